#!/bin/bash
# fwd/dgrad split-K target sweep over the layer-wise models (one MI355X): one JSON line per (target, model)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/split
for t in 512 0 128 256 1024; do
  for m in mnist_bn_cnn lenet5 mnist_mlp; do
    TDE_FWD_SPLIT_TARGET=$t timeout -k 10 120 python bench.py --model $m --steps 800 --warmup 64 > gpurun_out/split/${m}_$t.log 2>&1 || exit $?
    echo "target=$t $m $(grep -o '"value": [0-9.]*' gpurun_out/split/${m}_$t.log)"
  done
  TDE_FWD_SPLIT_TARGET=$t timeout -k 10 200 python bench.py --model resnet18 --steps 30 --warmup 5 > gpurun_out/split/resnet18_$t.log 2>&1 || exit $?
  echo "target=$t resnet18 $(grep -o '"value": [0-9.]*' gpurun_out/split/resnet18_$t.log)"
done
