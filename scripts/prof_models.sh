#!/bin/bash
# rocprofv3 kernel statistics for the layer-wise models (Model B, ResNet-18) and the torch baseline.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}" TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
}
run prof_bn_cnn 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bn -o run --output-format csv -- python bench.py --model mnist_bn_cnn --steps 160 --warmup 16
run prof_resnet18 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn -o run --output-format csv -- python bench.py --model resnet18 --steps 10 --warmup 3
run torch_resnet18 300 python bench/torch_baseline.py --model resnet18 --steps 30 --warmup 5 --channels-last
run torch_resnet18_nchw 300 python bench/torch_baseline.py --model resnet18 --steps 30 --warmup 5
echo "=== done"
