#!/bin/bash
# rocprofv3 kernel statistics of the layer-wise plan models (one MI355X).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in ${MODELS:-lenet5 mnist_bn_cnn mnist_mlp}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$m -o run --output-format csv -- \
    python bench.py --model $m --steps 160 --warmup 32 > gpurun_out/prof_$m.log 2>&1 || exit $?
done
