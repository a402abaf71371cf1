#!/bin/bash
# Fused DP exchange before / after: the 2-replica MirroredStrategy rehearsal on one
# GPU (one hipGraph per device, xGMI all-reduce with the optimizer fused), TDE_XGMI_PUSH=0 (backward, then
# the all-reduce pushes the whole bucket) vs 1 (the backward stores dW1 straight into the owners'
# windows): bench lines + rocprofv3 kernel statistics of each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}" TMPDIR=/tmp
mkdir -p gpurun_out
for model in mnist_cnn mnist_bn_cnn; do
  for push in 0 1; do
    name=push${push}_$model
    echo "=== $name ($(date +%T))"
    TDE_XGMI_PUSH=$push timeout -k 10 300 python bench.py --strategy mirrored --devices 0,0 --model $model \
        --steps 2000 --warmup 200 > gpurun_out/b_$name.log 2>&1 || { echo "STOP b_$name"; tail -5 gpurun_out/b_$name.log; exit 1; }
    tail -n 1 gpurun_out/b_$name.log
    TDE_XGMI_PUSH=$push timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d gpurun_out/prof_$name -o run -- python3 bench.py --strategy mirrored --devices 0,0 --model $model \
        --steps 400 --warmup 64 > gpurun_out/p_$name.log 2>&1 || { echo "STOP p_$name"; tail -5 gpurun_out/p_$name.log; exit 1; }
  done
done
echo "=== done"
