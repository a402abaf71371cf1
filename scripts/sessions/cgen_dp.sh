#!/bin/bash
# Data-parallel rehearsal of the generic plan (Model A wide, Mirrored(2) on one GPU): fused push vs the
# post-backward exchange, and the hand-tuned Model A for comparison.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/cgen_dp; mkdir -p $O
for m in mnist_cnn_wide mnist_cnn; do
  for push in 1 0; do
    TDE_XGMI_PUSH=$push timeout -k 10 300 python bench.py --strategy mirrored --devices 0,0 --model $m --steps 800 --warmup 64 > $O/${m}_push$push.log 2>&1 || exit $?
    echo "$m push=$push $(tail -1 $O/${m}_push$push.log | grep -o '"ms_per_step": [0-9.]*\|"exchange": "[a-z_]*"' | tr '\n' ' ')"
  done
done
