#!/bin/bash
# A/B on one box: the headline Model A (Conv2D(32)/Dense(64)) on the hand-tuned plan vs the generic fused plan
# (TDE_CONVNET_GENERIC=1), alternating runs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/cgen_ab; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > $O/tuned_$i.log 2>&1 || exit $?
  tail -1 $O/tuned_$i.log | cut -c1-200
  TDE_CONVNET_GENERIC=1 timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > $O/generic_$i.log 2>&1 || exit $?
  tail -1 $O/generic_$i.log | cut -c1-200
done
