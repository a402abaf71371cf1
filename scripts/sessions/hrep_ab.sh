#!/bin/bash
# Headline A/B (hand-tuned Model A): pre-activation split-K replicas TDE_CONVNET_HREP = 2 / 3 / 4.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/hrep_ab; mkdir -p $O
for i in 1 2; do
  for h in 4 2 3; do
    TDE_CONVNET_HREP=$h timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > $O/h${h}_$i.log 2>&1 || exit $?
    echo "hrep=$h $(tail -1 $O/h${h}_$i.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
