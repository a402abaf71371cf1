#!/bin/bash
# A/B on one box: the hand-tuned MNIST-CNN forward at 1 / 2 / 4 pooled positions per workgroup (TDE_CONVNET_FPW).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/fpw_ab; mkdir -p $O
for i in 1 2; do
  for f in 2 1 4; do
    TDE_CONVNET_FPW=$f timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > $O/fpw${f}_$i.log 2>&1 || exit $?
    echo "fpw=$f $(tail -1 $O/fpw${f}_$i.log | cut -c80-160)"
  done
done
