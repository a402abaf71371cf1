#!/bin/bash
# Generic plan: pre-activation replica count A/B (forward split-K contention vs the backward's reads),
# per-launch micro timings and the Model A-wide bench at each setting.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/cgen_hrep; mkdir -p $O
for h in 1 2 4; do
  timeout -k 10 200 python bench/cgen_micro.py --widths 64x128,32x64 --hrep $h > $O/micro_h$h.log 2>&1 || exit $?
  grep -v amdgpu $O/micro_h$h.log | grep cgen
  TDE_CONVNET_HREP=$h timeout -k 10 300 python bench.py --model mnist_cnn_wide --steps 2000 --warmup 200 > $O/wide_h$h.log 2>&1 || exit $?
  echo "hrep=$h $(tail -1 $O/wide_h$h.log | grep -o '"ms_per_step": [0-9.]*')"
done
