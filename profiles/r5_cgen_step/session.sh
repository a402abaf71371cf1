#!/bin/bash
# The generic fused CNN step as ONE launch (forward, grid barrier, backward: cgen_step_kernel) vs two launches
# (TDE_CGEN_STEP=0): generic-plan GPU tests, then alternating benches at the reference width (generic plan
# forced) and at Conv2D(64)/Dense(128), and the hand-tuned headline for reference.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/cgen_step; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_convnet_gen_gpu.py -x -v -rf --capture=sys --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 3; }
tail -3 $O/pytest.log
for w in 32x64 16x32 64x64 64x128; do
  timeout -k 10 300 python bench/cgen_step_phases.py --width $w > $O/phases_$w.log 2>&1 || exit $?
  tail -2 $O/phases_$w.log | cut -c1-600
done
[ -n "$PHASES_ONLY" ] && exit 0
for i in 1 2; do
  for st in 0 1; do
    TDE_CGEN_STEP=$st TDE_CONVNET_GENERIC=1 timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > $O/ref_step${st}_$i.log 2>&1 || exit $?
    echo "ref generic step=$st $(tail -1 $O/ref_step${st}_$i.log | cut -c1-190)"
    TDE_CGEN_STEP=$st timeout -k 10 300 python bench.py --model mnist_cnn_wide --steps 2000 --warmup 200 > $O/wide_step${st}_$i.log 2>&1 || exit $?
    echo "wide step=$st $(tail -1 $O/wide_step${st}_$i.log | cut -c1-190)"
  done
  timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > $O/tuned_$i.log 2>&1 || exit $?
  echo "tuned $(tail -1 $O/tuned_$i.log | cut -c1-190)"
done
