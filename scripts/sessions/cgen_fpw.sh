#!/bin/bash
# Generic plan: forward positions per workgroup A/B (TDE_CGEN_FPW = 1 / 2): kernel tests, micro timings with
# phase clocks, Model A wide bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/cgen_fpw; mkdir -p $O
for f in 2 1; do
  TDE_CGEN_FPW=$f timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_convnet_gen_gpu.py -k "kernels or trajectory" > $O/pytest_f$f.log 2>&1 || { tail -30 $O/pytest_f$f.log; exit 1; }
  tail -1 $O/pytest_f$f.log
  TDE_CGEN_FPW=$f timeout -k 10 200 python bench/cgen_micro.py --phases > $O/micro_f$f.log 2>&1 || exit $?
  grep '"cgen_fwd"\|fwd_phases' $O/micro_f$f.log
  TDE_CGEN_FPW=$f timeout -k 10 300 python bench.py --model mnist_cnn_wide --steps 2000 --warmup 200 > $O/wide_f$f.log 2>&1 || exit $?
  echo "fpw=$f $(tail -1 $O/wide_f$f.log | grep -o '"ms_per_step": [0-9.]*')"
done
