#!/bin/bash
# One GPU call: coalesced fused-push check (bitwise tests + before/after), hardware counters, fp32 torch baselines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD" TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -rf --timeout 240 --timeout-method thread \
  tests/test_mirrored_gpu.py::test_fused_push_exchange_is_bitwise_the_post_backward_exchange > gpurun_out/pytest_e.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_e.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/prof_push.sh > gpurun_out/prof_push.out 2>&1
echo "push rc=$?"; grep -o '"ms_per_step": [0-9.]*\|"exchange": "[a-z_]*"\|=== [a-z0-9_]*' gpurun_out/prof_push.out | paste - - - 
bash scripts/pmc_models.sh > gpurun_out/pmc_models.out 2>&1
rc=$?; echo "pmc rc=$rc"; tail -n 4 gpurun_out/pmc_models.out
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/gpu_session.sh baseline > gpurun_out/baseline.out 2>&1
echo "baseline rc=$?"; grep -h '"value"' gpurun_out/torch_*.log | cut -c1-200
