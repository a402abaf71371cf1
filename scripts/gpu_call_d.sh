#!/bin/bash
# One GPU call: xGMI hang diagnosis, the fused-push / eager MWMS tests, fused-push before/after profiles.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD" TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/diag_xgmi_hang.sh > gpurun_out/diag_hang2.out 2>&1
echo "diag rc=$?"; tail -n 3 gpurun_out/diag_hang2.out
timeout -k 10 600 python -u -m pytest -x -q -rf --timeout 240 --timeout-method thread \
  tests/test_mirrored_gpu.py::test_eager_mwms_2x2_rehearsal_runs_clean \
  tests/test_mirrored_gpu.py::test_fused_push_exchange_is_bitwise_the_post_backward_exchange > gpurun_out/pytest_d.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 4 gpurun_out/pytest_d.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/prof_push.sh > gpurun_out/prof_push.out 2>&1
echo "push rc=$?"; tail -n 12 gpurun_out/prof_push.out
bash scripts/rehearse_scale.sh 2 4 8 > gpurun_out/rehearse.out 2>&1
echo "rehearse rc=$?"; tail -n 12 gpurun_out/rehearse.out
