#!/bin/bash
# The copy_pairs kernel test, then the xGMI all-reduce per-block phase trace of the 2-replica rehearsal on the
# final tree (after the acquire removal; compare profiles/r5_xgmi_trace/mirrored2.log).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/copy_trace; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -rf -k copy_pairs --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log
[ $rc -ne 0 ] && { tail -30 $O/pytest.log; exit 3; }
TDE_XGMI_TRACE=64 timeout -k 10 300 python bench/mirrored_diag.py --devices 0,0 --spe 16 --execs 6 > $O/mirrored2.log 2>&1 || { tail -20 $O/mirrored2.log; exit 3; }
tail -25 $O/mirrored2.log
