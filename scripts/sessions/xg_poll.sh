#!/bin/bash
# xGMI flag polling without the s_sleep between polls vs the previous build (TDE_HIP_LIB=libtde_hip_base.so):
# the 2-replica rehearsal, alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/xg_poll; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py -x -q -rf --capture=sys --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log
[ $rc -ne 0 ] && { tail -30 $O/pytest.log; exit 3; }
for i in 1 2 3; do
  for lib in libtde_hip_base.so libtde_hip.so; do
    TDE_HIP_LIB=$lib timeout -k 10 300 python bench.py --strategy mirrored --devices 0,0 --model mnist_cnn --steps 800 --warmup 64 > $O/${lib}_$i.log 2>&1 || exit $?
    echo "$lib $(grep -h '"metric"' $O/${lib}_$i.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
