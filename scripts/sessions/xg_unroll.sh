#!/bin/bash
# xGMI phase loops with the loads of kXgU iterations issued before their stores vs the previous build
# (TDE_HIP_LIB=libtde_hip_base.so): data-parallel GPU tests on the new build, then the 2-replica rehearsal.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/xg_unroll; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_mirrored_gpu.py tests/test_xgmi_gpu.py -x -q -rf --capture=sys --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && { tail -40 $O/pytest.log; exit 3; }
for i in 1 2; do
  for lib in libtde_hip_base.so libtde_hip.so; do
    for m in mnist_cnn mnist_bn_cnn; do
      TDE_HIP_LIB=$lib timeout -k 10 300 python bench.py --strategy mirrored --devices 0,0 --model $m --steps 800 --warmup 64 > $O/${m}_${lib}_$i.log 2>&1 || exit $?
      echo "$lib $m $(grep -h '"metric"' $O/${m}_${lib}_$i.log | grep -o '"ms_per_step": [0-9.]*')"
    done
  done
done
