#!/bin/bash
# xGMI all-reduce on the uncached window without the waits' per-block system-scope acquire, vs with it
# (TDE_XGMI_ACQUIRE=1): data-parallel GPU tests, then the 2-replica Mirrored rehearsal on one GPU.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/xg_acq; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_mirrored_gpu.py tests/test_xgmi_gpu.py -x -q -rf --capture=sys --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && { tail -40 $O/pytest.log; exit 3; }
for i in 1 2; do
  for acq in ${ACQS:-1 0}; do
    for m in mnist_cnn mnist_bn_cnn; do
      TDE_XGMI_ACQUIRE=$acq timeout -k 10 300 python bench.py --strategy mirrored --devices 0,0 --model $m --steps 800 --warmup 64 > $O/${m}_acq${acq}_$i.log 2>&1 || exit $?
      echo "acq=$acq $m $(grep -h '"metric"' $O/${m}_acq${acq}_$i.log | grep -o '"ms_per_step": [0-9.]*')"
    done
  done
done
