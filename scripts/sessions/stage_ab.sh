#!/bin/bash
# Per-execution staging of a device-resident batch group as one fused copy launch vs two torch copies
# (TDE_STAGE_FUSED=0): plan / fp32 / generic-plan GPU tests, then alternating driver-length benches.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/stage_ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_plan_gpu.py tests/test_fp32_gpu.py tests/test_convnet_gen_gpu.py -x -q -rf --capture=sys --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && { tail -30 $O/pytest.log; exit 3; }
for i in 1 2 3; do
  for f in 0 1; do
    TDE_STAGE_FUSED=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/drv_f${f}_$i.log 2>&1 || exit $?
    echo "fused=$f $(grep -h '"metric"' $O/drv_f${f}_$i.log | grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*')"
  done
done
TDE_STAGE_FUSED=1 timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > $O/long.log 2>&1 || exit $?
echo "long $(grep -h '"metric"' $O/long.log | grep -o '"ms_per_step": [0-9.]*')"
