#!/bin/bash
# xGMI all-reduce latency work: correctness (bitwise tests), phase trace, rehearsal bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD" TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q -rf --capture=sys --timeout 240 --timeout-method thread \
  tests/test_xgmi_gpu.py tests/test_mirrored_gpu.py > gpurun_out/pytest_k.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_k.log
if [ $rc -ne 0 ]; then exit $rc; fi
TDE_XGMI_TRACE=64 timeout -k 10 200 python bench/mirrored_diag.py --devices 0,0 --spe 16 --execs 4 --trace-show 12 > gpurun_out/ar_trace_k.log 2>&1
echo "trace rc=$?"; grep "rank0 epoch" gpurun_out/ar_trace_k.log | head -4 | cut -c1-250
for push in 1; do
  TDE_XGMI_PUSH=$push timeout -k 10 300 python bench.py --strategy mirrored --devices 0,0 --steps 2000 --warmup 200 > gpurun_out/b_k_mirrored.log 2>&1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_k_mirrored.log
done
bash scripts/rehearse_scale.sh 2 4 > gpurun_out/rehearse_k.out 2>&1
echo "rehearse rc=$?"; grep -o '"n_gpus": [0-9]*\|"ms_per_step": [0-9.]*' gpurun_out/rehearse_k.out | paste - -
