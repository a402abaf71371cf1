#!/bin/bash
# Conv-gradient replicas in the data-parallel step (the all-reduce sums them) + pre-activation replica count.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD" TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -q -rf --capture=sys --timeout 240 --timeout-method thread \
  tests/test_fp32_gpu.py tests/test_xgmi_gpu.py tests/test_mirrored_gpu.py > gpurun_out/pytest_o.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_o.log
if [ $rc -ne 0 ]; then exit $rc; fi
for h in 4 8; do
  TDE_CONVNET_HREP=$h timeout -k 10 200 python bench.py --steps 2000 --warmup 200 > gpurun_out/b_hrep$h.log 2>&1
  echo "HREP=$h $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_hrep$h.log) $(grep -o '"repeat_ms_per_step": \[[0-9., ]*\]' gpurun_out/b_hrep$h.log)"
done
for g in 1 8; do
  TDE_CONVNET_GREP=$g timeout -k 10 300 python bench.py --strategy mirrored --devices 0,0 --steps 2000 --warmup 200 > gpurun_out/b_o_mirrored_g$g.log 2>&1
  echo "mirrored GREP=$g $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_o_mirrored_g$g.log)"
done
bash scripts/rehearse_scale.sh 2 4 > gpurun_out/rehearse_o.out 2>&1
echo "rehearse rc=$?"; grep -o '"n_gpus": [0-9]*\|"ms_per_step": [0-9.]*' gpurun_out/rehearse_o.out | paste - -
