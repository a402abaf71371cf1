#!/bin/bash
# Forward: conv weight / gradient-replica loads issued before the image staging.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD" TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -rf --capture=sys --timeout 240 --timeout-method thread \
  tests/test_fp32_gpu.py tests/test_plan_gpu.py tests/test_mirrored_gpu.py > gpurun_out/pytest_r.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_r.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 2000 --warmup 200 > gpurun_out/b_r.log 2>&1
echo "headline $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_r.log) $(grep -o '"repeat_ms_per_step": \[[0-9., ]*\]' gpurun_out/b_r.log)"
timeout -k 10 100 python bench/micro.py > gpurun_out/micro_r.json 2>/dev/null; echo "micro rc=$?"
