#!/bin/bash
# Replicated conv-gradient accumulation in the fused MNIST-CNN step: numerics (fused-step tests), then the
# headline bench per replica count (TDE_CONVNET_GREP) and the micro phase stamps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD" TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -rf --capture=sys --timeout 240 --timeout-method thread \
  tests/test_fp32_gpu.py tests/test_plan_gpu.py tests/test_kernels_gpu.py > gpurun_out/pytest_n.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_n.log
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2 4 8; do
  TDE_CONVNET_GREP=$r timeout -k 10 200 python bench.py --steps 2000 --warmup 200 > gpurun_out/b_grep$r.log 2>&1
  echo "GREP=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_grep$r.log) $(grep -o '"repeat_ms_per_step": \[[0-9., ]*\]' gpurun_out/b_grep$r.log)"
done
timeout -k 10 100 python bench/micro.py > gpurun_out/micro_grep8.json 2>/dev/null; echo "micro rc=$?"
timeout -k 10 100 python bench.py --steps 20 --warmup 5 > gpurun_out/b_driver_len.log 2>&1
echo "driver-length $(grep -o '"value": [0-9.]*, "unit": "images/sec", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*' gpurun_out/b_driver_len.log)"
