#!/bin/bash
# BN statistics slots 8 -> 32 (fewer same-address f64 atomics in the implicit-GEMM epilogue / BN reduce):
# layer-wise numerics + ResNet-18 bench + kernel statistics.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD" TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -rf --capture=sys --timeout 240 --timeout-method thread \
  tests/test_layers_gpu.py tests/test_layers_f32_gpu.py > gpurun_out/pytest_p.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_p.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --model resnet18 --steps 30 --warmup 5 > gpurun_out/b_rn_slots.log 2>&1
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/b_rn_slots.log | paste - -
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rn_slots -o run -- \
  python3 bench.py --model resnet18 --steps 10 --warmup 3 > gpurun_out/prof_rn_slots.log 2>&1
echo "prof rc=$?"
