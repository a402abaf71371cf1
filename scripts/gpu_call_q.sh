#!/bin/bash
# LDS row-stride padding of the head pieces (dlogits / W2 in the fused MNIST-CNN backward, the BN-CNN head):
# numerics + benches + PMC conflict counter of the backward.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD" TMPDIR=/tmp TDE_BENCH_WARM_MS=200
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -rf --capture=sys --timeout 240 --timeout-method thread \
  tests/test_fp32_gpu.py tests/test_bncnn_gpu.py tests/test_kernels_gpu.py tests/test_plan_gpu.py > gpurun_out/pytest_q.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_q.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 2000 --warmup 200 > gpurun_out/b_q.log 2>&1
echo "headline $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_q.log) $(grep -o '"repeat_ms_per_step": \[[0-9., ]*\]' gpurun_out/b_q.log)"
timeout -k 10 200 python bench.py --model mnist_bn_cnn --steps 800 --warmup 64 > gpurun_out/b_q_bn.log 2>&1
echo "bn_cnn $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_q_bn.log)"
export TDE_BENCH_WARM_MS=0
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv \
  -d gpurun_out/pmc_q -o run -- python3 bench.py --steps 64 --warmup 16 > gpurun_out/pmc_q.log 2>&1
echo "pmc rc=$?"
