#!/bin/bash
# The N=8 paths on one GPU: the xGMI kernel bitwise at 8 ranks, and the driver's bench command at N=8 with
# the xGMI communicator forced (the self-selection picks the fallback when 8 processes share one GPU).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD" TMPDIR=/tmp OMP_NUM_THREADS=2 TDE_HEARTBEAT=0
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q -rf --capture=sys --timeout 300 --timeout-method thread \
  "tests/test_xgmi_gpu.py::test_xgmi_allreduce_bitwise" > gpurun_out/pytest_l.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 gpurun_out/pytest_l.log
if [ $rc -ne 0 ]; then exit $rc; fi
TDE_ALLREDUCE=xgmi timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29781 bench.py --gpus 8 --steps 20 --warmup 5 > gpurun_out/rehearse_n8_xgmi.log 2>&1
rc=$?; echo "n8 rc=$rc"; grep -v amdgpu.ids gpurun_out/rehearse_n8_xgmi.log | grep '{"metric"\|replicas_identical' | cut -c1-400
