#!/bin/bash
# In-process / multi-process xGMI diagnostics (bench/mirrored_diag.py) with a short peer-wait timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TDE_XGMI_TIMEOUT=3 PYTHONPATH="$PWD" TDE_HEARTBEAT=0 OMP_NUM_THREADS=2 TDE_RCCL=0
run() { echo "=== $*"; timeout -k 10 100 python -u "$@" 2>&1 | grep -v amdgpu.ids; }
TDE_XGMI_BLOCKS=8 run -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
    --master-port=29611 bench/mirrored_diag.py --mwms 2 --spe 16 --execs 6 && \
TDE_GRAPH=0 run -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
    --master-port=29612 bench/mirrored_diag.py --mwms 2 --spe 16 --execs 6
