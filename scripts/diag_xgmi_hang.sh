#!/bin/bash
# Root-cause run for the eager MWMS 2x2 xGMI timeouts: two worker processes x two
# replicas, all on cuda:0, eager launches, a short peer-wait timeout and the per-block phase trace
# (TDE_XGMI_TRACE): every launch records, per block, its start / publish / arrival / end times on the
# device's 100 MHz clock (shared by both processes) and which source flag never arrived.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TDE_XGMI_TIMEOUT=${TDE_XGMI_TIMEOUT:-2} PYTHONPATH="$PWD" TDE_HEARTBEAT=0 OMP_NUM_THREADS=2 TDE_RCCL=0
export TDE_XGMI_TRACE=64
run() {  # name args...
  local name=$1; shift
  echo "=== $name: $*"
  timeout -k 10 150 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
      --master-port=$((29600 + RANDOM % 300)) bench/mirrored_diag.py "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -v amdgpu.ids "gpurun_out/$name.log" | grep "diag" | tail -n 40
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
TDE_GRAPH=0 run eager_2x2 --mwms 2 --spe 4 --execs 2 && \
TDE_GRAPH=1 run graph_2x2 --mwms 2 --spe 4 --execs 2 && \
TDE_GRAPH=0 TDE_ALLREDUCE=xgmi run eager_2x1 --mwms 1 --spe 4 --execs 2
echo "=== done"
