#!/bin/bash
# Root-cause runs for the eager MWMS 2x2 xGMI timeouts: two worker processes x two
# replicas, all on cuda:0, a short peer-wait timeout and the per-block phase trace (TDE_XGMI_TRACE):
# every launch records, per block, its start / publish / arrival / end times on the device's 100 MHz
# clock (shared by both processes), which source flag never arrived and the value that flag held.
#   r3 conditions: --spe 16 --execs 6, TDE_GRAPH=0; with and without the co-located-process spin cap (parallel/comm.spin_grid_caps).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TDE_XGMI_TIMEOUT=${TDE_XGMI_TIMEOUT:-3} PYTHONPATH="$PWD" TDE_HEARTBEAT=0 OMP_NUM_THREADS=2 TDE_RCCL=0
export TDE_XGMI_TRACE=64 TDE_HOST_TRACE=1
run() {  # name args...
  local name=$1; shift
  echo "=== $name: $*"
  timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
      --master-port=$((29600 + RANDOM % 300)) bench/mirrored_diag.py "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -v amdgpu.ids "gpurun_out/$name.log" | grep "diag" | grep -v " rank[01] epoch" | tail -n 60
  grep " rank[01] epoch" "gpurun_out/$name.log" | head -n 8
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
TDE_GRAPH=0 run eager_2x2_spincap --mwms 2 --spe 16 --execs 6 && \
TDE_GRAPH=0 TDE_XGMI_SPIN_CAP=0 run eager_2x2_nocap --mwms 2 --spe 16 --execs 6 && \
TDE_GRAPH=1 TDE_XGMI_SPIN_CAP=0 run graph_2x2_nocap --mwms 2 --spe 16 --execs 6 && \
TDE_GRAPH=0 TDE_XGMI_SPIN_CAP=0 run eager_2x2_nocap_bn --mwms 2 --spe 16 --execs 6 --model mnist_bn_cnn
echo "=== done"
