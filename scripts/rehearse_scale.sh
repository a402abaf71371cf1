#!/bin/bash
# The driver's multi-GPU bench command (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N)
# rehearsed on the ONE-GPU box: N ranks map onto cuda:0 (bench.py: local_rank % device_count), so this
# checks the N-rank code path end to end — xGMI windows over IPC, the fused push, graph capture, the
# rank-max timing and the single JSON line — not throughput (the N ranks share one GPU).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD" TMPDIR=/tmp OMP_NUM_THREADS=2 TDE_HEARTBEAT=0
mkdir -p gpurun_out
for n in ${*:-2 4 8}; do
  echo "=== N=$n ($(date +%T))"
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29700 + n)) bench.py --gpus $n --steps 200 --warmup 20 > gpurun_out/rehearse_n$n.log 2>&1
  rc=$?
  grep -v amdgpu.ids gpurun_out/rehearse_n$n.log | grep '{"metric"\|replicas_identical\|exchange\|Error\|error' | tail -n 5
  echo "=== N=$n rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo "=== done"
