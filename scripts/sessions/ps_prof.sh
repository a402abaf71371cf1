#!/bin/bash
# The PS device-plane exchange: device time (bench/ps_exchange_micro.py), the PS GPU tests, then Estimator
# throughput (pipelined loop vs synchronous, 1 and 2 ps tasks).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/ps_prof; mkdir -p $O
timeout -k 10 200 python bench/ps_exchange_micro.py > $O/micro.log 2>&1 || { tail -20 $O/micro.log; exit 3; }
tail -1 $O/micro.log
export OMP_NUM_THREADS=2 TDE_HEARTBEAT=0 TDE_PS_DEVICE=1
timeout -k 10 600 python -u -m pytest tests/test_ps_device_gpu.py -q -rf --timeout 250 --timeout-method thread > $O/pt_ps.log 2>&1; rc=$?; tail -3 $O/pt_ps.log
[ $rc -gt 1 ] && exit $rc
for pipe in 0 1; do
  for nps in 1 2; do
    TDE_PS_PIPELINE=$pipe TDE_PS_GRAPH=0 timeout -k 10 200 python -m tensorflow_distributed_example_amd.launch --ps $nps --master 1 --workers 1 --timeout 150 bench/ps_throughput.py --max-steps 4000 --warm 300 > $O/b_pipe${pipe}_ps${nps}.log 2>&1 || exit $?
    echo "pipe=$pipe ps=$nps $(grep -h '"metric"' $O/b_pipe${pipe}_ps${nps}.log | cut -c1-260)"
  done
done
