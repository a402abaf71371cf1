#!/bin/bash
# Round-5 GPU session: the sharded PS device data plane (tests + throughput on both planes).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD OMP_NUM_THREADS=2 TDE_HEARTBEAT=0; O=gpurun_out/r5ps; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ps_device_gpu.py -q -rf --timeout 250 --timeout-method thread > $O/pt_ps.log 2>&1; rc=$?; tail -3 $O/pt_ps.log
[ $rc -gt 1 ] && exit $rc
for plane in tcp device; do
  for nps in 1 2; do
    E=""; [ $plane = device ] && E="TDE_PS_DEVICE=1"
    env $E timeout -k 10 200 python -m tensorflow_distributed_example_amd.launch --ps $nps --master 1 --workers 1 --timeout 150 bench/ps_throughput.py --max-steps 4000 --warm 300 > $O/b_${plane}_ps$nps.log 2>&1 || exit $?
    grep -h '"metric"' $O/b_${plane}_ps$nps.log | cut -c1-330
  done
done
