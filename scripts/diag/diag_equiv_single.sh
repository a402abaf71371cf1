#!/bin/bash
# Repeat the single-replica equivalence run (bench/dp_equiv.py --strategy single) N times per
# configuration and group the final losses: which configuration shows the intermittent alternative
# trajectory.  Usage: diag_equiv_single.sh N "LABEL:ENV=V ENV2=V" ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD" TDE_HEARTBEAT=0 OMP_NUM_THREADS=2 TDE_BENCH_WARM_MS=0
O=gpurun_out/equiv1; mkdir -p $O
N=$1; shift
for cfg in "$@"; do
  label=${cfg%%:*}; envs=${cfg#*:}
  for i in $(seq 1 $N); do
    env $envs timeout -k 10 90 python bench/dp_equiv.py --strategy single --out $O/${label}_$i.npz > $O/${label}_$i.log 2>&1 || { echo "$label $i rc=$?"; tail -5 $O/${label}_$i.log; exit 1; }
    echo "$label $i $(grep -o 'loss=[0-9.]*' $O/${label}_$i.log)"
  done
done
