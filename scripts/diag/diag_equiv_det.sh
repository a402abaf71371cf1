#!/bin/bash
# Deterministic mode (TDE_DETERMINISTIC=1: ordered partial sums instead of float atomics) for the
# equivalence runs: single N times + Mirrored(2 on cuda:0) + MWMS 2 ranks, all compared with det single 1.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD" TDE_HEARTBEAT=0 OMP_NUM_THREADS=2 TDE_BENCH_WARM_MS=0 TDE_XGMI_TIMEOUT=20 TDE_DETERMINISTIC=1
O=gpurun_out/equivdet; mkdir -p $O
N=${1:-4}
for i in $(seq 1 $N); do
  timeout -k 10 90 python bench/dp_equiv.py --strategy single --out $O/single_$i.npz > $O/single_$i.log 2>&1 || { echo "single $i rc=$?"; tail -5 $O/single_$i.log; exit 1; }
done
timeout -k 10 90 python bench/dp_equiv.py --strategy mirrored --devices 0,0 --out $O/mirrored.npz > $O/mirrored.log 2>&1 || { echo "mirrored rc=$?"; tail -5 $O/mirrored.log; exit 1; }
TDE_RCCL=0 TDE_ALLREDUCE=xgmi timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29533 bench/dp_equiv.py --strategy mwms --out $O/mwms.npz > $O/mwms.log 2>&1 || { echo "mwms rc=$?"; tail -5 $O/mwms.log; exit 1; }
python - <<'PY'
import glob, numpy as np
O = "gpurun_out/equivdet"
ref = dict(np.load(f"{O}/single_1.npz"))
for f in sorted(glob.glob(f"{O}/*.npz")):
    w = dict(np.load(f))
    d = {k: float(np.abs(w[k] - ref[k]).max()) for k in ref if k in w}
    print(f.split("/")[-1], " ".join(f"{k}={v:.2e}" for k, v in d.items()))
PY
grep -h "\[dp_equiv\]" $O/*.log
