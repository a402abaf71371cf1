#!/bin/bash
# Repeat the single-replica and Mirrored(2 on cuda:0) equivalence runs of
# tests/test_mirrored_gpu.py and compare every run's weights with the first single run: which side
# of the intermittent conv2d/kernel mismatch varies between runs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD" TDE_HEARTBEAT=0 OMP_NUM_THREADS=2 TDE_BENCH_WARM_MS=0 TDE_XGMI_TIMEOUT=20
O=gpurun_out/equiv; mkdir -p $O
N=${1:-4}
for i in $(seq 1 $N); do
  timeout -k 10 90 python bench/dp_equiv.py --strategy single --out $O/single_$i.npz > $O/single_$i.log 2>&1 || { echo "single $i rc=$?"; exit 1; }
  timeout -k 10 90 python bench/dp_equiv.py --strategy mirrored --devices 0,0 --out $O/mirrored_$i.npz > $O/mirrored_$i.log 2>&1 || { echo "mirrored $i rc=$?"; exit 1; }
  echo "run $i done"
done
python - <<'PY'
import glob, numpy as np
O = "gpurun_out/equiv"
ref = dict(np.load(f"{O}/single_1.npz"))
for f in sorted(glob.glob(f"{O}/*.npz")):
    w = dict(np.load(f))
    d = {k: float(np.abs(w[k] - ref[k]).max()) for k in ref if k in w}
    print(f.split("/")[-1], " ".join(f"{k}={v:.2e}" for k, v in d.items()))
PY
grep -h "\[dp_equiv\]" $O/*.log
