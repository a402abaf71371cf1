#!/bin/bash
# Repeatability of the fused single-replica step against the CPU reference (bench/equiv_trace.py):
# N1 in-process trials without per-step tracing, then N2 separate processes of bench/dp_equiv.py
# (single + Mirrored), each compared with the CPU reference weights.  Usage: equiv_repeat.sh [N1] [N2]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
OUT=gpurun_out/equiv; mkdir -p $OUT
N1=${1:-30}; N2=${2:-6}
timeout -k 10 300 python -u bench/equiv_trace.py --trials "$N1" --no-trace > $OUT/inproc.log 2>&1 || exit $?
tail -1 $OUT/inproc.log
TDE_EXECUTOR=reference CUDA_VISIBLE_DEVICES= timeout -k 10 120 python bench/dp_equiv.py --strategy single --out $OUT/ref.npz > $OUT/ref.log 2>&1 || exit $?
for i in $(seq 1 "$N2"); do
  timeout -k 10 120 python bench/dp_equiv.py --strategy single --out $OUT/single_$i.npz > $OUT/single_$i.log 2>&1 || exit $?
  timeout -k 10 120 python bench/dp_equiv.py --strategy mirrored --devices 0,0 --out $OUT/mirrored_$i.npz > $OUT/mirrored_$i.log 2>&1 || exit $?
done
python - <<'PY'
import glob, numpy as np
ref = np.load("gpurun_out/equiv/ref.npz")
for f in sorted(glob.glob("gpurun_out/equiv/*_*.npz")):
    d = np.load(f)
    print(f.split("/")[-1], " ".join(f"{k}={np.abs(d[k] - ref[k]).max():.2e}" for k in ref.files))
PY
grep -h dp_equiv $OUT/*.log
