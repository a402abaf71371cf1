#!/bin/bash
# Round-5 GPU session: reverse-order bucket overlap of the per-device-group strategies (tests, a bf16
# run-to-run control, Mirrored ResNet-18 rehearsals with / without buckets, rocprofv3 overlap check).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD; O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_mirrored_gpu.py -k "group_buckets" -q -rf --timeout 150 --timeout-method thread > $O/pt_buckets.log 2>&1; rc=$?; tail -3 $O/pt_buckets.log
[ $rc -gt 1 ] && exit $rc
for i in 1 2; do
  TDE_OVERLAP=0 timeout -k 10 120 python bench/dp_equiv.py --strategy mirrored --devices 0,0 --model mini_resnet --dtype bf16 --out $O/ctl_$i.npz > $O/ctl_$i.log 2>&1 || exit $?
done
python -c "
import numpy as np; a=np.load('$O/ctl_1.npz'); b=np.load('$O/ctl_2.npz')
print('bf16 one-bucket run-to-run max diff:', max(float(np.abs(a[k]-b[k]).max()) for k in a.files))"
timeout -k 10 300 python bench.py --strategy mirrored --devices 0,0 --model resnet18 --steps 20 --warmup 5 > $O/rn_mirrored_buckets.log 2>&1 || exit $?
tail -1 $O/rn_mirrored_buckets.log | cut -c1-400
TDE_OVERLAP=0 timeout -k 10 300 python bench.py --strategy mirrored --devices 0,0 --model resnet18 --steps 20 --warmup 5 > $O/rn_mirrored_one.log 2>&1 || exit $?
tail -1 $O/rn_mirrored_one.log | cut -c1-400
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python bench.py --strategy mirrored --devices 0,0 --model resnet18 --steps 6 --warmup 2 > $O/rn_prof.log 2>&1 || exit $?
f=$(find $O/prof -name "*kernel_trace.csv" | head -1); python scripts/overlap_check.py $f
