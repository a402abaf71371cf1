#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pf; mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 100 python bench.py --steps 20 --warmup 5 > $OUT/cnn20.$i.log 2>&1 || exit 1
  echo "cnn 20-step $(grep -o '"value": [0-9.]*' $OUT/cnn20.$i.log)"
done
timeout -k 10 100 python bench.py --steps 2000 --warmup 200 > $OUT/cnn2000.log 2>&1 || exit 1
echo "cnn 2000-step $(grep -o '"value": [0-9.]*' $OUT/cnn2000.log)"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_xgmi_gpu.py > $OUT/xgmi.log 2>&1; tail -2 $OUT/xgmi.log
