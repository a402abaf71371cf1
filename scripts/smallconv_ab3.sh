#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/sc; mkdir -p $OUT
run() { env "$@" timeout -k 10 200 python bench.py --model mnist_bn_cnn --steps 800 --warmup 64 > $OUT/run.log 2>&1 || exit 1; echo "$* $(grep -o '"value": [0-9.]*' $OUT/run.log) $(grep -o 'loss=[0-9.]*' $OUT/run.log)"; }
for i in 1 2; do
  run TDE_X=0
  run TDE_SMALLWG_IM2COL=1 TDE_SMALLCONV_WGRAD_MAX=4096
  run TDE_SMALLWG_IM2COL=1 TDE_SMALLCONV_WGRAD_MAX=8192
done
TDE_SMALLWG_IM2COL=1 TDE_SMALLCONV_WGRAD_MAX=8192 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_layers_gpu.py -k "smallconv_wgrad or model_b" > $OUT/pytest_sw.log 2>&1; tail -3 $OUT/pytest_sw.log
