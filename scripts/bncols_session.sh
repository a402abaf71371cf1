#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/bncols; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_layers_gpu.py -k "few_rows or batchnorm or dropout or model_b" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run() { env "$@" timeout -k 10 200 python bench.py --model mnist_bn_cnn --steps 800 --warmup 64 > $OUT/run.log 2>&1 || exit 1; echo "$* $(grep -o '"value": [0-9.]*' $OUT/run.log) $(grep -o 'loss=[0-9.]*' $OUT/run.log)"; }
for i in 1 2; do run TDE_BN_COLS_OFF=1; run TDE_X=0; done
