#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/sc; mkdir -p $OUT
run() { env "$@" timeout -k 10 200 python bench.py --model mnist_bn_cnn --steps 800 --warmup 64 > $OUT/run.log 2>&1 || exit 1; echo "$* $(grep -o '"value": [0-9.]*' $OUT/run.log)"; }
for i in 1 2; do
  run TDE_X=0
  run TDE_SMALLCONV_WGRAD_PPT=1 TDE_SMALLCONV_WGRAD_GRID=1024
  run TDE_SMALLCONV_WGRAD_PPT=1 TDE_SMALLCONV_WGRAD_GRID=256
done
