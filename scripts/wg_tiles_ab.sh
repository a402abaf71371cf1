#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/wgt; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_layers_gpu.py -k "dense or conv_fwd_dgrad or wgrad or model_b or resnet" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  for m in 0 1; do
    TDE_WG_SMALL_TILES=$m timeout -k 10 200 python bench.py --model mnist_bn_cnn --steps 800 --warmup 64 > $OUT/bn$m.$i.log 2>&1 || exit 1
    echo "bn_cnn small_tiles=$m $(grep -o '"value": [0-9.]*' $OUT/bn$m.$i.log)"
  done
  for m in 0 1; do
    TDE_WG_SMALL_TILES=$m timeout -k 10 200 python bench.py --model resnet18 --steps 30 --warmup 5 > $OUT/r18_$m.$i.log 2>&1 || exit 1
    echo "resnet18 small_tiles=$m $(grep -o '"value": [0-9.]*' $OUT/r18_$m.$i.log)"
  done
done
