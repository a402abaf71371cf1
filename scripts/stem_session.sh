#!/bin/bash
# Fused stem BN+ReLU+MaxPool: GPU tests, ResNet-18 A/B (TDE_BN_POOL=0 / 1, twice each)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/stem
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_layers_gpu.py \
  -k "bn_relu_maxpool or fuses_stem or small_resnet or maxpool or batchnorm or resnet" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for i in 1 2; do
  for e in 0 1; do
    TDE_BN_POOL=$e timeout -k 10 200 python bench.py --model resnet18 --steps 30 --warmup 5 > $OUT/r18_pool$e.$i.log 2>&1 || exit 1
    echo "pool=$e $(grep -o '"value": [0-9.]*' $OUT/r18_pool$e.$i.log)"
  done
done
