#!/bin/bash
# wgrad side stream A/B (ResNet-18, Model B, LeNet-5 layer-wise), wgrad scratch A/B, GPU plan tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/s5; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_layers_gpu.py tests/test_plan_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
  for m in 0 1; do
    TDE_WGRAD_STREAM=$m timeout -k 10 200 python bench.py --model resnet18 --steps 30 --warmup 5 > $OUT/r18_side$m.$i.log 2>&1 || exit 1
    echo "resnet18 side=$m $(grep -o '"value": [0-9.]*' $OUT/r18_side$m.$i.log)"
    TDE_WGRAD_STREAM=$m timeout -k 10 200 python bench.py --model mnist_bn_cnn --steps 800 --warmup 64 > $OUT/bn_side$m.$i.log 2>&1 || exit 1
    echo "bn_cnn side=$m $(grep -o '"value": [0-9.]*' $OUT/bn_side$m.$i.log)"
  done
done
for m in 16 256; do
  TDE_WG_SCRATCH_MAX=$m timeout -k 10 200 python bench.py --model resnet18 --steps 30 --warmup 5 > $OUT/r18_wgs$m.log 2>&1 || exit 1
  echo "resnet18 wg_scratch_max=$m $(grep -o '"value": [0-9.]*' $OUT/r18_wgs$m.log)"
done
