#!/bin/bash
# A/B: weight-gradient split-K partials through scratch + one reduction pass (up to N splits) vs f32 atomics
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/wgs; mkdir -p $OUT
for i in 1 2; do
  for m in 16 256; do
    TDE_WG_SCRATCH_MAX=$m timeout -k 10 200 python bench.py --model resnet18 --steps 30 --warmup 5 > $OUT/r18_wgs$m.$i.log 2>&1 || exit 1
    echo "wg_scratch_max=$m $(grep -o '"value": [0-9.]*' $OUT/r18_wgs$m.$i.log)"
  done
done
TDE_WG_SCRATCH_MAX=256 timeout -k 10 300 python bench/resnet_layers.py > $OUT/layers256.log 2>&1 || exit 1
timeout -k 10 300 python bench/resnet_layers.py > $OUT/layers16.log 2>&1
