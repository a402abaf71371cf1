#!/bin/bash
# Round-5 GPU session: the width variants of Model A / Model B (layer-wise f32 plan vs stock torch fp32).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/r5w; mkdir -p $O
for m in mnist_cnn_wide mnist_bn_cnn_x2; do
  timeout -k 10 300 python bench.py --model $m --steps 400 --warmup 50 > $O/ours_$m.log 2>&1 || exit $?
  tail -1 $O/ours_$m.log | cut -c1-260
  timeout -k 10 300 python bench/torch_baseline.py --model $m --steps 400 --warmup 64 --graph --dtype fp32 > $O/torch_$m.log 2>&1 || exit $?
  tail -1 $O/torch_$m.log | cut -c1-200
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$m -o run --output-format csv -- python bench.py --model $m --steps 100 --warmup 20 > $O/prof_$m.log 2>&1 || exit $?
done
