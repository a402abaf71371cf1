#!/bin/bash
# Round-5 GPU session: the layer-wise float32 plan (kernel tests, width-variant benches, kernel statistics).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/r5f; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_layers_f32_gpu.py -x -q -rf --timeout 200 --timeout-method thread > $O/pt_f32.log 2>&1; rc=$?; tail -3 $O/pt_f32.log
[ $rc -ne 0 ] && exit $rc
for m in mnist_cnn_wide mnist_bn_cnn_x2; do
  timeout -k 10 300 python bench.py --model $m --steps 400 --warmup 50 > $O/ours_$m.log 2>&1 || exit $?
  tail -1 $O/ours_$m.log | cut -c1-220
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$m -o run --output-format csv -- python bench.py --model $m --steps 100 --warmup 20 > $O/prof_$m.log 2>&1 || exit $?
done
