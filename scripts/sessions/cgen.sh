#!/bin/bash
# Round-5 GPU session: the generic-width fused small-CNN plan (csrc/kernels/convnet_gen.hip): float64 tests,
# Model A-wide bench on it, rocprof kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/cgen; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_convnet_gen_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for m in mnist_cnn_wide; do
  timeout -k 10 300 python bench.py --model $m --steps 2000 --warmup 200 > $O/ours_$m.log 2>&1 || exit $?
  tail -1 $O/ours_$m.log | cut -c1-300
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$m -o run --output-format csv -- python bench.py --model $m --steps 200 --warmup 20 > $O/prof_$m.log 2>&1 || exit $?
done
