#!/bin/bash
# Round-5 GPU session: the generic-width fused small-CNN plan (csrc/kernels/convnet_gen.hip): float64 tests,
# data-parallel equivalence, per-launch micro timings, Model A-wide bench, rocprof kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/cgen; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_convnet_gen_gpu.py \
  tests/test_mirrored_gpu.py -k "generic or cgen" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for wv in 16 8; do TDE_CGEN_WAVES=$wv timeout -k 10 200 python bench/cgen_micro.py --phases > $O/micro_w$wv.log 2>&1 || { tail -20 $O/micro_w$wv.log; exit 1; }; echo "waves=$wv"; cat $O/micro_w$wv.log; done

TDE_CGEN_WAVES=8 timeout -k 10 200 python bench/cgen_micro.py --widths 64x128,32x64 --hrep 8 > $O/micro_h8.log 2>&1 || exit $?; cat $O/micro_h8.log
for m in mnist_cnn_wide; do
  timeout -k 10 300 python bench.py --model $m --steps 2000 --warmup 200 > $O/ours_$m.log 2>&1 || exit $?
  tail -1 $O/ours_$m.log | cut -c1-300
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$m -o run --output-format csv -- python bench.py --model $m --steps 200 --warmup 20 > $O/prof_$m.log 2>&1 || exit $?
done
