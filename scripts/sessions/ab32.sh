cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/ab32; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_layers_gpu.py -q -x -k "mfma32 or conv_fwd_dgrad or wgrad_lds or largest or dense_fwd" --timeout 120 --timeout-method thread > $O/pytest_layers.log 2>&1; rc=$?; tail -3 $O/pytest_layers.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_mirrored_gpu.py -q -x --timeout 120 --timeout-method thread > $O/pytest_mirrored.log 2>&1; rc=$?; tail -3 $O/pytest_mirrored.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench/resnet_layers.py --ab-mfma32 > $O/ab.log 2>&1; rc=$?; grep TOTAL $O/ab.log; [ $rc -le 1 ] || exit $rc
TDE_MFMA32=7 timeout -k 10 200 python bench.py --model resnet18 --steps 30 --warmup 5 > $O/bench_rn_m32.log 2>&1; tail -1 $O/bench_rn_m32.log | cut -c1-200
timeout -k 10 200 python bench.py --model resnet18 --steps 30 --warmup 5 > $O/bench_rn_m16.log 2>&1; tail -1 $O/bench_rn_m16.log | cut -c1-200
