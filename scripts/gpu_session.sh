#!/bin/bash
# One GPU-box session: tests, smoke, bench, rocprof.  Stops at the first step
# that ends in a fault/abort/timeout (exit codes other than 0/1).
#   bash scripts/gpu_session.sh [all|tests|bench|models|baseline|micro|prof|equiv|buckets|ps|f32|widths]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step pytest_gpu ${PYTEST_TIMEOUT:-1000} python -u -m pytest tests -m gpu -q -rf --capture=sys --timeout 120 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 600 python bench.py --steps 2000 --warmup 200
  step bench_nograph 600 python bench.py --steps 400 --warmup 64 --no-graph
fi
if [ "$MODE" = all ] || [ "$MODE" = models ]; then
  step bench_bn_cnn 600 python bench.py --model mnist_bn_cnn --steps 800 --warmup 64
  step bench_resnet18 600 python bench.py --model resnet18 --steps 30 --warmup 5
fi
if [ "$MODE" = all ] || [ "$MODE" = baseline ]; then
  step torch_cnn 600 python bench/torch_baseline.py --model mnist_cnn --steps 400 --warmup 64
  step torch_cnn_graph 600 python bench/torch_baseline.py --model mnist_cnn --steps 2000 --warmup 64 --graph
  step torch_bn_cnn_graph 600 python bench/torch_baseline.py --model mnist_bn_cnn --steps 800 --warmup 64 --graph
  step torch_resnet18 600 python bench/torch_baseline.py --model resnet18 --steps 30 --warmup 5 --channels-last
  step torch_cnn_graph_fp32 600 python bench/torch_baseline.py --model mnist_cnn --steps 2000 --warmup 64 --graph --dtype fp32
  step torch_bn_cnn_graph_fp32 600 python bench/torch_baseline.py --model mnist_bn_cnn --steps 800 --warmup 64 --graph --dtype fp32
fi
if [ "$MODE" = all ] || [ "$MODE" = micro ]; then
  step micro 300 python bench/micro.py
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps 400 --warmup 64
fi
# topic sessions of this round (scripts/sessions/<name>.sh): equiv | buckets | ps | f32 | widths | cgen
case "$MODE" in
  equiv) bash scripts/equiv_repeat.sh "${@:2}" || exit $? ;;
  buckets|ps|f32|widths|cgen|cgen_ab|fpw_ab|rn_knobs|final|cgen_dp|cgen_hrep|hrep_ab|cgen_fpw|ps_prof|xg_acq|stage_ab|drv_trace|xg_unroll|bnpool_ab|copy_trace|xg_poll|stats|copy_ab) bash "scripts/sessions/$MODE.sh" || exit $? ;;
esac
echo "=== done"
