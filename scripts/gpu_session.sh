#!/bin/bash
# One GPU-box session (run through gpurun): every step under its own time limit, stopping at the first step
# that ends in a fault / abort / timeout (exit codes other than 0 / 1).  Logs land in gpurun_out/<mode>/.
#   bash scripts/gpu_session.sh <mode> [args]
# modes:
#   tests     pytest -m gpu + smoke()                  bench     headline (2,000 steps) + eager
#   models    Model B + ResNet-18 benches              baseline  stock-PyTorch baselines (bench/torch_baseline.py)
#   final     end-of-round validation: tests, smoke, the headline at 2,000 steps and at the driver's length in
#             5 fresh processes, every benchmarked model
#   stats     rocprofv3 --kernel-trace --stats of the headline, Model B, ResNet-18, the PS exchange micro
#   layers    ResNet-18 per-layer GEMM timings (bench/resnet_layers.py [args], e.g. --ab-mfma32)
#   ps        PS device data plane: its GPU tests + throughput on both planes x 1 / 2 ps tasks
#   pytest    pytest on the given test files / -k expression ([args] passed through)
#   micro     bench/micro.py
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}" TMPDIR=/tmp
MODE=${1:-tests}
shift || true
O=gpurun_out/$MODE
mkdir -p "$O"
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  tail -n 3 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
stat() {  # name cmd...: rocprofv3 kernel statistics, the summary CSV copied next to the log
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$n" -o "$n" -- "$@" > "$O/$n.log" 2>&1 \
    || { tail -20 "$O/$n.log"; exit 3; }
  local f
  f=$(find "$O/$n" -name "*kernel_stats.csv" | head -1)
  cp "$f" "$O/${n}_kernel_stats.csv"
  head -6 "$f" | cut -d, -f1-5
}
PYT="python -u -m pytest -q -rf --timeout 120 --timeout-method thread"
case "$MODE" in
  tests)
    step pytest_gpu 1100 $PYT tests -m gpu
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
  bench)
    step bench 300 python bench.py --steps 2000 --warmup 200
    step bench_nograph 300 python bench.py --steps 400 --warmup 64 --no-graph ;;
  models)
    step bench_bn_cnn 300 python bench.py --model mnist_bn_cnn --steps 800 --warmup 64
    step bench_resnet18 300 python bench.py --model resnet18 --steps 30 --warmup 5 ;;
  baseline)
    for m in mnist_cnn mnist_bn_cnn; do
      step torch_${m}_graph 600 python bench/torch_baseline.py --model $m --steps 800 --warmup 64 --graph --dtype fp32
    done
    step torch_resnet18 600 python bench/torch_baseline.py --model resnet18 --steps 30 --warmup 5 --channels-last ;;
  final)
    step pytest_gpu 1100 $PYT tests -m gpu
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
    step bench 300 python bench.py --steps 2000 --warmup 200
    for i in 1 2 3 4 5; do step bench_driver_$i 200 python bench.py --steps 20 --warmup 5; done
    step bench_wide 300 python bench.py --model mnist_cnn_wide --steps 2000 --warmup 200
    step bench_bn_cnn 300 python bench.py --model mnist_bn_cnn --steps 800 --warmup 64
    step bench_lenet5 300 python bench.py --model lenet5 --steps 800 --warmup 64
    step bench_mlp 300 python bench.py --model mnist_mlp --steps 2000 --warmup 64
    step bench_resnet18 300 python bench.py --model resnet18 --steps 30 --warmup 5 ;;
  stats)
    stat mnist_cnn python3 bench.py --steps 2000 --warmup 200 --repeats 0
    stat mnist_bn_cnn python3 bench.py --model mnist_bn_cnn --steps 800 --warmup 64 --repeats 0
    stat resnet18 python3 bench.py --model resnet18 --steps 30 --warmup 5 --repeats 0
    stat ps_exchange python3 bench/ps_exchange_micro.py ;;
  layers)
    step resnet_layers 400 python -u bench/resnet_layers.py "$@" ;;
  ps)
    export OMP_NUM_THREADS=2 TDE_HEARTBEAT=0
    step pytest_ps 600 python -u -m pytest tests/test_ps_device_gpu.py -q -rf --timeout 250 --timeout-method thread
    for plane in tcp device; do
      for nps in 1 2; do
        E=""
        [ $plane = device ] && E="TDE_PS_DEVICE=1"
        step b_${plane}_ps$nps 200 env $E python -m tensorflow_distributed_example_amd.launch --ps $nps --master 1 \
          --workers 1 --timeout 150 bench/ps_throughput.py --max-steps 4000 --warm 300
      done
    done ;;
  pytest)
    step pytest 900 $PYT "$@" ;;
  micro)
    step micro 300 python bench/micro.py ;;
  *)
    echo "unknown mode $MODE"; exit 2 ;;
esac
echo "=== done"
