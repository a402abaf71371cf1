#!/bin/bash
# GPU-box session driver: runs the named steps in order, each under its own time limit, logs under
# gpurun_out/<step>.log, and stops at the first step that ends in a fault / abort / timeout (exit
# codes other than 0 and 1: a failing test is 1 and the session goes on).
#   bash scripts/gpu_steps.sh <step> [<step> ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT" profiles
PYT="python -u -m pytest -x -q -rf --timeout 120 --timeout-method thread"
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 30 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
prof() {  # name timeout cmd... : rocprofv3 kernel statistics of a command
  local name=$1 t=$2; shift 2
  rm -rf "$OUT/prof_$name"
  step "prof_$name" "$t" rocprofv3 --kernel-trace --stats -d "$OUT/prof_$name" -o run --output-format csv -- "$@"
  local f
  f=$(find "$OUT/prof_$name" -name '*kernel_stats.csv' | head -n 1)
  [ -n "$f" ] && cp "$f" "$OUT/${name}_kernel_stats.csv"
  return 0
}
for s in "$@"; do
  case "$s" in
    t_fp32) step t_fp32 300 $PYT tests/test_fp32_gpu.py ;;
    t_bncnn) step t_bncnn 300 $PYT tests/test_bncnn_gpu.py ;;
    t_convnet) step t_convnet 400 $PYT tests/test_kernels_gpu.py tests/test_plan_gpu.py ;;
    t_all) step t_all 1000 $PYT tests -m gpu ;;
    t_xgmi) step t_xgmi 400 $PYT tests/test_xgmi_gpu.py ;;
    t_mirrored) step t_mirrored 500 $PYT tests/test_mirrored_gpu.py ;;
    t_layers) step t_layers 600 $PYT tests/test_layers_gpu.py ;;
    t_smallnet) step t_smallnet 300 $PYT tests/test_smallnet_gpu.py ;;
    t_examples) step t_examples 400 $PYT tests/test_examples_gpu.py ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    b_fp32_20) step b_fp32_20 200 python bench.py --steps 20 --warmup 5 ;;
    b_fp32) step b_fp32 300 python bench.py --steps 2000 --warmup 200 ;;
    b_bf16_20) step b_bf16_20 200 python bench.py --steps 20 --warmup 5 --dtype bf16 ;;
    b_bf16) step b_bf16 300 python bench.py --steps 2000 --warmup 200 --dtype bf16 ;;
    b_fp32_nograph) step b_fp32_nograph 300 python bench.py --steps 400 --warmup 64 --no-graph ;;
    b_bn_cnn) step b_bn_cnn 300 python bench.py --model mnist_bn_cnn --steps 800 --warmup 64 ;;
    b_bn_cnn_bf16) step b_bn_cnn_bf16 300 python bench.py --model mnist_bn_cnn --steps 800 --warmup 64 --dtype bf16 ;;
    b_lenet5) step b_lenet5 300 python bench.py --model lenet5 --steps 800 --warmup 64 ;;
    b_mlp) step b_mlp 300 python bench.py --model mnist_mlp --steps 800 --warmup 64 ;;
    b_lenet5_m3) step b_lenet5_m3 300 env TDE_SN_MFMA=3 python bench.py --model lenet5 --steps 800 --warmup 64 ;;
    b_lenet5_m7) step b_lenet5_m7 300 env TDE_SN_MFMA=7 python bench.py --model lenet5 --steps 800 --warmup 64 ;;
    t_smallnet_m7) step t_smallnet_m7 300 env TDE_SN_MFMA=7 $PYT tests/test_smallnet_gpu.py ;;
    b_lenet5_m0) step b_lenet5_m0 300 env TDE_SN_MFMA=0 python bench.py --model lenet5 --steps 800 --warmup 64 ;;
    b_ps) step b_ps 300 python -m tensorflow_distributed_example_amd.launch --ps 1 --master 1 --workers 1 --timeout 280 bench/ps_throughput.py --max-steps 3000 --warm 200 ;;
    b_ps_legacy) step b_ps_legacy 300 env TDE_PS_FLAT=0 python -m tensorflow_distributed_example_amd.launch --ps 1 --master 1 --workers 1 --timeout 280 bench/ps_throughput.py --max-steps 3000 --warm 200 ;;
    phases) step phases 150 python bench/bncnn_phases.py ;;
    micro) step micro 200 python bench/micro.py ;;
    snphases) step snphases 150 python bench/smallnet_phases.py ;;
    p_lenet5) prof lenet5 300 python3 bench.py --model lenet5 --steps 400 --warmup 64 ;;
    p_mlp) prof mlp 300 python3 bench.py --model mnist_mlp --steps 400 --warmup 64 ;;
    b_mirrored) step b_mirrored 300 env TDE_XGMI_TIMEOUT=30 python bench.py --strategy mirrored --devices 0,0 --steps 2000 --warmup 200 ;;
    b_resnet18) step b_resnet18 400 python bench.py --model resnet18 --steps 30 --warmup 5 ;;
    p_fp32) prof fp32 300 python3 bench.py --steps 400 --warmup 64 ;;
    p_bf16) prof bf16 300 python3 bench.py --steps 400 --warmup 64 --dtype bf16 ;;
    p_bn_cnn) prof bn_cnn 300 python3 bench.py --model mnist_bn_cnn --steps 400 --warmup 64 ;;
    p_resnet18) prof resnet18 400 python3 bench.py --model resnet18 --steps 20 --warmup 5 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== done"
