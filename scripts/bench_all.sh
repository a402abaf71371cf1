#!/bin/bash
# Every benchmark row of BASELINE.md on one MI355X (ours + the stock-PyTorch baselines), one JSON line each
# into gpurun_out/bench_all/<name>.log.  Stops at the first step that faults / aborts / times out.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/bench_all
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $OUT/$name.log | head -1)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
run cnn 200 python bench.py --steps 2000 --warmup 200
run cnn_driver 100 python bench.py --steps 20 --warmup 5
run cnn_nograph 200 python bench.py --steps 400 --warmup 64 --no-graph
run bn_cnn 200 python bench.py --model mnist_bn_cnn --steps 800 --warmup 64
run lenet5 200 python bench.py --model lenet5 --steps 800 --warmup 64
run mlp 200 python bench.py --model mnist_mlp --steps 800 --warmup 64
run resnet18 300 python bench.py --model resnet18 --steps 30 --warmup 5
run torch_cnn_graph 300 python bench/torch_baseline.py --model mnist_cnn --steps 2000 --warmup 64 --graph
run torch_bn_cnn_graph 300 python bench/torch_baseline.py --model mnist_bn_cnn --steps 800 --warmup 64 --graph
run fit_pipeline 300 python bench/fit_pipeline.py
