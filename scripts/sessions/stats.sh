#!/bin/bash
# rocprofv3 kernel statistics of the final tree: headline MNIST CNN, Model B, ResNet-18, the PS exchange micro.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/stats; mkdir -p $O
run() {  # name cmd...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o $n -- "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 3; }
  f=$(find $O/$n -name "*kernel_stats.csv" | head -1); cp "$f" $O/${n}_kernel_stats.csv; head -6 "$f" | cut -d, -f1-5
}
run mnist_cnn python3 bench.py --steps 2000 --warmup 200 --repeats 0
run mnist_bn_cnn python3 bench.py --model mnist_bn_cnn --steps 800 --warmup 64 --repeats 0
run resnet18 python3 bench.py --model resnet18 --steps 30 --warmup 5 --repeats 0
run ps_exchange python3 bench/ps_exchange_micro.py
