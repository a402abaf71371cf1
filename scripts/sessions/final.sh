#!/bin/bash
# End-of-round validation on one box: the GPU test suite, smoke, the headline at 2,000 steps and at the
# driver's length in 5 fresh processes (the spread), and every benchmarked model.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/final; mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  tail -n 3 "$O/$name.log" | cut -c1-260
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
step pytest_gpu 1100 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py --steps 2000 --warmup 200
for i in 1 2 3 4 5; do step bench_driver_$i 200 python bench.py --steps 20 --warmup 5; done
step bench_wide 300 python bench.py --model mnist_cnn_wide --steps 2000 --warmup 200
step bench_bn_cnn 300 python bench.py --model mnist_bn_cnn --steps 800 --warmup 64
step bench_lenet5 300 python bench.py --model lenet5 --steps 800 --warmup 64
step bench_mlp 300 python bench.py --model mnist_mlp --steps 2000 --warmup 64
step bench_resnet18 300 python bench.py --model resnet18 --steps 30 --warmup 5
echo "=== done"
