set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 400 --warmup 64 > gpurun_out/prof.log 2>&1 || exit $?
for m in mnist_bn_cnn lenet5 mnist_mlp; do timeout -k 10 200 python bench.py --model $m --steps 800 --warmup 64 > gpurun_out/bench_$m.log 2>&1 || exit $?; done
timeout -k 10 300 python bench.py --model resnet18 --steps 30 --warmup 5 > gpurun_out/bench_resnet18.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || exit $?
