cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/sr
for i in 1 2 3; do timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/sr/bench_$i.log 2>&1 || exit $?; done
timeout -k 10 300 python bench/short_run.py > gpurun_out/sr/short_run.log 2>&1 || exit $?
for i in 4 5; do timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/sr/bench_$i.log 2>&1 || exit $?; done
grep -h '"value"' gpurun_out/sr/bench_*.log | cut -c1-200
tail -1 gpurun_out/sr/short_run.log
