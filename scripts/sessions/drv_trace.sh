#!/bin/bash
# Kernel timeline of the driver-length headline run (bench.py --steps 20 --warmup 5): where the ~30 us of
# per-run overhead sits (staging, graph start, the flush, the tail).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/drv_trace; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o drv -- python3 bench.py --steps 20 --warmup 5 --repeats 2 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 3; }
grep -h '"metric"' $O/run.log | grep -o '"ms_per_step": [0-9.]*'
find $O/prof -name "*kernel_trace.csv" | head -3
