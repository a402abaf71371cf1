#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 100 python scripts/diag/dbg_pool.py > gpurun_out/dbg_pool.log 2>&1 || { tail gpurun_out/dbg_pool.log; exit 1; }
tail -6 gpurun_out/dbg_pool.log
bash scripts/stem_session.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stem -o run --output-format csv -- python bench.py --model resnet18 --steps 20 --warmup 3 > gpurun_out/prof_stem.log 2>&1
