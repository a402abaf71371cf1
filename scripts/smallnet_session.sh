#!/bin/bash
# Small-net plan on one GPU: tests, LeNet-5 / MLP bench, kernel-trace profile of LeNet-5.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}" TMPDIR=/tmp
OUT=gpurun_out/sn
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_smallnet_gpu.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 120 python bench.py --model lenet5 --steps 800 --warmup 64 > $OUT/lenet5.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --model mnist_mlp --steps 800 --warmup 64 > $OUT/mlp.log 2>&1 || exit 1
grep -h '^{' $OUT/lenet5.log $OUT/mlp.log | python -c "import sys,json; [print(j['config']['model'], j['value'], j['ms_per_step']) for j in map(json.loads, sys.stdin)]"
timeout -k 10 100 python bench/smallnet_phases.py || exit 1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/prof -o lenet -- python $GRAFT_REPO_ROOT/bench.py --model lenet5 --steps 400 --warmup 32 > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python scripts/rocpd_stats.py $OUT/prof/lenet_results.db --last 800 | cut -c1-120
