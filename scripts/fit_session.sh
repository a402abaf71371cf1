#!/bin/bash
# GPU tests + smoke + end-to-end fit() throughput (bench/fit_pipeline.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD" TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python bench/fit_pipeline.py > $O/fit.log 2>&1 || { tail -20 $O/fit.log; exit 1; }
cat $O/fit.log
