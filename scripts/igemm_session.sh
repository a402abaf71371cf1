#!/bin/bash
# igemm change validation: layer/plan GPU numerics, then conv probe, per-layer ResNet-18 table, ResNet-18 bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/ig
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_layers_gpu.py tests/test_plan_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench/igemm_probe.py > $O/probe.log 2>&1 || exit $?
timeout -k 10 300 python bench/resnet_layers.py > $O/layers.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model resnet18 --steps 30 --warmup 5 > $O/resnet18.log 2>&1 || exit $?
cat $O/probe.log; tail -1 $O/layers.log; tail -1 $O/resnet18.log | cut -c1-200
