#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_layers_gpu.py -k "bn_relu_maxpool or stem or maxpool" > gpurun_out/stemtests.log 2>&1 || { tail -30 gpurun_out/stemtests.log; exit 1; }
tail -2 gpurun_out/stemtests.log
bash scripts/stem_session.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stem -o run --output-format csv -- python bench.py --model resnet18 --steps 20 --warmup 3 > gpurun_out/prof_stem.log 2>&1
