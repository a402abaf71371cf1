#!/bin/bash
# ResNet-18 stem BN + max-pool backward with the input row's y loads batched with dy / argmax vs the previous
# build (TDE_HIP_LIB=libtde_hip_base.so): layer GPU tests, kernel statistics of both, alternating benches.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/bnpool_ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_layers_gpu.py -x -q -rf --capture=sys --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log
[ $rc -ne 0 ] && { tail -30 $O/pytest.log; exit 3; }
for lib in libtde_hip_base.so libtde_hip.so; do
  TDE_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$lib -o rn -- python3 bench.py --model resnet18 --steps 20 --warmup 5 --repeats 0 > $O/prof_$lib.log 2>&1 || exit $?
  f=$(find $O/prof_$lib -name "*kernel_stats.csv" | head -1); grep -h "bn_pool_bwd\|bn_relu_maxpool" "$f" | cut -d, -f1-4
done
for i in 1 2; do
  for lib in libtde_hip_base.so libtde_hip.so; do
    TDE_HIP_LIB=$lib timeout -k 10 300 python bench.py --model resnet18 --steps 30 --warmup 5 > $O/rn_${lib}_$i.log 2>&1 || exit $?
    echo "$lib $(grep -h '"metric"' $O/rn_${lib}_$i.log | grep -o '"value": [0-9.]*')"
  done
done
