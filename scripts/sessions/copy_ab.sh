#!/bin/bash
# copy_pairs with 4 units per thread (loads before stores) vs the previous build (TDE_HIP_LIB=libtde_hip_base.so):
# its GPU test, kernel time in the headline, alternating driver-length benches.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/copy_ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k copy_pairs --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
for lib in libtde_hip_base.so libtde_hip.so; do
  TDE_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$lib -o h -- python3 bench.py --steps 2000 --warmup 200 --repeats 0 > $O/p_$lib.log 2>&1 || exit $?
  echo "$lib $(grep -h copy_pairs $(find $O/p_$lib -name '*kernel_stats.csv') | cut -d, -f1-4)"
done
for i in 1 2 3; do
  for lib in libtde_hip_base.so libtde_hip.so; do
    TDE_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/d_${lib}_$i.log 2>&1 || exit $?
    echo "$lib $(grep -h '"metric"' $O/d_${lib}_$i.log | grep -o '"value": [0-9.]*')"
  done
done
