#!/bin/bash
# Grid sweep of the streaming BN passes of the ResNet-18 layer-wise plan (TDE_BN_STREAM / TDE_BN_RED =
# "div,lo,hi"): rocprofv3 kernel statistics per configuration + the bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD" TMPDIR=/tmp
mkdir -p gpurun_out
i=0
while read -r stream red; do
  i=$((i+1))
  name=bn_sweep_$i
  echo "=== $name STREAM=$stream RED=$red"
  TDE_BN_STREAM=$stream TDE_BN_RED=$red timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/$name -o run -- python3 bench.py --model resnet18 --steps 20 --warmup 3 > gpurun_out/$name.log 2>&1
  rc=$?
  grep -o '"value": [0-9.]*' gpurun_out/$name.log
  if [ $rc -ne 0 ]; then echo "STOP rc=$rc"; exit $rc; fi
done <<LIST
16384,512,4096 32768,256,1024
16384,512,4096 8192,512,4096
16384,512,4096 4096,1024,8192
4096,1024,8192 32768,256,1024
8192,1024,8192 8192,512,4096
2048,2048,16384 4096,1024,8192
LIST
echo "=== done"
