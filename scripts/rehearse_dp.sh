#!/bin/bash
# 2-replica MirroredStrategy rehearsal on one GPU (both replicas on cuda:0, the in-process xGMI exchange):
# ms/step of the headline MNIST CNN and Model B, alternating rounds.  bash scripts/rehearse_dp.sh [rounds]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/rehearse; mkdir -p $O
for r in $(seq 1 ${1:-2}); do
  for m in mnist_cnn mnist_bn_cnn; do
    timeout -k 10 200 python bench.py --strategy mirrored --devices 0,0 --model $m --steps 800 --warmup 64 \
      --repeats 2 > $O/${m}_$r.log 2>&1 || exit $?
    echo "$m round $r: $(grep -o '"ms_per_step": [0-9.]*' $O/${m}_$r.log) $(grep -o '"repeat_ms_per_step": [^]]*' $O/${m}_$r.log)"
  done
done
