#!/bin/bash
# Model B fused step: the first layer's backward updates its own variables (last-arrival workgroup) and the
# other layers' reduce runs on a side stream, vs the separate reduce launch (TDE_BNCNN_FIN=0): BN-CNN GPU
# tests, then alternating benches, then phase clocks of both forms.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/bn_fin; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bncnn_gpu.py -x -v -rf --capture=sys --timeout 120 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -3 $O/pytest.log
# TDE_BNCNN_FIN: 0 separate reduce launch, 1 last-arrival update + reduce before the launch, 2 + side stream
for i in 1 2; do
  for f in 0 1 2; do
    TDE_BNCNN_FIN=$f timeout -k 10 300 python bench.py --model mnist_bn_cnn --steps 800 --warmup 64 > $O/fin${f}_$i.log 2>&1 || exit $?
    echo "fin=$f $(tail -1 $O/fin${f}_$i.log | cut -c1-200)"
  done
done
for f in 0 1 2; do
  TDE_BNCNN_FIN=$f timeout -k 10 300 python bench/bncnn_phases.py > $O/phases_fin$f.log 2>&1 || exit $?
  echo "fin=$f"; tail -3 $O/phases_fin$f.log | cut -c1-400
done
