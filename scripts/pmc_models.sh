#!/bin/bash
# rocprofv3 hardware-counter passes over the fused fp32 plans (headline MNIST CNN, Model B BN-CNN,
# LeNet-5, MLP) and the bf16 ResNet-18.  Counters only (no trace domains); one program per
# rocprofv3 call, placed directly after `--`; every pass within the per-block limits
# (<= 8 SQ, <= 4 TCC: FETCH_SIZE and WRITE_SIZE in passes of their own).
#   scripts/pmc_models.sh [models...]     (default: mnist_cnn mnist_bn_cnn lenet5 mnist_mlp)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}" TMPDIR=/tmp
export TDE_BENCH_WARM_MS=0      # counters serialise dispatches: no time-based warm-up
mkdir -p gpurun_out
MODELS=${*:-"mnist_cnn mnist_bn_cnn lenet5 mnist_mlp"}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE"
P3="FETCH_SIZE GRBM_GUI_ACTIVE"
P4="WRITE_SIZE GRBM_GUI_ACTIVE"
for m in $MODELS; do
  steps=64; warm=16
  [ "$m" = resnet18 ] && { steps=2; warm=1; }
  i=0
  for set in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    name=pmc_${m}_p$i
    echo "=== $name ($(date +%T))"
    timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d gpurun_out/$name -o run -- \
      python3 bench.py --model "$m" --steps $steps --warmup $warm > gpurun_out/$name.log 2>&1
    rc=$?
    tail -n 1 gpurun_out/$name.log
    if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  done
done
echo "=== done"
