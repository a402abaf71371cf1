#!/bin/bash
# rocprofv3 counter passes over bench/halo_probe.py (the halo-tile conv, stage-1 geometry): instruction mix,
# LDS bank conflicts, MFMA busy cycles, wait breakdown.  One counter group per pass, counters only.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmch_${1:-fwd}_$i -o run -- python bench/halo_probe.py ${1:-fwd} > gpurun_out/pmch_${1:-fwd}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmch_${1:-fwd}_$i.log; exit 1; }
done
echo done
