#!/bin/bash
# rocprofv3 hardware-counter runs (MFMA busy cycles, wait/active split, LDS bank conflicts) for the
# headline model and ResNet-18.  Counters only (no trace domains), one program per rocprofv3 call.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}" TMPDIR=/tmp
mkdir -p gpurun_out
PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 2 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
}
run pmc_list 120 rocprofv3 -L
run pmc_cnn 300 rocprofv3 --pmc $PMC --output-format csv -d gpurun_out/pmc_cnn -o run -- python bench.py --steps 64 --warmup 16
run pmc_rn 300 rocprofv3 --pmc $PMC --output-format csv -d gpurun_out/pmc_rn -o run -- python bench.py --model resnet18 --steps 4 --warmup 2
echo "=== done"
