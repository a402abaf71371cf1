#!/bin/bash
# Cross-process co-scheduling probe pairs (scripts/diag/xproc_probe.hip): two processes on one GPU whose
# grids wait for each other's flags; per grid size and number of extra streams per process.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
P=scripts/diag/xproc_probe
[ -x $P ] || { echo "build $P first"; exit 1; }
for extra in 0 4; do
  for blocks in 8 64 128 256 512; do
    d=$(mktemp -d /tmp/xprobe.XXXX)
    timeout -k 5 40 $P A $d $blocks $extra 2000 3 > gpurun_out/xprobe_A_${blocks}_${extra}.log 2>&1 &
    pa=$!
    timeout -k 5 40 $P B $d $blocks $extra 2000 3 > gpurun_out/xprobe_B_${blocks}_${extra}.log 2>&1
    rb=$?
    wait $pa
    ra=$?
    echo "=== blocks=$blocks extra_streams=$extra rcA=$ra rcB=$rb"
    cat gpurun_out/xprobe_A_${blocks}_${extra}.log gpurun_out/xprobe_B_${blocks}_${extra}.log
    rm -rf $d
    if [ $ra -ge 124 ] || [ $rb -ge 124 ]; then echo "STOP"; exit 1; fi
  done
done
echo "=== done"
