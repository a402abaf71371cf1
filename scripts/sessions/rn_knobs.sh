#!/bin/bash
# ResNet-18 (bf16, B=64) re-sweep of the implicit-GEMM knobs on one box: one bench per setting.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONPATH=$PWD TMPDIR=/tmp; O=gpurun_out/rn_knobs; mkdir -p $O
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --model resnet18 --steps 30 --warmup 5 > $O/$name.log 2>&1 || exit $?
  echo "$name $(tail -1 $O/$name.log | grep -o '"ms_per_step": [0-9.]*')"
}
run default A=1
run wgdma1 TDE_WGRAD_DMA=1
run wgdma2 TDE_WGRAD_DMA=2
run bigdgrad TDE_IGEMM_BIG_DGRAD=1
run tilemin1024 TDE_IGEMM_TILE_MIN=1024
run tilemin4096 TDE_IGEMM_TILE_MIN=4096
run scratch32 TDE_WG_SCRATCH_MAX=32
run xcd0 TDE_XCD_SWIZZLE=0
run default2 A=2
