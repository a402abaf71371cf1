set -e
mkdir -p gpurun_out
: > gpurun_out/ab.log
for m in mnist_bn_cnn lenet5 mnist_mlp; do
  for t in 512 2048; do
    echo "model=$m tile_min=$t $(TDE_IGEMM_TILE_MIN=$t timeout -k 10 120 python -u bench.py --model $m --steps 300 --warmup 30 2>/dev/null | tail -n1 | cut -c1-200)" >> gpurun_out/ab.log
  done
done
for t in 512 2048 512 2048; do
  echo "model=resnet18 tile_min=$t $(TDE_IGEMM_TILE_MIN=$t timeout -k 10 150 python -u bench.py --model resnet18 --steps 40 --warmup 5 2>/dev/null | tail -n1 | cut -c1-200)" >> gpurun_out/ab.log
done
