"""CPU checks of the layer-wise plan's fusion rules (which geometries the fused kernels take)."""
from tensorflow_distributed_example_amd.ops import layer_ops as O


def test_bn_pool_fusion_geometries():
    G = O.ConvGeom
    assert O.bn_pool_ok(G(64, 112, 112, 64, 56, 56, 64, 3, 3, 2, 2, 0, 0))      # the ResNet stem
    assert O.bn_pool_ok(G(8, 16, 16, 32, 8, 8, 32, 2, 2, 2, 2, 0, 0))           # 2x2/2
    assert not O.bn_pool_ok(G(8, 16, 16, 1024, 8, 8, 1024, 3, 3, 2, 2, 0, 0))   # > 512 channels
    assert not O.bn_pool_ok(G(8, 16, 16, 6, 8, 8, 6, 3, 3, 2, 2, 0, 0))         # not 8-channel vectors
    assert not O.bn_pool_ok(G(8, 16, 16, 96, 8, 8, 96, 3, 3, 2, 2, 0, 0))       # 256 % 12 != 0
    assert not O.bn_pool_ok(G(8, 16, 16, 64, 14, 14, 64, 3, 3, 1, 1, 1, 1))     # 3x3/1: 3 windows per pixel
    assert not O.bn_pool_ok(G(8, 200, 200, 64, 100, 100, 64, 2, 2, 2, 2, 0, 0))  # pooled row > 4096 elements
