"""CPU checks of the layer-wise plan's fusion rules (which geometries the fused kernels take)."""
import pytest

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


@pytest.mark.parametrize("which", ["mini_resnet", "model_a_wide", "model_b_doubled"])
def test_float32_layerwise_oracle_matches_reference_executor(which):
    """CPU: the float32 layer-wise plan compiles its stage graph without any bf16 buffer or weight shadow,
    and the float64 oracle that the GPU tests compare its kernels against (train/layerwise.emulate_step,
    nothing rounded under float32) equals the torch reference executor's gradients for the same model —
    so a GPU mismatch can only come from the kernels."""
    import numpy as np
    import torch

    import tensorflow_distributed_example_amd as tde
    from tensorflow_distributed_example_amd.train import program as PG
    from tensorflow_distributed_example_amd.train.layerwise import LayerwisePlan, emulate_step
    tde.backend.set_global_policy("float32")
    try:
        tde.backend.set_random_seed(2)
        L = tde.keras.layers
        if which == "mini_resnet":
            m = tde.zoo.resnet((1, 1), (8, 16), input_shape=(16, 16, 3), classes=10, name="mini_resnet")
            loss = tde.losses.SparseCategoricalCrossentropy(from_logits=True)
        elif which == "model_a_wide":
            m = tde.Sequential([L.Conv2D(64, 3, activation="relu", input_shape=(28, 28, 1)), L.MaxPooling2D(),
                                L.Flatten(), L.Dense(128, activation="relu"), L.Dense(10)])
            loss = tde.losses.SparseCategoricalCrossentropy(from_logits=True)
        else:
            m = tde.Sequential([
                L.Reshape(input_shape=(784,), target_shape=(28, 28, 1)),
                L.Conv2D(12, 3, padding="same", use_bias=False), L.BatchNormalization(scale=False), L.Activation("relu"),
                L.Conv2D(24, 6, padding="same", use_bias=False, strides=2), L.BatchNormalization(scale=False),
                L.Activation("relu"),
                L.Flatten(), L.Dense(400, use_bias=False), L.BatchNormalization(scale=False), L.Activation("relu"),
                L.Dropout(0.0), L.Dense(10, activation="softmax")])
            loss = "sparse_categorical_crossentropy"
        m.compile(loss=loss, optimizer=tde.optimizers.SGD(0.01))
        m.build()
        B = 8
        plan = LayerwisePlan(m, m._store, "cpu", B, B, m.optimizer, m.loss)
        assert plan.f32 and plan.compute_dtype == "fp32" and not plan.shadows
        assert all(t.buf is None or t.buf.dtype == torch.float32 for t in plan.T.values())
        rng = np.random.default_rng(3)
        x = torch.from_numpy(rng.standard_normal((B,) + tuple(m.input_shape[1:])).astype(np.float32))
        y = torch.from_numpy(rng.integers(0, 10, B)).int()
        want, _ = emulate_step(plan, x, y)
        ref = PG.ReferencePlan(m, m._store, "cpu", B, B, m.optimizer, m.loss)
        ref.train_step(x, y)
        st = m._store
        for n in st.names(trainable=True):
            g = st.grad(n).double()
            rel = float((g - want[n]).norm() / (want[n].norm() + 1e-30))
            assert rel < 1e-5, (which, n, rel)
    finally:
        tde.backend.set_global_policy(None)
