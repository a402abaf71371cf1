"""Which fused small-CNN step a DWK/TF2M-shaped model gets (train/program.py ``match_convnet``): the
hand-tuned Conv2D(32)/Dense(64) plan, the generic-width float32 plan, or a warning naming why neither fits
and the per-layer plan.  Pattern matching only: runs on the CPU."""
import warnings

import pytest


def _match(filters, units, policy, H=28, W=28, classes=10):
    import tensorflow_distributed_example_amd as tde
    from tensorflow_distributed_example_amd.models import layers as L
    from tensorflow_distributed_example_amd.train import program as PG
    tde.backend.set_global_policy(policy)
    try:
        m = tde.models.Sequential([
            L.Conv2D(filters, 3, activation="relu", input_shape=(H, W, 1)), L.MaxPooling2D(), L.Flatten(),
            L.Dense(units, activation="relu"), L.Dense(classes)])
        loss = tde.losses.SparseCategoricalCrossentropy(from_logits=True)
        with warnings.catch_warnings(record=True) as rec:
            warnings.simplefilter("always")
            pat = PG.match_convnet(m, loss)
        return pat, [str(w.message) for w in rec]
    finally:
        tde.backend.set_global_policy(None)


def test_reference_width_takes_the_hand_tuned_plan():
    for policy in ("float32", "mixed_bfloat16"):
        pat, warns = _match(32, 64, policy)
        assert pat is not None and not pat.get("generic") and not warns


@pytest.mark.parametrize("filters,units", [(64, 128), (16, 32), (48, 96), (32, 128), (64, 32), (32, 256), (16, 224),
                                           (48, 192), (64, 160)])
def test_generic_widths_take_the_generic_plan(filters, units):
    pat, warns = _match(filters, units, "float32")
    assert pat is not None and pat["generic"] and not warns


@pytest.mark.parametrize("filters,units,policy,H,W,classes,why", [
    (64, 128, "mixed_bfloat16", 28, 28, 10, "float32 policy"),
    (24, 64, "float32", 28, 28, 10, "filters must be one of"),
    (32, 288, "float32", 28, 28, 10, "multiple of 32 up to 256"),
    (64, 192, "float32", 28, 28, 10, "fits a CU's LDS"),
    (48, 224, "float32", 28, 28, 10, "fits a CU's LDS"),
    (64, 128, "float32", 28, 36, 10, "width a multiple of 4 up to 32"),
    (64, 128, "float32", 28, 28, 20, "at most 16 classes"),
])
def test_unfused_widths_warn_with_the_reason(filters, units, policy, H, W, classes, why):
    pat, warns = _match(filters, units, policy, H, W, classes)
    assert pat is None and len(warns) == 1 and why in warns[0] and "per-layer kernel plan" in warns[0], warns


def test_bncnn_family_near_miss_warns():
    """Model B (mnist_keras_distributed.py:79-109) matches the fused BN-CNN step silently; its doubled widths
    (48 filters, Dense(400)) fall back to the per-layer plan with a warning that names the limits."""
    import tensorflow_distributed_example_amd as tde
    from tensorflow_distributed_example_amd.train import bncnn
    for mult, fused in ((1, True), (2, False)):
        m = tde.zoo.mnist_bn_cnn(mult=mult)
        loss = tde.losses.SparseCategoricalCrossentropy()
        with warnings.catch_warnings(record=True) as rec:
            warnings.simplefilter("always")
            spec = bncnn.match_bncnn(m, loss)
        msgs = [str(w.message) for w in rec]
        if fused:
            assert spec is not None and not msgs, msgs
        else:
            assert spec is None and len(msgs) == 1 and "48 channels" in msgs[0] and "400 units" in msgs[0], msgs


def test_python_fit_rule_matches_the_kernel_family():
    """train/program.gen_fits mirrors the kernels' instantiation rule (csrc/kernels/convnet_gen.hip): 27 of
    the 32 (filters, units) pairs."""
    from tensorflow_distributed_example_amd.train import program as PG
    ok = {(f, u) for f in PG.GEN_FILTERS for u in PG.GEN_UNITS if PG.gen_fits(f, u)}
    assert len(ok) == 27 and (64, 160) in ok and (64, 192) not in ok and (48, 192) in ok and (48, 224) not in ok
