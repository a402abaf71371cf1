"""The fused per-image small-net plan (csrc/kernels/smallnet.hip, train/smallnet.py) vs the torch fp32
reference plan: per-variable gradients, metrics, eval and predict, the in-step optimizer ("local")
against the separate optimizer ("plain"), and fit() end to end (BASELINE.json config 2, LeNet-5).

Both sides compute in fp32, so the bounds are tight (reduction order only).  The reference runs on the
CPU (plain PyTorch fp32 ops, no GPU library in the oracle)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _models(tde):
    K = tde.keras.layers
    odd = tde.Sequential([   # same-padded bias-free conv + Activation layer, a pool over odd sizes,
        K.Conv2D(8, 3, padding="same", use_bias=False, input_shape=(15, 13, 2)),   # a conv feeding Dense
        K.Activation("relu"),
        K.MaxPooling2D(),
        K.Conv2D(12, 2, activation="relu"),
        K.Flatten(),
        K.Dense(33, activation="relu"),
        K.Dense(7, activation="softmax"),
    ], name="odd")
    narrow = tde.Sequential([K.Conv2D(5, 3, activation="relu", input_shape=(12, 12, 3)), K.MaxPooling2D(),
                             K.Flatten(), K.Dense(10)], name="narrow")
    return {"lenet5": (tde.zoo.lenet5(), True), "mnist_mlp": (tde.zoo.mnist_mlp(), True), "odd": (odd, False),
            "narrow": (narrow, True)}


def _build(tde, name, opt=None):
    m, logits = _models(tde)[name]
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=logits),
              optimizer=opt or tde.optimizers.SGD(0.01), metrics=["accuracy"])
    m.build()
    return m


def _data(m, n, seed):
    rng = np.random.default_rng(seed)
    shp = tuple(m.input_shape[1:])
    ncls = m.output_shape[-1]
    x = torch.from_numpy(rng.standard_normal((n,) + shp).astype(np.float32)).cuda()
    y = torch.from_numpy(rng.integers(0, ncls, n).astype(np.int32)).cuda()
    return x, y


def _rel(a, b):
    return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


@pytest.mark.parametrize("name", ["lenet5", "mnist_mlp", "odd", "narrow"])
@pytest.mark.parametrize("B,Bplan", [(128, 128), (37, 64)])
def test_smallnet_gradients_match_fp32_reference(name, B, Bplan):
    import tensorflow_distributed_example_amd as tde
    from tensorflow_distributed_example_amd.train import program as PG
    tde.backend.set_random_seed(1)
    m = _build(tde, name)
    st = m._store
    st_ref = st.clone_to("cpu")
    plan = PG.make_plan(m, st, "cuda", Bplan, Bplan, m.optimizer, m.loss)
    ref = PG.ReferencePlan(m, st_ref, "cpu", Bplan, Bplan, m.optimizer, m.loss)
    assert plan.kind == "fused_smallnet"
    x, y = _data(m, Bplan, 3)
    plan.train_step(x, y, B)
    torch.cuda.synchronize()
    ref.train_step(x.cpu(), y.long().cpu(), B)
    for n in st.names(trainable=True):
        r = _rel(st.grad(n).cpu(), st_ref.grad(n))
        assert r < 1e-4, (n, r)
    mf, mr = plan.metrics.cpu(), ref.metrics.cpu()
    assert abs(mf[0] - mr[0]) < 1e-4 * abs(mr[0]) and mf[1] == mr[1] and mf[2] == mr[2] == B
    assert plan.iterations.item() == 1


@pytest.mark.parametrize("name", ["lenet5", "odd"])
def test_smallnet_eval_and_predict_match_reference(name):
    import tensorflow_distributed_example_amd as tde
    from tensorflow_distributed_example_amd.train import program as PG
    tde.backend.set_random_seed(2)
    m = _build(tde, name)
    plan = PG.make_plan(m, m._store, "cuda", 50, 50, None, m.loss)
    ref = PG.ReferencePlan(m, m._store.clone_to("cpu"), "cpu", 50, 50, None, m.loss)
    x, y = _data(m, 50, 4)
    plan.eval_step(x, y, 50)
    p = plan.predict(x, 41).clone()
    torch.cuda.synchronize()
    ref.eval_step(x.cpu(), y.long().cpu(), 50)
    pr = ref.predict(x.cpu(), 41)
    assert _rel(p.cpu(), pr) < 1e-5
    mf, mr = plan.metrics.cpu(), ref.metrics.cpu()
    assert abs(mf[0] - mr[0]) < 1e-4 * abs(mr[0]) and mf[1] == mr[1] and mf[2] == mr[2]


@pytest.mark.parametrize("opt", ["sgd", "momentum", "adam"])
def test_smallnet_local_step_matches_plain(opt):
    """Step mode "local" (the optimizer applied where each gradient is finished) vs "plain" (gradients
    to the bucket + the multi-tensor optimizer kernel), three steps."""
    import tensorflow_distributed_example_amd as tde
    from tensorflow_distributed_example_amd.train import program as PG

    def mk():
        return {"sgd": tde.optimizers.SGD(0.05), "momentum": tde.optimizers.SGD(0.05, momentum=0.9),
                "adam": tde.optimizers.Adam(1e-3)}[opt]
    tde.backend.set_random_seed(3)
    m = _build(tde, "lenet5", mk())
    st = m._store
    st2 = st.clone_to("cuda")
    w0 = st.w.clone()
    a = PG.make_plan(m, st, "cuda", 64, 64, m.optimizer, m.loss)
    b = PG.make_plan(m, st2, "cuda", 64, 64, mk(), m.loss)
    a.set_step_mode("local")
    for s in range(3):
        x, y = _data(m, 64, 10 + s)
        a.train_step(x, y)
        b.train_step(x, y)
        b.apply()
    torch.cuda.synchronize()
    for n in st.names(trainable=True):
        sg = st.segments[n]
        w = w0[sg.offset: sg.offset + sg.numel].view(sg.shape)
        r = _rel(st.view(n) - w, st2.view(n) - w)    # the accumulated updates
        assert r < 1e-5, (n, r)
    assert a.iterations.item() == b.iterations.item() == 3


def test_smallnet_fit_lenet5():
    """fit() on LeNet-5 picks the fused small-net plan (hipGraph executions, the in-step optimizer) and
    learns a separable synthetic task."""
    import tensorflow_distributed_example_amd as tde
    tde.backend.set_random_seed(4)
    m = tde.zoo.lenet5()
    m.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=tde.optimizers.SGD(0.05),
              metrics=["accuracy"], steps_per_execution=4)
    rng = np.random.default_rng(0)
    y = rng.integers(0, 10, 2048)
    x = rng.random((2048, 28, 28, 1), dtype=np.float32) * 0.2
    for c in range(10):   # class c lights up row band c
        x[y == c, 2 * c + 4: 2 * c + 6, 4:24, 0] += 1.0
    h = m.fit(x, y, batch_size=128, epochs=3, verbose=0)
    prog = m._program("train", 128)
    assert prog.plan_kind == "fused_smallnet" and prog.use_graph
    assert prog.plans[0].step_mode == "local"
    assert h.history["loss"][-1] < 0.5 * h.history["loss"][0]
    assert h.history["accuracy"][-1] > 0.9
    ev = m.evaluate(x[:512], y[:512], batch_size=128, verbose=0, return_dict=True)
    assert ev["accuracy"] > 0.9
