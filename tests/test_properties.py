"""Property-based tests (hypothesis) of the host-side semantics — SURVEY.md §4.2 T0/T2:

* TF 'SAME' padding and the Conv2D reference path (the CPU backend's kernel library and the GPU
  numerics oracle) against an independent numpy direct convolution, over random geometries including
  the asymmetric TF pads;
* crc32c (native) against a bitwise pure-Python Castagnoli CRC;
* TensorBundle checkpoints and TFRecord event files round-tripped through the native writers;
* tf.data pipeline algebra (shuffle is a permutation, batch / repeat / take / skip / shard counts);
* TF_CONFIG <-> CLUSTER_SPEC/TASK_INDEX/JOB_NAME translation and the session device filters.

The GPU counterpart (random conv geometries through the HIP implicit-GEMM kernels) is
tests/test_layers_gpu.py::test_conv_kernels_random_geometries.
"""
import json

import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from tensorflow_distributed_example_amd import _native as N
from tensorflow_distributed_example_amd.data import dataset as D
from tensorflow_distributed_example_amd.io import events as EV
from tensorflow_distributed_example_amd.io import tensor_bundle as TB
from tensorflow_distributed_example_amd.models import layers as L
from tensorflow_distributed_example_amd.parallel import cluster as CL

FAST = settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow,
                                                                       HealthCheck.function_scoped_fixture])


# ------------------------------------------------------------------ padding / conv reference
def _np_conv_same_or_valid(x, w, s, padding):
    """Direct NHWC x HWIO convolution in float64 with TF padding semantics."""
    B, H, W, C = x.shape
    kh, kw, _, Co = w.shape
    if padding == "same":
        Ho, Wo = -(-H // s), -(-W // s)
        pt = max((Ho - 1) * s + kh - H, 0) // 2
        pl = max((Wo - 1) * s + kw - W, 0) // 2
    else:
        Ho, Wo = (H - kh) // s + 1, (W - kw) // s + 1
        pt = pl = 0
    y = np.zeros((B, Ho, Wo, Co))
    for oh in range(Ho):
        for ow in range(Wo):
            for i in range(kh):
                for j in range(kw):
                    ih, iw = oh * s - pt + i, ow * s - pl + j
                    if 0 <= ih < H and 0 <= iw < W:
                        y[:, oh, ow, :] += x[:, ih, iw, :] @ w[i, j]
    return y


@FAST
@given(n=st.integers(1, 64), k=st.integers(1, 9), s=st.integers(1, 4))
def test_tf_same_pads_formula(n, k, s):
    pb, pa = L.tf_same_pads(n, k, s)
    out = -(-n // s)
    assert pb + pa == max((out - 1) * s + k - n, 0) and pb == (pb + pa) // 2 and pa - pb in (0, 1)
    # every output window starts inside the padded input and ends inside it
    assert (out - 1) * s + k <= n + pb + pa


@FAST
@given(B=st.integers(1, 2), H=st.integers(3, 9), W=st.integers(3, 9), C=st.integers(1, 3),
       Co=st.integers(1, 4), k=st.integers(1, 4), s=st.integers(1, 3), padding=st.sampled_from(["same", "valid"]),
       seed=st.integers(0, 2 ** 16))
def test_conv2d_reference_matches_direct_convolution(B, H, W, C, Co, k, s, padding, seed):
    if padding == "valid" and (k > H or k > W):
        return
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((B, H, W, C))
    w = rng.standard_normal((k, k, C, Co))
    layer = L.Conv2D(Co, k, strides=s, padding=padding)
    assert layer.compute_output_shape((H, W, C))[:2] == _np_conv_same_or_valid(x[:1], w, s, padding).shape[1:3]
    layer.input_shape = (H, W, C)
    y = layer.ref_call(torch.from_numpy(x), {"kernel": torch.from_numpy(w)}, True)
    np.testing.assert_allclose(y.numpy(), _np_conv_same_or_valid(x, w, s, padding), rtol=1e-10, atol=1e-10)


# ------------------------------------------------------------------ crc32c
def _crc32c_py(data: bytes) -> int:
    crc = 0xFFFFFFFF
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (0x82F63B78 if crc & 1 else 0)
    return crc ^ 0xFFFFFFFF


@FAST
@given(data=st.binary(max_size=300))
def test_crc32c_matches_bitwise_reference(data):
    lib = N.host()
    c = lib.tde_crc32c(data, len(data))
    assert c == _crc32c_py(data)
    assert lib.tde_crc32c_unmask(lib.tde_crc32c_mask(c)) == c


# ------------------------------------------------------------------ TensorBundle / events
_names = st.text(alphabet="abcdefghijklmnopqrstuvwxyz_/0123456789", min_size=1, max_size=24)
_dtypes = st.sampled_from([np.float32, np.float64, np.int32, np.int64, np.uint8, np.float16])
_shapes = st.lists(st.integers(0, 5), min_size=0, max_size=4).map(tuple)
_f32 = st.floats(width=32, allow_nan=False, allow_infinity=False)


@FAST
@given(tensors=st.dictionaries(_names, st.tuples(_dtypes, _shapes, st.integers(0, 2 ** 16)), min_size=1,
                               max_size=8))
def test_tensor_bundle_roundtrip(tmp_path_factory, tensors):
    arrs = {}
    for name, (dt, shape, seed) in tensors.items():
        rng = np.random.default_rng(seed)
        arrs[name] = (rng.standard_normal(shape) * 100).astype(dt)
    prefix = str(tmp_path_factory.mktemp("tb") / "model.ckpt-1")
    TB.write_bundle(prefix, arrs)
    back = TB.read_bundle(prefix)
    assert sorted(back) == sorted(arrs)
    for k, a in arrs.items():
        assert back[k].dtype == a.dtype and back[k].shape == a.shape and np.array_equal(back[k], a)
    listed = [n for n, *_ in TB.list_variables(prefix)]
    assert listed == sorted(listed)   # SSTable keys are sorted


@FAST
@given(steps=st.lists(st.tuples(st.integers(0, 10 ** 9),
                                st.dictionaries(_names, _f32, min_size=1, max_size=4)),
                      min_size=1, max_size=6))
def test_event_file_roundtrip(tmp_path_factory, steps):
    w = EV.EventFileWriter(tmp_path_factory.mktemp("ev"))
    for step, vals in steps:
        w.add_scalars(step, vals)
    w.close()
    evs = EV.read_events(w.path)
    assert evs[0].get("file_version") == "brain.Event:2"
    got = [(e["step"], e["scalars"]) for e in evs[1:]]
    assert got == [(s, {k: float(np.float32(v)) for k, v in vals.items()}) for s, vals in steps]


# ------------------------------------------------------------------ tf.data algebra
def _flat(ds):
    out = []
    for b in ds:
        out.extend(np.asarray(b).reshape(-1).tolist())
    return out


@FAST
@given(n=st.integers(1, 200), buf=st.integers(1, 300), bs=st.integers(1, 40), seed=st.integers(0, 1000),
       drop=st.booleans())
def test_shuffle_batch_is_a_permutation(n, buf, bs, seed, drop):
    ds = D.Dataset.from_tensor_slices(np.arange(n)).shuffle(buf, seed=seed).batch(bs, drop_remainder=drop)
    batches = [np.asarray(b) for b in ds]
    sizes = [len(b) for b in batches]
    if drop:
        assert sizes == [bs] * (n // bs)
    else:
        assert sizes == [bs] * (n // bs) + ([n % bs] if n % bs else [])
    vals = _flat(batches)
    assert len(set(vals)) == len(vals) and set(vals) <= set(range(n))
    if not drop:
        assert sorted(vals) == list(range(n))


@FAST
@given(n=st.integers(1, 60), reps=st.integers(1, 4), take=st.integers(0, 300), skip=st.integers(0, 300))
def test_repeat_take_skip_counts(n, reps, take, skip):
    base = D.Dataset.from_tensor_slices(np.arange(n))
    rep = _flat(base.repeat(reps))
    assert rep == list(range(n)) * reps
    assert _flat(base.repeat(reps).skip(skip).take(take)) == rep[skip:][:take]


@FAST
@given(n=st.integers(1, 100), shards=st.integers(1, 8))
def test_shards_partition_the_data(n, shards):
    base = D.Dataset.from_tensor_slices(np.arange(n))
    parts = [_flat(base.shard(shards, i)) for i in range(shards)]
    assert sorted(sum(parts, [])) == list(range(n))
    assert all(p == list(range(i, n, shards)) for i, p in enumerate(parts))


# ------------------------------------------------------------------ cluster config
_addr = st.builds(lambda h, p: f"{h}:{p}", st.sampled_from(["localhost", "127.0.0.1", "node-a", "node-b"]),
                  st.integers(1024, 65535))


@FAST
@given(jobs=st.fixed_dictionaries({"ps": st.lists(_addr, min_size=0, max_size=3),
                                   "worker": st.lists(_addr, min_size=1, max_size=4)},
                                  optional={"master": st.lists(_addr, min_size=1, max_size=1)}),
       data=st.data())
def test_launcher_env_translation_and_device_filters(jobs, data):
    jobs = {k: v for k, v in jobs.items() if v}
    job = data.draw(st.sampled_from(sorted(jobs)))
    idx = data.draw(st.integers(0, len(jobs[job]) - 1))
    env = {"CLUSTER_SPEC": json.dumps(jobs), "TASK_INDEX": str(idx), "JOB_NAME": job}
    assert CL.translate_launcher_env(env, verbose=False)
    cfg = json.loads(env["TF_CONFIG"])
    assert cfg == {"cluster": jobs, "task": {"type": job, "index": idx}}
    r = CL.TFConfigClusterResolver(env)
    assert r.cluster_spec() == CL.ClusterSpec(jobs) and r.task_type == job and r.task_id == idx
    f = CL.device_filters(env)
    if job == "master":
        assert f == ["/job:ps", "/job:master"]
    elif job == "worker":
        assert f == ["/job:ps", f"/job:worker/task:{idx}"]
        # a worker never talks to another worker (async PS isolation, MKD:176-188)
        others = [i for i in range(len(jobs["worker"])) if i != idx]
        assert all(not CL.filter_allows(f, "worker", i) for i in others)
        assert CL.filter_allows(f, "ps", 0)
    else:
        assert f is None


if __name__ == "__main__":
    raise SystemExit(pytest.main([__file__, "-q"]))
