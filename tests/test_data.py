"""T2: tf.data-like pipeline semantics."""
import numpy as np
import pytest

import tensorflow_distributed_example_amd as tde
from tensorflow_distributed_example_amd.data import AutoShardPolicy, Dataset, Options
from tensorflow_distributed_example_amd.data.distributed import shard_pipeline


def test_from_tensor_slices_batch_and_cardinality():
    x = np.arange(10)
    ds = Dataset.from_tensor_slices((x, x * 2)).batch(4)
    bs = list(ds)
    assert [len(b[0]) for b in bs] == [4, 4, 2]
    assert ds.cardinality() == 3
    assert np.array_equal(bs[1][1], np.array([8, 10, 12, 14]))
    assert len(list(Dataset.from_tensor_slices(x).batch(4, drop_remainder=True))) == 2


def test_shuffle_is_permutation_and_seeded():
    x = np.arange(100)
    a = np.concatenate(list(Dataset.from_tensor_slices(x).shuffle(10, seed=1).batch(7)))
    b = np.concatenate(list(Dataset.from_tensor_slices(x).shuffle(10, seed=1).batch(7)))
    assert sorted(a.tolist()) == list(range(100))
    assert np.array_equal(a, b)
    assert not np.array_equal(a, x)
    # buffer semantics: element i can't be emitted before position i - buffer_size
    pos = {v: i for i, v in enumerate(a)}
    assert all(pos[v] >= v - 10 for v in range(100))


def test_repeat_take_skip_shard_map_cache():
    x = np.arange(6)
    assert list(Dataset.from_tensor_slices(x).repeat(2)) == list(range(6)) * 2
    assert list(Dataset.from_tensor_slices(x).repeat().take(8)) == [0, 1, 2, 3, 4, 5, 0, 1]
    assert list(Dataset.from_tensor_slices(x).skip(4)) == [4, 5]
    assert list(Dataset.from_tensor_slices(x).shard(2, 1)) == [1, 3, 5]
    calls = []

    def f(v):
        calls.append(v)
        return v * 10
    ds = Dataset.from_tensor_slices(x).map(f).cache()
    assert list(ds) == [0, 10, 20, 30, 40, 50]
    assert list(ds) == [0, 10, 20, 30, 40, 50]
    assert len(calls) == 6  # cached after the first pass


def test_map_tuple_and_prefetch():
    x = np.arange(20, dtype=np.float32)
    ds = Dataset.from_tensor_slices((x, x)).map(lambda a, b: (a / 2, b)).batch(5).prefetch(2)
    out = list(ds)
    assert len(out) == 4 and np.allclose(out[0][0], x[:5] / 2)


def test_options_autoshard_policy():
    ds = Dataset.from_tensor_slices(np.arange(8)).batch(4)
    assert ds.options().experimental_distribute.auto_shard_policy == AutoShardPolicy.AUTO
    o = Options()
    o.experimental_distribute.auto_shard_policy = AutoShardPolicy.OFF
    ds2 = ds.with_options(o)
    assert ds2.options().experimental_distribute.auto_shard_policy == AutoShardPolicy.OFF
    assert list(ds2)[0].tolist() == [0, 1, 2, 3]


def test_shard_pipeline_divides_batch():
    ds = Dataset.from_tensor_slices(np.arange(16)).batch(8)
    w0 = list(shard_pipeline(ds, 2, 0))
    w1 = list(shard_pipeline(ds, 2, 1))
    assert w0[0].tolist() == [0, 2, 4, 6] and w1[0].tolist() == [1, 3, 5, 7]


def test_mnist_synthetic_shapes():
    (xt, yt), (xe, ye) = tde.data.mnist.load_data()
    assert xt.shape == (60000, 28, 28) and xt.dtype == np.uint8
    assert xe.shape == (10000, 28, 28) and yt.shape == (60000,)
    assert set(np.unique(yt)) == set(range(10))


def _ref_ops(n, ops):
    """Plain-Python model of take/skip/shard/repeat over range(n)."""
    v = list(range(n))
    for op, *a in ops:
        if op == "shard":
            v = v[a[1]::a[0]]
        elif op == "skip":
            v = v[a[0]:]
        elif op == "take":
            v = v[:a[0]]
        elif op == "repeat":
            v = v * a[0]
    return v


@pytest.mark.parametrize("native", ["1", "0"])
def test_chunked_index_ops_across_chunk_boundaries(native, monkeypatch):
    """The index protocol runs in numpy chunks of 8192 (data/dataset.py _CHUNK): take/skip/shard/
    repeat and batching must not depend on where the chunk boundaries fall."""
    from tensorflow_distributed_example_amd.data import dataset as D
    monkeypatch.setattr(D, "_HOST", [])
    monkeypatch.setenv("TDE_NATIVE_DATA", native)
    n = 20011
    x = np.arange(n, dtype=np.int64)
    cases = [[("shard", 3, 1), ("skip", 5000), ("take", 4099)],
             [("skip", 8191), ("take", 8194)],
             [("repeat", 3), ("shard", 5, 4), ("skip", 7), ("take", 9000)],
             [("take", 0)], [("skip", 30000)]]
    for ops in cases:
        ds = Dataset.from_tensor_slices(x)
        for op, *a in ops:
            ds = getattr(ds, op)(*a)
        want = _ref_ops(n, ops)
        got = np.concatenate(list(ds.batch(1000))).tolist() if want else list(ds.batch(1000))
        assert got == want, ops


def test_native_shuffle_buffer_semantics_large():
    """Native shuffle buffer (csrc/data/pipeline.cpp): a permutation per epoch, seeded replay,
    reshuffled across repeat() epochs, and TF's locality bound (out position >= in position - buffer)."""
    from tensorflow_distributed_example_amd.data import dataset as D
    assert D._host_lib() is not None, "libtde_host.so pipeline engine missing"
    n, buf = 30000, 1000
    x = np.arange(n)
    ds = Dataset.from_tensor_slices(x).shuffle(buf, seed=7).repeat(2).batch(512)
    out = np.concatenate(list(ds))
    e0, e1 = out[:n], out[n:]
    assert sorted(e0.tolist()) == list(range(n)) and sorted(e1.tolist()) == list(range(n))
    assert not np.array_equal(e0, e1)
    pos = np.empty(n, np.int64)
    pos[e0] = np.arange(n)
    assert np.all(pos >= np.arange(n) - buf)
    again = np.concatenate(list(Dataset.from_tensor_slices(x).shuffle(buf, seed=7).repeat(2).batch(512)))
    assert np.array_equal(out, again)


def test_native_gather_matches_numpy_for_all_column_kinds():
    imgs = np.random.default_rng(0).random((3000, 28, 28, 1)).astype(np.float32)
    lab = np.arange(3000, dtype=np.int64)
    strided = np.arange(6000, dtype=np.int32)[::2]          # not contiguous: numpy take path
    ds = Dataset.from_tensor_slices((imgs, lab, strided)).shuffle(500, seed=3).batch(128)
    for bi, bl, bs in ds:
        assert np.array_equal(bi, imgs[bl]) and np.array_equal(bs, strided[bl])
        assert bi.dtype == np.float32 and bs.dtype == np.int32


@pytest.mark.parametrize("policy,workers,widx", [(None, 1, 0), (AutoShardPolicy.OFF, 2, 1),
                                                 (AutoShardPolicy.DATA, 2, 1)])
def test_device_source_index_stream_matches_iteration(policy, workers, widx):
    """The device feed (train/device_feed.py) gathers rows on the GPU from DistributedDataset.device_source's
    per-replica index stream: it must select exactly the rows iterating the dataset yields."""
    from types import SimpleNamespace
    from tensorflow_distributed_example_amd.data.distributed import DistributedDataset
    n = 203
    x = np.arange(n * 6, dtype=np.float32).reshape(n, 2, 3)
    y = np.arange(n) % 10

    def make():
        ds = Dataset.from_tensor_slices((x, y)).map(lambda a, b: (a * 0.5, b)).cache() \
            .shuffle(50, seed=3).repeat(2).batch(16).prefetch(2)
        if policy is not None:
            o = Options()
            o.experimental_distribute.auto_shard_policy = policy
            ds = ds.with_options(o)
        return ds
    st = SimpleNamespace(num_workers=workers, worker_index=widx, num_local_replicas=2,
                         num_replicas_in_sync=2 * workers, global_replica_id=lambda i: widx * 2 + i)
    ref = list(DistributedDataset(make(), st))
    cols, tup, index_iter = DistributedDataset(make(), st).device_source()
    got = list(index_iter())
    assert tup and len(got) == len(ref) and len(ref) > 10
    for rb, ib in zip(ref, got):
        assert len(rb) == len(ib) == 2
        for (rx, ry), idx in zip(rb, ib):
            assert np.array_equal(cols[0][idx], rx) and np.array_equal(cols[1][idx], ry)
    # pipelines that are not batches of in-memory rows have no device source
    assert Dataset.from_tensor_slices(x).batch(4).unbatch().batch(4).device_source() is None


def test_device_feed_row_eligibility():
    """the HIP row gather moves 4-byte words; an odd bf16 row must fall back to host staging."""
    import torch
    from tensorflow_distributed_example_amd.train.device_feed import DeviceFeed
    assert DeviceFeed.row_ok(784, torch.bfloat16) and DeviceFeed.row_ok(785, torch.float32)
    assert not DeviceFeed.row_ok(785, torch.bfloat16) and not DeviceFeed.row_ok(3, torch.bfloat16)


def test_philox_known_answers_and_keep_fraction():
    """ops/philox.py (the host twin of the fused plans' dropout generator) reproduces the Random123
    Philox4x32-10 known-answer vectors; keep scales are exactly 0 or 1/(1-rate) with a binomial keep
    fraction."""
    from tensorflow_distributed_example_amd.ops.philox import keep_scales, philox4x32_10
    kat = [(([0, 0, 0, 0], [0, 0]), [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
           (([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2), [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
           (([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0]),
            [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1])]
    for (ctr, key), want in kat:
        assert [int(v) for v in philox4x32_10(ctr, key)] == want
    n = 128 * 200
    for rate in (0.5, 0.3):
        k = keep_scales(rate, 0x1234_5678_9ABC, 7, 0, n)
        keep = np.float32(1) - np.float32(rate)
        assert set(np.unique(k)) <= {np.float32(0), np.float32(1) / keep}
        frac = float((k > 0).mean())
        assert abs(frac - (1 - rate)) < 5 * np.sqrt(rate * (1 - rate) / n)
    # a new step (or layer, or seed) draws a new mask
    a, b = keep_scales(0.5, 1, 1, 0, n), keep_scales(0.5, 1, 2, 0, n)
    assert (a != b).mean() > 0.4
