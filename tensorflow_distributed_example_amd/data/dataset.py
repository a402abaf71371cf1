"""tf.data-like input pipeline.

Ops used by the reference: ``from_tensor_slices``, ``map``, ``cache``,
``shuffle(buffer)``, ``repeat``, ``batch``, ``prefetch(n)``, ``with_options``
(distributed_with_keras.py:30,54-57; mnist_keras_distributed.py:142-147).

Design: elements are tuples of numpy arrays.  Chains made of a columnar source
(``from_tensor_slices`` or a filled ``cache``) followed by shuffle/repeat/take/
skip/shard are *indexable*: they produce a stream of row indices and ``batch``
gathers whole batches with one vectorised numpy take per column instead of
per-element Python work.  ``shuffle`` reproduces TF's buffer algorithm (fill a
buffer of ``buffer_size`` elements, emit a uniformly random slot, refill it) on
those indices.  ``prefetch`` runs the upstream iterator in a background thread.
"""
from __future__ import annotations

import enum
import os
import queue
import threading

import numpy as np

AUTOTUNE = -1


class AutoShardPolicy(enum.Enum):
    AUTO = 0
    FILE = 1
    DATA = 2
    OFF = -1
    HINT = 3


class _DistributeOptions:
    def __init__(self):
        self.auto_shard_policy = AutoShardPolicy.AUTO
        self.num_devices = None


class _ThreadingOptions:
    def __init__(self):
        self.private_threadpool_size = 0
        self.max_intra_op_parallelism = 1


class Options:
    def __init__(self):
        self.experimental_distribute = _DistributeOptions()
        self.experimental_deterministic = True
        self.deterministic = True
        self.threading = _ThreadingOptions()

    def merge(self, other: "Options") -> "Options":
        o = Options()
        o.experimental_distribute.auto_shard_policy = other.experimental_distribute.auto_shard_policy \
            if other.experimental_distribute.auto_shard_policy != AutoShardPolicy.AUTO \
            else self.experimental_distribute.auto_shard_policy
        o.experimental_deterministic = other.experimental_deterministic
        o.deterministic = other.deterministic
        return o


def _as_tuple(x):
    if isinstance(x, tuple):
        return x, True
    if isinstance(x, list):
        return tuple(x), True
    return (x,), False


def _np(a):
    try:
        import torch
        if isinstance(a, torch.Tensor):
            return a.detach().cpu().numpy()
    except Exception:  # pragma: no cover
        pass
    return np.asarray(a)


_CHUNK = 8192


def _chunked(it):
    buf = []
    for i in it:
        buf.append(i)
        if len(buf) == _CHUNK:
            yield np.asarray(buf, dtype=np.int64)
            buf = []
    if buf:
        yield np.asarray(buf, dtype=np.int64)


_HOST = []


def _host_lib():
    """libtde_host.so with the pipeline engine, or None (then numpy / Python paths are used)."""
    if not _HOST:
        lib = None
        if os.environ.get("TDE_NATIVE_DATA", "1") != "0":
            try:
                from .. import _native as N
                lib = N.host()
                if not hasattr(lib, "tde_shuffle_new"):
                    lib = None
            except Exception:  # no compiler / library: the pipeline still works
                lib = None
        _HOST.append(lib)
    return _HOST[0]


class Dataset:
    _parent = None

    def __init__(self):
        self._options = None

    # ------------------------------------------------------------------ constructors
    @staticmethod
    def from_tensor_slices(tensors):
        return _Source(tensors)

    @staticmethod
    def from_tensors(tensors):
        cols, is_tuple = _as_tuple(tensors)
        return _Source(tuple(np.expand_dims(_np(c), 0) for c in cols) if is_tuple else np.expand_dims(_np(tensors), 0))

    @staticmethod
    def range(*args):
        return _Source(np.arange(*args, dtype=np.int64))

    @staticmethod
    def from_generator(generator, output_types=None, output_shapes=None, output_signature=None):
        return _Generator(generator)

    # ------------------------------------------------------------------ transformations
    def map(self, map_func, num_parallel_calls=None, deterministic=None):
        return _Map(self, map_func)

    def cache(self, filename=""):
        return _Cache(self, filename)

    def shuffle(self, buffer_size, seed=None, reshuffle_each_iteration=True):
        return _Shuffle(self, int(buffer_size), seed, reshuffle_each_iteration)

    def repeat(self, count=None):
        return _Repeat(self, count)

    def batch(self, batch_size, drop_remainder=False, num_parallel_calls=None, deterministic=None):
        return _Batch(self, int(batch_size), drop_remainder)

    def prefetch(self, buffer_size):
        return _Prefetch(self, buffer_size)

    def take(self, count):
        return _Take(self, int(count))

    def skip(self, count):
        return _Skip(self, int(count))

    def shard(self, num_shards, index):
        return _Shard(self, int(num_shards), int(index))

    def unbatch(self):
        return _Unbatch(self)

    def device_source(self):
        """(columns, structured, batch node) when this pipeline is batches of rows of in-memory columns
        (source [-> map -> cache] -> shuffle/repeat/shard/take/skip -> batch [-> prefetch / options]), so
        a trainer may keep the columns resident on the device and gather batches there from the index
        stream; None otherwise."""
        d = self
        while isinstance(d, (_Prefetch, _WithOptions)):
            d = d._parent
        if not isinstance(d, _Batch) or not d._parent._indexable():
            return None
        return d._parent._columns(), d._parent._structure, d

    def with_options(self, options: Options):
        d = _WithOptions(self, options)
        return d

    def options(self) -> Options:
        o = Options()
        chain = []
        d = self
        while d is not None:
            chain.append(d)
            d = d._parent
        for d in reversed(chain):
            if d._options is not None:
                o = o.merge(d._options)
        return o

    # ------------------------------------------------------------------ iteration
    def __iter__(self):
        raise NotImplementedError

    def as_numpy_iterator(self):
        return iter(self)

    def cardinality(self):
        return -2  # UNKNOWN

    def __len__(self):
        c = self.cardinality()
        if c < 0:
            raise TypeError("dataset length is infinite or unknown")
        return c

    # indexable protocol -------------------------------------------------------------
    def _indexable(self):
        return False

    def _columns(self):
        raise NotImplementedError

    def _index_chunks(self, epoch_seed):
        """The element indices this op produces, as a stream of int64 numpy arrays (chunked so the
        per-element work — shuffling, sharding, batch gathers — runs in numpy / native code)."""
        raise NotImplementedError

    def _index_stream(self, epoch_seed):
        for c in self._index_chunks(epoch_seed):
            yield from c.tolist()

    @property
    def _structure(self):
        return self._parent._structure if self._parent is not None else True

    def _rebuild(self, new_parent):
        """Copy of this op applied to a different input (used by DistributedDataset)."""
        raise NotImplementedError


class _Source(Dataset):
    def __init__(self, tensors):
        super().__init__()
        if isinstance(tensors, dict):
            self._keys = list(tensors)
            cols = tuple(_np(tensors[k]) for k in self._keys)
            self._is_tuple = True
        else:
            self._keys = None
            cols, self._is_tuple = _as_tuple(tensors)
            cols = tuple(_np(c) for c in cols)
        n = {len(c) for c in cols}
        if len(n) != 1:
            raise ValueError("from_tensor_slices: all components need the same first dimension")
        self._cols = cols
        self._n = n.pop()

    @property
    def _structure(self):
        return self._is_tuple

    def _indexable(self):
        return True

    def _columns(self):
        return self._cols

    def _index_chunks(self, epoch_seed):
        for a in range(0, self._n, _CHUNK):
            yield np.arange(a, min(a + _CHUNK, self._n), dtype=np.int64)

    def _element(self, i):
        if self._keys is not None:
            return {k: c[i] for k, c in zip(self._keys, self._cols)}
        e = tuple(c[i] for c in self._cols)
        return e if self._is_tuple else e[0]

    def __iter__(self):
        for i in range(self._n):
            yield self._element(i)

    def cardinality(self):
        return self._n


class _Unary(Dataset):
    def __init__(self, parent):
        super().__init__()
        self._parent = parent

    def cardinality(self):
        return self._parent.cardinality()


class _Map(_Unary):
    def __init__(self, parent, fn):
        super().__init__(parent)
        self._fn = fn

    def __iter__(self):
        tup = self._parent._structure
        for e in self._parent:
            yield self._fn(*e) if (tup and isinstance(e, tuple)) else self._fn(e)

    def _rebuild(self, p):
        return _Map(p, self._fn)


class _Cache(_Unary):
    """Materialises the upstream elements into columnar arrays on first pass."""

    def __init__(self, parent, filename=""):
        super().__init__(parent)
        self._filename = filename
        self._filled = None

    def _fill(self):
        if self._filled is None:
            elems = list(iter(self._parent))
            if not elems:
                self._filled = _Source(np.zeros((0,)))
            elif isinstance(elems[0], tuple):
                self._filled = _Source(tuple(np.stack([e[k] for e in elems]) for k in range(len(elems[0]))))
            else:
                self._filled = _Source(np.stack(elems))
        return self._filled

    @property
    def _structure(self):
        return self._fill()._structure

    def _indexable(self):
        return True

    def _columns(self):
        return self._fill()._columns()

    def _index_chunks(self, epoch_seed):
        return self._fill()._index_chunks(epoch_seed)

    def _element(self, i):
        return self._fill()._element(i)

    def __iter__(self):
        return iter(self._fill())

    def cardinality(self):
        return self._fill().cardinality()

    def _rebuild(self, p):
        return _Cache(p, self._filename)


class _Shuffle(_Unary):
    def __init__(self, parent, buffer_size, seed, reshuffle):
        super().__init__(parent)
        self._buf = max(1, buffer_size)
        self._seed = seed
        self._reshuffle = reshuffle
        self._epoch = 0

    def _rng(self):
        from .. import backend as K
        base = self._seed if self._seed is not None else (K.get_seed() if K.get_seed() is not None else None)
        if base is None:
            rng = np.random.default_rng()
        else:
            rng = np.random.default_rng(base + (self._epoch if self._reshuffle else 0))
        self._epoch += 1
        return rng

    @staticmethod
    def _shuffle_stream(stream, size, rng):
        buf = []
        it = iter(stream)
        for x in it:
            buf.append(x)
            if len(buf) >= size:
                break
        # random draws in chunks to keep per-element Python cost low
        draws = iter(())
        for x in it:
            try:
                r = next(draws)
            except StopIteration:
                draws = iter(rng.random(4096))
                r = next(draws)
            j = int(r * len(buf))
            yield buf[j]
            buf[j] = x
        perm = rng.permutation(len(buf))
        for j in perm:
            yield buf[j]

    def _indexable(self):
        return self._parent._indexable()

    def _columns(self):
        return self._parent._columns()

    def _element(self, i):
        return self._parent._element(i)

    def _index_chunks(self, epoch_seed):
        rng = self._rng()
        parent = self._parent._index_chunks(epoch_seed)
        lib = _host_lib()
        if lib is None:   # pure-Python shuffle buffer (same semantics, numpy RNG)
            yield from _chunked(self._shuffle_stream((i for c in parent for i in c.tolist()), self._buf, rng))
            return
        h = lib.tde_shuffle_new(self._buf, int(rng.integers(0, 2 ** 63 - 1)))
        try:
            for c in parent:
                c = np.ascontiguousarray(c, dtype=np.int64)
                out = np.empty(len(c), np.int64)
                m = lib.tde_shuffle_feed(h, c.ctypes.data, len(c), out.ctypes.data)
                if m:
                    yield out[:m]
            out = np.empty(max(1, lib.tde_shuffle_size(h)), np.int64)
            m = lib.tde_shuffle_drain(h, out.ctypes.data)
            if m:
                yield out[:m]
        finally:
            lib.tde_shuffle_free(h)

    def __iter__(self):
        if self._indexable():
            for c in self._index_chunks(None):
                for i in c.tolist():
                    yield self._element(i)
        else:
            yield from self._shuffle_stream(iter(self._parent), self._buf, self._rng())

    def _rebuild(self, p):
        return _Shuffle(p, self._buf, self._seed, self._reshuffle)


class _Repeat(_Unary):
    def __init__(self, parent, count):
        super().__init__(parent)
        self._count = count if count is not None and count >= 0 else None

    def _indexable(self):
        return self._parent._indexable()

    def _columns(self):
        return self._parent._columns()

    def _element(self, i):
        return self._parent._element(i)

    def _index_chunks(self, epoch_seed):
        k = 0
        while self._count is None or k < self._count:
            empty = True
            for c in self._parent._index_chunks(epoch_seed):
                empty = empty and len(c) == 0
                yield c
            if empty:
                return
            k += 1

    def __iter__(self):
        k = 0
        while self._count is None or k < self._count:
            empty = True
            for e in self._parent:
                empty = False
                yield e
            if empty:
                return
            k += 1

    def cardinality(self):
        c = self._parent.cardinality()
        if self._count is None:
            return -1 if c != 0 else 0
        return c * self._count if c >= 0 else c

    def _rebuild(self, p):
        return _Repeat(p, self._count)


class _Take(_Unary):
    def __init__(self, parent, n):
        super().__init__(parent)
        self._n = n

    def _indexable(self):
        return self._parent._indexable()

    def _columns(self):
        return self._parent._columns()

    def _element(self, i):
        return self._parent._element(i)

    def _index_chunks(self, epoch_seed):
        if self._n < 0:
            yield from self._parent._index_chunks(epoch_seed)
            return
        left = self._n
        if left == 0:
            return
        for c in self._parent._index_chunks(epoch_seed):
            if len(c) >= left:
                yield c[:left]
                return
            left -= len(c)
            yield c

    def __iter__(self):
        for k, e in enumerate(self._parent):
            if self._n >= 0 and k >= self._n:
                return
            yield e

    def cardinality(self):
        c = self._parent.cardinality()
        if self._n < 0:
            return c
        return self._n if c == -1 else (min(c, self._n) if c >= 0 else c)

    def _rebuild(self, p):
        return _Take(p, self._n)


class _Skip(_Take):
    def _index_chunks(self, epoch_seed):
        left = max(self._n, 0)
        for c in self._parent._index_chunks(epoch_seed):
            if left:
                if len(c) <= left:
                    left -= len(c)
                    continue
                c, left = c[left:], 0
            yield c

    def __iter__(self):
        for k, e in enumerate(self._parent):
            if k >= self._n:
                yield e

    def cardinality(self):
        c = self._parent.cardinality()
        return max(c - self._n, 0) if c >= 0 else c

    def _rebuild(self, p):
        return _Skip(p, self._n)


class _Shard(_Unary):
    def __init__(self, parent, n, index):
        super().__init__(parent)
        if not 0 <= index < n:
            raise ValueError("shard index out of range")
        self._k, self._i = n, index

    def _indexable(self):
        return self._parent._indexable()

    def _columns(self):
        return self._parent._columns()

    def _element(self, i):
        return self._parent._element(i)

    def _index_chunks(self, epoch_seed):
        pos = 0   # position of c[0] in the parent stream: keep positions == index (mod k)
        for c in self._parent._index_chunks(epoch_seed):
            sel = c[(self._i - pos) % self._k::self._k]
            pos += len(c)
            if len(sel):
                yield sel

    def __iter__(self):
        for k, e in enumerate(self._parent):
            if k % self._k == self._i:
                yield e

    def cardinality(self):
        c = self._parent.cardinality()
        return (c - self._i + self._k - 1) // self._k if c >= 0 else c

    def _rebuild(self, p):
        return _Shard(p, self._k, self._i)


class _Batch(_Unary):
    def __init__(self, parent, batch_size, drop_remainder):
        super().__init__(parent)
        self.batch_size = batch_size
        self.drop_remainder = drop_remainder

    def index_batches(self):
        """Row indices of every batch of an indexable parent (the shuffle / repeat / shard / take / skip
        algebra runs on index streams; no row is gathered)."""
        bs = self.batch_size
        pend, npend = [], 0
        for c in self._parent._index_chunks(None):
            pend.append(c)
            npend += len(c)
            if npend < bs:
                continue
            cur = np.concatenate(pend) if len(pend) > 1 else pend[0]
            nfull = len(cur) // bs
            for k in range(nfull):
                yield cur[k * bs:(k + 1) * bs]
            rest = cur[nfull * bs:]
            pend, npend = ([rest] if len(rest) else []), len(rest)
        if npend and not self.drop_remainder:
            yield np.concatenate(pend)

    def __iter__(self):
        p = self._parent
        if p._indexable():
            cols = p._columns()
            tup = p._structure
            lib = _host_lib()
            for idx in self.index_batches():
                out = _gather(cols, idx, lib)
                yield out if tup else out[0]
            return
        buf = []
        for e in p:
            buf.append(e)
            if len(buf) == self.batch_size:
                yield _stack(buf)
                buf = []
        if buf and not self.drop_remainder:
            yield _stack(buf)

    def cardinality(self):
        c = self._parent.cardinality()
        if c < 0:
            return c
        return c // self.batch_size if self.drop_remainder else -(-c // self.batch_size)

    def _rebuild(self, p):
        return _Batch(p, self.batch_size, self.drop_remainder)


def _gather(cols, idx, lib):
    """Rows ``idx`` of every column: native multi-threaded row gather (csrc/data/pipeline.cpp) for
    plain contiguous arrays, numpy ``take`` otherwise."""
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    out = []
    for c in cols:
        if lib is not None and isinstance(c, np.ndarray) and c.flags.c_contiguous and c.dtype != object and len(c):
            dst = np.empty((len(idx),) + c.shape[1:], c.dtype)
            rc = lib.tde_gather_rows(c.ctypes.data, c.itemsize * (c.size // len(c)), len(c), idx.ctypes.data,
                                     len(idx), dst.ctypes.data, 8)
            if rc != 0:
                raise IndexError("dataset index out of range")
            out.append(dst)
        else:
            out.append(np.take(c, idx, axis=0))
    return tuple(out)


def _stack(buf):
    if isinstance(buf[0], tuple):
        return tuple(np.stack([b[k] for b in buf]) for k in range(len(buf[0])))
    if isinstance(buf[0], dict):
        return {k: np.stack([b[k] for b in buf]) for k in buf[0]}
    return np.stack(buf)


class _Unbatch(_Unary):
    def __iter__(self):
        for b in self._parent:
            if isinstance(b, tuple):
                for k in range(len(b[0])):
                    yield tuple(c[k] for c in b)
            else:
                yield from b

    def _rebuild(self, p):
        return _Unbatch(p)


_SENTINEL = object()


class _Prefetch(_Unary):
    """Background-thread prefetch of up to ``buffer_size`` upstream elements."""

    def __init__(self, parent, buffer_size):
        super().__init__(parent)
        self._size = 2 if buffer_size in (None, AUTOTUNE) else max(1, int(buffer_size))

    def __iter__(self):
        q: queue.Queue = queue.Queue(maxsize=self._size)
        stop = threading.Event()
        err = []

        def worker():
            try:
                for e in self._parent:
                    while not stop.is_set():
                        try:
                            q.put(e, timeout=0.1)
                            break
                        except queue.Full:
                            continue
                    if stop.is_set():
                        return
            except BaseException as ex:  # propagate to consumer
                err.append(ex)
            finally:
                while not stop.is_set():
                    try:
                        q.put(_SENTINEL, timeout=0.1)
                        break
                    except queue.Full:
                        continue

        th = threading.Thread(target=worker, daemon=True, name="tde-prefetch")
        th.start()
        try:
            while True:
                e = q.get()
                if e is _SENTINEL:
                    if err:
                        raise err[0]
                    return
                yield e
        finally:
            stop.set()

    def _rebuild(self, p):
        return _Prefetch(p, self._size)


class _WithOptions(_Unary):
    def __init__(self, parent, options):
        super().__init__(parent)
        self._options = options

    def _indexable(self):
        return self._parent._indexable()

    def _columns(self):
        return self._parent._columns()

    def _element(self, i):
        return self._parent._element(i)

    def _index_chunks(self, epoch_seed):
        return self._parent._index_chunks(epoch_seed)

    def __iter__(self):
        return iter(self._parent)

    def _rebuild(self, p):
        return _WithOptions(p, self._options)


class _Generator(Dataset):
    def __init__(self, gen):
        super().__init__()
        self._gen = gen

    def __iter__(self):
        return iter(self._gen())


class experimental:  # noqa: N801  (tf.data.experimental namespace)
    AutoShardPolicy = AutoShardPolicy
    AUTOTUNE = AUTOTUNE
