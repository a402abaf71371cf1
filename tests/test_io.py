"""T2: native host I/O — crc32c golden values, TensorBundle round trip + an
independent pure-Python SSTable/proto parse of the native writer's bytes, and
TensorBoard event files."""
import ctypes as C
import struct

import numpy as np
import pytest

from tensorflow_distributed_example_amd import _native as N
from tensorflow_distributed_example_amd.io import events as EV
from tensorflow_distributed_example_amd.io import tensor_bundle as TB


def _crc(b: bytes):
    return N.host().tde_crc32c(b, len(b))


def test_crc32c_golden():
    assert _crc(b"123456789") == 0xE3069283
    assert _crc(b"") == 0
    assert _crc(b"\x00" * 32) == 0x8A9136AA
    lib = N.host()
    for v in (0, 1, 0xDEADBEEF, 0xE3069283):
        assert lib.tde_crc32c_unmask(lib.tde_crc32c_mask(v)) == v
    assert lib.tde_crc32c_mask(0xE3069283) == (((0xE3069283 >> 15) | (0xE3069283 << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(b, i):
    r = s = 0
    while True:
        x = b[i]
        i += 1
        r |= (x & 0x7F) << s
        if x < 0x80:
            return r, i
        s += 7


def _block(buf, off, size):
    """Independent LevelDB block parser (prefix-compressed keys)."""
    data = buf[off: off + size]
    typ = buf[off + size]
    (stored,) = struct.unpack("<I", buf[off + size + 1: off + size + 5])
    lib = N.host()
    raw = bytes(data) + bytes([typ])
    assert lib.tde_crc32c_unmask(stored) == _crc(raw)
    assert typ == 0
    (nres,) = struct.unpack("<I", data[-4:])
    end = len(data) - 4 - 4 * nres
    i, key, out = 0, b"", []
    while i < end:
        shared, i = _varint(data, i)
        nonshared, i = _varint(data, i)
        vlen, i = _varint(data, i)
        key = key[:shared] + data[i:i + nonshared]
        i += nonshared
        out.append((key, data[i:i + vlen]))
        i += vlen
    return out


def _sstable(path):
    buf = open(path, "rb").read()
    assert struct.unpack("<Q", buf[-8:])[0] == 0xDB4775248B80FB57
    i = len(buf) - 48
    moff, i = _varint(buf, i)
    msize, i = _varint(buf, i)
    ioff, i = _varint(buf, i)
    isize, i = _varint(buf, i)
    rows = []
    for _, h in _block(buf, ioff, isize):
        bo, j = _varint(h, 0)
        bs, j = _varint(h, j)
        rows += _block(buf, bo, bs)
    return rows


def test_tensor_bundle_roundtrip_and_independent_parse(tmp_path):
    rng = np.random.default_rng(0)
    tensors = {"dense/kernel": rng.random((5408, 64), dtype=np.float32),
               "conv2d/kernel": rng.random((3, 3, 1, 32), dtype=np.float32),
               "conv2d/bias": np.zeros(32, np.float32),
               "global_step": np.array(469, dtype=np.int64)}
    for i in range(40):  # > 16 keys: exercises restart points
        tensors[f"extra/v{i:02d}"] = np.full((i + 1,), i, np.float32)
    prefix = str(tmp_path / "model.ckpt-469")
    TB.write_bundle(prefix, tensors)
    back = TB.read_bundle(prefix)
    assert set(back) == set(tensors)
    for k in tensors:
        assert back[k].shape == tensors[k].shape and np.array_equal(back[k], tensors[k])
    rows = _sstable(prefix + ".index")
    keys = [k for k, _ in rows]
    assert keys[0] == b"" and keys[1:] == sorted(k.encode() for k in tensors)
    # header proto: num_shards=1 (field 1), version{producer=1} (field 3)
    assert rows[0][1] == bytes([0x08, 0x01, 0x1A, 0x02, 0x08, 0x01])
    data = open(prefix + ".data-00000-of-00001", "rb").read()
    ent = dict(rows)[b"dense/kernel"]
    # BundleEntryProto: dtype DT_FLOAT (08 01), shape dims 5408, 64, offset, size, crc (fixed32 field 6)
    assert ent[:2] == bytes([0x08, 0x01])
    fields = {}
    i = 0
    while i < len(ent):
        tag, i = _varint(ent, i)
        f, wt = tag >> 3, tag & 7
        if wt == 0:
            v, i = _varint(ent, i)
        elif wt == 2:
            n, i = _varint(ent, i)
            v = ent[i:i + n]
            i += n
        else:
            v = struct.unpack("<I", ent[i:i + 4])[0]
            i += 4
        fields[f] = v
    off, size = fields.get(4, 0), fields[5]
    assert size == 5408 * 64 * 4
    blob = data[off: off + size]
    assert np.array_equal(np.frombuffer(blob, np.float32).reshape(5408, 64), tensors["dense/kernel"])
    assert N.host().tde_crc32c_unmask(fields[6]) == _crc(blob)


def test_bundle_detects_corruption(tmp_path):
    prefix = str(tmp_path / "c")
    TB.write_bundle(prefix, {"a": np.arange(100, dtype=np.float32)})
    d = bytearray(open(prefix + ".data-00000-of-00001", "rb").read())
    d[10] ^= 0xFF
    open(prefix + ".data-00000-of-00001", "wb").write(bytes(d))
    with pytest.raises(IOError, match="crc"):
        TB.read_bundle(prefix)


def test_checkpoint_state_file(tmp_path):
    TB.write_bundle(str(tmp_path / "model.ckpt-10"), {"x": np.ones(3, np.float32)})
    TB.write_checkpoint_state(tmp_path, "model.ckpt-10", ["model.ckpt-0", "model.ckpt-10"])
    st = TB.read_checkpoint_state(tmp_path)
    assert st["model_checkpoint_path"] == "model.ckpt-10"
    assert st["all_model_checkpoint_paths"] == ["model.ckpt-0", "model.ckpt-10"]
    assert TB.latest_checkpoint(tmp_path) == str(tmp_path / "model.ckpt-10")
    assert 'model_checkpoint_path: "model.ckpt-10"' in (tmp_path / "checkpoint").read_text()


def test_event_file_roundtrip(tmp_path):
    w = EV.EventFileWriter(tmp_path)
    w.add_scalars(100, {"loss": 0.5, "accuracy": 0.875})
    w.add_scalar("global_step/sec", 1234.5, 100)
    w.close()
    evs = EV.read_events(w.path)
    assert evs[0]["file_version"] == "brain.Event:2"
    assert evs[1]["step"] == 100 and evs[1]["scalars"] == {"loss": 0.5, "accuracy": 0.875}
    assert abs(evs[2]["scalars"]["global_step/sec"] - 1234.5) < 1e-3
    # TFRecord framing: first 8 bytes = length, then masked crc32c of the length
    raw = open(w.path, "rb").read()
    (ln,) = struct.unpack("<Q", raw[:8])
    (lc,) = struct.unpack("<I", raw[8:12])
    assert N.host().tde_crc32c_unmask(lc) == _crc(raw[:8])
    assert ln == len(raw[12:12 + ln])
