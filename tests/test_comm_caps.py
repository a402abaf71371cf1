"""CPU checks of the xGMI all-reduce grid sizing (parallel/comm.spin_chunk_cap): the spin limit applies only
when other processes share a GPU, shrinks with their number (the round-3 eager MWMS 2x2 timeouts: a
spinning grid on every CU starved a co-located process's whole-CU backward kernel), and is ONE number on
every rank of the world, whatever its own layout (the kernel's slices and flags assume equal chunk counts)."""
import types

import pytest
import torch

from tensorflow_distributed_example_amd.parallel import comm as CM


class _Props:
    def __init__(self, bus):
        self.pci_domain_id, self.pci_bus_id, self.pci_device_id = 0, bus, 0
        self.multi_processor_count = 256
        self.uuid = f"gpu-{bus}"


class _Ctl:
    """all_gather_json of a job whose other processes hold the given layouts ({device key: [nloc, CUs]})."""

    def __init__(self, others, caps=None):
        self.others = others
        self.caps = caps

    def all_gather_json(self, obj, tag):
        if tag.endswith("_agree"):
            return [obj] + (self.caps if self.caps is not None else [obj] * len(self.others))
        return [obj] + self.others


def _setup(monkeypatch):
    monkeypatch.setattr(CM.torch.cuda, "get_device_properties", lambda d: _Props(0x10 + torch.device(d).index))
    monkeypatch.setattr("socket.gethostname", lambda: "node0")
    return lambda i: CM._device_key(torch.device(f"cuda:{i}"))


def test_one_process_per_gpu_has_no_spin_limit(monkeypatch):
    key = _setup(monkeypatch)
    d0 = torch.device("cuda:0")
    assert CM.spin_chunk_cap(None, [d0], "t") is None
    # 8 processes, each on its own GPU (the driver's N=8 run)
    others = [{key(i): [1, 256]} for i in range(1, 8)]
    assert CM.spin_chunk_cap(_Ctl(others), [d0], "t") is None
    # one process, 8 replicas on 8 GPUs (MirroredStrategy)
    assert CM.spin_chunk_cap(None, [torch.device(f"cuda:{i}") for i in range(8)], "t") is None


def test_colocated_processes_leave_a_quarter_of_the_cus_free(monkeypatch):
    key = _setup(monkeypatch)
    d0 = torch.device("cuda:0")
    one = {key(0): [1, 256]}
    assert CM.spin_chunk_cap(_Ctl([one]), [d0], "t") == 192          # 2 processes on one GPU
    assert CM.spin_chunk_cap(_Ctl([one] * 3), [d0], "t") == 64       # 4
    assert CM.spin_chunk_cap(_Ctl([one] * 7), [d0], "t") == 27       # 8 (the N=8 rehearsal)
    monkeypatch.setenv("TDE_XGMI_SPIN_CAP", "0")
    assert CM.spin_chunk_cap(_Ctl([one] * 7), [d0], "t") is None


def test_uneven_colocation_gives_every_rank_the_same_cap(monkeypatch):
    """3 processes on 2 GPUs (A: 2 replicas on gpu0; B: 1 replica on gpu0; C: 1 on gpu1).  A
    per-process cap would give A's ranks 96 chunks and C's ranks none: owners would read contributions at
    the wrong offsets or wait on flags that never come.  The world-wide cap is the smallest per-rank share."""
    key = _setup(monkeypatch)
    lay_a = {key(0): [2, 256]}
    lay_b = {key(0): [1, 256]}
    lay_c = {key(1): [1, 256]}
    expect = 192 // 2    # gpu0: 2 processes -> grid 192; the largest group there has 2 ranks
    assert CM.chunk_cap_of([lay_a, lay_b, lay_c]) == expect
    assert CM.spin_chunk_cap(_Ctl([lay_b, lay_c]), [torch.device("cuda:0")] * 2, "t") == expect
    assert CM.spin_chunk_cap(_Ctl([lay_a, lay_c]), [torch.device("cuda:0")], "t") == expect
    assert CM.spin_chunk_cap(_Ctl([lay_a, lay_b]), [torch.device("cuda:1")], "t") == expect
    # two shared devices: the smaller share wins everywhere
    assert CM.chunk_cap_of([{key(0): [1, 256], key(1): [4, 256]}, {key(0): [1, 256], key(1): [1, 256]},
                            {key(0): [1, 256]}]) == 192 // 4


def test_disagreeing_caps_raise(monkeypatch):
    key = _setup(monkeypatch)
    one = {key(0): [1, 256]}
    with pytest.raises(RuntimeError, match="differ across ranks"):
        CM.spin_chunk_cap(_Ctl([one], caps=[None]), [torch.device("cuda:0")], "t")


def test_grid_sizes_respect_the_cap(monkeypatch):
    lib = types.SimpleNamespace(tde_xgmi_max_blocks=lambda: 128)
    xg = object.__new__(CM.XgmiCommunicator)
    xg.lib, xg.world, xg.nblocks_override = lib, 2, 0
    xg.chunk_cap = None
    assert xg.nblocks(347146) == 128
    xg.chunk_cap = 27
    assert xg.nblocks(347146) == 27
    pg = object.__new__(CM.PeerXgmiCommunicator)
    pg.lib, pg.world, pg.nblocks_override = lib, 4, 0
    pg.chunk_cap = None
    assert pg.nblocks(347146, 2, 0) == 128      # one process: the grouped grid may cover 2 x 128
    pg.chunk_cap = 96                           # co-located: 192 // 2 ranks per grid
    assert pg.nblocks(347146, 2, 0) == 96
    assert pg.nblocks(347146, 1, 0) == 96       # a 1-replica group of the same world: the same count
    assert pg.nblocks(1000, 2, 0) == 8


def test_gpu_sharing_decides_wide_allreduce_workgroups(monkeypatch):
    """GPU_SHARED (what the communicators pass to tde_xgmi_set_wide): 1024-thread all-reduce workgroups only when
    no GPU of the world runs two processes' all-reduces — independent of the TDE_XGMI_SPIN_CAP=0 diagnostics
    override, which lifts the chunk limit but not the co-location."""
    key = _setup(monkeypatch)
    d0 = torch.device("cuda:0")
    CM.spin_chunk_cap(_Ctl([{key(i): [1, 256]} for i in range(1, 8)]), [d0], "w8")
    assert CM.GPU_SHARED["w8"] is False                    # 8 processes, 8 GPUs
    CM.spin_chunk_cap(None, [d0, d0], "mirrored")
    assert CM.GPU_SHARED["mirrored"] is False              # in-process replicas on one GPU: one grid
    CM.spin_chunk_cap(_Ctl([{key(0): [1, 256]}]), [d0], "co")
    assert CM.GPU_SHARED["co"] is True                     # 2 processes on one GPU
    monkeypatch.setenv("TDE_XGMI_SPIN_CAP", "0")
    assert CM.spin_chunk_cap(_Ctl([{key(0): [1, 256]}]), [d0], "co0") is None
    assert CM.GPU_SHARED["co0"] is True
