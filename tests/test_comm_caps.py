"""CPU checks of the xGMI all-reduce grid sizing (parallel/comm.spin_grid_caps): the spin limit applies only
when other processes share a GPU, and shrinks with their number (the round-3 eager MWMS 2x2 timeouts:
a spinning grid on every CU starved a co-located process's whole-CU backward kernel)."""
import types

import torch

from tensorflow_distributed_example_amd.parallel import comm as CM


class _Props:
    def __init__(self, bus):
        self.pci_domain_id, self.pci_bus_id, self.pci_device_id = 0, bus, 0
        self.multi_processor_count = 256
        self.uuid = f"gpu-{bus}"


class _Ctl:
    """all_gather_json of a job whose other processes hold the given device-key lists."""

    def __init__(self, others):
        self.others = others

    def all_gather_json(self, obj, tag):
        return [obj] + self.others


def _setup(monkeypatch):
    monkeypatch.setattr(CM.torch.cuda, "get_device_properties", lambda d: _Props(0x10 + torch.device(d).index))
    monkeypatch.setattr("socket.gethostname", lambda: "node0")
    return lambda i: CM._device_key(torch.device(f"cuda:{i}"))


def test_one_process_per_gpu_has_no_spin_limit(monkeypatch):
    key = _setup(monkeypatch)
    d0 = torch.device("cuda:0")
    assert CM.spin_grid_caps(None, [d0], "t") == [None]
    # 8 processes, each on its own GPU (the driver's N=8 run)
    others = [[key(i)] for i in range(1, 8)]
    assert CM.spin_grid_caps(_Ctl(others), [d0], "t") == [None]


def test_colocated_processes_leave_a_quarter_of_the_cus_free(monkeypatch):
    key = _setup(monkeypatch)
    d0 = torch.device("cuda:0")
    assert CM.spin_grid_caps(_Ctl([[key(0)]]), [d0], "t") == [192]          # 2 processes on one GPU
    assert CM.spin_grid_caps(_Ctl([[key(0)]] * 3), [d0], "t") == [64]      # 4
    assert CM.spin_grid_caps(_Ctl([[key(0)]] * 7), [d0], "t") == [27]      # 8 (the N=8 rehearsal)
    monkeypatch.setenv("TDE_XGMI_SPIN_CAP", "0")
    assert CM.spin_grid_caps(_Ctl([[key(0)]] * 7), [d0], "t") == [None]


def test_grid_sizes_respect_the_cap(monkeypatch):
    lib = types.SimpleNamespace(tde_xgmi_max_blocks=lambda: 128)
    xg = object.__new__(CM.XgmiCommunicator)
    xg.lib, xg.world, xg.nblocks_override = lib, 2, 0
    xg.grid_cap = None
    assert xg.nblocks(347146) == 128
    xg.grid_cap = 27
    assert xg.nblocks(347146) == 27
    pg = object.__new__(CM.PeerXgmiCommunicator)
    pg.lib, pg.world, pg.nblocks_override = lib, 4, 0
    pg.grid_caps = [None]
    assert pg.nblocks(347146, 2, 0) == 128      # one process: the grouped grid may cover 2 x 128
    pg.grid_caps = [192]
    assert pg.nblocks(347146, 2, 0) == 96       # co-located: 2 x 96 <= 192
    assert pg.nblocks(1000, 2, 0) == 8
