"""xGMI peer-memory gradient all-reduce (csrc/comm/xgmi_allreduce.hip).

The GPU box has ONE MI355X, so the multi-rank tests run 2 and 4 processes that all map their
windows on cuda:0 through the same IPC path the 8-GPU node uses (hipIpcGetMemHandle /
hipIpcOpenMemHandle, system-scope flags).  The result must be BITWISE equal to the fp32 sum in
rank order, in eager launches and inside a replayed hipGraph, and MWMS training over it must keep
every replica bit-identical.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


WORKER = r"""
import json, os, sys
sys.path.insert(0, {root!r})
import torch
from tensorflow_distributed_example_amd.parallel import comm as CM, control as CP
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
cp = CP.ControlPlane(rank, world, "127.0.0.1", {port}, timeout=120)
fb = CM.StoreCommunicator(cp, 1)
xg = CM.XgmiCommunicator("cuda:0", rank, world, fb, cp, max_elems=1 << 20, timeout_s=30)
out = {{"self_test": xg.self_test()}}
bad = []
g = torch.Generator(device="cpu")
for it, n in enumerate([347146, 250466, 1, 5, 1023, 4096 * 8 + 3, 1 << 20]):
    parts = []
    for r in range(world):
        g.manual_seed(1000 * it + r)
        parts.append(torch.randn(n, generator=g).cuda())
    want = parts[0].clone()
    for p in parts[1:]:
        want += p
    t = parts[rank].clone()
    xg.all_reduce_([t])
    torch.cuda.synchronize()
    if not torch.equal(t, want):
        bad.append((n, float((t - want).abs().max())))
out["eager_bad"] = bad
# hipGraph: 5 all-reduces captured once, replayed 3 times (the epoch advances on the device)
n = 347146
buf = torch.zeros(n, device="cuda")
src = torch.zeros(n, device="cuda")
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    xg.all_reduce_([buf])      # warm-up outside capture
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
cp.barrier()
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    for k in range(5):
        buf.copy_(src)
        buf.mul_(float(k + 1))
        xg.all_reduce_([buf])
        src.copy_(buf)
gbad = []
for rep in range(3):
    torch.manual_seed(rep)
    base = [torch.rand(n) for _ in range(world)]
    src.copy_(base[rank].cuda())
    torch.cuda.synchronize()
    cp.barrier()
    graph.replay()
    torch.cuda.synchronize()
    # reference: x_r <- sum_r(x_r * (k+1)) five times, all ranks identical after the first
    ref = [b.cuda() for b in base]
    for k in range(5):
        sc = [r_ * float(k + 1) for r_ in ref]
        tot = sc[0].clone()
        for q in sc[1:]:
            tot += q
        ref = [tot.clone() for _ in range(world)]
    if not torch.equal(src, ref[rank]):
        gbad.append(rep)
out["graph_bad"] = gbad
out["calls"] = xg.calls()
out["err"] = int(xg.lib.tde_xgmi_error(xg.err))
cp.barrier()
xg.close()
print("RESULT" + json.dumps(out), flush=True)
cp.shutdown()
"""


@pytest.mark.parametrize("world", [2, 4, 8])
def test_xgmi_allreduce_bitwise(world, tmp_path):
    """world ranks (one process each, all on cuda:0; 8 = the N=8 kernel path with its co-located spin
    limit) vs the rank-ordered fp32 sum, eager and graph-captured."""
    port = _free_port()
    script = WORKER.format(root=ROOT, port=port)
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), OMP_NUM_THREADS="2")
        procs.append(subprocess.Popen([sys.executable, "-c", script], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        o, _ = p.communicate(timeout=240)
        assert p.returncode == 0, o[-4000:]
        outs.append(json.loads(o.split("RESULT")[1].strip()))
    for o in outs:
        assert o["self_test"], o
        assert o["eager_bad"] == [], o
        assert o["graph_bad"] == [], o
        assert o["err"] == 0, o
        assert o["calls"] == 3 + 7 + 1 + 15, o


def test_mwms_bench_two_ranks_on_xgmi(tmp_path):
    """bench.py under torchrun with 2 ranks sharing cuda:0: the gradient bucket goes through the
    xGMI kernel (captured in the step's hipGraph) and the run reports one JSON line."""
    env = dict(os.environ, TDE_RCCL="0", TDE_ALLREDUCE="xgmi", TDE_HEARTBEAT="0", OMP_NUM_THREADS="2", TDE_BENCH_WARM_MS="0",
               TDE_CHECK_XGMI="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "64", "--warmup", "16"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["value"] > 0
    assert res["config"]["allreduce"] == "xgmi", res
    assert res["config"]["hipgraph"] is True, res
    assert "replicas_identical=True" in r.stdout, r.stdout[-3000:]


FALLBACK = r"""
import json, os, sys
sys.path.insert(0, {root!r})
import torch
from tensorflow_distributed_example_amd.parallel import comm as CM, control as CP
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
cp = CP.ControlPlane(rank, world, "127.0.0.1", {port}, timeout=120)
fb = CM.StoreCommunicator(cp, 1)
c = CM.maybe_xgmi(fb, torch.device("cuda:0"), rank, world, cp)
t = torch.full((1000,), float(rank + 1), device="cuda")
c.all_reduce_([t])
torch.cuda.synchronize()
print("RESULT" + json.dumps({{"kind": type(c).__name__, "sum": float(t[0])}}), flush=True)
cp.shutdown()
"""


def test_xgmi_setup_failure_on_one_rank_falls_back_everywhere():
    """A window that fails on ONE rank must make every rank keep the fallback (no rank left waiting)."""
    port = _free_port()
    script = FALLBACK.format(root=ROOT, port=port)
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", OMP_NUM_THREADS="2", TDE_ALLREDUCE="xgmi",
                   TDE_XGMI_FAIL_RANK="1")
        procs.append(subprocess.Popen([sys.executable, "-c", script], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    for p in procs:
        o, _ = p.communicate(timeout=180)
        assert p.returncode == 0, o[-3000:]
        res = json.loads(o.split("RESULT")[1].strip())
        assert res["kind"] == "StoreCommunicator" and res["sum"] == 3.0, res


def test_bucketed_overlapped_allreduce_two_ranks():
    """Layer-wise plan (bf16 policy) under MWMS with small reverse-order buckets: each bucket's xGMI all-reduce is
    enqueued on the comm stream behind the backward stage that finalises it (captured in the step's
    hipGraph); replicas stay bit-identical and training matches the single post-backward all-reduce."""
    losses = {}
    for overlap in ("1", "0"):
        env = dict(os.environ, TDE_RCCL="0", TDE_ALLREDUCE="xgmi", TDE_HEARTBEAT="0", OMP_NUM_THREADS="2", TDE_BENCH_WARM_MS="0",
                   TDE_OVERLAP=overlap, TDE_BUCKET_MB="0.2")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
               "--gpus", "2", "--model", "mnist_bn_cnn", "--steps", "48", "--warmup", "16", "--dtype", "bf16"]
        r = subprocess.run(cmd, env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stdout[-4000:]
        res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
        assert res["config"]["allreduce"] == "xgmi" and res["config"]["hipgraph"] is True, res
        assert (res["config"]["grad_buckets"] > 1) == (overlap == "1"), res
        assert "replicas_identical=True" in r.stdout, r.stdout[-3000:]
        losses[overlap] = float(r.stdout.split("loss=")[1].split()[0])
    assert abs(losses["1"] - losses["0"]) < 0.05 * max(1.0, abs(losses["0"])), losses


def test_rccl_init_failure_falls_back_on_every_rank():
    """Two ranks on one GPU make ncclCommInitRank fail on both (duplicate GPU): the strategy agrees on
    the failure (through the native control plane), keeps the store for the control collectives and the
    xGMI kernel for the gradient bucket."""
    env = dict(os.environ, TDE_ALLREDUCE="xgmi", TDE_HEARTBEAT="0", OMP_NUM_THREADS="2", TDE_BENCH_WARM_MS="0")
    env.pop("TDE_RCCL", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "32", "--warmup", "8"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-4000:]
    assert "RCCL communicator init failed" in r.stdout, r.stdout[-3000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert res["config"]["allreduce"] == "xgmi", res
    assert "replicas_identical=True" in r.stdout


APPLY = r"""
import json, os, sys
sys.path.insert(0, {root!r})
import torch
from tensorflow_distributed_example_amd.parallel import comm as CM, control as CP
from tensorflow_distributed_example_amd.ops import kernels as K
from tensorflow_distributed_example_amd import optimizers as O
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
cp = CP.ControlPlane(rank, world, "127.0.0.1", {port}, timeout=120)
xg = CM.XgmiCommunicator("cuda:0", rank, world, CM.StoreCommunicator(cp, 1), cp, max_elems=1 << 20, timeout_s=30)
out = {{}}
n, lo, rows, cols = 347146 + 58, 64, 5408, 64
opts = {{"sgd": O.SGD(0.05), "momentum": O.SGD(0.05, momentum=0.9),
         "nesterov": O.SGD(0.05, momentum=0.9, nesterov=True), "adam": O.Adam(1e-3)}}
for name, opt in opts.items():
    g = torch.Generator(device="cpu").manual_seed(7)
    w = torch.randn(n, generator=g).cuda()
    m = torch.randn(n, generator=g).cuda() if opt.kind != "sgd" else None
    v = torch.rand(n, generator=g).cuda() if opt.kind == "adam" else None
    it = torch.full((1,), 3, dtype=torch.int64, device="cuda")
    grads = [torch.randn(n, generator=torch.Generator().manual_seed(100 + r)).cuda() for r in range(world)]
    gsum = grads[0].clone()
    for q in grads[1:]:
        gsum += q
    rw, rm, rv = w.clone(), None if m is None else m.clone(), None if v is None else v.clone()
    slots = {{}}
    if opt.kind in ("momentum", "nesterov"):
        slots["momentum"] = rm
    if opt.kind == "adam":
        slots["m"], slots["v"] = rm, rv
    opt.apply_reference(rw, gsum, slots, 2)   # Adam t = step + 1 = 3 = iterations
    sh = torch.zeros(rows * cols, dtype=torch.bfloat16, device="cuda")
    sht = torch.zeros(cols, rows, dtype=torch.bfloat16, device="cuda")
    hp = opt.hparams()
    spec = K.XgApply(opt.kind_id, opt.learning_rate, hp["mom"], hp["b1"], hp["b2"], hp["eps"], w.data_ptr(),
                     K._P(m), K._P(v), it.data_ptr(), sh.data_ptr(), lo, lo + rows * cols, sht.data_ptr(), cols,
                     rows)
    gb = grads[rank].clone()
    xg.all_reduce_apply_(gb, spec)
    torch.cuda.synchronize()
    rel = float((w - rw).norm() / (rw.norm()))
    res = {{"w_rel": rel, "w_max": float((w - rw).abs().max()), "grad_zero": bool((gb == 0).all()),
           "sh_ok": bool(torch.equal(sh, w[lo:lo + rows * cols].to(torch.bfloat16))),
           "sht_ok": bool(torch.equal(sht, w[lo:lo + rows * cols].view(rows, cols).t().to(torch.bfloat16)))}}
    if m is not None:
        res["m_max"] = float((m - rm).abs().max())
    if v is not None:
        res["v_max"] = float((v - rv).abs().max())
    # every rank must hold bit-identical weights
    allw = cp.all_gather_bytes(w.cpu().numpy().tobytes())
    res["identical"] = all(q == allw[0] for q in allw[1:])
    out[name] = res
out["err"] = int(xg.lib.tde_xgmi_error(xg.err))
cp.barrier()
xg.close()
print("RESULT" + json.dumps(out), flush=True)
cp.shutdown()
"""


def test_xgmi_allreduce_apply_matches_reference():
    """The fused all-reduce + optimizer (every kind) against the fp32 torch update of the rank-ordered
    gradient sum: weights, slots, bf16 shadows (row-major and transposed), zeroed bucket, and all ranks
    bit-identical."""
    world = 2
    port = _free_port()
    script = APPLY.format(root=ROOT, port=port)
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), OMP_NUM_THREADS="2")
        procs.append(subprocess.Popen([sys.executable, "-c", script], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    for p in procs:
        o, _ = p.communicate(timeout=240)
        assert p.returncode == 0, o[-4000:]
        res = json.loads(o.split("RESULT")[1].strip())
        assert res.pop("err") == 0, res
        for name, r in res.items():
            assert r["w_max"] < 1e-5 and r["grad_zero"] and r["sh_ok"] and r["sht_ok"] and r["identical"], (name, r)
            assert r.get("m_max", 0.0) < 1e-5 and r.get("v_max", 0.0) < 1e-5, (name, r)


def test_mwms_fused_allreduce_apply_matches_unfused():
    """bench.py with 2 ranks: the optimizer fused into the xGMI all-reduce (default) vs the separate
    optimizer launch (TDE_FUSED_STEP=0): replicas bit-identical in both, same JSON contract.  (The
    weight-level equivalence of the fused step is pinned by test_mirrored_gpu's N-replica tests.)"""
    for fused in ("1", "0"):
        env = dict(os.environ, TDE_RCCL="0", TDE_ALLREDUCE="xgmi", TDE_HEARTBEAT="0", OMP_NUM_THREADS="2", TDE_BENCH_WARM_MS="0",
                   TDE_FUSED_STEP=fused)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
               "--gpus", "2", "--steps", "48", "--warmup", "16", "--lr", "0.05"]
        r = subprocess.run(cmd, env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stdout[-4000:]
        res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
        assert res["config"]["allreduce"] == "xgmi" and res["config"]["hipgraph"] is True, res
        assert res["config"]["optimizer_placement"] == ("allreduce" if fused == "1" else "separate"), res
        assert "replicas_identical=True" in r.stdout, r.stdout[-3000:]


WIDE = r"""
import sys
sys.path.insert(0, {root!r})
import torch
torch.cuda.set_device(0)
from tensorflow_distributed_example_amd import _native as N
lib = N.hip()
cus = torch.cuda.get_device_properties(0).multi_processor_count
out = [lib.tde_xgmi_threads(2, 128)]        # not yet set: 256
lib.tde_xgmi_set_wide(1)
out += [lib.tde_xgmi_threads(2, 128), lib.tde_xgmi_threads(1, 128), lib.tde_xgmi_threads(8, 128)]
lib.tde_xgmi_set_wide(0)                    # a shared GPU: sticky off
lib.tde_xgmi_set_wide(1)
out += [lib.tde_xgmi_threads(1, 128)]
print("WIDE", cus, *out, flush=True)
"""


def test_allreduce_workgroup_width_rule():
    """The xGMI all-reduce runs 1024-thread workgroups only after a communicator declared the GPU unshared and only
    while the grid (local ranks x chunks) fits one workgroup per CU; a shared GPU turns it off for good."""
    r = subprocess.run([sys.executable, "-c", WIDE.format(root=ROOT)], stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-3000:]
    vals = [int(v) for v in r.stdout.split("WIDE")[1].split()]
    cus, before, two, one, eight, after = vals
    assert before == 256 and after == 256
    assert two == (1024 if 2 * 128 <= cus else 256) and one == 1024
    assert eight == (1024 if 8 * 128 <= cus else 256)
