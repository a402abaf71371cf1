#!/usr/bin/env python
"""Diagnostics of the in-process xGMI path (MirroredStrategy over replicas of one process): runs
``--execs`` executions of ``--spe`` steps and prints, after each, the wall time, the communicator's
error bits and every replica's all-reduce epoch.  Run with a short ``TDE_XGMI_TIMEOUT`` so a missed
peer ends each wait quickly and shows up as error bits instead of a hang."""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--devices", default="0,0")
    ap.add_argument("--spe", type=int, default=16)
    ap.add_argument("--execs", type=int, default=40)
    ap.add_argument("--model", default="mnist_cnn")
    ap.add_argument("--sync-every", type=int, default=1)
    ap.add_argument("--mwms", type=int, default=0, help="K > 0: MultiWorkerMirroredStrategy with K GPUs per worker "
                    "(launch with torchrun)")
    ap.add_argument("--trace-show", type=int, default=6, help="with TDE_XGMI_TRACE: calls printed per rank")
    a = ap.parse_args()
    import torch

    import tensorflow_distributed_example_amd as tde
    tde.backend.set_global_policy("float32")
    if a.mwms:
        strategy = tde.distribute.MultiWorkerMirroredStrategy(gpus_per_worker=a.mwms)
    else:
        strategy = tde.distribute.MirroredStrategy([f"cuda:{d}" for d in a.devices.split(",")])
    comm = strategy.comm
    tag = f"[diag w{strategy.worker_index}]"
    print(f"{tag} comm={type(comm).__name__} groups={getattr(comm, 'groups', None)}", flush=True)
    with strategy.scope():
        model = getattr(tde.zoo, a.model)()
        model.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=a.model != "mnist_bn_cnn"),
                      optimizer=tde.optimizers.SGD(0.01), metrics=["accuracy"], steps_per_execution=a.spe)
    n = strategy.num_replicas_in_sync
    nl = strategy.num_local_replicas
    prog = model._program("train", 64 * n)
    print(f"{tag} per_replica={prog.per_replica} graph={prog.use_graph} mode={prog.plans[0].step_mode}", flush=True)
    xs = [torch.rand((a.spe, 64) + tuple(prog.x_shape), device=d) for d in strategy.local_devices]
    ys = [torch.randint(0, 10, (a.spe, 64), device=d).to(torch.int32) for d in strategy.local_devices]
    for e in range(a.execs):
        t0 = time.perf_counter()
        prog.stage(list(zip(xs, ys)))
        prog.run()
        if (e + 1) % a.sync_every == 0 or e == a.execs - 1:
            prog.sync()
            dt = time.perf_counter() - t0
            if hasattr(comm, "error_bits"):       # PeerXgmiCommunicator: one entry per local replica
                bits = comm.error_bits()
                eps = [comm.calls(i) for i in range(nl)]
            elif hasattr(comm, "err"):            # XgmiCommunicator: one rank per process
                bits = [comm.lib.tde_xgmi_error(comm.err)]
                eps = [comm.calls()]
            else:
                bits = eps = None
            print(f"{tag} exec {e} {dt * 1e3:.2f} ms err={bits} epochs={eps}", flush=True)
            ht = getattr(prog, "_host_trace", None)
            if ht:   # host wall clock (shared by the workers) of this execution's all-reduce enqueues
                print(f"{tag} exec {e} host enqueue t%1000 = " + " ".join(f"{t % 1000:.4f}" for _, t in ht), flush=True)
                ht.clear()
            if bits and any(bits):
                print(f"{tag} STOP: error bits set", flush=True)
                break
    tr = getattr(comm, "trace", None)
    if tr:   # TDE_XGMI_TRACE=<calls>: per-block phase times of the recorded calls (device clock, us)
        from tensorflow_distributed_example_amd.parallel.comm import xg_trace_records
        torch.cuda.synchronize()
        nb = {}
        for li, buf in enumerate(tr):
            recs = xg_trace_records(buf, buf.shape[1])
            bad = [r for r in recs if any(m != 255 for m in r["miss1"] + r["miss2"])]
            for r in recs[: a.trace_show] + bad[:4]:
                used = [i for i, v in enumerate(r["start"]) if v]
                us = lambda k: [r[k][i] / 100.0 for i in used]   # noqa: E731
                mn = lambda k: min(us(k)) if used else 0.0         # noqa: E731
                mx = lambda k: max(us(k)) if used else 0.0         # noqa: E731
                miss = sorted({(r["miss1"][i], r["miss2"][i]) for i in used} - {(255, 255)})
                print(f"{tag} rank{li} epoch {r['epoch']} blocks {len(used)} start [{mn('start'):.1f}, "
                      f"{mx('start'):.1f}] pub1<= {mx('pub1'):.1f} arr1 [{mn('arr1'):.1f}, {mx('arr1'):.1f}] "
                      f"pub2<= {mx('pub2'):.1f} arr2<= {mx('arr2'):.1f} end<= {mx('end'):.1f} missing={miss} "
                      f"xcc={sorted(set(r['xcc'][i] for i in used))}", flush=True)
                if r in bad:   # per block: which source, the flag value seen, where the block ran
                    for i in used:
                        if r["miss1"][i] != 255 or r["miss2"][i] != 255:
                            print(f"{tag}   blk {i} miss1={r['miss1'][i]} seen1={r['seen1'][i]} "
                                  f"miss2={r['miss2'][i]} seen2={r['seen2'][i]} xcc={r['xcc'][i]} "
                                  f"start={r['start'][i] / 100.0:.1f} arr1={r['arr1'][i] / 100.0:.1f}", flush=True)
    print(f"{tag} done", flush=True)


if __name__ == "__main__":
    main()
