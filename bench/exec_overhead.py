"""Per-execution overhead of a short timed region (the driver's ``bench.py --steps 20``).

Times one execution of S steps (stage + graph replay + sync) split into its host phases, and the
same execution with parts removed, so the fixed cost that a 20-step timed region pays on top of
S x (device step time) can be attributed:

    python bench/exec_overhead.py [--spe 20] [--reps 30]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import tensorflow_distributed_example_amd as tde  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spe", type=int, default=20)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--model", default="mnist_cnn")
    a = ap.parse_args()
    tde.backend.set_random_seed(1234)
    strategy = tde.distribute.MultiWorkerMirroredStrategy()
    with strategy.scope():
        model = getattr(tde.zoo, a.model)()
        model.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=tde.optimizers.SGD(learning_rate=0.001), metrics=["accuracy"],
                      steps_per_execution=a.spe)
    B = 64
    prog = model._program("train", B)
    dev = strategy.local_devices[0]
    xs = torch.rand((4, a.spe, B) + tuple(prog.x_shape), device=dev)
    xb = xs.to(prog.x_ring[0].dtype)
    ys = torch.randint(0, 10, (4, a.spe, B), device=dev).to(torch.int32)
    sync = torch.cuda.synchronize

    def timed(fn):
        out = []
        for i in range(a.reps):
            sync()
            t0 = time.perf_counter()
            phases = fn(i)
            sync()
            t1 = time.perf_counter()
            out.append((t1 - t0, phases))
        out.sort(key=lambda r: r[0])
        med = out[len(out) // 2]
        return {"total_us": round(med[0] * 1e6, 1), "phases_us": [round(p * 1e6, 1) for p in med[1]]}

    def full(i):
        t0 = time.perf_counter()
        prog.stage([(xs[i % 4], ys[i % 4])])
        t1 = time.perf_counter()
        prog.run()
        t2 = time.perf_counter()
        return (t1 - t0, t2 - t1)

    def bf16_data(i):
        t0 = time.perf_counter()
        prog.stage([(xb[i % 4], ys[i % 4])])
        t1 = time.perf_counter()
        prog.run()
        t2 = time.perf_counter()
        return (t1 - t0, t2 - t1)

    def replay_only(i):
        t0 = time.perf_counter()
        prog.run()
        return (time.perf_counter() - t0,)

    def stage_only(i):
        t0 = time.perf_counter()
        prog.stage([(xs[i % 4], ys[i % 4])])
        return (time.perf_counter() - t0,)

    # the bench's sequence on a fresh program: the first execution captures, then each later
    # replay timed on its own (does the n-th replay of a fresh graph cost more than the median?)
    seq = []
    for i in range(8):
        sync()
        t0 = time.perf_counter()
        full(i)
        sync()
        seq.append(round((time.perf_counter() - t0) * 1e6, 1))
    res = {"spe": a.spe, "model": a.model, "fresh_sequence_us": seq}
    for name, fn in (("full", full), ("bf16_data", bf16_data), ("replay_only", replay_only),
                     ("stage_only", stage_only), ("full_again", full)):
        res[name] = timed(fn)
    # device time of the graph alone (events around the replay), for the per-step floor
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for i in range(a.reps):
        sync()
        e0.record(st)
        prog.run()
        e1.record(st)
        sync()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    res["replay_event_us"] = round(ts[len(ts) // 2], 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
