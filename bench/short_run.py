"""Where does a short timed region (the driver's ``bench.py --steps 20 --warmup 5``) lose time?

One fresh process: build the bench's program, then time single 20-step executions (stage + graph
replay + sync, as bench.py does) after different amounts of back-to-back warm-up work, recording
for each the wall time and the device time of the replay (HIP events):

    python bench/short_run.py [--spe 20] [--trials 5]

Prints one JSON line: {warm_ms: [[wall_us, device_us], ...]} per warm-up budget.
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
    ap.add_argument("--trials", type=int, default=5)
    a = ap.parse_args()
    tde.backend.set_random_seed(1234)
    strategy = tde.distribute.MultiWorkerMirroredStrategy()
    with strategy.scope():
        model = tde.zoo.mnist_cnn()
        model.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=tde.optimizers.SGD(learning_rate=0.001), metrics=["accuracy"],
                      steps_per_execution=a.spe)
    B = 64
    prog = model._program("train", B)
    dev = strategy.local_devices[0]
    xs = torch.rand((4, a.spe, B) + tuple(prog.x_shape), device=dev)
    ys = torch.randint(0, 10, (4, a.spe, B), device=dev).to(torch.int32)
    sync = torch.cuda.synchronize
    st = torch.cuda.current_stream()

    def run_exec(i):
        prog.stage([(xs[i % 4], ys[i % 4])])
        prog.run()

    # the bench's own warm-up: capture + one replay
    t0 = time.perf_counter()
    run_exec(0)
    run_exec(1)
    sync()
    res = {"spe": a.spe, "capture_and_first_ms": round((time.perf_counter() - t0) * 1e3, 2)}

    def timed_once(i):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        sync()
        t0 = time.perf_counter()
        e0.record(st)
        run_exec(i)
        e1.record(st)
        sync()
        wall = (time.perf_counter() - t0) * 1e6
        return [round(wall, 1), round(e0.elapsed_time(e1) * 1e3, 1)]

    # first timed execution exactly as bench.py's (right after its 2 warm-up executions)
    res["bench_like"] = timed_once(2)
    for warm_ms in (0, 1, 5, 20, 100, 400):
        out = []
        for t in range(a.trials):
            # idle gap like a fresh region start, then warm-up replays for warm_ms of wall time
            time.sleep(0.05)
            t0 = time.perf_counter()
            n = 0
            while (time.perf_counter() - t0) * 1e3 < warm_ms:
                run_exec(n)
                n += 1
                if n % 8 == 0:
                    sync()
            out.append(timed_once(n))
        res[f"warm_{warm_ms}ms"] = out
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
