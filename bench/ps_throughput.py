#!/usr/bin/env python
"""ParameterServerStrategy throughput (reference mnist_keras_distributed.py:242,
tf2_mnist_distributed.py:189): async PS training of Model B through the Estimator on a localhost cluster.

    python -m tensorflow_distributed_example_amd.launch --ps 1 --master 1 --workers 1 --timeout 600 \
        bench/ps_throughput.py --max-steps 2000

Every task runs this script; the ps task serves variables (csrc/ps/param_server.cpp), master and worker
train asynchronously (pull -> fwd/bwd on the local device -> push; the PS applies SGD).  The master times
the GLOBAL step (counted over all workers) from ``--warm`` to the end and prints one JSON line:
global steps/sec and images/sec (steps/s x batch), plus each trainer's own step rate.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _RateHook:
    def __init__(self, warm):
        self.warm = warm
        self.t0 = self.s0 = None
        self.local = 0
        self.lt0 = None

    def begin(self, ctx):
        pass

    def after_step(self, ctx):
        self.local += 1
        if self.t0 is None and ctx.global_step >= self.warm:
            self.t0, self.s0, self.lt0, self.l0 = time.perf_counter(), ctx.global_step, time.perf_counter(), self.local

    def end(self, ctx):
        self.t1, self.s1, self.l1 = time.perf_counter(), ctx.global_step, self.local


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-steps", type=int, default=2000)
    ap.add_argument("--warm", type=int, default=100)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--model", default="mnist_bn_cnn")
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--momentum", type=float, default=0.0)
    # K > 1: K consecutive train() sessions against the same ps tasks (max_steps = max_steps * (s + 1) / K),
    # the last one timed — every session must end at exactly its max_steps on the plane the first one chose
    ap.add_argument("--sessions", type=int, default=1)
    a, _ = ap.parse_known_args()
    import numpy as np

    import tensorflow_distributed_example_amd as tde
    from tensorflow_distributed_example_amd.parallel import cluster as CL

    CL.translate_launcher_env()
    cfg = json.loads(os.environ.get("TF_CONFIG", "{}"))
    task = cfg.get("task", {})
    role = task.get("type")
    if role == "ps":
        from tensorflow_distributed_example_amd.parallel.ps import run_ps_server
        run_ps_server(cfg["cluster"]["ps"][task.get("index", 0)], index=task.get("index", 0))
        return
    tde.backend.set_random_seed(1)
    rng = np.random.default_rng(5 + int(task.get("index", 0)))
    n = 60000
    x = rng.random((n, 784), dtype=np.float32)
    y = rng.integers(0, 10, (n, 1)).astype(np.int32)
    model = getattr(tde.zoo, a.model)()
    model.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=a.model != "mnist_bn_cnn"),
                  optimizer=tde.optimizers.SGD(learning_rate=a.lr, momentum=a.momentum), metrics=["accuracy"])
    rc = tde.estimator.RunConfig(
        experimental_distribute=tde.contrib.distribute.DistributeConfig(
            train_distribute=tde.contrib.distribute.ParameterServerStrategy()),
        model_dir=tempfile.mkdtemp(prefix="ps_bench_"), save_summary_steps=10 ** 9,
        log_step_count_steps=10 ** 9, save_checkpoints_steps=10 ** 9)
    est = tde.keras.estimator.model_to_estimator(keras_model=model, config=rc)

    def input_fn():
        return tde.data.Dataset.from_tensor_slices((x, y)).shuffle(1000).repeat().batch(a.batch).prefetch(100)

    ends, planes = [], []
    for s in range(a.sessions - 1):
        h0 = _RateHook(10 ** 12)
        est.train(input_fn, hooks=[h0], max_steps=a.max_steps * (s + 1) // a.sessions)
        ends.append(h0.s1)
        planes.append(getattr(est, "ps_data_plane", "tcp"))
    warm = a.warm + (a.max_steps * (a.sessions - 1) // a.sessions)
    hook = _RateHook(warm)
    est.train(input_fn, hooks=[hook], max_steps=a.max_steps)
    ends.append(hook.s1)
    planes.append(getattr(est, "ps_data_plane", "tcp"))
    dt = hook.t1 - hook.t0
    rate = (hook.s1 - hook.s0) / dt
    local = (hook.l1 - hook.l0) / (hook.t1 - hook.lt0)
    role = role or "local"
    print(f"[ps_bench] {role}:{task.get('index', 0)} local steps/s {local:.1f}", flush=True)
    if role in ("master", "chief", "local"):
        trainers = sum(len(cfg.get("cluster", {}).get(j, [])) for j in ("chief", "master", "worker")) or 1
        print(json.dumps({"metric": "PS async global steps/sec (Model B, localhost cluster)",
                          "value": round(rate, 1), "unit": "global steps/sec",
                          "images_per_sec": round(rate * a.batch, 1), "trainers": trainers,
                          "ps_tasks": len(cfg.get("cluster", {}).get("ps", [])), "batch": a.batch,
                          "model": a.model, "steps_timed": hook.s1 - hook.s0, "master_local_steps_per_sec":
                          round(local, 1), "device": str(model._store.device), "final_global_step": hook.s1,
                          "momentum": a.momentum, "data_plane": getattr(est, "ps_data_plane", "tcp"),
                          "pipelined": os.environ.get("TDE_PS_PIPELINE", "1") != "0",
                          "sessions": a.sessions, "session_end_steps": ends, "session_planes": planes}),
              flush=True)


if __name__ == "__main__":
    main()
