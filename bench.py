#!/usr/bin/env python
"""Headline benchmark: whole-job MNIST-CNN training images/sec on N MI355X GPUs.

Metric/config from BASELINE.json: "images/sec (whole node) MNIST CNN at 1/2/4/8
MI355X; step time ms".  Model = the reference's Keras MNIST CNN
(distributed_with_keras.py:33-43: Conv2D(32,3,relu) · MaxPool · Flatten ·
Dense(64,relu) · Dense(10), SCCE(from_logits), SGD(0.001)), random-init weights,
synthetic 28x28x1 inputs, per-GPU batch 64 (the reference's BATCH_SIZE per
worker, distributed_with_keras.py:13) -> weak scaling, global batch 64*N.
Distribution: MultiWorkerMirroredStrategy, one process per GPU, RCCL gradient
all-reduce over xGMI.  Every timed step runs the full forward, backward, gradient
all-reduce and SGD update.  Precision: float32 by default — the reference's
(distributed_with_keras.py:21), exact-f32 MFMA kernels over the f32 weights;
``--dtype bf16`` runs the mixed_bfloat16 kernel forms (bf16 MFMA, fp32 master weights).

    python bench.py [--gpus N] [--steps K] [--warmup W]     # N>1: MirroredStrategy, one process, N GPUs
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...   # MWMS, one process per GPU
"""
from __future__ import annotations

import argparse
import gc
import json
import math
import os
import sys
import time

METRIC = "images/sec (whole node) MNIST CNN at 1/2/4/8 MI355X; step time ms"


# model -> (per-GPU batch, steps_per_execution, lr, from_logits, image shape, metric); batches follow the
# reference: 64 per worker (distributed_with_keras.py:13), 128 per replica (mnist_keras_distributed.py:50-54)
MODELS = {
    "mnist_cnn": (64, 16, 0.001, True, (28, 28, 1), METRIC),
    "mnist_bn_cnn": (128, 16, 0.01, False, (784,), METRIC),
    # width variants (user edits of the reference models; the layer-wise plan or a generalised fused plan)
    "mnist_cnn_wide": (64, 16, 0.001, True, (28, 28, 1),
                       "images/sec (whole node) MNIST CNN Conv2D(64)/Dense(128) at 1/2/4/8 MI355X; step time ms"),
    "mnist_bn_cnn_x2": (128, 16, 0.01, False, (784,),
                        "images/sec (whole node) MNIST BN-CNN 2x widths at 1/2/4/8 MI355X; step time ms"),
    # the LeNet-5 label carries the precision actually run ({dtype}: fp32 by default, bf16 with --dtype bf16)
    "lenet5": (128, 16, 0.01, True, (28, 28, 1), "images/sec (whole node) MNIST LeNet-5 CNN {dtype} at 1/2/4/8 MI355X; step time ms"),
    "mnist_mlp": (128, 16, 0.01, True, (28, 28, 1), "images/sec (whole node) MNIST dense MLP at 1/2/4/8 MI355X; step time ms"),
    "resnet18": (64, 1, 0.1, True, (224, 224, 3),   # BASELINE.json names this config bf16
                 "images/sec (whole node) synthetic 224x224x3 ResNet-18 bf16 at 1/2/4/8 MI355X; step time ms"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of the job (default 1; with --devices: the length of that list)")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=64)
    ap.add_argument("--model", default="mnist_cnn", choices=sorted(MODELS))
    ap.add_argument("--batch-per-gpu", type=int, default=None)
    ap.add_argument("--spe", type=int, default=None, help="steps_per_execution (steps per hipGraph replay)")
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--executor", default=None, help="fused|reference (default: fused on GPU)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--dtype", choices=("fp32", "bf16"), default=None,
                    help="compute precision (default fp32; resnet18: bf16, as its BASELINE config)")
    ap.add_argument("--strategy", choices=("mwms", "mirrored"), default="mwms",
                    help="mwms: one process per GPU (torchrun; default); mirrored: ONE process driving --gpus "
                         "local GPUs (MirroredStrategy, in-process xGMI all-reduce, one hipGraph per GPU)")
    ap.add_argument("--gpus-per-worker", type=int, default=1,
                    help="mwms: local GPUs per worker process (torchrun --nproc-per-node = gpus / K)")
    ap.add_argument("--repeats", type=int, default=5,
                    help="after the reported measurement, repeat the K-step measurement R times (spread only)")
    ap.add_argument("--devices", default=None,
                    help="mirrored: explicit local device list, e.g. 0,1,2,3 (0,0 = a 2-replica rehearsal on one GPU)")
    return ap.parse_args()


def main():
    a = parse()
    if a.gpus is None:
        a.gpus = len(a.devices.split(",")) if a.devices else 1
    if a.no_graph:
        os.environ["TDE_GRAPH"] = "0"
    if a.executor:
        os.environ["TDE_EXECUTOR"] = a.executor
    import numpy as np
    import torch

    import tensorflow_distributed_example_amd as tde

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.strategy == "mwms" and world == 1 and a.gpus > max(1, a.gpus_per_worker):
        # `python bench.py --gpus N` with no launcher: ONE process drives N local GPUs with MirroredStrategy
        # (BASELINE config 3, "MNIST CNN MirroredStrategy on 8xMI355X"; the reference's in-process
        # strategy, mnist_keras_distributed.py:243).  torchrun keeps the one-process-per-GPU MWMS path.
        a.strategy = "mirrored"
    gpw = max(1, a.gpus_per_worker) if a.strategy == "mwms" else a.gpus
    if a.strategy == "mwms" and world * gpw != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} != WORLD_SIZE {world} x --gpus-per-worker {gpw}")
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device((local_rank * gpw) % torch.cuda.device_count())  # ranks > GPUs only in rehearsals
    tde.backend.set_random_seed(1234)
    dtype = a.dtype or ("bf16" if a.model == "resnet18" else "fp32")
    tde.backend.set_global_policy("float32" if dtype == "fp32" else "mixed_bfloat16")
    if a.strategy == "mirrored":
        if world != 1:
            raise SystemExit("--strategy mirrored runs in ONE process (no torchrun)")
        if a.devices:
            devs = [f"cuda:{d}" if d.isdigit() else d for d in a.devices.split(",")]
        elif torch.cuda.is_available():
            # fewer GPUs than --gpus (a 1-GPU box): replicas wrap onto the visible devices, a rehearsal of
            # the N-GPU layout (several replicas time-share a device; reported as distinct_devices)
            nd = torch.cuda.device_count()
            devs = [f"cuda:{i % nd}" for i in range(a.gpus)]
        else:
            devs = ["cpu"] * a.gpus   # CPU plumbing (tests/test_bench_contract.py)
        if len(devs) != a.gpus:
            raise SystemExit(f"--devices lists {len(devs)} devices for --gpus {a.gpus}")
        strategy = tde.distribute.MirroredStrategy(devs)
    else:
        strategy = tde.distribute.MultiWorkerMirroredStrategy(gpus_per_worker=gpw if gpw > 1 else None)
    n = strategy.num_replicas_in_sync
    n_local = strategy.num_local_replicas
    dB, dspe, dlr, from_logits, img, metric = MODELS[a.model]
    metric = metric.replace("{dtype}", dtype)
    B = a.batch_per_gpu or dB
    GB = B * n
    spe = a.spe or dspe
    if a.spe is None and dspe > 1 and a.steps <= 128:
        spe = a.steps   # short runs (the driver's --steps 20): the whole timed region is one graph replay
    a.lr = a.lr if a.lr is not None else dlr
    while a.steps % spe:
        spe -= 1
    with strategy.scope():
        model = getattr(tde.zoo, a.model)()
        model.compile(loss=tde.losses.SparseCategoricalCrossentropy(from_logits=from_logits),
                      optimizer=tde.optimizers.SGD(learning_rate=a.lr), metrics=["accuracy"],
                      steps_per_execution=spe)
    ncls = model.output_shape[-1]
    prog = model._program("train", GB)
    dev = strategy.local_devices[0]
    in_shape = prog.x_shape
    # Synthetic MNIST-shaped data resident on the device: a pool of batches,
    # staged into the program's input ring once per execution (D2D copy).
    pool_execs = 4
    xs, ys = [], []
    for r in range(n_local):   # replica r's batches live on its device
        g = torch.Generator(device="cpu").manual_seed(1000 + strategy.global_replica_id(r))
        xs.append(torch.rand((pool_execs, spe, B) + tuple(in_shape), generator=g).to(strategy.local_devices[r]))
        ys.append(torch.randint(0, ncls, (pool_execs, spe, B), generator=g).to(torch.int32)
                  .to(strategy.local_devices[r]))

    # Input pipeline with prefetch (tf.data ``prefetch``): execution i replays the step graph on the batch
    # group already in the input ring, and the next group is staged right behind it on the same stream
    # (it cannot overwrite the ring before the replay has read it), so staging overlaps the host's wait.
    def stage(i):
        k = i % pool_execs
        prog.stage([(xs[r][k], ys[r][k]) for r in range(n_local)])

    def run_exec(i, prefetch=True):
        prog.run()
        if prefetch:
            stage(i + 1)

    def barrier():
        strategy.barrier()   # the native control plane (parallel/control.py); no-op at 1 worker

    # warm-up: at least W steps, at least 2 executions (the first replay follows the capture) and at
    # least TDE_BENCH_WARM_MS of back-to-back work.  A GPU that idled runs the next ~0.5 ms of work
    # 25-35% slower (bench/short_run.py: 20-step device time 585-629 us after a 50 ms idle gap vs
    # 467-480 us after >= 1 ms of warm-up; profiles/r2_short_run.json), which alone decided the
    # driver's 20-step number (1.5-2.4 M img/s across boxes at 2 executions of warm-up).
    # Every rank runs the same number of executions (each holds collectives): the count is fixed from
    # the timed first two and agreed as the max over ranks.
    n_warm = max(2, math.ceil(a.warmup / spe))
    warm_s = float(os.environ.get("TDE_BENCH_WARM_MS", "200")) * 1e-3
    stage(0)
    run_exec(0)
    prog.sync()
    tw = time.perf_counter()
    run_exec(1, prefetch=False)
    prog.sync()
    per_exec = max(time.perf_counter() - tw, 1e-6)
    n_warm = max(n_warm, 2 + math.ceil(warm_s / per_exec))
    if world > 1:
        n_warm = int(strategy.control.all_reduce_max(n_warm))
    # no cyclic-GC pass inside a timed window (a collection is a host pause of up to ~1 ms against a 0.47 ms
    # 20-step window): collect now, BEFORE the warm-up — a collection between the warm-up and the window would
    # idle the GPU, and an idle GPU runs the next ~0.5 ms of work slowly (the warm-up note above) — and pause the collector until
    # the windows are done
    gc.collect()
    gc.disable()
    if n_warm > 2:
        stage(2)
    for i in range(2, n_warm):
        run_exec(i, prefetch=i + 1 < n_warm)
        if i % 8 == 0:
            prog.sync()   # bounded queue depth; the GPU never idles for long
    n_exec = a.steps // spe

    def timed(first):
        """K steps bracketed by a barrier + device sync on both sides; max over ranks.  The first timed
        execution's input group is staged inside the timed region (short and long runs count the same
        input work per execution); later ones overlap the previous replay."""
        prog.sync()
        barrier()
        prog.sync()
        t0 = time.perf_counter()
        stage(first)
        for i in range(n_exec):
            run_exec(first + i, prefetch=i + 1 < n_exec)
        prog.sync()
        barrier()
        el = time.perf_counter() - t0
        return strategy.control.all_reduce_max(el) if world > 1 else el

    try:
        elapsed = timed(n_warm)
        # spread evidence (outside the reported measurement): the same K-step measurement repeated
        repeats = [timed(n_warm + n_exec * (r + 1)) for r in range(max(0, a.repeats))]
    finally:
        gc.enable()
    logs = tde.metrics.logs_from(prog.global_metrics(), ["accuracy"])
    comm = strategy.comm
    ar = {"XgmiCommunicator": "xgmi", "PeerXgmiCommunicator": "xgmi_peer", "RcclCommunicator": "rccl",
          "StoreCommunicator": "store", "LocalCommunicator": "local"}.get(
        type(comm).__name__, "none")
    if n > 1:  # data-parallel invariant (outside the timed region): every replica bit-identical
        from tensorflow_distributed_example_amd.utils import debug
        fps = debug.replica_fingerprints(model)
        same = all(f[2] == fps[0][2] for f in fps)   # trainable weights (BN moving stats are per replica)
        if strategy.worker_index == 0:
            print(f"[bench] replicas_identical={same}", file=sys.stderr, flush=True)
    # where the optimizer update runs: fused into the step's kernels (1 replica), into the xGMI
    # gradient all-reduce (one replica per process), or its own multi-tensor launch
    placement = {"local": "in_step_kernels", "xgmi": "allreduce"}.get(prog.plans[0].step_mode, "separate")
    distinct = len({str(d) for d in strategy.local_devices}) * strategy.num_workers
    # n_gpus = the replicas the job runs (one per GPU on a real node); a rehearsal whose replicas share a
    # device says so in config.distinct_devices
    n_dev = n if a.strategy == "mirrored" else distinct
    ms = elapsed / a.steps * 1e3
    ips = GB * a.steps / elapsed
    if strategy.worker_index == 0:
        print(f"[bench] plan={prog.plan_kind} graph={prog.use_graph} spe={spe} world={n} local={n_local} "
              f"loss={logs['loss']:.4f} acc={logs['accuracy']:.4f}", file=sys.stderr)
        print(json.dumps({
            "metric": metric, "value": round(ips, 1), "unit": "images/sec", "n_gpus": n_dev, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms, 5), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": prog.plans[0].compute_dtype,
            "data": f"synthetic (random {'x'.join(map(str, img))} images, random labels; random-init weights)",
            "config": {"model": a.model, "global_batch": GB, "seq_len": None, "image_shape": list(img),
                       "per_gpu_batch": B, "parallelism": f"dp{n}", "strategy": strategy.name,
                       "replicas": n, "replicas_per_process": n_local, "distinct_devices": distinct,
                       "graphs_per_execution": (len(prog.groups) if prog.per_replica else 1) if prog.use_graph else 0,
                       "steps_per_execution": spe, "warmup_steps_run": n_warm * spe,
                       "input_staged_in_timed_region": True,
                       "optimizer": f"SGD(lr={a.lr})", "plan": prog.plan_kind,
                       "allreduce": ar,
                       "hipgraph": prog.use_graph, "grad_buckets": len(prog.buckets or prog.group_buckets or []) or 1,
                       # the same K-step measurement repeated after the reported one (ms/step; spread evidence)
                       "repeat_ms_per_step": [round(r / a.steps * 1e3, 5) for r in repeats],
                       "optimizer_placement": placement,
                       # fused_push: the backward stores the Dense(64) weight gradient straight into the
                       # xGMI owners' windows; post_backward: the all-reduce launch pushes the whole bucket
                       "exchange": getattr(prog, "exchange", "none")}}), flush=True)


if __name__ == "__main__":
    main()
