"""Keras ``fit`` / ``evaluate`` / ``predict`` loops.

``fit(x=dataset, epochs=3, steps_per_epoch=5)`` (distributed_with_keras.py:63):
the dataset iterator persists across epochs when ``steps_per_epoch`` is given,
per-replica batches come from the strategy's distributed dataset, and each
group of ``steps_per_execution`` full steps runs as one program execution
(a single hipGraph replay on GPU).  Metrics are device accumulators; the
progbar shows the chief's local values, epoch-end logs are globally reduced.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from ..data.dataset import Dataset, _Batch
from ..data.distributed import DistributedDataset
from ..metrics import logs_from
from . import callbacks as CB
from ..utils import fault


def _global_batch_of(ds):
    d = ds.dataset if isinstance(ds, DistributedDataset) else ds
    while d is not None:
        if isinstance(d, _Batch):
            return d.batch_size
        d = d._parent
    return None


def _to_dataset(x, y, batch_size, shuffle, seed=None):
    if isinstance(x, (Dataset, DistributedDataset)):
        return x
    if y is None:
        raise ValueError("y is required when x is an array")
    ds = Dataset.from_tensor_slices((np.asarray(x), np.asarray(y)))
    if shuffle:
        ds = ds.shuffle(len(np.asarray(y)), seed=seed)
    return ds.batch(batch_size or 32)


def _fix_x(x, shape):
    x = np.asarray(x) if not torch.is_tensor(x) else x
    want = (x.shape[0],) + tuple(shape)
    if tuple(x.shape) != want:
        x = x.reshape(want)
    return x


def _split_xy(elem):
    if isinstance(elem, tuple):
        return elem[0], elem[1]
    if isinstance(elem, dict):
        return elem["image"], elem["label"]
    raise ValueError("training batches must be (x, y) tuples")


def _stack_steps(batches):
    """list over steps of per-replica [(x,y)] -> per-replica (x[S,...], y[S,...]); numpy steps stay
    lists (the stager packs them straight into its pinned buffer)."""
    R = len(batches[0])
    out = []
    for r in range(R):
        xs = [b[r][0] for b in batches]
        ys = [b[r][1] for b in batches]
        if torch.is_tensor(xs[0]):
            out.append((torch.stack(xs), torch.stack(ys)))
        else:
            out.append((xs, ys))
    return out


def fit(model, x=None, y=None, batch_size=None, epochs=1, verbose="auto", callbacks=None, validation_data=None,
        steps_per_epoch=None, initial_epoch=0, shuffle=True, validation_steps=None, validation_freq=1):
    strategy = model._strategy
    ds = _to_dataset(x, y, batch_size, shuffle)
    gb = _global_batch_of(ds)
    if gb is None:
        raise ValueError("the training dataset must be batched (dataset.batch(GLOBAL_BATCH_SIZE))")
    dds = ds if isinstance(ds, DistributedDataset) else strategy.experimental_distribute_dataset(ds)
    prog = model._program("train", gb)
    S = prog.S
    in_shape = prog.x_shape
    verbose = 1 if verbose == "auto" else verbose
    chief = strategy.is_chief
    hist = CB.History()
    cbs = [hist] + list(callbacks or [])
    if verbose and chief:
        cbs.append(CB.ProgbarLogger(verbose))
    cl = CB.CallbackList(cbs, model, {"epochs": epochs, "steps": steps_per_epoch, "verbose": verbose})
    model.history = hist
    model.stop_training = False
    model._resume_epoch = None
    cl.on_train_begin()
    if model._resume_epoch is not None:      # BackupAndRestore restored a finished epoch
        initial_epoch = max(initial_epoch, model._resume_epoch)
    it = None
    persist = steps_per_epoch is not None

    def next_batch():
        nonlocal it
        if it is None:
            it = iter(dds)
        try:
            b = next(it)
        except StopIteration:
            it = None
            return None
        per = []
        for elem in b:
            xx, yy = _split_xy(elem)
            per.append((_fix_x(xx, in_shape), np.asarray(yy).reshape(-1) if not torch.is_tensor(yy) else yy.reshape(-1)))
        return per

    logs = {}
    import os
    check_every = int(os.environ.get("TDE_CHECK_REPLICAS", "0") or 0)   # utils/debug.py
    # in-memory (x, y) datasets on GPU replicas: HBM-resident cache + on-device gather (train/device_feed.py)
    from .device_feed import DeviceFeed
    feed = DeviceFeed.try_make(dds, prog)
    model._device_feed = feed is not None
    n_exec = 0
    for epoch in range(initial_epoch, epochs):
        if not persist:
            it = None
            if feed is not None:
                feed.reset()
        prog.reset_metrics()
        cl.on_epoch_begin(epoch)
        step = 0
        exhausted = False
        while (steps_per_epoch is None or step < steps_per_epoch) and not exhausted:
            want = S if steps_per_epoch is None else min(S, steps_per_epoch - step)
            group = []
            while len(group) < want:
                b = next_batch() if feed is None else feed.next()
                if b is None:
                    exhausted = True
                    break
                group.append(b)
            if not group:
                break
            if feed is not None:   # per-replica row-index arrays
                full = [all(len(r) == prog.B for r in g) for g in group]
            else:
                full = [all(len(r[1]) == prog.B for r in g) for g in group]
            cl.on_train_batch_begin(step)
            if len(group) == S and all(full):
                if feed is not None:
                    feed.stage(group)
                else:
                    prog.stage(_stack_steps(group))
                prog.run()
            else:
                for g in group:
                    if feed is not None:
                        g = feed.host_batch(g)
                    glob = sum(len(r[1]) for r in g) * strategy.num_workers
                    prog.run_single(g, glob)
            step += len(group)
            n_exec += 1
            if check_every and n_exec % check_every == 0:
                from ..utils import debug
                prog.sync()
                debug.check_replicas(model, f"after step {model.optimizer.iterations + step}")
            fault.maybe_inject(model.optimizer.iterations + step)
            cl.on_train_batch_end(step - 1, logs_from(prog.local_metrics(), model._metric_names)
                                  if chief and verbose == 1 and _due(prog) else None)
        if steps_per_epoch is not None and step < steps_per_epoch and exhausted:
            print("WARNING: your input ran out of data; interrupting training. Make sure that your dataset can "
                  f"generate at least `steps_per_epoch * epochs` batches ({steps_per_epoch * epochs}).")
        logs = logs_from(prog.global_metrics(), model._metric_names)
        model.optimizer.iterations += step
        if validation_data is not None and (epoch + 1) % validation_freq == 0:
            vx, vy = (validation_data if isinstance(validation_data, tuple) else (validation_data, None))
            vlogs = evaluate(model, vx, vy, batch_size=batch_size, steps=validation_steps, verbose=0,
                             return_dict=True)
            logs.update({f"val_{k}": v for k, v in vlogs.items()})
        cl.on_epoch_end(epoch, logs)
        if model.stop_training:
            break
        if exhausted and persist:
            break
    prog.sync()
    if feed is not None:
        feed.check()
    cl.on_train_end(logs)
    return hist


_last_read = [0.0]


def _due(prog):
    now = time.perf_counter()
    if now - _last_read[0] > 0.25:
        _last_read[0] = now
        return True
    return False


def evaluate(model, x=None, y=None, batch_size=None, verbose="auto", steps=None, return_dict=False,
             callbacks=None):
    strategy = model._strategy
    ds = _to_dataset(x, y, batch_size, shuffle=False)
    gb = _global_batch_of(ds) or 32
    dds = ds if isinstance(ds, DistributedDataset) else strategy.experimental_distribute_dataset(ds)
    prog = model._program("eval", gb)
    prog.on_weights_loaded()
    prog.reset_metrics()
    in_shape = prog.x_shape
    n = 0
    for b in dds:
        per = []
        for elem in b:
            xx, yy = _split_xy(elem)
            per.append((_fix_x(xx, in_shape), np.asarray(yy).reshape(-1)))
        prog.eval_batch(per)
        n += 1
        if steps is not None and n >= steps:
            break
    logs = logs_from(prog.global_metrics(), model._metric_names)
    if verbose not in (0, "auto") and strategy.is_chief:
        print(" - ".join(f"{k}: {v:.4f}" for k, v in logs.items()))
    if return_dict:
        return logs
    return [logs["loss"]] + ([logs["accuracy"]] if "accuracy" in logs else [])


def predict(model, x, batch_size=None, verbose=0, steps=None):
    bs = batch_size or 32
    if isinstance(x, Dataset):
        batches = [(_split_xy(e)[0] if isinstance(e, (tuple, dict)) else e) for e in x]
        bs = max(len(b) for b in batches)
    else:
        x = np.asarray(x)
        batches = [x[i:i + bs] for i in range(0, len(x), bs)]
    prog = model._program("predict", bs, single_replica=True)
    prog.on_weights_loaded()
    outs = [prog.predict_batch(_fix_x(b, prog.x_shape)) for b in batches]
    return np.concatenate(outs) if outs else np.zeros((0,))
