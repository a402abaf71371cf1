"""Metrics: ``'accuracy'`` (sparse categorical accuracy) and the
running loss mean.

Accumulators are device-resident ``[loss_sum, correct, count, 0]`` f32 vectors
updated inside the fused head kernel (no host sync per step).  Across replicas
they are SyncOnRead/SUM: ``read()`` all-reduces them only when a value is read
(progbar refresh, epoch end, evaluation end — SURVEY §2.6 C3/C5).
"""
from __future__ import annotations

import torch


class SparseCategoricalAccuracy:
    name = "accuracy"


class Mean:
    name = "loss"


def resolve(metrics):
    out = []
    for m in metrics or []:
        if m in ("accuracy", "acc", "sparse_categorical_accuracy") or isinstance(m, SparseCategoricalAccuracy):
            out.append("accuracy")
        else:
            raise ValueError(f"unsupported metric {m!r}")
    return out


def logs_from(acc: torch.Tensor, names):
    a = acc.detach().double().cpu()
    cnt = float(a[2])
    logs = {"loss": float(a[0]) / cnt if cnt else float("nan")}
    if "accuracy" in names:
        logs["accuracy"] = float(a[1]) / cnt if cnt else float("nan")
    return logs
