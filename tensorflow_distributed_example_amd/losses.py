"""Losses: SparseCategoricalCrossentropy and its string alias.

Keras semantics (distributed_with_keras.py:41, mnist_keras_distributed.py:114,
tf2_mnist_distributed.py:81-83):
  * ``from_logits=True``: softmax-CE on logits.
  * ``from_logits=False`` on the output of a softmax activation: computed from the
    pre-softmax logits (stable; quirk Q5).  On other probabilities: clip to
    [eps, 1-eps] and take -log p.
  * reduction AUTO/SUM_OVER_BATCH_SIZE: under a distribution strategy the
    per-replica loss is sum / GLOBAL batch, so SUM-all-reduced gradients equal
    the mean gradient.  NONE returns per-sample losses.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

EPSILON = 1e-7


class Reduction:
    AUTO = "auto"
    NONE = "none"
    SUM = "sum"
    SUM_OVER_BATCH_SIZE = "sum_over_batch_size"


class Loss:
    def __init__(self, reduction=Reduction.AUTO, name=None):
        self.reduction = reduction
        self.name = name

    def per_sample(self, y_true, y_pred, *, pred_is_logits=False):
        raise NotImplementedError

    def __call__(self, y_true, y_pred, sample_weight=None):
        ls = self.per_sample(y_true, y_pred)
        if sample_weight is not None:
            ls = ls * torch.as_tensor(sample_weight, dtype=ls.dtype, device=ls.device)
        if self.reduction == Reduction.NONE:
            return ls
        if self.reduction == Reduction.SUM:
            return ls.sum()
        return ls.sum() / max(ls.shape[0], 1)


class SparseCategoricalCrossentropy(Loss):
    def __init__(self, from_logits=False, reduction=Reduction.AUTO, name="sparse_categorical_crossentropy"):
        super().__init__(reduction, name)
        self.from_logits = from_logits

    def per_sample(self, y_true, y_pred, *, pred_is_logits=False):
        y = torch.as_tensor(y_true, device=y_pred.device).reshape(-1).long()
        if self.from_logits or pred_is_logits:
            return F.cross_entropy(y_pred.float(), y, reduction="none")
        p = y_pred.float().clamp(EPSILON, 1 - EPSILON)
        return -torch.log(p.gather(1, y[:, None]).squeeze(1))

    def get_config(self):
        return {"from_logits": self.from_logits, "reduction": self.reduction, "name": self.name}


def get(identifier):
    if isinstance(identifier, Loss):
        return identifier
    if identifier in ("sparse_categorical_crossentropy", "SparseCategoricalCrossentropy"):
        return SparseCategoricalCrossentropy()
    raise ValueError(f"unsupported loss {identifier!r}")
