"""Per-replica execution plans and the multi-step training program.

A *plan* executes one replica's work for one step on one device:

* ``ConvNetPlan`` (GPU): the DWK/TF2M small CNN as five
  fused gfx950 HIP kernels —
      conv+bias+ReLU+maxpool (VALU)  → Dense split-K MFMA (atomic f32)
      → head: bias+ReLU, Dense, softmax-CE, accuracy, and the whole head backward
      → dW of the big Dense (MFMA) → conv backward with the Dense input-gradient
        computed in-kernel (MFMA) and routed through pool argmax / ReLU mask;
  followed by the RCCL all-reduce of the flat gradient bucket and ONE
  multi-tensor optimizer kernel.
* ``LayerwisePlan`` (GPU): any Sequential model built from the supported layers,
  one HIP kernel family per layer (ops/layerwise.py) — Model B, ResNet-18.
* ``ReferencePlan`` (CPU, or GPU when explicitly requested for testing): torch
  ops + autograd — the CPU backend's kernel library and the numerics oracle.

``TrainProgram`` strings ``steps_per_execution`` steps (Keras
``compile(steps_per_execution=N)``) of every local replica together with the
gradient all-reduce and optimizer, and on a single-local-replica GPU captures the
whole N-step sequence — RCCL collective included — into one hipGraph replayed
per execution, so the host issues one launch per N steps.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from .. import backend as Kb
from ..models import layers as L
from . import params as P


def _round8(n):
    return (n + 7) // 8 * 8


class ReplicaPlan:
    kind = "base"

    def __init__(self, model, store, device, batch, global_batch, optimizer):
        self.model = model
        self.store = store
        self.device = torch.device(device)
        self.B = int(batch)
        self.global_batch = int(global_batch)
        self.scale = 1.0 / float(global_batch)
        self.optimizer = optimizer
        self.metrics = torch.zeros(4, dtype=torch.float32, device=self.device)
        self.iterations = torch.zeros(1, dtype=torch.int64, device=self.device)
        for s in optimizer.slot_names() if optimizer is not None else []:
            store.slot(s)

    def reset_metrics(self):
        self.metrics.zero_()

    def train_step(self, x, y, B=None):
        raise NotImplementedError

    def apply(self):
        raise NotImplementedError

    def eval_step(self, x, y, B=None):
        raise NotImplementedError

    def predict(self, x, B=None):
        raise NotImplementedError

    def on_weights_loaded(self):
        pass

    # How the optimizer runs (set by the Program): "plain" — gradients land in the flat bucket and
    # ``apply()`` runs the multi-tensor optimizer; fused plans may also support "local" (the update
    # happens inside the step's own kernels; ``finish()`` flushes what is deferred) and "xgmi" (the
    # communicator's fused all-reduce applies it).
    step_mode = "plain"
    input_dtype = torch.float32   # dtype of the Program's input ring for this plan
    compute_dtype = "fp32"        # what the plan's kernels compute in ("fp32" | "bf16"; bench / logs)
    parity = 0   # step parity of plans that double-buffer across steps (one hipGraph per start parity)

    def supports_step_mode(self, mode):
        return mode == "plain"

    def set_step_mode(self, mode):
        if not self.supports_step_mode(mode):
            raise ValueError(f"{self.kind} plan does not support step mode {mode!r}")
        self.step_mode = mode

    @property
    def applies_in_step(self):
        return self.step_mode == "local"

    def finish(self):
        """End of an execution (a run of steps): commit deferred updates."""

    def trace_tensors(self):
        """State recorded per step by ``Program.enable_trace`` (diagnostics)."""
        return [self.store.w, self.metrics]

    def refresh(self):
        """Before an execution is launched or captured: pick up optimizer hyper-parameter changes."""


# ---------------------------------------------------------------------------------------
def _last_softmax(model, loss):
    last = model.layers[-1]
    act = getattr(last, "activation", None)
    if act == "softmax" and not getattr(loss, "from_logits", False):
        return True
    return False


class ReferencePlan(ReplicaPlan):
    kind = "reference"

    def __init__(self, model, store, device, batch, global_batch, optimizer, loss):
        super().__init__(model, store, device, batch, global_batch, optimizer)
        self.loss = loss
        self.strip_softmax = _last_softmax(model, loss)
        self.rng = Kb.make_generator(1234)

    def _weights(self, wl):
        W = {}
        st = self.store
        for layer in self.model.layers:
            d = {}
            for s in layer.weight_specs:
                seg = st.segments[s.full_name]
                if seg.trainable and wl is not None:
                    d[s.name] = wl[seg.offset: seg.offset + seg.numel].view(seg.shape)
                else:
                    d[s.name] = st.view(s.full_name)
            W[layer.name] = d
        return W

    def _forward(self, x, W, training, updates=None):
        t = {0: x.float()}
        nodes = self.model._nodes()
        for i, (layer, ins, out) in enumerate(nodes):
            h = [t[j] for j in ins] if layer.multi_input else t[ins[0]]
            if i == len(nodes) - 1 and self.strip_softmax:
                act = layer.activation
                layer.activation = None
                try:
                    t[out] = layer.ref_call(h, W[layer.name], training, self.rng, updates)
                finally:
                    layer.activation = act
            else:
                t[out] = layer.ref_call(h, W[layer.name], training, self.rng, updates)
        return t[nodes[-1][2]]

    def train_step(self, x, y, B=None):
        B = x.shape[0] if B is None else B
        x, y = x[:B], y[:B]
        wl = self.store.w.detach().requires_grad_(True)
        W = self._weights(wl)
        updates = []
        out = self._forward(x, W, True, updates)
        ls = self.loss.per_sample(y, out, pred_is_logits=self.strip_softmax)
        (ls.sum() * self.scale).backward()
        with torch.no_grad():
            self.store.g.add_(wl.grad)
            for name, val in updates:
                self.store.view(name).copy_(val)
            self._acc(out, y, ls)

    def _acc(self, out, y, ls):
        yy = torch.as_tensor(y, device=out.device).reshape(-1).long()
        correct = (out.argmax(dim=1) == yy).sum().float()
        self.metrics += torch.stack([ls.sum().float(), correct, torch.tensor(float(ls.shape[0]), device=out.device),
                                     torch.zeros((), device=out.device)])

    @torch.no_grad()
    def apply(self):
        st = self.store
        slots = {n: st.slot(n) for n in self.optimizer.slot_names()}
        self.optimizer.apply_reference(st.w, st.g, slots, int(self.iterations.item()))
        st.g.zero_()
        self.iterations += 1

    @torch.no_grad()
    def eval_step(self, x, y, B=None):
        B = x.shape[0] if B is None else B
        out = self._forward(x[:B], self._weights(None), False)
        ls = self.loss.per_sample(y[:B], out, pred_is_logits=self.strip_softmax)
        self._acc(out, y[:B], ls)

    @torch.no_grad()
    def predict(self, x, B=None):
        B = x.shape[0] if B is None else B
        out = self._forward(x[:B], self._weights(None), False)
        if self.strip_softmax:
            out = torch.softmax(out, dim=-1)
        return out


# ---------------------------------------------------------------------------------------
class OptimizerKernel:
    """Device-side state for the multi-tensor optimizer kernel of one replica."""

    def __init__(self, store: P.ParamStore, optimizer, shadows: dict, iterations):
        from .. import _native as N
        self.N = N
        self.store = store
        self.optimizer = optimizer
        self.iterations = iterations
        segs = []
        sh_total = 0
        self.shadow_views = {}
        layout = []
        for name in store.names(trainable=True):
            seg = store.segments[name]
            # 2-D view [prod(shape[:-1]), shape[-1]]: Dense [in, out] and conv HWIO as [KH*KW*Cin, Cout],
            # so the transposed ("col") shadow is the K-contiguous [out, K] operand of the forward GEMM
            rows, cols = (int(np.prod(seg.shape[:-1])), seg.shape[-1]) if len(seg.shape) >= 2 else (1, seg.numel)
            sh = sht = -1
            if name in shadows:
                want = shadows[name]
                if "row" in want:
                    sh = sh_total
                    sh_total += _round8(seg.numel)
                if "col" in want:
                    sht = sh_total
                    sh_total += _round8(seg.numel)
            segs.append((seg.offset, rows, cols, sh, sht))
            layout.append((name, rows, cols, sh, sht))
        self.shadow = torch.zeros(max(sh_total, 8), dtype=torch.bfloat16, device=store.device)
        for name, rows, cols, sh, sht in layout:
            if sh >= 0:
                self.shadow_views[(name, "row")] = self.shadow[sh: sh + rows * cols].view(rows, cols)
            if sht >= 0:
                self.shadow_views[(name, "col")] = self.shadow[sht: sht + rows * cols].view(cols, rows)
        dt = np.dtype([("off", "<i8"), ("rows", "<i4"), ("cols", "<i4"), ("sh", "<i8"), ("sht", "<i8")])
        arr = np.array(segs, dtype=dt)
        self._segs_host = arr
        lib = N.hip()
        nb = lib.tde_optim_table_size(arr.ctypes.data, len(arr))
        table = np.zeros((max(nb, 1), 4), dtype=np.int32)
        lib.tde_optim_build_table(arr.ctypes.data, len(arr), table.ctypes.data)
        self.nblocks = nb
        self.segs_dev = torch.from_numpy(arr.view(np.uint8).copy()).to(store.device)
        self.table_dev = torch.from_numpy(table).to(store.device)
        self.refresh_shadows()

    def refresh_shadows(self):
        if not self.shadow_views:   # f32 plans read the master weights: nothing to refresh
            return
        N = self.N
        with torch.cuda.device(self.store.device):
            rc = N.hip().tde_shadow_refresh(self.store.w.data_ptr(), self.shadow.data_ptr(),
                                            self.segs_dev.data_ptr(), self.table_dev.data_ptr(), self.nblocks,
                                            N.stream_ptr())
        N.check(rc, "tde_shadow_refresh")

    def apply(self, zero_grad=True):
        N = self.N
        st = self.store
        opt = self.optimizer
        hp = opt.hparams()
        m = st.slot(opt.slot_names()[0]) if opt.slot_names() else None
        v = st.slot(opt.slot_names()[1]) if len(opt.slot_names()) > 1 else None
        rc = N.hip().tde_optim_apply(st.w.data_ptr(), st.g.data_ptr(), N.ptr(m), N.ptr(v), self.shadow.data_ptr(),
                                     self.segs_dev.data_ptr(), self.table_dev.data_ptr(), self.nblocks,
                                     self.iterations.data_ptr(), opt.kind_id,
                                     float(opt.learning_rate), hp["mom"], hp["b1"], hp["b2"], hp["eps"], 1.0,
                                     int(zero_grad), None, N.stream_ptr())
        N.check(rc, "tde_optim_apply")


def f32_xg_apply_spec(plan):
    """``XgApply`` of a plan whose weights are the f32 master store only (no bf16 shadows): the xGMI
    all-reduce applies the optimizer to ``store.w`` / slots (step mode "xgmi")."""
    from ..ops import kernels as K
    st, opt = plan.store, plan.optimizer
    sl = opt.slot_names()
    m = st.slot(sl[0]) if sl else None
    v = st.slot(sl[1]) if len(sl) > 1 else None
    hp = opt.hparams()
    # the plan's step pushed part of the bucket into the owners itself (fused exchange; a replica without
    # data this step pushed nothing)
    lo, hi = plan.push_range() if (getattr(plan, "_push", None) is not None and getattr(plan, "_pushed", False)) \
        else (0, 0)
    if hasattr(plan, "_pushed"):
        plan._pushed = False
    return K.XgApply(opt.kind_id, float(opt.learning_rate), hp["mom"], hp["b1"], hp["b2"], hp["eps"],
                     K._P(st.w), K._P(m), K._P(v), K._P(plan.iterations), None, 0, 0, None, 0, 0, lo, hi)


def match_convnet(model, loss):
    """Pattern of the DWK/TF2M small CNN: Conv2D(3x3,relu,bias) on 1 channel ·
    MaxPooling2D(2) · Flatten · Dense(bias[,relu]) · Dense(bias[,softmax]) + SCCE."""
    from ..losses import SparseCategoricalCrossentropy
    ls = [l for l in model.layers if not isinstance(l, L.InputLayer)]
    if ls and isinstance(ls[0], L.Reshape) and len(ls[0].target_shape) == 3:
        ls = ls[1:]
    if len(ls) != 5 or not isinstance(loss, SparseCategoricalCrossentropy):
        return None
    c, p, f, d1, d2 = ls
    ok = (isinstance(c, L.Conv2D) and c.kernel_size == (3, 3) and c.strides == (1, 1) and c.padding == "valid"
          and c.activation == "relu" and c.use_bias and c.input_shape[-1] == 1
          and c.input_shape[1] % 2 == 0
          and isinstance(p, L.MaxPooling2D) and p.pool_size == (2, 2) and p.strides == (2, 2) and p.padding == "valid"
          and isinstance(f, L.Flatten)
          and isinstance(d1, L.Dense) and d1.activation in (None, "relu")
          and isinstance(d2, L.Dense) and d2.use_bias and d2.activation in (None, "softmax"))
    if not ok:
        return None
    if (d2.activation == "softmax") == bool(loss.from_logits):
        return None  # probabilities fed to from_logits=True (or logits w/o from_logits): not fusable
    force_gen = os.environ.get("TDE_CONVNET_GENERIC", "0") == "1"   # A/B: the generic kernels at any width
    if c.filters != 32 or d1.units != 64 or force_gen:
        # the hand-tuned step is the reference's Conv2D(32)/Dense(64) (distributed_with_keras.py:34,37);
        # other widths run the generic fused kernels (float32 policy, ConvNetGenPlan) when they fit them,
        # and say so instead of silently dropping to the slower per-layer plan otherwise
        H, W = c.input_shape[0], c.input_shape[1]
        why = None
        if Kb.global_policy().compute_dtype != torch.float32:
            why = "the generic widths are implemented for the float32 policy"
        elif not gen_fits(c.filters, d1.units):
            why = (f"Conv2D filters must be one of {GEN_FILTERS} and Dense units a multiple of 32 up to 256 whose "
                   "backward fits a CU's LDS (Conv2D(48): up to 192 units, Conv2D(64): up to 160)")
        elif d2.units > 16 or W % 4 or W > 32 or H % 2:
            why = "at most 16 classes and an even height, width a multiple of 4 up to 32"
        if why is None:
            return dict(conv=c, pool=p, dense1=d1, dense2=d2, generic=True)
        import warnings
        warnings.warn(f"model {model.name!r}: no fused small-CNN step for Conv2D({c.filters}) + Dense({d1.units}) "
                      f"({why}); running the per-layer kernel plan")
        return None
    if d2.units > 16:
        import warnings
        warnings.warn(f"model {model.name!r}: the fused small-CNN step takes at most 16 classes (got {d2.units}); "
                      "running the per-layer kernel plan")
        return None
    return dict(conv=c, pool=p, dense1=d1, dense2=d2)


GEN_FILTERS = (16, 32, 48, 64)      # csrc/kernels/convnet_gen.hip instantiations
GEN_UNITS = tuple(range(32, 257, 32))


def gen_fits(filters, units):
    """Whether the generic fused kernels are instantiated for Conv2D(filters) / Dense(units): the backward's
    LDS carve at 8 waves (csrc/kernels/convnet_gen.hip BwdCfg) within a CU's 160 KB."""
    if filters not in GEN_FILTERS or units not in GEN_UNITS:
        return False
    cc, hd = filters, units
    rg = hd + 4
    lds = (64 * rg * 4 + cc * rg * 4 + cc * 68 * 4 + 64 * 16 * 4 + 64 * cc + 64 * (cc + 4) * 4
           + max(4096 + 64 * 17 * 4, 8 * 10 * cc * 4) + hd * 17 * 4 + 16 * 4 + 64 * 4)
    return lds <= 160 * 1024


class ConvNetPlan(ReplicaPlan):
    """The DWK/TF2M small CNN as two HIP launches per training step, in the precision of the global
    policy: float32 (the reference's; csrc/kernels/convnet_f32.hip, exact-f32 MFMA over the f32 master
    weights) or mixed_bfloat16 (csrc/kernels/convnet.hip, bf16 MFMA over bf16 weight shadows):

      forward   conv+bias+ReLU+pool fused with the Dense(64) matmul (split-K atomics into hpre[p])
      backward  the head recomputed from hpre[p] in every workgroup (softmax-CE, dlogits, Dense(64)
                input gradient), Dense(64) weight / input gradients, pool / ReLU routing and conv
                gradients; one extra workgroup makes the head's own gradients and the metrics; the
                other parity buffer hpre[1-p] is zeroed for the next forward

    followed, by step mode, by the multi-tensor optimizer ("plain"), nothing ("local": the update
    runs inside the two launches, the conv update deferred to the next step and flushed by
    ``finish()``), or the xGMI all-reduce that applies it ("xgmi").  ``parity`` alternates per step;
    the Program captures one hipGraph per starting parity."""
    kind = "fused_convnet"

    def __init__(self, model, store, device, batch, global_batch, optimizer, loss, pattern):
        super().__init__(model, store, device, batch, global_batch, optimizer)
        from ..ops import kernels as K
        self.K = K
        self.loss = loss
        c, d1, d2 = pattern["conv"], pattern["dense1"], pattern["dense2"]
        self.c, self.d1, self.d2 = c, d1, d2
        self.f32 = Kb.global_policy().compute_dtype == torch.float32
        self.compute_dtype = "fp32" if self.f32 else "bf16"
        H, W = c.input_shape[0], c.input_shape[1]
        self.H, self.W, self.C = H, W, c.filters
        Hp, Wp = (H - 2) // 2, (W - 2) // 2
        self.Kf = Hp * Wp * self.C
        self.Hd, self.Cls = d1.units, d2.units
        B, Bp = self.B, _round8(self.B)
        self.Bp = Bp
        dev = self.device
        self.Pt = torch.zeros(self.Kf, Bp, dtype=torch.float32 if self.f32 else torch.bfloat16, device=dev)
        self.amax = torch.zeros(self.Kf // 32, 4, Bp, dtype=torch.int64, device=dev)  # [P][C/8][B] argmax bytes
        # Dense(64) pre-activation: two training buffers by step parity + one for eval / predict
        # (training buffers: hrep replicas each, so the forward's ~85 split-K adders per address spread out)
        self.hrep = max(1, min(8, int(os.environ.get("TDE_CONVNET_HREP", "4"))))
        # TDE_DETERMINISTIC=1 (debugging): one pre-activation replica per forward workgroup (each address
        # receives exactly one add, into zeros; the consumer sums the replicas in order) and the conv
        # gradients as per-workgroup partials summed in order by an extra launch: bitwise-reproducible
        # training steps at the cost of 2.8 MB of replicas and one launch per step
        self.det = os.environ.get("TDE_DETERMINISTIC", "0") not in ("", "0")
        P_ = ((H - 2) // 2) * ((W - 2) // 2)
        if self.det:
            self.hrep = P_
        self.cpart = torch.zeros((P_ + 1) * 320, dtype=torch.float32, device=dev) if self.det else None
        self.n_cpart = P_
        self.hpre2 = torch.zeros(2, self.hrep, B, self.Hd, dtype=torch.float32, device=dev)
        self.hpre = torch.zeros(B, self.Hd, dtype=torch.float32, device=dev)
        self.parity = 0
        self.probs = torch.zeros(B, self.Cls, dtype=torch.float32, device=dev)
        self.pre_relu = d1.activation == "relu"
        self.logits_out = d2.activation is None
        n = lambda l, w: f"{l.name}/{w}"  # noqa: E731
        self.names = dict(wc=n(c, "kernel"), bc=n(c, "bias"), w1=n(d1, "kernel"),
                          b1=n(d1, "bias") if d1.use_bias else None, w2=n(d2, "kernel"), b2=n(d2, "bias"))
        # bf16: the forward reads the Dense(64) kernel from the row-major bf16 shadow (the one the
        # backward reads and the fused updates rewrite); TDE_CONVNET_W1=col keeps a transposed [64, K]
        # copy for it.  f32: both read the f32 master kernel itself (no shadow exists).
        self.w1_rows = self.f32 or os.environ.get("TDE_CONVNET_W1", "rows") != "col"
        if self.f32:
            shadows = {}
        else:
            shadows = {self.names["w1"]: ("row",) if self.w1_rows else ("row", "col")}
        self.opt = OptimizerKernel(store, optimizer, shadows, self.iterations) if optimizer is not None else None
        self._shadow_only = None
        if self.opt is None and shadows:
            # eval/predict-only plan still needs the bf16 weight copies
            from ..optimizers import SGD
            self._shadow_only = OptimizerKernel(store, SGD(0.0), shadows, self.iterations)
        if self.f32:
            self.W1row = store.view(self.names["w1"])
            self.W1col = None
        else:
            ok = self.opt or self._shadow_only
            self.W1row = ok.shadow_views[(self.names["w1"], "row")]
            self.W1col = None if self.w1_rows else ok.shadow_views[(self.names["w1"], "col")]
        self.W1fwd = self.W1row if self.w1_rows else self.W1col
        # fused step ("local"): conv gradients by step parity (the deferred update of step t is read by
        # forward t+1 while backward t+1 accumulates the next), their pending flags, and the step count
        # the deferred update belongs to
        seg = store.segments
        sw, sb = seg[self.names["wc"]], seg[self.names["bc"]]
        self._conv_lo = min(sw.offset, sb.offset)
        span = max(sw.offset + sw.numel, sb.offset + sb.numel) - self._conv_lo
        # the ~170 backward workgroups add their conv-gradient partials into crep replicas (workgroup x ->
        # replica x % crep, summed by the consumers): same-address float atomics from every workgroup cost
        # ~4 us of the backward (TDE_CONVNET_GREP, 1 = one buffer; the deterministic mode keeps one)
        self.crep = 1 if self.det else max(1, min(8, int(os.environ.get("TDE_CONVNET_GREP", "8"))))
        self._conv_span = span
        # data-parallel step (mode "xgmi", float32 form): the replicas of parity 0 take the conv gradients
        # and the all-reduce sums them into its push (only when nothing else lies between the two segments)
        others = [n for n in store.order if n not in (self.names["wc"], self.names["bc"]) and
                  self._conv_lo <= seg[n].offset < self._conv_lo + span]
        self._xg_rep = self.f32 and self.crep > 1 and not others
        self.gconv = torch.zeros(2, self.crep, span, dtype=torch.float32, device=dev)
        self.pend = torch.zeros(2, dtype=torch.int32, device=dev)
        # device counters of the deferred conv update (the local step's invariants, ``step_invariants``):
        # [0] updates committed (by the next backward's head workgroup or the flush), [1] forwards that
        # applied a pending update on the fly
        self.ucount = torch.zeros(2, dtype=torch.int64, device=dev)
        # fused step: the head variables as of this step's forward ([b1 | W2 | b2], written by the forward),
        # read by the backward's trunk workgroups while its head workgroup updates the originals
        C_ = self.Cls
        self.hsnap = torch.zeros(64 + 64 * C_ + C_, dtype=torch.float32, device=dev)
        self._hs_b1 = self.hsnap[:64]
        self._hs_w2 = self.hsnap[64: 64 + 64 * C_].view(64, C_)
        self._hs_b2 = self.hsnap[64 + 64 * C_:]
        self.iter_prev = torch.zeros(1, dtype=torch.int64, device=dev)
        self._fopt = self._bopt = self._flush = None
        # step mode "xgmi" with the fused exchange (set_push): the backward stores dW1 straight into the
        # xGMI owners' contribution areas; _pushed marks that the step's launch did so (xg_apply_spec)
        self._push = None
        self._pushed = False

    # ------------------------------------------------------------------ fused step modes
    def supports_step_mode(self, mode):
        if mode == "plain":
            return True
        return self.optimizer is not None and self.device.type == "cuda" and mode in ("local", "xgmi")

    def _gconv(self, q):
        """Pointer that indexes parity q's conv gradients with the flat-buffer offsets."""
        return self.gconv[q].data_ptr() - 4 * self._conv_lo

    def _gconv_views(self, q):
        seg = self.store.segments
        sw, sb = seg[self.names["wc"]], seg[self.names["bc"]]
        lo = self._conv_lo
        return (self.gconv[q, 0, sw.offset - lo: sw.offset - lo + sw.numel].view(sw.shape),
                self.gconv[q, 0, sb.offset - lo: sb.offset - lo + sb.numel].view(sb.shape))

    def set_step_mode(self, mode):
        super().set_step_mode(mode)
        if mode != "xgmi":
            self._push = None
        if mode != getattr(self, "_mode_set", None):
            self.gconv.zero_()   # the replicas change roles between the step modes
            self.pend.zero_()
        self._mode_set = mode
        self._fopt = self._bopt = self._flush = None
        self._slots = (None, None)
        if mode == "plain":
            return
        K, st, opt = self.K, self.store, self.optimizer
        sl = opt.slot_names()
        m = st.slot(sl[0]) if sl else None
        v = st.slot(sl[1]) if len(sl) > 1 else None
        self._slots = (m, v)
        self._opt_key_set = self._opt_key()
        if mode != "local":
            return
        seg = st.segments
        conv = [(seg[self.names["wc"]].offset, seg[self.names["wc"]].numel),
                (seg[self.names["bc"]].offset, seg[self.names["bc"]].numel)]
        hp = opt.hparams()
        P_ = K._P
        self._fopt, self._bopt, self._flush = [], [], []
        for q in (0, 1):
            # forward of parity q: the deferred update of the previous step (parity 1-q), t = iter_prev
            f = K.step_opt(opt, st.w, None, m, v, self.iter_prev, self.pend[1 - q])
            f.g = self._gconv(1 - q)
            f.grep, f.grep_stride = self.crep, self._conv_span
            f.fly_count = self.ucount[1].data_ptr()
            f.hsrc_w2, f.hsrc_b2 = self._v("w2").data_ptr(), self._v("b2").data_ptr()
            f.hsrc_b1 = self._v("b1").data_ptr() if self.names["b1"] is not None else None
            f.hsnap, f.hC = self.hsnap.data_ptr(), self.Cls
            self._fopt.append(f)
            commit = K.flat_apply_spec(opt, st.w, None, m, v, self.iterations, self.pend[1 - q], conv)
            commit.g = self._gconv(1 - q)
            commit.grep, commit.grep_stride = self.crep, self._conv_span
            commit.count = self.ucount[0].data_ptr()
            b1 = self.names["b1"]
            self._bopt.append(K.BwdOpt(
                opt.kind_id, float(opt.learning_rate), hp["mom"], hp["b1"], hp["b2"], hp["eps"], P_(st.w), P_(m),
                P_(v), seg[self.names["w1"]].offset, seg[self.names["w2"]].offset, seg[self.names["b2"]].offset,
                seg[b1].offset if b1 is not None else -1, P_(self.W1col),
                self.W1col.stride(0) if self.W1col is not None else 0, P_(self.iterations), P_(self.iter_prev),
                commit, self.pend[q].data_ptr(), self.crep, self._conv_span))
            fl = K.flat_apply_spec(opt, st.w, None, m, v, self.iterations, self.pend[q], conv)
            fl.g = self._gconv(q)
            fl.grep, fl.grep_stride = self.crep, self._conv_span
            fl.count = self.ucount[0].data_ptr()
            self._flush.append(fl)

    def push_range(self):
        """Bucket range the backward can push into the xGMI owners itself (the Dense(64) kernel's dW1:
        99.7 % of the gradient bytes), or None when this plan form cannot."""
        if not self.f32:
            return None
        seg = self.store.segments[self.names["w1"]]
        return seg.offset, seg.offset + seg.numel

    def set_push(self, spec):
        """Fused data-parallel exchange (step mode "xgmi"): ``spec`` is the communicator's ``XgPush`` for
        this replica (None: dW1 to the local bucket, the all-reduce pushes it)."""
        if spec is not None and (self.step_mode != "xgmi" or self.push_range() is None):
            raise ValueError("the fused exchange needs step mode 'xgmi' and the float32 plan")
        self._push = spec

    def _opt_key(self):
        o = self.optimizer
        return (o.kind_id, float(o.learning_rate), tuple(sorted(o.hparams().items())))

    def refresh(self):
        # the kernel argument structs carry lr / hyper-parameters by value
        if self.step_mode != "plain" and self._opt_key_set != self._opt_key():
            self.set_step_mode(self.step_mode)

    def xg_apply_spec(self):
        """``XgApply`` for the communicator's fused all-reduce (step mode "xgmi")."""
        st, opt = self.store, self.optimizer
        m, v = self._slots
        hp = opt.hparams()
        seg = st.segments[self.names["w1"]]
        K = self.K
        if self.f32:   # no shadow: the all-reduce updates the f32 master weights only
            # the step's backward pushed dW1 itself (a replica without data this step pushed nothing)
            lo, hi = self.push_range() if (self._push is not None and self._pushed) else (0, 0)
            self._pushed = False
            spec = K.XgApply(opt.kind_id, float(opt.learning_rate), hp["mom"], hp["b1"], hp["b2"], hp["eps"],
                             K._P(st.w), K._P(m), K._P(v), K._P(self.iterations), None, 0, 0, None, 0, 0, lo, hi)
            if self._xg_rep:   # the conv gradients wait in the replicas of parity 0
                spec.rep, spec.nrep = self.gconv[0].data_ptr(), self.crep
                spec.rep_lo, spec.rep_hi = self._conv_lo, self._conv_lo + self._conv_span
                spec.rep_stride = self._conv_span
            return spec
        return K.XgApply(opt.kind_id, float(opt.learning_rate), hp["mom"], hp["b1"], hp["b2"], hp["eps"],
                         K._P(st.w), K._P(m), K._P(v), K._P(self.iterations), K._P(self.W1row), seg.offset,
                         seg.offset + seg.numel, K._P(self.W1col), self.Hd,
                         self.W1col.stride(0) if self.W1col is not None else 0)

    def finish(self):
        if self.step_mode == "local":
            # only the last step's conv update can be pending (each backward commits the previous one)
            self.K.flat_apply(self._flush[1 - self.parity])

    def step_invariants(self):
        """The deferred conv update's state between executions (step mode "local"; synchronises): every
        step's update committed exactly once, nothing pending, every gradient replica consumed."""
        torch.cuda.synchronize(self.device)
        return dict(commits=int(self.ucount[0]), applied_on_the_fly=int(self.ucount[1]),
                    pending=[int(v) for v in self.pend.cpu()], gconv_abs_max=float(self.gconv.abs().max()))

    def trace_tensors(self):
        """Per-step state recorded by ``Program.enable_trace`` (diagnostics)."""
        return [self.store.w, self.gconv.view(-1), self.pend.float(), self.metrics]

    def effective_weights(self, trace):
        """From ``Program.enable_trace`` rows of this plan ([S, n]): the weights each step left for the next
        forward, [S, store.w.numel()] — in step mode "local" the stored conv weights lag by the pending
        (deferred) update, which the next forward applies on the fly (SGD: w - lr * sum of the pending
        parity's gradient replicas)."""
        nw, ng = self.store.w.numel(), self.gconv.numel()
        w = trace[:, :nw].clone()
        if self.step_mode != "local":
            return w
        if self.optimizer.kind_id != 0:
            raise NotImplementedError("effective_weights: the deferred update is reconstructed for SGD only")
        g = trace[:, nw: nw + ng].reshape(len(trace), 2, self.crep, self._conv_span).sum(dim=2)
        pend = trace[:, nw + ng: nw + ng + 2]
        lo, span = self._conv_lo, self._conv_span
        lr = float(self.optimizer.learning_rate)
        for q in (0, 1):
            w[:, lo: lo + span] -= lr * g[:, q] * (pend[:, q:q + 1] != 0)
        return w

    def on_weights_loaded(self):
        if not self.f32:
            (self.opt or self._shadow_only).refresh_shadows()
        # loaded weights replace whatever update was outstanding
        self.pend.zero_()
        self.gconv.zero_()
        self.store.g.zero_()

    def _v(self, key):
        nm = self.names[key]
        return None if nm is None else self.store.view(nm)

    def _g(self, key):
        nm = self.names[key]
        return None if nm is None else self.store.grad(nm)

    def _forward(self, x, B, hpre, with_pt, opt=None, train=False, hrep=1):
        # launch 1: conv+bias+ReLU+pool fused with the Dense(Hd) matmul (split-K atomics into hpre,
        # which the previous backward / head launch left zeroed)
        seg = self.store.segments
        self.K.convnet_fwd(x[:B], self._v("wc"), self._v("bc"), self.W1fwd, hpre,
                           self.Pt if with_pt else None, self.amax, opt=opt,
                           off_wc=seg[self.names["wc"]].offset, off_bc=seg[self.names["bc"]].offset,
                           inc_iter=self.iterations if train else None, hrep=hrep)

    def train_step(self, x, y, B=None):
        K = self.K
        B = self.B if B is None else B
        q = self.parity
        local = self.step_mode == "local"
        self._forward(x, B, self.hpre2[q], True, self._fopt[q] if local else None, train=True, hrep=self.hrep)
        # launch 2: head + trunk backward (fused step: the updates too)
        xg = self.step_mode == "xgmi"
        rep = xg and self._xg_rep
        if local or rep:
            dwc, dbc = self._gconv_views(q if local else 0)
        else:
            dwc, dbc = self._g("wc"), self._g("bc")
        push = self._push if xg else None
        if local:   # the head variables as of the forward (the backward's head workgroup updates the originals)
            b1, w2, b2 = (self._hs_b1 if self.names["b1"] is not None else None), self._hs_w2, self._hs_b2
        else:
            b1, w2, b2 = self._v("b1"), self._v("w2"), self._v("b2")
        K.convnet_bwd(x, self.amax, self.hpre2[q], self.hpre2[1 - q], b1, w2, b2, y,
                      scale=self.scale, pre_relu=self.pre_relu, metrics=self.metrics, W1row=self.W1row, Pt=self.Pt,
                      dW1=self._g("w1"), dwc=dwc, dbc=dbc, dW2=self._g("w2"), db2=self._g("b2"), db1=self._g("b1"),
                      B=B, opt=self._bopt[q] if local else None, cpart=self.cpart, push=push,
                      crep=self.crep if rep else 1, crep_stride=self._conv_span)
        self._pushed = push is not None
        if self.det:
            K.convnet_cgrad_reduce(self.cpart, self.n_cpart, dwc, dbc)
        self.parity = 1 - q

    def apply(self):
        # step mode "plain": multi-tensor optimizer (+ grad zeroing + bf16 shadow refresh)
        self.opt.apply()

    def eval_step(self, x, y, B=None):
        B = self.B if B is None else B
        self._forward(x, B, self.hpre, False)
        self.K.head_xent(self.hpre, self._v("w2"), self._v("b2"), y, B=B, scale=self.scale, pre_bias=self._v("b1"),
                         pre_relu=self.pre_relu, compute_grad=False, metrics=self.metrics, zero_hin=True)

    def predict(self, x, B=None):
        B = self.B if B is None else B
        self._forward(x, B, self.hpre, False)
        self.K.head_xent(self.hpre, self._v("w2"), self._v("b2"), self._dummy_labels(B), B=B, scale=1.0,
                         pre_bias=self._v("b1"), pre_relu=self.pre_relu, compute_grad=False, probs=self.probs,
                         probs_are_logits=self.logits_out, zero_hin=True)
        return self.probs[:B]

    def _dummy_labels(self, B):
        if not hasattr(self, "_zl") or self._zl.shape[0] < B:
            self._zl = torch.zeros(max(B, self.B), dtype=torch.int32, device=self.device)
        return self._zl


class ConvNetGenPlan(ReplicaPlan):
    """The DWK/TF2M small CNN at the user's own widths — Conv2D(F in 16/32/48/64) · MaxPool(2) · Flatten ·
    Dense(U in 32/64/96/128) · Dense(<= 16) (distributed_with_keras.py:33-43 and tf2_mnist_distributed.py:66-72
    with other filter / unit counts) — as two fused float32 HIP launches per step (csrc/kernels/convnet_gen.hip):

      forward   conv+bias+ReLU+pool fused with the Dense(U) matmul (split-K atomics into hpre replicas)
      backward  every workgroup recomputes the head from hpre, then the Dense(U) weight / input gradients
                of its pooled position, the pool / ReLU routing MFMA and the conv gradients; one extra
                workgroup makes the head's own gradients, the metrics and the step count

    followed, by step mode, by the multi-tensor optimizer ("plain"), nothing ("local": two launches per step —
    each backward workgroup applies the optimizer to the Dense(U) rows it owns in place, no other workgroup of
    the launch reading them; the head workgroup updates the head in place while the trunk reads the forward's
    snapshot of it; the conv update is deferred: the next forward applies it on the fly, the next backward's
    head workgroup commits it, ``finish()`` flushes the last one), or the xGMI all-reduce that applies it
    ("xgmi"; the backward pushes the Dense(U) gradient rows straight into the owners' windows).  The
    reference's own Conv2D(32)/Dense(64) keeps the hand-tuned ``ConvNetPlan``."""
    kind = "fused_convnet_generic"

    def __init__(self, model, store, device, batch, global_batch, optimizer, loss, pattern):
        super().__init__(model, store, device, batch, global_batch, optimizer)
        from ..ops import kernels as K
        self.K = K
        c, d1, d2 = pattern["conv"], pattern["dense1"], pattern["dense2"]
        if not K.cgen_supported(c.filters, d1.units):
            raise NotImplementedError(f"convnet_gen: Conv2D({c.filters}) + Dense({d1.units}) not instantiated")
        if os.environ.get("TDE_DETERMINISTIC", "0") not in ("", "0"):
            import warnings
            warnings.warn("TDE_DETERMINISTIC: the generic-width fused CNN step adds its split-K and conv-gradient "
                          "partials with float atomics; its steps are not bitwise reproducible")
        self.H, self.W, self.C = c.input_shape[0], c.input_shape[1], c.filters
        self.P = ((self.H - 2) // 2) * ((self.W - 2) // 2)
        self.Hd, self.Cls = d1.units, d2.units
        B, Bp, dev = self.B, _round8(self.B), self.device
        self.Pt = torch.zeros(self.P * self.C, Bp, dtype=torch.float32, device=dev)
        self.amax = torch.zeros(self.P, self.C // 8, Bp, dtype=torch.int64, device=dev)
        # split-K targets of the forward's ~P adders per address, summed by the consumers (TDE_CONVNET_HREP)
        self.hrep = max(1, min(8, int(os.environ.get("TDE_CONVNET_HREP", "4"))))
        self.hpre2 = torch.zeros(2, self.hrep, B, self.Hd, dtype=torch.float32, device=dev)
        self.hpre = torch.zeros(B, self.Hd, dtype=torch.float32, device=dev)
        self.probs = torch.zeros(B, self.Cls, dtype=torch.float32, device=dev)
        self.pre_relu = d1.activation == "relu"
        self.logits_out = d2.activation is None
        n = lambda l, w: f"{l.name}/{w}"  # noqa: E731
        self.names = dict(wc=n(c, "kernel"), bc=n(c, "bias"), w1=n(d1, "kernel"),
                          b1=n(d1, "bias") if d1.use_bias else None, w2=n(d2, "kernel"), b2=n(d2, "bias"))
        self.W1 = store.view(self.names["w1"])
        self.opt = OptimizerKernel(store, optimizer, {}, self.iterations) if optimizer is not None else None
        self.parity = 0
        self._copt = self._fly = self._hopt = self._commit = self._flush = None
        self._push, self._pushed = None, False
        # conv gradients: the ~170 backward workgroups add theirs into crep replicas of the conv segments
        # (workgroup x -> replica x % crep; same-address float atomics from every workgroup serialise at the
        # memory side), summed by the consumer: in the fused step the next forward (the update applied on the
        # fly) and the next backward's head workgroup (committed), one set per step parity; under data
        # parallelism the xGMI all-reduce (set 0).  TDE_CONVNET_GREP; plain steps add into the gradient bucket.
        seg = store.segments
        sw, sb = seg[self.names["wc"]], seg[self.names["bc"]]
        self._conv_lo = min(sw.offset, sb.offset)
        self._conv_span = max(sw.offset + sw.numel, sb.offset + sb.numel) - self._conv_lo
        others = [n for n in store.order if n not in (self.names["wc"], self.names["bc"]) and
                  self._conv_lo <= seg[n].offset < self._conv_lo + self._conv_span]
        self.crep = 1 if others else max(1, min(8, int(os.environ.get("TDE_CONVNET_GREP", "8"))))
        self.gconv = torch.zeros(2, self.crep, self._conv_span, dtype=torch.float32, device=dev)
        # fused step: the deferred conv update's flags by parity, Adam's t of the pending update, and the head
        # variables as of the forward ([b1 | W2 | b2]: the backward's trunk reads them while its head workgroup
        # updates the originals)
        self.pend = torch.zeros(2, dtype=torch.int32, device=dev)
        self.iter_prev = torch.zeros(1, dtype=torch.int64, device=dev)
        C_, H_ = self.Cls, self.Hd
        self.hsnap = torch.zeros(H_ + H_ * C_ + C_, dtype=torch.float32, device=dev)
        self._hs_b1 = self.hsnap[:H_]
        self._hs_w2 = self.hsnap[H_: H_ + H_ * C_].view(H_, C_)
        self._hs_b2 = self.hsnap[H_ + H_ * C_:]

    def supports_step_mode(self, mode):
        if mode == "plain":
            return True
        ok = self.optimizer is not None and self.device.type == "cuda"
        return ok and mode in ("xgmi", "local")

    def _gset(self, q, name):
        """Replica 0 of conv variable ``name``'s gradient in parity set q."""
        sg = self.store.segments[self.names[name]]
        lo = self._conv_lo
        return self.gconv[q, 0, sg.offset - lo: sg.offset - lo + sg.numel]

    def set_step_mode(self, mode):
        super().set_step_mode(mode)
        self._copt = self._fly = self._hopt = self._commit = self._flush = None
        if mode != "xgmi":
            self._push = None
        self.gconv.zero_()
        self.pend.zero_()
        if mode != "local":
            return
        K, st, o = self.K, self.store, self.optimizer
        sl = o.slot_names()
        m = st.slot(sl[0]) if sl else None
        v = st.slot(sl[1]) if len(sl) > 1 else None
        hp = o.hparams()
        seg = st.segments
        at = lambda t, name: None if t is None or name is None else t.data_ptr() + 4 * seg[self.names[name]].offset  # noqa: E731
        kind, lr = o.kind_id, float(o.learning_rate)
        self._copt = K.CgenOpt(kind, lr, hp["mom"], hp["b1"], hp["b2"], hp["eps"], at(st.w, "w1"), at(m, "w1"),
                               at(v, "w1"), self.iterations.data_ptr())
        conv = [(self._conv_lo, self._conv_span)]
        self._fly, self._hopt, self._commit, self._flush = [], [], [], []
        for q in (0, 1):
            # forward of parity q: the update of the previous step (set 1-q) on the fly, the head snapshot
            self._fly.append(K.CgenFly(
                kind, lr, hp["mom"], hp["b1"], hp["b2"], hp["eps"], self.pend[1 - q].data_ptr(),
                self._gset(1 - q, "wc").data_ptr(), self._gset(1 - q, "bc").data_ptr(), self.crep, self._conv_span,
                at(m, "wc"), at(m, "bc"), at(v, "wc"), at(v, "bc"), self.iter_prev.data_ptr(),
                at(st.w, "b1"), at(st.w, "w2"), at(st.w, "b2"), self.hsnap.data_ptr(), self.Cls))
            # backward of parity q: the head in place, the previous step's conv update committed, set q flagged
            b1 = self.names["b1"]
            self._hopt.append(K.CgenHead(
                kind, lr, hp["mom"], hp["b1"], hp["b2"], hp["eps"], st.w.data_ptr(), K._P(m), K._P(v),
                seg[self.names["w2"]].offset, seg[self.names["b2"]].offset, seg[b1].offset if b1 is not None else -1,
                self.iterations.data_ptr(), self.pend[q].data_ptr(), self.iter_prev.data_ptr()))
            for lst, qq in ((self._commit, 1 - q), (self._flush, q)):
                f = K.flat_apply_spec(o, st.w, None, m, v, self.iterations, self.pend[qq], conv)
                f.g = self.gconv[qq].data_ptr() - 4 * self._conv_lo   # indexed with the flat offsets
                f.grep, f.grep_stride = self.crep, self._conv_span
                lst.append(f)
        self._opt_key_set = self._opt_key()

    def finish(self):
        if self.step_mode == "local":
            # only the last step's conv update can be pending (each backward commits the previous one)
            self.K.flat_apply(self._flush[1 - self.parity])

    def _opt_key(self):
        o = self.optimizer
        return (o.kind_id, float(o.learning_rate), tuple(sorted(o.hparams().items())))

    def refresh(self):
        # the launch descriptors carry lr / hyper-parameters by value
        if self.step_mode == "local" and self._opt_key_set != self._opt_key():
            self.set_step_mode("local")

    def push_range(self):
        """Bucket range the backward can push into the xGMI owners itself: the Dense(U) kernel's gradient."""
        seg = self.store.segments[self.names["w1"]]
        return seg.offset, seg.offset + seg.numel

    def set_push(self, spec):
        """Fused data-parallel exchange (step mode "xgmi"): ``spec`` is the communicator's ``XgPush``."""
        if spec is not None and self.step_mode != "xgmi":
            raise ValueError("the fused exchange needs step mode 'xgmi'")
        self._push = spec

    def xg_apply_spec(self):
        spec = f32_xg_apply_spec(self)
        if self.crep > 1:   # the conv gradients wait in the replicas: the all-reduce sums (and zeroes) them
            spec.rep, spec.nrep = self.gconv[0].data_ptr(), self.crep
            spec.rep_lo, spec.rep_hi = self._conv_lo, self._conv_lo + self._conv_span
            spec.rep_stride = self._conv_span
        return spec

    def _conv_grads(self, q):
        """(dwc, dbc, crep, stride) the backward of parity q adds the conv gradients into."""
        if self.step_mode == "plain" or (self.step_mode == "xgmi" and self.crep == 1):
            return self._g("wc"), self._g("bc"), 1, 0
        qs = q if self.step_mode == "local" else 0
        return self._gset(qs, "wc"), self._gset(qs, "bc"), self.crep, self._conv_span

    def step_invariants(self):
        """The deferred conv update's state between executions (step mode "local"; synchronises): nothing
        pending, every gradient replica consumed."""
        torch.cuda.synchronize(self.device)
        return dict(pending=[int(v) for v in self.pend.cpu()], gconv_abs_max=float(self.gconv.abs().max()))

    def _v(self, key):
        nm = self.names[key]
        return None if nm is None else self.store.view(nm)

    def _g(self, key):
        nm = self.names[key]
        return None if nm is None else self.store.grad(nm)

    def on_weights_loaded(self):
        # loaded weights replace whatever gradients were outstanding
        self.store.g.zero_()
        self.gconv.zero_()
        self.pend.zero_()

    def train_step(self, x, y, B=None):
        K = self.K
        B = self.B if B is None else B
        q = self.parity
        local = self.step_mode == "local"
        # the fused step's Adam t is read by every backward workgroup: the forward advances the counter
        K.cgen_fwd(x, self._v("wc"), self._v("bc"), self.W1, self.hpre2[q], self.Pt, self.amax, B=B,
                   inc_iter=self.iterations if local else None, fly=self._fly[q] if local else None)
        dwc, dbc, crep, cstride = self._conv_grads(q)
        push = self._push if self.step_mode == "xgmi" else None
        if local:   # the head as of this step's forward (the head workgroup updates the originals)
            b1, w2, b2 = (self._hs_b1 if self.names["b1"] is not None else None), self._hs_w2, self._hs_b2
        else:
            b1, w2, b2 = self._v("b1"), self._v("w2"), self._v("b2")
        K.cgen_bwd(x, self.amax, self.hpre2[q], self.hpre2[1 - q], b1, w2, b2, y,
                   scale=self.scale, pre_relu=self.pre_relu, metrics=self.metrics, W1=self.W1, Pt=self.Pt,
                   dW1=None if local else self._g("w1"), dwc=dwc.view(self._v("wc").shape), dbc=dbc, dW2=self._g("w2"),
                   db2=self._g("b2"), db1=self._g("b1"), B=B, iterations=None if local else self.iterations,
                   opt=self._copt if local else None, crep=crep, crep_stride=cstride,
                   hopt=self._hopt[q] if local else None, fcommit=self._commit[q] if local else None, push=push)
        self._pushed = push is not None
        self.parity = 1 - q

    def apply(self):
        self.opt.apply()

    def _forward(self, x, B):
        self.K.cgen_fwd(x, self._v("wc"), self._v("bc"), self.W1, self.hpre, self.Pt, self.amax, B=B)

    def eval_step(self, x, y, B=None):
        B = self.B if B is None else B
        self._forward(x, B)
        self.K.head_xent(self.hpre, self._v("w2"), self._v("b2"), y, B=B, scale=self.scale, pre_bias=self._v("b1"),
                         pre_relu=self.pre_relu, compute_grad=False, metrics=self.metrics, zero_hin=True)

    def predict(self, x, B=None):
        B = self.B if B is None else B
        self._forward(x, B)
        if not hasattr(self, "_zl"):
            self._zl = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        self.K.head_xent(self.hpre, self._v("w2"), self._v("b2"), self._zl, B=B, scale=1.0,
                         pre_bias=self._v("b1"), pre_relu=self.pre_relu, compute_grad=False, probs=self.probs,
                         probs_are_logits=self.logits_out, zero_hin=True)
        return self.probs[:B]


# ---------------------------------------------------------------------------------------
def make_plan(model, store, device, batch, global_batch, optimizer, loss, prefer=None):
    device = torch.device(device)
    prefer = prefer or os.environ.get("TDE_EXECUTOR")
    if device.type == "cuda" and prefer != "reference":
        pat = match_convnet(model, loss)
        if pat is not None and prefer in (None, "fused"):
            cls = ConvNetGenPlan if pat.get("generic") else ConvNetPlan
            return cls(model, store, device, batch, global_batch, optimizer, loss, pat)
        if prefer in (None, "fused", "bncnn"):
            from . import bncnn
            plan = bncnn.try_make(model, store, device, batch, global_batch, optimizer, loss)
            if plan is not None:
                return plan
        if prefer in (None, "fused", "smallnet"):
            from . import smallnet
            plan = smallnet.try_make(model, store, device, batch, global_batch, optimizer, loss)
            if plan is not None:
                return plan
        from . import layerwise
        plan = layerwise.try_make(model, store, device, batch, global_batch, optimizer, loss)
        if plan is not None:
            return plan
        raise NotImplementedError(
            f"model {model.name!r} has layers without a HIP kernel path; set TDE_EXECUTOR=reference to run it "
            "with torch reference ops")
    return ReferencePlan(model, store, device, batch, global_batch, optimizer, loss)
