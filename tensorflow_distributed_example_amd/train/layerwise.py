"""Layer-wise HIP execution plan: any Sequential / functional model built from the
supported layers (Model B of mnist_keras_distributed.py:79-109 == tf2_mnist_distributed.py
:105-135, the ResNet-18 stress config, ...) runs its whole training step on the
gfx950 kernels of csrc/kernels/layers.hip — no torch compute op on the hot path.

The plan compiler walks the model's execution graph once and fuses layer chains
into *stages* (SURVEY.md §2.5 B1-B17):

    Conv2D/Dense  ->  implicit-GEMM MFMA (+bias, +ReLU, +BN batch statistics in the epilogue)
    BatchNormalization [-> Add(residual)] [-> ReLU] [-> Dropout]  ->  one bn_fwd pass
    standalone ReLU / Dropout / Add(+ReLU)  ->  bn_fwd in identity mode
    MaxPooling2D / GlobalAveragePooling2D / ZeroPadding2D  ->  dedicated kernels
    Flatten / Reshape  ->  buffer aliases (no kernel)
    last Dense (+softmax) + SparseCategoricalCrossentropy  ->  GEMM to f32 logits + fused
        softmax-CE / accuracy / dlogits kernel (probability-space loss on a softmax output
        is computed from the logits, Q5)

The backward replays the stages in reverse; tensors with several consumers (ResNet
shortcuts) accumulate their gradients in place (the first writer stores, later ones
add), BN+ReLU+dropout backward regenerates the dropout mask from the Philox counter
instead of storing it.  Weight gradients land in the replica's flat fp32 bucket (one
RCCL all-reduce) and one multi-tensor optimizer kernel applies them and refreshes the
bf16 weight shadows the GEMMs read.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from .. import _native as N
from .. import backend as Kb
from ..models import layers as L
from ..ops import layer_ops as O
from ..ops import layer_ops32 as O32
from . import program as PG

bf16 = torch.bfloat16


class Unsupported(Exception):
    pass


class _T:
    """One tensor of the execution graph (per-sample ``shape``)."""

    def __init__(self, tid, shape):
        self.id = tid
        self.shape = tuple(shape)
        self.numel = int(np.prod(self.shape)) if self.shape else 1
        self.alias = None          # Flatten/Reshape: same storage as another tensor
        self.consumers = []
        self.producer = None
        self.buf = None
        self.grad = None

    def root(self):
        t = self
        while t.alias is not None:
            t = t.alias
        return t

    @property
    def C(self):
        return self.shape[-1]

    def rows(self, B):
        return B * (self.numel // self.C)


def plan_grad_buckets(stage_params, segments, total, target_elems):
    """Bucket cuts for ``LayerwisePlan.grad_buckets``: ``stage_params[i]`` = variables written by the
    i-th backward stage, ``segments`` = (name, flat offset) of every trainable variable, ``total`` =
    bucket length.  Returns [(i, lo, hi)] covering [0, total) exactly, highest offsets first."""
    last = len(stage_params) - 1
    owner = {}
    for i, names in enumerate(stage_params):
        for n in names:
            owner.setdefault(n, i)
    segs = sorted(segments, key=lambda g: g[1], reverse=True)
    out = []
    hi = front = total
    k = 0
    for i in range(len(stage_params)):
        while k < len(segs) and owner.get(segs[k][0], last) <= i:
            front = segs[k][1]
            k += 1
        if k == len(segs):
            front = 0
        if front < hi and (hi - front >= target_elems or front == 0):
            out.append((i, front, hi))
            hi = front
    return out


class _Stage:
    inputs: list
    out: _T

    def fwd(self, p, B, training):
        raise NotImplementedError

    def bwd(self, p, B):
        raise NotImplementedError

    def param_names(self):
        """Trainable variables whose gradients this stage's backward writes (all of them, once)."""
        return [n for n in (getattr(self, "wname", None), getattr(self, "bname", None)) if n]


class LayerwisePlan(PG.ReplicaPlan):
    """Precision follows the global policy: ``float32`` (the reference's) runs every stage on the f32
    kernel forms (csrc/kernels/layers_f32.hip: f32 activations and gradients, the f32 master kernels read
    in place on the exact-f32 MFMA); ``mixed_bfloat16`` on the bf16 forms (csrc/kernels/layers.hip: bf16
    activations, bf16 weight shadows refreshed by the optimizer, f32 master weights)."""
    kind = "layerwise"

    def __init__(self, model, store, device, batch, global_batch, optimizer, loss):
        super().__init__(model, store, device, batch, global_batch, optimizer)
        self.loss = loss
        self.model = model
        self.f32 = Kb.global_policy().compute_dtype == torch.float32
        self.compute_dtype = "fp32" if self.f32 else "bf16"
        # TDE_DETERMINISTIC=1 (bf16 forms): every reduction in a fixed order (csrc/kernels/layers.hip g_det: sums by
        # the *_det kernels, split-K through the ordered scratch) and the kernels whose sums are atomics off (halo
        # conv statistics, fused BN + max-pool backward, narrow direct convs, fused head): two runs of one
        # configuration are bitwise identical
        self.det = (not self.f32 and torch.device(device).type == "cuda"
                    and bool(N.hip().tde_layers_is_deterministic()))
        self.adt = torch.float32 if self.f32 else bf16          # activation / activation-gradient dtype
        self.sdt = torch.float64 if self.f32 else torch.float32  # BN backward-sum dtype
        # bf16: inputs staged as bf16 (Keras mixed_bfloat16 casts them at the first layer anyway), no per-step
        # cast launch; TDE_BF16_INPUT=0 keeps f32 staging + the cast kernel.  f32: the ring is read in place.
        self.input_dtype = (torch.float32 if self.f32 or os.environ.get("TDE_BF16_INPUT", "1") == "0" else bf16)
        self._compile()
        self._alloc()
        # TDE_WGRAD_STREAM=1: weight gradients on a side stream, concurrent with the input-gradient chain
        # (joined at the end of the backward).  Off by default: measured slower in the captured step
        # (ResNet-18 20.7k -> 20.0k, Model B 511k -> 457k img/s; profiles/r2_ab_notes.md).
        self.side_stream = None
        if torch.device(device).type == "cuda" and os.environ.get("TDE_WGRAD_STREAM", "0") == "1":
            self.side_stream = torch.cuda.Stream(device=device)
        shadows = {}
        for st in self.stages:
            for name, want in getattr(st, "shadows", {}).items():
                shadows[name] = want
        self.shadows = shadows
        if optimizer is not None:
            self.opt = PG.OptimizerKernel(store, optimizer, shadows, self.iterations)
            self._sh = self.opt
        else:
            from ..optimizers import SGD
            self.opt = None
            self._sh = PG.OptimizerKernel(store, SGD(0.0), shadows, self.iterations)
        for st in self.stages:
            if hasattr(st, "bind_shadows"):
                st.bind_shadows(self._sh)

    # ------------------------------------------------------------------ compile
    def _compile(self):
        m = self.model
        nodes = m._nodes()
        T = {0: _T(0, m.input_shape[1:])}
        for i, (layer, ins, out) in enumerate(nodes):
            T[out] = _T(out, layer.output_shape)
            T[out].producer = i
            for j in ins:
                T[j].consumers.append(i)
        self.T = T
        self.nodes = nodes
        n_nodes = len(nodes)

        def single(t):
            return nodes[t.consumers[0]] if len(t.consumers) == 1 else None

        def is_relu(layer):
            return isinstance(layer, L.Activation) and layer.activation == "relu"

        fused = set()        # node indices absorbed into another stage
        deferred = {}        # Add node index -> BN stage emitted at that position
        stages = []
        bn_fed = {}          # BN node index -> GEMM stage that computes its statistics

        # pass 1: decide GEMM -> BN statistics fusion
        for i, (layer, ins, out) in enumerate(nodes):
            if isinstance(layer, (L.Conv2D, L.Dense)) and i != n_nodes - 1 and layer.activation is None:
                c = single(T[out])
                if c is not None and isinstance(c[0], L.BatchNormalization):
                    bn_fed[nodes.index(c)] = i

        last_layer = nodes[-1][0]
        if not isinstance(last_layer, L.Dense):
            raise Unsupported(f"last layer {last_layer.name} must be Dense (logits / softmax) for the fused head")
        strip = PG._last_softmax(m, self.loss)
        if last_layer.activation not in (None, "softmax") or (last_layer.activation == "softmax") != strip:
            raise Unsupported("head must be Dense logits with from_logits=True or Dense(softmax) with probabilities")
        from ..losses import SparseCategoricalCrossentropy
        if not isinstance(self.loss, SparseCategoricalCrossentropy):
            raise Unsupported(f"loss {type(self.loss).__name__} has no fused HIP kernel")

        lid = 0
        for i, (layer, ins, out) in enumerate(nodes):
            if i in fused:
                continue
            tin = [T[j] for j in ins]
            tout = T[out]
            if isinstance(layer, (L.Flatten, L.Reshape, L.InputLayer)):
                tout.alias = tin[0]
                continue
            if i == n_nodes - 1:
                stages.append(_Head(self, layer, tin[0], tout, logits_out=not strip))
                continue
            if isinstance(layer, (L.Conv2D, L.Dense)):
                if layer.activation not in (None, "relu"):
                    raise Unsupported(f"{layer.name}: activation {layer.activation!r}")
                stats = i in {v: k for k, v in bn_fed.items()}
                stages.append(_Gemm(self, layer, tin[0], tout, stats))
                continue
            if isinstance(layer, (L.BatchNormalization, L.Activation, L.Dropout, L.Add)):
                if isinstance(layer, L.Activation) and layer.activation != "relu":
                    raise Unsupported(f"{layer.name}: activation {layer.activation!r} inside the network")
                st = _Elementwise(self, layer, tin, tout, lid)
                lid += 1
                # absorb the chain that follows: [Add] [ReLU] [Dropout]
                cur = tout
                chain = [tout]
                if isinstance(layer, L.BatchNormalization):
                    st.stats_from_gemm = i in bn_fed
                    c = single(cur)
                    if c is not None and isinstance(c[0], L.Add) and len(c[1]) == 2 and nodes.index(c) not in fused:
                        k = nodes.index(c)
                        other = [T[j] for j in c[1] if j != out]
                        if len(other) == 1:
                            st.res = other[0]
                            fused.add(k)
                            cur = T[c[2]]
                            chain.append(cur)
                            st.defer_to = k
                if not isinstance(layer, L.Dropout) and not (isinstance(layer, L.Activation)):
                    c = single(cur)
                    if c is not None and is_relu(c[0]):
                        st.relu = True
                        fused.add(nodes.index(c))
                        cur = T[c[2]]
                        chain.append(cur)
                if not isinstance(layer, L.Dropout):
                    c = single(cur)
                    if c is not None and isinstance(c[0], L.Dropout):
                        st.set_dropout(c[0])
                        fused.add(nodes.index(c))
                        cur = T[c[2]]
                        chain.append(cur)
                st.out = cur
                for t in chain[:-1]:
                    t.alias = cur
                if st.defer_to is not None:
                    deferred.setdefault(st.defer_to, []).append(st)
                else:
                    stages.append(st)
                continue
            if isinstance(layer, L.MaxPooling2D):
                stages.append(_MaxPool(self, layer, tin[0], tout))
                continue
            if isinstance(layer, L.GlobalAveragePooling2D):
                stages.append(_GAP(self, layer, tin[0], tout))
                continue
            if isinstance(layer, L.ZeroPadding2D):
                stages.append(_Pad(self, layer, tin[0], tout))
                continue
            raise Unsupported(f"layer {layer.name} ({type(layer).__name__}) has no HIP kernel path")
        # emit deferred BN+Add stages at the Add's position (after both branches exist)
        if deferred:
            out_stages = []
            pending = sorted(deferred.items())
            for st in stages:
                while pending and st.node_index > pending[0][0]:
                    out_stages += pending.pop(0)[1]
                out_stages.append(st)
            for _, lst in pending:
                out_stages += lst
            stages = out_stages
        self.stages = stages
        # the fused head also takes over the ReLU mask and bias gradient of a Dense that feeds only it
        head = stages[-1]
        if isinstance(head, _Head) and head.fused and len(stages) > 1 and not self.f32:
            prev = stages[-2]
            if (isinstance(prev, _Gemm) and not prev.conv and prev.out.root() is head.inp.root()
                    and len(T[prev.out.id].consumers) == 1 and not prev.stats):
                head.absorb(prev)
        # BatchNorm + ReLU whose only consumer is a MaxPool (the ResNet stem): one pass reads the conv output
        # and writes the pooled output + argmax; the BN output itself is never stored (its backward recomputes
        # z from the conv output).  TDE_BN_POOL=0 keeps the two launches.
        if os.environ.get("TDE_BN_POOL", "1") != "0" and not self.f32 and not self.det:
            for i, st in enumerate(stages[:-1]):
                nxt = stages[i + 1]
                if (isinstance(st, _Elementwise) and st.bn and st.relu and st.res is None and st.drop.rate == 0
                        and isinstance(nxt, _MaxPool) and nxt.inp.root() is st.out.root()
                        and len(T[st.out.id].consumers) == 1 and O.bn_pool_ok(nxt.geo)
                        and st.inp.root().id != 0):
                    st.pool, nxt.fused = nxt, True
        # float32: Conv2D / Dense with ReLU whose only consumer is a non-overlapping MaxPool — the pool's
        # backward applies the ReLU mask (from the pooled value) and the bias gradient, and the separate
        # act_bwd pass over the 4x larger activation disappears.  TDE_POOL_RELU=0 keeps the two launches.
        if self.f32 and os.environ.get("TDE_POOL_RELU", "1") != "0":
            for i, st in enumerate(stages[:-1]):
                nxt = stages[i + 1]
                if (isinstance(st, _Gemm) and st.relu and not st.stats and isinstance(nxt, _MaxPool)
                        and nxt.inp.root() is st.out.root() and len(T[st.out.id].consumers) == 1
                        and O32.pool_relu_fusable(nxt.geo)):
                    st.act_done, nxt.relu_from = True, st
        # gradient accumulation flags: reverse order, first writer stores
        written = set()
        for st in reversed(stages):
            st.accum = {}
            for t in st.grad_inputs():
                r = t.root()
                st.accum[r.id] = r.id in written
                written.add(r.id)
        # TDE_BN_SUM_FUSE=1: BatchNormalization backward sums in the epilogue of the stride-1 input-gradient GEMM that
        # writes the BN output's gradient LAST (after every other consumer's contribution landed): that BN's
        # backward then runs its apply pass only — the bn_bwd_reduce pass over dout / y / res disappears
        # (csrc/kernels/layers.hip BnSum).  Off by default: on ResNet-18 the 9 eligible input gradients grow by
        # what the 9 reduction passes cost (reductions 231 -> 137 us, input gradients 414 -> 500 us per step;
        # 22,965 vs 22,948 img/s, profiles/r6_bnsum/)
        if not self.f32 and not self.det and os.environ.get("TDE_BN_SUM_FUSE", "0") == "1":
            for st in stages:
                if not (isinstance(st, _Elementwise) and st.bn and st.pool is None and st.drop.rate == 0):
                    continue
                T = st.out.root()
                writers = [w for w in reversed(stages) if any(t.root() is T for t in w.grad_inputs())]
                last = writers[-1] if writers else None
                if (isinstance(last, _Gemm) and last.conv and last.need_dgrad and last.inp.root() is T
                        and not (last.small_dgrad or last.halo or last.use_im2col or last.use_stem_pack)
                        and O.dgrad_bnsum_ok(last.geo)):
                    last.bnsum_of = st
                    st.sums_fused = True

    def _alloc(self):
        B, dev = self.B, self.device
        self.x_bf = torch.zeros(B * self.T[0].numel, dtype=self.adt, device=dev)
        self.T[0].buf = self.x_bf
        for t in self.T.values():
            if t.id == 0 or t.alias is not None:
                continue
            t.buf = torch.zeros(B * t.numel, dtype=self.adt, device=dev)
            t.grad = torch.zeros(B * t.numel, dtype=self.adt, device=dev)
        for t in self.T.values():
            if t.alias is not None:
                t.buf, t.grad = t.root().buf, t.root().grad
        for st in self.stages:
            st.alloc(B, dev)
        # one shared f32 split-K scratch (stages run in order on one stream; finalize re-zeroes it)
        need = max([st.scratch_need(B) for st in self.stages if hasattr(st, "scratch_need")] + [0])
        self.scratch = torch.zeros(max(need, 1), dtype=torch.float32, device=dev) if need else None
        # split-K weight gradients store per-split partials here and reduce them in one pass
        wneed = max([st.wscratch_need(B) for st in self.stages if hasattr(st, "wscratch_need")] + [0])
        self.wscratch = torch.empty(wneed, dtype=torch.float32, device=dev) if wneed else None
        # f32 forms: split-K weight-gradient partials (summed in split order by the second launch)
        pneed = max([st.wpart_need(B) for st in self.stages if hasattr(st, "wpart_need")] + [0]) if self.f32 else 0
        self.wpart = torch.empty(pneed, dtype=torch.float32, device=dev) if pneed else None

    # ------------------------------------------------------------------ plan interface
    def on_weights_loaded(self):
        self._sh.refresh_shadows()

    def _input(self, x, B):
        n = B * self.T[0].numel
        if self.f32:
            self._bind_input(x.reshape(-1)[:n].contiguous() if x.dtype == torch.float32 else x.float().reshape(-1)[:n])
            return
        if x.dtype == bf16:
            # the Program's input ring already holds bf16 (cast once per execution at staging): the
            # first layer reads the ring slot directly
            self._bind_input(x.reshape(-1)[:n])
        else:
            self._bind_input(self.x_bf)
            O.cast_bf16(x[:B].reshape(-1), self.x_bf[:n])

    def _bind_input(self, buf):
        if self.T[0].buf is buf:
            return
        for t in self.T.values():
            if t.root() is self.T[0]:
                t.buf = buf

    def train_step(self, x, y, B=None, after_bwd=None):
        """Forward + backward.  ``after_bwd(i)`` (optional) runs after the i-th backward stage (reverse
        order) has been enqueued — the hook the Program uses to start gradient-bucket all-reduces
        while the rest of the backward is still running (see ``grad_buckets``)."""
        B = self.B if B is None else B
        self._input(x, B)
        self._labels = y
        for st in self.stages:
            st.fwd(self, B, True)
        for i, st in enumerate(reversed(self.stages)):
            st.bwd(self, B)
            if after_bwd is not None:
                after_bwd(i)
        if self.side_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.side_stream)

    def grad_buckets(self, target_elems):
        """Reverse-order gradient buckets: [(i, lo, hi)] = once backward stage i (reverse order) is
        enqueued, the flat gradient range [lo, hi) is final (every variable in it has had its only
        writer run).  Variables sit in the flat bucket in layer order and backward visits layers in
        reverse, so the final region grows from the end of the bucket; a bucket is cut whenever it
        reaches ``target_elems`` (4-8 MB buckets issued as backward produces them)."""
        st = self.store
        segs = [(n, st.segments[n].offset) for n in st.names(trainable=True)]
        return plan_grad_buckets([s.param_names() for s in reversed(self.stages)], segs, st.g.numel(), target_elems)

    def apply(self):
        self.opt.apply()

    def eval_step(self, x, y, B=None):
        B = self.B if B is None else B
        self._input(x, B)
        self._labels = y
        tr = Kb.resolve_training(False)
        for st in self.stages:
            st.fwd(self, B, tr, mode="eval")
        if tr:
            self._reset_stats()

    def predict(self, x, B=None):
        B = self.B if B is None else B
        self._input(x, B)
        self._labels = self._zero_labels(B)
        tr = Kb.resolve_training(False)
        for st in self.stages:
            st.fwd(self, B, tr, mode="predict")
        if tr:
            self._reset_stats()
        return self.stages[-1].probs[: B * self.stages[-1].C].view(B, -1)

    def _reset_stats(self):
        for st in self.stages:
            if getattr(st, "colstats", None) is not None:
                st.colstats.zero_()

    def _zero_labels(self, B):
        if not hasattr(self, "_zl") or self._zl.shape[0] < B:
            self._zl = torch.zeros(max(B, self.B), dtype=torch.int32, device=self.device)
        return self._zl


# ---------------------------------------------------------------------------------------
class _Gemm(_Stage):
    def __init__(self, plan, layer, tin, tout, stats):
        self.layer, self.inp, self.out = layer, tin, tout
        self.node_index = tout.producer
        self.stats = stats
        self.relu = layer.activation == "relu"
        st = plan.store
        self.wname = f"{layer.name}/kernel"
        self.bname = f"{layer.name}/bias" if layer.use_bias else None
        self.W = st.view(self.wname)
        self.gW = st.grad(self.wname)
        self.b = st.view(self.bname) if self.bname else None
        self.gb = st.grad(self.bname) if self.bname else None
        self.conv = isinstance(layer, L.Conv2D)
        need_dgrad = tin.root().id != 0
        self.need_dgrad = need_dgrad
        self.f32 = plan.f32
        self.shadows = {} if self.f32 else {self.wname: ("row", "col") if need_dgrad else ("col",)}
        self.small_fwd = self.small_dgrad = self.small_wgrad = False
        self.use_im2col = self.use_stem_pack = False
        if self.conv and self.f32:   # the f32 implicit GEMM covers every geometry itself
            H, W_, C = tin.shape
            Ho, Wo, Co = tout.shape
            (pt, _), (pl, _) = layer.pads(tin.shape)
            self.geo = O.ConvGeom(plan.B, H, W_, C, Ho, Wo, Co, layer.kernel_size[0], layer.kernel_size[1],
                                  layer.strides[0], layer.strides[1], pt, pl)
        elif self.conv:
            H, W_, C = tin.shape
            Ho, Wo, Co = tout.shape
            (pt, _), (pl, _) = layer.pads(tin.shape)
            self.geo = O.ConvGeom(plan.B, H, W_, C, Ho, Wo, Co, layer.kernel_size[0], layer.kernel_size[1],
                                  layer.strides[0], layer.strides[1], pt, pl)
            # narrow layers (C_out / C_in <= 32, e.g. Model B) take the direct VALU kernels
            # (per-thread FMA count bounds: above ~1k a thread's serial chain loses to the MFMA GEMM)
            narrow = os.environ.get("TDE_SMALLCONV", "1") != "0" and not plan.det
            r8 = lambda c: -(-c // 8) * 8  # noqa: E731
            kh, kw = layer.kernel_size
            sh, sw = layer.strides
            fwd_work = kh * kw * C * r8(Co)
            dgrad_work = -(-kh // sh) * -(-kw // sw) * Co * r8(C)
            self.small_fwd = narrow and Co <= 32 and fwd_work <= 1024 and O.smallconv_ok(self.geo)
            self.small_dgrad = (narrow and need_dgrad and C <= 32 and dgrad_work <= 1024
                                and O.smallconv_ok(self.geo, True))
            if self.small_fwd:
                self.shadows = {self.wname: ("row", "col")}
            # channel counts that defeat 16-byte gathers (RGB stem): explicit im2col + vector GEMMs
            self.use_im2col = (not self.small_fwd and C % 8 != 0 and os.environ.get("TDE_IM2COL", "1") != "0")
            # the RGB stem as a packed virtual conv through the LDS-DMA implicit GEMM (no im2col matrix);
            # input layer only (no input gradient in the packed layout)
            self.use_stem_pack = (self.use_im2col and not need_dgrad and O.stem_pack_ok(self.geo)
                                  and os.environ.get("TDE_STEM_PACK", "1") != "0")
            if self.use_stem_pack:
                self.use_im2col = False
            # filters whose K*Co partial sums fit in registers (Model B conv1: 3x3x1 -> 6)
            # (TDE_SMALLWG_IM2COL=1: also for layers whose forward runs on an explicit im2col matrix)
            self.small_wgrad = (narrow and O.smallconv_wgrad_ok(self.geo)
                                and (not self.use_im2col or os.environ.get("TDE_SMALLWG_IM2COL", "0") == "1"))
        # 3x3 / stride-1 / SAME 64-channel convs without bias or activation (ResNet-18 stage 1): the persistent
        # halo-tile kernel (csrc/kernels/haloconv.hip) for the forward and the input gradient
        self.halo = (self.conv and not self.f32 and not plan.det
                     and not (self.small_fwd or self.use_im2col or self.use_stem_pack)
                     and self.b is None and not self.relu and O.halo_ok(self.geo))
        # ... and its weight gradient (one pass over x and dY for all 9 taps; ordered partial reduction, so also
        # under TDE_DETERMINISTIC)
        self.halo_wg = (self.conv and not self.f32 and not (self.small_wgrad or self.use_im2col or self.use_stem_pack)
                        and O.halo_wgrad_ok(self.geo))
        self.colstats = None
        self.dz = None
        self.act_done = False   # the consumer's launch already applied the ReLU mask / bias gradient
        self.bnsum_of = None    # _Elementwise BN whose backward sums this layer's input-gradient epilogue takes

    def wpart_need(self, B):
        """f32 split-K partials of this layer's GEMMs (weight gradient, forward, input gradient)."""
        if self.conv:
            g = self.geo.with_batch(B)
            need = [O32.wgrad_part_elems(g.K, g.Co, g.B * g.Ho * g.Wo),
                    O32.fd_part_elems(g.B * g.Ho * g.Wo, g.Co, g.K)]
            if self.need_dgrad and g.sh == 1 and g.sw == 1:
                need.append(O32.fd_part_elems(g.B * g.H * g.W, g.C, g.KH * g.KW * g.Co))
            return max(need)
        fin, fout, rows = self.W.shape[0], self.W.shape[1], self.inp.rows(B)
        need = [O32.wgrad_part_elems(fin, fout, rows), O32.fd_part_elems(rows, fout, fin)]
        if self.need_dgrad:
            need.append(O32.fd_part_elems(rows, fin, fout))
        return max(need)

    def scratch_need(self, B):
        if self.f32:
            return 0
        if self.conv:
            g = self.geo.with_batch(B)
            return max(O.scratch_elems(g.B * g.Ho * g.Wo, g.Co, g.K),
                       O.scratch_elems(g.B * g.H * g.W, g.C, g.KH * g.KW * g.Co) if self.need_dgrad else 0)
        rows, fin, out = self.inp.rows(B), self.W.shape[0], self.W.shape[1]
        return max(O.scratch_elems(rows, out, fin), O.scratch_elems(rows, fin, out) if self.need_dgrad else 0)

    def wscratch_need(self, B):
        if self.f32:
            return 0
        if self.conv:
            g = self.geo.with_batch(B)
            if self.halo_wg:
                return O.halo_wgrad_scratch_elems(g)
            if self.use_im2col or self.small_wgrad:
                return 0
            if self.use_stem_pack:
                gv = O.stem_geometry(g)
                if O.stem_wgrad_ok(gv):
                    return O.stem_wgrad_scratch_elems(gv)
                return O.wgrad_scratch_elems(gv.K, gv.Co, gv.B * gv.Ho * gv.Wo)
            return O.wgrad_scratch_elems(g.K, g.Co, g.B * g.Ho * g.Wo)
        return O.wgrad_scratch_elems(self.W.shape[0], self.W.shape[1], self.inp.rows(B))

    def alloc(self, B, dev):
        if self.conv and self.use_stem_pack:
            gv = O.stem_geometry(self.geo.with_batch(B))
            self.xp = torch.zeros(gv.B * gv.H * gv.W * 8, dtype=bf16, device=dev)
            self.Wv = torch.zeros(gv.Co * gv.K, dtype=bf16, device=dev)
            self.gWv = torch.zeros(gv.K * gv.Co, dtype=torch.float32, device=dev)
        if self.conv and self.use_im2col:
            g = self.geo.with_batch(B)
            self.Kp = -(-g.K // 8) * 8
            self.xcol = torch.zeros(B * g.Ho * g.Wo * self.Kp, dtype=bf16, device=dev)
            self.Wt_pad = torch.zeros(g.Co * self.Kp, dtype=bf16, device=dev)
        if self.stats:
            self.colstats = torch.zeros(2 * O.STAT_SLOTS * self.out.C, dtype=torch.float64, device=dev)
        if (self.relu or self.gb is not None) and not self.act_done:
            self.dz = torch.zeros(B * self.out.numel, dtype=self.inp_dt(), device=dev)

    def inp_dt(self):
        return torch.float32 if self.f32 else bf16

    def bind_shadows(self, sh):
        if self.f32:
            return
        self.Wt = sh.shadow_views[(self.wname, "col")]
        self.Wrow = sh.shadow_views.get((self.wname, "row"))

    def grad_inputs(self):
        return [self.inp] if self.need_dgrad else []

    def fwd(self, p, B, training, mode="train"):
        cs = self.colstats if (self.stats and training) else None
        if self.f32:
            if self.conv:
                O32.conv_fwd(self.inp.root().buf, self.W, self.out.root().buf, self.geo.with_batch(B), bias=self.b,
                             relu=self.relu, colstats=cs, part=p.wpart)
            else:
                O32.dense_fwd(self.inp.root().buf, self.W.view(-1, self.W.shape[-1]), self.inp.rows(B),
                              self.out.root().buf, bias=self.b, relu=self.relu, colstats=cs, part=p.wpart)
            return
        if self.conv and self.use_stem_pack:
            g = self.geo.with_batch(B)
            O.stem_pack(self.inp.buf, g, self.xp, self.Wt, self.Wv)
            gv = O.stem_geometry(g)
            if self.b is None and not self.relu and not p.det and O.stem_fwd_ok(gv):
                O.stem_fwd(self.xp, self.Wv, self.out.root().buf, gv, colstats=cs)   # the tile kernel
            else:
                O.conv_fwd(self.xp, self.Wv.view(g.Co, -1), self.out.root().buf, gv, bias=self.b,
                           relu=self.relu, colstats=cs, scratch=p.scratch)
        elif self.conv and self.use_im2col:
            g = self.geo.with_batch(B)
            O.im2col(self.inp.buf, g, self.xcol, self.Wt, self.Wt_pad)
            O.conv_fwd_im2col(self.xcol, self.Wt_pad, self.out.root().buf, g, self.Kp, bias=self.b, relu=self.relu,
                              colstats=cs, scratch=p.scratch)
        elif self.conv and self.halo:
            O.halo_conv(self.inp.buf, self.Wt, self.out.root().buf, self.geo.with_batch(B), colstats=cs)
        elif self.conv and self.small_fwd:
            O.smallconv_fwd(self.inp.buf, self.Wrow, self.out.root().buf, self.geo.with_batch(B), bias=self.b,
                            relu=self.relu, colstats=cs)
        elif self.conv:
            O.conv_fwd(self.inp.buf, self.Wt, self.out.root().buf, self.geo.with_batch(B), bias=self.b,
                       relu=self.relu, colstats=cs, scratch=p.scratch)
        else:
            rows = self.inp.rows(B)
            O.dense_fwd(self.inp.buf, self.Wt, rows, y=self.out.root().buf, bias=self.b, relu=self.relu,
                        colstats=cs, scratch=p.scratch)

    def bwd(self, p, B):
        dout = self.out.root().grad
        if self.dz is not None:
            (O32 if self.f32 else O).act_bwd(dout, self.out.root().buf, self.out.rows(B), self.out.C, relu=self.relu,
                                             dz=self.dz, dbias=self.gb)
            dout = self.dz
        if self.f32:
            self._wgrad(p, B, dout)
            if not self.need_dgrad:
                return
            acc = self.accum[self.inp.root().id]
            if self.conv:
                O32.conv_dgrad(dout, self.W, self.inp.root().grad, self.geo.with_batch(B), accum=acc, part=p.wpart)
            else:
                O32.dense_dgrad(dout, self.W.view(-1, self.W.shape[-1]), self.inp.root().grad, self.inp.rows(B),
                                accum=acc, part=p.wpart)
            return
        side = p.side_stream
        if side is not None:
            side.wait_stream(torch.cuda.current_stream(p.device))
            with torch.cuda.stream(side):
                self._wgrad(p, B, dout)
        else:
            self._wgrad(p, B, dout)
        if not self.need_dgrad:
            return
        if self.conv:
            g = self.geo.with_batch(B)
            if self.small_dgrad:
                O.smallconv_dgrad(dout, self.Wrow, self.inp.root().grad, g, accum=self.accum[self.inp.root().id])
            elif self.halo:
                O.halo_conv(dout, self.Wrow, self.inp.root().grad, g, dgrad=True, accum=self.accum[self.inp.root().id])
            else:
                bs = None
                if self.bnsum_of is not None:
                    b = self.bnsum_of
                    bs = dict(y=b.inp.root().buf, res=b.res.root().buf if b.res is not None else None, saved=b.saved,
                              gamma=b.gamma, beta=b.beta, relu=b.relu, dstats=b.dstats)
                O.conv_dgrad(dout, self.Wrow, self.inp.root().grad, g, accum=self.accum[self.inp.root().id],
                             scratch=p.scratch, bnsum=bs)
        else:
            O.dense_dgrad(dout, self.Wrow, self.inp.root().grad, self.inp.rows(B),
                          accum=self.accum[self.inp.root().id], scratch=p.scratch)

    def _wgrad(self, p, B, dout):
        """This layer's weight gradient (all of it on the plan's side stream when there is one)."""
        if self.f32:
            if self.conv:
                O32.conv_wgrad(self.inp.root().buf, dout, self.gW, self.geo.with_batch(B), part=p.wpart)
            else:
                O32.dense_wgrad(self.inp.root().buf, dout, self.gW.view(self.W.shape[0], -1), self.inp.rows(B),
                                part=p.wpart)
            return
        if self.conv:
            g = self.geo.with_batch(B)
            if self.use_stem_pack:
                gv = O.stem_geometry(g)
                if O.stem_wgrad_ok(gv):   # the tile kernel: every packed-input and dY byte loaded once
                    O.stem_wgrad(self.xp, dout, self.gWv, gv, p.wscratch)
                else:
                    O.conv_wgrad(self.xp, dout, self.gWv, gv, scratch=p.wscratch)
                O.stem_unpack_wgrad(self.gWv, g, self.gW)
            elif self.halo_wg:
                O.halo_wgrad(self.inp.buf, dout, self.gW, g, p.wscratch)
            elif self.small_wgrad:
                O.smallconv_wgrad(self.inp.buf, dout, self.gW, g)
            elif self.use_im2col:
                O.conv_wgrad_im2col(self.xcol, dout, self.gW, g, self.Kp)
            else:
                O.conv_wgrad(self.inp.buf, dout, self.gW, g, scratch=p.wscratch)
        else:
            O.dense_wgrad(self.inp.buf, dout, self.gW.view(self.W.shape[0], -1), self.inp.rows(B),
                          scratch=p.wscratch)


class _Elementwise(_Stage):
    """BatchNormalization / Activation(relu) / Dropout / Add, each optionally followed by the
    fused [Add] [ReLU] [Dropout] chain: out = dropout(relu(affine(y) + res))."""

    def __init__(self, plan, layer, tin, tout, lid):
        self.plan = plan
        self.layer = layer
        self.node_index = tout.producer
        self.bn = isinstance(layer, L.BatchNormalization)
        self.add = isinstance(layer, L.Add)
        if self.add and len(tin) != 2:
            raise Unsupported(f"{layer.name}: Add of {len(tin)} inputs")
        self.inp = tin[0]
        self.res = tin[1] if self.add else None
        self.out = tout
        self.relu = isinstance(layer, L.Activation)
        self.drop = O.DropSpec()
        self.lid = lid
        self.defer_to = None
        self.stats_from_gemm = False
        self.pool = None  # _MaxPool whose forward this BN+ReLU stage runs in the same pass
        self.sums_fused = False  # backward sums taken by the input-gradient GEMM that writes dout last
        if isinstance(layer, L.Dropout):
            self.set_dropout(layer)
        st = plan.store
        self.colstats = None
        if self.bn:
            n = layer.name
            self.gamma = st.view(f"{n}/gamma") if layer.scale else None
            self.beta = st.view(f"{n}/beta") if layer.center else None
            self.ggamma = st.grad(f"{n}/gamma") if layer.scale and st.segments[f"{n}/gamma"].trainable else None
            self.gbeta = st.grad(f"{n}/beta") if layer.center and st.segments[f"{n}/beta"].trainable else None
            self.mmean = st.view(f"{n}/moving_mean")
            self.mvar = st.view(f"{n}/moving_variance")
        self._pnames = []
        if self.bn:
            self._pnames = [f"{layer.name}/{v}" for v, g in (("gamma", self.ggamma), ("beta", self.gbeta))
                            if g is not None]

    def param_names(self):
        return self._pnames

    def set_dropout(self, layer):
        g = Kb.make_generator(7919 + self.lid)
        seed = int(torch.randint(0, 2 ** 62, (1,), generator=g).item()) if layer.seed is None else int(layer.seed)
        self.drop = O.DropSpec(layer.rate, seed, self.plan.iterations, self.lid)

    def alloc(self, B, dev):
        C = self.inp.C
        self.O = O32 if self.plan.f32 else O
        if self.bn:
            self.saved = torch.zeros(2 * C, dtype=torch.float32, device=dev)
            self.dstats = torch.zeros(2 * O.STAT_SLOTS * C, dtype=self.plan.sdt, device=dev)
            if self.stats_from_gemm:
                self.colstats = None   # bound below to the producing GEMM's buffer
            else:
                self.colstats = torch.zeros(2 * O.STAT_SLOTS * C, dtype=torch.float64, device=dev)
        if self.bn and self.stats_from_gemm:
            for st in self.plan.stages:
                if isinstance(st, _Gemm) and st.out.root() is self.inp.root():
                    self._gemm = st
                    break

    def _stats(self):
        if self.stats_from_gemm:
            return self._gemm.colstats
        return self.colstats

    def grad_inputs(self):
        out = []
        if self.inp.root().id != 0:
            out.append(self.inp)
        if self.res is not None and self.res.root().id != 0:
            out.append(self.res)
        return out

    def fwd(self, p, B, training, mode="train"):
        R, C = self.inp.rows(B), self.inp.C
        drop = self.drop if (training and self.drop.rate > 0) else O.DropSpec()
        kw = dict(res=self.res.root().buf if self.res is not None else None, relu=self.relu, drop=drop,
                  iter_offset=0)
        if not self.bn:
            self.O.bn_fwd(self.inp.root().buf, self.out.root().buf, R, C, mode=0, **kw)
            return
        L_ = self.layer
        if training:
            stats = self._stats()
            if not self.stats_from_gemm:
                self.O.colstats(self.inp.root().buf, R, C, stats)
            upd = mode == "train"
            bessel = (R / max(R - 1, 1)) if L_.fused else 1.0
            if self.pool is not None:
                O.bn_relu_maxpool_fwd(self.inp.root().buf, R, C, self.pool.out.root().buf, self.pool.idx,
                                      self.pool.geo.with_batch(B), mode=1, stats=stats, saved=self.saved,
                                      gamma=self.gamma, beta=self.beta, eps=L_.epsilon,
                                      mmean=self.mmean if upd else None, mvar=self.mvar if upd else None,
                                      momentum=L_.momentum, bessel=bessel, zero_buf=self.dstats if upd else None)
                return
            self.O.bn_fwd(self.inp.root().buf, self.out.root().buf, R, C, mode=1, stats=stats, saved=self.saved,
                     gamma=self.gamma, beta=self.beta, eps=L_.epsilon, mmean=self.mmean if upd else None,
                     mvar=self.mvar if upd else None, momentum=L_.momentum, bessel=bessel,
                     zero_buf=self.dstats if upd else None, **kw)
        elif self.pool is not None:
            O.bn_relu_maxpool_fwd(self.inp.root().buf, R, C, self.pool.out.root().buf, self.pool.idx,
                                  self.pool.geo.with_batch(B), mode=2, gamma=self.gamma, beta=self.beta,
                                  eps=L_.epsilon, mmean=self.mmean, mvar=self.mvar)
        else:
            self.O.bn_fwd(self.inp.root().buf, self.out.root().buf, R, C, mode=2, gamma=self.gamma, beta=self.beta,
                     eps=L_.epsilon, mmean=self.mmean, mvar=self.mvar, **kw)

    def bwd(self, p, B):
        R, C = self.inp.rows(B), self.inp.C
        ir = self.inp.root()
        rr = self.res.root() if self.res is not None else None
        dx = ir.grad if ir.id != 0 else None
        dres = rr.grad if (rr is not None and rr.id != 0) else None
        if self.pool is not None:
            O.bn_pool_bwd(self.pool.out.root().grad, self.pool.idx, ir.buf, R, C, self.pool.geo.with_batch(B),
                          saved=self.saved, dstats=self.dstats, dx=dx, gamma=self.gamma, beta=self.beta, relu=True,
                          dx_accum=self.accum.get(ir.id, False), dgamma=self.ggamma, dbeta=self.gbeta,
                          zero_fwd=self._stats())
            return
        self.O.bn_bwd(self.out.root().grad, ir.buf, R, C, mode=1 if self.bn else 0,
                 saved=self.saved if self.bn else None, gamma=self.gamma if self.bn else None,
                 beta=self.beta if self.bn else None, res=rr.buf if rr is not None else None, relu=self.relu,
                 drop=self.drop, iter_offset=-1, dstats=self.dstats if self.bn else None,
                 dx=dx, dx_accum=self.accum.get(ir.id, False), dres=dres,
                 dres_accum=self.accum.get(rr.id, False) if rr is not None else False,
                 dgamma=self.ggamma if self.bn else None, dbeta=self.gbeta if self.bn else None,
                 zero_fwd=self._stats() if self.bn else None,
                 **({"sums_ready": True} if self.bn and self.sums_fused else {}))


class _MaxPool(_Stage):
    def __init__(self, plan, layer, tin, tout):
        self.inp, self.out = tin, tout
        self.node_index = tout.producer
        H, W_, C = tin.shape
        Ho, Wo, _ = tout.shape
        if layer.padding == "same":
            pt = L.tf_same_pads(H, layer.pool_size[0], layer.strides[0])[0]
            pl = L.tf_same_pads(W_, layer.pool_size[1], layer.strides[1])[0]
        else:
            pt = pl = 0
        self.geo = O.ConvGeom(plan.B, H, W_, C, Ho, Wo, C, layer.pool_size[0], layer.pool_size[1],
                              layer.strides[0], layer.strides[1], pt, pl)
        self.fused = False  # the producing BN+ReLU stage runs this pool's forward (bn_relu_maxpool_fwd)
        self.relu_from = None   # f32: the producing ReLU GEMM whose mask / bias gradient this backward applies
        self.f32 = plan.f32

    def alloc(self, B, dev):
        self.idx = torch.zeros(B * self.out.numel, dtype=torch.uint8, device=dev)
        self.O = O32 if self.f32 else O

    def grad_inputs(self):
        return [self.inp] if self.inp.root().id != 0 else []

    def fwd(self, p, B, training, mode="train"):
        if self.fused:
            return
        self.O.maxpool_fwd(self.inp.root().buf, self.out.root().buf, self.idx, self.geo.with_batch(B))

    def bwd(self, p, B):
        if self.inp.root().id == 0 or self.fused:
            return
        if self.relu_from is not None:
            O32.maxpool_bwd_relu(self.out.root().grad, self.out.root().buf, self.idx, self.inp.root().grad,
                                 self.geo.with_batch(B), dbias=self.relu_from.gb, accum=self.accum[self.inp.root().id])
            return
        self.O.maxpool_bwd(self.out.root().grad, self.idx, self.inp.root().grad, self.geo.with_batch(B),
                      accum=self.accum[self.inp.root().id])


class _GAP(_Stage):
    def __init__(self, plan, layer, tin, tout):
        self.inp, self.out = tin, tout
        self.node_index = tout.producer
        self.HW = tin.shape[0] * tin.shape[1]
        self.C = tin.shape[2]
        self.O = O32 if plan.f32 else O

    def alloc(self, B, dev):
        pass

    def grad_inputs(self):
        return [self.inp] if self.inp.root().id != 0 else []

    def fwd(self, p, B, training, mode="train"):
        self.O.gap_fwd(self.inp.root().buf, self.out.root().buf, B, self.HW, self.C)

    def bwd(self, p, B):
        if self.inp.root().id == 0:
            return
        self.O.gap_bwd(self.out.root().grad, self.inp.root().grad, B, self.HW, self.C,
                  accum=self.accum[self.inp.root().id])


class _Pad(_Stage):
    def __init__(self, plan, layer, tin, tout):
        self.inp, self.out = tin, tout
        self.node_index = tout.producer
        H, W_, C = tin.shape
        Ho, Wo, _ = tout.shape
        (t, _), (l, _) = layer.padding
        self.geo = O.ConvGeom(plan.B, H, W_, C, Ho, Wo, C, 1, 1, 1, 1, t, l)
        self.O = O32 if plan.f32 else O

    def alloc(self, B, dev):
        pass

    def grad_inputs(self):
        return [self.inp] if self.inp.root().id != 0 else []

    def fwd(self, p, B, training, mode="train"):
        self.O.pad_fwd(self.inp.root().buf, self.out.root().buf, self.geo.with_batch(B))

    def bwd(self, p, B):
        if self.inp.root().id == 0:
            return
        self.O.pad_bwd(self.out.root().grad, self.inp.root().grad, self.geo.with_batch(B),
                  accum=self.accum[self.inp.root().id])


class _Head(_Stage):
    """Last Dense -> f32 logits (+bias) -> softmax cross-entropy / accuracy / dlogits.

    Fused (<= 16 classes, <= 256 input features, the usual MNIST heads): ONE launch of the head
    kernel (csrc/kernels/head.hip) at the head's forward position does the Dense on the bf16 input with
    exact f32 MFMA, softmax-CE, accuracy, dW / db and the input gradient — the five launches of the
    general path (logits GEMM, xent, bias-grad, wgrad GEMM, dgrad GEMM) become one.  Otherwise: GEMM to
    f32 logits, the fused softmax-CE kernel, and the backward GEMMs."""

    def __init__(self, plan, layer, tin, tout, logits_out):
        if len(tin.shape) != 1:
            raise Unsupported("the head Dense must see a flat [B, features] input")
        self.plan = plan
        self.inp, self.out = tin, tout
        self.node_index = tout.producer
        self.layer = layer
        self.logits_out = logits_out
        st = plan.store
        self.wname = f"{layer.name}/kernel"
        self.bname = f"{layer.name}/bias" if layer.use_bias else None
        self.b = st.view(self.bname) if self.bname else None
        self.gb = st.grad(self.bname) if self.bname else None
        self.gW = st.grad(self.wname)
        self.need_dgrad = tin.root().id != 0
        self.C = layer.units
        self.H = tin.shape[0]
        self.W = st.view(self.wname)
        self.f32 = plan.f32
        self.fused = (not self.f32 and not plan.det and self.C <= 16 and self.H <= 256 and self.H % 4 == 0
                      and os.environ.get("TDE_FUSED_HEAD", "1") != "0")
        self.shadows = {} if (self.fused or self.f32) else {self.wname: ("row", "col") if self.need_dgrad else ("col",)}
        self.pre = None   # absorbed Dense: its ReLU mask and bias gradient are applied by the head launch

    def absorb(self, gemm):
        self.pre = gemm
        gemm.act_done = True

    def alloc(self, B, dev):
        self.logits = torch.zeros(B * self.C, dtype=torch.float32, device=dev)
        self.dlogits = torch.zeros(B * self.C, dtype=torch.float32 if self.f32 else bf16, device=dev)
        self.probs = torch.zeros(B * self.C, dtype=torch.float32, device=dev)

    def bind_shadows(self, sh):
        if self.fused or self.f32:
            return
        self.Wt = sh.shadow_views[(self.wname, "col")]
        self.Wrow = sh.shadow_views.get((self.wname, "row"))

    def grad_inputs(self):
        return [self.inp] if self.need_dgrad else []

    def wpart_need(self, B):
        return O32.wgrad_part_elems(self.H, self.C, B)

    def _fused_fwd(self, p, B, mode):
        from ..ops import kernels as K
        h = self.inp.root().buf[: B * self.H].view(B, self.H)
        if mode == "train":
            G = self.inp.root().grad[: B * self.H].view(B, self.H) if self.need_dgrad else None
            # the input gradient is stored, never accumulated: the head is the first backward writer
            assert not self.need_dgrad or not self.accum[self.inp.root().id]
            pre = self.pre
            # (with an absorbed Dense: h is its ReLU output, so h > 0 is its ReLU mask)
            K.head_xent(h, self.W, self.b, p._labels, B=B, scale=p.scale, compute_grad=True,
                        dW2=self.gW.view(self.H, -1), db2=self.gb, G=G, metrics=p.metrics, iterations=p.iterations,
                        pre_relu=pre is not None and pre.relu, dpre_bias=pre.gb if pre is not None else None)
        elif mode == "eval":
            K.head_xent(h, self.W, self.b, p._labels, B=B, scale=p.scale, compute_grad=False, metrics=p.metrics)
        else:
            K.head_xent(h, self.W, self.b, p._labels, B=B, scale=1.0, compute_grad=False,
                        probs=self.probs[: B * self.C].view(B, self.C), probs_are_logits=self.logits_out)

    def fwd(self, p, B, training, mode="train"):
        if self.fused:
            self._fused_fwd(p, B, mode)
            return
        if self.f32:
            O32.dense_fwd(self.inp.root().buf, self.W, B, self.logits, bias=self.b)
            if mode == "train":
                O32.xent(self.logits, p._labels, B, self.C, scale=p.scale, dlogits=self.dlogits, metrics=p.metrics,
                         iterations=p.iterations)
            elif mode == "eval":
                O32.xent(self.logits, p._labels, B, self.C, scale=p.scale, metrics=p.metrics)
            else:
                O32.xent(self.logits, p._labels, B, self.C, probs=self.probs, probs_are_logits=self.logits_out)
            return
        O.dense_fwd(self.inp.root().buf, self.Wt, B, logits=self.logits, bias=self.b)
        if mode == "train":
            O.xent(self.logits, p._labels, B, self.C, scale=p.scale, dlogits=self.dlogits, metrics=p.metrics,
                   iterations=p.iterations)
        elif mode == "eval":
            O.xent(self.logits, p._labels, B, self.C, scale=p.scale, metrics=p.metrics)
        else:
            O.xent(self.logits, p._labels, B, self.C, probs=self.probs, probs_are_logits=self.logits_out)

    def bwd(self, p, B):
        if self.fused:
            return   # done by the forward's launch
        if self.f32:
            if self.gb is not None:
                O32.act_bwd(self.dlogits, None, B, self.C, relu=False, dbias=self.gb)
            O32.dense_wgrad(self.inp.root().buf, self.dlogits, self.gW.view(self.H, -1), B, part=p.wpart)
            if self.need_dgrad:
                O32.dense_dgrad(self.dlogits, self.W, self.inp.root().grad, B, accum=self.accum[self.inp.root().id])
            return
        if self.gb is not None:
            O.act_bwd(self.dlogits, None, B, self.C, relu=False, dbias=self.gb)
        O.dense_wgrad(self.inp.root().buf, self.dlogits, self.gW, B, scratch=p.wscratch)
        if self.need_dgrad:
            O.dense_dgrad(self.dlogits, self.Wrow, self.inp.root().grad, B, accum=self.accum[self.inp.root().id])


def try_make(model, store, device, batch, global_batch, optimizer, loss):
    try:
        return LayerwisePlan(model, store, device, batch, global_batch, optimizer, loss)
    except Unsupported:
        return None


# ---------------------------------------------------------------------------------------
class _QRound(torch.autograd.Function):
    """Round to bf16 in the forward AND the backward: a tensor the plan stores in bf16 has a
    bf16 gradient buffer too."""

    @staticmethod
    def forward(ctx, x):
        return x.to(bf16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(bf16).to(g.dtype)


class _QGrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        return g.to(bf16).to(g.dtype)


def emulate_step(plan: LayerwisePlan, x, y, B=None):
    """Numerics oracle for the layer-wise plan: the same stage graph in float64 torch autograd,
    rounding to bf16 exactly where the bf16 plan stores bf16 tensors (activations, their gradients,
    weight shadows; nothing is rounded for the float32 plan).  Returns {variable: gradient} plus the BN
    moving statistics after the step.  Dropout must be inactive (its Philox stream is not reproduced here)."""
    import torch.nn.functional as F
    B = plan.B if B is None else B
    st = plan.store
    dd = torch.float64
    W = {n: st.view(n).detach().to(dd).clone().requires_grad_(st.segments[n].trainable) for n in st.order}

    f32 = getattr(plan, "f32", False)
    QR = (lambda t: t) if f32 else _QRound.apply   # noqa: E731
    QG = (lambda t: t) if f32 else _QGrad.apply    # noqa: E731

    def qw(n):
        w = W[n]
        return w if f32 else w + (w.to(bf16).to(dd) - w).detach()

    vals = {0: QR(x[:B].to(dd).reshape((B,) + plan.T[0].shape))}

    def get(t):
        return vals[t.root().id].reshape((B,) + t.shape)

    moving = {}
    loss = None
    for stg in plan.stages:
        if isinstance(stg, _Gemm):
            a = get(stg.inp)
            if stg.conv:
                lay = stg.layer
                (pt, pb), (pl, pr) = lay.pads(stg.inp.shape)
                xc = F.pad(a.permute(0, 3, 1, 2), (pl, pr, pt, pb))
                k = qw(stg.wname).permute(3, 2, 0, 1)
                o = F.conv2d(xc, k, stride=lay.strides).permute(0, 2, 3, 1)
            else:
                o = a.reshape(-1, a.shape[-1]) @ qw(stg.wname)
            if stg.bname:
                o = o + W[stg.bname]
            if stg.relu:
                o = F.relu(o)
            vals[stg.out.root().id] = QR(o.reshape(B, -1))
        elif isinstance(stg, _Elementwise):
            a = get(stg.inp)
            if stg.drop.rate > 0:
                raise ValueError("emulate_step: dropout must be disabled")
            if stg.bn:
                lay = stg.layer
                axes = tuple(range(a.dim() - 1))
                mean, var = a.mean(axes), a.var(axes, unbiased=False)
                z = (a - mean) * torch.rsqrt(var + lay.epsilon)
                if stg.gamma is not None:
                    z = z * W[f"{lay.name}/gamma"]
                if stg.beta is not None:
                    z = z + W[f"{lay.name}/beta"]
                R = a.numel() // a.shape[-1]
                bes = R / max(R - 1, 1) if lay.fused else 1.0
                m = lay.momentum
                moving[f"{lay.name}/moving_mean"] = W[f"{lay.name}/moving_mean"] * m + mean.detach() * (1 - m)
                moving[f"{lay.name}/moving_variance"] = (W[f"{lay.name}/moving_variance"] * m
                                                         + var.detach() * bes * (1 - m))
            else:
                z = a
            if stg.res is not None:
                z = z + get(stg.res)
            if stg.relu:
                z = F.relu(z)
            vals[stg.out.root().id] = QR(z.reshape(B, -1))
        elif isinstance(stg, _MaxPool):
            g = stg.geo
            a = get(stg.inp).permute(0, 3, 1, 2)
            pb = max((g.Ho - 1) * g.sh + g.KH - g.H - g.pt, 0)
            pr = max((g.Wo - 1) * g.sw + g.KW - g.W - g.pl, 0)
            a = F.pad(a, (g.pl, pr, g.pt, pb), value=float("-inf"))
            o = F.max_pool2d(a, (g.KH, g.KW), (g.sh, g.sw)).permute(0, 2, 3, 1)
            vals[stg.out.root().id] = o.reshape(B, -1)
        elif isinstance(stg, _GAP):
            vals[stg.out.root().id] = QR(get(stg.inp).mean((1, 2)).reshape(B, -1))
        elif isinstance(stg, _Pad):
            g = stg.geo
            a = get(stg.inp)
            o = F.pad(a, (0, 0, g.pl, g.Wo - g.W - g.pl, g.pt, g.Ho - g.H - g.pt))
            vals[stg.out.root().id] = o.reshape(B, -1)
        elif isinstance(stg, _Head):
            a = get(stg.inp)
            if stg.fused:   # f32 weights, f32 dlogits (the input gradient is rounded where it is stored)
                logits = a @ W[stg.wname]
            else:
                logits = a @ qw(stg.wname)
            if stg.bname:
                logits = logits + W[stg.bname]
            if not stg.fused:
                logits = QG(logits)
            loss = F.cross_entropy(logits, y[:B].long(), reduction="sum") * plan.scale
    loss.backward()
    out = {n: W[n].grad for n in st.names(trainable=True)}
    out.update(moving)
    return out, loss.item()
