"""Multi-replica / multi-step programs driving the per-replica plans.

``TrainProgram.run()`` executes ``steps_per_execution`` training steps:
    for each step:  every local replica: fwd+bwd (HIP plan)      [compute stream]
                    RCCL all-reduce(SUM) of each replica's flat grad bucket
                    every local replica: optimizer kernel
On a GPU with one local replica and a capturable communicator the whole
sequence is captured ONCE into a hipGraph (torch.cuda.CUDAGraph) and replayed:
the host enqueues one graph launch per execution, the inputs arrive in static
device ring buffers [S, B, ...] filled by one async H2D (or D2D) copy.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
import time

import numpy as np
import torch

from .. import _native as N
from . import program as PG


def _ctx(dev):
    return torch.cuda.device(dev) if dev.type == "cuda" else contextlib.nullcontext()


def _cast_bf16(src, dst):
    from ..ops import layer_ops as O
    O.cast_bf16(src, dst)


class _Stager:
    """Double-buffered pinned host staging for async H2D copies into a ring."""

    def __init__(self, shape, dtype, device):
        self.device = device
        self.cuda = device.type == "cuda"
        self.bufs = [torch.empty(shape, dtype=dtype, pin_memory=self.cuda) for _ in range(2 if self.cuda else 1)]
        self.events = [None] * len(self.bufs)
        self.k = 0

    def stage(self, arr, dst):
        """Copy numpy/torch ``arr`` into device tensor ``dst`` (same numel).  ``arr`` may also be a
        list of per-step numpy arrays: they are packed straight into the pinned buffer (no stack)."""
        if isinstance(arr, (list, tuple)):
            buf = self._next_buf()
            flat = buf.view(-1).numpy()
            n = 0
            for part in arr:
                part = np.asarray(part)
                np.copyto(flat[n: n + part.size], part.reshape(-1), casting="unsafe")
                n += part.size
            self._launch(flat_t=buf.view(-1), n=n, dst=dst)
            return
        if torch.is_tensor(arr) and arr.device == dst.device:
            if self.cuda and arr.dtype == torch.float32 and dst.dtype == torch.bfloat16:
                _cast_bf16(arr.reshape(-1).contiguous(), dst.view(-1)[: arr.numel()])   # HIP cast kernel
            else:
                dst.view(-1)[: arr.numel()].copy_(arr.reshape(-1).to(dst.dtype), non_blocking=True)
            return
        if torch.is_tensor(arr):
            arr = arr.detach().cpu().numpy()
        arr = np.asarray(arr)
        buf = self._next_buf()
        flat = buf.view(-1)
        n = arr.size
        np.copyto(flat[:n].numpy(), arr.reshape(-1), casting="unsafe")
        self._launch(flat_t=flat, n=n, dst=dst)

    def _next_buf(self):
        buf = self.bufs[self.k]
        ev = self.events[self.k]
        if ev is not None:
            ev.synchronize()   # the H2D copy that last read this buffer is done
        return buf

    def _launch(self, flat_t, n, dst):
        if dst.dtype != flat_t.dtype:
            # e.g. a bf16 input ring: async H2D of the f32 staging, then one on-device cast
            if getattr(self, "dev_tmp", None) is None or self.dev_tmp.numel() < flat_t.numel():
                self.dev_tmp = torch.empty(flat_t.numel(), dtype=flat_t.dtype, device=dst.device)
            self.dev_tmp[:n].copy_(flat_t[:n], non_blocking=self.cuda)
            if self.cuda and self.dev_tmp.dtype == torch.float32 and dst.dtype == torch.bfloat16:
                _cast_bf16(self.dev_tmp[:n], dst.view(-1)[:n])
            else:
                dst.view(-1)[:n].copy_(self.dev_tmp[:n])
        else:
            dst.view(-1)[:n].copy_(flat_t[:n], non_blocking=self.cuda)
        if self.cuda:
            e = torch.cuda.Event()
            e.record(torch.cuda.current_stream(self.device))
            self.events[self.k] = e
        self.k = (self.k + 1) % len(self.bufs)


def _same_device_pair(src, ring):
    """A contiguous device tensor of the ring's dtype that fits it (copied without a cast or a host hop)."""
    return (os.environ.get("TDE_STAGE_FUSED", "1") != "0" and torch.is_tensor(src) and ring.is_cuda
            and src.device == ring.device and src.dtype == ring.dtype
            and src.is_contiguous() and src.numel() <= ring.numel()
            # tde_copy_pairs moves 4-byte words: odd bf16 counts / offsets take the staging path
            and (src.numel() * src.element_size()) % 4 == 0
            and src.data_ptr() % 4 == 0 and ring.data_ptr() % 4 == 0)


class Program:
    def __init__(self, model, strategy, global_batch, training, steps_per_execution=1):
        self.model = model
        self.strategy = strategy
        self.world = strategy.num_replicas_in_sync
        if global_batch % self.world:
            raise ValueError(f"global batch {global_batch} is not divisible by {self.world} replicas")
        self.global_batch = global_batch
        self.B = global_batch // self.world
        self.S = max(1, int(steps_per_execution)) if training else 1
        self.stores = model._replica_stores(strategy)
        self.devices = list(strategy.local_devices)
        opt = model.optimizer if training else None
        self.plans = [PG.make_plan(model, st, dev, self.B, global_batch, opt, model.loss)
                      for st, dev in zip(self.stores, self.devices)]
        self.comm = strategy.comm if self.world > 1 else None
        self.grad_comm = self.comm   # carries the gradient bucket (may differ from self.comm: _pick_step_mode)
        xs = tuple(model.input_shape[1:])
        self.x_shape = xs
        xdt = self.plans[0].input_dtype
        self.x_ring = [torch.zeros((self.S, self.B) + xs, dtype=xdt, device=d) for d in self.devices]
        self.y_ring = [torch.zeros((self.S, self.B), dtype=torch.int32, device=d) for d in self.devices]
        self.x_stage = [_Stager((self.S, self.B) + xs, torch.float32, d) for d in self.devices]
        self.y_stage = [_Stager((self.S, self.B), torch.int32, d) for d in self.devices]
        self.graph = None          # the last captured graph (diagnostics)
        self.graphs = {}           # start parities -> (hipGraph of one execution, end parities)
        self._graph_key = None
        cuda = all(d.type == "cuda" for d in self.devices)
        env = os.environ.get("TDE_GRAPH", "1") != "0"
        # several local replicas over a per-replica communicator (in-process xGMI): every device group's
        # steps run on a stream of their own and are captured into a hipGraph of their own
        pr = bool(training and cuda and len(self.devices) > 1 and getattr(self.comm, "per_replica", False))
        cut = self._group_cut() if pr else None
        # every all-reduce call must fit the xGMI window: the whole bucket, or each reverse-order bucket
        self.per_replica = pr and (all(p.store.g.numel() <= self.comm.max_elems for p in self.plans) or
                                   (cut is not None and max(hi - lo for _, lo, hi in cut) <= self.comm.max_elems))
        if (training and cuda and len(self.devices) > 1 and getattr(self.comm, "per_replica", False)
                and not self.per_replica):
            import warnings
            warnings.warn(f"gradient bucket of {self.plans[0].store.g.numel()} elements exceeds the in-process xGMI "
                          f"window ({self.comm.max_elems}; TDE_XGMI_MAX_ELEMS raises it): the replicas run eagerly "
                          "without per-device hipGraphs")
        # replicas grouped by device (the communicator's groups): one stream + one graph per group
        self.groups = list(self.comm.groups) if self.per_replica else None
        self.rstreams = [torch.cuda.Stream(self.devices[g[0]]) for g in self.groups] if self.per_replica else None
        self.use_graph = bool(training and cuda and env and self.plans[0].kind != "reference" and
                              ((len(self.devices) == 1 and (self.comm is None or self.comm.capturable))
                               or self.per_replica))
        self._comm_warm = False
        self._dbg = os.environ.get("TDE_DEBUG_SYNC", "0") not in ("", "0") and cuda
        self._host_trace = [] if os.environ.get("TDE_HOST_TRACE", "0") not in ("", "0") else None
        self._trace = None   # enable_trace(): per-step state buffers
        self.buckets = self._plan_buckets() if training else None
        self._comm_stream = torch.cuda.Stream(self.devices[0]) if self.buckets else None
        # per-device-group layouts (Mirrored / MWMS with K GPUs per worker): the same reverse-order buckets,
        # each issued by the group's launch on a comm stream of its own as soon as the group's last replica
        # has finished the backward stage that finalises it
        self.group_buckets = self._plan_group_buckets() if training else None
        self._gcomm = ([torch.cuda.Stream(self.devices[g[0]]) for g in self.groups] if self.group_buckets
                       else None)
        self.comm_applies = False
        self.exchange = "post_backward" if self.comm is not None else "none"
        if training:
            self._pick_step_mode()

    def _pick_step_mode(self):
        """Fused optimizer placement (TDE_FUSED_STEP=0 keeps the separate optimizer launch): with one
        replica the update runs inside the step's own kernels ("local"); with one replica per process
        under the xGMI communicator it runs inside the gradient all-reduce ("xgmi")."""
        from ..parallel.comm import XgmiCommunicator
        self._route_grads()
        if os.environ.get("TDE_FUSED_STEP", "1") == "0" or self.buckets or self.group_buckets:
            return
        if self.per_replica:
            if all(p.supports_step_mode("xgmi") for p in self.plans):
                for p in self.plans:
                    p.set_step_mode("xgmi")
                self.comm_applies = True
                self._setup_push()
            return
        if len(self.plans) != 1:
            return
        plan = self.plans[0]
        if self.comm is None and plan.supports_step_mode("local"):
            plan.set_step_mode("local")
        elif isinstance(self.comm, XgmiCommunicator) and plan.supports_step_mode("xgmi"):
            plan.set_step_mode("xgmi")
            self.comm_applies = True
            self.grad_comm = self.comm
            self._setup_push()

    def _setup_push(self):
        """Fused data-parallel exchange (TDE_XGMI_PUSH=0 disables): a plan whose backward can store its
        big weight gradient straight into the xGMI owners' windows does so, and the all-reduce launch
        after it only pushes the rest of the bucket — the exchange's push phase overlaps the backward."""
        self.exchange = "post_backward"
        if os.environ.get("TDE_XGMI_PUSH", "1") == "0" or not hasattr(self.comm, "push_spec"):
            return
        if not all(hasattr(p, "push_range") and p.push_range() is not None for p in self.plans):
            return
        for i, p in enumerate(self.plans):
            lo, _ = p.push_range()
            M = p.store.g.numel()
            spec = self.comm.push_spec(i, M, lo) if self.per_replica else self.comm.push_spec(M, lo)
            p.set_push(spec)
        self.exchange = "fused_push"

    def _route_grads(self):
        """The xGMI kernel keeps the bucket over a slightly faster RCCL only because it can also apply the
        update; a plan that cannot fuse it sends a plain all-reduce to whichever measured faster."""
        from ..parallel.comm import XgmiCommunicator
        if isinstance(self.comm, XgmiCommunicator) and not self.comm.plain_ok and self.comm.fallback is not None:
            self.grad_comm = self.comm.fallback

    def _plan_buckets(self):
        """Reverse-order gradient buckets all-reduced on a comm stream while backward still runs
        (one local replica, a stream-ordered collective, a plan that exposes its backward order).
        ``TDE_OVERLAP=0`` keeps the single post-backward all-reduce; ``TDE_BUCKET_MB`` sizes buckets."""
        if self.comm is None or len(self.plans) != 1 or self.devices[0].type != "cuda":
            return None
        if not getattr(self.comm, "capturable", False) or os.environ.get("TDE_OVERLAP", "1") == "0":
            return None
        plan = self.plans[0]
        if not hasattr(plan, "grad_buckets"):
            return None
        mb = float(os.environ.get("TDE_BUCKET_MB", "8"))
        bk = plan.grad_buckets(max(1, int(mb * 2 ** 20 / 4)))
        return bk if len(bk) > 1 else None

    def _plan_group_buckets(self):
        """``_plan_buckets`` for the per-device-group layouts (``per_replica``): every replica holds the same
        model, so one cut serves all; issued per group on the group's comm stream.  ``TDE_OVERLAP=0`` keeps
        the single post-backward launch per group."""
        if not self.per_replica:
            return None
        return self._group_cut()

    def _group_cut(self):
        if os.environ.get("TDE_OVERLAP", "1") == "0":
            return None
        if not all(hasattr(p, "grad_buckets") for p in self.plans):
            return None
        mb = float(os.environ.get("TDE_BUCKET_MB", "8"))
        bk = self.plans[0].grad_buckets(max(1, int(mb * 2 ** 20 / 4)))
        if len(bk) <= 1 or any(lo % 4 for _, lo, _ in bk):   # the xGMI launch takes 16-byte aligned slices
            return None
        return bk

    @property
    def plan_kind(self):
        return self.plans[0].kind

    # ------------------------------------------------------------------ staging
    def stage(self, per_replica_steps):
        """per_replica_steps[r] = (x [S,B,...], y [S,B]) for local replica r."""
        for r, (x, y) in enumerate(per_replica_steps):
            with _ctx(self.devices[r]):
                xr, yr = self.x_ring[r], self.y_ring[r]
                if _same_device_pair(x, xr) and _same_device_pair(y, yr):
                    # a device-resident batch group: x and y into the ring in ONE copy launch
                    N.check(N.hip().tde_copy_pairs(
                        2, (C.c_void_p * 2)(x.data_ptr(), y.data_ptr()), (C.c_void_p * 2)(xr.data_ptr(), yr.data_ptr()),
                        (C.c_longlong * 2)(x.numel() * x.element_size(), y.numel() * y.element_size()),
                        N.stream_ptr(xr.device)), "tde_copy_pairs")
                    continue
                self.x_stage[r].stage(x, xr)
                self.y_stage[r].stage(y, yr)

    # ------------------------------------------------------------------ training
    def _reduce_and_apply(self):
        """Gradient all-reduce + optimizer of every local replica (after their backward)."""
        if self.comm_applies:
            plan = self.plans[0]
            with _ctx(plan.device):
                self.comm.all_reduce_apply_(plan.store.g, plan.xg_apply_spec())
            self._debug_sync("gradient all-reduce + optimizer")
            return
        if self.comm is not None:
            self.grad_comm.all_reduce_([p.store.g for p in self.plans])
            self._debug_sync("gradient all-reduce")
        for plan in self.plans:
            if plan.applies_in_step:
                continue
            with _ctx(plan.device):
                plan.apply()
            self._debug_sync("optimizer")

    def _reduce_and_apply_group(self, gi):
        """Device group gi's gradient all-reduce (+ optimizer) as one launch on its stream."""
        idx = self.groups[gi]
        plans = [self.plans[r] for r in idx]
        if self.comm_applies:
            self.comm.all_reduce_group_(gi, [p.store.g for p in plans], [p.xg_apply_spec() for p in plans])
            return
        self.comm.all_reduce_group_(gi, [p.store.g for p in plans])
        for p in plans:
            if not p.applies_in_step:
                p.apply()

    def _steps_group(self, gi, S, B=None):
        """S training steps of device group gi (its launches only wait for the other groups on the device)."""
        idx = self.groups[gi]
        if self.group_buckets:
            for s in range(S):
                self._overlapped_group_step(gi, s, B)
            return
        for s in range(S):
            for r in idx:
                self.plans[r].train_step(self.x_ring[r][s], self.y_ring[r][s], B)
            if self._host_trace is not None:   # TDE_HOST_TRACE: host wall time of each all-reduce enqueue
                self._host_trace.append((gi, time.time()))
            self._reduce_and_apply_group(gi)
            self._debug_sync("train_step + gradient all-reduce")
        for r in idx:
            self.plans[r].finish()

    def _overlapped_group_step(self, gi, s, B=None):
        """Device group gi, one step with the reverse-order gradient buckets: the group's replicas run
        forward + backward in turn on the group's stream; while the LAST one's backward is still running,
        each bucket's group all-reduce launch (every replica's slice in one xGMI launch) is enqueued on the
        group's comm stream right after the backward stage that finalises it (event edges, captured into
        the group's hipGraph); the optimizer launches wait for the comm stream."""
        idx = self.groups[gi]
        plans = [self.plans[r] for r in idx]
        dev = self.devices[idx[0]]
        main = torch.cuda.current_stream(dev)
        cs = self._gcomm[gi]
        ready = {}
        for i, lo, hi in self.group_buckets:
            ready.setdefault(i, []).append((lo, hi))
        sides = [p.side_stream for p in plans if getattr(p, "side_stream", None) is not None]

        def after_bwd(i):
            for lo, hi in ready.get(i, ()):
                cs.wait_stream(main)
                for sd in sides:
                    cs.wait_stream(sd)
                with torch.cuda.stream(cs):
                    self.comm.all_reduce_group_(gi, [p.store.g[lo:hi] for p in plans])

        for r in idx[:-1]:
            self.plans[r].train_step(self.x_ring[r][s], self.y_ring[r][s], B)
        r = idx[-1]
        self.plans[r].train_step(self.x_ring[r][s], self.y_ring[r][s], B, after_bwd=after_bwd)
        main.wait_stream(cs)
        self._debug_sync("train_step + bucketed group all-reduce")
        for p in plans:
            p.apply()
        self._debug_sync("optimizer")

    @contextlib.contextmanager
    def _on_group(self, gi):
        """Group gi's stream, ordered after (and joined back into) the device's current stream, where the
        input staging runs."""
        dev, s = self.devices[self.groups[gi][0]], self.rstreams[gi]
        with torch.cuda.device(dev):
            cur = torch.cuda.current_stream(dev)
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                yield
            cur.wait_stream(s)

    def _finish(self):
        for plan in self.plans:
            with _ctx(plan.device):
                plan.finish()

    def _steps(self, S, B=None):
        if self.per_replica:
            for gi in range(len(self.groups)):
                with self._on_group(gi):
                    self._steps_group(gi, S, B)
            return
        for s in range(S):
            if self.buckets:
                self._overlapped_step(s, B)
                continue
            for r, plan in enumerate(self.plans):
                with _ctx(plan.device):
                    plan.train_step(self.x_ring[r][s], self.y_ring[r][s], B)
                self._debug_sync("train_step")
            self._reduce_and_apply()
            if self._trace is not None:
                self._record(s)
        self._finish()

    def enable_trace(self):
        """Diagnostics: after every step of an execution, copy each plan's ``trace_tensors()`` (weights and
        the plan's cross-step state) into ``self.trace[r][s]`` — captured into the hipGraph like the steps,
        so an execution's per-step states are readable after it (``sync()`` first).  Single-group layouts."""
        if self.per_replica:
            raise NotImplementedError("per-step traces are recorded for single-group layouts")
        self.graphs = {}
        self._trace = []
        for p in self.plans:
            n = sum(t.numel() for t in p.trace_tensors())
            self._trace.append(torch.zeros(self.S, n, dtype=torch.float32, device=p.device))
        self.trace = self._trace

    def _record(self, s):
        for r, p in enumerate(self.plans):
            with _ctx(p.device):
                o = 0
                for t in p.trace_tensors():
                    n = t.numel()
                    self._trace[r][s, o: o + n].copy_(t.reshape(-1))
                    o += n

    def _overlapped_step(self, s, B):
        """fwd + bwd on the compute stream; each gradient bucket's all-reduce is enqueued on the comm
        stream right after the backward stage that finalises it (event dependency), so it overlaps
        the remaining backward; the optimizer waits for the comm stream."""
        plan = self.plans[0]
        main = torch.cuda.current_stream(plan.device)
        cs = self._comm_stream
        g = plan.store.g
        ready = {}
        for i, lo, hi in self.buckets:
            ready.setdefault(i, []).append((lo, hi))

        side = getattr(plan, "side_stream", None)   # weight gradients of the layer-wise plan

        def after_bwd(i):
            for lo, hi in ready.get(i, ()):
                cs.wait_stream(main)
                if side is not None:
                    cs.wait_stream(side)
                with torch.cuda.stream(cs):
                    self.grad_comm.all_reduce_([g[lo:hi]])

        with _ctx(plan.device):
            plan.train_step(self.x_ring[0][s], self.y_ring[0][s], B, after_bwd=after_bwd)
            main.wait_stream(cs)
            self._debug_sync("train_step + bucketed gradient all-reduce")
            plan.apply()
            self._debug_sync("optimizer")

    def _debug_sync(self, what):
        if self._dbg:
            try:
                self.sync()
            except RuntimeError as e:
                raise RuntimeError(f"device fault surfaced after {what} (TDE_DEBUG_SYNC): {e}") from e

    def _warm_comm(self):
        if self.comm is not None and not self._comm_warm:
            scratch = [torch.zeros(64, device=d) for d in self.devices]
            self.comm.all_reduce_(scratch)
            for d in self.devices:
                if d.type == "cuda":
                    torch.cuda.synchronize(d)
            self._comm_warm = True

    def _key(self):
        o = self.model.optimizer
        return (float(o.learning_rate), o.kind, tuple(sorted(o.hparams().items())))

    def _parities(self):
        return tuple(p.parity for p in self.plans)

    def capture(self):
        """Capture one execution (S steps) as a hipGraph for the plans' current step parities; the
        parities are restored afterwards (capturing launches nothing)."""
        import gc
        self._warm_comm()
        for p in self.plans:
            p.refresh()
        start = self._parities()
        if self.per_replica:
            gs = []
            try:
                for gi, idx in enumerate(self.groups):
                    dev = self.devices[idx[0]]
                    with torch.cuda.device(dev):
                        torch.cuda.synchronize(dev)
                        g = torch.cuda.CUDAGraph()
                        gc.collect()
                        gc.disable()
                        try:
                            with torch.cuda.graph(g, stream=self.rstreams[gi]):
                                self._steps_group(gi, self.S)
                        finally:
                            gc.enable()
                        torch.cuda.synchronize(dev)
                    gs.append(g)
                self._end = self._parities()
            finally:
                for p, q in zip(self.plans, start):
                    p.parity = q
            self.graphs[start] = (gs, self._end)
            self._graph_key = self._key()
            self.graph = gs[0]
            return
        dev = self.devices[0]
        with torch.cuda.device(dev):
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            # no garbage collection while capturing: finalizers of unrelated dead objects (graphs,
            # events, device buffers of earlier programs) must not run inside the capture
            gc.collect()
            gc.disable()
            try:
                with torch.cuda.graph(g):
                    self._steps(self.S)
            finally:
                gc.enable()
                self._end = self._parities()
                for p, q in zip(self.plans, start):
                    p.parity = q
            torch.cuda.synchronize(dev)
        self.graphs[start] = (g, self._end)
        self._graph_key = self._key()
        self.graph = g

    def run(self):
        if self.use_graph:
            if self._graph_key != self._key():
                self.graphs = {}
            if self._parities() not in self.graphs:
                try:
                    self.capture()
                    end = self.graphs[self._parities()][1]
                    if end not in self.graphs:
                        # an odd number of steps per execution alternates the start parity: capture the
                        # other graph now too, so no later execution pays a capture
                        cur = self._parities()
                        for p, q in zip(self.plans, end):
                            p.parity = q
                        self.capture()
                        for p, q in zip(self.plans, cur):
                            p.parity = q
                except RuntimeError as e:
                    # e.g. a collective implementation that refuses stream capture: keep training
                    # with eager launches (same kernels, one host launch each) instead of failing
                    import warnings
                    warnings.warn(f"hipGraph capture of the training step failed ({e}); running eagerly")
                    self.use_graph = False
                    self.graph = None
                    self.graphs = {}
                    self.sync()
                    self._steps(self.S)
                    return
            g, end = self.graphs[self._parities()]
            if self.per_replica:
                for gi, gr in enumerate(g):   # one graph launch per device group, each on its stream
                    with self._on_group(gi):
                        gr.replay()
            else:
                with torch.cuda.device(self.devices[0]):
                    g.replay()
            for p, q in zip(self.plans, end):
                p.parity = q
        else:
            self._warm_comm()
            for p in self.plans:
                p.refresh()
            self._steps(self.S)

    def run_single(self, per_replica, global_actual):
        """One (possibly partial) step executed eagerly. per_replica[r] = (x[B_r,...], y[B_r])."""
        self._warm_comm()
        for r, (x, y) in enumerate(per_replica):
            with _ctx(self.devices[r]):
                n = len(y)
                self.x_stage[r].stage(x, self.x_ring[r][0])
                self.y_stage[r].stage(y, self.y_ring[r][0])
        for p in self.plans:
            p.refresh()
        scales = [p.scale for p in self.plans]
        for p in self.plans:
            p.scale = 1.0 / float(global_actual)
        try:
            if self.per_replica:   # every group issues its all-reduce, with or without data
                for gi, idx in enumerate(self.groups):
                    with self._on_group(gi):
                        for r in idx:
                            n = len(per_replica[r][1])
                            if n > 0:
                                self.plans[r].train_step(self.x_ring[r][0], self.y_ring[r][0], n)
                        if self.group_buckets:   # the same bucket calls as the captured steps, post-backward
                            plans = [self.plans[r] for r in idx]
                            for _, lo, hi in self.group_buckets:
                                self.comm.all_reduce_group_(gi, [p.store.g[lo:hi] for p in plans])
                            for p in plans:
                                p.apply()
                        else:
                            self._reduce_and_apply_group(gi)
                        for r in idx:
                            self.plans[r].finish()
                return
            if self.buckets:   # every rank issues the same bucket collectives, with or without data
                n = len(per_replica[0][1])
                if n > 0:
                    self._overlapped_step(0, n)
                else:
                    plan = self.plans[0]
                    with _ctx(plan.device):
                        for _, lo, hi in self.buckets:
                            self.grad_comm.all_reduce_([plan.store.g[lo:hi]])
                        plan.apply()
                return
            for r, plan in enumerate(self.plans):
                n = len(per_replica[r][1])
                with _ctx(plan.device):
                    if n > 0:
                        plan.train_step(self.x_ring[r][0], self.y_ring[r][0], n)
                    elif plan.applies_in_step:
                        continue   # no data, nothing to reduce: the fused step has no update to make
            self._reduce_and_apply()
            self._finish()
        finally:
            for p, s in zip(self.plans, scales):
                p.scale = s

    # ------------------------------------------------------------------ eval / predict
    def eval_batch(self, per_replica):
        for r, (x, y) in enumerate(per_replica):
            n = len(y)
            if n == 0:
                continue
            with _ctx(self.devices[r]):
                self.x_stage[r].stage(x, self.x_ring[r][0])
                self.y_stage[r].stage(y, self.y_ring[r][0])
                self.plans[r].eval_step(self.x_ring[r][0], self.y_ring[r][0], n)

    def predict_batch(self, x):
        n = len(x)
        with _ctx(self.devices[0]):
            self.x_stage[0].stage(x, self.x_ring[0][0])
            out = self.plans[0].predict(self.x_ring[0][0], n)
            return out[:n].float().cpu().numpy().copy()

    # ------------------------------------------------------------------ metrics
    def reset_metrics(self):
        for p in self.plans:
            p.reset_metrics()

    def local_metrics(self):
        acc = None
        for p in self.plans:
            m = p.metrics.detach().double().cpu()
            acc = m if acc is None else acc + m
        return acc

    def global_metrics(self):
        """SUM of the metric accumulators over ALL replicas (SyncOnRead SUM, C3/C5)."""
        if self.comm is None:
            return self.local_metrics()
        self.comm.check_health()   # surfaces a timed-out peer wait of the xGMI all-reduce
        bufs = [p.metrics.clone() for p in self.plans]
        self.comm.all_reduce_(bufs)
        for d in self.devices:
            if d.type == "cuda":
                torch.cuda.synchronize(d)
        return bufs[0].double().cpu()

    def on_weights_loaded(self):
        for p in self.plans:
            with _ctx(p.device):
                p.on_weights_loaded()

    def sync(self):
        for d in self.devices:
            if d.type == "cuda":
                torch.cuda.synchronize(d)
