#!/usr/bin/env python
"""Device time of one PS device-plane exchange (csrc/kernels/ps_device.hip ps_dev_step_kernel) for Model B's
variables on one shard (window allocated in-process): push (SGD / momentum) + pull + counters, and pull only.
Event-timed over many back-to-back launches; one JSON line per form."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tensorflow_distributed_example_amd as tde  # noqa: E402
from tensorflow_distributed_example_amd import _native as N  # noqa: E402
from tensorflow_distributed_example_amd.parallel import ps_device as PD  # noqa: E402


def main():
    m = tde.zoo.mnist_bn_cnn()
    m.compile(loss="sparse_categorical_crossentropy", optimizer=tde.optimizers.SGD(0.01))
    m.build()
    st = m._store
    lib = N.hip()
    out = {}
    for kind in (0, 1):
        segs, sizes = PD.layout(st, {n: 0 for n in st.order}, 1, slots=kind != 0)
        win = C.c_void_p()
        handle = (C.c_char * 64)()
        N.check(lib.tde_psdev_alloc(0, PD.shard_bytes(sizes[0]), C.byref(win), handle), "tde_psdev_alloc")
        wins = (C.c_void_p * 1)(win.value)
        segs_d = torch.from_numpy(segs.view(np.uint8).copy()).cuda()
        beg = np.zeros(len(segs) + 1, np.int64)
        beg[1:] = np.cumsum(segs["n"])
        beg_d = torch.from_numpy(beg).cuda()
        ns = max(st.state.numel(), 1)
        sp = torch.zeros(ns, device="cuda")
        mom = torch.full((ns,), 0.99, device="cuda")
        done = torch.zeros(1, dtype=torch.int32, device="cuda")
        g = torch.randn_like(st.g) * 1e-3

        def launch(push):
            if push:
                st.g.copy_(g)
            N.check(lib.tde_psdev_step(wins, 1, N.ptr(segs_d), N.ptr(beg_d), len(segs), int(beg[-1]), N.ptr(st.w),
                                       N.ptr(st.g) if push else None,
                                       N.ptr(st.state), N.ptr(sp), N.ptr(mom), 0.01, 0.9, kind, 1, 1, N.ptr(done),
                                       None, None, 0, N.stream_ptr()), "tde_psdev_step")

        for push in (True, False):
            for _ in range(5):
                launch(push)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 200
            e0.record()
            for _ in range(n):
                launch(push)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / n
            out[f"{'sgd' if kind == 0 else 'momentum'}_{'push_pull' if push else 'pull'}_us"] = round(us, 2)
        lib.tde_psdev_free(win)
    out["elements"] = int(st.w.numel())
    out["note"] = "push_pull includes a 1.2 MB device copy of the gradient before each launch"
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
