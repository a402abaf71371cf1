"""Profiling helpers.

* ``ProfilerHook`` (re-exported from train.hooks): Chrome-trace timelines every
  N steps, the reference's commented ``tf.estimator.ProfilerHook`` (MKD:235-237).
* ``trace(fn, path)``: one-off torch.profiler Chrome trace of a callable.
* ``rocprof_command(...)``: the rocprofv3 command lines used for the profiles
  committed under profiles/ (kernel trace + stats; PMC counters in a separate run).
* ``step_timer``: host perf_counter + HIP event timer for ms/step reporting.
"""
from __future__ import annotations

import contextlib
import time

from ..train.hooks import ProfilerHook  # noqa: F401


def trace(fn, path, *args, **kw):
    import torch
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts) as prof:
        out = fn(*args, **kw)
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    prof.export_chrome_trace(str(path))
    return out


def rocprof_command(cmd, out_dir="gpurun_out/prof", pmc=None):
    base = ["rocprofv3", "--kernel-trace", "--stats", "-d", out_dir, "-o", "run", "--output-format", "csv"]
    if pmc:
        base = ["rocprofv3", "--pmc", *pmc, "-d", out_dir, "-o", "pmc", "--output-format", "csv"]
    return base + ["--"] + list(cmd)


@contextlib.contextmanager
def step_timer(result: dict, key="ms"):
    import torch
    cuda = torch.cuda.is_available()
    if cuda:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    yield
    if cuda:
        torch.cuda.synchronize()
    result[key] = (time.perf_counter() - t0) * 1e3
