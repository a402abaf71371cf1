"""Estimator SessionRunHook equivalents.

The training loop calls ``begin()``, ``after_step(ctx)`` every execution and
``end(ctx)``; ``ctx`` exposes the global step, the interval metrics and the
model.  Built-in hooks reproduce what the reference's RunConfig turns on:
  * StepCounterHook    — ``global_step/sec`` every log_step_count_steps (MKD:247)
  * LoggingHook        — ``loss = X, step = N`` log lines (Estimator default)
  * SummarySaverHook   — TensorBoard scalars every save_summary_steps (MKD:246)
  * CheckpointSaverHook— chief-only checkpoints every N steps/secs (MKD:248)
  * ProfilerHook       — Chrome-trace timelines every save_steps (MKD:235-237)
"""
from __future__ import annotations

import json
import logging
import os
import time
from pathlib import Path

log = logging.getLogger("tensorflow_distributed_example_amd")


class SessionRunHook:
    def begin(self, ctx):
        pass

    def after_step(self, ctx):
        pass

    def end(self, ctx):
        pass


def _crossed(prev, cur, every):
    return every and every > 0 and (cur // every) > (prev // every)


class StepCounterHook(SessionRunHook):
    def __init__(self, every_n_steps=100, writer=None):
        self.every = every_n_steps
        self.writer = writer
        self._t = None
        self._s = 0

    def begin(self, ctx):
        self._t, self._s = time.perf_counter(), ctx.global_step

    def after_step(self, ctx):
        if _crossed(ctx.prev_step, ctx.global_step, self.every):
            now = time.perf_counter()
            rate = (ctx.global_step - self._s) / max(now - self._t, 1e-9)
            ctx.last_steps_per_sec = rate
            log.info("global_step/sec: %g", rate)
            if self.writer is not None:
                self.writer.add_scalars(ctx.global_step, {"global_step/sec": rate})
            self._t, self._s = now, ctx.global_step


class LoggingHook(SessionRunHook):
    def __init__(self, every_n_steps=100):
        self.every = every_n_steps

    def after_step(self, ctx):
        if _crossed(ctx.prev_step, ctx.global_step, self.every) or ctx.prev_step == ctx.start_step:
            m = ctx.interval_metrics()
            log.info("loss = %g, step = %d", m.get("loss", float("nan")), ctx.global_step)


class SummarySaverHook(SessionRunHook):
    def __init__(self, every_n_steps=100, writer=None):
        self.every = every_n_steps
        self.writer = writer

    def after_step(self, ctx):
        if self.writer is not None and _crossed(ctx.prev_step, ctx.global_step, self.every):
            m = ctx.interval_metrics(reset=True)
            self.writer.add_scalars(ctx.global_step, {k: v for k, v in m.items()})
            self.writer.flush()

    def end(self, ctx):
        if self.writer is not None:
            self.writer.flush()


class CheckpointSaverHook(SessionRunHook):
    def __init__(self, manager, save_steps=None, save_secs=None, saver_fn=None):
        self.manager = manager
        self.save_steps = save_steps
        self.save_secs = save_secs
        self.saver_fn = saver_fn
        self._last_t = time.time()
        self.saved = []
        self.listeners = []

    def _save(self, ctx):
        path = self.saver_fn(ctx.global_step) if self.saver_fn else self.manager.save(ctx.model, ctx.global_step)
        self.saved.append(ctx.global_step)
        self._last_t = time.time()
        log.info("Saving checkpoints for %d into %s.", ctx.global_step, path)
        for fn in self.listeners:
            fn(ctx, path)

    def begin(self, ctx):
        if ctx.manager_latest is None:   # Estimator saves step 0 at session creation
            self._save(ctx)

    def after_step(self, ctx):
        due = _crossed(ctx.prev_step, ctx.global_step, self.save_steps)
        if not due and self.save_secs and time.time() - self._last_t >= self.save_secs:
            due = True
        if due:
            self._save(ctx)

    def end(self, ctx):
        if not self.saved or self.saved[-1] != ctx.global_step:
            self._save(ctx)


class ProfilerHook(SessionRunHook):
    """tf.estimator.ProfilerHook(save_steps, output_dir, show_memory): every
    ``save_steps`` steps, profile ONE step with torch.profiler (ROCm activity via
    roctracer) and write ``timeline-<step>.json`` (Chrome trace format)."""

    def __init__(self, save_steps=None, save_secs=None, output_dir="", show_dataflow=True, show_memory=False):
        self.save_steps = save_steps or 100
        self.output_dir = Path(output_dir or ".")
        self.show_memory = show_memory
        self._prof = None
        self.written = []

    def before_step(self, ctx, next_step):
        if self._prof is None and (next_step % self.save_steps == 0 or next_step == 1):
            import torch
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self._prof = torch.profiler.profile(activities=acts, profile_memory=self.show_memory)
            self._prof.__enter__()

    def after_step(self, ctx):
        if self._prof is not None:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            self._prof.__exit__(None, None, None)
            self.output_dir.mkdir(parents=True, exist_ok=True)
            path = self.output_dir / f"timeline-{ctx.global_step}.json"
            try:
                self._prof.export_chrome_trace(str(path))
            except Exception as e:  # profiler export may fail without events; keep a stub trace
                path.write_text(json.dumps({"traceEvents": [], "error": str(e)}))
            self.written.append(str(path))
            self._prof = None
