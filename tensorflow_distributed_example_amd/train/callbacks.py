"""Keras-style callbacks: History, ProgbarLogger, ModelCheckpoint, plus the
progress bar that prints ``ms/step`` / loss / accuracy (the only timing the
reference's DWK path reports — distributed_with_keras.py:63)."""
from __future__ import annotations

import sys
import time


class Callback:
    def __init__(self):
        self.model = None
        self.params = {}

    def set_model(self, model):
        self.model = model

    def set_params(self, params):
        self.params = params

    def on_train_begin(self, logs=None): pass
    def on_train_end(self, logs=None): pass
    def on_epoch_begin(self, epoch, logs=None): pass
    def on_epoch_end(self, epoch, logs=None): pass
    def on_train_batch_begin(self, batch, logs=None): pass
    def on_train_batch_end(self, batch, logs=None): pass
    def on_test_begin(self, logs=None): pass
    def on_test_end(self, logs=None): pass


class History(Callback):
    def on_train_begin(self, logs=None):
        self.epoch = []
        self.history = {}

    def on_epoch_end(self, epoch, logs=None):
        self.epoch.append(epoch)
        for k, v in (logs or {}).items():
            self.history.setdefault(k, []).append(v)


class Progbar:
    def __init__(self, target, width=30, verbose=1, stream=None):
        self.target = target
        self.width = width
        self.verbose = verbose
        self.stream = stream or sys.stdout
        self.start = time.perf_counter()
        self._last = 0.0

    def update(self, current, values=None, finalize=False):
        if not self.verbose:
            return
        now = time.perf_counter()
        if not finalize and now - self._last < 0.1:
            return
        self._last = now
        elapsed = now - self.start
        vals = " - ".join(f"{k}: {v:.4f}" for k, v in (values or {}).items())
        if self.target:
            frac = min(current / self.target, 1.0)
            bar = "=" * int(self.width * frac)
            if frac < 1:
                bar = bar[:-1] + ">" if bar else ">"
            bar = bar.ljust(self.width, ".")
            per = elapsed / max(current, 1)
            unit = f"{per * 1e3:.0f}ms/step" if per >= 1e-3 else f"{per * 1e6:.0f}us/step"
            line = f"{current}/{self.target} [{bar}] - {elapsed:.0f}s {unit}"
        else:
            line = f"{current} - {elapsed:.0f}s"
        if vals:
            line += " - " + vals
        end = "\n" if finalize or self.verbose == 2 else "\r"
        if self.verbose == 2 and not finalize:
            return
        self.stream.write(line + end)
        self.stream.flush()


class ProgbarLogger(Callback):
    def __init__(self, verbose=1):
        super().__init__()
        self.verbose = verbose
        self.bar = None

    def on_epoch_begin(self, epoch, logs=None):
        if self.verbose:
            print(f"Epoch {epoch + 1}/{self.params.get('epochs', '?')}")
        self.bar = Progbar(self.params.get("steps"), verbose=self.verbose)

    def on_train_batch_end(self, batch, logs=None):
        if self.bar:
            self.bar.update(batch + 1, logs)

    def on_epoch_end(self, epoch, logs=None):
        if self.bar:
            self.bar.update(self.params.get("steps") or self.params.get("seen", 0), logs, finalize=True)


class ModelCheckpoint(Callback):
    def __init__(self, filepath, save_weights_only=True, save_freq="epoch", **kw):
        super().__init__()
        self.filepath = filepath
        self.save_weights_only = save_weights_only

    def on_epoch_end(self, epoch, logs=None):
        path = self.filepath.format(epoch=epoch + 1, **(logs or {}))
        st = self.model._strategy
        if st is None or st.is_chief:
            self.model.save_weights(path)
        else:
            self.model.state_dict()              # take part in the SyncOnRead collective only


class BackupAndRestore(Callback):
    """``tf.keras.callbacks.BackupAndRestore``: fault-tolerant fit for MultiWorkerMirroredStrategy.

    The chief backs up weights, optimizer slots, the step counter and the finished epoch into
    ``backup_dir`` (TensorBundle, atomic state file) at the end of every epoch; when ``fit`` starts
    and a backup exists, every worker restores it and training resumes with the next epoch — the
    recovery half of the failure handling in SURVEY.md §5.3 (parallel/health.py detects the
    failure and stops the job).  The backup is deleted when training finishes."""

    def __init__(self, backup_dir, save_freq="epoch", delete_checkpoint=True):
        super().__init__()
        if save_freq != "epoch":
            raise ValueError("BackupAndRestore: only save_freq='epoch' is supported")
        self.backup_dir = backup_dir
        self.delete_checkpoint = delete_checkpoint

    def _mgr(self):
        from .checkpoint import CheckpointManager
        return CheckpointManager(self.backup_dir, max_to_keep=1, prefix="backup")

    def on_train_begin(self, logs=None):
        r = self._mgr().restore(self.model)
        if r is None:
            return
        step, extras = r
        self.model._set_iterations(step)
        self.model._resume_epoch = int(extras.get("epoch", -1)) + 1

    def on_epoch_end(self, epoch, logs=None):
        st = self.model._strategy
        state = self.model.state_dict()          # collective (SyncOnRead MEAN) on every worker
        if st is None or st.is_chief:
            self._mgr().save(self.model, self.model.optimizer.iterations, extra={"epoch": epoch}, state=state)

    def on_train_end(self, logs=None):
        st = self.model._strategy
        if self.delete_checkpoint and (st is None or st.is_chief):
            import shutil
            shutil.rmtree(self.backup_dir, ignore_errors=True)


class ProfilerCallback(Callback):
    """Keras-side counterpart of the Estimator ProfilerHook (MKD:235-237; TF's TensorBoard
    ``profile_batch``): every ``every_n_steps`` training steps (and the first), one step is recorded with
    torch.profiler (host + ROCm activity) into ``<log_dir>/timeline-<step>.json`` (Chrome trace)."""

    def __init__(self, log_dir, every_n_steps=100, show_memory=True):
        super().__init__()
        from .hooks import ProfilerHook
        self._hook = ProfilerHook(save_steps=every_n_steps, output_dir=log_dir, show_memory=show_memory)
        self._step = 0

    @property
    def written(self):
        return self._hook.written

    def on_train_batch_begin(self, batch, logs=None):
        self._first = batch
        self._hook.before_step(None, self._step + 1)

    def on_train_batch_end(self, batch, logs=None):
        # fit() calls begin / end once per execution (steps_per_execution steps): batch is the index of
        # the execution's last step, so the global step advances by the execution's length
        self._step += batch - getattr(self, "_first", batch) + 1

        class _Ctx:
            global_step = self._step
        self._hook.after_step(_Ctx)


class LambdaCallback(Callback):
    def __init__(self, on_epoch_end=None, on_train_batch_end=None, **kw):
        super().__init__()
        self._oee = on_epoch_end
        self._otbe = on_train_batch_end

    def on_epoch_end(self, epoch, logs=None):
        if self._oee:
            self._oee(epoch, logs)

    def on_train_batch_end(self, batch, logs=None):
        if self._otbe:
            self._otbe(batch, logs)


class CallbackList:
    def __init__(self, cbs, model, params):
        self.cbs = list(cbs)
        for c in self.cbs:
            c.set_model(model)
            c.set_params(params)

    def __getattr__(self, name):
        def f(*a, **k):
            for c in self.cbs:
                getattr(c, name)(*a, **k)
        return f
