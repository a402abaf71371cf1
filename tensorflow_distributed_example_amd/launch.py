"""Localhost cluster launcher (SURVEY.md F11, §4.1 "multi-node without a real cluster").

    python -m tensorflow_distributed_example_amd.launch --workers 2 script.py [args]
    python -m tensorflow_distributed_example_amd.launch --ps 1 --master 1 --workers 1 --evaluator 1 script.py ...
    python -m tensorflow_distributed_example_amd.launch --workers 2 --gpus-per-worker 4 script.py   # MWMS 2x4

Spawns one process per task with ``TF_CONFIG`` (or, with ``--launcher-env``, the
``CLUSTER_SPEC``/``TASK_INDEX``/``JOB_NAME`` variables of mnist_keras_distributed.py
:221-225), picks free 127.0.0.1 ports, assigns GPUs (``LOCAL_RANK`` /
``TDE_GPUS_PER_WORKER``), prefixes output lines with the task name, and tears
the cluster down when the training tasks finish or one of them fails (ps tasks
block forever, like TF's server.join()).  Fault injection for tests:
``TDE_FAULT="task=worker:1,step=7,kind=exit"`` is forwarded to every task.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def build_cluster(ps=0, chief=0, master=0, workers=1, evaluator=0):
    c = {}
    for job, n in (("chief", chief), ("master", master), ("worker", workers), ("ps", ps)):
        if n:
            c[job] = [f"127.0.0.1:{free_port()}" for _ in range(n)]
    return c


def _pump(prefix, stream, out):
    for line in iter(stream.readline, ""):
        out.write(f"[{prefix}] {line}")
        out.flush()


def launch(script_args, ps=0, chief=0, master=0, workers=1, evaluator=0, gpus_per_worker=None,
           launcher_env=False, timeout=None, env_extra=None, out=None):
    out = out or sys.stdout
    cluster = build_cluster(ps, chief, master, workers, evaluator)
    tasks = [(job, i) for job in ("ps", "chief", "master", "worker") for i in range(len(cluster.get(job, [])))]
    tasks += [("evaluator", i) for i in range(evaluator)]
    procs = {}
    gpu_slot = 0
    for job, i in tasks:
        env = dict(os.environ, **(env_extra or {}))
        env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
        task = {"type": job, "index": i}
        if launcher_env:
            spec = {k: v for k, v in cluster.items()}
            env["CLUSTER_SPEC"] = json.dumps(spec)
            env["TASK_INDEX"] = str(i)
            env["JOB_NAME"] = job
            env.pop("TF_CONFIG", None)
        else:
            env["TF_CONFIG"] = json.dumps({"cluster": cluster, "task": task})
        if job in ("chief", "master", "worker"):
            env["LOCAL_RANK"] = str(gpu_slot)
            if gpus_per_worker:
                env["TDE_GPUS_PER_WORKER"] = str(gpus_per_worker)
            gpu_slot += 1
        else:
            env["LOCAL_RANK"] = "0"
        p = subprocess.Popen([sys.executable, *script_args], env=env, stdout=subprocess.PIPE,
                             stderr=subprocess.STDOUT, text=True, start_new_session=True)
        threading.Thread(target=_pump, args=(f"{job}:{i}", p.stdout, out), daemon=True).start()
        procs[(job, i)] = p
    trainers = [k for k in procs if k[0] != "ps"]
    t0 = time.time()
    rc = 0
    try:
        while True:
            done = {k: procs[k].poll() for k in trainers}
            failed = [k for k, v in done.items() if v not in (None, 0)]
            if failed:
                rc = procs[failed[0]].returncode
                out.write(f"[launch] task {failed[0][0]}:{failed[0][1]} failed with {rc}; stopping the cluster\n")
                break
            if all(v is not None for v in done.values()):
                break
            if timeout and time.time() - t0 > timeout:
                rc = 124
                out.write("[launch] timeout\n")
                break
            time.sleep(0.1)
    finally:
        for k, p in procs.items():
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        for p in procs.values():
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
    return rc, cluster


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--ps", type=int, default=0)
    ap.add_argument("--chief", type=int, default=0)
    ap.add_argument("--master", type=int, default=0)
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--evaluator", type=int, default=0)
    ap.add_argument("--gpus-per-worker", type=int, default=None)
    ap.add_argument("--launcher-env", action="store_true", help="use CLUSTER_SPEC/TASK_INDEX/JOB_NAME instead of TF_CONFIG")
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("script", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    if not a.script:
        ap.error("missing script")
    rc, _ = launch(a.script, a.ps, a.chief, a.master, a.workers, a.evaluator, a.gpus_per_worker, a.launcher_env,
                   a.timeout)
    return rc


if __name__ == "__main__":
    sys.exit(main())
