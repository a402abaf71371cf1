"""Cluster configuration: ``TF_CONFIG`` parsing, launcher-env translation,
session device filters and role resolution.

* ``TF_CONFIG`` = ``{"cluster": {job: ["host:port", ...]}, "task": {"type", "index"}}``
  (read by MWMS at construction — distributed_with_keras.py:16 — and by the PS
  strategy — tf2_mnist_distributed.py:189).
* ``translate_launcher_env()`` builds TF_CONFIG from ``CLUSTER_SPEC`` /
  ``TASK_INDEX`` / ``JOB_NAME`` exactly like mnist_keras_distributed.py:221-233.
* ``device_filters()`` reproduces ``_get_session_config_from_env_var``
  (mnist_keras_distributed.py:165-189): master talks to ps+master, worker i to
  ps+itself; our PS client only connects to the tasks the filter allows.
* torchrun-style env (RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT/LOCAL_RANK) is
  accepted as an equivalent worker-only cluster description.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass

ROLES = ("chief", "master", "worker", "ps", "evaluator")


class ClusterSpec:
    def __init__(self, cluster: dict | None = None):
        self._jobs = {k: list(v) if not isinstance(v, dict) else [v[i] for i in sorted(v)]
                      for k, v in (cluster or {}).items()}

    def as_dict(self):
        return {k: list(v) for k, v in self._jobs.items()}

    @property
    def jobs(self):
        return list(self._jobs)

    def job_tasks(self, job):
        return list(self._jobs.get(job, []))

    def num_tasks(self, job):
        return len(self._jobs.get(job, []))

    def task_address(self, job, index):
        return self._jobs[job][index]

    def __bool__(self):
        return bool(self._jobs)

    def __eq__(self, other):
        return isinstance(other, ClusterSpec) and self.as_dict() == other.as_dict()

    def __repr__(self):
        return f"ClusterSpec({self.as_dict()})"


@dataclass
class TaskInfo:
    type: str | None
    index: int


def tf_config(env=None) -> dict:
    env = os.environ if env is None else env
    raw = env.get("TF_CONFIG", "")
    if not raw:
        return {}
    cfg = json.loads(raw)
    if not isinstance(cfg, dict):
        raise ValueError("TF_CONFIG must be a JSON object")
    return cfg


def translate_launcher_env(env=None, verbose=True) -> bool:
    """CLUSTER_SPEC/TASK_INDEX/JOB_NAME -> TF_CONFIG (mnist_keras_distributed.py:221-233).

    Returns True if distribution got enabled.  Unlike the reference (quirk Q1), a
    missing CLUSTER_SPEC leaves a well-defined local task (chief, index 0)."""
    env = os.environ if env is None else env
    spec = env.get("CLUSTER_SPEC")
    if spec:
        cluster = json.loads(spec)
        job_index = int(env["TASK_INDEX"])
        job_type = env["JOB_NAME"]
        env["TF_CONFIG"] = json.dumps({"cluster": cluster, "task": {"type": job_type, "index": job_index}})
        if verbose:
            print("Distribution enabled: ", env["TF_CONFIG"])
        return True
    if verbose:
        print("Distribution is not enabled")
    return False


class TFConfigClusterResolver:
    """Equivalent of tf.distribute.cluster_resolver.TFConfigClusterResolver."""

    def __init__(self, env=None):
        cfg = tf_config(env)
        self._cfg = cfg
        self._spec = ClusterSpec(cfg.get("cluster", {}))
        task = cfg.get("task", {})
        self.task_type = task.get("type")
        self.task_id = int(task.get("index", 0)) if task else 0
        self.rpc_layer = cfg.get("rpc_layer", "grpc")

    def cluster_spec(self) -> ClusterSpec:
        return self._spec

    @property
    def is_distributed(self):
        return bool(self._spec)

    def master(self):
        for job in ("chief", "master", "worker"):
            if self._spec.num_tasks(job):
                return self._spec.task_address(job, 0)
        return ""

    def num_accelerators(self):
        import torch
        return {"GPU": torch.cuda.device_count()}


def device_filters(env=None):
    """Session device filters of mnist_keras_distributed.py:176-189 (None if undefined)."""
    cfg = tf_config(env)
    task = cfg.get("task") if cfg else None
    if task and "type" in task and "index" in task:
        if task["type"] == "master":
            return ["/job:ps", "/job:master"]
        if task["type"] == "worker":
            return ["/job:ps", "/job:worker/task:%d" % task["index"]]
    return None


def filter_allows(filters, job, index) -> bool:
    if filters is None:
        return True
    for f in filters:
        parts = dict(p.split(":", 1) for p in f.strip("/").split("/") if ":" in p)
        if parts.get("job") != job:
            continue
        if "task" not in parts or int(parts["task"]) == index:
            return True
    return False


@dataclass
class WorkerTopology:
    rank: int
    world: int
    master_addr: str
    master_port: int
    local_rank: int
    source: str  # "tf_config" | "torchrun" | "local"


def worker_topology(env=None) -> WorkerTopology:
    """Rank/world of this process among the synchronous (MWMS) workers."""
    env = os.environ if env is None else env
    cfg = tf_config(env)
    if cfg.get("cluster"):
        spec = ClusterSpec(cfg["cluster"])
        task = cfg.get("task", {})
        ttype, tidx = task.get("type", "worker"), int(task.get("index", 0))
        # MWMS workers: chief (if any) first, then workers.
        members = [("chief", i) for i in range(spec.num_tasks("chief"))] + \
                  [("worker", i) for i in range(spec.num_tasks("worker"))]
        if (ttype, tidx) not in members:
            raise ValueError(f"task {ttype}:{tidx} is not a MultiWorkerMirroredStrategy worker")
        rank = members.index((ttype, tidx))
        host, port = spec.task_address(*members[0]).rsplit(":", 1)
        local = int(env.get("LOCAL_RANK", rank if host in ("localhost", "127.0.0.1") else 0))
        return WorkerTopology(rank, len(members), host, int(port), local, "tf_config")
    if "WORLD_SIZE" in env and "RANK" in env:
        return WorkerTopology(int(env["RANK"]), int(env["WORLD_SIZE"]), env.get("MASTER_ADDR", "127.0.0.1"),
                              int(env.get("MASTER_PORT", "29500")), int(env.get("LOCAL_RANK", "0")), "torchrun")
    return WorkerTopology(0, 1, "127.0.0.1", 0, int(env.get("LOCAL_RANK", "0")), "local")


def is_chief(env=None) -> bool:
    cfg = tf_config(env)
    task = cfg.get("task") if cfg else None
    if not task:
        return True
    spec = ClusterSpec(cfg.get("cluster", {}))
    if task.get("type") in ("chief", "master"):
        return True
    if task.get("type") == "worker" and task.get("index", 0) == 0 and not (spec.num_tasks("chief") or spec.num_tasks("master")):
        return True
    return False
