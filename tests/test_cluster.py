"""T2: cluster config — TF_CONFIG parsing, CLUSTER_SPEC translation (Q1), device filters."""
import json

import pytest

from tensorflow_distributed_example_amd.parallel import cluster as CL


def test_translate_launcher_env():
    env = {"CLUSTER_SPEC": json.dumps({"ps": ["h:1"], "master": ["h:2"], "worker": ["h:3", "h:4"]}),
           "TASK_INDEX": "1", "JOB_NAME": "worker"}
    assert CL.translate_launcher_env(env, verbose=False)
    cfg = json.loads(env["TF_CONFIG"])
    assert cfg == {"cluster": {"ps": ["h:1"], "master": ["h:2"], "worker": ["h:3", "h:4"]},
                   "task": {"type": "worker", "index": 1}}
    env2 = {}
    assert not CL.translate_launcher_env(env2, verbose=False)
    assert "TF_CONFIG" not in env2


def test_device_filters_match_reference():
    mk = lambda t, i: {"TF_CONFIG": json.dumps({"cluster": {}, "task": {"type": t, "index": i}})}  # noqa: E731
    assert CL.device_filters(mk("master", 0)) == ["/job:ps", "/job:master"]
    assert CL.device_filters(mk("worker", 3)) == ["/job:ps", "/job:worker/task:3"]
    assert CL.device_filters(mk("ps", 0)) is None
    assert CL.device_filters({}) is None
    f = CL.device_filters(mk("worker", 3))
    assert CL.filter_allows(f, "ps", 1) and CL.filter_allows(f, "worker", 3)
    assert not CL.filter_allows(f, "worker", 2) and not CL.filter_allows(f, "master", 0)


def test_worker_topology_from_tf_config():
    env = {"TF_CONFIG": json.dumps({"cluster": {"worker": ["localhost:12345", "localhost:23456"]},
                                    "task": {"type": "worker", "index": 1}})}
    t = CL.worker_topology(env)
    assert (t.rank, t.world, t.master_addr, t.master_port) == (1, 2, "localhost", 12345)
    env = {"TF_CONFIG": json.dumps({"cluster": {"chief": ["a:1"], "worker": ["b:2"]},
                                    "task": {"type": "worker", "index": 0}})}
    t = CL.worker_topology(env)
    assert (t.rank, t.world) == (1, 2)
    with pytest.raises(ValueError):
        CL.worker_topology({"TF_CONFIG": json.dumps({"cluster": {"ps": ["a:1"], "worker": ["b:2"]},
                                                     "task": {"type": "ps", "index": 0}})})


def test_worker_topology_torchrun_and_local():
    t = CL.worker_topology({"RANK": "3", "WORLD_SIZE": "8", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "999",
                            "LOCAL_RANK": "3"})
    assert (t.rank, t.world, t.master_port, t.local_rank, t.source) == (3, 8, 999, 3, "torchrun")
    t = CL.worker_topology({})
    assert (t.rank, t.world, t.source) == (0, 1, "local")


def test_cluster_resolver_and_chief():
    env = {"TF_CONFIG": json.dumps({"cluster": {"master": ["m:1"], "worker": ["w:1"], "ps": ["p:1"]},
                                    "task": {"type": "master", "index": 0}})}
    r = CL.TFConfigClusterResolver(env)
    assert r.task_type == "master" and r.task_id == 0
    assert r.cluster_spec().num_tasks("ps") == 1
    assert r.master() == "m:1"
    assert CL.is_chief(env)
    env_w = {"TF_CONFIG": json.dumps({"cluster": {"master": ["m:1"], "worker": ["w:1"]},
                                      "task": {"type": "worker", "index": 0}})}
    assert not CL.is_chief(env_w)
    assert CL.is_chief({})
