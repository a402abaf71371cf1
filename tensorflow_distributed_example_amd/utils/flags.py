"""Framework command-line flags shared by the example scripts.

The reference scripts keep their own flags (``mnist_keras_distributed.py:33-65``); these are the
framework additions every example accepts on top of them:

    --devices cpu | gpu:0,gpu:1 | cuda:0   replicas a strategy built without devices uses
    --dtype fp32 | bf16                    compute policy: float32 (default; the reference's precision,
                                           exact-f32 MFMA kernel forms) / mixed_bfloat16 (bf16 MFMA)
    --synthetic                            synthetic MNIST even when a local mnist.npz exists
    --profile-steps N                      Chrome-trace timeline of one step every N steps
                                           (Estimator ProfilerHook, MKD:235-237; Keras ProfilerCallback)
"""
from __future__ import annotations

import os

from .. import backend as Kb

DTYPES = {"fp32": "float32", "bf16": "mixed_bfloat16"}


def add_framework_flags(parser):
    g = parser.add_argument_group("framework flags (SURVEY.md §5.6)")
    g.add_argument("--devices", default=None,
                   help="comma-separated replica devices (cpu, gpu:N, cuda:N); default: every local GPU, else CPU")
    g.add_argument("--dtype", choices=sorted(DTYPES), default=None,
                   help="compute dtype: fp32 (float32, the default and the reference's precision: exact-f32 "
                        "MFMA kernels) or bf16 (mixed_bfloat16: bf16 MFMA kernels, fp32 master weights)")
    g.add_argument("--synthetic", action="store_true", help="use synthetic MNIST even if a local mnist.npz exists")
    g.add_argument("--profile-steps", type=int, default=0,
                   help="write a Chrome-trace timeline of one step every N steps (0: off)")
    return parser


def apply_framework_flags(args):
    """Apply the parsed flags to the global framework state (before any strategy is built)."""
    devices = getattr(args, "devices", None)
    if devices:
        Kb.set_default_devices(devices.split(","))
    dtype = getattr(args, "dtype", None)
    if dtype:
        # the GPU plans pick their kernel form from the policy (train/program.py make_plan)
        Kb.set_global_policy(DTYPES[dtype])
    if getattr(args, "synthetic", False):
        os.environ["TDE_SYNTHETIC_MNIST"] = "1"
    return args


def profiler_hooks(args, output_dir):
    """Estimator hooks for ``--profile-steps`` (the reference's commented ProfilerHook, MKD:235-237)."""
    n = int(getattr(args, "profile_steps", 0) or 0)
    if n <= 0:
        return []
    from ..train.hooks import ProfilerHook
    return [ProfilerHook(save_steps=n, output_dir=output_dir, show_memory=True)]


def profiler_callbacks(args, output_dir):
    """Keras callbacks for ``--profile-steps``."""
    n = int(getattr(args, "profile_steps", 0) or 0)
    if n <= 0:
        return []
    from ..train.callbacks import ProfilerCallback
    return [ProfilerCallback(output_dir, every_n_steps=n)]
