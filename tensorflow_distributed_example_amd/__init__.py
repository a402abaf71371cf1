"""tensorflow_distributed_example_amd — an MI355X-native data-parallel training framework.

Keras / tf.distribute / tf.estimator-shaped API over PyTorch-ROCm tensors,
hand-written gfx950 HIP kernels (csrc/kernels) and RCCL over xGMI (csrc/comm),
with the capabilities of lowc1012/tensorflow-distributed-example:

    import tensorflow_distributed_example_amd as tde
    strategy = tde.distribute.MultiWorkerMirroredStrategy()
    with strategy.scope():
        model = tde.keras.Sequential([...]); model.compile(...)
    model.fit(ds, epochs=3, steps_per_epoch=5)

    est = tde.keras.estimator.model_to_estimator(keras_model=model, model_dir=D, config=run_config)
    tde.estimator.train_and_evaluate(est, train_spec, eval_spec)
"""
import os as _os

if _os.environ.get("TDE_DEBUG_SYNC", "0") not in ("", "0"):   # before any HIP call (utils/debug.py)
    _os.environ.setdefault("AMD_SERIALIZE_KERNEL", "3")
    _os.environ.setdefault("HIP_LAUNCH_BLOCKING", "1")
    _os.environ["TDE_GRAPH"] = "0"

import torch  # noqa: F401,E402  (first: our HIP library reuses torch's libamdhip64/librccl)

from . import backend  # noqa: F401
from . import data, losses, metrics, optimizers  # noqa: F401
from .data import tfds  # noqa: F401
from .io import export as _export
from .models import layers as _layers
from .models import zoo  # noqa: F401
from .models.model import Model, Sequential  # noqa: F401
from . import parallel as distribute  # noqa: F401
from .parallel import cluster as _cluster
from .train import estimator as _estimator
from .train import callbacks as _callbacks
from .train import hooks as _hooks
from .utils import logging as _logging
from .utils.tensorboard import start_tensorboard  # noqa: F401

__version__ = "0.1.0"

float32 = "float32"
int32 = "int32"
int64 = "int64"
bfloat16 = "bfloat16"


class _Namespace:
    def __init__(self, **kw):
        self.__dict__.update(kw)

    def __repr__(self):
        return f"<namespace {sorted(self.__dict__)}>"


def get_logger():
    return _logging.get_logger()


class _MixedPrecision:
    @staticmethod
    def set_global_policy(name):
        backend.set_global_policy(name)

    @staticmethod
    def global_policy():
        return backend.global_policy()

    Policy = backend.Policy


def _load_mnist(path=None):
    return data.mnist.load_data(path)


def _ps_strategy(*a, **k):
    from .parallel.ps import ParameterServerStrategy
    return ParameterServerStrategy(*a, **k)


estimator = _Namespace(
    Estimator=_estimator.Estimator, EstimatorSpec=_estimator.EstimatorSpec, ModeKeys=_estimator.ModeKeys,
    RunConfig=_estimator.RunConfig, TrainSpec=_estimator.TrainSpec, EvalSpec=_estimator.EvalSpec,
    FinalExporter=_estimator.FinalExporter, LatestExporter=_estimator.LatestExporter,
    train_and_evaluate=_estimator.train_and_evaluate, DistributeConfig=_estimator.DistributeConfig,
    SessionRunHook=_hooks.SessionRunHook, ProfilerHook=_hooks.ProfilerHook,
    export=_Namespace(TensorServingInputReceiver=_export.TensorServingInputReceiver,
                      ServingInputReceiver=_export.ServingInputReceiver),
)

keras = _Namespace(
    Sequential=Sequential,
    Model=Model,
    layers=_layers,
    losses=losses,
    optimizers=optimizers,
    metrics=metrics,
    backend=backend,
    mixed_precision=_MixedPrecision(),
    datasets=_Namespace(mnist=_Namespace(load_data=_load_mnist)),
    estimator=_Namespace(model_to_estimator=_estimator.model_to_estimator),
    callbacks=_callbacks,
    # (ReplicaConsistencyCheck lives in utils.debug; exposed below)
    Input=_layers.Input,
)

# tf.train.* names live on the real `train` subpackage (keeps `import ...train.estimator` working)
from . import train  # noqa: E402
from .io import tensor_bundle as _tb  # noqa: E402

train.GradientDescentOptimizer = optimizers.GradientDescentOptimizer
train.latest_checkpoint = _tb.latest_checkpoint
train.ClusterSpec = _cluster.ClusterSpec

compat = _Namespace(v1=_Namespace(placeholder=_export.placeholder, ConfigProto=_estimator.SessionConfig,
                                  logging=_Namespace(set_verbosity=_logging.set_verbosity)),
                    v2=_Namespace(optimizers=optimizers))

contrib = _Namespace(distribute=_Namespace(DistributeConfig=_estimator.DistributeConfig,
                                           MirroredStrategy=distribute.MirroredStrategy,
                                           ParameterServerStrategy=_ps_strategy))

saved_model = _Namespace(load=_export.load)
ConfigProto = _estimator.SessionConfig

from .utils import debug  # noqa: E402

_callbacks.ReplicaConsistencyCheck = debug.ReplicaConsistencyCheck
from . import utils  # noqa: E402
from .utils import flags as _flags  # noqa: E402,F401  (tde.utils.flags: the examples' framework flags)
