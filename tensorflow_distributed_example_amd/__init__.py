"""tensorflow_distributed_example_amd — an MI355X-native data-parallel training framework.

Keras/tf.distribute-shaped API over PyTorch-ROCm tensors, hand-written gfx950 HIP
kernels (csrc/kernels) and RCCL over xGMI (csrc/comm), with the capabilities of
lowc1012/tensorflow-distributed-example:

    import tensorflow_distributed_example_amd as tde
    strategy = tde.distribute.MultiWorkerMirroredStrategy()
    with strategy.scope():
        model = tde.keras.Sequential([...]); model.compile(...)
    model.fit(ds, epochs=3, steps_per_epoch=5)
"""
import torch  # noqa: F401  (first: our HIP library reuses torch's libamdhip64/librccl)

from . import backend  # noqa: F401
from . import data, losses, metrics, optimizers  # noqa: F401
from .models import layers as _layers
from .models import zoo  # noqa: F401
from .models.model import Model, Sequential  # noqa: F401
from . import parallel as distribute  # noqa: F401

__version__ = "0.1.0"


class _Namespace:
    def __init__(self, **kw):
        self.__dict__.update(kw)


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
)
