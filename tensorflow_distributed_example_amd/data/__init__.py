"""tf.data-like input pipeline and dataset loaders."""
from .dataset import AUTOTUNE, AutoShardPolicy, Dataset, Options, experimental  # noqa: F401
from .distributed import DistributedDataset  # noqa: F401
from . import mnist  # noqa: F401
