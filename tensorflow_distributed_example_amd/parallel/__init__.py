"""Distribution: strategies, communicators (RCCL over xGMI), cluster config, parameter server."""
from .strategy import (CommunicationImplementation, CommunicationOptions, MirroredStrategy,  # noqa: F401
                       MultiWorkerMirroredStrategy, OneDeviceStrategy, ReduceOp, Strategy, experimental,
                       get_strategy, has_strategy)
from .ps import ParameterServerStrategy  # noqa: F401,E402
from .cluster import ClusterSpec, TFConfigClusterResolver  # noqa: F401,E402
cluster_resolver = type("cluster_resolver", (), {"TFConfigClusterResolver": TFConfigClusterResolver})
