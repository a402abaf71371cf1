"""Distribution: strategies, communicators (RCCL over xGMI), cluster config, parameter server."""
from .strategy import (CommunicationImplementation, CommunicationOptions, MirroredStrategy,  # noqa: F401
                       MultiWorkerMirroredStrategy, OneDeviceStrategy, ReduceOp, Strategy, experimental,
                       get_strategy, has_strategy)
