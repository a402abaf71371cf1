"""Rank-prefixed logging and ``--verbosity`` handling (SURVEY.md F26;
mnist_keras_distributed.py:60-63,288-289, tf2_mnist_distributed.py:187)."""
from __future__ import annotations

import logging
import os
import sys

_NAME = "tensorflow_distributed_example_amd"
_LEVELS = {"DEBUG": logging.DEBUG, "INFO": logging.INFO, "WARN": logging.WARNING, "WARNING": logging.WARNING,
           "ERROR": logging.ERROR, "FATAL": logging.CRITICAL}


class _RankFilter(logging.Filter):
    def filter(self, record):
        record.rank = os.environ.get("RANK", os.environ.get("TASK_INDEX", "0"))
        return True


def get_logger():
    lg = logging.getLogger(_NAME)
    if not lg.handlers:
        h = logging.StreamHandler(sys.stderr)
        h.addFilter(_RankFilter())
        h.setFormatter(logging.Formatter("%(levelname)s:tde[r%(rank)s]:%(message)s"))
        lg.addHandler(h)
        lg.propagate = False
        lg.setLevel(logging.WARNING)
    return lg


def set_verbosity(level):
    lvl = _LEVELS[level.upper()] if isinstance(level, str) else int(level)
    get_logger().setLevel(lvl)
    return lvl
