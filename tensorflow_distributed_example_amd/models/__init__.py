"""Keras-style layers, Sequential model and the reference model zoo."""
from . import initializers, layers, zoo  # noqa: F401
from .model import Model, Sequential  # noqa: F401
