"""Logging, profiling, TensorBoard helpers."""
