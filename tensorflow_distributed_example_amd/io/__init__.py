"""Persistence: checkpoints (TensorBundle), export, summaries."""
