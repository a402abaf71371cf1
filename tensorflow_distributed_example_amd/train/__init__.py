"""Training runtime: flat parameter storage, per-replica plans, programs, fit loop, estimator."""
