"""Python entry points to the gfx950 HIP kernels (ops.kernels) and torch references."""
