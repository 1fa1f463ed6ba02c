"""Compute ops: NHWC layers backed by gfx950 HIP kernels (GPU) or PyTorch (CPU)."""
