"""Deterministic stand-in for ``torch.rand_like`` (test infrastructure).

The reference's training-mode drop-path draws ``torch.rand_like(updating, dtype=float32)``
once per iteration (``autograd_solvers/bfgs_solver.py:121-125``).  CPU and GPU generators
differ, so golden generation (reference, CPU) and the parity tests (product, GPU) both
replace it with draws from one seeded CPU generator, moved to the tensor's device.
"""
import torch


class deterministic_rand_like:
    """Stand-in for torch.rand_like: draws from a seeded CPU generator, then moves to the
    tensor's device, so the reference (CPU) and the product (GPU) see the same numbers."""

    def __init__(self, seed):
        self.gen = torch.Generator().manual_seed(seed)
        self.orig = torch.rand_like

    def __call__(self, t, dtype=None, **kw):
        return torch.rand(t.shape, generator=self.gen, dtype=dtype or torch.float32).to(t.device)

    def __enter__(self):
        torch.rand_like = self
        return self

    def __exit__(self, *exc):
        torch.rand_like = self.orig
