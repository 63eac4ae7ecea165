"""Stochastic magnitude quantisation (`util.py:65-70`).

``q = sign(a) * max|a| * Bernoulli(|a| / max|a|)`` -- unbiased (E[q] = a),
TernGrad-like.  Unused on the reference's main path (gradient-compression
leftover); kept as an optional gradient-compression hook.  On GPU the fused
HIP kernel ``mercury_amd.ops.quantize`` does abs-max + Philox Bernoulli in two
launches; this torch version is the CPU path and test oracle.
"""
from __future__ import annotations

import torch


def quantize_tensor(a, generator=None):
    sign = torch.sign(a)
    abs_a = torch.abs(a)
    max_a = torch.max(abs_a)
    if float(max_a) == 0.0:
        return torch.zeros_like(a)
    u = torch.rand(a.shape, generator=generator, device=a.device, dtype=torch.float32)
    sampled = (u < (abs_a / max_a)).to(a.dtype)
    return sign * max_a * sampled
