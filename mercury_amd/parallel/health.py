"""Replica-divergence detection for synchronous DP.

Synchronous data parallelism keeps every replica bit-identical: same initial
weights (broadcast), same averaged gradient, same optimizer.  A rank that
silently diverges -- a missed bucket, a race between the scoring stream and the
optimizer, a flaky link corrupting a message -- produces a model nobody trained.
The reference would never notice (it never compares replicas).

``replica_fingerprint`` reduces a flat parameter buffer to a tiny fp64 vector
(sum, sum of squares, and a position-weighted sum that catches permutations);
``check_replicas`` all-reduces MIN and MAX of that vector (two 24-byte
collectives) and reports the worst relative spread.  Cheap enough to run every
few hundred steps (``Config.check_replicas_every``).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def replica_fingerprint(flat):
    f = flat.detach().reshape(-1).double()
    w = torch.linspace(1.0, 2.0, f.numel(), device=f.device, dtype=torch.float64)
    return torch.stack([f.sum(), (f * f).sum(), (f * w).sum()])


def check_replicas(flat, group=None, rtol=0.0):
    """Returns ``(ok, spread)``: spread = max relative (max - min) over the fingerprint entries
    across ranks; ``ok`` iff spread <= rtol (0: bit-identical replicas expected)."""
    fp = replica_fingerprint(flat)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return True, 0.0
    lo, hi = fp.clone(), fp.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    spread = float(((hi - lo).abs() / hi.abs().clamp_min(1e-30)).max())
    return spread <= rtol, spread


class ReplicaDivergence(RuntimeError):
    pass
