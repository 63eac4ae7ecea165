"""Walker/Vose alias tables (reference implementation for the HIP sampler).

The reference draws with ``torch.multinomial`` (`pytorch_collab.py:114`,
`util.py:150`).  The MI355X sampler (``csrc/importance.hip``) builds an alias
table in LDS for pools up to 16k entries and draws each sample in O(1) with a
counter-based Philox stream, so a draw costs one table lookup instead of a
prefix-sum search.  This module is the host reference used by tests: same
construction (Vose's stable small/large worklists), numpy in float64.
"""
from __future__ import annotations

import numpy as np


def build_alias(p):
    """Return ``(prob, alias)`` so that drawing ``i = U[0,n)`` then keeping ``i``
    with probability ``prob[i]`` else ``alias[i]`` samples from ``p``."""
    p = np.asarray(p, dtype=np.float64)
    n = p.size
    scaled = p * n / p.sum()
    prob = np.zeros(n)
    alias = np.arange(n)
    small = [i for i in range(n) if scaled[i] < 1.0]
    large = [i for i in range(n) if scaled[i] >= 1.0]
    while small and large:
        s = small.pop()
        g = large.pop()
        prob[s] = scaled[s]
        alias[s] = g
        scaled[g] = (scaled[g] + scaled[s]) - 1.0
        (small if scaled[g] < 1.0 else large).append(g)
    for i in large + small:
        prob[i] = 1.0
    return prob, alias


def alias_draw(prob, alias, u_bin, u_coin):
    """Vectorised draw from uniform variates ``u_bin, u_coin`` in [0,1)."""
    n = prob.size
    i = np.minimum((np.asarray(u_bin) * n).astype(np.int64), n - 1)
    return np.where(np.asarray(u_coin) < prob[i], i, alias[i])


def alias_distribution(prob, alias):
    """Exact distribution implied by a table (for testing)."""
    n = prob.size
    out = np.zeros(n)
    for i in range(n):
        out[i] += prob[i] / n
        out[alias[i]] += (1.0 - prob[i]) / n
    return out
