"""Presample-pool importance sampling math (`pytorch_collab.py:89-117,132-145`).

Reference semantics, made explicit:

* the pool is ``n_batches`` (=10) loader batches of ``b`` (=32) samples;
* after *each* scored batch ``j`` the EMA is updated with the mean loss of the
  pool so far (``cat(losses[:j+1]).mean()``), i.e. 10 EMA updates per call
  (SURVEY F3);
* ``p_i = (l_i + alpha * ema) / sum_k(l_k + alpha * ema)``;
* the training batch is ``multinomial(p, b, replacement=True)``;
* the returned weights are ``p[idx] * N`` (N = pool size) and the training
  loss is ``mean(l_j / w_j)``, the unbiased estimator of the pool-mean loss.

Because every EMA update only depends on the cumulative means, scoring the
whole pool in ONE forward (ghost batch-norm per 32-sample group keeps the
per-batch BN statistics) and replaying the 10 updates afterwards gives
bit-for-bit the same EMA as the reference's 10 separate forwards.  That
replay is ``ema_replay``; the GPU path runs it inside the fused HIP scorer
kernel (``csrc/importance.hip``), this module is the torch reference
implementation and CPU path.
"""
from __future__ import annotations

import torch


def cumulative_means(losses, group):
    """Means of ``losses[:group*(j+1)]`` for every group boundary ``j``."""
    n = losses.numel()
    csum = torch.cumsum(losses.double(), 0)
    ends = torch.arange(group, n + 1, group, device=losses.device)
    return (csum[ends - 1] / ends.double()).to(losses.dtype)


def global_cumulative_means(gathered, group):
    """Cumulative pool means over every rank's pool: ``gathered`` is [W][P] (the score
    all-gather); the mean after batch ``j`` covers the first ``group*(j+1)`` samples of
    all W pools (the global-EMA mode; the fused kernel does the same on device)."""
    W, n = gathered.shape
    gs = gathered.double().reshape(W, n // group, group).sum((0, 2))
    ends = torch.arange(1, n // group + 1, device=gathered.device, dtype=torch.float64)
    return (torch.cumsum(gs, 0) / (ends * group * W)).to(gathered.dtype)


def classifier_gradnorm(logits, labels, feats):
    """Exact per-sample gradient norm of the classifier layer ``z = W h + b`` under CE:
    ``||softmax(z) - onehot(y)|| * sqrt(||h||^2 + 1)`` (an importance score that upper-bounds
    the full gradient norm up to a constant; Katharopoulos & Fleuret 2018).  Works for
    log-softmax outputs too (softmax is shift invariant)."""
    d = torch.softmax(logits.float(), 1)
    d[torch.arange(d.shape[0], device=d.device), labels] -= 1.0
    h2 = feats.float().reshape(feats.shape[0], -1).pow(2).sum(1)
    return d.norm(dim=1) * torch.sqrt(h2 + 1.0)


def ema_replay(ema, means):
    """Apply ``EMAverage.update`` for each cumulative mean in order (`util.py:207-213`).

    ``ema`` is a meter object (``first_update``/``value``/``alpha``)."""
    for m in means:
        ema.update(m)
    return ema


def importance_probs(losses, ema_value, alpha=0.5):
    """``(l + alpha*ema) / sum`` (`pytorch_collab.py:111-112`)."""
    shifted = losses + alpha * ema_value
    return shifted / shifted.sum()


def draw(probs, k, generator=None):
    """Weighted draw with replacement (`pytorch_collab.py:114`)."""
    return torch.multinomial(probs, k, replacement=True, generator=generator)


def is_weights(probs, idx):
    """Per-drawn-sample weights ``N * p_idx`` (`pytorch_collab.py:116`)."""
    return probs[idx] * probs.numel()


def weighted_loss(per_sample_losses, weights):
    """Unbiased IS estimator ``mean(l / w)`` (`pytorch_collab.py:137,145`)."""
    return torch.mean(per_sample_losses / weights)


def score_and_sample(losses, ema, alpha, batch_size, group, generator=None):
    """Full reference pipeline on an already-scored pool.

    Returns ``(weights, idx, pool_mean)``; mutates ``ema``."""
    ema_replay(ema, cumulative_means(losses, group))
    p = importance_probs(losses, ema.value, alpha)
    idx = draw(p, batch_size, generator)
    return is_weights(p, idx), idx, losses.mean()
