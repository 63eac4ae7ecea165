"""Importance-sampling kernels front-end (``csrc/importance.hip``)."""
from __future__ import annotations

import torch

from . import _chk, lib, ptr, stream_ptr
from ..data.transforms import CIFAR_MEAN, CIFAR_STD


def pool_build(shard, labels, ctrl, pool, pool_label, pool_index, P, batch, seed, pad=4,
               flip=True, augment=True, mean=CIFAR_MEAN, std=CIFAR_STD, shuffle=True, zero=None):
    """Build a P-sample presample pool on device from either the uint8 image shard
    [Ns][H][W][3] (crop/flip/normalise on the fly) or a pre-converted bf16 shard
    [Ns][H][W][8] (non-image inputs: plain gather, no augmentation).  ``zero``: an fp32
    buffer the same launch zeroes (the scoring pass's BN-statistics arena)."""
    _chk(labels, torch.int64, 'labels')
    prebuilt = shard.dtype == torch.bfloat16
    if not prebuilt:
        _chk(shard, torch.uint8, 'shard')
    elif shard.shape[-1] != 8:
        raise ValueError('pre-converted shard must be NHWC bf16 with 8 channels')
    Ns, H, W, _ = shard.shape
    _chk(pool, torch.bfloat16, 'pool', P * H * W * 8)
    lib().pool_build(ptr(shard), ptr(labels), ptr(ctrl), ptr(pool), ptr(pool_label),
                     ptr(pool_index), Ns, H, W, P, batch, pad, int(flip), int(augment), int(shuffle),
                     int(seed) & 0xffffffff, list(mean), [1.0 / s for s in std], stream_ptr(),
                     int(prebuilt), ptr(zero), zero.numel() if zero is not None else 0)


def is_sample(losses, ema, ctrl, idx, w, P, B, group, alpha=0.5, ema_alpha=0.9, seed=0,
              importance=True, meters=None, alias=True, gathered=None):
    """EMA replay + probabilities + B draws with replacement.  ``alias=True``: Walker alias
    table built in LDS and O(1) draws; ``alias=False``: inverse-CDF (prefix scan + search).
    ``gathered`` ([W][P] every rank's scores): the EMA is replayed over the global pool means
    (shared normaliser across ranks) while the draw still uses this rank's ``losses``."""
    _chk(losses, torch.float32, 'losses', P)
    _chk(idx, torch.int32, 'idx', B)
    lib().is_sample(ptr(losses), ptr(ema), ptr(ctrl), ptr(idx), ptr(w), ptr(meters), P, B, group,
                    int(importance), alpha, ema_alpha, int(seed) & 0xffffffff, stream_ptr(),
                    int(alias), ptr(gathered), gathered.shape[0] if gathered is not None else 1)


def gather(pool, pool_label, pool_index, idx, batch, batch_label, batch_index, B):
    per_img = pool[0].numel() * 2 // 16
    lib().gather(ptr(pool), ptr(pool_label), ptr(pool_index), ptr(idx), ptr(batch),
                 ptr(batch_label), ptr(batch_index), B, per_img, stream_ptr())
