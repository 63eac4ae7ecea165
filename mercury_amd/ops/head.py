"""Classifier head front-end: avg-pool + FC + (IS-weighted) CE (``csrc/head.hip``)."""
from __future__ import annotations

import torch

from . import _chk, lib, ptr, stream_ptr

MODE = {'score': 0, 'train': 1, 'eval': 2}


SCORE = {'loss': 0, 'gradnorm': 1}


def head_fwd(act, w, b, label, B, HW, C, classes, mode, pooled=None, logits=None, dlogits=None,
             losses=None, isw=None, meters=None, score='loss'):
    """``score``: what score mode writes into ``losses`` -- 'loss' (per-sample CE, the
    reference) or 'gradnorm' (exact per-sample gradient norm of the classifier layer)."""
    _chk(act, torch.bfloat16, 'act', B * HW * C)
    _chk(w, torch.float32, 'w', classes * C)
    _chk(label, torch.int32, 'label', B)
    lib().head_fwd(ptr(act), ptr(w), ptr(b), ptr(label), ptr(isw), ptr(pooled), ptr(logits),
                   ptr(dlogits), ptr(losses), ptr(meters), B, HW, C, classes, MODE[mode],
                   stream_ptr(), SCORE[score])


def head_bwd(pooled, dlogits, w, dw, db, dact, B, HW, C, classes):
    _chk(dact, torch.bfloat16, 'dact', B * HW * C)
    lib().head_bwd(ptr(pooled), ptr(dlogits), ptr(w), ptr(dw), ptr(db), ptr(dact), B, HW, C,
                   classes, stream_ptr())
