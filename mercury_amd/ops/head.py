"""Classifier head front-end: avg-pool + FC + (IS-weighted) CE (``csrc/head.hip``)."""
from __future__ import annotations

import torch

from . import _chk, lib, ptr, stream_ptr

MODE = {'score': 0, 'train': 1, 'eval': 2}


SCORE = {'loss': 0, 'gradnorm': 1}


_ACT = {'none': 0, 'relu': 1, 'relu6': 2}


def head_fwd(act, w, b, label, B, HW, C, classes, mode, pooled=None, logits=None, dlogits=None,
             losses=None, isw=None, meters=None, score='loss', bn=None):
    """``score``: what score mode writes into ``losses`` -- 'loss' (per-sample CE, the
    reference) or 'gradnorm' (exact per-sample gradient norm of the classifier layer).

    ``bn`` (scoring / eval): ``act`` is the last conv's raw output and the head pools
    act(bn(act) [+ res]) -- dict(gamma, beta, eps, act, res=None, and stats + count +
    group_imgs (ghost / batch statistics) or rmean + rvar (running)) -- instead of reading a
    block output that a bn_apply pass wrote."""
    _chk(act, torch.bfloat16, 'act', B * HW * C)
    _chk(w, torch.float32, 'w', classes * C)
    _chk(label, torch.int32, 'label', B)
    bnargs = (0, 0, 0, 0, 0, 0, 0.0, 0.0, 1, 0)
    if bn is not None:
        if pooled is None:
            raise ValueError('head_fwd: the BN prologue writes pooled[]')
        if bn.get('res') is not None:
            _chk(bn['res'], torch.bfloat16, 'bn res', B * HW * C)
        st = bn.get('stats')
        bnargs = (ptr(bn.get('res')), ptr(st), ptr(bn.get('rmean')), ptr(bn.get('rvar')),
                  ptr(bn['gamma']), ptr(bn['beta']),
                  1.0 / float(bn['count']) if st is not None else 0.0, float(bn['eps']),
                  int(bn.get('group_imgs') or B), _ACT[bn['act']])
    lib().head_fwd(ptr(act), ptr(w), ptr(b), ptr(label), ptr(isw), ptr(pooled), ptr(logits),
                   ptr(dlogits), ptr(losses), ptr(meters), B, HW, C, classes, MODE[mode],
                   stream_ptr(), SCORE[score], *bnargs)


def head_bwd(pooled, dlogits, w, dw, db, dact, B, HW, C, classes, bw=None):
    """Classifier-head backward.  ``bw`` (as conv_dgrad's): also reduce the BN-backward sums of
    the final BN whose activation the head read; returns True when it did (the per-sample
    path -- the wide GEMM path does not, and the caller then runs bn_bwd's reduce)."""
    from .conv import _bw_args
    _chk(dact, torch.bfloat16, 'dact', B * HW * C)
    return bool(lib().head_bwd(ptr(pooled), ptr(dlogits), ptr(w), ptr(dw), ptr(db), ptr(dact),
                               B, HW, C, classes, stream_ptr(), *_bw_args(bw, B * HW, C)))


def mlp_head_fwd(x, w1, b1, w2, b2, h1, logits, label, B, F, H1, classes, mode, isw=None,
                 dlogits=None, losses=None, meters=None, score='loss', splits=0):
    """Speech-VGG head (`pytorch_model.py:145-153`): h1 = x . W1^T + b1, logits = h1 . W2^T + b2,
    then log-softmax CE (loss / IS-weighted dlogits / meters / score) -- all HIP kernels.
    x: bf16 [B][F] (NHWC flatten), W1: bf16 [H1][F] in the same (H, W, C) column order."""
    _chk(x, torch.bfloat16, 'x', B * F)
    _chk(w1, torch.bfloat16, 'w1', H1 * F)
    for t, n, k in ((b1, 'b1', H1), (w2, 'w2', classes * H1), (b2, 'b2', classes),
                    (h1, 'h1', B * H1), (logits, 'logits', B * classes)):
        _chk(t, torch.float32, n, k)
    _chk(label, torch.int32, 'label', B)
    if not splits:
        # split the 7680-deep fc1 reduction so ~256 blocks run (64 x 64 output tiles)
        tiles = -(-B // 64) * -(-H1 // 64)
        splits = max(1, min(-(-F // 64), 256 // max(tiles, 1)))
    lib().mlp_head_fwd(ptr(x), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(h1), ptr(logits),
                       ptr(label), ptr(isw), ptr(dlogits), ptr(losses), ptr(meters), B, F, H1,
                       classes, MODE[mode], SCORE[score], splits, stream_ptr())


def mlp_head_bwd(dlogits, h1, x, w1, w2, dh1, dw1, db1, dw2, db2, dx, B, F, H1, classes):
    """Gradients of the speech-VGG head: dW2, db2, dh1, db1, dW1 (engine [H1][F] layout) and the
    bf16 activation gradient dx [B][F]."""
    _chk(dx, torch.bfloat16, 'dx', B * F)
    _chk(dw1, torch.float32, 'dw1', H1 * F)
    _chk(dh1, torch.float32, 'dh1', B * H1)
    lib().mlp_head_bwd(ptr(dlogits), ptr(h1), ptr(x), ptr(w1), ptr(w2), ptr(dh1), ptr(dw1),
                       ptr(db1), ptr(dw2), ptr(db2), ptr(dx), B, F, H1, classes, stream_ptr())
