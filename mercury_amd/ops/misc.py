"""Pooling, depthwise conv, quantisation front-ends (``csrc/misc.hip``)."""
from __future__ import annotations

import torch

from . import _chk, lib, ptr, stream_ptr


def quantize(x, out=None, ws=None, seed=0, counter=0):
    _chk(x, torch.float32, 'x')
    out = torch.empty_like(x) if out is None else out
    ws = torch.empty(1, dtype=torch.float32, device=x.device) if ws is None else ws
    lib().quantize(ptr(x), ptr(out), ptr(ws), x.numel(), int(seed) & 0xffffffff, int(counter),
                   stream_ptr())
    return out


def tern_pack(x, words, ws, seed=0, counter=0):
    """x fp32 [n] -> int32 message [1 + ceil(n/16)] (parallel/compress.py layout)."""
    _chk(x, torch.float32, 'x')
    n = x.numel()
    _chk(words, torch.int32, 'words', 1 + (n + 15) // 16)
    lib().tern_pack(ptr(x), n, ptr(ws), int(seed) & 0xffffffff, int(counter), ptr(words),
                    stream_ptr(), 0)
    return words


def tern_unpack(msgs, W, n, out, scale=None):
    """out[n] = scale * sum over W messages of max_r * code_r (scale defaults to 1/W)."""
    _chk(msgs, torch.int32, 'msgs', W * (1 + (n + 15) // 16))
    _chk(out, torch.float32, 'out', n)
    lib().tern_unpack(ptr(msgs), W, n, 1.0 / W if scale is None else float(scale), ptr(out),
                      stream_ptr())
    return out


ACT = {'none': 0, 'relu': 1, 'relu6': 2}


def pool2d_fwd(x, y, N, H, W, C, P, Q, k, stride, pad, is_max=True, argmax=None, bn=None):
    """NHWC bf16 max/avg pool.  ``argmax`` (uint8, N*P*Q*C) records the window tap of each
    maximum for ``maxpool2d_bwd``.  ``bn`` = dict(gamma, beta, act, eps and either stats
    [G][2][C] + group_imgs, or rmean + rvar): ``x`` is the raw conv output and its BatchNorm +
    activation are applied per tap (no separate bn_apply pass)."""
    _chk(x, torch.bfloat16, 'x', N * H * W * C)
    _chk(y, torch.bfloat16, 'y', N * P * Q * C)
    if argmax is not None:
        _chk(argmax, torch.uint8, 'argmax', N * P * Q * C)
    bn = bn or {}
    lib().pool2d_fwd(ptr(x), ptr(y), ptr(argmax), N, H, W, C, P, Q, k, stride, pad, int(is_max),
                     stream_ptr(), ptr(bn.get('stats')), ptr(bn.get('gamma')),
                     ptr(bn.get('beta')), ptr(bn.get('rmean')), ptr(bn.get('rvar')),
                     int(bn.get('group_imgs', 0)), ACT[bn.get('act', 'none')],
                     float(bn.get('eps', 1e-5)))


def maxpool2d_bwd(dy, argmax, dx, N, H, W, C, P, Q, k, stride, pad):
    _chk(argmax, torch.uint8, 'argmax', N * P * Q * C)
    lib().maxpool2d_bwd(ptr(dy), ptr(argmax), ptr(dx), N, H, W, C, P, Q, k, stride, pad,
                        stream_ptr())


_ACT = {None: 0, 'none': 0, 'relu': 1, 'relu6': 2}


def dwconv_fwd(x, w, y, N, H, W, C, P, Q, stride, pad, stats=None, group_rows=0, pro=None):
    """Depthwise 3x3 forward (+ BN sums).  ``pro``: x is the producer's raw output and
    act(bn(x)) is applied to each loaded chunk -- dict(stats=[G][2][C] | rmean/rvar, gamma,
    beta, act, eps, count, group_imgs, keep=optional activation output)."""
    pa = (0, 0, 0, 0, 0, 0, 0.0, 0.0, 0, 0)
    if pro is not None:
        for k in ('stats', 'rmean', 'rvar', 'gamma', 'beta'):
            _chk(pro.get(k), torch.float32, 'pro.' + k)
        _chk(pro.get('keep'), torch.bfloat16, 'pro.keep', N * H * W * C)
        if pro.get('stats') is None and pro.get('rmean') is None:
            raise ValueError('pro needs stats or running statistics')
        pa = (ptr(pro.get('stats')), ptr(pro.get('rmean')), ptr(pro.get('rvar')),
              ptr(pro['gamma']), ptr(pro['beta']), ptr(pro.get('keep')),
              1.0 / float(pro.get('count', 1)), float(pro.get('eps', 1e-5)),
              _ACT[pro.get('act')], int(pro.get('group_imgs') or N))
    lib().dwconv_fwd(ptr(x), ptr(w), ptr(y), ptr(stats), N, H, W, C, P, Q, stride, pad,
                     group_rows or N * P * Q, stream_ptr(), *pa)


def dwconv_dgrad(dy, w, dx, N, H, W, C, P, Q, stride, pad, bw=None):
    """Depthwise 3x3 data gradient.  ``bw``: dict(out=, y=, stats=[2][C], sums=[SUMS_R][3][C], act=,
    eps=) -- also reduce the BN-backward sums of the BN feeding this conv (its activation
    ``out``, input ``y``), as bn_bwd's reduce pass would (one batch group)."""
    ba = (0, 0, 0, 0, 0.0, 0.0, 0)
    if bw is not None:
        n_in = N * H * W * C
        for k in ('out', 'y'):
            _chk(bw[k], torch.bfloat16, 'bw.' + k, n_in)
        _chk(bw['stats'], torch.float32, 'bw.stats', 2 * C)
        _chk(bw['sums'], torch.float32, 'bw.sums', int(getattr(lib(), 'SUMS_R', 1)) * 3 * C)
        if bw.get('y2') is not None:
            raise ValueError('dwconv_dgrad: no shortcut-BN reduce')
        ba = (ptr(bw['out']), ptr(bw['y']), ptr(bw['stats']), ptr(bw['sums']),
              1.0 / (N * H * W), float(bw.get('eps', 1e-5)), _ACT[bw.get('act')])
    lib().dwconv_dgrad(ptr(dy), ptr(w), ptr(dx), N, H, W, C, P, Q, stride, pad, stream_ptr(), *ba)


def dwconv_bwd(dy, x, w, dx, dw, N, H, W, C, P, Q, stride, pad, slab, bw=None, reduce=True):
    """Depthwise dgrad (+ fused BN-backward sums ``bw``, as dwconv_dgrad) and slab wgrad in
    ONE launch.  ``slab`` (fp32, >= dwconv_wgrad_slab_floats): the wgrad blocks' partials;
    ``reduce=False`` leaves them for dwconv_wgrad_reduce_batch (dw is then not yet updated)."""
    _chk(slab, torch.float32, 'slab', dwconv_wgrad_slab_floats(N, P, Q, C))
    _chk(dy, torch.bfloat16, 'dy', N * P * Q * C)
    ba = (0, 0, 0, 0, 0.0, 0.0, 0)
    if bw is not None:
        n_in = N * H * W * C
        for k in ('out', 'y'):
            _chk(bw[k], torch.bfloat16, 'bw.' + k, n_in)
        _chk(bw['stats'], torch.float32, 'bw.stats', 2 * C)
        _chk(bw['sums'], torch.float32, 'bw.sums', int(getattr(lib(), 'SUMS_R', 1)) * 3 * C)
        if bw.get('y2') is not None:
            raise ValueError('dwconv_bwd: no shortcut-BN reduce')
        ba = (ptr(bw['out']), ptr(bw['y']), ptr(bw['stats']), ptr(bw['sums']),
              1.0 / (N * H * W), float(bw.get('eps', 1e-5)), _ACT[bw.get('act')])
    lib().dwconv_bwd(ptr(dy), ptr(x), ptr(w), ptr(dx), ptr(dw), N, H, W, C, P, Q, stride, pad,
                     ptr(slab), int(reduce), stream_ptr(), *ba)


def dwconv_wgrad_reduce_batch(items):
    """dw += the slab partials of several dwconv_bwd(reduce=False) launches in one kernel;
    ``items``: [(slab, dw, C, nblk)] with nblk = dwconv_wgrad_blocks(N, P, Q, C)."""
    if not items:
        return
    lib().dwconv_wgrad_reduce_batch([ptr(s) for s, _, _, _ in items],
                                    [ptr(d) for _, d, _, _ in items],
                                    [int(c) for _, _, c, _ in items],
                                    [int(n) for _, _, _, n in items], stream_ptr())


def dwconv_wgrad_blocks(N, P, Q, C):
    """wgrad blocks (= slab partial rows) of the train-batch depthwise wgrad."""
    return int(lib().dwconv_wgrad_blocks(N, P, Q, C))


def dwconv_wgrad_slab_floats(N, P, Q, C):
    """fp32 workspace for ``dwconv_wgrad(slab=...)`` (per-block partials)."""
    return int(lib().dwconv_wgrad_slab_floats(N, P, Q, C))


def dwconv_wgrad(dy, x, dw, N, H, W, C, P, Q, stride, pad, slab=None):
    """dw[C][9] += depthwise 3x3 weight gradient.  ``slab`` (fp32, >= dwconv_wgrad_slab_floats
    elements): column-segmented rows with the blocks' partials summed by a second kernel
    instead of atomics (faster at the train batch)."""
    _chk(slab, torch.float32, 'slab')
    lib().dwconv_wgrad(ptr(dy), ptr(x), ptr(dw), N, H, W, C, P, Q, stride, pad, stream_ptr(),
                       ptr(slab), 0 if slab is None else slab.numel())


def nchw_to_nhwc8(x, y):
    """float32 [N][C][H][W] -> bf16 [N][H][W][Cpad] (channels zero-padded), on device."""
    _chk(x, torch.float32, 'x')
    N, C, H, W = x.shape
    Cpad = y.shape[-1]
    _chk(y, torch.bfloat16, 'y', N * H * W * Cpad)
    lib().nchw_to_nhwc8(ptr(x), ptr(y), N, C, H, W, Cpad, stream_ptr())
    return y
