"""BatchNorm / activation / residual front-end (kernels in ``csrc/bn.hip``)."""
from __future__ import annotations

import torch

from . import _chk, lib, ptr, stream_ptr

ACT = {'none': 0, 'relu': 1, 'relu6': 2}


def bn_apply(y, stats, gamma, beta, out, M, C, group_rows=0, act='relu', eps=1e-5,
             running=None, res=None, res_bn=None):
    """out = act(bn(y) [+ res | + bn2(res)]).

    ``stats`` [G][2][C] fp32 sums (train) -- or ``running=(mean, var)`` for eval.
    ``res_bn = (stats2, gamma2, beta2[, (rmean2, rvar2)])`` normalises ``res`` first."""
    for t, n in ((y, 'y'), (out, 'out'), (res, 'res')):
        _chk(t, torch.bfloat16, n, None if t is None else M * C)
    if C % 8:
        raise ValueError('C must be a multiple of 8')
    res_mode = 0 if res is None else (2 if res_bn is not None else 1)
    s2 = g2 = b2 = rm2 = rv2 = None
    if res_bn is not None:
        s2, g2, b2 = res_bn[:3]
        if len(res_bn) > 3 and res_bn[3] is not None:
            rm2, rv2 = res_bn[3]
    rm = rv = None
    if running is not None:
        rm, rv = running
    lib().bn_apply(ptr(y), ptr(stats), ptr(gamma), ptr(beta), ptr(rm), ptr(rv),
                   int(running is not None), res_mode, ptr(res), ptr(s2), ptr(g2), ptr(b2),
                   ptr(rm2), ptr(rv2), ptr(out), M, C, group_rows or M, ACT[act], eps,
                   stream_ptr())
    return out


def sums_numel(C):
    """fp32 elements of a BN-backward sums workspace for C channels: [SUMS_R][3][C]."""
    return int(getattr(lib(), 'SUMS_R', 1)) * 3 * C     # (1: a build without replicas)


def sums_total(sums, C):
    """[3][C] totals of a [SUMS_R][3][C] BN-backward sums workspace."""
    return sums.reshape(-1, 3, C).sum(0)


def bn_bwd(dout, out, y, stats, gamma, sums, dy, M, C, act='relu', eps=1e-5, y2=None,
           stats2=None, gamma2=None, dy2=None, dz=None, dgamma=None, dbeta=None, dgamma2=None,
           dbeta2=None, zero_sums=True, reduce=True):
    """BN(+shortcut BN)+activation backward for one stat group.

    ``sums``: [SUMS_R][3][C] fp32 workspace (replicas the producers spread their atomics over,
    summed when applied: ``sums_total``) that must be zero on entry; ``zero_sums=False`` when
    the caller zeroes a whole arena once per step (one memset instead of one per layer).
    ``reduce=False``: the sums were already reduced by the producing dgrad's epilogue
    (``conv_dgrad(bw=...)``) -- only the apply pass runs."""
    _chk(sums, torch.float32, 'sums', sums_numel(C))
    if zero_sums and reduce:
        sums.zero_()
    lib().bn_bwd(ptr(dout), ptr(out), ptr(y), ptr(stats), ptr(gamma), ptr(y2), ptr(stats2),
                 ptr(gamma2), ptr(sums), ptr(dy), ptr(dy2), ptr(dz), ptr(dgamma), ptr(dbeta),
                 ptr(dgamma2), ptr(dbeta2), M, C, ACT[act], eps, stream_ptr(), 3 if reduce else 2)
    return dy


class BnRunTable(object):
    """Device table driving the one-launch running-stats update of every BN layer."""

    def __init__(self, rows, device):
        # rows: (rmean, rvar, stats_train, stats_score, nbt, C, n_train, n_score, cnt_tr, cnt_sc)
        packed = lib().pack_bn_table([[float(ptr(r[0])), float(ptr(r[1])), float(ptr(r[2])),
                                       float(ptr(r[3])), float(ptr(r[4])), r[5], r[6], r[7],
                                       r[8], r[9]] for r in rows])
        self.buf = torch.frombuffer(bytearray(packed), dtype=torch.uint8).to(device)
        self.n = len(rows)
        self.maxC = max(r[5] for r in rows)
        self._keep = rows

    def launch(self, momentum=0.1):
        lib().bn_running(ptr(self.buf), self.n, self.maxC, momentum, stream_ptr())
