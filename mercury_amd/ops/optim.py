"""Fused flat-buffer optimizer front-end (``csrc/optim.hip``).

``FlatOptimizer`` owns fp32 ``p``/``g``/``m``/``v`` flat buffers (4-element
aligned segments), a device segment table describing which segments are conv
weights (and where their bf16 MFMA operand copies live), and a device
hyper-parameter vector ``[lr, beta1, beta2, eps, weight_decay]``.  ``step``
is one launch; ``set_lr`` is a 4-byte host->device copy done outside graphs
(the cosine schedule changes lr once per epoch).
"""
from __future__ import annotations


import torch

from . import lib, ptr, stream_ptr

# kernel algorithm codes (csrc/kernels.h OptArgs.algo)
ALGOS = {'adam': 0, 'sgd': 1, 'adamw': 2}


def optimizer_spec(optimizer):
    """Map a ``torch.optim`` instance onto the fused kernel, or raise ``ValueError``.

    Only exact types are accepted (``AdamW`` subclasses ``Adam`` in torch 2.x, so an
    ``isinstance`` test would silently run it with coupled L2 decay), with one param group and
    no option the kernel does not implement.  Returns the ``FlatOptimizer`` keyword arguments."""
    groups = optimizer.param_groups
    if len(groups) != 1:
        raise ValueError('native optimizer: exactly one param group supported, got %d'
                         % len(groups))
    g = groups[0]
    t = type(optimizer)
    if g.get('maximize', False):
        raise ValueError('native optimizer: maximize=True is not supported')
    if g.get('differentiable', False):
        raise ValueError('native optimizer: differentiable=True is not supported')
    if t is torch.optim.Adam or t is torch.optim.AdamW:
        if g.get('amsgrad', False):
            raise ValueError('native optimizer: amsgrad=True is not supported')
        algo = 'adamw' if (t is torch.optim.AdamW or g.get('decoupled_weight_decay', False)) \
            else 'adam'
        lr = g['lr']
        if torch.is_tensor(lr):
            lr = float(lr)
        return dict(algo=algo, lr=lr, betas=tuple(g['betas']), eps=g['eps'],
                    weight_decay=g['weight_decay'], momentum=0.9)
    if t is torch.optim.SGD:
        if g.get('nesterov', False):
            raise ValueError('native optimizer: nesterov=True is not supported')
        if g.get('dampening', 0) != 0:
            raise ValueError('native optimizer: dampening != 0 is not supported')
        if g.get('momentum', 0) == 0:
            raise ValueError('native optimizer: SGD without momentum is not supported '
                             '(the kernel keeps a momentum buffer)')
        return dict(algo='sgd', lr=g['lr'], betas=(0.9, 0.999), eps=1e-8,
                    weight_decay=g['weight_decay'], momentum=g['momentum'])
    raise ValueError('native optimizer: %s is not supported (Adam, AdamW, SGD with momentum)'
                     % t.__name__)


class FlatOptimizer(object):

    def __init__(self, segments, total, device, algo='adam', lr=1e-3, betas=(0.9, 0.999),
                 eps=1e-8, weight_decay=0.0, momentum=0.9, fused=True):
        self.device = torch.device(device)
        self.total = int(total)
        self.segments = segments
        self.p = torch.zeros(self.total, dtype=torch.float32, device=device)
        self.g = torch.zeros_like(self.p)
        self.m = torch.zeros_like(self.p)
        if algo not in ALGOS:
            raise ValueError('FlatOptimizer algo must be one of %s, got %r' % (sorted(ALGOS), algo))
        adam = algo in ('adam', 'adamw')
        self.v = torch.zeros_like(self.p) if adam else torch.zeros(4, device=device)
        self.algo = ALGOS[algo]
        b1 = betas[0] if adam else momentum
        self.hyper = torch.tensor([lr, b1, betas[1], eps, weight_decay, 0, 0, 0],
                                  dtype=torch.float32, device=device)
        rows = []
        for s in segments:
            rows.append([s['off'], s['numel'], s['kind'], s.get('K', 0), s.get('R', 1),
                         s.get('S', 1), s.get('C', 1), s.get('Cpad', 1),
                         ptr(s.get('w_krsc')), ptr(s.get('w_crsk'))])
        self._seg_starts = set(int(s['off']) for s in segments)
        packed = lib().pack_opt_segs(rows)
        self.segbuf = torch.frombuffer(bytearray(packed), dtype=torch.uint8).to(device)
        self.nsegs = len(rows)
        # 64x64 transpose tiles producing the dgrad ([C][R][S][K]) weight copies
        jobs = []
        for i, s in enumerate(segments):
            if s['kind'] == 1 and s.get('w_crsk') is not None:
                for rs in range(s['R'] * s['S']):
                    for k0 in range(0, s['K'], 64):
                        for c0 in range(0, s['C'], 64):
                            jobs.append((i, rs, k0, c0))
        self.njobs = len(jobs)
        # jobs are ordered by segment, hence by flat offset: a range's jobs are a slice
        self._job_off = [segments[j[0]]['off'] for j in jobs]
        self.jobs = torch.tensor(jobs if jobs else [(0, 0, 0, 0)], dtype=torch.int32,
                                 device=device).contiguous()
        # fused full step (csrc/optim.hip optimizer_fused_kernel): 64x64 update tiles for conv
        # segments that carry a dgrad copy (their [C][R][S][K] copy is written from the update),
        # float4 elementwise ranges for everything else
        fjobs, ew = [], []
        for i, s in enumerate(segments):
            if s['kind'] == 1 and s.get('w_crsk') is not None and s['C'] % 4 == 0:
                for rs in range(s['R'] * s['S']):
                    for k0 in range(0, s['K'], 64):
                        for c0 in range(0, s['C'], 64):
                            fjobs.append((i, rs, k0, c0))
            else:
                ew.append((int(s['off']), (int(s['numel']) + 3) // 4 * 4))
        pre = [0]
        for _, n in ew:
            pre.append(pre[-1] + n // 4)
        self.fused = bool(fused)        # EngineOptions.fused_opt
        self.n_fjobs = len(fjobs)
        self.fjobs = torch.tensor(fjobs if fjobs else [(0, 0, 0, 0)], dtype=torch.int32,
                                  device=device).contiguous()
        self.ew = torch.tensor(ew if ew else [(0, 0)], dtype=torch.int64, device=device)
        self.ewp = torch.tensor(pre, dtype=torch.int64, device=device)
        self.n_ew, self.ew4 = len(ew), pre[-1]
        # dgrad copies of conv segments the tiles do not cover still go through the transpose
        fused_segs = set(j[0] for j in fjobs)
        rest = [j for j in jobs if j[0] not in fused_segs]
        self.n_rest = len(rest)
        self.rest_jobs = torch.tensor(rest if rest else [(0, 0, 0, 0)], dtype=torch.int32,
                                      device=device).contiguous()

    def _transpose(self, start=0, end=None):
        end = self.total if end is None else end
        j0 = next((i for i, o in enumerate(self._job_off) if o >= start), self.njobs)
        j1 = next((i for i, o in enumerate(self._job_off) if o >= end), self.njobs)
        if j1 > j0:
            lib().transpose_weights(ptr(self.segbuf), ptr(self.jobs) + 16 * j0, j1 - j0,
                                    stream_ptr())

    @property
    def lr(self):
        return float(self.hyper[0].item())

    def set_lr(self, lr):
        self.hyper[0].fill_(float(lr))

    def step(self, step_counter, zero_grad=True, start=0, end=None):
        """``step_counter``: device int64 scalar tensor/view holding t (already incremented).
        ``start``/``end``: update only the flat range [start, end) -- both must be segment
        starts (or ``total``); two range steps equal one full step."""
        end = self.total if end is None else end
        for b in (start, end):
            if b != self.total and b not in self._seg_starts:
                raise ValueError('optimizer range bound %d is not a segment start' % b)
        if self.fused and start == 0 and end == self.total:
            lib().optimizer_fused(ptr(self.p), ptr(self.g), ptr(self.m), ptr(self.v),
                                  ptr(self.segbuf), self.nsegs, self.total, ptr(self.hyper),
                                  ptr(step_counter), self.algo, int(zero_grad), ptr(self.fjobs),
                                  self.n_fjobs, ptr(self.ew), ptr(self.ewp), self.n_ew, self.ew4,
                                  stream_ptr())
            if self.n_rest:
                lib().transpose_weights(ptr(self.segbuf), ptr(self.rest_jobs), self.n_rest,
                                        stream_ptr())
            return
        lib().optimizer(ptr(self.p), ptr(self.g), ptr(self.m), ptr(self.v), ptr(self.segbuf),
                        self.nsegs, end, ptr(self.hyper), ptr(step_counter), self.algo,
                        int(zero_grad), stream_ptr(), start)
        self._transpose(start, end)

    def pack_weights(self):
        """Write the bf16 conv-weight copies from the fp32 master (after init / load)."""
        lib().pack_weights(ptr(self.p), ptr(self.segbuf), self.nsegs, self.total, stream_ptr())
        self._transpose()
