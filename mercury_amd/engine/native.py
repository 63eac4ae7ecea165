"""The MI355X-native training engine: fused HIP kernels + HIP graphs + RCCL.

One importance-sampled step (reference `pytorch_collab.py:127-164`) runs as:

    S1 (score stream)  : pool_build -> forward(B=320, ghost BN) -> CE scores
                         -> is_sample (EMA replay, p, draws, weights)
    S0 (main stream)   : forward(B=32) -> IS-weighted CE -> backward, segmented
                         at gradient-bucket boundaries; after each segment the
                         bucket's RCCL all-reduce (AVG) is issued on the NCCL
                         stream while later segments and S1 keep computing
    S0 after join      : BN running stats (train batch, then the 10 scoring
                         groups, in reference order) -> fused Adam (+bf16
                         weight packing, gradient zeroing) -> gather the drawn
                         samples into the next training batch

Scoring uses the same (pre-update) weights as training, exactly like the
reference, so it overlaps the whole train fwd/bwd and the all-reduce instead
of serialising after them (the reference's dead overlap code,
`pytorch_collab.py:154-156`, made real without the race).  Each stream's work
is captured once into HIP graphs (``torch.cuda.CUDAGraph``) and replayed, so
a step costs a handful of host calls.  All buffers are allocated up front.
"""
from __future__ import annotations

import gc
import math
import time
import weakref

import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from ..ops import hconv, tune
from ..ops.conv import (ConvSpec, cpad8, dgrad_plan, fwd_plan, pgemm_ok, pgemm_plain_wins,
                        pgemm_plan, pgemm_pro_wins, pro_plan, pwconv_ok, pwconv_plain_wins,
                        pwconv_pro_wins, slab_bytes,
                        stem_ok, wgrad_plan)
from ..ops.conv import pro_ok as conv_pro_ok
from ..parallel.buckets import default_bucket_bytes

_RELEASE = []    # (hipGraphExec_t, [hipEvent_t]) of un-closed collected engines


_HWQ_WARNED = []
LIVE = weakref.WeakSet()   # open engines of this process (close_all: test / program teardown)


def close_all():
    """Close every open engine of this process (deterministic teardown)."""
    for e in list(LIVE):
        e.close()


def _warn_hw_queues():
    """Once per process: the step's three streams need >= 16 hardware queues, set before HIP
    starts (mercury_amd/__init__.py); say so when that did not happen."""
    import warnings
    from .. import HW_QUEUES
    if HW_QUEUES['effective'] or _HWQ_WARNED:
        return
    _HWQ_WARNED.append(1)
    warnings.warn('mercury_amd: the HIP runtime started with GPU_MAX_HW_QUEUES=%s (< 16): the '
                  'scoring / train / comm streams can share hardware queues and the step runs '
                  'serially (~1.6x slower).  Import mercury_amd (or export GPU_MAX_HW_QUEUES=16) '
                  'before anything initialises the GPU.' % (HW_QUEUES['before'] or 'default 4'),
                  RuntimeWarning, stacklevel=3)


def _release_queued():
    """Destroy what collected (never closed) engines queued -- caller has synchronised."""
    while _RELEASE:
        ex, evs = _RELEASE.pop()
        if ex:
            ops.lib().graph_exec_destroy(ex)
        for e in evs:
            ops.lib().ext_event_destroy(e)


from ..trainer import Trainer
from ..utils import profiling as prof
from ..utils.meters import Accuracy, Average, EMAverage
from .lower import lower, supports  # noqa: F401

BN_EPS = 1e-5


class _Mode(object):
    """Per-batch-size buffers: activations, stats, plans, slabs."""

    def __init__(self, name, N, group_imgs, train):
        self.name = name
        self.N = N
        self.group_imgs = group_imgs   # images per BN stat group (0 = whole batch)
        self.train = train
        self.spec = {}
        self.plan = {}
        self.buf = {}
        self.stats = {}
        self.slab = None
        self.G = 1 if not group_imgs else N // group_imgs
        self.prereduced = {}             # block index -> BN sums already reduced by a dgrad
        self.dw_region = {}              # depthwise unit -> (slab offset, floats, wgrad blocks)
        self.dw_pending = []             # deferred depthwise wgrad reduces of this backward


class NativeEngine(object):

    def __init__(self, net, device, batch_size=32, pool_batches=10, num_classes=None,
                 image_hw=(32, 32), optimizer='adam', lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.0, momentum=0.9, seed=0, alpha=0.5, ema_alpha=0.9,
                 importance=True, world_size=1, bucket_bytes=None, use_graphs=True,
                 sampler='alias', exchange_scores=False, global_table=True, score='loss',
                 global_ema=False, autotune=None, force_buckets=False, comm='auto',
                 wire_bf16=False, debug=False, check_order=False, grad_compress=None,
                 opts=None):
        ops.lib()
        _warn_hw_queues()
        from ..config import EngineOptions
        self.opts = opts if opts is not None else EngineOptions.from_env()
        if autotune is not None:
            tune.enable(autotune)
        self.net = net
        self.device = torch.device(device)
        self.lw = lower(net)
        self.B = batch_size
        self.P = batch_size * pool_batches
        self.pool_batches = pool_batches
        self.classes = self.lw.num_classes
        self.H, self.W = image_hw
        self.seed = seed
        self.alpha, self.ema_alpha, self.importance = alpha, ema_alpha, importance
        self.world_size = world_size
        self.use_graphs = use_graphs and not debug
        self.debug = debug
        # data-parallel gradient path.  ``force_buckets`` runs the real bucketed all-reduces
        # even at W = 1 (the one-GPU box exercises the RCCL code path; AVG over one rank is the
        # identity, so results are bit-identical to the unbucketed step)
        self.dp = world_size > 1 or (force_buckets and dist.is_initialized())
        self._avg_op = None
        self.comm = None                 # own RCCL communicator (csrc/comm.hip)
        self.s_comm = None               # ... and the stream its bucket all-reduces run on
        rp = self.opts.role_prio
        self._role_prio = (-1 if self.dp else 0) if rp == 'auto' else int(rp)
        self.wire_bf16 = wire_bf16
        if self.dp:
            nccl = dist.get_backend() == 'nccl'
            self._avg_op = dist.ReduceOp.AVG if nccl else dist.ReduceOp.SUM
            if comm == 'auto':
                comm = 'rccl' if nccl else 'pg'
            if comm in ('rccl', 'xgmi'):
                from ..parallel.rccl import RcclComm
                self.comm = RcclComm.shared()
                self.s_comm = ops.role_stream(self.device, 'comm', self._role_prio)
            elif comm != 'pg':
                raise ValueError("comm must be 'auto', 'rccl', 'xgmi' or 'pg'")
        self.comm_kind = comm if self.dp else None
        self.xgmi = None                 # direct-xGMI two-shot all-reduce (parallel/xgmi.py)
        if grad_compress not in (None, 'none', 'ternary'):
            raise ValueError("grad_compress must be None, 'none' or 'ternary'")
        if grad_compress == 'ternary' and (wire_bf16 or comm == 'xgmi'):
            raise ValueError('grad_compress=ternary is its own wire format (no bf16 / xgmi)')
        self.grad_compress = grad_compress if grad_compress != 'none' else None
        self.tern = None                 # ternary-compressed all-reduce (parallel/compress.py)
        self._pg_works = []              # ProcessGroup works issued by the last step ('pg')
        self._closed = True              # (open once __init__ has finished: see its end)
        self._tern_ctr = 0
        # DP verification hook (tests): grad_probe(stage, i, t) sees bucket i's gradient slice as
        # the backward left it ('pre', on the stream that reduces it, before the collective) and
        # the whole flat gradient the optimizer will read ('post', i = None, on the train stream
        # before the tail).  Host-issued, so it sees every step, graphs or not.
        self.grad_probe = None
        self.bucket_bytes = bucket_bytes or default_bucket_bytes(world_size)
        # the last bucket (closed when the backward ends, so fully exposed) holds only the
        # leading blocks' parameters up to this many bytes (bucket_plan)
        self.last_bucket_bytes = int(self.opts.last_bucket_mb * (1 << 20))
        # measured all-reduce cost model (alpha, beta) and the plan derived from it: under DP on
        # the engine's RCCL communicator the bucket sizes come from timing the real collective
        # at start-up, not from an assumed link bandwidth (parallel/buckets.py)
        self.comm_calib = None
        cal = self.opts.bucket_calib
        if cal not in ('auto', 'on', 'off'):
            raise ValueError("EngineOptions.bucket_calib must be 'auto', 'on' or 'off'")
        if self.comm is not None and comm == 'rccl' and grad_compress in (None, 'none') and (
                cal == 'on' or (cal == 'auto' and bucket_bytes is None and
                                (self.comm.size > 1 or self.opts.rccl_one_rank))):
            from ..parallel.buckets import calibrate_allreduce, plan_from_calibration
            self.comm_calib = calibrate_allreduce(self.comm, self.device)
            bb, lb = plan_from_calibration(self.comm_calib)
            if bucket_bytes is None:
                self.bucket_bytes = bb
            self.last_bucket_bytes = lb
            self.comm_calib.update(bucket_bytes=self.bucket_bytes, last_bucket_bytes=lb)
        self.units = []
        for blk in self.lw.blocks:
            self.units += blk.units + ([blk.shortcut] if blk.shortcut else [])
        # conv bias (speech VGG) is added in the conv epilogue; under train-mode BN its gradient
        # is exactly zero (the batch mean absorbs it), so its grad segment is never written
        self._make_params(optimizer, lr, betas, eps, weight_decay, momentum)
        self.modes = {}
        self.ctrl = torch.zeros(8, dtype=torch.int64, device=self.device)
        self.ema = torch.zeros(2, dtype=torch.float32, device=self.device)
        self.meters = torch.zeros(8, dtype=torch.float32, device=self.device)
        self.eval_meters = torch.zeros(8, dtype=torch.float32, device=self.device)
        # (stream priorities, a CU-masked scoring stream, a weight-gradient side stream and an
        # early optimizer split were all measured neutral or slower on MI355X and removed:
        # profiles/ab_experiments_r1c.json)
        # the scoring and comm streams each own a hardware queue (ops.role_stream): a pooled
        # stream that lands on the train stream's queue serialises the step (1.37 -> 2.1 ms)
        self.s_score = ops.role_stream(self.device, 'score', self._role_prio)
        self.graphs = None
        self._bucket_evs = []            # event-record nodes of the one-graph DP replay
        self._train_exec = 0             # ... and that graph (hipGraphExec_t)
        self.shard = None
        self.primed = False              # a scored pool / drawn batch is pending
        self.scoring = True
        self.fuse_bn_bwd = True          # BN-backward reduce in the dgrad epilogue
        self.roctx = False               # per-phase roctx ranges around the step's host calls
        self.pair_bwd = True             # dgrad + wgrad of a conv in one launch
        # kernel-path switches (config.EngineOptions: defaults = the measured-best paths, each
        # with the A/B that keeps it)
        o = self.opts
        self.fuse_bn_fwd = o.fuse_bn_fwd
        self.use_hconv = o.hconv
        self.use_pgemm = o.pgemm
        self.use_pwconv = o.pwconv
        self.use_stem = o.stem
        self.dw_pro = o.dw_pro
        self.res_pro = o.fuse_bn_fwd and o.res_pro
        self.head_bw = o.head_bw
        self.dw_pair = o.dw_pair
        self.persist_bn = o.persist_bn if o.persist_bn in ('0', '1', 'row', 'stat') else (
            '1' if str(o.persist_bn).lower() in ('true', 'on', 'yes') else '0')
        self._apply_globals()

        if sampler not in ('alias', 'cdf', 'groupwise'):
            raise ValueError("sampler must be 'alias', 'cdf' or 'groupwise'")
        self.sampler = sampler
        if sampler == 'groupwise' and not global_table:
            raise ValueError("sampler='groupwise' draws from the global table (global_table=True)")
        if sampler == 'groupwise' and (exchange_scores or global_ema):
            raise ValueError("sampler='groupwise' has no pool EMA to share across ranks")
        if score not in ('loss', 'gradnorm'):
            raise ValueError('score must be loss or gradnorm')
        self.score = score
        self.global_table = global_table
        self.table = None
        self.score_exchange = None
        self.global_ema = global_ema
        if self.dp and (exchange_scores or global_ema):
            from ..parallel.scores import ScoreExchange
            # on an RCCL communicator of its own when the engine has one: stream-ordered on the
            # score stream, no ProcessGroup work in flight during a step or a capture, and not
            # queued in front of the gradient buckets (RCCL runs one communicator's operations
            # in issue order across streams, and the all-gather is issued first every step)
            xc = None
            if self.comm is not None:
                from ..parallel.rccl import RcclComm
                xc = RcclComm.shared(tag='score')
            self.score_exchange = ScoreExchange(self.P, self.device, force=world_size == 1,
                                                comm=xc)
        from .timing import StepTimer
        self.timer = StepTimer(self.device)   # per-phase device timing (off until enabled)
        self.wire = None
        # race detection: device-side stream-order assertions (csrc/runtime.hip);
        # debug mode also serialises the streams, runs eagerly and syncs after every phase
        self.check_order = check_order or debug
        self.order = torch.zeros(16, dtype=torch.int32, device=self.device)
        self.debug_log = self.opts.debug_log
        if self.comm_kind == 'xgmi':
            from ..parallel.xgmi import XgmiAllReduce
            cap = max(e - s_ for s_, e in self.bucket_plan().values())
            self.xgmi = XgmiAllReduce(cap, self.device, wire_bf16=wire_bf16)
        if self.dp and self.grad_compress == 'ternary':
            from ..parallel.compress import TernaryAllReduce
            cap = max(e - s_ for s_, e in self.bucket_plan().values())
            self.tern = TernaryAllReduce(cap, self.device, comm=self.comm, seed=seed)
        # registered for close_all() only once fully built: a constructor that raised leaves
        # nothing half-initialised for a later teardown to trip over
        self._closed = False
        LIVE.add(self)

    def _apply_globals(self):
        """The few EngineOptions that live in process-wide state (the halo-conv launcher's
        persistent grid / waves / plan overrides, the stride-2 dgrad switch) are re-applied by
        every phase of THIS engine that reads them -- plan building (set_shard / mode), eager
        launches and graph capture -- so engines with different options can share a process."""
        hconv.configure(self.opts)
        ops.conv.DGRAD_S2 = self.opts.dgrad_s2

    # ------------------------------------------------------------------ parameters
    def _final_chw(self):
        """(C, H, W) of the last block's output (speech VGG: 512 x 3 x 5 for 1x101x161)."""
        h, w = self.H, self.W
        for blk in self.lw.blocks:
            for u in blk.units:
                h = (h + 2 * u.pad - u.R) // u.stride + 1
                w = (w + 2 * u.pad - u.R) // u.stride + 1
            if blk.pool is not None:
                k, st, pd = blk.pool
                h = (h + 2 * pd - k) // st + 1
                w = (w + 2 * pd - k) // st + 1
        return self.lw.blocks[-1].units[-1].K, h, w

    def _make_params(self, optimizer, lr, betas, eps, wd, momentum):
        segs = []
        self.w_krsc, self.w_crsk = {}, {}
        # speech VGG: fc1's master weights live in [f1][H][W][C] order (the flatten order of the
        # NHWC activation), so fc1 is a plain GEMM on the activation rows; the optimizer writes
        # its bf16 copy like a conv weight's (torch's [f1][C][H][W] at the state-dict boundary)
        self.mlp_chw = None
        self.w1p = None
        if self.lw.head_pool == 'mlp2':
            c, h, w = self._final_chw()
            f1 = self.lw.fc1.out_features
            if c * h * w != self.lw.fc1.in_features:
                raise ValueError('fc1 expects %d inputs, the features give %d x %d x %d'
                                 % (self.lw.fc1.in_features, c, h, w))
            self.mlp_chw = (c, h, w)
            self.w1p = torch.zeros(f1, h, w, c, dtype=torch.bfloat16, device=self.device)
        for u in self.units:
            if u.depthwise:
                continue
            K, C, R = u.K, u.C, u.R
            self.w_krsc[u.name] = torch.zeros(K, R, R, cpad8(C), dtype=torch.bfloat16,
                                              device=self.device)
            if u.need_dgrad:
                self.w_crsk[u.name] = torch.zeros(C, R, R, K, dtype=torch.bfloat16,
                                                  device=self.device)
        unit_by_w = {id(u.w_seg): u for u in self.units}
        for s in self.lw.segs:
            d = dict(off=s.off, numel=s.numel, kind=0)
            u = unit_by_w.get(id(s))
            if u is not None and not u.depthwise:
                d.update(kind=1, K=u.K, R=u.R, S=u.R, C=u.C, Cpad=cpad8(u.C),
                         w_krsc=self.w_krsc[u.name], w_crsk=self.w_crsk.get(u.name))
            elif self.mlp_chw is not None and s is self.lw.fc1_w:
                c, h, w = self.mlp_chw
                d.update(kind=1, K=self.lw.fc1.out_features, R=h, S=w, C=c, Cpad=c,
                         w_krsc=self.w1p, w_crsk=None)
            segs.append(d)
        self.opt = ops.FlatOptimizer(segs, self.lw.total, self.device, optimizer, lr, betas, eps,
                                     wd, momentum, fused=self.opts.fused_opt)
        self.load_from_module()

    def _pview(self, seg, grad=False):
        buf = self.opt.g if grad else self.opt.p
        return buf[seg.off:seg.off + seg.numel]

    def _krsc_shape(self, seg):
        """[K][C][R][S] torch shape of a segment stored KRSC in the master, else None."""
        if seg.kind == 'conv':
            return tuple(seg.param.shape)
        if self.mlp_chw is not None and seg is self.lw.fc1_w:
            c, h, w = self.mlp_chw
            return (self.lw.fc1.out_features, c, h, w)
        return None

    @torch.no_grad()
    def load_from_module(self):
        """Module parameters (torch layout) -> flat master (engine layout) + bf16 copies."""
        for s in self.lw.segs:
            self._from_torch_layout(s, self.opt.p, s.param.detach())
        self.opt.pack_weights()

    @torch.no_grad()
    def sync_to_module(self):
        """Flat master -> module parameters (torch layout).  BN buffers are shared already."""
        for s in self.lw.segs:
            s.param.data.copy_(self._to_torch_layout(s, self.opt.p).reshape(s.param.shape))

    def _to_torch_layout(self, seg, flat):
        v = flat[seg.off:seg.off + seg.numel]
        sh = self._krsc_shape(seg)
        if sh is not None:
            k, c, r, s = sh
            return v.view(k, r, s, c).permute(0, 3, 1, 2).reshape(seg.param.shape).contiguous()
        return v.view(seg.param.shape).clone()

    def _from_torch_layout(self, seg, flat, t):
        t = t.to(self.device, torch.float32)
        sh = self._krsc_shape(seg)
        if sh is not None:
            t = t.reshape(sh).permute(0, 2, 3, 1)
        flat[seg.off:seg.off + seg.numel].copy_(t.reshape(-1))

    # ------------------------------------------------------------------ buffers
    def mode(self, name, N=None, group_imgs=0, train=False):
        if name in self.modes:
            return self.modes[name]
        self._apply_globals()
        m = _Mode(name, N, group_imgs, train)
        dev = self.device
        H, W = self.H, self.W
        C = cpad8(self.lw.in_channels)
        slab = 0
        dw_slab = 0
        coef = 0
        nstats = 0
        nsums = 0
        bf = torch.bfloat16

        def act(M, K):
            return torch.empty(M * K, dtype=bf, device=dev)

        for bi, blk in enumerate(self.lw.blocks):
            h, w = H, W
            main_hw = None
            for u in blk.units + ([blk.shortcut] if blk.shortcut else []):
                if u is blk.shortcut:
                    main_hw = (h, w)
                    h, w = H, W          # the shortcut reads the block input
                sp = ConvSpec(N, h, w, u.C, u.K, u.R, u.R, u.stride, u.pad)
                if group_imgs:
                    sp.group_rows = group_imgs * sp.P * sp.Q
                m.spec[u.name] = sp
                if u.depthwise and train:
                    # per-block weight-gradient partials (summed by a reduce kernel), a region
                    # per layer so the reduces can be deferred and batched at the end of the
                    # backward; its own buffer (the split-K slab's head holds tile counters)
                    m.dw_region[u.name] = (dw_slab, ops.dwconv_wgrad_slab_floats(
                        N, sp.P, sp.Q, sp.C), ops.dwconv_wgrad_blocks(N, sp.P, sp.Q, sp.C))
                    dw_slab += m.dw_region[u.name][1]
                if not u.depthwise:
                    # measured-best plans from the tuning cache (ops/tune.py) when present
                    # the scoring pass runs beside the latency-bound train chain: fewer, larger
                    # tiles leave the train kernels more room (measured, ResNet-18: 128-block
                    # target 1.656 vs 256-block 1.667 ms/step; split-K or 512 blocks slower)
                    mb = self.opts.score_min_blocks if group_imgs else 0
                    m.plan[u.name, 'fwd'] = p = tune.fwd_plan_for(
                        sp, fwd_plan(sp, min_blocks=mb) if mb else fwd_plan(sp))
                    slab = max(slab, slab_bytes(sp.M, sp.K, *p[:3]))
                    pp = pro_plan(sp) if self.opts.pro_plans else None
                    if pp is not None:
                        # the plan it runs with when it takes its input's BN in the prologue
                        m.plan[u.name, 'fwd_pro'] = pp
                        slab = max(slab, slab_bytes(sp.M, sp.K, *pp))
                    if self.use_pgemm and pgemm_ok(sp) and u.b_seg is None:
                        m.plan[u.name, 'pgemm'] = pgemm_plan(sp)
                        coef = max(coef, m.G * 2 * sp.Cp)
                    if self.use_stem and stem_ok(sp) and bi == 0 and u is blk.units[0]:
                        m.plan[u.name, 'stem'] = True
                    if self.use_pwconv and pwconv_ok(sp) and u.b_seg is None:
                        m.plan[u.name, 'pwconv'] = True
                        coef = max(coef, m.G * 2 * sp.Cp)
                    # stride-1 3x3 convs on the halo-tile kernel where it measured faster
                    uh = self.use_hconv == '1' or self.use_hconv == ('train' if train else 'score')
                    hp = hconv.engine_plan(sp, bias=u.b_seg is not None,
                                           train=train) if uh else None
                    if hp is not None:
                        m.plan[u.name, 'hconv'] = hp
                        slab = max(slab, slab_bytes(sp.M, sp.K, *hp[:3]))
                    # scoring pass: an intra-block conv on the persistent kernel takes its
                    # input's BN + activation in the halo staging (no residual there)
                    hb = None
                    if not train and group_imgs and self.persist_bn != '0' and \
                            u is not blk.units[0] and u is not blk.shortcut:
                        hb = hconv.persist_bn_plan(sp, group_imgs,
                                                   row_only=self.persist_bn in ('row', 'stat'),
                                                   stat_only=self.persist_bn == 'stat')
                    if hb is not None:
                        m.plan[u.name, 'hconv_bn'] = hb
                        slab = max(slab, slab_bytes(sp.M, sp.K, *hb[:3]))
                    if train:
                        if u.need_dgrad and sp.K % 8 == 0:
                            dp, wp = tune.bwd_plans_for(sp, dgrad_plan(sp), wgrad_plan(sp))
                        else:
                            dp, wp = dgrad_plan(sp), wgrad_plan(sp)
                        if u.need_dgrad:
                            m.plan[u.name, 'dgrad'] = dp
                            slab = max(slab, slab_bytes(N * h * w, sp.Cp, *dp))
                        m.plan[u.name, 'wgrad'] = wp
                m.buf[u.name, 'y'] = act(sp.M, u.K)
                m.stats[u.name] = nstats
                nstats += m.G * 2 * u.K
                if u is not blk.units[-1] and u is not blk.shortcut:
                    m.buf[u.name, 'a'] = act(sp.M, u.K)
                if train:
                    m.buf[u.name, 'dy'] = act(sp.M, u.K)
                    m.buf[u.name, 'sums'] = nsums
                    nsums += ops.sums_numel(u.K)      # [SUMS_R][3][K] replicas
                    if u is not blk.units[-1] and u is not blk.shortcut:
                        m.buf[u.name, 'da'] = act(sp.M, u.K)
                if u is not blk.shortcut:
                    h, w = sp.P, sp.Q
            if main_hw is not None:
                h, w = main_hw
            last = blk.units[-1]
            K = last.K
            m.buf[bi, 'out'] = act(N * h * w, K)
            if train:
                m.buf[bi, 'dout'] = act(N * h * w, K)
            if blk.pool is not None:
                k, st, pd = blk.pool
                P_ = (h + 2 * pd - k) // st + 1
                Q_ = (w + 2 * pd - k) // st + 1
                m.buf[bi, 'pre'] = m.buf[bi, 'out']
                m.buf[bi, 'out'] = act(N * P_ * Q_, K)
                m.buf[bi, 'pool_geom'] = (N, h, w, K, P_, Q_, k, st, pd)
                if train:
                    m.buf[bi, 'argmax'] = torch.empty(N * P_ * Q_ * K, dtype=torch.uint8,
                                                      device=dev)
                    m.buf[bi, 'dpre'] = m.buf[bi, 'dout']
                    m.buf[bi, 'dout'] = act(N * P_ * Q_, K)
                h, w = P_, Q_
            m.buf[bi, 'hw'] = (h, w)
            H, W, C = h, w, K
        m.stats_arena = torch.zeros(max(nstats, 1), device=dev)
        m.sums_arena = torch.zeros(max(nsums, 1), device=dev)
        for key, off in list(m.stats.items()):
            u = next(x for x in self.units if x.name == key)
            m.stats[key] = m.stats_arena[off:off + m.G * 2 * u.K]
            if train:
                so = m.buf[u.name, 'sums']
                m.buf[u.name, 'sums'] = m.sums_arena[so:so + ops.sums_numel(u.K)]
        m.final_hw = H * W
        m.final_C = C
        m.pooled = torch.zeros(N, C, device=dev)
        m.logits = torch.zeros(N, self.classes, device=dev)   # wide heads' FC output
        m.losses = torch.zeros(N, device=dev)
        if train:
            m.dlogits = torch.zeros(N, self.classes, device=dev)
        m.slab = torch.zeros(max(1, (slab + 3) // 4), dtype=torch.float32, device=dev)
        m.dw_slab = torch.empty(dw_slab, dtype=torch.float32, device=dev) if dw_slab else None
        # per-stream scale / shift workspace of the pointwise GEMM's input prologue (each fused
        # conv's coefficient kernel fills it right before the conv, on the same stream)
        m.coef = torch.zeros(max(1, coef), dtype=torch.float32, device=dev)
        m.input = torch.zeros(N, self.H, self.W, cpad8(self.lw.in_channels), dtype=bf, device=dev)
        m.label = torch.zeros(N, dtype=torch.int32, device=dev)
        m.index = torch.zeros(N, dtype=torch.int32, device=dev)
        self.modes[name] = m
        return m

    # ------------------------------------------------------------------ layer execution
    def _gamma(self, u, grad=False):
        return self._pview(u.g_seg, grad)

    def _beta(self, u, grad=False):
        return self._pview(u.beta_seg, grad)

    def _conv_fwd(self, m, u, x, y, stats, pro=None):
        sp = m.spec[u.name]
        if (u.name, 'stem') in m.plan and pro is None:
            ops.stem_fwd(x, self.w_krsc[u.name], y, sp, stats=stats,
                         bias=self._pview(u.b_seg) if u.b_seg is not None else None)
            return
        if pro is not None and pro.get('pw'):
            ops.pwconv_fwd(x, self.w_krsc[u.name], y, sp, stats=stats, pro=pro)
            return
        if pro is None and (u.name, 'pwconv') in m.plan and pwconv_plain_wins(sp) and \
                self.opts.pwconv_plain:
            ops.pwconv_fwd(x, self.w_krsc[u.name], y, sp, stats=stats)
            return
        pg = m.plan.get((u.name, 'pgemm'))
        if pg is not None and (pro is not None and pro.get('pg') or
                               pro is None and pgemm_plain_wins(sp)):
            ops.pgemm_fwd(x, self.w_krsc[u.name], y, sp, stats=stats, bn=pg, pro=pro)
            return
        if u.depthwise:
            ops.dwconv_fwd(x, self._pview(u.w_seg), y, sp.N, sp.H, sp.W, sp.C, sp.P, sp.Q,
                           sp.stride, sp.pad, stats=stats, group_rows=sp.group_rows or sp.M,
                           pro=pro if pro is not None and pro.get('dw') else None)
        elif pro is None and (u.name, 'hconv') in m.plan:
            hconv.hconv_fwd(x, self.w_krsc[u.name], y, sp, m.plan[u.name, 'hconv'], stats=stats,
                            slab=m.slab,
                            bias=self._pview(u.b_seg) if u.b_seg is not None else None)
        else:
            ops.conv_fwd(x, self.w_krsc[u.name], y, sp, stats=stats, slab=m.slab,
                         plan=self._pro_plan(m, u) if pro is not None else m.plan[u.name, 'fwd'],
                         bias=self._pview(u.b_seg) if u.b_seg is not None else None, pro=pro)

    def _pro_plan(self, m, u):
        """igemm plan of ``u`` when it applies its input's BN in the prologue."""
        return m.plan.get((u.name, 'fwd_pro'), m.plan[u.name, 'fwd'])

    def _igemm_only(self, m, u):
        """True when _conv_fwd(m, u, ..., pro=None) runs u on the plain igemm kernel."""
        if u.depthwise or u.b_seg is not None:
            return False
        if any((u.name, k) in m.plan for k in ('stem', 'hconv')):
            return False
        if (u.name, 'pwconv') in m.plan and pwconv_plain_wins(m.spec[u.name]) and \
                self.opts.pwconv_plain:
            return False
        return not ((u.name, 'pgemm') in m.plan and pgemm_plain_wins(m.spec[u.name]))

    def _dual_fwd(self, m, u, sc, x, stats_on):
        """A downsampling block's first conv and its shortcut conv (both read the block input x)
        in ONE launch (ops.conv_fwd_dual); False when the pair does not qualify."""
        if not self.opts.dual_fwd or not (self._igemm_only(m, u) and self._igemm_only(m, sc)):
            return False
        pa, pb = m.plan[u.name, 'fwd'], m.plan[sc.name, 'fwd']
        if tuple(pa[:2]) != tuple(pb[:2]):
            return False
        slab_b = m.slab
        if pa[2] > 1 and pb[2] > 1:
            # the shortcut's split-K partials and tile counters get a slab of their own
            slab_b = m.buf.get((sc.name, 'slab'))
            if slab_b is None:
                if torch.cuda.is_current_stream_capturing():
                    return False
                sp = m.spec[sc.name]
                slab_b = m.buf[sc.name, 'slab'] = torch.zeros(
                    (slab_bytes(sp.M, sp.K, *pb[:3]) + 3) // 4, dtype=torch.float32,
                    device=self.device)
        a = dict(x=x, w=self.w_krsc[u.name], out=m.buf[u.name, 'y'], spec=m.spec[u.name],
                 stats=m.stats[u.name] if stats_on else None, slab=m.slab, plan=pa)
        b = dict(x=x, w=self.w_krsc[sc.name], out=m.buf[sc.name, 'y'], spec=m.spec[sc.name],
                 stats=m.stats[sc.name] if stats_on else None, slab=slab_b, plan=pb)
        return ops.conv_fwd_dual(a, b)

    def _pro_for(self, m, u, nxt):
        """BN-apply of ``u`` folded into the load of its consumer ``nxt`` (csrc/igemm.h
        ProParams), or None when that conv/plan cannot take it.  Train mode also keeps the
        activation (backward reads it) through the consumer's centre-tap write-back."""
        if not self.fuse_bn_fwd or u.act not in ('relu', 'relu6', 'none'):
            return None
        if nxt.depthwise:
            # MobileNetV2's expand BN + ReLU6 applied to each chunk the depthwise conv loads
            if not self.dw_pro:
                return None
            su = m.spec[u.name]
            d = dict(dw=True, gamma=self._gamma(u), beta=self._beta(u), act=u.act, eps=BN_EPS,
                     keep=m.buf[u.name, 'a'] if m.train else None,
                     group_imgs=m.group_imgs or m.N)
            if m.train or m.group_imgs:
                d.update(stats=m.stats[u.name], count=su.group_rows or su.M)
            else:
                d.update(rmean=u.bn.running_mean, rvar=u.bn.running_var)
            return d
        pg = self._pg_pro(m, u, u.act, m.buf[u.name, 'a'] if m.train else None, nxt)
        if pg is not None:
            return pg
        sp = m.spec[nxt.name]
        if not conv_pro_ok(sp, self._pro_plan(m, nxt), keep=m.train):
            return None
        su = m.spec[u.name]
        d = dict(gamma=self._gamma(u), beta=self._beta(u), act=u.act, eps=BN_EPS,
                 keep=m.buf[u.name, 'a'] if m.train else None)
        if m.train or m.group_imgs:
            d.update(stats=m.stats[u.name], count=su.group_rows or su.M)
        else:
            d.update(rmean=u.bn.running_mean, rvar=u.bn.running_var)
        return d

    def _pg_pro(self, m, u, act, keep, nxt, res=None):
        """Input prologue of the pointwise GEMM running ``nxt`` on the raw output of ``u``:
        act(bn_u(y) [+ res]), activation written to ``keep`` (or None), or None when ``nxt``
        does not run on pgemm.  Narrow-input convs whose output spans several N-tiles take the
        panel-resident kernel instead (pwconv.hip: each element normalised once, not per tile)."""
        if act not in ('relu', 'relu6', 'none'):
            return None
        su, sn = m.spec[u.name], m.spec[nxt.name]
        if res is None and (nxt.name, 'pwconv') in m.plan and pwconv_pro_wins(sn):
            kind = 'pw'
        elif (nxt.name, 'pgemm') in m.plan and sn.stride == 1 and pgemm_pro_wins(sn):
            kind = 'pg'
        else:
            return None
        d = dict(gamma=self._gamma(u), beta=self._beta(u), act=act, eps=BN_EPS,
                 keep=keep, res=res, coef=m.coef, group_rows=su.group_rows or su.M)
        d[kind] = True
        if m.train or m.group_imgs:
            d.update(stats=m.stats[u.name], count=su.group_rows or su.M)
        else:
            d.update(rmean=u.bn.running_mean, rvar=u.bn.running_var)
        return d

    def _res_pro(self, m, u, act, out, nxt, res):
        """Block-final BN (+ identity residual ``res``) + activation folded into the
        register-staged load of the next block's first (pointwise) conv on igemm:
        a = act(bn_u(y) [+ res]), the block output ``out`` written once through the prologue's
        keep (MobileNetV2's linear-bottleneck outputs feeding the next expand conv), instead of
        a bn_apply pass."""
        if not self.res_pro or act not in ('relu', 'relu6', 'none') or nxt.depthwise:
            return None
        # (a pwconv plan only runs with its own prologue kind; with this prologue the conv runs
        # on igemm -- not where the persistent GEMM would have run it plain, e.g. ResNet-50)
        if any((nxt.name, k) in m.plan for k in ('stem', 'hconv')):
            return None
        sp = m.spec[nxt.name]
        if (nxt.name, 'pgemm') in m.plan and pgemm_plain_wins(sp):
            return None
        if sp.R != 1 or not conv_pro_ok(sp, self._pro_plan(m, nxt), keep=True):
            return None
        su = m.spec[u.name]
        d = dict(gamma=self._gamma(u), beta=self._beta(u), act=act, eps=BN_EPS, keep=out,
                 res=res)
        if m.train or m.group_imgs:
            d.update(stats=m.stats[u.name], count=su.group_rows or su.M)
        else:
            d.update(rmean=u.bn.running_mean, rvar=u.bn.running_var)
        return d

    def _pool_bn(self, m, u, act):
        d = dict(gamma=self._gamma(u), beta=self._beta(u), act=act, eps=BN_EPS)
        if m.group_imgs:
            d.update(stats=m.stats[u.name], group_imgs=m.group_imgs)
        else:
            d.update(rmean=u.bn.running_mean, rvar=u.bn.running_var)
        return d

    def _bn_apply(self, m, u, y, out, act, res=None, res_unit=None):
        sp = m.spec[u.name]
        kw = {}
        if m.train or m.group_imgs:
            stats, running = m.stats[u.name], None
        else:
            stats, running = None, (u.bn.running_mean, u.bn.running_var)
        if res_unit is not None:
            r2 = None if stats is not None else (res_unit.bn.running_mean,
                                                 res_unit.bn.running_var)
            kw['res_bn'] = (m.stats[res_unit.name] if stats is not None else None,
                            self._gamma(res_unit), self._beta(res_unit), r2)
        ops.bn_apply(y, stats, self._gamma(u), self._beta(u), out, sp.M, u.K,
                     group_rows=sp.group_rows or sp.M, act=act, eps=BN_EPS, running=running,
                     res=res, **kw)

    # -- BatchNorm folded into the halo conv (csrc/hconv.hip persistent / row-step MODE 1, the
    # scoring pass): an intra-block BN output that the next conv can stage itself stays
    # "pending" -- (raw conv output, its BN unit, activation) -- and that conv applies it while
    # loading its halo.  Plans: ``hconv.persist_bn_plan`` / ``m.plan[name, 'hconv_bn']``.
    def _pending(self, u, y, act):
        return dict(unit=u, y=y, act=act)

    def _can_take(self, m, u):
        return (u.name, 'hconv_bn') in m.plan and not u.depthwise

    def _hconv_pending(self, m, u, pend, y, stats):
        """conv ``u`` on the pending activation ``pend``: hconv with the BN applied in staging."""
        sp = m.spec[u.name]
        pu = pend['unit']
        su = m.spec[pu.name]
        pro = dict(gamma=self._gamma(pu), beta=self._beta(pu), act=pend['act'], eps=BN_EPS,
                   count=su.group_rows or su.M, group_imgs=m.group_imgs or m.N)
        if m.train or m.group_imgs:
            pro['stats'] = m.stats[pu.name]
        else:
            pro.update(rmean=pu.bn.running_mean, rvar=pu.bn.running_var)
        hconv.hconv_fwd(pend['y'], self.w_krsc[u.name], y, sp, m.plan[u.name, 'hconv_bn'],
                        stats=stats, slab=m.slab,
                        bias=self._pview(u.b_seg) if u.b_seg is not None else None, pro=pro)

    def forward(self, m, x=None):
        """Forward through all blocks; returns the final activation buffer."""
        x = m.input if x is None else x
        stats_on = m.train or m.group_imgs
        m.head_bn = None     # (set below when the head's pool applies the last block's BN)
        x_last = None
        pend = None          # an intra-block BN output the next conv applies in its staging
        nblk = len(self.lw.blocks)
        pool_bn = None       # BN + activation the block's max pool applies (scoring/eval stem)
        pgp = None           # the previous block's final BN (+ identity residual), applied by the
        #                      pointwise GEMM that consumes it (which writes the block output)
        for bi, blk in enumerate(self.lw.blocks):
            inp = x
            nu = len(blk.units)
            pro = None
            sc_done = False      # the shortcut conv already ran (with the first conv, one launch)
            for i, u in enumerate(blk.units):
                y = m.buf[u.name, 'y']
                st = m.stats[u.name] if stats_on else None
                if pgp is not None:
                    self._conv_fwd(m, u, pgp['y'], y, st, pro=pgp['pro'])
                    pgp = None
                elif (i == 0 and pend is None and blk.shortcut is not None and
                        self._dual_fwd(m, u, blk.shortcut, inp, stats_on)):
                    sc_done = True
                elif pend is not None:
                    # the previous unit's BN + act applied while staging (scoring pass: nothing
                    # reads the intra-block activation)
                    self._hconv_pending(m, u, pend, y, st)
                    pend = None
                else:
                    self._conv_fwd(m, u, inp, y, st, pro=pro)
                if i < nu - 1:
                    nxt = blk.units[i + 1]
                    if self._can_take(m, nxt) and u.act in ('relu', 'relu6', 'none'):
                        pend = self._pending(u, y, u.act)
                        continue
                    # intra-block BN + activation: inside the next conv's operand load when it
                    # can take it, else its own pass
                    pro = self._pro_for(m, u, nxt)
                    if pro is not None:
                        inp = y
                        continue
                    a = m.buf[u.name, 'a']
                    self._bn_apply(m, u, y, a, u.act)
                    inp = a
                else:
                    out = m.buf[bi, 'pre'] if blk.pool else m.buf[bi, 'out']
                    res, ru = None, None
                    if blk.shortcut is not None:
                        sc = blk.shortcut
                        if not sc_done:
                            self._conv_fwd(m, sc, x, m.buf[sc.name, 'y'],
                                           m.stats[sc.name] if stats_on else None)
                        res, ru = m.buf[sc.name, 'y'], sc
                    elif blk.identity:
                        res = x
                    nb = self.lw.blocks[bi + 1] if bi + 1 < nblk else None
                    pgd = None
                    if nb is not None and not blk.pool and nb.units and ru is None:
                        pgd = self._pg_pro(m, u, blk.final_act, out, nb.units[0], res=res)
                        if pgd is None:
                            pgd = self._res_pro(m, u, blk.final_act, out, nb.units[0], res)
                    if pgd is not None:
                        # the next block's first (pointwise) conv applies this BN (+ identity
                        # residual) + activation in its operand tiles and writes ``out``
                        pgp = dict(y=y, pro=pgd)
                    elif (nb is None and not m.train and not blk.pool and ru is None and
                          self.opts.head_bn and self.lw.head_pool != 'mlp2' and
                          blk.final_act in ('relu', 'relu6', 'none') and u.K % 8 == 0):
                        # scoring / eval: nothing reads the last block's output but the head's
                        # average pool, which applies this BN (+ identity residual) +
                        # activation itself (ops.head_fwd ``bn``): no bn_apply pass
                        hb = dict(gamma=self._gamma(u), beta=self._beta(u), act=blk.final_act,
                                  eps=BN_EPS, res=res)
                        if m.group_imgs:
                            su = m.spec[u.name]
                            hb.update(stats=m.stats[u.name], count=su.group_rows or su.M,
                                      group_imgs=m.group_imgs)
                        else:
                            hb.update(rmean=u.bn.running_mean, rvar=u.bn.running_var)
                        m.head_bn = hb
                        x_last = y
                    elif (blk.pool and not m.train and res is None and
                          blk.final_act in ('relu', 'relu6', 'none')):
                        # scoring / eval (nothing reads the pre-pool activation): the pool
                        # applies this BN + activation per tap, straight from the conv output
                        pool_bn = self._pool_bn(m, u, blk.final_act)
                    else:
                        self._bn_apply(m, u, y, out, blk.final_act, res=res, res_unit=ru)
            if blk.pool:
                N, h, w, K, P_, Q_, k, st, pd = m.buf[bi, 'pool_geom']
                src = m.buf[bi, 'pre']
                if pool_bn is not None:
                    src = m.buf[blk.units[-1].name, 'y']
                ops.pool2d_fwd(src, m.buf[bi, 'out'], N, h, w, K, P_, Q_, k, st, pd,
                               True, m.buf.get((bi, 'argmax')), bn=pool_bn)
                pool_bn = None
            x = m.buf[bi, 'out']
        if m.head_bn is not None:
            return x_last            # the raw last conv output: the head applies its BN
        return x

    # ------------------------------------------------------------------ speech-VGG head
    # flatten -> fc1 -> fc2 -> log_softmax (CE on log-probs == CE on logits), all HIP kernels
    # (csrc/head.hip mlp_head_*): fc1 runs on the NHWC activation rows against the [f1][H][W][C]
    # bf16 copy the optimizer writes, its weight gradient lands in the flat buffer in that order
    def _mlp_setup(self, m):
        f1 = self.lw.fc1.out_features
        m.h1 = torch.zeros(m.N, f1, device=self.device)
        if m.train:
            m.dh1 = torch.zeros(m.N, f1, device=self.device)

    def _mlp_head(self, m, x, mode, isw=None, meters=None):
        if getattr(m, 'h1', None) is None:
            self._mlp_setup(m)
        c, h, w = self.mlp_chw
        ops.mlp_head_fwd(x, self.w1p, self._pview(self.lw.fc1_b), self._pview(self.lw.fc_w),
                         self._pview(self.lw.fc_b), m.h1, m.logits, m.label, m.N, c * h * w,
                         self.lw.fc1.out_features, self.classes, mode, isw=isw,
                         dlogits=m.dlogits if mode == 'train' else None, losses=m.losses,
                         meters=meters if mode != 'score' else None,
                         score=self.score if mode == 'score' else 'loss')

    def _mlp_head_bwd(self, m, dout):
        """Grads of fc2 / fc1 into the flat buffer and d(activation) (NHWC bf16) into dout."""
        c, h, w = self.mlp_chw
        x = m.buf[len(self.lw.blocks) - 1, 'out']
        ops.mlp_head_bwd(m.dlogits, m.h1, x, self.w1p, self._pview(self.lw.fc_w), m.dh1,
                         self._pview(self.lw.fc1_w, True), self._pview(self.lw.fc1_b, True),
                         self._pview(self.lw.fc_w, True), self._pview(self.lw.fc_b, True), dout,
                         m.N, c * h * w, self.lw.fc1.out_features, self.classes)

    def head(self, m, x, mode, isw=None, meters=None):
        if self.lw.head_pool == 'mlp2':
            return self._mlp_head(m, x, mode, isw=isw, meters=meters)
        hb = getattr(m, 'head_bn', None) if mode != 'train' else None
        ops.head_fwd(x, self._pview(self.lw.fc_w), self._pview(self.lw.fc_b), m.label, m.N,
                     m.final_hw, m.final_C, self.classes, mode, pooled=m.pooled,
                     logits=m.logits,
                     dlogits=getattr(m, 'dlogits', None) if mode == 'train' else None,
                     losses=m.losses, isw=isw, meters=meters,
                     score=self.score if mode == 'score' else 'loss', bn=hb)

    def flush_dw_reduces(self, m):
        """The deferred depthwise wgrad reduces of this backward, in one launch."""
        ops.dwconv_wgrad_reduce_batch(m.dw_pending)
        m.dw_pending = []

    def _wgrad(self, m, u, dy, x):
        sp = m.spec[u.name]
        gw = self._pview(u.w_seg, grad=True)
        if u.depthwise:
            if m.dw_slab is not None:
                off, n, _ = m.dw_region[u.name]
                ops.dwconv_wgrad(dy, x, gw, sp.N, sp.H, sp.W, sp.C, sp.P, sp.Q, sp.stride,
                                 sp.pad, slab=m.dw_slab[off:off + n])
            else:
                ops.dwconv_wgrad(dy, x, gw, sp.N, sp.H, sp.W, sp.C, sp.P, sp.Q, sp.stride,
                                 sp.pad)
        else:
            ops.conv_wgrad(dy, x, gw, sp, plan=m.plan[u.name, 'wgrad'])

    def _conv_bwd(self, m, u, dy, x, dx, accumulate, bw=None):
        """Weight gradient, then the data gradient.  ``bw``: the dgrad epilogue also reduces
        the BN-backward sums of the unit feeding ``dx`` (returns True when it did, so the
        caller skips bn_bwd's reduce pass)."""
        sp = m.spec[u.name]
        if (dx is not None and not u.depthwise and self.pair_bwd and sp.K % 8 == 0):
            if bw is not None and (sp.Cp != sp.C or not self.fuse_bn_bwd):
                bw = None
            # dgrad + wgrad of this conv in ONE launch (they share dy and are independent)
            ops.conv_bwd(dy, self.w_crsk[u.name], dx, x, self._pview(u.w_seg, grad=True), sp,
                         dplan=m.plan[u.name, 'dgrad'], wplan=m.plan[u.name, 'wgrad'],
                         slab=m.slab, accumulate=accumulate, bw=bw)
            return bw is not None
        if u.depthwise and dx is not None and m.dw_slab is not None and self.dw_pair:
            assert not accumulate
            # the producer's BN-backward sums reduced in the depthwise dgrad (no bn_bwd reduce
            # pass; one batch group in train mode, no shortcut BN)
            if bw is not None and (not self.fuse_bn_bwd or bw.get('y2') is not None):
                bw = None
            # dgrad + wgrad in one launch; the wgrad partials' reduce is deferred to one batched
            # launch (flush_dw_reduces) -- nothing reads a depthwise weight gradient before the
            # optimizer or its bucket's all-reduce
            off, n, nblk = m.dw_region[u.name]
            region = m.dw_slab[off:off + n]
            gw = self._pview(u.w_seg, grad=True)
            # deferred to one batched launch: at the end of the backward, or (DP) before the
            # bucket all-reduce that carries this weight gradient (train_segments)
            defer = True
            ops.dwconv_bwd(dy, x, self._pview(u.w_seg), dx, gw, sp.N, sp.H, sp.W, sp.C, sp.P,
                           sp.Q, sp.stride, sp.pad, region, bw=bw, reduce=not defer)
            if defer:
                m.dw_pending.append((region, gw, sp.C, nblk))
            return bw is not None
        self._wgrad(m, u, dy, x)
        if u.depthwise:
            if dx is None:
                return False
            assert not accumulate
            if bw is not None and (not self.fuse_bn_bwd or bw.get('y2') is not None):
                bw = None
            ops.dwconv_dgrad(dy, self._pview(u.w_seg), dx, sp.N, sp.H, sp.W, sp.C, sp.P,
                             sp.Q, sp.stride, sp.pad, bw=bw)
            return bw is not None
        if dx is not None:
            if bw is not None and (sp.Cp != sp.C or not self.fuse_bn_bwd):
                bw = None
            ops.conv_dgrad(dy, self.w_crsk[u.name], dx, sp, slab=m.slab,
                           plan=m.plan[u.name, 'dgrad'], accumulate=accumulate, bw=bw)
            return bw is not None
        return False

    def _bwd_sc_ok(self, m, u, sc):
        """Can the shortcut ``sc``'s backward share one launch with ``u``'s (ops.conv_bwd_sc)?"""
        if not self.opts.dual_bwd or not self.pair_bwd or u.depthwise or sc.depthwise:
            return False
        su, ss = m.spec[u.name], m.spec[sc.name]
        if su.stride != 1 or su.K % 8 or ss.K % 8 or not ops.conv.dgrad_s2_ok(ss) or ss.N > 32:
            return False
        return (tuple(m.plan[u.name, 'dgrad'][:2]) == (64, 64) and
                tuple(m.plan[u.name, 'wgrad'][:2]) in ((64, 64), (128, 128)) and
                tuple(m.plan[sc.name, 'wgrad'][:2]) == (64, 64))

    def _conv_bwd_sc(self, m, u, dy, x, dx, bw, sc, xs, dxs):
        """``u``'s dgrad + wgrad (dx, fused BN-backward sums ``bw``) and the shortcut ``sc``'s
        (input ``xs``, writes ``dxs``) in one launch; two launches when the pair does not fit.
        Returns whether ``bw`` was reduced (as _conv_bwd)."""
        sp = m.spec[u.name]
        if bw is not None and (sp.Cp != sp.C or not self.fuse_bn_bwd):
            bw = None
        a = dict(dy=dy, wt=self.w_crsk[u.name], dx=dx, x=x, dw=self._pview(u.w_seg, grad=True),
                 spec=sp, dplan=m.plan[u.name, 'dgrad'], wplan=m.plan[u.name, 'wgrad'],
                 slab=m.slab, accumulate=False, bw=bw)
        b = dict(dy=m.buf[sc.name, 'dy'], wt=self.w_crsk[sc.name], dx=dxs, x=xs,
                 dw=self._pview(sc.w_seg, grad=True), spec=m.spec[sc.name],
                 wplan=m.plan[sc.name, 'wgrad'], accumulate=False)
        if ops.conv.conv_bwd_sc(a, b):
            return bw is not None
        self._conv_bwd(m, sc, m.buf[sc.name, 'dy'], xs, dxs, accumulate=False)
        return self._conv_bwd(m, u, dy, x, dx, accumulate=False, bw=bw)

    def _bw(self, m, u, out, act, unit2=None):
        """Fused-reduce descriptor for the BN of ``u`` (+ shortcut BN ``unit2``) whose activation
        output is ``out`` -- consumed by conv_dgrad(bw=...)."""
        d = dict(out=out, y=m.buf[u.name, 'y'], stats=m.stats[u.name], sums=m.buf[u.name, 'sums'],
                 act=act, eps=BN_EPS)
        if unit2 is not None:
            d.update(y2=m.buf[unit2.name, 'y'], stats2=m.stats[unit2.name])
        return d

    def _bn_bwd(self, m, u, dout, out, act, dy, unit2=None, dy2=None, dz=None, reduce=True):
        sp = m.spec[u.name]
        kw = {}
        if unit2 is not None:
            kw = dict(y2=m.buf[unit2.name, 'y'], stats2=m.stats[unit2.name],
                      gamma2=self._gamma(unit2), dy2=dy2, dgamma2=self._gamma(unit2, True),
                      dbeta2=self._beta(unit2, True))
        ops.bn_bwd(dout, out, m.buf[u.name, 'y'], m.stats[u.name], self._gamma(u),
                   m.buf[u.name, 'sums'], dy, sp.M, u.K, act=act, eps=BN_EPS, dz=dz,
                   dgamma=self._gamma(u, True), dbeta=self._beta(u, True), zero_sums=False,
                   reduce=reduce, **kw)

    def backward_block(self, m, bi):
        for _, f in self.backward_parts(m, bi):
            f()
        if bi == 0:                      # the backward is complete: deferred reduces
            self.flush_dw_reduces(m)

    def backward_parts(self, m, bi):
        """Block ``bi``'s backward as [(unit index, callable)] in execution order (last unit
        first): after part i, the gradients of units i..last, of the BNs of units i-1..last
        and of the shortcut are final -- so a gradient bucket may close between parts."""
        blk = self.lw.blocks[bi]
        x = m.buf[bi - 1, 'out'] if bi > 0 else m.input
        dx = m.buf[bi - 1, 'dout'] if (bi > 0 and blk.need_dx) else None
        units = blk.units
        last = units[-1]
        sc = blk.shortcut

        # the shortcut's backward runs in ONE launch with the last conv's (both start from the
        # block-final BN's backward; EngineOptions.dual_bwd)
        merge = (sc is not None and dx is not None and len(units) > 1 and
                 self._bwd_sc_ok(m, last, sc))

        def top():
            dout = m.buf[bi, 'dout']
            out = m.buf[bi, 'out']
            if blk.pool:
                N, h, w, K, P_, Q_, k, st, pd = m.buf[bi, 'pool_geom']
                ops.maxpool2d_bwd(dout, m.buf[bi, 'argmax'], m.buf[bi, 'dpre'], N, h, w, K, P_,
                                  Q_, k, st, pd)
                dout, out = m.buf[bi, 'dpre'], m.buf[bi, 'pre']
            dz = dx if (blk.identity and dx is not None) else None
            pre = m.prereduced.pop(bi, False) and not blk.pool
            self._bn_bwd(m, last, dout, out, blk.final_act, m.buf[last.name, 'dy'], unit2=sc,
                         dy2=m.buf[sc.name, 'dy'] if sc else None, dz=dz, reduce=not pre)
            if sc is not None and not merge:
                self._conv_bwd(m, sc, m.buf[sc.name, 'dy'], x, dx, accumulate=False)

        def unit(i):
            u = units[i]
            d = m.buf[u.name, 'dy']
            inp = x if i == 0 else m.buf[units[i - 1].name, 'a']
            if i > 0:
                prev = units[i - 1]
                da = m.buf[prev.name, 'da']
                bw = self._bw(m, prev, m.buf[prev.name, 'a'], prev.act)
                if merge and u is last:
                    fused = self._conv_bwd_sc(m, u, d, inp, da, bw, sc, x, dx)
                else:
                    fused = self._conv_bwd(m, u, d, inp, da, accumulate=False, bw=bw)
                self._bn_bwd(m, prev, da, m.buf[prev.name, 'a'], prev.act,
                             m.buf[prev.name, 'dy'], reduce=not fused)
            else:
                acc = blk.identity or sc is not None
                bw = None
                if bi > 0 and dx is not None:
                    # this dgrad is the LAST writer of the previous block's output gradient:
                    # reduce that block's final BN (+ shortcut BN) sums in its epilogue
                    pb = self.lw.blocks[bi - 1]
                    if not pb.pool:
                        bw = self._bw(m, pb.units[-1], m.buf[bi - 1, 'out'], pb.final_act,
                                      unit2=pb.shortcut)
                fused = self._conv_bwd(m, u, d, inp, dx if u.need_dgrad else None,
                                       accumulate=acc, bw=bw)
                if fused:
                    m.prereduced[bi - 1] = True

        parts = []
        for i in range(len(units) - 1, -1, -1):
            if i == len(units) - 1:
                parts.append((i, lambda i=i: (top(), unit(i))))
            else:
                parts.append((i, lambda i=i: unit(i)))
        return parts

    # ------------------------------------------------------------------ data
    def _device_inputs(self, images):
        """uint8 HWC images stay uint8 [N][H][W][3] (augmented on the fly); float inputs
        [N][C][H][W] (e.g. spectrograms) are converted ONCE to NHWC bf16 [N][H][W][8]."""
        x = torch.as_tensor(np.ascontiguousarray(images)) if not torch.is_tensor(images) \
            else images
        if x.dtype == torch.uint8:
            if x.dim() != 4 or tuple(x.shape[1:]) != (self.H, self.W, 3):
                raise ValueError('uint8 shard must be [N][%d][%d][3], got %s'
                                 % (self.H, self.W, tuple(x.shape)))
            return x.to(self.device).contiguous()
        C = self.lw.in_channels
        if x.dim() != 4 or tuple(x.shape[1:]) != (C, self.H, self.W):
            raise ValueError('float shard must be [N][%d][%d][%d], got %s'
                             % (C, self.H, self.W, tuple(x.shape)))
        out = torch.empty(x.shape[0], self.H, self.W, 8, dtype=torch.bfloat16, device=self.device)
        step = 4096
        for s0 in range(0, x.shape[0], step):
            blk = x[s0:s0 + step].to(self.device, torch.float32).contiguous()
            ops.nchw_to_nhwc8(blk, out[s0:s0 + step])
        return out

    def set_shard(self, images, labels):
        """Keep this rank's training shard resident in HBM: uint8 [Ns][H][W][3] images, or
        float [Ns][C][H][W] inputs pre-converted to NHWC bf16."""
        x = self._device_inputs(images)
        if x.shape[0] < 1:
            raise ValueError('empty shard')
        # (a shard smaller than one batch -- possible for a Dirichlet non-IID split at large
        # world size -- is cycled: every batch is the shard's epoch permutation, wrapped)
        self.shard = x
        self.shard_labels = torch.as_tensor(np.asarray(labels), dtype=torch.int64).to(self.device)
        self.train_mode = self.mode('train', self.B, 0, True)
        self.score_mode = self.mode('score', self.P, self.B, False)
        if self.lw.head_pool == 'mlp2':
            self._mlp_setup(self.train_mode)
            self._mlp_setup(self.score_mode)
        self.idx = torch.zeros(self.B, dtype=torch.int32, device=self.device)
        self._arange_b = torch.arange(self.B, dtype=torch.int32, device=self.device)
        self.isw = torch.ones(self.B, dtype=torch.float32, device=self.device)
        if self.global_table:
            # shard-wide importance table resident in HBM: every scored pool sample's latest
            # loss, stamped with the optimizer step that scored it
            self.table = ops.ImportanceTable(self.shard.shape[0], self.device)
        if self.sampler == 'groupwise':
            if self.shard.shape[0] < self.P:
                raise ValueError("sampler='groupwise' needs a shard of at least one pool "
                                 '(%d samples)' % self.P)
            self._draw_pos = torch.zeros(self.B, dtype=torch.int32, device=self.device)
            self._gstamp = torch.zeros(1, dtype=torch.int64, device=self.device)
        self._build_bn_table()

    def _build_bn_table(self):
        """Running-stat update table: the train batch, then (importance mode) the 10 scored
        pool batches, each a train-mode forward in the reference.  The uniform baseline
        scores nothing, so its table updates from the train batch only."""
        tables = []
        tm, sm = self.train_mode, self.score_mode
        for n_score in (sm.G, 0):
            rows = []
            for u in self.units:
                sp_t, sp_s = tm.spec[u.name], sm.spec[u.name]
                rows.append((u.bn.running_mean, u.bn.running_var, tm.stats[u.name],
                             sm.stats[u.name], u.bn.num_batches_tracked, u.K, 1, n_score,
                             float(sp_t.M), float(sp_s.group_rows or sp_s.M)))
            tables.append(ops.BnRunTable(rows, self.device))
        self.bn_table, self.bn_table_uniform = tables

    # ------------------------------------------------------------------ step pieces
    def score_branch(self):
        self.score_forward()
        if not self._split_score:
            self.score_sample()

    def score_forward(self):
        sm = self.score_mode
        if not self.scoring:
            # uniform-sampling baseline: the next batch is the next 32 shard samples
            # (epoch-shuffled, augmented), no pool forward, unit weights
            ops.pool_build(self.shard, self.shard_labels, self.ctrl, sm.input, sm.label,
                           sm.index, self.B, self.B, self.seed)
            self.ctrl[0:1].add_(1)
            self.idx.copy_(self._arange_b)
            self.isw.fill_(1.0)
            return
        # groupwise (Groupwise_Sampler, `util.py:114-138`): the pool is the next CONTIGUOUS slice
        # of the shard (cursor order, wrapping), which becomes this iteration's group.
        # Deviation (parity unpinned: no reference fixture covers it): when Ns % P != 0 the
        # slice that reaches the end of the shard wraps to its head and stays a full P-sample
        # group, where the reference truncates it at len(dataset) (a short group) and resets
        # the cursor.  Group sizes stay P, so the table weights need no short-group handling.
        ops.pool_build(self.shard, self.shard_labels, self.ctrl, sm.input, sm.label, sm.index,
                       self.P, self.B, self.seed, zero=sm.stats_arena,
                       shuffle=self.sampler != 'groupwise')
        # (the scoring convs keep their full occupancy: reserving extra LDS per scoring block
        # so train blocks fit beside them measured 1.70-2.21 ms/step vs 1.65 -- in the
        # concurrent step the GPU is throughput-bound, bench/ab_env.sh)
        x = self.forward(sm)
        self.head(sm, x, 'score')
        if self.table is not None:
            if self.sampler == 'groupwise':
                # a new group per scored slice (never 0: group 0 is the initial uniform table)
                torch.add(self.ctrl[0:1], 1, out=self._gstamp)
                self.table.scatter(sm.index, sm.losses, stamp=self._gstamp)
            else:
                self.table.scatter(sm.index, sm.losses, stamp=self.ctrl[2:3])

    def score_sample(self):
        if not self.scoring:
            return
        sm = self.score_mode
        if self.sampler == 'groupwise':
            # draw from the global HBM table over the current group (the slice just scattered,
            # stamped with this step's counter): p ~ imp + mean(imp) (`util.py:144-152`), then
            # pool slots + unbiased weights n_group * p
            self.table.draw_batch(self.B, self._gstamp, self._draw_pos, sm.index,
                                  self.shard.shape[0], self.P, self.idx, self.isw, seed=self.seed,
                                  meters=self.meters)
            self.ctrl[0:2].add_(1)       # pool and draw counters (is_sample bumps them otherwise)
            return
        gathered = self.score_exchange.gathered if self._split_score else None
        ops.is_sample(sm.losses, self.ema, self.ctrl, self.idx, self.isw, self.P, self.B, self.B,
                      self.alpha, self.ema_alpha, self.seed, self.importance, self.meters,
                      alias=self.sampler == 'alias', gathered=gathered)

    @property
    def _split_score(self):
        # global EMA: the all-gather of every rank's pool scores sits between the scoring
        # forward and the draw, so the score stream runs as two graphs around the collective
        return self.global_ema and self.score_exchange is not None and self.scoring

    def _score_stream_work(self, graphs):
        """Everything on the score stream for one step (caller sets the stream)."""
        if graphs:
            graphs['score'].replay()
        else:
            self.score_forward() if self._split_score else self.score_branch()
        if self.score_exchange is not None and self.scoring:
            # cross-worker importance-score all-gather, issued on the score stream
            # right after scoring; RCCL runs it beside the train backward
            cs = torch.cuda.current_stream(self.device)
            self.timer.mark('xchg0', cs)
            self.score_exchange.start(self.score_mode.losses)
            self.timer.mark('xchg1', cs)
        if self._split_score:
            self.score_exchange.wait()          # stream-side wait on RCCL
            if graphs:
                graphs['score_sample'].replay()
            else:
                self.score_sample()

    def gather_batch(self):
        sm, tm = self.score_mode, self.train_mode
        ops.gather(sm.input, sm.label, sm.index, self.idx, tm.input, tm.label, tm.index, self.B)

    def train_segments(self):
        """Train fwd + backward as a list of callables; bucket all-reduces go between them."""
        tm = self.train_mode
        segs = []

        def fwd_head():
            tm.dw_pending = []
            ops.lib().step_begin(ops.ptr(self.ctrl), ops.stream_ptr(), ops.ptr(tm.stats_arena),
                                 tm.stats_arena.numel(), ops.ptr(tm.sums_arena),
                                 tm.sums_arena.numel())
            x = self.forward(tm)
            self.head(tm, x, 'train', isw=self.isw, meters=self.meters)
            last = len(self.lw.blocks) - 1
            if self.lw.head_pool == 'mlp2':
                self._mlp_head_bwd(tm, tm.buf[last, 'dout'])
                return
            # the head's backward also reduces the final BN's backward sums (no bn_bwd reduce
            # pass at the top of the last block) where its per-sample path runs
            lb = self.lw.blocks[last]
            bw = None
            if self.head_bw and self.fuse_bn_bwd and not lb.pool:
                bw = self._bw(tm, lb.units[-1], tm.buf[last, 'out'], lb.final_act,
                              unit2=lb.shortcut)
            if ops.head_bwd(tm.pooled, tm.dlogits, self._pview(self.lw.fc_w),
                            self._pview(self.lw.fc_w, True), self._pview(self.lw.fc_b, True),
                            tm.buf[last, 'dout'], self.B, tm.final_hw, tm.final_C,
                            self.classes, bw=bw):
                tm.prereduced[last] = True
        cuts = self.bucket_plan()
        dw = any(u.depthwise for u in self.units)
        cur = [fwd_head]
        for bi in range(len(self.lw.blocks) - 1, -1, -1):
            for i, f in self.backward_parts(tm, bi):
                cur.append(f)
                if (bi, i) in cuts:
                    if dw:
                        # the bucket's depthwise weight gradients are complete before it
                        # all-reduces (a no-op when none is pending)
                        cur.append(lambda: self.flush_dw_reduces(tm))
                    segs.append((cur, cuts[bi, i]))
                    cur = []
        if cur:
            segs.append((cur, None))
        if dw:
            segs[-1][0].append(lambda: self.flush_dw_reduces(tm))
        if self.check_order:
            # every train segment ticks o[2]; the comm stream checks it before reducing
            for fs, _ in segs:
                fs.append(lambda: self._order(tick=2, at=1))
        return segs

    def _block_starts(self):
        starts = []
        for bi, blk in enumerate(self.lw.blocks):
            us = blk.units + ([blk.shortcut] if blk.shortcut else [])
            starts.append(min(min(s.off for s in (u.w_seg, u.g_seg, u.beta_seg)) for u in us))
        return starts

    def bucket_plan(self):
        """{(block, unit index): (flat_start, flat_end)} -- a bucket closes after that unit's
        backward part (backward_parts) once it holds >= ``bucket_bytes`` of gradient, and
        always after block 0's first unit.  Parameters are laid out in forward order, so the
        backward finishes them from the end of the flat buffer; cutting inside a block (not
        only at block boundaries) lets the first all-reduce start one conv earlier.  A block
        whose shortcut parameters precede its last unit's is cut only at its boundary."""
        if not self.dp:
            return {}
        if getattr(self, '_bucket_plan', None) is not None:
            return self._bucket_plan       # static: cached once (the issue loop reads it)
        starts = self._block_starts()
        cuts = {}
        end = self.lw.total
        # the last bucket: blocks 0 .. kl - 1, the largest leading run within last_bucket_bytes
        # (a cut at block kl's start is forced; 0: no forced cut)
        kl = 0
        for k in range(1, len(starts) if self.last_bucket_bytes > 0 else 1):
            if starts[k] * 4 > self.last_bucket_bytes:
                break
            kl = k
        for bi in range(len(self.lw.blocks) - 1, -1, -1):
            blk = self.lw.blocks[bi]
            ustart = [min(s.off for s in (u.w_seg, u.g_seg, u.beta_seg)) for u in blk.units]
            inner = blk.shortcut is None or min(
                s.off for s in (blk.shortcut.w_seg, blk.shortcut.g_seg,
                                blk.shortcut.beta_seg)) >= ustart[-1]
            inner = inner and all(ustart[i] < ustart[i + 1] for i in range(len(ustart) - 1))
            for i in range(len(blk.units) - 1, -1, -1):
                if i > 0 and not inner:
                    continue
                start = starts[bi] if i == 0 else ustart[i]
                if (bi == 0 and i == 0) or (end - start) * 4 >= self.bucket_bytes or (
                        bi == kl and i == 0 and kl > 0 and end > start):
                    cuts[bi, i] = (0 if (bi == 0 and i == 0) else start, end)
                    end = start
        self._bucket_plan = cuts
        return cuts

    def tail(self):
        if self.check_order:
            # the tail consumes the scoring stream's draw and (DP) every reduced bucket: both
            # must have finished this step -- o[0] / o[1] == steps completed + 1
            self._order(slot=0, ref=3, mult=1, add=1, at=3)
            if self.dp:
                self._order(slot=1, ref=3, mult=1, add=1, at=4)
            self._order(tick=3, at=5)
        (self.bn_table if self.scoring else self.bn_table_uniform).launch(0.1)
        self.opt.step(self.ctrl[2:3])
        self.gather_batch()

    def _order(self, slot=-1, ref=0, mult=0, add=0, ge=False, tick=-1, at=0):
        ops.lib().order_check(ops.ptr(self.order), slot, ref, mult, add, int(ge), tick, at,
                              ops.stream_ptr())

    def order_violations(self):
        """(count, first violation record) of the stream-order checks (``check_order``)."""
        o = self.order.tolist()
        return o[4], dict(slot=o[8], seen=o[9], want=o[10], at=o[11]) if o[4] else None

    # ------------------------------------------------------------------ graphs
    def _capture(self, fn, stream, keep=False):
        """Capture ``fn`` on ``stream`` in THREAD-LOCAL mode.  The default global mode forbids
        "unsafe" HIP calls on every thread of the process while a capture is open; the
        ProcessGroupNCCL watchdog thread polls its works' events every ~100 ms, and a poll that
        lands inside a global capture fails and aborts the process from that native thread (the
        round-4 driver suite abort).  Thread-local mode confines the restriction to this
        thread; build_graphs additionally quiesces the process before capturing."""
        g = torch.cuda.CUDAGraph(keep_graph=keep)
        with torch.cuda.graph(g, stream=stream, capture_error_mode='thread_local'):
            fn()
        if keep:
            g.instantiate()
        return g

    def _quiesce(self):
        """Nothing of this process may run a HIP call into an open capture: drain the device,
        the score exchange and every ProcessGroup work this engine issued, then run the
        collector NOW (finalizers of dead engines -- torch graphs, queued HIP objects -- execute
        here, not inside a capture) and release what dead engines queued."""
        torch.cuda.synchronize(self.device)
        if self.score_exchange is not None:
            self.score_exchange.wait()
        works, self._pg_works = self._pg_works, []
        if works and dist.is_initialized():      # (a destroyed group's works are moot)
            for w in works:
                w.wait()
        torch.cuda.synchronize(self.device)
        gc.collect()
        _release_queued()

    def build_graphs(self):
        self._check_open()
        self._quiesce()
        # no collector pass (and so no finalizer HIP call) while a capture is open
        gc_on = gc.isenabled()
        gc.disable()
        try:
            self._build_graphs()
        finally:
            if gc_on:
                gc.enable()

    def _build_graphs(self):
        self._apply_globals()
        cap = torch.cuda.Stream(self.device)
        segs = self.train_segments()
        comm_ev = (self.dp and self.s_comm is not None
                   and self.opts.comm_events and len(segs) > 1)
        if self._train_exec and not comm_ev:
            ops.lib().graph_exec_destroy(self._train_exec)
            self._train_exec = 0
        self.graphs = {
            'score': self._capture(self.score_forward if self._split_score else self.score_branch,
                                   cap),
            'train': [(self._capture(lambda fs=fs: [f() for f in fs], cap, keep=comm_ev), b)
                      for fs, b in segs],
            'tail': self._capture(self.tail, cap),
        }
        if self._split_score:
            self.graphs['score_sample'] = self._capture(self.score_sample, cap)
        if comm_ev:
            # ONE linear executable graph: the segment graphs as child nodes, an event-record
            # node after each bucket's segment; each bucket's host-issued all-reduce on the comm
            # stream waits on its node of this replay (segmented replays cost ~33 us per extra
            # segment at W = 1).  The segment graphs stay for the timed (phase-marked) path.
            L = ops.lib()
            if not self._bucket_evs:
                self._bucket_evs = [L.ext_event_create() for _, b in segs if b is not None]
            evs, k = [], 0
            for _, b in segs:
                evs.append(self._bucket_evs[k] if b is not None else 0)
                k += b is not None
            if self._train_exec:
                L.graph_exec_destroy(self._train_exec)
            self._train_exec = L.graph_chain(
                [g.raw_cuda_graph() for g, _ in self.graphs['train']], evs)
        self._graph_scoring = self.scoring
        torch.cuda.synchronize(self.device)

    def close(self):
        """Release everything this engine owns that is not plain device memory, in a fixed
        order, now: drain the device and outstanding collectives, drop the torch graphs
        (their executables and private pools), destroy the chained DP executable and its
        events, unmap / free the xGMI exchange buffers.  Idempotent; the engine cannot step
        afterwards.  The shared RCCL communicator is left to ``RcclComm.close`` (other engines
        of the process use it)."""
        if getattr(self, '_closed', True):
            return
        self._quiesce()
        if self.graphs:
            for v in self.graphs.values():
                for g in (v if isinstance(v, list) else [v]):
                    g = g[0] if isinstance(g, tuple) else g
                    g.reset()
        self.graphs = None
        L = ops.lib()
        if self._train_exec:
            L.graph_exec_destroy(self._train_exec)
            self._train_exec = 0
        for e in self._bucket_evs:
            L.ext_event_destroy(e)
        self._bucket_evs = []
        self.score_exchange = None
        torch.cuda.synchronize(self.device)
        self._closed = True
        LIVE.discard(self)
        x, self.xgmi = self.xgmi, None
        if x is not None:
            x.close()                    # collective at W > 1; raises XgmiTimeout last

    def _check_open(self):
        if self._closed:
            raise RuntimeError('NativeEngine was closed')

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def __del__(self):
        # an engine that was never closed: its chained DP executable and events are HIP objects
        # of the extension, not torch's.  No HIP call here (a collection can run at any point):
        # they are queued and released by the next _quiesce, after a device synchronisation
        try:
            if getattr(self, '_closed', True):
                return
            ex, evs = getattr(self, '_train_exec', 0), getattr(self, '_bucket_evs', ())
            if ex or evs:
                _RELEASE.append((ex, list(evs)))
        except Exception:       # interpreter shutdown
            pass

    def prime(self):
        """Score a first pool and gather the first training batch (reference `train()` entry)."""
        self._check_open()
        self._apply_globals()
        s0 = torch.cuda.current_stream(self.device)
        self.s_score.wait_stream(s0)
        with torch.cuda.stream(self.s_score):
            self._score_stream_work(None)
        s0.wait_stream(self.s_score)
        self.gather_batch()
        self.primed = True

    def step(self):
        """One importance-sampled DP step (all async; nothing syncs the host unless ``debug``).

        Streams: the scoring stream (next pool) and the train stream (this batch) start
        together; after each bucket segment of the backward the comm stream all-reduces that
        bucket (RCCL, AVG) while later segments and the scoring keep computing; the tail on the
        train stream waits for the scoring stream and the last bucket."""
        if self._closed:
            raise RuntimeError('NativeEngine was closed')
        s0 = torch.cuda.current_stream(self.device)
        graphs = self.graphs if self.use_graphs else None
        if not graphs:
            self._apply_globals()            # eager launches read the launcher globals
        if graphs and self._graph_scoring != self.scoring:
            raise RuntimeError('scoring was toggled after build_graphs(); rebuild the graphs')
        T = self.timer
        T.begin_step()
        T.mark('start', s0)
        rx = self.roctx
        debug = self.debug
        if rx:
            prof.push('score')
        if debug:
            # serialised: scoring first, on the train stream, checked before training starts
            self._score_stream_work(None)
            if self.check_order:
                self._order(tick=0, at=0)
            self._debug_sync('score')
        else:
            ev_start = torch.cuda.Event()
            ev_start.record(s0)
            self.s_score.wait_event(ev_start)
            with torch.cuda.stream(self.s_score):
                T.mark('score0', self.s_score)
                self._score_stream_work(graphs)
                if self.check_order:
                    self._order(tick=0, at=0)
                T.mark('score1', self.s_score)
        if rx:
            prof.pop()
            prof.push('train')
        works = []
        segs = graphs['train'] if graphs else self.train_segments()
        nb = 0
        if graphs and self._train_exec and not T.on and not debug:
            # one train replay; each bucket's all-reduce waits on its event node in it
            ops.lib().graph_launch(self._train_exec, s0.cuda_stream)
            for si, (_, bucket) in enumerate(segs):
                if bucket is not None:
                    works.append(self._reduce_bucket(s0, bucket, nb, si,
                                                     ev=self._bucket_evs[nb]))
                    nb += 1
            segs = []
        for si, (g, bucket) in enumerate(segs):
            if graphs:
                g.replay()
            else:
                for f in g:
                    f()
            if debug:
                self._debug_sync('train segment %d' % si)
            if bucket is not None and self.dp:
                works.append(self._reduce_bucket(s0, bucket, nb, si))
                nb += 1
        T.mark('train1', s0)
        if rx:
            prof.pop()
            prof.push('allreduce')
        if self.s_comm is not None and nb:
            if self.check_order:
                with torch.cuda.stream(self.s_comm):
                    self._order(tick=1, at=2)
            ev_c = torch.cuda.Event()
            ev_c.record(self.s_comm)
            s0.wait_event(ev_c)
        for wk in works:
            if wk is not None:
                self._finish_work(wk)
                if self.check_order and wk is works[-1]:
                    self._order(tick=1, at=2)
        # (kept until the next step / quiesce: drained before any capture)
        self._pg_works = [wk[0] for wk in works if wk is not None]
        if debug and self.dp:
            self._debug_sync('allreduce')
        if not debug:
            ev_score = torch.cuda.Event()
            ev_score.record(self.s_score)
            s0.wait_event(ev_score)
        if rx:
            prof.pop()
            prof.push('tail')
        T.mark('tail0', s0)
        if self.grad_probe is not None and self.dp:
            self.grad_probe('post', None, self.opt.g)
        if graphs:
            graphs['tail'].replay()
        else:
            self.tail()
        T.mark('end', s0)
        if debug:
            self._debug_sync('tail')
        if rx:
            prof.pop()

    def _reduce_bucket(self, s0, bucket, i, si, ev=None):
        """Issue bucket ``i``'s gradient all-reduce behind train segment ``si`` (or behind
        ``ev``, that segment's event node in the one-graph train replay)."""
        s, e = bucket
        g = self.opt.g[s:e]
        if self.tern is not None:
            self._tern_ctr += 1          # a fresh Philox stream per (step, bucket) (host path)
        if self.s_comm is None:          # torch ProcessGroup (gloo / CPU tests)
            if self.grad_probe is not None:
                self.grad_probe('pre', i, g)
            if self.tern is not None:
                self.tern.allreduce(g, self._tern_ctr)
                return None
            return [dist.all_reduce(g, op=self._avg_op, async_op=True), s, e, False]
        if ev is None:
            ev = torch.cuda.Event()
            ev.record(s0)
            self.s_comm.wait_event(ev)
        else:
            ops.lib().ext_event_wait(self.s_comm.cuda_stream, ev)
        with torch.cuda.stream(self.s_comm):
            if self.check_order:
                # the bucket's gradients are final: train segment si has ticked this step
                self._order(slot=2, ref=3, mult=self._nseg, add=si + 1, ge=True, at=6)
            self.timer.bucket(i, 0, self.s_comm)
            if self.grad_probe is not None:
                self.grad_probe('pre', i, g)
            if self.xgmi is not None:
                # direct two-shot over xGMI (all peers' exchange buffers mapped by IPC, device
                # flag barriers); consecutive buckets alternate the two exchange slots; the bf16
                # wire option lives in the exchange buffers
                self.xgmi.allreduce(g, avg=True, slot=i % 2)
                if i == len(self.bucket_plan()) - 1:
                    self.xgmi.end_step(i + 1)
            elif self.tern is not None:
                # 2-bit stochastic ternary codes + one scale per rank, all-gathered (1/16 of
                # the fp32 bytes), decoded to the same mean on every rank; Philox stream =
                # (device optimizer-step counter, bucket): fresh every replayed step
                self.tern.allreduce(g, i, dctr=self.ctrl[2:3])
            elif self.comm.size == 1 and not self.opts.rccl_one_rank:
                # one rank (forced buckets): the AVG is the identity -- the bucket plan, the
                # event waits and the comm stream run as at W > 1, RCCL's one-rank copy kernel
                # does not (EngineOptions.rccl_one_rank issues it: the tests)
                pass
            elif self.wire_bf16:
                # bf16 on the wire: half the bytes over xGMI; the sum is rounded once per hop
                if self.wire is None:
                    self.wire = torch.empty(self.lw.total, dtype=torch.bfloat16,
                                            device=self.device)
                w = self.wire[s:e]
                w.copy_(g)
                self.comm.allreduce(w, avg=True)
                g.copy_(w)
            else:
                self.comm.allreduce(g, avg=True)
            self.timer.bucket(i, 1, self.s_comm)
        return None

    @property
    def _nseg(self):
        plan = self.bucket_plan()
        return len(plan) + (0 if (0, 0) in plan else 1)

    def _debug_sync(self, what):
        """Debug mode: drain the device after every phase so a fault names its phase."""
        try:
            torch.cuda.synchronize(self.device)
        except RuntimeError as e:
            raise RuntimeError('device error after %s: %s' % (what, e)) from e
        if self.check_order:
            n, first = self.order_violations()
            if n:
                raise RuntimeError('stream-order violation after %s: %s' % (what, first))
        if self.debug_log:
            print('[mercury_amd debug] step phase done: %s' % what, flush=True)

    def _finish_work(self, wk):
        """Make the current stream wait for a bucket all-reduce (once per stream is harmless;
        the gloo SUM -> mean scaling runs once)."""
        w, s, e, done = wk
        w.wait()
        if not done and self._avg_op != dist.ReduceOp.AVG:   # gloo has no AVG
            self.opt.g[s:e].mul_(1.0 / self.world_size)
        wk[3] = True

    # ------------------------------------------------------------------ misc API
    def reset_ema(self):
        self.ema.zero_()

    def broadcast_from(self, src=0):
        """Initial replica sync (reference `pytorch_collab.py:84-87` averages parameters only;
        this broadcasts parameters AND BN running stats from ``src``).  On the engine's own
        RCCL communicator when it has one (stream-ordered, no ProcessGroup work left in flight
        for a later graph capture), else the ProcessGroup, drained before returning."""
        self._check_open()
        bufs = [self.opt.p]
        seen = set()
        for u in self.units:
            for b in (u.bn.running_mean, u.bn.running_var):
                if id(b) not in seen:
                    seen.add(id(b))
                    bufs.append(b)
        if self.comm is not None:
            for b in bufs:
                self.comm.broadcast(b, src)
        else:
            works = [dist.broadcast(b, src, async_op=True) for b in bufs]
            for w in works:
                w.wait()
            torch.cuda.synchronize(self.device)
        self.opt.pack_weights()

    @torch.no_grad()
    def evaluate_arrays(self, images, labels, batch=500):
        """Eval-mode (running-stats BN) loss / accuracy over uint8 HWC images (or float NCHW
        inputs) on device."""
        imgs = self._device_inputs(images)
        labs = torch.as_tensor(np.asarray(labels), dtype=torch.int64).to(self.device)
        n = imgs.shape[0]
        self.eval_meters.zero_()
        ctrl = torch.zeros(8, dtype=torch.int64, device=self.device)
        done = 0
        while done < n:
            b = min(batch, n - done)
            m = self.mode('eval%d' % b, b, 0, False)
            ops.pool_build(imgs[done:done + b], labs[done:done + b], ctrl, m.input, m.label,
                           m.index, b, b, self.seed, augment=False, shuffle=False)
            x = self.forward(m)
            self.head(m, x, 'eval', meters=self.eval_meters)
            done += b
        r = self.eval_meters[:3].tolist()
        return r[0] / max(r[1], 1), r[2] / max(r[1], 1), int(r[1])

    def global_share(self):
        """Each rank's fraction of total pool importance (needs ``exchange_scores``)."""
        if self.score_exchange is None:
            return torch.ones(1, device=self.device)
        return self.score_exchange.global_share()

    def read_meters(self):
        b = self.meters.tolist()
        if self.xgmi is not None:
            # host-synchronised already: a device barrier that gave up on a peer (its error word)
            # fails loudly here instead of turning into silent replica divergence
            self.xgmi.check()
        return {'loss_sum': b[0], 'count': b[1], 'correct': b[2], 'pool_mean': b[3], 'ema': b[4]}


# ---------------------------------------------------------------------- trainer
def _dataset_arrays(loader):
    ds = getattr(loader, 'dataset', None)
    x = getattr(ds, 'data', None)
    y = getattr(ds, 'target', None)
    if y is None:
        y = getattr(ds, 'targets', None)
    if x is None or y is None:
        raise ValueError('native engine needs a dataset with uint8 HWC .data and .target')
    return np.asarray(x), np.asarray(y)


class NativeTrainer(Trainer):
    """``Trainer`` whose step runs on the native engine (same public API)."""

    def __init__(self, net, optimizer, train_loader, presam_loader, test_loader, device,
                 config=None):
        from ..config import Config
        cfg = config or Config()
        self.cfg = cfg
        self.net = net
        self.optimizer = optimizer
        self.train_loader = train_loader
        self.presam_loader = presam_loader
        self.test_loader = test_loader
        self.device = torch.device(device)
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world_size = dist.get_world_size() if dist.is_initialized() else 1
        self.com_tensor = torch.ones(1)
        self.epoch, self.step, self.writer, self.scheduler = 0, 1, None, None
        self.epoch_step = 0
        self.next_batch_iter = None
        self.computed_samples = {'index': [], 'prob': []}
        self.should_compute_importance = True
        self.batch_size = getattr(train_loader, 'batch_size', None) or cfg.batch_size
        self.steps_per_epoch = len(train_loader) if train_loader is not None else 1
        self.flat = None
        self.bucketer = None
        from ..utils.logging import PhaseTimer
        self.timer = PhaseTimer(self.device)
        # the engine's fused kernel performs the optimizer step; tell the LR scheduler so it
        # does not warn that optimizer.step() was never called
        optimizer._opt_called = True
        osp = ops.optimizer_spec(optimizer)       # raises on anything the kernel cannot run
        x, y = _dataset_arrays(presam_loader)
        self.engine = NativeEngine(
            net, self.device, self.batch_size, cfg.presample_batches, image_hw=x.shape[1:3],
            optimizer=osp['algo'], lr=osp['lr'], betas=osp['betas'], eps=osp['eps'],
            weight_decay=osp['weight_decay'], momentum=osp['momentum'],
            seed=cfg.seed * 1000 + self.rank, alpha=cfg.alpha,
            ema_alpha=cfg.ema_alpha, importance=cfg.importance, world_size=self.world_size,
            bucket_bytes=int(cfg.bucket_mb * (1 << 20)) or None, use_graphs=cfg.use_graphs,
            sampler=cfg.sampler, exchange_scores=cfg.exchange_scores,
            score=cfg.score, global_ema=cfg.global_ema, wire_bf16=cfg.wire_bf16,
            grad_compress=cfg.grad_compress,
            comm=cfg.comm, debug=cfg.debug, check_order=cfg.check_order,
            force_buckets=cfg.force_buckets)
        self.engine.set_shard(x, y)
        self.engine.roctx = cfg.roctx
        from ..utils.profiling import StepWindow
        self.profile_window = StepWindow(cfg.profile_start, cfg.profile_steps)

    def _flat_params(self):
        return self.engine.opt.p

    def average_model(self):
        if self.world_size == 1:
            return
        if self.cfg.parity:
            dist.all_reduce(self.engine.opt.p, op=dist.ReduceOp.SUM)
            self.engine.opt.p /= float(self.world_size)
            self.engine.opt.pack_weights()
        else:
            self.engine.broadcast_from(0)

    def average_gradients(self):
        pass  # bucketed inside engine.step()

    def update_samples(self, ema_loss=None, alpha=None):
        """API-compatible scoring call: returns (weights, data NCHW, label, index, pool_mean).

        The native step scores the next pool inside ``step()``, so this is a read-only view of
        the pending (already scored and drawn) batch; only before the first step does it score
        a pool (``prime``)."""
        e = self.engine
        if not e.primed:
            e.prime()
        sm = e.score_mode
        idx = e.idx.long()
        data = sm.input[idx][..., :3].permute(0, 3, 1, 2).float()
        mean = e.meters[3].clone()
        if ema_loss is not None:
            ema_loss.first_update = False
            ema_loss.value = float(e.ema[0].item())
        return e.isw.clone(), data, sm.label[idx].long(), sm.index[idx].long(), mean

    def _sync_lr(self):
        self.engine.opt.set_lr(self.optimizer.param_groups[0]['lr'])

    def train(self):
        e = self.engine
        running_train_loss = Average()
        presam_ema_loss = EMAverage(self.cfg.ema_alpha)
        runing_train_acc = Accuracy()
        e.reset_ema()                      # reference: fresh EMAverage per epoch (`:121`)
        e.meters[:3].zero_()
        self._sync_lr()
        e.prime()
        t0 = time.perf_counter()
        pe = self.cfg.print_every
        for _ in range(max(0, self.steps_per_epoch - self.epoch_step)):
            # device-phase timing for the steps that are printed (events cost host time)
            e.timer.on = bool(pe) and self.step % pe == 0 and self.rank == 0
            if e.use_graphs and e.graphs is None:
                # the first step runs eagerly (warms every kernel), then the step is captured;
                # it is a real training step and counts like every other one
                e.step()
                e.build_graphs()
            else:
                e.step()
            self._health()
            if self.cfg.print_every and self.step % self.cfg.print_every == 0:
                self._log(t0)
                t0 = time.perf_counter()
            if self.cfg.eval_every and self.step % self.cfg.eval_every == 0 and (
                    self.rank == 0 or self.cfg.eval_all_ranks):
                self._eval_log()
            self._advance()
            if self._stop():
                break
        m = e.read_meters()
        running_train_loss.update(m['loss_sum'] / max(m['count'], 1), max(int(m['count']), 1))
        runing_train_acc.update_counts(m['correct'], int(m['count']))
        presam_ema_loss.update(m['ema'])
        return running_train_loss, runing_train_acc, presam_ema_loss

    def _log(self, t0):
        if self.rank != 0:
            return
        m = self.engine.read_meters()
        cnt = max(m['count'], 1)
        ph = self.engine.timer.collect()
        dev = ''
        if ph:
            # reference C27 fields (`pytorch_collab.py:129-178`), from device events: step, IS
            # (scoring stream), ff+bp, sync (all-reduce, and the part not hidden), opt (tail)
            dev = (', device ms: step {step:.3f} (critical path {critical:.3f}), IS {score:.3f}, '
                   'ff+bp {train:.3f}, sync {comm:.3f} (exposed {exp:.3f}), wait {wait:.3f}, '
                   'opt+tail {tail:.3f}, IS share {share:.1f}%').format(
                       exp=ph.get('comm_exposed', 0.0), share=100.0 * ph['score'] / max(
                           ph['score'] + ph['train'], 1e-9), **ph)
        print('step:{}, running train loss: {:.6f}, running train acc: {:.2f}%, '
              'presam_ema_loss: {:.6f}, pool_mean: {:.4f}, {:.3f} ms/step{}'.format(
                  self.step, m['loss_sum'] / cnt, 100 * m['correct'] / cnt, m['ema'],
                  m['pool_mean'], (time.perf_counter() - t0) * 1e3 / self.cfg.print_every, dev),
              flush=True)
        if self.engine.check_order:
            n, first = self.engine.order_violations()
            if n:
                raise RuntimeError('stream-order violation (%d): %s' % (n, first))

    def _eval_log(self):
        train_loss, train_acc, test_loss, test_acc = self.evaluate()
        if self.writer is not None:
            self.writer.add_scalar('train/acc', train_acc.accuracy, self.step)
            self.writer.add_scalar('test/acc', test_acc.accuracy, self.step)
            self.writer.add_scalar('train/loss', train_loss.average, self.step)
            self.writer.add_scalar('test/loss', test_loss.average, self.step)
        if self.rank == 0:
            print('(Eval) Step: {}, train loss: {}, train acc: {} test loss: {}, test acc: {}'
                  .format(self.step, train_loss, train_acc, test_loss, test_acc), flush=True)

    def evaluate(self, max_batches=None):
        out = []
        for loader in (self.train_loader, self.test_loader):
            lm, am = Average(), Accuracy()
            if loader is not None:
                x, y = _dataset_arrays(loader)
                bs = getattr(loader, 'batch_size', 32) or 32
                n = (len(x) // bs) * bs       # drop_last, as the reference loaders
                if max_batches is not None:
                    n = min(n, max_batches * bs)
                loss, acc, cnt = self.engine.evaluate_arrays(x[:n], y[:n])
                lm.update(loss, cnt)
                am.update_counts(acc * cnt, cnt)
            out += [lm, am]
        return out[0], out[1], out[2], out[3]

    def state_dict(self):
        e = self.engine
        e.sync_to_module()
        ost = self.optimizer.state_dict()
        state = {}
        t = int(e.ctrl[2].item())
        for i, s in enumerate(e.lw.segs):
            st = {'step': torch.tensor(float(t)), 'exp_avg': e._to_torch_layout(s, e.opt.m).cpu()}
            if e.opt.algo in (0, 2):
                st['exp_avg_sq'] = e._to_torch_layout(s, e.opt.v).cpu()
            else:
                st = {'momentum_buffer': st['exp_avg']}
            state[i] = st
        ost['state'] = state
        return {'model': {k: v.detach().cpu() for k, v in self.net.state_dict().items()},
                'optimizer': ost,
                'scheduler': self.scheduler.state_dict() if self.scheduler else None,
                'step': self.step, 'epoch': self.epoch, 'epoch_step': self.epoch_step,
                'engine': self._engine_state()}

    def _engine_state(self):
        e = self.engine
        out = {'ctrl': e.ctrl.cpu(), 'ema': e.ema.cpu()}
        if e.table is not None:
            # shard importance table with the Groupwise_Sampler field names (`util.py:106-107`)
            out['importance'] = e.table.importance.cpu()
            out['group_indicator'] = e.table.group.cpu().to(torch.int64)
        return out

    def load_state_dict(self, sd):
        e = self.engine
        self.net.load_state_dict(sd['model'])
        e.load_from_module()
        st = sd['optimizer'].get('state', {})
        for i, s in enumerate(e.lw.segs):
            if i in st:
                if 'exp_avg' in st[i]:
                    e._from_torch_layout(s, e.opt.m, st[i]['exp_avg'])
                if 'exp_avg_sq' in st[i] and e.opt.algo in (0, 2):
                    e._from_torch_layout(s, e.opt.v, st[i]['exp_avg_sq'])
                if 'momentum_buffer' in st[i]:
                    e._from_torch_layout(s, e.opt.m, st[i]['momentum_buffer'])
        if sd.get('scheduler') and self.scheduler is not None:
            self.scheduler.load_state_dict(sd['scheduler'])
        self.optimizer.param_groups[0]['lr'] = sd['optimizer']['param_groups'][0]['lr']
        self.step, self.epoch = sd['step'], sd['epoch']
        self.epoch_step = int(sd.get('epoch_step', 0))
        if 'engine' in sd:
            es = sd['engine']
            if e.table is not None and 'importance' in es:
                n = es['importance'].numel()
                if n != e.table.importance.numel():
                    raise ValueError(
                        'checkpoint importance table has %d entries but this rank\'s shard has '
                        '%d: resume each rank from its own file (Config.resume = a directory of '
                        'ckpt_rank<r>.pt files, or a path with {rank})'
                        % (n, e.table.importance.numel()))
            e.ctrl.copy_(es['ctrl'].to(e.device))
            e.ema.copy_(es['ema'].to(e.device))
            if e.table is not None and 'importance' in es:
                e.table.importance.copy_(es['importance'].to(e.device))
                e.table.group.copy_(es['group_indicator'].to(e.device, torch.int32))


# ---------------------------------------------------------------------- smoke
def smoke_step(device='cuda:0', steps=2):
    """Tiny end-to-end check used by ``__graft_entry__.smoke``."""
    from ..models import ResNet18
    torch.manual_seed(0)
    net = ResNet18(10).to(device)
    eng = NativeEngine(net, device, batch_size=32, pool_batches=10, use_graphs=True)
    rng = np.random.RandomState(0)
    eng.set_shard(rng.randint(0, 256, (640, 32, 32, 3), dtype=np.uint8),
                  rng.randint(0, 10, 640))
    eng.prime()
    eng.step()
    eng.build_graphs()
    for _ in range(steps):
        eng.step()
    torch.cuda.synchronize()
    m = eng.read_meters()
    assert math.isfinite(m['loss_sum']) and m['count'] == 32 * (steps + 1), m
    return m
