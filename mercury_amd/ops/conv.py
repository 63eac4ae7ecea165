"""Convolution front-end: geometry, tile selection and the three MFMA GEMMs.

``ConvSpec`` describes one conv layer at one batch size.  Tile choice targets
the MI355X's 256 CUs: a launch should have >= ~256 workgroups, so small-M
layers (layer3/4 of ResNet-18 at batch 32: M = 2048 / 512 rows) get split-K
(fp32 partial tiles reduced by a fused epilogue kernel) and big-M layers (the
B=320 scoring pass) use 128-row tiles.  Ghost-BN statistics need a tile never
to straddle a 32-image stat group; ``pick_tiles`` enforces that.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from . import _chk, lib, ptr, stream_ptr

CU = 256
WG_SEM_INTS = 1024          # tile counters at the head of a wgrad slab (csrc/wgrad_body.h)


def cpad8(c):
    return (c + 7) // 8 * 8


@dataclass
class ConvSpec:
    N: int
    H: int
    W: int
    C: int          # real input channels
    K: int          # output channels
    R: int
    S: int
    stride: int = 1
    pad: int = 0
    group_rows: int = 0   # rows per BN ghost group in the output (0 = whole batch)

    @property
    def Cp(self):
        return cpad8(self.C)

    @property
    def P(self):
        return (self.H + 2 * self.pad - self.R) // self.stride + 1

    @property
    def Q(self):
        return (self.W + 2 * self.pad - self.S) // self.stride + 1

    @property
    def M(self):
        return self.N * self.P * self.Q

    def flops(self):
        return 2.0 * self.M * self.K * self.R * self.S * self.C


def pick_tiles(M, Ncols, kchunks, group_rows=0, min_blocks=CU):
    """(bm, bn, splits) for the NT implicit GEMM."""
    bn = 64 if Ncols <= 64 else 128
    cands = [128, 64] if bn == 128 else [256, 128, 64]
    # ghost-BN groups need not be tile multiples: the epilogue splits a tile that straddles
    # one group boundary (requires group_rows >= bm)
    grp = group_rows if group_rows and group_rows < M else 0
    bm = None
    for c in cands:
        if grp and grp < c:
            continue
        bm = c
        if math.ceil(M / c) * math.ceil(Ncols / bn) >= min_blocks:
            break
    if bm is None:
        raise ValueError('BN ghost group (%d rows) smaller than every tile' % group_rows)
    blocks = math.ceil(M / bm) * math.ceil(Ncols / bn)
    ktiles = math.ceil(kchunks / 8)
    splits = 1
    if blocks < min_blocks * 3 // 4 and ktiles >= 8:
        splits = min(math.ceil(min_blocks / blocks), max(1, ktiles // 4), 16)
    return bm, bn, splits


SEM_BYTES = 4096   # per-tile split-K arrival counters at the head of a slab (csrc/igemm.hip)


def slab_bytes(M, Ncols, bm, bn, splits):
    """Split-K workspace: tile counters (must start zeroed) + fp32 partial tiles."""
    if splits <= 1:
        return 0
    return SEM_BYTES + splits * math.ceil(M / bm) * math.ceil(Ncols / bn) * bm * bn * 4


def fwd_plan(spec: ConvSpec, min_blocks=CU):
    kchunks = spec.R * spec.S * spec.Cp // 8
    return pick_tiles(spec.M, spec.K, kchunks, spec.group_rows, min_blocks=min_blocks)


def dgrad_plan(spec: ConvSpec):
    """dgrad tiles.  Measured at the train batch (bench/bwd_pair_sweep.py, MI355X): the dgrad
    half of the pair launch is fastest with narrow 64x64 tiles reaching ~2 blocks per CU
    before any K split (e.g. 32x32x64 3x3: 22 us vs 31 us with 128x64 tiles)."""
    kchunks = spec.R * spec.S * cpad8(spec.K) // 8
    M, N = spec.N * spec.H * spec.W, spec.Cp
    ktiles = math.ceil(kchunks / 8)
    tiles = math.ceil(M / 64) * math.ceil(N / 64)
    if tiles <= 2 * CU and ktiles >= 4:
        splits = max(1, min(2 * CU // tiles, ktiles // 4, 16))
        return 64, 64, splits
    return pick_tiles(M, N, kchunks, 0)


# Forward convs that take the BN-apply prologue (``pro``): the prologue adds per-chunk loads and
# VALU to every K stage, so deep-input / narrow-output convs at the train batch want more K
# splits than the plain-conv tuning picked.  MobileNetV2-CIFAR's project convs at B = 32, keyed
# (N, H, C, K) of a 1x1 conv (bench/pro_split_bench.py, graph-timed, profiles/r6/pro_split.jsonl),
# us vs the tuned plain plan: 960->160 @4 12.9 vs 16.4, 960->320 @4 14.9 vs 16.6, 576->160 @4
# 11.5 vs 15.6, 576->96 @8 12.3 vs 15.8, 384->64 @8 10.8 vs 13.1, 384->96 @8 11.2 vs 15.0; the
# narrow-input expansions want different tiles (profiles/r6/pro_split_all.jsonl): 64->96 @8 7.3
# vs 8.3, 32->192 @16 9.6 vs 11.1, 16->96 @32 14.7 vs 16.1
MEASURED_PRO = {
    (32, 4, 960, 160): (64, 64, 6), (32, 4, 960, 320): (64, 128, 6),
    (32, 4, 576, 160): (64, 64, 8), (32, 8, 576, 96): (64, 64, 8),
    (32, 8, 384, 64): (64, 64, 3), (32, 8, 384, 96): (64, 64, 4),
    (32, 8, 64, 96): (64, 64, 1), (32, 16, 32, 192): (128, 64, 1),
    (32, 32, 16, 96): (128, 64, 1),
}


def pro_plan(spec: ConvSpec):
    """The measured plan for this conv when it runs with the input prologue, or None."""
    if spec.R != 1 or spec.S != 1 or spec.H != spec.W or spec.group_rows not in (0, spec.M):
        return None
    return MEASURED_PRO.get((spec.N, spec.H, spec.C, spec.K))


ATOMIC_BUDGET = 1_200_000   # fp32 atomic adds per wgrad launch before splitting stops paying


# ResNet-50/224 train batch (B = 128): measured best atomic-split plans, keyed (N, H_in, C, K,
# R, stride) (bench/r50_bwd_cmp.py --sweep, profiles/r3/r50_bwd_sweep.jsonl).  At these pixel
# counts the wgrad is latency-bound per block: many more splits than the B = 32 atomic budget
# allows pay off (4.37 -> 3.02 ms over the net's wgrads).
MEASURED_WGRAD = {
    (128, 56, 64, 64, 1, 1): (64, 64, 128),   # 30.1 us (default 46.5)
    (128, 56, 256, 64, 1, 1): (64, 128, 128),   # 53.7 us (default 60.3)
    (128, 56, 64, 64, 3, 1): (64, 128, 128),   # 110.2 us (default 142.3)
    (128, 56, 64, 256, 1, 1): (128, 64, 128),   # 53.5 us (default 60.8)
    (128, 56, 256, 128, 1, 1): (128, 128, 128),   # 76.7 us (default 119.5)
    (128, 56, 128, 128, 3, 2): (128, 128, 32),   # 87.7 us (default 137.9)
    (128, 56, 256, 512, 1, 2): (64, 128, 32),   # 71.7 us (default 118.3)
    (128, 28, 512, 128, 1, 1): (128, 128, 64),   # 47.2 us (default 52.0)
    (128, 28, 128, 128, 3, 1): (64, 64, 64),   # 73.6 us (default 134.5)
    (128, 28, 128, 512, 1, 1): (128, 128, 64),   # 46.6 us (default 48.2)
    (128, 28, 512, 256, 1, 1): (64, 128, 32),   # 71.9 us (default 93.1)
    (128, 28, 256, 256, 3, 2): (64, 64, 16),   # 74.4 us (default 129.1)
    (128, 28, 512, 1024, 1, 2): (128, 128, 16),   # 66.9 us (default 117.6)
    (128, 14, 1024, 256, 1, 1): (64, 64, 16),   # 37.6 us (default 48.3)
    (128, 14, 256, 256, 3, 1): (64, 64, 16),   # 73.6 us (default 132.8)
    (128, 14, 256, 1024, 1, 1): (64, 128, 16),   # 39.1 us (default 49.1)
    (128, 14, 1024, 512, 1, 1): (128, 64, 8),   # 58.1 us (default 89.4)
    (128, 14, 512, 512, 3, 2): (64, 64, 4),   # 77.1 us (default 133.8)
    (128, 14, 1024, 2048, 1, 2): (128, 64, 2),   # 62.3 us (default 133.0)
    (128, 7, 2048, 512, 1, 1): (64, 64, 4),   # 37.1 us (default 46.8)
    (128, 7, 512, 512, 3, 1): (64, 64, 4),   # 76.0 us (default 135.6)
    (128, 7, 512, 2048, 1, 1): (64, 128, 4),   # 40.6 us (default 48.5)
}
WG_SPLIT_PIX = 4096          # pixels per split of the large-M heuristic
WG_SPLIT_MAX = 128


def _wgrad_plan_large(spec: ConvSpec):
    """Large pixel counts (>= 32k): splits ~ M / 4096 (a power of two, <= 128), the largest
    tile that still gives >= 256 blocks (fitted on the ResNet-50 sweep: 3.37 ms vs the 3.02
    per-shape optimum and 4.37 for the B = 32 rule)."""
    ncols = spec.R * spec.S * spec.Cp
    s = min(WG_SPLIT_MAX, 2 ** round(math.log2(max(1.0, spec.M / WG_SPLIT_PIX))))
    for bm, bn in ((128, 128), (128, 64), (64, 128), (64, 64)):
        if (bm > 64 and bm > spec.K) or (bn > 64 and bn > ncols):
            continue
        if math.ceil(spec.K / bm) * math.ceil(ncols / bn) * s >= 256:
            return bm, bn, s
    return 64, 64, s


def wgrad_plan(spec: ConvSpec):
    """wgrad tiles + pixel split.  Measured (bench/bwd_pair_sweep.py, MI355X, B=32): ~1 block
    per CU, each K-split covering >= 4 pixel tiles, and at most ~1.2M fp32 atomics per launch
    (layer4 3x3 512->512: split 1 = 22 us vs split 2 = 36 us); 64x64 tiles unless the weight
    gradient itself exceeds that budget (then 128x128, unsplit).  Large pixel counts (the
    ResNet-50 train batch): MEASURED_WGRAD, else _wgrad_plan_large."""
    p = MEASURED_WGRAD.get((spec.N, spec.H, spec.C, spec.K, spec.R, spec.stride))
    if p is not None and spec.H == spec.W:
        return p
    if spec.M >= 32768 and spec.N > 32:
        return _wgrad_plan_large(spec)
    ncols = spec.R * spec.S * spec.Cp
    out = spec.K * ncols                      # fp32 elements each K-split adds atomically
    if out <= ATOMIC_BUDGET:
        bm, bn = 64, 64
    else:
        bm, bn = 128, 128
    blocks = math.ceil(spec.K / bm) * math.ceil(ncols / bn)
    ptiles = math.ceil(spec.M / 64)
    splits = min(int(round(CU / blocks)), ATOMIC_BUDGET // out, ptiles // 4, 64)
    return bm, bn, max(1, splits)


def _slab(slab, need, device):
    if slab is not None and slab.numel() * slab.element_size() >= need:
        return slab
    if slab is None and not torch.cuda.is_current_stream_capturing():
        return torch.zeros((need + 3) // 4, dtype=torch.float32, device=device)
    raise ValueError('split-K slab too small (%d < %d bytes)' % (
        0 if slab is None else slab.numel() * slab.element_size(), need))


def pro_ok(spec: ConvSpec, plan, keep=False):
    """Can this forward conv take the BN-apply prologue (``conv_fwd(pro=...)``)?  Needs the
    register-staged loop, real channels a multiple of 8, ghost-BN groups that are whole tiles,
    and -- to keep the activation -- a stride-1 'same' conv (its centre tap is a bijection)."""
    bm = plan[0]
    if spec.C % 8:
        return False
    # pointwise convs only: a 3x3 conv re-loads every input chunk once per tap, and redoing the
    # normalisation 9x in VALU made the conv 2-2.5x slower than a separate bn_apply pass
    # (bench/pro_bench.py, MI355X: B=320 64->64 3x3 135 us vs 53 + 20 us)
    if spec.R != 1 or spec.S != 1:
        return False
    # every N-tile of the consumer redoes the normalisation of its A rows: worth it for one
    # tile, or a few at train-batch sizes (MobileNetV2 4.33 -> 4.26 ms/step), not for the wide
    # ResNet-50 expansions at large batch (53.6 -> 55.4 ms/step with every 1x1 fused)
    ntn = -(-spec.K // plan[1])
    if ntn > 1 and (ntn > 4 or spec.M > 32768):
        return False
    if spec.group_rows and spec.group_rows < spec.M and spec.group_rows % bm:
        return False
    if keep and not (spec.stride == 1 and spec.R == spec.S and spec.R % 2 == 1
                     and spec.pad == spec.R // 2):
        return False
    return True


def _pro_args(pro, spec):
    """ProParams (csrc/igemm.h) from a dict: the PRODUCER's BN -- stats=[G][2][C] batch sums
    (or rmean/rvar), gamma, beta, act, eps, count (= y pixels per stat group) -- and keep=
    (optional activation output, [N*H*W][C])."""
    for k in ('stats', 'rmean', 'rvar', 'gamma', 'beta'):
        _chk(pro.get(k), torch.float32, 'pro.' + k)
    _chk(pro.get('keep'), torch.bfloat16, 'pro.keep', spec.N * spec.H * spec.W * spec.Cp)
    _chk(pro.get('res'), torch.bfloat16, 'pro.res', spec.N * spec.H * spec.W * spec.Cp)
    if pro.get('stats') is None and pro.get('rmean') is None:
        raise ValueError('pro needs stats or running statistics')
    grp = spec.group_rows if spec.group_rows else spec.M
    return (ptr(pro.get('stats')), ptr(pro.get('rmean')), ptr(pro.get('rvar')), ptr(pro['gamma']),
            ptr(pro['beta']), ptr(pro.get('keep')), grp, 1.0 / float(pro.get('count', 1)),
            float(pro.get('eps', 1e-5)), _ACT[pro.get('act')], (spec.R // 2) * spec.S + spec.S // 2,
            ptr(pro.get('res')))


def conv_fwd(x, w, out, spec: ConvSpec, stats=None, bias=None, slab=None, plan=None,
             accumulate=False, pro=None):
    """out[M][K] = conv(x NHWC, w [K][R][S][Cp]); optional BN-sum epilogue.  ``pro``: x is the
    producer's raw conv output and its BN + activation are applied while loading (see
    ``pro_ok`` / ``_pro_args``)."""
    Cp = spec.Cp
    _chk(x, torch.bfloat16, 'x', spec.N * spec.H * spec.W * Cp)
    _chk(w, torch.bfloat16, 'w', spec.K * spec.R * spec.S * Cp)
    _chk(out, torch.bfloat16, 'out', spec.M * spec.K)
    _chk(stats, torch.float32, 'stats')
    plan = plan or fwd_plan(spec)
    bm, bn, splits = plan[:3]
    if splits > 1:
        slab = _slab(slab, slab_bytes(spec.M, spec.K, bm, bn, splits), x.device)
    grp = spec.group_rows if spec.group_rows else spec.M
    if pro is not None:
        if accumulate or not pro_ok(spec, (bm, bn, splits), keep=pro.get('keep') is not None):
            raise ValueError('BN-apply prologue not supported for this conv/plan')
        lib().igemm_pro(ptr(x), ptr(w), ptr(out), spec.K, ptr(bias), ptr(stats), spec.K, grp,
                        ptr(slab) if splits > 1 else 0, spec.H, spec.W, Cp, spec.P, spec.Q,
                        spec.R, spec.S, spec.stride, spec.pad, spec.R * spec.S * Cp // 8, spec.K,
                        spec.M, bm, bn, splits, stream_ptr(), *_pro_args(pro, spec))
        return out
    lib().igemm(ptr(x), ptr(w), ptr(out), spec.K, ptr(bias), ptr(stats), spec.K, grp,
                int(accumulate), ptr(slab) if splits > 1 else 0,
                spec.H, spec.W, Cp, spec.P, spec.Q, spec.R, spec.S, spec.stride, spec.pad,
                spec.R * spec.S * Cp // 8, spec.K, spec.M, bm, bn, splits, False, stream_ptr(),
                *_NO_BW)
    return out


def _dual_args(x, w, out, spec: ConvSpec, stats, slab, plan):
    _chk(x, torch.bfloat16, 'x', spec.N * spec.H * spec.W * spec.Cp)
    _chk(w, torch.bfloat16, 'w', spec.K * spec.R * spec.S * spec.Cp)
    _chk(out, torch.bfloat16, 'out', spec.M * spec.K)
    _chk(stats, torch.float32, 'stats')
    bm, bn, splits = plan[:3]
    if splits > 1:
        slab = _slab(slab, slab_bytes(spec.M, spec.K, bm, bn, splits), x.device)
    grp = spec.group_rows if spec.group_rows else spec.M
    return [ptr(x), ptr(w), ptr(out), spec.K, ptr(stats), spec.K, grp,
            ptr(slab) if splits > 1 else 0, spec.H, spec.W, spec.Cp, spec.P, spec.Q, spec.R,
            spec.S, spec.stride, spec.pad, spec.R * spec.S * spec.Cp // 8, spec.K, spec.M, splits]


def conv_fwd_dual(a, b):
    """Two independent forward convs (plain input, no bias) in ONE launch (csrc/igemm.hip
    igemm_dual_kernel): ``a`` and ``b`` are dicts x=, w=, out=, spec=, stats=, slab=, plan=
    with the same (bm, bn) tile and distinct slabs when both split K.  Returns False (nothing
    launched) when the pair has no instantiation; the caller then runs conv_fwd twice."""
    pa, pb = a['plan'], b['plan']
    if tuple(pa[:2]) != tuple(pb[:2]):
        return False
    if pa[2] > 1 and pb[2] > 1 and a.get('slab') is b.get('slab'):
        return False
    va = _dual_args(a['x'], a['w'], a['out'], a['spec'], a.get('stats'), a.get('slab'), pa)
    vb = _dual_args(b['x'], b['w'], b['out'], b['spec'], b.get('stats'), b.get('slab'), pb)
    return bool(lib().igemm_dual(va, vb, pa[0], pa[1], stream_ptr()))


PGEMM_BM = 256


def pgemm_ok(spec: ConvSpec):
    """Can the persistent pointwise GEMM (csrc/pgemm.hip) run this conv?  1x1, no padding,
    stride 1 or 2, channel counts multiples of 8, ghost-BN groups of >= one 256-row tile, and
    enough output tiles to fill the GPU (small-M layers stay on igemm's split-K)."""
    if spec.R != 1 or spec.S != 1 or spec.pad != 0 or spec.stride not in (1, 2):
        return False
    if spec.C % 8 or spec.K % 8:
        return False
    if spec.group_rows and spec.group_rows < spec.M and spec.group_rows < PGEMM_BM:
        return False
    # one block per CU walks the tiles: a persistent kernel pays off when every block has
    # several tiles (>= 64k rows); the latency-bound train-batch convs stay on igemm (measured:
    # MobileNetV2 at B = 32, 128 tiles, was slower on pgemm)
    return spec.M >= 65536


def pgemm_plan(spec: ConvSpec):
    """Output-tile width of the pointwise GEMM: the widest of 256 / 128 / 64 that the output
    channels fill (a 256-wide tile reads each activation row once for N <= 256)."""
    if spec.K >= 256:
        return 256
    if spec.K > 64:
        return 128
    return 64


def pgemm_plain_wins(spec: ConvSpec):
    """Plain (no input prologue) pointwise GEMM faster than igemm: measured at the ResNet-50
    scoring batch (profiles/r3/pgemm_cmp_v2.jsonl) on every shape with >= 256 input and
    >= 256 output channels (10-16 %), within noise or slower elsewhere."""
    return spec.C >= 256 and spec.K >= 256


def pgemm_pro_wins(spec: ConvSpec):
    """The input-BN prologue beats a bn_apply pass + igemm when the transformed operand tile is
    used by ONE output tile (N <= 128: each activation element normalised once) and the input is
    wide enough to be memory-bound on the pass it saves (profiles/r3/pgemm_pro_cmp.jsonl:
    ResNet-50 256->64 @56 1105 vs 1323 us, 256->128 1184 vs 1461; it loses where every element
    is re-normalised for 2-4 output tiles, e.g. 1024->512 @14 741 vs 592)."""
    # MobileNetV2's 32x32 expand / project shapes also gained in isolation (24->144 53 vs 73 us)
    # but the persistent kernel beside the latency-bound train stream lost 0.09 ms/step in the
    # engine (profiles/r3/mbv2_pgemm_ab.json): the narrow ones go to pwconv instead
    return spec.K <= 128 and spec.C >= 128


_PG_NO_PRO = (0, 0, 0, 0, 0, 0, 0.0, 0.0, 0, 1, 1, 0, 0, 0, 0, 0, 0)


def _pg_pro_args(pro, spec, x):
    """PgemmPro (csrc/igemm.h) from a dict: the PRODUCER's BN -- stats=[G][2][C] sums (or
    rmean/rvar), gamma, beta, act, eps, count (pixels per stats group), group_rows (input rows
    per group) -- plus res= (identity residual, mode 2), keep= (activation output), coef=
    (fp32 workspace >= G*2*C)."""
    for k in ('stats', 'rmean', 'rvar', 'gamma', 'beta', 'coef'):
        _chk(pro.get(k), torch.float32, 'pro.' + k)
    rows = spec.N * spec.H * spec.W
    _chk(pro.get('keep'), torch.bfloat16, 'pro.keep', rows * spec.Cp)
    _chk(pro.get('res'), torch.bfloat16, 'pro.res', rows * spec.Cp)
    if pro.get('stats') is None and pro.get('rmean') is None:
        raise ValueError('pro needs stats or running statistics')
    grp = int(pro.get('group_rows') or rows)
    G = rows // grp if pro.get('stats') is not None else 1
    if pro['coef'].numel() < G * 2 * spec.Cp:
        raise ValueError('pro.coef workspace too small')
    res, keep = pro.get('res'), pro.get('keep')
    return (2 if res is not None else 1, ptr(pro.get('stats')), ptr(pro.get('rmean')),
            ptr(pro.get('rvar')), ptr(pro['gamma']), ptr(pro['beta']),
            1.0 / float(pro.get('count', 1)), float(pro.get('eps', 1e-5)), _ACT[pro.get('act')],
            grp if G > 1 else max(grp, rows), G, ptr(pro['coef']), ptr(res), ptr(keep),
            0 if res is None else res.numel() * 2, 0 if keep is None else keep.numel() * 2,
            pro['coef'].numel() * 4)


def pgemm_fwd(x, w, out, spec: ConvSpec, stats=None, bn=None, grid=0, pro=None):
    """out[M][K] = conv1x1(x NHWC, w [K][Cp]) on the persistent LDS-DMA GEMM (+ BN sums).
    ``pro``: x is the producer's raw output; its BN + activation (+ identity residual) is
    applied to each operand tile in LDS (see ``_pg_pro_args``)."""
    if not (spec.R == 1 and spec.S == 1 and spec.pad == 0 and spec.stride in (1, 2)):
        raise ValueError('pgemm: 1x1 pad-0 stride-1/2 convs only')
    if pro is not None and spec.stride != 1:
        raise ValueError('pgemm: the input prologue needs a stride-1 conv')
    Cp = spec.Cp
    _chk(x, torch.bfloat16, 'x', spec.N * spec.H * spec.W * Cp)
    _chk(w, torch.bfloat16, 'w', spec.K * Cp)
    _chk(out, torch.bfloat16, 'out', spec.M * spec.K)
    _chk(stats, torch.float32, 'stats')
    grp = spec.group_rows if spec.group_rows else spec.M
    bn = bn or pgemm_plan(spec)
    if pro is not None and bn == 256:
        bn = 128      # the 256-wide tile has no register room for the prologue
    pa = _PG_NO_PRO if pro is None else _pg_pro_args(pro, spec, x)
    ok = lib().pgemm(ptr(x), ptr(w), ptr(out), ptr(stats), spec.M, spec.K, Cp, spec.K, spec.K,
                     grp, x.numel() * 2, w.numel() * 2, out.numel() * 2, spec.H, spec.W, spec.P,
                     spec.Q, spec.stride, bn, int(grid), stream_ptr(), *pa)
    if not ok:
        raise ValueError('pgemm: unsupported shape/tile %s bn=%s' % (spec, bn))
    return out


PWCONV_KMAX = 128


def pwconv_ok(spec: ConvSpec):
    """Narrow-input pointwise conv for the panel-resident kernel (csrc/pwconv.hip): 1x1 stride 1,
    <= 128 input channels (the whole 128-row A panel stays in LDS across every N-tile), ghost-BN
    groups of >= 128 rows."""
    if spec.R != 1 or spec.S != 1 or spec.pad != 0 or spec.stride != 1:
        return False
    if spec.C % 8 or spec.K % 8 or spec.Cp > PWCONV_KMAX:
        return False
    return not (spec.group_rows and spec.group_rows < spec.M and spec.group_rows < 128)


def pwconv_pro_wins(spec: ConvSpec):
    """Panel-resident input-BN prologue (pwconv) over a bn_apply pass + igemm / pgemm's
    per-tile prologue: the expansion convs -- narrow input (<= 128 channels) read and normalised
    once, >= 2x wider output -- at >= 64k rows (profiles/r3/pwconv_cmp_*.jsonl: ResNet-50 64->256
    @56 857 vs 993 us, 128->512 @28 472 vs 610; MobileNetV2 24->144 @32 46 vs 74; the project
    convs 96->24 lost, 54 vs 48)."""
    return pwconv_ok(spec) and spec.K >= 2 * spec.C and spec.M >= 65536


def pwconv_plain_wins(spec: ConvSpec):
    """Plain (no prologue) narrow-input expansion conv on the panel-resident kernel instead of
    igemm: ResNet-50's layer1.0 projection shortcut 64 -> 256 @56 at B = 1280 (write-bound,
    2 GB out), 817 vs 875 us with the statistics epilogue (scratch measurement, round 6)."""
    return pwconv_ok(spec) and spec.K >= 2 * spec.C and spec.M >= 65536


def pwconv_fwd(x, w, out, spec: ConvSpec, stats=None, pro=None):
    """out[M][K] = conv1x1(x, w) with the input panel normalised ONCE in LDS (``pro`` as in
    ``pgemm_fwd``, identity residual excluded) and reused by all output-channel tiles."""
    if not pwconv_ok(spec):
        raise ValueError('pwconv: unsupported conv %s' % (spec,))
    if pro is not None and pro.get('res') is not None:
        raise ValueError('pwconv: no residual prologue')
    Cp = spec.Cp
    _chk(x, torch.bfloat16, 'x', spec.N * spec.H * spec.W * Cp)
    _chk(w, torch.bfloat16, 'w', spec.K * Cp)
    _chk(out, torch.bfloat16, 'out', spec.M * spec.K)
    _chk(stats, torch.float32, 'stats')
    grp = spec.group_rows if spec.group_rows else spec.M
    pa = _PG_NO_PRO if pro is None else _pg_pro_args(pro, spec, x)
    ok = lib().pgemm(ptr(x), ptr(w), ptr(out), ptr(stats), spec.M, spec.K, Cp, spec.K, spec.K,
                     grp, x.numel() * 2, w.numel() * 2, out.numel() * 2, spec.H, spec.W, spec.P,
                     spec.Q, 1, 0, 0, stream_ptr(), *pa)
    if not ok:
        raise ValueError('pwconv: unsupported shape %s' % (spec,))
    return out


def stem_ok(spec: ConvSpec):
    """First-layer conv for the dense-k stem kernel (csrc/stem.hip): <= 4 input channels (input
    and weights padded to 8 in memory), 3x3 stride 1/2 or 7x7 stride 2, 32 or 64 outputs."""
    return (spec.C <= 4 and spec.Cp == 8 and spec.R == spec.S and
            (spec.R, spec.stride) in ((3, 1), (3, 2), (7, 2)) and spec.K in (32, 64))


def stem_fwd(x, w, y, spec: ConvSpec, stats=None, bias=None):
    """y[N][P][Q][K] = conv(x [N][H][W][8], w [K][R][R][8]) (+ bias) with the ghost-BN sums
    ([G][2][K], groups of ``spec.group_rows`` output rows = whole images)."""
    if not stem_ok(spec):
        raise ValueError('stem: unsupported conv %s' % (spec,))
    _chk(x, torch.bfloat16, 'x', spec.N * spec.H * spec.W * 8)
    _chk(w, torch.bfloat16, 'w', spec.K * spec.R * spec.S * 8)
    _chk(y, torch.bfloat16, 'y', spec.M * spec.K)
    _chk(stats, torch.float32, 'stats')
    _chk(bias, torch.float32, 'bias', spec.K)
    pq = spec.P * spec.Q
    grp = spec.group_rows or spec.M
    if grp % pq:
        raise ValueError('stem: BN groups must be whole images')
    ok = lib().stem_fwd(ptr(x), ptr(w), ptr(bias), ptr(y), ptr(stats), spec.N, spec.H, spec.W,
                        spec.K, spec.R, spec.stride, spec.pad, spec.P, spec.Q, grp // pq,
                        stream_ptr())
    if not ok:
        raise ValueError('stem: unsupported conv %s' % (spec,))
    return y


_NO_BW = (0, 0, 0, 0, 0, 0, 0.0, 0.0, 0)
_ACT = {None: 0, 'none': 0, 'relu': 1, 'relu6': 2}


def _bw_args(bw, Mx, Cp):
    """Fused BN-backward reduction of the dgrad output (see EpiParams in csrc/igemm.h).

    ``bw``: dict(out=, y=, stats=, sums=, act=, eps=, [y2=, stats2=]) -- the BN(+shortcut BN)
    + activation whose output gradient this dgrad produces."""
    if bw is None:
        return _NO_BW
    for k in ('out', 'y', 'y2'):
        if bw.get(k) is not None:
            _chk(bw[k], torch.bfloat16, 'bw.' + k, Mx * Cp)
    _chk(bw['sums'], torch.float32, 'bw.sums', int(getattr(lib(), 'SUMS_R', 1)) * 3 * Cp)
    _chk(bw['stats'], torch.float32, 'bw.stats', 2 * Cp)
    return (ptr(bw['out']), ptr(bw['y']), ptr(bw['stats']), ptr(bw.get('y2')),
            ptr(bw.get('stats2')), ptr(bw['sums']), 1.0 / Mx, float(bw.get('eps', 1e-5)),
            _ACT[bw.get('act')])


DGRAD_S2 = True    # EngineOptions.dgrad_s2 (the engine sets it)


def dgrad_s2_ok(spec: ConvSpec):
    """The stride-2 dgrad runs as four parity classes (csrc/igemm.hip dgrad_s2_launch): only
    the taps that reach an input pixel are multiplied (3x3: 9/4 per pixel instead of 9)."""
    return (DGRAD_S2 and spec.stride == 2 and spec.R == spec.S and spec.K % 64 == 0 and
            ((spec.R == 3 and spec.pad == 1) or (spec.R == 1 and spec.pad == 0)))


def dgrad_s2_plan(spec: ConvSpec):
    """Tiles of the class dgrad: the classes hold a quarter of the rows each, so the tile
    choice follows the total row count (one K slice per tile)."""
    M = spec.N * spec.H * spec.W
    N = spec.Cp
    bn = 128 if N >= 128 else 64
    bm = 128 if math.ceil(M / 128) * math.ceil(N / bn) >= 2 * CU else 64
    return bm, bn, 1


def conv_dgrad(dy, wt, dx, spec: ConvSpec, slab=None, plan=None, accumulate=False, bw=None):
    """dx[N*H*W][Cp] = dgrad(dy [M][K], wt [C][R][S][K]).  Stride 1 or 2 (stride 2 as parity
    classes where dgrad_s2_ok; ``plan`` then sizes its tiles).  ``bw``: also reduce the
    BN-backward sums of the (final, post-accumulate) dx in the epilogue."""
    if spec.stride not in (1, 2):
        raise ValueError('dgrad supports stride 1/2')
    if spec.K % 8:
        raise ValueError('dgrad needs K % 8 == 0')
    Cp = spec.Cp
    _chk(dy, torch.bfloat16, 'dy', spec.M * spec.K)
    _chk(wt, torch.bfloat16, 'wt', Cp * spec.R * spec.S * spec.K)
    _chk(dx, torch.bfloat16, 'dx', spec.N * spec.H * spec.W * Cp)
    Mx = spec.N * spec.H * spec.W
    if dgrad_s2_ok(spec):
        bm, bn, _ = plan or dgrad_s2_plan(spec)
        if lib().dgrad_s2(ptr(dy), ptr(wt), ptr(dx), Cp, int(accumulate), spec.P, spec.Q,
                          spec.K, spec.R, spec.S, spec.stride, spec.pad, Cp, bm, bn, spec.H,
                          spec.W, spec.N, stream_ptr(), *_bw_args(bw, Mx, Cp)):
            return dx
    bm, bn, splits = plan or dgrad_plan(spec)
    if splits > 1:
        slab = _slab(slab, slab_bytes(Mx, Cp, bm, bn, splits), dy.device)
    lib().igemm(ptr(dy), ptr(wt), ptr(dx), Cp, 0, 0, Cp, Mx, int(accumulate),
                ptr(slab) if splits > 1 else 0,
                spec.P, spec.Q, spec.K, spec.H, spec.W, spec.R, spec.S, spec.stride, spec.pad,
                spec.R * spec.S * spec.K // 8, Cp, Mx, bm, bn, splits, True, stream_ptr(),
                *_bw_args(bw, Mx, Cp))
    return dx


def wgrad_slab_bytes(spec: ConvSpec, plan):
    """Slab bytes of a split wgrad that reduces through a slab (csrc/wgrad_body.h): 4 KB of
    tile counters + one fp32 partial tile per (pixel split, output tile); 0 when unsplit."""
    bm, bn, splits = plan[:3]
    ncols = spec.R * spec.S * spec.Cp
    gx = math.ceil(spec.K / bm) * math.ceil(ncols / bn)
    ptiles = math.ceil(spec.M / 64)
    splits = max(1, min(splits, ptiles))
    per = math.ceil(ptiles / splits)
    gy = math.ceil(ptiles / per)
    if gy <= 1 or gx > WG_SEM_INTS:
        return 0
    return WG_SEM_INTS * 4 + gx * gy * bm * bn * 4


def conv_wgrad(dy, x, dw, spec: ConvSpec, plan=None, slab=None):
    """dw[K][R][S][C] (fp32, channel padding dropped) += / = wgrad(dy, x).  With ``slab``
    (>= wgrad_slab_bytes, zero-initialised once) the pixel splits reduce through it and dw is
    stored; without, split plans add into dw atomically (dw must start at zero)."""
    _chk(dy, torch.bfloat16, 'dy', spec.M * spec.K)
    _chk(x, torch.bfloat16, 'x', spec.N * spec.H * spec.W * spec.Cp)
    _chk(dw, torch.float32, 'dw', spec.K * spec.R * spec.S * spec.C)
    if spec.K % 8:
        raise ValueError('wgrad needs K % 8 == 0')
    _wg_range(spec)
    bm, bn, splits = (plan or wgrad_plan(spec))[:3]
    lib().wgrad(ptr(dy), ptr(x), ptr(dw), spec.N, spec.H, spec.W, spec.Cp, spec.P, spec.Q,
                spec.K, spec.R, spec.S, spec.stride, spec.pad, spec.C, bm, bn, splits,
                _wslab_ptr(spec, (bm, bn, splits), slab), stream_ptr())
    return dw


def _wg_range(spec):
    # the wgrad kernel addresses dy and x through buffer resources with 32-bit byte offsets
    if max(spec.M * spec.K, spec.N * spec.H * spec.W * spec.Cp) * 2 >= 2 ** 31:
        raise ValueError('wgrad: an operand exceeds 2 GiB (32-bit buffer offsets)')


def _wslab_ptr(spec, plan, slab):
    need = wgrad_slab_bytes(spec, plan)
    if slab is None or need == 0:
        return 0
    if slab.numel() * slab.element_size() < need:
        raise ValueError('wgrad slab too small (%d < %d bytes)'
                         % (slab.numel() * slab.element_size(), need))
    return ptr(slab)


def conv_bwd(dy, wt, dx, x, dw, spec: ConvSpec, dplan=None, wplan=None, slab=None,
             accumulate=False, bw=None, wslab=None):
    """Both backward GEMMs of one conv in ONE launch (csrc/igemm.hip bwd_pair_kernel):
    dx (= conv_dgrad, optional fused BN-backward reduce ``bw``) and dw (= conv_wgrad)."""
    if spec.stride not in (1, 2) or spec.K % 8:
        raise ValueError('conv_bwd needs stride 1/2 and K % 8 == 0')
    Cp = spec.Cp
    _chk(dy, torch.bfloat16, 'dy', spec.M * spec.K)
    _chk(wt, torch.bfloat16, 'wt', Cp * spec.R * spec.S * spec.K)
    _chk(dx, torch.bfloat16, 'dx', spec.N * spec.H * spec.W * Cp)
    _chk(x, torch.bfloat16, 'x', spec.N * spec.H * spec.W * Cp)
    _chk(dw, torch.float32, 'dw', spec.K * spec.R * spec.S * spec.C)
    _wg_range(spec)
    bm, bn, splits = dplan or dgrad_plan(spec)
    wbm, wbn, wsplits = (wplan or wgrad_plan(spec))[:3]
    Mx = spec.N * spec.H * spec.W
    if dgrad_s2_ok(spec):
        # stride 2: the dgrad as parity classes; at the small train batch in the same launch as
        # the wgrad (64 x 64 class tiles), else two launches with the class dgrad's own tiles
        if spec.N <= 32 and lib().conv_bwd_pair_s2(
                ptr(dy), ptr(wt), ptr(dx), Cp, int(accumulate), spec.P, spec.Q, spec.K, spec.R,
                spec.S, spec.stride, spec.pad, Cp, 64, 64, spec.H, spec.W, spec.N,
                *_bw_args(bw, Mx, Cp), ptr(x), ptr(dw), Cp, spec.P, spec.Q, spec.K, spec.C, wbm,
                wbn, wsplits, _wslab_ptr(spec, (wbm, wbn, wsplits), wslab), stream_ptr()):
            return dx, dw
        conv_wgrad(dy, x, dw, spec, plan=(wbm, wbn, wsplits), slab=wslab)
        conv_dgrad(dy, wt, dx, spec, plan=dgrad_s2_plan(spec), accumulate=accumulate, bw=bw)
        return dx, dw
    if splits > 1:
        slab = _slab(slab, slab_bytes(Mx, Cp, bm, bn, splits), dy.device)
    ok = lib().conv_bwd_pair(
        ptr(dy), ptr(wt), ptr(dx), Cp, int(accumulate), ptr(slab) if splits > 1 else 0,
        spec.P, spec.Q, spec.K, spec.H, spec.W, spec.R, spec.S, spec.stride, spec.pad,
        spec.R * spec.S * spec.K // 8, Cp, Mx, bm, bn, splits, *_bw_args(bw, Mx, Cp),
        ptr(x), ptr(dw), spec.N, spec.H, spec.W, Cp, spec.P, spec.Q, spec.K, spec.C, wbm, wbn,
        wsplits, _wslab_ptr(spec, (wbm, wbn, wsplits), wslab), stream_ptr())
    if not ok:
        conv_wgrad(dy, x, dw, spec, plan=(wbm, wbn, wsplits), slab=wslab)
        conv_dgrad(dy, wt, dx, spec, slab=slab, plan=(bm, bn, splits), accumulate=accumulate,
                   bw=bw)
    return dx, dw


def conv_bwd_sc(a, b):
    """A block's last-conv backward pair (stride 1: dgrad + wgrad) and its 1x1 stride-2
    shortcut's pair (parity-class dgrad + wgrad) in ONE launch (csrc/igemm.hip
    bwd_pair_sc_kernel).  ``a``: dict(dy, wt, dx, x, dw, spec, dplan, wplan, slab, accumulate,
    bw) as conv_bwd takes; ``b``: the shortcut's dict(dy, wt, dx, x, dw, spec, wplan,
    accumulate).  Returns False (nothing launched) when the pair is outside the kernel's
    instantiations; the caller then runs conv_bwd twice."""
    sa, sb = a['spec'], b['spec']
    if sa.stride != 1 or sa.K % 8 or not dgrad_s2_ok(sb) or sb.N > 32:
        return False
    bm, bn, splits = a.get('dplan') or dgrad_plan(sa)
    wbm, wbn, wsplits = (a.get('wplan') or wgrad_plan(sa))[:3]
    sbm, sbn, ssplits = (b.get('wplan') or wgrad_plan(sb))[:3]
    if (sbm, sbn) != (64, 64):
        return False
    for d, sp in ((a, sa), (b, sb)):
        _chk(d['dy'], torch.bfloat16, 'dy', sp.M * sp.K)
        _chk(d['wt'], torch.bfloat16, 'wt', sp.Cp * sp.R * sp.S * sp.K)
        _chk(d['dx'], torch.bfloat16, 'dx', sp.N * sp.H * sp.W * sp.Cp)
        _chk(d['x'], torch.bfloat16, 'x', sp.N * sp.H * sp.W * sp.Cp)
        _chk(d['dw'], torch.float32, 'dw', sp.K * sp.R * sp.S * sp.C)
        _wg_range(sp)
    Mx = sa.N * sa.H * sa.W
    slab = a.get('slab')
    if splits > 1:
        slab = _slab(slab, slab_bytes(Mx, sa.Cp, bm, bn, splits), a['dy'].device)
    ta = (ptr(a['dy']), ptr(a['wt']), ptr(a['dx']), sa.Cp, int(a.get('accumulate', False)),
          ptr(slab) if splits > 1 else 0, sa.P, sa.Q, sa.K, sa.H, sa.W, sa.R, sa.S, sa.stride,
          sa.pad, sa.R * sa.S * sa.K // 8, sa.Cp, Mx, bm, bn, splits,
          *_bw_args(a.get('bw'), Mx, sa.Cp), ptr(a['x']), ptr(a['dw']), sa.N, sa.H, sa.W, sa.Cp,
          sa.P, sa.Q, sa.K, sa.C, wbm, wbn, wsplits, 0)
    Mb = sb.N * sb.H * sb.W
    tb = (ptr(b['dy']), ptr(b['wt']), ptr(b['dx']), sb.Cp, int(b.get('accumulate', False)),
          sb.P, sb.Q, sb.K, sb.R, sb.S, sb.stride, sb.pad, sb.Cp, 64, 64, sb.H, sb.W, sb.N,
          *_bw_args(None, Mb, sb.Cp), ptr(b['x']), ptr(b['dw']), sb.Cp, sb.P, sb.Q, sb.K, sb.C,
          sbm, sbn, ssplits, 0)
    return bool(lib().conv_bwd_pair_sc(ta, tb, stream_ptr()))


# ----------------------------------------------------------------------- layout helpers
def to_nhwc(x, cpad=None):
    """NCHW float -> NHWC bf16 with channels padded to ``cpad`` (default: next multiple of 8)."""
    n, c, h, w = x.shape
    cp = cpad or cpad8(c)
    out = torch.zeros(n, h, w, cp, dtype=torch.bfloat16, device=x.device)
    out[..., :c] = x.permute(0, 2, 3, 1).to(torch.bfloat16)
    return out


def from_nhwc(y, c=None):
    """NHWC (padded) -> NCHW float32."""
    c = c or y.shape[-1]
    return y[..., :c].permute(0, 3, 1, 2).float()


def pack_conv_weight(w_kcrs):
    """fp32 torch conv weight [K][C][R][S] -> (bf16 [K][R][S][Cp], bf16 [C][R][S][K])."""
    k, c, r, s = w_kcrs.shape
    krsc = torch.zeros(k, r, s, cpad8(c), dtype=torch.bfloat16, device=w_kcrs.device)
    krsc[..., :c] = w_kcrs.permute(0, 2, 3, 1).to(torch.bfloat16)
    crsk = w_kcrs.permute(1, 2, 3, 0).contiguous().to(torch.bfloat16)
    return krsc.contiguous(), crsk
