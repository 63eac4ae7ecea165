"""Halo-tile conv (hconv) vs the generic implicit GEMM (igemm), timed by HIP-graph replay.

    python bench/hconv_sweep.py [--batch 320] [--reps 12]

Per ResNet-18 CIFAR conv shape with >= 64 input channels, one JSON line:
  igemm_us       generic implicit GEMM at its heuristic plan (plain input)
  bn_apply_us    the standalone BN + ReLU pass over the conv input that igemm needs first
  hconv_us       halo conv, plain input, best plan over tiles x 64-channel splits (split 0:
                 the persistent kernel)
  hconv_bn_us    halo conv with the producer's BN + ReLU applied while staging (+ the kept
                 activation where the halos tile the input) -- replaces bn_apply + igemm
"""
from __future__ import annotations

import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from gtime import gtime  # noqa: E402

SHAPES = [  # C, K, H, R, stride
    (64, 64, 32, 3, 1), (64, 128, 32, 3, 2), (128, 128, 16, 3, 1), (128, 256, 16, 3, 2),
    (256, 256, 8, 3, 1), (256, 512, 8, 3, 2), (512, 512, 4, 3, 1)]
# ResNet-50/224 bottleneck 3x3 convs (conv2 of each stage; the stride-2 ones open a stage)
R50_SHAPES = [(64, 64, 56, 3, 1), (128, 128, 56, 3, 2), (128, 128, 28, 3, 1),
              (256, 256, 28, 3, 2), (256, 256, 14, 3, 1), (512, 512, 14, 3, 2),
              (512, 512, 7, 3, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=320)
    ap.add_argument('--no-bn', action='store_true')
    ap.add_argument('--reps', type=int, default=12)
    ap.add_argument('--r50', action='store_true', help='ResNet-50/224 3x3 shapes')
    ap.add_argument('--group', type=int, default=0,
                    help='ghost-BN group in images (0: 32 above a batch of 32)')
    ap.add_argument('--miopen', action='store_true',
                    help='also time F.conv2d (MIOpen, bf16 channels_last) on the same shape')
    args = ap.parse_args()
    import torch
    from mercury_amd import ops
    from mercury_amd.ops import hconv as H
    from mercury_amd.ops.conv import ConvSpec, fwd_plan, slab_bytes
    dev = 'cuda'
    N = args.batch
    gimgs = args.group or (32 if N > 32 else 0)
    if gimgs >= N:
        gimgs = 0
    G = N // gimgs if gimgs else 1
    tot = dict(igemm=0.0, bn_apply=0.0, hconv=0.0, hconv_bn=0.0)
    for (C, K, Hh, R, st) in (R50_SHAPES if args.r50 else SHAPES):
        sp = ConvSpec(N, Hh, Hh, C, K, R, R, st, R // 2)
        if gimgs:
            sp.group_rows = gimgs * sp.P * sp.Q
        torch.manual_seed(0)
        y = ops.to_nhwc(torch.randn(N, C, Hh, Hh, device=dev))
        a = torch.empty_like(y)
        wk, _ = ops.pack_conv_weight(torch.randn(K, C, R, R, device=dev) * 0.05)
        out = torch.empty(sp.M * K, dtype=torch.bfloat16, device=dev)
        stats = torch.zeros(G * 2 * K, device=dev)
        ystats = torch.rand(G * 2 * C, device=dev) + 1.0
        gamma = torch.ones(C, device=dev)
        beta = torch.zeros(C, device=dev)
        cands = []
        for bm, bn, _ in H.TILES:
            g = H.geometry_cached(sp, bm, bn)
            if g is None:
                continue
            for s in (1, 2, 4):
                if s <= C // 64 and H.lds_bytes(g, bm, bn, s) <= H.LDS_MAX:
                    cands.append((bm, bn, s))
            if H.persistent_ok(sp, bm, bn) and H.lds_bytes(g, bm, bn, 0) <= H.LDS_MAX:
                cands.append((bm, bn, 0))      # persistent kernel
        hp = H.plan(sp)
        ip = fwd_plan(sp)
        slab = torch.zeros(max([slab_bytes(sp.M, K, *c) for c in cands + [ip]] + [4]) // 4 + 1,
                           device=dev)
        ti = gtime(lambda: ops.conv_fwd(y, wk, out, sp, stats=stats, slab=slab, plan=ip),
                   reps=args.reps)
        tb = gtime(lambda: ops.bn_apply(y, ystats, gamma, beta, a, N * Hh * Hh, C,
                                        group_rows=(gimgs or N) * Hh * Hh, act='relu'),
                   reps=args.reps)
        tm = -1.0
        if args.miopen:
            import torch.nn.functional as F
            xt = torch.randn(N, C, Hh, Hh, device=dev, dtype=torch.bfloat16).to(
                memory_format=torch.channels_last)
            wt = (torch.randn(K, C, R, R, device=dev) * 0.05).to(torch.bfloat16).to(
                memory_format=torch.channels_last)
            for _ in range(3):
                F.conv2d(xt, wt, stride=st, padding=R // 2)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(args.reps):
                F.conv2d(xt, wt, stride=st, padding=R // 2)
            e1.record()
            torch.cuda.synchronize()
            tm = e0.elapsed_time(e1) * 1e3 / args.reps
            del xt, wt
        res = {}
        for c in cands:
            res[c] = gtime(lambda: H.hconv_fwd(y, wk, out, sp, c, stats=stats, slab=slab),
                           reps=args.reps)
        if not res:
            print(json.dumps(dict(shape=[N, C, K, Hh, R, st], igemm_plan=list(ip),
                                  igemm_us=round(ti, 2),
                                  igemm_tflops=round(sp.flops() / ti / 1e6, 1),
                                  miopen_us=round(tm, 2),
                                  miopen_tflops=round(sp.flops() / tm / 1e6, 1) if tm > 0 else None,
                                  bn_apply_us=round(tb, 2), hconv=None)), flush=True)
            continue
        best = min(res, key=res.get)
        # input BN in the staging: persistent / row-step plans only (the per-tile modes were
        # removed in round 5)
        pro = dict(stats=ystats, gamma=gamma, beta=beta, act='relu', count=(gimgs or N) * Hh * Hh,
                   group_imgs=gimgs or N)
        tbn = -1.0 if args.no_bn or best[2] > 0 else gtime(
            lambda: H.hconv_fwd(y, wk, out, sp, best, stats=stats, slab=slab, pro=pro),
            reps=args.reps)
        row = dict(shape=[N, C, K, Hh, R, st], igemm_plan=list(ip), igemm_us=round(ti, 2),
                   miopen_us=round(tm, 2),
                   igemm_tflops=round(sp.flops() / ti / 1e6, 1), bn_apply_us=round(tb, 2),
                   hconv_heur=list(hp) if hp else None,
                   hconv_heur_us=round(res.get(tuple(hp), -1), 2) if hp else None,
                   hconv_best=list(best), hconv_us=round(res[best], 2),
                   hconv_tflops=round(sp.flops() / res[best] / 1e6, 1),
                   hconv_bn_us=round(tbn, 2),
                   all={'%dx%d/%d' % c: round(t, 2) for c, t in res.items()})
        print(json.dumps(row), flush=True)
        tot['igemm'] += ti
        tot['bn_apply'] += tb
        tot['hconv'] += res[best]
        tot['hconv_bn'] += tbn
    print(json.dumps({'batch': N, 'totals_us': {k: round(v, 1) for k, v in tot.items()}}),
          flush=True)


if __name__ == '__main__':
    main()
