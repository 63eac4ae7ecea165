"""Per-layer plan sweep for the implicit-GEMM conv kernels, timed by HIP-graph replay.

    python bench/kernel_sweep.py [--batch 32] [--kind fwd|bwd|both] [--write-cache PATH]

For every ResNet-18 CIFAR conv shape at one batch (train 32, or the 320-image scoring
pool with 10 ghost-BN groups) times each candidate plan -- forward: tile x K-split x
main-loop variant (register double buffer / LDS-DMA ring); backward: dgrad tile x split
with the wgrad tile x pixel-split of the paired launch -- with ``gtime`` (the in-graph
cost, not the host issue rate), and prints one JSON line per shape: the heuristic plan,
its time, the best plan and its time.  ``--write-cache`` stores the winners in the
``ops/tune.py`` cache format.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from gtime import gtime  # noqa: E402

SHAPES = [  # C, K, H, R, stride, pad
    (3, 64, 32, 3, 1, 1), (64, 64, 32, 3, 1, 1), (64, 128, 32, 3, 2, 1), (128, 128, 16, 3, 1, 1),
    (64, 128, 32, 1, 2, 0), (128, 256, 16, 3, 2, 1), (256, 256, 8, 3, 1, 1),
    (128, 256, 16, 1, 2, 0), (256, 512, 8, 3, 2, 1), (512, 512, 4, 3, 1, 1),
    (256, 512, 8, 1, 2, 0)]


def fwd_cands(sp):
    kt = math.ceil(sp.R * sp.S * sp.Cp / 64)
    out = []
    for bm, bn in ((256, 128), (256, 64), (128, 128), (128, 64), (64, 128), (64, 64)):
        if sp.group_rows and sp.group_rows < bm:
            continue
        if bn == 128 and sp.K <= 64:
            continue
        for s in (1, 2, 4, 8):
            if s <= max(1, kt // 2):
                out.append((bm, bn, s))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--kind', default='both', choices=('fwd', 'bwd', 'both'))
    ap.add_argument('--reps', type=int, default=12)
    ap.add_argument('--write-cache', default='')
    args = ap.parse_args()
    import torch
    from mercury_amd import ops
    from mercury_amd.ops import tune
    from mercury_amd.ops.conv import ConvSpec, dgrad_plan, fwd_plan, slab_bytes, wgrad_plan
    dev = 'cuda'
    N = args.batch
    gimgs = 32 if N > 32 else 0
    cache = {}
    tot = {'fwd_heur': 0.0, 'fwd_best': 0.0, 'bwd_heur': 0.0, 'bwd_best': 0.0}
    for (C, K, H, R, st, pd) in SHAPES:
        sp = ConvSpec(N, H, H, C, K, R, R, st, pd)
        if gimgs:
            sp.group_rows = gimgs * sp.P * sp.Q
        G = N // gimgs if gimgs else 1
        torch.manual_seed(0)
        x = ops.to_nhwc(torch.randn(N, C, H, H, device=dev))
        wk, wt = ops.pack_conv_weight(torch.randn(K, C, R, R, device=dev) * 0.05)
        row = {'shape': [N, C, K, H, R, st]}
        if args.kind in ('fwd', 'both'):
            y = torch.empty(sp.M * K, dtype=torch.bfloat16, device=dev)
            stats = torch.zeros(G * 2 * K, device=dev)
            cands = fwd_cands(sp)
            heur = tuple(fwd_plan(sp)) + (0,)
            slab = torch.zeros(max([slab_bytes(sp.M, K, *c[:3]) for c in cands + [heur]] + [4])
                               // 4 + 1, device=dev)

            def run(p):
                return gtime(lambda: ops.conv_fwd(x, wk, y, sp, stats=stats, slab=slab,
                                                  plan=p[:3]), reps=args.reps)
            th = run(heur)
            best = (th, heur)
            for c in cands:
                t = run(c)
                if t < best[0]:
                    best = (t, c)
            row.update(fwd_heur=list(heur), fwd_heur_us=round(th, 2), fwd_best=list(best[1]),
                       fwd_best_us=round(best[0], 2),
                       fwd_tflops=round(sp.flops() / best[0] / 1e6, 1))
            tot['fwd_heur'] += th
            tot['fwd_best'] += best[0]
            cache[tune._key('fwd', sp)] = list(best[1])
        if args.kind in ('bwd', 'both') and C % 8 == 0 and not gimgs:
            Mx = N * H * H
            dy = ops.to_nhwc(torch.randn(N, K, sp.P, sp.Q, device=dev))
            dx = torch.empty(Mx * sp.Cp, dtype=torch.bfloat16, device=dev)
            dw = torch.zeros(K * R * R * C, device=dev)
            dc, wc = tune._bwd_candidates(sp)
            dh, wh = tuple(dgrad_plan(sp)), tuple(wgrad_plan(sp))
            slab = torch.zeros(max([slab_bytes(Mx, sp.Cp, *p) for p in dc + [dh]] + [4]) // 4 + 1,
                               device=dev)

            def runb(d, w):
                return gtime(lambda: ops.conv_bwd(dy, wt, dx, x, dw, sp, dplan=d, wplan=w,
                                                  slab=slab), reps=args.reps)
            th = runb(dh, wh)
            dbest = min(((runb(d, wh), d) for d in dc), key=lambda t: t[0])
            best = min(((runb(dbest[1], w), w) for w in wc), key=lambda t: t[0])
            bt = best[0]
            pair = (dbest[1], best[1])
            if th <= bt:
                bt, pair = th, (dh, wh)
            row.update(bwd_heur=[list(dh), list(wh)], bwd_heur_us=round(th, 2),
                       bwd_best=[list(pair[0]), list(pair[1])], bwd_best_us=round(bt, 2))
            tot['bwd_heur'] += th
            tot['bwd_best'] += bt
            cache[tune._key('bwd', sp)] = [list(pair[0]), list(pair[1])]
        print(json.dumps(row), flush=True)
    print(json.dumps({'batch': N, 'totals_us': {k: round(v, 1) for k, v in tot.items()}}),
          flush=True)
    if args.write_cache:
        old = {}
        if os.path.exists(args.write_cache):
            with open(args.write_cache) as f:
                old = json.load(f)
        old.update(cache)
        with open(args.write_cache, 'w') as f:
            json.dump(dict(sorted(old.items())), f, indent=0)


if __name__ == '__main__':
    main()
