"""Tile / split sweep for the dgrad+wgrad pair launch at the train batch (B=32).

For every ResNet-18 CIFAR conv shape (and MobileNetV2's 1x1s) times ``ops.conv_bwd`` over
candidate (dgrad tile, dgrad split) x (wgrad tile, wgrad split) plans and prints the best
against the default plan -- the data behind ``dgrad_plan`` / ``wgrad_plan``.

    python bench/bwd_pair_sweep.py [--iters 30] > sweep.jsonl
"""
import argparse
import itertools
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # C, K, H, R, stride, pad
    (64, 64, 32, 3, 1, 1), (64, 128, 32, 3, 2, 1), (128, 128, 16, 3, 1, 1),
    (64, 128, 32, 1, 2, 0), (128, 256, 16, 3, 2, 1), (256, 256, 8, 3, 1, 1),
    (128, 256, 16, 1, 2, 0), (256, 512, 8, 3, 2, 1), (512, 512, 4, 3, 1, 1),
    (256, 512, 8, 1, 2, 0)]


def timeit(fn, iters):
    import torch
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(iters + 1)]
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev[0].record()
    for i in range(iters):
        fn()
        ev[i + 1].record()
    torch.cuda.synchronize()
    ts = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(iters))
    return ts[len(ts) // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=30)
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--default-only', action='store_true',
                    help='graph-timed default plans only (for same-box A/B of two builds)')
    args = ap.parse_args()
    import torch
    from mercury_amd import ops
    from mercury_amd.ops.conv import ConvSpec, dgrad_plan, slab_bytes, wgrad_plan
    dev = 'cuda'
    N = args.batch
    tot = 0.0
    for (C, K, H, R, st, pd) in SHAPES:
        sp = ConvSpec(N, H, H, C, K, R, R, st, pd)
        Mx = N * H * H
        x = ops.to_nhwc(torch.randn(N, C, H, H, device=dev))
        _, wt = ops.pack_conv_weight(torch.randn(K, C, R, R, device=dev) * 0.05)
        gy = ops.to_nhwc(torch.randn(N, K, sp.P, sp.Q, device=dev))
        dx = torch.empty(Mx, sp.Cp, dtype=torch.bfloat16, device=dev)
        dw = torch.zeros(K * R * R * C, device=dev)
        kt = math.ceil(R * R * K / 64)
        ptiles = math.ceil(sp.M / 64)
        dcands = []
        for bm, bn in ((128, 128), (128, 64), (64, 128), (64, 64)):
            for s in (1, 2, 4, 8):
                if s <= max(1, kt // 2):
                    dcands.append((bm, bn, s))
        wcands = []
        for bm, bn in ((128, 128), (128, 64), (64, 128), (64, 64)):
            for s in (1, 2, 4, 8, 16, 32, 64):
                if s <= ptiles:
                    wcands.append((bm, bn, s))
        slab = torch.zeros(max(slab_bytes(Mx, sp.Cp, bm, bn, s) for bm, bn, s in dcands) // 4 + 1,
                           device=dev)
        dp0, wp0 = dgrad_plan(sp), wgrad_plan(sp)
        if args.default_only:
            sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
            from gtime import gtime
            us = gtime(lambda: ops.conv_bwd(gy, wt, dx, x, dw, sp, dplan=dp0, wplan=wp0,
                                            slab=slab), reps=8)
            tot += us
            print(json.dumps({'shape': [N, C, K, H, R, st], 'us': round(us, 1),
                              'plan': [list(dp0), list(wp0)]}), flush=True)
            continue
        base = timeit(lambda: ops.conv_bwd(gy, wt, dx, x, dw, sp, dplan=dp0, wplan=wp0,
                                           slab=slab), args.iters)
        best = (base, dp0, wp0)
        for dp, wp in itertools.product(dcands, wcands):
            t = timeit(lambda: ops.conv_bwd(gy, wt, dx, x, dw, sp, dplan=dp, wplan=wp, slab=slab),
                       max(5, args.iters // 3))
            if t < best[0]:
                best = (t, dp, wp)
        print(json.dumps({'shape': [N, C, K, H, R, st], 'default_us': round(base, 1),
                          'default': [list(dp0), list(wp0)], 'best_us': round(best[0], 1),
                          'best': [list(best[1]), list(best[2])]}), flush=True)
    if args.default_only:
        print(json.dumps({'total_us': round(tot, 1)}), flush=True)


if __name__ == '__main__':
    main()
