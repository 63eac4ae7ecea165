"""Per-shape forward conv time of two main-loop variants at each candidate tile plan.

    python bench/pipe_cmp.py --batch 320 --pipes 0,1
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'bench'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=320)
    ap.add_argument('--pipes', default='0,1')
    ap.add_argument('--dgrad', action='store_true')
    args = ap.parse_args()
    import torch
    from gtime import gtime
    from kernel_sweep import SHAPES
    from mercury_amd import ops
    from mercury_amd.ops.conv import ConvSpec, slab_bytes
    pipes = [int(p) for p in args.pipes.split(',')]
    N = args.batch
    tot = {p: 0.0 for p in pipes}
    for (C, K, H, R, st, pd) in SHAPES:
        if args.dgrad and C % 8:
            continue
        sp = ConvSpec(N, H, H, C, K, R, R, st, pd)
        x = ops.to_nhwc(torch.randn(N, C, H, H, device='cuda'))
        wk, wt = ops.pack_conv_weight(torch.randn(K, C, R, R, device='cuda') * 0.05)
        y = torch.empty(sp.M * K, dtype=torch.bfloat16, device='cuda')
        stats = torch.zeros(2 * K, device='cuda')
        dy = ops.to_nhwc(torch.randn(N, K, sp.P, sp.Q, device='cuda'))
        dx = torch.empty(N * H * H * sp.Cp, dtype=torch.bfloat16, device='cuda')
        row = {'shape': [N, C, K, H, R, st]}
        plans = [(bm, bn, s) for bm, bn in ((256, 64), (128, 128), (128, 64), (64, 128), (64, 64))
                 for s in (1, 2, 4)]
        M = N * H * H if args.dgrad else sp.M
        Nc = sp.Cp if args.dgrad else K
        slab = torch.zeros(max(slab_bytes(M, Nc, *p) for p in plans) // 4 + 1, device='cuda')
        for p in pipes:
            best = None
            for pl in plans:
                if args.dgrad:
                    f = lambda: ops.conv_dgrad(dy, wt, dx, sp, slab=slab, plan=pl, pipe=p)
                else:
                    f = lambda: ops.conv_fwd(x, wk, y, sp, stats=stats, slab=slab, plan=pl, pipe=p)
                t = gtime(f, reps=10)
                if best is None or t < best[0]:
                    best = (t, pl)
            row['p%d' % p] = [round(best[0], 2), list(best[1])]
            tot[p] += best[0]
        print(json.dumps(row), flush=True)
    print(json.dumps({'totals_us': {p: round(v, 1) for p, v in tot.items()}}), flush=True)


if __name__ == '__main__':
    main()
