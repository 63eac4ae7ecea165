"""Row-step persistent conv (csrc/hconv.hip hrow_kernel) vs the per-tap persistent kernel on the
ResNet-18 scoring-pass stride-1 3x3 shapes (B = 320, 10 ghost-BN groups), graph-timed.

    python bench/hrow_bench.py [--grids 128,256]

One JSON line per (shape, grid): microseconds per conv for the engine's current plan, the
row-step plan (256 x 64 tiles, 8 waves), and TF/s."""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from gtime import gtime  # noqa: E402

SHAPES = [(320, 32, 64, 64), (320, 16, 128, 128), (320, 8, 256, 256), (320, 4, 512, 512)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--grids', default='128,256')
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--shapes', default='0,1,2,3', help='indices into SHAPES')
    ap.add_argument('--plans', default='engine,row4')
    ap.add_argument('--wm8', type=int, default=0, help='8-wave layout override (hconv_configure)')
    ap.add_argument('--swa', type=int, default=1, help='per-tile row-term halo swizzle (0: off)')
    ap.add_argument('--pro', action='store_true',
                    help="the input's ghost-BN + ReLU in the halo staging (MODE 1)")
    args = ap.parse_args()
    import torch
    from mercury_amd import ops
    from mercury_amd.ops import hconv as H
    from mercury_amd.ops.conv import ConvSpec, slab_bytes
    ops.lib()
    H._CFG['swa'] = bool(args.swa)
    dev = 'cuda'
    for grid in [int(x) for x in args.grids.split(',')]:
        ops.lib().hconv_configure(grid, 8, args.wm8)
        for (N, Hh, C, K) in [SHAPES[int(i)] for i in args.shapes.split(',')]:
            sp = ConvSpec(N, Hh, Hh, C, K, 3, 3, 1, 1)
            sp.group_rows = 32 * Hh * Hh
            torch.manual_seed(0)
            x = ops.to_nhwc((torch.randn(N, C, Hh, Hh, device=dev)).to(torch.bfloat16).float())
            wk, _ = ops.pack_conv_weight(torch.randn(K, C, 3, 3, device=dev) * 0.05)
            y = torch.empty(sp.M * K, dtype=torch.bfloat16, device=dev)
            stats = torch.zeros(10 * 2 * K, device=dev)
            pro = None
            if args.pro:
                st_in = torch.rand(10 * 2 * C, device=dev) + 1.0
                pro = dict(stats=st_in, gamma=torch.rand(C, device=dev) + 0.5,
                           beta=torch.randn(C, device=dev) * 0.1, act='relu', eps=1e-5,
                           count=32 * Hh * Hh, group_imgs=32)
            cur = H.engine_plan(sp)
            slab = torch.zeros(max(4, slab_bytes(sp.M, K, *cur[:3]) // 4 + 1), device=dev) \
                if cur and cur[2] > 0 else None
            row = {'shape': [N, Hh, C, K], 'grid': grid, 'pro': bool(args.pro), 'gflop': round(2 * sp.M * K * 9 * C / 1e9, 2)}
            cands = [('engine', cur)]
            bm = 256 if Hh >= 16 else 128
            cands += [('row4', (bm, 64, -1))]
            for name, p in cands:
                if p is None or name not in args.plans.split(','):
                    continue
                g = H.geometry_cached(sp, p[0], p[1])
                if p[2] < 0 and (g is None or H.row_lds_bytes(g, p[0], p[1], p[2]) > H.LDS_MAX):
                    row[name] = 'no-fit'
                    continue
                try:
                    us = gtime(lambda: H.hconv_fwd(x, wk, y, sp, p, stats=stats, slab=slab,
                                                   pro=pro), reps=args.reps)
                except Exception as e:  # noqa: BLE001
                    row[name] = 'error: %s' % e
                    continue
                row[name] = {'plan': list(p), 'us': round(us, 2),
                             'tflops': round(2 * sp.M * K * 9 * C / us / 1e6, 1)}
            print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
