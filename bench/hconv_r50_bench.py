"""ResNet-50's 3x3 convs on the persistent halo kernel with padded row tiles (csrc/hconv.hip
hconv_persist_kernel, ``ops.hconv.geometry(pad=True)``) vs the implicit GEMM, graph-timed.

    python bench/hconv_r50_bench.py [--batches 1280,128] [--pro]

The 56/28/14/7-wide images have no whole-row tile of 64/128/256 rows; the padded tile holds the
largest whole-row count that fits (2 x 56 or 4 x 28 = 112 of 128 rows) and drops the rest.  One
JSON line per (shape, plan): microseconds, TF/s (real FLOPs), and the max difference from the
implicit GEMM's output (bf16 ulp scale).  ``--pro``: the input's ghost-BN + ReLU in the halo
staging (MODE 1), which the scoring pass uses instead of a bn_apply pass.
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from gtime import gtime  # noqa: E402

# (H, C, K, stride) of ResNet-50's 3x3 convs (input size)
SHAPES = [(56, 64, 64, 1), (28, 128, 128, 1), (14, 256, 256, 1), (7, 512, 512, 1),
          (56, 128, 128, 2), (28, 256, 256, 2), (14, 512, 512, 2)]
PLANS = [(128, 64), (256, 64), (64, 64)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batches', default='1280,128')
    ap.add_argument('--grids', default='0,256')
    ap.add_argument('--shapes', default='')
    ap.add_argument('--reps', type=int, default=6)
    ap.add_argument('--pro', action='store_true')
    args = ap.parse_args()
    import torch
    from mercury_amd import ops
    from mercury_amd.ops import hconv as H
    from mercury_amd.ops.conv import ConvSpec, fwd_plan, slab_bytes
    ops.lib()
    dev = 'cuda'
    for B in [int(b) for b in args.batches.split(',')]:
        gi = 128 if B > 128 else B
        for si, (Hh, C, K, st) in enumerate(SHAPES):
            if args.shapes and str(si) not in args.shapes.split(','):
                continue
            sp = ConvSpec(B, Hh, Hh, C, K, 3, 3, st, 1)
            sp.group_rows = gi * sp.P * sp.Q
            G = B // gi
            torch.manual_seed(0)
            x = ops.to_nhwc(torch.randn(B, C, Hh, Hh, device=dev).to(torch.bfloat16).float())
            wk, _ = ops.pack_conv_weight(torch.randn(K, C, 3, 3, device=dev) * 0.03)
            flop = 2.0 * sp.M * K * 9 * C
            row = {'B': B, 'shape': [Hh, C, K, st], 'gflop': round(flop / 1e9, 1)}
            out_ref = torch.empty(sp.M * K, dtype=torch.bfloat16, device=dev)
            st_ref = torch.zeros(G * 2 * K, device=dev)
            ip = fwd_plan(sp)
            slab = torch.zeros(max(4, slab_bytes(sp.M, K, *ip[:3]) // 4 + 1), device=dev)

            def igemm():
                st_ref.zero_()
                ops.conv_fwd(x, wk, out_ref, sp, stats=st_ref, slab=slab, plan=ip)
            us = gtime(igemm, reps=args.reps)
            igemm()
            row['igemm'] = {'plan': list(ip[:3]), 'us': round(us, 1),
                            'tflops': round(flop / us / 1e6, 1)}
            pro = None
            if args.pro:
                stin = torch.empty(G, 2, C, device=dev)
                cnt = gi * Hh * Hh
                stin[:, 0] = torch.randn(G, C, device=dev) * cnt * 0.1
                stin[:, 1] = (torch.rand(G, C, device=dev) + 1.0) * cnt
                pro = dict(stats=stin.reshape(-1), gamma=torch.rand(C, device=dev) + 0.5,
                           beta=torch.randn(C, device=dev) * 0.1, act='relu', eps=1e-5,
                           count=cnt, group_imgs=gi)
            for bm, bn in PLANS:
                g = H.geometry(sp, bm, bn, pad=True)
                if g is None or not H.persistent_ok(sp, bm, bn):
                    continue
                if H.lds_bytes(g, bm, bn, 0) + H.persist_table_bytes(sp, pro) > H.LDS_MAX:
                    continue
                vr = g['IMG'] * g['TR'] * g['Q']
                for grid in [int(v) for v in args.grids.split(',')]:
                    out = torch.empty(sp.M * K, dtype=torch.bfloat16, device=dev)
                    stt = torch.zeros(G * 2 * K, device=dev)
                    p = (bm, bn, 0, grid)

                    def hc():
                        stt.zero_()
                        H.hconv_fwd(x, wk, out, sp, p, stats=stt, pro=pro)
                    try:
                        us = gtime(hc, reps=args.reps)
                    except Exception as e:  # noqa: BLE001
                        row['%dx%d_g%d' % (bm, bn, grid)] = 'error: %s' % e
                        continue
                    hc()
                    torch.cuda.synchronize()
                    d = None
                    if pro is None:
                        d = round((out.float() - out_ref.float()).abs().max().item(), 4)
                    row['%dx%d_g%d' % (bm, bn, grid)] = {
                        'vr': vr, 'us': round(us, 1), 'tflops': round(flop / us / 1e6, 1),
                        'maxdiff': d}
            print(json.dumps(row), flush=True)
            del x, out_ref, slab
            torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
