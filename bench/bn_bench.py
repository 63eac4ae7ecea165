"""bn_apply (csrc/bn.hip) variants on the engine's BN-pass shapes, graph-timed.

    python bench/bn_bench.py [--variants 0,1] [--reps 8]

Variants (``bn_configure``): 0 ordinary stores, 1 streaming (nontemporal) stores.  (A
software-pipelined loop -- the next trip's rows requested before this trip's stores -- measured
equal to the plain loop, 4.98 vs 4.99 TB/s on the layer-1 projection block end, and was
dropped: these passes run at the HBM rate for mixed read / write traffic.)
One JSON line per (shape, variant): microseconds and the HBM rate of the bytes the pass moves
(each input read once, the output written once).  Outputs are checked equal across variants.
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from gtime import gtime  # noqa: E402

# (name, M, C, groups, residual mode)
SHAPES = [
    ('r50_l1_proj_end', 1280 * 3136, 256, 10, 2),
    ('r50_l1_intra', 1280 * 3136, 64, 10, 0),
    ('r50_l3_id_end', 1280 * 196, 1024, 10, 1),
    ('r50_l2_intra', 1280 * 784, 128, 10, 0),
    ('r18_b320_l1', 320 * 1024, 64, 10, 1),
    ('r18_b32_l1', 32 * 1024, 64, 1, 0),
    ('r50_b128_l1_end', 128 * 3136, 256, 1, 1),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--variants', default='0,1')
    ap.add_argument('--reps', type=int, default=8)
    ap.add_argument('--shapes', default='')
    args = ap.parse_args()
    import torch
    from mercury_amd import ops
    lib = ops.lib()
    dev = 'cuda'
    for name, M, C, G, rm in SHAPES:
        if args.shapes and name not in args.shapes.split(','):
            continue
        torch.manual_seed(0)
        y = (torch.randn(M, C, device=dev) * 2).to(torch.bfloat16)
        res = torch.randn(M, C, device=dev).to(torch.bfloat16) if rm else None
        gr = M // G
        stats = torch.empty(G, 2, C, device=dev)
        stats[:, 0] = torch.randn(G, C, device=dev) * gr * 0.1
        stats[:, 1] = (torch.rand(G, C, device=dev) + 1.0) * gr * 4
        gamma = torch.rand(C, device=dev) + 0.5
        beta = torch.randn(C, device=dev) * 0.1
        res_bn = None
        if rm == 2:
            s2 = stats.clone()
            res_bn = (s2, gamma.clone(), beta.clone())
        out = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
        nbytes = M * C * 2 * (2 + (1 if rm else 0))
        ref = None
        for v in [int(x) for x in args.variants.split(',')]:
            lib.bn_configure(0 if v else 1 << 62)
            fn = lambda: ops.bn_apply(y, stats, gamma, beta, out, M, C, group_rows=gr,  # noqa
                                      act='relu', res=res, res_bn=res_bn)
            us = gtime(fn, reps=args.reps)
            fn()
            torch.cuda.synchronize()
            same = None
            if ref is None:
                ref = out.clone()
            else:
                same = bool(torch.equal(ref, out))
            print(json.dumps({'shape': name, 'M': M, 'C': C, 'res': rm, 'variant': v,
                              'us': round(us, 2), 'tbps': round(nbytes / us / 1e6, 2),
                              'equal': same}), flush=True)
        lib.bn_configure(256 << 20)
        del y, res, out, ref
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
