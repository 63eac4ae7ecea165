"""Tile / split / pipeline sweep for the forward implicit-GEMM conv (train and scoring batch).

    python bench/fwd_sweep.py [--iters 20] > fwd_sweep.jsonl

For each ResNet-18 CIFAR conv shape at batch 32 (train) and 320 (10 ghost groups of 32,
the scoring pass) times ``ops.conv_fwd`` with BN statistics over the candidate plans and
pipes and prints the best against ``fwd_plan``'s choice.
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bwd_pair_sweep import SHAPES, timeit  # noqa: E402

SHAPES = [(3, 64, 32, 3, 1, 1)] + SHAPES


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    args = ap.parse_args()
    import torch
    from mercury_amd import ops
    from mercury_amd.ops.conv import ConvSpec, fwd_plan, slab_bytes
    dev = 'cuda'
    for N, gimgs in ((32, 0), (320, 32)):
        for (C, K, H, R, st, pd) in SHAPES:
            sp = ConvSpec(N, H, H, C, K, R, R, st, pd)
            if gimgs:
                sp.group_rows = gimgs * sp.P * sp.Q
            G = N // gimgs if gimgs else 1
            x = ops.to_nhwc(torch.randn(N, C, H, H, device=dev))
            wk, _ = ops.pack_conv_weight(torch.randn(K, C, R, R, device=dev) * 0.05)
            y = torch.empty(sp.M, K, dtype=torch.bfloat16, device=dev)
            stats = torch.zeros(G, 2, K, device=dev)
            kt = math.ceil(R * R * sp.Cp / 64)
            cands = []
            for bm, bn in ((256, 64), (128, 128), (128, 64), (64, 128), (64, 64)):
                if sp.group_rows and sp.group_rows < bm:
                    continue
                for s in (1, 2, 4, 8):
                    if s <= max(1, kt // 2):
                        cands.append((bm, bn, s))
            slab = torch.zeros(max(slab_bytes(sp.M, K, *c) for c in cands) // 4 + 1, device=dev)
            p0 = fwd_plan(sp)
            base = timeit(lambda: ops.conv_fwd(x, wk, y, sp, stats=stats, slab=slab, plan=p0),
                          args.iters)
            best = (base, p0, 0)
            for c in cands:
                for pipe in (0, 3):
                    t = timeit(lambda: ops.conv_fwd(x, wk, y, sp, stats=stats, slab=slab, plan=c,
                                                    pipe=pipe), max(5, args.iters // 2))
                    if t < best[0]:
                        best = (t, c, pipe)
            print(json.dumps({'shape': [N, C, K, H, R, st], 'default_us': round(base, 1),
                              'default': list(p0), 'best_us': round(best[0], 1),
                              'best': list(best[1]), 'best_pipe': best[2]}), flush=True)


if __name__ == '__main__':
    main()
