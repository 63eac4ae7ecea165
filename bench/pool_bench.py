"""ImageNet-stem max pool (3x3/s2/p1, B x 112 x 112 x 64 bf16) timed by graph replay, with and
without the fused BN + ReLU, beside a bn_apply pass over the same tensor (the bandwidth
reference) -- bytes / time in TB/s.

    python bench/pool_bench.py [--batch 1280]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=1280)
    a = ap.parse_args()
    import torch
    from mercury_amd import ops
    ops.lib()
    N, H, C, G = a.batch, 112, 64, a.batch // 32
    P = 56
    x = torch.randn(N * H * H * C, device='cuda').to(torch.bfloat16)
    y = torch.empty(N * P * P * C, device='cuda', dtype=torch.bfloat16)
    a8 = torch.empty(N * P * P * C, device='cuda', dtype=torch.uint8)
    o = torch.empty_like(x)
    stats = torch.rand(G, 2, C, device='cuda') * 1000 + 1
    gamma, beta = torch.ones(C, device='cuda'), torch.zeros(C, device='cuda')
    bn = dict(stats=stats, group_imgs=32, gamma=gamma, beta=beta, act='relu', eps=1e-5)
    rin, rout = x.numel() * 2, y.numel() * 2
    res = {}
    for name, fn, by in (
            ('pool', lambda: ops.pool2d_fwd(x, y, N, H, H, C, P, P, 3, 2, 1, True), rin + rout),
            ('pool_argmax', lambda: ops.pool2d_fwd(x, y, N, H, H, C, P, P, 3, 2, 1, True, a8),
             rin + rout + a8.numel()),
            ('pool_bn', lambda: ops.pool2d_fwd(x, y, N, H, H, C, P, P, 3, 2, 1, True, bn=bn),
             rin + rout),
            ('bn_apply', lambda: ops.bn_apply(x, stats, gamma, beta, o, N * H * H, C,
                                              group_rows=32 * H * H, act='relu'), 2 * rin)):
        t = gtime(fn, reps=4)
        res[name] = dict(us=round(t, 1), tbs=round(by / t / 1e6, 2))
    print(json.dumps(dict(batch=N, **res)), flush=True)


if __name__ == '__main__':
    main()
