"""Depthwise 3x3 forward (csrc/dwconv.hip) at MobileNetV2-CIFAR's scoring shapes (B = 320, ten
ghost-BN groups of 32 images) with the input prologue, graph-timed with and without the fused
BN-statistics epilogue -- what the per-block statistics atomics cost at the scoring batch.

    python bench/dw_stats_bench.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from gtime import gtime  # noqa: E402

# (H, C, stride) of the depthwise convs
SHAPES = [(32, 96, 1), (32, 144, 1), (32, 144, 2), (16, 192, 1), (16, 192, 2), (8, 384, 1),
          (8, 576, 1), (8, 576, 2), (4, 960, 1)]


def main():
    import torch
    from mercury_amd import ops
    dev = 'cuda'
    N, gi = 320, 32
    for H, C, st in SHAPES:
        P = (H - 1) // st + 1
        x = torch.randn(N * H * H * C, device=dev).to(torch.bfloat16)
        w = torch.randn(C * 9, device=dev) * 0.2
        y = torch.empty(N * P * P * C, device=dev, dtype=torch.bfloat16)
        stats = torch.zeros(N // gi * 2 * C, device=dev)
        cnt = gi * H * H
        stin = torch.empty(N // gi, 2, C, device=dev)
        stin[:, 0] = torch.randn(N // gi, C, device=dev) * cnt * 0.1
        stin[:, 1] = (torch.rand(N // gi, C, device=dev) + 1.0) * cnt
        pro = dict(stats=stin.reshape(-1), gamma=torch.rand(C, device=dev) + 0.5,
                   beta=torch.randn(C, device=dev) * 0.1, act='relu6', eps=1e-5, count=cnt,
                   group_imgs=gi)
        row = {'shape': [N, H, C, st]}
        for name, s in (('stats', stats), ('nostats', None)):
            row[name] = round(gtime(lambda s=s: ops.dwconv_fwd(
                x, w, y, N, H, H, C, P, P, st, 1, stats=s, group_rows=gi * P * P, pro=pro),
                reps=8), 2)
        byt = (N * H * H * C + N * P * P * C) * 2
        row['tbps_stats'] = round(byt / row['stats'] / 1e6, 2)
        print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
