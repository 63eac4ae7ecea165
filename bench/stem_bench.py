"""Stem conv: the dense-k stem kernel (csrc/stem.hip) vs the generic implicit GEMM (igemm, 3
channels padded to 8 per tap), graph-timed, with the ghost-BN statistics epilogue both ways.

    python bench/stem_bench.py

One JSON line per preset stem: ResNet-50 7x7/2 at the scoring batch 1280 and train batch 128,
ResNet-18 3x3 at 320 / 32, MobileNetV2 3x3 -> 32 at 320, speech VGG 3x3 1 -> 64 at 320.
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from gtime import gtime  # noqa: E402

# name, N, H, W, C, K, R, stride, pad, group_imgs
STEMS = [('resnet50_224', 1280, 224, 224, 3, 64, 7, 2, 3, 32),
         ('resnet50_224', 128, 224, 224, 3, 64, 7, 2, 3, 0),
         ('resnet18_cifar', 320, 32, 32, 3, 64, 3, 1, 1, 32),
         ('resnet18_cifar', 32, 32, 32, 3, 64, 3, 1, 1, 0),
         ('mobilenetv2_cifar', 320, 32, 32, 3, 32, 3, 1, 1, 32),
         ('vgg11_speech', 320, 101, 161, 1, 64, 3, 1, 1, 32)]


def main():
    import torch
    from mercury_amd import ops
    from mercury_amd.ops.conv import ConvSpec, fwd_plan, slab_bytes
    ops.lib()
    for name, N, H, W, C, K, R, st, pad, gi in STEMS:
        sp = ConvSpec(N, H, W, C, K, R, R, st, pad)
        if gi:
            sp.group_rows = gi * sp.P * sp.Q
        G = N // gi if gi else 1
        x = torch.randn(N, H, W, 8, device='cuda').to(torch.bfloat16)
        x[..., C:] = 0
        w = torch.randn(K, R, R, 8, device='cuda').to(torch.bfloat16) * 0.1
        w[..., C:] = 0
        y = torch.empty(sp.M * K, device='cuda', dtype=torch.bfloat16)
        stats = torch.zeros(G * 2 * K, device='cuda')
        plan = fwd_plan(sp)
        slab = torch.zeros(max(1, slab_bytes(sp.M, K, *plan) // 4 + 1), device='cuda')
        t_ig = gtime(lambda: ops.conv_fwd(x, w, y, sp, stats=stats, slab=slab, plan=plan), reps=8)
        t_st = gtime(lambda: ops.stem_fwd(x, w, y, sp, stats=stats), reps=8)
        t_ns = gtime(lambda: ops.stem_fwd(x, w, y, sp), reps=8)
        print(json.dumps(dict(stem=name, N=N, R=R, stride=st, K=K, igemm_us=round(t_ig, 1),
                              stem_us=round(t_st, 1), stem_nostats_us=round(t_ns, 1),
                              stem_tfs=round(2.0 * sp.M * K * R * R * C / t_st / 1e6, 1),
                              stem_gbs=round((y.numel() * 2 + x.numel() * 2) / t_st / 1e3, 1))),
              flush=True)
        del x, w, y, stats, slab
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
