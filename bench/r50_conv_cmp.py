"""ResNet-50/224 forward convs at the scoring batch: the engine's igemm plan vs hipBLASLt.

    python bench/r50_conv_cmp.py [--batch 1280] [--group 32]

For every distinct conv of the ResNet-50 forward (with its count per forward) this times, by
HIP-graph replay (``gtime``): the igemm conv with the engine's plan and its ghost-BN-statistics
epilogue, and -- for the 1x1 stride-1 convs, which are plain GEMMs in NHWC -- ``torch.matmul``
(hipBLASLt) of the same bf16 operands without statistics.  One JSON line per shape plus a
summary: where the ResNet-50 scoring pass loses time against the library GEMM.
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

# C, K, H(in), R, stride, count per forward (torchvision-v1.5 bottleneck: stride on conv2)
SHAPES = [
    (3, 64, 224, 7, 2, 1),
    (64, 64, 56, 1, 1, 1), (256, 64, 56, 1, 1, 2), (64, 64, 56, 3, 1, 3), (64, 256, 56, 1, 1, 4),
    (256, 128, 56, 1, 1, 1), (128, 128, 56, 3, 2, 1), (256, 512, 56, 1, 2, 1),
    (512, 128, 28, 1, 1, 3), (128, 128, 28, 3, 1, 3), (128, 512, 28, 1, 1, 4),
    (512, 256, 28, 1, 1, 1), (256, 256, 28, 3, 2, 1), (512, 1024, 28, 1, 2, 1),
    (1024, 256, 14, 1, 1, 5), (256, 256, 14, 3, 1, 5), (256, 1024, 14, 1, 1, 6),
    (1024, 512, 14, 1, 1, 1), (512, 512, 14, 3, 2, 1), (1024, 2048, 14, 1, 2, 1),
    (2048, 512, 7, 1, 1, 2), (512, 512, 7, 3, 1, 2), (512, 2048, 7, 1, 1, 3),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=1280)
    ap.add_argument('--group', type=int, default=32)
    a = ap.parse_args()
    import torch
    from mercury_amd import ops
    from mercury_amd.ops.conv import ConvSpec, fwd_plan, slab_bytes
    ops.lib()
    dev = 'cuda'
    tot_ig = tot_best = 0.0
    for C, K, H, R, st, cnt in SHAPES:
        pad = R // 2
        sp = ConvSpec(a.batch, H, H, C, K, R, R, st, pad, 0)
        sp.group_rows = a.group * sp.P * sp.Q
        plan = fwd_plan(sp)
        x = torch.randn(a.batch * H * H * sp.Cp, device=dev).to(torch.bfloat16)
        w = (torch.randn(K * R * R * sp.Cp, device=dev) * 0.05).to(torch.bfloat16)
        y = torch.empty(sp.M * K, device=dev, dtype=torch.bfloat16)
        stats = torch.zeros(a.batch // a.group * 2 * K, device=dev)
        slab = torch.zeros(max(1, slab_bytes(sp.M, K, plan[0], plan[1], plan[2]) // 4 + 1),
                           device=dev)
        t_ig = gtime(lambda: ops.conv_fwd(x, w, y, sp, stats=stats, slab=slab, plan=plan), reps=4)
        rec = dict(C=C, K=K, H=H, R=R, stride=st, count=cnt, M=sp.M, plan=list(plan),
                   igemm_us=round(t_ig, 1), igemm_tfs=round(sp.flops() / t_ig / 1e6, 1))
        best = t_ig
        if R == 1 and st == 1:
            xa = x.view(sp.M, C)
            wt = w.view(K, C).t()
            ya = y.view(sp.M, K)
            t_mm = gtime(lambda: torch.matmul(xa, wt, out=ya), reps=4)
            rec.update(matmul_us=round(t_mm, 1), matmul_tfs=round(sp.flops() / t_mm / 1e6, 1))
            best = min(best, t_mm)
        tot_ig += cnt * t_ig
        tot_best += cnt * best
        print(json.dumps(rec), flush=True)
        del x, w, y, stats, slab
        torch.cuda.empty_cache()
    print(json.dumps(dict(summary=True, batch=a.batch, igemm_total_ms=round(tot_ig / 1e3, 2),
                          best_total_ms=round(tot_best / 1e3, 2))), flush=True)


if __name__ == '__main__':
    main()
