"""What the ghost-BN statistics epilogue costs the forward convs at the scoring batch: each conv
graph-timed with and without its stats (one atomic pair per channel per block), on the
ResNet-18 / MobileNetV2 B=320 shapes and the depthwise forward.

    python bench/stats_cost.py
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from gtime import gtime  # noqa: E402

# N, H, C, K, R, stride
SHAPES = [(320, 32, 64, 64, 3, 1), (320, 16, 128, 128, 3, 1), (320, 32, 64, 128, 1, 2),
          (320, 32, 16, 96, 1, 1), (320, 32, 96, 24, 1, 1), (320, 16, 32, 192, 1, 1),
          (320, 8, 64, 384, 1, 1), (32, 32, 64, 64, 3, 1), (32, 32, 16, 96, 1, 1)]
DW = [(320, 32, 96, 1), (320, 32, 144, 1), (320, 16, 192, 1), (32, 32, 96, 1), (32, 32, 144, 1)]


def main():
    import torch
    from mercury_amd import ops
    from mercury_amd.ops.conv import ConvSpec, fwd_plan, slab_bytes
    ops.lib()
    for N, H, C, K, R, st in SHAPES:
        sp = ConvSpec(N, H, H, C, K, R, R, st, R // 2)
        gi = 32 if N > 32 else 0
        if gi:
            sp.group_rows = gi * sp.P * sp.Q
        G = N // gi if gi else 1
        x = torch.randn(N * H * H * sp.Cp, device='cuda').to(torch.bfloat16)
        w = (torch.randn(K * R * R * sp.Cp, device='cuda') * 0.05).to(torch.bfloat16)
        y = torch.empty(sp.M * K, device='cuda', dtype=torch.bfloat16)
        stats = torch.zeros(G * 2 * K, device='cuda')
        plan = fwd_plan(sp)
        slab = torch.zeros(max(1, slab_bytes(sp.M, K, *plan) // 4 + 1), device='cuda')
        t1 = gtime(lambda: ops.conv_fwd(x, w, y, sp, stats=stats, slab=slab, plan=plan), reps=8)
        t0 = gtime(lambda: ops.conv_fwd(x, w, y, sp, slab=slab, plan=plan), reps=8)
        print(json.dumps(dict(kind='conv', N=N, H=H, C=C, K=K, R=R, stride=st, plan=list(plan),
                              stats_us=round(t1, 1), nostats_us=round(t0, 1))), flush=True)
    # the dgrad + wgrad pair with / without the fused BN-backward sums (train batch)
    from mercury_amd.ops.conv import dgrad_plan, wgrad_plan
    for N, H, C, K, R, st in [(32, 32, 64, 64, 3, 1), (32, 16, 128, 128, 3, 1),
                              (32, 32, 96, 16, 1, 1), (32, 32, 16, 96, 1, 1)]:
        sp = ConvSpec(N, H, H, C, K, R, R, st, R // 2)
        Mx = N * H * H
        x = torch.randn(Mx * sp.Cp, device='cuda').to(torch.bfloat16)
        wt = (torch.randn(C * R * R * K, device='cuda') * 0.05).to(torch.bfloat16)
        dy = torch.randn(sp.M * K, device='cuda').to(torch.bfloat16)
        dx = torch.empty(Mx * sp.Cp, device='cuda', dtype=torch.bfloat16)
        dw = torch.zeros(K * R * R * C, device='cuda')
        yb = torch.randn(Mx * sp.Cp, device='cuda').to(torch.bfloat16)
        ob = torch.relu(yb.float()).to(torch.bfloat16)
        bst = torch.stack([yb.float().view(Mx, -1).sum(0), yb.float().view(Mx, -1).pow(2).sum(0)])
        sums = torch.zeros(ops.sums_numel(sp.Cp), device='cuda')
        bw = dict(out=ob, y=yb, stats=bst.contiguous().view(-1), sums=sums, act='relu', eps=1e-5)
        dp, wp = dgrad_plan(sp), wgrad_plan(sp)
        slab = torch.zeros(max(1, slab_bytes(Mx, sp.Cp, *dp) // 4 + 1), device='cuda')
        t1 = gtime(lambda: ops.conv_bwd(dy, wt, dx, x, dw, sp, dplan=dp, wplan=wp, slab=slab,
                                        bw=bw), reps=8)
        t0 = gtime(lambda: ops.conv_bwd(dy, wt, dx, x, dw, sp, dplan=dp, wplan=wp, slab=slab),
                   reps=8)
        print(json.dumps(dict(kind='bwd_pair', N=N, H=H, C=C, K=K, R=R, dplan=list(dp),
                              bw_us=round(t1, 1), nobw_us=round(t0, 1))), flush=True)
    for N, H, C, st in DW:
        P = (H - 1) // st + 1
        x = torch.randn(N * H * H * C, device='cuda').to(torch.bfloat16)
        w = torch.randn(C * 9, device='cuda') * 0.1
        y = torch.empty(N * P * P * C, device='cuda', dtype=torch.bfloat16)
        gi = 32 if N > 32 else N
        stats = torch.zeros((N // gi) * 2 * C, device='cuda')
        t1 = gtime(lambda: ops.dwconv_fwd(x, w, y, N, H, H, C, P, P, st, 1, stats=stats,
                                          group_rows=gi * P * P), reps=8)
        t0 = gtime(lambda: ops.dwconv_fwd(x, w, y, N, H, H, C, P, P, st, 1), reps=8)
        print(json.dumps(dict(kind='dw', N=N, H=H, C=C, stride=st, stats_us=round(t1, 1),
                              nostats_us=round(t0, 1))), flush=True)


if __name__ == '__main__':
    main()
