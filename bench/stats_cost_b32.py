"""What the ghost-BN statistics epilogue costs the B = 32 train-forward convs (graph-timed):
each conv with and without its statistics output, on the engine's plan.

    python bench/stats_cost_b32.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from gtime import gtime  # noqa: E402

SHAPES = [(32, 32, 64, 64, 1), (32, 16, 128, 128, 1), (32, 8, 256, 256, 1), (32, 4, 512, 512, 1),
          (32, 32, 64, 128, 2), (32, 16, 128, 256, 2), (32, 8, 256, 512, 2)]


def main():
    import torch
    from mercury_amd import ops
    from mercury_amd.ops import hconv as H
    from mercury_amd.ops.conv import ConvSpec, fwd_plan, slab_bytes
    ops.lib()
    for (N, Hh, C, K, st) in SHAPES:
        sp = ConvSpec(N, Hh, Hh, C, K, 3, 3, st, 1)
        x = ops.to_nhwc(torch.randn(N, C, Hh, Hh, device='cuda').to(torch.bfloat16).float())
        wk, _ = ops.pack_conv_weight(torch.randn(K, C, 3, 3, device='cuda') * 0.05)
        y = torch.empty(sp.M * K, dtype=torch.bfloat16, device='cuda')
        stats = torch.zeros(2 * K, device='cuda')
        hp = H.engine_plan(sp, train=True)
        row = {'shape': [N, Hh, C, K, st]}
        if hp is not None:
            slab = torch.zeros(max(4, slab_bytes(sp.M, K, *hp) // 4 + 1), device='cuda')
            row['plan'] = ['hconv'] + list(hp)
            row['stats_us'] = round(gtime(lambda: H.hconv_fwd(x, wk, y, sp, hp, stats=stats,
                                                              slab=slab), reps=16), 2)
            row['nostats_us'] = round(gtime(lambda: H.hconv_fwd(x, wk, y, sp, hp, slab=slab),
                                            reps=16), 2)
        else:
            p = fwd_plan(sp)
            slab = torch.zeros(max(4, slab_bytes(sp.M, K, *p[:3]) // 4 + 1), device='cuda')
            row['plan'] = ['igemm'] + list(p)
            row['stats_us'] = round(gtime(lambda: ops.conv_fwd(x, wk, y, sp, stats=stats,
                                                               slab=slab, plan=p), reps=16), 2)
            row['nostats_us'] = round(gtime(lambda: ops.conv_fwd(x, wk, y, sp, slab=slab,
                                                                 plan=p), reps=16), 2)
        print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
