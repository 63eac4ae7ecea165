"""Standalone weight-gradient kernel (csrc/wgrad.hip) on engine shapes, graph-timed: the
engine's plan and 2x / 4x its pixel splits (atomic splits add into a zeroed gradient, which
the engine zeroes once per step; here the zeroing runs outside the timed graph).

    python bench/wgrad_bench.py

One JSON line per (shape, plan): microseconds, TF/s over the padded columns, and whether the
result matches the engine plan's (fp32 split sums: within 1e-3 relative).  (An XCD-grouped
block order measured equal, profiles/r6/wgrad_xcd_rejected.jsonl.)
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from gtime import gtime  # noqa: E402

# (name, N, H, C, K, R, stride, pad)
SHAPES = [
    ('r50_stem_b128', 128, 224, 3, 64, 7, 2, 3),
    ('r50_l1_3x3_b128', 128, 56, 64, 64, 3, 1, 1),
    ('r50_l1_1x1_b128', 128, 56, 256, 64, 1, 1, 0),
    ('r18_stem_b32', 32, 32, 3, 64, 3, 1, 1),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=8)
    args = ap.parse_args()
    import torch
    from mercury_amd import ops
    from mercury_amd.ops.conv import ConvSpec, wgrad_plan
    ops.lib()
    dev = 'cuda'
    for name, N, H, C, K, R, st, pd in SHAPES:
        sp = ConvSpec(N, H, H, C, K, R, R, st, pd)
        torch.manual_seed(0)
        x = ops.to_nhwc(torch.randn(N, C, H, H, device=dev).to(torch.bfloat16).float())
        dy = (torch.randn(sp.M * K, device=dev) * 0.1).to(torch.bfloat16)
        dw = torch.zeros(K * R * R * C, device=dev)
        base = wgrad_plan(sp)
        flop = 2.0 * sp.M * K * R * R * sp.Cp
        ref = None
        for mult in (1, 2, 4):
            plan = (base[0], base[1], base[2] * mult)

            def fn():      # atomic splits into the zeroed gradient, as the engine's stem runs it
                ops.conv_wgrad(dy, x, dw, sp, plan=plan)
            dw.zero_()
            fn()
            torch.cuda.synchronize()
            got = dw.clone()
            us = gtime(fn, reps=args.reps)
            ok = None
            if ref is None:
                ref = got
            else:
                ok = bool(((got - ref).abs().max() <= 1e-3 * ref.abs().max()).item())
            print(json.dumps({'shape': name, 'plan': list(plan), 'us': round(us, 2),
                              'tflops': round(flop / us / 1e6, 1), 'equal': ok}), flush=True)


if __name__ == '__main__':
    main()
