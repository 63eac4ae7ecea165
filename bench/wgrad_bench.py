"""Standalone weight-gradient kernel (csrc/wgrad.hip) on engine shapes, graph-timed, with and
without the XCD-aware block renumbering (``wgrad_configure``).

    python bench/wgrad_bench.py

One JSON line per (shape, xcd): the plan, microseconds, TF/s over the padded columns, and
whether the result equals the other setting's (fp32 split sums: within 1e-3 relative).
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
    from mercury_amd.ops.conv import ConvSpec, wgrad_plan, wgrad_slab_bytes
    lib = ops.lib()
    dev = 'cuda'
    for name, N, H, C, K, R, st, pd in SHAPES:
        sp = ConvSpec(N, H, H, C, K, R, R, st, pd)
        torch.manual_seed(0)
        x = ops.to_nhwc(torch.randn(N, C, H, H, device=dev).to(torch.bfloat16).float())
        dy = (torch.randn(sp.M * K, device=dev) * 0.1).to(torch.bfloat16)
        dw = torch.zeros(K * R * R * C, device=dev)
        plan = wgrad_plan(sp)
        nsl = wgrad_slab_bytes(sp, plan)
        slab = torch.zeros(max(1, (nsl + 3) // 4), device=dev) if nsl else None
        flop = 2.0 * sp.M * K * R * R * sp.Cp
        ref = None
        for xcd in (0, 1):
            lib.wgrad_configure(xcd)

            def fn():
                if slab is None:
                    dw.zero_()
                ops.conv_wgrad(dy, x, dw, sp, plan=plan, slab=slab)
            us = gtime(fn, reps=args.reps)
            fn()
            torch.cuda.synchronize()
            ok = None
            if ref is None:
                ref = dw.clone()
            else:
                ok = bool(((dw - ref).abs().max() <= 1e-3 * ref.abs().max()).item())
            print(json.dumps({'shape': name, 'plan': list(plan[:3]), 'xcd': xcd,
                              'us': round(us, 2), 'tflops': round(flop / us / 1e6, 1),
                              'equal': ok}), flush=True)
        lib.wgrad_configure(0)


if __name__ == '__main__':
    main()
