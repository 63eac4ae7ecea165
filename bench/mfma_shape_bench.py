"""v_mfma_f32_16x16x32_bf16 vs v_mfma_f32_32x32x16_bf16 on MI355X (csrc/tools/ubench.hip).

Same output tile per wave (64 x 64), one wave per SIMD (256-thread blocks, one per CU), random
bf16 operands, operands in registers (lds=0) or re-read from LDS every K step (lds=1).  The two
shapes are interleaved over several rounds in one process (cdna_hip_programming.md §5.4 rule
24) after a 2 s warm-up so the chip runs at the clock it holds under load.

    python bench/mfma_shape_bench.py [--trips 20000] [--rounds 5]

Prints one JSON line per (shape, lds) with median / min wall-clock TFLOP/s.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--trips', type=int, default=20000)
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--grid', type=int, default=256)
    args = ap.parse_args()
    import ctypes
    import torch
    from mercury_amd import _build
    from mercury_amd.ops import ptr, stream_ptr
    L = ctypes.CDLL(_build.build_tools(verbose=False))   # csrc/tools/ubench.hip (C ABI)
    L.ubench_mfma.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                              ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    src = (torch.rand(1 << 20, device='cuda') * 2 - 1).to(torch.bfloat16)
    out = torch.empty(args.grid * 256, device='cuda')
    flop = 524288.0 * 4 * args.grid * args.trips      # per trip per wave, 4 waves per block

    def run(shape, lds):
        L.ubench_mfma(shape, lds, ptr(src), args.trips, args.grid, ptr(out), stream_ptr())

    t_end = time.time() + 2.0                          # clock settles under sustained load
    while time.time() < t_end:
        run(16, 1)
        run(32, 1)
    torch.cuda.synchronize()
    res = {}
    for _ in range(args.rounds):
        for shape in (16, 32):
            for lds in (0, 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run(shape, lds)
                e1.record()
                torch.cuda.synchronize()
                res.setdefault((shape, lds), []).append(flop / (e0.elapsed_time(e1) * 1e-3) / 1e12)
    for (shape, lds), v in sorted(res.items()):
        v.sort()
        print(json.dumps({'mfma': '%dx%dx%d_bf16' % ((16, 16, 32) if shape == 16 else (32, 32, 16)),
                          'operands': 'lds' if lds else 'registers', 'grid': args.grid,
                          'tflops_median': round(v[len(v) // 2], 1), 'tflops_max': round(v[-1], 1),
                          'rounds': len(v)}), flush=True)


if __name__ == '__main__':
    main()
