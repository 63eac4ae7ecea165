"""Train-batch (B=32) MobileNetV2-CIFAR backward helpers, graph-timed: the BN-backward reduce
and the depthwise wgrad at every distinct shape of the net.  The launch knobs are read once per
process (MERCURY_BNRED_PT, MERCURY_DW_WG_THREADS), so run one process per setting.

    python bench/small_bwd_bench.py --tag T
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

# (C, H) of the expanded MobileNetV2-CIFAR layers (stride-1 depthwise input) at B=32
SHAPES = [(96, 32), (144, 32), (144, 16), (192, 16), (192, 8), (384, 8), (576, 8), (576, 4),
          (960, 4)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--tag', default='')
    ap.add_argument('--batch', type=int, default=32)
    a = ap.parse_args()
    import torch
    from mercury_amd import ops
    ops.lib()
    N = a.batch
    tot_red = tot_wg = 0.0
    rows = []
    for C, H in SHAPES:
        M = N * H * H
        t = lambda *s: torch.randn(*s, device='cuda')                       # noqa: E731
        dout, out, y = (t(M * C).to(torch.bfloat16) for _ in range(3))
        stats = torch.stack([t(C) * M * 0.1, (t(C).abs() + 1) * M]).contiguous()
        gamma = torch.ones(C, device='cuda')
        sums = torch.zeros(ops.sums_numel(C), device='cuda')
        dy = torch.empty_like(y)
        r = gtime(lambda: ops.bn_bwd(dout, out, y, stats, gamma, sums, dy, M, C,
                                     zero_sums=False, reduce=True), reps=8)
        x = t(M * C).to(torch.bfloat16)
        g = t(M * C).to(torch.bfloat16)
        dw = torch.zeros(C * 9, device='cuda')
        w = gtime(lambda: ops.dwconv_wgrad(g, x, dw, N, H, H, C, H, H, 1, 1), reps=8)
        tot_red += r
        tot_wg += w
        rows.append(dict(C=C, H=H, bn_bwd_us=round(r, 1), dw_wgrad_us=round(w, 1)))
    print(json.dumps(dict(tag=a.tag, env={k: v for k, v in os.environ.items()
                                           if k.startswith('MERCURY_')},
                          bn_bwd_total_us=round(tot_red, 1), dw_wgrad_total_us=round(tot_wg, 1),
                          rows=rows)), flush=True)


if __name__ == '__main__':
    main()
