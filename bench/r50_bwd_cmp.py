"""ResNet-50/224 backward convs at the train batch: the engine's dgrad / wgrad / pair plans
against alternative plans and hipBLASLt.

    python bench/r50_bwd_cmp.py [--batch 128] [--sweep]

Per distinct conv of the ResNet-50 forward (SHAPES of r50_conv_cmp.py, with its count) this
graph-times (``gtime``): the pair launch with the default plans, dgrad alone, wgrad alone, and
-- for the 1x1 stride-1 convs, plain GEMMs in NHWC -- ``torch.matmul`` for the dgrad
(dy[M][K] @ W[K][C]) and the wgrad (dy^T[K][M] @ x[M][C]).  ``--sweep`` also times a grid of
wgrad plans.  One JSON line per shape plus a summary.
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
from r50_conv_cmp import SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=128)
    ap.add_argument('--sweep', action='store_true')
    a = ap.parse_args()
    import torch
    from mercury_amd import ops
    from mercury_amd.ops.conv import ConvSpec, dgrad_plan, slab_bytes, wgrad_plan
    ops.lib()
    dev = 'cuda'
    tot = dict(pair=0.0, dgrad=0.0, wgrad=0.0, best=0.0)
    for C, K, H, R, st, cnt in SHAPES:
        if C < 8:
            continue                      # the stem has no dgrad; its wgrad is timed elsewhere
        pad = R // 2
        sp = ConvSpec(a.batch, H, H, C, K, R, R, st, pad, 0)
        Mx = a.batch * H * H
        x = torch.randn(Mx * sp.Cp, device=dev).to(torch.bfloat16)
        wt = (torch.randn(K * R * R * sp.Cp, device=dev) * 0.05).to(torch.bfloat16)
        dy = torch.randn(sp.M * K, device=dev).to(torch.bfloat16)
        dx = torch.empty(Mx * sp.Cp, device=dev, dtype=torch.bfloat16)
        dw = torch.zeros(K * R * R * C, device=dev)
        dp, wp = dgrad_plan(sp), wgrad_plan(sp)
        slab = torch.zeros(max(1, slab_bytes(Mx, sp.Cp, dp[0], dp[1], dp[2]) // 4 + 1),
                           device=dev)
        fl = sp.flops()                   # one GEMM's FLOPs (dgrad and wgrad each have this)
        t_pair = gtime(lambda: ops.conv_bwd(dy, wt, dx, x, dw, sp, dplan=dp, wplan=wp,
                                            slab=slab), reps=4)
        t_d = gtime(lambda: ops.conv_dgrad(dy, wt, dx, sp, slab=slab, plan=dp), reps=4)
        t_w = gtime(lambda: ops.conv_wgrad(dy, x, dw, sp, plan=wp), reps=4)
        rec = dict(C=C, K=K, H=H, R=R, stride=st, count=cnt, M=sp.M, dplan=list(dp),
                   wplan=list(wp), pair_us=round(t_pair, 1),
                   pair_tfs=round(2 * fl / t_pair / 1e6, 1), dgrad_us=round(t_d, 1),
                   dgrad_tfs=round(fl / t_d / 1e6, 1), wgrad_us=round(t_w, 1),
                   wgrad_tfs=round(fl / t_w / 1e6, 1))
        best_w = t_w
        if a.sweep:
            from mercury_amd.ops.conv import wgrad_slab_bytes
            cands = [(bm, bn, s) for bm, bn in ((128, 128), (64, 64), (128, 64), (64, 128))
                     for s in (1, 2, 4, 8, 16, 32, 64, 128)]
            wslab = torch.zeros(max(wgrad_slab_bytes(sp, c) for c in cands) // 4 + 1,
                                device=dev)
            sw = {}
            for c in cands:
                for mode in ('atomic', 'slab'):
                    if mode == 'slab' and wgrad_slab_bytes(sp, c) == 0:
                        continue
                    sl = wslab if mode == 'slab' else None
                    t = gtime(lambda: ops.conv_wgrad(dy, x, dw, sp, plan=c, slab=sl), reps=2,
                              iters=3)
                    sw['%s %d,%d,%d' % ((mode,) + c)] = round(t, 1)
            for mode in ('atomic', 'slab'):
                ks = [k for k in sw if k.startswith(mode)]
                if ks:
                    k = min(ks, key=sw.get)
                    rec['wgrad_best_' + mode] = [k, sw[k]]
                    best_w = min(best_w, sw[k])
            rec['sweep'] = sw
            del wslab
        if R == 1 and st == 1:
            dya = dy.view(sp.M, K)
            wa = wt.view(sp.Cp, K).t()    # wt is [C][K] for a 1x1: W^T as [K][C]
            dxa = dx.view(Mx, sp.Cp)
            xa = x.view(Mx, sp.Cp)
            dwa = torch.empty(K, sp.Cp, device=dev, dtype=torch.bfloat16)
            t_md = gtime(lambda: torch.matmul(dya, wa, out=dxa), reps=4)
            t_mw = gtime(lambda: torch.matmul(dya.t(), xa, out=dwa), reps=4)
            rec.update(mm_dgrad_us=round(t_md, 1), mm_dgrad_tfs=round(fl / t_md / 1e6, 1),
                       mm_wgrad_us=round(t_mw, 1), mm_wgrad_tfs=round(fl / t_mw / 1e6, 1))
        tot['pair'] += cnt * t_pair
        tot['dgrad'] += cnt * t_d
        tot['wgrad'] += cnt * t_w
        tot['best'] += cnt * (t_d + best_w)
        print(json.dumps(rec), flush=True)
        del x, wt, dy, dx, dw, slab
        torch.cuda.empty_cache()
    print(json.dumps(dict(summary=True, batch=a.batch,
                          **{k + '_ms': round(v / 1e3, 2) for k, v in tot.items()})), flush=True)


if __name__ == '__main__':
    main()
