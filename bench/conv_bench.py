"""Per-layer conv benchmark: our MFMA implicit-GEMM kernels vs PyTorch-ROCm (MIOpen).

Times forward / dgrad / wgrad for every distinct ResNet-18 CIFAR conv shape at the
train batch (32) and the scoring batch (320), interleaving the two implementations
in one process (methodology rule: A/B in one process, median of N).  MIOpen runs
bf16 NCHW via torch.nn.functional.conv2d / torch.ops.aten.convolution_backward.

    python bench/conv_bench.py [--iters 50] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [  # C, K, H, R, stride, pad
    (3, 64, 32, 3, 1, 1), (64, 64, 32, 3, 1, 1), (64, 128, 32, 3, 2, 1), (128, 128, 16, 3, 1, 1),
    (64, 128, 32, 1, 2, 0), (128, 256, 16, 3, 2, 1), (256, 256, 8, 3, 1, 1),
    (128, 256, 16, 1, 2, 0), (256, 512, 8, 3, 2, 1), (512, 512, 4, 3, 1, 1),
    (256, 512, 8, 1, 2, 0)]


def timeit(fn, iters):
    import torch
    st = [torch.cuda.Event(enable_timing=True) for _ in range(iters + 1)]
    fn()
    torch.cuda.synchronize()
    st[0].record()
    for i in range(iters):
        fn()
        st[i + 1].record()
    torch.cuda.synchronize()
    ts = sorted(st[i].elapsed_time(st[i + 1]) for i in range(iters))
    return ts[len(ts) // 2] * 1e3  # median us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=50)
    ap.add_argument('--json', default='')
    args = ap.parse_args()
    import torch
    import torch.nn.functional as F
    from mercury_amd import ops
    from mercury_amd.ops.conv import ConvSpec, dgrad_plan, fwd_plan, slab_bytes
    dev = 'cuda'
    rows = []
    for N in (32, 320):
        for (C, K, H, R, st, pd) in SHAPES:
            sp = ConvSpec(N, H, H, C, K, R, R, st, pd)
            x = torch.randn(N, C, H, H, device=dev, dtype=torch.bfloat16)
            w = torch.randn(K, C, R, R, device=dev, dtype=torch.bfloat16) * 0.05
            gy = torch.randn(N, K, sp.P, sp.Q, device=dev, dtype=torch.bfloat16)
            xn = ops.to_nhwc(x.float())
            wk, wt = ops.pack_conv_weight(w.float())
            gyn = ops.to_nhwc(gy.float())
            y = torch.empty(sp.M, K, dtype=torch.bfloat16, device=dev)
            stats = torch.zeros(2, K, device=dev)
            pf = fwd_plan(sp)
            slab = torch.zeros(max(1, slab_bytes(sp.M, K, *pf) // 4), device=dev)
            ours_f = timeit(lambda: ops.conv_fwd(xn, wk, y, sp, stats=stats, slab=slab, plan=pf),
                            args.iters)
            ref_f = timeit(lambda: F.conv2d(x, w, stride=st, padding=pd), args.iters)
            flops = sp.flops()
            r = dict(N=N, C=C, K=K, H=H, R=R, stride=st, gflop=flops / 1e9,
                     fwd_us=ours_f, fwd_miopen_us=ref_f, fwd_tflops=flops / ours_f / 1e6,
                     fwd_plan=list(pf))
            dw = torch.zeros(K, R, R, C, device=dev)
            r['wgrad_us'] = timeit(lambda: ops.conv_wgrad(gyn, xn, dw, sp), args.iters)
            if C % 8 == 0:
                dx = torch.empty(N * H * H, C, dtype=torch.bfloat16, device=dev)
                pd_ = dgrad_plan(sp)
                slab2 = torch.zeros(max(1, slab_bytes(N * H * H, C, *pd_) // 4), device=dev)
                r['dgrad_us'] = timeit(lambda: ops.conv_dgrad(gyn, wt, dx, sp, slab=slab2,
                                                              plan=pd_), args.iters)
                xr = x.clone().requires_grad_(False)

                def ref_bwd():
                    torch.ops.aten.convolution_backward(gy, xr, w, None, [st, st], [pd, pd],
                                                        [1, 1], False, [0, 0], 1,
                                                        [True, True, False])
                r['bwd_miopen_us'] = timeit(ref_bwd, args.iters)
            rows.append(r)
            print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v)
                              for k, v in r.items()}), flush=True)
    tot = {k: sum(r.get(k, 0) for r in rows) for k in
           ('fwd_us', 'fwd_miopen_us', 'wgrad_us', 'dgrad_us', 'bwd_miopen_us')}
    print(json.dumps({'totals_us': {k: round(v, 1) for k, v in tot.items()}}))
    if args.json:
        with open(args.json, 'w') as f:
            json.dump({'rows': rows, 'totals_us': tot}, f, indent=1)


if __name__ == '__main__':
    main()
