"""Split-K of the BN-prologue forward conv (igemm_pro) on MobileNetV2's train-batch project
convs (narrow output, deep input, 4x4 / 8x8 images at B = 32: 16-48 blocks per launch),
graph-timed.

    python bench/pro_split_bench.py [--all]

One JSON line per (shape, tile, splits): microseconds, with the tuned plain-conv plan marked.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from gtime import gtime  # noqa: E402

# (N, H, C, K): MobileNetV2-CIFAR project / expand convs at the train batch
SHAPES = [(32, 4, 960, 160), (32, 4, 960, 320), (32, 4, 576, 160), (32, 8, 576, 96),
          (32, 8, 384, 64), (32, 8, 384, 96), (32, 16, 192, 32), (32, 16, 144, 32),
          # expand / remaining 1x1 convs (--all)
          (32, 4, 160, 960), (32, 4, 320, 1280), (32, 4, 160, 320), (32, 8, 64, 384),
          (32, 8, 96, 576), (32, 8, 192, 64), (32, 8, 64, 96), (32, 16, 32, 192),
          (32, 32, 24, 144), (32, 32, 16, 96), (32, 32, 96, 24), (32, 32, 144, 24),
          (32, 32, 32, 16), (32, 32, 32, 32)]


def main():
    import torch
    from mercury_amd import ops
    from mercury_amd.ops import tune
    from mercury_amd.ops.conv import ConvSpec, fwd_plan, slab_bytes
    dev = 'cuda'
    for N, H, C, K in (SHAPES if '--all' in sys.argv else SHAPES[:8]):
        sp = ConvSpec(N, H, H, C, K, 1, 1, 1, 0)
        torch.manual_seed(0)
        y = ops.to_nhwc(torch.randn(N, C, H, H, device=dev))
        wk, _ = ops.pack_conv_weight(torch.randn(K, C, 1, 1, device=dev) * 0.05)
        cnt = N * H * H
        st = torch.empty(2, C, device=dev)
        st[0] = torch.randn(C, device=dev) * cnt * 0.1
        st[1] = (torch.rand(C, device=dev) + 1.0) * cnt
        pro = dict(stats=st.reshape(-1), gamma=torch.rand(C, device=dev) + 0.5,
                   beta=torch.randn(C, device=dev) * 0.1, act='relu6', eps=1e-5, count=cnt)
        out = torch.empty(sp.M * K, dtype=torch.bfloat16, device=dev)
        ost = torch.zeros(2 * K, device=dev)
        tuned = tuple(tune.fwd_plan_for(sp, fwd_plan(sp))[:3])
        ref = None
        for bm, bn in ((64, 64), (64, 128), (128, 64), (128, 128)):
            for s in (1, 2, 3, 4, 6, 8):
                if s > max(1, (C // 8 + 7) // 8):
                    continue
                p = (bm, bn, s)
                slab = torch.zeros(max(4, slab_bytes(sp.M, K, *p) // 4 + 1), device=dev)

                def fn():
                    ost.zero_()
                    ops.conv_fwd(y, wk, out, sp, stats=ost, slab=slab, plan=p, pro=pro)
                try:
                    us = gtime(fn, reps=16)
                except Exception as e:  # noqa: BLE001
                    print(json.dumps({'shape': [N, H, C, K], 'plan': list(p), 'error': str(e)}))
                    continue
                fn()
                torch.cuda.synchronize()
                if ref is None:
                    ref = out.float().clone()
                d = (out.float() - ref).abs().max().item()
                print(json.dumps({'shape': [N, H, C, K], 'plan': list(p), 'us': round(us, 2),
                                  'tuned': p == tuned, 'maxdiff': round(d, 4)}), flush=True)


if __name__ == '__main__':
    main()
