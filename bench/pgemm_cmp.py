"""ResNet-50/224 and MobileNetV2 1x1 convs: persistent pointwise GEMM (pgemm) vs the igemm plan
vs hipBLASLt (torch.matmul, no statistics), graph-timed, at the scoring batch.

    python bench/pgemm_cmp.py [--batch 1280] [--group 32] [--models r50,mbv2]

One JSON line per shape: us and TF/s of each; pgemm is timed at every tile width and with the
ghost-BN statistics epilogue (what the engine needs), like igemm.
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

# C, K, H(in), stride, count per forward
R50 = [(64, 64, 56, 1, 1), (256, 64, 56, 1, 2), (64, 256, 56, 1, 4), (256, 128, 56, 1, 1),
       (256, 512, 56, 2, 1), (512, 128, 28, 1, 3), (128, 512, 28, 1, 4), (512, 256, 28, 1, 1),
       (512, 1024, 28, 2, 1), (1024, 256, 14, 1, 5), (256, 1024, 14, 1, 6),
       (1024, 512, 14, 1, 1), (1024, 2048, 14, 2, 1), (2048, 512, 7, 1, 2), (512, 2048, 7, 1, 3)]
# MobileNetV2 (CIFAR, 32x32 input; stride-1 stem): expand C -> 6C, project 6C -> C'
MBV2 = [(32, 192, 32, 1, 1), (96, 16, 32, 1, 1), (16, 96, 32, 1, 1), (96, 24, 32, 1, 1),
        (24, 144, 32, 1, 2), (144, 24, 32, 1, 1), (144, 32, 16, 1, 1), (32, 192, 16, 1, 3),
        (192, 32, 16, 1, 2), (192, 64, 8, 1, 1), (64, 384, 8, 1, 4), (384, 64, 8, 1, 3),
        (384, 96, 8, 1, 1), (96, 576, 8, 1, 3), (576, 96, 8, 1, 2), (576, 160, 4, 1, 1),
        (160, 960, 4, 1, 3), (960, 160, 4, 1, 2), (960, 320, 4, 1, 1), (320, 1280, 4, 1, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=0)
    ap.add_argument('--group', type=int, default=32)
    ap.add_argument('--models', default='r50,mbv2')
    ap.add_argument('--pro', action='store_true',
                    help='also time the input-BN prologue (pgemm pro=, modes 1 and 2) against '
                         'the bn_apply pass + igemm the engine runs without it')
    a = ap.parse_args()
    import torch
    from mercury_amd import ops
    from mercury_amd.ops.conv import ConvSpec, fwd_plan, slab_bytes
    ops.lib()
    dev = 'cuda'
    for model in a.models.split(','):
        shapes, batch = (R50, a.batch or 1280) if model == 'r50' else (MBV2, a.batch or 320)
        tot = {}
        for C, K, H, st, cnt in shapes:
            sp = ConvSpec(batch, H, H, C, K, 1, 1, st, 0, 0)
            sp.group_rows = a.group * sp.P * sp.Q
            G = batch // a.group
            x = torch.randn(batch * H * H * sp.Cp, device=dev).to(torch.bfloat16)
            w = (torch.randn(K * sp.Cp, device=dev) * 0.05).to(torch.bfloat16)
            y = torch.empty(sp.M * K, device=dev, dtype=torch.bfloat16)
            stats = torch.zeros(G * 2 * K, device=dev)
            plan = fwd_plan(sp)
            slab = torch.zeros(max(1, slab_bytes(sp.M, K, *plan) // 4 + 1), device=dev)
            rec = dict(model=model, C=C, K=K, H=H, stride=st, count=cnt, M=sp.M)
            fl = sp.flops()

            def put(name, us):
                rec[name + '_us'] = round(us, 1)
                rec[name + '_tfs'] = round(fl / us / 1e6, 1)
                tot[name] = tot.get(name, 0.0) + cnt * us
            put('igemm', gtime(lambda: ops.conv_fwd(x, w, y, sp, stats=stats, slab=slab,
                                                    plan=plan), reps=4))
            for bn in (64, 128, 256):
                put('pgemm%d' % bn, gtime(lambda: ops.pgemm_fwd(x, w, y, sp, stats=stats, bn=bn),
                                          reps=4))
            pw = st == 1 and sp.Cp <= 128
            if pw:
                put('pwconv', gtime(lambda: ops.pwconv_fwd(x, w, y, sp, stats=stats), reps=4))
            if a.pro and st == 1:
                rows = batch * H * H
                gamma = torch.ones(C, device=dev)
                beta = torch.zeros(C, device=dev)
                pst = torch.rand(G * 2 * C, device=dev) * 100 + 1
                coef = torch.zeros(G * 2 * C, device=dev)
                act_buf = torch.empty_like(x)
                res = torch.randn(rows * sp.Cp, device=dev).to(torch.bfloat16)
                grp = a.group * H * H
                for mode, r in ((1, None), (2, res)):
                    pro = dict(stats=pst, gamma=gamma, beta=beta, act='relu', coef=coef,
                               group_rows=grp, count=grp, res=r, keep=act_buf)

                    def fused():
                        ops.pgemm_fwd(x, w, y, sp, stats=stats, pro=pro)

                    def unfused():
                        ops.bn_apply(x, pst, gamma, beta, act_buf, rows, C, group_rows=grp,
                                     act='relu', res=r)
                        ops.conv_fwd(act_buf, w, y, sp, stats=stats, slab=slab, plan=plan)
                    put('pro%d' % mode, gtime(fused, reps=4))
                    if pw and r is None:
                        put('pwpro', gtime(lambda: ops.pwconv_fwd(x, w, y, sp, stats=stats,
                                                                  pro=pro), reps=4))
                    put('bn%d_igemm' % mode, gtime(unfused, reps=4))
            if st == 1:
                xa, wt, ya = x.view(sp.M, C), w.view(K, C).t(), y.view(sp.M, K)
                put('matmul', gtime(lambda: torch.matmul(xa, wt, out=ya), reps=4))
            print(json.dumps(rec), flush=True)
            del x, w, y, stats, slab
            torch.cuda.empty_cache()
        print(json.dumps(dict(summary=True, model=model, batch=batch,
                              total_ms={k: round(v / 1e3, 3) for k, v in tot.items()})),
              flush=True)


if __name__ == '__main__':
    main()
