"""bn_apply / bn_bwd graph-timed at the ResNet-18 scoring (B=320, 10 ghost groups) and train
(B=32) shapes (bench/gtime.py)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from gtime import gtime  # noqa: E402


def main():
    import torch
    from mercury_amd import ops
    dev = 'cuda'
    tot = {}
    for N, C, H in ((320, 64, 32), (320, 128, 16), (320, 256, 8), (320, 512, 4),
                    (32, 64, 32), (32, 128, 16), (32, 256, 8), (32, 512, 4)):
        M = N * H * H
        G = N // 32
        y = torch.randn(M * C, device=dev).to(torch.bfloat16)
        res = torch.randn(M * C, device=dev).to(torch.bfloat16)
        out = torch.empty_like(y)
        st = torch.rand(G * 2 * C, device=dev) + 1
        gm, bt = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        gr = 32 * H * H
        t1 = gtime(lambda: ops.bn_apply(y, st, gm, bt, out, M, C, group_rows=gr, act='relu'))
        t2 = gtime(lambda: ops.bn_apply(y, st, gm, bt, out, M, C, group_rows=gr, act='relu',
                                        res=res))
        row = dict(N=N, C=C, H=H, apply_us=round(t1, 2), apply_res_us=round(t2, 2))
        if N == 32:
            sums = torch.zeros(ops.sums_numel(C), device=dev)
            dy = torch.empty_like(y)
            t3 = gtime(lambda: ops.bn_bwd(res, out, y, st, gm, sums, dy, M, C, act='relu',
                                          zero_sums=False, reduce=False))
            row['bwd_apply_us'] = round(t3, 2)
        for k, v in row.items():
            if k.endswith('_us'):
                tot[k] = tot.get(k, 0) + v
        print(row, flush=True)
    print({k: round(v, 1) for k, v in tot.items()})


if __name__ == '__main__':
    main()
