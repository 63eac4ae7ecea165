"""BN-apply prologue conv vs bn_apply + plain conv, graph-timed (bench/gtime.py)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from gtime import gtime  # noqa: E402


def main():
    import torch
    from mercury_amd import ops
    from mercury_amd.ops.conv import ConvSpec, fwd_plan, slab_bytes
    dev = 'cuda'
    for N, C, K, H, R, keep in ((32, 64, 64, 32, 3, 1), (320, 64, 64, 32, 3, 0),
                                (32, 64, 256, 32, 1, 1), (32, 128, 512, 16, 1, 1),
                                (32, 256, 1024, 8, 1, 1), (32, 144, 24, 32, 1, 1),
                                (32, 576, 96, 8, 1, 1), (320, 64, 256, 32, 1, 0),
                                (320, 144, 24, 32, 1, 0), (320, 576, 96, 8, 1, 0)):
        sp = ConvSpec(N, H, H, C, K, R, R, 1, R // 2)
        G = 1
        if N > 32:
            sp.group_rows = 32 * H * H
            G = N // 32
        yn = ops.to_nhwc(torch.randn(N, C, H, H, device=dev))
        wk, _ = ops.pack_conv_weight(torch.randn(K, C, R, R, device=dev) * 0.05)
        stats = torch.rand(G * 2 * C, device=dev) + 1
        gamma, beta = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        out = torch.empty(sp.M * K, dtype=torch.bfloat16, device=dev)
        an = torch.empty_like(yn)
        plan = fwd_plan(sp)
        slab = torch.zeros(max(1, slab_bytes(sp.M, K, *plan[:3]) // 4), device=dev)
        pro = dict(stats=stats, gamma=gamma, beta=beta, act='relu', count=32 * H * H,
                   keep=an if keep else None)
        from mercury_amd.ops import conv as cv
        grp = sp.group_rows or sp.M

        def fused():
            cv.lib().igemm_pro(cv.ptr(yn), cv.ptr(wk), cv.ptr(out), K, 0, 0, K, grp,
                               cv.ptr(slab) if plan[2] > 1 else 0, H, H, sp.Cp, sp.P, sp.Q, R, R,
                               1, R // 2, R * R * sp.Cp // 8, K, sp.M, plan[0], plan[1], plan[2],
                               cv.stream_ptr(), *cv._pro_args(pro, sp))
        t_f = gtime(fused)
        t_c = gtime(lambda: ops.conv_fwd(an, wk, out, sp, slab=slab, plan=plan))
        t_b = gtime(lambda: ops.bn_apply(yn, stats, gamma, beta, an, N * H * H, C,
                                         group_rows=sp.group_rows, act='relu'))
        print('N=%d C=%d K=%d H=%d R=%d plan=%s  fused %.1f us | conv %.1f + bn_apply %.1f = %.1f us'
              % (N, C, K, H, R, plan, t_f, t_c, t_b, t_c + t_b), flush=True)


if __name__ == '__main__':
    main()
