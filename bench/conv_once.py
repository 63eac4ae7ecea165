"""Run one conv configuration repeatedly (target for rocprofv3 --pmc counter runs).

    python bench/conv_once.py N C K H R stride pad [iters] [pipe]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from mercury_amd import ops
    from mercury_amd.ops.conv import ConvSpec, fwd_plan, slab_bytes
    N, C, K, H, R, st, pd = (int(v) for v in sys.argv[1:8])
    iters = int(sys.argv[8]) if len(sys.argv) > 8 else 20
    pipe = int(sys.argv[9]) if len(sys.argv) > 9 else 0
    sp = ConvSpec(N, H, H, C, K, R, R, st, pd)
    x = ops.to_nhwc(torch.randn(N, C, H, H, device='cuda'))
    wk, _ = ops.pack_conv_weight(torch.randn(K, C, R, R, device='cuda') * 0.05)
    y = torch.empty(sp.M, K, dtype=torch.bfloat16, device='cuda')
    stats = torch.zeros(2, K, device='cuda')
    plan = fwd_plan(sp)
    slab = torch.zeros(max(1, slab_bytes(sp.M, K, *plan) // 4), device='cuda')
    for _ in range(iters):
        ops.conv_fwd(x, wk, y, sp, stats=stats, slab=slab, plan=plan, pipe=pipe)
    torch.cuda.synchronize()
    print('plan', plan)


if __name__ == '__main__':
    main()
