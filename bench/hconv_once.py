"""Run one halo-conv plan repeatedly (target for rocprofv3 --pmc counter passes).

    python bench/hconv_once.py N C K H stride bm bn splits [iters]
Ghost-BN statistics groups of 32 images when N > 32 (the scoring pass's epilogue).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from mercury_amd import ops
    from mercury_amd.ops import hconv as H
    from mercury_amd.ops.conv import ConvSpec, slab_bytes
    N, C, K, Hh, st, bm, bn, splits = (int(v) for v in sys.argv[1:9])
    iters = int(sys.argv[9]) if len(sys.argv) > 9 else 20
    sp = ConvSpec(N, Hh, Hh, C, K, 3, 3, st, 1)
    G = 1
    if N > 32:
        sp.group_rows = 32 * sp.P * sp.Q
        G = N // 32
    x = ops.to_nhwc(torch.randn(N, C, Hh, Hh, device='cuda'))
    wk, _ = ops.pack_conv_weight(torch.randn(K, C, 3, 3, device='cuda') * 0.05)
    y = torch.empty(sp.M, K, dtype=torch.bfloat16, device='cuda')
    stats = torch.zeros(G * 2 * K, device='cuda')
    plan = (bm, bn, splits)
    slab = torch.zeros(max(1, slab_bytes(sp.M, K, *plan) // 4 + 1), device='cuda')
    for _ in range(iters):
        H.hconv_fwd(x, wk, y, sp, plan, stats=stats, slab=slab)
    torch.cuda.synchronize()
    print('plan', plan)


if __name__ == '__main__':
    main()
