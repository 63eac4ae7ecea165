"""Ternary-compressed gradient all-reduce (parallel/compress.py) on the CPU: message layout,
unbiasedness, and a two-rank gloo exchange whose replicas agree (reference quantize_tensor,
`util.py:65-70`, as a wire format)."""
import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mercury_amd.parallel.compress import (TernaryAllReduce, decode_sum_torch, encode_torch,
                                           quantize_codes_torch, tern_words)


def test_encode_decode_roundtrip_exact():
    g = torch.Generator().manual_seed(0)
    for n in (1, 15, 16, 17, 1000):
        codes = torch.randint(-1, 2, (n,), generator=g).to(torch.int8)
        msg = encode_torch(codes, 0.375)
        assert msg.dtype == torch.int32 and msg.numel() == tern_words(n)
        out = decode_sum_torch(msg.view(1, -1), n, avg=False)
        assert torch.equal(out, codes.float() * 0.375)


def test_decode_sums_and_averages_ranks():
    g = torch.Generator().manual_seed(1)
    n = 37
    cs = [torch.randint(-1, 2, (n,), generator=g).to(torch.int8) for _ in range(3)]
    sc = [0.5, 2.0, 1.25]
    msgs = torch.stack([encode_torch(c, s) for c, s in zip(cs, sc)])
    want = sum(c.float() * s for c, s in zip(cs, sc)) / 3
    assert torch.allclose(decode_sum_torch(msgs, n), want)


def test_quantizer_unbiased_and_ternary():
    x = torch.linspace(-1.5, 2.0, 64)
    gen = torch.Generator().manual_seed(3)
    acc = torch.zeros_like(x)
    reps = 3000
    for _ in range(reps):
        codes, m = quantize_codes_torch(x, gen)
        assert m == 2.0 and set(codes.unique().tolist()) <= {-1, 0, 1}
        acc += codes.float() * m
    # per element: var <= m |x| <= 4 -> std of the mean <= 2 / sqrt(reps)
    assert (acc / reps - x).abs().max() < 6 * 2 / reps ** 0.5
    # the max element is always kept, a zero never
    codes, m = quantize_codes_torch(torch.tensor([0.0, 2.0, -1.0]), gen)
    assert codes[0] == 0 and codes[1] == 1


def _worker(rank, ws, port, out):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=ws)
    try:
        g = torch.full((50,), 0.1 * (rank + 1))
        g[7] = -1.0 if rank == 0 else 3.0
        tern = TernaryAllReduce(64, 'cpu', seed=5)
        tern.allreduce(g, counter=1)
        out[rank] = g.clone()
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_replicas_agree():
    from mercury_amd.parallel.dist import free_port
    ws = 2
    with mp.Manager() as man:
        out = man.dict()
        mp.spawn(_worker, args=(ws, free_port(), out), nprocs=ws, join=True)
        a, b = out[0], out[1]
    assert torch.equal(a, b)
    # every element is (c0 * max0 + c1 * max1) / 2 with c in {-1, 0, 1}; max0 = 1, max1 = 3
    lattice = torch.tensor([(c0 * 1.0 + c1 * 3.0) / 2 for c0 in (-1, 0, 1) for c1 in (-1, 0, 1)])
    assert ((a.view(-1, 1) - lattice.view(1, -1)).abs().min(1).values < 1e-6).all()
    assert abs(float(a[7]) - 1.0) < 1e-6        # both maxima are kept: (-1 + 3) / 2
