"""Ternary-compressed gradient all-reduce: the reference's ``quantize_tensor`` (`util.py:65-70`,
SURVEY C15/K10 -- stochastic magnitude quantisation, unused on its main path) as a DP wire
format, selected with ``grad_compress='ternary'``.

Each rank sends its bucket as ONE int32 message: word 0 = max|g| (fp32 bits), then 16 elements
per word at 2 bits each, c in {0: 0, 1: +1, 2: -1} with P(c != 0) = |g| / max|g| -- unbiased
(E[max * c] = g), 1/16 of the fp32 bytes.  Messages are all-gathered (RCCL on the comm stream,
or the process group on CPU / gloo) and every rank decodes the same mean

    g  <-  (1 / W) * sum_r max_r * c_r

so replicas stay identical.  On the GPU the pack (abs-max + Philox Bernoulli + 2-bit packing)
and the decode-sum are HIP kernels (``csrc/misc.hip`` tern_pack / tern_unpack); the torch
functions here are the CPU path and the test oracle of the same message layout.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def tern_words(n):
    """int32 words of one rank's message for an n-element bucket."""
    return 1 + (n + 15) // 16


def encode_torch(codes, scale):
    """int32 message from ternary codes (int tensor in {-1, 0, 1}) and the bucket scale."""
    n = codes.numel()
    c = torch.where(codes > 0, 1, torch.where(codes < 0, 2, 0)).to(torch.int64)
    pad = (-n) % 16
    if pad:
        c = torch.cat([c, torch.zeros(pad, dtype=torch.int64, device=c.device)])
    c = c.view(-1, 16) << (2 * torch.arange(16, dtype=torch.int64, device=c.device))
    w = c.sum(1)
    w = torch.where(w >= 2 ** 31, w - 2 ** 32, w).to(torch.int32)
    head = torch.tensor([float(scale)], dtype=torch.float32).view(torch.int32).to(w.device)
    return torch.cat([head, w])


def quantize_codes_torch(g, generator=None):
    """(codes in {-1, 0, 1}, scale = max|g|) with P(code != 0) = |g| / max|g|."""
    m = float(g.abs().max()) if g.numel() else 0.0
    if m == 0.0:
        return torch.zeros_like(g, dtype=torch.int8), 0.0
    u = torch.rand(g.shape, generator=generator, dtype=torch.float32).to(g.device)
    keep = u < (g.abs() / m)
    return (torch.sign(g) * keep).to(torch.int8), m


def decode_sum_torch(msgs, n, avg=True):
    """msgs [W][tern_words(n)] int32 -> the (mean) decoded fp32 vector of n elements."""
    W = msgs.shape[0]
    scales = msgs[:, :1].contiguous().view(torch.float32).view(W)
    w = msgs[:, 1:].to(torch.int64) & 0xffffffff
    c = (w.unsqueeze(-1) >> (2 * torch.arange(16, dtype=torch.int64, device=w.device))) & 3
    v = torch.where(c == 1, 1.0, torch.where(c == 2, -1.0, 0.0)).view(W, -1)[:, :n]
    out = (v * scales.view(W, 1)).sum(0)
    return out / W if avg else out


class TernaryAllReduce(object):
    """In-place ternary-compressed mean all-reduce of fp32 buckets.

    ``comm``: the engine's RcclComm (GPU path: HIP pack / decode kernels, RCCL all-gather on the
    current stream); None: torch encode / decode and ``dist.all_gather`` on ``group`` (CPU)."""

    def __init__(self, capacity, device, group=None, comm=None, seed=0):
        self.device = torch.device(device)
        self.group = group
        self.comm = comm
        self.size = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.seed = (int(seed) * 1000003 + self.rank * 7919 + 17) & 0xffffffff
        nw = tern_words(capacity)
        self.send = torch.zeros(nw, dtype=torch.int32, device=self.device)
        self.recv = torch.zeros(self.size * nw, dtype=torch.int32, device=self.device)
        self.ws = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.gen = torch.Generator().manual_seed(self.seed)

    def allreduce(self, g, counter, dctr=None):
        """``counter``: the Philox stream of this (step, bucket).  ``dctr`` (GPU path, graph
        capture): an int64 device step counter -- the stream is then (dctr[0], counter), read
        at replay time, and ``counter`` is just the bucket index."""
        n = g.numel()
        nw = tern_words(n)
        if nw > self.send.numel():
            raise ValueError('ternary all-reduce: bucket of %d exceeds the capacity' % n)
        if self.comm is not None:
            from ..ops import lib, ptr, stream_ptr
            L, st = lib(), stream_ptr()
            send, recv = self.send[:nw], self.recv[:self.size * nw]
            L.tern_pack(ptr(g), n, ptr(self.ws), self.seed, int(counter), ptr(send), st,
                        ptr(dctr) if dctr is not None else 0)
            self.comm.all_gather(recv, send)
            L.tern_unpack(ptr(recv), self.size, n, 1.0 / self.size, ptr(g), st)
            return g
        codes, m = quantize_codes_torch(g, self.gen)
        msg = encode_torch(codes, m)
        if self.size > 1:
            parts = [torch.empty_like(msg) for _ in range(self.size)]
            dist.all_gather(parts, msg, group=self.group)
            msgs = torch.stack(parts)
        else:
            msgs = msg.view(1, -1)
        g.copy_(decode_sum_torch(msgs, n, avg=True))
        return g
