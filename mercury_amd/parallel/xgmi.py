"""Direct-xGMI two-shot all-reduce (``csrc/xgmi.hip``).

The reference reduces gradients with a hand-written CPU ring (`util.py:280-324`); RCCL's ring
algorithms are the GPU analogue and are per-link bound on MI355X's point-to-point xGMI (a ring
step moves every byte over one of the 7 links).  ``XgmiAllReduce`` instead maps every peer's
exchange buffer into this process (``hipIpcGetMemHandle`` / ``hipIpcOpenMemHandle``) and
reduces in two direct passes that pull from all peers at once:

    pack            own gradients -> own exchange buffer slot (fp32, or bf16 with ``wire_bf16``)
    barrier         every rank's slot is filled
    reduce-scatter  rank r sums chunk r over all W slots (W-1 remote reads in parallel)
                    and writes it back into its own slot
    barrier         every chunk is reduced
    all-gather      chunk p of peer p -> local gradients, for every p

The barriers are device-side and stream-ordered (``barrier='device'``, the default): a one-block
kernel stores this rank's barrier epoch into every peer's flag area (system-scope atomic stores
through the IPC mapping) and polls its own area until every peer's epoch has arrived, with a
time limit that raises ``XgmiTimeout`` on the next ``check()`` instead of spinning forever.
Two buffer slots alternate between consecutive buckets, so no third barrier is needed before a
slot is refilled: a rank refills slot s for bucket k + 2 only after passing bucket k + 1's
second barrier, which every peer reaches only after its all-gather of bucket k.  A step with an
odd bucket count ends with one trailing barrier (``end_step``) so the next step can start on
slot 0.  ``barrier='rccl'`` (a one-element RCCL all-reduce) and ``'host'`` (tests) remain.
Tests on one GPU also use emulated peers (``emulated_allreduce``: W local buffers stand for W
ranks).  RCCL stays the engine default (``comm='rccl'``); ``comm='xgmi'`` selects this path.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import lib, ptr, stream_ptr

MAX_RANKS = 8


class XgmiTimeout(RuntimeError):
    pass


class XgmiAllReduce(object):

    def __init__(self, capacity, device, group=None, wire_bf16=False, barrier='device',
                 timeout_s=30.0):
        if capacity % 4:
            capacity += 4 - capacity % 4
        if barrier not in ('device', 'rccl', 'host'):
            raise ValueError("barrier must be 'device', 'rccl' or 'host'")
        self.capacity = int(capacity)
        self.device = torch.device(device)
        self.group = group
        init = dist.is_initialized()
        self.rank = dist.get_rank(group) if init else 0
        self.size = dist.get_world_size(group) if init else 1
        if self.size > MAX_RANKS:
            raise ValueError('xgmi all-reduce: at most %d ranks (one node)' % MAX_RANKS)
        self.bf16 = bool(wire_bf16)
        L = lib()
        # one allocation per rank: [flag area][slot 0][slot 1], all three IPC-mapped by peers
        self.flag_bytes = int(L.xgmi_flag_bytes())
        self.slot_bytes = (self.capacity * (2 if self.bf16 else 4) + 255) // 256 * 256
        self.buf = L.xgmi_malloc(self.flag_bytes + 2 * self.slot_bytes)
        if not self.buf:
            raise RuntimeError('xgmi all-reduce: exchange buffer allocation failed')
        self._opened = []
        if self.size > 1:
            h = L.xgmi_ipc_handle(self.buf)
            if not h:
                raise RuntimeError('hipIpcGetMemHandle failed (HSA_ENABLE_IPC_MODE_LEGACY=0 '
                                   'must be set for dmabuf IPC)')
            hs = [None] * self.size
            dist.all_gather_object(hs, h, group=group)
            peers = []
            for r, hr in enumerate(hs):
                if r == self.rank:
                    peers.append(self.buf)
                    continue
                p = L.xgmi_ipc_open(hr)
                if not p:
                    raise RuntimeError('hipIpcOpenMemHandle failed for rank %d' % r)
                self._opened.append(p)
                peers.append(p)
            self.peers = peers
        else:
            self.peers = [self.buf]
        self.barrier_kind = barrier
        self.timeout_s = float(timeout_s)
        self._comm = None
        self._tick = torch.zeros(4, dtype=torch.float32, device=self.device)
        # device barrier state: this rank's epoch and the timeout error word (bit q: peer q late)
        self._epoch = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._err = torch.zeros(1, dtype=torch.int32, device=self.device)
        if barrier == 'rccl' and self.size > 1:
            from .rccl import RcclComm
            self._comm = RcclComm.shared(group)

    def slot_ptrs(self, slot):
        return [p + self.flag_bytes + slot * self.slot_bytes for p in self.peers]

    def barrier(self):
        """Every rank reaches this point of its stream (no host wait for 'device' / 'rccl')."""
        if self.size == 1:
            return
        if self.barrier_kind == 'device':
            lib().xgmi_barrier(self.peers, self.rank, ptr(self._epoch), self.timeout_s,
                               ptr(self._err), stream_ptr())
        elif self.barrier_kind == 'rccl':
            self._comm.allreduce(self._tick, avg=False)
        else:
            torch.cuda.current_stream(self.device).synchronize()
            dist.barrier(group=self.group)

    def check(self):
        """Raise ``XgmiTimeout`` if a device barrier gave up on a peer (host sync)."""
        e = int(self._err.item())
        if e:
            late = [q for q in range(32) if e >> q & 1]
            raise XgmiTimeout('xgmi barrier: peers %s did not arrive within %.1f s'
                              % (late, self.timeout_s))

    def end_step(self, nbuckets):
        """After a step's last bucket: an odd bucket count leaves slot 0 last used, so one
        trailing barrier lets the next step's first bucket refill it."""
        if nbuckets % 2:
            self.barrier()

    def allreduce(self, t, avg=True, slot=0):
        """In-place all-reduce of a contiguous fp32 device tensor (numel % 4 == 0) through
        exchange slot ``slot`` (alternate 0 / 1 between consecutive calls; see end_step)."""
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
            raise ValueError('xgmi all-reduce: contiguous fp32 device tensor expected')
        n = t.numel()
        if n % 4 or n > self.capacity:
            raise ValueError('xgmi all-reduce: numel %d (capacity %d, multiple of 4)'
                             % (n, self.capacity))
        L, st, bf = lib(), stream_ptr(), int(self.bf16)
        bufs = self.slot_ptrs(slot)
        L.xgmi_pack(ptr(t), bufs[self.rank], n, bf, st)
        self.barrier()
        L.xgmi_reduce_scatter(bufs, self.rank, n, bf, 1.0 / self.size if avg else 1.0, st)
        self.barrier()
        L.xgmi_all_gather(bufs, n, bf, ptr(t), st)
        return t

    def close(self, sync_peers=True):
        """Collective at W > 1 ON THE NORMAL PATH (every rank calls it): one last barrier of
        this exchange's kind -- whatever the kind, a peer may still be reading this rank's slot
        in its all-gather -- then a device drain, then unmap the peers' buffers and free our own
        (``sync_peers=False``: the caller has synchronised the ranks on the host already).

        If a device barrier of this exchange ever gave up on a peer (the peer is gone or
        desynchronised), nothing waits for it again: the mappings and the buffer are LEAKED
        (freeing memory a live peer may still read would be a cross-GPU use-after-free, and a
        host barrier with a vanished peer would block forever) and ``XgmiTimeout`` is raised."""
        L = lib()
        if not self.buf:
            return
        failed = bool(self._err.item()) if self.size > 1 else False
        if sync_peers and self.size > 1 and not failed:
            self.barrier()
            torch.cuda.synchronize(self.device)
            failed = bool(self._err.item())
        torch.cuda.synchronize(self.device)
        err = int(self._err.item())
        if failed:
            self._opened = []
            self.buf = 0
            late = [q for q in range(32) if err >> q & 1]
            raise XgmiTimeout('xgmi barrier: peers %s did not arrive within %.1f s (exchange '
                              'buffers left mapped)' % (late, self.timeout_s))
        for p in self._opened:
            L.xgmi_ipc_close(p)
        self._opened = []
        if self.buf:
            L.xgmi_free(self.buf)
            self.buf = 0
        if err:
            late = [q for q in range(32) if err >> q & 1]
            raise XgmiTimeout('xgmi barrier: peers %s did not arrive within %.1f s'
                              % (late, self.timeout_s))


def emulated_allreduce(tensors, avg=True, wire_bf16=False):
    """The two-shot algorithm with W local buffers as the W ranks' exchange buffers (one GPU).
    Returns one reduced copy per emulated rank (each produced by that rank's all-gather)."""
    W = len(tensors)
    n = tensors[0].numel()
    L, st, bf = lib(), stream_ptr(), int(wire_bf16)
    dt = torch.bfloat16 if wire_bf16 else torch.float32
    xb = [torch.zeros(n, dtype=dt, device=tensors[0].device) for _ in range(W)]
    peers = [ptr(b) for b in xb]
    for r in range(W):
        L.xgmi_pack(ptr(tensors[r]), peers[r], n, bf, st)
    for r in range(W):
        L.xgmi_reduce_scatter(peers, r, n, bf, 1.0 / W if avg else 1.0, st)
    outs = [torch.empty(n, dtype=torch.float32, device=tensors[0].device) for _ in range(W)]
    for r in range(W):
        L.xgmi_all_gather(peers, n, bf, ptr(outs[r]), st)
    return outs
