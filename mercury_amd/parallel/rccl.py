"""The framework's own RCCL communicator (C++ in ``csrc/comm.hip``).

``RcclComm(group)`` creates an RCCL communicator spanning a torch.distributed
group: rank 0 draws the 128-byte unique id, it is broadcast over the existing
group (any backend), every rank calls ``ncclCommInitRank`` on its current HIP
device.  Collectives are issued on the caller's current HIP stream and never
block the host:

* ``allreduce(t, avg=True)`` / ``all_gather(out, t)`` / ``broadcast(t, root)`` --
  RCCL's multi-channel algorithms (what the bucketed DP all-reduce uses);
* ``ring_allreduce(t)`` -- the explicit ring (reduce-scatter + all-gather of
  grouped ``ncclSend``/``ncclRecv`` pairs with an on-device add), the GPU
  counterpart of the reference's CPU ``util.allreduce`` (`util.py:280-324`).

This is independent of ``ProcessGroupNCCL``, so the engine can place a
collective on any stream it owns (e.g. the score stream) without an extra
ProcessGroup stream edge.

Lifetime is explicit.  ``RcclComm.shared(group, tag)`` hands out one communicator per
(torch.distributed group, tag) per process (engines share it).  RCCL runs the operations of ONE
communicator in issue order whatever stream they are issued on, so traffic that must not queue
behind the gradient buckets -- the per-step score all-gather, issued on the score stream before
the first bucket -- takes a communicator of its own (``tag='score'``).  ``close()`` synchronises
the device and destroys it.  Nothing is destroyed from ``__del__``: a garbage
collection pass can run at any point (inside another engine's construction, with
collectives in flight on a stream), and ncclCommDestroy there aborted the process
on the GPU box -- an un-closed communicator is released at process exit.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import lib, ptr, stream_ptr

_DTYPES = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int32: 3,
           torch.int64: 4}


class RcclComm(object):

    _shared = {}

    @classmethod
    def shared(cls, group=None, tag=None):
        """The process's communicator for (group, tag); creating one is collective over the
        group (every rank must ask for the same tags in the same order)."""
        init = dist.is_initialized()
        key = (id(group) if group is not None else None,
               dist.get_rank(group) if init else 0, dist.get_world_size(group) if init else 1,
               tag)
        c = cls._shared.get(key)
        if c is None or not c.handle:
            c = cls._shared[key] = cls(group)
        return c

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.size = dist.get_world_size(group) if dist.is_initialized() else 1
        L = lib()
        uid = L.comm_unique_id() if self.rank == 0 else b''
        if self.size > 1:
            box = [uid]
            dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group else 0,
                                       group=group)
            uid = box[0]
        self.handle = L.comm_init(uid, self.rank, self.size)
        self._work = None

    def close(self):
        if self.handle:
            torch.cuda.synchronize()
            lib().comm_destroy(self.handle)
            self.handle = 0

    @staticmethod
    def _code(t):
        if t.dtype not in _DTYPES:
            raise TypeError('rccl: unsupported dtype %s' % t.dtype)
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError('rccl: tensors must be contiguous HIP device tensors')
        return _DTYPES[t.dtype]

    def allreduce(self, t, avg=True):
        lib().comm_allreduce(self.handle, ptr(t), t.numel(), self._code(t), int(avg), stream_ptr())
        return t

    def all_gather(self, out, t):
        if out.numel() != t.numel() * self.size:
            raise ValueError('all_gather: out must hold world_size x input')
        self._code(out)
        lib().comm_allgather(self.handle, ptr(t), ptr(out), t.numel(), self._code(t), stream_ptr())
        return out

    def broadcast(self, t, root=0):
        lib().comm_broadcast(self.handle, ptr(t), t.numel(), self._code(t), root, stream_ptr())
        return t

    def ring_allreduce(self, t, avg=False):
        """Explicit ring all-reduce (fp32, in place); SUM by default like ``util.allreduce``."""
        if t.dtype != torch.float32:
            raise TypeError('ring_allreduce: fp32 only')
        self._code(t)
        need = (t.numel() + self.size - 1) // self.size + 8   # 16-B aligned chunks (comm.hip)
        if self._work is None or self._work.numel() < need or self._work.device != t.device:
            self._work = torch.empty(need, dtype=torch.float32, device=t.device)
        lib().comm_ring_allreduce(self.handle, ptr(t), t.numel(), ptr(self._work), int(avg),
                                  stream_ptr())
        return t
