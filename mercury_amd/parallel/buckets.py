"""Bucketed, backward-overlapped gradient all-reduce over RCCL.

Reference: one blocking 44.7 MB all-reduce after backward, plus two packing
copies (`pytorch_collab.py:236-249`).  Here gradients already live in a flat
buffer (``FlatParams``); buckets are contiguous slices in backward order and
each bucket's ``all_reduce`` is issued asynchronously the moment its last
gradient is accumulated, so RCCL (on its own HIP stream) overlaps with the
rest of backward.  ``finish()`` joins them before the optimizer step.

Bucket size is chosen for xGMI: an 8-GPU MI355X node is fully connected with
7 links per GPU (~153 GB/s each).  RCCL splits a bucket into per-channel ring
slices; for every link to carry a slice worth its latency the bucket should
be >= 7 x ~512 KB, while fewer, larger buckets amortise the ~10-20 us launch
latency of each collective.  ``default_bucket_bytes`` documents the size model
(see its docstring); the W = 8 choice is a model, not a measurement -- no
multi-GPU node has run this code yet.

``average`` uses ``ReduceOp.AVG`` on RCCL (folds the 1/W into the collective,
removing the reference's extra divide) and SUM + scale on gloo.  Optional
``wire_dtype=torch.bfloat16`` halves bytes on the links.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def default_bucket_bytes(world_size):
    """16 MiB buckets at every world size: each bucket costs the native step one more
    host-replayed graph segment and one RCCL launch (~15 us at W=1, more per-message latency over
    xGMI rings at W=8), and the scoring stream runs beside the whole backward, so a few large
    buckets still overlap.  Measured forced-bucket ResNet-18 step at W=1 (profiles/r3/
    bucket_size_sweep_w1.json): 4 MiB 1.514, 8 MiB 1.485, 16 MiB 1.469, 32 MiB 1.458 ms (no DP
    1.358).  (32 MiB would leave ResNet-18 two buckets -- the first 34 MB -- too little overlap
    at W=8.)"""
    return 16 << 20


class BucketedAllReduce(object):

    def __init__(self, flat, bucket_bytes=None, group=None, average=True, wire_dtype=None):
        self.flat = flat
        self.group = group
        self.ws = dist.get_world_size(group) if dist.is_initialized() else 1
        self.bucket_bytes = bucket_bytes or default_bucket_bytes(self.ws)
        self.buckets = flat.buckets(self.bucket_bytes)
        self.pidx = flat.param_bucket_index(self.buckets)
        self.need = [0] * len(self.buckets)
        for b in self.pidx:
            self.need[b] += 1
        self.count = [0] * len(self.buckets)
        self.average = average
        self.wire_dtype = wire_dtype
        self.handles = []
        self._hooks = []
        be = dist.get_backend(group) if dist.is_initialized() else 'gloo'
        self.use_avg_op = (be == 'nccl')

    # -- overlap with backward ---------------------------------------------------------------
    def attach(self):
        for p, b in zip(self.flat.params, self.pidx):
            self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(b)))
        return self

    def detach(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []

    def _make_hook(self, b):
        def hook(_p):
            self.count[b] += 1
            if self.count[b] == self.need[b]:
                self._launch(b)
        return hook

    def _launch(self, b):
        if self.ws == 1:
            return
        s, e = self.buckets[b]
        t = self.flat.grad[s:e]
        wire = t if self.wire_dtype is None else t.to(self.wire_dtype)
        op = dist.ReduceOp.AVG if (self.average and self.use_avg_op) else dist.ReduceOp.SUM
        h = dist.all_reduce(wire, op=op, group=self.group, async_op=True)
        self.handles.append((h, b, wire))

    def finish(self):
        """Launch any bucket whose hooks did not all fire, wait, and scale."""
        launched = {b for _, b, _ in self.handles}
        for b in range(len(self.buckets)):
            if b not in launched:
                self._launch(b)
        for h, b, wire in self.handles:
            h.wait()
            s, e = self.buckets[b]
            t = self.flat.grad[s:e]
            if wire is not t:
                t.copy_(wire)
            if self.average and not self.use_avg_op:
                t.div_(self.ws)
        self.handles = []
        self.count = [0] * len(self.buckets)

    def allreduce_now(self):
        """Non-overlapped path: all buckets, then wait."""
        self.handles = []
        for b in range(len(self.buckets)):
            self._launch(b)
        self.finish()
