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
    """16 MiB buckets at every world size, from this cost model:

    * a bucket of S bytes all-reduced by RCCL's rings at W ranks moves 2(W-1)/W * S bytes per
      GPU; on a fully connected 8-GPU MI355X node that traffic is spread over 7 xGMI links
      (153 GB/s each, spec), so T(S) = alpha + 2(W-1)/W * S / B_eff, with B_eff the achieved
      per-GPU bus bandwidth (NOT measured here: no multi-GPU node has run this code yet);
    * every bucket also costs the step a fixed amount: one more graph segment of the train
      graph plus the comm-stream event edges, measured at W = 1 as +0.065 ms for 3 buckets
      (~33 us per extra segment, dp_nocomm in profiles/r4/ab_hw_queues.json), plus RCCL's
      per-collective latency alpha (~10-20 us, assumed);
    * the backward produces ResNet-18's 44.7 MB of gradients over ~0.5 ms of train-stream time,
      so everything but the last bucket is hidden if T(S) stays under the backward time left
      after that bucket closes; the last bucket (stem + layer1, closed when the backward ends)
      is exposed.
    With B_eff ~ 300 GB/s (an assumption) at W = 8: the bandwidth term is 78 MB / 300 GB/s =
    0.26 ms per step in all; 16 MiB gives ResNet-18 3 buckets (18.9 / 17.1 / 8.7 MB): ~0.1 ms
    of fixed costs and ~70 us exposed for the last one, where 4 MiB buckets (7) would pay ~0.23
    ms of fixed costs and 64 MiB (1) would expose the whole 0.26 ms.  The W = 1 forced-bucket
    sweep (profiles/r3/bucket_size_sweep_w1.json: 4 MiB 1.514, 8 MiB 1.485, 16 MiB 1.469, 32
    MiB 1.458 ms) measures only the fixed costs and agrees with the n * 33 us term.
    One bucket is NOT better at W = 1 even though the bandwidth term is zero: RCCL's one-rank
    all-reduce is still a local pass over the bucket, and with one bucket it runs exposed after
    the backward (forced DP, same box: 1 bucket 1.480 ms, 16 MiB 1.437, non-DP 1.355,
    profiles/r4/session_r4s27/)."""
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
