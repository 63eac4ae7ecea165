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
    profiles/r4/session_r4s27/).

    The native engine replaces this model with measured numbers at start-up under DP
    (``calibrate_allreduce`` + ``plan_from_calibration``); this constant is the fallback when
    nothing was measured (ProcessGroup path, explicit sizes)."""
    return 16 << 20


# sizes timed by calibrate_allreduce (fp32 elements): 256 KiB, 4 MiB, 16 MiB
CALIB_SIZES = (1 << 16, 1 << 20, 1 << 22)


def calibrate_allreduce(comm, device, sizes=CALIB_SIZES, reps=5):
    """Time ``comm.allreduce`` (AVG, fp32) at a few sizes on a stream of its own and fit the
    linear model T(S) = alpha + S / beta (S in bytes) by least squares.  Collective: every rank
    of ``comm`` must call it.  Each size is issued once untimed, then ``reps`` times between two
    events; the per-rank fits are averaged over the communicator and rank 0's rounding of them is
    what every rank returns (the bucket plan built from them must be identical on every rank,
    or the ranks would issue mismatched collectives).

    Returns dict(alpha_us, beta_gbps, sizes_bytes, ms): ``ms`` the measured per-call times."""
    import numpy as np
    st = torch.cuda.Stream(device)
    cur = torch.cuda.current_stream(device)
    st.wait_stream(cur)
    buf = torch.zeros(max(sizes), dtype=torch.float32, device=device)
    ms = []
    with torch.cuda.stream(st):
        for n in sizes:
            t = buf[:n]
            comm.allreduce(t, avg=True)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(reps):
                comm.allreduce(t, avg=True)
            e1.record(st)
            e1.synchronize()
            ms.append(e0.elapsed_time(e1) / reps)
    cur.wait_stream(st)
    x = np.array([4.0 * n for n in sizes])
    y = np.array(ms) * 1e-3
    slope, icpt = np.polyfit(x, y, 1)
    alpha = max(float(icpt), 1e-6)                  # a collective costs at least 1 us
    beta = 1.0 / max(float(slope), 1e-15)           # bytes / s
    fit = torch.tensor([alpha * 1e6, beta / 1e9], dtype=torch.float32, device=device)
    if comm.size > 1:
        with torch.cuda.stream(st):
            comm.allreduce(fit, avg=True)
            comm.broadcast(fit, 0)
        st.synchronize()
    a_us, b_gbps = (float(v) for v in fit.tolist())
    return dict(alpha_us=round(a_us, 3), beta_gbps=round(b_gbps, 2),
                sizes_bytes=[4 * n for n in sizes], ms=[round(m, 5) for m in ms])


def plan_from_calibration(cal):
    """(bucket_bytes, last_bucket_bytes) from a calibration (``calibrate_allreduce``).

    * A bucket of S bytes costs alpha + S / beta; at S = 4 alpha beta the latency term is 20 %
      of it.  Buckets of that size (clamped to [4, 32] MiB) keep the per-bucket fixed costs (one
      more train-graph segment, the collective's latency) small against their transfer.
    * The LAST bucket closes when the backward ends, so all of it is exposed: it holds only the
      leading blocks' parameters (the ones the backward finishes last) up to alpha * beta bytes
      (where the transfer term equals the latency; clamped to [0.5, 4] MiB) -- for ResNet-18 the
      stem + layer1 (0.6 MB) or, on faster links, + layer2."""
    ab = cal['alpha_us'] * 1e-6 * cal['beta_gbps'] * 1e9
    mib = 1 << 20
    bucket = int(min(max(4.0 * ab, 4 * mib), 32 * mib))
    last = int(min(max(ab, mib // 2), 4 * mib))
    return bucket, last


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
