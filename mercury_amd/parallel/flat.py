"""Persistent flat parameter / gradient storage.

The reference flattens every gradient into a fresh 44.7 MB buffer per step and
divides into a second temporary (`pytorch_collab.py:236-249`).
``FlatParams`` instead re-homes every parameter of a module into ONE
contiguous fp32 buffer and points every ``.grad`` at a view of ONE contiguous
gradient buffer, once.  Gradient all-reduce then runs on contiguous slices of
that buffer with no packing copies, and a fused optimizer can sweep it in one
launch.  Buckets are contiguous flat ranges in *reverse* registration order,
which is the order backward produces gradients (last layer first), so the
first bucket is ready early in backward.
"""
from __future__ import annotations

import torch


class FlatParams(object):

    def __init__(self, module, dtype=torch.float32):
        self.params = [p for p in module.parameters() if p.requires_grad]
        dev = self.params[0].device
        self.numel = sum(p.numel() for p in self.params)
        self.data = torch.zeros(self.numel, dtype=dtype, device=dev)
        self.grad = torch.zeros(self.numel, dtype=dtype, device=dev)
        self.offsets = []
        off = 0
        for p in self.params:
            n = p.numel()
            self.data[off:off + n].copy_(p.detach().reshape(-1))
            p.data = self.data[off:off + n].view_as(p)
            p.grad = self.grad[off:off + n].view_as(p)
            self.offsets.append((off, n))
            off += n

    def zero_grad(self):
        self.grad.zero_()
        self.relink_grads()

    def relink_grads(self):
        """Re-point ``.grad`` at the flat views (after e.g. ``zero_grad(set_to_none=True)``)."""
        base = self.grad.data_ptr()
        esz = self.grad.element_size()
        for p, (off, n) in zip(self.params, self.offsets):
            g = p.grad
            view = self.grad[off:off + n].view_as(p)
            if g is None:
                view.zero_()
                p.grad = view
            elif g.data_ptr() != base + off * esz:
                view.copy_(g)
                p.grad = view

    def buckets(self, bucket_bytes):
        """Contiguous ``(start, end)`` flat ranges, last parameters first.

        Parameter boundaries are respected; a parameter larger than the cap
        gets its own bucket."""
        cap = max(1, bucket_bytes // self.grad.element_size())
        out = []
        end = self.numel
        cur_start = end
        for off, n in reversed(self.offsets):
            if end - off > cap and cur_start < end:
                out.append((cur_start, end))
                end = cur_start
            cur_start = off
        if cur_start < end:
            out.append((cur_start, end))
        return out

    def param_bucket_index(self, buckets):
        """For each parameter, the bucket id holding it."""
        idx = []
        for off, n in self.offsets:
            for b, (s, e) in enumerate(buckets):
                if s <= off < e:
                    idx.append(b)
                    break
        return idx
