"""Global importance table resident in HBM (``csrc/table.hip``).

``ImportanceTable`` owns one fp32 importance and one int32 group stamp per dataset
sample plus the small draw workspace.  Everything is stream-ordered and
allocation-free after construction, so writes and draws can be captured in HIP
graphs (pass ``stamp``/``group_dev`` device scalars instead of host ints).
"""
from __future__ import annotations

import torch

from . import _chk, lib, ptr, stream_ptr


class ImportanceTable(object):

    def __init__(self, n, device='cuda', init=1.0):
        self.N = int(n)
        self.device = torch.device(device)
        self.importance = torch.full((self.N,), float(init), dtype=torch.float32, device=self.device)
        self.group = torch.zeros(self.N, dtype=torch.int32, device=self.device)
        L = lib()
        nseg = L.table_num_segments(self.N)
        self._part = torch.zeros(nseg * 2, dtype=torch.float32, device=self.device)
        self._prefix = torch.zeros(nseg + 1, dtype=torch.float64, device=self.device)
        self._sc = torch.zeros(L.table_scalars_bytes() // 4, dtype=torch.int32, device=self.device)
        self.counter = torch.zeros(1, dtype=torch.int64, device=self.device)

    def write(self, start, losses, group_index):
        """Contiguous slice ``[start, start+n)`` <- losses, stamped ``group_index``."""
        losses = losses.detach().reshape(-1).to(self.device, torch.float32).contiguous()
        n = min(losses.numel(), self.N - int(start))
        lib().table_scatter(ptr(self.importance), ptr(self.group), ptr(losses), 0, 0, int(start), n,
                            self.N, int(group_index), stream_ptr())

    def scatter(self, index, losses, group_index=0, stamp=None):
        """``importance[index[i]] = losses[i]``; stamp from the device scalar ``stamp`` (int64)
        when given (graph-replay safe) else ``group_index``."""
        _chk(index, torch.int32, 'index')
        _chk(losses, torch.float32, 'losses', index.numel())
        lib().table_scatter(ptr(self.importance), ptr(self.group), ptr(losses), ptr(index),
                            ptr(stamp) if stamp is not None else 0, 0, index.numel(), self.N,
                            int(group_index), stream_ptr())

    def sample(self, ndraw, group_index=0, seed=0, out=None, out32=None, group_dev=None):
        """``ndraw`` weighted draws with replacement from the members of ``group_index``:
        ``p_i ~ imp_i + mean(imp over group)`` (`util.py:144-150`).  Returns int64 positions
        (-1 if the group is empty)."""
        if out is None and out32 is None:
            out = torch.empty(int(ndraw), dtype=torch.int64, device=self.device)
        lib().table_sample(ptr(self.importance), ptr(self.group), self.N, int(group_index),
                           ptr(group_dev) if group_dev is not None else 0, ptr(self._part),
                           ptr(self._prefix), ptr(self._sc), ptr(self.counter), int(ndraw),
                           int(seed) & 0xffffffff, ptr(out) if out is not None else 0,
                           ptr(out32) if out32 is not None else 0, stream_ptr())
        return out if out is not None else out32

    def draw_batch(self, ndraw, group_dev, pos32, pool_index, Ns, P, idx, isw, seed=0,
                   meters=None):
        """Native groupwise step: ``ndraw`` draws from the group stamped ``group_dev`` (device
        int64) into ``pos32``, then pool slots ``idx`` (the group is the contiguous slice that
        ``pool_index`` holds) and unbiased weights ``isw = n_group * p`` -- all on the current
        stream, graph-capturable."""
        _chk(pos32, torch.int32, 'pos32', ndraw)
        _chk(idx, torch.int32, 'idx', ndraw)
        _chk(isw, torch.float32, 'isw', ndraw)
        _chk(pool_index, torch.int32, 'pool_index', P)
        self.sample(ndraw, seed=seed, out32=pos32, group_dev=group_dev)
        lib().table_weights(ptr(pos32), int(ndraw), ptr(self.importance), ptr(self._sc),
                            ptr(pool_index), int(Ns), int(P), ptr(idx), ptr(isw), ptr(meters),
                            stream_ptr())

    def group_stats(self):
        """(mean importance, member count, total weight) of the last sampled group (syncs)."""
        f = self._sc[:2].view(torch.float32).tolist()
        total = self._sc[2:4].view(torch.float64).item()
        return f[0], int(f[1]), total
