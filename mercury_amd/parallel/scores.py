"""Cross-worker importance-score exchange (Mercury's global view).

Not in the reference code (no ``all_gather`` anywhere), but it is the paper's
cross-device importance idea and the BASELINE north star asks for it.  Each
rank contributes its pool scores (P fp32, 1.25 KB at P=320); the gathered
W x P matrix gives every rank the global loss distribution, from which

* ``global_pool_mean`` -- a shared EMA normaliser so every rank smooths its
  probabilities with the same alpha*EMA(mean loss) (``--global-ema``);
* ``global_share`` -- each rank's fraction of total importance (used to report
  how non-IID shards differ in difficulty).

The message is tiny and latency-bound, so it is issued asynchronously on the
communication stream right after scoring and waited for only when needed.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class ScoreExchange(object):

    def __init__(self, pool_size, device, group=None, force=False, comm=None):
        self.group = group
        self.force = force            # run the collective even at world size 1 (path testing)
        # the native engine's RcclComm: the all-gather is then stream-ordered on the caller's
        # stream (the score stream) and leaves no ProcessGroup work in flight
        self.comm = comm
        self.ws = comm.size if comm is not None else (
            dist.get_world_size(group) if dist.is_initialized() else 1)
        self.local = torch.zeros(pool_size, dtype=torch.float32, device=device)
        self.gathered = torch.zeros(self.ws, pool_size, dtype=torch.float32, device=device)
        self._h = None

    def start(self, scores):
        # order the previous exchange before ``local`` is overwritten (stream-side wait on
        # nccl, so the host does not block)
        self.wait()
        self.local.copy_(scores.reshape(-1))
        if self.ws == 1 and not self.force:
            self.gathered[0].copy_(self.local)
            return self
        if self.comm is not None:
            self.comm.all_gather(self.gathered.view(-1), self.local)
            return self
        self._h = dist.all_gather_into_tensor(self.gathered.view(-1), self.local, group=self.group,
                                              async_op=True)
        return self

    def wait(self):
        if self._h is not None:
            self._h.wait()
            self._h = None
        return self.gathered

    def global_pool_mean(self):
        return self.wait().mean()

    def global_share(self):
        g = self.wait().sum(1)
        return g / g.sum()
