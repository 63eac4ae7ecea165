"""In-situ plan tuner: chooses conv plans by the time of the WHOLE two-stream step.

``ops/tune.py`` times each conv alone, and its winners lost in the importance-sampled step
(its docstring: split-K and small tiles that shorten one kernel alone add blocks and slab
traffic that the concurrently running scoring stream pays for).  What the step needs is the
plan that costs the least *while the other stream is running*, which only the step itself can
measure.  So this tuner works on a live ``NativeEngine``:

* every distinct conv shape of every batch mode is one coordinate -- the cache key of
  ``tune.py`` (forward plan per (shape, ghost group, batch); dgrad + wgrad pair per train
  shape), so identical layers move together;
* for each coordinate, each candidate plan is written into the engine's plan table, the step
  graphs are re-captured, and the step is timed (median of a few chunks of replays);
* a candidate replaces the incumbent only if it is faster by more than ``threshold`` in the
  first measurement AND again in a confirming re-measurement of both, so run-to-run noise
  does not walk the plans;
* the result is a ``tune.py`` cache file (``MERCURY_TUNE_CACHE``, or shipped as the built-in
  ``tune_cache.json``): the engine then reads the step-tuned plans at mode allocation.

No counterpart in the reference (it has no kernels to plan; its convs are cuDNN's choice,
`pytorch_model.py:19-36`).
"""
from __future__ import annotations

import time

import torch

from . import tune
from .conv import slab_bytes


def time_steps(eng, steps=40, chunks=3):
    """Median ms per ``eng.step()`` over ``chunks`` timed runs of ``steps`` steps."""
    ts = []
    for _ in range(chunks):
        torch.cuda.synchronize(eng.device)
        t0 = time.perf_counter()
        for _ in range(steps):
            eng.step()
        torch.cuda.synchronize(eng.device)
        ts.append((time.perf_counter() - t0) * 1e3 / steps)
    ts.sort()
    return ts[len(ts) // 2]


def coordinates(eng):
    """[(kind, cache key, [(mode, unit name, spec)])] -- 'fwd' per forward shape and batch
    mode, 'bwd' per train shape whose dgrad + wgrad pair the engine plans from the cache."""
    out = {}
    for m in eng.modes.values():
        for (name, kind), _ in m.plan.items():
            if kind not in ('fwd', 'dgrad'):      # (halo-conv / pointwise / stem plans:
                continue                          # measured, not tuned; wgrad rides with dgrad)
            if kind == 'fwd' and ((name, 'hconv') in m.plan or (name, 'stem') in m.plan):
                continue                                  # (its igemm plan is never launched)
            sp = m.spec[name]
            ck = 'fwd' if kind == 'fwd' else 'bwd'
            if ck == 'bwd' and sp.K % 8:
                continue
            key = tune._key(ck, sp)
            out.setdefault((ck, key), []).append((m, name, sp))
    return [(k, key, users) for (k, key), users in out.items()]


def _ensure_slab(m, need):
    if m.slab.numel() * 4 < need:
        m.slab = torch.zeros((need + 3) // 4, dtype=torch.float32, device=m.slab.device)


def _get(kind, users):
    m, name, _ = users[0]
    if kind == 'fwd':
        p = m.plan[name, 'fwd']
        return (p[0], p[1], p[2], 0 if len(p) < 4 or p[3] is None else p[3])
    return (tuple(m.plan[name, 'dgrad']), tuple(m.plan[name, 'wgrad']))


def _set(kind, users, plan):
    for m, name, sp in users:
        if kind == 'fwd':
            m.plan[name, 'fwd'] = tuple(plan)
            _ensure_slab(m, slab_bytes(sp.M, sp.K, *plan[:3]))
        else:
            d, w = plan
            m.plan[name, 'dgrad'] = tuple(d)
            m.plan[name, 'wgrad'] = tuple(w)
            _ensure_slab(m, slab_bytes(sp.N * sp.H * sp.W, sp.Cp, *d))


def _candidates(kind, sp, cur, max_split):
    if kind == 'fwd':
        return [c for c in tune._fwd_candidates(sp) if c[2] <= max_split and c != cur]
    dc, wc = tune._bwd_candidates(sp)
    d0, w0 = cur
    return ([(d, w0) for d in dc if d[2] <= max_split and d != d0],
            [w for w in wc if w != w0])


def tune_step(eng, steps=40, chunks=3, threshold=0.004, max_split=4, budget_s=600.0,
              log=print, kinds=('fwd', 'bwd')):
    """Coordinate descent over the engine's conv plans, judged by step time.  Returns
    ({cache key: plan}, baseline ms, final ms).  ``eng`` must be primed and stepping."""
    t_start = time.perf_counter()

    def measure():
        eng.build_graphs()
        eng.step()
        return time_steps(eng, steps, chunks)

    base = measure()
    best_t = base
    coords = [c for c in coordinates(eng) if c[0] in kinds]
    # biggest work first: the scoring batch, then forward before backward
    coords.sort(key=lambda c: (-c[2][0][2].N, c[0] != 'fwd'))
    result = {}
    log('[step-tune] baseline %.4f ms/step, %d coordinates' % (base, len(coords)))

    def trial(kind, users, inc, cand):
        nonlocal best_t
        _set(kind, users, cand)
        t = measure()
        if t < best_t * (1.0 - threshold):
            # confirm against a fresh measurement of the incumbent
            _set(kind, users, inc)
            t_inc = measure()
            _set(kind, users, cand)
            t2 = measure()
            if t2 < t_inc * (1.0 - threshold):
                best_t = t2
                return True
            best_t = min(best_t, t_inc)
        _set(kind, users, inc)
        return False

    for kind, key, users in coords:
        if time.perf_counter() - t_start > budget_s:
            log('[step-tune] time budget reached')
            break
        sp = users[0][2]
        inc = _get(kind, users)
        if kind == 'fwd':
            for cand in _candidates(kind, sp, inc, max_split):
                if trial(kind, users, inc, cand):
                    inc = cand
        else:
            dpairs, wplans = _candidates(kind, sp, inc, max_split)
            for cand in dpairs:
                if trial(kind, users, inc, cand):
                    inc = cand
            for w in wplans:
                cand = (inc[0], w)
                if trial(kind, users, inc, cand):
                    inc = cand
        _set(kind, users, inc)
        result[key] = [list(inc[0]), list(inc[1])] if kind == 'bwd' else list(inc)
        log('[step-tune] %s -> %s  (%.4f ms/step, %.0f s)'
            % (key, result[key], best_t, time.perf_counter() - t_start))
    final = measure()
    log('[step-tune] final %.4f ms/step (baseline %.4f)' % (final, base))
    return result, base, final
