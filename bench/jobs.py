"""GPU job runner: every measurement this repo takes on an MI355X box, as named jobs.

    gpurun --timeout 1200 -- python3 bench/jobs.py <job> [--tag T] [job options]

Replaces the one-off ``bench/*.sh`` scripts of round 1.  Each step runs as a CHILD process
under its own time limit (``timeout -k 10``); a crash, fault, abort or time limit ends the job
there (exit code propagated), a plain test failure (pytest rc 1) does not stop later steps.
Outputs go to ``gpurun_out/<job>_<tag>/``.

jobs
  tests     [--select PYTEST_ARGS]   GPU test suite (default: every test marked gpu)
  bench     [--args BENCH_ARGS]      headline bench (and --args variants, ';'-separated)
  session                            tests + headline bench + forced-bucket RCCL bench + smoke
  trace     [--args BENCH_ARGS]      rocprofv3 kernel trace -> per-queue timeline + graph times
  pmc       [--counters C ...]       one PMC pass (<= 8 SQ counters) over the headline step
  presets                            every BASELINE config's bench (configs 2-5)
  ab        --env "A=1" "A=0" ...    same-box interleaved A/B of env settings (2 rounds;
            [--args BENCH_ARGS]      --args e.g. '--config mobilenetv2-cifar100')
  ab-ext    --old OLD.so             same-box A/B of another build (MERCURY_EXT_PATH)
  ab-preset --old OLD.so --args CFG  ... on one BASELINE preset
  ab-kernel --old OLD.so --args CMD  ... on a microbenchmark (bench/pool_bench.py, ...)
  sweep                              graph-timed conv plan sweeps (igemm and halo conv)
  learn                              learning check of the ResNet-50/224 preset
  multi     --args 'CMD1 ;; CMD2 ...'  ad-hoc steps, each a child under its own limit
                                     (--limit s); a plain test failure (rc 1) continues,
                                     a crash / abort / fault / time limit stops the job
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import shlex
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY = sys.executable


class Stop(Exception):
    pass


def run(cmd, out, limit, env=None, ok_codes=(0,)):
    """Run ``cmd`` (list) with stdout -> ``out``; raise Stop on a fatal exit."""
    e = dict(os.environ)
    e.setdefault('TMPDIR', '/tmp')
    if env:
        e.update(env)
    full = ['timeout', '-k', '10', str(limit)] + cmd
    with open(out, 'w') as f, open(out + '.err', 'w') as fe:
        rc = subprocess.call(full, cwd=ROOT, stdout=f, stderr=fe, env=e)
    print('[jobs] rc=%d %s -> %s' % (rc, ' '.join(cmd)[:160], os.path.relpath(out, ROOT)),
          flush=True)
    if rc not in ok_codes:
        with open(out + '.err') as fe:
            tail = fe.read()[-2000:]
        print(tail, flush=True)
        raise Stop(rc)
    return rc


def tail(path, n=3):
    with open(path) as f:
        lines = [l.rstrip() for l in f if l.strip()]
    for l in lines[-n:]:
        print(l, flush=True)


def job_tests(o, a):
    sel = shlex.split(a.select) if a.select else ['tests']
    out = os.path.join(o, 'tests.log')
    run([PY, '-u', '-m', 'pytest', '-v', '-m', 'gpu', '--timeout', '120',
         '--timeout-method', 'thread'] + sel, out, 900, ok_codes=(0, 1))
    tail(out, 2)


def job_bench(o, a):
    variants = [v.strip() for v in (a.args or '').split(';')] if a.args else ['']
    for i, v in enumerate(variants):
        out = os.path.join(o, 'bench%d.json' % i)
        run([PY, 'bench.py'] + shlex.split(v), out, 400)
        tail(out, 1)


def job_session(o, a):
    job_tests(o, a)
    for i, v in enumerate(['--steps 200 --warmup 20',
                           '--steps 100 --warmup 10 --no-overhead --force-buckets']):
        out = os.path.join(o, 'bench%d.json' % i)
        run([PY, 'bench.py'] + v.split(), out, 400)
        tail(out, 1)
    run([PY, '-c', 'import __graft_entry__ as g; g.smoke()'], os.path.join(o, 'smoke.log'), 300)
    tail(os.path.join(o, 'smoke.log'), 1)


def job_trace(o, a):
    tr = os.path.join(o, 'trace')
    run(['rocprofv3', '--kernel-trace', '--stats', '--output-format', 'csv', '-d', tr, '-o',
         'run', '--', PY, 'bench.py', '--steps', '60', '--warmup', '10', '--no-overhead'] +
        shlex.split(a.args or ''), os.path.join(o, 'bench.log'), 300)
    marker = 'optimizer_fused'
    if '--replay-only' in (a.args or ''):
        marker = 'step_begin' if 'train' in a.args else 'pool_build'
    run([PY, 'bench/trace_timeline.py', tr, marker, '40'],
        os.path.join(o, 'timeline.txt'), 120)
    tail(os.path.join(o, 'timeline.txt'), 30)
    if '--replay-only' in (a.args or ''):
        return
    run([PY, 'bench/host_overhead.py'], os.path.join(o, 'host_overhead.log'), 240)
    tail(os.path.join(o, 'host_overhead.log'), 12)


DEFAULT_PMC = ['SQ_WAVE_CYCLES', 'SQ_BUSY_CYCLES', 'SQ_VALU_MFMA_BUSY_CYCLES', 'SQ_INSTS_MFMA',
               'SQ_INSTS_VALU', 'SQ_INSTS_LDS', 'SQ_LDS_BANK_CONFLICT', 'SQ_WAIT_INST_ANY']


# MFMA utilisation pass (rocprofv3's MfmaUtil expression needs GRBM_GUI_ACTIVE beside the busy
# cycles; without it the round-5 summaries read 0)
MFMA_PMC = ['SQ_VALU_MFMA_BUSY_CYCLES', 'SQ_INSTS_VALU_MFMA_MOPS_BF16', 'SQ_INSTS_MFMA',
            'SQ_INSTS_VALU', 'SQ_INSTS_LDS', 'SQ_LDS_BANK_CONFLICT', 'SQ_WAIT_INST_LDS',
            'SQ_WAVE_CYCLES', 'GRBM_GUI_ACTIVE']


def job_pmc(o, a):
    ctr = a.counters or (MFMA_PMC if a.mfma else DEFAULT_PMC)
    if sum(1 for c in ctr if c.startswith('SQ_')) > 8:
        raise SystemExit('at most 8 SQ counters per pass')
    if sum(1 for c in ctr if c.startswith('GRBM_')) > 2:
        raise SystemExit('at most 2 GRBM counters per pass')
    bargs = shlex.split(a.args) if a.args else ['--steps', '10', '--warmup', '3', '--no-overhead']
    # (counters in their own pass, kernel trace only: no sys/runtime trace domains; the profiler
    # starts HIP before bench.py can raise the hardware-queue count)
    run(['timeout', '-s', 'KILL', '150', 'rocprofv3', '--pmc'] + ctr +
        ['--output-format', 'csv', '-d', os.path.join(o, 'p1'), '-o', 'run', '--', PY,
         'bench.py'] + bargs, os.path.join(o, 'p1.log'), 200, env={'GPU_MAX_HW_QUEUES': '16'})
    run([PY, 'bench/pmcsum.py', os.path.join(o, 'p1')], os.path.join(o, 'pmc_summary.txt'), 120)
    tail(os.path.join(o, 'pmc_summary.txt'), 30)


def job_presets(o, a):
    for c in ('resnet18-cifar10', 'mobilenetv2-cifar100', 'resnet50-imagenet', 'vgg11-speech'):
        out = os.path.join(o, c + '.json')
        extra = ['--steps', '300', '--warmup', '30'] if c == 'resnet18-cifar10' else \
            ['--steps', '100', '--warmup', '10', '--no-overhead']
        run([PY, 'bench.py', '--config', c] + extra, out, 400)
        tail(out, 1)


def job_ab(o, a):
    envs = a.env or []
    res = {e: [] for e in envs}
    solo = {}
    for rnd in range(a.rounds):
        for j, e in enumerate(envs):
            kv = dict(x.split('=', 1) for x in e.split())
            out = os.path.join(o, 'v%d_%d.json' % (j + 1, rnd + 1))
            run([PY, 'bench.py'] + shlex.split(a.args or '') +
                ['--steps', '300', '--warmup', '30', '--no-overhead'], out, 200, env=kv)
            with open(out) as f:
                d = json.loads(f.read().strip().splitlines()[-1])
            res[e].append(d['ms_per_step'])
            solo.setdefault(e, []).append(d.get('solo_ms'))
    for e, v in res.items():
        print('%-40s %s solo %s' % (e, v, solo.get(e)), flush=True)
    with open(os.path.join(o, 'ab.json'), 'w') as f:
        json.dump({'ms_per_step': res, 'solo_ms': solo}, f, indent=1)


def job_ab_ext(o, a):
    res = {'old': [], 'new': []}
    for rnd in range(a.rounds + 1):
        for name, env in (('old', {'MERCURY_EXT_PATH': a.old}), ('new', {})):
            out = os.path.join(o, '%s%d.json' % (name, rnd + 1))
            run([PY, 'bench.py', '--steps', '300', '--warmup', '30', '--no-overhead'], out, 200,
                env=env)
            with open(out) as f:
                res[name].append(json.loads(f.read().strip().splitlines()[-1])['ms_per_step'])
    print(res, flush=True)


def _last_ms(path):
    with open(path) as f:
        return json.loads(f.read().strip().splitlines()[-1])['ms_per_step']


def job_ab_preset(o, a):
    """same-box interleaved A/B of another build (--old OLD.so) on one preset (--args CONFIG)"""
    cfg = a.args or 'resnet18-cifar10'
    res = {'old': [], 'new': []}
    for rnd in range(a.rounds):
        for name, env in (('old', {'MERCURY_EXT_PATH': a.old}), ('new', {})):
            out = os.path.join(o, '%s%d.json' % (name, rnd + 1))
            run([PY, 'bench.py', '--config', cfg, '--steps', '100', '--warmup', '10',
                 '--no-overhead'], out, 200, env=env)
            res[name].append(_last_ms(out))
    print(json.dumps(res), flush=True)
    with open(os.path.join(o, 'ab.json'), 'w') as f:
        json.dump(res, f)


def job_ab_kernel(o, a):
    """same-box interleaved A/B of another build (--old OLD.so) on a microbenchmark
    (--args 'bench/pool_bench.py ...'); prints each run's last JSON line"""
    cmd = [PY] + shlex.split(a.args)
    for rnd in range(a.rounds + 1):
        for name, env in (('old', {'MERCURY_EXT_PATH': a.old}), ('new', {})):
            out = os.path.join(o, '%s%d.json' % (name, rnd + 1))
            run(cmd, out, 200, env=env)
            print(name, end=' ', flush=True)
            tail(out, 1)


def job_sweep(o, a):
    for b in (32, 320):
        run([PY, 'bench/kernel_sweep.py', '--batch', str(b), '--kind', 'fwd'],
            os.path.join(o, 'igemm%d.jsonl' % b), 400)
        run([PY, 'bench/hconv_sweep.py', '--batch', str(b)], os.path.join(o, 'hconv%d.jsonl' % b),
            400)
        tail(os.path.join(o, 'hconv%d.jsonl' % b), 1)


def job_learn(o, a):
    out = os.path.join(o, 'learn.json')
    run([PY, 'bench/learn_check.py', '--config', 'resnet50-imagenet', '--classes', '10',
         '--steps', '300'], out, 600)
    tail(out, 1)


def job_multi(o, a):
    for i, c in enumerate([c.strip() for c in (a.args or '').split(';;') if c.strip()]):
        out = os.path.join(o, 'step%d.log' % i)
        argv = shlex.split(c)
        if argv and argv[0] in ('python', 'python3'):
            argv[0] = PY
        run(argv, out, a.limit, ok_codes=(0, 1))
        tail(out, 4)


JOBS = {'multi': job_multi, 'tests': job_tests, 'bench': job_bench, 'session': job_session, 'trace': job_trace,
        'pmc': job_pmc, 'presets': job_presets, 'ab': job_ab, 'ab-ext': job_ab_ext,
        'sweep': job_sweep, 'learn': job_learn, 'ab-preset': job_ab_preset,
        'ab-kernel': job_ab_kernel}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('job', choices=sorted(JOBS))
    ap.add_argument('--tag', default='cur')
    ap.add_argument('--select', default='')
    ap.add_argument('--args', default='')
    ap.add_argument('--counters', nargs='*')
    ap.add_argument('--mfma', action='store_true', help='pmc: the MFMA-utilisation counter pass')
    ap.add_argument('--env', nargs='*')
    ap.add_argument('--old', default='')
    ap.add_argument('--rounds', type=int, default=2)
    ap.add_argument('--limit', type=int, default=400)
    a = ap.parse_args()
    o = os.path.join(ROOT, 'gpurun_out', '%s_%s' % (a.job, a.tag))
    os.makedirs(o, exist_ok=True)
    try:
        JOBS[a.job](o, a)
    except Stop as s:
        sys.exit(s.args[0] if s.args and s.args[0] else 1)


if __name__ == '__main__':
    main()
