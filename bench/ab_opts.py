"""Interleaved same-box A/B of EngineOptions on the headline step.

    python bench/ab_opts.py --out ab.json --rounds 3 "" "persist_bn=1" "hconv_row=0"

Runs ``bench.py --no-overhead`` once per option string per round (MERCURY_ENGINE_OPTS set to the
string; "" = defaults), interleaved so clock / thermal drift hits every arm alike, and writes
ms/step and solo graph times per arm.  The parent process never touches the GPU (each run is a
child process)."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('opts', nargs='+')
    ap.add_argument('--out', required=True)
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--steps', type=int, default=300)
    ap.add_argument('--config', default='resnet18-cifar10')
    ap.add_argument('--timeout', type=int, default=240)
    args = ap.parse_args()
    res = {o: [] for o in args.opts}
    for rnd in range(args.rounds):
        for o in args.opts:
            env = dict(os.environ, MERCURY_ENGINE_OPTS=o)
            cmd = [sys.executable, os.path.join(ROOT, 'bench.py'), '--steps', str(args.steps),
                   '--warmup', '30', '--no-overhead', '--config', args.config]
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=args.timeout)
            if p.returncode != 0:
                sys.stderr.write(p.stderr[-3000:])
                raise SystemExit('bench failed for %r (rc %d)' % (o, p.returncode))
            d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith('{')][-1])
            res[o].append({'ms_per_step': d['ms_per_step'], 'solo_ms': d.get('solo_ms')})
            print('%-60s %.4f %s' % (o or '(defaults)', d['ms_per_step'], d.get('solo_ms')),
                  flush=True)
    summ = {o or '(defaults)': sorted(r['ms_per_step'] for r in v) for o, v in res.items()}
    json.dump({'config': args.config, 'steps': args.steps, 'runs': res, 'ms_sorted': summ},
              open(args.out, 'w'), indent=1)


if __name__ == '__main__':
    main()
