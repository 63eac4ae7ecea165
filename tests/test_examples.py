"""The CPU plumbing example (BASELINE.json config 1) runs end to end and reports its line."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpu_reference_step_uniform_runs():
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'examples', 'cpu_reference_step.py'),
                        '--uniform', '--steps', '1', '--warmup', '0', '--threads', '4'],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out['value'] > 0 and out['sampler'] == 'uniform' and out['n_gpus'] == 0
