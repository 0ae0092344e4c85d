"""bench.py's own flows, end to end at small sizes (one process per case, each under a time
limit): the JSON line is printed and well formed, and its self-checks pass.

  * the one-GPU lazy owner path at the reference configs' 64-walk batch (the rows-major out
    step, eager warmup then graph replay) on an R-MAT 14 graph;
  * the headline composition (dense Adam, records path) with the batch64 line and its checked
    step, on an R-MAT 14 graph;
  * the C2 shape (HIP-graph replay, atomic scatter).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=240):
    env = dict(os.environ)
    env.pop('WORLD_SIZE', None)
    p = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), *args],
                       capture_output=True, text=True, timeout=timeout, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith('{')]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_lazy_owner_64_walks_small_graph():
    d = _bench('--scale', '14', '--edges', '100000', '--batch-walks', '64', '--n1-in-adam', 'lazy',
               '--steps', '32', '--warmup', '4', '--no-cpu-baseline', '--no-walk-bench',
               '--batch64-steps', '0')
    assert d['value'] > 0 and d['ms_per_step'] > 0
    assert 'owner path on one rank' in d['config']['parallelism']
    assert d['mean_loss'] is not None and 0 < d['mean_loss'] < 10


def test_bench_headline_with_batch64_small_graph():
    d = _bench('--scale', '14', '--edges', '100000', '--batch-walks', '512', '--steps', '8',
               '--warmup', '2', '--no-cpu-baseline', '--no-walk-bench', '--exact-steps', '0',
               '--batch64-steps', '32', '--batch64-long', '160')
    b = d['batch64']
    assert b['value'] > 0 and b['step_check']['ok'], b['step_check']
    # the steady-state leg: replays on to 160 steps, the last ones timed, then the check
    assert b['steady_state']['steps'] == 128 and b['steady_state']['ms_per_step'] > 0
    assert b['roofline']['touched_out_rows'] > 0 and b['roofline']['touched_in_rows'] > 0


def test_bench_c2_graph_replay():
    d = _bench('--config', 'c2', '--steps', '32', '--warmup', '2', '--no-cpu-baseline',
               '--no-walk-bench')
    assert d['value'] > 0 and d['roofline']['graph']
