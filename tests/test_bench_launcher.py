"""bench.py's multi-rank launcher on CPU (gloo): ``--gpus 2`` with no
WORLD_SIZE in the environment brings up two ranks itself (torch.distributed.run,
127.0.0.1), each worker checks that the process group is 2 wide, the timing
brackets and the metric all-reduce run, and rank 0 prints one JSON line
with n_gpus = 2 and the all-rank metric sums.  The HIP step is replaced by a
no-op (``--selftest-launcher``); everything around it is the bench's code."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    return env


def test_launcher_brings_up_two_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "3", "--warmup", "1", "--selftest-launcher"],
                       capture_output=True, text=True, env=_env(), timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["selftest"] is True
    # rank r contributes 4 rows of (r + 1): 4 * 1 + 4 * 2 per field
    assert d["metric_sums"] == [12.0] * 8


def test_worker_refuses_mismatched_world():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--selftest-launcher"], capture_output=True, text=True, env=env,
                       timeout=120, cwd=ROOT)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in (r.stderr + r.stdout)
