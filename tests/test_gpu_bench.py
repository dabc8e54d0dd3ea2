"""bench.py's multi-rank contract on the one-GPU box: `--gpus 2` without a
launcher starts the two rank processes itself (both on the one device), the
JSON line reports n_gpus 2 and the C2 replica aggregate, and the C4 sharded
sub-line (korali.Engine, Distributed conduit over the Host transport here:
RCCL refuses two ranks on one device) ends bit-identical to the one-rank
run."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus_2_spawns_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20", "--warmup", "3",
                        "--no-cpu-baseline"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "replicas2"
    assert out["value"] > 0
    c4 = out["c4_sharded"]
    assert c4["ranks"] == 2 and c4["bit_identical_to_1_rank"], c4
    print(json.dumps(c4))
