"""bench.py driver contract on CPU ranks: ``--gpus N`` self-launches N ranks under torch.distributed.run (child
process), the ranks form one communicator of that size, and rank 0 prints exactly one JSON line with the fields the
driver reads (the same path the 8-GPU scaling run takes, with gloo instead of RCCL)."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("gpus", [1, 2])
def test_bench_json_contract(gpus):
    env = dict(os.environ, OMP_NUM_THREADS="1", MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--device", "cpu",
                        "-n", "12", "--steps", "2", "--warmup", "1"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in out
    assert out["n_gpus"] == gpus and out["config"]["ranks"] == gpus
    assert out["config"]["backend"] == ("gloo" if gpus > 1 else "none")
    assert out["steps"] == 2 and out["warmup"] == 1 and out["value"] > 0
    assert out["config"]["global_batch"] == 12**3
    assert abs(out["value"] - 12**3 * 1000.0 / out["ms_per_step"]) < 1e-6 * out["value"]
    # the second headline config (Evrard with self-gravity) is timed in the same invocation
    assert out["evrard_value"] > 0 and out["evrard_ms_per_step"] > 0 and out["evrard_particles"] > 0
    assert abs(out["evrard_value"] - out["evrard_particles"] * 1000.0 / out["evrard_ms_per_step"]) < \
        1e-6 * out["evrard_value"]
