"""bench.py --gpus 2 end to end on one GPU: the launcher (torch.distributed.run), the gloo
rendezvous, two rank processes whose peer-mapped exchange opens its regions with hipIpc handles,
the timing with its barriers and max over ranks, the parity legs against a one-GPU engine, and
rank 0's one JSON line -- the path the
driver's multi-GPU bench takes, with both ranks on device 0 (PGCN_BENCH_SHARE_GPU=1, a rehearsal:
the value is not a scaling measurement)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus2_shared_gpu():
    env = dict(os.environ, PGCN_BENCH_SHARE_GPU="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps",
                        "3", "--warmup", "1", "--workload", "reddit-11.6M", "--no-cpu-baseline",
                        "--no-extra"], cwd=REPO, env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["warmup"] == 1
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert out["config"].get("exchange") == "peer", out["config"]
    # N > 1 lines carry their own parity: every rank's rows of the logits and the epoch lines
    # against a world-1 engine, after 2 fresh epochs and after the timed run
    par = out["parity"]
    assert par["pass"], par
    assert par["logits"]["gathered_from_ranks"] == 2
    assert par["logits"]["values"] == 232965 * 41
    assert par["after_timed"]["epochs"] == 2 + 1 + 3 + 2, par["after_timed"]
    assert par["after_timed"]["pass"], par["after_timed"]


def test_bench_one_gpu_default_line():
    """bench.py at N = 1 with its secondary measurements (the restricted-output and reference-
    order engines) -- the driver's default invocation minus the CPU leg, on the small
    reddit-11.6M workload: one JSON line with the contract's keys, the roofline object and the
    secondary values."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "3", "--warmup",
                        "1", "--workload", "reddit-11.6M", "--no-cpu-baseline"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in out, k
    assert out["n_gpus"] == 1 and out["steps"] == 3 and out["value"] > 0
    assert out["roofline"]["bound"] == "hbm" and 0 < out["roofline"]["frac"] < 1
    assert out["value_restricted"] > 0 and out["value_reference_order"] > 0
