"""bench.py's multi-rank launch path on the CPU: `--gpus N` without
torch.distributed's environment starts N rank processes through torch.distributed.run, each
rank joins the gloo rendezvous and stops cleanly at the point of GPU use when it has no device;
a WORLD_SIZE that disagrees with --gpus exits 2 before anything starts; `--dry-run` prints the
partition every rank would build."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kv):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["HIP_VISIBLE_DEVICES"] = ""  # a GPU box too: no device for the ranks
    env["CUDA_VISIBLE_DEVICES"] = ""
    env.update(kv)
    return env


def test_gpus2_launches_ranks_that_stop_without_a_device():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode != 0
    for rank in (0, 1):  # both ranks came up with their own env, through the rendezvous
        assert f"bench.py: rank {rank}/2 (local {rank}): no HIP device" in r.stderr, r.stderr[-3000:]
    assert r.stdout.strip() == ""  # no JSON line from a run that measured nothing


def test_world_size_mismatch_exits_2():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1"],
                       env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 2
    assert "--gpus 2 but WORLD_SIZE 3" in r.stderr


def test_dry_run_partition():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--dry-run", "--workload",
                        "reddit-11.6M"], env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout)
    ranks = out["ranks"]
    assert out["gpus"] == 4 and len(ranks) == 4
    assert ranks[0]["nodes"][0] == 0 and ranks[-1]["nodes"][1] == out["nodes"]
    for a, b in zip(ranks, ranks[1:]):
        assert a["nodes"][1] == b["nodes"][0]
    assert sum(x["column_block_nnz"] for x in ranks) == out["adjacency_nnz"]
    assert out["nnz_imbalance"] < 1.01  # nnz-balanced ranges
    assert max(x["rows"] for x in ranks) <= out["maxrows"]
    # every rank sends the partial sums of the other ranks' rows (16 floats each) per GraphSum
    for x in ranks:
        assert x["graphsum_send_bytes"]["16"] == (out["nodes"] - x["rows"]) * 64
