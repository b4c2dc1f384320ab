"""CPU, gloo: `bench.py --gpus 2` starts two ranks by itself (torch.distributed.run as a child,
before anything touches a GPU) and rank 0's JSON line reports n_gpus = 2 with the per-cloud
checksums of the single-process run over the same global clouds (contiguous batch split,
SURVEY.md §8(e); pointnet2_tensorflow/train_multi_gpu.py:181-190)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*argv):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only prints
    return json.loads(lines[0]), r.stderr


@pytest.mark.timeout(300)
def test_bench_self_launches_ranks():
    two, err = _bench("--gpus", "2", "--dry-run", "--batch", "2")
    assert "launching 2 ranks" in err
    assert two["n_gpus"] == 2 and two["dry_run"]
    assert two["clouds"] == 4 and two["config"]["global_batch"] == 4
    assert two["config"]["parallelism"] == "dp2 (batch split)"
    one, _ = _bench("--gpus", "1", "--dry-run", "--batch", "4")
    assert one["n_gpus"] == 1
    assert two["per_cloud_checksums"] == one["per_cloud_checksums"]
    assert two["elapsed_max_over_ranks"] > 0


@pytest.mark.timeout(600)
def test_bench_cfg4_split_dry_run():
    """cfg4's split (B = 128 over 8 GPUs, 16 per rank; train_multi_gpu.py:181-190) rehearsed on
    8 gloo ranks: rank r owns global clouds 16 r .. 16 r + 15 of every buffer set, the sets hold
    disjoint clouds, every rank's HIP would start with the config's hardware-queue count
    (<= 32, set before anything touches the GPU), and the gathered per-cloud checksums come
    back in global cloud order, equal to one process running all 128 clouds."""
    eight, err = _bench("--gpus", "8", "--dry-run", "--batch", "16")
    assert "launching 8 ranks" in err
    assert eight["n_gpus"] == 8 and eight["clouds"] == 128
    assert eight["config"]["parallelism"] == "dp8 (batch split)"
    ranks = eight["ranks"]
    assert [r["rank"] for r in ranks] == list(range(8))
    seen = set()
    for r in ranks:
        assert r["ids"] == list(range(16 * r["rank"], 16 * r["rank"] + 16))
        assert r["hw_queues"] is not None and 1 <= int(r["hw_queues"]) <= 32
        assert int(r["hw_queues"]) == int(ranks[0]["hw_queues"])
        assert len(r["set_ids"]) == eight["sets"]
        assert r["set_ids"][0] == r["ids"]
        for ids in r["set_ids"]:
            assert not seen & set(ids)
            seen |= set(ids)
    assert seen == set(range(128 * eight["sets"]))
    one, _ = _bench("--gpus", "1", "--dry-run", "--batch", "128")
    assert one["per_cloud_checksums"] == eight["per_cloud_checksums"]
