"""CPU, world_size 2 over gloo: the multi-GPU path of bench.py (contiguous batch split, no data
collective, max-over-ranks timing, per-cloud checksum gather) reproduces the single-process
result for the same global clouds. The per-rank compute is the oracle step (no GPU here)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _step_checksums(cloud_ids):
    import importlib
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
    inp = pkg.stack.make_inputs("cfg2", cloud_ids, "cpu")
    np_inp = dict(inp)
    np_inp["xyz"] = inp["xyz"].numpy()
    np_inp["sa_out"] = [t.numpy() for t in inp["sa_out"]]
    np_inp["fp_out"] = [t.numpy() for t in inp["fp_out"]]
    outs = [torch.from_numpy(o) for o in O.run_stack_cpu(np_inp, "cfg2")]
    return pkg, pkg.shard.cloud_checksums(outs, len(cloud_ids))


def _worker(rank, world, port, per_rank, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import importlib
        import sys
        sys.path.insert(0, ROOT)
        pkg = importlib.import_module("pointcloud-segmentation-attention_amd")
        ids = pkg.shard.shard_ids(rank, world, per_rank)
        _, sums = _step_checksums(ids)
        allsums = pkg.shard.gather_checksums(sums)
        elapsed = pkg.shard.max_over_ranks(0.25 * (rank + 1))
        if rank == 0:
            q.put((allsums.numpy(), elapsed))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_batch_split_matches_single_process():
    world, per_rank = 2, 1
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, per_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    allsums, elapsed = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    _, ref = _step_checksums(list(range(world * per_rank)))
    assert np.array_equal(allsums, ref.numpy())
    assert elapsed == 0.5  # max over ranks
