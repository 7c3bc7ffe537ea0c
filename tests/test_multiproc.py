"""world_size-2 gloo rehearsal of bench.py's multi-GPU plumbing on CPU: contiguous env shards keyed by
global env id, barrier + max-over-ranks timing, no data-path collective."""
import os
import socket

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

import bench  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    off, cnt = bench.shard(total, world, rank)
    ids = torch.arange(off, off + cnt)
    gathered = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(gathered, torch.tensor([off, cnt]))
    elapsed = torch.tensor([1.0 + rank], dtype=torch.float64)
    dist.barrier()
    dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    out[rank] = (int(ids.sum()), [tuple(g.tolist()) for g in gathered], float(elapsed))
    dist.destroy_process_group()


@pytest.mark.parametrize("total", [65536, 4097])
def test_two_rank_shards_and_max_timing(total):
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), total, out), nprocs=world, join=True)
    sums = sum(out[r][0] for r in range(world))
    assert sums == total * (total - 1) // 2           # every global env id exactly once
    shards = out[0][1]
    assert shards[0][0] == 0 and shards[1][0] == shards[0][1] and sum(c for _, c in shards) == total
    assert out[0][2] == out[1][2] == 2.0              # max over ranks


def test_shard_helper_covers_all_ids():
    for total in (1, 7, 65536, 65537):
        for world in (1, 2, 4, 8):
            spans = [bench.shard(total, world, r) for r in range(world)]
            assert spans[0][0] == 0
            for (o0, c0), (o1, _) in zip(spans, spans[1:]):
                assert o0 + c0 == o1
            assert sum(c for _, c in spans) == total
