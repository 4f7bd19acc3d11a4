"""N>1 path on CPU: two ranks over gloo exercise the gradient-arena exchange
(ArenaGradReducer, bucketed SUM all-reduce + 1/world folded into the optimizer),
rank initialisation from the torchrun environment, and the clip sharding."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sam2_video.training.ddp import ArenaGradReducer, init_from_env, shard_clips


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, bucket_bytes, async_op, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        r, w, local = init_from_env("gloo")
        assert (r, w, local) == (rank, world, rank)
        g = torch.arange(n, dtype=torch.float32) * (rank + 1) + rank
        red = ArenaGradReducer(g, bucket_bytes=bucket_bytes)
        works = red.reduce(async_op=async_op)
        for wk in works:
            wk.wait()
        base = torch.arange(n, dtype=torch.float32)
        expect = sum(base * (k + 1) + k for k in range(world))
        ok = torch.equal(g, expect) and red.grad_scale == 1.0 / world and len(red.buckets) == -(-n * 4 // bucket_bytes)
        # the averaged gradient the optimizer sees (grad_scale folded into AdamW)
        avg_ok = torch.allclose(g * red.grad_scale, expect / world)
        q.put((rank, bool(ok and avg_ok), ""))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, False, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("async_op", [False, True])
def test_arena_allreduce_two_ranks(async_op):
    world, n, bucket = 2, 300_001, 256 << 10  # ragged last bucket
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, bucket, async_op, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res


def test_single_process_is_a_noop():
    g = torch.ones(10)
    red = ArenaGradReducer(g)
    assert red.world == 1 and red.grad_scale == 1.0 and red.reduce() == []


def test_clip_sharding_is_disjoint_and_complete():
    world, steps = 4, 5
    shards = [shard_clips(steps, r, world) for r in range(world)]
    flat = sorted(i for s in shards for i in s)
    assert flat == list(range(world * steps))
