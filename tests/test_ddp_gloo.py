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


def _worker_overlap(rank, world, port, q):
    """region reduce (the overlap path): tracking region first (async), image-encoder tail after;
    then clip + AdamW on the averaged gradient equals one process on the mean of the rank
    gradients (torch's clip_grad_norm_ + AdamW as the arithmetic the fused kernels restate)"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        init_from_env("gloo")
        n, split = 50_003, 20_001
        cuts = [split, 23_000, 23_000, 41_517, n]  # staged backbone ranges (one empty), StepRunner.cuts
        torch.manual_seed(rank)
        g = torch.randn(n) * (rank + 1)
        mine = g.clone()
        red = ArenaGradReducer(g, bucket_bytes=64 << 10, split=split)
        works = red.reduce_range(0, red.split)  # issued before the tail is "computed"
        for lo, hi in zip(cuts, cuts[1:]):  # one range per completed backward segment
            works += red.reduce_range(lo, hi)
        for w in works:
            w.wait()
        allg = [torch.zeros(n) for _ in range(world)]
        dist.all_gather(allg, mine)
        mean = sum(allg) / world
        ok = torch.allclose(g * red.grad_scale, mean, atol=1e-6)
        p0 = torch.linspace(-1, 1, n)
        pa, pb = p0.clone().requires_grad_(True), p0.clone().requires_grad_(True)
        oa = torch.optim.AdamW([pa], lr=1e-3, weight_decay=0.01)
        ob = torch.optim.AdamW([pb], lr=1e-3, weight_decay=0.01)
        pa.grad = g * red.grad_scale
        pb.grad = mean.clone()
        for p_, o_ in ((pa, oa), (pb, ob)):
            torch.nn.utils.clip_grad_norm_([p_], 1.0)
            o_.step()
        ok = ok and torch.allclose(pa, pb, atol=1e-7)
        q.put((rank, bool(ok), ""))
    except Exception as e:  # pragma: no cover
        q.put((rank, False, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_region_reduce_then_adamw_equals_single_process_on_mean():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_overlap, args=(r, world, port, q)) for r in range(world)]
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
