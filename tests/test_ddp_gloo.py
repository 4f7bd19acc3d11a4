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


# ------------------------------------------------------------------------------------------------
# StepRunner on 4 ranks (round 5): the real fit-loop host logic -- accumulation windows, the
# all-reduce only at window boundaries (also the overlapped per-segment range reduces of the staged
# backward), 1/(world x accumulate) folded into the clip + AdamW -- over gloo, with a CPU stand-in for
# the GPU step: every rank's "backward" writes a synthetic per-clip gradient whose size depends on the
# clip's object count (ranks see different object counts, as real clips do).  Checked against one
# process on the mean gradient with torch's clip_grad_norm_ + AdamW.  The optimizer kernels are
# replaced by their torch restatement (they are checked against torch on the GPU:
# tests/test_kernels_gpu.py::test_clip_adamw_matches_torch).

N_ARENA, SPLIT, CUTS = 4_099, 2_500, [2_500, 3_100, 3_100, 4_099]


def _clip_grad(clip):
    """the synthetic gradient of clip `clip`: its object count (1..13) scales a fixed pattern"""
    n_obj = 1 + (clip * 7) % 13
    gen = torch.Generator().manual_seed(1000 + clip)
    return torch.randn(N_ARENA, generator=gen) * n_obj / 13.0


class _Arena:
    def __init__(self):
        self.n_grad, self.grad_split, self.grad_cuts = N_ARENA, SPLIT, list(CUTS)
        self.device = torch.device("cpu")
        self.grad = torch.zeros(N_ARENA)
        self.data = torch.linspace(-1, 1, N_ARENA)
        self.exp_avg = torch.zeros(N_ARENA)
        self.exp_avg_sq = torch.zeros(N_ARENA)
        self.shadow = None

    def grad_region(self):
        return self.grad[: self.n_grad]

    def zero_grad(self):
        self.grad.zero_()


class _AddGrad(torch.autograd.Function):
    """loss node whose backward writes [lo, hi) of the clip's gradient into the arena"""

    @staticmethod
    def forward(ctx, x, arena, g, lo, hi):
        ctx.arena, ctx.g, ctx.lo, ctx.hi = arena, g, lo, hi
        return x.sum() * 0.0

    @staticmethod
    def backward(ctx, go):
        ctx.arena.grad[ctx.lo:ctx.hi] += ctx.g[ctx.lo:ctx.hi]
        return torch.ones(1), None, None, None, None


class _Model:
    def __init__(self, overlap):
        self.arena = _Arena()
        self.frame_batched = overlap
        self.last_backbone_outputs = None

    def backbone_backward_segments(self, pend):
        """the backbone's staged backward: segment k completes arena range CUTS[k]:CUTS[k+1]"""
        segs = []
        for k in range(len(CUTS) - 1):
            def run(k=k):
                lo, hi = CUTS[k], CUTS[k + 1]
                self.arena.grad[lo:hi] += self._g[lo:hi]
            segs.append((run, k))
        return segs


class _Module:
    def __init__(self, overlap, clip_val):
        self.model = _Model(overlap)
        self.gradient_clip_val = clip_val
        self.logged, self.last_outputs, self.optimizer, self.lr_at = {}, None, None, None

    def configure_optimizers(self, total_steps=None):
        from sam2_video.training.optim import ArenaAdamW
        self.optimizer = ArenaAdamW(self.model.arena, lr=1e-3, weight_decay=0.01, max_grad_norm=self.gradient_clip_val)

    def log(self, name, value, **kw):
        self.logged[name] = value

    def training_step(self, clip, i):
        m = self.model
        g = _clip_grad(int(clip))
        m._g = g
        x = torch.ones(1, requires_grad=True)
        if m.frame_batched:  # phase 1 writes the tracking region; the segments write the backbone tail
            h = x * 1.0
            m.last_backbone_outputs = [h]
            return _AddGrad.apply(h, m.arena, g, 0, SPLIT)
        return _AddGrad.apply(x, m.arena, g, 0, N_ARENA)


def _torch_kernels(monkeypatch_ops):
    """the fused clip + AdamW kernels restated in torch (test double for the CPU ranks)"""
    import math

    def grad_norm(g, max_norm, ws, out, grad_scale=1.0):
        norm = float((g.double() * grad_scale).norm())
        c = min(1.0, max_norm / (norm + 1e-6)) if max_norm > 0 else 1.0
        out[0], out[1] = norm, c * grad_scale
        return out

    def adamw(p, g, m, v, clip, lr, beta1, beta2, eps, wd, step, shadow=None):
        gi = g * clip[1]
        p.mul_(1 - lr * wd)
        m.lerp_(gi, 1 - beta1)
        v.mul_(beta2).addcmul_(gi, gi, value=1 - beta2)
        bc1, bc2 = 1 - beta1 ** step, 1 - beta2 ** step
        p.addcdiv_(m, (v / bc2).sqrt() + eps, value=-lr / bc1)

    monkeypatch_ops.grad_norm, monkeypatch_ops.adamw = grad_norm, adamw
    return math


def _worker_runner(rank, world, port, acc, overlap, steps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        init_from_env("gloo")
        from sam2_video.kernels import ops
        from sam2_video.training import optim
        from sam2_video.training.trainer import StepRunner
        _torch_kernels(ops)
        optim.ops = ops
        mod = _Module(overlap, clip_val=1.0)
        run = StepRunner(mod, total_steps=steps, distributed=True, accumulate_grad_batches=acc)
        assert run.overlap == overlap
        clips = shard_clips(steps * acc, rank, world)
        took = [run(torch.tensor(c)) for c in clips]
        assert run.global_step == steps and run.micro_step == steps * acc
        assert len(took) == steps * acc
        q.put((rank, True, mod.model.arena.data.clone()))
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, False, traceback.format_exc() + repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [False, True])
def test_step_runner_four_ranks_accumulation_matches_single_process(overlap):
    world, acc, steps = 4, 3, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_runner, args=(r, world, port, acc, overlap, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), [r[2] for r in res if not r[1]]
    # every rank ends with the same weights
    for _, _, w in res[1:]:
        assert torch.equal(w, res[0][2])
    # one process: the mean over ranks of each window's summed micro-gradients / accumulate, then
    # torch's clip_grad_norm_(1.0) + AdamW; rank r's micro-step i of window s trains clip
    # shard_clips(...)[s * acc + i] -- object counts differ from rank to rank
    p = torch.linspace(-1, 1, N_ARENA).requires_grad_(True)
    opt = torch.optim.AdamW([p], lr=1e-3, weight_decay=0.01)
    shards = [shard_clips(steps * acc, r, world) for r in range(world)]
    counts = {1 + (c * 7) % 13 for s in shards for c in s}
    assert len(counts) > world  # the ranks really see different object counts
    for s in range(steps):
        g = sum(_clip_grad(shards[r][s * acc + i]) for r in range(world) for i in range(acc)) / (acc * world)
        p.grad = g.clone()
        torch.nn.utils.clip_grad_norm_([p], 1.0)
        opt.step()
    torch.testing.assert_close(res[0][2], p.detach(), atol=2e-6, rtol=1e-5)
