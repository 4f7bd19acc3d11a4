"""The N > 1 training path on the GPU box: two ranks sharing its one MI355X over gloo (RCCL needs
one GPU per rank; the collective's transport is the only difference), each training its own clip
with StepRunner(distributed=True, graph=True): the staged backbone backward with an all-reduce per
completed arena range (SAM2Model.backbone_backward_segments, arena.grad_cuts), clip + AdamW on the
averaged gradient.  After every step the two ranks' parameter arenas must be bit-identical -- a
range reduced before its gradients were complete (conv_s0 / conv_s1 were, in round 2) makes them
diverge."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path.insert(0, here)
        sys.path.insert(0, os.path.join(os.path.dirname(here), "sam2-video-training_amd"))
        torch.cuda.set_device(0)
        from sam2_video.data.synthetic import make_clip, sam2_collate_fn
        from sam2_video.kernels import functional as FN
        from sam2_video.model.sam2model import SAM2Model
        from sam2_video.training.ddp import init_from_env
        from sam2_video.training.trainer import SAM2LightningModule, StepRunner
        init_from_env("gloo")
        FN.set_seed(1234 + rank)
        ALL = ["image_encoder", "memory_attention", "memory_encoder", "mask_decoder", "prompt_encoder"]
        model = SAM2Model(None, "base_plus@256", trainable_modules=ALL, compute_dtype="bf16")
        loss = {"weight_dict": {"loss_mask": 20, "loss_dice": 1, "loss_iou": 1, "loss_class": 0},
                "supervise_all_iou": True, "iou_use_l1_loss": True}
        mod = SAM2LightningModule(model, loss, {"type": "AdamW", "lr": 1e-4}, {"enabled": False})
        mod.setup("fit", torch.device("cuda", 0))
        run = StepRunner(mod, total_steps=3, distributed=True, graph=True)
        ok = run.overlap and len(run.cuts) == len(model.image_encoder.trunk.stage_ends) + 2
        arena = model.arena
        before = arena.data.clone()
        sums = []
        for step in range(3):
            clip = make_clip(50 + 2 * step + rank, 3, 256, 4, 3)
            run(sam2_collate_fn([clip]).to("cuda"))
            torch.cuda.synchronize()
            t = arena.data.double().sum().cpu().view(1)
            allt = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
            dist.all_gather(allt, t)
            sums.append([float(x) for x in allt])
        # exact equality of the whole arena across ranks after the last step
        mine = arena.data.cpu()
        other = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(other, mine)
        ok = ok and all(a[0] == a[1] for a in sums) and torch.equal(other[0], other[1])
        ok = ok and not torch.equal(before.cpu(), mine)  # the parameters moved
        q.put((rank, bool(ok), f"overlap={run.overlap} sums={sums}"))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, False, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_two_ranks_stay_identical_with_staged_overlap():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=400) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
