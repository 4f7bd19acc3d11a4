"""Host side of the Lightning-shaped surface (CPU): the reference's Hydra config tree composes
and its `module` / `data_module` / `trainer` / `model` sections instantiate through this
build's `_target_` resolver; trainer settings (gradient_clip_val, accumulate_grad_batches,
precision) reach the optimizer and the step runner; the data module yields B == 1 clips of the
data section's shape; Lightning checkpoints round-trip with the `model.` prefix."""
import os
from types import SimpleNamespace

import pytest
import torch

REF_CONFIGS = "/root/reference/configs"
needs_ref = pytest.mark.skipif(not os.path.isdir(REF_CONFIGS), reason="reference config tree not present")


def _fake_arena():
    return SimpleNamespace(device=torch.device("cpu"), n_grad=0)


@needs_ref
def test_best_yaml_composes_and_instantiates():
    from sam2_video.model.build import instantiate
    from sam2_video.model.sam2model import SAM2Model
    from sam2_video.training.trainer import SAM2LightningDataModule, SAM2LightningModule, Trainer
    from sam2_video.utils.config import compose
    cfg = compose(REF_CONFIGS, "best", ["+trainer.max_steps=3", "data.video_clip_length=2", "data.image_size=128",
                                        "+data.synthetic_clips=2"])
    assert cfg["module"]["model"] == cfg["model"]  # ${model} interpolation keeps the dict
    assert cfg["data"]["name"] == "cholecseg8k" and cfg["data"]["num_categories"] == 13
    module = instantiate(cfg["module"], _recursive_=False)
    assert isinstance(module, SAM2LightningModule) and module.model is None
    assert isinstance(module.cfg.model, dict) and module.cfg.model["_target_"].endswith("SAM2Model")
    assert module.loss_gt_stride == 1
    dm = instantiate(cfg["data_module"], _recursive_=False)
    assert isinstance(dm, SAM2LightningDataModule)
    dm.setup("fit")
    b = next(iter(dm.train_dataloader()))
    assert tuple(b.img_batch.shape) == (2, 1, 3, 128, 128) and tuple(b.masks.shape) == (2, 13, 128, 128)
    tr = instantiate(cfg["trainer"])
    assert isinstance(tr, Trainer)
    assert tr.gradient_clip_val == 1.0 and tr.accumulate_grad_batches == 16 and tr.max_steps == 3
    # the configured checkpoint does not exist here: fail fast, as upstream build_sam2 does
    with pytest.raises(FileNotFoundError):
        instantiate(cfg["model"])
    # the model section builds the module tree (checkpoint_path=null: deterministic synthetic
    # weights); the reference's own sam2/sam2.1_hiera_t.yaml is image_size 384
    cfg = compose(REF_CONFIGS, "best", ["model.checkpoint_path=null"])
    model = instantiate(cfg["model"])
    assert isinstance(model, SAM2Model) and model.image_size == 384
    assert sorted(model.get_trainable_modules()) == ["memory_attention", "memory_encoder"]


@needs_ref
def test_trainer_clip_value_reaches_the_optimizer():
    """memory_overfit.yaml sets trainer.gradient_clip_val 0.1: the fused clip uses it;
    0 / None disable clipping like Lightning"""
    from sam2_video.model.build import instantiate
    from sam2_video.training.trainer import SAM2LightningModule
    from sam2_video.utils.config import compose
    cfg = compose(REF_CONFIGS, "memory_overfit")
    tr = instantiate(cfg["trainer"])
    assert tr.gradient_clip_val == 0.1 and tr.limit_train_batches == 1
    mod = SAM2LightningModule(SimpleNamespace(arena=_fake_arena()), cfg["loss"], cfg["optimizer"], cfg["scheduler"])
    mod.model = mod.cfg.model
    for clip, expect in ((tr.gradient_clip_val, 0.1), (0, 0.0), (None, 0.0), (3, 3.0)):
        mod.gradient_clip_val = clip
        opt = mod.configure_optimizers(10)["optimizer"]
        assert opt.max_grad_norm == expect
        assert opt.eps == 1e-8  # the YAML's eps is not forwarded (trainer.py:124-130)


def test_precision_maps_to_compute_dtype():
    from sam2_video.training.trainer import precision_dtype
    assert precision_dtype(16) == "bf16" and precision_dtype("bf16-mixed") == "bf16"
    assert precision_dtype("32-true") == "fp32" and precision_dtype(32) == "fp32"


def test_overrides_and_interpolation(tmp_path):
    from sam2_video.utils.config import compose
    (tmp_path / "grp").mkdir()
    (tmp_path / "grp" / "a.yaml").write_text("x: 1\ny: {z: 2}\n")
    (tmp_path / "base.yaml").write_text("defaults:\n  - grp: a\n  - _self_\nk: ${grp.y}\ns: run-${grp.x}\n"
                                        "d: ${hydra:run.dir}/ck\n")
    cfg = compose(str(tmp_path), "base", ["grp.x=5", "+new.v=[1, 2]"], run_dir="/tmp/r")
    assert cfg["k"] == {"z": 2} and cfg["s"] == "run-5" and cfg["d"] == "/tmp/r/ck"
    assert cfg["new"]["v"] == [1, 2]
    with pytest.raises(KeyError):
        compose(str(tmp_path), "base", ["nope.v=1"])


def test_lightning_checkpoint_prefix_strip(tmp_path):
    from sam2_video.model.sam2model import SAM2Model
    sd = {"model.a.weight": torch.ones(2), "model.b": torch.zeros(1)}
    assert set(SAM2Model.strip_lightning_prefix({"state_dict": sd})) == {"a.weight", "b"}
    assert SAM2Model.strip_lightning_prefix({"a": 1}) == {"a": 1}


def test_lightning_checkpoint_round_trip(tmp_path):
    """Trainer.save_checkpoint writes the Lightning layout (`state_dict` with the `model.` prefix,
    optimizer states, counters); load_lightning_checkpoint and the fintuned_model_path branch
    (reference sam2model.py:109-126 with train.py:146-157's unwrapping) restore every tensor of a
    differently initialised model exactly"""
    from sam2_video.model.sam2model import SAM2Model
    from sam2_video.training.trainer import Trainer
    src = SAM2Model(None, "tiny@128", trainable_modules=["memory_attention"], init_seed=3)
    opt_state = {"step": 7, "lr": 1e-4}
    module = SimpleNamespace(model=src, optimizer=SimpleNamespace(state_dict=lambda: opt_state))
    tr = Trainer(max_steps=1)
    path = str(tmp_path / "last.ckpt")
    tr.save_checkpoint(path, module)
    ck = torch.load(path, map_location="cpu", weights_only=True)
    assert all(k.startswith("model.") for k in ck["state_dict"]) and ck["optimizer_states"] == [opt_state]
    want = src.state_dict()
    dst = SAM2Model(None, "tiny@128", trainable_modules=["memory_attention"], init_seed=11)
    assert any(not torch.equal(want[k], v) for k, v in dst.state_dict().items())
    dst.load_lightning_checkpoint(path)
    assert all(torch.equal(want[k], v) for k, v in dst.state_dict().items())
    ft = SAM2Model(None, "tiny@128", fintuned_model_path=path, trainable_modules=["memory_attention"], init_seed=11)
    assert all(torch.equal(want[k], v) for k, v in ft.state_dict().items())
    # a checkpoint missing a tensor is refused under strict loading
    del ck["state_dict"]["model.no_mem_embed"]
    torch.save(ck, path)
    with pytest.raises(RuntimeError):
        SAM2Model(None, "tiny@128", init_seed=11).load_lightning_checkpoint(path)


def test_synthetic_clip_dataset_and_parts():
    from sam2_video.data.synthetic import SyntheticClipDataset, make_clip
    from sam2_video.utils.masks import cat_to_obj_mask
    ds = SyntheticClipDataset(3, 2, 128, 5, 3, parts=(2, 3))
    assert len(ds) == 3 and tuple(ds[0]["masks"].shape) == (2, 5, 128, 128)
    with pytest.raises(IndexError):
        ds[3]
    m = make_clip(7, 1, 256, 5, 3, (2, 3))["masks"][0]
    _, obj_to_cat, ncat = cat_to_obj_mask(m.unsqueeze(1))
    assert list(obj_to_cat) == [0, 0, 1, 1, 1, 2] and ncat == 5


def test_sam21_checkpoint_file_loads_and_missing_path_raises(tmp_path):
    """checkpoint_path: an upstream SAM2.1 `.pt` ({"model": state_dict}, the layout build_sam2
    loads) restores every tensor strictly; a path that does not exist raises instead of silently
    falling back to synthetic weights (upstream build_sam2, reference sam2model.py:80-82)"""
    from sam2_video.model.sam2model import SAM2Model
    src = SAM2Model(None, "tiny@128", trainable_modules=["memory_attention"], init_seed=5)
    want = src.state_dict()
    path = str(tmp_path / "sam2.1_hiera_tiny.pt")
    torch.save({"model": {k: v.clone() for k, v in want.items()}}, path)
    got = SAM2Model(path, "tiny@128", trainable_modules=["memory_attention"], init_seed=11).state_dict()
    assert set(got) == set(want) and all(torch.equal(want[k], got[k]) for k in want)
    with pytest.raises(FileNotFoundError):
        SAM2Model(str(tmp_path / "missing.pt"), "tiny@128")
    sd = {k: v.clone() for k, v in want.items()}
    del sd["no_mem_embed"]
    torch.save({"model": sd}, path)
    with pytest.raises(RuntimeError):  # strict, as upstream
        SAM2Model(path, "tiny@128")


def test_trainer_refuses_cpu_accelerator():
    from sam2_video.training.trainer import Trainer
    with pytest.raises(ValueError, match="accelerator='cpu'"):
        Trainer(accelerator="cpu")
    assert Trainer(accelerator="auto").accelerator == "auto"


class _Arena:
    def __init__(self, n):
        self.device = torch.device("cpu")
        self.grad = torch.zeros(n)
        self.data = torch.linspace(-1, 1, n)
        self.n_grad = self.grad_split = n

    def grad_region(self):
        return self.grad[: self.n_grad]

    def zero_grad(self):
        self.grad.zero_()


class _StubAdamW:
    """stands in for the fused clip + AdamW kernels of ArenaAdamW (CPU): records the gradient the
    kernels would consume (arena grad x grad_scale), the clip and the learning rate of each step"""

    def __init__(self, arena, lr=1e-4, **kw):
        self.arena = arena
        self.param_groups = [{"lr": lr}]
        self.seen, self.clips, self.lrs = [], [], []
        self.max_grad_norm = kw.get("max_grad_norm")

    def step(self, lr=None, grad_scale=1.0):
        self.seen.append(self.arena.grad_region() * grad_scale)
        self.clips.append(self.max_grad_norm)
        self.lrs.append(lr)

    def state_dict(self):
        return {"step": len(self.seen)}

    def load_state_dict(self, sd):
        pass


class _GradToArena(torch.autograd.Function):
    """a step's backward: adds `contrib` into the arena (the HIP backward kernels' contract)"""

    @staticmethod
    def forward(ctx, x, arena, contrib):
        ctx.arena, ctx.contrib = arena, contrib
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        ctx.arena.grad += ctx.contrib * g
        return g, None, None


class _StubModel(torch.nn.Module):
    """two parameters that are views of the arena's data, their `_s2h_grad` views of its gradient"""

    def __init__(self, arena):
        super().__init__()
        n = arena.n_grad
        self.arena = arena
        self.w = torch.nn.Parameter(arena.data[: n // 2].view(-1))
        self.b = torch.nn.Parameter(arena.data[n // 2:].view(-1))
        self.w._s2h_grad = arena.grad[: n // 2]
        self.b._s2h_grad = arena.grad[n // 2:]


def _stub_lightning_module(monkeypatch, n, rank, trainer):
    """SAM2LightningModule with the device parts stubbed (model forward, criterion, the fused AdamW
    kernels) and a (stub) Lightning trainer attached: what remains is the automatic-optimization
    surface -- configure_optimizers / ArenaOptimizer / configure_gradient_clipping -- under test"""
    from sam2_video.training import optim
    from sam2_video.training import trainer as T
    monkeypatch.setattr(optim, "ArenaAdamW", _StubAdamW)
    arena = _Arena(n)
    calls = {"n": 0}

    def forward(batch):
        calls["n"] += 1
        x = torch.ones((), requires_grad=True)
        contrib = torch.arange(n, dtype=torch.float32) * (rank + 1) + 10 * calls["n"]
        return [{"y": _GradToArena.apply(x, arena, contrib)}], [0]

    mod = T.SAM2LightningModule(SimpleNamespace(), {"gt_stride": 1, "iou_use_l1_loss": True,
                                                    "weight_dict": {"loss_mask": 1, "loss_dice": 1, "loss_iou": 1}},
                                {"lr": 1e-4, "warmup_factor": 0.25}, {"enabled": True})
    mod.model = _StubModel(arena)
    mod.forward = forward
    mod.criterion = _StubCriterion()
    mod._trainer = trainer
    mod.lightning_graph = False  # the eager module path: no StepRunner / graph on the stub model
    return mod, arena


class _StubCriterion(torch.nn.Module):
    def forward(self, outs, targets):
        return {"total_loss": outs[0]["y"]}


def _lightning_fit(mod, n_batches, acc, clip, scaler=None):
    """Lightning 2.x automatic optimization over n_batches (tests/lightning_stub.py: training_step,
    zero_grad on a window's first batch after it, the precision plugin's scaled module.backward; at a
    window boundary and on the epoch's last batch the optimizer step -- with precision=16 through
    GradScaler (unscale_, clip hook, scaler.step, update), else optimizer.step(closure) with the clip
    after the closure's backward -- then the per-step scheduler)"""
    from lightning_stub import StubFitLoop, lightning_fit
    tr = mod._trainer
    tr.fit_loop = StubFitLoop(acc, n_batches)
    tr.precision_plugin = SimpleNamespace(scaler=scaler)
    batch = SimpleNamespace(masks=torch.zeros(1, 1, 2, 2))
    opt = lightning_fit(mod, tr, [batch] * n_batches)
    assert isinstance(opt, torch.optim.Optimizer)
    return opt


@pytest.mark.parametrize("fp16", [False, True])
def test_lightning_automatic_optimization_clip_and_accumulate_on_the_trainer(monkeypatch, fp16):
    """the reference's Trainer section as written (best.yaml:103-106: precision 16,
    gradient_clip_val 1.0, accumulate_grad_batches 16 -- here 3): Lightning's automatic optimization
    drives the module with no user edit.  The optimizer is a torch.optim.Optimizer whose params'
    .grad are the arena slices (GradScaler unscales them in place), the window's micro-gradients
    are summed / accumulate_grad_batches, the clip reaches the fused kernel, the cosine schedule
    runs over estimated_stepping_batches (optimizer steps), and zero_grad keeps the bindings"""
    n, acc, nb = 16, 3, 7  # two full windows + a partial one (Lightning steps on the epoch's last batch)
    tr = SimpleNamespace(estimated_stepping_batches=3, accumulate_grad_batches=acc, gradient_clip_val=1.0,
                         precision="16-mixed" if fp16 else "32-true")
    mod, arena = _stub_lightning_module(monkeypatch, n, 0, tr)
    scaler = torch.amp.GradScaler("cpu", init_scale=256.0) if fp16 else None
    opt = _lightning_fit(mod, nb, acc, 1.0, scaler)
    impl = opt.impl
    base = torch.arange(n, dtype=torch.float32)
    exp = [(3 * base + 10 * (1 + 2 + 3)) / acc, (3 * base + 10 * (4 + 5 + 6)) / acc, (base + 70) / acc]
    assert len(impl.seen) == 3
    for got, want in zip(impl.seen, exp):
        torch.testing.assert_close(got, want)
    assert impl.clips == [1.0, 1.0, 1.0]
    assert impl.lrs[0] == 0.0 and 0.0 < impl.lrs[1] <= 1e-4  # warmup 0.25 x 3 steps, then cosine
    for p in mod.model.parameters():  # the bindings survive zero_grad
        assert p.grad is not None and p.grad.data_ptr() == p._s2h_grad.data_ptr()
    # Lightning zeroes a window's gradients at the next window's first micro-batch (after its
    # training_step), not after the optimizer step: the last window's stay in the arena
    torch.testing.assert_close(arena.grad, exp[-1])


def test_configure_gradient_clipping_routes_to_the_kernel(monkeypatch):
    tr = SimpleNamespace(estimated_stepping_batches=4, accumulate_grad_batches=1, gradient_clip_val=None)
    mod, _ = _stub_lightning_module(monkeypatch, 8, 0, tr)
    opt = mod.configure_optimizers()["optimizer"]
    assert opt.max_grad_norm == 0.0  # no clip on the trainer: none in the kernel
    mod.configure_gradient_clipping(SimpleNamespace(_optimizer=opt), 0.5, "norm")  # a LightningOptimizer
    assert opt.max_grad_norm == 0.5
    with pytest.raises(NotImplementedError):
        mod.configure_gradient_clipping(opt, 0.5, "value")
    sd = opt.state_dict()
    assert "param_groups_lr" in sd
    opt.load_state_dict(sd)


def _lightning_path_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        mp_ = pytest.MonkeyPatch()
        from sam2_video.training.ddp import init_from_env
        init_from_env("gloo")
        n, acc = 1000, 2
        tr = SimpleNamespace(estimated_stepping_batches=2, accumulate_grad_batches=acc, gradient_clip_val=1.0)
        mod, arena = _stub_lightning_module(mp_, n, rank, tr)
        opt = _lightning_fit(mod, 4, acc, 1.0)
        base = torch.arange(n, dtype=torch.float32)
        sumr = sum(base * (r + 1) for r in range(world))
        # window 1 = micro-steps 1, 2; window 2 = micro-steps 3, 4 (arena zeroed in between), averaged
        # over the ranks by the optimizer's arena all-reduce (grad_scale 1/world)
        exp1 = (2 * sumr + world * (10 + 20)) / (acc * world)
        exp2 = (2 * sumr + world * (30 + 40)) / (acc * world)
        seen = opt.impl.seen
        ok = opt.reducer is not None and len(seen) == 2 and torch.allclose(seen[0], exp1) and torch.allclose(seen[1], exp2)
        mp_.undo()
        q.put((rank, bool(ok), ""))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, False, traceback.format_exc()))
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def test_lightning_automatic_optimization_two_ranks_gloo():
    """the same under Lightning DDP without the DistributedDataParallel wrapper (arena_ddp_strategy)
    on 2 gloo ranks: ArenaOptimizer.step all-reduces the arena once per window"""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_lightning_path_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res


def _lightning_scaler_worker(rank, world, port, q):
    """precision=16 under DDP: rank 1's second micro-batch produces an inf gradient.  The arena is
    all-reduced in the module's backward hook (before GradScaler.unscale_ looks at it), so BOTH ranks
    find the inf, skip that window's step and lower the scale alike (with the reduce inside
    the optimizer step, only rank 1 skipped and the ranks' collectives paired up across iterations)"""
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        mp_ = pytest.MonkeyPatch()
        from sam2_video.training.ddp import init_from_env
        init_from_env("gloo")
        n, acc, nb = 64, 2, 6
        tr = SimpleNamespace(estimated_stepping_batches=3, accumulate_grad_batches=acc, gradient_clip_val=1.0,
                             precision="16-mixed")
        mod, arena = _stub_lightning_module(mp_, n, rank, tr)
        fwd = mod.forward
        calls = {"n": 0}

        def forward(batch):
            calls["n"] += 1
            outs, cats = fwd(batch)
            if rank == 1 and calls["n"] == 2:  # window 1's last micro-batch on rank 1 only
                y = outs[0]["y"]
                outs = [{"y": y * float("inf")}]
            return outs, cats
        mod.forward = forward
        scaler = torch.amp.GradScaler("cpu", init_scale=256.0)
        scales = []
        opt = _lightning_fit(mod, nb, acc, 1.0, scaler)
        scales.append(float(scaler.get_scale()))
        seen = opt.impl.seen
        ok = len(seen) == 2 and all(bool(torch.isfinite(x).all()) for x in seen)
        mp_.undo()
        q.put((rank, bool(ok), (len(seen), scales)))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, False, traceback.format_exc()))
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def test_lightning_grad_scaler_inf_on_one_rank_skips_on_every_rank():
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_lightning_scaler_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
    # the same skipped window and the same scale on both ranks (256 halved once by the skip)
    assert res[0][2] == res[1][2] and res[0][2][0] == 2 and res[0][2][1] == [128.0], res


def test_activation_checkpoint_flag_is_a_notice():
    """overfit.yaml:46 sets use_activation_checkpoint: the build accepts it, records it and says
    once at construction that it does not recompute (activations stay resident in HBM; results
    are identical, only peak memory differs from the reference's recompute)"""
    from sam2_video.model.modeling.sam2_base import ActivationCheckpointNotice
    from sam2_video.model.sam2model import SAM2Model
    with pytest.warns(ActivationCheckpointNotice, match="no recompute"):
        m = SAM2Model(None, "tiny@128", use_activation_checkpoint=True)
    assert m.use_activation_checkpoint
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("error", ActivationCheckpointNotice)
        assert not SAM2Model(None, "tiny@128").use_activation_checkpoint


@needs_ref
def test_overfit_fixture_matches_reference_composition():
    """tests/golden/overfit_cfg1.json (the GPU box's config-1 input) is exactly the reference's
    configs/overfit.yaml composed with oracle/gen_config_golden.py's overrides; its data module
    yields the reference fixture's clip (synthetic clip 7, 4 frames, 256^2, 4 of 13 categories)"""
    import json
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import gen_config_golden as gcg
    from sam2_video.data.synthetic import synthetic_batch
    from sam2_video.model.build import instantiate
    with open(gcg.OUT) as f:
        assert json.load(f) == json.loads(json.dumps(gcg.composed()))
    cfg = gcg.composed()
    dm = instantiate(cfg["data_module"], _recursive_=False)
    dm.setup("fit")
    dm.data.num_workers = 0
    b = next(iter(dm.train_dataloader()))
    ref = synthetic_batch(7, 4, 256, 13, 4)
    assert torch.equal(b.img_batch, ref.img_batch) and torch.equal(b.masks, ref.masks)


def test_data_module_shards_clips_across_ranks():
    """with a 2-rank process group the data module's loaders carry a DistributedSampler: the ranks
    see disjoint clip indices that together cover the split"""
    from torch.utils.data import DistributedSampler
    from sam2_video.data.synthetic import SyntheticClipDataset
    ds = SyntheticClipDataset(7, 1, 64, 2, 2)
    idx = [list(iter(DistributedSampler(ds, num_replicas=2, rank=r, shuffle=True, seed=0))) for r in range(2)]
    assert not (set(idx[0]) & set(idx[1]) - {idx[0][-1], idx[1][-1]})  # only the padding repeats
    assert set(idx[0]) | set(idx[1]) == set(range(7))


def test_arena_tail_ranks_follow_the_staged_backbone_backward():
    """the gradient arena ends with the parameters the staged backbone backward completes, in the
    order it completes them (SAM2Model._backbone_grad_rank): conv_s0 / conv_s1 and the neck (rank 0
    -- conv_s0 / s1 act on the backbone outputs, so their gradients are finished by phase 2, not
    phase 1), then the Hiera stages last to first, patch / position embedding with stage 1;
    grad_cuts are the rank boundaries"""
    from sam2_video.kernels.arena import ParamArena
    from sam2_video.model.sam2model import SAM2Model
    ALL = ["image_encoder", "memory_attention", "memory_encoder", "mask_decoder", "prompt_encoder"]
    m = SAM2Model(None, "tiny@128", trainable_modules=ALL)
    rank = m._backbone_grad_rank()
    never = set(m.never_grad_parameter_names())
    named = list(m.named_parameters())
    grad_names = [n for n, p in named if p.requires_grad and n not in never]
    a = ParamArena(named, grad_names, torch.float32, torch.device("cpu"), tail_rank=rank)
    nst = len(m.image_encoder.trunk.stage_ends)
    assert len(a.grad_cuts) == nst + 2 and a.grad_cuts[0] == a.grad_split and a.grad_cuts[-1] == a.n_grad
    assert all(x <= y for x, y in zip(a.grad_cuts, a.grad_cuts[1:]))
    by_off = sorted((a.offsets[n], n) for n in a.grad_names)
    ranks = [rank(n) for _, n in by_off if a.offsets[n] >= a.grad_split]
    assert None not in ranks and ranks == sorted(ranks)
    assert all(rank(n) is None for _, n in by_off if a.offsets[n] < a.grad_split)
    assert rank("sam_mask_decoder.conv_s0.weight") == 0 and rank("image_encoder.neck.convs.0.conv.weight") == 0
    last_block = m.image_encoder.trunk.stage_ends[-1]
    assert rank(f"image_encoder.trunk.blocks.{last_block}.mlp.layers.0.weight") == 1
    assert rank("image_encoder.trunk.blocks.0.norm1.weight") == nst == rank("image_encoder.trunk.patch_embed.proj.weight")
    for r in range(nst + 1):  # each rank's parameters lie inside its cut range
        for _, n in by_off:
            if rank(n) == r:
                assert a.grad_cuts[r] <= a.offsets[n] < a.grad_cuts[r + 1], (n, r)
    assert rank("memory_attention.layers.0.linear1.weight") is None


def test_vfold_key_rope_fusion_eligibility():
    """host decision of the fused key-gradient RoPE (frametape._vfold_k_rope): only when the keys
    come from ONE linear-with-RoPE op used by this attention alone, with one full-width head, the
    same tables and period in every frame and one L-row block per object; nrot per frame is passed
    through (object-pointer keys stay unrotated); S2H_VFOLD_DK_ROPE=0 turns it off"""
    import collections

    from sam2_video.kernels import frametape as ft
    cos, sin = torch.zeros(1024, 128), torch.zeros(1024, 128)
    lks = [1028, 2060]
    ropes = [(cos, sin, 1028, 1024, 1024, 256, 256), (cos, sin, 2060, 2048, 1024, 256, 256)]
    prod = SimpleNamespace(kind="linear", fattrs={"rope": ropes})
    tape = SimpleNamespace(producer={7: prod}, nuse=collections.Counter({7: 1}))
    got = ft._vfold_k_rope(tape, 7, lks, 256)
    assert got is not None and got[0] is cos and got[1] is sin and got[2] == 1024 and got[3] == [1024, 2048]
    tape.nuse[7] = 2  # the keys feed a second consumer: its gradient would not be rotated
    assert ft._vfold_k_rope(tape, 7, lks, 256) is None
    tape.nuse[7] = 1
    assert ft._vfold_k_rope(tape, 7, [1028, 2061], 256) is None  # block length != frame keys
    bad = [ropes[0], (torch.zeros(1024, 128), sin) + ropes[1][2:]]  # another table object
    tape.producer[7] = SimpleNamespace(kind="linear", fattrs={"rope": bad})
    assert ft._vfold_k_rope(tape, 7, lks, 256) is None
    tape.producer[7] = SimpleNamespace(kind="linear", fattrs={"rope": [r[:5] + (128, 128) for r in ropes]})
    assert ft._vfold_k_rope(tape, 7, lks, 256) is None  # multi-head / partial rotation
    tape.producer[7] = SimpleNamespace(kind="add", fattrs={})
    assert ft._vfold_k_rope(tape, 7, lks, 256) is None
    tape.producer[7] = prod
    old = os.environ.get("S2H_VFOLD_DK_ROPE")
    os.environ["S2H_VFOLD_DK_ROPE"] = "0"
    try:
        assert ft._vfold_k_rope(tape, 7, lks, 256) is None
    finally:
        if old is None:
            del os.environ["S2H_VFOLD_DK_ROPE"]
        else:
            os.environ["S2H_VFOLD_DK_ROPE"] = old
