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
    # the model section builds the module tree (weights: deterministic synthetic, the checkpoint
    # path does not exist here); the reference's own sam2/sam2.1_hiera_t.yaml is image_size 384
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
