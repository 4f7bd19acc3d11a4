"""Host-side pieces of the video predictor (no GPU): frame loading as upstream's
load_video_frames does it, hole filling / sprinkle removal, the upstream import paths and
config names."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sam2-video-training_amd"))


def test_load_frames_from_jpeg_folder(tmp_path):
    from PIL import Image
    from sam2_video.predictor import _load_frames
    rng = np.random.default_rng(0)
    frames = (rng.random((3, 30, 50, 3)) * 255).astype(np.uint8)
    for i, f in enumerate(frames):  # numeric order, not lexical: 10.jpg after 2.jpg
        Image.fromarray(f).save(tmp_path / f"{[0, 2, 10][i]}.jpg", quality=100)
    x, H, W = _load_frames(str(tmp_path), 64)
    assert x.shape == (3, 3, 64, 64) and (H, W) == (30, 50)
    y, _, _ = _load_frames(frames, 64)  # uint8 array path (no JPEG round trip)
    ref = np.asarray(Image.fromarray(frames[1]).resize((64, 64))).astype(np.float32) / 255.0
    mean, std = np.array([0.485, 0.456, 0.406]), np.array([0.229, 0.224, 0.225])
    np.testing.assert_allclose(y[1].permute(1, 2, 0).numpy(), (ref - mean) / std, atol=1e-5)


def test_fill_holes_and_remove_sprinkles():
    from sam2_video.predictor import fill_holes_in_mask_scores
    m = -torch.ones(1, 1, 20, 20)
    m[0, 0, 2:12, 2:12] = 3.0          # object (area 100)
    m[0, 0, 5:7, 5:7] = -2.0           # hole of area 4 -> 0.1
    m[0, 0, 15, 15] = 5.0              # sprinkle of area 1 -> -0.1
    m[0, 0, 9:12, 14:18] = -3.0        # already background
    out = fill_holes_in_mask_scores(m, 8)
    assert torch.all(out[0, 0, 5:7, 5:7] == 0.1)
    assert out[0, 0, 15, 15] == -0.1
    assert out[0, 0, 3, 3] == 3.0 and out[0, 0, 0, 0] == -1.0
    # a hole larger than max_area stays
    m2 = m.clone()
    m2[0, 0, 4:8, 4:8] = -2.0
    assert torch.all(fill_holes_in_mask_scores(m2, 8)[0, 0, 4:8, 4:8] == -2.0)
    # 8-connectivity: diagonal pixels form one component of area 2
    m3 = -torch.ones(1, 1, 6, 6)
    m3[0, 0, 1, 1] = m3[0, 0, 2, 2] = 1.0
    assert torch.all(fill_holes_in_mask_scores(m3, 1)[0, 0, 1:3, 1:3].diagonal() == 1.0)


def test_upstream_import_paths_and_config_names():
    from sam2.build_sam import build_sam2_video_predictor
    from sam2.sam2_video_predictor import SAM2VideoPredictor
    from sam2_video.model.build import load_model_config
    from sam2_video.predictor import SAM2VideoPredictor as P
    assert SAM2VideoPredictor is P and callable(build_sam2_video_predictor)
    cfg = load_model_config("configs/sam2.1/sam2.1_hiera_b+.yaml")
    assert cfg["image_size"] == 1024 and cfg["image_encoder"]["trunk"]["embed_dim"] == 112
    assert load_model_config("configs/sam2.1/sam2.1_hiera_l.yaml", 512)["image_encoder"]["trunk"]["embed_dim"] == 144
