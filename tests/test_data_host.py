"""Real-data input side on CPU: the COCO RLE codec against the reference's own
annotation files (tests/golden/rle_endovis18_sample.json: counts strings with the area / bbox
pycocotools wrote, extracted by oracle/gen_rle_golden.py), and the COCO clip dataset
(reference dataset.py:28-343) on a small COCO tree written here: keyframe filter, category
mapping, instance OR, resize / center-crop geometry, normalisation, clip stride, empty-mask
skip, and the data module's collated batches."""
import json
import os

import numpy as np
import pytest
import torch

from sam2_video.data import rle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rle_endovis18_sample.json")


def test_rle_decode_matches_reference_annotations():
    g = json.load(open(GOLD))
    assert len(g["original"]) >= 20 and len(g["opened"]) >= 20
    for a in g["original"]:  # string-repr dicts, area + bbox from the original conversion
        m = rle.decode(a["segmentation"])
        assert m.shape == (1024, 1280)
        assert int(m.sum()) == a["area"]
        assert rle.to_bbox(a["segmentation"]) == a["bbox"]
    for a in g["opened"]:  # dict RLEs re-encoded after the morphological opening
        m = rle.decode(a["segmentation"])
        assert int(m.sum()) == a["area"]
        assert rle.encode(m)["counts"] == a["segmentation"]["counts"]  # bit-exact re-encode


def test_rle_roundtrip_random_masks():
    rng = np.random.default_rng(0)
    for h, w in [(1, 1), (7, 5), (64, 48), (33, 100)]:
        for p in (0.0, 0.3, 1.0):
            m = (rng.random((h, w)) < p).astype(np.uint8)
            enc = rle.encode(m)
            assert np.array_equal(rle.decode(enc), m)
            assert rle.decode({"size": [h, w], "counts": rle.counts_from_string(enc["counts"])}).sum() == m.sum()


def _write_coco(root, H=90, W=120):
    from PIL import Image
    images, anns = [], []
    cats = [{"id": 7, "name": "b"}, {"id": 3, "name": "a"}]  # unsorted ids: contiguous by sorted id
    iid = 0
    truth = {}
    for v in range(2):
        for k in range(5):
            color = (10 * k + 40 * v, 100, 200 - 10 * k)
            path = os.path.join(root, f"v{v}_{k}.png")
            Image.fromarray(np.full((H, W, 3), color, np.uint8)).save(path)
            images.append({"id": iid, "path": path, "file_name": os.path.basename(path), "video_id": f"vid{v}",
                           "order_in_video": 4 - k, "is_det_keyframe": not (v == 1 and k == 2), "height": H,
                           "width": W})
            m = np.zeros((H, W), np.uint8)
            if not (v == 0 and k == 3):  # an empty-mask image
                m[10 + k:40 + k, 20:70] = 1
                m2 = np.zeros((H, W), np.uint8)
                m2[50:80, 90 - k:110] = 1
                anns.append({"id": len(anns), "image_id": iid, "category_id": 3, "segmentation": rle.encode(m)})
                anns.append({"id": len(anns), "image_id": iid, "category_id": 3, "segmentation": rle.encode(m2)})
                anns.append({"id": len(anns), "image_id": iid, "category_id": 7,
                             "segmentation": str(rle.encode(m2))})  # string-repr form
                truth[iid] = (m | m2, m2, color)
            iid += 1
    path = os.path.join(root, "ann.json")
    json.dump({"images": images, "annotations": anns, "categories": cats}, open(path, "w"))
    return path, truth


def test_coco_clip_dataset(tmp_path):
    from sam2_video.data.dataset import COCODataset, COCOImageDataset, IMAGENET_MEAN, IMAGENET_STD
    path, truth = _write_coco(str(tmp_path))
    cfg = {"image_size": 64, "video_clip_length": 2, "stride": 2, "num_categories": 3, "train_path": path}
    ids = COCOImageDataset(cfg, path)
    assert len(ids) == 9 and ids.catid_to_idx == {3: 0, 7: 1} and ids.num_categories == 3
    # frames of a video sorted by order_in_video (written in reverse)
    assert [im["order_in_video"] for im in ids.video_to_images["vid0"]] == [0, 1, 2, 3, 4]
    it = ids[ids.image_id_to_idx[1]]
    # geometry: 90x120 -> short side 64 (64 x 85, nearest) -> center crop 64 x 64 (left 10)
    u, m2, color = truth[1]
    ys = (np.arange(64) * 90 / 64).astype(int)
    xs = ((np.arange(64) + 10) * 120 / 85).astype(int)
    exp = torch.from_numpy(u[np.ix_(ys, xs)] > 0)
    assert torch.equal(it["masks"][0], exp)
    assert torch.equal(it["masks"][1], torch.from_numpy(m2[np.ix_(ys, xs)] > 0))
    assert not it["masks"][2].any()
    want = (torch.tensor(color, dtype=torch.float32) / 255 - torch.tensor(IMAGENET_MEAN)) / torch.tensor(IMAGENET_STD)
    assert torch.allclose(it["image"].mean(dim=(1, 2)), want, atol=1e-5)
    # the empty-mask image (video 0, k = 3) is replaced by the next index
    e = ids.image_id_to_idx[3]
    assert torch.equal(ids[e]["masks"], ids[(e + 1) % len(ids)]["masks"])
    ds = COCODataset(cfg, path)
    # vid0: 5 frames -> starts 0, 2; vid1: 4 keyframes -> starts 0, 2
    assert len(ds) == 4
    clip = ds[1]
    assert clip["images"].shape == (2, 3, 64, 64) and clip["masks"].shape == (2, 3, 64, 64)


def test_data_module_reads_coco_when_present(tmp_path):
    from sam2_video.training.trainer import SAM2LightningDataModule
    path, _ = _write_coco(str(tmp_path))
    dm = SAM2LightningDataModule({"train_path": path, "val_path": path, "image_size": 32, "video_clip_length": 3,
                                  "stride": 1, "num_categories": 2, "batch_size": 1, "num_workers": 0})
    dm.setup("fit")
    b = next(iter(dm.train_dataloader()))
    assert tuple(b.img_batch.shape) == (3, 1, 3, 32, 32) and tuple(b.masks.shape) == (3, 2, 32, 32)
    assert b.masks.dtype == torch.bool
    with pytest.raises(FileNotFoundError):
        from sam2_video.data.dataset import COCODataset
        COCODataset({"image_size": 8, "video_clip_length": 1, "stride": 1}, str(tmp_path / "missing.json"))
