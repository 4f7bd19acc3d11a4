"""The native prompt stage (csrc/prompts_host.cpp, host CPU code in libsam2hip.so) against the
oracle's scipy restatement of the reference's cv2 calls (masks.py:13-50, prompts.py:13-97):
object masks, their order and categories bit-exact, clicks and boxes exact, on random blob masks
and the edge cases (empty categories, borders, one-pixel specks, 1-row images, many objects)."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))

import sam2_oracle as O  # noqa: E402
from sam2_video.utils import masks as M  # noqa: E402
from sam2_video.utils import prompts as PR  # noqa: E402


def _blobs(rng, N, H, W, density):
    """category masks of random rectangles / discs, some touching the borders"""
    m = np.zeros((N, H, W), bool)
    yy, xx = np.mgrid[:H, :W]
    for c in range(N):
        for _ in range(rng.integers(0, 6)):
            if rng.random() < 0.5:
                y0, x0 = rng.integers(-4, H), rng.integers(-4, W)
                m[c, max(0, y0):y0 + rng.integers(1, H // 3 + 2), max(0, x0):x0 + rng.integers(1, W // 3 + 2)] = True
            else:
                cy, cx, r = rng.integers(0, H), rng.integers(0, W), rng.integers(1, max(2, H // 5))
                m[c] |= (yy - cy) ** 2 + (xx - cx) ** 2 <= r * r
        m[c] |= rng.random((H, W)) < density  # specks the opening removes (and some it joins)
    return m


CASES = [(3, 64, 64, 0.0), (4, 96, 80, 0.02), (2, 33, 47, 0.3), (5, 128, 128, 0.01), (1, 7, 9, 0.5), (2, 1, 40, 0.6),
         (13, 256, 256, 0.005)]


@pytest.mark.parametrize("N,H,W,density", CASES)
def test_objects_match_oracle(N, H, W, density):
    rng = np.random.default_rng(N * 1000 + H)
    cm = torch.from_numpy(_blobs(rng, N, H, W, density)).unsqueeze(1)
    want_objs, want_cats = [], []
    for c in range(N):
        if cm[c, 0].any():
            comps = O.opened_components(cm[c, 0].numpy())
            want_objs += comps
            want_cats += [c] * len(comps)
    cats, st, lab = M.object_moments(cm[:, 0], want_labels=True)
    assert cats.tolist() == want_cats
    if not want_objs:
        with pytest.raises(ValueError):
            M.cat_to_obj_mask(cm)
        return
    objs, obj_to_cat, n = M.cat_to_obj_mask(cm)
    assert n == N and obj_to_cat == want_cats
    assert torch.equal(objs[:, 0], torch.from_numpy(np.stack(want_objs)))
    # moments of each object = the oracle's click / box on its mask
    pts, lbl = O.point_prompt(objs)
    cp, cl = PR.center_prompt_from_moments(st)
    assert torch.equal(cp, pts) and torch.equal(cl, lbl)
    bp, bl = O.box_prompt(objs)
    mp, ml = PR.box_prompt_from_moments(st)
    assert torch.equal(mp, bp) and torch.equal(ml, bl)
    assert st[:, 0].tolist() == [int(o.sum()) for o in want_objs]


def test_find_connected_components_single_mask():
    m = torch.zeros(40, 40, dtype=torch.bool)
    m[2:10, 2:10] = True
    m[20:30, 5:35] = True
    m[35, 35] = True  # removed by the opening
    comps = M.find_connected_components(m)
    want = O.opened_components(m.numpy())
    assert len(comps) == len(want) == 2
    for a, b in zip(comps, want):
        assert torch.equal(a, torch.from_numpy(b))


def test_generate_prompts_match_oracle_with_random_clicks():
    rng = np.random.default_rng(7)
    cm = torch.from_numpy(_blobs(rng, 4, 64, 64, 0.0)).unsqueeze(1)
    objs, _, _ = M.cat_to_obj_mask(cm)
    p, lab = PR.generate_point_prompt(objs, 1, 0, True)
    po, lo = O.point_prompt(objs)
    assert torch.equal(p, po) and torch.equal(lab, lo)
    b, bl = PR.generate_box_prompt(objs)
    bo, blo = O.box_prompt(objs)
    assert torch.equal(b, bo) and torch.equal(bl, blo)
    # random positives / negatives land on the right pixels
    torch.manual_seed(0)
    p, lab = PR.generate_point_prompt(objs, 3, 2, True)
    assert p.shape == (objs.shape[0], 5, 2) and lab.tolist() == [[1, 1, 1, 0, 0]] * objs.shape[0]
    for k in range(objs.shape[0]):
        m = objs[k, 0] > 0
        for j in range(1, 5):
            x, y = int(p[k, j, 0]), int(p[k, j, 1])
            assert bool(m[y, x]) == (j < 3)


def test_empty_and_error_paths():
    with pytest.raises(ValueError):
        PR.generate_point_prompt(torch.zeros(1, 1, 8, 8), 1, 0, True)
    with pytest.raises(ValueError):
        PR.generate_box_prompt(torch.zeros(1, 1, 8, 8))
    cats, st, lab = M.object_moments(np.zeros((2, 8, 8), bool))
    assert len(cats) == 0 and st.shape == (0, 7) and lab is None


def test_many_objects_grow_the_buffer():
    """> the first capacity (64) objects: the call reports the count and is repeated"""
    m = np.zeros((1, 120, 120), bool)
    for i in range(10):
        for j in range(10):
            m[0, 12 * i:12 * i + 7, 12 * j:12 * j + 7] = True
    cats, st, _ = M.object_moments(m)
    want = O.opened_components(m[0])
    assert len(cats) == 100 and st[:, 0].tolist() == [int(o.sum()) for o in want]
    # raster order of first pixels
    first = st[:, 3] * 120 + st[:, 5]
    assert (np.diff(first) > 0).all()
