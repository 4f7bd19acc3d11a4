"""COCO run-length-encoded masks without pycocotools (not installed here).

The reference decodes annotation masks with pycocotools' `mask.decode` (dataset.py:123-137).  This
restates the published COCO RLE format it reads:
  * a mask [h, w] is flattened column-major (Fortran order) and described by alternating run
    lengths of 0s and 1s, starting with 0s;
  * the compressed string form (`counts` as str) stores each run length as a little-endian
    sequence of 5-bit groups, one character (group + 48) per group, bit 0x20 = "more groups
    follow", bit 0x10 of the last group = sign; from the 4th count on the value is the
    difference to the count two places earlier.
Host-side numpy, once per annotation (the reference caches decoded masks per image too).
"""
from __future__ import annotations

import ast
from typing import Dict, List, Union

import numpy as np


def counts_from_string(s: str) -> List[int]:
    cnts: List[int] = []
    p, n = 0, len(s)
    while p < n:
        x, k, more = 0, 0, 1
        while more:
            c = ord(s[p]) - 48
            x |= (c & 0x1F) << (5 * k)
            more = c & 0x20
            p += 1
            k += 1
            if not more and (c & 0x10):
                x |= -1 << (5 * k)
        if len(cnts) > 2:
            x += cnts[-2]
        cnts.append(x)
    return cnts


def counts_to_string(cnts: List[int]) -> str:
    out = []
    for i, x in enumerate(cnts):
        x = int(x)
        if i > 2:
            x -= int(cnts[i - 2])
        more = 1
        while more:
            c = x & 0x1F
            x >>= 5
            more = (x != -1) if (c & 0x10) else (x != 0)
            if more:
                c |= 0x20
            out.append(chr(c + 48))
    return "".join(out)


def _as_rle(rle: Union[Dict, str]) -> Dict:
    if isinstance(rle, str):  # some exports store the dict's repr (data/endovis18.json)
        rle = ast.literal_eval(rle)
    if not isinstance(rle, dict) or "counts" not in rle or "size" not in rle:
        raise ValueError("expected an RLE dict {'size': [h, w], 'counts': ...} (polygons are not supported)")
    return rle


def decode(rle: Union[Dict, str]) -> np.ndarray:
    """RLE (compressed or uncompressed counts) -> uint8 mask [h, w]"""
    rle = _as_rle(rle)
    h, w = (int(v) for v in rle["size"])
    cnts = rle["counts"]
    if isinstance(cnts, bytes):
        cnts = cnts.decode("ascii")
    if isinstance(cnts, str):
        cnts = counts_from_string(cnts)
    cnts = np.asarray(cnts, dtype=np.int64)
    if cnts.sum() != h * w:
        raise ValueError(f"RLE counts cover {int(cnts.sum())} pixels, mask has {h * w}")
    vals = np.zeros(len(cnts), dtype=np.uint8)
    vals[1::2] = 1
    flat = np.repeat(vals, cnts)
    return flat.reshape(w, h).T.copy()  # column-major


def encode(mask: np.ndarray) -> Dict:
    """uint8/bool mask [h, w] -> compressed RLE dict"""
    m = np.asarray(mask).astype(bool)
    h, w = m.shape
    flat = m.T.reshape(-1)
    change = np.flatnonzero(flat[1:] != flat[:-1]) + 1
    bounds = np.concatenate([[0], change, [flat.size]])
    runs = np.diff(bounds).tolist()
    if flat.size and flat[0]:
        runs = [0] + runs
    return {"size": [h, w], "counts": counts_to_string(runs)}


def area(rle) -> int:
    return int(decode(rle).sum())


def to_bbox(rle) -> List[float]:
    """[x, y, w, h] of the mask's nonzero pixels (pycocotools toBbox semantics)"""
    m = decode(rle)
    ys, xs = np.nonzero(m)
    if ys.size == 0:
        return [0.0, 0.0, 0.0, 0.0]
    return [float(xs.min()), float(ys.min()), float(xs.max() - xs.min() + 1), float(ys.max() - ys.min() + 1)]
