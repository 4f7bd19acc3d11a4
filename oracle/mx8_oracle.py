"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the MX-fp8 format the config-5 path computes
in (OCP Microscaling Formats v1.0, MXFP8 E4M3), the checker for s2h_mx8_quant / s2h_gemm_mx8.
Only tests/ may import this file; the product never does.

The reference has no fp8 path (it trains in fp32 or fp16/bf16 autocast, trainer.py:256-289
under Lightning `precision`), so there is no reference output to pin this against: parity
unpinned with respect to the reference.  It is pinned instead to (1) torch's own float ->
float8_e4m3fn conversion (round to nearest even, OCP encoding) in tests/test_mx8_host.py and
(2) the hardware conversion / MFMA lane maps checked by tools/probe_mx.hip.

Format restated (OCP MX v1.0 section 6.3): a block of 32 elements shares the E8M0 scale
X = 2^(floor(log2(max|v|)) - emax), emax = 8 for E4M3; elements are v / X rounded to
nearest-even E4M3 with saturation at +-448 (the spec's clamp); an all-zero block takes
X = 2^0 (any scale is exact for it).  E8M0 is stored as the biased exponent byte (127 = 2^0).
"""
from __future__ import annotations

import numpy as np

EMAX_E4M3 = 8
MAX_E4M3 = 448.0


def _e4m3_table():
    """float value of every e4m3fn code 0..255 (0x7f / 0xff NaN)"""
    v = np.zeros(256, dtype=np.float64)
    for c in range(256):
        s, e, m = c >> 7, (c >> 3) & 15, c & 7
        x = m / 8.0 * 2.0 ** -6 if e == 0 else (1 + m / 8.0) * 2.0 ** (e - 7)
        v[c] = -x if s else x
    v[0x7F] = v[0xFF] = np.nan
    return v


E4M3_VALUES = _e4m3_table()


def encode_e4m3(x):
    """float array -> e4m3fn codes, round to nearest even, saturating at +-448 (|x| finite);
    negative zero and negative underflow encode as 0x80"""
    x = np.asarray(x, dtype=np.float64)
    a = np.minimum(np.abs(x), MAX_E4M3)
    pos = E4M3_VALUES[:0x7F]  # 0 .. 448, increasing
    hi = np.clip(np.searchsorted(pos, a, side="left"), 0, 0x7E)  # first code with value >= a
    lo = np.maximum(hi - 1, 0)
    dlo, dhi = a - pos[lo], pos[hi] - a
    pick_hi = (dhi < dlo) | ((dhi == dlo) & (hi % 2 == 0))  # ties to the even code (even mantissa)
    code = np.where(pick_hi, hi, lo).astype(np.uint8)
    code = np.where(a == pos[hi], hi, code).astype(np.uint8)
    return np.where(np.signbit(x), code | 0x80, code).astype(np.uint8)  # -0 / underflow keep the sign (as v_cvt_pk_fp8_f32)


def _floor_log2(a):
    m, e = np.frexp(a)  # a = m * 2^e, m in [0.5, 1)
    return e - 1


def quantize(x, k=None):
    """rows of x [rows, K] (float32 values, e.g. bf16 inputs) -> (q [rows, Kp] uint8,
    e8 [rows, Kp / 32] uint8 biased exponents), Kp = K rounded up to 128, zero padded"""
    x = np.asarray(x, dtype=np.float32)
    rows, K = x.shape
    kp = (K + 127) // 128 * 128
    xp = np.zeros((rows, kp), dtype=np.float32)
    xp[:, :K] = x
    blk = xp.reshape(rows, kp // 32, 32).astype(np.float64)
    amax = np.abs(blk).max(axis=2)
    e8 = np.where(amax > 0, np.clip(_floor_log2(np.where(amax > 0, amax, 1.0)) - EMAX_E4M3 + 127, 0, 254), 127)
    scaled = blk / np.ldexp(1.0, (e8 - 127).astype(np.int64))[:, :, None]
    q = encode_e4m3(scaled).reshape(rows, kp)
    return q, e8.astype(np.uint8)


def scale_words(e8):
    """[rows, Kp/32] biased exponents -> the kernel's [Kp/128, rows] int32 words (byte b of word
    (kt, r) = block 4kt + b of row r)"""
    rows, nb = e8.shape
    e = e8.astype(np.uint32).reshape(rows, nb // 4, 4)
    w = e[:, :, 0] | (e[:, :, 1] << 8) | (e[:, :, 2] << 16) | (e[:, :, 3] << 24)
    return np.ascontiguousarray(w.T).view(np.int32)


def words_to_e8(words, rows):
    """inverse of scale_words: [Kp/128, >= rows] int32 -> [rows, Kp/32] uint8"""
    w = np.asarray(words).view(np.uint32)[:, :rows].T  # [rows, Kp/128]
    b = np.stack([(w >> (8 * i)) & 0xFF for i in range(4)], axis=2)
    return b.reshape(rows, -1).astype(np.uint8)


def dequantize(q, e8):
    """(q [rows, Kp], e8 [rows, Kp/32]) -> float64 values [rows, Kp]"""
    rows, kp = q.shape
    v = E4M3_VALUES[q].reshape(rows, kp // 32, 32) * np.ldexp(1.0, e8.astype(np.int64) - 127)[:, :, None]
    return v.reshape(rows, kp)
