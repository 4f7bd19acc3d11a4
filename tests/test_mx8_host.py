"""MX-fp8 oracle (oracle/mx8_oracle.py) pinned on the CPU: the e4m3 encoder against torch's
float -> float8_e4m3fn conversion (round to nearest even, OCP encoding), the block-scale rule
of OCP MX v1.0, and the scale-word layout round trip.  No GPU."""
import numpy as np
import torch

from oracle import mx8_oracle as mx


def test_e4m3_encoder_matches_torch():
    vals = mx.E4M3_VALUES[:0x7F]
    mids = 0.5 * (vals[:-1] + vals[1:])
    x = np.concatenate([vals, mids, np.nextafter(mids, 0), np.nextafter(mids, 1e9),
                        np.random.default_rng(0).uniform(-448, 448, 20000)]).astype(np.float32)
    x = np.concatenate([x, -x])
    want = torch.from_numpy(x).to(torch.float8_e4m3fn).view(torch.uint8).numpy()
    got = mx.encode_e4m3(x)
    nz = x != 0
    assert np.array_equal(got[nz], want[nz])
    # saturation (torch would give NaN above 464; the MX spec clamps)
    assert mx.encode_e4m3(np.array([500.0, -1e6]))[0] == 0x7E
    assert mx.encode_e4m3(np.array([500.0, -1e6]))[1] == 0xFE


def test_block_scale_rule():
    rng = np.random.default_rng(1)
    x = (rng.standard_normal((5, 200)) * np.ldexp(1.0, rng.integers(-20, 20, (5, 1)))).astype(np.float32)
    x[2, 32:64] = 0.0  # an all-zero block
    q, e8 = mx.quantize(x)
    assert q.shape == (5, 256) and e8.shape == (5, 8)
    assert np.all(q[:, 200:] == 0)
    amax = np.abs(np.pad(x, ((0, 0), (0, 56)))).reshape(5, 8, 32).max(2)
    for r in range(5):
        for b in range(8):
            if amax[r, b] == 0:
                assert e8[r, b] == 127
            else:
                # largest element lands in [256, 512) before the 448 clamp
                assert 256 <= amax[r, b] / 2.0 ** (int(e8[r, b]) - 127) < 512
    deq = mx.dequantize(q, e8)[:, :200]
    rel = np.abs(deq - x) / np.maximum(np.repeat(amax, 32, 1)[:, :200], 1e-30)
    assert rel.max() <= 2.0 ** -4 * 2  # half an e4m3 ulp of the block max (<= 2^-4), with the clamp edge


def test_scale_words_round_trip():
    e8 = np.random.default_rng(2).integers(0, 255, (7, 12)).astype(np.uint8)
    w = mx.scale_words(e8)
    assert w.shape == (3, 7) and w.dtype == np.int32
    assert np.array_equal(mx.words_to_e8(w, 7), e8)
    assert (w.view(np.uint32)[1, 4] >> 8) & 0xFF == e8[4, 5]
