"""SNAC oracle structure + the algebra the HIP kernels rely on (CPU only).

* window lengths: N frames -> 2048 N samples; NoiseBlock lengths 32N/256N/1024N/2048N;
* the polyphase ConvTranspose1d decomposition packed by mx_snac_finalize (capi.hip):
  out[co][s t + ph] = sum_ci W[ci][co][rm] x[ci][t+q] + W[ci][co][rm+s] x[ci][t+q-1],
  q = (ph + ceil(s/2)) // s, rm = (ph + ceil(s/2)) % s — equals F.conv_transpose1d;
* weight-norm folding used by the checkpoint loader.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from oracle import snac_ref
from project_morpheus_amd.weights import fold_weight_norm, snac_shapes, synthetic_snac_weights


@pytest.mark.parametrize("n", [1, 4, 7])
def test_window_lengths(n):
    w = synthetic_snac_weights()
    a = snac_ref.decode(w, [5] * n, [6] * (2 * n), [7] * (4 * n))
    assert a.shape == (1, 1, 2048 * n)
    assert snac_ref.noise_lengths(n) == [32 * n, 256 * n, 1024 * n, 2048 * n]
    assert sum(snac_ref.noise_lengths(n)) == 3360 * n
    assert float(a.abs().max()) <= 1.0


@pytest.mark.parametrize("s,cin,cout,T", [(8, 16, 8, 5), (4, 8, 4, 9), (2, 8, 8, 7), (8, 4, 4, 1)])
def test_polyphase_convtranspose(s, cin, cout, T):
    g = torch.Generator().manual_seed(s * 100 + T)
    W = torch.randn(cin, cout, 2 * s, generator=g, dtype=torch.float64)
    x = torch.randn(1, cin, T, generator=g, dtype=torch.float64)
    want = F.conv_transpose1d(x, W, stride=s, padding=math.ceil(s / 2), output_padding=s % 2)
    pad = (s + 1) // 2
    out = torch.zeros(1, cout, s * T, dtype=torch.float64)
    for ph in range(s):
        q, rm = (ph + pad) // s, (ph + pad) % s
        A = torch.cat([W[:, :, rm].T, W[:, :, rm + s].T], dim=1)          # [cout, 2 cin]
        for t in range(T):
            xs = []
            for d in (q, q - 1):
                i = t + d
                xs.append(x[0, :, i] if 0 <= i < T else torch.zeros(cin, dtype=torch.float64))
            out[0, :, s * t + ph] = A @ torch.cat(xs)
    assert want.shape == out.shape
    assert torch.allclose(out, want, atol=1e-12)


def test_weight_norm_fold_matches_torch():
    conv = torch.nn.utils.parametrizations.weight_norm(torch.nn.Conv1d(6, 4, 7))
    g = conv.parametrizations.weight.original0.detach()
    v = conv.parametrizations.weight.original1.detach()
    assert torch.allclose(fold_weight_norm(g, v), conv.weight.detach(), atol=1e-6)
    ct = torch.nn.utils.parametrizations.weight_norm(torch.nn.ConvTranspose1d(6, 4, 16, 8))
    g = ct.parametrizations.weight.original0.detach()
    v = ct.parametrizations.weight.original1.detach()
    assert torch.allclose(fold_weight_norm(g, v), ct.weight.detach(), atol=1e-6)


def test_synthetic_shapes_cover_decoder():
    w = synthetic_snac_weights()
    assert set(w) == set(snac_shapes())
    n = sum(v.numel() for k, v in w.items())
    assert 12.5e6 < n < 14.5e6   # ~13 M decoder + quantizer params


def _decode_window(w, codes, n, noise):
    c0 = [codes[7 * f] for f in range(n)]
    c1 = [codes[7 * f + j] for f in range(n) for j in (1, 4)]
    c2 = [codes[7 * f + j] for f in range(n) for j in (2, 3, 5, 6)]
    return snac_ref.decode(w, c0, c1, c2, noise=noise).reshape(-1)


def test_kept_slice_depends_on_the_first_five_frames_only():
    """schedule.frames_for_slice: the samples speechpipe keeps of a 49-code window, [2048, 4096)
    (speechpipe.py:122), do not depend on frames 5 and 6 (bit-identical when they change), so the
    serving path decodes the window's first 5 frames; with the NoiseBlock noise keyed by
    position (window_noise, the device's gauss_at) that decode gives the kept samples within
    fp32 summation order of the full one.  Frame 4 does reach them (the bound is tight)."""
    import numpy as np

    from project_morpheus_amd.schedule import frames_for_slice
    w = synthetic_snac_weights(seed=3)
    rng = np.random.default_rng(0)
    codes = [int(v) for v in rng.integers(0, 4096, 49)]
    full = _decode_window(w, codes, 7, snac_ref.window_noise(11, 7))[2048:4096]
    late = list(codes)
    for k in range(35, 49):
        late[k] = int(rng.integers(0, 4096))
    assert torch.equal(_decode_window(w, late, 7, snac_ref.window_noise(11, 7))[2048:4096], full)
    early = list(codes)
    for k in range(28, 35):
        early[k] = int(rng.integers(0, 4096))
    assert float((_decode_window(w, early, 7, snac_ref.window_noise(11, 7))[2048:4096] - full)
                 .abs().max()) > 1e-3
    n = frames_for_slice(7, 4096)
    assert n == 5 and frames_for_slice(4, 4096) == 4 and frames_for_slice(1, 2048) == 1
    short = _decode_window(w, codes[: 7 * n], n, snac_ref.window_noise(11, n))[2048:4096]
    d = (short - full).abs()
    assert float(d.max()) < 2e-5 and float(d.pow(2).mean().sqrt()) < 5e-6
