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


def _decode_cut(w, codes, n, noise, lo, hi, cut=None, poke=None):
    """The library's PCM-only decode (capi.hip snac_enqueue with snac_cut): input stage and
    block 0 whole, then blocks 1-3 and the output conv on block 0's positions [c0, c1) only,
    zero-padded at the cut edges, noise taken at the cut's origin; returns samples [lo, hi).
    cut=(0, 32 n) is the whole-window decode; poke=q adds 1 to block 0's Snake output at q."""
    from _snac_dispatch import snac_cut
    c0, c1 = cut if cut is not None else snac_cut(n, lo, hi)
    p = w
    cc = [codes[7 * f] for f in range(n)]
    c1c = [codes[7 * f + j] for f in range(n) for j in (1, 4)]
    c2c = [codes[7 * f + j] for f in range(n) for j in (2, 3, 5, 6)]
    with torch.no_grad():
        z = snac_ref.from_codes(p, [torch.as_tensor(c).reshape(1, -1) for c in (cc, c1c, c2c)])
        x = F.conv1d(z, p["in.dw.w"], p["in.dw.b"], padding=3, groups=z.shape[1])
        x = F.conv1d(x, p["in.pw.w"].unsqueeze(-1), p["in.pw.b"])
        org = 0
        for b, st in enumerate(snac_ref.RATES):
            x = snac_ref.snake(x, p[f"b{b}.alpha"])
            if b == 1:
                if poke is not None:
                    x = x.clone()
                    x[:, :, poke] += 1.0
                x, org = x[:, :, c0:c1], c0
            org *= st
            x = F.conv_transpose1d(x, p[f"b{b}.up.w"], p[f"b{b}.up.b"], stride=st,
                                   padding=math.ceil(st / 2), output_padding=st % 2)
            h = F.conv1d(x, p[f"b{b}.noise.w"].unsqueeze(-1))
            x = x + noise[b][:, :, org:org + x.shape[2]] * h
            for r, d in enumerate(snac_ref.DILATIONS):
                y = snac_ref.snake(x, p[f"b{b}.r{r}.alpha1"])
                y = F.conv1d(y, p[f"b{b}.r{r}.dw.w"], p[f"b{b}.r{r}.dw.b"], padding=3 * d,
                             dilation=d, groups=x.shape[1])
                y = snac_ref.snake(y, p[f"b{b}.r{r}.alpha2"])
                x = x + F.conv1d(y, p[f"b{b}.r{r}.pw.w"].unsqueeze(-1), p[f"b{b}.r{r}.pw.b"])
        x = snac_ref.snake(x, p["out.alpha"])
        x = torch.tanh(F.conv1d(x, p["out.conv.w"], p["out.conv.b"], padding=3)).reshape(-1)
    return x[lo - org:hi - org]


@pytest.mark.parametrize("n", [4, 5, 7])
def test_receptive_field_cut_keeps_the_kept_samples(n):
    """capi.hip snac_cut: a PCM-only call runs blocks 1-3 on the kept samples' receptive field
    in block 0's output (50 of 32 N positions for [2048, 4096), one of them margin on either
    side).  The cone is exact: a change to block 0's output just outside it leaves the kept
    samples of the whole-window decode bit-identical, one at its edge changes them; and the cut
    decode gives the kept samples within fp32 summation order (torch's conv algorithms vary
    with the length)."""
    import numpy as np

    from _snac_dispatch import serving_slice, snac_cut
    w = synthetic_snac_weights(seed=3)
    codes = [int(v) for v in np.random.default_rng(n).integers(0, 4096, 7 * n)]
    noise = snac_ref.window_noise(17, n)
    lo, hi = serving_slice(n)
    c0, c1 = snac_cut(n, lo, hi)
    assert (c0, c1) == (23, 73)
    whole = (0, 32 * n)
    full = _decode_cut(w, codes, n, noise, lo, hi, cut=whole)
    assert torch.equal(full, _decode_window(w, codes, n, noise)[lo:hi])
    for q in (c0, c1 - 1):  # the margin positions: outside the cone
        assert torch.equal(_decode_cut(w, codes, n, noise, lo, hi, cut=whole, poke=q), full)
    for q in (c0 + 1, c1 - 2):  # the cone's edges
        assert not torch.equal(_decode_cut(w, codes, n, noise, lo, hi, cut=whole, poke=q), full)
    d = (_decode_cut(w, codes, n, noise, lo, hi) - full).abs()
    assert float(d.max()) < 1e-5 and float(d.pow(2).mean().sqrt()) < 2e-6, float(d.max())
