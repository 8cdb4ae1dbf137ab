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
