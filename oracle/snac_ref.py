"""Oracle: torch-fp32 CPU restatement of the SNAC 24 kHz decoder (TEST INFRASTRUCTURE).

The reference calls ``snac.SNAC.decode(codes)`` (speechpipe.py:43,118) from the third-party
package ``snac>=1.2.1,<2`` (requirements.txt:8), which is neither vendored under
/root/reference nor installed here.  This module restates the published snac 1.2.x
algorithm for the 24 kHz configuration (hubertsiuzdak/snac_24khz):

    {encoder_rates [2,4,8,8], latent 768, decoder_dim 1024, decoder_rates [8,8,4,2],
     vq_strides [4,2,1], codebook 4096 x 8, noise true, depthwise true, attn_window None}

  decode(codes) = Decoder(ResidualVectorQuantize.from_codes(codes))          (snac.py)
  from_codes: sum_i repeat_interleave(out_proj_i(codebook_i[codes_i]^T), stride_i)  (vq.py)
  Decoder: dwconv k7 (768) -> 1x1 768->1024 -> 4 x DecoderBlock -> Snake -> conv k7 ->1 -> tanh
  DecoderBlock(s): Snake -> ConvTranspose1d(k=2s, stride s, pad ceil(s/2), outpad s%2)
                   -> NoiseBlock(x + randn(B,1,T) * W x) -> ResidualUnit(d=1,3,9)
  ResidualUnit(d): x + conv1x1(Snake(dwconv_k7_dil_d(Snake(x))))            (layers.py)
  Snake(x) = x + (alpha + 1e-9).reciprocal() * sin(alpha * x)^2

Weight norm is folded before this module sees the weights (the product's loader
``project_morpheus_amd.weights.fold_weight_norm``).  The NoiseBlock's ``torch.randn`` is
replaced by an explicit ``noise`` input (list of 4 tensors [B,1,T_b]) so that GPU and CPU
can be compared; ``noise=None`` means zero noise.

PARITY UNPINNED against snac itself (package and weights absent): the
restatement is pinned only structurally (shapes, lengths, 2048 samples per frame).
"""
from __future__ import annotations

import math

import numpy as np
from typing import Dict, List, Optional, Sequence

import torch
import torch.nn.functional as F

RATES = (8, 8, 4, 2)
STRIDES = (4, 2, 1)
DILATIONS = (1, 3, 9)


def snake(x: torch.Tensor, alpha: torch.Tensor) -> torch.Tensor:
    a = alpha.reshape(1, -1, 1)
    return x + (a + 1e-9).reciprocal() * torch.sin(a * x).pow(2)


def from_codes(p: Dict[str, torch.Tensor], codes: Sequence[torch.Tensor]) -> torch.Tensor:
    z = 0.0
    for i, c in enumerate(codes):
        e = F.embedding(c.long(), p[f"q{i}.codebook"]).transpose(1, 2)        # [B,8,Ti]
        zi = F.conv1d(e, p[f"q{i}.out_proj.w"].unsqueeze(-1), p[f"q{i}.out_proj.b"])
        z = z + zi.repeat_interleave(STRIDES[i], dim=-1)
    return z


def decoder(p: Dict[str, torch.Tensor], z: torch.Tensor,
            noise: Optional[List[torch.Tensor]] = None) -> torch.Tensor:
    c = z.shape[1]
    x = F.conv1d(z, p["in.dw.w"], p["in.dw.b"], padding=3, groups=c)
    x = F.conv1d(x, p["in.pw.w"].unsqueeze(-1), p["in.pw.b"])
    for b, s in enumerate(RATES):
        x = snake(x, p[f"b{b}.alpha"])
        x = F.conv_transpose1d(x, p[f"b{b}.up.w"], p[f"b{b}.up.b"], stride=s,
                               padding=math.ceil(s / 2), output_padding=s % 2)
        h = F.conv1d(x, p[f"b{b}.noise.w"].unsqueeze(-1))
        n = noise[b] if noise is not None else torch.zeros(x.shape[0], 1, x.shape[2])
        x = x + n * h
        co = x.shape[1]
        for r, d in enumerate(DILATIONS):
            y = snake(x, p[f"b{b}.r{r}.alpha1"])
            y = F.conv1d(y, p[f"b{b}.r{r}.dw.w"], p[f"b{b}.r{r}.dw.b"], padding=3 * d,
                         dilation=d, groups=co)
            y = snake(y, p[f"b{b}.r{r}.alpha2"])
            y = F.conv1d(y, p[f"b{b}.r{r}.pw.w"].unsqueeze(-1), p[f"b{b}.r{r}.pw.b"])
            x = x + y
    x = snake(x, p["out.alpha"])
    x = F.conv1d(x, p["out.conv.w"], p["out.conv.b"], padding=3)
    return torch.tanh(x)


def decode(p: Dict[str, torch.Tensor], c0, c1, c2,
           noise: Optional[List[torch.Tensor]] = None) -> torch.Tensor:
    """codes (lists or int tensors, batch 1 or [B,N]) -> audio [B,1,2048N] fp32."""
    def t(c):
        c = torch.as_tensor(c, dtype=torch.int64)
        return c.reshape(1, -1) if c.dim() == 1 else c
    with torch.no_grad():
        z = from_codes(p, (t(c0), t(c1), t(c2)))
        return decoder(p, z, noise)


def noise_lengths(n_frames: int) -> List[int]:
    """Latent length 4N, then x8, x8, x4, x2 -> the four NoiseBlock lengths."""
    t = 4 * n_frames
    out = []
    for s in RATES:
        t *= s
        out.append(t)
    return out


_M64 = (1 << 64) - 1


def _mix64(z: np.ndarray) -> np.ndarray:
    z = (z + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(_M64)
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(_M64)
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & np.uint64(_M64)
    return z ^ (z >> np.uint64(31))


def device_noise(seed: int, j) -> np.ndarray:
    """Restatement of the GPU's NoiseBlock noise for a window seeded ``seed`` (csrc/
    snac_kernels.hip gauss_at): element key j = Box-Muller of mix64(seed ^ mix64(j)), float32.
    Lets the end-to-end tests compare audio with the noise ON (host libm vs device ulps)."""
    with np.errstate(over="ignore"):
        j = np.asarray(j, dtype=np.uint64)
        h = _mix64(np.uint64(seed) ^ _mix64(j))
    u1 = ((h >> np.uint64(40)).astype(np.float32) + np.float32(1.0)) * np.float32(1.0 / 16777217.0)
    u2 = ((h >> np.uint64(16)) & np.uint64(0xFFFFFF)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return (np.sqrt(np.float32(-2.0) * np.log(u1)) *
            np.cos(np.float32(6.283185307179586) * u2)).astype(np.float32)


def window_noise(seed: int, n_frames: int) -> List[torch.Tensor]:
    """The four NoiseBlock inputs [1,1,T_b] of one window drawn as the device draws them: the
    value at (NoiseBlock s, position t) is keyed j = s << 24 | t (gauss_at), so a window decoded
    with fewer frames shares the full window's noise at every common position."""
    out = []
    for s, t in enumerate(noise_lengths(n_frames)):
        j = (np.uint64(s) << np.uint64(24)) | np.arange(t, dtype=np.uint64)
        out.append(torch.from_numpy(device_noise(seed, j)).reshape(1, 1, t))
    return out
