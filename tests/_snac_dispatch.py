"""Which SNAC kernel instantiations one window-batch decode runs.

A restatement of the library's SNAC dispatch, so that the parity tests' coverage of the
kernels the bench runs can be checked on the CPU (tests/test_snac_coverage.py):

* ``capi.hip`` ``snac_enqueue`` (the 36 launches of one call, 37 with the receptive-field cut
  of a PCM-only call: embed, input depthwise conv and 1x1 conv, then per DecoderBlock the polyphase ConvTranspose, the NoiseBlock and three
  ResidualUnits, then the output stage) and ``pick_tiles`` (block-tiled kernel from
  ``snac_tiled_min_batch()`` = 8 windows when M % 64 == 0; otherwise 16 x NSUB column tiles,
  NSUB = 4 from 2,048 input steps, and WK K-splitting waves doubled while the launch stays
  <= 2,048 waves);
* ``snac_kernels.hip`` ``launch_conv_gemm`` (WK = 1 -> ``conv_gemm1_kernel<NSUB>``, else
  ``conv_gemm_kernel<WK, NSUB>``) and ``launch_dwconv`` (64-step tiles from B x T = 16,384).

A key is the rocprofv3 kernel name (without ``void mx::`` and the argument list) plus the
edge class the launch's geometry puts the kernel in, so that a test reaching the
instantiation only with full tiles does not stand in for a ragged launch of it:

* block-tiled conv-GEMM: ``cols%128`` (a 128-column tile is cut by the end of the batch) and
  ``straddle`` (Tin % 128 != 0: a tile holds columns of two windows);
* one-wave conv-GEMMs: ``ragged`` (Tin % (16 NSUB) != 0: the last column tile is partial);
* depthwise conv: ``ragged`` (T % tile != 0).
"""
from __future__ import annotations

K_RATES = (8, 8, 4, 2)
K_DIL = (1, 3, 9)
TILED_MIN_BATCH = 8


def pick_tiles(M, Cin, Tin, B, nseg, nphase, tiled_min=TILED_MIN_BATCH):
    tiled = M % 64 == 0 and B >= tiled_min
    nsub = 4 if Tin >= 2048 else 2
    tiles = (M // 32) * (-(-Tin // (16 * nsub))) * nphase * B
    ktot = nseg * Cin
    wk = 1
    while wk < 8 and tiles * wk * 2 <= 2048 and ktot % (128 * wk) == 0 and ktot // (2 * wk) >= 64:
        wk *= 2
    return tiled, wk, nsub


def conv_gemm_key(M, Cin, Tin, B, nseg, nphase):
    tiled, wk, nsub = pick_tiles(M, Cin, Tin, B, nseg, nphase)
    if tiled:
        flags = []
        if (B * Tin) % 128:
            flags.append("cols%128")
        if Tin % 128:
            flags.append("straddle")
        return "conv_gemm_tiled_kernel<1>" + (f" [{','.join(flags)}]" if flags else "")
    name = f"conv_gemm1_kernel<{nsub}>" if wk == 1 else f"conv_gemm_kernel<{wk}, {nsub}>"
    return name + (" [ragged]" if Tin % (16 * nsub) else "")


def dwconv_key(B, T):
    tile = 64 if B * T >= 16384 else 16
    return f"dwconv_kernel<{tile}>" + (" [ragged]" if T % tile else "")


def name_of(key):
    """The instantiation a key names (its rocprofv3 name without namespace / arguments)."""
    return key.split(" [")[0]


def snac_cut(n_frames, lo, hi):
    """capi.hip snac_cut: block 0's output positions [c0, c1) the kept samples [lo, hi) depend on
    (output conv 7 taps; per block three residual units of 7 taps at dilations 1, 3, 9 and the
    ConvTranspose1d(k = 2s, stride s, pad ceil(s / 2))), one position of margin."""
    T1 = 32 * n_frames
    if hi <= lo:
        return 0, T1
    L, H = lo - 3, hi + 3
    for b in (3, 2, 1):
        L -= 3 * sum(K_DIL)
        H += 3 * sum(K_DIL)
        st = K_RATES[b]
        pad = (st + 1) // 2
        L = -((-(L + pad - 2 * st + 1)) // st)
        H = (H - 1 + pad) // st + 1
    return max(0, L - 1), min(T1, H + 1)


def window_keys(n_frames, B, lo=None, hi=None):
    """Every kernel key of one mx_snac_decode call of B windows of n_frames frames; with the
    kept slice [lo, hi) of a PCM-only call (the serving path), blocks 1-3 run on its receptive
    field (capi.hip snac_cut)."""
    T = 4 * n_frames
    c0, c1 = (0, 32 * n_frames) if lo is None else snac_cut(n_frames, lo, hi)
    keys = {"snac_embed_kernel", dwconv_key(B, T), conv_gemm_key(1024, 768, T, B, 1, 1)}
    for b in range(4):
        cin = 1024 >> b
        cout, sr = cin // 2, K_RATES[b]
        if b == 1 and c1 - c0 < T:
            keys.add("snac_cut_kernel")
            T = c1 - c0
        keys.add(conv_gemm_key(cout, cin, T, B, 2, sr))   # polyphase ConvTranspose (all phases)
        T *= sr
        keys.add(conv_gemm_key(cout, cout, T, B, 1, 1))   # NoiseBlock
        for _ in K_DIL:
            keys.add(dwconv_key(B, T))
            keys.add(conv_gemm_key(cout, cout, T, B, 1, 1))  # ResidualUnit 1x1
    keys.add("snac_out_kernel")
    return keys


# The window shapes the serving path decodes (schedule.WindowScheduler: the first window is 7
# codes = 1 frame, then 28 or 49 codes = 4 or 7 frames, the end-of-stream flush 4 or 7; a
# 7-frame window is decoded as its first 5 frames, schedule.frames_for_slice), in batches of 1
# (engine.Synthesizer) up to the SNAC decoder's max_batch (bench.py: 32).
SERVING_FRAMES = (1, 4, 5)


SLICE_LO, SLICE_HI = 2048, 4096  # speechpipe.py:122


def serving_slice(n):
    """engine.SnacDecoder.decode's slice of an n-frame window (clamped to the window)."""
    hi = min(SLICE_HI, 2048 * n)
    return min(SLICE_LO, hi), hi


def envelope(max_batch=32, frames=SERVING_FRAMES, cut=True):
    """cut=False: the library before snac_cut (round 6), for the traces recorded with it."""
    keys = set()
    for n in frames:
        for B in range(1, max_batch + 1):
            keys |= window_keys(n, B, *serving_slice(n)) if cut else window_keys(n, B)
    return keys
