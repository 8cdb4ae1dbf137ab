"""GPU parity of the SNAC 24 kHz decoder (HIP, fp32) vs the torch-fp32 CPU oracle.

Noise is passed explicitly (the reference's NoiseBlock draws torch.randn per call).
Tolerance (north_star): audio within 1e-4 RMS of the CPU path; PCM16 within 1 LSB
(truncation of x*32767 can flip on a last-ulp difference).
"""
import numpy as np
import pytest
import torch

from oracle import snac_ref
from project_morpheus_amd.weights import synthetic_snac_weights

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def snac_pair_32():
    from project_morpheus_amd.engine import SnacDecoder
    w = synthetic_snac_weights(seed=3)
    return w, SnacDecoder(w, device=0, max_frames=7, max_batch=32)


@pytest.fixture(scope="module")
def snac_pair():
    from project_morpheus_amd.engine import SnacDecoder
    w = synthetic_snac_weights(seed=3)
    return w, SnacDecoder(w, device=0, max_frames=7, max_batch=12)


def _noise(B, n, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(B, 3360 * n, generator=g)


def _split_noise(noise_row, n):
    out, off = [], 0
    for L in snac_ref.noise_lengths(n):
        out.append(noise_row[off:off + L].reshape(1, 1, L))
        off += L
    return out


@pytest.mark.parametrize("n_frames,B", [(1, 1), (4, 1), (7, 1), (7, 3), (2, 2), (1, 5), (4, 9),
                                        (7, 12), (5, 1), (5, 12)])
def test_snac_window_parity(snac_pair, n_frames, B):
    """(1, 5): the 2-wave conv-GEMM with a ragged column tile; (4, 9) and (7, 12): the
    block-tiled conv-GEMM below 32 windows, its last 128-column tile cut by the end of the
    batch and tiles holding columns of two windows (tests/_snac_dispatch.py keys); (5, *): the
    shape the serving path decodes a 7-frame window as (schedule.frames_for_slice)."""
    from _coverage import check_declared_snac
    check_declared_snac(n_frames, B)
    w, dec = snac_pair
    rng = np.random.default_rng(100 + n_frames + B)
    codes = rng.integers(0, 4096, size=(B, 7 * n_frames)).astype(np.int32)
    noise = _noise(B, n_frames, 7 + n_frames)
    pcm, audio = dec.decode(torch.from_numpy(codes).cuda(), noise=noise.cuda(), want_audio=True)
    torch.cuda.synchronize()
    audio = audio.cpu().numpy()
    pcm = pcm.cpu().numpy()
    for b in range(0, B, 1 if B <= 5 else 4):  # (every 4th window of the larger batches: CPU time)
        c = codes[b].tolist()
        c0 = [c[7 * f] for f in range(n_frames)]
        c1 = [c[7 * f + j] for f in range(n_frames) for j in (1, 4)]
        c2 = [c[7 * f + j] for f in range(n_frames) for j in (2, 3, 5, 6)]
        want = snac_ref.decode(w, c0, c1, c2, noise=_split_noise(noise[b], n_frames))
        want = want.reshape(-1).numpy()
        assert want.shape == audio[b].shape == (2048 * n_frames,)
        rms = float(np.sqrt(np.mean((audio[b] - want) ** 2)))
        assert rms < 1e-4, rms
        assert np.abs(audio[b] - want).max() < 1e-3
        ref_pcm = (want[2048:4096] * np.float32(32767)).astype(np.int16)
        assert pcm[b].shape == ref_pcm.shape
        if ref_pcm.size:  # a 1-frame window's [2048:4096] slice is empty (speechpipe.py:122)
            assert np.abs(pcm[b].astype(np.int32) - ref_pcm).max() <= 1


@pytest.mark.parametrize("n_frames,B", [(5, 1), (4, 5), (5, 12), (5, 32)])
def test_snac_cut_pcm_parity(snac_pair_32, n_frames, B):
    """PCM-only calls (the serving path) run blocks 1-3 on the kept samples' receptive field
    (capi.hip snac_cut, tests/test_oracle_snac.py): their PCM against the WHOLE-window oracle,
    within 1 LSB, for single windows, a 5-window batch (one-wave conv-GEMMs, ragged tiles) and
    12 / 32-window batches (the block-tiled conv-GEMM)."""
    from _coverage import check_declared_snac
    check_declared_snac(n_frames, B, cut=True)
    w, dec = snac_pair_32
    rng = np.random.default_rng(200 + n_frames + B)
    codes = rng.integers(0, 4096, size=(B, 7 * n_frames)).astype(np.int32)
    noise = _noise(B, n_frames, 9 + n_frames)
    pcm, audio = dec.decode(torch.from_numpy(codes).cuda(), noise=noise.cuda(), want_audio=False)
    torch.cuda.synchronize()
    assert audio is None
    pcm = pcm.cpu().numpy()
    hi = min(4096, 2048 * n_frames)
    for b in range(0, B, 1 if B <= 5 else 5):
        c = codes[b].tolist()
        c0 = [c[7 * f] for f in range(n_frames)]
        c1 = [c[7 * f + j] for f in range(n_frames) for j in (1, 4)]
        c2 = [c[7 * f + j] for f in range(n_frames) for j in (2, 3, 5, 6)]
        want = snac_ref.decode(w, c0, c1, c2, noise=_split_noise(noise[b], n_frames))
        ref_pcm = (want.reshape(-1).numpy()[2048:hi] * np.float32(32767)).astype(np.int16)
        assert pcm[b].shape == ref_pcm.shape
        assert np.abs(pcm[b].astype(np.int32) - ref_pcm).max() <= 1, b


def test_snac_audio_is_nontrivial(snac_pair):
    """Guard against a vacuous parity pass (all-zero or saturated audio)."""
    _, dec = snac_pair
    codes = torch.randint(0, 4096, (1, 49), dtype=torch.int32).cuda()
    _, audio = dec.decode(codes, want_audio=True, seed=5)
    a = audio.cpu().numpy()
    assert 0.01 < float(np.std(a)) < 0.99
    assert np.isfinite(a).all()


def test_device_noise_differs_per_seed(snac_pair):
    _, dec = snac_pair
    codes = torch.randint(0, 4096, (1, 28), dtype=torch.int32).cuda()
    _, a1 = dec.decode(codes, want_audio=True, seed=1)
    _, a2 = dec.decode(codes, want_audio=True, seed=2)
    _, a3 = dec.decode(codes, want_audio=True, seed=1)
    assert not torch.equal(a1, a2) and torch.equal(a1, a3)


def test_snac_batched_32_windows_matches_oracle(snac_pair):
    """The serving shape (B = 32 windows of 7 frames, the block-tiled conv-GEMM path)."""
    from project_morpheus_amd.engine import SnacDecoder

    from _coverage import check_declared_snac
    w, _ = snac_pair
    dec = SnacDecoder(w, device=0, max_frames=7, max_batch=32)
    n, B = 7, 32
    check_declared_snac(n, B)
    rng = np.random.default_rng(4242)
    codes = rng.integers(0, 4096, size=(B, 7 * n)).astype(np.int32)
    noise = _noise(B, n, 99)
    pcm, audio = dec.decode(torch.from_numpy(codes).cuda(), noise=noise.cuda(), want_audio=True)
    torch.cuda.synchronize()
    audio = audio.cpu().numpy()
    pcm = pcm.cpu().numpy()
    for b in range(0, B, 5):  # every 5th window against the oracle (CPU time)
        c = codes[b].tolist()
        c0 = [c[7 * f] for f in range(n)]
        c1 = [c[7 * f + j] for f in range(n) for j in (1, 4)]
        c2 = [c[7 * f + j] for f in range(n) for j in (2, 3, 5, 6)]
        want = snac_ref.decode(w, c0, c1, c2, _split_noise(noise[b], n)).reshape(-1).numpy()
        rms = float(np.sqrt(np.mean((audio[b] - want) ** 2)))
        assert rms < 1e-4, (b, rms)
        assert np.abs(audio[b] - want).max() < 1e-3
        ref_pcm = (want[2048:4096] * np.float32(32767)).astype(np.int16)
        assert np.abs(pcm[b].astype(np.int32) - ref_pcm).max() <= 1
