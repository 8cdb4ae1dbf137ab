"""CPU checks of the sampling oracle (oracle/sampling_ref.py): Philox known answer, the
nucleus definition against brute force, and the draw's distribution."""
import numpy as np

from oracle import sampling_ref as S


def test_philox_known_answer():
    # Random123 kat_vectors: philox4x32-10, counter 0, key 0 -> 6627e8d5 e169c58d ...
    assert int(S.philox_x0(np.array([0]), 0, 0)[0]) == 0x6627E8D5


def _brute_keep(e, f, thr):
    return np.array([int(f[e > e[i]].sum()) < thr and f[i] > 0 for i in range(len(e))])


def test_nucleus_matches_brute_force():
    rng = np.random.default_rng(0)
    for trial in range(40):
        n = int(rng.integers(2, 300))
        lg = rng.normal(0, float(rng.choice([0.1, 1, 5])), n).astype(np.float32)
        if trial % 4 == 0:  # ties
            lg = np.round(lg, 1)
        t = float(rng.choice([0.3, 0.6, 1.0, 1.7]))
        p = float(rng.choice([0.05, 0.5, 0.9, 0.999, 1.0]))
        e, kept, f, thr = S.nucleus(lg, t, p)
        np.testing.assert_array_equal(kept, _brute_keep(e, f, thr))
        assert kept[np.argmax(lg)]


def test_draw_distribution():
    lg = np.log(np.array([0.5, 0.25, 0.125, 0.0625, 0.0625], dtype=np.float32))
    # T = 1, top_p 0.8: nucleus {0, 1, 2} (mass above id 2 = 0.75 < 0.8), renormalised
    counts = np.zeros(5)
    for pos in range(6000):
        counts[S.sample(lg, 1.0, 0.8, 7, pos)] += 1
    freq = counts / counts.sum()
    np.testing.assert_allclose(freq[:3], np.array([4, 2, 1]) / 7, atol=0.02)
    assert counts[3:].sum() == 0


def test_greedy_is_argmax():
    lg = np.array([0.1, 3.0, 3.0, -1.0], dtype=np.float32)
    assert S.sample(lg, 0.0, 0.9, 1, 5) == 1
