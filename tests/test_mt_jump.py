"""MT19937 jump-ahead polynomials (csrc/mt_jump.cpp): the characteristic polynomial and
x^J mod phi, checked on the CPU against numpy's own generator (no GPU)."""
import numpy as np
import pytest


def _bits(words):
    return np.unpackbits(np.asarray(words, dtype=np.uint64).view(np.uint8), bitorder="little")


def test_charpoly_degree_weight_and_recurrence():
    from ddm_amd._capi import lib
    phi = np.zeros(313, np.uint64)
    assert lib.ddm_mt_charpoly(phi.ctypes.data) == 0
    b = _bits(phi)
    deg = int(np.flatnonzero(b).max())
    assert deg == 19937 and int(b.sum()) == 135       # MT19937's characteristic polynomial
    rs = np.random.RandomState(5)
    x = (rs.randint(0, 2**32, 45000, dtype=np.uint64) & 1).astype(np.int64)
    co = b[:deg + 1].astype(np.int64)
    for n in range(0, 25000, 997):
        assert int(co @ x[n:n + deg + 1]) % 2 == 0


def _horner(key, poly_words):
    """g(T) * key on the CPU: the window recurrence x_{k+624} = f(x_k, x_{k+1}, x_{k+397})."""
    g = _bits(poly_words)
    top = int(np.flatnonzero(g).max())
    S = np.asarray(key, dtype=np.uint32)
    seq = np.zeros(624 + top + 1, dtype=np.uint32)
    seq[:624] = S
    h = 0
    for i in range(top - 1, -1, -1):
        a, b2, c = int(seq[h]), int(seq[h + 1]), int(seq[h + 397])
        y = (a & 0x80000000) | (b2 & 0x7fffffff)
        seq[h + 624] = c ^ (y >> 1) ^ (0x9908b0df if y & 1 else 0)
        h += 1
        if g[i]:
            seq[h:h + 624] ^= S
    return seq[h:h + 624]


@pytest.mark.parametrize("jump", [624 * 5, 1000])
def test_jump_polys_advance_numpy_state(jump):
    from ddm_amd._capi import lib
    out = np.zeros((2, 312), np.uint64)
    assert lib.ddm_mt_jump_polys(jump, 2, out.ctypes.data) == 0
    rs = np.random.RandomState(17)
    key0 = rs.get_state()[1].copy()
    for k in (1, 2):
        win = _horner(key0, out[k - 1])
        # the jumped window with pos 624 continues numpy's stream after k*jump words
        a = np.random.RandomState()
        a.set_state(("MT19937", win, 624))
        b = np.random.RandomState()
        b.set_state(("MT19937", key0, 624))
        b.randint(0, 2**32, k * jump, dtype=np.uint64)
        assert np.array_equal(a.randint(0, 2**32, 2000, dtype=np.uint64), b.randint(0, 2**32, 2000, dtype=np.uint64))
