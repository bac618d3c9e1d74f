"""Host-side pieces of the GPU shuffle (ddm_amd/shuffle.py): untempering recovers numpy's
MT19937 key exactly, and the word-level Fisher-Yates / seed helpers equal numpy."""
import numpy as np

from ddm_amd.rng import MTStream
from ddm_amd.shuffle import _temper, _untemper, expected_draws_per_batch, fy_from_words, randint31_from_words


def raw_words(seed, n):
    """n tempered MT19937 outputs of RandomState(seed) (next_uint32 sequence)."""
    rs = np.random.RandomState(seed)
    return rs.randint(0, 2**32, n, dtype=np.uint64).astype(np.uint32)


def test_untemper_inverts_temper():
    x = np.random.RandomState(0).randint(0, 2**32, 100000, dtype=np.uint64).astype(np.uint32)
    assert np.array_equal(_temper(_untemper(x)), x)
    assert np.array_equal(_untemper(_temper(x)), x)


def test_untempered_block_is_numpy_key():
    rs = np.random.RandomState(3)
    w = raw_words(3, 624 * 3)           # fresh state: pos 624 -> first draw regenerates
    rs.randint(0, 2**32, 624 * 2, dtype=np.uint64)
    key = rs.get_state()[1]             # the block that produced draws 624..1247
    assert np.array_equal(_untemper(w[624:1248]), key)


def test_word_level_fisher_yates_and_seeds():
    for seed in (0, 7, 1000):
        w = raw_words(seed, 5000)
        rs = np.random.RandomState(seed)
        k = 0
        for L in (100, 100, 37, 2, 256):
            perm, used = fy_from_words(w[k:], L)
            assert np.array_equal(perm, rs.permutation(L))
            k += used
        seeds, used = randint31_from_words(w[k:], 100)
        assert np.array_equal(seeds, [rs.randint(2147483647) for _ in range(100)])
        mt = MTStream.from_seed(seed)
        mt.skip(k + used)
        assert np.array_equal(mt.key, rs.get_state()[1]) and mt.pos.value == rs.get_state()[2]


def test_expected_draws():
    assert abs(expected_draws_per_batch(100) - 141.3) < 0.2


def test_untemper_keys_rows_equal_per_stream_states():
    """The run end's one-pass read-back (BatchRunner._run: every stream's final 624-word window
    untempered at once) equals numpy's state of each stream, as untemper_state gives it."""
    from ddm_amd.shuffle import untemper_keys, untemper_state
    rows, keys = [], []
    for seed in (3, 4, 5):
        mt = MTStream.from_seed(seed)
        keys.append(mt.key.copy())
        rows.append(_temper(mt.key))
    words = np.stack(rows)
    got = untemper_keys(words)
    for k in range(3):
        assert np.array_equal(got[k], keys[k])
        assert np.array_equal(untemper_state(words[k], 624)[1], keys[k])
