"""numpy-compatible MT19937 stream driven by the native generator (ddm_mt_* in the C-ABI).

The reference consumes ONE global numpy RandomState per Python worker: a
`permutation(len(batch))` per batch (pandas `sample(frac=1)`, DDM_Process.py:187,
:190) and 100 `randint(2**31-1)` per refit (RandomForestClassifier with
random_state=None, DDM_Process.py:102).  `MTStream` holds that state as (key[624],
pos), generates batch permutations natively and converts to/from numpy's
`get_state()` tuple so the host refit (sklearn) can draw from exactly the same
position.
"""
import ctypes

import numpy as np

from ._capi import check, lib


class MTStream:
    __slots__ = ("key", "pos", "gauss")

    def __init__(self, key, pos, gauss=(0, 0.0)):
        self.key = np.ascontiguousarray(key, dtype=np.uint32).copy()
        self.pos = ctypes.c_int32(int(pos))
        # numpy's cached Gaussian (has_gauss, cached_gaussian): permutation and randint
        # leave it alone, so it is carried through untouched
        self.gauss = (int(gauss[0]), float(gauss[1]))
        assert self.key.shape == (624,)

    @classmethod
    def from_numpy_state(cls, state):
        name, key, pos = state[0], state[1], state[2]
        if name != "MT19937":
            raise ValueError(f"unsupported bit generator {name}")
        gauss = (state[3], state[4]) if len(state) >= 5 else (0, 0.0)
        return cls(key, pos, gauss)

    @classmethod
    def from_global(cls):
        return cls.from_numpy_state(np.random.get_state())

    @classmethod
    def from_seed(cls, seed):
        """numpy's RandomState(seed) state; 32-bit integer seeds natively (ddm_mt_seed)."""
        if isinstance(seed, (int, np.integer)) and 0 <= int(seed) < 2**32:
            st = cls.__new__(cls)
            st.key = np.empty(624, dtype=np.uint32)
            st.pos = ctypes.c_int32(0)
            st.gauss = (0, 0.0)
            check(lib.ddm_mt_seed(int(seed), st.key.ctypes.data, ctypes.byref(st.pos)), "ddm_mt_seed")
            return st
        return cls.from_numpy_state(np.random.RandomState(seed).get_state())

    def numpy_state(self):
        return ("MT19937", self.key.copy(), int(self.pos.value), self.gauss[0], self.gauss[1])

    def to_random_state(self):
        rs = np.random.RandomState()
        rs.set_state(self.numpy_state())
        return rs

    def load_random_state(self, rs):
        st = rs.get_state()
        self.key[:] = st[1]
        self.pos.value = int(st[2])
        self.gauss = (int(st[3]), float(st[4]))

    def snapshot(self):
        return self.key.copy(), int(self.pos.value)

    def restore(self, snap):
        self.key[:] = snap[0]
        self.pos.value = snap[1]

    def copy(self):
        return MTStream(self.key, self.pos.value, self.gauss)

    def perms(self, batch_len, out=None, draws=None):
        """Legacy `permutation(n)` for each n in batch_len (n <= 256), back to back as uint8."""
        batch_len = np.ascontiguousarray(batch_len, dtype=np.int32)
        total = int(batch_len.sum())
        if out is None:
            out = np.empty(total, dtype=np.uint8)
        assert out.dtype == np.uint8 and out.flags.c_contiguous and out.size >= total
        dptr = None
        if draws is not None:
            assert draws.dtype == np.int64 and draws.size >= batch_len.size
            dptr = draws.ctypes.data
        check(lib.ddm_mt_perms(self.key.ctypes.data, ctypes.byref(self.pos), batch_len.ctypes.data,
                               batch_len.size, out.ctypes.data, dptr), "ddm_mt_perms")
        return out

    def randint31(self, count):
        out = np.empty(count, dtype=np.int64)
        check(lib.ddm_mt_randint31(self.key.ctypes.data, ctypes.byref(self.pos), count, out.ctypes.data),
              "ddm_mt_randint31")
        return out

    def skip(self, n_draws):
        check(lib.ddm_mt_skip(self.key.ctypes.data, ctypes.byref(self.pos), int(n_draws)), "ddm_mt_skip")
