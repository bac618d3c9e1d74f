"""The classify pass's fill geometry (csrc/scan_batches.hip `fill_geo_at` and the incremental
step in `k_scan_batches_classify`), restated in numpy and checked against plain division.

A fill is 64 consecutive items (batches) of the flattened [n_streams][nb] batch grid, fill f
taken by wave f mod W.  The kernel carries each wave's first (stream, batch) from fill to fill
by a constant step instead of dividing, and derives each lane's stream offset with an fp32
reciprocal and one correction; the flush recomputes a ring slot's geometry from the stored
(s0, j0).  Every index it forms -- the lane's batch, its first row relative to the fill's
16-byte-aligned first row, its length, its flag byte -- must equal the direct form.  No GPU."""
import numpy as np
import pytest


def direct(items, L, nb, nbp, pb):
    s, j = np.divmod(items, nb)
    row = s * L + j * pb
    blen = np.minimum(pb, L - j * pb)
    return s, j, row, blen, s * nbp + j


def kernel_geo(base, s0, j0, n_items, L, nb, nbp, pb):
    """fill_geo_at for the 64 lanes of the fill whose first item is `base` = (s0, j0)."""
    lane = np.arange(64)
    delta = nb * pb - L
    b0 = s0 * L + j0 * pb
    a0 = b0 & ~15
    f0 = s0 * nbp + j0
    last = min(63, n_items - 1 - base)
    ln = np.minimum(lane, last)
    jl = j0 + ln
    inv_nb = 1.0 / nb
    if nb < (1 << 24):
        w = (np.float32(jl) * np.float32(inv_nb)).astype(np.int64)   # (int)((float)jl * (float)inv_nb)
    else:
        w = (jl.astype(np.float64) * inv_nb).astype(np.int64)
    w = np.where(w * nb > jl, w - 1, np.where((w + 1) * nb <= jl, w + 1, w))
    j = jl - w * nb
    o = (b0 - a0) + ln * pb - w * delta
    blen = np.minimum(pb, L - j * pb)
    return ln, lane <= last, a0 + o, blen, f0 + ln + w * (nbp - nb), s0 + w, j


SHAPES = [(s, L, pb) for pb in (1, 3, 16, 37, 64, 100, 128)
          for s, L in ((1, pb), (3, 5 * pb + 1), (7, 64 * pb), (5, 200 * pb - 1), (2, 333 * pb + 7))]


@pytest.mark.parametrize("n_streams,L,pb", SHAPES)
@pytest.mark.parametrize("n_waves", [1, 7, 64, 4096])
def test_fill_geometry_equals_division(n_streams, L, pb, n_waves):
    nb = -(-L // pb)
    nbp = -(-nb // 64) * 64
    n_items = n_streams * nb
    nfill = -(-n_items // 64)
    dstep = n_waves << 6
    ds, dj = divmod(dstep, nb)
    for wave in sorted({0, 1, n_waves // 2, n_waves - 1}):
        if wave >= nfill:
            continue
        s0, j0 = divmod(wave << 6, nb)          # fill_geo(wave): the general form once
        f = wave
        while f < nfill:
            base = f << 6
            assert (s0, j0) == divmod(base, nb)
            ln, valid, row, blen, fidx, s, j = kernel_geo(base, s0, j0, n_items, L, nb, nbp, pb)
            it = base + ln
            ds_, dj_, drow, dblen, dfidx = direct(it, L, nb, nbp, pb)
            np.testing.assert_array_equal(s, ds_)
            np.testing.assert_array_equal(j, dj_)
            np.testing.assert_array_equal(row, drow)
            np.testing.assert_array_equal(blen, dblen)
            np.testing.assert_array_equal(fidx, dfidx)
            assert valid.sum() == min(64, n_items - base)
            # the incremental step to the wave's next fill (wave-uniform)
            fn = f + n_waves
            if fn < nfill:
                sn, jn = s0 + ds, j0 + dj
                if jn >= nb:
                    jn -= nb
                    sn += 1
                s0, j0 = sn, jn
            f = fn
