/* ORACLE — plain-C DDM scan.  TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
 *
 * The same semantics as oracle/ddm.py:scan_stream, fast enough for C4-sized parity
 * tests: skmultiflow DDM as instantiated at DDM_Process.py:139 and fed batch by batch
 * as run_DDM does (DDM_Process.py:141-152: first warning per batch, first change
 * then break).  mode 0 = stop after the first change (controller), mode 1 = fresh
 * DDM at the next batch (DDM_Process.py:207-210 on a fixed error stream).
 *
 * Build (done by __graft_entry__.build / oracle/Makefile):
 *   gcc -O2 -ffp-contract=off -fno-fast-math -shared -fPIC ddm_scan.c -o _build/libddm_oracle.so -lm
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct {
    double p, s, p_min, s_min, ps_min;
    int64_t n;
    int32_t change, warn;
} oracle_state;

static void st_reset(oracle_state* st) {
    st->p = 1.0; st->s = 0.0;
    st->p_min = INFINITY; st->s_min = INFINITY; st->ps_min = INFINITY;
    st->n = 1; st->change = 0; st->warn = 0;
}

static void st_add(oracle_state* st, int x, int32_t min_inst, double wl, double cl) {
    if (st->change) st_reset(st);
    double n = (double)st->n;
    volatile double p = st->p + ((double)x - st->p) / n;   /* volatile: no contraction */
    volatile double v = p * (1.0 - p) / n;
    double s = sqrt(v);
    st->p = p; st->s = s;
    st->n += 1;
    st->change = 0; st->warn = 0;
    if (st->n < min_inst) return;
    volatile double ps = p + s;
    if (ps <= st->ps_min) { st->p_min = p; st->s_min = s; st->ps_min = ps; }
    volatile double tc = cl * st->s_min; tc = st->p_min + tc;
    volatile double tw = wl * st->s_min; tw = st->p_min + tw;
    if (ps > tc) st->change = 1;
    else if (ps > tw) st->warn = 1;
}

/* ev_out: [sum over streams of ceil(len/per_batch)][2] int32, written for every batch
 * (-1 where no event or past a stop).  stop_out[s]: batch of first change (mode 0) or -1.
 * state_out: [n_streams][8] doubles (p, s, p_min, s_min, ps_min, n, change, warn).
 * ps_out (nullable): [total rows][2] p,s per processed row, NaN elsewhere. */
int oracle_ddm_scan(const uint8_t* err, const int64_t* off, int64_t n_streams, int32_t per_batch,
                    int32_t min_inst, double wl, double cl, int32_t mode, int32_t* ev_out,
                    int32_t* stop_out, double* state_out, double* ps_out) {
    int64_t ev_base = 0;
    for (int64_t sidx = 0; sidx < n_streams; ++sidx) {
        int64_t lo = off[sidx], hi = off[sidx + 1], len = hi - lo;
        int64_t nb = (len + per_batch - 1) / per_batch;
        oracle_state st; st_reset(&st);
        int32_t stop = -1;
        if (ps_out) for (int64_t i = lo; i < hi; ++i) ps_out[2 * i] = ps_out[2 * i + 1] = NAN;
        for (int64_t b = 0; b < nb; ++b) {
            int32_t* ev = ev_out + 2 * (ev_base + b);
            ev[0] = -1; ev[1] = -1;
            if (stop >= 0) continue;
            int64_t blo = lo + b * per_batch, bhi = blo + per_batch < hi ? blo + per_batch : hi;
            for (int64_t i = blo; i < bhi; ++i) {
                st_add(&st, err[i] != 0, min_inst, wl, cl);
                if (ps_out) { ps_out[2 * i] = st.p; ps_out[2 * i + 1] = st.s; }
                if (st.warn && ev[0] < 0) ev[0] = (int32_t)(i - blo);
                if (st.change) { ev[1] = (int32_t)(i - blo); break; }
            }
            if (ev[1] >= 0) {
                if (mode == 0) stop = (int32_t)b;
                else st_reset(&st);
            }
        }
        stop_out[sidx] = stop;
        double* so = state_out + 8 * sidx;
        so[0] = st.p; so[1] = st.s; so[2] = st.p_min; so[3] = st.s_min; so[4] = st.ps_min;
        so[5] = (double)st.n; so[6] = st.change; so[7] = st.warn;
        ev_base += nb;
    }
    return 0;
}
