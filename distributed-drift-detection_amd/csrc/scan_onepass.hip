// ddm_scan_batches in one pass: run_DDM (DDM_Process.py:135-159) in mode 1 over many
// equal-length independent error streams (configs[3]: 1M streams x 4096 rows, reset-heavy),
// a change dropping the detector (DDM_Process.py:207-210) so that the next batch starts
// from a fresh one.
//
// One wave owns a stream at a time (grid-stride over streams, the next stream's bytes in
// flight while this one is decided) and finishes it before moving on: no second kernel, no
// per-batch scratch, one coalesced store of the stream's (warning, change) rows.
//   1. The stream's bytes (up to 64 batches at a time) come in by coalesced 16-byte loads and
//      are folded into an LDS bit image; lane b cuts batch b's row bits out of it.
//   2. Every batch is speculated from a FRESH detector, lane-parallel: two leading zeros
//      make the detector trivial (its first error is the change), or the 16-row prefix
//      table finds the change; the rest is marked for evaluation.  In a reset-heavy stream
//      nearly every batch follows a change, so the speculation stands for it.
//   3. The wave walks the batches in order with the true carried detector: runs of batches
//      whose speculation stands are skipped by bit operations, a trivial detector's batches
//      are decided from their first error row, and every other batch (a fresh one the
//      speculation left open, or one with a carried detector) is evaluated by all 64 lanes
//      at once: row i of the tile has k_i errors, p_i = k_i / n_i, s_i, the running arg-min
//      of p + s is a wave scan, and the tests are a ballot.
// The exact recurrence p += (x - p) / n rounds, so k_i / n_i is not its p: the rows are
// evaluated in fp32 and every comparison the reference makes (the arg-min update, the
// change test, the warning test, up to the decision) is CERTIFIED against a rigorous bound
// on both errors -- fp32 rounding (relative 2^-17, > 5x the analysed 2^-19.5) and the
// reference recurrence's own drift from k/n (absolute n * 2^-50) -- with rows whose p is
// exactly 0 or 1 (k = 0 or k = n, exact in both) compared exactly.  A batch with an
// uncertified comparison is evaluated exactly (xtile, the sequential p chain), from its
// exact starting detector: the fresh one, or the detector's exact state replayed from the
// row where it was created.  The carried state handed back is the exact detector (a
// detector carried to the stream's end is replayed exactly), so decisions AND states equal
// the sequential scan bit for bit (tests/test_gpu_scan_batches.py, C oracle).
#include "common.h"
#include "det.h"
#include "wave_det.h"

namespace {

constexpr int kMaxBatch = 128;
constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kChunkBatches = 64;               // batches per image (lane b owns batch b)
constexpr int kPre = 16;
constexpr int kPreN = 1 << kPre;
constexpr int64_t kNoCert = (int64_t)1 << 24;  // fp32 holds k and n exactly below this
// scratch counters: [0] replays that hit a change (never: the rows were certified); in a
// -DDDM_OP_COUNT build also [1] batches evaluated by certified rows, [2] of them not
// certified (exact path), [3] exact end-state replays
constexpr int kWalkCount = 4;

// ---------------------------------------------------------------- bit helpers
// byte k of the result = (byte k of w != 0)
__device__ __forceinline__ uint32_t nzbytes(uint32_t w) {
    return ((((w & 0x7f7f7f7fu) + 0x7f7f7f7fu) | w) & 0x80808080u) >> 7;
}

// 16 bytes of 0/1 -> 16 bits (bit t = byte t) by four v_dot4_u32_u8 with byte weights 1..128
__device__ __forceinline__ uint32_t fold16(uint4 v) {
    const uint32_t lo = __builtin_amdgcn_udot4(v.y, 0x80402010u, __builtin_amdgcn_udot4(v.x, 0x08040201u, 0u, false),
                                               false);
    const uint32_t hi = __builtin_amdgcn_udot4(v.w, 0x80402010u, __builtin_amdgcn_udot4(v.z, 0x08040201u, 0u, false),
                                               false);
    return lo | (hi << 8);
}

// first set bit of (m0 | m1 << 64) at or after i (128 if none)
__device__ __forceinline__ int mask_next(uint64_t m0, uint64_t m1, int i) {
    if (i < 64) {
        const uint64_t t = m0 & (~0ull << i);
        if (t) return __builtin_ctzll(t);
        return m1 ? 64 + __builtin_ctzll(m1) : 128;
    }
    if (i >= 128) return 128;
    const uint64_t t = m1 & (~0ull << (i - 64));
    return t ? 64 + __builtin_ctzll(t) : 128;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ float readlane_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------- the prefix table
// A fresh detector's first kPre rows depend only on their kPre error bits.  Entry m (bit t
// = row t is an error): (first warning row + 1) | (change row + 1) << 5 inside the prefix
// (0 = none), and pst[m] the detector after row kPre - 1 when there is no change (n = kPre
// + 1), stepped by det_add_fast (the production recurrence, bit for bit).
__global__ __launch_bounds__(256) void k_prefix_table(ddm_params P, uint16_t* __restrict__ ptab,
                                                      double4* __restrict__ pst) {
    __shared__ double rcp[kPre + 2];
    if (threadIdx.x < kPre + 2) rcp[threadIdx.x] = 1.0 / (double)(threadIdx.x > 0 ? threadIdx.x : 1);
    __syncthreads();
    const int m = blockIdx.x * 256 + threadIdx.x;
    if (m >= kPreN) return;
    Det d;
    det_reset(d);
    int wpos = -1, cpos = -1;
    for (int i = 0; i < kPre; ++i) {
        det_add_fast(d, (m >> i) & 1, P.min_num_instances, P.warning_level, P.out_control_level, rcp);
        if (d.warn && wpos < 0) wpos = i;
        if (d.chg) {
            cpos = i;
            break;
        }
    }
    ptab[m] = (uint16_t)((wpos + 1) | ((cpos + 1) << 5));
    pst[m] = make_double4(d.p, d.pmin, d.smin, d.psmin);      // the detector after row kPre - 1
}

// ---------------------------------------------------------------- certified rows
// A detector in the form the certified rows use: k errors among the n - 1 rows it has seen
// (sample_count n), and its running minimum (p, s, p + s at the arg-min row) in fp32;
// mex: that row's p is exactly 0 or 1 (s = 0), or there is none yet (+inf).
struct CDet {
    int64_t K, cc;
    float pm, sm, psm;
    int mex;
};

__device__ __forceinline__ void cdet_fresh(CDet& c) {
    c.K = 0;
    c.cc = 1;
    c.pm = c.sm = c.psm = __builtin_inff();
    c.mex = 1;
}

// from an exact detector (not pending a change): k = rint(p (n - 1)) is exact while the
// recurrence's drift from k / (n - 1) is far below 1 / (2 (n - 1)) (n < 2^24 here)
__device__ __forceinline__ void cdet_from(CDet& c, const Det& d) {
    c.cc = d.n;
    c.K = (int64_t)__builtin_rint(d.p * (double)(d.n - 1));
    c.pm = (float)d.pmin;
    c.sm = (float)d.smin;
    c.psm = (float)d.psmin;
    c.mex = (d.psmin == __builtin_huge_val()) || (d.smin == 0.0 && (d.pmin == 0.0 || d.pmin == 1.0));
}

// a comparison of a and b (both >= 0, finite) at sample count n decides as the reference's
// when they differ by more than this
__device__ __forceinline__ float cert_bound(float a, float b, float n) {
    return 7.62939453125e-06f * (a + b) + n * 8.881784197001252e-16f;   // 2^-17 rel + n 2^-50
}

// inclusive arg-min step (ties keep the later row), as wave_det.h's argmin_step in fp32
template <int kCtrl, int kRowMask>
__device__ __forceinline__ void argmin_f(float& v, int& idx) {
    const int ob = __builtin_amdgcn_update_dpp(0x7f800000, __float_as_int(v), kCtrl, kRowMask, 0xF, false);
    const int oi = __builtin_amdgcn_update_dpp(-1, idx, kCtrl, kRowMask, 0xF, false);
    const float ov = __int_as_float(ob);
    if (oi >= 0 && (idx < 0 || !(v <= ov))) {
        v = ov;
        idx = oi;
    }
}

struct TileRes {
    int kc;      // change row or -1
    int wr;      // first warning row (before the change) or -1
    int bad;     // some comparison up to the decision is not certified
};

// Rows [0, cnt) of a tile (bits m) from detector D, all lanes (lane = row).  D moves to the
// state after the tile's last row (no change), or after the change row.
__device__ __forceinline__ TileRes cert_tile(CDet& D, uint64_t m, int cnt, int min_inst, float wl, float cl) {
    const int lane = threadIdx.x & 63;
    const bool valid = lane < cnt;
    if (cnt < 64) m &= (1ull << cnt) - 1;
    const uint64_t incl = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    const int64_t k = D.K + __builtin_popcountll(m & incl);
    const int64_t c = D.cc + lane;                    // sample count this row divides by
    const float cf = (float)c, kf = (float)k;
    const bool ex = k == 0 || k == c;                 // p exactly 0 or 1 in both (s = 0)
    const float r = __builtin_amdgcn_rcpf(cf);
    const float p = ex ? (k == 0 ? 0.0f : 1.0f) : kf * r;
    const float q = kf * (float)(c - k) * r * r * r;  // p (1 - p) / n = k (n - k) / n^3
    const float s = ex ? 0.0f : __builtin_amdgcn_sqrtf(q);
    const float ps = p + s;
    const bool gated = valid && c + 1 >= (int64_t)min_inst;
    float mv = gated ? ps : __builtin_inff();
    int mi = gated ? lane : -1;
    argmin_f<0x111, 0xF>(mv, mi);
    argmin_f<0x112, 0xF>(mv, mi);
    argmin_f<0x114, 0xF>(mv, mi);
    argmin_f<0x118, 0xF>(mv, mi);
    argmin_f<0x142, 0xA>(mv, mi);
    argmin_f<0x143, 0xC>(mv, mi);
    // the minimum before this row (exclusive) and through it (inclusive), with the carried
    // one (the later row wins ties: the reference's `<=`)
    float xv = __shfl_up(mv, 1, 64);
    int xi = __shfl_up(mi, 1, 64);
    if (lane == 0) {
        xv = __builtin_inff();
        xi = -1;
    }
    const int si = mi >= 0 ? mi : 0, sx = xi >= 0 ? xi : 0;
    const float ip = __shfl(p, si, 64), is = __shfl(s, si, 64);
    const int iex = __shfl((int)ex, si, 64), xex = __shfl((int)ex, sx, 64);
    const bool tin = mi >= 0 && mv <= D.psm;
    const bool tex = xi >= 0 && xv <= D.psm;
    const float pm = tin ? ip : D.pm, sm = tin ? is : D.sm, psm = tin ? mv : D.psm;
    const bool mex = tin ? iex != 0 : D.mex != 0;
    const float pv = tex ? xv : D.psm;
    const bool pex = tex ? xex != 0 : D.mex != 0;
    const float thc = pm + cl * sm, thw = pm + wl * sm;
    const bool chg = gated && ps > thc;
    const bool wrn = gated && !chg && ps > thw;
    const bool exact_t = ex && mex;                   // both sides of the tests exact
    const bool ok_min = !gated || pv == __builtin_inff() || (ex && pex) ||
                        __builtin_fabsf(ps - pv) > cert_bound(ps, pv, cf);
    const bool ok_c = !gated || thc == __builtin_inff() || exact_t || __builtin_fabsf(ps - thc) > cert_bound(ps, thc, cf);
    const bool ok_w = !gated || chg || thw == __builtin_inff() || exact_t ||
                      __builtin_fabsf(ps - thw) > cert_bound(ps, thw, cf);
    const uint64_t Cm = __ballot(chg);
    const int kc = Cm ? __builtin_ctzll(Cm) : -1;
    const int last = __builtin_amdgcn_readfirstlane(kc >= 0 ? kc : cnt - 1);
    const bool row_ok = !valid || lane > last || (ok_min && ok_c && ok_w);
    TileRes t;
    t.bad = __ballot(!row_ok) != 0ull;
    const uint64_t upto = last >= 63 ? ~0ull : ((2ull << last) - 1);
    const uint64_t Wm = __ballot(wrn) & upto;
    t.kc = kc;
    t.wr = Wm ? __builtin_ctzll(Wm) : -1;
    D.K = (int64_t)readlane64((uint64_t)k, last);
    D.cc += last + 1;
    D.pm = readlane_f(pm, last);
    D.sm = readlane_f(sm, last);
    D.psm = readlane_f(psm, last);
    D.mex = __builtin_amdgcn_readlane((int)mex, last);
    return t;
}

struct BatchRes {
    int w, c, bad;
};

// one batch (blen <= 128 rows, bits m0 | m1 << 64) by certified rows
__device__ __forceinline__ BatchRes cert_batch(CDet& D, uint64_t m0, uint64_t m1, int blen, int min_inst, float wl,
                                               float cl) {
    BatchRes r{-1, -1, 0};
#ifdef DDM_OP_NOCERT      // timing variant (tools/build_variant.sh): results are NOT the scan's
    r.c = 0;
    return r;
#endif
    TileRes t = cert_tile(D, m0, min(blen, 64), min_inst, wl, cl);
    if (t.bad) {
        r.bad = 1;
        return r;
    }
    r.w = t.wr;
    if (t.kc >= 0) {
        r.c = t.kc;
        return r;
    }
    if (blen > 64) {
        t = cert_tile(D, m1, blen - 64, min_inst, wl, cl);
        if (t.bad) {
            r.bad = 1;
            return r;
        }
        if (r.w < 0 && t.wr >= 0) r.w = 64 + t.wr;
        if (t.kc >= 0) r.c = 64 + t.kc;
    }
    return r;
}

// An exact tile of up to 64 rows: wave_det.h's wave_tile (same operations, bit for bit)
// with the p chain in registers: row u's RN(1/n) is computed by lane u and read by
// readlane ahead of the chain, lane u keeps p_u.  Lighter on registers than wave_tile (no
// LDS scratch, no 8-row operand groups); only the rare exact paths run it.
__device__ __forceinline__ TileOut xtile(Det& d, uint64_t m, int cnt, int min_inst, double wl, double cl) {
    const int lane = threadIdx.x & 63;
    if (cnt < 64) m &= (1ull << cnt) - 1;
    if (det_trivial(d) && m == 0) {                 // zeros in the trivial state: only n moves
        d.n += cnt;
        d.warn = 0;
        return {-1, cnt - 1, 0ull};
    }
    const double nl = (double)d.n + (double)lane;   // divisor of row lane
    const double rl = 1.0 / nl;                     // RN(1/n), as det_add_fast's rcp[] / 1.0 / n
    double p = d.p, myp = 0.0;
    for (int u = 0; u < cnt; ++u) {
        const double nu = (double)d.n + (double)u;
        const double ru = readlane_d(rl, u);
        const double xu = (double)((m >> u) & 1ull);
        p = p + div_rn(xu - p, nu, ru);
        myp = lane == u ? p : myp;
    }
    const double s = sqrt_q(div_rn(myp * (1.0 - myp), nl, rl));
    const bool gated = lane < cnt && (d.n + lane + 1 >= (int64_t)min_inst);
    const double ps = myp + s;
    double mps = gated ? ps : __builtin_huge_val();
    int midx = gated ? lane : -1;
    argmin_step<0x111, 0xF>(mps, midx);
    argmin_step<0x112, 0xF>(mps, midx);
    argmin_step<0x114, 0xF>(mps, midx);
    argmin_step<0x118, 0xF>(mps, midx);
    argmin_step<0x142, 0xA>(mps, midx);
    argmin_step<0x143, 0xC>(mps, midx);
    const bool from_lane = midx >= 0 && mps <= d.psmin;
    const int src = midx >= 0 ? midx : 0;
    const double lp = shfl_d(myp, src), ls = shfl_d(s, src);
    const double pm = from_lane ? lp : d.pmin, sm = from_lane ? ls : d.smin;
    const double psm = from_lane ? mps : d.psmin;
    const bool chg = gated && ps > pm + cl * sm;
    const bool wrn = gated && !chg && ps > pm + wl * sm;
    const uint64_t C = __ballot(chg), W = __ballot(wrn);
    const int kc = C ? __builtin_ctzll(C) : -1;
    const int last = __builtin_amdgcn_readfirstlane(kc >= 0 ? kc : cnt - 1);
    d.p = readlane_d(myp, last);
    d.s = readlane_d(s, last);
    d.pmin = readlane_d(pm, last);
    d.smin = readlane_d(sm, last);
    d.psmin = readlane_d(psm, last);
    d.n += last + 1;
    d.chg = kc >= 0;
    d.warn = (int)((W >> last) & 1ull);
    return {kc, last, W};
}

// ---------------------------------------------------------------- the kernel
// A chunk of a stream: up to 64 batches, the image of their bytes.
struct ChunkGeo {
    int64_t row0;       // first row of the chunk in the stream
    int64_t a0;         // 16-aligned global byte the image starts at
    int off;            // bit of the chunk's first row in the image
    int rows, nbc, nch; // rows, batches, 16-byte pieces
};

__device__ __forceinline__ ChunkGeo chunk_geo(int64_t s, int64_t c, int64_t L, int pb) {
    ChunkGeo g;
    g.row0 = c * (int64_t)kChunkBatches * pb;
    const int64_t start = s * L + g.row0;
    g.a0 = start & ~(int64_t)15;
    g.off = (int)(start - g.a0);
    g.rows = (int)min((int64_t)kChunkBatches * pb, L - g.row0);
    g.nbc = (g.rows + pb - 1) / pb;
    g.nch = (g.off + g.rows + 15) >> 4;
    return g;
}

template <int kLoads>
__device__ __forceinline__ void chunk_load(const uint8_t* __restrict__ err, const ChunkGeo& g, int lane,
                                           uint4 (&v)[kLoads]) {
#pragma unroll
    for (int k = 0; k < kLoads; ++k) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4* a = reinterpret_cast<const u32x4*>(err + g.a0 + 16 * min(k * 64 + lane, g.nch - 1));
        const u32x4 t = __builtin_nontemporal_load(a);
        v[k] = make_uint4(t.x, t.y, t.z, t.w);
    }
}

enum : int { kFresh = 0, kTriv = 1, kCarr = 2 };

#ifndef DDM_OP_WAVES
#define DDM_OP_WAVES 4
#endif
template <bool kPmap, int kLoads>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(DDM_OP_WAVES))) void k_scan_onepass(
    const uint8_t* __restrict__ err, int64_t n_streams, int64_t L, int64_t nb, ddm_params P,
    ddm_state* __restrict__ state, int2* __restrict__ ev, int64_t* __restrict__ nev_out,
    const uint8_t* __restrict__ pmap, const uint16_t* __restrict__ ptab, int use_pre, uint32_t* __restrict__ cnt_out) {
    __shared__ uint64_t img_all[kWaves][kLoads * 16 + 2];
    __shared__ Det s_det[kWaves][2];                  // [0] the carried-in detector, [1] the exact one (xact)
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint64_t* const img = img_all[wv];
    uint16_t* const img16 = reinterpret_cast<uint16_t*>(img);
    const int pb = (int)P.per_batch;
    const int min_inst = P.min_num_instances;
    const double wl = P.warning_level, cl = P.out_control_level;
    const float wlf = (float)wl, clf = (float)cl;
    const bool shortcuts = min_inst == 3;            // the trivial state assumes the reference gate
    const int64_t wave = (int64_t)blockIdx.x * kWaves + wv;
    const int64_t n_waves = (int64_t)gridDim.x * kWaves;
    const int64_t nchunks = (nb + kChunkBatches - 1) / kChunkBatches;
    const int delta = (int)(nb * pb - L);            // rows missing from a stream's last batch

    // work: (stream, chunk) in order; a wave takes streams wave, wave + n_waves, ...
    int64_t s = wave, c = 0;
    if (s >= n_streams) return;
    ChunkGeo g = chunk_geo(s, c, L, pb);
    uint4 v[kLoads];
    chunk_load<kLoads>(err, g, lane, v);

    // the walk's detector (wave-uniform): kFresh, kTriv (sample count tn), or kCarr (the
    // certified form cd; xact: s_det[1] is its exact state; org: the stream row it was
    // created at, -1 = it is the carried-in one)
    int kind = kFresh;
    int64_t tn = 0, org = 0, nev = 0;
    CDet cd;
    cdet_fresh(cd);
    bool xact = false;

    for (;;) {
        const int64_t srow = s * L;                  // the stream's first global row
        if (c == 0) {
            // the carried-in detector (a pending change is dropped lazily: fresh)
            const ddm_state st = state[s];
            Det din;
            din.p = st.miss_prob;
            din.s = st.miss_std;
            din.pmin = st.miss_prob_min;
            din.smin = st.miss_sd_min;
            din.psmin = st.miss_prob_sd_min;
            din.n = st.sample_count;
            din.chg = st.in_concept_change;
            din.warn = st.in_warning_zone;
            nev = 0;
            xact = false;
            if (det_fresh(din)) {
                kind = kFresh;
            } else if (shortcuts && det_trivial(din)) {
                kind = kTriv;
                tn = din.n;
            } else {
                kind = kCarr;
                xact = true;
                org = -1;
                cdet_from(cd, din);
                if (lane == 0) s_det[wv][0] = s_det[wv][1] = din;
            }
        }
        // 1. the chunk's bytes -> the LDS bit image
        uint32_t odd = 0;
#pragma unroll
        for (int k = 0; k < kLoads; ++k) odd |= v[k].x | v[k].y | v[k].z | v[k].w;
        if (__ballot((odd & 0xfefefefeu) != 0u)) {       // bytes other than 0/1
#pragma unroll
            for (int k = 0; k < kLoads; ++k) {
                v[k].x = nzbytes(v[k].x);
                v[k].y = nzbytes(v[k].y);
                v[k].z = nzbytes(v[k].z);
                v[k].w = nzbytes(v[k].w);
            }
        }
        wave_sync_lds();                                 // the previous chunk's readers are done
#pragma unroll
        for (int k = 0; k < kLoads; ++k) img16[k * 64 + lane] = (uint16_t)fold16(v[k]);
        wave_sync_lds();
        const ChunkGeo cg = g;
        // the next chunk's loads (the same chunk again after the last one)
        int64_t ns = s, ncix = c + 1;
        if (ncix >= nchunks) {
            ncix = 0;
            ns = s + n_waves;
        }
        const bool more = ns < n_streams;
        g = chunk_geo(more ? ns : s, more ? ncix : c, L, pb);
        chunk_load<kLoads>(err, g, lane, v);
        const bool last_chunk = c == nchunks - 1;

        // 2. lane b: batch b's bits and its speculation from a fresh detector
        const int nbc = cg.nbc;
        const bool valid = lane < nbc;
        const int bl = valid ? lane : 0;
        const int blen = min(pb, cg.rows - bl * pb);
        const int o = cg.off + bl * pb;
        const int wo = o >> 6, sh = o & 63;
        const uint64_t x0 = img[wo], x1 = img[wo + 1], x2 = img[wo + 2];
        uint64_t m0 = sh ? (x0 >> sh) | (x1 << (64 - sh)) : x0;
        uint64_t m1 = sh ? (x1 >> sh) | (x2 << (64 - sh)) : x1;
        if (blen < 64) {
            m0 &= (1ull << blen) - 1;
            m1 = 0;
        } else if (blen < 128) {
            m1 &= (1ull << (blen - 64)) - 1;
        }
        const int fe = mask_next(m0, m1, 0);             // first error row (128: none)
        const bool triv = shortcuts && blen >= 2 && (m0 & 3ull) == 0;
        const int t2 = mask_next(m0, m1, 2);
        const uint32_t inf = ptab[(uint32_t)(m0 & (uint64_t)(kPreN - 1))];
        const bool pre = !triv && use_pre && blen >= kPre && (inf >> 5) != 0u;
        int rw = -1, rc = -1;
        bool dec = false;
        if (triv && t2 < blen) {
            rc = t2;
            dec = true;
        } else if (pre) {
            rc = (int)(inf >> 5) - 1;
            rw = (int)(inf & 31u) - 1;
            dec = true;
        }
        const uint64_t Cm = __ballot(valid && dec);               // the fresh speculation changes
        const uint64_t Nm = __ballot(valid && triv && t2 >= blen); // trivial, no error
        const uint64_t Zm = __ballot(valid && (m0 | m1) == 0ull);  // no error at all

        // 3. the walk with the true detector; exact work (rare) in one place below
        int j = 0;
        for (;;) {
            int job = 0;                                 // 1: batch j exactly, 2: the end state
            int64_t bstart = 0;
            int bj_len = 0;
            if (j < nbc) {
                bstart = cg.row0 + (int64_t)j * pb;      // stream row of batch j
                bj_len = min(pb, cg.rows - j * pb);
                if (kind == kFresh) {
                    const uint64_t R = Cm >> j;
                    const int run = min(nbc - j, R == ~0ull ? 64 : __builtin_ctzll(~R));
                    if (run > 0) {                       // the speculation stands
                        j += run;
                        continue;
                    }
                    if ((Nm >> j) & 1ull) {
                        kind = kTriv;
                        tn = 1 + bj_len;
                        ++j;
                        continue;
                    }
                    cdet_fresh(cd);
                    org = bstart;
                    xact = false;
                } else if (kind == kTriv) {
                    const uint64_t R = Zm >> j;
                    const int run = min(nbc - j, R == ~0ull ? 64 : __builtin_ctzll(~R));
                    if (run > 0) {
                        // no error: the detector stays trivial, n moves (the stream's last
                        // batch may be short)
                        tn += (int64_t)run * pb - ((last_chunk && j + run == nbc) ? delta : 0);
                        if (lane >= j && lane < j + run) rw = rc = -1;
                        j += run;
                        continue;
                    }
                    // an error in the trivial state: the change is the batch's first error row
                    const int e = __builtin_amdgcn_readlane(fe, j);
                    if (lane == j) {
                        rw = -1;
                        rc = e;
                    }
                    kind = kFresh;
                    ++j;
                    continue;
                }
                // batch j from a fresh (just set) or carried detector: certified rows (while
                // fp32 holds k and n exactly)
                if (cd.cc + bj_len < kNoCert) {
                    const uint64_t a0 = readlane64(m0, j), a1 = readlane64(m1, j);
                    const BatchRes r = cert_batch(cd, a0, a1, bj_len, min_inst, wlf, clf);
#ifdef DDM_OP_COUNT
                    if (lane == 0) atomicAdd(cnt_out + 1 + r.bad, 1u);
#endif
                    if (!r.bad) {
                        if (lane == j) {
                            rw = r.w;
                            rc = r.c;
                        }
                        xact = false;
                        kind = r.c >= 0 ? kFresh : kCarr;
                        ++j;
                        continue;
                    }
                }
                job = 1;
            } else if (last_chunk && kind == kCarr && !xact) {
                job = 2;
#ifdef DDM_OP_COUNT
                if (lane == 0) atomicAdd(cnt_out + 3, 1u);
#endif
            } else {
                break;
            }
            // the exact path: the detector's exact state at batch j (or at the stream's
            // end), replayed from where it was created when only its certified form is
            // known, then (job 1) batch j's rows
            Det d;
            int64_t from;
            if (xact) {
                d = s_det[wv][1];
                from = bstart;
            } else if (org < 0) {
                d = s_det[wv][0];
                from = 0;
            } else {
                det_reset(d);
                from = org;
            }
            const int64_t rb = job == 1 ? bstart : L, re = job == 1 ? bstart + bj_len : L;
            int w = -1, cpos = -1;
            for (int64_t rr = from; rr < re;) {
                const int cnt = (int)min((int64_t)64, (rr < rb ? rb : re) - rr);
                uint64_t mm;
                if (rr >= cg.row0) {
                    const int ob = cg.off + (int)(rr - cg.row0);
                    const int w2 = ob >> 6, s2 = ob & 63;
                    const uint64_t y0 = img[w2], y1 = img[w2 + 1];
                    mm = s2 ? (y0 >> s2) | (y1 << (64 - s2)) : y0;
                } else {                                 // an earlier chunk's rows
                    mm = __ballot(lane < cnt && err[srow + rr + lane] != 0);
                }
                const TileOut to = xtile(d, mm, cnt, min_inst, wl, cl);
                if (rr >= rb) {
                    const uint64_t upto = to.last >= 63 ? ~0ull : ((1ull << (to.last + 1)) - 1);
                    const uint64_t wb = to.warn & upto;
                    if (w < 0 && wb) w = (int)(rr - rb) + __builtin_ctzll(wb);
                    if (to.kc >= 0) {
                        cpos = (int)(rr - rb) + to.kc;
                        break;
                    }
                } else if (d.chg) {                      // cannot happen: those rows were certified
                    if (lane == 0) atomicAdd(cnt_out, 1u);
                    d.chg = 0;
                }
                rr += cnt;
            }
            if (cpos < 0) {
                if (lane == 0) s_det[wv][1] = d;
                wave_sync_lds();
                xact = true;
                cdet_from(cd, d);
            }
            if (job == 2) break;
            if (lane == j) {
                rw = w;
                rc = cpos;
            }
            kind = cpos >= 0 ? kFresh : kCarr;
            ++j;
        }

        // 4. the chunk's rows of (first warning, change), through perm_map
        if (valid) {
            int w = rw, cc = rc;
            if (kPmap) {
                const int64_t b0 = srow + cg.row0 + (int64_t)lane * pb;
                if (w >= 0) w = pmap[b0 + w];
                if (cc >= 0) cc = pmap[b0 + cc];
            }
            ev[s * nb + c * kChunkBatches + lane] = make_int2(w, cc);
        }
        nev += __popcll(__ballot(valid && (rw >= 0 || rc >= 0)));

        if (last_chunk) {
            // the stream's exact end state
            Det d;
            if (kind == kFresh) {
                det_reset(d);
            } else if (kind == kTriv) {
                d.p = d.s = d.pmin = d.smin = d.psmin = 0.0;
                d.n = tn;
                d.chg = d.warn = 0;
            } else {
                d = s_det[wv][1];                        // xact (job 2 above)
            }
            if (lane == 0) {
                ddm_state st;
                st.miss_prob = d.p;
                st.miss_std = d.s;
                st.miss_prob_min = d.pmin;
                st.miss_sd_min = d.smin;
                st.miss_prob_sd_min = d.psmin;
                st.sample_count = d.n;
                st.in_concept_change = d.chg;
                st.in_warning_zone = d.warn;
                state[s] = st;
                if (nev_out) nev_out[s] = nev;
            }
        }
        if (!more) break;
        s = ns;
        c = ncix;
    }
}

// ---------------------------------------------------------------- streams of <= 64 batches
// The same walk with exact rows only.  A wave classifies a GROUP of streams (at most kSlots,
// their open batches at most 64), then runs the open batches -- fresh detectors whose
// change the speculation did not find -- one per lane with the exact recurrence (all 64
// lanes busy: a batch costs ~1/64 of a wave per row, against a whole wave-wide tile), then
// walks the group's streams.  A batch with a carried detector (after an unchanged one, rare
// in a reset-heavy stream) runs wave-wide (xtile) from the exact detector the walk holds.
// Every detector the walk holds is exact, so the handed-back state is too.
constexpr int kSlots = 20;
constexpr int kBatchRcp = 2 * kMaxBatch + 2;

// 128-bit nonzero mask of the rows [bstart, bstart + blen), blen in 1..128, by nine 16-byte
// loads of this lane (the rare carried batches read their bytes again)
__device__ __forceinline__ void batch_mask(const uint8_t* __restrict__ err, int64_t bstart, int blen, uint64_t& m0,
                                           uint64_t& m1) {
    const int64_t c0 = bstart & ~(int64_t)15;
    const int64_t clast = (bstart + blen - 1) & ~(int64_t)15;
    uint32_t c[9];
    const int off = (int)(bstart & 15);
    const int nch = (off + blen + 15) >> 4;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        uint4 v = *reinterpret_cast<const uint4*>(err + min(c0 + 16 * k, clast));
        v.x = nzbytes(v.x);
        v.y = nzbytes(v.y);
        v.z = nzbytes(v.z);
        v.w = nzbytes(v.w);
        c[k] = k < nch ? fold16(v) : 0u;
    }
    const uint64_t a0 = (uint64_t)c[0] | ((uint64_t)c[1] << 16) | ((uint64_t)c[2] << 32) | ((uint64_t)c[3] << 48);
    const uint64_t a1 = (uint64_t)c[4] | ((uint64_t)c[5] << 16) | ((uint64_t)c[6] << 32) | ((uint64_t)c[7] << 48);
    const uint64_t a2 = c[8];
    m0 = off ? (a0 >> off) | (a1 << (64 - off)) : a0;
    m1 = off ? (a1 >> off) | (a2 << (64 - off)) : a1;
    if (blen < 64) {
        m0 &= (1ull << blen) - 1;
        m1 = 0;
    } else if (blen < 128) {
        m1 &= (1ull << (blen - 64)) - 1;
    }
}


// One exact row of a lane's detector whose p and s are already computed (det_add_fast's
// tests): 2 = change, 1 = warning.
__device__ __forceinline__ int lane_test(Det& d, double p, double s, int min_inst, double wl, double cl) {
    d.p = p;
    d.s = s;
    d.n += 1;
    d.warn = 0;
    if (d.n < min_inst) return 0;
    const double ps = p + s;
    if (ps <= d.psmin) {
        d.pmin = p;
        d.smin = s;
        d.psmin = ps;
    }
    if (ps > d.pmin + cl * d.smin) return 2;
    d.warn = ps > d.pmin + wl * d.smin ? 1 : 0;
    return d.warn;
}

__device__ __forceinline__ void write_ev(int2* __restrict__ ev, const uint8_t* __restrict__ pmap, int64_t item,
                                        int64_t brow, int w, int c) {
    if (pmap) {
        if (w >= 0) w = pmap[brow + w];
        if (c >= 0) c = pmap[brow + c];
    }
    ev[item] = make_int2(w, c);
}

template <bool kPmap, int kLoads>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(DDM_OP_WAVES))) void k_scan_group(
    const uint8_t* __restrict__ err, int64_t n_streams, int64_t L, int64_t nb, ddm_params P,
    ddm_state* __restrict__ state, int2* __restrict__ ev, int64_t* __restrict__ nev_out,
    const uint8_t* __restrict__ pmap, const uint16_t* __restrict__ ptab, const double4* __restrict__ pst, int use_pre,
    uint32_t* __restrict__ cnt_out) {
    __shared__ uint64_t img_all[kWaves][kLoads * 16 + 2];
    __shared__ uint64_t s_msk[kWaves][kSlots][4];     // per slot: C (speculation changes), N, X (open), Z
    __shared__ int64_t s_sid[kWaves][kSlots];
    __shared__ int32_t s_jb[kWaves][kSlots];          // the slot's first job
    __shared__ uint8_t s_fe[kWaves][kSlots][64];      // first error row of each batch
    __shared__ uint64_t j_m0[kWaves][64], j_m1[kWaves][64];
    __shared__ int32_t j_hdr[kWaves][64];             // batch | rows done by the prefix << 8 | (warning + 1) << 16
    __shared__ double rcp[kBatchRcp];
    for (int k = threadIdx.x; k < kBatchRcp; k += kThreads) rcp[k] = 1.0 / (double)(k > 0 ? k : 1);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint64_t* const img = img_all[wv];
    uint16_t* const img16 = reinterpret_cast<uint16_t*>(img);
    const int pb = (int)P.per_batch;
    const int min_inst = P.min_num_instances;
    const double wl = P.warning_level, cl = P.out_control_level;
    const bool shortcuts = min_inst == 3;
    const int64_t wave = (int64_t)blockIdx.x * kWaves + wv;
    const int64_t n_waves = (int64_t)gridDim.x * kWaves;
    const int nbi = (int)nb;                          // <= 64 here
    const uint64_t below = (1ull << lane) - 1;

    int64_t s = wave;
    if (s >= n_streams) return;
    ChunkGeo g = chunk_geo(s, 0, L, pb);
    uint4 v[kLoads];
    chunk_load<kLoads>(err, g, lane, v);

    // the classified stream not yet in a group (per lane: batch `lane`)
    bool pending = false;
    int64_t psid = 0;
    uint64_t pm0 = 0, pm1 = 0, pC = 0, pN = 0, pX = 0, pZ = 0;
    int pfe = 128, prw = -1, prc = -1, phdr = 0;

    for (;;) {
        // ---- 1. a group: classify streams until kSlots or 64 open batches
        int nslots = 0, njobs = 0;
        for (;;) {
            if (!pending) {
                if (s >= n_streams) break;
                uint32_t odd = 0;
#pragma unroll
                for (int k = 0; k < kLoads; ++k) odd |= v[k].x | v[k].y | v[k].z | v[k].w;
                if (__ballot((odd & 0xfefefefeu) != 0u)) {
#pragma unroll
                    for (int k = 0; k < kLoads; ++k) {
                        v[k].x = nzbytes(v[k].x);
                        v[k].y = nzbytes(v[k].y);
                        v[k].z = nzbytes(v[k].z);
                        v[k].w = nzbytes(v[k].w);
                    }
                }
                wave_sync_lds();
#pragma unroll
                for (int k = 0; k < kLoads; ++k) img16[k * 64 + lane] = (uint16_t)fold16(v[k]);
                wave_sync_lds();
                const ChunkGeo cg = g;
                const int64_t ns = s + n_waves;
                g = chunk_geo(ns < n_streams ? ns : s, 0, L, pb);
                chunk_load<kLoads>(err, g, lane, v);
                // lane b: batch b's bits and its speculation from a fresh detector
                const bool valid = lane < nbi;
                const int bl = valid ? lane : 0;
                const int blen = min(pb, cg.rows - bl * pb);
                const int o = cg.off + bl * pb;
                const int wo = o >> 6, sh = o & 63;
                const uint64_t x0 = img[wo], x1 = img[wo + 1], x2 = img[wo + 2];
                uint64_t m0 = sh ? (x0 >> sh) | (x1 << (64 - sh)) : x0;
                uint64_t m1 = sh ? (x1 >> sh) | (x2 << (64 - sh)) : x1;
                if (blen < 64) {
                    m0 &= (1ull << blen) - 1;
                    m1 = 0;
                } else if (blen < 128) {
                    m1 &= (1ull << (blen - 64)) - 1;
                }
                const bool triv = shortcuts && blen >= 2 && (m0 & 3ull) == 0;
                const int t2 = mask_next(m0, m1, 2);
                const uint32_t inf = ptab[(uint32_t)(m0 & (uint64_t)(kPreN - 1))];
                const bool pre_ok = !triv && use_pre && blen >= kPre;
                const bool pre = pre_ok && (inf >> 5) != 0u;
                int rw = -1, rc = -1;
                bool dec = false;
                if (triv && t2 < blen) {
                    rc = t2;
                    dec = true;
                } else if (pre) {
                    rc = (int)(inf >> 5) - 1;
                    rw = (int)(inf & 31u) - 1;
                    dec = true;
                }
                const bool open = valid && !dec && !(triv && t2 >= blen);
                pC = __ballot(valid && dec);
                pN = __ballot(valid && triv && t2 >= blen);
                pX = __ballot(open);
                pZ = __ballot(valid && (m0 | m1) == 0ull);
                pm0 = m0;
                pm1 = m1;
                pfe = mask_next(m0, m1, 0);
                prw = rw;
                prc = rc;
                // an open batch longer than the prefix starts after it (no change there)
                const bool from_pre = pre_ok && blen > kPre;
                phdr = lane | ((from_pre ? kPre : 0) << 8) | ((from_pre ? (int)(inf & 31u) : 0) << 16);
                psid = s;
                s = ns;
                pending = true;
            }
            const int xc = __popcll(pX);
            if (nslots == kSlots || njobs + xc > 64) break;
            // commit the pending stream into slot nslots
            if (lane == 0) {
                s_msk[wv][nslots][0] = pC;
                s_msk[wv][nslots][1] = pN;
                s_msk[wv][nslots][2] = pX;
                s_msk[wv][nslots][3] = pZ;
                s_sid[wv][nslots] = psid;
                s_jb[wv][nslots] = njobs;
            }
            s_fe[wv][nslots][lane] = (uint8_t)pfe;
            if ((pX >> lane) & 1ull) {
                const int jx = njobs + __popcll(pX & below);
                j_m0[wv][jx] = pm0;
                j_m1[wv][jx] = pm1;
                j_hdr[wv][jx] = phdr | (nslots << 24);
            }
            if (lane < nbi) write_ev(ev, kPmap ? pmap : nullptr, psid * nb + lane, psid * L + (int64_t)lane * pb, prw, prc);
            njobs += xc;
            ++nslots;
            pending = false;
        }
        if (nslots == 0) break;
        wave_sync_lds();

        // ---- 2. the open batches, one per lane, exact rows from a fresh detector (or the
        // detector after the prefix rows)
        Det d;
        det_reset(d);
        int jw = -1, jc = -1;
        bool busy = lane < njobs;
        uint64_t m0 = 0, m1 = 0;
        int i = 0, blen = 0;
        if (busy) {
            m0 = j_m0[wv][lane];
            m1 = j_m1[wv][lane];
            const int hdr = j_hdr[wv][lane];
            const int b = hdr & 255, slot = (hdr >> 24) & 255;
            blen = (int)min((int64_t)pb, L - (int64_t)b * pb);
            i = (hdr >> 8) & 255;
            jw = ((hdr >> 16) & 255) - 1;
            (void)slot;
            if (i) {
                const double4 t = pst[(uint32_t)(m0 & (uint64_t)(kPreN - 1))];
                d.p = t.x;
                d.pmin = t.y;
                d.smin = t.z;
                d.psmin = t.w;
                d.n = i + 1;
            }
        }
        // the batch's bits from row i on, consumed two at a time
        uint64_t q0 = i == 0 ? m0 : (m0 >> i) | (m1 << (64 - i)), q1 = i == 0 ? m1 : m1 >> i;   // i in {0, 16}
#ifdef DDM_OP_NOSTEP      // timing variant: results are NOT the scan's
        busy = false;
#endif
        while (__ballot(busy)) {
            if (busy) {
                const bool two = i + 1 < blen;
                const int n0 = (int)d.n;
                const double nd0 = (double)n0, r0 = rcp[n0], nd1 = (double)(n0 + 1), r1 = rcp[n0 + 1];
                const double x0 = (double)(int)(q0 & 1ull), x1 = two ? (double)(int)((q0 >> 1) & 1ull) : 0.0;
                q0 = (q0 >> 2) | (q1 << 62);
                q1 >>= 2;
                const double p0 = d.p + div_rn(x0 - d.p, nd0, r0);
                const double p1 = p0 + div_rn(x1 - p0, nd1, r1);
                const double s0 = sqrt_q(div_rn(p0 * (1.0 - p0), nd0, r0));
                const double s1 = sqrt_q(div_rn(p1 * (1.0 - p1), nd1, r1));
                int r = lane_test(d, p0, s0, min_inst, wl, cl);
                if (r == 1 && jw < 0) jw = i;
                ++i;
                if (r != 2 && two) {
                    r = lane_test(d, p1, s1, min_inst, wl, cl);
                    if (r == 1 && jw < 0) jw = i;
                    ++i;
                }
                if (r == 2) {
                    jc = i - 1;
                    busy = false;
                } else if (i >= blen) {
                    busy = false;
                }
            }
        }

        // ---- 3. the walks
#ifdef DDM_OP_NOWALK      // timing variant: results are NOT the scan's
        nslots = 0;
#endif
        for (int k = 0; k < nslots; ++k) {
            // wave-uniform values into scalar registers: the walk is scalar code
            const uint64_t C = uni64(s_msk[wv][k][0]), N = uni64(s_msk[wv][k][1]), X = uni64(s_msk[wv][k][2]),
                           Z = uni64(s_msk[wv][k][3]);
            const int64_t sid = (int64_t)uni64((uint64_t)s_sid[wv][k]);
            const int jb = __builtin_amdgcn_readfirstlane(s_jb[wv][k]);
            const int64_t srow = sid * L;
            const ddm_state st = state[sid];
            Det c;
            c.p = st.miss_prob;
            c.s = st.miss_std;
            c.pmin = st.miss_prob_min;
            c.smin = st.miss_sd_min;
            c.psmin = st.miss_prob_sd_min;
            c.n = st.sample_count;
            c.chg = st.in_concept_change;
            c.warn = st.in_warning_zone;
            int kind = kCarr;
            if (det_fresh(c)) kind = kFresh;
            else if (shortcuts && det_trivial(c)) kind = kTriv;
            uint64_t E = C;                              // batches with an event
            int j = 0;
            while (j < nbi) {
                const int bj_len = (int)min((int64_t)pb, L - (int64_t)j * pb);
                const int64_t brow = srow + (int64_t)j * pb;
                if (kind == kFresh) {
                    const uint64_t R = C >> j;
                    const int run = min(nbi - j, R == ~0ull ? 64 : __builtin_ctzll(~R));
                    if (run > 0) {
                        j += run;
                        continue;
                    }
                    if ((N >> j) & 1ull) {
                        det_reset(c);
                        c.p = c.s = c.pmin = c.smin = c.psmin = 0.0;
                        c.n = 1 + bj_len;
                        kind = kTriv;
                        ++j;
                        continue;
                    }
                    // open: the lane that ran it holds the result and the detector after it
                    const int jl = jb + __popcll(X & ((1ull << j) - 1));
                    const int w = __builtin_amdgcn_readlane(jw, jl), cp = __builtin_amdgcn_readlane(jc, jl);
                    if (lane == 0) write_ev(ev, kPmap ? pmap : nullptr, sid * nb + j, brow, w, cp);
                    if (w >= 0 || cp >= 0) E |= 1ull << j;
                    if (cp < 0) {
                        c.p = readlane_d(d.p, jl);
                        c.s = readlane_d(d.s, jl);
                        c.pmin = readlane_d(d.pmin, jl);
                        c.smin = readlane_d(d.smin, jl);
                        c.psmin = readlane_d(d.psmin, jl);
                        c.n = __builtin_amdgcn_readlane((int)d.n, jl);
                        c.warn = __builtin_amdgcn_readlane(d.warn, jl);
                        c.chg = 0;
                        kind = kCarr;
                    }
                    ++j;
                    continue;
                }
                if (kind == kTriv) {
                    const uint64_t R = Z >> j;
                    const int run = min(nbi - j, R == ~0ull ? 64 : __builtin_ctzll(~R));
                    if (run > 0) {
                        // no error: n moves (the stream's last batch may be short); no event
                        for (int u = 0; u < run; ++u) c.n += min((int64_t)pb, L - (int64_t)(j + u) * pb);
                        const uint64_t rm = run >= 64 ? ~0ull : ((1ull << run) - 1);
                        E &= ~(rm << j);                // (their rows were written as no event)
                        j += run;
                        continue;
                    }
                    const int e = __builtin_amdgcn_readfirstlane((int)s_fe[wv][k][j]);   // the change: the first error row
                    if (lane == 0) write_ev(ev, kPmap ? pmap : nullptr, sid * nb + j, brow, -1, e);
                    E |= 1ull << j;
                    kind = kFresh;
                    ++j;
                    continue;
                }
                // kCarr: batch j wave-wide from the exact detector
                uint64_t a0, a1;
                if ((X >> j) & 1ull) {
                    const int jl = jb + __popcll(X & ((1ull << j) - 1));
                    a0 = j_m0[wv][jl];
                    a1 = j_m1[wv][jl];
                } else {
                    uint64_t b0_, b1_;
                    batch_mask(err, brow, bj_len, b0_, b1_);
                    a0 = readlane64(b0_, 0);
                    a1 = readlane64(b1_, 0);
                }
                int w = -1, cp = -1;
                for (int ci = 0; ci < bj_len; ci += 64) {
                    const int cnt = min(64, bj_len - ci);
                    const TileOut to = xtile(c, ci == 0 ? a0 : a1, cnt, min_inst, wl, cl);
                    const uint64_t upto = to.last >= 63 ? ~0ull : ((1ull << (to.last + 1)) - 1);
                    const uint64_t wb = to.warn & upto;
                    if (w < 0 && wb) w = ci + __builtin_ctzll(wb);
                    if (to.kc >= 0) {
                        cp = ci + to.kc;
                        break;
                    }
                }
                if (lane == 0) write_ev(ev, kPmap ? pmap : nullptr, sid * nb + j, brow, w, cp);
                if (w >= 0 || cp >= 0) E |= 1ull << j;
                else E &= ~(1ull << j);
                if (cp >= 0) kind = kFresh;
                ++j;
            }
            if (kind == kFresh) det_reset(c);
            if (lane == 0) {
                ddm_state o;
                o.miss_prob = c.p;
                o.miss_std = c.s;
                o.miss_prob_min = c.pmin;
                o.miss_sd_min = c.smin;
                o.miss_prob_sd_min = c.psmin;
                o.sample_count = c.n;
                o.in_concept_change = 0;
                o.in_warning_zone = kind == kCarr ? c.warn : 0;
                state[sid] = o;
                if (nev_out) nev_out[sid] = __popcll(E);
            }
        }
        (void)cnt_out;
    }
}

int64_t onepass_waves() {
    static const int64_t w = [] {
        int dev = 0, cus = 256, per_cu = 4;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_scan_onepass<false, 7>, kThreads, 0) !=
                hipSuccess ||
            per_cu <= 0)
            per_cu = 4;
        return (int64_t)cus * per_cu * kWaves;
    }();
    return w;
}

}  // namespace

extern "C" int64_t ddm_scan_batches_scratch_bytes(int64_t n_streams, int64_t stream_len, int32_t per_batch) {
    if (n_streams < 0 || stream_len < 0 || per_batch <= 0) return -1;
    return 256 + 2 * (int64_t)kPreN + 32 * (int64_t)kPreN;
}

extern "C" int ddm_scan_batches(const uint8_t* err, int64_t n_streams, int64_t stream_len, const ddm_params* prm,
                                ddm_state* state_io, int32_t* ev_out, int64_t* nev_out, void* scratch,
                                const uint8_t* perm_map, ddm_stream_t stream, ddm_event_t ev_begin,
                                ddm_event_t ev_end) {
    if (!err || !prm || !state_io || !ev_out || !scratch || n_streams < 0 || n_streams >= ((int64_t)1 << 31) ||
        stream_len < 0 || stream_len >= ((int64_t)1 << 31) || prm->per_batch <= 0 || prm->per_batch > kMaxBatch) {
        ddm::set_error("ddm_scan_batches: invalid argument (per_batch must be 1..%d, streams and stream_len < 2^31)",
                       kMaxBatch);
        return DDM_E_ARG;
    }
    hipStream_t s = ddm::as_hip(stream);
    if (ev_begin)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_begin), s), "event record")) return rc;
    if (n_streams > 0 && stream_len > 0) {
        const int64_t nb = ddm::ceil_div(stream_len, prm->per_batch);
        uint8_t* b = static_cast<uint8_t*>(scratch);
        uint32_t* cnt = reinterpret_cast<uint32_t*>(b);
        uint16_t* ptab = reinterpret_cast<uint16_t*>(b + 256);
        double4* pst = reinterpret_cast<double4*>(b + 256 + 2 * (int64_t)kPreN);
        if (int rc = ddm::hip_status(hipMemsetAsync(cnt, 0, 4 * kWalkCount, s), "ddm_scan_batches: memset")) return rc;
        hipLaunchKernelGGL(k_prefix_table, dim3(kPreN / 256), dim3(256), 0, s, *prm, ptab, pst);
        if (int rc = ddm::launch_status("ddm_scan_batches/prefix")) return rc;
        // 16-byte pieces of a chunk: (64 * pb + 15) / 16 + 1, per 64 lanes
        const int64_t rows = std::min<int64_t>(stream_len, (int64_t)kChunkBatches * prm->per_batch);
        const int64_t loads = ddm::ceil_div((rows + 15) / 16 + 1, 64);
        const bool pm = perm_map != nullptr;
        const auto kern = loads <= 3 ? (pm ? k_scan_onepass<true, 3> : k_scan_onepass<false, 3>)
                        : loads <= 5 ? (pm ? k_scan_onepass<true, 5> : k_scan_onepass<false, 5>)
                        : loads <= 7 ? (pm ? k_scan_onepass<true, 7> : k_scan_onepass<false, 7>)
                                     : (pm ? k_scan_onepass<true, 9> : k_scan_onepass<false, 9>);
        const int64_t waves = std::min<int64_t>(onepass_waves(), n_streams);
        const int64_t blocks = ddm::ceil_div(waves, kWaves);
        const bool use_pre = prm->per_batch >= kPre;
        if (nb <= kChunkBatches) {
            const auto gk = loads <= 3 ? (pm ? k_scan_group<true, 3> : k_scan_group<false, 3>)
                          : loads <= 5 ? (pm ? k_scan_group<true, 5> : k_scan_group<false, 5>)
                          : loads <= 7 ? (pm ? k_scan_group<true, 7> : k_scan_group<false, 7>)
                                       : (pm ? k_scan_group<true, 9> : k_scan_group<false, 9>);
            hipLaunchKernelGGL(gk, dim3((unsigned)blocks), dim3(kThreads), 0, s, err, n_streams, stream_len, nb, *prm,
                               state_io, reinterpret_cast<int2*>(ev_out), nev_out, perm_map, ptab, pst, (int)use_pre,
                               cnt);
        } else {
            hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kThreads), 0, s, err, n_streams, stream_len, nb,
                               *prm, state_io, reinterpret_cast<int2*>(ev_out), nev_out, perm_map, ptab, (int)use_pre,
                               cnt);
        }
        if (int rc = ddm::launch_status("ddm_scan_batches/onepass")) return rc;
    }
    if (ev_end)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_end), s), "event record")) return rc;
    return 0;
}
