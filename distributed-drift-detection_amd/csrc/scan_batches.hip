// ddm_scan_batches: run_DDM (DDM_Process.py:135-159) in mode 1 over many equal-length
// independent error streams (configs[3]: 1M streams x 4096 rows, reset-heavy).
//
// In mode 1 a change drops the detector (DDM_Process.py:207-210), so a batch whose
// predecessor changed starts from a fresh detector and depends on nothing before it
// (98.8 % of C4's batches).  The scan is batch-parallel speculation plus a fix-up:
//   0. k_scan_prefix_table  a fresh detector's first 16 rows from their 16 bits;
//   1. k_scan_batches_classify  streaming pass: every batch from a fresh detector, with
//      the bytes read once by coalesced 16-byte loads and folded into an LDS bit image of
//      the wave's 64 batches; trivial batches (two leading zeros: the change is the first
//      error) and batches whose change lies inside the prefix table are final here, the
//      others (~7.5 % of C4's) go to a per-wave queue;
//   2. k_scan_batches_exact<0>  the queued batches' exact rows, one lane per batch with
//      lanes refilled as they finish; an unchanged batch stores its end state and queues
//      its successor;
//   3. k_scan_batches_exact<1>  level-1 rescans: the successor of each unchanged batch
//      from that batch's end state (what it is if the unchanged batch itself was fresh);
//   4. k_scan_batches_walk / k_scan_batches_chain  every stream: a fresh carry-in and a change
//      in every batch is final; the others are walked batch by batch over the flag bytes
//      (one lane per stream), the level-1 records resolving the common case; longer
//      carried chains run in the chain kernel, one wave per stream (wave_det.h).
// Every decision is the exact fp64 recurrence of det.h; the results equal ddm_scan_streams
// in mode 1 and the C oracle bit for bit.
#include "common.h"
#include "det.h"
#include "wave_det.h"

namespace {

constexpr int kMaxBatch = 128;
constexpr int kBatchRcp = 2 * kMaxBatch + 2;   // n <= 2 * 128 + 1 in a level-1 rescan

// phase: fold
// bit k set <=> byte k of w is nonzero
__device__ __forceinline__ uint32_t nz4(uint32_t w) {
    const uint32_t t = (((w & 0x7f7f7f7fu) + 0x7f7f7f7fu) | w) & 0x80808080u;
    return (((t >> 7) * 0x00204081u) >> 21) & 0xfu;
}

__device__ __forceinline__ uint32_t nz16(uint4 v) {
    return nz4(v.x) | (nz4(v.y) << 4) | (nz4(v.z) << 8) | (nz4(v.w) << 12);
}

// byte k of the result = (byte k of w != 0)
__device__ __forceinline__ uint32_t nzbytes(uint32_t w) {
    return ((((w & 0x7f7f7f7fu) + 0x7f7f7f7fu) | w) & 0x80808080u) >> 7;
}

// 16 bytes of 0/1 (what predict writes; other nonzero bytes are made 1 first) -> 16 bits,
// bit t = byte t: four v_dot4_u32_u8 with byte weights 1..128.
__device__ __forceinline__ uint32_t fold16(uint4 v) {
    const uint32_t lo = __builtin_amdgcn_udot4(v.y, 0x80402010u, __builtin_amdgcn_udot4(v.x, 0x08040201u, 0u, false),
                                               false);
    const uint32_t hi = __builtin_amdgcn_udot4(v.w, 0x80402010u, __builtin_amdgcn_udot4(v.z, 0x08040201u, 0u, false),
                                               false);
    return lo | (hi << 8);
}

// phase: other
// 128-bit nonzero mask of the rows [bstart, bstart + blen), blen in 1..128, by nine
// 16-byte loads of this lane (the scattered form: level-1 rescans and the fix-up).
__device__ __forceinline__ void batch_mask(const uint8_t* __restrict__ err, int64_t bstart, int blen, uint64_t& m0,
                                           uint64_t& m1) {
    const int64_t c0 = bstart & ~(int64_t)15;
    const int64_t clast = (bstart + blen - 1) & ~(int64_t)15;
    uint4 v[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) v[k] = *reinterpret_cast<const uint4*>(err + min(c0 + 16 * k, clast));
    const int off = (int)(bstart & 15);
    const int nch = (off + blen + 15) >> 4;
    // 16 bytes -> 16 bits by four v_dot4 (fold16) once bytes other than 0/1 are made 1
    // (rare: a ballot decides for the lanes loading together) instead of nz16's byte tests
    uint32_t odd = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) odd |= v[k].x | v[k].y | v[k].z | v[k].w;
    if (__ballot((odd & 0xfefefefeu) != 0u)) {
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            v[k].x = nzbytes(v[k].x);
            v[k].y = nzbytes(v[k].y);
            v[k].z = nzbytes(v[k].z);
            v[k].w = nzbytes(v[k].w);
        }
    }
    uint32_t c[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) c[k] = k < nch ? fold16(v[k]) : 0u;
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

// phase: decide
__device__ __forceinline__ int mask_bit(uint64_t m0, uint64_t m1, int i) {
    return (int)((i < 64 ? m0 >> i : m1 >> (i - 64)) & 1ull);
}

// first set bit at or after i (128 if none)
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

// phase: step_rows
struct SmallDet {          // a detector inside one or two batches: n <= 2 * kMaxBatch + 1
    double p, s, pmin, smin, psmin;
    int n;
};

__device__ __forceinline__ void small_fresh(SmallDet& d) {
    d.p = 1.0;
    d.s = 0.0;
    d.pmin = d.smin = d.psmin = __builtin_huge_val();
    d.n = 1;
}

// The tests of one row whose p and s are already computed: 2 = change, 1 = warning.
__device__ __forceinline__ int small_test(SmallDet& d, double p, double s, int min_inst, double wl, double cl) {
    d.p = p;
    d.s = s;
    d.n += 1;
    if (d.n < min_inst) return 0;
    const double ps = p + s;
    if (ps <= d.psmin) {
        d.pmin = p;
        d.smin = s;
        d.psmin = ps;
    }
    if (ps > d.pmin + cl * d.smin) return 2;
    return ps > d.pmin + wl * d.smin ? 1 : 0;
}

__device__ __forceinline__ int small_add(SmallDet& d, int x, int min_inst, double wl, double cl,
                                         const double* __restrict__ rcp) {
    const double n = (double)d.n;
    const double r = rcp[d.n];
    const double p = d.p + div_rn((double)x - d.p, n, r);
    const double s = sqrt_q(div_rn(p * (1.0 - p), n, r));
    return small_test(d, p, s, min_inst, wl, cl);
}

// phase: other
// Prefix table: a fresh detector's first kPre rows depend only on their kPre error bits.
// Entry m (bit t = row t is an error): ptab[m] = (first warning row + 1) | (change row + 1)
// << 5 inside the prefix (0 = none), and, without a change, pst[m] = the detector after
// row kPre - 1 (p, p_min, s_min, ps_min; n = kPre + 1).  Built with small_add and the same
// reciprocal table, so a looked-up prefix is the stepped one bit for bit.
constexpr int kPre = 16;
constexpr int kPreN = 1 << kPre;

__global__ __launch_bounds__(256) void k_scan_prefix_table(ddm_params P, double4* __restrict__ pst,
                                                           uint16_t* __restrict__ ptab) {
    __shared__ double rcp[kBatchRcp];
    for (int k = threadIdx.x; k < kBatchRcp; k += 256) rcp[k] = 1.0 / (double)(k > 0 ? k : 1);
    __syncthreads();
    const int m = blockIdx.x * 256 + threadIdx.x;
    if (m >= kPreN) return;
    SmallDet d;
    small_fresh(d);
    int wpos = -1, cpos = -1;
    for (int i = 0; i < kPre; ++i) {
        const int r = small_add(d, (m >> i) & 1, P.min_num_instances, P.warning_level, P.out_control_level, rcp);
        if (r == 1 && wpos < 0) wpos = i;
        if (r == 2) {
            cpos = i;
            break;
        }
    }
    ptab[m] = (uint16_t)((wpos + 1) | ((cpos + 1) << 5));
    pst[m] = make_double4(d.p, d.pmin, d.smin, d.psmin);
}

__device__ __forceinline__ bool state_fresh(const ddm_state& st) {
    return st.in_concept_change || (st.sample_count == 1 && st.miss_prob == 1.0 && st.miss_std == 0.0 &&
                                    st.miss_prob_sd_min == __builtin_huge_val() &&
                                    st.miss_prob_min == __builtin_huge_val() && st.miss_sd_min == __builtin_huge_val());
}

// Flag byte of a batch (classify / exact<0> -> fix): bit 0 change, bit 1 any event, bit 2
// end state stored (pend) and the successor's level-1 record written, and what a TRIVIAL
// carried detector (every error so far 0, gate passed) makes of the batch, without its
// bytes: bit 5 no error at all (it stays trivial), bit 3 an error in row 0 or 1 (the change
// is that row; bit 4: row 1), else the change is the batch's first error row, as the fresh
// speculation found.  Level-1 flag bytes (flags1): bit 0 change, bit 1 event, bit 2 end
// state stored (pend1).
// phase: decide
constexpr uint8_t kFlagLead01 = 8, kFlagLeadRow1 = 16, kFlagNoError = 32;

__device__ __forceinline__ uint8_t lead_bits(uint64_t m0, uint64_t m1) {
    if ((m0 | m1) == 0) return kFlagNoError;
    if (m0 & 3ull) return (uint8_t)(kFlagLead01 | ((m0 & 1ull) ? 0 : kFlagLeadRow1));
    return 0;
}

// phase: item_stream
// item -> (stream, batch in stream): a float quotient corrected by one
__device__ __forceinline__ int64_t item_stream(int64_t it, int64_t nb, double inv_nb) {
    int64_t s = (int64_t)((double)it * inv_nb);
    if (s * nb > it) --s;
    else if ((s + 1) * nb <= it) ++s;
    return s;
}

// phase: sync
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// A queued batch: its 128 row bits, the detector its exact rows start from (after the
// prefix-table rows when i0 > 0) and its offset in the wave's item range.
struct QEntry {
    uint64_t m0, m1;
    double p, pmin, smin, psmin;
    int64_t it;          // the item
    int32_t hdr;         // (first warning row + 1) | i0 << 8
    int32_t pad;
};

constexpr int kClsThreads = 256;
#ifndef DDM_RING
#define DDM_RING 8
#endif
#ifndef DDM_LQ
#define DDM_LQ 128
#endif
constexpr int kRing = DDM_RING;                 // fills whose results the classify pass holds in LDS (power of 2)
constexpr int kLQ = DDM_LQ;                     // per-wave LDS queue of batches needing exact rows (power of 2)
static_assert((kRing & (kRing - 1)) == 0 && kRing <= 8 && (kLQ & (kLQ - 1)) == 0, "ring / queue sizes");
#ifndef DDM_CLS_WAVES
#define DDM_CLS_WAVES 4
#endif
constexpr int kClsWavesPerEU = DDM_CLS_WAVES;   // occupancy target of the classify pass
constexpr int kClsLoads = 9;                    // (64 * kMaxBatch + 15) / 16 + 1 chunks <= 9 * 64
constexpr int kClsWords = kClsLoads * 64 / 4;   // the LDS bit image in u64 words

// 1. Streaming classification.  The items are taken 64 at a time (a fill, one item per
// lane), fill f by wave f mod W (grid-stride: at any moment the waves read neighbouring
// fills, one narrow window of the stream).  The 64 batches are contiguous rows, so the wave reads their bytes
// with 16-byte loads that are coalesced across lanes (1 KiB per instruction), folds each
// 16-byte chunk into 16 bits in LDS, and every lane cuts its batch's 128 bits out of the
// image.  The batch is then decided from a fresh detector by bit operations (two leading
// zeros: trivial, the change is the first error) or by the prefix table; the rest is queued.
// A fill's geometry: the first item (wave-uniform, 64-bit) and each lane's batch from it
// in 32-bit offsets (w stream boundaries lie between them).
struct FillGeo {
    int64_t base, a0, f0, s0, j0;
    int ln, w, j, o, blen, nch;
    bool valid;
};

// phase: geometry
// The geometry of the fill whose first item is `base` = batch j0 of stream s0 (wave-uniform):
// per lane, 32-bit arithmetic only (the batch's stream offset w by a float reciprocal and one
// correction) while nb < 2^24 -- the general form's 64-bit products and fp64 conversions
// were a measurable part of the classify pass's VALU work, which bounds it.
__device__ __forceinline__ FillGeo fill_geo_at(int64_t base, int64_t s0, int64_t j0, int64_t n_items, int64_t L,
                                               int64_t nb, int64_t nbp, int pb, int delta, double inv_nb, int lane) {
    FillGeo g;
    g.base = base;
    g.s0 = s0;
    g.j0 = j0;
    const int64_t b0 = s0 * L + j0 * pb;            // the fill's first row
    g.a0 = b0 & ~(int64_t)15;
    g.f0 = s0 * nbp + j0;
    const int last = (int)min((int64_t)63, n_items - 1 - base);
    g.valid = lane <= last;
    g.ln = min(lane, last);                          // lanes past the end repeat the last item
    int w, j;
    if (nb < (1 << 24)) {                            // wave-uniform
        const int nbi = (int)nb, jl = (int)j0 + g.ln;
        w = (int)((float)jl * (float)inv_nb);
        if (w * nbi > jl) --w;
        else if ((w + 1) * nbi <= jl) ++w;
        j = jl - w * nbi;
    } else {
        const int64_t jl = j0 + g.ln;
        w = (int)((double)jl * inv_nb);
        if ((int64_t)w * nb > jl) --w;
        else if ((int64_t)(w + 1) * nb <= jl) ++w;
        j = (int)(jl - (int64_t)w * nb);
    }
    g.w = w;
    g.j = j;
    g.o = (int)(b0 - g.a0) + g.ln * pb - w * delta;  // the batch's first row - a0
    g.blen = min(pb, (int)L - j * pb);               // L < 2^31 (ddm_scan_batches checks)
    g.nch = __builtin_amdgcn_readfirstlane((__shfl(g.o + g.blen, 63, 64) + 15) >> 4);
    return g;
}

__device__ __forceinline__ FillGeo fill_geo(int64_t f, int64_t n_items, int64_t L, int64_t nb, int64_t nbp, int pb,
                                            int delta, double inv_nb, int lane) {
    const int64_t base = f << 6;
    const int64_t s0 = item_stream(base, nb, inv_nb);
    return fill_geo_at(base, s0, base - s0 * nb, n_items, L, nb, nbp, pb, delta, inv_nb, lane);
}

// phase: loads
// The fill's chunks, one coalesced 16-byte load per k, issued back to back (chunks past the
// fill repeat its last one: no branch between them).
template <int kLoads, bool kNt = true>
__device__ __forceinline__ void fill_load(const uint8_t* __restrict__ err, const FillGeo& g, int lane,
                                          uint4 (&v)[kLoads]) {
#pragma unroll
    for (int k = 0; k < kLoads; ++k) {
        const u32x4* a = reinterpret_cast<const u32x4*>(err + g.a0 + 16 * min(k * 64 + lane, g.nch - 1));
        const u32x4 t = kNt ? __builtin_nontemporal_load(a) : *a;
        v[k] = make_uint4(t.x, t.y, t.z, t.w);
    }
}

// The same chunks through a buffer descriptor over the fill's bytes (wave-uniform base and
// size): the lane offset is one constant VGPR and the chunk offset a scalar, so the loads
// take no VALU address work; chunks past the fill are out of the descriptor's range and read
// as zeros without a memory access.  Non-temporal (aux 2: nt).
template <int kLoads>
__device__ __forceinline__ void fill_load_buf(const uint8_t* __restrict__ err, const FillGeo& g, int lane,
                                              uint4 (&v)[kLoads]) {
    const uint64_t a = reinterpret_cast<uint64_t>(err) + (uint64_t)g.a0;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const int nbytes = __builtin_amdgcn_readfirstlane(g.nch * 16);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, nbytes, 0x00020000);
#pragma unroll
    for (int k = 0; k < kLoads; ++k) {
        const u32x4 t = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, k * 1024, 2);
        v[k] = make_uint4(t.x, t.y, t.z, t.w);
    }
}

// The classify pass's per-wave LDS: the fill's bit image, the LDS queue of batches needing
// exact rows and the ring of the last kRing fills' events and flag bytes, stored to HBM whole
// when a fill leaves the ring: by then the batches the pass steps exactly have (nearly all)
// finished, so every 512-byte event row goes out as full lines.  (Stored as decided, the rows
// had a hole per exact batch and each exact result was a lone 8-byte store: partial lines,
// which HBM reads back to merge -- 0.12 B/row of extra fetches and 0.1 B/row of extra writes.)
struct ClsWaveLds {
    uint64_t img[kClsWords + 2];
    uint64_t lq_m0[kLQ], lq_m1[kLQ];
    int2 lq_sj[kLQ];             // the batch's stream and its batch in the stream
    int2 ring_ev[kRing][64];
    int64_t ring_f0[kRing];      // the slot's fill: its first batch's flag-byte index
    uint32_t lq_hdr[kLQ];
    uint8_t ring_fl[kRing][64];
};

template <bool kPmap, int kLoads>
__global__ __launch_bounds__(kClsThreads) __attribute__((amdgpu_waves_per_eu(kClsWavesPerEU))) void k_scan_batches_classify(
    const uint8_t* __restrict__ err, int64_t n_items, int64_t L, int64_t nb, int64_t nbp, ddm_params P,
    int2* __restrict__ ev, uint8_t* __restrict__ flags, const uint8_t* __restrict__ pmap, int64_t qcap,
    uint32_t* __restrict__ need, bool use_pre, const uint16_t* __restrict__ ptab, const double4* __restrict__ pst,
    QEntry* __restrict__ q, uint32_t* __restrict__ qcnt, int64_t* __restrict__ q1, uint32_t* __restrict__ q1cnt,
    double2* __restrict__ pend, int steps, int pop_min) {
    // phase: prologue
    // one struct per wave: a single LDS base (and immediate offsets) for all of them -- as
    // separate arrays each had its own base, which the compiler spilled (a v_readlane each)
    __shared__ ClsWaveLds wlds[kClsThreads / 64];
    __shared__ double rcp[kBatchRcp];
    for (int k = threadIdx.x; k < kBatchRcp; k += kClsThreads) rcp[k] = 1.0 / (double)(k > 0 ? k : 1);
    __syncthreads();
    const int pb = (int)P.per_batch;
    const int min_inst = P.min_num_instances;
    const double wl = P.warning_level, cl = P.out_control_level;
    const bool shortcuts = min_inst == 3;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    ClsWaveLds& W = wlds[wv];
    const uint64_t below = (1ull << lane) - 1;
    const int64_t wave = (int64_t)blockIdx.x * (kClsThreads / 64) + wv;
    const int64_t n_waves = (int64_t)gridDim.x * (kClsThreads / 64);
    const int64_t nfill = (n_items + 63) >> 6;
    int64_t iter = 0;                                   // this wave's fill count (wave-uniform)
    uint16_t* const img16 = reinterpret_cast<uint16_t*>(W.img);
    QEntry* const wq = q + wave * qcap;
    const double inv_nb = 1.0 / (double)nb;
    const int delta = (int)(nb * pb - L);            // rows missing from a stream's last batch
    uint32_t count = 0;
    // exact rows inside this pass: the wave's LDS queue (ring) of batches that need them and
    // one batch per busy lane (wave-uniform ring state; overflow goes to the global queue)
    uint32_t lq_head = 0, lq_count = 0, nq = 0;
    int64_t* const wq1 = q1 + wave * qcap;
    bool busy = false, popping = false;
    bool fin = false;                                 // the lane's batch finished in this fill's steps
    int fr = 0;                                       // ... with this test result of its last row
    SmallDet d;
    small_fresh(d);
    // the lane's exact batch: stream es, batch ej in it, and the queue entry's header
    // (first warning row + 1) | rows from the prefix table << 8 | its fill's count << 16
    int ei = 0, eblen = 0, ewp = -1, es = 0, ej = 0;
    uint32_t ehdr = 0;
    uint64_t em0 = 0, em1 = 0;
    const uint32_t nb32 = (uint32_t)nb;              // nb < 2^31 (ddm_scan_batches checks)
    // the stream offset w of every lane's batch in the ring's fills, a byte per fill
    // (slots 0-3 in wr0, 4-7 in wr1): the flag-byte index of a flushed fill without its
    // geometry recomputed
    uint32_t wr0 = 0, wr1 = 0;
    // phase: step_rows
    const auto step_rows = [&]() {
        // two exact rows of this lane's batch (as k_scan_batches_exact); a finished batch is
        // marked and written by finish() once per fill (a lane that finishes idles until the
        // next fill's pop anyway; per step, the compiler hoisted the result's addressing out
        // of its branch into every step)
        if (busy) {
            const bool two = ei + 1 < eblen;
            const int n0 = d.n;
            const double nd0 = (double)n0, r0 = rcp[n0], nd1 = (double)(n0 + 1), r1 = rcp[n0 + 1];
            const double p0 = d.p + div_rn((double)mask_bit(em0, em1, ei) - d.p, nd0, r0);
            const double p1 = p0 + div_rn((double)(two ? mask_bit(em0, em1, ei + 1) : 0) - p0, nd1, r1);
            const double s0 = sqrt_q(div_rn(p0 * (1.0 - p0), nd0, r0));
            const double s1 = sqrt_q(div_rn(p1 * (1.0 - p1), nd1, r1));
            int r = small_test(d, p0, s0, min_inst, wl, cl);
            if (r == 1 && ewp < 0) ewp = ei;
            ++ei;
            if (r != 2 && two) {
                r = small_test(d, p1, s1, min_inst, wl, cl);
                if (r == 1 && ewp < 0) ewp = ei;
                ++ei;
            }
            if (r == 2 || ei >= eblen) {
                busy = false;
                fin = true;
                fr = r;
            }
        }
    };
    // phase: step_finish
    // the results of the batches that finished in this fill's steps
    const auto finish = [&]() {
        bool enq = false;
        int64_t eit = 0;
        if (fin) {
            fin = false;
            {
                const int r = fr;
                const bool chg = r == 2;
                eit = (int64_t)((uint64_t)(uint32_t)es * nb32) + ej;
                int w = ewp, c = chg ? ei - 1 : -1;
                if (kPmap) {
                    const int64_t eb = (int64_t)es * L + (int64_t)ej * pb;
                    if (w >= 0) w = pmap[eb + w];
                    if (c >= 0) c = pmap[eb + c];
                }
                if (!chg) {
                    double2* const e = pend + 3 * eit;
                    e[0] = make_double2(d.p, d.s);
                    e[1] = make_double2(d.pmin, d.smin);
                    e[2] = make_double2(d.psmin, (double)(2 * d.n + (r == 1 ? 1 : 0)));
                    need[es] = 1u;
                    enq = ej + 1 < nb;
                }
                const uint8_t fl = (uint8_t)((chg ? 1 : 0) | ((chg || w >= 0) ? 2 : 0) | (chg ? 0 : 4) |
                                             lead_bits(em0, em1));
                // the fill of this batch, if still in the ring (fills iter - kRing + 1 .. iter):
                // its fill count mod 2^16 rides in the header (a queued batch waits a few
                // hundred fills at most: 128 entries ahead of it, <= 64 steps per batch).
                // A fill that left the ring stored a placeholder here from another lane of
                // this wave (flush); this later store of the same wave to the same address
                // lands after it, as a wave's vector memory operations issue in order and
                // one address's requests stay in order through its L2 channel (the full-size
                // C4 test checks every such batch: all unchanged exact batches outlive the ring)
                const uint32_t fit = ehdr >> 16;
                if ((((uint32_t)iter - fit) & 0xffffu) < (uint32_t)kRing) {
                    const int sl = (int)(fit & (kRing - 1));
                    W.ring_ev[sl][eit & 63] = make_int2(w, c);
                    W.ring_fl[sl][eit & 63] = fl;
                } else {
                    ev[eit] = make_int2(w, c);
                    flags[(int64_t)es * nbp + ej] = fl;
                }
            }
        }
        const uint64_t qm = __ballot(enq);
        if (enq) wq1[nq + __popcll(qm & below)] = eit;
        nq += (uint32_t)__popcll(qm);
    };
    // phase: pop
    // idle lanes take queued batches (lane order); returns the prefix-table index to look up
    const auto pop = [&]() -> uint32_t {
        popping = false;
        const uint64_t idle_m = __ballot(!busy);
        const int nidle = __popcll(idle_m);
        uint32_t ix = 0;
        if (lq_count > 0 && (nidle >= pop_min || nidle == 64)) {
            const uint32_t take = min((uint32_t)nidle, lq_count);
            const uint32_t rank = (uint32_t)__popcll(idle_m & below);
            if (!busy && rank < take) {
                const uint32_t sl = (lq_head + rank) & (kLQ - 1);
                em0 = W.lq_m0[sl];
                em1 = W.lq_m1[sl];
                const int2 sj = W.lq_sj[sl];
                es = sj.x;
                ej = sj.y;
                ehdr = W.lq_hdr[sl];
                popping = true;
                ix = (uint32_t)(em0 & (uint64_t)(kPreN - 1));
            }
            lq_head = (lq_head + take) & (kLQ - 1);
            lq_count -= take;
        }
        return ix;
    };
    // phase: start
    // a popped batch's starting detector (after the prefix rows when hdr says so)
    const auto start = [&](const double4& t) {
        if (popping) {
            busy = true;
            popping = false;
            ei = (int)((ehdr >> 8) & 255u);
            ewp = (int)(ehdr & 255u) - 1;
            d.p = ei ? t.x : 1.0;
            d.s = 0.0;
            d.pmin = ei ? t.y : __builtin_huge_val();
            d.smin = ei ? t.z : __builtin_huge_val();
            d.psmin = ei ? t.w : __builtin_huge_val();
            d.n = ei + 1;
            eblen = min(pb, (int)L - ej * pb);
        }
    };
    // phase: flush
    // a ring slot's fill to HBM: its 64 event records (whole lines) and flag bytes
    const auto flush = [&](int64_t fit) {
        const int64_t base = (wave + fit * n_waves) << 6;
        const int sl = (int)(fit & (kRing - 1));
        const int last = (int)min((int64_t)63, n_items - 1 - base);
        const int w = (int)(((sl < 4 ? wr0 : wr1) >> (8 * (sl & 3))) & 255u);
        if (lane <= last) {
            ev[base + lane] = W.ring_ev[sl][lane];
#if !(defined(DDM_TUNING) && defined(DDM_PROBE_NO_FLAGS))   // timing probe only: results wrong
            flags[W.ring_f0[sl] + lane + w * (int)(nbp - nb)] = W.ring_fl[sl][lane];
#endif
        }
    };
    // phase: prologue
    // software pipeline: the next fill's loads are issued before this fill's decisions
    // and stores, so every wave keeps a fill in flight
    FillGeo g = fill_geo(wave, n_items, L, nb, nbp, pb, delta, inv_nb, lane);
    // the next fill's first item, stream and batch advance by a constant step (wave-uniform)
    const int64_t dstep = n_waves << 6, ds = dstep / nb, dj = dstep - ds * nb;
    uint4 v[kLoads];
    if (wave < nfill) fill_load_buf<kLoads>(err, g, lane, v);
    for (int64_t f = wave; f < nfill; f += n_waves) {
        // phase: fold
        // A: the fill's bytes -> the LDS bit image -> this lane's 128 row bits
        uint32_t odd = 0;
#pragma unroll
        for (int k = 0; k < kLoads; ++k) odd |= v[k].x | v[k].y | v[k].z | v[k].w;
        if (__ballot((odd & 0xfefefefeu) != 0u)) {      // bytes other than 0/1 in the fill
#pragma unroll
            for (int k = 0; k < kLoads; ++k) {
                v[k].x = nzbytes(v[k].x);
                v[k].y = nzbytes(v[k].y);
                v[k].z = nzbytes(v[k].z);
                v[k].w = nzbytes(v[k].w);
            }
        }
#pragma unroll
        for (int k = 0; k < kLoads; ++k) img16[k * 64 + lane] = (uint16_t)fold16(v[k]);
        wave_sync_lds();
        // phase: cut
        const int wo = g.o >> 6, sh = g.o & 63;
        const uint64_t x0 = W.img[wo], x1 = W.img[wo + 1], x2 = W.img[wo + 2];
        wave_sync_lds();
        uint64_t m0 = sh ? (x0 >> sh) | (x1 << (64 - sh)) : x0;
        uint64_t m1 = sh ? (x1 >> sh) | (x2 << (64 - sh)) : x1;
        const int blen = g.blen;
        if (blen < 64) {
            m0 &= (1ull << blen) - 1;
            m1 = 0;
        } else if (blen < 128) {
            m1 &= (1ull << (blen - 64)) - 1;
        }
        // phase: decide
        // B: fresh + two zero rows = trivial state (n = 3): its first error row is the change
        // (p + s > 0 = p_min + cl * s_min) and zeros raise nothing.  Otherwise the prefix
        // table (and the detector after it, for the exact rows) is looked up now.
        // Both loads below are issued before the prefetch, so their uses wait only for them.
        // The table entry is read by the lanes that use it (scattered 4-byte reads; 1.3 %
        // faster than all 64 lanes); the popped state by every lane (mostly one shared
        // address; under a per-lane or a wave-uniform branch it measured 0.5-0.6 % slower).
        const bool triv = shortcuts && blen >= 2 && (m0 & 3ull) == 0;
        const bool pre = g.valid && !triv && use_pre && blen >= kPre;
        const uint32_t ix = (uint32_t)(m0 & (uint64_t)(kPreN - 1));
        uint32_t inf = 0u;
        if (pre) inf = ptab[ix];
        // phase: pop
        const uint32_t pix = steps > 0 ? pop() : 0u;
        const double4 ppt = pst[pix];
        // phase: geometry
        // C: the next fill's loads (the last iteration reloads its own fill)
        const int64_t fn = f + n_waves;
        FillGeo gn;
        if (fn < nfill) {
            int64_t sn = g.s0 + ds, jn = g.j0 + dj;
            if (jn >= nb) {
                jn -= nb;
                ++sn;
            }
            gn = fill_geo_at(fn << 6, sn, jn, n_items, L, nb, nbp, pb, delta, inv_nb, lane);
        } else {
            gn = fill_geo(nfill - 1, n_items, L, nb, nbp, pb, delta, inv_nb, lane);
        }
        fill_load_buf<kLoads>(err, gn, lane, v);
        // phase: decide
        // D: decisions and stores
        bool exact = false;
        int wp = -1, cp = -1;
        if (g.valid) {
            uint8_t fl = 0;
            if (triv) {
                const int t = mask_next(m0, m1, 2);
                if (t < blen) {
                    cp = t;
                    fl = 3;
                } else {
                    fl = kFlagNoError;
                    need[g.s0 + g.w] = 1u;
                }
            } else if (pre) {
                cp = (int)(inf >> 5) - 1;
                wp = (int)(inf & 31u) - 1;
                if (cp >= 0) fl = (uint8_t)(3 | lead_bits(m0, m1));
                else exact = true;
            } else {
                exact = true;
            }
            if (!exact) {
                if (kPmap) {
                    if (wp >= 0) wp = pmap[g.a0 + g.o + wp];
                    if (cp >= 0) cp = pmap[g.a0 + g.o + cp];
                }
            }
            // phase: ring
            // into the ring (an exact batch's slot is written when it finishes, or by
            // k_scan_batches_exact<0> after the pass when it overflows to the global queue)
            const int sl = (int)(iter & (kRing - 1));
            W.ring_ev[sl][lane] = make_int2(wp, cp);
            W.ring_fl[sl][lane] = fl;
        }
        {
            const int sl = (int)(iter & (kRing - 1));
            if (lane == 0) W.ring_f0[sl] = g.f0;
            const uint32_t sh = 8u * (uint32_t)(sl & 3), keep = ~(255u << sh), wb = (uint32_t)g.w << sh;
            if (sl < 4) wr0 = (wr0 & keep) | wb;
            else wr1 = (wr1 & keep) | wb;
        }
        // phase: start
        start(ppt);
        // phase: queue
        uint64_t xm = __ballot(exact);
        if (steps > 0 && xm) {
            // into the LDS queue while it has room (the prefix state is looked up at the pop)
            const uint32_t room = kLQ - lq_count;
            const uint32_t r = (uint32_t)__popcll(xm & below);
            if (exact && r < room) {
                const uint32_t sl = (lq_head + lq_count + r) & (kLQ - 1);
                W.lq_m0[sl] = m0;
                W.lq_m1[sl] = m1;
                W.lq_sj[sl] = make_int2((int)(g.s0 + g.w), g.j);
                W.lq_hdr[sl] = ((pre && blen > kPre) ? (uint32_t)((wp + 1) | (kPre << 8)) : 0u) | ((uint32_t)iter << 16);
                exact = false;
            }
            lq_count += min((uint32_t)__popcll(xm), room);
            xm = __ballot(exact);
        }
        if (exact) {
            // the detector after the prefix rows (no change there) when the batch is longer;
            // its prefix state is loaded only here (the LDS queue's batches look it up at the
            // pop): an unconditional 32-byte load per batch was 1.3 GB of L2 reads per C4 call
            // for the few batches that overflow to the global queue
            const double4 pt = pst[ix];
            QEntry e;
            e.m0 = m0;
            e.m1 = m1;
            const bool from_pre = pre && blen > kPre;
            e.p = from_pre ? pt.x : 1.0;
            e.pmin = from_pre ? pt.y : __builtin_huge_val();
            e.smin = from_pre ? pt.z : __builtin_huge_val();
            e.psmin = from_pre ? pt.w : __builtin_huge_val();
            e.it = g.base + g.ln;
            e.hdr = from_pre ? ((wp + 1) | (kPre << 8)) : 0;
            e.pad = 0;
            wq[count + __popcll(xm & below)] = e;
        }
        count += (uint32_t)__popcll(xm);
        // phase: step_rows
        // E: exact rows of the queued batches
        for (int k = 0; k < steps; ++k) {
            if (__ballot(busy) == 0ull) break;
            step_rows();
        }
        // phase: step_finish
        if (__ballot(fin)) finish();
        // phase: flush
        g = gn;
        ++iter;
        if (iter >= kRing) {                            // the slot the next fill takes
            wave_sync_lds();
            flush(iter - kRing);
        }
    }
    // phase: drain
    // drain the LDS queue (finished batches still land in the ring), then the ring
    if (steps > 0) {
        for (;;) {
            const uint32_t pix = pop();
            start(pst[pix]);
            if (__ballot(busy) == 0ull && lq_count == 0) break;
            step_rows();
            if (__ballot(fin)) finish();
        }
    }
    wave_sync_lds();
    for (int64_t fit = max((int64_t)0, iter - kRing + 1); fit < iter; ++fit) flush(fit);
    if (lane == 0) {
        qcnt[wave] = count;
        q1cnt[wave] = nq;
    }
}

// phase: other
#ifdef DDM_TUNING
// Timing probe (DDM_SCAN_PROBE=1, tuning builds only; results are NOT the scan's): the classify pass's reads,
// LDS image and bit extraction with one 8-byte store per batch and nothing else, to price
// its decision and queue work against the pure stream.
template <int kLoads, int kMode>
__global__ __launch_bounds__(kClsThreads) void k_scan_batches_probe(
    const uint8_t* __restrict__ err, int64_t n_items, int64_t L, int64_t nb, int64_t nbp, ddm_params P,
    int2* __restrict__ ev, uint32_t* __restrict__ qcnt, uint32_t* __restrict__ q1cnt) {
    // kMode 0: as the classify pass (non-temporal loads, one fill ahead); 1: plain loads;
    // 2: two fills ahead
    constexpr bool kNt = kMode != 1;
    __shared__ uint64_t img[kClsThreads / 64][kClsWords + 2];
    const int pb = (int)P.per_batch;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t wave = (int64_t)blockIdx.x * (kClsThreads / 64) + wv;
    const int64_t n_waves = (int64_t)gridDim.x * (kClsThreads / 64);
    const int64_t nfill = (n_items + 63) >> 6;
    uint16_t* const img16 = reinterpret_cast<uint16_t*>(img[wv]);
    const double inv_nb = 1.0 / (double)nb;
    const int delta = (int)(nb * pb - L);
    FillGeo g = fill_geo(wave, n_items, L, nb, nbp, pb, delta, inv_nb, lane);
    FillGeo g2 = fill_geo(min(wave + n_waves, nfill - 1), n_items, L, nb, nbp, pb, delta, inv_nb, lane);
    uint4 v[kLoads], v2[kLoads];
    if (wave < nfill) {
        fill_load<kLoads, kNt>(err, g, lane, v);
        if (kMode == 2) fill_load<kLoads, kNt>(err, g2, lane, v2);
    }
    for (int64_t f = wave; f < nfill; f += n_waves) {
#pragma unroll
        for (int k = 0; k < kLoads; ++k) img16[k * 64 + lane] = (uint16_t)fold16(v[k]);
        wave_sync_lds();
        const int wo = g.o >> 6, sh = g.o & 63;
        const uint64_t x0 = img[wv][wo], x1 = img[wv][wo + 1], x2 = img[wv][wo + 2];
        wave_sync_lds();
        const uint64_t m0 = sh ? (x0 >> sh) | (x1 << (64 - sh)) : x0;
        const uint64_t m1 = sh ? (x1 >> sh) | (x2 << (64 - sh)) : x1;
        FillGeo gn;
        if (kMode == 2) {
#pragma unroll
            for (int k = 0; k < kLoads; ++k) v[k] = v2[k];
            gn = g2;
            const int64_t f3 = f + 2 * n_waves;
            g2 = fill_geo(min(f3, nfill - 1), n_items, L, nb, nbp, pb, delta, inv_nb, lane);
            fill_load<kLoads, kNt>(err, g2, lane, v2);
        } else {
            const int64_t fn = f + n_waves;
            gn = fill_geo(min(fn, nfill - 1), n_items, L, nb, nbp, pb, delta, inv_nb, lane);
            fill_load<kLoads, kNt>(err, gn, lane, v);
        }
        if (g.valid) ev[g.base + g.ln] = make_int2((int)(m0 ^ m1), (int)((m0 ^ m1) >> 32));
        g = gn;
    }
    if (lane == 0) qcnt[wave] = q1cnt[wave] = 0;
}
#endif  // DDM_TUNING

// 2./3. Exact rows, one lane per queued batch.  Lanes that finish take the next entries of
// the wave's queue (one claim for all idle lanes, no atomics: the queue is the wave's own);
// each step runs two rows (p and s of row i + 1 depend on p_i alone, so both rows'
// arithmetic is issued before the tests).
//   kLevel 0: entries of the classify queue, a fresh detector (the prefix table gives the
//             first 16 rows when the batch is longer); writes ev / flags, and for an
//             unchanged batch its end state (pend) and its successor into the level-1 queue;
//   kLevel 1: the successor t = i + 1 of an unchanged batch i, from pend[i]: writes the
//             level-1 record of t (ev1, flags1, pend1 when t is unchanged too).
constexpr int kExThreads = 256;

template <int kLevel, bool kPmap>
__global__ __launch_bounds__(kExThreads) void k_scan_batches_exact(
    const uint8_t* __restrict__ err, int64_t n_items, int64_t L, int64_t nb, int64_t nbp, ddm_params P,
    int2* __restrict__ ev, uint8_t* __restrict__ flags, const uint8_t* __restrict__ pmap, int64_t qcap,
    uint32_t* __restrict__ need, const QEntry* __restrict__ q, const uint32_t* __restrict__ qcnt,
    int64_t* __restrict__ q1,
    uint32_t* __restrict__ q1cnt, double2* __restrict__ pend, int2* __restrict__ ev1, uint8_t* __restrict__ flags1,
    double2* __restrict__ pend1, int refill, uint32_t* __restrict__ ctr, int64_t* __restrict__ spec_list,
    int32_t* __restrict__ sidx, uint32_t spec_cap) {
    __shared__ double rcp[kBatchRcp];
    for (int k = threadIdx.x; k < kBatchRcp; k += kExThreads) rcp[k] = 1.0 / (double)(k > 0 ? k : 1);
    __syncthreads();
    const int pb = (int)P.per_batch;
    const int min_inst = P.min_num_instances;
    const double wl = P.warning_level, cl = P.out_control_level;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t below = (1ull << lane) - 1;
    const int64_t wave = (int64_t)blockIdx.x * (kExThreads / 64) + wv;
    const int64_t wq = wave * qcap;                 // this wave's queue slots
    const uint32_t n = kLevel == 0 ? qcnt[wave] : q1cnt[wave];
    const double inv_nb = 1.0 / (double)nb;
    uint32_t head = 0;                              // wave-uniform
    uint32_t nq = kLevel == 0 ? q1cnt[wave] : 0;    // after the classify pass's level-1 entries
    bool busy = false;
    int64_t it = 0, s = 0, j = 0, bstart = 0;
    int blen = 0, i = 0, wpos = -1;
    uint64_t m0 = 0, m1 = 0;
    SmallDet d;
    small_fresh(d);
    for (;;) {
        const uint64_t idle_m = __ballot(!busy);
        const int nidle = __popcll(idle_m);
        if (head < n && (nidle >= refill || nidle == 64)) {
            const uint32_t take = min((uint32_t)nidle, n - head);
            if (!busy) {
                const uint32_t rank = (uint32_t)__popcll(idle_m & below);
                if (rank < take) {
                    busy = true;
                    if (kLevel == 0) {
                        // the classify queue entry carries the starting detector (one load)
                        const QEntry e = q[wq + head + rank];
                        m0 = e.m0;
                        m1 = e.m1;
                        d.p = e.p;
                        d.s = 0.0;
                        d.pmin = e.pmin;
                        d.smin = e.smin;
                        d.psmin = e.psmin;
                        i = e.hdr >> 8;
                        d.n = i + 1;
                        wpos = (e.hdr & 255) - 1;
                        it = e.it;
                        s = item_stream(it, nb, inv_nb);
                        j = it - s * nb;
                        bstart = s * L + j * pb;
                        blen = (int)min((int64_t)pb, L - j * pb);
                    } else {
                        i = 0;
                        wpos = -1;
                        const int64_t ip = q1[wq + head + rank];
                        it = ip + 1;                // same stream: queued only when j + 1 < nb
                        s = item_stream(it, nb, inv_nb);
                        j = it - s * nb;
                        bstart = s * L + j * pb;
                        blen = (int)min((int64_t)pb, L - j * pb);
                        const double2* e = pend + 3 * ip;
                        const double2 a = e[0], b = e[1], c = e[2];
                        d.p = a.x;
                        d.s = a.y;
                        d.pmin = b.x;
                        d.smin = b.y;
                        d.psmin = c.x;
                        d.n = (int)((int64_t)c.y >> 1);
                        batch_mask(err, bstart, blen, m0, m1);
                    }
                }
            }
            head += take;
        }
        if (__ballot(busy) == 0ull) {
            if (head >= n) break;
            continue;
        }
        bool enq = false, spec = false;
        if (busy) {
            const bool two = i + 1 < blen;
            const int n0 = d.n;
            const double nd0 = (double)n0, r0 = rcp[n0], nd1 = (double)(n0 + 1), r1 = rcp[n0 + 1];
            const double p0 = d.p + div_rn((double)mask_bit(m0, m1, i) - d.p, nd0, r0);
            const double p1 = p0 + div_rn((double)(two ? mask_bit(m0, m1, i + 1) : 0) - p0, nd1, r1);
            const double s0 = sqrt_q(div_rn(p0 * (1.0 - p0), nd0, r0));
            const double s1 = sqrt_q(div_rn(p1 * (1.0 - p1), nd1, r1));
            int r = small_test(d, p0, s0, min_inst, wl, cl);
            if (r == 1 && wpos < 0) wpos = i;
            ++i;
            if (r != 2 && two) {
                r = small_test(d, p1, s1, min_inst, wl, cl);
                if (r == 1 && wpos < 0) wpos = i;
                ++i;
            }
            if (r == 2 || i >= blen) {
                const bool chg = r == 2;
                int w = wpos, c = chg ? i - 1 : -1;
                if (kPmap) {
                    if (w >= 0) w = pmap[bstart + w];
                    if (c >= 0) c = pmap[bstart + c];
                }
                double2* const e = (kLevel == 0 ? pend : pend1) + 3 * it;
                if (!chg) {
                    e[0] = make_double2(d.p, d.s);
                    e[1] = make_double2(d.pmin, d.smin);
                    e[2] = make_double2(d.psmin, (double)(2 * d.n + (r == 1 ? 1 : 0)));
                }
                const uint8_t fl = (uint8_t)((chg ? 1 : 0) | ((chg || w >= 0) ? 2 : 0) | (chg ? 0 : 4));
                if (kLevel == 0) {
                    ev[it] = make_int2(w, c);
                    flags[s * nbp + j] = (uint8_t)(fl | lead_bits(m0, m1));
                    if (!chg) {
                        need[s] = 1u;
                        enq = j + 1 < nb;
                    }
                } else {
                    ev1[it] = make_int2(w, c);
                    flags1[it] = fl;
                    spec = !chg && j + 1 < nb;   // a carried run from here on: the spec list
                }
                busy = false;
            }
        }
        if (kLevel == 1) {
            // an unchanged level-1 batch t: the run carried on from pend1[t] is computed ahead
            // by k_scan_batches_walk's spec blocks (beside the walk), its index in sidx[t]
            const uint64_t sm = __ballot(spec);
            if (sm) {
                uint32_t base = 0;
                const int lead = __builtin_ctzll(sm);
                if (lane == lead) base = atomicAdd(ctr + 3, (uint32_t)__popcll(sm));
                base = __shfl(base, lead);
                if (spec) {
                    const uint32_t k = base + (uint32_t)__popcll(sm & below);
                    if (k < spec_cap) spec_list[k] = it;
                    sidx[it] = k < spec_cap ? (int32_t)k : -1;
                }
            }
        }
        if (kLevel == 0) {
            const uint64_t em = __ballot(enq);
            if (enq) q1[wq + nq + __popcll(em & below)] = it;
            nq += (uint32_t)__popcll(em);
        }
    }
    if (kLevel == 0 && lane == 0) q1cnt[wave] = nq;
}

__device__ __forceinline__ void load_det(Det& d, const ddm_state& st) {
    d.p = st.miss_prob;
    d.s = st.miss_std;
    d.pmin = st.miss_prob_min;
    d.smin = st.miss_sd_min;
    d.psmin = st.miss_prob_sd_min;
    d.n = st.sample_count;
    d.chg = st.in_concept_change;
    d.warn = st.in_warning_zone;
}

__device__ __forceinline__ ddm_state store_det(const Det& d) {
    ddm_state st;
    st.miss_prob = d.p;
    st.miss_std = d.s;
    st.miss_prob_min = d.pmin;
    st.miss_sd_min = d.smin;
    st.miss_prob_sd_min = d.psmin;
    st.sample_count = d.n;
    st.in_concept_change = d.chg;
    st.in_warning_zone = d.warn;
    return st;
}

__device__ __forceinline__ void load_end_state(Det& d, const double2* __restrict__ e) {
    const double2 a = e[0], b = e[1], c = e[2];
    const int64_t nw = (int64_t)c.y;
    d.p = a.x;
    d.s = a.y;
    d.pmin = b.x;
    d.smin = b.y;
    d.psmin = c.x;
    d.n = nw >> 1;
    d.warn = (int)(nw & 1);
    d.chg = 0;
}

// 4. Fix-up of the streams with an unchanged batch or a carried-in detector: the walker
// (one lane per stream) resolves most of them from the flag bytes and the level-1 records;
// the rest -- a detector carried through two or more unchanged batches, at most a few
// thousand rows in C4 -- run in the chain kernel, one wave per stream.

// bits [i, i + 64) of the 128-bit mask (a0 | a1 << 64), i < 64
__device__ __forceinline__ uint64_t m0_shift(uint64_t a0, uint64_t a1, int i) {
    return i == 0 ? a0 : (a0 >> i) | (a1 << (64 - i));
}

struct LeadMasks {           // flag bits 3, 4, 5 of a 64-batch window as bit masks
    uint64_t l01, row1, none;
};

// One 64-batch window of flag bytes as bit masks: bit 0 of each byte (change) into the
// result, bit 2 (end state stored) into sm, bit 1 (event) into em.
__device__ __forceinline__ uint64_t change_window(const uint8_t* __restrict__ fl, int64_t wbase, int64_t nb,
                                                  uint64_t& sm, uint64_t& em, LeadMasks& lm) {
    uint64_t m = 0, ms = 0, me = 0, ml = 0, mr = 0, mz = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint4 v = *reinterpret_cast<const uint4*>(fl + wbase + 16 * q);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int sh = 16 * q + 4 * k;
            m |= (uint64_t)(((((w[k] >> 0) & 0x01010101u) * 0x00204081u) >> 21) & 0xfu) << sh;
            me |= (uint64_t)(((((w[k] >> 1) & 0x01010101u) * 0x00204081u) >> 21) & 0xfu) << sh;
            ms |= (uint64_t)(((((w[k] >> 2) & 0x01010101u) * 0x00204081u) >> 21) & 0xfu) << sh;
            ml |= (uint64_t)(((((w[k] >> 3) & 0x01010101u) * 0x00204081u) >> 21) & 0xfu) << sh;
            mr |= (uint64_t)(((((w[k] >> 4) & 0x01010101u) * 0x00204081u) >> 21) & 0xfu) << sh;
            mz |= (uint64_t)(((((w[k] >> 5) & 0x01010101u) * 0x00204081u) >> 21) & 0xfu) << sh;
        }
    }
    const int64_t valid = nb - wbase;
    const uint64_t vm = valid < 64 ? (1ull << valid) - 1 : ~0ull;
    sm = ms & vm;
    em = me & vm;
    lm.l01 = ml & vm;
    lm.row1 = mr & vm;
    lm.none = mz & vm;
    return m & vm;
}

// The flag-byte walk of one stream (fix-up "open"): from batch j with detector d, skip
// every batch whose result needs no rows -- runs whose speculative change stands, a
// trivial detector's batches (flag bits), an unchanged batch's stored end state with its
// successor's level-1 record -- and stop at the stream's end or at the first batch whose
// rows must be run with a carried detector.
struct Walk {
    Det d;
    int64_t sid, j, wbase, nev;
    int64_t lvl1;       // where walk_open stopped: the unchanged level-1 batch t it carries on from, or -1
    uint64_t chg_m, st_m, ev_m;
    LeadMasks lm;
};

__device__ __forceinline__ void walk_open(Walk& W, int64_t L, int64_t nb, int64_t nbp, int64_t pb, bool shortcuts,
                                          int2* __restrict__ ev, const uint8_t* __restrict__ flags,
                                          const uint8_t* __restrict__ pmap, const double2* __restrict__ pend,
                                          const int2* __restrict__ ev1, const uint8_t* __restrict__ flags1,
                                          const double2* __restrict__ pend1) {
    Det& d = W.d;
    int64_t& j = W.j;
    int64_t& wbase = W.wbase;
    int64_t& nev = W.nev;
    const int64_t sid = W.sid;
    uint64_t& chg_m = W.chg_m;
    uint64_t& st_m = W.st_m;
    uint64_t& ev_m = W.ev_m;
    LeadMasks& lm = W.lm;
    W.lvl1 = -1;
    for (;;) {
        if (j >= nb) break;
        if (j >= wbase + 64) {          // next 64-batch window (nb > 64 only)
            wbase = j & ~(int64_t)63;
            chg_m = change_window(flags + sid * nbp, wbase, nb, st_m, ev_m, lm);
        }
        if (shortcuts && det_trivial(d)) {
            // a trivial detector (after a batch of zeros): the batch's flag
            // bits give its result without its bytes (see kFlagNoError)
            const int o = (int)(j - wbase);
            if ((lm.none >> o) & 1ull) {
                d.n += min(pb, L - j * pb);
                d.warn = 0;
            } else {
                if ((lm.l01 >> o) & 1ull) {     // the change is row 0 or 1
                    const int t = (int)((lm.row1 >> o) & 1ull);
                    ev[sid * nb + j] = make_int2(-1, pmap ? (int)pmap[sid * L + j * pb + t] : t);
                }                               // else: the speculative change stands
                ++nev;
                det_reset(d);
            }
            ++j;
            continue;
        }
        if (!det_fresh(d)) break;
        if (shortcuts && ((lm.none >> (j - wbase)) & 1ull)) {
            // a fresh detector and a batch without an error: two zeros make it
            // trivial (n = 3), the rest only move n (no bytes needed)
            const int bl = (int)min(pb, L - j * pb);
            if (bl >= 2) {
                d.p = d.s = d.pmin = d.smin = d.psmin = 0.0;
                d.n = 1 + bl;
                d.chg = d.warn = 0;
                ++j;
                continue;
            }
        }
        const uint64_t rel = chg_m >> (j - wbase);
        const int run = (int)min((int64_t)(rel == ~0ull ? 64 : __builtin_ctzll(~rel)), wbase + 64 - j);
        if (run > 0) {
            nev += run;                 // batches whose speculative change stands
            j += run;
            det_reset(d);
            continue;
        }
        if (!((st_m >> (j - wbase)) & 1ull)) break;
        // fresh detector, unchanged batch whose end state the exact pass stored:
        // carry it on, and its successor's level-1 record is the successor's result
        load_end_state(d, pend + 3 * (sid * nb + j));
        nev += (int64_t)((ev_m >> (j - wbase)) & 1ull);
        ++j;
        if (j >= nb) break;
        const int64_t t = sid * nb + j;
        const uint8_t f1 = flags1[t];
        ev[t] = ev1[t];
        nev += (f1 >> 1) & 1;
        ++j;
        if (f1 & 1) {
            det_reset(d);
            continue;
        }
        load_end_state(d, pend1 + 3 * t);
        W.lvl1 = t;
        break;
    }
}

// A stream the walker hands to the fix-up kernel: where it stopped and the detector there.
struct FixEntry {
    Det d;
    int64_t sid, j, nev;
    int64_t lvl1;       // Walk::lvl1 where the walker stopped
};

// The carried run after an unchanged level-1 batch t, computed ahead (spec blocks of
// k_scan_batches_walk): batches t + 1 .. end_j of the stream from pend1[t], one event record
// each in spec_ev[k][...], kSpecBatches at most.  status 1: the run changed in batch end_j
// (the detector resets after it); 2: it reached the stream's end without a change, d the
// final detector; 3: cut after kSpecBatches batches, d the detector before batch end_j.
// Whether the run is the stream's (t's predecessor reached with a fresh detector) only the
// walk knows: the fix-up takes it where the walk stopped at t, ignores it elsewhere.
constexpr int kSpecBatches = 64;
struct SpecRes {
    Det d;
    int64_t end_j;
    int32_t status, nev;
};

// One batch of a stream from a carried detector c, by the wave: its bytes through the wave's
// LDS bit image (batches [ib, ib + 64) of the stream, refilled by coalesced loads when j
// leaves it), its rows through wave_tile tiles.  Returns the batch's event record (pmap
// applied); c is left as it stands after the batch (in a pending change when cp >= 0).
struct ChainImg {
    int64_t ib, ia0;
};

__device__ __forceinline__ int2 chain_batch(Det& c, int64_t sid, int64_t j, const uint8_t* __restrict__ err,
                                            int64_t L, int64_t pb, int min_inst, double wl, double cl,
                                            const uint8_t* __restrict__ pmap, uint64_t* img, double* tw,
                                            ChainImg& im, int& cp_out) {
    const int lane = threadIdx.x & 63;
    uint16_t* const img16 = reinterpret_cast<uint16_t*>(img);
    const int64_t srow = sid * L;
    if (j < im.ib || j >= im.ib + 64) {
        // batches [j & ~63, +64) of the stream into the image
        im.ib = j & ~(int64_t)63;
        im.ia0 = (srow + im.ib * pb) & ~(int64_t)15;
        const int64_t iend = srow + min(L, (im.ib + 64) * pb);
        const int nch = (int)((iend - im.ia0 + 15) >> 4);
        wave_sync_lds();
        for (int c0 = 0; c0 < nch; c0 += 64) {
            const int ch = min(c0 + lane, nch - 1);
            uint4 v = *reinterpret_cast<const uint4*>(err + im.ia0 + 16 * (int64_t)ch);
            v.x = nzbytes(v.x);
            v.y = nzbytes(v.y);
            v.z = nzbytes(v.z);
            v.w = nzbytes(v.w);
            img16[ch] = (uint16_t)fold16(v);
        }
        wave_sync_lds();
    }
    const int64_t bstart = srow + j * pb;
    const int blen = (int)min(pb, L - j * pb);
    const int o = (int)(bstart - im.ia0);
    const int wo = o >> 6, sh = o & 63;
    const uint64_t x0 = img[wo], x1 = img[wo + 1], x2 = img[wo + 2];
    const uint64_t a0 = sh ? (x0 >> sh) | (x1 << (64 - sh)) : x0;
    const uint64_t a1 = sh ? (x1 >> sh) | (x2 << (64 - sh)) : x1;
    c.chg = 0;
    int ci = 0, cw = -1, cp = -1;
    while (ci < blen) {
        const int cnt = min(64, blen - ci);
        const uint64_t m = ci < 64 ? m0_shift(a0, a1, ci) : (a1 >> (ci - 64));
        const TileOut to = wave_tile(c, m, cnt, min_inst, wl, cl, tw);
        const uint64_t upto = to.last >= 63 ? ~0ull : ((1ull << (to.last + 1)) - 1);
        const uint64_t wb = to.warn & upto;
        if (cw < 0 && wb) cw = ci + __builtin_ctzll(wb);
        if (to.kc >= 0) {
            cp = ci + to.kc;
            break;
        }
        ci += cnt;
    }
    int w = cw, cc = cp;
    if (pmap) {
        if (w >= 0) w = pmap[bstart + w];
        if (cc >= 0) cc = pmap[bstart + cc];
    }
    cp_out = cp;
    return make_int2(w, cc);
}

// 4a. The walker: one lane per listed stream (no cooperation, few registers, many lanes in
// flight), walk_open over its flag bytes from the carried-in state.  Most streams end here;
// a stream that needs rows with a carried detector (a chain longer than the level-1 records,
// or a carried-in state) goes to the fix-up list with its position.
//
// The same launch's first spec_blocks workgroups (dispatched first) run the speculative
// carried runs instead, one wave per spec-list entry t (an unchanged level-1 batch): the
// batches after t from pend1[t] until a change, into spec_ev / spec_res.  They need nothing
// of the walk, so the longest carried runs start with it instead of after it.
#ifndef DDM_WALK_THREADS
#define DDM_WALK_THREADS 256
#endif
constexpr int kWalkThreads = DDM_WALK_THREADS;
#ifndef DDM_WALK_WAVES
#define DDM_WALK_WAVES 4
#endif

__global__ __launch_bounds__(kWalkThreads) __attribute__((amdgpu_waves_per_eu(DDM_WALK_WAVES))) void k_scan_batches_walk(
    const uint8_t* __restrict__ err, int64_t n_streams, int64_t L, int64_t nb, int64_t nbp, ddm_params P,
    ddm_state* __restrict__ state, int2* __restrict__ ev, const uint8_t* __restrict__ flags,
    int64_t* __restrict__ nev_out, const uint8_t* __restrict__ pmap, const uint32_t* __restrict__ need,
    uint32_t* __restrict__ ctr, const double2* __restrict__ pend, const int2* __restrict__ ev1,
    const uint8_t* __restrict__ flags1, const double2* __restrict__ pend1, FixEntry* __restrict__ coop,
    int spec_blocks, const int64_t* __restrict__ spec_list, uint32_t spec_cap, SpecRes* __restrict__ spec_res,
    int2* __restrict__ spec_ev) {
    const int64_t pb = P.per_batch;
    const bool shortcuts = P.min_num_instances == 3;
    const int lane = threadIdx.x & 63;
    const uint64_t below = (1ull << lane) - 1;
    __shared__ int32_t s_list[kWalkThreads];
    __shared__ uint32_t s_cnt;
    __shared__ uint64_t img[kWalkThreads / 64][kClsWords + 2];
    __shared__ double s_tile[kWalkThreads / 64][kTileScratch];
    if ((int)blockIdx.x < spec_blocks) {
        // ---- spec role
        const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const uint32_t n_spec = min(__atomic_load_n(ctr + 3, __ATOMIC_RELAXED), spec_cap);
        const uint32_t n_waves = (uint32_t)spec_blocks * (kWalkThreads / 64);
        const double inv_nb = 1.0 / (double)nb;
        for (uint32_t k = blockIdx.x * (kWalkThreads / 64) + wv; k < n_spec; k += n_waves) {
            const int64_t t = spec_list[k];
            const int64_t sid = item_stream(t, nb, inv_nb);
            const int64_t j0 = t - sid * nb + 1;
            Det c;
            load_end_state(c, pend1 + 3 * t);
            ChainImg im{-((int64_t)1 << 40), 0};
            int32_t status = 3, nev = 0;
            int64_t j = j0;
            for (; j < nb && j < j0 + kSpecBatches; ++j) {
                int cp = -1;
                const int2 e = chain_batch(c, sid, j, err, L, pb, P.min_num_instances, P.warning_level,
                                           P.out_control_level, pmap, img[wv], s_tile[wv], im, cp);
                if (lane == 0) spec_ev[(int64_t)k * kSpecBatches + (j - j0)] = e;
                nev += (e.x >= 0 || e.y >= 0) ? 1 : 0;
                if (cp >= 0) {
                    status = 1;
                    break;
                }
            }
            if (status != 1 && j >= nb) {
                status = 2;
                j = nb - 1;
            }
            if (lane == 0) {
                SpecRes r;
                r.d = c;
                r.end_j = j;
                r.status = status;
                r.nev = nev;
                spec_res[k] = r;
            }
        }
        return;
    }
    // ---- walk role
    const int64_t wblk = (int64_t)blockIdx.x - spec_blocks;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    const int64_t t = wblk * kWalkThreads + threadIdx.x;
    if (t < n_streams) {
        const ddm_state st = state[t];
        if (need[t] == 0u && state_fresh(st)) {
            // a fresh carry-in and a change in every batch: the speculation is the result,
            // the reset state and nb batches with an event
            if (nb > 0) {
                ddm_state f;
                f.miss_prob = 1.0;
                f.miss_std = 0.0;
                f.miss_prob_min = f.miss_sd_min = f.miss_prob_sd_min = __builtin_huge_val();
                f.sample_count = 1;
                f.in_concept_change = 0;
                f.in_warning_zone = 0;
                state[t] = f;
            }
            if (nev_out) nev_out[t] = nb;
        } else {
            s_list[atomicAdd(&s_cnt, 1u)] = (int32_t)(t - wblk * kWalkThreads);
        }
    }
    __syncthreads();
    // the block's other streams, packed onto its first lanes
    const uint32_t cnt = s_cnt;
    if ((threadIdx.x & ~63u) >= cnt) return;
    bool defer = false;
    Walk W;
    if (threadIdx.x < cnt) {
        const int64_t u = wblk * kWalkThreads + s_list[threadIdx.x];
        W.sid = u;
        load_det(W.d, state[u]);
        W.j = W.wbase = W.nev = 0;
        W.chg_m = nb > 0 ? change_window(flags + u * nbp, 0, nb, W.st_m, W.ev_m, W.lm) : 0;
        walk_open(W, L, nb, nbp, pb, shortcuts, ev, flags, pmap, pend, ev1, flags1, pend1);
        if (W.j >= nb) {
            state[u] = store_det(W.d);
            if (nev_out) nev_out[u] = W.nev;
        } else {
            defer = true;
        }
    }
    const uint64_t dm = __ballot(defer);
    if (dm) {
        uint32_t base = 0;
        const int lead = __builtin_ctzll(dm);
        if (lane == lead) base = atomicAdd(ctr + 2, (uint32_t)__popcll(dm));
        base = __shfl(base, lead);
        if (defer) {
            FixEntry e;
            e.d = W.d;
            e.sid = W.sid;
            e.j = W.j;
            e.nev = W.nev;
            e.lvl1 = W.lvl1;
            coop[base + __popcll(dm & below)] = e;
        }
    }
}

// 4b. The fix-up: one wave per stream the walker handed over.  Where a carried run starts
// after an unchanged level-1 batch t (the walk stopped there, or got there again after a
// change), the spec blocks' run for t is taken as it stands (its event records copied);
// otherwise, or past a cut run, the batches run from the carried detector here (chain_batch:
// the stream's bytes 64 batches at a time in the wave's LDS image, rows through wave_tile),
// and walk_open skips what the flag bytes and records decide in between.
constexpr int kChainThreads = 256;

__global__ __launch_bounds__(kChainThreads) void k_scan_batches_chain(
    const uint8_t* __restrict__ err, int64_t L, int64_t nb, int64_t nbp, ddm_params P,
    ddm_state* __restrict__ state, int2* __restrict__ ev, const uint8_t* __restrict__ flags,
    int64_t* __restrict__ nev_out, const uint8_t* __restrict__ pmap, const FixEntry* __restrict__ coop,
    const uint32_t* __restrict__ ctr, const double2* __restrict__ pend, const int2* __restrict__ ev1,
    const uint8_t* __restrict__ flags1, const double2* __restrict__ pend1, const int32_t* __restrict__ sidx,
    const SpecRes* __restrict__ spec_res, const int2* __restrict__ spec_ev, uint64_t* __restrict__ cprof) {
    __shared__ uint64_t img[kChainThreads / 64][kClsWords + 2];
    __shared__ double s_tile[kChainThreads / 64][kTileScratch];
    const int64_t pb = P.per_batch;
    const int min_inst = P.min_num_instances;
    const double wl = P.warning_level, cl = P.out_control_level;
    const bool shortcuts = min_inst == 3;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t n_list = __atomic_load_n(ctr + 2, __ATOMIC_RELAXED);
    const uint32_t n_waves = gridDim.x * (kChainThreads / 64);
#ifdef DDM_TUNING
    // per-wave profile (tuning builds, DDM_CHAIN_PROF): start / end on the 100 MHz clock,
    // streams taken, rows run through wave_tile here (spec runs taken count none)
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    uint64_t p_streams = 0, p_rows = 0;
#endif
    for (uint32_t k = blockIdx.x * (kChainThreads / 64) + wv; k < n_list; k += n_waves) {
#ifdef DDM_TUNING
        ++p_streams;
#endif
        const FixEntry e = coop[k];
        Walk W;
        W.d = e.d;
        W.sid = e.sid;
        W.j = e.j;
        W.nev = e.nev;
        W.wbase = W.j & ~(int64_t)63;
        W.chg_m = change_window(flags + W.sid * nbp, W.wbase, nb, W.st_m, W.ev_m, W.lm);
        ChainImg im{-((int64_t)1 << 40), 0};
        int64_t lv = e.lvl1;                   // the walk stopped after this level-1 batch
        for (;;) {
            if (lv < 0) {
                walk_open(W, L, nb, nbp, pb, shortcuts, ev, flags, pmap, pend, ev1, flags1, pend1);
                if (W.j >= nb) break;
                lv = W.lvl1;
            }
            const int32_t sk = lv >= 0 ? sidx[lv] : -1;
            lv = -1;
            if (sk >= 0) {
                // the run carried on after the level-1 batch, computed ahead from the same
                // detector (pend1[t]): its records, then where it ended
                const SpecRes r = spec_res[sk];
                const int64_t j0 = W.j;
                const int64_t last = r.status == 3 ? r.end_j - 1 : r.end_j;
                for (int64_t b = j0 + lane; b <= last; b += 64)
                    ev[W.sid * nb + b] = spec_ev[(int64_t)sk * kSpecBatches + (b - j0)];
                W.nev += r.nev;
                if (r.status == 1) {
                    det_reset(W.d);            // DDM dropped (DDM_Process.py:209)
                    W.j = r.end_j + 1;
                } else {
                    W.d = r.d;
                    W.j = r.status == 2 ? nb : r.end_j;
                }
                if (W.j >= nb) break;
                if (r.status == 1) continue;   // fresh again: walk_open from there
            }
            // the batch W.j from the carried detector, here
            const int64_t j = W.j;
            Det c = W.d;
            int cp = -1;
            const int2 evj = chain_batch(c, W.sid, j, err, L, pb, min_inst, wl, cl, pmap, img[wv], s_tile[wv], im, cp);
#ifdef DDM_TUNING
            p_rows += (uint64_t)min(pb, L - j * pb);
#endif
            if (lane == 0) ev[W.sid * nb + j] = evj;
            W.nev += (evj.x >= 0 || evj.y >= 0);
            if (cp >= 0) det_reset(c);             // DDM dropped (DDM_Process.py:209)
            W.d = c;
            W.j = j + 1;
            if (W.j >= nb) break;
        }
        if (lane == 0) {
            state[W.sid] = store_det(W.d);
            if (nev_out) nev_out[W.sid] = W.nev;
        }
    }
#ifdef DDM_TUNING
    if (cprof) {
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        const uint32_t wid = blockIdx.x * (kChainThreads / 64) + wv;
        if (lane == 0) {
            uint64_t* const r = cprof + 4 * (uint64_t)wid;
            r[0] = t_start;
            r[1] = t_end;
            r[2] = p_streams;
            r[3] = p_rows;
        }
    }
#else
    (void)cprof;
#endif
}

// Scratch: counters, the fix-up list, flag bytes, the per-wave queues and the end states /
// level-1 records of unchanged batches (written sparsely, indexed by item).
constexpr int64_t kMaxWaves = 1 << 14;

struct BatchScratch {
    uint32_t* ctr;      // [2] streams handed to the chain kernel, [3] spec-list entries
    uint32_t* need;     // [n_streams]
    FixEntry* coop;     // [n_streams] streams the walker hands to the fix-up kernel
    uint8_t* flags;     // [n_streams * nbp], 64-byte aligned rows
    uint8_t* flags1;    // [n_items]
    int2* ev1;          // [n_items]
    double2* pend;      // [n_items][3]
    double2* pend1;     // [n_items][3]
    QEntry* q;          // [n_items + 64 * (kMaxWaves + 1)]: the waves' queues, qcap slots each
    int64_t* q1;        // [n_items + 64 * (kMaxWaves + 1)]
    uint32_t* qcnt;     // [kMaxWaves]
    uint32_t* q1cnt;    // [kMaxWaves]
    double4* pst;       // [kPreN]
    uint16_t* ptab;     // [kPreN]
    int64_t* spec_list; // [spec_cap] unchanged level-1 batches whose carried run is computed ahead
    int32_t* sidx;      // [n_items] spec-list index of an unchanged level-1 batch (-1: none, list full)
    SpecRes* spec_res;  // [spec_cap]
    int2* spec_ev;      // [spec_cap][kSpecBatches]
    uint32_t spec_cap;
    uint64_t* cprof;    // tuning builds: the chain kernel's per-wave profile [kChainProfWaves][4] (the scratch's end)
    int64_t bytes;
};
constexpr int64_t kChainProfWaves = 2048 * 4;

BatchScratch batch_scratch(void* base, int64_t n_streams, int64_t nb) {
    const auto up = [](int64_t x) { return (x + 255) & ~(int64_t)255; };
    const int64_t nbp = ddm::ceil_div(nb, 64) * 64;
    const int64_t n_items = n_streams * nb, nq = n_items + 64 * (kMaxWaves + 1);
    int64_t o = 256;
    const auto take = [&](int64_t bytes) {
        const int64_t at = o;
        o += up(bytes);
        return at;
    };
    const int64_t o_need = take(4 * n_streams), o_flags = take(n_streams * nbp);
    const int64_t o_coop = take((int64_t)sizeof(FixEntry) * n_streams);
    const int64_t o_flags1 = take(n_items), o_ev1 = take(8 * n_items), o_pend = take(48 * n_items);
    const int64_t o_pend1 = take(48 * n_items), o_q = take((int64_t)sizeof(QEntry) * nq), o_q1 = take(8 * nq);
    const int64_t o_qcnt = take(4 * kMaxWaves), o_q1cnt = take(4 * kMaxWaves), o_pst = take(32 * (int64_t)kPreN);
    const int64_t o_ptab = take(2 * (int64_t)kPreN);
    const int64_t spec_cap = std::min<int64_t>((int64_t)1 << 17, std::max<int64_t>(1, n_items));
    const int64_t o_slist = take(8 * spec_cap), o_sidx = take(4 * std::max<int64_t>(1, n_items));
    const int64_t o_sres = take((int64_t)sizeof(SpecRes) * spec_cap), o_sev = take(8 * kSpecBatches * spec_cap);
#ifdef DDM_TUNING
    const int64_t o_cprof = take(32 * kChainProfWaves);
#endif
    uint8_t* b = static_cast<uint8_t*>(base);
    BatchScratch sc;
    sc.ctr = reinterpret_cast<uint32_t*>(b);
    sc.need = reinterpret_cast<uint32_t*>(b + o_need);
    sc.coop = reinterpret_cast<FixEntry*>(b + o_coop);
    sc.flags = b + o_flags;
    sc.flags1 = b + o_flags1;
    sc.ev1 = reinterpret_cast<int2*>(b + o_ev1);
    sc.pend = reinterpret_cast<double2*>(b + o_pend);
    sc.pend1 = reinterpret_cast<double2*>(b + o_pend1);
    sc.q = reinterpret_cast<QEntry*>(b + o_q);
    sc.q1 = reinterpret_cast<int64_t*>(b + o_q1);
    sc.qcnt = reinterpret_cast<uint32_t*>(b + o_qcnt);
    sc.q1cnt = reinterpret_cast<uint32_t*>(b + o_q1cnt);
    sc.pst = reinterpret_cast<double4*>(b + o_pst);
    sc.ptab = reinterpret_cast<uint16_t*>(b + o_ptab);
    sc.spec_list = reinterpret_cast<int64_t*>(b + o_slist);
    sc.sidx = reinterpret_cast<int32_t*>(b + o_sidx);
    sc.spec_res = reinterpret_cast<SpecRes*>(b + o_sres);
    sc.spec_ev = reinterpret_cast<int2*>(b + o_sev);
    sc.spec_cap = (uint32_t)spec_cap;
#ifdef DDM_TUNING
    sc.cprof = getenv("DDM_CHAIN_PROF") ? reinterpret_cast<uint64_t*>(b + o_cprof) : nullptr;
#else
    sc.cprof = nullptr;
#endif
    sc.bytes = o;
    return sc;
}

// Tuning knobs read from the environment exist only in a tuning build (-DDDM_TUNING,
// tools/build_variant.sh); the production library always runs the defaults.
int env_int(const char* name, int dflt) {
#ifdef DDM_TUNING
    const char* e = getenv(name);
    return e ? atoi(e) : dflt;
#else
    (void)name;
    return dflt;
#endif
}

// Waves of the classify pass: one resident round (every wave owns an equal item range and
// streams through it), from the kernel's occupancy on this device.
int64_t classify_waves() {
    static const int64_t w = [] {
        const int over = env_int("DDM_SCAN_WAVES", 0);
        if (over > 0) return (int64_t)std::min<int64_t>(over, kMaxWaves);
        int dev = 0, cus = 256, per_cu = 8;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_scan_batches_classify<false, 7>, kClsThreads, 0) !=
                hipSuccess ||
            per_cu <= 0)
            per_cu = 8;
        return std::min<int64_t>((int64_t)cus * per_cu * (kClsThreads / 64), kMaxWaves / 4 * 4);
    }();
    return w;
}

}  // namespace

extern "C" int64_t ddm_scan_batches_scratch_bytes(int64_t n_streams, int64_t stream_len, int32_t per_batch) {
    if (n_streams < 0 || stream_len < 0 || per_batch <= 0) return -1;
    return batch_scratch(nullptr, n_streams, ddm::ceil_div(stream_len, per_batch)).bytes;
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
    const int64_t nb = ddm::ceil_div(stream_len, prm->per_batch);
    const int64_t nbp = ddm::ceil_div(nb, 64) * 64;
    const int64_t n_items = n_streams * nb;
    if (n_streams == 0) return 0;
    const BatchScratch sc = batch_scratch(scratch, n_streams, nb);
    hipStream_t s = ddm::as_hip(stream);
    static const int ex_refill = std::max(1, std::min(64, env_int("DDM_EXACT_REFILL", 24)));
    static const int fix_blocks_max = env_int("DDM_FIX_BLOCKS", 2048);
    static const int spec_blocks_max = std::max(0, env_int("DDM_SPEC_BLOCKS", 2048));
    static const bool use_pre = env_int("DDM_SCAN_PRE", 1) != 0;
    static const int cls_steps = std::max(0, env_int("DDM_SCAN_STEPS", 2));
    static const int cls_pop = std::max(1, std::min(64, env_int("DDM_SCAN_POP", 16)));
    if (ev_begin)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_begin), s), "event record")) return rc;
    if (int rc = ddm::hip_status(hipMemsetAsync(scratch, 0, (size_t)(256 + ((4 * n_streams + 255) & ~255)), s),
                                 "ddm_scan_batches: memset"))
        return rc;
    if (n_items > 0) {
        // whole workgroups of waves, each with a queue of qcap slots (its fills' items)
        const int64_t nfill = ddm::ceil_div(n_items, 64);
        const int64_t blocks = ddm::ceil_div(std::min<int64_t>(classify_waves(), nfill), kClsThreads / 64);
        const int64_t qcap = ddm::ceil_div(nfill, blocks * (kClsThreads / 64)) * 64;
        // the prefix table is built whatever the batch length (the classify pass reads it
        // unconditionally) and used when batches have at least kPre rows
        const bool pre = use_pre && prm->per_batch >= kPre;
        hipLaunchKernelGGL(k_scan_prefix_table, dim3(kPreN / 256), dim3(256), 0, s, *prm, sc.pst, sc.ptab);
        if (int rc = ddm::launch_status("ddm_scan_batches/prefix")) return rc;
        int2* ev = reinterpret_cast<int2*>(ev_out);
        // 16-byte chunks per fill: (63 * pb + 128 + 15) / 16 + 1, per 64 lanes
        const bool small = prm->per_batch <= 100;
        const auto cls = perm_map ? (small ? k_scan_batches_classify<true, 7> : k_scan_batches_classify<true, kClsLoads>)
                                  : (small ? k_scan_batches_classify<false, 7> : k_scan_batches_classify<false, kClsLoads>);
#ifdef DDM_TUNING
        static const bool probe = env_int("DDM_SCAN_PROBE", 0) != 0;
        if (probe)
        {
            static const int pm = env_int("DDM_SCAN_PROBE", 0);
            const auto pk = pm == 2 ? k_scan_batches_probe<7, 1>
                          : pm == 3 ? k_scan_batches_probe<7, 2> : k_scan_batches_probe<7, 0>;
            hipLaunchKernelGGL(pk, dim3((unsigned)blocks), dim3(kClsThreads), 0, s, err, n_items, stream_len, nb, nbp,
                               *prm, ev, sc.qcnt, sc.q1cnt);
        }
        else
#endif
            hipLaunchKernelGGL(cls, dim3((unsigned)blocks), dim3(kClsThreads), 0, s, err, n_items, stream_len, nb,
                               nbp, *prm, ev, sc.flags, perm_map, qcap, sc.need, pre, sc.ptab, sc.pst, sc.q,
                               sc.qcnt, sc.q1, sc.q1cnt, sc.pend, cls_steps, cls_pop);
        if (int rc = ddm::launch_status("ddm_scan_batches/classify")) return rc;
        const auto ex0 = perm_map ? k_scan_batches_exact<0, true> : k_scan_batches_exact<0, false>;
        const auto ex1 = perm_map ? k_scan_batches_exact<1, true> : k_scan_batches_exact<1, false>;
        hipLaunchKernelGGL(ex0, dim3((unsigned)blocks), dim3(kExThreads), 0, s, err, n_items, stream_len, nb, nbp, *prm, ev,
                           sc.flags, perm_map, qcap, sc.need, sc.q, sc.qcnt, sc.q1, sc.q1cnt,
                           sc.pend, sc.ev1, sc.flags1, sc.pend1, ex_refill, sc.ctr, sc.spec_list, sc.sidx, sc.spec_cap);
        if (int rc = ddm::launch_status("ddm_scan_batches/exact")) return rc;
        hipLaunchKernelGGL(ex1, dim3((unsigned)blocks), dim3(kExThreads), 0, s, err, n_items, stream_len, nb, nbp, *prm, ev,
                           sc.flags, perm_map, qcap, sc.need, sc.q, sc.qcnt, sc.q1, sc.q1cnt,
                           sc.pend, sc.ev1, sc.flags1, sc.pend1, ex_refill, sc.ctr, sc.spec_list, sc.sidx, sc.spec_cap);
        if (int rc = ddm::launch_status("ddm_scan_batches/exact1")) return rc;
    }
    // the speculative carried runs' workgroups first in the grid (dispatched first), then the walk's
    const int spec_blocks =
        n_items > 0 ? (int)std::min<int64_t>(spec_blocks_max, ddm::ceil_div((int64_t)sc.spec_cap, kWalkThreads / 64)) : 0;
    hipLaunchKernelGGL(k_scan_batches_walk, dim3((unsigned)(spec_blocks + ddm::ceil_div(n_streams, kWalkThreads))),
                       dim3(kWalkThreads), 0, s, err, n_streams, stream_len, nb, nbp, *prm, state_io,
                       reinterpret_cast<int2*>(ev_out), sc.flags, nev_out, perm_map, sc.need, sc.ctr, sc.pend, sc.ev1,
                       sc.flags1, sc.pend1, sc.coop, spec_blocks, sc.spec_list, sc.spec_cap, sc.spec_res, sc.spec_ev);
    if (int rc = ddm::launch_status("ddm_scan_batches/walk")) return rc;
    const int64_t fix_blocks =
        std::max<int64_t>(1, std::min<int64_t>(sc.cprof ? std::min(fix_blocks_max, 2048) : fix_blocks_max,
                                               ddm::ceil_div(n_streams, kChainThreads / 64)));
    hipLaunchKernelGGL(k_scan_batches_chain, dim3((unsigned)fix_blocks), dim3(kChainThreads), 0, s, err, stream_len,
                       nb, nbp, *prm, state_io, reinterpret_cast<int2*>(ev_out), sc.flags, nev_out, perm_map,
                       sc.coop, sc.ctr, sc.pend, sc.ev1, sc.flags1, sc.pend1, sc.sidx, sc.spec_res, sc.spec_ev,
                       sc.cprof);
    if (ev_end)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_end), s), "event record")) return rc;
    return ddm::launch_status("ddm_scan_batches");
}
