// Wave-cooperative exact DDM rows (used by scan_long.hip and the fix-up of ddm_scan.hip).
//
// run_DDM's detector (det.h, DDM_Process.py:135-159) over a tile of up to 64 rows whose
// error bits are m, by all 64 lanes of a wave holding the same detector:
//   * the p recurrence p += (x - p) / n is the only sequential part: the wave runs it once
//     (5 dependent fp64 operations per row; n and RN(1/n) of every row come from LDS by
//     broadcast reads issued ahead of the chain), and lane k keeps p_k;
//   * s_k, the running arg-min of p + s (an inclusive wave scan, the later row on ties: the
//     reference's `<=`), the change and warning tests and their ballots are lane-parallel.
// The detector comes back as it stands after the last committed row: the first change,
// or the tile's last row.  Bit for bit the sequential det_add_fast.
#pragma once
#include "det.h"

namespace {

__device__ __forceinline__ double shfl_d(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __shfl((int)b, src, 64);
    const int hi = __shfl((int)(b >> 32), src, 64);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// One step of the wave's inclusive arg-min scan of (value, index) through DPP: the pair
// from the lane kCtrl names (row_shr:n, or row_bcast:15/31 into the rows of kRowMask) is
// taken when it is valid and strictly smaller (ties keep the later row: the reference's
// `<=` minimum).  Lanes without a source get the identity (+inf, -1).
template <int kCtrl, int kRowMask>
__device__ __forceinline__ void argmin_step(double& v, int& idx) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, kCtrl, kRowMask, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0x7ff00000, (int)(b >> 32), kCtrl, kRowMask, 0xF, false);
    const int oi = __builtin_amdgcn_update_dpp(-1, idx, kCtrl, kRowMask, 0xF, false);
    const double ov = __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
    if (oi >= 0 && (idx < 0 || !(v <= ov))) {
        v = ov;
        idx = oi;
    }
}

__device__ __forceinline__ double readlane_d(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, src);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

struct TileOut {
    int kc;          // first change row of the tile or -1
    int last;        // last committed row (kc, or cnt - 1)
    uint64_t warn;   // rows with in_warning_zone set (committed rows only are meaningful)
};

// sc: this wave's LDS scratch of kTileScratch doubles (n, RN(1/n), x and p of every row).
// d must be uniform over the wave and not in a pending change (the caller resets it first);
// rows >= cnt are ignored.
constexpr int kTileScratch = 4 * 64;

__device__ __forceinline__ TileOut wave_tile(Det& d, uint64_t m, int cnt, int min_inst, double wl, double cl,
                                             double* sc) {
    const int lane = threadIdx.x & 63;
    if (cnt < 64) m &= (1ull << cnt) - 1;
    if (det_trivial(d) && m == 0) {                 // zeros in the trivial state: only n moves
        d.n += cnt;
        d.warn = 0;
        return {-1, cnt - 1, 0ull};
    }
    double* const s_n = sc;
    double* const s_r = sc + 64;
    double* const s_x = sc + 128;
    double* const s_p = sc + 192;
    const double nl = (double)d.n + (double)lane;   // divisor of row lane
    const double rl = 1.0 / nl;                     // RN(1/n), as det_add_fast's rcp[] / 1.0 / n
    // rows past cnt get n = 1, 1/n = 0: their step adds exactly 0 to p
    s_n[lane] = lane < cnt ? nl : 1.0;
    s_r[lane] = lane < cnt ? rl : 0.0;
    s_x[lane] = (double)((m >> lane) & 1ull);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the chain, 8 rows at a time: 5 dependent fp64 operations per row, the group's operands
    // read from LDS (broadcast) ahead of it, its p values written back by one lane after it
    double p = d.p;
    for (int k0 = 0; k0 < cnt; k0 += 8) {
        double xs[8], ns[8], rs[8], ps[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            xs[u] = s_x[k0 + u];
            ns[u] = s_n[k0 + u];
            rs[u] = s_r[k0 + u];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            p = p + div_rn(xs[u] - p, ns[u], rs[u]);
            ps[u] = p;
        }
        if (lane == 0) {
#pragma unroll
            for (int u = 0; u < 8; ++u) s_p[k0 + u] = ps[u];
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const double myp = lane < cnt ? s_p[lane] : 0.0;
    const double s = sqrt_q(div_rn(myp * (1.0 - myp), nl, rl));
    const bool gated = lane < cnt && (d.n + lane + 1 >= (int64_t)min_inst);
    const double ps = myp + s;
    double mps = gated ? ps : __builtin_huge_val();
    int midx = gated ? lane : -1;
    // inclusive arg-min scan: rows of 16 by row_shr 1/2/4/8, then across rows by row_bcast
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

}  // namespace
