// DDM detector arithmetic shared by the scan kernels (ddm_scan.hip, scan_long.hip):
// scikit-multiflow's DDM.add_element (used at DDM_Process.py:133-159)
// in fp64 with contraction off (-ffp-contract=off), plus the exact cheaper forms of its
// division and square root that the production kernels use.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

struct Det {
    double p, s, pmin, smin, psmin;
    int64_t n;
    int chg, warn;
};

__device__ __forceinline__ void det_reset(Det& d) {
    d.p = 1.0;
    d.s = 0.0;
    d.pmin = d.smin = d.psmin = __builtin_huge_val();
    d.n = 1;
    d.chg = 0;
    d.warn = 0;
}

// skmultiflow DDM.add_element (restated in SURVEY.md Appendix A).
__device__ __forceinline__ void det_add(Det& d, int x, int min_inst, double wl, double cl) {
    if (d.chg) det_reset(d);
    const double n = (double)d.n;
    const double p = d.p + ((double)x - d.p) / n;
    const double s = sqrt(p * (1.0 - p) / n);
    d.p = p;
    d.s = s;
    d.n += 1;
    d.chg = 0;
    d.warn = 0;
    if (d.n < min_inst) return;
    const double ps = p + s;
    if (ps <= d.psmin) {
        d.pmin = p;
        d.smin = s;
        d.psmin = ps;
    }
    if (ps > d.pmin + cl * d.smin) d.chg = 1;
    else if (ps > d.pmin + wl * d.smin) d.warn = 1;
}

// Every error so far was 0 and the gate has set the minimum: adding a 0 keeps
// (p, s, p_min, s_min, ps_min) = 0 and raises no flag.
__device__ __forceinline__ bool det_trivial(const Det& d) {
    return d.p == 0.0 && d.psmin == 0.0 && d.pmin == 0.0 && d.smin == 0.0 && d.chg == 0;
}

constexpr int kRcpN = 4096;

__device__ __forceinline__ double div_rn(double a, double n, double r) {
    const double q0 = a * r;
    const double e = __builtin_fma(-q0, n, a);
    return __builtin_fma(e, r, q0);
}

// sqrt for the DDM's q = p(1-p)/n: the operation sequence of the compiler's correctly
// rounded f64 sqrt (rsq seed, Goldschmidt step, two Newton corrections) without its
// denormal-range scaling and its inf check.  The scaling is the identity for
// q >= 2^-767 and q is either 0 or far above that (p and 1-p are 0 or >= 1/n with
// n < 2^63, so q >= 2^-190); q == 0 gives 0 as sqrt does.  Bit-identical to sqrt(q) on
// that domain (the scan parity tests compare with the C oracle's libm sqrt).
__device__ __forceinline__ double sqrt_q(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y;
    double h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    return x == 0.0 ? x : g;
}

__device__ __forceinline__ void det_add_fast(Det& d, int x, int min_inst, double wl, double cl,
                                             const double* __restrict__ rcp) {
    if (d.chg) det_reset(d);
    const double n = (double)d.n;
    const double r = d.n < kRcpN ? rcp[d.n] : 1.0 / n;
    const double p = d.p + div_rn((double)x - d.p, n, r);
    const double s = sqrt_q(div_rn(p * (1.0 - p), n, r));
    d.p = p;
    d.s = s;
    d.n += 1;
    d.chg = 0;
    d.warn = 0;
    if (d.n < min_inst) return;
    const double ps = p + s;
    if (ps <= d.psmin) {
        d.pmin = p;
        d.smin = s;
        d.psmin = ps;
    }
    if (ps > d.pmin + cl * d.smin) d.chg = 1;
    else if (ps > d.pmin + wl * d.smin) d.warn = 1;
}

__device__ __forceinline__ bool det_fresh(const Det& d) {
    return d.chg || (d.n == 1 && d.p == 1.0 && d.s == 0.0 && d.psmin == __builtin_huge_val() &&
                     d.pmin == __builtin_huge_val() && d.smin == __builtin_huge_val());
}

}  // namespace
