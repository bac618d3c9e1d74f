// MT19937 jump-ahead polynomials (host): x^(k*J) mod phi(x), k = 1..n, where phi is the
// characteristic polynomial of MT19937's state transition T (degree 19937).
//
// Why: each partition consumes ONE MT19937 stream (numpy's global RandomState,
// DDM_Process.py:187, :190, :102), ~1.4 draws per row.  Generated front to back that
// stream is a sequential recurrence per partition (one workgroup, the floor of a C3 step).
// T is linear over GF(2), so T^(kJ) = g_k(T) with g_k = x^(kJ) mod phi (Cayley-Hamilton);
// ddm_mt_jump (shuffle.hip) applies g_k to the partition's start state on the device
// (Horner), and the segments [kJ, (k+1)J) of the stream are then generated in parallel.
//
// phi is recovered once per process by Berlekamp-Massey from bit 0 of 2 * 19937 outputs
// of a seeded generator (the minimal polynomial of any nonzero linear output sequence of
// MT19937 is phi: it is irreducible).  Polynomials are bit vectors over 64-bit words,
// bit i = coefficient of x^i.
#include <stdint.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "../../include/ddm_amd.h"

namespace {

constexpr int kMexp = 19937;
constexpr int kW = DDM_MT_POLY_WORDS;                 // words of a reduced polynomial (deg < kMexp)
static_assert(kW * 64 >= kMexp, "poly words");
using Poly = std::vector<uint64_t>;

inline int bit(const Poly& p, int64_t i) { return (int)((p[(size_t)(i >> 6)] >> (i & 63)) & 1u); }
inline void flip(Poly& p, int64_t i) { p[(size_t)(i >> 6)] ^= 1ull << (i & 63); }

// dst ^= src << sh (word vectors; dst must be long enough)
void xor_shifted(Poly& dst, const Poly& src, int64_t sh, size_t src_words) {
    const int64_t ws = sh >> 6;
    const int bs = (int)(sh & 63);
    for (size_t k = 0; k < src_words; ++k) {
        const uint64_t v = src[k];
        if (!v) continue;
        dst[(size_t)ws + k] ^= v << bs;
        if (bs && (size_t)ws + k + 1 < dst.size()) dst[(size_t)ws + k + 1] ^= v >> (64 - bs);
    }
}

// bit 0 of successive tempered outputs of init_genrand(5489)
std::vector<uint8_t> output_bits(int n) {
    uint32_t mt[624];
    mt[0] = 5489u;
    for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    int pos = 624;
    std::vector<uint8_t> out((size_t)n);
    for (int k = 0; k < n; ++k) {
        if (pos == 624) {
            for (int i = 0; i < 624; ++i) {
                const uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % 624] & 0x7fffffffu);
                mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
            }
            pos = 0;
        }
        uint32_t y = mt[pos++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        out[(size_t)k] = (uint8_t)(y & 1u);
    }
    return out;
}

// Berlekamp-Massey over GF(2): connection polynomial C (c_0 = 1) of the sequence; the
// characteristic polynomial is its reciprocal x^L C(1/x).
Poly charpoly() {
    const int N = 2 * kMexp + 64;
    const std::vector<uint8_t> s = output_bits(N);
    const size_t W = (size_t)(N / 64 + 2);
    // rev[k] = s[N-1-k] packed, so sum_i c_i s[n-i] = parity(C & rev >> (N-1-n))
    Poly rev(W + 1, 0);
    for (int k = 0; k < N; ++k)
        if (s[(size_t)(N - 1 - k)]) rev[(size_t)k >> 6] |= 1ull << (k & 63);
    Poly C(W + 1, 0), B(W + 1, 0), T;
    C[0] = B[0] = 1;
    int L = 0, m = 1;
    for (int n = 0; n < N; ++n) {
        const int64_t off = (int64_t)(N - 1 - n);
        const int64_t ow = off >> 6;
        const int ob = (int)(off & 63);
        uint64_t acc = 0;
        const size_t cw = (size_t)(L / 64 + 1);
        for (size_t k = 0; k < cw; ++k) {
            const size_t a = (size_t)ow + k;
            uint64_t r = a < rev.size() ? rev[a] >> ob : 0;
            if (ob && a + 1 < rev.size()) r |= rev[a + 1] << (64 - ob);
            acc ^= C[k] & r;
        }
        if (L % 64 != 63) {                     // only coefficients 0..L count
            const int top = L % 64;
            const uint64_t keep = top == 63 ? ~0ull : ((1ull << (top + 1)) - 1);
            const size_t k = (size_t)(L / 64);
            // undo the bits of word k above L
            const size_t a = (size_t)ow + k;
            uint64_t r = a < rev.size() ? rev[a] >> ob : 0;
            if (ob && a + 1 < rev.size()) r |= rev[a + 1] << (64 - ob);
            acc ^= C[k] & r & ~keep;
        }
        const int d = __builtin_parityll(acc);
        if (!d) {
            ++m;
        } else if (2 * L <= n) {
            T = C;
            xor_shifted(C, B, m, W + 1 - (size_t)((m >> 6) + 1));
            L = n + 1 - L;
            B = T;
            m = 1;
        } else {
            xor_shifted(C, B, m, W + 1 - (size_t)((m >> 6) + 1));
            ++m;
        }
    }
    Poly phi((size_t)kW + 1, 0);                // degree L = 19937 needs bit 19937
    for (int i = 0; i <= L; ++i)
        if (bit(C, i)) flip(phi, L - i);
    return L == kMexp ? phi : Poly();
}

struct Field {
    Poly phi;                                   // kW + 1 words, bit kMexp set
    std::vector<Poly> phi_sh;                   // phi << k, k = 0..63
};

// a * b mod phi, a and b reduced (kW words)
Poly mulmod(const Poly& a, const Poly& b, const Field& F) {
    std::vector<Poly> bsh(64, Poly((size_t)kW + 1, 0));
    for (int k = 0; k < 64; ++k) {
        for (int w = 0; w < kW; ++w) {
            bsh[k][(size_t)w] ^= b[(size_t)w] << k;
            if (k) bsh[k][(size_t)w + 1] ^= b[(size_t)w] >> (64 - k);
        }
    }
    Poly prod(2 * (size_t)kW + 2, 0);
    for (int w = 0; w < kW; ++w) {
        uint64_t v = a[(size_t)w];
        while (v) {
            const int k = __builtin_ctzll(v);
            v &= v - 1;
            const Poly& s = bsh[k];
            for (int u = 0; u <= kW; ++u) prod[(size_t)(w + u)] ^= s[(size_t)u];
        }
    }
    for (int64_t t = 2 * (int64_t)kMexp; t >= kMexp; --t) {
        if (!bit(prod, t)) continue;
        const int64_t sh = t - kMexp;
        const Poly& p = F.phi_sh[(size_t)(sh & 63)];
        const size_t base = (size_t)(sh >> 6);
        for (int u = 0; u <= kW; ++u)
            if (base + (size_t)u < prod.size()) prod[base + (size_t)u] ^= p[(size_t)u];
    }
    prod.resize((size_t)kW);
    return prod;
}

Poly x_pow_mod(uint64_t e, const Field& F) {
    Poly r((size_t)kW, 0), x((size_t)kW, 0);
    r[0] = 1;
    x[0] = 2;
    while (e) {                                 // right-to-left binary powering
        if (e & 1) r = mulmod(r, x, F);
        e >>= 1;
        if (e) x = mulmod(x, x, F);
    }
    return r;
}

std::mutex g_mu;
Field* g_field = nullptr;
struct JumpCache {
    int64_t J = 0;
    std::vector<Poly> g;                        // g[k] = x^((k+1) J) mod phi
};
JumpCache g_cache;

const Field* field() {
    if (!g_field) {
        Poly phi = charpoly();
        if (phi.empty()) return nullptr;
        Field* F = new Field;
        F->phi = phi;
        F->phi_sh.assign(64, Poly((size_t)kW + 2, 0));
        for (int k = 0; k < 64; ++k)
            for (int w = 0; w <= kW; ++w) {
                F->phi_sh[(size_t)k][(size_t)w] ^= phi[(size_t)w] << k;
                if (k) F->phi_sh[(size_t)k][(size_t)w + 1] ^= phi[(size_t)w] >> (64 - k);
            }
        g_field = F;
    }
    return g_field;
}

}  // namespace

extern "C" int ddm_mt_charpoly(uint64_t* out) {
    if (!out) return DDM_E_ARG;
    std::lock_guard<std::mutex> lk(g_mu);
    const Field* F = field();
    if (!F) return DDM_E_ARG;
    memcpy(out, F->phi.data(), sizeof(uint64_t) * ((size_t)kW + 1));
    return 0;
}

extern "C" int ddm_mt_jump_polys(int64_t jump, int32_t n, uint64_t* out) {
    if (jump <= 0 || n < 0 || (!out && n > 0)) return DDM_E_ARG;
    std::lock_guard<std::mutex> lk(g_mu);
    const Field* F = field();
    if (!F) return DDM_E_ARG;
    if (g_cache.J != jump) {
        g_cache.J = jump;
        g_cache.g.clear();
    }
    while ((int32_t)g_cache.g.size() < n) {
        if (g_cache.g.empty()) g_cache.g.push_back(x_pow_mod((uint64_t)jump, *F));
        else g_cache.g.push_back(mulmod(g_cache.g.back(), g_cache.g.front(), *F));
    }
    for (int32_t k = 0; k < n; ++k) memcpy(out + (size_t)k * kW, g_cache.g[(size_t)k].data(), sizeof(uint64_t) * kW);
    return 0;
}
