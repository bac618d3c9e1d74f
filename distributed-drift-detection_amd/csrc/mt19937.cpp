// Host MT19937 in numpy's legacy RandomState layout (key[624], pos).
//
// The reference draws every shuffle and every forest seed from numpy's global
// RandomState (DDM_Process.py:187, :190 via pandas `sample(frac=1)`, and :102 via
// RandomForestClassifier(random_state=None)).  Reproducing those draws exactly is
// what makes the GPU path's batch order — and therefore every event index —
// identical to the reference's.  Semantics (numpy/random/src/legacy + distributions):
//   permutation(n): x = arange(n); for i = n-1 .. 1: j = random_interval(i); swap
//   random_interval(m): mask = smallest 2^k-1 >= m; draw next_uint32 & mask until <= m
//   randint(2**31-1):   random_interval(2**31 - 2)
#include <stdint.h>
#include <string.h>

#include <immintrin.h>

#include <algorithm>

#include "../../include/ddm_amd.h"

namespace {

constexpr int kN = 624, kM = 397;

void regen(uint32_t* mt) {
    int i = 0;
    for (; i < kN - kM; ++i) {
        const uint32_t y = (mt[i] & 0x80000000u) | (mt[i + 1] & 0x7fffffffu);
        mt[i] = mt[i + kM] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
    }
    for (; i < kN - 1; ++i) {
        const uint32_t y = (mt[i] & 0x80000000u) | (mt[i + 1] & 0x7fffffffu);
        mt[i] = mt[i + (kM - kN)] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
    }
    const uint32_t y = (mt[kN - 1] & 0x80000000u) | (mt[0] & 0x7fffffffu);
    mt[kN - 1] = mt[kM - 1] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
}

struct Gen {
    uint32_t* key;
    int32_t pos;
    int64_t draws = 0;

    inline uint32_t next() {
        if (pos >= kN) {
            regen(key);
            pos = 0;
        }
        uint32_t y = key[pos++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        ++draws;
        return y;
    }

    inline uint32_t interval(uint32_t mx) {
        if (mx == 0) return 0;
        uint32_t mask = mx;
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        mask |= mask >> 8;
        mask |= mask >> 16;
        uint32_t v;
        while ((v = (next() & mask)) > mx) {
        }
        return v;
    }
};


// Permutation stream, fast path: the current 624-word block is tempered once into a
// buffer, and each Fisher-Yates interval finds its first accepted draw among the next 8
// buffered words with one AVX2 compare + movemask (no unpredictable branch on the
// ~25% rejections).  Draw-for-draw identical to Gen::interval.
struct PermGen {
    uint32_t* key;
    int32_t pos;
    alignas(32) uint32_t tb[kN];
    int64_t draws = 0;

    void temper_from(int from) {
        for (int i = from; i < kN; ++i) {
            uint32_t y = key[i];
            y ^= y >> 11;
            y ^= (y << 7) & 0x9d2c5680u;
            y ^= (y << 15) & 0xefc60000u;
            y ^= y >> 18;
            tb[i] = y;
        }
    }
    PermGen(uint32_t* k, int32_t p) : key(k), pos(p) {
        if (pos < kN) temper_from(pos);
    }
    inline void refill() {
        regen(key);
        temper_from(0);
        pos = 0;
    }
};

#define PERM_FN perms_scalar
#define PERM_AVX2 0
#include "perm_loop.inc"
#undef PERM_FN
#undef PERM_AVX2

#pragma GCC push_options
#pragma GCC target("avx2")
#define PERM_FN perms_avx2
#define PERM_AVX2 1
#include "perm_loop.inc"
#undef PERM_FN
#undef PERM_AVX2
#pragma GCC pop_options

}  // namespace

extern "C" int ddm_mt_perms(uint32_t* key, int32_t* pos, const int32_t* batch_len, int64_t n_batches,
                            uint8_t* perm_out, int64_t* draws_out) {
    if (!key || !pos || (!batch_len && n_batches) || (!perm_out && n_batches) || n_batches < 0 || *pos < 0 ||
        *pos > kN)
        return DDM_E_ARG;
    static const bool avx2 = __builtin_cpu_supports("avx2");
    return avx2 ? perms_avx2(key, pos, batch_len, n_batches, perm_out, draws_out)
                : perms_scalar(key, pos, batch_len, n_batches, perm_out, draws_out);
}

extern "C" int ddm_mt_randint31(uint32_t* key, int32_t* pos, int64_t count, int64_t* out) {
    if (!key || !pos || (!out && count) || count < 0 || *pos < 0 || *pos > kN) return DDM_E_ARG;
    Gen g{key, *pos};
    for (int64_t i = 0; i < count; ++i) out[i] = (int64_t)g.interval(0x7ffffffeu);
    *pos = g.pos;
    return 0;
}

// ABI 24: numpy's legacy RandomState(seed) for a 32-bit integer seed (the reference's
// per-partition np.random.seed, DDM_Process.py): init_genrand into the key, pos = 624.
// Constructing a RandomState in Python costs ~0.1 ms (it seeds a fresh bit generator from
// the OS first), paid per partition at every run's start.
extern "C" int ddm_mt_seed(uint32_t seed, uint32_t* key, int32_t* pos) {
    if (!key || !pos) return DDM_E_ARG;
    uint32_t x = seed;
    for (int i = 0; i < kN; ++i) {
        key[i] = x;
        x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)(i + 1);
    }
    *pos = kN;
    return 0;
}

extern "C" int ddm_mt_skip(uint32_t* key, int32_t* pos, int64_t n_draws) {
    if (!key || !pos || n_draws < 0 || *pos < 0 || *pos > kN) return DDM_E_ARG;
    Gen g{key, *pos};
    // whole blocks of 624 can be regenerated without tempering
    while (n_draws > 0) {
        if (g.pos >= kN) {
            regen(g.key);
            g.pos = 0;
        }
        const int64_t take = std::min<int64_t>(n_draws, kN - g.pos);
        g.pos += (int32_t)take;
        n_draws -= take;
    }
    *pos = g.pos;
    return 0;
}

// From already tempered words of the stream (a read-back of the device copy R): one
// batch's legacy permutation(L) followed by T randint(2**31-1) tree seeds — the draws a
// refit consumes (DDM_Process.py:190 then :102).  used[0] / used[1] = words taken by the
// shuffle / the seeds.  DDM_E_ARG when n_words runs out (read more words).
extern "C" int ddm_words_perm_seeds(const uint32_t* words, int64_t n_words, int32_t L, int32_t T,
                                    uint8_t* perm_out, int64_t* seeds_out, int64_t* used) {
    if (!words || !used || L < 0 || L > 256 || T < 0 || (L && !perm_out) || (T && !seeds_out)) return DDM_E_ARG;
    int64_t k = 0;
    for (int32_t i = 0; i < L; ++i) perm_out[i] = (uint8_t)i;
    for (int32_t i = L - 1; i >= 1; --i) {
        const uint32_t mask = 0xffffffffu >> __builtin_clz((uint32_t)i);
        uint32_t j;
        do {
            if (k >= n_words) return DDM_E_ARG;
            j = words[k++] & mask;
        } while (j > (uint32_t)i);
        const uint8_t t = perm_out[i];
        perm_out[i] = perm_out[j];
        perm_out[j] = t;
    }
    used[0] = k;
    for (int32_t t = 0; t < T; ++t) {
        uint32_t v;
        do {
            if (k >= n_words) return DDM_E_ARG;
            v = words[k++] & 0x7fffffffu;
        } while (v > 0x7ffffffeu);
        seeds_out[t] = (int64_t)v;
    }
    used[1] = k - used[0];
    return 0;
}
