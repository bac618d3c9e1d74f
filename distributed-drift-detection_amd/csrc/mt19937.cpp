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

}  // namespace

extern "C" int ddm_mt_perms(uint32_t* key, int32_t* pos, const int32_t* batch_len, int64_t n_batches,
                            uint8_t* perm_out, int64_t* draws_out) {
    if (!key || !pos || (!batch_len && n_batches) || (!perm_out && n_batches) || n_batches < 0 || *pos < 0 ||
        *pos > kN)
        return DDM_E_ARG;
    Gen g{key, *pos};
    uint8_t* out = perm_out;
    for (int64_t b = 0; b < n_batches; ++b) {
        const int32_t n = batch_len[b];
        if (n < 0 || n > 256) {
            *pos = g.pos;
            return DDM_E_ARG;
        }
        const int64_t d0 = g.draws;
        for (int32_t i = 0; i < n; ++i) out[i] = (uint8_t)i;
        for (int32_t i = n - 1; i >= 1; --i) {
            const uint32_t j = g.interval((uint32_t)i);
            const uint8_t t = out[i];
            out[i] = out[j];
            out[j] = t;
        }
        out += n;
        if (draws_out) draws_out[b] = g.draws - d0;
    }
    *pos = g.pos;
    return 0;
}

extern "C" int ddm_mt_randint31(uint32_t* key, int32_t* pos, int64_t count, int64_t* out) {
    if (!key || !pos || (!out && count) || count < 0 || *pos < 0 || *pos > kN) return DDM_E_ARG;
    Gen g{key, *pos};
    for (int64_t i = 0; i < count; ++i) out[i] = (int64_t)g.interval(0x7ffffffeu);
    *pos = g.pos;
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
