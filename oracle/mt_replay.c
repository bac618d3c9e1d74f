/* ORACLE — plain-C replay of run_DDM_loop's global MT19937 consumption.
 * TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
 *
 * The reference draws from ONE global numpy RandomState per worker:
 *   batch 0:   permutation(len(B0))                         DDM_Process.py:187
 *   batch j:   permutation(len(Bj))                         DDM_Process.py:190
 *              then, if a refit is pending, 100 x randint(2**31-1), one per tree
 *              (RandomForestClassifier(random_state=None).fit, :98-105, :194-196)
 *   a change in batch j makes the refit pending for batch j+1 (:207-210).
 * Legacy numpy semantics restated here:
 *   seed(s)        init_genrand(s), position 624
 *   next_u32       the standard MT19937 twist of the whole key + tempering
 *   permutation(n) arange(n) shuffled by Fisher-Yates for i = n-1 .. 1 with
 *                  j = next_u32 & mask(i), rejected while j > i (mask = 2^bitlen(i) - 1)
 *   randint(2^31-1) next_u32 & 0x7fffffff, rejected while == 0x7fffffff
 * Given where the changes are, the replay yields the shuffled order of any batch and the
 * final generator state, with no GPU code involved: the bench's configs[2] property check
 * uses it to pin the exact drift row (the first new-class row in shuffled order) and the
 * RNG position the drop-in hands back.
 *
 * Built into oracle/_build/libddm_oracle.so with ddm_scan.c (oracle/Makefile).
 */
#include <stdint.h>
#include <string.h>

#define MT_N 624
#define MT_M 397

typedef struct {
    uint32_t key[MT_N];
    int32_t pos;
} mt_state;

static void mt_seed(mt_state* s, uint32_t seed) {
    s->key[0] = seed;
    for (int i = 1; i < MT_N; ++i)
        s->key[i] = 1812433253u * (s->key[i - 1] ^ (s->key[i - 1] >> 30)) + (uint32_t)i;
    s->pos = MT_N;
}

static inline uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t m) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return m ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

static void mt_twist(mt_state* s) {
    uint32_t* k = s->key;
    int i = 0;
    for (; i < MT_N - MT_M; ++i) k[i] = mt_mix(k[i], k[i + 1], k[i + MT_M]);
    for (; i < MT_N - 1; ++i) k[i] = mt_mix(k[i], k[i + 1], k[i + MT_M - MT_N]);
    k[MT_N - 1] = mt_mix(k[MT_N - 1], k[0], k[MT_M - 1]);
    s->pos = 0;
}

static uint32_t mt_next(mt_state* s) {
    if (s->pos >= MT_N) mt_twist(s);
    uint32_t y = s->key[s->pos++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

static void mt_permutation(mt_state* s, int32_t n, int32_t* out) {
    for (int32_t i = 0; i < n; ++i) out[i] = i;
    for (int32_t i = n - 1; i >= 1; --i) {
        uint32_t mask = (uint32_t)i;
        mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
        uint32_t j;
        while ((j = mt_next(s) & mask) > (uint32_t)i) {
        }
        int32_t t = out[i];
        out[i] = out[j];
        out[j] = t;
    }
}

static void mt_randint31(mt_state* s, int32_t count) {
    for (int32_t k = 0; k < count; ++k) {
        while ((mt_next(s) & 0x7fffffffu) == 0x7fffffffu) {
        }
    }
}

/* One partition of nb batches (per_batch rows each, the last last_len rows).  changes:
 * sorted batch indices (>= 1) whose DDM reported a change.  want: sorted batch indices
 * whose permutation is written to perm_out[k * per_batch ...] (k = index in want).
 * key_out / pos_out: the generator after the last batch (numpy get_state()[1:3]).
 * n_estimators: randint draws per refit.  Returns 0, or -1 on bad arguments. */
int oracle_mt_replay(uint32_t seed, int64_t nb, int32_t per_batch, int32_t last_len, int32_t n_estimators,
                     const int64_t* changes, int64_t n_changes, const int64_t* want, int64_t n_want,
                     int32_t* perm_out, uint32_t* key_out, int32_t* pos_out) {
    if (nb < 1 || per_batch < 1 || per_batch > 4096 || last_len < 1 || last_len > per_batch) return -1;
    mt_state s;
    mt_seed(&s, seed);
    int32_t buf[4096];
    int64_t ci = 0, wi = 0;
    int retrain = 1;
    for (int64_t b = 0; b < nb; ++b) {
        const int32_t len = b == nb - 1 ? last_len : per_batch;
        mt_permutation(&s, len, buf);
        if (wi < n_want && want[wi] == b) {
            memcpy(perm_out + wi * per_batch, buf, sizeof(int32_t) * (size_t)len);
            ++wi;
        }
        if (b == 0) continue;                       /* batch 0 is the first training batch */
        if (retrain) {
            mt_randint31(&s, n_estimators);
            retrain = 0;
        }
        while (ci < n_changes && changes[ci] < b) ++ci;
        if (ci < n_changes && changes[ci] == b) retrain = 1;
    }
    memcpy(key_out, s.key, sizeof(s.key));
    *pos_out = s.pos;
    return 0;
}
