// Batch shuffles on the GPU: pandas `sample(frac=1)` (DDM_Process.py:187, :190) ==
// numpy legacy RandomState.permutation on the global MT19937, reproduced draw for draw.
//
// The reference consumes one sequential MT19937 stream per partition: for every batch a
// Fisher-Yates pass whose intervals i = L-1..1 each take the first draw v with
// (v & mask(i)) <= i (mask(i) = smallest 2^k-1 >= i; rejected draws are skipped).  On
// the host that chain is latency bound (~10 ns/row).  Here it is made parallel:
//   1. k_mt_generate   one workgroup per partition emits the raw tempered stream R;
//                      a 624-word block is regenerated in LDS in three barrier phases.
//   2. k_fsm_prefix    interval acceptance is a finite-state machine whose state is the
//                      interval index s in [1, L-1] (s == 1 accepted -> batch done,
//                      s := L-1).  For every 8192-draw chunk and EVERY state it may be
//                      entered in: the state and batches done after each of its 64
//                      128-draw sub-chunks (prefix tables, coupled trajectories merged).
//   3. k_fsm_first     per window: classic per-sub-chunk tables for the rest of the
//                      chunk holding the window start P (entered mid-chunk).
//   4. k_fsm_walk      one lane walks from P (draws, first-chunk tables, then chunk
//                      tables) to find every piece's start (state, batch).
//   5. k_fsm_replay    one wave per chunk piece: lane t takes sub-chunk t's start from
//                      the prefix tables and replays its 128 draws, recording per batch
//                      the j of every interval and the draw that completes the batch.
//   6. k_fsm_perms     one lane per batch applies its L-1 swaps -> perm bytes in HBM.
// Steps 2-3 depend only on the RNG stream (not on drifts), so they run once per stream
// segment; 4-6 run per speculative window.  Tempering is invertible, so the host
// recovers the exact numpy (key, pos) state at any draw from R.
#include "common.h"

using ddm::as_global;
using ddm::gptr;

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kN = 624;
constexpr int kSub = 128;            // draws per sub-chunk
constexpr int kSubPerChunk = 64;     // sub-chunks per chunk
constexpr int64_t kChunk = (int64_t)kSub * kSubPerChunk;

__device__ __forceinline__ uint32_t temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

__device__ __forceinline__ uint32_t mt_word(uint32_t a, uint32_t b, uint32_t c) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

__device__ __forceinline__ uint32_t imask(uint32_t i) { return 0xffffffffu >> __builtin_clz(i); }

// state word: key[624] (untempered) followed by pos (number of words of key consumed).
// Double-buffered regeneration: the new block is computed from the old one in three
// dependency phases (words 0..226 need only old words; 227..453 need new 0..226;
// 454..623 need new 227..396 and new 0), each thread tempering and storing the words it
// produced, so a 624-word block costs three barriers.
__device__ void mt_generate(gptr<uint32_t> __restrict__ state, gptr<uint32_t> __restrict__ R, int64_t n) {
    __shared__ uint32_t buf[2][kN];
    for (int k = threadIdx.x; k < kN; k += 256) buf[0][k] = state[k];
    const int pos0 = (int)state[kN];
    __syncthreads();
    int cur = 0;
    int64_t out = 0;
    const int t = threadIdx.x;
    // the rest of the current block
    if (pos0 < kN) {
        const int take = (int)min((int64_t)(kN - pos0), n);
        for (int k = t; k < take; k += 256) R[k] = temper(buf[0][pos0 + k]);
        out = take;
    }
    int pos = pos0 < kN ? pos0 + (int)out : kN;
    while (out < n) {
        const uint32_t* o = buf[cur];
        uint32_t* w = buf[cur ^ 1];
        const int64_t base = out;
        const int64_t lim = n - base;   // words of this block to emit
        if (t < 227) {
            const uint32_t v = mt_word(o[t], o[t + 1], o[t + 397]);
            w[t] = v;
            if (t < lim) R[base + t] = temper(v);
        }
        __syncthreads();
        if (t < 227) {
            const int i = 227 + t;
            const uint32_t v = mt_word(o[i], o[i + 1], w[t]);
            w[i] = v;
            if (i < lim) R[base + i] = temper(v);
        }
        __syncthreads();
        if (t < 170) {
            const int i = 454 + t;
            const uint32_t v = (i < kN - 1) ? mt_word(o[i], o[i + 1], w[i - 227]) : mt_word(o[kN - 1], w[0], w[396]);
            w[i] = v;
            if (i < lim) R[base + i] = temper(v);
        }
        __syncthreads();
        cur ^= 1;
        const int take = (int)min((int64_t)kN, lim);
        out += take;
        pos = take;
    }
    for (int k = t; k < kN; k += 256) state[k] = buf[cur][k];
    if (t == 0) state[kN] = (uint32_t)pos;
}

__global__ __launch_bounds__(256) void k_mt_generate(uint32_t* __restrict__ state, uint32_t* __restrict__ R,
                                                     int64_t n) {
    mt_generate(as_global(state), as_global(R), n);
}

// g(T) * key on the device.  T^i(key) is the window (x_i .. x_{i+623}) of the MT19937
// word sequence that starts with key (x_{k+624} = f(x_k, x_{k+1}, x_{k+397})), so by
// linearity g(T) * key = XOR over the set coefficients i of g of those windows.  Thread j
// accumulates out[j] = XOR_i x_{i+j}, block by block of 624 exponents: the coefficients
// i in [624c, 624c + 624) read x_{624c} .. x_{624c + 1246}, i.e. sequence blocks c and
// c + 1, so only three blocks live in LDS (a ring; slot 3 mirrors slot 0 so that blocks c,
// c + 1 are always contiguous), block c + 2 is generated (three barrier phases) once block
// c's coefficients are done, and a workgroup takes ~12 KB of LDS instead of the whole
// ~85 KB sequence (several jumps share a CU, beside the epochs' kernels).  The
// coefficients are wave-uniform: their bits are walked on the scalar unit (readfirstlane,
// find-first-set), so a set bit costs the lanes one address add, one LDS read and a XOR.
struct JumpJob {
    const uint32_t* key;
    const uint64_t* poly;
    uint32_t* out;
    uint32_t* scratch;   // unused (the sequence lives in LDS)
};

constexpr int kJumpThreads = 640;    // >= 624 outputs, a multiple of 64

// block n of the sequence into ring slot n % 3 (and its mirror, slot 3, when n % 3 == 0)
// from block n - 1; three dependency phases, a barrier after each
__device__ __forceinline__ void jump_block(uint32_t* x, int n, int t) {
    const uint32_t* prev = x + ((n - 1) % 3) * kN;
    uint32_t* cur = x + (n % 3) * kN;
    uint32_t* mir = (n % 3 == 0) ? x + 3 * kN : nullptr;
    if (t < 227) {
        const uint32_t v = mt_word(prev[t], prev[t + 1], prev[t + 397]);
        cur[t] = v;
        if (mir) mir[t] = v;
    }
    __syncthreads();
    if (t < 227) {
        const int i = 227 + t;
        const uint32_t v = mt_word(prev[i], prev[i + 1], cur[t]);
        cur[i] = v;
        if (mir) mir[i] = v;
    }
    __syncthreads();
    if (t < 170) {
        const int i = 454 + t;
        const uint32_t v = mt_word(prev[i], i + 1 < kN ? prev[i + 1] : cur[0], cur[i - 227]);
        cur[i] = v;
        if (mir) mir[i] = v;
    }
    __syncthreads();
}

__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

__global__ __launch_bounds__(kJumpThreads) void k_mt_jump(const JumpJob* __restrict__ jobs) {
    __shared__ uint64_t P[DDM_MT_POLY_WORDS];
    __shared__ uint32_t x[4 * kN];
    __shared__ int top_s;
    const JumpJob jb = jobs[blockIdx.x];
    const int t = threadIdx.x;
    if (t == 0) top_s = -1;
    for (int k = t; k < DDM_MT_POLY_WORDS; k += kJumpThreads) P[k] = jb.poly[k];
    if (t < kN) {
        const uint32_t v = jb.key[t];
        x[t] = v;
        x[3 * kN + t] = v;
    }
    __syncthreads();
    for (int k = t; k < DDM_MT_POLY_WORDS; k += kJumpThreads)
        if (P[k]) atomicMax(&top_s, 64 * k + 63 - __builtin_clzll(P[k]));
    __syncthreads();
    const int top = top_s;
    if (top >= 0) jump_block(x, 1, t);
    uint32_t a = 0;
    const int tt = t < kN ? t : 0;       // lanes past the state read a valid word, store nothing
    for (int c = 0; c * kN <= top; ++c) {
        const int lo = c * kN, hi = min(lo + kN, top + 1);
        const uint32_t* xc = x + (c % 3) * kN + tt;   // x_{lo + r + t} == xc[r], r + t < 1248
        for (int wd = lo >> 6; wd * 64 < hi; ++wd) {
            uint64_t bits = uniform_u64(P[wd]);
            const int b_lo = lo - 64 * wd, b_hi = hi - 64 * wd;
            if (b_lo > 0) bits &= ~0ull << b_lo;
            if (b_hi < 64) bits &= (1ull << b_hi) - 1;
            const int base = 64 * wd - lo;
            int n = __builtin_popcountll(bits);
            for (; n >= 8; n -= 8) {
                uint32_t v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    v[u] = xc[base + __builtin_ctzll(bits)];
                    bits &= bits - 1;
                }
                a ^= (v[0] ^ v[1]) ^ (v[2] ^ v[3]) ^ (v[4] ^ v[5]) ^ (v[6] ^ v[7]);
            }
            for (; n > 0; --n) {
                a ^= xc[base + __builtin_ctzll(bits)];
                bits &= bits - 1;
            }
        }
        // block c + 2 into block c - 1's slot; its barriers also close block c's reads
        if ((c + 1) * kN <= top) jump_block(x, c + 2, t);
    }
    if (t < kN) jb.out[t] = top >= 0 ? a : 0u;
    if (t == 0) jb.out[kN] = kN;
}

struct GenJob {
    uint32_t* state;
    uint32_t* R;
    int64_t n;
};

__global__ __launch_bounds__(256) void k_mt_generate_batch(const GenJob* __restrict__ jobs) {
    const GenJob j = jobs[blockIdx.x];
    mt_generate(as_global(j.state), as_global(j.R), j.n);
}

__device__ __forceinline__ void fsm_step(uint32_t v, uint32_t& s, uint32_t& d, uint32_t S) {
    const bool acc = (v & imask(s)) <= s;
    const bool wrap = acc && s == 1;
    d += wrap ? 1u : 0u;
    s = wrap ? S : (acc ? s - 1 : s);
}

// Prefix tables.  For every chunk c of the stream and every interval state s it may be
// entered in: Tpre[c][k][s-1] = (state after sub-chunks 0..k of the chunk) | (batches
// completed since the chunk start) << 8, and Tchunk[c][s-1] = Tpre[c][63][s-1].
//
// The S trajectories of a chunk couple fast (two that reach the same state at the same
// draw never part again): for L = 100 about 27 distinct states are left after the first
// 128 draws, 10 after 512 and 3 after 8192.  A workgroup runs 16 chunks as ONE list of
// distinct (chunk, state) trajectories: per sub-chunk it steps every listed trajectory
// over the 128 draws (LDS rows, 16-byte reads), merges the ones that met (LDS atomicMin
// on the end state picks the survivor), renumbers the survivors in order, and writes
// every start state's entry through its trajectory index plus a done offset.  After the
// first sub-chunks ~16 trajectories per chunk remain, one pass of 128 lanes for all 8
// chunks: ~6x fewer FSM steps than stepping every start state through every sub-chunk.
// (8 chunks and 2 waves per workgroup: ~20 KB of LDS, so 8 workgroups share a CU.)
constexpr int kPreChunks = 8;
constexpr int kPreThreads = 128;    // 8 chunks x ~16 trajectories once they have coupled
constexpr int kPreRow = kSub + 4;   // LDS row stride in words: 16-byte rows, the chunks' rows in distinct banks

size_t prefix_lds_bytes(int L) {
    const size_t S = (size_t)L - 1, NP = kPreChunks * S;
    return (size_t)kPreChunks * kPreRow * 4 + (size_t)kPreChunks * (S + 1) * 4 + NP * (6 * 2 + 4 * 1);
}

struct TabJob {
    const uint32_t* R;
    int64_t chunk0, nchunk;
    uint32_t* Tpre;
    uint32_t* Tchunk;
};

__device__ void fsm_prefix(gptr<const uint32_t> __restrict__ R, int64_t chunk0, int64_t nchunk, int L,
                           gptr<uint32_t> __restrict__ Tpre, gptr<uint32_t> __restrict__ Tchunk, int64_t blk) {
    extern __shared__ __attribute__((aligned(16))) uint32_t pre_lds[];
    constexpr int kW = kPreThreads / 64;
    __shared__ int wsum[kW];
    __shared__ int n_sh;
    const int S = L - 1, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t cb = chunk0 + blk * kPreChunks;
    if (cb >= chunk0 + nchunk) return;
    const int nc = (int)min((int64_t)kPreChunks, chunk0 + nchunk - cb);
    const int NP = kPreChunks * S;
    uint32_t* draws = pre_lds;                                              // [16][kPreRow]
    int32_t* owner = reinterpret_cast<int32_t*>(draws + kPreChunks * kPreRow); // [16][S + 1]
    uint16_t* dn = reinterpret_cast<uint16_t*>(owner + kPreChunks * (S + 1));  // batches done, per trajectory
    uint16_t* dn2 = dn + NP;
    int16_t* nidx = reinterpret_cast<int16_t*>(dn2 + NP);                   // index after the merge
    int16_t* dlt = nidx + NP;                                               // done minus its survivor's
    int16_t* cls = dlt + NP;                                                // per start state: trajectory
    int16_t* off = cls + NP;                                                //   and done offset
    uint8_t* st = reinterpret_cast<uint8_t*>(off + NP);
    uint8_t* st2 = st + NP;
    uint8_t* ch = st2 + NP;
    uint8_t* ch2 = ch + NP;
    const int ns = nc * S;
    for (int e = tid; e < ns; e += kPreThreads) {
        st[e] = (uint8_t)(e % S + 1);
        dn[e] = 0;
        ch[e] = (uint8_t)(e / S);
        cls[e] = (int16_t)e;
        off[e] = 0;
    }
    if (tid == 0) n_sh = ns;
    // the sub-chunk's draws of all nc chunks: kPreLoads 16-byte loads per thread, the next
    // sub-chunk's issued right after this one's are in LDS so that they land while the
    // trajectories are stepped (the loop was waiting on a dependent HBM load 64 times)
    constexpr int kPreLoads = kPreChunks * (kSub / 4) / kPreThreads;
    static_assert(kPreLoads * kPreThreads == kPreChunks * (kSub / 4), "whole loads per thread");
    u32x4 nxt[kPreLoads];
    auto load_sub = [&](int k) {
#pragma unroll
        for (int u = 0; u < kPreLoads; ++u) {
            const int e = tid + u * kPreThreads, c = e / (kSub / 4), q = e % (kSub / 4);
            if (c < nc) nxt[u] = *(gptr<const u32x4>)(R + (cb + c) * kChunk + (int64_t)k * kSub + 4 * q);
        }
    };
    load_sub(0);
    for (int k = 0; k < kSubPerChunk; ++k) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kPreLoads; ++u) {
            const int e = tid + u * kPreThreads, c = e / (kSub / 4), q = e % (kSub / 4);
            if (c < nc) *reinterpret_cast<u32x4*>(draws + c * kPreRow + 4 * q) = nxt[u];
        }
        if (k + 1 < kSubPerChunk) load_sub(k + 1);
        __syncthreads();
        const int n = n_sh;
        for (int p = tid; p < n; p += kPreThreads) {
            uint32_t s = st[p], d = dn[p];
            const uint32_t* row = draws + ch[p] * kPreRow;
#pragma unroll 4
            for (int q = 0; q < kSub; q += 4) {
                const uint4 v = *reinterpret_cast<const uint4*>(row + q);
                fsm_step(v.x, s, d, (uint32_t)S);
                fsm_step(v.y, s, d, (uint32_t)S);
                fsm_step(v.z, s, d, (uint32_t)S);
                fsm_step(v.w, s, d, (uint32_t)S);
            }
            st2[p] = (uint8_t)s;
            dn2[p] = (uint16_t)d;
            ch2[p] = ch[p];
        }
        for (int e = tid; e < nc * (S + 1); e += kPreThreads) owner[e] = 0x7fffffff;
        __syncthreads();
        for (int p = tid; p < n; p += kPreThreads) atomicMin(&owner[ch2[p] * (S + 1) + st2[p]], p);
        __syncthreads();
        // survivors: the first trajectory of each (chunk, end state), renumbered in order
        const int per = (n + kPreThreads - 1) / kPreThreads;
        const int p0 = min(n, tid * per), p1 = min(n, p0 + per);
        int cnt = 0;
        for (int p = p0; p < p1; ++p) cnt += owner[ch2[p] * (S + 1) + st2[p]] == p ? 1 : 0;
        int inc = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(inc, o, 64);
            if (lane >= o) inc += y;
        }
        if (lane == 63) wsum[wv] = inc;
        __syncthreads();
        int base = 0;
        for (int w = 0; w < wv; ++w) base += wsum[w];
        int idx = base + inc - cnt;
        for (int p = p0; p < p1; ++p)
            if (owner[ch2[p] * (S + 1) + st2[p]] == p) nidx[p] = (int16_t)idx++;
        if (tid == kPreThreads - 1) n_sh = base + inc;
        __syncthreads();
        for (int p = tid; p < n; p += kPreThreads) {
            const int o = owner[ch2[p] * (S + 1) + st2[p]];
            if (o != p) {
                nidx[p] = nidx[o];
                dlt[p] = (int16_t)((int)dn2[p] - (int)dn2[o]);
            } else {
                dlt[p] = 0;
            }
        }
        __syncthreads();
        // every start state's entry; then its trajectory after the merge
        for (int e = tid; e < ns; e += kPreThreads) {
            const int i = cls[e], o = off[e];
            const uint32_t val = (uint32_t)st2[i] | ((uint32_t)((int)dn2[i] + o) << 8);
            const int64_t c = cb + e / S;
            const int s0 = e % S;
            Tpre[(c * kSubPerChunk + k) * S + s0] = val;
            if (k == kSubPerChunk - 1) Tchunk[c * S + s0] = val;
            cls[e] = nidx[i];
            off[e] = (int16_t)(o + dlt[i]);
        }
        for (int p = tid; p < n; p += kPreThreads)
            if (owner[ch2[p] * (S + 1) + st2[p]] == p) {
                const int q = nidx[p];
                st[q] = st2[p];
                dn[q] = dn2[p];
                ch[q] = ch2[p];
            }
    }
}

__global__ __launch_bounds__(kPreThreads) void k_fsm_prefix(const uint32_t* __restrict__ R, int64_t chunk0,
                                                            int64_t nchunk, int L, uint32_t* __restrict__ Tpre,
                                                            uint32_t* __restrict__ Tchunk) {
    fsm_prefix(as_global(R), chunk0, nchunk, L, as_global(Tpre), as_global(Tchunk), blockIdx.x);
}

__global__ __launch_bounds__(kPreThreads) void k_fsm_prefix_batch(const TabJob* __restrict__ jobs, int L) {
    const TabJob j = jobs[blockIdx.y];
    fsm_prefix(as_global(j.R), j.chunk0, j.nchunk, L, as_global(j.Tpre), as_global(j.Tchunk), blockIdx.x);
}

struct Job {
    const uint32_t* R;
    const uint32_t* Tpre;
    const uint32_t* Tchunk;
    int64_t avail, P, W;
    void* pieces;
    int64_t* info;
    uint8_t* J;
    int64_t* E;
    uint8_t* perm_out;
    const int32_t* stop;
    int64_t pick_offset, pick_last;
    int64_t* pick_out;
    uint16_t* first;   // [64][S]: sub-chunk tables of the chunk holding P (k_fsm_first)
};

struct ChunkStart {
    int64_t pos;      // first draw of this window piece
    int32_t state;    // interval index at pos
    int32_t batch;    // batches completed (relative to the window) before pos
};


__device__ __forceinline__ void put_piece(gptr<ChunkStart> out, int64_t k, int64_t pos, int32_t state, int32_t batch) {
    out[k].pos = pos;
    out[k].state = state;
    out[k].batch = batch;
}

__device__ __forceinline__ ChunkStart get_piece(gptr<const ChunkStart> in, int64_t k) {
    return ChunkStart{in[k].pos, in[k].state, in[k].batch};
}

// The prefix tables only describe chunks entered at their first draw.  A window starts at
// a batch boundary P anywhere in a chunk (the refit seeds before it are not shuffle draws),
// so the rest of that one chunk gets classic per-sub-chunk tables, every start state
// stepped through every sub-chunk after the one holding P: first[q][s-1] = end state |
// batches << 8.  One workgroup per (sub-chunk, job); they run side by side.
constexpr int kFirstThreads = 128;

__device__ void fsm_first(const Job& j, int L) {
    __shared__ __attribute__((aligned(16))) uint32_t dr[kSub];
    if (j.W <= 0) return;
    const int S = L - 1;
    const int64_t cstart = j.P / kChunk * kChunk;
    const int q = (int)((j.P - cstart) / kSub) + 1 + (int)blockIdx.x;
    if (q >= kSubPerChunk) return;
    const int64_t d0 = cstart + (int64_t)q * kSub;
    if (d0 + kSub > j.avail) return;
    if (threadIdx.x < kSub / 4)
        reinterpret_cast<u32x4*>(dr)[threadIdx.x] = ((gptr<const u32x4>)as_global(j.R + d0))[threadIdx.x];
    __syncthreads();
    for (int s0 = threadIdx.x + 1; s0 <= S; s0 += blockDim.x) {
        uint32_t s = (uint32_t)s0, d = 0;
#pragma unroll 4
        for (int k = 0; k < kSub; k += 4) {
            const uint4 v = reinterpret_cast<const uint4*>(dr)[k / 4];
            fsm_step(v.x, s, d, (uint32_t)S);
            fsm_step(v.y, s, d, (uint32_t)S);
            fsm_step(v.z, s, d, (uint32_t)S);
            fsm_step(v.w, s, d, (uint32_t)S);
        }
        as_global(j.first)[q * S + (s0 - 1)] = (uint16_t)(s | (d << 8));
    }
}

__global__ __launch_bounds__(kFirstThreads) void k_fsm_first(Job j, int L) { fsm_first(j, L); }

__global__ __launch_bounds__(kFirstThreads) void k_fsm_first_batch(const Job* __restrict__ jobs, int L) {
    const Job j = jobs[blockIdx.y];
    fsm_first(j, L);
}

constexpr int kWalkThreads = 256;    // stage the table rows; lane 0 walks them

// From draw P at a batch boundary: draw by draw to the next sub-chunk boundary, then by
// the first-chunk tables (k_fsm_first) to the chunk boundary, then chunk by chunk (Tchunk)
// until W batches are done.  Table rows are staged in LDS (all lanes load, lane 0 walks),
// so the serial walk does LDS lookups, not dependent HBM loads.
// Pieces: out[0] = [P, next sub-chunk boundary); then every sub-chunk of P's chunk; then
// chunk starts.  info = {pieces, end draw, batches reached}.
__device__ void fsm_walk(gptr<const uint32_t> __restrict__ R, gptr<const uint16_t> __restrict__ first,
                         gptr<const uint32_t> __restrict__ Tchunk, int64_t P, int64_t W, int L, int64_t avail,
                         gptr<ChunkStart> __restrict__ out, gptr<int64_t> __restrict__ info) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tab[];   // [64][S] chunk rows; phase A: draws + first-chunk rows
#ifdef DDM_WALK_PROFILE
    const uint64_t t_start = wall_clock64();
    uint64_t t_p0 = 0, t_p1 = 0, t_ld = 0;
#endif
    __shared__ int64_t sh_pos, sh_batch, sh_k;
    __shared__ uint32_t sh_s;
    const int S = L - 1;
    const int64_t sub_end = min(avail, (P / kSub + 1) * kSub);
    const int64_t chunk_end = min(avail, (P / kChunk + 1) * kChunk);
    const int n_draws = (int)max((int64_t)0, sub_end - P);
    const int q0 = (int)((sub_end % kChunk) / kSub);          // first sub-chunk after P's
    const int n_subrows = (int)max((int64_t)0, (chunk_end - sub_end) / kSub);
    uint32_t* a_draws = tab;
    uint16_t* a_first = reinterpret_cast<uint16_t*>(tab + kSub);
    for (int k = threadIdx.x; k < n_draws; k += kWalkThreads) a_draws[k] = R[P + k];
    const int of = (q0 * S) & 7;                      // 16-byte loads from the aligned element before
    {
        const gptr<const u32x4> src = (gptr<const u32x4>)(first + q0 * S - of);
        const int n8 = n_subrows > 0 ? (n_subrows * S + of + 7) / 8 : 0;
        for (int e = threadIdx.x; e < n8; e += kWalkThreads) reinterpret_cast<u32x4*>(a_first)[e] = src[e];
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        // draw by draw to the sub-chunk boundary, by the first wave: the next accepted draw
        // of the current interval is the first lane of a ballot over the next 64 draws
        const int lane = threadIdx.x;
        int64_t pos = P, batch = 0;
        uint32_t s = (uint32_t)S;
        for (int64_t base = P; batch < W && base < sub_end; base += 64) {
            // this lane's draw of the 64-draw window stays in a register; every accepted
            // draw is one ballot
            const bool in = base + lane < sub_end;
            const uint32_t v = in ? a_draws[base - P + lane] : 0u;
            int from = 0;
            pos = min(sub_end, base + 64);
            for (;;) {
                const uint64_t acc = __ballot(in && lane >= from && (v & imask(s)) <= s);
                if (!acc) break;
                const int f = __builtin_ctzll(acc);
                from = f + 1;
                if (s == 1) {
                    s = (uint32_t)S;
                    if (++batch >= W) {
                        pos = base + f + 1;
                        break;
                    }
                } else {
                    --s;
                }
            }
        }
#ifdef DDM_WALK_PROFILE
        t_p0 = wall_clock64();
#endif
        if (lane == 0) {                      // the rest of the walk is serial
            int64_t k = 0;
            put_piece(out, k++, P, S, 0);
            while (batch < W && pos % kChunk != 0 && pos + kSub <= avail) {
                put_piece(out, k++, pos, (int32_t)s, (int32_t)batch);
                const uint32_t e = a_first[of + ((pos - sub_end) / kSub) * S + (s - 1)];
                s = e & 0xffu;
                batch += e >> 8;
                pos += kSub;
            }
            sh_pos = pos;
            sh_batch = batch;
            sh_k = k;
            sh_s = s;
        }
#ifdef DDM_WALK_PROFILE
        t_p1 = wall_clock64();
#endif
    }
    __syncthreads();
    // chunk by chunk: the rows of up to 64 chunks per LDS buffer; waves 1-3 load the next
    // buffer while lane 0 walks the current one
    const int stride = (64 * S + 4 + 3) & ~3;
    auto load_rows = [&](uint32_t* buf, int64_t c0, int n, int t0) {
        // 16-byte loads from the aligned word at or before row c0 (Tchunk is 16-byte aligned
        // and padded by 4 words)
        const int o = (int)((c0 * S) & 3);
        const gptr<const u32x4> src = (gptr<const u32x4>)(Tchunk + c0 * S - o);
        const int n4 = (n * S + o + 3) / 4;
        for (int e = (int)threadIdx.x - t0; e < n4; e += kWalkThreads - t0) reinterpret_cast<u32x4*>(buf)[e] = src[e];
    };
    const int64_t covered = avail / kChunk;
    int64_t c_load = sh_pos / kChunk;
    int nload = (sh_batch < W && sh_pos % kChunk == 0) ? (int)max((int64_t)0, min((int64_t)64, covered - c_load)) : 0;
    if (nload > 0) load_rows(tab, c_load, nload, 0);
    __syncthreads();
    int cur = 0;
    while (nload > 0) {
        const int64_t c_next = c_load + nload;
        const int nnext = (int)max((int64_t)0, min((int64_t)64, covered - c_next));
        uint32_t* now = tab + cur * stride;
        if (threadIdx.x >= 64 && nnext > 0) load_rows(tab + (cur ^ 1) * stride, c_next, nnext, 64);
        if (threadIdx.x == 0) {
            const int o = (int)((c_load * S) & 3);
            int64_t pos = sh_pos, batch = sh_batch, k = sh_k;
            uint32_t s = sh_s;
            for (int c = 0; c < nload && batch < W; ++c) {
                put_piece(out, k++, pos, (int32_t)s, (int32_t)batch);
                const uint32_t e = now[o + c * S + (s - 1)];
                s = e & 0xffu;
                batch += e >> 8;
                pos += kChunk;
            }
            sh_pos = pos;
            sh_batch = batch;
            sh_k = k;
            sh_s = s;
        }
        __syncthreads();
        if (sh_batch >= W) break;
        c_load = c_next;
        nload = nnext;
        cur ^= 1;
    }
    if (threadIdx.x == 0) {
        info[0] = sh_k;
        info[1] = sh_pos;
        info[2] = sh_batch;
#ifdef DDM_WALK_PROFILE
        const uint64_t t_end = wall_clock64();
        info[3] = (int64_t)(t_p0 - t_start);
        info[4] = (int64_t)(t_p1 - t_start);
        info[5] = (int64_t)(t_end - t_start);
        info[6] = (int64_t)t_ld;
#endif
    }
}

__global__ __launch_bounds__(kWalkThreads) void k_fsm_walk(Job j, int L) {
    fsm_walk(as_global(j.R), as_global((const uint16_t*)j.first), as_global(j.Tchunk), j.P, j.W, L, j.avail,
             as_global(reinterpret_cast<ChunkStart*>(j.pieces)), as_global(j.info));
}

__global__ __launch_bounds__(kWalkThreads) void k_fsm_walk_batch(const Job* __restrict__ jobs, int L) {
    const Job j = jobs[blockIdx.x];
    if (j.W <= 0) return;
    fsm_walk(as_global(j.R), as_global((const uint16_t*)j.first), as_global(j.Tchunk), j.P, j.W, L, j.avail,
             as_global(reinterpret_cast<ChunkStart*>(j.pieces)), as_global(j.info));
}

// One wave per window piece.  A piece of at most one sub-chunk (the start of the window's
// first chunk) is replayed by lane 0; a chunk piece starts on a chunk boundary, so lane t
// reads sub-chunk t's start state and batch straight from the prefix tables and every
// lane replays its sub-chunk from HBM, 16 draws per round of loads: for each accepted draw
// of batch b < W the interval's j (v & mask(s)) is recorded and, when s == 1, E[b] = draw
// index.  Where a j goes: the batches that begin and end inside one chunk piece (nearly all
// of a window) are recorded in LDS and shuffled by the piece's own wave, which then writes
// their perm bytes contiguously; the others (the batches of the window's first chunk, cut
// into sub-chunk pieces, and the batch that straddles each chunk boundary) go to J in HBM
// for k_fsm_perms_batch.  J[b*L] (interval 0 never draws) tells k_fsm_perms_batch which:
// 1 = shuffled by the replay, 0 = its job.
constexpr int kReplayBatch = 16;

struct ReplaySink {
    gptr<uint8_t> J;
    gptr<int64_t> E;
    uint8_t* Jl;          // LDS rows of batches [b_lo, b_hi)
    int64_t b_lo, b_hi;
    int L;
    __device__ __forceinline__ bool local(int64_t b) const { return b >= b_lo && b < b_hi; }
    __device__ __forceinline__ void rec(int64_t b, uint32_t s, uint8_t m) const {
        if (local(b)) Jl[(b - b_lo) * L + s] = m;
        else J[b * L + s] = m;
    }
    __device__ __forceinline__ void done(int64_t b, int64_t q) const {
        E[b] = q;
        if (!local(b)) J[b * L] = 0;
    }
};

__device__ __forceinline__ void replay_step(uint32_t v, int64_t q, uint32_t& s, int64_t& b, uint32_t S,
                                            const ReplaySink& k) {
    const uint32_t m = v & imask(s);
    if (m <= s) {
        k.rec(b, s, (uint8_t)m);
        if (s == 1) {
            k.done(b, q);
            s = S;
            ++b;
        } else {
            --s;
        }
    }
}

__device__ __forceinline__ void replay_range(gptr<const uint32_t> __restrict__ R, int64_t beg, int64_t fin, uint32_t s,
                                             int64_t b, int64_t W, int L, const ReplaySink& k) {
    const uint32_t S = (uint32_t)(L - 1);
    if (fin - beg == kSub && (beg & 3) == 0) {
        // a whole sub-chunk: 64 words at a time in flight (sixteen 16-byte loads)
        const gptr<const u32x4> src = (gptr<const u32x4>)(R + beg);
        for (int h = 0; h < kSub / 64 && b < W; ++h) {
            u32x4 v[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = src[16 * h + q];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int64_t d = beg + 64 * h + 4 * q;
                if (b < W) replay_step(v[q].x, d, s, b, S, k);
                if (b < W) replay_step(v[q].y, d + 1, s, b, S, k);
                if (b < W) replay_step(v[q].z, d + 2, s, b, S, k);
                if (b < W) replay_step(v[q].w, d + 3, s, b, S, k);
            }
        }
        return;
    }
    for (int64_t q0 = beg; q0 < fin && b < W; q0 += kReplayBatch) {
        uint32_t v[kReplayBatch];
#pragma unroll
        for (int q = 0; q < kReplayBatch; ++q) v[q] = R[min(q0 + q, fin - 1)];
#pragma unroll
        for (int q = 0; q < kReplayBatch; ++q)
            if (q0 + q < fin && b < W) replay_step(v[q], q0 + q, s, b, S, k);
    }
}

// LDS of the fused replay: the j rows and the perms of a chunk piece's own batches (a
// batch takes at least L-1 draws, so a chunk holds at most kChunk / (L-1) + 1 of them)
__host__ __device__ inline int replay_local_batches(int L) { return (int)(kChunk / (L - 1)) + 2; }
size_t replay_lds_bytes(int L) { return ((size_t)2 * replay_local_batches(L) * L + 15) & ~(size_t)15; }

template <bool kFused>
__device__ void fsm_replay(gptr<const uint32_t> __restrict__ R, gptr<const uint32_t> __restrict__ Tpre,
                           gptr<const ChunkStart> __restrict__ pieces, gptr<const int64_t> __restrict__ info, int64_t W,
                           int L, gptr<uint8_t> __restrict__ J, gptr<int64_t> __restrict__ E,
                           gptr<uint8_t> __restrict__ perm_out, int64_t blk, int64_t nblk) {
    extern __shared__ __attribute__((aligned(16))) uint8_t rlds[];
    __shared__ uint32_t sdraws[kSub];
    const int64_t npieces = info[0], end = info[1];
    const int S = L - 1;
    const int lane = threadIdx.x;
    const int cap = replay_local_batches(L);
    for (int64_t pc = blk; pc < npieces; pc += nblk) {
        const ChunkStart c = get_piece(pieces, pc);
        const int64_t stop = (pc + 1 < npieces) ? pieces[pc + 1].pos : end;
        if (stop <= c.pos) continue;
        if (stop - c.pos <= kSub) {
            // a piece of at most one sub-chunk, stepped by lane 0: the wave stages its draws in
            // LDS with one load each first (lane 0 alone took 8 dependent rounds of 16-word
            // loads: ~30 us, on the critical path of small windows' epochs, C5 / c2)
            const ReplaySink k{J, E, nullptr, 0, 0, L};
            const int n = (int)(stop - c.pos);
            for (int q = lane; q < n; q += 64) sdraws[q] = R[c.pos + q];
            __syncthreads();
            if (lane == 0) {
                uint32_t s = (uint32_t)c.state;
                int64_t b = c.batch;
                const uint32_t S = (uint32_t)(L - 1);
                for (int q = 0; q < n && b < W; ++q) replay_step(sdraws[q], c.pos + q, s, b, S, k);
            }
            __syncthreads();
            continue;
        }
        // this piece's own batches: those that start in it and end in it
        int64_t b_lo = 0, b_hi = 0;
        if (kFused) {
            b_lo = c.batch + (c.state != S ? 1 : 0);
            b_hi = min(W, (pc + 1 < npieces) ? (int64_t)pieces[pc + 1].batch : W);
            b_hi = max(b_lo, min(b_hi, b_lo + cap));
        }
        const ReplaySink k{J, E, rlds, b_lo, b_hi, L};
        const int64_t chunk = c.pos / kChunk;        // c.pos % kChunk == 0 (a chunk piece)
        const int nsub = (int)((stop - c.pos + kSub - 1) / kSub);
        for (int t = lane; t < nsub; t += 64) {
            uint32_t s = (uint32_t)c.state;
            int64_t b = c.batch;
            if (t > 0) {
                const uint32_t e = Tpre[(chunk * kSubPerChunk + (t - 1)) * S + (c.state - 1)];
                s = e & 0xffu;
                b += e >> 8;
            }
#ifndef DDM_SHUF_NOREPLAY     // timing variant (tools/build_variant.sh): results are NOT the shuffle's
            replay_range(R, c.pos + (int64_t)t * kSub, min(stop, c.pos + (int64_t)(t + 1) * kSub), s, b, W, L, k);
#endif
        }
        if (!kFused) continue;
        const int nloc = (int)(b_hi - b_lo);
        uint8_t* Pl = rlds + (size_t)cap * L;
        __syncthreads();
        // Fisher-Yates of every own batch: lane k applies batch k's swaps i = L-1 .. 1
#ifdef DDM_SHUF_NOFY          // timing variant: results are NOT the shuffle's
        for (int q = lane; q < 0; q += 64) {
#else
        for (int q = lane; q < nloc; q += 64) {
#endif
            uint8_t* p = Pl + (size_t)q * L;
            const uint8_t* jr = rlds + (size_t)q * L;
            for (int e = 0; e < L; ++e) p[e] = (uint8_t)e;
            for (int i = L - 1; i >= 1; --i) {
                const int jj = jr[i];
                const uint8_t tmp = p[i];
                p[i] = p[jj];
                p[jj] = tmp;
            }
            J[(b_lo + q) * L] = 1;
        }
        __syncthreads();
        // their perm bytes, contiguous in the window
        const gptr<uint8_t> dst = perm_out + b_lo * L;
        const int nbytes = nloc * L;
        if (((uintptr_t)dst & 3) == 0) {
            const int nw = nbytes >> 2;
            for (int e = lane; e < nw; e += 64)
                ((gptr<uint32_t>)dst)[e] = reinterpret_cast<const uint32_t*>(Pl)[e];
            for (int e = 4 * nw + lane; e < nbytes; e += 64) dst[e] = Pl[e];
        } else {
            for (int e = lane; e < nbytes; e += 64) dst[e] = Pl[e];
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(64) void k_fsm_replay(Job j, int L) {
    fsm_replay<false>(as_global(j.R), as_global(j.Tpre), as_global(reinterpret_cast<const ChunkStart*>(j.pieces)),
                      as_global((const int64_t*)j.info), j.W, L, as_global(j.J), as_global(j.E), nullptr, blockIdx.x,
                      gridDim.x);
}

__global__ __launch_bounds__(64) void k_fsm_replay_batch(const Job* __restrict__ jobs, int L) {
    const Job j = jobs[blockIdx.y];
    if (j.W <= 0) return;
    fsm_replay<true>(as_global(j.R), as_global(j.Tpre), as_global(reinterpret_cast<const ChunkStart*>(j.pieces)),
                     as_global((const int64_t*)j.info), j.W, L, as_global(j.J), as_global(j.E), as_global(j.perm_out),
                     blockIdx.x, gridDim.x);
}

// One lane per batch: Fisher-Yates swaps i = L-1..1 with the recorded j's.
__device__ void fsm_perms(gptr<const uint8_t> __restrict__ J, int64_t W, int L, gptr<uint8_t> __restrict__ perm,
                          int64_t b0) {
    extern __shared__ uint8_t buf[];
    const int64_t b = b0 + threadIdx.x;
    if (b >= W) return;
    const gptr<const uint8_t> j = J + b * L;
    if (j[0]) return;                    // shuffled by the replay itself (fsm_replay<true>)
    uint8_t* p = buf + threadIdx.x * L;
    for (int k = 0; k < L; ++k) p[k] = (uint8_t)k;
    for (int i = L - 1; i >= 1; --i) {
        const int jj = j[i];
        const uint8_t t = p[i];
        p[i] = p[jj];
        p[jj] = t;
    }
    for (int k = 0; k < L; ++k) perm[b * L + k] = p[k];
}

__global__ __launch_bounds__(256) void k_fsm_perms(Job j, int L) {
    fsm_perms(as_global((const uint8_t*)j.J), j.W, L, as_global(j.perm_out), (int64_t)blockIdx.x * 256);
}

__global__ __launch_bounds__(256) void k_fsm_perms_batch(const Job* __restrict__ jobs, int L) {
    const Job j = jobs[blockIdx.y];
    for (int64_t b0 = (int64_t)blockIdx.x * 256; b0 < j.W; b0 += (int64_t)gridDim.x * 256)
        fsm_perms(as_global((const uint8_t*)j.J), j.W, L, as_global(j.perm_out), b0);
}

__global__ void k_pick(const int32_t* stop, const int64_t* E, int64_t W, int64_t offset, int64_t last, int64_t* out) {
    const int64_t k = (stop[0] >= 0 ? (int64_t)stop[0] : last) - offset;
    out[0] = (k >= 0 && k < W) ? E[k] : -1;
}

__global__ void k_pick_batch(const Job* __restrict__ jobs, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Job j = jobs[i];
    if (!j.pick_out) return;
    const int64_t k = (j.stop && j.stop[0] >= 0 ? (int64_t)j.stop[0] : j.pick_last) - j.pick_offset;
    j.pick_out[0] = (j.W > 0 && k >= 0 && k < j.W) ? j.E[k] : -1;
}

size_t walk_lds_bytes(int L) {
    return std::max((size_t)2 * ((64 * (L - 1) + 4 + 3) & ~3) * sizeof(uint32_t),
                    kSub * sizeof(uint32_t) + (size_t)kSubPerChunk * (L - 1) * sizeof(uint16_t));
}

}  // namespace

static_assert(sizeof(Job) == sizeof(ddm_shuffle_job), "ddm_shuffle_job layout");
static_assert(sizeof(GenJob) == sizeof(ddm_gen_job), "ddm_gen_job layout");

extern "C" int ddm_shuffle_generate_batch(const ddm_gen_job* jobs_dev, int32_t n_jobs, ddm_stream_t stream) {
    if (!jobs_dev || n_jobs < 0) {
        ddm::set_error("ddm_shuffle_generate_batch: invalid argument");
        return DDM_E_ARG;
    }
    if (n_jobs == 0) return 0;
    hipLaunchKernelGGL(k_mt_generate_batch, dim3((unsigned)n_jobs), dim3(256), 0, ddm::as_hip(stream),
                       reinterpret_cast<const GenJob*>(jobs_dev));
    return ddm::launch_status("ddm_shuffle_generate_batch");
}

extern "C" int ddm_shuffle_window_batch(const ddm_shuffle_job* jobs_dev, int32_t n_jobs, int64_t max_W,
                                        int64_t max_pieces, int32_t batch_len, ddm_stream_t stream,
                                        ddm_event_t ev_begin, ddm_event_t ev_end) {
    if (!jobs_dev || n_jobs < 0 || max_W < 0 || batch_len < 2 || batch_len > 256) {
        ddm::set_error("ddm_shuffle_window_batch: invalid argument");
        return DDM_E_ARG;
    }
    if (n_jobs == 0 || max_W == 0) return 0;
    hipStream_t s = ddm::as_hip(stream);
    const Job* jobs = reinterpret_cast<const Job*>(jobs_dev);
    if (ev_begin)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_begin), s), "event record")) return rc;
    hipLaunchKernelGGL(k_fsm_first_batch, dim3(kSubPerChunk - 1, (unsigned)n_jobs), dim3(kFirstThreads), 0, s, jobs,
                       (int)batch_len);
    if (int rc = ddm::launch_status("ddm_shuffle_window_batch/first")) return rc;
    hipLaunchKernelGGL(k_fsm_walk_batch, dim3((unsigned)n_jobs), dim3(kWalkThreads), walk_lds_bytes(batch_len), s, jobs,
                       (int)batch_len);
    if (int rc = ddm::launch_status("ddm_shuffle_window_batch/walk")) return rc;
    const int64_t pblocks = std::max<int64_t>(1, std::min<int64_t>(max_pieces, 2048));
    hipLaunchKernelGGL(k_fsm_replay_batch, dim3((unsigned)pblocks, (unsigned)n_jobs), dim3(64),
                       replay_lds_bytes(batch_len), s, jobs, (int)batch_len);
    if (int rc = ddm::launch_status("ddm_shuffle_window_batch/replay")) return rc;
    const int64_t bblocks = std::min<int64_t>(ddm::ceil_div(max_W, 256), 1024);
    hipLaunchKernelGGL(k_fsm_perms_batch, dim3((unsigned)bblocks, (unsigned)n_jobs), dim3(256),
                       (size_t)256 * batch_len, s, jobs, (int)batch_len);
    if (int rc = ddm::launch_status("ddm_shuffle_window_batch/perms")) return rc;
    if (ev_end)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_end), s), "event record")) return rc;
    return 0;
}

extern "C" int ddm_shuffle_pick_batch(const ddm_shuffle_job* jobs_dev, int32_t n_jobs, ddm_stream_t stream) {
    if (!jobs_dev || n_jobs < 0) {
        ddm::set_error("ddm_shuffle_pick_batch: invalid argument");
        return DDM_E_ARG;
    }
    if (n_jobs == 0) return 0;
    hipLaunchKernelGGL(k_pick_batch, dim3((unsigned)ddm::ceil_div(n_jobs, 64)), dim3(64), 0, ddm::as_hip(stream),
                       reinterpret_cast<const Job*>(jobs_dev), (int)n_jobs);
    return ddm::launch_status("ddm_shuffle_pick_batch");
}

extern "C" int ddm_shuffle_pick(const int32_t* stop, const int64_t* E, int64_t W, int64_t offset, int64_t last,
                                int64_t* out, ddm_stream_t stream) {
    if (!stop || !E || !out) {
        ddm::set_error("ddm_shuffle_pick: invalid argument");
        return DDM_E_ARG;
    }
    hipLaunchKernelGGL(k_pick, dim3(1), dim3(1), 0, ddm::as_hip(stream), stop, E, W, offset, last, out);
    return ddm::launch_status("ddm_shuffle_pick");
}

extern "C" int ddm_shuffle_generate(uint32_t* mt_state, uint32_t* R, int64_t n, ddm_stream_t stream) {
    if (!mt_state || !R || n < 0) {
        ddm::set_error("ddm_shuffle_generate: invalid argument");
        return DDM_E_ARG;
    }
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_mt_generate, dim3(1), dim3(256), 0, ddm::as_hip(stream), mt_state, R, n);
    return ddm::launch_status("ddm_shuffle_generate");
}

extern "C" int ddm_mt_jump(const ddm_jump_job* jobs_dev, int32_t n_jobs, ddm_stream_t stream) {
    if (!jobs_dev || n_jobs < 0) {
        ddm::set_error("ddm_mt_jump: invalid argument");
        return DDM_E_ARG;
    }
    if (n_jobs == 0) return 0;
    static_assert(sizeof(JumpJob) == sizeof(ddm_jump_job), "JumpJob must mirror ddm_jump_job");
    hipLaunchKernelGGL(k_mt_jump, dim3((unsigned)n_jobs), dim3(kJumpThreads), 0, ddm::as_hip(stream),
                       reinterpret_cast<const JumpJob*>(jobs_dev));
    return ddm::launch_status("ddm_mt_jump");
}

extern "C" int ddm_shuffle_tables(const uint32_t* R, int64_t chunk0, int64_t nchunk, int32_t batch_len,
                                  uint32_t* Tpre, uint32_t* Tchunk, ddm_stream_t stream) {
    if (!R || !Tpre || !Tchunk || chunk0 < 0 || nchunk < 0 || batch_len < 2 || batch_len > 256) {
        ddm::set_error("ddm_shuffle_tables: invalid argument");
        return DDM_E_ARG;
    }
    if (nchunk == 0) return 0;
    const int64_t blocks = ddm::ceil_div(nchunk, (int64_t)kPreChunks);
    hipLaunchKernelGGL(k_fsm_prefix, dim3((unsigned)blocks), dim3(kPreThreads), prefix_lds_bytes(batch_len),
                       ddm::as_hip(stream), R, chunk0, nchunk, (int)batch_len, Tpre, Tchunk);
    return ddm::launch_status("ddm_shuffle_tables");
}

extern "C" int ddm_shuffle_tables_batch(const ddm_table_job* jobs_dev, int32_t n_jobs, int64_t max_chunks,
                                        int32_t batch_len, ddm_stream_t stream) {
    if (!jobs_dev || n_jobs < 0 || max_chunks < 0 || batch_len < 2 || batch_len > 256) {
        ddm::set_error("ddm_shuffle_tables_batch: invalid argument");
        return DDM_E_ARG;
    }
    if (n_jobs == 0 || max_chunks == 0) return 0;
    static_assert(sizeof(TabJob) == sizeof(ddm_table_job), "TabJob must mirror ddm_table_job");
    const int64_t blocks = ddm::ceil_div(max_chunks, (int64_t)kPreChunks);
    hipLaunchKernelGGL(k_fsm_prefix_batch, dim3((unsigned)blocks, (unsigned)n_jobs), dim3(kPreThreads),
                       prefix_lds_bytes(batch_len), ddm::as_hip(stream), reinterpret_cast<const TabJob*>(jobs_dev),
                       (int)batch_len);
    return ddm::launch_status("ddm_shuffle_tables_batch");
}

extern "C" int ddm_shuffle_window(const uint32_t* R, const uint32_t* Tpre, const uint32_t* Tchunk, int64_t avail,
                                  int64_t P, int64_t W, int32_t batch_len, void* pieces, int64_t max_pieces,
                                  int64_t* info, uint8_t* J, int64_t* E, uint8_t* perm_out, uint16_t* first,
                                  ddm_stream_t stream, ddm_event_t ev_begin, ddm_event_t ev_end) {
    if (!R || !Tpre || !Tchunk || !pieces || !info || !J || !E || !perm_out || !first || P < 0 || W <= 0 ||
        batch_len < 2 || batch_len > 256 || max_pieces < 2 + kSubPerChunk + (W * batch_len * 3) / kChunk) {
        ddm::set_error("ddm_shuffle_window: invalid argument");
        return DDM_E_ARG;
    }
    hipStream_t s = ddm::as_hip(stream);
    Job j{R, Tpre, Tchunk, avail, P, W, pieces, info, J, E, perm_out, nullptr, 0, 0, nullptr, first};
    if (ev_begin)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_begin), s), "event record")) return rc;
    hipLaunchKernelGGL(k_fsm_first, dim3(kSubPerChunk - 1), dim3(kFirstThreads), 0, s, j, (int)batch_len);
    if (int rc = ddm::launch_status("ddm_shuffle_window/first")) return rc;
    hipLaunchKernelGGL(k_fsm_walk, dim3(1), dim3(kWalkThreads), walk_lds_bytes(batch_len), s, j, (int)batch_len);
    if (int rc = ddm::launch_status("ddm_shuffle_window/walk")) return rc;
    const int64_t blocks = std::min<int64_t>(max_pieces, 8192);
    hipLaunchKernelGGL(k_fsm_replay, dim3((unsigned)blocks), dim3(64), 0, s, j, (int)batch_len);
    if (int rc = ddm::launch_status("ddm_shuffle_window/replay")) return rc;
    hipLaunchKernelGGL(k_fsm_perms, dim3((unsigned)ddm::ceil_div(W, 256)), dim3(256), (size_t)256 * batch_len, s, j,
                       (int)batch_len);
    if (int rc = ddm::launch_status("ddm_shuffle_window/perms")) return rc;
    if (ev_end)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_end), s), "event record")) return rc;
    return 0;
}
