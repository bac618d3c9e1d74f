// Batch shuffles on the GPU: pandas `sample(frac=1)` (DDM_Process.py:187, :190) ==
// numpy legacy RandomState.permutation on the global MT19937, reproduced draw for draw.
//
// The reference consumes one sequential MT19937 stream per partition: for every batch a
// Fisher-Yates pass whose intervals i = L-1..1 each take the first draw v with
// (v & mask(i)) <= i (mask(i) = smallest 2^k-1 >= i; rejected draws are skipped).  On
// the host that chain is latency bound (~10 ns/row).  Here it is made parallel:
//   1. k_mt_generate   one workgroup per partition emits the raw tempered stream R;
//                      a 624-word block is regenerated in LDS in three barrier phases.
//   2. k_fsm_sub       interval acceptance is a finite-state machine whose state is the
//                      interval index s in [1, L-1] (s == 1 accepted -> batch done,
//                      s := L-1).  For every 128-draw sub-chunk and EVERY start state a
//                      lane simulates the sub-chunk: table (end state, batches done).
//   3. k_fsm_chunk     composes 64 sub-chunk tables into 8192-draw chunk tables.
//   4. k_fsm_walk      one lane walks chunk tables from a window start (a batch
//                      boundary at draw P) to find every chunk's start (state, batch).
//   5. k_fsm_replay    one wave per chunk: lane 0 composes the sub-chunk tables, then
//                      each lane replays its 128 draws and records, per batch, the j of
//                      every interval and the draw that completes the batch.
//   6. k_fsm_perms     one lane per batch applies its L-1 swaps -> perm bytes in HBM.
// Steps 2-3 depend only on the RNG stream (not on drifts), so they run once per stream
// segment; 4-6 run per speculative window.  Tempering is invertible, so the host
// recovers the exact numpy (key, pos) state at any draw from R.
#include "common.h"

namespace {

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
__device__ void mt_generate(uint32_t* __restrict__ state, uint32_t* __restrict__ R, int64_t n) {
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
    mt_generate(state, R, n);
}

// g(T) * key on the device.  T^i(key) is the window (x_i .. x_{i+623}) of the MT19937
// word sequence that starts with key (x_{k+624} = f(x_k, x_{k+1}, x_{k+397})), so by
// linearity g(T) * key = XOR over the set coefficients i of g of those windows:
//   1. the sequence x_0 .. x_{623 + deg g} (untempered) is generated into scratch, a
//      624-word block per three barrier phases;
//   2. thread j accumulates out[j] = XOR_i x_{i+j} over the ~10k set bits of g (coalesced
//      reads across the threads, the bit scan uniform).
struct JumpJob {
    const uint32_t* key;
    const uint64_t* poly;
    uint32_t* out;
    uint32_t* scratch;
};

__global__ __launch_bounds__(256) void k_mt_jump(const JumpJob* __restrict__ jobs) {
    __shared__ uint64_t P[DDM_MT_POLY_WORDS];
    __shared__ uint32_t blk[2][kN];
    __shared__ int top_s;
    const JumpJob jb = jobs[blockIdx.x];
    const int t = threadIdx.x;
    if (t == 0) top_s = -1;
    for (int k = t; k < DDM_MT_POLY_WORDS; k += 256) P[k] = jb.poly[k];
    for (int k = t; k < kN; k += 256) {
        blk[0][k] = jb.key[k];
        jb.scratch[k] = jb.key[k];
    }
    __syncthreads();
    for (int k = t; k < DDM_MT_POLY_WORDS; k += 256)
        if (P[k]) atomicMax(&top_s, 64 * k + 63 - __builtin_clzll(P[k]));
    __syncthreads();
    const int top = top_s;
    // 1. x_624 .. x_{623 + top}: whole blocks
    int cur = 0;
    for (int64_t base = kN; base < kN + top; base += kN) {
        const uint32_t* o = blk[cur];
        uint32_t* w = blk[cur ^ 1];
        if (t < 227) {
            const uint32_t v = mt_word(o[t], o[t + 1], o[t + 397]);
            w[t] = v;
            jb.scratch[base + t] = v;
        }
        __syncthreads();
        if (t < 227) {
            const int i = 227 + t;
            const uint32_t v = mt_word(o[i], o[i + 1], w[t]);
            w[i] = v;
            jb.scratch[base + i] = v;
        }
        __syncthreads();
        if (t < 170) {
            const int i = 454 + t;
            const uint32_t v = (i < kN - 1) ? mt_word(o[i], o[i + 1], w[i - 227]) : mt_word(o[kN - 1], w[0], w[396]);
            w[i] = v;
            jb.scratch[base + i] = v;
        }
        __syncthreads();
        cur ^= 1;
    }
    __threadfence_block();
    __syncthreads();
    // 2. out[j] = XOR over set bits i of x_{i+j}
    uint32_t a0 = 0, a1 = 0, a2 = 0;
    const uint32_t* x = jb.scratch;
    for (int wd = 0; wd * 64 <= top; ++wd) {
        uint64_t bits = P[wd];
        while (bits) {
            const int i = 64 * wd + __builtin_ctzll(bits);
            bits &= bits - 1;
            a0 ^= x[i + t];
            a1 ^= x[i + t + 256];
            if (t < kN - 512) a2 ^= x[i + t + 512];
        }
    }
    jb.out[t] = top >= 0 ? a0 : 0u;
    jb.out[t + 256] = top >= 0 ? a1 : 0u;
    if (t < kN - 512) jb.out[t + 512] = top >= 0 ? a2 : 0u;
    if (t == 0) jb.out[kN] = kN;
}

struct GenJob {
    uint32_t* state;
    uint32_t* R;
    int64_t n;
};

__global__ __launch_bounds__(256) void k_mt_generate_batch(const GenJob* __restrict__ jobs) {
    const GenJob j = jobs[blockIdx.x];
    mt_generate(j.state, j.R, j.n);
}

// Tsub[sub][s-1] = end_state | batches_done << 8, for s in [1, L-1].  A 256-thread block
// serves 256 / G sub-chunks at once, G = the start states rounded up to a wave multiple
// (L = 100: two sub-chunks of 99 states per block, 77% of the lanes busy).
__global__ __launch_bounds__(256) void k_fsm_sub(const uint32_t* __restrict__ R, int64_t sub0, int64_t nsub,
                                                 int L, uint16_t* __restrict__ Tsub) {
    __shared__ uint32_t draws[4][kSub];
    const int S = L - 1;
    const int G = (S + 63) & ~63;               // lanes per sub-chunk
    const int per = 256 / G >= 1 ? 256 / G : 1; // sub-chunks per block (1, 2 or 4)
    const int q = threadIdx.x / G, lane_s = threadIdx.x % G;
    for (int64_t sb0 = sub0 + (int64_t)blockIdx.x * per; sb0 < sub0 + nsub; sb0 += (int64_t)gridDim.x * per) {
        __syncthreads();
        for (int k = threadIdx.x; k < per * kSub; k += 256) {
            const int64_t sb = sb0 + k / kSub;
            draws[k / kSub][k % kSub] = sb < sub0 + nsub ? R[sb * kSub + k % kSub] : 0u;
        }
        __syncthreads();
        const int64_t sb = sb0 + q;
        if (q >= per || sb >= sub0 + nsub) continue;
        for (int s0 = lane_s + 1; s0 <= S; s0 += G) {
            uint32_t s = (uint32_t)s0, done = 0;
            for (int k = 0; k < kSub; ++k) {
                const bool acc = (draws[q][k] & imask(s)) <= s;
                const bool wrap = acc && s == 1;
                done += wrap ? 1u : 0u;
                s = wrap ? (uint32_t)S : (acc ? s - 1 : s);
            }
            Tsub[sb * S + (s0 - 1)] = (uint16_t)(s | (done << 8));
        }
    }
}

// Tchunk[c][s-1] = end_state | batches_done << 8 over 64 sub-chunks.
__global__ __launch_bounds__(256) void k_fsm_chunk(const uint16_t* __restrict__ Tsub, int64_t chunk0, int64_t nchunk,
                                                   int L, uint32_t* __restrict__ Tchunk) {
    const int S = L - 1;
    for (int64_t c = chunk0 + blockIdx.x; c < chunk0 + nchunk; c += gridDim.x) {
        for (int s0 = threadIdx.x + 1; s0 <= S; s0 += 256) {
            uint32_t s = (uint32_t)s0, done = 0;
            const uint16_t* t = Tsub + c * kSubPerChunk * S;
            for (int k = 0; k < kSubPerChunk; ++k) {
                const uint32_t e = t[(int64_t)k * S + (s - 1)];
                s = e & 0xffu;
                done += e >> 8;
            }
            Tchunk[c * S + (s0 - 1)] = s | (done << 8);
        }
    }
}

struct Job {
    const uint32_t* R;
    const uint16_t* Tsub;
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
};

struct ChunkStart {
    int64_t pos;      // first draw of this window piece
    int32_t state;    // interval index at pos
    int32_t batch;    // batches completed (relative to the window) before pos
};

// From draw P at a batch boundary, walk to the first chunk boundary (draw by draw, then
// by sub-chunk tables) and then chunk by chunk until W batches are done.  The chunk
// table rows are staged in LDS 64 chunks at a time (all lanes load, lane 0 walks), so
// the serial walk does LDS lookups, not dependent HBM loads.
// out[0] = the piece [P, first chunk boundary); out[k] = chunk starts.
// info = {pieces, end draw, batches reached}.
__device__ void fsm_walk(const uint32_t* __restrict__ R, const uint16_t* __restrict__ Tsub,
                         const uint32_t* __restrict__ Tchunk, int64_t P, int64_t W, int L, int64_t avail,
                         ChunkStart* __restrict__ out, int64_t* __restrict__ info) {
    extern __shared__ uint32_t tab[];   // [64][S] chunk rows; phase A: draws + sub-chunk rows
    __shared__ int64_t sh_pos, sh_batch, sh_k;
    __shared__ uint32_t sh_s;
    const int S = L - 1;
    // phase A inputs: the draws up to the next sub-chunk boundary and the sub-chunk rows up
    // to the next chunk boundary, staged in LDS by all lanes
    const int64_t sub_end = min(avail, (P / kSub + 1) * kSub);
    const int64_t chunk_end = min(avail, (P / kChunk + 1) * kChunk);
    const int n_draws = (int)max((int64_t)0, sub_end - P);
    const int64_t first_sub = sub_end / kSub;
    const int n_subrows = (int)max((int64_t)0, (chunk_end - sub_end) / kSub);
    uint32_t* a_draws = tab;
    uint16_t* a_sub = reinterpret_cast<uint16_t*>(tab + kSub);
#pragma unroll 2
    for (int k = threadIdx.x; k < n_draws; k += 64) a_draws[k] = R[P + k];
#pragma unroll 8
    for (int e = threadIdx.x; e < n_subrows * S; e += 64) a_sub[e] = Tsub[first_sub * S + e];
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t pos = P, batch = 0, k = 0;
        uint32_t s = (uint32_t)S;
        out[k++] = ChunkStart{pos, (int32_t)s, 0};
        while (batch < W && pos < sub_end) {
            const uint32_t v = a_draws[pos - P];
            ++pos;
            if ((v & imask(s)) <= s) {
                if (s == 1) {
                    s = (uint32_t)S;
                    ++batch;
                } else {
                    --s;
                }
            }
        }
        while (batch < W && pos % kChunk != 0 && pos + kSub <= avail) {
            const uint32_t e = a_sub[(pos / kSub - first_sub) * S + (s - 1)];
            s = e & 0xffu;
            batch += e >> 8;
            pos += kSub;
        }
        sh_pos = pos;
        sh_batch = batch;
        sh_k = k;
        sh_s = s;
    }
    __syncthreads();
    for (;;) {
        const int64_t pos0 = sh_pos;
        if (sh_batch >= W || pos0 + kChunk > avail) break;
        const int64_t c0 = pos0 / kChunk;
        const int nload = (int)min((int64_t)64, (avail - pos0) / kChunk);
        __syncthreads();
#pragma unroll 8
        for (int e = threadIdx.x; e < nload * S; e += 64) tab[e] = Tchunk[c0 * S + e];
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t pos = pos0, batch = sh_batch, k = sh_k;
            uint32_t s = sh_s;
            for (int c = 0; c < nload && batch < W; ++c) {
                out[k++] = ChunkStart{pos, (int32_t)s, (int32_t)batch};
                const uint32_t e = tab[c * S + (s - 1)];
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
    }
    if (threadIdx.x == 0) {
        info[0] = sh_k;
        info[1] = sh_pos;
        info[2] = sh_batch;
    }
}

__global__ __launch_bounds__(64) void k_fsm_walk(Job j, int L) {
    fsm_walk(j.R, j.Tsub, j.Tchunk, j.P, j.W, L, j.avail, reinterpret_cast<ChunkStart*>(j.pieces), j.info);
}

__global__ __launch_bounds__(64) void k_fsm_walk_batch(const Job* __restrict__ jobs, int L) {
    const Job j = jobs[blockIdx.x];
    if (j.W <= 0) return;
    fsm_walk(j.R, j.Tsub, j.Tchunk, j.P, j.W, L, j.avail, reinterpret_cast<ChunkStart*>(j.pieces), j.info);
}

// One wave per window piece.  The chunk's sub-chunk table rows are staged in LDS (16-byte
// loads) together with the draws of the piece's first and last sub-chunk (the only ones
// lane 0 may have to step draw by draw); lane 0 derives every sub-chunk's start (state,
// batch); then each lane replays one sub-chunk straight from HBM, 16 draws per round of
// loads: for each accepted draw of batch b < W record J[b*L + s] = v & mask(s) and, when
// s == 1, E[b] = draw index.  (LDS per wave ~13 KB, so a CU holds many pieces at once.)
constexpr int kReplayBatch = 16;

__device__ void fsm_replay(const uint32_t* __restrict__ R, const uint16_t* __restrict__ Tsub,
                           const ChunkStart* __restrict__ pieces, const int64_t* __restrict__ info, int64_t W, int L,
                           uint8_t* __restrict__ J, int64_t* __restrict__ E, int64_t blk, int64_t nblk) {
    extern __shared__ __attribute__((aligned(16))) uint32_t rep_lds[];   // [64][S] sub-chunk rows (u16)
    uint16_t* subtab = reinterpret_cast<uint16_t*>(rep_lds);
    __shared__ uint32_t edge[2][kSub];
    __shared__ int64_t sub_pos[kSubPerChunk + 2];
    __shared__ int32_t sub_state[kSubPerChunk + 2], sub_batch[kSubPerChunk + 2];
    __shared__ int n_subs;
    const int64_t npieces = info[0], end = info[1];
    const int S = L - 1;
    for (int64_t pc = blk; pc < npieces; pc += nblk) {
        const ChunkStart c = pieces[pc];
        const int64_t stop = (pc + 1 < npieces) ? pieces[pc + 1].pos : end;
        if (stop <= c.pos) continue;
        // the chunk's sub-chunk rows: 64 * S u16 = 8 * S uint4, 16-byte aligned (the chunk's
        // rows start at chunk * 128 * S bytes); rows past the piece are not read below
        const int64_t chunk = c.pos / kChunk;
        const int64_t first_sub = chunk * kSubPerChunk;
        {
            const uint4* src = reinterpret_cast<const uint4*>(Tsub + first_sub * S);
            uint4* dst = reinterpret_cast<uint4*>(subtab);
#pragma unroll 4
            for (int e = threadIdx.x; e < 8 * S; e += 64) dst[e] = src[e];
        }
        const int64_t sA = c.pos / kSub, sB = (stop - 1) / kSub;
        for (int k = threadIdx.x; k < kSub; k += 64) {
            edge[0][k] = R[sA * kSub + k];
            edge[1][k] = R[sB * kSub + k];
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t pos = c.pos;
            uint32_t s = (uint32_t)c.state;
            int32_t b = c.batch;
            int n = 0;
            while (pos < stop) {
                sub_pos[n] = pos;
                sub_state[n] = (int32_t)s;
                sub_batch[n] = b;
                ++n;
                const int64_t nxt = min(stop, (pos / kSub + 1) * kSub);
                if (pos % kSub == 0 && nxt - pos == kSub) {
                    const uint32_t e = subtab[(pos / kSub - first_sub) * S + (s - 1)];
                    s = e & 0xffu;
                    b += (int32_t)(e >> 8);
                } else {
                    const uint32_t* d = edge[pos / kSub == sA ? 0 : 1] - (pos / kSub) * kSub;
                    for (int64_t q = pos; q < nxt; ++q) {
                        const uint32_t v = d[q];
                        if ((v & imask(s)) <= s) {
                            if (s == 1) {
                                s = (uint32_t)S;
                                ++b;
                            } else {
                                --s;
                            }
                        }
                    }
                }
                pos = nxt;
            }
            sub_pos[n] = stop;
            n_subs = n;
        }
        __syncthreads();
        for (int t = threadIdx.x; t < n_subs; t += 64) {
            uint32_t s = (uint32_t)sub_state[t];
            int64_t b = sub_batch[t];
            const int64_t beg = sub_pos[t], fin = sub_pos[t + 1];
            for (int64_t q0 = beg; q0 < fin && b < W; q0 += kReplayBatch) {
                uint32_t v[kReplayBatch];
#pragma unroll
                for (int k = 0; k < kReplayBatch; ++k) v[k] = R[min(q0 + k, fin - 1)];
#pragma unroll
                for (int k = 0; k < kReplayBatch; ++k) {
                    if (q0 + k < fin && b < W) {
                        const uint32_t m = v[k] & imask(s);
                        if (m <= s) {
                            J[b * L + s] = (uint8_t)m;
                            if (s == 1) {
                                E[b] = q0 + k;
                                s = (uint32_t)S;
                                ++b;
                            } else {
                                --s;
                            }
                        }
                    }
                }
            }
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(64) void k_fsm_replay(Job j, int L) {
    fsm_replay(j.R, j.Tsub, reinterpret_cast<const ChunkStart*>(j.pieces), j.info, j.W, L, j.J, j.E, blockIdx.x,
               gridDim.x);
}

__global__ __launch_bounds__(64) void k_fsm_replay_batch(const Job* __restrict__ jobs, int L) {
    const Job j = jobs[blockIdx.y];
    if (j.W <= 0) return;
    fsm_replay(j.R, j.Tsub, reinterpret_cast<const ChunkStart*>(j.pieces), j.info, j.W, L, j.J, j.E, blockIdx.x,
               gridDim.x);
}

// One lane per batch: Fisher-Yates swaps i = L-1..1 with the recorded j's.
__device__ void fsm_perms(const uint8_t* __restrict__ J, int64_t W, int L, uint8_t* __restrict__ perm, int64_t b0) {
    extern __shared__ uint8_t buf[];
    const int64_t b = b0 + threadIdx.x;
    if (b >= W) return;
    uint8_t* p = buf + threadIdx.x * L;
    for (int k = 0; k < L; ++k) p[k] = (uint8_t)k;
    const uint8_t* j = J + b * L;
    for (int i = L - 1; i >= 1; --i) {
        const int jj = j[i];
        const uint8_t t = p[i];
        p[i] = p[jj];
        p[jj] = t;
    }
    for (int k = 0; k < L; ++k) perm[b * L + k] = p[k];
}

__global__ __launch_bounds__(256) void k_fsm_perms(Job j, int L) {
    fsm_perms(j.J, j.W, L, j.perm_out, (int64_t)blockIdx.x * 256);
}

__global__ __launch_bounds__(256) void k_fsm_perms_batch(const Job* __restrict__ jobs, int L) {
    const Job j = jobs[blockIdx.y];
    for (int64_t b0 = (int64_t)blockIdx.x * 256; b0 < j.W; b0 += (int64_t)gridDim.x * 256)
        fsm_perms(j.J, j.W, L, j.perm_out, b0);
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
    return std::max((size_t)64 * (L - 1) * sizeof(uint32_t),
                    kSub * sizeof(uint32_t) + (size_t)kSubPerChunk * (L - 1) * sizeof(uint16_t));
}

size_t replay_lds_bytes(int L) { return (size_t)kSubPerChunk * (L - 1) * sizeof(uint16_t); }

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
    hipLaunchKernelGGL(k_fsm_walk_batch, dim3((unsigned)n_jobs), dim3(64), walk_lds_bytes(batch_len), s, jobs,
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
    static_assert(DDM_MT_JUMP_SCRATCH_WORDS >= kN * ((kN + 64 * DDM_MT_POLY_WORDS + kN - 1) / kN + 1),
                  "jump scratch holds the whole blocks of x_0 .. x_{623 + deg}");
    hipLaunchKernelGGL(k_mt_jump, dim3((unsigned)n_jobs), dim3(256), 0, ddm::as_hip(stream),
                       reinterpret_cast<const JumpJob*>(jobs_dev));
    return ddm::launch_status("ddm_mt_jump");
}

extern "C" int ddm_shuffle_tables(const uint32_t* R, int64_t chunk0, int64_t nchunk, int32_t batch_len,
                                  uint16_t* Tsub, uint32_t* Tchunk, ddm_stream_t stream) {
    if (!R || !Tsub || !Tchunk || chunk0 < 0 || nchunk < 0 || batch_len < 2 || batch_len > 256) {
        ddm::set_error("ddm_shuffle_tables: invalid argument");
        return DDM_E_ARG;
    }
    if (nchunk == 0) return 0;
    hipStream_t s = ddm::as_hip(stream);
    const int64_t nsub = nchunk * kSubPerChunk;
    hipLaunchKernelGGL(k_fsm_sub, dim3((unsigned)std::min<int64_t>(nsub, 65536)), dim3(256), 0, s, R,
                       chunk0 * kSubPerChunk, nsub, (int)batch_len, Tsub);
    if (int rc = ddm::launch_status("ddm_shuffle_tables/sub")) return rc;
    hipLaunchKernelGGL(k_fsm_chunk, dim3((unsigned)std::min<int64_t>(nchunk, 65536)), dim3(256), 0, s, Tsub, chunk0,
                       nchunk, (int)batch_len, Tchunk);
    return ddm::launch_status("ddm_shuffle_tables/chunk");
}

extern "C" int ddm_shuffle_window(const uint32_t* R, const uint16_t* Tsub, const uint32_t* Tchunk, int64_t avail,
                                  int64_t P, int64_t W, int32_t batch_len, void* pieces, int64_t max_pieces,
                                  int64_t* info, uint8_t* J, int64_t* E, uint8_t* perm_out, ddm_stream_t stream,
                                  ddm_event_t ev_begin, ddm_event_t ev_end) {
    if (!R || !Tsub || !Tchunk || !pieces || !info || !J || !E || !perm_out || P < 0 || W <= 0 ||
        batch_len < 2 || batch_len > 256 || max_pieces < 2 + (W * batch_len * 3) / kChunk) {
        ddm::set_error("ddm_shuffle_window: invalid argument");
        return DDM_E_ARG;
    }
    hipStream_t s = ddm::as_hip(stream);
    Job j{R, Tsub, Tchunk, avail, P, W, pieces, info, J, E, perm_out, nullptr, 0, 0, nullptr};
    if (ev_begin)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_begin), s), "event record")) return rc;
    hipLaunchKernelGGL(k_fsm_walk, dim3(1), dim3(64), walk_lds_bytes(batch_len), s, j, (int)batch_len);
    if (int rc = ddm::launch_status("ddm_shuffle_window/walk")) return rc;
    const int64_t blocks = std::min<int64_t>(max_pieces, 8192);
    hipLaunchKernelGGL(k_fsm_replay, dim3((unsigned)blocks), dim3(64), replay_lds_bytes(batch_len), s, j,
                       (int)batch_len);
    if (int rc = ddm::launch_status("ddm_shuffle_window/replay")) return rc;
    hipLaunchKernelGGL(k_fsm_perms, dim3((unsigned)ddm::ceil_div(W, 256)), dim3(256), (size_t)256 * batch_len, s, j,
                       (int)batch_len);
    if (int rc = ddm::launch_status("ddm_shuffle_window/perms")) return rc;
    if (ev_end)
        if (int rc = ddm::hip_status(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_end), s), "event record")) return rc;
    return 0;
}
