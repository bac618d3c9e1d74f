// Epoch read-back staging: everything the host needs after an epoch, gathered on the
// device so that ONE device->host copy and ONE synchronisation close the epoch.
//
// After the batched shuffle / predict / scan of an epoch the controller has to learn,
// per partition (run_DDM_loop, DDM_Process.py:170-213):
//   * the batches with a warning or a change (DDM_Process.py:147-152, :204): compacted
//     here into (window batch, warning, change) records instead of copying every row;
//   * on a change in batch d (:207-210): the new training batch = batch d in its shuffled
//     order (`batch_a = batch_b`, :208), i.e. X rows d*pb + perm[d*pb + k] and labels, and
//     the stream words from the draw after batch d's shuffle, where batch d+1's shuffle
//     and then the refit's 100 tree seeds are drawn (:190, :102).
// It also draws what the reference draws next from the same stream: batch d+1's
// shuffle (written into the partition's perm array, DDM_Process.py:190) and the T tree
// seeds of the refit (:102), from words staged in LDS (one lane runs Fisher-Yates).
// One workgroup per partition; nothing here decides anything, the host still does.
#include <cstddef>

#include "common.h"
#include "ctl_dev.h"
#include "scan_fast.h"

namespace {

constexpr int kStageThreads = 1024;
constexpr int kStageWords = 1024;   // stream words in LDS for one shuffle + the seeds

using ddm::gptr;
struct Job {
    gptr<const float> X;
    int64_t ld;
    gptr<const int32_t> y;
    gptr<const uint8_t> perm;
    int64_t base;
    gptr<const int32_t> ev;
    gptr<const int32_t> stop;
    gptr<const int64_t> pick;
    gptr<const uint32_t> R;
    int64_t j, g0, nb, b_end, p_after_first, p_tail_after;
    int32_t pb, last_len, n_features, n_words, tail, max_events;
    gptr<float> x_out;
    gptr<int32_t> y_out;
    gptr<uint32_t> w_out;
    gptr<int64_t> info_out;
    gptr<int32_t> ev_out;
    gptr<uint8_t> perm_w;
    gptr<int64_t> seeds_out;
    int32_t n_trees, win_rule;
    int64_t p_now, win, max_win, seg_start, n_full, min_win, next_avail, dpb_x1024;
    gptr<int64_t> plan_out;
    ddm_shuffle_job* next_job;
    gptr<int32_t> log;
    gptr<int64_t> log_n;
    int64_t log_cap;
    gptr<const int32_t> stall;
};
static_assert(sizeof(Job) == sizeof(ddm_stage_job), "Job must mirror ddm_stage_job");

// The next window as BatchRunner._epoch_after + _epoch would set it (controller.py), for
// the common cases only: a change whose batch d+1 shuffle and seeds were drawn here (the
// refit goes through, on the device or the host, from the draw after the seeds), or no
// change at all; windows reaching a short last batch stay with the host.  Written by one
// thread; W = 0 when not planned.
__device__ void plan_next(const Job& jb, int32_t stop, bool drawn, int64_t p_seeds, int64_t pickv) {
    int64_t jn, Pn, g0n, winn;
    bool ok = true;
    if (stop >= 0) {
        const int64_t d = jb.j + stop;
        jn = d + 1;
        Pn = p_seeds;
        g0n = jn + 1;
        winn = drift_window(d - jb.seg_start + 1, jb.min_win, jb.win_rule);
        ok = drawn;
    } else {
        jn = jb.b_end;
        ok = jb.tail == 0;
        const int64_t Wg = max((int64_t)0, min(jb.b_end, jb.n_full) - jb.g0);
        Pn = Wg > 0 ? pickv + 1 : (jb.p_after_first >= 0 ? jb.p_after_first : jb.p_now);
        g0n = jn;
        winn = jb.win * 2;
    }
    int64_t Wn = 0, bn = 0;
    if (jn < jb.nb) {
        bn = min(jb.nb, jn + min(winn, jb.max_win));
        Wn = max((int64_t)0, min(bn, jb.n_full) - g0n);
        if (bn == jb.nb && jb.last_len != jb.pb && jb.nb - 1 >= g0n) ok = false;   // a host-shuffled tail
        // the draws the window may need (the host's window_draws, rounded up) are tabulated
        if (Pn + (Wn * jb.dpb_x1024 * 115 + 102399) / 102400 + 4 * 8192 > jb.next_avail) ok = false;
    } else {
        ok = false;
    }
    if (!ok) Wn = 0;
    gptr<int64_t> po = jb.plan_out;
    po[0] = Pn;
    po[1] = Wn;
    po[2] = g0n;
    po[3] = bn;
    po[4] = jn;
    po[5] = ok ? 1 : 0;
    if (jb.next_job) {
        jb.next_job->P = Pn;
        jb.next_job->W = Wn;
        jb.next_job->perm_out = (uint8_t*)(gptr<uint8_t>)jb.perm + jb.base + g0n * jb.pb;
        jb.next_job->avail = jb.next_avail;
    }
}

// One partition's staging (the workgroup's); pickv: the RNG position the pick found (the
// draw before the window's first unused batch shuffle), read where the host's pick is.
// pos_next >= 0: batch d + 1 of a change in batch d lies in the window, whose shuffles
// (ddm_shuffle_window_batch) already drew it from the draw after batch d's shuffle, as the
// reference does (DDM_Process.py:190 follows :187/:190 of batch d directly); its perm bytes
// are in place and pos_next is the draw after it, so only the seeds are drawn here.
__device__ void stage_body(const Job& jb, int64_t pickv, int64_t pos_next = -1) {
    __shared__ int counts[kStageThreads / 64];
#ifdef DDM_STAGE_PROFILE
    const uint64_t t0 = wall_clock64();
#define STAGE_MARK(k) do { if (threadIdx.x == 0) s_mark[k] = wall_clock64(); } while (0)
    __shared__ uint64_t s_mark[6];
#else
#define STAGE_MARK(k) do { } while (0)
#endif
    const int t = threadIdx.x;
    if (jb.stall && *jb.stall) {            // device-resident runner: this partition waits for the host
        if (t == 0) {
            jb.info_out[0] = -1;
            jb.info_out[1] = 0;
            jb.info_out[2] = 0;
            jb.info_out[3] = -1;
            jb.info_out[6] = 0;
        }
        return;
    }
    const int32_t stop = *jb.stop;
    const int64_t last = stop >= 0 ? jb.j + stop : jb.b_end - 1;   // last batch the scan covered
    const int64_t nrows = last - jb.j + 1;                         // window rows of ev to look at
    // ---- compact the event rows, in row order: per round every thread reads 8 consecutive
    // rows with four 16-byte loads (the whole block 2048 rows, coalesced, one memory
    // latency per round), then a block prefix of the per-thread counts places them
    const int lane = t & 63, wv = t >> 6;
    int total = 0;
    // device-resident runner: records go to the partition's event log (absolute batches)
    const int64_t log0 = jb.log ? *jb.log_n : 0;
    const int64_t cap = jb.log ? jb.log_cap - log0 : (int64_t)jb.max_events;
    // no log and no staging room: the scan logged the events itself (device-resident runner)
    const int64_t nscan = (jb.log || jb.max_events > 0) ? nrows : 0;
    for (int64_t base = 0; base < nscan; base += 8 * kStageThreads) {
        const int64_t r0 = base + 8 * (int64_t)t;
        int4 q[4];
        const bool vec = r0 + 8 <= nrows && ((reinterpret_cast<uintptr_t>(jb.ev + 2 * r0) & 15) == 0);
        if (vec) {
#pragma unroll
            for (int k = 0; k < 4; ++k) q[k] = ddm::ld_int4(jb.ev + 2 * r0 + 4 * k);
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int64_t ra = r0 + 2 * k, rb = ra + 1;
                q[k].x = ra < nrows ? jb.ev[2 * ra] : -1;
                q[k].y = ra < nrows ? jb.ev[2 * ra + 1] : -1;
                q[k].z = rb < nrows ? jb.ev[2 * rb] : -1;
                q[k].w = rb < nrows ? jb.ev[2 * rb + 1] : -1;
            }
        }
        uint32_t bits = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            bits |= (uint32_t)(q[k].x >= 0 || q[k].y >= 0) << (2 * k);
            bits |= (uint32_t)(q[k].z >= 0 || q[k].w >= 0) << (2 * k + 1);
        }
        int c = __popc(bits);
        int incl = c;                                   // inclusive prefix over the wave
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int u = __shfl_up(incl, o, 64);
            if (lane >= o) incl += u;
        }
        if (lane == 63) counts[wv] = incl;
        __syncthreads();
        int before = total;
        for (int w = 0; w < wv; ++w) before += counts[w];
        int round = 0;
#pragma unroll
        for (int w = 0; w < kStageThreads / 64; ++w) round += counts[w];
        int k = before + incl - c;
        gptr<int32_t> out = jb.log ? jb.log + 3 * log0 : jb.ev_out;
        const int32_t boff = jb.log ? (int32_t)jb.j : 0;
        while (bits && k < cap) {
            const int s = __builtin_ctz(bits);
            bits &= bits - 1;
            const int4 v = q[s >> 1];
            out[3 * k] = (int32_t)(r0 + s) + boff;
            out[3 * k + 1] = (s & 1) ? v.z : v.x;
            out[3 * k + 2] = (s & 1) ? v.w : v.y;
            ++k;
        }
        total += round;
        __syncthreads();
    }
    STAGE_MARK(0);
    if (t == 0) {
        jb.info_out[1] = total;
        jb.info_out[2] = total > cap ? 1 : 0;
        if (jb.log) *jb.log_n = log0 + min((int64_t)total, cap);
    }
    if (stop < 0) {
        if (t == 0) {
            jb.info_out[0] = -1;
            jb.info_out[3] = -1;
            if (jb.plan_out) plan_next(jb, stop, false, -1, pickv);
        }
        return;
    }
    // ---- a change in batch d: its rows in shuffled order and the words after its shuffle
    const int64_t d = jb.j + stop;
    const int L = d == jb.nb - 1 ? jb.last_len : jb.pb;
    int64_t P;
    if (d < jb.g0) P = jb.p_after_first;                        // the refit batch itself
    else if (jb.tail && d == jb.nb - 1) P = jb.p_tail_after;    // the short last batch
    else P = pickv + 1;
    if (t == 0) {
        jb.info_out[0] = P;
        jb.info_out[3] = d;
    }
    const int F = jb.n_features;
    // the batch's shuffle offsets once through LDS, then every thread's loads issued before
    // its stores (the pointers may alias as far as the compiler knows: a store between two
    // loads would keep the next load from being issued early)
    __shared__ uint8_t off_d[256];
    for (int kk = t; kk < L; kk += kStageThreads) off_d[kk] = jb.perm[jb.base + d * jb.pb + kk];
    __syncthreads();
    const int64_t row0 = d * jb.pb;
    for (int e0 = t; e0 < L * F; e0 += 4 * kStageThreads) {
        float xv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = e0 + u * kStageThreads;
            xv[u] = e < L * F ? jb.X[(int64_t)(e % F) * jb.ld + row0 + off_d[e / F]] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = e0 + u * kStageThreads;
            if (e < L * F) jb.x_out[e] = xv[u];
        }
    }
    for (int kk = t; kk < L; kk += kStageThreads) jb.y_out[kk] = jb.y[row0 + off_d[kk]];
    if (jb.R)
        for (int w = t; w < jb.n_words; w += kStageThreads) jb.w_out[w] = jb.R[P + w];
    STAGE_MARK(1);
    // ---- batch j = d + 1: its shuffle, then the refit's tree seeds
    __shared__ uint32_t words[kStageWords];
    __shared__ uint8_t perm[256];
    __shared__ uint8_t js[256];                 // the accepted j of every interval i
    __shared__ int64_t pos[2];
    __shared__ int ok;
    const int64_t j = d + 1;
    if (!jb.R || !jb.perm_w || !jb.seeds_out || j >= jb.nb) {
        if (t == 0) {
            jb.info_out[6] = 0;
            if (jb.plan_out) plan_next(jb, stop, false, -1, pickv);
        }
        return;
    }
    const int Lj = j == jb.nb - 1 ? jb.last_len : jb.pb;
    const bool pre = pos_next >= 0;                 // batch j shuffled by the window already
    const int64_t Pw = pre ? pos_next : P;
    for (int w = t; w < kStageWords; w += kStageThreads) words[w] = jb.R[Pw + w];
    __syncthreads();
    STAGE_MARK(2);
    if (wv == 0) {
        // legacy permutation(Lj), then randint(2**31 - 1) x n_trees, by the first wave.
        // Interval i accepts the first word w with (w & mask_i) <= i.  Speculation: lane l
        // tries interval i - l on word k + l (every interval accepting its first word); the
        // lanes before the first rejection are final, and the rejected interval searches
        // the words after it by a ballot over 64 at a time.  About a quarter of the rounds
        // of one interval per round.
        int k = 0;
        bool good = true;
        int i = pre ? 0 : Lj - 1;
        while (i >= 1) {
            const int il = i - lane, wi = k + lane;
            bool acc = false;
            uint32_t val = 0xffffffffu;
            if (il >= 1) {
                const uint32_t mask = 0xffffffffu >> __builtin_clz((uint32_t)il);
                val = wi < kStageWords ? (words[wi] & mask) : 0xffffffffu;
                acc = val <= (uint32_t)il;
            }
            const uint64_t rej = __ballot(!acc);          // lane i (il = 0) always counts
            const int r = rej ? __builtin_ctzll(rej) : 64;
            if (lane < r) js[il] = (uint8_t)val;           // swap il <-> val, applied below
            i -= r;
            k += r;
            if (i < 1 || r == 64) continue;
            // interval i rejected word k: its first accepted word after it
            const uint32_t mask = 0xffffffffu >> __builtin_clz((uint32_t)i);
            ++k;
            for (;;) {
                if (k >= kStageWords) { good = false; break; }
                const int w = k + lane;
                const uint32_t v = w < kStageWords ? (words[w] & mask) : 0xffffffffu;
                const uint64_t b = __ballot(v <= (uint32_t)i);
                if (b) {
                    const int f = __builtin_ctzll(b);
                    const int jv = __builtin_amdgcn_readlane((int)v, f);   // f is wave-uniform
                    k += f + 1;
                    if (lane == 0) js[i] = (uint8_t)jv;
                    --i;
                    break;
                }
                k += 64;
            }
            if (!good) break;
        }
        if (lane == 0) pos[0] = Pw + k;
        STAGE_MARK(3);
        int got = 0;                                                 // seeds drawn so far
        while (good && got < jb.n_trees) {
            if (k >= kStageWords) { good = false; break; }
            const int w = k + lane;
            const uint32_t v = w < kStageWords ? (words[w] & 0x7fffffffu) : 0xffffffffu;
            const bool acc = v <= 0x7ffffffeu;
            const uint64_t b = __ballot(acc);
            const int before = __popcll(b & ((1ull << lane) - 1ull));
            if (acc && got + before < jb.n_trees) jb.seeds_out[got + before] = (int64_t)v;
            const int need = jb.n_trees - got;
            const int nb = __popcll(b);
            if (nb >= need) {                                        // the need-th accepted word ends it
                uint64_t bb = b;
                for (int q = 1; q < need; ++q) bb &= bb - 1;
                k += __builtin_ctzll(bb) + 1;
                got = jb.n_trees;
            } else {
                got += nb;
                k += 64;
            }
        }
        if (lane == 0) {
            pos[1] = Pw + k;
            ok = good ? 1 : 0;
        }
    }
    __syncthreads();
    STAGE_MARK(4);
    if (!ok) {
        if (t == 0) {
            jb.info_out[6] = 0;
            if (jb.plan_out) plan_next(jb, stop, false, -1, pickv);
        }
        return;
    }
    // the swaps, all elements at once: element e starts at position e and follows the
    // transpositions i <-> js[i] for i = Lj-1 .. 1; it ends where Fisher-Yates puts it
    if (!pre && t < Lj) {
        int q = t;
#pragma unroll 8
        for (int i = Lj - 1; i >= 1; --i) {
            const int jv = js[i];
            q = q == i ? jv : (q == jv ? i : q);
        }
        perm[q] = (uint8_t)t;
    }
    __syncthreads();
    if (!pre)
        for (int i = t; i < Lj; i += kStageThreads) jb.perm_w[jb.base + j * jb.pb + i] = perm[i];
    if (t == 0) {
        jb.info_out[4] = pos[0];
        jb.info_out[5] = pos[1];
        jb.info_out[6] = 1;
        if (jb.plan_out) plan_next(jb, stop, true, pos[1], pickv);
    }
#ifdef DDM_STAGE_PROFILE
    __syncthreads();
    if (t == 0 && blockIdx.x == 0)
        printf("stage-prof compact %.2f gather %.2f words %.2f shuffle %.2f seeds %.2f swaps %.2f us\n",
               (s_mark[0] - t0) / 100.0, (s_mark[1] - s_mark[0]) / 100.0, (s_mark[2] - s_mark[1]) / 100.0,
               (s_mark[3] - s_mark[2]) / 100.0, (s_mark[4] - s_mark[3]) / 100.0, (wall_clock64() - s_mark[4]) / 100.0);
#endif
}

__global__ __launch_bounds__(kStageThreads) void k_stage(const Job* __restrict__ jobs) {
    const Job jb = jobs[blockIdx.x];
    stage_body(jb, jb.pick ? *jb.pick : -1);
}

// The one-lane DDM scan of the epoch's windows, when the fused kernel runs it (err set).
struct FoldScan {
    const uint8_t* err;
    const uint8_t* perm_map;
    ddm_params P;
    uint32_t* pub;           // non-null: the last workgroup stores pub_v there (ctl.hip's fork)
    uint32_t pub_v;
};

// The device-resident runner's epoch tail in one launch, a workgroup per partition: the
// partition's one-lane DDM scan (ddm_scan_streams_log's k_scan_fast worker; a window on
// ddm_scan_long was scanned before this launch), the pick of the RNG position
// (ddm_shuffle_pick_batch), the staging (k_stage), the partition's decisions (k_ctl's
// commit + plan); the last workgroup to finish splits the predict grid.
__global__ __launch_bounds__(kStageThreads) void k_stage_ctl(const Job* __restrict__ jobs,
                                                             const ddm_shuffle_job* __restrict__ sjobs,
                                                             const ddm_ctl c, const FoldScan fs) {
    __shared__ int64_t s_pick, s_next;
    __shared__ ddm_ctl_part s_part;
    __shared__ int s_last;
    __shared__ double s_rcp[kRcpN];
    const int t = threadIdx.x;
    const int i = (int)blockIdx.x;
    const Job jb = jobs[i];
#ifdef DDM_STAGE_PROFILE
    const uint64_t tk0 = wall_clock64();
#endif
    if (c.predict_clock && i == 0 && t < 64) {
        // the epoch's predict launch: its span on the device clock into the running sum (the
        // 16 shards read and reset by 16 lanes at once, then reduced over the wave)
        unsigned long long* clk = reinterpret_cast<unsigned long long*>(c.predict_clock);
        unsigned long long lo = ~0ull, hi = 0;
        if (t < 8) lo = atomicExch(clk + t, ~0ull);
        else if (t < 16) hi = atomicExch(clk + t, 0ull);
        for (int o = 32; o > 0; o >>= 1) {
            lo = min(lo, (unsigned long long)__shfl_xor(lo, o, 64));
            hi = max(hi, (unsigned long long)__shfl_xor(hi, o, 64));
        }
        if (t == 0 && lo != ~0ull && hi > lo) {
            atomicAdd(clk + 16, hi - lo);
            atomicAdd(clk + 17, 1ull);
        }
    }
    if (fs.err) {
        for (int k = t; k < kRcpN; k += kStageThreads) s_rcp[k] = 1.0 / (double)(k > 0 ? k : 1);
        __syncthreads();
        if (t == 0 && !(c.lend[i] > c.loff[i])) {
            const EvSink sink{nullptr, c.logs,
                              reinterpret_cast<int64_t*>(reinterpret_cast<uint8_t*>(c.parts) + offsetof(ddm_ctl_part, n_log)),
                              (int64_t)(sizeof(ddm_ctl_part) / sizeof(int64_t)), c.log_b0};
            scan_fast_worker(fs.err, c.off, c.n, fs.P, c.state, c.first, nullptr, sink, const_cast<int32_t*>(c.stop),
                             nullptr, 0, fs.perm_map, c.end, i, (int64_t)c.n, s_rcp);
            __threadfence();                        // stop, state and the log count for the block
        }
        __syncthreads();
    }
    if (t == 0) {
        const ddm_shuffle_job& sj = sjobs[i];
        int64_t v = -1, nx = -1;
        if (sj.pick_out) {
            const bool chg = sj.stop && sj.stop[0] >= 0;
            const int64_t k = (chg ? (int64_t)sj.stop[0] : sj.pick_last) - sj.pick_offset;
            v = (sj.W > 0 && k >= 0 && k < sj.W) ? sj.E[k] : -1;
            sj.pick_out[0] = v;
            // a change in batch d: batch d + 1 (window index k + 1) was shuffled by the window
            if (chg && sj.W > 0 && k + 1 >= 0 && k + 1 < sj.W) nx = sj.E[k + 1] + 1;
        }
        s_pick = v;
        s_next = nx;
    }
    __syncthreads();
#ifdef DDM_STAGE_PROFILE
    const uint64_t tk1 = wall_clock64();
#endif
    stage_body(jb, s_pick, s_next);
    __syncthreads();
#ifdef DDM_STAGE_PROFILE
    const uint64_t tk2 = wall_clock64();
#endif
    if (t < 64) ctl_record(c, i, &s_part, t, 0);
#ifdef DDM_STAGE_PROFILE
    const uint64_t tk3 = wall_clock64();
#endif
    __threadfence();
    __syncthreads();
    if (t == 0) s_last = atomicAdd(c.sync, 1u) == gridDim.x - 1;
    __syncthreads();
#ifdef DDM_STAGE_PROFILE
    const uint64_t tk4 = wall_clock64();
#endif
    if (s_last && t < 64) {
        __threadfence();
        ctl_split(c, t);
        if (t == 0) {
            c.sync[0] = 0;                          // the ticket, for the next epoch
            if (fs.pub) ddm::flag_publish(fs.pub, fs.pub_v);   // the fork (ctl.hip): every block's
        }                                                   // records are released before its ticket
    }
#ifdef DDM_STAGE_PROFILE
    if (t == 0)
        printf("stage-ctl block %d scan+pick %.2f stage %.2f record %.2f ticket %.2f split %.2f us%s\n", i,
               (tk1 - tk0) / 100.0, (tk2 - tk1) / 100.0, (tk3 - tk2) / 100.0, (tk4 - tk3) / 100.0,
               (wall_clock64() - tk4) / 100.0, s_last ? " (last)" : "");
#endif
}

}  // namespace

int epoch_stage_ctl_pub(const ddm_stage_job* jobs_dev, const ddm_shuffle_job* shuffle_jobs, const ddm_ctl* ctl,
                        const uint8_t* err, const ddm_params* prm, const uint8_t* perm_map, uint32_t* pub_flag,
                        uint32_t pub_v, ddm_stream_t stream);

// err != NULL: the kernel also runs the epoch's one-lane DDM scan (mode 0) on err with the
// params and perm_map given.
extern "C" int ddm_epoch_stage_ctl(const ddm_stage_job* jobs_dev, const ddm_shuffle_job* shuffle_jobs,
                                   const ddm_ctl* ctl, const uint8_t* err, const ddm_params* prm,
                                   const uint8_t* perm_map, ddm_stream_t stream) {
    if (!jobs_dev || !shuffle_jobs || !ctl || !ctl->sync || ctl->n <= 0 || (err && (!prm || prm->per_batch <= 0))) {
        ddm::set_error("ddm_epoch_stage_ctl: invalid argument");
        return DDM_E_ARG;
    }
    return epoch_stage_ctl_pub(jobs_dev, shuffle_jobs, ctl, err, prm, perm_map, nullptr, 0, stream);
}

// The same, storing pub_v into *pub_flag once every record is written (ctl.hip's fork).
int epoch_stage_ctl_pub(const ddm_stage_job* jobs_dev, const ddm_shuffle_job* shuffle_jobs, const ddm_ctl* ctl,
                        const uint8_t* err, const ddm_params* prm, const uint8_t* perm_map, uint32_t* pub_flag,
                        uint32_t pub_v, ddm_stream_t stream) {
    if (!jobs_dev || !shuffle_jobs || !ctl || !ctl->sync || ctl->n <= 0 || (err && (!prm || prm->per_batch <= 0))) {
        ddm::set_error("ddm_epoch_stage_ctl: invalid argument");
        return DDM_E_ARG;
    }
    FoldScan fs{err, perm_map, {}, pub_flag, pub_v};
    if (err) fs.P = *prm;
    hipLaunchKernelGGL(k_stage_ctl, dim3((unsigned)ctl->n), dim3(kStageThreads), 0, ddm::as_hip(stream),
                       reinterpret_cast<const Job*>(jobs_dev), shuffle_jobs, *ctl, fs);
    return ddm::launch_status("ddm_epoch_stage_ctl");
}

extern "C" int ddm_epoch_stage(const ddm_stage_job* jobs_dev, int32_t n_jobs, ddm_stream_t stream) {
    if (!jobs_dev || n_jobs < 0) {
        ddm::set_error("ddm_epoch_stage: invalid argument");
        return DDM_E_ARG;
    }
    if (n_jobs == 0) return 0;
    hipLaunchKernelGGL(k_stage, dim3((unsigned)n_jobs), dim3(kStageThreads), 0, ddm::as_hip(stream),
                       reinterpret_cast<const Job*>(jobs_dev));
    return ddm::launch_status("ddm_epoch_stage");
}
