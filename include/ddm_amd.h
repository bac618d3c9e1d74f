/* ddm_amd.h — C-ABI of the MI355X-native predict + DDM hot path.
 *
 * The reference hot path is the grouped-map pandas UDF `run_DDM_loop`
 * (DDM_Process.py:166-213) applied per partition (`groupby("device_id").apply`,
 * DDM_Process.py:226).  Its inner calls are replaced by these entry points:
 *
 *   ddm_forest_predict   <- predict_rf (DDM_Process.py:110-128): sklearn forest.predict
 *                           + `acc = y_pred != y` (:117), rows fed in the shuffled
 *                           order of `batch_b.sample(frac=1)` (:190)
 *   ddm_scan_streams     <- run_DDM (DDM_Process.py:135-159) over consecutive batches,
 *                           DDM state carried (:202), first warning / first change +
 *                           break per batch (:147-152), DDM dropped after a change
 *                           (:207-210)
 *   ddm_scan_long        <- run_DDM over long carried segments (wave-parallel tests,
 *                           chunk-chained carry)
 *   ddm_mt_perms         <- `DataFrame.sample(frac=1)` (:187, :190) on numpy's global
 *                           MT19937 (legacy RandomState.permutation)
 *   ddm_mt_randint31     <- the 100 `randint(2**31-1)` tree seeds RandomForestClassifier
 *                           .fit draws from the same global RNG (:102-103)
 *   ddm_mt_skip          <- re-positioning the global RNG after a speculative window
 *   ddm_rf_fit           <- train_rf (DDM_Process.py:98-105): RandomForestClassifier.fit
 *                           restated from scikit-learn 1.7.2 (identical trees), host code
 *   ddm_synth_*          <- synthetic rialto/outdoor-shaped inputs for the benchmark
 *                           (rialto.csv is not shipped, .MISSING_LARGE_BLOBS:1)
 *
 * Conventions: all device pointers are caller-owned (the library never allocates or
 * frees); every device entry point takes an explicit hipStream_t and is asynchronous,
 * re-entrant and stateless.  Return value 0 = ok, otherwise a hipError_t or one of
 * the DDM_E_* codes below; ddm_last_error() describes the last failure of the calling
 * thread.  No torch types cross this boundary.
 */
#ifndef DDM_AMD_H
#define DDM_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DDM_AMD_ABI_VERSION 24

#define DDM_E_ARG        1001   /* invalid argument (null pointer, bad size) */
#define DDM_E_FOREST     1002   /* forest shape not supported (classes > 256) */
#define DDM_E_NAN        1003   /* ddm_rf_fit: NaN in X (use sklearn for missing values) */
#define DDM_E_IMPURE     1004   /* ddm_rf_fit: impure forest needs a (larger) leaf_value buffer */

typedef struct ihipStream_t* ddm_stream_t;   /* == hipStream_t */
typedef struct ihipEvent_t* ddm_event_t;     /* == hipEvent_t  */

/* DDM parameters: DDM_Process.py:25,27-29 (PER_BATCH, MIN_NUM_DDM_VALS, WARNING_LEVEL,
 * CHANGE_LEVEL).  Reference values 100 / 3 / 0.5 / 1.5. */
typedef struct ddm_params {
    int32_t min_num_instances;
    int32_t per_batch;
    double  warning_level;
    double  out_control_level;
} ddm_params;

/* One DDM detector (scikit-multiflow DDM field names).  A freshly constructed DDM
 * (DDM_Process.py:139) is {1.0, 0.0, +inf, +inf, +inf, 1, 0, 0}. */
typedef struct ddm_state {
    double  miss_prob;          /* p      */
    double  miss_std;           /* s      */
    double  miss_prob_min;      /* p_min  */
    double  miss_sd_min;        /* s_min  */
    double  miss_prob_sd_min;   /* min of p+s */
    int64_t sample_count;       /* n      */
    int32_t in_concept_change;
    int32_t in_warning_zone;
} ddm_state;

/* Forest node, 16 bytes.  feature >= 0: internal node testing (double)x_f32[feature &
 * 0x3fffffff] <= threshold (bit 30 set: NaN goes left), children at child (left) and
 * child + 1 (right).  feature == -1: leaf, child = class index (pure forests) or row of
 * leaf_value (impure forests). */
typedef struct ddm_node {
    double  threshold;
    int32_t feature;
    int32_t child;
} ddm_node;

typedef struct ddm_forest {
    const ddm_node* nodes;       /* device [n_nodes]                               */
    const int32_t*  roots;       /* device [n_trees] root node of each tree        */
    const double*   leaf_value;  /* device [n_leaf_rows * n_classes] or NULL (pure) */
    const int32_t*  classes;     /* device [n_classes] class labels (classes_)     */
    int32_t n_trees;
    int32_t n_classes;           /* <= 64                                          */
    int32_t n_nodes;
    int32_t pure;                /* 1: every leaf is one-hot and n_trees <= 255    */
    const uint8_t*  cforest;     /* device blob of ddm_forest_compile, or NULL: then the
                                    node walk above is used                         */
    int32_t cf_slots;            /* the blob's n_slots, vote_regs, n_leaves and rank-table */
    int32_t cf_vote_regs;        /* words (kernel choice and LDS size without reading the  */
    int32_t cf_leaves;           /* blob)                                                   */
    int32_t cf_tab_words;
} ddm_forest;

/* ---- compiled forests (the fast predict path) -------------------------------------
 * A pure forest whose trees have <= 64 leaves, <= 16 classes and <= 32 distinct feature
 * columns is compiled on the host into one blob the predict kernels read with uniform
 * (scalar) loads:
 *   * the feature columns the forest reads become slots 0..n_slots-1 (a row loads only
 *     those: 4*n_slots bytes of X per row);
 *   * single-leaf trees fold into base_votes (u8 vote counters packed 4 per uint32);
 *   * stumps (one split, two leaves), NaN-right ones first: vote += right ? delta : 0
 *     with right = !(x <= thr) (NaN goes right) or x > thr (NaN goes left), thr the
 *     float32 image of the float64 threshold (x <= thr32 <=> (double)x <= thr for every
 *     float32 x) and base_votes already holding the left leaf's vote;
 *   * other trees are evaluated QuickScorer-style: every internal node whose test sends
 *     the row right clears the leaves of its left subtree from a 64-bit mask; the exit
 *     leaf is the lowest surviving bit (leaves numbered left to right).
 * Layout (byte offsets from the blob start, 16-byte aligned sections):
 *   ddm_cforest_head | stumps u32[S][stump_words] ({float32 thr bits, slot, delta[vote_regs]},
 *                                                  stump_words = 4 (vote_regs <= 2) or 8)
 *   | trees ddm_cforest_tree[n_general] | nodes ddm_cforest_node[] | leaf class u8[n_leaves]
 *   | slot records ddm_cforest_slot[n_slots] | extra thresholds float4[]
 *   | rank tables u32[entries][vote_regs]
 * The stump records are the forest's plain form (tests, tools); the kernel evaluates the
 * stumps through the per-slot rank tables (ddm_cforest_slot). */
typedef struct ddm_cforest_head {
    int32_t n_slots, n_classes, vote_regs, n_stumps;
    int32_t n_general, n_leaves, total_bytes, any_nanleft;
    int32_t stumps_off, stump_words, n_stumps_right, trees_off;  /* stumps [0, n_stumps_right)
                                                                     send NaN right */
    int32_t nodes_off, leafcls_off, pad0, pad1;
    uint32_t base_votes[4];
    int32_t cols[32];            /* feature column of each slot                          */
    int32_t classes[16];         /* classes_ labels                                      */
    int32_t slots_off, xthr_off, rank_tab_off, rank_tab_entries;  /* byte offsets, entries */
} ddm_cforest_head;

/* Per-slot stump ranks.  The m stumps on slot s have ascending thresholds t_0..t_{m-1},
 * stored as n4 = m/4 + 1 float4 groups padded with +inf (so at least one pad).  With
 * r = #{k : !(x <= t_k)} over the 4*n4 entries, r = #{t_k < x} <= m for every non-NaN x
 * (no pad counts) and r = 4*n4 for NaN (every compare counts).  The slot's votes are then
 * table[tab + r]: P[r] = the deltas of the r lowest stumps for r <= m, and entry 4*n4 the
 * deltas of the stumps that send NaN right.  Group 0 is inline, groups 1.. are at
 * extra thresholds[xthr..]. */
typedef struct ddm_cforest_slot {
    int32_t col;                 /* feature column                                       */
    int32_t n4;                  /* threshold groups (0: no stump reads this slot)       */
    int32_t tab;                 /* first table entry                                    */
    int32_t xthr;                /* first extra group                                    */
    float thr[4];                /* group 0                                              */
} ddm_cforest_slot;

typedef struct ddm_cforest_tree { int32_t node_begin, n_nodes, leaf_begin, n_leaves; } ddm_cforest_tree;
typedef struct ddm_cforest_node {
    float threshold; int32_t slot_nanleft;   /* slot | (NaN goes left) << 8 */
    uint32_t left_lo, left_hi;               /* leaves of the left subtree   */
} ddm_cforest_node;

/* Compile a packed host forest (nodes/roots as ddm_forest describes; classes host int32).
 * Returns 0 and *out_bytes = blob size when it fits `cap` (cap 0 / out NULL: size query),
 * DDM_E_FOREST when the forest is not compilable (impure, > 64 leaves in a tree, > 16
 * classes, > 32 feature columns): use the node walk. */
int ddm_forest_compile(const ddm_node* nodes, int32_t n_nodes, const int32_t* roots, int32_t n_trees,
                       const int32_t* classes, int32_t n_classes, int32_t pure, uint8_t* out,
                       int64_t cap, int64_t* out_bytes);

int ddm_abi_version(void);
const char* ddm_last_error(void);

/* predict_rf + error flag for DDM positions [pos_begin, pos_end) of one partition.
 * DDM position g lies in batch b = g / per_batch; its row is b*per_batch + perm[g]
 * (perm = the batch's shuffle, DDM_Process.py:190).  X is columnar float32
 * (X[f*ld + row], the float32 cast sklearn applies), y int32 labels.
 * err_out[g] = (classes[argmax] != y[row]); first_err (device uint64, may be NULL) is
 * set to the smallest g with an error, UINT64_MAX if none (written by this call);
 * pred_out (may be NULL) receives the predicted label per g.
 * ev_begin / ev_end (may be NULL) are recorded on `stream` immediately before and after
 * the kernel launch (launch-duration measurement without host gaps). */
int ddm_forest_predict(const float* X, int64_t ld, int32_t n_features, const int32_t* y,
                       const uint8_t* perm, int64_t pos_begin, int64_t pos_end,
                       int32_t per_batch, const ddm_forest* forest, uint8_t* err_out,
                       uint64_t* first_err, int32_t* pred_out, ddm_stream_t stream,
                       ddm_event_t ev_begin, ddm_event_t ev_end);

/* Batched predict: one segment per partition window (the same work as one
 * ddm_forest_predict call each), all in one launch per kernel variant.  segs_host must
 * stay valid (e.g. pinned) until the stream has consumed the table copy; block0/nblocks
 * are filled in by the call; segs_dev (device) receives the table (when every segment
 * has a compiled forest and n_segs <= 8 the table is passed in the kernel arguments
 * instead and segs_dev is not written).  first_err of every
 * segment (if non-NULL) is reset by the call. */
typedef struct ddm_predict_segment {
    const float* X; int64_t ld; const int32_t* y; const uint8_t* perm; uint8_t* err;
    int32_t* pred; uint64_t* first_err; int64_t pos_begin, pos_end;
    const ddm_node* nodes; const int32_t* roots; const double* leaf_value; const int32_t* classes;
    int32_t n_trees, n_classes, n_nodes, pure;
    int64_t row_base;       /* row = (g / per_batch) * per_batch + perm[g] - row_base (g: position) */
    int64_t block0, nblocks;
    const uint8_t* cforest; /* compiled forest (device) or NULL                              */
    int32_t cf_slots, cf_vote_regs;   /* its n_slots, vote_regs, n_leaves, rank-table words */
    int32_t cf_leaves, flags;         /* flags: DDM_SEG_FIRST_ERR_PRESET                     */
    int32_t cf_tab_words, pad;
} ddm_predict_segment;

/* ddm_predict_segment.flags: the caller already set *first_err to UINT64_MAX (e.g. in
 * the same host->device copy as its other inputs), so the call does not reset it. */
#define DDM_SEG_FIRST_ERR_PRESET 1

int ddm_forest_predict_batch(const ddm_predict_segment* segs_host, ddm_predict_segment* segs_dev,
                             int32_t n_segs, int32_t per_batch, ddm_stream_t stream,
                             ddm_event_t ev_begin, ddm_event_t ev_end);

/* run_DDM over every batch of every stream.  Stream s is err[stream_off[s] ..
 * stream_off[s+1]) (device int64 offsets; err readable up to the next multiple of 16
 * bytes past the last offset), cut into batches of per_batch rows (last one short).
 * state_io[s] (device) is the carried DDM, updated in place.
 * first_nz (device, may be NULL) is a hint: no nonzero byte of stream s lies in
 * [stream_off[s], first_nz[s]) (e.g. ddm_forest_predict's first_err).
 * ev_out (device int32 [n_batches_total][2]) receives per batch (first warning
 * position, change position) inside the batch, -1 = none; batch b of stream s is
 * row batch_base[s] + b (device int64).  This call fills ev_out with -1 first.
 * mode 0: stop a stream after its first batch with a change (controller mode);
 * mode 1: fresh DDM at the next batch after a change (DDM-only streams).
 * stop_out (device int32, may be NULL): batch of the first change or -1 (mode 0).
 * nev_out (device int64, may be NULL): number of batches with an event per stream.
 * ps_out (device double [rows][2], may be NULL): p and s after each processed row.
 * stream_end (device int64, may be NULL): when given, stream s is [stream_off[s],
 * stream_end[s]) (streams need not be adjacent), else [stream_off[s], stream_off[s+1]).
 * perm_map (device uint8, may be NULL): when given, events are reported as the ROW
 * offset inside the batch, perm_map[batch start + position] (the label the reference
 * records at DDM_Process.py:148,151), instead of the DDM position.
 * ev_begin / ev_end (may be NULL): as for ddm_forest_predict. */
int ddm_scan_streams(const uint8_t* err, const int64_t* stream_off, int64_t n_streams,
                     const ddm_params* prm, ddm_state* state_io, const uint64_t* first_nz,
                     const int64_t* batch_base, int64_t n_batches_total, int32_t* ev_out,
                     int32_t* stop_out, int64_t* nev_out, int32_t mode, double* ps_out,
                     const uint8_t* perm_map, const int64_t* stream_end, ddm_stream_t stream,
                     ddm_event_t ev_begin, ddm_event_t ev_end);

/* run_DDM in mode 1 (fresh DDM at the batch after a change) over n_streams independent
 * streams of stream_len rows each, back to back: stream s is err[s*stream_len ..
 * (s+1)*stream_len) (err readable up to the next multiple of 16 bytes past the end).
 * Replaces the per-row DDM loop of run_DDM (DDM_Process.py:135-159) for DDM-only
 * streams (SURVEY.md §8 a4/a5, configs[3]); results are those of ddm_scan_streams in
 * mode 1 with offsets s*stream_len and batch_base s*nb, nb = ceil(stream_len/per_batch).
 * Batch-parallel (csrc/scan_batches.hip): every batch is scanned speculatively with a
 * fresh detector, then each stream is walked over its batches' flags and the batches whose
 * carry-in was not fresh are rescanned with the carried detector.
 * per_batch must be 1..128, n_streams and stream_len < 2^31 (ABI 13).  ev_out: int32
 * [n_streams*nb][2] (every entry written); nev_out (may be NULL): batches with an event per
 * stream; scratch: device memory of ddm_scan_batches_scratch_bytes(...) bytes, 256-byte
 * aligned (about 140 bytes per batch: speculative records, queues, end states);
 * perm_map: as for ddm_scan_streams.  err must be 16-byte aligned. */
int64_t ddm_scan_batches_scratch_bytes(int64_t n_streams, int64_t stream_len, int32_t per_batch);
int ddm_scan_batches(const uint8_t* err, int64_t n_streams, int64_t stream_len, const ddm_params* prm,
                     ddm_state* state_io, int32_t* ev_out, int64_t* nev_out, void* scratch,
                     const uint8_t* perm_map, ddm_stream_t stream, ddm_event_t ev_begin,
                     ddm_event_t ev_end);

/* ddm_scan_streams (mode, state, stop, perm_map and first_nz as there) with the events
 * appended to per-stream logs instead of dense rows: for every batch b of stream s with an
 * event, logs[s][3 * k] = (log_b0[s] + b, first warning pos, change pos) at
 * k = log_n[s * log_n_stride]++ (the device-resident runner's event logs, csrc/ctl.hip). */
int ddm_scan_streams_log(const uint8_t* err, const int64_t* stream_off, int64_t n_streams, const ddm_params* prm,
                         ddm_state* state_io, const uint64_t* first_nz, int32_t* const* logs, int64_t* log_n,
                         int64_t log_n_stride, const int64_t* log_b0, int32_t* stop_out, int32_t mode,
                         const uint8_t* perm_map, const int64_t* stream_end, ddm_stream_t stream);

/* run_DDM over LONG carried segments (DDM_Process.py:135-159 with the DDM carried across
 * batches, :144-152, :202): the results of ddm_scan_streams (same stream_off / stream_end /
 * batch_base / ev_out / stop_out / nev_out / mode / perm_map meaning) for streams whose
 * detector runs exact rows for very long (no change for millions of rows while not in
 * its trivial state).  One wave per chunk of 64 * per_batch rows: the p recurrence is the
 * only sequential part, s, the running arg-min of p + s and the tests are lane-parallel
 * over 64-row tiles, and chunks are chained by a one-step look-back on the carried
 * detector (each chunk loads and masks its bytes before the carry reaches it).
 * Differences from ddm_scan_streams: streams with an empty range are left untouched
 * (state, stop, nev and events); ev_out is written for every batch of a non-empty stream
 * (-1 where none), never memset as a whole; max_rows bounds every stream's length (grid
 * size); per_batch must be 1..256; scratch is ddm_scan_long_scratch_bytes(...) bytes of
 * device memory, 256-byte aligned (its second uint32 is set to 1 if a chunk ever gave up
 * waiting for its predecessor).  A stream whose look-back gave up gets stop_out =
 * DDM_STOP_FAILED, nev_out = 0, events -1 and its state untouched: its results are void
 * and the caller must fail (or rescan it another way), never use them. */
#define DDM_STOP_FAILED (-2)
int64_t ddm_scan_long_scratch_bytes(int64_t n_streams, int64_t max_rows, int32_t per_batch);
int ddm_scan_long(const uint8_t* err, const int64_t* stream_off, const int64_t* stream_end, int64_t n_streams,
                  int64_t max_rows, const ddm_params* prm, ddm_state* state_io, const int64_t* batch_base,
                  int32_t* ev_out, int32_t* stop_out, int64_t* nev_out, int32_t mode, const uint8_t* perm_map,
                  void* scratch, ddm_stream_t stream, ddm_event_t ev_begin, ddm_event_t ev_end);
/* Test hook: look-back spins before a chunk gives up (default 2^24, about 1 s). */
int ddm_scan_long_set_spin_limit(uint32_t spins);

/* run_DDM over long carried segments, row-parallel with CERTIFIED decisions
 * (DDM_Process.py:135-159, the DDM carried across batches at :144-152, :202; the same
 * arguments and results as ddm_scan_long).  Every row is evaluated from the running mean
 * pa_i = (c0 p0 + K_i) / c_i (prefix error counts) instead of the reference's rounded
 * recurrence; every decision (the arg-min update, the change and warning tests) carries a
 * rigorous bound on the recurrence's rounding since the compared row (csrc/scan_cert.hip),
 * and a stream with any decision inside its bound is rescanned by ddm_scan_long.  Events,
 * stop, event counts, n and the flags are therefore the reference's exactly; p, s, p_min,
 * s_min and p_min+s_min are pa's, within bound_io's bound of the reference's.
 *   bound_io  NULL (the incoming states are the reference's) or double[2 * n_streams]:
 *             in: (bound of |p - p_ref|, bound of |p_min - p_min_ref|) of the incoming
 *             state; out: the same for the state handed back (0 for exact rescans).
 *   status_out NULL or int32[n_streams]: 0 certified, 1 rescanned exactly (a decision
 *             within its bound), 2 (mode 1) rescanned exactly after 4 certified rounds.
 * Mode 1 runs a certified round per change (the batch after a change starts fresh), up to
 * 4, then ddm_scan_long.  scratch: ddm_scan_certified_scratch_bytes(...) bytes, 256-byte
 * aligned; per_batch 1..256.  Streams with an empty range are left untouched. */
int64_t ddm_scan_certified_scratch_bytes(int64_t n_streams, int64_t max_rows, int32_t per_batch);
int ddm_scan_certified(const uint8_t* err, const int64_t* stream_off, const int64_t* stream_end, int64_t n_streams,
                       int64_t max_rows, const ddm_params* prm, ddm_state* state_io, double* bound_io,
                       const int64_t* batch_base, int32_t* ev_out, int32_t* stop_out, int64_t* nev_out, int32_t mode,
                       const uint8_t* perm_map, int32_t* status_out, void* scratch, ddm_stream_t stream,
                       ddm_event_t ev_begin, ddm_event_t ev_end);
/* Test hook: multiply every decision bound by scale (>= 1; huge forces the exact rescans). */
int ddm_scan_certified_set_tol_scale(double scale);

/* Timing events for the ev_begin / ev_end arguments (hipEventCreate / Destroy /
 * ElapsedTime; elapsed needs both events completed, e.g. after a stream sync). */
int ddm_event_create(ddm_event_t* ev);
/* ABI 19: an event for stream ordering only (hipEventDisableTiming): fork / join events. */
int ddm_event_create_sync(ddm_event_t* ev);
int ddm_event_destroy(ddm_event_t ev);
int ddm_event_record(ddm_event_t ev, ddm_stream_t stream);
int ddm_event_synchronize(ddm_event_t ev);
int ddm_event_elapsed_ms(ddm_event_t begin, ddm_event_t end, float* ms);

/* ABI 22: a stream on a subset of the current device's CUs (hipExtStreamCreateWithCUMask):
 * CU i belongs to it when i % stride == offset % stride; *n_cus (nullable) = their count.
 * The device epochs can put the next windows' shuffles on such a stream so that they leave
 * the other CUs to the predict (DDM_Process.py:110-128 beside :187/:190's shuffles; off by
 * default).  Measured in round 6 (tools/cu_probe.hip, profiles/r06/cu_probe.txt): on the
 * MI355X pool the runtime accepts the mask but does not apply it -- the workgroups of a
 * stride-2 / 4 / 8 stream still ran on all 256 CUs -- so *n_cus is the requested count. */
int ddm_stream_create_cu_stride(int32_t stride, int32_t offset, ddm_stream_t* out, int32_t* n_cus);
/* ABI 22: the number of CUs a stream may run on (hipExtStreamGetCUMask). */
int ddm_stream_cu_count(ddm_stream_t stream, int32_t* n_cus);
int ddm_stream_destroy(ddm_stream_t stream);
/* ABI 22: the decoupled epochs' predict launch (row order into err + delta; clk, join_flag and
 * timeouts nullable), exported for the bench's back-to-back replays of an epoch's tables. */
int ddm_forest_predict_dev_orig(const ddm_predict_segment* segs_dev, const int64_t* const* res_dev, int32_t n_segs,
                                int32_t per_batch, int64_t grid, int32_t* stall, int64_t delta, uint64_t* clk,
                                const uint32_t* join_flag, uint32_t join_v, uint32_t* timeouts, ddm_stream_t stream);

/* ---- host-side MT19937 (numpy legacy RandomState layout: key[624], pos) ---------- */

/* Legacy `permutation(len)` for consecutive batches (Fisher-Yates, mask rejection).
 * batch_len[i] <= 256; perms are written back to back into perm_out (uint8);
 * draws_out[i] (may be NULL) = 32-bit words consumed by batch i. */
int ddm_mt_perms(uint32_t* key, int32_t* pos, const int32_t* batch_len, int64_t n_batches,
                 uint8_t* perm_out, int64_t* draws_out);

/* `randint(2**31 - 1)` x count (the per-tree seeds of RandomForestClassifier.fit). */
int ddm_mt_randint31(uint32_t* key, int32_t* pos, int64_t count, int64_t* out);

/* Advance the generator by n_draws 32-bit words. */
int ddm_mt_skip(uint32_t* key, int32_t* pos, int64_t n_draws);

/* ABI 24: numpy's legacy RandomState(seed) state for a seed < 2^32 (init_genrand, pos 624):
 * the per-partition np.random.seed of the reference's UDF, without constructing a Python
 * RandomState (~0.1 ms each) at every run's start. */
int ddm_mt_seed(uint32_t seed, uint32_t* key, int32_t* pos);

/* One batch's permutation(L) then T randint(2**31-1) seeds from already tempered words
 * of the stream (e.g. read back from the device copy); used[0], used[1] = words each
 * consumed.  DDM_E_ARG when the words run out. */
int ddm_words_perm_seeds(const uint32_t* words, int64_t n_words, int32_t L, int32_t T,
                         uint8_t* perm_out, int64_t* seeds_out, int64_t* used);

/* ---- batch shuffles on the GPU (csrc/shuffle.hip) -------------------------------- */
/* The partition's MT19937 stream as raw tempered words R[0..), generated on the device,
 * plus interval-FSM tables that make the Fisher-Yates draws of many batches parallel.
 * Batches handled here all have batch_len rows (2..256); draws are indexed from the
 * stream start (the state uploaded into mt_state). */
#define DDM_SHUFFLE_SUB   128    /* draws per sub-chunk table   */
#define DDM_SHUFFLE_CHUNK 8192   /* draws per chunk table       */

/* Append n tempered words to R (device).  mt_state (device uint32[625]) = numpy key[624]
 * followed by pos; it is advanced in place (one workgroup, 624-word blocks in LDS). */
int ddm_shuffle_generate(uint32_t* mt_state, uint32_t* R, int64_t n, ddm_stream_t stream);

/* FSM tables for chunks [chunk0, chunk0+nchunk) of R, for a chunk entered in interval
 * state s (1..batch_len-1): Tpre uint32 [chunk][64][batch_len-1] = interval state after
 * sub-chunks 0..k | batches completed since the chunk start << 8, and Tchunk uint32
 * [chunk][batch_len-1] = Tpre[chunk][63]. */
int ddm_shuffle_tables(const uint32_t* R, int64_t chunk0, int64_t nchunk, int32_t batch_len,
                       uint32_t* Tpre, uint32_t* Tchunk, ddm_stream_t stream);
/* The same for many streams in one launch (jobs_dev: device array; max_chunks >= every
 * job's nchunk). */
typedef struct ddm_table_job {
    const uint32_t* R; int64_t chunk0, nchunk; uint32_t* Tpre; uint32_t* Tchunk;
} ddm_table_job;
int ddm_shuffle_tables_batch(const ddm_table_job* jobs_dev, int32_t n_jobs, int64_t max_chunks,
                             int32_t batch_len, ddm_stream_t stream);

/* Shuffles of W consecutive batches whose first draw is R[P] (a batch boundary):
 * perm_out[b*batch_len + k] (uint8) and E[b] = index of the draw completing batch b.
 * avail = draws covered by tables (multiple of DDM_SHUFFLE_CHUNK); pieces (device,
 * >= max_pieces * 16 bytes, max_pieces >= 66 + W*batch_len*3/DDM_SHUFFLE_CHUNK), J
 * (device, W*batch_len bytes) and first (device, 64*(batch_len-1) uint16: tables of the
 * chunk holding P) are scratch; info (device int64[3]) = {pieces, end draw, batches
 * reached} (batches reached < W means avail was too small). */
int ddm_shuffle_window(const uint32_t* R, const uint32_t* Tpre, const uint32_t* Tchunk, int64_t avail,
                       int64_t P, int64_t W, int32_t batch_len, void* pieces, int64_t max_pieces,
                       int64_t* info, uint8_t* J, int64_t* E, uint8_t* perm_out, uint16_t* first,
                       ddm_stream_t stream, ddm_event_t ev_begin, ddm_event_t ev_end);

/* Batched forms (one job per partition, device array of jobs; W = 0 skips a job). */
typedef struct ddm_gen_job { uint32_t* mt_state; uint32_t* R; int64_t n; } ddm_gen_job;
typedef struct ddm_shuffle_job {
    const uint32_t* R; const uint32_t* Tpre; const uint32_t* Tchunk;
    int64_t avail, P, W;
    void* pieces; int64_t* info; uint8_t* J; int64_t* E; uint8_t* perm_out;
    const int32_t* stop;            /* ddm_shuffle_pick_batch: scan stop flag (may be NULL) */
    int64_t pick_offset, pick_last; /* pick E[(stop >= 0 ? stop : pick_last) - pick_offset] */
    int64_t* pick_out;              /* may be NULL: no pick for this job                   */
    uint16_t* first;                /* scratch, 64*(batch_len-1) uint16 (see ddm_shuffle_window) */
} ddm_shuffle_job;

int ddm_shuffle_generate_batch(const ddm_gen_job* jobs_dev, int32_t n_jobs, ddm_stream_t stream);

/* MT19937 jump-ahead, so one partition's stream is generated in parallel segments.
 * A reduced GF(2) polynomial is DDM_MT_POLY_WORDS uint64 words, bit i = coefficient of x^i.
 * ddm_mt_charpoly (host): the characteristic polynomial phi of MT19937's transition
 *   (degree 19937, DDM_MT_POLY_WORDS + 1 words; Berlekamp-Massey, computed once).
 * ddm_mt_jump_polys (host): out[k] = x^((k+1)*jump) mod phi for k < n (cached per jump).
 * ddm_mt_jump (device): per job, out[0..623] = the MT19937 state (numpy key layout,
 *   pos 624) T^e(key) for the polynomial x^e mod phi in poly, and out[624] = 624.  The
 *   lower 31 bits of out[0] are not part of the state (never read by the generator).
 *   scratch: unused, may be NULL (the word sequence x_0 .. x_{623 + deg} is generated in
 *   the workgroup's LDS, three 624-word blocks at a time since round 6; the sequence's
 *   whole length, DDM_MT_JUMP_SCRATCH_WORDS, is kept for callers sizing scratch).
 *   Replaces nothing in the reference: the streams are those of DDM_Process.py:187,190,102. */
#define DDM_MT_POLY_WORDS 312
#define DDM_MT_JUMP_SCRATCH_WORDS 21216
typedef struct ddm_jump_job {
    const uint32_t* key; const uint64_t* poly; uint32_t* out; uint32_t* scratch;
} ddm_jump_job;
int ddm_mt_charpoly(uint64_t* out);
int ddm_mt_jump_polys(int64_t jump, int32_t n, uint64_t* out);
int ddm_mt_jump(const ddm_jump_job* jobs_dev, int32_t n_jobs, ddm_stream_t stream);
int ddm_shuffle_window_batch(const ddm_shuffle_job* jobs_dev, int32_t n_jobs, int64_t max_W,
                             int64_t max_pieces, int32_t batch_len, ddm_stream_t stream,
                             ddm_event_t ev_begin, ddm_event_t ev_end);
int ddm_shuffle_pick_batch(const ddm_shuffle_job* jobs_dev, int32_t n_jobs, ddm_stream_t stream);

/* out[0] = E[k] with k = (stop[0] >= 0 ? stop[0] : last) - offset if 0 <= k < W, else -1
 * (device scalars; lets the controller read the RNG position with the control block). */
int ddm_shuffle_pick(const int32_t* stop, const int64_t* E, int64_t W, int64_t offset, int64_t last,
                     int64_t* out, ddm_stream_t stream);

/* ---- epoch read-back staging (csrc/stage.hip) ------------------------------------ */
/* After an epoch's kernels, per partition: the event rows of the scanned batches
 * compacted into ev_out[max_events][3] = (window batch, warning pos, change pos) and,
 * when the scan stopped at a change in batch d = j + *stop, batch d's rows in shuffled
 * order (x_out [L][n_features] float32, y_out [L]) and n_words stream words from the draw
 * P after batch d's shuffle (P = p_after_first if d < g0, p_tail_after for the host-
 * shuffled short last batch when tail, else *pick + 1).  Then, if batch d+1 exists, its
 * shuffle is drawn from P into perm_w (at base + (d+1)*pb) and the n_trees refit seeds
 * after it into seeds_out.  info_out = {P or -1, event count, overflow (count >
 * max_events), d or -1, draw after batch d+1's shuffle, draw after the seeds, 1 if those
 * two were drawn}.  ev holds the partition's window rows [(b - j)][2] as
 * ddm_scan_streams wrote them. */
typedef struct ddm_stage_job {
    const float* X; int64_t ld; const int32_t* y; const uint8_t* perm; int64_t base;
    const int32_t* ev; const int32_t* stop; const int64_t* pick; const uint32_t* R;
    int64_t j, g0, nb, b_end, p_after_first, p_tail_after;
    int32_t pb, last_len, n_features, n_words, tail, max_events;
    float* x_out; int32_t* y_out; uint32_t* w_out; int64_t* info_out; int32_t* ev_out;
    uint8_t* perm_w;        /* perm array to receive batch d+1's shuffle (may be NULL)   */
    int64_t* seeds_out;     /* [n_trees] refit seeds drawn after it (may be NULL)        */
    int32_t n_trees;
    int32_t win_rule;       /* ABI 20: window after a change (ddm_ctl_part.win_rule)      */
    /* next-window plan (plan_out may be NULL): the controller's window policy applied on
     * the device, so the next window's shuffles can run before the host has seen this
     * epoch.  plan_out = {P, W (0: not planned), g0, b_end, j, planned}; next_job (may be
     * NULL) = this partition's ddm_shuffle_job whose P, W, perm_out and avail are set. */
    int64_t p_now, win, max_win, seg_start, n_full, min_win, next_avail, dpb_x1024;
    int64_t* plan_out;
    ddm_shuffle_job* next_job;
    /* device-resident runner (ddm_ctl, log != NULL): the event rows go to log[3 * (*log_n + k)]
     * = (batch, first warning pos, change pos) (absolute batch of the partition, at most
     * log_cap records) instead of ev_out, and *log_n advances; stall (may be NULL): when
     * *stall != 0 the partition is skipped (info = no change, nothing gathered or drawn). */
    int32_t* log; int64_t* log_n; int64_t log_cap; const int32_t* stall;
} ddm_stage_job;

int ddm_epoch_stage(const ddm_stage_job* jobs_dev, int32_t n_jobs, ddm_stream_t stream);

/* ---- host forest refit ------------------------------------------------------------ */

/* RandomForestClassifier(n_estimators=n_trees).fit(X, y) exactly as scikit-learn 1.7.2
 * builds it (bootstrap, max_features=sqrt, Gini, fully grown), given the per-tree seeds
 * the forest draws from the global RNG (ddm_mt_randint31 x n_trees).  X: host float32
 * [n][n_features] row-major (no NaN), y_idx: class index per row (np.unique inverse).
 * Writes the packed forest: nodes (capacity >= n_trees*(2n-1)), roots[n_trees];
 * leaf_value [leaf_rows_cap][n_classes] is only used when some leaf is not one-hot
 * (DDM_E_IMPURE if it is NULL or too small).  out_info = {n_nodes, pure, n_leaf_rows}. */
int ddm_rf_fit(const float* X, int32_t n, int32_t n_features, const int32_t* y_idx, int32_t n_classes,
               const int64_t* seeds, int32_t n_trees, int32_t max_features, ddm_node* nodes,
               int64_t nodes_cap, int32_t* roots, double* leaf_value, int64_t leaf_rows_cap,
               int64_t* out_info);

/* Many refits at once (one per partition that drifted): every (job, tree) pair is fitted
 * on a persistent pool of n_threads host threads (the calling thread included), then each
 * job is packed like ddm_rf_fit and, when `blob` is given and the forest compiles,
 * compiled with ddm_forest_compile (blob_bytes > 0, cf_* filled).  status per job: 0,
 * DDM_E_NAN (use sklearn), DDM_E_IMPURE or DDM_E_ARG; the call returns the first
 * non-zero status (the other jobs are still done). */
typedef struct ddm_fit_job {
    const float* X; const int32_t* y_idx; const int64_t* seeds; const int32_t* classes;
    int32_t n, n_features, n_classes, n_trees, max_features, status;
    ddm_node* nodes; int64_t nodes_cap; int32_t* roots; double* leaf_value; int64_t leaf_rows_cap;
    int64_t info[3];                   /* out: n_nodes, pure, n_leaf_rows */
    uint8_t* blob; int64_t blob_cap; int64_t blob_bytes;
    int32_t cf_slots, cf_vote_regs, cf_leaves, cf_tab_words;
} ddm_fit_job;

int ddm_rf_fit_many(ddm_fit_job* jobs, int32_t n_jobs, int32_t n_threads);

/* ---- device forest refit ---------------------------------------
 * train_rf (DDM_Process.py:98-105) on the GPU, tree for tree what ddm_rf_fit builds
 * (scikit-learn 1.7.2: bootstrap from RandomState(seed), BestSplitter with our_rand_r
 * feature draws, Gini, fully grown), then packed and compiled as ddm_rf_fit_many does,
 * so that the refit after a change never leaves the device: the training batch, its
 * labels and the tree seeds are the ones ddm_epoch_stage gathered and drew.  One wave
 * builds one tree.  Limits: L <= 256 rows, F <= 256 features, k_cap <= 64 classes;
 * a job outside them, or with NaN in X, reports a status and is refit on the host. */
typedef struct ddm_dfit_job {
    const float* X;          /* device [L][F] float32 row-major (ddm_stage_job.x_out)      */
    const int32_t* y;        /* device [L] labels (ddm_stage_job.y_out)                      */
    const int64_t* seeds;    /* device [n_trees] tree seeds (ddm_stage_job.seeds_out)        */
    const int64_t* gate;     /* device: the job runs only when *gate >= 0 (NULL: always),
                                e.g. ddm_stage_job.info_out (the change's stream position) */
    const int64_t* gate2;    /* device: and only when *gate2 == 1 (NULL: no condition),
                                e.g. info_out + 6 (the seeds were drawn on the device)      */
    int32_t L, F, n_trees, max_features;
    int32_t k_cap, pad;      /* classes the job's buffers hold (<= 64)                       */
    uint8_t* scratch;        /* device, ddm_rf_device_scratch_bytes(L, F, n_trees, k_cap)   */
    ddm_node* nodes;         /* device outputs, as ddm_rf_fit writes them: [n_trees*(2L-1)] */
    int32_t* roots;          /* [n_trees]                                                    */
    double* leaf_value;      /* [n_trees*L][k_cap] (impure forests)                          */
    int32_t* classes;        /* [k_cap] sorted labels (classes_)                             */
    uint8_t* blob;           /* the ddm_forest_compile blob, when the forest compiles        */
    int64_t blob_cap;
    int64_t* result;         /* device int64[12]: DDM_DFIT_* indices                        */
} ddm_dfit_job;

#define DDM_DFIT_STATUS    0   /* 0 ok, DDM_E_NAN / DDM_E_FOREST / DDM_E_ARG; a gated-off job writes nothing */
#define DDM_DFIT_CLASSES   1
#define DDM_DFIT_NODES     2
#define DDM_DFIT_PURE      3
#define DDM_DFIT_LEAF_ROWS 4
#define DDM_DFIT_BLOB      5   /* blob bytes; 0: not compilable (node walk)                  */
#define DDM_DFIT_CF_SLOTS  6
#define DDM_DFIT_CF_VR     7
#define DDM_DFIT_CF_LEAVES 8
#define DDM_DFIT_CF_TAB    9

int64_t ddm_rf_device_scratch_bytes(int32_t L, int32_t F, int32_t n_trees, int32_t k_cap);

/* Fits every job (device table of n_jobs records) on `stream`; max_trees bounds the
 * jobs' n_trees (grid size).  Asynchronous: results land in each job's result[]. */
int ddm_rf_fit_device(const ddm_dfit_job* jobs_dev, int32_t n_jobs, int32_t max_trees, ddm_stream_t stream);
/* The same with max_lf >= every job's L*F: batches of at most 4096 values are gated, checked
 * and presorted inside the tree kernel (one launch fewer); max_lf <= 0: unknown. */
int ddm_rf_fit_device_lf(const ddm_dfit_job* jobs_dev, int32_t n_jobs, int32_t max_trees, int64_t max_lf,
                         ddm_stream_t stream);

/* ---- epoch executor (csrc/epoch.hip) -------------------------------------------- */
/* One call enqueues a BatchRunner epoch on `stream`: ctrl_d[0, upload_bytes) <- ctrl_h
 * (pinned), ddm_shuffle_window_batch (n_shuffle > 0), ddm_forest_predict_batch (n_segs >
 * 0), ddm_scan_streams (mode 0), ddm_scan_long (long_max_rows > 0), ddm_shuffle_pick_batch,
 * ddm_epoch_stage (n_stage > 0), ddm_rf_fit_device (n_dfit > 0), then ctrl_h[0,
 * download_bytes) <- ctrl_d.  ev (may hold NULLs): begin/end pairs around the shuffles,
 * predict, scan, long scan and refits.  Replaces the per-launch calls the controller
 * makes for DDM_Process.py:187-210 (one batch loop iteration per partition and batch). */
typedef struct ddm_epoch {
    ddm_stream_t stream;
    void* ctrl_d; void* ctrl_h; int64_t upload_bytes, download_bytes;
    const ddm_shuffle_job* shuffle_jobs; int32_t n_shuffle, per_batch; int64_t max_W, max_pieces;
    const ddm_predict_segment* segs_h; ddm_predict_segment* segs_d; int32_t n_segs, n_stage;
    const uint8_t* err; const int64_t* offsets; const int64_t* ends; int64_t n_streams;
    const ddm_params* params; ddm_state* state; const uint64_t* first_nz; const int64_t* batch_base;
    int64_t n_batches_total; int32_t* ev_out; int32_t* stop; int64_t* nev; const uint8_t* perm_map;
    const int64_t* long_off; const int64_t* long_end; int64_t long_max_rows; void* long_scratch;
    const ddm_stage_job* stage_jobs; const ddm_dfit_job* dfit_jobs; int32_t n_dfit, max_trees;
    ddm_event_t ev[10];
    /* shuffle_jobs drive the shuffles, pick_jobs (all partitions with a window) the pick */
    const ddm_shuffle_job* pick_jobs; int32_t n_pick, n_next;
    /* the next windows' shuffles (n_next > 0): next_jobs planned by the staging, run on
     * side_stream between fork_ev (after the staging) and join_ev (before the read-back),
     * beside the device refits */
    const ddm_shuffle_job* next_jobs; int64_t next_max_W, next_max_pieces;
    ddm_stream_t side_stream; ddm_event_t fork_ev, join_ev;
    /* split read-back (mid_ev != NULL): the slab right after the staging, then mid_ev,
     * and after the refits only ctrl[tail_off, tail_off + tail_bytes) (their results) */
    ddm_event_t mid_ev; int64_t tail_off, tail_bytes;
    int64_t dfit_max_lf;     /* ddm_rf_fit_device_lf's max_lf (<= 0: unknown)              */
} ddm_epoch;
int ddm_epoch_launch(const ddm_epoch* e);
int64_t ddm_epoch_struct_bytes(void);   /* sizeof(ddm_epoch), for binding checks */

/* ---- device-resident epoch controller (csrc/ctl.hip) ------------------------------
 * The per-epoch decisions of the BatchRunner (ddm_amd/controller.py: the window after a
 * change or after a clean window, the RNG position, the DDM state carried or dropped, the
 * forest a refit produced, DDM_Process.py:189-210) taken on the device, so epochs are
 * enqueued ahead and the host only collects events.  One record per partition: the static
 * part (its buffers and the job / segment / staging templates) is written by the host when
 * the runner enters device mode, the dynamic part mirrors the host controller's state at
 * the start of an epoch.  Partitions that need the host (a refit that reported a status or
 * did not compile, stream words that ran out, a look-back that gave up) get `stall`;
 * partitions whose short last batch still needs its shuffle get `park`. */
typedef struct ddm_ctl_part {
    ddm_shuffle_job job;         /* window job template: R, Tpre, Tchunk, pieces, info, J, E, first, stop, pick_out */
    ddm_predict_segment seg;     /* segment template: X, ld, y, perm, err, first_err, row_base, flags + host forest */
    ddm_stage_job stage;         /* staging template (plan_out / next_job NULL, log / log_n / stall set) */
    const int64_t* res;          /* the partition's device refit result words (ddm_dfit_job.result) */
    const ddm_node* dnodes; const int32_t* droots; const double* dleaf; const int32_t* dclasses;
    const uint8_t* dblob;        /* the device refit's forest buffers */
    int64_t nb, n_full, base, max_win, min_win, long_min_rows, long_cap_rows, dpb_x1024;
    int32_t pb, last_len, n_words, dtrees;
    int32_t host_slots;          /* feature slots the host forest reads (statistics) */
    int32_t win_rule;            /* ABI 20: the window after a change covers the concept just
                                    closed plus max(concept >> (win_rule & 255),
                                    (win_rule >> 8) & 255) batches, and at least min_win unless
                                    the concept was at most win_rule >> 16 batches
                                    (DDMSettings drift_window_shift / _pad / _short) */
    /* dynamic: the host controller's state at the start of an epoch */
    int64_t j, P, win, seg_start, P1, P2, avail;
    int32_t retrain, done, stall, park, forest_dev, applied, idle, pad1;
    int64_t g0, b_end, Wg, P_after_first, p0, p1;
    ddm_state state;
    int64_t n_log, predicted_rows, predict_bytes, epochs, refits;
    int64_t log_mark;            /* n_log before this epoch's scans: restored when the epoch stalls */
    int64_t long_scans;          /* windows that ran on ddm_scan_long (statistics) */
    int64_t permute_rows;        /* ABI 20: rows of decoupled epochs (row-order predict +
                                    k_err_permute into DDM order; statistics) */
    int64_t pad2;
} ddm_ctl_part;

/* Stall reasons (ddm_ctl_part.stall) */
#define DDM_CTL_STALL_REFIT 1    /* the device refit reported a status / did not compile     */
#define DDM_CTL_STALL_WORDS 2    /* batch d+1's shuffle or the seeds ran past the staged words */
#define DDM_CTL_STALL_SCAN  3    /* ddm_scan_long gave up (DDM_STOP_FAILED)                   */
#define DDM_CTL_STALL_LONG  4    /* a carried window needs ddm_scan_long, not enqueued          */

typedef struct ddm_ctl {
    ddm_ctl_part* parts; int32_t n, entry;       /* entry: plan the first window only     */
    ddm_shuffle_job* jobs; ddm_predict_segment* segs; const int64_t** seg_res; ddm_stage_job* stage;
    int64_t* off; int64_t* end; ddm_state* state; uint64_t* first; const int32_t* stop; const int64_t* pick;
    int64_t* loff; int64_t* lend; int32_t* pstall;   /* per partition: set by the predict    */
    int64_t predict_blocks;                        /* grid of ddm_forest_predict_dev          */
    int64_t* status;                               /* [4]: active, stalled, parked, done       */
    int32_t* const* logs;                          /* per partition: its event log             */
    int64_t* log_b0;                               /* per partition: the window's first batch  */
    uint32_t* sync;                                /* NULL or uint32[2], zeroed: [0] the fused
                                                      staging's block ticket (left 0), [1] set
                                                      when the next epoch has a long window    */
    int32_t decoupled;                             /* ABI 20: set by ddm_ctl_epochs for the
                                                      decisions kernel: this epoch's predict
                                                      wrote row-order errors (statistics)      */
    int32_t long_ok;                               /* ABI 20: ddm_scan_long runs in the epochs
                                                      (long_max_rows > 0); 0: a window that
                                                      needs it stalls (DDM_CTL_STALL_LONG)
                                                      instead, and no long-scan launch is
                                                      enqueued                                 */
    uint64_t* predict_clock;                       /* ABI 21: NULL or device words [18], set
                                                      once to 8 x ~0, 8 x 0, 0, 0: every
                                                      epoch's predict stamps its first
                                                      workgroups' starts and every workgroup's
                                                      end on the 100 MHz device clock (8
                                                      shards), the staging kernel after it adds
                                                      max(end) - min(start) to [16] and 1 to
                                                      [17] and resets the shards              */
} ddm_ctl;

typedef struct ddm_ctl_epoch {
    ddm_stream_t stream, side_stream; ddm_event_t fork_ev, join_ev;
    ddm_ctl ctl;                                   /* device pointers, by value                */
    const ddm_ctl* ctl_d;                          /* unused (reserved)                        */
    int32_t n, per_batch;
    const uint8_t* err; const ddm_params* params; const int64_t* batch_base; int64_t n_batches_total;
    int32_t* ev_out; int64_t* nev; const uint8_t* perm_map;
    int64_t long_max_rows; void* long_scratch;
    const ddm_dfit_job* dfit_jobs; int32_t n_dfit, max_trees;
    int64_t max_W, max_pieces;                     /* shuffle grid bounds (windows never exceed) */
    int64_t dfit_max_lf;                           /* ddm_rf_fit_device_lf's max_lf             */
    ddm_event_t ev[12];                            /* optional begin/end pairs: predict, scan, long,
                                                      stage + ctl, refit, next shuffles        */
    int64_t row_order_delta;                       /* ABI 19: a buffer shaped like err at err +
                                                      delta (0: none) for decoupled epochs     */
    int32_t decouple, pad_dc;                      /* 1: the predict writes row-order errors
                                                      there without waiting for the window's
                                                      shuffles, which are waited for only by
                                                      the permutation into err (DDM order)     */
    const ddm_event_t* predict_evs;                /* ABI 20: NULL or [2 * n_epochs] timing
                                                      events recorded right before / after each
                                                      epoch's predict launch (ev[0] / ev[1] are
                                                      used when NULL)                          */
    uint32_t* sync_flags;                          /* ABI 21: NULL (fork / join by fork_ev /
                                                      join_ev) or device words [4], zeroed once
                                                      for the streams' life: [0] / [1] the last
                                                      fork / join number published, [2] waits
                                                      that gave up (nonzero voids the results),
                                                      [3] the join polls' give-up limit in
                                                      10-ns ticks (0: 2 s, as the fork wait's
                                                      always; a hang guard)                    */
    uint32_t* sync_seq;                            /* ABI 21: host words [3], the fork / join
                                                      numbers enqueued so far and the last
                                                      join the epoch stream polled (advanced
                                                      by ddm_ctl_epochs; zero with the flags)  */
} ddm_ctl_epoch;
int64_t ddm_ctl_part_bytes(void);
int64_t ddm_ctl_epoch_bytes(void);
/* entry: plan every partition's first window and shuffle it (on e->stream). */
int ddm_ctl_enter(const ddm_ctl_epoch* e);
/* n_epochs device epochs on e->stream: predict, scan (+ long), pick, staging, decisions and
 * the next windows' plan, then the next windows' shuffles on side_stream beside the device
 * refits.  Epochs after every partition is done, parked or stalled do no work.  With
 * ctl.sync, pick + staging + decisions are one kernel (the last workgroup splits the predict
 * grid) and the long scan's blocks return at once in epochs without a long window. */
int ddm_ctl_epochs(const ddm_ctl_epoch* e, int32_t n_epochs);
/* ABI 20: n_epochs of ddm_ctl_epochs captured once into an executable hipGraph (both streams
 * and their fork / join edges; no timing events: e->ev and e->predict_evs must be empty, HIP
 * does not time events a graph records), replayed by ddm_ctl_graph_launch on
 * e->stream.  Every decision is in device memory, so one graph serves every group of the
 * same runner (the tables never move).  A replayed group starts without the join of the
 * group before it and ends with its own. */
int ddm_ctl_graph_create(const ddm_ctl_epoch* e, int32_t n_epochs, void** exec_out);
int ddm_ctl_graph_launch(void* exec, ddm_stream_t stream);
int ddm_ctl_graph_destroy(void* exec);

/* Forest predict for the device-resident runner: one launch, fixed grid, segments and block
 * split from the device table; a segment with res[s] != NULL takes its compiled forest's shape
 * from those refit result words (and sets stall[s] instead when the refit is unusable). */
int ddm_forest_predict_dev(const ddm_predict_segment* segs_dev, const int64_t* const* res_dev, int32_t n_segs,
                           int32_t per_batch, int64_t grid, int32_t* stall, ddm_stream_t stream,
                           ddm_event_t ev_begin, ddm_event_t ev_end);

/* ---- synthetic inputs (benchmark configs) ------------------------- */

/* Labels of a class-block stream partitioned as DDM_Process.py:225 (row % n_parts):
 * partition row r is global row g = r*n_parts + part, class (g / block_rows) % n_classes. */
int ddm_synth_block_labels(int32_t* y, int64_t n_rows, int64_t part, int64_t n_parts,
                           int64_t block_rows, int32_t n_classes, ddm_stream_t stream);

/* configs[4] (C5) labels: global row g = r*n_parts + part lies in block k, whose global
 * boundaries are k*period + jitter_k (jitter_k ~ U[-jitter, jitter] from a counter hash of
 * (seed, k), jitter_0 = 0, 2*jitter < period); class k % n_classes, flipped to another
 * class with probability flip (label noise).  Blocks of 150-300 partition rows over 8
 * partitions: period 1800, jitter 300 (block lengths 1800 +- 600). */
int ddm_synth_jitter_labels(int32_t* y, int64_t n_rows, int64_t part, int64_t n_parts, int64_t period,
                            int64_t jitter, int32_t n_classes, double flip, uint64_t seed,
                            ddm_stream_t stream);

/* Noise-free separable features for labels y: X[f*ld + r] = base(y[r], f) + noise*u,
 * u ~ U[0,1) from a counter hash of (seed, row0 + r*row_stride, f). */
int ddm_synth_features(float* X, int64_t ld, int32_t n_features, const int32_t* y, int64_t n_rows,
                       int64_t row0, int64_t row_stride, uint64_t seed, float noise,
                       ddm_stream_t stream);

/* C4 streams: stream s has Bernoulli(r0) errors, r0 ~ U(0.01, 0.2), switching at a random
 * row to r0 + U(0.05, 0.3).  err is [n_streams][len] bytes. */
int ddm_synth_bernoulli_streams(uint8_t* err, int64_t n_streams, int64_t len, uint64_t seed,
                                ddm_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* DDM_AMD_H */
