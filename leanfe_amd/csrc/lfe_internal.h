// Internal declarations shared by the leanfe HIP engine translation units.
// Target: gfx950 (MI355X, CDNA4) only.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "../../include/leanfe_hip.h"

namespace lfe {

constexpr int kMaxFE = 8;        // FE dimensions supported per regression
constexpr int kMaxCl = 16;       // cluster columns per CGM subset
constexpr int kMaxCols = 63;     // p = 1 + k (+ instruments) <= 63 -> Gram width <= 64
constexpr int kColStatHead = 64; // colstat: max |x_c| bits of every column before the per-chunk sums
// iscratch (prepare_layout): [2 F] level counts, [2 kMaxFE] dropped rows, [+1] any-singleton flag,
// [kIscratchCmax, + F) largest kept count per FE
constexpr int kIscratchCmax = 2 * kMaxFE + 8;
constexpr int kIsDnPre = 2 * kMaxFE + 6;  // iscratch: a primary level of > 65535 rows in the pre-filter table build
constexpr int kIsCmaxOver = 2 * kMaxFE + 7;  // iscratch: ranks whose primary FE keeps a level of > 65535 rows (owner)
constexpr int kIsAny = 2 * kMaxFE + 1;   // iscratch: groups with a pre-filter count of 1 (0: nothing to mark)
constexpr int kIscratchInts = kIscratchCmax + kMaxFE;
// iscratch's allocation: the counts above, then lfe_load_clusters' per (cluster column, FE) flags
// (allocated whole at the first use, so that loading clusters after the drop keeps the counts)
constexpr int kIsClFlags = kIscratchInts;
constexpr int kIscratchAll = kIsClFlags + 30 * kMaxFE;
constexpr int kBlock = 256;      // threads per workgroup for simple streaming kernels
constexpr int kSweepThreads = 512;   // sweep kernels (8 waves)
constexpr int kLdsBudget = 64 * 1024;  // bytes of LDS tables per sweep workgroup (2 WG per CU)
constexpr int kItemRows = 8192;      // rows per work item (a bucket is split into items)
constexpr int kLdsHistMax = 16384;   // int32 counters in an LDS histogram
constexpr size_t kPinD2H = 128 * 1024;   // pinned staging: device -> host results
constexpr size_t kPinSmall = 192 * 1024; // pinned staging total (D2H + small H2D)

void set_error(const std::string& msg);

// Test / A-B knobs: a process-wide name -> value table that only lfe_test_set_knob writes (tests,
// bench --knob).  The engine never reads the environment, so a stray variable cannot change which
// kernels run; with no knob set every path is the production one.  nullptr = not set.  The value
// is a copy in a small per-thread ring: read it at once (e[0], atoi), do not keep the pointer.
const char* knob(const char* name);

// hipFuncSetAttribute(fn, MaxDynamicSharedMemorySize, bytes) once per (device, kernel) and size: the
// limit only grows, and the call (~µs of host time on the launch path) is skipped when it is already
// high enough
hipError_t set_max_lds(const void* fn, int bytes);

#define LFE_HIP(expr)                                                                    \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess) {                                                              \
      ::lfe::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));             \
      return (_e == hipErrorOutOfMemory) ? LFE_ENOMEM : LFE_EHIP;                        \
    }                                                                                    \
  } while (0)

#define LFE_TRY(expr)                                                                    \
  do {                                                                                   \
    int _rc = (expr);                                                                    \
    if (_rc != LFE_OK) return _rc;                                                       \
  } while (0)

// Per-FE device state.  Group tables are row-major [G][p] so that the p values
// of one group are contiguous (one 8*p-byte gather per row and FE).
struct FeState {
  int32_t G = 0;               // n_levels
  int32_t* code = nullptr;     // [ld] input codes (context-owned copy, input row order)
  int32_t* cnt_pre = nullptr;  // [G] pre-filter counts
  int32_t* drops = nullptr;    // [G] dropped-row counts (singleton filter)
  int32_t* cnt = nullptr;      // [G] kept counts
  int32_t cmax = 0;            // largest kept count (host copy, after the singleton drop)
  double* W = nullptr;         // [G] sum of weights over kept rows (weighted fits only)
  double* S = nullptr;         // [G*p] sum_{i in g} w_i x_i  (constant per solve)
  double* Sy = nullptr;        // [G] unweighted sum of y (weighted fits; the check is unweighted)
  double* T = nullptr;         // [G*p] cross term of the current projection
  double* alpha = nullptr;     // [G*p] group effect subtracted so far
  double* R = nullptr;         // [G] check cross term (y column, unweighted)
  double* alpha_g = nullptr;   // [G][alpha_pitch(p)] copy of alpha the general sweeps gather (whole lines)
  size_t alpha_g_cap = 0;
  double* alpha_y = nullptr;   // [G] the y column of alpha, dense (the y-only check passes gather it)
  size_t alpha_y_cap = 0;
  double* hi = nullptr;        // [G*p] coarse limbs of the sum being formed (S, W, Sy, T or R), all
                               // zero between sums: the conversion that reads an entry clears it
  // segment layout (general sweeps, lfe_seg.hip): kept rows sorted by this FE's code
  int32_t* seg_off = nullptr;  // [G + 1]
  size_t seg_off_cap = 0;
  int32_t* seg_cur = nullptr;  // [G] scatter cursors
  size_t seg_cur_cap = 0;
  int32_t* oc = nullptr;       // [F - 1][ld] the other FEs' codes, segment order
  size_t oc_cap = 0;
  int32_t* perm = nullptr;     // [ld] the layout row of every segment position (sorted build)
  size_t perm_cap = 0;
  bool perm_ok = false;        // perm holds the current segment order
  double* ws = nullptr;        // [ld] weights, segment order (weighted fits)
  size_t ws_cap = 0;
  int32_t* ufirst = nullptr;   // [units] segment holding each work unit's first row
  size_t ufirst_cap = 0;
  int32_t dims = 0, card = 0;
};

// kernel ids for per-launch event timing (lfe_profile / lfe_kernel_stats)
enum KernelId {
  K_PART_HIST = 0, K_SCAN, K_PART_SCATTER, K_COUNT, K_MARK, K_GROUP_SUMS, K_CROSS, K_CHECK, K_FINALIZE,
  K_CHECK_MAX, K_GRAM_DESIGN, K_GRAM_RESID, K_GRAM_TABLE, K_REDUCE, K_CLUSTER_SCATTER, K_MISC, K_SYNTH,
  K_TP, K_TQ, K_SEG_BUILD, K_CLUSTER_SORT, K_GRAM_TABLES, K_LAYOUT_HIST, K_LAYOUT_BASE, K_LAYOUT_SCATTER,
  K_TQ_REDUCE, K_FIX_SUMS, K_CLUSTER_FIX, K_NUM_KERNELS
};
extern const char* const kKernelNames[K_NUM_KERNELS];

struct Prof {
  bool on = false;
  std::vector<hipEvent_t> pool;  // free events
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;
  double total_ms[K_NUM_KERNELS] = {0};
  int64_t count[K_NUM_KERNELS] = {0};
  hipEvent_t open_ev = nullptr;
  int open_id = -1;
};

// cluster workspace (lfe_cluster.hip)
struct ClusterWS {
  // one-column subsets on a dense key table (no sort): the score columns' statistics and quanta,
  // the per-cluster fine limbs
  double* fixst = nullptr;      // [kColStatHead + k * nchunks] max |s_c| bits, per-chunk sums of s_c^2
  size_t fixst_cap = 0;
  double* fixq = nullptr;       // [kFqRows][kFqCols]
  size_t fixq_cap = 0;
  double* segst = nullptr;      // subsets on an FE's segments: the score rows' statistics (fixst form)
  size_t segst_cap = 0;
  bool segst_ok = false;        // segst holds this launch_cluster_subsets call's statistics
  uint64_t* keys[2] = {nullptr, nullptr};  // radix sort ping-pong
  size_t keys_cap[2] = {0, 0};
  int32_t* rows[2] = {nullptr, nullptr};
  size_t rows_cap[2] = {0, 0};
  int32_t* counts = nullptr;    // [bins][blocks] digit counts
  size_t counts_cap = 0;
  int32_t* flag = nullptr;      // [ld + 1] segment heads -> indices
  size_t flag_cap = 0;
  int32_t* seg_off = nullptr;   // [ld + 1]
  size_t seg_off_cap = 0;
  int32_t* ufirst = nullptr;
  size_t ufirst_cap = 0;
  bool lay_move = false;        // the partition moves the cluster columns into lay (prepare_layout)
  // owner-partitioned exchange (multi-rank, many clusters)
  uint64_t* skey = nullptr;     // [G_local] segment keys -> send order
  size_t skey_cap = 0;
  double* srec = nullptr;       // [G_local][k] send records
  size_t srec_cap = 0;
  double* rsum = nullptr;       // one double summed over ranks (sum_over_ranks)
  size_t rsum_cap = 0;
  uint64_t* rkey = nullptr;     // received keys
  size_t rkey_cap = 0;
  double* rrec = nullptr;       // received records
  size_t rrec_cap = 0;
  int32_t* ocnt = nullptr;      // [world] owner counts + cursors, [world * world] count matrix
  size_t ocnt_cap = 0;
  // mostly-singleton subsets: the clusters of two or more rows, compacted
  int32_t* r2 = nullptr;        // [N2] their rows, cluster by cluster (sorted order)
  size_t r2_cap = 0;
  int32_t* off2 = nullptr;      // [G + 1] scans: positions / cluster index of the multi-row clusters
  size_t off2_cap = 0;
  int32_t* idx2 = nullptr;
  size_t idx2_cap = 0;
  int32_t* seg2 = nullptr;      // [G2 + 1] their offsets in r2
  size_t seg2_cap = 0;
  double* t2 = nullptr;         // [N2][k] their score rows
  size_t t2_cap = 0;
  double* s2 = nullptr;         // [G2][k] their sums
  size_t s2_cap = 0;
  std::vector<int32_t*> lay;    // loaded cluster columns in layout order
  std::vector<size_t> lay_cap;
  bool lay_valid = false;
};

// per-phase device time of the latest call (prep, demean, gram, resid, cluster): begin/end
// events recorded on the stream, read only when lfe_timings asks (no host wait per phase)
struct Timings {
  double ms[5] = {0, 0, 0, 0, 0};
  double last = 0;
  hipEvent_t ev[5][2] = {};
  unsigned pending = 0;  // phases whose events are not read yet
  int last_phase = -1;
  bool on = false;       // lfe_phase_timing
};

// Row layout used by every pass after the singleton drop: rows grouped by
// buckets of the primary (highest-cardinality) FE, bucket b holding codes
// [b << s, (b+1) << s).  Work item = contiguous row range inside one bucket.
struct PartGeom {  // partition scatter launch geometry (lfe_prep.hip)
  int nth = 0, per = 0, nw = 0;
  size_t lds = 0;
};

struct Layout {
  int P = -1;          // primary FE (-1: no FE)
  int s = 0;           // bucket shift
  int nb = 1;          // buckets
  bool permuted = false;
  double* X = nullptr;          // [p][ld] (aliases input when !permuted)
  double* w = nullptr;          // [ld] or nullptr
  int32_t* code[kMaxFE] = {};   // per FE, bucket order; code[P][i] = -1 marks a dropped row
  int32_t* orig = nullptr;      // [ld] input row index of each layout row (nullptr = identity)
  bool orig_pending = false;    // orig not written yet (ensure_layout_orig)
  PartGeom part;
  int n_items = 0;
  std::vector<int32_t> hitems;  // host copy of the work items
  std::vector<int32_t> bstart;  // host [nb + 1]
};

}  // namespace lfe

struct lfe_ctx {
  int device = 0;
  int n_cu = 256;        // compute units of the device
  hipStream_t stream = nullptr;
  // data (row shard, input order)
  int64_t n = 0;      // rows in this shard
  int64_t ld = 0;     // leading dimension of column storage (n rounded up)
  int p = 0;          // columns: y + x (+ instruments)
  int F = 0;
  double* X = nullptr;       // [p][ld]
  double* w = nullptr;       // [ld] or nullptr
  std::vector<lfe::FeState> fe;
  // layout (bucket order) storage
  lfe::Layout L;
  int64_t dense_cells = 0;        // cells of the last demean's dense count tables (0: row layouts)
  uint16_t* dn_na = nullptr;      // dense cross-term count tables (lfe_dense.hip)
  size_t dn_na_cap = 0;
  uint16_t* dn_nb = nullptr;
  size_t dn_nb_cap = 0;
  // exact integer form of the dense passes (lfe_dense.hip, "dn8"): i8 count tables in MFMA fragment
  // order, per-block flags of cells over 127 (those blocks' counts stay in dn_na / dn_nb as u16),
  // and the secondary effects' base-128 digit fragments with their per-tile scales
  bool dn8 = false;
  int8_t* dn8_a = nullptr;
  size_t dn8_a_cap = 0;
  int8_t* dn8_b = nullptr;
  size_t dn8_b_cap = 0;
  uint8_t* dn8_fa = nullptr;
  size_t dn8_fa_cap = 0;
  uint8_t* dn8_fb = nullptr;
  size_t dn8_fb_cap = 0;
  int8_t* dn8_dq = nullptr;
  size_t dn8_dq_cap = 0;
  double* dn8_eq = nullptr;
  size_t dn8_eq_cap = 0;
  // the digits' dynamic-range guard (lfe_dense.hip dn8_tile_digits): [0] nonzero when some tile of
  // effects held most of its values 2^16 below its largest; lfe_demean then redoes the solve
  // without the dense cross terms (dense_off), and dense_coarse records that it did
  double* rflag = nullptr;
  bool any_ready = false;    // this solve's pre-filter count kernel also counted the singleton groups
  bool fixq_ready = false;   // k_finish_counts formed the group sums' quanta (lfe_fast.hip sums4)
  const double* q_first = nullptr;  // the two-FE sums' epilogue wrote alpha_Q = S_Q / n_Q there (and zeroed rflag)
  size_t rflag_cap = 0;
  bool dense_off = false;
  bool dense_coarse = false;
  // general dense sweeps (lfe_dense3.hip, three or more FEs): per ordered FE pair (a, b) the i8
  // count table of a's levels x b's levels in the K2 fragment form of the two-FE passes ([tile of 512
  // b levels][16-row block of a][8 k blocks][1 KB]), its block flags and the flagged blocks' u16
  // counts; per FE the slots of its cross term (one per tile of every other FE)
  struct D3WS {
    bool on = false;                // the last demean ran the pair-table sweeps
    int8_t* tab[lfe::kMaxFE][lfe::kMaxFE] = {};
    size_t tab_cap[lfe::kMaxFE][lfe::kMaxFE] = {};
    uint8_t* flg[lfe::kMaxFE][lfe::kMaxFE] = {};
    size_t flg_cap[lfe::kMaxFE][lfe::kMaxFE] = {};
    uint16_t* X[lfe::kMaxFE][lfe::kMaxFE] = {};
    size_t X_cap[lfe::kMaxFE][lfe::kMaxFE] = {};
    double* runs[lfe::kMaxFE] = {};
    size_t runs_cap[lfe::kMaxFE] = {};
    uint64_t* part = nullptr;       // kept rows' a & 63 and partner codes, partitioned by a >> 6
    size_t part_cap = 0;
    int32_t* hist = nullptr;        // [bins][workgroups] counts -> scanned bases
    size_t hist_cap = 0;
    int32_t* tiles = nullptr;       // [128] 0, 1, 2, ...: the passes' tile list
    int64_t table_bytes = 0;        // i8 table bytes over all ordered pairs
    uint32_t t_final = 0;           // FEs whose fe[f].T holds the cross term of the final effects
  } d3;
  double* colsum_part = nullptr;  // [p][blocks][G] fine-limb columns of k_col_sums (lfe_fast.hip)
  size_t colsum_part_cap = 0;
  double* Xp = nullptr;          // [p][ld] permuted columns
  double* wp = nullptr;          // [ld] permuted weights
  int32_t* codes_p = nullptr;    // [F][ld] permuted / working codes
  int32_t* origp = nullptr;      // [ld]
  int32_t* items_d = nullptr;    // device work items [n_items][4]
  size_t items_cap = 0;
  int32_t* bitems_d = nullptr;   // device [nb + 1]: first work item of each bucket (in items_d)
  int32_t* xitems_d = nullptr;   // device [n_xgrid]: work item of each block, XCD-grouped (-1: idle; in items_d)
  int n_xgrid = 0;
  int32_t* blist_d = nullptr;    // device [nbe]: the buckets that hold rows, in order (in items_d)
  int nbe = 0;                   // buckets that hold rows (an owner shard: its own levels' buckets)
  // segment layout (fast path, F == 2): kept rows sorted by the primary code
  int32_t* seg_off = nullptr;    // [nb * B + 1] local row offsets of each primary group
  size_t seg_off_cap = 0;
  int32_t* seg_q = nullptr;      // [ld] secondary codes in segment order
  size_t seg_q_cap = 0;
  int32_t* seg_aux = nullptr;    // [n_items * B] per-item counts -> bases
  size_t seg_aux_cap = 0;
  int32_t* seg_units = nullptr;  // [n_units] K1 work unit descriptors (int4: first / end segment, first / end row)
  size_t seg_units_cap = 0;
  // run layout (fast path): kept rows of each bucket sorted by the secondary code
  int32_t* run_off = nullptr;    // [nb * G_Q + 1] offsets of the (bucket, q) runs
  size_t run_off_cap = 0;
  uint16_t* run_h = nullptr;     // [ld] primary code - bucket base, run order
  size_t run_h_cap = 0;
  int n_units = 0;
  double* alpha_spare = nullptr; // [G_Q * p] double buffer for the secondary alpha
  size_t alpha_spare_cap = 0;
  // clusters (input row order)
  std::vector<int32_t*> cl;
  std::vector<int32_t> cl_levels;
  std::vector<int> cl_fe;  // per cluster column: the FE column it repeats (equal codes), or -1
  // the one cluster column is the primary FE: its sums came out of the residual pass (no score rows;
  // lfe_gram.hip k_resid_rows<.., true>, finished by lfe_cluster.hip)
  bool clfused = false;
  int clfused_j = -1;            // that cluster column
  bool clfused_scores = false;   // the pass wrote the score rows too (other subsets need them)
  std::vector<double> clfused_beta;  // beta_full of that pass (to redo it with score rows)
  bool clfused_done = false;         // its meat formed (the sums are converted in place: kept here)
  std::vector<double> clfused_meat;
  int64_t clfused_G = 0;
  // its sums (kept apart from the other subsets' work buffers): fine limbs, coarse limbs, counts
  // with [G, max, flag] after them, quanta
  double* clf_S = nullptr;
  double* clf_hi = nullptr;
  int32_t* clf_cnt = nullptr;
  double* clf_fq = nullptr;
  size_t clf_S_cap = 0, clf_hi_cap = 0, clf_cnt_cap = 0, clf_fq_cap = 0;
  lfe::ClusterWS clw;
  // pinned host staging (small transfers avoid the runtime's pageable path)
  char* hpin = nullptr;            // kPinSmall bytes: [0, kPinD2H) D2H results
  char* hup = nullptr;             // kPinSmall - kPinD2H bytes of small-upload staging (mapped, coherent)
  char* hup_dev = nullptr;         // its device address
  // mapped, coherent host memory the device writes small results into (no copy kernel, no event):
  // msg[0] = sequence number, msg[1..] = values; the host spins on the sequence (host_msg_wait)
  unsigned long long* hmsg = nullptr;   // host view
  unsigned long long* dmsg = nullptr;   // device view
  unsigned long long msg_seq = 0;
  hipEvent_t hpin_ev = nullptr;    // last H2D from the staging region
  hipEvent_t aux_ev = nullptr;     // completion of an asynchronous D2H into the staging region
  // the layout's work-item upload runs on its own stream while the partition scatter runs:
  // up_ev0 (main stream, before the scatter: earlier readers of items_d are done), up_ev1 (upload done)
  hipStream_t up_stream = nullptr;
  hipEvent_t up_ev0 = nullptr, up_ev1 = nullptr;
  char* hpin_items = nullptr;      // work-item upload staging
  char* hpin_items_dev = nullptr;  // its device address (mapped, coherent)
  size_t hpin_items_cap = 0;
  double* scores = nullptr;  // row-major [ld][score_k] score rows u r (w), layout order (p * ld allocated)
  double* dbeta = nullptr;   // [64] beta_full staging
  bool scores_valid = false;
  // sum over kept rows of s s' for the score rows s (the residual pass's meat tile, unweighted
  // one-process fits): the cluster meats of mostly-singleton subsets start from it (lfe_cluster.hip)
  std::vector<double> score_meat;
  bool score_meat_ok = false;
  int score_k = 0;           // score width: p - 1 (u = x~), or p with the intercept (IV, u = [1, x~, z~])
  // YOCO records (lfe_compress): the loaded rows are compressed records, weight = n_g (or sum w);
  // no singleton drop, weighted convergence check, lfe_resid_yoco's sufficient-statistic residuals
  bool records = false;
  int64_t rows_in = 0;           // rows before compression
  double* rec_sy = nullptr;      // [ld] sum (w) y per record, input (record) order
  double* rec_syy = nullptr;     // [ld] sum (w) y^2 per record
  double* rec_lay = nullptr;     // [2][ld] the two above in layout order
  size_t rec_sy_cap = 0, rec_syy_cap = 0, rec_lay_cap = 0;
  // Gram from group tables (two FEs, unweighted, one process): the group-sum pass also forms
  // the raw Gram of the shifted data columns, so lfe_gram_resid needs no design pass
  double* raw_part = nullptr;    // [blocks][256] per-block raw tiles
  size_t raw_part_cap = 0;
  double* qpart = nullptr;       // [blocks][G_Q * p] per-block secondary-FE sums (k_sums2_raw)
  size_t qpart_cap = 0;
  double* raw_slots = nullptr;   // [world][272] every rank's raw tile + shift (one grouped all-reduce)
  size_t raw_slots_cap = 0;
  // exact cross terms of the general sweeps (lfe_seg.hip): per-FE column max |alpha| (u64 bits)
  // and the quanta of the cross term being formed
  double* amax = nullptr;        // [kMaxFE][kMaxCols]
  size_t amax_cap = 0;
  double* astat = nullptr;       // [kMaxFE][kAstatBlocks][64]: per-block sum cnt alpha^2 (col 63: sum cnt)
  size_t astat_cap = 0;
  double* xq = nullptr;          // [kFqRows][kFqCols] quanta of the cross term being formed
  size_t xq_cap = 0;
  bool hi_dirty = false;         // a sum may have left coarse limbs in fe[].hi (hi_begin clears them)
  // f64 segmented sums (lfe_seg.hip, lfe_cluster.hip): the partials of segments cut by work-unit /
  // wave edges, [2][units][cols], added in unit order by a fix-up pass instead of f64 atomics
  double* chain = nullptr;
  size_t chain_cap = 0;
  double* raw_tile = nullptr;    // [256] raw tile: slots 0..p-1 data (shifted by raw_shift), slot 15 intercept
  size_t raw_tile_cap = 0;
  double* raw_shift = nullptr;   // [32]: [0, 16) the shift of raw_tile (rank 0's first row on every rank),
  size_t raw_shift_cap = 0;      //       [16, 32) this rank's own first row
  bool raw_ready = false;        // raw_tile holds this layout's kept rows
  bool tq_final = false;         // fe[Q].T = sum over q of the final alpha_P (demean_fast)
  bool hists_kept = false;       // seg_aux holds the kept rows' per-item histograms (no row dropped)
  bool dn_pre = false;           // prepare_layout built the dense tables on every row (pre-filter counts)
  bool dn_pre_valid = false;     // ... and they hold the kept rows (nothing dropped, no 16-bit overflow)
  bool sums_zeroed = false;      // prepare_layout zeroed the S tables (sums4 skips its memsets)
  // scratch
  double* scratch = nullptr;     // device partials
  size_t scratch_elems = 0;
  double* dred = nullptr;        // device reduced output (small)
  unsigned long long* scan_status = nullptr;  // k_scan_fused: per-block sums tagged with the launch's epoch
  unsigned int scan_epoch = 0;
  unsigned int* gsync = nullptr; // [kGsyncSlots] grid-completion counters (last_block_done), zero between launches
  size_t dred_elems = 0;
  int32_t* iscratch = nullptr;   // device int scratch
  size_t iscratch_elems = 0;
  int32_t* pcounts = nullptr;    // partition histogram matrix / scan
  size_t pcounts_elems = 0;
  int32_t* psums = nullptr;      // scan block sums
  size_t psums_elems = 0;
  double* clS = nullptr;         // cluster score table [C][k]
  size_t clS_elems = 0;
  int32_t* clP = nullptr;        // cluster presence flags [C] + counter
  size_t clP_elems = 0;
  // chunked upload (lfe_load_begin / lfe_load_rows / lfe_load_finish)
  hipEvent_t load_ev[2] = {nullptr, nullptr};
  int64_t load_calls = 0, load_rows_done = 0;
  bool loading = false;
  // state
  int64_t n_kept = 0;
  int64_t n_kept_local = 0;  // kept rows of this shard
  // owner-sharded ranks whose primary FE keeps a level of more than 65535 rows (summed with the kept
  // rows): the dense-path decisions use it so that every rank takes the same sweeps
  int32_t cmax_over_ranks = 0;
  bool loaded = false, prepared = false, demeaned = false;
  bool sums_ready = false;  // S (and W, Sy) already enqueued by lfe_drop_singletons
  bool seg_ready = false;   // segment layouts built for the current drop_singletons
  // distributed: an RCCL communicator, or (tests) an in-process emulated group
  ncclComm_t comm = nullptr;
  struct lfe_emu* emu = nullptr;
  int rank = 0, world = 1;
  // owner-sharded rows (lfe_ctx_set_owner): this rank holds every row whose code of FE owner_fe
  // lies in [owner_lo, owner_hi); owner_on (prepare_layout): the primary FE's tables stay local
  int owner_fe = -1;
  int32_t owner_lo = 0, owner_hi = 0;
  bool owner_on = false;
  int test_hooks = 0;
  int64_t synth_row0 = 0;  // lfe_synth_load_codes_at: the synthetic panel's global index of row 0  // lfe_ctx_test_hooks (LFE_TEST_* bits; tests only, 0 in production)
  // deterministic T_Q: per-(bucket, q) run sums reduced in bucket order (no cross-bucket atomics)
  double* tq_runs = nullptr;     // [nb * G_Q][p]
  size_t tq_runs_cap = 0;
  // exact group sums (k_sums2_raw): the column statistics of the loaded rows (written by the
  // partition, or k_col_stats) fix a per-column 2^-e quantum, and the group sums accumulate
  // round(x / quantum) in int64, so their order never changes a bit (lfe_fast.hip)
  double* colstat = nullptr;     // [kColStatHead + p * nchunks]: max |x_c| bits (as u64), then sum x_c^2 per column and chunk
  size_t colstat_cap = 0;
  int colstat_chunks = 0;        // chunks of per-chunk sums of squares written for this layout
  double* fixq = nullptr;        // [kFqRows][kFqCols] quanta of the group sums (fix_quanta_col)
  double* colq = nullptr;        // [kMaxCols + 1] column sums of squares (k_finish_counts' quanta)
  size_t colq_cap = 0;
  size_t fixq_cap = 0;
  bool exact_sums = false;       // the group sums of this layout were formed (always two-limb fixed point)
  // speculative Gram tile + Cholesky of the converged tables (gram_spec_enqueue), valid until the
  // next load / drop / demean: [0, 256) tile, 516 ok, [520, 532) beta, 532 guard (launch_gram_resid)
  double* dspec = nullptr;
  size_t dspec_elems = 0;
  bool gram_spec = false;
  // out-of-core X (lfe_load_codes + lfe_stream_*): codes resident, X streamed in row chunks
  struct StreamWS {
    bool on = false;       // codes-only context
    int pass = 0;          // 0 idle, 1 group sums + raw Gram, 2 residual, 3 design Gram
    int64_t rows_done = 0;
    double* x = nullptr;   // [p][cld] the chunk's columns
    size_t x_cap = 0;
    double* s64 = nullptr;   // [sum_f G_f p] chunk group sums, int64 bits (exact path)
    size_t s64_cap = 0;
    double* sdbl = nullptr;  // the same in f64 (a chunk whose range defeats the fixed point)
    size_t sdbl_cap = 0;
    double* tile = nullptr;  // [ts * ts + 4] tile (+ statistics) accumulated over the chunks, in order
    size_t tile_cap = 0;
    int ts = 16;             // tile stride: 16 for p <= 11 (row-per-lane passes), else 16 * ceil((p + 1) / 16)
    double* red = nullptr;   // wide passes: the chunk's reduced MFMA blocks (+ statistics)
    size_t red_cap = 0;
    double* toff = nullptr;  // [4 kMaxFE] 8-byte slots: table ends (int64), S / W / Sy pointers per FE
    size_t toff_cap = 0;
    int icpt = 0;            // pass 4: the IV residual over u = [1, x~, z~]
    // pass 5 (lfe_stream_materialize): the chunks' demeaned columns into a caller's matrix
    double* mD = nullptr;    // [cols][mld], input row order (0 on dropped rows)
    int64_t mld = 0;
    int64_t mbase = 0, mrows = -1;  // lfe_stream_materialize_rows: D row = row - mbase over mrows rows (-1: all)
    int mcol0 = 0, mmask = -1;  // first target column; kept-row indicator column (-1: none)
    // clustered SEs (lfe_stream_clusters): every subset's dense cluster id per input row, and the
    // per-cluster score sums the residual passes add in chunk order
    std::vector<int32_t> masks;
    std::vector<int32_t*> cid;   // [n] per subset (-1: dropped row)
    std::vector<int32_t> G;      // clusters per subset
    std::vector<double*> S;      // [G][ks] per subset
    std::vector<uint64_t*> ukey; // multi-rank: [G] the intersection key of every local cluster per subset
    std::vector<uint64_t> span;  // key span per subset
    std::vector<size_t> S_cap;
    int ks = 0;                  // score width of the sums in S
    double* sc = nullptr;        // [rows][ks] the chunk's score rows
    size_t sc_cap = 0;
  } sw;
  lfe::Timings tm;
  lfe::Prof prof;
};

namespace lfe {

// --- prep / partition (lfe_prep.hip) ---
int prepare_layout(lfe_ctx* c);   // partition + counts + singleton marks
int ensure_layout_orig(lfe_ctx* c);  // L.orig written (deferred by prepare_layout)
int exact_sums_on(lfe_ctx* c, int* on);  // did the last group sums take the exact (int64) path
// coarse-limb tables fe[].hi: clean (zero) on return; the caller's kernels may then write them
// until the conversions that read and clear them are enqueued (hi_end)
int hi_begin(lfe_ctx* c);
inline void hi_end(lfe_ctx* c) { c->hi_dirty = false; }

// --- group sums (lfe_fast.hip) ---
int sums4(lfe_ctx* c);
// --- two-FE sweeps (lfe_iter.hip) ---
bool fast_path_ok(const lfe_ctx* c, const std::vector<int>& order);
bool fast_layout_ok(const lfe_ctx* c);            // the two-FE layouts fit (any FE order)
int layout_hists(lfe_ctx* c, int Q);              // per-item histograms of both codes -> seg_aux
int demean_fast(lfe_ctx* c, double tol, int max_iter, int check_from, int* iterations_out, double* last_out);
// lfe_dense.hip: the two-FE cross terms as count-table products on the matrix cores
bool dense_ok(const lfe_ctx* c);
int dense_build(lfe_ctx* c, bool pre = false);  // pre: before the marks, every row, with the pre-filter counts
bool dense_pre_ok(const lfe_ctx* c);
// the guard's flag: zeroed at the start of a dense solve; read with the stop test (read_check)
int range_flag_reset(lfe_ctx* c);
int64_t dense_table_cells(const lfe_ctx* c);
int dense_tp(lfe_ctx* c, const double* alphaQ, double* zero_check);
int dense_tq(lfe_ctx* c, double* runs);
// the secondary effects' digit fragments for the exact K1 pass (after every alpha_Q update)
int dense_digits_q(lfe_ctx* c, const double* alphaQ);
// one product pass over a pair table in the K2 fragment form (lfe_dense.hip): slots
// runs[t][G_rows][ldo] (columns [0, pc)) = the table's tile t times alpha_k's rows of that tile
struct PairPass {
  const int8_t* tab;
  const uint8_t* flg;
  const uint16_t* X;
  const int32_t* tiles;   // [ntile_k] 0, 1, ...
  int ntile_k, nrb;       // tiles of the k-side FE, 16-row blocks of the output FE
  int G_rows, G_k, pc;    // levels of both FEs, columns of this pass (<= 16)
  int lda, ldo;           // row strides of alpha_k and of the slots
  const double* alpha;    // alpha_k (+ the column offset)
  double* runs;           // the slots (+ the column offset)
};
int dn8_pair_pass(lfe_ctx* c, const PairPass& pp);
int dn8_pair_passes(lfe_ctx* c, const PairPass* pp, int n);  // up to 8 per launch
// lfe_dense3.hip: three or more FEs, unweighted - every cross term from the pair tables
bool dense3_ok(const lfe_ctx* c, const std::vector<int>& order, int check_from);
int demean_dense3(lfe_ctx* c, const std::vector<int>& order, double tol, int max_iter, int check_from,
                  int* iterations_out, double* last_out);
void free_dense3(lfe_ctx* c);
// the cross terms fe[f].T of every FE from the final effects (the Gram from the tables)
int dense3_final_T(lfe_ctx* c);

// --- constant sums (lfe_sweep.hip) ---
int sweep_group_sums(lfe_ctx* c);
// --- general sweeps (lfe_seg.hip) ---
int seg_build(lfe_ctx* c);
int demean_generic(lfe_ctx* c, const std::vector<int>& order, double tol, int max_iter, int check_from,
                   int* iterations_out, double* last_out);

// --- Gram / residual / clusters (lfe_gram.hip) ---
int launch_gram(lfe_ctx* c, double* host_gram);
int launch_resid(lfe_ctx* c, const double* beta_full, double* stats, double* hc1, int keep_scores, int icpt);
int launch_gram_resid(lfe_ctx* c, double* host_gram, double* beta_full, double* stats, double* hc1, int keep_scores);
// speculative Gram-from-tables + device Cholesky, enqueued behind a convergence check's read-back
// so that the GPU keeps working while the host decides (lfe_gram.hip); *queued = 1 if enqueued
int gram_spec_enqueue(lfe_ctx* c, int* queued, const unsigned long long* gate = nullptr, double tol = 0.0);
// out-of-core X (lfe_fast.hip / lfe_gram.hip): one streamed chunk ([p][ld] on the device)
int stream_sums_chunk(lfe_ctx* c, const double* X, int64_t ld, int64_t row0, int64_t rows, bool first);
int stream_weight_stats(lfe_ctx* c);
// clustered SEs of streamed fits (lfe_stream.hip)
int stream_clusters_prep(lfe_ctx* c, int n_subsets, const int32_t* masks);
int stream_clusters_chunk(lfe_ctx* c, int64_t row0, int64_t rows);
int stream_cluster_meats(lfe_ctx* c, double* meats, int64_t* G_out);
void free_stream_clusters(lfe_ctx* c);
// clusters of sorted (key, row) pairs: segment offsets in clw.seg_off, per-cluster sums of the rows'
// records in c->clS (lfe_cluster.hip)
int group_sorted(lfe_ctx* c, int64_t n, uint64_t drop, const uint64_t* K, const int32_t* R, const double* table,
                 int k, int32_t* G_out);  // weighted streamed fits: w's max / rms into fixq column p
int cluster_fused_col(const lfe_ctx* c);                       // lfe_cluster.hip (-1: none)
int cluster_fused_prepare(lfe_ctx* c);                         // buffers and counts, before the pass
int cluster_fused_reset(lfe_ctx* c, const double* tile, const double* beta);  // zeroed sums + quanta
int launch_resid(lfe_ctx* c, const double* beta_full, double* stats, double* hc1, int keep_scores, int icpt);
int launch_codes_differ(lfe_ctx* c, const int32_t* a, const int32_t* b, int64_t n, int32_t* flag);  // lfe_cluster.hip
int stream_materialize_chunk(lfe_ctx* c, const double* X, int64_t ld, int64_t row0, int64_t rows);  // lfe_wide.hip
int stream_rows_chunk(lfe_ctx* c, int mode, int icpt, const double* X, int64_t ld, int64_t row0, int64_t rows,
                      double* scores);
// streamed tile stride for p data columns: the p <= 11 row-per-lane passes use the 16 x 16 tile of
// the resident kernels; wider fits the MFMA passes' 16 * ceil((p + 1) / 16) (design Gram of [1, y~, x~])
inline int stream_tile_stride(int p) { return p <= 11 ? 16 : 16 * ((p + 1 + 15) / 16); }
inline size_t stream_tile_len(int p) { const size_t t = (size_t)stream_tile_stride(p); return t * t + 4; }
void stream_tile_add(lfe_ctx* c, const double* t, int m);
int launch_table_gram(lfe_ctx* c, const double* table, int64_t rows, int k, double* meat,
                      const int32_t* idx = nullptr);  // idx: row q of the Gram = table row idx[q]
// lfe_fast.hip: quanta of `ncols` columns from colstat-form statistics (max count: the max of cmax[0..nfe)),
// and a [m] two-limb table (fine limbs' bits in S, coarse limbs in hi) -> double in place
int launch_fix_quanta(lfe_ctx* c, const double* st, int nchunks, int64_t n, const int32_t* cmax, int nfe, double* fq,
                      int ncols);
int launch_fix_convert(lfe_ctx* c, double* S, double* hi, int64_t m, int p, const double* fq);
void reduce_tiles(lfe_ctx* c, const double* part, int nblocks, double* out);  // sum of [nblocks][256] tiles
// --- YOCO records (lfe_compress.hip) ---
int records_layout(lfe_ctx* c);   // rec_sy / rec_syy in layout order -> rec_lay
// --- device keys (lfe_keys.hip) ---
int bit_length(uint64_t v);
int ensure_sort_ws(lfe_ctx* c, size_t n);
int radix_sort(lfe_ctx* c, int64_t n, int bits, int* out_buf);
int radix_pass(lfe_ctx* c, int64_t n, int shift, int cur, int kid);
// --- clusters (lfe_cluster.hip) ---
int launch_cluster_subsets(lfe_ctx* c, int n_subsets, const int32_t* masks, double* meats, int64_t* G_out);
// per-row cluster ids (input row order) of subset `mask` over the loaded cluster columns; rows with
// kept[i] == 0 get -1; *G_out: the id range (a column's levels, or an intersection's segments)
int cluster_ids_input(lfe_ctx* c, int mask, const double* kept, int32_t* cid, int32_t* G_out);
// multi-rank: per-cluster score rows S[G][k] (keys K[seg_off[h]], or K[h] with seg_off null) exchanged
// to their owner ranks, merged by key; the k x k meat and the global cluster count
int owner_meat(lfe_ctx* c, const uint64_t* K, const int32_t* seg_off, const double* S, int32_t G, int k,
               uint64_t span, double* meat, int64_t* G_out);
void free_cluster_ws(lfe_ctx* c);
// --- segmented gather-sums (lfe_seg.hip) ---
// cluster score sums over FE f's segments (the sorted build's permutation), two-limb (lfe_seg.hip)
int seg_score_sums(lfe_ctx* c, int f, const double* table, int cols, const double* xq, double* S, double* Shi,
                   int kid);
int seg_gather_sum(lfe_ctx* c, const int32_t* seg_off, int32_t G, int32_t* ufirst, int64_t n_pos,
                   const int32_t* rows, const double* table, int stride, int cols, double* out, int kid);
int seg_units_needed(int64_t n_pos);
int launch_copy_demeaned(lfe_ctx* c, double* dev_out);
int launch_validate_codes(const int32_t* code, int64_t n, int32_t G, int32_t* flag, hipStream_t s);

// --- synthetic panel (lfe_synth.hip) ---
int synth_cols_chunk(lfe_ctx* c, int K, int c_lo, const int32_t* levels, const double* beta, uint64_t seed,
                     int64_t row0, int64_t rows, double* X, int64_t ld);
int synth_chunk(lfe_ctx* c, int k, const int32_t* levels, const double* beta, uint64_t seed, int64_t row0,
                int64_t rows, double* X, int64_t ld);
int synth_codes(lfe_ctx* c, const int32_t* levels, uint64_t seed, int64_t row0);
int launch_synth(lfe_ctx* c, int k, const int32_t* levels, const double* beta, uint64_t seed,
                 int64_t row_offset);
// owner-sharded synthetic shard: count the rows of [0, n_total) whose code of FE f is in [lo, hi)
// (per-chunk bases, *n_local), then (after alloc_data(n_local)) generate them in row order
int synth_count_owned(lfe_ctx* c, int64_t n_total, int f, int32_t L, int32_t lo, int32_t hi, uint64_t seed,
                      std::vector<int64_t>& base, int64_t* n_local);
int launch_synth_owned(lfe_ctx* c, int64_t n_total, int k, const int32_t* levels, const double* beta, uint64_t seed,
                       int f, int32_t lo, int32_t hi, const std::vector<int64_t>& base);
// flag (atomic max into *flag) any code outside [lo, hi)
int launch_validate_range(const int32_t* code, int64_t n, int32_t lo, int32_t hi, int32_t* flag, hipStream_t s);

// --- owner re-shard (lfe_shard.hip) ---
int reshard_owner(lfe_ctx* c, int fe, int32_t* lo_out, int32_t* hi_out);

// --- helpers (lfe_capi.hip) ---
// (re)allocate the shard's buffers for n rows (frees every derived table and the cluster columns)
int alloc_shard(lfe_ctx* c, int64_t n, int p, int F, const int32_t* n_levels, bool weighted);
int ensure_scratch(lfe_ctx* c, size_t elems);
int ensure_dred(lfe_ctx* c, size_t elems);
int ensure_iscratch(lfe_ctx* c, size_t elems);
int ensure_pcounts(lfe_ctx* c, size_t elems, size_t sums);
int ensure_items(lfe_ctx* c, size_t n_items);
int ensure_i32(lfe_ctx* c, int32_t*& p, size_t& cap, size_t elems);
int ensure_f64(lfe_ctx* c, double*& p, size_t& cap, size_t elems);
int ensure_u16(lfe_ctx* c, uint16_t*& p, size_t& cap, size_t elems);
int ensure_u64(lfe_ctx* c, uint64_t*& p, size_t& cap, size_t elems);
int ensure_i8(lfe_ctx* c, int8_t*& p, size_t& cap, size_t elems);
int ensure_u8(lfe_ctx* c, uint8_t*& p, size_t& cap, size_t elems);
template <typename T>
inline void dfree_any(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}
int exclusive_scan(lfe_ctx* c, int32_t* a, int64_t m);
// two independent exclusive scans in one set of launches (a2 may be null)
int exclusive_scan2(lfe_ctx* c, int32_t* a1, int64_t m1, int32_t* a2, int64_t m2);
// *any += 1 (per wave) if some level of cnt[0, G) has a count of one (a singleton test)
int launch_any_eq1(lfe_ctx* c, const int32_t* cnt, int32_t G, int32_t* any);
// zero up to 32 device ranges (byte counts multiples of 4) in one launch instead of a memset each
int zero_ranges(lfe_ctx* c, const std::vector<std::pair<void*, size_t>>& ranges);
// the same ranges as kernel arguments, for a kernel that zeroes them beside its own work
// (lfe_prep.hip k_part_hist): range j covers words [end[j - 1], end[j]) of the concatenation
struct ZeroArgs {
  uint32_t* p[32];
  int64_t end[32];
  int n;
};
int build_zero_args(const std::vector<std::pair<void*, size_t>>& ranges, ZeroArgs* a, int64_t* words);
// thread t of nt: every range in turn, its 16-byte-aligned body in 16-byte stores
__device__ inline void zero_ranges_part(const ZeroArgs& a, int64_t t, int64_t nt) {
  for (int j = 0; j < a.n; ++j) {
    uint32_t* p = a.p[j];
    const int64_t len = a.end[j] - (j ? a.end[j - 1] : 0);
    const int64_t head = min(len, (int64_t)(((16 - (reinterpret_cast<uintptr_t>(p) & 15)) & 15) / 4));
    const int64_t nb = (len - head) / 4;
    uint4* q = reinterpret_cast<uint4*>(p + head);
    for (int64_t e = t; e < head; e += nt) p[e] = 0u;
    for (int64_t e = t; e < nb; e += nt) q[e] = uint4{0u, 0u, 0u, 0u};
    for (int64_t e = head + 4 * nb + t; e < len; e += nt) p[e] = 0u;
  }
}
// device -> host copy of a small result through pinned staging, synchronizing the stream
int d2h_sync(lfe_ctx* c, void* dst, const void* src_dev, size_t bytes);
// device -> host copy into the pinned staging region without waiting; d2h_wait finishes it
int d2h_async(lfe_ctx* c, const void* src_dev, size_t bytes);
int d2h_wait(lfe_ctx* c, void* dst, size_t bytes);
int host_msg_wait(lfe_ctx* c, unsigned long long seq, double* vals, int nvals);
// small device results go to the host through the mapped message (one rank; knob LFE_HOST_MSG=0: copies)
bool host_msg_on(const lfe_ctx* c);
// the next message's sequence number (its 32-bit tag is never 0: the zeroed buffer's)
inline unsigned long long next_msg_seq(lfe_ctx* c) {
  if (((++c->msg_seq) & 0xffffffffull) == 0) ++c->msg_seq;
  return c->msg_seq;
}
int host_msg_wait_i32(lfe_ctx* c, unsigned long long seq, int32_t* vals, int n);
// host -> device copy of a small argument through pinned staging (asynchronous)
int h2d_small(lfe_ctx* c, void* dst_dev, const void* src, size_t bytes);
// pinned upload buffer of at least `bytes` (work items)
int ensure_pinned_items(lfe_ctx* c, size_t bytes);
// blocks of `fn` that fit on the whole device at once (occupancy API x CUs)
int resident_blocks(lfe_ctx* c, const void* fn, int threads, size_t dyn_lds);
// grid of a row pass over the work items (block_rows splits the rows evenly over the grid):
// the resident blocks, but no more than one per kRowBlockMin rows or per item, whichever is more
// (a small fit's few items no longer leave CUs idle: 1M rows = ~160 items for 256 CUs)
constexpr int64_t kRowBlockMin = 2048;
inline int row_blocks(const lfe_ctx* c, int resident) {
  const auto& h = c->L.hitems;
  const int64_t rows = h.size() >= 4 ? h[h.size() - 2] : 0;
  const int64_t want = std::max<int64_t>(c->L.n_items, (rows + kRowBlockMin - 1) / kRowBlockMin);
  return (int)std::max<int64_t>(1, std::min<int64_t>(resident, want));
}
int ensure_cluster_ws(lfe_ctx* c, size_t table_elems, size_t flag_elems);
int allreduce_sum_f64(lfe_ctx* c, double* dev, size_t count);
int allreduce_sum_f64_many(lfe_ctx* c, const std::vector<std::pair<double*, size_t>>& bufs);
int allreduce_sum_i32(lfe_ctx* c, int32_t* dev, size_t count);
int allreduce_max_f64(lfe_ctx* c, double* dev, size_t count);
int allreduce_max_u64(lfe_ctx* c, uint64_t* dev, size_t count);
int allreduce_max_i32(lfe_ctx* c, int32_t* dev, size_t count);
int alltoallv_bytes(lfe_ctx* c, const char* send, const size_t* send_off, const size_t* send_bytes, char* recv,
                    const size_t* recv_off, const size_t* recv_bytes);
void prof_begin(lfe_ctx* c, int kid);
void prof_end(lfe_ctx* c);
int prof_fold(lfe_ctx* c);

// RAII bracket around one launch
struct ProfScope {
  lfe_ctx* c;
  ProfScope(lfe_ctx* c_, int kid) : c(c_) { prof_begin(c, kid); }
  ~ProfScope() { prof_end(c); }
};

inline int grid_for(int64_t n, int block = kBlock, int cap = 256 * 8) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// group-by equality of f64 values (keys of distinct rows and YOCO records):
// -0.0 == 0.0 and every NaN alike
__device__ __forceinline__ uint64_t canon_bits(double v) {
  if (v != v) return 0x7ff8000000000000ull;
  if (v == 0.0) return 0ull;
  return (uint64_t)__double_as_longlong(v);
}

// Element (row, col) of a row-major [rows][p] f64 table in LDS, addressed with one 24-bit
// multiply-add on byte offsets (v_mad_u32_u24; a 32-bit v_mul_lo_u32 issues at quarter rate).
// row < 2^24 and p8 = 8 p, col8 = 8 col.
__device__ __forceinline__ double lds_row(const double* t, uint32_t row, uint32_t p8, uint32_t col8) {
  return *reinterpret_cast<const double*>(reinterpret_cast<const char*>(t) + (__umul24(row, p8) + col8));
}
// Stage n contiguous doubles (global, 16-byte aligned) into LDS (16-byte aligned) as dst[0, n),
// or, with pitch > 0, row g of `width` doubles to dst + g * pitch (rows of a table into padded LDS
// rows).  Every thread issues up to 8 16-byte loads before its stores, so a staging loop no longer
// waits out one global latency per element per thread (K1 / K2 / residual-pass prologues).
template <int NTH>
__device__ __forceinline__ void stage_lds(double* __restrict__ dst, const double* __restrict__ src, int n, int tid,
                                          int width = 0, int pitch = 0) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  const int n2 = n >> 1;
  const d2* s2 = reinterpret_cast<const d2*>(src);
  auto put = [&](int j, double v) {
    if (pitch > 0) {
      const int g = j / width;
      dst[g * pitch + (j - g * width)] = v;
    } else {
      dst[j] = v;
    }
  };
  for (int base = 0; base < n2; base += 8 * NTH) {
    d2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = base + u * NTH + tid;
      v[u] = i < n2 ? s2[i] : d2{0.0, 0.0};
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = base + u * NTH + tid;
      if (i < n2) {
        put(2 * i, v[u].x);
        put(2 * i + 1, v[u].y);
      }
    }
  }
  if ((n & 1) && tid == 0) put(n - 1, src[n - 1]);
}

__device__ __forceinline__ double* lds_row_ptr(double* t, uint32_t row, uint32_t p8, uint32_t col8) {
  return reinterpret_cast<double*>(reinterpret_cast<char*>(t) + (__umul24(row, p8) + col8));
}

// one 64-bit DPP lane move (two 32-bit halves); lanes without a source (or outside ROWMASK)
// get idv
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp64(double v, double idv) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(idv), __double2loint(v), CTRL, ROWMASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(idv), __double2hiint(v), CTRL, ROWMASK, 0xF, false);
  return __hiloint2double(hi, lo);
}
// reductions over VALU lane moves (no LDS traffic) in a fixed order, so the result is the
// same every run.  row16: row_shr 1/2/4/8 (a scan within each row of 16; lane 15 of a row
// holds its total); wave63: then row_bcast:15 and row_bcast:31 - lane 63 holds the total
template <class Op>
__device__ __forceinline__ double row16_reduce15(double v, double idv, Op op) {
  v = op(v, dpp64<0x111, 0xF>(v, idv));
  v = op(v, dpp64<0x112, 0xF>(v, idv));
  v = op(v, dpp64<0x114, 0xF>(v, idv));
  v = op(v, dpp64<0x118, 0xF>(v, idv));
  return v;
}
// Grid completion of a fused reduction (one launch instead of a kernel and a one-block finisher):
// every workgroup calls it once, with all its threads, after its global writes; it returns true in
// exactly one workgroup - the last to arrive - which then sees every other workgroup's writes
// (agent-scope release before the count, acquire after it).  *counter is 0 at launch and 0 again
// when the last workgroup leaves, so a slot serves one launch at a time on its context's stream.
// Host messages (lfe_ctx::dmsg, mapped coherent host memory): every word carries the low 32 bits of
// the message's sequence number above 32 payload bits, so the host checks each word by itself and
// the device needs no release fence (a system-scope release writes the whole L2 back): relaxed
// system-scope stores only.  A double takes two words (low, high half).
__device__ __forceinline__ void host_msg_word(unsigned long long* msg, int i, unsigned long long seq, unsigned int v) {
  __hip_atomic_store(&msg[i], ((seq & 0xffffffffull) << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void host_msg_publish(unsigned long long* msg, unsigned long long seq, const double* v, int nv) {
  for (int i = 0; i < nv; ++i) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v[i]);
    host_msg_word(msg, 2 * i, seq, (unsigned int)b);
    host_msg_word(msg, 2 * i + 1, seq, (unsigned int)(b >> 32));
  }
}
// ... n int32 values (agent-scope loads of what other workgroups wrote), one word each
__device__ __forceinline__ void host_msg_publish_i32(unsigned long long* msg, unsigned long long seq,
                                                     const int32_t* v, int n) {
  for (int i = 0; i < n; ++i)
    host_msg_word(msg, i, seq, (unsigned int)__hip_atomic_load(&v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

constexpr int kGsyncSlots = 16;
constexpr size_t kHostMsgBytes = 16384;  // lfe_ctx::hmsg: 2048 tagged words (1024 doubles)
enum GsyncSlot { GS_SPARE = 0, GS_RESID = 1, GS_FINISH = 2, GS_SPARE2 = 3, GS_SPARE1 = 4, GS_SCAN = 5, GS_TQ_REDUCE = 6, GS_SCAN_DONE = 7 };
__device__ __forceinline__ bool last_block_done(unsigned int* counter) {
  __shared__ unsigned int amlast;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned int total = gridDim.x * gridDim.y * gridDim.z;
    const unsigned int t = atomicAdd(counter, 1u);
    amlast = t == total - 1 ? 1u : 0u;
    if (amlast) atomicExch(counter, 0u);
  }
  __syncthreads();
  if (amlast) __threadfence();
  return amlast != 0;
}

template <class Op>
__device__ __forceinline__ double wave_reduce63(double v, double idv, Op op) {
  v = row16_reduce15(v, idv, op);
  v = op(v, dpp64<0x142, 0xA>(v, idv));
  v = op(v, dpp64<0x143, 0xC>(v, idv));
  return v;
}

// row pitch (doubles) of the gathered effect tables: a row of p <= 16 doubles in one 32/64/128-byte
// aligned segment, so a random gather touches one cache line instead of up to two
inline int alpha_pitch(int p) { return p <= 4 ? 4 : p <= 8 ? 8 : (p + 15) / 16 * 16; }

// ---------------------------------------------------------------------------
// Two-limb fixed-point sums: every group sum, cross term and weight sum of the demeaning loop
// is order-independent, so its bits do not depend on which wave or block adds first.
//
// Per column a quanta table fixes a coarse quantum Qc = 2^b and a fine scale sf = 2^s.  A value
// v enters a sum as
//     h  = round(v / Qc)                  (the coarse limb: an integer-valued double)
//     lo = round((v - h Qc) * sf)         (the fine limb: int64)
// Qc / 2 exceeds every typical value (min(max |v|, 64 rms)), so h = 0 for them and only
// outliers touch the coarse limb.  The bounds keep both limbs exact whatever the order: a sum
// of |h| over one group stays below 2^51 (f64 adds of integers below 2^53 are exact, so the
// coarse limbs may use f64 atomics), a sum of |lo| below 2^62 (int64 adds commute).  A
// non-finite v goes to the coarse limb itself (NaN / Inf propagate as in an f64 sum, in any
// order).  The sum is then lo_sum / sf + h_sum Qc.  Per value the rounding is at most
// 1 / (2 sf) = Qc 2^-min(64 - e_N, 53) (N < 2^e_N rows per group): 2^-41 of 64 rms at N = 2^16.
// ---------------------------------------------------------------------------
constexpr int kFqCols = kMaxCols + 3;
constexpr int kAstatBlocks = 256;       // blocks of the effect-table statistics (k_alpha_stats)   // quanta table columns: p data columns (+ w, raw y)
enum { FQ_SF = 0, FQ_QF = 1, FQ_BIG = 2, FQ_IQC = 3, FQ_QC = 4, FQ_RMS = 5, FQ_MAX = 6, FQ_SF2 = 7, kFqRows = 8 };
constexpr double kFixRange = 64.0;      // typical values: |v| <= kFixRange * rms
constexpr double kFixMagic = 6755399441055744.0;  // 1.5 * 2^52: fma(v, s, magic) - magic = round(v s)
constexpr unsigned long long kFixMagicBits = 0x4338000000000000ull;

struct FixCol {
  double sf = 0.0, iqc = 0.0, qc = 0.0;
  double sf2 = 1.0;  // the fine scale is sf * sf2 (two exact powers of two: 2^s overflows past s = 1023)
  bool big = false;  // some value of the column may have a coarse limb
};
__device__ __forceinline__ FixCol fix_col(const double* __restrict__ fq, int c) {
  FixCol q;
  q.sf = fq[FQ_SF * kFqCols + c];
  q.sf2 = fq[FQ_SF2 * kFqCols + c];
  q.big = fq[FQ_BIG * kFqCols + c] != 0.0;
  q.iqc = fq[FQ_IQC * kFqCols + c];
  q.qc = fq[FQ_QC * kFqCols + c];
  return q;
}
// the fine limb of v (returned) and its coarse limb h (0 for a typical value)
__device__ __forceinline__ unsigned long long fix_split(double v, const FixCol& q, double& h) {
  h = 0.0;
  if (q.big) {
    h = __builtin_fma(v, q.iqc, kFixMagic) - kFixMagic;     // round(v / Qc); NaN / Inf stay
    v = __builtin_isfinite(h) ? __builtin_fma(-h, q.qc, v) : 0.0;  // exact remainder, |.| <= Qc / 2
  }
  return (unsigned long long)__double_as_longlong(__builtin_fma(v * q.sf2, q.sf, kFixMagic)) - kFixMagicBits;
}
// the sum of a table entry from its limbs (fine: int64 bits, coarse: f64)
__device__ __forceinline__ double fix_value(unsigned long long lo, double hi, const double* __restrict__ fq, int c) {
  const double v = (double)(long long)lo * fq[FQ_QF * kFqCols + c];
  return hi != 0.0 ? v + hi * fq[FQ_QC * kFqCols + c] : v;
}
// quanta of one column from its statistics: M = max |v| (maybe Inf), rms (maybe NaN), N = the
// largest number of values one sum adds (all written to fq[r * kFqCols + c])
__device__ inline void fix_quanta_col(double M, double rms, double N, double* __restrict__ fq, int c) {
  const bool finite = __builtin_isfinite(M) && __builtin_isfinite(rms);
  int eN = 0;
  (void)frexp(fmax(N, 1.0), &eN);  // N < 2^eN
  int b = 0;                        // Qc = 2^b
  if (finite && M > 0.0) {
    const double T = fmin(M, kFixRange * rms);
    int a = 0;
    (void)frexp(T > 0.0 ? T : M, &a);  // T < 2^a: |v| <= T rounds to h = 0 with Qc = 2^(a + 1)
    b = a + 1;
    while (fmax(N, 1.0) * (ldexp(M, -b) + 1.0) >= 0x1p51) ++b;  // sum of |h| over one group < 2^51
    b = min(b, 1023);  // Qc finite (a column of values near DBL_MAX)
  }
  // sum of |lo| <= N 2^(b-1) 2^s < 2^62, |lo| <= 2^51; s <= 1074 keeps the quantum 2^-s a (subnormal)
  // double, and the scale goes in two factors once s passes 1000 (a column of values near 1e-300)
  const int s = min(min(63 - eN, 52) - b, 1074);
  const int s2 = s > 1000 ? s - 1000 : 0;
  fq[FQ_SF * kFqCols + c] = ldexp(1.0, s - s2);
  fq[FQ_SF2 * kFqCols + c] = ldexp(1.0, s2);
  fq[FQ_QF * kFqCols + c] = ldexp(1.0, -s);
  // (a margin below Qc / 2: a value may exceed its bound M by the rounding of the sum it came from)
  fq[FQ_BIG * kFqCols + c] = (!finite || M >= ldexp(1.0 - 0x1p-20, b - 1)) ? 1.0 : 0.0;
  fq[FQ_IQC * kFqCols + c] = ldexp(1.0, -b);
  fq[FQ_QC * kFqCols + c] = ldexp(1.0, b);
  fq[FQ_RMS * kFqCols + c] = rms;
  fq[FQ_MAX * kFqCols + c] = M;
}

// Balanced row ranges for the streaming X passes: block b of the grid walks layout rows
// [lo, hi) (equal shares, multiples of 64), i.e. the items from `first` on, each clipped to
// [lo, hi) (whole items per block left some blocks a full 8192-row item more than others: +30%
// at 3 items per block).  Every wave finds `first` - the first item ending after lo - by a
// 64-ary search over the items' ends (3 dependent loads at ~6K items).
struct BlockRows {
  int first, lo, hi;
};
__device__ __forceinline__ BlockRows block_rows(const int4* __restrict__ items, int n_items, int lane,
                                                int64_t b = -1, int64_t nb = -1) {
  BlockRows r{0, 0, 0};
  if (n_items <= 0) return r;
  if (b < 0) {  // block b of nb (default: this block of the grid)
    b = blockIdx.x;
    nb = gridDim.x;
  }
  const int64_t total = items[n_items - 1].z;
  r.lo = (int)((total * b / nb) & ~63ll);
  r.hi = b + 1 == nb ? (int)total : (int)((total * (b + 1) / nb) & ~63ll);
  int lo = 0, hi = n_items;  // the answer lies in [lo, hi]
  while (lo < hi) {
    const int step = (hi - lo + 63) / 64;
    const int idx = lo + lane * step;
    const bool inr = idx < hi;
    const bool past = inr && items[idx].z > r.lo;  // monotone in idx
    const int f = __popcll(__ballot(inr && !past));
    const int cand = lo + f * step;
    hi = cand < hi ? cand : hi;
    lo = step == 1 ? hi : (f > 0 ? lo + (f - 1) * step + 1 : lo);
  }
  r.first = lo;
  return r;
}

__device__ __forceinline__ uint64_t fmix64(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  h ^= h >> 33;
  return h;
}

// What every sweep / Gram kernel needs to evaluate x~_i = x_i - sum_f alpha_f[g_f(i)]
// on the layout: codes in layout order, alpha tables, primary FE bucket geometry.
struct LayoutArgs {
  int F, p, P, s;
  const int32_t* code[kMaxFE];
  const double* alpha[kMaxFE];
  const int4* items;
  int n_items;
};
LayoutArgs layout_args(const lfe_ctx* c);

}  // namespace lfe
