// Internal declarations shared by the leanfe HIP engine translation units.
// Target: gfx950 (MI355X, CDNA4) only.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/leanfe_hip.h"

namespace lfe {

constexpr int kMaxFE = 8;        // FE dimensions supported per regression
constexpr int kMaxCols = 63;     // p = 1 + k (+ instruments) <= 63 -> Gram width <= 64
constexpr int kBlock = 256;      // threads per workgroup for streaming kernels (4 waves)

void set_error(const std::string& msg);

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
  int32_t G = 0;             // n_levels
  int32_t* code = nullptr;   // [ld] int32 codes (context-owned)
  int32_t* cnt_pre = nullptr;  // [G] pre-filter counts
  int32_t* cnt = nullptr;      // [G] kept counts
  double* W = nullptr;         // [G] sum of weights (or counts) over kept rows
  double* S = nullptr;         // [G*p] sum_{i in g} w_i x_i  (constant)
  double* T = nullptr;         // [G*p] cross term of the current projection
  double* alpha = nullptr;     // [G*p] accumulated group effect (the "subtracted mean")
  double* R = nullptr;         // [G] check sums (unweighted y residual)
  int32_t dims = 0, card = 0;
};

// Kernel-argument bundle (passed by value) describing all FEs.
struct FeArgs {
  int F;
  int p;
  const int32_t* code[kMaxFE];
  const double* alpha[kMaxFE];
};

// kernel ids for per-launch event timing (lfe_profile / lfe_kernel_stats)
enum KernelId {
  K_COUNT_PRE = 0, K_KEEP, K_GROUP_SUMS, K_CROSS_SUMS, K_FINALIZE, K_CHECK_SUMS, K_CHECK_MAX, K_GRAM_DESIGN,
  K_GRAM_RESID, K_GRAM_TABLE, K_REDUCE, K_CLUSTER_SCATTER, K_COUNT_NONZERO, K_SYNTH, K_NUM_KERNELS
};
extern const char* const kKernelNames[K_NUM_KERNELS];

struct Prof {
  bool on = false;
  std::vector<hipEvent_t> pool;        // free events
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;
  double total_ms[K_NUM_KERNELS] = {0};
  int64_t count[K_NUM_KERNELS] = {0};
  hipEvent_t open_ev = nullptr;
  int open_id = -1;
};

struct Timings {
  double prep = 0, demean = 0, gram = 0, resid = 0, cluster = 0, last = 0;
};

}  // namespace lfe

struct lfe_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // data (row shard)
  int64_t n = 0;      // rows in this shard
  int64_t ld = 0;     // leading dimension of column storage (n rounded up)
  int p = 0;          // columns: y + x (+ instruments)
  int F = 0;
  double* X = nullptr;       // [p][ld]
  double* w = nullptr;       // [ld] or nullptr
  uint8_t* keep = nullptr;   // [ld]
  std::vector<lfe::FeState> fe;
  // clusters
  std::vector<int32_t*> cl;
  std::vector<int32_t> cl_levels;
  double* scores = nullptr;  // [k][ld] x~ r (w)
  double* dbeta = nullptr;   // [64] beta_full staging
  bool scores_valid = false;
  // scratch
  double* scratch = nullptr;     // device partials
  size_t scratch_elems = 0;
  double* dred = nullptr;        // device reduced output (small)
  size_t dred_elems = 0;
  double* hpinned = nullptr;     // pinned host staging
  size_t hpinned_elems = 0;
  int32_t* iscratch = nullptr;   // device int scratch
  size_t iscratch_elems = 0;
  // state
  int64_t n_kept = 0;
  bool loaded = false, prepared = false, demeaned = false;
  // distributed
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
  lfe::Timings tm;
  lfe::Prof prof;
};

namespace lfe {

// --- launchers (lfe_kernels.hip) ---
int launch_count_pre(lfe_ctx* c);
int launch_keep(lfe_ctx* c);
int launch_group_sums(lfe_ctx* c);
int launch_cross_sums(lfe_ctx* c, int f);
int launch_finalize(lfe_ctx* c, int f);
int launch_check(lfe_ctx* c, double* host_max);
int launch_gram(lfe_ctx* c, double* host_gram);
int launch_resid(lfe_ctx* c, const double* beta_full, double* stats, double* hc1, int keep_scores);
int launch_cluster(lfe_ctx* c, double* meats, int64_t* G_out);
int launch_count_dims(lfe_ctx* c, int32_t* dims, int32_t* card);
int launch_validate_codes(const int32_t* code, int64_t n, int32_t G, int32_t* flag, hipStream_t s);
int launch_copy_demeaned(lfe_ctx* c, double* dev_out);

// --- synthetic panel (lfe_synth.hip) ---
int launch_synth(lfe_ctx* c, int k, const int32_t* levels, const double* beta, uint64_t seed,
                 int64_t row_offset);

// --- helpers (lfe_capi.hip) ---
int ensure_scratch(lfe_ctx* c, size_t elems);
int ensure_dred(lfe_ctx* c, size_t elems);
int ensure_pinned(lfe_ctx* c, size_t elems);
int ensure_iscratch(lfe_ctx* c, size_t elems);
int allreduce_sum_f64(lfe_ctx* c, double* dev, size_t count);
int allreduce_sum_i32(lfe_ctx* c, int32_t* dev, size_t count);
int allreduce_max_f64(lfe_ctx* c, double* dev, size_t count);
FeArgs fe_args(const lfe_ctx* c);
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

}  // namespace lfe
