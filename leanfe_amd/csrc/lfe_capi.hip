// leanfe HIP engine — C ABI (include/leanfe_hip.h), context management, RCCL.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <map>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "lfe_internal.h"

namespace lfe {

static std::mutex g_knob_mu;
static std::map<std::string, std::string> g_knobs;

const char* knob(const char* name) {
  thread_local std::string ring[8];
  thread_local int slot = 0;
  std::lock_guard<std::mutex> lk(g_knob_mu);
  if (g_knobs.empty()) return nullptr;
  const auto it = g_knobs.find(name);
  if (it == g_knobs.end()) return nullptr;
  std::string& out = ring[slot];
  slot = (slot + 1) & 7;
  out = it->second;
  return out.c_str();
}

static std::mutex g_lds_mu;
static std::map<std::pair<int, const void*>, int> g_lds_set;

hipError_t set_max_lds(const void* fn, int bytes) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lk(g_lds_mu);
  int& have = g_lds_set[{dev, fn}];
  if (bytes <= have) return hipSuccess;
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) have = bytes;
  return e;
}

static thread_local std::string g_err;

void set_error(const std::string& msg) { g_err = msg; }

static int fail(int code, const std::string& msg) {
  set_error(msg);
  return code;
}

#define LFE_NCCL(expr)                                                                                  \
  do {                                                                                                  \
    ncclResult_t _r = (expr);                                                                           \
    if (_r != ncclSuccess) return fail(LFE_ERCCL, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
  } while (0)

// Device allocations are plain hipMalloc: the stream-ordered allocator is not
// used anywhere in the engine (a hipMallocAsync'd table raced with later
// hipMalloc/hipFree in an early version).
template <typename T>
static int dalloc(T** p, size_t elems) {
  *p = nullptr;
  if (elems == 0) elems = 1;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(p), sizeof(T) * elems);
  if (e != hipSuccess) {
    set_error(std::string("hipMalloc(") + std::to_string(sizeof(T) * elems) + " B): " + hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? LFE_ENOMEM : LFE_EHIP;
  }
  return LFE_OK;
}

template <typename T>
static void dfree(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

template <typename T>
static int ensure(T*& p, size_t& have, size_t want) {
  if (have >= want) return LFE_OK;
  dfree(p);
  have = 0;
  LFE_TRY(dalloc(&p, want));
  have = want;
  return LFE_OK;
}

int ensure_scratch(lfe_ctx* c, size_t elems) { return ensure(c->scratch, c->scratch_elems, elems); }
int ensure_dred(lfe_ctx* c, size_t elems) { return ensure(c->dred, c->dred_elems, elems); }
int ensure_iscratch(lfe_ctx* c, size_t elems) { return ensure(c->iscratch, c->iscratch_elems, elems); }
int d2h_sync(lfe_ctx* c, void* dst, const void* src_dev, size_t bytes) {
  if (bytes == 0) return LFE_OK;
  if (bytes > kPinD2H) {
    LFE_HIP(hipMemcpyAsync(dst, src_dev, bytes, hipMemcpyDeviceToHost, c->stream));
    LFE_HIP(hipStreamSynchronize(c->stream));
    return LFE_OK;
  }
  LFE_HIP(hipMemcpyAsync(c->hpin, src_dev, bytes, hipMemcpyDeviceToHost, c->stream));
  LFE_HIP(hipStreamSynchronize(c->stream));
  memcpy(dst, c->hpin, bytes);
  return LFE_OK;
}

int d2h_async(lfe_ctx* c, const void* src_dev, size_t bytes) {
  if (bytes > kPinD2H) return fail(LFE_EINVAL, "d2h_async: transfer too large");
  LFE_HIP(hipMemcpyAsync(c->hpin, src_dev, bytes, hipMemcpyDeviceToHost, c->stream));
  LFE_HIP(hipEventRecord(c->aux_ev, c->stream));
  return LFE_OK;
}

// the n tagged words a kernel published under sequence number seq; a bounded spin per word (the
// stream is synchronized after ~2 s without it, which then must be there)
static int host_msg_words(lfe_ctx* c, unsigned long long seq, unsigned int* out, int n) {
  const unsigned long long tag = seq & 0xffffffffull;
  if ((size_t)n > kHostMsgBytes / 8) return fail(LFE_EINVAL, "host message too long");
  for (int i = 0; i < n; ++i) {
    unsigned long long w = __atomic_load_n(&c->hmsg[i], __ATOMIC_ACQUIRE);
    for (long spin = 0; (w >> 32) != tag; ++spin) {
      if (spin == (1l << 26)) {
        LFE_HIP(hipStreamSynchronize(c->stream));
        w = __atomic_load_n(&c->hmsg[i], __ATOMIC_ACQUIRE);
        if ((w >> 32) != tag) return fail(LFE_EHIP, "device message lost");
        break;
      }
      w = __atomic_load_n(&c->hmsg[i], __ATOMIC_ACQUIRE);
    }
    out[i] = (unsigned int)w;
  }
  return LFE_OK;
}

int host_msg_wait(lfe_ctx* c, unsigned long long seq, double* vals, int nvals) {
  std::vector<unsigned int> w((size_t)2 * nvals);
  LFE_TRY(host_msg_words(c, seq, w.data(), 2 * nvals));
  for (int i = 0; i < nvals; ++i) {
    const unsigned long long b = (unsigned long long)w[2 * i] | ((unsigned long long)w[2 * i + 1] << 32);
    memcpy(&vals[i], &b, sizeof(double));
  }
  return LFE_OK;
}

// off by default: with a kernel storing into the mapped host words the 8-rank shard solved in
// 1.10 vs 0.91 ms and config 3 in 4.78-4.83 vs 4.62-4.63 ms, config 1 0.385-0.391 vs 0.390-0.403
// (same box, profiles/r06/ab_hostmsg.txt); LFE_HOST_MSG=1 turns them on
bool host_msg_on(const lfe_ctx* c) {
  if (c->world != 1) return false;
  const char* e = knob("LFE_HOST_MSG");
  return e && e[0] == '1';
}

int host_msg_wait_i32(lfe_ctx* c, unsigned long long seq, int32_t* vals, int n) {
  std::vector<unsigned int> w((size_t)n);
  LFE_TRY(host_msg_words(c, seq, w.data(), n));
  for (int i = 0; i < n; ++i) vals[i] = (int32_t)w[i];
  return LFE_OK;
}

int d2h_wait(lfe_ctx* c, void* dst, size_t bytes) {
  LFE_HIP(hipEventSynchronize(c->aux_ev));  // work enqueued after the copy keeps running
  memcpy(dst, c->hpin, bytes);
  return LFE_OK;
}

// small uploads from mapped, coherent staging by a copy kernel: a kernel-to-kernel dependency in the
// stream (~2 us) where an SDMA copy cost ~15-20 us of idle GPU on each side
__global__ void k_copy_up(const char* __restrict__ src, char* __restrict__ dst, int64_t bytes) {
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
  if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) | (uintptr_t)bytes) & 3) == 0) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
    for (int64_t i = t0; i < bytes / 4; i += st) d[i] = s[i];
  } else {
    for (int64_t i = t0; i < bytes; i += st) dst[i] = src[i];
  }
}

int h2d_small(lfe_ctx* c, void* dst_dev, const void* src, size_t bytes) {
  if (bytes == 0) return LFE_OK;
  if (bytes > kPinSmall - kPinD2H || knob("LFE_H2D_SDMA")) {  // (the knob: the SDMA form, for A/B)
    LFE_HIP(hipMemcpyAsync(dst_dev, src, bytes, hipMemcpyHostToDevice, c->stream));
    LFE_HIP(hipStreamSynchronize(c->stream));
    return LFE_OK;
  }
  LFE_HIP(hipEventSynchronize(c->hpin_ev));  // the previous upload from the staging has been read
  memcpy(c->hup, src, bytes);
  hipLaunchKernelGGL(k_copy_up, dim3((unsigned)std::min<size_t>(16, (bytes / 4 + 255) / 256 + 1)), dim3(256), 0,
                     c->stream, c->hup_dev, static_cast<char*>(dst_dev), (int64_t)bytes);
  LFE_HIP(hipGetLastError());
  LFE_HIP(hipEventRecord(c->hpin_ev, c->stream));
  return LFE_OK;
}

int ensure_pinned_items(lfe_ctx* c, size_t bytes) {
  if (c->hpin_items_cap >= bytes) return LFE_OK;
  if (c->hpin_items) {
    LFE_HIP(hipStreamSynchronize(c->stream));  // no upload from the old buffer in flight
    (void)hipHostFree(c->hpin_items);
    c->hpin_items = nullptr;
    c->hpin_items_dev = nullptr;
    c->hpin_items_cap = 0;
  }
  const size_t cap = (std::max<size_t>(bytes, 1 << 20) + 15) & ~(size_t)15;  // whole 16-byte words
  // mapped and coherent: a kernel copies it to the device (k_copy_staged), a dependency of ~2 us in
  // the stream where an SDMA upload behind the partition scatter cost ~15-20 us of idle GPU
  LFE_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->hpin_items), cap, hipHostMallocMapped | hipHostMallocCoherent));
  LFE_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->hpin_items_dev), c->hpin_items, 0));
  c->hpin_items_cap = cap;
  return LFE_OK;
}

// the occupancy query costs several µs of host time on the launch path: cached per (device, kernel,
// block size, dynamic LDS)
int resident_blocks(lfe_ctx* c, const void* fn, int threads, size_t dyn_lds) {
  static std::mutex mu;
  static std::map<std::tuple<int, const void*, int, size_t>, int> cache;
  const auto key = std::make_tuple(c->device, fn, threads, dyn_lds);
  {
    std::lock_guard<std::mutex> lk(mu);
    const auto it = cache.find(key);
    if (it != cache.end()) return it->second * c->n_cu;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, dyn_lds) != hipSuccess || per_cu < 1)
    per_cu = 1;
  std::lock_guard<std::mutex> lk(mu);
  cache[key] = per_cu;
  return per_cu * c->n_cu;
}

int ensure_items(lfe_ctx* c, size_t n_items) { return ensure(c->items_d, c->items_cap, 4 * n_items); }
int ensure_i32(lfe_ctx*, int32_t*& p, size_t& cap, size_t elems) { return ensure(p, cap, elems); }
int ensure_f64(lfe_ctx*, double*& p, size_t& cap, size_t elems) { return ensure(p, cap, elems); }
int ensure_u16(lfe_ctx*, uint16_t*& p, size_t& cap, size_t elems) { return ensure(p, cap, elems); }
int ensure_u64(lfe_ctx*, uint64_t*& p, size_t& cap, size_t elems) { return ensure(p, cap, elems); }
int ensure_i8(lfe_ctx*, int8_t*& p, size_t& cap, size_t elems) { return ensure(p, cap, elems); }
int ensure_u8(lfe_ctx*, uint8_t*& p, size_t& cap, size_t elems) { return ensure(p, cap, elems); }

__global__ void k_zero_ranges(ZeroArgs a) {
  zero_ranges_part(a, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x);
}

int build_zero_args(const std::vector<std::pair<void*, size_t>>& ranges, ZeroArgs* a, int64_t* words) {
  *a = ZeroArgs{};
  int64_t off = 0;
  for (const auto& r : ranges) {
    if (!r.first || r.second == 0) continue;
    if (a->n == 32) return fail(LFE_EINVAL, "zero_ranges: at most 32 ranges");
    a->p[a->n] = static_cast<uint32_t*>(r.first);
    off += (int64_t)(r.second / 4);
    a->end[a->n++] = off;
  }
  if (words) *words = off;
  return LFE_OK;
}

int zero_ranges(lfe_ctx* c, const std::vector<std::pair<void*, size_t>>& ranges) {
  ZeroArgs a{};
  int64_t off = 0;
  LFE_TRY(build_zero_args(ranges, &a, &off));
  if (a.n == 0) return LFE_OK;
  hipLaunchKernelGGL(k_zero_ranges, dim3(grid_for((off + 3) / 4, 256, 1024)), dim3(256), 0, c->stream, a);
  LFE_HIP(hipGetLastError());
  return LFE_OK;
}

int ensure_pcounts(lfe_ctx* c, size_t elems, size_t sums) {
  LFE_TRY(ensure(c->pcounts, c->pcounts_elems, elems));
  return ensure(c->psums, c->psums_elems, sums);
}

int ensure_cluster_ws(lfe_ctx* c, size_t table_elems, size_t flag_elems) {
  LFE_TRY(ensure(c->clS, c->clS_elems, table_elems));
  return ensure(c->clP, c->clP_elems, flag_elems);
}

}  // namespace lfe

// In-process emulated communicator (tests only): `world` contexts of one process,
// each driven by its own host thread, exchange all-reduce buffers through host
// memory behind a barrier.  It exercises the engine's multi-rank code paths (the
// same collective calls, in the same order, as with RCCL) on a single GPU.
struct lfe_emu {
  int world = 0;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  int64_t generation = 0;
  std::vector<std::vector<char>> slots;
  std::vector<char> result;
  // all-to-all: every rank publishes its device send buffer and per-peer blocks
  std::vector<const char*> a2a_send;
  std::vector<std::vector<size_t>> a2a_off, a2a_bytes;
  bool aborted = false;  // lfe_emu_abort: a member failed; every waiting and later barrier fails
  bool barrier() {
    std::unique_lock<std::mutex> lk(m);
    if (aborted) return false;
    const int64_t gen = generation;
    if (++arrived == world) {
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return generation != gen || aborted; });
    }
    return !aborted;
  }
};

namespace lfe {

enum EmuOp { EMU_SUM_F64, EMU_SUM_I32, EMU_MAX_F64, EMU_MAX_U64, EMU_MAX_I32 };

static int emu_allreduce(lfe_ctx* c, void* dev, size_t count, EmuOp op) {
  lfe_emu* e = c->emu;
  const size_t esz = (op == EMU_SUM_I32 || op == EMU_MAX_I32) ? sizeof(int32_t) : sizeof(double);
  const size_t bytes = count * esz;
  LFE_HIP(hipStreamSynchronize(c->stream));
  e->slots[c->rank].resize(bytes);
  // copies on this context's stream, waited for: a plain hipMemcpy runs on the null stream, which
  // a non-blocking context stream does not order against (a later kernel could read the result
  // before a host-to-device copy lands)
  LFE_HIP(hipMemcpyAsync(e->slots[c->rank].data(), dev, bytes, hipMemcpyDeviceToHost, c->stream));
  LFE_HIP(hipStreamSynchronize(c->stream));
  if (!e->barrier()) return fail(LFE_ESTATE, "group aborted by a member");
  if (c->rank == 0) {  // fixed rank order: deterministic
    e->result = e->slots[0];
    for (int r = 1; r < e->world; ++r)
      for (size_t i = 0; i < count; ++i) {
        if (op == EMU_SUM_I32) {
          reinterpret_cast<int32_t*>(e->result.data())[i] += reinterpret_cast<const int32_t*>(e->slots[r].data())[i];
        } else if (op == EMU_MAX_I32) {
          int32_t& acc = reinterpret_cast<int32_t*>(e->result.data())[i];
          acc = std::max(acc, reinterpret_cast<const int32_t*>(e->slots[r].data())[i]);
        } else if (op == EMU_MAX_U64) {
          uint64_t& acc = reinterpret_cast<uint64_t*>(e->result.data())[i];
          acc = std::max(acc, reinterpret_cast<const uint64_t*>(e->slots[r].data())[i]);
        } else {
          double& acc = reinterpret_cast<double*>(e->result.data())[i];
          const double v = reinterpret_cast<const double*>(e->slots[r].data())[i];
          acc = op == EMU_SUM_F64 ? acc + v : std::max(acc, v);
        }
      }
  }
  if (!e->barrier()) return fail(LFE_ESTATE, "group aborted by a member");
  LFE_HIP(hipMemcpyAsync(dev, e->result.data(), bytes, hipMemcpyHostToDevice, c->stream));
  LFE_HIP(hipStreamSynchronize(c->stream));
  if (!e->barrier()) return fail(LFE_ESTATE, "group aborted by a member");  // copies done before reuse
  return LFE_OK;
}

// peer r receives this rank's block [send_off[r], + send_bytes[r]); this rank
// receives peer r's block for it at recv_off[r] (recv_bytes[r] bytes)
int alltoallv_bytes(lfe_ctx* c, const char* send, const size_t* send_off, const size_t* send_bytes, char* recv,
                    const size_t* recv_off, const size_t* recv_bytes) {
  const int W = c->world;
  if (W <= 1) {
    if (send_bytes[0])
      LFE_HIP(hipMemcpyAsync(recv + recv_off[0], send + send_off[0], send_bytes[0], hipMemcpyDeviceToDevice,
                             c->stream));
    return LFE_OK;
  }
  if (c->emu) {  // all contexts of an emulated group share one device: peer copies are D2D
    lfe_emu* e = c->emu;
    LFE_HIP(hipStreamSynchronize(c->stream));
    {
      std::lock_guard<std::mutex> lk(e->m);
      e->a2a_send.resize(W);
      e->a2a_off.resize(W);
      e->a2a_bytes.resize(W);
      e->a2a_send[c->rank] = send;
      e->a2a_off[c->rank].assign(send_off, send_off + W);
      e->a2a_bytes[c->rank].assign(send_bytes, send_bytes + W);
    }
    if (!e->barrier()) return fail(LFE_ESTATE, "group aborted by a member");
    for (int q = 0; q < W; ++q) {
      const size_t b = e->a2a_bytes[q][c->rank];
      if (b != recv_bytes[q]) return fail(LFE_EINVAL, "alltoallv: peer block size mismatch");
      if (b) LFE_HIP(hipMemcpyAsync(recv + recv_off[q], e->a2a_send[q] + e->a2a_off[q][c->rank], b,
                                    hipMemcpyDeviceToDevice, c->stream));
    }
    // the copies complete before the peers go on (a plain device-to-device hipMemcpy may return
    // before its copy is done, and runs on the null stream, unordered with this context's stream)
    LFE_HIP(hipStreamSynchronize(c->stream));
    if (!e->barrier()) return fail(LFE_ESTATE, "group aborted by a member");  // peers read this buffer
    return LFE_OK;
  }
  LFE_NCCL(ncclGroupStart());
  for (int r = 0; r < W; ++r) {
    if (r == c->rank) continue;
    if (send_bytes[r]) LFE_NCCL(ncclSend(send + send_off[r], send_bytes[r], ncclUint8, r, c->comm, c->stream));
    if (recv_bytes[r]) LFE_NCCL(ncclRecv(recv + recv_off[r], recv_bytes[r], ncclUint8, r, c->comm, c->stream));
  }
  LFE_NCCL(ncclGroupEnd());
  if (send_bytes[c->rank])
    LFE_HIP(hipMemcpyAsync(recv + recv_off[c->rank], send + send_off[c->rank], send_bytes[c->rank],
                           hipMemcpyDeviceToDevice, c->stream));
  return LFE_OK;
}

int allreduce_sum_f64(lfe_ctx* c, double* dev, size_t count) {
  if (c->world <= 1 || count == 0) return LFE_OK;
  if (c->emu) return emu_allreduce(c, dev, count, EMU_SUM_F64);
  LFE_NCCL(ncclAllReduce(dev, dev, count, ncclFloat64, ncclSum, c->comm, c->stream));
  return LFE_OK;
}

// several independent f64 sums in one RCCL group (one launch, one latency)
int allreduce_sum_f64_many(lfe_ctx* c, const std::vector<std::pair<double*, size_t>>& bufs) {
  if (c->world <= 1) return LFE_OK;
  if (c->emu) {
    for (auto& b : bufs)
      if (b.second) LFE_TRY(emu_allreduce(c, b.first, b.second, EMU_SUM_F64));
    return LFE_OK;
  }
  LFE_NCCL(ncclGroupStart());
  for (auto& b : bufs)
    if (b.second) LFE_NCCL(ncclAllReduce(b.first, b.first, b.second, ncclFloat64, ncclSum, c->comm, c->stream));
  LFE_NCCL(ncclGroupEnd());
  return LFE_OK;
}

int allreduce_sum_i32(lfe_ctx* c, int32_t* dev, size_t count) {
  if (c->world <= 1 || count == 0) return LFE_OK;
  if (c->emu) return emu_allreduce(c, dev, count, EMU_SUM_I32);
  LFE_NCCL(ncclAllReduce(dev, dev, count, ncclInt32, ncclSum, c->comm, c->stream));
  return LFE_OK;
}

int allreduce_max_i32(lfe_ctx* c, int32_t* dev, size_t count) {
  if (c->world <= 1 || count == 0) return LFE_OK;
  if (c->emu) return emu_allreduce(c, dev, count, EMU_MAX_I32);
  LFE_NCCL(ncclAllReduce(dev, dev, count, ncclInt32, ncclMax, c->comm, c->stream));
  return LFE_OK;
}

// max of u64 (the bits of non-negative doubles, NaN above every number: a max that keeps NaN)
int allreduce_max_u64(lfe_ctx* c, uint64_t* dev, size_t count) {
  if (c->world <= 1 || count == 0) return LFE_OK;
  if (c->emu) return emu_allreduce(c, dev, count, EMU_MAX_U64);
  LFE_NCCL(ncclAllReduce(dev, dev, count, ncclUint64, ncclMax, c->comm, c->stream));
  return LFE_OK;
}

int allreduce_max_f64(lfe_ctx* c, double* dev, size_t count) {
  if (c->world <= 1 || count == 0) return LFE_OK;
  if (c->emu) return emu_allreduce(c, dev, count, EMU_MAX_F64);
  LFE_NCCL(ncclAllReduce(dev, dev, count, ncclFloat64, ncclMax, c->comm, c->stream));
  return LFE_OK;
}

// ---------------------------------------------------------------------------
// per-kernel event profiling
// ---------------------------------------------------------------------------

const char* const kKernelNames[K_NUM_KERNELS] = {
    "part_hist", "scan", "part_scatter", "count", "mark", "group_sums", "cross", "check", "finalize",
    "check_max", "gram_design", "gram_resid", "gram_table", "reduce_partials", "cluster_scatter", "misc", "synth",
    "tp", "tq", "seg_build", "cluster_sort", "gram_tables", "layout_hist", "layout_base", "layout_scatter",
    "tq_reduce", "fix_sums", "cluster_fix"};

static hipEvent_t prof_event(lfe_ctx* c) {
  if (!c->prof.pool.empty()) {
    hipEvent_t e = c->prof.pool.back();
    c->prof.pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

void prof_begin(lfe_ctx* c, int kid) {
  if (!c->prof.on) return;
  hipEvent_t e = prof_event(c);
  if (!e) return;
  (void)hipEventRecord(e, c->stream);
  c->prof.open_ev = e;
  c->prof.open_id = kid;
}

void prof_end(lfe_ctx* c) {
  if (!c->prof.on || !c->prof.open_ev) return;
  hipEvent_t e = prof_event(c);
  if (!e) return;
  (void)hipEventRecord(e, c->stream);
  c->prof.pending.push_back({c->prof.open_id, {c->prof.open_ev, e}});
  c->prof.open_ev = nullptr;
  if (c->prof.pending.size() > 4096) (void)prof_fold(c);
}

int prof_fold(lfe_ctx* c) {
  if (c->prof.pending.empty()) return LFE_OK;
  LFE_HIP(hipStreamSynchronize(c->stream));
  for (auto& r : c->prof.pending) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, r.second.first, r.second.second) == hipSuccess) {
      c->prof.total_ms[r.first] += ms;
      c->prof.count[r.first] += 1;
    }
    c->prof.pool.push_back(r.second.first);
    c->prof.pool.push_back(r.second.second);
  }
  c->prof.pending.clear();
  return LFE_OK;
}

// ---------------------------------------------------------------------------
// data buffers
// ---------------------------------------------------------------------------

static void free_data(lfe_ctx* c) {
  dfree(c->X);
  dfree(c->w);
  dfree(c->Xp);
  dfree(c->wp);
  dfree(c->codes_p);
  dfree(c->origp);
  dfree(c->scores);
  for (auto& fe : c->fe) {
    dfree(fe.code);
    dfree(fe.cnt_pre);
    dfree(fe.drops);
    dfree(fe.cnt);
    dfree(fe.W);
    dfree(fe.S);
    dfree(fe.Sy);
    dfree(fe.T);
    dfree(fe.alpha);
    dfree(fe.R);
    dfree(fe.hi);
    dfree(fe.alpha_g);
    fe.alpha_g_cap = 0;
    dfree(fe.alpha_y);
    fe.alpha_y_cap = 0;
    dfree(fe.seg_off);
    dfree(fe.seg_cur);
    dfree(fe.oc);
    dfree(fe.perm);
    dfree(fe.ws);
    dfree(fe.ufirst);
  }
  c->fe.clear();
  for (auto& p : c->cl) dfree(p);
  c->cl.clear();
  c->cl_levels.clear();
  c->cl_fe.clear();
  c->clfused = false;
  dfree(c->clf_S);
  dfree(c->clf_hi);
  dfree(c->clf_cnt);
  dfree(c->clf_fq);
  c->clf_S_cap = c->clf_hi_cap = c->clf_cnt_cap = c->clf_fq_cap = 0;
  free_cluster_ws(c);
  dfree(c->rec_sy);
  dfree(c->rec_syy);
  dfree(c->rec_lay);
  c->rec_sy_cap = c->rec_syy_cap = c->rec_lay_cap = 0;
  dfree(c->raw_part);
  dfree(c->qpart);
  dfree(c->colsum_part);
  c->colsum_part_cap = 0;
  dfree(c->dn_na);
  dfree(c->dn_nb);
  c->dn_na_cap = c->dn_nb_cap = 0;
  dfree(c->dn8_a);
  dfree(c->dn8_b);
  dfree(c->dn8_fa);
  dfree(c->dn8_fb);
  dfree(c->dn8_dq);
  dfree(c->dn8_eq);
  dfree(c->rflag);
  c->rflag_cap = 0;
  c->dn8_a_cap = c->dn8_b_cap = c->dn8_fa_cap = c->dn8_fb_cap = c->dn8_dq_cap = c->dn8_eq_cap = 0;
  c->dn8 = false;
  free_dense3(c);
  dfree(c->raw_slots);
  c->raw_slots_cap = 0;
  dfree(c->amax);
  dfree(c->astat);
  c->astat_cap = 0;
  dfree(c->xq);
  dfree(c->chain);
  c->amax_cap = c->xq_cap = c->chain_cap = 0;
  dfree(c->sw.x);
  dfree(c->sw.s64);
  dfree(c->sw.sdbl);
  dfree(c->sw.tile);
  dfree(c->sw.red);
  dfree(c->sw.toff);
  free_stream_clusters(c);
  c->sw = lfe_ctx::StreamWS();
  dfree(c->dspec);
  c->dspec_elems = 0;
  c->gram_spec = false;
  c->qpart_cap = 0;
  dfree(c->raw_tile);
  dfree(c->raw_shift);
  c->raw_part_cap = c->raw_tile_cap = c->raw_shift_cap = 0;
  c->raw_ready = c->tq_final = false;
  c->records = false;
  c->rows_in = 0;
  c->loading = false;
  c->L = Layout();
  dfree(c->tq_runs);
  c->tq_runs_cap = 0;
  dfree(c->colstat);
  dfree(c->fixq);
  dfree(c->colq);
  c->colstat_cap = c->fixq_cap = c->colq_cap = 0;
  c->fixq_ready = c->any_ready = false;
  c->q_first = nullptr;
  c->colstat_chunks = 0;
  c->owner_fe = -1;
  c->owner_on = false;
  c->loaded = c->prepared = c->demeaned = c->scores_valid = c->seg_ready = false;
  c->n = c->ld = 0;
  c->p = c->F = 0;
}

// allocate all per-shard buffers for (n, p, F, levels)
static int alloc_data(lfe_ctx* c, int64_t n, int p, int F, const int32_t* n_levels, bool weighted,
                      bool codes_only = false) {
  free_data(c);
  if (p < 1 || p > kMaxCols) return fail(LFE_EINVAL, "p must be in [1, 63] (y plus up to 62 regressors)");
  if (F < 0 || F > kMaxFE) return fail(LFE_EINVAL, "number of fixed effects must be in [0, 8]");
  if (n < 0 || n >= (int64_t)INT32_MAX) return fail(LFE_EINVAL, "rows per shard must be in [0, 2^31 - 1)");
  for (int f = 0; f < F; ++f)
    if (n_levels[f] < 1) return fail(LFE_EINVAL, "n_levels must be >= 1");
  c->n = n;
  c->ld = std::max<int64_t>((n + 63) / 64 * 64, 64);
  c->hi_dirty = false;
  c->p = p;
  c->F = F;
  c->sw.on = codes_only;  // streamed X: no resident columns, no permuted copy
  if (!codes_only) LFE_TRY(dalloc(&c->X, (size_t)p * c->ld));
  if (weighted) LFE_TRY(dalloc(&c->w, (size_t)c->ld));
  if (F > 0) LFE_TRY(dalloc(&c->codes_p, (size_t)F * c->ld));
  c->fe.resize(F);
  bool need_perm = false;
  for (int f = 0; f < F; ++f) {
    auto& fe = c->fe[f];
    fe.G = n_levels[f];
    need_perm = need_perm || fe.G > 256;
    LFE_TRY(dalloc(&fe.code, (size_t)c->ld));
    LFE_TRY(dalloc(&fe.cnt_pre, (size_t)fe.G));
    LFE_TRY(dalloc(&fe.drops, (size_t)fe.G));
    LFE_TRY(dalloc(&fe.cnt, (size_t)fe.G));
    LFE_TRY(dalloc(&fe.S, (size_t)fe.G * p));
    LFE_TRY(dalloc(&fe.T, (size_t)fe.G * p));
    LFE_TRY(dalloc(&fe.alpha, (size_t)fe.G * p));
    LFE_TRY(dalloc(&fe.R, (size_t)fe.G));
    LFE_TRY(dalloc(&fe.hi, (size_t)fe.G * p));
    LFE_HIP(hipMemsetAsync(fe.hi, 0, sizeof(double) * (size_t)fe.G * p, c->stream));
    if (weighted) {
      LFE_TRY(dalloc(&fe.W, (size_t)fe.G));
      LFE_TRY(dalloc(&fe.Sy, (size_t)fe.G));
    }
  }
  if (need_perm) {  // bucketed layout storage (rows regrouped by the primary FE)
    if (!codes_only) LFE_TRY(dalloc(&c->Xp, (size_t)p * c->ld));
    if (weighted) LFE_TRY(dalloc(&c->wp, (size_t)c->ld));
    LFE_TRY(dalloc(&c->origp, (size_t)c->ld));
  }
  return LFE_OK;
}

int alloc_shard(lfe_ctx* c, int64_t n, int p, int F, const int32_t* n_levels, bool weighted) {
  return alloc_data(c, n, p, F, n_levels, weighted);
}

enum { PH_PREP, PH_DEMEAN, PH_GRAM, PH_RESID, PH_CLUSTER };

struct PhaseTimer {
  lfe_ctx* c;
  int ph;
  // (opt-in, lfe_phase_timing: an event record costs several µs of host time, on the launch path)
  PhaseTimer(lfe_ctx* c_, int ph_) : c(c_), ph(ph_) {
    if (c->tm.on) (void)hipEventRecord(c->tm.ev[ph][0], c->stream);
  }
  ~PhaseTimer() {
    if (!c->tm.on) return;
    (void)hipEventRecord(c->tm.ev[ph][1], c->stream);
    c->tm.pending |= 1u << ph;
    c->tm.last_phase = ph;
  }
};

#define LFE_CTX(c)                                     \
  do {                                                 \
    if (!(c)) return fail(LFE_EINVAL, "null context"); \
    LFE_HIP(hipSetDevice((c)->device));                \
  } while (0)

// entry points that read resident data columns
#define LFE_NO_STREAM(c)                                                                                 \
  do {                                                                                                   \
    if ((c)->sw.on)                                                                                      \
      return fail(LFE_ESTATE, "not available with streamed X (lfe_load_codes): use the lfe_stream passes"); \
  } while (0)

// Runs right after the copies of lfe_load / lfe_load_finish: every return path has waited for
// the stream, so no copy from the caller's host arrays is still in flight when it returns.
static int validate_all(lfe_ctx* c) {
  int32_t bad = 0;
  auto run = [&]() -> int {
    LFE_TRY(ensure_iscratch(c, 16));
    LFE_HIP(hipMemsetAsync(c->iscratch, 0, sizeof(int32_t), c->stream));
    for (int f = 0; f < c->F && c->n > 0; ++f)
      LFE_TRY(launch_validate_codes(c->fe[f].code, c->n, c->fe[f].G, c->iscratch, c->stream));
    LFE_HIP(hipMemcpyAsync(&bad, c->iscratch, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    return LFE_OK;
  };
  const int rc = run();
  const hipError_t e = hipStreamSynchronize(c->stream);
  if (rc != LFE_OK) return rc;
  if (e != hipSuccess) return fail(LFE_EHIP, std::string("hipStreamSynchronize: ") + hipGetErrorString(e));
  if (bad) {
    free_data(c);
    return fail(LFE_EINVAL, "FE codes must be dense int32 in [0, n_levels)");
  }
  return LFE_OK;
}

}  // namespace lfe

using namespace lfe;

extern "C" {

const char* lfe_last_error(void) { return g_err.c_str(); }

const char* lfe_version(void) { return "leanfe_amd-hip 0.2.0 (gfx950)"; }

int lfe_ctx_create(lfe_ctx** out, int device) {
  if (!out) return fail(LFE_EINVAL, "out is null");
  *out = nullptr;
  int ndev = 0;
  LFE_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(LFE_EINVAL, "device ordinal out of range");
  LFE_HIP(hipSetDevice(device));
  lfe_ctx* c = new lfe_ctx();
  c->device = device;
  (void)hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device);
  if (c->n_cu <= 0) c->n_cu = 256;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->hpin_ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->aux_ev, hipEventDisableTiming) != hipSuccess ||
      hipStreamCreateWithFlags(&c->up_stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->up_ev0, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->up_ev1, hipEventDisableTiming) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&c->hpin), kPinSmall, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&c->hmsg), kHostMsgBytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&c->dmsg), c->hmsg, 0) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&c->hup), kPinSmall - kPinD2H, hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&c->hup_dev), c->hup, 0) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&c->dbeta), 64 * sizeof(double)) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&c->gsync), kGsyncSlots * sizeof(unsigned int)) != hipSuccess ||
      hipMemsetAsync(c->gsync, 0, kGsyncSlots * sizeof(unsigned int), c->stream) != hipSuccess) {
    delete c;
    return fail(LFE_EHIP, "stream/event/buffer creation failed");
  }
  memset(c->hmsg, 0, kHostMsgBytes);
  for (auto& pair : c->tm.ev)
    for (auto& e : pair)
      if (hipEventCreate(&e) != hipSuccess) {
        e = nullptr;
        lfe_ctx_destroy(c);
        return fail(LFE_EHIP, "event creation failed");
      }
  *out = c;
  return LFE_OK;
}

void lfe_ctx_destroy(lfe_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  free_data(c);
  dfree(c->scratch);
  dfree(c->dred);
  if (c->gsync) (void)hipFree(c->gsync);
  if (c->scan_status) (void)hipFree(c->scan_status);
  c->scan_status = nullptr;
  c->gsync = nullptr;
  dfree(c->iscratch);
  dfree(c->pcounts);
  dfree(c->psums);
  dfree(c->items_d);
  c->bitems_d = c->xitems_d = nullptr;  // views into items_d
  dfree(c->seg_off);
  dfree(c->seg_q);
  dfree(c->seg_aux);
  dfree(c->seg_units);
  dfree(c->run_off);
  dfree(c->run_h);
  dfree(c->alpha_spare);
  dfree(c->dbeta);
  if (c->hpin) (void)hipHostFree(c->hpin);
  if (c->hmsg) (void)hipHostFree(c->hmsg);
  if (c->hup) (void)hipHostFree(c->hup);
  if (c->hpin_items) (void)hipHostFree(c->hpin_items);
  if (c->hpin_ev) (void)hipEventDestroy(c->hpin_ev);
  for (auto& e : c->load_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->aux_ev) (void)hipEventDestroy(c->aux_ev);
  if (c->up_ev0) (void)hipEventDestroy(c->up_ev0);
  if (c->up_ev1) (void)hipEventDestroy(c->up_ev1);
  if (c->up_stream) (void)hipStreamDestroy(c->up_stream);
  dfree(c->clS);
  dfree(c->clP);
  if (c->comm) ncclCommDestroy(c->comm);
  for (auto& r : c->prof.pending) {
    (void)hipEventDestroy(r.second.first);
    (void)hipEventDestroy(r.second.second);
  }
  for (auto e : c->prof.pool) (void)hipEventDestroy(e);
  for (auto& pair : c->tm.ev)
    for (auto e : pair)
      if (e) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int lfe_comm_unique_id(void* out128) {
  if (!out128) return fail(LFE_EINVAL, "out is null");
  static_assert(sizeof(ncclUniqueId) == 128, "unique id size");
  ncclUniqueId id;
  LFE_NCCL(ncclGetUniqueId(&id));
  std::memcpy(out128, &id, sizeof(id));
  return LFE_OK;
}

int lfe_emu_create(int world, lfe_emu** out) {
  if (!out || world < 1) return fail(LFE_EINVAL, "bad arguments");
  lfe_emu* e = new lfe_emu();
  e->world = world;
  e->slots.resize(world);
  *out = e;
  return LFE_OK;
}

void lfe_emu_destroy(lfe_emu* e) { delete e; }

void lfe_emu_abort(lfe_emu* e) {
  if (!e) return;
  std::lock_guard<std::mutex> lk(e->m);
  e->aborted = true;
  e->cv.notify_all();
}

int lfe_ctx_set_emu(lfe_ctx* c, lfe_emu* e, int rank) {
  LFE_CTX(c);
  if (!e || rank < 0 || rank >= e->world) return fail(LFE_EINVAL, "bad emulated group / rank");
  if (c->comm) {
    ncclCommDestroy(c->comm);
    c->comm = nullptr;
  }
  c->emu = e;
  c->rank = rank;
  c->world = e->world;
  return LFE_OK;
}

int lfe_ctx_set_comm(lfe_ctx* c, const void* unique_id128, int rank, int world) {
  LFE_CTX(c);
  if (world < 1 || rank < 0 || rank >= world) return fail(LFE_EINVAL, "bad rank/world");
  if (c->comm) {
    ncclCommDestroy(c->comm);
    c->comm = nullptr;
  }
  c->emu = nullptr;
  c->rank = rank;
  c->world = world;
  if (world == 1) return LFE_OK;
  if (!unique_id128) return fail(LFE_EINVAL, "unique id is null");
  ncclUniqueId id;
  std::memcpy(&id, unique_id128, sizeof(id));
  LFE_NCCL(ncclCommInitRank(&c->comm, world, id, rank));
  return LFE_OK;
}

int lfe_load(lfe_ctx* c, int64_t n, int p, const double* const* cols, int F, const int32_t* const* fe_codes,
             const int32_t* n_levels, const double* weights, int where) {
  LFE_CTX(c);
  if (where != LFE_HOST && where != LFE_DEVICE) return fail(LFE_EINVAL, "where must be LFE_HOST or LFE_DEVICE");
  if (n > 0 && (!cols || (F > 0 && (!fe_codes || !n_levels)))) return fail(LFE_EINVAL, "null input pointer");
  if (F > 0 && !n_levels) return fail(LFE_EINVAL, "n_levels is null");
  LFE_TRY(alloc_data(c, n, p, F, n_levels, weights != nullptr));
  const hipMemcpyKind kind = where == LFE_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
  hipError_t e = hipSuccess;
  for (int j = 0; j < p && n > 0 && e == hipSuccess; ++j)
    e = hipMemcpyAsync(c->X + (size_t)j * c->ld, cols[j], sizeof(double) * n, kind, c->stream);
  if (weights && n > 0 && e == hipSuccess) e = hipMemcpyAsync(c->w, weights, sizeof(double) * n, kind, c->stream);
  for (int f = 0; f < F && n > 0 && e == hipSuccess; ++f)
    e = hipMemcpyAsync(c->fe[f].code, fe_codes[f], sizeof(int32_t) * n, kind, c->stream);
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(c->stream);  // no copy from the caller's arrays outlives the call
    return fail(LFE_EHIP, std::string("hipMemcpyAsync: ") + hipGetErrorString(e));
  }
  LFE_TRY(validate_all(c));
  c->loaded = true;
  return LFE_OK;
}

// ---------------------------------------------------------------------------
// out-of-core X: codes resident, the data columns streamed in row chunks
// ---------------------------------------------------------------------------
int lfe_load_codes(lfe_ctx* c, int64_t n, int p, int F, const int32_t* const* fe_codes, const int32_t* n_levels,
                   const double* weights, int kind) {
  LFE_CTX(c);
  if (F < 1 || F > kMaxFE) return fail(LFE_EINVAL, "streamed X (lfe_load_codes) needs 1 to 8 fixed effects");
  if (!n_levels || (n > 0 && !fe_codes)) return fail(LFE_EINVAL, "null input pointer");
  if (kind != LFE_HOST && kind != LFE_DEVICE) return fail(LFE_EINVAL, "kind must be LFE_HOST or LFE_DEVICE");
  if (weights && p + 2 > kColStatHead)  // the weighted sums add w and the raw y as two more columns
    return fail(LFE_EINVAL, "weighted streamed X supports p <= 62 columns");
  LFE_TRY(alloc_data(c, n, p, F, n_levels, weights != nullptr, true));
  const hipMemcpyKind mk = kind == LFE_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
  hipError_t e = hipSuccess;
  if (weights && n > 0) e = hipMemcpyAsync(c->w, weights, sizeof(double) * n, mk, c->stream);
  for (int f = 0; f < F && n > 0 && e == hipSuccess; ++f)
    e = hipMemcpyAsync(c->fe[f].code, fe_codes[f], sizeof(int32_t) * n, mk, c->stream);
  if (e != hipSuccess) {
    (void)hipStreamSynchronize(c->stream);
    return fail(LFE_EHIP, std::string("hipMemcpyAsync: ") + hipGetErrorString(e));
  }
  LFE_TRY(validate_all(c));
  c->loaded = true;
  return LFE_OK;
}

int lfe_stream_begin(lfe_ctx* c, int pass, const double* beta_full) {
  LFE_CTX(c);
  auto& w = c->sw;
  if (!w.on) return fail(LFE_ESTATE, "lfe_stream_*: the context holds resident columns (use lfe_load_codes)");
  if (pass < 1 || pass > 4)
    return fail(LFE_EINVAL, "pass must be 1 (group sums), 2 (residual), 3 (design Gram) or 4 (IV residual)");
  if (!c->prepared) return fail(LFE_ESTATE, "lfe_drop_singletons first");
  if (pass > 1 && !c->demeaned) return fail(LFE_ESTATE, "lfe_demean first");
  if (pass == 2 || pass == 4) {
    if (!beta_full) return fail(LFE_EINVAL, "beta_full is null");
    LFE_TRY(h2d_small(c, c->dbeta, beta_full, sizeof(double) * c->p));
    w.icpt = pass == 4 ? 1 : 0;
    if (!w.cid.empty()) {  // clustered SEs: zeroed per-cluster score sums of width ks
      w.ks = c->p - 1 + w.icpt;
      for (size_t s = 0; s < w.cid.size(); ++s) {
        const size_t m = (size_t)std::max(w.G[s], 1) * std::max(w.ks, 1);
        LFE_TRY(ensure_f64(c, w.S[s], w.S_cap[s], m));
        LFE_HIP(hipMemsetAsync(w.S[s], 0, sizeof(double) * m, c->stream));
      }
    }
  }
  if (pass > 1) {
    w.ts = stream_tile_stride(c->p);
    const size_t tl = stream_tile_len(c->p);
    LFE_TRY(ensure_f64(c, w.tile, w.tile_cap, tl));
    LFE_HIP(hipMemsetAsync(w.tile, 0, sizeof(double) * tl, c->stream));
  }
  if (pass == 1) c->sums_ready = c->raw_ready = false;
  w.pass = pass;
  w.rows_done = 0;
  return LFE_OK;
}

// one streamed chunk (columns in c->sw.x, leading dimension cld) through the current pass
static int stream_chunk(lfe_ctx* c, int64_t cld, int64_t row0, int64_t rows) {
  auto& w = c->sw;
  PhaseTimer t(c, w.pass == 1 ? PH_PREP : w.pass == 3 ? PH_GRAM : PH_RESID);
  if (w.pass == 1) {
    LFE_TRY(stream_sums_chunk(c, w.x, cld, row0, rows, w.rows_done == 0));
  } else if (w.pass == 5) {
    LFE_TRY(stream_materialize_chunk(c, w.x, cld, row0, rows));
  } else {
    const bool resid = w.pass == 2 || w.pass == 4;
    const bool scored = resid && !w.cid.empty();
    if (scored) LFE_TRY(ensure_f64(c, w.sc, w.sc_cap, (size_t)std::max<int64_t>(rows, 1) * std::max(w.ks, 1)));
    LFE_TRY(stream_rows_chunk(c, resid ? 0 : 1, resid ? w.icpt : 0, w.x, cld, row0, rows, scored ? w.sc : nullptr));
    if (scored) LFE_TRY(stream_clusters_chunk(c, row0, rows));
  }
  w.rows_done += rows;
  return LFE_OK;
}

int lfe_stream_rows(lfe_ctx* c, int64_t row0, int64_t rows, const double* const* cols, int kind) {
  LFE_CTX(c);
  auto& w = c->sw;
  if (!w.on || w.pass == 0) return fail(LFE_ESTATE, "lfe_stream_begin first");
  if (row0 < 0 || rows < 0 || row0 + rows > c->n) return fail(LFE_EINVAL, "rows outside the loaded codes");
  if (rows == 0) return LFE_OK;
  if (!cols) return fail(LFE_EINVAL, "cols is null");
  if (kind != LFE_HOST && kind != LFE_DEVICE) return fail(LFE_EINVAL, "kind must be LFE_HOST or LFE_DEVICE");
  const int64_t cld = (rows + 63) / 64 * 64;
  LFE_TRY(ensure_f64(c, w.x, w.x_cap, (size_t)c->p * cld));
  const hipMemcpyKind mk = kind == LFE_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
  for (int j = 0; j < c->p; ++j) {
    if (!cols[j]) return fail(LFE_EINVAL, "null column pointer");
    LFE_HIP(hipMemcpyAsync(w.x + (size_t)j * cld, cols[j], sizeof(double) * rows, mk, c->stream));
  }
  LFE_TRY(stream_chunk(c, cld, row0, rows));
  if (kind == LFE_HOST) LFE_HIP(hipStreamSynchronize(c->stream));  // the caller may reuse its buffers
  return LFE_OK;
}

// benchmark / test helpers: the synthetic panel of lfe_synth_load with the codes resident and
// the columns generated chunk by chunk on the device (no host copy of data larger than HBM)
int lfe_synth_load_codes_at(lfe_ctx* c, int64_t n, int64_t row0, int k, int n_fe, const int32_t* n_levels,
                            uint64_t seed) {
  LFE_CTX(c);
  if (n_fe < 1 || n_fe > kMaxFE || !n_levels) return fail(LFE_EINVAL, "streamed X needs 1 to 8 fixed effects");
  if (k < 1 || k + 1 > kMaxCols) return fail(LFE_EINVAL, "k out of range");
  if (row0 < 0) return fail(LFE_EINVAL, "row0 must be >= 0");
  LFE_TRY(alloc_data(c, n, k + 1, n_fe, n_levels, false, true));
  LFE_TRY(synth_codes(c, n_levels, seed, row0));
  c->synth_row0 = row0;
  c->loaded = true;
  return LFE_OK;
}

int lfe_synth_load_codes(lfe_ctx* c, int64_t n, int k, int n_fe, const int32_t* n_levels, uint64_t seed) {
  return lfe_synth_load_codes_at(c, n, 0, k, n_fe, n_levels, seed);
}

int lfe_stream_synth_rows(lfe_ctx* c, int64_t row0, int64_t rows, int k, const int32_t* n_levels,
                          const double* beta, uint64_t seed) {
  LFE_CTX(c);
  auto& w = c->sw;
  if (!w.on || w.pass == 0) return fail(LFE_ESTATE, "lfe_stream_begin first");
  if (k + 1 != c->p || !n_levels || !beta) return fail(LFE_EINVAL, "k must match the loaded p - 1");
  if (row0 < 0 || rows < 0 || row0 + rows > c->n) return fail(LFE_EINVAL, "rows outside the loaded codes");
  if (rows == 0) return LFE_OK;
  const int64_t cld = (rows + 63) / 64 * 64;
  LFE_TRY(ensure_f64(c, w.x, w.x_cap, (size_t)c->p * cld));
  LFE_TRY(synth_chunk(c, k, n_levels, beta, seed, c->synth_row0 + row0, rows, w.x, cld));
  LFE_TRY(stream_chunk(c, cld, row0, rows));
  return LFE_OK;
}

int lfe_stream_synth_cols(lfe_ctx* c, int64_t row0, int64_t rows, int K, int c_lo, const int32_t* n_levels,
                          const double* beta, uint64_t seed) {
  LFE_CTX(c);
  auto& w = c->sw;
  if (!w.on || w.pass == 0) return fail(LFE_ESTATE, "lfe_stream_begin first");
  if (K < 0 || c_lo < 0 || c_lo + c->p > K + 1 || !n_levels || (K > 0 && !beta))
    return fail(LFE_EINVAL, "the column block must lie in [0, K]");
  if (row0 < 0 || rows < 0 || row0 + rows > c->n) return fail(LFE_EINVAL, "rows outside the loaded codes");
  if (rows == 0) return LFE_OK;
  const int64_t cld = (rows + 63) / 64 * 64;
  LFE_TRY(ensure_f64(c, w.x, w.x_cap, (size_t)c->p * cld));
  LFE_TRY(synth_cols_chunk(c, K, c_lo, n_levels, beta, seed, c->synth_row0 + row0, rows, w.x, cld));
  LFE_TRY(stream_chunk(c, cld, row0, rows));
  return LFE_OK;
}

int lfe_stream_end(lfe_ctx* c, double* out) {
  LFE_CTX(c);
  auto& w = c->sw;
  if (!w.on || w.pass == 0) return fail(LFE_ESTATE, "lfe_stream_begin first");
  const int pass = w.pass;
  w.pass = 0;
  const int64_t want = pass == 5 && w.mrows >= 0 ? w.mrows : c->n;  // (a row range of lfe_stream_materialize_rows)
  if (w.rows_done != want) return fail(LFE_EINVAL, "the streamed chunks did not cover the loaded rows");
  const int p = c->p, k = p - 1;
  if (pass == 5) {  // lfe_stream_materialize: nothing to reduce; D is written when this returns (other
    w.mD = nullptr;  // contexts' streams read it next: the column blocks of a wide fit)
    w.mbase = 0;
    w.mrows = -1;
    LFE_HIP(hipStreamSynchronize(c->stream));
    return LFE_OK;
  }
  if (pass == 1) {
    LFE_TRY(ensure_f64(c, c->raw_tile, c->raw_tile_cap, 256));
    if (c->n > 0) LFE_HIP(hipMemcpyAsync(c->raw_tile, w.tile, sizeof(double) * 256, hipMemcpyDeviceToDevice, c->stream));
    // the raw Gram tile stands for the Gram from the group tables only in the unweighted two-FE case
    // of one process (ranks' tiles have their own shifts: a sharded fit streams the design Gram) and
    // when it fits one 16 x 16 MFMA tile (intercept in slot 15)
    c->raw_ready = c->F == 2 && !c->w && c->world == 1 && p <= 15;
    if (c->world > 1) {  // every rank streamed its own rows: the group sums over all ranks
      std::vector<std::pair<double*, size_t>> bufs;
      for (auto& fe : c->fe) {
        bufs.push_back({fe.S, (size_t)fe.G * p});
        if (c->w) {
          bufs.push_back({fe.W, (size_t)fe.G});
          bufs.push_back({fe.Sy, (size_t)fe.G});
        }
      }
      LFE_TRY(allreduce_sum_f64_many(c, bufs));
    }
    c->sums_ready = true;
    c->sums_zeroed = false;
    LFE_TRY(stream_weight_stats(c));
    c->exact_sums = true;
    return LFE_OK;
  }
  if (!out) return fail(LFE_EINVAL, "out is null");
  // tile (i, j) at i * ts + j, the statistics after ts * ts (ts = 16: the p <= 11 passes)
  const size_t ts = (size_t)w.ts, tl = ts * ts + 4;
  LFE_TRY(allreduce_sum_f64(c, w.tile, tl));  // sharded: every rank's rows
  std::vector<double> h(tl);
  LFE_TRY(d2h_sync(c, h.data(), w.tile, sizeof(double) * tl));
  if (pass == 2 || pass == 4) {  // stats[4] (sum r^2 w, sum r^2, sum y~, sum y~^2), then the HC1 meat
    const int km = k + (pass == 4 ? 1 : 0);  // pass 4: over u = [1, x~, z~]
    for (int e = 0; e < 4; ++e) out[e] = h[ts * ts + e];
    for (int i = 0; i < km; ++i)
      for (int j = 0; j < km; ++j) out[4 + i * km + j] = h[(size_t)(1 + i) * ts + (1 + j)];
  } else {  // the (p + 1) x (p + 1) Gram of [1, y~, x~]
    for (int i = 0; i <= p; ++i)
      for (int j = 0; j <= p; ++j) out[i * (p + 1) + j] = h[(size_t)i * ts + j];
  }
  return LFE_OK;
}

int lfe_stream_clusters(lfe_ctx* c, int n_subsets, const int32_t* masks) {
  LFE_CTX(c);
  if (!c->sw.on) return fail(LFE_ESTATE, "lfe_stream_clusters: the context holds resident columns");
  if (!c->prepared) return fail(LFE_ESTATE, "lfe_drop_singletons first");
  if (n_subsets < 1 || !masks) return fail(LFE_EINVAL, "bad subsets");
  if (c->sw.pass != 0) return fail(LFE_ESTATE, "lfe_stream_clusters: a streamed pass is open (lfe_stream_end first)");
  return stream_clusters_prep(c, n_subsets, masks);
}

int lfe_stream_cluster_meats(lfe_ctx* c, double* meats_out, int64_t* G_out) {
  LFE_CTX(c);
  if (c->sw.cid.empty() || c->sw.ks == 0)
    return fail(LFE_ESTATE, "lfe_stream_clusters and a residual pass (2 or 4) first");
  if (!meats_out || !G_out) return fail(LFE_EINVAL, "null output pointer");
  PhaseTimer t(c, PH_CLUSTER);
  return stream_cluster_meats(c, meats_out, G_out);
}

int lfe_load_begin(lfe_ctx* c, int64_t n, int p, int F, const int32_t* n_levels, int weighted) {
  LFE_CTX(c);
  if (F > 0 && !n_levels) return fail(LFE_EINVAL, "n_levels is null");
  LFE_TRY(alloc_data(c, n, p, F, n_levels, weighted != 0));
  for (auto& e : c->load_ev)
    if (!e) LFE_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  c->load_calls = 0;
  c->load_rows_done = 0;
  c->loading = true;
  return LFE_OK;
}

int lfe_load_rows(lfe_ctx* c, int64_t row0, int64_t rows, const double* const* cols, const int32_t* const* fe_codes,
                  const double* weights) {
  LFE_CTX(c);
  if (!c->loading) return fail(LFE_ESTATE, "lfe_load_begin first");
  if (row0 < 0 || rows < 0 || row0 + rows > c->n) return fail(LFE_EINVAL, "rows outside the shard");
  if (rows > 0 && (!cols || (c->F > 0 && !fe_codes) || ((c->w != nullptr) != (weights != nullptr))))
    return fail(LFE_EINVAL, "null input pointer (or weights given to an unweighted shard)");
  // the copies issued two calls ago have finished: the caller may release those host arrays
  const int slot = (int)(c->load_calls & 1);
  LFE_HIP(hipEventSynchronize(c->load_ev[slot]));
  for (int j = 0; j < c->p && rows > 0; ++j)
    LFE_HIP(hipMemcpyAsync(c->X + (size_t)j * c->ld + row0, cols[j], sizeof(double) * rows, hipMemcpyHostToDevice,
                           c->stream));
  if (c->w && rows > 0)
    LFE_HIP(hipMemcpyAsync(c->w + row0, weights, sizeof(double) * rows, hipMemcpyHostToDevice, c->stream));
  for (int f = 0; f < c->F && rows > 0; ++f)
    LFE_HIP(hipMemcpyAsync(c->fe[f].code + row0, fe_codes[f], sizeof(int32_t) * rows, hipMemcpyHostToDevice,
                           c->stream));
  LFE_HIP(hipEventRecord(c->load_ev[slot], c->stream));
  ++c->load_calls;
  c->load_rows_done += rows;
  return LFE_OK;
}

int lfe_load_finish(lfe_ctx* c) {
  LFE_CTX(c);
  if (!c->loading) return fail(LFE_ESTATE, "lfe_load_begin first");
  c->loading = false;
  if (c->load_rows_done != c->n) return fail(LFE_EINVAL, "lfe_load_rows did not cover the shard's rows");
  LFE_HIP(hipStreamSynchronize(c->stream));
  LFE_TRY(validate_all(c));
  c->loaded = true;
  return LFE_OK;
}

int lfe_synth_load(lfe_ctx* c, int64_t n, int k, int n_fe, const int32_t* n_levels, const double* beta,
                   uint64_t seed, int64_t row_offset) {
  LFE_CTX(c);
  if (k < 0 || k + 1 > kMaxCols) return fail(LFE_EINVAL, "k out of range");
  if (n_fe > 0 && !n_levels) return fail(LFE_EINVAL, "n_levels is null");
  LFE_TRY(alloc_data(c, n, k + 1, n_fe, n_levels, false));
  LFE_TRY(launch_synth(c, k, n_levels, beta, seed, row_offset));
  LFE_HIP(hipStreamSynchronize(c->stream));
  c->loaded = true;
  return LFE_OK;
}

int lfe_ctx_set_owner(lfe_ctx* c, int fe, int32_t lo, int32_t hi) {
  LFE_CTX(c);
  if (fe < 0) {
    c->owner_fe = -1;
    c->prepared = false;
    return LFE_OK;
  }
  if (!c->loaded) return fail(LFE_ESTATE, "load the shard before lfe_ctx_set_owner");
  if (fe >= c->F || lo < 0 || hi < lo || hi > c->fe[fe].G) return fail(LFE_EINVAL, "bad owner FE / level range");
  if (c->n == 0) return fail(LFE_EINVAL, "owner sharding needs at least one row on every rank");
  LFE_TRY(ensure_iscratch(c, 16));
  LFE_HIP(hipMemsetAsync(c->iscratch, 0, sizeof(int32_t), c->stream));
  LFE_TRY(launch_validate_range(c->fe[fe].code, c->n, lo, hi, c->iscratch, c->stream));
  int32_t bad = 0;
  LFE_HIP(hipMemcpyAsync(&bad, c->iscratch, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  LFE_HIP(hipStreamSynchronize(c->stream));
  if (bad) return fail(LFE_EINVAL, "owner sharding: a row's owner-FE code lies outside [lo, hi)");
  c->owner_fe = fe;
  c->owner_lo = lo;
  c->owner_hi = hi;
  c->prepared = false;  // the layout decides again which tables stay rank-local
  return LFE_OK;
}

int lfe_reshard_owner(lfe_ctx* c, int fe, int32_t* lo_out, int32_t* hi_out) {
  LFE_CTX(c);
  if (!c->loaded) return fail(LFE_ESTATE, "load the shard before lfe_reshard_owner");
  if (!lo_out || !hi_out) return fail(LFE_EINVAL, "null output pointer");
  int32_t lo = 0, hi = 0;
  LFE_TRY(reshard_owner(c, fe, &lo, &hi));
  *lo_out = lo;
  *hi_out = hi;
  return lfe_ctx_set_owner(c, fe, lo, hi);
}

int lfe_synth_load_owned(lfe_ctx* c, int64_t n_total, int k, int n_fe, const int32_t* n_levels, const double* beta,
                         uint64_t seed, int owner_fe, int32_t lo, int32_t hi) {
  LFE_CTX(c);
  if (k < 0 || k + 1 > kMaxCols) return fail(LFE_EINVAL, "k out of range");
  if (n_fe < 1 || !n_levels || owner_fe < 0 || owner_fe >= n_fe) return fail(LFE_EINVAL, "bad owner FE");
  if (n_total < 0 || lo < 0 || hi < lo || hi > n_levels[owner_fe]) return fail(LFE_EINVAL, "bad owner level range");
  std::vector<int64_t> base;
  int64_t n_local = 0;
  LFE_TRY(synth_count_owned(c, n_total, owner_fe, n_levels[owner_fe], lo, hi, seed, base, &n_local));
  LFE_TRY(alloc_data(c, n_local, k + 1, n_fe, n_levels, false));
  LFE_TRY(launch_synth_owned(c, n_total, k, n_levels, beta, seed, owner_fe, lo, hi, base));
  c->loaded = true;
  return lfe_ctx_set_owner(c, owner_fe, lo, hi);
}

int lfe_load_clusters(lfe_ctx* c, int m, const int32_t* const* cl_codes, const int32_t* cl_levels, int where) {
  LFE_CTX(c);
  if (!c->loaded) return fail(LFE_ESTATE, "lfe_load must precede lfe_load_clusters");
  if (m < 0 || (m > 0 && (!cl_codes || !cl_levels))) return fail(LFE_EINVAL, "bad cluster arrays");
  if (m > 30) return fail(LFE_EINVAL, "at most 30 cluster columns");
  for (int j = 0; j < m; ++j)  // every argument checked before the first copy is issued
    if (cl_levels[j] < 1) return fail(LFE_EINVAL, "cluster n_levels must be >= 1");
  for (auto& p : c->cl) dfree(p);
  free_cluster_ws(c);
  // the residual pass's one-way sums (and the meat cached from them) belong to the old columns;
  // c->clfused stays, so a subset of the new columns reruns that pass writing score rows
  c->clfused_done = false;
  c->clfused_j = -1;
  c->cl.assign(m, nullptr);
  c->cl_levels.assign(cl_levels, cl_levels + m);
  const hipMemcpyKind kind = where == LFE_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
  // [0]: a code out of range; [kIsClFlags + j kMaxFE + f]: column j differs from FE f (of the same
  // level count) - past the drop's counts, which a later demean still reads
  LFE_TRY(ensure_iscratch(c, kIscratchAll));
  LFE_HIP(hipMemsetAsync(c->iscratch, 0, sizeof(int32_t), c->stream));
  LFE_HIP(hipMemsetAsync(c->iscratch + kIsClFlags, 0, sizeof(int32_t) * (size_t)m * kMaxFE, c->stream));
  int rc = LFE_OK;
  for (int j = 0; j < m && rc == LFE_OK; ++j) {
    rc = dalloc(&c->cl[j], (size_t)c->ld);
    if (rc == LFE_OK && c->n > 0) {
      const hipError_t e = hipMemcpyAsync(c->cl[j], cl_codes[j], sizeof(int32_t) * c->n, kind, c->stream);
      rc = e == hipSuccess ? launch_validate_codes(c->cl[j], c->n, cl_levels[j], c->iscratch, c->stream)
                           : fail(LFE_EHIP, std::string("hipMemcpyAsync: ") + hipGetErrorString(e));
    }
  }
  if (rc != LFE_OK) {
    // copies from the caller's (pageable) arrays may still be in flight: finish them before
    // the caller can release those arrays
    (void)hipStreamSynchronize(c->stream);
    return rc;
  }
  // a cluster column that repeats an FE column (reg_test.py:55, 61 cluster on the FEs): its sums
  // can use the layout's bucket slices when that FE is the primary one (lfe_cluster.hip)
  for (int j = 0; j < m && c->n > 0; ++j)
    for (int f = 0; f < c->F; ++f)
      if (c->fe[f].G == cl_levels[j]) LFE_TRY(launch_codes_differ(c, c->cl[j], c->fe[f].code, c->n,
                                                                  c->iscratch + kIsClFlags + j * kMaxFE + f));
  // several ranks: a bad code anywhere fails every rank, and a column repeats an FE only if it does
  // on every rank's rows (the owner-local cluster forms are then a decision all ranks take alike)
  LFE_TRY(allreduce_sum_i32(c, c->iscratch, 1));
  LFE_TRY(allreduce_sum_i32(c, c->iscratch + kIsClFlags, (size_t)m * kMaxFE));
  std::vector<int32_t> h(kIsClFlags + (size_t)m * kMaxFE, 0);
  LFE_HIP(hipMemcpyAsync(h.data(), c->iscratch, sizeof(int32_t) * h.size(), hipMemcpyDeviceToHost, c->stream));
  LFE_HIP(hipStreamSynchronize(c->stream));
  if (h[0]) return fail(LFE_EINVAL, "cluster codes must be dense int32 in [0, n_levels)");
  c->cl_fe.assign(m, -1);
  for (int j = 0; j < m && c->n > 0; ++j)
    for (int f = 0; f < c->F && c->cl_fe[j] < 0; ++f)
      if (c->fe[f].G == cl_levels[j] && h[kIsClFlags + j * kMaxFE + f] == 0) c->cl_fe[j] = f;
  return LFE_OK;
}

int lfe_drop_singletons(lfe_ctx* c, int64_t* n_kept, int32_t* fe_dims_out, int32_t* fe_card_out) {
  LFE_CTX(c);
  if (!c->loaded) return fail(LFE_ESTATE, "lfe_load first");
  {
    PhaseTimer t(c, PH_PREP);
    LFE_TRY(prepare_layout(c));
  }
  for (int f = 0; f < c->F; ++f) {
    if (fe_dims_out) fe_dims_out[f] = c->fe[f].dims;
    if (fe_card_out) fe_card_out[f] = c->fe[f].card;
  }
  if (n_kept) *n_kept = c->n_kept;
  c->prepared = true;
  c->demeaned = false;
  c->scores_valid = false;
  c->clfused = false;
  return LFE_OK;
}

int lfe_demean(lfe_ctx* c, const int* fe_order, double tol, int max_iter, int check_from, int* iterations_out,
               double* last_check_out) {
  LFE_CTX(c);
  if (!c->prepared) return fail(LFE_ESTATE, "lfe_drop_singletons first");
  std::vector<int> order(c->F);
  for (int f = 0; f < c->F; ++f) order[f] = fe_order ? fe_order[f] : f;
  {
    std::vector<int> chk(order);
    std::sort(chk.begin(), chk.end());
    for (int f = 0; f < c->F; ++f)
      if (chk[f] != f) return fail(LFE_EINVAL, "fe_order must be a permutation of 0..F-1");
  }
  if (check_from > 0 && max_iter < 1) return fail(LFE_EINVAL, "max_iter must be >= 1");
  int iterations = 0;
  double last = -1.0;
  c->dense_coarse = c->dense_off = false;
  {
    PhaseTimer t(c, PH_DEMEAN);
    // a second attempt only when the i8 digits' dynamic-range guard fired on the first (every rank
    // sees the same flag): the same solve without the dense cross terms (lfe_dense.hip)
    for (int attempt = 0; attempt < 2; ++attempt) {
      c->dense_cells = 0;  // demean_fast sets it when the dense cross terms run
      c->d3.on = false;    // ... demean_dense3 this
      c->tq_final = false;
      c->gram_spec = false;
      const bool fast = c->F > 0 && check_from > 0 && fast_path_ok(c, order);
      if (!fast)  // the two-FE sweeps write every alpha entry before reading any
        for (auto& fe : c->fe) LFE_HIP(hipMemsetAsync(fe.alpha, 0, sizeof(double) * (size_t)fe.G * c->p, c->stream));
      if (c->F > 0) {
        if (!c->sums_ready) {
          if (c->sw.on) return fail(LFE_ESTATE, "streamed X: stream the group-sums pass (lfe_stream pass 1) first");
          LFE_TRY(sweep_group_sums(c));
        }
        if (fast) {
          // two FEs, unweighted: segment layout + one fused codes-only kernel per sweep
          LFE_TRY(demean_fast(c, tol, max_iter, check_from, &iterations, &last));
        } else if (dense3_ok(c, order, check_from)) {
          // three or more FEs, unweighted, small pair tables: every cross term on the matrix cores
          LFE_TRY(demean_dense3(c, order, tol, max_iter, check_from, &iterations, &last));
        } else {
          LFE_TRY(demean_generic(c, order, tol, max_iter, check_from, &iterations, &last));
        }
      }
      c->q_first = nullptr;  // (demean_fast consumed it, or another path ran)
      if (!c->dense_coarse || c->dense_off) break;
      c->dense_off = true;
    }
    c->dense_off = false;
  }
  if (iterations_out) *iterations_out = iterations;
  if (last_check_out) *last_check_out = last;
  c->demeaned = true;
  return LFE_OK;
}

int lfe_gram(lfe_ctx* c, double* gram_out) {
  LFE_CTX(c);
  if (!c->demeaned) return fail(LFE_ESTATE, "lfe_demean first");
  if (!gram_out) return fail(LFE_EINVAL, "gram_out is null");
  PhaseTimer t(c, PH_GRAM);
  const int rc = launch_gram(c, gram_out);
  if (rc == 2)
    return fail(LFE_ENEEDPASS, "streamed X: the Gram from the group tables is unavailable or failed its "
                               "cancellation guard; stream the design-Gram pass (lfe_stream_begin pass 3)");
  return rc;
}

int lfe_resid(lfe_ctx* c, const double* beta_full, double* stats_out, double* hc1_meat, int keep_scores) {
  LFE_CTX(c);
  LFE_NO_STREAM(c);
  if (!c->demeaned) return fail(LFE_ESTATE, "lfe_demean first");
  if (!beta_full || !stats_out) return fail(LFE_EINVAL, "null pointer");
  if (keep_scores && !c->scores && c->p > 1) LFE_TRY(dalloc(&c->scores, (size_t)c->p * c->ld));
  PhaseTimer t(c, PH_RESID);
  return launch_resid(c, beta_full, stats_out, hc1_meat, keep_scores, 0);
}

int lfe_resid_iv(lfe_ctx* c, const double* coef, double* stats_out, double* meat_out, int keep_scores) {
  LFE_CTX(c);
  LFE_NO_STREAM(c);
  if (!c->demeaned) return fail(LFE_ESTATE, "lfe_demean first");
  if (!coef || !stats_out) return fail(LFE_EINVAL, "null pointer");
  if (keep_scores && !c->scores) LFE_TRY(dalloc(&c->scores, (size_t)c->p * c->ld));
  PhaseTimer t(c, PH_RESID);
  return launch_resid(c, coef, stats_out, meat_out, keep_scores, 1);
}

int lfe_gram_resid(lfe_ctx* c, double* gram_out, double* beta_full_out, double* stats_out, double* hc1_meat,
                   int keep_scores) {
  LFE_CTX(c);
  LFE_NO_STREAM(c);
  if (!c->demeaned) return fail(LFE_ESTATE, "lfe_demean first");
  if (!gram_out || !beta_full_out || !stats_out) return fail(LFE_EINVAL, "null pointer");
  if (keep_scores && !c->scores && c->p > 1) LFE_TRY(dalloc(&c->scores, (size_t)c->p * c->ld));
  PhaseTimer t(c, PH_RESID);
  return launch_gram_resid(c, gram_out, beta_full_out, stats_out, hc1_meat, keep_scores);
}

int lfe_cluster_meat(lfe_ctx* c, double* meats_out, int64_t* G_out) {
  LFE_CTX(c);
  if (!c->scores_valid) return fail(LFE_ESTATE, "lfe_resid(keep_scores=1) first");
  if (!meats_out || !G_out) return fail(LFE_EINVAL, "null pointer");
  PhaseTimer t(c, PH_CLUSTER);
  std::vector<int32_t> masks(c->cl.size());
  for (size_t j = 0; j < masks.size(); ++j) masks[j] = 1 << j;
  return launch_cluster_subsets(c, (int)masks.size(), masks.data(), meats_out, G_out);
}

int lfe_cluster_meat_subsets(lfe_ctx* c, int n_subsets, const int32_t* masks, double* meats_out, int64_t* G_out) {
  LFE_CTX(c);
  if (!c->scores_valid) return fail(LFE_ESTATE, "lfe_resid(keep_scores=1) first");
  if (n_subsets < 0 || (n_subsets > 0 && (!masks || !meats_out || !G_out))) return fail(LFE_EINVAL, "null pointer");
  PhaseTimer t(c, PH_CLUSTER);
  return launch_cluster_subsets(c, n_subsets, masks, meats_out, G_out);
}

int lfe_copy_demeaned(lfe_ctx* c, double* const* cols_out, int64_t* n_out) {
  LFE_CTX(c);
  LFE_NO_STREAM(c);
  if (!c->demeaned) return fail(LFE_ESTATE, "lfe_demean first");
  double* d = nullptr;
  LFE_TRY(dalloc(&d, (size_t)c->p * std::max<int64_t>(c->n, 1)));
  int rc = launch_copy_demeaned(c, d);
  if (rc == LFE_OK) {
    for (int j = 0; j < c->p && c->n > 0; ++j)
      if (hipMemcpyAsync(cols_out[j], d + (size_t)j * c->n, sizeof(double) * c->n, hipMemcpyDeviceToHost,
                         c->stream) != hipSuccess)
        rc = fail(LFE_EHIP, "copy out failed");
    (void)hipStreamSynchronize(c->stream);
  }
  dfree(d);
  if (n_out) *n_out = c->n;
  return rc;
}

int lfe_copy_inputs(lfe_ctx* c, double* const* cols_out, int32_t* const* codes_out) {
  LFE_CTX(c);
  LFE_NO_STREAM(c);
  if (!c->loaded) return fail(LFE_ESTATE, "nothing loaded");
  for (int j = 0; j < c->p && c->n > 0 && cols_out; ++j)
    LFE_HIP(hipMemcpyAsync(cols_out[j], c->X + (size_t)j * c->ld, sizeof(double) * c->n, hipMemcpyDeviceToHost,
                           c->stream));
  for (int f = 0; f < c->F && c->n > 0 && codes_out; ++f)
    LFE_HIP(hipMemcpyAsync(codes_out[f], c->fe[f].code, sizeof(int32_t) * c->n, hipMemcpyDeviceToHost, c->stream));
  LFE_HIP(hipStreamSynchronize(c->stream));
  return LFE_OK;
}

int lfe_shard_rows(lfe_ctx* c, int64_t* n_out) {
  if (!c || !n_out) return fail(LFE_EINVAL, "null pointer");
  *n_out = c->loaded ? c->n : 0;
  return LFE_OK;
}

int lfe_exact_sums(lfe_ctx* c, int* on) {
  LFE_CTX(c);
  if (!on) return fail(LFE_EINVAL, "null pointer");
  return exact_sums_on(c, on);
}

// host: (min, max) of an integer column in one pass over up to 8 threads (the dense-code test of
// frame.factorize; NumPy's two single-threaded reductions took 14 ms per 50M-row column)
// one slice: min / max reductions the compiler vectorizes; compiled for AVX2 and for the baseline
#define LFE_RANGE_SLICE(NAME, ATTR)                                                            \
  template <typename T>                                                                        \
  ATTR static void NAME(const T* __restrict__ v, int64_t a, int64_t b, int64_t* lo, int64_t* hi) { \
    T l = v[a], h = v[a];                                                                      \
    _Pragma("clang loop vectorize(enable) interleave(enable)")                                 \
    for (int64_t j = a; j < b; ++j) {                                                          \
      l = std::min(l, v[j]);                                                                   \
      h = std::max(h, v[j]);                                                                   \
    }                                                                                          \
    *lo = l;                                                                                   \
    *hi = h;                                                                                   \
  }
extern "C++" {
LFE_RANGE_SLICE(range_slice_avx2, __attribute__((target("avx2"))))
LFE_RANGE_SLICE(range_slice_base, )

template <typename T>
static void int_range_t(const T* v, int64_t n, int64_t* mn, int64_t* mx) {
  const int64_t t = std::max<int64_t>(1, std::min<int64_t>(8, n >> 22));
  const bool avx2 = __builtin_cpu_supports("avx2");
  std::vector<int64_t> lo((size_t)t), hi((size_t)t);
  auto work = [&](int64_t i) {
    const int64_t a = n * i / t, b = n * (i + 1) / t;
    if (avx2) range_slice_avx2(v, a, b, &lo[(size_t)i], &hi[(size_t)i]);
    else range_slice_base(v, a, b, &lo[(size_t)i], &hi[(size_t)i]);
  };
  std::vector<std::thread> th;
  for (int64_t i = 1; i < t; ++i) th.emplace_back(work, i);
  work(0);
  for (auto& x : th) x.join();
  *mn = *std::min_element(lo.begin(), lo.end());
  *mx = *std::max_element(hi.begin(), hi.end());
}
}

int lfe_int_range(const void* values, int64_t n, int width, int64_t* min_out, int64_t* max_out) {
  if (!min_out || !max_out || n < 1 || !values) return fail(LFE_EINVAL, "lfe_int_range: bad arguments");
  switch (width) {
    case 1: int_range_t(static_cast<const int8_t*>(values), n, min_out, max_out); break;
    case 2: int_range_t(static_cast<const int16_t*>(values), n, min_out, max_out); break;
    case 4: int_range_t(static_cast<const int32_t*>(values), n, min_out, max_out); break;
    case 8: int_range_t(static_cast<const int64_t*>(values), n, min_out, max_out); break;
    default: return fail(LFE_EINVAL, "lfe_int_range: width must be 1, 2, 4 or 8 (signed)");
  }
  return LFE_OK;
}

int lfe_test_set_knob(const char* name, const char* value) {
  if (!name || !name[0]) return fail(LFE_EINVAL, "knob name is empty");
  std::lock_guard<std::mutex> lk(g_knob_mu);
  if (value)
    g_knobs[name] = value;
  else if (name[0] == '*' && !name[1])
    g_knobs.clear();
  else
    g_knobs.erase(name);
  return LFE_OK;
}

int lfe_ctx_test_hooks(lfe_ctx* c, int flags) {
  LFE_CTX(c);
  if (flags & ~(LFE_TEST_SHORT_MEMORY | LFE_TEST_CLUSTER_SORTED | LFE_TEST_CLUSTER_STATS | LFE_TEST_SEG_SCATTER))
    return fail(LFE_EINVAL, "unknown test hook");
  c->test_hooks = flags;
  return LFE_OK;
}

int lfe_dense_cells(lfe_ctx* c, int64_t* cells) {
  LFE_CTX(c);
  if (!cells) return fail(LFE_EINVAL, "null pointer");
  *cells = c->dense_cells;
  return LFE_OK;
}

int lfe_dense_cell_bytes(lfe_ctx* c, int32_t* bytes) {
  LFE_CTX(c);
  if (!bytes) return fail(LFE_EINVAL, "null output pointer");
  *bytes = c->dense_cells ? (c->dn8 ? 1 : 2) : 0;
  return LFE_OK;
}

int lfe_sync(lfe_ctx* c) {
  LFE_CTX(c);
  LFE_HIP(hipStreamSynchronize(c->stream));
  return LFE_OK;
}

int lfe_profile(lfe_ctx* c, int enable) {
  LFE_CTX(c);
  LFE_TRY(prof_fold(c));
  for (int k = 0; k < K_NUM_KERNELS; ++k) {
    c->prof.total_ms[k] = 0;
    c->prof.count[k] = 0;
  }
  c->prof.on = enable != 0;
  return LFE_OK;
}

int lfe_phase_timing(lfe_ctx* c, int enable) {
  if (!c) return fail(LFE_EINVAL, "null context");
  c->tm.on = enable != 0;
  return LFE_OK;
}

int lfe_kernel_stats(lfe_ctx* c, int max, char* names, double* total_ms, int64_t* launches, int* n_out) {
  LFE_CTX(c);
  LFE_TRY(prof_fold(c));
  int n = 0;
  for (int k = 0; k < K_NUM_KERNELS && n < max; ++k) {
    if (c->prof.count[k] == 0) continue;
    if (names) {
      std::strncpy(names + 32 * n, kKernelNames[k], 31);
      names[32 * n + 31] = 0;
    }
    if (total_ms) total_ms[n] = c->prof.total_ms[k];
    if (launches) launches[n] = c->prof.count[k];
    ++n;
  }
  if (n_out) *n_out = n;
  return LFE_OK;
}

int lfe_timings(lfe_ctx* c, double* out6) {
  if (!c || !out6) return fail(LFE_EINVAL, "null pointer");
  for (int ph = 0; ph < 5; ++ph) {
    if (!(c->tm.pending & (1u << ph))) continue;
    float ms = 0.f;
    if (hipEventSynchronize(c->tm.ev[ph][1]) == hipSuccess &&
        hipEventElapsedTime(&ms, c->tm.ev[ph][0], c->tm.ev[ph][1]) == hipSuccess)
      c->tm.ms[ph] = ms;
  }
  c->tm.pending = 0;
  if (c->tm.last_phase >= 0) c->tm.last = c->tm.ms[c->tm.last_phase];
  for (int ph = 0; ph < 5; ++ph) out6[ph] = c->tm.ms[ph];
  out6[5] = c->tm.last;
  return LFE_OK;
}

}  // extern "C"
