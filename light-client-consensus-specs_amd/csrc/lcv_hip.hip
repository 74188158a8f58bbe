// lcv_hip.hip — HIP/gfx950 backend of liblcv.so (the product): streams, memory, events and the
// C ABI (lcv_driver.inc).  One lane per item; every stage of lcv_items.hpp is one kernel launch on
// the context's stream; HIP events bracket the stages so the per-stage kernel time is reported by
// lcv_last_timings() (and cross-checked with rocprofv3).  The kernels themselves live in the
// lcv_k_*.hip units (one heavy stage per unit so they compile in parallel).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <chrono>
#include <new>
#include <thread>
#include <type_traits>
#include <string>
#include <vector>

#define LCV_HD __device__
#include "lcv_common.hpp"  // LCV_SLOTS, EV_*

struct lcv_ctx;

// two streams per work-space slot; a stream per hardware queue when GPU_MAX_HW_QUEUES >= 2 x the slots in
// use (bench.py sets it; with HIP's default of 4 the streams share queues, which orders more than the
// events require)
enum { BE_STREAMS = 2 * LCV_SLOTS };
struct Backend {
  hipStream_t st[BE_STREAMS] = {};  // st[0]: main stream (copies, serial stages); st[k]: forked work
  int cur = 0;                      // stream of the next launch / copy
  int device = 0;
  struct Mark { int stage; hipEvent_t a, b; };
  std::vector<hipEvent_t> pool;
  size_t used = 0;
  std::vector<Mark> marks;
  int open_stage[BE_STREAMS];  // set to -1 by be_init
  hipEvent_t open_ev[BE_STREAMS] = {};
  hipEvent_t fork_ev[BE_STREAMS] = {}, join_ev[BE_STREAMS] = {};
  int base = 0;                          // work-space slot s uses streams st[2s] (main), st[2s + 1] (side)
  hipEvent_t ev[LCV_SLOTS][EV_COUNT] = {};  // run_bls's ordering events, per slot
  ncclComm_t comm = nullptr;  // RCCL communicator (lcv_comm_init), collectives on st[0]
  double* comm_scalar = nullptr;       // device scalar of lcv_comm_allreduce_max
  double* comm_host_scalar = nullptr;  // its pinned host staging (copies never block the bounded wait)
  uint32_t* hold_flag = nullptr;       // lcv_debug_hold_slot's release word: pinned, mapped, this context's
};

static int be_init(lcv_ctx* ctx, int device);
static void be_destroy(lcv_ctx* ctx);
static int be_alloc(lcv_ctx* ctx, void** p, size_t bytes);
static void be_free(lcv_ctx* ctx, void* p);
static int be_h2d(lcv_ctx* ctx, void* dst, const void* src, size_t bytes);
static int be_d2h(lcv_ctx* ctx, void* dst, const void* src, size_t bytes);
static int be_d2d(lcv_ctx* ctx, void* dst, const void* src, size_t bytes);
static int be_memset(lcv_ctx* ctx, void* p, int v, size_t bytes);
static int be_sync(lcv_ctx* ctx);
static int be_fork_to(lcv_ctx* ctx, int k);
static int be_join_from(lcv_ctx* ctx, int k);
static int be_nstreams() { return BE_STREAMS; }
template <class F> static int be_launch(lcv_ctx* ctx, const F& f, uint32_t n);
template <class F> static int be_launch_team(lcv_ctx* ctx, const F& f, uint32_t n);
template <class F> static int be_launch_sop(lcv_ctx* ctx, const F& f, uint32_t n, uint32_t g);
template <class F> static int be_launch_sop_fan(lcv_ctx* ctx, const F& f, uint32_t n);
static int be_fork(lcv_ctx* ctx);
static int be_join(lcv_ctx* ctx);
static void be_use_stream(lcv_ctx* ctx, int k);
static void be_set_slot(lcv_ctx* ctx, int slot);
static int be_mark(lcv_ctx* ctx, int ev, int k);
static int be_wait(lcv_ctx* ctx, int k, int ev);
static int be_sync_slot(lcv_ctx* ctx);
static void be_stage_begin(lcv_ctx* ctx, int stage);
static void be_stage_end(lcv_ctx* ctx, int stage);
static void be_reset_timings(lcv_ctx* ctx);
static void be_collect_timings(lcv_ctx* ctx);
static int be_comm_unique_id(uint8_t* id);
static int be_comm_init(lcv_ctx* ctx, int nranks, int rank, const uint8_t* id);
static void be_comm_destroy(lcv_ctx* ctx);
static int be_comm_allgather(lcv_ctx* ctx, const uint8_t* send, uint8_t* recv, size_t per_rank);
static int be_comm_allreduce_max(lcv_ctx* ctx, double* inout);
static int be_comm_count(lcv_ctx* ctx, int* out);
static int be_comm_wait(lcv_ctx* ctx);
static int be_comm_shrink(lcv_ctx* ctx, const int* exclude, int nexclude, int* rank, int* nranks);
static void be_comm_abort(lcv_ctx* ctx);
static int be_host_alloc(lcv_ctx* ctx, void** p, size_t bytes);
static void be_host_free(lcv_ctx* ctx, void* p);
static int be_wait_event(lcv_ctx* ctx, int ev);
static size_t be_event_pool_size(lcv_ctx* ctx);

#include "lcv_driver.inc"
#include "lcv_launch.hpp"

static int hip_fail(lcv_ctx* ctx, hipError_t e, const char* what) {
  return fail(ctx, LCV_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}
#define HIPCHK(ctx, x)                                  \
  do {                                                  \
    hipError_t _e = (x);                                \
    if (_e != hipSuccess) return hip_fail(ctx, _e, #x); \
  } while (0)

static hipStream_t cur_stream(lcv_ctx* ctx) { return ctx->be.st[ctx->be.base + ctx->be.cur]; }

static int be_init(lcv_ctx* ctx, int device) {
  int nd = 0;
  HIPCHK(ctx, hipGetDeviceCount(&nd));
  if (device < 0 || device >= nd) return fail(ctx, LCV_EDEVICE, "lcv_init: no such HIP device");
  ctx->be.device = device;
  HIPCHK(ctx, hipSetDevice(device));
  for (int k = 0; k < BE_STREAMS; ++k) {
    HIPCHK(ctx, hipStreamCreateWithFlags(&ctx->be.st[k], hipStreamNonBlocking));
    HIPCHK(ctx, hipEventCreateWithFlags(&ctx->be.fork_ev[k], hipEventDisableTiming));
    HIPCHK(ctx, hipEventCreateWithFlags(&ctx->be.join_ev[k], hipEventDisableTiming));
  }
  for (int s = 0; s < LCV_SLOTS; ++s)
    for (int e = 0; e < EV_COUNT; ++e) HIPCHK(ctx, hipEventCreateWithFlags(&ctx->be.ev[s][e], hipEventDisableTiming));
  for (int k = 0; k < BE_STREAMS; ++k) ctx->be.open_stage[k] = -1;
  return LCV_OK;
}

static void be_destroy(lcv_ctx* ctx) {
  (void)hipSetDevice(ctx->be.device);
  for (hipEvent_t e : ctx->be.pool) (void)hipEventDestroy(e);
  for (int k = 0; k < BE_STREAMS; ++k) {
    if (ctx->be.st[k]) (void)hipStreamDestroy(ctx->be.st[k]);
    if (ctx->be.fork_ev[k]) (void)hipEventDestroy(ctx->be.fork_ev[k]);
    if (ctx->be.join_ev[k]) (void)hipEventDestroy(ctx->be.join_ev[k]);
  }
  for (int s = 0; s < LCV_SLOTS; ++s)
    for (int e = 0; e < EV_COUNT; ++e)
      if (ctx->be.ev[s][e]) (void)hipEventDestroy(ctx->be.ev[s][e]);
  if (ctx->be.hold_flag) (void)hipHostFree(ctx->be.hold_flag);
  ctx->be.hold_flag = nullptr;
}

static int be_alloc(lcv_ctx* ctx, void** p, size_t bytes) {
  HIPCHK(ctx, hipSetDevice(ctx->be.device));
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) {
    *p = nullptr;
    return fail(ctx, LCV_ENOMEM, std::string("hipMalloc(") + std::to_string(bytes) + "): " + hipGetErrorString(e));
  }
  return LCV_OK;
}
static void be_free(lcv_ctx* ctx, void* p) {
  if (!p) return;
  (void)hipSetDevice(ctx->be.device);
  for (int k = 0; k < BE_STREAMS; ++k) (void)hipStreamSynchronize(ctx->be.st[k]);
  (void)hipFree(p);
}
static int be_h2d(lcv_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!bytes) return LCV_OK;
  HIPCHK(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, cur_stream(ctx)));
  return LCV_OK;
}
// pinned host memory (the staging buffers of lcv_validate_async): copies from it are DMA, asynchronous
// to the host, so a batch's upload overlaps the kernels of the other slots
static int be_host_alloc(lcv_ctx* ctx, void** p, size_t bytes) {
  HIPCHK(ctx, hipSetDevice(ctx->be.device));
  hipError_t e = hipHostMalloc(p, bytes ? bytes : 1, hipHostMallocDefault);
  if (e != hipSuccess) {
    *p = nullptr;
    return fail(ctx, LCV_ENOMEM, std::string("hipHostMalloc(") + std::to_string(bytes) + "): " + hipGetErrorString(e));
  }
  return LCV_OK;
}
static void be_host_free(lcv_ctx* ctx, void* p) {
  if (!p) return;
  (void)hipSetDevice(ctx->be.device);
  (void)hipHostFree(p);
}
// the host waits for the active slot's event `ev` (returns at once if it was never recorded)
static int be_wait_event(lcv_ctx* ctx, int ev) {
  HIPCHK(ctx, hipEventSynchronize(ctx->be.ev[ctx->be.base / 2][ev]));
  return LCV_OK;
}
static int be_d2h(lcv_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!bytes) return LCV_OK;
  HIPCHK(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, cur_stream(ctx)));
  return LCV_OK;
}
static int be_d2d(lcv_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!bytes) return LCV_OK;
  HIPCHK(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, cur_stream(ctx)));
  return LCV_OK;
}
static int be_memset(lcv_ctx* ctx, void* p, int v, size_t bytes) {
  if (!bytes) return LCV_OK;
  HIPCHK(ctx, hipMemsetAsync(p, v, bytes, cur_stream(ctx)));
  return LCV_OK;
}
static int be_sync(lcv_ctx* ctx) {
  for (int k = BE_STREAMS - 1; k >= 0; --k) HIPCHK(ctx, hipStreamSynchronize(ctx->be.st[k]));
  return LCV_OK;
}
static void be_use_stream(lcv_ctx* ctx, int k) { ctx->be.cur = (k > 0 && ctx->be.base + k < BE_STREAMS) ? k : 0; }
static void be_set_slot(lcv_ctx* ctx, int slot) {
  ctx->be.base = 2 * slot;
  ctx->be.cur = 0;
}
static int be_mark(lcv_ctx* ctx, int ev, int k) {
  HIPCHK(ctx, hipEventRecord(ctx->be.ev[ctx->be.base / 2][ev], ctx->be.st[ctx->be.base + k]));
  return LCV_OK;
}
static int be_wait(lcv_ctx* ctx, int k, int ev) {
  HIPCHK(ctx, hipStreamWaitEvent(ctx->be.st[ctx->be.base + k], ctx->be.ev[ctx->be.base / 2][ev], 0));
  return LCV_OK;
}
static int be_sync_slot(lcv_ctx* ctx) {
  HIPCHK(ctx, hipStreamSynchronize(ctx->be.st[ctx->be.base + 1]));
  HIPCHK(ctx, hipStreamSynchronize(ctx->be.st[ctx->be.base]));
  return LCV_OK;
}
// stream k starts after everything queued so far on the main stream
static int be_fork_to(lcv_ctx* ctx, int k) {
  const int b = ctx->be.base;
  HIPCHK(ctx, hipEventRecord(ctx->be.fork_ev[b + k], ctx->be.st[b]));
  HIPCHK(ctx, hipStreamWaitEvent(ctx->be.st[b + k], ctx->be.fork_ev[b + k], 0));
  return LCV_OK;
}
// the main stream continues after everything queued so far on stream k
static int be_join_from(lcv_ctx* ctx, int k) {
  const int b = ctx->be.base;
  HIPCHK(ctx, hipEventRecord(ctx->be.join_ev[b + k], ctx->be.st[b + k]));
  HIPCHK(ctx, hipStreamWaitEvent(ctx->be.st[b], ctx->be.join_ev[b + k], 0));
  return LCV_OK;
}
static int be_fork(lcv_ctx* ctx) { return be_fork_to(ctx, 1); }
static int be_join(lcv_ctx* ctx) { return be_join_from(ctx, 1); }

template <class F> static int be_launch(lcv_ctx* ctx, const F& f, uint32_t n) {
  if (n == 0) return LCV_OK;
  HIPCHK(ctx, hipSetDevice(ctx->be.device));
  HIPCHK(ctx, lcv_hip_launch<F>(f, n, cur_stream(ctx)));  // defined in the lcv_k_*.hip kernel units
  return LCV_OK;
}
template <class F> static int be_launch_team(lcv_ctx* ctx, const F& f, uint32_t n) {
  if (n == 0) return LCV_OK;
  HIPCHK(ctx, hipSetDevice(ctx->be.device));
  HIPCHK(ctx, lcv_hip_launch_team<F>(f, n, cur_stream(ctx)));
  return LCV_OK;
}

// g items per one-wave block (launch_sop, lcv_driver.inc)
template <class F> static int be_launch_sop(lcv_ctx* ctx, const F& f, uint32_t n, uint32_t g) {
  if (n == 0) return LCV_OK;
  HIPCHK(ctx, hipSetDevice(ctx->be.device));
  HIPCHK(ctx, lcv_hip_launch_sop<F>(f, n, cur_stream(ctx), g));
  return LCV_OK;
}

template <class F> static int be_launch_sop_fan(lcv_ctx* ctx, const F& f, uint32_t n) {
  if (n == 0) return LCV_OK;
  HIPCHK(ctx, hipSetDevice(ctx->be.device));
  HIPCHK(ctx, lcv_hip_launch_sop_fan<F>(f, n, cur_stream(ctx)));  // lcv_k_fan.hip
  return LCV_OK;
}

static hipEvent_t take_event(lcv_ctx* ctx) {
  Backend& b = ctx->be;
  if (b.used == b.pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    b.pool.push_back(e);
  }
  return b.pool[b.used++];
}
// stage marks: HIP events on the stream the stage's kernels are launched on
static size_t be_event_pool_size(lcv_ctx* ctx) { return ctx->be.pool.size(); }
static void be_stage_begin(lcv_ctx* ctx, int stage) {
  if (ctx->marks_off) return;
  hipEvent_t e = take_event(ctx);
  if (!e) return;
  const int k = ctx->be.base + ctx->be.cur;
  (void)hipEventRecord(e, cur_stream(ctx));
  ctx->be.open_stage[k] = stage;
  ctx->be.open_ev[k] = e;
}
static void be_stage_end(lcv_ctx* ctx, int stage) {
  if (ctx->marks_off) return;
  const int k = ctx->be.base + ctx->be.cur;
  if (ctx->be.open_stage[k] != stage || !ctx->be.open_ev[k]) return;
  hipEvent_t e = take_event(ctx);
  if (!e) return;
  (void)hipEventRecord(e, cur_stream(ctx));
  ctx->be.marks.push_back({stage, ctx->be.open_ev[k], e});
  ctx->be.open_stage[k] = -1;
  ctx->be.open_ev[k] = nullptr;
}
static void be_reset_timings(lcv_ctx* ctx) {
  ctx->be.marks.clear();
  ctx->be.used = 0;
  for (int k = 0; k < BE_STREAMS; ++k) ctx->be.open_stage[k] = -1;
  for (int s = 0; s < ST_COUNT; ++s) ctx->stage_ms[s] = 0.f;
}
static void be_collect_timings(lcv_ctx* ctx) {
  for (auto& m : ctx->be.marks) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, m.a, m.b) == hipSuccess) ctx->stage_ms[m.stage] += ms;
  }
  ctx->be.marks.clear();
  ctx->be.used = 0;
}

// ---- RCCL (over xGMI between the GPUs of one node): the verdict all-gather of lcv_validate_sharded
static int nccl_fail(lcv_ctx* ctx, ncclResult_t r, const char* what) {
  return fail(ctx, LCV_EDEVICE, std::string(what) + ": " + ncclGetErrorString(r));
}
static int be_comm_unique_id(uint8_t* id) {
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return LCV_EDEVICE;
  memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return LCV_OK;
}
static int be_comm_init(lcv_ctx* ctx, int nranks, int rank, const uint8_t* id) {
  HIPCHK(ctx, hipSetDevice(ctx->be.device));
  ncclUniqueId u;
  memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclResult_t r = ncclCommInitRank(&ctx->be.comm, nranks, u, rank);
  if (r != ncclSuccess) {
    ctx->be.comm = nullptr;
    return nccl_fail(ctx, r, "ncclCommInitRank");
  }
  HIPCHK(ctx, hipMalloc((void**)&ctx->be.comm_scalar, sizeof(double)));
  HIPCHK(ctx, hipHostMalloc((void**)&ctx->be.comm_host_scalar, sizeof(double), hipHostMallocDefault));
  return LCV_OK;
}
static void be_comm_free_scalars(lcv_ctx* ctx) {
  if (ctx->be.comm_scalar) (void)hipFree(ctx->be.comm_scalar);
  if (ctx->be.comm_host_scalar) (void)hipHostFree(ctx->be.comm_host_scalar);
  ctx->be.comm_scalar = nullptr;
  ctx->be.comm_host_scalar = nullptr;
}
static void be_comm_destroy(lcv_ctx* ctx) {
  (void)hipSetDevice(ctx->be.device);
  if (ctx->be.comm) (void)ncclCommDestroy(ctx->be.comm);
  ctx->be.comm = nullptr;
  be_comm_free_scalars(ctx);
}
static int be_comm_allgather(lcv_ctx* ctx, const uint8_t* send, uint8_t* recv, size_t per_rank) {
  HIPCHK(ctx, hipSetDevice(ctx->be.device));
  ncclResult_t r = ncclAllGather(send, recv, per_rank, ncclUint8, ctx->be.comm, cur_stream(ctx));
  return r == ncclSuccess ? LCV_OK : nccl_fail(ctx, r, "ncclAllGather");
}
static int be_comm_count(lcv_ctx* ctx, int* out) {
  int c = 0;
  ncclResult_t r = ncclCommCount(ctx->be.comm, &c);
  if (r != ncclSuccess) return nccl_fail(ctx, r, "ncclCommCount");
  *out = c;
  return LCV_OK;
}
// Waits for the current stream (a collective and what follows it) with a bound: polls the stream and
// RCCL's asynchronous error; a peer that died or hangs fails the call (LCV_EDEVICE, the context's
// communicator marked failed) instead of blocking this rank forever in the collective.
static int be_comm_wait_stream(lcv_ctx* ctx, hipStream_t s) {
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned it = 0;; ++it) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return LCV_OK;
    if (q != hipErrorNotReady) {
      ctx->comm_failed = true;
      return fail(ctx, LCV_EDEVICE, std::string("collective: ") + hipGetErrorString(q));
    }
    ncclResult_t ae = ncclSuccess;
    if (ncclCommGetAsyncError(ctx->be.comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
      ctx->comm_failed = true;
      return fail(ctx, LCV_EDEVICE, std::string("RCCL asynchronous error: ") + ncclGetErrorString(ae));
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > ctx->comm_timeout_s) {
      ctx->comm_failed = true;
      return fail(ctx, LCV_EDEVICE, "collective did not complete within the communicator timeout (a peer rank died or hangs)");
    }
    if (it >= 256) std::this_thread::sleep_for(std::chrono::microseconds(50));  // spin briefly first
  }
}
static int be_comm_wait(lcv_ctx* ctx) { return be_comm_wait_stream(ctx, cur_stream(ctx)); }
// the survivors' communicator: ncclCommShrink terminates the failed parent's operations (a collective
// stuck on a dead peer) and builds the new one; the parent is then aborted
static int be_comm_shrink(lcv_ctx* ctx, const int* exclude, int nexclude, int* rank, int* nranks) {
  HIPCHK(ctx, hipSetDevice(ctx->be.device));
  ncclComm_t nc = nullptr;
  // a failed parent first has its outstanding operations terminated (NCCL_SHRINK_ABORT)
  const int flags = ctx->comm_failed ? NCCL_SHRINK_ABORT : NCCL_SHRINK_DEFAULT;
  ncclResult_t r = ncclCommShrink(ctx->be.comm, const_cast<int*>(exclude), nexclude, &nc, nullptr, flags);
  if (r != ncclSuccess || !nc) return nccl_fail(ctx, r, "ncclCommShrink");
  (void)ncclCommAbort(ctx->be.comm);
  ctx->be.comm = nc;
  if ((r = ncclCommUserRank(nc, rank)) != ncclSuccess) return nccl_fail(ctx, r, "ncclCommUserRank");
  if ((r = ncclCommCount(nc, nranks)) != ncclSuccess) return nccl_fail(ctx, r, "ncclCommCount");
  return be_sync(ctx);  // the aborted collective no longer holds the streams
}
static void be_comm_abort(lcv_ctx* ctx) {
  (void)hipSetDevice(ctx->be.device);
  if (ctx->be.comm) (void)ncclCommAbort(ctx->be.comm);
  ctx->be.comm = nullptr;
  be_comm_free_scalars(ctx);
}
static int be_comm_allreduce_max(lcv_ctx* ctx, double* inout) {
  HIPCHK(ctx, hipSetDevice(ctx->be.device));
  hipStream_t s = ctx->be.st[0];
  // both copies go through pinned memory (DMA, asynchronous to the host), so the host reaches the
  // bounded wait even when the collective can never complete; the caller's double is written after it
  // (every earlier call ended with its wait, or failed the communicator, which refuses further calls)
  *ctx->be.comm_host_scalar = *inout;
  HIPCHK(ctx, hipMemcpyAsync(ctx->be.comm_scalar, ctx->be.comm_host_scalar, sizeof(double), hipMemcpyHostToDevice, s));
  ncclResult_t r = ncclAllReduce(ctx->be.comm_scalar, ctx->be.comm_scalar, 1, ncclFloat64, ncclMax, ctx->be.comm, s);
  if (r != ncclSuccess) return nccl_fail(ctx, r, "ncclAllReduce");
  HIPCHK(ctx, hipMemcpyAsync(ctx->be.comm_host_scalar, ctx->be.comm_scalar, sizeof(double), hipMemcpyDeviceToHost, s));
  LCV_TRY(be_comm_wait_stream(ctx, s));
  *inout = *ctx->be.comm_host_scalar;
  return LCV_OK;
}

// ---- test entries: hold a slot's main stream (a one-wave kernel that spins until the host releases it or
// `max_seconds` of the device's constant-rate clock pass — every wave reaches the exit), so that a
// collective enqueued behind it cannot complete: the bounded collective waits must then fail the call
// within the communicator timeout (tests/test_multi_gpu.py)
__global__ __launch_bounds__(64) void k_hold(const volatile uint32_t* flag, uint64_t max_ticks) {
  const uint64_t t0 = wall_clock64();
  while (*flag == 0u && wall_clock64() - t0 < max_ticks) __builtin_amdgcn_s_sleep(127);
}
// The release word is the context's own (allocated on its device on first use, freed by be_destroy), so
// lcv_debug_release_slots(ctx) releases only this context's holds.
extern "C" int lcv_debug_hold_slot(lcv_ctx* ctx, int slot, double max_seconds) {
  if (!ctx || slot < 0 || slot >= LCV_SLOTS || !(max_seconds > 0.0) || max_seconds > 120.0)
    return fail(ctx, LCV_EINVAL, "lcv_debug_hold_slot: slot 0..7, 0 < max_seconds <= 120");
  HIPCHK(ctx, hipSetDevice(ctx->be.device));
  if (!ctx->be.hold_flag)
    HIPCHK(ctx, hipHostMalloc((void**)&ctx->be.hold_flag, 64, hipHostMallocMapped | hipHostMallocCoherent));
  __atomic_store_n(ctx->be.hold_flag, 0u, __ATOMIC_SEQ_CST);
  uint32_t* dflag = nullptr;
  HIPCHK(ctx, hipHostGetDevicePointer((void**)&dflag, ctx->be.hold_flag, 0));
  int khz = 0;
  HIPCHK(ctx, hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->be.device));
  const uint64_t ticks = (uint64_t)(max_seconds * 1e3 * (double)(khz > 0 ? khz : 100000));
  hipLaunchKernelGGL(k_hold, dim3(1), dim3(64), 0, ctx->be.st[2 * slot], (const volatile uint32_t*)dflag, ticks);
  HIPCHK(ctx, hipGetLastError());
  return LCV_OK;
}
extern "C" int lcv_debug_release_slots(lcv_ctx* ctx) {
  if (!ctx) return LCV_EINVAL;
  if (ctx->be.hold_flag) __atomic_store_n(ctx->be.hold_flag, 1u, __ATOMIC_SEQ_CST);
  return LCV_OK;
}

extern "C" int lcv_device_count(int* out) {
  if (!out) return LCV_EINVAL;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *out = n;
  return LCV_OK;
}
