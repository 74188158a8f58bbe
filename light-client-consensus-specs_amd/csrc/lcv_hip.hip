// lcv_hip.hip — HIP/gfx950 backend of liblcv.so (the product): streams, memory, events and the
// C ABI (lcv_driver.inc).  One lane per item; every stage of lcv_items.hpp is one kernel launch on
// the context's stream; HIP events bracket the stages so the per-stage kernel time is reported by
// lcv_last_timings() (and cross-checked with rocprofv3).  The kernels themselves live in the
// lcv_k_*.hip units (one heavy stage per unit so they compile in parallel).
#include <hip/hip_runtime.h>

#include <new>
#include <string>
#include <vector>

#define LCV_HD __device__

struct lcv_ctx;

struct Backend {
  hipStream_t stream = nullptr;   // main stream: copies + the current launch stream when cur == 0
  hipStream_t side = nullptr;     // second stream for independent stages (be_fork / be_join)
  int cur = 0;
  int device = 0;
  struct Mark { int stage; hipEvent_t a, b; };
  std::vector<hipEvent_t> pool;
  size_t used = 0;
  std::vector<Mark> marks;
  int open_stage[2] = {-1, -1};
  hipEvent_t open_ev[2] = {nullptr, nullptr};
  hipEvent_t fork_ev = nullptr, join_ev = nullptr;
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
template <class F> static int be_launch(lcv_ctx* ctx, const F& f, uint32_t n);
template <class F> static int be_launch_team(lcv_ctx* ctx, const F& f, uint32_t n);
static int be_fork(lcv_ctx* ctx);
static int be_join(lcv_ctx* ctx);
static void be_use_stream(lcv_ctx* ctx, int k);
static void be_stage_begin(lcv_ctx* ctx, int stage);
static void be_stage_end(lcv_ctx* ctx, int stage);
static void be_reset_timings(lcv_ctx* ctx);
static void be_collect_timings(lcv_ctx* ctx);

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

static int be_init(lcv_ctx* ctx, int device) {
  int nd = 0;
  HIPCHK(ctx, hipGetDeviceCount(&nd));
  if (device < 0 || device >= nd) return fail(ctx, LCV_EDEVICE, "lcv_init: no such HIP device");
  ctx->be.device = device;
  HIPCHK(ctx, hipSetDevice(device));
  HIPCHK(ctx, hipStreamCreateWithFlags(&ctx->be.stream, hipStreamNonBlocking));
  HIPCHK(ctx, hipStreamCreateWithFlags(&ctx->be.side, hipStreamNonBlocking));
  HIPCHK(ctx, hipEventCreateWithFlags(&ctx->be.fork_ev, hipEventDisableTiming));
  HIPCHK(ctx, hipEventCreateWithFlags(&ctx->be.join_ev, hipEventDisableTiming));
  return LCV_OK;
}

static void be_destroy(lcv_ctx* ctx) {
  (void)hipSetDevice(ctx->be.device);
  for (hipEvent_t e : ctx->be.pool) (void)hipEventDestroy(e);
  if (ctx->be.stream) (void)hipStreamDestroy(ctx->be.stream);
  if (ctx->be.side) (void)hipStreamDestroy(ctx->be.side);
  if (ctx->be.fork_ev) (void)hipEventDestroy(ctx->be.fork_ev);
  if (ctx->be.join_ev) (void)hipEventDestroy(ctx->be.join_ev);
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
  (void)hipStreamSynchronize(ctx->be.stream);
  (void)hipStreamSynchronize(ctx->be.side);
  (void)hipFree(p);
}
static int be_h2d(lcv_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!bytes) return LCV_OK;
  HIPCHK(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->be.stream));
  return LCV_OK;
}
static int be_d2h(lcv_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!bytes) return LCV_OK;
  HIPCHK(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->be.stream));
  return LCV_OK;
}
static int be_d2d(lcv_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!bytes) return LCV_OK;
  HIPCHK(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ctx->be.stream));
  return LCV_OK;
}
static int be_memset(lcv_ctx* ctx, void* p, int v, size_t bytes) {
  if (!bytes) return LCV_OK;
  HIPCHK(ctx, hipMemsetAsync(p, v, bytes, ctx->be.stream));
  return LCV_OK;
}
static int be_sync(lcv_ctx* ctx) {
  HIPCHK(ctx, hipStreamSynchronize(ctx->be.side));
  HIPCHK(ctx, hipStreamSynchronize(ctx->be.stream));
  return LCV_OK;
}
static hipStream_t cur_stream(lcv_ctx* ctx) { return ctx->be.cur ? ctx->be.side : ctx->be.stream; }
static void be_use_stream(lcv_ctx* ctx, int k) { ctx->be.cur = k ? 1 : 0; }
// side stream starts after everything queued so far on the main stream
static int be_fork(lcv_ctx* ctx) {
  HIPCHK(ctx, hipEventRecord(ctx->be.fork_ev, ctx->be.stream));
  HIPCHK(ctx, hipStreamWaitEvent(ctx->be.side, ctx->be.fork_ev, 0));
  return LCV_OK;
}
// main stream continues after everything queued so far on the side stream
static int be_join(lcv_ctx* ctx) {
  HIPCHK(ctx, hipEventRecord(ctx->be.join_ev, ctx->be.side));
  HIPCHK(ctx, hipStreamWaitEvent(ctx->be.stream, ctx->be.join_ev, 0));
  return LCV_OK;
}

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
static void be_stage_begin(lcv_ctx* ctx, int stage) {
  hipEvent_t e = take_event(ctx);
  if (!e) return;
  const int k = ctx->be.cur;
  (void)hipEventRecord(e, cur_stream(ctx));
  ctx->be.open_stage[k] = stage;
  ctx->be.open_ev[k] = e;
}
static void be_stage_end(lcv_ctx* ctx, int stage) {
  const int k = ctx->be.cur;
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
  ctx->be.open_stage[0] = ctx->be.open_stage[1] = -1;
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

extern "C" int lcv_device_count(int* out) {
  if (!out) return LCV_EINVAL;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *out = n;
  return LCV_OK;
}
