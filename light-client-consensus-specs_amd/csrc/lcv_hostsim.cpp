// lcv_hostsim.cpp — TEST-ONLY host simulation of liblcv.so (built as liblcv_hostsim.so).
// Runs the exact per-item device code of lcv_items.hpp in plain host loops (OpenMP), so the CPU-only
// test suite can check the device arithmetic against the oracle.  The product package `lcv` never
// loads this library; it exists only for tests/ (see DESIGN.md "Testing without a GPU").
#define LCV_HOSTSIM 1
#include <atomic>
#include <chrono>
#include <fstream>
#include <new>
#include <thread>
#include <errno.h>
#include <sys/stat.h>
#include <unistd.h>
#include <stdlib.h>
#include <string>
#include <vector>

#define LCV_HD

struct lcv_ctx;

#ifdef LCV_OPCOUNT
namespace lcv { std::atomic<unsigned long long> g_ops[4]; }
#endif

// Stage marks are kept per (simulated) stream, like the HIP backend's, so that marks opened on
// different streams never overwrite each other; the driver's marks do not nest on one stream.
struct Backend {
  int cur = 0;
  int open_stage[4] = {-1, -1, -1, -1};
  std::chrono::steady_clock::time_point t0[4];
  unsigned long long ops0[4][4] = {};
  unsigned long long ops[16][4] = {};
  // test-only stand-in for the RCCL communicator: collectives through files in a directory shared by
  // the ranks (the "unique id" is its path), so the multi-process path runs on the CPU (tests/test_multi.py)
  std::string comm_dir;
  int comm_rank = 0, comm_n = 1;
  unsigned long long comm_round = 0;
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
template <class F> static int be_launch_sop(lcv_ctx* ctx, const F& f, uint32_t n, uint32_t g = 0);
// the latency engine's launches run the same per-item code (the device spreads products over lanes)
// the fan engine (device latency mode) computes the batch engine's values: the simulation runs the latter
template <class F> static int be_launch_sop_fan(lcv_ctx* ctx, const F& f, uint32_t n) { return be_launch_sop(ctx, f, n); }
static int be_fork(lcv_ctx*) { return 0; }
static int be_join(lcv_ctx*) { return 0; }
static void be_use_stream(lcv_ctx* ctx, int k);
static int be_fork_to(lcv_ctx*, int) { return 0; }
static int be_join_from(lcv_ctx*, int) { return 0; }
static int be_nstreams() { return 4; }
// the host simulation runs every launch in program order: slots and events order nothing
static void be_set_slot(lcv_ctx*, int) {}
static int be_mark(lcv_ctx*, int, int) { return 0; }
static int be_wait(lcv_ctx*, int, int) { return 0; }
static int be_sync_slot(lcv_ctx*) { return 0; }
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
static void be_host_free(lcv_ctx*, void* p) { free(p); }
static int be_wait_event(lcv_ctx*, int) { return 0; }
static size_t be_event_pool_size(lcv_ctx*) { return 0; }

#include "lcv_driver.inc"

static int be_init(lcv_ctx* ctx, int device) {
  if (device != 0) return fail(ctx, LCV_EDEVICE, "hostsim: only device 0");
  return LCV_OK;
}
static void be_destroy(lcv_ctx*) {}
static int be_alloc(lcv_ctx* ctx, void** p, size_t bytes) {
  *p = calloc(1, bytes ? bytes : 1);
  return *p ? LCV_OK : fail(ctx, LCV_ENOMEM, "hostsim: out of memory");
}
static void be_free(lcv_ctx*, void* p) { free(p); }
static int be_host_alloc(lcv_ctx* ctx, void** p, size_t bytes) { return be_alloc(ctx, p, bytes); }
static int be_h2d(lcv_ctx*, void* dst, const void* src, size_t bytes) { memcpy(dst, src, bytes); return LCV_OK; }
static int be_d2h(lcv_ctx*, void* dst, const void* src, size_t bytes) { memcpy(dst, src, bytes); return LCV_OK; }
static int be_d2d(lcv_ctx*, void* dst, const void* src, size_t bytes) { memmove(dst, src, bytes); return LCV_OK; }
static int be_memset(lcv_ctx*, void* p, int v, size_t bytes) { memset(p, v, bytes); return LCV_OK; }
static int be_sync(lcv_ctx*) { return LCV_OK; }
template <class F> static int be_launch(lcv_ctx*, const F& f, uint32_t n) {
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t i = 0; i < (int64_t)n; ++i) f((uint32_t)i);
  return LCV_OK;
}
// team kernels: the rounds of one item run in order; within a round every lane of the team runs
// (sequentially here, in lockstep on the device) — programs never read a slot written in the same round
template <class F> static int be_launch_team(lcv_ctx*, const F& f, uint32_t n) {
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    std::vector<uint32_t> lds(F::LDS_WORDS, 0u), shared(F::SHARED_WORDS + 1, 0u);
    const uint32_t R = f.rounds();
    for (uint32_t r = 0; r < R; ++r)
      for (uint32_t lane = 0; lane < F::TEAM; ++lane) f((uint32_t)i, lane, r, lds.data(), shared.data());
  }
  return LCV_OK;
}
static void be_use_stream(lcv_ctx* ctx, int k) { ctx->be.cur = (k > 0 && k < 4) ? k : 0; }
// SOP team kernels: every lane of a round reads the item's LDS as it was when the round began (the
// device's lockstep wave), so the rounds run lane by lane against a snapshot
template <class F> static int be_launch_sop(lcv_ctx*, const F& f, uint32_t n, uint32_t) {
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    std::vector<uint32_t> lds(F::LDS_WORDS, 0u), snap(F::LDS_WORDS, 0u), cl(F::SHARED_WORDS + 1, 0u);
    for (uint32_t k = 0; k < F::SHARED_WORDS; ++k) cl[k] = f.P.consts[k];
    for (uint32_t lane = 0; lane < F::TEAM; ++lane) f.prologue((uint32_t)i, lane, lds.data());
    const uint32_t* io_in = f.io_in((uint32_t)i);
    uint32_t* io_out = f.io_out((uint32_t)i);
    for (uint32_t r = 0; r < f.P.rounds; ++r) {
      snap = lds;
      for (uint32_t lane = 0; lane < F::TEAM; ++lane)
        lcv::sop_round(f.P, r, lane, snap.data(), lds.data(), cl.data(), io_in, io_out);
    }
    for (uint32_t lane = 0; lane < F::TEAM; ++lane) f.epilogue((uint32_t)i, lane, lds.data());
  }
  return LCV_OK;
}

static void be_stage_begin(lcv_ctx* ctx, int stage) {
  if (ctx->marks_off) return;
  Backend& b = ctx->be;
  b.open_stage[b.cur] = stage;
  b.t0[b.cur] = std::chrono::steady_clock::now();
#ifdef LCV_OPCOUNT
  for (int k = 0; k < 4; ++k) b.ops0[b.cur][k] = lcv::g_ops[k].load();
#endif
}
static void be_stage_end(lcv_ctx* ctx, int stage) {
  if (ctx->marks_off) return;
  Backend& b = ctx->be;
  if (b.open_stage[b.cur] != stage) return;
  const auto t1 = std::chrono::steady_clock::now();
  ctx->stage_ms[stage] += std::chrono::duration<float, std::milli>(t1 - b.t0[b.cur]).count();
#ifdef LCV_OPCOUNT
  for (int k = 0; k < 4; ++k) b.ops[stage][k] += lcv::g_ops[k].load() - b.ops0[b.cur][k];
#endif
  b.open_stage[b.cur] = -1;
}
static void be_reset_timings(lcv_ctx* ctx) {
  for (int k = 0; k < 4; ++k) ctx->be.open_stage[k] = -1;
  for (int s = 0; s < ST_COUNT; ++s) ctx->stage_ms[s] = 0.f;
  for (int s = 0; s < 16; ++s) for (int k = 0; k < 4; ++k) ctx->be.ops[s][k] = 0;
}
static void be_collect_timings(lcv_ctx*) {}

static int be_comm_unique_id(uint8_t* id) {
  char tmpl[] = "/tmp/lcv_comm_XXXXXX";
  if (!mkdtemp(tmpl)) return LCV_EDEVICE;
  memset(id, 0, 128);
  memcpy(id, tmpl, strlen(tmpl));
  return LCV_OK;
}
static int be_comm_init(lcv_ctx* ctx, int nranks, int rank, const uint8_t* id) {
  ctx->be.comm_dir.assign((const char*)id, strnlen((const char*)id, 128));
  ctx->be.comm_rank = rank;
  ctx->be.comm_n = nranks;
  ctx->be.comm_round = 0;
  return LCV_OK;
}
static void be_comm_destroy(lcv_ctx* ctx) { ctx->be.comm_dir.clear(); }
// every rank writes <dir>/<round>.<rank> (atomically: temp file + rename), then reads all of them
static int comm_exchange(lcv_ctx* ctx, const void* mine, size_t bytes, uint8_t* all) {
  Backend& b = ctx->be;
  const unsigned long long r = b.comm_round++;
  auto name = [&](int k) { return b.comm_dir + "/" + std::to_string(r) + "." + std::to_string(k); };
  {
    const std::string tmp = name(b.comm_rank) + ".tmp";
    std::ofstream f(tmp, std::ios::binary);
    f.write((const char*)mine, (std::streamsize)bytes);
    f.close();
    if (!f || rename(tmp.c_str(), name(b.comm_rank).c_str()) != 0) return fail(ctx, LCV_EDEVICE, "hostsim comm: write");
  }
  for (int k = 0; k < b.comm_n; ++k) {
    for (int t = 0;; ++t) {
      std::ifstream f(name(k), std::ios::binary);
      if (f) {
        f.read((char*)all + (size_t)k * bytes, (std::streamsize)bytes);
        if ((size_t)f.gcount() == bytes) break;
      }
      if (t > 1000.0 * ctx->comm_timeout_s) {
        ctx->comm_failed = true;
        return fail(ctx, LCV_EDEVICE, "hostsim comm: collective did not complete within the communicator timeout");
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  }
  return LCV_OK;
}
static int be_comm_allgather(lcv_ctx* ctx, const uint8_t* send, uint8_t* recv, size_t per_rank) {
  return comm_exchange(ctx, send, per_rank, recv);
}
static int be_comm_count(lcv_ctx* ctx, int* out) {
  *out = ctx->be.comm_n;
  return LCV_OK;
}
static int be_comm_wait(lcv_ctx*) { return LCV_OK; }  // the stand-in's exchanges are synchronous
// the survivors renumber in rank order and continue in a sub-directory every survivor names alike
static int be_comm_shrink(lcv_ctx* ctx, const int* exclude, int nexclude, int* rank, int* nranks) {
  Backend& b = ctx->be;
  std::vector<bool> gone((size_t)b.comm_n, false);
  for (int i = 0; i < nexclude; ++i) gone[(size_t)exclude[i]] = true;
  std::string sub = b.comm_dir + "/shrink";
  int r = 0, n = 0;
  for (int k = 0; k < b.comm_n; ++k) {
    if (gone[(size_t)k]) {
      sub += "_" + std::to_string(k);
      continue;
    }
    if (k == b.comm_rank) r = n;
    ++n;
  }
  if (mkdir(sub.c_str(), 0700) != 0 && errno != EEXIST) return fail(ctx, LCV_EDEVICE, "hostsim comm: shrink directory");
  b.comm_dir = sub;
  b.comm_rank = r;
  b.comm_n = n;
  b.comm_round = 0;
  *rank = r;
  *nranks = n;
  return LCV_OK;
}
static void be_comm_abort(lcv_ctx* ctx) { ctx->be.comm_dir.clear(); }
static int be_comm_allreduce_max(lcv_ctx* ctx, double* inout) {
  std::vector<double> all((size_t)ctx->be.comm_n);
  LCV_TRY(comm_exchange(ctx, inout, sizeof(double), (uint8_t*)all.data()));
  for (double x : all) *inout = x > *inout ? x : *inout;
  return LCV_OK;
}

// the stream-hold test entries need a device queue (lcv_hip.hip); the host simulation refuses them
extern "C" int lcv_debug_hold_slot(lcv_ctx* ctx, int, double) {
  return fail(ctx, LCV_EINVAL, "lcv_debug_hold_slot: device backend only");
}
extern "C" int lcv_debug_release_slots(lcv_ctx* ctx) { return ctx ? LCV_OK : LCV_EINVAL; }

extern "C" int lcv_device_count(int* out) {
  if (!out) return LCV_EINVAL;
  *out = 1;
  return LCV_OK;
}

// test/tool-only: per-stage operation counts of the last validate call (needs -DLCV_OPCOUNT):
// out[4 * s + k], k = 0 Fp multiplications, 1 Fp additions/subtractions/halvings, 2 SHA-256 compressions,
// 3 SOP half-multiplications (a 12x12-limb product or a Montgomery reduction)
extern "C" int lcv_debug_opcounts(lcv_ctx* ctx, unsigned long long* out, int max_stages) {
  if (!ctx || !out) return LCV_EINVAL;
  for (int s = 0; s < max_stages && s < 16; ++s)
    for (int k = 0; k < 4; ++k) out[4 * s + k] = ctx->be.ops[s][k];
  return LCV_OK;
}
