// quadtrace.hip — where a LONE wave's SOP round goes (the latency path, lcv_set_latency_mode): runs the
// generated fexp program (csrc/lcv_sop_programs.inc) for ONE item through (a) the batch engine's round
// (one lane per op, lcv::sop_exec) and (b) the quad engine's round (four lanes per op,
// lcv_sop_quad.hpp), lane 0 stamping the shader clock (s_memtime) between the phases of every round:
//   batch: header/record | products + reduction + tail          (sop_exec as one piece)
//   quad:  header/record | products | transpose | reduction | tail
// Prints the mean shader cycles per round for each phase.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../light-client-consensus-specs_amd/csrc quadtrace.hip -o quadtrace
#define LCV_HD __device__
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "lcv_sop_quad.hpp"
#include "lcv_sop_programs.inc"

using namespace lcv;

__device__ inline uint64_t stamp() { return __builtin_readcyclecounter(); }

__global__ __launch_bounds__(64) void k_batch(SopView P, uint64_t* ph) {
  constexpr uint32_t T = LCV_SOP_FEXP_TEAM;
  extern __shared__ uint32_t lds[];
  const uint32_t lane = threadIdx.x;
  const bool active = lane < T;
  const uint32_t shared = P.nconst * 12;
  uint32_t* my = lds + shared;
  for (uint32_t k = threadIdx.x; k < shared; k += 64) lds[k] = P.consts[k];
  for (uint32_t s = lane; s < P.nslots && active; s += T)
    for (int j = 0; j < 12; ++j) my[12 * s + j] = j == 11 ? 0x01000000u + s : 0x9e3779b9u * (7 * s + j + 1);
  __syncthreads();
  uint64_t acc[2] = {0, 0};
  for (uint32_t r = 0; r < P.rounds; ++r) {
    const uint64_t t0 = stamp();
    const uint32_t h0 = __builtin_amdgcn_readfirstlane(P.hdr[4 * r]);
    const uint32_t off = __builtin_amdgcn_readfirstlane(P.hdr[4 * r + 1]);
    const uint32_t words = __builtin_amdgcn_readfirstlane(P.hdr[4 * r + 2]);
    const uint32_t h3 = __builtin_amdgcn_readfirstlane(P.hdr[4 * r + 3]);
    const uint32_t* w = P.rec + off + (active ? lane : 0) * words;
    const SopPre pre = sop_pre(h0, w);
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t t1 = stamp();
    if (active) sop_exec(h0, h3, w, pre, my, my, lds, P.nslots, nullptr, nullptr);
    __syncthreads();
    const uint64_t t2 = stamp();
    acc[0] += t1 - t0;
    acc[1] += t2 - t1;
  }
  if (threadIdx.x == 0) { ph[0] = acc[0]; ph[1] = acc[1]; }
}

__global__ __launch_bounds__(64) void k_quad(SopView P, uint64_t* ph) {
  constexpr uint32_t T = LCV_SOP_FEXP_TEAM;
  extern __shared__ uint32_t lds[];
  const uint32_t op = threadIdx.x >> 2, q = threadIdx.x & 3u;
  const bool active = op < T;
  const uint32_t shared = P.nconst * 12;
  const uint32_t item_words = (P.nslots * 12 + 4 + 1) & ~1u;
  uint32_t* my = lds + shared;
  uint64_t* scratch = (uint64_t*)(lds + shared + item_words);
  uint64_t* S = scratch + (active ? op : 0) * QUAD_SCRATCH_U64;
  for (uint32_t k = threadIdx.x; k < shared; k += 64) lds[k] = P.consts[k];
  for (uint32_t k = threadIdx.x; k < T * QUAD_SCRATCH_U64; k += 64) scratch[k] = 0;
  if (active && q == 0)
    for (uint32_t s = op; s < P.nslots; s += T)
      for (int j = 0; j < 12; ++j) my[12 * s + j] = j == 11 ? 0x01000000u + s : 0x9e3779b9u * (7 * s + j + 1);
  __syncthreads();
  uint32_t pz[16];
  quad_ptable(pz, q);
  uint64_t acc[5] = {0, 0, 0, 0, 0};
  for (uint32_t r = 0; r < P.rounds; ++r) {
    const uint64_t t0 = stamp();
    const uint32_t h0 = __builtin_amdgcn_readfirstlane(P.hdr[4 * r]);
    const uint32_t off = __builtin_amdgcn_readfirstlane(P.hdr[4 * r + 1]);
    const uint32_t words = __builtin_amdgcn_readfirstlane(P.hdr[4 * r + 2]);
    const uint32_t h3 = __builtin_amdgcn_readfirstlane(P.hdr[4 * r + 3]);
    const uint32_t* w = P.rec + off + (active ? op : 0) * words;
    const SopPre pre = sop_pre(h0, w);
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t t1 = stamp();
    uint64_t t2 = t1, t3 = t1, t4 = t1;
    if (active) {
      const uint32_t K = h0 & 15u;
      const bool mflag = (h0 >> 6) & 1u;
      uint32_t rr[13];
      if (K == 0) {
        for (int j = 0; j < 13; ++j) rr[j] = 0;
      } else {
        const SopBase base{my, lds, (int32_t)((const char*)lds - (const char*)my)};
        uint64_t pc[26], A[7];
        quad_products(pc, w + 4, K, h3, mflag, base, q, pre.x, pre.y, pre.m);
        t2 = stamp();
        quad_transpose(A, pc, S, q);
        __builtin_amdgcn_s_waitcnt(0);
        t3 = stamp();
        quad_redc(rr, A, pz);
        t4 = stamp();
      }
      sop_tail(h0, w, pre, my, my, lds, P.nslots, nullptr, nullptr, rr);
    }
    __syncthreads();
    const uint64_t t5 = stamp();
    acc[0] += t1 - t0;
    acc[1] += t2 - t1;
    acc[2] += t3 - t2;
    acc[3] += t4 - t3;
    acc[4] += t5 - t4;
  }
  if (threadIdx.x == 0)
    for (int k = 0; k < 5; ++k) ph[k] = acc[k];
}

int main() {
  SopView P{};
  uint32_t *hdr, *rec, *cst;
  hipMalloc(&hdr, sizeof(kSop_fexp_hdr));
  hipMalloc(&rec, sizeof(kSop_fexp_rec));
  hipMalloc(&cst, sizeof(kSop_fexp_consts));
  hipMemcpy(hdr, kSop_fexp_hdr, sizeof(kSop_fexp_hdr), hipMemcpyHostToDevice);
  hipMemcpy(rec, kSop_fexp_rec, sizeof(kSop_fexp_rec), hipMemcpyHostToDevice);
  hipMemcpy(cst, kSop_fexp_consts, sizeof(kSop_fexp_consts), hipMemcpyHostToDevice);
  P.hdr = hdr; P.rec = rec; P.consts = cst;
  P.rounds = LCV_SOP_FEXP_ROUNDS; P.nslots = LCV_SOP_FEXP_SLOTS; P.nconst = LCV_SOP_FEXP_NCONST;
  uint64_t* ph;
  hipMalloc(&ph, 8 * sizeof(uint64_t));
  const size_t lds_b = 4 * (P.nconst * 12 + P.nslots * 12 + 4);
  const size_t lds_q = 4 * (P.nconst * 12 + ((P.nslots * 12 + 4 + 1) & ~1u)) + 8 * LCV_SOP_FEXP_TEAM * QUAD_SCRATCH_U64;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int rep = 0; rep < 3; ++rep) {
    float ms;
    uint64_t h[8];
    hipEventRecord(a);
    hipLaunchKernelGGL(k_batch, dim3(1), dim3(64), lds_b, 0, P, ph);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    hipMemcpy(h, ph, 2 * 8, hipMemcpyDeviceToHost);
    printf("batch engine: %.3f ms, per round cycles: header/record %.0f | op %.0f\n", ms, (double)h[0] / P.rounds,
           (double)h[1] / P.rounds);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_quad, dim3(1), dim3(64), lds_q, 0, P, ph);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b);
    hipMemcpy(h, ph, 5 * 8, hipMemcpyDeviceToHost);
    printf("quad engine : %.3f ms, per round cycles: header/record %.0f | products %.0f | transpose %.0f | "
           "reduction %.0f | tail %.0f\n", ms, (double)h[0] / P.rounds, (double)h[1] / P.rounds,
           (double)h[2] / P.rounds, (double)h[3] / P.rounds, (double)h[4] / P.rounds);
  }
  return 0;
}
