// soptrace.hip — where the SOP programs spend their time: runs each generated program (lines, miller_acc,
// fexp, h2c; csrc/lcv_sop_programs.inc) through the same round loop as k_sop (csrc/lcv_functors_sop.hpp)
// at the production block count for 10^4 updates, with lane 0 of every block stamping the wall clock
// (100 MHz) at each round.  Prints the kernel time, the mean cost per round by round shape (K, operand
// flags, reduction steps, inversion / load / emit) and the most expensive rounds.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../light-client-consensus-specs_amd/csrc soptrace.hip -o soptrace
#define LCV_HD __device__
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <map>
#include <string>
#include <vector>

#include "lcv_sop.hpp"
#include "lcv_sop_programs.inc"

struct Prog {
  const char* name;
  const uint32_t *hdr, *rec, *consts;
  uint32_t nhdr, nrec, rounds, slots, nconst, team, items, io_words;
};

// W: the program's VGPR budget in waves per SIMD (F::WAVES in csrc/lcv_functors_sop.hpp); the 2-wave
// programs scan products three at a time, as k_sop does
template <uint32_t T, uint32_t W>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(W))) void k_trace(lcv::SopView P, uint32_t n,
                                                                                      uint32_t lds_words, uint32_t* io,
                                                                                      uint32_t io_words, uint64_t* trace,
                                                                                      uint32_t* hwid) {
  constexpr uint32_t G = 64 / T;
  extern __shared__ uint32_t lds[];
  const uint32_t team = threadIdx.x / T, lane = threadIdx.x % T;
  const uint32_t item = blockIdx.x * G + team;
  const bool active = team < G && item < n;
  const uint32_t shared = P.nconst * 12;
  uint32_t* my = lds + shared + (team < G ? team : 0) * lds_words;
  for (uint32_t k = threadIdx.x; k < shared; k += 64) lds[k] = P.consts[k];
  if (active)  // slot values below p: limbs with a small top word
    for (uint32_t s = lane; s < P.nslots; s += T)
      for (int j = 0; j < 12; ++j) my[12 * s + j] = j == 11 ? 0x01000000u + item + s : 0x9e3779b9u * (item + 7 * s + j + 1);
  __syncthreads();
  uint32_t* io_item = io + (size_t)(active ? item : 0) * io_words;
  const uint32_t R = P.rounds;
  uint64_t* tr = trace + (size_t)blockIdx.x * (R + 1);
  for (uint32_t r = 0; r < R; ++r) {
    if (threadIdx.x == 0) tr[r] = wall_clock64();
    const uint32_t h0 = __builtin_amdgcn_readfirstlane(P.hdr[4 * r]);
    const uint32_t off = __builtin_amdgcn_readfirstlane(P.hdr[4 * r + 1]);
    const uint32_t words = __builtin_amdgcn_readfirstlane(P.hdr[4 * r + 2]);
    if (active) lcv::sop_exec(h0, __builtin_amdgcn_readfirstlane(P.hdr[4 * r + 3]), P.rec + off + lane * words, lcv::sop_pre(h0, P.rec + off + lane * words), my, my, lds, P.nslots, io_item, io_item);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    tr[R] = wall_clock64();
    hwid[2 * blockIdx.x] = __builtin_amdgcn_s_getreg((31 << 11) | 4);       // HW_ID: wave, SIMD, CU, SH, SE
    hwid[2 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
  }
}

template <uint32_t T, uint32_t W>
void run(const Prog& pg) {
  auto up = [](const uint32_t* h, size_t n) {
    uint32_t* d;
    hipMalloc(&d, n * 4);
    hipMemcpy(d, h, n * 4, hipMemcpyHostToDevice);
    return d;
  };
  lcv::SopView P{up(pg.hdr, pg.nhdr), up(pg.rec, pg.nrec), up(pg.consts, pg.nconst * 12), pg.rounds, pg.slots,
                 pg.nconst};
  const uint32_t G = 64 / T, blocks = (pg.items + G - 1) / G, lds_words = pg.slots * 12 + 1;
  const size_t lds_bytes = 4 * (size_t)(pg.nconst * 12 + G * lds_words);
  uint32_t* io;
  hipMalloc(&io, (size_t)pg.items * pg.io_words * 4);
  hipMemset(io, 0, (size_t)pg.items * pg.io_words * 4);
  uint64_t* trace;
  const size_t tn = (size_t)blocks * (pg.rounds + 1);
  hipMalloc(&trace, tn * 8);
  uint32_t* hw;
  hipMalloc(&hw, (size_t)blocks * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((k_trace<T, W>), dim3(blocks), dim3(64), lds_bytes, 0, P, pg.items, lds_words, io, pg.io_words, trace, hw);
  hipDeviceSynchronize();
  hipEventRecord(a);
  hipLaunchKernelGGL((k_trace<T, W>), dim3(blocks), dim3(64), lds_bytes, 0, P, pg.items, lds_words, io, pg.io_words, trace, hw);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  std::vector<uint64_t> t(tn);
  hipMemcpy(t.data(), trace, tn * 8, hipMemcpyDeviceToHost);
  std::vector<double> per(pg.rounds, 0.0);
  double span = 0;
  for (uint32_t bk = 0; bk < blocks; ++bk) {
    const uint64_t* tb = t.data() + (size_t)bk * (pg.rounds + 1);
    for (uint32_t r = 0; r < pg.rounds; ++r) per[r] += (double)(tb[r + 1] - tb[r]) * 10.0 / blocks;  // ns
    span += (double)(tb[pg.rounds] - tb[0]) * 10.0 / blocks;
  }
  uint64_t s0 = ~0ull, s1 = 0, e0 = ~0ull, e1 = 0;
  for (uint32_t bk = 0; bk < blocks; ++bk) {
    const uint64_t* tb = t.data() + (size_t)bk * (pg.rounds + 1);
    s0 = std::min(s0, tb[0]); s1 = std::max(s1, tb[0]);
    e0 = std::min(e0, tb[pg.rounds]); e1 = std::max(e1, tb[pg.rounds]);
  }
  printf("== %s: team %u, %u items, %u blocks, %u rounds: kernel %.3f ms, mean block round span %.3f ms; "
         "first round starts over %.3f ms, last rounds end over %.3f ms, first start to last end %.3f ms\n",
         pg.name, T, pg.items, blocks, pg.rounds, ms, span * 1e-6, (s1 - s0) * 1e-5, (e1 - e0) * 1e-5,
         (e1 - s0) * 1e-5);
  {  // waves per SIMD (blocks are one wave) and the mean block span by that count
    std::vector<uint32_t> h(2 * (size_t)blocks);
    hipMemcpy(h.data(), hw, h.size() * 4, hipMemcpyDeviceToHost);
    std::map<uint64_t, int> per_simd;
    auto key = [&](uint32_t b) {
      const uint32_t id = h[2 * b], x = h[2 * b + 1] & 15u;
      const uint32_t simd = (id >> 4) & 3u, cu = (id >> 8) & 15u, sh = (id >> 12) & 1u, se = (id >> 13) & 7u;
      return ((uint64_t)x << 24) | (se << 16) | (sh << 12) | (cu << 4) | simd;
    };
    for (uint32_t b = 0; b < blocks; ++b) per_simd[key(b)]++;
    std::map<int, std::pair<int, double>> byw;
    std::map<uint32_t, int> cus;
    for (uint32_t b = 0; b < blocks; ++b) {
      const uint64_t* tb = t.data() + (size_t)b * (pg.rounds + 1);
      auto& e = byw[per_simd[key(b)]];
      e.first++;
      e.second += (double)(tb[pg.rounds] - tb[0]) * 1e-5;
      cus[(uint32_t)(key(b) >> 4)]++;
    }
    std::map<uint32_t, std::pair<int, double>> byx;
    std::vector<double> spans;
    for (uint32_t b = 0; b < blocks; ++b) {
      const uint64_t* tb = t.data() + (size_t)b * (pg.rounds + 1);
      const double sp = (double)(tb[pg.rounds] - tb[0]) * 1e-5;
      spans.push_back(sp);
      auto& e = byx[(uint32_t)(key(b) >> 24)];
      e.first++;
      e.second += sp;
    }
    std::sort(spans.begin(), spans.end());
    printf("  span percentiles (ms): p0 %.3f p10 %.3f p50 %.3f p90 %.3f p99 %.3f p100 %.3f; by XCC:", spans[0],
           spans[spans.size() / 10], spans[spans.size() / 2], spans[spans.size() * 9 / 10], spans[spans.size() * 99 / 100],
           spans.back());
    for (auto& kv : byx) printf(" %u: %.3f", kv.first, kv.second.second / kv.second.first);
    printf("\n");
    printf("  %zu SIMDs and %zu CUs used;", per_simd.size(), cus.size());
    for (auto& kv : byw) printf(" %d waves/SIMD: %d blocks, mean span %.3f ms;", kv.first, kv.second.first, kv.second.second / kv.second.first);
    printf("\n");
  }
  std::map<std::string, std::pair<int, double>> by;
  for (uint32_t r = 0; r < pg.rounds; ++r) {
    const uint32_t h0 = pg.hdr[4 * r];
    char key[128];
    snprintf(key, sizeof key, "K%2u add%u m%u x2%u y2%u red%2u%s%s%s%s used%2u", h0 & 15, (h0 >> 4) & 3, (h0 >> 6) & 1,
             (h0 >> 7) & 1, (h0 >> 8) & 1, (h0 >> 16) & 31, (h0 >> 10) & 1 ? " INV" : "", (h0 >> 11) & 1 ? " LOAD" : "",
             (h0 >> 12) & 1 ? " EMIT" : "", (h0 >> 13) & 1 ? " SHADOW" : "", h0 >> 24);
    auto& e = by[key];
    e.first += 1;
    e.second += per[r];
  }
  std::vector<std::pair<double, std::string>> rows;
  for (auto& kv : by) rows.push_back({kv.second.second, kv.first});
  std::sort(rows.rbegin(), rows.rend());
  for (auto& rw : rows) {
    const auto& e = by[rw.second];
    printf("  %-62s rounds %4d  total %8.1f us (%5.1f%%)  per round %7.2f us\n", rw.second.c_str(), e.first,
           e.second * 1e-3, 100.0 * e.second / span, e.second * 1e-3 / e.first);
  }
  std::vector<std::pair<double, uint32_t>> top;
  for (uint32_t r = 0; r < pg.rounds; ++r) top.push_back({per[r], r});
  std::sort(top.rbegin(), top.rend());
  printf("  top rounds:");
  for (int k = 0; k < 8 && k < (int)top.size(); ++k) printf(" r%u %.1fus", top[k].second, top[k].first * 1e-3);
  printf("\n");
  hipFree(io);
  hipFree(trace);
  hipFree(hw);
}

#define PROG(nm, N, items, iow)                                                                              \
  Prog{#nm, kSop_##nm##_hdr, kSop_##nm##_rec, kSop_##nm##_consts, sizeof(kSop_##nm##_hdr) / 4,              \
       sizeof(kSop_##nm##_rec) / 4, LCV_SOP_##N##_ROUNDS, LCV_SOP_##N##_SLOTS, LCV_SOP_##N##_NCONST,          \
       LCV_SOP_##N##_TEAM, items, iow}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 10000;
  const uint32_t line_words = 2 * 6 * LCV_SOP_LINES_NSTEPS * 12;
  run<LCV_SOP_LINES_TEAM, 3>(PROG(lines, LINES, n, line_words));
  run<LCV_SOP_MILLER_ACC_TEAM, 2>(PROG(miller_acc, MILLER_ACC, n, line_words));
  run<LCV_SOP_FEXP_TEAM, 2>(PROG(fexp, FEXP, n, 12));
  run<LCV_SOP_H2C_TEAM, 2>(PROG(h2c, H2C, n, 12));
  return 0;
}
