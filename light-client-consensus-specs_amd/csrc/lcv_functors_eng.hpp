// lcv_functors_eng.hpp — team functors of the generated pairing programs (lcv_engine.hpp); kept
// apart from lcv_functors.hpp so that only the engine unit and the driver depend on the programs.
#pragma once
#include "lcv_engine.hpp"
#include "lcv_functors.hpp"

// pairing programs on the team engine (lcv_engine.hpp); one team of TEAM lanes per update
struct F_eng_miller {
  static constexpr bool ENGINE = true;
  Work W; ProgView P;
  static constexpr uint32_t TEAM = LCV_PROG_MILLER_TEAM, LDS_WORDS = LCV_PROG_MILLER_SLOTS * 12,
                            SHARED_WORDS = LCV_PROG_MILLER_NCONST * 12;
  LCV_HD uint32_t rounds() const { return P.rounds + 2; }
  LCV_HD void operator()(uint32_t i, uint32_t lane, uint32_t r, uint32_t* lds, uint32_t* cl) const { item_miller_team(i, lane, r, lds, cl, P, W); }
};
struct F_eng_fexp {
  static constexpr bool ENGINE = true;
  Work W; ProgView P;
  static constexpr uint32_t TEAM = LCV_PROG_FEXP_TEAM, LDS_WORDS = LCV_PROG_FEXP_SLOTS * 12,
                            SHARED_WORDS = LCV_PROG_FEXP_NCONST * 12;
  LCV_HD uint32_t rounds() const { return P.rounds + 2; }
  LCV_HD void operator()(uint32_t i, uint32_t lane, uint32_t r, uint32_t* lds, uint32_t* cl) const { item_fexp_team(i, lane, r, lds, cl, P, W); }
};
struct F_eng_h2c {
  static constexpr bool ENGINE = true;
  Work W; ProgView P;
  static constexpr uint32_t TEAM = LCV_PROG_H2C_TEAM, LDS_WORDS = LCV_PROG_H2C_SLOTS * 12,
                            SHARED_WORDS = LCV_PROG_H2C_NCONST * 12;
  LCV_HD uint32_t rounds() const { return P.rounds + 2; }
  LCV_HD void operator()(uint32_t i, uint32_t lane, uint32_t r, uint32_t* lds, uint32_t* cl) const { item_h2c_team(i, lane, r, lds, cl, P, W); }
};
struct F_eng_g2sub {
  static constexpr bool ENGINE = true;
  Work W; ProgView P;
  static constexpr uint32_t TEAM = LCV_PROG_G2SUB_TEAM, LDS_WORDS = LCV_PROG_G2SUB_SLOTS * 12,
                            SHARED_WORDS = LCV_PROG_G2SUB_NCONST * 12;
  LCV_HD uint32_t rounds() const { return P.rounds + 2; }
  LCV_HD void operator()(uint32_t i, uint32_t lane, uint32_t r, uint32_t* lds, uint32_t* cl) const { item_g2sub_team(i, lane, r, lds, cl, P, W); }
};

#ifdef LCV_KERNEL_UNIT
// The engine's round loop (one wave per block, TEAM lanes per update): prologue (r = 0), the
// program's rounds, epilogue (r = rounds + 1).  Round r+1's lane record (two 16-byte loads) and
// header are loaded while round r executes; the header is wave-uniform (readfirstlane), so the
// interpreter's term loops and reductions branch on SGPRs.  Blocks are one wave, so the barrier
// between rounds is a wave barrier (LDS operations of one wave complete in order).
template <class F>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3))) void k_eng(F f, uint32_t n) {
  constexpr uint32_t T = F::TEAM, G = 64 / F::TEAM;
  static_assert(lcv::ENG_REC_WORDS == 8, "lane record = two 16-byte loads");
  __shared__ uint32_t lds[F::SHARED_WORDS + G * F::LDS_WORDS];
  const uint32_t team = threadIdx.x / T, lane = threadIdx.x % T;
  const uint32_t item = blockIdx.x * G + team;
  const bool active = team < G && item < n;
  uint32_t* my = lds + F::SHARED_WORDS + (team < G ? team : 0) * F::LDS_WORDS;
  const uint32_t R = f.P.rounds, ns = f.P.nslots;
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  typedef uint32_t u2 __attribute__((ext_vector_type(2)));
  typedef const __attribute__((address_space(1))) u4 g4;
  typedef const __attribute__((address_space(1))) u2 g2;
  g4* rec = (g4*)f.P.rec + 2 * lane;
  g2* hdr = (g2*)f.P.hdr;
  if (active) f(item, lane, 0u, my, lds);
  __syncthreads();
  u4 q0 = rec[0], q1 = rec[1];
  u2 h = hdr[0];
  for (uint32_t r = 0; r < R; ++r) {
    const uint32_t w[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
    const uint32_t h0 = __builtin_amdgcn_readfirstlane(h.x), h1 = __builtin_amdgcn_readfirstlane(h.y);
    if (r + 1 < R) {
      const size_t o = (size_t)(r + 1) * (2 * T);
      q0 = rec[o];
      q1 = rec[o + 1];
      h = hdr[r + 1];
    }
    if (active) lcv::eng_exec(w, h0, h1, my, lds, ns, 0u);
    __syncthreads();
  }
  if (active) f(item, lane, R + 1, my, lds);
}
#endif
