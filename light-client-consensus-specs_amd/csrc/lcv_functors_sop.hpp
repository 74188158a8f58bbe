// lcv_functors_sop.hpp — team functors of the SOP programs (lcv_sop.hpp, tools/gen_sop.py): the pairing
// check of bls.FastAggregateVerify (reference call site sync-protocol.md:464) as three kernels:
//   F_sop_lines  one team of LCV_SOP_LINES_TEAM lanes per (update, pairing): the T walk over |x|,
//                streaming the 68 sparse lines (a, b, c) of that pairing to W.lines (HBM, L2-resident);
//   F_sop_acc    one team of 12 lanes (one Fp coefficient each) per update: f <- f^2 l1 l2 per step,
//                the lines side-loaded one round ahead; output conj(f) to W.f;
//   F_sop_fexp   one team of 12 lanes per update: final exponentiation (result e^3) and "== 1".
#pragma once
#include "lcv_functors.hpp"
#include "lcv_sop.hpp"
#include "lcv_sop_programs.inc"
#if defined(LCV_KERNEL_UNIT)
#include "lcv_sop_fan.hpp"
#include "lcv_sop_row.hpp"
#endif
// the fan engine's lanes per product (lcv_sop_fan.hpp; also known to lcv_launch.hpp): 3 = Karatsuba parts split
#ifndef LCV_FAN_SPLIT
#define LCV_FAN_SPLIT 1
#endif
#ifndef LCV_FAN_PARTS
#define LCV_FAN_PARTS (LCV_FAN_SPLIT ? 3u : 1u)
#endif

enum { SOP_LINE_VALS = 6 * LCV_SOP_LINES_NSTEPS, SOP_LINE_WORDS = 2 * SOP_LINE_VALS * 12 };
// W.lines: item i's two pairings' line values (pairing k at + k * SOP_LINE_VALS * 12 words)
LCV_HDFN size_t lines_index(size_t i) { return i * (size_t)SOP_LINE_WORDS; }
// per-item LDS pitch = 12 * slots + SOP_PITCH_PAD words: 4 keeps every value 16-byte aligned for the
// b128 LDS accesses (LCV_SOP_B128, lcv_sop.hpp); 1 (odd) staggers the teams' banks for 32-bit accesses
enum { SOP_PITCH_PAD = LCV_SOP_B128 ? 4 : 1 };

// Round 2 padded the pitch to an odd word count so the teams of a wave start on different LDS banks for
// 32-bit accesses (a bank model: 1.3-1.4x the conflict-free LDS cycles instead of 2.7-3.4x); since r03
// v13 the pitch is 4 mod 8 words and values move as 16-byte accesses, three instead of six LDS
// instructions per value: 1.448 -> 1.472 M updates/s in a same-box A/B (profiles/r03_v13)
// the SOP kernels' VGPR budget in waves per SIMD (3 = 168 VGPRs, no spills; an experiment knob)
#ifndef LCV_SOP_WAVES
#define LCV_SOP_WAVES 3
#endif
struct F_sop_lines {
  Work W; SopView P;
  uint32_t mode;  // 0: items t = 2i + k (both pairings); 1: t = i, k = 1 (signature); 2: t = i, k = 0 (message)
  static constexpr uint32_t WAVES = LCV_SOP_WAVES;  // waves per SIMD the kernel's VGPR budget targets
  static constexpr uint32_t MAXK = LCV_SOP_LINES_MAXK;  // the fan engine's lanes per op
  static constexpr uint32_t FAN_PARTS = LCV_FAN_PARTS;    // the fan engine's lanes per product
  static constexpr uint32_t TEAM = LCV_SOP_LINES_TEAM, LDS_WORDS = LCV_SOP_LINES_SLOTS * 12 + SOP_PITCH_PAD,
                            SHARED_WORDS = LCV_SOP_LINES_NCONST * 12;
  // pairing k of update i: k = 0 e(PK_agg, H(m)), k = 1 e(-G1, signature)
  LCV_HD uint32_t upd(uint32_t t) const { return mode == 0 ? t >> 1 : t; }
  LCV_HD uint32_t pk(uint32_t t) const { return mode == 0 ? (t & 1u) : (mode == 1 ? 1u : 0u); }
  LCV_HD const uint32_t* io_in(uint32_t) const { return nullptr; }
  LCV_HD uint32_t* io_out(uint32_t t) const {
    return W.lines + lines_index(upd(t)) + (size_t)pk(t) * SOP_LINE_VALS * 12;
  }
  // T = (Qx, Qy, 1), Q affine; (-xP, yP).  An identity Q becomes (G2 generator, P = (0, 0)): constant
  // lines, killed by the final exponentiation (e(P, O) = 1).
  LCV_HD void prologue(uint32_t t, uint32_t lane, uint32_t* lds) const {
    const uint32_t i = upd(t), k = pk(t);
    const bool id = k == 0 ? W.qh_inf[i] != 0 : W.sig_status[i] != PT_OK;
    for (uint32_t v = lane; v < 12; v += TEAM) {
      fp x;
      uint32_t slot;
      if (v < 8) {  // qx0 qx1 qy0 qy1, then the same into tx0 tx1 ty0 ty1
        const uint32_t c = v & 3u;
        if (id) {
          fp2 g;
          if (c < 2) LCV_FP2_SET(g, LCV_G2X);
          else LCV_FP2_SET(g, LCV_G2Y);
          x = (c & 1u) ? g.c1 : g.c0;
        } else {
          soa_ld_fp(x, k == 0 ? W.qh : W.qs, W.cap, i, c);
        }
        constexpr uint32_t QS[4] = {LCV_SOP_LINES_SLOT_QX0, LCV_SOP_LINES_SLOT_QX1, LCV_SOP_LINES_SLOT_QY0,
                                    LCV_SOP_LINES_SLOT_QY1};
        constexpr uint32_t TS[4] = {LCV_SOP_LINES_SLOT_TX0, LCV_SOP_LINES_SLOT_TX1, LCV_SOP_LINES_SLOT_TY0,
                                    LCV_SOP_LINES_SLOT_TY1};
        slot = v < 4 ? QS[c] : TS[c];
      } else if (v < 10) {  // tz = (1, 0)
        if (v == 8) fp_one(x);
        else fp_zero(x);
        slot = v == 8 ? LCV_SOP_LINES_SLOT_TZ0 : LCV_SOP_LINES_SLOT_TZ1;
      } else {  // nxP, yP
        if (k == 0) {
          soa_ld_fp(x, W.pk, W.cap, i, v - 10);
          if (v == 10) fp_neg(x, x);
        } else if (v == 10) {
          LCV_FP_SET(x, LCV_G1X_INIT);
          fp_neg(x, x);
        } else {
          LCV_FP_SET(x, LCV_G1NEGY_INIT);
        }
        if (id) fp_zero(x);
        slot = v == 10 ? LCV_SOP_LINES_SLOT_NXP : LCV_SOP_LINES_SLOT_YP;
      }
      LCV_UNROLL for (int j = 0; j < 12; ++j) lds[12 * slot + j] = x.v[j];
    }
  }
  // the signature pairing's walk ends at T = [|x|]Q: the G2 subgroup check of the signature
  // (psi(Q) == [x]Q, program rounds e1/e2) turns PT_OK into PT_BAD for a non-member
  LCV_HD void epilogue(uint32_t t, uint32_t lane, const uint32_t* lds) const {
    if (lane != 0 || pk(t) != 1u) return;
    const uint32_t i = upd(t);
    if (W.sig_status[i] != PT_OK) return;
    uint32_t e = 0, z = 0;
    for (int j = 0; j < 12; ++j) {
      e |= lds[12 * LCV_SOP_LINES_SLOT_E10 + j] | lds[12 * LCV_SOP_LINES_SLOT_E11 + j] |
           lds[12 * LCV_SOP_LINES_SLOT_E20 + j] | lds[12 * LCV_SOP_LINES_SLOT_E21 + j];
      z |= lds[12 * LCV_SOP_LINES_SLOT_TZ0 + j] | lds[12 * LCV_SOP_LINES_SLOT_TZ1 + j];
    }
    if (e != 0 || z == 0) W.sig_status[i] = PT_BAD;
  }
};

struct F_sop_acc {
  Work W; SopView P;
  static constexpr uint32_t WAVES = LCV_SOP_WAVES;  // waves per SIMD the kernel's VGPR budget targets
  static constexpr uint32_t MAXK = LCV_SOP_MILLER_ACC_MAXK;  // the fan engine's lanes per op
  static constexpr uint32_t FAN_PARTS = LCV_FAN_PARTS;         // the fan engine's lanes per product
  static constexpr uint32_t TEAM = LCV_SOP_MILLER_ACC_TEAM, LDS_WORDS = LCV_SOP_MILLER_ACC_SLOTS * 12 + SOP_PITCH_PAD,
                            SHARED_WORDS = LCV_SOP_MILLER_ACC_NCONST * 12;
  static_assert(LCV_SOP_MILLER_ACC_SLOT_F0_0 == 0 && LCV_SOP_MILLER_ACC_SLOT_F5_1 == 11, "f in slots 0..11");
  LCV_HD const uint32_t* io_in(uint32_t i) const { return W.lines + lines_index(i); }
  LCV_HD uint32_t* io_out(uint32_t) const { return nullptr; }
  // lane l handles the Fp12 coefficients l, l + TEAM, ... (any team size)
  LCV_HD void prologue(uint32_t, uint32_t lane, uint32_t* lds) const {  // f = 1
    for (uint32_t s = lane; s < 12; s += TEAM) {
      fp x;
      if (s == 0) fp_one(x);
      else fp_zero(x);
      LCV_UNROLL for (int j = 0; j < 12; ++j) lds[12 * s + j] = x.v[j];
    }
  }
  LCV_HD void epilogue(uint32_t i, uint32_t lane, const uint32_t* lds) const {  // slot 2g + c -> W.f
    for (uint32_t s = lane; s < 12; s += TEAM) {
      uint32_t x[12];
      LCV_UNROLL for (int j = 0; j < 12; ++j) x[j] = lds[12 * s + j];
      f12_st_coeff(W.f, i, s, x);
    }
  }
};

// Latency mode's Miller loop as one program (tools/gen_sop.py miller_program): both pairings' walks
// (slots m_* for e(PK_agg, H(m)), s_* for e(-G1, signature) with its G2 subgroup check) beside the
// accumulation, one step behind, the lines passing through LDS; fan engine only (one update per block,
// one lane per product: its K = 7 accumulation rounds would fill 11 waves with split products)
struct F_sop_miller {
  Work W; SopView P;
  static constexpr uint32_t MAXK = LCV_SOP_MILLER_MAXK;
  static constexpr uint32_t FAN_PARTS = 1;
  static constexpr uint32_t TEAM = LCV_SOP_MILLER_TEAM, LDS_WORDS = LCV_SOP_MILLER_SLOTS * 12 + SOP_PITCH_PAD,
                            SHARED_WORDS = LCV_SOP_MILLER_NCONST * 12;
  static_assert(LCV_SOP_MILLER_SLOT_F0_0 == 0 && LCV_SOP_MILLER_SLOT_F5_1 == 11, "f in slots 0..11");
  LCV_HD const uint32_t* io_in(uint32_t) const { return nullptr; }
  LCV_HD uint32_t* io_out(uint32_t) const { return nullptr; }
  // 36 values: each walk's Q, T = (Q, 1) and (-xP, yP) as F_sop_lines' prologue, then f = 1
  LCV_HD void prologue(uint32_t i, uint32_t lane, uint32_t* lds) const {
    constexpr uint32_t QS[2][4] = {{LCV_SOP_MILLER_SLOT_M_QX0, LCV_SOP_MILLER_SLOT_M_QX1, LCV_SOP_MILLER_SLOT_M_QY0,
                                    LCV_SOP_MILLER_SLOT_M_QY1},
                                   {LCV_SOP_MILLER_SLOT_S_QX0, LCV_SOP_MILLER_SLOT_S_QX1, LCV_SOP_MILLER_SLOT_S_QY0,
                                    LCV_SOP_MILLER_SLOT_S_QY1}};
    constexpr uint32_t TS[2][6] = {{LCV_SOP_MILLER_SLOT_M_TX0, LCV_SOP_MILLER_SLOT_M_TX1, LCV_SOP_MILLER_SLOT_M_TY0,
                                    LCV_SOP_MILLER_SLOT_M_TY1, LCV_SOP_MILLER_SLOT_M_TZ0, LCV_SOP_MILLER_SLOT_M_TZ1},
                                   {LCV_SOP_MILLER_SLOT_S_TX0, LCV_SOP_MILLER_SLOT_S_TX1, LCV_SOP_MILLER_SLOT_S_TY0,
                                    LCV_SOP_MILLER_SLOT_S_TY1, LCV_SOP_MILLER_SLOT_S_TZ0, LCV_SOP_MILLER_SLOT_S_TZ1}};
    constexpr uint32_t PS[2][2] = {{LCV_SOP_MILLER_SLOT_M_NXP, LCV_SOP_MILLER_SLOT_M_YP},
                                   {LCV_SOP_MILLER_SLOT_S_NXP, LCV_SOP_MILLER_SLOT_S_YP}};
    for (uint32_t u = lane; u < 36; u += TEAM) {
      fp x;
      uint32_t slot;
      if (u < 24) {
        const uint32_t k = u / 12, v = u % 12;
        const bool id = k == 0 ? W.qh_inf[i] != 0 : W.sig_status[i] != PT_OK;
        if (v < 8) {
          const uint32_t c = v & 3u;
          if (id) {
            fp2 g;
            if (c < 2) LCV_FP2_SET(g, LCV_G2X);
            else LCV_FP2_SET(g, LCV_G2Y);
            x = (c & 1u) ? g.c1 : g.c0;
          } else {
            soa_ld_fp(x, k == 0 ? W.qh : W.qs, W.cap, i, c);
          }
          slot = v < 4 ? QS[k][c] : TS[k][c];
        } else if (v < 10) {
          if (v == 8) fp_one(x);
          else fp_zero(x);
          slot = TS[k][v - 4];
        } else {
          if (k == 0) {
            soa_ld_fp(x, W.pk, W.cap, i, v - 10);
            if (v == 10) fp_neg(x, x);
          } else if (v == 10) {
            LCV_FP_SET(x, LCV_G1X_INIT);
            fp_neg(x, x);
          } else {
            LCV_FP_SET(x, LCV_G1NEGY_INIT);
          }
          if (id) fp_zero(x);
          slot = PS[k][v - 10];
        }
      } else {
        slot = u - 24;  // f = 1
        if (slot == 0) fp_one(x);
        else fp_zero(x);
      }
      LCV_UNROLL for (int j = 0; j < 12; ++j) lds[12 * slot + j] = x.v[j];
    }
  }
  // f -> W.f (as F_sop_acc), and the signature's G2 subgroup check (as F_sop_lines)
  LCV_HD void epilogue(uint32_t i, uint32_t lane, const uint32_t* lds) const {
    for (uint32_t s = lane; s < 12; s += TEAM) {
      uint32_t x[12];
      LCV_UNROLL for (int j = 0; j < 12; ++j) x[j] = lds[12 * s + j];
      f12_st_coeff(W.f, i, s, x);
    }
    if (lane != 0 || W.sig_status[i] != PT_OK) return;
    uint32_t e = 0, z = 0;
    for (int j = 0; j < 12; ++j) {
      e |= lds[12 * LCV_SOP_MILLER_SLOT_S_E10 + j] | lds[12 * LCV_SOP_MILLER_SLOT_S_E11 + j] |
           lds[12 * LCV_SOP_MILLER_SLOT_S_E20 + j] | lds[12 * LCV_SOP_MILLER_SLOT_S_E21 + j];
      z |= lds[12 * LCV_SOP_MILLER_SLOT_S_TZ0 + j] | lds[12 * LCV_SOP_MILLER_SLOT_S_TZ1 + j];
    }
    if (e != 0 || z == 0) W.sig_status[i] = PT_BAD;
  }
};

struct F_sop_fexp {
  Work W; SopView P;
  static constexpr uint32_t WAVES = LCV_SOP_WAVES;  // waves per SIMD the kernel's VGPR budget targets
  static constexpr uint32_t MAXK = LCV_SOP_FEXP_MAXK;  // the fan engine's lanes per op
  static constexpr uint32_t FAN_PARTS = LCV_FAN_PARTS;   // the fan engine's lanes per product
  static constexpr uint32_t TEAM = LCV_SOP_FEXP_TEAM, LDS_WORDS = LCV_SOP_FEXP_SLOTS * 12 + SOP_PITCH_PAD,
                            SHARED_WORDS = LCV_SOP_FEXP_NCONST * 12;
  static_assert(LCV_SOP_FEXP_SLOT_F0_0 == 0 && LCV_SOP_FEXP_SLOT_F5_1 == 11, "f in slots 0..11");
  // the result's 12 coefficients (slot order 2 g + c; the generator places them anywhere)
  static constexpr uint32_t RS[12] = {LCV_SOP_FEXP_SLOT_R0_0, LCV_SOP_FEXP_SLOT_R0_1, LCV_SOP_FEXP_SLOT_R1_0,
                                      LCV_SOP_FEXP_SLOT_R1_1, LCV_SOP_FEXP_SLOT_R2_0, LCV_SOP_FEXP_SLOT_R2_1,
                                      LCV_SOP_FEXP_SLOT_R3_0, LCV_SOP_FEXP_SLOT_R3_1, LCV_SOP_FEXP_SLOT_R4_0,
                                      LCV_SOP_FEXP_SLOT_R4_1, LCV_SOP_FEXP_SLOT_R5_0, LCV_SOP_FEXP_SLOT_R5_1};
  LCV_HD const uint32_t* io_in(uint32_t) const { return nullptr; }
  LCV_HD uint32_t* io_out(uint32_t) const { return nullptr; }
  LCV_HD void prologue(uint32_t i, uint32_t lane, uint32_t* lds) const {
    for (uint32_t s = lane; s < 12; s += TEAM) {
      uint32_t x[12];
      f12_ld_coeff(x, W.f, i, s);
      LCV_UNROLL for (int j = 0; j < 12; ++j) lds[12 * s + j] = x[j];
    }
  }
  // the pairing value (e^3) to W.f; "== 1" to W.pair_ok
  LCV_HD void epilogue(uint32_t i, uint32_t lane, const uint32_t* lds) const {
    for (uint32_t s = lane; s < 12; s += TEAM) {
      uint32_t x[12];
      LCV_UNROLL for (int j = 0; j < 12; ++j) x[j] = lds[12 * RS[s] + j];
      f12_st_coeff(W.f, i, s, x);
    }
    if (lane == 0) {
      fp x, one;
      LCV_UNROLL for (int j = 0; j < 12; ++j) x.v[j] = lds[12 * RS[0] + j];
      fp_one(one);
      bool ok = fp_eq(x, one);
      for (uint32_t k = 1; k < 12; ++k) {
        uint32_t z = 0;
        for (int j = 0; j < 12; ++j) z |= lds[12 * RS[k] + j];
        ok = ok && z == 0;
      }
      W.pair_ok[i] = ok ? 1 : 0;
    }
  }
};

// hash_to_G2 tail after the two SSWU maps (W.qmap): isogeny, addition, cofactor clearing (complete
// formulas), affine H(m) -> W.qh and its identity flag -> W.qh_inf
struct F_sop_h2c {
  Work W; SopView P;
  static constexpr uint32_t WAVES = LCV_SOP_WAVES;  // waves per SIMD the kernel's VGPR budget targets
  static constexpr uint32_t MAXK = LCV_SOP_H2C_MAXK;  // the fan engine's lanes per op
  static constexpr uint32_t FAN_PARTS = LCV_FAN_PARTS;  // the fan engine's lanes per product
  static constexpr uint32_t TEAM = LCV_SOP_H2C_TEAM, LDS_WORDS = LCV_SOP_H2C_SLOTS * 12 + SOP_PITCH_PAD,
                            SHARED_WORDS = LCV_SOP_H2C_NCONST * 12;
  static_assert(LCV_SOP_H2C_SLOT_M0X0 == 0 && LCV_SOP_H2C_SLOT_M1Y1 == 7, "SSWU points in slots 0..7");
  static_assert(LCV_SOP_H2C_SLOT_HY1 == LCV_SOP_H2C_SLOT_HX0 + 3, "hx, hy in consecutive slots");
  LCV_HD const uint32_t* io_in(uint32_t) const { return nullptr; }
  LCV_HD uint32_t* io_out(uint32_t) const { return nullptr; }
  LCV_HD void prologue(uint32_t i, uint32_t lane, uint32_t* lds) const {
    for (uint32_t v = lane; v < 8; v += TEAM) {
      fp x;
      soa_ld_fp(x, W.qmap, W.cap, i, v);
      LCV_UNROLL for (int j = 0; j < 12; ++j) lds[12 * v + j] = x.v[j];
    }
  }
  LCV_HD void epilogue(uint32_t i, uint32_t lane, const uint32_t* lds) const {
    if (lane < 4) {
      fp x;
      LCV_UNROLL for (int j = 0; j < 12; ++j) x.v[j] = lds[12 * (LCV_SOP_H2C_SLOT_HX0 + lane) + j];
      soa_st_fp(W.qh, W.cap, i, lane, x);
    } else if (lane == 4) {
      uint32_t z = 0;
      for (int j = 0; j < 12; ++j) z |= lds[12 * LCV_SOP_H2C_SLOT_HZ0 + j] | lds[12 * LCV_SOP_H2C_SLOT_HZ1 + j];
      W.qh_inf[i] = z == 0 ? 1 : 0;
    }
  }
};

#ifdef LCV_KERNEL_UNIT
// The SOP round loop: one wave per block, g <= 64 / TEAM teams (items) per wave, lanes past the last
// team idle.  The round header is wave-uniform (scalar loads); each lane reads its record from global
// memory (L2-resident program).  Blocks are one wave, so the barrier between rounds is a wave barrier.
template <class F>
// LDS is dynamic (sized at launch): with a static size the compiler derives its occupancy target from
// a smaller LDS than gfx950's 160 KB and gives the kernel 256 VGPRs (2 waves/SIMD).
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(F::WAVES))) void k_sop(F f, uint32_t n, uint32_t g) {
  constexpr uint32_t T = F::TEAM, G = 64 / F::TEAM;
  if (g == 0 || g > G) g = G;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];  // 16-byte aligned values (LCV_SOP_B128)
  const uint32_t team = threadIdx.x / T, lane = threadIdx.x % T;
  const uint32_t item = blockIdx.x * g + team;
  const bool active = team < g && item < n;
  // LDS: the program's constants, the q p table of the reductions (lcv::sop_reduce), the items' slots
  static_assert(lcv::SOP_QP_WORDS == LCV_SOP_QP_WORDS, "k_sop's LDS size (lcv_launch.hpp)");
  uint32_t* qp = lds + F::SHARED_WORDS;
  uint32_t* my = qp + lcv::SOP_QP_WORDS + (team < g ? team : 0) * F::LDS_WORDS;
  for (uint32_t k = threadIdx.x; k < F::SHARED_WORDS; k += 64) lds[k] = f.P.consts[k];
  if (threadIdx.x < lcv::SOP_QP_N) lcv::sop_qp_entry(qp + 16 * threadIdx.x, threadIdx.x);
  if (active) f.prologue(item, lane, my);
  __syncthreads();
  const uint32_t* io_in = active ? f.io_in(item) : nullptr;
  uint32_t* io_out = active ? f.io_out(item) : nullptr;
  const uint32_t R = f.P.rounds, ns = f.P.nslots;
  // round r + 1's header and the lane's first record words are loaded at the top of round r
  // (lcv::sop_pre), so their latency overlaps round r's products instead of opening round r + 1
  uint32_t h0 = 0, h3 = 0;
  const uint32_t* wn = f.P.rec;
  lcv::SopPre pre{0, 0, 0, 0, 0};
  if (R) {
    h0 = __builtin_amdgcn_readfirstlane(f.P.hdr[0]);
    const uint32_t off = __builtin_amdgcn_readfirstlane(f.P.hdr[1]);
    const uint32_t words = __builtin_amdgcn_readfirstlane(f.P.hdr[2]);
    h3 = __builtin_amdgcn_readfirstlane(f.P.hdr[3]);
    wn = f.P.rec + off + lane * words;
    if (active) pre = lcv::sop_pre(h0, wn);
  }
  for (uint32_t r = 0; r < R; ++r) {
    const uint32_t ch0 = h0, ch3 = h3;
    const uint32_t* w = wn;  // this round's record (its address computed once, a round ahead)
    const lcv::SopPre cur = pre;
    if (r + 1 < R) {
      h0 = __builtin_amdgcn_readfirstlane(f.P.hdr[4 * r + 4]);
      const uint32_t off = __builtin_amdgcn_readfirstlane(f.P.hdr[4 * r + 5]);
      const uint32_t words = __builtin_amdgcn_readfirstlane(f.P.hdr[4 * r + 6]);
      h3 = __builtin_amdgcn_readfirstlane(f.P.hdr[4 * r + 7]);
      wn = f.P.rec + off + lane * words;
      if (active) pre = lcv::sop_pre(h0, wn);
    }
    if (active) lcv::sop_exec(ch0, ch3, w, cur, my, my, lds, ns, io_in, io_out, qp);
    __syncthreads();
  }
  if (active) f.epilogue(item, lane, my);
}

// The fan engine's round loop (lcv_sop_fan.hpp; latency mode): ONE item per block of TEAM x MAXK x S lanes
// (S = LCV_FAN_PARTS, 3 when the products' Karatsuba parts are split; lcv_hip_launch_sop_fan sizes it to
// whole waves), lane (k S + part) TEAM + o computes part `part` of product k of op o, so the ops'
// product-0 part-0 lanes — which also run the reductions and tails — are lanes 0 .. TEAM - 1 of the first
// wave, whose lockstep orders every tail's reads before any store; a round of K products keeps its
// K x S x TEAM busy lanes in the first waves.  The products' columns meet in the op's 28-column LDS
// accumulator by 64-bit LDS atomic adds (ds_add_u64); the op's tail lane reads the sums and zeroes the
// accumulator for the next round.  Two block barriers per round: after the products (the sums are
// complete) and after the stores (the next round reads them).
// LCV_FAN_X_TIMING (experiments only): per-phase clock sums of the first and the last wave, printed.
#ifndef LCV_FAN_X_TIMING
#define LCV_FAN_X_TIMING 0
#endif
#ifndef LCV_FAN_FLAT_COLS
#define LCV_FAN_FLAT_COLS 1
#endif
#ifndef LCV_FAN_FLAT_FETCH
#define LCV_FAN_FLAT_FETCH 1
#endif
#ifndef LCV_FAN_LATE_FETCH
#define LCV_FAN_LATE_FETCH 1
#endif
#ifndef LCV_FAN_X_NOATOMIC
#define LCV_FAN_X_NOATOMIC 0
#endif
// LCV_FAN_ROW (lcv_launch.hpp, the default) for the programs of at most LCV_FAN_ROW_MAX_TEAM ops a round
// (lcv_fan_rows<F>: the final exponentiation and hash_to_G2's tail): op o's tail runs on the 16-lane row of lanes
// 16 o .. 16 o + 15 (lcv_sop_row.hpp: the reduction as two column passes, one column pair per lane; the add-ins,
// the quotient step and the store with a limb or word per lane), instead of on one lane of the first wave.  The
// tails then sit in several waves, so a row reads its add-in terms at the top of the round, before any tail of
// the round stores (ops update slots in place).  Inversion, side-load and emit rounds gather the value on the
// row's lane 0, which runs the inversion flag and sop_tail_store as the one-lane tail does.
template <class F>
__global__ __launch_bounds__(lcv_fan_threads<F>()) void k_sop_fan(F f, uint32_t n) {
  constexpr uint32_t T = F::TEAM, KM = F::MAXK, S = F::FAN_PARTS, NT = lcv_fan_threads<F>();
  constexpr bool ROWS = lcv_fan_rows<F>();
  constexpr uint32_t ITEM_WORDS = (F::LDS_WORDS + 1u) & ~1u;  // 8-byte aligned scratch after the slots
  static_assert(T <= 64, "every op's tail lane in the first wave");
  static_assert(S == 1 || S == 3, "one lane per product, or one per Karatsuba part");
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t L = threadIdx.x, k = L / (S * T), part = (L / T) % S, o = L % T;
  const uint32_t item = blockIdx.x;
  const bool active = k < KM && item < n;
  uint32_t* qp = lds + F::SHARED_WORDS;
  uint32_t* my = qp + lcv::SOP_QP_WORDS;
  uint64_t* acc = (uint64_t*)(my + ITEM_WORDS) + (size_t)o * lcv::FAN_COLS;  // op o's column accumulator
  for (uint32_t x = L; x < F::SHARED_WORDS; x += NT) lds[x] = f.P.consts[x];
  if (L < lcv::SOP_QP_N) lcv::sop_qp_entry(qp + 16 * L, L);
  if (L < T) LCV_UNROLL for (int c = 0; c < 28; ++c) acc[c] = 0;
  if (L < T && item < n) f.prologue(item, L, my);
  __syncthreads();
  const uint32_t* io_in = item < n ? f.io_in(item) : nullptr;
  uint32_t* io_out = item < n ? f.io_out(item) : nullptr;
  const uint32_t R = f.P.rounds, ns = f.P.nslots;
  const lcv::SopBase base{my, lds, (int32_t)((const char*)lds - (const char*)my)};
  // the tail's op and lane: op L >> 4 on its row's lane 0 (ROWS), else op L on lane L < T
  const uint32_t orow = L >> 4;
  const bool rowact = ROWS && orow < T && item < n;
  const uint32_t to = ROWS ? orow : o;
  const bool tail_lane = ROWS ? rowact && (L & 15u) == 0u : L < T && item < n;
  uint64_t* racc = (uint64_t*)(my + ITEM_WORDS) + (size_t)(orow < T ? orow : 0u) * lcv::FAN_COLS;
  lcv::RowTabs rtabs;
  if constexpr (ROWS) lcv::rw_tabs(rtabs);
  // round r + 1's header and this lane's record words (its product's operand pair and scale; the tail's dst / io
  // words; a row's dst, shadow and add-in words) are loaded at the top of round r, so their latency overlaps
  // round r's work
  // The round headers come one round earlier still (round r + 2's at the top of round r), through vector loads
  // (an opaque zero lane offset keeps them off the scalar path), so the record addresses of round r + 1 do not
  // wait on a header load: the vector loads of a wave complete in order, and a header's is older than the
  // record loads of the round before it.
  struct Hdr { uint32_t h0, off, words, h3; };
  auto load_hdr = [&](uint32_t r) {
    uint32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    const uint32_t* p = f.P.hdr + 4 * r + z;
    return Hdr{p[0], p[1], p[2], p[3]};
  };
  struct Rec { uint32_t h0, h3, x, y, m; lcv::SopPre pre; const uint32_t* w; uint32_t a0, a1, d0, d1; };
  auto fetch = [&](const Hdr& hd) {
    Rec c;
    c.h0 = __builtin_amdgcn_readfirstlane(hd.h0);
    const uint32_t off = __builtin_amdgcn_readfirstlane(hd.off);
    const uint32_t words = __builtin_amdgcn_readfirstlane(hd.words);
    c.h3 = __builtin_amdgcn_readfirstlane(hd.h3);
    c.w = f.P.rec + off + __umul24(o, words);  // (o < 64, words < 2^10: the full-rate 24-bit multiply)
    const uint32_t* wt = f.P.rec + off + __umul24(to < T ? to : 0u, words);  // the tail's op's record
    const uint32_t K = c.h0 & 15u;
#if LCV_FAN_FLAT_FETCH
    // branch-free: every lane loads (a lone wave pays each exec-mask region and branch in series).  Product k is
    // clamped into op o's record (4 + 3 K words: its first words when K = 0); the values are used only by the lanes
    // they belong to (active, k < K; a row's add-in words only when the header counts them)
    const uint32_t kk = k < K ? k : (K ? K - 1u : 0u);
    const uint32_t* pw = c.w + (K ? 4u + 3u * kk : 0u);
    c.x = pw[0]; c.y = pw[1]; c.m = pw[2];
    c.pre = lcv::SopPre{0, 0, 0, 0, 0};
    if (!ROWS && tail_lane) c.pre = lcv::sop_pre(c.h0, wt);
    c.d0 = c.d1 = c.a0 = c.a1 = 0;
    if constexpr (ROWS) {
      c.d0 = wt[0]; c.d1 = wt[1]; c.a0 = wt[2]; c.a1 = wt[3];
    }
#else
    c.x = c.y = c.m = 0;
    if (active && k < K) {
      const uint32_t* pw = c.w + 4 + 3 * k;
      c.x = pw[0]; c.y = pw[1]; c.m = pw[2];
    }
    c.pre = lcv::SopPre{0, 0, 0, 0, 0};
    c.a0 = c.a1 = c.d0 = c.d1 = 0;
    if (tail_lane && !ROWS) c.pre = lcv::sop_pre(c.h0, wt);  // (rows: the dst / io words are d0 / d1 below)
    if (rowact) {
      const uint32_t nadd = (c.h0 >> 4) & 3u;
      c.d0 = wt[0];
      c.d1 = wt[1];
      if (nadd > 0) c.a0 = wt[2];
      if (nadd > 1) c.a1 = wt[3];
    }
#endif
    return c;
  };
  Hdr hn = load_hdr(0);
  Rec nx = fetch(hn);
  if (R > 1) hn = load_hdr(1);
#if LCV_FAN_X_TIMING
  uint64_t tq[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, tp = clock64();
#define LCV_FAN_T(i) do { const uint64_t tn = clock64(); tq[i] += tn - tp; tp = tn; } while (0)
#else
#define LCV_FAN_T(i) ((void)0)
#endif
  // round r reads its record `cur` and fetches round r + 1's into `nxr` (unconditionally: past the last round it
  // re-reads the last round's record).  The loop runs two rounds a trip with the two records swapping roles, so
  // no record is copied at the back edge: such a copy waits on the record's loads, issued only a round earlier
  auto prefetch = [&](uint32_t r, Rec& nxr) {
    nxr = fetch(hn);
    hn = load_hdr(r + 2 < R ? r + 2 : R - 1);
  };
  auto round = [&](const uint32_t r, const Rec& cur, Rec& nxr) __attribute__((always_inline)) {
    if (!LCV_FAN_LATE_FETCH) prefetch(r, nxr);
    const uint32_t h0 = cur.h0, K = h0 & 15u;
    LCV_FAN_T(0);
    if (active && k < K) {
      if constexpr (S == 3) {
      int64_t c13[13];
      lcv::sop_fan_part(c13, cur.x, cur.y, cur.m, k, cur.h3, (h0 >> 6) & 1u, part, base);
      const uint32_t at = part == 0 ? 0u : (part == 1 ? 14u : 7u);
#if LCV_FAN_X_NOATOMIC  // timing experiment only (wrong results): one atomic per lane instead of 13 or 26
      { uint64_t xs = 0; LCV_UNROLL for (int c = 0; c < 13; ++c) xs ^= (uint64_t)c13[c];
        __hip_atomic_fetch_add(acc + at, xs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
      if (false)
#endif
      LCV_UNROLL for (int c = 0; c < 13; ++c)
        __hip_atomic_fetch_add(acc + at + c, (uint64_t)c13[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (part != 2 && !LCV_FAN_X_NOATOMIC)
        LCV_UNROLL for (int c = 0; c < 13; ++c)
          __hip_atomic_fetch_add(acc + 7 + c, (uint64_t)c13[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else {
      uint64_t col[28];
      lcv::sop_fan_product(col, cur.x, cur.y, cur.m, k, cur.h3, (h0 >> 6) & 1u, base);
      LCV_UNROLL for (int c = 0; c < 28; ++c) __hip_atomic_fetch_add(acc + c, col[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    // a row's add-in terms are read now (the two words holding a lane's limb): after the products' operand reads and
    // before the barrier, so before any tail of this round stores; the limbs are cut out in the tail
    uint32_t tw[4] = {0, 0, 0, 0};
    if (rowact) {
      const uint32_t nadd = (h0 >> 4) & 3u;
      if (nadd > 0) lcv::rw_limb_words(lcv::sop_src(cur.a0 & 0xFFFu, my, lds, ns), tw[0], tw[1]);
      if (nadd > 1) lcv::rw_limb_words(lcv::sop_src(cur.a1 & 0xFFFu, my, lds, ns), tw[2], tw[3]);
    }
    // LCV_FAN_LATE_FETCH: round r + 1's record loads (and round r + 2's header) are issued here, while the column
    // atomics drain before the barrier (it waits on LDS only), instead of at the top of the round, where a lone wave
    // pays their issue in series with its products; they are still a whole tail ahead of their use
    if (LCV_FAN_LATE_FETCH) prefetch(r, nxr);
    LCV_FAN_T(1);
    __syncthreads();
    LCV_FAN_T(2);
    if constexpr (ROWS) {
      if (rowact) {  // K and the header flags are wave-uniform: the whole row takes one branch
        uint32_t rl = 0;  // r = REDC(T): limb j on lane j (partly normalised)
        if (K != 0) {
          const uint32_t jj = L & 15u;
          uint64_t lo = 0, hi = 0;
#if LCV_FAN_FLAT_COLS
          {  // branch-free: lanes 14, 15 read and zero lane 13's pair again (the reads precede the writes in the wave)
            const uint32_t jc = jj < 14u ? jj : 13u;
            const uint64_t cl = racc[jc], ch = racc[jc + 14];
            racc[jc] = 0;
            racc[jc + 14] = 0;
            lo = jj < 14u ? cl : 0ull;
            hi = jj < 14u ? ch : 0ull;
          }
#else
          if (jj < 14u) {
            lo = racc[jj];
            hi = racc[jj + 14];
            racc[jj] = 0;
            racc[jj + 14] = 0;
          }
#endif
#if LCV_FAN_X_TIMING > 1
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          LCV_FAN_T(5);
#endif
          rl = lcv::rw_redc_limbs(lo, hi, rtabs);
#if LCV_FAN_X_TIMING > 1
          asm volatile("" :: "v"(rl));
          LCV_FAN_T(6);
#endif
        }
        const uint32_t vl = lcv::rw_value(rl, (h0 >> 4) & 3u, cur.a0, cur.a1, lcv::rw_limb_of(tw[0], tw[1]),
                                          lcv::rw_limb_of(tw[2], tw[3]), (h0 >> 16) & 31u, rtabs);
#if LCV_FAN_X_TIMING > 1
        asm volatile("" :: "v"(vl));
        LCV_FAN_T(7);
#endif
        if (h0 & ((1u << 10) | (1u << 11) | (1u << 12))) {  // inversion, side-load and emit rounds: on lane 0
          uint32_t w[13];
          lcv::rw_gather(w, lcv::rw_word(vl));
          if (tail_lane) {
            lcv::fp v;
            w[12] = 0;
            const lcv::SopPre pre{cur.d0, cur.d1, 0, 0, 0};
            lcv::sop_tail_finish(v, h0 & ~(31u << 16), pre, w, qp);  // (reduced already)
            lcv::sop_tail_store(h0, pre, my, io_in, io_out, v);
          }
        } else {
          lcv::rw_store(vl, h0, cur.d0, cur.d1, my, rtabs);
        }
      }
    } else if (tail_lane) {  // op o's tail, in the first wave: every read of the round precedes its stores
      uint32_t res[13];
      if (K == 0) {
        LCV_UNROLL for (int j = 0; j < 13; ++j) res[j] = 0;
      } else {
        uint64_t col[28];
        LCV_UNROLL for (int c = 0; c < 28; ++c) col[c] = acc[c];
        LCV_UNROLL for (int c = 0; c < 28; ++c) acc[c] = 0;
#if LCV_FAN_X_TIMING > 1  // sub-phases of the tail (the sums wait for their reads: the clock reads data)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        LCV_FAN_T(5);
#endif
        lcv::sop_redc28(res, col);
#if LCV_FAN_X_TIMING > 1
        asm volatile("" :: "v"(res[12]));
        LCV_FAN_T(6);
#endif
      }
      lcv::fp v;
      lcv::sop_tail_value(v, h0, cur.w, cur.pre, my, lds, ns, res, qp);
#if LCV_FAN_X_TIMING > 1
      asm volatile("" :: "v"(v.v[11]));
      LCV_FAN_T(7);
#endif
      lcv::sop_tail_store(h0, cur.pre, my, io_in, io_out, v);
    }
    LCV_FAN_T(3);
#if LCV_FAN_X_TIMING > 1
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    LCV_FAN_T(8);
#endif
    __syncthreads();
    LCV_FAN_T(4);
  };
  Rec rb = nx;
  for (uint32_t r = 0; r < R; r += 2) {
    round(r, nx, rb);
    if (r + 1 < R) round(r + 1, rb, nx);
  }
#if LCV_FAN_X_TIMING
  if (item == 0 && (L == 0 || L == NT - 64))
    printf("fan T=%u KM=%u S=%u R=%u rows=%d wave=%u: fetch %lu products %lu barrier1 %lu tail %lu barrier2 %lu | "
           "tail: columns %lu redc %lu value %lu store %lu\n", T, KM, S, R, (int)ROWS, L / 64, tq[0], tq[1], tq[2], tq[3],
           tq[4], tq[5], tq[6], tq[7], tq[8]);
#endif
#undef LCV_FAN_T
  if (L < T && item < n) f.epilogue(item, L, my);
}
#endif
