// lcv_items.hpp — per-item bodies of every stage of the batched verifier.  Each function processes
// ONE item (an update, a committee key, a (update, pairing) pair ...) and is called by
//   * the HIP kernels in lcv_hip.hip (one lane per item), and
//   * the host-simulation test build lcv_hostsim.cpp (a plain loop), so the exact device
//     arithmetic can be checked against the CPU oracle in the CPU-only test suite.
// All intermediate device buffers are structure-of-arrays with stride `cap` (lane i of a wave reads
// consecutive 32-bit words -> coalesced).
//
// Stage map onto the reference's validate_light_client_update (sync-protocol.md:386-465):
//   item_nsc_team   hash_tree_root(next_sync_committee) + default / store-equality tests (:439-449)
//   item_pre        every non-BLS assert (:392-449) -> first failing reason, committee id
//   item_sigroot    signing root (:460-463) -> W.msg
//   item_h2c_map + SOP h2c program   hash_to_G2(signing_root)                  -+
//   item_sig + SOP line walk          signature decode + G2 subgroup check      |  bls.FastAggregate-
//   item_agg                          masked G1 aggregation of participant keys |  Verify (:464)
//   SOP lines / miller_acc / fexp     the two-pairing product check             -+
//   (SOP programs: tools/gen_sop.py -> lcv_sop_programs.inc, interpreter lcv_sop.hpp)
//   item_verdict    conjunction + reason code
#pragma once
#include "lcv_h2c.hpp"
#include "lcv_pairing.hpp"
#include "lcv_ssz.hpp"

namespace lcv {

struct BatchDev {
  const uint8_t* att_beacon;
  const uint8_t* att_exec;
  const uint8_t* att_branch;
  const uint8_t* fin_beacon;
  const uint8_t* fin_exec;
  const uint8_t* fin_branch;
  const uint8_t* nsc_pool;
  const uint32_t* nsc_index;
  const uint8_t* nsc_branch;
  const uint8_t* finality_branch;
  const uint8_t* bits;
  const uint8_t* sig;
  const uint64_t* sig_slot;
  uint32_t n;
  uint32_t npool;
};

struct Params {
  NetConfig cfg;
  uint64_t current_slot;
  uint64_t store_fin_slot;
  uint32_t next_known;
  uint32_t gvr[8];  // big-endian words
};

struct CommitteeDev {
  const uint8_t* next_raw;   // store.next_sync_committee SSZ bytes (24624)
  uint32_t* pts;             // [ncomm][512][24]  affine x,y (Montgomery)
  uint32_t* sum_all;         // [ncomm][36]       Jacobian sum of all valid keys
  uint32_t* badmask;         // [ncomm][16]       invalid-key bitmap
  uint8_t* key_status;       // [ncomm][512]      PT_OK, or PT_BAD (undecodable / identity / not in G1)
  const uint8_t* raw;        // [ncomm][raw_stride] compressed pubkeys, key j at +48 j
  uint32_t raw_stride;       // 24624 for SSZ SyncCommittee, 24576 for bare key tables
  uint32_t ncomm;
};

struct Work {
  uint32_t cap;
  uint32_t pool_cap;
  uint32_t* msg;         // [8][cap]
  uint8_t* pre_reason;   // [cap]
  uint32_t* comm_id;     // [cap] committee used for the signature (0 current, 1 next)
  uint32_t* nsc_root;    // [8][pool_cap]
  uint8_t* nsc_flags;    // [pool_cap] bit0: all-zero, bit1: equals store.next_sync_committee
  uint32_t* qmap;        // [96][cap] the two SSWU outputs on E2' (affine, 8 Fp: x0,x1,y0,y1 per map)
  uint32_t* qh;          // [48][cap] H(m) affine (x0,x1,y0,y1)
  uint8_t* qh_inf;       // [cap]
  uint32_t* qs;          // [48][cap] signature affine
  uint8_t* sig_status;   // [cap]
  uint32_t* pk;          // [24][cap] aggregate pubkey affine
  uint8_t* agg_status;   // [cap]
  uint32_t* f;           // [cap][144]   Miller output, then the pairing value (item-major: f12_st_coeff)
  uint8_t* pair_ok;      // [cap]
  uint8_t* verdict;      // [cap]
  uint8_t* reason;       // [cap]
  uint32_t* lines;       // [item][2 pairings][6 * 68 line values][12]  (SOP Miller loop: lines -> accumulation)
  uint32_t msg_b0;       // 1: W.msg already holds expand_message_xmd's b0 (arbitrary-length messages)
};

// fp2 coefficient g_i (of w^i) -> its fp2 slot in the SoA Fp12 layout of soa_st_fp12 (c0.c0, c0.c1,
// c0.c2, c1.c0, c1.c1, c1.c2 = g0, g2, g4, g1, g3, g5)
LCV_FN uint32_t fp12_soa_slot(uint32_t g) { return (g & 1u) ? 3u + (g >> 1) : (g >> 1); }

// ---- element addressing of the Work / batch arrays: every accessor below and the host-side layout
// check (lcv_debug_work_check, lcv_driver.inc) go through these, so the check sees the kernels' addresses
// SoA: row `row` of item i of an array with stride cap
LCV_HDFN size_t soa_index(size_t cap, size_t i, size_t row) { return row * cap + i; }
// item-major W.f: coefficient s of item i (12 words each, 144 per item)
LCV_HDFN size_t f12_index(size_t i, uint32_t s) { return (i * 12 + s) * 12; }
enum : uint32_t { F12_ITEM_WORDS = 144 };

// ---- SoA helpers
LCV_FN void soa_ld_fp(fp& r, const uint32_t* base, size_t cap, size_t i, size_t slot) {
  LCV_UNROLL for (int k = 0; k < 12; ++k) r.v[k] = base[soa_index(cap, i, slot * 12 + k)];
}
LCV_FN void soa_st_fp(uint32_t* base, size_t cap, size_t i, size_t slot, const fp& a) {
  LCV_UNROLL for (int k = 0; k < 12; ++k) base[soa_index(cap, i, slot * 12 + k)] = a.v[k];
}
// W.f (the Miller loop's output, the final exponentiation's e^3): item-major, the 12 Fp coefficients of
// item i in the SOP programs' slot order (2 g + c for the w^g coefficient, component c), 48 contiguous
// bytes each, so a team's lanes move their coefficients as 16-byte accesses of one 576-byte row
LCV_FN void f12_st_coeff(uint32_t* base, size_t i, uint32_t s, const uint32_t v[12]) {
  uint32_t* d = base + f12_index(i, s);
#if defined(__HIP_DEVICE_COMPILE__)
  uint4* q = (uint4*)d;
  LCV_UNROLL for (int k = 0; k < 3; ++k) q[k] = make_uint4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
#else
  LCV_UNROLL for (int k = 0; k < 12; ++k) d[k] = v[k];
#endif
}
LCV_FN void f12_ld_coeff(uint32_t v[12], const uint32_t* base, size_t i, uint32_t s) {
  const uint32_t* d = base + f12_index(i, s);
#if defined(__HIP_DEVICE_COMPILE__)
  const uint4* q = (const uint4*)d;
  LCV_UNROLL for (int k = 0; k < 3; ++k) {
    const uint4 t = q[k];
    v[4 * k] = t.x; v[4 * k + 1] = t.y; v[4 * k + 2] = t.z; v[4 * k + 3] = t.w;
  }
#else
  LCV_UNROLL for (int k = 0; k < 12; ++k) v[k] = d[k];
#endif
}
LCV_FN void soa_ld_fp2(fp2& r, const uint32_t* base, size_t cap, size_t i, size_t slot) {
  soa_ld_fp(r.c0, base, cap, i, 2 * slot);
  soa_ld_fp(r.c1, base, cap, i, 2 * slot + 1);
}
LCV_FN void soa_st_fp2(uint32_t* base, size_t cap, size_t i, size_t slot, const fp2& a) {
  soa_st_fp(base, cap, i, 2 * slot, a.c0);
  soa_st_fp(base, cap, i, 2 * slot + 1, a.c1);
}
LCV_FN void soa_ld_fp12(fp12& r, const uint32_t* base, size_t cap, size_t i) {
  soa_ld_fp2(r.c0.c0, base, cap, i, 0); soa_ld_fp2(r.c0.c1, base, cap, i, 1); soa_ld_fp2(r.c0.c2, base, cap, i, 2);
  soa_ld_fp2(r.c1.c0, base, cap, i, 3); soa_ld_fp2(r.c1.c1, base, cap, i, 4); soa_ld_fp2(r.c1.c2, base, cap, i, 5);
}
LCV_FN void soa_st_fp12(uint32_t* base, size_t cap, size_t i, const fp12& a) {
  soa_st_fp2(base, cap, i, 0, a.c0.c0); soa_st_fp2(base, cap, i, 1, a.c0.c1); soa_st_fp2(base, cap, i, 2, a.c0.c2);
  soa_st_fp2(base, cap, i, 3, a.c1.c0); soa_st_fp2(base, cap, i, 4, a.c1.c1); soa_st_fp2(base, cap, i, 5, a.c1.c2);
}
LCV_FN void soa_ld_h256(h256& r, const uint32_t* base, size_t cap, size_t i) {
  LCV_UNROLL for (int k = 0; k < 8; ++k) r.w[k] = base[k * cap + i];
}
LCV_FN void soa_st_h256(uint32_t* base, size_t cap, size_t i, const h256& a) {
  LCV_UNROLL for (int k = 0; k < 8; ++k) base[k * cap + i] = a.w[k];
}

// ============================================================================ SSZ stage
// hash_tree_root(next_sync_committee) + default / store-equality tests (:439-449), one team per pool row.
// Team version (64 lanes per committee): lane l hashes keys 8l..8l+7 into a depth-3 subtree root,
// then 6 rounds halve the 64 roots (ping-pong LDS buffers), and lane 0 mixes in the aggregate key.
// The all-zero / equals-store tests are split over the lanes (flags reduced by lane 0).
enum { NSC_TEAM = 64, NSC_ROUNDS = 8, NSC_LDS = 2 * 64 * 8 + 64 };
LCV_FN void item_nsc_team(uint32_t j, uint32_t lane, uint32_t r, uint32_t* lds, const BatchDev& B,
                          const CommitteeDev& C, const Work& W) {
  const uint8_t* sc = B.nsc_pool + (size_t)K_SC * j;
  uint32_t* buf0 = lds;
  uint32_t* buf1 = lds + 64 * 8;
  uint32_t* flags = lds + 2 * 64 * 8;
  if (r == 0) {
    h256 n[8];
    LCV_NOUNROLL for (int k = 0; k < 8; ++k) htr_pubkey(n[k], sc + 48 * (8 * lane + k));
    hash_pair(n[0], n[0], n[1]);
    hash_pair(n[2], n[2], n[3]);
    hash_pair(n[4], n[4], n[5]);
    hash_pair(n[6], n[6], n[7]);
    hash_pair(n[0], n[0], n[2]);
    hash_pair(n[4], n[4], n[6]);
    hash_pair(n[0], n[0], n[4]);
    LCV_UNROLL for (int k = 0; k < 8; ++k) buf0[8 * lane + k] = n[0].w[k];
    const uint32_t* a = (const uint32_t*)sc;
    const uint32_t* b = (const uint32_t*)C.next_raw;
    uint32_t orz = 0, dif = 0;
    for (int k = lane; k < K_SC / 4; k += 64) {
      const uint32_t x = a[k];
      orz |= x;
      dif |= x ^ b[k];
    }
    flags[lane] = (orz != 0 ? 1u : 0u) | (dif != 0 ? 2u : 0u);
  } else if (r < 7) {
    const uint32_t* src = (r & 1) ? buf0 : buf1;
    uint32_t* dst = (r & 1) ? buf1 : buf0;
    if (lane < (64u >> r)) {
      h256 x, y;
      LCV_UNROLL for (int k = 0; k < 8; ++k) { x.w[k] = src[16 * lane + k]; y.w[k] = src[16 * lane + 8 + k]; }
      hash_pair(x, x, y);
      LCV_UNROLL for (int k = 0; k < 8; ++k) dst[8 * lane + k] = x.w[k];
    }
  } else if (lane == 0) {  // r == 7: the 6 halving rounds ended in buf0 (r = 6 writes buf0)
    h256 root, agg;
    LCV_UNROLL for (int k = 0; k < 8; ++k) root.w[k] = buf0[k];
    htr_pubkey(agg, sc + 48 * 512);
    hash_pair(root, root, agg);
    soa_st_h256(W.nsc_root, W.pool_cap, j, root);
    uint32_t f = 0;
    for (int k = 0; k < 64; ++k) f |= flags[k];
    W.nsc_flags[j] = (uint8_t)(((f & 1u) ? 0u : 1u) | ((f & 2u) ? 0u : 2u));
  }
}

LCV_FN uint32_t popcount_bits(const uint8_t* bits) {
  uint32_t pc = 0;
  LCV_UNROLL for (int w = 0; w < 16; ++w) pc += (uint32_t)__builtin_popcount(((const uint32_t*)bits)[w]);
  return pc;
}

LCV_FN void item_pre(uint32_t i, const BatchDev& B, const CommitteeDev& C, const Params& P, const Work& W) {
  (void)C;
  const uint8_t* ab = B.att_beacon + (size_t)K_BEACON * i;
  const uint8_t* ae = B.att_exec + (size_t)K_EXEC * i;
  const uint8_t* abr = B.att_branch + (size_t)K_EXEC_BRANCH * i;
  const uint8_t* fb = B.fin_beacon + (size_t)K_BEACON * i;
  const uint8_t* fe = B.fin_exec + (size_t)K_EXEC * i;
  const uint8_t* fbr = B.fin_branch + (size_t)K_EXEC_BRANCH * i;
  const uint8_t* nbr = B.nsc_branch + (size_t)K_NSC_BRANCH * i;
  const uint8_t* finb = B.finality_branch + (size_t)K_FIN_BRANCH * i;
  const uint32_t pool = B.nsc_index[i];
  const uint64_t sig_slot = B.sig_slot[i];
  const uint64_t att_slot = ld_le64(ab);
  const uint64_t fin_slot = ld_le64(fb);
  uint32_t reason = 0;
#define LCV_FAIL(k) do { if (reason == 0) reason = (k); } while (0)
  // :392 participants
  if (popcount_bits(B.bits + 64 * (size_t)i) < 1) LCV_FAIL(1);
  // :395 attested header
  if (!lc_header_valid(ab, ae, abr, P.cfg)) LCV_FAIL(2);
  // :398 slot ordering
  if (!(P.current_slot >= sig_slot && sig_slot > att_slot && att_slot >= fin_slot)) LCV_FAIL(3);
  const uint64_t store_period = period_of_slot(P.store_fin_slot, P.cfg);
  const uint64_t sig_period = period_of_slot(sig_slot, P.cfg);
  const bool next_known = P.next_known != 0;
  if (next_known) {
    if (!(sig_period == store_period || sig_period == store_period + 1)) LCV_FAIL(4);  // :402
  } else {
    if (sig_period != store_period) LCV_FAIL(5);  // :404
  }
  // :407-414 relevance
  const uint64_t att_period = period_of_slot(att_slot, P.cfg);
  const bool is_sc = !bytes_all_zero(nbr, K_NSC_BRANCH / 4);
  const bool has_next = !next_known && is_sc && att_period == store_period;
  if (!(att_slot > P.store_fin_slot || has_next)) LCV_FAIL(6);
  // :419-434 finality
  h256 state_root;
  ld_chunk(state_root, ab + 48);
  const bool is_fin = !bytes_all_zero(finb, K_FIN_BRANCH / 4);
  const bool fin_default = bytes_all_zero(fb, K_BEACON / 4) && bytes_all_zero(fe, K_EXEC / 4) &&
                           bytes_all_zero(fbr, K_EXEC_BRANCH / 4);
  if (!is_fin) {
    if (!fin_default) LCV_FAIL(7);
  } else {
    h256 leaf;
    if (fin_slot == 0) {
      if (!fin_default) LCV_FAIL(8);
      h256_zero(leaf);
    } else {
      if (!lc_header_valid(fb, fe, fbr, P.cfg)) LCV_FAIL(9);
      htr_beacon(leaf, fb);
    }
    if (!merkle_branch_ok(leaf, finb, 6, 41, state_root)) LCV_FAIL(10);
  }
  // :438-449 next sync committee
  const uint32_t nflags = W.nsc_flags[pool];
  if (!is_sc) {
    if (!(nflags & 1u)) LCV_FAIL(11);
  } else {
    if (att_period == store_period && next_known && !(nflags & 2u)) LCV_FAIL(12);
    h256 leaf;
    soa_ld_h256(leaf, W.nsc_root, W.pool_cap, pool);
    if (!merkle_branch_ok(leaf, nbr, 5, 23, state_root)) LCV_FAIL(13);
  }
#undef LCV_FAIL
  // :452-459 committee selection (the signing root is item_sigroot's)
  W.comm_id[i] = sig_period != store_period ? 1u : 0u;
  W.pre_reason[i] = (uint8_t)reason;
}

// :460-463 fork version, domain and signing root of the attested header -> W.msg.  A kernel of its own
// (16 SHA-256 compressions per update against item_pre's 162), so hash_to_G2 starts without waiting
// for the branch checks, which run beside it on another stream.
LCV_FN void item_sigroot(uint32_t i, const BatchDev& B, const Params& P, const Work& W) {
  const uint8_t* ab = B.att_beacon + (size_t)K_BEACON * i;
  h256 gvr, msg;
  LCV_UNROLL for (int k = 0; k < 8; ++k) gvr.w[k] = P.gvr[k];
  signing_root(msg, ab, B.sig_slot[i], gvr, P.cfg);
  soa_st_h256(W.msg, W.cap, i, msg);
}

// ============================================================================ BLS stages
LCV_FN void st_g2a(uint32_t* base, size_t cap, size_t i, const g2a& q) {
  soa_st_fp2(base, cap, i, 0, q.x);
  soa_st_fp2(base, cap, i, 1, q.y);
}
LCV_FN void ld_g2a(g2a& q, const uint32_t* base, size_t cap, size_t i) {
  soa_ld_fp2(q.x, base, cap, i, 0);
  soa_ld_fp2(q.y, base, cap, i, 1);
}

// hash_to_field + simplified SWU for u_m of update i (item t: i = t >> 1, m = t & 1): the serial part
// of hash_to_G2 (two Fp exponentiations for the square root), two lanes per update; the isogeny,
// addition, cofactor clearing and affine conversion run as the SOP program `h2c` (F_sop_h2c)
LCV_FN void item_h2c_map(uint32_t t, const Work& W) {
  const uint32_t i = t >> 1, m = t & 1u;
  h256 msg;
  soa_ld_h256(msg, W.msg, W.cap, i);
  fp2 u, x, y;
  if (W.msg_b0) hash_to_field_u_b0(u, msg, m);
  else hash_to_field_u(u, msg, m);
  sswu_e2prime(x, y, u);
  soa_st_fp2(W.qmap, W.cap, i, 2 * m, x);
  soa_st_fp2(W.qmap, W.cap, i, 2 * m + 1, y);
}

// signature decode (flags, x < p, on-curve square root); the G2 subgroup check (psi(Q) == [x]Q) is fused
// into the signature pairing's SOP line walk (F_sop_lines mode 1), which may downgrade PT_OK to PT_BAD
LCV_FN void item_sig(uint32_t i, const BatchDev& B, const Work& W) {
  g2a s;
  fp2_zero(s.x);
  fp2_zero(s.y);
  const int st = g2_decompress(s, B.sig + 96 * (size_t)i);
  st_g2a(W.qs, W.cap, i, s);
  W.sig_status[i] = (uint8_t)st;
}

LCV_FN void ld_g1a_tbl(g1a& p, const uint32_t* pts, size_t idx) {
  const uint32_t* q = pts + idx * 24;
  LCV_UNROLL for (int k = 0; k < 12; ++k) { p.x.v[k] = q[k]; p.y.v[k] = q[12 + k]; }
}

// masked aggregation of the selected committee (sync-protocol.md:452-459 + FastAggregateVerify's
// aggregate).  Complement trick: with more than 256 participants, sum_all - sum(non-participants).
LCV_FN void item_agg(uint32_t i, const BatchDev& B, const CommitteeDev& C, const Work& W) {
  const uint32_t c = W.comm_id[i];
  const uint32_t* bw = (const uint32_t*)(B.bits + 64 * (size_t)i);
  const uint32_t* bad = C.badmask + 16 * c;
  uint32_t pc = 0, anybad = 0;
  LCV_UNROLL for (int w = 0; w < 16; ++w) {
    pc += (uint32_t)__builtin_popcount(bw[w]);
    anybad |= bw[w] & bad[w];
  }
  const bool comp = pc > 256;
  g1j acc;
  if (comp) {
    const uint32_t* s = C.sum_all + 36 * c;
    LCV_UNROLL for (int k = 0; k < 12; ++k) { acc.x.v[k] = s[k]; acc.y.v[k] = s[12 + k]; acc.z.v[k] = s[24 + k]; }
  } else {
    jac_set_inf(acc);
  }
  const uint32_t* pts = C.pts + (size_t)c * 512 * 24;
  LCV_NOUNROLL for (int w = 0; w < 16; ++w) {
    uint32_t m = comp ? (~bw[w] & ~bad[w]) : bw[w];
    while (m) {
      const int b = __builtin_ctz(m);
      m &= m - 1;
      g1a p;
      ld_g1a_tbl(p, pts, 32 * w + b);
      if (comp) fp_neg(p.y, p.y);
      jac_madd(acc, acc, p);
    }
  }
  const bool inf = jac_is_inf(acc);
  g1a a;
  jac_to_aff(a, acc);
  soa_st_fp(W.pk, W.cap, i, 0, a.x);
  soa_st_fp(W.pk, W.cap, i, 1, a.y);
  W.agg_status[i] = (uint8_t)(anybad ? PT_BAD : (inf || pc == 0 ? PT_INF : PT_OK));
}

// Jacobian G1 point <-> 36 LDS words (team kernels)
LCV_FN void ld_g1j_lds(g1j& p, const uint32_t* s) {
  LCV_UNROLL for (int k = 0; k < 12; ++k) { p.x.v[k] = s[k]; p.y.v[k] = s[12 + k]; p.z.v[k] = s[24 + k]; }
}
LCV_FN void st_g1j_lds(uint32_t* s, const g1j& p) {
  LCV_UNROLL for (int k = 0; k < 12; ++k) { s[k] = p.x.v[k]; s[12 + k] = p.y.v[k]; s[24 + k] = p.z.v[k]; }
}

// The same masked aggregation on a team of AGG_TEAM = 4 lanes per item (16 items per wave): round 0,
// lane l sums the gathered points of mask words 4l .. 4l + 3 (128 keys); rounds 1-2, a pairwise tree
// over the 4 partial sums in LDS; round 3, lane 0 adds the committee sum (complement case), converts to
// affine and writes the aggregate.  One lane per item ran a serial chain as long as the wave's longest
// (up to 170 mixed additions at 342-512 random participants); here each lane's chain covers a quarter
// of the bits (north star: wavefront-level reductions for point aggregation).
enum { AGG_TEAM = 4, AGG_ROUNDS = 4, AGG_LDS = AGG_TEAM * 36 };
LCV_FN void item_agg_team(uint32_t i, uint32_t lane, uint32_t r, uint32_t* lds, const BatchDev& B,
                          const CommitteeDev& C, const Work& W) {
  const uint32_t c = W.comm_id[i];
  const uint32_t* bw = (const uint32_t*)(B.bits + 64 * (size_t)i);
  const uint32_t* bad = C.badmask + 16 * c;
  uint32_t* part = lds + 36 * lane;
  if (r == 0) {
    uint32_t pc = 0;
    LCV_UNROLL for (int w = 0; w < 16; ++w) pc += (uint32_t)__builtin_popcount(bw[w]);
    const bool comp = pc > 256;
    const uint32_t* pts = C.pts + (size_t)c * 512 * 24;
    g1j acc;
    jac_set_inf(acc);
    LCV_NOUNROLL for (uint32_t w = 4 * lane; w < 4 * lane + 4; ++w) {
      uint32_t m = comp ? (~bw[w] & ~bad[w]) : bw[w];
      while (m) {
        const int b = __builtin_ctz(m);
        m &= m - 1;
        g1a p;
        ld_g1a_tbl(p, pts, 32 * w + b);
        if (comp) fp_neg(p.y, p.y);
        jac_madd(acc, acc, p);
      }
    }
    st_g1j_lds(part, acc);
  } else if (r < AGG_ROUNDS - 1) {
    const uint32_t step = 1u << (r - 1);
    if ((lane & (2 * step - 1)) == 0) {
      g1j a, b;
      ld_g1j_lds(b, lds + 36 * (lane + step));
      if (!jac_is_inf(b)) {
        ld_g1j_lds(a, part);
        jac_add(a, a, b);
        st_g1j_lds(part, a);
      }
    }
  } else if (lane == 0) {
    uint32_t pc = 0, anybad = 0;
    LCV_UNROLL for (int w = 0; w < 16; ++w) {
      pc += (uint32_t)__builtin_popcount(bw[w]);
      anybad |= bw[w] & bad[w];
    }
    g1j acc;
    ld_g1j_lds(acc, part);
    if (pc > 256) {  // sum_all - sum(non-participants)
      g1j all;
      const uint32_t* s = C.sum_all + 36 * c;
      LCV_UNROLL for (int k = 0; k < 12; ++k) { all.x.v[k] = s[k]; all.y.v[k] = s[12 + k]; all.z.v[k] = s[24 + k]; }
      if (jac_is_inf(acc)) acc = all;
      else jac_add(acc, acc, all);
    }
    const bool inf = jac_is_inf(acc);
    g1a a;
    jac_to_aff(a, acc);
    soa_st_fp(W.pk, W.cap, i, 0, a.x);
    soa_st_fp(W.pk, W.cap, i, 1, a.y);
    W.agg_status[i] = (uint8_t)(anybad ? PT_BAD : (inf || pc == 0 ? PT_INF : PT_OK));
  }
}

// FastAggregateVerify with more keys than one 512-key table: items 0..m-1 hold the masked aggregates
// of consecutive 512-key slices of the caller's list; item 0 becomes their sum (any invalid key ->
// PT_BAD, an identity sum -> PT_INF).  One lane; m = ceil(npk / 512) is small.
LCV_FN void item_agg_fold(uint32_t m, const Work& W) {
  g1j acc;
  jac_set_inf(acc);
  bool bad = false;
  for (uint32_t k = 0; k < m; ++k) {
    if (W.agg_status[k] == PT_BAD) bad = true;
    if (W.agg_status[k] != PT_OK) continue;
    g1a p;
    soa_ld_fp(p.x, W.pk, W.cap, k, 0);
    soa_ld_fp(p.y, W.pk, W.cap, k, 1);
    jac_madd(acc, acc, p);
  }
  const bool inf = jac_is_inf(acc);
  g1a a;
  jac_to_aff(a, acc);
  soa_st_fp(W.pk, W.cap, 0, 0, a.x);
  soa_st_fp(W.pk, W.cap, 0, 1, a.y);
  W.agg_status[0] = (uint8_t)(bad ? PT_BAD : (inf ? PT_INF : PT_OK));
}

LCV_FN void item_verdict(uint32_t i, const Work& W) {
  uint32_t reason = W.pre_reason[i];
  if (reason == 0) {
    const bool ok = W.agg_status[i] == PT_OK && W.sig_status[i] != PT_BAD && W.pair_ok[i] != 0;
    reason = ok ? 0 : 14;  // :464
  }
  W.reason[i] = (uint8_t)reason;
  W.verdict[i] = reason == 0 ? 1 : 0;
}

// ============================================================================ committee setup
LCV_FN void item_committee_key(uint32_t t, const CommitteeDev& C) {
  const uint32_t c = t / 512, j = t % 512;
  g1a p;
  fp_zero(p.x);
  fp_zero(p.y);
  int st = g1_decompress(p, C.raw + (size_t)c * C.raw_stride + 48 * j);
  if (st == PT_OK && !g1_in_subgroup(p)) st = PT_BAD;
  if (st == PT_INF) st = PT_BAD;  // KeyValidate rejects the identity
  uint32_t* q = C.pts + (size_t)t * 24;
  LCV_UNROLL for (int k = 0; k < 12; ++k) { q[k] = p.x.v[k]; q[12 + k] = p.y.v[k]; }
  C.key_status[t] = (uint8_t)st;
}

// per committee: sum of all valid keys (for the complement trick) and the invalid-key bitmap, on a
// team of 64 lanes (one wave per committee): round 0, lane l sums keys 8l .. 8l + 7 and records their
// validity byte; rounds 1..6, a pairwise tree over the 64 partial sums in LDS (lane l adds lane
// l + 2^(k-1)'s sum when l % 2^k == 0); round 7 writes the sum and the 16 mask words.
enum { SUM_TEAM = 64, SUM_ROUNDS = 8, SUM_LDS = 64 * 36 + 16 };
LCV_FN void item_committee_sum_team(uint32_t c, uint32_t lane, uint32_t r, uint32_t* lds, const CommitteeDev& C) {
  uint32_t* part = lds + 36 * lane;
  uint8_t* mbytes = (uint8_t*)(lds + 64 * 36);
  if (r == 0) {
    g1j acc;
    jac_set_inf(acc);
    const uint32_t* pts = C.pts + (size_t)c * 512 * 24;
    uint32_t m = 0;
    LCV_NOUNROLL for (int b = 0; b < 8; ++b) {
      const uint32_t j = 8 * lane + b;
      if (C.key_status[(size_t)c * 512 + j] != PT_OK) {
        m |= 1u << b;
        continue;
      }
      g1a p;
      ld_g1a_tbl(p, pts, j);
      jac_madd(acc, acc, p);
    }
    st_g1j_lds(part, acc);
    mbytes[lane] = (uint8_t)m;
  } else if (r < 7) {
    const uint32_t step = 1u << (r - 1);
    if ((lane & (2 * step - 1)) == 0) {
      g1j a, b;
      ld_g1j_lds(a, part);
      ld_g1j_lds(b, lds + 36 * (lane + step));
      jac_add(a, a, b);
      st_g1j_lds(part, a);
    }
  } else {
    if (lane < 16) {
      const uint32_t* mw = (const uint32_t*)mbytes;  // bytes 4w .. 4w + 3 = keys 32w .. 32w + 31
      C.badmask[c * 16 + lane] = mw[lane];
    }
    if (lane == 0) {
      uint32_t* s = C.sum_all + 36 * c;
      LCV_UNROLL for (int k = 0; k < 36; ++k) s[k] = lds[k];
    }
  }
}

}  // namespace lcv
