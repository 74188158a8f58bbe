// lcv_functors.hpp — one functor per kernel: each wraps a per-item body of lcv_items.hpp so the
// same code runs as a HIP kernel (one lane per item, lcv_k_*.hip) or as a host loop (hostsim tests).
// The including file defines LCV_HD (the call-operator qualifier: __device__ or empty).
#pragma once
#include "lcv_items.hpp"

using namespace lcv;

struct F_nsc_team {
  BatchDev B; CommitteeDev C; Work W;
  static constexpr uint32_t TEAM = NSC_TEAM, LDS_WORDS = NSC_LDS, SHARED_WORDS = 0;
  LCV_HD uint32_t rounds() const { return NSC_ROUNDS; }
  LCV_HD void operator()(uint32_t j, uint32_t lane, uint32_t r, uint32_t* lds, uint32_t*) const { item_nsc_team(j, lane, r, lds, B, C, W); }
};
struct F_pre { BatchDev B; CommitteeDev C; Params P; Work W; LCV_HD void operator()(uint32_t i) const { item_pre(i, B, C, P, W); } };
struct F_sigroot { BatchDev B; Params P; Work W; LCV_HD void operator()(uint32_t i) const { item_sigroot(i, B, P, W); } };
struct F_h2c_map { Work W; LCV_HD void operator()(uint32_t t) const { item_h2c_map(t, W); } };
struct F_sig { BatchDev B; Work W; LCV_HD void operator()(uint32_t i) const { item_sig(i, B, W); } };
// latency-mode twins of the two one-lane-per-map/update kernels (lcv_k_lat.hip, compiled with LCV_FP_CALL=0:
// the field products inlined, no call per product — ~14 % faster for a lone wave, ~2 % more chip cycles at
// full batches, so batches keep the forms above; and one item per wave, its square-root chains spread over the
// wave, lcv_wave.hpp)
struct F_h2c_map_lat { Work W; LCV_HD void operator()(uint32_t t) const { item_h2c_map(t, W); } };
struct F_sig_lat { BatchDev B; Work W; LCV_HD void operator()(uint32_t i) const { item_sig(i, B, W); } };
struct F_agg { BatchDev B; CommitteeDev C; Work W; LCV_HD void operator()(uint32_t i) const { item_agg(i, B, C, W); } };
struct F_agg_fold { Work W; uint32_t m; LCV_HD void operator()(uint32_t) const { item_agg_fold(m, W); } };
struct F_verdict { Work W; LCV_HD void operator()(uint32_t i) const { item_verdict(i, W); } };
struct F_key { CommitteeDev C; LCV_HD void operator()(uint32_t t) const { item_committee_key(t, C); } };
struct F_agg_team {  // AGG_TEAM lanes per update (item_agg_team)
  BatchDev B; CommitteeDev C; Work W;
  static constexpr uint32_t TEAM = AGG_TEAM, LDS_WORDS = AGG_LDS, SHARED_WORDS = 0;
  LCV_HD uint32_t rounds() const { return AGG_ROUNDS; }
  LCV_HD void operator()(uint32_t i, uint32_t lane, uint32_t r, uint32_t* lds, uint32_t*) const {
    item_agg_team(i, lane, r, lds, B, C, W);
  }
};
struct F_sum {  // one wave per committee (item_committee_sum_team)
  CommitteeDev C;
  static constexpr uint32_t TEAM = SUM_TEAM, LDS_WORDS = SUM_LDS, SHARED_WORDS = 0;
  LCV_HD uint32_t rounds() const { return SUM_ROUNDS; }
  LCV_HD void operator()(uint32_t c, uint32_t lane, uint32_t r, uint32_t* lds, uint32_t*) const {
    item_committee_sum_team(c, lane, r, lds, C);
  }
};

struct F_msg_import {  // 32-byte messages -> W.msg (big-endian words, SoA)
  const uint8_t* msg; Work W;
  LCV_HD void operator()(uint32_t i) const {
    h256 m;
    LCV_UNROLL for (int k = 0; k < 8; ++k) m.w[k] = ld_be32(msg + 32 * (size_t)i + 4 * k);
    soa_st_h256(W.msg, W.cap, i, m);
  }
};
struct F_msg_import_b0 {  // one message of any length -> expand_message_xmd's b0 in W.msg (W.msg_b0 = 1)
  const uint8_t* msg; uint64_t len; Work W;
  LCV_HD void operator()(uint32_t i) const {
    h256 b0;
    xmd_b0_bytes(b0, msg, len);
    soa_st_h256(W.msg, W.cap, i, b0);
  }
};
struct F_merkle {
  const uint8_t* leaf; const uint8_t* branch; const uint8_t* root; uint8_t* out; uint32_t depth; uint64_t index;
  LCV_HD void operator()(uint32_t i) const {
    h256 l, r;
    ld_chunk(l, leaf + 32 * (size_t)i);
    ld_chunk(r, root + 32 * (size_t)i);
    out[i] = merkle_branch_ok(l, branch + (size_t)32 * depth * i, (int)depth, index, r) ? 1 : 0;
  }
};
struct F_htr_sc {
  const uint8_t* sc; uint8_t* out;
  LCV_HD void operator()(uint32_t i) const {
    h256 r;
    htr_sync_committee(r, sc + (size_t)K_SC * i);
    st_chunk(out + 32 * (size_t)i, r);
  }
};
struct F_sk_to_pk {
  const uint8_t* sk; uint8_t* out;
  LCV_HD void operator()(uint32_t i) const {
    g1a g;
    g1_generator(g);
    g1j p;
    jac_mul_scalar_be32(p, g, sk + 32 * (size_t)i);
    const bool inf = jac_is_inf(p);
    g1a a;
    jac_to_aff(a, p);
    g1_compress(out + 48 * (size_t)i, a, inf);
  }
};
struct F_sign {
  const uint8_t* sk; const uint8_t* msg; uint8_t* out;
  LCV_HD void operator()(uint32_t i) const {
    h256 m;
    LCV_UNROLL for (int k = 0; k < 8; ++k) m.w[k] = ld_be32(msg + 32 * (size_t)i + 4 * k);
    g2j h;
    hash_to_g2(h, m);
    g2a ha;
    jac_to_aff(ha, h);
    g2j s;
    jac_mul_scalar_be32(s, ha, sk + 32 * (size_t)i);
    const bool inf = jac_is_inf(s) || jac_is_inf(h);
    g2a a;
    jac_to_aff(a, s);
    g2_compress(out + 96 * (size_t)i, a, inf);
  }
};
struct F_dbg_fp {
  const uint8_t* a48; const uint8_t* b48; uint8_t* out; uint8_t* ok;
  LCV_HD void operator()(uint32_t i) const {
    fp a, b, r;
    fp_from_be48_mont(a, a48 + 48 * (size_t)i);
    fp_from_be48_mont(b, b48 + 48 * (size_t)i);
    uint8_t* o = out + 288 * (size_t)i;
    fp_mul(r, a, b); fp_to_be48(o, r);
    fp_add(r, a, b); fp_to_be48(o + 48, r);
    fp_sub(r, a, b); fp_to_be48(o + 96, r);
    fp_inv(r, a); fp_to_be48(o + 144, r);
    fp2 x, y;
    x.c0 = a;
    x.c1 = b;
    const bool s = fp2_sqrt(y, x);
    fp_to_be48(o + 192, y.c0);
    fp_to_be48(o + 240, y.c1);
    ok[i] = s ? 1 : 0;
  }
};
struct F_dbg_pow {  // the sqrt-candidate exponentiations (sliding window, fp_pow_p1d4 / fp_pow_p3d4)
  const uint8_t* a48; uint8_t* out;
  LCV_HD void operator()(uint32_t i) const {
    fp a, r;
    fp_from_be48_mont(a, a48 + 48 * (size_t)i);
    uint8_t* o = out + 96 * (size_t)i;
    fp_pow_p1d4(r, a); fp_to_be48(o, r);
    fp_pow_p3d4(r, a); fp_to_be48(o + 48, r);
  }
};
struct F_dbg_pow_lat { F_dbg_pow f; LCV_HD void operator()(uint32_t i) const { f(i); } };  // lcv_k_lat.hip's chains
struct F_export_g2 {  // SoA affine G2 -> canonical bytes
  const uint32_t* base; uint32_t cap; uint8_t* out;
  LCV_HD void operator()(uint32_t i) const {
    g2a q;
    ld_g2a(q, base, cap, i);
    uint8_t* o = out + 192 * (size_t)i;
    fp_to_be48(o, q.x.c0); fp_to_be48(o + 48, q.x.c1); fp_to_be48(o + 96, q.y.c0); fp_to_be48(o + 144, q.y.c1);
  }
};
struct F_export_g1 {
  const uint32_t* base; uint32_t cap; uint8_t* out;
  LCV_HD void operator()(uint32_t i) const {
    fp x, y;
    soa_ld_fp(x, base, cap, i, 0);
    soa_ld_fp(y, base, cap, i, 1);
    fp_to_be48(out + 96 * (size_t)i, x);
    fp_to_be48(out + 96 * (size_t)i + 48, y);
  }
};
struct F_export_fp12 {  // W.f (item-major, coefficient order w^0 .. w^5, f12_ld_coeff) -> big-endian bytes
  const uint32_t* base; uint32_t cap; uint8_t* out;
  LCV_HD void operator()(uint32_t i) const {
    uint8_t* o = out + 576 * (size_t)i;
    for (uint32_t s = 0; s < 12; ++s) {
      fp x;
      f12_ld_coeff(x.v, base, i, s);
      fp_to_be48(o + 48 * s, x);
    }
  }
};
struct F_import_pq {  // debug pairing inputs: P -> W.pk, Q -> W.qh (no validation: test entry point)
  const uint8_t* p96; const uint8_t* q192; Work W;
  LCV_HD void operator()(uint32_t i) const {
    fp x, y;
    fp_from_be48_mont(x, p96 + 96 * (size_t)i);
    fp_from_be48_mont(y, p96 + 96 * (size_t)i + 48);
    soa_st_fp(W.pk, W.cap, i, 0, x);
    soa_st_fp(W.pk, W.cap, i, 1, y);
    g2a q;
    const uint8_t* b = q192 + 192 * (size_t)i;
    fp_from_be48_mont(q.x.c0, b); fp_from_be48_mont(q.x.c1, b + 48);
    fp_from_be48_mont(q.y.c0, b + 96); fp_from_be48_mont(q.y.c1, b + 144);
    st_g2a(W.qh, W.cap, i, q);
    W.qh_inf[i] = 0;
    W.sig_status[i] = PT_BAD;  // second pairing contributes identity lines
  }
};

// initialize_light_client_store's checks (sync-protocol.md:353-362), one lane per bootstrap:
// reason 0 ok, 1 is_valid_light_client_header (:353), 2 hash_tree_root(header.beacon) ==
// trusted_block_root (:354), 3 current_sync_committee branch (:356-362; CURRENT_SYNC_COMMITTEE_GINDEX
// 54 -> depth 5, subtree index 22, rooted at header.beacon.state_root)
struct F_bootstrap {
  const uint8_t* beacon; const uint8_t* exec; const uint8_t* branch; const uint8_t* sc; const uint8_t* sc_branch;
  const uint8_t* trusted; uint8_t* out; NetConfig cfg;
  LCV_HD void operator()(uint32_t i) const {
    const uint8_t* b = beacon + (size_t)K_BEACON * i;
    uint8_t r = 0;
    if (!lc_header_valid(b, exec + (size_t)K_EXEC * i, branch + (size_t)K_EXEC_BRANCH * i, cfg)) {
      r = 1;
    } else {
      h256 root, t;
      htr_beacon(root, b);
      ld_chunk(t, trusted + 32 * (size_t)i);
      if (!h256_eq(root, t)) {
        r = 2;
      } else {
        h256 leaf, state;
        htr_sync_committee(leaf, sc + (size_t)K_SC * i);
        ld_chunk(state, b + 48);
        if (!merkle_branch_ok(leaf, sc_branch + 160 * (size_t)i, 5, 22, state)) r = 3;
      }
    }
    out[i] = r;
  }
};
