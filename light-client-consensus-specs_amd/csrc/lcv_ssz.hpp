// lcv_ssz.hpp — SSZ hash_tree_root of the light-client containers on the device, in the packed
// layouts of include/lcv.h:
//   BeaconBlockHeader   112 B SSZ (slot, proposer_index, parent_root, state_root, body_root)
//   execution record    832 B: 17 leaf chunks (leaf 4 = logs_bloom, computed; leaf 10 = extra_data
//                       padded), logs_bloom 256 B @544, extra_len u32 @800
//   SyncCommittee       24624 B SSZ (512 x 48 B pubkeys, 48 B aggregate_pubkey)
// Reference: get_lc_execution_root (sync-protocol.md:186-214), is_valid_light_client_header
// (:220-240), hash_tree_root call sites (:427, :444, :463).
#pragma once
#include "lcv_sha.hpp"

namespace lcv {

enum {
  K_BEACON = 112,
  K_EXEC = 832,
  K_EXEC_BLOOM_OFF = 544,
  K_EXEC_EXTRALEN_OFF = 800,
  K_EXEC_BRANCH = 128,
  K_NSC_BRANCH = 160,
  K_FIN_BRANCH = 192,
  K_SC = 24624,
};

// The network configuration the light-client path reads (lcv_set_config; mainnet by default): the
// preset's SLOTS_PER_EPOCH and EPOCHS_PER_SYNC_COMMITTEE_PERIOD (UPDATE_TIMEOUT's factors,
// compute_sync_committee_period_at_slot), the config's fork epochs (is_valid_light_client_header
// sync-protocol.md:220-240, get_lc_execution_root :186-214) and fork versions (compute_fork_version
// at :461), and DOMAIN_SYNC_COMMITTEE (:462).  SYNC_COMMITTEE_SIZE stays the mainnet preset's 512
// (the packed layouts of include/lcv.h).
struct NetConfig {
  uint64_t slots_per_epoch;
  uint64_t epochs_per_period;
  uint64_t fork_epoch[4];          // ALTAIR, BELLATRIX, CAPELLA, DENEB
  uint32_t fork_version[5];        // GENESIS, ALTAIR, BELLATRIX, CAPELLA, DENEB (big-endian words)
  uint32_t domain_sync_committee;  // big-endian word
};
enum { FORK_ALTAIR = 0, FORK_BELLATRIX = 1, FORK_CAPELLA = 2, FORK_DENEB = 3 };

inline NetConfig net_config_mainnet() {
  NetConfig c;
  c.slots_per_epoch = 32;
  c.epochs_per_period = 256;
  c.fork_epoch[FORK_ALTAIR] = 74240;
  c.fork_epoch[FORK_BELLATRIX] = 144896;
  c.fork_epoch[FORK_CAPELLA] = 194048;
  c.fork_epoch[FORK_DENEB] = 269568;
  for (uint32_t k = 0; k < 5; ++k) c.fork_version[k] = k << 24;  // 0x0k000000
  c.domain_sync_committee = 0x07000000u;
  return c;
}

LCV_FN uint64_t epoch_of_slot(uint64_t slot, const NetConfig& c) { return slot / c.slots_per_epoch; }
LCV_FN uint64_t period_of_slot(uint64_t slot, const NetConfig& c) {
  return slot / (c.slots_per_epoch * c.epochs_per_period);
}

// hash_tree_root(BeaconBlockHeader): 5 leaves -> 8, 6 hashes
LCV_FN void htr_beacon(h256& root, const uint8_t* b) {
  h256 l0, l1, l2, l3, z, n0, n1, n2;
  u64_chunk(l0, ld_le64(b));
  u64_chunk(l1, ld_le64(b + 8));
  hash_pair(n0, l0, l1);
  ld_chunk(l2, b + 16);
  ld_chunk(l3, b + 48);
  hash_pair(n1, l2, l3);
  ld_chunk(l0, b + 80);
  zero_hash(z, 0);
  hash_pair(n2, l0, z);
  hash_pair(n0, n0, n1);
  zero_hash(z, 1);
  hash_pair(n2, n2, z);
  hash_pair(root, n0, n2);
}

LCV_FN void exec_leaf(h256& r, const uint8_t* rec, int k, const h256& bloom_root, const h256& extra_root) {
  if (k == 4) r = bloom_root;
  else if (k == 10) r = extra_root;
  else ld_chunk(r, rec + 32 * k);
}

// hash_tree_root of the Deneb (17 fields) or Capella (15 fields) ExecutionPayloadHeader
LCV_FN void htr_exec(h256& root, const uint8_t* rec, bool deneb) {
  h256 bloom_root, extra_root, a, b;
  {
    h256 n[4];
    LCV_UNROLL for (int k = 0; k < 4; ++k) {
      ld_chunk(a, rec + K_EXEC_BLOOM_OFF + 64 * k);
      ld_chunk(b, rec + K_EXEC_BLOOM_OFF + 64 * k + 32);
      hash_pair(n[k], a, b);
    }
    hash_pair(n[0], n[0], n[1]);
    hash_pair(n[2], n[2], n[3]);
    hash_pair(bloom_root, n[0], n[2]);
  }
  {
    h256 len;
    ld_chunk(a, rec + 32 * 10);
    u64_chunk(len, (uint64_t)(*(const uint32_t*)(rec + K_EXEC_EXTRALEN_OFF)));
    hash_pair(extra_root, a, len);  // mix_in_length(merkleize([chunk], limit=1), len)
  }
  h256 z;
  if (deneb) {
    h256 l1[9];
    LCV_UNROLL for (int k = 0; k < 8; ++k) {
      exec_leaf(a, rec, 2 * k, bloom_root, extra_root);
      exec_leaf(b, rec, 2 * k + 1, bloom_root, extra_root);
      hash_pair(l1[k], a, b);
    }
    exec_leaf(a, rec, 16, bloom_root, extra_root);
    zero_hash(z, 0);
    hash_pair(l1[8], a, z);
    LCV_UNROLL for (int k = 0; k < 4; ++k) hash_pair(l1[k], l1[2 * k], l1[2 * k + 1]);
    zero_hash(z, 1);
    hash_pair(l1[4], l1[8], z);
    hash_pair(l1[0], l1[0], l1[1]);
    hash_pair(l1[1], l1[2], l1[3]);
    zero_hash(z, 2);
    hash_pair(l1[2], l1[4], z);
    hash_pair(l1[0], l1[0], l1[1]);
    zero_hash(z, 3);
    hash_pair(l1[1], l1[2], z);
    hash_pair(root, l1[0], l1[1]);
  } else {
    h256 l1[8];
    LCV_UNROLL for (int k = 0; k < 7; ++k) {
      exec_leaf(a, rec, 2 * k, bloom_root, extra_root);
      exec_leaf(b, rec, 2 * k + 1, bloom_root, extra_root);
      hash_pair(l1[k], a, b);
    }
    exec_leaf(a, rec, 14, bloom_root, extra_root);
    zero_hash(z, 0);
    hash_pair(l1[7], a, z);
    LCV_UNROLL for (int k = 0; k < 4; ++k) hash_pair(l1[k], l1[2 * k], l1[2 * k + 1]);
    hash_pair(l1[0], l1[0], l1[1]);
    hash_pair(l1[1], l1[2], l1[3]);
    hash_pair(root, l1[0], l1[1]);
  }
}

// is_valid_light_client_header (sync-protocol.md:220-240)
LCV_FN bool lc_header_valid(const uint8_t* beacon, const uint8_t* exec, const uint8_t* branch, const NetConfig& cfg) {
  const uint64_t epoch = epoch_of_slot(ld_le64(beacon), cfg);
  const uint64_t blob = ld_le64(exec + 32 * 15);
  const uint64_t excess = ld_le64(exec + 32 * 16);
  if (epoch < cfg.fork_epoch[FORK_DENEB] && (blob | excess) != 0) return false;
  if (epoch < cfg.fork_epoch[FORK_CAPELLA])
    return bytes_all_zero(exec, K_EXEC / 4) && bytes_all_zero(branch, K_EXEC_BRANCH / 4);
  h256 root, body;
  htr_exec(root, exec, epoch >= cfg.fork_epoch[FORK_DENEB]);
  ld_chunk(body, beacon + 80);
  return merkle_branch_ok(root, branch, 4, 9, body);
}

// incremental merkleization of 512 leaves with a statically indexed stack (uniform leaf index j)
template <int L> LCV_FN void merkle_push(h256 (&s)[10], h256& node, uint32_t j) {
  if constexpr (L >= 9) {
    s[9] = node;
  } else {
    if ((j >> L) & 1u) {
      hash_pair(node, s[L], node);
      merkle_push<L + 1>(s, node, j);
    } else {
      s[L] = node;
    }
  }
}

LCV_FN void htr_pubkey(h256& r, const uint8_t* pk) {
  h256 a, b;
  ld_chunk(a, pk);
  LCV_UNROLL for (int i = 0; i < 4; ++i) b.w[i] = bswap32(*(const uint32_t*)(pk + 32 + 4 * i));
  LCV_UNROLL for (int i = 4; i < 8; ++i) b.w[i] = 0;
  hash_pair(r, a, b);
}

// hash_tree_root(SyncCommittee): 512 pubkey roots -> depth-9 tree, then H(root || HTR(aggregate))
LCV_FN void htr_sync_committee(h256& root, const uint8_t* sc) {
  h256 s[10], node;
  LCV_NOUNROLL for (uint32_t j = 0; j < 512; ++j) {
    htr_pubkey(node, sc + 48 * j);
    merkle_push<0>(s, node, j);
  }
  h256 agg;
  htr_pubkey(agg, sc + 48 * 512);
  hash_pair(root, s[9], agg);
}

// compute_fork_version (its fork cascade, sync-protocol.md:461)
LCV_FN uint32_t fork_version_word(uint64_t epoch, const NetConfig& c) {
  uint32_t v = c.fork_version[0];
  LCV_UNROLL for (int k = 0; k < 4; ++k)
    if (epoch >= c.fork_epoch[k]) v = c.fork_version[k + 1];
  return v;
}

// compute_signing_root(attested.beacon, compute_domain(DOMAIN_SYNC_COMMITTEE, fork_version, gvr))
// (sync-protocol.md:460-463)
LCV_FN void signing_root(h256& out, const uint8_t* att_beacon, uint64_t signature_slot, const h256& gvr,
                         const NetConfig& cfg) {
  const uint64_t fslot = (signature_slot > 1 ? signature_slot : 1) - 1;
  h256 ver, fdr, dom, obj;
  h256_zero(ver);
  ver.w[0] = fork_version_word(epoch_of_slot(fslot, cfg), cfg);
  hash_pair(fdr, ver, gvr);
  dom.w[0] = cfg.domain_sync_committee;
  LCV_UNROLL for (int i = 1; i < 8; ++i) dom.w[i] = fdr.w[i - 1];
  htr_beacon(obj, att_beacon);
  hash_pair(out, obj, dom);
}

}  // namespace lcv
