// SSZ wire decode of light-client messages into the packed SoA rows of include/lcv.h.
//
// Containers (reference sync-protocol.md:96-101 LightClientHeader, :120-133 LightClientUpdate,
// :138-148 LightClientFinalityUpdate, :153-160 LightClientOptimisticUpdate; Req/Resp and gossip
// payloads p2p-interface.md) in SSZ wire form: fixed parts in field order, 4-byte little-endian
// offsets for the variable-size fields (every LightClientHeader, because its ExecutionPayloadHeader
// ends in extra_data: ByteList[32]).  Decoding is strict, as upstream SSZ deserialisation is: the
// first offset must equal the fixed size, offsets are monotonic and in bounds, no trailing bytes,
// extra_data <= 32 bytes.  A malformed message yields status 1 and an all-zero row.
//
// Finality / optimistic updates become the LightClientUpdate the reference builds from them
// (sync-protocol.md:563-571 / :582-590): default next_sync_committee, zero next-committee branch,
// and for optimistic updates a default finalized header and zero finality branch.
//
// Distinct next_sync_committee values are deduplicated by content (the device computes
// HTR(SyncCommittee) once per pool row): pool_src[k] = byte offset in `buf` of pool row k's first
// occurrence, or UINT64_MAX for SyncCommittee() (all zero).  Pure host code, no device work.
#include <cstdint>
#include <cstring>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/lcv.h"

namespace {

constexpr uint64_t kCommittee = 24624, kBeacon = 112, kExecRec = 832, kExecBranch = 128;
constexpr uint64_t kNscBranch = 160, kFinBranch = 192, kBits = 64, kSig = 96;
constexpr uint64_t kHeaderFixed = kBeacon + 4 + kExecBranch;  // 244
constexpr uint64_t kExtraOffPos = 436;                        // extra_data offset inside the exec header
constexpr uint64_t kMaxExtra = 32;

inline uint32_t rd32(const uint8_t* p) { uint32_t v; std::memcpy(&v, p, 4); return v; }

// ExecutionPayloadHeader (Deneb 17 fields / Capella 15) -> 832 B record (layout: include/lcv.h)
bool decode_exec(const uint8_t* p, uint64_t len, bool deneb, uint8_t* rec) {
  const uint64_t fixed = deneb ? 584 : 568;
  if (len < fixed || rd32(p + kExtraOffPos) != fixed) return false;
  const uint64_t elen = len - fixed;
  if (elen > kMaxExtra) return false;
  std::memset(rec, 0, kExecRec);
  uint64_t o = 0;
  auto chunk = [&](int leaf, uint64_t n) { std::memcpy(rec + 32 * leaf, p + o, n); o += n; };
  chunk(0, 32);                                   // parent_hash
  chunk(1, 20);                                   // fee_recipient
  chunk(2, 32);                                   // state_root
  chunk(3, 32);                                   // receipts_root
  std::memcpy(rec + 544, p + o, 256); o += 256;   // logs_bloom
  chunk(5, 32);                                   // prev_randao
  chunk(6, 8); chunk(7, 8); chunk(8, 8); chunk(9, 8);  // block_number, gas_limit, gas_used, timestamp
  o += 4;                                         // extra_data offset (checked above)
  chunk(11, 32);                                  // base_fee_per_gas (uint256 LE)
  chunk(12, 32);                                  // block_hash
  chunk(13, 32);                                  // transactions_root
  chunk(14, 32);                                  // withdrawals_root
  if (deneb) { chunk(15, 8); chunk(16, 8); }      // blob_gas_used, excess_blob_gas
  std::memcpy(rec + 32 * 10, p + fixed, elen);    // extra_data
  const uint32_t e32 = (uint32_t)elen;
  std::memcpy(rec + 800, &e32, 4);
  return true;
}

// LightClientHeader: beacon (112) | offset(execution) | execution_branch (128) | execution
bool decode_header(const uint8_t* p, uint64_t len, bool deneb, uint8_t* beacon, uint8_t* rec, uint8_t* branch) {
  if (len < kHeaderFixed || rd32(p + kBeacon) != kHeaderFixed) return false;
  if (!decode_exec(p + kHeaderFixed, len - kHeaderFixed, deneb, rec)) return false;
  std::memcpy(beacon, p, kBeacon);
  std::memcpy(branch, p + kBeacon + 4, kExecBranch);
  return true;
}

struct Row {
  const lcv_update_batch* b;
  uint64_t i;
  uint8_t* at(const uint8_t* col, uint64_t w) const { return const_cast<uint8_t*>(col) + i * w; }
};

void zero_row(const Row& r) {
  const lcv_update_batch* b = r.b;
  std::memset(r.at(b->attested.beacon, kBeacon), 0, kBeacon);
  std::memset(r.at(b->attested.execution, kExecRec), 0, kExecRec);
  std::memset(r.at(b->attested.exec_branch, kExecBranch), 0, kExecBranch);
  std::memset(r.at(b->finalized.beacon, kBeacon), 0, kBeacon);
  std::memset(r.at(b->finalized.execution, kExecRec), 0, kExecRec);
  std::memset(r.at(b->finalized.exec_branch, kExecBranch), 0, kExecBranch);
  std::memset(r.at(b->nsc_branch, kNscBranch), 0, kNscBranch);
  std::memset(r.at(b->finality_branch, kFinBranch), 0, kFinBranch);
  std::memset(r.at(b->sync_bits, kBits), 0, kBits);
  std::memset(r.at(b->sync_signature, kSig), 0, kSig);
  const_cast<uint64_t*>(b->signature_slot)[r.i] = 0;
}

enum { FORK_DENEB = 0, FORK_CAPELLA = 1, FORK_ALTAIR = 2 };

// Altair-format messages (ALTAIR .. BELLATRIX fork versions, p2p-interface.md:82-85, 112-115, 157-160,
// 197-200): LightClientHeader = {beacon} is fixed-size, so every container is fixed-size.  The rows
// are the Capella upgrade of the data (upgrade_lc_header_to_capella: empty execution and branch).
bool decode_one_altair(const uint8_t* p, uint64_t len, int kind, const Row& r, uint64_t* committee) {
  const lcv_update_batch* b = r.b;
  const uint64_t size = kind == 0 ? kBeacon + kCommittee + kNscBranch + kBeacon + kFinBranch + kBits + kSig + 8
                        : kind == 1 ? kBeacon + kBeacon + kFinBranch + kBits + kSig + 8
                                    : kBeacon + kBits + kSig + 8;
  if (len != size) return false;
  uint64_t pos = 0;
  std::memcpy(r.at(b->attested.beacon, kBeacon), p, kBeacon);
  pos += kBeacon;
  if (kind == 0) {
    *committee = pos;
    pos += kCommittee;
    std::memcpy(r.at(b->nsc_branch, kNscBranch), p + pos, kNscBranch);
    pos += kNscBranch;
  }
  if (kind != 2) {
    std::memcpy(r.at(b->finalized.beacon, kBeacon), p + pos, kBeacon);
    pos += kBeacon;
    std::memcpy(r.at(b->finality_branch, kFinBranch), p + pos, kFinBranch);
    pos += kFinBranch;
  }
  std::memcpy(r.at(b->sync_bits, kBits), p + pos, kBits);
  pos += kBits;
  std::memcpy(r.at(b->sync_signature, kSig), p + pos, kSig);
  pos += kSig;
  uint64_t slot;
  std::memcpy(&slot, p + pos, 8);
  const_cast<uint64_t*>(b->signature_slot)[r.i] = slot;
  return true;
}

// Decodes one message into row r; *committee = offset (within the message) of next_sync_committee,
// or UINT64_MAX when the message carries none.
bool decode_one(const uint8_t* p, uint64_t len, int kind, int fork, const Row& r, uint64_t* committee) {
  const lcv_update_batch* b = r.b;
  *committee = UINT64_MAX;
  if (fork == FORK_ALTAIR) return decode_one_altair(p, len, kind, r, committee);
  const bool deneb = fork == FORK_DENEB;
  uint64_t fixed, att_off_pos, fin_off_pos = 0, pos;
  if (kind == 0) fixed = 4 + kCommittee + kNscBranch + 4 + kFinBranch + kBits + kSig + 8;  // 25152
  else if (kind == 1) fixed = 4 + 4 + kFinBranch + kBits + kSig + 8;                       // 368
  else fixed = 4 + kBits + kSig + 8;                                                       // 172
  if (len < fixed || rd32(p) != fixed) return false;
  att_off_pos = 0;
  pos = 4;
  if (kind == 0) {
    *committee = pos;
    pos += kCommittee;
    std::memcpy(r.at(b->nsc_branch, kNscBranch), p + pos, kNscBranch);
    pos += kNscBranch;
  }
  if (kind != 2) {
    fin_off_pos = pos;
    pos += 4;
    std::memcpy(r.at(b->finality_branch, kFinBranch), p + pos, kFinBranch);
    pos += kFinBranch;
  }
  std::memcpy(r.at(b->sync_bits, kBits), p + pos, kBits);
  pos += kBits;
  std::memcpy(r.at(b->sync_signature, kSig), p + pos, kSig);
  pos += kSig;
  uint64_t slot;
  std::memcpy(&slot, p + pos, 8);
  const_cast<uint64_t*>(b->signature_slot)[r.i] = slot;
  const uint64_t a0 = rd32(p + att_off_pos);
  const uint64_t a1 = kind == 2 ? len : rd32(p + fin_off_pos);
  if (a1 < a0 || a1 > len) return false;
  if (!decode_header(p + a0, a1 - a0, deneb, r.at(b->attested.beacon, kBeacon),
                     r.at(b->attested.execution, kExecRec), r.at(b->attested.exec_branch, kExecBranch)))
    return false;
  if (kind != 2 &&
      !decode_header(p + a1, len - a1, deneb, r.at(b->finalized.beacon, kBeacon),
                     r.at(b->finalized.execution, kExecRec), r.at(b->finalized.exec_branch, kExecBranch)))
    return false;
  return true;
}

// Dedup key of a committee: a hash of its first pubkey and its aggregate_pubkey (96 sampled bytes);
// every key hit is confirmed by a full 24,624-byte compare, so the sample only has to spread rows.
uint64_t committee_key(const uint8_t* p) {
  uint64_t h = 0x9e3779b97f4a7c15ull;
  auto mix = [&](const uint8_t* q) {
    for (int k = 0; k < 48; k += 8) {
      uint64_t w;
      std::memcpy(&w, q + k, 8);
      h = (h ^ w) * 0xff51afd7ed558ccdull;
      h ^= h >> 29;
    }
  };
  mix(p);
  mix(p + kCommittee - 48);
  return h;
}

bool all_zero(const uint8_t* p, uint64_t n) {  // n multiple of 8
  for (uint64_t k = 0; k < n; k += 512) {
    uint64_t acc = 0;
    const uint64_t e = k + 512 < n ? k + 512 : n;
    for (uint64_t j = k; j < e; j += 8) {
      uint64_t w;
      std::memcpy(&w, p + j, 8);
      acc |= w;
    }
    if (acc) return false;
  }
  return true;
}

// rows are independent: split [0, n) over host threads (the batch path; small batches stay inline)
template <class Fn> void parallel_rows(uint64_t n, Fn fn) {
  unsigned t = std::thread::hardware_concurrency();
  t = t < 1 ? 1 : (t > 16 ? 16 : t);
  if (n < 1024 || t == 1) { fn(0, n); return; }
  std::vector<std::thread> pool;
  const uint64_t step = (n + t - 1) / t;
  for (unsigned k = 0; k < t; ++k) {
    const uint64_t lo = k * step, hi = lo + step < n ? lo + step : n;
    if (lo < hi) pool.emplace_back(fn, lo, hi);
  }
  for (auto& th : pool) th.join();
}

}  // namespace

// the batch decode; fork_of(i) gives message i's fork (one per call, or one per Req/Resp chunk)
template <class ForkOf>
static int decode_updates(const uint8_t* buf, const uint64_t* offsets, const uint64_t* lengths, uint64_t n, int kind,
                          ForkOf fork_of, const lcv_update_batch* out, uint64_t* pool_src, uint64_t* npool_out,
                          uint8_t* status) {
  if ((n && (!buf || !offsets || !lengths || !out || !pool_src || !status)) || !npool_out) return LCV_EINVAL;
  if (kind < 0 || kind > 2) return LCV_EINVAL;
  if (n && (!out->attested.beacon || !out->attested.execution || !out->attested.exec_branch ||
            !out->finalized.beacon || !out->finalized.execution || !out->finalized.exec_branch ||
            !out->nsc_index || !out->nsc_branch || !out->finality_branch || !out->sync_bits ||
            !out->sync_signature || !out->signature_slot))
    return LCV_EINVAL;
  constexpr uint64_t kNone = UINT64_MAX;
  std::vector<uint64_t> csrc(n, kNone), key(n, 0);  // committee offset in buf (kNone: SyncCommittee())
  // 1. decode every row (parallel)
  parallel_rows(n, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t i = lo; i < hi; ++i) {
      const Row r{out, i};
      zero_row(r);
      uint64_t c = kNone;
      const int fork = fork_of(i);
      const bool ok = fork >= FORK_DENEB && fork <= FORK_ALTAIR &&
                      decode_one(buf + offsets[i], lengths[i], kind, fork, r, &c);
      status[i] = ok ? 0 : 1;
      if (!ok) {
        zero_row(r);
        continue;
      }
      if (c != kNone && !all_zero(buf + offsets[i] + c, kCommittee)) {
        csrc[i] = offsets[i] + c;
        key[i] = committee_key(buf + csrc[i]);
      }
    }
  });
  // 2. pool rows in first-occurrence order; each row tentatively takes the first pool row of its key
  uint32_t* nsc_index = const_cast<uint32_t*>(out->nsc_index);
  std::unordered_map<uint64_t, std::vector<uint32_t>> seen;
  uint64_t npool = 0;
  int64_t zero_ix = -1;  // pool row of SyncCommittee(), created on first use
  for (uint64_t i = 0; i < n; ++i) {
    if (csrc[i] == kNone) {
      if (zero_ix < 0) { zero_ix = (int64_t)npool; pool_src[npool++] = kNone; }
      nsc_index[i] = (uint32_t)zero_ix;
      continue;
    }
    std::vector<uint32_t>& cands = seen[key[i]];
    if (cands.empty()) { cands.push_back((uint32_t)npool); pool_src[npool++] = csrc[i]; }
    nsc_index[i] = cands[0];
  }
  // 3. confirm every tentative assignment with a full compare (parallel)
  std::vector<uint8_t> mismatch(n, 0);
  parallel_rows(n, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t i = lo; i < hi; ++i)
      if (csrc[i] != kNone && pool_src[nsc_index[i]] != csrc[i])
        mismatch[i] = std::memcmp(buf + pool_src[nsc_index[i]], buf + csrc[i], kCommittee) != 0;
  });
  // 4. sampled-key collisions (distinct committees sharing first and aggregate pubkeys): exact search
  for (uint64_t i = 0; i < n; ++i) {
    if (!mismatch[i]) continue;
    std::vector<uint32_t>& cands = seen[key[i]];
    int64_t hit = -1;
    for (uint32_t k : cands)
      if (std::memcmp(buf + pool_src[k], buf + csrc[i], kCommittee) == 0) { hit = k; break; }
    if (hit < 0) { hit = (int64_t)npool; cands.push_back((uint32_t)npool); pool_src[npool++] = csrc[i]; }
    nsc_index[i] = (uint32_t)hit;
  }
  *npool_out = npool;
  return LCV_OK;
}

extern "C" int lcv_ssz_decode_updates(const uint8_t* buf, const uint64_t* offsets, const uint64_t* lengths,
                                      uint64_t n, int kind, int fork, const lcv_update_batch* out,
                                      uint64_t* pool_src, uint64_t* npool_out, uint8_t* status) {
  if (fork < FORK_DENEB || fork > FORK_ALTAIR) return LCV_EINVAL;
  return decode_updates(buf, offsets, lengths, n, kind, [fork](uint64_t) { return fork; }, out, pool_src, npool_out,
                        status);
}

extern "C" int lcv_ssz_decode_updates_mixed(const uint8_t* buf, const uint64_t* offsets, const uint64_t* lengths,
                                            uint64_t n, int kind, const uint8_t* forks, const lcv_update_batch* out,
                                            uint64_t* pool_src, uint64_t* npool_out, uint8_t* status) {
  if (n && !forks) return LCV_EINVAL;
  return decode_updates(buf, offsets, lengths, n, kind, [forks](uint64_t i) { return (int)forks[i]; }, out, pool_src,
                        npool_out, status);
}

// LightClientBootstrap (sync-protocol.md:109-115): header (offset) | current_sync_committee (24624) |
// current_sync_committee_branch (5 x 32) | header.  Input of initialize_light_client_store (:351-373).
extern "C" int lcv_ssz_decode_bootstrap(const uint8_t* buf, uint64_t len, int fork, uint8_t* beacon112,
                                        uint8_t* exec832, uint8_t* exec_branch128, uint8_t* committee24624,
                                        uint8_t* committee_branch160, uint8_t* status) {
  if (!buf || !beacon112 || !exec832 || !exec_branch128 || !committee24624 || !committee_branch160 || !status)
    return LCV_EINVAL;
  if (fork < FORK_DENEB || fork > FORK_ALTAIR) return LCV_EINVAL;
  constexpr uint64_t fixed = 4 + kCommittee + kNscBranch;  // 24788
  bool ok;
  uint64_t cpos = 4;
  if (fork == FORK_ALTAIR) {  // header (112, fixed) | committee | branch
    ok = len == kBeacon + kCommittee + kNscBranch;
    if (ok) {
      std::memcpy(beacon112, buf, kBeacon);
      std::memset(exec832, 0, kExecRec);
      std::memset(exec_branch128, 0, kExecBranch);
    }
    cpos = kBeacon;
  } else {
    ok = len >= fixed && rd32(buf) == fixed &&
         decode_header(buf + fixed, len - fixed, fork == FORK_DENEB, beacon112, exec832, exec_branch128);
  }
  if (ok) {
    std::memcpy(committee24624, buf + cpos, kCommittee);
    std::memcpy(committee_branch160, buf + cpos + kCommittee, kNscBranch);
  } else {
    std::memset(beacon112, 0, kBeacon);
    std::memset(exec832, 0, kExecRec);
    std::memset(exec_branch128, 0, kExecBranch);
    std::memset(committee24624, 0, kCommittee);
    std::memset(committee_branch160, 0, kNscBranch);
  }
  *status = ok ? 0 : 1;
  return LCV_OK;
}
