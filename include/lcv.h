/* lcv.h — C ABI of liblcv.so, the MI355X (gfx950) batched light-client verifier.
 *
 * Drop-in boundary for the hot path of Inspector-Butters/light-client-consensus-specs:
 *   validate_light_client_update(store, update, current_slot, genesis_validators_root)
 *       reference sync-protocol.md:386-465           -> lcv_set_store + lcv_validate_updates
 *   bls.FastAggregateVerify(pubkeys, message, signature)
 *       reference call site sync-protocol.md:464      -> lcv_fast_aggregate_verify(_batch)
 *   is_valid_merkle_branch(leaf, branch, depth, index, root)
 *       reference call sites sync-protocol.md:234,356,428,443 -> lcv_merkle_branch_batch
 *   hash_tree_root(SyncCommittee)
 *       reference call site sync-protocol.md:444      -> lcv_htr_sync_committee_batch
 *
 * Conventions: plain pointers and sizes, caller owns every host buffer, the library copies in and
 * out.  Every function returns 0 (LCV_OK) or a negative lcv_status; lcv_last_error() explains.
 * No C++ exception crosses the ABI.  One lcv_ctx per device, not shared between threads.
 * Byte layouts of the packed update batch (structure of arrays, one row per update) are given
 * next to lcv_update_batch and in DESIGN.md.
 */
#ifndef LCV_H
#define LCV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LCV_SYNC_COMMITTEE_SIZE 512
#define LCV_PUBKEY_BYTES 48
#define LCV_SIGNATURE_BYTES 96
#define LCV_SYNC_COMMITTEE_BYTES 24624 /* SSZ SyncCommittee: 512 x 48 B pubkeys + 48 B aggregate */
#define LCV_BEACON_HEADER_BYTES 112    /* SSZ BeaconBlockHeader */
#define LCV_EXEC_RECORD_BYTES 832      /* packed ExecutionPayloadHeader, see below */
#define LCV_EXEC_BRANCH_BYTES 128      /* ExecutionBranch 4 x 32 */
#define LCV_NSC_BRANCH_BYTES 160       /* NextSyncCommitteeBranch 5 x 32 */
#define LCV_FINALITY_BRANCH_BYTES 192  /* FinalityBranch 6 x 32 */
#define LCV_SYNC_BITS_BYTES 64         /* SSZ Bitvector[512] */

enum lcv_status { LCV_OK = 0, LCV_EINVAL = -1, LCV_EDEVICE = -2, LCV_ENOMEM = -3, LCV_ESTATE = -4 };

/* reason codes: k = the k-th assert of validate_light_client_update in source order */
enum lcv_reason {
  LCV_VALID = 0,
  LCV_R_PARTICIPANTS = 1,            /* :392 */
  LCV_R_ATTESTED_HEADER = 2,         /* :395 */
  LCV_R_SLOT_ORDER = 3,              /* :398 */
  LCV_R_SIG_PERIOD_NEXT_KNOWN = 4,   /* :402 */
  LCV_R_SIG_PERIOD_NEXT_UNKNOWN = 5, /* :404 */
  LCV_R_NOT_RELEVANT = 6,            /* :411-414 */
  LCV_R_FINALIZED_NOT_EMPTY = 7,     /* :420 */
  LCV_R_FINALIZED_GENESIS = 8,       /* :423 */
  LCV_R_FINALIZED_HEADER = 9,        /* :426 */
  LCV_R_FINALITY_BRANCH = 10,        /* :428-434 */
  LCV_R_NSC_NOT_EMPTY = 11,          /* :439 */
  LCV_R_NSC_MISMATCH = 12,           /* :442 */
  LCV_R_NSC_BRANCH = 13,             /* :443-449 */
  LCV_R_SIGNATURE = 14               /* :464 */
};

typedef struct lcv_ctx lcv_ctx;
typedef struct lcv_dbatch lcv_dbatch;

/* Packed ExecutionPayloadHeader record (832 B): 17 SSZ leaf chunks of 32 B in field order
 * (parent_hash, fee_recipient (20 B + 12 zero), state_root, receipts_root, [leaf 4 unused: zero],
 * prev_randao, block_number, gas_limit, gas_used, timestamp (uint64 LE + 24 zero),
 * extra_data (zero padded), base_fee_per_gas (uint256 LE), block_hash, transactions_root,
 * withdrawals_root, blob_gas_used, excess_blob_gas), then logs_bloom (256 B) at offset 544,
 * extra_data length (uint32 LE) at 800, 28 zero bytes.  All-zero == ExecutionPayloadHeader(). */
typedef struct lcv_header_cols {
  const uint8_t* beacon;      /* n x 112 */
  const uint8_t* execution;   /* n x 832 */
  const uint8_t* exec_branch; /* n x 128 */
} lcv_header_cols;

typedef struct lcv_update_batch {
  lcv_header_cols attested;
  lcv_header_cols finalized;
  const uint8_t* nsc_pool;        /* npool x 24624: distinct next_sync_committee values */
  const uint32_t* nsc_index;      /* n: pool row holding update i's next_sync_committee */
  const uint8_t* nsc_branch;      /* n x 160 */
  const uint8_t* finality_branch; /* n x 192 */
  const uint8_t* sync_bits;       /* n x 64 */
  const uint8_t* sync_signature;  /* n x 96 */
  const uint64_t* signature_slot; /* n */
  uint64_t n;
  uint64_t npool;
} lcv_update_batch;

/* ---- context */
int lcv_device_count(int* out);
int lcv_init(int device, lcv_ctx** out);
void lcv_destroy(lcv_ctx* ctx);
const char* lcv_last_error(const lcv_ctx* ctx);

/* ---- network configuration, runtime (mainnet by default): the values sync-protocol.md reads from
 * the preset / config — SLOTS_PER_EPOCH and EPOCHS_PER_SYNC_COMMITTEE_PERIOD (periods, UPDATE_TIMEOUT),
 * fork_epochs4 = ALTAIR, BELLATRIX, CAPELLA, DENEB _FORK_EPOCH (is_valid_light_client_header :220-240,
 * get_lc_execution_root :186-214, compute_fork_version :461), fork_versions20 = GENESIS, ALTAIR,
 * BELLATRIX, CAPELLA, DENEB _FORK_VERSION (5 x 4 B), domain_sync_committee4 = DOMAIN_SYNC_COMMITTEE
 * (:462).  Fork epochs non-decreasing.  Applies to every later validate / bootstrap call on ctx.
 * SYNC_COMMITTEE_SIZE is the mainnet preset's 512 (the packed layouts above). */
int lcv_set_config(lcv_ctx* ctx, uint64_t slots_per_epoch, uint64_t epochs_per_sync_committee_period,
                   const uint64_t* fork_epochs4, const uint8_t* fork_versions20, const uint8_t* domain_sync_committee4);

/* ---- validate_light_client_update (sync-protocol.md:386-465) against one store snapshot.
 * The store's two committees (SSZ SyncCommittee bytes; an all-zero next committee means
 * "not known", sync-protocol.md:316-317) are decoded and KeyValidated once, device resident.
 * key_status_out (optional, 1024 B): 0 valid key, 2 invalid. */
int lcv_set_store(lcv_ctx* ctx, uint64_t finalized_slot, const uint8_t* current_sync_committee,
                  const uint8_t* next_sync_committee, uint8_t* key_status_out);
/* host batch in, verdict (1 = valid) and reason code (lcv_reason) out, one byte per update */
int lcv_validate_updates(lcv_ctx* ctx, const lcv_update_batch* batch, uint64_t current_slot,
                         const uint8_t* genesis_validators_root, uint8_t* verdict_out, uint8_t* reason_out);
/* device-resident batches: upload once, validate many times (timed region excludes the upload) */
int lcv_batch_upload(lcv_ctx* ctx, const lcv_update_batch* batch, lcv_dbatch** out);
void lcv_batch_free(lcv_ctx* ctx, lcv_dbatch* b);
int lcv_validate_resident(lcv_ctx* ctx, lcv_dbatch* b, uint64_t current_slot, const uint8_t* genesis_validators_root,
                          uint8_t* verdict_out, uint8_t* reason_out);
/* same, verdicts written to a DEVICE buffer of n bytes (for an RCCL all-gather); no host copy */
int lcv_validate_resident_dev(lcv_ctx* ctx, lcv_dbatch* b, uint64_t current_slot,
                              const uint8_t* genesis_validators_root, uint8_t* verdict_dev);
/* Several batches in flight (multi-buffered serving loop; no reference counterpart: the reference
 * validates one update per call, sync-protocol.md:386).  lcv_validate_resident_async enqueues the whole
 * pipeline for b (at most 65536 updates) on the two HIP streams of work-space slot `slot` (0..7) and
 * returns without waiting; lcv_slot_wait waits for that slot and copies the first n verdicts / reason
 * codes out (either pointer may be NULL).  A slot's next batch starts on the device after its previous
 * one; alternate the slots and wait for a slot before reading or reusing it.  Synchronous calls use
 * slot 0 (and, for batches of several 64k chunks, every slot): wait for pending slots before them. */
int lcv_validate_resident_async(lcv_ctx* ctx, lcv_dbatch* b, uint64_t current_slot,
                                const uint8_t* genesis_validators_root, int slot);
int lcv_slot_wait(lcv_ctx* ctx, int slot, uint64_t n, uint8_t* verdict_out, uint8_t* reason_out);
/* Host-input serving entry (the per-batch form of lcv_validate_updates; callers sync-protocol.md:512 per
 * update and the gossip / Req/Resp ingress p2p-interface.md:69,99 per batch): the batch (at most 65536
 * updates) is copied into slot `slot`'s pinned staging buffer, uploaded by one DMA on the slot's stream
 * (overlapping the other slots' kernels), validated, and its verdicts / reasons copied back to pinned
 * memory — all enqueued without waiting; lcv_slot_wait(slot) waits and copies them out.  The caller's
 * buffers may be reused as soon as the call returns. */
int lcv_validate_async(lcv_ctx* ctx, const lcv_update_batch* batch, uint64_t current_slot,
                       const uint8_t* genesis_validators_root, int slot);
/* multi-GPU form of lcv_slot_wait: after slot `slot`'s batch (n <= per_rank rows), all-gather every rank's
 * verdict bytes over RCCL (rank-major, each slice zero padded to per_rank) into verdict_all_out
 * (nranks * per_rank bytes) and wait.  Collective: every rank calls it in the same order. */
int lcv_slot_allgather(lcv_ctx* ctx, int slot, uint64_t n, uint64_t per_rank, uint8_t* verdict_all_out);
/* Execution shape of lcv_validate_*: each 64k-update chunk is cut into `chunks` slices whose whole
 * stage chains run on min(streams, 4) HIP streams, so different slices' kernels overlap.  streams = 1
 * (default) runs the stages one after another over the whole chunk (per-stage timings available);
 * verdicts are identical either way.  Performance knob only, no reference counterpart. */
int lcv_set_pipeline(lcv_ctx* ctx, int streams, int chunks);
/* Latency mode for small batches (the reference's per-update usage: validate_light_client_update and
 * bls.FastAggregateVerify once per update, sync-protocol.md:512, :464): calls whose batch (or chunk) has
 * at most max_rows rows run
 *   - the SOP programs (hash_to_G2 tail, final exponentiation) on the fan engine — an op's K products on
 *     K lanes and its reduction and tail on a 16-lane row, one update per block — instead of one op per lane,
 *   - both Miller line walks and the accumulation as ONE fan-engine program (lines through LDS), and
 *   - the SSWU maps and the signature decoding on their one-item-per-wave twins (each square-root
 *     product spread over the 64 lanes of a wave).
 * Results are identical to the batch engine's (bit for bit).  Default 64: one update 2.8 ms through
 * lcv_validate_updates on the MI355X (6.0 ms on the batch engine); 0 = the batch engine
 * always.  Performance knob only. */
int lcv_set_latency_mode(lcv_ctx* ctx, uint64_t max_rows);
/* test hook: which engines ran since the last reset (reset != 0 clears after reading).  out8[0] fan-engine
 * SOP launches, [1] batch-engine SOP launches, [2] one-item-per-wave twin launches (SSWU / signature),
 * [3] one-lane-per-item SSWU / signature launches, [4..7] items per wave of the last batch-engine launch of
 * the line walk, Miller accumulation, final exponentiation, hash_to_G2 tail (0 = not launched) */
int lcv_debug_engine_log(lcv_ctx* ctx, uint64_t* out8, int reset);
/* kernel time of the last validate call: total and per stage (ms); names via lcv_stage_name
 * (stage times are recorded by the serial shape only: zero under a multi-stream pipeline) */
int lcv_last_timings(lcv_ctx* ctx, float* ms_out, int max_stages, int* nstages);
const char* lcv_stage_name(int stage);

/* ---- multi-GPU: one process and one context per GPU, updates sharded by contiguous
 * index range, RCCL over xGMI for the one collective (the per-update verdict all-gather).  No reference
 * counterpart: the reference is single-process (p2p-interface.md:69,99 is the ingress producing batches).
 * lcv_comm_unique_id: rank 0 makes the 128-byte id (ncclGetUniqueId) and hands it to every rank. */
int lcv_comm_unique_id(uint8_t* id128);
int lcv_comm_init(lcv_ctx* ctx, int nranks, int rank, const uint8_t* id128);
int lcv_comm_destroy(lcv_ctx* ctx);
/* ranks in the communicator as RCCL reports them (ncclCommCount) */
int lcv_comm_count(lcv_ctx* ctx, int* nranks_out);
/* validate this rank's resident shard (n <= per_rank), all-gather every rank's per_rank verdict bytes
 * (zero padded) into verdict_all_out (nranks * per_rank bytes, rank-major) */
int lcv_validate_sharded(lcv_ctx* ctx, lcv_dbatch* b, uint64_t current_slot, const uint8_t* genesis_validators_root,
                         uint64_t per_rank, uint8_t* verdict_all_out);
/* max over ranks of one double (in place); doubles as a barrier */
int lcv_comm_allreduce_max(lcv_ctx* ctx, double* inout);
/* Failure containment (a failed GPU's shard is re-run).  Every collective completes within
 * the communicator timeout (default 60 s) or the call fails with LCV_EDEVICE: the wait polls the stream and
 * RCCL's asynchronous error (ncclCommGetAsyncError), so a rank whose peer died or hangs returns instead of
 * blocking in ncclAllGather.  The communicator is then marked failed (collectives refused, LCV_ESTATE) until
 * the surviving ranks all call lcv_comm_shrink with the same list of excluded ranks (ncclCommShrink with
 * NCCL_SHRINK_ABORT: the failed parent's operations are terminated, the survivors renumbered in rank
 * order; new_rank / new_nranks out), or lcv_comm_abort (ncclCommAbort) drops it. */
int lcv_comm_set_timeout(lcv_ctx* ctx, double seconds);
int lcv_comm_shrink(lcv_ctx* ctx, const int* exclude_ranks, int nexclude, int* new_rank, int* new_nranks);
int lcv_comm_abort(lcv_ctx* ctx);

/* ---- bls.FastAggregateVerify (sync-protocol.md:464); py_ecc semantics (every key KeyValidated).
 * Any number of pubkeys (npk = 0 -> False), a message of any length (the light-client call site passes
 * a 32-byte signing root; other lengths take the device's byte-streamed expand_message_xmd). */
int lcv_fast_aggregate_verify(lcv_ctx* ctx, const uint8_t* pubkeys48, uint64_t npk, const uint8_t* msg,
                              uint64_t msg_len, const uint8_t* sig96, int* result);
/* batched: committee table (ncomm x 512 x 48 B), per item committee id + participation bits */
int lcv_fast_aggregate_verify_batch(lcv_ctx* ctx, const uint8_t* committees, uint64_t ncomm,
                                    const uint32_t* committee_id, const uint8_t* bits64, const uint8_t* msg32,
                                    const uint8_t* sig96, uint64_t n, uint8_t* verdict_out);

/* ---- SSZ */
int lcv_merkle_branch_batch(lcv_ctx* ctx, const uint8_t* leaf32, const uint8_t* branch, uint32_t depth,
                            uint64_t index, const uint8_t* root32, uint64_t n, uint8_t* out);
int lcv_htr_sync_committee_batch(lcv_ctx* ctx, const uint8_t* committees, uint64_t n, uint8_t* roots32_out);
/* initialize_light_client_store's asserts (sync-protocol.md:353-362), one bootstrap per row (header rows
 * as lcv_header_cols, committee 24624 B, current_sync_committee_branch 5 x 32 B, trusted_block_root 32 B):
 * reason 0 ok, 1 header invalid (:353), 2 beacon root != trusted root (:354), 3 committee branch (:356) */
int lcv_bootstrap_check_batch(lcv_ctx* ctx, const uint8_t* beacon112, const uint8_t* exec832,
                              const uint8_t* exec_branch128, const uint8_t* committees, const uint8_t* committee_branch160,
                              const uint8_t* trusted_root32, uint64_t n, uint8_t* reason_out);

/* ---- SSZ wire decode (host only, no device work; csrc/lcv_wire.cpp).  Replaces the upstream SSZ
 * deserialisation of the reference's containers (sync-protocol.md:109-115 LightClientBootstrap,
 * :120-133 LightClientUpdate, :138-148 LightClientFinalityUpdate, :153-160 LightClientOptimisticUpdate)
 * as received over Req/Resp / gossip (p2p-interface.md).  kind: 0 update, 1 finality update,
 * 2 optimistic update (converted as sync-protocol.md:563-571 / :582-590 do); fork: 0 Deneb
 * ExecutionPayloadHeader (17 fields), 1 Capella (15), 2 Altair (LightClientHeader = beacon only; the
 * row is its Capella upgrade: empty execution and branch).  Message i = buf[offsets[i] .. + lengths[i]] ->
 * row i of `out` (caller-allocated columns of n rows; out->nsc_pool is ignored).  status[i] = 0 ok,
 * 1 malformed (row zeroed).  Distinct next_sync_committee values: pool row k is the committee at
 * buf + pool_src[k] (UINT64_MAX = SyncCommittee()), *npool_out rows (<= n + 1). */
int lcv_ssz_decode_updates(const uint8_t* buf, const uint64_t* offsets, const uint64_t* lengths, uint64_t n,
                           int kind, int fork, const lcv_update_batch* out, uint64_t* pool_src,
                           uint64_t* npool_out, uint8_t* status);
/* the same with a fork per message (a Req/Resp response's chunks each carry their own ForkDigest
 * context, p2p-interface.md:189-200, so one response may straddle a fork boundary) */
int lcv_ssz_decode_updates_mixed(const uint8_t* buf, const uint64_t* offsets, const uint64_t* lengths, uint64_t n,
                                 int kind, const uint8_t* forks, const lcv_update_batch* out, uint64_t* pool_src,
                                 uint64_t* npool_out, uint8_t* status);
int lcv_ssz_decode_bootstrap(const uint8_t* buf, uint64_t len, int fork, uint8_t* beacon112, uint8_t* exec832,
                             uint8_t* exec_branch128, uint8_t* committee24624, uint8_t* committee_branch160,
                             uint8_t* status);

/* ---- synthetic-data signer (producer side).  Secret keys 32 B big-endian. */
int lcv_sk_to_pk_batch(lcv_ctx* ctx, const uint8_t* sk32, uint64_t n, uint8_t* pk48_out);
int lcv_sign_batch(lcv_ctx* ctx, const uint8_t* sk32, const uint8_t* msg32, uint64_t n, uint8_t* sig96_out);

/* ---- parity-test entry points (intermediate values, canonical big-endian bytes) */
/* field ops on (a, b) < p: out per item = a*b, a+b, a-b, a^-1, sqrt_fp2(a + b u) (2 x 48); ok = sqrt exists */
/* test hook: rows per validate chunk (multiple of 64, <= 65536; default 65536) */
int lcv_debug_set_chunk(lcv_ctx* ctx, uint64_t rows);
/* test hook (host arithmetic only): allocates work-space slots 0 .. nslots-1 for `cap` rows and checks
 * (1) for slices of `slice` rows, that item j of each slice's work view is item base + j of the slot's
 * work space in every per-item field, element for element, as the kernels address them, and (2) that the
 * byte ranges of every field of every slot — the committee-pool fields (HTR roots and flags of a pool of 5
 * distinct committees) included — are pairwise disjoint.  LCV_EINVAL + lcv_last_error names the first
 * field that fails. */
int lcv_debug_work_check(lcv_ctx* ctx, uint64_t cap, uint64_t slice, int nslots);
/* test hook (device backend): hold work-space slot `slot`'s main stream with a kernel that waits for
 * lcv_debug_release_slots or max_seconds (<= 120), so that a collective behind it cannot complete */
int lcv_debug_hold_slot(lcv_ctx* ctx, int slot, double max_seconds);
int lcv_debug_release_slots(lcv_ctx* ctx);
/* build provenance: a hash of the sources liblcv.so was compiled from (tools/build_id.py: csrc/, include/,
 * tools/gen_sop.py, the Makefile), NUL-terminated into out (cap >= 17); LCV_EINVAL if cap is too small */
int lcv_build_id(char* out, uint64_t cap);
/* test hook: HIP events held by the context's stage-timing pool (bounded under asynchronous calls) */
int lcv_debug_event_pool(lcv_ctx* ctx, uint64_t* events_out);
int lcv_debug_fp(lcv_ctx* ctx, const uint8_t* a48, const uint8_t* b48, uint64_t n, uint8_t* out288, uint8_t* ok);
/* a^((p+1)/4) || a^((p-3)/4) (2 x 48 B) for a < p: the windowed sqrt exponentiations of decompression / SSWU */
int lcv_debug_fp_pow(lcv_ctx* ctx, const uint8_t* a48, uint64_t n, uint8_t* out96);
/* hash_to_G2(msg) affine (x0 || x1 || y0 || y1, 4 x 48 B); inf flag */
int lcv_debug_hash_to_g2(lcv_ctx* ctx, const uint8_t* msg32, uint64_t n, uint8_t* out192, uint8_t* inf);
/* signature decode + subgroup check: affine point + status (0 ok, 1 identity, 2 invalid) */
int lcv_debug_g2_decompress(lcv_ctx* ctx, const uint8_t* sig96, uint64_t n, uint8_t* out192, uint8_t* status);
/* masked aggregate (affine x || y) + status (0 ok, 1 identity, 2 invalid key among participants) */
int lcv_debug_aggregate(lcv_ctx* ctx, const uint8_t* committees, uint64_t ncomm, const uint32_t* committee_id,
                        const uint8_t* bits64, uint64_t n, uint8_t* out96, uint8_t* status);
/* e(P, Q)^3 after final exponentiation (12 x 48 B, coefficient order g0..g5 of w^i, each c0 || c1) */
int lcv_debug_pairing(lcv_ctx* ctx, const uint8_t* p96, const uint8_t* q192, uint64_t n, uint8_t* out576);

#ifdef __cplusplus
}
#endif
#endif /* LCV_H */
