/*
 * ygm.h -- C ABI of the MI355X batched Yjs update engine ("ygm" = Yjs GPU Merge).
 *
 * The drop-in boundary for Hocuspocus's persistence / sync hot path.  Plain
 * pointers and sizes only (no torch, no HIP types in signatures).  Each entry
 * point replaces a per-document yjs call that the reference makes one document
 * at a time on the Node event loop:
 *
 *   ygm_merge_v1           <- Y.mergeUpdates(updates)                  (yjs Y@37704; the
 *                             store path packages/extension-database/src/Database.ts:55-60
 *                             persists Y.encodeStateAsUpdate(doc); the GPU extension persists
 *                             mergeUpdates([snapshot, ...onChange updates]) instead,
 *                             packages/server/src/Hocuspocus.ts:244-277,417-447)
 *   ygm_diff_v1            <- Y.diffUpdate(update, stateVector)        (yjs Y@41210; the Step1 ->
 *                             Step2 reply of packages/server/src/MessageReceiver.ts:137-155)
 *   ygm_sv_from_update_v1  <- Y.encodeStateVectorFromUpdate(update)    (yjs Y@38304; the SV a
 *                             server sends in SyncStep1, packages/server/src/OutgoingMessage.ts:93-99)
 *
 * Byte-for-byte identical to yjs 13.6.26 by default; YGM_F_COMPAT_135 selects
 * the yjs 13.5.16 / lib0 0.2.42 behaviours.  A document whose
 * content yjs would re-encode (non-canonical Any/JSON) is
 * refused with YGM_ENONCANON instead of being silently copied.
 *
 * Error behaviour mirrors the reference: yjs throws per document; here the
 * batch call succeeds and the failing document carries a non-zero status
 * (the extension then rejects only that document's hook, Hocuspocus.ts:431-435).
 */
#ifndef YGM_H
#define YGM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- per-document status codes ------------------------------------------ */
#define YGM_OK 0
#define YGM_EMALFORMED 1   /* yjs throws: truncated input, bad UTF-8, unknown content/Any tag, bad JSON */
#define YGM_ERANGE 2       /* yjs throws "Integer out of Range": varuint > 2^53 */
#define YGM_ENONCANON 3    /* yjs would re-encode content (non-canonical Any/JSON): refused, not copied */
#define YGM_ESURROGATE 4   /* compat 13.5 only: lib0 0.2.42 throws writing a lone surrogate */
#define YGM_EDEPTH 5       /* Any/JSON nesting deeper than YGM_MAX_DEPTH */
#define YGM_ENOMEM 6
#define YGM_EDEVICE 7      /* HIP error / device fault */
#define YGM_EINVAL 8       /* bad call arguments */
#define YGM_EUNSUPPORTED 9 /* snapshot / step2 / contains only: the update repeats a client block or overlaps
                              structs (yjs's writers never do), or names a non-type item as a parent
                              -- the caller keeps its yjs path for that document */

#define YGM_MAX_DEPTH 32

/* ---- context flags -------------------------------------------------------- */
#define YGM_F_COMPAT_135 1u   /* delete-set clients in first-seen order; lone surrogate -> error */
#define YGM_F_FORCE_SEQ 2u    /* route every merge through the exact sequential kernel (testing) */
#define YGM_F_KEEP_SUB 4u     /* internal to ygm_sync_step2_v1: diffs keep each struct's parentSub bit (0x20) */
#define YGM_F_SNAP_STATE 16u  /* internal to ygm_contains_v1: such a state's snapshot is its integrated part alone
                                 (Y.snapshot(doc): the store's state vector and delete set) */

typedef struct ygm_ctx ygm_ctx;

/* Result of one host-API batch call.  Owned by the context (pinned host
 * memory); valid until the next call on the same context or ygm_close.
 * Document d's output is data[off[d] .. off[d]+len[d]) when status[d] ==
 * YGM_OK (len[d] = 0 otherwise); outputs are packed in document order.
 * The host API moves a batch in chunks of whole documents through two
 * stage streams (pinned staging, H2D of chunk i+1 beside the kernels of
 * chunk i, device-side packing, D2H of the packed outputs only); h2d_ms /
 * d2h_ms in ygm_stats_t are those copies' event times. */
typedef struct {
  const uint8_t *data;
  const uint64_t *off;
  const uint64_t *len;
  const int32_t *status;
  uint32_t n_docs;
  uint64_t data_bytes;
} ygm_result;

typedef struct {
  uint64_t calls, docs, updates;
  uint64_t bytes_in, bytes_out;       /* algorithmic bytes */
  uint64_t docs_fast, docs_seq;        /* documents finished by the general tiers (merge: wave / workgroup kernels;
                                          SV / diff: the exact per-document kernel) / by the sequential merge kernel */
  double kernel_ms, h2d_ms, d2h_ms;    /* cumulative, HIP-event timed */
  uint64_t docs_lean;                  /* documents finished by the lean kernels (merge: the debounce-log kernels; SV / diff:
                                          lane-per-document walker) */
  double lean_ms;                      /* HIP-event time of the lean kernel launches (part of kernel_ms): one span
                                          from the first launch after a finish to that finish */
  uint64_t lean_launches;              /* lean kernel launches timed in lean_ms */
  uint64_t docs_big;                   /* merges finished by the large-document ([snapshot, ...log]) kernel */
  uint64_t docs_lean_wide;             /* merges of docs_lean finished by the wide lean kernel (updates <= 64 B,
                                          documents <= 7 KB: the narrow kernel's deferrals) */
  uint64_t host_syncs;                 /* host waits on the device inside the calls (counter reads between the merge
                                          tiers, snapshot workspace sizing, ...): one per call for a batch the lean
                                          kernels finish, two when the general tiers are needed, more for the
                                          large-document and sequential tiers */
  uint64_t docs_pending;               /* snapshots of updates that leave pending structs / a pending delete set
                                          (finished by merging [state, pendingDs, pending structs] on the GPU) */
} ygm_stats_t;

/* Opens the engine on HIP device `device` (one context per GPU; contexts are
 * independent, not thread-safe: one batch in flight per context). */
int ygm_open(int device, uint32_t flags, ygm_ctx **out);
void ygm_close(ygm_ctx *ctx);

/* ---- host-memory batch API (what the N-API addon / ctypes binding call) ---
 * arena      concatenated V1 updates
 * upd_off    n_upd+1 byte offsets into arena
 * upd_doc    n_upd document ids, non-decreasing; updates of a document keep
 *            their order (the order of yjs's `updates` array) */
int ygm_merge_v1(ygm_ctx *ctx, const uint8_t *arena, const uint64_t *upd_off, const uint32_t *upd_doc,
                 uint32_t n_upd, uint32_t n_docs, ygm_result *out);
/* doc_off: n_docs+1 offsets of one update per document; sv_off: n_docs+1
 * offsets of one encoded state vector per document in sv_arena. */
int ygm_diff_v1(ygm_ctx *ctx, const uint8_t *arena, const uint64_t *doc_off, const uint8_t *sv_arena,
                const uint64_t *sv_off, uint32_t n_docs, ygm_result *out);
int ygm_sv_from_update_v1(ygm_ctx *ctx, const uint8_t *arena, const uint64_t *doc_off, uint32_t n_docs,
                          ygm_result *out);

/* Doc-normalized snapshot: Y.encodeStateAsUpdate(Y.applyUpdate(new Y.Doc(), update)) per document
 * -- the bytes extension-database stores (packages/extension-database/src/Database.ts:55-60,
 * Y.encodeStateAsUpdate of the live document): YATA-integrated, deleted content garbage-collected,
 * adjacent structs merged (yjs Y@20500-32900 readUpdate / cleanupTransactions, Y@23300
 * encodeStateAsUpdate).  One update per document (e.g. the output of ygm_merge_v1).  An update whose
 * document keeps pending structs / a pending delete set (lost or out-of-order updates) gives yjs's bytes
 * too: mergeUpdates([state, pendingDs, pending structs]) (Y@23300), run by the merge kernels.  Sub-documents
 * (ContentDoc) are integrated like any one-clock content.  Documents outside the envelope (repeated client
 * blocks, overlapping structs) carry YGM_EUNSUPPORTED. */
int ygm_snapshot_v1(ygm_ctx *ctx, const uint8_t *arena, const uint64_t *doc_off, uint32_t n_docs, ygm_result *out);
/* Read-only SyncStep2: Y.snapshotContainsUpdate(Y.snapshot(doc), update) per document
 * (packages/server/src/MessageReceiver.ts:156-179; yjs 13.6 snapshotContainsUpdate).  states: each
 * document's state (any update: its Y.snapshot view -- the store's integrated part, without pending structs or
 * a pending delete set -- is taken by the snapshot kernels first; a ygm_snapshot_v1 output is its own view);
 * updates: the received update per document.  Document d's output is one byte, 1 = contained (the
 * server acks with SyncStatus true), 0 = new content (SyncStatus false). */
int ygm_contains_v1(ygm_ctx *ctx, const uint8_t *states, const uint64_t *state_off, const uint8_t *updates,
                    const uint64_t *update_off, uint32_t n_docs, ygm_result *out);
/* SyncStep2 payload of a stored document: Y.encodeStateAsUpdate(doc, sv) for doc = Y.applyUpdate(new Y.Doc(), state)
 * -- what the reference sends in reply to a SyncStep1 (packages/server/src/MessageReceiver.ts:137-138) for a
 * document loaded from stored bytes (extension-database Database.ts:44-50).  Computed as the doc-normalized
 * snapshot of `state` (ygm_snapshot_v1) followed by diffUpdate(snapshot, sv) in which every struct keeps its
 * parentSub bit (Item.write of an integrated item, yjs Y@80416).  states / state_off as ygm_snapshot_v1;
 * sv_arena / sv_off one encoded state vector per document.  A state that leaves pending structs / a pending delete
 * set is answered as yjs does: mergeUpdates([writeStateAsUpdate(doc, sv), pendingDs, diffUpdate(pending structs,
 * sv)]) (Y@23300; the pending structs diffed without the kept bit).  A document outside the snapshot envelope
 * carries YGM_EUNSUPPORTED (the caller names it and keeps its yjs path). */
int ygm_sync_step2_v1(ygm_ctx *ctx, const uint8_t *states, const uint64_t *state_off, const uint8_t *sv_arena,
                      const uint64_t *sv_off, uint32_t n_docs, ygm_result *out);

/* ---- update format V2 ------------------------------------
 * The same operations over yjs's column-encoded update format V2 (UpdateEncoderV2 / UpdateDecoderV2,
 * yjs Y@15400-18900; lib0 RLE column coders), used by yjs providers other than Hocuspocus's V1 path:
 *   ygm_merge_v2            <- Y.mergeUpdatesV2(updates)                 (yjs Y@39011, V2 coders)
 *   ygm_diff_v2             <- Y.diffUpdateV2(update, stateVector)       (yjs Y@40711)
 *   ygm_sv_from_update_v2   <- Y.encodeStateVectorFromUpdateV2(update)   (yjs Y@37728; V1 state vector out)
 *   ygm_convert_v1_to_v2    <- Y.convertUpdateFormatV1ToV2(update)       (yjs 13.6)
 *   ygm_convert_v2_to_v1    <- Y.convertUpdateFormatV2ToV1(update)       (yjs 13.6)
 * Arguments as the V1 forms.  The conversions take updates in the lazy writer's normal form (what every
 * yjs encoder writes) and refuse others with YGM_ENONCANON, as they refuse V2 -> V1 of embed / format values
 * holding non-integer numbers (their JSON.stringify decimal is not reproduced).  mergeUpdatesV2 of one
 * update returns it as it is, as yjs does. */
int ygm_merge_v2(ygm_ctx *ctx, const uint8_t *arena, const uint64_t *upd_off, const uint32_t *upd_doc,
                 uint32_t n_upd, uint32_t n_docs, ygm_result *out);
int ygm_diff_v2(ygm_ctx *ctx, const uint8_t *arena, const uint64_t *doc_off, const uint8_t *sv_arena,
                const uint64_t *sv_off, uint32_t n_docs, ygm_result *out);
int ygm_sv_from_update_v2(ygm_ctx *ctx, const uint8_t *arena, const uint64_t *doc_off, uint32_t n_docs,
                          ygm_result *out);
int ygm_convert_v1_to_v2(ygm_ctx *ctx, const uint8_t *arena, const uint64_t *doc_off, uint32_t n_docs, ygm_result *out);
int ygm_convert_v2_to_v1(ygm_ctx *ctx, const uint8_t *arena, const uint64_t *doc_off, uint32_t n_docs, ygm_result *out);

/* ---- device-resident API (inputs already in HBM; used by bench.py) --------
 * All pointers are device pointers.  doc_upd: n_docs+1 update-index offsets
 * (document d owns updates doc_upd[d] .. doc_upd[d+1]); upd_off must be
 * non-decreasing.  Results stay on the device: the data/off/len/status
 * pointers of the result point into context-owned device memory.  Outputs
 * are NOT packed: document d's bytes are data[off[d] .. off[d]+len[d]) inside
 * its own slot (2*in_off + 64*d, capacity 2*|in| + 64) or, for documents the
 * lean kernels defer, in a region after the slots (merge: overflow cursor;
 * SV / diff: packed by the exact per-document kernel); data_bytes is the used
 * extent of `data`, payload_bytes the sum of len[].  `stream` is a
 * hipStream_t (NULL = the context's stream); the call returns after one
 * read of the launch counters.
 * Tail padding: the kernels read inputs in aligned 16-byte pieces and 64-byte chunks, so at least
 * 64 readable bytes must follow d_arena + arena_bytes and the end of d_sv_arena (zeroed or not: they
 * are never taken as input).  The host API pads its own staging copies. */
typedef struct {
  uint8_t *data;
  uint64_t *off;
  uint64_t *len;
  int32_t *status;
  uint64_t data_bytes;
  uint64_t payload_bytes;
} ygm_device_result;

int ygm_merge_v1_device(ygm_ctx *ctx, const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_upd_off,
                        const uint32_t *d_doc_upd, uint32_t n_upd, uint32_t n_docs, void *stream,
                        ygm_device_result *out);
/* Asynchronous form of ygm_merge_v1_device for GPU-resident pipelines: enqueues
 * the counter reset and the lean kernel on `stream` and returns without waiting.
 * Documents the lean kernel finishes are complete when the stream reaches this
 * point; every other document (deferred to the wave / workgroup / sequential
 * tiers) is completed by ygm_merge_v1_device_finish, which waits for the stream,
 * runs the tiers the device counters ask for, checks the fault flag and fills
 * out->data_bytes / payload_bytes.  A context holds one batch: the next enqueue
 * on it reuses the result buffers.
 * (Replaces no single reference interface: the batched form of Y.mergeUpdates,
 * yjs Y@37704, for GPU-resident pipelines.) */
int ygm_merge_v1_device_async(ygm_ctx *ctx, const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_upd_off,
                              const uint32_t *d_doc_upd, uint32_t n_upd, uint32_t n_docs, void *stream);
int ygm_merge_v1_device_finish(ygm_ctx *ctx, ygm_device_result *out);
/* Compact input form of ygm_merge_v1_device(_async): the documents' updates are contiguous in the arena, so
 * d_doc_off[d] (u64, n_docs + 1 entries) is the byte offset of document d's first update, d_doc_off[n_docs] the
 * end of the last, and d_upd_len[i] (u16, n_upd entries) the byte length of update i (every update < 64 KiB; a
 * batch with a larger one takes the u64 form).  2 bytes per update instead of 8 -- for a log of one-character
 * inserts the table is a third of the input bytes -- and no u64 table at all unless a document leaves the lean
 * kernel (the context then builds its entries on the device).  Lengths that do not add up to the document's bytes
 * give that document YGM_EMALFORMED (yjs reading past an update's end throws).  Results, finish and reuse as ygm_merge_v1_device(_async).
 * (Replaces no single reference interface: the batched form of Y.mergeUpdates, yjs Y@37704.) */
int ygm_merge_v1_device_lens(ygm_ctx *ctx, const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_doc_off,
                             const uint16_t *d_upd_len, const uint32_t *d_doc_upd, uint32_t n_upd, uint32_t n_docs, void *stream,
                             ygm_device_result *out);
int ygm_merge_v1_device_lens_async(ygm_ctx *ctx, const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_doc_off,
                                   const uint16_t *d_upd_len, const uint32_t *d_doc_upd, uint32_t n_upd, uint32_t n_docs,
                                   void *stream);
int ygm_diff_v1_device(ygm_ctx *ctx, const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_doc_off,
                       const uint8_t *d_sv_arena, const uint64_t *d_sv_off, uint32_t n_docs, void *stream,
                       ygm_device_result *out);
int ygm_sv_from_update_v1_device(ygm_ctx *ctx, const uint8_t *d_arena, uint64_t arena_bytes,
                                 const uint64_t *d_doc_off, uint32_t n_docs, void *stream,
                                 ygm_device_result *out);

int ygm_snapshot_v1_device(ygm_ctx *ctx, const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_doc_off,
                           uint32_t n_docs, void *stream, ygm_device_result *out);

int ygm_contains_v1_device(ygm_ctx *ctx, const uint8_t *d_states, const uint64_t *d_state_off, const uint8_t *d_updates,
                           const uint64_t *d_update_off, uint32_t n_docs, void *stream, ygm_device_result *out);
int ygm_sync_step2_v1_device(ygm_ctx *ctx, const uint8_t *d_states, uint64_t states_bytes, const uint64_t *d_state_off,
                             const uint8_t *d_sv_arena, const uint64_t *d_sv_off, uint32_t n_docs, void *stream,
                             ygm_device_result *out);

/* update V2, device-resident (outputs packed in document order: off[d] increasing) */
int ygm_merge_v2_device(ygm_ctx *ctx, const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_upd_off,
                        const uint32_t *d_doc_upd, uint32_t n_upd, uint32_t n_docs, void *stream, ygm_device_result *out);
int ygm_diff_v2_device(ygm_ctx *ctx, const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_doc_off,
                       const uint8_t *d_sv_arena, const uint64_t *d_sv_off, uint32_t n_docs, void *stream,
                       ygm_device_result *out);
int ygm_sv_from_update_v2_device(ygm_ctx *ctx, const uint8_t *d_arena, uint64_t arena_bytes,
                                 const uint64_t *d_doc_off, uint32_t n_docs, void *stream, ygm_device_result *out);
int ygm_convert_v1_to_v2_device(ygm_ctx *ctx, const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_doc_off,
                                uint32_t n_docs, void *stream, ygm_device_result *out);
int ygm_convert_v2_to_v1_device(ygm_ctx *ctx, const uint8_t *d_arena, uint64_t arena_bytes, const uint64_t *d_doc_off,
                                uint32_t n_docs, void *stream, ygm_device_result *out);

int ygm_stats(ygm_ctx *ctx, ygm_stats_t *out);
const char *ygm_strerror(int code);
const char *ygm_version(void);

#ifdef __cplusplus
}
#endif
#endif /* YGM_H */
