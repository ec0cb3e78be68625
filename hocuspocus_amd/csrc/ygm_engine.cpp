// ygm_engine.cpp -- host runtime behind include/ygm.h.
//
// One context per GPU: a HIP stream, grow-only device workspaces, host result
// buffers and HIP-event timers.  A batch call = H2D of the packed inputs, one
// fast-path launch (look-back placed, packed output), an 8-byte-class meta
// read, the sequential kernel only when some document needed it, D2H.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "../../include/ygm.h"

extern "C" {
size_t ygm_k_meta_bytes();
int ygm_k_meta_layout(size_t* sz, size_t* off_big_started, size_t* off_big_scur, size_t* off_payload_sh);
size_t ygm_k_seq_reader_bytes();
size_t ygm_k_drec_bytes();
int ygm_k_launch_doc(int mode, const uint8_t* arena, const uint64_t* doc_off, const uint8_t* sv_arena, const uint64_t* sv_off,
                     const uint32_t* docs, uint64_t out_base, uint32_t n_docs, uint32_t flags, uint8_t* out, uint64_t* out_off,
                     uint64_t* out_len, int32_t* status, unsigned long long* lb, void* meta, uint64_t out_cap, hipStream_t s);
size_t ygm_k_sv_table_bytes(uint32_t n_docs);
int ygm_k_launch_snap_plan(const uint8_t* arena, const uint64_t* doc_off, uint32_t n_docs, uint32_t flags, void* cnt, uint64_t* ws_off,
                           uint64_t* bs, const uint8_t* claim, hipStream_t s);
int ygm_k_launch_snap_text(const uint8_t* arena, const uint64_t* doc_off, uint32_t n_docs, uint32_t flags, uint8_t* out, uint64_t* out_off,
                           uint64_t* out_len, int32_t* status, uint8_t* claim, unsigned long long* pay, int again, uint64_t slot_total, hipStream_t s);
int ygm_k_launch_cont_plan(const uint8_t* st_arena, const uint64_t* st_off, uint32_t n_docs, uint32_t flags, uint64_t* ws_off, uint64_t* bs,
                           hipStream_t s);
int ygm_k_launch_cont(const uint8_t* st_arena, const uint64_t* st_off, const uint8_t* up_arena, const uint64_t* up_off, uint32_t n_docs,
                      uint32_t flags, const uint64_t* ws_off, uint8_t* ws, uint8_t* out, uint64_t* out_off, uint64_t* out_len,
                      int32_t* status, hipStream_t s);
int ygm_k_launch_snap(const uint8_t* arena, const uint64_t* doc_off, uint32_t n_docs, uint32_t flags, const void* cnt, const uint64_t* ws_off,
                      uint8_t* ws, uint64_t* out_off, uint64_t* out_len, int32_t* status, unsigned long long* payload, const uint8_t* claim,
                      uint64_t base, uint32_t* pend_list, unsigned int* pend_n, hipStream_t s);
int ygm_k_launch_pend_plan(const uint32_t* list, uint32_t P, const uint8_t* ws, const uint64_t* out_off, uint64_t* upd_off, uint32_t* doc_upd,
                           hipStream_t s);
int ygm_k_launch_pend_copy(const uint32_t* list, uint32_t P, const uint8_t* ws, const uint64_t* out_off, const uint64_t* upd_off, uint8_t* dst,
                           hipStream_t s);
int ygm_k_launch_pend_fix(const uint32_t* list, uint32_t P, const uint64_t* m_off, const uint64_t* m_len, const int32_t* m_st,
                          const int32_t* pst, uint64_t tail, uint64_t* out_off, uint64_t* out_len, int32_t* status, hipStream_t s);
int ygm_k_launch_pend_split(const uint32_t* list, uint32_t P, const uint8_t* ws, const uint64_t* out_off, const uint8_t* sv,
                            const uint64_t* sv_off, uint64_t* offs, uint8_t* da, uint8_t* db, uint8_t* dc, uint8_t* dsv, int pass,
                            hipStream_t s);
int ygm_k_launch_pend_join(uint32_t P, const uint8_t* ad, const uint64_t* a_off, const uint64_t* a_len, const int32_t* a_st, const uint8_t* bd,
                           const uint64_t* offs, const uint8_t* cd, const uint64_t* c_off, const uint64_t* c_len, const int32_t* c_st,
                           uint64_t* upd_off, uint32_t* doc_upd, int32_t* pst, uint8_t* dst, int pass, hipStream_t s);
int ygm_k_launch_pack(const uint8_t* src, const uint64_t* off, const uint64_t* len, const int32_t* status, uint32_t n, uint64_t* bsum,
                      uint8_t* dst, uint64_t* poff, hipStream_t s);
int ygm_k_launch_doc_lean(int mode, const uint8_t* arena, uint64_t arena_bytes, const uint64_t* doc_off, const uint8_t* sv_arena,
                          uint64_t sv_bytes, const uint64_t* sv_off, uint32_t n_docs, uint32_t flags, uint8_t* out, uint64_t* out_off,
                          uint64_t* out_len, int32_t* status, void* meta, uint32_t* defer_list, uint64_t out_cap, uint8_t* tbl,
                          uint32_t* tbl_n, hipStream_t s);
uint32_t ygm_k_lean_stage_bytes();
int ygm_k_launch_merge_lean(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, uint32_t n_docs, uint32_t flags,
                            uint8_t* out, uint64_t* out_off, uint64_t* out_len, int32_t* status, void* meta, void* meta_next,
                            uint32_t* defer_list, uint64_t out_cap, hipStream_t s, const uint64_t* doc_off, const uint16_t* upd_len);
int ygm_k_launch_big_wait(void* meta, uint32_t n_large, hipStream_t s);
int ygm_k_launch_build_off(const uint64_t* doc_off, const uint16_t* upd_len, const uint32_t* doc_upd, const uint32_t* list, uint32_t n,
                           uint64_t* upd_off, hipStream_t s);
int ygm_k_launch_merge_lean_wide(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, uint32_t n_docs, const uint32_t* list,
                                 uint32_t n_list, uint32_t flags, uint8_t* out, uint64_t* out_off, uint64_t* out_len, int32_t* status,
                                 void* meta, void* meta_next, uint32_t* defer_list, uint64_t out_cap, const uint16_t* upd_len,
                                 hipStream_t s);
int ygm_k_launch_merge_wave(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, const uint32_t* docs,
                            const unsigned int* n_dev, uint32_t n_docs, uint32_t flags, uint8_t* out, uint64_t* out_off, uint64_t* out_len,
                            int32_t* status, void* meta, uint32_t* defer_list, uint32_t* fb_list, uint64_t out_cap, hipStream_t s);
int ygm_k_launch_route_big(const uint64_t* upd_off, const uint32_t* doc_upd, const uint32_t* docs, const unsigned int* n_dev, uint32_t n_docs,
                           uint32_t flags, uint64_t* out_off, uint64_t* out_len, int32_t* status, void* meta, uint32_t* fb_list, uint32_t* rest,
                           hipStream_t s);
int ygm_k_launch_merge_fast(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, const uint32_t* docs,
                            const unsigned int* n_dev, uint32_t n_docs, uint32_t flags, uint8_t* out, uint64_t* out_off, uint64_t* out_len,
                            int32_t* status, uint64_t slot_total, void* meta, uint32_t* fb_list, uint64_t out_cap, hipStream_t s);
int ygm_k_launch_merge_seq(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, const uint32_t* fb_list, uint32_t n_fb,
                           uint32_t flags, uint8_t* out, uint64_t* out_off, uint64_t* out_len, int32_t* status, void* meta,
                           void* readers, int* order, int* tmp, const uint8_t** ubase, uint32_t* ulen, uint64_t upd_cap,
                           uint32_t* cnt, void* drec, uint64_t byte_cap, uint64_t slot_total, uint64_t out_cap, hipStream_t s);
int ygm_k_launch_scan(uint64_t* v, uint32_t n, uint64_t* bs, hipStream_t s);
size_t ygm_k_v2_cols();
int ygm_k_launch_v21(int pass, const uint8_t* arena, const uint64_t* upd_off, uint32_t n_upd, const uint32_t* doc_upd, uint32_t n_docs,
                     uint32_t mode, uint32_t flags, uint64_t* len_or_off, int32_t* st, uint8_t* out, uint8_t* cl, hipStream_t s);
int ygm_k_launch_v12_count(const uint8_t* v1, const uint64_t* v1_off, const uint64_t* v1_len, const int32_t* v1_st, const uint8_t* v2a,
                           uint64_t v2n, const uint64_t* upd_off, const uint32_t* doc_upd, const int32_t* ust, uint32_t n_docs, uint32_t mode,
                           uint32_t flags, uint32_t* L, uint64_t* tot, int32_t* st, const uint8_t* claim, hipStream_t s);
int ygm_k_launch_v12_write(const uint8_t* v1, const uint64_t* v1_off, const uint64_t* v1_len, const uint8_t* v2a, uint64_t v2n,
                           const uint64_t* upd_off, const uint32_t* doc_upd, uint32_t n_docs, uint32_t mode, uint32_t flags, const uint32_t* L,
                           const uint64_t* off, int32_t* st, uint8_t* out, uint64_t* out_len, const uint8_t* claim, uint64_t base, uint64_t* fo,
                           hipStream_t s);
int ygm_k_launch_v12_fast(const uint8_t* v1, const uint64_t* v1_off, const uint64_t* v1_len, const int32_t* v1_st, const uint64_t* slot_off,
                          const uint32_t* doc_upd, const int32_t* ust, uint32_t n_docs, uint8_t* out, uint64_t* fo, uint64_t* olen, int32_t* ost,
                          uint8_t* claim, unsigned long long* payload, uint8_t* scr, uint64_t slot_total, hipStream_t s);
size_t ygm_k_v12_fast_scratch();
int ygm_k_launch_v2_status(const int32_t* ust, uint32_t n, int32_t* status, uint64_t* len, hipStream_t s);
int ygm_k_launch_v2_lens(const uint64_t* off, const int32_t* st, uint32_t n, uint64_t* len, hipStream_t s);
size_t ygm_k_big_blk_bytes();
size_t ygm_k_big_rec_bytes();
int ygm_k_launch_big_scan(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, const uint32_t* fb_list,
                          uint32_t n_fb, uint32_t flags, void* scan, uint64_t fb_bytes, hipStream_t s);
int ygm_k_launch_merge_big(int large, const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, const uint32_t* fb_list,
                           uint32_t n_fb, const uint32_t* fbx, uint32_t n, uint32_t* up_list, uint32_t flags, uint8_t* out,
                           uint64_t* out_off, uint64_t* out_len, int32_t* status, void* meta, uint32_t* fb2_list, void* blk,
                           uint64_t blk_cap, void* rec, uint64_t rec_cap, uint64_t slot_total, uint64_t out_cap, void* scan,
                           uint64_t fb_bytes, hipStream_t s);
size_t ygm_k_big_scan_bytes(uint32_t n_fb, uint64_t fb_bytes);
void ygm_k_big_lists(void* scan, uint32_t n_fb, uint64_t fb_bytes, unsigned long long** cnt, uint32_t** llist, uint32_t** mlist);
}

namespace {

// mirrors ygm::DocMeta (ygm_docmeta.hpp) field for field; sizeof is a multiple of 16.  ygm_open checks the layout
// against the kernels' own (ygm_k_meta_layout): read_meta and the counter memsets depend on it
struct Meta {
  unsigned int ticket, fault, fb_count, defer_count, lean_defer, big_defer, wide_defer, mid_defer, big_started, route_n;
  unsigned long long big_scur;
  unsigned long long fast_total, cursor, payload, fb_upds, fb_bytes, scr_upd_cursor, scr_byte_cursor, big_cursor;
  unsigned long long payload_sh[16 * 16];
  unsigned long long payload_total() const {
    unsigned long long t = payload;
    for (unsigned long long x : payload_sh) t += x;
    return t;
  }
};

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  // keep > 0: the first `keep` bytes survive a regrowth (copied on stream s, which is then synchronised)
  bool ensure(size_t n, size_t keep = 0, hipStream_t s = nullptr) {
    if (n <= cap && p) return true;
    if (p && keep) {
      void* q = nullptr;
      size_t c = n + n / 4;
      if (hipMalloc(&q, c) != hipSuccess) return false;
      if (hipMemcpyAsync(q, p, std::min(keep, cap), hipMemcpyDeviceToDevice, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {
        (void)hipFree(q); return false;
      }
      (void)hipFree(p); p = q; cap = c;
      return true;
    }
    if (p) { (void)hipFree(p); p = nullptr; cap = 0; }
    size_t c = std::max<size_t>(n, 256);
    c += c / 4;  // grow with headroom
    if (hipMalloc(&p, c) != hipSuccess) { p = nullptr; return false; }
    cap = c;
    return true;
  }
  void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
  template <class T> T* as() const { return (T*)p; }
};

// pinned (page-locked) host memory: DMA-able staging for the host API's copies
struct PinBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool ensure(size_t n, size_t keep = 0) {   // keep: leading bytes preserved across a regrowth
    if (n <= cap && p) return true;
    size_t c = std::max<size_t>(n, 4096);
    c += c / 4;
    void* q = nullptr;
    if (hipHostMalloc(&q, c, hipHostMallocDefault) != hipSuccess) return false;
    if (p) { if (keep) memcpy(q, p, std::min(keep, cap)); (void)hipHostFree(p); }
    p = q; cap = c;
    return true;
  }
  void release() { if (p) (void)hipHostFree(p); p = nullptr; cap = 0; }
  template <class T> T* as() const { return (T*)p; }
};

}  // namespace

struct ygm_ctx {
  int device = 0;
  uint32_t flags = 0;
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;   // the large-document tier's 16-wave launch, beside the mid size's on `stream`
  hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr, e3 = nullptr;
  // device inputs (host API staging)
  DevBuf arena, offs, docs, sv_arena, sv_offs;
  // device outputs + state
  DevBuf out, out_off, out_len, status, lb, meta, fb_list, defer_list, defer2_list, defer_w_list, route_list;
  Meta* h_meta = nullptr;  // pinned read-back of the per-launch counters
  int mslot = 0;           // counter slot of the next merge launch
  void* meta_slot(int i) const { return (uint8_t*)meta.p + (size_t)i * sizeof(Meta); }
  DevBuf s_readers, s_order, s_tmp, s_ubase, s_ulen, s_cnt, s_drec;
  DevBuf big_blk, big_rec, big_list, big_scan, big_up;   // large-document tier: block tables, struct records, documents sent on, scan
  DevBuf sv_tbl, sv_tn;                // diff: sorted state-vector tables (k_sv_table) and their entry counts
  DevBuf sn_cnt, sn_off, sn_bs, sn_ws, sn_claim, sn_pay;
  DevBuf sn_pend, pn_off, pn_du, pn_arena;   // snapshot: documents left pending, their three-update batch for the merge
  DevBuf pq_off, pq_a, pq_b, pq_c, pq_s, pq_st;   // step2 of pending documents: their parts and state vectors, statuses
  ygm_ctx* pend_ctx = nullptr;               // ... merged on this child context (its own buffers and counters)
  ygm_ctx* pend_dx[2] = {nullptr, nullptr};  // ... and the step2 diffs of their parts on these  // snapshot: per-document counts, workspace offsets, scan scratch,
  // [LDS-tier output slots | workspaces], LDS-tier claims, its payload / claimed counters
  // update V2: per-update V1 sizes -> offsets, transcoding statuses, scan scratch, the V1 arena, per-document column
  // lengths, the V2 outputs (packed), their offsets / lengths / statuses
  DevBuf v2_len, v2_st, v2_bs, v2_v1, v2_L, v2_out, v2_off, v2_olen, v2_ost, v2_fo, v2_claim, v2_pay, v2_scr, v21_cl;
  // host API: results in pinned memory (packed outputs, per-document offset / length / status), the
  // pinned input staging of this context when it serves as a pipeline stage, the packed device copy,
  // and the two stage contexts (own streams and buffers) that double-buffer a batch's chunks
  PinBuf h_data, h_off, h_len, h_status, h_in;
  DevBuf pk_data, pk_off, pk_bsum;
  DevBuf s2_data, s2_off, s2_bsum, s2_st;   // sync step2: packed snapshots, their offsets, scan scratch, snapshot statuses
  ygm_ctx* kid[2] = {nullptr, nullptr};
  std::vector<uint32_t> h_doc_upd;
  ygm_stats_t stats{};
  // the batch enqueued by ygm_merge_v1_device_async, completed by ygm_merge_v1_device_finish
  struct Pending {
    bool live = false;
    hipStream_t s = nullptr;
    const uint8_t* arena = nullptr; const uint64_t* upd_off = nullptr; const uint32_t* doc_upd = nullptr;
    uint64_t arena_bytes = 0, slot_total = 0, out_cap = 0;
    uint32_t n_upd = 0, n_docs = 0;
    void* meta = nullptr;   // counter slot of the launch
    bool wide_route = false;   // the launch was the wide lean kernel over the whole batch
    // the compact input form (ygm_merge_v1_device_lens): upd_off is the context's table, built for deferred documents
    const uint64_t* doc_off = nullptr; const uint16_t* upd_len = nullptr;
  } pend;
  DevBuf lens_off;   // update-offset table of a compact-form batch (entries of the documents the lean kernel defers)
  uint32_t lean_span_n = 0;   // lean launches enqueued since the last finish (timed as one span, e0 .. e1)
};

static int herr(hipError_t e) { return e == hipSuccess ? YGM_OK : YGM_EDEVICE; }
#define HIPCHK(x) do { hipError_t _e = (x); if (_e != hipSuccess) return YGM_EDEVICE; } while (0)

extern "C" {

const char* ygm_version(void) { return "ygm 0.1 (gfx950; yjs 13.6.26 update-v1 semantics)"; }

const char* ygm_strerror(int code) {
  switch (code) {
    case YGM_OK: return "ok";
    case YGM_EMALFORMED: return "Unexpected end of array / malformed update";
    case YGM_ERANGE: return "Integer out of Range";
    case YGM_ENONCANON: return "non-canonical content (yjs would re-encode it)";
    case YGM_ESURROGATE: return "lone surrogate in string slice (yjs 13.5 compat)";
    case YGM_EDEPTH: return "Any/JSON nesting too deep";
    case YGM_ENOMEM: return "out of device memory";
    case YGM_EDEVICE: return "HIP device error";
    case YGM_EINVAL: return "invalid argument";
    case YGM_EUNSUPPORTED: return "outside the snapshot kernel's envelope (pending structs / delete set, sub-documents, ...)";
  }
  return "unknown error";
}

int ygm_open(int device, uint32_t flags, ygm_ctx** out) {
  if (!out) return YGM_EINVAL;
  *out = nullptr;
  {   // the host mirror of the device counters must match the kernels' struct
    size_t sz = 0, o1 = 0, o2 = 0, o3 = 0;
    ygm_k_meta_layout(&sz, &o1, &o2, &o3);
    if (sz != sizeof(Meta) || o1 != offsetof(Meta, big_started) || o2 != offsetof(Meta, big_scur) || o3 != offsetof(Meta, payload_sh)) {
      fprintf(stderr, "ygm: host / device counter layouts differ (%zu vs %zu bytes)\n", sz, sizeof(Meta));
      return YGM_EINVAL;
    }
  }
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return YGM_EDEVICE;
  ygm_ctx* c = new ygm_ctx();
  c->device = device; c->flags = flags;
  // stream2 (the large-document tier's 16-wave size) is created at the high priority on first use: a queue of its own
  // (a process with more streams than hardware queues shares them, and two streams on one queue run their kernels
  // one after the other); contexts that never run that size (the host API's stage contexts, most pool members) do
  // not hold one
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->e0) != hipSuccess || hipEventCreate(&c->e1) != hipSuccess || hipEventCreate(&c->e2) != hipSuccess ||
      hipEventCreate(&c->e3) != hipSuccess) {
    delete c;
    return YGM_EDEVICE;
  }
  // counter slots: 0 / 1 alternate between merge launches (each lean launch zeroes the other
  // slot for the next one: no reset kernel per batch), 2 = SV / diff (reset per call)
  if (!c->meta.ensure(3 * sizeof(Meta)) || hipMemset(c->meta.p, 0, 3 * sizeof(Meta)) != hipSuccess) { ygm_close(c); return YGM_ENOMEM; }
  if (hipHostMalloc((void**)&c->h_meta, sizeof(Meta), hipHostMallocDefault) != hipSuccess) { c->h_meta = nullptr; ygm_close(c); return YGM_ENOMEM; }
  *out = c;
  return YGM_OK;
}

void ygm_close(ygm_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->stream2) (void)hipStreamSynchronize(c->stream2);
  for (DevBuf* b : {&c->arena, &c->offs, &c->docs, &c->sv_arena, &c->sv_offs, &c->out, &c->out_off, &c->out_len, &c->status,
                    &c->lb, &c->meta, &c->fb_list, &c->defer_list, &c->defer2_list, &c->defer_w_list, &c->route_list, &c->s_readers, &c->s_order, &c->s_tmp, &c->s_ubase, &c->s_ulen, &c->s_cnt,
                    &c->s_drec, &c->big_blk, &c->big_rec, &c->big_list, &c->big_scan, &c->big_up, &c->lens_off, &c->sv_tbl, &c->sv_tn, &c->sn_cnt, &c->sn_off, &c->sn_bs, &c->sn_ws, &c->sn_claim, &c->sn_pay,
                    &c->sn_pend, &c->pn_off, &c->pn_du, &c->pn_arena,
                    &c->pq_off, &c->pq_a, &c->pq_b, &c->pq_c, &c->pq_s, &c->pq_st, &c->v2_len, &c->v2_st, &c->v2_bs, &c->v2_v1, &c->v2_L, &c->v2_out, &c->v2_off, &c->v2_olen, &c->v2_ost, &c->v2_fo, &c->v2_claim, &c->v2_pay, &c->v2_scr, &c->v21_cl})
    b->release();
  for (ygm_ctx* k : c->kid) if (k) ygm_close(k);
  if (c->pend_ctx) ygm_close(c->pend_ctx);
  for (ygm_ctx* k : c->pend_dx) if (k) ygm_close(k);
  for (DevBuf* b : {&c->pk_data, &c->pk_off, &c->pk_bsum}) b->release();
  for (PinBuf* b : {&c->h_data, &c->h_off, &c->h_len, &c->h_status, &c->h_in}) b->release();
  for (hipEvent_t e : {c->e0, c->e1, c->e2, c->e3}) if (e) (void)hipEventDestroy(e);
  if (c->h_meta) (void)hipHostFree(c->h_meta);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->stream2) (void)hipStreamDestroy(c->stream2);
  delete c;
}

int ygm_stats(ygm_ctx* c, ygm_stats_t* out) {
  if (!c || !out) return YGM_EINVAL;
  *out = c->stats;
  return YGM_OK;
}

// ------------------------------------------------------------------ device API
static int prep_outputs(ygm_ctx* c, uint32_t n_docs, uint64_t out_cap, hipStream_t s, bool lookback) {
  const size_t tiles = (size_t)n_docs / 256 + 2;  // look-back tiles of the SV/diff kernels (256 documents each)
  if (!c->out.ensure(out_cap + 64) || !c->out_off.ensure((size_t)n_docs * 8 + 8) || !c->out_len.ensure((size_t)n_docs * 8 + 8) ||
      !c->status.ensure((size_t)n_docs * 4 + 4) || !c->lb.ensure(tiles * 8) || !c->fb_list.ensure((size_t)n_docs * 4 + 4) ||
      !c->defer_list.ensure((size_t)n_docs * 4 + 4) || !c->defer2_list.ensure((size_t)n_docs * 4 + 4) ||
      !c->defer_w_list.ensure((size_t)n_docs * 4 + 4) || !c->route_list.ensure((size_t)n_docs * 4 + 4))
    return YGM_ENOMEM;
  if (lookback) {   // SV / diff: look-back tiles and counter slot 2 reset per call
    HIPCHK(hipMemsetAsync(c->lb.p, 0, tiles * 8, s));
    HIPCHK(hipMemsetAsync(c->meta_slot(2), 0, sizeof(Meta), s));
  }
  return YGM_OK;
}

static int read_meta(ygm_ctx* c, hipStream_t s, Meta& m, const void* slot) {
  c->stats.host_syncs++;
  HIPCHK(hipMemcpyAsync(c->h_meta, slot, sizeof(Meta), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  m = *c->h_meta;
  return YGM_OK;
}

static void fill_dev_result(ygm_ctx* c, uint64_t data_bytes, ygm_device_result* out) {
  out->data = c->out.as<uint8_t>();
  out->off = c->out_off.as<uint64_t>();
  out->len = c->out_len.as<uint64_t>();
  out->status = c->status.as<int32_t>();
  out->data_bytes = data_bytes;
  out->payload_bytes = data_bytes;
}

// offsets of the DocMeta counters the tier kernels read as device-side counts
static int merge_async(ygm_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes, const uint64_t* d_upd_off, const uint32_t* d_doc_upd,
                       uint32_t n_upd, uint32_t n_docs, void* stream, const uint64_t* d_doc_off, const uint16_t* d_upd_len) {
  if (!c) return YGM_EINVAL;
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  (void)hipSetDevice(c->device);
  // output arena: one slot per document (2|in| + 64 B, no cross-document dependency),
  // then the overflow region for outputs that outgrow their slot (<= 3|in| + 16/doc)
  const uint64_t slot_total = 2 * arena_bytes + 64ull * n_docs;
  const uint64_t out_cap = slot_total + 3 * arena_bytes + 16ull * n_docs + 64;
  int e = prep_outputs(c, n_docs, out_cap, s, false);
  if (e) return e;
  // the wide route: a batch whose average document outgrows the narrow kernel's staging (multi-character inserts,
  // many clients: the realistic logs of c2_mixed) would be deferred by it almost whole -- a pass that only reads
  // headers yet costs as much as merging a C2 batch (latency-bound) -- so the wide kernel takes every document
  const bool wide_route = n_docs && arena_bytes / n_docs > (uint64_t)ygm_k_lean_stage_bytes() && getenv("YGM_NO_WIDE_ROUTE") == nullptr;
  if (d_doc_off) {   // compact form: the table every tier after the narrow kernel reads (only deferred documents' entries)
    if (!c->lens_off.ensure(8ull * n_upd + 16)) return YGM_ENOMEM;
    d_upd_off = c->lens_off.as<uint64_t>();
    if (wide_route && ygm_k_launch_build_off(d_doc_off, d_upd_len, d_doc_upd, nullptr, n_docs, c->lens_off.as<uint64_t>(), s))
      return YGM_EDEVICE;
  }
  // tier 1: lean wave-per-document kernel (debounce-log shape); everything else is deferred.
  // Timing: one event before the first launch since the last finish, one in finish after the
  // last -- per-launch event pairs between back-to-back launches cost ~8 us of stream time each.
  if (c->lean_span_n == 0) HIPCHK(hipEventRecord(c->e0, s));
  c->lean_span_n++;
  void* meta = c->meta_slot(c->mslot);
  void* meta_next = c->meta_slot(1 - c->mslot);   // zeroed by this launch for the next one
  if (wide_route) {
    if (ygm_k_launch_merge_lean_wide(d_arena, d_upd_off, d_doc_upd, n_docs, nullptr, n_docs, c->flags, c->out.as<uint8_t>(),
                                     c->out_off.as<uint64_t>(), c->out_len.as<uint64_t>(), c->status.as<int32_t>(), meta, meta_next,
                                     c->defer_w_list.as<uint32_t>(), out_cap, d_upd_len, s))
      return YGM_EDEVICE;
  } else if (ygm_k_launch_merge_lean(d_arena, d_upd_off, d_doc_upd, n_docs, c->flags, c->out.as<uint8_t>(), c->out_off.as<uint64_t>(),
                                     c->out_len.as<uint64_t>(), c->status.as<int32_t>(), meta, meta_next, c->defer_list.as<uint32_t>(), out_cap, s,
                                     d_doc_off, d_upd_len))
    return YGM_EDEVICE;
  c->pend.wide_route = wide_route;
  if (n_docs) c->mslot = 1 - c->mslot;   // (an empty batch launches nothing: the slot stays current)
  c->pend.live = true; c->pend.s = s;
  c->pend.arena = d_arena; c->pend.upd_off = d_upd_off; c->pend.doc_upd = d_doc_upd;
  c->pend.arena_bytes = arena_bytes; c->pend.slot_total = slot_total; c->pend.out_cap = out_cap;
  c->pend.n_upd = n_upd; c->pend.n_docs = n_docs; c->pend.meta = meta;
  c->pend.doc_off = wide_route ? nullptr : d_doc_off; c->pend.upd_len = d_upd_len;   // (wide route: the table is whole)
  return YGM_OK;
}
int ygm_merge_v1_device_async(ygm_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes, const uint64_t* d_upd_off,
                              const uint32_t* d_doc_upd, uint32_t n_upd, uint32_t n_docs, void* stream) {
  return merge_async(c, d_arena, arena_bytes, d_upd_off, d_doc_upd, n_upd, n_docs, stream, nullptr, nullptr);
}
int ygm_merge_v1_device_lens_async(ygm_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes, const uint64_t* d_doc_off,
                                   const uint16_t* d_upd_len, const uint32_t* d_doc_upd, uint32_t n_upd, uint32_t n_docs, void* stream) {
  if (!d_doc_off || !d_upd_len) return YGM_EINVAL;
  return merge_async(c, d_arena, arena_bytes, nullptr, d_doc_upd, n_upd, n_docs, stream, d_doc_off, d_upd_len);
}

int ygm_merge_v1_device_finish(ygm_ctx* c, ygm_device_result* out) {
  if (!c || !out || !c->pend.live) return YGM_EINVAL;
  ygm_ctx::Pending& P = c->pend;
  P.live = false;
  hipStream_t s = P.s;
  (void)hipSetDevice(c->device);
  HIPCHK(hipEventRecord(c->e1, s));
  Meta m;
  int e = read_meta(c, s, m, P.meta);
  if (e) return e;
  if (m.fault) return YGM_EDEVICE;
  float ms0 = 0;
  if (c->lean_span_n && hipEventElapsedTime(&ms0, c->e0, c->e1) == hipSuccess) { c->stats.kernel_ms += ms0; c->stats.lean_ms += ms0; }
  c->stats.lean_launches += c->lean_span_n;
  c->lean_span_n = 0;
  uint32_t n_gen = 0;   // documents for the general tiers
  // The general tiers are chained on the device: the wide lean kernel (host count: the narrow kernel's deferrals),
  // then the wave and workgroup kernels, each reading its count from the counter the kernel before it wrote (stream
  // order; the host count is only the bound that sizes the persistent grid) -- one host wait for all three.
  const unsigned int* d_wide_defer = (const unsigned int*)((const char*)P.meta + offsetof(Meta, wide_defer));
  const unsigned int* d_defer_count = (const unsigned int*)((const char*)P.meta + offsetof(Meta, defer_count));
  const unsigned int* d_route_n = (const unsigned int*)((const char*)P.meta + offsetof(Meta, route_n));
  // the large-document tier's documents leave the chain before the wave kernel (k_route_big): the rest go on to it
  auto route = [&](const uint32_t* list, const unsigned int* n_dev, uint32_t n) {
    return ygm_k_launch_route_big(P.upd_off, P.doc_upd, list, n_dev, n, c->flags, c->out_off.as<uint64_t>(), c->out_len.as<uint64_t>(),
                                  c->status.as<int32_t>(), P.meta, c->fb_list.as<uint32_t>(), c->route_list.as<uint32_t>(), s);
  };
  uint32_t bound = 0;   // documents the chain may see (0: no chain)
  HIPCHK(hipEventRecord(c->e0, s));
  if (P.wide_route) {  // the wide kernel took the whole batch (async): its deferrals go on
    n_gen = bound = m.wide_defer;
    c->stats.docs_lean_wide += P.n_docs - m.wide_defer;
    if (n_gen && route(c->defer_w_list.as<uint32_t>(), nullptr, n_gen)) return YGM_EDEVICE;
    if (n_gen && ygm_k_launch_merge_wave(P.arena, P.upd_off, P.doc_upd, c->route_list.as<uint32_t>(), d_route_n, n_gen, c->flags,
                                         c->out.as<uint8_t>(), c->out_off.as<uint64_t>(), c->out_len.as<uint64_t>(), c->status.as<int32_t>(),
                                         P.meta, c->defer2_list.as<uint32_t>(), c->fb_list.as<uint32_t>(), P.out_cap, s))
      return YGM_EDEVICE;
  } else if (m.lean_defer) {  // tier 1b: the wide lean kernel (updates <= 64 bytes, documents <= 7 KB) over tier 1's deferred list
    bound = m.lean_defer;
    if (P.doc_off && ygm_k_launch_build_off(P.doc_off, P.upd_len, P.doc_upd, c->defer_list.as<uint32_t>(), m.lean_defer,
                                            const_cast<uint64_t*>(P.upd_off), s))   // (compact form: the deferred documents' offsets)
      return YGM_EDEVICE;
    if (ygm_k_launch_merge_lean_wide(P.arena, P.upd_off, P.doc_upd, P.n_docs, c->defer_list.as<uint32_t>(), m.lean_defer, c->flags,
                                     c->out.as<uint8_t>(), c->out_off.as<uint64_t>(), c->out_len.as<uint64_t>(), c->status.as<int32_t>(),
                                     P.meta, nullptr, c->defer_w_list.as<uint32_t>(), P.out_cap, P.upd_len, s))
      return YGM_EDEVICE;
    // tier 2: the general wave-per-document kernel over the lean kernels' deferred list, after the routing pass
    if (route(c->defer_w_list.as<uint32_t>(), d_wide_defer, bound)) return YGM_EDEVICE;
    if (ygm_k_launch_merge_wave(P.arena, P.upd_off, P.doc_upd, c->route_list.as<uint32_t>(), d_route_n, bound, c->flags,
                                c->out.as<uint8_t>(), c->out_off.as<uint64_t>(), c->out_len.as<uint64_t>(), c->status.as<int32_t>(),
                                P.meta, c->defer2_list.as<uint32_t>(), c->fb_list.as<uint32_t>(), P.out_cap, s))
      return YGM_EDEVICE;
  }
  if (bound) {  // tier 3: documents over the wave class, one workgroup per document
    if (ygm_k_launch_merge_fast(P.arena, P.upd_off, P.doc_upd, c->defer2_list.as<uint32_t>(), d_defer_count, bound, c->flags,
                                c->out.as<uint8_t>(), c->out_off.as<uint64_t>(), c->out_len.as<uint64_t>(), c->status.as<int32_t>(),
                                P.slot_total, P.meta, c->fb_list.as<uint32_t>(), P.out_cap, s))
      return YGM_EDEVICE;
    HIPCHK(hipEventRecord(c->e1, s));
    const uint32_t lean_defer = m.lean_defer;
    if ((e = read_meta(c, s, m, P.meta))) return e;
    if (m.fault) return YGM_EDEVICE;
    if (hipEventElapsedTime(&ms0, c->e0, c->e1) == hipSuccess) c->stats.kernel_ms += ms0;
    if (!P.wide_route) { n_gen = m.wide_defer; c->stats.docs_lean_wide += lean_defer - m.wide_defer; }
  }
  uint32_t n_seq = 0;
  if (m.fb_count) {  // tier 4: large [snapshot, ...log] documents, one wave each; the rest go on to tier 5
    const uint64_t blk_cap = m.fb_bytes / 4 + 2ull * m.fb_count + 16, rec_cap = m.fb_bytes + 2ull * m.fb_count + 16;
    if (!c->big_blk.ensure(blk_cap * ygm_k_big_blk_bytes()) || !c->big_rec.ensure(rec_cap * ygm_k_big_rec_bytes()) ||
        !c->big_list.ensure((size_t)m.fb_count * 4 + 4) || !c->big_up.ensure((size_t)m.fb_count * 4 + 4) ||
        !c->big_scan.ensure(ygm_k_big_scan_bytes(m.fb_count, m.fb_bytes)))
      return YGM_ENOMEM;
    HIPCHK(hipEventRecord(c->e0, s));
    // the snapshot scan; then documents with a snapshot over BIG_MID_U0 on the 16-wave size (stream2) beside the mid
    // size over the rest (stream); a log over the mid size's LDS goes on to the 16-wave size after it
    if (ygm_k_launch_big_scan(P.arena, P.upd_off, P.doc_upd, c->fb_list.as<uint32_t>(), m.fb_count, c->flags, c->big_scan.p, m.fb_bytes, s))
      return YGM_EDEVICE;
    unsigned long long* d_cnt; uint32_t *llist, *mlist;
    ygm_k_big_lists(c->big_scan.p, m.fb_count, m.fb_bytes, &d_cnt, &llist, &mlist);
    unsigned long long cnt[4];
    c->stats.host_syncs++;
    HIPCHK(hipMemcpyAsync(c->h_meta, d_cnt, sizeof cnt, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    memcpy(cnt, c->h_meta, sizeof cnt);
    auto launch = [&](int large, const uint32_t* list, uint32_t n, hipStream_t st) {
      return ygm_k_launch_merge_big(large, P.arena, P.upd_off, P.doc_upd, c->fb_list.as<uint32_t>(), m.fb_count, list, n,
                                    c->big_up.as<uint32_t>(), c->flags, c->out.as<uint8_t>(), c->out_off.as<uint64_t>(),
                                    c->out_len.as<uint64_t>(), c->status.as<int32_t>(), P.meta, c->big_list.as<uint32_t>(), c->big_blk.p,
                                    blk_cap, c->big_rec.p, rec_cap, P.slot_total, P.out_cap, c->big_scan.p, m.fb_bytes, st);
    };
    // once the 16-wave size runs on stream2, every exit waits for it: its kernels write the outputs, the counters
    // and the tier's scratch, which the next call on this context reuses on `stream`
    struct Join2 {
      hipStream_t st = nullptr;
      ~Join2() { if (st) (void)hipStreamSynchronize(st); }
    } join2;
    if (cnt[2]) {
      if (!c->stream2) {   // created on first use, only on contexts that run the 16-wave size
        int prio_lo = 0, prio_hi = 0;
        HIPCHK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
#ifndef YGM_S2_PRIO
#define YGM_S2_PRIO 1
#endif
        HIPCHK(hipStreamCreateWithPriority(&c->stream2, hipStreamNonBlocking, YGM_S2_PRIO ? prio_hi : prio_lo));
      }
      HIPCHK(hipEventRecord(c->e2, s));
      HIPCHK(hipStreamWaitEvent(c->stream2, c->e2, 0));
      join2.st = c->stream2;
      if (launch(1, llist, (uint32_t)cnt[2], c->stream2)) return YGM_EDEVICE;
      HIPCHK(hipEventRecord(c->e3, c->stream2));
      if (cnt[3] && ygm_k_launch_big_wait(P.meta, (uint32_t)cnt[2], s)) return YGM_EDEVICE;   // (their workgroups resident first)
    }
    if (launch(0, mlist, (uint32_t)cnt[3], s)) return YGM_EDEVICE;
    if ((e = read_meta(c, s, m, P.meta))) return e;
    if (m.fault) return YGM_EDEVICE;
    if (m.mid_defer && launch(1, c->big_up.as<uint32_t>(), m.mid_defer, s)) return YGM_EDEVICE;
    if (cnt[2]) { HIPCHK(hipStreamWaitEvent(s, c->e3, 0)); join2.st = nullptr; }
    HIPCHK(hipEventRecord(c->e1, s));
    if ((e = read_meta(c, s, m, P.meta))) return e;
    if (m.fault) return YGM_EDEVICE;
    if (hipEventElapsedTime(&ms0, c->e0, c->e1) == hipSuccess) c->stats.kernel_ms += ms0;
    c->stats.docs_big += m.fb_count - m.big_defer;
    n_seq = m.big_defer;
  }
  if (n_seq) {  // tier 5: the exact sequential replay (scratch sized from the tier-4 counters: an upper bound)
    const uint64_t upd_cap = m.fb_upds + 1, byte_cap = m.fb_bytes + 8ull * m.fb_count + 8;
    if (!c->s_readers.ensure(upd_cap * ygm_k_seq_reader_bytes()) || !c->s_order.ensure(upd_cap * 4) || !c->s_tmp.ensure(upd_cap * 4) ||
        !c->s_ubase.ensure(upd_cap * 8) || !c->s_ulen.ensure(upd_cap * 4) || !c->s_cnt.ensure(byte_cap * 4) ||
        !c->s_drec.ensure((byte_cap / 2 + 1) * ygm_k_drec_bytes()))
      return YGM_ENOMEM;
    HIPCHK(hipEventRecord(c->e0, s));
    if (ygm_k_launch_merge_seq(P.arena, P.upd_off, P.doc_upd, c->big_list.as<uint32_t>(), n_seq, c->flags, c->out.as<uint8_t>(),
                               c->out_off.as<uint64_t>(), c->out_len.as<uint64_t>(), c->status.as<int32_t>(), P.meta,
                               c->s_readers.p, c->s_order.as<int>(), c->s_tmp.as<int>(), c->s_ubase.as<const uint8_t*>(),
                               c->s_ulen.as<uint32_t>(), upd_cap, c->s_cnt.as<uint32_t>(), c->s_drec.p, byte_cap, P.slot_total, P.out_cap, s))
      return YGM_EDEVICE;
    HIPCHK(hipEventRecord(c->e1, s));
    if ((e = read_meta(c, s, m, P.meta))) return e;
    if (hipEventElapsedTime(&ms0, c->e0, c->e1) == hipSuccess) c->stats.kernel_ms += ms0;
    c->stats.docs_seq += n_seq;
  }
  const uint64_t extent = P.slot_total + m.cursor;
  c->stats.calls++; c->stats.docs += P.n_docs; c->stats.updates += P.n_upd;
  c->stats.docs_fast += n_gen - m.fb_count;   // finished by the wave / workgroup tiers (tier 4 counted above)
  c->stats.docs_lean += P.n_docs - n_gen;      // finished by the lean kernels (narrow + wide)
  c->stats.bytes_in += P.arena_bytes; c->stats.bytes_out += m.payload_total();
  fill_dev_result(c, extent, out);
  out->payload_bytes = m.payload_total();
  return YGM_OK;
}

int ygm_merge_v1_device(ygm_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes, const uint64_t* d_upd_off,
                        const uint32_t* d_doc_upd, uint32_t n_upd, uint32_t n_docs, void* stream, ygm_device_result* out) {
  if (!c || !out) return YGM_EINVAL;
  const int e = ygm_merge_v1_device_async(c, d_arena, arena_bytes, d_upd_off, d_doc_upd, n_upd, n_docs, stream);
  if (e) return e;
  return ygm_merge_v1_device_finish(c, out);
}
int ygm_merge_v1_device_lens(ygm_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes, const uint64_t* d_doc_off,
                             const uint16_t* d_upd_len, const uint32_t* d_doc_upd, uint32_t n_upd, uint32_t n_docs, void* stream,
                             ygm_device_result* out) {
  if (!c || !out) return YGM_EINVAL;
  const int e = ygm_merge_v1_device_lens_async(c, d_arena, arena_bytes, d_doc_off, d_upd_len, d_doc_upd, n_upd, n_docs, stream);
  if (e) return e;
  return ygm_merge_v1_device_finish(c, out);
}

static int run_doc_kernel(ygm_ctx* c, int mode, const uint8_t* d_arena, uint64_t arena_bytes, const uint64_t* d_doc_off,
                          const uint8_t* d_sv, uint64_t sv_bytes, const uint64_t* d_sv_off, uint32_t n_docs, void* stream,
                          ygm_device_result* out, uint32_t extra_flags = 0) {
  const uint32_t flags = c ? c->flags | extra_flags : 0;
  if (!c || !out) return YGM_EINVAL;
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  (void)hipSetDevice(c->device);
  // per-document slots (lean kernel), then the packed region of the exact kernel's deferred documents
  const uint64_t slot_total = 2 * arena_bytes + 64ull * n_docs;
  const uint64_t out_cap = slot_total + 2 * arena_bytes + 32ull * n_docs + 64;
  int e = prep_outputs(c, n_docs, out_cap, s, true);
  if (e) return e;
  void* meta = c->meta_slot(2);
  if (mode == 1 && (!c->sv_tbl.ensure(ygm_k_sv_table_bytes(n_docs)) || !c->sv_tn.ensure(4ull * n_docs + 4))) return YGM_ENOMEM;
  HIPCHK(hipEventRecord(c->e0, s));
  if (ygm_k_launch_doc_lean(mode, d_arena, arena_bytes, d_doc_off, d_sv, sv_bytes, d_sv_off, n_docs, flags, c->out.as<uint8_t>(),
                            c->out_off.as<uint64_t>(), c->out_len.as<uint64_t>(), c->status.as<int32_t>(), meta,
                            c->defer_list.as<uint32_t>(), out_cap, c->sv_tbl.as<uint8_t>(), c->sv_tn.as<uint32_t>(), s))
    return YGM_EDEVICE;
  HIPCHK(hipEventRecord(c->e1, s));
  Meta m;
  if ((e = read_meta(c, s, m, meta))) return e;
  if (m.fault) return YGM_EDEVICE;
  float ms = 0;
  if (hipEventElapsedTime(&ms, c->e0, c->e1) == hipSuccess) { c->stats.kernel_ms += ms; c->stats.lean_ms += ms; c->stats.lean_launches++; }
  if (m.lean_defer) {   // the exact per-document kernel over the deferred list, packed after the slots
    HIPCHK(hipEventRecord(c->e0, s));
    if (ygm_k_launch_doc(mode, d_arena, d_doc_off, d_sv, d_sv_off, c->defer_list.as<uint32_t>(), slot_total, m.lean_defer, flags,
                         c->out.as<uint8_t>(), c->out_off.as<uint64_t>(), c->out_len.as<uint64_t>(), c->status.as<int32_t>(),
                         c->lb.as<unsigned long long>(), meta, out_cap, s))
      return YGM_EDEVICE;
    HIPCHK(hipEventRecord(c->e1, s));
    if ((e = read_meta(c, s, m, meta))) return e;
    if (m.fault) return YGM_EDEVICE;
    if (hipEventElapsedTime(&ms, c->e0, c->e1) == hipSuccess) c->stats.kernel_ms += ms;
  }
  const uint64_t payload = m.payload_total() + m.fast_total;
  c->stats.calls++; c->stats.docs += n_docs; c->stats.docs_fast += m.lean_defer; c->stats.docs_lean += n_docs - m.lean_defer;
  c->stats.bytes_in += arena_bytes; c->stats.bytes_out += payload;
  fill_dev_result(c, slot_total + m.fast_total, out);
  out->payload_bytes = payload;
  return YGM_OK;
}

// Documents k_snap left pending (ST_PEND: PendHdr, then [state, pendingDs, pending structs]): encodeStateAsUpdate
// returns mergeUpdates of the three (Y@23300).  They are packed into one arena as three-update documents (k_pend_plan /
// k_pend_copy) and merged by the merge kernels on the child context c->pend_ctx; the merged bytes are appended to the
// snapshot's output region at `used` and the documents' offsets, lengths and statuses rewritten (k_pend_fix).
// the pending documents' three-update batch (c->pn_arena / pn_off / pn_du, `total` bytes) merged on the child context
// c->pend_ctx; the merged bytes appended to `dst` at `used` and the documents' places, lengths and statuses written
// (pst: statuses decided before the merge, nullable)
static uint64_t read_u64(ygm_ctx* c, hipStream_t s, const uint64_t* d_p, int& e) {
  uint64_t v = 0;
  c->stats.host_syncs++;
  e = hipMemcpyAsync(c->h_meta, d_p, 8, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess ? YGM_EDEVICE : 0;
  memcpy(&v, c->h_meta, 8);
  return v;
}
static int pend_merge_place(ygm_ctx* c, hipStream_t s, uint32_t P, uint64_t total, const int32_t* pst, DevBuf& dst, uint64_t used,
                            uint64_t& data_bytes, unsigned long long& payload) {
  if (!c->pend_ctx) { const int e = ygm_open(c->device, c->flags, &c->pend_ctx); if (e) return e; }
  int e = ygm_merge_v1_device_async(c->pend_ctx, c->pn_arena.as<uint8_t>(), total, c->pn_off.as<uint64_t>(), c->pn_du.as<uint32_t>(), 3 * P, P, s);
  ygm_device_result r;
  if (!e) e = ygm_merge_v1_device_finish(c->pend_ctx, &r);
  if (e) return e;
  if (!dst.ensure(used + r.data_bytes + 64, used, s)) return YGM_ENOMEM;
  if (r.data_bytes) HIPCHK(hipMemcpyAsync(dst.as<uint8_t>() + used, r.data, r.data_bytes, hipMemcpyDeviceToDevice, s));
  if (ygm_k_launch_pend_fix(c->sn_pend.as<uint32_t>(), P, r.off, r.len, r.status, pst, used, c->out_off.as<uint64_t>(), c->out_len.as<uint64_t>(),
                            c->status.as<int32_t>(), s))
    return YGM_EDEVICE;
  data_bytes = used + r.data_bytes;
  payload += r.payload_bytes;
  c->stats.docs_pending += P;
  return YGM_OK;
}
static int snap_resolve_pending(ygm_ctx* c, hipStream_t s, uint32_t P, uint64_t used, uint64_t& data_bytes, unsigned long long& payload) {
  if (!c->pn_off.ensure(8ull * (3ull * P + 1) + 16) || !c->pn_du.ensure(4ull * (P + 1) + 16)) return YGM_ENOMEM;
  if (ygm_k_launch_pend_plan(c->sn_pend.as<uint32_t>(), P, c->sn_ws.as<uint8_t>(), c->out_off.as<uint64_t>(), c->pn_off.as<uint64_t>(),
                             c->pn_du.as<uint32_t>(), s))
    return YGM_EDEVICE;
  int e = 0;
  const uint64_t total = read_u64(c, s, c->pn_off.as<uint64_t>() + 3ull * P, e);
  if (e) return e;
  if (!c->pn_arena.ensure(total + 64)) return YGM_ENOMEM;
  HIPCHK(hipMemsetAsync(c->pn_arena.as<uint8_t>() + total, 0, 64, s));   // (the merge kernels' tail padding)
  if (ygm_k_launch_pend_copy(c->sn_pend.as<uint32_t>(), P, c->sn_ws.as<uint8_t>(), c->out_off.as<uint64_t>(), c->pn_off.as<uint64_t>(),
                             c->pn_arena.as<uint8_t>(), s))
    return YGM_EDEVICE;
  return pend_merge_place(c, s, P, total, nullptr, c->sn_ws, used, data_bytes, payload);
}

// the snapshot batch; xf: YGM_F_SNAP_STATE (contains) for states that leave pending parts
// leave: when non-null, documents left pending are not resolved: their count goes there (list c->sn_pend, statuses
// ST_PEND, their PendHdr layouts at out_off)
static int snapshot_dev(ygm_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes, const uint64_t* d_doc_off, uint32_t n_docs,
                        hipStream_t s, ygm_device_result* out, uint32_t xf, uint32_t* leave = nullptr) {
  if (leave) *leave = 0;
  const uint32_t fl = c->flags | xf;
  const uint32_t nb = (n_docs + 1 + 255) / 256;
  if (!c->sn_cnt.ensure(16ull * n_docs + 16) || !c->sn_off.ensure(8ull * n_docs + 16) || !c->sn_bs.ensure(8ull * nb + 16) ||
      !c->out_off.ensure(8ull * n_docs + 8) || !c->out_len.ensure(8ull * n_docs + 8) || !c->status.ensure(4ull * n_docs + 4))
    return YGM_ENOMEM;
  void* meta = c->meta_slot(2);
  HIPCHK(hipMemsetAsync(meta, 0, sizeof(Meta), s));
  HIPCHK(hipEventRecord(c->e0, s));
  // tier 1: k_snap_text (flat text; input + workspace in LDS) into per-document slots; the documents it leaves go to
  // the count / scan / k_snap path, whose workspaces follow the slot region
  const bool lds = n_docs && getenv("YGM_SNAP_NOLDS") == nullptr;
  const uint64_t slot_total = lds ? 2 * arena_bytes + 64ull * n_docs + 64 : 0;
  uint64_t lds_pay[2] = {0, 0};
  if (lds) {
    if (!c->sn_ws.ensure(slot_total + 64) || !c->sn_claim.ensure((size_t)n_docs + 16) || !c->sn_pay.ensure(16)) return YGM_ENOMEM;
    HIPCHK(hipMemsetAsync(c->sn_pay.p, 0, 16, s));
    for (int again = 0; again < 2 && lds_pay[1] < n_docs; again++) {   // 6 KiB per document, then 24 KiB for what it left
      if (ygm_k_launch_snap_text(d_arena, d_doc_off, n_docs, fl, c->sn_ws.as<uint8_t>(), c->out_off.as<uint64_t>(), c->out_len.as<uint64_t>(),
                                 c->status.as<int32_t>(), c->sn_claim.as<uint8_t>(), c->sn_pay.as<unsigned long long>(), again, slot_total, s))
        return YGM_EDEVICE;
      HIPCHK(hipMemcpyAsync(c->h_meta, c->sn_pay.p, 16, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      memcpy(lds_pay, c->h_meta, 16);
    }
  }
  uint64_t total = 0;   // workspace bytes: one read of the scanned total
  uint64_t total_out = 0;   // the output region's extent when pending documents' merged bytes follow the workspaces
  Meta m;
  memset(&m, 0, sizeof(m));
  if (!lds || lds_pay[1] < n_docs) {
    const uint8_t* claim = lds ? c->sn_claim.as<uint8_t>() : nullptr;
    if (ygm_k_launch_snap_plan(d_arena, d_doc_off, n_docs, fl, c->sn_cnt.p, c->sn_off.as<uint64_t>(), c->sn_bs.as<uint64_t>(), claim, s))
      return YGM_EDEVICE;
    if (n_docs) {
      HIPCHK(hipMemcpyAsync(c->h_meta, c->sn_off.as<uint64_t>() + n_docs, 8, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      memcpy(&total, c->h_meta, 8);
    }
    if (!c->sn_ws.ensure(slot_total + total + 64, slot_total, s) || !c->sn_pend.ensure(4ull * n_docs + 16)) return YGM_ENOMEM;
    if (ygm_k_launch_snap(d_arena, d_doc_off, n_docs, fl, c->sn_cnt.p, c->sn_off.as<uint64_t>(), c->sn_ws.as<uint8_t>(),
                          c->out_off.as<uint64_t>(), c->out_len.as<uint64_t>(), c->status.as<int32_t>(),
                          (unsigned long long*)((uint8_t*)meta + offsetof(Meta, payload)), claim, slot_total, c->sn_pend.as<uint32_t>(),
                          (unsigned int*)((uint8_t*)meta + offsetof(Meta, fb_count)), s))
      return YGM_EDEVICE;
    int e = read_meta(c, s, m, meta);
    if (e) return e;
    if (m.fb_count && leave) *leave = m.fb_count;
    else if (m.fb_count && (e = snap_resolve_pending(c, s, m.fb_count, slot_total + total, total_out, m.payload))) return e;
    HIPCHK(hipEventRecord(c->e1, s));
    HIPCHK(hipEventSynchronize(c->e1));
  } else {
    HIPCHK(hipEventRecord(c->e1, s));
    HIPCHK(hipEventSynchronize(c->e1));
  }
  m.payload += lds_pay[0];
  float ms = 0;
  if (hipEventElapsedTime(&ms, c->e0, c->e1) == hipSuccess) c->stats.kernel_ms += ms;
  c->stats.calls++; c->stats.docs += n_docs; c->stats.bytes_in += arena_bytes; c->stats.bytes_out += m.payload;
  out->data = c->sn_ws.as<uint8_t>(); out->off = c->out_off.as<uint64_t>(); out->len = c->out_len.as<uint64_t>();
  out->status = c->status.as<int32_t>(); out->data_bytes = total_out ? total_out : slot_total + total; out->payload_bytes = m.payload;
  return YGM_OK;
}
int ygm_snapshot_v1_device(ygm_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes, const uint64_t* d_doc_off, uint32_t n_docs,
                           void* stream, ygm_device_result* out) {
  if (!c || !out) return YGM_EINVAL;
  (void)hipSetDevice(c->device);
  return snapshot_dev(c, d_arena, arena_bytes, d_doc_off, n_docs, stream ? (hipStream_t)stream : c->stream, out, 0);
}
// a snapshot batch's outputs packed into one arena on the device (k_pack_*: offsets n + 1, the total at [n]) with its
// statuses, for kernels that read documents by offsets (step2's diff, contains)
static int pack_snapshots(ygm_ctx* c, hipStream_t s, const ygm_device_result& r1, uint32_t n_docs) {
  const uint32_t nb = (n_docs + 255) / 256;
  if (!c->s2_data.ensure(r1.payload_bytes + 64) || !c->s2_off.ensure(8ull * n_docs + 16) || !c->s2_bsum.ensure(8ull * nb + 16) ||
      !c->s2_st.ensure(4ull * n_docs + 4))
    return YGM_ENOMEM;
  HIPCHK(hipMemsetAsync((uint8_t*)c->s2_data.p + r1.payload_bytes, 0, 64, s));   // readable tail for the walker's chunks
  if (n_docs) {
    if (ygm_k_launch_pack(r1.data, r1.off, r1.len, r1.status, n_docs, c->s2_bsum.as<uint64_t>(), c->s2_data.as<uint8_t>(),
                          c->s2_off.as<uint64_t>(), s))
      return YGM_EDEVICE;
    HIPCHK(hipMemcpyAsync(c->s2_off.as<uint64_t>() + n_docs, c->s2_bsum.as<uint64_t>() + nb, 8, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(c->s2_st.p, r1.status, 4ull * n_docs, hipMemcpyDeviceToDevice, s));
  } else HIPCHK(hipMemsetAsync(c->s2_off.p, 0, 8, s));
  return YGM_OK;
}

// Read-only SyncStep2: the states' Y.snapshot view first -- the snapshot batch with YGM_F_SNAP_STATE (a state that
// leaves pending structs / a pending delete set is seen through its integrated part, as Y.snapshot(doc) sees the
// store) -- packed, then the containment kernels over it; the snapshot's per-document refusals carried into the result
int ygm_contains_v1_device(ygm_ctx* c, const uint8_t* d_states_in, const uint64_t* d_state_off_in, const uint8_t* d_updates,
                           const uint64_t* d_update_off, uint32_t n_docs, void* stream, ygm_device_result* out) {
  if (!c || !out) return YGM_EINVAL;
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  (void)hipSetDevice(c->device);
  uint64_t states_bytes = 0;
  if (n_docs) {
    c->stats.host_syncs++;
    HIPCHK(hipMemcpyAsync(c->h_meta, d_state_off_in + n_docs, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    memcpy(&states_bytes, c->h_meta, 8);
  }
  ygm_device_result r1;
  int e0 = snapshot_dev(c, d_states_in, states_bytes, d_state_off_in, n_docs, s, &r1, YGM_F_SNAP_STATE);
  if (e0 || (e0 = pack_snapshots(c, s, r1, n_docs))) return e0;
  const uint8_t* d_states = c->s2_data.as<uint8_t>();
  const uint64_t* d_state_off = c->s2_off.as<uint64_t>();
  const uint32_t nb = (n_docs + 1 + 255) / 256;
  if (!c->sn_off.ensure(8ull * n_docs + 16) || !c->sn_bs.ensure(8ull * nb + 16) || !c->out.ensure((uint64_t)n_docs + 64) ||
      !c->out_off.ensure(8ull * n_docs + 8) || !c->out_len.ensure(8ull * n_docs + 8) || !c->status.ensure(4ull * n_docs + 4))
    return YGM_ENOMEM;
  HIPCHK(hipEventRecord(c->e0, s));
  if (ygm_k_launch_cont_plan(d_states, d_state_off, n_docs, c->flags, c->sn_off.as<uint64_t>(), c->sn_bs.as<uint64_t>(), s)) return YGM_EDEVICE;
  uint64_t total = 0;
  if (n_docs) {
    HIPCHK(hipMemcpyAsync(c->h_meta, c->sn_off.as<uint64_t>() + n_docs, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    memcpy(&total, c->h_meta, 8);
  }
  if (!c->sn_ws.ensure(total + 64)) return YGM_ENOMEM;
  if (ygm_k_launch_cont(d_states, d_state_off, d_updates, d_update_off, n_docs, c->flags, c->sn_off.as<uint64_t>(), c->sn_ws.as<uint8_t>(),
                        c->out.as<uint8_t>(), c->out_off.as<uint64_t>(), c->out_len.as<uint64_t>(), c->status.as<int32_t>(), s))
    return YGM_EDEVICE;
  if (n_docs && ygm_k_launch_v2_status(c->s2_st.as<int32_t>(), n_docs, c->status.as<int32_t>(), c->out_len.as<uint64_t>(), s))
    return YGM_EDEVICE;
  HIPCHK(hipEventRecord(c->e1, s));
  HIPCHK(hipStreamSynchronize(s));
  float ms = 0;
  if (hipEventElapsedTime(&ms, c->e0, c->e1) == hipSuccess) c->stats.kernel_ms += ms;
  c->stats.calls++; c->stats.docs += n_docs;
  out->data = c->out.as<uint8_t>(); out->off = c->out_off.as<uint64_t>(); out->len = c->out_len.as<uint64_t>();
  out->status = c->status.as<int32_t>(); out->data_bytes = n_docs; out->payload_bytes = n_docs;
  return YGM_OK;
}

int ygm_diff_v1_device(ygm_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes, const uint64_t* d_doc_off, const uint8_t* d_sv_arena,
                       const uint64_t* d_sv_off, uint32_t n_docs, void* stream, ygm_device_result* out) {
  // (the state-vector arena's extent is the last offset; its 16-byte window reads stay inside its padding)
  uint64_t sv_end = 0;
  if (n_docs && hipMemcpy(&sv_end, d_sv_off + n_docs, 8, hipMemcpyDeviceToHost) != hipSuccess) return YGM_EDEVICE;
  return run_doc_kernel(c, 1, d_arena, arena_bytes, d_doc_off, d_sv_arena, sv_end, d_sv_off, n_docs, stream, out);
}

int ygm_sv_from_update_v1_device(ygm_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes, const uint64_t* d_doc_off, uint32_t n_docs,
                                 void* stream, ygm_device_result* out) {
  return run_doc_kernel(c, 0, d_arena, arena_bytes, d_doc_off, nullptr, 0, nullptr, n_docs, stream, out);
}

// SyncStep2 of the documents the snapshot left pending (P of them, list c->sn_pend, PendHdr layouts in its output
// region: split off before the main diff, finished after it): encodeStateAsUpdate(doc, sv) = mergeUpdates([writeStateAsUpdate(doc, sv), pendingDs, diffUpdate(pending
// structs, sv)]) (Y@23300) -- the state part diffed keeping each struct's parentSub bit (an integrated item's write),
// the pending structs by the plain diff (the lazy writer's), on two child contexts; the three merged on a third, and
// appended to the step2 result (`out`, the diff kernels' output region) in the documents' places
// split (before the main diff reuses the snapshot's out_off): parts and state vectors into c->pq_*; tot: their bytes
static int step2_pending_split(ygm_ctx* c, hipStream_t s, uint32_t P, const uint8_t* d_sv_arena, const uint64_t* d_sv_off, uint64_t (&tot)[4]) {
  const uint64_t np = (uint64_t)P + 1;
  if (!c->pq_off.ensure(8ull * 4 * np + 16) || !c->pq_st.ensure(4ull * P + 16) || !c->pn_off.ensure(8ull * (3ull * P + 1) + 16) ||
      !c->pn_du.ensure(4ull * np + 16))
    return YGM_ENOMEM;
  uint64_t* offs = c->pq_off.as<uint64_t>();
  if (ygm_k_launch_pend_split(c->sn_pend.as<uint32_t>(), P, c->sn_ws.as<uint8_t>(), c->out_off.as<uint64_t>(), d_sv_arena, d_sv_off, offs,
                              nullptr, nullptr, nullptr, nullptr, 0, s))
    return YGM_EDEVICE;
  c->stats.host_syncs++;
  for (int k = 0; k < 4; k++) HIPCHK(hipMemcpyAsync((uint64_t*)c->h_meta + k, offs + (uint64_t)k * np + P, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  memcpy(tot, c->h_meta, sizeof tot);
  DevBuf* part[4] = {&c->pq_a, &c->pq_b, &c->pq_c, &c->pq_s};
  for (int k = 0; k < 4; k++) {
    if (!part[k]->ensure(tot[k] + 64)) return YGM_ENOMEM;
    HIPCHK(hipMemsetAsync(part[k]->as<uint8_t>() + tot[k], 0, 64, s));   // (readable tail padding for the kernels)
  }
  if (ygm_k_launch_pend_split(c->sn_pend.as<uint32_t>(), P, c->sn_ws.as<uint8_t>(), c->out_off.as<uint64_t>(), d_sv_arena, d_sv_off, offs,
                              c->pq_a.as<uint8_t>(), c->pq_b.as<uint8_t>(), c->pq_c.as<uint8_t>(), c->pq_s.as<uint8_t>(), 1, s))
    return YGM_EDEVICE;
  return YGM_OK;
}
// finish (after the main diff): the two diffs, the join, the merge, the places in `out`
static int step2_pending_finish(ygm_ctx* c, hipStream_t s, uint32_t P, const uint64_t (&tot)[4], ygm_device_result* out) {
  const uint64_t np = (uint64_t)P + 1;
  uint64_t* offs = c->pq_off.as<uint64_t>();
  for (ygm_ctx*& k : c->pend_dx) if (!k) { const int e = ygm_open(c->device, c->flags, &k); if (e) return e; }
  ygm_device_result ra, rc;
  int e = run_doc_kernel(c->pend_dx[0], 1, c->pq_a.as<uint8_t>(), tot[0], offs, c->pq_s.as<uint8_t>(), tot[3], offs + 3 * np, P, s, &ra,
                         YGM_F_KEEP_SUB);
  if (!e) e = run_doc_kernel(c->pend_dx[1], 1, c->pq_c.as<uint8_t>(), tot[2], offs + 2 * np, c->pq_s.as<uint8_t>(), tot[3], offs + 3 * np, P,
                             s, &rc, 0);
  if (e) return e;
  if (ygm_k_launch_pend_join(P, ra.data, ra.off, ra.len, ra.status, c->pq_b.as<uint8_t>(), offs, rc.data, rc.off, rc.len, rc.status,
                             c->pn_off.as<uint64_t>(), c->pn_du.as<uint32_t>(), c->pq_st.as<int32_t>(), nullptr, 0, s))
    return YGM_EDEVICE;
  const uint64_t total = read_u64(c, s, c->pn_off.as<uint64_t>() + 3ull * P, e);
  if (e) return e;
  if (!c->pn_arena.ensure(total + 64)) return YGM_ENOMEM;
  HIPCHK(hipMemsetAsync(c->pn_arena.as<uint8_t>() + total, 0, 64, s));
  if (ygm_k_launch_pend_join(P, ra.data, ra.off, ra.len, ra.status, c->pq_b.as<uint8_t>(), offs, rc.data, rc.off, rc.len, rc.status,
                             c->pn_off.as<uint64_t>(), c->pn_du.as<uint32_t>(), c->pq_st.as<int32_t>(), c->pn_arena.as<uint8_t>(), 1, s))
    return YGM_EDEVICE;
  uint64_t db = 0;
  unsigned long long pay = out->payload_bytes;
  if ((e = pend_merge_place(c, s, P, total, c->pq_st.as<int32_t>(), c->out, out->data_bytes, db, pay))) return e;
  out->data = c->out.as<uint8_t>(); out->data_bytes = db; out->payload_bytes = pay;
  return YGM_OK;
}

// SyncStep2 of stored documents (MessageReceiver.ts:137-138): the snapshot batch, its outputs packed into one arena
// on the device (k_pack_*: offsets n + 1, the total at [n]), the diff kernels over it with F_KEEP_SUB, and the
// snapshot's per-document refusals (EUNSUPPORTED, malformed states) carried into the result; states that leave
// pending parts by step2_pending_split / _finish
int ygm_sync_step2_v1_device(ygm_ctx* c, const uint8_t* d_states, uint64_t states_bytes, const uint64_t* d_state_off,
                             const uint8_t* d_sv_arena, const uint64_t* d_sv_off, uint32_t n_docs, void* stream,
                             ygm_device_result* out) {
  if (!c || !out) return YGM_EINVAL;
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  (void)hipSetDevice(c->device);
  ygm_device_result r1;
  const bool dbg = getenv("YGM_DEBUG") != nullptr;
#define S2CHK(x) do { hipError_t _e = (x); if (_e != hipSuccess) { if (dbg) fprintf(stderr, "ygm step2: %s: %s\n", #x, hipGetErrorString(_e)); return YGM_EDEVICE; } } while (0)
  uint32_t P = 0;   // documents the snapshot leaves pending (their parts split off now, answered after the diff)
  uint64_t ptot[4] = {0, 0, 0, 0};
  int e = snapshot_dev(c, d_states, states_bytes, d_state_off, n_docs, s, &r1, 0, &P);
  if (!e && P) e = step2_pending_split(c, s, P, d_sv_arena, d_sv_off, ptot);
  if (dbg) fprintf(stderr, "ygm step2: snapshot rc %d payload %llu\n", e, (unsigned long long)r1.payload_bytes);
  if (e || (e = pack_snapshots(c, s, r1, n_docs))) return e;
  uint64_t sv_end = 0;
  if (n_docs && hipMemcpy(&sv_end, d_sv_off + n_docs, 8, hipMemcpyDeviceToHost) != hipSuccess) return YGM_EDEVICE;
  e = run_doc_kernel(c, 1, c->s2_data.as<uint8_t>(), r1.payload_bytes, c->s2_off.as<uint64_t>(), d_sv_arena, sv_end, d_sv_off, n_docs, s,
                     out, YGM_F_KEEP_SUB);
  if (dbg) fprintf(stderr, "ygm step2: diff rc %d\n", e);
  if (e) return e;
  if (n_docs && ygm_k_launch_v2_status(c->s2_st.as<int32_t>(), n_docs, out->status, out->len, s)) return YGM_EDEVICE;
  if (P && (e = step2_pending_finish(c, s, P, ptot, out))) return e;
  S2CHK(hipStreamSynchronize(s));
  return YGM_OK;
#undef S2CHK
}

// ------------------------------------------------------------------ update V2 (device API)
// V2 -> V1 of n units (merge: updates, with doc_upd so single-input documents are skipped; otherwise one per
// document): sizes, scan (c->v2_len becomes the V1 offsets, total at [n]), bytes into c->v2_v1
static int v21_pass(ygm_ctx* c, hipStream_t s, const uint8_t* arena, const uint64_t* off, uint32_t n, const uint32_t* doc_upd,
                    uint32_t n_docs, uint32_t mode, uint64_t& total) {
  const size_t nb = ((size_t)n + 1 + 255) / 256 + 2;
  if (!c->v2_len.ensure(8ull * n + 16) || !c->v2_st.ensure(4ull * n + 4) || !c->v2_bs.ensure(8 * nb) || !c->v21_cl.ensure((size_t)n + 16))
    return YGM_ENOMEM;
  // the register-resident transcoder first (claims), the general one for the rest; the public conversion: general only
  uint8_t* cl = (mode & 1u) || getenv("YGM_V21_NOFAST") ? nullptr : c->v21_cl.as<uint8_t>();
  total = 0;
  if (n == 0) { HIPCHK(hipMemsetAsync(c->v2_len.p, 0, 8, s)); }
  else {
    if (ygm_k_launch_v21(0, arena, off, n, doc_upd, n_docs, mode, c->flags, c->v2_len.as<uint64_t>(), c->v2_st.as<int32_t>(), nullptr, cl, s) ||
        ygm_k_launch_scan(c->v2_len.as<uint64_t>(), n, c->v2_bs.as<uint64_t>(), s))
      return YGM_EDEVICE;
    HIPCHK(hipMemcpyAsync(c->h_meta, c->v2_len.as<uint64_t>() + n, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    memcpy(&total, c->h_meta, 8);
  }
  if (!c->v2_v1.ensure(total + 64)) return YGM_ENOMEM;   // (the V1 kernels read up to 64 bytes past the arena)
  if (n && ygm_k_launch_v21(1, arena, off, n, doc_upd, n_docs, mode, c->flags, c->v2_len.as<uint64_t>(), c->v2_st.as<int32_t>(),
                            c->v2_v1.as<uint8_t>(), cl, s))
    return YGM_EDEVICE;
  return YGM_OK;
}
// V1 -> V2 per document with final statuses.  Documents in the fast encoder's shape (ygm_v2_fast.hpp) are done by
// k_v12_fast into slots of c->v2_out placed from slot_off (the V2 input offsets: merge_slot of the document's input
// bytes); the rest take k_v12_count / scan / k_v12_write, packed after the slot region.  slot_off == nullptr (the
// public conversion): the general kernels only.
static int v12_pass(ygm_ctx* c, hipStream_t s, const uint8_t* v1, const uint64_t* v1_off, const uint64_t* v1_len, const int32_t* v1_st,
                    const uint8_t* v2a, uint64_t v2n, const uint64_t* upd_off, const uint32_t* doc_upd, const int32_t* ust, uint32_t n_docs,
                    uint32_t mode, const uint64_t* slot_off, ygm_device_result* out) {
  const size_t nb = ((size_t)n_docs + 1 + 255) / 256 + 2;
  if (!c->v2_L.ensure(4ull * ygm_k_v2_cols() * n_docs + 16) || !c->v2_off.ensure(8ull * n_docs + 16) || !c->v2_olen.ensure(8ull * n_docs + 8) ||
      !c->v2_ost.ensure(4ull * n_docs + 4) || !c->v2_bs.ensure(8 * nb) || !c->v2_fo.ensure(8ull * n_docs + 8) ||
      !c->v2_claim.ensure((size_t)n_docs + 16) || !c->v2_pay.ensure(16))
    return YGM_ENOMEM;
  const bool fast = slot_off != nullptr && !(mode & 1u) && getenv("YGM_V2_NOFAST") == nullptr;
  const uint64_t slot_total = fast ? 2 * v2n + 64ull * n_docs : 0;
  uint8_t* claim = fast ? c->v2_claim.as<uint8_t>() : nullptr;
  uint64_t total = 0, fast_bytes = 0, fast_docs = 0;
  if (fast && n_docs) {
    if (!c->v2_out.ensure(slot_total + 64) || !c->v2_scr.ensure(ygm_k_v12_fast_scratch())) return YGM_ENOMEM;
    HIPCHK(hipMemsetAsync(c->v2_pay.p, 0, 16, s));
    if (ygm_k_launch_v12_fast(v1, v1_off, v1_len, v1_st, slot_off, doc_upd, ust, n_docs, c->v2_out.as<uint8_t>(), c->v2_fo.as<uint64_t>(),
                              c->v2_olen.as<uint64_t>(), c->v2_ost.as<int32_t>(), claim, c->v2_pay.as<unsigned long long>(),
                              c->v2_scr.as<uint8_t>(), slot_total, s))
      return YGM_EDEVICE;
    HIPCHK(hipMemcpyAsync(c->h_meta, c->v2_pay.p, 16, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    memcpy(&fast_bytes, c->h_meta, 8); memcpy(&fast_docs, (uint8_t*)c->h_meta + 8, 8);
  }
  if (fast && fast_docs == n_docs) {   // every document done by the fast encoder: no general pass
    out->data = c->v2_out.as<uint8_t>(); out->off = c->v2_fo.as<uint64_t>(); out->len = c->v2_olen.as<uint64_t>();
    out->status = c->v2_ost.as<int32_t>(); out->data_bytes = slot_total; out->payload_bytes = fast_bytes;
    return YGM_OK;
  }
  if (n_docs) {
    if (ygm_k_launch_v12_count(v1, v1_off, v1_len, v1_st, v2a, v2n, upd_off, doc_upd, ust, n_docs, mode, c->flags, c->v2_L.as<uint32_t>(),
                               c->v2_off.as<uint64_t>(), c->v2_ost.as<int32_t>(), claim, s) ||
        ygm_k_launch_scan(c->v2_off.as<uint64_t>(), n_docs, c->v2_bs.as<uint64_t>(), s))
      return YGM_EDEVICE;
    HIPCHK(hipMemcpyAsync(c->h_meta, c->v2_off.as<uint64_t>() + n_docs, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    memcpy(&total, c->h_meta, 8);
  }
  if (!c->v2_out.ensure(slot_total + total + 64, slot_total, s)) return YGM_ENOMEM;
  if (n_docs && ygm_k_launch_v12_write(v1, v1_off, v1_len, v2a, v2n, upd_off, doc_upd, n_docs, mode, c->flags, c->v2_L.as<uint32_t>(),
                                       c->v2_off.as<uint64_t>(), c->v2_ost.as<int32_t>(), c->v2_out.as<uint8_t>(), c->v2_olen.as<uint64_t>(),
                                       claim, slot_total, c->v2_fo.as<uint64_t>(), s))
    return YGM_EDEVICE;
  out->data = c->v2_out.as<uint8_t>(); out->off = c->v2_fo.as<uint64_t>(); out->len = c->v2_olen.as<uint64_t>();
  out->status = c->v2_ost.as<int32_t>(); out->data_bytes = slot_total + total; out->payload_bytes = total + fast_bytes;
  return YGM_OK;
}
static const uint32_t V2_EXPORT = 1u, V2_STRUCTS_ONLY = 2u;

// the span of a V2 call's own kernels (the V1 operation inside times itself)
struct V2Timer {
  ygm_ctx* c; hipStream_t s; float pre = 0;
  V2Timer(ygm_ctx* c_, hipStream_t s_) : c(c_), s(s_) { (void)hipEventRecord(c->e2, s); }
  void split() { (void)hipEventRecord(c->e3, s); (void)hipEventSynchronize(c->e3); float ms = 0; if (hipEventElapsedTime(&ms, c->e2, c->e3) == hipSuccess) pre += ms; }
  void resume() { (void)hipEventRecord(c->e2, s); }
  void done() { split(); c->stats.kernel_ms += pre; }
};

int ygm_merge_v2_device(ygm_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes, const uint64_t* d_upd_off, const uint32_t* d_doc_upd,
                        uint32_t n_upd, uint32_t n_docs, void* stream, ygm_device_result* out) {
  if (!c || !out) return YGM_EINVAL;
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  (void)hipSetDevice(c->device);
  V2Timer T(c, s);
  uint64_t v1_bytes = 0;
  int e = v21_pass(c, s, d_arena, d_upd_off, n_upd, d_doc_upd, n_docs, 0, v1_bytes);
  if (e) return e;
  T.split();
  ygm_device_result r1;
  if ((e = ygm_merge_v1_device(c, c->v2_v1.as<uint8_t>(), v1_bytes, c->v2_len.as<uint64_t>(), d_doc_upd, n_upd, n_docs, s, &r1))) return e;
  T.resume();
  e = v12_pass(c, s, r1.data, r1.off, r1.len, r1.status, d_arena, arena_bytes, d_upd_off, d_doc_upd, c->v2_st.as<int32_t>(), n_docs, 0, d_upd_off, out);
  T.done();
  return e;
}
int ygm_diff_v2_device(ygm_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes, const uint64_t* d_doc_off, const uint8_t* d_sv_arena,
                       const uint64_t* d_sv_off, uint32_t n_docs, void* stream, ygm_device_result* out) {
  if (!c || !out) return YGM_EINVAL;
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  (void)hipSetDevice(c->device);
  V2Timer T(c, s);
  uint64_t v1_bytes = 0;
  int e = v21_pass(c, s, d_arena, d_doc_off, n_docs, nullptr, n_docs, 0, v1_bytes);
  if (e) return e;
  T.split();
  ygm_device_result r1;
  if ((e = ygm_diff_v1_device(c, c->v2_v1.as<uint8_t>(), v1_bytes, c->v2_len.as<uint64_t>(), d_sv_arena, d_sv_off, n_docs, s, &r1))) return e;
  T.resume();
  e = v12_pass(c, s, r1.data, r1.off, r1.len, r1.status, d_arena, arena_bytes, nullptr, nullptr, c->v2_st.as<int32_t>(), n_docs, 0, d_doc_off, out);
  T.done();
  return e;
}
int ygm_sv_from_update_v2_device(ygm_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes, const uint64_t* d_doc_off, uint32_t n_docs,
                                 void* stream, ygm_device_result* out) {
  if (!c || !out) return YGM_EINVAL;
  (void)arena_bytes;
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  (void)hipSetDevice(c->device);
  V2Timer T(c, s);
  uint64_t v1_bytes = 0;
  int e = v21_pass(c, s, d_arena, d_doc_off, n_docs, nullptr, n_docs, V2_STRUCTS_ONLY, v1_bytes);
  if (e) return e;
  T.split();
  if ((e = ygm_sv_from_update_v1_device(c, c->v2_v1.as<uint8_t>(), v1_bytes, c->v2_len.as<uint64_t>(), n_docs, s, out))) return e;
  T.resume();
  if (ygm_k_launch_v2_status(c->v2_st.as<int32_t>(), n_docs, out->status, out->len, s)) return YGM_EDEVICE;
  T.done();
  return YGM_OK;
}
int ygm_convert_v1_to_v2_device(ygm_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes, const uint64_t* d_doc_off, uint32_t n_docs,
                                void* stream, ygm_device_result* out) {
  if (!c || !out) return YGM_EINVAL;
  (void)arena_bytes;
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  (void)hipSetDevice(c->device);
  V2Timer T(c, s);
  const int e = v12_pass(c, s, d_arena, d_doc_off, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr, n_docs, V2_EXPORT, nullptr, out);
  T.done();
  if (!e) { c->stats.calls++; c->stats.docs += n_docs; }
  return e;
}
int ygm_convert_v2_to_v1_device(ygm_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes, const uint64_t* d_doc_off, uint32_t n_docs,
                                void* stream, ygm_device_result* out) {
  if (!c || !out) return YGM_EINVAL;
  (void)arena_bytes;
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  (void)hipSetDevice(c->device);
  V2Timer T(c, s);
  uint64_t v1_bytes = 0;
  int e = v21_pass(c, s, d_arena, d_doc_off, n_docs, nullptr, n_docs, V2_EXPORT, v1_bytes);
  if (e) return e;
  if (!c->v2_olen.ensure(8ull * n_docs + 8)) return YGM_ENOMEM;
  if (ygm_k_launch_v2_lens(c->v2_len.as<uint64_t>(), c->v2_st.as<int32_t>(), n_docs, c->v2_olen.as<uint64_t>(), s)) return YGM_EDEVICE;
  T.done();
  c->stats.calls++; c->stats.docs += n_docs;
  out->data = c->v2_v1.as<uint8_t>(); out->off = c->v2_len.as<uint64_t>(); out->len = c->v2_olen.as<uint64_t>();
  out->status = c->v2_st.as<int32_t>(); out->data_bytes = v1_bytes; out->payload_bytes = v1_bytes;
  return YGM_OK;
}

// ------------------------------------------------------------------ host API
// A batch is cut into chunks of whole documents (about YGM_CHUNK_BYTES of input each) that alternate
// between two stage contexts, each with its own stream and device buffers:
//   stage i+1: host arena -> pinned staging (CPU copy) -> H2D        (stream of stage (i+1) % 2)
//   chunk i:   kernels -> device-side packing of the outputs -> D2H   (stream of stage i % 2)
// so the CPU copy and the H2D of one chunk overlap the kernels of the previous one, and the D2H moves
// only the packed outputs (not the per-document slots).  h2d_ms / d2h_ms are the copies' HIP-event
// times (summed over chunks); the results live in the parent context's pinned buffers.
static const uint64_t YGM_CHUNK_BYTES = 64ull << 20;
// A batch of large [snapshot, ...log] documents runs the large-document tier once per chunk, each run as long as its
// largest document: a third of the batch per chunk (at least 64 MB) keeps the copies overlapped and the tier's runs
// few (tools/host_probe.py, profiles/r06_final/host_chunks.jsonl).  YGM_CHUNK_MB overrides (experiments).
static uint64_t chunk_bytes(uint64_t in_bytes) {
  const char* e = getenv("YGM_CHUNK_MB");
  if (e && atoi(e) > 0) return (uint64_t)atoi(e) << 20;
  return in_bytes / 3 > YGM_CHUNK_BYTES ? in_bytes / 3 : YGM_CHUNK_BYTES;
}

namespace {
struct Chunk {   // documents [d0, d1): merge updates [u0, u1) / SV-diff documents
  uint32_t d0, d1, u0, u1;
  uint64_t pos = 0, payload = 0;   // packed output position in the parent's result, bytes
  hipEvent_t h0 = nullptr, h1 = nullptr, o0 = nullptr, o1 = nullptr;
};
struct HostCall {
  int mode;   // 0 sv, 1 diff, 2 merge, 3 snapshot, 4 contains (second arena in the sv slots); update V2: 5 merge, 6 diff,
              // 7 sv, 8 V1 -> V2, 9 V2 -> V1; 10 sync step2 (states + state vectors)
  const uint8_t* arena; const uint64_t* off; const uint32_t* upd_doc; const uint8_t* sv_arena; const uint64_t* sv_off;
  uint32_t n_upd, n_docs;
};
}  // namespace

static int stage_ctx(ygm_ctx* c, int i, ygm_ctx** out) {
  if (!c->kid[i]) { int e = ygm_open(c->device, c->flags, &c->kid[i]); if (e) return e; }
  *out = c->kid[i];
  return YGM_OK;
}

// large host copies split over threads (one core copies ~10 GB/s; PCIe takes ~55 GB/s)
static void par_memcpy(uint8_t* dst, const uint8_t* src, size_t n) {
  const size_t per = 8u << 20;
  unsigned t = (unsigned)std::min<size_t>((n + per - 1) / per, 8);
  const unsigned hw = std::thread::hardware_concurrency();
  if (hw && t > hw) t = hw;
  if (t <= 1) { memcpy(dst, src, n); return; }
  std::vector<std::thread> th;
  const size_t part = (n + t - 1) / t;
  for (unsigned i = 1; i < t; i++) {
    const size_t a = i * part, b = std::min(n, a + part);
    if (a < b) th.emplace_back([=] { memcpy(dst + a, src + a, b - a); });
  }
  memcpy(dst, src, std::min(n, part));
  for (auto& x : th) x.join();
}

// f(begin, end) over [0, n) split over threads when n is large
extern "C++" template <class F>
static void par_for(size_t n, F f) {
  const size_t per = 1u << 20;
  unsigned t = (unsigned)std::min<size_t>((n + per - 1) / per, 8);
  const unsigned hw = std::thread::hardware_concurrency();
  if (hw && t > hw) t = hw;
  if (t <= 1) { f((size_t)0, n); return; }
  std::vector<std::thread> th;
  const size_t part = (n + t - 1) / t;
  for (unsigned i = 1; i < t; i++) {
    const size_t a = i * part, b = std::min(n, a + part);
    if (a < b) th.emplace_back([=] { f(a, b); });
  }
  f((size_t)0, std::min(n, part));
  for (auto& x : th) x.join();
}

// CPU copy of a chunk's inputs into the stage's pinned buffer, then the async H2D copies
static bool is_merge(int mode) { return mode == 2 || mode == 5; }
static int chunk_stage(ygm_ctx* k, const HostCall& H, Chunk& C) {
  const bool two = H.mode == 1 || H.mode == 4 || H.mode == 6 || H.mode == 10;   // a second arena per document (diff: state vectors, contains: updates)
  const uint32_t nd = C.d1 - C.d0;
  const uint64_t a0 = is_merge(H.mode) ? H.off[C.u0] : H.off[C.d0], a1 = is_merge(H.mode) ? H.off[C.u1] : H.off[C.d1];
  const uint64_t bytes = a1 - a0, ab = (bytes + 64 + 15) & ~15ull;
  const uint32_t nu = is_merge(H.mode) ? C.u1 - C.u0 : nd;
  uint64_t s0 = 0, s1 = 0, sb = 0;
  if (two) { s0 = H.sv_off[C.d0]; s1 = H.sv_off[C.d1]; sb = ((s1 - s0) + 64 + 15) & ~15ull; }
  const uint64_t n_off = (uint64_t)nu + 1, n_doc = is_merge(H.mode) ? (uint64_t)nd + 1 : 0, n_sv = two ? (uint64_t)nd + 1 : 0;
  const uint64_t need = ab + 8 * n_off + sb + 8 * n_sv + 4 * n_doc + 64;
  if (!k->h_in.ensure(need)) return YGM_ENOMEM;
  uint8_t* P = k->h_in.as<uint8_t>();
  par_memcpy(P, H.arena + a0, bytes); memset(P + bytes, 0, ab - bytes);
  uint64_t* ro = (uint64_t*)(P + ab);
  const uint64_t* src_off = is_merge(H.mode) ? H.off + C.u0 : H.off + C.d0;
  par_for(n_off, [=](size_t a, size_t b) { for (size_t j = a; j < b; j++) ro[j] = src_off[j] - a0; });
  uint8_t* q = P + ab + 8 * n_off;
  if (two) {
    memcpy(q, H.sv_arena + s0, s1 - s0); memset(q + (s1 - s0), 0, sb - (s1 - s0));
    uint64_t* rs = (uint64_t*)(q + sb);
    for (uint64_t j = 0; j < n_sv; j++) rs[j] = H.sv_off[C.d0 + j] - s0;
    q += sb + 8 * n_sv;
  }
  if (is_merge(H.mode)) {   // per-document update ranges, relative to the chunk (one walk over its updates: a binary
                            // search per document measured 2-3x slower end to end, tools/host_probe.py)
    uint32_t* du = (uint32_t*)q;
    du[0] = 0;
    uint32_t u = C.u0;
    for (uint32_t d = 0; d < nd; d++) { while (u < C.u1 && H.upd_doc[u] == C.d0 + d) u++; du[d + 1] = u - C.u0; }
  }
  if (!k->arena.ensure(ab) || !k->offs.ensure(8 * n_off) || (two && (!k->sv_arena.ensure(sb) || !k->sv_offs.ensure(8 * n_sv))) ||
      (is_merge(H.mode) && !k->docs.ensure(4 * n_doc)))
    return YGM_ENOMEM;
  HIPCHK(hipEventRecord(C.h0, k->stream));
  HIPCHK(hipMemcpyAsync(k->arena.p, P, ab, hipMemcpyHostToDevice, k->stream));
  HIPCHK(hipMemcpyAsync(k->offs.p, ro, 8 * n_off, hipMemcpyHostToDevice, k->stream));
  if (two) {
    HIPCHK(hipMemcpyAsync(k->sv_arena.p, P + ab + 8 * n_off, sb, hipMemcpyHostToDevice, k->stream));
    HIPCHK(hipMemcpyAsync(k->sv_offs.p, P + ab + 8 * n_off + sb, 8 * n_sv, hipMemcpyHostToDevice, k->stream));
  }
  if (is_merge(H.mode)) HIPCHK(hipMemcpyAsync(k->docs.p, q, 4 * n_doc, hipMemcpyHostToDevice, k->stream));
  HIPCHK(hipEventRecord(C.h1, k->stream));
  return YGM_OK;
}

// kernels of a staged chunk, packing, and the async D2H into the parent's pinned results
static int chunk_run(ygm_ctx* c, ygm_ctx* k, const HostCall& H, Chunk& C, uint64_t& pos, bool merge_enqueued) {
  const uint32_t nd = C.d1 - C.d0;
  const uint64_t bytes = (is_merge(H.mode) ? H.off[C.u1] - H.off[C.u0] : H.off[C.d1] - H.off[C.d0]);
  ygm_device_result dr;
  int e;
  if (H.mode == 5) e = ygm_merge_v2_device(k, k->arena.as<uint8_t>(), bytes, k->offs.as<uint64_t>(), k->docs.as<uint32_t>(), C.u1 - C.u0, nd,
                                           nullptr, &dr);
  else if (H.mode == 6) e = ygm_diff_v2_device(k, k->arena.as<uint8_t>(), bytes, k->offs.as<uint64_t>(), k->sv_arena.as<uint8_t>(),
                                               k->sv_offs.as<uint64_t>(), nd, nullptr, &dr);
  else if (H.mode == 7) e = ygm_sv_from_update_v2_device(k, k->arena.as<uint8_t>(), bytes, k->offs.as<uint64_t>(), nd, nullptr, &dr);
  else if (H.mode == 8) e = ygm_convert_v1_to_v2_device(k, k->arena.as<uint8_t>(), bytes, k->offs.as<uint64_t>(), nd, nullptr, &dr);
  else if (H.mode == 9) e = ygm_convert_v2_to_v1_device(k, k->arena.as<uint8_t>(), bytes, k->offs.as<uint64_t>(), nd, nullptr, &dr);
  else if (H.mode == 2) e = merge_enqueued ? ygm_merge_v1_device_finish(k, &dr)
                                      : ygm_merge_v1_device(k, k->arena.as<uint8_t>(), bytes, k->offs.as<uint64_t>(), k->docs.as<uint32_t>(),
                                                            C.u1 - C.u0, nd, nullptr, &dr);
  else if (H.mode == 4) e = ygm_contains_v1_device(k, k->arena.as<uint8_t>(), k->offs.as<uint64_t>(), k->sv_arena.as<uint8_t>(),
                                                   k->sv_offs.as<uint64_t>(), nd, nullptr, &dr);
  else if (H.mode == 3) e = ygm_snapshot_v1_device(k, k->arena.as<uint8_t>(), bytes, k->offs.as<uint64_t>(), nd, nullptr, &dr);
  else if (H.mode == 10) e = ygm_sync_step2_v1_device(k, k->arena.as<uint8_t>(), bytes, k->offs.as<uint64_t>(), k->sv_arena.as<uint8_t>(),
                                                      k->sv_offs.as<uint64_t>(), nd, nullptr, &dr);
  else if (H.mode == 1) e = ygm_diff_v1_device(k, k->arena.as<uint8_t>(), bytes, k->offs.as<uint64_t>(), k->sv_arena.as<uint8_t>(),
                                               k->sv_offs.as<uint64_t>(), nd, nullptr, &dr);
  else e = ygm_sv_from_update_v1_device(k, k->arena.as<uint8_t>(), bytes, k->offs.as<uint64_t>(), nd, nullptr, &dr);
  if (e) return e;
  const uint32_t nb = (nd + 255) / 256;
  if (!k->pk_data.ensure(dr.payload_bytes + 64) || !k->pk_off.ensure(8ull * nd + 8) || !k->pk_bsum.ensure(8ull * nb + 16)) return YGM_ENOMEM;
  if (nd && ygm_k_launch_pack(dr.data, dr.off, dr.len, dr.status, nd, k->pk_bsum.as<uint64_t>(), k->pk_data.as<uint8_t>(),
                              k->pk_off.as<uint64_t>(), k->stream))
    return YGM_EDEVICE;
  C.pos = pos; C.payload = dr.payload_bytes;
  if (pos + dr.payload_bytes + 1 > c->h_data.cap) {   // regrowth moves the bytes copied so far: let those copies land first
    for (ygm_ctx* x : c->kid) if (x) HIPCHK(hipStreamSynchronize(x->stream));
    if (!c->h_data.ensure(pos + dr.payload_bytes + 1, pos)) return YGM_ENOMEM;
  }
  HIPCHK(hipEventRecord(C.o0, k->stream));
  if (dr.payload_bytes) HIPCHK(hipMemcpyAsync(c->h_data.as<uint8_t>() + pos, k->pk_data.p, dr.payload_bytes, hipMemcpyDeviceToHost, k->stream));
  if (nd) {
    HIPCHK(hipMemcpyAsync(c->h_off.as<uint64_t>() + C.d0, k->pk_off.p, 8ull * nd, hipMemcpyDeviceToHost, k->stream));
    HIPCHK(hipMemcpyAsync(c->h_len.as<uint64_t>() + C.d0, dr.len, 8ull * nd, hipMemcpyDeviceToHost, k->stream));
    HIPCHK(hipMemcpyAsync(c->h_status.as<int32_t>() + C.d0, dr.status, 4ull * nd, hipMemcpyDeviceToHost, k->stream));
  }
  HIPCHK(hipEventRecord(C.o1, k->stream));
  pos += dr.payload_bytes;
  return YGM_OK;
}

static int host_call(ygm_ctx* c, const HostCall& H, ygm_result* out) {
  (void)hipSetDevice(c->device);
  const uint32_t n = H.n_docs;
  // chunks of whole documents
  std::vector<Chunk> ch;
  {
    const uint64_t CB = chunk_bytes(n ? (is_merge(H.mode) ? H.off[H.n_upd] - H.off[0] : H.off[n] - H.off[0]) : 0);
    uint32_t d = 0, u = 0;
    while (d < n || ch.empty()) {
      Chunk C{};
      C.d0 = d; C.u0 = u;
      const uint64_t base = is_merge(H.mode) ? H.off[u] : H.off[d];
      // the input end of documents [C.d0, x): binary searches over the ascending upd_doc / offsets (a walk over every
      // update took milliseconds per call on batches of millions of updates)
      auto first_upd = [&](uint32_t x) { return (uint32_t)(std::lower_bound(H.upd_doc, H.upd_doc + H.n_upd, x) - H.upd_doc); };
      auto end_of = [&](uint32_t x) { return is_merge(H.mode) ? H.off[first_upd(x)] : H.off[x]; };
      uint32_t lo = d + 1, hi = n;   // the last x in [d + 1, n] whose documents fit in CB (at least one document)
      if (n > d && end_of(n) - base <= CB) lo = n;
      else if (n > d) {
        while (lo < hi) { const uint32_t mid = lo + (hi - lo + 1) / 2; if (end_of(mid) - base <= CB) lo = mid; else hi = mid - 1; }
      }
      if (n > d) { d = lo; u = is_merge(H.mode) ? first_upd(d) : d; }
      C.d1 = d; C.u1 = u;
      ch.push_back(C);
      if (n == 0) break;
    }
  }
  // (outputs are usually no larger than the inputs: sized so, grown when a chunk needs more)
  const uint64_t in_bytes = n ? (is_merge(H.mode) ? H.off[H.n_upd] - H.off[0] : H.off[n] - H.off[0]) : 0;
  if (!c->h_off.ensure(8ull * n + 8) || !c->h_len.ensure(8ull * n + 8) || !c->h_status.ensure(4ull * n + 4) ||
      !c->h_data.ensure(in_bytes + 16ull * n + 4096))
    return YGM_ENOMEM;
  int e = YGM_OK;
  ygm_ctx* k[2];
  if ((e = stage_ctx(c, 0, &k[0])) || (ch.size() > 1 && (e = stage_ctx(c, 1, &k[1])))) return e;
  for (Chunk& C : ch)
    if (hipEventCreate(&C.h0) != hipSuccess || hipEventCreate(&C.h1) != hipSuccess || hipEventCreate(&C.o0) != hipSuccess ||
        hipEventCreate(&C.o1) != hipSuccess) { e = YGM_EDEVICE; break; }
  ygm_stats_t s0[2] = {k[0]->stats, ch.size() > 1 ? k[1]->stats : ygm_stats_t{}};
  uint64_t pos = 0;
  if (!e) e = chunk_stage(k[0], H, ch[0]);
  for (size_t i = 0; i < ch.size() && !e; i++) {
    ygm_ctx* ki = k[i & 1];
    bool enq = false;
    if (H.mode == 2) {   // the lean kernel of chunk i runs while chunk i + 1 is staged
      const uint64_t bytes = H.off[ch[i].u1] - H.off[ch[i].u0];
      if ((e = ygm_merge_v1_device_async(ki, ki->arena.as<uint8_t>(), bytes, ki->offs.as<uint64_t>(), ki->docs.as<uint32_t>(),
                                         ch[i].u1 - ch[i].u0, ch[i].d1 - ch[i].d0, nullptr)))
        break;
      enq = true;
    }
    if (i + 1 < ch.size()) {
      ygm_ctx* kn = k[(i + 1) & 1];
      // the stage's previous chunk (i - 1) has left its pinned staging (its kernels have run)
      if ((e = chunk_stage(kn, H, ch[i + 1]))) break;
    }
    e = chunk_run(c, ki, H, ch[i], pos, enq);
  }
  for (int j = 0; j < (ch.size() > 1 ? 2 : 1); j++) if (hipStreamSynchronize(k[j]->stream) != hipSuccess && !e) e = YGM_EDEVICE;
  if (!e) {
    float ms = 0;
    for (Chunk& C : ch) {
      if (hipEventElapsedTime(&ms, C.h0, C.h1) == hipSuccess) c->stats.h2d_ms += ms;
      if (hipEventElapsedTime(&ms, C.o0, C.o1) == hipSuccess) c->stats.d2h_ms += ms;
      uint64_t* off = c->h_off.as<uint64_t>() + C.d0;
      for (uint32_t d = 0; d < C.d1 - C.d0; d++) off[d] += C.pos;
    }
    for (int j = 0; j < (ch.size() > 1 ? 2 : 1); j++) {   // device work of the stages, into this context's counters
      const ygm_stats_t& a = k[j]->stats; const ygm_stats_t& b = s0[j];
      c->stats.calls += a.calls - b.calls; c->stats.docs += a.docs - b.docs; c->stats.updates += a.updates - b.updates;
      c->stats.bytes_in += a.bytes_in - b.bytes_in; c->stats.bytes_out += a.bytes_out - b.bytes_out;
      c->stats.docs_fast += a.docs_fast - b.docs_fast; c->stats.docs_seq += a.docs_seq - b.docs_seq;
      c->stats.kernel_ms += a.kernel_ms - b.kernel_ms; c->stats.docs_lean += a.docs_lean - b.docs_lean;
      c->stats.lean_ms += a.lean_ms - b.lean_ms; c->stats.lean_launches += a.lean_launches - b.lean_launches;
      c->stats.docs_big += a.docs_big - b.docs_big; c->stats.docs_lean_wide += a.docs_lean_wide - b.docs_lean_wide;
      c->stats.host_syncs += a.host_syncs - b.host_syncs;
      c->stats.docs_pending += a.docs_pending - b.docs_pending;
    }
    int32_t* st = c->h_status.as<int32_t>();
    uint64_t* ln = c->h_len.as<uint64_t>();
    for (uint32_t d = 0; d < n; d++) {
      if (st[d] >= 100 || st[d] < 0) st[d] = YGM_EDEVICE;   // never leaves internal codes
      if (st[d] != YGM_OK) ln[d] = 0;
    }
    out->data = c->h_data.as<uint8_t>(); out->off = c->h_off.as<uint64_t>(); out->len = ln; out->status = st;
    out->n_docs = n; out->data_bytes = pos;
  }
  for (Chunk& C : ch) for (hipEvent_t ev : {C.h0, C.h1, C.o0, C.o1}) if (ev) (void)hipEventDestroy(ev);
  return e;
}

int ygm_merge_v1(ygm_ctx* c, const uint8_t* arena, const uint64_t* upd_off, const uint32_t* upd_doc, uint32_t n_upd, uint32_t n_docs,
                 ygm_result* out) {
  if (!c || !out || (n_upd && (!arena || !upd_off || !upd_doc))) return YGM_EINVAL;
  // document ids non-decreasing, offsets non-decreasing
  std::atomic<int> bad{0};
  par_for(n_upd, [&](size_t a, size_t b) {
    for (size_t i = a; i < b; i++)
      if (upd_doc[i] >= n_docs || (i && upd_doc[i] < upd_doc[i - 1]) || upd_off[i + 1] < upd_off[i]) { bad = 1; return; }
  });
  if (bad) return YGM_EINVAL;
  static const uint64_t zero_off[1] = {0};
  HostCall H{2, arena, n_upd ? upd_off : zero_off, upd_doc, nullptr, nullptr, n_upd, n_docs};
  return host_call(c, H, out);
}

int ygm_merge_v2(ygm_ctx* c, const uint8_t* arena, const uint64_t* upd_off, const uint32_t* upd_doc, uint32_t n_upd, uint32_t n_docs,
                 ygm_result* out) {
  if (!c || !out || (n_upd && (!arena || !upd_off || !upd_doc))) return YGM_EINVAL;
  for (uint32_t i = 0; i < n_upd; i++)
    if (upd_doc[i] >= n_docs || (i && upd_doc[i] < upd_doc[i - 1]) || upd_off[i + 1] < upd_off[i]) return YGM_EINVAL;
  static const uint64_t zero_off[1] = {0};
  HostCall H{5, arena, n_upd ? upd_off : zero_off, upd_doc, nullptr, nullptr, n_upd, n_docs};
  return host_call(c, H, out);
}

static int host_doc_call(ygm_ctx* c, int mode, const uint8_t* arena, const uint64_t* doc_off, const uint8_t* sv_arena,
                         const uint64_t* sv_off, uint32_t n_docs, ygm_result* out) {
  if (!c || !out || (n_docs && (!arena || !doc_off))) return YGM_EINVAL;
  const bool two = mode == 1 || mode == 4 || mode == 6 || mode == 10;
  if (two && n_docs && (!sv_arena || !sv_off)) return YGM_EINVAL;
  for (uint32_t d = 0; d < n_docs; d++) {
    if (doc_off[d + 1] < doc_off[d]) return YGM_EINVAL;
    if (two && sv_off[d + 1] < sv_off[d]) return YGM_EINVAL;
  }
  static const uint64_t zero_off[1] = {0};
  HostCall H{mode, arena, n_docs ? doc_off : zero_off, nullptr, sv_arena, n_docs ? sv_off : zero_off, 0, n_docs};
  return host_call(c, H, out);
}

int ygm_contains_v1(ygm_ctx* c, const uint8_t* states, const uint64_t* state_off, const uint8_t* updates, const uint64_t* update_off,
                    uint32_t n_docs, ygm_result* out) {
  return host_doc_call(c, 4, states, state_off, updates, update_off, n_docs, out);
}

int ygm_snapshot_v1(ygm_ctx* c, const uint8_t* arena, const uint64_t* doc_off, uint32_t n_docs, ygm_result* out) {
  return host_doc_call(c, 3, arena, doc_off, nullptr, nullptr, n_docs, out);
}

int ygm_sync_step2_v1(ygm_ctx* c, const uint8_t* states, const uint64_t* state_off, const uint8_t* sv_arena, const uint64_t* sv_off,
                      uint32_t n_docs, ygm_result* out) {
  return host_doc_call(c, 10, states, state_off, sv_arena, sv_off, n_docs, out);
}

int ygm_diff_v1(ygm_ctx* c, const uint8_t* arena, const uint64_t* doc_off, const uint8_t* sv_arena, const uint64_t* sv_off,
                uint32_t n_docs, ygm_result* out) {
  return host_doc_call(c, 1, arena, doc_off, sv_arena, sv_off, n_docs, out);
}

int ygm_sv_from_update_v1(ygm_ctx* c, const uint8_t* arena, const uint64_t* doc_off, uint32_t n_docs, ygm_result* out) {
  return host_doc_call(c, 0, arena, doc_off, nullptr, nullptr, n_docs, out);
}

int ygm_diff_v2(ygm_ctx* c, const uint8_t* arena, const uint64_t* doc_off, const uint8_t* sv_arena, const uint64_t* sv_off,
                uint32_t n_docs, ygm_result* out) {
  return host_doc_call(c, 6, arena, doc_off, sv_arena, sv_off, n_docs, out);
}
int ygm_sv_from_update_v2(ygm_ctx* c, const uint8_t* arena, const uint64_t* doc_off, uint32_t n_docs, ygm_result* out) {
  return host_doc_call(c, 7, arena, doc_off, nullptr, nullptr, n_docs, out);
}
int ygm_convert_v1_to_v2(ygm_ctx* c, const uint8_t* arena, const uint64_t* doc_off, uint32_t n_docs, ygm_result* out) {
  return host_doc_call(c, 8, arena, doc_off, nullptr, nullptr, n_docs, out);
}
int ygm_convert_v2_to_v1(ygm_ctx* c, const uint8_t* arena, const uint64_t* doc_off, uint32_t n_docs, ygm_result* out) {
  return host_doc_call(c, 9, arena, doc_off, nullptr, nullptr, n_docs, out);
}

}  // extern "C"
