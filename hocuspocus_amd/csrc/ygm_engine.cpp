// ygm_engine.cpp -- host runtime behind include/ygm.h.
//
// One context per GPU: a HIP stream, grow-only device workspaces, host result
// buffers and HIP-event timers.  A batch call = H2D of the packed inputs, one
// fast-path launch (look-back placed, packed output), an 8-byte-class meta
// read, the sequential kernel only when some document needed it, D2H.
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/ygm.h"

extern "C" {
size_t ygm_k_meta_bytes();
size_t ygm_k_seq_reader_bytes();
size_t ygm_k_drec_bytes();
int ygm_k_launch_doc(int mode, const uint8_t* arena, const uint64_t* doc_off, const uint8_t* sv_arena, const uint64_t* sv_off,
                     const uint32_t* docs, uint64_t out_base, uint32_t n_docs, uint32_t flags, uint8_t* out, uint64_t* out_off,
                     uint64_t* out_len, int32_t* status, unsigned long long* lb, void* meta, uint64_t out_cap, hipStream_t s);
size_t ygm_k_sv_table_bytes(uint32_t n_docs);
int ygm_k_launch_doc_lean(int mode, const uint8_t* arena, uint64_t arena_bytes, const uint64_t* doc_off, const uint8_t* sv_arena,
                          uint64_t sv_bytes, const uint64_t* sv_off, uint32_t n_docs, uint32_t flags, uint8_t* out, uint64_t* out_off,
                          uint64_t* out_len, int32_t* status, void* meta, uint32_t* defer_list, uint64_t out_cap, uint8_t* tbl,
                          uint32_t* tbl_n, hipStream_t s);
int ygm_k_launch_merge_lean(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, uint32_t n_docs, uint32_t flags,
                            uint8_t* out, uint64_t* out_off, uint64_t* out_len, int32_t* status, void* meta, void* meta_next,
                            uint32_t* defer_list, uint64_t out_cap, hipStream_t s);
int ygm_k_launch_merge_wave(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, const uint32_t* docs,
                            const unsigned int* n_dev, uint32_t n_docs, uint32_t flags, uint8_t* out, uint64_t* out_off, uint64_t* out_len,
                            int32_t* status, void* meta, uint32_t* defer_list, uint32_t* fb_list, uint64_t out_cap, hipStream_t s);
int ygm_k_launch_merge_fast(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, const uint32_t* docs,
                            const unsigned int* n_dev, uint32_t n_docs, uint32_t flags, uint8_t* out, uint64_t* out_off, uint64_t* out_len,
                            int32_t* status, uint64_t slot_total, void* meta, uint32_t* fb_list, uint64_t out_cap, hipStream_t s);
int ygm_k_launch_merge_seq(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, const uint32_t* fb_list, uint32_t n_fb,
                           uint32_t flags, uint8_t* out, uint64_t* out_off, uint64_t* out_len, int32_t* status, void* meta,
                           void* readers, int* order, int* tmp, const uint8_t** ubase, uint32_t* ulen, uint64_t upd_cap,
                           uint32_t* cnt, void* drec, uint64_t byte_cap, uint64_t slot_total, uint64_t out_cap, hipStream_t s);
size_t ygm_k_big_blk_bytes();
size_t ygm_k_big_rec_bytes();
int ygm_k_launch_merge_big(const uint8_t* arena, const uint64_t* upd_off, const uint32_t* doc_upd, const uint32_t* fb_list,
                           uint32_t n_fb, uint32_t flags, uint8_t* out, uint64_t* out_off, uint64_t* out_len, int32_t* status,
                           void* meta, uint32_t* fb2_list, void* blk, uint64_t blk_cap, void* rec, uint64_t rec_cap,
                           uint64_t slot_total, uint64_t out_cap, hipStream_t s);
}

namespace {

// mirrors ygm::DocMeta (ygm_kernels.hip); sizeof is a multiple of 16
struct Meta {
  unsigned int ticket, fault, fb_count, defer_count, lean_defer, big_defer;
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
  bool ensure(size_t n) {
    if (n <= cap && p) return true;
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

}  // namespace

struct ygm_ctx {
  int device = 0;
  uint32_t flags = 0;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr, e2 = nullptr, e3 = nullptr;
  // device inputs (host API staging)
  DevBuf arena, offs, docs, sv_arena, sv_offs;
  // device outputs + state
  DevBuf out, out_off, out_len, status, lb, meta, fb_list, defer_list, defer2_list;
  Meta* h_meta = nullptr;  // pinned read-back of the per-launch counters
  int mslot = 0;           // counter slot of the next merge launch
  void* meta_slot(int i) const { return (uint8_t*)meta.p + (size_t)i * sizeof(Meta); }
  DevBuf s_readers, s_order, s_tmp, s_ubase, s_ulen, s_cnt, s_drec;
  DevBuf big_blk, big_rec, big_list;   // large-document tier: block tables, struct records, documents sent on
  DevBuf sv_tbl, sv_tn;                // diff: sorted state-vector tables (k_sv_table) and their entry counts
  // host results
  std::vector<uint8_t> h_data;
  std::vector<uint64_t> h_off, h_len;
  std::vector<int32_t> h_status;
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
  } pend;
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
  }
  return "unknown error";
}

int ygm_open(int device, uint32_t flags, ygm_ctx** out) {
  if (!out) return YGM_EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return YGM_EDEVICE;
  ygm_ctx* c = new ygm_ctx();
  c->device = device; c->flags = flags;
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
  for (DevBuf* b : {&c->arena, &c->offs, &c->docs, &c->sv_arena, &c->sv_offs, &c->out, &c->out_off, &c->out_len, &c->status,
                    &c->lb, &c->meta, &c->fb_list, &c->defer_list, &c->defer2_list, &c->s_readers, &c->s_order, &c->s_tmp, &c->s_ubase, &c->s_ulen, &c->s_cnt,
                    &c->s_drec, &c->big_blk, &c->big_rec, &c->big_list, &c->sv_tbl, &c->sv_tn})
    b->release();
  for (hipEvent_t e : {c->e0, c->e1, c->e2, c->e3}) if (e) (void)hipEventDestroy(e);
  if (c->h_meta) (void)hipHostFree(c->h_meta);
  if (c->stream) (void)hipStreamDestroy(c->stream);
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
      !c->defer_list.ensure((size_t)n_docs * 4 + 4) || !c->defer2_list.ensure((size_t)n_docs * 4 + 4))
    return YGM_ENOMEM;
  if (lookback) {   // SV / diff: look-back tiles and counter slot 2 reset per call
    HIPCHK(hipMemsetAsync(c->lb.p, 0, tiles * 8, s));
    HIPCHK(hipMemsetAsync(c->meta_slot(2), 0, sizeof(Meta), s));
  }
  return YGM_OK;
}

static int read_meta(ygm_ctx* c, hipStream_t s, Meta& m, const void* slot) {
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
int ygm_merge_v1_device_async(ygm_ctx* c, const uint8_t* d_arena, uint64_t arena_bytes, const uint64_t* d_upd_off,
                              const uint32_t* d_doc_upd, uint32_t n_upd, uint32_t n_docs, void* stream) {
  if (!c) return YGM_EINVAL;
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  (void)hipSetDevice(c->device);
  // output arena: one slot per document (2|in| + 64 B, no cross-document dependency),
  // then the overflow region for outputs that outgrow their slot (<= 3|in| + 16/doc)
  const uint64_t slot_total = 2 * arena_bytes + 64ull * n_docs;
  const uint64_t out_cap = slot_total + 3 * arena_bytes + 16ull * n_docs + 64;
  int e = prep_outputs(c, n_docs, out_cap, s, false);
  if (e) return e;
  // tier 1: lean wave-per-document kernel (debounce-log shape); everything else is deferred.
  // Timing: one event before the first launch since the last finish, one in finish after the
  // last -- per-launch event pairs between back-to-back launches cost ~8 us of stream time each.
  if (c->lean_span_n == 0) HIPCHK(hipEventRecord(c->e0, s));
  c->lean_span_n++;
  void* meta = c->meta_slot(c->mslot);
  void* meta_next = c->meta_slot(1 - c->mslot);   // zeroed by this launch for the next one
  if (ygm_k_launch_merge_lean(d_arena, d_upd_off, d_doc_upd, n_docs, c->flags, c->out.as<uint8_t>(), c->out_off.as<uint64_t>(),
                              c->out_len.as<uint64_t>(), c->status.as<int32_t>(), meta, meta_next, c->defer_list.as<uint32_t>(), out_cap, s))
    return YGM_EDEVICE;
  if (n_docs) c->mslot = 1 - c->mslot;   // (an empty batch launches nothing: the slot stays current)
  c->pend.live = true; c->pend.s = s;
  c->pend.arena = d_arena; c->pend.upd_off = d_upd_off; c->pend.doc_upd = d_doc_upd;
  c->pend.arena_bytes = arena_bytes; c->pend.slot_total = slot_total; c->pend.out_cap = out_cap;
  c->pend.n_upd = n_upd; c->pend.n_docs = n_docs; c->pend.meta = meta;
  return YGM_OK;
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
  if (m.lean_defer) {  // tier 2: general wave-per-document kernel over the lean kernel's deferred list
    HIPCHK(hipEventRecord(c->e0, s));
    if (ygm_k_launch_merge_wave(P.arena, P.upd_off, P.doc_upd, c->defer_list.as<uint32_t>(), nullptr, m.lean_defer, c->flags,
                                c->out.as<uint8_t>(), c->out_off.as<uint64_t>(), c->out_len.as<uint64_t>(), c->status.as<int32_t>(),
                                P.meta, c->defer2_list.as<uint32_t>(), c->fb_list.as<uint32_t>(), P.out_cap, s))
      return YGM_EDEVICE;
    HIPCHK(hipEventRecord(c->e1, s));
    if ((e = read_meta(c, s, m, P.meta))) return e;
    if (m.fault) return YGM_EDEVICE;
    if (hipEventElapsedTime(&ms0, c->e0, c->e1) == hipSuccess) c->stats.kernel_ms += ms0;
  }
  if (m.defer_count) {  // tier 3: documents over the wave class, one workgroup per document
    HIPCHK(hipEventRecord(c->e0, s));
    if (ygm_k_launch_merge_fast(P.arena, P.upd_off, P.doc_upd, c->defer2_list.as<uint32_t>(), nullptr, m.defer_count, c->flags,
                                c->out.as<uint8_t>(), c->out_off.as<uint64_t>(), c->out_len.as<uint64_t>(), c->status.as<int32_t>(),
                                P.slot_total, P.meta, c->fb_list.as<uint32_t>(), P.out_cap, s))
      return YGM_EDEVICE;
    HIPCHK(hipEventRecord(c->e1, s));
    if ((e = read_meta(c, s, m, P.meta))) return e;
    if (m.fault) return YGM_EDEVICE;
    if (hipEventElapsedTime(&ms0, c->e0, c->e1) == hipSuccess) c->stats.kernel_ms += ms0;
  }
  uint32_t n_seq = 0;
  if (m.fb_count) {  // tier 4: large [snapshot, ...log] documents, one wave each; the rest go on to tier 5
    const uint64_t blk_cap = m.fb_bytes / 4 + 2ull * m.fb_count + 16, rec_cap = m.fb_bytes / 2 + 2ull * m.fb_count + 16;
    if (!c->big_blk.ensure(blk_cap * ygm_k_big_blk_bytes()) || !c->big_rec.ensure(rec_cap * ygm_k_big_rec_bytes()) ||
        !c->big_list.ensure((size_t)m.fb_count * 4 + 4))
      return YGM_ENOMEM;
    HIPCHK(hipEventRecord(c->e0, s));
    if (ygm_k_launch_merge_big(P.arena, P.upd_off, P.doc_upd, c->fb_list.as<uint32_t>(), m.fb_count, c->flags, c->out.as<uint8_t>(),
                               c->out_off.as<uint64_t>(), c->out_len.as<uint64_t>(), c->status.as<int32_t>(), P.meta,
                               c->big_list.as<uint32_t>(), c->big_blk.p, blk_cap, c->big_rec.p, rec_cap, P.slot_total, P.out_cap, s))
      return YGM_EDEVICE;
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
  c->stats.docs_fast += m.lean_defer - m.fb_count;   // finished by the wave / workgroup tiers (tier 4 counted above)
  c->stats.docs_lean += P.n_docs - m.lean_defer;
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

static int run_doc_kernel(ygm_ctx* c, int mode, const uint8_t* d_arena, uint64_t arena_bytes, const uint64_t* d_doc_off,
                          const uint8_t* d_sv, uint64_t sv_bytes, const uint64_t* d_sv_off, uint32_t n_docs, void* stream,
                          ygm_device_result* out) {
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
  if (ygm_k_launch_doc_lean(mode, d_arena, arena_bytes, d_doc_off, d_sv, sv_bytes, d_sv_off, n_docs, c->flags, c->out.as<uint8_t>(),
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
    if (ygm_k_launch_doc(mode, d_arena, d_doc_off, d_sv, d_sv_off, c->defer_list.as<uint32_t>(), slot_total, m.lean_defer, c->flags,
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

// ------------------------------------------------------------------ host API
static int h2d(ygm_ctx* c, DevBuf& b, const void* src, size_t n, size_t pad) {
  if (!b.ensure(n + pad)) return YGM_ENOMEM;
  if (n) HIPCHK(hipMemcpyAsync(b.p, src, n, hipMemcpyHostToDevice, c->stream));
  if (pad) HIPCHK(hipMemsetAsync((uint8_t*)b.p + n, 0, pad, c->stream));
  return YGM_OK;
}

static int fetch_results(ygm_ctx* c, uint32_t n_docs, const ygm_device_result& dr, ygm_result* out) {
  c->h_off.resize(n_docs); c->h_len.resize(n_docs); c->h_status.resize(n_docs);
  c->h_data.resize(dr.data_bytes ? dr.data_bytes : 1);
  HIPCHK(hipEventRecord(c->e2, c->stream));
  if (n_docs) {
    HIPCHK(hipMemcpyAsync(c->h_off.data(), dr.off, n_docs * 8ull, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(c->h_len.data(), dr.len, n_docs * 8ull, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(c->h_status.data(), dr.status, n_docs * 4ull, hipMemcpyDeviceToHost, c->stream));
  }
  if (dr.data_bytes) HIPCHK(hipMemcpyAsync(c->h_data.data(), dr.data, dr.data_bytes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipEventRecord(c->e3, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  float ms = 0;
  if (hipEventElapsedTime(&ms, c->e2, c->e3) == hipSuccess) c->stats.d2h_ms += ms;
  for (uint32_t d = 0; d < n_docs; d++)
    if (c->h_status[d] >= 100 || c->h_status[d] < 0) c->h_status[d] = YGM_EDEVICE;  // never left internal codes
  out->data = c->h_data.data(); out->off = c->h_off.data(); out->len = c->h_len.data(); out->status = c->h_status.data();
  out->n_docs = n_docs; out->data_bytes = dr.data_bytes;
  return YGM_OK;
}

int ygm_merge_v1(ygm_ctx* c, const uint8_t* arena, const uint64_t* upd_off, const uint32_t* upd_doc, uint32_t n_upd, uint32_t n_docs,
                 ygm_result* out) {
  if (!c || !out || (n_upd && (!arena || !upd_off || !upd_doc))) return YGM_EINVAL;
  (void)hipSetDevice(c->device);
  // per-document update ranges; document ids must be non-decreasing
  c->h_doc_upd.assign((size_t)n_docs + 1, 0);
  for (uint32_t i = 0; i < n_upd; i++) {
    if (upd_doc[i] >= n_docs || (i && upd_doc[i] < upd_doc[i - 1])) return YGM_EINVAL;
    if (upd_off[i + 1] < upd_off[i]) return YGM_EINVAL;
    c->h_doc_upd[upd_doc[i] + 1]++;
  }
  for (uint32_t d = 0; d < n_docs; d++) c->h_doc_upd[d + 1] += c->h_doc_upd[d];
  const uint64_t bytes = n_upd ? upd_off[n_upd] - upd_off[0] : 0;
  // offsets are rebased to the first update
  std::vector<uint64_t> rel(n_upd + 1);
  for (uint32_t i = 0; i <= n_upd; i++) rel[i] = n_upd ? upd_off[i] - upd_off[0] : 0;
  HIPCHK(hipEventRecord(c->e2, c->stream));
  int e;
  if ((e = h2d(c, c->arena, n_upd ? arena + upd_off[0] : nullptr, bytes, 64))) return e;
  if ((e = h2d(c, c->offs, rel.data(), rel.size() * 8, 0))) return e;
  if ((e = h2d(c, c->docs, c->h_doc_upd.data(), c->h_doc_upd.size() * 4, 0))) return e;
  HIPCHK(hipEventRecord(c->e3, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  float ms = 0;
  if (hipEventElapsedTime(&ms, c->e2, c->e3) == hipSuccess) c->stats.h2d_ms += ms;
  ygm_device_result dr;
  if ((e = ygm_merge_v1_device(c, c->arena.as<uint8_t>(), bytes, c->offs.as<uint64_t>(), c->docs.as<uint32_t>(), n_upd, n_docs,
                               nullptr, &dr)))
    return e;
  return fetch_results(c, n_docs, dr, out);
}

static int host_doc_call(ygm_ctx* c, int mode, const uint8_t* arena, const uint64_t* doc_off, const uint8_t* sv_arena,
                         const uint64_t* sv_off, uint32_t n_docs, ygm_result* out) {
  if (!c || !out || (n_docs && (!arena || !doc_off))) return YGM_EINVAL;
  if (mode == 1 && n_docs && (!sv_arena || !sv_off)) return YGM_EINVAL;
  (void)hipSetDevice(c->device);
  for (uint32_t d = 0; d < n_docs; d++) {
    if (doc_off[d + 1] < doc_off[d]) return YGM_EINVAL;
    if (mode == 1 && sv_off[d + 1] < sv_off[d]) return YGM_EINVAL;
  }
  const uint64_t bytes = n_docs ? doc_off[n_docs] - doc_off[0] : 0;
  std::vector<uint64_t> rel(n_docs + 1), srel;
  for (uint32_t d = 0; d <= n_docs; d++) rel[d] = n_docs ? doc_off[d] - doc_off[0] : 0;
  HIPCHK(hipEventRecord(c->e2, c->stream));
  int e;
  if ((e = h2d(c, c->arena, n_docs ? arena + doc_off[0] : nullptr, bytes, 64))) return e;
  if ((e = h2d(c, c->offs, rel.data(), rel.size() * 8, 0))) return e;
  uint64_t sv_bytes = 0;
  if (mode == 1) {
    sv_bytes = n_docs ? sv_off[n_docs] - sv_off[0] : 0;
    srel.resize(n_docs + 1);
    for (uint32_t d = 0; d <= n_docs; d++) srel[d] = n_docs ? sv_off[d] - sv_off[0] : 0;
    if ((e = h2d(c, c->sv_arena, n_docs ? sv_arena + sv_off[0] : nullptr, sv_bytes, 64))) return e;
    if ((e = h2d(c, c->sv_offs, srel.data(), srel.size() * 8, 0))) return e;
  }
  HIPCHK(hipEventRecord(c->e3, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  float ms = 0;
  if (hipEventElapsedTime(&ms, c->e2, c->e3) == hipSuccess) c->stats.h2d_ms += ms;
  ygm_device_result dr;
  if (mode == 1)
    e = ygm_diff_v1_device(c, c->arena.as<uint8_t>(), bytes, c->offs.as<uint64_t>(), c->sv_arena.as<uint8_t>(), c->sv_offs.as<uint64_t>(),
                           n_docs, nullptr, &dr);
  else
    e = ygm_sv_from_update_v1_device(c, c->arena.as<uint8_t>(), bytes, c->offs.as<uint64_t>(), n_docs, nullptr, &dr);
  if (e) return e;
  return fetch_results(c, n_docs, dr, out);
}

int ygm_diff_v1(ygm_ctx* c, const uint8_t* arena, const uint64_t* doc_off, const uint8_t* sv_arena, const uint64_t* sv_off,
                uint32_t n_docs, ygm_result* out) {
  return host_doc_call(c, 1, arena, doc_off, sv_arena, sv_off, n_docs, out);
}

int ygm_sv_from_update_v1(ygm_ctx* c, const uint8_t* arena, const uint64_t* doc_off, uint32_t n_docs, ygm_result* out) {
  return host_doc_call(c, 0, arena, doc_off, nullptr, nullptr, n_docs, out);
}

}  // extern "C"
