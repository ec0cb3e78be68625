/*
 * ygm_napi.c -- N-API addon: the thin extern "C" bridge between Node and libygm.so
 * (include/ygm.h).  Every engine handle (one GPU context) owns ONE native worker
 * thread with its own job queue; a batch runs there and its result is handed back to
 * the event loop through a napi_threadsafe_function, so the Hocuspocus event loop
 * never blocks on the GPU and an 8-GPU pool keeps 8 batches in flight (libuv's
 * shared 4-thread pool -- napi_async_work -- would cap it at 4 and compete with
 * fs / dns / crypto).  Results come back as a Promise of
 * { status: Int32Array, outputs: (Uint8Array|null)[] }.
 *
 * JS surface (see ../index.d.ts):
 *   open(device, flags)                                  -> handle
 *   mergeMany(h, arena:Buffer, lens:Uint32Array, docs:Uint32Array, nDocs)  -> Promise
 *   diffMany(h, arena, lens, svArena, svLens)           -> Promise
 *   svMany(h, arena, lens)                              -> Promise
 *   stats(h) -> object ; close(h) ; strerror(code) -> string
 * Input bytes are copied into native memory before the worker runs (JS owns its
 * typed arrays; SURVEY.md §8b "Ownership"); outputs are fresh Buffers.
 */
#include <node_api.h>
#include <pthread.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

#include "../../../include/ygm.h"

#define NAPI_CALL(env, call) do { if ((call) != napi_ok) { napi_throw_error((env), NULL, "N-API call failed: " #call); return NULL; } } while (0)

typedef struct Job Job;
typedef struct {
  ygm_ctx *ctx;
  int busy;
  /* the handle's worker: a FIFO of jobs, run one at a time on `thread` */
  pthread_t thread; int has_thread;
  pthread_mutex_t mu; pthread_cond_t cv;
  Job *head, *tail; int stop;
  napi_threadsafe_function tsfn;   /* worker -> event loop: settles a finished job's promise */
  int refs;                        /* jobs whose completion is pending (the tsfn keeps the loop alive meanwhile) */
  int closing;                     /* close() arrived while a job was in flight: stop once it has settled */
  int owners;                      /* the JS external and the threadsafe function: freed when both are finalized */
} Handle;

struct Job {
  int op; /* 0 merge, 1 diff, 2 sv, ... 99 test sleep */
  Handle *h;
  Job *next;
  uint32_t sleep_ms; double t_start, t_end;   /* op 99 */
  uint8_t *arena; uint64_t *off; uint32_t *docs; uint32_t n_upd, n_docs;
  uint8_t *sv; uint64_t *sv_off;
  int rc;
  /* copied results */
  uint8_t *data; uint64_t *roff, *rlen; int32_t *status; uint32_t rn;
  napi_deferred deferred;
  /* mergeMany: the caller's arena Buffer is read in place by the worker (held by a reference until the
     batch completes), not copied on the main thread */
  napi_ref arena_ref; int arena_borrowed;
  /* the handle's JS external, held until the job settles: a dropped engine cannot be finalized (and its
     Handle freed) while the worker or the threadsafe-function queue still refers to it */
  napi_ref handle_ref;
  double exec_ms;       /* worker: the engine call + copy-out of its context-owned results */
};

static double now_ms(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec * 1e3 + t.tv_nsec / 1e6; }
static void free_data(napi_env env, void *data, void *hint) { (void)env; (void)hint; free(data); }

static void job_execute(Job *j);
static void job_complete(napi_env env, Job *j);

static void *worker_main(void *arg) {
  Handle *h = (Handle *)arg;
  for (;;) {
    pthread_mutex_lock(&h->mu);
    while (!h->head && !h->stop) pthread_cond_wait(&h->cv, &h->mu);
    if (!h->head) { pthread_mutex_unlock(&h->mu); break; }   /* stop, queue drained */
    Job *j = h->head;
    h->head = j->next; if (!h->head) h->tail = NULL;
    pthread_mutex_unlock(&h->mu);
    job_execute(j);
    napi_call_threadsafe_function(h->tsfn, j, napi_tsfn_blocking);
  }
  return NULL;
}

static void handle_stop(Handle *h);

/* runs on the event loop for every finished job (env NULL: the environment is being torn down, the
   promise cannot settle; the job's memory is released with the process) */
static void tsfn_call(napi_env env, napi_value js_cb, void *context, void *data) {
  (void)js_cb;
  Handle *h = (Handle *)context;
  Job *j = (Job *)data;
  if (!env) return;
  job_complete(env, j);
  if (--h->refs == 0) napi_unref_threadsafe_function(env, h->tsfn);
  if (h->closing && !h->busy) handle_stop(h);   /* a close() that waited for this job (last use of h here) */
}

/* joins the worker (after the jobs queued so far), releases the threadsafe function and frees the
   context; the Handle itself is freed by the threadsafe function's finalizer, which runs only after every
   queued completion has been delivered */
static void handle_stop(Handle *h) {
  h->closing = 0;
  const int had = h->has_thread;
  if (had) {
    pthread_mutex_lock(&h->mu); h->stop = 1; pthread_cond_signal(&h->cv); pthread_mutex_unlock(&h->mu);
    pthread_join(h->thread, NULL);
    h->has_thread = 0;
  }
  if (h->ctx) { ygm_close(h->ctx); h->ctx = NULL; }
  if (had) napi_release_threadsafe_function(h->tsfn, napi_tsfn_release);   /* last: may finalize (free) h */
}

static void handle_release(Handle *h) {   /* (both finalizers run on the event loop) */
  if (--h->owners > 0) return;
  pthread_mutex_destroy(&h->mu); pthread_cond_destroy(&h->cv);
  free(h);
}
static void tsfn_finalize(napi_env env, void *data, void *hint) {
  (void)env; (void)hint;
  handle_release((Handle *)data);
}

/* the JS external was collected: no job can be pending (each holds a reference to it) */
static void handle_finalize(napi_env env, void *data, void *hint) {
  (void)env; (void)hint;
  Handle *h = (Handle *)data;
  handle_stop(h);
  handle_release(h);
}

static napi_value noop(napi_env env, napi_callback_info info) { (void)env; (void)info; return NULL; }

/* a handle with its worker; ctx may be NULL (openNull: the threading test's sleep jobs only) */
static napi_value make_handle(napi_env env, ygm_ctx *ctx) {
  Handle *h = (Handle *)calloc(1, sizeof(Handle));
  h->ctx = ctx;
  h->owners = 1;   /* the threadsafe function; the external adds itself below */
  pthread_mutex_init(&h->mu, NULL); pthread_cond_init(&h->cv, NULL);
  napi_value fn, name, ext;
  if (napi_create_function(env, "ygmSettle", NAPI_AUTO_LENGTH, noop, NULL, &fn) != napi_ok ||
      napi_create_string_utf8(env, "ygm.worker", NAPI_AUTO_LENGTH, &name) != napi_ok ||
      napi_create_threadsafe_function(env, fn, NULL, name, 0, 1, h, tsfn_finalize, h, tsfn_call, &h->tsfn) != napi_ok) {
    if (ctx) ygm_close(ctx);
    pthread_mutex_destroy(&h->mu); pthread_cond_destroy(&h->cv);
    free(h); napi_throw_error(env, NULL, "ygm: cannot create the worker's threadsafe function"); return NULL;
  }
  napi_unref_threadsafe_function(env, h->tsfn);   /* an idle engine does not keep Node alive */
  if (pthread_create(&h->thread, NULL, worker_main, h) != 0) {
    if (ctx) { ygm_close(ctx); h->ctx = NULL; }
    napi_release_threadsafe_function(h->tsfn, napi_tsfn_abort);   /* its finalizer frees h */
    napi_throw_error(env, NULL, "ygm: cannot start the engine's worker thread"); return NULL;
  }
  h->has_thread = 1;
  h->owners = 2;
  if (napi_create_external(env, h, handle_finalize, NULL, &ext) != napi_ok) {
    h->owners = 1;
    handle_stop(h);
    napi_throw_error(env, NULL, "ygm: cannot create the engine handle"); return NULL;
  }
  return ext;
}

static Handle *get_handle_any(napi_env env, napi_value v) {
  Handle *h = NULL;
  if (napi_get_value_external(env, v, (void **)&h) != napi_ok || !h || !h->has_thread || h->closing) {
    napi_throw_error(env, NULL, "ygm: closed or invalid engine handle");
    return NULL;
  }
  return h;
}
static Handle *get_handle(napi_env env, napi_value v) {
  Handle *h = NULL;
  if (napi_get_value_external(env, v, (void **)&h) != napi_ok || !h || !h->ctx || !h->has_thread || h->closing) {
    napi_throw_error(env, NULL, "ygm: closed or invalid engine handle");
    return NULL;
  }
  return h;
}

static napi_value js_open(napi_env env, napi_callback_info info) {
  size_t argc = 2; napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  int32_t device = 0; uint32_t flags = 0;
  if (argc > 0) napi_get_value_int32(env, argv[0], &device);
  if (argc > 1) napi_get_value_uint32(env, argv[1], &flags);
  ygm_ctx *ctx = NULL;
  int rc = ygm_open(device, flags, &ctx);
  if (rc != YGM_OK) { napi_throw_error(env, "YGM_EOPEN", ygm_strerror(rc)); return NULL; }
  return make_handle(env, ctx);
}

/* openNull(): a handle with a worker but no GPU context -- accepts only sleep() jobs (threading test) */
static napi_value js_open_null(napi_env env, napi_callback_info info) { (void)info; return make_handle(env, NULL); }

static napi_value js_close(napi_env env, napi_callback_info info) {
  size_t argc = 1; napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  Handle *h = NULL;
  if (napi_get_value_external(env, argv[0], (void **)&h) == napi_ok && h && h->has_thread) {
    if (h->busy) h->closing = 1;   /* stops when the in-flight job has settled (tsfn_call) */
    else handle_stop(h);
  }
  return NULL;
}

static napi_value js_strerror(napi_env env, napi_callback_info info) {
  size_t argc = 1; napi_value argv[1]; int32_t code = 0;
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  napi_get_value_int32(env, argv[0], &code);
  napi_value s;
  NAPI_CALL(env, napi_create_string_utf8(env, ygm_strerror(code), NAPI_AUTO_LENGTH, &s));
  return s;
}

static napi_value js_stats(napi_env env, napi_callback_info info) {
  size_t argc = 1; napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  Handle *h = get_handle(env, argv[0]);
  if (!h) return NULL;
  ygm_stats_t s; ygm_stats(h->ctx, &s);
  napi_value o, v;
  NAPI_CALL(env, napi_create_object(env, &o));
#define SETN(name, val) NAPI_CALL(env, napi_create_double(env, (double)(val), &v)); NAPI_CALL(env, napi_set_named_property(env, o, name, v));
  SETN("calls", s.calls) SETN("docs", s.docs) SETN("updates", s.updates) SETN("bytesIn", s.bytes_in) SETN("bytesOut", s.bytes_out)
  SETN("docsFast", s.docs_fast) SETN("docsSeq", s.docs_seq) SETN("kernelMs", s.kernel_ms) SETN("h2dMs", s.h2d_ms) SETN("d2hMs", s.d2h_ms) SETN("docsLean", s.docs_lean) SETN("leanMs", s.lean_ms) SETN("leanLaunches", s.lean_launches) SETN("docsBig", s.docs_big) SETN("docsLeanWide", s.docs_lean_wide) SETN("hostSyncs", s.host_syncs) SETN("docsPending", s.docs_pending)
#undef SETN
  return o;
}

/* copies a Buffer / TypedArray argument into malloc'd memory */
static int get_bytes(napi_env env, napi_value v, void **out, size_t *len) {
  bool is_ta = false, is_buf = false; void *data = NULL; size_t n = 0;
  napi_is_typedarray(env, v, &is_ta);
  napi_is_buffer(env, v, &is_buf);
  if (is_buf) { if (napi_get_buffer_info(env, v, &data, &n) != napi_ok) return -1; }
  else if (is_ta) {
    napi_typedarray_type t; size_t cnt; napi_value ab; size_t boff;
    if (napi_get_typedarray_info(env, v, &t, &cnt, &data, &ab, &boff) != napi_ok) return -1;
    size_t el = (t == napi_uint32_array || t == napi_int32_array || t == napi_float32_array) ? 4 : (t == napi_float64_array || t == napi_bigint64_array || t == napi_biguint64_array) ? 8 : (t == napi_uint16_array || t == napi_int16_array) ? 2 : 1;
    n = cnt * el;
  } else return -1;
  *out = malloc(n ? n : 1);
  if (!*out) return -1;
  if (n) memcpy(*out, data, n);
  *len = n;
  return 0;
}

static uint64_t *lens_to_off(const uint32_t *lens, uint32_t n) {
  uint64_t *off = (uint64_t *)malloc(sizeof(uint64_t) * (n + 1));
  off[0] = 0;
  for (uint32_t i = 0; i < n; i++) off[i + 1] = off[i] + lens[i];
  return off;
}

static void job_execute(Job *j) {
  const double t0 = now_ms();
  ygm_result r; memset(&r, 0, sizeof r);
  if (j->op == 99) {   /* threading test: occupy the worker */
    j->t_start = t0;
    struct timespec ts = { j->sleep_ms / 1000, (long)(j->sleep_ms % 1000) * 1000000L };
    nanosleep(&ts, NULL);
    j->t_end = now_ms(); j->rc = YGM_OK; return;
  }
  if (j->op == 0) j->rc = ygm_merge_v1(j->h->ctx, j->arena, j->off, j->docs, j->n_upd, j->n_docs, &r);
  else if (j->op == 1) j->rc = ygm_diff_v1(j->h->ctx, j->arena, j->off, j->sv, j->sv_off, j->n_docs, &r);
  else if (j->op == 3) j->rc = ygm_snapshot_v1(j->h->ctx, j->arena, j->off, j->n_docs, &r);
  else if (j->op == 4) j->rc = ygm_contains_v1(j->h->ctx, j->arena, j->off, j->sv, j->sv_off, j->n_docs, &r);
  else if (j->op == 5) j->rc = ygm_sync_step2_v1(j->h->ctx, j->arena, j->off, j->sv, j->sv_off, j->n_docs, &r);
  else if (j->op == 10) j->rc = ygm_merge_v2(j->h->ctx, j->arena, j->off, j->docs, j->n_upd, j->n_docs, &r);
  else if (j->op == 11) j->rc = ygm_diff_v2(j->h->ctx, j->arena, j->off, j->sv, j->sv_off, j->n_docs, &r);
  else if (j->op == 12) j->rc = ygm_sv_from_update_v2(j->h->ctx, j->arena, j->off, j->n_docs, &r);
  else if (j->op == 13) j->rc = ygm_convert_v1_to_v2(j->h->ctx, j->arena, j->off, j->n_docs, &r);
  else if (j->op == 14) j->rc = ygm_convert_v2_to_v1(j->h->ctx, j->arena, j->off, j->n_docs, &r);
  else j->rc = ygm_sv_from_update_v1(j->h->ctx, j->arena, j->off, j->n_docs, &r);
  if (j->rc != YGM_OK) return;
  /* results are context-owned: copy out before the next batch may reuse them */
  j->rn = r.n_docs;
  j->data = (uint8_t *)malloc(r.data_bytes ? r.data_bytes : 1);
  j->roff = (uint64_t *)malloc(sizeof(uint64_t) * (r.n_docs + 1));
  j->rlen = (uint64_t *)malloc(sizeof(uint64_t) * (r.n_docs + 1));
  j->status = (int32_t *)malloc(sizeof(int32_t) * (r.n_docs + 1));
  if (r.data_bytes) memcpy(j->data, r.data, r.data_bytes);
  if (r.n_docs) {
    memcpy(j->roff, r.off, sizeof(uint64_t) * r.n_docs);
    memcpy(j->rlen, r.len, sizeof(uint64_t) * r.n_docs);
    memcpy(j->status, r.status, sizeof(int32_t) * r.n_docs);
  }
  j->exec_ms = now_ms() - t0;
}

static void job_free(Job *j) {
  if (!j->arena_borrowed) free(j->arena);
  free(j->off); free(j->docs); free(j->sv); free(j->sv_off);
  free(j->data); free(j->roff); free(j->rlen); free(j->status);
  free(j);
}

static void job_complete(napi_env env, Job *j) {
  const double t0 = now_ms();
  j->h->busy = 0;
  if (j->arena_ref) { napi_delete_reference(env, j->arena_ref); j->arena_ref = NULL; }
  if (j->handle_ref) { napi_delete_reference(env, j->handle_ref); j->handle_ref = NULL; }
  napi_value result = NULL, err = NULL;
  if (j->op == 99) {
    napi_value a, b;
    napi_create_object(env, &result);
    napi_create_double(env, j->t_start, &a); napi_create_double(env, j->t_end, &b);
    napi_set_named_property(env, result, "start", a); napi_set_named_property(env, result, "end", b);
    napi_resolve_deferred(env, j->deferred, result);
  } else if (j->rc != YGM_OK) {
    napi_value msg, code;
    napi_create_string_utf8(env, ygm_strerror(j->rc), NAPI_AUTO_LENGTH, &msg);
    napi_create_string_utf8(env, "YGM_EBATCH", NAPI_AUTO_LENGTH, &code);
    napi_create_error(env, code, msg, &err);
    napi_reject_deferred(env, j->deferred, err);
  } else {
    napi_value status_ab, status_arr, outs;
    void *sp = NULL;
    napi_create_arraybuffer(env, sizeof(int32_t) * j->rn, &sp, &status_ab);
    if (j->rn) memcpy(sp, j->status, sizeof(int32_t) * j->rn);
    napi_create_typedarray(env, napi_int32_array, j->rn, status_ab, 0, &status_arr);
    napi_create_array_with_length(env, j->rn, &outs);
    /* outputs: Uint8Array views of ONE external ArrayBuffer that owns the packed result bytes (no copy and
       no allocation per document); per-document Buffer copies if external buffers are unavailable */
    napi_value rab = NULL;
    size_t rbytes = 0;
    for (uint32_t d = 0; d < j->rn; d++) if (j->status[d] == YGM_OK && j->roff[d] + j->rlen[d] > rbytes) rbytes = j->roff[d] + j->rlen[d];
    if (rbytes && napi_create_external_arraybuffer(env, j->data, rbytes, free_data, NULL, &rab) == napi_ok) j->data = NULL;
    else rab = NULL;
    for (uint32_t d = 0; d < j->rn; d++) {
      napi_value b;
      if (j->status[d] != YGM_OK) napi_get_null(env, &b);
      else if (rab) napi_create_typedarray(env, napi_uint8_array, j->rlen[d], rab, j->roff[d], &b);
      else napi_create_buffer_copy(env, j->rlen[d], j->data + j->roff[d], NULL, &b);
      napi_set_element(env, outs, d, b);
    }
    napi_value ems, cms;
    napi_create_object(env, &result);
    napi_set_named_property(env, result, "status", status_arr);
    napi_set_named_property(env, result, "outputs", outs);
    napi_create_double(env, j->exec_ms, &ems);
    napi_create_double(env, now_ms() - t0, &cms);
    napi_set_named_property(env, result, "execMs", ems);
    napi_set_named_property(env, result, "completeMs", cms);
    napi_resolve_deferred(env, j->deferred, result);
  }
  job_free(j);
}

/* queues the job on its handle's worker thread */
static napi_value submit(napi_env env, Job *j, napi_value handle) {
  napi_value promise;
  Handle *h = j->h;
  if (h->busy) {
    if (j->arena_ref) napi_delete_reference(env, j->arena_ref);
    job_free(j); napi_throw_error(env, "YGM_EBUSY", "ygm: one batch in flight per engine handle"); return NULL;
  }
  if (napi_create_reference(env, handle, 1, &j->handle_ref) != napi_ok || napi_create_promise(env, &j->deferred, &promise) != napi_ok) {
    if (j->arena_ref) napi_delete_reference(env, j->arena_ref);
    if (j->handle_ref) napi_delete_reference(env, j->handle_ref);
    job_free(j); napi_throw_error(env, NULL, "ygm: cannot queue the batch"); return NULL;
  }
  h->busy = 1;
  if (h->refs++ == 0) napi_ref_threadsafe_function(env, h->tsfn);   /* keep the loop alive until it settles */
  pthread_mutex_lock(&h->mu);
  j->next = NULL;
  if (h->tail) h->tail->next = j; else h->head = j;
  h->tail = j;
  pthread_cond_signal(&h->cv);
  pthread_mutex_unlock(&h->mu);
  return promise;
}

/* sleep(h, ms) -> Promise<{start, end}>: occupies the handle's worker for ms (threading test) */
static napi_value js_sleep(napi_env env, napi_callback_info info) {
  size_t argc = 2; napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  Handle *h = argc > 0 ? get_handle_any(env, argv[0]) : NULL;
  if (!h) return NULL;
  Job *j = (Job *)calloc(1, sizeof(Job)); j->op = 99; j->h = h;
  if (argc > 1) napi_get_value_uint32(env, argv[1], &j->sleep_ms);
  return submit(env, j, argv[0]);
}

/* mergeMany(h, arena, lens, docs, nDocs) */
static napi_value js_merge(napi_env env, napi_callback_info info) {
  size_t argc = 5; napi_value argv[5];
  void *opd = NULL;
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, &opd));
  if (argc < 5) { napi_throw_type_error(env, NULL, "mergeMany(handle, arena, lens, docs, nDocs)"); return NULL; }
  Handle *h = get_handle(env, argv[0]);
  if (!h) return NULL;
  Job *j = (Job *)calloc(1, sizeof(Job)); j->op = opd ? (int)(intptr_t)opd : 0; j->h = h;
  size_t an = 0, ln, dn; void *lens = NULL;
  bool is_buf = false;
  napi_is_buffer(env, argv[1], &is_buf);
  if (is_buf && napi_get_buffer_info(env, argv[1], (void **)&j->arena, &an) == napi_ok &&
      napi_create_reference(env, argv[1], 1, &j->arena_ref) == napi_ok) {
    j->arena_borrowed = 1;   /* read in place by the worker; the reference keeps it alive */
  } else if (get_bytes(env, argv[1], (void **)&j->arena, &an)) {
    job_free(j); napi_throw_type_error(env, NULL, "mergeMany: expected Buffer / Uint32Array arguments"); return NULL;
  }
  if (get_bytes(env, argv[2], &lens, &ln) || get_bytes(env, argv[3], (void **)&j->docs, &dn)) {
    if (j->arena_ref) napi_delete_reference(env, j->arena_ref);
    free(lens); job_free(j); napi_throw_type_error(env, NULL, "mergeMany: expected Buffer / Uint32Array arguments"); return NULL;
  }
  napi_get_value_uint32(env, argv[4], &j->n_docs);
  j->n_upd = (uint32_t)(ln / 4);
  if (dn / 4 != j->n_upd) {
    if (j->arena_ref) napi_delete_reference(env, j->arena_ref);
    free(lens); job_free(j); napi_throw_range_error(env, NULL, "mergeMany: lens/docs length mismatch"); return NULL;
  }
  j->off = lens_to_off((const uint32_t *)lens, j->n_upd);
  free(lens);
  if (j->off[j->n_upd] != an) {
    if (j->arena_ref) napi_delete_reference(env, j->arena_ref);
    job_free(j); napi_throw_range_error(env, NULL, "mergeMany: sum(lens) != arena length"); return NULL;
  }
  return submit(env, j, argv[0]);
}

/* diffMany(h, arena, lens, svArena, svLens) */
static napi_value js_diff(napi_env env, napi_callback_info info) {
  size_t argc = 5; napi_value argv[5];
  void *opd = NULL;
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, &opd));
  if (argc < 5) { napi_throw_type_error(env, NULL, "diffMany(handle, arena, lens, svArena, svLens)"); return NULL; }
  Handle *h = get_handle(env, argv[0]);
  if (!h) return NULL;
  Job *j = (Job *)calloc(1, sizeof(Job)); j->op = opd ? (int)(intptr_t)opd : 1; j->h = h;
  size_t an, ln, sn, sln; void *lens = NULL, *slens = NULL;
  if (get_bytes(env, argv[1], (void **)&j->arena, &an) || get_bytes(env, argv[2], &lens, &ln) || get_bytes(env, argv[3], (void **)&j->sv, &sn) ||
      get_bytes(env, argv[4], &slens, &sln) || ln != sln) {
    free(lens); free(slens); job_free(j); napi_throw_type_error(env, NULL, "diffMany: bad arguments"); return NULL;
  }
  j->n_docs = (uint32_t)(ln / 4);
  j->off = lens_to_off((const uint32_t *)lens, j->n_docs);
  j->sv_off = lens_to_off((const uint32_t *)slens, j->n_docs);
  free(lens); free(slens);
  if (j->off[j->n_docs] != an || j->sv_off[j->n_docs] != sn) { job_free(j); napi_throw_range_error(env, NULL, "diffMany: lengths do not match arenas"); return NULL; }
  return submit(env, j, argv[0]);
}

/* svMany(h, arena, lens) */
static napi_value js_sv(napi_env env, napi_callback_info info) {
  size_t argc = 3; napi_value argv[3];
  void *opd = NULL;
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, &opd));
  if (argc < 3) { napi_throw_type_error(env, NULL, "svMany(handle, arena, lens)"); return NULL; }
  Handle *h = get_handle(env, argv[0]);
  if (!h) return NULL;
  Job *j = (Job *)calloc(1, sizeof(Job)); j->op = opd ? (int)(intptr_t)opd : 2; j->h = h;
  size_t an, ln; void *lens = NULL;
  if (get_bytes(env, argv[1], (void **)&j->arena, &an) || get_bytes(env, argv[2], &lens, &ln)) {
    free(lens); job_free(j); napi_throw_type_error(env, NULL, "svMany: bad arguments"); return NULL;
  }
  j->n_docs = (uint32_t)(ln / 4);
  j->off = lens_to_off((const uint32_t *)lens, j->n_docs);
  free(lens);
  if (j->off[j->n_docs] != an) { job_free(j); napi_throw_range_error(env, NULL, "svMany: sum(lens) != arena length"); return NULL; }
  return submit(env, j, argv[0]);
}

/* containsMany(h, states, stateLens, updates, updateLens): snapshotContainsUpdate per pair (1 byte) */
static napi_value js_contains(napi_env env, napi_callback_info info) {
  size_t argc = 5; napi_value argv[5];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 5) { napi_throw_type_error(env, NULL, "containsMany(handle, states, lens, updates, lens)"); return NULL; }
  Handle *h = get_handle(env, argv[0]);
  if (!h) return NULL;
  Job *j = (Job *)calloc(1, sizeof(Job)); j->op = 4; j->h = h;
  size_t an, ln, sn, sln; void *lens = NULL, *slens = NULL;
  if (get_bytes(env, argv[1], (void **)&j->arena, &an) || get_bytes(env, argv[2], &lens, &ln) || get_bytes(env, argv[3], (void **)&j->sv, &sn) ||
      get_bytes(env, argv[4], &slens, &sln) || ln != sln) {
    free(lens); free(slens); job_free(j); napi_throw_type_error(env, NULL, "containsMany: bad arguments"); return NULL;
  }
  j->n_docs = (uint32_t)(ln / 4);
  j->off = lens_to_off((const uint32_t *)lens, j->n_docs);
  j->sv_off = lens_to_off((const uint32_t *)slens, j->n_docs);
  free(lens); free(slens);
  if (j->off[j->n_docs] != an || j->sv_off[j->n_docs] != sn) { job_free(j); napi_throw_range_error(env, NULL, "containsMany: lengths do not match arenas"); return NULL; }
  return submit(env, j, argv[0]);
}

/* snapshotMany(h, arena, lens): Y.encodeStateAsUpdate(Y.applyUpdate(new Y.Doc(), u)) per update */
static napi_value js_snapshot(napi_env env, napi_callback_info info) {
  size_t argc = 3; napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 3) { napi_throw_type_error(env, NULL, "snapshotMany(handle, arena, lens)"); return NULL; }
  Handle *h = get_handle(env, argv[0]);
  if (!h) return NULL;
  Job *j = (Job *)calloc(1, sizeof(Job)); j->op = 3; j->h = h;
  size_t an, ln; void *lens = NULL;
  if (get_bytes(env, argv[1], (void **)&j->arena, &an) || get_bytes(env, argv[2], &lens, &ln)) {
    free(lens); job_free(j); napi_throw_type_error(env, NULL, "snapshotMany: bad arguments"); return NULL;
  }
  j->n_docs = (uint32_t)(ln / 4);
  j->off = lens_to_off((const uint32_t *)lens, j->n_docs);
  free(lens);
  if (j->off[j->n_docs] != an) { job_free(j); napi_throw_range_error(env, NULL, "snapshotMany: sum(lens) != arena length"); return NULL; }
  return submit(env, j, argv[0]);
}

static napi_value init(napi_env env, napi_value exports) {
  napi_property_descriptor d[] = {
    { "open", NULL, js_open, NULL, NULL, NULL, napi_default, NULL },
    { "openNull", NULL, js_open_null, NULL, NULL, NULL, napi_default, NULL },
    { "sleep", NULL, js_sleep, NULL, NULL, NULL, napi_default, NULL },
    { "close", NULL, js_close, NULL, NULL, NULL, napi_default, NULL },
    { "mergeMany", NULL, js_merge, NULL, NULL, NULL, napi_default, NULL },
    { "diffMany", NULL, js_diff, NULL, NULL, NULL, napi_default, NULL },
    /* SyncStep2 of stored documents: encodeStateAsUpdate(applyUpdate(new Doc, state), sv) (MessageReceiver.ts:137-138) */
    { "step2Many", NULL, js_diff, NULL, NULL, NULL, napi_default, (void *)(intptr_t)5 },
    { "svMany", NULL, js_sv, NULL, NULL, NULL, napi_default, NULL },
    { "snapshotMany", NULL, js_snapshot, NULL, NULL, NULL, napi_default, NULL },
    { "containsMany", NULL, js_contains, NULL, NULL, NULL, napi_default, NULL },
    /* update format V2 (yjs mergeUpdatesV2 / diffUpdateV2 / encodeStateVectorFromUpdateV2 / 13.6 convertUpdateFormat*) */
    { "mergeManyV2", NULL, js_merge, NULL, NULL, NULL, napi_default, (void *)(intptr_t)10 },
    { "diffManyV2", NULL, js_diff, NULL, NULL, NULL, napi_default, (void *)(intptr_t)11 },
    { "svManyV2", NULL, js_sv, NULL, NULL, NULL, napi_default, (void *)(intptr_t)12 },
    { "convertManyV1ToV2", NULL, js_sv, NULL, NULL, NULL, napi_default, (void *)(intptr_t)13 },
    { "convertManyV2ToV1", NULL, js_sv, NULL, NULL, NULL, napi_default, (void *)(intptr_t)14 },
    { "stats", NULL, js_stats, NULL, NULL, NULL, napi_default, NULL },
    { "strerror", NULL, js_strerror, NULL, NULL, NULL, napi_default, NULL },
  };
  napi_define_properties(env, exports, sizeof d / sizeof d[0], d);
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
