/*
 * synth.c -- seeded synthetic Yjs update-v1 corpora for bench.py and the GPU
 * parity tests (there is no yjs on the GPU box).  Emits update bytes directly
 * (SURVEY.md App. A), following the Y.Text editing model of SURVEY.md §8d:
 *
 *  text_updates: config C2 -- every document gets `n_updates` single-character
 *    inserts at uniform random positions from 1..4 clients (uint32 client ids),
 *    each insert one V1 update whose origin/rightOrigin are the neighbouring
 *    characters' ids (exactly what Y.Text.insert records); `del_pct` percent of
 *    the operations are single-character deletes (delete-set-only updates).
 *  text_updates_gen: config C2 with one PRNG stream per document (global index), so any subset of
 *    a document set (a rank's shard) is generated alone, in parallel.
 *  text_states: config C4 -- the merged state of such a session written as one
 *    update (client blocks descending, clocks ascending; 1-16 clients, log-uniform
 *    1-8 KB) plus a per-document state vector with a uniform clock per client
 *    (10 % empty); documents generated in parallel from per-document streams.
 *
 * xorshift64* PRNG; identical bytes for identical (seed, parameters).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <pthread.h>

typedef struct { uint64_t s; } Rng;
static uint64_t rnext(Rng *r) { uint64_t x = r->s; x ^= x >> 12; x ^= x << 25; x ^= x >> 27; r->s = x; return x * 2685821657736338717ULL; }
static uint64_t rbelow(Rng *r, uint64_t n) { return n ? rnext(r) % n : 0; }

static size_t vu(uint8_t *o, uint64_t v) { size_t n = 0; while (v > 127) { o[n++] = (uint8_t)(0x80 | (v & 127)); v >>= 7; } o[n++] = (uint8_t)v; return n; }

typedef struct { uint32_t client, clock; uint8_t ch; uint8_t deleted; } Ch;
typedef struct { uint32_t client, clock; uint8_t ch; int32_t oi, ri; uint32_t oc, ok, rc, rk; } Rec;  /* one insert */

/* Runs one document's editing session; returns number of chars, fills recs/ops.
 * `vis` tracks the visible characters (no scan when nothing was deleted). */
static int session(Rng *r, int n_ops, int nclients, uint32_t *clients, uint32_t *clocks, Ch *doc, int *ndoc,
                   uint8_t *buf, size_t *blen, uint64_t *upd_off, uint32_t *nupd, int del_pct, int max_run) {
  int len = 0, visible = 0, ndel = 0; size_t b = *blen;
  for (int op = 0; op < n_ops; op++) {
    const int ci = (int)rbelow(r, nclients);
    const uint32_t client = clients[ci];
    if (visible > 0 && (int)rbelow(r, 100) < del_pct) {
      /* delete one visible char: DS-only update */
      int k = (int)rbelow(r, visible), i = 0;
      for (;; i++) if (!doc[i].deleted && k-- == 0) break;
      doc[i].deleted = 1; visible--; ndel++;
      upd_off[(*nupd)++] = b;
      buf[b++] = 0;                       /* no structs */
      buf[b++] = 1;                       /* 1 DS client */
      b += vu(buf + b, doc[i].client); buf[b++] = 1;
      b += vu(buf + b, doc[i].clock); buf[b++] = 1;
      continue;
    }
    /* insert at a uniform visible position; neighbours = adjacent chars in the list */
    int pos = (int)rbelow(r, (uint64_t)visible + 1), at = 0, seen = 0;
    if (ndel == 0) at = pos;
    else for (at = 0; at < len; at++) { if (seen == pos) break; if (!doc[at].deleted) seen++; }
    /* one Item of k ASCII characters (k = 1 unless max_run > 1: pastes / typed words of one transaction) */
    const int k = max_run > 1 ? 1 + (int)rbelow(r, (uint64_t)max_run) : 1;
    char chs[256];
    for (int j = 0; j < k; j++) chs[j] = "abcdefghijklmnopqrstuvwxyz"[rbelow(r, 26)];
    const int has_o = at > 0, has_r = at < len;
    memmove(doc + at + k, doc + at, (size_t)(len - at) * sizeof(Ch));
    for (int j = 0; j < k; j++) { doc[at + j].client = client; doc[at + j].clock = clocks[ci] + (uint32_t)j; doc[at + j].ch = (uint8_t)chs[j]; doc[at + j].deleted = 0; }
    len += k; visible += k;
    upd_off[(*nupd)++] = b;
    buf[b++] = 1; buf[b++] = 1;
    b += vu(buf + b, client); b += vu(buf + b, clocks[ci]);
    buf[b++] = (uint8_t)(4 | (has_o ? 0x80 : 0) | (has_r ? 0x40 : 0));
    if (has_o) { b += vu(buf + b, doc[at - 1].client); b += vu(buf + b, doc[at - 1].clock); }
    if (has_r) { b += vu(buf + b, doc[at + k].client); b += vu(buf + b, doc[at + k].clock); }
    if (!has_o && !has_r) { buf[b++] = 1; buf[b++] = 1; buf[b++] = 't'; }
    buf[b++] = (uint8_t)k; memcpy(buf + b, chs, (size_t)k); b += (size_t)k;
    buf[b++] = 0;                         /* empty delete set */
    clocks[ci] += (uint32_t)k;
  }
  *blen = b; *ndoc = len;
  return len;
}

static void pick_clients(Rng *r, int n, uint32_t *c) {
  for (int i = 0; i < n; i++) {
    for (;;) { c[i] = (uint32_t)rnext(r); int dup = 0; for (int j = 0; j < i; j++) dup |= c[j] == c[i]; if (!dup) break; }
  }
}

/* Config C2.  buf must hold n_docs*n_updates*40 bytes; upd_off n_docs*n_updates+1;
 * doc_upd n_docs+1.  Returns bytes written. */
size_t synth_text_updates(uint64_t seed, uint32_t n_docs, uint32_t n_updates, uint32_t min_clients, uint32_t max_clients,
                          int del_pct, uint8_t *buf, uint64_t *upd_off, uint32_t *doc_upd, int max_run) {
  Rng r = { seed * 0x9E3779B97F4A7C15ULL + 1 };
  if (max_run < 1) max_run = 1;
  if (max_run > 200) max_run = 200;
  Ch *doc = (Ch *)malloc(sizeof(Ch) * ((size_t)n_updates * (size_t)max_run + 1));
  size_t b = 0; uint32_t nupd = 0;
  for (uint32_t d = 0; d < n_docs; d++) {
    doc_upd[d] = nupd;
    uint32_t clients[64], clocks[64] = {0};
    int nc = (int)(min_clients + rbelow(&r, max_clients - min_clients + 1));
    if (nc > 64) nc = 64;
    pick_clients(&r, nc, clients);
    int nd;
    session(&r, (int)n_updates, nc, clients, clocks, doc, &nd, buf, &b, upd_off, &nupd, del_pct, max_run);
  }
  doc_upd[n_docs] = nupd; upd_off[nupd] = b;
  free(doc);
  return b;
}

/* Config C4: one merged state update per document + a state vector.
 * Document d is generated from its own PRNG stream (seed, d), so documents are built in parallel
 * (pthreads) and the bytes do not depend on the thread count.  The op count is log-uniform so that
 * the state is log-uniform in [min_bytes, max_bytes] (about 16 bytes per one-character Item with both origins).
 * Two calls: synth_text_states_gen builds the corpus into a handle and returns its sizes;
 * synth_text_states_take copies it into caller arrays and frees the handle. */
typedef struct { uint8_t *buf, *sv; uint64_t *doff, *soff; size_t nb, ns; } C4Part;
typedef struct { uint64_t seed; uint32_t d0, d1, min_cl, max_cl; double lo, hi; C4Part *p; const uint32_t *idx; } C4Job;

static void c4_doc(uint64_t seed, uint32_t d, uint32_t ops, uint32_t min_cl, uint32_t max_cl, Rng *r,
                   Ch *doc, uint8_t *tmp, uint64_t *toff, uint32_t *uidx, C4Part *P) {
  uint32_t clients[64], clocks[64] = {0};
  int nc = (int)(min_cl + rbelow(r, max_cl - min_cl + 1));
  if (nc > 64) nc = 64;
  pick_clients(r, nc, clients);
  int nd; size_t tl = 0; uint32_t nu = 0;
  session(r, (int)ops, nc, clients, clocks, doc, &nd, tmp, &tl, toff, &nu, 0, 1);
  toff[nu] = tl;
  /* update index of each (client, clock): inserts of a client arrive in clock order */
  uint32_t base[65]; base[0] = 0; for (int i = 0; i < nc; i++) base[i + 1] = base[i] + clocks[i];
  uint32_t fill[64] = {0};
  for (uint32_t u = 0; u < nu; u++) {
    const uint8_t *p = tmp + toff[u]; size_t i = 2; uint64_t cl = 0; int sh = 0;
    do { cl |= (uint64_t)(p[i] & 127) << sh; sh += 7; } while (p[i++] & 128);
    int ci = 0; while (clients[ci] != (uint32_t)cl) ci++;
    uidx[base[ci] + fill[ci]++] = u;
  }
  /* merged state: client blocks in descending client order; a client's inserts in clock order
   * (each insert's struct re-emitted from its update: structs start at 2 + vu(client) + vu(clock)) */
  int ord[64]; for (int i = 0; i < nc; i++) ord[i] = i;
  for (int i = 1; i < nc; i++) { int t = ord[i], j = i; while (j > 0 && clients[ord[j - 1]] < clients[t]) { ord[j] = ord[j - 1]; j--; } ord[j] = t; }
  int nblocks = 0; for (int i = 0; i < nc; i++) nblocks += clocks[i] > 0;
  uint8_t *o = P->buf; size_t b = P->nb;
  P->doff[d] = b;
  b += vu(o + b, (uint64_t)nblocks);
  for (int q = 0; q < nc; q++) {
    const int ci = ord[q];
    if (!clocks[ci]) continue;
    b += vu(o + b, clocks[ci]); b += vu(o + b, clients[ci]); o[b++] = 0;
    for (uint32_t k = 0; k < clocks[ci]; k++) {
      const uint32_t u = uidx[base[ci] + k];
      const uint8_t *p = tmp + toff[u]; size_t i = 2;
      while (p[i++] & 128) {}
      while (p[i++] & 128) {}
      const size_t end = toff[u + 1] - 1; /* drop the update's empty DS byte */
      memcpy(o + b, p + i, end - toff[u] - i); b += end - toff[u] - i;
    }
  }
  o[b++] = 0; /* empty delete set */
  P->nb = b;
  (void)seed;
  /* state vector: each client with probability 0.9, clock uniform in [0, end] */
  int empty = rbelow(r, 10) == 0;
  uint8_t *sp = P->sv + P->ns; size_t sn = 0; int ne = 0;
  uint8_t ent[64 * 20]; size_t el = 0;
  if (!empty) for (int i = 0; i < nc; i++) {
    if (!clocks[i]) continue;
    el += vu(ent + el, clients[i]); el += vu(ent + el, rbelow(r, (uint64_t)clocks[i] + 1)); ne++;
  }
  P->soff[d] = P->ns;
  sn += vu(sp, (uint64_t)ne); memcpy(sp + sn, ent, el); sn += el; P->ns += sn;
}

static void *c4_run(void *arg) {
  C4Job *J = (C4Job *)arg;
  const uint32_t max_ops = (uint32_t)exp(J->hi) + 2;
  Ch *doc = (Ch *)malloc(sizeof(Ch) * (max_ops + 1));
  uint8_t *tmp = (uint8_t *)malloc((size_t)max_ops * 40 + 64);
  uint64_t *toff = (uint64_t *)malloc(sizeof(uint64_t) * (max_ops + 2));
  uint32_t *uidx = (uint32_t *)malloc(sizeof(uint32_t) * (max_ops + 2));
  const size_t n = J->d1 - J->d0;
  C4Part *P = J->p;
  size_t cap = 1 << 20, scap = n * (1 + (size_t)J->max_cl * 16) + 64;
  P->buf = (uint8_t *)malloc(cap); P->sv = (uint8_t *)malloc(scap); P->nb = 0; P->ns = 0;
  for (uint32_t d = J->d0; d < J->d1; d++) {
    const uint32_t gi = J->idx ? J->idx[d] : d;   /* the document's global index: its PRNG stream */
    Rng r = { (J->seed * 0x9E3779B97F4A7C15ULL) ^ ((uint64_t)(gi + 1) * 0xD1B54A32D192ED03ULL) };
    rnext(&r); rnext(&r);
    const double u = (double)(rnext(&r) >> 11) * (1.0 / 9007199254740992.0);
    const uint32_t ops = (uint32_t)exp(J->lo + u * (J->hi - J->lo));
    if (P->nb + (size_t)ops * 40 + 64 > cap) { while (P->nb + (size_t)ops * 40 + 64 > cap) cap *= 2; P->buf = (uint8_t *)realloc(P->buf, cap); }
    c4_doc(J->seed, d - J->d0, ops < 1 ? 1 : ops, J->min_cl, J->max_cl, &r, doc, tmp, toff, uidx, P);
  }
  free(doc); free(tmp); free(toff); free(uidx);
  return NULL;
}

typedef struct { uint32_t n_docs, n_parts; C4Part *parts; uint32_t *pd0; size_t nb, ns; } C4Handle;

void *synth_text_states_gen(uint64_t seed, const uint32_t *idx, uint32_t n_docs, uint32_t min_bytes, uint32_t max_bytes,
                            uint32_t min_clients, uint32_t max_clients, uint32_t threads, uint64_t *out_bytes, uint64_t *out_sv_bytes) {
  if (threads < 1) threads = 1;
  if (threads > n_docs) threads = n_docs ? n_docs : 1;
  C4Handle *H = (C4Handle *)calloc(1, sizeof(C4Handle));
  H->n_docs = n_docs; H->n_parts = threads;
  H->parts = (C4Part *)calloc(threads, sizeof(C4Part));
  H->pd0 = (uint32_t *)calloc(threads + 1, sizeof(uint32_t));
  C4Job *jobs = (C4Job *)calloc(threads, sizeof(C4Job));
  pthread_t *th = (pthread_t *)calloc(threads, sizeof(pthread_t));
  const double lo = log((double)min_bytes / 16.0), hi = log((double)max_bytes / 16.0);
  for (uint32_t t = 0; t < threads; t++) {
    jobs[t].seed = seed; jobs[t].d0 = (uint32_t)((uint64_t)n_docs * t / threads); jobs[t].d1 = (uint32_t)((uint64_t)n_docs * (t + 1) / threads);
    jobs[t].min_cl = min_clients; jobs[t].max_cl = max_clients; jobs[t].lo = lo; jobs[t].hi = hi; jobs[t].p = &H->parts[t]; jobs[t].idx = idx;
    H->pd0[t] = jobs[t].d0;
    const size_t n = jobs[t].d1 - jobs[t].d0;
    H->parts[t].doff = (uint64_t *)malloc(sizeof(uint64_t) * (n + 1)); H->parts[t].soff = (uint64_t *)malloc(sizeof(uint64_t) * (n + 1));
    pthread_create(&th[t], NULL, c4_run, &jobs[t]);
  }
  H->pd0[threads] = n_docs;
  for (uint32_t t = 0; t < threads; t++) { pthread_join(th[t], NULL); H->nb += H->parts[t].nb; H->ns += H->parts[t].ns; }
  free(jobs); free(th);
  *out_bytes = H->nb; *out_sv_bytes = H->ns;
  return H;
}

void synth_text_states_take(void *h, uint8_t *buf, uint64_t *doc_off, uint8_t *sv, uint64_t *sv_off) {
  C4Handle *H = (C4Handle *)h;
  size_t b = 0, s = 0;
  for (uint32_t t = 0; t < H->n_parts; t++) {
    C4Part *P = &H->parts[t];
    memcpy(buf + b, P->buf, P->nb); memcpy(sv + s, P->sv, P->ns);
    for (uint32_t i = 0; i < H->pd0[t + 1] - H->pd0[t]; i++) { doc_off[H->pd0[t] + i] = b + P->doff[i]; sv_off[H->pd0[t] + i] = s + P->soff[i]; }
    b += P->nb; s += P->ns;
    free(P->buf); free(P->sv); free(P->doff); free(P->soff);
  }
  doc_off[H->n_docs] = b; sv_off[H->n_docs] = s;
  free(H->parts); free(H->pd0); free(H);
}

/* ---- configs C3 / C5: [snapshot, ...log] documents of a target size --------------------------
 * The snapshot is one merged update: client blocks in descending client order, each a run of
 * structs with contiguous clocks -- Item ContentString (ASCII and 2-byte UTF-8), ContentDeleted,
 * GC, and with `xml` ContentType (XmlElement "paragraph" / XmlText), ContentFormat and
 * ContentEmbed, and XmlElement attributes (map entries: parent id, parentSub key, ContentAny) -- every
 * other Item after a block's first carrying an origin (and sometimes a right
 * origin) on a random earlier id; then a sorted, merged delete set over the deleted runs.  The
 * log holds k-1 updates: inserts continuing a client's clock (1-3 string structs) and
 * delete-set-only updates over random existing ids.  Sizes follow size(r) = max_bytes * r^-0.8
 * for the document of rank r = d + 1 (floored at min_bytes).
 * buf capacity: sum of the sizes + n_docs * 64 KiB; upd_off: n_docs * 200 + 1; doc_upd: n_docs + 1. */
typedef struct { uint32_t client, clock; } Id;
static size_t w_str(uint8_t *o, const char *s, size_t n) { size_t b = vu(o, n); memcpy(o + b, s, n); return b + n; }
size_t synth_big_docs(uint64_t seed, uint32_t n_docs, uint64_t max_bytes, uint64_t min_bytes, uint32_t max_clients,
                      uint32_t max_k, int xml, uint8_t *buf, uint64_t *upd_off, uint32_t *doc_upd) {
  Rng r = { seed * 0x9E3779B97F4A7C15ULL + 11 };
  size_t b = 0; uint32_t nu = 0;
  uint32_t *clients = (uint32_t *)malloc(sizeof(uint32_t) * max_clients);
  uint32_t *ends = (uint32_t *)malloc(sizeof(uint32_t) * max_clients);
  /* deleted runs of the snapshot, per client in clock order: (client index, clock, len) */
  size_t dcap = 1 << 16, nd = 0;
  uint32_t *dcl = (uint32_t *)malloc(sizeof(uint32_t) * dcap), *dck = (uint32_t *)malloc(sizeof(uint32_t) * dcap), *dln = (uint32_t *)malloc(sizeof(uint32_t) * dcap);
  static const char *words[] = {"lorem", "ipsum", "dolor", "sit", "amet", "caf\xc3\xa9", "na\xc3\xafve", "x"};
  for (uint32_t d = 0; d < n_docs; d++) {
    doc_upd[d] = nu;
    const double sz = (double)max_bytes * pow((double)(d + 1), -0.8);   /* size(r) = max * r^-0.8 */
    uint64_t target = (uint64_t)sz; if (target < min_bytes) target = min_bytes;
    uint32_t nc = 1 + (uint32_t)rbelow(&r, max_clients);
    if (xml && max_clients > 64) nc = max_clients;   /* C5: every snapshot over exactly max_clients client blocks */
    pick_clients(&r, (int)nc, clients);
    /* descending client order */
    for (uint32_t i = 1; i < nc; i++) { uint32_t t = clients[i], j = i; while (j > 0 && clients[j - 1] < t) { clients[j] = clients[j - 1]; j--; } clients[j] = t; }
    /* per-client struct budget */
    uint64_t per = target / nc + 1;
    upd_off[nu++] = b;
    b += vu(buf + b, nc);
    nd = 0;
    for (uint32_t c = 0; c < nc; c++) {
      /* count structs first into a temp region: write block body after a header placeholder */
      const size_t bstart = b; b += 16;         /* header slot: the body is moved up behind the real header */
      const size_t body0 = b;
      uint32_t clock = 0, nst = 0; int last_gc = 0;
      while ((uint64_t)(b - body0) < per || nst == 0) {
        const uint32_t kind = (uint32_t)rbelow(&r, 100);
        if (nst > 0 && kind < 6 && !last_gc) {           /* GC run (never two in a row) */
          const uint32_t ln = 1 + (uint32_t)rbelow(&r, 20);
          buf[b++] = 0; b += vu(buf + b, ln); clock += ln; nst++; last_gc = 1; continue;
        }
        last_gc = 0;
        if (xml && kind >= 47 && kind < 53) {            /* XmlElement attribute: a map entry (parent id + parentSub key), ContentAny */
          buf[b++] = 8 | 0x20; buf[b++] = 0;
          b += vu(buf + b, clients[rbelow(&r, nc)]); b += vu(buf + b, (uint32_t)rbelow(&r, 50));
          if (rbelow(&r, 2)) b += w_str(buf + b, "level", 5); else b += w_str(buf + b, "class", 5);
          b += vu(buf + b, 1);
          if (rbelow(&r, 2)) { buf[b++] = 119; b += w_str(buf + b, "heading", 7); } else { buf[b++] = 125; buf[b++] = (uint8_t)rbelow(&r, 60); }
          clock += 1; nst++; continue;
        }
        uint8_t info; int has_o = nst > 0, has_r = nst > 0 && rbelow(&r, 3) == 0;
        uint32_t ref;
        if (kind < 26) ref = 1;                          /* ContentDeleted */
        else if (xml && kind < 34) ref = 7;              /* ContentType */
        else if (xml && kind < 44) ref = 6;              /* ContentFormat */
        else if (xml && kind < 47) ref = 5;              /* ContentEmbed */
        else ref = 4;                                    /* ContentString */
        info = (uint8_t)(ref | (has_o ? 0x80 : 0) | (has_r ? 0x40 : 0));
        buf[b++] = info;
        if (has_o) { const uint32_t oc = (uint32_t)rbelow(&r, c + 1); b += vu(buf + b, clients[oc]); b += vu(buf + b, oc == c ? clock - 1 : (uint32_t)rbelow(&r, 50)); }
        if (has_r) { const uint32_t oc = (uint32_t)rbelow(&r, nc); b += vu(buf + b, clients[oc]); b += vu(buf + b, (uint32_t)rbelow(&r, 50)); }
        if (!has_o && !has_r) { buf[b++] = 1; b += w_str(buf + b, xml ? "prosemirror" : "t", xml ? 11 : 1); }
        uint32_t len = 1;
        if (ref == 1) { len = 1 + (uint32_t)rbelow(&r, 30); b += vu(buf + b, len);
          if (nd == dcap) { dcap *= 2; dcl = realloc(dcl, 4 * dcap); dck = realloc(dck, 4 * dcap); dln = realloc(dln, 4 * dcap); }
          dcl[nd] = c; dck[nd] = clock; dln[nd] = len; nd++; }
        else if (ref == 7) { const int el = rbelow(&r, 2) == 0; b += vu(buf + b, el ? 3 : 6); if (el) b += w_str(buf + b, "paragraph", 9); }
        else if (ref == 6) { const uint32_t f = (uint32_t)rbelow(&r, 3);
          if (f == 0) { b += w_str(buf + b, "bold", 4); b += w_str(buf + b, "true", 4); }
          else if (f == 1) { b += w_str(buf + b, "italic", 6); b += w_str(buf + b, "1.5", 3); }
          else { b += w_str(buf + b, "link", 4); b += w_str(buf + b, "{\"href\":\"https://x.y/z\"}", 24); } }
        else if (ref == 5) { b += w_str(buf + b, "{\"image\":\"a.png\"}", 17); }
        else { char s[256]; size_t sl = 0; uint32_t units = 0; const uint32_t nw = 1 + (uint32_t)rbelow(&r, 8);
          for (uint32_t w = 0; w < nw; w++) { const char *t = words[rbelow(&r, 8)]; size_t tl = strlen(t);
            memcpy(s + sl, t, tl); sl += tl; s[sl++] = ' ';
            for (size_t q = 0; q < tl; q++) units += (t[q] & 0xC0) != 0x80;   /* UTF-16 units (all BMP) */
            units++; }
          len = units; b += w_str(buf + b, s, sl); }
        clock += len; nst++;
      }
      ends[c] = clock;
      /* header: nst, client, clock 0 -- written in front of the body (shift the body left) */
      uint8_t h[16]; size_t hl = 0; hl += vu(h + hl, nst); hl += vu(h + hl, clients[c]); h[hl++] = 0;
      memmove(buf + bstart + hl, buf + body0, b - body0);
      memcpy(buf + bstart, h, hl);
      b = bstart + hl + (b - body0);
    }
    /* delete set of the snapshot: clients descending (the block order), runs merged */
    { uint32_t ncl = 0; for (size_t i = 0; i < nd; i++) if (i == 0 || dcl[i] != dcl[i - 1]) ncl++;
      b += vu(buf + b, ncl);
      size_t i = 0;
      while (i < nd) { size_t j = i; while (j < nd && dcl[j] == dcl[i]) j++;
        /* runs: merge adjacent */
        uint32_t nr = 0; for (size_t q = i; q < j; q++) if (q == i || dck[q] != dck[q - 1] + dln[q - 1]) nr++;
        b += vu(buf + b, clients[dcl[i]]); b += vu(buf + b, nr);
        size_t q = i; while (q < j) { uint32_t s0 = dck[q], e0 = dck[q] + dln[q]; q++; while (q < j && dck[q] == e0) { e0 += dln[q]; q++; } b += vu(buf + b, s0); b += vu(buf + b, e0 - s0); }
        i = j; } }
    /* the log */
    const uint32_t k = 2 + (uint32_t)rbelow(&r, max_k - 1);
    for (uint32_t u = 1; u < k; u++) {
      upd_off[nu++] = b;
      if (rbelow(&r, 100) < 40) {                         /* deletion: DS only */
        buf[b++] = 0;
        const uint32_t c = (uint32_t)rbelow(&r, nc);
        const uint32_t nr = 1 + (uint32_t)rbelow(&r, 3);
        buf[b++] = 1; b += vu(buf + b, clients[c]); b += vu(buf + b, nr);
        for (uint32_t q = 0; q < nr; q++) { b += vu(buf + b, (uint32_t)rbelow(&r, ends[c] + 1)); b += vu(buf + b, 1 + (uint32_t)rbelow(&r, 4)); }
      } else {                                            /* insert: 1-3 strings continuing a client */
        const uint32_t c = (uint32_t)rbelow(&r, nc), ns = 1 + (uint32_t)rbelow(&r, 3);
        buf[b++] = 1; b += vu(buf + b, ns); b += vu(buf + b, clients[c]); b += vu(buf + b, ends[c]);
        for (uint32_t s = 0; s < ns; s++) {
          buf[b++] = 0x84; b += vu(buf + b, clients[c]); b += vu(buf + b, ends[c] > 0 ? ends[c] - 1 : 0);
          const char ch = (char)('a' + rbelow(&r, 26)); b += w_str(buf + b, &ch, 1); ends[c]++;
        }
        buf[b++] = 0;
      }
    }
  }
  doc_upd[n_docs] = nu; upd_off[nu] = b;
  free(clients); free(ends); free(dcl); free(dck); free(dln);
  return b;
}

/* ---- per-document C2 (documents from their own PRNG streams; a rank generates only its shard) ---- */
typedef struct { uint8_t *buf; uint64_t *uoff; uint32_t *cnt; size_t nb; uint32_t nu; } C2Part;
typedef struct { uint64_t seed; const uint32_t *idx; uint32_t d0, d1, n_updates, min_cl, max_cl; int del_pct; C2Part *p; } C2Job;
static void *c2_run(void *arg) {
  C2Job *J = (C2Job *)arg;
  const uint32_t n = J->d1 - J->d0;
  C2Part *P = J->p;
  P->buf = (uint8_t *)malloc((size_t)n * J->n_updates * 40 + 64);
  P->uoff = (uint64_t *)malloc(sizeof(uint64_t) * ((size_t)n * J->n_updates + 1));
  P->cnt = (uint32_t *)malloc(sizeof(uint32_t) * (n + 1));
  P->nb = 0; P->nu = 0;
  Ch *doc = (Ch *)malloc(sizeof(Ch) * (J->n_updates + 1));
  for (uint32_t d = J->d0; d < J->d1; d++) {
    const uint32_t gi = J->idx ? J->idx[d] : d;
    Rng r = { (J->seed * 0x9E3779B97F4A7C15ULL) ^ ((uint64_t)(gi + 1) * 0xC2B2AE3D27D4EB4FULL) };
    rnext(&r); rnext(&r);
    uint32_t clients[64], clocks[64] = {0};
    int nc = (int)(J->min_cl + rbelow(&r, J->max_cl - J->min_cl + 1));
    if (nc > 64) nc = 64;
    pick_clients(&r, nc, clients);
    const uint32_t u0 = P->nu;
    int nd;
    session(&r, (int)J->n_updates, nc, clients, clocks, doc, &nd, P->buf, &P->nb, P->uoff, &P->nu, J->del_pct, 1);
    P->cnt[d - J->d0] = P->nu - u0;
  }
  free(doc);
  return NULL;
}
typedef struct { uint32_t n, parts; uint32_t *pd0; C2Part *p; size_t nb; uint64_t nu; } C2Handle;
void *synth_text_updates_gen(uint64_t seed, const uint32_t *idx, uint32_t n, uint32_t n_updates, uint32_t min_cl, uint32_t max_cl,
                             int del_pct, uint32_t threads, uint64_t *out_bytes, uint64_t *out_upds) {
  if (threads < 1) threads = 1;
  if (threads > n) threads = n ? n : 1;
  C2Handle *H = (C2Handle *)calloc(1, sizeof(C2Handle));
  H->n = n; H->parts = threads;
  H->p = (C2Part *)calloc(threads, sizeof(C2Part)); H->pd0 = (uint32_t *)calloc(threads + 1, sizeof(uint32_t));
  C2Job *jobs = (C2Job *)calloc(threads, sizeof(C2Job));
  pthread_t *th = (pthread_t *)calloc(threads, sizeof(pthread_t));
  for (uint32_t t = 0; t < threads; t++) {
    C2Job j = { seed, idx, (uint32_t)((uint64_t)n * t / threads), (uint32_t)((uint64_t)n * (t + 1) / threads), n_updates, min_cl, max_cl, del_pct, &H->p[t] };
    jobs[t] = j; H->pd0[t] = j.d0;
    pthread_create(&th[t], NULL, c2_run, &jobs[t]);
  }
  H->pd0[threads] = n;
  for (uint32_t t = 0; t < threads; t++) { pthread_join(th[t], NULL); H->nb += H->p[t].nb; H->nu += H->p[t].nu; }
  free(jobs); free(th);
  *out_bytes = H->nb; *out_upds = H->nu;
  return H;
}
void synth_text_updates_take(void *h, uint8_t *buf, uint64_t *upd_off, uint32_t *doc_upd) {
  C2Handle *H = (C2Handle *)h;
  size_t b = 0; uint64_t u = 0;
  for (uint32_t t = 0; t < H->parts; t++) {
    C2Part *P = &H->p[t];
    memcpy(buf + b, P->buf, P->nb);
    for (uint32_t i = 0; i < P->nu; i++) upd_off[u + i] = b + P->uoff[i];
    uint64_t uu = u;
    for (uint32_t d = H->pd0[t]; d < H->pd0[t + 1]; d++) { doc_upd[d] = (uint32_t)uu; uu += P->cnt[d - H->pd0[t]]; }
    b += P->nb; u += P->nu;
    free(P->buf); free(P->uoff); free(P->cnt);
  }
  upd_off[u] = b; doc_upd[H->n] = (uint32_t)u;
  free(H->p); free(H->pd0); free(H);
}

/* Documents of `n_total` named prefix + decimal index owned by `rank`: fnv1a64(utf8(name)) mod world
 * (the same hash as hocuspocus_amd/shard.py and the Node GpuEnginePool).  Returns the count. */
uint32_t synth_partition(const char *prefix, uint32_t n_total, uint32_t world, uint32_t rank, uint32_t *out) {
  uint32_t k = 0;
  char name[96];
  const size_t pl = strlen(prefix);
  if (pl > 64) return 0;
  memcpy(name, prefix, pl);
  for (uint32_t i = 0; i < n_total; i++) {
    char dig[16]; int nd = 0; uint32_t v = i;
    do { dig[nd++] = (char)('0' + v % 10); v /= 10; } while (v);
    size_t len = pl;
    while (nd) name[len++] = dig[--nd];
    uint64_t h = 0xCBF29CE484222325ULL;
    for (size_t j = 0; j < len; j++) { h ^= (uint8_t)name[j]; h *= 0x100000001B3ULL; }
    if (h % world == rank) out[k++] = i;
  }
  return k;
}
