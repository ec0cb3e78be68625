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
 *  text_states: config C4 -- the merged state of such a session written as one
 *    update (client blocks descending, clocks ascending) plus a per-document
 *    state vector with a uniform clock per client (10 % empty).
 *
 * xorshift64* PRNG; identical bytes for identical (seed, parameters).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { uint64_t s; } Rng;
static uint64_t rnext(Rng *r) { uint64_t x = r->s; x ^= x >> 12; x ^= x << 25; x ^= x >> 27; r->s = x; return x * 2685821657736338717ULL; }
static uint64_t rbelow(Rng *r, uint64_t n) { return n ? rnext(r) % n : 0; }

static size_t vu(uint8_t *o, uint64_t v) { size_t n = 0; while (v > 127) { o[n++] = (uint8_t)(0x80 | (v & 127)); v >>= 7; } o[n++] = (uint8_t)v; return n; }

typedef struct { uint32_t client, clock; uint8_t ch; uint8_t deleted; } Ch;
typedef struct { uint32_t client, clock; uint8_t ch; int32_t oi, ri; uint32_t oc, ok, rc, rk; } Rec;  /* one insert */

/* Runs one document's editing session; returns number of chars, fills recs/ops. */
static int session(Rng *r, int n_ops, int nclients, uint32_t *clients, uint32_t *clocks, Ch *doc, int *ndoc,
                   uint8_t *buf, size_t *blen, uint64_t *upd_off, uint32_t *nupd, int del_pct) {
  int len = 0; size_t b = *blen;
  for (int op = 0; op < n_ops; op++) {
    const int ci = (int)rbelow(r, nclients);
    const uint32_t client = clients[ci];
    int visible = 0; for (int i = 0; i < len; i++) visible += !doc[i].deleted;
    if (visible > 0 && (int)rbelow(r, 100) < del_pct) {
      /* delete one visible char: DS-only update */
      int k = (int)rbelow(r, visible), i = 0;
      for (;; i++) if (!doc[i].deleted && k-- == 0) break;
      doc[i].deleted = 1;
      upd_off[(*nupd)++] = b;
      buf[b++] = 0;                       /* no structs */
      buf[b++] = 1;                       /* 1 DS client */
      b += vu(buf + b, doc[i].client); buf[b++] = 1;
      b += vu(buf + b, doc[i].clock); buf[b++] = 1;
      continue;
    }
    /* insert at a uniform visible position; neighbours = adjacent chars in the list */
    int pos = (int)rbelow(r, (uint64_t)visible + 1), at = 0, seen = 0;
    for (at = 0; at < len; at++) { if (seen == pos) break; if (!doc[at].deleted) seen++; }
    const char ch = "abcdefghijklmnopqrstuvwxyz"[rbelow(r, 26)];
    const int has_o = at > 0, has_r = at < len;
    memmove(doc + at + 1, doc + at, (size_t)(len - at) * sizeof(Ch));
    doc[at].client = client; doc[at].clock = clocks[ci]; doc[at].ch = (uint8_t)ch; doc[at].deleted = 0;
    len++;
    upd_off[(*nupd)++] = b;
    buf[b++] = 1; buf[b++] = 1;
    b += vu(buf + b, client); b += vu(buf + b, clocks[ci]);
    buf[b++] = (uint8_t)(4 | (has_o ? 0x80 : 0) | (has_r ? 0x40 : 0));
    if (has_o) { b += vu(buf + b, doc[at - 1].client); b += vu(buf + b, doc[at - 1].clock); }
    if (has_r) { b += vu(buf + b, doc[at + 1].client); b += vu(buf + b, doc[at + 1].clock); }
    if (!has_o && !has_r) { buf[b++] = 1; buf[b++] = 1; buf[b++] = 't'; }
    buf[b++] = 1; buf[b++] = (uint8_t)ch;
    buf[b++] = 0;                         /* empty delete set */
    clocks[ci]++;
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
                          int del_pct, uint8_t *buf, uint64_t *upd_off, uint32_t *doc_upd) {
  Rng r = { seed * 0x9E3779B97F4A7C15ULL + 1 };
  Ch *doc = (Ch *)malloc(sizeof(Ch) * (n_updates + 1));
  size_t b = 0; uint32_t nupd = 0;
  for (uint32_t d = 0; d < n_docs; d++) {
    doc_upd[d] = nupd;
    uint32_t clients[64], clocks[64] = {0};
    int nc = (int)(min_clients + rbelow(&r, max_clients - min_clients + 1));
    if (nc > 64) nc = 64;
    pick_clients(&r, nc, clients);
    int nd;
    session(&r, (int)n_updates, nc, clients, clocks, doc, &nd, buf, &b, upd_off, &nupd, del_pct);
  }
  doc_upd[n_docs] = nupd; upd_off[nupd] = b;
  free(doc);
  return b;
}

/* Config C4: one merged state update per document + a state vector.
 * ops per doc uniform in [min_ops, max_ops].  buf: n_docs*max_ops*40; sv: n_docs*(1+max_clients*16). */
size_t synth_text_states(uint64_t seed, uint32_t n_docs, uint32_t min_ops, uint32_t max_ops, uint32_t min_clients, uint32_t max_clients,
                         uint8_t *buf, uint64_t *doc_off, uint8_t *sv, uint64_t *sv_off, size_t *sv_bytes) {
  Rng r = { seed * 0x9E3779B97F4A7C15ULL + 7 };
  Ch *doc = (Ch *)malloc(sizeof(Ch) * (max_ops + 1));
  uint8_t *tmp = (uint8_t *)malloc((size_t)max_ops * 40 + 64);
  uint64_t *toff = (uint64_t *)malloc(sizeof(uint64_t) * (max_ops + 2));
  size_t b = 0, s = 0;
  for (uint32_t d = 0; d < n_docs; d++) {
    doc_off[d] = b; sv_off[d] = s;
    uint32_t clients[64], clocks[64] = {0};
    int nc = (int)(min_clients + rbelow(&r, max_clients - min_clients + 1));
    if (nc > 64) nc = 64;
    pick_clients(&r, nc, clients);
    const int ops = (int)(min_ops + rbelow(&r, max_ops - min_ops + 1));
    int nd; size_t tl = 0; uint32_t nu = 0;
    session(&r, ops, nc, clients, clocks, doc, &nd, tmp, &tl, toff, &nu, 0);
    /* merged state: client blocks in descending client order; a client's inserts in clock order.
     * Re-emit each insert's struct from the per-update bytes (structs start at offset 2+vu(client)+vu(clock)). */
    int ord[64]; for (int i = 0; i < nc; i++) ord[i] = i;
    for (int i = 1; i < nc; i++) { int t = ord[i], j = i; while (j > 0 && clients[ord[j - 1]] < clients[t]) { ord[j] = ord[j - 1]; j--; } ord[j] = t; }
    int nblocks = 0; for (int i = 0; i < nc; i++) nblocks += clocks[i] > 0;
    b += vu(buf + b, (uint64_t)nblocks);
    for (int q = 0; q < nc; q++) {
      const int ci = ord[q];
      if (!clocks[ci]) continue;
      b += vu(buf + b, clocks[ci]); b += vu(buf + b, clients[ci]); buf[b++] = 0;
      for (uint32_t k = 0; k < clocks[ci]; k++) {
        /* find update of (client, k): scan updates (insert-only sessions) */
        for (uint32_t u = 0; u < nu; u++) {
          const uint8_t *p = tmp + toff[u]; size_t i = 2; uint64_t cl = 0, ck = 0; int sh = 0;
          do { cl |= (uint64_t)(p[i] & 127) << sh; sh += 7; } while (p[i++] & 128);
          sh = 0; do { ck |= (uint64_t)(p[i] & 127) << sh; sh += 7; } while (p[i++] & 128);
          if (cl == clients[ci] && ck == k) {
            const size_t end = (u + 1 < nu ? toff[u + 1] : tl) - 1; /* drop the update's empty DS byte */
            memcpy(buf + b, p + i, end - toff[u] - i); b += end - toff[u] - i;
            break;
          }
        }
      }
    }
    buf[b++] = 0; /* empty delete set */
    /* state vector: each client with probability 0.9, clock uniform in [0, end] */
    int empty = rbelow(&r, 10) == 0;
    uint8_t *sp = sv + s; size_t sn = 0; int ne = 0;
    uint8_t ent[64 * 20]; size_t el = 0;
    if (!empty) for (int i = 0; i < nc; i++) {
      if (!clocks[i]) continue;
      el += vu(ent + el, clients[i]); el += vu(ent + el, rbelow(&r, (uint64_t)clocks[i] + 1)); ne++;
    }
    sn += vu(sp, (uint64_t)ne); memcpy(sp + sn, ent, el); sn += el; s += sn;
  }
  doc_off[n_docs] = b; sv_off[n_docs] = s; *sv_bytes = s;
  free(doc); free(tmp); free(toff);
  return b;
}
