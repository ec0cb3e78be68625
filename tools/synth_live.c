/*
 * synth_live.c -- "live session" documents for the doc-normalized snapshot (f-1) at BASELINE sizes: a simulated
 * Y.Doc editing session written as yjs writes its updates, so that Y.applyUpdate integrates every struct (no pending
 * structs, no ids that do not exist, every origin / right origin / parent in the same parent list as the item).
 *
 * The corpora of synth.c (configs C3 / C5) are built for mergeUpdates, which never integrates: their origins point at
 * random ids, and yjs 13.5.16's applyUpdate throws on them ("Cannot read property 'origin' of undefined" inside
 * Item.integrate).  A server document never looks like that, and the snapshot the extension stores by default is
 * encodeStateAsUpdate(applyUpdate(new Doc, merged)) -- so the store is measured on these documents instead.
 *
 * Model (xml = 1, config C5: Tiptap / ProseMirror): the root XmlFragment "prosemirror" holds XmlElement "paragraph"
 * items; each paragraph holds one XmlText whose list holds ContentString runs (ASCII and 2-byte UTF-8 words),
 * ContentFormat marks and ContentEmbed images; paragraphs carry attributes (map entries "level" / "class" with
 * ContentAny values, an overwrite deleting the previous entry).  xml = 0 (config C3 shape): one root Y.Text "t",
 * strings only, heavy deletions.  Inserts land after a random item of a list or inside a string item (splitting it:
 * origin = the unit before, right origin = the unit after, as Y.Text.insert records); deletions cut ranges out of
 * string items.  Every item is written with the origin / right origin / parent it was created with (a gc:false
 * document's encoding: deleted items keep their content), so the bytes are exactly a valid yjs update.
 *
 * Documents d0 .. d0 + n_docs - 1 of a corpus (each from its own PRNG stream: chunks are generated in parallel).
 * Per document: [state, ...log] -- state = every struct of the session's first part (client blocks descending by
 * client, clocks from 0) + its delete set (clients descending, ranges sorted and merged); log = k - 1 later updates
 * of the same session (inserts of 1-3 structs by one client, or delete-set-only updates).  The state's size follows
 * max_bytes * r^-0.8 for the document of rank r (floored at min_bytes).  With xml and n_clients > 64 the state holds
 * exactly n_clients client blocks (every client edits at least once).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

typedef struct { uint64_t s; } LRng;
static uint64_t lnext(LRng *r) { uint64_t x = r->s; x ^= x >> 12; x ^= x << 25; x ^= x >> 27; r->s = x; return x * 2685821657736338717ULL; }
static uint64_t lbelow(LRng *r, uint64_t n) { return n ? lnext(r) % n : 0; }
static size_t lvu(uint8_t *o, uint64_t v) { size_t n = 0; while (v > 127) { o[n++] = (uint8_t)(0x80 | (v & 127)); v >>= 7; } o[n++] = (uint8_t)v; return n; }
static size_t lstr(uint8_t *o, const char *s, size_t n) { size_t b = lvu(o, n); memcpy(o + b, s, n); return b + n; }

enum { K_STR = 4, K_EMBED = 5, K_FORMAT = 6, K_TYPE = 7, K_ANY = 8 };
typedef struct {
  uint32_t ci, clock, len;          /* client index, first clock, length (UTF-16 units for strings, else 1) */
  int32_t parent;                   /* type item index, -1 = the root type */
  int32_t key;                      /* parentSub: -1 none, else attribute key index */
  int32_t prev, next;               /* neighbours in the parent's list (map entries: unused) */
  int32_t o_ci, r_ci;               /* origin / right origin client index (-1: none) */
  uint32_t o_clk, r_clk;
  uint32_t coff, clen;              /* content bytes in the pool: string UTF-8 / format key,value / embed JSON / any value */
  uint8_t kind, deleted, sub;       /* sub: type ref (3 XmlElement, 6 XmlText) or format / any variant */
} LItem;

typedef struct {
  LItem *it; uint32_t n, cap;
  char *pool; size_t pn, pcap;
  int32_t *head;                    /* per type slot: first item of its list (-1 empty) */
  int32_t **members; uint32_t *nmem, *cmem;   /* per type slot: its list's items (any order, for random picks) */
  uint32_t ntypes, ctypes;
  int32_t *type_item;               /* type slot -> the ContentType item (-1: the root) */
  int32_t *slot_of;                 /* item -> its type slot, if it is a type (else -1) */
  uint32_t *paras; uint32_t npara, cpara;     /* paragraph type slots */
  uint32_t *texts; uint32_t ntext, ctext;     /* XmlText / root Y.Text type slots */
  int32_t *attr;                    /* paragraph slot * 2 + key -> current map entry item (-1) */
  uint32_t *clock;                  /* per client: next clock */
  uint32_t nc; const uint32_t *cid;
  /* deletions: (ci, clock, len) */
  uint32_t *dci, *dck, *dln; size_t nd, dcap;
} LDoc;

static void *grow(void *p, uint32_t *cap, uint32_t need, size_t sz) {
  if (need <= *cap) return p;
  uint32_t c = *cap ? *cap : 16; while (c < need) c *= 2;
  p = realloc(p, (size_t)c * sz); *cap = c; return p;
}
static uint32_t pool_add(LDoc *D, const char *s, size_t n) {
  if (D->pn + n > D->pcap) { while (D->pn + n > D->pcap) D->pcap = D->pcap ? D->pcap * 2 : 1 << 16; D->pool = realloc(D->pool, D->pcap); }
  memcpy(D->pool + D->pn, s, n); D->pn += n; return (uint32_t)(D->pn - n);
}
static int32_t new_item(LDoc *D, uint32_t ci, uint32_t len, uint8_t kind) {
  D->it = grow(D->it, &D->cap, D->n + 1, sizeof(LItem));
  D->slot_of = realloc(D->slot_of, sizeof(int32_t) * D->cap);
  LItem *x = &D->it[D->n];
  memset(x, 0, sizeof *x);
  x->ci = ci; x->clock = D->clock[ci]; x->len = len; x->kind = kind; x->parent = -1; x->key = -1; x->prev = x->next = -1;
  x->o_ci = x->r_ci = -1;
  D->clock[ci] += len;
  D->slot_of[D->n] = -1;
  return (int32_t)D->n++;
}
static uint32_t new_type_slot(LDoc *D, int32_t item) {
  if (D->ntypes == D->ctypes) {
    D->ctypes = D->ctypes ? D->ctypes * 2 : 64;
    D->head = realloc(D->head, sizeof(int32_t) * D->ctypes);
    D->members = realloc(D->members, sizeof(int32_t *) * D->ctypes);
    D->nmem = realloc(D->nmem, sizeof(uint32_t) * D->ctypes);
    D->cmem = realloc(D->cmem, sizeof(uint32_t) * D->ctypes);
    D->type_item = realloc(D->type_item, sizeof(int32_t) * D->ctypes);
    D->attr = realloc(D->attr, sizeof(int32_t) * 2 * D->ctypes);
  }
  const uint32_t s = D->ntypes++;
  D->head[s] = -1; D->members[s] = NULL; D->nmem[s] = 0; D->cmem[s] = 0; D->type_item[s] = item;
  D->attr[2 * s] = D->attr[2 * s + 1] = -1;
  if (item >= 0) D->slot_of[item] = (int32_t)s;
  return s;
}
static void add_member(LDoc *D, uint32_t slot, int32_t item) {
  D->members[slot] = grow(D->members[slot], &D->cmem[slot], D->nmem[slot] + 1, sizeof(int32_t));
  D->members[slot][D->nmem[slot]++] = item;
}
/* links item x into list `slot` after item `left` (-1: at the head) and sets its origin / right origin from the
 * neighbours (origin = left's last unit, right origin = right's first unit; parent when neither) */
static void link_after(LDoc *D, uint32_t slot, int32_t left, int32_t x) {
  LItem *X = &D->it[x];
  const int32_t right = left >= 0 ? D->it[left].next : D->head[slot];
  X->prev = left; X->next = right;
  if (left >= 0) { D->it[left].next = x; X->o_ci = (int32_t)D->it[left].ci; X->o_clk = D->it[left].clock + D->it[left].len - 1; }
  else D->head[slot] = x;
  if (right >= 0) { D->it[right].prev = x; X->r_ci = (int32_t)D->it[right].ci; X->r_clk = D->it[right].clock; }
  X->parent = D->type_item[slot];
  add_member(D, slot, x);
}
/* byte offset of unit k of a string item (all BMP: one unit per code point) */
static uint32_t unit_off(const LDoc *D, const LItem *X, uint32_t k) {
  uint32_t b = 0, u = 0;
  while (u < k) { b++; while (b < X->clen && (D->pool[X->coff + b] & 0xC0) == 0x80) b++; u++; }
  return b;
}
/* splits string item x at unit k (0 < k < len): x keeps [0, k), the new right part [k, len) follows it in the list
 * with origin = x's unit k - 1 and x's right origin (Item split, yjs splitItem) */
static int32_t split_at(LDoc *D, uint32_t slot, int32_t x, uint32_t k) {
  const uint32_t b = unit_off(D, &D->it[x], k);
  D->it = grow(D->it, &D->cap, D->n + 1, sizeof(LItem));
  D->slot_of = realloc(D->slot_of, sizeof(int32_t) * D->cap);
  const int32_t y = (int32_t)D->n++;
  LItem *X = &D->it[x], *Y = &D->it[y];
  *Y = *X;
  D->slot_of[y] = -1;
  Y->clock = X->clock + k; Y->len = X->len - k; Y->coff = X->coff + b; Y->clen = X->clen - b;
  Y->o_ci = (int32_t)X->ci; Y->o_clk = X->clock + k - 1;
  X->len = k; X->clen = b;
  Y->prev = x; Y->next = X->next;
  if (X->next >= 0) D->it[X->next].prev = y;
  X->next = y;
  add_member(D, slot, y);
  return y;
}
static void del_range(LDoc *D, uint32_t ci, uint32_t clock, uint32_t len) {
  if (D->nd == D->dcap) {
    D->dcap = D->dcap ? D->dcap * 2 : 1024;
    D->dci = realloc(D->dci, 4 * D->dcap); D->dck = realloc(D->dck, 4 * D->dcap); D->dln = realloc(D->dln, 4 * D->dcap);
  }
  D->dci[D->nd] = ci; D->dck[D->nd] = clock; D->dln[D->nd] = len; D->nd++;
}

static const char *WORDS[] = {"lorem ", "ipsum ", "dolor ", "sit ", "amet ", "caf\xc3\xa9 ", "na\xc3\xafve ", "x", "\xc3\xbc" "ber ", "q"};
static uint32_t units_of(const char *s, size_t n) { uint32_t u = 0; for (size_t i = 0; i < n; i++) u += ((uint8_t)s[i] & 0xC0) != 0x80; return u; }
static int32_t new_string(LDoc *D, LRng *r, uint32_t ci) {
  char s[128]; size_t sl = 0;
  const uint32_t nw = 1 + (uint32_t)lbelow(r, 6);
  for (uint32_t w = 0; w < nw; w++) { const char *t = WORDS[lbelow(r, 10)]; const size_t tl = strlen(t); memcpy(s + sl, t, tl); sl += tl; }
  const int32_t x = new_item(D, ci, units_of(s, sl), K_STR);
  D->it[x].coff = pool_add(D, s, sl); D->it[x].clen = (uint32_t)sl;
  return x;
}
/* a random live list position of type slot t: (left item, or -1 for the head); may split a string item */
static int32_t pick_left(LDoc *D, LRng *r, uint32_t t, int *mid_split) {
  *mid_split = 0;
  if (!D->nmem[t] || lbelow(r, 8) == 0) return -1;
  const int32_t x = D->members[t][lbelow(r, D->nmem[t])];
  LItem *X = &D->it[x];
  if (X->kind == K_STR && !X->deleted && X->len > 1 && lbelow(r, 2)) {
    split_at(D, t, x, 1 + (uint32_t)lbelow(r, X->len - 1));
    *mid_split = 1;
  }
  return x;
}
static void op_text(LDoc *D, LRng *r, uint32_t ci, int xml) {
  const uint32_t t = D->texts[lbelow(r, D->ntext)];
  int ms;
  const int32_t left = pick_left(D, r, t, &ms);
  const uint32_t k = (uint32_t)lbelow(r, 100);
  int32_t x;
  if (xml && k < 12) {        /* a formatting mark */
    static const char *F[] = {"bold", "true", "italic", "true", "link", "{\"href\":\"https://x.y/z\"}", "bold", "null"};
    const uint32_t f = (uint32_t)lbelow(r, 4);
    char b[96]; size_t bl = 0;
    bl += lstr((uint8_t *)b + bl, F[2 * f], strlen(F[2 * f])); bl += lstr((uint8_t *)b + bl, F[2 * f + 1], strlen(F[2 * f + 1]));
    x = new_item(D, ci, 1, K_FORMAT); D->it[x].coff = pool_add(D, b, bl); D->it[x].clen = (uint32_t)bl;
  } else if (xml && k < 16) { /* an embed */
    static const char e[] = "{\"image\":\"a.png\"}";
    x = new_item(D, ci, 1, K_EMBED); D->it[x].coff = pool_add(D, e, sizeof e - 1); D->it[x].clen = sizeof e - 1;
  } else x = new_string(D, r, ci);
  link_after(D, t, left, x);
}
static void op_para(LDoc *D, LRng *r, uint32_t ci) {
  const uint32_t root = 0;
  int ms;
  const int32_t left = pick_left(D, r, root, &ms);
  const int32_t p = new_item(D, ci, 1, K_TYPE);
  D->it[p].sub = 3;
  link_after(D, root, left, p);
  const uint32_t ps = new_type_slot(D, p);
  D->paras = grow(D->paras, &D->cpara, D->npara + 1, 4); D->paras[D->npara++] = ps;
  const int32_t tx = new_item(D, ci, 1, K_TYPE);
  D->it[tx].sub = 6;
  link_after(D, ps, -1, tx);
  const uint32_t ts = new_type_slot(D, tx);
  D->texts = grow(D->texts, &D->ctext, D->ntext + 1, 4); D->texts[D->ntext++] = ts;
  const int32_t s = new_string(D, r, ci);
  link_after(D, ts, -1, s);
}
static void op_attr(LDoc *D, LRng *r, uint32_t ci) {
  const uint32_t ps = D->paras[lbelow(r, D->npara)], key = (uint32_t)lbelow(r, 2);
  const int32_t prev = D->attr[2 * ps + key];
  const int32_t x = new_item(D, ci, 1, K_ANY);
  LItem *X = &D->it[x];
  X->sub = (uint8_t)lbelow(r, 2); X->coff = (uint32_t)lbelow(r, 60);
  X->parent = D->type_item[ps]; X->key = (int32_t)key;
  if (prev >= 0) {   /* the overwrite: left = the key's current entry, which is deleted */
    X->o_ci = (int32_t)D->it[prev].ci; X->o_clk = D->it[prev].clock;
    D->it[prev].deleted = 1; del_range(D, D->it[prev].ci, D->it[prev].clock, 1);
  }
  D->attr[2 * ps + key] = x;
}
static void op_delete(LDoc *D, LRng *r) {
  const uint32_t t = D->texts[lbelow(r, D->ntext)];
  if (!D->nmem[t]) return;
  int32_t x = D->members[t][lbelow(r, D->nmem[t])];
  if (D->it[x].deleted) return;
  const uint32_t len = D->it[x].len;
  if (D->it[x].kind == K_STR && len > 2 && lbelow(r, 2)) {   /* a range [a, b) inside the string */
    const uint32_t a = (uint32_t)lbelow(r, len - 1), b = a + 1 + (uint32_t)lbelow(r, len - a - 1);
    if (b < len) split_at(D, t, x, b);
    if (a > 0) x = split_at(D, t, x, a);
  }
  D->it[x].deleted = 1;
  del_range(D, D->it[x].ci, D->it[x].clock, D->it[x].len);
}

/* the struct of item x, as Item.write writes it (V1) */
static size_t w_item(const LDoc *D, const LItem *X, const char *rootname, uint8_t *o) {
  static const char *KEYS[] = {"level", "class"};
  size_t b = 0;
  const int has_o = X->o_ci >= 0, has_r = X->r_ci >= 0;
  o[b++] = (uint8_t)(X->kind | (has_o ? 0x80 : 0) | (has_r ? 0x40 : 0) | (X->key >= 0 ? 0x20 : 0));
  if (has_o) { b += lvu(o + b, D->cid[X->o_ci]); b += lvu(o + b, X->o_clk); }
  if (has_r) { b += lvu(o + b, D->cid[X->r_ci]); b += lvu(o + b, X->r_clk); }
  if (!has_o && !has_r) {
    if (X->parent < 0) { o[b++] = 1; b += lstr(o + b, rootname, strlen(rootname)); }
    else { o[b++] = 0; b += lvu(o + b, D->cid[D->it[X->parent].ci]); b += lvu(o + b, D->it[X->parent].clock); }
    if (X->key >= 0) b += lstr(o + b, KEYS[X->key], strlen(KEYS[X->key]));
  }
  switch (X->kind) {
    case K_STR: b += lstr(o + b, D->pool + X->coff, X->clen); break;
    case K_FORMAT: case K_EMBED:
      if (X->kind == K_EMBED) b += lvu(o + b, X->clen);
      memcpy(o + b, D->pool + X->coff, X->clen); b += X->clen; break;
    case K_TYPE: b += lvu(o + b, X->sub); if (X->sub == 3) b += lstr(o + b, "paragraph", 9); break;
    case K_ANY: o[b++] = 1; if (X->sub) { o[b++] = 119; b += lstr(o + b, "heading", 7); } else { o[b++] = 125; o[b++] = (uint8_t)X->coff; } break;
  }
  return b;
}
typedef struct { uint64_t key; uint64_t idx; } LKey;
static int cmp_lkey(const void *a, const void *b) {
  const uint64_t x = ((const LKey *)a)->key, y = ((const LKey *)b)->key; return x < y ? -1 : x > y;
}
/* the delete set of deletions [d0, d1): clients descending (rank_of: 0 = the largest id), ranges sorted and merged */
static size_t w_ds(LDoc *D, size_t d0, size_t d1, uint8_t *o, const uint32_t *rank_of) {
  const size_t n = d1 - d0;
  LKey *k = (LKey *)malloc(sizeof(LKey) * (n + 1));
  for (size_t i = 0; i < n; i++) { k[i].key = ((uint64_t)rank_of[D->dci[d0 + i]] << 32) | D->dck[d0 + i]; k[i].idx = d0 + i; }
  qsort(k, n, sizeof(LKey), cmp_lkey);
  size_t b = 0, ncl = 0;
  for (size_t i = 0; i < n; i++) if (i == 0 || D->dci[k[i].idx] != D->dci[k[i - 1].idx]) ncl++;
  b += lvu(o + b, ncl);
  size_t i = 0;
  while (i < n) {
    const uint32_t c = D->dci[k[i].idx];
    size_t j = i; while (j < n && D->dci[k[j].idx] == c) j++;
    uint32_t nr = 0, e = 0;
    for (size_t q = i; q < j; q++) {
      const uint32_t s = D->dck[k[q].idx], l = D->dln[k[q].idx];
      if (q == i || s > e) nr++;
      if (q == i || s + l > e) e = s + l;
    }
    b += lvu(o + b, D->cid[c]); b += lvu(o + b, nr);
    size_t q = i;
    while (q < j) {
      const uint32_t s0 = D->dck[k[q].idx]; uint32_t e0 = s0 + D->dln[k[q].idx]; q++;
      while (q < j && D->dck[k[q].idx] <= e0) { const uint32_t e1 = D->dck[k[q].idx] + D->dln[k[q].idx]; if (e1 > e0) e0 = e1; q++; }
      b += lvu(o + b, s0); b += lvu(o + b, e0 - s0);
    }
    i = j;
  }
  free(k);
  return b;
}
static int cmp_item_key(const void *a, const void *b) {
  const uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b; return x < y ? -1 : x > y;
}

/* buf capacity: max(sum of the state sizes, ...) * 1.5 + n_docs * (max_k * 96 + 64 KiB); upd_off: n_docs * max_k + 1 */
size_t synth_live_docs(uint64_t seed, uint32_t d0, uint32_t n_docs, uint64_t max_bytes, uint64_t min_bytes, uint32_t n_clients, uint32_t max_k, int xml,
                       uint8_t *buf, uint64_t *upd_off, uint32_t *doc_upd) {
  size_t b = 0; uint32_t nu = 0;
  const char *rootname = xml ? "prosemirror" : "t";
  for (uint32_t d = 0; d < n_docs; d++) {
    LRng rr = { (seed * 0x9E3779B97F4A7C15ULL) ^ ((uint64_t)(d0 + d + 1) * 0xD6E8FEB86659FD93ULL) };
    LRng *r = &rr; lnext(r); lnext(r);
    doc_upd[d] = nu;
    const double sz = (double)max_bytes * pow((double)(d0 + d + 1), -0.8);
    uint64_t target = (uint64_t)sz; if (target < min_bytes) target = min_bytes;
    uint32_t nc = xml && n_clients > 64 ? n_clients : 1 + (uint32_t)lbelow(r, n_clients);
    uint32_t *cid = (uint32_t *)malloc(4 * nc), *rank_of = (uint32_t *)malloc(4 * nc);
    /* distinct client ids: an odd multiplier over a random start (a bijection of 2^32) */
    const uint32_t a = (uint32_t)lnext(r) | 1u, c0 = (uint32_t)lnext(r);
    for (uint32_t i = 0; i < nc; i++) cid[i] = a * (c0 + i) + 0x9E3779B9u;
    LDoc D; memset(&D, 0, sizeof D);
    D.nc = nc; D.cid = cid; D.clock = (uint32_t *)calloc(nc, 4);
    new_type_slot(&D, -1);                      /* slot 0: the root type */
    if (!xml) { D.texts = grow(D.texts, &D.ctext, 1, 4); D.texts[D.ntext++] = 0; }
    /* the session until the state reaches its size; every client edits at least once first (xml, many clients) */
    uint64_t est = 16;
    uint32_t turn = 0;
    uint8_t scratch[512];
    const uint32_t del_pct = xml ? 12 : 40;
    while (est < target || (xml && nc > 64 && turn < nc)) {
      const uint32_t ci = turn < nc && (xml && nc > 64) ? turn : (uint32_t)lbelow(r, nc);
      turn++;
      const uint32_t n0 = D.n, k = (uint32_t)lbelow(r, 100);
      if (xml && (D.npara == 0 || k < 6)) op_para(&D, r, ci);
      else if (xml && k < 10) op_attr(&D, r, ci);
      else if (k < 10 + del_pct && D.n > 4) { op_delete(&D, r); if (D.clock[ci] == 0) op_text(&D, r, ci, xml); }
      else op_text(&D, r, ci, xml);
      for (uint32_t q = n0; q < D.n; q++) est += w_item(&D, &D.it[q], rootname, scratch);
      if (D.nd) est += 3;
    }
    /* the state: client blocks descending by client id (rank 0 = the largest id), structs in clock order */
    {
      uint64_t *ord = (uint64_t *)malloc(sizeof(uint64_t) * nc);
      for (uint32_t i = 0; i < nc; i++) ord[i] = ((uint64_t)(0xFFFFFFFFu - cid[i]) << 32) | i;
      qsort(ord, nc, 8, cmp_item_key);
      for (uint32_t i = 0; i < nc; i++) rank_of[(uint32_t)ord[i]] = i;
      free(ord);
    }
    LKey *kv = (LKey *)malloc(sizeof(LKey) * (D.n + 1));
    for (uint32_t i = 0; i < D.n; i++) { kv[i].key = ((uint64_t)rank_of[D.it[i].ci] << 32) | D.it[i].clock; kv[i].idx = i; }
    qsort(kv, D.n, sizeof(LKey), cmp_lkey);
    upd_off[nu++] = b;
    uint32_t nblocks = 0;
    for (uint32_t i = 0; i < nc; i++) nblocks += D.clock[i] > 0;
    b += lvu(buf + b, nblocks);
    uint32_t i = 0;
    while (i < D.n) {
      const uint32_t ci = D.it[kv[i].idx].ci;
      uint32_t j = i; while (j < D.n && D.it[kv[j].idx].ci == ci) j++;
      b += lvu(buf + b, j - i); b += lvu(buf + b, cid[ci]); b += lvu(buf + b, 0);
      for (uint32_t q = i; q < j; q++) b += w_item(&D, &D.it[kv[q].idx], rootname, buf + b);
      i = j;
    }
    b += w_ds(&D, 0, D.nd, buf + b, rank_of);
    free(kv);
    /* the log: k - 1 later updates of the same session */
    const uint32_t k = 2 + (uint32_t)lbelow(r, max_k - 1);
    for (uint32_t u = 1; u < k; u++) {
      upd_off[nu++] = b;
      const size_t nd0 = D.nd;
      if (lbelow(r, 100) < 40) {
        for (uint32_t t = 0; t < 1 + (uint32_t)lbelow(r, 3); t++) op_delete(&D, r);
        buf[b++] = 0;
        if (D.nd > nd0) b += w_ds(&D, nd0, D.nd, buf + b, rank_of);
        else buf[b++] = 0;
      } else {
        const uint32_t ci = (uint32_t)lbelow(r, nc), n0 = D.n, ck = D.clock[ci];
        const uint32_t ns = 1 + (uint32_t)lbelow(r, 3);
        for (uint32_t s = 0; s < ns; s++) {
          if (xml && lbelow(r, 10) == 0) op_para(&D, r, ci);
          else op_text(&D, r, ci, xml);
        }
        /* the new items of client ci (splits of earlier items keep their clocks and are not re-sent) */
        uint32_t cnt = 0;
        for (uint32_t q = n0; q < D.n; q++) cnt += D.it[q].ci == ci && D.it[q].clock >= ck;
        buf[b++] = 1; b += lvu(buf + b, cnt); b += lvu(buf + b, cid[ci]); b += lvu(buf + b, ck);
        /* in clock order: the items were created in clock order (splits of new items cannot happen in one update) */
        for (uint32_t q = n0; q < D.n; q++) if (D.it[q].ci == ci && D.it[q].clock >= ck) b += w_item(&D, &D.it[q], rootname, buf + b);
        buf[b++] = 0;
      }
    }
    free(cid); free(rank_of); free(D.clock);
    free(D.it); free(D.pool); free(D.head); free(D.nmem); free(D.cmem); free(D.type_item); free(D.slot_of);
    for (uint32_t s = 0; s < D.ntypes; s++) free(D.members[s]);
    free(D.members); free(D.attr); free(D.paras); free(D.texts); free(D.dci); free(D.dck); free(D.dln);
  }
  doc_upd[n_docs] = nu; upd_off[nu] = b;
  return b;
}
