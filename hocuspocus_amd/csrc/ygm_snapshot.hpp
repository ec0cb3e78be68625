// ygm_snapshot.hpp -- doc-normalized snapshot:
//
//     snapshot(u) = Y.encodeStateAsUpdate(Y.applyUpdate(new Y.Doc(), u))
//
// what extension-database stores (packages/extension-database/src/Database.ts:55-60): the update a
// fresh document holds after integrating u in one transaction -- deleted content garbage-collected,
// split and adjacent structs merged.  Restated from yjs 13.5.16 (the bundle this image carries;
// offsets "Y@" into 3502.fbe0c610be82ba1360db.js):
//   readUpdate / readClientsStructRefs  Y@20500-21900   integrateStructs (dependency stack)  Y@21000-22500
//   Item.getMissing / Item.integrate    Y@77700-79900   splitItem Y@76300   getItemClean* Y@29900-30100
//   readAndApplyDeleteSet               Y@11500-12200   Item.delete / ContentType.delete / gc  Y@73600, Y@80200
//   cleanupTransactions: tryGcDeleteSet, tryMergeDeleteSet, afterState merge   Y@30900-32900
//   Item.mergeWith / content mergeWith  Y@79900, Y@69000-73400   encodeStateAsUpdate Y@23300-23900
//
// One thread runs one document, sequentially, over a private workspace carved from global memory
// (index-based records, explicit stacks, no allocation, no recursion).  The structure is the
// reference's: struct store per client (input structs in clock order, each a chain of its split
// parts), document lists through left/right item indices, a type table (root types by name,
// nested types per ContentType item) with per-type key lists for map entries.
//
// Pending structs and a pending delete set (missing dependencies, clock gaps, Skips followed by structs, ranges past
// the state): integrateStructs' dependency stack is followed as the reference runs it, its quirks included (the rest
// of a walled client is the slice from its refs cursor, a client met again on the stack keeps only that struct), and
// readAndApplyDeleteSet keeps the ranges past the state.  encodeStateAsUpdate then returns
// mergeUpdates([state, pendingDs, diffUpdate(pendingStructs.update)]) (Y@23300): the document's output is those three
// updates (ST_PEND, the layout at pend_hdr) and the engine merges them with the merge kernels.
// Sub-documents (ContentDoc, one clock, never split) integrate like any other content; their options are written as
// read when canonical (ContentDoc's constructor rebuilds them: read_struct's check), refused (ST_NONCANON) if not.
// Envelope: an update that repeats a client block, overlaps structs, carries content with non-minimal varuints in a
// verbatim field, or whose parent id names a non-type item, returns ST_UNSUP: the caller keeps its yjs path for it.
// After one transaction on a fresh document every struct is a merge candidate, so the reference's
// three merge passes (delete-set ranges, afterState, _mergeStructs) reduce to one right-to-left
// pass per client: mergeability is preserved along a merged run, so maximal runs are unique.
#pragma once
#include "ygm_v1.hpp"

namespace ygm {
namespace snap {

constexpr int ST_UNSUP = 9;   // YGM_EUNSUPPORTED
constexpr int ST_PEND = 64;   // internal: the output is [state, pendingDs, pending structs] for the merge kernels
constexpr uint32_t F_SNAP_STATE = 16u;   // YGM_F_SNAP_STATE: a pending document's output is its integrated state
// a pending document's output: this header, then the three V1 updates back to back (an absent one as the empty update)
struct PendHdr { uint32_t len[3]; uint32_t magic; };
constexpr uint32_t PEND_MAGIC = 0x444E4550u;

enum : uint8_t { F_DEL = 1, F_HO = 2, F_HR = 4, F_INT = 8, F_GONE = 16 };
enum : uint8_t { SK_ITEM = 0, SK_GC = 1, SK_SKIP = 2 };
constexpr int32_t P_NONE = -1, P_ID = -2;

struct SI {
  uint32_t client, clock, len;       // id and length (clock units)
  int32_t left, right;               // document-list neighbours (item indices, -1 null)
  int32_t nxt;                       // next part of the same input struct (clock order)
  int32_t orig;                      // the input struct (ref index) this part comes from
  uint32_t oc, ok, rc, rk;           // origin / right origin ids (F_HO / F_HR)
  int32_t parent;                    // type index, P_NONE (none / GC), P_ID (pc, pk unresolved)
  uint32_t pc, pk;
  uint32_t sub_off; int32_t sub_len; // parentSub key bytes in the input (-1: null)
  int32_t type;                      // ContentType items: their type
  int32_t p0, p1;                    // content pieces (String / JSON / Any / Deleted)
  uint32_t c_start, c_end;           // content bytes in the input (verbatim kinds)
  uint32_t ms, mr;                   // integrate's conflict sets (epoch marks)
  uint8_t kind, ref, flags, pad;
};
// String: UTF-8 bytes [off, end) with a U+FFFD before (pre) / after (post) from surrogate-pair splits,
// cnt = UTF-16 units.  JSON / Any: the encoded elements [off, end), cnt elements.  Deleted: cnt.
struct Piece { uint32_t off, end, cnt; int32_t next; uint8_t pre, post, pad0, pad1; };
struct TypeRec { int32_t item; uint32_t name_off, name_len; int32_t start, map; };
struct MapEnt { int32_t type; uint32_t key_off, key_len; int32_t item, next; };
// rest0 / restn: the client's pending structs (refs [rest0, rest0 + restn)); gone: taken off integrateStructs' map
struct Cli { uint32_t id; int32_t r0, rn, ri; uint32_t state; int32_t ins, ni, rest0, restn; uint32_t gone; };
struct Rng { uint32_t client, clock, len, pad; };

// workspace capacities of a document, from its counts (input structs S, delete-set ranges D, client
// blocks C, bytes n)
struct Caps {
  uint32_t it, pc, ty, me, cl, tx, dsin, st, seq, out, hc;   // hc: client hash slots (a power of two >= 2 cl)
};
YDEV Caps caps_of(uint32_t S, uint32_t D, uint32_t C, uint32_t n) {
  Caps k;
  k.it = 3u * S + 2u * D + 4u;
  k.pc = k.it; k.ty = S + 2u; k.me = S + 2u; k.cl = C + 1u; k.tx = k.it + 2u; k.dsin = D + 1u;
  k.st = k.it + k.ty + 4u; k.seq = k.it + 1u;
  k.out = n + 48u * k.it + 16u * k.cl + 64u;
  k.hc = 16u;
  while (k.hc < 2u * k.cl) k.hc <<= 1;
  return k;
}
YDEV uint64_t al16(uint64_t x) { return (x + 15u) & ~15ull; }
YDEV uint64_t ws_core_bytes(const Caps& k) {   // the workspace without its output region
  return al16((uint64_t)k.it * sizeof(SI)) + al16((uint64_t)k.pc * sizeof(Piece)) + al16((uint64_t)k.ty * sizeof(TypeRec)) +
         al16((uint64_t)k.me * sizeof(MapEnt)) + al16((uint64_t)k.cl * sizeof(Cli)) + al16((uint64_t)k.tx * sizeof(Rng)) +
         al16((uint64_t)k.dsin * sizeof(Rng)) + al16((uint64_t)k.dsin * sizeof(Rng)) + al16(4ull * k.st) + al16(4ull * k.seq) +
         al16(4ull * k.hc);
}
YDEV uint64_t ws_bytes(const Caps& k) { return ws_core_bytes(k) + al16(k.out); }
// the encoder's writer: stores stop at cap (the caller's region), n counts on (> cap: the output did not fit)
struct OutCap {
  uint8_t* p; uint32_t n, cap;
  YDEV void b(uint8_t v) { if (n < cap) p[n] = v; n++; }
  YDEV void vu(uint64_t v) { while (v > 127) { b((uint8_t)(0x80 | (v & 127))); v >>= 7; } b((uint8_t)v); }
  YDEV void vu32(uint32_t v) { while (v > 127u) { b((uint8_t)(0x80u | (v & 127u))); v >>= 7; } b((uint8_t)v); }
  YDEV void copy(const uint8_t* s, uint32_t len) { for (uint32_t i = 0; i < len; i++) b(s[i]); }
};

// counts of a document (a light parse; errors are found again by the full pass)
YDEV_NI void count_doc(const uint8_t* p, uint32_t n, uint32_t flags, uint32_t& S, uint32_t& D, uint32_t& C) {
  S = D = C = 0;
  Cur c{p, 0, n, 0, 0};
  const uint64_t nb = c.vu();
  for (uint64_t b = 0; b < nb && !c.err; b++) {
    const uint64_t ns = c.vu(); c.vu(); c.vu();
    C++;
    for (uint64_t s = 0; s < ns && !c.err; s++) { SInfo si; read_struct_fast(c, si, flags); S++; }
  }
  const uint64_t nd = c.err ? 0 : c.vu();
  for (uint64_t k = 0; k < nd && !c.err; k++) {
    c.vu(); const uint64_t nr = c.vu();
    for (uint64_t r = 0; r < nr && !c.err; r++) { c.vu(); c.vu(); D++; }
  }
  if (S > (1u << 26) || D > (1u << 26)) { S = D = C = 0; }
}

struct Doc {
  const uint8_t* in; uint32_t n; uint32_t flags;
  SI* it; uint32_t n_it, cap_it;
  Piece* pc; uint32_t n_pc, cap_pc;
  TypeRec* ty; uint32_t n_ty, cap_ty;
  MapEnt* me; uint32_t n_me, cap_me;
  Cli* cl; uint32_t n_cl, cap_cl;
  int32_t* ch; uint32_t ch_mask;   // client id -> slot, open addressing (built once the table is sorted)
  Rng* tx; uint32_t n_tx, cap_tx;
  Rng* dsin; uint32_t n_dsin, cap_dsin;
  Rng* pds; uint32_t n_pds;        // the pending delete set: ranges (or their parts) past the state, in input order
  uint32_t n_rest;                 // clients with pending structs
  int32_t* st; uint32_t cap_st;
  int32_t* seq; uint32_t cap_seq;
  uint8_t* out; uint32_t cap_out;
  uint32_t epoch, n_ins;
  int err;
  bool pend;   // the output is the pending layout (PendHdr)

  YDEV void fail(int e) { if (!err) err = e; }

  // ------------------------------------------------------------------ lookups
  uint32_t hint_id; int32_t hint_k;   // the last client looked up (most lookups repeat it: a struct's own client)
  YDEV int32_t cli_slot(uint32_t id) {   // client table sorted by id
    if (hint_k >= 0 && hint_id == id) return hint_k;
    const int32_t k = cli_search(id);
    if (k >= 0) { hint_id = id; hint_k = k; }
    return k;
  }
  YDEV static uint32_t cli_hash(uint32_t id) { return (id * 0x9E3779B1u) ^ (id >> 15); }
  YDEV int32_t cli_search(uint32_t id) const {   // one or two dependent reads, not a binary search's ~log2(clients)
    for (uint32_t h = cli_hash(id) & ch_mask;; h = (h + 1u) & ch_mask) {
      const int32_t k = ch[h];
      if (k < 0 || cl[k].id == id) return k;
    }
  }
  YDEV uint32_t state_of(uint32_t id) { const int32_t k = cli_slot(id); return k < 0 ? 0u : cl[k].state; }
  // the integrated part holding (client, clock) (Y@29348 findIndexSS + the split chain); clock < state
  YDEV int32_t find(uint32_t client, uint32_t clock) {
    const int32_t k = cli_slot(client);
    if (k < 0 || clock >= cl[k].state) { fail(ST_UNSUP); return -1; }
    int32_t lo = cl[k].r0, hi = cl[k].r0 + cl[k].ni - 1, r = -1;
    {   // the last input struct starting at or before clock: first a guess by the clock distance -- exact when the
        // client's structs before it are single-clock (typed text) -- checked with one round trip of two reads
        // (each probe of the binary search below is a dependent global-memory read)
      const int64_t g = (int64_t)lo + ((int64_t)clock - (int64_t)it[lo].clock);
      if (g >= lo && g <= hi) {
        const int32_t x = (int32_t)g;
        if (it[x].clock <= clock && (x == hi || it[x + 1].clock > clock)) { r = x; lo = hi + 1; }
      }
    }
    while (lo <= hi) {   // last input struct starting at or before clock
      const int32_t m = (lo + hi) >> 1;
      if (it[m].clock <= clock) { r = m; lo = m + 1; } else hi = m - 1;
    }
    if (r < 0) { fail(ST_UNSUP); return -1; }
    int32_t x = r;
    while (x >= 0 && !(clock < it[x].clock + it[x].len)) x = it[x].nxt;
    if (x < 0) fail(ST_UNSUP);
    return x;
  }
  // the next struct of the same client in clock order
  YDEV int32_t next_part(int32_t x) {
    if (it[x].nxt >= 0) return it[x].nxt;
    const int32_t o = it[x].orig, k = cli_slot(it[x].client);
    return (k >= 0 && o + 1 < cl[k].r0 + cl[k].ni) ? o + 1 : -1;
  }
  YDEV bool key_eq(uint32_t a, uint32_t al, uint32_t b, uint32_t bl) const {
    if (al != bl) return false;
    for (uint32_t i = 0; i < al; i++) if (in[a + i] != in[b + i]) return false;
    return true;
  }
  YDEV int32_t map_get(int32_t t, uint32_t ko, uint32_t kl) const {
    for (int32_t e = ty[t].map; e >= 0; e = me[e].next) if (key_eq(me[e].key_off, me[e].key_len, ko, kl)) return me[e].item;
    return -1;
  }
  YDEV void map_set(int32_t t, uint32_t ko, uint32_t kl, int32_t item) {
    for (int32_t e = ty[t].map; e >= 0; e = me[e].next)
      if (key_eq(me[e].key_off, me[e].key_len, ko, kl)) { me[e].item = item; return; }
    if (n_me >= cap_me) { fail(ST_NOMEM); return; }
    MapEnt& m = me[n_me]; m.type = t; m.key_off = ko; m.key_len = kl; m.item = item; m.next = ty[t].map; ty[t].map = (int32_t)n_me++;
  }
  YDEV int32_t new_type(int32_t item, uint32_t no, uint32_t nl) {
    if (n_ty >= cap_ty) { fail(ST_NOMEM); return -1; }
    TypeRec& t = ty[n_ty]; t.item = item; t.name_off = no; t.name_len = nl; t.start = -1; t.map = -1;
    return (int32_t)n_ty++;
  }
  YDEV int32_t root_type(uint32_t no, uint32_t nl) {   // doc.get(name) (Y@ Doc.get): one root type per name
    for (uint32_t t = 0; t < n_ty; t++) if (ty[t].item == -1 && key_eq(ty[t].name_off, ty[t].name_len, no, nl)) return (int32_t)t;
    return new_type(-1, no, nl);
  }
  YDEV int32_t new_piece(uint32_t off, uint32_t end, uint32_t cnt, uint8_t pre, uint8_t post) {
    if (n_pc >= cap_pc) { fail(ST_NOMEM); return -1; }
    Piece& q = pc[n_pc]; q.off = off; q.end = end; q.cnt = cnt; q.next = -1; q.pre = pre; q.post = post;
    return (int32_t)n_pc++;
  }
  YDEV void tx_add(uint32_t client, uint32_t clock, uint32_t len) {   // addToDeleteSet (Y@10900)
    if (n_tx >= cap_tx) { fail(ST_NOMEM); return; }
    tx[n_tx].client = client; tx[n_tx].clock = clock; tx[n_tx].len = len; n_tx++;
  }
  YDEV bool deleted(int32_t x) const { return it[x].kind == SK_GC || (it[x].flags & F_DEL); }

  // ------------------------------------------------------------------ read (readClientsStructRefs)
  YDEV void parse() {
    Cur c{in, 0, n, 0, 0};
    const uint64_t nb = c.vu();
    for (uint64_t b = 0; b < nb && !c.err && !err; b++) {
      const uint64_t ns = c.vu(), client = c.vu(); uint64_t clock = c.vu();
      if (c.err) break;
      if (client > 0xFFFFFFFFull || n_cl >= cap_cl) { fail(ST_UNSUP); return; }
      Cli& k = cl[n_cl++];
      k.id = (uint32_t)client; k.r0 = (int32_t)n_it; k.rn = 0; k.ri = 0; k.state = 0; k.ins = -1; k.ni = 0; k.rest0 = 0; k.restn = 0; k.gone = 0;
      for (uint64_t s = 0; s < ns && !c.err; s++) {
        SInfo si; read_struct_fast(c, si, flags);
        if (c.err) break;
        if (clock + si.len > 0xFFFFFFFFull) { fail(ST_UNSUP); return; }
        if (n_it >= cap_it) { fail(ST_NOMEM); return; }
        SI& x = it[n_it];
        x.client = (uint32_t)client; x.clock = (uint32_t)clock; x.len = (uint32_t)si.len;
        x.left = x.right = x.nxt = -1; x.orig = (int32_t)n_it;
        x.oc = x.ok = x.rc = x.rk = 0; x.parent = P_NONE; x.pc = x.pk = 0; x.sub_off = 0; x.sub_len = -1; x.type = -1;
        x.p0 = x.p1 = -1; x.c_start = si.cstart; x.c_end = si.end; x.ms = x.mr = 0; x.flags = 0; x.pad = 0;
        x.kind = si.kind == K_GC ? SK_GC : si.kind == K_SKIP ? SK_SKIP : SK_ITEM;
        x.ref = si.ref;
        if (x.kind == SK_ITEM) {
          if (si.nc) { fail(ST_NONCANON); return; }
          Cur h{in, si.start + 1, si.cstart, 0, 0};
          const uint8_t info = si.info;
          if (info & 0x80) { x.oc = (uint32_t)h.vu(); x.ok = (uint32_t)h.vu(); x.flags |= F_HO; }
          if (info & 0x40) { x.rc = (uint32_t)h.vu(); x.rk = (uint32_t)h.vu(); x.flags |= F_HR; }
          if ((info & 0xC0) == 0) {
            const uint64_t pi = h.vu();
            if (pi == 1) { uint32_t l; const uint32_t s0 = h.buf(l); x.parent = root_type(s0, l); }
            else { x.pc = (uint32_t)h.vu(); x.pk = (uint32_t)h.vu(); x.parent = P_ID; }
            if (info & 0x20) { uint32_t l; x.sub_off = h.buf(l); x.sub_len = (int32_t)l; }
          }
          if (si.renc && x.ref != 1 && x.ref != 4 && x.ref != 8) { fail(ST_UNSUP); return; }   // verbatim fields must be minimal
          // content pieces
          Cur q{in, si.cstart, si.end, 0, 0};
          if (x.ref == 1) x.p0 = x.p1 = new_piece(0, 0, x.len, 0, 0);
          else if (x.ref == 4) { uint32_t l; const uint32_t s0 = q.buf(l); x.p0 = x.p1 = new_piece(s0, s0 + l, x.len, 0, 0); }
          else if (x.ref == 2 || x.ref == 8) { q.vu(); x.p0 = x.p1 = new_piece(q.pos, si.end, x.len, 0, 0); }
        }
        clock += si.len;
        n_it++; k.rn++;
      }
    }
    if (c.err) { fail(c.err); return; }
    if (err) return;
    // delete set (read now, applied after the structs: readAndApplyDeleteSet)
    const uint64_t nd = c.vu();
    for (uint64_t q = 0; q < nd && !c.err; q++) {
      const uint64_t client = c.vu(), nr = c.vu();
      for (uint64_t r = 0; r < nr && !c.err; r++) {
        const uint64_t ck = c.vu(), ln = c.vu();
        if (c.err) break;
        if (client > 0xFFFFFFFFull || ck + ln > 0xFFFFFFFFull) { fail(ST_UNSUP); return; }
        if (n_dsin >= cap_dsin) { fail(ST_NOMEM); return; }
        dsin[n_dsin].client = (uint32_t)client; dsin[n_dsin].clock = (uint32_t)ck; dsin[n_dsin].len = (uint32_t)ln; n_dsin++;
      }
    }
    if (c.err) { fail(c.err); return; }
    if (c.pos != c.end) { /* yjs ignores trailing bytes of an update */ }
    // client table by id (a repeated client block replaces the earlier one in yjs: refused).  yjs writes client blocks
    // in descending order: reversed in one pass; anything else by heapsort (an insertion sort was quadratic: ~5e7
    // moves through global memory for a Tiptap document of 10 000 clients)
    bool desc = true;
    for (uint32_t a = 1; a < n_cl && desc; a++) desc = cl[a - 1].id > cl[a].id;
    if (desc) {
      for (uint32_t a = 0, b = n_cl ? n_cl - 1 : 0; a < b; a++, b--) { const Cli t = cl[a]; cl[a] = cl[b]; cl[b] = t; }
    } else {
      auto sift = [&](uint32_t r, uint32_t m) {   // max-heap by id over cl[0, m)
        for (;;) {
          uint32_t c = 2u * r + 1u;
          if (c >= m) return;
          if (c + 1u < m && cl[c + 1u].id > cl[c].id) c++;
          if (cl[r].id >= cl[c].id) return;
          const Cli t = cl[r]; cl[r] = cl[c]; cl[c] = t;
          r = c;
        }
      };
      for (uint32_t r = n_cl / 2; r-- > 0;) sift(r, n_cl);
      for (uint32_t m = n_cl; m-- > 1;) { const Cli t = cl[0]; cl[0] = cl[m]; cl[m] = t; sift(0, m); }
    }
    for (uint32_t a = 1; a < n_cl; a++) if (cl[a].id == cl[a - 1].id) { fail(ST_UNSUP); return; }
    hint_k = -1;   // (slots moved)
    for (uint32_t h = 0; h <= ch_mask; h++) ch[h] = -1;
    for (uint32_t a = 0; a < n_cl; a++) {
      uint32_t h = cli_hash(cl[a].id) & ch_mask;
      while (ch[h] >= 0) h = (h + 1u) & ch_mask;
      ch[h] = (int32_t)a;
    }
  }

  // ------------------------------------------------------------------ content splice
  YDEV int32_t piece_split(int32_t p, uint32_t t, uint8_t ref) {   // content.splice(t): p keeps [0, t), returns the rest
    Piece& a = pc[p];
    if (ref == 1) { const int32_t r = new_piece(0, 0, a.cnt - t, 0, 0); if (r >= 0) pc[p].cnt = t; return r; }
    if (ref == 4) {   // ContentString.splice (Y@73100): UTF-16 offset, a cut surrogate pair becomes U+FFFD twice
      uint32_t u = a.pre ? 1u : 0u, i = a.off;
      if (a.pre && t == 1) {
        const int32_t r = new_piece(a.off, a.end, a.cnt - 1, 0, a.post);
        if (r >= 0) { pc[p].end = pc[p].off; pc[p].post = 0; pc[p].cnt = 1; }
        return r;
      }
      while (i < a.end && u < t) {
        const uint8_t ch = in[i];
        const uint32_t k = ch < 0x80 ? 1 : (ch & 0xE0) == 0xC0 ? 2 : (ch & 0xF0) == 0xE0 ? 3 : 4;
        if (k == 4 && u + 1 == t) {   // between the two halves of a pair
          const int32_t r = new_piece(i + 4, a.end, a.cnt - t, 1, a.post);
          if (r >= 0) { pc[p].end = i; pc[p].post = 1; pc[p].cnt = t; }
          return r;
        }
        u += k == 4 ? 2u : 1u; i += k;
      }
      const int32_t r = new_piece(i, a.end, a.cnt - t, 0, a.post);   // (i == end with post: the rest is the U+FFFD alone)
      if (r >= 0) { if (i == a.end && a.post && u == t) pc[r].pre = 1, pc[r].post = 0; pc[p].end = i; pc[p].post = 0; pc[p].cnt = t; }
      return r;
    }
    // JSON / Any: element boundary
    Cur q{in, a.off, a.end, 0, 0};
    for (uint32_t e = 0; e < t && !q.err; e++) {
      if (ref == 2) { uint32_t l; q.buf(l); } else any_skip(q);
    }
    if (q.err) { fail(ST_MALFORMED); return -1; }
    const int32_t r = new_piece(q.pos, a.end, a.cnt - t, 0, 0);
    if (r >= 0) { pc[p].end = q.pos; pc[p].cnt = t; }
    return r;
  }

  // splitItem (Y@76300): x keeps [0, diff), returns the right part
  YDEV int32_t split(int32_t x, uint32_t diff) {
    if (n_it >= cap_it) { fail(ST_NOMEM); return -1; }
    if (it[x].ref != 1 && it[x].ref != 2 && it[x].ref != 4 && it[x].ref != 8) { fail(ST_UNSUP); return -1; }
    const int32_t r = (int32_t)n_it++;
    SI& a = it[x]; SI& b = it[r];
    b = a;
    b.clock = a.clock + diff; b.len = a.len - diff;
    b.left = x; b.oc = a.client; b.ok = a.clock + diff - 1; b.flags = (uint8_t)((a.flags & (F_DEL | F_HR | F_INT)) | F_HO);
    b.right = a.right;
    b.ms = b.mr = 0;
    b.p0 = b.p1 = piece_split(a.p0, diff, a.ref);
    if (err) return -1;
    a.right = r;
    if (b.right >= 0) it[b.right].left = r;
    if (b.sub_len >= 0 && b.right < 0 && b.parent >= 0) map_set(b.parent, b.sub_off, (uint32_t)b.sub_len, r);
    a.len = diff;
    b.nxt = a.nxt; a.nxt = r;
    return r;
  }
  YDEV int32_t clean_end(uint32_t client, uint32_t clock) {   // getItemCleanEnd (Y@30000)
    const int32_t x = find(client, clock);
    if (x < 0) return -1;
    if (clock != it[x].clock + it[x].len - 1 && it[x].kind != SK_GC) split(x, clock - it[x].clock + 1);
    return x;
  }
  YDEV int32_t clean_start(uint32_t client, uint32_t clock) {   // getItemCleanStart (Y@29900)
    const int32_t x = find(client, clock);
    if (x < 0) return -1;
    if (it[x].clock < clock && it[x].kind == SK_ITEM) return split(x, clock - it[x].clock);
    return x;
  }

  // ------------------------------------------------------------------ integration
  // Item.getMissing (Y@77700): the client of a missing dependency, or -1 (then left / right / parent set)
  YDEV int64_t get_missing(int32_t x) {
    SI* u = &it[x];
    if ((u->flags & F_HO) && u->oc != u->client && u->ok >= state_of(u->oc)) return u->oc;
    if ((u->flags & F_HR) && u->rc != u->client && u->rk >= state_of(u->rc)) return u->rc;
    if (u->parent == P_ID && u->client != u->pc && u->pk >= state_of(u->pc)) return u->pc;
    if (u->flags & F_HO) {
      const int32_t l = clean_end(u->oc, u->ok);
      u = &it[x];
      u->left = l;
      if (l >= 0) { u->oc = it[l].client; u->ok = it[l].clock + it[l].len - 1; }
    }
    if (u->flags & F_HR) {
      const int32_t r = clean_start(u->rc, u->rk);
      u = &it[x];
      u->right = r;
      if (r >= 0) { u->rc = it[r].client; u->rk = it[r].clock; }
    }
    if (err) return -1;
    const bool lgc = u->left >= 0 && it[u->left].kind == SK_GC, rgc = u->right >= 0 && it[u->right].kind == SK_GC;
    // (a GC origin with an item on the right leaves yjs with an undefined origin id: refused)
    if (lgc && u->right >= 0 && it[u->right].kind == SK_ITEM) { fail(ST_UNSUP); return -1; }
    if (lgc || rgc) u->parent = P_NONE;
    if (u->parent == P_NONE) {   // items with origins take the parent (and key) of a neighbour
      if (u->left >= 0 && it[u->left].kind == SK_ITEM) { u->parent = it[u->left].parent; u->sub_off = it[u->left].sub_off; u->sub_len = it[u->left].sub_len; }
      if (u->right >= 0 && it[u->right].kind == SK_ITEM) { u->parent = it[u->right].parent; u->sub_off = it[u->right].sub_off; u->sub_len = it[u->right].sub_len; }
    } else if (u->parent == P_ID) {
      const int32_t p = find(u->pc, u->pk);
      if (p < 0) return -1;
      if (it[p].kind == SK_GC) u->parent = P_NONE;
      else if (it[p].ref != 7 || it[p].type < 0) { fail(ST_UNSUP); return -1; }
      else u->parent = it[p].type;
    }
    return -1;
  }

  YDEV bool same_origin(uint32_t ha, uint32_t ac, uint32_t ak, uint32_t hb, uint32_t bc, uint32_t bk) const {
    return (!ha && !hb) || (ha && hb && ac == bc && ak == bk);
  }

  YDEV void add_struct(int32_t x) {   // Un (addStruct): the client's state advances
    const int32_t k = cli_slot(it[x].client);
    if (cl[k].ins < 0) cl[k].ins = (int32_t)n_ins++;
    cl[k].state = it[x].clock + it[x].len;
    cl[k].ni = it[x].orig - cl[k].r0 + 1;
    it[x].flags |= F_INT;
  }

  YDEV void integrate(int32_t x) {   // Item.integrate(transaction, 0) (Y@78600)
    SI* u = &it[x];
    if (u->kind == SK_GC || u->parent < 0) {   // GC, or an item without parent: a GC struct
      u->kind = SK_GC;
      add_struct(x);
      return;
    }
    const int32_t P = u->parent;
    const bool sub = u->sub_len >= 0;
    if ((u->left < 0 && (u->right < 0 || it[u->right].left >= 0)) || (u->left >= 0 && it[u->left].right != u->right)) {
      int32_t e = u->left, o;
      if (e >= 0) o = it[e].right;
      else if (sub) { o = map_get(P, u->sub_off, (uint32_t)u->sub_len); while (o >= 0 && it[o].left >= 0) o = it[o].left; }
      else o = ty[P].start;
      const uint32_t eS = ++epoch;   // set s (cleared by bumping)
      uint32_t eR = eS;              // set r (never cleared within this call)
      uint32_t curS = eS;
      while (o >= 0 && o != u->right) {
        it[o].mr = eR; it[o].ms = curS;
        if (same_origin(u->flags & F_HO, u->oc, u->ok, it[o].flags & F_HO, it[o].oc, it[o].ok)) {
          if (it[o].client < u->client) { e = o; curS = ++epoch; }
          else if (same_origin(u->flags & F_HR, u->rc, u->rk, it[o].flags & F_HR, it[o].rc, it[o].rk)) break;
        } else if ((it[o].flags & F_HO)) {
          const int32_t g = find(it[o].oc, it[o].ok);
          if (g < 0) return;
          if (it[g].mr == eR) { if (it[g].ms != curS) { e = o; curS = ++epoch; } }
          else break;
        } else break;
        o = it[o].right;
        u = &it[x];
      }
      u = &it[x];
      u->left = e;
    }
    if (u->left >= 0) { const int32_t r = it[u->left].right; u->right = r; it[u->left].right = x; }
    else {
      int32_t r;
      if (sub) { r = map_get(P, u->sub_off, (uint32_t)u->sub_len); while (r >= 0 && it[r].left >= 0) r = it[r].left; }
      else { r = ty[P].start; ty[P].start = x; }
      u->right = r;
    }
    if (u->right >= 0) it[u->right].left = x;
    else if (sub) {
      map_set(P, u->sub_off, (uint32_t)u->sub_len, x);
      u = &it[x];
      if (u->left >= 0) item_delete(u->left);
    }
    add_struct(x);
    u = &it[x];
    // content.integrate
    if (u->ref == 1) { tx_add(u->client, u->clock, u->len); u->flags |= F_DEL; }
    else if (u->ref == 7) { const int32_t t = new_type(x, 0, 0); it[x].type = t; }
    u = &it[x];
    const int32_t pi = ty[P].item;
    if ((pi >= 0 && (it[pi].flags & F_DEL)) || (sub && u->right >= 0)) item_delete(x);
  }

  // Item.delete (Y@80200) with ContentType.delete (Y@73600): an explicit stack instead of recursion
  YDEV void item_delete(int32_t x0) {
    uint32_t sp = 0;
    st[sp++] = x0;
    while (sp && !err) {
      const int32_t x = st[--sp];
      if (it[x].kind != SK_ITEM || (it[x].flags & F_DEL)) continue;
      it[x].flags |= F_DEL;
      tx_add(it[x].client, it[x].clock, it[x].len);
      if (it[x].ref == 7 && it[x].type >= 0) {
        const int32_t t = it[x].type;
        // (pushed in reverse so the list is deleted front to back, as the reference walks it)
        uint32_t base = sp;
        for (int32_t c = ty[t].start; c >= 0; c = it[c].right)
          if (!(it[c].flags & F_DEL) && it[c].kind == SK_ITEM) { if (sp >= cap_st) { fail(ST_NOMEM); return; } st[sp++] = c; }
        for (int32_t e = ty[t].map; e >= 0; e = me[e].next) {
          const int32_t c = me[e].item;
          if (c >= 0 && it[c].kind == SK_ITEM && !(it[c].flags & F_DEL)) { if (sp >= cap_st) { fail(ST_NOMEM); return; } st[sp++] = c; }
        }
        for (uint32_t a = base, b = sp - 1; a < b && sp > base; a++, b--) { const int32_t tmp = st[a]; st[a] = st[b]; st[b] = tmp; }
      }
    }
  }

  // integrateStructs (Y@21000 Me): highest client first, a dependency stack.  A struct past its client's state (a gap)
  // or one whose dependency's client has no refs left walls the stack: every struct on it goes to the pending set
  // (addStackToRestSS): a client still on the map gives the slice of its refs from its cursor (one back) and leaves the
  // map; a client already off it gives that one struct (replacing what it gave before).  Skips are passed over.
  YDEV void rest_stack(uint32_t& sp, int32_t* stk) {
    for (uint32_t i = 0; i < sp; i++) {
      const int32_t t = stk[i];
      const int32_t k = cli_slot(it[t].client);
      if (!cl[k].gone) {
        cl[k].ri--;
        cl[k].rest0 = cl[k].r0 + cl[k].ri; cl[k].restn = cl[k].rn - cl[k].ri;
        cl[k].gone = 1; cl[k].ri = cl[k].rn;   // (refs emptied: its cursor at the end)
      } else { cl[k].rest0 = t; cl[k].restn = 1; }
    }
    sp = 0;
  }
  YDEV void integrate_all() {
    for (uint32_t k = 0; k < n_cl; k++) cl[k].ri = 0;
    int32_t ci = (int32_t)n_cl - 1;   // current client (ascending table, taken from the end)
    auto next_client = [&]() -> int32_t {
      while (ci >= 0 && (cl[ci].gone || cl[ci].ri >= cl[ci].rn)) ci--;
      return ci;
    };
    int32_t cur = next_client();
    if (cur < 0) return;
    int32_t u = cl[cur].r0 + cl[cur].ri++;
    uint32_t sp = 0;   // the reference's stack `s`
    int32_t* stk = seq;   // (seq is free until the merge pass)
    for (;;) {
      if (err) return;
      if (it[u].kind != SK_SKIP) {
        const int32_t k = cli_slot(it[u].client);
        const int64_t diff = (int64_t)cl[k].state - (int64_t)it[u].clock;
        if (diff < 0) {   // a gap: the struct and the stack go pending
          if (sp >= cap_seq) { fail(ST_NOMEM); return; }
          stk[sp++] = u;
          rest_stack(sp, stk);
        } else {
          const int64_t m = get_missing(u);
          if (err) return;
          if (m >= 0) {
            if (sp >= cap_seq) { fail(ST_NOMEM); return; }
            stk[sp++] = u;
            const int32_t mk = cli_slot((uint32_t)m);
            if (mk < 0 || cl[mk].gone || cl[mk].ri >= cl[mk].rn) rest_stack(sp, stk);   // the dependency is not in the update
            else { u = cl[mk].r0 + cl[mk].ri++; continue; }
          } else if (diff == 0) integrate(u);
          else if (diff < (int64_t)it[u].len) { fail(ST_UNSUP); return; }   // overlapping structs (integrate with an offset)
          // (else: every clock of it is integrated already)
        }
      }
      if (sp) u = stk[--sp];
      else if (cur >= 0 && !cl[cur].gone && cl[cur].ri < cl[cur].rn) u = cl[cur].r0 + cl[cur].ri++;
      else {
        cur = next_client();
        if (cur < 0) break;
        u = cl[cur].r0 + cl[cur].ri++;
      }
    }
    for (uint32_t k = 0; k < n_cl; k++) n_rest += cl[k].restn > 0 ? 1u : 0u;
  }

  YDEV void pds_add(uint32_t client, uint32_t clock, uint32_t len) {   // addToDeleteSet on the pending set (one per input range)
    Rng& r = pds[n_pds++];
    r.client = client; r.clock = clock; r.len = len; r.pad = 0;
  }
  // readAndApplyDeleteSet (Y@11500): split at range ends, delete; ranges past the state are pending
  YDEV void apply_ds() {
    for (uint32_t r = 0; r < n_dsin && !err; r++) {
      const uint32_t client = dsin[r].client, a = dsin[r].clock, b = dsin[r].clock + dsin[r].len;
      const uint32_t s = state_of(client);
      if (!(a < s)) { pds_add(client, a, b - a); continue; }   // past the state: pending
      if (s < b) pds_add(client, s, b - s);                    // its part past the state: pending
      int32_t x = find(client, a);
      if (x < 0) return;
      if (!deleted(x) && it[x].clock < a) { split(x, a - it[x].clock); x = it[x].nxt; }
      while (x >= 0 && !err) {
        if (it[x].clock < b) {
          if (!deleted(x)) {
            if (b < it[x].clock + it[x].len) split(x, b - it[x].clock);
            item_delete(x);
          }
        } else break;
        x = next_part(x);
      }
    }
  }

  // cleanupTransactions, gc branch (Y@30900 tryGcDeleteSet): deleted items -> ContentDeleted, their
  // children (ContentType.gc, Y@73900) -> GC structs
  YDEV void gc_item(int32_t x0, bool parent_gcd) {
    uint32_t sp = 0;
    st[sp++] = x0 * 2 + (parent_gcd ? 1 : 0);
    while (sp && !err) {
      const int32_t v = st[--sp], x = v >> 1;
      const bool pg = v & 1;
      if (it[x].kind == SK_GC) continue;
      if (!(it[x].flags & F_DEL)) { fail(ST_UNSUP); return; }   // yjs throws unexpectedCase
      if (it[x].ref == 7 && it[x].type >= 0) {
        const int32_t t = it[x].type;
        for (int32_t c = ty[t].start; c >= 0; c = it[c].right) { if (sp >= cap_st) { fail(ST_NOMEM); return; } st[sp++] = c * 2 + 1; }
        for (int32_t e = ty[t].map; e >= 0; e = me[e].next)
          for (int32_t c = me[e].item; c >= 0; c = it[c].left) { if (sp >= cap_st) { fail(ST_NOMEM); return; } st[sp++] = c * 2 + 1; }
        ty[t].start = -1; ty[t].map = -1;
      }
      if (pg) it[x].kind = SK_GC;   // replaceStruct(new GC)
      else {                        // content = new ContentDeleted(length)
        it[x].ref = 1;
        it[x].p0 = it[x].p1 = new_piece(0, 0, it[x].len, 0, 0);
      }
    }
  }
  YDEV void gc_pass() {
    for (uint32_t r = 0; r < n_tx && !err; r++) {
      const uint32_t a = tx[r].clock, b = tx[r].clock + tx[r].len;
      int32_t x = find(tx[r].client, a);
      while (x >= 0 && it[x].clock < b && !err) {
        if (it[x].kind == SK_ITEM && (it[x].flags & F_DEL)) gc_item(x, false);
        x = next_part(x);
      }
    }
  }

  // tryToMergeWithLeft over every client (Y@31000 Yn, Item.mergeWith Y@79900, GC.mergeWith)
  YDEV bool mergeable(int32_t a, int32_t b) const {
    const SI& L = it[a]; const SI& R = it[b];
    if (deleted(a) != deleted(b) || L.kind != R.kind) return false;
    if (L.kind == SK_GC) return true;
    if (!((R.flags & F_HO) && R.oc == L.client && R.ok == L.clock + L.len - 1)) return false;
    if (L.right != b) return false;
    if (!same_origin(L.flags & F_HR, L.rc, L.rk, R.flags & F_HR, R.rc, R.rk)) return false;
    if (L.clock + L.len != R.clock) return false;
    if (L.ref != R.ref) return false;
    return L.ref == 1 || L.ref == 2 || L.ref == 4 || L.ref == 8;
  }
  YDEV void absorb(int32_t a, int32_t b) {
    SI& L = it[a]; SI& R = it[b];
    if (L.kind == SK_ITEM) {
      L.right = R.right;
      if (L.right >= 0) it[L.right].left = a;
      if (L.ref == 1) pc[L.p0].cnt += R.len;
      else { pc[L.p1].next = R.p0; L.p1 = R.p1; }
    }
    L.len += R.len;
    R.flags |= F_GONE;
  }
  YDEV uint32_t client_seq(uint32_t k) {   // the client's structs in clock order -> seq[]
    uint32_t m = 0;
    for (int32_t o = cl[k].r0; o < cl[k].r0 + cl[k].ni; o++)
      for (int32_t x = o; x >= 0; x = it[x].nxt)
        if (!(it[x].flags & F_GONE)) { if (m >= cap_seq) { fail(ST_NOMEM); return 0; } seq[m++] = x; }
    return m;
  }
  YDEV void merge_pass() {
    for (uint32_t k = 0; k < n_cl && !err; k++) {
      const uint32_t m = client_seq(k);
      for (uint32_t e = m; e-- > 1;) if (mergeable(seq[e - 1], seq[e])) absorb(seq[e - 1], seq[e]);
    }
  }

  // ------------------------------------------------------------------ encodeStateAsUpdate (Y@23300)
  YDEV void w(OutCap& o, uint32_t a, uint32_t l) { o.copy(in + a, l); }
  YDEV void write_item(OutCap& o, int32_t x) {
    const SI& u = it[x];
    if (u.kind == SK_GC) { o.b(0); o.vu(u.len); return; }
    const bool ho = u.flags & F_HO, hr = u.flags & F_HR, hs = u.sub_len >= 0;
    o.b((uint8_t)((u.ref & 31) | (ho ? 0x80 : 0) | (hr ? 0x40 : 0) | (hs ? 0x20 : 0)));
    if (ho) { o.vu(u.oc); o.vu(u.ok); }
    if (hr) { o.vu(u.rc); o.vu(u.rk); }
    if (!ho && !hr) {
      if (u.parent == P_ID) { o.b(0); o.vu(u.pc); o.vu(u.pk); }   // (a pending item: its parent id as read)
      else {
        const TypeRec& t = ty[u.parent];
        if (t.item < 0) { o.b(1); o.vu(t.name_len); w(o, t.name_off, t.name_len); }
        else { o.b(0); o.vu(it[t.item].client); o.vu(it[t.item].clock); }
      }
      if (hs) { o.vu((uint32_t)u.sub_len); w(o, u.sub_off, (uint32_t)u.sub_len); }
    }
    switch (u.ref) {
      case 1: o.vu(u.len); break;
      case 4: {
        uint32_t nb = 0;
        for (int32_t p = u.p0; p >= 0; p = pc[p].next) nb += pc[p].end - pc[p].off + 3u * (pc[p].pre + pc[p].post);
        o.vu(nb);
        for (int32_t p = u.p0; p >= 0; p = pc[p].next) {
          if (pc[p].pre) { o.b(0xEF); o.b(0xBF); o.b(0xBD); }
          w(o, pc[p].off, pc[p].end - pc[p].off);
          if (pc[p].post) { o.b(0xEF); o.b(0xBF); o.b(0xBD); }
        }
        break;
      }
      case 2: case 8: {
        o.vu(u.len);
        for (int32_t p = u.p0; p >= 0; p = pc[p].next) w(o, pc[p].off, pc[p].end - pc[p].off);
        break;
      }
      default: w(o, u.c_start, u.c_end - u.c_start);   // Binary / Embed / Format / Type: as read (canonical)
    }
  }
  YDEV void encode_state(OutCap& o) {
    uint32_t nc = 0;
    for (uint32_t k = 0; k < n_cl; k++) nc += cl[k].ni > 0 ? 1u : 0u;
    o.vu(nc);
    for (uint32_t kk = n_cl; kk-- > 0;) {   // clients descending
      if (!cl[kk].ni) continue;
      const uint32_t m = client_seq(kk);
      o.vu(m); o.vu(cl[kk].id); o.vu(it[seq[0]].clock);
      for (uint32_t i = 0; i < m; i++) write_item(o, seq[i]);
      if (o.n + 64u > o.cap) { fail(ST_NOMEM); return; }
    }
    // delete set from the struct store (createDeleteSetFromStructStore, Y@10600): store insertion order
    // (13.5 writeDeleteSet keeps the Map order; 13.6 sorts clients descending)
    uint32_t nds = 0;
    for (uint32_t k = 0; k < n_cl; k++) {
      if (!cl[k].ni) continue;
      const uint32_t m = client_seq(k);
      for (uint32_t i = 0; i < m; i++) if (deleted(seq[i])) { nds++; break; }
    }
    o.vu(nds);
    for (uint32_t r = 0; r < n_cl; r++) {
      int32_t k = -1;
      if (flags & F_COMPAT_135) { for (uint32_t j = 0; j < n_cl; j++) if (cl[j].ins == (int32_t)r) k = (int32_t)j; }
      else k = (int32_t)(n_cl - 1 - r);
      if (k < 0 || !cl[k].ni) continue;
      const uint32_t m = client_seq((uint32_t)k);
      uint32_t runs = 0;
      for (uint32_t i = 0; i < m; i++) if (deleted(seq[i]) && (i == 0 || !deleted(seq[i - 1]))) runs++;
      if (!runs) continue;
      o.vu(cl[k].id); o.vu(runs);
      for (uint32_t i = 0; i < m;) {
        if (!deleted(seq[i])) { i++; continue; }
        const uint32_t c0 = it[seq[i]].clock; uint32_t len = 0;
        while (i < m && deleted(seq[i])) len += it[seq[i++]].len;
        o.vu(c0); o.vu(len);
      }
      if (o.n + 64u > o.cap) { fail(ST_NOMEM); return; }
    }
  }
  // the pending delete set as encodeStateAsUpdate merges it (pendingDs converted to V1): no structs, then the ranges
  // by client in first-seen order (addToDeleteSet's Map), each client's in input order
  YDEV void encode_pds(OutCap& o) {
    o.vu(0);
    if (n_pds > 4096u) { fail(ST_UNSUP); return; }   // (the first-seen grouping below is quadratic)
    auto first = [&](uint32_t i) { for (uint32_t j = 0; j < i; j++) if (pds[j].client == pds[i].client) return false; return true; };
    uint32_t nc = 0;
    for (uint32_t i = 0; i < n_pds; i++) nc += first(i) ? 1u : 0u;
    o.vu(nc);
    for (uint32_t i = 0; i < n_pds; i++) {
      if (!first(i)) continue;
      uint32_t cnt = 0;
      for (uint32_t j = i; j < n_pds; j++) cnt += pds[j].client == pds[i].client ? 1u : 0u;
      o.vu(pds[i].client); o.vu(cnt);
      for (uint32_t j = i; j < n_pds; j++) if (pds[j].client == pds[i].client) { o.vu(pds[j].clock); o.vu(pds[j].len); }
    }
  }
  // the pending structs as encodeStateAsUpdate merges them: diffUpdate(pendingStructs.update, [0]) converted to V1 --
  // clients descending (writeClientsStructs), a client's leading Skips dropped (diffUpdate), every struct as written
  // by Item.write at offset 0 from what was read (never integrated: origins, parent id / key as read), no delete set
  YDEV void encode_rest(OutCap& o) {
    auto lead = [&](uint32_t k) {   // the client's first pending struct that is not a Skip (rest0 + restn: none)
      int32_t x = cl[k].rest0;
      while (x < cl[k].rest0 + cl[k].restn && it[x].kind == SK_SKIP) x++;
      return x;
    };
    uint32_t nc = 0;
    for (uint32_t k = 0; k < n_cl; k++) nc += (cl[k].restn && lead(k) < cl[k].rest0 + cl[k].restn) ? 1u : 0u;
    o.vu(nc);
    for (uint32_t kk = n_cl; kk-- > 0;) {
      if (!cl[kk].restn) continue;
      const int32_t x0 = lead(kk), x1 = cl[kk].rest0 + cl[kk].restn;
      if (x0 >= x1) continue;
      o.vu((uint32_t)(x1 - x0)); o.vu(cl[kk].id); o.vu(it[x0].clock);
      for (int32_t x = x0; x < x1; x++) {
        if (it[x].kind == SK_SKIP) { o.b(10); o.vu(it[x].len); }
        else write_item(o, x);
      }
      if (o.n + 64u > o.cap) { fail(ST_NOMEM); return; }
    }
    o.vu(0);
  }
  YDEV uint32_t encode() {
    if ((!n_rest && !n_pds) || (flags & F_SNAP_STATE)) {
      OutCap o{out, 0, cap_out};
      encode_state(o);
      if (err) return 0;
      if (o.n > cap_out) { fail(ST_NOMEM); return 0; }
      return o.n;
    }
    // pending: PendHdr, then the state, the pending delete set and the pending structs (each the empty update if absent)
    if (cap_out < sizeof(PendHdr) + 64u) { fail(ST_NOMEM); return 0; }
    PendHdr h;
    OutCap o{out + sizeof(PendHdr), 0, cap_out - (uint32_t)sizeof(PendHdr)};
    encode_state(o); h.len[0] = o.n;
    if (n_pds) encode_pds(o); else { o.b(0); o.b(0); }
    h.len[1] = o.n - h.len[0];
    if (n_rest) encode_rest(o); else { o.b(0); o.b(0); }
    h.len[2] = o.n - h.len[0] - h.len[1];
    if (err) return 0;
    if (o.n > o.cap) { fail(ST_NOMEM); return 0; }
    h.magic = PEND_MAGIC;
    const uint8_t* hb = (const uint8_t*)&h;
    for (uint32_t i = 0; i < sizeof(PendHdr); i++) out[i] = hb[i];
    pend = true;
    return (uint32_t)sizeof(PendHdr) + o.n;
  }

  YDEV uint32_t run() {
    parse();
    if (!err) integrate_all();
    if (!err) apply_ds();
    if (!err) gc_pass();
    if (!err) merge_pass();
    return err ? 0u : encode();
  }
};

// carves a workspace (ws, ws_core_bytes(caps)) and runs the document, writing at most out_cap bytes at out
YDEV_NI int snapshot_run(const uint8_t* in, uint32_t n, uint32_t flags, uint8_t* ws, const Caps& k, uint8_t* out, uint32_t out_cap,
                         uint32_t& out_len) {
  Doc D;
  uint8_t* p = ws;
  D.in = in; D.n = n; D.flags = flags; D.err = 0; D.epoch = 0; D.n_ins = 0; D.hint_id = 0; D.hint_k = -1; D.pend = false;
  D.n_pds = 0; D.n_rest = 0;
  D.it = (SI*)p; D.n_it = 0; D.cap_it = k.it; p += al16((uint64_t)k.it * sizeof(SI));
  D.pc = (Piece*)p; D.n_pc = 0; D.cap_pc = k.pc; p += al16((uint64_t)k.pc * sizeof(Piece));
  D.ty = (TypeRec*)p; D.n_ty = 0; D.cap_ty = k.ty; p += al16((uint64_t)k.ty * sizeof(TypeRec));
  D.me = (MapEnt*)p; D.n_me = 0; D.cap_me = k.me; p += al16((uint64_t)k.me * sizeof(MapEnt));
  D.cl = (Cli*)p; D.n_cl = 0; D.cap_cl = k.cl; p += al16((uint64_t)k.cl * sizeof(Cli));
  D.tx = (Rng*)p; D.n_tx = 0; D.cap_tx = k.tx; p += al16((uint64_t)k.tx * sizeof(Rng));
  D.dsin = (Rng*)p; D.n_dsin = 0; D.cap_dsin = k.dsin; p += al16((uint64_t)k.dsin * sizeof(Rng));
  D.pds = (Rng*)p; p += al16((uint64_t)k.dsin * sizeof(Rng));
  D.st = (int32_t*)p; D.cap_st = k.st; p += al16(4ull * k.st);
  D.seq = (int32_t*)p; D.cap_seq = k.seq; p += al16(4ull * k.seq);
  D.ch = (int32_t*)p; D.ch_mask = k.hc - 1u;
  D.out = out; D.cap_out = out_cap;
  out_len = D.run();
  return D.err ? D.err : D.pend ? ST_PEND : 0;
}
// document d's workspace from caps_of, its output region at the end
YDEV int snapshot_doc(const uint8_t* in, uint32_t n, uint32_t flags, uint8_t* ws, const Caps& k, uint32_t& out_off, uint32_t& out_len) {
  out_off = (uint32_t)ws_core_bytes(k);
  return snapshot_run(in, n, flags, ws, k, ws + out_off, k.out, out_len);
}

}  // namespace snap
}  // namespace ygm
