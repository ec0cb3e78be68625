// ygm_seqdoc.hpp -- per-document (one lane = one document) algorithms:
//   * encodeStateVectorFromUpdate  (yjs Y@37728, rule R-SV)
//   * diffUpdate                   (yjs Y@40711, rule R-D,  SURVEY.md App. B.2)
//   * delete-set read/write helpers (Y@11346 readDeleteSet, Y@11105 writeDeleteSet)
// Each runs twice per document: a size pass (Out.p == nullptr) and a write
// pass at the offset the decoupled look-back assigned.
#pragma once
#include "ygm_v1.hpp"

namespace ygm {

// Sequential struct stream over one update (LazyStructReader with filterSkips=false).
struct Stream {
  Cur c;
  uint64_t blocks_left, structs_left, client, clock;
  bool has;
  SInfo cur;
  uint64_t cur_client, cur_clock;
  uint32_t flags;
  YDEV void init(const uint8_t* p, uint32_t n, uint32_t f) {
    c = Cur{p, 0, n, 0, 0};
    flags = f;
    structs_left = 0; client = 0; clock = 0; has = false;
    blocks_left = c.vu();
    next();
  }
  YDEV void next() {
    has = false;
    if (c.err) return;
    while (structs_left == 0) {
      if (blocks_left == 0) return;
      blocks_left--;
      structs_left = c.vu();
      client = c.vu();
      clock = c.vu();
      if (c.err) return;
    }
    structs_left--;
    read_struct_fast(c, cur, flags);
    if (c.err) return;
    if (clock + cur.len > MAX_SAFE) { c.fail(ST_RANGE); return; }
    cur_client = client; cur_clock = clock;
    clock += cur.len;
    has = true;
  }
};

// ---------------------------------------------------------------- SV
// Returns status; o.n = output size.  `count` is computed in the size pass and
// consumed by the write pass (the varuint count precedes the entries).
YDEV_NI int sv_doc(const uint8_t* p, uint32_t n, uint32_t flags, Out& o, uint64_t& count, bool write) {
  Stream s; s.init(p, n, flags);
  if (s.c.err) return s.c.err;
  uint64_t size = 0;
  Out body{write ? o.p : nullptr, 0};
  if (write) { o.vu(count); body.p = o.p + o.n; }
  if (s.has) {
    uint64_t cc = s.cur_client;
    bool stop = s.cur_clock != 0;
    uint64_t clk = stop ? 0 : s.cur_clock + s.cur.len;
    while (s.has) {
      if (cc != s.cur_client) {
        if (clk != 0) { size++; body.vu(cc); body.vu(clk); }
        cc = s.cur_client; clk = 0; stop = s.cur_clock != 0;
      }
      if (s.cur.kind == K_SKIP) stop = true;
      if (!stop) clk = s.cur_clock + s.cur.len;
      s.next();
      if (s.c.err) return s.c.err;
    }
    if (clk != 0) { size++; body.vu(cc); body.vu(clk); }
  }
  if (!write) { count = size; o.n = vu_len(size) + body.n; }
  else o.n += body.n;
  return ST_OK;
}

// ---------------------------------------------------------------- delete sets
// DS entries are read in place; clients with 0 ranges are dropped and repeated
// clients are merged into their first non-empty entry (Map semantics of
// readDeleteSet).  Output order: client-descending (yjs 13.6 writeDeleteSet) or
// first-seen (13.5 compat).  O(C^2) client scans: delete sets are small.
YDEV_NI bool ds_seen_before(const uint8_t* p, uint32_t dstart, uint32_t dend, uint32_t upto, uint64_t client);
// validates the DS at c and counts its distinct clients with >= 1 range
YDEV_NI int ds_validate(Cur c, uint64_t& nclients_out) {
  const uint32_t dstart = c.pos;
  const uint64_t n = c.vu();
  uint64_t distinct = 0;
  for (uint64_t i = 0; i < n && !c.err; i++) {
    const uint32_t at = c.pos;
    const uint64_t cl = c.vu(); const uint64_t nd = c.vu();
    for (uint64_t k = 0; k < nd && !c.err; k++) { c.vu(); c.vu(); }
    if (!c.err && nd > 0 && !ds_seen_before(c.p, dstart, c.end, at, cl)) distinct++;
  }
  nclients_out = distinct;
  return c.err;
}
// entry i: position of its client varuint (after the count)
YDEV_NI bool ds_seen_before(const uint8_t* p, uint32_t dstart, uint32_t dend, uint32_t upto, uint64_t client) {
  Cur c{p, dstart, dend, 0, 0};
  const uint64_t n = c.vu();
  for (uint64_t i = 0; i < n && !c.err; i++) {
    if (c.pos >= upto) return false;
    const uint64_t cl = c.vu(); const uint64_t nd = c.vu();
    if (nd > 0 && cl == client) return true;
    for (uint64_t k = 0; k < nd && !c.err; k++) { c.vu(); c.vu(); }
  }
  return false;
}
// writes all ranges of `client` in entry order; returns number of ranges
YDEV_NI uint64_t ds_client_ranges(const uint8_t* p, uint32_t dstart, uint32_t dend, uint64_t client, Out* o) {
  Cur c{p, dstart, dend, 0, 0};
  const uint64_t n = c.vu(); uint64_t cnt = 0;
  for (uint64_t i = 0; i < n && !c.err; i++) {
    const uint64_t cl = c.vu(); const uint64_t nd = c.vu();
    for (uint64_t k = 0; k < nd && !c.err; k++) {
      const uint64_t a = c.vu(), b = c.vu();
      if (cl == client) { cnt++; if (o) { o->vu(a); o->vu(b); } }
    }
  }
  return cnt;
}
// readDeleteSet + writeDeleteSet (unsorted ranges) of the DS at [dstart, dend)
YDEV_NI void ds_copy(const uint8_t* p, uint32_t dstart, uint32_t dend, uint64_t nclients, uint32_t flags, Out& o) {
  o.vu(nclients);
  if (nclients == 0) return;
  if (flags & F_COMPAT_135) {  // first-seen order
    Cur c{p, dstart, dend, 0, 0};
    const uint64_t n = c.vu();
    for (uint64_t i = 0; i < n && !c.err; i++) {
      const uint32_t at = c.pos;
      const uint64_t cl = c.vu(); const uint64_t nd = c.vu();
      for (uint64_t k = 0; k < nd && !c.err; k++) { c.vu(); c.vu(); }
      if (nd == 0 || ds_seen_before(p, dstart, dend, at, cl)) continue;
      o.vu(cl);
      o.vu(ds_client_ranges(p, dstart, dend, cl, nullptr));
      ds_client_ranges(p, dstart, dend, cl, &o);
    }
    return;
  }
  // client-descending: repeatedly take the largest client below the previous one
  uint64_t prev = ~0ull; bool first = true;
  for (uint64_t q = 0; q < nclients; q++) {
    Cur c{p, dstart, dend, 0, 0};
    const uint64_t n = c.vu();
    bool found = false; uint64_t best = 0;
    for (uint64_t i = 0; i < n && !c.err; i++) {
      const uint64_t cl = c.vu(); const uint64_t nd = c.vu();
      for (uint64_t k = 0; k < nd && !c.err; k++) { c.vu(); c.vu(); }
      if (nd == 0) continue;
      if ((first || cl < prev) && (!found || cl > best)) { best = cl; found = true; }
    }
    if (!found) break;
    o.vu(best);
    o.vu(ds_client_ranges(p, dstart, dend, best, nullptr));
    ds_client_ranges(p, dstart, dend, best, &o);
    prev = best; first = false;
  }
}

// ---------------------------------------------------------------- diff
// decodeStateVector lookup: last entry for `client` wins (Map.set)
YDEV uint64_t sv_lookup(const uint8_t* sv, uint32_t svn, uint64_t client) {
  Cur c{sv, 0, svn, 0, 0};
  const uint64_t n = c.vu(); uint64_t r = 0;
  for (uint64_t i = 0; i < n && !c.err; i++) { const uint64_t cl = c.vu(), k = c.vu(); if (cl == client) r = k; }
  return r;
}
YDEV int sv_validate(const uint8_t* sv, uint32_t svn) {
  Cur c{sv, 0, svn, 0, 0};
  const uint64_t n = c.vu();
  for (uint64_t i = 0; i < n && !c.err; i++) { c.vu(); c.vu(); }
  return c.err;
}

// The diffUpdateV2 loop (Y@40711) as an event generator: each event is one
// writeStructToLazyStructWriter(struct, offset) call.
struct DiffGen {
  Stream s;
  const uint8_t* sv; uint32_t svn;
  int mode;  // 0 top, 1 write rest of client, 2 skip covered
  uint64_t run_client, svclock;
  YDEV void init(const uint8_t* p, uint32_t n, const uint8_t* svp, uint32_t svlen, uint32_t flags) {
    s.init(p, n, flags); sv = svp; svn = svlen; mode = 0; run_client = 0; svclock = 0;
  }
  // returns false at end (or on error: check s.c.err)
  YDEV bool next(SInfo& ev, uint64_t& client, uint64_t& clock, uint64_t& off) {
    for (;;) {
      if (s.c.err || !s.has) return false;
      if (mode == 0) {
        const uint64_t cl = s.cur_client;
        const uint64_t svc = sv_lookup(sv, svn, cl);
        if (s.cur.kind == K_SKIP) { s.next(); continue; }
        if (s.cur_clock + s.cur.len > svc) {
          ev = s.cur; client = cl; clock = s.cur_clock; off = svc > s.cur_clock ? svc - s.cur_clock : 0;
          run_client = cl; mode = 1;
          s.next();
          return true;
        }
        run_client = cl; svclock = svc; mode = 2;
        continue;
      }
      if (mode == 1) {
        if (s.cur_client == run_client) { ev = s.cur; client = s.cur_client; clock = s.cur_clock; off = 0; s.next(); return true; }
        mode = 0; continue;
      }
      if (s.cur_client == run_client && s.cur_clock + s.cur.len <= svclock) { s.next(); continue; }
      mode = 0;
    }
  }
};

// blk[]: per-lane scratch (LDS) recording each output block's struct count in
// the size pass; blocks beyond `blk_cap` are counted again by look-ahead in
// the write pass.
YDEV_NI int diff_doc(const uint8_t* p, uint32_t n, const uint8_t* sv, uint32_t svn, uint32_t flags, Out& o,
                  bool write, uint64_t& nblocks, uint32_t* blk, int blk_cap) {
  int e = sv_validate(sv, svn);
  if (e) return e;
  DiffGen g; g.init(p, n, sv, svn, flags);
  if (g.s.c.err) return g.s.c.err;
  bool nc = false;
  if (write) o.vu(nblocks);
  uint64_t written = 0, wclient = 0, bi = 0;
  SInfo ev; uint64_t cl, ck, off;
  while (g.next(ev, cl, ck, off)) {
    if (written > 0 && wclient != cl) {
      if (!write && bi < (uint64_t)blk_cap) blk[bi] = (uint32_t)written;
      bi++; written = 0;
    }
    if (written == 0) {
      wclient = cl;
      uint64_t cnt;
      if (!write) cnt = 1;  // header size needs the count: patched below
      else if (bi < (uint64_t)blk_cap) cnt = blk[bi];
      else {  // look-ahead: count events until the writer would flush
        DiffGen h = g; cnt = 1;
        SInfo e2; uint64_t c2, k2, o2;
        while (h.next(e2, c2, k2, o2) && c2 == cl) cnt++;
      }
      if (write) { o.vu(cnt); o.vu(cl); o.vu(ck + off); }
      else { o.vu(cl); o.vu(ck + off); }  // count varuint added when the block closes
    }
    const int we = write_struct(o, p, ev, cl, ck, off, false, flags);
    if (we == ST_NONCANON) nc = true;  // reported after the rest has been validated
    else if (we) return we;
    written++;
  }
  if (g.s.c.err) return g.s.c.err;
  if (written > 0) { if (!write && bi < (uint64_t)blk_cap) blk[bi] = (uint32_t)written; bi++; }
  if (!write) {
    nblocks = bi;
    // add the varuint sizes of every block count and of the block total
    uint64_t extra = vu_len(bi);
    if (bi <= (uint64_t)blk_cap) { for (uint64_t i = 0; i < bi; i++) extra += vu_len(blk[i]); }
    else {  // recount block sizes by replay (rare: more blocks than scratch)
      DiffGen h; h.init(p, n, sv, svn, flags);
      uint64_t wr = 0, wc = 0; SInfo e2; uint64_t c2, k2, o2;
      while (h.next(e2, c2, k2, o2)) {
        if (wr > 0 && wc != c2) { extra += vu_len(wr); wr = 0; }
        if (wr == 0) wc = c2;
        wr++;
      }
      if (wr > 0) extra += vu_len(wr);
    }
    o.n += (uint32_t)extra;
  }
  // delete set: readDeleteSet + writeDeleteSet
  const uint32_t dstart = g.s.c.pos;
  uint64_t ncl;
  e = ds_validate(Cur{p, dstart, n, 0, 0}, ncl);
  if (e) return e;
  if (nc) return ST_NONCANON;
  ds_copy(p, dstart, n, ncl, flags, o);
  return ST_OK;
}

}  // namespace ygm
