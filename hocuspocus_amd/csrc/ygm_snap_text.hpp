// ygm_snap_text.hpp -- the doc-normalized snapshot of ygm_snapshot.hpp (SURVEY.md §8f-1,
// encodeStateAsUpdate(applyUpdate(new Doc, u))) for documents of flat text, over a compact workspace that fits in
// LDS next to the document's bytes.
//
// Why: the general kernel's integration is a serial chain of dependent accesses into a per-document workspace in
// global memory (≈ 1 µs a step; a 160-struct document takes ≈ 10 ms however many documents run beside it).  Here
// the same steps run on 26-byte part records in LDS.
//
// Envelope (anything else returns false and the document goes to the general kernel, which decides its status):
// Items with ContentDeleted / ASCII ContentString only (no GC, Skip, types, maps, embeds), items without origins
// under one root type named in the update (no parent ids, no parentSub), <= 16 client blocks (distinct), every
// client's clocks < 2^16, input < 64 KiB, the parts (input structs + splits) within the workspace, an update that
// integrates completely (no pending structs or delete set).  Inside it every step is ygm_snapshot.hpp's (cited
// there against yjs 13.5.16), specialised:
//   * parts: the struct store's items and their split parts (Doc::it), ids of origins as (client slot, clock);
//   * one root type: its list head (TypeRec::start); no nested types, so Item.delete is a flag and the GC of a
//     deleted item (tryGcDeleteSet) turns its content into ContentDeleted -- done for every deleted part at once
//     (every deleted part lies in a range the transaction's delete set recorded);
//   * ASCII content: a part's bytes are its input slice [coff, coff + len); a split cuts the slice at the clock
//     offset, and a merged part's bytes are its own slice followed by those of the parts it absorbed (they follow
//     it in the client's clock order), so no piece lists.
#pragma once
#include "ygm_snapshot.hpp"

namespace ygm {
namespace snapt {

#ifdef YGM_HOST_BUILD
#define YSN_CONST
#else
#define YSN_CONST __attribute__((address_space(4)))   // the input is read-only for the kernel: scalar-cache loads
#endif
typedef const YSN_CONST uint32_t* InW;

constexpr uint16_t NIL = 0xFFFFu;
constexpr uint32_t CMAX = 16;
enum : uint8_t { T_HO = 1, T_HR = 2, T_DEL = 4, T_INT = 8, T_GONE = 16, T_STR = 32 };

struct P {                         // a part: Doc::SI for flat text (26 bytes)
  uint16_t clock, len, ok, rk;     // id clock and length, origin / right origin clocks
  uint16_t left, right, nxt, orig; // document list, next split part, input struct
  uint16_t coff, ms, mr;           // own ASCII slice start (its length: len until merged), integrate's conflict marks
  uint8_t cl, ocl, rcl, fl;        // client slot (block order), origin / right origin client slots, T_* flags
};
struct CT { uint32_t id, state; uint16_t r0, rn, ri, ni; int16_t ins, pad; };

// workspace bytes besides the input: client table, id order, parts and their sequence / stack array
YDEV uint32_t ws_fixed() { return CMAX * (uint32_t)sizeof(CT) + CMAX; }
YDEV uint32_t part_bytes() { return (uint32_t)sizeof(P) + 2u; }

struct TDoc {
  InW w32; uint32_t sh, n, flags;   // the input: byte i at bit 8 * ((i + sh) & 3) of w32[(i + sh) >> 2] (readable past n)
  P* p; uint32_t np, cap;
  CT* ct; uint8_t* ord; uint32_t nc;
  uint16_t* sq;
  uint32_t name_off, name_len, ds_pos, epoch, n_ins;
  uint16_t start;
  bool have_name, bad;

  YDEV uint32_t at(uint32_t i) const { const uint32_t j = i + sh; return (w32[j >> 2] >> (8u * (j & 3u))) & 0xFFu; }

  YDEV int slot(uint32_t id) const {
    for (uint32_t k = 0; k < nc; k++) if (ct[k].id == id) return (int)k;
    return -1;
  }

  // ------------------------------------------------------------------ read (Doc::parse)
  // A lean reader for the envelope's shapes: varuints of <= 5 bytes below 2^32 (larger ones, any read past the end,
  // a struct of another kind, a non-ASCII string: outside the envelope), the same values as read_struct / Cur::vu.
  uint32_t pos;
  YDEV uint32_t vu() {   // one 8-byte window (two aligned dwords) holds the <= 5 bytes
    const uint32_t j = pos + sh;
    uint64_t win = (((uint64_t)w32[(j >> 2) + 1] << 32) | w32[j >> 2]) >> (8u * (j & 3u));
    uint32_t v = 0;
#pragma unroll 1
    for (uint32_t k = 0; k < 5u; k++) {
      if (pos >= n) { bad = true; return 0; }
      const uint32_t x = (uint32_t)win & 0xFFu;
      win >>= 8; pos++;
      v |= (x & 127u) << (7u * k);
      if (x < 128u) { if (k == 4u && (x & 0x70u)) bad = true; return v; }
    }
    bad = true;
    return 0;
  }
  YDEV bool ascii(uint32_t a, uint32_t l) const {   // a dword at a time: no byte of [a, a + l) has its top bit set
    for (uint32_t i = 0; i < l;) {
      const uint32_t j = a + i + sh, q = j & 3u, take = 4u - q < l - i ? 4u - q : l - i;
      const uint32_t w = w32[j >> 2] >> (8u * q);
      const uint32_t m = take == 4u ? 0x80808080u : 0x80808080u & ((1u << (8u * take)) - 1u);
      if (w & m) return false;
      i += take;
    }
    return true;
  }
  template <class O>
  YDEV void copy_in(O& o, uint32_t a, uint32_t l) const {   // input bytes [a, a + l) to o, a dword fetched per 4 bytes
    for (uint32_t i = 0; i < l;) {
      const uint32_t j = a + i + sh, q = j & 3u, take = 4u - q < l - i ? 4u - q : l - i;
      uint32_t w = w32[j >> 2] >> (8u * q);
      for (uint32_t t = 0; t < take; t++) { o.b((uint8_t)w); w >>= 8; }
      i += take;
    }
  }
  YDEV void parse() {
    pos = 0;
    const uint32_t nb = vu();
    for (uint32_t b = 0; b < nb && !bad; b++) {
      const uint32_t ns = vu(), client = vu(); uint32_t clock = vu();
      if (bad || nc >= CMAX || slot(client) >= 0) { bad = true; return; }
      CT& k = ct[nc];
      k.id = client; k.state = 0; k.r0 = (uint16_t)np; k.rn = 0; k.ri = 0; k.ni = 0; k.ins = -1; k.pad = 0;
      for (uint32_t s = 0; s < ns && !bad; s++) {
        if (pos >= n || np >= cap) { bad = true; return; }
        const uint8_t info = (uint8_t)at(pos++);
        const uint32_t ref = info & 31u;
        if (ref != 1u && ref != 4u) { bad = true; return; }   // GC / Skip / other content: the general path
        P& x = p[np];
        x.orig = (uint16_t)np; x.nxt = NIL; x.left = x.right = 0; x.ms = x.mr = 0; x.ok = x.rk = 0; x.ocl = x.rcl = 0;
        x.cl = (uint8_t)nc; x.fl = ref == 4u ? T_STR : 0; x.coff = 0;
        if (info & 0x80) {   // origin id: the client id parks in (ms, mr) until the client table is complete
          const uint32_t oc = vu(), ok = vu();
          if (ok > 0xFFFFu) bad = true;
          x.ms = (uint16_t)(oc >> 16); x.mr = (uint16_t)oc; x.ok = (uint16_t)ok; x.fl |= T_HO;
        }
        if (info & 0x40) {   // right origin: the client id parks in (left, right)
          const uint32_t rc = vu(), rk = vu();
          if (rk > 0xFFFFu) bad = true;
          x.left = (uint16_t)(rc >> 16); x.right = (uint16_t)rc; x.rk = (uint16_t)rk; x.fl |= T_HR;
        }
        if ((info & 0xC0) == 0) {   // the root type by name (ASCII), the same one for the whole update
          if (vu() != 1u || (info & 0x20)) { bad = true; return; }
          const uint32_t l = vu();
          if (bad || l > n - pos || !ascii(pos, l)) { bad = true; return; }
          if (!have_name) { name_off = pos; name_len = l; have_name = true; }
          else {
            if (l != name_len) { bad = true; return; }
            for (uint32_t i = 0; i < l; i++) if (at(pos + i) != at(name_off + i)) { bad = true; return; }
          }
          pos += l;
        }
        uint32_t len;
        if (ref == 1u) len = vu();                  // ContentDeleted
        else {                                      // ContentString, ASCII: UTF-16 length == bytes
          len = vu();
          if (bad || len > n - pos || !ascii(pos, len)) { bad = true; return; }
          x.coff = (uint16_t)pos;
          pos += len;
        }
        if (bad || len == 0 || clock + len > 0xFFFFu) { bad = true; return; }
        x.clock = (uint16_t)clock; x.len = (uint16_t)len;
        clock += len;
        np++; k.rn++;
      }
      nc++;
    }
    if (bad) return;
    ds_pos = pos;   // the delete set, checked now, applied after the structs
    const uint32_t nd = vu();
    for (uint32_t q = 0; q < nd && !bad; q++) {
      (void)vu(); const uint32_t nr = vu();
      for (uint32_t r = 0; r < nr && !bad; r++) {
        const uint64_t ck = vu(), ln = vu();
        if (ck + ln > 0xFFFFFFFFull) { bad = true; return; }
      }
    }
    if (bad) return;
    for (uint32_t i = 0; i < np; i++) {   // origin client ids -> slots (an unknown client leaves the item pending)
      P& x = p[i];
      if (x.fl & T_HO) { const int k = slot(((uint32_t)x.ms << 16) | x.mr); if (k < 0) { bad = true; return; } x.ocl = (uint8_t)k; }
      if (x.fl & T_HR) { const int k = slot(((uint32_t)x.left << 16) | x.right); if (k < 0) { bad = true; return; } x.rcl = (uint8_t)k; }
      x.ms = x.mr = 0; x.left = x.right = NIL;
    }
    for (uint32_t a = 0; a < nc; a++) ord[a] = (uint8_t)a;   // slots by id
    for (uint32_t a = 1; a < nc; a++) {
      const uint8_t v = ord[a]; uint32_t b = a;
      while (b > 0 && ct[ord[b - 1]].id > ct[v].id) { ord[b] = ord[b - 1]; b--; }
      ord[b] = v;
    }
  }

  // ------------------------------------------------------------------ lookups and splits (Doc::find / split)
  YDEV uint16_t find(uint32_t k, uint32_t clock) {
    const CT kk = ct[k];
    if (clock >= kk.state) { bad = true; return NIL; }
    // the last input struct starting at or before clock: an interpolated guess over the client's integrated input
    // structs (they tile [0, state) in clock order), then a walk to it -- a step or two for typed text
    const int32_t lo = kk.r0, hi = (int32_t)kk.r0 + kk.ni - 1;
    int32_t g = lo + (int32_t)(((uint32_t)(hi - lo + 1) * clock) / kk.state);
    g = g > hi ? hi : g;
    while (g > lo && p[g].clock > clock) g--;
    while (g < hi && p[g + 1].clock <= clock) g++;
    uint16_t x = (uint16_t)g;
    while (x != NIL && !(clock < (uint32_t)p[x].clock + p[x].len)) x = p[x].nxt;
    if (x == NIL) bad = true;
    return x;
  }
  YDEV uint16_t next_part(uint16_t x) const {
    if (p[x].nxt != NIL) return p[x].nxt;
    const CT& k = ct[p[x].cl];
    return (uint32_t)p[x].orig + 1 < (uint32_t)k.r0 + k.ni ? (uint16_t)(p[x].orig + 1) : NIL;
  }
  YDEV uint16_t split(uint16_t x, uint32_t diff) {   // x keeps [0, diff)
    if (np >= cap) { bad = true; return NIL; }
    const uint16_t r = (uint16_t)np++;
    P b = p[x];
    b.clock = (uint16_t)(b.clock + diff); b.len = (uint16_t)(b.len - diff);
    b.left = x; b.ocl = p[x].cl; b.ok = (uint16_t)(p[x].clock + diff - 1);
    b.fl = (uint8_t)((p[x].fl & (T_DEL | T_HR | T_INT | T_STR)) | T_HO);
    b.ms = b.mr = 0;
    if (b.fl & T_STR) b.coff = (uint16_t)(b.coff + diff);
    b.nxt = p[x].nxt;
    p[r] = b;
    p[x].nxt = r; p[x].right = r; p[x].len = (uint16_t)diff;
    if (b.right != NIL) p[b.right].left = r;
    return r;
  }
  YDEV uint16_t clean_end(uint32_t k, uint32_t clock) {
    const uint16_t x = find(k, clock);
    if (x != NIL && clock != (uint32_t)p[x].clock + p[x].len - 1) split(x, clock - p[x].clock + 1);
    return x;
  }
  YDEV uint16_t clean_start(uint32_t k, uint32_t clock) {
    const uint16_t x = find(k, clock);
    if (x != NIL && p[x].clock < clock) return split(x, clock - p[x].clock);
    return x;
  }

  // ------------------------------------------------------------------ integration (Doc::get_missing / integrate)
  // Item.getMissing on u (its record read once into pu): the client of a missing dependency, or -1 with the left /
  // right neighbours found (getItemCleanEnd / getItemCleanStart split the parts they land in; u itself is not
  // integrated yet, so no split touches its record)
  YDEV int get_missing(const P& pu, uint16_t& L, uint16_t& R) {
    if ((pu.fl & T_HO) && pu.ocl != pu.cl && pu.ok >= ct[pu.ocl].state) return pu.ocl;
    if ((pu.fl & T_HR) && pu.rcl != pu.cl && pu.rk >= ct[pu.rcl].state) return pu.rcl;
    L = (pu.fl & T_HO) ? clean_end(pu.ocl, pu.ok) : NIL;
    R = (pu.fl & T_HR) ? clean_start(pu.rcl, pu.rk) : NIL;
    return -1;
  }
  YDEV bool same(bool ha, uint32_t ac, uint32_t ak, bool hb, uint32_t bc, uint32_t bk) const {
    return (!ha && !hb) || (ha && hb && ac == bc && ak == bk);
  }
  YDEV void integrate(uint16_t x, const P& pu, uint16_t left, const uint16_t right) {
    const uint8_t fl = pu.fl;
    const bool ho = fl & T_HO, hr = fl & T_HR;
    const uint32_t oc = pu.ocl, ok = pu.ok, rc = pu.rcl, rk = pu.rk, myid = ct[pu.cl].id;
    if ((left == NIL && (right == NIL || p[right].left != NIL)) || (left != NIL && p[left].right != right)) {
      uint16_t e = left;
      uint16_t o = left != NIL ? p[left].right : start;
      if (epoch >= 0xFF00u) { bad = true; return; }
      const uint32_t eR = ++epoch;
      uint32_t curS = eR;
      while (o != NIL && o != right) {
        p[o].mr = (uint16_t)eR; p[o].ms = (uint16_t)curS;
        const uint8_t f2 = p[o].fl;
        if (same(ho, oc, ok, f2 & T_HO, p[o].ocl, p[o].ok)) {
          if (ct[p[o].cl].id < myid) { e = o; curS = ++epoch; }
          else if (same(hr, rc, rk, f2 & T_HR, p[o].rcl, p[o].rk)) break;
        } else if (f2 & T_HO) {
          const uint16_t g = find(p[o].ocl, p[o].ok);
          if (bad) return;
          if (p[g].mr == (uint16_t)eR) { if (p[g].ms != (uint16_t)curS) { e = o; curS = ++epoch; } }
          else break;
        } else break;
        if (epoch >= 0xFF00u) { bad = true; return; }
        o = p[o].right;
      }
      left = e;
    }
    uint16_t r;
    if (left != NIL) { r = p[left].right; p[left].right = x; }
    else { r = start; start = x; }
    p[x].left = left; p[x].right = r;
    if (r != NIL) p[r].left = x;
    CT& k = ct[pu.cl];   // addStruct
    if (k.ins < 0) k.ins = (int16_t)n_ins++;
    k.state = (uint32_t)pu.clock + pu.len;
    k.ni = (uint16_t)(pu.orig - k.r0 + 1);
    p[x].fl = (uint8_t)(fl | T_INT | ((fl & T_STR) ? 0 : T_DEL));   // ContentDeleted.integrate: deleted at once
  }
  YDEV void integrate_all() {   // Doc::integrate_all: highest client first, the dependency stack
    int32_t ci = (int32_t)nc - 1;
    auto next_client = [&]() -> int32_t {
      while (ci >= 0 && ct[ord[ci]].ri >= ct[ord[ci]].rn) ci--;
      return ci;
    };
    int32_t cur = next_client();
    if (cur < 0) return;
    uint16_t u = (uint16_t)(ct[ord[cur]].r0 + ct[ord[cur]].ri++);
    uint32_t sp = 0;
    for (;;) {
      if (bad) return;
      const P pu = p[u];
      const int64_t diff = (int64_t)ct[pu.cl].state - (int64_t)pu.clock;
      if (diff < 0) { bad = true; return; }
      uint16_t L = NIL, R = NIL;
      const int m = get_missing(pu, L, R);
      if (bad) return;
      if (m >= 0) {
        if (sp >= cap || ct[m].ri >= ct[m].rn) { bad = true; return; }
        sq[sp++] = u;
        u = (uint16_t)(ct[m].r0 + ct[m].ri++);
        continue;
      }
      if (diff != 0) { bad = true; return; }
      integrate(u, pu, L, R);
      if (sp) u = sq[--sp];
      else if (cur >= 0 && ct[ord[cur]].ri < ct[ord[cur]].rn) u = (uint16_t)(ct[ord[cur]].r0 + ct[ord[cur]].ri++);
      else {
        cur = next_client();
        if (cur < 0) break;
        u = (uint16_t)(ct[ord[cur]].r0 + ct[ord[cur]].ri++);
      }
    }
  }

  // ------------------------------------------------------------------ delete set, GC, merge (Doc::apply_ds ..)
  YDEV void apply_ds() {
    pos = ds_pos;
    const uint32_t nd = vu();
    for (uint64_t q = 0; q < nd && !bad; q++) {
      const uint32_t client = vu(), nr = vu();
      const int k = slot(client);
      for (uint64_t r = 0; r < nr && !bad; r++) {
        const uint64_t a = vu(); const uint64_t b = a + vu();
        if (k < 0) { bad = true; return; }   // (state 0: pending)
        const uint32_t s = ct[k].state;
        if (!(a < s) || s < b) { bad = true; return; }
        uint16_t x = find((uint32_t)k, (uint32_t)a);
        if (bad) return;
        if (!(p[x].fl & T_DEL) && p[x].clock < a) { split(x, (uint32_t)a - p[x].clock); x = p[x].nxt; }
        while (x != NIL && !bad) {
          if (p[x].clock < b) {
            if (!(p[x].fl & T_DEL)) {
              if (b < (uint64_t)p[x].clock + p[x].len) split(x, (uint32_t)b - p[x].clock);
              p[x].fl |= T_DEL;
            }
          } else break;
          x = next_part(x);
        }
      }
    }
  }
  // the client's parts in clock order into sq (GONE ones included when all); returns the count
  YDEV uint32_t client_seq(uint32_t k, bool all) {
    uint32_t m = 0;
    for (uint32_t o = ct[k].r0; o < (uint32_t)ct[k].r0 + ct[k].ni; o++)
      for (uint16_t x = (uint16_t)o; x != NIL; x = p[x].nxt)
        if (all || !(p[x].fl & T_GONE)) sq[m++] = x;
    return m;
  }
  YDEV void gc_merge() {
    for (uint32_t i = 0; i < np; i++) if (p[i].fl & T_DEL) p[i].fl = (uint8_t)(p[i].fl & ~T_STR);   // tryGcDeleteSet
    for (uint32_t k = 0; k < nc; k++) {   // one right-to-left tryToMergeWithLeft pass per client
      const uint32_t m = client_seq(k, false);
      for (uint32_t e = m; e-- > 1;) {
        const uint16_t a = sq[e - 1], b = sq[e];
        const P L = p[a], R = p[b];   // (both records read at once)
        if (((L.fl ^ R.fl) & (T_DEL | T_STR)) != 0) continue;
        if (!((R.fl & T_HO) && R.ocl == L.cl && R.ok == (uint32_t)L.clock + L.len - 1)) continue;
        if (L.right != b) continue;
        if (!same(L.fl & T_HR, L.rcl, L.rk, R.fl & T_HR, R.rcl, R.rk)) continue;
        if ((uint32_t)L.clock + L.len != R.clock) continue;
        const uint16_t rr = R.right;
        p[a].right = rr;
        if (rr != NIL) p[rr].left = a;
        p[a].len = (uint16_t)(p[a].len + p[b].len);
        p[b].fl |= T_GONE;
      }
    }
  }

  // ------------------------------------------------------------------ encodeStateAsUpdate (Doc::encode)
  template <class O>
  YDEV void encode(O& o) {
    uint32_t cnt = 0;
    for (uint32_t k = 0; k < nc; k++) cnt += ct[k].ni > 0 ? 1u : 0u;
    o.vu32(cnt);
    for (uint32_t i = nc; i-- > 0;) {
      const uint32_t k = ord[i];
      if (!ct[k].ni) continue;
      const uint32_t m = client_seq(k, true);
      uint32_t live = 0;
      for (uint32_t j = 0; j < m; j++) live += (p[sq[j]].fl & T_GONE) ? 0u : 1u;
      o.vu32(live); o.vu32(ct[k].id); o.vu32(p[sq[0]].clock);
      for (uint32_t j = 0; j < m; j++) {
        const P u = p[sq[j]];
        if (!(u.fl & T_GONE)) {
          const bool ho = u.fl & T_HO, hr = u.fl & T_HR;
          o.b((uint8_t)(((u.fl & T_STR) ? 4 : 1) | (ho ? 0x80 : 0) | (hr ? 0x40 : 0)));
          if (ho) { o.vu32(ct[u.ocl].id); o.vu32(u.ok); }
          if (hr) { o.vu32(ct[u.rcl].id); o.vu32(u.rk); }
          if (!ho && !hr) { o.b(1); o.vu32(name_len); copy_in(o, name_off, name_len); }
          o.vu32(u.len);
        }
        if (u.fl & T_STR) {   // a merged part's bytes: its own, then those it absorbed (the GONE parts after it,
                              // each of whose len counts its own bytes and those it absorbed in turn)
          const uint32_t nx = j + 1 < m && (p[sq[j + 1]].fl & T_GONE) ? p[sq[j + 1]].len : 0u;
          copy_in(o, u.coff, u.len - nx);
        }
      }
    }
    // delete set from the struct store: runs of deleted parts; clients in store order (13.5) or descending (13.6)
    uint32_t nds = 0;
    for (uint32_t k = 0; k < nc; k++) {
      if (!ct[k].ni) continue;
      const uint32_t m = client_seq(k, false);
      for (uint32_t j = 0; j < m; j++) if (p[sq[j]].fl & T_DEL) { nds++; break; }
    }
    o.vu32(nds);
    for (uint32_t r = 0; r < nc; r++) {
      int32_t k = -1;
      if (flags & F_COMPAT_135) { for (uint32_t j = 0; j < nc; j++) if (ct[j].ins == (int32_t)r) k = (int32_t)j; }
      else k = ord[nc - 1 - r];
      if (k < 0 || !ct[k].ni) continue;
      const uint32_t m = client_seq((uint32_t)k, false);
      uint32_t runs = 0;
      for (uint32_t j = 0; j < m; j++) if ((p[sq[j]].fl & T_DEL) && (j == 0 || !(p[sq[j - 1]].fl & T_DEL))) runs++;
      if (!runs) continue;
      o.vu32(ct[k].id); o.vu32(runs);
      for (uint32_t j = 0; j < m;) {
        if (!(p[sq[j]].fl & T_DEL)) { j++; continue; }
        const uint32_t c0 = p[sq[j]].clock; uint32_t len = 0;
        while (j < m && (p[sq[j]].fl & T_DEL)) len += p[sq[j++]].len;
        o.vu32(c0); o.vu32(len);
      }
    }
  }

  template <class O>
  YDEV bool run(O& o) {
    parse();
    if (!bad) integrate_all();
    if (!bad) apply_ds();
    if (!bad) gc_merge();
    if (bad) return false;
    encode(o);
    return true;
  }
};

// The snapshot of in[0, n) over a workspace of ws_bytes at ws (4-aligned), written through o (OutCap: stops at its
// cap); false: outside the envelope or the workspace (the general kernel takes the document).
template <class O>
YDEV bool snapshot_text(const uint8_t* in, uint32_t n, uint32_t flags, uint8_t* ws, uint32_t ws_bytes, O& o) {
  if (n >= 0xFFFFu || ws_bytes < ws_fixed() + 16u * part_bytes()) return false;
  TDoc D;
  D.sh = (uint32_t)((uintptr_t)in & 3u); D.w32 = (InW)(in - D.sh); D.n = n; D.flags = flags;
  D.ct = (CT*)ws; D.ord = ws + CMAX * sizeof(CT); D.nc = 0;
  D.cap = (ws_bytes - ws_fixed()) / part_bytes();
  if (D.cap > 0xFFF0u) D.cap = 0xFFF0u;
  D.p = (P*)(ws + ws_fixed()); D.np = 0;
  D.sq = (uint16_t*)(ws + ws_fixed() + D.cap * (uint32_t)sizeof(P));
  D.name_off = D.name_len = 0; D.ds_pos = 0; D.epoch = 0; D.n_ins = 0; D.start = NIL; D.have_name = false; D.bad = false;
  return D.run(o);
}

}  // namespace snapt
}  // namespace ygm
