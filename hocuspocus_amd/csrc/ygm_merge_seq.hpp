// ygm_merge_seq.hpp -- the exact sequential mergeUpdates kernel body (one lane = one document).
//
// Runs yjs's mergeUpdatesV2 loop (Y@39011-40710) literally,
// including the per-iteration re-sort of the struct decoders with V8's TimSort
// (third_party/v8 builtins/array-sort.tq) because yjs's comparator is
// inconsistent for GC-vs-Item ties (App. B.5): only an exact replay of V8's
// comparison sequence reproduces which struct wins.  Used for the documents
// the workgroup fast path cannot prove overlap-free, or that exceed its LDS
// capacity.  Scratch lives in global memory (reserved per document with
// atomic cursors by the launcher).
#pragma once
#include "ygm_seqdoc.hpp"

namespace ygm {

// A filtered reader (LazyStructReader(decoder, filterSkips=true))
YDEV void rd_next_nonskip(Stream& r) {
  do { r.next(); } while (r.has && r.cur.kind == K_SKIP && !r.c.err);
}
YDEV void rd_init(Stream& r, const uint8_t* p, uint32_t n, uint32_t flags) {
  r.init(p, n, flags);
  while (r.has && r.cur.kind == K_SKIP && !r.c.err) r.next();
}

// comparator of Y@39011 over reader heads
struct DecCmp {
  Stream* R;
  YDEV int operator()(int x, int y) const {
    const Stream& a = R[x]; const Stream& b = R[y];
    if (a.cur_client == b.cur_client) {
      if (a.cur_clock == b.cur_clock) return a.cur.kind == b.cur.kind ? 0 : (a.cur.kind == K_SKIP ? 1 : -1);
      return a.cur_clock < b.cur_clock ? -1 : 1;
    }
    return b.cur_client < a.cur_client ? -1 : 1;
  }
};

// ---------------------------------------------------------------- V8 TimSort
// Comparator-call-exact port (validated against V8 by the CPU oracle's
// v8_timsort_vectors fixtures; this copy is checked against the oracle on the GPU).
template <class C>
struct V8Sort {
  int* a; int* tmp; C cmp; int min_gallop; int rb[85], rl[85]; int nruns;
  YDEV static int min_run(int n) { int r = 0; while (n >= 64) { r |= n & 1; n >>= 1; } return n + r; }
  YDEV void reverse(int lo, int hi) { hi--; while (lo < hi) { const int t = a[lo]; a[lo] = a[hi]; a[hi] = t; lo++; hi--; } }
  YDEV int count_run(int lo_arg, int high) {
    const int low = lo_arg + 1;
    if (low == high) return 1;
    int run = 2;
    int order = cmp(a[low], a[low - 1]);
    const bool desc = order < 0;
    int prev = a[low];
    for (int i = low + 1; i < high; i++) {
      const int cur = a[i]; order = cmp(cur, prev);
      if (desc) { if (order >= 0) break; } else { if (order < 0) break; }
      prev = cur; run++;
    }
    if (desc) reverse(lo_arg, lo_arg + run);
    return run;
  }
  YDEV void binary_insertion(int low, int start_arg, int high) {
    int start = low == start_arg ? start_arg + 1 : start_arg;
    for (; start < high; start++) {
      int left = low, right = start; const int pivot = a[start];
      while (left < right) { const int mid = left + ((right - left) >> 1); if (cmp(pivot, a[mid]) < 0) right = mid; else left = mid + 1; }
      for (int p = start; p > left; p--) a[p] = a[p - 1];
      a[left] = pivot;
    }
  }
  YDEV int gallop_left(int* arr, int key, int base, int length, int hint) {
    int last = 0, ofs = 1;
    int order = cmp(arr[base + hint], key);
    if (order < 0) {
      const int mx = length - hint;
      while (ofs < mx) { order = cmp(arr[base + hint + ofs], key); if (order >= 0) break; last = ofs; ofs = (ofs << 1) + 1; if (ofs <= 0) ofs = mx; }
      if (ofs > mx) ofs = mx;
      last += hint; ofs += hint;
    } else {
      const int mx = hint + 1;
      while (ofs < mx) { order = cmp(arr[base + hint - ofs], key); if (order < 0) break; last = ofs; ofs = (ofs << 1) + 1; if (ofs <= 0) ofs = mx; }
      if (ofs > mx) ofs = mx;
      const int t = last; last = hint - ofs; ofs = hint - t;
    }
    last++;
    while (last < ofs) { const int m = last + ((ofs - last) >> 1); if (cmp(arr[base + m], key) < 0) last = m + 1; else ofs = m; }
    return ofs;
  }
  YDEV int gallop_right(int* arr, int key, int base, int length, int hint) {
    int last = 0, ofs = 1;
    int order = cmp(key, arr[base + hint]);
    if (order < 0) {
      const int mx = hint + 1;
      while (ofs < mx) { order = cmp(key, arr[base + hint - ofs]); if (order >= 0) break; last = ofs; ofs = (ofs << 1) + 1; if (ofs <= 0) ofs = mx; }
      if (ofs > mx) ofs = mx;
      const int t = last; last = hint - ofs; ofs = hint - t;
    } else {
      const int mx = length - hint;
      while (ofs < mx) { order = cmp(key, arr[base + hint + ofs]); if (order < 0) break; last = ofs; ofs = (ofs << 1) + 1; if (ofs <= 0) ofs = mx; }
      if (ofs > mx) ofs = mx;
      last += hint; ofs += hint;
    }
    last++;
    while (last < ofs) { const int m = last + ((ofs - last) >> 1); if (cmp(key, arr[base + m]) < 0) ofs = m; else last = m + 1; }
    return ofs;
  }
  YDEV static void cpy(int* d, const int* s, int n) { for (int i = 0; i < n; i++) d[i] = s[i]; }
  YDEV static void mv(int* d, const int* s, int n) {
    if (d < s) { for (int i = 0; i < n; i++) d[i] = s[i]; } else { for (int i = n - 1; i >= 0; i--) d[i] = s[i]; }
  }
  YDEV void merge_low(int baseA, int lenA, int baseB, int lenB) {
    int* w = a; int* t = tmp;
    cpy(t, w + baseA, lenA);
    int dest = baseA, ct = 0, cb = baseB;
    w[dest++] = w[cb++];
    if (--lenB == 0) goto succeed;
    if (lenA == 1) goto copyB;
    {
      int mg = min_gallop;
      for (;;) {
        int wa = 0, wb = 0;
        for (;;) {
          if (cmp(w[cb], t[ct]) < 0) { w[dest++] = w[cb++]; wb++; lenB--; wa = 0; if (lenB == 0) goto succeed; if (wb >= mg) break; }
          else { w[dest++] = t[ct++]; wa++; lenA--; wb = 0; if (lenA == 1) goto copyB; if (wa >= mg) break; }
        }
        mg++;
        bool first = true;
        while (wa >= 7 || wb >= 7 || first) {
          first = false;
          mg = mg - 1 > 1 ? mg - 1 : 1; min_gallop = mg;
          wa = gallop_right(t, w[cb], ct, lenA, 0);
          if (wa > 0) { cpy(w + dest, t + ct, wa); dest += wa; ct += wa; lenA -= wa; if (lenA == 1) goto copyB; if (lenA == 0) goto succeed; }
          w[dest++] = w[cb++];
          if (--lenB == 0) goto succeed;
          wb = gallop_left(w, t[ct], cb, lenB, 0);
          if (wb > 0) { mv(w + dest, w + cb, wb); dest += wb; cb += wb; lenB -= wb; if (lenB == 0) goto succeed; }
          w[dest++] = t[ct++];
          if (--lenA == 1) goto copyB;
        }
        mg++; min_gallop = mg;
      }
    }
  succeed:
    if (lenA > 0) cpy(w + dest, t + ct, lenA);
    return;
  copyB:
    mv(w + dest, w + cb, lenB);
    w[dest + lenB] = t[ct];
  }
  YDEV void merge_high(int baseA, int lenA, int baseB, int lenB) {
    int* w = a; int* t = tmp;
    cpy(t, w + baseB, lenB);
    int dest = baseB + lenB - 1, ct = lenB - 1, ca = baseA + lenA - 1;
    w[dest--] = w[ca--];
    if (--lenA == 0) goto succeed;
    if (lenB == 1) goto copyA;
    {
      int mg = min_gallop;
      for (;;) {
        int wa = 0, wb = 0;
        for (;;) {
          if (cmp(t[ct], w[ca]) < 0) { w[dest--] = w[ca--]; wa++; lenA--; wb = 0; if (lenA == 0) goto succeed; if (wa >= mg) break; }
          else { w[dest--] = t[ct--]; wb++; lenB--; wa = 0; if (lenB == 1) goto copyA; if (wb >= mg) break; }
        }
        mg++;
        bool first = true;
        while (wa >= 7 || wb >= 7 || first) {
          first = false;
          mg = mg - 1 > 1 ? mg - 1 : 1; min_gallop = mg;
          int k = gallop_right(w, t[ct], baseA, lenA, lenA - 1);
          wa = lenA - k;
          if (wa > 0) { dest -= wa; ca -= wa; mv(w + dest + 1, w + ca + 1, wa); lenA -= wa; if (lenA == 0) goto succeed; }
          w[dest--] = t[ct--];
          if (--lenB == 1) goto copyA;
          k = gallop_left(t, w[ca], 0, lenB, lenB - 1);
          wb = lenB - k;
          if (wb > 0) { dest -= wb; ct -= wb; cpy(w + dest + 1, t + ct + 1, wb); lenB -= wb; if (lenB == 1) goto copyA; if (lenB == 0) goto succeed; }
          w[dest--] = w[ca--];
          if (--lenA == 0) goto succeed;
        }
        mg++; min_gallop = mg;
      }
    }
  succeed:
    if (lenB > 0) cpy(w + dest - (lenB - 1), t, lenB);
    return;
  copyA:
    dest -= lenA; ca -= lenA;
    mv(w + dest + 1, w + ca + 1, lenA);
    w[dest] = t[ct];
  }
  YDEV void merge_at(int i) {
    const int n = nruns;
    int baseA = rb[i], lenA = rl[i]; const int baseB = rb[i + 1]; int lenB = rl[i + 1];
    rl[i] = lenA + lenB;
    if (i == n - 3) { rb[i + 1] = rb[i + 2]; rl[i + 1] = rl[i + 2]; }
    nruns = n - 1;
    const int k = gallop_right(a, a[baseB], baseA, lenA, 0);
    baseA += k; lenA -= k;
    if (lenA == 0) return;
    lenB = gallop_left(a, a[baseA + lenA - 1], baseB, lenB, lenB - 1);
    if (lenB == 0) return;
    if (lenA <= lenB) merge_low(baseA, lenA, baseB, lenB); else merge_high(baseA, lenA, baseB, lenB);
  }
  YDEV bool inv(int n) { if (n < 2) return true; return rl[n - 2] > rl[n - 1] + rl[n]; }
  YDEV void collapse() {
    while (nruns > 1) {
      int n = nruns - 2;
      if (!inv(n + 1) || !inv(n)) { if (rl[n - 1] < rl[n + 1]) n--; merge_at(n); }
      else if (rl[n] <= rl[n + 1]) merge_at(n);
      else break;
    }
  }
  YDEV void force_collapse() {
    while (nruns > 1) { int n = nruns - 2; if (n > 0 && rl[n - 1] < rl[n + 1]) n--; merge_at(n); }
  }
  YDEV void sort(int n) {
    if (n < 2) return;
    min_gallop = 7; nruns = 0;
    int remaining = n, low = 0; const int minrun = min_run(n);
    while (remaining) {
      int run = count_run(low, low + remaining);
      if (run < minrun) { const int forced = minrun < remaining ? minrun : remaining; binary_insertion(low, low + run, low + forced); run = forced; }
      rb[nruns] = low; rl[nruns] = run; nruns++;
      collapse();
      low += run; remaining -= run;
    }
    force_collapse();
  }
};

// ---------------------------------------------------------------- writer
// currWrite: an input struct (maybe sliced by `cut`) or a synthetic Skip
struct CW {
  SInfo s; const uint8_t* base;
  uint64_t client, clock0;  // clock0: clock of the unsliced struct
  uint64_t cut;             // sliceStruct offset applied (Items: splice)
  uint64_t len;             // current length (GC/Skip merges and shrinks)
  YDEV uint64_t clock() const { return clock0 + cut; }
  YDEV uint64_t end() const { return clock0 + cut + len; }
};
YDEV CW cw_from(const Stream& r) {
  CW w; w.s = r.cur; w.base = r.c.p; w.client = r.cur_client; w.clock0 = r.cur_clock; w.cut = 0; w.len = r.cur.len; return w;
}

// LazyStructWriter; in the count pass it records each block's struct count.
struct LW {
  Out* o; bool write; uint32_t flags;
  uint64_t written, curr_client, bi;
  uint32_t* cnt; uint64_t cnt_cap;
  int err;
  bool nc;  // NONCANON content written: reported only if nothing else throws
  YDEV void flush() {
    if (written > 0) {
      if (!write) { if (bi < cnt_cap) cnt[bi] = (uint32_t)written; else err = ST_NOMEM; o->n += vu_len(written); }
      bi++; written = 0;
    }
  }
  YDEV void put(const CW& w) {
    if (err) return;
    if (written > 0 && curr_client != w.client) flush();
    if (written == 0) {
      curr_client = w.client;
      if (write) o->vu(cnt[bi]);
      o->vu(w.client); o->vu(w.clock());
    }
    int e = ST_OK;
    if (w.s.kind == K_GC) { o->b(0); o->vu(w.len); }
    else if (w.s.kind == K_SKIP) { o->b(10); o->vu(w.len); }
    else e = write_struct(*o, w.base, w.s, w.client, w.clock0, w.cut, true, flags);
    if (e == ST_NONCANON) nc = true;
    else if (e) err = e;
    written++;
  }
};

YDEV bool cw_try_merge(CW& w, const CW& n) {  // GC.mergeWith / Skip.mergeWith; Items never merge lazily
  if (w.s.kind == n.s.kind && w.s.kind != K_ITEM) { w.len += n.len; return true; }
  return false;
}

// One full pass of the mergeUpdatesV2 struct loop.  Returns status.
YDEV_NI int merge_pass(Stream* R, int* order, int* tmp, int k, const uint8_t* const* ubase, const uint32_t* ulen,
                    uint32_t flags, LW& lw) {
  for (int i = 0; i < k; i++) { rd_init(R[i], ubase[i], ulen[i], flags); if (R[i].c.err) return R[i].c.err; order[i] = i; }
  int nd = k;
  CW cw; bool has_cw = false;
  V8Sort<DecCmp> vs; vs.a = order; vs.tmp = tmp; vs.cmp.R = R;
  for (;;) {
    int m = 0;
    for (int i = 0; i < nd; i++) if (R[order[i]].has) order[m++] = order[i];
    nd = m;
    vs.sort(nd);
    if (nd == 0) break;
    Stream& t = R[order[0]];
    const uint64_t first_client = t.cur_client;
    if (has_cw) {
      bool iterated = false;
      while (t.has && t.cur_clock + t.cur.len <= cw.end() && t.cur_client >= cw.client) {
        rd_next_nonskip(t); if (t.c.err) return t.c.err; iterated = true;
      }
      if (!t.has || t.cur_client != first_client || (iterated && t.cur_clock > cw.end())) continue;
      if (first_client != cw.client) {
        lw.put(cw); cw = cw_from(t); rd_next_nonskip(t);
      } else if (cw.end() < t.cur_clock) {
        if (cw.s.kind == K_SKIP) { cw.len = t.cur_clock + t.cur.len - cw.clock(); }
        else {
          lw.put(cw);
          CW sk; sk.s.kind = K_SKIP; sk.s.info = 10; sk.s.nc = false; sk.base = nullptr;
          sk.client = first_client; sk.clock0 = cw.end(); sk.cut = 0; sk.len = t.cur_clock - cw.end();
          cw = sk;
        }
      } else {
        const uint64_t diff = cw.end() - t.cur_clock;
        CW n = cw_from(t);
        if (diff > 0) {
          if (cw.s.kind == K_SKIP) cw.len -= diff;
          else { n.cut = diff; n.len = n.s.len - diff; }  // sliceStruct (Y@38665)
        }
        if (!cw_try_merge(cw, n)) { lw.put(cw); cw = n; rd_next_nonskip(t); }
      }
    } else {
      cw = cw_from(t); has_cw = true; rd_next_nonskip(t);
    }
    if (t.c.err) return t.c.err;
    while (t.has && t.cur_client == first_client && t.cur_clock == cw.end() && t.cur.kind != K_SKIP) {
      lw.put(cw); cw = cw_from(t);
      rd_next_nonskip(t); if (t.c.err) return t.c.err;
    }
    if (lw.err) return lw.err;
  }
  if (has_cw) lw.put(cw);
  lw.flush();
  return lw.err;
}

// ---------------------------------------------------------------- DS union
// mergeDeleteSets (Y@10486) + sortAndMergeDeleteSet (Y@10246) + writeDeleteSet.
struct DRec { uint64_t client, clock, len, seq, fs; };
YDEV bool drec_less(const DRec& x, const DRec& y, int mode) {
  if (mode == 0) { if (x.client != y.client) return x.client > y.client; return x.seq < y.seq; }       // group, first-seen
  if (mode == 1) { if (x.client != y.client) return x.client > y.client; return x.clock < y.clock; }   // 13.6 order
  if (x.fs != y.fs) return x.fs < y.fs; return x.clock < y.clock;                                      // 13.5 order
}
YDEV_NI void drec_heapsort(DRec* a, uint64_t n, int mode) {
  if (n < 2) return;
  for (int64_t start = (int64_t)(n / 2) - 1; start >= 0; start--) {
    uint64_t root = (uint64_t)start;
    for (;;) { uint64_t ch = 2 * root + 1; if (ch >= n) break; if (ch + 1 < n && drec_less(a[ch], a[ch + 1], mode)) ch++; if (drec_less(a[root], a[ch], mode)) { DRec t = a[root]; a[root] = a[ch]; a[ch] = t; root = ch; } else break; }
  }
  for (uint64_t end = n - 1; end > 0; end--) {
    DRec t = a[0]; a[0] = a[end]; a[end] = t;
    uint64_t root = 0;
    for (;;) { uint64_t ch = 2 * root + 1; if (ch >= end) break; if (ch + 1 < end && drec_less(a[ch], a[ch + 1], mode)) ch++; if (drec_less(a[root], a[ch], mode)) { DRec q = a[root]; a[root] = a[ch]; a[ch] = q; root = ch; } else break; }
  }
}
// Reads every update's DS (cursors positioned at their DS), returns #records or -err.
YDEV_NI int64_t ds_collect(Stream* R, int k, DRec* recs, uint64_t cap) {
  uint64_t n = 0;
  for (int i = 0; i < k; i++) {
    Cur& c = R[i].c;
    const uint64_t nc = c.vu();
    for (uint64_t q = 0; q < nc && !c.err; q++) {
      const uint64_t cl = c.vu(), nd = c.vu();
      for (uint64_t r = 0; r < nd && !c.err; r++) {
        const uint64_t ck = c.vu(), ln = c.vu();
        if (c.err) break;
        if (n >= cap) return -ST_NOMEM;
        recs[n].client = cl; recs[n].clock = ck; recs[n].len = ln; recs[n].seq = n; recs[n].fs = 0; n++;
      }
    }
    if (c.err) return -c.err;
  }
  return (int64_t)n;
}
// sorts and writes the merged delete set (o.p == nullptr -> size only)
YDEV_NI void ds_union_write(DRec* a, uint64_t n, uint32_t flags, Out& o) {
  // first-seen sequence per client
  drec_heapsort(a, n, 0);
  uint64_t fs = 0;
  for (uint64_t i = 0; i < n; i++) { if (i == 0 || a[i].client != a[i - 1].client) fs = a[i].seq; a[i].fs = fs; }
  drec_heapsort(a, n, (flags & F_COMPAT_135) ? 2 : 1);
  uint64_t nclients = 0;
  for (uint64_t i = 0; i < n; i++) if (i == 0 || a[i].client != a[i - 1].client) nclients++;
  o.vu(nclients);
  uint64_t i = 0;
  while (i < n) {
    uint64_t j = i; while (j < n && a[j].client == a[i].client) j++;
    // merge runs in [i, j): clock-sorted; run continues while clock <= running end
    uint64_t runs = 0, q = i;
    while (q < j) { uint64_t e = a[q].clock + a[q].len; uint64_t r = q + 1; while (r < j && a[r].clock <= e) { if (a[r].clock + a[r].len > e) e = a[r].clock + a[r].len; r++; } runs++; q = r; }
    o.vu(a[i].client); o.vu(runs);
    q = i;
    while (q < j) { uint64_t e = a[q].clock + a[q].len; uint64_t r = q + 1; while (r < j && a[r].clock <= e) { if (a[r].clock + a[r].len > e) e = a[r].clock + a[r].len; r++; } o.vu(a[q].clock); o.vu(e - a[q].clock); q = r; }
    i = j;
  }
}

}  // namespace ygm
