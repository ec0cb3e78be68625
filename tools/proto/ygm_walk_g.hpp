// Prototype (round 4, not product): the register-window SV walker timed by walkg.hip; kept with its harness.
// ygm_walk_g.hpp -- encodeStateVectorFromUpdate / diffUpdate walker with the document read through
// the cache hierarchy into a register window (no LDS ring).  One lane per document: per iteration a
// lane decodes ONE unit (struct, block header, update header) from a 32-byte register window at its
// parse position, loaded by two dword-aligned 16-byte loads and one dword, funnel-shifted by
// v_alignbyte; varuint ends come from the window's terminator mask (bit i: byte i < 0x80, by two
// v_dot4 per 8 bytes).  Without a ring there is no LDS per wave, so occupancy is set by registers.
#pragma once
#include "../../hocuspocus_amd/csrc/ygm_doc_walk.hpp"

namespace ygm {

typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

// 32 bytes of `src` from byte p (v[0] = bytes p..p+3) and their terminator mask.  Reads the 36 bytes
// from p & ~3: callers keep 40 readable bytes past every position they parse.
YDEV void gw_load(const uint8_t* __restrict__ src, uint64_t p, uint32_t (&v)[8], uint32_t& T) {
  const uint32_t* s = (const uint32_t*)(src + (p & ~3ull));
  const u32x4a4 a = *(const u32x4a4*)s, b = *(const u32x4a4*)(s + 4);
  const uint32_t c = s[8];
  const uint32_t sh = (uint32_t)p & 3u;
  v[0] = __builtin_amdgcn_alignbyte(a.y, a.x, sh);
  v[1] = __builtin_amdgcn_alignbyte(a.z, a.y, sh);
  v[2] = __builtin_amdgcn_alignbyte(a.w, a.z, sh);
  v[3] = __builtin_amdgcn_alignbyte(b.x, a.w, sh);
  v[4] = __builtin_amdgcn_alignbyte(b.y, b.x, sh);
  v[5] = __builtin_amdgcn_alignbyte(b.z, b.y, sh);
  v[6] = __builtin_amdgcn_alignbyte(b.w, b.z, sh);
  v[7] = __builtin_amdgcn_alignbyte(c, b.w, sh);
  T = ~(hibits8(v[0], v[1]) | (hibits8(v[2], v[3]) << 8) | (hibits8(v[4], v[5]) << 16) | (hibits8(v[6], v[7]) << 24));
}
// byte i (< 32) of the window: a three-level select, no indexed register access
YDEV uint32_t gw_byte(const uint32_t (&v)[8], uint32_t i) {
  const uint32_t k = i >> 2;
  const bool k0 = k & 1u, k1 = k & 2u, k2 = k & 4u;
  const uint32_t a = k0 ? v[1] : v[0], b = k0 ? v[3] : v[2], c = k0 ? v[5] : v[4], d = k0 ? v[7] : v[6];
  const uint32_t e = k1 ? b : a, f = k1 ? d : c;
  return __builtin_amdgcn_ubfe(k2 ? f : e, (i & 3u) * 8u, 8u);
}
// 8 bytes from byte o (o < 8) of the window
YDEV uint64_t gw_at8(const uint32_t (&v)[8], uint32_t o) {
  const uint64_t lo = (uint64_t)v[0] | ((uint64_t)v[1] << 32), hi = (uint64_t)v[2] | ((uint64_t)v[3] << 32);
  return dw_fsh(lo, hi, 8u * o);
}
YDEV uint32_t gw_ctz(uint32_t x) { return (uint32_t)__builtin_ctz(x | 0x80000000u) | (x ? 0u : 32u); }
YDEV uint32_t gw_clr(uint32_t x) { return x & (x - 1u); }
YDEV uint32_t gw_low(uint32_t n) { return n >= 32u ? 0xFFFFFFFFu : ((1u << n) - 1u); }

enum : uint32_t { G_IDLE = 0, G_UPD, G_BLK, G_ST, G_FIN };

// One unit per lane and iteration (MODE 0 = state vector).  Documents: wave w owns
// [n*w/G, n*(w+1)/G), lanes take the next one as they finish.  Output into the document's merge slot
// (merge_slot / merge_slot_cap, see ygm_kernels.hip): body from slot + 16, the count right-aligned in
// front.  Anything outside the fast shapes: status ST_FALLBACK + defer_list.
template <int MODE>
__global__ __launch_bounds__(WAVE) void k_walk_g(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ doc_off,
                                                 uint32_t n_docs, uint8_t* __restrict__ out, uint64_t* __restrict__ out_off,
                                                 uint64_t* __restrict__ out_len, int32_t* __restrict__ status,
                                                 unsigned int* __restrict__ defer_cnt, uint32_t* __restrict__ defer_list,
                                                 uint64_t out_cap, unsigned long long* __restrict__ payload_out) {
  const uint32_t l = threadIdx.x;
  const uint32_t D1 = (uint32_t)((uint64_t)n_docs * (blockIdx.x + 1) / gridDim.x);
  uint32_t next = (uint32_t)((uint64_t)n_docs * blockIdx.x / gridDim.x);
  uint64_t pa = 0, pb = 0;
  auto prefetch = [&]() {
    pa = 0; pb = 0;
    if (next + l < D1) { pa = doc_off[next + l]; pb = doc_off[next + l + 1]; }
  };
  prefetch();
  uint32_t ph = G_IDLE, d = 0, bad = 0;
  uint64_t p = 0, e = 0, slot = 0;
  uint32_t n_left = 0, st_left = 0, cc = 0, clk = 0, clock = 0, count = 0, t = 0, tend = 0, prevc = 0;
  bool stop = false, fst = false, have_prev = false;
  uint64_t payload = 0;
  uint8_t* ob = out;
  for (uint32_t iter = 0;; iter++) {
    if (ph == G_FIN) {
      const uint64_t bm = __ballot(bad != 0u);
      if (bm) {
        uint32_t base = 0;
        if (l == (uint32_t)__builtin_ctzll(bm)) base = atomicAdd(defer_cnt, (uint32_t)__popcll(bm));
        base = (uint32_t)__shfl((int)base, (int)__builtin_ctzll(bm));
        if (bad) { defer_list[base + lanes_below(bm)] = d; status[d] = ST_FALLBACK; }
      }
      if (!bad) {
        const uint32_t hl = dw_vulen(count);
        dw_st16(ob, 0ull, dw_vu_enc(count) << (64u - 8u * hl));
        out_off[d] = slot + 16u - hl; out_len[d] = hl + (t - 16u); status[d] = ST_OK;
        payload += hl + (t - 16u);
      }
      ph = G_IDLE;
    }
    const bool want = ph == G_IDLE;
    const uint64_t wm = __ballot(want);
    if (wm) {
      const uint32_t rank = lanes_below(wm) & 63u;
      const uint64_t na = dw_shfl64(pa, rank), nb = dw_shfl64(pb, rank);
      const uint32_t avail = next < D1 ? D1 - next : 0u;
      const uint32_t npop = (uint32_t)__popcll(wm);
      if (want && rank < avail) {
        d = next + rank; bad = 0; count = 0; have_prev = false;
        p = na; e = nb;
        slot = merge_slot(na, d);
        ob = out + slot;
        const uint64_t cap = merge_slot_cap(nb - na), room = out_cap > slot ? out_cap - slot : 0ull;
        const uint64_t lim = cap < room ? cap : room;
        tend = lim > 16u ? (uint32_t)(lim - 16u) : 0u;
        t = 16u;
        bad |= (nb < na || ((nb - na) >> 30)) ? 1u : 0u;
        ph = bad ? G_FIN : G_UPD;
      }
      if (avail) { next += npop < avail ? npop : avail; prefetch(); }
    }
    if (__ballot(ph != G_IDLE) == 0 && next >= D1) break;
    if (ph == G_IDLE || ph == G_FIN) continue;
    uint32_t v[8], T;
    gw_load(arena, p, v, T);
    const uint32_t b0 = v[0] & 0xFFu;
    if (ph == G_ST) {
      const uint32_t info = b0, hoh = info >> 6, ref = info & 31u;
      const uint32_t T1 = T & ~1u;
      uint32_t len = 0, end = 0;
      bool skip = false;
      if (ref == 0u || info == 10u) {   // GC / Skip: a varuint length
        const uint32_t e1 = gw_ctz(T1);
        bad |= (info != 0u && info != 10u) || e1 > 5u ? 1u : 0u;
        const uint64_t w = gw_at8(v, 1u);
        len = (uint32_t)pext7(w, e1 < 5u ? e1 : 5u);
        bad |= (e1 == 5u && ((uint32_t)(w >> 32) & 0x70u)) || len == 0u ? 1u : 0u;
        end = e1 + 1u;
        skip = info == 10u;
      } else {
        bad |= ((info & 0xC0u) && (info & 0x20u)) || (ref != 1u && ref != 4u) ? 1u : 0u;
        uint32_t cs;
        if (hoh) {   // origin and/or right origin: the content starts after the 2nd / 4th terminator
          const uint32_t c1 = gw_clr(T1), c3 = gw_clr(gw_clr(c1));
          cs = gw_ctz(hoh == 3u ? c3 : c1) + 1u;
        } else {     // parent: y-key string (parentInfo 1) or parent id (0); parentSub string with bit 0x20
          const uint32_t pi = (v[0] >> 8) & 0xFFu;
          bad |= (pi > 1u || !((T >> 1) & 1u)) ? 1u : 0u;
          if (pi == 1u) {
            const uint32_t kl = (v[0] >> 16) & 0xFFu;
            bad |= (!((T >> 2) & 1u) || kl > 28u || ((~T >> 3) & gw_low(kl))) ? 1u : 0u;
            cs = 3u + (kl & 31u);
          } else cs = gw_ctz(gw_clr(T & ~3u)) + 1u;
          if ((info & 0x20u) && cs < 31u) {
            const uint32_t sl = gw_byte(v, cs);
            bad |= (!((T >> cs) & 1u) || sl > 30u || ((~T >> (cs + 1u)) & gw_low(sl))) ? 1u : 0u;
            cs += 1u + (sl & 31u);
          }
        }
        bad |= cs >= 31u ? 1u : 0u;
        const uint32_t cq = cs & 31u;
        const uint32_t lb = gw_byte(v, cq);
        bad |= (!((T >> cq) & 1u) || lb == 0u) ? 1u : 0u;   // a one-byte length
        len = lb;
        end = cq + 1u + (ref == 4u ? lb : 0u);
        if (ref == 4u) bad |= (end > 32u || ((~T >> ((cq + 1u) & 31u)) & gw_low(lb))) ? 1u : 0u;   // ASCII
      }
      // varuints of >= 6 bytes (five non-terminators in a row after the info byte)
      const uint32_t H = ~T & gw_low(end) & ~1u;
      bad |= (H & (H >> 1) & (H >> 2) & (H >> 3) & (H >> 4)) ? 1u : 0u;
      const uint64_t ce64 = (uint64_t)clock + len;
      bad |= (ce64 >> 32) ? 1u : 0u;
      const uint32_t ce = (uint32_t)ce64;
      if (fst && !stop) clk = ce;
      fst = false;
      if (skip) stop = true;
      if (!stop) clk = ce;
      clock = ce;
      p += end;
      if (--st_left == 0u) {
        if (clk) {
          const uint32_t el = dw_vulen(cc) + dw_vulen(clk);
          if (t + el > tend) bad = 1;
          else {
            uint64_t lo = dw_vu_enc(cc), hi = 0;
            uint32_t at = dw_vulen(cc);
            dw_app(lo, hi, at, clk);
            dw_st16(ob + t, lo, hi);
            t += el; count++;
          }
        }
        ph = --n_left ? G_BLK : G_FIN;
      }
    } else if (ph == G_BLK) {   // block header: structs (<= 2 bytes), client, clock
      const uint32_t e1 = gw_ctz(T), x = gw_clr(T), e2 = gw_ctz(x), e3 = gw_ctz(gw_clr(x));
      const uint32_t cn = e2 - e1, kn = e3 - e2;
      const uint64_t cw = gw_at8(v, (e1 + 1u) & 7u), kw = gw_at8(v, (e2 + 1u) & 7u);
      bad |= (e1 > 1u || cn - 1u > 4u || kn - 1u > 4u || e2 + 1u > 7u) ? 1u : 0u;
      bad |= ((cn == 5u && ((uint32_t)(cw >> 32) & 0x70u)) || (kn == 5u && ((uint32_t)(kw >> 32) & 0x70u))) ? 1u : 0u;
      const uint32_t nst = (uint32_t)pext7(gw_at8(v, 0u), e1 + 1u);
      const uint32_t cl = (uint32_t)pext7(cw, cn < 5u ? cn : 5u), ck = (uint32_t)pext7(kw, kn < 5u ? kn : 5u);
      bad |= (nst == 0u || (have_prev && cl >= prevc)) ? 1u : 0u;
      fst = !have_prev;
      prevc = cl; have_prev = true;
      st_left = nst; cc = cl; clock = ck; stop = ck != 0u; clk = 0u;
      p += e3 + 1u;
      ph = G_ST;
    } else {   // G_UPD: the block count
      const uint32_t e1 = gw_ctz(T);
      const uint32_t nb = (uint32_t)pext7(gw_at8(v, 0u), e1 < 5u ? e1 + 1u : 5u);
      bad |= e1 > 3u ? 1u : 0u;
      p += e1 + 1u;
      n_left = nb; have_prev = false;
      ph = nb ? G_BLK : G_FIN;
    }
    if (p > e) bad = 1;
    if (bad) ph = G_FIN;
    else if (ph == G_FIN && MODE == 0) {}   // (the state vector does not read the delete set)
    if (iter > (1u << 28)) break;
  }
  payload = wave_sum(payload);
  if (l == 0 && payload) atomicAdd(payload_out, (unsigned long long)payload);
}

}  // namespace ygm
