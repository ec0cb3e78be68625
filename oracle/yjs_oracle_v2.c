/*
 * yjs_oracle_v2.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 * #included at the end of yjs_oracle.c (shares its decoder, Any / JSON checks, lazy reader and writer).
 *
 * Update format V2: yjs's UpdateDecoderV2 / UpdateEncoderV2 (Y@15400-18900 of the
 * 13.5.16 bundle) over lib0 0.2.42's column coders (chunk 8086: RleDecoder `N`, UintOptRleDecoder `P`,
 * IntDiffOptRleDecoder `G`, StringDecoder `$`; RleEncoder `$`, UintOptRleEncoder `K`,
 * IntDiffOptRleEncoder `H`, StringEncoder `W`).  An update V2 is
 *
 *   varUint 0 | 9 x varUint8Array column (keyClock G, client P, leftClock G, rightClock G, info N,
 *   string $, parentInfo N, typeRef P, len P) | rest (block headers, Skip lengths, Any / Buf content,
 *   the delete set with clocks diff-coded per client: readDsClock += v, readDsLen = v + 1)
 *
 * yjs's V2 functions are its V1 functions with V2 coders: the struct objects they read and the
 * writer calls they make do not depend on the format.  So this file restates the two coders as
 * transcoders, and the V2 operations as  V2 -> V1 -> (the V1 restatement above) -> V1 -> V2:
 *
 *   v2_to_v1   the lazy reader's field-by-field reads through UpdateDecoderV2 (Y@36564 generator,
 *              content readers Y@69266-74200), written out as a V1 update of the same structs; the
 *              JSON values of ContentEmbed / ContentFormat (an Any in V2, a JSON string in V1) become
 *              a placeholder number (an index into a table of their Any bytes) -- yjs re-encodes
 *              them with writeAny(readAny(..)) and never looks inside -- or, for the public
 *              conversion, JSON.stringify of the Any;
 *   v1_to_v2   convertUpdateFormat(V1 -> V2) of yjs 13.6 (lazy reader, writeStructToLazyStructWriter
 *              through UpdateEncoderV2, readDeleteSet / writeDeleteSet), placeholders resolved back to
 *              the Any bytes or, for the public conversion, JSON.parse + writeAny.
 *
 * The column decoders keep JavaScript's reads past a column's end (`arr[pos++]` is undefined): readVarInt
 * returns 0, readVarUint throws, a RleDecoder's last run repeats (and one read past the end throws),
 * UintOptRle returns 0, IntDiffOptRle repeats its value, StringDecoder.read returns "".  Strings are
 * slices of the column's joined string at UTF-16 offsets; a slice that splits a surrogate pair is
 * refused (YO_ENONCANON: its V1 form does not exist), as is a readKey cache hit (keyClock below the
 * keys read so far: only hand-made updates do that; yjs 13.5 and 13.6 read ContentFormat keys
 * differently there).  Pinned by tests/golden/yjs13516_v2_vectors.jsonl.gz (tests/golden/gen/gen_v2.js).
 */

/* ------------------------------------------------ lib0 0.2.42 column decoders */
typedef struct { const uint8_t *a; size_t n, p; } Col;   /* p keeps counting past n, as JS `pos` does */
#define V2_UNDEF (-1)

/* readVarUint (`U`): 32-bit shifts (count mod 32); past the end `undefined < 128` is false -> throw at n > 35 */
static uint32_t col_rdu(Col *c, int *err) {
  uint32_t s = 0; int n = 0;
  for (;;) {
    const int have = c->p < c->n; const uint32_t e = have ? c->a[c->p] : 0; c->p++;
    if (have) s |= (e & 127u) << (n & 31);
    n += 7;
    if (have && e < 128) return s;
    if (n > 35) { if (!*err) *err = YO_EMALFORMED; return 0; }
  }
}
/* readVarInt (`T`): sign in bit 6 of the first byte; returns the magnitude (uint32) and the sign bit */
static uint32_t col_rdi(Col *c, int *neg, int *err) {
  int have = c->p < c->n; uint32_t s = have ? c->a[c->p] : 0; c->p++;
  uint32_t n = s & 63; *neg = (s & 64) != 0;
  if (!(s & 128)) return n;
  int e = 6;
  for (;;) {
    have = c->p < c->n; s = have ? c->a[c->p] : 0; c->p++;
    if (have) n |= (s & 127u) << (e & 31);
    e += 7;
    if (have && s < 128) return n;
    if (e > 41) { if (!*err) *err = YO_EMALFORMED; return 0; }
  }
}
/* ToInt32 of a readVarInt result (+-uint32) */
static int32_t js_i32(uint32_t mag, int neg) { uint32_t v = neg ? (uint32_t)(0u - mag) : mag; return (int32_t)v; }

typedef struct { Col c; int64_t count; int s; } RleD;                /* RleDecoder(readUint8) */
typedef struct { Col c; int64_t count; uint64_t s; } UoD;             /* UintOptRleDecoder */
typedef struct { Col c; int64_t count; int64_t s, diff; } IdD;        /* IntDiffOptRleDecoder */

static int rle_read(RleD *d, int *err) {
  if (d->count == 0) {
    const int have = d->c.p < d->c.n; d->s = have ? d->c.a[d->c.p] : V2_UNDEF; d->c.p++;
    if (d->c.p != d->c.n) d->count = (int64_t)col_rdu(&d->c, err) + 1;   /* hasContent: pos !== length */
    else d->count = -1;
  }
  d->count--;
  return d->s;
}
static uint64_t uo_read(UoD *d, int *err) {
  if (d->count == 0) {
    int neg; const uint32_t m = col_rdi(&d->c, &neg, err);
    d->s = m; d->count = 1;
    if (neg) d->count = (int64_t)col_rdu(&d->c, err) + 2;   /* isNegativeZero-or-negative: a run */
  }
  d->count--;
  return d->s;
}
static int64_t id_read(IdD *d, int *err) {
  if (d->count == 0) {
    int neg; const uint32_t m = col_rdi(&d->c, &neg, err);
    const int32_t t = js_i32(m, neg);
    d->diff = t >> 1; d->count = 1;
    if (t & 1) d->count = (int64_t)col_rdu(&d->c, err) + 2;
  }
  d->s += d->diff;
  d->count--;
  return d->s;
}

typedef struct {
  Dec rest;
  IdD kc, lc, rc; UoD cl, tr, ln, lens; RleD info, pi;
  const uint8_t *str; size_t sn;   /* the joined string (validated UTF-8) */
  size_t sb; uint64_t su;          /* byte / UTF-16 position of StringDecoder.spos */
  uint64_t nkeys;                  /* readKey: keys read so far */
  int err;
} V2Dec;

static void v2_fail(V2Dec *v, int e) { if (!v->err) v->err = e; }
static int v2_err(V2Dec *v) { return v->err ? v->err : v->rest.err; }

/* UpdateDecoderV2 constructor (Y@15400): feature flag, nine columns, the string column decoded eagerly */
static void v2_open(V2Dec *v, const uint8_t *u, size_t n) {
  memset(v, 0, sizeof *v);
  v->rest.a = u; v->rest.n = n;
  rdu(&v->rest);
  Col cols[9];
  for (int i = 0; i < 9; i++) {
    size_t l; const uint8_t *p = rdbuf(&v->rest, &l);
    cols[i].a = p; cols[i].n = l; cols[i].p = 0;
    if (v->rest.err) return;
    if (i == 5) {   /* StringDecoder: readVarString over the column, then the lengths decoder continues */
      Col sc = cols[5]; int e = 0;
      const uint32_t sl = col_rdu(&sc, &e);
      if (e) { v2_fail(v, e); return; }
      /* lib0 0.2.42 readVarString: the first byte, then (length - 1 < 100) byte by byte -- a missing byte is
       * fromCodePoint(undefined), a throw -- or in clamped subarray chunks that never throw.  0.2.104 reads a
       * bounded Uint8Array view: always a throw. */
      size_t avail = sc.p < sc.n ? sc.n - sc.p : 0;
      if (sl > 0 && (avail == 0 || ((sl - 1 < 100 || !(g_flags & YO_COMPAT_135)) && (uint64_t)sl > avail))) { v2_fail(v, YO_EMALFORMED); return; }
      v->str = sc.a + sc.p; v->sn = (uint64_t)sl < avail ? sl : avail; sc.p += sl;
      if (utf8_check(v->str, v->sn) < 0) { v2_fail(v, YO_EMALFORMED); return; }          /* URI malformed */
      v->lens.c = sc;
    }
  }
  v->kc.c = cols[0]; v->cl.c = cols[1]; v->lc.c = cols[2]; v->rc.c = cols[3]; v->info.c = cols[4];
  v->pi.c = cols[6]; v->tr.c = cols[7]; v->ln.c = cols[8];
}
/* StringDecoder.read: str.slice(spos, spos + len) at UTF-16 offsets */
static const uint8_t *v2_string(V2Dec *v, size_t *len) {
  int e = 0;
  const uint64_t L = uo_read(&v->lens, &e);
  if (e) { v2_fail(v, e); *len = 0; return NULL; }
  const size_t b0 = v->sb;
  uint64_t want = L;
  while (want > 0 && v->sb < v->sn) {
    const uint8_t ch = v->str[v->sb];
    const int k = ch < 0x80 ? 1 : (ch & 0xE0) == 0xC0 ? 2 : (ch & 0xF0) == 0xE0 ? 3 : 4;
    if (k == 4) { if (want == 1) { v2_fail(v, YO_ENONCANON); *len = 0; return NULL; } want -= 2; }
    else want -= 1;
    v->sb += (size_t)k;
  }
  v->su += L;
  *len = v->sb - b0;
  return v->str + b0;
}
static uint64_t v2_client(V2Dec *v) { int e = 0; const uint64_t x = uo_read(&v->cl, &e); if (e) v2_fail(v, e); return x; }
static uint64_t v2_len(V2Dec *v) { int e = 0; const uint64_t x = uo_read(&v->ln, &e); if (e) v2_fail(v, e); return x; }
static uint64_t v2_clock(V2Dec *v, IdD *d) {
  int e = 0; const int64_t x = id_read(d, &e);
  if (e) v2_fail(v, e);
  if (x < 0 || (uint64_t)x > MAX_SAFE) v2_fail(v, YO_ENONCANON);   /* a clock V1 cannot carry (hand-made input) */
  return x < 0 ? 0 : (uint64_t)x;
}

/* ---------------------------------------------- Any -> JSON.stringify (public V2 -> V1) */
static void js_quote(Buf *o, const uint8_t *s, size_t n) {
  static const char hx[] = "0123456789abcdef";
  bbyte(o, '"');
  for (size_t i = 0; i < n; i++) {
    const uint8_t c = s[i];
    if (c == '"') bput(o, "\\\"", 2); else if (c == '\\') bput(o, "\\\\", 2);
    else if (c == 8) bput(o, "\\b", 2); else if (c == 9) bput(o, "\\t", 2); else if (c == 10) bput(o, "\\n", 2);
    else if (c == 12) bput(o, "\\f", 2); else if (c == 13) bput(o, "\\r", 2);
    else if (c < 0x20) { char u[6] = { '\\', 'u', '0', '0', hx[c >> 4], hx[c & 15] }; bput(o, u, 6); }
    else bbyte(o, c);
  }
  bbyte(o, '"');
}
/* one Any value (already validated canonical by rd_any) as JSON.stringify writes it; numbers other than
 * varInt integers are refused (their shortest round-trip decimal is not reproduced here) */
static int any_json(Dec *d, Buf *o, int depth) {
  if (depth > ANY_MAX_DEPTH) return YO_EDEPTH;
  const uint8_t tag = rd8(d);
  if (d->err) return d->err;
  switch (tag) {
    case 126: bput(o, "null", 4); return 0;
    case 120: bput(o, "true", 4); return 0;
    case 121: bput(o, "false", 5); return 0;
    case 125: {
      const uint8_t r = rd8(d); uint64_t num = r & 63; int sh = 6; const int neg = (r & 64) != 0;
      if (r & 128) for (;;) { const uint8_t c = rd8(d); if (d->err) return d->err; num |= (uint64_t)(c & 127) << sh; sh += 7; if (c < 128) break; }
      char t[32]; const int k = snprintf(t, sizeof t, "%s%llu", neg && num ? "-" : "", (unsigned long long)num);
      bput(o, t, (size_t)k); return 0;
    }
    case 119: { size_t l; const uint8_t *s = rdbuf(d, &l); if (d->err) return d->err; js_quote(o, s, l); return 0; }
    case 117: {
      const uint64_t n = rdu(d); bbyte(o, '[');
      for (uint64_t i = 0; i < n; i++) { if (i) bbyte(o, ','); const int e = any_json(d, o, depth + 1); if (e) return e; }
      bbyte(o, ']'); return 0;
    }
    case 118: {
      const uint64_t n = rdu(d); bbyte(o, '{');
      for (uint64_t i = 0; i < n; i++) {
        if (i) bbyte(o, ',');
        size_t l; const uint8_t *k = rdbuf(d, &l); if (d->err) return d->err;
        js_quote(o, k, l); bbyte(o, ':');
        const size_t at = d->p; if (at < d->n && d->a[at] == 127) return YO_ENONCANON;   /* undefined member: dropped by stringify */
        const int e = any_json(d, o, depth + 1); if (e) return e;
      }
      bbyte(o, '}'); return 0;
    }
    case 122: return YO_EMALFORMED;   /* JSON.stringify throws on a BigInt */
    default: return YO_ENONCANON;     /* floats, undefined, Uint8Array */
  }
}

/* ---------------------------------------------- JSON.parse -> writeAny (public V1 -> V2) */
/* s is canonical (json_check without nc): no whitespace, keys without escapes, strings with the short
 * escapes or \u00xx for control characters, numbers of <= 15 significant digits without exponent */
static void any_vi(Buf *o, uint64_t m, int neg) {   /* lib0 writeVarInt of a magnitude m < 2^32 */
  bbyte(o, (uint8_t)((m > 63 ? 0x80 : 0) | (neg ? 0x40 : 0) | (m & 63)));
  m >>= 6;
  while (m > 0) { bbyte(o, (uint8_t)((m > 127 ? 0x80 : 0) | (m & 127))); m >>= 7; }
}
static size_t json_str_any(const uint8_t *s, size_t n, size_t i, Buf *o) {   /* s[i] == '"'; writes varString */
  Buf t; memset(&t, 0, sizeof t);
  i++;
  while (i < n && s[i] != '"') {
    if (s[i] == '\\') {
      const uint8_t e = s[i + 1];
      if (e == 'u') { int v = 0; for (int k = 0; k < 4; k++) v = v * 16 + hexv(s[i + 2 + k]); bbyte(&t, (uint8_t)v); i += 6; continue; }
      bbyte(&t, e == 'b' ? 8 : e == 'f' ? 12 : e == 'n' ? 10 : e == 'r' ? 13 : e == 't' ? 9 : e);
      i += 2; continue;
    }
    bbyte(&t, s[i]); i++;
  }
  bstr(o, t.b, t.n); free(t.b);
  return i + 1;
}
static size_t json_any2(const uint8_t *s, size_t n, size_t i, Buf *o);
static size_t json_num_any(const uint8_t *s, size_t n, size_t i, Buf *o) {
  size_t j = i; char b[64]; size_t k = 0;
  while (j < n && (s[j] == '-' || s[j] == '.' || (s[j] >= '0' && s[j] <= '9'))) { if (k < 63) b[k++] = (char)s[j]; j++; }
  b[k] = 0;
  const double x = strtod(b, NULL);
  if (js_small_int(x)) { bbyte(o, 125); any_vi(o, (uint64_t)fmod(fabs(x), 4294967296.0), x < 0); }
  else if ((double)(float)x == x) { const float f = (float)x; uint32_t u; memcpy(&u, &f, 4); bbyte(o, 124); for (int q = 3; q >= 0; q--) bbyte(o, (uint8_t)(u >> (8 * q))); }
  else { uint64_t u; memcpy(&u, &x, 8); bbyte(o, 123); for (int q = 7; q >= 0; q--) bbyte(o, (uint8_t)(u >> (8 * q))); }
  return j;
}
static size_t json_any2(const uint8_t *s, size_t n, size_t i, Buf *o) {
  const uint8_t c = s[i];
  if (c == '{' || c == '[') {
    size_t cnt = 0, j = i + 1; int dpt = 0, instr = 0;
    if (s[j] != (c == '{' ? '}' : ']')) {
      cnt = 1;
      for (; j < n; j++) {
        const uint8_t ch = s[j];
        if (instr) { if (ch == '\\') j++; else if (ch == '"') instr = 0; continue; }
        if (ch == '"') instr = 1;
        else if (ch == '{' || ch == '[') dpt++;
        else if (ch == '}' || ch == ']') { if (dpt == 0) break; dpt--; }
        else if (ch == ',' && dpt == 0) cnt++;
      }
    }
    bbyte(o, c == '{' ? 118 : 117); bvu(o, cnt);
    i++;
    if (cnt == 0) return i + 1;
    for (size_t k = 0; k < cnt; k++) {
      if (c == '{') { i = json_str_any(s, n, i, o); i++; }
      i = json_any2(s, n, i, o);
      i++;
    }
    return i;
  }
  if (c == '"') { bbyte(o, 119); return json_str_any(s, n, i, o); }
  if (c == 't') { bbyte(o, 120); return i + 4; }
  if (c == 'f') { bbyte(o, 121); return i + 5; }
  if (c == 'n') { bbyte(o, 126); return i + 4; }
  return json_num_any(s, n, i, o);
}
/* writeAny(JSON.parse(s)) */
static void json_to_any(const uint8_t *s, size_t n, Buf *o) { json_any2(s, n, 0, o); }

/* ---------------------------------------------- V2 -> V1 */
/* JSON values of embeds / formats: placeholders into this table (internal transcoding) */
typedef struct { const uint8_t **p; size_t *n; size_t cnt, cap; } JTab;
static size_t jtab_add(JTab *t, const uint8_t *p, size_t n) {
  if (t->cnt == t->cap) { t->cap = t->cap ? 2 * t->cap : 16; t->p = (const uint8_t **)realloc(t->p, t->cap * sizeof *t->p); t->n = (size_t *)realloc(t->n, t->cap * sizeof *t->n); }
  t->p[t->cnt] = p; t->n[t->cnt] = n; return t->cnt++;
}
static void jtab_free(JTab *t) { free(t->p); free(t->n); memset(t, 0, sizeof *t); }

/* readJSON of the V2 decoder (readAny) written as the V1 JSON string: a placeholder (jt != NULL) -- " N"
 * with a leading blank when writeAny would not reproduce the Any, so the V1 layer refuses the struct
 * exactly when it writes it -- or JSON.stringify of the value */
static int v2_json(V2Dec *v, Buf *o, JTab *jt) {
  const size_t a = v->rest.p; int nc = 0;
  v->rest.nm = 0; rd_any(&v->rest, 0, &nc);
  if (v->rest.err) return v->rest.err;
  if (v->rest.nm) nc = 1;
  if (jt) {
    char t[32]; const size_t id = jtab_add(jt, v->rest.a + a, v->rest.p - a);
    const int k = snprintf(t, sizeof t, "%s%zu", nc ? " " : "", id);
    bstr(o, (const uint8_t *)t, (size_t)k);
    return 0;
  }
  if (nc) return YO_ENONCANON;
  Dec q = { v->rest.a + a, v->rest.p - a, 0, 0, 0 };
  Buf j; memset(&j, 0, sizeof j);
  const int e = any_json(&q, &j, 0);
  if (!e) bstr(o, j.b, j.n);
  free(j.b);
  return e;
}

/* Transcodes one V2 update into V1 (same blocks, structs, info bytes and delete set entries).
 * structs_only: stop after the structs (encodeStateVectorFromUpdateV2 reads no delete set) and write
 * an empty delete set. */
static int v2_to_v1(const uint8_t *u, size_t n, Buf *o, JTab *jt, int structs_only) {
  V2Dec V; V2Dec *v = &V;
  v2_open(v, u, n);
  if (v2_err(v)) return v2_err(v);
  const uint64_t nb = rdu(&v->rest); bvu(o, nb);
  for (uint64_t b = 0; b < nb && !v2_err(v); b++) {
    const uint64_t ns = rdu(&v->rest); const uint64_t client = v2_client(v); const uint64_t clock = rdu(&v->rest);
    if (v2_err(v)) break;
    bvu(o, ns); bvu(o, client); bvu(o, clock);
    for (uint64_t s = 0; s < ns && !v2_err(v); s++) {
      int e = 0; const int info = rle_read(&v->info, &e);
      if (e) { v2_fail(v, e); break; }
      if (info == 10) { const uint64_t l = rdu(&v->rest); bbyte(o, 10); bvu(o, l); continue; }
      if (info == V2_UNDEF || (info & 31) == 0) { bbyte(o, 0); bvu(o, v2_len(v)); continue; }   /* GC */
      bbyte(o, (uint8_t)info);
      const int cant_copy = (info & 0xC0) == 0;
      if (info & 0x80) { bvu(o, v2_client(v)); bvu(o, v2_clock(v, &v->lc)); }
      if (info & 0x40) { bvu(o, v2_client(v)); bvu(o, v2_clock(v, &v->rc)); }
      if (cant_copy) {
        const int p = rle_read(&v->pi, &e); if (e) { v2_fail(v, e); break; }
        if (p == 1) { size_t l; const uint8_t *t = v2_string(v, &l); bvu(o, 1); bstr(o, t, l); }
        else { bvu(o, 0); bvu(o, v2_client(v)); bvu(o, v2_clock(v, &v->lc)); }
        if (info & 0x20) { size_t l; const uint8_t *t = v2_string(v, &l); bstr(o, t, l); }
      }
      if (v2_err(v)) break;
      switch (info & 31) {
        case 1: bvu(o, v2_len(v)); break;                                        /* ContentDeleted */
        case 2: { const uint64_t k = v2_len(v); bvu(o, k);                       /* ContentJSON */
          for (uint64_t i = 0; i < k && !v2_err(v); i++) { size_t l; const uint8_t *t = v2_string(v, &l); if (v2_err(v)) break; bstr(o, t, l);
            if (!(l == 9 && !memcmp(t, "undefined", 9))) { int nc = 0; const int je = json_check(t, l, &nc); if (je) v2_fail(v, je); } }
          break; }
        case 3: { size_t l; const uint8_t *t = rdbuf(&v->rest, &l); if (!v->rest.err) bstr(o, t, l); break; }   /* ContentBinary */
        case 4: { size_t l; const uint8_t *t = v2_string(v, &l); bstr(o, t, l); break; }                     /* ContentString */
        case 5: { const int je = v2_json(v, o, jt); if (je) v2_fail(v, je); break; }                         /* ContentEmbed */
        case 6: { size_t l; const uint8_t *t = v2_string(v, &l); if (v2_err(v)) break; bstr(o, t, l);      /* ContentFormat */
          const int je = v2_json(v, o, jt); if (je) v2_fail(v, je); break; }
        case 7: { const uint64_t tr = uo_read(&v->tr, &e); if (e) { v2_fail(v, e); break; }                  /* ContentType */
          if (tr > 6) { v2_fail(v, YO_EMALFORMED); break; }   /* typeRefs[tr] is not a function */
          bvu(o, tr);
          if (tr == 3 || tr == 5) {   /* readKey */
            const int64_t kc = id_read(&v->kc, &e); if (e) { v2_fail(v, e); break; }
            if (kc < 0 || (uint64_t)kc < v->nkeys) { v2_fail(v, YO_ENONCANON); break; }
            size_t l; const uint8_t *t = v2_string(v, &l); bstr(o, t, l); v->nkeys++;
          }
          break; }
        case 8: { const uint64_t k = v2_len(v); bvu(o, k);                                                  /* ContentAny */
          const size_t a = v->rest.p; int nc = 0;
          for (uint64_t i = 0; i < k && !v2_err(v); i++) rd_any(&v->rest, 0, &nc);
          if (!v2_err(v)) bput(o, v->rest.a + a, v->rest.p - a);
          break; }
        case 9: { size_t l; const uint8_t *t = v2_string(v, &l); if (v2_err(v)) break; bstr(o, t, l);      /* ContentDoc */
          const size_t a = v->rest.p; int nc = 0; rd_any(&v->rest, 0, &nc);
          if (!v2_err(v)) bput(o, v->rest.a + a, v->rest.p - a);
          break; }
        default: v2_fail(v, YO_EMALFORMED); break;   /* contentRefs[10] -> unexpectedCase */
      }
    }
  }
  if (v2_err(v)) return v2_err(v);
  if (structs_only) { bvu(o, 0); return o->oom ? YO_ENOMEM : 0; }
  /* readDeleteSet through the V2 decoder: clocks diff-coded per client, lengths + 1 */
  const uint64_t nc = rdu(&v->rest); bvu(o, nc);
  for (uint64_t i = 0; i < nc && !v2_err(v); i++) {
    uint64_t cur = 0;
    const uint64_t client = rdu(&v->rest), nd = rdu(&v->rest);
    if (v2_err(v)) break;
    bvu(o, client); bvu(o, nd);
    for (uint64_t k = 0; k < nd && !v2_err(v); k++) {
      cur += rdu(&v->rest); const uint64_t clock = cur;
      const uint64_t len = rdu(&v->rest) + 1; cur += len;
      if (cur > MAX_SAFE) { v2_fail(v, YO_ERANGE); break; }
      bvu(o, clock); bvu(o, len);
    }
  }
  if (v2_err(v)) return v2_err(v);
  return o->oom ? YO_ENOMEM : 0;
}

/* ---------------------------------------------- V1 -> V2 (UpdateEncoderV2 + lazy writer) */
typedef struct { Buf b; int64_t count; int s; } RleE;               /* RleEncoder(writeUint8), s = -1: null */
typedef struct { Buf b; int64_t count; uint64_t s; } UoE;            /* UintOptRleEncoder */
typedef struct { Buf b; int64_t count; int64_t s, diff; } IdE;       /* IntDiffOptRleEncoder */
static void rle_w(RleE *e, int v) {
  if (e->s == v) { e->count++; return; }
  if (e->count > 0) bvu(&e->b, (uint64_t)(e->count - 1));
  e->count = 1; bbyte(&e->b, (uint8_t)v); e->s = v;
}
static void uo_flush(UoE *e) {
  if (e->count > 0) { any_vi(&e->b, e->s & 0xFFFFFFFFull, e->count != 1); if (e->count > 1) bvu(&e->b, (uint64_t)(e->count - 2)); }
}
static void uo_w(UoE *e, uint64_t v) { if (e->s == v) { e->count++; return; } uo_flush(e); e->count = 1; e->s = v; }
static void id_flush(IdE *e) {
  if (e->count > 0) {
    const int32_t v = (int32_t)(((uint32_t)(int32_t)(uint32_t)(uint64_t)e->diff << 1) | (e->count == 1 ? 0u : 1u));   /* diff << 1 | run (int32) */
    any_vi(&e->b, v < 0 ? (uint64_t)(0u - (uint32_t)v) : (uint64_t)v, v < 0);
    if (e->count > 1) bvu(&e->b, (uint64_t)(e->count - 2));
  }
}
static void id_w(IdE *e, int64_t v) { if (e->diff == v - e->s) { e->s = v; e->count++; return; } id_flush(e); e->count = 1; e->diff = v - e->s; e->s = v; }

typedef struct {
  IdE kc, lc, rc; UoE cl, tr, ln, lens; RleE info, pi;
  Buf str;           /* joined string */
  uint64_t keyclock;
  /* lazy writer: rest parts per client block */
  Buf rest; uint64_t written, curr_client;
  Buf parts; uint64_t nparts;
  int err, nc;
} V2Enc;
static void v2e_str(V2Enc *w, const uint8_t *s, size_t n) { bput(&w->str, s, n); uo_w(&w->lens, (uint64_t)utf8_check(s, n)); }
static void v2e_key(V2Enc *w, const uint8_t *s, size_t n) { id_w(&w->kc, (int64_t)w->keyclock++); v2e_str(w, s, n); }
/* writeJSON(JSON.parse(s)) or the placeholder's Any bytes */
static int v2e_json(V2Enc *w, const uint8_t *s, size_t n, const JTab *jt) {
  if (jt) {
    size_t i = 0; while (i < n && s[i] == ' ') i++;
    size_t id = 0; for (; i < n; i++) id = id * 10 + (size_t)(s[i] - '0');
    if (id >= jt->cnt) return YO_EMALFORMED;
    bput(&w->rest, jt->p[id], jt->n[id]);
    return 0;
  }
  json_to_any(s, n, &w->rest);
  return 0;
}
/* Item.write / GC.write / Skip.write through UpdateEncoderV2 (Y@80416, Y@68955, Y@81211) */
static int v2e_struct(V2Enc *w, const St *s, const JTab *jt) {
  if (s->kind == K_GC) { rle_w(&w->info, 0); uo_w(&w->ln, s->len); return 0; }
  if (s->kind == K_SKIP) { rle_w(&w->info, 10); bvu(&w->rest, s->len); return 0; }
  if (s->nc) return YO_ENONCANON;
  const uint8_t info = (uint8_t)((s->ref & 31) | (s->has_origin ? 0x80 : 0) | (s->has_right ? 0x40 : 0) | (s->has_sub ? 0x20 : 0));
  rle_w(&w->info, info);
  if (s->has_origin) { uo_w(&w->cl, s->oc); id_w(&w->lc, (int64_t)s->ok); }
  if (s->has_right) { uo_w(&w->cl, s->rc); id_w(&w->rc, (int64_t)s->rk); }
  if (!s->has_origin && !s->has_right) {
    if (s->parent_is_key) { rle_w(&w->pi, 1); v2e_str(w, s->pkey, s->pkey_len); }
    else { rle_w(&w->pi, 0); uo_w(&w->cl, s->pc); id_w(&w->lc, (int64_t)s->pk); }
    if (s->has_sub) v2e_str(w, s->sub, s->sub_len);
  }
  Dec d = { s->content, s->content_len, 0, 0, 0 };
  switch (s->ref) {
    case 1: uo_w(&w->ln, rdu(&d)); return 0;
    case 2: { const uint64_t k = rdu(&d); uo_w(&w->ln, k); for (uint64_t i = 0; i < k; i++) { size_t l; const uint8_t *t = rdbuf(&d, &l); v2e_str(w, t, l); } return 0; }
    case 3: { size_t l; const uint8_t *t = rdbuf(&d, &l); bstr(&w->rest, t, l); return 0; }
    case 4: { size_t l; const uint8_t *t = rdbuf(&d, &l); v2e_str(w, t, l); return 0; }
    case 5: { size_t l; const uint8_t *t = rdbuf(&d, &l); return v2e_json(w, t, l, jt); }
    case 6: { size_t l; const uint8_t *t = rdbuf(&d, &l); v2e_key(w, t, l); t = rdbuf(&d, &l); return v2e_json(w, t, l, jt); }
    case 7: { const uint64_t tr = rdu(&d); uo_w(&w->tr, tr); if (tr == 3 || tr == 5) { size_t l; const uint8_t *t = rdbuf(&d, &l); v2e_key(w, t, l); } return 0; }
    case 8: { const uint64_t k = rdu(&d); uo_w(&w->ln, k); bput(&w->rest, d.a + d.p, d.n - d.p); return 0; }
    case 9: { size_t l; const uint8_t *t = rdbuf(&d, &l); v2e_str(w, t, l); bput(&w->rest, d.a + d.p, d.n - d.p); return 0; }
  }
  return YO_EMALFORMED;
}
static void v2e_flush(V2Enc *w) {
  if (w->written > 0) { bvu(&w->parts, w->written); bput(&w->parts, w->rest.b, w->rest.n); w->nparts++; w->rest.n = 0; w->written = 0; }
}
static void v2e_write(V2Enc *w, const St *s, const JTab *jt) {   /* writeStructToLazyStructWriter(w, s, 0) */
  if (w->err) return;
  if (w->written > 0 && w->curr_client != s->client) v2e_flush(w);
  if (w->written == 0) { w->curr_client = s->client; uo_w(&w->cl, s->client); bvu(&w->rest, s->clock); }
  const int e = v2e_struct(w, s, jt);
  if (e == YO_ENONCANON) w->nc = 1; else if (e) w->err = e;
  w->written++;
}
static void v2e_col(Buf *o, Buf *c) { bstr(o, c->b, c->n); }
static void v2e_free(V2Enc *w) {
  Buf *bs[] = { &w->kc.b, &w->lc.b, &w->rc.b, &w->cl.b, &w->tr.b, &w->ln.b, &w->lens.b, &w->info.b, &w->pi.b, &w->str, &w->rest, &w->parts };
  for (size_t i = 0; i < sizeof bs / sizeof *bs; i++) free(bs[i]->b);
}
/* convertUpdateFormat(u, id, UpdateDecoderV1, UpdateEncoderV2) -- yjs 13.6 convertUpdateFormatV1ToV2 */
static int v1_to_v2(const uint8_t *u, size_t n, Buf *o, const JTab *jt, int flags) {
  V2Enc W; memset(&W, 0, sizeof W); V2Enc *w = &W;
  w->info.s = -1; w->pi.s = -1;
  Reader r; reader_init(&r, u, n, 0);
  int err = r.d.err;
  while (!err && r.has_cur) {
    v2e_write(w, &r.cur, jt);
    reader_next(&r); err = r.d.err;
    if (!err && w->err) err = w->err;
  }
  if (!err) {
    v2e_flush(w);
    /* finishLazyStructWriting: the rest gets the part count, then every part */
    Buf rest; memset(&rest, 0, sizeof rest);
    bvu(&rest, w->nparts); bput(&rest, w->parts.b, w->parts.n);
    /* readDeleteSet (V1) / writeDeleteSet (V2: resetDsCurVal per client, clock deltas, lengths - 1) */
    DS ds; memset(&ds, 0, sizeof ds);
    ds_read(&r.d, &ds); err = r.d.err;
    if (!err) {
      bvu(&rest, ds.n);
      size_t *ord = (size_t *)malloc((ds.n + 1) * sizeof(size_t));
      for (size_t i = 0; i < ds.n; i++) ord[i] = i;
      if (!(flags & YO_COMPAT_135))
        for (size_t i = 1; i < ds.n; i++) { size_t t = ord[i]; size_t j = i; while (j > 0 && ds.c[ord[j - 1]].client < ds.c[t].client) { ord[j] = ord[j - 1]; j--; } ord[j] = t; }
      for (size_t q = 0; q < ds.n && !err; q++) {
        const DClient *c = &ds.c[ord[q]];
        bvu(&rest, c->client); bvu(&rest, c->n);
        uint64_t cur = 0;
        for (size_t k = 0; k < c->n; k++) {
          const int64_t dl = (int64_t)c->it[k].clock - (int64_t)cur;
          if (dl < 0) bbyte(&rest, (uint8_t)(dl & 127)); else bvu(&rest, (uint64_t)dl);   /* writeVarUint(negative): one byte */
          cur = c->it[k].clock;
          if (c->it[k].len == 0) { err = YO_EMALFORMED; break; }   /* writeDsLen(0): unexpectedCase */
          bvu(&rest, c->it[k].len - 1); cur += c->it[k].len;
        }
      }
      free(ord);
    }
    ds_free(&ds);
    if (!err) {
      /* UpdateEncoderV2.toUint8Array: flag 0, the nine columns, then the rest */
      bvu(o, 0);
      id_flush(&w->kc); v2e_col(o, &w->kc.b);
      uo_flush(&w->cl); v2e_col(o, &w->cl.b);
      id_flush(&w->lc); v2e_col(o, &w->lc.b);
      id_flush(&w->rc); v2e_col(o, &w->rc.b);
      v2e_col(o, &w->info.b);
      Buf sc; memset(&sc, 0, sizeof sc);
      bstr(&sc, w->str.b, w->str.n); uo_flush(&w->lens); bput(&sc, w->lens.b.b, w->lens.b.n);
      v2e_col(o, &sc); free(sc.b);
      v2e_col(o, &w->pi.b);
      uo_flush(&w->tr); v2e_col(o, &w->tr.b);
      uo_flush(&w->ln); v2e_col(o, &w->ln.b);
      bput(o, rest.b, rest.n);
    }
    free(rest.b);
  }
  if (!err && w->nc) err = YO_ENONCANON;
  v2e_free(w);
  if (!err && o->oom) err = YO_ENOMEM;
  return err;
}

/* yjs 13.6 convertUpdateFormat(V1 -> V1) through the lazy writer: the normal form v2_to_v1 must take
 * for the public conversion (same-client blocks joined, info bytes and the delete set rewritten) */
static int v1_normalize(const uint8_t *u, size_t n, Buf *o, int flags) {
  LWriter W; memset(&W, 0, sizeof W);
  Reader r; reader_init(&r, u, n, 0);
  int err = r.d.err;
  while (!err && r.has_cur) { lw_write(&W, &r.cur, 0, flags); reader_next(&r); err = r.d.err; if (!err && W.err) err = W.err; }
  if (!err) {
    lw_finish(&W, o);
    DS ds; memset(&ds, 0, sizeof ds);
    ds_read(&r.d, &ds); err = r.d.err;
    if (!err) ds_write(o, &ds, flags);
    ds_free(&ds);
  }
  if (!err && W.nc) err = YO_ENONCANON;
  lw_free(&W);
  return err;
}

static int take(Buf *b, int err, uint8_t **out, size_t *out_len) {
  if (!err && b->oom) err = YO_ENOMEM;
  if (err) { free(b->b); return err; }
  if (!b->b) { b->b = (uint8_t *)malloc(1); }
  *out = b->b; *out_len = b->n;
  return 0;
}

/* ---------------------------------------------- public functions */
/* mergeUpdatesV2(us) (Y@39011 with UpdateDecoderV2 / UpdateEncoderV2) */
int yo_merge_v2(const uint8_t *const *ups, const size_t *lens, size_t n, int flags, uint8_t **out, size_t *out_len) {
  g_flags = flags;
  *out = NULL; *out_len = 0;
  if (n == 1) { Buf b; memset(&b, 0, sizeof b); bput(&b, ups[0], lens[0]); return take(&b, 0, out, out_len); }
  JTab jt; memset(&jt, 0, sizeof jt);
  Buf *v1 = (Buf *)calloc(n ? n : 1, sizeof(Buf));
  int err = 0, refuse = 0;
  for (size_t i = 0; i < n; i++) {   /* a throw in any input wins over a refusal in another */
    const int e = v2_to_v1(ups[i], lens[i], &v1[i], &jt, 0);
    if (e == YO_ENONCANON) { if (!refuse) refuse = e; }
    else if (e && !err) err = e;
  }
  if (!err) err = refuse;
  Buf res; memset(&res, 0, sizeof res);
  if (!err) {
    const uint8_t **p = (const uint8_t **)malloc((n ? n : 1) * sizeof *p); size_t *l = (size_t *)malloc((n ? n : 1) * sizeof *l);
    for (size_t i = 0; i < n; i++) { p[i] = v1[i].b ? v1[i].b : (const uint8_t *)""; l[i] = v1[i].n; }
    uint8_t *m = NULL; size_t ml = 0;
    err = yo_merge(p, l, n, flags, &m, &ml);
    g_flags = flags;
    if (!err) err = v1_to_v2(m, ml, &res, &jt, flags);
    free(m); free(p); free(l);
  }
  for (size_t i = 0; i < n; i++) free(v1[i].b);
  free(v1); jtab_free(&jt);
  return take(&res, err, out, out_len);
}

/* diffUpdateV2(u, sv) (Y@40711) */
int yo_diff_v2(const uint8_t *u, size_t ulen, const uint8_t *sv, size_t svlen, int flags, uint8_t **out, size_t *out_len) {
  g_flags = flags;
  *out = NULL; *out_len = 0;
  JTab jt; memset(&jt, 0, sizeof jt);
  Buf v1; memset(&v1, 0, sizeof v1); Buf res; memset(&res, 0, sizeof res);
  int err = v2_to_v1(u, ulen, &v1, &jt, 0);
  if (!err) {
    uint8_t *m = NULL; size_t ml = 0;
    err = yo_diff(v1.b ? v1.b : (const uint8_t *)"", v1.n, sv, svlen, flags, &m, &ml);
    g_flags = flags;
    if (!err) err = v1_to_v2(m, ml, &res, &jt, flags);
    free(m);
  }
  free(v1.b); jtab_free(&jt);
  return take(&res, err, out, out_len);
}

/* encodeStateVectorFromUpdateV2(u) (Y@37728): reads the structs only */
int yo_sv_v2(const uint8_t *u, size_t ulen, int flags, uint8_t **out, size_t *out_len) {
  g_flags = flags;
  *out = NULL; *out_len = 0;
  JTab jt; memset(&jt, 0, sizeof jt);
  Buf v1; memset(&v1, 0, sizeof v1);
  int err = v2_to_v1(u, ulen, &v1, &jt, 1);
  jtab_free(&jt);
  if (err) { free(v1.b); return err; }
  err = yo_sv(v1.b ? v1.b : (const uint8_t *)"", v1.n, flags, out, out_len);
  free(v1.b);
  return err;
}

/* yjs 13.6 convertUpdateFormatV1ToV2 / convertUpdateFormatV2ToV1 */
int yo_v1_to_v2(const uint8_t *u, size_t ulen, int flags, uint8_t **out, size_t *out_len) {
  g_flags = flags;
  *out = NULL; *out_len = 0;
  Buf res; memset(&res, 0, sizeof res);
  const int err = v1_to_v2(u, ulen, &res, NULL, flags);
  return take(&res, err, out, out_len);
}
int yo_v2_to_v1(const uint8_t *u, size_t ulen, int flags, uint8_t **out, size_t *out_len) {
  g_flags = flags;
  *out = NULL; *out_len = 0;
  Buf v1; memset(&v1, 0, sizeof v1); Buf res; memset(&res, 0, sizeof res);
  int err = v2_to_v1(u, ulen, &v1, NULL, 0);
  if (!err) err = v1_normalize(v1.b ? v1.b : (const uint8_t *)"", v1.n, &res, flags);
  free(v1.b);
  return take(&res, err, out, out_len);
}
