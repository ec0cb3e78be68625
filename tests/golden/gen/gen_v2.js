// Golden vectors for the update-V2 codec (SURVEY.md §8f-4; test-fixture tooling, build container only).
//
// Drives the yjs 13.5.16 bundle (tools/yjs_bundle.js) and records, as hex:
//   mergeUpdatesV2(us)                 (Y@39011 with UpdateDecoderV2 / UpdateEncoderV2)
//   diffUpdateV2(u, sv)                (Y@40711)
//   encodeStateVectorFromUpdateV2(u)   (Y@37728)
//   conv pairs {v1, v2}: the same writer calls through UpdateEncoderV1 and UpdateEncoderV2 -- a
//     transaction's 'update' / 'updateV2' events, encodeStateAsUpdate / encodeStateAsUpdateV2 of one
//     document, mergeUpdates / mergeUpdatesV2 of corresponding logs -- which pin yjs 13.6's
//     convertUpdateFormatV1ToV2 / V2ToV1 (not exported by 13.5.16) on lazy-writer-normal updates.
// Sessions are random multi-client Y.Doc edits (text with formats / embeds, arrays of Any and binary,
// maps with nested types and sub-documents, XmlFragment trees with attributes and hooks); then
// truncated and byte-flipped V2 inputs.
//
// Usage:  node tests/golden/gen/gen_v2.js [out.jsonl.gz]
'use strict'
const zlib = require('zlib')
const fs = require('fs')
const path = require('path')
const { load } = require('../../../tools/yjs_bundle')
const Y = load()

function mulberry32 (a) {
  return function () {
    a |= 0; a = a + 0x6D2B79F5 | 0
    let t = Math.imul(a ^ a >>> 15, 1 | a)
    t = t + Math.imul(t ^ t >>> 7, 61 | t) ^ t
    return ((t ^ t >>> 14) >>> 0) / 4294967296
  }
}
const rnd = mulberry32(20261017)
const ri = n => Math.floor(rnd() * n)
const pick = a => a[ri(a.length)]
const hex = u => Buffer.from(u).toString('hex')
function shuffle (a) { a = a.slice(); for (let i = a.length - 1; i > 0; i--) { const j = ri(i + 1); const t = a[i]; a[i] = a[j]; a[j] = t } return a }

const cases = []
function run (c, f) {
  try { c.out = hex(f()); c.err = null } catch (e) { c.out = null; c.err = String(e && e.message) }
  cases.push(c)
  return c.out
}
const merge2 = (family, us, note) => run({ family, op: 'merge_v2', in: us.map(hex), note }, () => Y.mergeUpdatesV2(us))
const diff2 = (family, u, sv, note) => run({ family, op: 'diff_v2', update: hex(u), sv: hex(sv), note }, () => Y.diffUpdateV2(u, sv))
const sv2 = (family, u, note) => run({ family, op: 'sv_v2', update: hex(u), note }, () => Y.encodeStateVectorFromUpdateV2(u))
// conversion pairs in the lazy writer's normal form: an update re-written by a two-input merge with an
// empty update (the V1 and V2 merges read the same structs and make the same writer calls)
const E1 = Y.encodeStateAsUpdate(new Y.Doc()); const E2 = Y.encodeStateAsUpdateV2(new Y.Doc())
const conv = (family, v1, v2, note) => cases.push({ family, op: 'conv', v1: hex(Y.mergeUpdates([v1, E1])), v2: hex(Y.mergeUpdatesV2([v2, E2])), note })

const ASCII = 'abcdefghijklmnopqrstuvwxyz ABCDEFG0123456789.,!?'
const UNI = ['é', 'ß', '中', '😀', '👍🏽', '𝄞', 'Ω', '\u0000', '"', '\\', '\n', ' ']
function randStr (maxLen, uni) {
  const n = 1 + ri(maxLen); let s = ''
  for (let i = 0; i < n; i++) s += (uni && rnd() < 0.25) ? pick(UNI) : ASCII[ri(ASCII.length)]
  return s
}
function randAny (depth) {
  switch (ri(depth > 0 ? 13 : 10)) {
    case 0: return ri(100)
    case 1: return -ri(1 << 20)
    case 2: return ri(2147483647)
    case 3: return rnd() * 1000
    case 4: return pick([0.5, 1.5, -2.25, 1e-7, 1e300])
    case 5: return randStr(6, true)
    case 6: return rnd() < 0.5
    case 7: return null
    case 8: return ''
    case 9: return new Uint8Array([ri(256), ri(256), ri(256)])
    case 10: { const o = {}; const n = ri(4); for (let i = 0; i < n; i++) o[pick(['a', 'b', 'key', 'x y', 'é'])] = randAny(depth - 1); return o }
    case 11: { const a = []; const n = ri(4); for (let i = 0; i < n; i++) a.push(randAny(depth - 1)); return a }
    default: return [randAny(depth - 1)]
  }
}
// format / embed values: JSON-able; floats included (V2 carries them as Any float32 / float64)
const FORMATS = [{ bold: true }, { italic: 1.5 }, { bold: null }, { link: { href: 'https://x.y/1' } }, { size: 12 }, { color: 'réd' },
  { font: { family: 'a"b', w: -3 } }, { tags: ['x', 2, false] }]
const EMBEDS = [{ image: 'a.png' }, { video: { src: 'v', w: 7 } }, 'emb', { n: 2.5 }, [1, 'two'], { esc: 'q"\\\n\u0001' }]

function session (nClients, nOps, kinds, syncP) {
  const docs = []; const logs1 = []; const logs2 = []
  for (let i = 0; i < nClients; i++) {
    const d = new Y.Doc(); d.clientID = pick([1 + ri(9), 100 + ri(1000), ri(2 ** 31), 2 ** 31 + ri(2 ** 31), 4294967295 - ri(3)])
    while (docs.some(o => o.clientID === d.clientID)) d.clientID++
    const l1 = []; const l2 = []
    d.on('update', (u, origin) => { if (origin !== 'remote') l1.push(u) })
    d.on('updateV2', (u, origin) => { if (origin !== 'remote') l2.push(u) })
    docs.push(d); logs1.push(l1); logs2.push(l2)
  }
  for (let op = 0; op < nOps; op++) {
    const d = docs[ri(nClients)]
    const k = pick(kinds)
    d.transact(() => {
      if (k === 'text') {
        const t = d.getText('t'); const L = t.length; const r = rnd()
        if (r < 0.5 || L === 0) t.insert(ri(L + 1), randStr(4, true), rnd() < 0.3 ? pick(FORMATS) : undefined)
        else if (r < 0.75) { const p = ri(L); t.delete(p, 1 + ri(Math.min(3, L - p))) } else if (r < 0.9) { const p = ri(L); t.format(p, 1 + ri(Math.min(3, L - p)), pick(FORMATS)) } else t.insertEmbed(ri(L + 1), pick(EMBEDS))
      } else if (k === 'array') {
        const a = d.getArray('a'); const L = a.length; const r = rnd()
        if (r < 0.6 || L === 0) { const n = 1 + ri(3); const vals = []; for (let i = 0; i < n; i++) vals.push(randAny(2)); a.insert(ri(L + 1), vals) } else if (r < 0.85) { const p = ri(L); a.delete(p, 1 + ri(Math.min(2, L - p))) } else { a.insert(ri(L + 1), [pick([new Y.Map(), new Y.Array(), new Y.Text('nt'), new Y.XmlText()])]) }
      } else if (k === 'map') {
        const m = d.getMap('m'); const r = rnd(); const key = pick(['a', 'b', 'c', 'long key ' + ri(3), 'é'])
        if (r < 0.7) m.set(key, randAny(2)); else if (r < 0.8) m.set(key, pick([new Y.Map(), new Y.Array(), new Y.Text()])); else if (r < 0.9) { const sd = new Y.Doc({ guid: 'sub-' + ri(100), gc: rnd() < 0.5, autoLoad: rnd() < 0.5 }); m.set(key, sd) } else m.delete(key)
      } else if (k === 'xml') {
        const f = d.getXmlFragment('prosemirror'); const L = f.length; const r = rnd()
        if (r < 0.45 || L === 0) { const el = new Y.XmlElement(pick(['paragraph', 'heading', 'blockquote', 'p'])); el.setAttribute('level', String(ri(3))); const tx = new Y.XmlText(); el.insert(0, [tx]); f.insert(ri(L + 1), [el]); tx.insert(0, randStr(5, true)); if (rnd() < 0.5) tx.format(0, 1, pick(FORMATS)) } else if (r < 0.7) { const el = f.get(ri(L)); if (el instanceof Y.XmlElement && el.length > 0) { const tx = el.get(0); if (tx instanceof Y.XmlText) { const tl = tx.length; if (rnd() < 0.6 || tl === 0) tx.insert(ri(tl + 1), randStr(3, true), rnd() < 0.3 ? { italic: true } : undefined); else tx.delete(ri(tl), 1) } } } else if (r < 0.8) { const p = ri(L); f.delete(p, 1) } else if (r < 0.9) { f.insert(ri(L + 1), [new Y.XmlHook(pick(['mention', 'card']))]) } else { const el = f.get(ri(L)); if (el instanceof Y.XmlElement) el.setAttribute(pick(['class', 'level', 'id']), randStr(3, false)) }
      } else if (k === 'bin') {
        const a = d.getArray('b'); a.insert(ri(a.length + 1), [new Uint8Array(Array.from({ length: ri(5) }, () => ri(256)))])
      }
    })
    if (rnd() < syncP) {
      const a = docs[ri(nClients)]; const b = docs[ri(nClients)]
      if (a !== b) {
        Y.applyUpdateV2(b, Y.encodeStateAsUpdateV2(a, Y.encodeStateVector(b)), 'remote')
        Y.applyUpdateV2(a, Y.encodeStateAsUpdateV2(b, Y.encodeStateVector(a)), 'remote')
      }
    }
  }
  return { docs, logs1, logs2 }
}

function family (F, nClients, nOps, kinds, syncP) {
  const { docs, logs1, logs2 } = session(nClients, nOps, kinds, syncP)
  const all1 = [].concat(...logs1); const all2 = [].concat(...logs2)
  if (all1.length !== all2.length) throw new Error('update / updateV2 logs differ in length')
  for (let i = 0; i < all1.length; i++) if (rnd() < 0.3) conv(F, all1[i], all2[i], 'transaction')
  for (const d of docs) conv(F, Y.encodeStateAsUpdate(d), Y.encodeStateAsUpdateV2(d), 'doc state')
  if (all2.length === 0) return
  const idx = all2.map((_, i) => i)
  const sel = ix => ix.map(i => all2[i])
  const order = shuffle(idx)
  const full = merge2(F, sel(order), 'all-shuffled')
  merge2(F, all2, 'all-in-order')
  conv(F, Y.mergeUpdates(sel(order).map((_, j) => all1[order[j]])), Y.mergeUpdatesV2(sel(order)), 'merged log')
  const sub = shuffle(idx).slice(0, 1 + ri(idx.length)); merge2(F, sel(sub), 'subset')
  if (idx.length >= 4) {
    const s = shuffle(idx); const cut = 1 + ri(s.length - 2)
    const p1 = Y.mergeUpdatesV2(sel(s.slice(0, cut))); const p2 = Y.mergeUpdatesV2(sel(s.slice(cut)))
    merge2(F, [p1, p2], 'two-disjoint-premerged')
    merge2(F, [p2].concat(sel(shuffle(s.slice(0, cut)))), 'premerged+log')
  }
  const snap = Y.encodeStateAsUpdateV2(docs[0])
  merge2(F, [snap].concat(sel(shuffle(idx).slice(0, ri(4)))), 'snapshot+log(overlap)')
  merge2(F, sel(shuffle(idx.concat(shuffle(idx).slice(0, 1 + ri(3))))), 'duplicates')
  merge2(F, [pick(all2)], 'single input')
  if (full) {
    const fb = Buffer.from(full, 'hex')
    sv2(F, fb, 'sv(full)')
    diff2(F, fb, Y.encodeStateVectorFromUpdateV2(Y.mergeUpdatesV2(sel(sub))), 'diff(sv subset)')
    diff2(F, fb, Y.encodeStateVector(docs[ri(docs.length)]), 'diff(sv peer)')
    diff2(F, fb, Y.encodeStateVector(new Y.Doc()), 'diff(empty sv)')
    // random clocks: may split items (and surrogate pairs)
    const svm = Y.decodeStateVector(Y.encodeStateVectorFromUpdateV2(fb)); const enc = []
    for (const [c, k] of svm) if (rnd() < 0.7) enc.push([c, ri(k + 1)])
    const o = [enc.length]; const vu = n => { while (n > 127) { o.push(0x80 | (n % 128)); n = Math.floor(n / 128) } o.push(n) }
    o.length = 0; vu(enc.length); for (const [c, k] of enc) { vu(c); vu(k) }
    diff2(F, fb, new Uint8Array(o), 'diff(random sv)')
  }
  sv2(F, snap, 'sv(snapshot)')
  sv2(F, pick(all2), 'sv(single)')
  diff2(F, snap, Y.encodeStateVector(docs[ri(docs.length)]), 'diff(snapshot, sv peer)')
  // malformed: truncations and byte flips of V2 inputs
  for (let t = 0; t < 3; t++) {
    const u = pick(all2.concat([snap]))
    const cut = u.slice(0, ri(u.length))
    merge2(F + '-bad', [cut, pick(all2)], 'truncated')
    sv2(F + '-bad', cut, 'truncated')
    diff2(F + '-bad', cut, Y.encodeStateVector(docs[0]), 'truncated')
    const fl = Uint8Array.from(u); fl[ri(fl.length)] = ri(256)
    merge2(F + '-bad', [pick(all2), fl], 'flipped')
    sv2(F + '-bad', fl, 'flipped')
    diff2(F + '-bad', fl, Y.encodeStateVector(docs[0]), 'flipped')
  }
}

function main () {
  const out = process.argv[2] || path.join(__dirname, '..', 'yjs13516_v2_vectors.jsonl.gz')
  for (let s = 0; s < 40; s++) family('text', 1 + ri(3), 5 + ri(40), ['text'], 0.3)
  for (let s = 0; s < 30; s++) family('mixed', 1 + ri(4), 5 + ri(40), ['text', 'array', 'map', 'xml', 'bin'], 0.3)
  for (let s = 0; s < 25; s++) family('xml', 1 + ri(4), 5 + ri(50), ['xml', 'text'], 0.4)
  for (let s = 0; s < 15; s++) family('map', 1 + ri(3), 5 + ri(30), ['map', 'array'], 0.3)
  // hand edge cases
  merge2('edge', [], 'empty list')
  merge2('edge', [Y.encodeStateAsUpdateV2(new Y.Doc())], 'single empty doc')
  merge2('edge', [Y.encodeStateAsUpdateV2(new Y.Doc()), Y.encodeStateAsUpdateV2(new Y.Doc())], 'two empty docs')
  sv2('edge', Y.encodeStateAsUpdateV2(new Y.Doc()), 'empty doc')
  const hdr = { generator: 'tests/golden/gen/gen_v2.js', yjs: '13.5.16 (JupyterLab bundle)', count: cases.length }
  const body = [JSON.stringify(hdr)].concat(cases.map(c => JSON.stringify(c))).join('\n') + '\n'
  fs.writeFileSync(out, zlib.gzipSync(body, { level: 9 }))
  const by = {}; for (const c of cases) by[c.op] = (by[c.op] || 0) + 1
  console.log(out, cases.length, JSON.stringify(by), 'errors', cases.filter(c => c.err).length)
}
main()
