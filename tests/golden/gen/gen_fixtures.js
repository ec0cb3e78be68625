// Golden-vector generator (test-fixture tooling; runs only in the build container).
//
// Drives the yjs 13.5.16 bundle (see tools/yjs_bundle.js) and records
//   mergeUpdates(us)                 -> out   (yjs Y@37704 / Y@39011)
//   diffUpdate(u, sv)                -> out   (Y@41210 -> Y@40711)
//   encodeStateVectorFromUpdate(u)   -> out   (Y@38304 -> Y@37728)
// as hex byte vectors in tests/golden/yjs13516_vectors.jsonl.gz.  The
// reference path these functions stand in for is Hocuspocus's persistence
// and sync path (packages/extension-database/src/Database.ts:44-60,
// packages/server/src/MessageReceiver.ts:137-213; SURVEY.md §8a rows a11-a16).
//
// Usage:  node tests/golden/gen/gen_fixtures.js [out.jsonl.gz]
'use strict'
const zlib = require('zlib')
const fs = require('fs')
const path = require('path')
const { load } = require('../../../tools/yjs_bundle')
const Y = load()

// ---------------------------------------------------------------- utilities
function mulberry32 (a) {
  return function () {
    a |= 0; a = a + 0x6D2B79F5 | 0
    let t = Math.imul(a ^ a >>> 15, 1 | a)
    t = t + Math.imul(t ^ t >>> 7, 61 | t) ^ t
    return ((t ^ t >>> 14) >>> 0) / 4294967296
  }
}
let rnd = mulberry32(1)
const ri = n => Math.floor(rnd() * n)
const pick = a => a[ri(a.length)]
const hex = u => Buffer.from(u).toString('hex')
const unhex = s => new Uint8Array(Buffer.from(s, 'hex'))
function shuffle (a) { a = a.slice(); for (let i = a.length - 1; i > 0; i--) { const j = ri(i + 1); const t = a[i]; a[i] = a[j]; a[j] = t } return a }

const cases = []
function rec (c) { cases.push(c) }
function runMerge (family, inputs, note) {
  const c = { family, op: 'merge', in: inputs.map(hex) }
  try { c.out = hex(Y.mergeUpdates(inputs)); c.err = null } catch (e) { c.out = null; c.err = String(e && e.message) }
  if (note) c.note = note
  rec(c)
  return c.out
}
function runDiff (family, u, sv, note) {
  const c = { family, op: 'diff', update: hex(u), sv: hex(sv) }
  try { c.out = hex(Y.diffUpdate(u, sv)); c.err = null } catch (e) { c.out = null; c.err = String(e && e.message) }
  if (note) c.note = note
  rec(c)
}
function runSV (family, u, note) {
  const c = { family, op: 'sv', update: hex(u) }
  try { c.out = hex(Y.encodeStateVectorFromUpdate(u)); c.err = null } catch (e) { c.out = null; c.err = String(e && e.message) }
  if (note) c.note = note
  rec(c)
}

// ------------------------------------------- raw V1 writer (own encoder, App. A)
function vu (n) { const o = []; while (n > 127) { o.push(0x80 | (n % 128)); n = Math.floor(n / 128) } o.push(n); return o }
function vs (s) { const b = Buffer.from(s, 'utf8'); return vu(b.length).concat(Array.from(b)) }
// struct builders: each returns { len, bytes }
const GC = len => ({ len, bytes: [0].concat(vu(len)) })
const SKIP = len => ({ len, bytes: [10].concat(vu(len)) })
function ITEM ({ origin = null, right = null, parentKey = 't', parentId = null, sub = null, content }) {
  let info = content.ref | (origin ? 0x80 : 0) | (right ? 0x40 : 0) | (sub !== null && !origin && !right ? 0x20 : 0)
  let b = []
  if (origin) b = b.concat(vu(origin[0]), vu(origin[1]))
  if (right) b = b.concat(vu(right[0]), vu(right[1]))
  if (!origin && !right) {
    if (parentId) b = b.concat([0], vu(parentId[0]), vu(parentId[1]))
    else b = b.concat([1], vs(parentKey))
    if (sub !== null) b = b.concat(vs(sub))
  }
  return { len: content.len, bytes: [info].concat(b, content.bytes) }
}
const STR = s => { let n = 0; for (const _ of s) n += (_.codePointAt(0) > 0xffff ? 2 : 1); return { ref: 4, len: n, bytes: vs(s) } }
const DEL = n => ({ ref: 1, len: n, bytes: vu(n) })
const BIN = arr => ({ ref: 3, len: 1, bytes: vu(arr.length).concat(arr) })
// blocks: [{client, clock, structs:[...]}], ds: [[client, [[clock,len],...]], ...]
function UPD (blocks, ds = []) {
  let b = vu(blocks.length)
  for (const bl of blocks) {
    b = b.concat(vu(bl.structs.length), vu(bl.client), vu(bl.clock))
    for (const s of bl.structs) b = b.concat(s.bytes)
  }
  b = b.concat(vu(ds.length))
  for (const [c, rs] of ds) { b = b.concat(vu(c), vu(rs.length)); for (const [k, l] of rs) b = b.concat(vu(k), vu(l)) }
  return new Uint8Array(b)
}

// ------------------------------------------------ family 1: SURVEY App. C KATs
function appC () {
  const F = 'appc'
  const c1 = ['01010100040101740568656c6c6f00', '010101058401040620776f726c6400', '000101010001'].map(unhex)
  const m1 = Y.mergeUpdates(c1)
  runMerge(F, c1, 'C-1')
  // sv bytes 01 01 01 05 decode as {1:1} plus a trailing byte (readStateVector stops after its count)
  runDiff(F, m1, unhex('01010105'), 'C-1 diff sv{1:1} + trailing byte')
  runDiff(F, m1, unhex('010105'), 'C-1 diff sv{1:5}')   // SURVEY App. C-1: 010101058401040620776f726c640101010001
  const a0 = unhex('01010700040101740368656c00'); const a1 = unhex('01010703840702026c6f00'); const st = unhex('01010700040101740568656c6c6f00')
  runMerge(F, [a0, a1, a0], 'C-2'); runMerge(F, [st, a0], 'C-2'); runMerge(F, [a0, st], 'C-2')
  const c4 = unhex('0201ac02004403000151010300040101740378797a0103010002')
  runSV(F, c4, 'C-4'); runDiff(F, c4, unhex('010302'), 'C-4')
  runMerge(F, [unhex('00020501000102010001')], 'C-5 single input passthrough')
  const c8 = unhex('01010500040101740661f09f98806200')
  runDiff(F, c8, unhex('01050100'.slice(0, 6)), 'C-8 sv{5:1}')
  runDiff(F, c8, unhex('010503'), 'C-8 sv{5:3}')
  runDiff(F, c8, unhex('010502'), 'C-8 sv{5:2} lone surrogate (throws in 13.5.16)')
  const U1 = UPD([{ client: 5, clock: 0, structs: [GC(1), GC(1)] }]); const U2 = UPD([{ client: 5, clock: 2, structs: [GC(1)] }])
  runMerge(F, [U1, U2], 'C-10')
  const G0 = UPD([{ client: 5, clock: 0, structs: [GC(1)] }]); const G3 = UPD([{ client: 5, clock: 3, structs: [GC(1)] }]); const G12 = UPD([{ client: 5, clock: 1, structs: [GC(2)] }])
  runMerge(F, [G0, G3, G12], 'C-10'); runMerge(F, [G0, G3], 'C-10')
  const A = UPD([{ client: 5, clock: 0, structs: [GC(2)] }])
  const B = UPD([{ client: 5, clock: 0, structs: [ITEM({ content: DEL(1) })] }])
  const C = UPD([{ client: 5, clock: 0, structs: [ITEM({ content: STR('ab') })] }])
  runMerge(F, [A, B], 'C-11'); runMerge(F, [B, A], 'C-11'); runMerge(F, [B, C], 'C-12'); runMerge(F, [C, B], 'C-12')
  const U7 = UPD([{ client: 9, clock: 4, structs: [GC(1)] }]); const U4 = UPD([{ client: 5, clock: 0, structs: [GC(1)] }])
  const m13 = Y.mergeUpdates([U7, U4]); runMerge(F, [U7, U4], 'C-13'); runSV(F, m13, 'C-13')
  const d2 = UPD([], [[2, [[0, 1]]]]); const d9 = UPD([], [[9, [[0, 1]]]])
  runMerge(F, [d2, d9], 'C-14'); runMerge(F, [d9, d2], 'C-14')
  runMerge(F, [], 'C-15'); runMerge(F, [unhex('0000'), unhex('0000')], 'C-15')
  const B16 = unhex('01010500040101740661f09f98806200')
  runMerge(F, [B16, A], 'C-16'); runMerge(F, [A, B16], 'C-16')
}

// ------------------------------------ family 2: real Y.Doc editing sessions
const ASCII = 'abcdefghijklmnopqrstuvwxyz ABCDEFG0123456789.,!?'
const UNI = ['é', 'ß', '中', '文', '😀', '👍🏽', '𝄞', 'Ω', '\u0000', '"', '\\', '\n']
function randStr (maxLen, uni) {
  const n = 1 + ri(maxLen); let s = ''
  for (let i = 0; i < n; i++) s += (uni && rnd() < 0.25) ? pick(UNI) : ASCII[ri(ASCII.length)]
  return s
}
function randAny (depth) {
  const r = ri(depth > 0 ? 14 : 11)
  switch (r) {
    case 0: return ri(100)
    case 1: return -ri(1 << 20)
    case 2: return ri(2147483647)
    case 3: return rnd() * 1000
    case 4: return pick([0.5, 1.5, -2.25, 3.4028234663852886e38, 1e-7, 1e300, -1e-300])
    case 5: return randStr(6, true)
    case 6: return rnd() < 0.5
    case 7: return null
    case 8: return pick([4294967296, 2 ** 40, 2 ** 53 - 1, 1 << 30])
    case 9: return ''
    case 10: return new Uint8Array([ri(256), ri(256), ri(256)])
    case 11: { const o = {}; const n = ri(4); for (let i = 0; i < n; i++) o[pick(['a', 'b', 'key', 'x y', '10', '2', 'é'])] = randAny(depth - 1); return o }
    case 12: { const a = []; const n = ri(4); for (let i = 0; i < n; i++) a.push(randAny(depth - 1)); return a }
    default: return [randAny(depth - 1)]
  }
}
function randJSONable (depth) {
  const v = randAny(depth)
  return JSON.parse(JSON.stringify(v, (k, x) => x instanceof Uint8Array ? Array.from(x) : x) || 'null')
}

function session (nClients, nOps, kinds, syncP) {
  const docs = []; const logs = []
  for (let i = 0; i < nClients; i++) {
    const d = new Y.Doc(); d.clientID = pick([1 + ri(9), 100 + ri(1000), ri(2 ** 31), 2 ** 31 + ri(2 ** 31), 4294967295 - ri(3)])
    while (docs.some(o => o.clientID === d.clientID)) d.clientID++
    const log = []
    d.on('update', (u, origin) => { if (origin !== 'remote') log.push(u) })
    docs.push(d); logs.push(log)
  }
  for (let op = 0; op < nOps; op++) {
    const ci = ri(nClients); const d = docs[ci]
    const k = pick(kinds)
    d.transact(() => {
      if (k === 'text') {
        const t = d.getText('t'); const L = t.length; const r = rnd()
        if (r < 0.55 || L === 0) t.insert(ri(L + 1), randStr(4, true), rnd() < 0.2 ? { bold: true } : undefined)
        else if (r < 0.8) { const p = ri(L); t.delete(p, 1 + ri(Math.min(3, L - p))) } else if (r < 0.92) { const p = ri(L); t.format(p, 1 + ri(Math.min(3, L - p)), pick([{ bold: true }, { italic: 1.5 }, { bold: null }, { link: { href: 'https://x.y/' + ri(9) } }])) } else t.insertEmbed(ri(L + 1), pick([{ image: 'a.png' }, { video: { src: 'v', w: ri(9) } }, 'emb']))
      } else if (k === 'array') {
        const a = d.getArray('a'); const L = a.length; const r = rnd()
        if (r < 0.6 || L === 0) { const n = 1 + ri(3); const vals = []; for (let i = 0; i < n; i++) vals.push(randAny(2)); a.insert(ri(L + 1), vals) } else if (r < 0.85) { const p = ri(L); a.delete(p, 1 + ri(Math.min(2, L - p))) } else { a.insert(ri(L + 1), [pick([new Y.Map(), new Y.Array(), new Y.Text('nt'), new Y.XmlText()])]) }
      } else if (k === 'map') {
        const m = d.getMap('m'); const r = rnd(); const key = pick(['a', 'b', 'c', 'long key ' + ri(3), 'é'])
        if (r < 0.7) m.set(key, randAny(2)); else if (r < 0.8) m.set(key, pick([new Y.Map(), new Y.Array(), new Y.Text()])); else if (r < 0.9) { const sd = new Y.Doc({ guid: 'sub-' + ri(100), gc: rnd() < 0.5, autoLoad: rnd() < 0.5 }); m.set(key, sd) } else m.delete(key)
      } else if (k === 'xml') {
        const f = d.getXmlFragment('prosemirror'); const L = f.length; const r = rnd()
        if (r < 0.5 || L === 0) { const el = new Y.XmlElement(pick(['paragraph', 'heading', 'blockquote'])); el.setAttribute('level', String(ri(3))); const tx = new Y.XmlText(); el.insert(0, [tx]); f.insert(ri(L + 1), [el]); tx.insert(0, randStr(5, true)); if (rnd() < 0.5) tx.format(0, 1, { bold: true }) } else if (r < 0.75) { const el = f.get(ri(L)); if (el instanceof Y.XmlElement && el.length > 0) { const tx = el.get(0); if (tx instanceof Y.XmlText) { const tl = tx.length; if (rnd() < 0.6 || tl === 0) tx.insert(ri(tl + 1), randStr(3, true), rnd() < 0.3 ? { italic: true } : undefined); else tx.delete(ri(tl), 1) } } } else if (r < 0.9) { const p = ri(L); f.delete(p, 1) } else { const el = f.get(ri(L)); if (el instanceof Y.XmlElement) el.setAttribute(pick(['class', 'level', 'id']), randStr(3, false)) }
      } else if (k === 'nested') {
        const a = d.getArray('n'); if (a.length === 0 || rnd() < 0.3) { a.push([new Y.Map()]) } else { const m = a.get(ri(a.length)); if (m instanceof Y.Map) { if (rnd() < 0.7) m.set(pick(['p', 'q']), randAny(1)); else a.delete(ri(a.length), 1) } }
      }
    })
    if (rnd() < syncP) { // sync two random clients both ways
      const a = docs[ri(nClients)]; const b = docs[ri(nClients)]
      if (a !== b) {
        Y.applyUpdate(b, Y.encodeStateAsUpdate(a, Y.encodeStateVector(b)), 'remote')
        Y.applyUpdate(a, Y.encodeStateAsUpdate(b, Y.encodeStateVector(a)), 'remote')
      }
    }
  }
  return { docs, logs }
}

function mergeFamily (F, logs, docs) {
  const all = [].concat(...logs)
  if (all.length === 0) return
  // overlap-free: all updates in random order; random subsets; pre-merged disjoint chunks
  const full = Y.mergeUpdates(shuffle(all))
  runMerge(F, shuffle(all), 'all-shuffled')
  runMerge(F, all, 'all-in-order')
  const sub = shuffle(all).slice(0, 1 + ri(all.length)); runMerge(F, sub, 'subset')
  if (all.length >= 4) {
    const s = shuffle(all); const cut = 1 + ri(s.length - 2)
    const p1 = Y.mergeUpdates(s.slice(0, cut)); const p2 = Y.mergeUpdates(s.slice(cut))
    runMerge(F, [p1, p2], 'two-disjoint-premerged')
    runMerge(F, [p2].concat(shuffle(s.slice(0, cut))), 'premerged+log')
  }
  // snapshot (doc-level re-encode, may hold GC) + log of later updates: the Hocuspocus store shape
  const d0 = docs[0]
  const snap = Y.encodeStateAsUpdate(d0)
  runMerge(F, [snap].concat(shuffle(all).slice(0, ri(4))), 'snapshot+log(overlap)')
  // overlap/duplicates: repeat some updates, overlapping premerged chunks
  const dup = shuffle(all.concat(shuffle(all).slice(0, 1 + ri(3)))); runMerge(F, dup, 'duplicates')
  if (all.length >= 3) {
    const s = shuffle(all); const a = 1 + ri(s.length - 1); const b = ri(a)
    runMerge(F, [Y.mergeUpdates(s.slice(0, a)), Y.mergeUpdates(s.slice(b))], 'overlapping-premerged')
  }
  // state vectors
  runSV(F, full, 'sv(full)')
  runSV(F, pick(all), 'sv(single)')
  runSV(F, Y.mergeUpdates(sub), 'sv(subset)')
  runSV(F, snap, 'sv(snapshot)')
  // diffs: sv of random subset, sv of a peer doc, random clocks (may split items and surrogate pairs)
  runDiff(F, full, Y.encodeStateVectorFromUpdate(Y.mergeUpdates(sub)), 'diff(sv subset)')
  runDiff(F, full, Y.encodeStateVector(docs[ri(docs.length)]), 'diff(sv peer)')
  runDiff(F, snap, Y.encodeStateVector(docs[ri(docs.length)]), 'diff(snapshot, sv peer)')
  const svm = Y.decodeStateVector(Y.encodeStateVectorFromUpdate(full))
  for (let rep = 0; rep < 3; rep++) {
    const ents = []
    svm.forEach((clock, client) => { if (rnd() < 0.8) ents.push([client, ri(clock + 2)]) })
    if (rnd() < 0.2) ents.push([12345, 3])
    const sv = [].concat(vu(ents.length), ...ents.map(([c, k]) => vu(c).concat(vu(k))))
    runDiff(F, full, new Uint8Array(sv), 'diff(random sv)')
  }
  runDiff(F, full, new Uint8Array([0]), 'diff(empty sv)')
  runDiff(F, pick(all), new Uint8Array([0]), 'diff(single, empty sv)')
}

function sessions () {
  const kindsets = [['text'], ['array'], ['map'], ['xml'], ['nested'], ['text', 'array', 'map'], ['text', 'xml', 'map', 'nested', 'array']]
  for (let s = 0; s < 260; s++) {
    const kinds = kindsets[s % kindsets.length]
    const { docs, logs } = session(1 + ri(4), 3 + ri(30), kinds, 0.3)
    mergeFamily('session-' + kinds.join('+'), logs, docs)
  }
}

// ---------------- family 3: GC-heavy docs (gc on, deleted nested types -> GC structs)
function gcFamily () {
  for (let s = 0; s < 60; s++) {
    const d = new Y.Doc(); d.clientID = 1 + ri(50); const log = []; d.on('update', u => log.push(u))
    const a = d.getArray('a')
    for (let i = 0; i < 3 + ri(6); i++) { const m = new Y.Map(); a.insert(ri(a.length + 1), [m]); m.set('k', i); m.set('k2', 'v' + i); if (rnd() < 0.5) { const t = new Y.Text(); m.set('t', t); t.insert(0, 'xyz') } }
    for (let i = 0; i < 2 + ri(3) && a.length > 0; i++) a.delete(ri(a.length), 1)
    const snap = Y.encodeStateAsUpdate(d) // GC'd content of deleted maps
    const d2 = new Y.Doc(); d2.clientID = d.clientID + 1000; const log2 = []; d2.on('update', (u, o) => { if (o !== 'remote') log2.push(u) })
    Y.applyUpdate(d2, snap, 'remote')
    const a2 = d2.getArray('a'); for (let i = 0; i < 1 + ri(4); i++) a2.insert(ri(a2.length + 1), [i, 'x'])
    if (a2.length > 0) a2.delete(ri(a2.length), 1)
    runMerge('gc', [snap].concat(log2), 'snapshot(GC)+log')
    runMerge('gc', shuffle([snap].concat(log2)), 'snapshot(GC)+log shuffled')
    runMerge('gc', [Y.encodeStateAsUpdate(d2), snap], 'snap2+snap1 (overlap)')
    runSV('gc', snap); runDiff('gc', snap, Y.encodeStateVector(d2)); runDiff('gc', Y.encodeStateAsUpdate(d2), Y.encodeStateVectorFromUpdate(Y.mergeUpdates(log.slice(0, 1 + ri(log.length)))))
    // split snapshot GC runs into pieces from different sources (C-10 provenance rule)
    runMerge('gc', [snap, Y.mergeUpdates(log)], 'snapshot+full log')
  }
}

// --------------------------------- family 4: hand-built raw update structure
function rawFamily () {
  const F = 'raw'
  for (let s = 0; s < 400; s++) {
    // build a client's struct sequence, then cut it into pieces spread over k updates
    const nClients = 1 + ri(3); const pieces = []
    const clients = shuffle([3, 7, 300, 2 ** 31 + 5, 65, 128, 16383, 16384]).slice(0, nClients)
    for (const c of clients) {
      let clock = rnd() < 0.2 ? ri(5) : 0
      const n = 1 + ri(8)
      for (let i = 0; i < n; i++) {
        const kind = ri(10); let st
        if (kind < 3) st = GC(1 + ri(3))
        else if (kind < 5) st = ITEM({ origin: clock > 0 && rnd() < 0.7 ? [c, clock - 1] : null, content: STR(randStr(3, true)) })
        else if (kind < 6) st = ITEM({ origin: rnd() < 0.5 ? [c, Math.max(0, clock - 1)] : null, right: rnd() < 0.3 ? [clients[0], 0] : null, content: DEL(1 + ri(3)) })
        else if (kind < 7) st = ITEM({ parentId: [clients[0], 0], sub: rnd() < 0.5 ? 'key' : null, content: BIN([1, 2, 3]) })
        else if (kind < 8) st = ITEM({ origin: [c, clock], sub: 'k', content: STR('q') }) // 0x20 not set when origin (builder); see nonCanonical below
        else st = GC(1)
        pieces.push({ client: c, clock, st })
        clock += st.len
        if (rnd() < 0.25) clock += 1 + ri(3) // gap: missing structs -> Skip in merge
      }
    }
    // distribute pieces over k updates; within an update, group into client blocks (maybe ascending order!)
    const k = 1 + ri(4); const ups = []; for (let i = 0; i < k; i++) ups.push([])
    for (const p of pieces) ups[ri(k)].push(p)
    const updates = ups.map(ps => {
      const byClient = new Map()
      for (const p of ps) { if (!byClient.has(p.client)) byClient.set(p.client, []); byClient.get(p.client).push(p) }
      let order = Array.from(byClient.keys()).sort((a, b) => b - a)
      if (rnd() < 0.15) order = order.reverse()
      const blocks = []
      for (const c of order) {
        const list = byClient.get(c)
        // split into contiguous runs; a gap inside a run is filled with a Skip sometimes
        let cur = null
        for (const p of list) {
          if (cur && cur.end === p.clock) { cur.structs.push(p.st); cur.end += p.st.len } else if (cur && rnd() < 0.3) { cur.structs.push(SKIP(p.clock - cur.end)); cur.structs.push(p.st); cur.end = p.clock + p.st.len } else { cur = { client: c, clock: p.clock, structs: [p.st], end: p.clock + p.st.len }; blocks.push(cur) }
        }
      }
      const ds = []
      if (rnd() < 0.5) { const nd = 1 + ri(3); for (let i = 0; i < nd; i++) { const rs = []; const nr = ri(4); for (let j = 0; j < nr; j++) rs.push([ri(20), ri(5)]); ds.push([pick(clients.concat([11, 12])), rs]) } }
      return UPD(blocks, ds)
    })
    runMerge(F, updates)
    if (updates.length > 1) runMerge(F, shuffle(updates))
    for (const u of updates) runSV(F, u)
    const m = Y.mergeUpdates(updates)
    runSV(F, m)
    const ents = clients.filter(() => rnd() < 0.8).map(c => [c, ri(12)])
    runDiff(F, m, new Uint8Array([].concat(vu(ents.length), ...ents.map(([c, kk]) => vu(c).concat(vu(kk))))))
    runDiff(F, updates[0], new Uint8Array([].concat(vu(ents.length), ...ents.map(([c, kk]) => vu(c).concat(vu(kk))))))
  }
  // DS-only updates: union rules (R-DS), first-seen order, 0-range clients, duplicate clients
  for (let s = 0; s < 150; s++) {
    const k = 1 + ri(5); const ups = []
    for (let i = 0; i < k; i++) {
      const ds = []; const nd = ri(4)
      for (let j = 0; j < nd; j++) { const rs = []; const nr = ri(5); for (let q = 0; q < nr; q++) rs.push([ri(30), ri(6)]); ds.push([pick([1, 2, 9, 200, 70000, 2 ** 32 - 1]), rs]) }
      ups.push(UPD([], ds))
    }
    runMerge('ds', ups)
    runDiff('ds', ups[0], new Uint8Array([0]))
  }
}

// ------------------------------ family 5: non-canonical and malformed inputs
function edgeFamily () {
  const F = 'edge'
  const base = unhex('01010500040101740568656c6c6f00')
  const other = unhex('01010502840504016f00') // overlapping-ish
  // non-minimal varuint for clock (0x80 0x00)
  runMerge(F, [unhex('0101058000040101740161' + '00'), unhex('0000')], 'non-minimal varuint clock')
  // bit 0x20 with origin present (parentSub not read; info rewritten)
  runMerge(F, [unhex('0101050184050001620' + '0'), unhex('01010500040101740161' + '00')], 'info 0x80 sliced-free')
  runMerge(F, [unhex('01010501a405000162' + '00'), unhex('01010500040101740161' + '00')], 'info 0x20|0x80 (parentSub bit with origin)')
  runMerge(F, [unhex('01010501e4050005010162' + '00'), unhex('01010500040101740161' + '00')], 'info 0x20|0x80|0x40')
  // parentInfo = 2 (treated as ID)
  runMerge(F, [unhex('01010500040205000161' + '00'), unhex('0000')], 'parentInfo 2')
  // GC info with high bits
  runMerge(F, [unhex('0101050080020000'.slice(0, 14) + '00'), unhex('0000')], 'GC info 0x80')
  runMerge(F, [unhex('010105004002' + '00'), unhex('0000')], 'GC info 0x40')
  // trailing garbage, empty, truncated
  runMerge(F, [unhex('0000ffff'), unhex('0000')], 'trailing garbage')
  runMerge(F, [unhex('01'), unhex('0000')], 'truncated header')
  runMerge(F, [base.slice(0, 10), unhex('0000')], 'truncated struct')
  runMerge(F, [unhex('00'), unhex('0000')], 'missing DS')
  runMerge(F, [unhex(''), unhex('0000')], 'empty update')
  runSV(F, unhex(''), 'sv(empty)'); runSV(F, unhex('0000')); runSV(F, base.slice(0, 10), 'sv truncated')
  runDiff(F, base, unhex(''), 'diff empty sv bytes'); runDiff(F, base.slice(0, 9), unhex('00'), 'diff truncated')
  runMerge(F, [base, other])
  // invalid UTF-8 / overlong / surrogate in string content
  runMerge(F, [unhex('0101050004010174' + '02c0af' + '00'), unhex('0000')], 'overlong utf8')
  runMerge(F, [unhex('0101050004010174' + '03eda080' + '00'), unhex('0000')], 'utf8 surrogate')
  runMerge(F, [unhex('0101050004010174' + '01ff' + '00'), unhex('0000')], 'invalid utf8 byte')
  runMerge(F, [unhex('0101050004010174' + '03efbbbf' + '00'), unhex('0000')], 'BOM kept')
  // content ref 10 / 0x8A, unknown refs
  runMerge(F, [unhex('0101050a0a05000100'), unhex('0000')], 'info 10 with garbage')
  runMerge(F, [unhex('010105008a050001' + '00'), unhex('0000')], 'content ref 10')
  runMerge(F, [unhex('010105000b0101740000'), unhex('0000')], 'content ref 11')
  // Any: non-canonical numbers (C-9), unknown tag, objects with index keys
  const anyItem = hexAny => unhex('0101050008010161' + '01' + hexAny + '00')
  for (const a of ['7b3ff0000000000000', '7b3ff8000000000000', '7c3f800000', '7c3fc00000', '7d01', '7d4100'.slice(0, 4), '7d8100', '7d41', '7dc001', '7b7ff8000000000000', '7c7fc00000', '7b4000000000000000',
    '7a0000000000000001', '7f', '7e', '79', '78', '7703616263', '760201617d0101627d02', '760201327d0101317d02', '760201317d0101317d02', '7602095f5f70726f746f5f5f7d0101617d02', '7602095f5f70726f746f5f5f7e0101617d02', '750277017d02', '75027701617d02', '7b7ff8000000000001', '7bfff8000000000000', '7b8000000000000000', '7c80000000', '7c7f800000', '7d8080808008', '7d80808080088000', '7dbfffffff0f', '7dffffffff0f', '7b41e0000000000000', '7bc1e0000000200000', '76017600', '760201317d0101307d02', '7602023130017d0101397d02', '760203303031017d0101317d02', '74020102', '7300', 'ff']) {
    runMerge(F, [anyItem(a), unhex('0000')], 'any ' + a)
  }
  // JSON content (ref 2) canonical / non-canonical, 'undefined'
  const jsonItem = strs => unhex('0101050002010161' + Buffer.from(vu(strs.length).concat(...strs.map(vs))).toString('hex') + '00')
  for (const js of [['1'], ['1.0'], ['{"a":1}'], ['{ "a" : 1 }'], ['undefined'], ['"x"', 'true', 'null'], ['[1,2]'], ['{"b":1,"a":2}'], ['{"2":1,"1":2}'], ['1e21'], ['0.1'], ['"\\u0041"'], ['"\\/"'], ['-0'], ['1E2'], ['bad']]) {
    runMerge(F, [jsonItem(js), unhex('0000')], 'json ' + JSON.stringify(js))
  }
  // embed / format JSON
  runMerge(F, [unhex('0101050005010161' + Buffer.from(vs('{"image":"a.png"}')).toString('hex') + '00'), unhex('0000')], 'embed canonical')
  runMerge(F, [unhex('0101050005010161' + Buffer.from(vs('{ "image":"a.png"}')).toString('hex') + '00'), unhex('0000')], 'embed non-canonical')
  runMerge(F, [unhex('0101050006010161' + Buffer.from(vs('bold').concat(vs('true'))).toString('hex') + '00'), unhex('0000')], 'format canonical')
  runMerge(F, [unhex('0101050006010161' + Buffer.from(vs('italic').concat(vs('1.50'))).toString('hex') + '00'), unhex('0000')], 'format non-canonical')
  // type refs incl. XmlElement / XmlHook names, unknown type ref
  for (const t of ['00', '01', '02', '03' + Buffer.from(vs('p')).toString('hex'), '04', '05' + Buffer.from(vs('h')).toString('hex'), '06', '07', '8000']) runMerge(F, [unhex('0101050007010161' + t + '00'), unhex('0000')], 'type ' + t)
  // ContentDoc
  runMerge(F, [unhex('0101050009010161' + Buffer.from(vs('guid-1')).toString('hex') + '7600' + '00'), unhex('0000')], 'doc {}')
  runMerge(F, [unhex('0101050009010161' + Buffer.from(vs('guid-1')).toString('hex') + '760102676379' + '00'), unhex('0000')], 'doc {gc:false}')
  runMerge(F, [unhex('0101050009010161' + Buffer.from(vs('guid-1')).toString('hex') + '7601086175746f4c6f616478' + '00'), unhex('0000')], 'doc {autoLoad:true}')
  runMerge(F, [unhex('0101050009010161' + Buffer.from(vs('guid-1')).toString('hex') + '7601026763' + '78' + '00'), unhex('0000')], 'doc {gc:true}')
  // large clocks / clients (>= 2^31, 32-bit boundary)
  runMerge(F, [UPD([{ client: 4294967295, clock: 2147483647, structs: [GC(1)] }]), UPD([{ client: 4294967295, clock: 2147483648, structs: [GC(3)] }])], 'u32 max client')
  // non-descending client blocks, same client twice in one update
  runMerge(F, [UPD([{ client: 1, clock: 0, structs: [GC(1)] }, { client: 5, clock: 0, structs: [GC(1)] }]), UPD([{ client: 5, clock: 1, structs: [GC(1)] }])], 'ascending blocks')
  runMerge(F, [UPD([{ client: 5, clock: 0, structs: [GC(1)] }, { client: 5, clock: 3, structs: [GC(1)] }]), UPD([{ client: 5, clock: 1, structs: [GC(2)] }])], 'repeated client block')
  runSV(F, UPD([{ client: 5, clock: 0, structs: [GC(1)] }, { client: 7, clock: 0, structs: [GC(1)] }, { client: 5, clock: 1, structs: [GC(1)] }]), 'sv repeated client')
  runSV(F, UPD([{ client: 5, clock: 0, structs: [SKIP(3), GC(2)] }]), 'sv first skip')
  runSV(F, UPD([{ client: 9, clock: 0, structs: [GC(2)] }, { client: 5, clock: 0, structs: [SKIP(3), GC(2)] }]), 'sv second skip')
  runDiff(F, UPD([{ client: 5, clock: 0, structs: [SKIP(2), GC(2), SKIP(1), GC(1)] }, { client: 5, clock: 10, structs: [GC(1)] }]), unhex('010501'), 'diff skips + repeated client')
  // Skips in merge input (filtered), merge where a Skip must be extended
  runMerge(F, [UPD([{ client: 5, clock: 0, structs: [GC(1), SKIP(2), GC(1)] }]), UPD([{ client: 5, clock: 6, structs: [GC(1)] }])], 'skips in input')
}

// ------------------------------------------------ family 6: config-2 shapes
function c2Family () {
  for (let s = 0; s < 20; s++) {
    const nC = 1 + ri(4); const docs = []; const log = []
    for (let i = 0; i < nC; i++) { const d = new Y.Doc(); d.clientID = ri(2 ** 32); docs.push(d); d.on('update', (u, o) => { if (o !== 'remote') log.push(u) }) }
    // single shared doc model: all clients see each other's edits (server doc), like Hocuspocus
    const server = new Y.Doc()
    for (let i = 0; i < 60; i++) {
      const d = pick(docs)
      Y.applyUpdate(d, Y.encodeStateAsUpdate(server, Y.encodeStateVector(d)), 'remote')
      const t = d.getText('t'); t.insert(ri(t.length + 1), ASCII[ri(26)])
      Y.applyUpdate(server, Y.encodeStateAsUpdate(d, Y.encodeStateVector(server)), 'remote')
    }
    runMerge('c2', log, 'c2 log order'); runMerge('c2', shuffle(log), 'c2 shuffled')
    const m = Y.mergeUpdates(log); runSV('c2', m); runDiff('c2', m, Y.encodeStateVectorFromUpdate(Y.mergeUpdates(log.slice(0, ri(log.length)))))
  }
}

// ---------------------------------------------------------------------- main
const out = process.argv[2] || path.join(__dirname, '..', 'yjs13516_vectors.jsonl.gz')
rnd = mulberry32(20251024)
appC(); sessions(); gcFamily(); rawFamily(); edgeFamily(); c2Family()
const lines = cases.map((c, i) => JSON.stringify(Object.assign({ id: i }, c)))
const header = JSON.stringify({ oracle: 'yjs13.5.16/lib0-0.2.42', source: 'JupyterLab bundle 3502.fbe0c610be82ba1360db.js (md5 11700b19974fc00b67cd4223f97475ea)', seed: 20251024, count: cases.length })
fs.writeFileSync(out, zlib.gzipSync(Buffer.from([header].concat(lines).join('\n') + '\n'), { level: 9 }))
const errs = cases.filter(c => c.err).length
console.log(`wrote ${cases.length} cases (${errs} throwing) to ${out}`)
