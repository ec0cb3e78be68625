'use strict'
// Doc-normalized snapshot corpus (SURVEY.md §8f-1; test / measurement tooling).
// Random multi-peer editing sessions on the image's yjs 13.5.16 bundle -- Y.Text inserts and deletes
// (ASCII, 2/3/4-byte UTF-8 so surrogate pairs get split), formatting and embeds, Y.Array of JSON
// values and nested types, Y.Map sets / overwrites / deletes, XmlFragment trees with attributes,
// deleted nested types -- with peers syncing now and then (concurrent inserts).  For each session:
//   u        = Y.mergeUpdates(every local update of every peer)     (what GpuMerge stores today)
//   expected = Y.encodeStateAsUpdate(Y.applyUpdate(new Y.Doc(), u))  (what extension-database stores)
// Writes `out.bin` (u32 n, then (u32 len, u) per session) and `exp.bin` (i32 status 0, u32 len, bytes),
// the formats tools/snapdev and tests read.
//   node tools/snap_corpus.js <n> <seed> <out.bin> <exp.bin> [maxOps] [text|pending|textpending|subdoc|subpending]
// subdoc: the general sessions with sub-documents (Y.Doc values in a map and an array, some of them deleted)
// pending: the same sessions with 1-3 of the log's updates lost (out-of-order delivery: later updates depend on the
// missing ones) -- u merges what is left, so Y.applyUpdate leaves pending structs and / or a pending delete set
const fs = require('fs')
const path = require('path')
const Y = require(path.join(__dirname, 'yjs_bundle.js')).load()

function rng (seed) {
  let x = (seed >>> 0) || 1
  return () => { x ^= x << 13; x >>>= 0; x ^= x >>> 17; x ^= x << 5; x >>>= 0; return x / 4294967296 }
}

const ALPH = ['a', 'b', 'c', 'd', 'e', ' ', 'é', 'ß', '€', '中', '😀', '🎉', 'x']

// text: flat Y.Text sessions only -- ASCII inserts of 1-8 characters (in the middle of earlier runs too) and
// deletions over 1-4 peers that sync now and then (concurrent inserts at one position, splits by origins and by
// delete ranges): the envelope of the flat-text snapshot kernel (ygm_snap_text.hpp)
// drop 1-3 random updates of the log (pending mode), from a stream of its own (the sessions stay the same)
function dropSome (log, seed) {
  if (log.length < 2) return log
  const R = rng(seed * 2246822519 + 99)
  const out = log.slice()
  const k = 1 + Math.floor(R() * Math.min(3, out.length - 1))
  for (let i = 0; i < k; i++) out.splice(Math.floor(R() * out.length), 1)
  return out
}

function textSession (seed, maxOps, drop) {
  const R = rng(seed * 2654435761 + 777)
  const ri = n => Math.floor(R() * n)
  const nPeers = 1 + ri(4)
  const peers = []
  const log = []
  for (let p = 0; p < nPeers; p++) {
    const d = new Y.Doc()
    d.clientID = 1 + ri(R() < 0.5 ? 100 : 0x7ffffff0)
    d.on('update', (u, origin, doc, tr) => { if (tr.local) log.push(u) })
    peers.push(d)
  }
  const ops = 1 + ri(maxOps)
  for (let o = 0; o < ops; o++) {
    const p = ri(nPeers)
    const d = peers[p]
    if (R() < 0.12) {
      const q = ri(nPeers)
      if (q !== p) Y.applyUpdate(peers[q], Y.encodeStateAsUpdate(d, Y.encodeStateVector(peers[q])), 'remote')
      continue
    }
    d.transact(() => {
      const t = d.getText('text')
      if (t.length > 0 && R() < 0.3) { const at = ri(t.length); t.delete(at, 1 + ri(Math.min(5, t.length - at))) }
      else { let s = ''; const k = 1 + ri(R() < 0.7 ? 2 : 8); for (let i = 0; i < k; i++) s += 'abcdefgh xyz'[ri(12)]; t.insert(ri(t.length + 1), s) }
    })
  }
  const kept = drop ? dropSome(log, seed) : log
  const u = kept.length ? Y.mergeUpdates(kept) : Y.encodeStateAsUpdate(new Y.Doc())
  const fresh = new Y.Doc()
  Y.applyUpdate(fresh, u)
  return [u, Y.encodeStateAsUpdate(fresh)]
}

function session (seed, maxOps, drop, subdoc) {
  const R = rng(seed * 2654435761 + 12345)
  const ri = n => Math.floor(R() * n)
  const nPeers = 1 + ri(3)
  const peers = []
  const log = []
  for (let p = 0; p < nPeers; p++) {
    const d = new Y.Doc()
    d.clientID = 1 + ri(0x7ffffff0)
    d.on('update', (u, origin, doc, tr) => { if (tr.local) log.push(u) })
    peers.push(d)
  }
  const str = n => { let s = ''; for (let i = 0; i < n; i++) s += ALPH[ri(ALPH.length)]; return s }
  const ops = 1 + ri(maxOps)
  const nested = []   // nested shared types created so far: [peerIndex, type]
  for (let o = 0; o < ops; o++) {
    const p = ri(nPeers)
    const d = peers[p]
    const k = ri(16)
    d.transact(() => {
      if (subdoc && R() < 0.15) {
        // sub-documents (ContentDoc): set in a map (an overwrite deletes the previous one) or inserted in an array
        const opts = [{}, { autoLoad: true }, { meta: { v: ri(9) } }, { gc: false }, { gc: false, autoLoad: true, meta: 'm' }][ri(5)]
        const sd = new Y.Doc(Object.assign({ guid: 'sub-' + ri(1e9) }, opts))   // (a seeded guid: the vectors regenerate)
        if (R() < 0.6) d.getMap('docs').set('d' + ri(3), sd)
        else { const a = d.getArray('subs'); if (a.length && R() < 0.3) a.delete(ri(a.length), 1); else a.insert(ri(a.length + 1), [sd]) }
      } else if (k < 5) {
        const t = d.getText('text')
        if (t.length > 0 && R() < 0.35) { const at = ri(t.length); t.delete(at, 1 + ri(Math.min(6, t.length - at))) }
        else t.insert(ri(t.length + 1), str(1 + ri(R() < 0.8 ? 3 : 12)), R() < 0.15 ? { bold: true } : undefined)
        if (R() < 0.05 && t.length > 1) { const at = ri(t.length - 1); t.format(at, 1 + ri(Math.min(2, t.length - at - 1)), { italic: R() < 0.5 ? 1.5 : null }) }
        if (R() < 0.03) t.insertEmbed(ri(t.length + 1), { image: 'x.png' })
      } else if (k < 8) {
        const a = d.getArray('arr')
        if (a.length > 0 && R() < 0.3) { const at = ri(a.length); a.delete(at, 1 + ri(Math.min(3, a.length - at))) }
        else {
          const v = ri(6)
          let item
          if (v === 0) item = ri(1000)
          else if (v === 1) item = str(2)
          else if (v === 2) item = { k: ri(10), s: str(1) }
          else if (v === 3) item = [true, null, ri(5)]
          else if (v === 4) { item = new Y.Map(); nested.push([p, item]) }
          else { item = new Y.Array(); nested.push([p, item]) }
          a.insert(ri(a.length + 1), [item])
          if (v === 4) item.set('n', ri(100))
          if (v === 5) item.push([str(1), ri(9)])
        }
      } else if (k < 11) {
        const m = d.getMap('map')
        const key = 'k' + ri(5)
        if (R() < 0.2) m.delete(key)
        else if (R() < 0.15) { const t = new Y.Text(); m.set(key, t); t.insert(0, str(3)); nested.push([p, t]) }
        else m.set(key, R() < 0.5 ? ri(100) : str(2))
      } else if (k < 13) {
        const f = d.getXmlFragment('xml')
        if (f.length > 0 && R() < 0.25) f.delete(ri(f.length), 1)
        else {
          const e = new Y.XmlElement(R() < 0.5 ? 'paragraph' : 'heading')
          f.insert(ri(f.length + 1), [e])
          e.setAttribute('level', String(1 + ri(3)))
          const tx = new Y.XmlText()
          e.insert(0, [tx])
          tx.insert(0, str(2 + ri(5)), R() < 0.3 ? { bold: true } : undefined)
          nested.push([p, tx])
        }
      } else if (k < 15 && nested.length) {
        const [q, t] = nested[ri(nested.length)]
        if (q === p && t.doc === d && !(t._item && t._item.deleted)) {
          if (t instanceof Y.Text) { if (t.length > 1 && R() < 0.4) t.delete(ri(t.length - 1), 1); else t.insert(ri(t.length + 1), str(2)) }
          else if (t instanceof Y.Array) { if (t.length && R() < 0.4) t.delete(0, 1); else t.push([ri(50)]) }
          else if (t instanceof Y.Map) t.set('m' + ri(3), str(1))
        }
      } else {
        // sync: another peer receives this peer's state (concurrency afterwards)
        const q = ri(nPeers)
        if (q !== p) Y.applyUpdate(peers[q], Y.encodeStateAsUpdate(d, Y.encodeStateVector(peers[q])), 'remote')
      }
    })
  }
  const kept = drop ? dropSome(log, seed) : log
  const u = kept.length ? Y.mergeUpdates(kept) : Y.encodeStateAsUpdate(new Y.Doc())
  const fresh = new Y.Doc()
  Y.applyUpdate(fresh, u)
  return [u, Y.encodeStateAsUpdate(fresh)]
}

function write (file, arr, withStatus) {
  const parts = [Buffer.from(new Uint32Array([arr.length]).buffer)]
  for (const b of arr) {
    if (withStatus) parts.push(Buffer.from(new Int32Array([0]).buffer))
    parts.push(Buffer.from(new Uint32Array([b.length]).buffer), Buffer.from(b))
  }
  fs.writeFileSync(file, Buffer.concat(parts))
}

if (require.main === module) {
  const n = parseInt(process.argv[2] || '100', 10)
  const seed = parseInt(process.argv[3] || '1', 10)
  const maxOps = parseInt(process.argv[6] || '60', 10)
  const mode = process.argv[7] || ''
  const gen = mode === 'text' || mode === 'textpending' ? textSession : session
  const drop = mode === 'pending' || mode === 'textpending' || mode === 'subpending'
  const subdoc = mode === 'subdoc' || mode === 'subpending'
  const us = []; const ex = []
  for (let i = 0; i < n; i++) { const [u, e] = gen(seed * 100003 + i, maxOps, drop, subdoc); us.push(u); ex.push(e) }
  write(process.argv[4], us, false)
  const eb = [Buffer.from(new Uint32Array([ex.length]).buffer)]
  for (const b of ex) eb.push(Buffer.from(new Int32Array([0]).buffer), Buffer.from(new Uint32Array([b.length]).buffer), Buffer.from(b))
  fs.writeFileSync(process.argv[5], Buffer.concat(eb.slice(1)))
}

module.exports = { session, textSession }
