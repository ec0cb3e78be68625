'use strict'
// Step2 wire corpus (MessageReceiver.ts:137-138; test tooling, runs against the image's yjs 13.5.16 bundle).
// The reference answers a SyncStep1 with Y.encodeStateAsUpdate(doc, sv) of the LIVE document.  For a document
// loaded from a stored state `u` (Database.ts:44-50) that is encodeStateAsUpdate(applyUpdate(new Doc, u), sv).
// For every session of the committed f-1 corpora (tests/golden/snapshot_v135.json.gz, snapshot_text_v135.json.gz)
// this records that payload for three state vectors: empty, a random cut of every client, the document's own.
// Also records whether it equals Y.diffUpdate(encodeStateAsUpdate(doc), sv) (the responder's computation:
// diffUpdate of the doc-normalized snapshot).
// pending: the corpora of states with lost updates (snapshot_pending_v135, snapshot_subdoc_v135), pending ones kept:
// encodeStateAsUpdate(doc, sv) then merges [writeStateAsUpdate(doc, sv), pendingDs, diffUpdate(pending structs, sv)]
//   node tools/step2_corpus.js <out.json.gz> [pending]
const fs = require('fs')
const zlib = require('zlib')
const path = require('path')
const Y = require(path.join(__dirname, 'yjs_bundle.js')).load()

function rng (seed) { let x = (seed >>> 0) || 1; return () => { x ^= x << 13; x >>>= 0; x ^= x >>> 17; x ^= x << 5; x >>>= 0; return x / 4294967296 } }
const pendingMode = process.argv[3] === 'pending'
const R = rng(pendingMode ? 20261018 : 20261017)
const hex = b => Buffer.from(b).toString('hex')
const unhex = h => Uint8Array.from(Buffer.from(h, 'hex'))
const rows = []
let same = 0; let differ = 0; let skipped = 0; let throws = 0
for (const f of pendingMode ? ['snapshot_pending_v135.json.gz', 'snapshot_subdoc_v135.json.gz'] : ['snapshot_v135.json.gz', 'snapshot_text_v135.json.gz']) {
  const src = JSON.parse(zlib.gunzipSync(fs.readFileSync(path.join(__dirname, '..', 'tests', 'golden', f))).toString())
  for (const [u] of src.rows) {
    const doc = new Y.Doc()
    Y.applyUpdate(doc, unhex(u))
    if (!pendingMode && (doc.store.pendingStructs || doc.store.pendingDs)) { skipped++; continue }   // (the pending corpus keeps them)
    const snap = Y.encodeStateAsUpdate(doc)
    const own = Y.decodeStateVector(pendingMode ? Y.encodeStateVectorFromUpdate(snap) : Y.encodeStateVector(doc))
    const cut = new Map()
    own.forEach((clock, client) => { if (R() < 0.8) cut.set(client, Math.floor(R() * (clock + 1))) })
    const svs = [new Uint8Array([0]), Y.encodeStateVector(cut), Y.encodeStateVector(doc)]
    if (pendingMode) svs.push(Y.encodeStateVectorFromUpdate(snap))   // (past the store's own: cuts inside the pending structs)
    for (const sv of svs) {
      // 13.5.16 throws where the cut splits a surrogate pair (writeString of a lone surrogate): recorded as null
      let step2 = null
      try { step2 = Y.encodeStateAsUpdate(doc, sv) } catch (e) { step2 = null; throws++ }
      let viaDiff = null
      try { viaDiff = Y.diffUpdate(snap, sv) } catch (e) { viaDiff = null }
      const eq = step2 === null ? viaDiff === null : viaDiff !== null && Buffer.compare(Buffer.from(viaDiff), Buffer.from(step2)) === 0
      if (eq) same++; else differ++
      rows.push([u, hex(sv), step2 === null ? null : hex(step2), eq ? 1 : 0])
    }
  }
}
const out = process.argv[2] || path.join(__dirname, '..', 'tests', 'golden', 'step2_v135.json.gz')
fs.writeFileSync(out, zlib.gzipSync(Buffer.from(JSON.stringify({
  source: 'tools/step2_corpus.js' + (pendingMode ? ' pending' : '') + ' (yjs 13.5.16 bundle) over the f-1 corpora; rows [state, sv, encodeStateAsUpdate(applyUpdate(new Doc, state), sv), equals diffUpdate(snapshot, sv)]',
  rows
})), { level: 9 }))
console.log(JSON.stringify({ rows: rows.length, diff_equal: same, diff_differs: differ, throws, pending_skipped: skipped }))
