'use strict'
// Read-only SyncStep2 corpus (MessageReceiver.ts:156-179; test tooling).  For each session of
// tools/snap_corpus.js the document is loaded fresh from its merged history; then:
//   contained updates : single updates of the history (every one is already in the document)
//   new structs       : an edit by a peer that synced the document first
//   new deletions     : a delete-only update of that peer removing live text
// The state handed to the GPU is Y.encodeStateAsUpdate(doc) (its delete set is Y.snapshot(doc).ds).
// Expected answer: Y.equalSnapshots(Y.snapshot(doc), Y.snapshot(doc after applying the update)) -- the
// meaning of yjs 13.6 snapshotContainsUpdate for updates that apply completely (no Skips, no pending
// structs or delete ranges), which is all this corpus makes; 13.6 itself is not in the image.
// pending: the sessions lose 1-3 updates (snap_corpus.js pending mode) and the state handed to the GPU is their merge
// `u` itself, whose loaded document keeps pending structs / a pending delete set.  Y.snapshot(doc) sees the store
// alone, so the expected answers are taken on the document of its integrated part A (encodeStateAsUpdate with the
// pending parts cleared), whose updates here all apply completely.
//   node tools/contains_corpus.js <n> <seed> <states.bin> <updates.bin> <expect.bin> [pending]
const fs = require('fs')
const path = require('path')
const Y = require(path.join(__dirname, 'yjs_bundle.js')).load()
const { session } = require('./snap_corpus.js')

function rng (seed) { let x = (seed >>> 0) || 1; return () => { x ^= x << 13; x >>>= 0; x ^= x >>> 17; x ^= x << 5; x >>>= 0; return x / 4294967296 } }
function writeBlobs (file, arr) {
  const parts = [Buffer.from(new Uint32Array([arr.length]).buffer)]
  for (const b of arr) parts.push(Buffer.from(new Uint32Array([b.length]).buffer), Buffer.from(b))
  fs.writeFileSync(file, Buffer.concat(parts))
}

const n = parseInt(process.argv[2] || '100', 10)
const seed = parseInt(process.argv[3] || '1', 10)
const R = rng(seed * 7919 + 1)
const pending = process.argv[7] === 'pending'
const states = []; const updates = []; const expect = []
for (let i = 0; i < n; i++) {
  const [u0] = session(seed * 100003 + i, pending ? 80 : 50, pending)
  const doc = new Y.Doc()
  Y.applyUpdate(doc, u0)
  if (pending) { doc.store.pendingStructs = null; doc.store.pendingDs = null }
  const state = Y.encodeStateAsUpdate(doc)
  const u = pending ? state : u0   // (the document the expectations are taken on)
  const snap = Y.snapshot(doc)
  const cand = []
  // parts of the history: the whole state, and its diff against a random earlier state vector
  cand.push(state)
  const cut = new Map()
  Y.decodeStateVector(Y.encodeStateVector(doc)).forEach((clock, client) => cut.set(client, Math.floor(R() * (clock + 1))))
  try { cand.push(Y.diffUpdate(u, Y.encodeStateVector(cut))) } catch (e) { /* 13.5 throws cutting a surrogate pair */ }
  // a peer that synced the document, then edits
  const peer = new Y.Doc(); peer.clientID = 0x7ffffff1 - i
  Y.applyUpdate(peer, state)
  const grab = []
  peer.on('update', (x, o, d, tr) => { if (tr.local) grab.push(x) })
  const t = peer.getText('text')
  if (R() < 0.5 || t.length === 0) t.insert(Math.floor(R() * (t.length + 1)), 'zq')
  else t.delete(Math.floor(R() * t.length), 1)
  cand.push(...grab)
  for (const c of cand) {
    const probe = new Y.Doc()
    Y.applyUpdate(probe, u)
    Y.applyUpdate(probe, c)
    states.push(pending ? u0 : state); updates.push(c)
    expect.push(Y.equalSnapshots(snap, Y.snapshot(probe)) ? 1 : 0)
  }
}
writeBlobs(process.argv[4], states)
writeBlobs(process.argv[5], updates)
fs.writeFileSync(process.argv[6], Buffer.from(Uint8Array.from(expect)))
console.log(JSON.stringify({ pairs: expect.length, contained: expect.reduce((a, b) => a + b, 0) }))
