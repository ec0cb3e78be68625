'use strict'
// Extension tests: node test/run.js --cpu|--gpu
//  --cpu : the extension's hook logic with an injected engine double (Y.mergeUpdates of
//          the bundled yjs) -- no GPU in the build container
//  --gpu : the same scenarios through the real N-API addon on the MI355X, plus byte parity
//          of the stored state with yjs and batching checks
const path = require('path')
const assert = require('assert')
const { GpuMerge, GpuEnginePool, fnv1a64 } = require('../src/index.js')
const { frame, decodeSyncMessage, MessageType, SyncStep, SyncResponder } = require('../src/sync.js')
const { RedisFanout } = require('../src/redis.js')
const { MiniHocuspocus } = require('./harness.js')
const { UpdateLog, jobUpdates } = require('../src/log.js')
const { packJobs } = require('../src/engine.js')

const mode = process.argv.includes('--gpu') ? 'gpu' : 'cpu'
const Y = require(path.join(__dirname, '..', '..', '..', 'tools', 'yjs_bundle.js')).load()   // the test oracle: yjs from the image's bundle

// a per-document status, as GpuEngine rejects a refused document (YgmError code)
const refusal = fn => { try { return fn() } catch (e) { throw Object.assign(new Error(e.message), { code: 'EMALFORMED' }) } }

// an update whose struct section names a client twice (yjs's writers never do: outside the snapshot envelope)
function repeatsClient (u) {
  const seen = new Set()
  for (const [client] of Y.parseUpdateMeta(u).from) seen.add(client)
  let pos = 0
  const vu = () => { let v = 0; let m = 1; for (;;) { const b = u[pos++]; v += (b & 127) * m; if (b < 128) return v; m *= 128 } }
  const nb = vu()
  return nb > seen.size
}
class CpuDouble { // test double (never shipped): same API as GpuEngine
  constructor (device = 0) { this.calls = 0; this.device = device }
  async mergeUpdates (u) { this.calls++; return refusal(() => Y.mergeUpdates(u)) }
  async mergePacked (job) { this.calls++; return refusal(() => Y.mergeUpdates(jobUpdates(job))) }
  async mergeMany (docs) { this.calls++; return docs.map(u => { try { return Y.mergeUpdates(u) } catch (e) { return e } }) }   // per-document errors, as GpuEngine
  async diffMany (states, svs) { this.calls++; return states.map((u, i) => Y.diffUpdate(u, svs[i])) }
  async step2Many (states, svs) {   // the reference's reply for a document loaded from each state
    this.calls++
    return states.map((u, i) => {
      const d = new Y.Doc(); Y.applyUpdate(d, u)
      // the snapshot kernel's envelope: a repeated client block is EUNSUPPORTED (ygm_snapshot.hpp)
      if (repeatsClient(u)) return Object.assign(new Error('EUNSUPPORTED'), { code: 'EUNSUPPORTED' })
      return Y.encodeStateAsUpdate(d, svs[i])
    })
  }
  async stateVectorsMany (states) { this.calls++; return states.map(u => Y.encodeStateVectorFromUpdate(u)) }
  async snapshot (u) { this.calls++; const d = new Y.Doc(); Y.applyUpdate(d, u); return Y.encodeStateAsUpdate(d) }
  async snapshotMany (states) {
    this.calls++
    return states.map(u => {
      const d = new Y.Doc(); Y.applyUpdate(d, u)
      return Y.encodeStateAsUpdate(d)
    })
  }
  async containsMany (states, updates) {   // snapshotContainsUpdate(Y.snapshot(doc loaded from the state), update)
    this.calls++
    const { snapshotContains } = require('../src/sync.js')
    return states.map((s, i) => { const d = new Y.Doc(); Y.applyUpdate(d, s); return snapshotContains(Y, Y.snapshot(d), updates[i]) })
  }
  async mergeManyV2 (docs) { this.calls++; return docs.map(u => Y.mergeUpdatesV2(u)) }
  async diffManyV2 (states, svs) { this.calls++; return states.map((u, i) => Y.diffUpdateV2(u, svs[i])) }
  async stateVectorsManyV2 (states) { this.calls++; return states.map(u => Y.encodeStateVectorFromUpdateV2(u)) }
  stats () { return { calls: this.calls, device: this.device } }
  close () {}
}

function makeEngine () {
  if (mode === 'cpu') return new CpuDouble()
  const { GpuEngine } = require('../src/engine.js')
  return new GpuEngine({ device: 0, batchWindowMs: 5 })
}

const sleep = ms => new Promise(resolve => setTimeout(resolve, ms))
const tests = []
const test = (name, fn) => tests.push({ name, fn })

function memoryDb () {
  const rows = new Map()
  return { rows, fetch: async ({ documentName }) => rows.get(documentName) || null, store: async ({ documentName, state }) => { rows.set(documentName, state) } }
}

// tests/extension-s3/fetch.ts:92-114 -- stored state round-trips through fetch + applyUpdate
test('store -> fetch -> applyUpdate preserves content', async (engine) => {
  const db = memoryDb()
  const ext = new GpuMerge({ ...db, Y, engine })
  const hp = new MiniHocuspocus({ extensions: [ext], Y })
  const doc = await hp.loadDocument('hocuspocus-test')
  doc.transact(() => doc.getMap('map').set('attribute', 'value'), 'connection')
  await hp.flushAll(); await hp.lastStore
  assert.ok(db.rows.get('hocuspocus-test') instanceof Buffer)
  const hp2 = new MiniHocuspocus({ extensions: [new GpuMerge({ ...db, Y, engine })], Y })
  const doc2 = await hp2.loadDocument('hocuspocus-test')
  assert.strictEqual(doc2.getMap('map').get('attribute'), 'value')
})

// tests/server/onStoreDocument.ts:521-630 -- two debounced saves, a new client sees ["foo","bar"]
test('two saves then reload sees both', async (engine) => {
  const db = memoryDb()
  const hp = new MiniHocuspocus({ extensions: [new GpuMerge({ ...db, Y, engine })], Y })
  const doc = await hp.loadDocument('doc')
  doc.transact(() => doc.getArray('foo').push(['foo']), 'c1')
  await hp.flushAll(); await hp.lastStore
  doc.transact(() => doc.getArray('foo').push(['bar']), 'c1')
  await hp.flushAll(); await hp.lastStore
  const hp2 = new MiniHocuspocus({ extensions: [new GpuMerge({ ...db, Y, engine })], Y })
  const d2 = await hp2.loadDocument('doc')
  assert.deepStrictEqual(d2.getArray('foo').toArray(), ['foo', 'bar'])
})

// tests/server/onStoreDocument.ts:110-145 -- five changes, one store
test('five changes debounce into one store', async (engine) => {
  const db = memoryDb()
  const hp = new MiniHocuspocus({ extensions: [new GpuMerge({ ...db, Y, engine })], Y, debounce: 40 })
  const doc = await hp.loadDocument('d5')
  for (let i = 0; i < 5; i++) doc.transact(() => doc.getText('t').insert(0, String(i)), 'c1')
  await sleep(120); await hp.lastStore
  assert.strictEqual(hp.stores, 1)
  const d2 = await new MiniHocuspocus({ extensions: [new GpuMerge({ ...db, Y, engine })], Y }).loadDocument('d5')
  assert.strictEqual(d2.getText('t').toString(), '43210')
})

// tests/server/onChange.ts:60-80 + SURVEY.md §8b hazard 2: content added during load is persisted
test('content added by another extension during load is captured', async (engine) => {
  const db = memoryDb()
  const seeder = { priority: 50, async onLoadDocument ({ document }) { document.getText('t').insert(0, 'seeded') } }
  const hp = new MiniHocuspocus({ extensions: [new GpuMerge({ ...db, Y, engine }), seeder], Y })
  const doc = await hp.loadDocument('seeded')
  doc.transact(() => doc.getText('t').insert(6, '!'), 'c1')
  await hp.flushAll(); await hp.lastStore
  const d2 = await new MiniHocuspocus({ extensions: [new GpuMerge({ ...db, Y, engine })], Y }).loadDocument('seeded')
  assert.strictEqual(d2.getText('t').toString(), 'seeded!')
})

// normalize: false -- the stored state is byte-identical to Y.mergeUpdates([base, ...updates])
test('stored bytes == yjs mergeUpdates([snapshot, ...log]) (normalize: false)', async (engine) => {
  const db = memoryDb()
  const ext = new GpuMerge({ ...db, Y, engine, normalize: false })
  const hp = new MiniHocuspocus({ extensions: [ext], Y })
  const doc = await hp.loadDocument('bytes')
  const log = []
  doc.on('update', (u, o) => { if (o) log.push(u) })
  for (let i = 0; i < 20; i++) doc.transact(() => doc.getText('t').insert(Math.floor(Math.random() * (doc.getText('t').length + 1)), 'x' + i), 'c1')
  await hp.flushAll(); await hp.lastStore
  const first = db.rows.get('bytes')
  assert.strictEqual(Buffer.from(Y.mergeUpdates(log)).toString('hex'), first.toString('hex'))
  const log2 = []
  doc.on('update', (u, o) => { if (o) log2.push(u) })
  doc.transact(() => doc.getText('t').delete(0, 3), 'c1')
  doc.transact(() => doc.getText('t').insert(0, 'héllo 😀'), 'c1')
  await hp.flushAll(); await hp.lastStore
  assert.strictEqual(Buffer.from(Y.mergeUpdates([first].concat(log2))).toString('hex'), db.rows.get('bytes').toString('hex'))
})

// many documents storing in the same window share one GPU batch
test('concurrent stores of many documents', async (engine) => {
  const db = memoryDb()
  const hp = new MiniHocuspocus({ extensions: [new GpuMerge({ ...db, Y, engine })], Y })
  const docs = []
  for (let d = 0; d < 64; d++) docs.push(await hp.loadDocument('many-' + d))
  docs.forEach((doc, d) => { for (let i = 0; i < 10; i++) doc.transact(() => doc.getText('t').insert(0, String.fromCharCode(97 + ((d + i) % 26))), 'c') })
  const before = mode === 'gpu' ? engine.stats().calls : 0
  await hp.flushAll(); await hp.lastStore
  await sleep(20)
  for (let d = 0; d < 64; d++) {
    const d2 = await new MiniHocuspocus({ extensions: [new GpuMerge({ ...db, Y, engine })], Y }).loadDocument('many-' + d)
    assert.strictEqual(d2.getText('t').toString(), docs[d].getText('t').toString())
  }
  if (mode === 'gpu') assert.ok(engine.stats().calls - before <= 3, 'stores were batched')
})

// a failing document rejects only its own store (Hocuspocus.ts:431-435) -- with onRefused 'throw';
// by default it stores the live document's Y.encodeStateAsUpdate like extension-database instead
test('refused document: throws only its store, or stores the reference bytes', async (engine) => {
  const db = memoryDb()
  const payload = name => { const document = new Y.Doc(); document.getText('t').insert(0, 'live ' + name); return { documentName: name, document, context: {} } }
  const logOf = ups => { const l = new UpdateLog(); ups.forEach(u => l.push(u)); return l }
  const bad = () => ({ base: Uint8Array.from([1, 1, 5, 0, 4, 1, 1, 0x74]), log: logOf([Uint8Array.from([0, 0])]) }) // truncated base
  const strict = new GpuMerge({ ...db, Y, engine, onRefused: 'throw' })
  strict.docs.set('bad', bad())
  strict.docs.set('good', { base: null, log: logOf([Uint8Array.from([0, 0]), Uint8Array.from([0, 0])]) })
  const r = await Promise.allSettled([strict.onStoreDocument(payload('bad')), strict.onStoreDocument(payload('good'))])
  assert.strictEqual(r[0].status, 'rejected')
  assert.strictEqual(r[1].status, 'fulfilled')
  const lax = new GpuMerge({ ...db, Y, engine })
  lax.docs.set('bad', bad())
  const p = payload('bad')
  await lax.onStoreDocument(p)
  assert.strictEqual(lax.refused.length, 1)
  assert.strictEqual(db.rows.get('bad').toString('hex'), Buffer.from(Y.encodeStateAsUpdate(p.document)).toString('hex'))
  assert.strictEqual(lax.docs.get('bad').log.length, 0)
})

// a failed batch (device lost, out of memory, a rejected native call) is not a refusal: the store hook rejects
// (Hocuspocus.ts:431-435 logs and rethrows) instead of silently storing CPU bytes; the log is kept for a retry
test('failed batch rejects the store; no CPU fallback', async (engine) => {
  const db = memoryDb()
  const failing = { // engine double whose every batch fails as a dead device would
    async mergePacked () { throw Object.assign(new Error('hipErrorLaunchFailure'), { code: 'EDEVICE' }) },
    async mergeUpdates () { throw new Error('addon: batch rejected') },
    async snapshot () { throw Object.assign(new Error('out of device memory'), { code: 'ENOMEM' }) },
    close () {}
  }
  for (const onRefused of ['reference', 'throw']) {
    const ext = new GpuMerge({ ...db, Y, engine: failing, onRefused })
    const document = new Y.Doc()
    const log = new UpdateLog()
    document.on('update', u => log.push(u))
    document.getText('t').insert(0, 'a'); document.getText('t').insert(1, 'b')
    ext.docs.set('dead', { base: null, log })
    await assert.rejects(ext.onStoreDocument({ documentName: 'dead', document, context: {} }), /hipErrorLaunchFailure/)
    assert.strictEqual(db.rows.has('dead'), false)
    assert.strictEqual(ext.refused.length, 0)
    assert.strictEqual(ext.docs.get('dead').log.length, 2)   // nothing dropped
  }
  // the merge succeeds but the normalizing snapshot batch fails: still a rejection
  const ext = new GpuMerge({ ...db, Y, engine: { ...failing, mergePacked: async job => Y.mergeUpdates(jobUpdates(job)) } })
  const log = new UpdateLog(); log.push(Y.encodeStateAsUpdate(new Y.Doc())); log.push(Uint8Array.from([0, 0]))
  ext.docs.set('dead2', { base: null, log })
  await assert.rejects(ext.onStoreDocument({ documentName: 'dead2', document: new Y.Doc(), context: {} }), /out of device memory/)
  assert.strictEqual(db.rows.has('dead2'), false)
})

// the stored base is a copy of the document's bytes, not a view into the batch's shared result buffer
test('stored base does not pin the batch result buffer', async (engine) => {
  const db = memoryDb()
  const ext = new GpuMerge({ ...db, Y, engine })
  const hp = new MiniHocuspocus({ extensions: [ext], Y })
  const docs = []
  for (let d = 0; d < 8; d++) docs.push(await hp.loadDocument('pin-' + d))
  docs.forEach((doc, d) => doc.transact(() => doc.getText('t').insert(0, 'x'.repeat(d + 1)), 'c'))
  await hp.flushAll(); await hp.lastStore
  await sleep(20)
  for (let d = 0; d < 8; d++) {
    const b = ext.docs.get('pin-' + d).base
    assert.ok(b && b.byteLength === b.buffer.byteLength, 'base owns its buffer')
  }
})

// the log is captured by a document listener: an earlier extension whose onChange throws, or one that
// awaits I/O before a store / unload, cannot drop an update (Hocuspocus.ts:263, 465-479)
test('updates captured even when an earlier onChange throws or stalls', async (engine) => {
  const db = memoryDb()
  const thrower = { priority: 2000, async onChange () { throw new Error('boom') } }
  const staller = { priority: 1500, async onChange () { await sleep(50) } }
  for (const early of [thrower, staller]) {
    const ext = new GpuMerge({ ...db, Y, engine })
    const hp = new MiniHocuspocus({ extensions: [early, ext], Y })
    const name = 'guard-' + early.priority
    const doc = await hp.loadDocument(name)
    doc.transact(() => doc.getText('t').insert(0, 'abc'), 'c1')
    doc.transact(() => doc.getText('t').insert(3, 'def'), 'c1')
    await ext.onStoreDocument({ documentName: name, document: doc, context: {} })   // store right away
    await hp.unloadDocument(name)
    const d2 = await new MiniHocuspocus({ extensions: [new GpuMerge({ ...db, Y, engine })], Y }).loadDocument(name)
    assert.strictEqual(d2.getText('t').toString(), 'abcdef')
    assert.ok(!ext.docs.has(name))                                      // no orphan entry after unload
  }
})

// a reload of a document with deletions does not queue a duplicate of its delete set
test('afterLoadDocument adds nothing when the load added nothing', async (engine) => {
  const db = memoryDb()
  const hp = new MiniHocuspocus({ extensions: [new GpuMerge({ ...db, Y, engine })], Y })
  const doc = await hp.loadDocument('dels')
  doc.transact(() => doc.getText('t').insert(0, 'hello world'), 'c1')
  doc.transact(() => doc.getText('t').delete(0, 6), 'c1')
  await hp.flushAll(); await hp.lastStore
  const ext2 = new GpuMerge({ ...db, Y, engine })
  await new MiniHocuspocus({ extensions: [ext2], Y }).loadDocument('dels')
  assert.strictEqual(ext2.docs.get('dels').log.length, 0)
})

// SURVEY.md §8e: documents sharded over the node's GPUs by fnv1a64(documentName) mod N
// SURVEY.md §8f-1: normalize stores what extension-database stores for a fresh load of the merge --
// encodeStateAsUpdate(applyUpdate(new Doc, mergeUpdates(log))): deleted text garbage-collected
test('the default store is the doc-normalized snapshot of the merge', async (engine) => {
  const db = memoryDb()
  const ext = new GpuMerge({ ...db, Y, engine })
  const hp = new MiniHocuspocus({ extensions: [ext], Y })
  const doc = await hp.loadDocument('norm')
  doc.clientID = 7
  const log = []
  doc.on('update', u => log.push(u))
  const t = doc.getText('t')
  for (let i = 0; i < 40; i++) doc.transact(() => t.insert(i % 5 === 0 ? 0 : t.length, 'abc'.charAt(i % 3)), 'c1')
  doc.transact(() => t.delete(3, 20), 'c1')
  await hp.flushAll(); await hp.lastStore
  const merged = Y.mergeUpdates(log)
  const fresh = new Y.Doc(); Y.applyUpdate(fresh, merged)
  const expected = Buffer.from(Y.encodeStateAsUpdate(fresh))
  const stored = db.rows.get('norm')
  assert.strictEqual(Buffer.compare(stored, expected), 0)
  assert.ok(stored.length < Buffer.from(merged).length, 'garbage-collected snapshot is smaller than the merge')
  const back = new Y.Doc(); Y.applyUpdate(back, stored)
  assert.strictEqual(back.getText('t').toString(), t.toString())
  assert.deepStrictEqual(ext.unnormalized, [])
})

// a stored state whose history lost an update (its document keeps pending structs and a pending delete set) is
// normalized on the GPU as well: encodeStateAsUpdate merges [state, pendingDs, pending structs] (VERDICT r5 #9)
test('a state with pending structs and deletions is normalized like yjs', async (engine) => {
  const db = memoryDb()
  const src = new Y.Doc(); src.clientID = 11
  const ups = []; src.on('update', u => ups.push(u))
  const t0 = src.getText('t')
  t0.insert(0, 'abcdef'); t0.insert(6, 'ghij'); t0.delete(2, 5); t0.insert(1, 'XY')
  const base = Y.mergeUpdates([ups[0], ups[2], ups[3]])   // ups[1] never arrived
  db.rows.set('lost', Buffer.from(base))
  const ext = new GpuMerge({ ...db, Y, engine })
  const hp = new MiniHocuspocus({ extensions: [ext], Y })
  const doc = await hp.loadDocument('lost')
  doc.clientID = 12
  const log = []
  doc.on('update', u => log.push(u))
  doc.transact(() => doc.getText('t').insert(0, 'zz'), 'c1')
  await hp.flushAll(); await hp.lastStore
  const fresh = new Y.Doc(); Y.applyUpdate(fresh, Y.mergeUpdates([base, ...log]))
  assert.ok(fresh.store.pendingStructs && fresh.store.pendingDs, 'the state keeps pending structs and deletions')
  assert.strictEqual(Buffer.compare(db.rows.get('lost'), Buffer.from(Y.encodeStateAsUpdate(fresh))), 0)
  assert.deepStrictEqual(ext.unnormalized, [])
})

// normalizeMaxBytes: a merged state over the limit is stored as the bare merge (the snapshot kernel runs a document on
// one GPU thread: seconds for megabyte documents), counted in sizeSkipped; one under it is normalized as before
test('merged states over normalizeMaxBytes are stored as the bare merge', async (engine) => {
  const db = memoryDb()
  const ext = new GpuMerge({ ...db, Y, engine, normalizeMaxBytes: 200 })
  const hp = new MiniHocuspocus({ extensions: [ext], Y })
  const logs = {}
  for (const [name, n] of [['small', 4], ['large', 60]]) {
    const doc = await hp.loadDocument(name)
    doc.clientID = 9
    logs[name] = []
    doc.on('update', u => logs[name].push(u))
    const t = doc.getText('t')
    for (let i = 0; i < n; i++) doc.transact(() => t.insert(t.length, 'xy'), 'c1')
    doc.transact(() => t.delete(0, 2), 'c1')
  }
  await hp.flushAll(); await hp.lastStore
  const mergedLarge = Buffer.from(Y.mergeUpdates(logs.large))
  assert.ok(mergedLarge.length > 200)
  assert.strictEqual(Buffer.compare(db.rows.get('large'), mergedLarge), 0)
  const fresh = new Y.Doc(); Y.applyUpdate(fresh, Y.mergeUpdates(logs.small))
  assert.ok(Y.mergeUpdates(logs.small).length <= 200)
  assert.strictEqual(Buffer.compare(db.rows.get('small'), Buffer.from(Y.encodeStateAsUpdate(fresh))), 0)
  assert.strictEqual(ext.sizeSkipped, 1)
})

// SURVEY.md §8f-3 (Redis.ts:210-219, 336-372): changes publish Step1 in one batch; a remote instance's
// SyncStep1 is answered (SyncReply Step1 + Step2) in one batch, published back on the document channel
test('redis fan-out: batched first sync steps and remote Step2 replies', async (engine) => {
  const bus = []   // published [channel, buffer]
  const docs = new Map()
  const names = Array.from({ length: 12 }, (_, i) => `r-${i}`)
  for (const n of names) {
    const d = new Y.Doc(); d.clientID = 100 + docs.size
    d.getText('t').insert(0, 'hello ' + n)
    docs.set(n, d)
  }
  const getState = async n => Y.encodeStateAsUpdate(docs.get(n))
  const A = new RedisFanout({ engine, getState, publish: async (c, m) => bus.push([c, m]), identifier: 'host-A' })
  await Promise.all(names.map(n => A.onChange({ documentName: n, document: docs.get(n), transactionOrigin: 'connection' })))
  assert.strictEqual(A.batches.step1, 1)
  assert.strictEqual(bus.length, names.length)
  for (const [channel, buf] of bus) {
    const [id, msg] = A.decodeMessage(buf)
    assert.strictEqual(id, 'host-A')
    const d = decodeSyncMessage(msg)
    assert.strictEqual(channel, `hocuspocus:${d.documentName}`)
    assert.strictEqual(d.step, SyncStep.Step1)
    assert.deepStrictEqual(Array.from(Y.decodeStateVector(d.payload)), Array.from(Y.decodeStateVector(Y.encodeStateVector(docs.get(d.documentName)))))
  }
  // Redis-origin changes publish nothing; own messages are ignored
  await A.onChange({ documentName: names[0], transactionOrigin: A.redisTransactionOrigin })
  assert.strictEqual(bus.length, names.length)
  assert.strictEqual(await A.handleIncomingMessage('x', bus[0][1]), null)
  // instance B holds newer content and answers A's Step1 messages
  const bdocs = new Map(names.map(n => { const d = new Y.Doc(); Y.applyUpdate(d, Y.encodeStateAsUpdate(docs.get(n))); d.clientID = 900; d.getText('t').insert(0, 'B:'); return [n, d] }))
  const back = []
  const B = new RedisFanout({ engine, getState: async n => Y.encodeStateAsUpdate(bdocs.get(n)), publish: async (c, m) => back.push([c, m]), identifier: 'host-B' })
  const res = await Promise.all(bus.map(([c, m]) => B.handleIncomingMessage(c, m)))
  assert.strictEqual(B.batches.replies, 1)
  assert.ok(res.every(r => r.replied === 2))
  assert.strictEqual(back.length, 2 * names.length)
  for (let k = 0; k < names.length; k++) {
    const [, m1] = B.decodeMessage(back[2 * k][1]); const [, m2] = B.decodeMessage(back[2 * k + 1][1])
    const s1 = decodeSyncMessage(m1); const s2 = decodeSyncMessage(m2)
    assert.strictEqual(s1.messageType, MessageType.SyncReply); assert.strictEqual(s1.step, SyncStep.Step1)
    assert.strictEqual(s2.step, SyncStep.Step2)
    const sv = decodeSyncMessage(A.decodeMessage(bus[k][1])[1]).payload
    assert.strictEqual(Buffer.compare(Buffer.from(s2.payload), Buffer.from(Y.diffUpdate(Y.encodeStateAsUpdate(bdocs.get(s2.documentName)), sv))), 0)
    // A applies B's Step2 (what the host's MessageReceiver does with the returned message)
    const got = await A.handleIncomingMessage('x', back[2 * k + 1][1])
    Y.applyUpdate(docs.get(got.documentName), decodeSyncMessage(got.message).payload)
    assert.strictEqual(docs.get(got.documentName).getText('t').toString(), bdocs.get(got.documentName).getText('t').toString())
  }
})

// GpuMerge.redisFanout: the fan-out reads the extension's captured state (stored base + updates since)
test('redis fan-out over GpuMerge captured state', async (engine) => {
  const db = memoryDb()
  const ext = new GpuMerge({ ...db, Y, engine })
  const hp = new MiniHocuspocus({ extensions: [ext], Y })
  const doc = await hp.loadDocument('rf')
  doc.transact(() => doc.getText('t').insert(0, 'captured'), 'c1')
  const bus = []
  const fan = ext.redisFanout({ publish: async (c, m) => bus.push([c, m]), identifier: 'host-X', prefix: 'pfx' })
  await fan.onChange({ documentName: 'rf', transactionOrigin: 'c1' })
  assert.strictEqual(bus.length, 1)
  assert.strictEqual(bus[0][0], 'pfx:rf')
  const d = decodeSyncMessage(fan.decodeMessage(bus[0][1])[1])
  assert.deepStrictEqual(Array.from(Y.decodeStateVector(d.payload)), Array.from(Y.decodeStateVector(Y.encodeStateVector(doc))))
})

// MessageReceiver.ts:156-179: a read-only client's SyncStep2 is acked SyncStatus(true) when the document
// already contains it (Y.snapshotContainsUpdate), SyncStatus(false) otherwise -- one batch
test('read-only SyncStep2 acks through snapshotContainsUpdate, batched', async (engine) => {
  const doc = new Y.Doc(); doc.clientID = 5
  doc.getText('t').insert(0, 'abcdef'); doc.getText('t').delete(1, 2)
  const state = Y.encodeStateAsUpdate(doc)
  const peer = new Y.Doc(); Y.applyUpdate(peer, state); peer.clientID = 6
  const old = Y.encodeStateAsUpdate(doc)
  const grab = []; peer.on('update', u => grab.push(u))
  peer.getText('t').insert(0, 'new')
  const r = new SyncResponder({ engine, getState: async () => state })
  const msgs = [frame('ro', MessageType.Sync, SyncStep.Step2, old), frame('ro', MessageType.Sync, SyncStep.Step2, grab[0]), frame('ro', MessageType.Sync, SyncStep.Step1, Y.encodeStateVector(doc))]
  const out = await r.answerReadOnlyMany(msgs)
  assert.deepStrictEqual(Array.from(out[0]), [2, 0x72, 0x6f, 8, 1])
  assert.deepStrictEqual(Array.from(out[1]), [2, 0x72, 0x6f, 8, 0])
  assert.strictEqual(out[2], null)
})

// ADVICE r2: a store on the encodeStateAsUpdate path keeps the updates that arrive while storeMany is pending
test('refused store keeps updates applied while the database write is pending', async (engine) => {
  const rows = new Map()
  let release = null
  const slow = { fetch: async () => null, store: ({ documentName, state }) => new Promise(resolve => { release = () => { rows.set(documentName, state); resolve() } }) }
  const ext = new GpuMerge({ ...slow, Y, engine })
  const hp = new MiniHocuspocus({ extensions: [ext], Y })
  const doc = await hp.loadDocument('pending')
  doc.transact(() => doc.getText('t').insert(0, 'abc'), 'c1')
  const entry = ext.docs.get('pending')
  entry.base = Uint8Array.from([1, 1, 5, 0, 4, 1, 1, 0x74])   // a corrupt base: the engine refuses the merge
  const store = ext.onStoreDocument({ documentName: 'pending', document: doc, context: {} })
  while (!release) await sleep(1)
  doc.transact(() => doc.getText('t').insert(3, 'XYZ'), 'c1')   // arrives during storeMany
  release(); await store
  assert.strictEqual(ext.refused.length, 1)
  assert.strictEqual(entry.log.length, 1, 'the update applied during the write stays in the log')
  const back = new Y.Doc(); Y.applyUpdate(back, rows.get('pending'))
  assert.strictEqual(back.getText('t').toString(), 'abc')
  const next = Y.mergeUpdates([entry.base].concat(entry.log.toArray()))
  const full = new Y.Doc(); Y.applyUpdate(full, next)
  assert.strictEqual(full.getText('t').toString(), 'abcXYZ')
})

// ADVICE r2 / VERDICT r2 missing 5: a refused merge answers only its own read-only messages with the Error;
// a state outside the snapshot kernel's envelope (pending structs) gets the reference's answer (ADVICE r3):
// snapshotContainsUpdate(snapshot(doc), update) of the document loaded from it -- its integrated part holds `state`
test('read-only batch with a refused and a pending-struct document', async (engine) => {
  const doc = new Y.Doc(); doc.clientID = 5
  doc.getText('t').insert(0, 'abcdef')
  const state = Y.encodeStateAsUpdate(doc)
  const peer = new Y.Doc(); peer.clientID = 9; Y.applyUpdate(peer, state)
  const grab = []; peer.on('update', u => grab.push(u))
  peer.getText('t').insert(0, 'x'); peer.getText('t').insert(0, 'y')
  const pending = grab[1]                                            // client 9 clock 1 without clock 0: pending
  const states = { ok: [state], bad: [Uint8Array.from([1, 1, 5, 0, 4, 1, 1, 0x74]), Uint8Array.from([0, 0])], pend: [state, pending] }
  const r = new SyncResponder({ engine, getState: async n => states[n], Y })
  const msgs = [frame('ok', MessageType.Sync, SyncStep.Step2, state), frame('bad', MessageType.Sync, SyncStep.Step2, state),
    frame('pend', MessageType.Sync, SyncStep.Step2, state), frame('ok', MessageType.Sync, SyncStep.Step2, grab[0])]
  const out = await r.answerReadOnlyMany(msgs)
  assert.deepStrictEqual(Array.from(out[0]), [2, 0x6f, 0x6b, 8, 1])
  assert.ok(out[1] instanceof Error)
  assert.deepStrictEqual(Array.from(out[2]), [4, 0x70, 0x65, 0x6e, 0x64, 8, 1])
  assert.deepStrictEqual(Array.from(out[3]), [2, 0x6f, 0x6b, 8, 0])
  // ... and an update with the pending struct itself is new content for the live document
  const out2 = await r.answerReadOnlyMany([frame('pend', MessageType.Sync, SyncStep.Step2, pending)])
  assert.deepStrictEqual(Array.from(out2[0]), [4, 0x70, 0x65, 0x6e, 0x64, 8, 0])
})

// ADVICE r2: a failing Step1 batch is reported, never an unhandled rejection
test('redis fan-out reports a failed Step1 batch', async (engine) => {
  const seen = []
  const fan = new RedisFanout({ engine, getState: async () => { throw new Error('db down') }, publish: async () => {}, onError: e => seen.push(e) })
  await fan.onChange({ documentName: 'x', transactionOrigin: 'c1' })
  await sleep(5)
  assert.strictEqual(seen.length, 1)
  assert.strictEqual(seen[0].message, 'db down')
})

// the packed capture log and the batch packer (one copy per document at store time)
test('UpdateLog packs, drops and views captured updates; packJobs builds the batch arena', async () => {
  const log = new UpdateLog()
  const ups = []
  for (let i = 0; i < 300; i++) { const u = Uint8Array.from({ length: 1 + (i * 7) % 40 }, (_, k) => (i + k) & 255); ups.push(u); log.push(u) }
  assert.strictEqual(log.length, 300)
  const view = log.packed(120)
  const held = Buffer.from(view.arena)
  assert.deepStrictEqual(jobUpdates({ head: [], ...view }).map(u => Buffer.from(u).toString('hex')), ups.slice(0, 120).map(u => Buffer.from(u).toString('hex')))
  log.drop(120)
  log.push(Uint8Array.from([9, 9, 9]))
  assert.strictEqual(Buffer.compare(Buffer.from(view.arena), held), 0, 'a view handed to a batch keeps its bytes')
  assert.deepStrictEqual(log.toArray().map(u => Buffer.from(u).toString('hex')), ups.slice(120).concat([Uint8Array.from([9, 9, 9])]).map(u => Buffer.from(u).toString('hex')))
  const head = Uint8Array.from([1, 2])
  const jobs = [[Uint8Array.from([5]), Uint8Array.from([6, 7])], { head: [head], ...log.packed(3) }, []]
  const { arena, lens, docs } = packJobs(jobs)
  const flat = [Uint8Array.from([5]), Uint8Array.from([6, 7]), head].concat(log.toArray(3))
  assert.strictEqual(Buffer.compare(arena, Buffer.concat(flat.map(u => Buffer.from(u)))), 0)
  assert.deepStrictEqual(Array.from(lens), flat.map(u => u.length))
  assert.deepStrictEqual(Array.from(docs), [0, 0, 1, 1, 1, 1])
})

test('engine pool shards by fnv1a64(name) and keeps caller order', async () => {
  assert.strictEqual(fnv1a64('').toString(16), 'cbf29ce484222325')     // FNV-1a 64 published vectors
  assert.strictEqual(fnv1a64('foobar').toString(16), '85944171f73967e8')
  const pool = mode === 'cpu'
    ? new GpuEnginePool({ devices: [0, 1, 2], makeEngine: d => new CpuDouble(d) })
    : new GpuEnginePool({ devices: [0, 0], batchWindowMs: 1 })            // two contexts on the box's one GPU
  const names = []; const docs = []
  for (let d = 0; d < 24; d++) {
    const doc = new Y.Doc(); const ups = []
    doc.on('update', u => ups.push(u))
    for (let i = 0; i < 5; i++) doc.getText('t').insert(0, 'p' + d + i)
    names.push('shard-' + d); docs.push(ups)
  }
  const merged = await pool.mergeMany(names, docs)
  merged.forEach((m, i) => assert.strictEqual(Buffer.from(m).toString('hex'), Buffer.from(Y.mergeUpdates(docs[i])).toString('hex')))
  names.forEach(n => assert.strictEqual(pool.shardOf(n), Number(fnv1a64(n) % BigInt(pool.engines.length))))
  if (mode === 'cpu') {
    const used = new Set(names.map(n => pool.shardOf(n)))
    pool.engines.forEach((e, k) => assert.strictEqual(e.calls, used.has(k) ? 1 : 0))
  }
  const one = await pool.mergeUpdates(docs[3], names[3])
  assert.strictEqual(Buffer.from(one).toString('hex'), Buffer.from(Y.mergeUpdates(docs[3])).toString('hex'))
  // node-wide totals: the per-device counters summed (calls: one batch per used shard, then the single merge)
  const per = pool.stats(); const tot = pool.statsTotal()
  assert.strictEqual(tot.devices, pool.engines.length)
  assert.strictEqual(tot.calls, per.reduce((a, s) => a + s.calls, 0))
  assert.ok(tot.calls >= 2)
  pool.close()
})

// SURVEY.md §8f-2: a reconnect storm -- SyncStep1 from many clients -- answered in one batch
// every engine handle owns a native worker thread (addon/ygm_napi.c): an 8-GPU pool keeps 8 batches in flight at
// once, where libuv's 4-thread pool (napi_async_work) would serialize half of them
test('eight engine handles run eight native jobs at once', async () => {
  const { loadAddon } = require('../src/engine.js')
  const a = loadAddon()
  const hs = Array.from({ length: 8 }, () => a.openNull())
  const t0 = Date.now()
  const r = await Promise.all(hs.map(h => a.sleep(h, 150)))
  const lastStart = Math.max(...r.map(x => x.start)); const firstEnd = Math.min(...r.map(x => x.end))
  assert.ok(lastStart < firstEnd, 'all eight jobs were running at the same time')
  assert.ok(Date.now() - t0 < 8 * 150 / 2, 'not serialized')
  hs.forEach(h => a.close(h))
  if (mode === 'gpu') {   // eight contexts on the box's GPU, one batch each, all in flight together
    const { GpuEngine } = require('../src/engine.js')
    const engines = Array.from({ length: 8 }, () => new GpuEngine({ device: 0 }))
    const docs = Array.from({ length: 64 }, (_, d) => { const y = new Y.Doc(); const ups = []; y.on('update', u => ups.push(u)); for (let i = 0; i < 20; i++) y.getText('t').insert(0, String.fromCharCode(97 + (d + i) % 26)); return ups })
    const res = await Promise.all(engines.map(e => e.mergeMany(docs)))
    res.forEach(rr => rr.forEach((m, d) => assert.strictEqual(Buffer.from(m).toString('hex'), Buffer.from(Y.mergeUpdates(docs[d])).toString('hex'))))
    engines.forEach(e => e.close())
  }
})

// close() while a job is in flight: the job still settles, the handle stops after it, and later calls throw
// (the handle is freed only after its last completion has been delivered: addon/ygm_napi.c tsfn_finalize)
test('close during an in-flight job settles the job, then closes', async () => {
  const { loadAddon } = require('../src/engine.js')
  const a = loadAddon()
  const h = a.openNull()
  const p = a.sleep(h, 100)
  a.close(h)
  assert.throws(() => a.sleep(h, 1), /closed or invalid/)
  const r = await p
  assert.ok(r.end >= r.start + 90)
  assert.throws(() => a.sleep(h, 1), /closed or invalid/)
  a.close(h)   // idempotent
  // a handle dropped with a job pending is kept alive by the job (no use-after-free when it is collected)
  let h2 = a.openNull()
  const p2 = a.sleep(h2, 50)
  h2 = null
  if (global.gc) global.gc()
  const r2 = await p2
  assert.ok(r2.end >= r2.start + 40)
  if (global.gc) global.gc()
})

test('sync responder answers a SyncStep1 batch', async (engine) => {
  const db = memoryDb()
  const ext = new GpuMerge({ ...db, Y, engine })
  const hp = new MiniHocuspocus({ extensions: [ext], Y })
  const names = ['room-a', 'room-b', 'room-c']
  const snaps = {}
  for (const n of names) {
    const doc = await hp.loadDocument(n)
    doc.transact(() => doc.getText('t').insert(0, 'hello ' + n), 'c1')
    await hp.flushAll(); await hp.lastStore
    snaps[n] = Y.encodeStateVector(doc)                                   // a client that saw the first store
    doc.transact(() => doc.getText('t').insert(0, '> '), 'c2')          // captured log, not stored yet
    doc.transact(() => doc.getText('t').delete(2, 3), 'c2')
  }
  const msgs = []; const want = []
  for (const n of names) {
    for (const sv of [Uint8Array.from([0]), snaps[n]]) { msgs.push(frame(n, MessageType.Sync, SyncStep.Step1, sv)); want.push({ n, sv }) }
  }
  msgs.push(frame('room-a', 1, 0, Uint8Array.from([1, 2, 3])))          // awareness: not a sync message
  msgs.push(Uint8Array.from([5, 0x72, 0x6f]))                           // truncated
  const replies = await ext.syncResponder().answerMany(msgs)
  assert.strictEqual(replies[msgs.length - 2], null)
  assert.ok(replies[msgs.length - 1] instanceof Error)
  want.forEach(({ n, sv }, i) => {
    const e = ext.docs.get(n)
    const state = Y.mergeUpdates([e.base].concat(e.log.toArray()))
    const [step1, step2] = replies[i]                                   // the reference's order: server Step1, then Step2
    const a = decodeSyncMessage(step2); const b = decodeSyncMessage(step1)
    assert.strictEqual(a.documentName, n); assert.strictEqual(a.messageType, MessageType.Sync); assert.strictEqual(a.step, SyncStep.Step2)
    // the reference's bytes (MessageReceiver.ts:137-138) for the document loaded from the stored state
    const loaded = new Y.Doc(); Y.applyUpdate(loaded, state)
    assert.strictEqual(Buffer.from(a.payload).toString('hex'), Buffer.from(Y.encodeStateAsUpdate(loaded, sv)).toString('hex'))
    assert.ok(!replies[i].unnormalized)
    assert.strictEqual(b.step, SyncStep.Step1)
    assert.strictEqual(Buffer.from(b.payload).toString('hex'), Buffer.from(Y.encodeStateVectorFromUpdate(state)).toString('hex'))
    // a client at `sv` that applies the reply ends up with the server's content
    const client = new Y.Doc()
    if (sv.length > 1) Y.applyUpdate(client, db.rows.get(n))
    Y.applyUpdate(client, a.payload)
    assert.strictEqual(client.getText('t').toString(), hp.documents.get(n).getText('t').toString())
  })
})

// a state outside the snapshot envelope (a client block written twice: yjs keeps the second) is answered with
// diffUpdate(state, sv) and named, never sent silently as if it were the reference's bytes; a state whose history
// lost an update (pending structs in yjs) gets the reference's own reply
test('sync responder names Step2 replies outside the snapshot envelope', async (engine) => {
  const src = new Y.Doc(); const ups = []
  src.on('update', u => ups.push(u))
  src.getText('t').insert(0, 'ab'); src.getText('t').insert(2, 'cd')
  const pending = ups[1]                                            // depends on the first update: pending alone
  const good = Y.mergeUpdates(ups)
  const twice = Uint8Array.from([2, 1, 5, 0, 4, 1, 1, 0x74, 1, 0x61, 1, 5, 1, 0x84, 5, 0, 1, 0x62, 0])   // client 5's block twice
  const states = { pend: pending, good, twice }
  const r = new SyncResponder({ engine, getState: async n => states[n] })
  const msgs = ['pend', 'good', 'twice'].map(n => frame(n, MessageType.Sync, SyncStep.Step1, Uint8Array.from([0])))
  const out = await r.answerMany(msgs)
  for (const [k, state] of [[0, pending], [1, good]]) {
    assert.ok(!out[k].unnormalized)
    const loaded = new Y.Doc(); Y.applyUpdate(loaded, state)
    assert.strictEqual(Buffer.from(decodeSyncMessage(out[k][1]).payload).toString('hex'), Buffer.from(Y.encodeStateAsUpdate(loaded, Uint8Array.from([0]))).toString('hex'))
  }
  assert.strictEqual(out[2].unnormalized, true)
  assert.deepStrictEqual(r.unnormalized, ['twice'])
  assert.strictEqual(Buffer.from(decodeSyncMessage(out[2][1]).payload).toString('hex'), Buffer.from(Y.diffUpdate(twice, Uint8Array.from([0]))).toString('hex'))
})

test('update V2 batches match yjs mergeUpdatesV2 / diffUpdateV2 / encodeStateVectorFromUpdateV2', async (engine) => {
  const docs = []; const logs = []
  for (let k = 0; k < 24; k++) {
    const a = new Y.Doc(); a.clientID = 1000 + k; const b = new Y.Doc(); b.clientID = 5000 + k
    const log = []
    for (const d of [a, b]) d.on('updateV2', (u, origin) => { if (origin !== 'remote') log.push(u) })
    a.transact(() => a.getText('t').insert(0, 'hello ' + k, { bold: true }))
    Y.applyUpdateV2(b, Y.encodeStateAsUpdateV2(a), 'remote')
    b.transact(() => { b.getText('t').insert(2, 'é😀'); b.getMap('m').set('k', { n: k, s: 'x' }) })
    a.transact(() => a.getText('t').delete(0, 3))
    a.getXmlFragment('x').insert(0, [new Y.XmlElement('p')])
    docs.push(a); logs.push(log)
  }
  const merged = await engine.mergeManyV2(logs)
  logs.forEach((l, i) => assert.strictEqual(Buffer.from(merged[i]).toString('hex'), Buffer.from(Y.mergeUpdatesV2(l)).toString('hex')))
  const svs = await engine.stateVectorsManyV2(merged)
  merged.forEach((m, i) => assert.strictEqual(Buffer.from(svs[i]).toString('hex'), Buffer.from(Y.encodeStateVectorFromUpdateV2(m)).toString('hex')))
  const peer = logs.map(l => Y.encodeStateVectorFromUpdateV2(Y.mergeUpdatesV2(l.slice(0, 2))))
  const diffs = await engine.diffManyV2(merged, peer)
  merged.forEach((m, i) => assert.strictEqual(Buffer.from(diffs[i]).toString('hex'), Buffer.from(Y.diffUpdateV2(m, peer[i])).toString('hex')))
})

async function main () {
  const engine = makeEngine()
  let failed = 0
  for (const t of tests) {
    try { await t.fn(engine); console.log('ok   ' + t.name) } catch (e) { failed++; console.log('FAIL ' + t.name + '\n     ' + (e && e.stack)) }
  }
  engine.close()
  console.log(`${tests.length - failed}/${tests.length} passed (${mode})`)
  process.exit(failed ? 1 : 0)
}
main()
