'use strict'
// C1-shaped store window (SURVEY.md §8d C1; measurement tooling, runs on the GPU box):
// 1 000 Y.Text documents, each edited by 200 single-character inserts at random positions from one
// client, then every document's debounced store fires in the same window (the flush of
// Hocuspocus.ts:417-447 storeDocumentHooks).  Timed both ways, in one process, on the same documents:
//   reference : extension-database's onStoreDocument -- Y.encodeStateAsUpdate(document) per document
//               (packages/extension-database/src/Database.ts:55-60), yjs 13.5.16 from the image's bundle
//   gpumerge  : GpuMerge.onStoreDocument -- Y.mergeUpdates([base, ...log]) for the window in one
//               batched ygm_merge_v1 call through the N-API addon (src/index.js)
// Prints one JSON line: window latency (first store call -> last store resolved) for each path, and a
// byte-parity count of the GPU-stored states against yjs mergeUpdates of the same logs.
//   node tools/c1_store_latency.js [docs] [inserts]
const path = require('path')
const ROOT = path.join(__dirname, '..')
const Y = require(path.join(ROOT, 'tools', 'yjs_bundle.js')).load()
const { GpuMerge } = require(path.join(ROOT, 'packages', 'extension-gpu-merge', 'src', 'index.js'))
const { GpuEngine } = require(path.join(ROOT, 'packages', 'extension-gpu-merge', 'src', 'engine.js'))
const { MiniHocuspocus } = require(path.join(ROOT, 'packages', 'extension-gpu-merge', 'test', 'harness.js'))

const nDocs = parseInt(process.argv[2] || '1000', 10)
const nIns = parseInt(process.argv[3] || '200', 10)

function rng (seed) {   // xorshift32, seeded per document
  let x = (seed * 2654435761) >>> 0 || 1
  return () => { x ^= x << 13; x >>>= 0; x ^= x >>> 17; x ^= x << 5; x >>>= 0; return x }
}

class ReferenceStore {   // extension-database's store path (Database.ts:55-60)
  constructor (rows) { this.rows = rows; this.priority = 100 }
  async onStoreDocument ({ documentName, document }) { this.rows.set(documentName, Buffer.from(Y.encodeStateAsUpdate(document))) }
}

async function build (ext) {
  const hp = new MiniHocuspocus({ extensions: [ext], Y, debounce: 1e9, maxDebounce: 1e12 })
  const logs = []
  for (let d = 0; d < nDocs; d++) {
    const doc = await hp.loadDocument(`c1-${d}`)
    doc.clientID = 1 + (rng(d + 7)() % 0x7fffffff)
    const r = rng(d + 1)
    const log = []
    doc.on('update', u => log.push(u))
    const t = doc.getText('t')
    for (let i = 0; i < nIns; i++) t.doc.transact(() => t.insert(r() % (t.length + 1), String.fromCharCode(97 + (r() % 26))), 'connection')
    logs.push(log)
  }
  return { hp, logs }
}

async function window (hp) {
  const t0 = process.hrtime.bigint()
  await hp.flushAll()
  return Number(process.hrtime.bigint() - t0) / 1e6
}

async function main () {
  // reference path
  const refRows = new Map()
  const ref = await build(new ReferenceStore(refRows))
  const refMs = await window(ref.hp)
  // GPU path, in steady state: one untimed window of the same shape first, so the engine's device buffers and
  // pinned staging already have this window's size (a server sizes them on its first windows; growing them --
  // hipHostMalloc + the first DMA through new pinned pages -- is a one-off cost, not the store path's)
  const engine = new GpuEngine({ device: 0, batchWindowMs: 2, maxBatchDocs: 65536 })
  {
    const ext = new GpuMerge({ store: async () => {}, Y, engine })
    const warm = await build(ext)
    await window(warm.hp)
  }
  // the bare merge (normalize: false) first, then the default store (merge + GPU doc-normalized snapshot)
  const bareRows = new Map()
  const bare = await build(new GpuMerge({ store: async ({ documentName, state }) => bareRows.set(documentName, state), Y, engine, normalize: false }))
  const bareMs = await window(bare.hp)
  let sameBare = 0
  for (let d = 0; d < nDocs; d++) if (Buffer.compare(Buffer.from(Y.mergeUpdates(bare.logs[d])), Buffer.from(bareRows.get(`c1-${d}`))) === 0) sameBare++
  {
    const ext = new GpuMerge({ store: async () => {}, Y, engine })
    const warm = await build(ext)
    await window(warm.hp)
  }
  const gpuRows = new Map()
  const ext = new GpuMerge({ store: async ({ documentName, state }) => gpuRows.set(documentName, state), Y, engine })
  const gpu = await build(ext)
  const calls0 = engine.stats ? engine.stats().calls : null
  const gpuMs = await window(gpu.hp)
  const calls = engine.stats && calls0 !== null ? engine.stats().calls - calls0 : null
  const split = engine.timing.merge || null   // the window's merge batch: wait / pack / native / settle
  let same = 0, sameRef = 0
  for (let d = 0; d < nDocs; d++) {
    const fresh = new Y.Doc(); Y.applyUpdate(fresh, Y.mergeUpdates(gpu.logs[d]))
    const got = Buffer.from(gpuRows.get(`c1-${d}`))
    if (Buffer.compare(Buffer.from(Y.encodeStateAsUpdate(fresh)), got) === 0) same++
    if (Buffer.compare(Buffer.from(refRows.get(`c1-${d}`)), got) === 0) sameRef++
  }
  let inBytes = 0
  for (const l of gpu.logs) for (const u of l) inBytes += u.length
  engine.close()
  console.log(JSON.stringify({
    config: `C1: ${nDocs} Y.Text docs x ${nIns} single-char inserts (1 client each), one store window`,
    reference_store_ms: Math.round(refMs * 1000) / 1000,
    reference: 'extension-database onStoreDocument: Y.encodeStateAsUpdate(document) per document (yjs 13.5.16 bundle, Node ' + process.version + ')',
    gpumerge_store_ms: Math.round(gpuMs * 1000) / 1000,
    gpumerge: 'GpuMerge.onStoreDocument (default): Y.mergeUpdates([base, ...log]) batched through ygm_merge_v1, then the doc-normalized snapshot batched through ygm_snapshot_v1 (N-API addon)',
    gpumerge_bare_store_ms: Math.round(bareMs * 1000) / 1000,
    gpumerge_bare: 'GpuMerge({ normalize: false }): the merge batch only',
    gpumerge_engine_calls: calls,
    gpumerge_batch_split_ms: split && Object.fromEntries(Object.entries(split).map(([k, v]) => [k, typeof v === 'number' && !Number.isInteger(v) ? Math.round(v * 1000) / 1000 : v])),
    gpumerge_split_note: 'wait: first store -> batch flush (batch window); pack: JS batch arena (one copy per document, logs packed at capture); napi_in: addon call on the main thread; native: call -> promise settled, of which exec (worker: ygm_merge_v1 with pinned staging, H2D, kernels, D2H, result copy) and copy_out (result views); h2d / kernel / d2h: the engine\'s HIP-event times; settle: resolving the documents\' promises',
    log_bytes: inBytes,
    parity: `default: ${same}/${nDocs} stored states byte-identical to yjs encodeStateAsUpdate(applyUpdate(new Doc, mergeUpdates(log))), ${sameRef}/${nDocs} to the extension-database rows; normalize false: ${sameBare}/${nDocs} byte-identical to yjs mergeUpdates`
  }))
}

main().catch(e => { console.error(e); process.exit(1) })
