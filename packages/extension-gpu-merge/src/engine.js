'use strict'
/**
 * GpuEngine -- Promise API over the N-API addon (addon/ygm_napi.c -> libygm.so).
 *
 * Requests from many documents that arrive within `batchWindowMs` (or until
 * `maxBatchDocs`) are packed into ONE GPU batch: the batch formation point is
 * the debounced store of Hocuspocus (packages/server/src/Hocuspocus.ts:417-447,
 * SURVEY.md §8a row a4).  One batch is in flight per engine; later requests
 * queue for the next batch.  A document whose status is not OK rejects only its
 * own promise, with yjs's error text (SURVEY.md §8b "Errors").
 */
const path = require('path')
const { jobUpdates } = require('./log')
const now = () => Number(process.hrtime.bigint()) / 1e6

let addon = null
function loadAddon () {
  if (!addon) addon = require(path.join(__dirname, '..', 'build', 'ygm_napi.node'))
  return addon
}

const STATUS = ['OK', 'EMALFORMED', 'ERANGE', 'ENONCANON', 'ESURROGATE', 'EDEPTH', 'ENOMEM', 'EDEVICE', 'EINVAL', 'EUNSUPPORTED']

class YgmError extends Error {
  constructor (code, message) {
    super(message)
    this.name = 'YgmError'
    this.code = STATUS[code] || String(code)
    this.status = code
  }
}

class Batcher {
  constructor (engine, op) {
    this.engine = engine
    this.op = op
    this.queue = []
    this.timer = null
    this.inflight = false
  }

  push (job) {
    return new Promise((resolve, reject) => {
      if (this.queue.length === 0) this.t_first = now()
      this.queue.push({ job, resolve, reject })
      if (this.queue.length >= this.engine.maxBatchDocs) this.kick(0)
      else this.kick(this.engine.batchWindowMs)
    })
  }

  kick (delay) {
    if (this.inflight) return
    if (delay === 0) { if (this.timer) { clearTimeout(this.timer); this.timer = null } setImmediate(() => this.flush()); return }
    if (!this.timer) this.timer = setTimeout(() => { this.timer = null; this.flush() }, delay)
  }

  async flush () {
    if (this.inflight || this.queue.length === 0) return
    const batch = this.queue.splice(0, this.engine.maxBatchDocs)
    this.inflight = true
    const t0 = now()
    try {
      const res = await this.engine._run(this.op, batch.map(b => b.job))
      const t1 = now()
      batch.forEach((b, i) => {
        const st = res.status[i]
        if (st === 0) b.resolve(res.outputs[i])
        else b.reject(new YgmError(st, loadAddon().strerror(st)))
      })
      // the last batch's time split (engine.timing[op]): window wait, JS packing, the native call (worker
      // execution + copy-out), settling the documents' promises
      this.engine.timing[this.op] = { docs: batch.length, wait_ms: t0 - (this.t_first || t0), ...this.engine._last, settle_ms: now() - t1 }
    } catch (e) {
      batch.forEach(b => b.reject(e))
    } finally {
      this.inflight = false
      if (this.queue.length) this.kick(this.queue.length >= this.engine.maxBatchDocs ? 0 : this.engine.batchWindowMs)
    }
  }
}

// one batch arena from merge jobs: an array of updates, or { head: Uint8Array[], arena, lens } whose log part is
// already packed (UpdateLog): one copy per document, and the per-update lengths / document ids by typed-array
// fills instead of per-update pushes
function packJobs (jobs) {
  let nUpd = 0; let total = 0
  for (const j of jobs) {
    if (Array.isArray(j)) { nUpd += j.length; for (const u of j) total += u.length } else {
      nUpd += j.head.length + j.lens.length; total += j.arena.length
      for (const u of j.head) total += u.length
    }
  }
  const arena = Buffer.allocUnsafe(total)
  const lens = new Uint32Array(nUpd)
  const docs = new Uint32Array(nUpd)
  let o = 0; let k = 0
  jobs.forEach((j, d) => {
    const k0 = k
    const ups = Array.isArray(j) ? j : j.head
    for (const u of ups) { arena.set(u, o); o += u.length; lens[k++] = u.length }
    if (!Array.isArray(j)) { arena.set(j.arena, o); o += j.arena.length; lens.set(j.lens, k); k += j.lens.length }
    docs.fill(d, k0, k)
  })
  return { arena, lens, docs }
}

function packBlobs (blobs) {
  const lens = new Uint32Array(blobs.length)
  let total = 0
  for (let i = 0; i < blobs.length; i++) { lens[i] = blobs[i].length; total += blobs[i].length }
  const arena = Buffer.allocUnsafe(total)
  let o = 0
  for (const b of blobs) { arena.set(b, o); o += b.length }
  return { arena, lens }
}

class GpuEngine {
  /**
   * @param {{device?: number, compat135?: boolean, batchWindowMs?: number, maxBatchDocs?: number}} [opts]
   */
  constructor (opts = {}) {
    this.device = opts.device || 0
    this.flags = opts.compat135 ? 1 : 0
    this.batchWindowMs = opts.batchWindowMs === undefined ? 2 : opts.batchWindowMs
    this.maxBatchDocs = opts.maxBatchDocs || 65536
    this.handle = loadAddon().open(this.device, this.flags)
    this.batchers = { merge: new Batcher(this, 'merge'), diff: new Batcher(this, 'diff'), sv: new Batcher(this, 'sv'), snapshot: new Batcher(this, 'snapshot') }
    this.timing = {}
    this._last = {}
    this.chain = Promise.resolve()
  }

  // one native batch at a time per handle (the addon enforces it; chain them here)
  _run (op, jobs) {
    const run = () => {
      const a = loadAddon()
      if (op === 'merge' || op === 'mergeV2') {
        const t0 = now()
        const { arena, lens, docs } = packJobs(jobs)
        const t1 = now()
        const s0 = this.stats()
        const p = (op === 'merge' ? a.mergeMany : a.mergeManyV2)(this.handle, arena, lens, docs, jobs.length)
        const t2 = now()
        return p.then(r => {
          const s1 = this.stats()
          this._last = { pack_ms: t1 - t0, napi_in_ms: t2 - t1, native_ms: now() - t2, exec_ms: r.execMs, copy_out_ms: r.completeMs,
            h2d_ms: s1.h2dMs - s0.h2dMs, kernel_ms: s1.kernelMs - s0.kernelMs, d2h_ms: s1.d2hMs - s0.d2hMs, bytes: arena.length }
          return r
        })
      }
      if (op === 'diff' || op === 'contains' || op === 'diffV2' || op === 'step2') {
        const u = packBlobs(jobs.map(j => j[0])); const s = packBlobs(jobs.map(j => j[1]))
        return ({ diff: a.diffMany, contains: a.containsMany, diffV2: a.diffManyV2, step2: a.step2Many })[op](this.handle, u.arena, u.lens, s.arena, s.lens)
      }
      const u = packBlobs(jobs)
      const unary = { snapshot: a.snapshotMany, sv: a.svMany, svV2: a.svManyV2, v1ToV2: a.convertManyV1ToV2, v2ToV1: a.convertManyV2ToV1 }
      return unary[op](this.handle, u.arena, u.lens)
    }
    const p = this.chain.then(run, run)
    this.chain = p.catch(() => {})
    return p
  }

  /** Y.mergeUpdates(updates), batched with concurrent callers. */
  mergeUpdates (updates) { return this.batchers.merge.push(updates.map(u => u instanceof Uint8Array ? u : Uint8Array.from(u))) }
  /** Y.mergeUpdates([...head, ...the packed updates]) for { head: Uint8Array[], arena, lens } (UpdateLog.packed) */
  mergePacked (job) { return this.batchers.merge.push(job) }
  /** Y.diffUpdate(update, stateVector) */
  diffUpdate (update, sv) { return this.batchers.diff.push([update, sv]) }
  /** Y.encodeStateVectorFromUpdate(update) */
  encodeStateVectorFromUpdate (update) { return this.batchers.sv.push(update) }
  /** Y.encodeStateAsUpdate(Y.applyUpdate(new Y.Doc(), update)): the doc-normalized snapshot (GC'd, merged) */
  snapshot (update) { return this.batchers.snapshot.push(update) }

  /** explicit batches (sync responders, bulk snapshot jobs) */
  async mergeMany (docs) { const r = await this._run('merge', docs); return unpack(r) }
  async diffMany (states, svs) { const r = await this._run('diff', states.map((s, i) => [s, svs[i]])); return unpack(r) }
  /** SyncStep2 payloads of stored documents: Y.encodeStateAsUpdate(doc, sv) of doc = Y.applyUpdate(new Y.Doc(), state)
   *  (MessageReceiver.ts:137-138) -- the snapshot, then a diff keeping each struct's parentSub bit; EUNSUPPORTED
   *  outside the snapshot envelope */
  async step2Many (states, svs) { const r = await this._run('step2', states.map((s, i) => [s, svs[i]])); return unpack(r) }
  async stateVectorsMany (states) { const r = await this._run('sv', states); return unpack(r) }
  async snapshotMany (states) { const r = await this._run('snapshot', states); return unpack(r) }
  /** Y.snapshotContainsUpdate(Y.snapshot(doc), update) per pair, `states` being normalized (snapshotMany) states */
  async containsMany (states, updates) {
    const r = await this._run('contains', states.map((s, i) => [s, updates[i]]))
    return unpack(r).map(x => x instanceof Error ? x : x[0] === 1)
  }

  /** update format V2 (yjs providers other than Hocuspocus's V1 path): Y.mergeUpdatesV2 / Y.diffUpdateV2 /
   *  Y.encodeStateVectorFromUpdateV2 / yjs 13.6 Y.convertUpdateFormatV1ToV2 / V2ToV1, as explicit batches */
  async mergeManyV2 (docs) { const r = await this._run('mergeV2', docs); return unpack(r) }
  async diffManyV2 (states, svs) { const r = await this._run('diffV2', states.map((s, i) => [s, svs[i]])); return unpack(r) }
  async stateVectorsManyV2 (states) { const r = await this._run('svV2', states); return unpack(r) }
  async convertManyV1ToV2 (updates) { const r = await this._run('v1ToV2', updates); return unpack(r) }
  async convertManyV2ToV1 (updates) { const r = await this._run('v2ToV1', updates); return unpack(r) }

  stats () { return loadAddon().stats(this.handle) }
  close () { if (this.handle) { loadAddon().close(this.handle); this.handle = null } }
}

function unpack (r) {
  return Array.from(r.status, (st, i) => st === 0 ? r.outputs[i] : new YgmError(st, loadAddon().strerror(st)))
}

const FNV_OFFSET = BigInt('0xcbf29ce484222325')
const FNV_PRIME = BigInt('0x100000001b3')
const U64 = BigInt('0xffffffffffffffff')
/** FNV-1a 64 over the UTF-8 bytes of a document name (SURVEY.md §8e: gpu = fnv1a64(name) mod N). */
function fnv1a64 (name) {
  let h = FNV_OFFSET
  for (const b of Buffer.from(String(name), 'utf8')) h = ((h ^ BigInt(b)) * FNV_PRIME) & U64
  return h
}

/**
 * Documents sharded over several GPUs of one node: one GpuEngine (context, stream, batcher) per
 * device, document -> device by fnv1a64(documentName) mod N, no cross-device traffic (documents
 * are independent; the reference scales by document too, docs/guides/scalability.md:12-14).
 * Same API as GpuEngine with a trailing document name; the *Many forms split a batch by shard,
 * run the shards concurrently (one native worker thread per device handle, addon/ygm_napi.c) and return results in caller order.
 */
class GpuEnginePool {
  constructor (opts = {}) {
    const devices = opts.devices && opts.devices.length ? opts.devices : [opts.device || 0]
    const make = opts.makeEngine || (device => new GpuEngine({ ...opts, device }))
    this.engines = devices.map(make)
  }

  shardOf (documentName) { return Number(fnv1a64(documentName) % BigInt(this.engines.length)) }
  engineFor (documentName) { return this.engines[this.shardOf(documentName)] }
  mergeUpdates (updates, documentName = '') { return this.engineFor(documentName).mergeUpdates(updates) }
  mergePacked (job, documentName = '') {
    const e = this.engineFor(documentName)
    return e.mergePacked ? e.mergePacked(job) : e.mergeUpdates(jobUpdates(job))
  }
  diffUpdate (update, sv, documentName = '') { return this.engineFor(documentName).diffUpdate(update, sv) }
  encodeStateVectorFromUpdate (update, documentName = '') { return this.engineFor(documentName).encodeStateVectorFromUpdate(update) }
  snapshot (update, documentName = '') { return this.engineFor(documentName).snapshot(update) }

  async _many (names, cols, run) {
    const parts = this.engines.map(() => [])
    names.forEach((n, i) => parts[this.shardOf(n)].push(i))
    const out = new Array(names.length)
    await Promise.all(parts.map(async (idx, e) => {
      if (!idx.length) return
      const r = await run(this.engines[e], ...cols.map(c => idx.map(i => c[i])))
      idx.forEach((i, k) => { out[i] = r[k] })
    }))
    return out
  }

  mergeMany (names, docs) { return this._many(names, [docs], (e, d) => e.mergeMany(d)) }
  diffMany (names, states, svs) { return this._many(names, [states, svs], (e, a, b) => e.diffMany(a, b)) }
  step2Many (names, states, svs) { return this._many(names, [states, svs], (e, a, b) => e.step2Many(a, b)) }
  stateVectorsMany (names, states) { return this._many(names, [states], (e, a) => e.stateVectorsMany(a)) }
  snapshotMany (names, states) { return this._many(names, [states], (e, a) => e.snapshotMany(a)) }
  containsMany (names, states, updates) { return this._many(names, [states, updates], (e, a, b) => e.containsMany(a, b)) }
  stats () { return this.engines.map(e => e.stats()) }
  /**
   * Node-wide totals (the reference's server-wide counters, Hocuspocus.ts:138-160): every numeric field of the
   * per-device stats summed over the pool's engines, plus `devices`.  Read on the host from each context's counters:
   * no collective, nothing crosses GPUs.
   */
  statsTotal () {
    const t = { devices: this.engines.length }
    for (const s of this.stats()) for (const [k, v] of Object.entries(s)) if (typeof v === 'number') t[k] = (t[k] || 0) + v
    return t
  }
  close () { this.engines.forEach(e => e.close()) }
}

module.exports = { packJobs, GpuEngine, GpuEnginePool, fnv1a64, YgmError, STATUS, loadAddon }
