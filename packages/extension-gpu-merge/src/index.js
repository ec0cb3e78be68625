'use strict'
/**
 * @hocuspocus/extension-gpu-merge -- drop-in persistence extension whose
 * merge / diff / state-vector work runs on MI355X.
 *
 * Mirrors the reference's persistence contract:
 *   interface Extension            packages/server/src/types.ts:36-63
 *   DatabaseConfiguration{fetch,store}  packages/extension-database/src/Database.ts:10-20
 *   storePayload.state: Buffer     packages/server/src/types.ts:329-331
 *
 * What changes versus extension-database: instead of Y.encodeStateAsUpdate(doc)
 * on every debounced store (Database.ts:55-60), the stored state is
 * Y.mergeUpdates([base, ...updates since base]) computed in a GPU batch with
 * every other document whose store fires in the same window.  The stored bytes
 * are a valid V1 update of the same document state (mergeUpdates semantics,
 * byte-identical to yjs); loading applies it exactly as Database.ts:44-50 does.
 */
const { GpuEngine, GpuEnginePool, fnv1a64, YgmError } = require('./engine')
const { SyncResponder } = require('./sync')
const { RedisFanout } = require('./redis')
const { UpdateLog } = require('./log')

/**
 * A batched document store.  `fromDatabase` adapts any DatabaseConfiguration
 * (sqlite / s3 / custom) document by document.
 */
class DocumentStore {
  /** @returns {Promise<(Uint8Array|Uint8Array[]|null)[]>} */
  async fetchMany (payloads) { return payloads.map(() => null) }
  /** @param {{payload: any, state: Buffer}[]} entries */
  async storeMany (entries) {}

  static fromDatabase (config) {
    const s = new DocumentStore()
    s.fetchMany = payloads => Promise.all(payloads.map(p => config.fetch ? config.fetch(p) : null))
    s.storeMany = entries => Promise.all(entries.map(e => config.store ? config.store({ ...e.payload, state: e.state }) : undefined))
    return s
  }
}

class GpuMerge {
  /**
   * @param {{store?: DocumentStore|Function, fetch?: Function, device?: number, Y?: any,
   *          engine?: GpuEngine, batchWindowMs?: number, maxBatchDocs?: number, compat135?: boolean,
   *          onRefused?: 'reference'|'throw', normalize?: boolean, normalizeMaxBytes?: number}} configuration
   *   onRefused: what a store does when the engine refuses ONE document (a per-document status: content
   *   yjs would re-encode, ENONCANON; a corrupt stored base, EMALFORMED / ERANGE / ESURROGATE / EDEPTH) --
   *   'reference' (default): store Y.encodeStateAsUpdate(document) like extension-database and record it in
   *   `refused`; 'throw': reject the store.  A failed batch (EDEVICE, ENOMEM, EINVAL, an addon or driver
   *   error) always rejects the store (Hocuspocus logs and rethrows, Hocuspocus.ts:431-435): the product has
   *   no CPU fallback for a lost or failing GPU (SURVEY.md §5)
   *   normalize (default true): store the doc-normalized snapshot of the merge, Y.encodeStateAsUpdate(
   *   Y.applyUpdate(new Y.Doc(), merged)) computed on the GPU (SURVEY.md §8f-1) -- deleted content
   *   garbage-collected and adjacent structs merged, the bytes extension-database stores for a fresh load of
   *   the same updates (Database.ts:55-60); a document outside the snapshot kernel's envelope keeps its merged
   *   bytes (`unnormalized`).  normalize: false stores the bare Y.mergeUpdates bytes.
   *   normalizeMaxBytes (default 32768): merged states larger than this are stored as the bare merge (counted in
   *   `sizeSkipped`): the snapshot kernel runs a document on ONE GPU thread (yjs's integration is a serial chain),
   *   3-5 us per byte, and a batch takes its largest document's time: ~0.1-0.15 s at the limit, seconds for the ~1 MB
   *   documents of BASELINE config C5, whose merge takes milliseconds (DESIGN.md 6.R6, tools/snap_probe.py).  Both
   *   forms load identically.
   */
  constructor (configuration = {}) {
    this.extensionName = 'GpuMerge'
    // after Redis (priority 1000, which takes the store lock first), before plain storage extensions (100)
    this.priority = configuration.priority || 900
    this.configuration = configuration
    this.normalize = configuration.normalize !== false
    this.normalizeMaxBytes = configuration.normalizeMaxBytes === undefined ? 32768 : configuration.normalizeMaxBytes
    /** stores whose merged state was over normalizeMaxBytes (kept as the bare merge) */
    this.sizeSkipped = 0
    // drop-in for `new Database({ fetch, store })`, or a batched DocumentStore instance
    const st = configuration.store
    this.store = st && typeof st.storeMany === 'function'
      ? st
      : DocumentStore.fromDatabase({ fetch: configuration.fetch, store: typeof st === 'function' ? st : undefined })
    this.Y = configuration.Y || null
    this.engine = configuration.engine || null
    /** documentName -> { base: Uint8Array|null, log: UpdateLog (packed captured updates), doc?: Y.Doc, onUpdate?: Function } */
    this.docs = new Map()
    /** stores that fell back to Y.encodeStateAsUpdate(document) because the engine refused the merge */
    this.refused = []
    /** normalize: stores that kept the merged bytes (snapshot outside the kernel's envelope) */
    this.unnormalized = []
  }

  _Y () { if (!this.Y) this.Y = require('yjs'); return this.Y }
  _engine () {
    if (!this.engine) {
      const c = this.configuration
      const opts = { device: c.device || 0, compat135: c.compat135, batchWindowMs: c.batchWindowMs, maxBatchDocs: c.maxBatchDocs }
      // several GPUs of the node: documents sharded by fnv1a64(documentName) mod N (SURVEY.md §8e)
      this.engine = c.devices && c.devices.length > 1 ? new GpuEnginePool({ ...opts, devices: c.devices }) : new GpuEngine(opts)
    }
    return this.engine
  }

  /**
   * A batched SyncStep1 responder over this extension's captured state (stored snapshot + the
   * updates since): reconnect storms answered by one GPU diff batch (SURVEY.md §8f-2, src/sync.js).
   */
  syncResponder () {
    return new SyncResponder({
      engine: this._engine(),
      getState: async name => { const e = this.docs.get(name); return e ? (e.base ? [e.base] : []).concat(e.log.toArray()) : null }
    })
  }

  /** Batched extension-redis fan-out over the same captured state (SURVEY.md §8f-3, src/redis.js) */
  redisFanout ({ publish, identifier, prefix, windowMs }) {
    return new RedisFanout({ engine: this._engine(), getState: this.syncResponder().getState, publish, identifier, prefix, windowMs })
  }

  async onConfigure () { this._engine() }

  /** fetch -> (GPU merge of snapshot + log rows) -> Y.applyUpdate, as Database.onLoadDocument (Database.ts:44-50) */
  async onLoadDocument (data) {
    const [fetched] = await this.store.fetchMany([data])
    let state = null
    if (Array.isArray(fetched)) {
      const parts = fetched.filter(Boolean)
      state = parts.length === 0 ? null : parts.length === 1 ? parts[0] : await this._engine().mergeUpdates(parts, data.documentName)
    } else if (fetched) state = fetched
    if (state) this._Y().applyUpdate(data.document, state)
    this.docs.set(data.documentName, { base: state, log: new UpdateLog() })
  }

  /**
   * Content added while loading (other extensions' onLoadDocument, a returned Doc,
   * Hocuspocus.ts:357-372) never reaches onChange (the listener is registered after
   * load, :382-391): capture it once here (SURVEY.md §8b log-capture hazard 2) -- only when it
   * adds something (new structs, or deletions the base does not hold: encodeStateAsUpdate always
   * carries the whole delete set).  From here on every update of the document is captured by a
   * synchronous Y.Doc 'update' listener, not by onChange: Hocuspocus runs onChange through the
   * extension promise chain (Hocuspocus.ts:263, 465-479), where an earlier extension that throws or
   * awaits I/O would drop or delay it.
   */
  async afterLoadDocument (data) {
    const Y = this._Y()
    const entry = this.docs.get(data.documentName) || { base: null, log: new UpdateLog() }
    this.docs.set(data.documentName, entry)
    const baseSV = entry.base ? Y.encodeStateVectorFromUpdate(entry.base) : new Uint8Array([0])
    const missing = Y.encodeStateAsUpdate(data.document, baseSV)
    if (await addsToBase(this._engine(), missing, entry.base, data.documentName)) entry.log.push(missing)
    if (entry.doc && entry.onUpdate) entry.doc.off('update', entry.onUpdate)
    entry.doc = data.document
    entry.onUpdate = update => entry.log.push(update)
    data.document.on('update', entry.onUpdate)
  }

  /** every post-load update, whatever its origin (Hocuspocus.ts:263; hazard 1): captured by the
   * document listener of afterLoadDocument; onChange only covers a host that never ran that hook */
  async onChange (data) {
    let entry = this.docs.get(data.documentName)
    if (entry && entry.onUpdate) return
    if (!entry) { entry = { base: null, log: new UpdateLog() }; this.docs.set(data.documentName, entry) }
    entry.log.push(data.update)
  }

  /** store = mergeUpdates([base, ...log]) on the GPU, then the same store payload shape (Database.ts:55-60) */
  async onStoreDocument (data) {
    const entry = this.docs.get(data.documentName) || { base: null, log: new UpdateLog() }
    this.docs.set(data.documentName, entry)
    const taken = entry.log.length
    const nparts = (entry.base ? 1 : 0) + taken
    let state
    // updates the stored state holds: the `taken` ones, or -- when the state is the live document's
    // encodeStateAsUpdate -- every update captured up to that synchronous call (updates that arrive
    // while storeMany is pending are not in it and stay in the log)
    let cut = taken
    if (nparts === 0) { state = this._Y().encodeStateAsUpdate(data.document); cut = entry.log.length } // nothing captured: extension-database's bytes
    else if (nparts === 1) state = entry.base || new Uint8Array(entry.log.toArray(1)[0])   // (a copy: the log's buffer is reused)
    else {
      try {
        // the captured updates go to the batch as one packed range (UpdateLog): one copy per document
        const job = { head: entry.base ? [entry.base] : [], ...entry.log.packed(taken) }
        const eng = this._engine()
        state = await (eng.mergePacked ? eng.mergePacked(job, data.documentName) : eng.mergeUpdates(job.head.concat(entry.log.toArray(taken)), data.documentName))
        if (this.normalize && state.byteLength <= this.normalizeMaxBytes) state = await this._normalize(state, data.documentName)
        else if (this.normalize) this.sizeSkipped++
      } catch (e) {
        // a document the engine refuses (content yjs would re-encode, YGM_ENONCANON; a corrupt stored
        // base): unless configured to throw, store what extension-database stores for it -- the live
        // document's Y.encodeStateAsUpdate (Database.ts:58) -- so it keeps persisting.  Anything else (the
        // device, memory, a rejected batch) rejects the hook.
        if (!isRefusal(e) || this.configuration.onRefused === 'throw') throw e
        this.refused.push({ documentName: data.documentName, code: e.code || String(e) })
        state = this._Y().encodeStateAsUpdate(data.document)
        cut = entry.log.length
      }
    }
    // engine results are views into one buffer per batch: keep a copy of exactly this document's bytes, so
    // the long-lived base (and the stored Buffer) do not pin the whole batch's result buffer
    if (state.byteLength !== state.buffer.byteLength) state = new Uint8Array(state)
    await this.store.storeMany([{ payload: data, state: Buffer.from(state.buffer, state.byteOffset, state.byteLength) }])
    // the stored state becomes the new base (under the document's saveMutex, Hocuspocus.ts:427)
    entry.base = state
    entry.log.drop(cut)
  }

  // the doc-normalized snapshot of a merged state; outside the kernel's envelope the merge is kept
  async _normalize (state, documentName) {
    try {
      return await this._engine().snapshot(state, documentName)
    } catch (e) {
      if (e && e.code === 'EUNSUPPORTED') { this.unnormalized.push({ documentName, code: e.code }); return state }
      throw e
    }
  }

  async afterUnloadDocument (data) {
    const entry = this.docs.get(data.documentName)
    if (entry && entry.doc && entry.onUpdate) entry.doc.off('update', entry.onUpdate)
    this.docs.delete(data.documentName)
  }

  async onDestroy () { if (this.engine && !this.configuration.engine) this.engine.close(); this.engine = null }
}

// per-document statuses (the batch ran; this document's input was refused), as opposed to batch failures
const REFUSALS = new Set(['EMALFORMED', 'ERANGE', 'ENONCANON', 'ESURROGATE', 'EDEPTH'])
function isRefusal (e) { return !!e && REFUSALS.has(e.code) }

// does `missing` (encodeStateAsUpdate(doc, baseSV)) add structs, or deletions that `base` does not hold?
// Without structs its delete set is the document's whole delete set: it adds nothing iff merging it
// into the base leaves the base's (sorted, merged) delete set unchanged -- decided by two engine merges.
async function addsToBase (engine, missing, base, name) {
  if (missing.length > 0 && missing[0] !== 0) return true                  // struct blocks
  if (missing.length === 2 && missing[1] === 0) return false               // nothing at all
  if (!base) return true
  const [withIt, without] = await Promise.all([engine.mergeUpdates([base, missing], name), engine.mergeUpdates([base, Uint8Array.from([0, 0])], name)])
  return Buffer.compare(Buffer.from(withIt), Buffer.from(without)) !== 0
}

module.exports = { GpuMerge, DocumentStore, isRefusal, GpuEngine, GpuEnginePool, SyncResponder, RedisFanout, UpdateLog, fnv1a64, YgmError }
