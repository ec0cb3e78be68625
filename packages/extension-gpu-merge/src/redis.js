'use strict'
// Batched Redis fan-out (SURVEY.md §8f-3): the per-change work of @hocuspocus/extension-redis done as
// GPU batches.  The reference, per document and per event:
//   onChange (non-Redis origin)  -> publishFirstSyncStep: [Sync, Step1, encodeStateVector(doc)]
//                                   published on `${prefix}:${documentName}` (Redis.ts:210-219, 368-372)
//   a remote instance's message  -> MessageReceiver(message, redisOrigin).apply(doc, undefined, reply):
//                                   a SyncStep1 is answered with [SyncReply, Step1] and [Sync, Step2,
//                                   encodeStateAsUpdate(doc, sv)] published back (Redis.ts:336-363)
// Here changes arriving within `windowMs` share one GPU state-vector batch (stateVectorsMany over
// the documents' captured states), and remote SyncStep1 messages arriving within the window are
// answered by one SyncResponder batch (GPU diffMany).  Every other incoming message (Update,
// Step2, awareness) is handed back to the caller to apply as the reference does.
// Messages are framed as the reference frames them: [identifier length][identifier][message]
// (Redis.ts:142-180); an instance ignores its own messages.
// The state vector is encodeStateVectorFromUpdate(state) -- the same (client, clock) entries as the
// live document's encodeStateVector; yjs writes the latter's entries in struct-store order, so the
// bytes can differ in entry order while decoding to the same map.
const crypto = require('crypto')
const { SyncResponder, decodeSyncMessage, frame, MessageType, SyncStep } = require('./sync')

class RedisFanout {
  /**
   * @param {{engine: any, getState: (name: string) => Promise<Uint8Array|Uint8Array[]|null>,
   *          publish: (channel: string, message: Buffer) => any, identifier?: string, prefix?: string,
   *          windowMs?: number}} opts
   *   getState: the document's stored update or [snapshot, ...log] (GpuMerge: syncResponder()'s source)
   *   publish: the Redis client's publish (ioredis pub.publish)
   */
  constructor ({ engine, getState, publish, identifier, prefix = 'hocuspocus', windowMs = 2, onError }) {
    this.engine = engine
    this.getState = getState
    this.publish = publish
    this.identifier = identifier || `host-${crypto.randomBytes(8).toString('hex')}`
    this.prefix = prefix
    this.windowMs = windowMs
    this.redisTransactionOrigin = '__hocuspocus__redis__origin__'
    const id = Buffer.from(this.identifier, 'utf8')
    this.messagePrefix = Buffer.concat([Buffer.from([id.length]), id])
    this.responder = new SyncResponder({ engine, getState })
    this.pendingStep1 = new Map()   // documentName -> [resolve]
    this.pendingAsks = []           // { message, resolve, reject }
    this.t1 = null
    this.t2 = null
    this.batches = { step1: 0, replies: 0 }
    this.onError = onError || null
    this.errors = []   // failed Step1 publish batches (the change's onChange has already resolved)
  }

  // a failed background batch must not become an unhandled rejection (which ends a Node server):
  // it is recorded and reported, as the reference logs a failed publish
  _report (e) {
    this.errors.push(e)
    if (this.onError) this.onError(e)
    else console.error('[GpuMerge RedisFanout] Step1 publish batch failed:', e && e.message ? e.message : e)
  }

  pubKey (documentName) { return `${this.prefix}:${documentName}` }
  encodeMessage (message) { return Buffer.concat([this.messagePrefix, Buffer.from(message)]) }
  decodeMessage (buffer) {
    const n = buffer[0]
    return [buffer.toString('utf-8', 1, n + 1), buffer.slice(n + 1)]
  }

  _pooled () { return typeof this.engine.shardOf === 'function' }

  /** Redis.onChange: changes not made by Redis publish the document's first sync step (batched) */
  onChange (data) {
    if (data.transactionOrigin === this.redisTransactionOrigin) return Promise.resolve()
    return new Promise(resolve => {
      const waiters = this.pendingStep1.get(data.documentName) || []
      waiters.push(resolve)
      this.pendingStep1.set(data.documentName, waiters)
      if (!this.t1) this.t1 = setTimeout(() => { this.t1 = null; this._flushStep1().catch(e => this._report(e)) }, this.windowMs)
    })
  }

  async _flushStep1 () {
    const batch = this.pendingStep1
    this.pendingStep1 = new Map()
    const names = Array.from(batch.keys())
    if (!names.length) return
    this.batches.step1++
    try {
      const fetched = await Promise.all(names.map(n => this.getState(n)))
      const state = new Array(names.length)
      const toMerge = []
      fetched.forEach((f, k) => {
        const parts = Array.isArray(f) ? f.filter(Boolean) : (f ? [f] : [])
        if (parts.length > 1) toMerge.push(k)
        else state[k] = parts.length ? parts[0] : new Uint8Array([0, 0])
      })
      if (toMerge.length) {
        const parts = toMerge.map(k => (Array.isArray(fetched[k]) ? fetched[k] : [fetched[k]]).filter(Boolean))
        const merged = this._pooled() ? await this.engine.mergeMany(toMerge.map(k => names[k]), parts) : await this.engine.mergeMany(parts)
        toMerge.forEach((k, j) => { state[k] = merged[j] })
      }
      const okIdx = names.map((_, k) => k).filter(k => !(state[k] instanceof Error))
      const svs = this._pooled()
        ? await this.engine.stateVectorsMany(okIdx.map(k => names[k]), okIdx.map(k => state[k]))
        : await this.engine.stateVectorsMany(okIdx.map(k => state[k]))
      await Promise.all(okIdx.map((k, j) => svs[j] instanceof Error
        ? null
        : this.publish(this.pubKey(names[k]), this.encodeMessage(frame(names[k], MessageType.Sync, SyncStep.Step1, svs[j])))))
    } finally {
      batch.forEach(ws => ws.forEach(r => r()))
    }
  }

  /**
   * Redis.handleIncomingMessage: own messages are ignored; SyncStep1 requests are answered in a batch
   * (the replies are published back); anything else resolves to { documentName, message } for the host
   * to apply with its MessageReceiver (origin redisTransactionOrigin), as the reference does.
   */
  handleIncomingMessage (channel, data) {
    const [identifier, message] = this.decodeMessage(Buffer.from(data))
    if (identifier === this.identifier) return Promise.resolve(null)
    let d = null
    try { d = decodeSyncMessage(message) } catch (e) { d = null }
    if (!d || d.step !== SyncStep.Step1) return Promise.resolve({ documentName: d ? d.documentName : null, message })
    return new Promise((resolve, reject) => {
      this.pendingAsks.push({ message, resolve, reject })
      if (!this.t2) this.t2 = setTimeout(() => { this.t2 = null; this._flushAsks() }, this.windowMs)
    })
  }

  async _flushAsks () {
    const asks = this.pendingAsks
    this.pendingAsks = []
    if (!asks.length) return
    this.batches.replies++
    try {
      const out = await this.responder.answerMany(asks.map(a => a.message), { path: 'reply' })
      for (let i = 0; i < asks.length; i++) {   // in arrival order: a document's replies stay in the reference's wire order
        const a = asks[i]
        if (out[i] instanceof Error) { a.reject(out[i]); continue }
        const d = decodeSyncMessage(a.message)
        for (const r of out[i] || []) await this.publish(this.pubKey(d.documentName), this.encodeMessage(r))
        a.resolve({ documentName: d.documentName, replied: (out[i] || []).length })
      }
    } catch (e) {
      asks.forEach(a => a.reject(e))
    }
  }
}

module.exports = { RedisFanout }
