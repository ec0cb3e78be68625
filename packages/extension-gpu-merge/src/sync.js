'use strict'
// Batched sync responder (SURVEY.md §8f-2): answers many SyncStep1 messages -- a reconnect storm --
// with one GPU diff batch instead of one encodeStateAsUpdate(doc, sv) per connection.
//
// Wire format (packages/server/src/types.ts:12-23 MessageType, OutgoingMessage.ts:17-50,
// Connection.ts:180-186, MessageReceiver.ts:29-60 / 120-155, y-protocols/sync):
//   message = varString(documentName) varUint(MessageType) payload
//   Sync payload: varUint(step: 0 Step1 | 1 Step2 | 2 Update) varUint8Array(stateVector | update)
// The reference replies to Step1 with [Sync, Step2, encodeStateAsUpdate(doc, sv)] and then sends its
// own first sync step [SyncReply (or Sync), Step1, encodeStateVector(doc)] (MessageReceiver.ts:137-155).
// Here a document's state is its stored update (snapshot + captured log, merged on the GPU) and the
// Step2 payload is the reference's own bytes for a document loaded from that state:
// encodeStateAsUpdate(applyUpdate(new Doc, state), sv) -- the GPU snapshot of the state (§8f-1), then a diff
// in which every struct keeps its parentSub bit (step2Many, ygm_sync_step2_v1; pinned against yjs by
// tests/test_step2.py).  A state outside the snapshot kernel's envelope (pending structs or delete set,
// sub-documents) is answered with diffUpdate(state, sv) -- the same content, not the same bytes -- and
// NAMED: its reply array carries `unnormalized: true` and the document is listed in
// responder.unnormalized.  The server's Step1 carries encodeStateVectorFromUpdate(state).

const MessageType = { Sync: 0, SyncReply: 4 }
const SyncStep = { Step1: 0, Step2: 1, Update: 2 }

// lib0 decoding (L0@2955 readVarUint, L0@3467 readVarString): a reader over one message
class Reader {
  constructor (buf) { this.buf = buf; this.pos = 0 }
  varUint () {
    let num = 0; let mult = 1
    for (;;) {
      if (this.pos >= this.buf.length) throw new Error('Unexpected end of array')
      const r = this.buf[this.pos++]
      num += (r & 127) * mult
      mult *= 128
      if (r < 128) return num
      if (num > Number.MAX_SAFE_INTEGER) throw new Error('Integer out of Range')
    }
  }
  varUint8Array () {
    const n = this.varUint()
    if (this.pos + n > this.buf.length) throw new Error('Unexpected end of array')
    const s = this.buf.subarray(this.pos, this.pos + n); this.pos += n; return s
  }
  varString () { return Buffer.from(this.varUint8Array()).toString('utf8') }
}

// lib0 encoding (L0@7250 writeVarUint, L0@7454 writeVarString)
function varUintBytes (v) {
  const out = []
  while (v > 127) { out.push(0x80 | (v % 128)); v = Math.floor(v / 128) }
  out.push(v)
  return out
}
function frame (documentName, type, step, payload) {
  const name = Buffer.from(documentName, 'utf8')
  const head = [...varUintBytes(name.length), ...name, ...varUintBytes(type), ...varUintBytes(step), ...varUintBytes(payload.length)]
  const out = new Uint8Array(head.length + payload.length)
  out.set(head, 0); out.set(payload, head.length)
  return out
}

/** { documentName, messageType, step, payload } of a Sync / SyncReply message, or null for other types. */
function decodeSyncMessage (message) {
  const r = new Reader(message)
  const documentName = r.varString()
  const messageType = r.varUint()
  if (messageType !== MessageType.Sync && messageType !== MessageType.SyncReply) return null
  const step = r.varUint()
  return { documentName, messageType, step, payload: r.varUint8Array() }
}

class SyncResponder {
  /**
   * @param {{ engine: any, getState: (documentName: string) => Promise<Uint8Array | Uint8Array[] | null> }} opts
   *   engine: GpuEngine or GpuEnginePool; getState: the document's stored update, or [snapshot, ...log]
   */
  constructor ({ engine, getState, Y = null }) {
    this.engine = engine; this.getState = getState
    this.Y = Y   // yjs, for the read-only answer of a document outside the snapshot envelope (loaded lazily)
    /** Step1 replies sent as diffUpdate(state, sv) because the state is outside the snapshot envelope */
    this.unnormalized = []
  }

  _pooled () { return typeof this.engine.shardOf === 'function' }
  _Y () { if (!this.Y) this.Y = require('yjs'); return this.Y }
  _merge (names, docs) { return this._pooled() ? this.engine.mergeMany(names, docs) : this.engine.mergeMany(docs) }
  _diff (names, states, svs) { return this._pooled() ? this.engine.diffMany(names, states, svs) : this.engine.diffMany(states, svs) }
  _step2 (names, states, svs) { return this._pooled() ? this.engine.step2Many(names, states, svs) : this.engine.step2Many(states, svs) }
  _svs (names, states) { return this._pooled() ? this.engine.stateVectorsMany(names, states) : this.engine.stateVectorsMany(states) }

  /**
   * Answers a batch of incoming messages.  For each SyncStep1 message the result is [server Step1,
   * Step2 reply] (the reference's wire order): path 'connection' (Connection.handleMessage -> MessageReceiver.apply(doc, connection),
   * the websocket path) always sends the server Step1 as a Sync message; path 'reply' (apply with a
   * reply callback) sends it as SyncReply, and only for Sync requests (requestFirstSync,
   * MessageReceiver.ts:39-47 / 137-155); path 'none' omits it.  Other messages give null; a
   * malformed message or document gives an Error for that message only.
   */
  async answerMany (messages, { path = 'connection' } = {}) {
    const requestFirstSync = path !== 'none'
    const out = new Array(messages.length).fill(null)
    const asks = []
    messages.forEach((m, i) => {
      try {
        const d = decodeSyncMessage(m)
        if (d && d.step === SyncStep.Step1) asks.push({ i, ...d })
      } catch (e) { out[i] = e }
    })
    if (!asks.length) return out
    // one state per document: fetched in parallel, multi-part logs merged in one GPU batch
    const names = Array.from(new Set(asks.map(a => a.documentName)))
    const fetched = await Promise.all(names.map(n => this.getState(n)))
    const state = new Map()
    const toMerge = []
    names.forEach((n, k) => {
      const f = fetched[k]
      const parts = Array.isArray(f) ? f.filter(Boolean) : (f ? [f] : [])
      if (parts.length > 1) toMerge.push({ n, parts })
      else state.set(n, parts.length ? parts[0] : new Uint8Array([0, 0]))
    })
    if (toMerge.length) {
      const merged = await this._merge(toMerge.map(t => t.n), toMerge.map(t => t.parts))
      toMerge.forEach((t, k) => state.set(t.n, merged[k]))
    }
    const live = asks.filter(a => !(state.get(a.documentName) instanceof Error))
    asks.filter(a => state.get(a.documentName) instanceof Error).forEach(a => { out[a.i] = state.get(a.documentName) })
    const diffs = await this._step2(live.map(a => a.documentName), live.map(a => state.get(a.documentName)), live.map(a => a.payload))
    // states the snapshot kernel does not take: diffUpdate of the state itself, named as such
    const unsup = live.map((a, k) => diffs[k] instanceof Error && diffs[k].code === 'EUNSUPPORTED' ? k : -1).filter(k => k >= 0)
    if (unsup.length) {
      const plain = await this._diff(unsup.map(k => live[k].documentName), unsup.map(k => state.get(live[k].documentName)), unsup.map(k => live[k].payload))
      unsup.forEach((k, j) => {
        diffs[k] = plain[j]
        if (!(plain[j] instanceof Error)) { plain[j].unnormalized = true; this.unnormalized.push(live[k].documentName) }
      })
    }
    let ownSv = new Map()
    if (requestFirstSync) {
      const svs = await this._svs(names, names.map(n => state.get(n) instanceof Error ? new Uint8Array([0, 0]) : state.get(n)))
      ownSv = new Map(names.map((n, k) => [n, svs[k]]))
    }
    live.forEach((a, k) => {
      if (diffs[k] instanceof Error) { out[a.i] = diffs[k]; return }
      // wire order of the reference: the server Step1 is sent while the request is read
      // (MessageReceiver.ts:141-153), the Step2 reply after it (apply(), :50-61)
      const replies = []
      const sv = ownSv.get(a.documentName)
      if (sv && !(sv instanceof Error)) {
        if (path === 'connection') replies.push(frame(a.documentName, MessageType.Sync, SyncStep.Step1, sv))
        else if (path === 'reply' && a.messageType === MessageType.Sync) replies.push(frame(a.documentName, MessageType.SyncReply, SyncStep.Step1, sv))
      }
      replies.push(frame(a.documentName, MessageType.Sync, SyncStep.Step2, diffs[k]))
      if (diffs[k].unnormalized) replies.unnormalized = true
      out[a.i] = replies
    })
    return out
  }
}

// yjs 13.6 snapshotContainsUpdate(snapshot, update) for a yjs that does not export it (13.5): every struct of the
// update (Skips included: the lazy reader does not filter them) inside the snapshot's state vector -- parseUpdateMeta's
// per-client end clocks -- and the snapshot's delete set unchanged by merging the update's in (mergeDeleteSets +
// sortAndMergeDeleteSet: ranges sorted by clock, a range that reaches the next one's clock absorbs it; then
// equalDeleteSets).  The update's delete set: diffUpdate against its own state vector leaves only it.
function snapshotContains (Y, snap, update) {
  for (const [client, clock] of Y.parseUpdateMeta(update).to) if ((snap.sv.get(client) || 0) < clock) return false
  const r = new Reader(Y.diffUpdate(update, Y.encodeStateVectorFromUpdate(update)))
  if (r.varUint() !== 0) return false
  const ds = new Map()
  for (let c = r.varUint(); c > 0; c--) {
    const client = r.varUint(); const items = ds.get(client) || []
    for (let n = r.varUint(); n > 0; n--) items.push({ clock: r.varUint(), len: r.varUint() })
    ds.set(client, items)
  }
  for (const [client, items] of ds) {
    const base = snap.ds.clients.get(client) || []
    const all = base.concat(items).map(d => ({ clock: d.clock, len: d.len })).sort((x, y) => x.clock - y.clock)
    const runs = []
    for (const d of all) {
      const last = runs[runs.length - 1]
      if (last && last.clock + last.len >= d.clock) last.len = Math.max(last.len, d.clock + d.len - last.clock)
      else runs.push(d)
    }
    if (runs.length !== base.length || runs.some((r, i) => r.clock !== base[i].clock || r.len !== base[i].len)) return false
  }
  return true
}

// [varString(documentName) varUint(SyncStatus = 8) varUint(saved ? 1 : 0)] (OutgoingMessage.ts:128-135)
function syncStatusFrame (documentName, saved) {
  const name = Buffer.from(documentName, 'utf8')
  return Uint8Array.from([...varUintBytes(name.length), ...name, 8, saved ? 1 : 0])
}

/**
 * Read-only connections (MessageReceiver.ts:156-179): a SyncStep2 from a read-only client is not
 * applied; the server acks SyncStatus(true) when Y.snapshotContainsUpdate(Y.snapshot(doc), update)
 * (nothing new) and SyncStatus(false) otherwise.  Batched: the documents' states merged on the GPU, then
 * one GPU containment batch (which normalizes the states to their Y.snapshot view itself).  Returns per
 * message the SyncStatus frame, null for other messages, or an Error.
 */
SyncResponder.prototype.answerReadOnlyMany = async function (messages) {
  const out = new Array(messages.length).fill(null)
  const asks = []
  messages.forEach((m, i) => {
    try {
      const d = decodeSyncMessage(m)
      if (d && d.step === SyncStep.Step2) asks.push({ i, ...d })
    } catch (e) { out[i] = e }
  })
  if (!asks.length) return out
  const names = Array.from(new Set(asks.map(a => a.documentName)))
  const fetched = await Promise.all(names.map(n => this.getState(n)))
  const parts = fetched.map(f => Array.isArray(f) ? f.filter(Boolean) : (f ? [f] : []))
  const merged = await this._merge(names, parts.map(p => p.length ? p : [new Uint8Array([0, 0])]))
  const mergedOf = new Map(names.map((n, k) => [n, merged[k]]))
  // a document whose merge the engine refuses answers with that Error; the other states go to one containment batch as
  // merged: the engine takes their Y.snapshot view itself (the snapshot kernels; for a state that leaves pending
  // structs or a pending delete set, its integrated part -- what Y.snapshot(doc) sees in the store)
  asks.filter(a => mergedOf.get(a.documentName) instanceof Error).forEach(a => { out[a.i] = mergedOf.get(a.documentName) })
  const live = asks.filter(a => !(mergedOf.get(a.documentName) instanceof Error))
  if (!live.length) return out
  const stateOf = a => mergedOf.get(a.documentName)
  const res = await (this._pooled()
    ? this.engine.containsMany(live.map(a => a.documentName), live.map(stateOf), live.map(a => a.payload))
    : this.engine.containsMany(live.map(stateOf), live.map(a => a.payload)))
  live.forEach((a, k) => {
    const r = res[k]
    if (r instanceof Error && r.code === 'EUNSUPPORTED') {
      // a state outside the snapshot kernel's envelope (sub-documents, repeated client blocks) is answered as the
      // reference does (MessageReceiver.ts:157-179) on the host: the document loaded from the merged state,
      // Y.snapshotContainsUpdate(Y.snapshot(doc), update) (yjs 13.6; with a yjs that lacks it, the same algorithm:
      // snapshotContains above)
      const Y = this._Y()
      const doc = new Y.Doc()
      Y.applyUpdate(doc, stateOf(a))
      const snap = Y.snapshot(doc)
      const yes = typeof Y.snapshotContainsUpdate === 'function' ? Y.snapshotContainsUpdate(snap, a.payload) : snapshotContains(Y, snap, a.payload)
      out[a.i] = syncStatusFrame(a.documentName, yes)
      this.unnormalized.push(a.documentName)
    } else out[a.i] = r instanceof Error ? r : syncStatusFrame(a.documentName, r)
  })
  return out
}

module.exports = { SyncResponder, decodeSyncMessage, frame, syncStatusFrame, snapshotContains, MessageType, SyncStep }
