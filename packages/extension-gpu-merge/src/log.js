'use strict'
/**
 * UpdateLog -- a document's captured updates (every V1 update applied after load, SURVEY.md §8b
 * log-capture hazard 1) kept PACKED as they arrive: one growing byte buffer plus a length per update.
 *
 * The store window (Hocuspocus.ts:417-447) then hands each document to the GPU batch as one contiguous
 * byte range, so building the batch arena costs one copy per document instead of one per update: with
 * 200 updates per document, packing 200 000 small Uint8Arrays at store time cost 30-60 ms of the event
 * loop on Node 12 -- more than the whole reference store (Database.ts:55-60, 47 ms for 1 000 documents).
 * The copy moves to capture time, one update at a time, where it is spread over the editing session.
 */
class UpdateLog {
  constructor () {
    this.buf = Buffer.allocUnsafe(1024)
    this.used = 0
    this.lens = new Uint32Array(64)
    this.n = 0
  }

  get length () { return this.n }

  push (u) {
    const need = this.used + u.length
    if (need > this.buf.length) {
      let cap = this.buf.length * 2
      while (cap < need) cap *= 2
      const b = Buffer.allocUnsafe(cap)
      this.buf.copy(b, 0, 0, this.used)
      this.buf = b
    }
    this.buf.set(u, this.used)
    this.used = need
    if (this.n === this.lens.length) {
      const l = new Uint32Array(this.lens.length * 2)
      l.set(this.lens)
      this.lens = l
    }
    this.lens[this.n++] = u.length
    return this.n
  }

  /** bytes of the first k updates */
  bytes (k = this.n) {
    if (k === this.n) return this.used
    let s = 0
    for (let i = 0; i < k; i++) s += this.lens[i]
    return s
  }

  /** the first k updates as one packed view: { arena: Uint8Array (a view, not a copy), lens: Uint32Array view } */
  packed (k = this.n) {
    return { arena: this.buf.subarray(0, this.bytes(k)), lens: this.lens.subarray(0, k) }
  }

  /** the first k updates as separate Uint8Array views (for callers that take update arrays) */
  toArray (k = this.n) {
    const out = new Array(k)
    let o = 0
    for (let i = 0; i < k; i++) { out[i] = this.buf.subarray(o, o + this.lens[i]); o += this.lens[i] }
    return out
  }

  /** drops the first k updates (those a store has persisted); later ones move to the front */
  drop (k) {
    if (k <= 0) return
    // always a new buffer: views handed out by packed() / toArray() (an in-flight batch, a stored base)
    // keep their bytes, so later pushes never write under them
    if (k >= this.n) { this.buf = Buffer.allocUnsafe(1024); this.used = 0; this.n = 0; return }
    const b = this.bytes(k)
    const nb = Buffer.allocUnsafe(Math.max(1024, this.buf.length))
    this.buf.copy(nb, 0, b, this.used)
    this.buf = nb
    this.used -= b
    this.lens = this.lens.slice(k, Math.max(this.n, 64))
    this.n -= k
  }
}

/** the updates of a packed merge job ({ head, arena, lens }) as one array of Uint8Array views */
function jobUpdates (job) {
  if (Array.isArray(job)) return job
  const out = job.head.slice()
  let o = 0
  for (let i = 0; i < job.lens.length; i++) { out.push(job.arena.subarray(o, o + job.lens[i])); o += job.lens[i] }
  return out
}

module.exports = { UpdateLog, jobUpdates }
