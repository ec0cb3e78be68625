// The reference CPU path for bench.py's cpu_baseline "yjs" leg (BASELINE.md, SURVEY.md §8d): yjs on
// Node worker_threads, one worker per host core granted, each running Y.mergeUpdates /
// Y.diffUpdate / Y.encodeStateVectorFromUpdate per document over a contiguous shard of a corpus
// that bench.py wrote to disk.  Only the op loops are timed: every worker loads its shard, then waits
// at a start barrier (SharedArrayBuffer + Atomics); the job's time is the last worker's end minus the
// common start (process-wide monotonic clock), so workers that the host time-slices are counted in full.
//
//   node tools/yjs_cpu_baseline.js <dir> <op: merge|merge_v2|sv|diff|snapshot> <workers>
//   (merge_v2: Y.mergeUpdatesV2 over update-V2 inputs)
//   (snapshot: Y.encodeStateAsUpdate(Y.applyUpdate(new Y.Doc(), u)), what extension-database stores)
//   <dir>/arena.bin, <dir>/off.bin (u64 update or document offsets), <dir>/docs.bin (u32 update index
//   per document, merge), <dir>/sv.bin + <dir>/svoff.bin (diff)
// Prints one JSON line: {op, docs, workers, seconds, algo_bytes}.
'use strict'
const { Worker, isMainThread, parentPort, workerData } = require('worker_threads')
const fs = require('fs')
const path = require('path')

function u64 (buf) { const a = new BigUint64Array(buf.buffer, buf.byteOffset, buf.length / 8); return Array.from(a, Number) }
function u32 (buf) { return new Uint32Array(buf.buffer, buf.byteOffset, buf.length / 4) }

if (isMainThread) {
  const [dir, op, nw] = process.argv.slice(2)
  const workers = parseInt(nw, 10)
  const docs = op.startsWith('merge') ? u32(fs.readFileSync(path.join(dir, 'docs.bin'))).length - 1 : u64(fs.readFileSync(path.join(dir, 'off.bin'))).length - 1
  const sync = new Int32Array(new SharedArrayBuffer(8))   // [0]: workers loaded, [1]: start flag
  let done = 0; let slowest = 0; let algo = 0; let t0 = null; let t1 = 0n
  for (let w = 0; w < workers; w++) {
    const d0 = Math.floor(docs * w / workers); const d1 = Math.floor(docs * (w + 1) / workers)
    const wk = new Worker(__filename, { workerData: { dir, op, d0, d1, sync } })
    wk.on('message', m => {
      if (m.ready) {
        if (Atomics.add(sync, 0, 1) + 1 === workers) { Atomics.store(sync, 1, 1); Atomics.notify(sync, 1) }
        return
      }
      slowest = Math.max(slowest, m.seconds); algo += m.algo
      const s = BigInt(m.start); const e = BigInt(m.end)
      if (t0 === null || s < t0) t0 = s
      if (e > t1) t1 = e
      if (++done === workers) {
        console.log(JSON.stringify({ op, docs, workers, seconds: Number(t1 - t0) / 1e9, slowest_worker_seconds: slowest, algo_bytes: algo }))
      }
    })
    wk.on('error', e => { console.error(e); process.exit(1) })
  }
} else {
  const Y = require('./yjs_bundle.js').load()
  const { dir, op, d0, d1, sync } = workerData
  const arena = fs.readFileSync(path.join(dir, 'arena.bin'))
  const off = u64(fs.readFileSync(path.join(dir, 'off.bin')))
  const jobs = []
  if (op.startsWith('merge')) {
    const docs = u32(fs.readFileSync(path.join(dir, 'docs.bin')))
    for (let d = d0; d < d1; d++) {
      const us = []
      for (let u = docs[d]; u < docs[d + 1]; u++) us.push(new Uint8Array(arena.buffer, arena.byteOffset + off[u], off[u + 1] - off[u]))
      jobs.push(us)
    }
  } else {
    const sv = op === 'diff' ? fs.readFileSync(path.join(dir, 'sv.bin')) : null
    const svoff = op === 'diff' ? u64(fs.readFileSync(path.join(dir, 'svoff.bin'))) : null
    for (let d = d0; d < d1; d++) {
      const u = new Uint8Array(arena.buffer, arena.byteOffset + off[d], off[d + 1] - off[d])
      jobs.push(op === 'diff' ? [u, new Uint8Array(sv.buffer, sv.byteOffset + svoff[d], svoff[d + 1] - svoff[d])] : u)
    }
  }
  let algo = 0
  parentPort.postMessage({ ready: true })
  Atomics.wait(sync, 1, 0)   // the common start: every worker has loaded its shard
  const t0 = process.hrtime.bigint()
  for (const j of jobs) {
    let out
    if (op.startsWith('merge')) { out = op === 'merge' ? Y.mergeUpdates(j) : Y.mergeUpdatesV2(j); for (const u of j) algo += u.length } else if (op === 'diff') { out = Y.diffUpdate(j[0], j[1]); algo += j[0].length + j[1].length } else if (op === 'snapshot') { const d = new Y.Doc(); Y.applyUpdate(d, j); out = Y.encodeStateAsUpdate(d); algo += j.length } else { out = Y.encodeStateVectorFromUpdate(j); algo += j.length }
    algo += out.length
  }
  const t1 = process.hrtime.bigint()
  parentPort.postMessage({ seconds: Number(t1 - t0) / 1e9, algo, start: t0.toString(), end: t1.toString() })
}
