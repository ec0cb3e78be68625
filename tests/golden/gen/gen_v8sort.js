// Test-fixture tooling: records how V8's Array.prototype.sort (TimSort, the
// algorithm mergeUpdates' per-iteration decoder re-sort runs on, Y@39011)
// orders arrays under INCONSISTENT comparators (yjs's comparator returns -1
// both ways for GC-vs-Item ties, SURVEY.md App. B.5).  Each case: n, a
// comparator T(a,b) = key order, ties -> 0 if same kind else -1 (both ways),
// then `noise` overrides [a,b,v]; plus the permutation V8 produced.
'use strict'
const fs = require('fs'); const zlib = require('zlib'); const path = require('path')
function mulberry32 (a) { return function () { a |= 0; a = a + 0x6D2B79F5 | 0; let t = Math.imul(a ^ a >>> 15, 1 | a); t = t + Math.imul(t ^ t >>> 7, 61 | t) ^ t; return ((t ^ t >>> 14) >>> 0) / 4294967296 } }
const rnd = mulberry32(7); const ri = n => Math.floor(rnd() * n)
const cases = []
const sizes = [2, 3, 5, 8, 13, 22, 40, 63, 64, 65, 100, 130, 200, 260, 600]
for (let rep = 0; rep < 40; rep++) {
  for (const n of sizes) {
    // mostly-consistent key order with random inconsistent pairs (like equal-key GC/Item ties)
    const key = []; for (let i = 0; i < n; i++) key.push(ri(rep % 3 === 0 ? 4 : n))
    const kind = []; for (let i = 0; i < n; i++) kind.push(ri(2))
    const T = new Int8Array(n * n)
    for (let a = 0; a < n; a++) for (let b = 0; b < n; b++) {
      if (key[a] !== key[b]) T[a * n + b] = key[a] < key[b] ? -1 : 1
      else T[a * n + b] = kind[a] === kind[b] ? 0 : -1 // inconsistent tie
    }
    const noise = []
    if (rep % 5 === 4) for (let q = 0; q < n; q++) { const a = ri(n); const b = ri(n); const v = ri(3) - 1; T[a * n + b] = v; noise.push([a, b, v]) } // noise
    const arr = []; for (let i = 0; i < n; i++) arr.push(i)
    // a pre-ordered start (like the previous iteration's order) half of the time
    if (rep % 2 === 0) arr.sort((a, b) => key[a] - key[b] || a - b)
    const input = arr.slice()
    let calls = 0
    arr.sort((a, b) => { calls++; return T[a * n + b] })
    cases.push({ n, key, kind, noise, input, out: arr, calls })
  }
}
const out = path.join(__dirname, '..', 'v8_timsort_vectors.json.gz')
fs.writeFileSync(out, zlib.gzipSync(JSON.stringify({ node: process.version, v8: process.versions.v8, cases }), { level: 9 }))
console.log('wrote', cases.length, 'cases to', out, 'v8', process.versions.v8)
