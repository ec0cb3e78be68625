'use strict'
// yjs expectation of the doc-normalized snapshot for a file of updates (test tooling):
// exp = Y.encodeStateAsUpdate(Y.applyUpdate(new Y.Doc(), u)) with the image's yjs 13.5.16 bundle.
//   node tools/snap_expect.js in.bin exp.bin      (in: u32 n, (u32 len, bytes)*; exp: (i32 status, u32 len, bytes)*)
// status 1 = yjs threw reading the update.
const fs = require('fs')
const path = require('path')
const Y = require(path.join(__dirname, 'yjs_bundle.js')).load()
const b = fs.readFileSync(process.argv[2])
const n = b.readUInt32LE(0)
let i = 4
const out = []
for (let k = 0; k < n; k++) {
  const len = b.readUInt32LE(i); i += 4
  const u = new Uint8Array(b.buffer, b.byteOffset + i, len); i += len
  let st = 0; let e = new Uint8Array(0)
  try { const d = new Y.Doc(); Y.applyUpdate(d, u); e = Y.encodeStateAsUpdate(d) } catch (err) { st = 1 }
  out.push(Buffer.from(new Int32Array([st]).buffer), Buffer.from(new Uint32Array([e.length]).buffer), Buffer.from(e))
}
fs.writeFileSync(process.argv[3], Buffer.concat(out))
