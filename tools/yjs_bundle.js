// Loads the yjs 13.5.16 / lib0 0.2.42 copy that JupyterLab bundles in this image
// (/opt/conda/share/jupyter/lab/static) where it lies -- the reference yjs CPU path for bench.py's
// cpu_baseline "yjs" leg.  Nothing of the bundle is copied into the repository: this is a small
// webpack-chunk runtime that evaluates the bundle's own chunks.
'use strict'
const path = require('path')

const STATIC = process.env.YJS_BUNDLE_DIR || '/opt/conda/share/jupyter/lab/static'
const CHUNKS = ['3502.fbe0c610be82ba1360db.js', '8086.1dfabaac37d971e2cc4c.js', '1057.1a1aee857cdaddbae1d3.js']
const YJS_MODULE_ID = 73502

let cached = null
function load () {
  if (cached) return cached   // one evaluation per process (a second one finds the chunk registry consumed)
  const modules = {}
  global.self = global
  global.window = undefined
  global.crypto = { getRandomValues: a => require('crypto').randomFillSync(a) }
  global.self.webpackChunk_jupyterlab_application_top = { push: ([, mods]) => Object.assign(modules, mods) }
  for (const f of CHUNKS) require(path.join(STATIC, f))
  const cache = {}
  function req (id) {
    if (cache[id]) return cache[id].exports
    const m = cache[id] = { exports: {} }
    modules[id].call(m.exports, m, m.exports, req)
    return m.exports
  }
  req.r = e => Object.defineProperty(e, '__esModule', { value: true })
  req.d = (e, d) => { for (const k in d) if (!Object.prototype.hasOwnProperty.call(e, k)) Object.defineProperty(e, k, { enumerable: true, get: d[k] }) }
  req.n = m => { const g = m && m.__esModule ? () => m.default : () => m; req.d(g, { a: g }); return g }
  req.o = (o, p) => Object.prototype.hasOwnProperty.call(o, p)
  req.g = global
  cached = req(YJS_MODULE_ID)
  return cached
}

module.exports = { load, STATIC, present: () => require('fs').existsSync(path.join(STATIC, CHUNKS[0])) }
