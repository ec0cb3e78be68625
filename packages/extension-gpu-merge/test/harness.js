'use strict'
// A minimal stand-in for the parts of Hocuspocus's document lifecycle the
// extension hooks into (packages/server/src/Hocuspocus.ts:244-277 handleDocumentUpdate,
// :321-415 loadDocument, :417-447 storeDocumentHooks, :454-487 hooks; util/debounce.ts).
// The real server cannot run in this image (Node 12, no node_modules; SURVEY.md §0-6).
class Mutex {
  constructor () { this.p = Promise.resolve() }
  runExclusive (fn) { const r = this.p.then(fn, fn); this.p = r.catch(() => {}); return r }
}

class MiniHocuspocus {
  constructor ({ extensions, Y, debounce = 30, maxDebounce = 200 }) {
    this.Y = Y
    this.extensions = extensions.slice().sort((a, b) => (b.priority || 100) - (a.priority || 100))
    this.debounce = debounce
    this.maxDebounce = maxDebounce
    this.documents = new Map()
    this.timers = new Map()
    this.stores = 0
  }

  // sequential hook chain; a rejection stops it (Hocuspocus.ts:454-487)
  async hooks (name, payload, callback) {
    for (const ext of this.extensions) {
      if (typeof ext[name] !== 'function') continue
      const r = await ext[name](payload)
      if (callback) callback(r)
    }
  }

  async loadDocument (documentName) {
    const Y = this.Y
    const document = new Y.Doc()
    document.name = documentName
    document.saveMutex = new Mutex()
    const payload = { instance: this, context: {}, document, documentName, socketId: '', requestHeaders: {}, requestParameters: new Map(), connectionConfig: { readOnly: false, isAuthenticated: true } }
    await this.hooks('onLoadDocument', payload, loaded => {
      if (loaded && (loaded.constructor.name === 'Doc' || loaded.constructor.name === 'Document')) Y.applyUpdate(document, Y.encodeStateAsUpdate(loaded))
    })
    await this.hooks('afterLoadDocument', payload)
    document.on('update', (update, origin) => this.handleDocumentUpdate(document, origin, update))
    this.documents.set(documentName, document)
    return document
  }

  handleDocumentUpdate (document, connection, update) {
    const payload = { instance: this, clientsCount: 1, context: {}, document, documentName: document.name, requestHeaders: {}, requestParameters: new Map(), socketId: '', update, transactionOrigin: connection }
    this.hooks('onChange', payload)
    if (!connection || connection === '__hocuspocus__redis__origin__') return
    this.scheduleStore(document, payload)
  }

  scheduleStore (document, payload) {
    const id = document.name
    const t = this.timers.get(id)
    const start = t ? t.start : Date.now()
    if (t) clearTimeout(t.handle)
    const run = () => { this.timers.delete(id); return this.runStore(document, payload) }
    if (Date.now() - start >= this.maxDebounce) { run(); return }
    this.timers.set(id, { start, handle: setTimeout(run, this.debounce), run })
  }

  runStore (document, payload) {
    const p = document.saveMutex.runExclusive(async () => {
      this.stores++
      await this.hooks('onStoreDocument', payload)
      await this.hooks('afterStoreDocument', payload)
    })
    this.lastStore = p
    return p
  }

  // executeNow for every pending debounce (last disconnect / tests)
  async flushAll () {
    const pending = Array.from(this.timers.values())
    this.timers.clear()
    pending.forEach(t => clearTimeout(t.handle))
    await Promise.all(pending.map(t => t.run()))
  }

  async unloadDocument (documentName) {
    this.documents.delete(documentName)
    await this.hooks('afterUnloadDocument', { instance: this, documentName })
  }
}

module.exports = { MiniHocuspocus }
