// Type declarations for @hocuspocus/extension-gpu-merge (see src/index.js).
import type { Extension, fetchPayload, storePayload, onLoadDocumentPayload, afterLoadDocumentPayload,
  onChangePayload, onStoreDocumentPayload, afterUnloadDocumentPayload } from '@hocuspocus/server'

export declare class YgmError extends Error {
  code: 'EMALFORMED' | 'ERANGE' | 'ENONCANON' | 'ESURROGATE' | 'EDEPTH' | 'ENOMEM' | 'EDEVICE' | 'EINVAL' | 'EUNSUPPORTED' | string
  status: number
}

export interface GpuEngineOptions { device?: number; compat135?: boolean; batchWindowMs?: number; maxBatchDocs?: number }

export declare class GpuEngine {
  constructor (opts?: GpuEngineOptions)
  mergeUpdates (updates: Uint8Array[]): Promise<Uint8Array>
  diffUpdate (update: Uint8Array, stateVector: Uint8Array): Promise<Uint8Array>
  encodeStateVectorFromUpdate (update: Uint8Array): Promise<Uint8Array>
  mergeMany (docs: Uint8Array[][]): Promise<(Uint8Array | YgmError)[]>
  diffMany (states: Uint8Array[], svs: Uint8Array[]): Promise<(Uint8Array | YgmError)[]>
  stateVectorsMany (states: Uint8Array[]): Promise<(Uint8Array | YgmError)[]>
  /** update format V2: Y.mergeUpdatesV2 / Y.diffUpdateV2 / Y.encodeStateVectorFromUpdateV2 / Y.convertUpdateFormat* (yjs 13.6) */
  mergeManyV2 (docs: Uint8Array[][]): Promise<(Uint8Array | YgmError)[]>
  diffManyV2 (states: Uint8Array[], stateVectors: Uint8Array[]): Promise<(Uint8Array | YgmError)[]>
  stateVectorsManyV2 (states: Uint8Array[]): Promise<(Uint8Array | YgmError)[]>
  convertManyV1ToV2 (updates: Uint8Array[]): Promise<(Uint8Array | YgmError)[]>
  convertManyV2ToV1 (updates: Uint8Array[]): Promise<(Uint8Array | YgmError)[]>
  /** Y.encodeStateAsUpdate(Y.applyUpdate(new Y.Doc(), update)) (doc-normalized snapshot, SURVEY.md §8f-1) */
  snapshot (update: Uint8Array): Promise<Uint8Array>
  snapshotMany (states: Uint8Array[]): Promise<(Uint8Array | YgmError)[]>
  /** Y.snapshotContainsUpdate(Y.snapshot(doc), update), states being normalized (snapshotMany) states */
  containsMany (states: Uint8Array[], updates: Uint8Array[]): Promise<(boolean | YgmError)[]>
  stats (): Record<string, number>
  close (): void
}

/** FNV-1a 64 of the UTF-8 document name: the device of a document is fnv1a64(name) % devices.length */
export declare function fnv1a64 (name: string): bigint

/** One GpuEngine per device; documents sharded by fnv1a64(documentName) mod N (SURVEY.md §8e). */
export declare class GpuEnginePool {
  constructor (opts?: GpuEngineOptions & { devices?: number[] })
  shardOf (documentName: string): number
  engineFor (documentName: string): GpuEngine
  mergeUpdates (updates: Uint8Array[], documentName?: string): Promise<Uint8Array>
  diffUpdate (update: Uint8Array, stateVector: Uint8Array, documentName?: string): Promise<Uint8Array>
  encodeStateVectorFromUpdate (update: Uint8Array, documentName?: string): Promise<Uint8Array>
  mergeMany (names: string[], docs: Uint8Array[][]): Promise<(Uint8Array | YgmError)[]>
  diffMany (names: string[], states: Uint8Array[], svs: Uint8Array[]): Promise<(Uint8Array | YgmError)[]>
  stateVectorsMany (names: string[], states: Uint8Array[]): Promise<(Uint8Array | YgmError)[]>
  snapshot (update: Uint8Array, documentName?: string): Promise<Uint8Array>
  snapshotMany (names: string[], states: Uint8Array[]): Promise<(Uint8Array | YgmError)[]>
  containsMany (names: string[], states: Uint8Array[], updates: Uint8Array[]): Promise<(boolean | YgmError)[]>
  stats (): Record<string, number>[]
  /** node-wide totals: every per-device counter summed over the pool, plus `devices` */
  statsTotal (): Record<string, number>
  close (): void
}

/** Batched SyncStep1 -> SyncStep2 responder (SURVEY.md §8f-2; src/sync.js). */
export declare class SyncResponder {
  constructor (opts: { engine: GpuEngine | GpuEnginePool, getState: (documentName: string) => Promise<Uint8Array | Uint8Array[] | null> })
  /** per message: [Step2 reply, server Step1] for SyncStep1, null for other messages, an Error if malformed */
  answerMany (messages: Uint8Array[], opts?: { path?: 'connection' | 'reply' | 'none' }): Promise<(Uint8Array[] | Error | null)[]>
  /** read-only connections' SyncStep2 (MessageReceiver.ts:156-179): the SyncStatus(contained) frame per message */
  answerReadOnlyMany (messages: Uint8Array[]): Promise<(Uint8Array | Error | null)[]>
}

/** Batched Redis fan-out (SURVEY.md §8f-3; src/redis.js): extension-redis's per-change Step1 publishes and
 * remote SyncStep1 replies as GPU batches, with the reference's channel names and message framing. */
export declare class RedisFanout {
  constructor (opts: { engine: GpuEngine | GpuEnginePool, getState: (documentName: string) => Promise<Uint8Array | Uint8Array[] | null>,
    publish: (channel: string, message: Buffer) => any, identifier?: string, prefix?: string, windowMs?: number })
  identifier: string
  redisTransactionOrigin: string
  onChange (data: { documentName: string, transactionOrigin?: any }): Promise<void>
  /** null for own messages; answers SyncStep1 (replies published); otherwise the message for the host to apply */
  handleIncomingMessage (channel: string | Buffer, data: Buffer): Promise<null | { documentName: string | null, message?: Buffer, replied?: number }>
}

export declare class DocumentStore {
  fetchMany (payloads: fetchPayload[]): Promise<(Uint8Array | Uint8Array[] | null)[]>
  storeMany (entries: { payload: onStoreDocumentPayload; state: Buffer }[]): Promise<void>
  static fromDatabase (config: { fetch?: (p: fetchPayload) => Promise<Uint8Array | Uint8Array[] | null>; store?: (p: storePayload) => Promise<void> }): DocumentStore
}

export interface GpuMergeConfiguration extends GpuEngineOptions {
  /** several GPUs: documents sharded by fnv1a64(documentName) mod devices.length */
  devices?: number[]
  /** a batched DocumentStore, or the DatabaseConfiguration.store function (Database.ts:19) */
  store?: DocumentStore | ((p: storePayload) => Promise<void>)
  fetch?: (p: fetchPayload) => Promise<Uint8Array | Uint8Array[] | null>
  priority?: number
  engine?: GpuEngine
  Y?: any
  /** a refused merge: store Y.encodeStateAsUpdate(document) ('reference', default) or reject the store ('throw') */
  onRefused?: 'reference' | 'throw'
  /** store the GPU doc-normalized snapshot of the merge (GC'd, merged: the shape extension-database stores); default true, false stores the bare merge */
  normalize?: boolean
  /** merged states over this many bytes are stored as the bare merge (the snapshot kernel runs one thread per document); default 32768 */
  normalizeMaxBytes?: number
}

export declare class GpuMerge implements Extension {
  extensionName: string
  priority: number
  constructor (configuration?: GpuMergeConfiguration)
  onConfigure (): Promise<void>
  onLoadDocument (data: onLoadDocumentPayload): Promise<void>
  afterLoadDocument (data: afterLoadDocumentPayload): Promise<void>
  onChange (data: onChangePayload): Promise<void>
  onStoreDocument (data: onStoreDocumentPayload): Promise<void>
  afterUnloadDocument (data: afterUnloadDocumentPayload): Promise<void>
  onDestroy (): Promise<void>
  /** batched SyncStep1 responder over the captured state (snapshot + updates since) */
  syncResponder (): SyncResponder
  /** batched extension-redis fan-out over the same captured state */
  redisFanout (opts: { publish: (channel: string, message: Buffer) => any, identifier?: string, prefix?: string, windowMs?: number, onError?: (e: Error) => void }): RedisFanout
}
