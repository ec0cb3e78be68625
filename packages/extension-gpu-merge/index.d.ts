// Type declarations for @hocuspocus/extension-gpu-merge (see src/index.js).
import type { Extension, fetchPayload, storePayload, onLoadDocumentPayload, afterLoadDocumentPayload,
  onChangePayload, onStoreDocumentPayload, afterUnloadDocumentPayload } from '@hocuspocus/server'

export declare class YgmError extends Error {
  code: 'EMALFORMED' | 'ERANGE' | 'ENONCANON' | 'ESURROGATE' | 'EDEPTH' | 'ENOMEM' | 'EDEVICE' | 'EINVAL' | string
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
  stats (): Record<string, number>[]
  close (): void
}

/** Batched SyncStep1 -> SyncStep2 responder (SURVEY.md §8f-2; src/sync.js). */
export declare class SyncResponder {
  constructor (opts: { engine: GpuEngine | GpuEnginePool, getState: (documentName: string) => Promise<Uint8Array | Uint8Array[] | null> })
  /** per message: [Step2 reply, server Step1] for SyncStep1, null for other messages, an Error if malformed */
  answerMany (messages: Uint8Array[], opts?: { path?: 'connection' | 'reply' | 'none' }): Promise<(Uint8Array[] | Error | null)[]>
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
}
