/*
 * crdtenc.h -- C ABI of the MI355X-native crdt-enc compaction/ingest hot path.
 *
 * Every entry point replaces one reference interface (Rust, chpio/crdt-enc @ /root/reference):
 *   Cryptor  trait   crdt-enc/src/cryptor.rs:11-27         -> ce_cryptor_*
 *            impl    crdt-enc-xchacha20poly1305/src/lib.rs:28-101 (EncHandler)
 *   Storage  trait   crdt-enc/src/storage.rs:8-43          -> ce_storage_*
 *            impl    crdt-enc-tokio/src/lib.rs:48-316       (local-dir layout)
 *   Core     API     crdt-enc/src/lib.rs:226 open, :332 compact, :390 read_remote,
 *                    :666 apply_ops, :325 with_state        -> ce_core_*
 * INTEGRATION.md shows the Rust FFI binding a maintainer would add on the reference side.
 *
 * Conventions: plain pointers and sizes; no torch/HIP types.  Functions return a ce_status
 * (0 = CE_OK).  Buffers returned in a ce_buf are owned by the caller and released with
 * ce_buf_free.  All entry points are thread-safe per ce_ctx (internally serialized; the
 * reference issues <= 16 concurrent decrypts, crdt-enc/src/lib.rs:452,512).
 */
#ifndef CRDTENC_H
#define CRDTENC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Per-file / per-call status, numbered in the reference's check order. */
enum ce_status {
  CE_OK = 0,
  CE_ERR_OUTER_LEN = 1,     /* VersionBytes::deserialize InvalidLength (version_bytes.rs:187)  */
  CE_ERR_OUTER_VERSION = 2, /* ensure_versions_phf(SUPPORTED_VERSIONS) (lib.rs:435,501)        */
  CE_ERR_KEY_VERSION = 3,   /* "not matching key version" (xchacha lib.rs:74-75)               */
  CE_ERR_KEY_LEN = 4,       /* "Invalid key length" (xchacha lib.rs:76-78)                     */
  CE_ERR_PARSE_VBOX = 5,    /* "failed to parse version box" (xchacha lib.rs:82-83)            */
  CE_ERR_DATA_VERSION = 6,  /* "not matching version of encryption box" (xchacha lib.rs:84-86) */
  CE_ERR_PARSE_ENCBOX = 7,  /* "failed to parse encryption box" (xchacha lib.rs:87-88)         */
  CE_ERR_NONCE_LEN = 8,     /* "Invalid nonce length" (xchacha lib.rs:89-91)                   */
  CE_ERR_AUTH = 9,          /* "Decryption failed" (xchacha lib.rs:92-97)                      */
  CE_ERR_PT_LEN = 10,       /* clear text VersionBytesRef::deserialize (lib.rs:443,504)        */
  CE_ERR_PT_VERSION = 11,   /* ensure_versions(supported_data_versions) (lib.rs:444,505)       */
  CE_ERR_DECODE = 12,       /* rmp_serde::from_slice of ops / StateWrapper (lib.rs:447,507)    */
  CE_ERR_OP_VERSION = 13,   /* "Unexpected op version" (lib.rs:527-531)                        */
  CE_ERR_INVALID_ARG = 64,
  CE_ERR_DEVICE = 65,       /* HIP runtime failure / no GPU: the product has no CPU path       */
  CE_ERR_NO_KEY = 66,       /* "no latest key" (lib.rs:420,490)                                */
  CE_ERR_IO = 67,
  CE_ERR_NO_LOCAL_META = 68, /* "local meta does not exist, and `create` option is not set"    */
  CE_ERR_SHARD = 69          /* sharded ingest: a rank's batch breaks the partition contract (the
                                windows must come from ce_shard_window_exact) or the ranks'
                                next_op_versions differ                                        */
};

typedef struct ce_buf {
  uint8_t *data;
  size_t len;
} ce_buf;

void ce_buf_free(ce_buf *b);
const char *ce_status_str(int status);

/* ---------------------------------------------------------------------------------------- */
/* Context: one per GPU (one process per GPU).                                               */
/* ---------------------------------------------------------------------------------------- */
typedef struct ce_ctx ce_ctx;

int ce_ctx_create(int device, ce_ctx **out);
void ce_ctx_destroy(ce_ctx *ctx);
/* Use an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL = own. */
int ce_ctx_set_stream(ce_ctx *ctx, void *hip_stream);
void ce_ctx_synchronize(ce_ctx *ctx);
/* Human readable detail of the last failure on this context. */
const char *ce_ctx_last_error(ce_ctx *ctx);
/* Kernel timing with HIP events recorded on the context stream around every launch (off by
 * default).  ce_ctx_timing_read synchronizes and returns the summed milliseconds and launch
 * count of one kernel ("open_setup", "segments_open", "finalize_open", "decode", "merge",
 * "seal_setup", "segments_seal", "finalize_seal"). */
int ce_ctx_set_timing(ce_ctx *ctx, int enable);
/* Restrict the timing to one kernel name (NULL = every launch): each timed launch adds two
 * event markers to the stream, so a timed step measures only the kernel it reports. */
int ce_ctx_set_timing_only(ce_ctx *ctx, const char *kernel);
int ce_ctx_timing_read(ce_ctx *ctx, const char *kernel, double *total_ms, uint64_t *launches);
void ce_ctx_timing_reset(ce_ctx *ctx);
/* Diagnostics (no reference counterpart): the shader clock while other work runs.  Launches
 * `blocks` one-wave blocks on hip_stream (NULL = the context stream); each reads the shader
 * cycle counter against the 100 MHz reference clock every `ticks` reference ticks, `samples`
 * times, and writes (cycles, ticks) of every interval to d_out (device memory, blocks * samples
 * * 2 uint64).  Asynchronous; at most 4096 blocks, samples * ticks <= 10^8 (1 s). */
int ce_ctx_clock_probe(ce_ctx *ctx, void *hip_stream, uint64_t *d_out, uint32_t blocks,
                       uint32_t samples, uint32_t ticks);

/* ---------------------------------------------------------------------------------------- */
/* Cryptor: XChaCha20-Poly1305 EncHandler on the GPU                                          */
/*   (trait crdt-enc/src/cryptor.rs:11-27; impl crdt-enc-xchacha20poly1305/src/lib.rs:28-101) */
/* ---------------------------------------------------------------------------------------- */
/* Cryptor::gen_key (xchacha lib.rs:29-38): out = VersionBytes(KEY_VERSION, 32 random bytes)
 * in the raw framing (16-byte version || 32-byte key; version_bytes.rs:198-208). */
int ce_cryptor_gen_key(ce_ctx *ctx, ce_buf *out);

/* Cryptor::encrypt (xchacha lib.rs:40-71): out = msgpack(VersionBytesRef(DATA_VERSION,
 * msgpack(EncBox{nonce, enc_data}))).  nonce: 24 bytes, or NULL to draw from the OS RNG
 * (the reference uses rand::rng(), lib.rs:51-54). */
int ce_cryptor_encrypt(ce_ctx *ctx, const uint8_t key_version[16], const uint8_t *key,
                       size_t key_len, const uint8_t *nonce, const uint8_t *clear,
                       size_t clear_len, ce_buf *out);

/* Cryptor::decrypt (xchacha lib.rs:73-101): enc = VersionBytes content (the outer 16-byte
 * version already stripped by the caller, lib.rs:502).  No plaintext is returned for a file
 * whose tag fails. */
int ce_cryptor_decrypt(ce_ctx *ctx, const uint8_t key_version[16], const uint8_t *key,
                       size_t key_len, const uint8_t *enc, size_t enc_len, ce_buf *out);

/* Length of Cryptor::encrypt's output for a clear text of clear_len bytes. */
size_t ce_cryptor_sealed_len(size_t clear_len);

/* Batched Cryptor::decrypt over host buffers: input i = blob[offs[i], offs[i+1]).
 * out_blob must hold offs[n] + 16*n bytes; plaintext i is written at out_offs[i] with length
 * out_lens[i] (both outputs, n entries).  status[i] receives the per-file status; the call
 * returns CE_OK when every file opened, else the status of the lowest failing index.  A file
 * whose tag fails has its output region zeroed (verify-before-release). */
int ce_cryptor_decrypt_batch(ce_ctx *ctx, const uint8_t key_version[16], const uint8_t *key,
                             size_t key_len, const uint8_t *blob, const uint64_t *offs,
                             uint32_t n, uint8_t *out_blob, uint64_t *out_offs,
                             uint64_t *out_lens, int32_t *status);

/* Batched Cryptor::encrypt: clear text i = blob[offs[i], offs[i+1]); nonces = n*24 bytes or
 * NULL (OS RNG).  Output i is written at out_offs[i] (n+1 entries, computed by the call; size
 * out_offs[n] = sum of ce_cryptor_sealed_len) into out_blob (capacity out_cap). */
int ce_cryptor_encrypt_batch(ce_ctx *ctx, const uint8_t key_version[16], const uint8_t *key,
                             size_t key_len, const uint8_t *blob, const uint64_t *offs,
                             uint32_t n, const uint8_t *nonces, uint8_t *out_blob,
                             size_t out_cap, uint64_t *out_offs);

/* Device-resident variants: every pointer is a device pointer (hipMalloc / torch tensor);
 * the work is enqueued on the context stream and the call returns after enqueueing unless
 * noted.  d_offs has n+1 entries.  d_out must hold offs[n] + 16*n + 64 bytes; plaintext i
 * lands at align16(offs[i]) (see DESIGN.md "HBM layout").  d_status may be NULL. */
int ce_cryptor_decrypt_batch_device(ce_ctx *ctx, const uint8_t key_version[16],
                                    const uint8_t *key, size_t key_len, const uint8_t *d_blob,
                                    const uint64_t *d_offs, uint32_t n, uint8_t *d_out,
                                    int32_t *d_status, uint32_t *n_failed);
/* Seal n clear texts of d_clear[d_offs[i], d_offs[i+1]) into op files
 * CURRENT_VERSION || Cryptor::encrypt(...) at d_out[d_out_offs[i], ...).  d_nonces = n*24
 * device bytes.  outer_version: 16 bytes or NULL (no outer prefix). */
int ce_cryptor_encrypt_batch_device(ce_ctx *ctx, const uint8_t key_version[16],
                                    const uint8_t *key, size_t key_len,
                                    const uint8_t *outer_version, const uint8_t *d_clear,
                                    const uint64_t *d_offs, uint32_t n, const uint8_t *d_nonces,
                                    uint8_t *d_out, const uint64_t *d_out_offs);

/* ---------------------------------------------------------------------------------------- */
/* Storage: crdt-enc-tokio local-dir layout (crdt-enc-tokio/src/lib.rs)                        */
/*   local/meta-data.msgpack, remote/{meta,states}/<BASE32_NOPAD(SHA3-256)>,                   */
/*   remote/ops/<uuid>/<version>                                                              */
/* ---------------------------------------------------------------------------------------- */
typedef struct ce_storage ce_storage;

/* Storage::new (tokio lib.rs:29-45): both paths must be absolute. */
int ce_storage_open(const char *local_path, const char *remote_path, ce_storage **out);
void ce_storage_close(ce_storage *s);
/* list_op_actors (tokio lib.rs:204-220): out = m*16 bytes of actor UUIDs */
int ce_storage_list_op_actors(ce_storage *s, ce_buf *out);
/* load_ops (tokio lib.rs:222-278): for each (actor, first) read ops/<actor>/<v> for
 * v = first.. until the first missing file.  Outputs (caller frees with ce_buf_free):
 * blob = concatenated files, offs = (k+1) u64, actor_idx = k u32 (index into actors),
 * versions = k u64. */
int ce_storage_load_ops(ce_storage *s, const uint8_t *actors, const uint64_t *first, uint32_t m,
                        ce_buf *blob, ce_buf *offs, ce_buf *actor_idx, ce_buf *versions);
/* store_ops (tokio lib.rs:280-293): create-new + fsync */
int ce_storage_store_ops(ce_storage *s, const uint8_t actor[16], uint64_t version,
                         const uint8_t *data, size_t len);
/* remove_ops (tokio lib.rs:295-315): NotFound is not an error */
int ce_storage_remove_ops(ce_storage *s, const uint8_t *actors, const uint64_t *versions,
                          uint32_t m);
/* list_state_names (tokio lib.rs:138-153): out = NUL-separated names */
int ce_storage_list_state_names(ce_storage *s, ce_buf *out);
/* store_state (tokio lib.rs:174-179): name = BASE32_NOPAD(SHA3-256(bytes)), 52 chars + NUL */
int ce_storage_store_state(ce_storage *s, const uint8_t *data, size_t len, char name_out[64]);
int ce_storage_load_state(ce_storage *s, const char *name, ce_buf *out);
int ce_storage_remove_state(ce_storage *s, const char *name);
/* content address of a blob: BASE32_NOPAD(SHA3-256(data)) (tokio lib.rs:403-417) */
int ce_content_name(const uint8_t *data, size_t len, char name_out[64]);
/* the same name computed on the library's own host thread (store_state's hash off the caller's
   thread, e.g. while the next compaction runs): *ticket identifies the job; data must stay valid
   until ce_content_name_wait(ticket) returns.  Jobs run in submission order; a ticket is waited
   once. */
int ce_content_name_async(const uint8_t *data, size_t len, uint64_t *ticket);
/* ce_content_name of n buffers at once: eight SHA3-256 sponges per AVX-512 core step (the
 * pipelined compactions' names, crdt-enc-tokio/src/lib.rs:403-432); names_out[i] as
 * ce_content_name's.  Same result as n ce_content_name calls. */
int ce_content_names(const uint8_t *const *data, const size_t *lens, uint32_t n, char (*names_out)[64]);
int ce_content_name_wait(uint64_t ticket, char name_out[64]);

/* ---------------------------------------------------------------------------------------- */
/* Core (crdt-enc/src/lib.rs)                                                                */
/* ---------------------------------------------------------------------------------------- */
typedef struct ce_core ce_core;

/* StateWrapper<S> state type S (crdts 7 types; Orswot and MVReg over u64 members / values) */
enum ce_state_kind {
  CE_STATE_VCLOCK = 0,   /* VClock<Uuid>                                                      */
  CE_STATE_GCOUNTER = 1, /* GCounter<Uuid>                                                    */
  CE_STATE_ORSWOT = 2,   /* Orswot<u64, Uuid>: op = orswot::Op {Add{dot, members}, Rm{clock,
                            members}}; entries/deferred serialized in canonical order (members
                            ascending, deferred clocks by their msgpack bytes): the reference's
                            HashMap order is random                           */
  CE_STATE_MVREG = 3     /* MVReg<u64, Uuid>: op = mvreg::Op::Put{clock, val}                 */
};

enum ce_open_flags {
  CE_OPEN_CREATE = 1,            /* OpenOptions.create (lib.rs:729)                          */
  CE_COMPACT_INGEST_FORMAT = 2,  /* write compacted states in the format read_remote_states
                                    reads (outer CURRENT_VERSION + inner data-version prefix)
                                    instead of the reference's compact() bytes   */
  CE_OPEN_MULTI_KEY = 4          /* beyond the reference (opt-in): files that fail
                                    authentication under the latest key are opened again under
                                    the other keys of the set given to ce_core_set_keys, in id
                                    order; the batch is rejected only if some file opens under
                                    none.  Off, every file must open under Keys::latest_key, as
                                    the reference requires (lib.rs:414-420,484-490) */
};

typedef struct ce_open_options {
  int state_kind;                        /* ce_state_kind                                  */
  const uint8_t *supported_data_versions; /* n_supported * 16 bytes (lib.rs:730)             */
  size_t n_supported;
  const uint8_t *current_data_version;   /* 16 bytes (lib.rs:731)                          */
  const char *local_path;                /* NULL: no storage (ingest API only)             */
  const char *remote_path;
  uint32_t flags;                        /* ce_open_flags                                  */
} ce_open_options;

/* Core::open (lib.rs:226-311) minus the key-cryptor handshake: the latest data key is
 * supplied with ce_core_set_latest_key (Keys::latest_key, key_cryptor.rs:59-70). */
int ce_core_open(ce_ctx *ctx, const ce_open_options *opts, ce_core **out);
void ce_core_close(ce_core *c);
int ce_core_set_latest_key(ce_core *c, const uint8_t key_version[16], const uint8_t *key,
                           size_t key_len);
/* Core::info().actor() (lib.rs:313-322) */
int ce_core_info_actor(ce_core *c, uint8_t out[16]);
/* Core::read_remote (lib.rs:390-399): read_remote_states then read_remote_ops via Storage */
int ce_core_read_remote(ce_core *c);
/* Core::compact (lib.rs:332-380).  name_out (may be NULL) receives the new state's name. */
int ce_core_compact(ce_core *c, char name_out[64]);
/* Core::apply_ops (lib.rs:666-722): ops = rmp-serde msgpack of Vec<S::Op> (Vec<Dot<Uuid>>). */
int ce_core_apply_ops(ce_core *c, const uint8_t *ops, size_t len);
/* n successive Core::apply_ops calls (lib.rs:666-722) as one batch: ops i =
 * ops[offs[i], offs[i+1]) (offs: n+1 entries); every clear text sealed by one GPU launch; file i
 * stored (with storage) as ops/<local actor>/<next_op_versions.get(actor) + i>; the ops applied
 * in order; next_op_versions bumped by n.  All n ops blobs are decoded before anything is sealed
 * or written.  nonces: n*24 bytes or NULL (OS RNG).  files / file_offs (may be NULL) receive
 * the op files back to back and their n+1 u64 offsets (what Storage::store_ops got). */
int ce_core_apply_ops_batch(ce_core *c, const uint8_t *ops, const uint64_t *offs, uint32_t n,
                            const uint8_t *nonces, ce_buf *files, ce_buf *file_offs);
/* rmp_serde::to_vec_named(&StateWrapper) (lib.rs:336, 739-743) */
int ce_core_state_bytes(ce_core *c, ce_buf *out);
/* Back to the empty StateWrapper (Default, lib.rs:240-243), keeping registered actors and the
 * read key; used to compact the same batch repeatedly in benchmarks. */
int ce_core_reset(ce_core *c);
/* Wait for the core's queued device work and return its deferred status: CE_OK, or the error a
 * fold / merge that already returned CE_OK found on the device (a dot-set table overflow).  Such
 * an error is sticky: every later call fails with it until ce_core_reset.  Callers that must act
 * on an ingest's exact status before the next call (the sharded ingest's all_reduce of statuses)
 * settle first.  No reference counterpart: the reference's apply loop is synchronous
 * (crdt-enc/src/lib.rs:533-535). */
int ce_core_settle(ce_core *c);

/* Storage-less ingest: what read_remote_ops does after Storage::load_ops (lib.rs:495-546).
 * files i = blob[offs[i], offs[i+1]) (outer version || cryptor box); the writer of file i is
 * actors[file_actor[i]] (m actors, 16 bytes each) with version file_version[i].  status may
 * be NULL.  Returns CE_OK, the lowest failing file's status (nothing folded), or
 * CE_ERR_OP_VERSION (fold stopped at the gap, as the reference's loop). */
int ce_core_ingest_ops(ce_core *c, const uint8_t *blob, const uint64_t *offs, uint32_t n,
                       const uint8_t *actors, uint32_t m, const uint32_t *file_actor,
                       const uint64_t *file_version, int32_t *status);
/* Same with the batch resident in HBM: d_blob/d_offs (n+1 entries, blob_len = offs[n]) and
 * the per-file metadata d_file_actor (u32) / d_file_version (u64) are device pointers; the m
 * writer actors (16 bytes each) and status (may be NULL) are host memory.  Batches in
 * Storage::load_ops order (each actor's files contiguous with consecutive versions) are gated
 * on the GPU; any other order is gated on the host with identical results. */
int ce_core_ingest_ops_device(ce_core *c, const uint8_t *d_blob, const uint64_t *d_offs,
                              uint32_t n, uint64_t blob_len, const uint8_t *actors, uint32_t m,
                              const uint32_t *d_file_actor, const uint64_t *d_file_version,
                              int32_t *status);
/* The same from the per-file host buffers Storage::load_ops returns (one Vec<u8> per file,
 * crdt-enc-tokio/src/lib.rs:222-278): files[i] holds lens[i] bytes.  The files are gathered
 * into pinned staging chunks by host threads and DMA'd while the next chunk fills; no
 * concatenated copy is needed on the caller's side. */
int ce_core_ingest_ops_iov(ce_core *c, const uint8_t *const *files, const size_t *lens, uint32_t n,
                           const uint8_t *actors, uint32_t m, const uint32_t *file_actor,
                           const uint64_t *file_version, int32_t *status);
/* What read_remote_states does after Storage::load_states (lib.rs:425-466). */
int ce_core_ingest_states(ce_core *c, const uint8_t *blob, const uint64_t *offs, uint32_t n,
                          int32_t *status);
/* ce_core_ingest_states over per-file host buffers (what Storage::load_states returns as
 * Vec<u8>s, crdt-enc/src/lib.rs:425-431): files[i] holds lens[i] bytes, uploaded through the
 * pinned staging ring (no concatenated copy). */
int ce_core_ingest_states_iov(ce_core *c, const uint8_t *const *files, const size_t *lens, uint32_t n,
                              int32_t *status);
/* The same with the state files resident in HBM: d_blob / d_offs (n + 1 entries, blob_len =
 * offs[n]) are device pointers (file i = CURRENT_VERSION || cryptor box, as load_states returns
 * it); status (may be NULL) is host memory. */
int ce_core_ingest_states_device(ce_core *c, const uint8_t *d_blob, const uint64_t *d_offs, uint32_t n,
                                 uint64_t blob_len, int32_t *status);
/* Core::compact (crdt-enc/src/lib.rs:332-380) over a batch resident in HBM: read_remote_ops over
 * the op files exactly as ce_core_ingest_ops_device, then the compaction output as
 * ce_core_compact_to_buffer.  For VClock/GCounter the compaction is queued on the device behind
 * the ingest's commit (one host synchronisation for both).  A read_remote error is returned
 * before anything is written (file untouched).  nonce: 24 bytes or NULL; name_out may be NULL. */
int ce_core_compact_ops_device(ce_core *c, const uint8_t *d_blob, const uint64_t *d_offs, uint32_t n,
                               uint64_t blob_len, const uint8_t *actors, uint32_t m,
                               const uint32_t *d_file_actor, const uint64_t *d_file_version,
                               const uint8_t *nonce, ce_buf *file, char name_out[64]);
/* ce_core_compact_ops_device into a caller-owned buffer (pinned host memory: the sealed file is
 * downloaded straight into it, no intermediate copy): *len = the file size.  cap should be at
 * least 16 + ce_cryptor_sealed_len(bound of the serialized state); when the file does not fit
 * CE_ERR_INVALID_ARG is returned with *len set (the state is then already folded: call
 * ce_core_compact_into for the file).  On an error dst's contents are unspecified. */
int ce_core_compact_ops_device_into(ce_core *c, const uint8_t *d_blob, const uint64_t *d_offs,
                                    uint32_t n, uint64_t blob_len, const uint8_t *actors, uint32_t m,
                                    const uint32_t *d_file_actor, const uint64_t *d_file_version,
                                    const uint8_t *nonce, uint8_t *dst, size_t cap, size_t *len,
                                    char name_out[64]);
/* ce_core_compact_ops_device over per-file host buffers (upload as ce_core_ingest_ops_iov,
 * then the device path; file_actor / file_version are host arrays). */
int ce_core_compact_ops_iov(ce_core *c, const uint8_t *const *files, const size_t *lens, uint32_t n,
                            const uint8_t *actors, uint32_t m, const uint32_t *file_actor,
                            const uint64_t *file_version, const uint8_t *nonce, ce_buf *file,
                            char name_out[64]);
/* compact() without storage: serialize the state, seal it on the GPU with the latest key and
 * return the state file bytes and its content name.  nonce: 24 bytes or NULL (OS RNG). */
int ce_core_compact_to_buffer(ce_core *c, const uint8_t *nonce, ce_buf *file, char name_out[64]);
/* The same into a caller-owned buffer (no per-call allocation): *len = the file size.  When
 * cap < *len nothing is written and CE_ERR_INVALID_ARG is returned with *len set, so the caller
 * can grow its buffer and call again (the state is unchanged; the nonce is drawn again). */
int ce_core_compact_into(ce_core *c, const uint8_t *nonce, uint8_t *dst, size_t cap, size_t *len,
                         char name_out[64]);

/* ce_core_compact_into with the sealed file's download left in flight (pipelined
 * compactions: the download overlaps the caller's next batch on the device, and the call returns
 * without waiting for the device at all).  *ticket = 0 when the file is already complete in dst
 * (*len = its length), else *len = 0 and ce_core_compact_wait(ticket, &len) gives the length once
 * the file is in dst (dst must stay allocated until then; a dst the device cannot write -- not
 * pinned -- takes the synchronous path, ticket 0).  Returns the same statuses as
 * ce_core_compact_into; a dst too small for the file is reported by ce_core_compact_wait
 * (CE_ERR_INVALID_ARG).  A ticket stays valid for the next 15 compactions of the core. */
int ce_core_compact_into_async(ce_core *c, const uint8_t *nonce, uint8_t *dst, size_t cap, size_t *len,
                               uint64_t *ticket);
int ce_core_compact_wait(ce_core *c, uint64_t ticket, uint64_t *len);

/* Pinned host memory for the asynchronous paths (ce_core_compact_into_async's dst, the *_iov
 * host-buffer ingests): the device's DMA engines copy it without staging and without occupying
 * the compute units.  NULL when the allocation fails.  (No reference counterpart: the Rust
 * caller's Vec<u8> buffers, lib.rs:349-363, would be allocated here for the zero-copy form.) */
void *ce_host_alloc(size_t bytes);
void ce_host_free(void *p);

/* What read_remote_states does with one decrypted state (lib.rs:447, 458-466):
 * rmp_serde::from_slice::<StateWrapper<S>>(sw) then state.merge + next_op_versions.merge.
 * Also the exchange step of the dot-set kinds across GPUs (all-gather of partial states). */
int ce_core_merge_state(ce_core *c, const uint8_t *sw, size_t len);
/* The multi-GPU dot-set exchange without a host hop (read_remote_states' merge, lib.rs:446-466,
 * with the partial state travelling GPU to GPU over RCCL): ce_core_state_bytes written into
 * device memory d_dst (cap bytes; *len = its length; CE_ERR_INVALID_ARG, nothing written, when
 * cap < *len -- grow and call again), and ce_core_merge_state of a StateWrapper resident in HBM
 * (d_sw, len bytes).  Orswot states are written and read by the device serializer / state
 * reader (only the head and the deferred tail reach the host); the small VClock, GCounter and
 * MVReg states are serialized / parsed on the host and copied. */
int ce_core_state_bytes_device(ce_core *c, uint8_t *d_dst, uint64_t cap, uint64_t *len);
int ce_core_merge_state_device(ce_core *c, const uint8_t *d_sw, uint64_t len);

/* The multi-GPU dot-set exchange as columns: an Orswot's live (member, actor, counter) pairs, its
 * clock, next_op_versions and actor UUIDs written into device memory d_dst (cap bytes) -- no
 * msgpack, no parse on the receiving side -- and, when the state holds deferred removals, its
 * deferred map as a final section of CSR arrays (removal clocks by the partial's actor index and
 * their members; format in INTEGRATION.md).  *len = the bytes written, or needed when cap is too
 * small (CE_ERR_INVALID_ARG).  Another kind than Orswot has no column form: CE_ERR_INVALID_ARG
 * with *len = 0, and the caller exchanges ce_core_state_bytes_device instead.
 * d_dst NULL with cap 0 is a query: CE_ERR_INVALID_ARG with *len = 1 when the state has a column
 * form, 0 when not (nothing is collected).
 * Complete on return.  Replaces, for the exchange only, the serialize -> parse round trip of
 * read_remote_states' merge (crdt-enc/src/lib.rs:458-466). */
int ce_core_export_columns_device(ce_core *c, uint8_t *d_dst, uint64_t cap, uint64_t *len);
/* Merge k <= 64 column partials (device pointers d_parts[i], lens[i] bytes) into the state at once:
 * Orswot::merge of every part, deferred removals on either side included (the same result as
 * merging their StateWrappers one by one, in any order), next_op_versions max-merged.  Complete
 * on return (the parts may be reused).  CE_ERR_DECODE when a part is not a column partial or its
 * deferred section is malformed (checked on the device before this state is touched). */
int ce_core_merge_columns_device(ce_core *c, const uint8_t *const *d_parts, const uint64_t *lens, uint32_t k);

/* Dense state exchange for multi-GPU merges (one process per GPU): actors registered in the
 * same order on every rank get the same dense index.  export copies the dense state counters
 * (u64[cap]) and next_op_versions (u64[cap]) into device buffers; import max-merges them back.
 * cap = ce_core_dense_capacity(). */
int ce_core_register_actors(ce_core *c, const uint8_t *actors, uint32_t m);
/* export/import_dense: VClock / GCounter only (CE_ERR_INVALID_ARG for the dot-set kinds). */
uint32_t ce_core_dense_capacity(ce_core *c);
int ce_core_export_dense(ce_core *c, uint64_t *d_state, uint64_t *d_nov);
int ce_core_import_dense(ce_core *c, const uint64_t *d_state, const uint64_t *d_nov);
/* 1 when every actor the state (or next_op_versions) holds has a registered dense slot, so
 * export/import_dense can carry it; 0 otherwise (a Dot named an actor outside
 * register_actors -- VClock::apply takes any actor, lib.rs:533-535).  Ranks then exchange
 * ce_core_state_bytes + ce_core_merge_state instead (crdtenc shard.exchange_vclock). */
int ce_core_dense_ready(ce_core *c);

/* ---------------------------------------------------------------------------------------- */
/* Multi-GPU partition of VClock / GCounter op files (one process per GPU).  North star: files */
/* sharded by address across the GPUs.  An op file's address is its path ops/<actor>/<version> */
/* (crdt-enc-tokio/src/lib.rs:280-293; op files are not content-named): its owner   */
/* rank is a hash of it, so every rank (and a directory listing) agrees on the partition.     */
/* Replaces, across ranks, the version gate of read_remote_ops (crdt-enc/src/lib.rs:516-544).  */
/* ---------------------------------------------------------------------------------------- */
/* owner rank of ops/<actor>/<version> among `world` ranks */
uint32_t ce_shard_owner(const uint8_t actor[16], uint64_t version, uint32_t world);
/* owner_out[i] = ce_shard_owner(actors[file_actor[i]], file_version[i], world) */
int ce_shard_owners(const uint8_t *actors, uint32_t m, const uint32_t *file_actor,
                    const uint64_t *file_version, uint64_t n, uint32_t world, uint32_t *owner_out);
/* ShardStats words for m writers (2m + 3 int64; layout in csrc/ce_common.h) */
uint32_t ce_shard_stats_len(uint32_t m);
/* This rank's ShardStats over its batch, resident in HBM (d_fa indexes the writer list shared by
 * every rank, in that shared order; each writer's files one run of ascending versions, as
 * Storage::load_ops returns them, storage.rs:36-40).  The stats are complete on return; the
 * ranks then all_reduce(MAX) them (int64). */
int ce_core_shard_stats(ce_core *c, const uint8_t *actors, uint32_t m, const uint32_t *d_fa,
                        const uint64_t *d_fv, uint32_t n, uint32_t rank, uint32_t world,
                        int64_t *d_stats);
/* The windows from the reduced stats: d_hi[a] = end of writer a's applied versions (from its
 * next_op_versions), d_hi[m] = flags (1 contract broken, 2 gap, 4 ranks' next_op_versions
 * differ).  Queued on the context's stream. */
int ce_core_shard_window(ce_core *c, const uint8_t *actors, uint32_t m, const int64_t *d_stats,
                         uint64_t *d_hi);
/* read_remote_ops over this rank's files with the windows as the gate: every file with
 * e0 <= version < hi is folded, into a PENDING batch -- nothing is committed until
 * ce_core_pending_commit, so a failure on any rank can leave every rank's state unchanged
 * (lib.rs:497-514).  Returns CE_OK, the lowest failing file's status, CE_ERR_OP_VERSION when the
 * windows stop at a gap (the files before it are folded, lib.rs:527-531), or CE_ERR_SHARD (flags
 * 1 or 4: nothing folded; compute the windows with ce_shard_window_exact and call again). */
int ce_core_ingest_ops_device_sharded(ce_core *c, const uint8_t *d_blob, const uint64_t *d_offs,
                                      uint32_t n, uint64_t blob_len, const uint8_t *actors,
                                      uint32_t m, const uint32_t *d_fa, const uint64_t *d_fv,
                                      const uint64_t *d_hi, int32_t *status);
/* The pending batch as a dense u64[ce_core_dense_capacity] over the registered slots (for the
 * all_reduce(MAX)); d_batch holds cap_words u64.  *ready = 0, and nothing is written, when the
 * batch names an actor outside register_actors or the actor table has grown past cap_words since
 * the caller sized d_batch (then commit it locally and exchange serialized states instead). */
int ce_core_pending_export(ce_core *c, uint64_t *d_batch, uint64_t cap_words, int *ready);
/* accept: state = max(state, d_import ? d_import (the reduced batch, import_words u64; at least
 * ce_core_dense_capacity) : the local pending batch), next_op_versions from the windows;
 * !accept: drop the pending batch. */
int ce_core_pending_commit(ce_core *c, int accept, const uint64_t *d_import, uint64_t import_words);
/* next_op_versions.get(writer) for each of m writers (host) */
int ce_core_writer_versions(ce_core *c, const uint8_t *actors, uint32_t m, uint64_t *e0_out);
/* Host twins (CPU ranks, tests): ShardStats over host metadata; the windows from reduced stats;
 * the exact windows from every rank's gathered (writer, version) metadata -- the reference's
 * loop over the batch in (writer, version) order (lib.rs:516-544). */
int ce_shard_stats_host(const uint8_t *actors, uint32_t m, const uint64_t *e0, const uint32_t *fa,
                        const uint64_t *fv, uint64_t n, uint32_t rank, uint32_t world,
                        int64_t *stats);
int ce_shard_window_host(uint32_t m, const uint64_t *e0, const int64_t *stats, uint64_t *hi);
int ce_shard_window_exact(uint32_t m, const uint64_t *e0, const uint32_t *fa, const uint64_t *fv,
                          uint64_t n, uint64_t *hi);

/* Diagnostics: how many times a code path ran on this core ("states_device_read",
 * "states_host_parse", "compact_device_writer"; per multi-segment op file "segdec_records"
 * (folded from the segment pass's records) and "segdec_fallback" (decoded whole)); lets tests
 * show which path did the work. */
uint64_t ce_core_path_count(ce_core *c, const char *path);

/* ---------------------------------------------------------------------------------------- */
/* Keys (crdt-enc/src/key_cryptor.rs:35-82): the data keys the core reads and writes with     */
/* ---------------------------------------------------------------------------------------- */
typedef struct ce_keys ce_keys;
/* rmp_serde::from_slice::<Keys>: Keys { latest_key_id: MVReg<Uuid, Uuid>,
 * keys: Orswot<Key, Uuid> }, Key { id: Uuid, key: VersionBytes } (key_cryptor.rs:35-40,85-89). */
int ce_keys_decode(const uint8_t *msgpack, size_t len, ce_keys **out);
/* The remote meta files (each VersionBytes(CURRENT_VERSION, msgpack(RemoteMeta)), lib.rs:
 * 647-664) merged as Core::read_remote_meta_ does (lib.rs:553-612), then the key cryptor's
 * register decoded as the gpgme KeyHandler does (crdt-enc-gpgme/src/lib.rs:79-105;
 * utils/mod.rs:94-126): every value VersionBytes(gpgme version, msgpack(Keys)), merged.
 * blob[offs[i], offs[i+1]) = file i as Storage::load_remote_metas returns it. */
int ce_keys_from_remote_metas(const uint8_t *blob, const uint64_t *offs, uint32_t n, ce_keys **out);
/* Keys::merge (key_cryptor.rs:42-50): MVReg::merge + Orswot::merge */
int ce_keys_merge(ce_keys *k, const ce_keys *other);
void ce_keys_free(ce_keys *k);
/* keys.read().val.len() */
uint32_t ce_keys_count(const ce_keys *k);
/* Keys::latest_key (key_cryptor.rs:59-70): the min-id key among the register's latest ids.
 * CE_ERR_NO_KEY when the register is empty; CE_ERR_DECODE when a latest id names no key (the
 * reference panics, :67).  Outputs may be NULL; key_out needs *key_len bytes (cap). */
int ce_keys_latest(const ce_keys *k, uint8_t id_out[16], uint8_t key_version_out[16],
                   uint8_t *key_out, size_t cap, size_t *key_len);
/* Keys::get_key (key_cryptor.rs:55-57): CE_ERR_NO_KEY when absent */
int ce_keys_get(const ce_keys *k, const uint8_t id[16], uint8_t key_version_out[16],
                uint8_t *key_out, size_t cap, size_t *key_len);
/* the i-th key of keys.read().val in id order (enumeration) */
int ce_keys_at(const ce_keys *k, uint32_t i, uint8_t id_out[16], uint8_t key_version_out[16],
               uint8_t *key_out, size_t cap, size_t *key_len);
/* CoreSubHandle::set_keys (lib.rs:382-388): the core reads and writes with Keys::latest_key
 * from now on; the other keys are kept for CE_OPEN_MULTI_KEY.  (ce_core_set_latest_key sets
 * one key and drops any others.) */
int ce_core_set_keys(ce_core *c, const ce_keys *k);

/* Framing helpers (crdt-enc/src/utils/version_bytes.rs): VersionBytesBuf chunk/advance. */
typedef struct ce_vbuf {
  size_t pos;
  uint8_t version[16];
  const uint8_t *content;
  size_t content_len;
} ce_vbuf;
void ce_vbuf_init(ce_vbuf *b, const uint8_t version[16], const uint8_t *content, size_t len);
size_t ce_vbuf_remaining(const ce_vbuf *b);
/* current chunk; returns its length */
size_t ce_vbuf_chunk(const ce_vbuf *b, const uint8_t **chunk);
/* returns 0, or -1 when cnt > remaining (the reference panics, version_bytes.rs:281) */
int ce_vbuf_advance(ce_vbuf *b, size_t cnt);
/* chunks_vectored (version_bytes.rs:285-308): fills up to n_dst (ptr,len) pairs */
size_t ce_vbuf_chunks_vectored(const ce_vbuf *b, const uint8_t **dst_ptr, size_t *dst_len,
                               size_t n_dst);

#ifdef __cplusplus
}
#endif
#endif
