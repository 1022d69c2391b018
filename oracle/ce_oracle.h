/*
 * ce_oracle.h -- CPU restatement of crdt-enc's compaction/ingest hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker, never the product: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product path lives in crdt-enc_amd/ (HIP) and must never call into this.
 *
 * Parity anchors (the reference is Rust; it cannot be built in this image, see
 * DESIGN.md "Oracle"):
 *   - AEAD: chacha20poly1305 0.10 XChaCha20Poly1305, called at
 *     crdt-enc-xchacha20poly1305/src/lib.rs:56-58 (encrypt) and :95-97 (decrypt).
 *     Restated from draft-irtf-cfrg-xchacha-03 + RFC 8439; pinned by the draft's
 *     KATs and by OpenSSL-generated fixtures (tests/golden/make_golden.py).
 *   - Boxes: crdt-enc-xchacha20poly1305/src/lib.rs:40-113 (EncBox, VersionBytesRef),
 *     rmp-serde 1.x rules; pinned by Python msgpack fixtures.
 *   - Fold: crdt-enc/src/lib.rs:401-547 (read_remote_states / read_remote_ops),
 *     crdts 7 VClock/GCounter.
 *   - Naming: crdt-enc-tokio/src/lib.rs:403-432 (SHA3-256 + BASE32_NOPAD).
 */
#ifndef CE_ORACLE_H
#define CE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes: identical numbering to include/crdtenc.h (reference check order) */
enum {
  OC_OK = 0,
  OC_ERR_OUTER_LEN = 1,      /* VersionBytes::deserialize InvalidLength (version_bytes.rs:187) */
  OC_ERR_OUTER_VERSION = 2,  /* ensure_versions_phf(SUPPORTED_VERSIONS) (lib.rs:435,501)     */
  OC_ERR_KEY_VERSION = 3,    /* xchacha lib.rs:74-75 */
  OC_ERR_KEY_LEN = 4,        /* xchacha lib.rs:76-78 */
  OC_ERR_PARSE_VBOX = 5,     /* xchacha lib.rs:82-83 */
  OC_ERR_DATA_VERSION = 6,   /* xchacha lib.rs:84-86 */
  OC_ERR_PARSE_ENCBOX = 7,   /* xchacha lib.rs:87-88 */
  OC_ERR_NONCE_LEN = 8,      /* xchacha lib.rs:89-91 */
  OC_ERR_AUTH = 9,           /* xchacha lib.rs:92-97 "Decryption failed" */
  OC_ERR_PT_LEN = 10,        /* VersionBytesRef::deserialize on clear text (lib.rs:443,504) */
  OC_ERR_PT_VERSION = 11,    /* ensure_versions(supported_data_versions) (lib.rs:444,505)   */
  OC_ERR_DECODE = 12,        /* rmp_serde::from_slice (lib.rs:447,507) */
  OC_ERR_OP_VERSION = 13     /* "Unexpected op version" (lib.rs:527-531) */
};

/* ---- primitives ---- */
void oc_chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce12[12],
                       uint8_t out[64]);
void oc_hchacha20(const uint8_t key[32], const uint8_t n16[16], uint8_t out[32]);
void oc_poly1305(const uint8_t key[32], const uint8_t *msg, size_t len, uint8_t tag[16]);
/* out = ct || tag16 ; empty AAD */
void oc_xchacha_seal(const uint8_t key[32], const uint8_t nonce[24], const uint8_t *pt,
                     size_t len, uint8_t *out);
/* with associated data (KAT only; the reference always passes empty AAD) */
void oc_xchacha_seal_aad(const uint8_t key[32], const uint8_t nonce[24], const uint8_t *aad,
                         size_t aad_len, const uint8_t *pt, size_t len, uint8_t *out);
/* ct includes the trailing tag; returns 0 on success, OC_ERR_AUTH otherwise */
int oc_xchacha_open(const uint8_t key[32], const uint8_t nonce[24], const uint8_t *ct,
                    size_t ct_len, uint8_t *out);
void oc_sha3_256(const uint8_t *msg, size_t len, uint8_t out[32]);
/* BASE32_NOPAD (RFC 4648 upper case, no padding); out must hold ceil(len*8/5)+1 */
size_t oc_base32_nopad(const uint8_t *in, size_t len, char *out);

/* ---- EncHandler (crdt-enc-xchacha20poly1305/src/lib.rs) ---- */
/* Cryptor::encrypt with an explicit nonce (the reference draws it from rand::rng()).
 * out must hold oc_cryptor_sealed_len(clear_len). Returns status. */
size_t oc_cryptor_sealed_len(size_t clear_len);
int oc_cryptor_encrypt(const uint8_t key_version[16], const uint8_t *key, size_t key_len,
                       const uint8_t nonce[24], const uint8_t *clear, size_t clear_len,
                       uint8_t *out, size_t *out_len);
/* Cryptor::decrypt: enc = VersionBytes content (after the outer 16-byte version).
 * out must hold enc_len bytes. Returns status. */
int oc_cryptor_decrypt(const uint8_t key_version[16], const uint8_t *key, size_t key_len,
                       const uint8_t *enc, size_t enc_len, uint8_t *out, size_t *out_len);

/* ---- VClock / GCounter state (crdts 7; sorted by actor bytes = BTreeMap order) ---- */
typedef struct {
  uint8_t (*actor)[16];
  uint64_t *counter;
  size_t n, cap;
} oc_vclock;

void oc_vclock_init(oc_vclock *v);
void oc_vclock_free(oc_vclock *v);
uint64_t oc_vclock_get(const oc_vclock *v, const uint8_t actor[16]);
void oc_vclock_apply(oc_vclock *v, const uint8_t actor[16], uint64_t counter);

/* state kinds for StateWrapper<S> */
enum { OC_STATE_VCLOCK = 0, OC_STATE_GCOUNTER = 1 };

typedef struct {
  int kind;
  oc_vclock next_op_versions; /* StateWrapper.next_op_versions (lib.rs:741) */
  oc_vclock state;            /* VClock or GCounter.inner */
} oc_core;

void oc_core_init(oc_core *c, int kind);
void oc_core_free(oc_core *c);

/* rmp_serde::to_vec_named(&StateWrapper) (lib.rs:336). Returns needed length; writes if out
 * != NULL and cap is large enough. */
size_t oc_core_serialize(const oc_core *c, uint8_t *out, size_t cap);
/* rmp_serde::from_slice::<StateWrapper<S>> into (merged into) c; returns status */
int oc_core_merge_serialized(oc_core *c, const uint8_t *buf, size_t len);

/* Decode rmp Vec<Dot<Uuid>> (lib.rs:507) and apply in order.  Returns OC_OK or OC_ERR_DECODE.
 * When dry_run != 0 only validates. */
int oc_decode_apply_dots(oc_core *c, const uint8_t *buf, size_t len, int dry_run);

/*
 * Core::read_remote_ops (lib.rs:471-547) over an in-memory batch as Storage::load_ops returns
 * it: files[i] = whole op file (outer version || cryptor box), in per-actor version order.
 * supported: sorted list of n_supported data versions.  status[i] receives the per-file status.
 * Semantics: every file is opened and decoded first; if any fails nothing is folded and the
 * first failing file's status is returned.  Then the per-actor version gate runs in the given
 * order (skip < expected; > expected -> OC_ERR_OP_VERSION and the fold stops there, keeping
 * what was applied before it, exactly like the reference's loop).
 */
int oc_read_remote_ops(oc_core *c, const uint8_t key_version[16], const uint8_t *key,
                       size_t key_len, const uint8_t (*supported)[16], size_t n_supported,
                       const uint8_t *blob, const uint64_t *offs, const uint8_t (*file_actor)[16],
                       const uint64_t *file_version, size_t n_files, int32_t *status);

/* Core::read_remote_states (lib.rs:401-469); state files in the ingest format (outer
 * CURRENT_VERSION, inner VersionBytes(data_version, msgpack(StateWrapper))). */
int oc_read_remote_states(oc_core *c, const uint8_t key_version[16], const uint8_t *key,
                          size_t key_len, const uint8_t (*supported)[16], size_t n_supported,
                          const uint8_t *blob, const uint64_t *offs, size_t n_files,
                          int32_t *status);

/* multi-threaded batch open used by the CPU baseline: decrypt + decode check per file.
 * Returns number of files that opened OK. */
size_t oc_open_batch_mt(const uint8_t key[32], const uint8_t data_version[16],
                        const uint8_t *blob, const uint64_t *offs, size_t n_files, int n_threads,
                        int32_t *status);

/* CPU baseline: whole read_remote_ops + serialize, with n_threads AEAD workers (decode and
 * fold on the calling thread, mirroring lib.rs:497-544).  Returns serialized length. */
size_t oc_compact_ops_baseline(int kind, const uint8_t key[32], const uint8_t data_version[16],
                               const uint8_t *blob, const uint64_t *offs,
                               const uint8_t (*file_actor)[16], const uint64_t *file_version,
                               size_t n_files, int n_threads, uint8_t *out, size_t cap,
                               int *err);

/* Best-CPU baseline (SURVEY.md §8d mode ii): the same result with every stage on n_threads
 * threads -- open + decode check parallel over files, then the version gate and the fold
 * parallel over actors (thread t folds the files of the actors it owns, in batch order, into a
 * private StateWrapper), then the private states merged (VClock::merge, pointwise max).  A
 * batch with a version gap is folded sequentially instead (the reference stops at the gap in
 * batch order, lib.rs:527-531).  Returns serialized length. */
size_t oc_compact_ops_best(int kind, const uint8_t key[32], const uint8_t data_version[16],
                           const uint8_t *blob, const uint64_t *offs,
                           const uint8_t (*file_actor)[16], const uint64_t *file_version,
                           size_t n_files, int n_threads, uint8_t *out, size_t cap, int *err);

/* Orswot<u64, Uuid> CPU baseline (C3): a C restatement of oracle/crdts.py (crdts 7 Orswot
 * apply / apply_rm / apply_deferred / merge, Core.read_remote_states then read_remote_ops).
 * Every state and op file is opened and decoded on n_threads threads; the state merges, the
 * version gate and the op fold then run in file order on the calling thread (the fold is
 * order-dependent: removals defer on the clock).  Returns the length of the canonical
 * StateWrapper (crdts.py serialize; writes it when out != NULL and it fits in cap); seal != 0
 * also seals it as Core::compact does (version prefix, Cryptor::encrypt, SHA3-256 name).
 * phase_s (nullable) receives [open+decode, state merges, op fold, serialize(+seal)] seconds. */
size_t oc_compact_orswot_best(const uint8_t key[32], const uint8_t data_version[16],
                              const uint8_t *state_blob, const uint64_t *state_offs,
                              size_t n_states, const uint8_t *blob, const uint64_t *offs,
                              const uint8_t (*file_actor)[16], const uint64_t *file_version,
                              size_t n_files, int n_threads, int seal, uint8_t *out, size_t cap,
                              int *err, double phase_s[4]);

#ifdef __cplusplus
}
#endif
#endif
