// ce_common.h -- definitions shared by the HIP kernels and the host library.
//
// Contents:
//   * the reference's version UUIDs (raw big-endian bytes, as Uuid::from_u128 stores them)
//   * status codes (reference check order; see include/crdtenc.h)
//   * a bounds-checked msgpack reader implementing rmp-serde 1.x `from_slice` acceptance for the
//     boxes on the hot path (VersionBytesRef, EncBox, Vec<Dot>, StateWrapper<VClock|GCounter>),
//     compiled for both host and device (CE_HD).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "crdtenc.h"

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define CE_HD __host__ __device__ __forceinline__
#else
#define CE_HD inline
#endif

namespace ce {

// crdt-enc/src/lib.rs:26  CURRENT_VERSION e834d789-101b-4634-9823-9de990a9051f
static constexpr uint8_t kCoreVersion[16] = {0xe8, 0x34, 0xd7, 0x89, 0x10, 0x1b, 0x46, 0x34,
                                             0x98, 0x23, 0x9d, 0xe9, 0x90, 0xa9, 0x05, 0x1f};
// crdt-enc-xchacha20poly1305/src/lib.rs:11  DATA_VERSION c7f269be-0ff5-4a77-99c3-7c23c96d5cb4
static constexpr uint8_t kBoxVersion[16] = {0xc7, 0xf2, 0x69, 0xbe, 0x0f, 0xf5, 0x4a, 0x77,
                                            0x99, 0xc3, 0x7c, 0x23, 0xc9, 0x6d, 0x5c, 0xb4};
// crdt-enc-xchacha20poly1305/src/lib.rs:13  KEY_VERSION 5df28591-439a-4cef-8ca6-8433276cc9ed
static constexpr uint8_t kKeyVersion[16] = {0x5d, 0xf2, 0x85, 0x91, 0x43, 0x9a, 0x4c, 0xef,
                                            0x8c, 0xa6, 0x84, 0x33, 0x27, 0x6c, 0xc9, 0xed};

// internal status: the device envelope parser met a form it does not decode in place
// (a byte string encoded as an array of u8, or nesting deeper than kMaxDepth); the host
// normalizes the envelope and resubmits the file (ce_batch.cpp).
static constexpr int32_t kStatusHostParse = 100;
static constexpr int kMaxDepth = 32;

// ---------------------------------------------------------------------------------------
// msgpack reader
// ---------------------------------------------------------------------------------------
struct Rd {
  const uint8_t* p;
  uint64_t n;
  uint64_t i;
};
// byte x of a reader's input.  The helpers below are templates over the reader type R, so a
// parser can supply its own byte source with the same grammar code.  (A 16-byte register window
// over HBM for the lane-per-file op decode measured slower than byte loads: C3 ds_count 0.41 ->
// 0.62 ms, ds_emit 0.67 -> 0.93 ms.)
CE_HD uint8_t rb(const Rd& r, uint64_t x) { return r.p[x]; }

template <typename R>
CE_HD bool rd_take(R& r, uint64_t k, uint64_t* at) {
  if (r.n - r.i < k) return false;
  *at = r.i;
  r.i += k;
  return true;
}

template <typename R>
CE_HD bool rd_be(R& r, int k, uint64_t* v) {
  uint64_t at;
  if (!rd_take(r, (uint64_t)k, &at)) return false;
  uint64_t x = 0;
  for (int j = 0; j < k; j++) x = (x << 8) | rb(r, at + j);
  *v = x;
  return true;
}

// serde u64 visitor: any non-negative msgpack integer
template <typename R>
CE_HD bool rd_u64(R& r, uint64_t* v) {
  uint64_t at, x;
  if (!rd_take(r, 1, &at)) return false;
  const uint8_t m = rb(r, at);
  if (m <= 0x7f) { *v = m; return true; }
  switch (m) {
    case 0xcc: return rd_be(r, 1, v);
    case 0xcd: return rd_be(r, 2, v);
    case 0xce: return rd_be(r, 4, v);
    case 0xcf: return rd_be(r, 8, v);
    case 0xd0: if (!rd_be(r, 1, &x) || (x & 0x80)) return false; *v = x; return true;
    case 0xd1: if (!rd_be(r, 2, &x) || (x & 0x8000)) return false; *v = x; return true;
    case 0xd2: if (!rd_be(r, 4, &x) || (x & 0x80000000ull)) return false; *v = x; return true;
    case 0xd3: if (!rd_be(r, 8, &x) || (x >> 63)) return false; *v = x; return true;
    default: return false;
  }
}

CE_HD bool is_array_marker(uint8_t m) { return (m & 0xf0) == 0x90 || m == 0xdc || m == 0xdd; }
CE_HD bool is_map_marker(uint8_t m) { return (m & 0xf0) == 0x80 || m == 0xde || m == 0xdf; }
CE_HD bool is_binstr_marker(uint8_t m) {
  return (m & 0xe0) == 0xa0 || m == 0xc4 || m == 0xc5 || m == 0xc6 || m == 0xd9 || m == 0xda ||
         m == 0xdb;
}

template <typename R>
CE_HD bool rd_array_hdr(R& r, uint64_t* len) {
  uint64_t at;
  if (!rd_take(r, 1, &at)) return false;
  const uint8_t m = rb(r, at);
  if ((m & 0xf0) == 0x90) { *len = m & 0x0f; return true; }
  if (m == 0xdc) return rd_be(r, 2, len);
  if (m == 0xdd) return rd_be(r, 4, len);
  return false;
}

template <typename R>
CE_HD bool rd_map_hdr(R& r, uint64_t* len) {
  uint64_t at;
  if (!rd_take(r, 1, &at)) return false;
  const uint8_t m = rb(r, at);
  if ((m & 0xf0) == 0x80) { *len = m & 0x0f; return true; }
  if (m == 0xde) return rd_be(r, 2, len);
  if (m == 0xdf) return rd_be(r, 4, len);
  return false;
}

// bin/str: kind 1 = bin, 2 = str; payload [*off, *off + *len)
template <typename R>
CE_HD bool rd_binstr(R& r, int* kind, uint64_t* off, uint64_t* len) {
  uint64_t at, l;
  if (!rd_take(r, 1, &at)) return false;
  const uint8_t m = rb(r, at);
  if ((m & 0xe0) == 0xa0) { l = m & 0x1f; *kind = 2; }
  else if (m == 0xc4 || m == 0xd9) { if (!rd_be(r, 1, &l)) return false; *kind = m == 0xc4 ? 1 : 2; }
  else if (m == 0xc5 || m == 0xda) { if (!rd_be(r, 2, &l)) return false; *kind = m == 0xc5 ? 1 : 2; }
  else if (m == 0xc6 || m == 0xdb) { if (!rd_be(r, 4, &l)) return false; *kind = m == 0xc6 ? 1 : 2; }
  else return false;
  if (!rd_take(r, l, off)) return false;
  *len = l;
  return true;
}

CE_HD bool utf8_valid(const uint8_t* s, uint64_t n) {
  uint64_t i = 0;
  while (i < n) {
    const uint8_t c = s[i];
    if (c < 0x80) { i++; continue; }
    int k;
    uint32_t cp;
    if ((c & 0xe0) == 0xc0) { k = 1; cp = c & 0x1f; }
    else if ((c & 0xf0) == 0xe0) { k = 2; cp = c & 0x0f; }
    else if ((c & 0xf8) == 0xf0) { k = 3; cp = c & 0x07; }
    else return false;
    for (int j = 1; j <= k; j++) {
      if (i + j >= n || (s[i + j] & 0xc0) != 0x80) return false;
      cp = (cp << 6) | (s[i + j] & 0x3f);
    }
    if ((k == 1 && cp < 0x80) || (k == 2 && cp < 0x800) || (k == 3 && cp < 0x10000)) return false;
    if (cp > 0x10ffff || (cp >= 0xd800 && cp <= 0xdfff)) return false;
    i += (uint64_t)k + 1;
  }
  return true;
}

// Uuid, non-human-readable (uuid 1.x serde: deserialize_bytes, visit_bytes only): bin of 16,
// or a str that is not valid UTF-8 (rmp-serde then calls visit_bytes) of 16.
template <typename R>
CE_HD bool rd_uuid(R& r, uint64_t* off) {
  int kind;
  uint64_t l;
  if (!rd_binstr(r, &kind, off, &l)) return false;
  if (l != 16) return false;
  if (kind == 2 && utf8_valid(r.p + *off, 16)) return false;
  return true;
}

// skip one value (serde IgnoredAny), iterative with a bounded stack.  Returns 1 ok, 0 error,
// -1 too deep (host must handle).
template <typename R>
CE_HD int rd_skip(R& r) {
  uint64_t stack[kMaxDepth];
  int sp = 0;
  uint64_t remaining = 1;
  for (;;) {
    while (remaining == 0) {
      if (sp == 0) return 1;
      remaining = stack[--sp];
    }
    remaining--;
    uint64_t at, len;
    if (!rd_take(r, 1, &at)) return 0;
    const uint8_t m = rb(r, at);
    if (m <= 0x7f || m >= 0xe0 || m == 0xc0 || m == 0xc2 || m == 0xc3) continue;
    uint64_t cnt = 0;
    bool container = false;
    if ((m & 0xf0) == 0x80) { cnt = 2ull * (m & 0x0f); container = true; }
    else if ((m & 0xf0) == 0x90) { cnt = m & 0x0f; container = true; }
    else if ((m & 0xe0) == 0xa0) { if (!rd_take(r, m & 0x1f, &at)) return 0; continue; }
    else {
      switch (m) {
        case 0xc4: case 0xd9: if (!rd_be(r, 1, &len) || !rd_take(r, len, &at)) return 0; continue;
        case 0xc5: case 0xda: if (!rd_be(r, 2, &len) || !rd_take(r, len, &at)) return 0; continue;
        case 0xc6: case 0xdb: if (!rd_be(r, 4, &len) || !rd_take(r, len, &at)) return 0; continue;
        case 0xcc: case 0xd0: if (!rd_take(r, 1, &at)) return 0; continue;
        case 0xcd: case 0xd1: if (!rd_take(r, 2, &at)) return 0; continue;
        case 0xce: case 0xd2: case 0xca: if (!rd_take(r, 4, &at)) return 0; continue;
        case 0xcf: case 0xd3: case 0xcb: if (!rd_take(r, 8, &at)) return 0; continue;
        case 0xd4: if (!rd_take(r, 2, &at)) return 0; continue;
        case 0xd5: if (!rd_take(r, 3, &at)) return 0; continue;
        case 0xd6: if (!rd_take(r, 5, &at)) return 0; continue;
        case 0xd7: if (!rd_take(r, 9, &at)) return 0; continue;
        case 0xd8: if (!rd_take(r, 17, &at)) return 0; continue;
        case 0xc7: if (!rd_be(r, 1, &len) || !rd_take(r, len + 1, &at)) return 0; continue;
        case 0xc8: if (!rd_be(r, 2, &len) || !rd_take(r, len + 1, &at)) return 0; continue;
        case 0xc9: if (!rd_be(r, 4, &len) || !rd_take(r, len + 1, &at)) return 0; continue;
        case 0xdc: if (!rd_be(r, 2, &cnt)) return 0; container = true; break;
        case 0xdd: if (!rd_be(r, 4, &cnt)) return 0; container = true; break;
        case 0xde: if (!rd_be(r, 2, &cnt)) return 0; cnt *= 2; container = true; break;
        case 0xdf: if (!rd_be(r, 4, &cnt)) return 0; cnt *= 2; container = true; break;
        default: return 0;  // 0xc1
      }
    }
    if (container && cnt) {
      if (cnt > r.n - r.i) return 0;  // each element takes >= 1 byte
      if (sp == kMaxDepth) return -1;
      stack[sp++] = remaining;
      remaining = cnt;
    }
  }
}

// Struct field identifier (serde derive __FieldVisitor): str/bin compared to the names,
// non-negative integers are field indices; returns field index, nf = ignored, -1 error.
template <int NF, typename R>
CE_HD int rd_field(R& r, const char* const (&names)[NF]) {
  if (r.i >= r.n) return -1;
  const uint8_t m = rb(r, r.i);
  if (is_binstr_marker(m)) {
    int kind;
    uint64_t off, l;
    if (!rd_binstr(r, &kind, &off, &l)) return -1;
    for (int f = 0; f < NF; f++) {
      const char* s = names[f];
      uint64_t k = 0;
      while (s[k] && k < l && (uint8_t)s[k] == rb(r, off + k)) k++;
      if (k == l && s[k] == 0) return f;
    }
    return NF;
  }
  uint64_t v;
  if (!rd_u64(r, &v)) return -1;
  return v < (uint64_t)NF ? (int)v : NF;
}

// Byte string for serde_bytes fields: bin or str (borrowed).  An array-of-u8 form is legal for
// serde_bytes but not contiguous in the input: report "host parse" (-1).
template <typename R>
CE_HD int rd_bytes(R& r, uint64_t* off, uint64_t* len) {
  if (r.i >= r.n) return 0;
  const uint8_t m = rb(r, r.i);
  if (is_array_marker(m)) return -1;
  int kind;
  return rd_binstr(r, &kind, off, len) ? 1 : 0;
}

// ---------------------------------------------------------------------------------------
// The cryptor envelope: msgpack(VersionBytesRef(DATA_VERSION, msgpack(EncBox{nonce,enc_data})))
// (crdt-enc-xchacha20poly1305/src/lib.rs:82-91).  `enc` is the VersionBytes content after the
// outer 16-byte version.  On success: nonce and enc_data offsets relative to `enc`.
// ---------------------------------------------------------------------------------------
struct Envelope {
  uint64_t nonce_off, nonce_len, enc_off, enc_len;
};

CE_HD int32_t parse_envelope(const uint8_t* enc, uint64_t enc_len, Envelope* e) {
  Rd r{enc, enc_len, 0};
  // VersionBytesRef: tuple struct -> visit_seq only: array of exactly 2
  uint64_t cnt;
  if (r.n == 0 || !is_array_marker(r.p[0])) return CE_ERR_PARSE_VBOX;
  if (!rd_array_hdr(r, &cnt) || cnt != 2) return CE_ERR_PARSE_VBOX;
  uint64_t ver_off;
  if (!rd_uuid(r, &ver_off)) return CE_ERR_PARSE_VBOX;
  uint64_t box_off, box_len;
  int b = rd_bytes(r, &box_off, &box_len);
  if (b < 0) return kStatusHostParse;
  if (b == 0) return CE_ERR_PARSE_VBOX;
  for (int k = 0; k < 16; k++)
    if (enc[ver_off + k] != kBoxVersion[k]) return CE_ERR_DATA_VERSION;
  // EncBox: map (any order, unknown keys ignored, duplicates rejected) or array of exactly 2
  Rd q{enc + box_off, box_len, 0};
  static constexpr const char* kF[2] = {"nonce", "enc_data"};
  uint64_t off[2] = {0, 0}, len[2] = {0, 0};
  if (q.n == 0) return CE_ERR_PARSE_ENCBOX;
  const uint8_t m = q.p[0];
  if (is_array_marker(m)) {
    if (!rd_array_hdr(q, &cnt) || cnt != 2) return CE_ERR_PARSE_ENCBOX;
    for (int f = 0; f < 2; f++) {
      int bb = rd_bytes(q, &off[f], &len[f]);
      if (bb < 0) return kStatusHostParse;
      if (bb == 0) return CE_ERR_PARSE_ENCBOX;
    }
  } else {
    if (!rd_map_hdr(q, &cnt)) return CE_ERR_PARSE_ENCBOX;
    unsigned seen = 0;
    for (uint64_t k = 0; k < cnt; k++) {
      int f = rd_field<2>(q, kF);
      if (f < 0) return CE_ERR_PARSE_ENCBOX;
      if (f == 2) {
        int s = rd_skip(q);
        if (s < 0) return kStatusHostParse;
        if (s == 0) return CE_ERR_PARSE_ENCBOX;
        continue;
      }
      if (seen & (1u << f)) return CE_ERR_PARSE_ENCBOX;
      seen |= 1u << f;
      int bb = rd_bytes(q, &off[f], &len[f]);
      if (bb < 0) return kStatusHostParse;
      if (bb == 0) return CE_ERR_PARSE_ENCBOX;
    }
    if (seen != 3u) return CE_ERR_PARSE_ENCBOX;
  }
  if (len[0] != 24) return CE_ERR_NONCE_LEN;
  if (len[1] < 16) return CE_ERR_AUTH;  // aead decrypt of a too-short buffer -> "Decryption failed"
  e->nonce_off = box_off + off[0];
  e->nonce_len = len[0];
  e->enc_off = box_off + off[1];
  e->enc_len = len[1];
  return CE_OK;
}

// canonical envelope size produced by EncHandler::encrypt (xchacha lib.rs:59-67)
CE_HD uint64_t bin_hdr_len(uint64_t l) { return l <= 0xff ? 2 : (l <= 0xffff ? 3 : 5); }
CE_HD uint64_t encbox_len(uint64_t clear_len) {
  const uint64_t ct = clear_len + 16;
  return 1 + 6 + 2 + 24 + 9 + bin_hdr_len(ct) + ct;
}
CE_HD uint64_t sealed_len(uint64_t clear_len) {
  const uint64_t eb = encbox_len(clear_len);
  return 1 + 2 + 16 + bin_hdr_len(eb) + eb;
}
CE_HD uint64_t put_bin_hdr(uint8_t* o, uint64_t l) {
  if (l <= 0xff) { o[0] = 0xc4; o[1] = (uint8_t)l; return 2; }
  if (l <= 0xffff) { o[0] = 0xc5; o[1] = (uint8_t)(l >> 8); o[2] = (uint8_t)l; return 3; }
  o[0] = 0xc6; o[1] = (uint8_t)(l >> 24); o[2] = (uint8_t)(l >> 16); o[3] = (uint8_t)(l >> 8);
  o[4] = (uint8_t)l;
  return 5;
}
// writes the canonical header (everything before the ciphertext); returns its length.
CE_HD uint64_t put_envelope_header(uint8_t* o, uint64_t clear_len, const uint8_t nonce[24]) {
  uint64_t k = 0;
  o[k++] = 0x92;                        // VersionBytesRef tuple -> array(2)
  o[k++] = 0xc4; o[k++] = 0x10;         // bin8(16) DATA_VERSION
  for (int j = 0; j < 16; j++) o[k++] = kBoxVersion[j];
  k += put_bin_hdr(o + k, encbox_len(clear_len));
  o[k++] = 0x82;                        // EncBox map(2)
  o[k++] = 0xa5; o[k++] = 'n'; o[k++] = 'o'; o[k++] = 'n'; o[k++] = 'c'; o[k++] = 'e';
  o[k++] = 0xc4; o[k++] = 24;
  for (int j = 0; j < 24; j++) o[k++] = nonce[j];
  o[k++] = 0xa8; o[k++] = 'e'; o[k++] = 'n'; o[k++] = 'c'; o[k++] = '_'; o[k++] = 'd';
  o[k++] = 'a'; o[k++] = 't'; o[k++] = 'a';
  k += put_bin_hdr(o + k, clear_len + 16);
  return k;
}

}  // namespace ce

namespace ce {

// Dot<Uuid> (crdts 7, derive(Deserialize)): map {"actor", "counter"} in any order (unknown keys
// ignored, duplicates rejected, both required) or an array of exactly 2.  Returns 1 ok,
// 0 decode error, -1 nesting too deep for the device (host handles).
template <typename R>
CE_HD int parse_dot(R& r, uint64_t* actor_off, uint64_t* counter) {
  static constexpr const char* kF[2] = {"actor", "counter"};
  if (r.i >= r.n) return 0;
  const uint8_t m = rb(r, r.i);
  uint64_t cnt;
  if (is_array_marker(m)) {
    if (!rd_array_hdr(r, &cnt) || cnt != 2) return 0;
    if (!rd_uuid(r, actor_off)) return 0;
    return rd_u64(r, counter) ? 1 : 0;
  }
  if (!rd_map_hdr(r, &cnt)) return 0;
  unsigned seen = 0;
  for (uint64_t k = 0; k < cnt; k++) {
    int f = rd_field<2>(r, kF);
    if (f < 0) return 0;
    if (f == 2) {
      int s = rd_skip(r);
      if (s <= 0) return s;
      continue;
    }
    if (seen & (1u << f)) return 0;
    seen |= 1u << f;
    if (f == 0) { if (!rd_uuid(r, actor_off)) return 0; }
    else if (!rd_u64(r, counter)) return 0;
  }
  return seen == 3u ? 1 : 0;
}

// actor table hash (shared by host table builder and device lookups)
CE_HD uint32_t actor_hash(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
  uint32_t h = (k0 * 0x9E3779B1u) ^ (k1 * 0x85EBCA77u) ^ (k2 * 0xC2B2AE3Du) ^ (k3 * 0x27D4EB2Fu);
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h;
}

// ---------------------------------------------------------------------------------------
// Multi-GPU partition of op files (VClock / GCounter): an op file is addressed by its path
// ops/<actor>/<version> (crdt-enc-tokio/src/lib.rs:280-293; op files are not content-named,
// SURVEY F8), and its owner rank is a hash of that address, so every rank -- and the storage
// listing -- agrees on the partition without reading a file.  Each rank folds only its files;
// the version gate (crdt-enc/src/lib.rs:519-531) becomes per-writer windows [e0, hi) agreed
// through one all_reduce(MAX) of ShardStats (ce_shard.hip / ce_shard.cpp).
// ---------------------------------------------------------------------------------------
CE_HD uint64_t shard_mix64(uint64_t x) {
  x ^= x >> 31;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 29;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 32;
  return x;
}
// owner rank of ops/<actor>/<version> among `world` ranks (multiply-shift range reduction)
CE_HD uint32_t shard_owner(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3, uint64_t v,
                           uint32_t world) {
  const uint64_t a = ((uint64_t)k1 << 32 | k0) * 0x9E3779B97F4A7C15ull ^ ((uint64_t)k3 << 32 | k2);
  const uint64_t x = shard_mix64(a ^ shard_mix64(v + 0xD1B54A32D192ED03ull));
  return (uint32_t)(((x & 0xffffffffull) * world) >> 32);
}
// ShardStats: int64[2m + 3] per rank, reduced with all_reduce(MAX).  Every word is a u64 with
// its top bit flipped (u64 order == int64 order):
//   [a]       ~cand[a]: cand = the smallest version >= e0[a] that this rank owns and does not
//             hold (MAX of ~cand = the global MIN: the first missing version of writer a)
//   [m + a]   vmax[a] + 1 over held versions >= e0[a] (0: none)
//   [2m]      1 when a rank's batch breaks the contract (a writer split into several runs,
//             versions descending inside a run, a file the partition gives to another rank, a
//             walk past kShardWalkLimit): the windows are then computed exactly from the
//             gathered metadata instead (ce_shard_window_exact)
//   [2m + 1]  h(e0), [2m + 2] ~h(e0): MAX(h) == ~MAX(~h) iff every rank started from the same
//             next_op_versions (the partition needs the replicated starting state)
static constexpr uint64_t kShardFlip = 0x8000000000000000ull;
static constexpr uint64_t kShardWalkLimit = 1u << 16;
// window flags word (hi[m]): bit 0 = contract broken (exact fallback), bit 1 = a gap (the fold
// stops there, CE_ERR_OP_VERSION), bit 2 = the ranks' next_op_versions differ
static constexpr uint64_t kShardBad = 1, kShardGap = 2, kShardE0Mismatch = 4;
CE_HD uint64_t shard_e0_hash(const uint64_t* e0, uint32_t m) {
  uint64_t h = 0x243F6A8885A308D3ull ^ m;
  for (uint32_t a = 0; a < m; a++) h = shard_mix64(h ^ e0[a]) + a;
  return h;
}
// windows from the reduced stats (plain u64, flips removed): hi[a] = the end of writer a's
// applied versions, hi[m] = flags.  The reference's loop over the batch in (writer, version)
// order applies every version from e0 while they are consecutive; the first writer (in the
// shared writer order) whose run has a missing version below its largest held one stops the
// fold there: its versions up to the hole are applied, later writers get nothing (lib.rs:
// 519-531, the error returned after the files before it are folded).
template <typename Get>
CE_HD uint32_t shard_first_gap(uint32_t m, Get&& cand_vmaxp1) {
  for (uint32_t a = 0; a < m; a++) {
    uint64_t cand, vmaxp1;
    cand_vmaxp1(a, &cand, &vmaxp1);
    if (vmaxp1 != 0 && cand < vmaxp1) return a;
  }
  return m;
}
CE_HD uint64_t shard_hi(uint32_t a, uint32_t astar, uint64_t e0, uint64_t cand, uint64_t vmaxp1) {
  if (a > astar) return e0;
  if (a == astar) return cand;          // cand >= e0: versions e0..cand-1 are all held somewhere
  return vmaxp1 > e0 ? vmaxp1 : e0;     // no hole below vmax: e0..vmax all applied
}

// one actor-table entry: 16-byte UUID key + occupancy (32 bytes, two dwordx4 loads)
struct alignas(16) ActorSlot {
  uint32_t k[4];
  uint32_t used;
  uint32_t pad[3];
};

}  // namespace ce
