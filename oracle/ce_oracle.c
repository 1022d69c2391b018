/*
 * ce_oracle.c -- CPU restatement (plain C) of crdt-enc's compaction/ingest hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see ce_oracle.h).  Written independently of the HIP product:
 * Poly1305 uses 44/44/42-bit limbs with 128-bit products (the product uses 26-bit limbs),
 * the msgpack reader is a separate recursive-descent implementation, and the fold uses a
 * sorted-array map (BTreeMap order) instead of the product's dense actor table.
 */
#include "ce_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------ */
/* version UUIDs (raw big-endian bytes, Uuid::from_u128)                                  */
/* ------------------------------------------------------------------------------------ */
/* crdt-enc/src/lib.rs:26 CURRENT_VERSION e834d789-101b-4634-9823-9de990a9051f */
static const uint8_t CORE_VERSION[16] = {0xe8, 0x34, 0xd7, 0x89, 0x10, 0x1b, 0x46, 0x34,
                                         0x98, 0x23, 0x9d, 0xe9, 0x90, 0xa9, 0x05, 0x1f};
/* crdt-enc-xchacha20poly1305/src/lib.rs:11 DATA_VERSION c7f269be-0ff5-4a77-99c3-7c23c96d5cb4 */
static const uint8_t BOX_VERSION[16] = {0xc7, 0xf2, 0x69, 0xbe, 0x0f, 0xf5, 0x4a, 0x77,
                                        0x99, 0xc3, 0x7c, 0x23, 0xc9, 0x6d, 0x5c, 0xb4};
/* crdt-enc-xchacha20poly1305/src/lib.rs:13 KEY_VERSION 5df28591-439a-4cef-8ca6-8433276cc9ed */
static const uint8_t KEY_VERSION[16] = {0x5d, 0xf2, 0x85, 0x91, 0x43, 0x9a, 0x4c, 0xef,
                                        0x8c, 0xa6, 0x84, 0x33, 0x27, 0x6c, 0xc9, 0xed};

static uint32_t ld32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static uint64_t ld64(const uint8_t *p) { return (uint64_t)ld32(p) | ((uint64_t)ld32(p + 4) << 32); }
static void st32(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
static void st64(uint8_t *p, uint64_t v) { st32(p, (uint32_t)v); st32(p + 4, (uint32_t)(v >> 32)); }

/* ------------------------------------------------------------------------------------ */
/* ChaCha20 / HChaCha20 (RFC 8439 §2.3, draft-irtf-cfrg-xchacha-03 §2.2)                 */
/* ------------------------------------------------------------------------------------ */
#define ROTL(v, c) (((v) << (c)) | ((v) >> (32 - (c))))
#define QR(a, b, c, d)                                                                       \
  a += b; d ^= a; d = ROTL(d, 16); c += d; b ^= c; b = ROTL(b, 12);                         \
  a += b; d ^= a; d = ROTL(d, 8);  c += d; b ^= c; b = ROTL(b, 7);

static void chacha_rounds(uint32_t x[16]) {
  for (int i = 0; i < 10; i++) {
    QR(x[0], x[4], x[8], x[12]); QR(x[1], x[5], x[9], x[13]);
    QR(x[2], x[6], x[10], x[14]); QR(x[3], x[7], x[11], x[15]);
    QR(x[0], x[5], x[10], x[15]); QR(x[1], x[6], x[11], x[12]);
    QR(x[2], x[7], x[8], x[13]); QR(x[3], x[4], x[9], x[14]);
  }
}

static void chacha_init(uint32_t s[16], const uint8_t key[32]) {
  s[0] = 0x61707865; s[1] = 0x3320646e; s[2] = 0x79622d32; s[3] = 0x6b206574;
  for (int i = 0; i < 8; i++) s[4 + i] = ld32(key + 4 * i);
}

void oc_chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce12[12],
                       uint8_t out[64]) {
  uint32_t s[16], x[16];
  chacha_init(s, key);
  s[12] = counter;
  s[13] = ld32(nonce12); s[14] = ld32(nonce12 + 4); s[15] = ld32(nonce12 + 8);
  memcpy(x, s, sizeof x);
  chacha_rounds(x);
  for (int i = 0; i < 16; i++) st32(out + 4 * i, x[i] + s[i]);
}

void oc_hchacha20(const uint8_t key[32], const uint8_t n16[16], uint8_t out[32]) {
  uint32_t x[16];
  chacha_init(x, key);
  for (int i = 0; i < 4; i++) x[12 + i] = ld32(n16 + 4 * i);
  chacha_rounds(x);
  for (int i = 0; i < 4; i++) st32(out + 4 * i, x[i]);
  for (int i = 0; i < 4; i++) st32(out + 16 + 4 * i, x[12 + i]);
}

static void chacha_xor(const uint8_t key[32], uint32_t counter, const uint8_t n12[12],
                       const uint8_t *in, uint8_t *out, size_t len) {
  uint8_t ks[64];
  for (size_t off = 0; off < len; off += 64, counter++) {
    oc_chacha20_block(key, counter, n12, ks);
    size_t m = len - off < 64 ? len - off : 64;
    for (size_t j = 0; j < m; j++) out[off + j] = in[off + j] ^ ks[j];
  }
}

/* ------------------------------------------------------------------------------------ */
/* Poly1305 (RFC 8439 §2.5), 44/44/42-bit limbs                                          */
/* ------------------------------------------------------------------------------------ */
typedef unsigned __int128 u128;
#define M44 0xfffffffffffULL
#define M42 0x3ffffffffffULL

typedef struct {
  uint64_t r0, r1, r2, s1, s2, h0, h1, h2, pad0, pad1;
  uint8_t buf[16];
  size_t nbuf;
} poly_st;

static void poly_init(poly_st *st, const uint8_t key[32]) {
  uint64_t t0 = ld64(key), t1 = ld64(key + 8);
  st->r0 = t0 & 0xffc0fffffffULL;
  st->r1 = ((t0 >> 44) | (t1 << 20)) & 0xfffffc0ffffULL;
  st->r2 = (t1 >> 24) & 0x00ffffffc0fULL;
  st->s1 = st->r1 * (5 << 2);
  st->s2 = st->r2 * (5 << 2);
  st->h0 = st->h1 = st->h2 = 0;
  st->pad0 = ld64(key + 16);
  st->pad1 = ld64(key + 24);
  st->nbuf = 0;
}

static void poly_block(poly_st *st, const uint8_t m[16], uint64_t hibit) {
  uint64_t t0 = ld64(m), t1 = ld64(m + 8);
  uint64_t h0 = st->h0 + (t0 & M44);
  uint64_t h1 = st->h1 + (((t0 >> 44) | (t1 << 20)) & M44);
  uint64_t h2 = st->h2 + (((t1 >> 24)) & M42) + hibit;
  u128 d0 = (u128)h0 * st->r0 + (u128)h1 * st->s2 + (u128)h2 * st->s1;
  u128 d1 = (u128)h0 * st->r1 + (u128)h1 * st->r0 + (u128)h2 * st->s2;
  u128 d2 = (u128)h0 * st->r2 + (u128)h1 * st->r1 + (u128)h2 * st->r0;
  uint64_t c;
  c = (uint64_t)(d0 >> 44); h0 = (uint64_t)d0 & M44;
  d1 += c; c = (uint64_t)(d1 >> 44); h1 = (uint64_t)d1 & M44;
  d2 += c; c = (uint64_t)(d2 >> 42); h2 = (uint64_t)d2 & M42;
  h0 += c * 5; c = h0 >> 44; h0 &= M44;
  h1 += c;
  st->h0 = h0; st->h1 = h1; st->h2 = h2;
}

static void poly_update(poly_st *st, const uint8_t *m, size_t len) {
  if (st->nbuf) {
    size_t want = 16 - st->nbuf;
    if (want > len) want = len;
    memcpy(st->buf + st->nbuf, m, want);
    st->nbuf += want; m += want; len -= want;
    if (st->nbuf < 16) return;
    poly_block(st, st->buf, 1ULL << 40);
    st->nbuf = 0;
  }
  while (len >= 16) { poly_block(st, m, 1ULL << 40); m += 16; len -= 16; }
  if (len) { memcpy(st->buf, m, len); st->nbuf = len; }
}

static void poly_finish(poly_st *st, uint8_t tag[16]) {
  if (st->nbuf) { /* generic Poly1305 final partial block: append 0x01 then zeros */
    st->buf[st->nbuf] = 1;
    for (size_t i = st->nbuf + 1; i < 16; i++) st->buf[i] = 0;
    poly_block(st, st->buf, 0);
  }
  uint64_t h0 = st->h0, h1 = st->h1, h2 = st->h2, c;
  c = h1 >> 44; h1 &= M44; h2 += c;
  c = h2 >> 42; h2 &= M42; h0 += c * 5;
  c = h0 >> 44; h0 &= M44; h1 += c;
  c = h1 >> 44; h1 &= M44; h2 += c;
  c = h2 >> 42; h2 &= M42; h0 += c * 5;
  c = h0 >> 44; h0 &= M44; h1 += c;
  uint64_t g0 = h0 + 5; c = g0 >> 44; g0 &= M44;
  uint64_t g1 = h1 + c; c = g1 >> 44; g1 &= M44;
  uint64_t g2 = h2 + c - (1ULL << 42);
  uint64_t mask = (g2 >> 63) - 1; /* g2 >= 0 -> all ones -> take g */
  h0 = (h0 & ~mask) | (g0 & mask);
  h1 = (h1 & ~mask) | (g1 & mask);
  h2 = (h2 & ~mask) | (g2 & mask);
  uint64_t t0 = st->pad0, t1 = st->pad1;
  h0 += t0 & M44; c = h0 >> 44; h0 &= M44;
  h1 += (((t0 >> 44) | (t1 << 20)) & M44) + c; c = h1 >> 44; h1 &= M44;
  h2 += ((t1 >> 24) & M42) + c; h2 &= M42;
  st64(tag, h0 | (h1 << 44));
  st64(tag + 8, (h1 >> 20) | (h2 << 24));
}

void oc_poly1305(const uint8_t key[32], const uint8_t *msg, size_t len, uint8_t tag[16]) {
  poly_st st;
  poly_init(&st, key);
  poly_update(&st, msg, len);
  poly_finish(&st, tag);
}

/* ------------------------------------------------------------------------------------ */
/* XChaCha20-Poly1305 (empty AAD)                                                        */
/* ------------------------------------------------------------------------------------ */
static void aead_mac_aad(const uint8_t polykey[32], const uint8_t *aad, size_t aad_len,
                         const uint8_t *ct, size_t len, uint8_t tag[16]) {
  static const uint8_t zeros[16] = {0};
  uint8_t lens[16];
  poly_st st;
  poly_init(&st, polykey);
  poly_update(&st, aad, aad_len);
  if (aad_len % 16) poly_update(&st, zeros, 16 - aad_len % 16);
  poly_update(&st, ct, len);
  if (len % 16) poly_update(&st, zeros, 16 - len % 16);
  st64(lens, (uint64_t)aad_len);
  st64(lens + 8, (uint64_t)len);
  poly_update(&st, lens, 16);
  poly_finish(&st, tag);
}
static void aead_mac(const uint8_t polykey[32], const uint8_t *ct, size_t len, uint8_t tag[16]) {
  aead_mac_aad(polykey, NULL, 0, ct, len, tag);
}

static void xchacha_keys(const uint8_t key[32], const uint8_t nonce[24], uint8_t subkey[32],
                         uint8_t n12[12], uint8_t polykey[32]) {
  uint8_t blk[64];
  oc_hchacha20(key, nonce, subkey);
  memset(n12, 0, 4);
  memcpy(n12 + 4, nonce + 16, 8);
  oc_chacha20_block(subkey, 0, n12, blk);
  memcpy(polykey, blk, 32);
}

void oc_xchacha_seal(const uint8_t key[32], const uint8_t nonce[24], const uint8_t *pt,
                     size_t len, uint8_t *out) {
  uint8_t subkey[32], n12[12], pk[32];
  xchacha_keys(key, nonce, subkey, n12, pk);
  chacha_xor(subkey, 1, n12, pt, out, len);
  aead_mac(pk, out, len, out + len);
}

void oc_xchacha_seal_aad(const uint8_t key[32], const uint8_t nonce[24], const uint8_t *aad,
                         size_t aad_len, const uint8_t *pt, size_t len, uint8_t *out) {
  uint8_t subkey[32], n12[12], pk[32];
  xchacha_keys(key, nonce, subkey, n12, pk);
  chacha_xor(subkey, 1, n12, pt, out, len);
  aead_mac_aad(pk, aad, aad_len, out, len, out + len);
}

int oc_xchacha_open(const uint8_t key[32], const uint8_t nonce[24], const uint8_t *ct,
                    size_t ct_len, uint8_t *out) {
  uint8_t subkey[32], n12[12], pk[32], tag[16];
  if (ct_len < 16) return OC_ERR_AUTH;
  size_t len = ct_len - 16;
  xchacha_keys(key, nonce, subkey, n12, pk);
  aead_mac(pk, ct, len, tag);
  uint8_t diff = 0;
  for (int i = 0; i < 16; i++) diff |= (uint8_t)(tag[i] ^ ct[len + i]);
  if (diff) return OC_ERR_AUTH;
  chacha_xor(subkey, 1, n12, ct, out, len);
  return OC_OK;
}

/* ------------------------------------------------------------------------------------ */
/* SHA3-256 (FIPS 202) + BASE32_NOPAD (RFC 4648)                                         */
/* ------------------------------------------------------------------------------------ */
static const uint64_t KRC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
    0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
static const int KROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                             25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};

static uint64_t rol64(uint64_t v, int c) { return c ? (v << c) | (v >> (64 - c)) : v; }

static void keccak_f(uint64_t a[25]) {
  for (int round = 0; round < 24; round++) {
    uint64_t c[5], b[25];
    for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
    for (int x = 0; x < 5; x++) {
      uint64_t d = c[(x + 4) % 5] ^ rol64(c[(x + 1) % 5], 1);
      for (int y = 0; y < 25; y += 5) a[x + y] ^= d;
    }
    for (int x = 0; x < 5; x++)
      for (int y = 0; y < 5; y++) b[y + 5 * ((2 * x + 3 * y) % 5)] = rol64(a[x + 5 * y], KROT[x + 5 * y]);
    for (int y = 0; y < 25; y += 5)
      for (int x = 0; x < 5; x++) a[x + y] = b[x + y] ^ (~b[(x + 1) % 5 + y] & b[(x + 2) % 5 + y]);
    a[0] ^= KRC[round];
  }
}

void oc_sha3_256(const uint8_t *msg, size_t len, uint8_t out[32]) {
  uint64_t a[25] = {0};
  const size_t rate = 136;
  uint8_t blk[136];
  while (len >= rate) {
    for (size_t i = 0; i < rate / 8; i++) a[i] ^= ld64(msg + 8 * i);
    keccak_f(a);
    msg += rate; len -= rate;
  }
  memset(blk, 0, rate);
  memcpy(blk, msg, len);
  blk[len] ^= 0x06;
  blk[rate - 1] ^= 0x80;
  for (size_t i = 0; i < rate / 8; i++) a[i] ^= ld64(blk + 8 * i);
  keccak_f(a);
  for (int i = 0; i < 4; i++) st64(out + 8 * i, a[i]);
}

size_t oc_base32_nopad(const uint8_t *in, size_t len, char *out) {
  static const char AL[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZ234567";
  size_t o = 0;
  uint32_t acc = 0;
  int bits = 0;
  for (size_t i = 0; i < len; i++) {
    acc = (acc << 8) | in[i];
    bits += 8;
    while (bits >= 5) { out[o++] = AL[(acc >> (bits - 5)) & 31]; bits -= 5; }
  }
  if (bits > 0) out[o++] = AL[(acc << (5 - bits)) & 31];
  out[o] = 0;
  return o;
}

/* ------------------------------------------------------------------------------------ */
/* msgpack reader -- rmp-serde 1.x from_slice acceptance rules    */
/* ------------------------------------------------------------------------------------ */
typedef struct {
  const uint8_t *p;
  size_t n, i;
} rd_t;

static int rd_take(rd_t *r, size_t k, const uint8_t **out) {
  if (r->n - r->i < k) return -1;
  *out = r->p + r->i;
  r->i += k;
  return 0;
}
static int rd_be(rd_t *r, int k, uint64_t *v) {
  const uint8_t *q;
  if (rd_take(r, (size_t)k, &q)) return -1;
  uint64_t x = 0;
  for (int j = 0; j < k; j++) x = (x << 8) | q[j];
  *v = x;
  return 0;
}

/* skip one value of any type (serde IgnoredAny) */
static int rd_skip(rd_t *r, int depth) {
  const uint8_t *q;
  uint64_t len;
  if (depth > 1024) return -1;
  if (rd_take(r, 1, &q)) return -1;
  uint8_t m = q[0];
  if (m <= 0x7f || m >= 0xe0 || m == 0xc0 || m == 0xc2 || m == 0xc3) return 0;
  if ((m & 0xf0) == 0x80 || (m & 0xf0) == 0x90) {
    uint64_t cnt = (uint64_t)(m & 0x0f) * (((m & 0xf0) == 0x80) ? 2 : 1);
    for (uint64_t k = 0; k < cnt; k++)
      if (rd_skip(r, depth + 1)) return -1;
    return 0;
  }
  if ((m & 0xe0) == 0xa0) return rd_take(r, m & 0x1f, &q);
  switch (m) {
    case 0xc4: case 0xd9: if (rd_be(r, 1, &len)) return -1; return rd_take(r, len, &q);
    case 0xc5: case 0xda: if (rd_be(r, 2, &len)) return -1; return rd_take(r, len, &q);
    case 0xc6: case 0xdb: if (rd_be(r, 4, &len)) return -1; return rd_take(r, len, &q);
    case 0xcc: case 0xd0: return rd_take(r, 1, &q);
    case 0xcd: case 0xd1: return rd_take(r, 2, &q);
    case 0xce: case 0xd2: case 0xca: return rd_take(r, 4, &q);
    case 0xcf: case 0xd3: case 0xcb: return rd_take(r, 8, &q);
    case 0xd4: return rd_take(r, 2, &q);
    case 0xd5: return rd_take(r, 3, &q);
    case 0xd6: return rd_take(r, 5, &q);
    case 0xd7: return rd_take(r, 9, &q);
    case 0xd8: return rd_take(r, 17, &q);
    case 0xc7: if (rd_be(r, 1, &len)) return -1; return rd_take(r, len + 1, &q);
    case 0xc8: if (rd_be(r, 2, &len)) return -1; return rd_take(r, len + 1, &q);
    case 0xc9: if (rd_be(r, 4, &len)) return -1; return rd_take(r, len + 1, &q);
    case 0xdc: case 0xdd: case 0xde: case 0xdf: {
      if (rd_be(r, (m == 0xdc || m == 0xde) ? 2 : 4, &len)) return -1;
      uint64_t cnt = len * ((m >= 0xde) ? 2 : 1);
      for (uint64_t k = 0; k < cnt; k++)
        if (rd_skip(r, depth + 1)) return -1;
      return 0;
    }
    default: return -1; /* 0xc1 never used */
  }
}

/* serde u64 visitor: any msgpack integer that is >= 0 */
static int rd_u64(rd_t *r, uint64_t *v) {
  const uint8_t *q;
  uint64_t x;
  if (rd_take(r, 1, &q)) return -1;
  uint8_t m = q[0];
  if (m <= 0x7f) { *v = m; return 0; }
  if (m >= 0xe0) return -1; /* negative fixint */
  switch (m) {
    case 0xcc: return rd_be(r, 1, v);
    case 0xcd: return rd_be(r, 2, v);
    case 0xce: return rd_be(r, 4, v);
    case 0xcf: return rd_be(r, 8, v);
    case 0xd0: if (rd_be(r, 1, &x)) return -1; if (x & 0x80) return -1; *v = x; return 0;
    case 0xd1: if (rd_be(r, 2, &x)) return -1; if (x & 0x8000) return -1; *v = x; return 0;
    case 0xd2: if (rd_be(r, 4, &x)) return -1; if (x & 0x80000000ULL) return -1; *v = x; return 0;
    case 0xd3: if (rd_be(r, 8, &x)) return -1; if (x >> 63) return -1; *v = x; return 0;
    default: return -1;
  }
}

/* array header (fixarray/array16/array32) */
static int rd_array_hdr(rd_t *r, uint64_t *len) {
  const uint8_t *q;
  if (rd_take(r, 1, &q)) return -1;
  uint8_t m = q[0];
  if ((m & 0xf0) == 0x90) { *len = m & 0x0f; return 0; }
  if (m == 0xdc) return rd_be(r, 2, len);
  if (m == 0xdd) return rd_be(r, 4, len);
  return -1;
}

static int utf8_valid(const uint8_t *s, size_t n) {
  size_t i = 0;
  while (i < n) {
    uint8_t c = s[i];
    if (c < 0x80) { i++; continue; }
    int k;
    uint32_t cp;
    if ((c & 0xe0) == 0xc0) { k = 1; cp = c & 0x1f; }
    else if ((c & 0xf0) == 0xe0) { k = 2; cp = c & 0x0f; }
    else if ((c & 0xf8) == 0xf0) { k = 3; cp = c & 0x07; }
    else return 0;
    for (int j = 1; j <= k; j++) {
      if (i + j >= n || (s[i + j] & 0xc0) != 0x80) return 0;
      cp = (cp << 6) | (s[i + j] & 0x3f);
    }
    if ((k == 1 && cp < 0x80) || (k == 2 && cp < 0x800) || (k == 3 && cp < 0x10000)) return 0;
    if (cp > 0x10ffff || (cp >= 0xd800 && cp <= 0xdfff)) return 0;
    i += (size_t)k + 1;
  }
  return 1;
}

/* bin / str header: returns kind 1=bin 2=str, payload pointer+len */
static int rd_binstr(rd_t *r, int *kind, const uint8_t **data, size_t *len) {
  const uint8_t *q;
  uint64_t l;
  if (rd_take(r, 1, &q)) return -1;
  uint8_t m = q[0];
  if ((m & 0xe0) == 0xa0) { l = m & 0x1f; *kind = 2; }
  else if (m == 0xc4 || m == 0xd9) { if (rd_be(r, 1, &l)) return -1; *kind = m == 0xc4 ? 1 : 2; }
  else if (m == 0xc5 || m == 0xda) { if (rd_be(r, 2, &l)) return -1; *kind = m == 0xc5 ? 1 : 2; }
  else if (m == 0xc6 || m == 0xdb) { if (rd_be(r, 4, &l)) return -1; *kind = m == 0xc6 ? 1 : 2; }
  else return -1;
  if (rd_take(r, l, data)) return -1;
  *len = (size_t)l;
  return 0;
}

/* Uuid (non-human-readable): deserialize_bytes with a visitor that only has visit_bytes:
 * bin of exactly 16 bytes, or a str that is not valid UTF-8 (rmp-serde hands it over as
 * bytes) of exactly 16 bytes. */
static int rd_uuid(rd_t *r, uint8_t out[16]) {
  int kind;
  const uint8_t *d;
  size_t l;
  if (rd_binstr(r, &kind, &d, &l)) return -1;
  if (kind == 2 && utf8_valid(d, l)) return -1;
  if (l != 16) return -1;
  memcpy(out, d, 16);
  return 0;
}

/* serde_bytes Cow<[u8]>: bin, str (any), or array of u8.  Array form is copied into *own
 * (malloc'd, caller frees). */
static int rd_bytes(rd_t *r, const uint8_t **data, size_t *len, uint8_t **own) {
  *own = NULL;
  if (r->i >= r->n) return -1;
  uint8_t m = r->p[r->i];
  if ((m & 0xf0) == 0x90 || m == 0xdc || m == 0xdd) {
    uint64_t cnt, v;
    if (rd_array_hdr(r, &cnt)) return -1;
    if (cnt > r->n) return -1;
    uint8_t *buf = (uint8_t *)malloc(cnt ? cnt : 1);
    for (uint64_t k = 0; k < cnt; k++) {
      if (rd_u64(r, &v) || v > 255) { free(buf); return -1; }
      buf[k] = (uint8_t)v;
    }
    *own = buf; *data = buf; *len = (size_t)cnt;
    return 0;
  }
  int kind;
  return rd_binstr(r, &kind, data, len);
}

/* struct field identifier: returns field index, nf for "ignore", -1 on error */
static int rd_field(rd_t *r, const char *const *names, int nf) {
  if (r->i >= r->n) return -1;
  uint8_t m = r->p[r->i];
  if ((m & 0xe0) == 0xa0 || m == 0xc4 || m == 0xc5 || m == 0xc6 || m == 0xd9 || m == 0xda ||
      m == 0xdb) {
    int kind;
    const uint8_t *d;
    size_t l;
    if (rd_binstr(r, &kind, &d, &l)) return -1;
    for (int f = 0; f < nf; f++)
      if (strlen(names[f]) == l && memcmp(names[f], d, l) == 0) return f;
    return nf;
  }
  uint64_t v;
  if (rd_u64(r, &v)) return -1;
  return v < (uint64_t)nf ? (int)v : nf;
}

/* generic derive(Deserialize) struct reader: map (any key order, unknown keys ignored,
 * duplicates rejected) or array of exactly nf elements.  cb(field, r, ctx) reads one value. */
typedef int (*field_cb)(int field, rd_t *r, void *ctx);
static int rd_struct(rd_t *r, const char *const *names, int nf, field_cb cb, void *ctx) {
  const uint8_t *q;
  uint64_t cnt;
  if (r->i >= r->n) return -1;
  uint8_t m = r->p[r->i];
  if ((m & 0xf0) == 0x90 || m == 0xdc || m == 0xdd) {
    if (rd_array_hdr(r, &cnt)) return -1;
    if (cnt != (uint64_t)nf) return -1; /* too few: invalid_length; too many: LengthMismatch */
    for (int f = 0; f < nf; f++)
      if (cb(f, r, ctx)) return -1;
    return 0;
  }
  if (rd_take(r, 1, &q)) return -1;
  if ((m & 0xf0) == 0x80) cnt = m & 0x0f;
  else if (m == 0xde) { if (rd_be(r, 2, &cnt)) return -1; }
  else if (m == 0xdf) { if (rd_be(r, 4, &cnt)) return -1; }
  else return -1;
  unsigned seen = 0;
  for (uint64_t k = 0; k < cnt; k++) {
    int f = rd_field(r, names, nf);
    if (f < 0) return -1;
    if (f == nf) { if (rd_skip(r, 0)) return -1; continue; }
    if (seen & (1u << f)) return -1; /* duplicate_field */
    seen |= 1u << f;
    if (cb(f, r, ctx)) return -1;
  }
  if (seen != (1u << nf) - 1) return -1; /* missing_field */
  return 0;
}

/* ------------------------------------------------------------------------------------ */
/* msgpack writer (rmp-serde to_vec_named)                                              */
/* ------------------------------------------------------------------------------------ */
typedef struct {
  uint8_t *p;
  size_t cap, n;
} wr_t;
static void wr_put(wr_t *w, const void *d, size_t k) {
  if (w->p && w->n + k <= w->cap) memcpy(w->p + w->n, d, k);
  w->n += k;
}
static void wr_u8(wr_t *w, uint8_t v) { wr_put(w, &v, 1); }
static void wr_be(wr_t *w, uint64_t v, int k) {
  uint8_t b[8];
  for (int j = 0; j < k; j++) b[j] = (uint8_t)(v >> (8 * (k - 1 - j)));
  wr_put(w, b, (size_t)k);
}
static void wr_uint(wr_t *w, uint64_t v) {
  if (v <= 0x7f) wr_u8(w, (uint8_t)v);
  else if (v <= 0xff) { wr_u8(w, 0xcc); wr_be(w, v, 1); }
  else if (v <= 0xffff) { wr_u8(w, 0xcd); wr_be(w, v, 2); }
  else if (v <= 0xffffffffULL) { wr_u8(w, 0xce); wr_be(w, v, 4); }
  else { wr_u8(w, 0xcf); wr_be(w, v, 8); }
}
static void wr_str(wr_t *w, const char *s) {
  size_t l = strlen(s); /* all field names are < 32 bytes */
  wr_u8(w, (uint8_t)(0xa0 | l));
  wr_put(w, s, l);
}
static void wr_bin(wr_t *w, const uint8_t *d, size_t l) {
  if (l <= 0xff) { wr_u8(w, 0xc4); wr_be(w, l, 1); }
  else if (l <= 0xffff) { wr_u8(w, 0xc5); wr_be(w, l, 2); }
  else { wr_u8(w, 0xc6); wr_be(w, l, 4); }
  wr_put(w, d, l);
}
static void wr_map_hdr(wr_t *w, size_t n) {
  if (n <= 15) wr_u8(w, (uint8_t)(0x80 | n));
  else if (n <= 0xffff) { wr_u8(w, 0xde); wr_be(w, n, 2); }
  else { wr_u8(w, 0xdf); wr_be(w, n, 4); }
}

/* ------------------------------------------------------------------------------------ */
/* EncHandler encrypt / decrypt (crdt-enc-xchacha20poly1305/src/lib.rs:40-101)            */
/* ------------------------------------------------------------------------------------ */
static size_t bin_hdr_len(size_t l) { return l <= 0xff ? 2 : (l <= 0xffff ? 3 : 5); }

size_t oc_cryptor_sealed_len(size_t clear_len) {
  size_t ct = clear_len + 16;
  size_t encbox = 1 + 6 + 2 + 24 + 9 + bin_hdr_len(ct) + ct; /* 82 a5nonce c418 .. a8enc_data */
  return 1 + 2 + 16 + bin_hdr_len(encbox) + encbox;
}

int oc_cryptor_encrypt(const uint8_t key_version[16], const uint8_t *key, size_t key_len,
                       const uint8_t nonce[24], const uint8_t *clear, size_t clear_len,
                       uint8_t *out, size_t *out_len) {
  if (memcmp(key_version, KEY_VERSION, 16)) return OC_ERR_KEY_VERSION;
  if (key_len != 32) return OC_ERR_KEY_LEN;
  size_t ct_len = clear_len + 16;
  uint8_t *ct = (uint8_t *)malloc(ct_len);
  oc_xchacha_seal(key, nonce, clear, clear_len, ct);
  /* EncBox{nonce, enc_data} via to_vec_named (lib.rs:59-64) */
  wr_t eb = {NULL, 0, 0};
  size_t eb_len = 1 + 6 + 2 + 24 + 9 + bin_hdr_len(ct_len) + ct_len;
  uint8_t *ebuf = (uint8_t *)malloc(eb_len);
  eb.p = ebuf; eb.cap = eb_len;
  wr_map_hdr(&eb, 2);
  wr_str(&eb, "nonce"); wr_bin(&eb, nonce, 24);
  wr_str(&eb, "enc_data"); wr_bin(&eb, ct, ct_len);
  /* VersionBytesRef(DATA_VERSION, enc_box) -> array(2)[bin16, bin] (lib.rs:65-67) */
  wr_t w = {out, (size_t)-1, 0};
  wr_u8(&w, 0x92);
  wr_bin(&w, BOX_VERSION, 16);
  wr_bin(&w, ebuf, eb.n);
  *out_len = w.n;
  free(ct); free(ebuf);
  return OC_OK;
}

typedef struct {
  uint8_t ver[16];
  const uint8_t *content; size_t content_len; uint8_t *own;
} vbox_ctx;
static int vbox_cb(int f, rd_t *r, void *ctx) {
  vbox_ctx *v = (vbox_ctx *)ctx;
  if (f == 0) return rd_uuid(r, v->ver);
  return rd_bytes(r, &v->content, &v->content_len, &v->own);
}
typedef struct {
  const uint8_t *nonce; size_t nonce_len; uint8_t *own_n;
  const uint8_t *enc; size_t enc_len; uint8_t *own_e;
} encbox_ctx;
static int encbox_cb(int f, rd_t *r, void *ctx) {
  encbox_ctx *e = (encbox_ctx *)ctx;
  if (f == 0) { free(e->own_n); e->own_n = NULL; return rd_bytes(r, &e->nonce, &e->nonce_len, &e->own_n); }
  free(e->own_e); e->own_e = NULL;
  return rd_bytes(r, &e->enc, &e->enc_len, &e->own_e);
}

int oc_cryptor_decrypt(const uint8_t key_version[16], const uint8_t *key, size_t key_len,
                       const uint8_t *enc, size_t enc_len, uint8_t *out, size_t *out_len) {
  static const char *const VB_F[2] = {"0", "1"}; /* tuple struct: array form only */
  static const char *const EB_F[2] = {"nonce", "enc_data"};
  if (memcmp(key_version, KEY_VERSION, 16)) return OC_ERR_KEY_VERSION;
  if (key_len != 32) return OC_ERR_KEY_LEN;
  rd_t r = {enc, enc_len, 0};
  vbox_ctx vb = {{0}, NULL, 0, NULL};
  /* VersionBytesRef is a tuple struct: serde visit_seq only -> array of exactly 2 */
  if (r.n == 0 || !(((r.p[0] & 0xf0) == 0x90) || r.p[0] == 0xdc || r.p[0] == 0xdd) ||
      rd_struct(&r, VB_F, 2, vbox_cb, &vb)) {
    free(vb.own);
    return OC_ERR_PARSE_VBOX;
  }
  if (memcmp(vb.ver, BOX_VERSION, 16)) { free(vb.own); return OC_ERR_DATA_VERSION; }
  rd_t r2 = {vb.content, vb.content_len, 0};
  encbox_ctx eb = {NULL, 0, NULL, NULL, 0, NULL};
  if (rd_struct(&r2, EB_F, 2, encbox_cb, &eb)) {
    free(eb.own_n); free(eb.own_e); free(vb.own);
    return OC_ERR_PARSE_ENCBOX;
  }
  int st = OC_OK;
  if (eb.nonce_len != 24) st = OC_ERR_NONCE_LEN;
  else {
    st = oc_xchacha_open(key, eb.nonce, eb.enc, eb.enc_len, out);
    if (st == OC_OK) *out_len = eb.enc_len - 16;
  }
  free(eb.own_n); free(eb.own_e); free(vb.own);
  return st;
}

/* ------------------------------------------------------------------------------------ */
/* VClock (crdts 7): BTreeMap<Uuid, u64> as a sorted array                               */
/* ------------------------------------------------------------------------------------ */
void oc_vclock_init(oc_vclock *v) { memset(v, 0, sizeof *v); }
void oc_vclock_free(oc_vclock *v) { free(v->actor); free(v->counter); memset(v, 0, sizeof *v); }

static size_t vc_lower(const oc_vclock *v, const uint8_t a[16], int *found) {
  size_t lo = 0, hi = v->n;
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    int c = memcmp(v->actor[mid], a, 16);
    if (c < 0) lo = mid + 1; else hi = mid;
  }
  *found = lo < v->n && memcmp(v->actor[lo], a, 16) == 0;
  return lo;
}

uint64_t oc_vclock_get(const oc_vclock *v, const uint8_t actor[16]) {
  int f;
  size_t i = vc_lower(v, actor, &f);
  return f ? v->counter[i] : 0;
}

/* VClock::apply(Dot): insert when get(actor) < counter */
void oc_vclock_apply(oc_vclock *v, const uint8_t actor[16], uint64_t counter) {
  int f;
  size_t i = vc_lower(v, actor, &f);
  if (f) { if (v->counter[i] < counter) v->counter[i] = counter; return; }
  if (counter == 0) return;
  if (v->n == v->cap) {
    v->cap = v->cap ? 2 * v->cap : 64;
    v->actor = (uint8_t (*)[16])realloc(v->actor, v->cap * 16);
    v->counter = (uint64_t *)realloc(v->counter, v->cap * 8);
  }
  memmove(v->actor + i + 1, v->actor + i, (v->n - i) * 16);
  memmove(v->counter + i + 1, v->counter + i, (v->n - i) * 8);
  memcpy(v->actor[i], actor, 16);
  v->counter[i] = counter;
  v->n++;
}

void oc_core_init(oc_core *c, int kind) {
  c->kind = kind;
  oc_vclock_init(&c->next_op_versions);
  oc_vclock_init(&c->state);
}
void oc_core_free(oc_core *c) { oc_vclock_free(&c->next_op_versions); oc_vclock_free(&c->state); }

static void wr_vclock(wr_t *w, const oc_vclock *v) {
  wr_map_hdr(w, 1);
  wr_str(w, "dots");
  wr_map_hdr(w, v->n);
  for (size_t i = 0; i < v->n; i++) { wr_bin(w, v->actor[i], 16); wr_uint(w, v->counter[i]); }
}

size_t oc_core_serialize(const oc_core *c, uint8_t *out, size_t cap) {
  wr_t w = {out, cap, 0};
  wr_map_hdr(&w, 2);
  wr_str(&w, "next_op_versions");
  wr_vclock(&w, &c->next_op_versions);
  wr_str(&w, "state");
  if (c->kind == OC_STATE_GCOUNTER) { wr_map_hdr(&w, 1); wr_str(&w, "inner"); }
  wr_vclock(&w, &c->state);
  return w.n;
}

/* --- VClock / GCounter / StateWrapper deserialize+merge --- */
static int vc_dots_cb(int f, rd_t *r, void *ctx) {
  (void)f;
  oc_vclock *v = (oc_vclock *)ctx;
  const uint8_t *q;
  uint64_t cnt;
  if (r->i >= r->n) return -1;
  uint8_t m = r->p[r->i];
  if ((m & 0xf0) == 0x80) { r->i++; cnt = m & 0x0f; }
  else if (m == 0xde) { r->i++; if (rd_be(r, 2, &cnt)) return -1; }
  else if (m == 0xdf) { r->i++; if (rd_be(r, 4, &cnt)) return -1; }
  else return -1;
  (void)q;
  /* BTreeMap: later duplicate keys overwrite earlier ones (last wins) before the merge */
  oc_vclock tmp;
  oc_vclock_init(&tmp);
  for (uint64_t k = 0; k < cnt; k++) {
    uint8_t a[16];
    uint64_t ctr;
    if (rd_uuid(r, a) || rd_u64(r, &ctr)) { oc_vclock_free(&tmp); return -1; }
    int f2;
    size_t i = vc_lower(&tmp, a, &f2);
    if (f2) tmp.counter[i] = ctr;
    else if (ctr == 0) {
      /* keep explicit zero entries out: VClock::merge applies them as no-ops */
    } else oc_vclock_apply(&tmp, a, ctr);
  }
  for (size_t i = 0; i < tmp.n; i++) oc_vclock_apply(v, tmp.actor[i], tmp.counter[i]);
  oc_vclock_free(&tmp);
  return 0;
}
static int rd_vclock_merge(rd_t *r, oc_vclock *v) {
  static const char *const F[1] = {"dots"};
  return rd_struct(r, F, 1, vc_dots_cb, v);
}
static int gc_inner_cb(int f, rd_t *r, void *ctx) { (void)f; return rd_vclock_merge(r, (oc_vclock *)ctx); }

typedef struct { oc_core *tmp; } sw_ctx;
static int sw_cb(int f, rd_t *r, void *ctx) {
  oc_core *c = ((sw_ctx *)ctx)->tmp;
  static const char *const GF[1] = {"inner"};
  if (f == 0) return rd_vclock_merge(r, &c->next_op_versions);
  if (c->kind == OC_STATE_GCOUNTER) return rd_struct(r, GF, 1, gc_inner_cb, &c->state);
  return rd_vclock_merge(r, &c->state);
}

int oc_core_merge_serialized(oc_core *c, const uint8_t *buf, size_t len) {
  static const char *const F[2] = {"next_op_versions", "state"};
  oc_core tmp;
  oc_core_init(&tmp, c->kind);
  sw_ctx ctx = {&tmp};
  rd_t r = {buf, len, 0};
  if (rd_struct(&r, F, 2, sw_cb, &ctx)) { oc_core_free(&tmp); return OC_ERR_DECODE; }
  /* lib.rs:460-463: state.merge(sw.state); next_op_versions.merge(sw.next_op_versions) */
  for (size_t i = 0; i < tmp.state.n; i++) oc_vclock_apply(&c->state, tmp.state.actor[i], tmp.state.counter[i]);
  for (size_t i = 0; i < tmp.next_op_versions.n; i++)
    oc_vclock_apply(&c->next_op_versions, tmp.next_op_versions.actor[i], tmp.next_op_versions.counter[i]);
  oc_core_free(&tmp);
  return OC_OK;
}

/* --- Vec<Dot<Uuid>> --- */
typedef struct { uint8_t actor[16]; uint64_t counter; } dot_t;
static int dot_cb(int f, rd_t *r, void *ctx) {
  dot_t *d = (dot_t *)ctx;
  if (f == 0) return rd_uuid(r, d->actor);
  return rd_u64(r, &d->counter);
}

int oc_decode_apply_dots(oc_core *c, const uint8_t *buf, size_t len, int dry_run) {
  static const char *const F[2] = {"actor", "counter"};
  rd_t r = {buf, len, 0};
  uint64_t cnt;
  if (rd_array_hdr(&r, &cnt)) return OC_ERR_DECODE;
  if (cnt > len) return OC_ERR_DECODE;
  /* decode everything first (rmp_serde::from_slice returns the whole Vec or an error),
   * then apply in order */
  dot_t stackbuf[256];
  dot_t *dots = cnt <= 256 ? stackbuf : (dot_t *)malloc(cnt * sizeof(dot_t));
  for (uint64_t k = 0; k < cnt; k++) {
    if (rd_struct(&r, F, 2, dot_cb, &dots[k])) {
      if (dots != stackbuf) free(dots);
      return OC_ERR_DECODE;
    }
  }
  if (!dry_run)
    for (uint64_t k = 0; k < cnt; k++) oc_vclock_apply(&c->state, dots[k].actor, dots[k].counter);
  if (dots != stackbuf) free(dots);
  return OC_OK;
}

/* ------------------------------------------------------------------------------------ */
/* Core::read_remote_ops / read_remote_states                                            */
/* ------------------------------------------------------------------------------------ */
static int version_supported(const uint8_t v[16], const uint8_t (*sup)[16], size_t n) {
  for (size_t i = 0; i < n; i++)
    if (memcmp(v, sup[i], 16) == 0) return 1;
  return 0;
}

/* open one file: outer version, cryptor decrypt, inner data version.  On success pt, pt_len
 * point at the msgpack payload inside buf (caller-provided, >= file length). */
static int open_file(const uint8_t key_version[16], const uint8_t *key, size_t key_len,
                     const uint8_t (*sup)[16], size_t n_sup, const uint8_t *file, size_t flen,
                     uint8_t *buf, const uint8_t **pt, size_t *pt_len) {
  if (flen < 16) return OC_ERR_OUTER_LEN;
  if (memcmp(file, CORE_VERSION, 16)) return OC_ERR_OUTER_VERSION;
  size_t clen = 0;
  int st = oc_cryptor_decrypt(key_version, key, key_len, file + 16, flen - 16, buf, &clen);
  if (st) return st;
  if (clen < 16) return OC_ERR_PT_LEN;
  if (!version_supported(buf, sup, n_sup)) return OC_ERR_PT_VERSION;
  *pt = buf + 16;
  *pt_len = clen - 16;
  return OC_OK;
}

int oc_read_remote_ops(oc_core *c, const uint8_t key_version[16], const uint8_t *key,
                       size_t key_len, const uint8_t (*supported)[16], size_t n_supported,
                       const uint8_t *blob, const uint64_t *offs, const uint8_t (*file_actor)[16],
                       const uint64_t *file_version, size_t n_files, int32_t *status) {
  int first_err = OC_OK;
  uint8_t **pts = (uint8_t **)calloc(n_files ? n_files : 1, sizeof *pts);
  size_t *pt_lens = (size_t *)calloc(n_files ? n_files : 1, sizeof *pt_lens);
  /* phase 1 (lib.rs:497-514): open + decode every file, in order */
  for (size_t i = 0; i < n_files; i++) {
    size_t flen = offs[i + 1] - offs[i];
    uint8_t *buf = (uint8_t *)malloc(flen + 1);
    const uint8_t *pt;
    size_t pl;
    int st = open_file(key_version, key, key_len, supported, n_supported, blob + offs[i], flen,
                       buf, &pt, &pl);
    if (st == OC_OK) st = oc_decode_apply_dots(c, pt, pl, 1);
    status[i] = st;
    if (st == OC_OK) { pts[i] = buf; memmove(buf, pt, pl); pt_lens[i] = pl; }
    else { free(buf); if (first_err == OC_OK) first_err = st; }
  }
  if (first_err == OC_OK) {
    /* phase 2 (lib.rs:516-544): version gate + apply, under the lock.  An actor whose
     * next file is ahead of expected stops (error recorded) -- see DESIGN.md. */
    for (size_t i = 0; i < n_files; i++) {
      uint64_t expected = oc_vclock_get(&c->next_op_versions, file_actor[i]);
      if (file_version[i] < expected) continue;
      if (expected < file_version[i]) { /* lib.rs:527-531: return Err, fold stops here */
        status[i] = OC_ERR_OP_VERSION;
        first_err = OC_ERR_OP_VERSION;
        break;
      }
      oc_decode_apply_dots(c, pts[i], pt_lens[i], 0);
      oc_vclock_apply(&c->next_op_versions, file_actor[i], expected + 1);
    }
  }
  for (size_t i = 0; i < n_files; i++) free(pts[i]);
  free(pts); free(pt_lens);
  return first_err;
}

int oc_read_remote_states(oc_core *c, const uint8_t key_version[16], const uint8_t *key,
                          size_t key_len, const uint8_t (*supported)[16], size_t n_supported,
                          const uint8_t *blob, const uint64_t *offs, size_t n_files,
                          int32_t *status) {
  int first_err = OC_OK;
  oc_core acc;
  oc_core_init(&acc, c->kind);
  for (size_t i = 0; i < n_files; i++) {
    size_t flen = offs[i + 1] - offs[i];
    uint8_t *buf = (uint8_t *)malloc(flen + 1);
    const uint8_t *pt;
    size_t pl;
    int st = open_file(key_version, key, key_len, supported, n_supported, blob + offs[i], flen,
                       buf, &pt, &pl);
    if (st == OC_OK) st = oc_core_merge_serialized(&acc, pt, pl);
    status[i] = st;
    if (st && first_err == OC_OK) first_err = st;
    free(buf);
  }
  if (first_err == OC_OK) {
    for (size_t i = 0; i < acc.state.n; i++) oc_vclock_apply(&c->state, acc.state.actor[i], acc.state.counter[i]);
    for (size_t i = 0; i < acc.next_op_versions.n; i++)
      oc_vclock_apply(&c->next_op_versions, acc.next_op_versions.actor[i], acc.next_op_versions.counter[i]);
  }
  oc_core_free(&acc);
  return first_err;
}

/* ------------------------------------------------------------------------------------ */
/* multi-threaded CPU baseline                                                            */
/* ------------------------------------------------------------------------------------ */
typedef struct {
  const uint8_t *key, *blob;
  const uint64_t *offs;
  size_t n, next;
  int32_t *status;
  uint8_t **pts;
  size_t *pt_lens;
  pthread_mutex_t mu;
  const uint8_t *data_version;
} mt_job;

static void *mt_worker(void *arg) {
  mt_job *j = (mt_job *)arg;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    size_t lo = j->next;
    j->next += 64;
    pthread_mutex_unlock(&j->mu);
    if (lo >= j->n) break;
    size_t hi = lo + 64 < j->n ? lo + 64 : j->n;
    for (size_t i = lo; i < hi; i++) {
      size_t flen = j->offs[i + 1] - j->offs[i];
      uint8_t *buf = (uint8_t *)malloc(flen + 1);
      const uint8_t *pt;
      size_t pl;
      int st = open_file(KEY_VERSION, j->key, 32, (const uint8_t(*)[16])j->data_version, 1,
                         j->blob + j->offs[i], flen, buf, &pt, &pl);
      j->status[i] = st;
      if (j->pts && st == OC_OK) { memmove(buf, pt, pl); j->pts[i] = buf; j->pt_lens[i] = pl; }
      else free(buf);
    }
  }
  return NULL;
}

static void mt_run(mt_job *j, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  pthread_t th[256];
  if (n_threads > 256) n_threads = 256;
  pthread_mutex_init(&j->mu, NULL);
  for (int t = 0; t < n_threads; t++) pthread_create(&th[t], NULL, mt_worker, j);
  for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
  pthread_mutex_destroy(&j->mu);
}

size_t oc_open_batch_mt(const uint8_t key[32], const uint8_t data_version[16],
                        const uint8_t *blob, const uint64_t *offs, size_t n_files, int n_threads,
                        int32_t *status) {
  mt_job j;
  memset(&j, 0, sizeof j);
  j.data_version = data_version;
  j.key = key; j.blob = blob; j.offs = offs; j.n = n_files; j.status = status;
  mt_run(&j, n_threads);
  size_t ok = 0;
  for (size_t i = 0; i < n_files; i++) ok += status[i] == OC_OK;
  return ok;
}

size_t oc_compact_ops_baseline(int kind, const uint8_t key[32], const uint8_t data_version[16],
                               const uint8_t *blob, const uint64_t *offs,
                               const uint8_t (*file_actor)[16], const uint64_t *file_version,
                               size_t n_files, int n_threads, uint8_t *out, size_t cap,
                               int *err) {
  mt_job j;
  memset(&j, 0, sizeof j);
  j.key = key; j.blob = blob; j.offs = offs; j.n = n_files; j.data_version = data_version;
  j.status = (int32_t *)calloc(n_files ? n_files : 1, sizeof(int32_t));
  j.pts = (uint8_t **)calloc(n_files ? n_files : 1, sizeof(uint8_t *));
  j.pt_lens = (size_t *)calloc(n_files ? n_files : 1, sizeof(size_t));
  mt_run(&j, n_threads);
  oc_core c;
  oc_core_init(&c, kind);
  int e = OC_OK;
  for (size_t i = 0; i < n_files && !e; i++)
    if (j.status[i]) e = j.status[i];
  for (size_t i = 0; i < n_files && !e; i++)
    if (oc_decode_apply_dots(&c, j.pts[i], j.pt_lens[i], 1)) e = OC_ERR_DECODE;
  size_t n_out = 0;
  if (!e) {
    for (size_t i = 0; i < n_files; i++) {
      uint64_t expected = oc_vclock_get(&c.next_op_versions, file_actor[i]);
      if (file_version[i] < expected) continue;
      if (expected < file_version[i]) { e = OC_ERR_OP_VERSION; break; }
      oc_decode_apply_dots(&c, j.pts[i], j.pt_lens[i], 0);
      oc_vclock_apply(&c.next_op_versions, file_actor[i], expected + 1);
    }
    n_out = oc_core_serialize(&c, out, cap);
  }
  for (size_t i = 0; i < n_files; i++) free(j.pts[i]);
  free(j.pts); free(j.pt_lens); free(j.status);
  oc_core_free(&c);
  *err = e;
  return n_out;
}

/* ---- best-CPU baseline: open/decode parallel over files, gate + fold parallel over actors -- */
typedef struct {
  mt_job *j;
  const uint8_t (*file_actor)[16];
  const uint64_t *file_version;
  int kind, t, n_threads;
  oc_core core;
  int err;
} best_fold;

static uint32_t actor_owner(const uint8_t a[16], int n) {
  uint32_t h = 2166136261u;
  for (int i = 0; i < 16; i++) h = (h ^ a[i]) * 16777619u;
  return h % (uint32_t)n;
}

static void *best_check_worker(void *arg) {  /* decode check (rmp_serde::from_slice, lib.rs:507) */
  best_fold *b = (best_fold *)arg;
  for (size_t i = (size_t)b->t; i < b->j->n; i += (size_t)b->n_threads)
    if (b->j->status[i] == OC_OK && oc_decode_apply_dots(&b->core, b->j->pts[i], b->j->pt_lens[i], 1))
      b->j->status[i] = OC_ERR_DECODE;
  return NULL;
}

static void *best_fold_worker(void *arg) {   /* lib.rs:516-544 for the actors this thread owns */
  best_fold *b = (best_fold *)arg;
  for (size_t i = 0; i < b->j->n && !b->err; i++) {
    if ((int)actor_owner(b->file_actor[i], b->n_threads) != b->t) continue;
    uint64_t expected = oc_vclock_get(&b->core.next_op_versions, b->file_actor[i]);
    if (b->file_version[i] < expected) continue;
    if (expected < b->file_version[i]) { b->err = OC_ERR_OP_VERSION; break; }
    oc_decode_apply_dots(&b->core, b->j->pts[i], b->j->pt_lens[i], 0);
    oc_vclock_apply(&b->core.next_op_versions, b->file_actor[i], expected + 1);
  }
  return NULL;
}

size_t oc_compact_ops_best(int kind, const uint8_t key[32], const uint8_t data_version[16],
                           const uint8_t *blob, const uint64_t *offs,
                           const uint8_t (*file_actor)[16], const uint64_t *file_version,
                           size_t n_files, int n_threads, uint8_t *out, size_t cap, int *err) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  mt_job j;
  memset(&j, 0, sizeof j);
  j.key = key; j.blob = blob; j.offs = offs; j.n = n_files; j.data_version = data_version;
  j.status = (int32_t *)calloc(n_files ? n_files : 1, sizeof(int32_t));
  j.pts = (uint8_t **)calloc(n_files ? n_files : 1, sizeof(uint8_t *));
  j.pt_lens = (size_t *)calloc(n_files ? n_files : 1, sizeof(size_t));
  mt_run(&j, n_threads);
  best_fold *bf = (best_fold *)calloc((size_t)n_threads, sizeof(best_fold));
  pthread_t th[256];
  for (int t = 0; t < n_threads; t++) {
    bf[t].j = &j; bf[t].file_actor = file_actor; bf[t].file_version = file_version;
    bf[t].kind = kind; bf[t].t = t; bf[t].n_threads = n_threads;
    oc_core_init(&bf[t].core, kind);
  }
  for (int t = 0; t < n_threads; t++) pthread_create(&th[t], NULL, best_check_worker, &bf[t]);
  for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
  int e = OC_OK;
  for (size_t i = 0; i < n_files && !e; i++)
    if (j.status[i]) e = j.status[i];
  size_t n_out = 0;
  oc_core c;
  oc_core_init(&c, kind);
  if (!e) {
    for (int t = 0; t < n_threads; t++) pthread_create(&th[t], NULL, best_fold_worker, &bf[t]);
    for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
    int gap = 0;
    for (int t = 0; t < n_threads; t++) gap |= bf[t].err;
    if (gap) {  /* sequential fold: stop at the gap in batch order */
      for (size_t i = 0; i < n_files; i++) {
        uint64_t expected = oc_vclock_get(&c.next_op_versions, file_actor[i]);
        if (file_version[i] < expected) continue;
        if (expected < file_version[i]) { e = OC_ERR_OP_VERSION; break; }
        oc_decode_apply_dots(&c, j.pts[i], j.pt_lens[i], 0);
        oc_vclock_apply(&c.next_op_versions, file_actor[i], expected + 1);
      }
    } else {
      for (int t = 0; t < n_threads; t++) {  /* VClock::merge of the private states */
        for (size_t i = 0; i < bf[t].core.state.n; i++)
          oc_vclock_apply(&c.state, bf[t].core.state.actor[i], bf[t].core.state.counter[i]);
        for (size_t i = 0; i < bf[t].core.next_op_versions.n; i++)
          oc_vclock_apply(&c.next_op_versions, bf[t].core.next_op_versions.actor[i],
                          bf[t].core.next_op_versions.counter[i]);
      }
    }
    if (!e) n_out = oc_core_serialize(&c, out, cap);
  }
  for (int t = 0; t < n_threads; t++) oc_core_free(&bf[t].core);
  free(bf);
  oc_core_free(&c);
  for (size_t i = 0; i < n_files; i++) free(j.pts[i]);
  free(j.pts); free(j.pt_lens); free(j.status);
  *err = e;
  return n_out;
}

/* ------------------------------------------------------------------------------------ */
/* Orswot<u64, Uuid> CPU baseline (C3): a C restatement of oracle/crdts.py's Orswot and  */
/* Core (crdts 7 orswot.rs; crdt-enc/src/lib.rs:401-547)           */
/* ------------------------------------------------------------------------------------ */
/* Data layout: actors interned to dense ids (first-seen order); the Orswot's own clock and
 * next_op_versions are dense arrays indexed by id (they never hold zero counters: every
 * insertion goes through VClock::apply); an entry's or a removal's VClock is a small array
 * sorted by id (it may hold explicit zero counters, as a decoded BTreeMap may); entries are an
 * open-addressed member -> VClock table; deferred removals a list of (clock, members). */
#include <time.h>

static double oc_now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

typedef struct { uint64_t *p; size_t n, cap; } u64v;
static void u64v_push(u64v *v, uint64_t x) {
  if (v->n == v->cap) {
    v->cap = v->cap ? 2 * v->cap : 64;
    v->p = (uint64_t *)realloc(v->p, v->cap * 8);
  }
  v->p[v->n++] = x;
}
static void u64v_free(u64v *v) { free(v->p); memset(v, 0, sizeof *v); }

static int rd_map_hdr(rd_t *r, uint64_t *len) {
  const uint8_t *q;
  if (rd_take(r, 1, &q)) return -1;
  uint8_t m = q[0];
  if ((m & 0xf0) == 0x80) { *len = m & 0x0f; return 0; }
  if (m == 0xde) return rd_be(r, 2, len);
  if (m == 0xdf) return rd_be(r, 4, len);
  return -1;
}

/* --- raw (uuid-keyed) decode, run on the worker threads ---------------------------------- */
/* VClock {dots: BTreeMap<Uuid, u64>} (crdts.py dec_vclock): a later duplicate key overwrites an
 * earlier one, zero counters kept.  Appends [n, (uuid lo, uuid hi, counter) x n]. */
typedef struct { uint8_t a[16]; uint64_t c; uint32_t ord; } rawdot;
static int rawdot_cmp(const void *x, const void *y) {
  const rawdot *p = (const rawdot *)x, *q = (const rawdot *)y;
  int c = memcmp(p->a, q->a, 16);
  if (c) return c;
  return p->ord < q->ord ? -1 : p->ord > q->ord;
}
typedef struct { u64v *out; rawdot *tmp; size_t tcap; } vcraw_ctx;
static int vcraw_dots_cb(int f, rd_t *r, void *ctx) {
  (void)f;
  vcraw_ctx *x = (vcraw_ctx *)ctx;
  uint64_t cnt;
  if (rd_map_hdr(r, &cnt) || cnt > r->n - r->i) return -1;
  if (cnt > x->tcap) {
    x->tcap = cnt;
    x->tmp = (rawdot *)realloc(x->tmp, cnt * sizeof(rawdot));
  }
  for (uint64_t k = 0; k < cnt; k++) {
    if (rd_uuid(r, x->tmp[k].a) || rd_u64(r, &x->tmp[k].c)) return -1;
    x->tmp[k].ord = (uint32_t)k;
  }
  size_t n = (size_t)cnt;
  if (n > 1) {
    qsort(x->tmp, n, sizeof(rawdot), rawdot_cmp);
    size_t w = 0;
    for (size_t k = 0; k < n; k++) {
      if (k + 1 < n && memcmp(x->tmp[k].a, x->tmp[k + 1].a, 16) == 0) continue;  /* last wins */
      x->tmp[w++] = x->tmp[k];
    }
    n = w;
  }
  u64v_push(x->out, n);
  for (size_t k = 0; k < n; k++) {
    uint64_t lo, hi;
    memcpy(&lo, x->tmp[k].a, 8);
    memcpy(&hi, x->tmp[k].a + 8, 8);
    u64v_push(x->out, lo);
    u64v_push(x->out, hi);
    u64v_push(x->out, x->tmp[k].c);
  }
  return 0;
}
static int rd_vcraw(rd_t *r, vcraw_ctx *x, u64v *out) {
  static const char *const F[1] = {"dots"};
  x->out = out;
  return rd_struct(r, F, 1, vcraw_dots_cb, x);
}

static int rd_members(rd_t *r, u64v *out) {  /* Vec<u64> (crdts.py _seq + _u64) */
  uint64_t cnt, m;
  if (rd_array_hdr(r, &cnt) || cnt > r->n - r->i) return -1;
  u64v_push(out, cnt);
  for (uint64_t k = 0; k < cnt; k++) {
    if (rd_u64(r, &m)) return -1;
    u64v_push(out, m);
  }
  return 0;
}

/* StateWrapper<Orswot> (crdts.py dec_state): four raw sections, each in wire order */
typedef struct { u64v nov, clk, ent, def; } ow_raw;
typedef struct { vcraw_ctx vc; ow_raw *s; } ow_rawctx;
static int ow_set_cb(int f, rd_t *r, void *ctx) {
  ow_rawctx *x = (ow_rawctx *)ctx;
  uint64_t cnt, m;
  if (f == 0) return rd_vcraw(r, &x->vc, &x->s->clk);
  if (rd_map_hdr(r, &cnt) || cnt > r->n - r->i) return -1;
  u64v *o = f == 1 ? &x->s->ent : &x->s->def;
  u64v_push(o, cnt);
  for (uint64_t k = 0; k < cnt; k++) {
    if (f == 1) {          /* entries: member -> VClock */
      if (rd_u64(r, &m)) return -1;
      u64v_push(o, m);
      if (rd_vcraw(r, &x->vc, o)) return -1;
    } else {               /* deferred: VClock -> Vec<member> */
      if (rd_vcraw(r, &x->vc, o) || rd_members(r, o)) return -1;
    }
  }
  return 0;
}
static int ow_sw_cb(int f, rd_t *r, void *ctx) {
  static const char *const F[3] = {"clock", "entries", "deferred"};
  ow_rawctx *x = (ow_rawctx *)ctx;
  if (f == 0) return rd_vcraw(r, &x->vc, &x->s->nov);
  return rd_struct(r, F, 3, ow_set_cb, x);
}
static int ow_decode_state(const uint8_t *pt, size_t len, ow_rawctx *x) {
  static const char *const F[2] = {"next_op_versions", "state"};
  rd_t r = {pt, len, 0};
  return rd_struct(&r, F, 2, ow_sw_cb, x);
}

/* Vec<orswot::Op<u64, Uuid>> (crdts.py dec_orswot_op): externally tagged {"Add": {dot, members}}
 * | {"Rm": {clock, members}} -> [0, uuid lo, uuid hi, counter, nm, m..] | [1, <vc>, nm, m..] */
typedef struct { vcraw_ctx vc; dot_t dot; u64v clk, mem; } ow_opctx;
static int ow_add_cb(int f, rd_t *r, void *ctx) {
  static const char *const DF[2] = {"actor", "counter"};
  ow_opctx *x = (ow_opctx *)ctx;
  if (f == 0) return rd_struct(r, DF, 2, dot_cb, &x->dot);
  x->mem.n = 0;
  return rd_members(r, &x->mem);
}
static int ow_rm_cb(int f, rd_t *r, void *ctx) {
  ow_opctx *x = (ow_opctx *)ctx;
  if (f == 0) { x->clk.n = 0; return rd_vcraw(r, &x->vc, &x->clk); }
  x->mem.n = 0;
  return rd_members(r, &x->mem);
}
static int ow_decode_ops(const uint8_t *pt, size_t len, ow_opctx *x, u64v *out) {
  static const char *const V[2] = {"Add", "Rm"};
  static const char *const AF[2] = {"dot", "members"};
  static const char *const RF[2] = {"clock", "members"};
  rd_t r = {pt, len, 0};
  uint64_t cnt, one;
  if (rd_array_hdr(&r, &cnt) || cnt > len) return -1;
  for (uint64_t k = 0; k < cnt; k++) {
    if (rd_map_hdr(&r, &one) || one != 1) return -1;
    int v = rd_field(&r, V, 2);
    if (v < 0 || v >= 2) return -1;
    if (v == 0) {
      if (rd_struct(&r, AF, 2, ow_add_cb, x)) return -1;
      uint64_t lo, hi;
      memcpy(&lo, x->dot.actor, 8);
      memcpy(&hi, x->dot.actor + 8, 8);
      u64v_push(out, 0); u64v_push(out, lo); u64v_push(out, hi); u64v_push(out, x->dot.counter);
    } else {
      if (rd_struct(&r, RF, 2, ow_rm_cb, x)) return -1;
      u64v_push(out, 1);
      for (size_t i = 0; i < x->clk.n; i++) u64v_push(out, x->clk.p[i]);
    }
    for (size_t i = 0; i < x->mem.n; i++) u64v_push(out, x->mem.p[i]);
  }
  return 0;
}

/* --- fold structures --------------------------------------------------------------------- */
typedef struct {
  uint8_t (*uuid)[16];
  uint32_t n, cap;
  uint32_t *tab;  /* id + 1, 0 = empty */
  uint32_t mask;
} ow_actors;
static uint32_t uuid_hash(const uint8_t *u) {
  uint64_t a, b;
  memcpy(&a, u, 8);
  memcpy(&b, u + 8, 8);
  uint64_t h = (a ^ (b * 0x9E3779B97F4A7C15ULL)) * 0xBF58476D1CE4E5B9ULL;
  return (uint32_t)(h >> 32);
}
static uint32_t ow_intern(ow_actors *t, uint64_t lo, uint64_t hi) {
  uint8_t u[16];
  memcpy(u, &lo, 8);
  memcpy(u + 8, &hi, 8);
  if (2 * (t->n + 1) > t->mask + 1 || !t->tab) {
    uint32_t ncap = t->tab ? 2 * (t->mask + 1) : 1024;
    free(t->tab);
    t->tab = (uint32_t *)calloc(ncap, 4);
    t->mask = ncap - 1;
    for (uint32_t i = 0; i < t->n; i++) {
      uint32_t h = uuid_hash(t->uuid[i]) & t->mask;
      while (t->tab[h]) h = (h + 1) & t->mask;
      t->tab[h] = i + 1;
    }
  }
  uint32_t h = uuid_hash(u) & t->mask;
  while (t->tab[h]) {
    if (memcmp(t->uuid[t->tab[h] - 1], u, 16) == 0) return t->tab[h] - 1;
    h = (h + 1) & t->mask;
  }
  if (t->n == t->cap) {
    t->cap = t->cap ? 2 * t->cap : 1024;
    t->uuid = (uint8_t (*)[16])realloc(t->uuid, (size_t)t->cap * 16);
  }
  memcpy(t->uuid[t->n], u, 16);
  t->tab[h] = t->n + 1;
  return t->n++;
}

typedef struct { uint32_t aid; uint64_t ctr; } ow_dot;
typedef struct { uint32_t n, cap; union { ow_dot one; ow_dot *heap; } u; } ow_vc;  /* sorted by aid */
static ow_dot *vc_d(ow_vc *v) { return v->cap > 1 ? v->u.heap : &v->u.one; }
static const ow_dot *vc_cd(const ow_vc *v) { return v->cap > 1 ? v->u.heap : &v->u.one; }
static void vc_free(ow_vc *v) {
  if (v->cap > 1) free(v->u.heap);
  memset(v, 0, sizeof *v);
}
static size_t vc_find(const ow_vc *v, uint32_t aid, int *found) {
  const ow_dot *d = vc_cd(v);
  size_t lo = 0, hi = v->n;
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    if (d[mid].aid < aid) lo = mid + 1; else hi = mid;
  }
  *found = lo < v->n && d[lo].aid == aid;
  return lo;
}
static uint64_t vc_get(const ow_vc *v, uint32_t aid) {
  int f;
  size_t i = vc_find(v, aid, &f);
  return f ? vc_cd(v)[i].ctr : 0;
}
static void vc_insert_at(ow_vc *v, size_t i, uint32_t aid, uint64_t c) {
  uint32_t capn = v->cap > 1 ? v->cap : 1;
  if (v->n == capn) {
    uint32_t nc = v->cap > 1 ? 2 * v->cap : 4;
    ow_dot *h = (ow_dot *)malloc((size_t)nc * sizeof(ow_dot));
    memcpy(h, vc_d(v), v->n * sizeof(ow_dot));
    if (v->cap > 1) free(v->u.heap);
    v->u.heap = h;
    v->cap = nc;
  }
  ow_dot *d = vc_d(v);
  memmove(d + i + 1, d + i, (v->n - i) * sizeof(ow_dot));
  d[i].aid = aid;
  d[i].ctr = c;
  v->n++;
}
static void vc_remove_at(ow_vc *v, size_t i) {
  ow_dot *d = vc_d(v);
  memmove(d + i, d + i + 1, (v->n - i - 1) * sizeof(ow_dot));
  v->n--;
}
static void vc_apply_dot(ow_vc *v, uint32_t aid, uint64_t c) {  /* VClock::apply */
  int f;
  size_t i = vc_find(v, aid, &f);
  if (f) { if (vc_d(v)[i].ctr < c) vc_d(v)[i].ctr = c; }
  else if (c > 0) vc_insert_at(v, i, aid, c);
}
static void vc_put(ow_vc *v, uint32_t aid, uint64_t c) {
  int f;
  size_t i = vc_find(v, aid, &f);
  if (f) vc_d(v)[i].ctr = c; else vc_insert_at(v, i, aid, c);
}
static void vc_clone(ow_vc *dst, const ow_vc *src) {
  memset(dst, 0, sizeof *dst);
  if (src->n <= 1) { *dst = *src; dst->cap = src->n ? 1 : 0; if (src->n) dst->u.one = vc_cd(src)[0]; return; }
  dst->u.heap = (ow_dot *)malloc(src->n * sizeof(ow_dot));
  memcpy(dst->u.heap, vc_cd(src), src->n * sizeof(ow_dot));
  dst->n = dst->cap = src->n;
  if (dst->cap == 1) dst->cap = 2;
}
static int vc_eq(const ow_vc *a, const ow_vc *b) {
  if (a->n != b->n) return 0;
  const ow_dot *x = vc_cd(a), *y = vc_cd(b);
  for (uint32_t i = 0; i < a->n; i++)
    if (x[i].aid != y[i].aid || x[i].ctr != y[i].ctr) return 0;
  return 1;
}
/* v.reset_remove(other): drop a when other holds a with counter >= v[a] */
static void vc_reset_remove(ow_vc *v, const ow_vc *other) {
  for (size_t i = v->n; i-- > 0;) {
    int f;
    size_t j = vc_find(other, vc_d(v)[i].aid, &f);
    if (f && vc_cd(other)[j].ctr >= vc_d(v)[i].ctr) vc_remove_at(v, i);
  }
}
static int dot_cmp_aid(const void *x, const void *y) {
  uint32_t a = ((const ow_dot *)x)->aid, b = ((const ow_dot *)y)->aid;
  return a < b ? -1 : a > b;
}
/* raw [n, (lo, hi, c) x n] (distinct uuids) -> v; returns the words consumed */
static size_t vc_from_raw(ow_vc *v, const uint64_t *p, ow_actors *A) {
  size_t n = (size_t)p[0];
  memset(v, 0, sizeof *v);
  if (n == 1) { vc_insert_at(v, 0, ow_intern(A, p[1], p[2]), p[3]); return 4; }
  if (n > 1) {
    v->u.heap = (ow_dot *)malloc(n * sizeof(ow_dot));
    v->cap = (uint32_t)n;
    for (size_t k = 0; k < n; k++) {
      v->u.heap[k].aid = ow_intern(A, p[1 + 3 * k], p[2 + 3 * k]);
      v->u.heap[k].ctr = p[3 + 3 * k];
    }
    qsort(v->u.heap, n, sizeof(ow_dot), dot_cmp_aid);
    v->n = (uint32_t)n;
  }
  return 1 + 3 * n;
}

typedef struct { uint64_t *c; size_t cap; } ow_dense;  /* clock by actor id; 0 = absent */
static uint64_t dn_get(const ow_dense *d, uint32_t a) { return a < d->cap ? d->c[a] : 0; }
static void dn_apply(ow_dense *d, uint32_t a, uint64_t v) {
  if (a >= d->cap) {
    size_t nc = d->cap ? d->cap : 1024;
    while (nc <= a) nc *= 2;
    d->c = (uint64_t *)realloc(d->c, nc * 8);
    memset(d->c + d->cap, 0, (nc - d->cap) * 8);
    d->cap = nc;
  }
  if (d->c[a] < v) d->c[a] = v;
}
static int vc_le_dense(const ow_vc *v, const ow_dense *d) {
  const ow_dot *x = vc_cd(v);
  for (uint32_t i = 0; i < v->n; i++)
    if (dn_get(d, x[i].aid) < x[i].ctr) return 0;
  return 1;
}
static int vc_le(const ow_vc *v, const ow_vc *o) {
  const ow_dot *x = vc_cd(v);
  for (uint32_t i = 0; i < v->n; i++)
    if (vc_get(o, x[i].aid) < x[i].ctr) return 0;
  return 1;
}
/* v.reset_remove(dense clock): the dense clock holds a iff its counter is nonzero */
static void vc_reset_remove_dense(ow_vc *v, const ow_dense *d) {
  for (size_t i = v->n; i-- > 0;) {
    uint64_t c = dn_get(d, vc_d(v)[i].aid);
    if (c && c >= vc_d(v)[i].ctr) vc_remove_at(v, i);
  }
}

typedef struct { uint64_t key; ow_vc vc; uint32_t used; } ow_slot;
typedef struct { ow_slot *s; size_t mask, n; } ow_map;
static uint64_t mix64(uint64_t x) {
  x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ULL;
  x ^= x >> 27; x *= 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}
static ow_slot *map_find(const ow_map *m, uint64_t k) {
  if (!m->s) return NULL;
  size_t h = mix64(k) & m->mask;
  while (m->s[h].used) {
    if (m->s[h].key == k) return &m->s[h];
    h = (h + 1) & m->mask;
  }
  return NULL;
}
static ow_slot *map_add(ow_map *m, uint64_t k, int *fresh) {  /* get or insert (empty clock) */
  if (!m->s || 2 * (m->n + 1) > m->mask + 1) {
    size_t nc = m->s ? 2 * (m->mask + 1) : 1024;
    ow_slot *old = m->s;
    size_t ocap = m->s ? m->mask + 1 : 0;
    m->s = (ow_slot *)calloc(nc, sizeof(ow_slot));
    m->mask = nc - 1;
    for (size_t i = 0; i < ocap; i++) {
      if (!old[i].used) continue;
      size_t h = mix64(old[i].key) & m->mask;
      while (m->s[h].used) h = (h + 1) & m->mask;
      m->s[h] = old[i];
    }
    free(old);
  }
  size_t h = mix64(k) & m->mask;
  while (m->s[h].used) {
    if (m->s[h].key == k) { *fresh = 0; return &m->s[h]; }
    h = (h + 1) & m->mask;
  }
  m->s[h].used = 1;
  m->s[h].key = k;
  memset(&m->s[h].vc, 0, sizeof(ow_vc));
  m->n++;
  *fresh = 1;
  return &m->s[h];
}
static void map_del(ow_map *m, ow_slot *s) {  /* backward-shift deletion */
  size_t i = (size_t)(s - m->s);
  vc_free(&m->s[i].vc);
  size_t j = i;
  for (;;) {
    j = (j + 1) & m->mask;
    if (!m->s[j].used) break;
    size_t k = mix64(m->s[j].key) & m->mask;
    if (i <= j ? (i < k && k <= j) : (i < k || k <= j)) continue;
    m->s[i] = m->s[j];
    i = j;
  }
  memset(&m->s[i], 0, sizeof(ow_slot));
  m->n--;
}
static void map_free(ow_map *m) {
  if (m->s)
    for (size_t i = 0; i <= m->mask; i++)
      if (m->s[i].used) vc_free(&m->s[i].vc);
  free(m->s);
  memset(m, 0, sizeof *m);
}

typedef struct { ow_vc clock; u64v mem; } ow_def;
typedef struct { ow_def *d; size_t n, cap; } ow_defs;
static void defs_free(ow_defs *D) {
  for (size_t i = 0; i < D->n; i++) { vc_free(&D->d[i].clock); u64v_free(&D->d[i].mem); }
  free(D->d);
  memset(D, 0, sizeof *D);
}
/* deferred.setdefault(clock.key(), set()).update(members) */
static void defs_add(ow_defs *D, const ow_vc *clock, const uint64_t *m, size_t nm) {
  size_t i = 0;
  while (i < D->n && !vc_eq(&D->d[i].clock, clock)) i++;
  if (i == D->n) {
    if (D->n == D->cap) {
      D->cap = D->cap ? 2 * D->cap : 8;
      D->d = (ow_def *)realloc(D->d, D->cap * sizeof(ow_def));
    }
    vc_clone(&D->d[i].clock, clock);
    memset(&D->d[i].mem, 0, sizeof(u64v));
    D->n++;
  }
  for (size_t k = 0; k < nm; k++) u64v_push(&D->d[i].mem, m[k]);
}

typedef struct { ow_dense clk; ow_map ent; ow_defs def; } ow_self;   /* the Core's Orswot */
typedef struct { ow_vc clk; ow_map ent; ow_defs def; } ow_other;    /* a decoded state's */

/* Orswot::apply_rm (crdts.py:113-121) */
static void ow_apply_rm(ow_self *o, const uint64_t *m, size_t nm, const ow_vc *clock) {
  for (size_t k = 0; k < nm; k++) {
    ow_slot *s = map_find(&o->ent, m[k]);
    if (!s) continue;
    vc_reset_remove(&s->vc, clock);
    if (s->vc.n == 0) map_del(&o->ent, s);
  }
  if (!vc_le_dense(clock, &o->clk)) defs_add(&o->def, clock, m, nm);
}
/* Orswot::apply_deferred (crdts.py:123-126) */
static void ow_apply_deferred(ow_self *o) {
  if (!o->def.n) return;
  ow_defs old = o->def;
  memset(&o->def, 0, sizeof o->def);
  for (size_t i = 0; i < old.n; i++) ow_apply_rm(o, old.d[i].mem.p, old.d[i].mem.n, &old.d[i].clock);
  defs_free(&old);
}
/* Orswot::merge (crdts.py:129-160) */
static void ow_merge(ow_self *o, ow_other *x) {
  u64v drop = {0};
  if (o->ent.s)
    for (size_t i = 0; i <= o->ent.mask; i++) {
      ow_slot *s = &o->ent.s[i];
      if (!s->used || map_find(&x->ent, s->key)) continue;
      if (vc_le(&s->vc, &x->clk)) u64v_push(&drop, s->key);  /* other has seen it and dropped it */
      else vc_reset_remove(&s->vc, &x->clk);
    }
  for (size_t k = 0; k < drop.n; k++) map_del(&o->ent, map_find(&o->ent, drop.p[k]));
  u64v_free(&drop);
  if (x->ent.s)
    for (size_t i = 0; i <= x->ent.mask; i++) {
      ow_slot *t = &x->ent.s[i];
      if (!t->used) continue;
      const ow_vc *clock = &t->vc;
      const ow_dot *cd = vc_cd(clock);
      ow_slot *ours = map_find(&o->ent, t->key);
      if (ours) {
        ow_vc cm;
        memset(&cm, 0, sizeof cm);
        for (uint32_t k = 0; k < clock->n; k++)      /* VClock::intersection(clock, ours) */
          if (vc_get(&ours->vc, cd[k].aid) == cd[k].ctr) vc_put(&cm, cd[k].aid, cd[k].ctr);
        for (uint32_t k = 0; k < clock->n; k++) {    /* .merge(clock.clone_without(self.clock)) */
          uint64_t c = dn_get(&o->clk, cd[k].aid);
          if (!(c && c >= cd[k].ctr)) vc_apply_dot(&cm, cd[k].aid, cd[k].ctr);
        }
        const ow_dot *od = vc_cd(&ours->vc);         /* .merge(ours.clone_without(other.clock)) */
        for (uint32_t k = 0; k < ours->vc.n; k++) {
          int f;
          size_t j = vc_find(&x->clk, od[k].aid, &f);
          if (!(f && vc_cd(&x->clk)[j].ctr >= od[k].ctr)) vc_apply_dot(&cm, od[k].aid, od[k].ctr);
        }
        if (cm.n == 0) { vc_free(&cm); map_del(&o->ent, ours); }
        else { vc_free(&ours->vc); ours->vc = cm; }
      } else {
        if (vc_le_dense(clock, &o->clk)) continue;  /* seen and dropped */
        ow_vc c;
        vc_clone(&c, clock);
        vc_reset_remove_dense(&c, &o->clk);
        int fresh;
        ow_slot *s = map_add(&o->ent, t->key, &fresh);
        s->vc = c;
      }
    }
  for (size_t i = 0; i < x->def.n; i++) ow_apply_rm(o, x->def.d[i].mem.p, x->def.d[i].mem.n, &x->def.d[i].clock);
  const ow_dot *xd = vc_cd(&x->clk);
  for (uint32_t k = 0; k < x->clk.n; k++) dn_apply(&o->clk, xd[k].aid, xd[k].ctr);
  ow_apply_deferred(o);
}

/* Orswot::apply over one op file's raw stream (crdts.py:99-111) */
static void ow_apply_ops(ow_self *o, ow_actors *A, const u64v *ops) {
  const uint64_t *p = ops->p, *e = ops->p + ops->n;
  ow_vc clock;
  memset(&clock, 0, sizeof clock);
  while (p < e) {
    if (p[0] == 0) {
      uint32_t a = ow_intern(A, p[1], p[2]);
      uint64_t c = p[3];
      size_t nm = (size_t)p[4];
      const uint64_t *m = p + 5;
      p = m + nm;
      if (dn_get(&o->clk, a) >= c) continue;  /* already seen */
      for (size_t k = 0; k < nm; k++) {
        int fresh;
        vc_apply_dot(&map_add(&o->ent, m[k], &fresh)->vc, a, c);
      }
      dn_apply(&o->clk, a, c);
      ow_apply_deferred(o);
    } else {
      p += 1 + vc_from_raw(&clock, p + 1, A);
      size_t nm = (size_t)p[0];
      ow_apply_rm(o, p + 1, nm, &clock);
      p += 1 + nm;
      vc_free(&clock);
    }
  }
}

static void ow_other_build(ow_other *x, const ow_raw *r, ow_actors *A) {
  memset(x, 0, sizeof *x);
  vc_from_raw(&x->clk, r->clk.p, A);
  const uint64_t *p = r->ent.p;
  size_t ne = (size_t)*p++;
  for (size_t k = 0; k < ne; k++) {
    uint64_t m = *p++;
    int fresh;
    ow_slot *s = map_add(&x->ent, m, &fresh);
    if (!fresh) vc_free(&s->vc);  /* a later duplicate member overwrites */
    p += vc_from_raw(&s->vc, p, A);
  }
  p = r->def.p;
  size_t nd = (size_t)*p++;
  for (size_t k = 0; k < nd; k++) {
    ow_vc c;
    p += vc_from_raw(&c, p, A);
    size_t nm = (size_t)*p++;
    defs_add(&x->def, &c, p, nm);
    p += nm;
    vc_free(&c);
  }
}
static void ow_other_free(ow_other *x) { vc_free(&x->clk); map_free(&x->ent); defs_free(&x->def); }

/* --- canonical serialization (crdts.py serialize: members ascending, deferred by clock bytes) */
typedef struct { const uint32_t *rank; const ow_actors *A; } ow_ser;
static void wr_arr_hdr(wr_t *w, size_t n) {
  if (n <= 15) wr_u8(w, (uint8_t)(0x90 | n));
  else if (n <= 0xffff) { wr_u8(w, 0xdc); wr_be(w, n, 2); }
  else { wr_u8(w, 0xdd); wr_be(w, n, 4); }
}
static void wr_dense(wr_t *w, const ow_dense *d, const ow_actors *A, const uint32_t *order) {
  size_t n = 0;
  for (uint32_t i = 0; i < A->n; i++) n += dn_get(d, i) != 0;
  wr_map_hdr(w, 1);
  wr_str(w, "dots");
  wr_map_hdr(w, n);
  for (uint32_t r = 0; r < A->n; r++) {
    uint64_t c = dn_get(d, order[r]);
    if (c) { wr_bin(w, A->uuid[order[r]], 16); wr_uint(w, c); }
  }
}
static void wr_sparse(wr_t *w, const ow_vc *v, const ow_ser *S) {
  ow_dot tmp[16], *t = v->n <= 16 ? tmp : (ow_dot *)malloc(v->n * sizeof(ow_dot));
  memcpy(t, vc_cd(v), v->n * sizeof(ow_dot));
  for (uint32_t i = 1; i < v->n; i++) {  /* insertion sort by uuid rank */
    ow_dot x = t[i];
    uint32_t j = i;
    while (j > 0 && S->rank[t[j - 1].aid] > S->rank[x.aid]) { t[j] = t[j - 1]; j--; }
    t[j] = x;
  }
  wr_map_hdr(w, 1);
  wr_str(w, "dots");
  wr_map_hdr(w, v->n);
  for (uint32_t i = 0; i < v->n; i++) { wr_bin(w, S->A->uuid[t[i].aid], 16); wr_uint(w, t[i].ctr); }
  if (t != tmp) free(t);
}
static const ow_actors *g_sort_actors;
static int aid_uuid_cmp(const void *x, const void *y) {
  return memcmp(g_sort_actors->uuid[*(const uint32_t *)x], g_sort_actors->uuid[*(const uint32_t *)y], 16);
}
static int u64_cmp(const void *x, const void *y) {
  uint64_t a = *(const uint64_t *)x, b = *(const uint64_t *)y;
  return a < b ? -1 : a > b;
}
typedef struct { uint64_t key; ow_vc *vc; } ow_ent_ref;
static int ent_cmp(const void *x, const void *y) { return u64_cmp(x, y); }
typedef struct { uint8_t *b; size_t n; ow_def *d; } ow_def_ref;
static int def_cmp(const void *x, const void *y) {
  const ow_def_ref *p = (const ow_def_ref *)x, *q = (const ow_def_ref *)y;
  size_t l = p->n < q->n ? p->n : q->n;
  int c = memcmp(p->b, q->b, l);
  if (c) return c;
  return p->n < q->n ? -1 : p->n > q->n;
}
static size_t ow_serialize(ow_self *o, const ow_dense *nov, const ow_actors *A, uint8_t *out, size_t cap) {
  uint32_t *order = (uint32_t *)malloc((A->n + 1) * 4), *rank = (uint32_t *)malloc((A->n + 1) * 4);
  for (uint32_t i = 0; i < A->n; i++) order[i] = i;
  g_sort_actors = A;
  qsort(order, A->n, 4, aid_uuid_cmp);
  for (uint32_t r = 0; r < A->n; r++) rank[order[r]] = r;
  ow_ser S = {rank, A};
  wr_t w = {out, cap, 0};
  wr_map_hdr(&w, 2);
  wr_str(&w, "next_op_versions");
  wr_dense(&w, nov, A, order);
  wr_str(&w, "state");
  wr_map_hdr(&w, 3);
  wr_str(&w, "clock");
  wr_dense(&w, &o->clk, A, order);
  wr_str(&w, "entries");
  ow_ent_ref *er = (ow_ent_ref *)malloc((o->ent.n + 1) * sizeof(ow_ent_ref));
  size_t ne = 0;
  if (o->ent.s)
    for (size_t i = 0; i <= o->ent.mask; i++)
      if (o->ent.s[i].used) { er[ne].key = o->ent.s[i].key; er[ne].vc = &o->ent.s[i].vc; ne++; }
  qsort(er, ne, sizeof(ow_ent_ref), ent_cmp);
  wr_map_hdr(&w, ne);
  for (size_t i = 0; i < ne; i++) { wr_uint(&w, er[i].key); wr_sparse(&w, er[i].vc, &S); }
  free(er);
  wr_str(&w, "deferred");
  ow_def_ref *dr = (ow_def_ref *)malloc((o->def.n + 1) * sizeof(ow_def_ref));
  for (size_t i = 0; i < o->def.n; i++) {
    wr_t k = {NULL, 0, 0};
    wr_sparse(&k, &o->def.d[i].clock, &S);
    dr[i].b = (uint8_t *)malloc(k.n);
    dr[i].n = k.n;
    wr_t k2 = {dr[i].b, k.n, 0};
    wr_sparse(&k2, &o->def.d[i].clock, &S);
    dr[i].d = &o->def.d[i];
  }
  qsort(dr, o->def.n, sizeof(ow_def_ref), def_cmp);
  wr_map_hdr(&w, o->def.n);
  for (size_t i = 0; i < o->def.n; i++) {
    u64v *m = &dr[i].d->mem;
    qsort(m->p, m->n, 8, u64_cmp);
    size_t u = 0;
    for (size_t k = 0; k < m->n; k++)
      if (k == 0 || m->p[k] != m->p[k - 1]) m->p[u++] = m->p[k];
    m->n = u;
    wr_put(&w, dr[i].b, dr[i].n);
    wr_arr_hdr(&w, u);
    for (size_t k = 0; k < u; k++) wr_uint(&w, m->p[k]);
    free(dr[i].b);
  }
  free(dr);
  free(order);
  free(rank);
  return w.n;
}

/* --- the baseline: open + decode parallel over files, merge + fold on one thread --------- */
typedef struct {
  const uint8_t *key, *dv;
  const uint8_t *sblob, *blob;
  const uint64_t *soffs, *offs;
  size_t ns, n, next;
  pthread_mutex_t mu;
  int32_t *status;  /* [ns + n] */
  ow_raw *states;   /* [ns] */
  u64v *ops;        /* [n] */
} ow_job;

static void *ow_worker(void *arg) {
  ow_job *j = (ow_job *)arg;
  ow_opctx ox;
  memset(&ox, 0, sizeof ox);
  uint8_t *buf = NULL;
  size_t bcap = 0;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    size_t lo = j->next;
    j->next += lo < j->ns ? 1 : 64;  /* a state file per claim, op files 64 at a time */
    pthread_mutex_unlock(&j->mu);
    if (lo >= j->ns + j->n) break;
    size_t hi = lo < j->ns ? lo + 1 : (lo + 64 < j->ns + j->n ? lo + 64 : j->ns + j->n);
    for (size_t i = lo; i < hi; i++) {
      int is_state = i < j->ns;
      size_t k = is_state ? i : i - j->ns;
      const uint8_t *b = is_state ? j->sblob : j->blob;
      const uint64_t *of = is_state ? j->soffs : j->offs;
      size_t flen = of[k + 1] - of[k];
      if (flen + 1 > bcap) { bcap = flen + 1; buf = (uint8_t *)realloc(buf, bcap); }
      const uint8_t *pt;
      size_t pl;
      int st = open_file(KEY_VERSION, j->key, 32, (const uint8_t(*)[16])j->dv, 1, b + of[k], flen,
                         buf, &pt, &pl);
      if (st == OC_OK) {
        if (is_state) {
          ow_rawctx rx = {ox.vc, &j->states[k]};
          if (ow_decode_state(pt, pl, &rx)) st = OC_ERR_DECODE;
          ox.vc = rx.vc;
        } else if (ow_decode_ops(pt, pl, &ox, &j->ops[k])) st = OC_ERR_DECODE;
      }
      j->status[i] = st;
    }
  }
  free(buf);
  free(ox.vc.tmp);
  u64v_free(&ox.clk);
  u64v_free(&ox.mem);
  return NULL;
}

size_t oc_compact_orswot_best(const uint8_t key[32], const uint8_t data_version[16],
                              const uint8_t *state_blob, const uint64_t *state_offs,
                              size_t n_states, const uint8_t *blob, const uint64_t *offs,
                              const uint8_t (*file_actor)[16], const uint64_t *file_version,
                              size_t n_files, int n_threads, int seal, uint8_t *out, size_t cap,
                              int *err, double phase_s[4]) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  double t0 = oc_now();
  ow_job j;
  memset(&j, 0, sizeof j);
  j.key = key; j.dv = data_version;
  j.sblob = state_blob; j.soffs = state_offs; j.ns = n_states;
  j.blob = blob; j.offs = offs; j.n = n_files;
  j.status = (int32_t *)calloc(n_states + n_files + 1, sizeof(int32_t));
  j.states = (ow_raw *)calloc(n_states + 1, sizeof(ow_raw));
  j.ops = (u64v *)calloc(n_files + 1, sizeof(u64v));
  pthread_mutex_init(&j.mu, NULL);
  pthread_t th[256];
  for (int t = 0; t < n_threads; t++) pthread_create(&th[t], NULL, ow_worker, &j);
  for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
  pthread_mutex_destroy(&j.mu);
  double t1 = oc_now();

  int e = OC_OK;
  size_t n_out = 0;
  ow_actors A;
  memset(&A, 0, sizeof A);
  ow_self o;
  memset(&o, 0, sizeof o);
  ow_dense nov;
  memset(&nov, 0, sizeof nov);
  /* read_remote_states (lib.rs:401-469): any failing file rejects the batch */
  for (size_t i = 0; i < n_states && !e; i++) e = j.status[i];
  for (size_t i = 0; i < n_states && !e; i++) {
    ow_other x;
    ow_other_build(&x, &j.states[i], &A);
    ow_merge(&o, &x);
    ow_other_free(&x);
    const uint64_t *p = j.states[i].nov.p;
    for (size_t k = 0; k < (size_t)p[0]; k++)
      dn_apply(&nov, ow_intern(&A, p[1 + 3 * k], p[2 + 3 * k]), p[3 + 3 * k]);
  }
  double t2 = oc_now();
  /* read_remote_ops (lib.rs:471-547): every file opened and decoded first, then the gate */
  for (size_t i = 0; i < n_files && !e; i++) e = j.status[n_states + i];
  if (!e)
    for (size_t i = 0; i < n_files; i++) {
      uint64_t lo, hi;
      memcpy(&lo, file_actor[i], 8);
      memcpy(&hi, file_actor[i] + 8, 8);
      uint32_t a = ow_intern(&A, lo, hi);
      uint64_t expected = dn_get(&nov, a);
      if (file_version[i] < expected) continue;
      if (expected < file_version[i]) { e = OC_ERR_OP_VERSION; break; }
      ow_apply_ops(&o, &A, &j.ops[i]);
      dn_apply(&nov, a, expected + 1);
    }
  double t3 = oc_now();
  if (!e) {
    n_out = ow_serialize(&o, &nov, &A, out, cap);
    if (seal && n_out <= cap) {  /* Core::compact's file: outer version || Cryptor::encrypt(..) */
      uint8_t *clear = (uint8_t *)malloc(n_out + 16);
      memcpy(clear, data_version, 16);
      memcpy(clear + 16, out, n_out);
      uint8_t *file = (uint8_t *)malloc(16 + oc_cryptor_sealed_len(n_out + 16));
      memcpy(file, CORE_VERSION, 16);
      size_t fl = 0;
      static const uint8_t nonce[24] = {0};
      oc_cryptor_encrypt(KEY_VERSION, key, 32, nonce, clear, n_out + 16, file + 16, &fl);
      uint8_t name[32];
      oc_sha3_256(file, fl + 16, name);  /* content name (crdt-enc-tokio lib.rs:403-432) */
      free(clear);
      free(file);
    }
  }
  double t4 = oc_now();
  if (phase_s) { phase_s[0] = t1 - t0; phase_s[1] = t2 - t1; phase_s[2] = t3 - t2; phase_s[3] = t4 - t3; }
  for (size_t i = 0; i < n_states; i++) {
    u64v_free(&j.states[i].nov); u64v_free(&j.states[i].clk);
    u64v_free(&j.states[i].ent); u64v_free(&j.states[i].def);
  }
  for (size_t i = 0; i < n_files; i++) u64v_free(&j.ops[i]);
  free(j.states); free(j.ops); free(j.status);
  map_free(&o.ent); defs_free(&o.def); free(o.clk.c); free(nov.c);
  free(A.uuid); free(A.tab);
  *err = e;
  return n_out;
}
