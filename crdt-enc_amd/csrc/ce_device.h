// ce_device.h -- gfx950 device helpers shared by the kernels: ChaCha20/HChaCha20, Poly1305
// in radix 2^26, key schedule, actor-table lookup, msgpack window helpers.
#pragma once
#include "ce_kernels.h"

#ifndef CE_ROT16_SDWA
#define CE_ROT16_SDWA 1
#endif

namespace ce {

// ----------------------------------------------------------------------------------------
// ChaCha20 (RFC 8439 §2.3) / HChaCha20 (draft-irtf-cfrg-xchacha-03 §2.2)
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int c) {
  return __builtin_amdgcn_alignbit(x, x, 32 - c);
}

// rotl32(d ^ a, 16) as two SDWA xors, one per 16-bit half of the result.  Measured on
// MI355X (tools/ubench_chacha, profiles/r02_ubench_chacha.txt): ChaCha20 at 2 waves/SIMD runs
// 2.50 TB/s of keystream this way against 2.26 TB/s with xor + v_alignbit_b32.
template <bool SD>
__device__ __forceinline__ uint32_t xor_rotl16_t(uint32_t d, uint32_t a) {
  if (!SD) return rotl32(d ^ a, 16);
  uint32_t r;
  asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n\t"
      "v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0"
      : "=&v"(r) : "v"(d), "v"(a));
  return r;
}
__device__ __forceinline__ uint32_t xor_rotl16(uint32_t d, uint32_t a) {
  return xor_rotl16_t<CE_ROT16_SDWA != 0>(d, a);
}

#define CE_QR_T(SD, a, b, c, d)                                                             \
  a += b; d = xor_rotl16_t<SD>(d, a); c += d; b ^= c; b = rotl32(b, 12);                   \
  a += b; d ^= a; d = rotl32(d, 8);  c += d; b ^= c; b = rotl32(b, 7);
#define CE_QR(a, b, c, d) CE_QR_T(CE_ROT16_SDWA != 0, a, b, c, d)

__device__ __forceinline__ void chacha_rounds(uint32_t (&x)[16]) {
#pragma unroll
  for (int i = 0; i < 10; i++) {
    CE_QR(x[0], x[4], x[8], x[12]); CE_QR(x[1], x[5], x[9], x[13]);
    CE_QR(x[2], x[6], x[10], x[14]); CE_QR(x[3], x[7], x[11], x[15]);
    CE_QR(x[0], x[5], x[10], x[15]); CE_QR(x[1], x[6], x[11], x[12]);
    CE_QR(x[2], x[7], x[8], x[13]); CE_QR(x[3], x[4], x[9], x[14]);
  }
}

__device__ __forceinline__ void chacha_block(const uint32_t (&k)[8], uint32_t ctr, uint32_t n0,
                                             uint32_t n1, uint32_t n2, uint32_t (&out)[16]) {
  uint32_t x[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, k[0], k[1], k[2], k[3],
                    k[4], k[5], k[6], k[7], ctr, n0, n1, n2};
  chacha_rounds(x);
  out[0] = x[0] + 0x61707865u; out[1] = x[1] + 0x3320646eu;
  out[2] = x[2] + 0x79622d32u; out[3] = x[3] + 0x6b206574u;
#pragma unroll
  for (int i = 0; i < 8; i++) out[4 + i] = x[4 + i] + k[i];
  out[12] = x[12] + ctr; out[13] = x[13] + n0; out[14] = x[14] + n1; out[15] = x[15] + n2;
}

// Counter-independent part of a ChaCha20 block (key, 96-bit nonce n0 n1 n2 fixed, counter
// varying): the first column round's quarter rounds on columns 1..3 and the first add of
// column 0.  Computed once per file and reused for every block of it (13 words).
struct ChachaPre {
  uint32_t c[12];  // x1 x5 x9 x13 | x2 x6 x10 x14 | x3 x7 x11 x15 after the first column round
  uint32_t a0;     // x0 + x4
};

__device__ __forceinline__ ChachaPre chacha_pre(const uint32_t (&k)[8], uint32_t n0, uint32_t n1,
                                                uint32_t n2) {
  uint32_t x1 = 0x3320646eu, x5 = k[1], x9 = k[5], x13 = n0;
  uint32_t x2 = 0x79622d32u, x6 = k[2], x10 = k[6], x14 = n1;
  uint32_t x3 = 0x6b206574u, x7 = k[3], x11 = k[7], x15 = n2;
  CE_QR(x1, x5, x9, x13);
  CE_QR(x2, x6, x10, x14);
  CE_QR(x3, x7, x11, x15);
  ChachaPre p;
  p.c[0] = x1; p.c[1] = x5; p.c[2] = x9; p.c[3] = x13;
  p.c[4] = x2; p.c[5] = x6; p.c[6] = x10; p.c[7] = x14;
  p.c[8] = x3; p.c[9] = x7; p.c[10] = x11; p.c[11] = x15;
  p.a0 = 0x61707865u + k[0];
  return p;
}

// chacha_block with the counter-independent first-round work taken from `pre`.  UNR = double
// rounds per trip of the 9-trip loop (9: straight-line code; 1 or 3: a rolled loop, a fraction
// of the instruction bytes for kernels whose loop body would otherwise crowd the I-cache).
template <bool SD = (CE_ROT16_SDWA != 0), int UNR = 9>
__device__ __forceinline__ void chacha_block_pre(const ChachaPre& pre, const uint32_t (&k)[8],
                                                 uint32_t ctr, uint32_t n0, uint32_t n1,
                                                 uint32_t n2, uint32_t (&out)[16]) {
  uint32_t x[16];
  x[1] = pre.c[0]; x[5] = pre.c[1]; x[9] = pre.c[2]; x[13] = pre.c[3];
  x[2] = pre.c[4]; x[6] = pre.c[5]; x[10] = pre.c[6]; x[14] = pre.c[7];
  x[3] = pre.c[8]; x[7] = pre.c[9]; x[11] = pre.c[10]; x[15] = pre.c[11];
  // column 0 of the first round, after its first add
  x[0] = pre.a0; x[4] = k[0]; x[8] = k[4]; x[12] = ctr;
  x[12] = xor_rotl16_t<SD>(x[12], x[0]); x[8] += x[12]; x[4] ^= x[8]; x[4] = rotl32(x[4], 12);
  x[0] += x[4]; x[12] ^= x[0]; x[12] = rotl32(x[12], 8); x[8] += x[12]; x[4] ^= x[8]; x[4] = rotl32(x[4], 7);
  // first diagonal round, then 9 double rounds
  CE_QR_T(SD, x[0], x[5], x[10], x[15]); CE_QR_T(SD, x[1], x[6], x[11], x[12]);
  CE_QR_T(SD, x[2], x[7], x[8], x[13]); CE_QR_T(SD, x[3], x[4], x[9], x[14]);
  auto dround = [&] {
    CE_QR_T(SD, x[0], x[4], x[8], x[12]); CE_QR_T(SD, x[1], x[5], x[9], x[13]);
    CE_QR_T(SD, x[2], x[6], x[10], x[14]); CE_QR_T(SD, x[3], x[7], x[11], x[15]);
    CE_QR_T(SD, x[0], x[5], x[10], x[15]); CE_QR_T(SD, x[1], x[6], x[11], x[12]);
    CE_QR_T(SD, x[2], x[7], x[8], x[13]); CE_QR_T(SD, x[3], x[4], x[9], x[14]);
  };
  if constexpr (UNR == 1) {
#pragma unroll 1
    for (int i = 0; i < 9; i++) dround();
  } else if constexpr (UNR == 3) {
#pragma unroll 1
    for (int i = 0; i < 3; i++) { dround(); dround(); dround(); }
  } else {
#pragma unroll
    for (int i = 0; i < 9; i++) dround();
  }
  out[0] = x[0] + 0x61707865u; out[1] = x[1] + 0x3320646eu;
  out[2] = x[2] + 0x79622d32u; out[3] = x[3] + 0x6b206574u;
#pragma unroll
  for (int i = 0; i < 8; i++) out[4 + i] = x[4 + i] + k[i];
  out[12] = x[12] + ctr; out[13] = x[13] + n0; out[14] = x[14] + n1; out[15] = x[15] + n2;
}

// two chacha_block_pre blocks (counters ca, cb) with their quarter rounds interleaved: eight
// independent ARX chains per round instead of four
template <int UNR = 9>
__device__ __forceinline__ void chacha_block_pre2(const ChachaPre& pre, const uint32_t (&k)[8],
                                                  uint32_t ca, uint32_t cb, uint32_t n0, uint32_t n1,
                                                  uint32_t n2, uint32_t (&oa)[16], uint32_t (&ob)[16]) {
  uint32_t x[16], y[16];
  x[1] = pre.c[0]; x[5] = pre.c[1]; x[9] = pre.c[2]; x[13] = pre.c[3];
  x[2] = pre.c[4]; x[6] = pre.c[5]; x[10] = pre.c[6]; x[14] = pre.c[7];
  x[3] = pre.c[8]; x[7] = pre.c[9]; x[11] = pre.c[10]; x[15] = pre.c[11];
#pragma unroll
  for (int i = 1; i < 16; i++) y[i] = x[i];
  x[0] = pre.a0; x[4] = k[0]; x[8] = k[4]; x[12] = ca;
  y[0] = pre.a0; y[4] = k[0]; y[8] = k[4]; y[12] = cb;
  x[12] = xor_rotl16_t<true>(x[12], x[0]); y[12] = xor_rotl16_t<true>(y[12], y[0]);
  x[8] += x[12]; y[8] += y[12]; x[4] ^= x[8]; y[4] ^= y[8];
  x[4] = rotl32(x[4], 12); y[4] = rotl32(y[4], 12);
  x[0] += x[4]; y[0] += y[4]; x[12] ^= x[0]; y[12] ^= y[0];
  x[12] = rotl32(x[12], 8); y[12] = rotl32(y[12], 8);
  x[8] += x[12]; y[8] += y[12]; x[4] ^= x[8]; y[4] ^= y[8];
  x[4] = rotl32(x[4], 7); y[4] = rotl32(y[4], 7);
#define CE_QR2(a, b, c, d) CE_QR_T(true, x[a], x[b], x[c], x[d]); CE_QR_T(true, y[a], y[b], y[c], y[d]);
  CE_QR2(0, 5, 10, 15); CE_QR2(1, 6, 11, 12); CE_QR2(2, 7, 8, 13); CE_QR2(3, 4, 9, 14);
  auto dround2 = [&] {
    CE_QR2(0, 4, 8, 12); CE_QR2(1, 5, 9, 13); CE_QR2(2, 6, 10, 14); CE_QR2(3, 7, 11, 15);
    CE_QR2(0, 5, 10, 15); CE_QR2(1, 6, 11, 12); CE_QR2(2, 7, 8, 13); CE_QR2(3, 4, 9, 14);
  };
  if constexpr (UNR == 1) {
#pragma unroll 1
    for (int i = 0; i < 9; i++) dround2();
  } else {
#pragma unroll
    for (int i = 0; i < 9; i++) dround2();
  }
#undef CE_QR2
  const uint32_t c4[4] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
#pragma unroll
  for (int i = 0; i < 4; i++) { oa[i] = x[i] + c4[i]; ob[i] = y[i] + c4[i]; }
#pragma unroll
  for (int i = 0; i < 8; i++) { oa[4 + i] = x[4 + i] + k[i]; ob[4 + i] = y[4 + i] + k[i]; }
  oa[12] = x[12] + ca; ob[12] = y[12] + cb;
  oa[13] = x[13] + n0; ob[13] = y[13] + n0;
  oa[14] = x[14] + n1; ob[14] = y[14] + n1;
  oa[15] = x[15] + n2; ob[15] = y[15] + n2;
}

__device__ __forceinline__ void hchacha20(const uint32_t (&k)[8], const uint32_t (&n)[4],
                                          uint32_t (&sub)[8]) {
  uint32_t x[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, k[0], k[1], k[2], k[3],
                    k[4], k[5], k[6], k[7], n[0], n[1], n[2], n[3]};
  chacha_rounds(x);
  sub[0] = x[0]; sub[1] = x[1]; sub[2] = x[2]; sub[3] = x[3];
  sub[4] = x[12]; sub[5] = x[13]; sub[6] = x[14]; sub[7] = x[15];
}

// ----------------------------------------------------------------------------------------
// Poly1305 over GF(2^130 - 5), radix 2^26 (5 limbs), v_mad_u64_u32 products
// ----------------------------------------------------------------------------------------
static constexpr uint32_t M26 = 0x3ffffffu;

struct L5 {
  uint32_t v[5];
};

// h * r mod p; h limbs < 2^28, r limbs < 2^26 + 2^9  ->  result limbs < 2^26 (v[1] < 2^26+2^9)
__device__ __forceinline__ L5 mulmod(const L5& h, const L5& r) {
  const uint32_t s1 = r.v[1] * 5, s2 = r.v[2] * 5, s3 = r.v[3] * 5, s4 = r.v[4] * 5;
  uint64_t d0 = (uint64_t)h.v[0] * r.v[0] + (uint64_t)h.v[1] * s4 + (uint64_t)h.v[2] * s3 +
                (uint64_t)h.v[3] * s2 + (uint64_t)h.v[4] * s1;
  uint64_t d1 = (uint64_t)h.v[0] * r.v[1] + (uint64_t)h.v[1] * r.v[0] + (uint64_t)h.v[2] * s4 +
                (uint64_t)h.v[3] * s3 + (uint64_t)h.v[4] * s2;
  uint64_t d2 = (uint64_t)h.v[0] * r.v[2] + (uint64_t)h.v[1] * r.v[1] + (uint64_t)h.v[2] * r.v[0] +
                (uint64_t)h.v[3] * s4 + (uint64_t)h.v[4] * s3;
  uint64_t d3 = (uint64_t)h.v[0] * r.v[3] + (uint64_t)h.v[1] * r.v[2] + (uint64_t)h.v[2] * r.v[1] +
                (uint64_t)h.v[3] * r.v[0] + (uint64_t)h.v[4] * s4;
  uint64_t d4 = (uint64_t)h.v[0] * r.v[4] + (uint64_t)h.v[1] * r.v[3] + (uint64_t)h.v[2] * r.v[2] +
                (uint64_t)h.v[3] * r.v[1] + (uint64_t)h.v[4] * r.v[0];
  L5 o;
  d1 += d0 >> 26; o.v[0] = (uint32_t)d0 & M26;
  d2 += d1 >> 26; o.v[1] = (uint32_t)d1 & M26;
  d3 += d2 >> 26; o.v[2] = (uint32_t)d2 & M26;
  d4 += d3 >> 26; o.v[3] = (uint32_t)d3 & M26;
  const uint64_t c = d4 >> 26; o.v[4] = (uint32_t)d4 & M26;
  const uint64_t t0 = (uint64_t)o.v[0] + c * 5;
  o.v[0] = (uint32_t)t0 & M26;
  o.v[1] += (uint32_t)(t0 >> 26);
  return o;
}

// A multiplier with its 5x limbs (2^130 = 5 mod p), for sums of products reduced once:
// mac5 adds h * r into five 64-bit column sums without carrying, reduce5 carries them.  Each
// product adds < 5 * 2^27 * 2^28.4 < 2^57.7 per column (h limbs < 2^27), so up to 64 products
// fit a column; reduce5 keeps every carry in 64 bits.
struct MulR {
  uint32_t v[5], s[4];  // s[i] = 5 * v[i + 1]
};

__device__ __forceinline__ MulR mul_r(const L5& r) {
  MulR o;
#pragma unroll
  for (int i = 0; i < 5; i++) o.v[i] = r.v[i];
#pragma unroll
  for (int i = 0; i < 4; i++) o.s[i] = r.v[i + 1] * 5;
  return o;
}

__device__ __forceinline__ void mac5(uint64_t (&d)[5], const L5& h, const MulR& r) {
  d[0] += (uint64_t)h.v[0] * r.v[0] + (uint64_t)h.v[1] * r.s[3] + (uint64_t)h.v[2] * r.s[2] +
          (uint64_t)h.v[3] * r.s[1] + (uint64_t)h.v[4] * r.s[0];
  d[1] += (uint64_t)h.v[0] * r.v[1] + (uint64_t)h.v[1] * r.v[0] + (uint64_t)h.v[2] * r.s[3] +
          (uint64_t)h.v[3] * r.s[2] + (uint64_t)h.v[4] * r.s[1];
  d[2] += (uint64_t)h.v[0] * r.v[2] + (uint64_t)h.v[1] * r.v[1] + (uint64_t)h.v[2] * r.v[0] +
          (uint64_t)h.v[3] * r.s[3] + (uint64_t)h.v[4] * r.s[2];
  d[3] += (uint64_t)h.v[0] * r.v[3] + (uint64_t)h.v[1] * r.v[2] + (uint64_t)h.v[2] * r.v[1] +
          (uint64_t)h.v[3] * r.v[0] + (uint64_t)h.v[4] * r.s[3];
  d[4] += (uint64_t)h.v[0] * r.v[4] + (uint64_t)h.v[1] * r.v[3] + (uint64_t)h.v[2] * r.v[2] +
          (uint64_t)h.v[3] * r.v[1] + (uint64_t)h.v[4] * r.v[0];
}

__device__ __forceinline__ L5 reduce5(uint64_t (&d)[5]) {
  L5 o;
  d[1] += d[0] >> 26; o.v[0] = (uint32_t)d[0] & M26;
  d[2] += d[1] >> 26; o.v[1] = (uint32_t)d[1] & M26;
  d[3] += d[2] >> 26; o.v[2] = (uint32_t)d[2] & M26;
  d[4] += d[3] >> 26; o.v[3] = (uint32_t)d[3] & M26;
  o.v[4] = (uint32_t)d[4] & M26;
  const uint64_t t = (d[4] >> 26) * 5 + o.v[0];
  o.v[0] = (uint32_t)t & M26;
  o.v[1] += (uint32_t)(t >> 26);
  return o;
}

__device__ __forceinline__ L5 add5(const L5& a, const L5& b) {
  L5 o;
#pragma unroll
  for (int i = 0; i < 5; i++) o.v[i] = a.v[i] + b.v[i];
  return o;
}

// partial carry: limbs back under 2^26 (+ small in v[1])
__device__ __forceinline__ L5 carry5(L5 h) {
  uint32_t c;
  c = h.v[0] >> 26; h.v[0] &= M26; h.v[1] += c;
  c = h.v[1] >> 26; h.v[1] &= M26; h.v[2] += c;
  c = h.v[2] >> 26; h.v[2] &= M26; h.v[3] += c;
  c = h.v[3] >> 26; h.v[3] &= M26; h.v[4] += c;
  c = h.v[4] >> 26; h.v[4] &= M26; h.v[0] += c * 5;
  c = h.v[0] >> 26; h.v[0] &= M26; h.v[1] += c;
  return h;
}

// 16-byte little-endian block (+2^128 pad bit) -> limbs
__device__ __forceinline__ L5 block_limbs(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  L5 m;
  m.v[0] = w0 & M26;
  m.v[1] = __builtin_amdgcn_alignbit(w1, w0, 26) & M26;
  m.v[2] = __builtin_amdgcn_alignbit(w2, w1, 20) & M26;
  m.v[3] = __builtin_amdgcn_alignbit(w3, w2, 14) & M26;
  m.v[4] = __builtin_amdgcn_alignbit(1u, w3, 8);  // (w3 >> 8) | 2^24 in one instruction
  return m;
}

// full reduction mod p, then (h + s) mod 2^128 -> 4 LE words
__device__ __forceinline__ void poly_tag(L5 h, const uint32_t (&s)[4], uint32_t (&tag)[4]) {
  h = carry5(h);
  uint32_t c;
  // limbs 0..3 < 2^26, h4 <= 2^26 (+small): value < 2^130 + 2^104
  c = h.v[1] >> 26; h.v[1] &= M26; h.v[2] += c;
  c = h.v[2] >> 26; h.v[2] &= M26; h.v[3] += c;
  c = h.v[3] >> 26; h.v[3] &= M26; h.v[4] += c;
  // g = h + 5 - 2^130 ; select g when non-negative (h >= p)
  uint32_t g[5];
  g[0] = h.v[0] + 5; c = g[0] >> 26; g[0] &= M26;
  g[1] = h.v[1] + c; c = g[1] >> 26; g[1] &= M26;
  g[2] = h.v[2] + c; c = g[2] >> 26; g[2] &= M26;
  g[3] = h.v[3] + c; c = g[3] >> 26; g[3] &= M26;
  g[4] = h.v[4] + c - (1u << 26);
  const uint32_t mask = (g[4] >> 31) - 1;  // all ones when g >= 0
#pragma unroll
  for (int i = 0; i < 5; i++) h.v[i] = (h.v[i] & ~mask) | (g[i] & mask);
  const uint32_t w0 = h.v[0] | (h.v[1] << 26);
  const uint32_t w1 = (h.v[1] >> 6) | (h.v[2] << 20);
  const uint32_t w2 = (h.v[2] >> 12) | (h.v[3] << 14);
  const uint32_t w3 = (h.v[3] >> 18) | (h.v[4] << 8);
  uint64_t f = (uint64_t)w0 + s[0]; tag[0] = (uint32_t)f;
  f = (uint64_t)w1 + s[1] + (f >> 32); tag[1] = (uint32_t)f;
  f = (uint64_t)w2 + s[2] + (f >> 32); tag[2] = (uint32_t)f;
  f = (uint64_t)w3 + s[3] + (f >> 32); tag[3] = (uint32_t)f;
}

__device__ __forceinline__ L5 load_l5(const uint32_t* p) {
  L5 o;
#pragma unroll
  for (int i = 0; i < 5; i++) o.v[i] = p[i];
  return o;
}

__device__ __forceinline__ uint32_t ld_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// key schedule shared by open/seal setup: subkey, (r, s), r^(2^k); nonce as 6 LE words
__device__ __forceinline__ void key_schedule_w(const DevKey& key, const uint32_t (&nw)[6], FileParams& P) {
  uint32_t k[8], n16[4], sub[8];
#pragma unroll
  for (int i = 0; i < 8; i++) k[i] = key.k[i];
#pragma unroll
  for (int i = 0; i < 4; i++) n16[i] = nw[i];
  hchacha20(k, n16, sub);
  const uint32_t n2a = nw[4], n2b = nw[5];
  uint32_t b0[16];
  chacha_block(sub, 0, 0, n2a, n2b, b0);
#pragma unroll
  for (int i = 0; i < 8; i++) P.subkey[i] = sub[i];
  P.n2[0] = n2a; P.n2[1] = n2b;
  // r = le128(b0[0..4]) clamped
  const uint32_t r0 = b0[0] & 0x0fffffffu, r1 = b0[1] & 0x0ffffffcu, r2 = b0[2] & 0x0ffffffcu,
                 r3 = b0[3] & 0x0ffffffcu;
  L5 r;
  r.v[0] = r0 & M26;
  r.v[1] = __builtin_amdgcn_alignbit(r1, r0, 26) & M26;
  r.v[2] = __builtin_amdgcn_alignbit(r2, r1, 20) & M26;
  r.v[3] = __builtin_amdgcn_alignbit(r3, r2, 14) & M26;
  r.v[4] = r3 >> 8;
  P.s[0] = b0[4]; P.s[1] = b0[5]; P.s[2] = b0[6]; P.s[3] = b0[7];
#pragma unroll
  for (int i = 0; i < 5; i++) P.rpow[0][i] = r.v[i];
  L5 p = r;
#pragma unroll  // constant rpow indices: P stays in registers (no scratch in the setup kernels)
  for (int kk = 1; kk < 7; kk++) {
    p = mulmod(p, p);
#pragma unroll
    for (int i = 0; i < 5; i++) P.rpow[kk][i] = p.v[i];
  }
}

// PolyAux of an opened file whose FileParams (rpow, len, s, tag) are set (lane per file)
__device__ __forceinline__ void poly_aux(const FileParams& P, PolyAux& X) {
  const L5 r = load_l5(P.rpow[0]), r2 = load_l5(P.rpow[1]), r4 = load_l5(P.rpow[2]);
  const L5 r3 = mulmod(r2, r);
  const L5 r12 = mulmod(load_l5(P.rpow[3]), r4);
  const L5 r48 = mulmod(load_l5(P.rpow[5]), load_l5(P.rpow[4]));
  const uint32_t npc = (P.len + 15) >> 4, nblk = (P.len + 63) >> 6;
  const uint32_t delta = 4 * nblk - npc;  // 0..3
  const L5 r5 = mulmod(r4, r), r6 = mulmod(r4, r2);
  const L5 e6 = delta == 0 ? r6 : delta == 1 ? r5 : delta == 2 ? r4 : r3;
  const L5 lr = mulmod(block_limbs(0u, 0u, P.len, 0u), r);  // le64(0) || le64(len), pad bit
#pragma unroll
  for (int i = 0; i < 5; i++) {
    X.r3[i] = r3.v[i]; X.r12[i] = r12.v[i]; X.r48[i] = r48.v[i];
    X.e6[i] = e6.v[i]; X.lr[i] = lr.v[i];
  }
  uint64_t b = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint64_t d = (uint64_t)P.tag[i] - P.s[i] - b;
    X.ts[i] = (uint32_t)d;
    b = (d >> 32) & 1;
  }
  X.pad[0] = X.pad[1] = X.pad[2] = 0;
}

// h (limbs < 2^31, v[1] < 2^31) fully reduced mod p, its low 128 bits == ts (the expected tag
// less s, mod 2^128): the tag check of (h + s) mod 2^128 == tag without the 128-bit add
__device__ __forceinline__ bool poly_check(L5 h, const uint32_t (&ts)[4]) {
  uint32_t c;
  c = h.v[0] >> 26; h.v[0] &= M26; h.v[1] += c;
  c = h.v[1] >> 26; h.v[1] &= M26; h.v[2] += c;
  c = h.v[2] >> 26; h.v[2] &= M26; h.v[3] += c;
  c = h.v[3] >> 26; h.v[3] &= M26; h.v[4] += c;
  c = h.v[4] >> 26; h.v[4] &= M26; h.v[0] += c * 5;
  c = h.v[0] >> 26; h.v[0] &= M26; h.v[1] += c;
  c = h.v[1] >> 26; h.v[1] &= M26; h.v[2] += c;
  c = h.v[2] >> 26; h.v[2] &= M26; h.v[3] += c;
  c = h.v[3] >> 26; h.v[3] &= M26; h.v[4] += c;
  // limbs 0..3 < 2^26, h4 <= 2^26 (+small): g = h + 5 - 2^130, kept when non-negative (h >= p)
  uint32_t g[5];
  g[0] = h.v[0] + 5; c = g[0] >> 26; g[0] &= M26;
  g[1] = h.v[1] + c; c = g[1] >> 26; g[1] &= M26;
  g[2] = h.v[2] + c; c = g[2] >> 26; g[2] &= M26;
  g[3] = h.v[3] + c; c = g[3] >> 26; g[3] &= M26;
  g[4] = h.v[4] + c - (1u << 26);
  const uint32_t mask = (g[4] >> 31) - 1;  // all ones when g >= 0
#pragma unroll
  for (int i = 0; i < 5; i++) h.v[i] = (h.v[i] & ~mask) | (g[i] & mask);
  const uint32_t w0 = h.v[0] | (h.v[1] << 26);
  const uint32_t w1 = (h.v[1] >> 6) | (h.v[2] << 20);
  const uint32_t w2 = (h.v[2] >> 12) | (h.v[3] << 14);
  const uint32_t w3 = (h.v[3] >> 18) | (h.v[4] << 8);
  return ((w0 ^ ts[0]) | (w1 ^ ts[1]) | (w2 ^ ts[2]) | (w3 ^ ts[3])) == 0;
}

__device__ __forceinline__ void key_schedule(const DevKey& key, const uint8_t* nonce, FileParams& P) {
  uint32_t nw[6];
#pragma unroll
  for (int i = 0; i < 6; i++) nw[i] = ld_le32(nonce + 4 * i);
  key_schedule_w(key, nw, P);
}

// Segment bookkeeping of a file (lane per file).  Every lane of the wave calls it, `mine` =
// the lane holds a file to set up (the others only help): a file's (file, segment) work items go
// to extra_list, up to 32 by its own lane, longer runs (a 35 MB compaction has 2,200) by the
// whole wave, one file at a time.
__device__ __forceinline__ void reserve_segments(FileParams& P, uint32_t f, SegScratch sc, bool mine = true) {
  const uint64_t nblk = ((uint64_t)P.len + 15) / 16 + 1;
  const uint32_t nseg = mine ? (uint32_t)((nblk + sc.seg_blocks - 1) / sc.seg_blocks) : 0u;
  if (mine) {
    P.nseg = nseg;
    P.extra_base = 0;
  }
  uint32_t e = 0;
  if (nseg > 1) {
    e = atomicAdd(&sc.counters[0], nseg - 1);
    const uint32_t pb = atomicAdd(&sc.counters[6], nseg);
    const uint32_t mf = atomicAdd(&sc.counters[1], 1u);
    P.extra_base = pb;
    sc.multi_files[mf] = f;
    if (nseg <= 33)
      for (uint32_t j = 1; j < nseg; j++) sc.extra_list[e + j - 1] = make_uint2(f, j);
  }
  // the lanes running here (every lane of the wave, for the callers above): rank among them
  const unsigned long long act = __ballot(true);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t rank = (uint32_t)__builtin_popcountll(act & ((1ull << lane) - 1ull));
  const uint32_t nact = (uint32_t)__builtin_popcountll(act);
  for (unsigned long long big = __ballot(nseg > 33); big; big &= big - 1) {
    const int src = (int)__builtin_ctzll(big);
    const uint32_t fe = (uint32_t)__shfl((int)e, src), ff = (uint32_t)__shfl((int)f, src);
    const uint32_t fn = (uint32_t)__shfl((int)nseg, src);
    for (uint32_t j = 1 + rank; j < fn; j += nact) sc.extra_list[fe + j - 1] = make_uint2(ff, j);
  }
}


static constexpr int kKsStride = 80;  // LDS bytes per keystream block (64 + 16 pad: no conflicts)

__device__ __forceinline__ uint32_t bcast(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// atomicMax into the batch state, skipped when a plain read already shows a value >= v: the
// state only grows during a launch, so a stale (smaller) read costs at most a redundant atomic.
// Dots of many actors with random counters (C2 variant B) otherwise issue one L2 atomic each.
__device__ __forceinline__ void batch_max(unsigned long long* p, unsigned long long v) {
  if (v > *p) atomicMax(p, v);
}

__device__ __forceinline__ uint32_t lookup_slot(const ActorSlot* __restrict__ tab, uint32_t mask,
                                                uint32_t k0, uint32_t k1, uint32_t k2,
                                                uint32_t k3) {
  uint32_t h = actor_hash(k0, k1, k2, k3) & mask;
  for (uint32_t probe = 0; probe <= mask; probe++) {
    const uint4 a = *reinterpret_cast<const uint4*>(tab[h].k);
    const uint32_t used = tab[h].used;
    if (!used) return 0xffffffffu;
    if (a.x == k0 && a.y == k1 && a.z == k2 && a.w == k3) return h;
    h = (h + 1) & mask;
  }
  return 0xffffffffu;
}

// lookup_slot with one 16-byte load per probe: an empty slot's key is all zero (ActorSlot{}), and
// a used slot's key is zero only for the nil UUID, so the key alone decides unless the nil UUID
// is the key looked up or is in the table (nil_in_table: the host's probe at launch time).  C2
// variant B (a lookup per Dot) spends its time in these L2 requests.
__device__ __forceinline__ uint32_t lookup_slot1(const ActorSlot* __restrict__ tab, uint32_t mask,
                                                 int nil_in_table, uint32_t k0, uint32_t k1,
                                                 uint32_t k2, uint32_t k3) {
  if (nil_in_table || (k0 | k1 | k2 | k3) == 0) return lookup_slot(tab, mask, k0, k1, k2, k3);
  uint32_t h = actor_hash(k0, k1, k2, k3) & mask;
  for (uint32_t probe = 0; probe <= mask; probe++) {
    const uint4 a = *reinterpret_cast<const uint4*>(tab[h].k);
    if (a.x == k0 && a.y == k1 && a.z == k2 && a.w == k3) return h;
    if ((a.x | a.y | a.z | a.w) == 0) return 0xffffffffu;
    h = (h + 1) & mask;
  }
  return 0xffffffffu;
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// bytes [b, b+4) of a 48-byte window held as 12 LE words (b compile-time)
__device__ __forceinline__ uint32_t win_word(const uint32_t (&w)[12], int b) {
  const int i = b >> 2, s = b & 3;
  if (s == 0) return w[i];
  return __builtin_amdgcn_alignbyte(w[i + 1], w[i], s);
}

// canonical rmp-serde Dot: 82 a5"actor" c4 10 <16> a7"counter" <uint>: length from the marker
// (positive fixint 34; cc/cd/ce/cf = 34 + 1/2/4/8; anything else 0).  Branch-free.
__device__ __forceinline__ uint32_t dot_len_of_marker(uint32_t mk) {
  const uint32_t t = mk - 0xccu;
  return mk < 0x80u ? 34u : (t < 4u ? 34u + (1u << t) : 0u);
}

// check one canonical Dot of length L in the window w (bytes cand..cand+47); extract fields.
// Branch-free: every test is evaluated; the counter is one shift of the big-endian 8 bytes.
__device__ __forceinline__ bool canon_dot(const uint32_t (&w)[12], uint32_t L, uint32_t& k0,
                                          uint32_t& k1, uint32_t& k2, uint32_t& k3,
                                          unsigned long long& ctr) {
  const uint32_t mk = (w[8] >> 8) & 0xff;
  const uint32_t Lc = dot_len_of_marker(mk);
  const uint32_t ok = (uint32_t)(w[0] == 0x6361a582u) & (uint32_t)(w[1] == 0xc4726f74u) &
                      (uint32_t)((w[2] & 0xffu) == 0x10u) &
                      (uint32_t)(win_word(w, 25) == 0x756f63a7u) &
                      (uint32_t)(win_word(w, 29) == 0x7265746eu) & (uint32_t)(Lc == L);
  k0 = win_word(w, 9); k1 = win_word(w, 13); k2 = win_word(w, 17); k3 = win_word(w, 21);
  const unsigned long long be =
      ((unsigned long long)bswap32(win_word(w, 34)) << 32) | bswap32(win_word(w, 38));
  const uint32_t t = (mk - 0xccu) & 3u;   // cc..cf -> 1, 2, 4, 8 bytes
  ctr = mk < 0x80u ? (unsigned long long)mk : be >> (64u - (8u << t));
  return ok != 0;
}

}  // namespace ce
