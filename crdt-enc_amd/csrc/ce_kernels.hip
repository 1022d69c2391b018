// ce_kernels.hip -- gfx950 kernels of the compaction/ingest hot path.
//
//  k_open_setup     one lane per file: outer version (crdt-enc/src/lib.rs:501), envelope parse
//                   (crdt-enc-xchacha20poly1305/src/lib.rs:82-91), HChaCha20 subkey, Poly1305
//                   key (ChaCha20 block 0) and r^(2^k) k=0..6.
//  k_seal_setup     one lane per file: writes CURRENT_VERSION || msgpack header
//                   (xchacha lib.rs:59-67, crdt-enc/src/lib.rs:695), key schedule.
//  k_segments       one wavefront per 16 KiB segment: ChaCha20 keystream (one 64-byte block
//                   per lane, transposed through LDS), coalesced 16-byte pieces, Poly1305 as a
//                   64-way strided Horner in r^64 + a 6-level cross-lane tree in r^(2^k);
//                   single-segment files finalize in place (tag compare, scrub on failure).
//  k_finalize_multi one lane per multi-segment file: Horner over segment partials.
//  k_decode_dots    one wavefront per file: rmp-serde Vec<Dot<Uuid>> (crdt-enc/src/lib.rs:507)
//                   decoded 64 dots at a time by speculating on the canonical encoding, general
//                   grammar by lane 0 otherwise; dots of applied files max-folded
//                   (VClock::apply) into a dense batch state.
#include "ce_kernels.h"

namespace ce {

// ----------------------------------------------------------------------------------------
// ChaCha20 (RFC 8439 §2.3) / HChaCha20 (draft-irtf-cfrg-xchacha-03 §2.2)
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int c) {
  return __builtin_amdgcn_alignbit(x, x, 32 - c);
}

#define CE_QR(a, b, c, d)                                                                   \
  a += b; d ^= a; d = rotl32(d, 16); c += d; b ^= c; b = rotl32(b, 12);                    \
  a += b; d ^= a; d = rotl32(d, 8);  c += d; b ^= c; b = rotl32(b, 7);

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
  m.v[4] = (w3 >> 8) | (1u << 24);
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

// key schedule shared by open/seal setup: subkey, (r, s), r^(2^k)
__device__ void key_schedule(const DevKey& key, const uint8_t* nonce, FileParams& P) {
  uint32_t k[8], n16[4], sub[8];
#pragma unroll
  for (int i = 0; i < 8; i++) k[i] = key.k[i];
#pragma unroll
  for (int i = 0; i < 4; i++) n16[i] = ld_le32(nonce + 4 * i);
  hchacha20(k, n16, sub);
  const uint32_t n2a = ld_le32(nonce + 16), n2b = ld_le32(nonce + 20);
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
  for (int kk = 1; kk < 7; kk++) {
    p = mulmod(p, p);
#pragma unroll
    for (int i = 0; i < 5; i++) P.rpow[kk][i] = p.v[i];
  }
}

__device__ __forceinline__ void reserve_segments(FileParams& P, uint32_t f, SegScratch sc) {
  const uint64_t nblk = ((uint64_t)P.len + 15) / 16 + 1;
  const uint32_t nseg = (uint32_t)((nblk + kSegBlocks - 1) / kSegBlocks);
  P.nseg = nseg;
  P.extra_base = 0;
  if (nseg > 1) {
    const uint32_t e = atomicAdd(&sc.counters[0], nseg - 1);
    const uint32_t pb = atomicAdd(&sc.counters[6], nseg);
    const uint32_t mf = atomicAdd(&sc.counters[1], 1u);
    P.extra_base = pb;
    sc.multi_files[mf] = f;
    for (uint32_t j = 1; j < nseg; j++) sc.extra_list[e + j - 1] = make_uint2(f, j);
  }
}

// ----------------------------------------------------------------------------------------
// setup kernels
// ----------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_open_setup(const uint8_t* __restrict__ blob,
                                                    const uint64_t* __restrict__ offs, uint32_t n,
                                                    int outer, DevKey key, int32_t key_status,
                                                    FileParams* __restrict__ params,
                                                    int32_t* __restrict__ status, SegScratch sc) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n) return;
  const uint64_t off = offs[f];
  const uint64_t flen = offs[f + 1] - off;
  const uint8_t* enc = blob + off;
  uint64_t enc_len = flen;
  int32_t st = CE_OK;
  if (outer) {
    // Storage: VersionBytes::deserialize (tokio lib.rs:241), then the core's
    // ensure_versions_phf(SUPPORTED_VERSIONS) (crdt-enc/src/lib.rs:501)
    if (flen < 16) st = CE_ERR_OUTER_LEN;
    else {
      for (int i = 0; i < 16; i++)
        if (enc[i] != kCoreVersion[i]) { st = CE_ERR_OUTER_VERSION; break; }
      enc += 16;
      enc_len -= 16;
    }
  }
  if (st == CE_OK) st = key_status;  // key version / length (xchacha lib.rs:74-78)
  Envelope e{};
  if (st == CE_OK) st = parse_envelope(enc, enc_len, &e);
  FileParams P;
  P.status = st;
  P.len = 0;
  P.in_off = 0;
  P.out_off = (off + 15) & ~15ull;
  P.nseg = 0;
  P.extra_base = 0;
  if (st == CE_OK) {
    const uint64_t ct_off = (uint64_t)(enc - blob) + e.enc_off;
    P.in_off = ct_off;
    P.len = (uint32_t)(e.enc_len - 16);
    const uint8_t* t = blob + ct_off + P.len;
    for (int i = 0; i < 4; i++) P.tag[i] = ld_le32(t + 4 * i);
    key_schedule(key, enc + e.nonce_off, P);
    reserve_segments(P, f, sc);
  }
  params[f] = P;
  status[f] = st;
  if (st == kStatusHostParse) atomicAdd(&sc.counters[7], 1u);
  else if (st != CE_OK) {
    atomicAdd(&sc.counters[8], 1u);
    atomicMin(&sc.counters[5], f);
  }
}

__global__ __launch_bounds__(256) void k_seal_setup(const uint8_t* __restrict__ clear,
                                                    const uint64_t* __restrict__ offs, uint32_t n,
                                                    const uint8_t* __restrict__ outer_version,
                                                    const uint8_t* __restrict__ nonces,
                                                    uint8_t* __restrict__ out,
                                                    const uint64_t* __restrict__ out_offs,
                                                    DevKey key, FileParams* __restrict__ params,
                                                    SegScratch sc) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n) return;
  const uint64_t off = offs[f];
  const uint64_t len = offs[f + 1] - off;
  uint8_t* o = out + out_offs[f];
  uint64_t k = 0;
  if (outer_version) {
    for (int i = 0; i < 16; i++) o[i] = outer_version[i];
    k = 16;
  }
  uint8_t hdr[96];
  const uint8_t* nonce = nonces + 24ull * f;
  uint8_t nb[24];
  for (int i = 0; i < 24; i++) nb[i] = nonce[i];
  const uint64_t h = put_envelope_header(hdr, len, nb);
  for (uint64_t i = 0; i < h; i++) o[k + i] = hdr[i];
  FileParams P;
  P.status = CE_OK;
  P.in_off = off;
  P.out_off = out_offs[f] + k + h;
  P.len = (uint32_t)len;
  key_schedule(key, nb, P);
  reserve_segments(P, f, sc);
  params[f] = P;
}

// ----------------------------------------------------------------------------------------
// segment kernel: one wavefront per (file, 16 KiB segment)
// ----------------------------------------------------------------------------------------
static constexpr int kWavesPerBlock = 4;
static constexpr int kKsStride = 80;  // LDS bytes per keystream block (64 + 16 pad: no conflicts)

__device__ __forceinline__ uint32_t bcast(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

template <bool SEAL>
__global__ __launch_bounds__(256) void k_segments(const uint8_t* __restrict__ in,
                                                  uint8_t* __restrict__ out,
                                                  const FileParams* __restrict__ params, uint32_t n,
                                                  int32_t* __restrict__ status, SegScratch sc) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWavesPerBlock * 64 * kKsStride];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wib = threadIdx.x >> 6;
  uint8_t* ks = lds + wib * 64 * kKsStride;
  const uint32_t total = n + *((volatile uint32_t*)&sc.counters[0]);
  const uint32_t stride = gridDim.x * kWavesPerBlock;

  for (uint32_t w = bcast(blockIdx.x * kWavesPerBlock + wib); w < total; w += stride) {
    uint32_t f, j;
    if (w < n) { f = w; j = 0; }
    else { const uint2 e = sc.extra_list[w - n]; f = bcast(e.x); j = bcast(e.y); }
    const FileParams* Pp = params + f;
    if (Pp->status != CE_OK) continue;  // setup status (never rewritten: read-only here)
    const uint32_t len = Pp->len;
    const uint32_t nseg = Pp->nseg;
    uint32_t key[8];
#pragma unroll
    for (int i = 0; i < 8; i++) key[i] = Pp->subkey[i];
    const uint32_t n2a = Pp->n2[0], n2b = Pp->n2[1];
    const L5 R = load_l5(Pp->rpow[6]);
    const uint8_t* src = in + Pp->in_off;
    uint8_t* dst = out + Pp->out_off;

    const uint32_t nblk_ct = (len + 15) >> 4;
    const uint32_t nblk = nblk_ct + 1;
    const uint32_t b_lo = j * kSegBlocks;
    const uint32_t b_hi = min(nblk, b_lo + kSegBlocks);
    const uint32_t nb = b_hi - b_lo;
    const uint32_t rows = (nb + 63) >> 6;

    L5 acc = {{0, 0, 0, 0, 0}};
    for (uint32_t row = 0; row < rows; row++) {
      const uint32_t rb = b_lo + row * 64;  // first block of this row
      if ((row & 3) == 0) {
        const uint32_t page_byte = rb * 16;
        __builtin_amdgcn_wave_barrier();
        if (page_byte < len) {
          uint32_t kb[16];
          chacha_block(key, 1u + (page_byte >> 6) + lane, 0u, n2a, n2b, kb);
          uint4* kd = reinterpret_cast<uint4*>(ks + lane * kKsStride);
          kd[0] = make_uint4(kb[0], kb[1], kb[2], kb[3]);
          kd[1] = make_uint4(kb[4], kb[5], kb[6], kb[7]);
          kd[2] = make_uint4(kb[8], kb[9], kb[10], kb[11]);
          kd[3] = make_uint4(kb[12], kb[13], kb[14], kb[15]);
        }
        __builtin_amdgcn_wave_barrier();
      }
      const uint32_t blk = rb + lane;
      if (blk < nblk_ct) {
        const uint32_t boff = blk * 16;
        const uint32_t q = (row & 3) * 64 + lane;  // piece within the page
        const uint4 k4 = *reinterpret_cast<const uint4*>(ks + (q >> 2) * kKsStride + (q & 3) * 16);
        uint4 x;
        const bool full = boff + 16 <= len;
        if (full) {
          x = *reinterpret_cast<const uint4*>(src + boff);
        } else {
          uint32_t wv[4] = {0, 0, 0, 0};
          for (uint32_t b = 0; b < len - boff; b++) wv[b >> 2] |= (uint32_t)src[boff + b] << (8 * (b & 3));
          x = make_uint4(wv[0], wv[1], wv[2], wv[3]);
        }
        uint4 y = make_uint4(x.x ^ k4.x, x.y ^ k4.y, x.z ^ k4.z, x.w ^ k4.w);
        if (full) {
          *reinterpret_cast<uint4*>(dst + boff) = y;
        } else {
          const uint32_t rem = len - boff;
          const uint32_t wv[4] = {y.x, y.y, y.z, y.w};
          for (uint32_t b = 0; b < rem; b++) dst[boff + b] = (uint8_t)(wv[b >> 2] >> (8 * (b & 3)));
          // zero the pad bytes of the MAC input
          uint32_t mw[4];
          const uint32_t c[4] = {SEAL ? y.x : x.x, SEAL ? y.y : x.y, SEAL ? y.z : x.z, SEAL ? y.w : x.w};
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const int lo = 4 * i;
            const uint32_t keep = rem >= (uint32_t)(lo + 4) ? 0xffffffffu
                                  : (rem <= (uint32_t)lo ? 0u : ((1u << (8 * (rem - lo))) - 1));
            mw[i] = c[i] & keep;
          }
          if (SEAL) y = make_uint4(mw[0], mw[1], mw[2], mw[3]);
          else x = make_uint4(mw[0], mw[1], mw[2], mw[3]);
        }
        const uint4 m = SEAL ? y : x;
        acc = add5(mulmod(acc, R), block_limbs(m.x, m.y, m.z, m.w));
      } else if (blk == nblk_ct) {
        // length block: le64(aad_len = 0) || le64(ct_len)
        acc = add5(mulmod(acc, R), block_limbs(0u, 0u, len, 0u));
      }
    }
    // rotate so position p = lane holds the lane whose last block has weight r^(64 - p)
    L5 v;
    {
      const int srcl = (int)((lane + nb) & 63);
#pragma unroll
      for (int i = 0; i < 5; i++) v.v[i] = __shfl(acc.v[i], srcl);
    }
#pragma unroll
    for (int k = 0; k < 6; k++) {
      const L5 rk = load_l5(Pp->rpow[k]);
      L5 o;
#pragma unroll
      for (int i = 0; i < 5; i++) o.v[i] = __shfl_down(v.v[i], 1u << k);
      v = carry5(add5(mulmod(v, rk), o));
    }
    L5 tot = mulmod(v, load_l5(Pp->rpow[0]));
#pragma unroll
    for (int i = 0; i < 5; i++) tot.v[i] = bcast(tot.v[i]);

    if (nseg == 1) {
      const uint32_t sv[4] = {Pp->s[0], Pp->s[1], Pp->s[2], Pp->s[3]};
      uint32_t tag[4];
      poly_tag(tot, sv, tag);
      if (SEAL) {
        if (lane < 4) {
          const uint32_t tv = lane == 0 ? tag[0] : lane == 1 ? tag[1] : lane == 2 ? tag[2] : tag[3];
          uint8_t* tp = dst + len + 4 * lane;
          tp[0] = (uint8_t)tv; tp[1] = (uint8_t)(tv >> 8); tp[2] = (uint8_t)(tv >> 16);
          tp[3] = (uint8_t)(tv >> 24);
        }
      } else {
        const bool ok = ((tag[0] ^ Pp->tag[0]) | (tag[1] ^ Pp->tag[1]) | (tag[2] ^ Pp->tag[2]) |
                         (tag[3] ^ Pp->tag[3])) == 0;
        if (!ok) {
          // verify-before-release: scrub the speculative plaintext
          for (uint32_t b = lane * 16; b < len; b += 64 * 16) {
            if (b + 16 <= len) *reinterpret_cast<uint4*>(dst + b) = make_uint4(0, 0, 0, 0);
            else for (uint32_t t = b; t < len; t++) dst[t] = 0;
          }
          if (lane == 0) {
            status[f] = CE_ERR_AUTH;
            atomicAdd(&sc.counters[2], 1u);
            atomicMin(&sc.counters[5], f);
          }
        }
      }
    } else if (lane == 0) {
      uint32_t* pp = sc.partials + 5ull * (Pp->extra_base + j);
#pragma unroll
      for (int i = 0; i < 5; i++) pp[i] = tot.v[i];
    }
  }
}

// ----------------------------------------------------------------------------------------
// multi-segment finalize: one lane per multi-segment file (grid-stride)
// ----------------------------------------------------------------------------------------
__device__ L5 rpow_any(const FileParams& P, uint32_t e) {
  // r^e, 1 <= e <= 1024, from r^(2^k) (k <= 6) and further squarings
  L5 acc = {{1, 0, 0, 0, 0}};
  L5 p = load_l5(P.rpow[0]);
  for (int k = 0; k < 11; k++) {
    if (k <= 6) p = load_l5(P.rpow[k]);
    else p = mulmod(p, p);
    if (e & (1u << k)) acc = mulmod(acc, p);
  }
  return acc;
}

template <bool SEAL>
__global__ __launch_bounds__(256) void k_finalize_multi(uint8_t* __restrict__ out,
                                                        const FileParams* __restrict__ params,
                                                        int32_t* __restrict__ status,
                                                        SegScratch sc) {
  const uint32_t nm = sc.counters[1];
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < nm; t += gridDim.x * blockDim.x) {
    const uint32_t f = sc.multi_files[t];
    const FileParams& P = params[f];
    const uint32_t nblk = ((P.len + 15) >> 4) + 1;
    const L5 rseg = rpow_any(P, kSegBlocks);
    L5 acc = load_l5(sc.partials + 5ull * P.extra_base);
    for (uint32_t j = 1; j < P.nseg; j++) {
      const uint32_t nb = min(nblk - j * kSegBlocks, kSegBlocks);
      const L5 rj = nb == kSegBlocks ? rseg : rpow_any(P, nb);
      acc = carry5(add5(mulmod(acc, rj), load_l5(sc.partials + 5ull * (P.extra_base + j))));
    }
    uint32_t tag[4];
    const uint32_t sv[4] = {P.s[0], P.s[1], P.s[2], P.s[3]};
    poly_tag(acc, sv, tag);
    uint8_t* dst = out + P.out_off;
    if (SEAL) {
      for (int i = 0; i < 16; i++) dst[P.len + i] = (uint8_t)(tag[i >> 2] >> (8 * (i & 3)));
    } else {
      const bool ok = ((tag[0] ^ P.tag[0]) | (tag[1] ^ P.tag[1]) | (tag[2] ^ P.tag[2]) |
                       (tag[3] ^ P.tag[3])) == 0;
      if (!ok) {
        for (uint32_t b = 0; b < P.len; b++) dst[b] = 0;
        status[f] = CE_ERR_AUTH;
        atomicAdd(&sc.counters[2], 1u);
        atomicMin(&sc.counters[5], f);
      }
    }
  }
}

// ----------------------------------------------------------------------------------------
// decode + fold: one wavefront per file
// ----------------------------------------------------------------------------------------
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

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// bytes [b, b+4) of a 48-byte window held as 12 LE words (b compile-time or uniform small)
__device__ __forceinline__ uint32_t win_word(const uint32_t (&w)[12], int b) {
  const int i = b >> 2, s = b & 3;
  if (s == 0) return w[i];
  return __builtin_amdgcn_alignbyte(w[i + 1], w[i], s);
}

struct FoldState {
  uint32_t slot;             // wave-uniform pending slot (0xffffffff = none)
  unsigned long long best;   // pending max
};

__device__ __forceinline__ void fold_lane(const DecodeArgs& a, uint32_t f, bool active,
                                          uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3,
                                          unsigned long long ctr, FoldState& fs) {
  uint32_t slot = 0xffffffffu;
  if (active) {
    slot = lookup_slot(a.table, a.mask, k0, k1, k2, k3);
    if (slot == 0xffffffffu) {
      const uint32_t mi = atomicAdd(&a.counters[4], 1u);
      if (mi < a.miss_cap) a.miss_list[mi] = make_uint4(k0, k1, k2, k3);
      a.refold[f] = 1;
    }
  }
  const bool live = active && slot != 0xffffffffu;
  // common case: every live lane folds into one slot -> one wave max, one pending update
  const uint32_t first_live = __builtin_ctzll(__ballot(live) | (1ull << 63));
  const uint32_t s0 = __shfl(slot, first_live);
  const bool same = __ballot(live && slot != s0) == 0;
  if (same && __ballot(live) != 0) {
    unsigned long long v = live ? ctr : 0ull;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      const unsigned long long o = __shfl_xor(v, d);
      v = o > v ? o : v;
    }
    if (fs.slot != s0) {
      if (fs.slot != 0xffffffffu && __lane_id() == 0) atomicMax(&a.batch[fs.slot], fs.best);
      fs.slot = s0;
      fs.best = v;
    } else if (v > fs.best) {
      fs.best = v;
    }
  } else if (live) {
    atomicMax(&a.batch[slot], ctr);
  }
}

__device__ __forceinline__ void fold_flush(const DecodeArgs& a, FoldState& fs) {
  if (fs.slot != 0xffffffffu && __lane_id() == 0) atomicMax(&a.batch[fs.slot], fs.best);
  fs.slot = 0xffffffffu;
  fs.best = 0;
}

__global__ __launch_bounds__(256) void k_decode_dots(DecodeArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t stride = gridDim.x * kWavesPerBlock;
  for (uint32_t f = bcast(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)); f < a.n; f += stride) {
    if (a.only && !a.only[f]) continue;
    const FileParams* Pp = a.params + f;
    if (a.status[f] != CE_OK) continue;
    const uint8_t* pt = a.pt + Pp->out_off;
    const uint32_t len = Pp->len;
    int32_t st = CE_OK;
    // clear text = VersionBytes(data_version, msgpack(Vec<Op>)) (crdt-enc/src/lib.rs:504-507)
    if (len < 16) st = CE_ERR_PT_LEN;
    else {
      const uint4 dv = *reinterpret_cast<const uint4*>(pt);
      bool found = false;
      for (uint32_t s = 0; s < a.n_supported; s++) {
        const uint4 sv = *reinterpret_cast<const uint4*>(a.supported + 16 * s);
        found |= dv.x == sv.x && dv.y == sv.y && dv.z == sv.z && dv.w == sv.w;
      }
      if (!found) st = CE_ERR_PT_VERSION;
    }
    const bool do_fold = st == CE_OK && (a.apply == nullptr || a.apply[f]);
    FoldState fs{0xffffffffu, 0ull};
    if (st == CE_OK) {
      const uint8_t* body = pt + 16;
      const uint32_t blen = len - 16;
      Rd r{body, blen, 0};
      uint64_t count = 0;
      if (!rd_array_hdr(r, &count)) st = CE_ERR_DECODE;
      uint32_t pos = (uint32_t)r.i;
      uint64_t remaining = st == CE_OK ? count : 0;
      if (remaining > blen) st = CE_ERR_DECODE, remaining = 0;  // each Dot takes >= 1 byte
      while (remaining > 0 && st == CE_OK) {
        // canonical rmp-serde Dot: 82 a5"actor" c4 10 <16> a7"counter" <uint>  (33 + 1..9 bytes)
        uint32_t L = 0;
        if (pos + 34 <= blen) {
          const uint8_t mk = body[pos + 33];
          L = mk <= 0x7f ? 34 : mk == 0xcc ? 35 : mk == 0xcd ? 36 : mk == 0xce ? 38 : mk == 0xcf ? 42 : 0;
        }
        bool valid = false;
        uint32_t k0 = 0, k1 = 0, k2 = 0, k3 = 0;
        unsigned long long ctr = 0;
        if (L) {
          const uint32_t cand = pos + lane * L;
          if (lane < remaining && cand + L <= blen) {
            uint32_t w[12];
            const uint4 A = *reinterpret_cast<const uint4*>(body + cand);
            const uint4 B = *reinterpret_cast<const uint4*>(body + cand + 16);
            const uint4 C = *reinterpret_cast<const uint4*>(body + cand + 32);
            w[0] = A.x; w[1] = A.y; w[2] = A.z; w[3] = A.w;
            w[4] = B.x; w[5] = B.y; w[6] = B.z; w[7] = B.w;
            w[8] = C.x; w[9] = C.y; w[10] = C.z; w[11] = C.w;
            const uint32_t mk = (w[8] >> 8) & 0xff;
            const uint32_t Lc = mk <= 0x7f ? 34 : mk == 0xcc ? 35 : mk == 0xcd ? 36 : mk == 0xce ? 38 : mk == 0xcf ? 42 : 0;
            valid = w[0] == 0x6361a582u && w[1] == 0xc4726f74u && (w[2] & 0xffu) == 0x10u &&
                    win_word(w, 25) == 0x756f63a7u && win_word(w, 29) == 0x7265746eu && Lc == L;
            k0 = win_word(w, 9); k1 = win_word(w, 13); k2 = win_word(w, 17); k3 = win_word(w, 21);
            const uint32_t hi = bswap32(win_word(w, 34)), lo = bswap32(win_word(w, 38));
            ctr = L == 34 ? mk
                : L == 35 ? (hi >> 24)
                : L == 36 ? (hi >> 16)
                : L == 38 ? hi
                : (((unsigned long long)hi << 32) | lo);
          }
        }
        const unsigned long long vm = __ballot(valid);
        // leading run of valid lanes (ctz of 0 is undefined: all 64 valid -> 64)
        const uint32_t k = vm == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~vm);
        if (k > 0) {
          if (do_fold) fold_lane(a, f, lane < k, k0, k1, k2, k3, ctr, fs);
          pos += k * L;
          remaining -= k;
        } else {
          // general grammar for one element (lane 0), e.g. reordered keys / array form
          int ok = 0;
          uint32_t g0 = 0, g1 = 0, g2 = 0, g3 = 0;
          unsigned long long gc = 0;
          uint32_t npos = pos;
          if (lane == 0) {
            Rd q{body, blen, pos};
            uint64_t aoff = 0, c = 0;
            ok = parse_dot(q, &aoff, &c);
            if (ok == 1) {
              g0 = ld_le32(body + aoff); g1 = ld_le32(body + aoff + 4);
              g2 = ld_le32(body + aoff + 8); g3 = ld_le32(body + aoff + 12);
              gc = c;
              npos = (uint32_t)q.i;
            }
          }
          ok = __shfl(ok, 0);
          if (ok != 1) { st = CE_ERR_DECODE; break; }
          npos = bcast(npos);
          if (do_fold) fold_lane(a, f, lane == 0, g0, g1, g2, g3, gc, fs);
          pos = npos;
          remaining -= 1;
        }
      }
      if (do_fold) fold_flush(a, fs);
    }
    if (st != CE_OK && lane == 0) {
      a.status[f] = st;
      atomicAdd(&a.counters[3], 1u);
      atomicMin(&a.counters[5], f);
    }
  }
}

__global__ void k_merge_max(unsigned long long* __restrict__ dst,
                            const unsigned long long* __restrict__ src, uint32_t n) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const unsigned long long s = src[i];
    if (s > dst[i]) dst[i] = s;
  }
}

// ----------------------------------------------------------------------------------------
// launchers
// ----------------------------------------------------------------------------------------
hipError_t launch_open_setup(hipStream_t s, const uint8_t* blob, const uint64_t* offs, uint32_t n,
                             bool outer, DevKey key, int32_t key_status, FileParams* params,
                             int32_t* status, SegScratch sc) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_open_setup, dim3((n + 255) / 256), dim3(256), 0, s, blob, offs, n,
                     outer ? 1 : 0, key, key_status, params, status, sc);
  return hipGetLastError();
}

hipError_t launch_seal_setup(hipStream_t s, const uint8_t* clear, const uint64_t* offs, uint32_t n,
                             const uint8_t* outer_version, const uint8_t* nonces, uint8_t* out,
                             const uint64_t* out_offs, DevKey key, FileParams* params,
                             SegScratch sc) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_seal_setup, dim3((n + 255) / 256), dim3(256), 0, s, clear, offs, n,
                     outer_version, nonces, out, out_offs, key, params, sc);
  return hipGetLastError();
}

hipError_t launch_segments(hipStream_t s, bool seal, const uint8_t* in, uint8_t* out,
                           const FileParams* params, uint32_t n, int32_t* status, SegScratch sc,
                           uint32_t grid_waves) {
  if (n == 0) return hipSuccess;
  const uint32_t blocks = (grid_waves + kWavesPerBlock - 1) / kWavesPerBlock;
  if (seal)
    hipLaunchKernelGGL(k_segments<true>, dim3(blocks), dim3(256), 0, s, in, out, params, n,
                       status, sc);
  else
    hipLaunchKernelGGL(k_segments<false>, dim3(blocks), dim3(256), 0, s, in, out, params, n,
                       status, sc);
  return hipGetLastError();
}

hipError_t launch_finalize_multi(hipStream_t s, bool seal, uint8_t* out, const FileParams* params,
                                 int32_t* status, SegScratch sc) {
  if (seal)
    hipLaunchKernelGGL(k_finalize_multi<true>, dim3(64), dim3(256), 0, s, out, params, status, sc);
  else
    hipLaunchKernelGGL(k_finalize_multi<false>, dim3(64), dim3(256), 0, s, out, params, status, sc);
  return hipGetLastError();
}

hipError_t launch_decode_dots(hipStream_t s, const DecodeArgs& a, uint32_t grid_waves) {
  if (a.n == 0) return hipSuccess;
  const uint32_t blocks = (grid_waves + kWavesPerBlock - 1) / kWavesPerBlock;
  hipLaunchKernelGGL(k_decode_dots, dim3(blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_merge_max(hipStream_t s, unsigned long long* dst, const unsigned long long* src,
                            uint32_t n) {
  if (n == 0) return hipSuccess;
  const uint32_t blocks = min((n + 255) / 256, 1024u);
  hipLaunchKernelGGL(k_merge_max, dim3(blocks), dim3(256), 0, s, dst, src, n);
  return hipGetLastError();
}

}  // namespace ce
