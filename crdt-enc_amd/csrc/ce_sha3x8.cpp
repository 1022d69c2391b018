// ce_sha3x8.cpp -- SHA3-256 of up to eight messages at once, one per 64-bit lane of AVX-512
// registers (multi-buffer Keccak-f[1600]: the 25 state words of the eight sponges in 25 zmm
// registers, every step lane-wise, pi a renaming of registers).
//
// A compaction's content name is the SHA3-256 of its sealed file (crdt-enc-tokio/src/lib.rs:
// 403-432), a sequential sponge: ~48 ms per 35 MB file on one core of the GPU box (OpenSSL,
// ~7 cycles/byte).  Pipelined compactions produce one such file every ~2.6 ms, so the names --
// not the GPU -- bounded the C3 step.  Eight sponges per core in the time of about one make the
// hashing a small fraction of the host.  Messages may differ in length: the common
// full blocks run eight-wide, each message's remainder and padding finish on its own sponge
// (the portable permutation in ce_storage.cpp).  Without AVX-512F: sha3_256 per message.
#include <immintrin.h>
#include <stdint.h>
#include <string.h>

#include <string>

#include "ce_core.h"

namespace ce {
void keccakf_portable(uint64_t s[25]);  // ce_storage.cpp
void sha3_256(const uint8_t* msg, size_t len, uint8_t out[32]);
std::string base32_nopad(const uint8_t* in, size_t len);

namespace {

constexpr uint64_t kRCx8[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull, 0x8000000080008000ull,
    0x000000000000808bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
    0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800aull, 0x800000008000000aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

#define CE_ROL(x, n) ((n) ? _mm512_rol_epi64((x), (n)) : (x))

__attribute__((target("avx512f"))) inline void keccakf_x8(__m512i s[25]) {
  for (int r = 0; r < 24; r++) {
    __m512i c[5], d[5], b[25];
#define CE_C(x) c[x] = _mm512_ternarylogic_epi64(_mm512_ternarylogic_epi64(s[x], s[x + 5], s[x + 10], 0x96), s[x + 15], s[x + 20], 0x96)
    CE_C(0); CE_C(1); CE_C(2); CE_C(3); CE_C(4);
#undef CE_C
#define CE_D(x) d[x] = _mm512_xor_si512(c[((x) + 4) % 5], _mm512_rol_epi64(c[((x) + 1) % 5], 1))
    CE_D(0); CE_D(1); CE_D(2); CE_D(3); CE_D(4);
#undef CE_D
    // theta + rho + pi: B[y, 2x + 3y] = rot(A[x, y] ^ D[x], r[x, y])
#define CE_B(x, y, rho) b[(y) + 5 * ((2 * (x) + 3 * (y)) % 5)] = CE_ROL(_mm512_xor_si512(s[(x) + 5 * (y)], d[x]), rho)
    CE_B(0, 0, 0);  CE_B(1, 0, 1);  CE_B(2, 0, 62); CE_B(3, 0, 28); CE_B(4, 0, 27);
    CE_B(0, 1, 36); CE_B(1, 1, 44); CE_B(2, 1, 6);  CE_B(3, 1, 55); CE_B(4, 1, 20);
    CE_B(0, 2, 3);  CE_B(1, 2, 10); CE_B(2, 2, 43); CE_B(3, 2, 25); CE_B(4, 2, 39);
    CE_B(0, 3, 41); CE_B(1, 3, 45); CE_B(2, 3, 15); CE_B(3, 3, 21); CE_B(4, 3, 8);
    CE_B(0, 4, 18); CE_B(1, 4, 2);  CE_B(2, 4, 61); CE_B(3, 4, 56); CE_B(4, 4, 14);
#undef CE_B
    // chi: a ^ (~b & c) as one ternary-logic op (0xD2); iota
#define CE_CHI(y, x) s[(y) + (x)] = _mm512_ternarylogic_epi64(b[(y) + (x)], b[(y) + ((x) + 1) % 5], b[(y) + ((x) + 2) % 5], 0xD2)
#define CE_ROW(y) CE_CHI(y, 0); CE_CHI(y, 1); CE_CHI(y, 2); CE_CHI(y, 3); CE_CHI(y, 4)
    CE_ROW(0); CE_ROW(5); CE_ROW(10); CE_ROW(15); CE_ROW(20);
#undef CE_ROW
#undef CE_CHI
    s[0] = _mm512_xor_si512(s[0], _mm512_set1_epi64((long long)kRCx8[r]));
  }
}

// 8x8 transpose of 64-bit words: c[i] lane j = row j word i
__attribute__((target("avx512f"))) inline void transpose8(__m512i r0, __m512i r1, __m512i r2, __m512i r3, __m512i r4,
                                                           __m512i r5, __m512i r6, __m512i r7, __m512i c[8]) {
  const __m512i t0 = _mm512_unpacklo_epi64(r0, r1), t1 = _mm512_unpackhi_epi64(r0, r1);
  const __m512i t2 = _mm512_unpacklo_epi64(r2, r3), t3 = _mm512_unpackhi_epi64(r2, r3);
  const __m512i t4 = _mm512_unpacklo_epi64(r4, r5), t5 = _mm512_unpackhi_epi64(r4, r5);
  const __m512i t6 = _mm512_unpacklo_epi64(r6, r7), t7 = _mm512_unpackhi_epi64(r6, r7);
  const __m512i u0 = _mm512_shuffle_i64x2(t0, t2, 0x88), u1 = _mm512_shuffle_i64x2(t0, t2, 0xDD);
  const __m512i u2 = _mm512_shuffle_i64x2(t1, t3, 0x88), u3 = _mm512_shuffle_i64x2(t1, t3, 0xDD);
  const __m512i u4 = _mm512_shuffle_i64x2(t4, t6, 0x88), u5 = _mm512_shuffle_i64x2(t4, t6, 0xDD);
  const __m512i u6 = _mm512_shuffle_i64x2(t5, t7, 0x88), u7 = _mm512_shuffle_i64x2(t5, t7, 0xDD);
  c[0] = _mm512_shuffle_i64x2(u0, u4, 0x88);
  c[4] = _mm512_shuffle_i64x2(u0, u4, 0xDD);
  c[2] = _mm512_shuffle_i64x2(u1, u5, 0x88);
  c[6] = _mm512_shuffle_i64x2(u1, u5, 0xDD);
  c[1] = _mm512_shuffle_i64x2(u2, u6, 0x88);
  c[5] = _mm512_shuffle_i64x2(u2, u6, 0xDD);
  c[3] = _mm512_shuffle_i64x2(u3, u7, 0x88);
  c[7] = _mm512_shuffle_i64x2(u3, u7, 0xDD);
}

__attribute__((target("avx512f"))) void sha3_256_x8_avx512(const uint8_t* const* msg, const size_t* len, int n,
                                                            uint8_t out[][32]) {
  constexpr size_t rate = 136;
  size_t common = ~(size_t)0;
  for (int j = 0; j < n; j++) common = len[j] / rate < common ? len[j] / rate : common;
  __m512i s[25];
  for (int i = 0; i < 25; i++) s[i] = _mm512_setzero_si512();
  // lane j reads message j (lanes past n repeat message 0; their results are dropped)
  long long base[8];
  for (int j = 0; j < 8; j++) base[j] = (long long)(uintptr_t)msg[j < n ? j : 0];
  __m512i addr = _mm512_loadu_si512(base);
  const __m512i step = _mm512_set1_epi64((long long)rate);
  const uint8_t* pf[8];
  for (int j = 0; j < 8; j++) pf[j] = msg[j < n ? j : 0];
  for (size_t blk = 0; blk < common; blk++) {
    // the eight streams' blocks 6 ahead into L1 (the gathers alone leave the prefetchers idle:
    // eight sponges ran at 1.4 GB/s of input without this)
    if (blk + 6 < common) {
      const size_t o = (blk + 6) * rate;
      for (int j = 0; j < n; j++) {
        _mm_prefetch((const char*)pf[j] + o, _MM_HINT_T0);
        _mm_prefetch((const char*)pf[j] + o + 64, _MM_HINT_T0);
        _mm_prefetch((const char*)pf[j] + o + 128, _MM_HINT_T0);
      }
    }
    // words 0-15: each message's two 64-byte rows, transposed 8x8 (a gather per word was most of
    // the time: eight scattered lines per instruction), word 16 by one gather
    const size_t o = blk * rate;
#pragma GCC unroll 2
    for (int h = 0; h < 2; h++) {
      __m512i c[8];
      transpose8(_mm512_loadu_si512(pf[0] + o + 64 * h), _mm512_loadu_si512(pf[1] + o + 64 * h),
                 _mm512_loadu_si512(pf[2] + o + 64 * h), _mm512_loadu_si512(pf[3] + o + 64 * h),
                 _mm512_loadu_si512(pf[4] + o + 64 * h), _mm512_loadu_si512(pf[5] + o + 64 * h),
                 _mm512_loadu_si512(pf[6] + o + 64 * h), _mm512_loadu_si512(pf[7] + o + 64 * h), c);
#pragma GCC unroll 8
      for (int i = 0; i < 8; i++) s[8 * h + i] = _mm512_xor_si512(s[8 * h + i], c[i]);
    }
    s[16] = _mm512_xor_si512(s[16], _mm512_i64gather_epi64(_mm512_add_epi64(addr, _mm512_set1_epi64(128)), nullptr, 1));
    keccakf_x8(s);
    addr = _mm512_add_epi64(addr, step);
  }
  // each message's remaining blocks and its padding on its own sponge
  alignas(64) uint64_t lanes[25][8];
  for (int i = 0; i < 25; i++) _mm512_store_si512(lanes[i], s[i]);
  for (int j = 0; j < n; j++) {
    uint64_t st[25];
    for (int i = 0; i < 25; i++) st[i] = lanes[i][j];
    const uint8_t* p = msg[j] + common * rate;
    size_t rem = len[j] - common * rate;
    auto absorb = [&](const uint8_t* bl) {
      for (size_t i = 0; i < rate / 8; i++) {
        uint64_t w;
        memcpy(&w, bl + 8 * i, 8);
        st[i] ^= w;
      }
      keccakf_portable(st);
    };
    while (rem >= rate) {
      absorb(p);
      p += rate;
      rem -= rate;
    }
    uint8_t last[rate] = {0};
    memcpy(last, p, rem);
    last[rem] ^= 0x06;
    last[rate - 1] ^= 0x80;
    absorb(last);
    memcpy(out[j], st, 32);
  }
}

bool have_avx512f() {
  static const bool v = __builtin_cpu_supports("avx512f") && !getenv("CE_NO_SHA3X8");
  return v;
}

}  // namespace

void sha3_256_multi(const uint8_t* const* msg, const size_t* len, int n, uint8_t out[][32]) {
  for (int b = 0; b < n; b += 8) {
    const int k = n - b < 8 ? n - b : 8;
    if (have_avx512f() && k > 1) {
      sha3_256_x8_avx512(msg + b, len + b, k, out + b);
    } else {
      for (int j = 0; j < k; j++) sha3_256(msg[b + j], len[b + j], out[b + j]);
    }
  }
}

}  // namespace ce

extern "C" int ce_content_names(const uint8_t* const* data, const size_t* lens, uint32_t n, char (*names_out)[64]) {
  if (n && (!data || !lens || !names_out)) return CE_ERR_INVALID_ARG;
  for (uint32_t i = 0; i < n; i++)
    if (!data[i] && lens[i]) return CE_ERR_INVALID_ARG;
  std::string nm;
  for (uint32_t b = 0; b < n; b += 8) {
    const uint32_t k = n - b < 8 ? n - b : 8;
    uint8_t h[8][32];
    ce::sha3_256_multi(data + b, lens + b, (int)k, h);
    for (uint32_t j = 0; j < k; j++) {
      nm = ce::base32_nopad(h[j], 32);
      snprintf(names_out[b + j], 64, "%s", nm.c_str());
    }
  }
  return CE_OK;
}
