// Microbenchmark: ChaCha20 block throughput on gfx950 with different rotate lowerings, and the
// issue cost of the integer instructions the open kernel is made of (full occupancy).
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_chacha.hip -o tools/ubench_chacha
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int IMPL>
__device__ __forceinline__ uint32_t rot(uint32_t x, int c) {
  if (IMPL == 0) return __builtin_amdgcn_alignbit(x, x, 32 - c);             // v_alignbit_b32
  if (IMPL == 1) {                                                           // v_perm for 16/8
    if (c == 16) return __builtin_amdgcn_perm(x, x, 0x01000302u);
    if (c == 8) return __builtin_amdgcn_perm(x, x, 0x02010003u);
    return __builtin_amdgcn_alignbit(x, x, 32 - c);
  }
  if (IMPL == 2) return (x << c) | (x >> (32 - c));                           // shl, shr, or
  if (IMPL == 4) return __builtin_amdgcn_alignbit(x, x, 32 - c);
  if (IMPL >= 5) {  // full-rate VOP2 only: shl, shr, or (asm so the compiler cannot fold it back)
    if (IMPL == 7 && c == 8) return __builtin_amdgcn_perm(x, x, 0x02010003u);
    uint32_t h, l, r;
    asm("v_lshlrev_b32 %0, %1, %2" : "=v"(h) : "i"(c), "v"(x));
    asm("v_lshrrev_b32 %0, %1, %2" : "=v"(l) : "i"(32 - c), "v"(x));
    asm("v_or_b32 %0, %1, %2" : "=v"(r) : "v"(h), "v"(l));
    return r;
  }
  // IMPL 3: v_lshl_or_b32(x, c, x >> (32 - c))
  uint32_t r;
  asm volatile("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "i"(c), "v"(x >> (32 - c)));
  return r;
}

// rot16(d ^ a): IMPL 4 writes the two halves with two SDWA xors (full-rate VOP2) instead of
// a xor plus a (half-rate) v_alignbit_b32
template <int IMPL>
__device__ __forceinline__ uint32_t xr16(uint32_t d, uint32_t a) {
  if (IMPL != 4 && IMPL != 6 && IMPL != 7) return rot<IMPL>(d ^ a, 16);
  uint32_t r;
  asm(
      "v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n"
      "v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0"
      : "=&v"(r) : "v"(d), "v"(a));
  return r;
}

#define QR(a, b, c, d)                                                          \
  a += b; d = xr16<IMPL>(d, a); c += d; b ^= c; b = rot<IMPL>(b, 12);     \
  a += b; d ^= a; d = rot<IMPL>(d, 8);  c += d; b ^= c; b = rot<IMPL>(b, 7);

template <int IMPL, int NB>
__global__ void k_chacha(uint32_t* out, uint32_t seed, int iters) {
  uint32_t acc = 0;
  for (int it = 0; it < iters; it++) {
    uint32_t x[NB][16];
#pragma unroll
    for (int b = 0; b < NB; b++)
#pragma unroll
      for (int i = 0; i < 16; i++) x[b][i] = seed * (i + 1) + threadIdx.x + b + it;
#pragma unroll
    for (int r = 0; r < 10; r++)
#pragma unroll
      for (int b = 0; b < NB; b++) {
        QR(x[b][0], x[b][4], x[b][8], x[b][12]); QR(x[b][1], x[b][5], x[b][9], x[b][13]);
        QR(x[b][2], x[b][6], x[b][10], x[b][14]); QR(x[b][3], x[b][7], x[b][11], x[b][15]);
        QR(x[b][0], x[b][5], x[b][10], x[b][15]); QR(x[b][1], x[b][6], x[b][11], x[b][12]);
        QR(x[b][2], x[b][7], x[b][8], x[b][13]); QR(x[b][3], x[b][4], x[b][9], x[b][14]);
      }
#pragma unroll
    for (int b = 0; b < NB; b++)
#pragma unroll
      for (int i = 0; i < 16; i++) acc ^= x[b][i];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <typename K>
float run(K kern, uint32_t* out, int grid, int block, int iters) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(block), 0, 0, out, 1u, iters);
  (void)hipEventRecord(a);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(kern, dim3(grid), dim3(block), 0, 0, out, 1u, iters);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  const int block = 256, iters = 64;
  uint32_t* o;
  CHECK(hipMalloc(&o, (size_t)256 * 16 * block * 4));
  const char* names[8] = {"alignbit", "perm16/8+alignbit", "shl|shr", "lshl_or+shr", "sdwa-xor rot16", "shl/shr/or asm", "sdwa16+shl/shr/or", "sdwa16+perm8+shl/shr/or"};
  for (int occ : {2, 8}) {  // waves per SIMD
    const int grid = 256 * occ;  // 4 waves per block -> occ waves per SIMD
    const double blocks = (double)grid * block * iters;
    float t[8][2];
    t[0][0] = run(k_chacha<0, 1>, o, grid, block, iters); t[0][1] = run(k_chacha<0, 2>, o, grid, block, iters);
    t[1][0] = run(k_chacha<1, 1>, o, grid, block, iters); t[1][1] = run(k_chacha<1, 2>, o, grid, block, iters);
    t[2][0] = run(k_chacha<2, 1>, o, grid, block, iters); t[2][1] = run(k_chacha<2, 2>, o, grid, block, iters);
    t[3][0] = run(k_chacha<3, 1>, o, grid, block, iters); t[3][1] = run(k_chacha<3, 2>, o, grid, block, iters);
    t[4][0] = run(k_chacha<4, 1>, o, grid, block, iters); t[4][1] = run(k_chacha<4, 2>, o, grid, block, iters);
    t[5][0] = run(k_chacha<5, 1>, o, grid, block, iters); t[5][1] = run(k_chacha<5, 2>, o, grid, block, iters);
    t[6][0] = run(k_chacha<6, 1>, o, grid, block, iters); t[6][1] = run(k_chacha<6, 2>, o, grid, block, iters);
    t[7][0] = run(k_chacha<7, 1>, o, grid, block, iters); t[7][1] = run(k_chacha<7, 2>, o, grid, block, iters);
    for (int i = 0; i < 8; i++)
      printf("%d waves/SIMD %-20s 1 blk/lane %7.1f GB/s keystream   2 blk/lane %7.1f GB/s\n", occ, names[i],
             blocks * 64 / (t[i][0] * 1e-3) / 1e9, blocks * 2 * 64 / (t[i][1] * 1e-3) / 1e9);
  }
  return 0;
}
