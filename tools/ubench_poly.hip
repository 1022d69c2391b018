// Microbenchmark: Poly1305 mulmod formulations on gfx950 (radix 2^26, 5 limbs), throughput at
// full occupancy, NCHAIN independent Horner chains per lane.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_poly.hip -o tools/ubench_poly
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "../crdt-enc_amd/csrc/ce_device.h"

using namespace ce;

// variant 1: carries folded into the next limb's first v_mad_u64_u32 (32-bit carry words)
__device__ __forceinline__ L5 mulmod_fold(const L5& h, const L5& r) {
  const uint32_t s1 = r.v[1] * 5, s2 = r.v[2] * 5, s3 = r.v[3] * 5, s4 = r.v[4] * 5;
  L5 o;
  uint64_t d = (uint64_t)h.v[0] * r.v[0] + (uint64_t)h.v[1] * s4 + (uint64_t)h.v[2] * s3 +
               (uint64_t)h.v[3] * s2 + (uint64_t)h.v[4] * s1;
  o.v[0] = (uint32_t)d & M26;
  uint32_t c = __builtin_amdgcn_alignbit((uint32_t)(d >> 32), (uint32_t)d, 26);
  d = (uint64_t)c + (uint64_t)h.v[0] * r.v[1] + (uint64_t)h.v[1] * r.v[0] + (uint64_t)h.v[2] * s4 +
      (uint64_t)h.v[3] * s3 + (uint64_t)h.v[4] * s2;
  o.v[1] = (uint32_t)d & M26;
  c = __builtin_amdgcn_alignbit((uint32_t)(d >> 32), (uint32_t)d, 26);
  d = (uint64_t)c + (uint64_t)h.v[0] * r.v[2] + (uint64_t)h.v[1] * r.v[1] + (uint64_t)h.v[2] * r.v[0] +
      (uint64_t)h.v[3] * s4 + (uint64_t)h.v[4] * s3;
  o.v[2] = (uint32_t)d & M26;
  c = __builtin_amdgcn_alignbit((uint32_t)(d >> 32), (uint32_t)d, 26);
  d = (uint64_t)c + (uint64_t)h.v[0] * r.v[3] + (uint64_t)h.v[1] * r.v[2] + (uint64_t)h.v[2] * r.v[1] +
      (uint64_t)h.v[3] * r.v[0] + (uint64_t)h.v[4] * s4;
  o.v[3] = (uint32_t)d & M26;
  c = __builtin_amdgcn_alignbit((uint32_t)(d >> 32), (uint32_t)d, 26);
  d = (uint64_t)c + (uint64_t)h.v[0] * r.v[4] + (uint64_t)h.v[1] * r.v[3] + (uint64_t)h.v[2] * r.v[2] +
      (uint64_t)h.v[3] * r.v[1] + (uint64_t)h.v[4] * r.v[0];
  o.v[4] = (uint32_t)d & M26;
  c = __builtin_amdgcn_alignbit((uint32_t)(d >> 32), (uint32_t)d, 26);
  const uint64_t t = (uint64_t)c * 5 + o.v[0];
  o.v[0] = (uint32_t)t & M26;
  o.v[1] += __builtin_amdgcn_alignbit((uint32_t)(t >> 32), (uint32_t)t, 26);
  return o;
}

// variant 2: five independent 64-bit sums, then 32-bit carry words added with add_co/addc
__device__ __forceinline__ L5 mulmod_par(const L5& h, const L5& r) {
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
  auto cw = [](uint64_t d) { return __builtin_amdgcn_alignbit((uint32_t)(d >> 32), (uint32_t)d, 26); };
  L5 o;
  d1 += cw(d0); o.v[0] = (uint32_t)d0 & M26;
  d2 += cw(d1); o.v[1] = (uint32_t)d1 & M26;
  d3 += cw(d2); o.v[2] = (uint32_t)d2 & M26;
  d4 += cw(d3); o.v[3] = (uint32_t)d3 & M26;
  o.v[4] = (uint32_t)d4 & M26;
  const uint64_t t = (uint64_t)cw(d4) * 5 + o.v[0];
  o.v[0] = (uint32_t)t & M26;
  o.v[1] += cw(t);
  return o;
}

template <int V, int NCHAIN>
__global__ void k_horner(uint32_t* out, uint32_t seed, int iters) {
  L5 acc[NCHAIN], R;
  for (int i = 0; i < 5; i++) R.v[i] = (seed * 0x9e3779b1u + i) & M26;
#pragma unroll
  for (int c = 0; c < NCHAIN; c++)
    for (int i = 0; i < 5; i++) acc[c].v[i] = (threadIdx.x + c + i) & M26;
  for (int it = 0; it < iters; it++) {
    const L5 m = block_limbs(it, it * 3, it * 7, threadIdx.x);
#pragma unroll
    for (int c = 0; c < NCHAIN; c++) {
      L5 p = V == 0 ? mulmod(acc[c], R) : V == 1 ? mulmod_fold(acc[c], R) : mulmod_par(acc[c], R);
      acc[c] = add5(p, m);
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < NCHAIN; c++)
    for (int i = 0; i < 5; i++) s ^= acc[c].v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
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

// equality of the variants on random inputs (host-checked)
__global__ void k_check(uint32_t* bad, uint32_t seed) {
  uint32_t x = seed ^ (blockIdx.x * 256 + threadIdx.x) * 0x9e3779b1u;
  auto rnd = [&]() { x ^= x << 13; x ^= x >> 17; x ^= x << 5; return x; };
  for (int k = 0; k < 64; k++) {
    L5 h, r;
    for (int i = 0; i < 5; i++) { h.v[i] = rnd() & 0x7ffffff; r.v[i] = rnd() & M26; }
    r.v[1] &= 0x3fffffc; r.v[2] &= 0x3fffffc; r.v[3] &= 0x3fffffc; r.v[4] &= 0xfffff;
    const L5 a = carry5(mulmod(h, r)), b = carry5(mulmod_fold(h, r)), c = carry5(mulmod_par(h, r));
    for (int i = 0; i < 5; i++)
      if (a.v[i] != b.v[i] || a.v[i] != c.v[i]) atomicAdd(bad, 1u);
  }
}

int main() {
  const int block = 256, iters = 256;
  uint32_t* o;
  if (hipMalloc(&o, (size_t)256 * 8 * block * 4) != hipSuccess) return 1;
  uint32_t* bad;
  (void)hipMalloc(&bad, 4);
  (void)hipMemset(bad, 0, 4);
  hipLaunchKernelGGL(k_check, dim3(1024), dim3(256), 0, 0, bad, 12345u);
  uint32_t hb = 0;
  (void)hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
  printf("variants agree on 16M random products: %s (%u mismatches)\n", hb ? "NO" : "yes", hb);
  const char* names[3] = {"mulmod (current)", "carry folded into mad", "parallel sums + 32-bit carries"};
  for (int occ : {2, 8}) {
    const int grid = 256 * occ;
    const double steps = (double)grid * block * iters;
    float t[3][2];
    t[0][0] = run(k_horner<0, 1>, o, grid, block, iters); t[0][1] = run(k_horner<0, 2>, o, grid, block, iters);
    t[1][0] = run(k_horner<1, 1>, o, grid, block, iters); t[1][1] = run(k_horner<1, 2>, o, grid, block, iters);
    t[2][0] = run(k_horner<2, 1>, o, grid, block, iters); t[2][1] = run(k_horner<2, 2>, o, grid, block, iters);
    for (int i = 0; i < 3; i++)
      printf("%d waves/SIMD %-32s 1 chain %7.1f G steps/s   2 chains %7.1f G steps/s\n", occ, names[i],
             steps / (t[i][0] * 1e-3) / 1e9, 2 * steps / (t[i][1] * 1e-3) / 1e9);
  }
  return 0;
}
