// ubench_lds_unaligned: are unaligned ds_read_b32 / b64 / b128 correct on gfx950 (MI355X), and
// what do they cost against aligned reads + v_alignbyte windowing?
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_lds_unaligned.hip -o tools/ubench_lds_unaligned
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef uint32_t u32a1 __attribute__((aligned(1)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef v2u u2a1 __attribute__((aligned(1)));
typedef v4u u4a1 __attribute__((aligned(1)));

__global__ void k_check(uint32_t* out) {
  __shared__ uint8_t lds[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) lds[i] = (uint8_t)(i * 7 + 3);
  __syncthreads();
  const uint32_t off = threadIdx.x * 37 + 1;  // every alignment
  const uint32_t a = *reinterpret_cast<const u32a1*>(lds + off);
  const v2u b = *reinterpret_cast<const u2a1*>(lds + off + 5);
  const v4u c = *reinterpret_cast<const u4a1*>(lds + off + 11);
  out[threadIdx.x * 7 + 0] = a;
  out[threadIdx.x * 7 + 1] = b.x; out[threadIdx.x * 7 + 2] = b.y;
  out[threadIdx.x * 7 + 3] = c.x; out[threadIdx.x * 7 + 4] = c.y;
  out[threadIdx.x * 7 + 5] = c.z; out[threadIdx.x * 7 + 6] = c.w;
}

constexpr int IT = 4096;
// 48-byte windows at a per-lane byte offset: 3 unaligned b128 reads vs 13 aligned b32 + 12 alignbyte
__global__ void k_unal(uint32_t* out, uint32_t stride) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[16384];
  for (int i = threadIdx.x; i < 16384; i += blockDim.x) lds[i] = (uint8_t)i;
  __syncthreads();
  uint32_t acc = 0, o = (threadIdx.x & 63) * stride;
  for (int it = 0; it < IT; it++) {
    const uint8_t* p = lds + ((o + it * 38) & 8191);
    v4u w0 = *reinterpret_cast<const u4a1*>(p);
    v4u w1 = *reinterpret_cast<const u4a1*>(p + 16);
    v4u w2 = *reinterpret_cast<const u4a1*>(p + 32);
    acc += w0.x ^ w0.y ^ w0.z ^ w0.w ^ w1.x ^ w1.y ^ w1.z ^ w1.w ^ w2.x ^ w2.y ^ w2.z ^ w2.w;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
__global__ void k_align(uint32_t* out, uint32_t stride) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[16384];
  for (int i = threadIdx.x; i < 16384; i += blockDim.x) lds[i] = (uint8_t)i;
  __syncthreads();
  uint32_t acc = 0, o = (threadIdx.x & 63) * stride;
  for (int it = 0; it < IT; it++) {
    const uint32_t c = (o + it * 38) & 8191;
    const uint32_t* d = reinterpret_cast<const uint32_t*>(lds) + (c >> 2);
    uint32_t dd[13], w = 0;
#pragma unroll
    for (int q = 0; q < 13; q++) dd[q] = d[q];
#pragma unroll
    for (int q = 0; q < 12; q++) w ^= __builtin_amdgcn_alignbyte(dd[q + 1], dd[q], c & 3);
    acc += w;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  uint32_t* o;
  CHECK(hipMalloc(&o, 1 << 24));
  hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, o);
  std::vector<uint32_t> h(64 * 7);
  CHECK(hipMemcpy(h.data(), o, h.size() * 4, hipMemcpyDeviceToHost));
  std::vector<uint8_t> ref(4096);
  for (int i = 0; i < 4096; i++) ref[i] = (uint8_t)(i * 7 + 3);
  int bad = 0;
  for (int t = 0; t < 64; t++) {
    const uint32_t off = t * 37 + 1;
    auto rd = [&](uint32_t p) { return ref[p] | ref[p + 1] << 8 | ref[p + 2] << 16 | (uint32_t)ref[p + 3] << 24; };
    uint32_t want[7] = {rd(off), rd(off + 5), rd(off + 9), rd(off + 11), rd(off + 15), rd(off + 19), rd(off + 23)};
    for (int k = 0; k < 7; k++) bad += h[t * 7 + k] != want[k];
  }
  printf("unaligned ds_read b32/b64/b128 correct: %s (%d mismatches)\n", bad ? "NO" : "yes", bad);
  for (int rep = 0; rep < 2; rep++)
    for (int which = 0; which < 2; which++) {
      hipEvent_t a, b;
      (void)hipEventCreate(&a); (void)hipEventCreate(&b);
      auto k = which ? k_align : k_unal;
      hipLaunchKernelGGL(k, dim3(256 * 8), dim3(128), 0, 0, o, 38u);
      (void)hipEventRecord(a);
      for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k, dim3(256 * 8), dim3(128), 0, 0, o, 38u);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b);
      printf("%s: %.3f ms per launch (2048 blocks x 128 lanes x %d windows of 48 B)\n",
             which ? "13 aligned b32 + 12 alignbyte" : "3 unaligned b128", ms / 5, IT);
    }
  return 0;
}
