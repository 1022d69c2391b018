// Sustained ChaCha20 keystream rate and the shader clock it runs at: the tools/ubench_chacha.hip
// kernel (SDWA rot16, one block per lane) launched back to back for ~150 ms at 2 and 8 waves per
// SIMD, with 8 one-wave probes on a second stream reading the shader cycle counter against the
// 100 MHz reference clock every 100 us (as ce_ctx_clock_probe).  Prints the keystream rate of
// the first and of the last launches and the clock over the first 10 ms and the last 50 ms.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_chacha_clock.hip -o tools/ubench_chacha_clock
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t rot(uint32_t x, int c) { return __builtin_amdgcn_alignbit(x, x, 32 - c); }
__device__ __forceinline__ uint32_t xr16(uint32_t d, uint32_t a) {
  uint32_t r;
  asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n"
      "v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0"
      : "=&v"(r) : "v"(d), "v"(a));
  return r;
}
#define QR(a, b, c, d)                                                  \
  a += b; d = xr16(d, a); c += d; b ^= c; b = rot(b, 12);               \
  a += b; d ^= a; d = rot(d, 8);  c += d; b ^= c; b = rot(b, 7);

__global__ void k_chacha(uint32_t* out, uint32_t seed, int iters) {
  uint32_t acc = 0;
  for (int it = 0; it < iters; it++) {
    uint32_t x[16];
#pragma unroll
    for (int i = 0; i < 16; i++) x[i] = seed * (i + 1) + threadIdx.x + it;
#pragma unroll
    for (int r = 0; r < 10; r++) {
      QR(x[0], x[4], x[8], x[12]); QR(x[1], x[5], x[9], x[13]);
      QR(x[2], x[6], x[10], x[14]); QR(x[3], x[7], x[11], x[15]);
      QR(x[0], x[5], x[10], x[15]); QR(x[1], x[6], x[11], x[12]);
      QR(x[2], x[7], x[8], x[13]); QR(x[3], x[4], x[9], x[14]);
    }
#pragma unroll
    for (int i = 0; i < 16; i++) acc ^= x[i];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void k_probe(unsigned long long* out, uint32_t samples, uint32_t ticks) {
  const uint32_t lane = threadIdx.x;
  unsigned long long c0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t k = 0; k < samples; k++) {
    unsigned long long r = r0;
    while (r - r0 < ticks) {
      __builtin_amdgcn_s_sleep(2);
      r = __builtin_amdgcn_s_memrealtime();
    }
    const unsigned long long c = __builtin_amdgcn_s_memtime();
    if (lane < 2) out[2ull * ((unsigned long long)blockIdx.x * samples + k) + lane] = lane ? r - r0 : c - c0;
    c0 = c;
    r0 = r;
  }
}

int main() {
  const int block = 256, probes = 8;
  const uint32_t samples = 1500, ticks = 10000;  // 150 ms
  uint32_t* o;
  unsigned long long* po;
  CHECK(hipMalloc(&o, (size_t)256 * 8 * block * 4));
  CHECK(hipMalloc(&po, (size_t)probes * samples * 16));
  hipStream_t s1, s2;
  CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  for (int occ : {2, 8}) {
    const int grid = 256 * occ;
    const int iters = occ == 2 ? 512 : 128;  // ~3.5 ms per launch at either occupancy
    const int nl = 80;
    std::vector<hipEvent_t> ev(nl + 1);
    for (int l = 0; l <= nl; l++) CHECK(hipEventCreate(&ev[l]));
    hipLaunchKernelGGL(k_chacha, dim3(grid), dim3(block), 0, s1, o, 1u, 4);  // load the code
    CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_probe, dim3(probes), dim3(64), 0, s2, po, samples, ticks);
    CHECK(hipEventRecord(ev[0], s1));
    for (int l = 0; l < nl; l++) {
      hipLaunchKernelGGL(k_chacha, dim3(grid), dim3(block), 0, s1, o, 1u, iters);
      CHECK(hipEventRecord(ev[l + 1], s1));
    }
    CHECK(hipDeviceSynchronize());
    std::vector<unsigned long long> h((size_t)probes * samples * 2);
    CHECK(hipMemcpy(h.data(), po, h.size() * 8, hipMemcpyDeviceToHost));
    auto ghz = [&](uint32_t k0, uint32_t k1) {
      std::vector<double> v;
      for (int b = 0; b < probes; b++)
        for (uint32_t k = k0; k < k1; k++) {
          const unsigned long long* p = &h[2ull * ((size_t)b * samples + k)];
          v.push_back((double)p[0] / (double)std::max(p[1], 1ull) * 0.1);
        }
      std::sort(v.begin(), v.end());
      return v[v.size() / 2];
    };
    auto rate = [&](int l0, int l1) {
      float ms;
      (void)hipEventElapsedTime(&ms, ev[l0], ev[l1]);
      const double bytes = (double)grid * block * iters * 64 * (l1 - l0);
      return bytes / (ms * 1e-3) / 1e9;
    };
    float total;
    (void)hipEventElapsedTime(&total, ev[0], ev[nl]);
    printf("%d waves/SIMD: %d launches in %.1f ms; keystream first 3 launches %.1f GB/s, last 10 "
           "%.1f GB/s; clock first 10 ms %.3f GHz, 50-100 ms %.3f GHz\n",
           occ, nl, total, rate(0, 3), rate(nl - 10, nl), ghz(0, 100), ghz(500, 1000));
    for (auto& e : ev) (void)hipEventDestroy(e);
  }
  return 0;
}
