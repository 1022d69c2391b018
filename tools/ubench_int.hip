// Microbenchmark: integer VALU rates on gfx950 that decide the Poly1305 limb design, and
// whether unaligned 16-byte global loads are correct + fast.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_int.hip -o tools/ubench_int
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <cstring>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;
constexpr int CH = 8;  // independent chains per lane

__global__ void k_add(uint32_t* out, uint32_t seed) {
  uint32_t a[CH];
  for (int c = 0; c < CH; c++) a[c] = seed + threadIdx.x + c;
  for (int i = 0; i < ITERS; i++)
#pragma unroll
    for (int c = 0; c < CH; c++) a[c] = (a[c] + 0x9e3779b9u) ^ (a[c] >> 3);
  uint32_t s = 0;
  for (int c = 0; c < CH; c++) s ^= a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_rot(uint32_t* out, uint32_t seed) {  // ChaCha-like ARX: add, xor, rotate
  uint32_t a[CH], b[CH];
  for (int c = 0; c < CH; c++) { a[c] = seed + threadIdx.x + c; b[c] = a[c] * 7; }
  for (int i = 0; i < ITERS; i++)
#pragma unroll
    for (int c = 0; c < CH; c++) { a[c] += b[c]; b[c] ^= a[c]; b[c] = __builtin_amdgcn_alignbit(b[c], b[c], 16); }
  uint32_t s = 0;
  for (int c = 0; c < CH; c++) s ^= a[c] ^ b[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mad64(uint32_t* out, uint32_t seed) {  // v_mad_u64_u32
  uint64_t acc[CH];
  uint32_t m[CH];
  for (int c = 0; c < CH; c++) { acc[c] = seed + threadIdx.x + c; m[c] = 0x3ffffff - c; }
  for (int i = 0; i < ITERS; i++)
#pragma unroll
    for (int c = 0; c < CH; c++) acc[c] = (uint64_t)(uint32_t)acc[c] * m[c] + (acc[c] >> 32);
  uint32_t s = 0;
  for (int c = 0; c < CH; c++) s ^= (uint32_t)acc[c] ^ (uint32_t)(acc[c] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mullo(uint32_t* out, uint32_t seed) {  // v_mul_lo_u32
  uint32_t a[CH];
  for (int c = 0; c < CH; c++) a[c] = seed + threadIdx.x + c;
  for (int i = 0; i < ITERS; i++)
#pragma unroll
    for (int c = 0; c < CH; c++) a[c] = a[c] * 0x9e3779b9u + 1;
  uint32_t s = 0;
  for (int c = 0; c < CH; c++) s ^= a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul24(uint32_t* out, uint32_t seed) {  // v_mad_u32_u24 + v_mul_hi_u32_u24
  uint32_t a[CH], h[CH];
  for (int c = 0; c < CH; c++) { a[c] = seed + threadIdx.x + c; h[c] = 0; }
  for (int i = 0; i < ITERS; i++)
#pragma unroll
    for (int c = 0; c < CH; c++) {
      uint32_t x = a[c] & 0xffffff;
      uint32_t hi, lo;
      asm volatile("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(hi) : "v"(x), "v"(0x9e3779u));
      asm volatile("v_mul_u32_u24 %0, %1, %2" : "=v"(lo) : "v"(x), "v"(0x9e3779u));
      h[c] += hi;
      a[c] = lo + h[c];
    }
  uint32_t s = 0;
  for (int c = 0; c < CH; c++) s ^= a[c] ^ h[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma64(double* out, double seed) {  // v_fma_f64
  double a[CH];
  for (int c = 0; c < CH; c++) a[c] = seed + threadIdx.x + c;
  for (int i = 0; i < ITERS; i++)
#pragma unroll
    for (int c = 0; c < CH; c++) a[c] = __builtin_fma(a[c], 0.999999, 1e-9);
  double s = 0;
  for (int c = 0; c < CH; c++) s += a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_load16(const uint8_t* __restrict__ in, size_t n16, uint32_t* out, int misalign) {
  const uint8_t* base = in + misalign;
  uint32_t s = 0;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    uint4 v = *reinterpret_cast<const uint4*>(base + 16 * i);
    s ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K, typename T>
float run(K kern, T* out, T seed, int grid, int block) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(block), 0, 0, out, seed);
  (void)hipEventRecord(a);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(kern, dim3(grid), dim3(block), 0, 0, out, seed);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  int grid = 256 * 8, block = 256;
  uint32_t* o32; double* of;
  CHECK(hipMalloc(&o32, (size_t)grid * block * 4));
  CHECK(hipMalloc(&of, (size_t)grid * block * 8));
  double lanes = (double)grid * block;
  struct { const char* n; float ms; double ops_per_iter; } r[6];
  r[0] = {"add+xor+shr (3 ops)", run(k_add, o32, 1u, grid, block), 3};
  r[1] = {"add+xor+alignbit (3 ops)", run(k_rot, o32, 1u, grid, block), 3};
  r[2] = {"mad_u64_u32 (+shift)", run(k_mad64, o32, 1u, grid, block), 1};
  r[3] = {"mul_lo_u32 (+add)", run(k_mullo, o32, 1u, grid, block), 1};
  r[4] = {"mul_u24+mulhi_u24+2add", run(k_mul24, o32, 1u, grid, block), 2};
  r[5] = {"fma_f64", run(k_fma64, of, 1.0, grid, block), 1};
  for (auto& x : r) {
    double n = lanes * ITERS * CH * x.ops_per_iter;
    printf("%-28s %8.3f ms  %8.2f Tlane-ops/s (per listed op)\n", x.n, x.ms, n / (x.ms * 1e-3) / 1e12);
  }
  // unaligned 16-B loads
  size_t bytes = (size_t)1 << 30;
  uint8_t* buf;
  CHECK(hipMalloc(&buf, bytes + 64));
  CHECK(hipMemset(buf, 0x5a, bytes + 64));
  size_t n16 = bytes / 16;
  for (int mis : {0, 3, 8, 13}) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k_load16, dim3(grid), dim3(block), 0, 0, buf, n16, o32, mis);
    (void)hipEventRecord(a);
    for (int rr = 0; rr < 5; rr++) hipLaunchKernelGGL(k_load16, dim3(grid), dim3(block), 0, 0, buf, n16, o32, mis);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b); ms /= 5;
    printf("load16 misalign=%2d : %.3f ms  %.1f GB/s\n", mis, ms, bytes / (ms * 1e-3) / 1e9);
  }
  // correctness of an unaligned load
  std::vector<uint8_t> h(64);
  for (int i = 0; i < 64; i++) h[i] = (uint8_t)i;
  CHECK(hipMemcpy(buf, h.data(), 64, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_load16, dim3(1), dim3(1), 0, 0, buf, (size_t)1, o32, 3);
  uint32_t got;
  CHECK(hipMemcpy(&got, o32, 4, hipMemcpyDeviceToHost));
  uint32_t w[4];
  std::memcpy(w, h.data() + 3, 16);
  printf("unaligned load correct: %s (got %08x want %08x)\n", got == (w[0] ^ w[1] ^ w[2] ^ w[3]) ? "yes" : "NO", got, w[0] ^ w[1] ^ w[2] ^ w[3]);
  return 0;
}
