// How a device->host copy slows kernels running beside it: a 512 MB HBM fill timed alone, then
// beside a 35 MB copy into pinned host memory (copy kernel with B blocks, or hipMemcpyAsync),
// for pinned memory from hipHostMalloc and from a THP-backed mmap + hipHostRegister.
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#define CK(x) do { hipError_t e_ = (x); if (e_) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
__global__ void k_fill4(uint4* p, uint64_t n, uint32_t v) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = make_uint4(v, v, v, v);
}
__global__ void k_copy(uint4* dst, const uint4* src, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}
int main() {
  const uint64_t FB = 512ull << 20, CB = 35ull << 20;
  uint4 *dfill, *dsrc;
  CK(hipMalloc(&dfill, FB)); CK(hipMalloc(&dsrc, CB));
  CK(hipMemset(dsrc, 7, CB));
  void* hm; CK(hipHostMalloc(&hm, CB, 0));
  void* thp = mmap(nullptr, CB + (2 << 20), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  uint8_t* thpa = (uint8_t*)(((uintptr_t)thp + (2 << 20) - 1) & ~(uintptr_t)((2 << 20) - 1));
  int adv = madvise(thpa, CB, MADV_HUGEPAGE);
  memset(thpa, 1, CB);
  CK(hipHostRegister(thpa, CB, hipHostRegisterMapped));
  void* thpd; CK(hipHostGetDevicePointer(&thpd, thpa, 0));
  void* hmd; CK(hipHostGetDevicePointer(&hmd, hm, 0));
  printf("madvise %d\n", adv);
  hipStream_t s1, s2; CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t a, b, c, d; hipEventCreate(&a); hipEventCreate(&b); hipEventCreate(&c); hipEventCreate(&d);
  auto fill = [&] { hipLaunchKernelGGL(k_fill4, dim3(4096), dim3(256), 0, s1, dfill, FB / 16, 0u); };
  for (int rep = 0; rep < 2; rep++) {
    float t;
    hipEventRecord(a, s1); fill(); hipEventRecord(b, s1); CK(hipEventSynchronize(b));
    hipEventElapsedTime(&t, a, b); printf("fill alone          %8.1f us\n", t * 1e3);
    const char* names[2] = {"hipHostMalloc", "THP+register"};
    void* dsts[2] = {hmd, thpd}; void* hdst[2] = {hm, thpa};
    for (int m = 0; m < 2; m++) {
      for (int blocks : {8, 32, 128}) {
        float tc, tf;
        hipEventRecord(c, s2);
        hipLaunchKernelGGL(k_copy, dim3(blocks), dim3(256), 0, s2, (uint4*)dsts[m], dsrc, CB / 16);
        hipEventRecord(d, s2);
        hipEventRecord(a, s1); fill(); hipEventRecord(b, s1);
        CK(hipEventSynchronize(b)); CK(hipEventSynchronize(d));
        hipEventElapsedTime(&tf, a, b); hipEventElapsedTime(&tc, c, d);
        printf("%-14s copy kernel %3d blocks: copy %8.1f us (%5.1f GB/s), fill beside it %8.1f us\n", names[m], blocks, tc * 1e3, CB / (tc * 1e6), tf * 1e3);
        hipEventRecord(c, s2);
        hipLaunchKernelGGL(k_copy, dim3(blocks), dim3(256), 0, s2, (uint4*)dsts[m], dsrc, CB / 16);
        hipEventRecord(d, s2); CK(hipEventSynchronize(d));
        hipEventElapsedTime(&tc, c, d);
        printf("%-14s copy kernel %3d blocks alone: %8.1f us\n", names[m], blocks, tc * 1e3);
      }
      float tc, tf;
      hipEventRecord(c, s2);
      CK(hipMemcpyAsync(hdst[m], dsrc, CB, hipMemcpyDeviceToHost, s2));
      hipEventRecord(d, s2);
      hipEventRecord(a, s1); fill(); hipEventRecord(b, s1);
      CK(hipEventSynchronize(b)); CK(hipEventSynchronize(d));
      hipEventElapsedTime(&tf, a, b); hipEventElapsedTime(&tc, c, d);
      printf("%-14s hipMemcpyAsync: copy %8.1f us, fill beside it %8.1f us\n", names[m], tc * 1e3, tf * 1e3);
    }
  }
  return 0;
}
