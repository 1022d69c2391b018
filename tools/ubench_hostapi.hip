// Host cost of the HIP calls a C3 step issues (no GPU sync between calls): us per call.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdint>
__global__ void k_nop(uint32_t* p) { if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345u) p[1] = 1; }
template <typename F> double per_call(int n, F f, hipStream_t s) {
  hipStreamSynchronize(s);
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; i++) f();
  auto t1 = std::chrono::steady_clock::now();
  hipStreamSynchronize(s);
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}
int main() {
  hipStream_t s; hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  uint32_t *d, *d2; void* h;
  hipMalloc(&d, 64 << 20); hipMalloc(&d2, 64 << 20); hipHostMalloc(&h, 1 << 20, 0);
  hipEvent_t ev; hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  const int n = 2000;
  for (int rep = 0; rep < 2; rep++) {
    printf("launch    %.2f\n", per_call(n, [&] { hipLaunchKernelGGL(k_nop, dim3(64), dim3(256), 0, s, d); }, s));
    printf("memset64  %.2f\n", per_call(n, [&] { hipMemsetAsync(d, 0, 64, s); }, s));
    printf("memset4M  %.2f\n", per_call(n / 4, [&] { hipMemsetAsync(d, 0, 4 << 20, s); }, s));
    printf("memcpyDD  %.2f\n", per_call(n, [&] { hipMemcpyAsync(d2, d, 64, hipMemcpyDeviceToDevice, s); }, s));
    printf("memcpyDH  %.2f\n", per_call(n, [&] { hipMemcpyAsync(h, d, 64, hipMemcpyDeviceToHost, s); }, s));
    printf("memcpyHD  %.2f\n", per_call(n, [&] { hipMemcpyAsync(d, h, 64, hipMemcpyHostToDevice, s); }, s));
    printf("evrecord  %.2f\n", per_call(n, [&] { hipEventRecord(ev, s); }, s));
    printf("evwait    %.2f\n", per_call(n, [&] { hipStreamWaitEvent(s, ev, 0); }, s));
    printf("devprops  %.2f\n", per_call(50, [&] { hipDeviceProp_t p; hipGetDeviceProperties(&p, 0); }, s));
    printf("ptrattr   %.2f\n", per_call(n, [&] { hipPointerAttribute_t a; hipPointerGetAttributes(&a, h); }, s));
    printf("sync_rt   %.2f\n", per_call(500, [&] { hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, s, d); hipStreamSynchronize(s); }, s));
    printf("memcpyDH_sync %.2f\n", per_call(500, [&] { hipMemcpyAsync(h, d, 64, hipMemcpyDeviceToHost, s); hipStreamSynchronize(s); }, s));
  }
  return 0;
}
