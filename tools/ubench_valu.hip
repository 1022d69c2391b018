// ubench_valu: issue cost of the VALU instructions the fused open kernel is made of, per wave64
// instruction per SIMD, at 1/2/4/8 waves per SIMD, with the in-kernel clock measured (s_memtime
// over s_memrealtime) so a DVFS clock drop is not mistaken for a slower issue rate.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_valu.hip -o tools/ubench_valu && tools/ubench_valu
// Each kernel runs 8 independent register chains of one instruction (inline asm, so the exact
// opcode is what issues), ITERS x 8 instructions per wave.  A workgroup is 4 waves (one per
// SIMD); the grid is 256 CUs x W workgroups, so every SIMD holds W waves.
//   cycles/instr/SIMD = (in-kernel cycles of the launch) / (W x instructions per wave)
// Evidence for the bench's roofline: profiles/r02_ubench_valu.txt.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

constexpr int ITERS = 32768;

#define R8(OP) OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)

// clock stamps of lane 0: [cycles, realtime ticks (100 MHz)]
__device__ __forceinline__ void stamp_out(unsigned long long* st, unsigned long long t0c,
                                          unsigned long long t0r) {
  const unsigned long long t1c = __builtin_amdgcn_s_memtime();
  const unsigned long long t1r = __builtin_amdgcn_s_memrealtime();
  const uint32_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0) {
    st[2 * w] = t1c - t0c;
    st[2 * w + 1] = t1r - t0r;
  }
}

#define U32_KERNEL(NAME, ASM)                                                          \
  __global__ void NAME(uint32_t* out, unsigned long long* st, uint32_t seed) {        \
    uint32_t r0 = seed + threadIdx.x, r1 = r0 * 3, r2 = r0 * 5, r3 = r0 * 7, r4 = r0 * 9, \
             r5 = r0 * 11, r6 = r0 * 13, r7 = r0 * 15;                                 \
    const uint32_t k = seed * 0x9e3779b9u, k2 = seed ^ 0x5bd1e995u;                  \
    const unsigned long long t0c = __builtin_amdgcn_s_memtime();                     \
    const unsigned long long t0r = __builtin_amdgcn_s_memrealtime();                 \
    for (int i = 0; i < ITERS; i++) {                                                  \
      asm volatile(ASM : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5),     \
                   "+v"(r6), "+v"(r7) : "v"(k), "v"(k2));                              \
    }                                                                                  \
    stamp_out(st, t0c, t0r);                                                           \
    out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7; \
  }

#define S_ADD(i) "v_add_u32 %" #i ", %" #i ", %8\n"
#define S_XOR(i) "v_xor_b32 %" #i ", %" #i ", %8\n"
#define S_ALIGN(i) "v_alignbit_b32 %" #i ", %" #i ", %" #i ", 20\n"
#define S_ADD3(i) "v_add3_u32 %" #i ", %" #i ", %8, %9\n"
#define S_XAD(i) "v_xad_u32 %" #i ", %" #i ", %8, %9\n"
#define S_PERM(i) "v_perm_b32 %" #i ", %" #i ", %8, %9\n"
#define S_AND(i) "v_and_b32 %" #i ", %" #i ", %8\n"
#define S_FMA(i) "v_fma_f32 %" #i ", %" #i ", %8, %9\n"
#define S_MULLO(i) "v_mul_lo_u32 %" #i ", %" #i ", %8\n"
// one ChaCha20 quarter-round step mix: add, xor, rotate on chains (i, i^1)
#define S_ARX(i) "v_add_u32 %" #i ", %" #i ", %8\n v_xor_b32 %" #i ", %" #i ", %9\n v_alignbit_b32 %" #i ", %" #i ", %" #i ", 16\n"

// issue-rule probes: the same three ARX instructions grouped by kind (consecutive instructions
// independent), add/xor only (dependent), the rot16 fused into the xor by two SDWA word moves,
// v_bitop3_b32, and 2 full-rate : 1 half-rate on independent chains
#define S_ARXG "v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n" \
  "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n"            \
  "v_xor_b32 %0, %0, %9\n v_xor_b32 %1, %1, %9\n v_xor_b32 %2, %2, %9\n v_xor_b32 %3, %3, %9\n"            \
  "v_xor_b32 %4, %4, %9\n v_xor_b32 %5, %5, %9\n v_xor_b32 %6, %6, %9\n v_xor_b32 %7, %7, %9\n"            \
  R8(S_ALIGN)
#define S_AX(i) "v_add_u32 %" #i ", %" #i ", %8\n v_xor_b32 %" #i ", %" #i ", %9\n"
#define S_XR16(i) "v_xor_b32_sdwa %" #i ", %" #i ", %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n" \
  "v_xor_b32_sdwa %" #i ", %" #i ", %9 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n"
#define S_BOP3(i) "v_bitop3_b32 %" #i ", %" #i ", %8, %9 bitop3:0x96\n"
#define S_221 "v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_alignbit_b32 %2, %2, %2, 20\n" \
  "v_xor_b32 %3, %3, %9\n v_xor_b32 %4, %4, %9\n v_alignbit_b32 %5, %5, %5, 20\n" \
  "v_add_u32 %6, %6, %8\n v_xor_b32 %7, %7, %9\n"

U32_KERNEL(k_arxg, S_ARXG)
U32_KERNEL(k_ax, R8(S_AX))
U32_KERNEL(k_xr16, R8(S_XR16))
U32_KERNEL(k_bop3, R8(S_BOP3))
U32_KERNEL(k_221, S_221)
U32_KERNEL(k_add, R8(S_ADD))
U32_KERNEL(k_xor, R8(S_XOR))
U32_KERNEL(k_align, R8(S_ALIGN))
U32_KERNEL(k_add3, R8(S_ADD3))
U32_KERNEL(k_xad, R8(S_XAD))
U32_KERNEL(k_perm, R8(S_PERM))
U32_KERNEL(k_and, R8(S_AND))
U32_KERNEL(k_fma, R8(S_FMA))
U32_KERNEL(k_mullo, R8(S_MULLO))
U32_KERNEL(k_arx, R8(S_ARX))

// v_mad_u64_u32 (the Poly1305 limb product): 64-bit accumulators, written in C (the compiler
// emits v_mad_u64_u32 with a discarded carry)
__global__ void k_mad64(uint32_t* out, unsigned long long* st, uint32_t seed) {
  uint64_t a[8];
  uint32_t m[8];
  for (int c = 0; c < 8; c++) {
    a[c] = seed + threadIdx.x + c;
    m[c] = 0x3ffffffu - c;
  }
  const unsigned long long t0c = __builtin_amdgcn_s_memtime();
  const unsigned long long t0r = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < 8; c++) a[c] = (uint64_t)m[c] * (uint32_t)a[c] + a[c];
  }
  stamp_out(st, t0c, t0r);
  uint32_t s = 0;
  for (int c = 0; c < 8; c++) s ^= (uint32_t)a[c] ^ (uint32_t)(a[c] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// v_pk_fma_f32 (two f32 FMAs per lane per instruction)
__global__ void k_pkfma(uint32_t* out, unsigned long long* st, uint32_t seed) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 r[8];
  for (int c = 0; c < 8; c++) r[c] = f2{(float)(seed + c), (float)threadIdx.x};
  const f2 k = {0.999f, 0.998f}, k2 = {1e-3f, 2e-3f};
  const unsigned long long t0c = __builtin_amdgcn_s_memtime();
  const unsigned long long t0r = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < ITERS; i++) {
    asm volatile(
        "v_pk_fma_f32 %0, %0, %8, %9\n v_pk_fma_f32 %1, %1, %8, %9\n"
        "v_pk_fma_f32 %2, %2, %8, %9\n v_pk_fma_f32 %3, %3, %8, %9\n"
        "v_pk_fma_f32 %4, %4, %8, %9\n v_pk_fma_f32 %5, %5, %8, %9\n"
        "v_pk_fma_f32 %6, %6, %8, %9\n v_pk_fma_f32 %7, %7, %8, %9\n"
        : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]),
          "+v"(r[7])
        : "v"(k), "v"(k2));
  }
  stamp_out(st, t0c, t0r);
  float s = 0;
  for (int c = 0; c < 8; c++) s += r[c].x + r[c].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = __float_as_uint(s);
}

typedef void (*KFn)(uint32_t*, unsigned long long*, uint32_t);

struct Res {
  double wall_ms, cyc, ghz;
};

static int run(KFn k, int W, int cus, uint32_t* out, unsigned long long* st, Res& r) {
  const int grid = cus * W, block = 256;
  const int waves = grid * 4;
  hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, out, st, 1u);  // warm-up (clock ramp)
  for (int i = 0; i < 20; i++) hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, out, st, 1u);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, out, st, 1u);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  std::vector<unsigned long long> h(2 * waves);
  CHECK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
  std::vector<double> cyc(waves), ghz(waves);
  for (int w = 0; w < waves; w++) {
    cyc[w] = (double)h[2 * w];
    ghz[w] = (double)h[2 * w] / ((double)h[2 * w + 1] * 10.0);  // ticks of 10 ns
  }
  std::sort(cyc.begin(), cyc.end());
  std::sort(ghz.begin(), ghz.end());
  r.wall_ms = ms;
  r.cyc = cyc[waves / 2];
  r.ghz = ghz[waves / 2];
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return 0;
}

int main() {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  uint32_t* out;
  unsigned long long* st;
  CHECK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
  CHECK(hipMalloc(&st, (size_t)cus * 8 * 4 * 16));
  struct K {
    const char* name;
    KFn fn;
    double lane_ops;  // lane-ops per listed instruction (2 for v_pk_fma_f32)
    int instr_per_iter;
  } ks[] = {
      {"v_add_u32", k_add, 1, 8},        {"v_xor_b32", k_xor, 1, 8},
      {"v_and_b32", k_and, 1, 8},        {"v_alignbit_b32", k_align, 1, 8},
      {"v_perm_b32", k_perm, 1, 8},      {"v_add3_u32", k_add3, 1, 8},
      {"v_xad_u32", k_xad, 1, 8},        {"add/xor/alignbit (ARX)", k_arx, 1, 24},
      {"v_mul_lo_u32", k_mullo, 1, 8},   {"v_mad_u64_u32 (C)", k_mad64, 1, 8},
      {"v_fma_f32", k_fma, 1, 8},        {"v_pk_fma_f32", k_pkfma, 2, 8},
      {"ARX grouped by kind", k_arxg, 1, 24}, {"add/xor dependent", k_ax, 1, 16},
      {"xor+rot16 as 2 SDWA xors", k_xr16, 1, 16}, {"v_bitop3_b32", k_bop3, 1, 8},
      {"6 full-rate : 2 alignbit", k_221, 1, 8},
  };
  printf("# %d CUs; cycles per wave64 instruction per SIMD (in-kernel clock), chip lane-op rate\n", cus);
  printf("# %-24s %2s %9s %9s %8s %10s %12s\n", "instruction", "W", "wall_ms", "cyc/instr", "GHz",
         "Tlane-op/s", "T@2.4GHz-eq");
  for (const K& k : ks) {
    for (int W : {1, 2, 4, 8}) {
      Res r{};
      if (run(k.fn, W, cus, out, st, r)) return 1;
      const double per_wave = (double)ITERS * k.instr_per_iter;
      const double cyc_per = r.cyc / (W * per_wave);
      const double lane_ops = (double)cus * 4 * W * per_wave * 64 * k.lane_ops;
      const double tops = lane_ops / (r.wall_ms * 1e-3) / 1e12;
      printf("  %-24s %2d %9.4f %9.3f %8.3f %10.2f %12.2f\n", k.name, W, r.wall_ms, cyc_per, r.ghz,
             tops, (double)cus * 4 * 64 * k.lane_ops * 2.4 / cyc_per / 1e3);
    }
  }
  return 0;
}
