// valu_rates.hip -- issue rate of the VALU instructions the int16 / fp32
// scan kernels spend their time in, measured on the whole chip: every SIMD
// runs 8 waves, each wave issues ITER x 8 independent copies of one
// instruction (inline asm, so the compiler cannot fold or reorder them).
// Reported: wave-instructions per SIMD-cycle at the measured clock
// (1.0 = one wave64 instruction every cycle per SIMD, 0.25 = every 4).
//
// build: make -C tools/tune valu_rates ; run: tools/tune/valu_rates
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                    \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) {                                                                      \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);     \
      exit(1);                                                                                   \
    }                                                                                            \
  } while (0)

constexpr int ITER = 2048;

#define REP8(S) S S S S S S S S

// 32-bit destination ops: v0..v7 independent accumulators
#define K32(NAME, ASM)                                                                           \
  __global__ __launch_bounds__(256) void NAME(unsigned* out, unsigned seed) {                    \
    unsigned a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11,     \
             a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19, b = seed ^ 0x5555;                        \
    for (int i = 0; i < ITER; ++i) {                                                             \
      asm volatile(ASM : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),  \
                   "+v"(a7) : "v"(b));                                                           \
    }                                                                                            \
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                  \
  }
#define OP32(OP) OP " %0, %0, %8\n" OP " %1, %1, %8\n" OP " %2, %2, %8\n" OP " %3, %3, %8\n" \
                 OP " %4, %4, %8\n" OP " %5, %5, %8\n" OP " %6, %6, %8\n" OP " %7, %7, %8\n"
K32(k_add_u32, OP32("v_add_u32"))
K32(k_mul_hi_u32, OP32("v_mul_hi_u32"))
K32(k_perm, "v_perm_b32 %0, %0, %8, %8\n v_perm_b32 %1, %1, %8, %8\n v_perm_b32 %2, %2, %8, %8\n v_perm_b32 %3, %3, %8, %8\n"
            "v_perm_b32 %4, %4, %8, %8\n v_perm_b32 %5, %5, %8, %8\n v_perm_b32 %6, %6, %8, %8\n v_perm_b32 %7, %7, %8, %8\n")
K32(k_sub_sdwa, "v_sub_u32_sdwa %0, %0, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1\n"
                "v_sub_u32_sdwa %1, %1, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1\n"
                "v_sub_u32_sdwa %2, %2, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1\n"
                "v_sub_u32_sdwa %3, %3, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1\n"
                "v_sub_u32_sdwa %4, %4, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1\n"
                "v_sub_u32_sdwa %5, %5, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1\n"
                "v_sub_u32_sdwa %6, %6, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1\n"
                "v_sub_u32_sdwa %7, %7, %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1\n")
K32(k_dot2_i16, "v_dot2_i32_i16 %0, %8, %8, %0\n v_dot2_i32_i16 %1, %8, %8, %1\n v_dot2_i32_i16 %2, %8, %8, %2\n v_dot2_i32_i16 %3, %8, %8, %3\n"
                "v_dot2_i32_i16 %4, %8, %8, %4\n v_dot2_i32_i16 %5, %8, %8, %5\n v_dot2_i32_i16 %6, %8, %8, %6\n v_dot2_i32_i16 %7, %8, %8, %7\n")
K32(k_bfe_i32, "v_bfe_i32 %0, %0, 16, 16\n v_bfe_i32 %1, %1, 16, 16\n v_bfe_i32 %2, %2, 16, 16\n v_bfe_i32 %3, %3, 16, 16\n"
               "v_bfe_i32 %4, %4, 16, 16\n v_bfe_i32 %5, %5, 16, 16\n v_bfe_i32 %6, %6, 16, 16\n v_bfe_i32 %7, %7, 16, 16\n")

// 64-bit register pairs (f64 ops)
#define K64(NAME, ASM)                                                                           \
  __global__ __launch_bounds__(256) void NAME(unsigned* out, unsigned seed) {                    \
    double a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11,       \
           a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19, b = 1.0000001;                              \
    for (int i = 0; i < ITER; ++i) {                                                             \
      asm volatile(ASM : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),  \
                   "+v"(a7) : "v"(b));                                                           \
    }                                                                                            \
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);     \
  }
K64(k_add_f64, OP32("v_add_f64"))
K64(k_mul_f64, OP32("v_mul_f64"))
// cvt round trips: i32 -> f64 -> i32 and f32 -> f64 -> f32 (two instructions per copy)
#define KRT(NAME, A, B)                                                                          \
  __global__ __launch_bounds__(256) void NAME(unsigned* out, unsigned seed) {                    \
    unsigned a[8];                                                                               \
    double d[8];                                                                                 \
    for (int j = 0; j < 8; ++j) a[j] = seed * (j + 1) + threadIdx.x;                             \
    for (int i = 0; i < ITER; ++i) {                                                             \
      _Pragma("unroll") for (int j = 0; j < 8; ++j) asm volatile(A " %0, %1" : "=v"(d[j]) : "v"(a[j])); \
      _Pragma("unroll") for (int j = 0; j < 8; ++j) asm volatile(B " %0, %1" : "=v"(a[j]) : "v"(d[j])); \
    }                                                                                            \
    unsigned r = 0;                                                                              \
    for (int j = 0; j < 8; ++j) r ^= a[j];                                                       \
    out[blockIdx.x * 256 + threadIdx.x] = r;                                                     \
  }
KRT(k_cvt_f64_i32_rt, "v_cvt_f64_i32", "v_cvt_i32_f64")
KRT(k_cvt_f64_f32_rt, "v_cvt_f64_f32", "v_cvt_f32_f64")
K64(k_fma_f64, "v_fma_f64 %0, %0, %8, %8\n v_fma_f64 %1, %1, %8, %8\n v_fma_f64 %2, %2, %8, %8\n v_fma_f64 %3, %3, %8, %8\n"
               "v_fma_f64 %4, %4, %8, %8\n v_fma_f64 %5, %5, %8, %8\n v_fma_f64 %6, %6, %8, %8\n v_fma_f64 %7, %7, %8, %8\n")

int main() {
  int dev = 0, cus = 0, clk = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev));  // kHz
  const int grid = cus * 8;  // 8 workgroups of 4 waves per CU = 8 waves per SIMD
  unsigned* out;
  CK(hipMalloc(&out, (size_t)grid * 256 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct K { const char* name; void (*f)(unsigned*, unsigned); int insts_per_iter; };
  K ks[] = {{"v_add_u32", k_add_u32, 8},         {"v_mul_hi_u32", k_mul_hi_u32, 8},
            {"v_perm_b32", k_perm, 8},           {"v_sub_u32_sdwa", k_sub_sdwa, 8},
            {"v_dot2_i32_i16", k_dot2_i16, 8},   {"v_bfe_i32", k_bfe_i32, 8},
            {"v_add_f64", k_add_f64, 8},         {"v_mul_f64", k_mul_f64, 8},
            {"v_fma_f64", k_fma_f64, 8},         {"cvt_i32_f64+cvt_f64_i32", k_cvt_f64_i32_rt, 16},
            {"cvt_f32_f64+cvt_f64_f32", k_cvt_f64_f32_rt, 16}};
  printf("CUs=%d nominal clock %.0f MHz; wave-instructions per SIMD-cycle at that clock\n", cus, clk / 1e3);
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(grid), dim3(256), 0, 0, out, 1u);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k.f, dim3(grid), dim3(256), 0, 0, out, (unsigned)r);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    const double wave_insts = (double)grid * 4 * ITER * k.insts_per_iter;  // 4 waves per workgroup
    const double simd_cycles = (double)cus * 4 * (best * 1e-3) * (clk * 1e3);
    printf("%-28s %8.3f ms  %.3f per SIMD-cycle (%.1f cycles per wave-instruction)\n", k.name, best,
           wave_insts / simd_cycles, simd_cycles / wave_insts);
  }
  return 0;
}
