// membw.hip -- MI355X HBM calibration for a 1-read + 1-write stream of 16-B
// units: read-only, write-only and copy kernels in two access shapes
//   gs  : grid-stride (all workgroups sweep the buffer together)
//   seg : each workgroup streams its own contiguous segment (the scan's shape)
// with plain / non-temporal loads and stores.  Interleaved rounds in one
// process; median GB/s reported (bytes actually moved by the kernel).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

template <int NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  if constexpr (NT & 2) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
  if constexpr (NT & 1) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// ---- grid-stride ----
template <int NT, int UNR, int MODE>  // MODE 0 copy, 1 read, 2 write
__global__ __launch_bounds__(256) void k_gs(const u32x4* __restrict__ in, u32x4* __restrict__ out, long long n4,
                                            u32x4* sink) {
  const long long stride = (long long)gridDim.x * 256 * UNR;
  u32x4 acc = {0, 0, 0, 0};
  for (long long i = (long long)blockIdx.x * 256 * UNR + threadIdx.x; i < n4; i += stride) {
    u32x4 v[UNR];
    if constexpr (MODE != 2) {
#pragma unroll
      for (int u = 0; u < UNR; ++u) v[u] = ld<NT>(in + i + u * 256);
    } else {
#pragma unroll
      for (int u = 0; u < UNR; ++u) v[u] = u32x4{(uint32_t)i, 1u, 2u, (uint32_t)u};
    }
    if constexpr (MODE == 1) {
#pragma unroll
      for (int u = 0; u < UNR; ++u) acc ^= v[u];
    } else {
#pragma unroll
      for (int u = 0; u < UNR; ++u) st<NT>(out + i + u * 256, v[u]);
    }
  }
  if constexpr (MODE == 1)
    if (acc.x == 0x12345678u && acc.y == 7u) sink[0] = acc;
}

// ---- per-workgroup contiguous segment; PD register chunks in flight ----
template <int NT, int UNR, int MODE>
__global__ __launch_bounds__(256) void k_seg(const u32x4* __restrict__ in, u32x4* __restrict__ out, long long n4,
                                             u32x4* sink) {
  const long long seg = (n4 + gridDim.x - 1) / gridDim.x;
  const long long b = (long long)blockIdx.x * seg;
  const long long e = min(b + seg, n4);
  u32x4 acc = {0, 0, 0, 0};
  for (long long i = b + threadIdx.x; i < e; i += 256 * UNR) {
    u32x4 v[UNR];
    if constexpr (MODE != 2) {
#pragma unroll
      for (int u = 0; u < UNR; ++u)
        if (i + u * 256 < e) v[u] = ld<NT>(in + i + u * 256);
    } else {
#pragma unroll
      for (int u = 0; u < UNR; ++u) v[u] = u32x4{(uint32_t)i, 1u, 2u, (uint32_t)u};
    }
    if constexpr (MODE == 1) {
#pragma unroll
      for (int u = 0; u < UNR; ++u) acc ^= v[u];
    } else {
#pragma unroll
      for (int u = 0; u < UNR; ++u)
        if (i + u * 256 < e) st<NT>(out + i + u * 256, v[u]);
    }
  }
  if constexpr (MODE == 1)
    if (acc.x == 0x12345678u && acc.y == 7u) sink[0] = acc;
}

// ---- flat: workgroup b handles units [b*256*UNR, (b+1)*256*UNR), no loop ----
template <int NT, int UNR, int MODE>
__global__ __launch_bounds__(256) void k_flat(const u32x4* __restrict__ in, u32x4* __restrict__ out, long long n4,
                                              u32x4* sink) {
  const long long i = (long long)blockIdx.x * 256 * UNR + threadIdx.x;
  u32x4 v[UNR];
  u32x4 acc = {0, 0, 0, 0};
  if constexpr (MODE != 2) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) v[u] = ld<NT>(in + i + u * 256);
  } else {
#pragma unroll
    for (int u = 0; u < UNR; ++u) v[u] = u32x4{(uint32_t)i, 1u, 2u, (uint32_t)u};
  }
  if constexpr (MODE == 1) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) acc ^= v[u];
    if (acc.x == 0x12345678u && acc.y == 7u) sink[0] = acc;
  } else {
#pragma unroll
    for (int u = 0; u < UNR; ++u) st<NT>(out + i + u * 256, v[u]);
  }
}

struct V {
  std::string name;
  double bytes;
  std::function<void(hipStream_t)> go;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 30;  // floats per buffer
  const int rounds = argc > 2 ? atoi(argv[2]) : 8;
  const long long n = 1LL << lg, n4 = n / 4;
  u32x4 *x, *y, *sink;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y, n * 4));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(x, 1, n * 4));
  CK(hipMemset(y, 2, n * 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  std::vector<V> vs;
  const double B = (double)n * 4;
#define GS(NT, U, M, G)                                                                              \
  vs.push_back({std::string(M == 0 ? "copy" : M == 1 ? "read" : "write") + " gs  NT" #NT " U" #U " g" #G, \
                (M == 0 ? 2 : 1) * B, [=](hipStream_t st) {                                           \
                  hipLaunchKernelGGL((k_gs<NT, U, M>), dim3(G), dim3(256), 0, st, x, y, n4, sink);     \
                }});
#define SG(NT, U, M, G)                                                                              \
  vs.push_back({std::string(M == 0 ? "copy" : M == 1 ? "read" : "write") + " seg NT" #NT " U" #U " g" #G, \
                (M == 0 ? 2 : 1) * B, [=](hipStream_t st) {                                           \
                  hipLaunchKernelGGL((k_seg<NT, U, M>), dim3(G), dim3(256), 0, st, x, y, n4, sink);    \
                }});
#define FL(NT, U, M)                                                                                  \
  vs.push_back({std::string(M == 0 ? "copy" : M == 1 ? "read" : "write") + " flat NT" #NT " U" #U,           \
                (M == 0 ? 2 : 1) * B, [=](hipStream_t st) {                                               \
                  hipLaunchKernelGGL((k_flat<NT, U, M>), dim3((unsigned)(n4 / (256 * U))), dim3(256), 0, st, x, y, \
                                     n4, sink);                                                           \
                }});
  // read-only and write-only ceilings
  GS(2, 4, 1, 4096) FL(0, 1, 1) FL(2, 1, 1) FL(2, 4, 1) SG(2, 4, 1, 1024)
  GS(0, 4, 2, 4096) FL(0, 1, 2) FL(1, 1, 2) FL(0, 4, 2) FL(0, 2, 2) SG(0, 4, 2, 1024) SG(0, 4, 2, 4096)
  // copy, grid-stride
  GS(3, 2, 0, 8192) GS(3, 2, 0, 16384) GS(3, 1, 0, 32768) GS(2, 2, 0, 16384) GS(0, 2, 0, 16384)
  // copy, flat
  FL(0, 1, 0) FL(2, 1, 0) FL(3, 1, 0) FL(0, 2, 0) FL(2, 2, 0) FL(3, 2, 0) FL(2, 4, 0) FL(3, 4, 0) FL(2, 8, 0)
  // copy, contiguous segment per workgroup: segment-count sweep
  SG(3, 4, 0, 1024) SG(3, 4, 0, 1534) SG(3, 4, 0, 1536) SG(3, 4, 0, 2048) SG(3, 4, 0, 3072) SG(3, 4, 0, 4096)
  SG(3, 4, 0, 8192) SG(3, 4, 0, 16384) SG(3, 4, 0, 65536) SG(2, 4, 0, 4096) SG(2, 4, 0, 16384)
  vs.push_back({"hipMemcpyDtoD", 2 * B, [=](hipStream_t st) { hipMemcpyAsync(y, x, n * 4, hipMemcpyDeviceToDevice, st); }});
  vs.push_back({"hipMemsetD32 (write)", B, [=](hipStream_t st) { hipMemsetD32Async((hipDeviceptr_t)y, 7, n, st); }});

  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (auto& v : vs) v.go(s);
  CK(hipStreamSynchronize(s));
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vs) {
      CK(hipEventRecord(a, s));
      v.go(s);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      v.ms.push_back(ms);
    }
  printf("buffers 2 x %.2f GiB\n%-30s %9s %9s %9s\n", B / (1 << 30), "kernel", "med_ms", "GB/s", "frac8T");
  for (auto& v : vs) {
    auto m = v.ms;
    std::sort(m.begin(), m.end());
    const double gbs = v.bytes / (m[m.size() / 2] * 1e-3) / 1e9;
    printf("%-30s %9.4f %9.1f %9.4f\n", v.name.c_str(), m[m.size() / 2], gbs, gbs / 8000.0);
  }
  return 0;
}
