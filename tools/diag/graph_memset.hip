// graph_memset.hip -- does a byte-valued hipMemsetAsync captured into a HIP
// graph write the same bytes as the eager call?  (Evidence for why the
// look-back scan resets its workspace with its own kernel.)  Reads only
// inside its own buffer.
// build: hipcc --offload-arch=gfx950 -O2 -o graph_memset graph_memset.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

static int check(const char* what, unsigned char* d, size_t n, size_t cap) {
  std::vector<unsigned char> h(cap);
  CK(hipMemcpy(h.data(), d, cap, hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (size_t i = 0; i < n; ++i) bad += h[i] != 0x80;
  size_t spill = 0;
  for (size_t i = n; i < cap; ++i) spill += h[i] != 0;
  printf("%-28s bytes=%zu wrong=%zu beyond_end_written=%zu first8=%02x %02x %02x %02x %02x %02x %02x %02x\n", what, n,
         bad, spill, h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]);
  return 0;
}

int main() {
  const size_t cap = 1 << 16;
  unsigned char* d;
  CK(hipMalloc(&d, cap));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  for (size_t n : {4168ul, 4096ul, 4104ul, 4194560ul > cap ? 32768ul : 4194560ul}) {
    CK(hipMemset(d, 0, cap));
    CK(hipMemsetAsync(d, 0x80, n, s));
    CK(hipStreamSynchronize(s));
    check("eager", d, n, cap);
    CK(hipMemset(d, 0, cap));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    CK(hipMemsetAsync(d, 0x80, n, s));
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    check("captured + replayed", d, n, cap);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
