// hbm_probe.hip — achievable HBM bandwidth on this MI355X for the access
// shapes the Jacobian kernel uses (streaming 8-B and 16-B per lane stores,
// streaming reads, copy).  Build + run:
//   hipcc --offload-arch=gfx950 -O3 tools/hbm_probe.hip -o /tmp/hbm_probe && /tmp/hbm_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

__global__ void write16(double2* __restrict__ d, size_t n, double v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    d[i] = make_double2(v, v + 1.0);
}
__global__ void write8(double* __restrict__ d, size_t n, double v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    d[i] = v;
}
__global__ void read16(const double2* __restrict__ s, size_t n, double* out) {
  double acc = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const double2 x = s[i];
    acc += x.x + x.y;
  }
  if (acc == 1234.5) out[0] = acc;
}
__global__ void copy16(const double2* __restrict__ s, double2* __restrict__ d, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    d[i] = s[i];
}

int main() {
  const size_t bytes = (size_t)2700 << 20;
  double *a, *b;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMalloc(&b, bytes));
  CHECK(hipMemset(a, 0, bytes));
  CHECK(hipMemset(b, 0, bytes));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int grids[] = {1024, 4096, 16384};
  for (int g : grids) {
    for (int k = 0; k < 4; ++k) {
      auto launch = [&]() {
        if (k == 0) hipLaunchKernelGGL(write16, dim3(g), dim3(256), 0, 0, (double2*)a, bytes / 16, 1.0);
        if (k == 1) hipLaunchKernelGGL(write8, dim3(g), dim3(256), 0, 0, a, bytes / 8, 1.0);
        if (k == 2) hipLaunchKernelGGL(read16, dim3(g), dim3(256), 0, 0, (const double2*)a, bytes / 16, b);
        if (k == 3) hipLaunchKernelGGL(copy16, dim3(g), dim3(256), 0, 0, (const double2*)a, (double2*)b, bytes / 32);
      };
      launch();
      CHECK(hipEventRecord(e0));
      const int reps = 10;
      for (int r = 0; r < reps; ++r) launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double moved = (k == 3) ? (double)bytes : (double)bytes;  // copy: bytes/2 read + bytes/2 written
      const char* nm[] = {"write16", "write8", "read16", "copy16"};
      std::printf("{\"kernel\": \"%s\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", nm[k], g, ms / reps,
                  moved / (ms / reps * 1e-3) / 1e9);
    }
  }
  return 0;
}
