#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dvec4 __attribute__((ext_vector_type(4)));
// lane l supplies a = fa(l), b = fb(l); D values printed per (lane, r)
__global__ void k(int mode, double* D) {
  int l = threadIdx.x;
  double a, b;
  if (mode == 0) { a = (l / 16 == 0) ? (l % 16 + 1) : 0.0; b = (l / 16 == 0) ? 100.0 * (l % 16 + 1) : 0.0; }
  else { a = l + 1; b = (l == 0) ? 1.0 : 0.0; }  // probe: which lanes' a meet lane 0's b
  dvec4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[l * 4 + r] = acc[r];
}
int main() {
  double* dD; double D[256];
  hipMalloc(&dD, 2048);
  for (int mode = 0; mode < 2; ++mode) {
    k<<<1, 64>>>(mode, dD);
    hipMemcpy(D, dD, 2048, hipMemcpyDeviceToHost);
    printf("mode %d\n", mode);
    for (int l = 0; l < 64; ++l) { printf("l%02d:", l); for (int r = 0; r < 4; ++r) printf(" %8g", D[l*4+r]); printf("\n"); }
  }
  return 0;
}
