// Resident workgroups per CU of the kernels whose hand-offs use sc1 loads
// without an acquire (csrc/cholesky.cpp: blocks_per_cu must be 1 for them).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/occupancy_probe.cpp -lrocsolver -lrocblas -o tools/probes/occupancy_probe.bin
#include "../../semantic-bundle-adjustment-colmap_amd/csrc/cholesky.cpp"

#include <cstdio>

int main() {
  using namespace miba;
  constexpr CholConfig kDef{};
  printf("panel_factor_kernel<%d, true, %d>: %d per CU\n", kDef.tile_factor, kDef.panel_wait,
         blocks_per_cu(reinterpret_cast<const void*>(&panel_factor_kernel<kDef.tile_factor, true, kDef.panel_wait>), 256));
  printf("trsv_sweep_kernel<true, true>: %d per CU\n",
         blocks_per_cu(reinterpret_cast<const void*>(&trsv_sweep_kernel<true, true>), 64 * kSweepWaves));
  printf("trsv_sweep_kernel<false, true>: %d per CU\n",
         blocks_per_cu(reinterpret_cast<const void*>(&trsv_sweep_kernel<false, true>), 64 * kSweepWaves));
  printf("sweep_sc1_ok %d\n", (int)sweep_sc1_ok());
  return 0;
}
