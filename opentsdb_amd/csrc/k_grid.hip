// k_grid.hip -- instantiates the general kernel k_grid for ONE downsample function
// (F_ID, set by the Makefile), so the eleven functions compile as parallel objects.
#include "kcommon.h"

#ifndef F_ID
#error "compile with -DF_ID=<downsample function class>"
#endif

namespace tsdb {

template <int F, bool G>
static hipError_t launch_grid_t(const GridParams& p, hipStream_t s) {
  const int64_t nl = p.n_launch > 0 ? p.n_launch : p.n_tiles;
  const int64_t blocks = (nl + p.waves - 1) / p.waves;
  const size_t lds = (size_t)p.wave_lds * p.waves;
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)k_grid<F, G>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((k_grid<F, G>), dim3((unsigned)blocks), dim3(64 * p.waves), lds, s, p);
  return hipGetLastError();
}

template <>
hipError_t launch_grid_inst<F_ID>(const GridParams& p, hipStream_t s) {
  return p.g_dense ? launch_grid_t<F_ID, true>(p, s) : launch_grid_t<F_ID, false>(p, s);
}

}  // namespace tsdb
