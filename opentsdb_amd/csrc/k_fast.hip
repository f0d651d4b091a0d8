// k_fast.hip -- instantiates the streaming kernel k_fast for ONE downsample function
// (F_ID, set by the Makefile) and the four uniform row classes (qualifier width 2/4 x
// value length 4/8).
#include "kcommon.h"

#ifndef F_ID
#error "compile with -DF_ID=<downsample function class>"
#endif

#ifndef SHORT_D0
#define SHORT_D0 2     // k_short ring depth, vle class
#endif
#ifndef SHORT_D
#define SHORT_D 2      // k_short ring depth, 4-byte float class
#endif
#ifndef SHORT6_VL4
#define SHORT6_VL4 0   // 4: the float32 class takes 6 a lane too (measured no faster: profiles/r04ab)
#endif
#ifndef ROWS_D
#define ROWS_D 2       // k_rows ring depth (a power of two: 64 rows per descriptor batch)
#endif

namespace tsdb {

template <int F, int QW, int VL, int KR>
static hipError_t launch_fast_k(const GridParams& p, hipStream_t s) {
  constexpr int D = (QW * 2 + VL * 2 <= 16) ? 3 : 2;   // ring depth: chunk registers per lane
  const int64_t nl = p.n_launch > 0 ? p.n_launch : p.n_tiles;
  const int64_t blocks = (nl + p.waves - 1) / p.waves;
  const size_t lds = (size_t)p.wave_lds * p.waves;
  if constexpr (KR == 4 || KR == 5) {   // the staged column layout / the sampled window: k_short only (shortk 1)
    if (p.shortk != 1) return hipErrorNotSupported;
    constexpr int DS = VL == 0 ? SHORT_D0 : (QW * 2 + VL * 2 <= 16) ? SHORT_D : 2;
    if constexpr (QW == 2 && (VL == 0 || VL == SHORT6_VL4)) {
      if (p.short6) {
        if (lds > 65536) {
          hipError_t e = hipFuncSetAttribute((const void*)k_short<F, QW, VL, DS, KR, 6>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
          if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL((k_short<F, QW, VL, DS, KR, 6>), dim3((unsigned)blocks), dim3(64 * p.waves), lds, s, p, p.rows,
                           p.series_row_ptr, p.tile_begin, p.tile_end);
        return hipGetLastError();
      }
    }
    if (lds > 65536) {
      hipError_t e = hipFuncSetAttribute((const void*)k_short<F, QW, VL, DS, KR>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((k_short<F, QW, VL, DS, KR>), dim3((unsigned)blocks), dim3(64 * p.waves), lds, s, p, p.rows,
                       p.series_row_ptr, p.tile_begin, p.tile_end);
    return hipGetLastError();
  } else {
  if (p.shortk == 2) {   // k_rows: multi-row series of rows <= CH (a batch is 64 / DR ring turns)
    constexpr int DR = ROWS_D;
    if (lds > 65536) {
      hipError_t e = hipFuncSetAttribute((const void*)k_rows<F, QW, VL, DR, KR>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((k_rows<F, QW, VL, DR, KR>), dim3((unsigned)blocks), dim3(64 * p.waves), lds, s, p, p.rows,
                       p.series_row_ptr, p.tile_begin, p.tile_end);
    return hipGetLastError();
  }
  if (p.shortk) {
    constexpr int DS = VL == 0 ? SHORT_D0 : (QW * 2 + VL * 2 <= 16) ? SHORT_D : 2;
    if constexpr (QW == 2 && (VL == 0 || VL == SHORT6_VL4)) {
      if (p.short6) {   // rows of <= 384 points: 6 a lane (the kernel hands longer rows back)
        if (lds > 65536) {
          hipError_t e = hipFuncSetAttribute((const void*)k_short<F, QW, VL, DS, KR, 6>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
          if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL((k_short<F, QW, VL, DS, KR, 6>), dim3((unsigned)blocks), dim3(64 * p.waves), lds, s, p, p.rows,
                           p.series_row_ptr, p.tile_begin, p.tile_end);
        return hipGetLastError();
      }
    }
    if (lds > 65536) {
      hipError_t e = hipFuncSetAttribute((const void*)k_short<F, QW, VL, DS, KR>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((k_short<F, QW, VL, DS, KR>), dim3((unsigned)blocks), dim3(64 * p.waves), lds, s, p, p.rows,
                       p.series_row_ptr, p.tile_begin, p.tile_end);
    return hipGetLastError();
  }
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)k_fast<F, QW, VL, D, KR>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((k_fast<F, QW, VL, D, KR>), dim3((unsigned)blocks), dim3(64 * p.waves), lds, s, p, p.rows,
                     p.series_row_ptr, p.tile_begin, p.tile_end);
  return hipGetLastError();
  }
}

// register partials when every slot has its own lane and the series emit needs no rate pass
// (KR 1: the group-by alone; KR 3: with the per-series outputs of the percentile / ordered /
// dense paths; KR 2: every decomposable aggregator's partials at once, tsdbhip_run_multi)
template <int F, int QW, int VL>
static hipError_t launch_fast_t(const GridParams& p, hipStream_t s) {
  if (p.shortk == 3) {   // k_hwin: K > 64 buckets tiling the hour, window by window
    const int64_t nl = (p.n_launch > 0 ? p.n_launch : p.n_tiles) * std::max(1, (int)p.win_split);
    const int64_t blocks = (nl + p.waves - 1) / p.waves;
    const size_t lds = (size_t)p.wave_lds * p.waves;
    if constexpr (QW == 2 && (VL == 0 || VL == 4)) {
      if (p.short6) {   // vle / float32 rows of <= 384 points: 6 a lane (the kernel hands longer rows back)
        if (p.multi)
          hipLaunchKernelGGL((k_hwin<F, QW, VL, 2, true, 6>), dim3((unsigned)blocks), dim3(64 * p.waves), lds, s, p,
                             p.rows, p.series_row_ptr, p.tile_begin, p.tile_end);
        else
          hipLaunchKernelGGL((k_hwin<F, QW, VL, 2, false, 6>), dim3((unsigned)blocks), dim3(64 * p.waves), lds, s, p,
                             p.rows, p.series_row_ptr, p.tile_begin, p.tile_end);
        return hipGetLastError();
      }
    }
    if (p.multi)
      hipLaunchKernelGGL((k_hwin<F, QW, VL, 2, true>), dim3((unsigned)blocks), dim3(64 * p.waves), lds, s, p, p.rows,
                         p.series_row_ptr, p.tile_begin, p.tile_end);
    else
      hipLaunchKernelGGL((k_hwin<F, QW, VL, 2>), dim3((unsigned)blocks), dim3(64 * p.waves), lds, s, p, p.rows,
                         p.series_row_ptr, p.tile_begin, p.tile_end);
    return hipGetLastError();
  }
  if (p.K <= 64 && !p.rate) {
    if (p.multi) return launch_fast_k<F, QW, VL, 2>(p, s);
    if (p.sel_direct && p.sel_win && p.shortk == 1) return launch_fast_k<F, QW, VL, 5>(p, s);   // (k_short, sampled window)
    if (p.sel_direct && p.sel_stage) return launch_fast_k<F, QW, VL, 4>(p, s);   // (k_short, staged columns)
    return (p.sel_direct || p.dense_out) ? launch_fast_k<F, QW, VL, 3>(p, s) : launch_fast_k<F, QW, VL, 1>(p, s);
  }
  if (p.multi) return hipErrorNotSupported;
  return launch_fast_k<F, QW, VL, 0>(p, s);
}

template <>
hipError_t launch_fast_inst<F_ID>(const GridParams& p, int qw, int vl, hipStream_t s) {
  if (qw == 2 && vl == 4) return launch_fast_t<F_ID, 2, 4>(p, s);
  if (qw == 2 && vl == 8) return launch_fast_t<F_ID, 2, 8>(p, s);
  if (qw == 4 && vl == 4) return launch_fast_t<F_ID, 4, 4>(p, s);
  if (qw == 4 && vl == 8) return launch_fast_t<F_ID, 4, 8>(p, s);
  if (qw == 2 && vl == 0) return launch_fast_t<F_ID, 2, 0>(p, s);
  return hipErrorNotSupported;
}

}  // namespace tsdb
