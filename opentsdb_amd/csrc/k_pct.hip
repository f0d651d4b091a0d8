// k_pct.hip -- downsampling with order-statistic functions: p999 ... p50, ep*r3, ep*r7
// and median (Aggregators.PercentileAgg, src/core/Aggregators.java:657-708; Median
// :397-431), then the group-by step over the resulting bucket values.
//
//  * k_pct   one wave per series.  Decodes the series' rows in 512-datapoint chunks
//            (decode_generic: every row class), gathers each bucket's non-NaN values in
//            an LDS buffer, and at the bucket's end sorts them -- in registers with a
//            64-lane bitonic network when <= 512 values (8 per lane), in LDS otherwise
//            (<= PCT_CAP) -- and selects.  Downsampler.runDouble is always called, and
//            PercentileAgg.runDouble ignores the estimation type (:690), so every
//            percentile uses commons-math3 3.4.1 LEGACY: pos = p (n + 1).
//  * k_emit  one wave per tile: the bucket values -> SpanGroup contributions (LERP, fill,
//            rate), exactly emit_series of k_grid, into tile partials for k_reduce.
#include "kcommon.h"

namespace tsdb {

// compare-exchange keeping (lo, hi); ties keep both values (multiset preserved)
__device__ __forceinline__ void cx(double& a, double& b, bool up) {
  const bool sw = up ? (b < a) : (a < b);
  const double t = sw ? b : a;
  b = sw ? a : b;
  a = t;
}

// Bitonic sort of 512 doubles held 8 per lane (element e = lane * 8 + j), ascending.
__device__ __forceinline__ void sort512(double v[DPL]) {
  const int lane = lane_id();
#pragma unroll
  for (int k = 2; k <= 512; k <<= 1) {
#pragma unroll
    for (int jj = k >> 1; jj > 0; jj >>= 1) {
      if (jj >= DPL) {
        const int lm = jj / DPL;
#pragma unroll
        for (int j = 0; j < DPL; j++) {
          const double o = __shfl_xor(v[j], lm, 64);
          const int e = lane * DPL + j;
          const bool up = (e & k) == 0;
          const bool lower = (e & jj) == 0;
          // the lower element of an ascending pair keeps the min
          v[j] = (up == lower) ? ((o < v[j]) ? o : v[j]) : ((v[j] < o) ? o : v[j]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < DPL; j++) {
          const int q = j ^ jj;
          if (q > j) {
            const int e = lane * DPL + j;
            cx(v[j], v[q], (e & k) == 0);
          }
        }
      }
    }
  }
}

// Bitonic sort of the first N (power of two) doubles of an LDS buffer by one wave.
__device__ __forceinline__ void sort_lds(double* buf, int N) {
  const int lane = lane_id();
  for (int k = 2; k <= N; k <<= 1) {
    for (int jj = k >> 1; jj > 0; jj >>= 1) {
      for (int i = lane; i < N / 2; i += 64) {
        const int a = 2 * jj * (i / jj) + (i % jj);
        const int b = a + jj;
        double x = buf[a], y = buf[b];
        cx(x, y, (a & k) == 0);
        buf[a] = x;
        buf[b] = y;
      }
      WAVE_SYNC();
    }
  }
}

__device__ __forceinline__ double pct_quantile(int fn) {
  const int i = (fn - TSDB_AGG_P999) % 6;
  return i == 0 ? 99.9 : i == 1 ? 99.0 : i == 2 ? 95.0 : i == 3 ? 90.0 : i == 4 ? 75.0 : 50.0;
}

// Order statistic of the n sorted values; get(i) returns element i (wave-uniform i).
template <class Get>
__device__ __forceinline__ double select_sorted(int fn, int n, Get get) {
  if (fn == TSDB_AGG_MEDIAN) return get(n / 2);   // Median.runDouble: sorted[size / 2]
  if (n == 1) return get(0);
  // Percentile.evaluate, LEGACY: pos = p (n + 1); estimate() (commons-math3 3.4.1)
  const double p = pct_quantile(fn) / 100.0;
  const double pos = (p == 0.0) ? 0.0 : (p == 1.0 ? (double)n : p * (double)(n + 1));
  const double fpos = floor(pos);
  const int ip = (int)fpos;
  const double dif = pos - fpos;
  if (pos < 1) return get(0);
  if (pos >= (double)n) return get(n - 1);
  const double lower = get(ip - 1);
  const double upper = get(ip);
  return lower + dif * (upper - lower);
}

__device__ __forceinline__ double reg_at(const double v[DPL], int i) {
  double t = v[0];
#pragma unroll
  for (int j = 1; j < DPL; j++) if ((i & (DPL - 1)) == j) t = v[j];
  return __shfl(t, i / DPL, 64);
}

// value of a finished bucket holding n non-NaN values in buf (tot values incl. NaN)
__device__ __forceinline__ double bucket_value(const GridParams& p, double* buf, int n) {
  const int lane = lane_id();
  if (n == 0) return (double)NAN;
  if (n > PCT_CAP) {
    if (lane == 0) set_err(p.err, TSDB_E_NOT_IMPLEMENTED);
    return (double)NAN;
  }
  if (n <= CH) {
    double v[DPL];
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      const int e = lane * DPL + j;
      v[j] = e < n ? buf[e] : (double)INFINITY;
    }
    sort512(v);
    return select_sorted(p.sel_fn, n, [&](int i) { return reg_at(v, i); });
  }
  int N = CH;
  while (N < n) N <<= 1;
  for (int e = n + lane; e < N; e += 64) buf[e] = (double)INFINITY;
  WAVE_SYNC();
  sort_lds(buf, N);
  return select_sorted(p.sel_fn, n, [&](int i) { return buf[i]; });
}

__global__ __launch_bounds__(128) void k_pct(GridParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  unsigned char* base = smem + (int64_t)wave * (VBUF + PCT_CAP * 8);
  WaveLds W;
  W.dpv = (double*)base;
  W.vbuf = base;
  W.mq = (uint32_t*)base;
  W.mv = (uint32_t*)(base + CH * 4);
  double* buf = (double*)(base + VBUF);
  const int K = (int)p.K;
  const int64_t s = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave;
  if (s >= p.n_series) return;
  double* dense = p.pre_dense + s * K;
  uint8_t* pres = p.pre_pres + s * K;
  for (int k = lane; k < K; k += 64) pres[k] = 0;
  int cur = -1;      // open bucket
  int cnt = 0;       // its non-NaN values (in buf)
  const int64_t r0 = p.series_row_ptr[s], r1 = p.series_row_ptr[s + 1];
  for (int64_t r = r0; r < r1; r++) {
    const RowDesc d = p.rows[r];
    if ((int64_t)d.base < p.ss) continue;
    if ((int64_t)d.base >= p.se) break;
    if (d.flags & ROW_ERR) { if (lane == 0) set_err(p.err, TSDB_E_ILLEGAL_DATA); continue; }
    const RowGeom g = row_geom(p, d.base);
    int64_t vcur = 0;
    for (int64_t c0 = 0; c0 < (int64_t)d.ndp; c0 += CH) {
      int slot[DPL];
      double val[DPL];
      decode_generic(p, d, g, c0, W, vcur, slot, val);
      bool left[DPL];
#pragma unroll
      for (int j = 0; j < DPL; j++) left[j] = slot[j] >= 0;
      for (;;) {
        int mn = INT32_MAX;
#pragma unroll
        for (int j = 0; j < DPL; j++) if (left[j]) mn = min(mn, slot[j]);
        mn = wave_min(mn);
        if (mn == INT32_MAX) break;
        if (mn != cur) {
          if (cur >= 0) {
            const double x = bucket_value(p, buf, cnt);
            if (lane == 0) { dense[cur] = x; pres[cur] = 1; }
          }
          cur = mn;
          cnt = 0;
          WAVE_SYNC();
        }
        int mine = 0;
#pragma unroll
        for (int j = 0; j < DPL; j++) if (left[j] && slot[j] == mn && !isnan(val[j])) mine++;
        const int incl = wave_incl_sum(mine);
        int o = cnt + incl - mine;
#pragma unroll
        for (int j = 0; j < DPL; j++) {
          if (left[j] && slot[j] == mn) {
            if (!isnan(val[j])) {
              if (o < PCT_CAP) buf[o] = val[j];
              o++;
            }
            left[j] = false;
          }
        }
        cnt += __shfl(incl, 63, 64);
        WAVE_SYNC();
      }
    }
  }
  if (cur >= 0) {
    const double x = bucket_value(p, buf, cnt);
    if (lane == 0) { dense[cur] = x; pres[cur] = 1; }
  }
}

// One wave per tile: SpanGroup contributions of precomputed bucket values.
__global__ __launch_bounds__(256) void k_emit(GridParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t tile = (int64_t)blockIdx.x * p.waves + wave;
  if (tile >= p.n_tiles) return;
  const int K = (int)p.K;
  unsigned char* b = smem + (int64_t)wave * p.wave_lds;
  WaveLds W;
  if (p.g_dense) {   // large K: tile scratch in HBM
    W.rate = p.rate ? p.g_rate + tile * K : nullptr;
    W.part.a = p.part.a + tile * K;
    W.part.b = p.part.b + tile * K;
    W.part.n = p.part.n + tile * K;
    W.part.f = p.part.f + tile * K;
  } else {
    int64_t o = 0;
    W.part.a = (double*)(b + o); o += align16(K * 8);
    W.part.b = (double*)(b + o); o += align16(K * 8);
    W.part.n = (uint32_t*)(b + o); o += align16(K * 4);
    W.part.f = (uint32_t*)(b + o); o += align16(K * 4);
    W.rate = p.rate ? (double*)(b + o) : nullptr;
  }
  for (int k = lane; k < K; k += 64) part_init(p.ga, W.part, k);
  bool active = false;
  for (int64_t s = p.tile_begin[tile]; s < p.tile_end[tile]; s++) {
    bool any = false;
    for (int64_t r = p.series_row_ptr[s]; r < p.series_row_ptr[s + 1]; r++) {
      const uint32_t base = p.rows[r].base;
      if ((int64_t)base >= p.ss && (int64_t)base < p.se) { any = true; break; }
    }
    if (!any) continue;
    active = true;
    W.dense = p.pre_dense + s * K;
    W.pres = p.pre_pres + s * K;
    emit_series(p, W, K);
  }
  if (active && lane == 0) atomicOr(&p.group_active[p.tile_group[tile]], 1u);
  if (!p.g_dense) {
    WAVE_SYNC();
    for (int k = lane; k < K; k += 64) {
      p.part.a[tile * K + k] = W.part.a[k];
      p.part.b[tile * K + k] = W.part.b[k];
      p.part.n[tile * K + k] = W.part.n[k];
      p.part.f[tile * K + k] = W.part.f[k];
    }
  }
}

hipError_t launch_pct(const GridParams& p, hipStream_t s) {
  if (p.n_series == 0) return hipSuccess;
  const size_t lds = 2 * (size_t)(VBUF + PCT_CAP * 8);
  hipError_t e = hipFuncSetAttribute((const void*)k_pct, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_pct, dim3((unsigned)((p.n_series + 1) / 2)), dim3(128), lds, s, p);
  return hipGetLastError();
}

hipError_t launch_emit(const GridParams& p, hipStream_t s) {
  if (p.n_tiles == 0) return hipSuccess;
  const int64_t blocks = (p.n_tiles + p.waves - 1) / p.waves;
  const size_t lds = (size_t)p.wave_lds * p.waves;
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)k_emit, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_emit, dim3((unsigned)blocks), dim3(64 * p.waves), lds, s, p);
  return hipGetLastError();
}

}  // namespace tsdb
