// k_pct.hip -- downsampling with order-statistic functions: p999 ... p50, ep*r3, ep*r7
// and median (Aggregators.PercentileAgg, src/core/Aggregators.java:657-708; Median
// :397-431), then the group-by step over the resulting bucket values.
//
//  * k_pct   one wave per series.  Decodes the series' rows in 512-datapoint chunks
//            (prefetched register decode for uniform rows, decode_generic otherwise),
//            gathers each bucket's non-NaN values in an LDS buffer, and at the bucket's
//            end sorts them -- in registers with a 64-lane bitonic network (<= 512
//            values, 8 per lane); series with larger buckets go to a second pass that
//            sorts in LDS (<= PCT_CAP values) -- and selects.  Downsampler.runDouble is always called, and
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

// one DPP step of a 64-lane max / min of a double (identity where the source is invalid)
template <bool MAX, int CTRL, int RMASK>
__device__ __forceinline__ double dpp_ext_step(double x) {
  const double id = MAX ? -(double)INFINITY : (double)INFINITY;
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(id), __double2loint(x), CTRL, RMASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(id), __double2hiint(x), CTRL, RMASK, 0xF, false);
  const double y = __hiloint2double(hi, lo);
  return MAX ? fmax(x, y) : fmin(x, y);
}

// 64-lane max / min of a double with DPP (row_shr + row_bcast), result in every lane
template <bool MAX>
__device__ __forceinline__ double wave_ext_f64(double x) {
  x = dpp_ext_step<MAX, 0x111, 0xF>(x);   // row_shr:1
  x = dpp_ext_step<MAX, 0x112, 0xF>(x);   // row_shr:2
  x = dpp_ext_step<MAX, 0x114, 0xF>(x);   // row_shr:4
  x = dpp_ext_step<MAX, 0x118, 0xF>(x);   // row_shr:8
  x = dpp_ext_step<MAX, 0x142, 0xA>(x);   // row_bcast:15 -> rows 1, 3
  x = dpp_ext_step<MAX, 0x143, 0xC>(x);   // row_bcast:31 -> rows 2, 3
  const int lo = __builtin_amdgcn_readlane(__double2loint(x), 63);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(x), 63);
  return __hiloint2double(hi, lo);
}

// Order statistics by extraction: the k largest (MAX) or smallest values of the multiset
// held 8 per lane (pads = the opposite infinity), one per step, one occurrence removed per
// step; returns the last two extracted (e_k, e_{k-1}).  Used when the requested order
// statistics lie within 24 of either end (p95..p999 of 1 h @10 s buckets: 1..19 steps)
// instead of a 512-element bitonic sort; the values are the same order statistics.
template <bool MAX>
__device__ __forceinline__ void extract_k(double v[DPL], int k, double& ek, double& ek1) {
  const int lane = lane_id();
  const double gone = MAX ? -(double)INFINITY : (double)INFINITY;
  ek = ek1 = gone;
  for (int t = 0; t < k; t++) {
    double m = v[0];
#pragma unroll
    for (int j = 1; j < DPL; j++) m = MAX ? fmax(m, v[j]) : fmin(m, v[j]);
    const double w = wave_ext_f64<MAX>(m);
    const uint64_t holders = __ballot(m == w);
    const int first = __ffsll((long long)holders) - 1;
    if (lane == first) {
      bool done = false;
#pragma unroll
      for (int j = 0; j < DPL; j++) {
        if (!done && v[j] == w) { v[j] = gone; done = true; }
      }
    }
    ek1 = ek;
    ek = w;
  }
}

// LEGACY estimate from the extremes when the needed order statistics are within 24 of an
// end; false = use the sort
__device__ __forceinline__ bool select_extreme(int fn, int n, const double* buf, double& out) {
  if (fn == TSDB_AGG_MEDIAN || n < 2 || n > CH) return false;
  const int lane = lane_id();
  const double q = pct_quantile(fn) / 100.0;
  const double pos = q * (double)(n + 1);
  const int ip = (int)floor(pos);
  // ascending indices lo_i, hi_i (select_sorted / Percentile.estimate)
  int lo_i, hi_i;
  if (pos < 1) { lo_i = hi_i = 0; }
  else if (pos >= (double)n) { lo_i = hi_i = n - 1; }
  else { lo_i = ip - 1; hi_i = ip; }
  const int ktop = n - lo_i, kbot = hi_i + 1;
  if (min(ktop, kbot) > 24) return false;
  double v[DPL];
  double a, b;   // extracted values at lo_i / hi_i
  if (ktop <= kbot) {
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      const int e = lane * DPL + j;
      v[j] = e < n ? buf[e] : -(double)INFINITY;
    }
    double ek, ek1;
    extract_k<true>(v, ktop, ek, ek1);   // e_ktop is index lo_i, e_{ktop-1} index lo_i + 1
    a = ek;
    b = (hi_i == lo_i) ? ek : ek1;
  } else {
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      const int e = lane * DPL + j;
      v[j] = e < n ? buf[e] : (double)INFINITY;
    }
    double ek, ek1;
    extract_k<false>(v, kbot, ek, ek1);  // m_kbot is index hi_i, m_{kbot-1} index hi_i - 1
    b = ek;
    a = (hi_i == lo_i) ? ek : ek1;
  }
  if (lo_i == hi_i) { out = a; return true; }
  const double dif = pos - floor(pos);
  out = a + dif * (b - a);
  return true;
}

// value of a finished bucket holding n non-NaN values in buf (tot values incl. NaN)
__device__ __forceinline__ double bucket_value(const GridParams& p, double* buf, int n) {
  const int lane = lane_id();
  if (n == 0) return (double)NAN;
  if (n > PCT_CAP) {   // only the BIG pass gets here
    if (lane == 0) set_err(p.err, TSDB_E_NOT_IMPLEMENTED);
    return (double)NAN;
  }
  double sel;
  if (select_extreme(p.sel_fn, n, buf, sel)) return sel;
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

// Order statistics per (series, bucket).  BIG = false: every series, buckets of at most
// CH values (register sort), 4 waves per block; a series with a larger bucket is appended
// to p.redo_list and left to the BIG pass (one wave per listed series, LDS buffer of
// PCT_CAP values).  Uniform rows are decoded from registers with a one-chunk prefetch
// (load_raw / decode_raw, as k_grid); other row classes through decode_generic.
template <bool BIG>
__global__ __launch_bounds__(256) void k_pct(GridParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int CAP = BIG ? PCT_CAP : CH;
  const int lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  unsigned char* base = smem + (int64_t)wave * (VBUF + CAP * 8);
  WaveLds W;
  W.dpv = (double*)base;
  W.vbuf = base;
  W.mq = (uint32_t*)base;
  W.mv = (uint32_t*)(base + CH * 4);
  double* buf = (double*)(base + VBUF);
  const int K = (int)p.K;
  int64_t s = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave;
  if (BIG) {
    if (s >= (int64_t)*p.redo_n) return;
    s = p.redo_list[s];
  }
  if (s >= p.n_series) return;
  double* dense = p.pre_dense + s * K;
  uint8_t* pres = p.pre_pres + s * K;
  for (int k = lane; k < K; k += 64) pres[k] = 0;
  // rows of the series inside the scan range: [ra, rb) (rows are in base-time order)
  const int64_t r0 = p.series_row_ptr[s], r1 = p.series_row_ptr[s + 1];
  int64_t ra = r0;
  while (ra < r1 && (int64_t)p.rows[ra].base < p.ss) ra++;
  int64_t rb = ra;
  while (rb < r1 && (int64_t)p.rows[rb].base < p.se) rb++;
  int cur = -1;      // open bucket
  int cnt = 0;       // its non-NaN values (in buf)
  bool big = false;
  Raw rc = {}, rn = {};
  RowDesc d = {};
  if (ra < rb) {
    d = p.rows[ra];
    if (row_uniform(d)) load_raw(p, d, 0, rc);
  }
  for (int64_t r = ra; r < rb && !big; r++) {
    const bool has_next = r + 1 < rb;
    RowDesc nd = {};
    if (has_next) nd = p.rows[r + 1];
    if (d.flags & ROW_ERR) {
      if (lane == 0) set_err(p.err, TSDB_E_ILLEGAL_DATA);
      if (has_next && row_uniform(nd)) load_raw(p, nd, 0, rc);
      d = nd;
      continue;
    }
    const RowGeom g = row_geom(p, d.base);
    const bool uni = row_uniform(d);
    int64_t vcur = 0;
    for (int64_t c0 = 0; c0 < (int64_t)d.ndp && !big; c0 += CH) {
      // prefetch the next chunk (same row, or the first chunk of the next row)
      if (c0 + CH < (int64_t)d.ndp) {
        if (uni) load_raw(p, d, c0 + CH, rn);
      } else if (has_next && row_uniform(nd)) {
        load_raw(p, nd, 0, rn);
      }
      int slot[DPL];
      double val[DPL];
      if (uni) decode_raw(p, d, g, c0, rc, slot, val);
      else decode_generic(p, d, g, c0, W, vcur, slot, val);
      rc = rn;
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
        const int total = __shfl(incl, 63, 64);
        if (!BIG && cnt + total > CAP) {   // bucket too large for the register sort
          big = true;
          break;
        }
        int o = cnt + incl - mine;
#pragma unroll
        for (int j = 0; j < DPL; j++) {
          if (left[j] && slot[j] == mn) {
            if (!isnan(val[j])) {
              if (o < CAP) buf[o] = val[j];
              o++;
            }
            left[j] = false;
          }
        }
        cnt += total;
        WAVE_SYNC();
      }
    }
    d = nd;
  }
  if (big) {
    if (lane == 0) p.redo_list[atomicAdd(p.redo_n, 1)] = (int32_t)s;
    return;
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

hipError_t launch_pct(const GridParams& p, bool big, int64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (big) {
    const size_t lds = 2 * (size_t)(VBUF + PCT_CAP * 8);
    hipError_t e = hipFuncSetAttribute((const void*)k_pct<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pct<true>, dim3((unsigned)((n + 1) / 2)), dim3(128), lds, s, p);
  } else {
    const size_t lds = 4 * (size_t)(VBUF + CH * 8);
    hipLaunchKernelGGL(k_pct<false>, dim3((unsigned)((n + 3) / 4)), dim3(256), lds, s, p);
  }
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
