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
#include "ksel.h"

#include <cstdlib>

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

// ---- the wave-local radix select (k_pct's large buckets, keys from ksel.h,
//      k_raw_sel) ---------------------------------------------------------------------

constexpr int SELW = 4;
constexpr int RAW_SEL_B = 8;        // operand rows of 64 loaded together (k_raw_sel staging)
constexpr int RAW_SEL_LDS = 4096;   // keys per wave staged in LDS (4 x 32 KB a block)
struct SelWave {
  uint32_t hist[256];
  uint64_t cand[64];
  uint32_t n;
};

__device__ __forceinline__ int wave_sum_int(int v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// Key of rank r (0-based ascending) among keys[0..n); called by all 64 lanes of the wave.
__device__ uint64_t wave_radix_select(const uint64_t* keys, int64_t ks, int n, int r, SelWave& W) {
  const int lane = lane_id();
  // skip the leading digits every key shares (counters, clustered values): they would put
  // all n keys into one histogram bin, pass after pass
  uint64_t kand = ~0ULL, kor = 0;
  for (int j = lane; j < n; j += 64) {
    const uint64_t k = keys[j * ks];
    kand &= k;
    kor |= k;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    kand &= shfl_u64(kand, lane ^ d);
    kor |= shfl_u64(kor, lane ^ d);
  }
  const uint64_t diff = kand ^ kor;
  if (diff == 0) return kand;   // all keys equal
  const int top = (63 - __clzll((long long)diff)) & ~7;   // lowest bit of the first differing digit
  uint64_t mask = top == 56 ? 0 : ~((1ULL << (top + 8)) - 1ULL);
  uint64_t prefix = kand & mask;
  for (int shift = top; shift >= 0; shift -= 8) {
#pragma unroll
    for (int q = 0; q < 4; q++) W.hist[lane * 4 + q] = 0;
    WAVE_SYNC();
    for (int j = lane; j < n; j += 64) {
      const uint64_t k = keys[j * ks];
      if ((k & mask) == prefix) atomicAdd(&W.hist[(k >> shift) & 255], 1u);
    }
    WAVE_SYNC();
    uint32_t c[4], t = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) { c[q] = W.hist[lane * 4 + q]; t += c[q]; }
    const int incl = wave_incl_sum((int)t);
    int ex = incl - (int)t;
    const bool found = ex <= r && r < incl;
    int bin = 0, rr = 0, nc = 0;
    if (found) {
      int q = 0;
      for (; q < 3; q++) {
        if (r < ex + (int)c[q]) break;
        ex += (int)c[q];
      }
      bin = lane * 4 + q;
      rr = r - ex;
      nc = (int)c[q];
    }
    const int src = __ffsll((long long)__ballot(found)) - 1;
    bin = __shfl(bin, src, 64);
    rr = __shfl(rr, src, 64);
    nc = __shfl(nc, src, 64);
    prefix |= (uint64_t)bin << shift;
    mask |= 255ULL << shift;
    r = rr;
    WAVE_SYNC();
    if (shift == 0) break;
    if (nc <= 64) {
      if (lane == 0) W.n = 0;
      WAVE_SYNC();
      for (int j = lane; j < n; j += 64) {
        const uint64_t k = keys[j * ks];
        if ((k & mask) == prefix) W.cand[atomicAdd(&W.n, 1u)] = k;
      }
      WAVE_SYNC();
      const uint64_t x = lane < nc ? W.cand[lane] : ~0ULL;
      int less = 0, eq = 0;
      for (int q = 0; q < nc; q++) {
        const uint64_t y = W.cand[q];
        less += y < x;
        eq += y == x;
      }
      const bool hit = lane < nc && less <= r && r < less + eq;
      const uint64_t res = shfl_u64(x, __ffsll((long long)__ballot(hit)) - 1);
      WAVE_SYNC();
      return res;
    }
  }
  return prefix;
}


// Ranks select_sorted reads for n sorted values (r1 = -1: one value); Median.runDouble
// sorted[n / 2], PercentileAgg.runDouble commons-math3 LEGACY pos = p (n + 1).
__device__ __forceinline__ void sel_ranks(int fn, int64_t n, int64_t& r0, int64_t& r1) {
  r0 = 0;
  r1 = -1;
  if (fn == TSDB_AGG_MEDIAN) { r0 = n / 2; return; }
  if (n <= 1) return;
  const double q = pct_quantile(fn) / 100.0;
  const double pos = (q == 0.0) ? 0.0 : (q == 1.0 ? (double)n : q * (double)(n + 1));
  if (pos < 1) r0 = 0;
  else if (pos >= (double)n) r0 = n - 1;
  else { r0 = (int64_t)floor(pos) - 1; r1 = r0 + 1; }
}

// Order statistic of n > PCT_CAP values: buf[0 .. PCT_CAP) in LDS, the rest at gbuf[PCT_CAP ..)
// (the wave's region of the global overflow buffer).  The values become order-preserving
// keys in gbuf[0 .. n) and the one or two ranks select_sorted reads are radix-selected --
// no sort and no size limit (the reference collects any number of values, Aggregators.java:657-708).
__device__ double bucket_value_big(const GridParams& p, const double* buf, int64_t n, double* gbuf, SelWave& SW) {
  const int lane = lane_id();
  uint64_t* keys = reinterpret_cast<uint64_t*>(gbuf);
  for (int e = lane; e < PCT_CAP; e += 64) keys[e] = f2key(buf[e]);
  for (int64_t e = PCT_CAP + lane; e < n; e += 64) keys[e] = f2key(gbuf[e]);
  __threadfence_block();
  WAVE_SYNC();
  int64_t r0, r1;
  sel_ranks(p.sel_fn, n, r0, r1);
  const uint64_t k0 = wave_radix_select(keys, 1, (int)n, (int)r0, SW);
  uint64_t k1 = k0;
  if (r1 >= 0) {
    // rank r0 + 1: the same key when more than r0 + 1 keys are <= k0, else the next larger key
    int le = 0;
    uint64_t gt = ~0ULL;
    for (int64_t j = lane; j < n; j += 64) {
      const uint64_t kk = keys[j];
      if (kk <= k0) le++;
      else gt = kk < gt ? kk : gt;
    }
    le = wave_sum_int(le);
    gt = wave_min_u64(gt);
    k1 = le > r1 ? k0 : gt;
  }
  const double v0 = key2f(k0), v1 = key2f(k1);
  WAVE_SYNC();
  return select_sorted(p.sel_fn, (int)n, [&](int i) { return (int64_t)i == r0 ? v0 : v1; });
}

// value of a finished bucket holding n non-NaN values in buf (and gbuf beyond PCT_CAP)
__device__ __forceinline__ double bucket_value(const GridParams& p, double* buf, int64_t n, double* gbuf, SelWave* SW) {
  const int lane = lane_id();
  if (n == 0) return (double)NAN;
  if (n > PCT_CAP) return bucket_value_big(p, buf, n, gbuf, *SW);   // only the BIG pass gets here
  double sel;
  if (select_extreme(p.sel_fn, (int)n, buf, sel)) return sel;
  if (n <= CH) {
    double v[DPL];
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      const int e = lane * DPL + j;
      v[j] = e < n ? buf[e] : (double)INFINITY;
    }
    sort512(v);
    return select_sorted(p.sel_fn, (int)n, [&](int i) { return reg_at(v, i); });
  }
  int N = CH;
  while (N < n) N <<= 1;
  for (int e = (int)n + lane; e < N; e += 64) buf[e] = (double)INFINITY;
  WAVE_SYNC();
  sort_lds(buf, N);
  return select_sorted(p.sel_fn, (int)n, [&](int i) { return buf[i]; });
}

// Order statistics per (series, bucket) of series s.  BIG = false: buckets of at most CH
// values (register sort); false = the series has a larger bucket (left to the BIG pass).
// BIG = true: buckets up to PCT_CAP values sorted in the LDS buffer, larger ones spill to the
// wave's global region gbuf (p.big_cap values) and are radix-selected.  Uniform rows are
// decoded from registers with a one-chunk prefetch (load_raw / decode_raw, as k_grid);
// other row classes through decode_generic.
template <bool BIG>
__device__ bool pct_series(const GridParams& p, int64_t s, const WaveLds& W, double* buf, double* gbuf, SelWave* SW) {
  constexpr int CAP = BIG ? PCT_CAP : CH;
  const int lane = lane_id();
  const int K = (int)p.K;
  double* dense = p.pre_dense + s * K;
  uint8_t* pres = p.pre_pres + s * K;
  for (int k = lane; k < K; k += 64) pres[k] = 0;
  // rows of the series inside the scan range: [ra, rb) (rows are in base-time order)
  const int64_t r0 = p.series_row_ptr[s], r1 = p.series_row_ptr[s + 1];
  int64_t ra = r0;
  while (ra < r1 && (int64_t)p.rows[ra].base < p.ss) ra++;
  int64_t rb = ra;
  while (rb < r1 && (int64_t)p.rows[rb].base < p.se) rb++;
  int cur = -1;        // open bucket
  int64_t cnt = 0;     // its non-NaN values (in buf / gbuf)
  StreamOrd so{-1};    // stored order (kcommon.h so_apply)
  Raw rc = {}, rn = {};
  RowDesc d = {};
  if (ra < rb) {
    d = p.rows[ra];
    if (row_uniform(d)) load_raw(p, d, 0, rc);
  }
  for (int64_t r = ra; r < rb; r++) {
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
    const bool skip = so_row_skip(p, so, d, !has_next);
    int64_t vcur = 0;
    for (int64_t c0 = 0; c0 < (int64_t)d.ndp; c0 += CH) {
      // prefetch the next chunk (same row, or the first chunk of the next row)
      if (c0 + CH < (int64_t)d.ndp) {
        if (uni) load_raw(p, d, c0 + CH, rn);
      } else if (has_next && row_uniform(nd)) {
        load_raw(p, nd, 0, rn);
      }
      int slot[DPL];
      double val[DPL];
      if (uni) decode_raw<true>(p, d, g, c0, rc, slot, val);
      else decode_generic<true>(p, d, g, c0, W, vcur, slot, val);
      so_apply(p, so, slot, skip);
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
            const double x = bucket_value(p, buf, cnt, gbuf, SW);
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
        if (!BIG && cnt + total > CAP) return false;   // bucket too large for the register sort
        int64_t o = cnt + incl - mine;
#pragma unroll
        for (int j = 0; j < DPL; j++) {
          if (left[j] && slot[j] == mn) {
            if (!isnan(val[j])) {
              if (o < CAP) buf[o] = val[j];
              else if (BIG && o < p.big_cap) gbuf[o] = val[j];
              o++;
            }
            left[j] = false;
          }
        }
        cnt += total;
        if (BIG && cnt > p.big_cap && lane == 0) set_err(p.err, TSDB_E_HIP);   // host sizing bug; never silent
        WAVE_SYNC();
      }
    }
    d = nd;
  }
  if (cur >= 0) {
    const double x = bucket_value(p, buf, cnt, gbuf, SW);
    if (lane == 0) { dense[cur] = x; pres[cur] = 1; }
  }
  return true;
}

// BIG = false: one wave per series (LIST: the series k_pct_rows handed back), 4 waves a
// block; a series with a bucket of more than CH values goes to p.redo_list.  BIG = true:
// p.n_launch waves loop over p.redo_list, each with a region of p.big_cap values of
// p.big_scratch for buckets above PCT_CAP.
template <bool BIG, bool LIST>
__global__ __launch_bounds__(256) void k_pct(GridParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ SelWave SWs[BIG ? 2 : 1];
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
  const int64_t gw = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave;
  if (BIG) {
    double* gbuf = p.big_scratch + gw * p.big_cap;
    const int64_t n = *p.redo_n;
    for (int64_t i = gw; i < n; i += p.n_launch) pct_series<true>(p, p.redo_list[i], W, buf, gbuf, &SWs[wave]);
    return;
  }
  int64_t s = gw;
  if (LIST) {   // series k_pct_rows handed back
    if (s >= (int64_t)*p.tile_list_n) return;
    s = p.tile_list[s];
  }
  if (s >= p.n_series) return;
  if (!pct_series<false>(p, s, W, buf, nullptr, nullptr) && lane == 0) p.redo_list[atomicAdd(p.redo_n, 1)] = (int32_t)s;
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

// k_emit for K <= 64 without rate: lane k owns slot k (emit_series_reg, as k_fast's register
// partials), the tile's series are checked for scan-range rows one a lane up front, and the
// next series' buckets are loaded while the current one is folded -- k_emit walks each series'
// rows for that check and stages the partials in LDS (0.62 ms over a 1M-series rollup table).
// GA: the group aggregator the instantiation is specialised for (< 0: p.ga at run time) -- the
// per-series work is a few dozen instructions, and the aggregator switch was a good part of them.
// The ring loads unconditionally (the index clamped to the last active series): with conditional
// loads the compiler waited for every outstanding load at each series (vmcnt(0)).
template <int GA>
__global__ __launch_bounds__(256) void k_emit_reg(GridParams p) {
  const int lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t tile = (int64_t)blockIdx.x * p.waves + wave;
  if (tile >= p.n_tiles) return;
  const int K = (int)p.K;
  const int ga = GA < 0 ? p.ga : GA;
  const int64_t s0 = p.tile_begin[tile], s1 = p.tile_end[tile];
  bool mine = false;   // lane i: series s0 + i has a row in the scan range (tiles hold <= 64 series)
  if (s0 + lane < s1) {
    const int64_t s = s0 + lane;
    for (int64_t r = p.series_row_ptr[s]; r < p.series_row_ptr[s + 1]; r++) {
      const uint32_t base = p.rows[r].base;
      if ((int64_t)base >= p.ss && (int64_t)base < p.se) { mine = true; break; }
    }
  }
  const uint64_t act = __ballot(mine);
  if (act && lane == 0) atomicOr(&p.group_active[p.tile_group[tile]], 1u);
  RegPart RP;
  rp_init(ga, RP);
  if (!act) {
    rp_store(p, tile, K, RP);
    return;
  }
  const bool inK = lane < K;
  const int64_t kl = inK ? lane : 0;   // (lanes past K read slot 0: in bounds, ignored)
  const int nact = __popcll(act);
  const int last = 63 - __clzll((long long)act);
  uint64_t rem = act;
  auto next = [&]() {   // the next active series of the tile (the last one again once none is left)
    const int i = rem ? __ffsll((long long)rem) - 1 : last;
    rem &= rem - 1;
    return s0 + i;
  };
  constexpr int EMIT_D = 16;
  uint8_t pr[EMIT_D];
  double v[EMIT_D];
#pragma unroll
  for (int d = 0; d < EMIT_D; d++) {
    const int64_t s = next();
    pr[d] = p.pre_pres[s * K + kl];
    v[d] = p.pre_dense[s * K + kl];
  }
  for (int j = 0; j < nact; j += EMIT_D) {
#pragma unroll
    for (int d = 0; d < EMIT_D; d++) {
      if (j + d < nact) emit_series_reg(p, K, inK && pr[d] != 0, v[d], RP, ga);
      const int64_t s = next();
      pr[d] = p.pre_pres[s * K + kl];
      v[d] = p.pre_dense[s * K + kl];
    }
  }
  rp_store(p, tile, K, RP);
}

// slot_contribution for a half wave (K <= 32): lanes 32h .. 32h + 31 are slots 0 .. 31 of one
// series; presence, neighbours and shuffles stay inside the half
__device__ __forceinline__ bool slot_contribution_half(const GridParams& p, int K, bool pr_in, bool valid, double v,
                                                       double& cv, bool& uni) {
  const int lane = lane_id(), h = lane >> 5, sl = lane & 31;
  const bool inK = valid && sl < K;
  const bool pr = inK && pr_in;
  uni = false;
  if (p.fill != TSDB_FILL_NONE && p.mode != MODE_ALL) {
    const double fillv = (p.fill == TSDB_FILL_ZERO) ? 0.0 : (double)NAN;
    if (!inK) return false;
    if (!pr && p.fill == TSDB_FILL_SCALAR) set_err(p.err, TSDB_E_RUNTIME);
    if (sl == 0 && p.skip0) return false;
    cv = pr ? v : fillv;
    uni = true;
    return true;
  }
  const uint32_t pm = (uint32_t)(__ballot(pr) >> (32 * h));
  if (pm == (K >= 32 ? 0xFFFFFFFFu : ((1u << K) - 1))) {   // every slot present: no interpolation
    cv = v;
    uni = inK;
    return inK;
  }
  const uint32_t below = pm & ((1u << sl) - 1);
  const uint32_t above = sl == 31 ? 0u : (pm & ~((2u << sl) - 1));
  const int prv = below ? 31 - __clz((int)below) : -1;
  const int nxt = above ? __ffs((int)above) - 1 : 32;
  const bool need = inK && !pr && prv >= 0 && nxt < K;
  double y0 = 0.0, y1 = 0.0;
  if (__ballot(need)) {
    y0 = __shfl(v, 32 * h + max(prv, 0), 64);
    y1 = __shfl(v, 32 * h + min(nxt, 31), 64);
  }
  if (pr) {
    cv = v;
    uni = true;
    return true;
  }
  if (need) {
    cv = interp(p.interp, p, prv, y0, nxt, y1, sl);
    return true;
  }
  return false;
}

// k_emit_reg for K <= 32: two series a step, the lower half wave the earlier one -- both halves
// find their contributions (presence ballots, LERP neighbours) at once, and the lower half's
// lanes fold the two into the slot's partial in series order, so the partial is the one-series-
// a-step kernel's bit for bit.  Half the serial steps a tile, and every load instruction feeds
// 2K lanes instead of K.
template <int GA>
__global__ __launch_bounds__(256) void k_emit_reg2(GridParams p) {
  const int lane = lane_id(), h = lane >> 5, sl = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t tile = (int64_t)blockIdx.x * p.waves + wave;
  if (tile >= p.n_tiles) return;
  const int K = (int)p.K;
  const int ga = GA < 0 ? p.ga : GA;
  const int64_t s0 = p.tile_begin[tile], s1 = p.tile_end[tile];
  bool mine = false;   // lane i: series s0 + i has a row in the scan range (tiles hold <= 64 series)
  if (s0 + lane < s1) {
    const int64_t s = s0 + lane;
    for (int64_t r = p.series_row_ptr[s]; r < p.series_row_ptr[s + 1]; r++) {
      const uint32_t base = p.rows[r].base;
      if ((int64_t)base >= p.ss && (int64_t)base < p.se) { mine = true; break; }
    }
  }
  const uint64_t act = __ballot(mine);
  if (act && lane == 0) atomicOr(&p.group_active[p.tile_group[tile]], 1u);
  RegPart RP;
  rp_init(ga, RP);
  if (!act) {
    rp_store(p, tile, K, RP);
    return;
  }
  const int64_t kl = sl < K ? sl : 0;   // (lanes past K read slot 0: in bounds, ignored)
  const int nact = __popcll(act);
  const int npair = (nact + 1) >> 1;
  const int last = 63 - __clzll((long long)act);
  uint64_t rem = act;
  auto next = [&]() {   // this half's series of the next pair (the last one again once none is left)
    const int a = rem ? __ffsll((long long)rem) - 1 : last;
    rem &= rem - 1;
    const int b = rem ? __ffsll((long long)rem) - 1 : last;
    rem &= rem - 1;
    return s0 + (h ? b : a);
  };
  constexpr int EMIT_D = 8;
  uint8_t pr[EMIT_D];
  double v[EMIT_D];
#pragma unroll
  for (int d = 0; d < EMIT_D; d++) {
    const int64_t s = next();
    pr[d] = p.pre_pres[s * K + kl];
    v[d] = p.pre_dense[s * K + kl];
  }
  for (int j = 0; j < npair; j += EMIT_D) {
#pragma unroll
    for (int d = 0; d < EMIT_D; d++) {
      if (j + d < npair) {
        const bool valid = 2 * (j + d) + h < nact;
        double cv = 0.0;
        bool uni = false;
        const bool c = slot_contribution_half(p, K, pr[d] != 0, valid, v[d], cv, uni);
        const double cv1 = __shfl(cv, sl + 32, 64);
        const int cu1 = __shfl((c ? 1 : 0) | (uni ? 2 : 0), sl + 32, 64);
        if (h == 0) {
          if (c) contribute_slot(ga, RP, cv, uni);
          if (cu1 & 1) contribute_slot(ga, RP, cv1, (cu1 & 2) != 0);
        }
      }
      const int64_t s = next();
      pr[d] = p.pre_pres[s * K + kl];
      v[d] = p.pre_dense[s * K + kl];
    }
  }
  rp_store(p, tile, K, RP);
}

// k_emit for K > 64 without rate (a day of 1m buckets: K = 1440): one wave per (tile, window of
// 64 slots), lane = slot, the window's tile partials in registers -- k_emit keeps K slots of
// partials in LDS (35 KB a wave at K = 1440: one wave a block, four a CU).  The contributions of
// a slot still arrive in series order.  A missing slot interpolates between the nearest present
// buckets of its series as emit_series_to does (both must exist); when one lies outside the
// window the wave finds it by scanning the series' presence bytes 64 at a time.
__device__ __forceinline__ int pres_prev(const uint8_t* pres, int k) {   // last present slot < k, -1 if none
  for (int b = k - 64; b > -64; b -= 64) {
    const int j = b + lane_id();
    const uint64_t m = __ballot(j >= 0 && j < k && pres[j] != 0);
    if (m) return b + 63 - __clzll((long long)m);
  }
  return -1;
}
__device__ __forceinline__ int pres_next(const uint8_t* pres, int k, int K) {   // first present slot >= k, K if none
  for (int b = k; b < K; b += 64) {
    const int j = b + lane_id();
    const uint64_t m = __ballot(j < K && pres[j] != 0);
    if (m) return b + __ffsll((long long)m) - 1;
  }
  return K;
}

__global__ __launch_bounds__(256) void k_emit_win(GridParams p, int nwin) {
  const int lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t gw = (int64_t)blockIdx.x * 4 + wave;
  const int64_t tile = gw / nwin;
  if (tile >= p.n_tiles) return;
  const int K = (int)p.K;
  const int w0 = (int)(gw % nwin) * 64;
  const int k = w0 + lane;
  const bool inK = k < K;
  const int64_t s0 = p.tile_begin[tile], s1 = p.tile_end[tile];
  bool mine = false;   // lane i: series s0 + i has a row in the scan range (tiles hold <= 64 series)
  if (s0 + lane < s1) {
    const int64_t s = s0 + lane;
    for (int64_t r = p.series_row_ptr[s]; r < p.series_row_ptr[s + 1]; r++) {
      const uint32_t base = p.rows[r].base;
      if ((int64_t)base >= p.ss && (int64_t)base < p.se) { mine = true; break; }
    }
  }
  const uint64_t act = __ballot(mine);
  if (act && w0 == 0 && lane == 0) atomicOr(&p.group_active[p.tile_group[tile]], 1u);
  RegPart RP;
  rp_init(p.ga, RP);
  const bool fill = p.fill != TSDB_FILL_NONE && p.mode != MODE_ALL;
  const double fillv = (p.fill == TSDB_FILL_ZERO) ? 0.0 : (double)NAN;
  const uint64_t win_mask = K - w0 >= 64 ? ~0ull : ((1ull << (K - w0)) - 1);
  for (int64_t s = s0; s < s1; s++) {
    if (!((act >> (s - s0)) & 1)) continue;
    const uint8_t* pres = p.pre_pres + s * K;
    const double* dense = p.pre_dense + s * K;
    const bool pr = inK && pres[k] != 0;
    const double v = inK ? dense[k] : 0.0;
    if (fill) {   // FillingDownsampler: every slot, missing -> NaN / 0 / RuntimeException
      if (inK) {
        if (!pr && p.fill == TSDB_FILL_SCALAR) set_err(p.err, TSDB_E_RUNTIME);
        if (!(k == 0 && p.skip0)) contribute_slot(p.ga, RP, pr ? v : fillv, true);
      }
      continue;
    }
    const uint64_t pm = __ballot(pr);
    if (pm == win_mask) {   // every slot of the window present: no interpolation
      if (inK) contribute_slot(p.ga, RP, v, true);
      continue;
    }
    // nearest present slots in the window, else outside it (scanned only when a lane needs them)
    const uint64_t below = pm & ((1ull << lane) - 1);
    const uint64_t above = lane == 63 ? 0ull : (pm & ~((2ull << lane) - 1));
    int prv = below ? w0 + 63 - __clzll((long long)below) : -2;
    int nxt = above ? w0 + __ffsll((long long)above) - 1 : -2;
    const bool miss = inK && !pr;
    if (__ballot(miss && prv == -2)) { const int q = pres_prev(pres, w0); if (prv == -2) prv = q; }
    if (__ballot(miss && nxt == -2)) { const int q = pres_next(pres, w0 + 64, K); if (nxt == -2) nxt = q; }
    const bool need = miss && prv >= 0 && nxt >= 0 && nxt < K;
    double y0 = 0.0, y1 = 0.0;
    if (need) {
      y0 = dense[prv];
      y1 = dense[nxt];
    }
    if (pr) contribute_slot(p.ga, RP, v, true);
    else if (need) contribute_slot(p.ga, RP, interp(p.interp, p, prv, y0, nxt, y1, k), false);
  }
  if (inK) {
    const int64_t o = tile * K + k;
    p.part.a[o] = RP.pa;
    p.part.b[o] = RP.pb;
    p.part.n[o] = RP.pn;
    p.part.f[o] = RP.pf;
  }
}

// ---- k_pct_rows: buckets inside rows, order statistics near the ends ------------------
//
// When the interval divides one hour (and slot 0 is interval-aligned, as the Downsampler's
// seek makes it) no bucket spans two rows, so every row is independent work: a wave takes a
// series, loads all its row descriptors at once (lane i: row i of a 64-row window) and runs
// a two-deep load ring over the rows with no walker.  Each bucket's order statistics come
// from extraction over the decoded registers (select_extreme's arithmetic, values removed
// through a per-lane keep mask), so the per-wave state is ~60 VGPRs and the kernel keeps
// far more waves in flight than k_pct.  A series that breaks a premise -- a row of another
// class, > CH datapoints, unsorted or malformed, an offset >= 1 h, a repeated base time, or a
// bucket whose statistic lies more than EXT_MAX from both ends -- is appended to
// p.redo_list for k_pct (which recomputes it whole).

static constexpr int EXT_MAX = 24;
#ifndef PCT_KEYS_OCC
#define PCT_KEYS_OCC 1   // min waves / SIMD the key kernel is compiled for (8: 18.7 ms with spills vs 18.1 at 7)
#endif
#ifndef PCT_VKEYS_OCC
#define PCT_VKEYS_OCC 7  // the values-only key kernel (8 spills 3-10 VGPRs)
#endif

// DPP int min across the wave (uniform result)
__device__ __forceinline__ int wave_min_dpp(int x) {
  x = min(x, __builtin_amdgcn_update_dpp(INT32_MAX, x, 0x111, 0xF, 0xF, false));
  x = min(x, __builtin_amdgcn_update_dpp(INT32_MAX, x, 0x112, 0xF, 0xF, false));
  x = min(x, __builtin_amdgcn_update_dpp(INT32_MAX, x, 0x114, 0xF, 0xF, false));
  x = min(x, __builtin_amdgcn_update_dpp(INT32_MAX, x, 0x118, 0xF, 0xF, false));
  x = min(x, __builtin_amdgcn_update_dpp(INT32_MAX, x, 0x142, 0xA, 0xF, false));
  x = min(x, __builtin_amdgcn_update_dpp(INT32_MAX, x, 0x143, 0xC, 0xF, false));
  return __builtin_amdgcn_readlane(x, 63);
}

// k-th largest (MAX) / smallest value of the multiset {val[j] : keep bit j}, and the
// (k-1)-th; one occurrence removed per step (ties kept as a multiset)
template <bool MAX>
__device__ __forceinline__ void extract_masked(const double val[DPL], uint32_t keep, int k, double& ek, double& ek1) {
  const int lane = lane_id();
  const double gone = MAX ? -(double)INFINITY : (double)INFINITY;
  ek = ek1 = gone;
  for (int t = 0; t < k; t++) {
    double m = gone;
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      const double c = MAX ? fmax(m, val[j]) : fmin(m, val[j]);
      m = ((keep >> j) & 1) ? c : m;
    }
    const double w = wave_ext_f64<MAX>(m);
    const uint64_t holders = __ballot(keep != 0 && m == w);
    const int first = __ffsll((long long)holders) - 1;
    if (lane == first) {
      uint32_t hit = 0;
#pragma unroll
      for (int j = DPL - 1; j >= 0; j--) if (((keep >> j) & 1) && val[j] == w) hit = 1u << j;
      keep &= ~hit;
    }
    ek1 = ek;
    ek = w;
  }
}

struct RowLite {
  uint64_t qoff, voff;
  uint32_t base, ndp, flags;
};

__device__ __forceinline__ RowLite row_of_lane(const RowDesc& d, int l) {
  RowLite r;
  r.qoff = rl64(d.qoff, l);
  r.voff = rl64(d.voff, l);
  r.base = (uint32_t)__builtin_amdgcn_readlane((int)d.base, l);
  r.ndp = (uint32_t)__builtin_amdgcn_readlane((int)d.ndp, l);
  r.flags = (uint32_t)__builtin_amdgcn_readlane((int)d.flags, l);
  return r;
}

template <int QW, int VL>
struct RawT {
  uint4 q[QW / 2];
  uint4 v[VL <= 2 ? 1 : VL / 2];
};

template <int QW, int VL>
__device__ __forceinline__ void load_row(const GridParams& p, const RowLite& d, RawT<QW, VL>& rw) {
  const int64_t i0 = (int64_t)lane_id() * DPL;
  if (i0 >= (int64_t)d.ndp) return;
  const uint8_t* q = p.qual + d.qoff + i0 * QW;
  const uint8_t* v = p.val + d.voff + i0 * VL;
#pragma unroll
  for (int i = 0; i < QW / 2; i++) rw.q[i] = reinterpret_cast<const uint4*>(q)[i];
  if (VL == 1) {
    const uint2 t = *reinterpret_cast<const uint2*>(v);
    rw.v[0] = make_uint4(t.x, t.y, 0, 0);
  } else {
#pragma unroll
    for (int i = 0; i < (VL <= 2 ? 1 : VL / 2); i++) rw.v[i] = reinterpret_cast<const uint4*>(v)[i];
  }
}

// the lane's 8 datapoints: slot (-1 = none), value, and whether every offset is < 1 h.
// slot0 = the row base's slot (exact: base and slot 0 are multiples of I); a datapoint at
// offset off lies in slot0 + off / I (one bucket per row when I = 1 h).
template <int QW, int VL>
__device__ __forceinline__ bool decode_row(const GridParams& p, const RowLite& d, int slot0, bool one,
                                           const RawT<QW, VL>& rw, int slot[DPL], double val[DPL]) {
  const int i0 = lane_id() * DPL;
  const int nv = max(0, min(DPL, (int)d.ndp - i0));
  uint32_t off[DPL], fl[DPL];
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    if (QW == 2) {
      const uint32_t w = (&rw.q[0].x)[j >> 1];
      const uint32_t be = __builtin_bswap32(w);
      const uint32_t qq = (j & 1) ? (be & 0xFFFF) : (be >> 16);
      off[j] = (qq >> 4) * 1000u;
      fl[j] = qq & 0xF;
    } else {
      const uint32_t qq = __builtin_bswap32((&rw.q[0].x)[j]);
      off[j] = (qq & 0x0FFFFFC0u) >> 6;
      fl[j] = qq & 0xF;
    }
  }
  const uint32_t* vw = &rw.v[0].x;
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    if (VL == 4) {
      const uint32_t be = __builtin_bswap32(vw[j]);
      val[j] = (fl[j] & 8) ? (double)__uint_as_float(be) : (double)(int32_t)be;
    } else if (VL == 8) {
      const uint64_t a = ((uint64_t)__builtin_bswap32(vw[2 * j]) << 32) | __builtin_bswap32(vw[2 * j + 1]);
      val[j] = (fl[j] & 8) ? __longlong_as_double((long long)a) : (double)(long long)a;
    } else if (VL == 2) {
      const uint32_t be = __builtin_bswap32(vw[j >> 1]);
      const uint32_t x = (j & 1) ? (be & 0xFFFF) : (be >> 16);
      val[j] = (double)(int16_t)(uint16_t)x;
    } else {
      val[j] = (double)(int8_t)((vw[j >> 2] >> ((j & 3) * 8)) & 0xFF);
    }
  }
  bool ok = true;
  const uint32_t I32 = (uint32_t)p.I;
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    int sl = slot0;
    if (!one) {
      // off < 3.6e6 (exact in float): reciprocal estimate, corrected to the exact quotient
      uint32_t qq = (uint32_t)((float)off[j] * p.rcpI);
      int64_t r = (int64_t)off[j] - (int64_t)qq * I32;
      if (r < 0) { qq--; r += I32; }
      if (r >= (int64_t)I32) { qq++; r -= I32; }
      if (r >= (int64_t)I32) { qq++; }
      sl += (int)qq;
    }
    slot[j] = (j < nv && sl >= 0 && sl < (int)p.K) ? sl : -1;
    ok = ok && (j >= nv || off[j] < 3600000u);
  }
  return ok;
}

// order statistic of the bucket {val[j] : keep bit j} holding n non-NaN values (n >= 1)
// by extraction; false = more than EXT_MAX from both ends
__device__ __forceinline__ bool select_keep(const double val[DPL], uint32_t keep, int n, double q, double& x) {
  // select_sorted / select_extreme: LEGACY pos = p (n + 1)
  const double pos = q * (double)(n + 1);
  const int ip = (int)floor(pos);
  int lo_i, hi_i;
  if (pos < 1) { lo_i = hi_i = 0; }
  else if (pos >= (double)n) { lo_i = hi_i = n - 1; }
  else { lo_i = ip - 1; hi_i = ip; }
  const int ktop = n - lo_i, kbot = hi_i + 1;
  if (min(ktop, kbot) > EXT_MAX) return false;
  double a, b, ek, ek1;
  if (ktop <= kbot) {
    extract_masked<true>(val, keep, ktop, ek, ek1);
    a = ek;
    b = (hi_i == lo_i) ? ek : ek1;
  } else {
    extract_masked<false>(val, keep, kbot, ek, ek1);
    b = ek;
    a = (hi_i == lo_i) ? ek : ek1;
  }
  x = (lo_i == hi_i) ? a : a + (pos - floor(pos)) * (b - a);
  return true;
}

// ---- one-bucket rows of 4-byte values: order statistics over 32-bit keys ----------------
// A 1 h bucket in a row of 4-byte values that are all float32 (or all int32): the values map
// to order-preserving uint32 keys (NaN and absent datapoints -> 0, below every key), each lane
// sorts its 8 keys once, and the k-th largest is found by popping the wave maximum of the lane
// heads -- every lane holding the maximum pops it at once, so a round costs one DPP max and a
// shift of the popped lanes' lists.  The arithmetic is 32-bit until the two selected values are
// converted back (exact: float32 / int32 -> double), so the result equals select_keep's.
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false));
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

__device__ __forceinline__ void cas_desc(uint32_t& a, uint32_t& b) {
  const uint32_t hi = max(a, b), lo = min(a, b);
  a = hi;
  b = lo;
}

// 8 keys, descending (Batcher's odd-even merge network, 19 comparators)
__device__ __forceinline__ void sort8_desc(uint32_t k[DPL]) {
  cas_desc(k[0], k[1]); cas_desc(k[2], k[3]); cas_desc(k[4], k[5]); cas_desc(k[6], k[7]);
  cas_desc(k[0], k[2]); cas_desc(k[1], k[3]); cas_desc(k[4], k[6]); cas_desc(k[5], k[7]);
  cas_desc(k[1], k[2]); cas_desc(k[5], k[6]);
  cas_desc(k[0], k[4]); cas_desc(k[1], k[5]); cas_desc(k[2], k[6]); cas_desc(k[3], k[7]);
  cas_desc(k[2], k[4]); cas_desc(k[3], k[5]);
  cas_desc(k[1], k[2]); cas_desc(k[3], k[4]); cas_desc(k[5], k[6]);
}

// 6 keys, descending (the optimal 12-comparator network, depth 5)
__device__ __forceinline__ void sort6_desc(uint32_t k[6]) {
  cas_desc(k[0], k[5]); cas_desc(k[1], k[3]); cas_desc(k[2], k[4]);
  cas_desc(k[1], k[2]); cas_desc(k[3], k[4]);
  cas_desc(k[0], k[3]); cas_desc(k[2], k[5]);
  cas_desc(k[0], k[1]); cas_desc(k[2], k[3]); cas_desc(k[4], k[5]);
  cas_desc(k[1], k[2]); cas_desc(k[3], k[4]);
}

// N keys a lane (8, or 6 for rows of <= 384 values: 60 lanes of a 360-value hour row busy
// instead of 45)
template <int N>
__device__ __forceinline__ void sortN_desc(uint32_t k[N]) {
  static_assert(N == 8 || N == 6, "8 or 6 keys a lane");
  if constexpr (N == 8) sort8_desc(k);
  else sort6_desc(k);
}

// k-th and (k-1)-th largest key (k >= 1) of the wave's keys (0 = none); sorts k[] in place
template <int N = DPL>
__device__ __forceinline__ void topk_u32(uint32_t k[N], int kk, uint32_t& ek, uint32_t& ek1) {
  sortN_desc<N>(k);
  int cum = 0;
  ek = ek1 = 0;
  while (cum < kk) {
    const uint32_t w = wave_max_u32(k[0]);
    const bool pop = k[0] == w;
    const int c = __popcll(__ballot(pop));
    if (cum < kk - 1 && kk - 1 <= cum + c) ek1 = w;
    if (kk <= cum + c) ek = w;
    cum += c;
    if (pop) {
#pragma unroll
      for (int j = 0; j < N - 1; j++) k[j] = k[j + 1];
      k[N - 1] = 0;
    }
  }
}

// float32 bits / int32 -> order key (> 0); NaN -> 0
__device__ __forceinline__ uint32_t key32(uint32_t bits, bool isf) {
  if (!isf) return bits ^ 0x80000000u;
  if ((bits & 0x7FFFFFFFu) > 0x7F800000u) return 0u;   // NaN
  return (bits & 0x80000000u) ? ~bits : (bits | 0x80000000u);
}
__device__ __forceinline__ double unkey32(uint32_t k, bool isf) {
  if (!isf) return (double)(int32_t)(k ^ 0x80000000u);
  return (double)__uint_as_float((k & 0x80000000u) ? (k ^ 0x80000000u) : ~k);
}

// keys of the lane (sorted descending) below t: the keys >= t are a prefix, found by a
// branch-free binary search over the N keys.  (The keys are copied to values first: a
// conditional over two array elements is an lvalue in C++, so clang selects between their
// addresses, and the AMDGPU backend then moved the whole key array to LDS for the indexed load --
// one ds_write per key and a ds_read per search step, seen in the ISA.)
template <int N = DPL>
__device__ __forceinline__ int lane_below(const uint32_t key[N], uint32_t t) {
  if constexpr (N == 6) {
    const uint32_t k0 = key[0], k1 = key[1], k2 = key[2], k3 = key[3], k4 = key[4], k5 = key[5];
    const bool c3 = k2 >= t;
    const bool c2 = (c3 ? k4 : k0) >= t;
    const int ge = c3 ? (c2 ? 5 : 3) : (c2 ? 1 : 0);
    const uint32_t x = c3 ? (c2 ? k5 : k3) : (c2 ? k1 : k0);
    return N - (ge + ((c2 || c3) && x >= t ? 1 : 0));
  } else {
    const uint32_t k0 = key[0], k1 = key[1], k2 = key[2], k3 = key[3], k4 = key[4], k5 = key[5], k6 = key[6],
                   k7 = key[7];
    const bool c4 = k3 >= t;
    int ge = c4 ? 4 : 0;
    const bool c2 = (c4 ? k5 : k1) >= t;
    ge += c2 ? 2 : 0;
    const uint32_t x = c4 ? (c2 ? k6 : k4) : (c2 ? k2 : k0);
    ge += x >= t ? 1 : 0;
    if (k7 >= t) ge = 8;   // (the search above resolves 0..7)
    return N - ge;
  }
}

template <int N = DPL>
__device__ __forceinline__ uint32_t next_key32(const uint32_t key[N], uint32_t k0, int target);

// Keys of rank `target` and `target + 1` (0-based, ascending; k1 only when want1) among the
// wave's 512 keys (absent = 0, counted first; any order in a lane).  Mid-rank
// statistics (median, p50, p75) take it instead of popping ~n/2 wave maxima.
// Phase 1, a bitwise binary search over the key bits below the prefix every present key
// shares, narrows [ans, ans + 2^b) until it holds <= 64 keys (the counts below both ends come
// free with each step).  Phase 2 compacts those keys one per lane through the wave's LDS row and
// finishes the remaining bits with one compare + ballot each.  (The kernel is VALU-bound -- r03h
// PMC: VALU issue ~100 % of SIMD cycles -- and phase 2's bits cost 1 VALU instead of ~16.)
template <int N = DPL>
__device__ __forceinline__ void kth_pair32(const uint32_t key[N], int target, bool want1, uint32_t& k0,
                                           uint32_t& k1, int zeros) {
  __shared__ uint32_t cand_lds[4][64];
  uint32_t* cand_row = cand_lds[threadIdx.x >> 6];
  // the prefix every present key shares = the common prefix of the smallest and largest present
  // key (absent keys are 0: the max ignores them, the min of key - 1 wraps them to the top)
  uint32_t kmx = 0u, kmn1 = ~0u;
#pragma unroll
  for (int j = 0; j < N; j++) {
    kmx = max(kmx, key[j]);
    kmn1 = min(kmn1, key[j] - 1u);
  }
  // wave max / min by DPP (row shifts, then the row broadcasts; lane 63 ends with the whole wave)
  kmx = max(kmx, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)kmx, 0x111, 0xF, 0xF, false));
  kmn1 = min(kmn1, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)kmn1, 0x111, 0xF, 0xF, false));
  kmx = max(kmx, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)kmx, 0x112, 0xF, 0xF, false));
  kmn1 = min(kmn1, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)kmn1, 0x112, 0xF, 0xF, false));
  kmx = max(kmx, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)kmx, 0x114, 0xF, 0xF, false));
  kmn1 = min(kmn1, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)kmn1, 0x114, 0xF, 0xF, false));
  kmx = max(kmx, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)kmx, 0x118, 0xF, 0xF, false));
  kmn1 = min(kmn1, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)kmn1, 0x118, 0xF, 0xF, false));
  kmx = max(kmx, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)kmx, 0x142, 0xA, 0xF, false));
  kmn1 = min(kmn1, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)kmn1, 0x142, 0xA, 0xF, false));
  kmx = max(kmx, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)kmx, 0x143, 0xC, 0xF, false));
  kmn1 = min(kmn1, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)kmn1, 0x143, 0xC, 0xF, false));
  kmx = (uint32_t)__builtin_amdgcn_readlane((int)kmx, 63);
  const uint32_t kmn = (uint32_t)__builtin_amdgcn_readlane((int)kmn1, 63) + 1u;   // (n >= 1 present keys)
  const uint32_t diff = kmn ^ kmx;
  if (diff == 0) { k0 = k1 = kmn; return; }   // every present key equal
  int b = 32 - __clz((int)diff);   // width of the open interval [ans, ans + 2^b)
  uint32_t ans = b == 32 ? 0u : (kmn & ~((1u << b) - 1u));
  // count of keys below ans / below ans + 2^b (the absent keys, 0, below every present key)
  int lowc = zeros, highc = 64 * N;
  while (b > 0 && highc - lowc > 64) {
    b--;
    const uint32_t t = ans | (1u << b);
    // keys below t: one compare and one popcount a key slot (the scalar unit adds; a DPP sum
    // of per-lane counts cost ~15 more VALU instructions a step)
    int c = 0;
#pragma unroll
    for (int j = 0; j < N; j++) c += __popcll(__ballot(key[j] < t));
    if (c <= target) { ans = t; lowc = c; } else { highc = c; }
  }
  if (b == 0) {   // more than 64 keys equal ans
    k0 = ans;
    k1 = want1 ? next_key32<N>(key, ans, target) : ans;
    return;
  }
  const uint32_t span = b == 32 ? ~0u : (1u << b) - 1u;   // keys in the interval: key - ans <= span
  // present keys in [ans, ans + span] with one compare: key - lo <= hb, lo = max(ans, 1) keeps the
  // absent keys (0) out when ans is 0
  const uint32_t lo = ans ? ans : 1u, hb = span - (lo - ans);
  int m = 0;
#pragma unroll
  for (int j = 0; j < N; j++) m += (key[j] - lo <= hb) ? 1 : 0;
  int pos = wave_incl_sum_dpp(m) - m;
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < N; j++) {
    if (key[j] - lo <= hb) cand_row[pos++] = key[j];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int M = highc - lowc;
  const bool live = lane_id() < M;
  const uint32_t c = live ? cand_row[lane_id()] : ~0u;
  __builtin_amdgcn_wave_barrier();
  const int t2 = target - lowc;   // rank among the candidates
  // The candidates sorted across the wave (bitonic, one per lane; lanes past them hold ~0u and
  // sort last): ranks t2 and t2 + 1 are lanes t2 and t2 + 1.  21 compare-exchange steps of a
  // shuffle, a min and a max -- the bit-by-bit search it replaces cost one compare and ~8 scalar
  // instructions for each of the ~20 open key bits, and the kernel is bound by the scalar unit.
  const int lane = lane_id();
  uint32_t v = c;
  // (the flip form: each stage starts by comparing lane l with l ^ (k - 1), then half-cleaners
  // with l ^ j; the lower lane always keeps the minimum, so the lane predicate is one bit of the
  // lane id -- six wave-constant masks -- instead of two)
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const int x = j == (k >> 1) ? k - 1 : j;
      const uint32_t o = (uint32_t)__shfl_xor((int)v, x, 64);
      const bool keep_min = (lane & j) == 0;
      v = keep_min ? min(v, o) : max(v, o);
    }
  }
  (void)ans;
  k0 = (uint32_t)__builtin_amdgcn_readlane((int)v, t2);
  if (!want1) { k1 = k0; return; }
  if (t2 + 1 < M) { k1 = (uint32_t)__builtin_amdgcn_readlane((int)v, t2 + 1); return; }
  k1 = next_key32<N>(key, k0, target);   // rank target + 1 lies above the interval
}

// The key of rank target + 1 given k0 = the key of rank target.
template <int N>
__device__ __forceinline__ uint32_t next_key32(const uint32_t key[N], uint32_t k0, int target) {
  int le = 0;
  uint32_t gt = ~0u;
#pragma unroll
  for (int j = 0; j < N; j++) {
    le += __popcll(__ballot(key[j] <= k0));
    if (key[j] > k0) gt = min(gt, key[j]);
  }
  if (le > target + 1) return k0;
  return ~wave_max_u32(~gt);
}

// The statistic of one bucket from the wave's 32-bit keys (absent = 0), n present values (n >= 1),
// wf = the keys are float32 (else int32).  Near the ends the k largest / smallest keys are popped
// (topk_u32); mid ranks take the bitwise search.  0 = more than EXT_MAX from both ends (near-end
// variant): the caller hands the series back.
template <bool MID, int N = DPL>
__device__ __forceinline__ int keys_stat(const GridParams& p, uint32_t key[N], int n, bool wf, double q, double& x) {
  // select_sorted: PercentileAgg LEGACY pos = p (n + 1); Median.runDouble sorted[n / 2]
  const double pos = q * (double)(n + 1);
  int lo_i, hi_i;
  if (MID && p.sel_fn == TSDB_AGG_MEDIAN) { lo_i = hi_i = n / 2; }
  else {
    const int ip = (int)floor(pos);
    if (pos < 1) { lo_i = hi_i = 0; }
    else if (pos >= (double)n) { lo_i = hi_i = n - 1; }
    else { lo_i = ip - 1; hi_i = ip; }
  }
  const int ktop = n - lo_i, kbot = hi_i + 1;
  double a, b;
  uint32_t ek, ek1;
  if (min(ktop, kbot) > EXT_MAX) {
    if constexpr (!MID) return 0;   // (the near-end variant keeps its registers for the extraction)
    // (kth_pair32 needs no per-lane order: its counts, candidate list and next key compare every slot)
    const int zeros = 64 * N - n;
    uint32_t k0, k1;
    kth_pair32<N>(key, zeros + lo_i, hi_i != lo_i, k0, k1, zeros);
    a = unkey32(k0, wf);
    b = unkey32(k1, wf);
  } else if (ktop <= kbot) {
    topk_u32<N>(key, ktop, ek, ek1);
    a = unkey32(ek, wf);
    b = (hi_i == lo_i) ? a : unkey32(ek1, wf);
  } else {
#pragma unroll
    for (int j = 0; j < N; j++) key[j] = key[j] ? ~key[j] : 0u;   // ascending order as descending keys
    topk_u32<N>(key, kbot, ek, ek1);
    b = unkey32(~ek, wf);
    a = (hi_i == lo_i) ? b : unkey32(~ek1, wf);
  }
  x = (lo_i == hi_i) ? a : a + (pos - floor(pos)) * (b - a);
  return 1;
}

// The statistic of a one-bucket row of 4-byte values; 0 = not this path's case (mixed float /
// int row): the caller hands the series to k_pct.  Near the ends the k largest / smallest keys
// are popped (topk_u32); mid ranks take the bitwise search.
template <int QW, bool MID>
__device__ __forceinline__ int pct_row_keys(const GridParams& p, const RowLite& d, const RawT<QW, 4>& rw, double q,
                                            double& x) {
  const int i0 = lane_id() * DPL;
  const int nv = max(0, min(DPL, (int)d.ndp - i0));
  uint32_t key[DPL];
  bool ok = true, anyf = false, anyi = false;
  int n = 0;
  const uint32_t* vw = &rw.v[0].x;
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    uint32_t off, fl;
    if (QW == 2) {
      const uint32_t be = __builtin_bswap32((&rw.q[0].x)[j >> 1]);
      const uint32_t qq = (j & 1) ? (be & 0xFFFF) : (be >> 16);
      off = (qq >> 4) * 1000u;
      fl = qq & 0xF;
    } else {
      const uint32_t qq = __builtin_bswap32((&rw.q[0].x)[j]);
      off = (qq & 0x0FFFFFC0u) >> 6;
      fl = qq & 0xF;
    }
    const bool v = j < nv;
    const bool isf = (fl & 8) != 0;
    ok = ok && (!v || off < 3600000u);
    anyf = anyf || (v && isf);
    anyi = anyi || (v && !isf);
    const uint32_t bits = __builtin_bswap32(vw[j]);
    key[j] = v ? key32(bits, isf) : 0u;
    n += key[j] != 0;
    ok = ok && !(v && !isf && bits == 0x80000000u);   // int32 MIN keys to 0 (= absent): not this path's
  }
  if (__ballot(!ok)) return -1;   // offset >= 1 h (or an int32 MIN value): hand the series back
  const bool wf = __ballot(anyf) != 0, wi = __ballot(anyi) != 0;
  if (wf && wi) return 0;   // mixed row
  n = __builtin_amdgcn_readlane(wave_incl_sum_dpp(n), 63);
  if (n == 0) {
    x = (double)NAN;
    return 1;
  }
  return keys_stat<MID>(p, key, n, wf, q, x);
}

// ---- values-only key rows (KEYS & 4) ----------------------------------------------------
// When every row of the batch's key class was certified at load (k_index flags) as all-float32
// without NaN or all-int32 -- sorted, 4-byte values -- a 1 h bucket needs no qualifier but the
// row's last: offsets strictly increase, so the row lies inside its hour iff its last offset is
// < 1 h.  The kernel then reads 4 B a datapoint (+ one qualifier a row), forms each key with a
// byte swap and a sign flip, and n is the row's datapoint count (no NaN to drop).
struct RawV {
  uint4 v[2];
  uint32_t lq;   // the row's last qualifier, as loaded (little-endian load of big-endian bytes)
};

template <int QW>
__device__ __forceinline__ void load_row_v(const GridParams& p, const RowLite& d, RawV& rw) {
  const uint8_t* q = p.qual + (d.ndp ? d.qoff + (uint64_t)(d.ndp - 1) * QW : 0);
  rw.lq = QW == 2 ? (uint32_t)*reinterpret_cast<const uint16_t*>(q) : *reinterpret_cast<const uint32_t*>(q);
  const int64_t i0 = (int64_t)lane_id() * DPL;
  if (i0 >= (int64_t)d.ndp) return;
  const uint4* v = reinterpret_cast<const uint4*>(p.val + d.voff + i0 * 4);
  rw.v[0] = v[0];
  rw.v[1] = v[1];
}

// 6 values a lane (KEYS & 8): rows of <= 384 values, 24 B a lane
struct RawV6 {
  uint2 v[3];
  uint32_t lq;
};

template <int QW>
__device__ __forceinline__ void load_row_v6(const GridParams& p, const RowLite& d, RawV6& rw) {
  const uint8_t* q = p.qual + (d.ndp ? d.qoff + (uint64_t)(d.ndp - 1) * QW : 0);
  rw.lq = QW == 2 ? (uint32_t)*reinterpret_cast<const uint16_t*>(q) : *reinterpret_cast<const uint32_t*>(q);
  const int64_t i0 = (int64_t)lane_id() * 6;
  if (i0 >= (int64_t)d.ndp) return;
  const uint2* v = reinterpret_cast<const uint2*>(p.val + d.voff + i0 * 4);
  rw.v[0] = v[0];
  rw.v[1] = v[1];
  rw.v[2] = v[2];
}

template <int QW, bool MID, int N = DPL, class R>
__device__ __forceinline__ int pct_row_vkeys(const GridParams& p, const RowLite& d, const R& rw, double q,
                                             double& x) {
  const uint32_t lq = (uint32_t)__builtin_amdgcn_readfirstlane((int)rw.lq);
  const uint32_t off = QW == 2 ? (((((lq & 0xFFu) << 8) | ((lq >> 8) & 0xFFu)) >> 4) * 1000u)
                               : ((__builtin_bswap32(lq) & 0x0FFFFFC0u) >> 6);
  if (off >= 3600000u) return -1;   // the row reaches past its hour: hand the series back
  const bool isf = (d.flags & ROW_ALLF) != 0;
  const int n = (int)d.ndp;
  const int i0 = lane_id() * N;
  uint32_t key[N];
  const uint32_t* vw = &rw.v[0].x;
  if (isf) {
#pragma unroll
    for (int j = 0; j < N; j++) {
      const uint32_t b = __builtin_bswap32(vw[j]);
      key[j] = b ^ ((uint32_t)((int32_t)b >> 31) | 0x80000000u);   // key32 of a non-NaN float32
    }
  } else {
    bool mn = false;
#pragma unroll
    for (int j = 0; j < N; j++) {
      key[j] = __builtin_bswap32(vw[j]) ^ 0x80000000u;
      mn = mn || (i0 + j < n && key[j] == 0u);
    }
    if (__ballot(mn)) return -1;   // an int32 MIN value keys to 0 (= absent)
  }
  if (i0 + N > n) {
#pragma unroll
    for (int j = 0; j < N; j++) key[j] = i0 + j < n ? key[j] : 0u;
  }
  return keys_stat<MID, N>(p, key, n, isf, q, x);
}

// one in-range row: its buckets' order statistics into dense / pres; false = hand the
// series back (offset >= 1 h, or a statistic more than EXT_MAX from both ends)
template <int QW, int VL, int KEYS, class R>
__device__ __forceinline__ bool pct_row(const GridParams& p, const RowLite& cd, const R& rc, double q,
                                        double* dense, uint8_t* pres) {
  const int lane = lane_id();
  RowLite d;
  d.base = (uint32_t)__builtin_amdgcn_readfirstlane((int)cd.base);
  d.ndp = (uint32_t)__builtin_amdgcn_readfirstlane((int)cd.ndp);
  d.flags = (uint32_t)__builtin_amdgcn_readfirstlane((int)cd.flags);
  // slot of the row base: (base * 1000 - B0) / I, an exact multiple (double division exact)
  const int64_t rel = (int64_t)d.base * 1000 - p.B0;
  const int slot0 = (int)__builtin_amdgcn_readfirstlane((int)((double)rel / (double)p.I));
  const bool one = p.I == 3600000;
  if (one && (slot0 < 0 || slot0 >= (int)p.K)) return true;   // the row's bucket is out of range
  if constexpr (KEYS) {
    // 1 h buckets of 4-byte values (host-checked): the key path alone, the rest to k_pct
    if constexpr (VL == 4) {
      if (d.ndp == 0) return true;
      double x;
      int r;
      if constexpr ((KEYS & 8) != 0) r = pct_row_vkeys<QW, (KEYS & 3) == 2, 6>(p, d, rc, q, x);
      else if constexpr ((KEYS & 4) != 0) r = pct_row_vkeys<QW, (KEYS & 3) == 2>(p, d, rc, q, x);
      else r = pct_row_keys<QW, (KEYS & 3) == 2>(p, d, rc, q, x);
      if (r <= 0) return false;
      if (lane == 0) { dense[slot0] = x; pres[slot0] = 1; }
      return true;
    } else {
      return false;
    }
  } else {
  static_assert(std::is_same<R, RawT<QW, VL>>::value, "extraction rows are raw qualifier + value registers");
  int slot[DPL];
  double val[DPL];
  const bool ok = decode_row<QW, VL>(p, d, slot0, one, rc, slot, val);
  if (__ballot(!ok)) return false;
  if (one) {
    uint32_t keep = 0;
    bool any = false;
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      any = any || slot[j] >= 0;
      keep |= (slot[j] >= 0 && !isnan(val[j]) ? 1u : 0u) << j;
    }
    if (!__ballot(any)) return true;
    const int n = __builtin_amdgcn_readlane(wave_incl_sum_dpp(__popc(keep)), 63);
    double x = (double)NAN;
    if (n > 0 && (q < 0 || !select_keep(val, keep, n, q, x))) return false;
    if (lane == 0) { dense[slot0] = x; pres[slot0] = 1; }
    return true;
  }
  uint32_t left = 0;
#pragma unroll
  for (int j = 0; j < DPL; j++) left |= (slot[j] >= 0 ? 1u : 0u) << j;
  for (;;) {
    int mn = INT32_MAX;
#pragma unroll
    for (int j = 0; j < DPL; j++) if ((left >> j) & 1) mn = min(mn, slot[j]);
    mn = wave_min_dpp(mn);
    if (mn == INT32_MAX) break;
    uint32_t keep = 0;
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      if (((left >> j) & 1) && slot[j] == mn) {
        left &= ~(1u << j);
        if (!isnan(val[j])) keep |= 1u << j;
      }
    }
    const int n = __builtin_amdgcn_readlane(wave_incl_sum_dpp(__popc(keep)), 63);
    double x = (double)NAN;
    if (n > 0 && (q < 0 || !select_keep(val, keep, n, q, x))) return false;
    if (lane == 0) { dense[mn] = x; pres[mn] = 1; }
  }
  return true;
  }
}

// KEYS: 0 = extraction over doubles; 1 = the 32-bit key kernel, statistics near the ends;
// 2 = the key kernel ranking any statistic (median, p50, p75: the bitwise rank search);
// | 4 = the key kernel over load-certified rows, values read alone (RawV); | 8 as well, 6 values a
// lane (RawV6, rows of <= 384 values)
template <int QW, int VL, int KEYS>
__device__ __forceinline__ void load_ring_row(const GridParams& p, const RowLite& d, RawT<QW, VL>& rw) {
  load_row<QW, VL>(p, d, rw);
}
template <int QW, int VL, int KEYS>
__device__ __forceinline__ void load_ring_row(const GridParams& p, const RowLite& d, RawV& rw) {
  load_row_v<QW>(p, d, rw);
}
template <int QW, int VL, int KEYS>
__device__ __forceinline__ void load_ring_row(const GridParams& p, const RowLite& d, RawV6& rw) {
  load_row_v6<QW>(p, d, rw);
}

template <int QW, int VL, int D, int KEYS>
__global__ __launch_bounds__(256, (KEYS & 4) ? PCT_VKEYS_OCC : KEYS ? PCT_KEYS_OCC : 1) void k_pct_rows(GridParams p) {
  const int lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t s = (int64_t)blockIdx.x * 4 + wave;
  if (s >= p.n_series) return;
  const int K = (int)p.K;
  double* dense = p.pre_dense + s * K;
  uint8_t* pres = p.pre_pres + s * K;
  for (int k = lane; k < K; k += 64) pres[k] = 0;
  // (median: no quantile; the extraction path hands such series back, the key path ranks them)
  const double q = p.sel_fn == TSDB_AGG_MEDIAN ? -1.0 : pct_quantile(p.sel_fn) / 100.0;
  const int64_t r0 = p.series_row_ptr[s], r1 = p.series_row_ptr[s + 1];
  int64_t last_base = -1;   // base of the previous in-range row (repeated bases: redo)
  for (int64_t w0 = r0; w0 < r1; w0 += 64) {
    const int nr = (int)min((int64_t)64, r1 - w0);
    RowDesc d = {};   // only qoff / voff / base / ndp / flags are read
    bool in = false, bad = false;
    if (lane < nr) {
      const RowDesc* src = p.rows + w0 + lane;
      d.qoff = src->qoff;
      d.voff = src->voff;
      d.base = src->base;
      d.ndp = src->ndp;
      d.flags = src->flags;
      in = (int64_t)d.base >= p.ss && (int64_t)d.base < p.se;
      const uint32_t f = d.flags;
      bad = in && ((f & (ROW_ERR | ROW_UNSORTED)) || (d.base % 3600u) != 0 || (int)(f & ROW_QW_MASK) != QW ||
                   (int)((f & ROW_VL_MASK) >> ROW_VL_SHIFT) != VL || d.ndp > (uint32_t)CH);
      if ((KEYS & 4) != 0) bad = bad || (in && !(((f & ROW_ALLF) && !(f & ROW_NAN)) || (f & ROW_ALLI)));
      if ((KEYS & 8) != 0) bad = bad || (in && d.ndp > 384u);
    }
    // strictly increasing bases (rows of one series are in base order; equal = two cells)
    const int prev = __shfl_up((int)d.base, 1, 64);
    if (in && lane > 0 && (uint32_t)prev >= d.base) bad = true;
    if (in && lane == 0 && last_base >= (int64_t)d.base) bad = true;
    if (__ballot(bad)) {
      if (lane == 0) p.redo_list[atomicAdd(p.redo_n, 1)] = (int32_t)s;
      return;
    }
    uint64_t m = __ballot(in);
    if (!m) continue;
    // rows of a series are in base order, so the in-range rows are the contiguous lanes
    // [lo, hi] of this window
    const int lo = __ffsll((long long)m) - 1, hi = 63 - __clzll((long long)m);
    last_base = (uint32_t)__builtin_amdgcn_readlane((int)d.base, hi);
    const int nin = hi - lo + 1;
    // D-deep ring, shifted by one row per step: ring[0] is row t, ring[1 .. D-1] rows
    // t+1 .. t+D-1 in flight
    using Ring = typename std::conditional<(KEYS & 8) != 0, RawV6,
                                           typename std::conditional<(KEYS & 4) != 0, RawV, RawT<QW, VL>>::type>::type;
    Ring ring[D];
    RowLite rl[D];
#pragma unroll
    for (int u = 0; u < D; u++) {
      ring[u] = {};
      if (u < D - 1 && u < nin) {
        rl[u] = row_of_lane(d, lo + u);
        load_ring_row<QW, VL, KEYS>(p, rl[u], ring[u]);
      }
    }
    for (int t = 0; t < nin; t++) {
      if (t + D - 1 < nin) {
        rl[D - 1] = row_of_lane(d, lo + t + D - 1);
        load_ring_row<QW, VL, KEYS>(p, rl[D - 1], ring[D - 1]);
      }
      if (!pct_row<QW, VL, KEYS>(p, rl[0], ring[0], q, dense, pres)) {
        if (lane == 0) p.redo_list[atomicAdd(p.redo_n, 1)] = (int32_t)s;
        return;
      }
#pragma unroll
      for (int u = 0; u < D - 1; u++) {
        ring[u] = ring[u + 1];
        rl[u] = rl[u + 1];
      }
    }
  }
}

hipError_t launch_pct(const GridParams& p, int pass, int64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (pass == 2) {
    // n = waves (p.n_launch, even): a persistent loop over the listed series
    const size_t lds = 2 * (size_t)(VBUF + PCT_CAP * 8);
    hipError_t e = hipFuncSetAttribute((const void*)k_pct<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_pct<true, false>), dim3((unsigned)((n + 1) / 2)), dim3(128), lds, s, p);
  } else {
    const size_t lds = 4 * (size_t)(VBUF + CH * 8);
    if (pass == 1)
      hipLaunchKernelGGL((k_pct<false, true>), dim3((unsigned)((n + 3) / 4)), dim3(256), lds, s, p);
    else
      hipLaunchKernelGGL((k_pct<false, false>), dim3((unsigned)((n + 3) / 4)), dim3(256), lds, s, p);
  }
  return hipGetLastError();
}

bool pct_rows_supported(int qw, int vl) { return (qw == 2 || qw == 4) && (vl == 1 || vl == 2 || vl == 4 || vl == 8); }

// ---- percentile / median as the group-by aggregator ----------------------------------
//
// AggregationIterator feeds PercentileAgg.runDouble / Median.runDouble with one value per
// span at every union timestamp (the span's bucket value, or its LERP between neighbouring
// buckets; src/core/AggregationIterator.java:735-797), and runDouble drops NaNs
// (src/core/Aggregators.java:689-706, :416-430).  k_emit_vals writes each series' value for
// every slot ([series][slot], NaN = no value); k_sel_seg stages one (group, slot) column in
// LDS as order-preserving integer keys and finds the one or two order statistics
// select_sorted needs by an 8-pass radix select -- no sort.


// One wave per tile (<= 64 series of one group).
__global__ __launch_bounds__(256) void k_emit_vals(GridParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t tile = (int64_t)blockIdx.x * p.waves + wave;
  if (tile >= p.n_tiles) return;
  const int K = (int)p.K;
  const int32_t g = p.tile_group[tile];
  uint8_t* uni = p.sel_uni + (int64_t)g * K;
  WaveLds W;
  W.rate = !p.rate ? nullptr : (p.g_rate ? p.g_rate + tile * K : (double*)(smem + (int64_t)wave * p.wave_lds));
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
    double* row = p.sel_vals + s * K;
    emit_series_to(p, W, K, [&](int k, double v, bool u) {
      row[k] = canon_nan(v);
      if (u) uni[k] = 1;
    });
  }
  if (active && lane_id() == 0) atomicOr(&p.group_active[g], 1u);
}


// The key of rank r (0-based, ascending) among keys[0..n): MSB-first radix select, 8 bits a
// pass; the bin holding rank r is found by wave 0 with a prefix sum over its lanes' 4 bins,
// and once at most SEL_FIN keys share the selected prefix they are gathered and ranked
// directly (one thread per candidate).  Called by the whole block.
constexpr int SEL_FIN = 256;
struct SelShared {
  uint32_t hist[256];
  uint64_t cand[SEL_FIN];
  uint64_t bin, rr, res;
  uint32_t ncand;
};
__device__ uint64_t radix_select(const uint64_t* keys, int64_t n, int64_t r, SelShared& S) {
  const int tid = threadIdx.x;
  // the leading digits all keys share are skipped (clustered values would otherwise put every
  // key into one bin, pass after pass): block AND / OR of the keys
  uint64_t kand = ~0ULL, kor = 0;
  for (int64_t j = tid; j < n; j += blockDim.x) {
    kand &= keys[j];
    kor |= keys[j];
  }
  if (tid == 0) { S.bin = ~0ULL; S.rr = 0; }
  __syncthreads();
  atomicAnd(reinterpret_cast<unsigned long long*>(&S.bin), (unsigned long long)kand);
  atomicOr(reinterpret_cast<unsigned long long*>(&S.rr), (unsigned long long)kor);
  __syncthreads();
  const uint64_t band = S.bin, bor = S.rr;
  __syncthreads();
  if ((band ^ bor) == 0) return band;   // all keys equal
  const int top = (63 - __clzll((long long)(band ^ bor))) & ~7;
  uint64_t mask = top == 56 ? 0 : ~((1ULL << (top + 8)) - 1ULL);
  uint64_t prefix = band & mask;
  for (int shift = top; shift >= 0; shift -= 8) {
    for (int b = tid; b < 256; b += blockDim.x) S.hist[b] = 0;
    __syncthreads();
    for (int64_t j = tid; j < n; j += blockDim.x) {
      const uint64_t k = keys[j];
      if ((k & mask) == prefix) atomicAdd(&S.hist[(k >> shift) & 255], 1u);
    }
    __syncthreads();
    if (tid < 64) {
      uint32_t c[4], t = 0;
#pragma unroll
      for (int q = 0; q < 4; q++) { c[q] = S.hist[tid * 4 + q]; t += c[q]; }
      const int64_t incl = wave_incl_sum((int)t);
      int64_t ex = incl - t;
      if (ex <= r && r < incl) {
        int q = 0;
        for (; q < 3; q++) {
          if (r < ex + c[q]) break;
          ex += c[q];
        }
        S.bin = (uint64_t)(tid * 4 + q);
        S.rr = (uint64_t)(r - ex);
        S.ncand = c[q];
      }
    }
    __syncthreads();
    prefix |= S.bin << shift;
    mask |= 255ULL << shift;
    r = (int64_t)S.rr;
    const uint32_t nc = S.ncand;
    __syncthreads();
    if (shift == 0) break;
    if (nc <= SEL_FIN) {
      if (tid == 0) S.ncand = 0;
      __syncthreads();
      for (int64_t j = tid; j < n; j += blockDim.x) {
        const uint64_t k = keys[j];
        if ((k & mask) == prefix) S.cand[atomicAdd(&S.ncand, 1u)] = k;
      }
      __syncthreads();
      if ((uint32_t)tid < nc) {
        const uint64_t x = S.cand[tid];
        uint32_t less = 0, eq = 0;
        for (uint32_t q = 0; q < nc; q++) {
          const uint64_t y = S.cand[q];
          less += y < x;
          eq += y == x;
        }
        if ((int64_t)less <= r && r < (int64_t)(less + eq)) S.res = x;
      }
      __syncthreads();
      const uint64_t res = S.res;
      __syncthreads();
      return res;
    }
  }
  return prefix;
}

// One block per (group, slot).  Blocks are dealt to the 8 XCDs in contiguous runs of
// segments, so the K columns of one group (interleaved in memory) share an L2.
__global__ __launch_bounds__(1024) void k_sel_seg(SelParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ SelShared S;
  __shared__ unsigned long long red[2];
  const int64_t nseg = p.G * p.K;
  const int64_t per = (nseg + 7) / 8;
  const int64_t i = (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
  if (i >= nseg) return;
  const int tid = threadIdx.x;
  if (!p.uni[i]) {
    if (tid == 0) { p.out_val[i] = 0.0; p.out_flag[i] = 0; }
    return;
  }
  const int64_t g = i / p.K, k = i - g * p.K;
  const int64_t gs0 = p.group_series_ptr[g], n = p.group_series_ptr[g + 1] - gs0;
  uint64_t* keys = n <= SEL_CAP ? reinterpret_cast<uint64_t*>(smem) : reinterpret_cast<uint64_t*>(p.scratch) + gs0 * p.K + k * n;
  if (tid == 0) red[0] = 0;
  __syncthreads();
  uint32_t nan_local = 0;
  // SEL_UNROLL independent loads in flight per thread (the column is strided by K: one cache
  // line per value, so the staging is latency-bound, not bandwidth-bound)
  constexpr int SEL_UNROLL = 8;
  const int bs = blockDim.x;
  for (int64_t j0 = tid; j0 < n; j0 += (int64_t)SEL_UNROLL * bs) {
    double x[SEL_UNROLL];
#pragma unroll
    for (int u = 0; u < SEL_UNROLL; u++) {
      const int64_t j = j0 + (int64_t)u * bs;
      const int64_t jj = j < n ? j : j0;
      x[u] = p.cols ? p.vals[gs0 * p.K + k * n + jj] : p.vals[(gs0 + jj) * p.K + k];
    }
#pragma unroll
    for (int u = 0; u < SEL_UNROLL; u++) {
      const int64_t j = j0 + (int64_t)u * bs;
      if (j < n) {
        nan_local += isnan(x[u]) ? 1u : 0u;
        keys[j] = f2key(canon_nan(x[u]));
      }
    }
  }
  if (nan_local) atomicAdd(&red[0], (unsigned long long)nan_local);
  __syncthreads();
  const int64_t m = n - (int64_t)red[0];   // non-NaN values (they hold ranks 0 .. m-1)
  // the indices select_sorted reads (src/core/Aggregators.java runDouble; commons-math3 LEGACY)
  int64_t r0 = 0, r1 = -1;
  if (m > 0) {
    if (p.fn == TSDB_AGG_MEDIAN) {
      r0 = m / 2;
    } else if (m > 1) {
      const double q = pct_quantile(p.fn) / 100.0;
      const double pos = (q == 0.0) ? 0.0 : (q == 1.0 ? (double)m : q * (double)(m + 1));
      if (pos < 1) r0 = 0;
      else if (pos >= (double)m) r0 = m - 1;
      else { r0 = (int64_t)floor(pos) - 1; r1 = r0 + 1; }
    }
  }
  double v0 = NAN, v1 = NAN;
  if (m > 0) {
    const uint64_t k0 = radix_select(keys, n, r0, S);
    v0 = key2f(k0);
    if (r1 >= 0) {
      // rank r0 + 1: the same key when more than r0 + 1 keys are <= k0, else the next larger key
      if (tid == 0) { red[0] = 0; red[1] = ~0ULL; }
      __syncthreads();
      uint32_t le = 0;
      uint64_t gt = ~0ULL;
      for (int64_t j = tid; j < n; j += blockDim.x) {
        const uint64_t kk = keys[j];
        if (kk <= k0) le++;
        else gt = kk < gt ? kk : gt;
      }
      atomicAdd(&red[0], (unsigned long long)le);
      atomicMin(&red[1], (unsigned long long)gt);
      __syncthreads();
      v1 = (int64_t)red[0] > r1 ? v0 : key2f(red[1]);
    }
  }
  if (tid == 0) {
    const double r = m == 0 ? (double)NAN
                            : select_sorted(p.fn, (int)m, [&](int j) { return (int64_t)j == r0 ? v0 : v1; });
    if (isinf(r)) set_err(p.err, TSDB_E_ILLEGAL_STATE);   // AggregationIterator.doubleValue :640-643
    p.out_val[i] = r;
    p.out_flag[i] = 1;
  }
}

// k_sel_reg: k_sel_seg for segments of at most SEL_REG_T * SEL_REG_R values, the keys held in
// registers (SEL_REG_R per thread) instead of staged in LDS: no 96 KB LDS buffer, so two
// blocks share a CU, and every radix pass reads registers.  Same ranks, same result.
constexpr int SEL_REG_T = 1024;
constexpr int SEL_REG_R = 12;

__device__ __forceinline__ uint64_t wave_and_u64(uint64_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x &= shfl_u64(x, lane_id() ^ d);
  return x;
}
__device__ __forceinline__ uint64_t wave_or_u64(uint64_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x |= shfl_u64(x, lane_id() ^ d);
  return x;
}

// One LDS histogram increment per lane with `in`: the lanes whose bin is the first such lane's
// add as one atomic of their count, the others one by one.  A column of similar values shares its
// leading digits, so a pass's keys pile into a few bins and a plain per-lane atomic serialises
// up to 64 same-address updates per instruction.
__device__ __forceinline__ void hist_add_agg(uint32_t* hist, bool in, uint32_t bin) {
  const uint64_t act = __ballot(in);
  if (!act) return;
  const int leader = __ffsll((long long)act) - 1;
  const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)bin, leader);
  const bool same = in && bin == b0;
  const uint64_t sm = __ballot(same);
  if (lane_id() == leader) atomicAdd(&hist[b0], (uint32_t)__popcll(sm));
  if (in && !same) atomicAdd(&hist[bin], 1u);
}

// WIDE: the first digit is the 12 bits below the prefix every key shares (a 4096-bin histogram,
// H, in LDS; WT: the 16 waves' totals of its block-wide scan), then 8-bit digits as before.  A
// column of similar doubles differs first in its exponent: the 12 bits take the exponent and the
// leading mantissa bits in one pass, and the bin of rank r usually holds few enough keys to rank
// directly -- one histogram pass instead of three.
template <int R, bool AGG = false, bool WIDE = false, int T = SEL_REG_T, class V = uint32_t>
__device__ uint64_t reg_radix_select(const uint64_t (&key)[R], V valid, int64_t r, SelShared& S,
                                     unsigned long long* red, uint32_t* H = nullptr, int* WT = nullptr) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  uint64_t kand = ~0ULL, kor = 0;
#pragma unroll
  for (int u = 0; u < R; u++) {
    if (valid >> u & 1) {
      kand &= key[u];
      kor |= key[u];
    }
  }
  kand = wave_and_u64(kand);
  kor = wave_or_u64(kor);
  if (tid == 0) { red[0] = ~0ULL; red[1] = 0; }
  __syncthreads();
  if (lane == 0) {
    atomicAnd(&red[0], (unsigned long long)kand);
    atomicOr(&red[1], (unsigned long long)kor);
  }
  __syncthreads();
  const uint64_t band = red[0], bor = red[1];
  if ((band ^ bor) == 0) return band;   // all keys equal
  // the keys sharing the selected prefix, ranked directly (nc <= SEL_FIN of them)
  auto gather_rank = [&](uint64_t mask, uint64_t prefix, int64_t rr, uint32_t nc) {
    if (tid == 0) S.ncand = 0;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < R; u++)
      if ((valid >> u & 1) && (key[u] & mask) == prefix) S.cand[atomicAdd(&S.ncand, 1u)] = key[u];
    __syncthreads();
    if ((uint32_t)tid < nc) {
      const uint64_t x = S.cand[tid];
      uint32_t less = 0, eq = 0;
      for (uint32_t q = 0; q < nc; q++) {
        const uint64_t y = S.cand[q];
        less += y < x;
        eq += y == x;
      }
      if ((int64_t)less <= rr && rr < (int64_t)(less + eq)) S.res = x;
    }
    __syncthreads();
    const uint64_t res = S.res;
    __syncthreads();
    return res;
  };
  int shift;
  uint64_t mask, prefix;
  if constexpr (WIDE) {
    const int h = 63 - __clzll((long long)(band ^ bor));   // the highest bit the keys differ in
    const int sw = h >= 11 ? h - 11 : 0;                   // digit [sw, sw + 12) (bits above h shared)
    const uint64_t above = h == 63 ? 0 : ~((1ULL << (h + 1)) - 1ULL);
    prefix = band & above;
    constexpr int BPT = 4096 / T;   // bins a thread scans (4096 bins: T x BPT)
#pragma unroll
    for (int b = 0; b < BPT / 4; b++) reinterpret_cast<uint4*>(H)[tid * (BPT / 4) + b] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < R; u++)
      if (valid >> u & 1) atomicAdd(&H[(key[u] >> sw) & 0xFFFu], 1u);
    __syncthreads();
    uint32_t c[BPT];
#pragma unroll
    for (int b = 0; b < BPT / 4; b++) {
      const uint4 c4 = reinterpret_cast<const uint4*>(H)[tid * (BPT / 4) + b];
      c[4 * b] = c4.x;
      c[4 * b + 1] = c4.y;
      c[4 * b + 2] = c4.z;
      c[4 * b + 3] = c4.w;
    }
    uint32_t t = 0;
#pragma unroll
    for (int q = 0; q < BPT; q++) t += c[q];
    const int incl = (int)wave_incl_sum((int)t);
    if (lane == 63) WT[tid >> 6] = incl;
    __syncthreads();
    int woff = 0;
    for (int w2 = 0; w2 < (tid >> 6); w2++) woff += WT[w2];
    int64_t ex = (int64_t)woff + incl - t;
    if (ex <= r && r < ex + (int64_t)t) {
      int q = 0;
      for (; q < BPT - 1; q++) {
        if (r < ex + c[q]) break;
        ex += c[q];
      }
      S.bin = (uint64_t)(tid * BPT + q);
      S.rr = (uint64_t)(r - ex);
      S.ncand = c[q];
    }
    __syncthreads();
    prefix |= S.bin << sw;
    mask = above | (0xFFFULL << sw);
    r = (int64_t)S.rr;
    const uint32_t nc = S.ncand;
    __syncthreads();
    if (sw == 0) return prefix;
    if (nc <= SEL_FIN) return gather_rank(mask, prefix, r, nc);
    shift = sw >= 8 ? sw - 8 : 0;   // (below 8: bits [sw, 8) of the next digit are already fixed)
  } else {
    shift = (63 - __clzll((long long)(band ^ bor))) & ~7;
    mask = shift == 56 ? 0 : ~((1ULL << (shift + 8)) - 1ULL);
    prefix = band & mask;
  }
  // (after the 12-bit first digit the 8-bit digits need not end on bit 0: the last one is taken at
  // shift 0, its bits above the remaining ones already fixed -- ending at shift < 0 left the low
  // bits of a key tied more than SEL_FIN times unresolved)
  for (; shift >= 0; shift = shift >= 8 ? shift - 8 : (shift > 0 ? 0 : -1)) {
    for (int b = tid; b < 256; b += blockDim.x) S.hist[b] = 0;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < R; u++) {
      const bool in = (valid >> u & 1) && (key[u] & mask) == prefix;
      if (AGG) hist_add_agg(S.hist, in, (uint32_t)(key[u] >> shift) & 255u);
      else if (in) atomicAdd(&S.hist[(key[u] >> shift) & 255], 1u);
    }
    __syncthreads();
    if (tid < 64) {
      uint32_t c[4], t = 0;
#pragma unroll
      for (int q = 0; q < 4; q++) { c[q] = S.hist[tid * 4 + q]; t += c[q]; }
      const int64_t incl = wave_incl_sum((int)t);
      int64_t ex = incl - t;
      if (ex <= r && r < incl) {
        int q = 0;
        for (; q < 3; q++) {
          if (r < ex + c[q]) break;
          ex += c[q];
        }
        S.bin = (uint64_t)(tid * 4 + q);
        S.rr = (uint64_t)(r - ex);
        S.ncand = c[q];
      }
    }
    __syncthreads();
    prefix |= S.bin << shift;
    mask |= 255ULL << shift;
    r = (int64_t)S.rr;
    const uint32_t nc = S.ncand;
    __syncthreads();
    if (shift == 0) break;
    if (nc <= SEL_FIN) return gather_rank(mask, prefix, r, nc);
  }
  return prefix;
}

template <int OCC, bool AGG = false, bool WIDE = true, int T = SEL_REG_T, int R = SEL_REG_R>
__global__ __launch_bounds__(T, OCC) void k_sel_reg(SelParams p) {
  __shared__ SelShared S;
  __shared__ unsigned long long red[2];
  __shared__ uint32_t H[WIDE ? 4096 : 1];
  __shared__ int WT[T / 64];
  const int64_t nseg = p.G * p.K;
  const int64_t per = (nseg + 7) / 8;
  const int64_t i = (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
  if (i >= nseg) return;
  const int tid = threadIdx.x;
  if (!p.uni[i]) {
    if (tid == 0) { p.out_val[i] = 0.0; p.out_flag[i] = 0; }
    return;
  }
  const int64_t g = i / p.K, k = i - g * p.K;
  const int64_t gs0 = p.group_series_ptr[g], n = p.group_series_ptr[g + 1] - gs0;
  // all loads issued before any is consumed (strided column: latency-bound)
  double x[R];
#pragma unroll
  for (int u = 0; u < R; u++) {
    const int64_t j = tid + (int64_t)u * T;
    const int64_t jj = j < n ? j : 0;
    x[u] = p.cols ? p.vals[gs0 * p.K + k * n + jj] : p.vals[(gs0 + jj) * p.K + k];
  }
  uint64_t key[R];
  using V = std::conditional_t<(R > 32), uint64_t, uint32_t>;   // a bit a key slot
  V valid = 0;
  int nan_local = 0;
#pragma unroll
  for (int u = 0; u < R; u++) {
    const bool v = tid + (int64_t)u * T < n;
    valid |= (V)(v ? 1u : 0u) << u;
    nan_local += (v && isnan(x[u])) ? 1 : 0;
    key[u] = f2key(canon_nan(x[u]));
  }
  nan_local = wave_sum_int(nan_local);
  if (tid == 0) red[0] = 0;
  __syncthreads();
  if ((tid & 63) == 0 && nan_local) atomicAdd(&red[0], (unsigned long long)nan_local);
  __syncthreads();
  const int64_t m = n - (int64_t)red[0];   // non-NaN values (they hold ranks 0 .. m-1)
  __syncthreads();
  int64_t r0 = 0, r1 = -1;
  if (m > 0) {
    if (p.fn == TSDB_AGG_MEDIAN) {
      r0 = m / 2;
    } else if (m > 1) {
      const double q = pct_quantile(p.fn) / 100.0;
      const double pos = (q == 0.0) ? 0.0 : (q == 1.0 ? (double)m : q * (double)(m + 1));
      if (pos < 1) r0 = 0;
      else if (pos >= (double)m) r0 = m - 1;
      else { r0 = (int64_t)floor(pos) - 1; r1 = r0 + 1; }
    }
  }
  double v0 = NAN, v1 = NAN;
  if (m > 0) {
    const uint64_t k0 = reg_radix_select<R, AGG, WIDE, T, V>(key, valid, r0, S, red, H, WT);
    v0 = key2f(k0);
    if (r1 >= 0) {
      // rank r0 + 1: the same key when more than r0 + 1 keys are <= k0, else the next larger key
      __syncthreads();
      if (tid == 0) { red[0] = 0; red[1] = ~0ULL; }
      __syncthreads();
      int le = 0;
      uint64_t gt = ~0ULL;
#pragma unroll
      for (int u = 0; u < R; u++) {
        if (valid >> u & 1) {
          if (key[u] <= k0) le++;
          else gt = key[u] < gt ? key[u] : gt;
        }
      }
      le = wave_sum_int(le);
      gt = wave_min_u64(gt);
      if ((tid & 63) == 0) {
        atomicAdd(&red[0], (unsigned long long)le);
        atomicMin(&red[1], (unsigned long long)gt);
      }
      __syncthreads();
      v1 = (int64_t)red[0] > r1 ? v0 : key2f(red[1]);
    }
  }
  if (tid == 0) {
    const double r = m == 0 ? (double)NAN
                            : select_sorted(p.fn, (int)m, [&](int j) { return (int64_t)j == r0 ? v0 : v1; });
    if (isinf(r)) set_err(p.err, TSDB_E_ILLEGAL_STATE);   // AggregationIterator.doubleValue :640-643
    p.out_val[i] = r;
    p.out_flag[i] = 1;
  }
}


template <int KPL>
__device__ uint64_t wave_radix_select_reg(const uint64_t (&kr)[KPL], uint64_t vm, int r, SelWave& W);

// ---- the sampled-window select (engine.cpp sel_window) ------------------------------------
// One wave a (group, slot) column, four a block, no block barriers: the sample and the kept values
// are at most WIN_SCAP / WIN_CCAP = 1024, 16 keys a lane, and wave_radix_select_reg (k_raw_sel's
// register select) ranks them.  (A block of 256 a column with k_sel_reg's select, barrier-bound:
// bounds 0.47 ms + select 0.46 ms over config 3's 60000 columns, profiles/r05ao.)
constexpr int WIN_KPL = 16;   // keys a lane
__device__ __forceinline__ int64_t win_column(int64_t nseg) {
  const int64_t nblk = (nseg + 3) / 4;
  const int64_t per = (nblk + 7) / 8;   // blocks dealt to the XCDs in contiguous runs
  return ((int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8) * 4 + (threadIdx.x >> 6);
}

// k_win_bounds: the window [lo, hi] of each column from the sample pass's values (the sampled
// positions of the column layout): the sample ranks around the target ranks (estimated from the
// sample's non-NaN fraction) with a binomial margin of 6 standard deviations + 2 (~1e-9 a column
// and side: a 60000-column query falls back about once in 10^4); an end past the sample is
// unbounded, as are both for fewer than 32 sampled values.  The window only decides which values
// the main pass keeps: k_win_select checks with exact counts that it holds the ranks.
__global__ __launch_bounds__(256) void k_win_bounds(WinParams p) {
  __shared__ SelWave WS[4];
  const int64_t i = win_column(p.G * p.K);
  if (i >= p.G * p.K) return;   // (whole waves)
  const int lane = lane_id();
  SelWave& W = WS[threadIdx.x >> 6];
  const int64_t g = i / p.K, k = i - g * p.K;
  const int64_t g0 = p.group_series_ptr[g], n = p.group_series_ptr[g + 1] - g0;
  const int32_t sa = p.samp_ptr[g], np = min(p.samp_ptr[g + 1] - sa, 64 * WIN_KPL);
  const double* col = p.vals + g0 * p.K + k * n;
  uint64_t kr[WIN_KPL];
  uint64_t vm = 0;
  int nv = 0;
#pragma unroll
  for (int u = 0; u < WIN_KPL; u++) {
    const int j = lane + 64 * u;
    // (a sampled position the sample pass did not write -- a handed-back tile's series without
    // rows in the scan range -- holds a stale value: it only shifts the window)
    const double x = j < np ? col[p.samp_pos[sa + j]] : 0.0;
    const bool v = j < np && !isnan(x);
    vm |= (uint64_t)v << u;
    nv += v ? 1 : 0;
    kr[u] = f2key(x);
  }
  const int64_t nsv = wave_sum_int(nv);
  double lo = -(double)INFINITY, hi = (double)INFINITY;
  if (nsv >= 32) {
    const double m_est = (double)nsv * (double)n / (double)max(1, np);
    int64_t r0, r1;
    sel_ranks(p.fn, max<int64_t>(1, (int64_t)llround(m_est)), r0, r1);
    const double me = max(1.0, m_est);
    const double f0 = (double)r0 / me, f1 = (double)(r1 >= 0 ? r1 : r0) / me;
    const double sd0 = sqrt((double)nsv * f0 * (1.0 - f0)), sd1 = sqrt((double)nsv * f1 * (1.0 - f1));
    const int64_t q0 = (int64_t)floor(f0 * (double)nsv - 6.0 * sd0 - 2.0);
    const int64_t q1 = (int64_t)ceil(f1 * (double)nsv + 6.0 * sd1 + 2.0);
    if (q0 >= 0) lo = key2f(wave_radix_select_reg<WIN_KPL>(kr, vm, (int)min(q0, nsv - 1), W));
    if (q1 < nsv) hi = key2f(wave_radix_select_reg<WIN_KPL>(kr, vm, (int)max<int64_t>(q1, 0), W));
  }
  if (lane == 0) {
    p.lo[i] = lo;
    p.hi[i] = hi;
  }
}

// k_win_select: one wave a column over its window counts and values (the main pass, k_short KR 5,
// adds each tile's counts and appends its values inside): m = below + above + inside (the non-NaN
// contributions, as the full path's m), the ranks select_sorted reads (as k_sel_reg), and when the
// window holds them (below <= r0, the upper rank < below + inside, inside <= WIN_CCAP) their keys
// among the inside values -- the full path's keys, so its result; else the column sets p.fail.
__global__ __launch_bounds__(256) void k_win_select(WinParams p) {
  __shared__ SelWave WS[4];
  const int64_t i = win_column(p.G * p.K);
  if (i >= p.G * p.K) return;   // (whole waves)
  const int lane = lane_id();
  SelWave& W = WS[threadIdx.x >> 6];
  // the flags, counts and values loaded together (the column's region holds WIN_CCAP values)
  const double* cand = p.cand + i * WIN_CCAP;
  const uint8_t un = p.uni[i];
  const unsigned long long ba = p.gcnt[i];
  const uint32_t cc = p.cur[i];
  double x[WIN_KPL];
#pragma unroll
  for (int u = 0; u < 4; u++) x[u] = cand[lane + 64 * u];   // (typical p99 columns keep ~450)
  if (!un) {
    if (lane == 0) { p.out_val[i] = 0.0; p.out_flag[i] = 0; }
    return;
  }
  const int64_t B = (int64_t)(ba & 0xFFFFFFFFull), C = cc;
  const int64_t m = B + (int64_t)(ba >> 32) + C;
  if (m == 0) {
    if (lane == 0) { p.out_val[i] = (double)NAN; p.out_flag[i] = 1; }
    return;
  }
  int64_t r0, r1;
  sel_ranks(p.fn, m, r0, r1);
  const int64_t rhi = r1 >= 0 ? r1 : r0;
  if (C > WIN_CCAP || r0 < B || rhi >= B + C) {
    if (lane == 0) atomicOr(p.fail, 1);
    return;
  }
#pragma unroll
  for (int u = 4; u < WIN_KPL; u++) x[u] = lane + 64 * u < C ? cand[lane + 64 * u] : 0.0;
  uint64_t kr[WIN_KPL];
  uint64_t vm = 0;
#pragma unroll
  for (int u = 0; u < WIN_KPL; u++) {
    const bool v = lane + 64 * u < C;
    vm |= (uint64_t)v << u;
    kr[u] = v ? f2key(x[u]) : ~0ULL;
  }
  const uint64_t k0 = wave_radix_select_reg<WIN_KPL>(kr, vm, (int)(r0 - B), W);
  const double v0 = key2f(k0);
  double v1 = v0;
  if (r1 >= 0) {
    // rank r1 = r0 + 1: the same key when more than r1 - B kept keys are <= k0, else the next larger
    int le = 0;
    uint64_t gt = ~0ULL;
#pragma unroll
    for (int u = 0; u < WIN_KPL; u++) {
      if ((vm >> u) & 1ULL) {
        if (kr[u] <= k0) le++;
        else gt = kr[u] < gt ? kr[u] : gt;
      }
    }
    le = wave_sum_int(le);
    gt = wave_min_u64(gt);
    v1 = (int64_t)le > r1 - B ? v0 : key2f(gt);
  }
  if (lane == 0) {
    const double r = select_sorted(p.fn, (int)m, [&](int j) { return (int64_t)j == r0 ? v0 : v1; });
    if (isinf(r)) set_err(p.err, TSDB_E_ILLEGAL_STATE);   // AggregationIterator.doubleValue :640-643
    p.out_val[i] = r;
    p.out_flag[i] = 1;
  }
}

// k_sel_wave<KPL>: k_sel_reg for columns of at most 64 KPL values -- one wave a (group, slot)
// column, four a block (adjacent columns: in the [series][K] layout they read the same row lines),
// the keys in registers and wave_radix_select_reg, no block barriers.  k_sel_reg spends a
// 512-thread block and a 4096-bin histogram on each column, whatever its size: the multi-device
// owners' selection (a day of 1m slots, ~250-1000 spans a column) ran at ~12 G values/s on it.
// NaN contributions (no value) are left out of the mask: they are the largest keys, so ranks
// 0 .. m-1 of the non-NaN values are k_sel_reg's, and so is the result.
template <int KPL>
__global__ __launch_bounds__(256) void k_sel_wave(SelParams p) {
  __shared__ SelWave WS[4];
  const int64_t i = win_column(p.G * p.K);
  if (i >= p.G * p.K) return;   // (whole waves)
  const int lane = lane_id();
  SelWave& W = WS[threadIdx.x >> 6];
  if (!p.uni[i]) {
    if (lane == 0) { p.out_val[i] = 0.0; p.out_flag[i] = 0; }
    return;
  }
  const int64_t g = i / p.K, k = i - g * p.K;
  const int64_t gs0 = p.group_series_ptr[g], n = p.group_series_ptr[g + 1] - gs0;
  double x[KPL];
#pragma unroll
  for (int u = 0; u < KPL; u++) {
    const int64_t j = lane + 64 * u;
    x[u] = j < n ? (p.cols ? p.vals[gs0 * p.K + k * n + j] : p.vals[(gs0 + j) * p.K + k]) : (double)NAN;
  }
  uint64_t kr[KPL];
  uint64_t vm = 0;
  int nv = 0;
#pragma unroll
  for (int u = 0; u < KPL; u++) {
    const bool v = !isnan(x[u]);
    vm |= (uint64_t)v << u;
    nv += v ? 1 : 0;
    kr[u] = v ? f2key(x[u]) : ~0ULL;
  }
  const int64_t m = wave_sum_int(nv);
  if (m == 0) {
    if (lane == 0) { p.out_val[i] = (double)NAN; p.out_flag[i] = 1; }
    return;
  }
  int64_t r0, r1;
  sel_ranks(p.fn, m, r0, r1);
  const uint64_t k0 = wave_radix_select_reg<KPL>(kr, vm, (int)r0, W);
  const double v0 = key2f(k0);
  double v1 = v0;
  if (r1 >= 0) {
    // rank r1 = r0 + 1: the same key when more than r1 keys are <= k0, else the next larger key
    int le = 0;
    uint64_t gt = ~0ULL;
#pragma unroll
    for (int u = 0; u < KPL; u++) {
      if ((vm >> u) & 1ULL) {
        if (kr[u] <= k0) le++;
        else gt = kr[u] < gt ? kr[u] : gt;
      }
    }
    le = wave_sum_int(le);
    gt = wave_min_u64(gt);
    v1 = (int64_t)le > r1 ? v0 : key2f(gt);
  }
  if (lane == 0) {
    const double r = select_sorted(p.fn, (int)m, [&](int j) { return (int64_t)j == r0 ? v0 : v1; });
    if (isinf(r)) set_err(p.err, TSDB_E_ILLEGAL_STATE);   // AggregationIterator.doubleValue :640-643
    p.out_val[i] = r;
    p.out_flag[i] = 1;
  }
}

hipError_t launch_win_bounds(const WinParams& p, hipStream_t s) {
  const int64_t n = p.G * p.K;
  if (n == 0) return hipSuccess;
  const int64_t nblk = (n + 3) / 4;
  hipLaunchKernelGGL(k_win_bounds, dim3((unsigned)(((nblk + 7) / 8) * 8)), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_win_select(const WinParams& p, hipStream_t s) {
  const int64_t n = p.G * p.K;
  if (n == 0) return hipSuccess;
  const int64_t nblk = (n + 3) / 4;
  hipLaunchKernelGGL(k_win_select, dim3((unsigned)(((nblk + 7) / 8) * 8)), dim3(256), 0, s, p);
  return hipGetLastError();
}


// One thread per (group, slot), consecutive slots in consecutive lanes (coalesced rows):
// contribute_slot over the group's spans in index order, then ps_final.  A span without a
// value at the slot holds sel_values' fill pattern (0x7FF87FF87FF87FF8), distinct from the
// canonical NaN of a real NaN value (which MULT / FIRST / LAST see).
// The fold is a dependent chain over the group's spans and only G * K threads run it, so the
// kernel is memory-latency bound: ORD_U loads per batch are issued one batch AHEAD of the fold
// (two register buffers), and the aggregator is a template parameter so that a fold step is a
// few instructions (the runtime switch cost more issue slots than the loads).
constexpr int ORD_U = 32;

template <int GA>
__device__ __forceinline__ void ord_fold(RegPart& R, const double (&v)[ORD_U]) {
#pragma unroll
  for (int u = 0; u < ORD_U; u++)
    if ((uint64_t)__double_as_longlong(v[u]) != 0x7FF87FF87FF87FF8ULL) contribute_slot(GA, R, v[u], false);
}

template <int GA>
__global__ __launch_bounds__(256) void k_ordered(OrdParams p) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.G * p.K) return;
  const int64_t g = i / p.K, k = i - g * p.K;
  RegPart R;
  regpart_init(GA, R);
  const int64_t s1 = p.group_series_ptr[g + 1];
  const double* col = p.vals + k;
  int64_t s = p.group_series_ptr[g];
  double va[ORD_U], vb[ORD_U];
  if (s + ORD_U <= s1) {
#pragma unroll
    for (int u = 0; u < ORD_U; u++) va[u] = col[(s + u) * p.K];
  }
  while (s + 2 * ORD_U <= s1) {
#pragma unroll
    for (int u = 0; u < ORD_U; u++) vb[u] = col[(s + ORD_U + u) * p.K];
    ord_fold<GA>(R, va);
#pragma unroll
    for (int u = 0; u < ORD_U; u++) va[u] = vb[u];
    s += ORD_U;
  }
  if (s + ORD_U <= s1) {
    ord_fold<GA>(R, va);
    s += ORD_U;
  }
  for (; s < s1; s++) {
    const double v = col[s * p.K];
    if ((uint64_t)__double_as_longlong(v) == 0x7FF87FF87FF87FF8ULL) continue;
    contribute_slot(GA, R, v, false);
  }
  const bool emit = p.uni[i] != 0;
  PState S;
  S.a = R.pa;
  S.b = R.pb;
  S.n = R.pn;
  S.f = R.pf | (emit ? PF_UNION : 0u);
  p.out_val[i] = emit ? ps_final(GA, S, p.err) : 0.0;
  p.out_flag[i] = emit ? 1 : 0;
}

hipError_t launch_ordered(const OrdParams& p, hipStream_t s) {
  const int64_t n = p.G * p.K;
  if (n == 0) return hipSuccess;
  const dim3 grid((unsigned)((n + 255) / 256)), block(256);
  switch (p.ga) {
#define ORD_CASE(G_) \
  case G_: hipLaunchKernelGGL(k_ordered<G_>, grid, block, 0, s, p); break;
    ORD_CASE(GA_SUM) ORD_CASE(GA_AVG) ORD_CASE(GA_COUNT) ORD_CASE(GA_SQUARESUM) ORD_CASE(GA_MIN) ORD_CASE(GA_MAX)
    ORD_CASE(GA_DEV) ORD_CASE(GA_FIRST) ORD_CASE(GA_LAST) ORD_CASE(GA_DIFF) ORD_CASE(GA_MULT) ORD_CASE(GA_NONE)
#undef ORD_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_emit_vals(const GridParams& p, hipStream_t s) {
  if (p.n_tiles == 0) return hipSuccess;
  const int64_t blocks = (p.n_tiles + p.waves - 1) / p.waves;
  const size_t lds = (size_t)p.wave_lds * p.waves;
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)k_emit_vals, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_emit_vals, dim3((unsigned)blocks), dim3(64 * p.waves), lds, s, p);
  return hipGetLastError();
}

hipError_t launch_sel_seg(const SelParams& p, hipStream_t s, int64_t maxn) {
  const int64_t n = p.G * p.K;
  if (n == 0) return hipSuccess;
  const int64_t per = (n + 7) / 8;
  // columns of at most 2048 values: a wave each (k_sel_wave); option SEL_WAVE = 0 keeps the block
  if (maxn <= 64 * 32 && !opt_off(OPT_SEL_WAVE)) {
    const int64_t nblk = (n + 3) / 4;
    const dim3 grid((unsigned)(((nblk + 7) / 8) * 8));
    if (maxn <= 64 * 4) hipLaunchKernelGGL(k_sel_wave<4>, grid, dim3(256), 0, s, p);
    else if (maxn <= 64 * 16) hipLaunchKernelGGL(k_sel_wave<16>, grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL(k_sel_wave<32>, grid, dim3(256), 0, s, p);
    return hipGetLastError();
  }
  if (maxn <= (int64_t)SEL_REG_T * SEL_REG_R && !opt_off(OPT_SEL_REG)) {
    // 512 threads x 24 keys, two blocks a CU without spills: config 3 p99:1m-avg 7.40 ms a step,
    // against 7.90 for 1024 x 12 at two blocks (spilling), 7.72 for 512 x 24 at three, 7.58 for
    // 256 x 48, 8.54 for 1024 x 12 unspilled, 7.44 for 32-bit keys of the upper words (k_sel_hl),
    // 10.4 -> 11.4 for two slots a block (profiles/r03g, r05z, r05ad); those variants are gone
    hipLaunchKernelGGL((k_sel_reg<4, false, true, 512, 24>), dim3((unsigned)(per * 8)), dim3(512), 0, s, p);
    return hipGetLastError();
  }
  const size_t lds = (size_t)SEL_CAP * 8;
  hipError_t e = hipFuncSetAttribute((const void*)k_sel_seg, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_sel_seg, dim3((unsigned)(per * 8)), dim3(1024), lds, s, p);
  return hipGetLastError();
}

hipError_t launch_pct_rows(const GridParams& p, int qw, int vl, hipStream_t s) {
  if (p.n_series == 0) return hipSuccess;
  const dim3 grid((unsigned)((p.n_series + 3) / 4)), block(256);
  // ring depth: 3 rows for the general kernel; 2 for the key kernel (config 5 1h-p99: 18.1 /
  // 19.7 / 22.0 ms at D = 2 / 3 / 4 -- occupancy beats depth)
  const int D = vl == 4 && p.I == 3600000 ? 2 : 3;
  // 1 h buckets of 4-byte values: the 32-bit key kernel (its misses go to k_pct)
  const bool keys = vl == 4 && p.I == 3600000 && !opt_off(OPT_PCT_KEYS);
  const int sel_i = (p.sel_fn - TSDB_AGG_P999) % 6;
  const bool mid = p.sel_fn == TSDB_AGG_MEDIAN || sel_i >= 4;   // median, p75, p50 (and their ep* forms)
#define PCT_ROWS_CASE(Q, V)                                                                                  \
  if (qw == Q && vl == V) {                                                                                \
    if (V == 4 && keys && p.pct_vonly && p.pct_v6) {                                                       \
      if (mid) hipLaunchKernelGGL((k_pct_rows<Q, V, 2, 14>), grid, block, 0, s, p);                       \
      else hipLaunchKernelGGL((k_pct_rows<Q, V, 2, 13>), grid, block, 0, s, p);                            \
      return hipGetLastError();                                                                            \
    }                                                                                                      \
    if (V == 4 && keys && p.pct_vonly) {                                                                   \
      if (mid) hipLaunchKernelGGL((k_pct_rows<Q, V, 2, 6>), grid, block, 0, s, p);                        \
      else hipLaunchKernelGGL((k_pct_rows<Q, V, 2, 5>), grid, block, 0, s, p);                             \
      return hipGetLastError();                                                                            \
    }                                                                                                      \
    if (V == 4 && keys) {                                                                                  \
      if (mid) hipLaunchKernelGGL((k_pct_rows<Q, V, 2, 2>), grid, block, 0, s, p);                        \
      else hipLaunchKernelGGL((k_pct_rows<Q, V, 2, 1>), grid, block, 0, s, p);                             \
      return hipGetLastError();                                                                            \
    }                                                                                                      \
    if (D == 2) hipLaunchKernelGGL((k_pct_rows<Q, V, 2, 0>), grid, block, 0, s, p);                        \
    else hipLaunchKernelGGL((k_pct_rows<Q, V, 3, 0>), grid, block, 0, s, p);                               \
    return hipGetLastError();                                                                              \
  }
  PCT_ROWS_CASE(2, 1) PCT_ROWS_CASE(2, 2) PCT_ROWS_CASE(2, 4) PCT_ROWS_CASE(2, 8)
  PCT_ROWS_CASE(4, 1) PCT_ROWS_CASE(4, 2) PCT_ROWS_CASE(4, 4) PCT_ROWS_CASE(4, 8)
#undef PCT_ROWS_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_emit(const GridParams& p, hipStream_t s) {
  if (p.n_tiles == 0) return hipSuccess;
  if (p.K <= 32 && !p.rate && !opt_off(OPT_EMIT_HALF)) {   // two series a step (half waves)
    GridParams q = p;
    q.waves = 4;
    const dim3 grid((unsigned)((p.n_tiles + 3) / 4));
    switch (p.ga) {
      case GA_SUM: hipLaunchKernelGGL(k_emit_reg2<GA_SUM>, grid, dim3(256), 0, s, q); break;
      case GA_AVG: hipLaunchKernelGGL(k_emit_reg2<GA_AVG>, grid, dim3(256), 0, s, q); break;
      case GA_COUNT: hipLaunchKernelGGL(k_emit_reg2<GA_COUNT>, grid, dim3(256), 0, s, q); break;
      case GA_MIN: hipLaunchKernelGGL(k_emit_reg2<GA_MIN>, grid, dim3(256), 0, s, q); break;
      case GA_MAX: hipLaunchKernelGGL(k_emit_reg2<GA_MAX>, grid, dim3(256), 0, s, q); break;
      case GA_DEV: hipLaunchKernelGGL(k_emit_reg2<GA_DEV>, grid, dim3(256), 0, s, q); break;
      default: hipLaunchKernelGGL(k_emit_reg2<-1>, grid, dim3(256), 0, s, q); break;
    }
    return hipGetLastError();
  }
  if (p.K <= 64 && !p.rate) {
    GridParams q = p;
    q.waves = 4;
    const dim3 grid((unsigned)((p.n_tiles + 3) / 4));
    switch (p.ga) {
      case GA_SUM: hipLaunchKernelGGL(k_emit_reg<GA_SUM>, grid, dim3(256), 0, s, q); break;
      case GA_AVG: hipLaunchKernelGGL(k_emit_reg<GA_AVG>, grid, dim3(256), 0, s, q); break;
      case GA_COUNT: hipLaunchKernelGGL(k_emit_reg<GA_COUNT>, grid, dim3(256), 0, s, q); break;
      case GA_MIN: hipLaunchKernelGGL(k_emit_reg<GA_MIN>, grid, dim3(256), 0, s, q); break;
      case GA_MAX: hipLaunchKernelGGL(k_emit_reg<GA_MAX>, grid, dim3(256), 0, s, q); break;
      case GA_DEV: hipLaunchKernelGGL(k_emit_reg<GA_DEV>, grid, dim3(256), 0, s, q); break;
      default: hipLaunchKernelGGL(k_emit_reg<-1>, grid, dim3(256), 0, s, q); break;
    }
    return hipGetLastError();
  }
  if (p.K > 64 && !p.rate) {
    const int nwin = (int)((p.K + 63) / 64);
    const int64_t waves = p.n_tiles * nwin;
    hipLaunchKernelGGL(k_emit_win, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, p, nwin);
    return hipGetLastError();
  }
  const int64_t blocks = (p.n_tiles + p.waves - 1) / p.waves;
  const size_t lds = (size_t)p.wave_lds * p.waves;
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)k_emit, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_emit, dim3((unsigned)blocks), dim3(64 * p.waves), lds, s, p);
  return hipGetLastError();
}

// ---- percentile / median group-by without downsampling (raw timestamp union) --------------
// One block per union point.  The point's span operands (k_raw_vals) are staged in LDS as
// order-preserving keys; the order statistics come from radix_select.  isInteger at the point
// (AggregationIterator.isInteger :612-625) picks the reducer, as longValue / doubleValue do:
//   runLong   (src/core/Aggregators.java:403-413 Median, :675-686 PercentileAgg): every span
//             operand, the estimation type honoured (LEGACY / R_3 / R_7), (long) of the estimate;
//   runDouble (:416-430, :689-706): NaNs skipped, LEGACY always.

// One WAVE per union point of the batch's strips (4 waves a block, no block barriers):
// point pt -> strip pt / RAW_STRIP, position j.  Wave-local radix select: 8-bit digits, a
// 256-bin LDS histogram per wave, the digit holding rank r found by a wave prefix sum over
// the lanes' 4 bins; once <= 64 keys share the prefix they are ranked directly.
__global__ __launch_bounds__(256) void k_raw_sel(RawParams p, int32_t kcap) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ SelWave WS[SELW];
  const int wv = threadIdx.x >> 6;
  const int lane = lane_id();
  const int64_t pt = (int64_t)blockIdx.x * SELW + wv;
  const int64_t sl = pt / RAW_STRIP;
  const int64_t j = pt - sl * RAW_STRIP;
  if (sl >= p.n_strips) return;   // whole waves leave; no block barrier follows
  const int64_t gi = p.strip_g[sl];
  const int64_t u = (int64_t)p.strip_t[sl] * RAW_STRIP + j;
  if (u >= p.U[gi]) return;
  const int64_t idx = p.out_off[gi] + u;
  const int64_t g = gi + p.g0;
  const int k = (int)(p.grp_ser[g + 1] - p.grp_ser[g]);
  const int64_t vb = p.vals_off[sl] + j;
  constexpr int64_t US = RAW_STRIP;   // operand stride between spans
  const bool is_int = p.out_int[idx] != 0;
  SelWave& W = WS[wv];
  // keys in LDS, or (groups beyond kcap) in place over the strided operands themselves
  const bool in_lds = k <= kcap;
  const int64_t ks = in_lds ? 1 : US;
  uint64_t* keys = in_lds ? reinterpret_cast<uint64_t*>(smem) + (int64_t)wv * kcap
                          : reinterpret_cast<uint64_t*>(is_int ? (void*)p.vals_l : (void*)p.vals_d) + vb;
  const uint64_t below = (1ULL << lane) - 1ULL;   // lanes < lane
  int m = 0;
  // RAW_SEL_B rows of 64 operands loaded before any is used: the operands are strided by
  // RAW_STRIP (one line each), so a load-use chain per row left the kernel waiting on memory
  // latency 25 times a point for config 4's 1560-span groups
  if (is_int) {
    // present long operands, compacted (their order does not matter to a selection)
    for (int base = 0; base < k; base += 64 * RAW_SEL_B) {
      bool pres[RAW_SEL_B];
      uint64_t key[RAW_SEL_B];
#pragma unroll
      for (int u = 0; u < RAW_SEL_B; u++) {
        const int i = base + 64 * u + lane;
        const int ic = i < k ? i : 0;
        pres[u] = i < k && p.vals_p[vb + ic * US];
        key[u] = (uint64_t)p.vals_l[vb + ic * US] ^ 0x8000000000000000ULL;
      }
      WAVE_SYNC();   // in place: every lane has read its operands before any is overwritten
#pragma unroll
      for (int u = 0; u < RAW_SEL_B; u++) {
        const uint64_t bal = (uint64_t)__ballot(pres[u]);
        if (pres[u]) keys[(m + __popcll(bal & below)) * ks] = key[u];
        m += __popcll(bal);
      }
    }
  } else {
    int nan = 0;
    for (int base = 0; base < k; base += 64 * RAW_SEL_B) {
      double x[RAW_SEL_B];
#pragma unroll
      for (int u = 0; u < RAW_SEL_B; u++) {
        const int i = base + 64 * u + lane;
        x[u] = p.vals_d[vb + (int64_t)(i < k ? i : 0) * US];
      }
      WAVE_SYNC();
#pragma unroll
      for (int u = 0; u < RAW_SEL_B; u++) {
        const int i = base + 64 * u + lane;
        bool isn = false;
        if (i < k) {
          isn = isnan(x[u]);
          keys[i * ks] = f2key(canon_nan(x[u]));
        }
        nan += __popcll((uint64_t)__ballot(isn));
      }
    }
    m = k - nan;
  }
  WAVE_SYNC();
  const int n = is_int ? m : k;   // keys staged
  const int fn = p.sel_fn;
  int r0, r1;
  double dif;
  raw_sel_ranks(fn, is_int, m, r0, r1, dif);
  uint64_t k0 = 0, k1 = 0;
  if (m > 0) {
    k0 = wave_radix_select(keys, ks, n, r0, W);
    k1 = k0;
    if (r1 >= 0) {
      // rank r0 + 1: the same key when more than r0 + 1 keys are <= k0, else the next larger key
      int le = 0;
      uint64_t gt = ~0ULL;
      for (int jj = lane; jj < n; jj += 64) {
        const uint64_t kk = keys[jj * ks];
        if (kk <= k0) le++;
        else gt = kk < gt ? kk : gt;
      }
      le = wave_sum_int(le);
      gt = wave_min_u64(gt);
      k1 = le > r1 ? k0 : gt;
    }
  }
  if (lane == 0) raw_sel_store(p, idx, is_int, fn, m, r1, dif, k0, k1);
}

// Register-resident variant (groups of <= 64 KPL spans): lane l holds operands l, l + 64, ...
// as keys (all KPL loads in flight together), a validity mask stands in for the compaction,
// and the radix passes read registers.  The wave's LDS is the 256-bin histogram and the
// candidate list only, so residency is set by registers (k_raw_sel: a 12.5-KB key stage per
// wave for config 4's 1560-span groups, 3 waves a SIMD).  Same ranks, same keys, same result.
template <int KPL>
__device__ uint64_t wave_radix_select_reg(const uint64_t (&kr)[KPL], uint64_t vm, int r, SelWave& W) {
  const int lane = lane_id();
  uint64_t kand = ~0ULL, kor = 0;
#pragma unroll
  for (int u = 0; u < KPL; u++)
    if ((vm >> u) & 1ULL) { kand &= kr[u]; kor |= kr[u]; }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    kand &= shfl_u64(kand, lane ^ d);
    kor |= shfl_u64(kor, lane ^ d);
  }
  const uint64_t diff = kand ^ kor;
  if (diff == 0) return kand;
  const int top = (63 - __clzll((long long)diff)) & ~7;
  uint64_t mask = top == 56 ? 0 : ~((1ULL << (top + 8)) - 1ULL);
  uint64_t prefix = kand & mask;
  for (int shift = top; shift >= 0; shift -= 8) {
#pragma unroll
    for (int q = 0; q < 4; q++) W.hist[lane * 4 + q] = 0;
    WAVE_SYNC();
#pragma unroll
    for (int u = 0; u < KPL; u++)
      if (((vm >> u) & 1ULL) && (kr[u] & mask) == prefix) atomicAdd(&W.hist[(kr[u] >> shift) & 255], 1u);
    WAVE_SYNC();
    uint32_t c[4], t = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) { c[q] = W.hist[lane * 4 + q]; t += c[q]; }
    const int incl = wave_incl_sum((int)t);
    int ex = incl - (int)t;
    const bool found = ex <= r && r < incl;
    int bin = 0, rr = 0, nc = 0;
    if (found) {
      int q = 0;
      for (; q < 3; q++) {
        if (r < ex + (int)c[q]) break;
        ex += (int)c[q];
      }
      bin = lane * 4 + q;
      rr = r - ex;
      nc = (int)c[q];
    }
    const int src = __ffsll((long long)__ballot(found)) - 1;
    bin = __shfl(bin, src, 64);
    rr = __shfl(rr, src, 64);
    nc = __shfl(nc, src, 64);
    prefix |= (uint64_t)bin << shift;
    mask |= 255ULL << shift;
    r = rr;
    WAVE_SYNC();
    if (shift == 0) break;
    if (nc <= 64) {
      if (lane == 0) W.n = 0;
      WAVE_SYNC();
#pragma unroll
      for (int u = 0; u < KPL; u++)
        if (((vm >> u) & 1ULL) && (kr[u] & mask) == prefix) W.cand[atomicAdd(&W.n, 1u)] = kr[u];
      WAVE_SYNC();
      const uint64_t x = lane < nc ? W.cand[lane] : ~0ULL;
      int less = 0, eq = 0;
      for (int q = 0; q < nc; q++) {
        const uint64_t y = W.cand[q];
        less += y < x;
        eq += y == x;
      }
      const bool hit = lane < nc && less <= r && r < less + eq;
      const uint64_t res = shfl_u64(x, __ffsll((long long)__ballot(hit)) - 1);
      WAVE_SYNC();
      return res;
    }
  }
  return prefix;
}

template <int KPL>
__global__ __launch_bounds__(256) void k_raw_sel_reg(RawParams p) {
  __shared__ SelWave WS[SELW];
  const int wv = threadIdx.x >> 6;
  const int lane = lane_id();
  const int64_t pt = (int64_t)blockIdx.x * SELW + wv;
  const int64_t sl = pt / RAW_STRIP;
  const int64_t j = pt - sl * RAW_STRIP;
  if (sl >= p.n_strips) return;   // whole waves leave; no block barrier follows
  const int64_t gi = p.strip_g[sl];
  const int64_t u0 = (int64_t)p.strip_t[sl] * RAW_STRIP + j;
  if (u0 >= p.U[gi]) return;
  const int64_t idx = p.out_off[gi] + u0;
  const int64_t g = gi + p.g0;
  const int k = (int)(p.grp_ser[g + 1] - p.grp_ser[g]);   // <= 64 KPL (host-checked)
  const int64_t vb = p.vals_off[sl] + j;
  constexpr int64_t US = RAW_STRIP;
  const bool is_int = p.out_int[idx] != 0;
  SelWave& W = WS[wv];
  uint64_t kr[KPL];
  uint64_t vm = 0;
  int m;
  if (is_int) {
    bool pr[KPL];
#pragma unroll
    for (int u = 0; u < KPL; u++) {
      const int i = 64 * u + lane;
      const int64_t ic = i < k ? i : 0;
      pr[u] = i < k && p.vals_p[vb + ic * US];
      kr[u] = (uint64_t)p.vals_l[vb + ic * US] ^ 0x8000000000000000ULL;
    }
#pragma unroll
    for (int u = 0; u < KPL; u++) vm |= (uint64_t)pr[u] << u;
    m = wave_sum_int(__popcll(vm));
  } else {
    int nan = 0;
#pragma unroll
    for (int u = 0; u < KPL; u++) {
      const int i = 64 * u + lane;
      const double x = p.vals_d[vb + (int64_t)(i < k ? i : 0) * US];
      kr[u] = f2key(canon_nan(x));
      if (i < k) {
        vm |= 1ULL << u;
        nan += isnan(x) ? 1 : 0;
      }
    }
    m = k - wave_sum_int(nan);   // NaN keys sort above every number; ranks < m never reach them
  }
  const int fn = p.sel_fn;
  int r0, r1;
  double dif;
  raw_sel_ranks(fn, is_int, m, r0, r1, dif);
  uint64_t k0 = 0, k1 = 0;
  if (m > 0) {
    k0 = wave_radix_select_reg<KPL>(kr, vm, r0, W);
    k1 = k0;
    if (r1 >= 0) {
      int le = 0;
      uint64_t gt = ~0ULL;
#pragma unroll
      for (int u = 0; u < KPL; u++) {
        if (!((vm >> u) & 1ULL)) continue;
        if (kr[u] <= k0) le++;
        else gt = kr[u] < gt ? kr[u] : gt;
      }
      le = wave_sum_int(le);
      gt = wave_min_u64(gt);
      k1 = le > r1 ? k0 : gt;
    }
  }
  if (lane == 0) raw_sel_store(p, idx, is_int, fn, m, r1, dif, k0, k1);
}

// The order statistics near the top (p90 ... p999 of large groups; any rank of small ones):
// one WAVE per 64 consecutive union points of a strip, lane = point.  The operands of span i
// for those points are adjacent (k_raw_vals writes [span][RAW_STRIP points]), so every load
// instruction reads 512 contiguous bytes -- the per-point kernels above read one 8-byte operand
// per 4 KB line and lane, and wait on the texture path.  Each lane streams its point's k
// operands in chunks of 8 and keeps the T largest keys in registers, sorted descending (a
// compare-exchange chain per insertion, only for operands above the current T-th).  Ranks from
// the top below T (host-checked bound) are then read from the registers; the keys and the
// estimate are those of the selections above.
template <int T, int MODE>   // MODE 0: every point long, 1: every point double, 2: mixed
__device__ __forceinline__ void topk_stream(const RawParams& p, int64_t vb, int k, bool is_int, uint64_t (&b)[T],
                                            int& m) {
  constexpr int64_t US = RAW_STRIP;
  for (int i0 = 0; i0 < k; i0 += 8) {
    uint64_t x[8];
    uint32_t cm = 0;
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int i = i0 + u;
      const int64_t o = vb + (int64_t)(i < k ? i : k - 1) * US;
      bool ok;
      if (MODE == 0 || (MODE == 2 && is_int)) {
        ok = i < k && p.vals_p[o];
        x[u] = (uint64_t)p.vals_l[o] ^ 0x8000000000000000ULL;
      } else {
        const double d = p.vals_d[o];
        ok = i < k && !isnan(d);   // runDouble drops NaN operands
        x[u] = f2key(d);
      }
      m += ok ? 1 : 0;
      if (ok && x[u] > b[T - 1]) cm |= 1u << u;
    }
    // insertions, operand by operand where some lane holds a candidate (static register
    // indices: a dynamically indexed x[] went to scratch)
#pragma unroll
    for (int u = 0; u < 8; u++)
      if (__any((cm >> u) & 1u))
        if ((cm >> u) & 1u) topk_insert<T>(b, x[u]);
  }
}

template <int T>
__global__ __launch_bounds__(256) void k_raw_sel_top(RawParams p) {
  const int wv = threadIdx.x >> 6;
  const int lane = lane_id();
  constexpr int WPS = RAW_STRIP / 64;   // waves per strip
  const int64_t wid = (int64_t)blockIdx.x * 4 + wv;
  const int64_t sl = wid / WPS;
  if (sl >= p.n_strips) return;
  const int64_t j = (wid - sl * WPS) * 64 + lane;   // point of the strip
  const int64_t gi = p.strip_g[sl];
  const int64_t u0 = (int64_t)p.strip_t[sl] * RAW_STRIP + j;
  if (!__any(u0 < p.U[gi])) return;   // the strip's tail
  const bool live = u0 < p.U[gi];
  const int64_t idx = p.out_off[gi] + u0;
  const int64_t g = gi + p.g0;
  const int k = (int)(p.grp_ser[g + 1] - p.grp_ser[g]);
  const int64_t vb = p.vals_off[sl] + j;
  const bool is_int = live && p.out_int[idx] != 0;
  uint64_t b[T];
#pragma unroll
  for (int t = 0; t < T; t++) b[t] = 0;   // the smallest key: pads rank below every operand
  int m = 0;
  if (__all(is_int || !live)) topk_stream<T, 0>(p, vb, k, true, b, m);
  else if (__all(!is_int)) topk_stream<T, 1>(p, vb, k, false, b, m);
  else topk_stream<T, 2>(p, vb, k, is_int, b, m);
  if (!live) return;
  const int fn = p.sel_fn;
  int r0, r1;
  double dif;
  raw_sel_ranks(fn, is_int, m, r0, r1, dif);
  uint64_t k0 = 0, k1 = 0;
  if (m > 0) {
    const int i0 = m - 1 - r0, i1 = r1 >= 0 ? m - 1 - r1 : i0;   // positions from the top
    if (i0 >= T || i0 < 0 || i1 < 0) {
      set_err(p.err, TSDB_E_HIP);   // planning error: the rank is not among the kept keys
      return;
    }
    k0 = topk_at<T>(b, i0);
    k1 = topk_at<T>(b, i1);
  }
  raw_sel_store(p, idx, is_int, fn, m, r1, dif, k0, k1);
}

// T for k_raw_sel_top when every rank it can be asked for lies within T of the top (ksel.h
// raw_top_need over m <= k_max operands, both reducers); 0 = no.
int raw_sel_top_t(int fn, int64_t k_max) {
  if (opt_off(OPT_RAW_SEL_TOP)) return 0;   // option RAW_SEL_TOP = 0: the per-point kernels
  const int need = raw_top_need(fn, k_max, 32);
  return need <= 16 ? 16 : need <= 32 ? 32 : 0;
}

// k_max: the largest group of the batch; each wave stages k_max keys in LDS.
hipError_t launch_raw_sel(const RawParams& p, int64_t k_max, hipStream_t s) {
  if (p.n_strips == 0) return hipSuccess;
  if (const int T = raw_sel_top_t(p.sel_fn, k_max)) {
    const dim3 grid((unsigned)((p.n_strips * (RAW_STRIP / 64) + 3) / 4)), block(256);
    if (T == 16) hipLaunchKernelGGL(k_raw_sel_top<16>, grid, block, 0, s, p);
    else hipLaunchKernelGGL(k_raw_sel_top<32>, grid, block, 0, s, p);
    return hipGetLastError();
  }
  if (k_max <= 64 * 32 && !opt_off(OPT_RAW_SEL_REG)) {   // option RAW_SEL_REG = 0: the LDS-staged kernel
    const dim3 grid((unsigned)((p.n_strips * RAW_STRIP + SELW - 1) / SELW)), block(64 * SELW);
    if (k_max <= 64 * 8) hipLaunchKernelGGL(k_raw_sel_reg<8>, grid, block, 0, s, p);
    else if (k_max <= 64 * 16) hipLaunchKernelGGL(k_raw_sel_reg<16>, grid, block, 0, s, p);
    // 26 keys a lane (groups of <= 1664 spans, config 4's 1560) still fit 4 waves a SIMD; 32 take 3
    else if (k_max <= 64 * 26) hipLaunchKernelGGL(k_raw_sel_reg<26>, grid, block, 0, s, p);
    else hipLaunchKernelGGL(k_raw_sel_reg<32>, grid, block, 0, s, p);
    return hipGetLastError();
  }
  const int32_t kcap = (int32_t)std::max<int64_t>(1, std::min<int64_t>(k_max, RAW_SEL_LDS));
  const size_t lds = (size_t)kcap * 8 * SELW;
  hipError_t e = hipFuncSetAttribute((const void*)k_raw_sel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)((size_t)RAW_SEL_LDS * 8 * SELW));
  if (e != hipSuccess) return e;
  const int64_t pts = p.n_strips * RAW_STRIP;
  hipLaunchKernelGGL(k_raw_sel, dim3((unsigned)((pts + SELW - 1) / SELW)), dim3(64 * SELW), lds, s, p, kcap);
  return hipGetLastError();
}

}  // namespace tsdb
