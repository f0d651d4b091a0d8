// ksel.h -- order statistics shared by the percentile kernels (k_pct.hip) and the raw
// path's fused selection (k_raw_eval.hip): quantiles, order-preserving keys, and the ranks /
// estimate of PercentileAgg and Median (src/core/Aggregators.java:397-431, :657-708).
#pragma once
#include <algorithm>

#include "kcommon.h"

namespace tsdb {

__host__ __device__ inline double pct_quantile(int fn) {
  const int i = (fn - TSDB_AGG_P999) % 6;
  return i == 0 ? 99.9 : i == 1 ? 99.0 : i == 2 ? 95.0 : i == 3 ? 90.0 : i == 4 ? 75.0 : 50.0;
}

__device__ __forceinline__ uint64_t f2key(double x) {   // ascending double order == unsigned key order
  const uint64_t b = (uint64_t)__double_as_longlong(x);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ULL);
}
__device__ __forceinline__ double key2f(uint64_t k) {
  return __longlong_as_double((long long)((k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFULL) : ~k));
}

__device__ __forceinline__ int64_t sel_d2l(double d) {   // Java (long) of a double
  if (isnan(d)) return 0;
  if (d >= 9223372036854775807.0) return 0x7FFFFFFFFFFFFFFFLL;
  if (d <= -9223372036854775808.0) return (int64_t)0x8000000000000000ULL;
  return (int64_t)d;
}

// The ranks select_sorted reads among m values at a union point (r1 = -1: one value) and the
// interpolation weight: Median.runLong / runDouble sorted[m / 2]; PercentileAgg with its
// estimation type for runLong, LEGACY for runDouble (src/core/Aggregators.java:403-430, :675-706).
__host__ __device__ inline void raw_sel_ranks(int fn, bool is_int, int m, int& r0, int& r1, double& dif) {
  r0 = 0;
  r1 = -1;
  dif = 0.0;
  const int est = fn == TSDB_AGG_MEDIAN ? 0 : (is_int ? (fn - TSDB_AGG_P999) / 6 : 0);   // runDouble: LEGACY
  if (m > 1 && fn != TSDB_AGG_MEDIAN) {
    const double q = pct_quantile(fn) / 100.0;
    double pos;
    if (est == 1) {            // R_3
      pos = (q <= 0.5 / (double)m) ? 0.0 : rint((double)m * q);
    } else if (est == 2) {     // R_7
      pos = (q == 0.0) ? 0.0 : (q == 1.0 ? (double)m : 1.0 + (double)(m - 1) * q);
    } else {                   // LEGACY
      pos = (q == 0.0) ? 0.0 : (q == 1.0 ? (double)m : q * (double)(m + 1));
    }
    const double fpos = floor(pos);
    if (pos < 1) r0 = 0;
    else if (pos >= (double)m) r0 = m - 1;
    else { r0 = (int)fpos - 1; r1 = r0 + 1; dif = pos - fpos; }
  } else if (m > 0 && fn == TSDB_AGG_MEDIAN) {
    r0 = m / 2;
  }
}

// longValue / doubleValue of the selection (k0, k1: keys of ranks r0, r0 + 1) into out_bits.
__device__ __forceinline__ void raw_sel_store(const RawParams& p, int64_t idx, bool is_int, int fn, int m, int r1,
                                              double dif, uint64_t k0, uint64_t k1) {
  uint64_t bits;
  if (is_int) {
    const int64_t l0 = (int64_t)(k0 ^ 0x8000000000000000ULL), l1 = (int64_t)(k1 ^ 0x8000000000000000ULL);
    int64_t r;
    if (fn == TSDB_AGG_MEDIAN) {
      if (m == 0) set_err(p.err, TSDB_E_ILLEGAL_STATE);   // "Shouldn't be here without any data"
      r = l0;
    } else if (m == 0) {
      r = 0;                                               // (long) NaN
    } else if (r1 < 0) {
      r = sel_d2l((double)l0);
    } else {
      const double lower = (double)l0, upper = (double)l1;
      r = sel_d2l(lower + dif * (upper - lower));
    }
    bits = (uint64_t)r;
  } else {
    double r;
    if (m == 0) r = NAN;
    else if (r1 < 0) r = key2f(k0);
    else {
      const double lower = key2f(k0), upper = key2f(k1);
      r = lower + dif * (upper - lower);
    }
    if (isinf(r)) set_err(p.err, TSDB_E_ILLEGAL_STATE);   // doubleValue (:640-643)
    bits = (uint64_t)__double_as_longlong(r);
  }
  p.out_bits[idx] = bits;
}

// 64-bit shuffles and the wave minimum of 64-bit keys
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint64_t o = shfl_u64(v, lane_id() ^ d);
    v = o < v ? o : v;
  }
  return v;
}

// The T largest keys seen, sorted descending (k_raw_sel_top, k_raw_top): insertion is a
// compare-exchange chain; inserting key 0 (below every operand's key) changes nothing.
template <int T>
__device__ __forceinline__ void topk_insert(uint64_t (&b)[T], uint64_t c) {
#pragma unroll
  for (int t = 0; t < T; t++) {
    const uint64_t hi = b[t] > c ? b[t] : c;
    c = b[t] > c ? c : b[t];
    b[t] = hi;
  }
}

// b[i] for a lane-varying i, as masks (a select chain is turned back into a dynamically
// indexed array, which lives in scratch)
template <int T>
__device__ __forceinline__ uint64_t topk_at(const uint64_t (&b)[T], int i) {
  uint64_t r = 0;
#pragma unroll
  for (int t = 0; t < T; t++) r |= b[t] & (0ULL - (uint64_t)(i == t));
  return r;
}

// The largest number of keys from the top a point of at most k_max operands needs for
// function fn (positions m - 1 - r0 and m - 1 - r1 of raw_sel_ranks, both reducers), capped
// at cap + 1 (more than any register buffer holds)
inline int raw_top_need(int fn, int64_t k_max, int cap) {
  int need = 0;
  for (int64_t m = 1; m <= k_max && need <= cap; m++) {
    for (int is_int = 0; is_int < 2; is_int++) {
      int r0, r1;
      double dif;
      raw_sel_ranks(fn, is_int != 0, (int)m, r0, r1, dif);
      need = std::max(need, (int)(m - r0));   // position m - 1 - r0 (r1 = r0 + 1 lies above it)
    }
  }
  return need;
}

}  // namespace tsdb
