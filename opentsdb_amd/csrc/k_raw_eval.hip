// k_raw_eval.hip -- evaluation kernel of the raw path, instantiated for ONE group
// aggregator class (GA_ID, set by the Makefile) so each aggregator keeps only its own
// state in registers.
//
// One wave per strip of RAW_STRIP = 64 x RAW_W union points of one group.  Lane l owns
// the union points ua + 64 w + l (w < RAW_W) and keeps one aggregator state per point.
// Spans are visited sequentially in SpanGroup index order (the order in which
// AggregationIterator.nextDoubleValue / nextLongValue hand values to the aggregator,
// src/core/AggregationIterator.java:667-797), so every aggregator -- float sums included --
// sees the reference's operand order.  Per (strip, span):
//   c = cursor[strip][span]  counted points of the span with rank < ua
//   m = cursor[strip+1][span] - c  the span's points inside the strip
// m == 0 (the common case for groups of many spans): one segment for the whole strip;
// its two end points are wave-uniform loads and every window is a plain LERP.
// m > 0: the span's in-strip ranks are OR-ed into RAW_W 64-bit window masks in LDS; a
// lane's segment is cursor + popcount(mask bits at or below its position).
#include "ksel.h"

#ifndef GA_ID
#error "compile with -DGA_ID=<group aggregator class>"
#endif

namespace tsdb {

// Java long arithmetic (wrapping) and the LERP of nextLongValue (:682-729):
//   y0 + (x - x0) * (y1 - y0) / (x1 - x0)   with truncating division
__device__ __forceinline__ int64_t jdiv_pos(int64_t num, int64_t den) {
  // den > 0.  |num| < 2^53: double quotient, corrected to the exact truncated one.
  const uint64_t an = num < 0 ? (uint64_t)0 - (uint64_t)num : (uint64_t)num;
  if (an < (1ULL << 53) && den < (1LL << 53)) {
    int64_t q = (int64_t)((double)num / (double)den);
    const int64_t r = num - q * den;
    if (num >= 0) {
      if (r < 0) q--;
      else if (r >= den) q++;
    } else {
      if (r > 0) q++;
      else if (r <= -den) q--;
    }
    return q;
  }
  return num / den;
}

__device__ __forceinline__ int64_t jlerp(int interp, int64_t x, int64_t x0, int64_t y0, int64_t x1, int64_t y1) {
  switch (interp) {
    case TSDB_INTERP_LERP: {
      const uint64_t prod = (uint64_t)(x - x0) * ((uint64_t)y1 - (uint64_t)y0);
      return (int64_t)((uint64_t)y0 + (uint64_t)jdiv_pos((int64_t)prod, x1 - x0));
    }
    case TSDB_INTERP_ZIM: return 0;
    case TSDB_INTERP_MAX: return 0x7FFFFFFFFFFFFFFFLL;
    case TSDB_INTERP_MIN: return (int64_t)0x8000000000000000ULL;
    default: return y0;
  }
}

// The long LERP of one span window shared by a whole strip (k_raw_eval's m == 0 case: x0, y0,
// x1, y1 wave-uniform, x0 < x < x1 at every lane).  When x1 - x0 < 2^32 and |y1 - y0| (x1 - x0)
// < 2^51 the wrapping product cannot wrap and every quantity is an exact double: the product is
// one multiply, the quotient one multiply by the window's reciprocal (off by at most one), an
// FMA gives its exact remainder and a compare corrects it -- ~15 instructions a point instead of
// the general path's 64-bit multiplies, IEEE division and conversions.  Same result bit for bit.
struct LerpW {
  double dyd, dend, rd;
  int64_t x0, y0;
  bool pos, ok;
};
__device__ __forceinline__ LerpW lerpw_init(int interp, bool uns, int64_t x0, int64_t y0, int64_t x1, int64_t y1) {
  LerpW L;
  const int64_t den = x1 - x0;
  const int64_t dy = (int64_t)((uint64_t)y1 - (uint64_t)y0);
  const uint64_t ady = dy < 0 ? (uint64_t)0 - (uint64_t)dy : (uint64_t)dy;
  L.ok = interp == TSDB_INTERP_LERP && !uns && den > 0 && den < (1LL << 32) && ady < (1ULL << 51) &&
         (double)ady * (double)den < 1125899906842624.0;   // 2^50 on the rounded product: the exact one < 2^51
  L.dyd = (double)dy;
  L.dend = (double)den;
  L.rd = 1.0 / L.dend;
  L.x0 = x0;
  L.y0 = y0;
  L.pos = dy >= 0;
  return L;
}
__device__ __forceinline__ int64_t lerpw_eval(const LerpW& L, int64_t x) {
  const double nd = (double)(uint32_t)(x - L.x0) * L.dyd;   // exact: |nd| < 2^51
  double q = trunc(nd * L.rd);
  const double r = fma(-q, L.dend, nd);                      // exact remainder of q
  if (L.pos) q += (r >= L.dend ? 1.0 : 0.0) - (r < 0.0 ? 1.0 : 0.0);
  else q += (r > 0.0 ? 1.0 : 0.0) - (r <= -L.dend ? 1.0 : 0.0);
  // |q| < 2^51: its integer from the mantissa of q + 1.5 * 2^52
  const int64_t qi = (int64_t)__double_as_longlong(q + 6755399441055744.0) - 0x4338000000000000LL;
  return (int64_t)((uint64_t)L.y0 + (uint64_t)qi);
}

// nextDoubleValue (:735-797), evaluated with exactly Java's association and no FMA
__device__ __forceinline__ double dlerp(int interp, int64_t x, int64_t x0, double y0, int64_t x1, double y1) {
  switch (interp) {
    case TSDB_INTERP_LERP: return y0 + (double)(x - x0) * (y1 - y0) / (double)(x1 - x0);
    case TSDB_INTERP_ZIM: return 0.0;
    case TSDB_INTERP_MAX: return DBL_MAX;
    case TSDB_INTERP_MIN: return 4.9e-324;   // Double.MIN_VALUE
    default: return y0;
  }
}

// nextLongValue / nextDoubleValue of a span that does not own the union point (:682-797): y0
// at x == x0, y1 at x == x1, else the interpolation.  With points in time order x0 < x < x1
// always holds; over cells with unsorted datapoints (RawParams.uns) x may sit on either end of
// the window and x1 - x0 may be <= 0 (Java long division truncates; / 0 throws
// ArithmeticException, reported through dz where the long result is the one used).
__device__ __forceinline__ int64_t jlerp_u(int interp, int64_t x, int64_t x0, int64_t y0, int64_t x1, int64_t y1,
                                           bool& dz) {
  if (x == x0) return y0;
  if (x == x1) return y1;
  if (interp != TSDB_INTERP_LERP || x1 > x0) return jlerp(interp, x, x0, y0, x1, y1);
  if (x1 == x0) { dz = true; return 0; }
  const int64_t num = (int64_t)((uint64_t)(x - x0) * ((uint64_t)y1 - (uint64_t)y0));
  const int64_t den = x1 - x0;
  const int64_t q = (num == INT64_MIN && den == -1) ? INT64_MIN : num / den;
  return (int64_t)((uint64_t)y0 + (uint64_t)q);
}
__device__ __forceinline__ double dlerp_u(int interp, int64_t x, int64_t x0, double y0, int64_t x1, double y1) {
  if (x == x0) return y0;
  if (x == x1) return y1;
  return dlerp(interp, x, x0, y0, x1, y1);
}

__device__ __forceinline__ int64_t jd2l(double d) {   // Java (long) of a double
  if (isnan(d)) return 0;
  if (d >= 9223372036854775807.0) return 0x7FFFFFFFFFFFFFFFLL;
  if (d <= -9223372036854775808.0) return (int64_t)0x8000000000000000ULL;
  return (int64_t)d;
}

// Aggregator.runLong / runDouble as a stream over the spans' values in index order
// (src/core/Aggregators.java: Sum :237-259, SquareSum :269-293, Min :303-327,
// Max :337-361, Avg :371-393, None :445-460, Multiply :470-485, StdDev :504-569,
// Diff :582-617, Count :626-645, First :815-829, Last :837-851).
struct RAcc {
  double da, db;      // runDouble
  int64_t la;         // runLong
  double lm, lM2;     // runLong dev (Welford in double)
  uint64_t lfirst;    // runLong diff
  int32_t dn, ln;
  int32_t dst, lst;
  bool bad;           // None: more than one value
};

template <int GA>
__device__ __forceinline__ void racc_init(RAcc& a) {
  a.da = (GA == GA_MIN) ? INFINITY : (GA == GA_MAX ? -INFINITY : 0.0);
  a.db = 0.0;
  a.la = 0;
  a.lm = 0.0;
  a.lM2 = 0.0;
  a.lfirst = 0;
  a.dn = 0;
  a.ln = 0;
  a.dst = 0;
  a.lst = 0;
  a.bad = false;
}

template <int GA>
__device__ __forceinline__ void racc_double(RAcc& a, double x) {
  if constexpr (GA == GA_SUM || GA == GA_AVG) { if (!isnan(x)) { a.da += x; a.dn++; } }
  else if constexpr (GA == GA_SQUARESUM) { if (!isnan(x)) { a.da += x * x; a.dn++; } }
  else if constexpr (GA == GA_COUNT) { if (!isnan(x)) a.dn++; }
  else if constexpr (GA == GA_MIN) { if (!isnan(x) && x < a.da) a.da = x; }
  else if constexpr (GA == GA_MAX) { if (!isnan(x) && x > a.da) a.da = x; }
  else if constexpr (GA == GA_DEV) {
    if (a.dst == 0) {
      if (!isnan(x)) { a.da = x; a.dst = 1; a.dn = 2; }
    } else if (!isnan(x)) {
      const double nm = a.da + (x - a.da) / (double)a.dn;
      a.db += (x - a.da) * (x - nm);
      a.da = nm;
      a.dn++;
    }
  } else if constexpr (GA == GA_DIFF) {
    if (a.dst == 0) { if (!isnan(x)) { a.da = x; a.dst = 1; } }
    else { a.db = x; a.dst = 2; }
  } else if constexpr (GA == GA_FIRST) { if (a.dst == 0) { a.da = x; a.dst = 1; } }
  else if constexpr (GA == GA_LAST) { a.da = x; }
  else if constexpr (GA == GA_MULT) { a.da = a.dst ? a.da * x : x; a.dst = 1; }
  else if constexpr (GA == GA_NONE) { if (a.dst) a.bad = true; a.da = x; a.dst = 1; }
}

template <int GA>
__device__ __forceinline__ double racc_double_final(const RAcc& a) {
  if constexpr (GA == GA_SUM || GA == GA_SQUARESUM) return a.dn == 0 ? (double)NAN : a.da;
  else if constexpr (GA == GA_AVG) return a.dn == 0 ? (double)NAN : a.da / (double)a.dn;
  else if constexpr (GA == GA_COUNT) return (double)a.dn;
  else if constexpr (GA == GA_MIN) return a.da == INFINITY ? (double)NAN : a.da;
  else if constexpr (GA == GA_MAX) return a.da == -INFINITY ? (double)NAN : a.da;
  else if constexpr (GA == GA_DEV) return a.dst == 0 ? (double)NAN : (a.dn == 2 ? 0.0 : sqrt(a.db / (double)(a.dn - 1)));
  else if constexpr (GA == GA_DIFF) return a.dst == 0 ? (double)NAN : (a.dst == 1 ? 0.0 : a.db - a.da);
  else return a.da;
}

template <int GA>
__device__ __forceinline__ void racc_long(RAcc& a, int64_t x) {
  const uint64_t ux = (uint64_t)x;
  if constexpr (GA == GA_SUM) a.la = (int64_t)((uint64_t)a.la + ux);
  else if constexpr (GA == GA_AVG) { a.la = (int64_t)((uint64_t)a.la + ux); a.ln++; }
  else if constexpr (GA == GA_SQUARESUM) a.la = (int64_t)((uint64_t)a.la + ux * ux);
  else if constexpr (GA == GA_COUNT) a.ln++;
  else if constexpr (GA == GA_MIN) { if (a.lst == 0 || x < a.la) a.la = x; a.lst = 1; }
  else if constexpr (GA == GA_MAX) { if (a.lst == 0 || x > a.la) a.la = x; a.lst = 1; }
  else if constexpr (GA == GA_DEV) {
    if (a.lst == 0) { a.lm = (double)x; a.lst = 1; a.ln = 2; }
    else {
      const double xd = (double)x;
      const double nm = a.lm + (xd - a.lm) / (double)a.ln;
      a.lM2 += (xd - a.lm) * (xd - nm);
      a.lm = nm;
      a.ln++;
      a.lst = 2;
    }
  } else if constexpr (GA == GA_DIFF) {
    if (a.lst == 0) { a.lfirst = ux; a.lst = 1; }
    else { a.la = x; a.lst = 2; }
  } else if constexpr (GA == GA_FIRST) { if (a.lst == 0) { a.la = x; a.lst = 1; } }
  else if constexpr (GA == GA_LAST) a.la = x;
  else if constexpr (GA == GA_MULT) { a.la = a.lst ? (int64_t)((uint64_t)a.la * ux) : x; a.lst = 1; }
  else if constexpr (GA == GA_NONE) { if (a.lst) a.bad = true; a.la = x; a.lst = 1; }
}

template <int GA>
__device__ __forceinline__ int64_t racc_long_final(const RAcc& a) {
  if constexpr (GA == GA_AVG) return a.ln == 0 ? 0 : a.la / (int64_t)a.ln;
  else if constexpr (GA == GA_COUNT) return a.ln;
  else if constexpr (GA == GA_DEV) return a.lst < 2 ? 0 : jd2l(sqrt(a.lM2 / (double)(a.ln - 1)));
  else if constexpr (GA == GA_DIFF) return a.lst < 2 ? 0 : (int64_t)((uint64_t)a.la - a.lfirst);
  else return a.la;
}

// One value (exact or interpolated) of a span at union time x.
template <int GA, bool DL, bool DD>
__device__ __forceinline__ void feed(RAcc& acc, int interp, bool own, int64_t x, const RawPt& a, const RawPt& b,
                                     bool uns, bool& dz) {
  if (own) {
    if (DL) racc_long<GA>(acc, (int64_t)a.bits);
    if (DD) racc_double<GA>(acc, pt_double(a.tsf, a.bits));
  } else if (uns) {
    const int64_t x0 = a.tsf & RAW_TIME_MASK, x1 = b.tsf & RAW_TIME_MASK;
    if (DL) racc_long<GA>(acc, jlerp_u(interp, x, x0, (int64_t)a.bits, x1, (int64_t)b.bits, dz));
    if (DD) racc_double<GA>(acc, dlerp_u(interp, x, x0, pt_double(a.tsf, a.bits), x1, pt_double(b.tsf, b.bits)));
  } else {
    const int64_t x0 = a.tsf & RAW_TIME_MASK, x1 = b.tsf & RAW_TIME_MASK;
    if (DL) racc_long<GA>(acc, jlerp(interp, x, x0, (int64_t)a.bits, x1, (int64_t)b.bits));
    if (DD) racc_double<GA>(acc, dlerp(interp, x, x0, pt_double(a.tsf, a.bits), x1, pt_double(b.tsf, b.bits)));
  }
}

template <int GA, bool DL, bool DD, bool RATE>
__global__ __launch_bounds__(64) void k_raw_eval(RawParams p) {
  __shared__ uint64_t wmask[RAW_W];
  const int lane = lane_id();
  const int64_t strip = blockIdx.x;
  if (strip >= p.n_strips) return;
  const int64_t gi = p.strip_g[strip];
  const int64_t t = p.strip_t[strip];
  const int64_t g = gi + p.g0;
  const int64_t U = p.U[gi];
  const int64_t ns = (U + RAW_STRIP - 1) / RAW_STRIP;
  const int64_t ua = t * RAW_STRIP;
  const int64_t ub = min(U, ua + (int64_t)RAW_STRIP);
  const int64_t sb = p.grp_ser[g];
  const int k = (int)(p.grp_ser[g + 1] - sb);
  constexpr int first = RATE ? 1 : 0;
  const int interp = p.interp;
  const int32_t* crow = p.cur + p.cur_off[gi] + t * k;
  const int32_t* cnext = (t + 1 < ns) ? crow + k : nullptr;
  const int64_t obase = p.out_off[gi];
  const uint64_t below = (lane == 63) ? ~0ULL : ((2ULL << lane) - 1ULL);

  int64_t x[RAW_W];
  RAcc acc[RAW_W];
  uint32_t flt = 0;   // bit w: some slot at union point w holds a double (isInteger, :612-625)
  uint32_t dzm = 0;   // bit w: a long LERP at union point w divided by zero (unsorted cells)
  const bool uns = p.uns != 0;
#pragma unroll
  for (int w = 0; w < RAW_W; w++) {
    const int64_t u = ua + 64 * w + lane;
    x[w] = (u < ub) ? p.out_ts[obase + u] : 0;
    racc_init<GA>(acc[w]);
  }

  for (int i = 0; i < k; i++) {
    const int64_t s = sb + i;
    const int n = p.sp_n[s];
    if (n < (RATE ? 2 : 1)) continue;   // empty span; rate: endReached with nothing current (:448-459)
    const int nc = n - first;
    const RawPt* pts = p.pts + p.sp_off[s];
    const int c = crow[i];
    const int m = (cnext ? cnext[i] : nc) - c;
    if (m == 0) {
      // one segment for the whole strip (wave-uniform)
      if (RATE) {
        if (c == nc) continue;   // ended after its last rate (the zeroing, :521-526)
        const double y = __longlong_as_double((long long)pts[c].bits);   // step / PREV (:744-753)
#pragma unroll
        for (int w = 0; w < RAW_W; w++) racc_double<GA>(acc[w], y);
      } else {
        if (c == 0) {            // not started: its next slot still counts for isInteger
          if (pts[0].tsf & RAW_FLOAT) flt = (1u << RAW_W) - 1;
          continue;
        }
        if (c == n) continue;    // ended
        const RawPt a = pts[c - 1], b = pts[c];
        if ((a.tsf | b.tsf) & RAW_FLOAT) flt = (1u << RAW_W) - 1;
        if (DL && p.lerp_fast) {
          const int64_t x0 = a.tsf & RAW_TIME_MASK, x1 = b.tsf & RAW_TIME_MASK;
          const LerpW L = lerpw_init(interp, uns, x0, (int64_t)a.bits, x1, (int64_t)b.bits);
          if (L.ok) {
#pragma unroll
            for (int w = 0; w < RAW_W; w++) {
              racc_long<GA>(acc[w], lerpw_eval(L, x[w]));
              if (DD) racc_double<GA>(acc[w], dlerp(interp, x[w], x0, pt_double(a.tsf, a.bits), x1, pt_double(b.tsf, b.bits)));
            }
            continue;
          }
        }
#pragma unroll
        for (int w = 0; w < RAW_W; w++) {
          bool dz = false;
          feed<GA, DL, DD>(acc[w], interp, false, x[w], a, b, uns, dz);
          if (dz) dzm |= 1u << w;
        }
      }
      continue;
    }
    // the span has points inside the strip: window masks of their ranks
    if (lane < RAW_W) wmask[lane] = 0;
    WAVE_SYNC();
    const int32_t* rk = p.rank + p.sp_off[s] + first + c;
    for (int l = lane; l < m; l += 64) {
      const int64_t o = rk[l] - ua;
      __hip_atomic_fetch_or(&wmask[o >> 6], 1ULL << (o & 63), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    WAVE_SYNC();
    int tb = 0;
#pragma unroll
    for (int w = 0; w < RAW_W; w++) {
      const uint64_t M = wmask[w];
      const int cnt = c + tb + __popcll(M & below);   // counted points with rank <= u
      const bool own = (M >> lane) & 1ULL;
      tb += __popcll(M);
      if (RATE) {
        if (cnt == nc && !own) continue;
        racc_double<GA>(acc[w], __longlong_as_double((long long)pts[cnt].bits));
      } else {
        if (cnt == 0) {
          if (pts[0].tsf & RAW_FLOAT) flt |= 1u << w;
          continue;
        }
        const int j = cnt - 1;
        const RawPt a = pts[j];
        if (j == n - 1) {
          if (!own) continue;
          if (a.tsf & RAW_FLOAT) flt |= 1u << w;
          if (DL) racc_long<GA>(acc[w], (int64_t)a.bits);
          if (DD) racc_double<GA>(acc[w], pt_double(a.tsf, a.bits));
          continue;
        }
        const RawPt b = pts[j + 1];
        if ((a.tsf | b.tsf) & RAW_FLOAT) flt |= 1u << w;
        bool dz = false;
        feed<GA, DL, DD>(acc[w], interp, own, x[w], a, b, uns, dz);
        if (dz) dzm |= 1u << w;
      }
    }
    WAVE_SYNC();
  }

#pragma unroll
  for (int w = 0; w < RAW_W; w++) {
    const int64_t u = ua + 64 * w + lane;
    if (u >= ub) continue;
    const bool is_int = !RATE && !((flt >> w) & 1);
    uint64_t bits = 0;
    if (is_int) {
      if (DL) bits = (uint64_t)racc_long_final<GA>(acc[w]);
      else set_err(p.err, TSDB_E_HIP);   // planning error: integer output without the long path
    } else {
      double r = 0.0;
      if (DD) r = racc_double_final<GA>(acc[w]);
      else set_err(p.err, TSDB_E_HIP);
      if (isinf(r)) set_err(p.err, TSDB_E_ILLEGAL_STATE);   // doubleValue (:640-643)
      bits = (uint64_t)__double_as_longlong(r);
    }
    if (acc[w].bad) set_err(p.err, TSDB_E_ILLEGAL_DATA);   // None: "More than one value" (:454-460)
    if (is_int && ((dzm >> w) & 1)) set_err(p.err, TSDB_E_ILLEGAL_STATE);   // ArithmeticException: / by zero
    p.out_bits[obase + u] = bits;
    p.out_int[obase + u] = is_int ? 1 : 0;
  }
}

template <>
hipError_t launch_raw_eval_inst<GA_ID>(const RawParams& p, hipStream_t s) {
  const dim3 grid((unsigned)p.n_strips), block(64);
  if (p.rate) hipLaunchKernelGGL((k_raw_eval<GA_ID, false, true, true>), grid, block, 0, s, p);
  else if (p.do_long && p.do_double) hipLaunchKernelGGL((k_raw_eval<GA_ID, true, true, false>), grid, block, 0, s, p);
  else if (p.do_long) hipLaunchKernelGGL((k_raw_eval<GA_ID, true, false, false>), grid, block, 0, s, p);
  else hipLaunchKernelGGL((k_raw_eval<GA_ID, false, true, false>), grid, block, 0, s, p);
  return hipGetLastError();
}

#if GA_ID == 11
// Percentile / median as the group-by aggregator without downsampling (PercentileAgg and
// Median collect the span values of each union point, src/core/Aggregators.java:397-431,
// :657-708): the traversal of k_raw_eval, but each span's operand (exact or interpolated,
// long and/or double as nextLongValue / nextDoubleValue produce it) is stored at
// vals_off[strip] + i * RAW_STRIP + (u - ua) instead of being folded; k_raw_sel (k_pct.hip)
// selects.
template <bool DL, bool DD, bool RATE>
__global__ __launch_bounds__(64) void k_raw_vals(RawParams p) {
  __shared__ uint64_t wmask[RAW_W];
  const int lane = lane_id();
  const int64_t strip = blockIdx.x;
  if (strip >= p.n_strips) return;
  // blockIdx.y: a run of RAW_SEL_SPANS spans of the strip (the spans are independent here)
  const int64_t gi = p.strip_g[strip];
  const int64_t t = p.strip_t[strip];
  const int64_t g = gi + p.g0;
  const int64_t U = p.U[gi];
  const int64_t ns = (U + RAW_STRIP - 1) / RAW_STRIP;
  const int64_t ua = t * RAW_STRIP;
  const int64_t ub = min(U, ua + (int64_t)RAW_STRIP);
  const int64_t sb = p.grp_ser[g];
  const int k = (int)(p.grp_ser[g + 1] - sb);
  const int i0 = (int)blockIdx.y * RAW_SEL_SPANS;
  if (i0 >= k) return;
  const int i1 = min(k, i0 + RAW_SEL_SPANS);
  constexpr int first = RATE ? 1 : 0;
  const int interp = p.interp;
  const int32_t* crow = p.cur + p.cur_off[gi] + t * k;
  const int32_t* cnext = (t + 1 < ns) ? crow + k : nullptr;
  const int64_t obase = p.out_off[gi];
  const int64_t vbase = p.vals_off[strip];
  const uint64_t below = (lane == 63) ? ~0ULL : ((2ULL << lane) - 1ULL);

  int64_t x[RAW_W];
  bool in[RAW_W];
  uint32_t flt = 0;
  const bool uns = p.uns != 0;
#pragma unroll
  for (int w = 0; w < RAW_W; w++) {
    const int64_t u = ua + 64 * w + lane;
    in[w] = u < ub;
    x[w] = in[w] ? p.out_ts[obase + u] : 0;
  }
  auto put_l = [&](int i, int w, int64_t v) {
    if (!in[w]) return;
    const int64_t o = vbase + (int64_t)i * RAW_STRIP + 64 * w + lane;
    p.vals_l[o] = v;
    p.vals_p[o] = 1;
  };
  auto put_d = [&](int i, int w, double v) {
    if (!in[w]) return;
    p.vals_d[vbase + (int64_t)i * RAW_STRIP + 64 * w + lane] = v;
  };
  // a non-owning span's operands (see jlerp_u); a long division by zero marks the point
  auto put_lerp = [&](int i, int w, const RawPt& a, const RawPt& b) {
    const int64_t x0 = a.tsf & RAW_TIME_MASK, x1 = b.tsf & RAW_TIME_MASK;
    if (uns) {
      bool dz = false;
      if (DL) put_l(i, w, jlerp_u(interp, x[w], x0, (int64_t)a.bits, x1, (int64_t)b.bits, dz));
      if (DD) put_d(i, w, dlerp_u(interp, x[w], x0, pt_double(a.tsf, a.bits), x1, pt_double(b.tsf, b.bits)));
      if (dz && in[w]) p.dz[obase + ua + 64 * w + lane] = 1;
    } else {
      if (DL) put_l(i, w, jlerp(interp, x[w], x0, (int64_t)a.bits, x1, (int64_t)b.bits));
      if (DD) put_d(i, w, dlerp(interp, x[w], x0, pt_double(a.tsf, a.bits), x1, pt_double(b.tsf, b.bits)));
    }
  };

  for (int i = i0; i < i1; i++) {
    const int64_t s = sb + i;
    const int n = p.sp_n[s];
    if (n < (RATE ? 2 : 1)) continue;
    const int nc = n - first;
    const RawPt* pts = p.pts + p.sp_off[s];
    const int c = crow[i];
    const int m = (cnext ? cnext[i] : nc) - c;
    if (m == 0) {
      if (RATE) {
        if (c == nc) continue;
        const double y = __longlong_as_double((long long)pts[c].bits);
#pragma unroll
        for (int w = 0; w < RAW_W; w++) put_d(i, w, y);
      } else {
        if (c == 0) {
          if (pts[0].tsf & RAW_FLOAT) flt = (1u << RAW_W) - 1;
          continue;
        }
        if (c == n) continue;
        const RawPt a = pts[c - 1], b = pts[c];
        if ((a.tsf | b.tsf) & RAW_FLOAT) flt = (1u << RAW_W) - 1;
        if (DL && p.lerp_fast) {   // the strip-wide window (lerpw_*, as in k_raw_eval)
          const int64_t x0 = a.tsf & RAW_TIME_MASK, x1 = b.tsf & RAW_TIME_MASK;
          const LerpW L = lerpw_init(interp, uns, x0, (int64_t)a.bits, x1, (int64_t)b.bits);
          if (L.ok) {
#pragma unroll
            for (int w = 0; w < RAW_W; w++) {
              put_l(i, w, lerpw_eval(L, x[w]));
              if (DD) put_d(i, w, dlerp(interp, x[w], x0, pt_double(a.tsf, a.bits), x1, pt_double(b.tsf, b.bits)));
            }
            continue;
          }
        }
#pragma unroll
        for (int w = 0; w < RAW_W; w++) put_lerp(i, w, a, b);
      }
      continue;
    }
    if (lane < RAW_W) wmask[lane] = 0;
    WAVE_SYNC();
    const int32_t* rk = p.rank + p.sp_off[s] + first + c;
    for (int l = lane; l < m; l += 64) {
      const int64_t o = rk[l] - ua;
      __hip_atomic_fetch_or(&wmask[o >> 6], 1ULL << (o & 63), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    WAVE_SYNC();
    int tb = 0;
#pragma unroll
    for (int w = 0; w < RAW_W; w++) {
      const uint64_t M = wmask[w];
      const int cnt = c + tb + __popcll(M & below);
      const bool own = (M >> lane) & 1ULL;
      tb += __popcll(M);
      if (RATE) {
        if (cnt == nc && !own) continue;
        put_d(i, w, __longlong_as_double((long long)pts[cnt].bits));
      } else {
        if (cnt == 0) {
          if (pts[0].tsf & RAW_FLOAT) flt |= 1u << w;
          continue;
        }
        const int j = cnt - 1;
        const RawPt a = pts[j];
        if (j == n - 1 && !own) continue;
        if (j == n - 1 || own) {
          if (a.tsf & RAW_FLOAT) flt |= 1u << w;
          if (j < n - 1 && (pts[j + 1].tsf & RAW_FLOAT)) flt |= 1u << w;
          if (DL) put_l(i, w, (int64_t)a.bits);
          if (DD) put_d(i, w, pt_double(a.tsf, a.bits));
          continue;
        }
        const RawPt b = pts[j + 1];
        if ((a.tsf | b.tsf) & RAW_FLOAT) flt |= 1u << w;
        put_lerp(i, w, a, b);
      }
    }
    WAVE_SYNC();
  }

#pragma unroll
  for (int w = 0; w < RAW_W; w++) {
    const int64_t u = ua + 64 * w + lane;
    if (u >= ub) continue;
    // out_int starts at 1; any run of spans that sees a double at the point clears it
    if (RATE || ((flt >> w) & 1)) p.out_int[obase + u] = 0;
  }
}

// Percentile / median group-by without downsampling, fused (config 4 p99): k_raw_vals'
// traversal, but each span operand goes into its union point's T largest keys, held in
// registers (ksel.h topk_insert), instead of the operand arrays -- 9 to 17 B a (span, point),
// 5e10 operands in config 4, written by k_raw_vals and read back by k_raw_sel_top.  A wave
// covers RW of a strip's RAW_W windows (64 x RW points; lane l: points ua + 64 (q RW + w) + l),
// so one strip is RAW_W / RW waves; a span's in-strip ranks still come from the whole strip's
// window masks.  Valid when every rank the query can ask for lies within T of the top
// (host: raw_top_need); keys, counts, ranks and estimate are k_raw_sel_top's (runLong keys
// for long points, runDouble's NaN-free double keys otherwise), so results are bit-identical.
// MODE 0: long operands only, 1: double only (rate too), 2: both (a key list each).
template <int T, int RW, int MODE, bool RATE>
__global__ __launch_bounds__(64) void k_raw_top(RawParams p) {
  constexpr bool DL = MODE != 1, DD = MODE != 0;
  constexpr int NL = DL ? T : 1, ND = DD ? T : 1;
  static_assert(RAW_W % RW == 0, "a strip is a whole number of waves");
  __shared__ uint64_t wmask[RAW_W];
  const int lane = lane_id();
  constexpr int SUB = RAW_W / RW;
  const int64_t strip = blockIdx.x / SUB;
  if (strip >= p.n_strips) return;
  const int q = (int)(blockIdx.x % SUB);
  const int64_t gi = p.strip_g[strip];
  const int64_t t = p.strip_t[strip];
  const int64_t g = gi + p.g0;
  const int64_t U = p.U[gi];
  const int64_t ns = (U + RAW_STRIP - 1) / RAW_STRIP;
  const int64_t ua = t * RAW_STRIP;
  const int64_t ub = min(U, ua + (int64_t)RAW_STRIP);
  const int64_t uq = ua + 64 * q * RW;   // this wave's first point
  if (uq >= ub) return;
  const int64_t sb = p.grp_ser[g];
  const int k = (int)(p.grp_ser[g + 1] - sb);
  constexpr int first = RATE ? 1 : 0;
  const int interp = p.interp;
  const int32_t* crow = p.cur + p.cur_off[gi] + t * k;
  const int32_t* cnext = (t + 1 < ns) ? crow + k : nullptr;
  const int64_t obase = p.out_off[gi];
  const uint64_t below = (lane == 63) ? ~0ULL : ((2ULL << lane) - 1ULL);
  const bool uns = p.uns != 0;

  int64_t x[RW];
  bool in[RW];
  uint64_t bl[RW][NL], bd[RW][ND];
  int ml[RW], md[RW];
  uint32_t flt = 0, dzm = 0;
#pragma unroll
  for (int w = 0; w < RW; w++) {
    const int64_t u = uq + 64 * w + lane;
    in[w] = u < ub;
    x[w] = in[w] ? p.out_ts[obase + u] : 0;
    ml[w] = md[w] = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) bl[w][j] = 0;
#pragma unroll
    for (int j = 0; j < ND; j++) bd[w][j] = 0;
  }
  // one operand of span i at window w (every lane: a lane without one passes ok = false)
  // thr: the wave's smallest T-th key over its points (wave-uniform, refreshed after an
  // insertion): a span whose operands all lie below it cannot enter any point's top T
  uint64_t thr = 0;
  auto refresh = [&]() {
    uint64_t t = ~0ULL;
#pragma unroll
    for (int w = 0; w < RW; w++) {
      if (DL && in[w]) t = min(t, bl[w][NL - 1]);
      if (DD && in[w]) t = min(t, bd[w][ND - 1]);
    }
    thr = wave_min_u64(t);
  };
  auto put_l = [&](int w, int64_t v, bool ok) {
    if constexpr (DL) {
      ok = ok && in[w];
      const uint64_t key = (uint64_t)v ^ 0x8000000000000000ULL;
      const bool cand = ok && key > bl[w][NL - 1];
      ml[w] += ok ? 1 : 0;
      if (__any(cand)) {
        topk_insert<NL>(bl[w], cand ? key : 0);
        refresh();
      }
    }
  };
  auto put_d = [&](int w, double v, bool ok) {
    if constexpr (DD) {
      ok = ok && in[w] && !isnan(v);   // runDouble drops NaN operands
      const uint64_t key = f2key(v);
      const bool cand = ok && key > bd[w][ND - 1];
      md[w] += ok ? 1 : 0;
      if (__any(cand)) {
        topk_insert<ND>(bd[w], cand ? key : 0);
        refresh();
      }
    }
  };
  // every point of the wave takes one operand of this span, none of which can enter a top T
  auto skip_all = [&](bool count_l, bool count_d) {
#pragma unroll
    for (int w = 0; w < RW; w++) {
      if (count_l) ml[w] += in[w] ? 1 : 0;
      if (count_d) md[w] += in[w] ? 1 : 0;
    }
  };
  auto put_lerp = [&](int w, const RawPt& a, const RawPt& b, bool ok) {
    const int64_t x0 = a.tsf & RAW_TIME_MASK, x1 = b.tsf & RAW_TIME_MASK;
    if (uns) {
      bool dz = false;
      if (DL) put_l(w, jlerp_u(interp, x[w], x0, (int64_t)a.bits, x1, (int64_t)b.bits, dz), ok);
      if (DD) put_d(w, dlerp_u(interp, x[w], x0, pt_double(a.tsf, a.bits), x1, pt_double(b.tsf, b.bits)), ok);
      if (dz && ok) dzm |= 1u << w;
    } else {
      if (DL) put_l(w, jlerp(interp, x[w], x0, (int64_t)a.bits, x1, (int64_t)b.bits), ok);
      if (DD) put_d(w, dlerp(interp, x[w], x0, pt_double(a.tsf, a.bits), x1, pt_double(b.tsf, b.bits)), ok);
    }
  };

  // A span's cursors and window ends are loads that depend on each other (cursor, then the
  // points at it), and with RAW_W / RW waves a strip each wave has few points to work on between
  // them: the next span's points and the one after's cursors are loaded a step ahead.
  struct SpanPre {
    int n, c, m;
    const RawPt* pts;
  };
  auto meta = [&](int i) {
    SpanPre M;
    const int64_t s = sb + i;
    M.n = p.sp_n[s];
    M.pts = p.pts + p.sp_off[s];
    M.c = crow[i];
    M.m = (cnext ? cnext[i] : M.n - first) - M.c;
    return M;
  };
  auto ends = [&](const SpanPre& M, RawPt& A, RawPt& B) {   // pts[c - 1], pts[c] (clamped)
    const int hi = max(M.n - 1, 0);
    const RawPt* base = M.n > 0 ? M.pts : p.pts;
    A = base[min(max(M.c - 1, 0), hi)];
    B = base[min(max(M.c, 0), hi)];
  };
  SpanPre M0{}, M1{};
  RawPt A0{}, B0{}, A1{}, B1{};
  if (k > 0) {
    M0 = meta(0);
    M1 = k > 1 ? meta(1) : M0;
    ends(M0, A0, B0);
  }
  for (int i = 0; i < k; i++) {
    const SpanPre cur = M0;
    const RawPt ea = A0, eb = B0;
    if (i + 1 < k) ends(M1, A1, B1);
    SpanPre M2 = M1;
    if (i + 2 < k) M2 = meta(i + 2);
    M0 = M1;
    A0 = A1;
    B0 = B1;
    M1 = M2;
    const int n = cur.n;
    if (n < (RATE ? 2 : 1)) continue;
    const int nc = n - first;
    const RawPt* pts = cur.pts;
    const int c = cur.c;
    const int m = cur.m;
    if (m == 0) {
      if (RATE) {
        if (c == nc) continue;
        const double y = __longlong_as_double((long long)eb.bits);   // pts[c]
        if (!isnan(y) && f2key(y) < thr) { skip_all(false, true); continue; }   // (the same operand at every point)
#pragma unroll
        for (int w = 0; w < RW; w++) put_d(w, y, true);
      } else {
        if (c == 0) {
          if (eb.tsf & RAW_FLOAT) flt = (1u << RW) - 1;   // pts[0]
          continue;
        }
        if (c == n) continue;
        const RawPt a = ea, b = eb;   // pts[c - 1], pts[c]
        if ((a.tsf | b.tsf) & RAW_FLOAT) flt = (1u << RW) - 1;
        const int64_t x0 = a.tsf & RAW_TIME_MASK, x1 = b.tsf & RAW_TIME_MASK;
        if (MODE == 1 && !uns && interp == TSDB_INTERP_LERP) {
          // a double LERP strictly inside (x0, x1) stays within [y0, y1] up to a few ulps of
          // rounding: skipped when even 8 key steps (ulps) above the larger end lie below thr
          const double y0 = pt_double(a.tsf, a.bits), y1 = pt_double(b.tsf, b.bits);
          if (isfinite(y0) && isfinite(y1) && f2key(fmax(y0, y1)) + 8 < thr) { skip_all(false, true); continue; }
        }
        if (MODE == 0 && !uns && interp == TSDB_INTERP_LERP && x1 > x0) {
          // a long LERP strictly inside the window whose product (x - x0) dy cannot wrap:
          // y0 + trunc((x - x0) dy / (x1 - x0)) lies within [y0, y1] (wave-uniform test, before
          // any per-lane work)
          const int64_t ya = (int64_t)a.bits, yb = (int64_t)b.bits;
          int64_t dy, prod;
          if (((uint64_t)max(ya, yb) ^ 0x8000000000000000ULL) < thr && !__builtin_sub_overflow(yb, ya, &dy) &&
              !__builtin_mul_overflow(dy, x1 - x0, &prod)) {
            skip_all(true, false);
            continue;
          }
        }
        if (DL && p.lerp_fast) {   // the strip-wide window (lerpw_*, as in k_raw_eval)
          const LerpW L = lerpw_init(interp, uns, x0, (int64_t)a.bits, x1, (int64_t)b.bits);
          if (L.ok) {
#pragma unroll
            for (int w = 0; w < RW; w++) {
              put_l(w, lerpw_eval(L, x[w]), true);
              if (DD) put_d(w, dlerp(interp, x[w], x0, pt_double(a.tsf, a.bits), x1, pt_double(b.tsf, b.bits)), true);
            }
            continue;
          }
        }
#pragma unroll
        for (int w = 0; w < RW; w++) put_lerp(w, a, b, true);
      }
      continue;
    }
    if (!RATE && MODE == 0 && !uns && interp == TSDB_INTERP_LERP && c >= 1 && c + m <= n - 1) {
      // points inside the strip, with one before and one after it: every point of the wave takes an
      // operand (its own value, or a LERP between two of pts[c - 1 .. c + m]); below thr when the
      // largest of those values is and no LERP product can wrap
      int64_t ymax = INT64_MIN;
      bool safe = true;
      for (int t = c - 1; t < c + m && safe; t++) {
        const RawPt a = pts[t], b = pts[t + 1];
        const int64_t ya = (int64_t)a.bits, yb = (int64_t)b.bits;
        const int64_t xa = a.tsf & RAW_TIME_MASK, xb = b.tsf & RAW_TIME_MASK;
        int64_t dy, prod;
        safe = xb > xa && !__builtin_sub_overflow(yb, ya, &dy) && !__builtin_mul_overflow(dy, xb - xa, &prod);
        ymax = max(ymax, max(ya, yb));
      }
      if (safe && ((uint64_t)ymax ^ 0x8000000000000000ULL) < thr) {
        skip_all(true, false);
        continue;
      }
    }
    if (lane < RAW_W) wmask[lane] = 0;
    WAVE_SYNC();
    const int32_t* rk = p.rank + (pts - p.pts) + first + c;   // (sp_off[s] + ...)
    for (int l = lane; l < m; l += 64) {
      const int64_t o = rk[l] - ua;
      __hip_atomic_fetch_or(&wmask[o >> 6], 1ULL << (o & 63), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    WAVE_SYNC();
    int tb = 0;
    for (int w2 = 0; w2 < q * RW; w2++) tb += __popcll(wmask[w2]);   // the span's ranks before this wave's points
#pragma unroll
    for (int w = 0; w < RW; w++) {
      const uint64_t M = wmask[q * RW + w];
      const int cnt = c + tb + __popcll(M & below);
      const bool own = (M >> lane) & 1ULL;
      tb += __popcll(M);
      if (RATE) {
        const bool ok = !(cnt == nc && !own);
        put_d(w, ok ? __longlong_as_double((long long)pts[cnt].bits) : 0.0, ok);   // (n = nc + 1 points)
      } else {
        if (cnt == 0) {
          if (pts[0].tsf & RAW_FLOAT) flt |= 1u << w;
          put_l(w, 0, false);
          put_d(w, 0.0, false);
          continue;
        }
        const int j = cnt - 1;
        const RawPt a = pts[j];
        const bool exact = j == n - 1 || own;   // the span's own point (or its last one)
        const bool ok = !(j == n - 1 && !own);
        if (exact) {
          if (ok) {
            if (a.tsf & RAW_FLOAT) flt |= 1u << w;
            if (j < n - 1 && (pts[j + 1].tsf & RAW_FLOAT)) flt |= 1u << w;
          }
          put_l(w, (int64_t)a.bits, ok);
          put_d(w, pt_double(a.tsf, a.bits), ok);
          continue;
        }
        const RawPt b = pts[j + 1];
        if ((a.tsf | b.tsf) & RAW_FLOAT) flt |= 1u << w;
        put_lerp(w, a, b, true);
      }
    }
    WAVE_SYNC();
  }

  const int fn = p.sel_fn;
#pragma unroll
  for (int w = 0; w < RW; w++) {
    if (!in[w]) continue;
    const int64_t idx = obase + uq + 64 * w + lane;
    const bool is_int = !RATE && !((flt >> w) & 1);
    if (uns && ((dzm >> w) & 1)) p.dz[idx] = 1;
    const int m = is_int ? ml[w] : md[w];
    int r0, r1;
    double dif;
    raw_sel_ranks(fn, is_int, m, r0, r1, dif);
    uint64_t k0 = 0, k1 = 0;
    if (m > 0) {
      const int i0 = m - 1 - r0, i1 = r1 >= 0 ? m - 1 - r1 : i0;   // positions from the top
      if (i0 >= T || i0 < 0 || i1 < 0) {
        set_err(p.err, TSDB_E_HIP);   // planning error: the rank is not among the kept keys
        continue;
      }
      if (is_int) {
        if (DL) { k0 = topk_at<NL>(bl[w], i0); k1 = topk_at<NL>(bl[w], i1); }
        else set_err(p.err, TSDB_E_HIP);   // planning error: an integer point without long operands
      } else {
        if (DD) { k0 = topk_at<ND>(bd[w], i0); k1 = topk_at<ND>(bd[w], i1); }
        else set_err(p.err, TSDB_E_HIP);
      }
    }
    raw_sel_store(p, idx, is_int, fn, m, r1, dif, k0, k1);
    p.out_int[idx] = is_int ? 1 : 0;
  }
}

// T: keys kept a point (8 / 16 / 32, >= raw_top_need); 0 when the query is not fused
hipError_t launch_raw_top(const RawParams& p, int T, hipStream_t s) {
  if (p.n_strips == 0) return hipSuccess;
  const int mode = p.rate ? 1 : (p.do_long && p.do_double) ? 2 : p.do_long ? 0 : 1;
#define RAW_TOP(TT, RW)                                                                                        \
  do {                                                                                                        \
    const dim3 grid((unsigned)(p.n_strips * (RAW_W / (RW)))), block(64);                                     \
    if (p.rate) hipLaunchKernelGGL((k_raw_top<TT, RW, 1, true>), grid, block, 0, s, p);                       \
    else if (mode == 0) hipLaunchKernelGGL((k_raw_top<TT, RW, 0, false>), grid, block, 0, s, p);              \
    else if (mode == 1) hipLaunchKernelGGL((k_raw_top<TT, RW, 1, false>), grid, block, 0, s, p);              \
    else hipLaunchKernelGGL((k_raw_top<TT, (RW > 1 ? RW / 2 : 1), 2, false>),                                \
                            dim3((unsigned)(p.n_strips * (RAW_W / (RW > 1 ? RW / 2 : 1)))), block, 0, s, p);  \
  } while (0)
  if (T == 8) RAW_TOP(8, 4);
  else if (T == 16) RAW_TOP(16, 2);
  else if (T == 32) RAW_TOP(32, 1);
  else return hipErrorInvalidValue;
#undef RAW_TOP
  return hipGetLastError();
}

hipError_t launch_raw_vals(const RawParams& p, int64_t k_max, hipStream_t s) {
  if (p.n_strips == 0) return hipSuccess;
  const dim3 grid((unsigned)p.n_strips, (unsigned)((k_max + RAW_SEL_SPANS - 1) / RAW_SEL_SPANS)), block(64);
  if (p.rate) hipLaunchKernelGGL((k_raw_vals<false, true, true>), grid, block, 0, s, p);
  else if (p.do_long && p.do_double) hipLaunchKernelGGL((k_raw_vals<true, true, false>), grid, block, 0, s, p);
  else if (p.do_long) hipLaunchKernelGGL((k_raw_vals<true, false, false>), grid, block, 0, s, p);
  else hipLaunchKernelGGL((k_raw_vals<false, true, false>), grid, block, 0, s, p);
  return hipGetLastError();
}
#endif

}  // namespace tsdb
