// k_expr.hip -- expression functions over query results (src/query/expression/).
//
//   k_expr_map   thread per point: Scale / Absolute / TimeShift (Scale.java:86-112,
//                Absolute.java:64-83, TimeShift.java:121-141)
//   k_expr_mavg  thread per point: MovingAverageAggregator.runDouble (MovingAverage.java:262-330)
//                -- the window walks back from the point, newest first, as the aggregator's
//                LinkedList does, so the sum is the reference's in its order
//   k_expr_zip   thread per (joined set, position): ExpressionIterator.next(index)
//                (ExpressionIterator.java:452-485) through EDPtoDPS, the program over doubles
//   k_expr_sync  thread per (joined set, step): ExpressionIterator.next(timestamp) (:323-358) over
//                the join iterator's time-synchronised steps
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/tsdbhip.h"
#include "expr.h"

namespace tsdb {
namespace {

__device__ __forceinline__ double pt_double(uint64_t bits, uint8_t is_int) {   // DataPoint.toDouble()
  return is_int ? (double)(int64_t)bits : __longlong_as_double((long long)bits);
}
__device__ __forceinline__ int64_t java_d2l(double d) {   // (long) d
  if (d != d) return 0;
  if (d >= 9223372036854775807.0) return INT64_MAX;
  if (d <= -9223372036854775808.0) return INT64_MIN;
  return (int64_t)d;
}
__device__ __forceinline__ void set_err(int32_t* err, int code) { atomicCAS(err, 0, code); }

__global__ void k_expr_map(ExprMapParams p) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  const uint64_t bits = p.bits[i];
  const uint8_t is_int = p.is_int[i];
  int64_t ts = p.ts[i];
  uint64_t ob;
  uint8_t oi;
  if (p.fn == TSDB_EXPR_SCALE) {
    if (is_int && p.scale_is_int) {
      ob = (uint64_t)java_d2l(p.fparam) * bits;   // (long) scale_factor * longValue(), Java wrap
      oi = 1;
    } else {
      ob = (uint64_t)__double_as_longlong(p.fparam * pt_double(bits, is_int));
      oi = 0;
    }
  } else if (p.fn == TSDB_EXPR_ABSOLUTE) {
    if (is_int) {
      const int64_t v = (int64_t)bits;
      ob = (uint64_t)(v < 0 ? (int64_t)(0 - (uint64_t)v) : v);   // Math.abs(long): MIN_VALUE stays
      oi = 1;
    } else {
      ob = bits & 0x7FFFFFFFFFFFFFFFull;                          // Math.abs(double)
      oi = 0;
    }
  } else {   // TSDB_EXPR_SHIFT: ofLongValue(ts + shift, longValue())
    if (!is_int) set_err(p.err, TSDB_E_CLASS_CAST);
    ts += p.iparam;
    ob = bits;
    oi = 1;
  }
  p.out_ts[i] = ts;
  p.out_bits[i] = ob;
  p.out_int[i] = oi;
}

// MovingAverageAggregator.runDouble over the points [lo, i] of one series (lo = the first point
// the one-span AggregationIterator emits); every emitted value is a double.
__global__ void k_expr_mavg(ExprMapParams p) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  const int64_t lo = p.lo[i];
  if (lo < 0) return;   // not emitted (outside the AggregationIterator's range)
  double sum = 0;
  int32_t count = 0;
  bool met = false;
  if (p.time_window) {
    if (i == lo) {      // the first point of a time window: no previous timestamp, 0
      p.out_ts[i] = p.ts[i];
      p.out_bits[i] = 0;
      p.out_int[i] = 0;
      return;
    }
    int64_t cum = 0, last = -1;
    for (int64_t j = i; j >= lo; j--) {
      const int64_t t = p.ts[j];
      if (last < 0) {
        last = t;
      } else {
        cum += last - t;
        last = t;
        if (cum >= p.iparam) { met = true; break; }
      }
      const double v = pt_double(p.bits[j], p.is_int[j]);
      if (v == v) { sum += v; count++; }
    }
  } else {
    for (int64_t j = i; j >= lo; j--) {
      const double v = pt_double(p.bits[j], p.is_int[j]);
      if (v == v) { sum += v; count++; }
      if (count >= p.iparam) { met = true; break; }
    }
  }
  const double r = (!met || count == 0) ? 0.0 : sum / (double)count;
  p.out_ts[i] = p.ts[i];
  p.out_bits[i] = (uint64_t)__double_as_longlong(r);
  p.out_int[i] = 0;
}

// The postfix program of one expression evaluation (JEXL 2.1.1 arithmetic, Interpreter.visit of
// the arithmetic and comparison nodes): the operands are Doubles (variables) or constants the host
// folded; a division or modulo error yields Double 0.0 (the lenient interpreter), comparisons give
// Boolean -> 1.0 / 0.0 (ExpressionIterator.java:347-351).  var(v) loads variable v.
template <class Var>
__device__ __forceinline__ double expr_eval(const int32_t* prog, int n_ops, const double* consts, Var&& var) {
  double stack[EXPR_STACK];
  int sp = 0;
  for (int o = 0; o < n_ops; o++) {
    const int op = prog[2 * o], arg = prog[2 * o + 1];
    if (op == TSDB_XOP_VAR) {
      stack[sp++] = var(arg);
    } else if (op == TSDB_XOP_CONST) {
      stack[sp++] = consts[arg];
    } else if (op == TSDB_XOP_NEG) {
      stack[sp - 1] = -stack[sp - 1];
    } else if (op == TSDB_XOP_NOT) {
      stack[sp - 1] = stack[sp - 1] != 0.0 ? 0.0 : 1.0;
    } else {
      const double r = stack[--sp], l = stack[--sp];
      double x;
      switch (op) {
        case TSDB_XOP_ADD: x = l + r; break;
        case TSDB_XOP_SUB: x = l - r; break;
        case TSDB_XOP_MUL: x = l * r; break;
        case TSDB_XOP_DIV: x = r == 0.0 ? 0.0 : l / r; break;          // JexlArithmetic.divide
        case TSDB_XOP_MOD: x = r == 0.0 ? 0.0 : fmod(l, r); break;     // JexlArithmetic.mod (Java %)
        case TSDB_XOP_IDIV: x = r == 0.0 ? 0.0 : trunc(l / r); break;  // BigInteger.divide
        case TSDB_XOP_IMOD: {                                          // BigInteger.mod: r > 0, result >= 0
          if (r <= 0.0) { x = 0.0; break; }
          x = fmod(l, r);
          if (x < 0.0) x += r;
          break;
        }
        case TSDB_XOP_LT: x = l < r ? 1.0 : 0.0; break;
        case TSDB_XOP_GT: x = l > r ? 1.0 : 0.0; break;
        case TSDB_XOP_LE: x = l <= r ? 1.0 : 0.0; break;
        case TSDB_XOP_GE: x = l >= r ? 1.0 : 0.0; break;
        case TSDB_XOP_EQ: x = l == r ? 1.0 : 0.0; break;
        default: x = l != r ? 1.0 : 0.0; break;
      }
      stack[sp++] = x;
    }
  }
  return stack[0];
}

__global__ void k_expr_zip(ExprZipParams p) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= p.n_out) return;
  // the joined set of output point t: set_off is an exclusive scan of the sets' lengths
  int64_t a = 0, b = p.n_sets;
  while (b - a > 1) {
    const int64_t m = (a + b) / 2;
    if (p.set_off[m] <= t) a = m; else b = m;
  }
  const int64_t j = a, k = t - p.set_off[j];
  int64_t ts = INT64_MAX;
  for (int v = 0; v < p.n_vars; v++) {   // timestamps of the present series at position k
    const int32_t s = p.set_series[j * p.n_vars + v];
    if (s < 0) continue;
    const int64_t q = p.ptr[s] + k;
    if (q >= p.ptr[s + 1]) { set_err(p.err, TSDB_E_RUNTIME); return; }   // "No more elements"
    ts = min(ts, p.ts[q]);
  }
  const double r = expr_eval(p.prog, p.n_ops, p.consts, [&](int v) {
    const int32_t s = p.set_series[j * p.n_vars + v];
    double x = 0.0;   // UnionIterator's fill_dp: a default MutableDataPoint reads 0
    if (s >= 0) {
      const int64_t q = p.ptr[s] + k;
      x = pt_double(p.bits[q], p.is_int[q]);
      if (x != x) x = p.var_fill[v];
    }
    return x;
  });
  p.out_ts[t] = ts;
  p.out_bits[t] = (uint64_t)__double_as_longlong(r);
  p.out_int[t] = 0;
}

// ---- time-synchronised evaluation (tsdbhip_expr_sync) -----------------------------------
// keys of the step timestamps: the active series' points inside [start, end]
__global__ void k_expr_sync_keys(ExprSyncParams p, int64_t* keys) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n_pts) return;
  const int64_t t = p.ts[i];
  const bool in = p.pt_active[i] && t >= p.start && t <= p.end;
  keys[i] = !in ? INT64_MAX : p.rep == 1 ? t : (t - p.base) * p.rep + p.rank[i];
}

// thread per (joined set, step): every variable's value at the step's timestamp -- its series'
// point there (binary search: the series are in time order; the step's copy of a repeated
// timestamp), else the variable's fill; then the
// program (ExpressionIterator.next(long), :323-358)
__global__ void k_expr_sync(ExprSyncParams p) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= p.n_sets * p.U) return;
  const int64_t j = t / p.U, u = t - j * p.U;
  const int64_t key = p.uts[u];
  const int64_t x = p.rep == 1 ? key : p.base + key / p.rep;   // the step's timestamp
  const int64_t c = p.rep == 1 ? 0 : key % p.rep;              // and copy of it
  const double r = expr_eval(p.prog, p.n_ops, p.consts, [&](int v) {
    const int32_t s = p.set_series[j * p.n_vars + v];
    double y = p.absent;
    if (s >= 0) {
      int64_t lo = p.ptr[s], hi = p.ptr[s + 1];
      while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        if (p.ts[m] < x) lo = m + 1; else hi = m;
      }
      lo += c;
      y = (lo < p.ptr[s + 1] && p.ts[lo] == x) ? pt_double(p.bits[lo], p.is_int[lo]) : p.var_fill[v];
    }
    return y != y ? p.var_fill[v] : y;
  });
  p.out_ts[t] = x;
  p.out_bits[t] = (uint64_t)__double_as_longlong(r);
  p.out_int[t] = 0;
}

// ---- highestMax / highestCurrent ------------------------------------------------------
// The state of span i at union point x, as AggregationIterator holds it after next() moved the
// spans at x (AggregationIterator.java:514-567, slots :482-494, zeroing :521-526): lo = the
// constructor's seek(start) position, hi = points <= x.  `flt`: a double in the span's current
// or next slot (isInteger :612-625); `act`: hasNextValue sees the span (ts[i] != 0).
struct TopSpan {
  bool act, flt, own;
  int64_t j;   // current point (act)
};
__device__ __forceinline__ TopSpan top_span(const ExprTopParams& p, int64_t i, int64_t x) {
  TopSpan r = {false, false, false, 0};
  const int64_t a = p.ptr[i], n = p.ptr[i + 1] - a, lo = p.lo[i];
  if (lo >= n) return r;                       // ended in the constructor
  int64_t l = lo, h = n;                       // hi = first point > x
  while (l < h) {
    const int64_t m = (l + h) >> 1;
    if (p.ts[a + m] <= x) l = m + 1; else h = m;
  }
  if (l == lo) {                               // not started: its next slot holds point lo
    r.flt = !p.is_int[a + lo];
    return r;
  }
  r.j = l - 1;
  r.own = p.ts[a + r.j] == x;
  if (r.j == n - 1) {                          // no next point: ended once its last one passed
    if (r.own) { r.act = true; r.flt = !p.is_int[a + r.j]; }
    return r;
  }
  r.act = true;
  r.flt = !p.is_int[a + r.j] || !p.is_int[a + r.j + 1];
  return r;
}

// nextLongValue / nextDoubleValue of an active span (:682-797): its own value, else the LERP
// between its current and next points (x0 < x < x1: the series are in time order)
__device__ __forceinline__ int64_t top_long(const ExprTopParams& p, int64_t i, const TopSpan& t, int64_t x) {
  const int64_t q = p.ptr[i] + t.j;
  const int64_t y0 = (int64_t)p.bits[q];
  if (t.own) return y0;
  const int64_t x0 = p.ts[q], x1 = p.ts[q + 1], y1 = (int64_t)p.bits[q + 1];
  const int64_t num = (int64_t)((uint64_t)(x - x0) * ((uint64_t)y1 - (uint64_t)y0));
  return (int64_t)((uint64_t)y0 + (uint64_t)(num / (x1 - x0)));
}
__device__ __forceinline__ double top_double(const ExprTopParams& p, int64_t i, const TopSpan& t, int64_t x) {
  const int64_t q = p.ptr[i] + t.j;
  const double y0 = pt_double(p.bits[q], p.is_int[q]);
  if (t.own) return y0;
  const int64_t x0 = p.ts[q], x1 = p.ts[q + 1];
  const double y1 = pt_double(p.bits[q + 1], p.is_int[q + 1]);
  return y0 + (double)(x - x0) * (y1 - y0) / (double)(x1 - x0);
}

__device__ __forceinline__ uint64_t dkey(double d) {   // Math.max order: -0.0 < 0.0, NaN on top
  uint64_t b = (uint64_t)__double_as_longlong(d);
  if (d != d) b = 0x7FF8000000000000ull;
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__device__ __forceinline__ int lanes_before(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// One wave per union point u: isInteger over every span's slots, then the operands in span
// order, each at its position among the spans with a value (MaxCacheAggregator.runLong /
// runDouble: longs[ix++], HighestMax.java:226-266), folded with Math.max per position.
// Positions past the point's operand count read 0: min_m records the smallest count.
__global__ __launch_bounds__(256) void k_expr_topn(ExprTopParams p) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t u = wave; u < p.U; u += nwaves) {
    const int64_t x = p.uts[u];
    bool flt = false;
    for (int64_t i0 = 0; i0 < p.n_series; i0 += 64) {
      const int64_t i = i0 + lane;
      if (i < p.n_series && top_span(p, i, x).flt) flt = true;
    }
    const bool is_int = !__any(flt);
    int64_t run = 0;
    for (int64_t i0 = 0; i0 < p.n_series; i0 += 64) {
      const int64_t i = i0 + lane;
      TopSpan t = {false, false, false, 0};
      if (i < p.n_series) t = top_span(p, i, x);
      const uint64_t m = __ballot(t.act);
      const int64_t pos = run + lanes_before(m);
      if (t.act && !p.current) {
        if (is_int) atomicMax((long long*)&p.max_l[pos], (long long)top_long(p, i, t, x));
        else atomicMax((unsigned long long*)&p.max_d[pos], (unsigned long long)dkey(top_double(p, i, t, x)));
      }
      run += __popcll(m);
    }
    if (lane == 0) {
      const int w = is_int ? 0 : 1;
      atomicOr(&p.has[w], 1);
      if (p.current) atomicMax((unsigned long long*)&p.last_u[w], (unsigned long long)u);
      else atomicMin(&p.min_m[w], (int32_t)run);
    }
  }
}

// MaxLatestAggregator: `ts > latest_ts` always holds (latest_ts is never updated,
// HighestCurrent.java:228-260), so each array is the positional operands of the LAST long /
// double point, zeros past its operand count (System.arraycopy of the zero-filled array).
__global__ __launch_bounds__(64) void k_expr_topn_at(ExprTopParams p) {
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x;   // 0: long point, 1: double point
  if (!p.has[w]) return;
  const int64_t u = p.last_u[w];
  const int64_t x = p.uts[u];
  int64_t run = 0;
  for (int64_t i0 = 0; i0 < p.n_series; i0 += 64) {
    const int64_t i = i0 + lane;
    TopSpan t = {false, false, false, 0};
    if (i < p.n_series) t = top_span(p, i, x);
    const uint64_t m = __ballot(t.act);
    const int64_t pos = run + lanes_before(m);
    if (t.act) {
      if (w == 0) p.max_l[pos] = top_long(p, i, t, x);
      else p.max_d[pos] = dkey(top_double(p, i, t, x));
    }
    run += __popcll(m);
  }
  for (int64_t q = run + lane; q < p.n_series; q += 64) {
    if (w == 0) p.max_l[q] = 0;
    else p.max_d[q] = dkey(0.0);
  }
}

}  // namespace

hipError_t expr_topn(const ExprTopParams& p, hipStream_t s) {
  if (p.U <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((p.U + 3) / 4, 65536);
  hipLaunchKernelGGL(k_expr_topn, dim3((unsigned)blocks), dim3(256), 0, s, p);
  return hipGetLastError();
}
hipError_t expr_topn_at(const ExprTopParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_expr_topn_at, dim3(2), dim3(64), 0, s, p);
  return hipGetLastError();
}

hipError_t expr_map(const ExprMapParams& p, hipStream_t s) {
  if (p.n <= 0) return hipSuccess;
  if (p.fn == TSDB_EXPR_MOVING_AVG) hipLaunchKernelGGL(k_expr_mavg, dim3((unsigned)((p.n + 255) / 256)), dim3(256), 0, s, p);
  else hipLaunchKernelGGL(k_expr_map, dim3((unsigned)((p.n + 255) / 256)), dim3(256), 0, s, p);
  return hipGetLastError();
}
hipError_t expr_sync_keys(const ExprSyncParams& p, int64_t* keys, hipStream_t s) {
  if (p.n_pts <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_expr_sync_keys, dim3((unsigned)((p.n_pts + 255) / 256)), dim3(256), 0, s, p, keys);
  return hipGetLastError();
}
hipError_t expr_sync(const ExprSyncParams& p, hipStream_t s) {
  const int64_t n = p.n_sets * p.U;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_expr_sync, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p);
  return hipGetLastError();
}
hipError_t expr_zip(const ExprZipParams& p, hipStream_t s) {
  if (p.n_out <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_expr_zip, dim3((unsigned)((p.n_out + 255) / 256)), dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace tsdb
