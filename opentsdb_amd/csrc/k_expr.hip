// k_expr.hip -- expression functions over query results (src/query/expression/).
//
//   k_expr_map   thread per point: Scale / Absolute / TimeShift (Scale.java:86-112,
//                Absolute.java:64-83, TimeShift.java:121-141)
//   k_expr_mavg  thread per point: MovingAverageAggregator.runDouble (MovingAverage.java:262-330)
//                -- the window walks back from the point, newest first, as the aggregator's
//                LinkedList does, so the sum is the reference's in its order
//   k_expr_zip   thread per (joined set, position): ExpressionIterator.next(index)
//                (ExpressionIterator.java:282-318) through EDPtoDPS, the program over doubles
#include <hip/hip_runtime.h>
#include <stdint.h>

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
  double stack[EXPR_STACK];
  int sp = 0;
  int64_t ts = INT64_MAX;
  for (int v = 0; v < p.n_vars; v++) {   // timestamps of the present series at position k
    const int32_t s = p.set_series[j * p.n_vars + v];
    if (s < 0) continue;
    const int64_t q = p.ptr[s] + k;
    if (q >= p.ptr[s + 1]) { set_err(p.err, TSDB_E_RUNTIME); return; }   // "No more elements"
    ts = min(ts, p.ts[q]);
  }
  for (int o = 0; o < p.n_ops; o++) {
    const int op = p.prog[2 * o], arg = p.prog[2 * o + 1];
    if (op == TSDB_XOP_VAR) {
      const int32_t s = p.set_series[j * p.n_vars + arg];
      double v = 0.0;   // UnionIterator's fill_dp: a default MutableDataPoint reads 0
      if (s >= 0) {
        const int64_t q = p.ptr[s] + k;
        v = pt_double(p.bits[q], p.is_int[q]);
        if (v != v) v = p.var_fill[arg];
      }
      stack[sp++] = v;
    } else if (op == TSDB_XOP_CONST) {
      stack[sp++] = p.consts[arg];
    } else if (op == TSDB_XOP_NEG) {
      stack[sp - 1] = -stack[sp - 1];
    } else {
      const double r = stack[--sp], l = stack[--sp];
      double x;
      switch (op) {
        case TSDB_XOP_ADD: x = l + r; break;
        case TSDB_XOP_SUB: x = l - r; break;
        case TSDB_XOP_MUL: x = l * r; break;
        case TSDB_XOP_DIV:
          if (r == 0.0) { set_err(p.err, TSDB_E_RUNTIME); return; }   // JexlArithmetic.divide
          x = l / r;
          break;
        default:
          if (r == 0.0) { set_err(p.err, TSDB_E_RUNTIME); return; }   // JexlArithmetic.mod
          x = fmod(l, r);
          break;
      }
      stack[sp++] = x;
    }
  }
  p.out_ts[t] = ts;
  p.out_bits[t] = (uint64_t)__double_as_longlong(stack[0]);
  p.out_int[t] = 0;
}

}  // namespace

hipError_t expr_map(const ExprMapParams& p, hipStream_t s) {
  if (p.n <= 0) return hipSuccess;
  if (p.fn == TSDB_EXPR_MOVING_AVG) hipLaunchKernelGGL(k_expr_mavg, dim3((unsigned)((p.n + 255) / 256)), dim3(256), 0, s, p);
  else hipLaunchKernelGGL(k_expr_map, dim3((unsigned)((p.n + 255) / 256)), dim3(256), 0, s, p);
  return hipGetLastError();
}
hipError_t expr_zip(const ExprZipParams& p, hipStream_t s) {
  if (p.n_out <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_expr_zip, dim3((unsigned)((p.n_out + 255) / 256)), dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace tsdb
