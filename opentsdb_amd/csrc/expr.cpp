// expr.cpp -- host side of the expression functions over query results:
// tsdbhip_expr_map, tsdbhip_expr_zip.  Kernels in k_expr.hip; the function names, parameter
// parsing and the union join by tags live in the host mirror (opentsdb_amd/expression.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/tsdbhip.h"
#include "expr.h"

namespace tsdb {
hipStream_t ctx_stream(tsdbhip_ctx* c);
int ctx_device(tsdbhip_ctx* c);
std::mutex& ctx_mutex(tsdbhip_ctx* c);
int set_error(int code, const std::string& msg);
tsdbhip_result* new_result(int64_t n_groups, int64_t n_points);
}  // namespace tsdb

using namespace tsdb;

namespace {

#define XOK(expr)                                                                              \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) { release(); return set_error(TSDB_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); } \
  } while (0)

// device copies of one call's arrays (expression inputs are query results: small, per call)
struct Scratch {
  std::vector<void*> bufs;
  hipError_t alloc(void** p, size_t bytes) {
    hipError_t e = hipMalloc(p, bytes ? bytes : 16);
    if (e == hipSuccess) bufs.push_back(*p);
    return e;
  }
  ~Scratch() {
    for (void* b : bufs) (void)hipFree(b);
  }
};

int check_set(const tsdbhip_series_set* in) {
  if (!in || in->n_series < 0 || !in->ptr || (in->ptr[in->n_series] > 0 && (!in->ts_ms || !in->value_bits || !in->is_int)))
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "malformed series set");
  return 0;
}

}  // namespace

extern "C" int tsdbhip_expr_map(tsdbhip_ctx* c, int fn, double fparam, int64_t iparam, int64_t start_ms, int64_t end_ms,
                                const tsdbhip_series_set* in, tsdbhip_result** out) {
  if (!c || !out) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  *out = nullptr;
  if (int rc = check_set(in)) return rc;
  if (fn < TSDB_EXPR_SCALE || fn > TSDB_EXPR_MOVING_AVG) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "unknown expression function");
  if (fn == TSDB_EXPR_MOVING_AVG && iparam <= 0)
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "Moving average window must be an integer greater than zero");
  std::lock_guard<std::mutex> lk(ctx_mutex(c));
  if (hipSetDevice(ctx_device(c)) != hipSuccess) return set_error(TSDB_E_HIP, "hipSetDevice");
  hipStream_t st = ctx_stream(c);
  const int64_t S = in->n_series, N = in->ptr[S];
  // moving average: the one-span AggregationIterator over [start, end] emits the points from its
  // seek(start) on while their timestamps stay <= end (AggregationIterator.java:395-460)
  std::vector<int64_t> lo(N > 0 ? N : 1, -1);
  std::vector<uint8_t> emit(N > 0 ? N : 1, 1);
  if (fn == TSDB_EXPR_MOVING_AVG) {
    for (int64_t s = 0; s < S; s++) {
      int64_t first = -1;
      for (int64_t q = in->ptr[s]; q < in->ptr[s + 1]; q++) {
        const bool keep = in->ts_ms[q] >= start_ms && in->ts_ms[q] <= end_ms && (first >= 0 || in->ts_ms[q] >= start_ms);
        if (first < 0 && in->ts_ms[q] >= start_ms) first = q;
        if (first >= 0 && in->ts_ms[q] > end_ms) { for (int64_t r = q; r < in->ptr[s + 1]; r++) emit[r] = 0; break; }
        emit[q] = first >= 0 && keep;
        lo[q] = emit[q] ? first : -1;
      }
    }
  }
  Scratch sc;
  auto release = [&]() {};
  ExprMapParams p{};
  void *d_ts, *d_bits, *d_int, *d_lo, *o_ts, *o_bits, *o_int, *d_err;
  XOK(sc.alloc(&d_ts, N * 8));
  XOK(sc.alloc(&d_bits, N * 8));
  XOK(sc.alloc(&d_int, N));
  XOK(sc.alloc(&d_lo, N * 8));
  XOK(sc.alloc(&o_ts, N * 8));
  XOK(sc.alloc(&o_bits, N * 8));
  XOK(sc.alloc(&o_int, N));
  XOK(sc.alloc(&d_err, 16));
  if (N) {
    XOK(hipMemcpyAsync(d_ts, in->ts_ms, N * 8, hipMemcpyHostToDevice, st));
    XOK(hipMemcpyAsync(d_bits, in->value_bits, N * 8, hipMemcpyHostToDevice, st));
    XOK(hipMemcpyAsync(d_int, in->is_int, N, hipMemcpyHostToDevice, st));
    XOK(hipMemcpyAsync(d_lo, lo.data(), N * 8, hipMemcpyHostToDevice, st));
  }
  XOK(hipMemsetAsync(d_err, 0, 16, st));
  p.n = N;
  p.ts = (const int64_t*)d_ts;
  p.bits = (const uint64_t*)d_bits;
  p.is_int = (const uint8_t*)d_int;
  p.lo = (const int64_t*)d_lo;
  p.fn = fn;
  p.fparam = fparam;
  p.scale_is_int = fparam == std::floor(fparam) && !std::isinf(fparam);
  p.time_window = fn == TSDB_EXPR_MOVING_AVG && fparam != 0.0;
  p.iparam = iparam;
  p.out_ts = (int64_t*)o_ts;
  p.out_bits = (uint64_t*)o_bits;
  p.out_int = (uint8_t*)o_int;
  p.err = (int32_t*)d_err;
  XOK(expr_map(p, st));
  std::vector<int64_t> ots(N > 0 ? N : 1);
  std::vector<uint64_t> obits(N > 0 ? N : 1);
  std::vector<uint8_t> oint(N > 0 ? N : 1);
  int32_t err = 0;
  if (N) {
    XOK(hipMemcpyAsync(ots.data(), o_ts, N * 8, hipMemcpyDeviceToHost, st));
    XOK(hipMemcpyAsync(obits.data(), o_bits, N * 8, hipMemcpyDeviceToHost, st));
    XOK(hipMemcpyAsync(oint.data(), o_int, N, hipMemcpyDeviceToHost, st));
  }
  XOK(hipMemcpyAsync(&err, d_err, 4, hipMemcpyDeviceToHost, st));
  XOK(hipStreamSynchronize(st));
  if (err) return set_error(err, err == TSDB_E_CLASS_CAST ? "Not a long (TimeShift of a double data point)" : "expression");
  int64_t n_out = 0;
  for (int64_t q = 0; q < N; q++) n_out += emit[q];
  tsdbhip_result* r = new_result(S, n_out);
  if (!r) return set_error(TSDB_E_NOMEM, "result");
  auto* gid = const_cast<int32_t*>(r->group_id);
  auto* gptr = const_cast<int64_t*>(r->group_ptr);
  auto* rts = const_cast<int64_t*>(r->ts_ms);
  auto* rb = const_cast<uint64_t*>(r->value_bits);
  auto* ri = const_cast<uint8_t*>(r->is_int);
  int64_t o = 0;
  gptr[0] = 0;
  for (int64_t s = 0; s < S; s++) {
    gid[s] = (int32_t)s;
    for (int64_t q = in->ptr[s]; q < in->ptr[s + 1]; q++) {
      if (!emit[q]) continue;
      rts[o] = ots[q];
      rb[o] = obits[q];
      ri[o] = oint[q];
      o++;
    }
    gptr[s + 1] = o;
  }
  *out = r;
  return 0;
}

extern "C" int tsdbhip_expr_zip(tsdbhip_ctx* c, const int32_t* program, int n_ops, const double* consts, int n_vars,
                                int64_t n_sets, const int32_t* set_series, const double* var_fill,
                                const tsdbhip_series_set* in, tsdbhip_result** out) {
  if (!c || !out || !program || n_ops <= 0 || n_vars <= 0 || n_sets < 0 || (n_sets && !set_series) || !var_fill)
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  *out = nullptr;
  if (int rc = check_set(in)) return rc;
  // validate the program: stack depth, operands, indices
  int depth = 0, maxd = 0, n_consts = 0;
  for (int o = 0; o < n_ops; o++) {
    const int op = program[2 * o], arg = program[2 * o + 1];
    if (op == TSDB_XOP_VAR) { if (arg < 0 || arg >= n_vars) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "bad variable"); depth++; }
    else if (op == TSDB_XOP_CONST) { if (arg < 0) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "bad constant"); n_consts = std::max(n_consts, arg + 1); depth++; }
    else if (op == TSDB_XOP_NEG) { if (depth < 1) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "bad program"); }
    else if (op >= TSDB_XOP_ADD && op <= TSDB_XOP_MOD) { if (depth < 2) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "bad program"); depth--; }
    else return set_error(TSDB_E_ILLEGAL_ARGUMENT, "bad opcode");
    maxd = std::max(maxd, depth);
  }
  if (depth != 1) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "bad program");
  if (maxd > EXPR_STACK) return set_error(TSDB_E_NOT_IMPLEMENTED, "expression deeper than the evaluation stack");
  if (n_consts && !consts) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "missing constants");
  const int64_t S = in->n_series, N = in->ptr[S];
  for (int64_t i = 0; i < n_sets * n_vars; i++)
    if (set_series[i] >= S) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "set series out of range");
  // output length of each set: EDPtoDPS iterates while some present series has a point
  std::vector<int64_t> off(n_sets + 1, 0);
  for (int64_t j = 0; j < n_sets; j++) {
    int64_t len = 0;
    for (int v = 0; v < n_vars; v++) {
      const int32_t s = set_series[j * n_vars + v];
      if (s >= 0) len = std::max<int64_t>(len, in->ptr[s + 1] - in->ptr[s]);
    }
    off[j + 1] = off[j] + len;
  }
  const int64_t n_out = off[n_sets];
  std::lock_guard<std::mutex> lk(ctx_mutex(c));
  if (hipSetDevice(ctx_device(c)) != hipSuccess) return set_error(TSDB_E_HIP, "hipSetDevice");
  hipStream_t st = ctx_stream(c);
  Scratch sc;
  auto release = [&]() {};
  void *d_prog, *d_consts, *d_sets, *d_fill, *d_ptr, *d_ts, *d_bits, *d_int, *d_off, *o_ts, *o_bits, *o_int, *d_err;
  XOK(sc.alloc(&d_prog, n_ops * 8));
  XOK(sc.alloc(&d_consts, n_consts * 8));
  XOK(sc.alloc(&d_sets, n_sets * n_vars * 4));
  XOK(sc.alloc(&d_fill, n_vars * 8));
  XOK(sc.alloc(&d_ptr, (S + 1) * 8));
  XOK(sc.alloc(&d_ts, N * 8));
  XOK(sc.alloc(&d_bits, N * 8));
  XOK(sc.alloc(&d_int, N));
  XOK(sc.alloc(&d_off, (n_sets + 1) * 8));
  XOK(sc.alloc(&o_ts, n_out * 8));
  XOK(sc.alloc(&o_bits, n_out * 8));
  XOK(sc.alloc(&o_int, n_out));
  XOK(sc.alloc(&d_err, 16));
  XOK(hipMemcpyAsync(d_prog, program, n_ops * 8, hipMemcpyHostToDevice, st));
  if (n_consts) XOK(hipMemcpyAsync(d_consts, consts, n_consts * 8, hipMemcpyHostToDevice, st));
  if (n_sets) XOK(hipMemcpyAsync(d_sets, set_series, n_sets * n_vars * 4, hipMemcpyHostToDevice, st));
  XOK(hipMemcpyAsync(d_fill, var_fill, n_vars * 8, hipMemcpyHostToDevice, st));
  XOK(hipMemcpyAsync(d_ptr, in->ptr, (S + 1) * 8, hipMemcpyHostToDevice, st));
  if (N) {
    XOK(hipMemcpyAsync(d_ts, in->ts_ms, N * 8, hipMemcpyHostToDevice, st));
    XOK(hipMemcpyAsync(d_bits, in->value_bits, N * 8, hipMemcpyHostToDevice, st));
    XOK(hipMemcpyAsync(d_int, in->is_int, N, hipMemcpyHostToDevice, st));
  }
  XOK(hipMemcpyAsync(d_off, off.data(), (n_sets + 1) * 8, hipMemcpyHostToDevice, st));
  XOK(hipMemsetAsync(d_err, 0, 16, st));
  ExprZipParams p{(const int32_t*)d_prog, n_ops, (const double*)d_consts, n_vars, n_sets, (const int32_t*)d_sets,
                  (const double*)d_fill, (const int64_t*)d_ptr, (const int64_t*)d_ts, (const uint64_t*)d_bits,
                  (const uint8_t*)d_int, (const int64_t*)d_off, n_out, (int64_t*)o_ts, (uint64_t*)o_bits,
                  (uint8_t*)o_int, (int32_t*)d_err};
  XOK(expr_zip(p, st));
  tsdbhip_result* r = new_result(n_sets, n_out);
  if (!r) return set_error(TSDB_E_NOMEM, "result");
  int32_t err = 0;
  if (n_out) {
    XOK(hipMemcpyAsync(const_cast<int64_t*>(r->ts_ms), o_ts, n_out * 8, hipMemcpyDeviceToHost, st));
    XOK(hipMemcpyAsync(const_cast<uint64_t*>(r->value_bits), o_bits, n_out * 8, hipMemcpyDeviceToHost, st));
    XOK(hipMemcpyAsync(const_cast<uint8_t*>(r->is_int), o_int, n_out, hipMemcpyDeviceToHost, st));
  }
  XOK(hipMemcpyAsync(&err, d_err, 4, hipMemcpyDeviceToHost, st));
  XOK(hipStreamSynchronize(st));
  if (err) {
    tsdbhip_result_free(r);
    return set_error(err, "expression evaluation: a series ended before another (No more elements) or a division by zero");
  }
  for (int64_t j = 0; j <= n_sets; j++) const_cast<int64_t*>(r->group_ptr)[j] = off[j];
  for (int64_t j = 0; j < n_sets; j++) const_cast<int32_t*>(r->group_id)[j] = (int32_t)j;
  *out = r;
  return 0;
}
