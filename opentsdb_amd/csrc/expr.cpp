// expr.cpp -- host side of the expression functions over query results:
// tsdbhip_expr_map, tsdbhip_expr_zip, tsdbhip_expr_sync, tsdbhip_expr_topn.  Kernels in k_expr.hip; the function names, parameter
// parsing and the union join by tags live in the host mirror (opentsdb_amd/expression.py).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>
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

// the postfix program: stack depth, operands, indices, opcodes
int check_program(const int32_t* program, int n_ops, int n_vars, const double* consts, int* n_consts_out) {
  int depth = 0, maxd = 0, n_consts = 0;
  for (int o = 0; o < n_ops; o++) {
    const int op = program[2 * o], arg = program[2 * o + 1];
    if (op == TSDB_XOP_VAR) { if (arg < 0 || arg >= n_vars) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "bad variable"); depth++; }
    else if (op == TSDB_XOP_CONST) { if (arg < 0) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "bad constant"); n_consts = std::max(n_consts, arg + 1); depth++; }
    else if (op == TSDB_XOP_NEG || op == TSDB_XOP_NOT) { if (depth < 1) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "bad program"); }
    else if ((op >= TSDB_XOP_ADD && op <= TSDB_XOP_MOD) || (op >= TSDB_XOP_LT && op <= TSDB_XOP_NE) ||
             op == TSDB_XOP_IDIV || op == TSDB_XOP_IMOD) {
      if (depth < 2) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "bad program");
      depth--;
    } else return set_error(TSDB_E_ILLEGAL_ARGUMENT, "bad opcode");
    maxd = std::max(maxd, depth);
  }
  if (depth != 1) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "bad program");
  if (maxd > EXPR_STACK) return set_error(TSDB_E_NOT_IMPLEMENTED, "expression deeper than the evaluation stack");
  if (n_consts && !consts) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "missing constants");
  *n_consts_out = n_consts;
  return 0;
}

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
  int n_consts = 0;
  if (int rc = check_program(program, n_ops, n_vars, consts, &n_consts)) return rc;
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
    return set_error(err, "expression evaluation: a series ended before another (No more elements)");
  }
  for (int64_t j = 0; j <= n_sets; j++) const_cast<int64_t*>(r->group_ptr)[j] = off[j];
  for (int64_t j = 0; j < n_sets; j++) const_cast<int32_t*>(r->group_id)[j] = (int32_t)j;
  *out = r;
  return 0;
}

extern "C" int tsdbhip_expr_sync(tsdbhip_ctx* c, const int32_t* program, int n_ops, const double* consts, int n_vars,
                                 int64_t n_sets, const int32_t* set_series, const double* var_fill, double absent_value,
                                 const uint8_t* active, int64_t start_ms, int64_t end_ms, const tsdbhip_series_set* in,
                                 tsdbhip_result** out) {
  if (!c || !out || !program || n_ops <= 0 || n_vars <= 0 || n_sets < 0 || (n_sets && !set_series) || !var_fill)
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  *out = nullptr;
  if (int rc = check_set(in)) return rc;
  int n_consts = 0;
  if (int rc = check_program(program, n_ops, n_vars, consts, &n_consts)) return rc;
  const int64_t S = in->n_series, N = in->ptr[S];
  for (int64_t i = 0; i < n_sets * n_vars; i++)
    if (set_series[i] >= S) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "set series out of range");
  // per point: does its series drive the steps, and its rank among the series' points at the
  // same timestamp.  Series may repeat a timestamp (non-decreasing); a decreasing one is refused.
  // The step walk over repeats (TimeSyncedIterator.next(long) :125-144 consumes one point per
  // series and step, nextTimestamp :147-158 the smallest current one): timestamp t is stepped
  // R_t times, R_t = the most copies of t any active series holds; at its j-th step a series
  // reads its j-th copy of t, else its fill.
  std::vector<uint8_t> pact(N > 0 ? N : 1, 0);
  std::vector<int32_t> prank;
  int64_t rep = 1, tmin = INT64_MAX, tmax = INT64_MIN;
  for (int64_t s = 0; s < S; s++) {
    const int64_t a = in->ptr[s], b = in->ptr[s + 1];
    if (b < a) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "malformed series set");
    const uint8_t act = active ? active[s] : 1;
    int64_t run = 0;
    for (int64_t q = a; q < b; q++) {
      pact[q] = act;
      const int64_t t = in->ts_ms[q];
      if (q > a && t < in->ts_ms[q - 1])
        return set_error(TSDB_E_NOT_IMPLEMENTED, "time-synchronised expression over a series out of time order");
      run = (q > a && t == in->ts_ms[q - 1]) ? run + 1 : 0;
      if (run) {
        if (prank.empty()) prank.assign(N, 0);
        prank[q] = (int32_t)std::min<int64_t>(run, INT32_MAX);
      }
      if (act && t >= start_ms && t <= end_ms) {
        rep = std::max(rep, run + 1);
        tmin = std::min(tmin, t);
        tmax = std::max(tmax, t);
      }
    }
  }
  // repeats: step key (t - tmin) * rep + rank, below the INT64_MAX sentinel
  if (rep > 1 && ((uint64_t)tmax - (uint64_t)tmin) > (uint64_t)((INT64_MAX - rep) / rep))
    return set_error(TSDB_E_NOT_IMPLEMENTED, "repeated timestamps over a time range too wide for the step keys");
  std::lock_guard<std::mutex> lk(ctx_mutex(c));
  if (hipSetDevice(ctx_device(c)) != hipSuccess) return set_error(TSDB_E_HIP, "hipSetDevice");
  hipStream_t st = ctx_stream(c);
  Scratch sc;
  auto release = [&]() {};
  void *d_prog, *d_consts, *d_sets, *d_fill, *d_ptr, *d_ts, *d_bits, *d_int, *d_act, *d_keys, *d_sorted, *d_uni, *d_nu;
  XOK(sc.alloc(&d_prog, n_ops * 8));
  XOK(sc.alloc(&d_consts, n_consts * 8));
  XOK(sc.alloc(&d_sets, n_sets * n_vars * 4));
  XOK(sc.alloc(&d_fill, n_vars * 8));
  XOK(sc.alloc(&d_ptr, (S + 1) * 8));
  XOK(sc.alloc(&d_ts, N * 8));
  XOK(sc.alloc(&d_bits, N * 8));
  XOK(sc.alloc(&d_int, N));
  XOK(sc.alloc(&d_act, N));
  XOK(sc.alloc(&d_keys, N * 8));
  XOK(sc.alloc(&d_sorted, N * 8));
  XOK(sc.alloc(&d_uni, N * 8));
  XOK(sc.alloc(&d_nu, 8));
  void* d_rank = nullptr;
  if (rep > 1) {
    XOK(sc.alloc(&d_rank, N * 4));
    XOK(hipMemcpyAsync(d_rank, prank.data(), N * 4, hipMemcpyHostToDevice, st));
  }
  XOK(hipMemcpyAsync(d_prog, program, n_ops * 8, hipMemcpyHostToDevice, st));
  if (n_consts) XOK(hipMemcpyAsync(d_consts, consts, n_consts * 8, hipMemcpyHostToDevice, st));
  if (n_sets) XOK(hipMemcpyAsync(d_sets, set_series, n_sets * n_vars * 4, hipMemcpyHostToDevice, st));
  XOK(hipMemcpyAsync(d_fill, var_fill, n_vars * 8, hipMemcpyHostToDevice, st));
  XOK(hipMemcpyAsync(d_ptr, in->ptr, (S + 1) * 8, hipMemcpyHostToDevice, st));
  if (N) {
    XOK(hipMemcpyAsync(d_ts, in->ts_ms, N * 8, hipMemcpyHostToDevice, st));
    XOK(hipMemcpyAsync(d_bits, in->value_bits, N * 8, hipMemcpyHostToDevice, st));
    XOK(hipMemcpyAsync(d_int, in->is_int, N, hipMemcpyHostToDevice, st));
    XOK(hipMemcpyAsync(d_act, pact.data(), N, hipMemcpyHostToDevice, st));
  }
  ExprSyncParams p{};
  p.prog = (const int32_t*)d_prog;
  p.n_ops = n_ops;
  p.consts = (const double*)d_consts;
  p.n_vars = n_vars;
  p.n_sets = n_sets;
  p.set_series = (const int32_t*)d_sets;
  p.var_fill = (const double*)d_fill;
  p.absent = absent_value;
  p.ptr = (const int64_t*)d_ptr;
  p.ts = (const int64_t*)d_ts;
  p.bits = (const uint64_t*)d_bits;
  p.is_int = (const uint8_t*)d_int;
  p.n_pts = N;
  p.pt_active = (const uint8_t*)d_act;
  p.start = start_ms;
  p.end = end_ms;
  p.rank = (const int32_t*)d_rank;
  p.rep = rep;
  p.base = rep > 1 ? tmin : 0;
  // the steps: the join iterator's nextTimestamp sequence = the distinct timestamps of the
  // active series (each in time order; with repeats the distinct (timestamp, rank) keys), sorted
  // and made unique on the device
  int64_t U = 0;
  if (N) {
    XOK(expr_sync_keys(p, (int64_t*)d_keys, st));
    size_t tmp1 = 0, tmp2 = 0;
    XOK(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp1, (const int64_t*)d_keys, (int64_t*)d_sorted, (int)N, 0, 64, st));
    XOK(hipcub::DeviceSelect::Unique(nullptr, tmp2, (const int64_t*)d_sorted, (int64_t*)d_uni, (int64_t*)d_nu, (int)N, st));
    void* d_tmp;
    size_t t1 = std::max(tmp1, tmp2), t2 = t1;
    XOK(sc.alloc(&d_tmp, t1));
    XOK(hipcub::DeviceRadixSort::SortKeys(d_tmp, t1, (const int64_t*)d_keys, (int64_t*)d_sorted, (int)N, 0, 64, st));
    XOK(hipcub::DeviceSelect::Unique(d_tmp, t2, (const int64_t*)d_sorted, (int64_t*)d_uni, (int64_t*)d_nu, (int)N, st));
    int64_t nu = 0, last = 0;
    XOK(hipMemcpyAsync(&nu, d_nu, 8, hipMemcpyDeviceToHost, st));
    XOK(hipStreamSynchronize(st));
    if (nu > 0) {
      XOK(hipMemcpyAsync(&last, (int64_t*)d_uni + nu - 1, 8, hipMemcpyDeviceToHost, st));
      XOK(hipStreamSynchronize(st));
    }
    U = nu - (nu > 0 && last == INT64_MAX ? 1 : 0);
  }
  const int64_t n_out = n_sets * U;
  void *o_ts, *o_bits, *o_int;
  XOK(sc.alloc(&o_ts, n_out * 8));
  XOK(sc.alloc(&o_bits, n_out * 8));
  XOK(sc.alloc(&o_int, n_out));
  p.uts = (const int64_t*)d_uni;
  p.U = U;
  p.out_ts = (int64_t*)o_ts;
  p.out_bits = (uint64_t*)o_bits;
  p.out_int = (uint8_t*)o_int;
  XOK(expr_sync(p, st));
  tsdbhip_result* r = new_result(n_sets, n_out);
  if (!r) return set_error(TSDB_E_NOMEM, "result");
  if (n_out) {
    XOK(hipMemcpyAsync(const_cast<int64_t*>(r->ts_ms), o_ts, n_out * 8, hipMemcpyDeviceToHost, st));
    XOK(hipMemcpyAsync(const_cast<uint64_t*>(r->value_bits), o_bits, n_out * 8, hipMemcpyDeviceToHost, st));
    XOK(hipMemcpyAsync(const_cast<uint8_t*>(r->is_int), o_int, n_out, hipMemcpyDeviceToHost, st));
  }
  XOK(hipStreamSynchronize(st));
  for (int64_t j = 0; j <= n_sets; j++) const_cast<int64_t*>(r->group_ptr)[j] = j * U;
  for (int64_t j = 0; j < n_sets; j++) const_cast<int32_t*>(r->group_id)[j] = (int32_t)j;
  *out = r;
  return 0;
}

namespace {

__global__ void k_topn_keys(const int64_t* ts, int64_t n, int64_t start, int64_t end, int64_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (ts[i] >= start && ts[i] <= end) ? ts[i] : INT64_MAX;
}

double key_double(uint64_t k) {   // inverse of k_expr.hip's dkey
  const uint64_t b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  double d;
  std::memcpy(&d, &b, 8);
  return d;
}
double java_max(double a, double b) {   // Math.max(double, double)
  if (a != a || b != b) return NAN;
  if (a == 0.0 && b == 0.0) return std::signbit(a) ? b : a;
  return a > b ? a : b;
}
int java_compare(double a, double b) {  // Double.compare
  if (a < b) return -1;
  if (a > b) return 1;
  const bool na = a != a, nb = b != b;
  if (na || nb) return na == nb ? 0 : (na ? 1 : -1);
  const bool sa = std::signbit(a), sb = std::signbit(b);   // -0.0 < 0.0
  return sa == sb ? 0 : (sa ? -1 : 1);
}

}  // namespace

extern "C" int tsdbhip_expr_topn(tsdbhip_ctx* c, int fn, int32_t topn, int64_t start_ms, int64_t end_ms,
                                 const tsdbhip_series_set* in, int32_t* out_index, int32_t* out_n) {
  if (!c || !out_n || (!out_index && in && in->n_series > 0)) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  *out_n = 0;
  if (int rc = check_set(in)) return rc;
  if (fn != TSDB_EXPR_HIGHEST_MAX && fn != TSDB_EXPR_HIGHEST_CURRENT)
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "unknown top-n function");
  if (topn < 1) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "Top n value must be greater than zero");
  const bool current = fn == TSDB_EXPR_HIGHEST_CURRENT;
  // the series the AggregationIterator walks: all of them (HighestMax.java:75-100) or those with
  // points (HighestCurrent.java:81-101); their points in one contiguous block each
  std::vector<int32_t> sel;
  std::vector<int64_t> ptr{0}, lo;
  for (int64_t s = 0; s < in->n_series; s++) {
    const int64_t a = in->ptr[s], b = in->ptr[s + 1];
    if (b < a) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "malformed series set");
    if (current && b == a) continue;
    for (int64_t q = a + 1; q < b; q++)
      if (in->ts_ms[q] <= in->ts_ms[q - 1]) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "series out of time order");
    sel.push_back((int32_t)s);
    ptr.push_back(ptr.back() + (b - a));
    lo.push_back(std::lower_bound(in->ts_ms + a, in->ts_ms + b, start_ms) - (in->ts_ms + a));   // seek(start)
  }
  const int64_t S = (int64_t)sel.size(), N = ptr.back();
  if (S == 0) return 0;
  std::lock_guard<std::mutex> lk(ctx_mutex(c));
  if (hipSetDevice(ctx_device(c)) != hipSuccess) return set_error(TSDB_E_HIP, "hipSetDevice");
  hipStream_t st = ctx_stream(c);
  Scratch sc;
  auto release = [&]() {};
  void *d_ptr, *d_ts, *d_bits, *d_int, *d_lo, *d_keys, *d_sorted, *d_uni, *d_nu, *d_ml, *d_md, *d_minm, *d_has, *d_last,
      *d_err;
  XOK(sc.alloc(&d_ptr, (S + 1) * 8));
  XOK(sc.alloc(&d_ts, N * 8));
  XOK(sc.alloc(&d_bits, N * 8));
  XOK(sc.alloc(&d_int, N));
  XOK(sc.alloc(&d_lo, S * 8));
  XOK(sc.alloc(&d_keys, N * 8));
  XOK(sc.alloc(&d_sorted, N * 8));
  XOK(sc.alloc(&d_uni, N * 8));
  XOK(sc.alloc(&d_nu, 8));
  XOK(sc.alloc(&d_ml, S * 8));
  XOK(sc.alloc(&d_md, S * 8));
  XOK(sc.alloc(&d_minm, 8));
  XOK(sc.alloc(&d_has, 8));
  XOK(sc.alloc(&d_last, 16));
  XOK(sc.alloc(&d_err, 16));
  XOK(hipMemcpyAsync(d_ptr, ptr.data(), (S + 1) * 8, hipMemcpyHostToDevice, st));
  XOK(hipMemcpyAsync(d_lo, lo.data(), S * 8, hipMemcpyHostToDevice, st));
  for (int64_t k = 0, o = 0; k < S; k++) {   // the selected series' points, back to back
    const int64_t a = in->ptr[sel[k]], n = in->ptr[sel[k] + 1] - a;
    if (!n) continue;
    XOK(hipMemcpyAsync((int64_t*)d_ts + o, in->ts_ms + a, n * 8, hipMemcpyHostToDevice, st));
    XOK(hipMemcpyAsync((uint64_t*)d_bits + o, in->value_bits + a, n * 8, hipMemcpyHostToDevice, st));
    XOK(hipMemcpyAsync((uint8_t*)d_int + o, in->is_int + a, n, hipMemcpyHostToDevice, st));
    o += n;
  }
  // union timestamps in [start, end]: the points the iterator emits (series in time order, seek
  // to start, hasNext while <= end), sorted and made unique on the device
  int64_t U = 0;
  if (N) {
    hipLaunchKernelGGL(k_topn_keys, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, (const int64_t*)d_ts, N, start_ms,
                       end_ms, (int64_t*)d_keys);
    XOK(hipGetLastError());
    size_t tmp1 = 0, tmp2 = 0;
    XOK(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp1, (const int64_t*)d_keys, (int64_t*)d_sorted, (int)N, 0, 64, st));
    XOK(hipcub::DeviceSelect::Unique(nullptr, tmp2, (const int64_t*)d_sorted, (int64_t*)d_uni, (int64_t*)d_nu, (int)N, st));
    void* d_tmp;
    XOK(sc.alloc(&d_tmp, std::max(tmp1, tmp2)));
    size_t t1 = std::max(tmp1, tmp2), t2 = t1;
    XOK(hipcub::DeviceRadixSort::SortKeys(d_tmp, t1, (const int64_t*)d_keys, (int64_t*)d_sorted, (int)N, 0, 64, st));
    XOK(hipcub::DeviceSelect::Unique(d_tmp, t2, (const int64_t*)d_sorted, (int64_t*)d_uni, (int64_t*)d_nu, (int)N, st));
    int64_t nu = 0, last = 0;
    XOK(hipMemcpyAsync(&nu, d_nu, 8, hipMemcpyDeviceToHost, st));
    XOK(hipStreamSynchronize(st));
    if (nu > 0) {
      XOK(hipMemcpyAsync(&last, (int64_t*)d_uni + nu - 1, 8, hipMemcpyDeviceToHost, st));
      XOK(hipStreamSynchronize(st));
    }
    U = nu - (nu > 0 && last == INT64_MAX ? 1 : 0);
  }
  // MaxCacheAggregator / MaxLatestAggregator initial arrays (HighestMax.java:212-215)
  std::vector<int64_t> ml(S, INT64_MIN);
  std::vector<uint64_t> md(S);
  {
    const double dmin = 4.9e-324;   // Double.MIN_VALUE
    uint64_t b;
    std::memcpy(&b, &dmin, 8);
    std::fill(md.begin(), md.end(), b | 0x8000000000000000ull);
  }
  const int32_t minm0[2] = {INT32_MAX, INT32_MAX}, has0[2] = {0, 0};
  const int64_t last0[2] = {0, 0};
  XOK(hipMemcpyAsync(d_ml, ml.data(), S * 8, hipMemcpyHostToDevice, st));
  XOK(hipMemcpyAsync(d_md, md.data(), S * 8, hipMemcpyHostToDevice, st));
  XOK(hipMemcpyAsync(d_minm, minm0, 8, hipMemcpyHostToDevice, st));
  XOK(hipMemcpyAsync(d_has, has0, 8, hipMemcpyHostToDevice, st));
  XOK(hipMemcpyAsync(d_last, last0, 16, hipMemcpyHostToDevice, st));
  XOK(hipMemsetAsync(d_err, 0, 16, st));
  ExprTopParams p{};
  p.n_series = S;
  p.ptr = (const int64_t*)d_ptr;
  p.ts = (const int64_t*)d_ts;
  p.bits = (const uint64_t*)d_bits;
  p.is_int = (const uint8_t*)d_int;
  p.lo = (const int64_t*)d_lo;
  p.uts = (const int64_t*)d_uni;
  p.U = U;
  p.current = current ? 1 : 0;
  p.max_l = (int64_t*)d_ml;
  p.max_d = (uint64_t*)d_md;
  p.min_m = (int32_t*)d_minm;
  p.has = (int32_t*)d_has;
  p.last_u = (int64_t*)d_last;
  p.err = (int32_t*)d_err;
  XOK(expr_topn(p, st));
  if (current) XOK(expr_topn_at(p, st));
  int32_t minm[2], has[2];
  XOK(hipMemcpyAsync(ml.data(), d_ml, S * 8, hipMemcpyDeviceToHost, st));
  XOK(hipMemcpyAsync(md.data(), d_md, S * 8, hipMemcpyDeviceToHost, st));
  XOK(hipMemcpyAsync(minm, d_minm, 8, hipMemcpyDeviceToHost, st));
  XOK(hipMemcpyAsync(has, d_has, 8, hipMemcpyDeviceToHost, st));
  XOK(hipStreamSynchronize(st));
  // the ranking over S values (HighestMax.java:118-146): positions past a point's operand count
  // read 0 (MaxCache: Math.max with it), then (double) / Math.max of the two arrays, then
  // TopNSortingEntry order (descending Double.compare; Arrays.sort is stable)
  std::vector<double> val(S);
  for (int64_t i = 0; i < S; i++) {
    int64_t l = ml[i];
    double d = key_double(md[i]);
    if (!current && has[0] && i >= minm[0]) l = std::max<int64_t>(l, 0);
    if (!current && has[1] && i >= minm[1]) d = java_max(d, 0.0);
    val[i] = has[0] && has[1] ? java_max((double)l, d) : (has[0] ? (double)l : d);
  }
  if (!has[0] && !has[1]) return set_error(TSDB_E_NULL_POINTER, "no datapoint in the query range (TopNSortingEntry left null)");
  std::vector<int32_t> order(S);
  for (int64_t i = 0; i < S; i++) order[i] = (int32_t)i;
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return java_compare(val[a], val[b]) > 0; });
  const int32_t cnt = (int32_t)std::min<int64_t>(topn, S);
  for (int32_t k = 0; k < cnt; k++) out_index[k] = sel[order[k]];
  *out_n = cnt;
  return 0;
}
