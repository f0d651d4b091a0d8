// expr.h -- internal declarations of the expression functions shared by
// expr.cpp and k_expr.hip.  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tsdb {

static constexpr int EXPR_STACK = 32;   // postfix program depth

struct ExprMapParams {
  int64_t n;                 // points
  const int64_t* ts;
  const uint64_t* bits;
  const uint8_t* is_int;
  const int64_t* lo;         // moving average: first emitted point of the point's series (-1: not emitted)
  int32_t fn;
  double fparam;
  int32_t scale_is_int;      // Scale: factor == floor(factor) && !isInfinite(factor)
  int32_t time_window;       // moving average: window in ms (else a point count)
  int64_t iparam;
  int64_t* out_ts;
  uint64_t* out_bits;
  uint8_t* out_int;
  int32_t* err;
};

struct ExprZipParams {
  const int32_t* prog;       // [2 * n_ops]
  int32_t n_ops;
  const double* consts;
  int32_t n_vars;
  int64_t n_sets;
  const int32_t* set_series; // [n_sets * n_vars]
  const double* var_fill;    // [n_vars]
  const int64_t* ptr;        // input series
  const int64_t* ts;
  const uint64_t* bits;
  const uint8_t* is_int;
  const int64_t* set_off;    // [n_sets + 1] output offsets
  int64_t n_out;
  int64_t* out_ts;
  uint64_t* out_bits;
  uint8_t* out_int;
  int32_t* err;
};

// time-synchronised evaluation (tsdbhip_expr_sync): steps = distinct timestamps of the active
// series' points in [start, end]
struct ExprSyncParams {
  const int32_t* prog;
  int32_t n_ops;
  const double* consts;
  int32_t n_vars;
  int64_t n_sets;
  const int32_t* set_series; // [n_sets * n_vars]
  const double* var_fill;    // [n_vars]
  double absent;             // a variable without a series in the set (UnionIterator fill_dp)
  const int64_t* ptr;        // input series
  const int64_t* ts;
  const uint64_t* bits;
  const uint8_t* is_int;
  int64_t n_pts;
  const uint8_t* pt_active;  // [n_pts] the point's series drives the steps
  int64_t start, end;
  const int32_t* rank;       // [n_pts] copies of the point's timestamp before it in its series (rep > 1)
  int64_t rep, base;         // rep > 1: step key = (ts - base) * rep + rank; rep == 1: key = ts
  const int64_t* uts;        // [U] step keys
  int64_t U;
  int64_t* out_ts;           // [n_sets * U]
  uint64_t* out_bits;
  uint8_t* out_int;
};
hipError_t expr_sync_keys(const ExprSyncParams& p, int64_t* keys, hipStream_t s);
hipError_t expr_sync(const ExprSyncParams& p, hipStream_t s);

// highestMax / highestCurrent: an AggregationIterator (LERP) over every result series, one
// wave per union point; operands kept by position among the spans that have a value
struct ExprTopParams {
  int64_t n_series;
  const int64_t* ptr;
  const int64_t* ts;
  const uint64_t* bits;
  const uint8_t* is_int;
  const int64_t* lo;          // [n_series] first point >= start (the constructor's seek)
  const int64_t* uts;         // [U] union timestamps in [start, end], ascending
  int64_t U;
  int32_t current;            // 1: MaxLatestAggregator, 0: MaxCacheAggregator
  int64_t* max_l;             // [n_series] positional long maxima (MaxCache) / latest (MaxLatest)
  uint64_t* max_d;            // [n_series] positional double maxima as order-preserving keys
  int32_t* min_m;             // [2] fewest spans with a value at a long / double point
  int32_t* has;               // [2] some long / double point ran
  int64_t* last_u;            // [2] MaxLatest: last long / double point
  int32_t* err;
};
hipError_t expr_topn(const ExprTopParams& p, hipStream_t s);      // the walk over every union point
hipError_t expr_topn_at(const ExprTopParams& p, hipStream_t s);   // MaxLatest: operands at the last points

hipError_t expr_map(const ExprMapParams& p, hipStream_t s);
hipError_t expr_zip(const ExprZipParams& p, hipStream_t s);

}  // namespace tsdb
