// kcommon.h -- device-side building blocks of libtsdbhip shared by the kernel
// translation units (k_grid.hip, k_fast.hip, k_misc.hip).  Header-only: every function is
// inline or a template, so each TU instantiates only the kernels it launches.
#pragma once
//
// The OpenTSDB query-time aggregation hot path (decode compacted cells -> per-series downsample -> cross-series group-by).
//
// The path is HBM-bound integer/byte work: no MFMA.  Design (DESIGN.md has the numbers):
//  * k_index   one wave per compacted row: classifies qualifier width / value length so
//              the main kernel can address datapoints directly (built once at load).
//  * k_grid    one wave per "tile" (<= T consecutive series of ONE SpanGroup).  For each
//              series the wave streams its rows in 512-datapoint chunks with 16-byte
//              coalesced loads, decodes qualifier+value in registers, stages the decoded
//              doubles in LDS, reduces every (series, bucket) segment sequentially in time
//              order (bit-exact with Downsampler's runDouble), then turns the series'
//              bucket stream into SpanGroup contributions (LERP / ZIM / MAX / MIN / PREV
//              interpolation, fill policies, RateSpan) accumulated into the tile's
//              per-slot partial state in LDS.  No atomics on the data path.
//  * k_reduce  merges tile partials of each group in tile (= series) order and finalises
//              the aggregator (AggregationIterator.doubleValue semantics).
#include "engine.h"

#include <float.h>
#include <math.h>
#include <type_traits>

#include "../../include/tsdbhip.h"

namespace tsdb {

#define WAVE_SYNC()                                          \
  do {                                                       \
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");   \
    __builtin_amdgcn_wave_barrier();                         \
  } while (0)

static constexpr int CH = CH_ROWS;      // datapoints per chunk (64 lanes x 8)
static constexpr int DPL = 8;           // datapoints per lane
static constexpr int VBUF = 4224;       // value staging bytes (aliases the decoded-double area)

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ void set_err(int32_t* err, int code) { atomicCAS(err, 0, code); }

// ---- wave scans (64 lanes) ------------------------------------------------
// ballot-based (no LDS round trip): lanes below this one in a 64-bit lane mask
__device__ __forceinline__ int lanes_below(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// inclusive prefix sum with DPP (gfx9 row_shr / row_bcast): 6 VALU ops, no LDS round trip
__device__ __forceinline__ int wave_incl_sum_dpp(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);   // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);   // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);   // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);   // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);   // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);   // row_bcast:31 -> rows 2, 3
  return x;
}
// exclusive prefix sum of small non-negative values (< 2^B), bit-sliced over ballots
template <int B>
__device__ __forceinline__ int wave_excl_sum_small(int x) {
  int r = 0;
#pragma unroll
  for (int b = 0; b < B; b++) r += lanes_below(__ballot((x >> b) & 1)) << b;
  return r;
}

__device__ __forceinline__ int wave_incl_sum(int x) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int y = __shfl_up(x, d, 64);
    if (l >= d) x += y;
  }
  return x;
}
__device__ __forceinline__ int wave_incl_max(int x) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int y = __shfl_up(x, d, 64);
    if (l >= d) x = max(x, y);
  }
  return x;
}
// Butterfly reductions: every lane holds the result; readfirstlane tells the compiler so
// (keeps loop-carried state that depends on it in SGPRs / uniform control flow).
__device__ __forceinline__ int wave_max(int x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x = max(x, __shfl_xor(x, d, 64));
  return __builtin_amdgcn_readfirstlane(x);
}
__device__ __forceinline__ int wave_min(int x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x = min(x, __shfl_xor(x, d, 64));
  return __builtin_amdgcn_readfirstlane(x);
}
__device__ __forceinline__ long long wave_sum64(long long x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
  return __builtin_amdgcn_readfirstlane(x);
}
// value of lane l (uniform result)
__device__ __forceinline__ int lane_bcast(int x, int l) { return __builtin_amdgcn_readlane(x, l); }

// Wave reduction by DPP (the inclusive-scan pattern of wave_incl_sum_dpp; lane 63 ends with the
// whole wave, returned as a uniform value).  op(a, b) combines, id is its identity; every lane
// must be active.
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_mov_f64(double x, double id) {
  const long long b = __double_as_longlong(x), ib = __double_as_longlong(id);
  const int lo = __builtin_amdgcn_update_dpp((int)ib, (int)b, CTRL, ROWS, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(ib >> 32), (int)(b >> 32), CTRL, ROWS, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
template <class Op>
__device__ __forceinline__ double wave_reduce_f64(double x, double id, Op op) {
  x = op(x, dpp_mov_f64<0x111, 0xF>(x, id));
  x = op(x, dpp_mov_f64<0x112, 0xF>(x, id));
  x = op(x, dpp_mov_f64<0x114, 0xF>(x, id));
  x = op(x, dpp_mov_f64<0x118, 0xF>(x, id));
  x = op(x, dpp_mov_f64<0x142, 0xA>(x, id));
  x = op(x, dpp_mov_f64<0x143, 0xC>(x, id));
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)b, 63), hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
template <class Op>
__device__ __forceinline__ int wave_reduce_i32(int x, int id, Op op) {
  x = op(x, __builtin_amdgcn_update_dpp(id, x, 0x111, 0xF, 0xF, false));
  x = op(x, __builtin_amdgcn_update_dpp(id, x, 0x112, 0xF, 0xF, false));
  x = op(x, __builtin_amdgcn_update_dpp(id, x, 0x114, 0xF, 0xF, false));
  x = op(x, __builtin_amdgcn_update_dpp(id, x, 0x118, 0xF, 0xF, false));
  x = op(x, __builtin_amdgcn_update_dpp(id, x, 0x142, 0xA, 0xF, false));
  x = op(x, __builtin_amdgcn_update_dpp(id, x, 0x143, 0xC, 0xF, false));
  return __builtin_amdgcn_readlane(x, 63);
}

// ---- big-endian value decode (RowSeq.extractIntegerValue / extractFloatingPointValue,
//      src/core/RowSeq.java:233-266); returns false on an illegal length -------------
__device__ __forceinline__ bool decode_value(uint64_t be_bits, int len, bool is_float, double& out) {
  // be_bits holds the len value bytes big-endian in its low len*8 bits
  if (is_float) {
    if (len == 4) { out = (double)__uint_as_float((uint32_t)be_bits); return true; }
    if (len == 8) { out = __longlong_as_double((long long)be_bits); return true; }
    return false;
  }
  switch (len) {
    case 1: out = (double)(int8_t)(uint8_t)be_bits; return true;
    case 2: out = (double)(int16_t)(uint16_t)be_bits; return true;
    case 4: out = (double)(int32_t)(uint32_t)be_bits; return true;
    case 8: out = (double)(long long)be_bits; return true;
  }
  return false;
}

// ---- slot of a datapoint ---------------------------------------------------
struct RowGeom {
  int64_t q0;   // slot index at the row base (when rel >= 0)
  int64_t r0;   // remainder (or negative rel)
};

__device__ __forceinline__ RowGeom row_geom(const GridParams& p, uint32_t base) {
  RowGeom g;
  const int64_t rel = (int64_t)base * 1000 - p.B0;
  if (rel >= 0) {
    g.q0 = rel / p.I;
    g.r0 = rel - g.q0 * p.I;
  } else {
    g.q0 = 0;
    g.r0 = rel;
  }
  return g;
}

// slot code of offset off_ms inside the row: its slot, -1 before slot 0 (before the seek point;
// ds_all: before the start), K at or after the last slot's end (ds_all: at or past the end)
__device__ __forceinline__ int slot_code(const GridParams& p, const RowGeom& g, uint32_t base, uint32_t off_ms) {
  if (p.mode == MODE_ALL) {
    const int64_t ts = (int64_t)base * 1000 + off_ms;
    return ts < p.qs ? -1 : ts < p.qe ? 0 : 1;
  }
  if (p.mode == MODE_TABLE) {   // variable-width calendar slots: bounds[lo] <= ts < bounds[lo + 1]
    const int64_t ts = (int64_t)base * 1000 + off_ms;
    if (ts < p.seek_ms || ts < p.bounds[0]) return -1;
    if (ts >= p.bounds[p.K]) return (int)p.K;
    int lo = 0, hi = (int)p.K;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (p.bounds[mid] <= ts) lo = mid; else hi = mid;
    }
    return lo;
  }
  const int64_t n = g.r0 + (int64_t)off_ms;
  if (n < 0) return -1;
  int64_t q;
  if (p.I < (1LL << 31)) {
    // n < I + 3.6e6 < 2^32: float reciprocal estimate, corrected to the exact quotient
    const uint32_t un = (uint32_t)n;
    const uint32_t I32 = (uint32_t)p.I;
    uint32_t qq = (uint32_t)((float)un * p.rcpI);
    int64_t r = (int64_t)un - (int64_t)qq * I32;
    if (r < 0) { qq--; r += I32; }
    if (r >= (int64_t)I32) { qq++; r -= I32; }
    if (r >= (int64_t)I32) { qq++; }
    q = qq;
  } else {
    q = n / p.I;
  }
  const int64_t s = g.q0 + q;
  return s < p.K ? (int)s : (int)p.K;
}

// slot of offset off_ms inside the row, -1 if before slot 0 or at/after K
__device__ __forceinline__ int slot_of(const GridParams& p, const RowGeom& g, uint32_t base, uint32_t off_ms) {
  const int k = slot_code(p, g, base, off_ms);
  return k < p.K ? k : -1;
}

// ---- stream order -----------------------------------------------------------------
// A span yields its datapoints as stored: Span.Iterator the rows in base-time order
// (Span.java:420-452), RowSeq.Iterator a row's cells in column order (RowSeq.java:552-568).
// ValuesInInterval takes every next value below the current interval's end
// (Downsampler.java:464-471) and otherwise moves the end past the value (:388-406), so a
// datapoint falls in the interval of the LARGEST timestamp its span has yielded so far: its own
// when the points are in time order, the one it follows when it recedes (cells out of order).
// Over slot codes (slot_code) that is a running max along the stored order.  The span starts at
// the seek point (Span.seekRow :360-380: the first row whose LAST cell is at or past it, then
// RowSeq.Iterator.seek :612-636: the first cell there that is): the max turns >= 0 at that
// cell, and so_row_skip drops the rows seekRow passes over.  Once the max reaches K the span
// has ended for the query.  ds_all (MODE_ALL) filters each value by [start, end) instead and
// ends the span at the first value past the end (ValuesInInterval.moveToNextValue :357-382).
// Over sorted rows every code is its own running max: the transform is the identity.
#define SLOT_NONE INT32_MIN   // no datapoint (lane past the row's end)
struct StreamOrd {
  int smax;   // running max slot code of the span's points so far (-1: not started)
};

// Timestamp (ms) of row d's last cell in column order (Internal.inMilliseconds per qualifier).
__device__ __forceinline__ int64_t row_last_ms(const GridParams& p, const RowDesc& d) {
  const uint8_t* q = p.qual + d.qoff;
  const int qw = d.flags & ROW_QW_MASK;
  uint32_t pos = 0;
  if (qw == 2 || qw == 4) {
    pos = (d.ndp - 1) * (uint32_t)qw;
  } else {
    uint32_t at = 0;
    for (uint32_t i = 0; i < d.ndp && at < d.qlen; i++) {
      pos = at;
      at += (q[at] & 0xF0) == 0xF0 ? 4 : 2;
    }
  }
  int64_t off;
  if (qw == 4 || (qw != 2 && (q[pos] & 0xF0) == 0xF0)) {
    const uint32_t w = ((uint32_t)q[pos] << 24) | ((uint32_t)q[pos + 1] << 16) | ((uint32_t)q[pos + 2] << 8) | q[pos + 3];
    off = (w & 0x0FFFFFC0u) >> 6;
  } else {
    off = (int64_t)(((((uint32_t)q[pos] << 8) | q[pos + 1]) >> 4) & 0xFFF) * 1000;
  }
  return (int64_t)d.base * 1000 + off;
}

// true: Span.seekRow passes over row d (the span has not started, d is not its last row in the
// scan, and d's last cell lies before the seek point -- only a row out of order can hold a cell
// at or past the seek point before that one)
__device__ __forceinline__ bool so_row_skip(const GridParams& p, const StreamOrd& so, const RowDesc& d,
                                            bool last_row) {
  if (so.smax >= 0 || last_row || !(d.flags & ROW_UNSORTED) || d.ndp == 0) return false;
  return row_last_ms(p, d) < p.seek_any;
}

// Slot codes of the lane's DPL consecutive points (lanes in stored order) -> slots (-1: none).
__device__ __forceinline__ void so_apply(const GridParams& p, StreamOrd& so, int slot[DPL], bool skip_row) {
  const int K = (int)p.K;
  const int lane = lane_id();
  int run[DPL];
  int m = INT32_MIN;
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    if (skip_row) slot[j] = SLOT_NONE;
    if (slot[j] != SLOT_NONE) m = max(m, slot[j]);
    run[j] = m;
  }
  int incl = m;   // inclusive max scan over the lanes
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o, 64);
    if (lane >= o) incl = max(incl, y);
  }
  int excl = __shfl_up(incl, 1, 64);
  if (lane == 0) excl = INT32_MIN;
  excl = max(excl, so.smax);
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    if (slot[j] == SLOT_NONE) { slot[j] = -1; continue; }
    const int e = max(excl, run[j]);
    if (p.mode == MODE_ALL) slot[j] = (slot[j] == 0 && e < K) ? 0 : -1;
    else slot[j] = (e >= 0 && e < K) ? e : -1;
  }
  so.smax = max(so.smax, __shfl(incl, 63, 64));
}

// ---- per-bucket downsample state (Aggregator.runDouble over a bucket, in order) ----
struct BState {
  double a, b;
  long long n;
};

template <int F>
__device__ __forceinline__ void bs_init(BState& s) {
  s.b = 0.0;
  s.n = 0;
  if (F == F_MIN) s.a = INFINITY;
  else if (F == F_MAX) s.a = -INFINITY;
  else if (F == F_DIFF) { s.a = 0.0; s.n = -1; }
  else s.a = 0.0;
}

// Aggregators.java: Sum :246-259, SquareSum :280-293, Min :315-327, Max :349-361, Avg :382-393,
// StdDev :526-569, Diff :598-617, Count :636-645, Multiply :479-485, First :823-829, Last :845-851
template <int F>
__device__ __forceinline__ void bs_add(BState& s, double x) {
  if (F == F_SUM || F == F_AVG) {
    if (!isnan(x)) { s.a += x; s.n++; }
  } else if (F == F_SQUARESUM) {
    if (!isnan(x)) { s.a += x * x; s.n++; }
  } else if (F == F_COUNT) {
    if (!isnan(x)) s.n++;
  } else if (F == F_MIN) {
    if (!isnan(x) && x < s.a) s.a = x;
  } else if (F == F_MAX) {
    if (!isnan(x) && x > s.a) s.a = x;
  } else if (F == F_DEV) {
    if (!isnan(x)) {
      if (s.n == 0) {
        s.a = x;
      } else {
        const double old = s.a;
        const double nm = old + (x - old) / (double)(s.n + 1);
        s.b += (x - old) * (x - nm);
        s.a = nm;
      }
      s.n++;
    }
  } else if (F == F_FIRST) {
    if (s.n == 0) s.a = x;
    s.n++;
  } else if (F == F_LAST) {
    s.a = x;
    s.n++;
  } else if (F == F_DIFF) {
    if (s.n < 0) {
      if (!isnan(x)) { s.a = x; s.n = 0; }
    } else {
      s.n++;
    }
    s.b = x;
  } else if (F == F_MULT) {
    s.a = (s.b != 0.0) ? s.a * x : x;   // b used as "has value" flag
    s.b = 1.0;
  }
}

template <int F>
__device__ __forceinline__ double bs_final(const BState& s) {
  if (F == F_SUM || F == F_SQUARESUM) return s.n == 0 ? (double)NAN : s.a;
  if (F == F_AVG) return s.n == 0 ? (double)NAN : s.a / (double)(int)s.n;
  if (F == F_COUNT) return (double)s.n;
  if (F == F_MIN) return s.a == INFINITY ? (double)NAN : s.a;
  if (F == F_MAX) return s.a == -INFINITY ? (double)NAN : s.a;
  if (F == F_DEV) return s.n == 0 ? (double)NAN : (s.n == 1 ? 0.0 : sqrt(s.b / (double)s.n));
  if (F == F_FIRST || F == F_LAST) return s.a;
  if (F == F_DIFF) return s.n < 0 ? (double)NAN : (s.n == 0 ? 0.0 : s.b - s.a);
  if (F == F_MULT) return s.a;
  return NAN;
}

// ---- SpanGroup contributions into the tile's per-slot partial state ----------------
struct LdsPart {
  double* a;
  double* b;
  uint32_t* n;
  uint32_t* f;
};

__device__ __forceinline__ void part_init(int ga, const LdsPart& P, int k) {
  P.a[k] = (ga == GA_MIN) ? INFINITY : (ga == GA_MAX ? -INFINITY : 0.0);
  P.b[k] = 0.0;
  P.n[k] = 0;
  P.f[k] = 0;
}

// Slot accessors: the same contribution code updates LDS partials (slot s of a tile
// array) or register partials (the lane's own slot, K <= 64).
struct LdsSlot {
  const LdsPart& P;
  int s;
  __device__ double& a() const { return P.a[s]; }
  __device__ double& b() const { return P.b[s]; }
  __device__ uint32_t& n() const { return P.n[s]; }
  __device__ uint32_t& f() const { return P.f[s]; }
};

struct RegPart {
  double pa, pb;
  uint32_t pn, pf;
  __device__ double& a() { return pa; }
  __device__ double& b() { return pb; }
  __device__ uint32_t& n() { return pn; }
  __device__ uint32_t& f() { return pf; }
};

// AggregationIterator feeding Aggregator.runDouble, one span at a time in index order.
template <class S>
__device__ __forceinline__ void contribute_slot(int ga, S&& P, double v, bool uni) {
  uint32_t f = P.f();
  switch (ga) {
    case GA_SUM: case GA_AVG:
      if (!isnan(v)) { P.a() += v; P.n()++; }
      break;
    case GA_SQUARESUM:
      if (!isnan(v)) { P.a() += v * v; P.n()++; }
      break;
    case GA_COUNT:
      if (!isnan(v)) P.n()++;
      break;
    case GA_MIN:
      if (!isnan(v) && v < P.a()) P.a() = v;
      break;
    case GA_MAX:
      if (!isnan(v) && v > P.a()) P.a() = v;
      break;
    case GA_DEV:
      if (!isnan(v)) {
        const uint32_t c = P.n();
        if (c == 0) {
          P.a() = v;
        } else {
          const double m = P.a();
          const double nm = m + (v - m) / (double)(c + 1);
          P.b() += (v - m) * (v - nm);
          P.a() = nm;
        }
        P.n() = c + 1;
      }
      break;
    case GA_FIRST: case GA_NONE:
      if (!(f & PF_HAS)) { P.a() = v; f |= PF_HAS; }
      f += 4;
      break;
    case GA_LAST:
      P.a() = v;
      f |= PF_HAS;
      f += 4;
      break;
    case GA_DIFF:
      if (!(f & PF_HAS)) {
        if (!isnan(v)) { P.a() = v; f |= PF_HAS; P.n() = 0; }
      } else {
        P.n()++;
      }
      P.b() = v;
      f += 4;
      break;
    case GA_MULT:
      P.a() = (f & PF_HAS) ? P.a() * v : v;
      f |= PF_HAS;
      f += 4;
      break;
  }
  if (uni) f |= PF_UNION;
  P.f() = f;
}

__device__ __forceinline__ void contribute(int ga, const LdsPart& P, int s, double v, bool uni) {
  contribute_slot(ga, LdsSlot{P, s}, v, uni);
}

__device__ __forceinline__ void regpart_init(int ga, RegPart& P) {
  P.pa = (ga == GA_MIN) ? INFINITY : (ga == GA_MAX ? -INFINITY : 0.0);
  P.pb = 0.0;
  P.pn = 0;
  P.pf = 0;
}

// Interpolation of a missing slot (AggregationIterator.nextDoubleValue, :773-793)
// timestamp of slot k relative to slot 0 (ms)
__device__ __forceinline__ long long slot_rel(const GridParams& p, int k) {
  return p.mode == MODE_TABLE ? (long long)(p.bounds[k] - p.bounds[0]) : (long long)k * p.I;
}

__device__ __forceinline__ double interp(int method, const GridParams& p, int k0, double y0, int k1, double y1, int k) {
  switch (method) {
    case TSDB_INTERP_LERP: {
      const long long x = slot_rel(p, k), x0 = slot_rel(p, k0), x1 = slot_rel(p, k1);
      return y0 + (double)(x - x0) * (y1 - y0) / (double)(x1 - x0);
    }
    case TSDB_INTERP_ZIM: return 0.0;
    case TSDB_INTERP_MAX: return DBL_MAX;
    case TSDB_INTERP_MIN: return 4.9e-324;
    default: return y0;
  }
}

// value of a raw datapoint as a double (DataPoint.toDouble)
__device__ __forceinline__ double pt_double(int64_t tsf, uint64_t bits) {
  return (tsf & RAW_FLOAT) ? __longlong_as_double((long long)bits) : (double)(long long)bits;
}

// ---- exactness certificate helpers ---------------------------------------------------
// lsb(x): exponent of the least significant set bit of a finite non-zero double.
__device__ __forceinline__ int lsb_exp(double x) {
  const unsigned long long bits = (unsigned long long)__double_as_longlong(x);
  const int E = (int)((bits >> 52) & 0x7FF);
  const unsigned long long M = bits & 0xFFFFFFFFFFFFFULL;
  if (E == 0) return -1074 + __ffsll((long long)M) - 1;
  return E - 1075 + __ffsll((long long)(M | 0x10000000000000ULL)) - 1;
}


// ---- k_grid ---------------------------------------------------------------------
struct WaveLds {
  double* dpv;          // [CH] decoded values; aliases the vle byte staging and mixed-row scratch
  uint8_t* vbuf;
  uint32_t* mq;         // [CH] mixed-row scratch: off_ms
  uint32_t* mv;         // [CH] mixed-row scratch: value offset | len<<24 | float<<31
  int32_t* seg_slot;    // [CH]
  uint16_t* seg_start;  // [CH+1]
  double* dense;        // [K] per-series bucket values
  uint8_t* pres;        // [K] bucket present
  double* rate;         // [K] rate values (rate mode)
  LdsPart part;         // [K] tile partials
};

__host__ __device__ inline int64_t align16(int64_t x) { return (x + 15) & ~(int64_t)15; }

// fixed per-wave LDS (decode staging + segment lists)
__host__ __device__ constexpr int64_t fixed_lds_bytes() { return VBUF + CH * 4 + ((CH + 1) * 2 + 15) / 16 * 16; }

__host__ __device__ inline int64_t slot_lds_bytes(int64_t K, bool rate) {
  int64_t o = align16(K * 8) + align16(K);
  if (rate) o += align16(K * 8);
  o += align16(K * 8) * 2 + align16(K * 4) * 2;
  return o;
}

template <bool GSLOT>
__device__ inline WaveLds carve(const GridParams& p, unsigned char* base, int64_t tile, int64_t K, bool rate) {
  WaveLds w;
  int64_t o = 0;
  w.dpv = (double*)(base + o);
  w.vbuf = base + o;
  w.mq = (uint32_t*)(base + o);
  w.mv = (uint32_t*)(base + o + CH * 4);
  o += VBUF;
  w.seg_slot = (int32_t*)(base + o); o += CH * 4;
  w.seg_start = (uint16_t*)(base + o); o += align16((CH + 1) * 2);
  if (GSLOT) {
    w.dense = p.g_dense + tile * K;
    w.pres = p.g_pres + tile * K;
    w.rate = rate ? p.g_rate + tile * K : nullptr;
    w.part.a = p.part.a + tile * K;
    w.part.b = p.part.b + tile * K;
    w.part.n = p.part.n + tile * K;
    w.part.f = p.part.f + tile * K;
  } else {
    w.dense = (double*)(base + o); o += align16(K * 8);
    w.pres = base + o; o += align16(K);
    if (rate) { w.rate = (double*)(base + o); o += align16(K * 8); } else { w.rate = nullptr; }
    w.part.a = (double*)(base + o); o += align16(K * 8);
    w.part.b = (double*)(base + o); o += align16(K * 8);
    w.part.n = (uint32_t*)(base + o); o += align16(K * 4);
    w.part.f = (uint32_t*)(base + o); o += align16(K * 4);
  }
  return w;
}

// Raw bytes of one lane's 8 datapoints of a uniform row (qualifier width 2/4, value length 1/2/4/8)
struct Raw {
  uint4 q0, q1;
  uint4 v0, v1, v2, v3;
};

__device__ __forceinline__ bool row_uniform(const RowDesc& d) {
  return (d.flags & ROW_QW_MASK) != 0 && (d.flags & ROW_VL_MASK) != 0 && !(d.flags & ROW_ERR);
}

__device__ __forceinline__ void load_raw(const GridParams& p, const RowDesc& d, int64_t c0, Raw& rw) {
  const int lane = lane_id();
  const int64_t i0 = c0 + (int64_t)lane * DPL;
  if (i0 >= (int64_t)d.ndp) return;
  const int qw = d.flags & ROW_QW_MASK;
  const int vl = (d.flags & ROW_VL_MASK) >> ROW_VL_SHIFT;
  const uint8_t* q = p.qual + d.qoff + i0 * qw;
  const uint8_t* v = p.val + d.voff + i0 * vl;
  rw.q0 = *reinterpret_cast<const uint4*>(q);
  if (qw == 4) rw.q1 = *reinterpret_cast<const uint4*>(q + 16);
  if (vl == 1) {
    const uint2 t = *reinterpret_cast<const uint2*>(v);
    rw.v0 = make_uint4(t.x, t.y, 0, 0);
  } else {
    rw.v0 = *reinterpret_cast<const uint4*>(v);
    if (vl >= 4) rw.v1 = *reinterpret_cast<const uint4*>(v + 16);
    if (vl == 8) {
      rw.v2 = *reinterpret_cast<const uint4*>(v + 32);
      rw.v3 = *reinterpret_cast<const uint4*>(v + 48);
    }
  }
}

// Decodes the lane's 8 datapoints of a uniform row from raw registers into (slot, value).
// CODE: slot codes (slot_code, SLOT_NONE past the row's end) for so_apply, else slots
template <bool CODE = false>
__device__ __forceinline__ void decode_raw(const GridParams& p, const RowDesc& d, const RowGeom& g, int64_t c0,
                                           const Raw& rw, int slot[DPL], double val[DPL]) {
  const int lane = lane_id();
  const int64_t i0 = c0 + (int64_t)lane * DPL;
  const int nv = (int)max((int64_t)0, min((int64_t)DPL, (int64_t)d.ndp - i0));
  const int qw = d.flags & ROW_QW_MASK;
  const int vl = (d.flags & ROW_VL_MASK) >> ROW_VL_SHIFT;
  uint32_t off[DPL], fl[DPL];
  if (qw == 2) {
    const uint32_t ws[4] = {rw.q0.x, rw.q0.y, rw.q0.z, rw.q0.w};
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      const uint32_t be = __builtin_bswap32(ws[j >> 1]);
      const uint32_t qq = (j & 1) ? (be & 0xFFFF) : (be >> 16);
      off[j] = (qq >> 4) * 1000u;
      fl[j] = qq & 0xF;
    }
  } else {
    const uint32_t ws[8] = {rw.q0.x, rw.q0.y, rw.q0.z, rw.q0.w, rw.q1.x, rw.q1.y, rw.q1.z, rw.q1.w};
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      const uint32_t qq = __builtin_bswap32(ws[j]);
      off[j] = (qq & 0x0FFFFFC0u) >> 6;
      fl[j] = qq & 0xF;
    }
  }
  if (vl == 4) {
    const uint32_t ws[8] = {rw.v0.x, rw.v0.y, rw.v0.z, rw.v0.w, rw.v1.x, rw.v1.y, rw.v1.z, rw.v1.w};
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      const uint32_t be = __builtin_bswap32(ws[j]);
      val[j] = (fl[j] & 8) ? (double)__uint_as_float(be) : (double)(int32_t)be;
    }
  } else if (vl == 8) {
    const uint32_t ws[16] = {rw.v0.x, rw.v0.y, rw.v0.z, rw.v0.w, rw.v1.x, rw.v1.y, rw.v1.z, rw.v1.w,
                             rw.v2.x, rw.v2.y, rw.v2.z, rw.v2.w, rw.v3.x, rw.v3.y, rw.v3.z, rw.v3.w};
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      const uint64_t a = ((uint64_t)__builtin_bswap32(ws[2 * j]) << 32) | __builtin_bswap32(ws[2 * j + 1]);
      val[j] = (fl[j] & 8) ? __longlong_as_double((long long)a) : (double)(long long)a;
    }
  } else if (vl == 2) {
    const uint32_t ws[4] = {rw.v0.x, rw.v0.y, rw.v0.z, rw.v0.w};
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      const uint32_t be = __builtin_bswap32(ws[j >> 1]);
      const uint32_t x = (j & 1) ? (be & 0xFFFF) : (be >> 16);
      val[j] = (double)(int16_t)(uint16_t)x;
    }
  } else {
    const uint32_t ws[2] = {rw.v0.x, rw.v0.y};
#pragma unroll
    for (int j = 0; j < DPL; j++) val[j] = (double)(int8_t)((ws[j >> 2] >> ((j & 3) * 8)) & 0xFF);
  }
#pragma unroll
  for (int j = 0; j < DPL; j++)
    slot[j] = (j < nv) ? (CODE ? slot_code(p, g, d.base, off[j]) : slot_of(p, g, d.base, off[j])) : (CODE ? SLOT_NONE : -1);
}

// Generic decode (variable-length values, mixed qualifier widths); loads inside.
template <bool CODE = false>
__device__ __forceinline__ void decode_generic(const GridParams& p, const RowDesc& d, const RowGeom& g, int64_t c0,
                               const WaveLds& W, int64_t& vcur, int slot[DPL], double val[DPL]) {
  const int lane = lane_id();
  const int64_t i0 = c0 + (int64_t)lane * DPL;
  const int nv = (int)max((int64_t)0, min((int64_t)DPL, (int64_t)d.ndp - i0));
  const int qw = d.flags & ROW_QW_MASK;
  const uint8_t* q = p.qual + d.qoff;
  const uint8_t* v = p.val + d.voff;
  uint32_t off[DPL], fl[DPL];
#pragma unroll
  for (int j = 0; j < DPL; j++) { off[j] = 0; fl[j] = 0; slot[j] = CODE ? SLOT_NONE : -1; val[j] = 0.0; }
  WAVE_SYNC();
  if (qw == 2 || qw == 4) {
    if (nv > 0) {
      if (qw == 2) {
        const uint4 w = *reinterpret_cast<const uint4*>(q + i0 * 2);
        const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int j = 0; j < DPL; j++) {
          const uint32_t be = __builtin_bswap32(ws[j >> 1]);
          const uint32_t qq = (j & 1) ? (be & 0xFFFF) : (be >> 16);
          off[j] = (qq >> 4) * 1000u;
          fl[j] = qq & 0xF;
        }
      } else {
        const uint4 w0 = *reinterpret_cast<const uint4*>(q + i0 * 4);
        const uint4 w1 = *reinterpret_cast<const uint4*>(q + i0 * 4 + 16);
        const uint32_t ws[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
        for (int j = 0; j < DPL; j++) {
          const uint32_t qq = __builtin_bswap32(ws[j]);
          off[j] = (qq & 0x0FFFFFC0u) >> 6;
          fl[j] = qq & 0xF;
        }
      }
    }
    // variable-length values: wave prefix scan of lengths, stage the chunk's bytes in LDS
    int len[DPL];
    int loc = 0;
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      len[j] = (j < nv) ? (int)(fl[j] & 7) + 1 : 0;
      loc += len[j];
    }
    const int incl = wave_incl_sum(loc);
    const int total = __shfl(incl, 63, 64);
    const int excl = incl - loc;
    const int64_t start = (int64_t)d.voff + vcur;
    const int64_t a0 = start & ~(int64_t)15;
    const int64_t lead = start - a0;
    const int npieces = (int)((lead + total + 15) >> 4);
    for (int pc = lane; pc < npieces; pc += 64)
      reinterpret_cast<uint4*>(W.vbuf)[pc] = *reinterpret_cast<const uint4*>(p.val + a0 + pc * 16);
    WAVE_SYNC();
    int o = (int)lead + excl;
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      if (j < nv) {
        uint64_t bits = 0;
        for (int b = 0; b < len[j]; b++) bits = (bits << 8) | W.vbuf[o + b];
        double x = 0.0;
        if (!decode_value(bits, len[j], (fl[j] & 8) != 0, x)) set_err(p.err, TSDB_E_ILLEGAL_DATA);
        val[j] = x;
        slot[j] = CODE ? slot_code(p, g, d.base, off[j]) : slot_of(p, g, d.base, off[j]);
      }
      o += len[j];
    }
    vcur += total;
  } else {
    // mixed s/ms row: lane 0 walks the chunk (RowSeq.Iterator.next, :552-568); positions in vcur
    if (lane == 0) {
      uint32_t qi = (uint32_t)(vcur & 0xFFFFFFFF), vi = (uint32_t)(vcur >> 32);
      for (int t = 0; t < CH && c0 + t < (int64_t)d.ndp; t++) {
        const bool ms = (q[qi] & 0xF0) == 0xF0;
        uint32_t qq;
        if (ms) { qq = ((uint32_t)q[qi] << 24) | ((uint32_t)q[qi + 1] << 16) | ((uint32_t)q[qi + 2] << 8) | q[qi + 3]; qi += 4; }
        else { qq = ((uint32_t)q[qi] << 8) | q[qi + 1]; qi += 2; }
        const uint32_t f = qq & 0xF;
        const uint32_t len = (f & 7) + 1;
        W.mq[t] = ms ? ((qq & 0x0FFFFFC0u) >> 6) : ((qq >> 4) & 0xFFF) * 1000u;
        W.mv[t] = vi | (len << 24) | ((f & 8) ? 0x80000000u : 0u);
        vi += len;
      }
      vcur = ((int64_t)vi << 32) | qi;
    }
    vcur = __shfl(vcur, 0, 64);
    WAVE_SYNC();
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      if (j < nv) {
        const int t = lane * DPL + j;
        const uint32_t mvv = W.mv[t];
        const uint32_t vo = mvv & 0xFFFFFF;
        const int len = (mvv >> 24) & 0x7F;
        uint64_t bits = 0;
        for (int b = 0; b < len; b++) bits = (bits << 8) | v[vo + b];
        double x = 0.0;
        if (!decode_value(bits, len, (mvv >> 31) != 0, x)) set_err(p.err, TSDB_E_ILLEGAL_DATA);
        val[j] = x;
        slot[j] = CODE ? slot_code(p, g, d.base, W.mq[t]) : slot_of(p, g, d.base, W.mq[t]);
      }
    }
  }
  WAVE_SYNC();
}

// ---- fast per-bucket reduction: order-free state combined across lanes ----------------
// Used for downsample functions whose result is exact in any association order: min, max,
// count, first, last, and sum / avg / squareSum under the exactness certificate.
template <int F>
__device__ __forceinline__ constexpr bool fast_capable() {
  return F == F_SUM || F == F_AVG || F == F_COUNT || F == F_SQUARESUM || F == F_MIN || F == F_MAX ||
         F == F_FIRST || F == F_LAST;
}
template <int F>
__device__ __forceinline__ constexpr bool needs_cert() {
  return F == F_SUM || F == F_AVG || F == F_SQUARESUM;
}

struct FS {
  double v;
  int n;
};

template <int F>
__device__ __forceinline__ FS fs_id() {
  FS s;
  s.v = (F == F_MIN) ? (double)INFINITY : (F == F_MAX ? -(double)INFINITY : 0.0);
  s.n = 0;
  return s;
}
template <int F>
__device__ __forceinline__ FS fs_of(double x) {
  FS s = fs_id<F>();
  if (F == F_FIRST || F == F_LAST) { s.v = x; s.n = 1; return s; }
  if (isnan(x)) return s;
  if (F == F_SQUARESUM) s.v = x * x;
  else if (F != F_COUNT) s.v = x;
  s.n = 1;
  return s;
}
template <int F>
__device__ __forceinline__ FS fs_op(const FS& a, const FS& b) {
  FS r;
  if (F == F_MIN) { r = (b.v < a.v) ? b : a; return r; }
  if (F == F_MAX) { r = (b.v > a.v) ? b : a; return r; }
  if (F == F_FIRST) return a.n ? a : b;
  if (F == F_LAST) return b.n ? b : a;
  r.v = (F == F_COUNT) ? 0.0 : a.v + b.v;
  r.n = a.n + b.n;
  return r;
}
template <int F>
__device__ __forceinline__ double fs_final(const FS& s) {
  if (F == F_SUM || F == F_SQUARESUM) return s.n == 0 ? (double)NAN : s.v;
  if (F == F_AVG) return s.n == 0 ? (double)NAN : s.v / (double)s.n;
  if (F == F_COUNT) return (double)s.n;
  if (F == F_MIN) return s.v == INFINITY ? (double)NAN : s.v;
  if (F == F_MAX) return s.v == -INFINITY ? (double)NAN : s.v;
  return s.v;
}

__device__ __forceinline__ FS shfl_up_fs(const FS& s, int d) {
  FS r;
  r.v = __shfl_up(s.v, d, 64);
  r.n = __shfl_up(s.n, d, 64);
  return r;
}
__device__ __forceinline__ FS shfl_fs(const FS& s, int src) {
  FS r;
  r.v = __shfl(s.v, src, 64);
  r.n = __shfl(s.n, src, 64);
  return r;
}

// Per-series state carried across chunks / rows.
struct SeriesState {
  int carry_slot;
  FS fcarry;       // fast-path open bucket
  BState scarry;   // slow-path open bucket
  int nmax;        // largest bucket (datapoint count) emitted by the fast path
};

template <int F>
__device__ __forceinline__ void emit_bucket(const WaveLds& W, int k, double v) {
  W.dense[k] = v;
  W.pres[k] = 1;
}

// Fast path: segmented reduction of one decoded chunk, keys = slots (non-decreasing).
template <int F>
__device__ __forceinline__ void fast_chunk(const WaveLds& W, SeriesState& st, const int slot[DPL], const double val[DPL]) {
  const int lane = lane_id();
  int kf = -1, kl = -1, cur_key = -1, nruns = 0;
  FS Pf = fs_id<F>(), cur = fs_id<F>();
  int mymax = 0;
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    if (slot[j] < 0) continue;
    const FS x = fs_of<F>(val[j]);
    if (slot[j] != cur_key) {
      if (cur_key >= 0) {
        if (nruns == 1) { Pf = cur; kf = cur_key; }
        else { emit_bucket<F>(W, cur_key, fs_final<F>(cur)); mymax = max(mymax, cur.n); }
      }
      cur_key = slot[j];
      cur = x;
      nruns++;
    } else {
      cur = fs_op<F>(cur, x);
    }
  }
  FS Pl = cur;
  kl = cur_key;
  if (nruns == 1) { kf = kl; Pf = Pl; }
  const bool has = nruns > 0;
  const bool multi = nruns >= 2;
  const unsigned long long hm = __ballot(has);
  if (hm == 0) return;
  const int fv = __ffsll((long long)hm) - 1;          // first lane with datapoints
  const int lv = 63 - __clzll((long long)hm);        // last lane with datapoints
  // open bucket from the previous chunk
  const int kf_fv = __shfl(kf, fv, 64);
  if (st.carry_slot >= 0) {
    if (kf_fv == st.carry_slot) {
      if (lane == fv) {
        Pf = fs_op<F>(st.fcarry, Pf);
        if (!multi) Pl = Pf;
      }
    } else if (lane == 0) {
      emit_bucket<F>(W, st.carry_slot, fs_final<F>(st.fcarry));
      mymax = max(mymax, st.fcarry.n);
    }
  }
  // segmented inclusive scan of the last runs
  const int kl_prev = __shfl_up(kl, 1, 64);
  int h = (!has || multi || lane == 0 || kl_prev != kf) ? 1 : 0;
  FS T = has ? Pl : fs_id<F>();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const FS To = shfl_up_fs(T, d);
    const int ho = __shfl_up(h, d, 64);
    if (lane >= d) {
      if (!h) T = fs_op<F>(To, T);
      h |= ho;
    }
  }
  const FS Tprev = shfl_up_fs(T, 1);
  const int kf_next = __shfl_down(kf, 1, 64);
  if (has && multi) {
    const FS tot = (lane > 0 && kl_prev == kf && lane > fv) ? fs_op<F>(Tprev, Pf) : Pf;
    emit_bucket<F>(W, kf, fs_final<F>(tot));
    mymax = max(mymax, tot.n);
  }
  if (has && lane != lv && kf_next != kl) {
    emit_bucket<F>(W, kl, fs_final<F>(T));
    mymax = max(mymax, T.n);
  }
  st.carry_slot = __shfl(kl, lv, 64);
  st.fcarry = shfl_fs(T, lv);
  st.nmax = max(st.nmax, wave_max(mymax));
}

// Slow path: every (series, bucket) reduced sequentially in time order (bit-exact always).
template <int F>
__device__ __forceinline__ void slow_chunk(const WaveLds& W, SeriesState& st, const int slot[DPL], const double val[DPL]) {
  const int lane = lane_id();
  WAVE_SYNC();
#pragma unroll
  for (int j = 0; j < DPL; j++) W.dpv[lane * DPL + j] = val[j];
  const int prev_last = __shfl_up(slot[DPL - 1], 1, 64);
  int h = 0;
  bool head[DPL];
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    const int ps = (j == 0) ? (lane == 0 ? -2 : prev_last) : slot[j - 1];
    head[j] = slot[j] >= 0 && (ps < 0 || ps != slot[j]);
    h += head[j];
  }
  int vend = 0;
#pragma unroll
  for (int j = 0; j < DPL; j++) if (slot[j] >= 0) vend = lane * DPL + j + 1;
  vend = wave_max(vend);
  const int hincl = wave_incl_sum(h);
  const int nseg = __shfl(hincl, 63, 64);
  int pos = hincl - h;
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    if (head[j]) {
      W.seg_start[pos] = (uint16_t)(lane * DPL + j);
      W.seg_slot[pos] = slot[j];
      pos++;
    }
  }
  if (lane == 0) W.seg_start[nseg] = (uint16_t)vend;
  WAVE_SYNC();
  if (nseg == 0) return;
  const int first_slot = W.seg_slot[0];
  if (st.carry_slot >= 0 && first_slot != st.carry_slot) {
    if (lane == 0) emit_bucket<F>(W, st.carry_slot, bs_final<F>(st.scarry));
    st.carry_slot = -1;
    bs_init<F>(st.scarry);
  }
  for (int b0 = 0; b0 < nseg; b0 += 64) {
    const int si = b0 + lane;
    const bool act = si < nseg;
    BState s;
    bs_init<F>(s);
    int myslot = -1;
    if (act) {
      myslot = W.seg_slot[si];
      if (si == 0 && myslot == st.carry_slot) s = st.scarry;
      const int e = W.seg_start[si + 1];
      int i = W.seg_start[si];
      // 4 LDS reads in flight per step
      for (; i + 4 <= e; i += 4) {
        const double x0 = W.dpv[i], x1 = W.dpv[i + 1], x2 = W.dpv[i + 2], x3 = W.dpv[i + 3];
        bs_add<F>(s, x0); bs_add<F>(s, x1); bs_add<F>(s, x2); bs_add<F>(s, x3);
      }
      for (; i < e; i++) bs_add<F>(s, W.dpv[i]);
      if (si != nseg - 1) emit_bucket<F>(W, myslot, bs_final<F>(s));
    }
    if (b0 + 64 >= nseg) {
      const int src = (nseg - 1) & 63;
      st.scarry.a = __shfl(s.a, src, 64);
      st.scarry.b = __shfl(s.b, src, 64);
      st.scarry.n = __shfl(s.n, src, 64);
      st.carry_slot = __shfl(myslot, src, 64);
    }
  }
  WAVE_SYNC();
}

// ---- series -> SpanGroup contributions over the K slots -----------------------------
// put(slot, value, union) receives each contribution of the series, at most one per slot.
template <class Put>
__device__ __forceinline__ void emit_series_to(const GridParams& p, const WaveLds& W, int K, Put&& put) {
  const int lane = lane_id();
  const double fillv = (p.fill == TSDB_FILL_ZERO) ? 0.0 : (double)NAN;
  WAVE_SYNC();
  if (!p.rate) {
    if (p.fill != TSDB_FILL_NONE && p.mode != MODE_ALL) {
      // FillingDownsampler (:172-301): every slot, missing -> NaN / 0 / RuntimeException
      for (int k = lane; k < K; k += 64) {
        const bool pr = W.pres[k] != 0;
        if (!pr && p.fill == TSDB_FILL_SCALAR) set_err(p.err, TSDB_E_RUNTIME);
        if (k == 0 && p.skip0) continue;   // before start_time: AggregationIterator ctor :424-441
        put(k, pr ? W.dense[k] : fillv, true);
      }
    } else {
      int prev_present = -1;
      for (int kb = 0; kb < K; kb += 64) {
        const int k = kb + lane;
        const bool pr = k < K && W.pres[k] != 0;
        const int incl = wave_incl_max(pr ? k : -1);
        int pp = __shfl_up(incl, 1, 64);
        if (lane == 0) pp = -1;
        pp = max(pp, prev_present);
        if (pr) {
          const double v = W.dense[k];
          if (pp >= 0 && pp < k - 1) {
            const double y0 = W.dense[pp];
            for (int s2 = pp + 1; s2 < k; s2++) put(s2, interp(p.interp, p, pp, y0, k, v, s2), false);
          }
          put(k, v, true);
        }
        prev_present = max(prev_present, lane_bcast(incl, 63));
      }
    }
  } else {
    // RateSpan over the bucket stream (:121-180), aggregated with PREV semantics
    // (AggregationIterator ctor rate branch :448-459, nextDoubleValue :744-753)
    int prev_item = -1, last_surv = -1;
    long long nsurv = 0;
    const bool dense_stream = p.fill != TSDB_FILL_NONE && p.mode != MODE_ALL;
    for (int kb = 0; kb < K; kb += 64) {
      const int k = kb + lane;
      const bool inK = k < K;
      const bool pr = inK && W.pres[k] != 0;
      const bool item = inK && (dense_stream || pr);
      if (item && !pr && p.fill == TSDB_FILL_SCALAR) set_err(p.err, TSDB_E_RUNTIME);
      const int iincl = wave_incl_max(item ? k : -1);
      int pi = __shfl_up(iincl, 1, 64);
      if (lane == 0) pi = -1;
      pi = max(pi, prev_item);
      bool sv = false;
      double r = 0.0;
      if (item) {
        const double v1 = pr ? W.dense[k] : fillv;
        double v0 = 0.0;
        long long t0 = 0;
        if (pi >= 0) { v0 = W.pres[pi] ? W.dense[pi] : fillv; t0 = p.B0 + slot_rel(p, pi); }
        const long long t1 = (p.mode == MODE_ALL) ? p.qs : p.B0 + slot_rel(p, k);
        if (t1 <= t0) set_err(p.err, TSDB_E_ILLEGAL_STATE);
        const double dt = (double)(t1 - t0) / 1000.0;
        double diff = v1 - v0;
        sv = true;
        if (p.counter && diff < 0) {
          if (p.drop) {
            sv = false;
          } else {
            diff = (double)p.counter_max - v0 + v1;
            r = diff / dt;
            if (p.reset_value > 0 && r > (double)p.reset_value) r = 0.0;
          }
        } else {
          r = diff / dt;
        }
        if (k == 0 && p.skip0) sv = false;   // its rate is dropped with the point (ctor :424-441)
        if (sv) W.rate[k] = r;
      }
      WAVE_SYNC();
      const int cincl = wave_incl_sum(sv ? 1 : 0);
      const long long m = nsurv + (cincl - (sv ? 1 : 0));
      const int sincl = wave_incl_max(sv ? k : -1);
      int ps = __shfl_up(sincl, 1, 64);
      if (lane == 0) ps = -1;
      ps = max(ps, last_surv);
      if (sv) {
        if (m == 1) {
          const double r0 = W.rate[ps];
          for (int s2 = 0; s2 < k; s2++) put(s2, r0, false);
          put(k, r, true);
        } else if (m >= 2) {
          const double rp = W.rate[ps];
          for (int s2 = ps + 1; s2 < k; s2++) put(s2, rp, false);
          put(k, r, true);
        }
      }
      prev_item = max(prev_item, lane_bcast(iincl, 63));
      last_surv = max(last_surv, lane_bcast(sincl, 63));
      nsurv += lane_bcast(cincl, 63);
      WAVE_SYNC();
    }
  }
  WAVE_SYNC();
}

__device__ __forceinline__ void emit_series(const GridParams& p, const WaveLds& W, int K) {
  const int ga = p.ga;
  emit_series_to(p, W, K, [&](int s, double v, bool uni) { contribute(ga, W.part, s, v, uni); });
}

// emit_series for K <= 64 without rate: lane k owns slot k; the series' bucket k arrives
// in registers (pr, v) and the tile partial of slot k lives in the lane's registers, so
// neither the bucket values nor the partials round-trip through LDS.  Same contributions,
// same per-slot order (one per series) as emit_series.
__device__ __forceinline__ double canon_nan(double v) {
  return isnan(v) ? __longlong_as_double(0x7FF8000000000000LL) : v;   // +NaN: the largest key
}

// The SpanGroup contribution of lane k's slot (K <= 64, no rate): the bucket value, its LERP
// between the neighbouring present buckets, the fill value, or none (returns false).  *uni:
// the slot holds a real bucket of the span (a union timestamp).  Called by the whole wave.
__device__ __forceinline__ bool slot_contribution(const GridParams& p, int K, bool pr_in, double v, double& cv,
                                                  bool& uni) {
  const int lane = lane_id();
  const bool inK = lane < K;
  const bool pr = inK && pr_in;
  uni = false;
  if (p.fill != TSDB_FILL_NONE && p.mode != MODE_ALL) {
    // FillingDownsampler (:172-301): every slot, missing -> NaN / 0 / RuntimeException
    const double fillv = (p.fill == TSDB_FILL_ZERO) ? 0.0 : (double)NAN;
    if (!inK) return false;
    if (!pr && p.fill == TSDB_FILL_SCALAR) set_err(p.err, TSDB_E_RUNTIME);
    if (lane == 0 && p.skip0) return false;   // before start_time: AggregationIterator ctor :424-441
    cv = pr ? v : fillv;
    uni = true;
    return true;
  }
  // previous and next present slot of every lane, from the presence ballot
  const uint64_t pm = __ballot(pr);
  if (pm == (K >= 64 ? ~0ull : ((1ull << K) - 1))) {   // every slot present: no interpolation
    cv = v;
    uni = inK;
    return inK;
  }
  const uint64_t below = pm & ((1ull << lane) - 1);
  const uint64_t above = lane == 63 ? 0ull : (pm & ~((2ull << lane) - 1));
  const int prv = below ? 63 - __clzll((long long)below) : -1;
  const int nxt = above ? __ffsll((long long)above) - 1 : 64;
  const bool need = inK && !pr && prv >= 0 && nxt < K;
  double y0 = 0.0, y1 = 0.0;
  if (__ballot(need)) {
    y0 = __shfl(v, max(prv, 0), 64);
    y1 = __shfl(v, min(nxt, 63), 64);
  }
  if (pr) {
    cv = v;
    uni = true;
    return true;
  }
  if (need) {
    cv = interp(p.interp, p, prv, y0, nxt, y1, lane);
    return true;
  }
  return false;
}

// (ga: the group aggregator, a compile-time constant where the caller is specialised for it)
__device__ __forceinline__ void emit_series_reg(const GridParams& p, int K, bool pr_in, double v, RegPart& P, int ga) {
  double cv;
  bool uni;
  if (slot_contribution(p, K, pr_in, v, cv, uni)) contribute_slot(ga, P, cv, uni);
}
__device__ __forceinline__ void emit_series_reg(const GridParams& p, int K, bool pr_in, double v, RegPart& P) {
  emit_series_reg(p, K, pr_in, v, P, p.ga);
}

// Several group-by aggregators over one downsampling in one pass (tsdbhip_run_multi,
// p.multi): the lane's slot keeps the SpanGroup state of sum / avg (sum, nl), min, max, dev
// (Welford mean, m2 over the same nl) and count (nz), all fed the same contribution sequence
// contribute_slot would feed each of them alone -- so every aggregator's tile partial is
// bit-identical to its own pass.  Count interpolates with ZIM (Aggregators.java:620-647), the
// others with LERP: they differ only where a slot is interpolated, where count reads 0.0.
struct MultiReg {
  double sum, mn, mx, mean, m2;
  uint32_t nl, nz, f;
};

__device__ __forceinline__ void rp_init(int ga, RegPart& P) { regpart_init(ga, P); }
__device__ __forceinline__ void rp_init(int, MultiReg& M) {
  M.sum = 0.0;
  M.mn = INFINITY;
  M.mx = -INFINITY;
  M.mean = 0.0;
  M.m2 = 0.0;
  M.nl = 0;
  M.nz = 0;
  M.f = 0;
}

__device__ __forceinline__ void emit_series_reg(const GridParams& p, int K, bool pr_in, double v, MultiReg& M) {
  double cv;
  bool uni;
  if (!slot_contribution(p, K, pr_in, v, cv, uni)) return;   // p.interp is LERP
  const bool interpolated = (p.fill == TSDB_FILL_NONE || p.mode == MODE_ALL) && !(lane_id() < K && pr_in);
  if (!isnan(cv)) {
    M.sum += cv;
    if (cv < M.mn) M.mn = cv;
    if (cv > M.mx) M.mx = cv;
    const uint32_t c = M.nl;
    if (p.multi & MULTI_DEV) {   // contribute_slot's GA_DEV step (a division: only when asked for)
      if (c == 0) {
        M.mean = cv;
      } else {
        const double m = M.mean;
        const double nm = m + (cv - m) / (double)(c + 1);
        M.m2 += (cv - m) * (cv - nm);
        M.mean = nm;
      }
    }
    M.nl = c + 1;
    M.nz++;
  } else if (interpolated) {
    M.nz++;   // ZIM reads 0.0 where LERP produced NaN
  }
  if (uni) M.f |= PF_UNION;
}

// the tile's partial states, lane = slot (K <= 64)
__device__ __forceinline__ void rp_store(const GridParams& p, int64_t tile, int K, const RegPart& P) {
  const int lane = lane_id();
  if (lane < K) {
    const int64_t o = tile * K + lane;
    p.part.a[o] = P.pa;
    p.part.b[o] = P.pb;
    p.part.n[o] = P.pn;
    p.part.f[o] = P.pf;
  }
}
__device__ __forceinline__ void rp_store(const GridParams& p, int64_t tile, int K, const MultiReg& M) {
  const int lane = lane_id();
  if (lane < K) {
    const int64_t o = tile * K + lane;
    p.mp.sum[o] = M.sum;
    p.mp.mn[o] = M.mn;
    p.mp.mx[o] = M.mx;
    p.mp.mean[o] = M.mean;
    p.mp.m2[o] = M.m2;
    p.mp.nl[o] = M.nl;
    p.mp.nz[o] = M.nz;
    p.mp.f[o] = M.f;
  }
}

// Percentile / median (and ordered) group-by, fused into the downsampling pass (p.sel_direct,
// K <= 64, no rate): series s of group g writes its contribution to every slot straight into
// sel_vals[s * K + k] (one coalesced row per series; the fill pattern where it has none) and
// marks the union slots -- k_emit_vals' output without the bucket values round-tripping
// through pre_dense.
// stage (k_short, column layout): the row goes to LDS and sel_cols_flush writes 8 series'
// column pieces at once.
// uacc: the caller's per-lane union flag for the tile (all its series are of group g), stored
// once at the tile's end (sel_uni_flush) -- a load of the flag at every series end makes the wave
// wait for every load issued before it, the streaming kernels' whole ring of rows.
template <bool MARK = true>   // MARK: flag the row written (k_short flags its whole tile at the end)
__device__ __forceinline__ void sel_direct_out(const GridParams& p, int K, int32_t g, int64_t s, bool pr_in,
                                               double v, double* stage = nullptr, bool* uacc = nullptr) {
  double cv = 0.0;
  bool uni;
  const bool has = slot_contribution(p, K, pr_in, v, cv, uni);
  const int lane = lane_id();
  if (stage) {
    if (lane < K) stage[lane] = has ? canon_nan(cv) : __longlong_as_double(0x7FF87FF87FF87FF8LL);
  } else if (lane < K) {
    int64_t at = s * K + lane;
    if (p.sel_cols) {   // the (group, slot) column layout: each column contiguous for the select
      const int64_t g0 = p.group_series_ptr[g], ng = p.group_series_ptr[g + 1] - g0;
      at = g0 * K + (int64_t)lane * ng + (s - g0);
    }
    p.sel_vals[at] = has ? canon_nan(cv) : __longlong_as_double(0x7FF87FF87FF87FF8LL);
  }
  // every series of a group sets the same G x K flags: store only while unset (config 2: 1M
  // series' byte stores into 64 x 60 flags serialised on a few L2 lines, 6.5 vs 3.9 ms)
  if (uacc) *uacc |= uni;
  else if (uni && !p.sel_uni[(int64_t)g * K + lane]) p.sel_uni[(int64_t)g * K + lane] = 1;
  if (MARK && lane == 0 && p.sel_wr) p.sel_wr[s] = 1;
}

// Sampled window (KR 5): the series' contribution to lane k's column is counted below / above
// the column's window [lo, hi] (w.pa, w.pb: loaded once a tile) or kept among the tile's window
// values (wv: the tile's [K][WIN_CAP] block, WIN_CAP = 64 holds a tile's whole column); w.pn =
// below | above << 8, w.pf = values inside.  NaN and
// no contribution count nowhere (runDouble drops NaN; the full path's fill pattern is NaN).
__device__ __forceinline__ void sel_window_out(const GridParams& p, int K, bool pr_in, double v, RegPart& w,
                                               double* wv, double* ws, bool* uacc) {
  double cv = 0.0;
  bool uni;
  const bool has = slot_contribution(p, K, pr_in, v, cv, uni);
  *uacc |= uni;
  const int lane = lane_id();
  if (has && lane < K && !isnan(cv)) {
    if (cv < w.pa) {
      w.pn += 1u;
    } else if (cv > w.pb) {
      w.pn += 1u << 8;
    } else {
      // the first WIN_LDS a lane in the wave's LDS stage, the rest in the tile's global slot
      if (w.pf < (uint32_t)WIN_LDS) ws[lane * WIN_LDS + w.pf] = cv;
      else if (w.pf < (uint32_t)WIN_CAP) wv[lane * WIN_CAP + w.pf] = cv;
      w.pf++;
    }
  }
}

__device__ __forceinline__ void sel_uni_flush(const GridParams& p, int K, int32_t g, bool uacc) {
  const int lane = lane_id();
  if (uacc && lane < K && !p.sel_uni[(int64_t)g * K + lane]) p.sel_uni[(int64_t)g * K + lane] = 1;
}

// The staged rows of series sa .. sa + nb - 1 (group g, nb <= 8; stage [nb][K]) into their
// columns: lanes 8c .. 8c + 7 store column k's nb consecutive values (64 B pieces instead of one
// 8-B store per line).
// (g0, ng: the group's first series and its series count, loaded by the caller before its load
// ring starts -- a global load here, consumed at once, would wait for every ring load in flight)
__device__ __forceinline__ void sel_cols_flush(const GridParams& p, int K, int64_t g0, int64_t ng, int64_t sa, int nb,
                                               const double* stage) {
  WAVE_SYNC();
  double* base = p.sel_vals + g0 * K + (sa - g0);
  const int lane = lane_id();
  if (nb == 8) {
    for (int e = lane; e < 8 * K; e += 64) {
      const int k = e >> 3, i = e & 7;
      base[(int64_t)k * ng + i] = stage[i * K + k];
    }
  } else {
    for (int e = lane; e < nb * K; e += 64) {
      const int k = e / nb, i = e - k * nb;
      base[(int64_t)k * ng + i] = stage[i * K + k];
    }
  }
  WAVE_SYNC();
}

// End of series s (group g): its SpanGroup contributions, (dense_out) its bucket values, or
// (sel_direct) its percentile group-by contributions.
__device__ __forceinline__ void series_out(const GridParams& p, const WaveLds& W, int K, int64_t s, int32_t g) {
  if (p.sel_direct) {   // K <= 64 (host-checked)
    const int lane = lane_id();
    WAVE_SYNC();
    const bool pr = lane < K && W.pres[lane] != 0;
    sel_direct_out(p, K, g, s, pr, pr ? W.dense[lane] : 0.0);
    WAVE_SYNC();
    return;
  }
  if (p.dense_out) {
    const int lane = lane_id();
    WAVE_SYNC();
    for (int k = lane; k < K; k += 64) {
      p.dense_out[s * K + k] = W.dense[k];
      p.pres_out[s * K + k] = W.pres[k];
    }
    WAVE_SYNC();
    return;
  }
  emit_series(p, W, K);
}

// Next row of the tile inside the scan range, starting at (s, r) inclusive.
__device__ __forceinline__ bool seek_row(const GridParams& p, int64_t s_end, int64_t& s, int64_t& r, RowDesc& d) {
  while (s < s_end) {
    const int64_t r1 = p.series_row_ptr[s + 1];
    for (; r < r1; r++) {
      d = p.rows[r];
      if ((int64_t)d.base < p.ss) continue;
      if ((int64_t)d.base >= p.se) break;
      return true;
    }
    s++;
    if (s < s_end) r = p.series_row_ptr[s];
  }
  return false;
}

// The slow path over one whole series (after a failed certificate, or for
// order-sensitive downsample functions).
template <int F>
__device__ __forceinline__ void series_slow(const GridParams& p, const WaveLds& W, int64_t s, int K) {
  const int lane = lane_id();
  for (int k = lane; k < K; k += 64) W.pres[k] = 0;
  WAVE_SYNC();
  SeriesState st;
  st.carry_slot = -1;
  bs_init<F>(st.scarry);
  StreamOrd so{-1};
  const int64_t r0 = p.series_row_ptr[s], r1 = p.series_row_ptr[s + 1];
  for (int64_t r = r0; r < r1; r++) {
    const RowDesc d = p.rows[r];
    if ((int64_t)d.base < p.ss) continue;
    if ((int64_t)d.base >= p.se) break;
    if (d.flags & ROW_ERR) { if (lane == 0) set_err(p.err, TSDB_E_ILLEGAL_DATA); continue; }
    const RowGeom g = row_geom(p, d.base);
    const bool skip = so_row_skip(p, so, d, r + 1 >= r1 || (int64_t)p.rows[r + 1].base >= p.se);
    int64_t vcur = 0;
    for (int64_t c0 = 0; c0 < (int64_t)d.ndp; c0 += CH) {
      int slot[DPL];
      double val[DPL];
      if (row_uniform(d)) {   // uniform rows: the register decode (no byte staging)
        Raw rw = {};
        load_raw(p, d, c0, rw);
        decode_raw<true>(p, d, g, c0, rw, slot, val);
      } else {
        decode_generic<true>(p, d, g, c0, W, vcur, slot, val);
      }
      so_apply(p, so, slot, skip);
      slow_chunk<F>(W, st, slot, val);
    }
  }
  if (st.carry_slot >= 0 && lane == 0) emit_bucket<F>(W, st.carry_slot, bs_final<F>(st.scarry));
  WAVE_SYNC();
}

template <int F, bool GSLOT>
__global__ __launch_bounds__(256) void k_grid(GridParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform (scalar) tile index
  int64_t tile = (int64_t)blockIdx.x * p.waves + wave;
  if (p.tile_list) {
    if (tile >= (int64_t)*p.tile_list_n) return;
    tile = p.tile_list[tile];
  }
  if (tile >= p.n_tiles) return;
  const int K = (int)p.K;
  const WaveLds W = carve<GSLOT>(p, smem + (int64_t)wave * p.wave_lds, tile, K, p.rate != 0);
  for (int k = lane; k < K; k += 64) part_init(p.ga, W.part, k);

  const int64_t s_end = p.tile_end[tile];
  int64_t cs = p.tile_begin[tile];
  int64_t cr = (cs < s_end) ? p.series_row_ptr[cs] : 0;
  RowDesc cd;
  bool cok = seek_row(p, s_end, cs, cr, cd);
  if (cok && lane == 0) atomicOr(&p.group_active[p.tile_group[tile]], 1u);
  // one row of look-ahead (descriptor prefetch)
  int64_t ns = cs, nr = cr + 1;
  RowDesc nd;
  bool nok = cok ? seek_row(p, s_end, ns, nr, nd) : false;

  SeriesState st;
  st.carry_slot = -1;
  st.fcarry = fs_id<F>();
  bs_init<F>(st.scarry);
  st.nmax = 0;
  int lsb = INT32_MAX;
  double amax = 0.0;
  bool force_slow = !fast_capable<F>();
  for (int k = lane; k < K; k += 64) W.pres[k] = 0;
  WAVE_SYNC();

  int64_t c0 = 0;
  int64_t vcur = 0;
  Raw rc = {};
  if (cok && !force_slow && row_uniform(cd)) load_raw(p, cd, 0, rc);
  bool row_start = true;
  // seq: this series' first row already rules the exactness certificate out (two values of its
  // magnitude and resolution cannot add exactly), so its chunks go straight through the
  // sequential in-bucket order (slow_chunk) -- one pass instead of the fast pass plus a re-walk
  bool series_first = true, seq = false;
  StreamOrd so{-1};
  bool skip_row = false;
  while (cok) {
    if (row_start) {
      if (cd.flags & ROW_ERR) { if (lane == 0) set_err(p.err, TSDB_E_ILLEGAL_DATA); }
      lsb = min(lsb, cd.lsb);
      amax = fmax(amax, cd.absmax);
      row_start = false;
      skip_row = !force_slow && so_row_skip(p, so, cd, !nok || ns != cs);
      if (series_first) {
        series_first = false;
        if (needs_cert<F>() && !force_slow && cd.lsb != INT32_MAX && cd.absmax != 0.0) {
          const int L = (F == F_SQUARESUM) ? 2 * cd.lsb : cd.lsb;
          const double A = (F == F_SQUARESUM) ? cd.absmax * cd.absmax : cd.absmax;
          seq = isinf(A) || 2.0 * A * (1.0 + 1e-12) > ldexp(1.0, 52 + L);   // (row_nocert for sums)
        }
      }
    }
    const bool more_in_row = c0 + CH < (int64_t)cd.ndp;
    // prefetch the next chunk (same row, or the first chunk of the next row)
    Raw rn = {};
    if (!force_slow) {
      if (more_in_row) {
        if (row_uniform(cd)) load_raw(p, cd, c0 + CH, rn);
      } else if (nok && row_uniform(nd)) {
        load_raw(p, nd, 0, rn);
      }
    }
    if (!force_slow && !(cd.flags & ROW_ERR)) {
      const RowGeom g = row_geom(p, cd.base);
      int slot[DPL];
      double val[DPL];
      if (row_uniform(cd)) decode_raw<true>(p, cd, g, c0, rc, slot, val);
      else decode_generic<true>(p, cd, g, c0, W, vcur, slot, val);
      so_apply(p, so, slot, skip_row);
      if (seq) slow_chunk<F>(W, st, slot, val);
      else fast_chunk<F>(W, st, slot, val);
    }
    if (more_in_row) {
      c0 += CH;
      rc = rn;
      continue;
    }
    // row done
    const bool series_end = !nok || ns != cs;
    if (series_end) {
      bool slow = force_slow;
      if (seq) {
        if (st.carry_slot >= 0 && lane == 0) emit_bucket<F>(W, st.carry_slot, bs_final<F>(st.scarry));
        WAVE_SYNC();
      } else if (!slow) {
        if (st.carry_slot >= 0 && lane == 0) emit_bucket<F>(W, st.carry_slot, fs_final<F>(st.fcarry));
        if (st.carry_slot >= 0) st.nmax = max(st.nmax, st.fcarry.n);
        if (needs_cert<F>()) {
          // all partial sums exactly representable => any association order == Java's order
          const int L = (F == F_SQUARESUM) ? 2 * lsb : lsb;
          const double A = (F == F_SQUARESUM) ? amax * amax : amax;
          const bool ok = (A == 0.0) ||
                          (lsb != INT32_MAX && !isinf(A) && (double)st.nmax * A * (1.0 + 1e-12) <= ldexp(1.0, 52 + L));
          slow = !ok;
        }
      }
      if (slow) series_slow<F>(p, W, cs, K);
      series_out(p, W, K, cs, p.tile_group[tile]);
      // next series
      for (int k = lane; k < K; k += 64) W.pres[k] = 0;
      WAVE_SYNC();
      st.carry_slot = -1;
      st.fcarry = fs_id<F>();
      bs_init<F>(st.scarry);
      st.nmax = 0;
      lsb = INT32_MAX;
      amax = 0.0;
      series_first = true;
      seq = false;
      so.smax = -1;
    }
    cs = ns;
    cr = nr;
    cd = nd;
    cok = nok;
    c0 = 0;
    vcur = 0;
    rc = rn;
    row_start = true;
    if (cok) {
      ns = cs;
      nr = cr + 1;
      nok = seek_row(p, s_end, ns, nr, nd);
    }
  }

  if (!GSLOT) {
    WAVE_SYNC();
    double* ga_ = p.part.a + tile * K;
    double* gb_ = p.part.b + tile * K;
    uint32_t* gn_ = p.part.n + tile * K;
    uint32_t* gf_ = p.part.f + tile * K;
    for (int k = lane; k < K; k += 64) {
      ga_[k] = W.part.a[k];
      gb_[k] = W.part.b[k];
      gn_[k] = W.part.n[k];
      gf_[k] = W.part.f[k];
    }
  }
}

// ---- k_fast: the streaming kernel ------------------------------------------------
// For tiles whose rows are all "uniform float" cells of one (qualifier width QW, value
// length VL) class, sorted, NaN-free, and whose buckets pass the exactness certificate,
// the order in which a bucket's values are added cannot change the bit pattern of the
// result.  k_fast therefore reduces each lane's 8 datapoints in registers (at most two
// bucket runs per lane) and folds them into per-series slot accumulators in LDS with
// LDS atomics -- no per-chunk wave scan, no carry -- while a D-deep ring of chunk loads
// keeps ~D x 3 KB per wave in flight.  A tile that breaks any premise (other row class,
// malformed / NaN row, failed certificate) is appended to the redo list and recomputed
// by k_grid, the general (sequential-order) kernel.
struct FMeta {
  uint32_t bits;   // datapoints of the row from this chunk's start | FM_* flags
  int32_t rrel;    // row index relative to the tile's first row
};
enum : uint32_t { FM_NV = 0x1FFFFFFFu, FM_OK = 1u << 29, FM_NEWSER = 1u << 30, FM_NEWROW = 1u << 31 };

// VL == 0: the vle-integer class (values of 1 or 2 bytes, rows of <= CH datapoints): the
// lane loads a fixed 16-byte slice of the row's value bytes; values are located after a
// wave prefix sum of the qualifier lengths and read back from an LDS stage.
template <int QW, int VL>
struct FRaw {
  uint4 q[QW / 2];               // 8 qualifiers of QW bytes
  uint4 v[VL == 0 ? 1 : VL / 2]; // 8 values of VL bytes / a 16-B slice of the row's values
};

template <int F>
__device__ __forceinline__ constexpr bool fast_f() {
  return F == F_SUM || F == F_AVG || F == F_COUNT || F == F_SQUARESUM || F == F_MIN || F == F_MAX;
}

__host__ __device__ inline int64_t fast_slot_bytes(int64_t K, bool rate, bool part = true) {
  // acc (f64, also the dense bucket values), cnt (u32), pres (u8), [rate f64], [partials: not
  // when the kernel writes the series' buckets to HBM for a later group-by step (dense_out)]
  return align16(K * 8) + align16(K * 4) + align16(K) + (rate ? align16(K * 8) : 0) +
         (part ? align16(K * 8) * 2 + align16(K * 4) * 2 : 0);
}

struct FastLds {
  double* acc;
  uint32_t* cnt;
  WaveLds w;          // dense == acc, pres, rate, part
  uint8_t* vstage;    // VL == 0: the row's value bytes (64 lanes x 16 B)
  double* wstage;     // KR 5: the kept values, WIN_LDS a lane (sel_window_out)
};

__device__ __forceinline__ FastLds fast_carve(unsigned char* base, int64_t K, bool rate, bool part = true) {
  FastLds f;
  int64_t o = 0;
  f.vstage = base;    // used only by the VL == 0 instantiations (fast_wave_lds reserves it)
  o += 1024;
  f.acc = (double*)(base + o); o += align16(K * 8);
  f.cnt = (uint32_t*)(base + o); o += align16(K * 4);
  f.w.dense = f.acc;
  f.w.pres = base + o; o += align16(K);
  if (rate) { f.w.rate = (double*)(base + o); o += align16(K * 8); } else { f.w.rate = nullptr; }
  if (part) {
    f.w.part.a = (double*)(base + o); o += align16(K * 8);
    f.w.part.b = (double*)(base + o); o += align16(K * 8);
    f.w.part.n = (uint32_t*)(base + o); o += align16(K * 4);
    f.w.part.f = (uint32_t*)(base + o); o += align16(K * 4);
  } else {
    f.w.part.a = f.w.part.b = nullptr;
    f.w.part.n = f.w.part.f = nullptr;
  }
  f.w.dpv = nullptr; f.w.vbuf = nullptr; f.w.mq = nullptr; f.w.mv = nullptr;
  f.w.seg_slot = nullptr; f.w.seg_start = nullptr;
  f.wstage = nullptr;
  return f;
}

template <int F>
__device__ __forceinline__ double fast_identity() {
  return F == F_MIN ? (double)INFINITY : (F == F_MAX ? -(double)INFINITY : 0.0);
}

template <int F>
__device__ __forceinline__ void fast_fold(const FastLds& L, int k, double v, uint32_t n) {
  if (F == F_MIN) __hip_atomic_fetch_min(&L.acc[k], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  else if (F == F_MAX) __hip_atomic_fetch_max(&L.acc[k], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  else if (F != F_COUNT) __hip_atomic_fetch_add(&L.acc[k], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  __hip_atomic_fetch_add(&L.cnt[k], n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

template <int QW, int VL>
__device__ __forceinline__ bool fast_row_ok(uint32_t flags, bool minmax, bool cert = false) {
  // cert: an order-free sum (F_SUM / F_AVG) -- a row whose values can never add exactly goes
  // to k_grid's sequential path at once instead of after a full streaming pass
  if (VL == 0) {
    const uint32_t want = (uint32_t)QW | ROW_ALLI | ROW_VLE2;
    const uint32_t mask = ROW_QW_MASK | ROW_ALLI | ROW_VLE2 | ROW_ERR | ROW_UNSORTED | (cert ? ROW_NOCERT : 0u);
    return (flags & mask) == want;
  }
  const uint32_t want = (uint32_t)QW | ((uint32_t)VL << ROW_VL_SHIFT) | ROW_ALLF;
  const uint32_t mask = ROW_QW_MASK | ROW_VL_MASK | ROW_ALLF | ROW_ERR | ROW_NAN | ROW_UNSORTED |
                        (minmax ? ROW_NEGZ : 0u) | (cert ? ROW_NOCERT : 0u);
  return (flags & mask) == want;
}

// Row walker: the tile's rows in order, filtered to the scan range, cut in CH-datapoint
// chunks.  Descriptors are read with scalar loads, one row ahead.
struct FDesc {       // the descriptor fields the walker needs
  uint64_t qoff, voff;
  uint32_t base, ndp, flags;
};

__device__ __forceinline__ FDesc fdesc(const RowDesc* __restrict__ rows, int64_t r) {
  const RowDesc& x = rows[r];
  FDesc d;
  d.qoff = x.qoff; d.voff = x.voff; d.base = x.base; d.ndp = x.ndp; d.flags = x.flags;
  return d;
}

struct FWalk {
  int64_t r0;        // first row of the tile
  int32_t r, rend;   // current row, end of the tile's rows (relative to r0)
  int32_t c0;        // next chunk offset inside row r
  int32_t sf;        // a series start was passed since the last issued chunk
  FDesc d, nd;       // rows r and r + 1
};

__device__ __forceinline__ void fwalk_next_row(const RowDesc* __restrict__ rows, FWalk& w) {
  w.r++;
  w.c0 = 0;
  w.d = w.nd;
  if (w.r + 1 < w.rend) w.nd = fdesc(rows, w.r0 + w.r + 1);
}

// 0 = chunk issued, 1 = end of tile, 2 = row the kernel cannot take (redo the tile)
template <int F, int QW, int VL>
__device__ __forceinline__ int fast_issue(const GridParams& p, const RowDesc* __restrict__ rows, FWalk& w,
                                          FRaw<QW, VL>& b, FMeta& m) {
  m.bits = 0;
  for (;;) {
    if (w.r >= w.rend) return 1;
    if (w.c0 == 0) {
      w.sf |= (w.d.flags & ROW_SFIRST) != 0;
      if ((int64_t)w.d.base < p.ss || (int64_t)w.d.base >= p.se) { fwalk_next_row(rows, w); continue; }
      if (!fast_row_ok<QW, VL>(w.d.flags, F == F_MIN || F == F_MAX, F == F_SUM || F == F_AVG)) return 2;
      if (VL == 0 && w.d.ndp > CH) return 2;
    }
    if (w.c0 < (int64_t)w.d.ndp) break;
    fwalk_next_row(rows, w);
  }
  const int lane = lane_id();
  const int nv0 = (int)w.d.ndp - w.c0;
  m.bits = (uint32_t)nv0 | FM_OK | (w.sf ? FM_NEWSER : 0u) | (w.c0 == 0 ? FM_NEWROW : 0u);
  m.rrel = w.r;
  w.sf = 0;
  // lanes past the end of the row re-read its first datapoints (in bounds, ignored)
  const int64_t i0 = (lane * DPL < nv0) ? w.c0 + (int64_t)lane * DPL : 0;
  const uint4* q = reinterpret_cast<const uint4*>(p.qual + w.d.qoff + i0 * QW);
#pragma unroll
  for (int k = 0; k < QW / 2; k++) b.q[k] = q[k];
  if (VL == 0) {
    b.v[0] = *reinterpret_cast<const uint4*>(p.val2 + w.d.qoff + i0 * 2);   // the lane's 8 int16 values
  } else {
    const uint4* v = reinterpret_cast<const uint4*>(p.val + w.d.voff + i0 * VL);
#pragma unroll
    for (int k = 0; k < VL / 2; k++) b.v[k] = v[k];
  }
  w.c0 += CH;
  return 0;
}

// offset field of datapoint j (seconds for QW == 2, milliseconds for QW == 4)
template <int QW, int VL>
__device__ __forceinline__ uint32_t f_field(const FRaw<QW, VL>& b, int j) {
  if (QW == 2) {
    const uint32_t wd = (j >> 1) == 0 ? b.q[0].x : (j >> 1) == 1 ? b.q[0].y : (j >> 1) == 2 ? b.q[0].z : b.q[0].w;
    const uint32_t t = __builtin_bswap32(wd);
    return (j & 1) ? ((t >> 4) & 0xFFF) : (t >> 20);
  } else {
    const uint4 u = b.q[j >> 2];
    const uint32_t wd = (j & 3) == 0 ? u.x : (j & 3) == 1 ? u.y : (j & 3) == 2 ? u.z : u.w;
    return (__builtin_bswap32(wd) >> 6) & 0x3FFFFF;
  }
}

template <int QW, int VL>
__device__ __forceinline__ double f_value(const FRaw<QW, VL>& b, int j) {
  if (VL == 4) {
    const uint4 u = b.v[j >> 2];
    const uint32_t wd = (j & 3) == 0 ? u.x : (j & 3) == 1 ? u.y : (j & 3) == 2 ? u.z : u.w;
    return (double)__uint_as_float(__builtin_bswap32(wd));
  } else {
    const uint4 u = b.v[j >> 1];
    const uint32_t hi = (j & 1) ? u.z : u.x;
    const uint32_t lo = (j & 1) ? u.w : u.y;
    return __longlong_as_double((long long)(((uint64_t)__builtin_bswap32(hi) << 32) | __builtin_bswap32(lo)));
  }
}

// qualifier flags (low nibble) of datapoint j
template <int QW, int VL>
__device__ __forceinline__ uint32_t f_flags(const FRaw<QW, VL>& b, int j) {
  if (QW == 2) {
    const uint32_t wd = (j >> 1) == 0 ? b.q[0].x : (j >> 1) == 1 ? b.q[0].y : (j >> 1) == 2 ? b.q[0].z : b.q[0].w;
    const uint32_t t = __builtin_bswap32(wd);
    return (j & 1) ? (t & 0xF) : ((t >> 16) & 0xF);
  } else {
    const uint4 u = b.q[j >> 2];
    const uint32_t wd = (j & 3) == 0 ? u.x : (j & 3) == 1 ? u.y : (j & 3) == 2 ? u.z : u.w;
    return __builtin_bswap32(wd) & 0xF;
  }
}

// VL == 0: the lane's 8 vle integers (1 or 2 bytes, RowSeq.extractIntegerValue
// src/core/RowSeq.java:233-245), read from the load-time int16 copy of the row's values
// (k_index writes val2[qoff + 2 i] for every 1-2-byte integer of a 2-byte-qualifier row), so
// the query needs no in-wave prefix sum of value lengths and no LDS staging.
template <int QW, int VL>
__device__ __forceinline__ int f_int16(const FRaw<QW, VL>& b, int j) {
  const uint32_t wd = (j >> 1) == 0 ? b.v[0].x : (j >> 1) == 1 ? b.v[0].y : (j >> 1) == 2 ? b.v[0].z : b.v[0].w;
  return (j & 1) ? ((int)wd >> 16) : (int)(int16_t)(wd & 0xFFFF);
}

template <int QW, int VL>
__device__ __forceinline__ void f_values_vle(const FastLds& L, const FRaw<QW, VL>& b, int nvl, double xs[DPL]) {
#pragma unroll
  for (int j = 0; j < DPL; j++) xs[j] = (double)f_int16<QW, VL>(b, j);
}

template <int QW, int VL, int NP = DPL>
__device__ __forceinline__ void f_values_vle_i(const FastLds& L, const FRaw<QW, VL>& b, int nvl, int xi[NP]) {
#pragma unroll
  for (int j = 0; j < NP; j++) xi[j] = f_int16<QW, VL>(b, j);
}

struct FGeom {
  int q0, r0;   // slot at the row base, remainder in n-units (r0 < 0: row starts before slot 0)
};

__device__ __forceinline__ FGeom fgeom(const GridParams& p, uint32_t base) {
  const int64_t rel = p.unit_s ? (int64_t)base - p.B0n : (int64_t)base * 1000 - p.B0n;
  FGeom g;
  if (rel >= 0) {
    g.q0 = (int)((double)rel * p.rcpn);
    g.r0 = (int)(rel - (int64_t)g.q0 * p.In);
  } else {
    g.q0 = 0;
    g.r0 = (int)rel;
  }
  return g;
}

__device__ __forceinline__ int f_slot(const GridParams& p, const FGeom& m, int n) {
  return m.q0 + (int)((double)n * p.rcpn);
}

// Folds one chunk into the series' slot accumulators.
template <int F, int QW, int VL, bool FULL, int NP = DPL>
__device__ __forceinline__ void fast_chunk(const GridParams& p, const FastLds& L, const FRaw<QW, VL>& b,
                                           const FGeom& m, int nv0, int K) {
  const int lane = lane_id();
  const int nvl = FULL ? NP : max(0, min(NP, nv0 - lane * NP));
  const int uq = (QW == 2 && !p.unit_s) ? 1000 : 1;
  uint32_t fld[NP];
#pragma unroll
  for (int j = 0; j < NP; j++) fld[j] = f_field<QW, VL>(b, j);
  // vle integers (1-2 bytes): the in-lane runs are folded in int32 (8 values of |x| < 2^15
  // sum exactly) and converted once per run; squareSum stays in double
  constexpr bool IP = (VL == 0) && (F != F_SQUARESUM);
  double xs[NP];
  int xi[NP];
  if (VL == 0) {
    f_values_vle_i<QW, VL, NP>(L, b, nvl, xi);
    if (!IP) {
#pragma unroll
      for (int j = 0; j < NP; j++) xs[j] = (double)xi[j];
    }
  } else {
#pragma unroll
    for (int j = 0; j < NP; j++) xs[j] = f_value<QW, VL>(b, j);
  }
  uint32_t flast = fld[NP - 1];
  if (!FULL) {
#pragma unroll
    for (int j = 0; j < NP - 1; j++) if (j == nvl - 1) flast = fld[j];
  }
  const int n0 = m.r0 + (int)fld[0] * uq;
  const int nl = m.r0 + (int)flast * uq;
  const int sfirst = n0 >= 0 ? f_slot(p, m, n0) : -1;
  const int slast = nl >= 0 ? f_slot(p, m, nl) : -1;
  const bool simple = nvl == 0 || (n0 >= 0 && slast < K && slast <= sfirst + 1);
  if (__builtin_expect(__all(simple), 1)) {
    if (nvl == 0) return;
    // first run: offsets below the next bucket boundary
    const int Dn = (sfirst - m.q0 + 1) * p.In - m.r0;   // > 0
    uint32_t Tf;
    if (uq == 1) Tf = (uint32_t)Dn;                      // uniform branch: no runtime integer division
    else Tf = (uint32_t)((Dn + 999) / 1000);
    if constexpr (IP) {
      constexpr int ID = F == F_MIN ? INT32_MAX : (F == F_MAX ? INT32_MIN : 0);
      int P = ID, sF = 0, mL = ID, cF = 0;
#pragma unroll
      for (int j = 0; j < NP; j++) {
        const bool valid = FULL || j < nvl;
        const bool inF = valid && fld[j] < Tf;
        const int x = xi[j];
        if (F == F_MIN) {
          P = min(P, valid ? x : INT32_MAX);
          if (!inF && valid) mL = min(mL, x);
        } else if (F == F_MAX) {
          P = max(P, valid ? x : INT32_MIN);
          if (!inF && valid) mL = max(mL, x);
        } else if (F != F_COUNT) {
          P += valid ? x : 0;
        }
        if (inF) { sF = P; cF = j + 1; }
      }
      const int nL = nvl - cF;
      const int iL = (F == F_MIN || F == F_MAX) ? mL : P - sF;
      fast_fold<F>(L, sfirst, (double)sF, (uint32_t)cF);
      if (nL > 0) fast_fold<F>(L, sfirst + 1, (double)iL, (uint32_t)nL);
      return;
    }
    double P = fast_identity<F>(), sF = 0.0, mL = fast_identity<F>();
    int cF = 0;
#pragma unroll
    for (int j = 0; j < NP; j++) {
      const bool valid = FULL || j < nvl;
      const bool inF = valid && fld[j] < Tf;
      double x = xs[j];
      if (F == F_SQUARESUM) x = x * x;
      if (F == F_MIN) {
        P = fmin(P, valid ? x : (double)INFINITY);
        if (!inF && valid) mL = fmin(mL, x);
      } else if (F == F_MAX) {
        P = fmax(P, valid ? x : -(double)INFINITY);
        if (!inF && valid) mL = fmax(mL, x);
      } else if (F != F_COUNT) {
        P += valid ? x : 0.0;
      }
      if (inF) { sF = P; cF = j + 1; }
    }
    const int nL = nvl - cF;
    double sL;
    if (F == F_MIN || F == F_MAX) sL = mL;
    else sL = P - sF;   // exact: every partial sum is representable (certificate)
    fast_fold<F>(L, sfirst, sF, (uint32_t)cF);
    if (nL > 0) fast_fold<F>(L, sfirst + 1, sL, (uint32_t)nL);
  } else {
    // some lane spans more than two buckets or the edge of the slot range: per datapoint
#pragma unroll
    for (int j = 0; j < NP; j++) {
      if (j < nvl) {
        const int n = m.r0 + (int)fld[j] * uq;
        if (n >= 0) {
          const int s = f_slot(p, m, n);
          if (s < K) {
            double x = IP ? (double)xi[j] : xs[j];
            if (F == F_SQUARESUM) x = x * x;
            fast_fold<F>(L, s, x, 1u);
          }
        }
      }
    }
  }
}

// The whole chunk in one bucket (an hour bucket over an hour row, GridParams.oneb): one wave
// reduction and one fold.  A fold a lane would serialise ~45 LDS atomics on one slot.  Any
// association is exact here (the series' certificate covers every partial sum), min / max are
// order-free.  Called by the whole wave; false = not one bucket (nothing folded).
template <int F, int QW, int VL, int NP = DPL>
__device__ __forceinline__ bool fast_chunk_oneb(const GridParams& p, const FastLds& L, const FRaw<QW, VL>& b,
                                                const FGeom& m, int nv0, int K) {
  const int lane = lane_id();
  const int n = min(nv0, 64 * NP);
  const int nvl = max(0, min(NP, n - lane * NP));
  const int uq = (QW == 2 && !p.unit_s) ? 1000 : 1;
  const int ll = (n - 1) / NP, jl = (n - 1) % NP;   // the chunk's last datapoint: lane, slot
  uint32_t fl = 0;
#pragma unroll
  for (int j = 0; j < NP; j++) if (j == jl) fl = f_field<QW, VL>(b, j);
  const int n0 = m.r0 + (int)__builtin_amdgcn_readfirstlane((int)f_field<QW, VL>(b, 0)) * uq;
  const int nl = m.r0 + (int)__builtin_amdgcn_readlane((int)fl, ll) * uq;
  if (n0 < 0) return false;
  const int s0 = f_slot(p, m, n0);
  if (f_slot(p, m, nl) != s0 || s0 >= K) return false;
  const uint32_t cnt = (uint32_t)n;
  if constexpr (F == F_COUNT) {
    if (lane == 0) fast_fold<F>(L, s0, 0.0, cnt);
  } else if constexpr (VL == 0 && F != F_SQUARESUM) {   // vle integers: |x| < 2^15, 512 of them add in int32
    constexpr int ID = F == F_MIN ? INT32_MAX : (F == F_MAX ? INT32_MIN : 0);
    int P = ID;
#pragma unroll
    for (int j = 0; j < NP; j++) {
      const int x = j < nvl ? f_int16<QW, VL>(b, j) : ID;
      P = F == F_MIN ? min(P, x) : (F == F_MAX ? max(P, x) : P + x);
    }
    const int tot = wave_reduce_i32(P, ID, [](int a, int c) { return F == F_MIN ? min(a, c) : (F == F_MAX ? max(a, c) : a + c); });
    if (lane == 0) fast_fold<F>(L, s0, (double)tot, cnt);
  } else {
    const double ID = fast_identity<F>();
    double P = ID;
#pragma unroll
    for (int j = 0; j < NP; j++) {
      double x = VL == 0 ? (double)f_int16<QW, VL>(b, j) : f_value<QW, VL>(b, j);
      if (F == F_SQUARESUM) x = x * x;
      if (j >= nvl) x = ID;
      P = F == F_MIN ? fmin(P, x) : (F == F_MAX ? fmax(P, x) : P + x);
    }
    const double tot = wave_reduce_f64(P, ID, [](double a, double c) {
      return F == F_MIN ? fmin(a, c) : (F == F_MAX ? fmax(a, c) : a + c);
    });
    if (lane == 0) fast_fold<F>(L, s0, tot, cnt);
  }
  return true;
}

// A chunk of a row shorter than CH: when every lane is either full or empty (a row of a
// multiple of 8 datapoints, e.g. 360), the full-lane code runs on the non-empty lanes.
template <int F, int QW, int VL, int NP = DPL>
__device__ __forceinline__ void fast_chunk_any(const GridParams& p, const FastLds& L, const FRaw<QW, VL>& b,
                                               const FGeom& m, int nv0, int K) {
#ifndef TSDBHIP_NO_ONEB
  if (p.oneb && fast_chunk_oneb<F, QW, VL, NP>(p, L, b, m, nv0, K)) return;
#endif
  const int nvl = max(0, min(NP, nv0 - lane_id() * NP));
  if (__all(nvl == 0 || nvl == NP)) {
    if (nvl) fast_chunk<F, QW, VL, true, NP>(p, L, b, m, nv0, K);
  } else {
    fast_chunk<F, QW, VL, false, NP>(p, L, b, m, nv0, K);
  }
}

// Series end: buckets -> dense values, certificate, SpanGroup contributions, reset.
template <int F>
__device__ __forceinline__ bool fast_cert(uint32_t nmax, int lsb, double amax) {
  if (!needs_cert<F>()) return true;
  const int Lb = (F == F_SQUARESUM) ? 2 * lsb : lsb;
  const double A = (F == F_SQUARESUM) ? amax * amax : amax;
  return (A == 0.0) || (lsb != INT32_MAX && Lb >= -1022 && !isinf(A) &&
                        (double)nmax * A * (1.0 + 1e-12) <= ldexp(1.0, 52 + Lb));
}

template <int F>
__device__ __forceinline__ double fast_bucket_value(uint32_t c, double a) {
  if (F == F_SUM || F == F_SQUARESUM) return c ? a : (double)NAN;
  if (F == F_AVG) return c ? a / (double)(int)c : (double)NAN;
  if (F == F_COUNT) return (double)c;
  if (F == F_MIN) return a == INFINITY ? (double)NAN : a;
  return a == -INFINITY ? (double)NAN : a;
}

// K <= 64, no rate: the register-partial variant (emit_series_reg; RP = RegPart, or MultiReg
// for the fused multi-aggregator pass).  OUT: the instantiation also serves the per-series
// output modes (sel_direct / dense_out); without it the group-by kernels carry no such branch.
// (OUT 2: the per-series select output only -- k_short KR 4 -- without the other branches'
// registers; OUT 3: the sampled window's counts and values -- KR 5)
template <int F, bool MARK = true, int OUT = 1, class RP>
__device__ __forceinline__ bool fast_series_end_reg(const GridParams& p, const FastLds& L, int K, int lsb, double amax,
                                                    RP& P, int64_t s, int32_t g, uint32_t nbound = 0,
                                                    double* stage = nullptr, bool* uacc = nullptr) {
  const int lane = lane_id();
  WAVE_SYNC();
  uint32_t c = 0;
  double a = 0.0;
  if (lane < K) {
    c = L.cnt[lane];
    a = L.acc[lane];
  }
  // certificate: the series' datapoint count bounds every bucket count (nbound), else the
  // bucket maximum
  if (!(nbound && fast_cert<F>(nbound, lsb, amax))) {
    const uint32_t nmax = (uint32_t)wave_max((int)c);
    if (!fast_cert<F>(nmax, lsb, amax)) return false;
  }
  if constexpr (OUT == 3) {   // (KR 5: P holds the window state, stage the tile's window values)
    if constexpr (std::is_same_v<RP, RegPart>) sel_window_out(p, K, c != 0, fast_bucket_value<F>(c, a), P, stage, L.wstage, uacc);
  } else if (OUT == 2 || (OUT && p.sel_direct)) {
    sel_direct_out<MARK>(p, K, g, s, c != 0, fast_bucket_value<F>(c, a), stage, uacc);
  } else if (OUT == 2) {
  } else if (OUT && p.dense_out) {
    if (lane < K) {
      p.dense_out[s * K + lane] = fast_bucket_value<F>(c, a);
      p.pres_out[s * K + lane] = c != 0;
    }
  } else {
    emit_series_reg(p, K, c != 0, fast_bucket_value<F>(c, a), P);
  }
  if (lane < K) {
    L.acc[lane] = fast_identity<F>();
    L.cnt[lane] = 0;
  }
  WAVE_SYNC();
  return true;
}

template <int F>
__device__ __forceinline__ bool fast_series_end(const GridParams& p, const FastLds& L, int K, int lsb, double amax,
                                                int64_t s, int32_t g) {
  const int lane = lane_id();
  WAVE_SYNC();
  uint32_t nmax = 0;
  for (int k = lane; k < K; k += 64) {
    const uint32_t c = L.cnt[k];
    const double a = L.acc[k];
    nmax = max(nmax, c);
    L.w.pres[k] = c != 0;
    double v;
    if (F == F_SUM || F == F_SQUARESUM) v = c ? a : (double)NAN;
    else if (F == F_AVG) v = c ? a / (double)(int)c : (double)NAN;
    else if (F == F_COUNT) v = (double)c;
    else if (F == F_MIN) v = a == INFINITY ? (double)NAN : a;
    else v = a == -INFINITY ? (double)NAN : a;
    L.acc[k] = v;
  }
  nmax = (uint32_t)wave_max((int)nmax);
  if (needs_cert<F>()) {
    const int Lb = (F == F_SQUARESUM) ? 2 * lsb : lsb;
    const double A = (F == F_SQUARESUM) ? amax * amax : amax;
    const bool ok = (A == 0.0) || (lsb != INT32_MAX && Lb >= -1022 && !isinf(A) &&
                                   (double)nmax * A * (1.0 + 1e-12) <= ldexp(1.0, 52 + Lb));
    if (!ok) return false;
  }
  series_out(p, L.w, K, s, g);
  for (int k = lane; k < K; k += 64) {
    L.acc[k] = fast_identity<F>();
    L.cnt[k] = 0;
    L.w.pres[k] = 0;
  }
  WAVE_SYNC();
  return true;
}

// KR: 0 = LDS partials (rate, K > 64), 1 = register partials, 2 = the fused multi-aggregator
// registers, 3 = register partials with the per-series output modes (sel_direct / dense_out).
template <int F, int QW, int VL, int D, int KR>
__global__ __launch_bounds__(256) void k_fast(GridParams p, const RowDesc* __restrict__ rows,
                                              const int64_t* __restrict__ srp, const int64_t* __restrict__ tbeg,
                                              const int64_t* __restrict__ tend) {
  constexpr bool OUT = KR == 0 || KR == 3;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform (scalar) tile index
  int64_t tile = (int64_t)blockIdx.x * p.waves + wave;
  if (p.tile_list) {   // chained launch over the tiles an earlier k_fast class handed back
    if (tile >= (int64_t)*p.tile_list_n) return;
    tile = p.tile_list[tile];
  }
  if (tile >= p.n_tiles) return;
  const int K = (int)p.K;
  // KR 0 writing the series' buckets to HBM (dense_out: a group-by step over them follows) keeps
  // no partials or rate values in LDS, so large K (a day of 1m buckets) fits the streaming kernels
  const bool dense0 = KR == 0 && p.dense_out != nullptr;
  const FastLds L = fast_carve(smem + (int64_t)wave * p.wave_lds, K, p.rate != 0 && !dense0, !KR && !dense0);
  for (int k = lane; k < K; k += 64) {
    if (!KR && !dense0) part_init(p.ga, L.w.part, k);
    L.acc[k] = fast_identity<F>();
    L.cnt[k] = 0;
    L.w.pres[k] = 0;
  }
  const int32_t tgrp = p.tile_group[tile];   // (loaded once: see k_short)
  std::conditional_t<KR == 2, MultiReg, RegPart> RP;   // KR 2: the fused multi-aggregator pass
  bool uacc = false;   // sel_direct: this tile's union flags (sel_uni_flush)
  rp_init(p.ga, RP);
  FWalk w;
  w.r0 = srp[tbeg[tile]];
  w.r = 0;
  w.rend = (int32_t)(srp[tend[tile]] - w.r0);
  w.c0 = 0;
  w.sf = 0;
  if (w.rend > 0) w.d = fdesc(rows, w.r0);
  if (w.rend > 1) w.nd = fdesc(rows, w.r0 + 1);
  WAVE_SYNC();

  FRaw<QW, VL> buf[D];
  FMeta meta[D];
  bool redo = false;
#pragma unroll
  for (int i = 0; i < D; i++) {
    if (fast_issue<F, QW, VL>(p, rows, w, buf[i], meta[i]) == 2) redo = true;
  }
  if ((meta[0].bits & FM_OK) && !redo && lane == 0) atomicOr(&p.group_active[tgrp], 1u);
  bool have = false;
  int64_t scur = tbeg[tile];   // series of the rows being folded (dense_out / sel_direct)
  int64_t snb = scur + 1 < tend[tile] ? srp[scur + 1] : INT64_MAX;
  int lsb = INT32_MAX;
  double amax = 0.0;
  FGeom g = {0, 0};
  int32_t last_rrel = 0;
  bool done = redo;
  while (!done) {
#pragma unroll
    for (int i = 0; i < D; i++) {
      if (!done) {
        const uint32_t mb = meta[i].bits;
        if (!(mb & FM_OK) || (mb & FM_NEWSER)) {
          if (have) {
            int64_t s = -1;
            if (OUT && (p.dense_out || p.sel_direct)) {   // the series of the last row folded (dense output only)
              // rows come in series order: the cursor only moves forward (a scan from the
              // tile's first series at every series end was quadratic in the tile's series:
              // config 2 ordered 6.5 vs 3.9 ms)
              // snb (the next series' first row) is loaded one series ahead, so the common
              // case waits on no load; only series without rows loop here
              const int64_t row = w.r0 + last_rrel;
              while (snb <= row) {
                scur++;
                snb = scur + 1 < tend[tile] ? srp[scur + 1] : INT64_MAX;
              }
              s = scur;
            }
            const bool ok =
                KR ? fast_series_end_reg<F, true, OUT>(p, L, K, lsb, amax, RP, s, tgrp, 0, nullptr, &uacc)
                   : fast_series_end<F>(p, L, K, lsb, amax, s, tgrp);
            if (!ok) { redo = true; done = true; }
            if (OUT && (p.dense_out || p.sel_direct)) {   // the next series end is a later series
              scur++;
              snb = scur + 1 < tend[tile] ? srp[scur + 1] : INT64_MAX;
            }
          }
          lsb = INT32_MAX;
          amax = 0.0;
          have = true;
          if (!(mb & FM_OK)) done = true;
        }
        if (!done) {
          if (mb & FM_NEWROW) {
            last_rrel = meta[i].rrel;
            const RowDesc& x = rows[w.r0 + meta[i].rrel];
            lsb = min(lsb, x.lsb);
            amax = fmax(amax, x.absmax);
            g = fgeom(p, x.base);
          }
          const int nv0 = (int)(mb & FM_NV);
#ifndef TSDBHIP_NO_ONEB
          if (p.oneb && fast_chunk_oneb<F, QW, VL>(p, L, buf[i], g, nv0, K)) {
          } else
#endif
          if (nv0 >= CH) fast_chunk<F, QW, VL, true>(p, L, buf[i], g, nv0, K);
          else fast_chunk<F, QW, VL, false>(p, L, buf[i], g, nv0, K);
          if (fast_issue<F, QW, VL>(p, rows, w, buf[i], meta[i]) == 2) { redo = true; done = true; }
        }
      }
    }
  }
  if (redo) {
    if (lane == 0) p.redo_list[atomicAdd(p.redo_n, 1)] = (int32_t)tile;
    return;
  }
  if (OUT && p.sel_direct) sel_uni_flush(p, K, tgrp, uacc);
  WAVE_SYNC();
  double* ga_ = p.part.a + tile * K;
  double* gb_ = p.part.b + tile * K;
  uint32_t* gn_ = p.part.n + tile * K;
  uint32_t* gf_ = p.part.f + tile * K;
  if (KR) {
    rp_store(p, tile, K, RP);
    return;
  }
  if (dense0) return;   // (the buckets went to dense_out; no tile partials)
  for (int k = lane; k < K; k += 64) {
    ga_[k] = L.w.part.a[k];
    gb_[k] = L.w.part.b[k];
    gn_[k] = L.w.part.n[k];
    gf_[k] = L.w.part.f[k];
  }
}

// ---- k_short: tiles whose series have exactly one row each (short windows) --------------
// config 3 (10M series x 1 h @10 s) is one 360-point row per series: k_fast's per-row walker
// (scalar descriptor chain, chunk metadata) costs as much as the decode there.  Here lane i
// loads the descriptor of the tile's series i up front, so every chunk address is known and
// the D-deep load ring runs across series with no walker.  Same chunk fold and series end
// as k_fast (bit-identical partials); a tile that breaks a premise goes to the redo list.
template <int QW, int VL>
__device__ __forceinline__ void short_issue(const GridParams& p, uint64_t qoff, uint64_t voff, int ndp,
                                            FRaw<QW, VL>& b) {
  const int lane = lane_id();
#ifdef TSDBHIP_KDBG
  if (p.dbg & 32) { qoff = 0; voff = 0; }
#endif
  const int64_t i0 = (lane * DPL < ndp) ? (int64_t)lane * DPL : 0;
  const uint4* q = reinterpret_cast<const uint4*>(p.qual + qoff + i0 * QW);
#pragma unroll
  for (int k = 0; k < QW / 2; k++) b.q[k] = q[k];
  if (VL == 0) {
    b.v[0] = *reinterpret_cast<const uint4*>(p.val2 + qoff + i0 * 2);   // the lane's 8 int16 values
  } else {
    const uint4* v = reinterpret_cast<const uint4*>(p.val + voff + i0 * VL);
#pragma unroll
    for (int k = 0; k < VL / 2; k++) b.v[k] = v[k];
  }
}

// NP = 6 (vle class, rows of <= 384 datapoints): 6 datapoints a lane, 12 bytes of qualifiers and
// 12 of int16 values (dwordx3 loads at lane * 12), so a 360-point row keeps 60 lanes busy, not 45
template <int QW, int VL, int NP>
__device__ __forceinline__ void short_issue_np(const GridParams& p, uint64_t qoff, uint64_t voff, int ndp,
                                               FRaw<QW, VL>& b) {
  if constexpr (NP == DPL) {
    short_issue<QW, VL>(p, qoff, voff, ndp, b);
  } else {
    static_assert(NP == 6 && QW == 2 && (VL == 0 || VL == 4), "6 a lane: 2-byte qualifiers, vle or 4-byte values");
    const int lane = lane_id();
    const int64_t i0 = (lane * NP < ndp) ? (int64_t)lane * NP : 0;
    const uint3 q = *reinterpret_cast<const uint3*>(p.qual + qoff + i0 * 2);
    b.q[0] = make_uint4(q.x, q.y, q.z, 0u);
    if constexpr (VL == 0) {
      const uint3 v = *reinterpret_cast<const uint3*>(p.val2 + qoff + i0 * 2);
      b.v[0] = make_uint4(v.x, v.y, v.z, 0u);
    } else {   // 24 bytes of float32 values at lane * 24 (16-byte and 8-byte loads)
      const uint8_t* vp = p.val + voff + i0 * 4;
      b.v[0] = *reinterpret_cast<const uint4*>(vp);
      const uint2 t = *reinterpret_cast<const uint2*>(vp + 16);
      b.v[1] = make_uint4(t.x, t.y, 0u, 0u);
    }
  }
}

__device__ __forceinline__ uint64_t rl64(uint64_t x, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

#ifndef SHORT_OCC
// waves per SIMD k_short is compiled for (VGPR budget). Config 3 (round 1): 3-5 -> 3.8 ms,
// 6 -> 4.5 ms, 8 -> 9.4 ms.  Round 2: the 4- and 8-byte classes grew past 5 waves' budget and
// spilled (48-280 B/lane of scratch): they compile for 4, the vle class (93 VGPRs) stays at 5.
#define SHORT_OCC(VL) ((VL) == 0 ? 5 : 4)
#endif
#ifndef SHORT_OCC2_VLE
// The fused multi-aggregator variant (KR 2, tsdbhip_run_multi) holds 13 more registers of
// SpanGroup state: it compiles for 4 (vle at 5 spilled 20 B/lane).
#define SHORT_OCC2_VLE 4
#endif
#define SHORT_OCC2(VL) ((VL) == 0 ? SHORT_OCC2_VLE : 4)
// KR as k_fast.  The profiling switches of TSDBHIP_DBG exist only in a -DTSDBHIP_KDBG build.
template <int F, int QW, int VL, int D, int KR, int NP = DPL>
__global__ __launch_bounds__(256, (KR) == 2 ? SHORT_OCC2(VL) : SHORT_OCC(VL)) void k_short(GridParams p, const RowDesc* __restrict__ rows,
                                               const int64_t* __restrict__ srp, const int64_t* __restrict__ tbeg,
                                               const int64_t* __restrict__ tend) {
  constexpr bool OUT = KR == 0 || KR == 3 || KR == 4 || KR == 5;
  // KR 4: KR 3's percentile output in the (group, slot) column layout, staged in LDS (COLS)
  constexpr bool COLS = KR == 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int64_t tile = (int64_t)blockIdx.x * p.waves + wave;
  if (p.tile_list) {
    if (tile >= (int64_t)*p.tile_list_n) return;
    tile = p.tile_list[tile];
  }
  if (tile >= p.n_tiles) return;
  const int K = (int)p.K;
  const int64_t s0 = tbeg[tile];
  const int ns = (int)(tend[tile] - s0);
  const int64_t r0 = srp[s0];
  // the tile's group bounds for the column layout, loaded before the ring starts (a global load
  // consumed inside the loop waits for every ring load issued before it)
  // (and the tile's group: p.tile_group[tile] read inside the loop is reloaded after every store
  // the compiler cannot tell apart from it -- a load consumed at once, behind the whole ring)
  const int32_t tgrp = p.tile_group[tile];
  int64_t cg0 = 0, cgn = 0;
  if (COLS) {
    cg0 = p.group_series_ptr[tgrp];
    cgn = p.group_series_ptr[tgrp + 1] - cg0;
  }
  // KR 5: lane k's window of column (tgrp, k), loaded before the ring as the group bounds above
  double wlo = 0.0, whi = 0.0;
  double* wbase = nullptr;
  if constexpr (KR == 5) {
    if (lane < K) {
      wlo = p.win_lo[(int64_t)tgrp * K + lane];
      whi = p.win_hi[(int64_t)tgrp * K + lane];
    }
    wbase = p.win_val + tile * K * WIN_CAP;
  }
  // premise: one row per series, in the scan range, of this kernel's class, one chunk long
  bool ok = ns <= 64 && srp[s0 + ns] - r0 == ns;
  uint64_t dq = 0, dv = 0, damax = 0;
  int dbase = 0, dndp = 0, dlsb = INT32_MAX;
  if (ok && lane < ns) {
    const RowDesc& x = rows[r0 + lane];
    dq = x.qoff;
    dv = x.voff;
    dbase = (int)x.base;
    dndp = (int)x.ndp;
    dlsb = x.lsb;
    damax = (uint64_t)__double_as_longlong(x.absmax);
    const uint32_t fl = x.flags;
    ok = (int64_t)x.base >= p.ss && (int64_t)x.base < p.se && dndp >= 1 && dndp <= 64 * NP &&
         fast_row_ok<QW, VL>(fl, F == F_MIN || F == F_MAX, F == F_SUM || F == F_AVG);
  }
  if (!__all(ok)) {
    if (lane == 0) p.redo_list[atomicAdd(p.redo_n, 1)] = (int32_t)tile;
    return;
  }
#ifdef TSDBHIP_KDBG
  if (p.dbg & 16) return;
#endif
  // bucket geometry of every series' row, computed once per tile (lane = series)
  int gq0, gr0;
  {
    const FGeom g = fgeom(p, (uint32_t)dbase);
    gq0 = g.q0;
    gr0 = g.r0;
  }
  // KR 0 writing the series' buckets to HBM (dense_out: a group-by step over them follows) keeps
  // no partials or rate values in LDS, so large K (a day of 1m buckets) fits the streaming kernels
  const bool dense0 = KR == 0 && p.dense_out != nullptr;
  FastLds L = fast_carve(smem + (int64_t)wave * p.wave_lds, K, p.rate != 0 && !dense0, !KR && !dense0);
  if constexpr (KR == 5) L.wstage = (double*)(smem + (int64_t)wave * p.wave_lds + p.win_stage);
  for (int k = lane; k < K; k += 64) {
    if (!KR && !dense0) part_init(p.ga, L.w.part, k);
    L.acc[k] = fast_identity<F>();
    L.cnt[k] = 0;
    L.w.pres[k] = 0;
  }
  std::conditional_t<KR == 2, MultiReg, RegPart> RP;   // KR 2: the fused multi-aggregator pass
  rp_init(p.ga, RP);
  if constexpr (KR == 5) {   // the window state (sel_window_out)
    RP.pa = wlo;
    RP.pb = whi;
    RP.pn = 0;
    RP.pf = 0;
  }
  if (ns > 0 && lane == 0) atomicOr(&p.group_active[tgrp], 1u);
  WAVE_SYNC();
  // The ring issues unconditionally (series index clamped to the last one) so that the
  // compiler's vmcnt bookkeeping stays exact: a conditional issue makes it wait for every
  // outstanding load (vmcnt(0)) and the ring degenerates to one series in flight.
  FRaw<QW, VL> buf[D];
  const int nlast = ns - 1;
#pragma unroll
  for (int i = 0; i < D; i++) {
    const int jn = min(i, nlast);
    short_issue_np<QW, VL, NP>(p, rl64(dq, jn), rl64(dv, jn), __builtin_amdgcn_readlane(dndp, jn), buf[i]);
  }
  bool redo = false;
  auto series = [&](const FRaw<QW, VL>& b, int j) {
    const int nv0 = __builtin_amdgcn_readlane(dndp, j);
    const FGeom g = {__builtin_amdgcn_readlane(gq0, j), __builtin_amdgcn_readlane(gr0, j)};
#ifdef TSDBHIP_KDBG
    if (!(p.dbg & 2)) {   // TSDBHIP_DBG profiling switches (results invalid when set)
      fast_chunk_any<F, QW, VL, NP>(p, L, b, g, nv0, K);
    } else if (p.dbg & 8) {
      uint32_t x = b.q[0].x ^ b.v[0].x;
      if (x == 0x12345678u) L.cnt[0] = x;
    }
#else
    fast_chunk_any<F, QW, VL, NP>(p, L, b, g, nv0, K);
#endif
    return nv0;
  };
  // sel_direct into the column layout (COLS): two LDS stages of 8 series' rows.  Every series end
  // stores one slice (8 columns x 8 series: 64-B pieces) of the previous 8 series' stage, so
  // each iteration issues exactly one store: a store only every 8th series made the compiler's
  // vmcnt count assume none, and the waits for the ring's loads then also waited for the stores
  // (68 % of wave cycles waiting, round-5 PMC).  Before the first 8 are staged the slice stores
  // go to the first 8 series' own entries (rewritten later), masked to this tile.
  double* stage = COLS ? (double*)(smem + (int64_t)wave * p.wave_lds + p.sel_stage) : nullptr;
  const int sl_c = lane >> 3, sl_i = lane & 7;   // a slice lane: column 8 t + sl_c, series sl_i
  double* colbase = COLS ? p.sel_vals + cg0 * K + (s0 - cg0) : nullptr;
  auto slice = [&](int t, int grp, int nrow) {   // slice t of 8-series group grp (rows < nrow)
    const int k = 8 * t + sl_c;
    const double v = stage[((grp & 1) * 8 + sl_i) * K + min(k, K - 1)];
    if (k < K && sl_i < nrow) colbase[(int64_t)k * cgn + grp * 8 + sl_i] = v;
  };
  bool uacc = false;
  auto series_end = [&](int j, int nv0) {
#ifdef TSDBHIP_KDBG
    if (p.dbg & 1) return;
#endif
    const int lsb = __builtin_amdgcn_readlane(dlsb, j);
    const double amax = __longlong_as_double((long long)rl64(damax, j));
    const bool fine =
        KR ? fast_series_end_reg<F, false, KR == 5 ? 3 : KR == 4 ? 2 : (int)OUT>(p, L, K, lsb, amax, RP, s0 + j, tgrp, (uint32_t)nv0,
                                                COLS ? stage + (((j >> 3) & 1) * 8 + (j & 7)) * K : wbase, &uacc)
           : fast_series_end<F>(p, L, K, lsb, amax, s0 + j, tgrp);
    if (!fine) redo = true;
    if constexpr (COLS) {
      WAVE_SYNC();
      const int g = (j >> 3) - 1;   // the previous group (-1: none yet)
      slice(j & 7, max(g, 0), g >= 0 ? 8 : min(8, ns));
    }
  };
  int j = 0;
  for (; j + D <= ns; j += D) {
#pragma unroll
    for (int i = 0; i < D; i++) {
      const int nv0 = series(buf[i], j + i);
      const int jn = min(j + i + D, nlast);
      short_issue_np<QW, VL, NP>(p, rl64(dq, jn), rl64(dv, jn), __builtin_amdgcn_readlane(dndp, jn), buf[i]);
      series_end(j + i, nv0);
    }
    if (redo) break;
  }
  if (!redo) {
#pragma unroll
    for (int i = 0; i < D; i++) {
      if (j + i < ns) {
        const int nv0 = series(buf[i], j + i);
        series_end(j + i, nv0);
      }
    }
  }
  if (redo) {
    if (lane == 0) p.redo_list[atomicAdd(p.redo_n, 1)] = (int32_t)tile;
    return;
  }
  if (COLS && ns > 0) {   // the slices left: the last full group's rest, then the last group whole
    WAVE_SYNC();
    const int last = (ns - 1) >> 3, nb = ns - 8 * last;
    if (last >= 1)
      for (int t = nb; t < 8; t++) slice(t, last - 1, 8);
    for (int t = 0; t < 8; t++) slice(t, last, nb);
  }
  if constexpr (KR == 5) {   // the tile's window counts into its column's, its values inside to the candidates
    if (lane < K && ns > 0) {
      const int64_t col = (int64_t)tgrp * K + lane;
      const uint32_t nin = RP.pf;
      const unsigned long long ba = (unsigned long long)(RP.pn & 0xFFu) | ((unsigned long long)(RP.pn >> 8) << 32);
      if (ba) atomicAdd(&p.win_gcnt[col], ba);
      if (nin) {
        const uint32_t at = atomicAdd(&p.win_cur[col], nin);
        const double* src = wbase + lane * WIN_CAP;
        const double* sl = L.wstage + lane * WIN_LDS;
        double* dst = p.win_cand + col * WIN_CCAP;
        for (uint32_t e = 0; e < nin && at + e < (uint32_t)WIN_CCAP; e++) dst[at + e] = e < (uint32_t)WIN_LDS ? sl[e] : src[e];
      }
    }
    sel_uni_flush(p, K, tgrp, uacc);
    return;
  }
  if (OUT && p.sel_wr && lane < ns) p.sel_wr[s0 + lane] = 1;   // sel_direct: every series of the tile was written
  if (OUT && p.sel_direct) sel_uni_flush(p, K, tgrp, uacc);
  WAVE_SYNC();
  double* ga_ = p.part.a + tile * K;
  double* gb_ = p.part.b + tile * K;
  uint32_t* gn_ = p.part.n + tile * K;
  uint32_t* gf_ = p.part.f + tile * K;
  if (KR) {
    rp_store(p, tile, K, RP);
    return;
  }
  if (dense0) return;   // (the buckets went to dense_out; no tile partials)
  for (int k = lane; k < K; k += 64) {
    ga_[k] = L.w.part.a[k];
    gb_[k] = L.w.part.b[k];
    gn_[k] = L.w.part.n[k];
    gf_[k] = L.w.part.f[k];
  }
}

// ---- k_rows: tiles whose series have several rows, each at most CH datapoints -------------
// A day of 10 s points kept as hour rows (24 rows of 360 per series): k_fast's walker reads
// every row's descriptor with a dependent scalar load before it can issue the row's chunk.
// Here the descriptors come in batches of 64 rows, lane i holding row b*64 + i, two batches
// in registers (the one being folded and the next), so the D-deep ring issues across rows
// and series with no walker.  A series ends at the row where some series' row range ends
// (a ballot over the tile's series ends, lane = series).  Same chunk fold, certificate and
// series end as k_fast (bit-identical partials); a tile that breaks a premise is handed back.
struct RowBatch {
  uint64_t qoff, voff, amax;
  int ndp;    // > 0 in the scan range, 0 out of it (or past the tile), -1 not this kernel's row
  uint32_t base;
  int lsb;
};

template <int F, int QW, int VL, int NP = DPL>
__device__ __forceinline__ void rows_batch(const GridParams& p, const RowDesc* __restrict__ rows, int64_t r0,
                                           int nr, int b, RowBatch& B) {
  const int jr = b * 64 + lane_id();
  const RowDesc& x = rows[r0 + min(jr, nr - 1)];
  B.qoff = x.qoff;
  B.voff = x.voff;
  B.base = x.base;
  B.lsb = x.lsb;
  B.amax = (uint64_t)__double_as_longlong(x.absmax);
  const int n = (int)x.ndp;
  const uint32_t fl = x.flags;   // (no short-circuit: a lane-conditional load waits for all loads)
  const bool in = (jr < nr) & ((int64_t)x.base >= p.ss) & ((int64_t)x.base < p.se);
  const bool ok = (n <= 64 * NP) & fast_row_ok<QW, VL>(fl, F == F_MIN || F == F_MAX, F == F_SUM || F == F_AVG);
  B.ndp = !in ? 0 : (ok ? n : -1);
}

template <int F, int QW, int VL, int D, int KR, int NP = DPL>
__global__ __launch_bounds__(256, (KR) == 2 ? SHORT_OCC2(VL) : SHORT_OCC(VL)) void k_rows(GridParams p, const RowDesc* __restrict__ rows,
                                              const int64_t* __restrict__ srp, const int64_t* __restrict__ tbeg,
                                              const int64_t* __restrict__ tend) {
  static_assert(64 % D == 0, "a batch is a whole number of ring turns");
  constexpr bool OUT = KR == 0 || KR == 3;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int64_t tile = (int64_t)blockIdx.x * p.waves + wave;
  if (p.tile_list) {
    if (tile >= (int64_t)*p.tile_list_n) return;
    tile = p.tile_list[tile];
  }
  if (tile >= p.n_tiles) return;
  const int K = (int)p.K;
  const int64_t s0 = tbeg[tile];
  const int ns = (int)(tend[tile] - s0);
  const int64_t r0 = srp[s0];
  const int64_t nr64 = srp[s0 + ns] - r0;
  if (ns > 64 || nr64 <= 0 || nr64 > INT32_MAX) {
    if (lane == 0) p.redo_list[atomicAdd(p.redo_n, 1)] = (int32_t)tile;
    return;
  }
  const int nr = (int)nr64;
  const int nb = (nr + 63) >> 6;
  // lane = series of the tile: the end of its rows (tile-relative)
  int send = lane < ns ? (int)(srp[s0 + lane + 1] - r0) : INT32_MAX;
  asm volatile("" : "+v"(send));   // kept in its register (not re-loaded from srp at every series end)
  RowBatch cur, nxt;
  rows_batch<F, QW, VL, NP>(p, rows, r0, nr, 0, cur);
  rows_batch<F, QW, VL, NP>(p, rows, r0, nr, min(1, nb - 1), nxt);
  const bool dense0 = KR == 0 && p.dense_out != nullptr;
  const FastLds L = fast_carve(smem + (int64_t)wave * p.wave_lds, K, p.rate != 0 && !dense0, !KR && !dense0);
  for (int k = lane; k < K; k += 64) {
    if (!KR && !dense0) part_init(p.ga, L.w.part, k);
    L.acc[k] = fast_identity<F>();
    L.cnt[k] = 0;
    L.w.pres[k] = 0;
  }
  const int32_t tgrp = p.tile_group[tile];   // (loaded once: see k_short)
  std::conditional_t<KR == 2, MultiReg, RegPart> RP;
  bool uacc = false;
  rp_init(p.ga, RP);
  WAVE_SYNC();
  // ring: rows issued unconditionally (past the tile: its last row, 0 datapoints)
  FRaw<QW, VL> buf[D];
  // (in ring order: the scheduler is kept from issuing buf[1] before buf[0], which made the
  // first fold in the loop wait for every load)
#pragma unroll
  for (int i = 0; i < D; i++) {
    short_issue_np<QW, VL, NP>(p, rl64(cur.qoff, i), rl64(cur.voff, i), max(0, __builtin_amdgcn_readlane(cur.ndp, i)), buf[i]);
    __builtin_amdgcn_sched_barrier(0);
  }
  bool redo = false, have = false, any = false;
  int lsb = INT32_MAX;
  double amax = 0.0;
  uint32_t nser = 0;
  // One loop over the rows (D a turn); the next batch is loaded when a batch is finished.  (A
  // nested batch/row loop was rotated by the compiler so that the loads at the loop's entry
  // made it wait for every outstanding load -- vmcnt(0) -- on every row: no ring at all.)
  for (int j = 0; j < nr && !redo; j += D) {
#pragma unroll
    for (int i = 0; i < D; i++) {
      const int jr = j + i, jl = jr & 63;
      const int nd = __builtin_amdgcn_readlane(cur.ndp, jl);
      if (jr < nr && nd < 0) redo = true;
      if (jr < nr && nd > 0) {
        const FGeom g = fgeom(p, (uint32_t)__builtin_amdgcn_readlane((int)cur.base, jl));
        fast_chunk_any<F, QW, VL, NP>(p, L, buf[i], g, nd, K);
        have = true;
        lsb = min(lsb, __builtin_amdgcn_readlane(cur.lsb, jl));
        amax = fmax(amax, __longlong_as_double((long long)rl64(cur.amax, jl)));
        nser += (uint32_t)nd;
      }
      const int jn = jl + D;   // the ring's next row: this batch or the next
      const uint64_t iq = jn < 64 ? rl64(cur.qoff, jn) : rl64(nxt.qoff, jn - 64);
      const uint64_t iv = jn < 64 ? rl64(cur.voff, jn) : rl64(nxt.voff, jn - 64);
      const int in = jn < 64 ? __builtin_amdgcn_readlane(cur.ndp, jn) : __builtin_amdgcn_readlane(nxt.ndp, jn - 64);
      short_issue_np<QW, VL, NP>(p, iq, iv, max(0, in), buf[i]);
      if (jr < nr && !redo && __ballot(send == jr + 1) != 0) {   // the last row of its series
        if (have) {
          const int64_t s = s0 + __popcll(__ballot(send <= jr));
          const bool fine = KR ? fast_series_end_reg<F, true, OUT>(p, L, K, lsb, amax, RP, s, tgrp, nser, nullptr, &uacc)
                               : fast_series_end<F>(p, L, K, lsb, amax, s, tgrp);
          if (!fine) redo = true;
          any = true;
        }
        have = false;
        lsb = INT32_MAX;
        amax = 0.0;
        nser = 0;
      }
    }
    if (((j + D) & 63) == 0) {
      cur = nxt;
      rows_batch<F, QW, VL, NP>(p, rows, r0, nr, min(((j + D) >> 6) + 1, nb - 1), nxt);
    }
  }
  if (redo) {
    if (lane == 0) p.redo_list[atomicAdd(p.redo_n, 1)] = (int32_t)tile;
    return;
  }
  if (any && lane == 0) atomicOr(&p.group_active[tgrp], 1u);
  if (OUT && p.sel_direct) sel_uni_flush(p, K, tgrp, uacc);
  WAVE_SYNC();
  if (KR) {
    rp_store(p, tile, K, RP);
    return;
  }
  if (dense0) return;
  double* ga_ = p.part.a + tile * K;
  double* gb_ = p.part.b + tile * K;
  uint32_t* gn_ = p.part.n + tile * K;
  uint32_t* gf_ = p.part.f + tile * K;
  for (int k = lane; k < K; k += 64) {
    ga_[k] = L.w.part.a[k];
    gb_[k] = L.w.part.b[k];
    gn_[k] = L.w.part.n[k];
    gf_[k] = L.w.part.f[k];
  }
}

// ---- k_hwin: K > 64 buckets that tile the hour (a day of 1m buckets over hour rows) ---------
// Buckets dividing the hour with slot 0 on an hour (GridParams.win_w = W = 3600 s / interval
// <= 64 slots): every hour row falls in one window of W slots.  The tile is walked window by
// window; in a window every series contributes at most its one row, so the series' buckets and
// the tile's partials of the window fit the wave (registers, KR 1's emit) -- no [series][K]
// bucket store and no group-by pass over it (the dense split).  LERP needs neighbours across
// windows, so a series with a bucket missing inside its data span hands the tile back (the
// general kernel takes it); regular data never does.
// MULTI: the fused multi-aggregator pass (tsdbhip_run_multi, p.multi): every decomposable
// aggregator's window partials at once (MultiReg, as k_short / k_rows KR 2).
// Blocks are dispatched round-robin over the 8 XCDs (block b on XCD b % 8, each XCD its own L2):
// the logical block of b when every XCD takes a contiguous run of logical blocks, so that
// neighbouring logical blocks share an L2 (a bijection of [0, nb)).
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nb) {
  const int64_t q = nb >> 3, r = nb & 7, x = b & 7, j = b >> 3;
  return x * q + min(x, r) + j;
}

template <int F, int QW, int VL, int D, bool MULTI = false, int NP = DPL>
__global__ __launch_bounds__(256, MULTI ? SHORT_OCC2(VL) : SHORT_OCC(VL)) void k_hwin(GridParams p, const RowDesc* __restrict__ rows,
                                                             const int64_t* __restrict__ srp, const int64_t* __restrict__ tbeg,
                                                             const int64_t* __restrict__ tend) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // a work item is a contiguous range of one tile's windows (p.win_split items a tile): the
  // launch's last round of whole tiles left most of the GPU idle (a day: 24 windows a tile)
  const int S = max(1, p.win_split);
  // a tile's window items on one XCD: hour rows h and h + 1 of a series share their edge lines,
  // fetched once into that L2 instead of into two (config 3's day shard: FETCH 1.05x -> 1.01x of
  // the algorithmic bytes for the float class, 1.07x -> 1.02x vle; profiles/r06w)
  const int64_t item = xcd_block(blockIdx.x, gridDim.x) * p.waves + wave;
  int64_t tile = item / S;
  const int part = (int)(item - tile * S);
  if (p.tile_list) {
    if (tile >= (int64_t)*p.tile_list_n) return;
    tile = p.tile_list[tile];
  }
  if (tile >= p.n_tiles) return;
  const int K = (int)p.K;
  const int W = p.win_w;
  const int NW = (K + W - 1) / W;
  const int h0 = (int)((int64_t)part * NW / S), h1 = (int)((int64_t)(part + 1) * NW / S);
  const int64_t s0 = tbeg[tile];
  const int ns = (int)(tend[tile] - s0);
  // a tile goes on the redo list once, whichever of its items hands it back (p.redo_mark: a
  // zeroed word a tile; the list holds one entry a tile)
  auto hand_back = [&]() {
    if (lane == 0 && atomicOr(&p.redo_mark[tile], 1u) == 0) p.redo_list[atomicAdd(p.redo_n, 1)] = (int32_t)tile;
  };
  if (ns > 64) {
    hand_back();
    return;
  }
  int64_t cur = lane < ns ? srp[s0 + lane] : 0;
  const int64_t end = lane < ns ? srp[s0 + lane + 1] : 0;
  bool seen = false;   // the lane's series had a row in an earlier window (of this item or before it)
  if (h0 > 0 && cur < end) {
    // a later item: jump to the series' row of window h0 (one row an hour: first row + h0 - its
    // window), kept when the row before the jump lies in an earlier window; else the window
    // loop below walks the rows from the first
    const RowDesc& x0 = rows[cur];
    const int64_t b0 = (int64_t)x0.base;
    const int64_t rel0 = p.unit_s ? b0 - p.B0n : b0 * 1000 - p.B0n;
    if (b0 >= p.ss && b0 < p.se && rel0 >= 0) {
      const FGeom g0 = fgeom(p, (uint32_t)b0);
      const int w0 = g0.q0 / W;
      const int64_t guess = cur + (h0 - w0);
      if (g0.r0 == 0 && g0.q0 % W == 0 && w0 < h0 && guess <= end) {
        const int64_t bp = (int64_t)rows[guess - 1].base;
        const FGeom gp = fgeom(p, (uint32_t)bp);
        if (bp < p.se && gp.q0 / W < h0) {
          cur = guess;
          seen = true;
        }
      }
    }
  }
  const FastLds L = fast_carve(smem + (int64_t)wave * p.wave_lds, W, false, false);
  for (int k = lane; k < W; k += 64) {
    L.acc[k] = fast_identity<F>();
    L.cnt[k] = 0;
  }
  std::conditional_t<MULTI, MultiReg, RegPart> RP;
  rp_init(p.ga, RP);
  WAVE_SYNC();
  bool redo = false, any = false;
  const bool lerp = p.fill == TSDB_FILL_NONE;   // (the host routes fill policies elsewhere)
  for (int h = h0; h < h1 && !redo; h++) {
    const int Wh = min(W, K - h * W);
    // the lane's row of window h: rows outside the scan range or before slot 0 are passed over
    bool has = false, bad = false;
    uint64_t dq = 0, dv = 0, damax = 0;
    int dndp = 0, dlsb = INT32_MAX, gr0 = 0;
    while (cur < end) {
      const RowDesc& x = rows[cur];
      const int64_t base = (int64_t)x.base;
      const int64_t rel = p.unit_s ? base - p.B0n : base * 1000 - p.B0n;
      if (base < p.ss || base >= p.se || rel < 0) { cur++; continue; }
      const FGeom g = fgeom(p, (uint32_t)base);
      if (g.r0 != 0 || g.q0 % W != 0) { bad = true; break; }   // (host-checked alignment)
      const int wi = g.q0 / W;
      if (wi < h) { seen = true; cur++; continue; }   // (a row of a window before this item's)
      if (wi == h) {
        has = true;
        dq = x.qoff;
        dv = x.voff;
        dndp = (int)x.ndp;
        dlsb = x.lsb;
        damax = (uint64_t)__double_as_longlong(x.absmax);
        gr0 = g.r0;
        bad = !(dndp >= 1 && dndp <= 64 * NP &&
                fast_row_ok<QW, VL>(x.flags, F == F_MIN || F == F_MAX, F == F_SUM || F == F_AVG));
      }
      break;
    }
    // a series without a row here but with rows on both sides: LERP would fill this window
    if (lerp && !has && seen && cur < end) bad = true;
    if (__ballot(bad)) { redo = true; break; }
    uint64_t act = __ballot(has);
    if (act) any = true;
    // the window's series, in order: the ring over them
    FRaw<QW, VL> buf[D];
    int lanes_[D];
    uint64_t rest = act;
#pragma unroll
    for (int i = 0; i < D; i++) {
      const int ln = rest ? (int)__builtin_ctzll(rest) : -1;
      if (rest) rest &= rest - 1;
      lanes_[i] = ln;
      const int l2 = ln < 0 ? 0 : ln;
      short_issue_np<QW, VL, NP>(p, rl64(dq, l2), rl64(dv, l2), ln < 0 ? 0 : __builtin_amdgcn_readlane(dndp, l2), buf[i]);
    }
    const int nact = __popcll(act);
    for (int j = 0; j < nact && !redo; j += D) {
#pragma unroll
      for (int i = 0; i < D; i++) {
        const int ln = lanes_[i];
        if (j + i < nact) {
          const int nv0 = __builtin_amdgcn_readlane(dndp, ln);
          const FGeom g = {0, __builtin_amdgcn_readlane(gr0, ln)};   // window-relative: the row starts at slot 0
          // the row's last datapoint inside the window (a second qualifier can reach 4095 s)
          const int ll = (nv0 - 1) / NP, jl = (nv0 - 1) % NP;
          uint32_t fl = 0;
#pragma unroll
          for (int jj = 0; jj < NP; jj++) if (jj == jl) fl = f_field<QW, VL>(buf[i], jj);
          const int uq = (QW == 2 && !p.unit_s) ? 1000 : 1;
          const int64_t lastn = (int64_t)g.r0 + (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)fl, ll) * uq;
          if (lastn >= (int64_t)W * p.In) redo = true;
          if (!redo) {
            fast_chunk_any<F, QW, VL, NP>(p, L, buf[i], g, nv0, Wh);
            WAVE_SYNC();
            // every bucket of the window present, or fill: the window's emit needs no neighbour
            // from another window
            if (lerp && __ballot(lane < Wh && L.cnt[lane] == 0)) redo = true;
            const int lsb = __builtin_amdgcn_readlane(dlsb, ln);
            const double amax = __longlong_as_double((long long)rl64(damax, ln));
            if (!redo && !fast_series_end_reg<F, false, false>(p, L, Wh, lsb, amax, RP, s0 + ln, p.tile_group[tile],
                                                               (uint32_t)nv0))
              redo = true;
          }
        }
        // next series of the window into this ring slot (issued unconditionally)
        const int ln2 = rest ? (int)__builtin_ctzll(rest) : -1;
        if (rest) rest &= rest - 1;
        lanes_[i] = ln2;
        const int l2 = ln2 < 0 ? 0 : ln2;
        short_issue_np<QW, VL, NP>(p, rl64(dq, l2), rl64(dv, l2), ln2 < 0 ? 0 : __builtin_amdgcn_readlane(dndp, l2), buf[i]);
      }
    }
    if (redo) break;
    // the window's partials: slots h W .. h W + Wh - 1 of the tile
    if (lane < Wh) {
      const int64_t o = tile * K + (int64_t)h * W + lane;
      if constexpr (MULTI) {
        p.mp.sum[o] = RP.sum;
        p.mp.mn[o] = RP.mn;
        p.mp.mx[o] = RP.mx;
        p.mp.mean[o] = RP.mean;
        p.mp.m2[o] = RP.m2;
        p.mp.nl[o] = RP.nl;
        p.mp.nz[o] = RP.nz;
        p.mp.f[o] = RP.f;
      } else {
        p.part.a[o] = RP.pa;
        p.part.b[o] = RP.pb;
        p.part.n[o] = RP.pn;
        p.part.f[o] = RP.pf;
      }
    }
    rp_init(p.ga, RP);
    if (has) { seen = true; cur++; }
  }
  if (redo) {
    hand_back();
    return;
  }
  if (any && lane == 0) atomicOr(&p.group_active[p.tile_group[tile]], 1u);
}

// ---- k_reduce -------------------------------------------------------------------
struct PState {
  double a, b;
  uint32_t n, f;
};

__device__ __forceinline__ PState ps_identity(int ga) {
  PState s;
  s.a = (ga == GA_MIN) ? INFINITY : (ga == GA_MAX ? -INFINITY : 0.0);
  s.b = 0.0;
  s.n = 0;
  s.f = 0;
  return s;
}

// merge B (later series) into A (earlier series)
__device__ __forceinline__ PState ps_merge(int ga, PState A, const PState& B) {
  const uint32_t uni = (A.f | B.f) & PF_UNION;
  switch (ga) {
    case GA_SUM: case GA_AVG: case GA_SQUARESUM:
      A.a += B.a; A.n += B.n; break;
    case GA_COUNT:
      A.n += B.n; break;
    case GA_MIN:
      if (B.a < A.a) A.a = B.a;
      break;
    case GA_MAX:
      if (B.a > A.a) A.a = B.a;
      break;
    case GA_DEV:
      if (B.n == 0) break;
      if (A.n == 0) { A.a = B.a; A.b = B.b; A.n = B.n; break; }
      {
        const double na = A.n, nb = B.n, n = na + nb;
        const double delta = B.a - A.a;
        A.a = A.a + delta * nb / n;
        A.b = A.b + B.b + delta * delta * na * nb / n;
        A.n = A.n + B.n;
      }
      break;
    case GA_FIRST: case GA_NONE:
      if (!(A.f & PF_HAS) && (B.f & PF_HAS)) { A.a = B.a; }
      A.f = (A.f & 3u) | (B.f & PF_HAS) | ((((A.f >> 2) + (B.f >> 2))) << 2);
      break;
    case GA_LAST:
      if (B.f & PF_HAS) A.a = B.a;
      A.f = (A.f & 3u) | (B.f & PF_HAS) | ((((A.f >> 2) + (B.f >> 2))) << 2);
      break;
    case GA_DIFF: {
      const uint32_t totb = B.f >> 2;
      if (A.f & PF_HAS) { A.n += totb; }
      else if (B.f & PF_HAS) { A.a = B.a; A.n = B.n; }
      if (totb > 0) A.b = B.b;
      A.f = (A.f & 3u) | (B.f & PF_HAS) | ((((A.f >> 2) + totb)) << 2);
      break;
    }
    case GA_MULT:
      if (B.f & PF_HAS) A.a = (A.f & PF_HAS) ? A.a * B.a : B.a;
      A.f = (A.f & 3u) | (B.f & PF_HAS) | ((((A.f >> 2) + (B.f >> 2))) << 2);
      break;
  }
  A.f = (A.f & ~PF_UNION) | uni;
  return A;
}

// Aggregator.runDouble results (see bs_final) + AggregationIterator.doubleValue's Inf check
__device__ __forceinline__ double ps_final(int ga, const PState& s, int32_t* err, bool chk_inf = true) {
  double r;
  switch (ga) {
    case GA_SUM: case GA_SQUARESUM: r = s.n == 0 ? (double)NAN : s.a; break;
    case GA_AVG: r = s.n == 0 ? (double)NAN : s.a / (double)(int)s.n; break;
    case GA_COUNT: r = (double)s.n; break;
    case GA_MIN: r = s.a == INFINITY ? (double)NAN : s.a; break;
    case GA_MAX: r = s.a == -INFINITY ? (double)NAN : s.a; break;
    case GA_DEV: r = s.n == 0 ? (double)NAN : (s.n == 1 ? 0.0 : sqrt(s.b / (double)s.n)); break;
    case GA_FIRST: case GA_LAST: case GA_MULT: r = s.a; break;
    case GA_NONE:
      if ((s.f >> 2) > 1) set_err(err, TSDB_E_ILLEGAL_DATA);
      r = s.a;
      break;
    case GA_DIFF: r = !(s.f & PF_HAS) ? (double)NAN : (s.n == 0 ? 0.0 : s.b - s.a); break;
    default: r = NAN;
  }
  if (chk_inf && isinf(r)) set_err(err, TSDB_E_ILLEGAL_STATE);
  return r;
}

}  // namespace tsdb
