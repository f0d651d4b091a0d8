// k_raw.hip -- the raw path: queries without downsampling.
//
// AggregationIterator (src/core/AggregationIterator.java:395-797) walks the UNION of the
// group's datapoint timestamps.  At every union timestamp x it feeds the aggregator one
// value per span, in SpanGroup index order: the span's own value at x, a LERP / ZIM / MAX /
// MIN / PREV value between the span's points around x, or nothing (not started / ended).
// With integer data the LERP is long arithmetic with truncating division, so the
// reference is O(U * k) per group and the values cannot be factored.
//
// GPU formulation (one group chunk at a time):
//   k_raw_decode  one wave per compacted row: every datapoint -> RawPt {ts | FLOAT, bits}
//   k_raw_rate    (rate mode) one wave per series: RateSpan over the points, kept rates
//                 compacted in place (a rate depends only on the point and its predecessor)
//   k_raw_mark    one wave per series: set the point's bit in its group's timestamp bitmap
//   k_raw_scan    one block per group: exclusive popcount prefix over the bitmap -> U
//   k_raw_rank    one wave per series: rank[p] = union points strictly before p
//   k_raw_ts      one thread per bitmap word: the union timestamps, in order
//   k_raw_eval    one wave per strip of RAW_STRIP union points: lanes own union points;
//                 spans are visited sequentially in SpanGroup order, so every aggregator
//                 (float sums included) sees its values in the reference's order.  Per
//                 64-point window a lane-parallel pre-pass advances every span's cursor
//                 (points with rank < window start) and records which window positions
//                 are the span's own points (a 64-bit mask); a lane then finds its
//                 segment with one popcount.
#include "kcommon.h"

namespace tsdb {

// ---- decode -------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_raw_decode(RawParams p) {
  const int lane = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = wave; r < p.n_rows; r += nwaves) {
    const int64_t po = p.row_pt_off[r];
    if (po < 0) continue;
    const RowDesc d = p.rows[r];
    if (d.flags & ROW_ERR) {
      if (lane == 0) set_err(p.err, TSDB_E_ILLEGAL_DATA);
      continue;
    }
    const uint8_t* q = p.qual + d.qoff;
    const uint8_t* v = p.val + d.voff;
    const uint32_t qw = d.flags & ROW_QW_MASK;
    const int64_t base_ms = (int64_t)d.base * 1000;
    long long vcarry = 0;
    uint32_t qcarry = 0;
    for (uint32_t i0 = 0; i0 < d.ndp; i0 += 64) {
      const uint32_t i = i0 + lane;
      const bool in = i < d.ndp;
      uint32_t qpos = 0, w = 2;
      if (qw) {
        w = qw;
        qpos = i * w;
      } else {
        // mixed second / millisecond qualifiers (MS_MIXED_COMPACT): positions by a walk
        uint32_t pos = qcarry, mypos = 0, myw = 2;
        for (int t = 0; t < 64 && i0 + t < d.ndp; t++) {
          const uint32_t ww = ((q[pos] & 0xF0) == 0xF0) ? 4 : 2;
          if (t == lane) { mypos = pos; myw = ww; }
          pos += ww;
        }
        qpos = mypos;
        w = myw;
        qcarry = __shfl(pos, 0, 64);
      }
      uint32_t qq = 0;
      if (in) {
        if (w == 4) qq = ((uint32_t)q[qpos] << 24) | ((uint32_t)q[qpos + 1] << 16) | ((uint32_t)q[qpos + 2] << 8) | q[qpos + 3];
        else qq = ((uint32_t)q[qpos] << 8) | q[qpos + 1];
      }
      const uint32_t fl = qq & 0xF;
      const int len = in ? (int)(fl & 7) + 1 : 0;
      const int incl = wave_incl_sum(len);
      const long long vo = vcarry + incl - len;
      vcarry += __shfl(incl, 63, 64);
      if (in) {
        // Internal.getOffsetFromQualifier (src/core/Internal.java:647-658)
        const int64_t off = (w == 4) ? (int64_t)((qq & 0x0FFFFFC0u) >> 6) : (int64_t)(qq >> 4) * 1000;
        uint64_t bits = 0;
        for (int b = 0; b < len; b++) bits = (bits << 8) | v[vo + b];
        RawPt pt;
        pt.tsf = base_ms + off;
        const bool is_float = (fl & 8) != 0;
        if (is_float) {
          // RowSeq.extractFloatingPointValue (src/core/RowSeq.java:256-266)
          if (len == 4) pt.bits = (uint64_t)__double_as_longlong((double)__uint_as_float((uint32_t)bits));
          else if (len == 8) pt.bits = bits;
          else set_err(p.err, TSDB_E_ILLEGAL_DATA);
          pt.tsf |= RAW_FLOAT;
        } else {
          // RowSeq.extractIntegerValue (src/core/RowSeq.java:233-245)
          switch (len) {
            case 1: pt.bits = (uint64_t)(int64_t)(int8_t)(uint8_t)bits; break;
            case 2: pt.bits = (uint64_t)(int64_t)(int16_t)(uint16_t)bits; break;
            case 4: pt.bits = (uint64_t)(int64_t)(int32_t)(uint32_t)bits; break;
            case 8: pt.bits = bits; break;
            default: pt.bits = 0; set_err(p.err, TSDB_E_ILLEGAL_DATA);
          }
        }
        p.pts[po + i] = pt;
      }
    }
  }
}

// ---- RateSpan over raw points ----------------------------------------------------------
__device__ __forceinline__ double pt_double(int64_t tsf, uint64_t bits) {
  return (tsf & RAW_FLOAT) ? __longlong_as_double((long long)bits) : (double)(long long)bits;
}

// RateSpan.populateNextRate (src/core/RateSpan.java:121-180): the rate at every point
// against its predecessor (the first against (t=0, long 0), :112); with drop_resets a
// negative counter delta drops the point but it stays the predecessor of the next one.
__global__ __launch_bounds__(256) void k_raw_rate(RawParams p) {
  const int lane = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t s = wave; s < p.n_series; s += nwaves) {
    const int64_t b0 = p.sp_off[s];
    const int64_t n = p.sp_off[s + 1] - b0;
    int64_t prev_tsf = 0;            // (0, long 0)
    uint64_t prev_bits = 0;
    int64_t kept = 0;
    for (int64_t i0 = 0; i0 < n; i0 += 64) {
      const int64_t i = i0 + lane;
      const bool in = i < n;
      RawPt cur = {0, 0};
      if (in) cur = p.pts[b0 + i];
      int64_t ptsf = __shfl_up(cur.tsf, 1, 64);
      uint64_t pbits = __shfl_up(cur.bits, 1, 64);
      if (lane == 0) { ptsf = prev_tsf; pbits = prev_bits; }
      bool keep = false;
      double rate = 0.0;
      if (in) {
        const int64_t t0 = ptsf & RAW_TIME_MASK, t1 = cur.tsf & RAW_TIME_MASK;
        if (t1 <= t0) set_err(p.err, TSDB_E_ILLEGAL_STATE);
        const double dt = (double)(t1 - t0) / 1000.0;
        const bool ints = !(ptsf & RAW_FLOAT) && !(cur.tsf & RAW_FLOAT);
        double diff = ints ? (double)(long long)(cur.bits - pbits) : pt_double(cur.tsf, cur.bits) - pt_double(ptsf, pbits);
        keep = true;
        if (p.counter && diff < 0) {
          if (p.drop) {
            keep = false;
          } else {
            if (ints) diff = (double)(long long)((uint64_t)p.counter_max - pbits + cur.bits);
            else diff = (double)p.counter_max - pt_double(ptsf, pbits) + pt_double(cur.tsf, cur.bits);
            rate = diff / dt;
            if (p.reset_value > 0 && rate > (double)p.reset_value) rate = 0.0;
          }
        } else {
          rate = diff / dt;
        }
      }
      const int incl = wave_incl_sum(keep ? 1 : 0);
      const int64_t pos = kept + incl - (keep ? 1 : 0);
      const int last = (int)min((int64_t)63, n - 1 - i0);
      prev_tsf = __shfl(cur.tsf, last, 64);
      prev_bits = __shfl(cur.bits, last, 64);
      kept += __shfl(incl, 63, 64);
      if (keep) {
        RawPt o;
        o.tsf = (cur.tsf & RAW_TIME_MASK) | RAW_FLOAT;
        o.bits = (uint64_t)__double_as_longlong(rate);
        p.pts[b0 + pos] = o;   // pos <= i: every lane read its point before any store
      }
    }
    if (lane == 0) p.sp_n[s] = (int32_t)kept;
  }
}

// ---- union bitmap -------------------------------------------------------------------
__device__ __forceinline__ int64_t group_of_series(const RawParams& p, int64_t s) {
  // grp_ser is monotonic; series s of the chunk belongs to the last g with grp_ser[g] <= s
  int64_t lo = p.g0, hi = p.g1;
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (p.grp_ser[mid] <= s) lo = mid; else hi = mid;
  }
  return lo;
}

// first counted point of a series: in rate mode the first kept rate is not a union member
// (the AggregationIterator constructor pre-advances every span, :448-459)
__device__ __forceinline__ int64_t first_counted(const RawParams& p, int64_t n) { return p.rate ? 1 : 0; }

__global__ __launch_bounds__(256) void k_raw_mark(RawParams p, int64_t s_begin, int64_t s_end) {
  const int lane = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t s = s_begin + wave; s < s_end; s += nwaves) {
    const int64_t g = group_of_series(p, s);
    const int64_t n = p.sp_n[s];
    if (p.rate && n < 2) continue;
    uint32_t* bm = p.bitmap + (g - p.g0) * p.W;
    const RawPt* pts = p.pts + p.sp_off[s];
    for (int64_t j = first_counted(p, n) + lane; j < n; j += 64) {
      const int64_t bit = ((pts[j].tsf & RAW_TIME_MASK) - p.start_ms) / p.gran;
      if (bit < 0 || bit >= p.W * 32) { set_err(p.err, TSDB_E_ILLEGAL_DATA); continue; }
      atomicOr(&bm[bit >> 5], 1u << (bit & 31));
    }
  }
}

__global__ __launch_bounds__(256) void k_raw_scan(RawParams p) {
  __shared__ int64_t part[256];
  const int64_t gi = blockIdx.x;
  const uint32_t* bm = p.bitmap + gi * p.W;
  uint32_t* wb = p.wbase + gi * p.W;
  const int64_t per = (p.W + 255) / 256;
  const int64_t a = min(p.W, (int64_t)threadIdx.x * per), b = min(p.W, a + per);
  int64_t sum = 0;
  for (int64_t w = a; w < b; w++) sum += __popc(bm[w]);
  part[threadIdx.x] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t run = 0;
    for (int t = 0; t < 256; t++) { const int64_t x = part[t]; part[t] = run; run += x; }
    p.U[gi] = (int32_t)run;
  }
  __syncthreads();
  int64_t run = part[threadIdx.x];
  for (int64_t w = a; w < b; w++) { wb[w] = (uint32_t)run; run += __popc(bm[w]); }
}

__device__ __forceinline__ int32_t rank_of(const RawParams& p, int64_t gi, int64_t ts) {
  const int64_t bit = (ts - p.start_ms) / p.gran;
  const int64_t w = bit >> 5;
  const uint32_t m = p.bitmap[gi * p.W + w] & ((1u << (bit & 31)) - 1u);
  return (int32_t)(p.wbase[gi * p.W + w] + __popc(m));
}

__global__ __launch_bounds__(256) void k_raw_rank(RawParams p, int64_t s_begin, int64_t s_end) {
  const int lane = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t s = s_begin + wave; s < s_end; s += nwaves) {
    const int64_t gi = group_of_series(p, s) - p.g0;
    const int64_t n = p.sp_n[s];
    const int64_t b0 = p.sp_off[s];
    for (int64_t j = lane; j < n; j += 64) p.rank[b0 + j] = rank_of(p, gi, p.pts[b0 + j].tsf & RAW_TIME_MASK);
  }
}

__global__ __launch_bounds__(256) void k_raw_ts(RawParams p) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = (p.g1 - p.g0) * p.W;
  if (i >= n) return;
  const int64_t gi = i / p.W, w = i - gi * p.W;
  uint32_t m = p.bitmap[i];
  int64_t o = p.out_off[gi] + p.wbase[i];
  while (m) {
    const int b = __ffs(m) - 1;
    m &= m - 1;
    p.out_ts[o++] = p.start_ms + (w * 32 + b) * p.gran;
  }
}

// ---- evaluation ---------------------------------------------------------------------
// Java long arithmetic (wrapping) and the LERP of nextLongValue (:682-729):
//   y0 + (x - x0) * (y1 - y0) / (x1 - x0)   with truncating division
__device__ __forceinline__ int64_t jdiv_pos(int64_t num, int64_t den) {
  // den > 0.  |num| < 2^53: double quotient, corrected to the exact truncated one.
  const uint64_t an = num < 0 ? (uint64_t)0 - (uint64_t)num : (uint64_t)num;
  if (an < (1ULL << 53) && den < (1LL << 53)) {
    int64_t q = (int64_t)((double)num / (double)den);
    int64_t r = num - q * den;
    if (num >= 0) {
      if (r < 0) { q--; r += den; }
      if (r >= den) { q++; }
    } else {
      if (r > 0) { q++; r -= den; }
      if (r <= -den) { q--; }
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

// nextDoubleValue (:735-797)
__device__ __forceinline__ double dlerp(int interp, int64_t x, int64_t x0, double y0, int64_t x1, double y1) {
  switch (interp) {
    case TSDB_INTERP_LERP: return y0 + (double)(x - x0) * (y1 - y0) / (double)(x1 - x0);
    case TSDB_INTERP_ZIM: return 0.0;
    case TSDB_INTERP_MAX: return DBL_MAX;
    case TSDB_INTERP_MIN: return 4.9e-324;   // Double.MIN_VALUE
    default: return y0;
  }
}

// Aggregator.runLong / runDouble as a stream over the spans' values in index order
// (src/core/Aggregators.java; the oracle's agg_run_long / agg_run_double).
struct RAcc {
  double da, db;      // runDouble state
  int64_t la;         // runLong state
  double lm, lM2;     // runLong dev (Welford in double)
  int32_t dn, ln;     // counts
  int32_t dst, lst;   // stage flags
  uint64_t lfirst;    // runLong diff: first value
  bool bad;           // NONE with more than one value
};

__device__ __forceinline__ void racc_init(RAcc& a, int ga) {
  a.da = (ga == GA_MIN) ? INFINITY : (ga == GA_MAX ? -INFINITY : 0.0);
  a.db = 0.0;
  a.la = 0;
  a.lm = 0.0;
  a.lM2 = 0.0;
  a.dn = 0;
  a.ln = 0;
  a.dst = 0;
  a.lst = 0;
  a.lfirst = 0;
  a.bad = false;
}

__device__ __forceinline__ void racc_double(RAcc& a, int ga, double x) {
  switch (ga) {
    case GA_SUM: case GA_AVG: if (!isnan(x)) { a.da += x; a.dn++; } break;
    case GA_SQUARESUM: if (!isnan(x)) { a.da += x * x; a.dn++; } break;
    case GA_COUNT: if (!isnan(x)) a.dn++; break;
    case GA_MIN: if (!isnan(x) && x < a.da) a.da = x; break;
    case GA_MAX: if (!isnan(x) && x > a.da) a.da = x; break;
    case GA_DEV:
      if (a.dst == 0) {
        if (!isnan(x)) { a.da = x; a.dst = 1; a.dn = 2; }
      } else if (!isnan(x)) {
        const double nm = a.da + (x - a.da) / (double)a.dn;
        a.db += (x - a.da) * (x - nm);
        a.da = nm;
        a.dn++;
      }
      break;
    case GA_DIFF:
      if (a.dst == 0) { if (!isnan(x)) { a.da = x; a.dst = 1; } }
      else { a.db = x; a.dst = 2; }
      break;
    case GA_FIRST: if (a.dst == 0) { a.da = x; a.dst = 1; } break;
    case GA_LAST: a.da = x; break;
    case GA_MULT: a.da = a.dst ? a.da * x : x; a.dst = 1; break;
    case GA_NONE: if (a.dst) a.bad = true; a.da = x; a.dst = 1; break;
  }
}

__device__ __forceinline__ double racc_double_final(const RAcc& a, int ga) {
  switch (ga) {
    case GA_SUM: case GA_SQUARESUM: return a.dn == 0 ? (double)NAN : a.da;
    case GA_AVG: return a.dn == 0 ? (double)NAN : a.da / (double)a.dn;
    case GA_COUNT: return (double)a.dn;
    case GA_MIN: return a.da == INFINITY ? (double)NAN : a.da;
    case GA_MAX: return a.da == -INFINITY ? (double)NAN : a.da;
    case GA_DEV: return a.dst == 0 ? (double)NAN : (a.dn == 2 ? 0.0 : sqrt(a.db / (double)(a.dn - 1)));
    case GA_DIFF: return a.dst == 0 ? (double)NAN : (a.dst == 1 ? 0.0 : a.db - a.da);
    default: return a.da;
  }
}

__device__ __forceinline__ void racc_long(RAcc& a, int ga, int64_t x) {
  const uint64_t ux = (uint64_t)x;
  switch (ga) {
    case GA_SUM: a.la = (int64_t)((uint64_t)a.la + ux); break;
    case GA_AVG: a.la = (int64_t)((uint64_t)a.la + ux); a.ln++; break;
    case GA_SQUARESUM: a.la = (int64_t)((uint64_t)a.la + ux * ux); break;
    case GA_COUNT: a.ln++; break;
    case GA_MIN: if (a.lst == 0 || x < a.la) a.la = x; a.lst = 1; break;
    case GA_MAX: if (a.lst == 0 || x > a.la) a.la = x; a.lst = 1; break;
    case GA_DEV:
      if (a.lst == 0) { a.lm = (double)x; a.lst = 1; a.ln = 2; }
      else {
        const double xd = (double)x;
        const double nm = a.lm + (xd - a.lm) / (double)a.ln;
        a.lM2 += (xd - a.lm) * (xd - nm);
        a.lm = nm;
        a.ln++;
        a.lst = 2;
      }
      break;
    case GA_DIFF:
      if (a.lst == 0) { a.lfirst = ux; a.lst = 1; }
      else { a.la = x; a.lst = 2; }
      break;
    case GA_FIRST: if (a.lst == 0) { a.la = x; a.lst = 1; } break;
    case GA_LAST: a.la = x; break;
    case GA_MULT: a.la = a.lst ? (int64_t)((uint64_t)a.la * ux) : x; a.lst = 1; break;
    case GA_NONE: if (a.lst) a.bad = true; a.la = x; a.lst = 1; break;
  }
}

__device__ __forceinline__ int64_t jd2l(double d) {
  if (isnan(d)) return 0;
  if (d >= 9223372036854775807.0) return 0x7FFFFFFFFFFFFFFFLL;
  if (d <= -9223372036854775808.0) return (int64_t)0x8000000000000000ULL;
  return (int64_t)d;
}

__device__ __forceinline__ int64_t racc_long_final(const RAcc& a, int ga) {
  switch (ga) {
    case GA_AVG: return a.ln == 0 ? 0 : (a.la == (int64_t)0x8000000000000000ULL && a.ln == -1 ? a.la : a.la / a.ln);
    case GA_COUNT: return a.ln;
    case GA_DEV: return a.lst < 2 ? 0 : jd2l(sqrt(a.lM2 / (double)(a.ln - 1)));
    case GA_DIFF: return a.lst < 2 ? 0 : (int64_t)((uint64_t)a.la - a.lfirst);
    default: return a.la;
  }
}

template <bool DL, bool DD>
__device__ __forceinline__ void raw_eval_strip(const RawParams& p, int64_t strip, int32_t* cur, uint64_t* mask) {
  const int lane = lane_id();
  const int64_t gi = p.strip_g[strip];
  const int64_t g = gi + p.g0;
  const int64_t U = p.U[gi];
  const int64_t ua = p.strip_u[strip];
  const int64_t ub = min(U, ua + (int64_t)RAW_STRIP);
  const int64_t sb = p.grp_ser[g];
  const int k = (int)(p.grp_ser[g + 1] - sb);
  const int first = p.rate ? 1 : 0;
  const int ga = p.ga;
  // cursors at the strip start: counted points with rank < ua (binary search)
  for (int i = lane; i < k; i += 64) {
    const int64_t s = sb + i;
    const int n = p.sp_n[s];
    const int32_t* rk = p.rank + p.sp_off[s];
    int lo = first, hi = max(first, n);
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (rk[mid] < ua) lo = mid + 1; else hi = mid;
    }
    cur[i] = lo - first;
  }
  WAVE_SYNC();
  const int64_t obase = p.out_off[gi];
  for (int64_t u0 = ua; u0 < ub; u0 += 64) {
    // pre-pass: each span's own points in [u0, u0 + 64)
    for (int i = lane; i < k; i += 64) {
      const int64_t s = sb + i;
      const int n = p.sp_n[s];
      const int32_t* rk = p.rank + p.sp_off[s];
      int c = cur[i] + first;
      uint64_t M = 0;
      while (c < n) {
        const int32_t r = rk[c];
        if (r >= u0 + 64) break;
        M |= 1ULL << (r - u0);
        c++;
      }
      mask[i] = M;
    }
    WAVE_SYNC();
    const int64_t u = u0 + lane;
    const int64_t x = (u < ub) ? (p.out_ts[obase + u] & RAW_TIME_MASK) : 0;
    const uint64_t below = (lane == 63) ? ~0ULL : ((2ULL << lane) - 1ULL);
    RAcc acc;
    racc_init(acc, ga);
    bool flt = false;
    for (int i = 0; i < k; i++) {
      const int64_t s = sb + i;
      const int n = p.sp_n[s];
      if (p.rate && n < 2) continue;
      const RawPt* pts = p.pts + p.sp_off[s];
      const uint64_t M = mask[i];
      const int cnt = cur[i] + __popcll(M & below);
      const bool own = (M >> lane) & 1ULL;
      if (p.rate) {
        // step semantics (:744-753): the latest rate at or before x, the first kept rate
        // before the span's second one; ended after its last rate (the zeroing, :521-526)
        if (cnt == n - 1 && !own) continue;
        const RawPt r = pts[cnt];
        racc_double(acc, ga, __longlong_as_double((long long)r.bits));
        continue;
      }
      if (cnt == 0) {   // not started: its next slot still counts for isInteger (:612-625)
        flt |= (pts[0].tsf & RAW_FLOAT) != 0;
        continue;
      }
      const int j = cnt - 1;
      const RawPt a = pts[j];
      if (j == n - 1) {
        if (!own) continue;   // ended
        flt |= (a.tsf & RAW_FLOAT) != 0;
        if (DL) racc_long(acc, ga, (int64_t)a.bits);
        if (DD) racc_double(acc, ga, pt_double(a.tsf, a.bits));
        continue;
      }
      const RawPt b = pts[j + 1];
      flt |= ((a.tsf | b.tsf) & RAW_FLOAT) != 0;
      if (own) {
        if (DL) racc_long(acc, ga, (int64_t)a.bits);
        if (DD) racc_double(acc, ga, pt_double(a.tsf, a.bits));
      } else {
        const int64_t x0 = a.tsf & RAW_TIME_MASK, x1 = b.tsf & RAW_TIME_MASK;
        if (DL) racc_long(acc, ga, jlerp(p.interp, x, x0, (int64_t)a.bits, x1, (int64_t)b.bits));
        if (DD) racc_double(acc, ga, dlerp(p.interp, x, x0, pt_double(a.tsf, a.bits), x1, pt_double(b.tsf, b.bits)));
      }
    }
    if (u < ub) {
      const bool is_int = !p.rate && !flt;
      uint64_t bits;
      if (is_int) {
        bits = DL ? (uint64_t)racc_long_final(acc, ga) : 0;
        if (!DL) set_err(p.err, TSDB_E_HIP);   // planning error: integer output without the long path
      } else {
        const double r = DD ? racc_double_final(acc, ga) : 0.0;
        if (!DD) set_err(p.err, TSDB_E_HIP);
        if (isinf(r)) set_err(p.err, TSDB_E_ILLEGAL_STATE);   // doubleValue (:640-643)
        bits = (uint64_t)__double_as_longlong(r);
      }
      if (acc.bad) set_err(p.err, TSDB_E_ILLEGAL_DATA);   // None: "More than one value" (:454-460)
      p.out_bits[obase + u] = bits;
      p.out_int[obase + u] = is_int ? 1 : 0;
    }
    WAVE_SYNC();
    for (int i = lane; i < k; i += 64) cur[i] += __popcll(mask[i]);
    WAVE_SYNC();
  }
}

template <bool DL, bool DD>
__global__ __launch_bounds__(64) void k_raw_eval(RawParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int64_t strip = blockIdx.x;
  if (strip >= p.n_strips) return;
  int32_t* cur;
  uint64_t* mask;
  if (p.kmax <= RAW_LDS_SPANS) {
    mask = reinterpret_cast<uint64_t*>(smem);
    cur = reinterpret_cast<int32_t*>(smem + (size_t)p.kmax * 8);
  } else {
    mask = p.g_mask + strip * p.kmax;
    cur = p.g_cur + strip * p.kmax;
  }
  raw_eval_strip<DL, DD>(p, strip, cur, mask);
}

// ---- launchers --------------------------------------------------------------------
static unsigned wave_blocks(int64_t n_waves) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n_waves + 3) / 4, 65536));
}

hipError_t launch_raw_decode(const RawParams& p, hipStream_t s) {
  if (p.n_rows == 0) return hipSuccess;
  hipLaunchKernelGGL(k_raw_decode, dim3(wave_blocks(p.n_rows)), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_raw_rate(const RawParams& p, hipStream_t s) {
  if (p.n_series == 0) return hipSuccess;
  hipLaunchKernelGGL(k_raw_rate, dim3(wave_blocks(p.n_series)), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_raw_union(const RawParams& p, int64_t s_begin, int64_t s_end, hipStream_t s) {
  if (s_end > s_begin) {
    hipLaunchKernelGGL(k_raw_mark, dim3(wave_blocks(s_end - s_begin)), dim3(256), 0, s, p, s_begin, s_end);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (p.g1 > p.g0) hipLaunchKernelGGL(k_raw_scan, dim3((unsigned)(p.g1 - p.g0)), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_raw_rank(const RawParams& p, int64_t s_begin, int64_t s_end, hipStream_t s) {
  if (s_end > s_begin) {
    hipLaunchKernelGGL(k_raw_rank, dim3(wave_blocks(s_end - s_begin)), dim3(256), 0, s, p, s_begin, s_end);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const int64_t nw = (p.g1 - p.g0) * p.W;
  if (nw > 0) hipLaunchKernelGGL(k_raw_ts, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_raw_eval(const RawParams& p, hipStream_t s) {
  if (p.n_strips == 0) return hipSuccess;
  const size_t lds = p.kmax <= RAW_LDS_SPANS ? (size_t)p.kmax * 12 + 16 : 16;
  const dim3 grid((unsigned)p.n_strips), block(64);
  if (p.do_long && p.do_double) hipLaunchKernelGGL((k_raw_eval<true, true>), grid, block, lds, s, p);
  else if (p.do_long) hipLaunchKernelGGL((k_raw_eval<true, false>), grid, block, lds, s, p);
  else hipLaunchKernelGGL((k_raw_eval<false, true>), grid, block, lds, s, p);
  return hipGetLastError();
}

}  // namespace tsdb
