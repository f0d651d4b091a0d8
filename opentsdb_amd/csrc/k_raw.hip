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
//   k_raw_cursor  one wave per series: the span's cursor at every strip start
//   k_raw_eval    (k_raw_eval.hip) one wave per strip of RAW_STRIP union points.
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

// ---- strip cursors -----------------------------------------------------------------
// cur[t][i] = counted points of span i with rank < t * RAW_STRIP.  Counted point q (rank
// r_q, strictly increasing) is the cursor of the strips t with r_{q-1} < t * S <= r_q.
__global__ __launch_bounds__(256) void k_raw_cursor(RawParams p, int64_t s_begin, int64_t s_end) {
  const int lane = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t s = s_begin + wave; s < s_end; s += nwaves) {
    const int64_t g = group_of_series(p, s);
    const int64_t gi = g - p.g0;
    const int64_t U = p.U[gi];
    const int64_t ns = (U + RAW_STRIP - 1) / RAW_STRIP;
    const int64_t n = p.sp_n[s];
    const int first = p.rate ? 1 : 0;
    const int64_t nc = max((int64_t)0, n - first);
    const int64_t k = p.grp_ser[g + 1] - p.grp_ser[g];
    const int64_t i = s - p.grp_ser[g];
    int32_t* cur = p.cur + p.cur_off[gi] + i;
    const int32_t* rk = p.rank + p.sp_off[s] + first;
    for (int64_t q = lane; q <= nc; q += 64) {
      const int64_t t_lo = q == 0 ? 0 : (int64_t)rk[q - 1] / RAW_STRIP + 1;
      const int64_t t_hi = q == nc ? ns - 1 : (int64_t)rk[q] / RAW_STRIP;
      for (int64_t t = t_lo; t <= t_hi; t++) cur[t * k] = (int32_t)q;
    }
  }
}

// ---- greedy merge over cells with unsorted datapoints -------------------------------
// AggregationIterator.next (src/core/AggregationIterator.java:514-567) emits the smallest next
// timestamp of the group's spans and advances every span whose next point has it; a span's
// points are consumed in stored order whatever their timestamps (RowSeq.Iterator.next,
// src/core/RowSeq.java:552-568, does not sort), so over unsorted cells the emitted sequence is
// not the sorted union and a timestamp may be emitted more than once.  One wave per group
// walks those steps: lane l keeps the minimum next timestamp of its spans (l, l + 64, ...),
// the wave minimum is the step's timestamp and the lanes holding it advance their spans.
// Every counted point gets its step as rank (strictly increasing along a span), so
// k_raw_cursor and the evaluation kernels run unchanged on top.
__device__ __forceinline__ int64_t wave_min64(int64_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) x = min(x, (int64_t)__shfl_xor((long long)x, d, 64));
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ int64_t merge_head(const RawParams& p, const RawPt* pts, int pos, int n) {
  if (pos >= n) return INT64_MAX;
  const int64_t t = pts[pos].tsf & RAW_TIME_MASK;
  const int64_t bit = (t - p.start_ms) / p.gran;
  if (t < p.start_ms || bit >= p.W * 32) set_err(p.err, TSDB_E_ILLEGAL_DATA);   // as k_raw_mark
  return t;
}

__global__ __launch_bounds__(256) void k_raw_merge(RawParams p) {
  const int lane = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int first = p.rate ? 1 : 0;   // rate: the constructor pre-advances every span (:448-459)
  for (int64_t gi = wave; gi < p.g1 - p.g0; gi += nwaves) {
    const int64_t g = gi + p.g0;
    const int64_t sb = p.grp_ser[g];
    const int64_t k = p.grp_ser[g + 1] - sb;
    int64_t* mts = p.mts + p.bnd_off[gi];
    if (k == 1) {   // one span: every point is a step of its own, in stored order
      const int n = p.sp_n[sb];
      const RawPt* pts = p.pts + p.sp_off[sb];
      for (int j = first + lane; j < n; j += 64) {
        mts[j - first] = merge_head(p, pts, j, n);
        p.rank[p.sp_off[sb] + j] = j - first;
      }
      if (lane == 0) p.U[gi] = max(0, n - first);
      continue;
    }
    int64_t lm = INT64_MAX;
    for (int64_t i = lane; i < k; i += 64) {
      const int64_t s = sb + i;
      const int64_t h = merge_head(p, p.pts + p.sp_off[s], first, p.sp_n[s]);
      p.m_pos[s] = first;
      p.m_head[s] = h;
      lm = min(lm, h);
    }
    int32_t step = 0;
    for (;;) {
      const int64_t m = wave_min64(lm);
      if (m == INT64_MAX) break;
      if (lane == 0) mts[step] = m;
      if (lm == m) {
        int64_t nm = INT64_MAX;
        for (int64_t i = lane; i < k; i += 64) {
          const int64_t s = sb + i;
          int64_t h = p.m_head[s];
          if (h == m) {
            const int pos = p.m_pos[s];
            p.rank[p.sp_off[s] + pos] = step;
            h = merge_head(p, p.pts + p.sp_off[s], pos + 1, p.sp_n[s]);
            p.m_pos[s] = pos + 1;
            p.m_head[s] = h;
          }
          nm = min(nm, h);
        }
        lm = nm;
      }
      step++;
    }
    if (lane == 0) p.U[gi] = step;
  }
}

// step timestamps from the per-group bound layout into the output layout
__global__ __launch_bounds__(256) void k_raw_merge_ts(RawParams p) {
  const int lane = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t gi = wave; gi < p.g1 - p.g0; gi += nwaves) {
    const int64_t U = p.U[gi];
    const int64_t* src = p.mts + p.bnd_off[gi];
    int64_t* dst = p.out_ts + p.out_off[gi];
    for (int64_t u = lane; u < U; u += 64) dst[u] = src[u];
  }
}

// a long LERP that divided by zero raises ArithmeticException only where nextLongValue ran,
// i.e. at points whose result is an integer (k_raw_vals records it per point)
__global__ __launch_bounds__(256) void k_raw_dz_check(RawParams p, int64_t n_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_out && p.dz[i] && p.out_int[i]) set_err(p.err, TSDB_E_ILLEGAL_STATE);
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

hipError_t launch_raw_merge(const RawParams& p, hipStream_t s) {
  if (p.g1 <= p.g0) return hipSuccess;
  hipLaunchKernelGGL(k_raw_merge, dim3(wave_blocks(p.g1 - p.g0)), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_raw_merge_ts(const RawParams& p, hipStream_t s) {
  if (p.g1 <= p.g0) return hipSuccess;
  hipLaunchKernelGGL(k_raw_merge_ts, dim3(wave_blocks(p.g1 - p.g0)), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_raw_dz_check(const RawParams& p, int64_t n_out, hipStream_t s) {
  if (n_out <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_raw_dz_check, dim3((unsigned)((n_out + 255) / 256)), dim3(256), 0, s, p, n_out);
  return hipGetLastError();
}

hipError_t launch_raw_cursor(const RawParams& p, int64_t s_begin, int64_t s_end, hipStream_t s) {
  if (s_end <= s_begin) return hipSuccess;
  hipLaunchKernelGGL(k_raw_cursor, dim3(wave_blocks(s_end - s_begin)), dim3(256), 0, s, p, s_begin, s_end);
  return hipGetLastError();
}

hipError_t launch_raw_eval(const RawParams& p, hipStream_t s) {
  if (p.n_strips == 0) return hipSuccess;
  switch (p.ga) {
    case GA_SUM: return launch_raw_eval_inst<GA_SUM>(p, s);
    case GA_AVG: return launch_raw_eval_inst<GA_AVG>(p, s);
    case GA_COUNT: return launch_raw_eval_inst<GA_COUNT>(p, s);
    case GA_SQUARESUM: return launch_raw_eval_inst<GA_SQUARESUM>(p, s);
    case GA_MIN: return launch_raw_eval_inst<GA_MIN>(p, s);
    case GA_MAX: return launch_raw_eval_inst<GA_MAX>(p, s);
    case GA_DEV: return launch_raw_eval_inst<GA_DEV>(p, s);
    case GA_FIRST: return launch_raw_eval_inst<GA_FIRST>(p, s);
    case GA_LAST: return launch_raw_eval_inst<GA_LAST>(p, s);
    case GA_DIFF: return launch_raw_eval_inst<GA_DIFF>(p, s);
    case GA_MULT: return launch_raw_eval_inst<GA_MULT>(p, s);
    case GA_NONE: return launch_raw_eval_inst<GA_NONE>(p, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace tsdb
