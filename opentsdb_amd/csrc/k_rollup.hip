// k_rollup.hip -- rollup generation: the per-series downsampled
// buckets of one function (dense [series][slot] outputs of the NONE-aggregator query,
// engine.cpp) -> rollup cells [agg id][BE16 offset|flags] + value bytes.
//
// k_rollup_agg reads every series once and reduces each bucket with the four rollup
// functions at the same time (Aggregators Sum :246-259, Count :636-645, Max :349-361,
// Min :315-327 as runDouble applies them to the Downsampler's bucket, src/core/Downsampler.java
// :223): one wave per series, its rows decoded in 512-datapoint chunks, the open bucket carried
// across chunks and rows.  A series whose datapoint count, largest magnitude and least
// significant bit certify that every partial sum is exact (kcommon.h fast_cert) reduces its
// buckets with a segmented wave scan; any other series reduces each bucket run sequentially in
// time order with one lane.  Both give Java's left-to-right sum bit for bit.  Output: the four functions' dense [series][slot] values and
// the bucket presence.
//
// Then, per function, two passes over the (series, slot) grid in batch series order:
// k_rollup_size writes a cell flag and the value length of every present bucket, two
// device-wide exclusive scans turn them into cell and byte offsets, k_rollup_write writes the
// cells.  The grid is 1 thread per (series, slot): a few bytes read and written per bucket.
#include <hipcub/hipcub.hpp>

#include "kcommon.h"
#include "rollup_codec.h"
#include "../../include/tsdbhip.h"

namespace tsdb {

struct RAcc {
  double sum, mn, mx;
  int n;   // non-NaN values
};

__device__ __forceinline__ void racc_init(RAcc& a) {
  a.sum = 0.0;
  a.mn = INFINITY;
  a.mx = -INFINITY;
  a.n = 0;
}

__device__ __forceinline__ void racc_add(RAcc& a, double x) {
  if (!isnan(x)) {
    a.sum += x;
    a.n++;
    if (x < a.mn) a.mn = x;
    if (x > a.mx) a.mx = x;
  }
}

// a then b (time order): the sum is exact in any association order under the series'
// certificate, count / min / max always are
__device__ __forceinline__ RAcc racc_op(const RAcc& a, const RAcc& b) {
  RAcc r;
  r.sum = a.sum + b.sum;
  r.mn = b.mn < a.mn ? b.mn : a.mn;
  r.mx = b.mx > a.mx ? b.mx : a.mx;
  r.n = a.n + b.n;
  return r;
}

__device__ __forceinline__ RAcc shfl_up_racc(const RAcc& a, int d) {
  RAcc r;
  r.sum = __shfl_up(a.sum, d, 64);
  r.mn = __shfl_up(a.mn, d, 64);
  r.mx = __shfl_up(a.mx, d, 64);
  r.n = __shfl_up(a.n, d, 64);
  return r;
}

__device__ __forceinline__ RAcc shfl_racc(const RAcc& a, int src) {
  RAcc r;
  r.sum = __shfl(a.sum, src, 64);
  r.mn = __shfl(a.mn, src, 64);
  r.mx = __shfl(a.mx, src, 64);
  r.n = __shfl(a.n, src, 64);
  return r;
}

// runDouble of each function over the bucket: sum / max / min NaN when no non-NaN value (and
// min +Inf / max -Inf -> NaN), count the non-NaN values
__device__ __forceinline__ void racc_emit(const RollupAggParams& p, int64_t s, int k, const RAcc& a) {
  const int64_t o = s * p.K + k;
  const double nan = (double)NAN;
  p.out[0 * p.stride + o] = a.n == 0 ? nan : a.sum;
  p.out[1 * p.stride + o] = (double)a.n;
  p.out[2 * p.stride + o] = a.mx == -INFINITY ? nan : a.mx;
  p.out[3 * p.stride + o] = a.mn == INFINITY ? nan : a.mn;
  p.pres[o] = 1;
}

// Certified series: a segmented wave reduction of the chunk's bucket runs (keys = slots,
// non-decreasing in time order).  Each lane folds its DPL values into its first and last run
// (runs wholly inside the lane are emitted directly), the last runs are combined across lanes
// by a segmented inclusive scan, and the chunk's last run stays open in the carry.
__device__ __forceinline__ void rfast_chunk(const RollupAggParams& rp, int64_t s, int& carry_slot, RAcc& carry,
                                            const int slot[DPL], const double val[DPL]) {
  const int lane = lane_id();
  int kf = -1, cur_key = -1, nruns = 0;
  RAcc Pf, cur;
  racc_init(Pf);
  racc_init(cur);
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    if (slot[j] < 0) continue;
    if (slot[j] != cur_key) {
      if (cur_key >= 0) {
        if (nruns == 1) { Pf = cur; kf = cur_key; }
        else racc_emit(rp, s, cur_key, cur);
      }
      cur_key = slot[j];
      racc_init(cur);
      nruns++;
    }
    racc_add(cur, val[j]);
  }
  RAcc Pl = cur;
  const int kl = cur_key;
  if (nruns == 1) { kf = kl; Pf = Pl; }
  const bool has = nruns > 0;
  const bool multi = nruns >= 2;
  const unsigned long long hm = __ballot(has);
  if (hm == 0) return;
  const int fv = __ffsll((long long)hm) - 1;
  const int lv = 63 - __clzll((long long)hm);
  const int kf_fv = __shfl(kf, fv, 64);
  if (carry_slot >= 0) {
    if (kf_fv == carry_slot) {
      if (lane == fv) {
        Pf = racc_op(carry, Pf);
        if (!multi) Pl = Pf;
      }
    } else if (lane == 0) {
      racc_emit(rp, s, carry_slot, carry);
    }
  }
  const int kl_prev = __shfl_up(kl, 1, 64);
  int h = (!has || multi || lane == 0 || kl_prev != kf) ? 1 : 0;
  RAcc T;
  if (has) T = Pl;
  else racc_init(T);
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const RAcc To = shfl_up_racc(T, d);
    const int ho = __shfl_up(h, d, 64);
    if (lane >= d) {
      if (!h) T = racc_op(To, T);
      h |= ho;
    }
  }
  const RAcc Tprev = shfl_up_racc(T, 1);
  const int kf_next = __shfl_down(kf, 1, 64);
  if (has && multi) racc_emit(rp, s, kf, (lane > 0 && kl_prev == kf && lane > fv) ? racc_op(Tprev, Pf) : Pf);
  if (has && lane != lv && kf_next != kl) racc_emit(rp, s, kl, T);
  carry_slot = __shfl(kl, lv, 64);
  carry = shfl_racc(T, lv);
}

// Uncertified series: every bucket run of the chunk reduced sequentially in time order by one
// lane (the sum is bit-exact whatever the values), the last run carried.
__device__ __forceinline__ void rslow_chunk(const RollupAggParams& rp, const WaveLds& W, int64_t s, int& carry_slot,
                                            RAcc& carry, const int slot[DPL], const double val[DPL]) {
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
  if (nseg > 0) {
    if (carry_slot >= 0 && W.seg_slot[0] != carry_slot) {
      if (lane == 0) racc_emit(rp, s, carry_slot, carry);
      carry_slot = -1;
      racc_init(carry);
    }
    for (int b0 = 0; b0 < nseg; b0 += 64) {
      const int si = b0 + lane;
      RAcc a;
      racc_init(a);
      int myslot = -1;
      if (si < nseg) {
        myslot = W.seg_slot[si];
        if (si == 0 && myslot == carry_slot) a = carry;
        const int e = W.seg_start[si + 1];
        for (int i = W.seg_start[si]; i < e; i++) racc_add(a, W.dpv[i]);
        if (si != nseg - 1) racc_emit(rp, s, myslot, a);
      }
      if (b0 + 64 >= nseg) {   // the chunk's last run stays open
        const int src = (nseg - 1) & 63;
        carry = shfl_racc(a, src);
        carry_slot = __shfl(myslot, src, 64);
      }
    }
  }
  WAVE_SYNC();
}

__device__ __forceinline__ void rollup_series(const GridParams& p, const RollupAggParams& rp, const WaveLds& W,
                                              int64_t s) {
  const int lane = lane_id();
  const int K = (int)p.K;
  for (int k = lane; k < K; k += 64) rp.pres[s * K + k] = 0;
  const int64_t r0 = p.series_row_ptr[s], r1 = p.series_row_ptr[s + 1];
  int64_t ra = r0;
  while (ra < r1 && (int64_t)p.rows[ra].base < p.ss) ra++;
  int64_t rb = ra;
  // exactness certificate of the order-free sum (kcommon.h fast_cert): the series' datapoint
  // count bounds every bucket's
  uint32_t nb = 0;
  int lsb = INT32_MAX;
  double amax = 0.0;
  while (rb < r1 && (int64_t)p.rows[rb].base < p.se) {
    nb += p.rows[rb].ndp;
    lsb = min(lsb, p.rows[rb].lsb);
    amax = fmax(amax, p.rows[rb].absmax);
    rb++;
  }
  const bool fast = fast_cert<F_SUM>(nb, lsb, amax);
  int carry_slot = -1;
  RAcc carry;
  racc_init(carry);
  StreamOrd so{-1};   // stored order (kcommon.h so_apply)
  Raw rc = {}, rn = {};
  RowDesc d = {};
  if (ra < rb) {
    d = p.rows[ra];
    if (row_uniform(d)) load_raw(p, d, 0, rc);
  }
  for (int64_t r = ra; r < rb; r++) {
    const bool has_next = r + 1 < rb;
    RowDesc nd = {};
    if (has_next) nd = p.rows[r + 1];
    if (d.flags & ROW_ERR) {
      if (lane == 0) set_err(p.err, TSDB_E_ILLEGAL_DATA);
      if (has_next && row_uniform(nd)) load_raw(p, nd, 0, rc);
      d = nd;
      continue;
    }
    const RowGeom g = row_geom(p, d.base);
    const bool uni = row_uniform(d);
    const bool skip = so_row_skip(p, so, d, !has_next);
    int64_t vcur = 0;
    for (int64_t c0 = 0; c0 < (int64_t)d.ndp; c0 += CH) {
      if (c0 + CH < (int64_t)d.ndp) {
        if (uni) load_raw(p, d, c0 + CH, rn);
      } else if (has_next && row_uniform(nd)) {
        load_raw(p, nd, 0, rn);
      }
      int slot[DPL];
      double val[DPL];
      if (uni) decode_raw<true>(p, d, g, c0, rc, slot, val);
      else decode_generic<true>(p, d, g, c0, W, vcur, slot, val);
      so_apply(p, so, slot, skip);
      rc = rn;
      if (fast) rfast_chunk(rp, s, carry_slot, carry, slot, val);
      else rslow_chunk(rp, W, s, carry_slot, carry, slot, val);
    }
    d = nd;
  }
  if (carry_slot >= 0 && lane == 0) racc_emit(rp, s, carry_slot, carry);
  WAVE_SYNC();
}

// One wave per series; over a list (the series k_rollup_fast handed back) the n_launch waves
// stride through it.
__global__ __launch_bounds__(256) void k_rollup_agg(GridParams p, RollupAggParams rp) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  unsigned char* base = smem + (int64_t)wave * fixed_lds_bytes();
  WaveLds W;
  W.dpv = (double*)base;
  W.vbuf = base;
  W.mq = (uint32_t*)base;
  W.mv = (uint32_t*)(base + CH * 4);
  W.seg_slot = (int32_t*)(base + VBUF);
  W.seg_start = (uint16_t*)(base + VBUF + CH * 4);
  const int64_t gw = (int64_t)blockIdx.x * 4 + wave;
  if (p.tile_list) {
    const int64_t n = *p.tile_list_n;
    for (int64_t i = gw; i < n; i += (int64_t)gridDim.x * 4) rollup_series(p, rp, W, p.tile_list[i]);
    return;
  }
  if (gw < p.n_series) rollup_series(p, rp, W, gw);
}

hipError_t launch_rollup_agg(const GridParams& p, const RollupAggParams& rp, hipStream_t s) {
  const int64_t n = p.n_launch > 0 ? p.n_launch : p.n_series;
  if (n <= 0) return hipSuccess;
  const size_t lds = 4 * (size_t)fixed_lds_bytes();
  hipLaunchKernelGGL(k_rollup_agg, dim3((unsigned)((n + 3) / 4)), dim3(256), lds, s, p, rp);
  return hipGetLastError();
}

// ---- k_rollup_fast: the streaming variant -------------------------------------------------
// For a series whose rows are all of one uniform class (k_fast's premises: sorted, NaN-free,
// no negative zero) and whose buckets pass the exactness certificate, each bucket's sum, count,
// min and max do not depend on the order the values are combined in.  One wave per series:
// the row walker and D-deep chunk ring of k_fast (kcommon.h fast_issue).  A chunk inside one
// bucket folds into lane-resident accumulators (RfAcc); a chunk over several buckets reduces
// each lane's 8 datapoints into at most two runs folded into per-slot LDS accumulators with LDS
// atomics.  The series end writes the four dense outputs.  A series
// that breaks a premise is appended to the redo list for k_rollup_agg.
struct RfLds {
  double* sum;
  double* mn;
  double* mx;
  uint32_t* cnt;
};

__host__ __device__ inline int64_t rollup_fast_wave_lds(int64_t K) { return align16(K * 8) * 3 + align16(K * 4); }

__device__ __forceinline__ void rf_fold(const RfLds& L, int k, double s, double mn, double mx, uint32_t n) {
  __hip_atomic_fetch_add(&L.sum[k], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  __hip_atomic_fetch_min(&L.mn[k], mn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  __hip_atomic_fetch_max(&L.mx[k], mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  __hip_atomic_fetch_add(&L.cnt[k], n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

// DPP move of a double (both halves; lanes without a source keep `old`)
template <int C, int RM>
__device__ __forceinline__ double dpp_f64(double old, double x) {
  const long long o = __double_as_longlong(old), v = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp((int)o, (int)v, C, RM, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(v >> 32), C, RM, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(uint32_t)lo);
}

template <int C, int RM>
__device__ __forceinline__ void racc_dpp_step(RAcc& a) {
  a.sum += dpp_f64<C, RM>(0.0, a.sum);
  a.mn = fmin(a.mn, dpp_f64<C, RM>(INFINITY, a.mn));
  a.mx = fmax(a.mx, dpp_f64<C, RM>(-INFINITY, a.mx));
  a.n += __builtin_amdgcn_update_dpp(0, a.n, C, RM, 0xF, false);
}

// inclusive DPP scan (row_shr 1/2/4/8, row_bcast 15/31): lane 63 ends with the wave total.
// The sum's association order differs from time order -- exact under the certificate.
__device__ __forceinline__ void wave_total_racc(RAcc& a) {
  racc_dpp_step<0x111, 0xF>(a);
  racc_dpp_step<0x112, 0xF>(a);
  racc_dpp_step<0x114, 0xF>(a);
  racc_dpp_step<0x118, 0xF>(a);
  racc_dpp_step<0x142, 0xA>(a);
  racc_dpp_step<0x143, 0xC>(a);
}

// Lane-resident accumulator of the wave's open bucket in the class's native value type
// (float32 / float64 / vle integer): min and max exact in that type, the sum in double (in
// int64 for integers) -- a chunk inside one bucket costs a few VALU ops per datapoint and no
// cross-lane traffic; the accumulator is reduced across the wave (DPP) only when the bucket
// changes.
template <int VL>
struct RfAcc {
  using V = typename std::conditional<VL == 4, float, typename std::conditional<VL == 8, double, int>::type>::type;
  using S = typename std::conditional<VL == 0, long long, double>::type;
  V mn, mx;
  S s;
  int n;      // wave-uniform: datapoints accumulated
  int slot;   // wave-uniform: the bucket being accumulated (-1: none)
};

// DPP move of a 32- or 64-bit value (lanes without a source keep `old`)
template <int C, int RM, class T>
__device__ __forceinline__ T dpp_mov(T old, T x) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, x),
                                                             C, RM, 0xF, false));
  } else {
    const long long o = __builtin_bit_cast(long long, old), v = __builtin_bit_cast(long long, x);
    const int lo = __builtin_amdgcn_update_dpp((int)o, (int)v, C, RM, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(v >> 32), C, RM, 0xF, false);
    return __builtin_bit_cast(T, ((long long)hi << 32) | (long long)(uint32_t)lo);
  }
}

template <int VL>
__device__ __forceinline__ typename RfAcc<VL>::V rf_vmax() {
  if constexpr (VL == 4) return INFINITY;
  else if constexpr (VL == 8) return (double)INFINITY;
  else return INT32_MAX;
}

template <int VL>
__device__ __forceinline__ void rf_reset(RfAcc<VL>& a) {
  a.mn = rf_vmax<VL>();
  a.mx = -rf_vmax<VL>();
  a.s = 0;
  a.n = 0;
}

template <int QW, int VL>
__device__ __forceinline__ typename RfAcc<VL>::V rf_value(const FRaw<QW, VL>& b, int j) {
  if constexpr (VL == 0) {
    return f_int16<QW, VL>(b, j);
  } else if constexpr (VL == 4) {
    const uint4 u = b.v[j >> 2];
    const uint32_t wd = (j & 3) == 0 ? u.x : (j & 3) == 1 ? u.y : (j & 3) == 2 ? u.z : u.w;
    return __uint_as_float(__builtin_bswap32(wd));
  } else {
    return f_value<QW, VL>(b, j);
  }
}

template <int VL, int C, int RM>
__device__ __forceinline__ void rf_dpp_step(RfAcc<VL>& a) {
  using V = typename RfAcc<VL>::V;
  using S = typename RfAcc<VL>::S;
  a.s += dpp_mov<C, RM, S>((S)0, a.s);
  a.mn = min(a.mn, dpp_mov<C, RM, V>(rf_vmax<VL>(), a.mn));
  a.mx = max(a.mx, dpp_mov<C, RM, V>(-rf_vmax<VL>(), a.mx));
}

// the open bucket's lane accumulators -> one fold into the slot (lane 63 holds the wave total
// after the inclusive DPP scan: row_shr 1/2/4/8, row_bcast 15/31)
template <int VL>
__device__ __forceinline__ void rf_flush(const RfLds& L, RfAcc<VL>& a) {
  if (a.slot < 0) return;
  if (a.n) {
    rf_dpp_step<VL, 0x111, 0xF>(a);
    rf_dpp_step<VL, 0x112, 0xF>(a);
    rf_dpp_step<VL, 0x114, 0xF>(a);
    rf_dpp_step<VL, 0x118, 0xF>(a);
    rf_dpp_step<VL, 0x142, 0xA>(a);
    rf_dpp_step<VL, 0x143, 0xC>(a);
    if (lane_id() == 63) rf_fold(L, a.slot, (double)a.s, (double)a.mn, (double)a.mx, (uint32_t)a.n);
  }
  rf_reset<VL>(a);
  a.slot = -1;
}

template <int VL, bool FULL>
__device__ __forceinline__ void rf_accum(RfAcc<VL>& A, const typename RfAcc<VL>::V xv[DPL], int nvl) {
  typename RfAcc<VL>::S ps = 0;
  if constexpr (VL == 0) {
    int pi = 0;   // 8 values of |x| < 2^15
#pragma unroll
    for (int j = 0; j < DPL; j++) pi += (FULL || j < nvl) ? xv[j] : 0;
    ps = pi;
  } else {
#pragma unroll
    for (int j = 0; j < DPL; j++) ps += (FULL || j < nvl) ? (double)xv[j] : 0.0;
  }
  A.s += ps;
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    const bool valid = FULL || j < nvl;
    A.mn = min(A.mn, valid ? xv[j] : rf_vmax<VL>());
    A.mx = max(A.mx, valid ? xv[j] : -rf_vmax<VL>());
  }
}

template <int QW, int VL, bool FULL>
__device__ __forceinline__ void rf_chunk(const GridParams& p, const RfLds& L, RfAcc<VL>& A, const FRaw<QW, VL>& b,
                                         const FGeom& m, int nv0, int K) {
  using V = typename RfAcc<VL>::V;
  const int lane = lane_id();
  const int nvl = FULL ? DPL : max(0, min(DPL, nv0 - lane * DPL));
  const int uq = (QW == 2 && !p.unit_s) ? 1000 : 1;
  uint32_t fld[DPL];
  V xv[DPL];
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    fld[j] = f_field<QW, VL>(b, j);
    xv[j] = rf_value<QW, VL>(b, j);
  }
  uint32_t flast = fld[DPL - 1];
  if (!FULL) {
#pragma unroll
    for (int j = 0; j < DPL - 1; j++) if (j == nvl - 1) flast = fld[j];
  }
  // the chunk's first and last datapoints (lane 0 and the last lane with datapoints: lanes hold
  // the chunk in time order) decide whether it lies inside one bucket of the slot range
  {
    const int w0 = m.r0 + (int)__builtin_amdgcn_readfirstlane(fld[0]) * uq;
    const int w1 = m.r0 + (int)__builtin_amdgcn_readlane(flast, min(63, (nv0 - 1) >> 3)) * uq;
    if (w0 >= 0) {
      const int s0 = f_slot(p, m, w0), s1 = f_slot(p, m, w1);
      if (s0 == s1 && s1 < K) {
        if (s0 != A.slot) {
          rf_flush<VL>(L, A);
          A.slot = s0;
        }
        A.n += nv0;
        // a chunk whose lanes are all full or empty (rows of a multiple of 8 datapoints, e.g.
        // 360) takes the unmasked loop on its full lanes
        const bool whole = FULL || __all(nvl == 0 || nvl == DPL);
        if (whole) {
          if (nvl) rf_accum<VL, true>(A, xv, DPL);
        } else {
          rf_accum<VL, false>(A, xv, nvl);
        }
        return;
      }
    }
  }
  // several buckets: per-lane runs folded into the slot accumulators with LDS atomics
  double xs[DPL];
#pragma unroll
  for (int j = 0; j < DPL; j++) xs[j] = (double)xv[j];
  const int n0 = m.r0 + (int)fld[0] * uq;
  const int nl = m.r0 + (int)flast * uq;
  const int sfirst = n0 >= 0 ? f_slot(p, m, n0) : -1;
  const int slast = nl >= 0 ? f_slot(p, m, nl) : -1;
  const bool simple = nvl == 0 || (n0 >= 0 && slast < K && slast <= sfirst + 1);
  if (__builtin_expect(__all(simple), 1)) {
    if (nvl == 0) return;
    const int Dn = (sfirst - m.q0 + 1) * p.In - m.r0;   // offsets below the next bucket boundary
    const uint32_t Tf = uq == 1 ? (uint32_t)Dn : (uint32_t)((Dn + 999) / 1000);
    double sF = 0.0, sL = 0.0, mnF = INFINITY, mxF = -INFINITY, mnL = INFINITY, mxL = -INFINITY;
    int cF = 0;
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      const bool valid = FULL || j < nvl;
      const bool inF = valid && fld[j] < Tf;
      const bool inL = valid && !inF;
      const double x = xs[j];
      sF += inF ? x : 0.0;
      mnF = (inF && x < mnF) ? x : mnF;
      mxF = (inF && x > mxF) ? x : mxF;
      cF += inF;
      sL += inL ? x : 0.0;
      mnL = (inL && x < mnL) ? x : mnL;
      mxL = (inL && x > mxL) ? x : mxL;
    }
    const int nL = nvl - cF;
    if (cF) rf_fold(L, sfirst, sF, mnF, mxF, (uint32_t)cF);
    if (nL) rf_fold(L, sfirst + 1, sL, mnL, mxL, (uint32_t)nL);
  } else {
    // some lane spans more than two buckets or the edge of the slot range: per datapoint
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      if (j < nvl) {
        const int n = m.r0 + (int)fld[j] * uq;
        if (n >= 0) {
          const int sl = f_slot(p, m, n);
          if (sl < K) rf_fold(L, sl, xs[j], xs[j], xs[j], 1u);
        }
      }
    }
  }
}

// Series end: the open bucket folded, the certificate checked, the dense outputs written (a
// failing series goes to the redo list).
template <int VL>
__device__ __forceinline__ void rf_series_end(const GridParams& p, const RollupAggParams& rp, const RfLds& L,
                                              RfAcc<VL>& A, int K, int64_t s, int lsb, double amax) {
  const int lane = lane_id();
  rf_flush<VL>(L, A);
  WAVE_SYNC();
  uint32_t nmax = 0;
  for (int k = lane; k < K; k += 64) nmax = max(nmax, L.cnt[k]);
  nmax = (uint32_t)wave_max((int)nmax);
  if (!fast_cert<F_SUM>(nmax, lsb, amax)) {
    if (lane == 0) p.redo_list[atomicAdd(p.redo_n, 1)] = (int32_t)s;
  } else {
    const double nan = (double)NAN;
    for (int k = lane; k < K; k += 64) {
      const uint32_t c = L.cnt[k];
      const int64_t o = s * K + k;
      rp.out[0 * rp.stride + o] = c ? L.sum[k] : nan;
      rp.out[1 * rp.stride + o] = (double)c;
      rp.out[2 * rp.stride + o] = c ? L.mx[k] : nan;
      rp.out[3 * rp.stride + o] = c ? L.mn[k] : nan;
      rp.pres[o] = c != 0;
    }
  }
}

// One wave per series (a tile of several series, the chunk ring running across them, measured
// slower on config 5: the series-end code inside the unrolled ring costs registers and
// occupancy, and its stores count against the ring's vmcnt waits).
template <int QW, int VL, int D>
__global__ __launch_bounds__(256) void k_rollup_fast(GridParams p, RollupAggParams rp) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int64_t s = (int64_t)blockIdx.x * p.waves + wave;
  if (p.tile_list) {
    if (s >= (int64_t)*p.tile_list_n) return;
    s = p.tile_list[s];
  }
  if (s >= p.n_series) return;
  const int K = (int)p.K;
  RfLds L;
  {
    unsigned char* base = smem + (int64_t)wave * p.wave_lds;
    L.sum = (double*)base;
    L.mn = (double*)(base + align16(K * 8));
    L.mx = (double*)(base + 2 * align16(K * 8));
    L.cnt = (uint32_t*)(base + 3 * align16(K * 8));
  }
  for (int k = lane; k < K; k += 64) {
    L.sum[k] = 0.0;
    L.mn[k] = INFINITY;
    L.mx[k] = -INFINITY;
    L.cnt[k] = 0;
  }
  const RowDesc* __restrict__ rows = p.rows;
  FWalk w;
  w.r0 = p.series_row_ptr[s];
  w.r = 0;
  w.rend = (int32_t)(p.series_row_ptr[s + 1] - w.r0);
  w.c0 = 0;
  w.sf = 0;
  if (w.rend > 0) w.d = fdesc(rows, w.r0);
  if (w.rend > 1) w.nd = fdesc(rows, w.r0 + 1);
  WAVE_SYNC();
  FRaw<QW, VL> buf[D];
  FMeta meta[D];
  bool redo = false;
#pragma unroll
  for (int i = 0; i < D; i++)
    if (fast_issue<F_MIN, QW, VL>(p, rows, w, buf[i], meta[i]) == 2) redo = true;
  int lsb = INT32_MAX;
  double amax = 0.0;
  FGeom g = {0, 0};
  RfAcc<VL> A;
  rf_reset<VL>(A);
  A.slot = -1;
  bool done = redo;
  while (!done) {
#pragma unroll
    for (int i = 0; i < D; i++) {
      if (!done) {
        const uint32_t mb = meta[i].bits;
        if (!(mb & FM_OK)) {
          done = true;
        } else {
          if (mb & FM_NEWROW) {
            const RowDesc& x = rows[w.r0 + meta[i].rrel];
            lsb = min(lsb, x.lsb);
            amax = fmax(amax, x.absmax);
            g = fgeom(p, x.base);
          }
          const int nv0 = (int)(mb & FM_NV);
          if (nv0 >= CH) rf_chunk<QW, VL, true>(p, L, A, buf[i], g, nv0, K);
          else rf_chunk<QW, VL, false>(p, L, A, buf[i], g, nv0, K);
          if (fast_issue<F_MIN, QW, VL>(p, rows, w, buf[i], meta[i]) == 2) { redo = true; done = true; }
        }
      }
    }
  }
  if (redo) {
    if (lane == 0) p.redo_list[atomicAdd(p.redo_n, 1)] = (int32_t)s;
    return;
  }
  rf_series_end<VL>(p, rp, L, A, K, s, lsb, amax);
}

template <int QW, int VL>
static hipError_t launch_rollup_fast_t(const GridParams& p, const RollupAggParams& rp, hipStream_t s) {
  constexpr int D = (QW * 2 + VL * 2 <= 16) ? 3 : 2;
  const int64_t n = p.tile_list ? p.n_launch : p.n_series;
  if (n <= 0) return hipSuccess;
  const int64_t blocks = (n + p.waves - 1) / p.waves;
  const size_t lds = (size_t)p.wave_lds * p.waves;
  hipLaunchKernelGGL((k_rollup_fast<QW, VL, D>), dim3((unsigned)blocks), dim3(64 * p.waves), lds, s, p, rp);
  return hipGetLastError();
}

bool rollup_fast_supported(int qw, int vl) { return ((qw == 2 || qw == 4) && (vl == 4 || vl == 8)) || (qw == 2 && vl == 0); }

int64_t rollup_fast_lds(int64_t K) { return rollup_fast_wave_lds(K); }

hipError_t launch_rollup_fast(const GridParams& p, const RollupAggParams& rp, int qw, int vl, hipStream_t s) {
  if (qw == 2 && vl == 4) return launch_rollup_fast_t<2, 4>(p, rp, s);
  if (qw == 2 && vl == 8) return launch_rollup_fast_t<2, 8>(p, rp, s);
  if (qw == 4 && vl == 4) return launch_rollup_fast_t<4, 4>(p, rp, s);
  if (qw == 4 && vl == 8) return launch_rollup_fast_t<4, 8>(p, rp, s);
  if (qw == 2 && vl == 0) return launch_rollup_fast_t<2, 0>(p, rp, s);
  return hipErrorNotSupported;
}

__global__ void k_series_allint(const RowDesc* __restrict__ rows, const int64_t* __restrict__ srp, int64_t n,
                                uint8_t* __restrict__ allint) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  uint8_t a = 1;
  for (int64_t r = srp[g]; r < srp[g + 1]; r++)
    if (!(rows[r].flags & ROW_ALLI)) a = 0;
  allint[g] = a;
}

__device__ __forceinline__ bool rollup_cell(const RollupParams& p, int64_t idx, int64_t& g, int64_t& ts,
                                            double& v) {
  const int64_t i = idx / p.K;
  const int64_t k = idx - i * p.K;
  g = p.ord[i];
  if (!p.flag[g * p.K + k]) return false;
  ts = p.B0 + k * p.I;
  if (ts < p.start_ms || ts >= p.end_ms) return false;
  v = p.val[g * p.K + k];
  return true;
}

__global__ void k_rollup_size(RollupParams p) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= p.n) return;
  int64_t g, ts;
  double v;
  uint32_t c = 0, len = 0;
  if (rollup_cell(p, idx, g, ts, v)) {
    int16_t flags;
    uint64_t be;
    const int l = rc_value(v, p.as_long_all || p.allint[g], flags, be);
    int32_t base;
    uint8_t q[3];
    if (l == 0 || !rc_basetime(ts / 1000, p.iv, base) || !rc_qualifier(ts / 1000, base, flags, p.agg_id, p.iv, q)) {
      atomicCAS(p.err, 0, (int32_t)TSDB_E_ILLEGAL_ARGUMENT);
    } else {
      c = 1;
      len = (uint32_t)l;
    }
  }
  p.cnt[idx] = c;
  p.vsz[idx] = len;
}

__global__ void k_rollup_write(RollupParams p) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= p.n) return;
  if (!p.cnt[idx]) return;
  int64_t g, ts;
  double v;
  rollup_cell(p, idx, g, ts, v);
  int16_t flags;
  uint64_t be;
  const int len = rc_value(v, p.as_long_all || p.allint[g], flags, be);
  int32_t base;
  uint8_t q[3];
  rc_basetime(ts / 1000, p.iv, base);
  rc_qualifier(ts / 1000, base, flags, p.agg_id, p.iv, q);
  const int64_t c = p.coff[idx];
  const uint64_t vo = p.voff[idx];
  p.o_series[c] = p.orig[g];
  p.o_base[c] = (uint32_t)base;
  p.o_qual[3 * c] = q[0];
  p.o_qual[3 * c + 1] = q[1];
  p.o_qual[3 * c + 2] = q[2];
  p.o_voff[c] = vo;
  for (int b = 0; b < len; b++) p.o_val[vo + b] = (uint8_t)(be >> (8 * (len - 1 - b)));
}

hipError_t launch_series_allint(const RowDesc* rows, const int64_t* srp, int64_t n, uint8_t* allint, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_series_allint, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, rows, srp, n, allint);
  return hipGetLastError();
}

hipError_t launch_rollup_size(const RollupParams& p, hipStream_t s) {
  if (p.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_rollup_size, dim3((unsigned)((p.n + 255) / 256)), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_rollup_write(const RollupParams& p, hipStream_t s) {
  if (p.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_rollup_write, dim3((unsigned)((p.n + 255) / 256)), dim3(256), 0, s, p);
  return hipGetLastError();
}

template <class T>
struct Widen {
  __host__ __device__ T operator()(uint32_t x) const { return (T)x; }
};

// exclusive prefix sums: uint32 -> int64 / uint64, accumulated in 64 bits (temp storage
// grown on demand)
hipError_t rollup_scan(const uint32_t* cnt_, int64_t* coff, const uint32_t* vsz_, uint64_t* voff, int64_t n,
                       void** tmp, size_t* tmp_bytes, hipStream_t s) {
  hipcub::TransformInputIterator<int64_t, Widen<int64_t>, const uint32_t*> cnt(cnt_, Widen<int64_t>());
  hipcub::TransformInputIterator<uint64_t, Widen<uint64_t>, const uint32_t*> vsz(vsz_, Widen<uint64_t>());
  size_t need1 = 0, need2 = 0;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, need1, cnt, coff, (int)n, s);
  if (e != hipSuccess) return e;
  e = hipcub::DeviceScan::ExclusiveSum(nullptr, need2, vsz, voff, (int)n, s);
  if (e != hipSuccess) return e;
  const size_t need = need1 > need2 ? need1 : need2;
  if (need > *tmp_bytes) {
    if (*tmp) (void)hipFree(*tmp);
    *tmp = nullptr;
    e = hipMalloc(tmp, need);
    if (e != hipSuccess) { *tmp_bytes = 0; return e; }
    *tmp_bytes = need;
  }
  size_t t = *tmp_bytes;
  e = hipcub::DeviceScan::ExclusiveSum(*tmp, t, cnt, coff, (int)n, s);
  if (e != hipSuccess) return e;
  t = *tmp_bytes;
  return hipcub::DeviceScan::ExclusiveSum(*tmp, t, vsz, voff, (int)n, s);
}

}  // namespace tsdb
