// k_index.hip -- the load-time row index of libtsdbhip.
//
// RowSeq's per-datapoint view (src/core/RowSeq.java:233-266, 552-614; Internal.java:621-810)
// reduced to the row facts the query kernels branch on: qualifier width, uniform value
// length, all-float / all-integer, NaN / -0.0, offset order, malformed cells, and the
// exactness certificate (least significant set bit, max |value|).  Written once per load into
// RowDesc; 2-byte-qualifier rows also get their 1-2-byte integers as little-endian int16 at
// val2 + qoff + 2 i (the same offsets as the qualifiers), the layout k_short / k_fast read for
// vle rows.
//
//  * k_index_hint     one thread per row: the row's class -- qualifier width (first byte) x
//                     value length (L when the value bytes are exactly ndp x L (+ meta byte),
//                     else variable) -- and per-class row counts.
//  * k_index_scatter  per-class row lists.
//  * k_index_cls<QW,L>  one wave per row of its class (grid-stride over the list), 8 datapoints
//                     per lane per 512-datapoint chunk.  Every lane issues the same loads for
//                     every chunk (lanes past the row re-read its start), so the next chunk --
//                     or the next row's first chunk -- is prefetched while this one decodes and
//                     the wait before use covers only the older loads.  Uniform classes read
//                     values at i x L; the variable class stages value bytes in LDS after a
//                     wave prefix sum of the lengths (its first 1 KB prefetched).  Statistics
//                     are kept in the integer domain (bit patterns, magnitudes).
//  * k_index_short    rows of 2-byte qualifiers that fit one chunk (<= 512 datapoints) with
//                     4-byte values or 1-2-byte integers (config 3's hour rows of 10 s points),
//                     hinted by k_index_hint: no row lists, a 64-row descriptor batch per wave
//                     (lane l loads row l's descriptor, the row loop reads them with readlane),
//                     the next row's loads in flight while one decodes, each row's results kept
//                     in its own lane and stored with the batch.
//  * k_index_generic  rows no class kernel takes (mixed second / millisecond qualifiers, odd or
//                     empty qualifier arrays, a class hypothesis that failed): sequential.
#include "kcommon.h"

namespace tsdb {

static constexpr int IDX_STAGE = 4224;   // bytes of value staging per wave: 512 x 8 B + alignment
static constexpr int IDX_NCLS = 11;      // 0 generic, 1 + qwi * 5 + li (qwi: 2 / 4 bytes; li: var, 1, 2, 4, 8)
static constexpr uint8_t HINT_SHORT = 0x80;   // hint bit: the row is k_index_short's (low bits: its class)
// IndexBufs.cnt slots past the classes: k_index_short's rows (4-byte values / 1-2-byte integers)
// and the rows it handed back to k_index_generic
static constexpr int IDX_C_SHORT4 = 12, IDX_C_SHORTV = 13, IDX_C_FAIL = 14;
#ifndef IDX_SHORT_D
#define IDX_SHORT_D 2   // k_index_short's load ring depth
#endif
#ifndef IDX_SHORT_BLOCKS
#define IDX_SHORT_BLOCKS 16384   // k_index_short's grid cap (4 waves a block, 64-row batches grid-strided)
#endif

struct IdxAcc {
  bool bad, allf, alli, vmax2, nan, negz, unsorted;
  int lsb, lmin, lmax;
  double amax;
};

__device__ __forceinline__ void idx_acc_init(IdxAcc& a) {
  a.bad = false; a.allf = a.alli = a.vmax2 = true; a.nan = a.negz = a.unsorted = false;
  a.lsb = INT32_MAX; a.lmin = 99; a.lmax = -1; a.amax = 0.0;
}

// 8 bytes of the LDS stage from byte offset b (little-endian memory order)
__device__ __forceinline__ uint64_t stage_u64(const uint32_t* s, int b) {
  const int w = b >> 2, sh = (b & 3) * 8;
  const uint32_t w0 = s[w], w1 = s[w + 1], w2 = s[w + 2];
  const uint32_t lo = sh ? (w0 >> sh) | (w1 << (32 - sh)) : w0;
  const uint32_t hi = sh ? (w1 >> sh) | (w2 << (32 - sh)) : w1;
  return ((uint64_t)hi << 32) | lo;
}

__device__ __noinline__ void index_row_generic(const uint8_t* __restrict__ qual, const uint8_t* __restrict__ val,
                                  uint8_t* __restrict__ val2, RowDesc* __restrict__ rows, int64_t r, int32_t* err) {
  const int lane = lane_id();
  {
    RowDesc d = rows[r];
    const uint8_t* q = qual + d.qoff;
    const uint8_t* v = val + d.voff;
    const uint32_t qlen = d.qlen;
    // hypotheses: all 2-byte, all 4-byte
    bool ok2 = (qlen % 2) == 0 && qlen > 0;
    bool ok4 = (qlen % 4) == 0 && qlen > 0;
    int lmin2 = 99, lmax2 = -1, lmin4 = 99, lmax4 = -1;
    for (uint32_t p0 = (uint32_t)lane * 16; p0 < qlen; p0 += 64 * 16) {
      const uint4 w = *reinterpret_cast<const uint4*>(q + p0);
      const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int b = 0; b < 16; b += 2) {
        if (p0 + b >= qlen) break;
        const uint32_t b0 = (ws[b >> 2] >> ((b & 3) * 8)) & 0xFF;
        const uint32_t b1 = (ws[(b + 1) >> 2] >> (((b + 1) & 3) * 8)) & 0xFF;
        if ((b0 & 0xF0) == 0xF0) ok2 = false;
        const int len = (b1 & 7) + 1;
        lmin2 = min(lmin2, len);
        lmax2 = max(lmax2, len);
        if ((b & 3) == 0) {
          if ((b0 & 0xF0) != 0xF0) ok4 = false;
          const uint32_t b3 = (ws[(b + 3) >> 2] >> (((b + 3) & 3) * 8)) & 0xFF;
          const int l4 = (b3 & 7) + 1;
          lmin4 = min(lmin4, l4);
          lmax4 = max(lmax4, l4);
        }
      }
    }
    ok2 = __all(ok2);
    ok4 = __all(ok4);
    lmin2 = wave_min(lmin2); lmax2 = wave_max(lmax2);
    lmin4 = wave_min(lmin4); lmax4 = wave_max(lmax4);
    uint32_t flags = 0, ndp = 0;
    if (ok2) {
      ndp = qlen / 2; flags = 2;
      if (lmin2 == lmax2) flags |= (uint32_t)lmin2 << ROW_VL_SHIFT;
    } else if (ok4) {
      ndp = qlen / 4; flags = 4;
      if (lmin4 == lmax4) flags |= (uint32_t)lmin4 << ROW_VL_SHIFT;
    } else {
      // mixed second/millisecond qualifiers (meta bit MS_MIXED_COMPACT): count sequentially
      if (lane == 0) {
        uint32_t i = 0;
        while (i < qlen) {
          const uint32_t w = ((q[i] & 0xF0) == 0xF0) ? 4 : 2;
          if (i + w > qlen) break;
          ndp++;
          i += w;
        }
      }
      ndp = __shfl(ndp, 0, 64);
    }
    // walk every datapoint: validate qualifier/value lengths, certificate stats
    bool bad = qlen == 0;
    bool allf = true, alli = true, vmax2 = true, hasnan = false, negz = false, unsorted = false;
    int lsbmin = INT32_MAX;
    double amax = 0.0;
    long long vcarry = 0;
    uint32_t qcarry = 0;
    long long prev_off = -1;   // offset (ms) of the previous datapoint
    for (uint32_t i0 = 0; i0 < ndp; i0 += 64) {
      const uint32_t i = i0 + lane;
      const bool in = i < ndp;
      uint32_t qpos = 0, w = 2;
      if (flags & ROW_QW_MASK) {
        w = flags & ROW_QW_MASK;
        qpos = i * w;
      } else {
        // mixed: positions found by the sequential walk below
      }
      uint32_t fb = 0;
      if (flags & ROW_QW_MASK) {
        if (in) fb = q[qpos + w - 1];
      } else {
        // mixed rows are rare: lane 0 computes every width sequentially, then broadcasts through shuffles
        uint32_t pos = qcarry, mypos = 0, myw = 2;
        for (int t = 0; t < 64 && i0 + t < ndp; t++) {
          const uint32_t ww = ((q[pos] & 0xF0) == 0xF0) ? 4 : 2;
          if (t == lane) { mypos = pos; myw = ww; }
          pos += ww;
        }
        qpos = mypos;
        w = myw;
        if (in) fb = q[qpos + w - 1];
        qcarry = __shfl(pos, 0, 64);
      }
      const int len = in ? (int)(fb & 7) + 1 : 0;
      const bool fl = (fb & 8) != 0;
      // offset order (strictly increasing in a well-formed compacted cell)
      long long off = -1;
      if (in) {
        if (w == 4) off = (long long)((((uint32_t)q[qpos] << 24) | ((uint32_t)q[qpos + 1] << 16) |
                                       ((uint32_t)q[qpos + 2] << 8) | q[qpos + 3]) & 0x0FFFFFC0u) >> 6;
        else off = (long long)((((uint32_t)q[qpos] << 8) | q[qpos + 1]) >> 4) * 1000;
      }
      long long po = __shfl_up(off, 1, 64);
      if (lane == 0) po = prev_off;
      if (in && off <= po) unsorted = true;
      prev_off = __shfl(off, (int)min((uint32_t)63, ndp - 1 - i0), 64);
      if (in && !fl) allf = false;
      if (in && fl) alli = false;
      if (in && len > 2) vmax2 = false;
      if (in && (fl ? (len != 4 && len != 8) : (len == 3 || (len >= 5 && len <= 7)))) bad = true;
      const int incl = wave_incl_sum(len);
      const long long vo = vcarry + incl - len;
      vcarry += __shfl(incl, 63, 64);
      if (in && !bad && vo + len <= (long long)d.vlen) {
        uint64_t bits = 0;
        for (int b = 0; b < len; b++) bits = (bits << 8) | v[vo + b];
        double x = 0.0;
        decode_value(bits, len, fl, x);
        if (val2 && w == 2 && (flags & ROW_QW_MASK) == 2 && !fl && len <= 2)
          reinterpret_cast<int16_t*>(val2 + d.qoff)[i] = (int16_t)(long long)x;
        if (isnan(x)) hasnan = true;
        if (x == 0.0 && signbit(x)) negz = true;
        if (!isnan(x)) {
          const double ax = fabs(x);
          if (ax > amax || isinf(ax)) amax = fmax(amax, ax);
          if (x != 0.0 && !isinf(x)) lsbmin = min(lsbmin, lsb_exp(x));
        }
      }
    }
    if (vcarry > (long long)d.vlen) bad = true;
    bad = __any(bad);
    allf = __all(allf);
    alli = __all(alli);
    vmax2 = __all(vmax2);
    hasnan = __any(hasnan);
    negz = __any(negz);
    unsorted = __any(unsorted);
    lsbmin = wave_min(lsbmin);
#pragma unroll
    for (int dd = 32; dd >= 1; dd >>= 1) amax = fmax(amax, __shfl_xor(amax, dd, 64));
    if (lane == 0) {
      if (bad) {
        flags |= ROW_ERR;
        set_err(err, TSDB_E_ILLEGAL_DATA);
      }
      if (allf) flags |= ROW_ALLF;
      if (alli) flags |= ROW_ALLI;
      if (vmax2) flags |= ROW_VLE2;
      if (hasnan) flags |= ROW_NAN;
      if (negz) flags |= ROW_NEGZ;
      if (unsorted) flags |= ROW_UNSORTED;
      flags |= d.flags & ROW_SFIRST;
      if (row_nocert(lsbmin, amax)) flags |= ROW_NOCERT;
      d.ndp = ndp;
      d.flags = flags;
      d.lsb = lsbmin;
      d.absmax = amax;
      rows[r] = d;
    }
  }
}


// ---- classes ----------------------------------------------------------------------------
__host__ __device__ constexpr int idx_cls(int qw, int L) {
  return 1 + (qw == 4 ? 5 : 0) + (L == 0 ? 0 : L == 1 ? 1 : L == 2 ? 2 : L == 4 ? 3 : 4);
}

// A row fits k_index_short: 2-byte qualifiers (by its first one), one chunk, 4-byte values or
// 1-2-byte-integer value bytes (uniform 1 / 2 or variable within ndp .. 2 ndp + meta).
__device__ __forceinline__ bool idx_short_ok(int qw, uint32_t L, uint64_t ndp, uint32_t vlen, bool uni) {
  if (qw != 2 || ndp == 0 || ndp > (uint64_t)CH) return false;
  if (uni) return L == 1 || L == 2 || L == 4;
  return (uint64_t)vlen >= ndp && (uint64_t)vlen <= 2 * ndp + 1;
}

__global__ __launch_bounds__(256) void k_index_hint(const uint8_t* __restrict__ qual, const RowDesc* __restrict__ rows,
                                                    int64_t n_rows, uint8_t* __restrict__ hint, uint32_t* cnt) {
  __shared__ uint32_t h[16];
  if (threadIdx.x < 16) h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int cls = -1, slot = -1;
  if (r < n_rows) {
    const RowDesc& d = rows[r];
    const uint32_t qlen = d.qlen, vlen = d.vlen;
    cls = 0;
    bool sh = false;
    if (qlen > 0) {
      const uint32_t w = *reinterpret_cast<const uint32_t*>(qual + d.qoff);   // qoff is 16-B aligned
      const int qw = (w & 0xF0) == 0xF0 ? 4 : 2;
      if (qlen % qw == 0) {
        const uint32_t L = ((w >> (8 * (qw - 1))) & 7) + 1;
        const uint64_t ndp = qlen / qw;
        const bool uni = (L == 1 || L == 2 || L == 4 || L == 8) && (uint64_t)vlen == ndp * L + (ndp > 1 ? 1 : 0);
        cls = idx_cls(qw, uni ? (int)L : 0);
        sh = idx_short_ok(qw, L, ndp, vlen, uni);
      }
    }
    hint[r] = (uint8_t)(cls | (sh ? HINT_SHORT : 0));
    slot = sh ? (cls == idx_cls(2, 4) ? IDX_C_SHORT4 : IDX_C_SHORTV) : cls;
  }
  // wave-aggregated counts (a class per ballot): one LDS atomic per class present in the wave
  const int lane = lane_id();
  for (int c = 0; c < 16; c++) {
    const uint64_t m = __ballot(slot == c);
    if (m && lane == 0) atomicAdd(&h[c], (uint32_t)__popcll(m));
  }
  __syncthreads();
  if (threadIdx.x < 16 && h[threadIdx.x]) atomicAdd(&cnt[threadIdx.x], h[threadIdx.x]);
}

// cursor[c] starts at class c's list offset
__global__ __launch_bounds__(256) void k_index_scatter(const uint8_t* __restrict__ hint, int64_t n_rows, uint32_t* cursor,
                                                       int32_t* __restrict__ list) {
  __shared__ uint32_t h[16], base[16];
  if (threadIdx.x < 16) h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int cls = 0;
  uint32_t local = 0;
  if (r < n_rows) {
    cls = hint[r];
    if (cls & HINT_SHORT) cls = 0;   // (k_index_short's: not listed)
    local = atomicAdd(&h[cls], 1u);
  }
  __syncthreads();
  if (threadIdx.x < IDX_NCLS && h[threadIdx.x]) base[threadIdx.x] = atomicAdd(&cursor[threadIdx.x], h[threadIdx.x]);
  __syncthreads();
  if (r < n_rows && cls) list[base[cls] + local] = (int32_t)r;
}

struct IdxRow {          // wave-uniform row state
  int64_t r;
  uint64_t qoff, voff;
  uint32_t qlen, vlen, flags_in, ndp;
};

template <int QW>
__device__ __forceinline__ IdxRow idx_row(const RowDesc* __restrict__ rows, int64_t r) {
  IdxRow w;
  const RowDesc& d = rows[r];
  w.r = r;
  w.qoff = d.qoff;
  w.voff = d.voff;
  w.qlen = d.qlen;
  w.vlen = d.vlen;
  w.flags_in = d.flags;
  w.ndp = w.qlen / QW;
  return w;
}

template <int QW, int L>
struct IdxLd {           // one chunk's loads
  uint4 q[QW / 2];
  uint4 v[L <= 2 ? 1 : L / 2];
};

// Chunk c's loads: the same for every lane and every chunk (lanes past the row's datapoints
// re-read its start; the variable class always loads a 16-B slice of the first 1 KB).
template <int QW, int L>
__device__ __forceinline__ void idx_issue(const uint8_t* __restrict__ qual, const uint8_t* __restrict__ val,
                                          const IdxRow& w, uint32_t c, IdxLd<QW, L>& ld) {
  const int lane = lane_id();
  int64_t i = (int64_t)c * CH + (int64_t)lane * DPL;
  if (i >= (int64_t)w.ndp) i = 0;
  const uint4* q = reinterpret_cast<const uint4*>(qual + w.qoff + i * QW);
#pragma unroll
  for (int k = 0; k < QW / 2; k++) ld.q[k] = q[k];
  const uint8_t* v = val + w.voff;
  if (L == 0) {
    ld.v[0] = *reinterpret_cast<const uint4*>(v + ((uint32_t)lane * 16 < w.vlen ? lane * 16 : 0));
  } else if (L == 1) {
    const uint2 t = *reinterpret_cast<const uint2*>(v + i);
    ld.v[0] = make_uint4(t.x, t.y, 0, 0);
  } else {
    const uint4* p = reinterpret_cast<const uint4*>(v + i * L);
#pragma unroll
    for (int k = 0; k < (L <= 2 ? 1 : L / 2); k++) ld.v[k] = p[k];
  }
}

// value statistics in the integer domain (bit patterns / magnitudes), one conversion per
// chunk: NaN, -0.0, max |x| (Inf included, NaN excluded), least significant set bit
__device__ __forceinline__ void idx_stats(IdxAcc& a, const uint32_t qq[DPL], const int len[DPL], const uint64_t be[DPL],
                                          int nin, int64_t vo, uint32_t vlen) {
  uint32_t fmax_bits = 0;      // float32 |x| bits
  uint64_t dmax_bits = 0;      // float64 |x| bits
  uint64_t imax = 0;           // |long|
  int64_t o = vo;
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    if (j < nin && o + len[j] <= (int64_t)vlen) {
      const uint64_t b = be[j];
      if (qq[j] & 8) {
        if (len[j] == 4) {
          const uint32_t ab = (uint32_t)b & 0x7FFFFFFFu;
          if (ab > 0x7F800000u) {
            a.nan = true;
          } else {
            a.negz |= (uint32_t)b == 0x80000000u;
            fmax_bits = max(fmax_bits, ab);
            const uint32_t E = ab >> 23, M = ab & 0x7FFFFFu;
            if (ab != 0 && E != 0xFF) a.lsb = min(a.lsb, E == 0 ? -149 + __ffs(M) - 1 : (int)E - 150 + __ffs(M | 0x800000u) - 1);
          }
        } else if (len[j] == 8) {
          const uint64_t ab = b & 0x7FFFFFFFFFFFFFFFULL;
          if (ab > 0x7FF0000000000000ULL) {
            a.nan = true;
          } else {
            a.negz |= b == 0x8000000000000000ULL;
            dmax_bits = ab > dmax_bits ? ab : dmax_bits;
            const uint32_t E = (uint32_t)(ab >> 52);
            const uint64_t M = ab & 0xFFFFFFFFFFFFFULL;
            if (ab != 0 && E != 0x7FF)
              a.lsb = min(a.lsb, E == 0 ? -1074 + __ffsll((long long)M) - 1
                                        : (int)E - 1075 + __ffsll((long long)(M | 0x10000000000000ULL)) - 1);
          }
        }
      } else {
        const int sh = 64 - 8 * len[j];   // sign-extended integer of len bytes
        const int64_t x = (int64_t)(b << sh) >> sh;
        const uint64_t ax = x < 0 ? (uint64_t)0 - (uint64_t)x : (uint64_t)x;
        imax = ax > imax ? ax : imax;
        if (ax != 0) a.lsb = min(a.lsb, ax <= (1ULL << 53) ? __ffsll((long long)ax) - 1 : lsb_exp((double)x));
      }
    }
    o += len[j];
  }
  a.amax = fmax(a.amax, fmax(fmax((double)__uint_as_float(fmax_bits), __longlong_as_double((long long)dmax_bits)),
                             (double)imax));
}

// The row's offset order (Internal.compareQualifiers order of a compacted cell: strictly
// increasing), lane-local then across lanes and chunks.
__device__ __forceinline__ void idx_order(const int off[DPL], int nin, int64_t i0, const IdxRow& w, int& prev_off,
                                          IdxAcc& a) {
  const int lane = lane_id();
  bool uns = false;
#pragma unroll
  for (int j = 1; j < DPL; j++) uns |= (j < nin) & (off[j] <= off[j - 1]);
  const int last = off[max(0, nin - 1)];
  int pl = __shfl_up(last, 1, 64);
  if (lane == 0) pl = prev_off;
  uns |= (nin > 0) & (off[0] <= pl);
  a.unsorted |= uns;
  prev_off = __shfl(last, (int)((min((int64_t)CH, (int64_t)w.ndp - i0) - 1) / DPL), 64);
}

// int16 copy of the lane's 8 values (1-2-byte integers; other lanes' slots are never read:
// val2 is consulted only for rows whose every value is a 1-2-byte integer)
__device__ __forceinline__ void idx_val2(uint8_t* __restrict__ val2, const IdxRow& w, int64_t i, const int len[DPL],
                                         const uint32_t lo[DPL]) {
  uint32_t h[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t x0 = len[2 * k] == 1 ? (uint32_t)(int32_t)(int8_t)(lo[2 * k] & 0xFF) : lo[2 * k];
    const uint32_t x1 = len[2 * k + 1] == 1 ? (uint32_t)(int32_t)(int8_t)(lo[2 * k + 1] & 0xFF) : lo[2 * k + 1];
    h[k] = (x0 & 0xFFFF) | (x1 << 16);
  }
  *reinterpret_cast<uint4*>(val2 + w.qoff + 2 * i) = make_uint4(h[0], h[1], h[2], h[3]);
}

// Statistics of the lane's integer values (sign-extended from len bytes), branch-free.
__device__ __forceinline__ void idx_int_stats(IdxAcc& a, const uint64_t be[DPL], const int len[DPL], int nin) {
  uint64_t imax = 0;
  int lsb = INT32_MAX;
  bool big = false;
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    const int sh = 64 - 8 * max(1, len[j]);
    const int64_t x = (int64_t)(be[j] << sh) >> sh;
    const uint64_t ax = x < 0 ? (uint64_t)0 - (uint64_t)x : (uint64_t)x;
    const bool ok = (j < nin) & (ax != 0);
    imax = ok && ax > imax ? ax : imax;
    lsb = min(lsb, ok ? (int)__builtin_ctzll(ax) : INT32_MAX);
    big |= ok & (ax > (1ULL << 53));
  }
  if (big) {   // |x| > 2^53: the double rounds, take its least significant bit
    lsb = INT32_MAX;
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      const int sh = 64 - 8 * max(1, len[j]);
      const int64_t x = (int64_t)(be[j] << sh) >> sh;
      if (j < nin && x != 0) lsb = min(lsb, lsb_exp((double)x));
    }
  }
  a.lsb = min(a.lsb, lsb);
  a.amax = fmax(a.amax, (double)imax);
}

// Chunk decode of the variable-length class: wave prefix sum of the lengths, the chunk's
// value bytes staged in LDS (the first 1 KB from the prefetch; never past the row's
// 16-B-aligned extent).  false: a qualifier of the other width -> the generic path.
template <int QW, bool V2>
__device__ __forceinline__ bool idx_chunk_var(const uint8_t* __restrict__ val, uint8_t* __restrict__ val2,
                                              const IdxRow& w, uint32_t c, const IdxLd<QW, 0>& ld, uint32_t* stage,
                                              int64_t& carry, int& prev_off, IdxAcc& a) {
  const int lane = lane_id();
  const int64_t i0 = (int64_t)c * CH;
  const int nin = (int)min((int64_t)DPL, max((int64_t)0, (int64_t)w.ndp - i0 - (int64_t)lane * DPL));
  uint32_t qq[DPL];
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    const uint32_t* ws = &ld.q[0].x;
    if (QW == 2) {
      const uint32_t b = __builtin_bswap32(ws[j >> 1]);
      qq[j] = (j & 1) ? (b & 0xFFFF) : (b >> 16);
    } else {
      qq[j] = __builtin_bswap32(ws[j]);
    }
  }
  bool fail = false, bad = false, vmax2 = true;
  uint32_t fl_or = 0, fl_and = 8;
  int len[DPL], off[DPL];
  int lsum = 0, lmin = 99, lmax = -1;
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    const bool in = j < nin;
    fail |= in & (QW == 2 ? (qq[j] >> 12) == 0xF : (qq[j] >> 28) != 0xF);
    len[j] = in ? (int)(qq[j] & 7) + 1 : 0;
    lsum += len[j];
    const uint32_t f = qq[j] & 8;
    fl_or |= in ? f : 0u;
    fl_and &= in ? f : 8u;
    lmin = min(lmin, in ? len[j] : 99);
    lmax = max(lmax, len[j] - (in ? 0 : 1));
    vmax2 &= len[j] <= 2;
    bad |= in & (f ? (len[j] != 4 && len[j] != 8) : (len[j] == 3 || (len[j] >= 5 && len[j] <= 7)));
    off[j] = QW == 2 ? (int)(qq[j] >> 4) * 1000 : (int)((qq[j] & 0x0FFFFFC0u) >> 6);
  }
  if (__any(fail)) return false;
  a.allf &= fl_and != 0;
  a.alli &= fl_or == 0;
  a.vmax2 &= vmax2;
  a.bad |= bad;
  a.lmin = min(a.lmin, lmin);
  a.lmax = max(a.lmax, lmax);
  idx_order(off, nin, i0, w, prev_off, a);
  // stage the chunk's value bytes
  const uint8_t* v = val + w.voff;
  const int incl = wave_incl_sum_dpp(lsum);
  const int total = __builtin_amdgcn_readlane(incl, 63);
  const int64_t a0 = carry & ~(int64_t)15;
  const int lead = (int)(carry - a0);
  const int64_t vlen16 = ((int64_t)w.vlen + 15) & ~(int64_t)15;
  const int64_t nst = min((int64_t)(lead + total + 15) & ~(int64_t)15, vlen16 - a0);
  WAVE_SYNC();
  int64_t o0 = 0;
  if (c == 0) {   // the prefetched first 1 KB
    if ((int64_t)lane * 16 < nst) *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(stage) + lane * 16) = ld.v[0];
    o0 = 64 * 16;
  }
  for (int64_t o = o0 + (int64_t)lane * 16; o < nst; o += 64 * 16)
    *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(stage) + o) = *reinterpret_cast<const uint4*>(v + a0 + o);
  WAVE_SYNC();
  uint64_t be[DPL];
  int b = lead + incl - lsum;
  const int64_t vo = carry + incl - lsum;
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    const bool ok = (j < nin) & (b + len[j] <= nst);
    const uint64_t raw = __builtin_bswap64(stage_u64(stage, min(b, IDX_STAGE - 12)));
    be[j] = ok ? raw >> (64 - 8 * max(1, len[j])) : 0;
    b += len[j];
  }
  if (V2 && nin > 0) {
    uint32_t lo[DPL];
#pragma unroll
    for (int j = 0; j < DPL; j++) lo[j] = (uint32_t)be[j];
    idx_val2(val2, w, i0 + (int64_t)lane * DPL, len, lo);
  }
  if (__all(fl_or == 0)) idx_int_stats(a, be, len, nin);
  else idx_stats(a, qq, len, be, nin, vo, w.vlen);
  carry += total;
  return true;
}

// Branch-free chunk decode of a uniform class (every length == L): per-datapoint conditions
// are selects, not branches, and the value statistics take the float32-only / integer-only
// fast path when the wave's chunk allows.  false: the class hypothesis failed.
template <int QW, int L, bool V2>
__device__ __forceinline__ bool idx_chunk_uni(uint8_t* __restrict__ val2, const IdxRow& w, uint32_t c,
                                              const IdxLd<QW, L>& ld, int& prev_off, IdxAcc& a) {
  const int lane = lane_id();
  const int64_t i0 = (int64_t)c * CH;
  const int nin = (int)min((int64_t)DPL, max((int64_t)0, (int64_t)w.ndp - i0 - (int64_t)lane * DPL));
  uint32_t qq[DPL];
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    const uint32_t* ws = &ld.q[0].x;
    if (QW == 2) {
      const uint32_t b = __builtin_bswap32(ws[j >> 1]);
      qq[j] = (j & 1) ? (b & 0xFFFF) : (b >> 16);
    } else {
      qq[j] = __builtin_bswap32(ws[j]);
    }
  }
  bool fail = false;
  uint32_t fl_or = 0, fl_and = 8;
  int off[DPL];
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    const bool in = j < nin;
    const bool ww = QW == 2 ? (qq[j] >> 12) == 0xF : (qq[j] >> 28) != 0xF;
    fail |= in & (ww | ((qq[j] & 7) != (uint32_t)(L - 1)));
    const uint32_t f = qq[j] & 8;
    fl_or |= in ? f : 0u;
    fl_and &= in ? f : 8u;
    off[j] = QW == 2 ? (int)(qq[j] >> 4) * 1000 : (int)((qq[j] & 0x0FFFFFC0u) >> 6);
  }
  if (__any(fail)) return false;
  a.allf &= fl_and != 0;
  a.alli &= fl_or == 0;
  if (L <= 2) a.bad |= fl_or != 0;   // a float of 1 or 2 bytes
  idx_order(off, nin, i0, w, prev_off, a);
  const uint32_t* vw = &ld.v[0].x;
  int len[DPL];
#pragma unroll
  for (int j = 0; j < DPL; j++) len[j] = L;
  if (L == 8) {
    uint64_t be[DPL];
#pragma unroll
    for (int j = 0; j < DPL; j++) be[j] = ((uint64_t)__builtin_bswap32(vw[2 * j]) << 32) | __builtin_bswap32(vw[2 * j + 1]);
    if (__all(fl_or == 0)) idx_int_stats(a, be, len, nin);
    else idx_stats(a, qq, len, be, nin, 0, 0xFFFFFFFFu);
    return true;
  }
  uint32_t be[DPL];
#pragma unroll
  for (int j = 0; j < DPL; j++) {
    if (L == 1) be[j] = (vw[j >> 2] >> ((j & 3) * 8)) & 0xFF;
    else if (L == 2) { const uint32_t b = __builtin_bswap32(vw[j >> 1]); be[j] = (j & 1) ? (b & 0xFFFF) : (b >> 16); }
    else be[j] = __builtin_bswap32(vw[j]);
  }
  if (V2 && QW == 2 && L <= 2 && nin > 0) idx_val2(val2, w, i0 + (int64_t)lane * DPL, len, be);
  if (L == 4 && __all(fl_and != 0)) {
    // every value of the chunk float32: bit-pattern statistics
    uint32_t fmax_bits = 0;
    bool nan = false, negz = false;
    int lsb = INT32_MAX;
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      const bool in = j < nin;
      const uint32_t ab = be[j] & 0x7FFFFFFFu;
      const bool isn = ab > 0x7F800000u;
      const bool ok = in & !isn;
      nan |= in & isn;
      negz |= ok & (be[j] == 0x80000000u);
      fmax_bits = max(fmax_bits, ok ? ab : 0u);
      const uint32_t E = ab >> 23, M = ab & 0x7FFFFFu;
      const int lj = E == 0 ? (int)__builtin_ctz(M | 0x80000000u) - 149 : (int)E - 150 + (int)__builtin_ctz(M | 0x800000u);
      lsb = min(lsb, (ok & (ab != 0) & (E != 0xFF)) ? lj : INT32_MAX);
    }
    a.nan |= nan;
    a.negz |= negz;
    a.lsb = min(a.lsb, lsb);
    a.amax = fmax(a.amax, (double)__uint_as_float(fmax_bits));
    return true;
  }
  if (__all(fl_or == 0)) {
    // integers of L <= 4 bytes: magnitude and trailing zeros (|x| <= 2^31: exact as doubles)
    uint32_t imax = 0;
    int lsb = INT32_MAX;
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      const int sh = 32 - 8 * L;
      const int32_t x = L == 4 ? (int32_t)be[j] : (int32_t)(be[j] << (sh & 31)) >> (sh & 31);
      const uint32_t ax = x < 0 ? 0u - (uint32_t)x : (uint32_t)x;
      const bool ok = (j < nin) & (ax != 0);
      imax = max(imax, ok ? ax : 0u);
      lsb = min(lsb, ok ? (int)__builtin_ctz(ax) : INT32_MAX);
    }
    a.lsb = min(a.lsb, lsb);
    a.amax = fmax(a.amax, (double)imax);
    return true;
  }
  // integers and floats mixed in the chunk
  uint64_t be64[DPL];
#pragma unroll
  for (int j = 0; j < DPL; j++) be64[j] = be[j];
  idx_stats(a, qq, len, be64, nin, 0, 0xFFFFFFFFu);
  return true;
}

// One wave per row of class (QW, L) (grid-stride over the class list); V2: also write the
// int16 copy of 1-2-byte integers (2-byte-qualifier integer classes, when val2 is allocated).
// Rows whose hypothesis fails get hint 0 (k_index_generic).
template <int QW, int L, bool V2>
__global__ __launch_bounds__(256) void k_index_cls(const uint8_t* __restrict__ qual, const uint8_t* __restrict__ val,
                                                   uint8_t* __restrict__ val2, RowDesc* __restrict__ rows,
                                                   uint8_t* __restrict__ hint, const int32_t* __restrict__ list,
                                                   int64_t n, int32_t* err) {
  __shared__ uint32_t stage_all[4][L == 0 ? IDX_STAGE / 4 : 1];
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* stage = stage_all[wv];
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  int64_t i = (int64_t)blockIdx.x * 4 + wv;
  if (i >= n) return;
  IdxRow cur = idx_row<QW>(rows, list[i]);
  IdxRow nxt = i + nw < n ? idx_row<QW>(rows, list[i + nw]) : cur;
  IdxLd<QW, L> ld;
  idx_issue<QW, L>(qual, val, cur, 0, ld);
  for (;;) {
    const bool has_next = i + nw < n;
    const IdxRow nxt2 = i + 2 * nw < n ? idx_row<QW>(rows, list[i + 2 * nw]) : nxt;
    IdxAcc a;
    idx_acc_init(a);
    int64_t carry = 0;
    int prev_off = -1;
    bool ok = true;
    const uint32_t nch = (cur.ndp + CH - 1) / CH;
    for (uint32_t c = 0; c < nch; c++) {
      IdxLd<QW, L> nl;
      idx_issue<QW, L>(qual, val, c + 1 < nch ? cur : nxt, c + 1 < nch ? c + 1 : 0, nl);
      if (ok) {
        if constexpr (L != 0) ok = idx_chunk_uni<QW, L, V2>(val2, cur, c, ld, prev_off, a);
        else ok = idx_chunk_var<QW, V2>(val, val2, cur, c, ld, stage, carry, prev_off, a);
      }
      ld = nl;
    }
    if (!ok) {
      if (lane == 0) hint[cur.r] = 0;   // k_index_generic takes the row
    } else {
      if (L == 0 && carry > (int64_t)cur.vlen) a.bad = true;   // (uniform classes: vlen matches by construction)
      const bool bad = __any(a.bad);
      const bool allf = __all(a.allf), alli = __all(a.alli);
      const bool vmax2 = L != 0 ? L <= 2 : __all(a.vmax2);
      const bool hasnan = __any(a.nan), negz = __any(a.negz), unsorted = __any(a.unsorted);
      const int lsbmin = wave_min(a.lsb);
      const int lmin = L != 0 ? L : wave_min(a.lmin), lmax = L != 0 ? L : wave_max(a.lmax);
      double amax = a.amax;
#pragma unroll
      for (int dd = 32; dd >= 1; dd >>= 1) amax = fmax(amax, __shfl_xor(amax, dd, 64));
      if (lane == 0) {
        uint32_t flags = (uint32_t)QW;
        if (lmin == lmax) flags |= (uint32_t)lmin << ROW_VL_SHIFT;
        if (bad) {
          flags |= ROW_ERR;
          set_err(err, TSDB_E_ILLEGAL_DATA);
        }
        if (allf) flags |= ROW_ALLF;
        if (alli) flags |= ROW_ALLI;
        if (vmax2) flags |= ROW_VLE2;
        if (hasnan) flags |= ROW_NAN;
        if (negz) flags |= ROW_NEGZ;
        if (unsorted) flags |= ROW_UNSORTED;
        flags |= cur.flags_in & ROW_SFIRST;
        if (row_nocert(lsbmin, amax)) flags |= ROW_NOCERT;
        RowDesc& o = rows[cur.r];
        o.ndp = cur.ndp;
        o.flags = flags;
        o.lsb = lsbmin;
        o.absmax = amax;
      }
    }
    if (!has_next) break;
    i += nw;
    cur = nxt;
    nxt = nxt2;
  }
}


// ---- k_index_short: one-chunk rows of 2-byte qualifiers (config 3's hour rows) ----------
//
// A wave takes 64 consecutive rows.  Lane l loads row l's descriptor once (one 48-B line a lane),
// the rows the hint marks short are walked in order with their fields read by readlane (no
// dependent descriptor load in the loop), and the next row's qualifier / value loads are issued
// before the current row decodes.  Lane i covers datapoints 8i .. 8i + 7 (45 lanes for 360):
//   * 4-byte values (float32, or int32 vle): 32 B of values a lane at 4 x its first datapoint;
//   * 1-2-byte integers (uniform or variable): the row's value bytes (<= 1 KB) staged in LDS
//     by 16-B lane slices, each lane's start from a DPP prefix sum of its lengths, its <= 16
//     bytes read as three 8-B LDS words and consumed value by value from a 128-bit window;
//     the int16 copy (val2) is one 16-B store a lane.
// A row breaking a premise (a 4-byte qualifier inside, a float of 1-2 bytes, a 4- or 8-byte
// integer among the short ones, 4-byte values mixing floats and integers) is handed to
// k_index_generic (hint 0).  Results are k_index_cls's for the same row: the same flags, lsb and
// max |value| (tests/test_gpu_scale.py checks every RowDesc against the generic path).
struct ShortLd {
  uint4 q;       // qualifiers of the lane's 8 datapoints
  uint4 v0, v1;  // 4-byte values: 32 B at 4 x 8 lane; 1-2-byte values: v0 = bytes 16 lane .. + 15
};

__device__ __forceinline__ void short_issue(const uint8_t* __restrict__ qual, const uint8_t* __restrict__ val,
                                            uint64_t qoff, uint64_t voff, uint32_t ndp, bool u4, ShortLd& ld) {
  const int lane = lane_id();
  const uint32_t i = (uint32_t)lane * DPL < ndp ? (uint32_t)lane * DPL : 0u;   // lanes past the row re-read its start
  ld.q = *reinterpret_cast<const uint4*>(qual + qoff + 2 * (uint64_t)i);
  const uint64_t vb = voff + (u4 ? 4 * (uint64_t)i : 2 * (uint64_t)i);
  ld.v0 = *reinterpret_cast<const uint4*>(val + vb);
  ld.v1 = *reinterpret_cast<const uint4*>(val + vb + (u4 ? 16 : 0));
}

// Row j's results (every lane calls it; the values are wave-uniform).
static constexpr uint32_t SHORT_FAIL = 0x80000000u;   // (a result flag of k_index_short's batch, not a RowDesc flag)
struct ShortRes {
  uint32_t flags;
  int32_t lsb;
  double amax;
  bool fail;
};

__device__ __forceinline__ ShortRes short_row_general(const ShortLd& ld, uint8_t* __restrict__ val2, const uint8_t* st8,
                                                      uint4* stage, uint64_t cq, uint32_t cn, uint32_t cvl, bool cu4) {
  const int lane = lane_id();
  const int i0 = lane * DPL;
  const int nin = min(DPL, max(0, (int)cn - i0));
  uint32_t qq[DPL];
  {
    const uint32_t ws[4] = {ld.q.x, ld.q.y, ld.q.z, ld.q.w};
#pragma unroll
    for (int k = 0; k < DPL; k++) {
      const uint32_t b = __builtin_bswap32(ws[k >> 1]);
      qq[k] = (k & 1) ? (b & 0xFFFF) : (b >> 16);
    }
  }
  bool fail = false, bad = false, uns = false;
  uint32_t fl_or = 0, fl_and = 8;
  int len[DPL], lsum = 0, lmin = 99, lmax = -1;
  int prev = -1;
#pragma unroll
  for (int k = 0; k < DPL; k++) {
    const bool in = k < nin;
    const uint32_t f = qq[k] & 8;
    len[k] = in ? (int)(qq[k] & 7) + 1 : 0;
    fail |= in & ((qq[k] >> 12) == 0xF);                    // a 4-byte qualifier inside
    fl_or |= in ? f : 0u;
    fl_and &= in ? f : 8u;
    lsum += len[k];
    lmin = min(lmin, in ? len[k] : 99);
    lmax = max(lmax, in ? len[k] : -1);
    const int off = (int)(qq[k] >> 4);                       // seconds: strictly increasing
    uns |= in & (k > 0) & (off <= prev);
    prev = in ? off : prev;
  }
  {   // order across lanes: this lane's first offset against the previous lane's last
    const int last = (int)(qq[max(0, nin - 1)] >> 4);
    const int pl = __builtin_amdgcn_update_dpp(-1, nin > 0 ? last : -1, 0x138, 0xF, 0xF, false);   // wave_shr:1
    uns |= (lane > 0) & (nin > 0) & ((int)(qq[0] >> 4) <= pl);
  }
  uint32_t flags = 2;
  int lsb = INT32_MAX;
  uint32_t amax_bits = 0;   // float32 |x| bits, or |int32|
  bool isf = false, nan = false, negz = false;
  if (cu4) {
    // ---- 4-byte values: float32 or int32
#pragma unroll
    for (int k = 0; k < DPL; k++) fail |= (k < nin) & (len[k] != 4);
    const bool allf = __all(fl_and != 0), alli = __all(fl_or == 0);
    fail |= !allf && !alli;                                  // floats and integers mixed: generic
    isf = allf;
    const uint32_t vw[8] = {ld.v0.x, ld.v0.y, ld.v0.z, ld.v0.w, ld.v1.x, ld.v1.y, ld.v1.z, ld.v1.w};
#pragma unroll
    for (int k = 0; k < DPL; k++) {
      const bool in = k < nin;
      const uint32_t be = __builtin_bswap32(vw[k]);
      // float32: bit-pattern statistics; int32: magnitude and trailing zeros (branch-free select)
      const uint32_t ab = be & 0x7FFFFFFFu;
      const bool isn = allf & (ab > 0x7F800000u);
      const uint32_t E = ab >> 23, M = ab & 0x7FFFFFu;
      const int lf = E == 0 ? (int)__builtin_ctz(M | 0x80000000u) - 149 : (int)E - 150 + (int)__builtin_ctz(M | 0x800000u);
      const uint32_t ai = (int32_t)be < 0 ? 0u - be : be;
      const uint32_t mag = allf ? ab : ai;
      const bool ok = in & !isn & (mag != 0) & (!allf | (E != 0xFF));
      nan |= in & isn;
      negz |= allf & in & (be == 0x80000000u);
      amax_bits = max(amax_bits, (in & !isn) ? mag : 0u);
      lsb = min(lsb, ok ? (allf ? lf : (int)__builtin_ctz(ai)) : INT32_MAX);
    }
    flags |= (4u << ROW_VL_SHIFT) | (allf ? ROW_ALLF : 0u) | (alli ? ROW_ALLI : 0u);
  } else {
    // ---- 1-2-byte integers: stage the value bytes, each lane's start by prefix sum
    fail |= (fl_or != 0) | (lmax > 2);
    const int incl = wave_incl_sum_dpp(lsum);
    const int total = __builtin_amdgcn_readlane(incl, 63);
    bad |= lane == 0 && (uint32_t)total > cvl;              // values past the row's value bytes
    // (LDS order within the wave: the previous row's reads are done before this write lands,
    // and the write before the reads below -- lgkmcnt waits, no memory fence)
    __builtin_amdgcn_wave_barrier();
    stage[lane] = ld.v0;
    __builtin_amdgcn_s_waitcnt(0xC07F);                     // lgkmcnt(0), vmcnt / expcnt untouched
    __builtin_amdgcn_wave_barrier();
    const int b = min(incl - lsum, 1024);
    const int b8 = b & ~7, d = (b - b8) * 8;
    const uint64_t x0 = *reinterpret_cast<const uint64_t*>(st8 + b8);
    const uint64_t x1 = *reinterpret_cast<const uint64_t*>(st8 + b8 + 8);
    const uint64_t x2 = *reinterpret_cast<const uint64_t*>(st8 + b8 + 16);
    uint64_t lo = d ? (x0 >> d) | (x1 << (64 - d)) : x0;
    uint64_t hi = d ? (x1 >> d) | (x2 << (64 - d)) : x1;
    uint32_t h16[4] = {0, 0, 0, 0};
    uint32_t imax = 0;
    const int vend = (int)((cvl + 15) & ~15u);   // (k_index_cls decodes up to the 16-B-aligned extent)
    int pos = b;
#pragma unroll
    for (int k = 0; k < DPL; k++) {
      const int L = len[k];
      // big-endian: first byte most significant
      const uint32_t b0 = (uint32_t)lo & 0xFF, b1 = (uint32_t)(lo >> 8) & 0xFF;
      const int32_t xv = L == 2 ? (int32_t)(int16_t)(uint16_t)((b0 << 8) | b1) : (int32_t)(int8_t)(uint8_t)b0;
      const int32_t x = pos + L <= vend ? xv : 0;
      pos += L;
      const uint32_t ax = x < 0 ? 0u - (uint32_t)x : (uint32_t)x;
      const bool ok = (k < nin) & (ax != 0);
      imax = max(imax, ok ? ax : 0u);
      lsb = min(lsb, ok ? (int)__builtin_ctz(ax) : INT32_MAX);
      h16[k >> 1] |= ((uint32_t)x & 0xFFFF) << ((k & 1) * 16);
      const int sh = 8 * max(L, 1);
      if (L) {
        lo = (lo >> sh) | (hi << (64 - sh));
        hi >>= sh;
      }
    }
    amax_bits = imax;
    if (val2 && nin > 0)
      *reinterpret_cast<uint4*>(val2 + cq + 2 * (uint64_t)i0) = make_uint4(h16[0], h16[1], h16[2], h16[3]);
    const int wl = wave_reduce_i32(lmin, 99, [](int a, int c) { return min(a, c); });
    const int wh = wave_reduce_i32(lmax, -1, [](int a, int c) { return max(a, c); });
    flags |= ROW_ALLI | ROW_VLE2 | (wl == wh ? (uint32_t)wl << ROW_VL_SHIFT : 0u);
  }
  ShortRes R;
  R.fail = __any(fail);
  R.lsb = wave_reduce_i32(lsb, INT32_MAX, [](int a, int c) { return min(a, c); });
  const uint32_t wmax = (uint32_t)wave_reduce_i32((int)amax_bits, 0,
                                                  [](int a, int c) { return (int)max((uint32_t)a, (uint32_t)c); });
  R.amax = isf ? (double)__uint_as_float(wmax) : (double)wmax;
  if (__any(bad)) flags |= ROW_ERR;
  if (__any(nan)) flags |= ROW_NAN;
  if (__any(negz)) flags |= ROW_NEGZ;
  if (__any(uns)) flags |= ROW_UNSORTED;
  R.flags = flags;   // (ROW_NOCERT: k_index_short, per lane at the batch end)
  return R;
}


// ---- full-lane fast paths: every lane 0 or 8 datapoints (rows of a multiple of 8, 360 among them)
// The common rows' premises checked on packed qualifier words (two 2-byte qualifiers a word)
// and value bit patterns; false = a premise fails (a flag nibble off the class, offsets not
// strictly increasing or a 4-byte qualifier, NaN, a denormal, values past the row, ...) and
// short_row_general decodes the row -- whose results these equal wherever they return true.
__device__ __forceinline__ bool short_full_order(const uint32_t t[4], bool act) {
  uint32_t o[DPL];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    o[2 * i] = t[i] >> 20;
    o[2 * i + 1] = (t[i] >> 4) & 0xFFF;
  }
  bool inc = true;
#pragma unroll
  for (int k = 1; k < DPL; k++) inc &= o[k - 1] < o[k];
  const int pl = __builtin_amdgcn_update_dpp(-1, act ? (int)o[DPL - 1] : -1, 0x138, 0xF, 0xF, false);   // wave_shr:1
  // (a 2-byte qualifier's offset field is below 0xF00: a top nibble 0xF is a 4-byte qualifier)
  return inc & ((int)o[0] > pl) & (o[DPL - 1] < 0xF00u);
}

__device__ __forceinline__ bool short_full_u4(const ShortLd& ld, bool act, ShortRes& R) {
  const uint32_t t[4] = {__builtin_bswap32(ld.q.x), __builtin_bswap32(ld.q.y), __builtin_bswap32(ld.q.z),
                         __builtin_bswap32(ld.q.w)};
  // float32 of 4 bytes everywhere: flag nibble 0xB
  const uint32_t fx = ((t[0] ^ 0x000B000Bu) | (t[1] ^ 0x000B000Bu) | (t[2] ^ 0x000B000Bu) | (t[3] ^ 0x000B000Bu)) & 0x000F000Fu;
  const bool ord = short_full_order(t, act);   // (every lane: a DPP step inside)
  if (!__all(!act || (fx == 0 && ord))) return false;
  const uint32_t vw[8] = {ld.v0.x, ld.v0.y, ld.v0.z, ld.v0.w, ld.v1.x, ld.v1.y, ld.v1.z, ld.v1.w};
  uint32_t amax = 0, lsbk = 0xFFFFFFFFu;
  bool odd = false;
#pragma unroll
  for (int k = 0; k < DPL; k++) {
    const uint32_t be = __builtin_bswap32(vw[k]);
    const uint32_t ab = be & 0x7FFFFFFFu;
    const uint32_t E = ab >> 23;
    amax = max(amax, ab);
    // normal numbers only: a zero (-0.0 included), a denormal, an infinity or a NaN sends the row
    // to the general path; the least significant set bit as E + its place in the significand
    // (-150 once at the end)
    odd |= (E - 1u) >= 254u;
    lsbk = min(lsbk, E + (uint32_t)__builtin_ctz(be | 0x00800000u));
  }
  if (!act) { amax = 0; lsbk = 0xFFFFFFFFu; odd = false; }
  if (__any(odd)) return false;
  const uint32_t wmax = (uint32_t)wave_reduce_i32((int)amax, 0, [](int a, int c) { return (int)max((uint32_t)a, (uint32_t)c); });
  const uint32_t wl = (uint32_t)wave_reduce_i32((int)lsbk, -1, [](int a, int c) { return (int)min((uint32_t)a, (uint32_t)c); });
  R.fail = false;
  R.lsb = wl == 0xFFFFFFFFu ? INT32_MAX : (int)wl - 150;
  R.amax = (double)__uint_as_float(wmax);
  R.flags = 2u | (4u << ROW_VL_SHIFT) | ROW_ALLF;
  return true;
}

__device__ __forceinline__ bool short_full_vle(const ShortLd& ld, uint8_t* __restrict__ val2, const uint8_t* st8,
                                               uint4* stage, uint64_t cq, uint32_t cvl, bool act, ShortRes& R) {
  const int lane = lane_id();
  const uint32_t t[4] = {__builtin_bswap32(ld.q.x), __builtin_bswap32(ld.q.y), __builtin_bswap32(ld.q.z),
                         __builtin_bswap32(ld.q.w)};
  // integers of 1 or 2 bytes everywhere: flag nibble 0 or 1
  const uint32_t fx = (t[0] | t[1] | t[2] | t[3]) & 0x000E000Eu;
  const bool ord = short_full_order(t, act);   // (every lane: a DPP step inside)
  if (!__all(!act || (fx == 0 && ord))) return false;
  // 2-byte values: bit k of lb (datapoint k of the lane)
  uint32_t lb = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) lb |= (((t[i] >> 16) & 1u) << (2 * i)) | ((t[i] & 1u) << (2 * i + 1));
  const int lsum = act ? DPL + __builtin_popcount(lb) : 0;
  const int incl = wave_incl_sum_dpp(lsum);
  const int total = __builtin_amdgcn_readlane(incl, 63);
  if ((uint32_t)total > cvl) return false;   // values past the row's bytes: the general path flags the row
  __builtin_amdgcn_wave_barrier();
  stage[lane] = ld.v0;
  __builtin_amdgcn_s_waitcnt(0xC07F);        // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  // the lane's 16 value bytes from byte b: five staged dwords, funnel-shifted by b & 3
  const int b = min(incl - lsum, 1024);
  const uint32_t* sw = reinterpret_cast<const uint32_t*>(st8) + (b >> 2);
  const uint32_t sh = (uint32_t)(b & 3);
  const uint32_t d0 = sw[0], d1 = sw[1], d2 = sw[2], d3 = sw[3], d4 = sw[4];
  uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh), w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
  uint32_t w2 = __builtin_amdgcn_alignbyte(d3, d2, sh), w3 = __builtin_amdgcn_alignbyte(d4, d3, sh);
  int32_t mx = INT32_MIN, mn = INT32_MAX, xp = 0;
  uint32_t ox = 0, h16[4];
#pragma unroll
  for (int k = 0; k < DPL; k++) {
    const uint32_t two = (lb >> k) & 1u;
    // big-endian: one byte, or two with the first the more significant
    const int32_t x1 = (int32_t)(int8_t)(uint8_t)w0;
    const int32_t x2 = (int32_t)(int16_t)(uint16_t)__builtin_amdgcn_perm(w0, w0, 0x0C0C0001u);
    const int32_t x = two ? x2 : x1;
    ox |= (uint32_t)x;          // ctz of the OR = the least significant set bit over the values
    mx = max(mx, x);
    mn = min(mn, x);
    if (k & 1) h16[k >> 1] = __builtin_amdgcn_perm((uint32_t)x, (uint32_t)xp, 0x05040100u);   // (x << 16) | (xp & 0xFFFF)
    xp = x;
    // consume 1 or 2 bytes (the upper words only while later values can still reach them)
    const uint32_t s = 1u + two;
    w0 = __builtin_amdgcn_alignbyte(w1, w0, s);
    if (k < 6) w1 = __builtin_amdgcn_alignbyte(w2, w1, s);
    if (k < 4) w2 = __builtin_amdgcn_alignbyte(w3, w2, s);
    if (k < 2) w3 = w3 >> (8 * s);
  }
  if (val2 && act)
    *reinterpret_cast<uint4*>(val2 + cq + 16 * (uint64_t)lane) = make_uint4(h16[0], h16[1], h16[2], h16[3]);
  uint32_t imax = (uint32_t)max(mx, -mn);   // |x| <= 32768
  uint32_t lsbk = ox ? (uint32_t)__builtin_ctz(ox) : 0xFFFFFFFFu;
  if (!act) { imax = 0; lsbk = 0xFFFFFFFFu; }
  const uint32_t wmax = (uint32_t)wave_reduce_i32((int)imax, 0, [](int a, int c) { return (int)max((uint32_t)a, (uint32_t)c); });
  const uint32_t wl = (uint32_t)wave_reduce_i32((int)lsbk, -1, [](int a, int c) { return (int)min((uint32_t)a, (uint32_t)c); });
  const bool all1 = __all(!act || lb == 0), all2 = __all(!act || lb == 0xFFu);
  R.fail = false;
  R.lsb = wl == 0xFFFFFFFFu ? INT32_MAX : (int)wl;
  R.amax = (double)wmax;
  R.flags = 2u | ROW_ALLI | ROW_VLE2 | (all1 ? 1u << ROW_VL_SHIFT : all2 ? 2u << ROW_VL_SHIFT : 0u);
  return true;
}

__device__ __forceinline__ ShortRes short_row(const ShortLd& ld, uint8_t* __restrict__ val2, const uint8_t* st8,
                                              uint4* stage, uint64_t cq, uint32_t cn, uint32_t cvl, bool cu4) {
  const int nin = min(DPL, max(0, (int)cn - lane_id() * DPL));
  ShortRes R;
  if (__all(nin == 0 || nin == DPL)) {
    if (cu4 ? short_full_u4(ld, nin > 0, R) : short_full_vle(ld, val2, st8, stage, cq, cvl, nin > 0, R)) return R;
  }
  return short_row_general(ld, val2, st8, stage, cq, cn, cvl, cu4);
}

// SD: the load ring's depth (rows in flight while one decodes); 64 is a multiple of it.
// CLS: the kernel classifies every row itself (k_index_hint's rule, from the batch's descriptors
// already in its lanes) and writes every hint and class count (cnt) -- no separate hint pass.
template <int SD, bool CLS>
__global__ __launch_bounds__(256) void k_index_short(const uint8_t* __restrict__ qual, const uint8_t* __restrict__ val,
                                                     uint8_t* __restrict__ val2, RowDesc* __restrict__ rows,
                                                     uint8_t* __restrict__ hint, int64_t n_rows, uint32_t* cnt,
                                                     int32_t* err) {
  uint32_t* fails = cnt + IDX_C_FAIL;
  static_assert(64 % SD == 0, "ring depth divides the 64-row batch");
  __shared__ uint4 stage_all[4][66];   // per wave: 1 KB of value bytes + a 32-B tail
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint4* stage = stage_all[wv];
  const uint8_t* st8 = reinterpret_cast<const uint8_t*>(stage);
  if (lane < 2) stage[64 + lane] = make_uint4(0, 0, 0, 0);
  const int64_t n_tiles = (n_rows + 63) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t t = (int64_t)blockIdx.x * 4 + wv; t < n_tiles; t += nw) {
    const int64_t r = (t << 6) + lane;
    uint8_t h = (!CLS && r < n_rows) ? hint[r] : 0;
    if (!CLS && !__any(h & HINT_SHORT)) continue;
    // lane l: row l's descriptor (rows not this kernel's keep their own valid offsets: the ring
    // issues their loads too, unused, so that every slot issues the same loads)
    uint64_t qoff = 0, voff = 0;
    uint32_t qlen = 0, vlen = 0, fin = 0;
    if (r < n_rows) {
      const RowDesc& d = rows[r];
      qoff = d.qoff;
      voff = d.voff;
      qlen = d.qlen;
      vlen = d.vlen;
      fin = d.flags;
    }
    if constexpr (CLS) {   // k_index_hint's classification, and the batch's class counts
      int slot = -1;
      if (r < n_rows) {
        int cls = 0;
        bool sh = false;
        if (qlen > 0) {
          const uint32_t w = *reinterpret_cast<const uint32_t*>(qual + qoff);   // qoff is 16-B aligned
          const int qw = (w & 0xF0) == 0xF0 ? 4 : 2;
          if (qlen % qw == 0) {
            const uint32_t L = ((w >> (8 * (qw - 1))) & 7) + 1;
            const uint64_t ndp = qlen / qw;
            const bool uni = (L == 1 || L == 2 || L == 4 || L == 8) && (uint64_t)vlen == ndp * L + (ndp > 1 ? 1 : 0);
            cls = idx_cls(qw, uni ? (int)L : 0);
            sh = idx_short_ok(qw, L, ndp, vlen, uni);
          }
        }
        h = (uint8_t)(cls | (sh ? HINT_SHORT : 0));
        slot = sh ? (cls == idx_cls(2, 4) ? IDX_C_SHORT4 : IDX_C_SHORTV) : cls;
      }
      for (int c = 0; c < 16; c++) {
        const uint64_t m = __ballot(slot == c);
        if (m && lane == 0) atomicAdd(&cnt[c], (uint32_t)__popcll(m));
      }
      if (r < n_rows && !(h & HINT_SHORT)) hint[r] = h;
    }
    const bool mine = (h & HINT_SHORT) != 0;
    const uint64_t todo = __ballot(mine);
    if (CLS && !todo) continue;
    if (!mine) qlen = 0;
    const uint32_t u4m = (uint32_t)((h & 0x7F) == idx_cls(2, 4));
    uint32_t o_flags = 0, o_alo = 0, o_ahi = 0;
    int32_t o_lsb = INT32_MAX;
    auto issue = [&](int jj, ShortLd& ld) {
      const uint64_t qo = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(qoff >> 32), jj) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)qoff, jj);
      const uint64_t vo = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(voff >> 32), jj) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)voff, jj);
      short_issue(qual, val, qo, vo, (uint32_t)__builtin_amdgcn_readlane((int)qlen, jj) >> 1,
                  __builtin_amdgcn_readlane((int)u4m, jj) != 0, ld);
    };
    ShortLd buf[SD];
#pragma unroll
    for (int i = 0; i < SD; i++) issue(i, buf[i]);
    for (int j0 = 0; j0 < 64; j0 += SD) {
#pragma unroll
      for (int i = 0; i < SD; i++) {
        const int j = j0 + i;
        if ((todo >> j) & 1) {   // (wave-uniform)
          const uint64_t cq = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(qoff >> 32), j) << 32) |
                              (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)qoff, j);
          const ShortRes R = short_row(buf[i], val2, st8, stage, cq, (uint32_t)__builtin_amdgcn_readlane((int)qlen, j) >> 1,
                                       (uint32_t)__builtin_amdgcn_readlane((int)vlen, j),
                                       __builtin_amdgcn_readlane((int)u4m, j) != 0);
          // the row's (uniform) results into lane j
          const uint64_t ab = (uint64_t)__double_as_longlong(R.amax);
          const bool me = lane == j;
          o_flags = me ? (R.flags | (R.fail ? SHORT_FAIL : 0u)) : o_flags;
          o_lsb = me ? R.lsb : o_lsb;
          o_alo = me ? (uint32_t)ab : o_alo;
          o_ahi = me ? (uint32_t)(ab >> 32) : o_ahi;
        }
        issue(min(j + SD, 63), buf[i]);
      }
    }
    if (mine) {
      if (o_flags & SHORT_FAIL) {
        hint[r] = 0;   // k_index_generic takes the row
        atomicAdd(fails, 1u);
      } else {
        if (CLS) hint[r] = h;
        const double amax = __longlong_as_double((long long)(((uint64_t)o_ahi << 32) | o_alo));
        RowDesc& o = rows[r];
        o.ndp = qlen >> 1;
        o.flags = (o_flags | (fin & ROW_SFIRST)) | (row_nocert(o_lsb, amax) ? ROW_NOCERT : 0u);
        o.lsb = o_lsb;
        o.absmax = amax;
        if (o_flags & ROW_ERR) set_err(err, TSDB_E_ILLEGAL_DATA);
      }
    }
  }
}

// Rows of class 0 (hint 0), or every row (all = 1: test hook), through the sequential path.
// A wave scans 64 hints at a time and walks the rows its ballot selects.
__global__ __launch_bounds__(256) void k_index_generic(const uint8_t* __restrict__ qual, const uint8_t* __restrict__ val,
                                                       uint8_t* __restrict__ val2, RowDesc* __restrict__ rows,
                                                       const uint8_t* __restrict__ hint, int64_t n_rows, int32_t* err,
                                                       int all, const uint32_t* need) {
  // need (non-null): the count of rows handed back by k_index_short -- the only rows left to
  // this kernel when no class kernel ran and k_index_hint found none for it
  if (need && *need == 0) return;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int lane = lane_id();
  for (int64_t r0 = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 64; r0 < n_rows; r0 += nw * 64) {
    const int64_t r = r0 + lane;
    uint64_t m = __ballot(r < n_rows && (all || hint[r] == 0));
    while (m) {
      const int l = __ffsll((long long)m) - 1;
      m &= m - 1;
      index_row_generic(qual, val, val2, rows, r0 + l, err);
    }
  }
}

template <int QW, int L>
static hipError_t launch_cls(const uint8_t* qual, const uint8_t* val, uint8_t* val2, RowDesc* rows, const IndexBufs& b,
                             const uint32_t* off, const uint32_t* cnt, int32_t* err, hipStream_t s) {
  const int c = idx_cls(QW, L);
  if (!cnt[c]) return hipSuccess;
  const int64_t blocks = std::min<int64_t>(((int64_t)cnt[c] + 3) / 4, 8192);
  if (QW == 2 && L <= 2 && val2)
    hipLaunchKernelGGL((k_index_cls<QW, L, true>), dim3((unsigned)blocks), dim3(256), 0, s, qual, val, val2, rows,
                       b.hint, b.list + off[c], (int64_t)cnt[c], err);
  else
    hipLaunchKernelGGL((k_index_cls<QW, L, false>), dim3((unsigned)blocks), dim3(256), 0, s, qual, val, val2, rows,
                       b.hint, b.list + off[c], (int64_t)cnt[c], err);
  return hipGetLastError();
}

hipError_t index_classes(const uint8_t* qual, const RowDesc* rows, const IndexBufs& b, int64_t n_rows,
                         IndexClasses* out, hipStream_t s) {
  // (k_index_hint's counts: classes 0 .. IDX_NCLS - 1 for the listed rows and k_index_generic,
  // IDX_C_SHORT4 / IDX_C_SHORTV for k_index_short's rows)
  *out = IndexClasses{};
  if (n_rows == 0) return hipSuccess;
  if (n_rows > 0x7FFFFFFFLL) return hipErrorInvalidValue;   // int32 row lists
  hipError_t e;
  const unsigned tb = (unsigned)((n_rows + 255) / 256);
  if ((e = hipMemsetAsync(b.cnt, 0, 16 * 4, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_index_hint, dim3(tb), dim3(256), 0, s, qual, rows, n_rows, b.hint, b.cnt);
  uint32_t cnt[16] = {}, cur[16] = {};
  if ((e = hipMemcpyAsync(cnt, b.cnt, 16 * 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
  for (int c = 0; c < 16; c++) out->cnt[c] = cnt[c];
  for (int c = 2; c < IDX_NCLS; c++) out->off[c] = out->off[c - 1] + cnt[c - 1];
  for (int c = 1; c < IDX_NCLS; c++) out->listed += cnt[c];
  out->short_rows = cnt[IDX_C_SHORT4] + cnt[IDX_C_SHORTV];
  out->vle_capable = cnt[idx_cls(2, 0)] + cnt[idx_cls(2, 1)] + cnt[idx_cls(2, 2)] + cnt[IDX_C_SHORTV];
  if (out->listed) {   // class row lists (the cursors; k_index_short's hand-back counter at 0)
    for (int c = 0; c < 16; c++) cur[c] = out->off[c];
    if ((e = hipMemcpyAsync(b.cnt, cur, 16 * 4, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_index_scatter, dim3(tb), dim3(256), 0, s, b.hint, n_rows, b.cnt, b.list);
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;   // `cur` leaves scope
  } else if ((e = hipMemsetAsync(b.cnt + IDX_C_FAIL, 0, 4, s)) != hipSuccess) {
    return e;
  }
  return hipGetLastError();
}

// index_classes + k_index_short in one pass over the batch (val2 allocated up front): the short
// rows indexed while the rest are classified; then, only if some row is not short, the class
// row lists.  index_rows runs the rest (class kernels, k_index_generic).
hipError_t index_fused(const uint8_t* qual, const uint8_t* val, uint8_t* val2, RowDesc* rows, const IndexBufs& b,
                       int64_t n_rows, int32_t* err, IndexClasses* out, hipStream_t s) {
  *out = IndexClasses{};
  if (n_rows == 0) return hipSuccess;
  if (n_rows > 0x7FFFFFFFLL) return hipErrorInvalidValue;   // int32 row lists
  hipError_t e;
  if ((e = hipMemsetAsync(b.cnt, 0, 16 * 4, s)) != hipSuccess) return e;
  const int64_t tiles = (n_rows + 63) / 64;
  hipLaunchKernelGGL((k_index_short<IDX_SHORT_D, true>), dim3((unsigned)std::min<int64_t>((tiles + 3) / 4, IDX_SHORT_BLOCKS)),
                     dim3(256), 0, s, qual, val, val2, rows, b.hint, n_rows, b.cnt, err);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  uint32_t cnt[16] = {}, cur[16] = {};
  if ((e = hipMemcpyAsync(cnt, b.cnt, 16 * 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
  for (int c = 0; c < 16; c++) out->cnt[c] = cnt[c];
  for (int c = 2; c < IDX_NCLS; c++) out->off[c] = out->off[c - 1] + cnt[c - 1];
  for (int c = 1; c < IDX_NCLS; c++) out->listed += cnt[c];
  out->short_rows = cnt[IDX_C_SHORT4] + cnt[IDX_C_SHORTV];
  out->short_done = true;
  out->vle_capable = cnt[idx_cls(2, 0)] + cnt[idx_cls(2, 1)] + cnt[idx_cls(2, 2)] + cnt[IDX_C_SHORTV];
  if (out->listed) {   // class row lists; the hand-back counter (k_index_generic's early-out) kept
    for (int c = 0; c < 16; c++) cur[c] = out->off[c];
    cur[IDX_C_FAIL] = cnt[IDX_C_FAIL];
    if ((e = hipMemcpyAsync(b.cnt, cur, 16 * 4, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    const unsigned tb = (unsigned)((n_rows + 255) / 256);
    hipLaunchKernelGGL(k_index_scatter, dim3(tb), dim3(256), 0, s, b.hint, n_rows, b.cnt, b.list);
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;   // `cur` leaves scope
  }
  return hipGetLastError();
}

hipError_t index_rows(const uint8_t* qual, const uint8_t* val, uint8_t* val2, RowDesc* rows, const IndexBufs& b,
                      const IndexClasses& k, int64_t n_rows, int32_t* err, bool generic, hipStream_t s) {
  if (n_rows == 0) return hipSuccess;
  const int64_t gblocks = std::min<int64_t>((n_rows + 3) / 4, 16384);
  if (generic) {
    hipLaunchKernelGGL(k_index_generic, dim3((unsigned)gblocks), dim3(256), 0, s, qual, val, val2, rows, b.hint, n_rows,
                       err, 1, nullptr);
    return hipGetLastError();
  }
  hipError_t e;
  if (k.short_rows && !k.short_done) {
    const int64_t tiles = (n_rows + 63) / 64;
    hipLaunchKernelGGL((k_index_short<IDX_SHORT_D, false>), dim3((unsigned)std::min<int64_t>((tiles + 3) / 4, IDX_SHORT_BLOCKS)),
                       dim3(256), 0, s, qual, val, val2, rows, b.hint, n_rows, b.cnt, err);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
#define IDX_CLS(Q, LL) if ((e = launch_cls<Q, LL>(qual, val, val2, rows, b, k.off, k.cnt, err, s)) != hipSuccess) return e;
  IDX_CLS(2, 0) IDX_CLS(2, 1) IDX_CLS(2, 2) IDX_CLS(2, 4) IDX_CLS(2, 8)
  IDX_CLS(4, 0) IDX_CLS(4, 1) IDX_CLS(4, 2) IDX_CLS(4, 4) IDX_CLS(4, 8)
#undef IDX_CLS
  // rows of no class, or handed back by a class kernel: known only on the device when just
  // k_index_short ran (its hand-back counter); otherwise the kernel scans every hint
  const bool early_out = k.cnt[0] == 0 && k.listed == 0;
  hipLaunchKernelGGL(k_index_generic, dim3((unsigned)std::min<int64_t>(gblocks, 4096)), dim3(256), 0, s, qual, val,
                     nullptr, rows, b.hint, n_rows, err, 0, early_out ? b.cnt + IDX_C_FAIL : nullptr);
  return hipGetLastError();
}

// ---- k_recede: datapoints going back in time across a series' rows -------------------------
// Span.Iterator yields a series' rows in base-time order and each row's cells in column order;
// the downsamplers and AggregationIterator read that stream as it comes (kcommon.h "stream
// order").  A row whose first datapoint is not after every datapoint of the series' earlier rows
// (two rows of one hour, an offset past the hour in the row before) breaks the time order
// across rows as an unsorted cell does inside one, so it is flagged ROW_UNSORTED too: every
// streaming kernel hands it to the stored-order paths (k_grid's running max, k_raw_merge's
// greedy walk).  One thread a series, rows in their (sorted) order.
__device__ __forceinline__ int64_t qual_ms_at(const uint8_t* q, uint32_t pos, int qw) {
  if (qw == 4 || (qw != 2 && (q[pos] & 0xF0) == 0xF0)) {
    const uint32_t w = ((uint32_t)q[pos] << 24) | ((uint32_t)q[pos + 1] << 16) | ((uint32_t)q[pos + 2] << 8) | q[pos + 3];
    return (w & 0x0FFFFFC0u) >> 6;
  }
  return (int64_t)(((((uint32_t)q[pos] << 8) | q[pos + 1]) >> 4) & 0xFFF) * 1000;
}

__global__ __launch_bounds__(256) void k_recede(RowDesc* __restrict__ rows, const int64_t* __restrict__ srp,
                                                const uint8_t* __restrict__ qual, int64_t n_series) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_series) return;
  int64_t M = INT64_MIN;   // latest datapoint of the earlier rows
  for (int64_t r = srp[s]; r < srp[s + 1]; r++) {
    const RowDesc d = rows[r];
    if ((d.flags & ROW_ERR) || d.ndp == 0) continue;
    const uint8_t* q = qual + d.qoff;
    const int qw = d.flags & ROW_QW_MASK;
    const int64_t b = (int64_t)d.base * 1000;
    const int64_t first = b + qual_ms_at(q, 0, qw);
    int64_t mx;
    if (!(d.flags & ROW_UNSORTED) && (qw == 2 || qw == 4)) {
      mx = b + qual_ms_at(q, (d.ndp - 1) * (uint32_t)qw, qw);
    } else {   // a mixed-width row: walk to its last cell; a row out of order: its latest cell
      mx = INT64_MIN;
      uint32_t pos = 0;
      for (uint32_t i = 0; i < d.ndp && pos < d.qlen; i++) {
        const int w = qw ? qw : ((q[pos] & 0xF0) == 0xF0 ? 4 : 2);
        const int64_t t = b + qual_ms_at(q, pos, qw);
        mx = (d.flags & ROW_UNSORTED) ? max(mx, t) : t;
        pos += w;
      }
    }
    if (first <= M) rows[r].flags = d.flags | ROW_UNSORTED;
    M = max(M, mx);
  }
}

hipError_t index_recede(RowDesc* rows, const int64_t* srp, const uint8_t* qual, int64_t n_series, hipStream_t s) {
  if (n_series <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_recede, dim3((unsigned)((n_series + 255) / 256)), dim3(256), 0, s, rows, srp, qual, n_series);
  return hipGetLastError();
}

}  // namespace tsdb
