// k_misc.hip -- row index, cross-tile group reduction, synthetic store and the
// per-function dispatch of libtsdbhip (the k_grid / k_fast instantiations live in
// k_grid.hip / k_fast.hip, compiled once per downsample function).
#include "kcommon.h"

namespace tsdb {

// ---- k_index: classify every row, validate it, certificate stats ---------------------
// RowSeq's per-datapoint view (src/core/RowSeq.java:233-266, 552-614; Internal.java:621-810)
// reduced to the row facts the query kernels branch on: qualifier width, uniform value
// length, all-float / all-integer, NaN / -0.0, offset order, malformed cells, and the
// exactness certificate (least significant set bit, max |value|).
//
// index_row_fast: rows whose qualifiers all have the width of the first one (2 = seconds,
// 4 = ms).  8 datapoints per lane per 512-datapoint chunk, 16-byte loads of qualifiers and --
// while every length so far equals the first one -- of values at i * L; otherwise the
// chunk's value bytes are staged in LDS after a wave prefix sum of the lengths.  One pass.
// VAL2: the second pass over rows of the vle-integer class (2-byte qualifiers, 1-2-byte
// integers): only writes each value as a little-endian int16 at val2 + qoff + 2 i (same
// offsets as the qualifiers), the layout k_short / k_fast read.
// index_row_generic: the rest (mixed second/millisecond rows, empty rows), sequentially.
static constexpr int IDX_STAGE = 4224;   // bytes of value staging per wave: 512 x 8 B + alignment

struct IdxAcc {
  bool bad, allf, alli, vmax2, nan, negz, unsorted;
  int lsb, lmin, lmax;
  double amax;
};

// 8 bytes of the LDS stage from byte offset b (little-endian memory order)
__device__ __forceinline__ uint64_t stage_u64(const uint32_t* s, int b) {
  const int w = b >> 2, sh = (b & 3) * 8;
  const uint32_t w0 = s[w], w1 = s[w + 1], w2 = s[w + 2];
  const uint32_t lo = sh ? (w0 >> sh) | (w1 << (32 - sh)) : w0;
  const uint32_t hi = sh ? (w1 >> sh) | (w2 << (32 - sh)) : w1;
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ void idx_value(IdxAcc& a, uint64_t be, int len, bool fl) {
  double x = 0.0;
  decode_value(be, len, fl, x);
  if (isnan(x)) { a.nan = true; return; }
  if (x == 0.0 && signbit(x)) a.negz = true;
  const double ax = fabs(x);
  if (ax > a.amax || isinf(ax)) a.amax = fmax(a.amax, ax);
  if (x != 0.0 && !isinf(x)) a.lsb = min(a.lsb, lsb_exp(x));
}

// false: the width hypothesis failed (the row mixes widths); the caller takes the generic path
template <int QW, bool VAL2>
__device__ bool index_row_fast(const uint8_t* __restrict__ q, const uint8_t* __restrict__ v, uint8_t* __restrict__ v2,
                               uint32_t qlen, uint32_t vlen, uint32_t* stage, IdxAcc& a) {
  const int lane = lane_id();
  const uint32_t ndp = qlen / QW;
  const int L0 = (q[QW - 1] & 7) + 1;              // length of datapoint 0 (uniform value)
  const bool L0ok = L0 == 1 || L0 == 2 || L0 == 4 || L0 == 8;
  const int64_t vlen16 = ((int64_t)vlen + 15) & ~(int64_t)15;
  bool uni = L0ok;                                  // every length so far == L0: values at i * L0
  int64_t carry = 0;                                // value bytes before this chunk
  long long prev_off = -1;
  for (uint32_t i0 = 0; i0 < ndp; i0 += CH) {
    const int nin = (int)min((int64_t)DPL, max((int64_t)0, (int64_t)ndp - i0 - (int64_t)lane * DPL));
    uint32_t qq[DPL];
#pragma unroll
    for (int j = 0; j < DPL; j++) qq[j] = 0;
    if (nin > 0) {
      if (QW == 2) {
        const uint4 w = *reinterpret_cast<const uint4*>(q + 2 * ((int64_t)i0 + lane * DPL));
        const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int j = 0; j < DPL; j++) {
          const uint32_t be = __builtin_bswap32(ws[j >> 1]);
          qq[j] = (j & 1) ? (be & 0xFFFF) : (be >> 16);
        }
      } else {
        const uint4 w0 = *reinterpret_cast<const uint4*>(q + 4 * ((int64_t)i0 + lane * DPL));
        const uint4 w1 = *reinterpret_cast<const uint4*>(q + 4 * ((int64_t)i0 + lane * DPL) + 16);
        const uint32_t ws[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
        for (int j = 0; j < DPL; j++) qq[j] = __builtin_bswap32(ws[j]);
      }
    }
    int len[DPL];
    int lsum = 0;
    bool wbad = false, cuni = true;
    long long off[DPL];
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      const bool in = j < nin;
      if (in) wbad |= QW == 2 ? (qq[j] >> 12) == 0xF : (qq[j] >> 28) != 0xF;
      len[j] = in ? (int)(qq[j] & 7) + 1 : 0;
      lsum += len[j];
      cuni &= !in || len[j] == L0;
      off[j] = QW == 2 ? (long long)(qq[j] >> 4) * 1000 : (long long)((qq[j] & 0x0FFFFFC0u) >> 6);
    }
    if (__any(wbad)) return false;   // uniform over the wave
    uni = uni && __all(cuni);
    if (!VAL2) {
      // offsets strictly increasing (Internal.compareQualifiers order of a compacted cell)
      long long last = nin > 0 ? off[0] : -1;
#pragma unroll
      for (int j = 1; j < DPL; j++)
        if (j < nin) { a.unsorted |= off[j] <= off[j - 1]; last = off[j]; }
      long long pl = __shfl_up(last, 1, 64);
      if (lane == 0) pl = prev_off;
      if (nin > 0 && off[0] <= pl) a.unsorted = true;
      const int lastl = (int)((min((int64_t)CH, (int64_t)ndp - i0) - 1) / DPL);
      prev_off = __shfl(last, lastl, 64);
#pragma unroll
      for (int j = 0; j < DPL; j++) {
        if (j < nin) {
          const bool fl = (qq[j] & 8) != 0;
          a.allf &= fl;
          a.alli &= !fl;
          a.vmax2 &= len[j] <= 2;
          a.lmin = min(a.lmin, len[j]);
          a.lmax = max(a.lmax, len[j]);
          a.bad |= fl ? (len[j] != 4 && len[j] != 8) : (len[j] == 3 || (len[j] >= 5 && len[j] <= 7));
        }
      }
    }
    // value bytes of the lane's datapoints
    uint64_t be[DPL];
#pragma unroll
    for (int j = 0; j < DPL; j++) be[j] = 0;
    int64_t total;
    int64_t vo;          // byte offset (in the row's values) of the lane's first value
    if (uni) {
      total = (int64_t)min((int64_t)CH, (int64_t)ndp - i0) * L0;
      vo = carry + (int64_t)lane * DPL * L0;
      if (nin > 0 && vo + (int64_t)nin * L0 <= (int64_t)vlen) {
        const uint8_t* p = v + vo;
        if (L0 == 1) {
          const uint2 t = *reinterpret_cast<const uint2*>(p);
#pragma unroll
          for (int j = 0; j < DPL; j++) be[j] = ((j < 4 ? t.x : t.y) >> ((j & 3) * 8)) & 0xFF;
        } else if (L0 == 2) {
          const uint4 t = *reinterpret_cast<const uint4*>(p);
          const uint32_t ws[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
          for (int j = 0; j < DPL; j++) {
            const uint32_t b = __builtin_bswap32(ws[j >> 1]);
            be[j] = (j & 1) ? (b & 0xFFFF) : (b >> 16);
          }
        } else if (L0 == 4) {
          const uint4 t0 = *reinterpret_cast<const uint4*>(p);
          const uint4 t1 = *reinterpret_cast<const uint4*>(p + 16);
          const uint32_t ws[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
#pragma unroll
          for (int j = 0; j < DPL; j++) be[j] = __builtin_bswap32(ws[j]);
        } else {
          const uint4 t0 = *reinterpret_cast<const uint4*>(p);
          const uint4 t1 = *reinterpret_cast<const uint4*>(p + 16);
          const uint4 t2 = *reinterpret_cast<const uint4*>(p + 32);
          const uint4 t3 = *reinterpret_cast<const uint4*>(p + 48);
          const uint32_t ws[16] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w,
                                   t2.x, t2.y, t2.z, t2.w, t3.x, t3.y, t3.z, t3.w};
#pragma unroll
          for (int j = 0; j < DPL; j++)
            be[j] = ((uint64_t)__builtin_bswap32(ws[2 * j]) << 32) | __builtin_bswap32(ws[2 * j + 1]);
        }
      }
    } else {
      // variable lengths: wave prefix sum, the chunk's value bytes staged in LDS
      const int incl = wave_incl_sum_dpp(lsum);
      total = __builtin_amdgcn_readlane(incl, 63);
      const int64_t a0 = carry & ~(int64_t)15;
      const int lead = (int)(carry - a0);
      vo = carry + incl - lsum;
      const int64_t nst = min((int64_t)(lead + total + 15) & ~(int64_t)15, vlen16 - a0);   // never past the row
      WAVE_SYNC();
      for (int64_t o = (int64_t)lane * 16; o < nst; o += 64 * 16)
        *reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(stage) + o) = *reinterpret_cast<const uint4*>(v + a0 + o);
      WAVE_SYNC();
      int b = lead + incl - lsum;
#pragma unroll
      for (int j = 0; j < DPL; j++) {
        be[j] = 0;
        if (j < nin && b + len[j] <= nst) be[j] = __builtin_bswap64(stage_u64(stage, b)) >> (64 - 8 * len[j]);
        b += len[j];
      }
    }
    // decode
    if (VAL2) {
      if (nin > 0) {
        uint32_t h[4] = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < DPL; j++) {
          const int16_t x = len[j] == 1 ? (int16_t)(int8_t)(uint8_t)be[j] : (int16_t)(uint16_t)be[j];
          h[j >> 1] |= (uint32_t)(uint16_t)x << ((j & 1) * 16);
        }
        *reinterpret_cast<uint4*>(v2 + 2 * ((int64_t)i0 + lane * DPL)) = make_uint4(h[0], h[1], h[2], h[3]);
      }
    } else {
      int64_t o = vo;
#pragma unroll
      for (int j = 0; j < DPL; j++) {
        if (j < nin && o + len[j] <= (int64_t)vlen) idx_value(a, be[j], len[j], (qq[j] & 8) != 0);
        o += len[j];
      }
    }
    carry += total;
  }
  if (!VAL2 && carry > (int64_t)vlen) a.bad = true;
  return true;
}

__device__ void index_row_generic(const uint8_t* __restrict__ qual, const uint8_t* __restrict__ val,
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
      d.ndp = ndp;
      d.flags = flags;
      d.lsb = lsbmin;
      d.absmax = amax;
      rows[r] = d;
    }
  }
}

template <bool VAL2>
__global__ __launch_bounds__(256) void k_index(const uint8_t* __restrict__ qual, const uint8_t* __restrict__ val,
                                               uint8_t* __restrict__ val2, RowDesc* __restrict__ rows, int64_t n_rows,
                                               int32_t* err, int generic) {
  __shared__ uint32_t stage_all[4][IDX_STAGE / 4];
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* stage = stage_all[wv];
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = (int64_t)blockIdx.x * 4 + wv; r < n_rows; r += nwaves) {
    const RowDesc d = rows[r];
    const uint8_t* q = qual + d.qoff;
    const uint8_t* v = val + d.voff;
    if (VAL2) {
      // rows of the vle-integer class only (flags from the first pass)
      if ((d.flags & (ROW_QW_MASK | ROW_ALLI | ROW_VLE2 | ROW_ERR)) != (2u | ROW_ALLI | ROW_VLE2)) continue;
      IdxAcc a{};
      index_row_fast<2, true>(q, v, val2 + d.qoff, d.qlen, d.vlen, stage, a);
      continue;
    }
    IdxAcc a;
    a.bad = false; a.allf = a.alli = a.vmax2 = true; a.nan = a.negz = a.unsorted = false;
    a.lsb = INT32_MAX; a.lmin = 99; a.lmax = -1; a.amax = 0.0;
    const int qw = d.qlen == 0 ? 0 : ((q[0] & 0xF0) == 0xF0 ? 4 : 2);
    bool ok = false;
    if (generic) {}   // test hook: every row through the sequential path
    else if (qw == 2 && d.qlen % 2 == 0) ok = index_row_fast<2, false>(q, v, nullptr, d.qlen, d.vlen, stage, a);
    else if (qw == 4 && d.qlen % 4 == 0) ok = index_row_fast<4, false>(q, v, nullptr, d.qlen, d.vlen, stage, a);
    if (!ok) {
      index_row_generic(qual, val, val2, rows, r, err);   // val2: the generic test hook's second pass
      continue;
    }
    const bool bad = __any(a.bad);
    const bool allf = __all(a.allf), alli = __all(a.alli), vmax2 = __all(a.vmax2);
    const bool hasnan = __any(a.nan), negz = __any(a.negz), unsorted = __any(a.unsorted);
    const int lsbmin = wave_min(a.lsb), lmin = wave_min(a.lmin), lmax = wave_max(a.lmax);
    double amax = a.amax;
#pragma unroll
    for (int dd = 32; dd >= 1; dd >>= 1) amax = fmax(amax, __shfl_xor(amax, dd, 64));
    if (lane == 0) {
      RowDesc o = d;
      uint32_t flags = (uint32_t)qw;
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
      flags |= d.flags & ROW_SFIRST;
      o.ndp = d.qlen / qw;
      o.flags = flags;
      o.lsb = lsbmin;
      o.absmax = amax;
      rows[r] = o;
    }
  }
}

__global__ __launch_bounds__(256) void k_reduce(ReduceParams p) {
  __shared__ PState sh[4][64];
  const int lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform (scalar) tile index
  const int64_t g = blockIdx.x;
  const int64_t k = (int64_t)blockIdx.y * 64 + lane;
  const int64_t t0 = p.group_tile_ptr[g], t1 = p.group_tile_ptr[g + 1];
  const int64_t n = t1 - t0;
  const int64_t a = t0 + n * wave / 4, b = t0 + n * (wave + 1) / 4;
  PState S = ps_identity(p.ga);
  if (k < p.K) {
    for (int64_t t = a; t < b; t++) {
      PState X;
      const int64_t idx = t * p.K + k;
      X.a = p.part.a[idx];
      X.b = p.part.b[idx];
      X.n = p.part.n[idx];
      X.f = p.part.f[idx];
      S = ps_merge(p.ga, S, X);
    }
  }
  sh[wave][lane] = S;
  __syncthreads();
  if (wave == 0 && k < p.K) {
    PState T = sh[0][lane];
    for (int w = 1; w < 4; w++) T = ps_merge(p.ga, T, sh[w][lane]);
    const int64_t o = g * p.K + k;
    if (p.state.a) {
      p.state.a[o] = T.a;
      p.state.b[o] = T.b;
      p.state.n[o] = T.n;
      p.state.f[o] = T.f;
    } else {
      const bool emit = (T.f & PF_UNION) != 0;
      const double r = emit ? ps_final(p.ga, T, p.err, !p.no_inf) : 0.0;
      p.out_val[o] = r;
      p.out_flag[o] = emit ? 1 : 0;
    }
  }
}

// ---- k_rank_merge: multi-GPU exchange step ------------------------------------------
// Rank r holds series shard r of the group-sorted span order, so merging the gathered
// per-rank states in rank order continues ps_merge's series order across GPUs.
__global__ __launch_bounds__(256) void k_rank_merge(RankMergeParams p) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = p.G * p.K;
  if (i < n) {
    PState S = ps_identity(p.ga);
    for (int r = 0; r < p.n_ranks; r++) {
      const unsigned char* b = p.base + (int64_t)r * p.stride;
      PState X;
      X.a = reinterpret_cast<const double*>(b)[i];
      X.b = reinterpret_cast<const double*>(b + p.off_b)[i];
      X.n = reinterpret_cast<const uint32_t*>(b + p.off_n)[i];
      X.f = reinterpret_cast<const uint32_t*>(b + p.off_f)[i];
      S = ps_merge(p.ga, S, X);
    }
    const bool emit = (S.f & PF_UNION) != 0;
    p.out_val[i] = emit ? ps_final(p.ga, S, p.err) : 0.0;
    p.out_flag[i] = emit ? 1 : 0;
  }
  if (i < p.G) {
    uint32_t act = 0;
    for (int r = 0; r < p.n_ranks; r++)
      act |= reinterpret_cast<const uint32_t*>(p.base + (int64_t)r * p.stride + p.off_act)[i];
    p.out_act[i] = act;
  }
}

// ---- synthetic MockBase-equivalent store, generated in HBM -------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

__device__ __forceinline__ void synth_series(const SynthParams& p, int64_t pos, int64_t& gsid, int32_t& grp) {
  // batch position -> (group, global series id): series i belongs to group i % G
  int64_t lo = 0, hi = p.n_groups;
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (p.grp_off[mid] <= pos) lo = mid; else hi = mid;
  }
  grp = (int32_t)lo;
  gsid = lo + (pos - p.grp_off[lo]) * p.n_groups;
}

// value of point k of global series i: (is_int, long, float)
__device__ __forceinline__ void synth_value(const SynthParams& p, int64_t i, int64_t k, bool& is_int, int64_t& lv,
                                            float& fv) {
  const uint64_t u = splitmix64(p.seed ^ ((uint64_t)i << 32) ^ (uint64_t)k);
  is_int = p.value_kind == 1 || (p.value_kind == 2 && (i % 2) == 0);
  if (is_int) {
    lv = (int64_t)(u % (uint64_t)p.int_mod);
  } else {
    const double d = (double)(u >> 11) * (1.0 / 9007199254740992.0);
    fv = (float)(50.0 + 10.0 * (d - 0.5));
  }
}

__device__ __forceinline__ int vle_len(int64_t v) {
  if (v >= -128 && v <= 127) return 1;
  if (v >= -32768 && v <= 32767) return 2;
  if (v >= -2147483648LL && v <= 2147483647LL) return 4;
  return 8;
}

// pass 1: value bytes per row (wave per row)
__global__ __launch_bounds__(256) void k_synth_sizes(SynthParams p) {
  const int lane = lane_id();
  const int64_t R = p.n_rows_per_series;
  const int64_t nr = p.n_series * R;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t row = wave; row < nr; row += nwaves) {
    const int64_t pos = row / R, h = row % R;
    int64_t i;
    int32_t grp;
    synth_series(p, pos, i, grp);
    const int64_t k0 = p.row_k0[h];
    const int n = p.row_n[h];
    long long bytes = 0;
    for (int t = lane; t < n; t += 64) {
      bool isi; int64_t lv; float fv;
      synth_value(p, i, k0 + t, isi, lv, fv);
      bytes += isi ? vle_len(lv) : 4;
    }
    bytes = wave_sum64(bytes);
    if (lane == 0) p.row_vbytes[row] = (uint32_t)(bytes + (n > 1 ? 1 : 0));
  }
}

// pass 2: write qualifiers, values, meta byte and the row index (wave per row)
__global__ __launch_bounds__(256) void k_synth_write(SynthParams p) {
  const int lane = lane_id();
  const int64_t R = p.n_rows_per_series;
  const int64_t nr = p.n_series * R;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t row = wave; row < nr; row += nwaves) {
    const int64_t pos = row / R, h = row % R;
    int64_t i;
    int32_t grp;
    synth_series(p, pos, i, grp);
    if (h == 0 && lane == 0) p.group_id[pos] = grp;
    RowDesc d = p.rows[row];   // qoff / voff / qlen / vlen set by the host
    const int64_t k0 = p.row_k0[h];
    const int n = p.row_n[h];
    uint8_t* q = p.qual + d.qoff;
    uint8_t* v = p.val + d.voff;
    const int64_t base_ms = (int64_t)p.row_base[h] * 1000;
    int64_t vo_carry = 0;
    for (int t0 = 0; t0 < n; t0 += 64) {
      const int t = t0 + lane;
      bool isi = false; int64_t lv = 0; float fv = 0.f;
      int len = 0;
      if (t < n) {
        synth_value(p, i, k0 + t, isi, lv, fv);
        len = isi ? vle_len(lv) : 4;
      }
      const int incl = wave_incl_sum(len);
      const int64_t vo = vo_carry + incl - len;
      vo_carry += __shfl(incl, 63, 64);
      if (t < n) {
        const int64_t ts = p.start_ms + (k0 + t) * p.period_ms;
        const int64_t off = ts - base_ms;
        const uint32_t flags = isi ? (uint32_t)(len - 1) : 0xBu;
        if (p.ms_qual) {
          const uint32_t qq = 0xF0000000u | ((uint32_t)off << 6) | flags;
          q[t * 4 + 0] = qq >> 24; q[t * 4 + 1] = (qq >> 16) & 0xFF; q[t * 4 + 2] = (qq >> 8) & 0xFF; q[t * 4 + 3] = qq & 0xFF;
        } else {
          const uint32_t qq = ((uint32_t)(off / 1000) << 4) | flags;
          q[t * 2 + 0] = (qq >> 8) & 0xFF; q[t * 2 + 1] = qq & 0xFF;
        }
        uint64_t be;
        if (isi) be = (uint64_t)lv; else be = __float_as_uint(fv);
        for (int b = 0; b < len; b++) v[vo + b] = (uint8_t)(be >> (8 * (len - 1 - b)));
      }
    }
    if (lane == 0 && n > 1) v[vo_carry] = 0;   // CompactionQueue meta byte (no s/ms mix)
  }
}

// ---- launchers -------------------------------------------------------------------
hipError_t launch_index(const uint8_t* qual, const uint8_t* val, uint8_t* val2, RowDesc* rows, int64_t n_rows,
                        int32_t* err, hipStream_t s, bool generic) {
  if (n_rows == 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((n_rows + 3) / 4, 65536);
  if (val2 && !generic) hipLaunchKernelGGL(k_index<true>, dim3((unsigned)blocks), dim3(256), 0, s, qual, val, val2, rows, n_rows, err, 0);
  else hipLaunchKernelGGL(k_index<false>, dim3((unsigned)blocks), dim3(256), 0, s, qual, val, val2, rows, n_rows, err,
                          generic ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_grid(const GridParams& p, int f, hipStream_t s) {
  if (p.n_tiles == 0) return hipSuccess;
  switch (f) {
    case F_SUM: return launch_grid_inst<F_SUM>(p, s);
    case F_AVG: return launch_grid_inst<F_AVG>(p, s);
    case F_COUNT: return launch_grid_inst<F_COUNT>(p, s);
    case F_SQUARESUM: return launch_grid_inst<F_SQUARESUM>(p, s);
    case F_MIN: return launch_grid_inst<F_MIN>(p, s);
    case F_MAX: return launch_grid_inst<F_MAX>(p, s);
    case F_DEV: return launch_grid_inst<F_DEV>(p, s);
    case F_FIRST: return launch_grid_inst<F_FIRST>(p, s);
    case F_LAST: return launch_grid_inst<F_LAST>(p, s);
    case F_DIFF: return launch_grid_inst<F_DIFF>(p, s);
    case F_MULT: return launch_grid_inst<F_MULT>(p, s);
  }
  return hipErrorInvalidValue;
}

bool fast_supported(int f, int qw, int vl) {
  return (f == F_SUM || f == F_AVG || f == F_COUNT || f == F_SQUARESUM || f == F_MIN || f == F_MAX) &&
         (((qw == 2 || qw == 4) && (vl == 4 || vl == 8)) || (qw == 2 && vl == 0));
}

hipError_t launch_fast(const GridParams& p, int f, int qw, int vl, hipStream_t s) {
  if (p.n_tiles == 0) return hipSuccess;
  switch (f) {
    case F_SUM: return launch_fast_inst<F_SUM>(p, qw, vl, s);
    case F_AVG: return launch_fast_inst<F_AVG>(p, qw, vl, s);
    case F_COUNT: return launch_fast_inst<F_COUNT>(p, qw, vl, s);
    case F_SQUARESUM: return launch_fast_inst<F_SQUARESUM>(p, qw, vl, s);
    case F_MIN: return launch_fast_inst<F_MIN>(p, qw, vl, s);
    case F_MAX: return launch_fast_inst<F_MAX>(p, qw, vl, s);
  }
  return hipErrorNotSupported;
}

int64_t fast_wave_lds(int64_t K, bool rate) { return align16(1024 + fast_slot_bytes(K, rate)); }   // + VL==0 value stage

int64_t grid_wave_lds(int64_t K, bool rate, bool gslot) {
  return align16(fixed_lds_bytes() + (gslot ? 0 : slot_lds_bytes(K, rate)));
}

hipError_t launch_reduce(const ReduceParams& p, hipStream_t s) {
  if (p.G == 0 || p.K == 0) return hipSuccess;
  hipLaunchKernelGGL(k_reduce, dim3((unsigned)p.G, (unsigned)((p.K + 63) / 64)), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_rank_merge(const RankMergeParams& p, hipStream_t s) {
  const int64_t n = std::max(p.G * p.K, p.G);
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rank_merge, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_synth_sizes(const SynthParams& p, hipStream_t s) {
  const int64_t nr = p.n_series * p.n_rows_per_series;
  const int64_t blocks = std::min<int64_t>((nr + 3) / 4, 1 << 16);
  hipLaunchKernelGGL(k_synth_sizes, dim3((unsigned)blocks), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_synth_write(const SynthParams& p, hipStream_t s) {
  const int64_t nr = p.n_series * p.n_rows_per_series;
  const int64_t blocks = std::min<int64_t>((nr + 3) / 4, 1 << 16);
  hipLaunchKernelGGL(k_synth_write, dim3((unsigned)blocks), dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace tsdb
