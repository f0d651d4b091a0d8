// k_misc.hip -- cross-tile group reduction, synthetic store and the
// per-function dispatch of libtsdbhip (the k_grid / k_fast instantiations live in
// k_grid.hip / k_fast.hip, compiled once per downsample function).
#include "kcommon.h"
#include <cstdlib>

namespace tsdb {

// values of datapoints i0 .. i0 + 7 of a uniform row (value length vl; fl: the qualifier flags)
__device__ __forceinline__ void seq_values(const uint8_t* vb, int64_t i0, int vl, const uint32_t fl[DPL], double val[DPL]) {
  if (vl == 8) {
    const uint4* v = reinterpret_cast<const uint4*>(vb + i0 * 8);
    const uint4 a0 = v[0], a1 = v[1], a2 = v[2], a3 = v[3];
    const uint32_t ws[16] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w,
                             a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      const uint64_t b = ((uint64_t)__builtin_bswap32(ws[2 * j]) << 32) | __builtin_bswap32(ws[2 * j + 1]);
      val[j] = (fl[j] & 8) ? __longlong_as_double((long long)b) : (double)(long long)b;
    }
  } else if (vl == 4) {
    const uint4* v = reinterpret_cast<const uint4*>(vb + i0 * 4);
    const uint4 a0 = v[0], a1 = v[1];
    const uint32_t ws[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      const uint32_t be = __builtin_bswap32(ws[j]);
      val[j] = (fl[j] & 8) ? (double)__uint_as_float(be) : (double)(int32_t)be;
    }
  } else if (vl == 2) {
    const uint4 a0 = *reinterpret_cast<const uint4*>(vb + i0 * 2);
    const uint32_t ws[4] = {a0.x, a0.y, a0.z, a0.w};
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      const uint32_t be = __builtin_bswap32(ws[j >> 1]);
      val[j] = (double)(int16_t)(uint16_t)((j & 1) ? (be & 0xFFFF) : (be >> 16));
    }
  } else {
    const uint2 a0 = *reinterpret_cast<const uint2*>(vb + i0);
    const uint32_t ws[2] = {a0.x, a0.y};
#pragma unroll
    for (int j = 0; j < DPL; j++) val[j] = (double)(int8_t)((ws[j >> 2] >> ((j & 3) * 8)) & 0xFF);
  }
}

// values of datapoints i0 .. i0 + 3 (i0 a multiple of 4) of a uniform row: seq_values' decode
// in half the registers (the rollup pair walk, one hour row a thread)
__device__ __forceinline__ void seq_values4(const uint8_t* vb, int64_t i0, int vl, const uint32_t fl[4], double val[4],
                                            bool ints) {
  if (vl == 8) {
    const uint4* v = reinterpret_cast<const uint4*>(vb + i0 * 8);
    const uint4 a0 = v[0], a1 = v[1];
    const uint32_t ws[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint64_t b = ((uint64_t)__builtin_bswap32(ws[2 * j]) << 32) | __builtin_bswap32(ws[2 * j + 1]);
      val[j] = (!ints && (fl[j] & 8)) ? __longlong_as_double((long long)b) : (double)(long long)b;
    }
  } else if (vl == 4) {
    const uint4 a0 = *reinterpret_cast<const uint4*>(vb + i0 * 4);
    const uint32_t ws[4] = {a0.x, a0.y, a0.z, a0.w};
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t be = __builtin_bswap32(ws[j]);
      val[j] = (!ints && (fl[j] & 8)) ? (double)__uint_as_float(be) : (double)(int32_t)be;
    }
  } else if (vl == 2) {
    const uint2 a0 = *reinterpret_cast<const uint2*>(vb + i0 * 2);
    const uint32_t ws[2] = {a0.x, a0.y};
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t be = __builtin_bswap32(ws[j >> 1]);
      val[j] = (double)(int16_t)(uint16_t)((j & 1) ? (be & 0xFFFF) : (be >> 16));
    }
  } else {
    const uint32_t w = *reinterpret_cast<const uint32_t*>(vb + i0);
#pragma unroll
    for (int j = 0; j < 4; j++) val[j] = (double)(int8_t)((w >> (j * 8)) & 0xFF);
  }
}

// ---- k_seq_dense: Java's bucket order, one series per thread -------------------------
// Sum / avg downsampling of rows whose values cannot add exactly in any order (ROW_NOCERT):
// each thread walks its series' uniform rows in stored order, adding every bucket's values one
// after the other as Downsampler.ValuesInInterval hands them to runDouble, and writes the
// bucket values to [series][K] (pre_dense / pre_pres) for the group-by step (k_emit).  Uniform
// rows: 16-byte loads of qualifiers and values, eight datapoints decoded per step; other rows
// datapoint by datapoint.
template <int F>
__global__ __launch_bounds__(256) void k_seq_dense(GridParams p, double* __restrict__ dense, uint8_t* __restrict__ pres,
                                                   int64_t n_series) {
  int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_series) return;
  if (p.tile_list) {   // the series k_seq_rows handed back
    if (s >= (int64_t)*p.tile_list_n) return;
    s = p.tile_list[s];
  }
  const int64_t K = p.K;
  BState st;
  bs_init<F>(st);
  int cur = -1;
  auto flush = [&]() {
    if (cur >= 0) {
      dense[s * K + cur] = bs_final<F>(st);
      pres[s * K + cur] = 1;
    }
  };
  for (int64_t r = p.series_row_ptr[s]; r < p.series_row_ptr[s + 1]; r++) {
    const RowDesc d = p.rows[r];
    if ((int64_t)d.base < p.ss) continue;
    if ((int64_t)d.base >= p.se) break;
    if (d.flags & ROW_ERR) { set_err(p.err, TSDB_E_ILLEGAL_DATA); continue; }
    const int qw = d.flags & ROW_QW_MASK;
    const int vl = (d.flags & ROW_VL_MASK) >> ROW_VL_SHIFT;
    const RowGeom g = row_geom(p, d.base);
    const uint8_t* qb = p.qual + d.qoff;
    const uint8_t* vb = p.val + d.voff;
    if (!((qw == 2 || qw == 4) && (vl == 1 || vl == 2 || vl == 4 || vl == 8))) {
      // mixed qualifier widths or variable value lengths: datapoint by datapoint
      // (RowSeq.Iterator: the width from the qualifier's first byte, the length from its flags)
      uint64_t qi = 0, vi = 0;
      for (uint32_t j = 0; j < d.ndp; j++) {
        uint32_t off, fl;
        if ((qb[qi] & 0xF0) == 0xF0) {
          const uint32_t qq = ((uint32_t)qb[qi] << 24) | ((uint32_t)qb[qi + 1] << 16) | ((uint32_t)qb[qi + 2] << 8) | qb[qi + 3];
          off = (qq & 0x0FFFFFC0u) >> 6;
          fl = qq & 0xF;
          qi += 4;
        } else {
          const uint32_t qq = ((uint32_t)qb[qi] << 8) | qb[qi + 1];
          off = (qq >> 4) * 1000u;
          fl = qq & 0xF;
          qi += 2;
        }
        const int len = (int)(fl & 7) + 1;
        uint64_t be = 0;
        for (int t = 0; t < len; t++) be = (be << 8) | vb[vi + t];
        vi += len;
        double x;
        if (fl & 8) x = len == 4 ? (double)__uint_as_float((uint32_t)be) : __longlong_as_double((long long)be);
        else x = (double)((long long)(be << (64 - 8 * len)) >> (64 - 8 * len));
        const int k = slot_of(p, g, d.base, off);
        if (k < 0) continue;
        if (k != cur) {
          flush();
          bs_init<F>(st);
          cur = k;
        }
        bs_add<F>(st, x);
      }
      continue;
    }
    for (int64_t i0 = 0; i0 < (int64_t)d.ndp; i0 += DPL) {
      const int nv = (int)min((int64_t)DPL, (int64_t)d.ndp - i0);
      uint32_t off[DPL], fl[DPL];
      if (qw == 2) {
        const uint4 q = *reinterpret_cast<const uint4*>(qb + i0 * 2);
        const uint32_t ws[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int j = 0; j < DPL; j++) {
          const uint32_t be = __builtin_bswap32(ws[j >> 1]);
          const uint32_t qq = (j & 1) ? (be & 0xFFFF) : (be >> 16);
          off[j] = (qq >> 4) * 1000u;
          fl[j] = qq & 0xF;
        }
      } else {
        const uint4 q0 = *reinterpret_cast<const uint4*>(qb + i0 * 4);
        const uint4 q1 = *reinterpret_cast<const uint4*>(qb + i0 * 4 + 16);
        const uint32_t ws[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
        for (int j = 0; j < DPL; j++) {
          const uint32_t qq = __builtin_bswap32(ws[j]);
          off[j] = (qq & 0x0FFFFFC0u) >> 6;
          fl[j] = qq & 0xF;
        }
      }
      double val[DPL];
      seq_values(vb, i0, vl, fl, val);
#pragma unroll
      for (int j = 0; j < DPL; j++) {
        if (j >= nv) break;
        const int k = slot_of(p, g, d.base, off[j]);
        if (k < 0) continue;
        if (k != cur) {
          flush();
          bs_init<F>(st);
          cur = k;
        }
        bs_add<F>(st, val[j]);
      }
    }
  }
  flush();
}

// The same sums with one WAVE per series (K <= 64): a row's datapoints are loaded by the whole
// wave in 512-point chunks (lane l: points 8l .. 8l + 7, so the 16-byte loads of neighbouring
// lanes are neighbouring bytes) and staged in LDS with their slots; lane b then folds bucket
// b's values in stored order.  Slots never decrease along a sorted series, so a bucket's values
// in a chunk are one run [start, end), found by the lanes that own its edges.  k_seq_dense's
// one-series-per-lane walk reads 16 bytes of a different line per lane and instruction (1M
// rollup rows: 3.9 ms).  Rows of mixed widths are decoded by lane 0, in order, into the same stage.
constexpr int SEQW_DP = 512;
constexpr int SEQW_WAVES = 4;
template <int F>
__global__ __launch_bounds__(64 * SEQW_WAVES) void k_seq_wave(GridParams p, double* __restrict__ dense,
                                                             uint8_t* __restrict__ pres, int64_t n_series) {
  __shared__ double sval[SEQW_WAVES][SEQW_DP];
  __shared__ int32_t sslot[SEQW_WAVES][SEQW_DP];
  __shared__ int32_t srun[SEQW_WAVES][2][64];
  const int wv = threadIdx.x >> 6;
  const int lane = lane_id();
  const int64_t s = (int64_t)blockIdx.x * SEQW_WAVES + wv;
  if (s >= n_series) return;   // whole waves leave; no block barrier follows
  const int K = (int)p.K;      // <= 64 (host-checked)
  double* V = sval[wv];
  int32_t* S = sslot[wv];
  int32_t* RS = srun[wv][0];
  int32_t* RE = srun[wv][1];
  BState st;
  bs_init<F>(st);
  bool has = false;
  for (int64_t r = p.series_row_ptr[s]; r < p.series_row_ptr[s + 1]; r++) {
    const RowDesc d = p.rows[r];
    if ((int64_t)d.base < p.ss) continue;
    if ((int64_t)d.base >= p.se) break;
    if (d.flags & ROW_ERR) { if (lane == 0) set_err(p.err, TSDB_E_ILLEGAL_DATA); continue; }
    const int qw = d.flags & ROW_QW_MASK;
    const int vl = (d.flags & ROW_VL_MASK) >> ROW_VL_SHIFT;
    const bool uni = (qw == 2 || qw == 4) && (vl == 1 || vl == 2 || vl == 4 || vl == 8);
    const RowGeom g = row_geom(p, d.base);
    const uint8_t* qb = p.qual + d.qoff;
    const uint8_t* vb = p.val + d.voff;
    const int64_t ndp = d.ndp;
    uint64_t qi = 0, vi = 0;   // lane 0's cursor through a row of mixed widths
    for (int64_t c0 = 0; c0 < ndp; c0 += SEQW_DP) {
      const int n = (int)min((int64_t)SEQW_DP, ndp - c0);
      if (uni) {
        const int64_t i0 = c0 + (int64_t)lane * DPL;
        if (lane * DPL < n) {
          uint32_t off[DPL], fl[DPL];
          if (qw == 2) {
            const uint4 q = *reinterpret_cast<const uint4*>(qb + i0 * 2);
            const uint32_t ws[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int j = 0; j < DPL; j++) {
              const uint32_t be = __builtin_bswap32(ws[j >> 1]);
              const uint32_t qq = (j & 1) ? (be & 0xFFFF) : (be >> 16);
              off[j] = (qq >> 4) * 1000u;
              fl[j] = qq & 0xF;
            }
          } else {
            const uint4 q0 = *reinterpret_cast<const uint4*>(qb + i0 * 4);
            const uint4 q1 = *reinterpret_cast<const uint4*>(qb + i0 * 4 + 16);
            const uint32_t ws[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
            for (int j = 0; j < DPL; j++) {
              const uint32_t qq = __builtin_bswap32(ws[j]);
              off[j] = (qq & 0x0FFFFFC0u) >> 6;
              fl[j] = qq & 0xF;
            }
          }
          double val[DPL];
          if (vl == 8) {
            const uint4* v = reinterpret_cast<const uint4*>(vb + i0 * 8);
            const uint4 a0 = v[0], a1 = v[1], a2 = v[2], a3 = v[3];
            const uint32_t ws[16] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w,
                                     a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
#pragma unroll
            for (int j = 0; j < DPL; j++) {
              const uint64_t b = ((uint64_t)__builtin_bswap32(ws[2 * j]) << 32) | __builtin_bswap32(ws[2 * j + 1]);
              val[j] = (fl[j] & 8) ? __longlong_as_double((long long)b) : (double)(long long)b;
            }
          } else if (vl == 4) {
            const uint4* v = reinterpret_cast<const uint4*>(vb + i0 * 4);
            const uint4 a0 = v[0], a1 = v[1];
            const uint32_t ws[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
            for (int j = 0; j < DPL; j++) {
              const uint32_t be = __builtin_bswap32(ws[j]);
              val[j] = (fl[j] & 8) ? (double)__uint_as_float(be) : (double)(int32_t)be;
            }
          } else if (vl == 2) {
            const uint4 a0 = *reinterpret_cast<const uint4*>(vb + i0 * 2);
            const uint32_t ws[4] = {a0.x, a0.y, a0.z, a0.w};
#pragma unroll
            for (int j = 0; j < DPL; j++) {
              const uint32_t be = __builtin_bswap32(ws[j >> 1]);
              val[j] = (double)(int16_t)(uint16_t)((j & 1) ? (be & 0xFFFF) : (be >> 16));
            }
          } else {
            const uint2 a0 = *reinterpret_cast<const uint2*>(vb + i0);
            const uint32_t ws[2] = {a0.x, a0.y};
#pragma unroll
            for (int j = 0; j < DPL; j++) val[j] = (double)(int8_t)((ws[j >> 2] >> ((j & 3) * 8)) & 0xFF);
          }
#pragma unroll
          for (int j = 0; j < DPL; j++) {
            const int i = lane * DPL + j;
            if (i < n) {
              V[i] = val[j];
              S[i] = slot_of(p, g, d.base, off[j]);
            }
          }
        }
      } else if (lane == 0) {
        // RowSeq.Iterator: the width from the qualifier's first byte, the length from its flags
        for (int i = 0; i < n; i++) {
          uint32_t off, fl;
          if ((qb[qi] & 0xF0) == 0xF0) {
            const uint32_t qq = ((uint32_t)qb[qi] << 24) | ((uint32_t)qb[qi + 1] << 16) | ((uint32_t)qb[qi + 2] << 8) | qb[qi + 3];
            off = (qq & 0x0FFFFFC0u) >> 6;
            fl = qq & 0xF;
            qi += 4;
          } else {
            const uint32_t qq = ((uint32_t)qb[qi] << 8) | qb[qi + 1];
            off = (qq >> 4) * 1000u;
            fl = qq & 0xF;
            qi += 2;
          }
          const int len = (int)(fl & 7) + 1;
          uint64_t be = 0;
          for (int t = 0; t < len; t++) be = (be << 8) | vb[vi + t];
          vi += len;
          double x;
          if (fl & 8) x = len == 4 ? (double)__uint_as_float((uint32_t)be) : __longlong_as_double((long long)be);
          else x = (double)((long long)(be << (64 - 8 * len)) >> (64 - 8 * len));
          V[i] = x;
          S[i] = slot_of(p, g, d.base, off);
        }
      }
      RS[lane] = -1;
      WAVE_SYNC();
      // the run of each slot in this chunk: its first and one-past-last point
      for (int i = lane; i < n; i += 64) {
        const int k = S[i];
        if (k < 0) continue;
        if (i == 0 || S[i - 1] != k) RS[k] = i;
        if (i == n - 1 || S[i + 1] != k) RE[k] = i + 1;
      }
      WAVE_SYNC();
      if (lane < K && RS[lane] >= 0) {
        for (int i = RS[lane]; i < RE[lane]; i++) bs_add<F>(st, V[i]);
        has = true;
      }
      WAVE_SYNC();
    }
  }
  if (lane < K && has) {
    dense[s * K + lane] = bs_final<F>(st);
    pres[s * K + lane] = 1;
  }
}

// ---- k_seq_rows: Java's bucket order, one row per thread ---------------------------------
// When the interval divides one hour and slot 0 is interval-aligned, a bucket of an hour row
// holds only that row's datapoints -- unless the row starts off the hour, reaches past it
// (2-byte qualifiers go to 4095 s), repeats the previous row's base (two cells of one hour),
// or is not uniform / sorted.  Each row is then its own sequential walk: the thread adds its
// buckets' values in stored order (ValuesInInterval -> runDouble) and writes them to
// [series][K].  Neighbouring threads read neighbouring descriptors and cells, and write
// neighbouring buckets, where k_seq_dense's one-series-a-thread walk reads one row after the
// other (rollup tables read as hour rows: 24 rows of a few cells a series).  A row that breaks
// the premise hands its series back (redo_list, once per series: redo_mark), and k_seq_dense
// recomputes those series whole afterwards, overwriting every bucket they hold.
template <int F>
__global__ __launch_bounds__(256) void k_seq_rows(GridParams p, double* __restrict__ dense, uint8_t* __restrict__ pres,
                                                  int64_t n_rows) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  const RowDesc d = p.rows[r];
  if ((int64_t)d.base < p.ss || (int64_t)d.base >= p.se) return;
  const int64_t s = p.row_series[r];
  const int qw = d.flags & ROW_QW_MASK;
  const int vl = (d.flags & ROW_VL_MASK) >> ROW_VL_SHIFT;
  bool back = (d.flags & (ROW_ERR | ROW_UNSORTED)) || (d.base % 3600u) != 0 ||
              !((qw == 2 || qw == 4) && (vl == 1 || vl == 2 || vl == 4 || vl == 8));
  // two cells of one hour: the previous row of the series has the same base (ROW_SFIRST: none)
  if (!back && r > 0 && !(d.flags & ROW_SFIRST) && p.rows[r - 1].base == d.base) back = true;
  if (back) {
    if (atomicExch(&p.redo_mark[s], 1u) == 0u) p.redo_list[atomicAdd(p.redo_n, 1)] = (int32_t)s;
    return;
  }
  const int64_t K = p.K;
  // slot of the row base without a 64-bit division: rel and I are exact doubles, the quotient
  // is corrected to the exact one
  RowGeom g;
  {
    const int64_t rel = (int64_t)d.base * 1000 - p.B0;
    if (rel >= 0) {
      int64_t q0 = (int64_t)((double)rel / (double)p.I);
      int64_t r0 = rel - q0 * p.I;
      if (r0 < 0) { q0--; r0 += p.I; }
      if (r0 >= p.I) { q0++; r0 -= p.I; }
      g.q0 = q0;
      g.r0 = r0;
    } else {
      g.q0 = 0;
      g.r0 = rel;
    }
  }
  const uint8_t* qb = p.qual + d.qoff;
  const uint8_t* vb = p.val + d.voff;
  BState st;
  bs_init<F>(st);
  int cur = -1;
  for (int64_t i0 = 0; i0 < (int64_t)d.ndp; i0 += DPL) {
    const int nv = (int)min((int64_t)DPL, (int64_t)d.ndp - i0);
    uint32_t off[DPL], fl[DPL];
    if (qw == 2) {
      const uint4 q = *reinterpret_cast<const uint4*>(qb + i0 * 2);
      const uint32_t ws[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int j = 0; j < DPL; j++) {
        const uint32_t be = __builtin_bswap32(ws[j >> 1]);
        const uint32_t qq = (j & 1) ? (be & 0xFFFF) : (be >> 16);
        off[j] = (qq >> 4) * 1000u;
        fl[j] = qq & 0xF;
      }
    } else {
      const uint4 q0 = *reinterpret_cast<const uint4*>(qb + i0 * 4);
      const uint4 q1 = *reinterpret_cast<const uint4*>(qb + i0 * 4 + 16);
      const uint32_t ws[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
      for (int j = 0; j < DPL; j++) {
        const uint32_t qq = __builtin_bswap32(ws[j]);
        off[j] = (qq & 0x0FFFFFC0u) >> 6;
        fl[j] = qq & 0xF;
      }
    }
    double val[DPL];
    seq_values(vb, i0, vl, fl, val);
    // a datapoint past the row's hour (2-byte qualifiers reach 4095 s): its bucket takes the next
    // row's datapoints too, so the series goes to k_seq_dense, which rewrites every bucket of it
    // (the ones this row wrote already included)
    bool past = false;
#pragma unroll
    for (int j = 0; j < DPL; j++) past = past || (j < nv && off[j] >= 3600000u);
    if (past) {
      if (atomicExch(&p.redo_mark[s], 1u) == 0u) p.redo_list[atomicAdd(p.redo_n, 1)] = (int32_t)s;
      return;
    }
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      if (j >= nv) break;
      const int k = slot_of(p, g, d.base, off[j]);
      if (k < 0) continue;
      if (k != cur) {
        if (cur >= 0) {
          dense[s * K + cur] = bs_final<F>(st);
          pres[s * K + cur] = 1;
        }
        bs_init<F>(st);
        cur = k;
      }
      bs_add<F>(st, val[j]);
    }
  }
  if (cur >= 0) {
    dense[s * K + cur] = bs_final<F>(st);
    pres[s * K + cur] = 1;
  }
}

hipError_t launch_seq_rows(const GridParams& p, int f, double* dense, uint8_t* pres, int64_t n_rows, hipStream_t s) {
  if (n_rows <= 0) return hipSuccess;
  const unsigned nb = (unsigned)((n_rows + 255) / 256);
#define SEQR_CASE(FF)                                                                          \
  case FF:                                                                                     \
    hipLaunchKernelGGL(k_seq_rows<FF>, dim3(nb), dim3(256), 0, s, p, dense, pres, n_rows);     \
    break;
  switch (f) {
    SEQR_CASE(F_SUM) SEQR_CASE(F_AVG) SEQR_CASE(F_COUNT) SEQR_CASE(F_SQUARESUM) SEQR_CASE(F_MIN) SEQR_CASE(F_MAX)
    SEQR_CASE(F_DEV) SEQR_CASE(F_FIRST) SEQR_CASE(F_LAST) SEQR_CASE(F_DIFF) SEQR_CASE(F_MULT)
    default: return hipErrorInvalidValue;
  }
#undef SEQR_CASE
  return hipGetLastError();
}

// ---- k_seq_rows_ro: rollup avg / count downsampling, a value row with its count row ------
// A rollup batch with count cells holds, for every value series, a count series whose hour rows
// the load wrote in lock step with the value rows (tsdbhip_load_rollup: same bases, same
// offsets).  With k_seq_rows' premise (buckets inside hour rows), one thread takes a value row
// and its count row: Σsum in Java's order (the SUM downsampler over the value cells), Σcount
// (exact integer sums), and writes the bucket as k_rollup_combine would: Σsum / Σcount (0 when
// Σcount is 0) for avg, Σcount for count.  No thread for the count rows, no combine pass.  A row
// pair that breaks a premise (k_seq_rows' checks, rows out of lock step, a count row that is not
// uniform integers) hands both series to k_seq_dense, and k_rollup_combine_list combines them.
template <int AVG>
__global__ __launch_bounds__(256) void k_seq_rows_ro(GridParams p, double* __restrict__ dense, uint8_t* __restrict__ pres,
                                                     const int64_t* __restrict__ cmap, int64_t n_rows) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  const int32_t rc = p.ro_partner[r];   // the count row (loaded beside the series and descriptor)
  const int64_t s = p.row_series[r];
  if (rc == -1) return;                 // a count row: its value row takes it
  const RowDesc d = p.rows[r];
  if ((int64_t)d.base < p.ss || (int64_t)d.base >= p.se) return;
  const int qw = d.flags & ROW_QW_MASK;
  const int vl = (d.flags & ROW_VL_MASK) >> ROW_VL_SHIFT;
  auto hand_back = [&]() {
    if (atomicExch(&p.redo_mark[s], 1u) == 0u) {
      const int32_t at = atomicAdd(p.redo_n, 2);
      p.redo_list[at] = (int32_t)s;
      p.redo_list[at + 1] = (int32_t)cmap[s];
    }
  };
  bool back = rc < 0 || (d.flags & (ROW_ERR | ROW_UNSORTED)) || (d.base % 3600u) != 0 ||
              !((qw == 2 || qw == 4) && (vl == 1 || vl == 2 || vl == 4 || vl == 8));
  if (!back && r > 0 && !(d.flags & ROW_SFIRST) && p.rows[r - 1].base == d.base) back = true;
  RowDesc dc{};
  if (!back) dc = p.rows[rc];
  const int qwc = dc.flags & ROW_QW_MASK;
  const int vlc = (dc.flags & ROW_VL_MASK) >> ROW_VL_SHIFT;
  if (!back && (dc.base != d.base || dc.ndp != d.ndp || (dc.flags & (ROW_ERR | ROW_UNSORTED)) || !(dc.flags & ROW_ALLI) ||
                qwc != 2 || !(vlc == 1 || vlc == 2 || vlc == 4 || vlc == 8)))
    back = true;
  if (back) {
    hand_back();
    return;
  }
  const int64_t K = p.K;
  RowGeom g;
  {
    const int64_t rel = (int64_t)d.base * 1000 - p.B0;
    if (rel >= 0) {
      int64_t q0 = (int64_t)((double)rel / (double)p.I);
      int64_t r0 = rel - q0 * p.I;
      if (r0 < 0) { q0--; r0 += p.I; }
      if (r0 >= p.I) { q0++; r0 -= p.I; }
      g.q0 = q0;
      g.r0 = r0;
    } else {
      g.q0 = 0;
      g.r0 = rel;
    }
  }
  const uint8_t* qb = p.qual + d.qoff;
  const uint8_t* vb = p.val + d.voff;
  const uint8_t* vbc = p.val + dc.voff;
  BState sv, sc;
  bs_init<F_SUM>(sv);
  bs_init<F_SUM>(sc);
  int cur = -1;
  auto flush = [&]() {
    if (cur < 0) return;
    const double sum = bs_final<F_SUM>(sv), count = bs_final<F_SUM>(sc);
    dense[s * K + cur] = AVG ? (count == 0.0 ? 0.0 : sum / count) : count;
    pres[s * K + cur] = 1;
  };
  const uint32_t fl_int[DPL] = {0, 0, 0, 0, 0, 0, 0, 0};   // count cells: integers
  for (int64_t i0 = 0; i0 < (int64_t)d.ndp; i0 += DPL) {
    const int nv = (int)min((int64_t)DPL, (int64_t)d.ndp - i0);
    uint32_t off[DPL], fl[DPL];
    if (qw == 2) {
      const uint4 q = *reinterpret_cast<const uint4*>(qb + i0 * 2);
      const uint32_t ws[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int j = 0; j < DPL; j++) {
        const uint32_t be = __builtin_bswap32(ws[j >> 1]);
        const uint32_t qq = (j & 1) ? (be & 0xFFFF) : (be >> 16);
        off[j] = (qq >> 4) * 1000u;
        fl[j] = qq & 0xF;
      }
    } else {
      const uint4 q0 = *reinterpret_cast<const uint4*>(qb + i0 * 4);
      const uint4 q1 = *reinterpret_cast<const uint4*>(qb + i0 * 4 + 16);
      const uint32_t ws[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
      for (int j = 0; j < DPL; j++) {
        const uint32_t qq = __builtin_bswap32(ws[j]);
        off[j] = (qq & 0x0FFFFFC0u) >> 6;
        fl[j] = qq & 0xF;
      }
    }
    bool past = false;
#pragma unroll
    for (int j = 0; j < DPL; j++) past = past || (j < nv && off[j] >= 3600000u);
    if (past) {
      hand_back();
      return;
    }
    double val[DPL], cnt[DPL];
    seq_values(vb, i0, vl, fl, val);
    seq_values(vbc, i0, vlc, fl_int, cnt);
#pragma unroll
    for (int j = 0; j < DPL; j++) {
      if (j >= nv) break;
      const int k = slot_of(p, g, d.base, off[j]);
      if (k < 0) continue;
      if (k != cur) {
        flush();
        bs_init<F_SUM>(sv);
        bs_init<F_SUM>(sc);
        cur = k;
      }
      bs_add<F_SUM>(sv, val[j]);
      bs_add<F_SUM>(sc, cnt[j]);
    }
  }
  flush();
}

// ---- k_ro_pack / k_ro_pairs: k_seq_rows_ro over packed row pairs ------------------------
// A rollup table read as hour rows is mostly row metadata: 6 cells an hour row (10m rollups),
// and k_seq_rows_ro reads two 48-B descriptors, the partner and the series for every value row
// and a thread's worth of lookups for every count row (1M series x 1 d: 2.3 GB of descriptors
// for 1.9 GB of cells).  At load, k_ro_pack evaluates k_seq_rows_ro's query-independent
// premises once per value row (row class, hour-aligned base, no second row of the hour, a count
// row in lock step, no offset past the hour) and packs what the walk needs into 24 B
// (RoPair); k_ro_pairs then walks the pairs as k_seq_rows_ro walks the rows -- same buckets,
// same order, same hand-back -- and only the scan range is tested per query.
__global__ __launch_bounds__(256) void k_ro_pack(const RowDesc* __restrict__ rows, const int32_t* __restrict__ partner,
                                                 const int32_t* __restrict__ vrows, const int32_t* __restrict__ vser,
                                                 const uint8_t* __restrict__ qual, int64_t n, RoPair* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = vrows[i];
  const int32_t rc = partner ? partner[r] : -2;   // (a table without count cells: value rows alone)
  const RowDesc d = rows[r];
  const int qw = d.flags & ROW_QW_MASK;
  const int vl = (d.flags & ROW_VL_MASK) >> ROW_VL_SHIFT;
  // vok: k_seq_rows' premises for the value row alone; ok: k_seq_rows_ro's for the pair
  bool vok = !(d.flags & (ROW_ERR | ROW_UNSORTED)) && (d.base % 3600u) == 0 && (qw == 2 || qw == 4) &&
             (vl == 1 || vl == 2 || vl == 4 || vl == 8) && d.ndp < 65536 && d.qoff < (1ULL << 32) && d.voff < (1ULL << 32);
  if (vok && r > 0 && !(d.flags & ROW_SFIRST) && rows[r - 1].base == d.base) vok = false;   // two rows of one hour
  if (vok) {   // an offset past the hour (2-byte qualifiers reach 4095 s): the walk hands the series back
    const uint8_t* q = qual + d.qoff;
    for (uint32_t j = 0; j < d.ndp && vok; j++) {
      uint32_t off;
      if (qw == 2) off = ((((uint32_t)q[2 * j] << 8) | q[2 * j + 1]) >> 4) * 1000u;
      else off = ((((uint32_t)q[4 * j] << 24) | ((uint32_t)q[4 * j + 1] << 16) | ((uint32_t)q[4 * j + 2] << 8) | q[4 * j + 3]) &
                  0x0FFFFFC0u) >> 6;
      if (off >= 3600000u) vok = false;
    }
  }
  bool ok = vok && rc >= 0;
  RowDesc dc{};
  if (ok) dc = rows[rc];
  const int vlc = (dc.flags & ROW_VL_MASK) >> ROW_VL_SHIFT;
  if (ok && (dc.base != d.base || dc.ndp != d.ndp || (dc.flags & (ROW_ERR | ROW_UNSORTED)) || !(dc.flags & ROW_ALLI) ||
             (dc.flags & ROW_QW_MASK) != 2 || !(vlc == 1 || vlc == 2 || vlc == 4 || vlc == 8) || dc.voff >= (1ULL << 32)))
    ok = false;
  auto lg = [](int v) { return v == 1 ? 0u : v == 2 ? 1u : v == 4 ? 2u : 3u; };
  RoPair o;
  o.base = d.base;
  o.qoff = (uint32_t)d.qoff;
  o.voff = (uint32_t)d.voff;
  o.cvoff = (uint32_t)dc.voff;
  o.meta = (d.ndp & 0xFFFFu) | (lg(vl) << 16) | (lg(vlc) << 18) | (qw == 4 ? 1u << 20 : 0u) | (ok ? RP_OK : 0u) |
           (vok ? RP_VOK : 0u);
  o.series = vser[i];
  out[i] = o;
}

hipError_t launch_ro_pack(const RowDesc* rows, const int32_t* partner, const int32_t* vrows, const int32_t* vser,
                          const uint8_t* qual, int64_t n, RoPair* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_ro_pack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, rows, partner, vrows, vser, qual, n,
                     out);
  return hipGetLastError();
}

template <int AVG>
__device__ __forceinline__ void ro_pair(const GridParams& p, double* __restrict__ dense, uint8_t* __restrict__ pres,
                                        const int64_t* __restrict__ cmap, const RoPair& P) {
  if ((int64_t)P.base < p.ss || (int64_t)P.base >= p.se) return;
  const int64_t s = P.series;
  if (!(P.meta & RP_OK)) {   // as k_seq_rows_ro: both series to k_seq_dense, then k_rollup_combine_list
    if (atomicExch(&p.redo_mark[s], 1u) == 0u) {
      const int32_t at = atomicAdd(p.redo_n, 2);
      p.redo_list[at] = (int32_t)s;
      p.redo_list[at + 1] = (int32_t)cmap[s];
    }
    return;
  }
  const int ndp = (int)(P.meta & 0xFFFFu);
  const int vl = 1 << ((P.meta >> 16) & 3), vlc = 1 << ((P.meta >> 18) & 3);
  const bool q4 = (P.meta >> 20) & 1;
  const int64_t K = p.K;
  RowGeom g;
  {
    const int64_t rel = (int64_t)P.base * 1000 - p.B0;
    if (rel >= 0) {
      int64_t q0 = (int64_t)((double)rel / (double)p.I);
      int64_t r0 = rel - q0 * p.I;
      if (r0 < 0) { q0--; r0 += p.I; }
      if (r0 >= p.I) { q0++; r0 -= p.I; }
      g.q0 = q0;
      g.r0 = r0;
    } else {
      g.q0 = 0;
      g.r0 = rel;
    }
  }
  const uint8_t* qb = p.qual + P.qoff;
  const uint8_t* vb = p.val + P.voff;
  const uint8_t* vbc = p.val + P.cvoff;
  BState sv, sc;
  bs_init<F_SUM>(sv);
  bs_init<F_SUM>(sc);
  int cur = -1;
  auto flush = [&]() {
    if (cur < 0) return;
    const double sum = bs_final<F_SUM>(sv), count = bs_final<F_SUM>(sc);
    dense[s * K + cur] = AVG ? (count == 0.0 ? 0.0 : sum / count) : count;
    pres[s * K + cur] = 1;
  };
  // four datapoints a step (seq_values4): half the registers of an 8-point step, so more waves a
  // SIMD hide the row loads (an hour row of 10m cells is 6 points)
  for (int64_t i0 = 0; i0 < (int64_t)ndp; i0 += 4) {
    const int nv = (int)min((int64_t)4, (int64_t)ndp - i0);
    uint32_t off[4], fl[4];
    if (!q4) {
      const uint2 q = *reinterpret_cast<const uint2*>(qb + i0 * 2);
      const uint32_t ws[2] = {q.x, q.y};
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t be = __builtin_bswap32(ws[j >> 1]);
        const uint32_t qq = (j & 1) ? (be & 0xFFFF) : (be >> 16);
        off[j] = (qq >> 4) * 1000u;
        fl[j] = qq & 0xF;
      }
    } else {
      const uint4 q0 = *reinterpret_cast<const uint4*>(qb + i0 * 4);
      const uint32_t ws[4] = {q0.x, q0.y, q0.z, q0.w};
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t qq = __builtin_bswap32(ws[j]);
        off[j] = (qq & 0x0FFFFFC0u) >> 6;
        fl[j] = qq & 0xF;
      }
    }
    double val[4], cnt[4];
    seq_values4(vb, i0, vl, fl, val, false);
    seq_values4(vbc, i0, vlc, fl, cnt, true);   // (count cells: integers)
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (j >= nv) break;
      const int k = slot_of(p, g, P.base, off[j]);
      if (k < 0) continue;
      if (k != cur) {
        flush();
        bs_init<F_SUM>(sv);
        bs_init<F_SUM>(sc);
        cur = k;
      }
      bs_add<F_SUM>(sv, val[j]);
      bs_add<F_SUM>(sc, cnt[j]);
    }
  }
  flush();
}

// pair i: from the packed table, or (RUN) from its run
template <bool RUN>
__device__ __forceinline__ RoPair ro_get(const GridParams& p, int64_t i) {
  if (RUN) return ro_run_pair(p.ro_runs[p.ro_rid[i]], (uint32_t)i);
  return p.ro_pairs[i];
}

template <int AVG, bool RUN>
__global__ __launch_bounds__(256) void k_ro_pairs(GridParams p, double* __restrict__ dense, uint8_t* __restrict__ pres,
                                                  const int64_t* __restrict__ cmap, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  ro_pair<AVG>(p, dense, pres, cmap, ro_get<RUN>(p, i));
}

// k_seq_rows over a rollup batch's packed value rows (sum / min / max ... downsampling reads the
// value series alone): the pair table's value fields, RP_VOK for k_seq_rows' premises.
template <int F, bool RUN>
__global__ __launch_bounds__(256) void k_ro_rows(GridParams p, double* __restrict__ dense, uint8_t* __restrict__ pres,
                                                 int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const RoPair P = ro_get<RUN>(p, i);
  if ((int64_t)P.base < p.ss || (int64_t)P.base >= p.se) return;
  const int64_t s = P.series;
  if (!(P.meta & RP_VOK)) {
    if (atomicExch(&p.redo_mark[s], 1u) == 0u) p.redo_list[atomicAdd(p.redo_n, 1)] = (int32_t)s;
    return;
  }
  const int ndp = (int)(P.meta & 0xFFFFu);
  const int vl = 1 << ((P.meta >> 16) & 3);
  const bool q4 = (P.meta >> 20) & 1;
  const int64_t K = p.K;
  RowGeom g;
  {
    const int64_t rel = (int64_t)P.base * 1000 - p.B0;
    if (rel >= 0) {
      int64_t q0 = (int64_t)((double)rel / (double)p.I);
      int64_t r0 = rel - q0 * p.I;
      if (r0 < 0) { q0--; r0 += p.I; }
      if (r0 >= p.I) { q0++; r0 -= p.I; }
      g.q0 = q0;
      g.r0 = r0;
    } else {
      g.q0 = 0;
      g.r0 = rel;
    }
  }
  const uint8_t* qb = p.qual + P.qoff;
  const uint8_t* vb = p.val + P.voff;
  BState st;
  bs_init<F>(st);
  int cur = -1;
  for (int64_t i0 = 0; i0 < (int64_t)ndp; i0 += 4) {   // four datapoints a step (as k_ro_pairs)
    const int nv = (int)min((int64_t)4, (int64_t)ndp - i0);
    uint32_t off[4], fl[4];
    if (!q4) {
      const uint2 q = *reinterpret_cast<const uint2*>(qb + i0 * 2);
      const uint32_t ws[2] = {q.x, q.y};
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t be = __builtin_bswap32(ws[j >> 1]);
        const uint32_t qq = (j & 1) ? (be & 0xFFFF) : (be >> 16);
        off[j] = (qq >> 4) * 1000u;
        fl[j] = qq & 0xF;
      }
    } else {
      const uint4 q0 = *reinterpret_cast<const uint4*>(qb + i0 * 4);
      const uint32_t ws[4] = {q0.x, q0.y, q0.z, q0.w};
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t qq = __builtin_bswap32(ws[j]);
        off[j] = (qq & 0x0FFFFFC0u) >> 6;
        fl[j] = qq & 0xF;
      }
    }
    double val[4];
    seq_values4(vb, i0, vl, fl, val, false);
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (j >= nv) break;
      const int k = slot_of(p, g, P.base, off[j]);
      if (k < 0) continue;
      if (k != cur) {
        if (cur >= 0) {
          dense[s * K + cur] = bs_final<F>(st);
          pres[s * K + cur] = 1;
        }
        bs_init<F>(st);
        cur = k;
      }
      bs_add<F>(st, val[j]);
    }
  }
  if (cur >= 0) {
    dense[s * K + cur] = bs_final<F>(st);
    pres[s * K + cur] = 1;
  }
}

hipError_t launch_ro_rows(const GridParams& p, int f, double* dense, uint8_t* pres, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const unsigned nb = (unsigned)((n + 255) / 256);
#define RORO_CASE(FF)                                                                      \
  case FF:                                                                                 \
    if (p.ro_runs) hipLaunchKernelGGL((k_ro_rows<FF, true>), dim3(nb), dim3(256), 0, s, p, dense, pres, n); \
    else hipLaunchKernelGGL((k_ro_rows<FF, false>), dim3(nb), dim3(256), 0, s, p, dense, pres, n);         \
    break;
  switch (f) {
    RORO_CASE(F_SUM) RORO_CASE(F_AVG) RORO_CASE(F_COUNT) RORO_CASE(F_SQUARESUM) RORO_CASE(F_MIN) RORO_CASE(F_MAX)
    RORO_CASE(F_DEV) RORO_CASE(F_FIRST) RORO_CASE(F_LAST) RORO_CASE(F_DIFF) RORO_CASE(F_MULT)
    default: return hipErrorInvalidValue;
  }
#undef RORO_CASE
  return hipGetLastError();
}

hipError_t launch_ro_pairs(const GridParams& p, int avg, double* dense, uint8_t* pres, const int64_t* cmap, int64_t n,
                           hipStream_t s) {
  if (n <= 0) return hipSuccess;
  // (2 or 4 pairs a thread, every descriptor loaded first, measured no faster: profiles/r05au)
  const unsigned nb = (unsigned)((n + 255) / 256);
  if (p.ro_runs) {
    if (avg) hipLaunchKernelGGL((k_ro_pairs<1, true>), dim3(nb), dim3(256), 0, s, p, dense, pres, cmap, n);
    else hipLaunchKernelGGL((k_ro_pairs<0, true>), dim3(nb), dim3(256), 0, s, p, dense, pres, cmap, n);
  } else {
    if (avg) hipLaunchKernelGGL((k_ro_pairs<1, false>), dim3(nb), dim3(256), 0, s, p, dense, pres, cmap, n);
    else hipLaunchKernelGGL((k_ro_pairs<0, false>), dim3(nb), dim3(256), 0, s, p, dense, pres, cmap, n);
  }
  return hipGetLastError();
}

// k_rollup_combine over the listed series (the ones k_seq_rows_ro handed back; count series in
// the list have no count map entry and are skipped)
__global__ __launch_bounds__(256) void k_rollup_combine_list(double* __restrict__ dense, const uint8_t* __restrict__ pres,
                                                             const int64_t* __restrict__ cmap, const int32_t* __restrict__ list,
                                                             const int32_t* __restrict__ list_n, int64_t K, int avg) {
  const int64_t n = *list_n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n * K; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = list[i / K];
    const int64_t cs = cmap[s];
    const int64_t k = i % K;
    if (cs < 0 || !pres[s * K + k]) continue;
    const double sum = dense[s * K + k];
    const double count = pres[cs * K + k] ? dense[cs * K + k] : 0.0;
    dense[s * K + k] = avg ? (count == 0.0 ? 0.0 : sum / count) : count;
  }
}

hipError_t launch_seq_rows_ro(const GridParams& p, int avg, double* dense, uint8_t* pres, const int64_t* cmap, int64_t n_rows,
                              hipStream_t s) {
  if (n_rows <= 0) return hipSuccess;
  const unsigned nb = (unsigned)((n_rows + 255) / 256);
  if (avg) hipLaunchKernelGGL(k_seq_rows_ro<1>, dim3(nb), dim3(256), 0, s, p, dense, pres, cmap, n_rows);
  else hipLaunchKernelGGL(k_seq_rows_ro<0>, dim3(nb), dim3(256), 0, s, p, dense, pres, cmap, n_rows);
  return hipGetLastError();
}

hipError_t launch_rollup_combine_list(double* dense, const uint8_t* pres, const int64_t* cmap, const int32_t* list,
                                      const int32_t* list_n, int64_t n_max, int64_t K, int avg, hipStream_t s) {
  if (n_max * K <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((n_max * K + 255) / 256, 2048);
  hipLaunchKernelGGL(k_rollup_combine_list, dim3((unsigned)blocks), dim3(256), 0, s, dense, pres, cmap, list, list_n, K, avg);
  return hipGetLastError();
}

hipError_t launch_seq_dense(const GridParams& p, int f, double* dense, uint8_t* pres, int64_t n_series, hipStream_t s,
                            bool uniform) {
  if (n_series <= 0) return hipSuccess;
  const unsigned nb = (unsigned)((n_series + 255) / 256);
  // (option SEQ_WAVE = 0: one series per lane) uniform rows of 64+ points on average only (engine.cpp seq_dense_wanted): a row of mixed
  // widths is decoded by one lane, and short rows leave the wave waiting on each row's descriptor
  const bool wave = uniform && p.K <= 64 && !opt_off(OPT_SEQ_WAVE);
  const unsigned nw = (unsigned)((n_series + SEQW_WAVES - 1) / SEQW_WAVES);
#define SEQ_CASE(FF)                                                                                          \
  case FF:                                                                                                    \
    if (wave) hipLaunchKernelGGL(k_seq_wave<FF>, dim3(nw), dim3(64 * SEQW_WAVES), 0, s, p, dense, pres, n_series); \
    else hipLaunchKernelGGL(k_seq_dense<FF>, dim3(nb), dim3(256), 0, s, p, dense, pres, n_series);           \
    break;
  switch (f) {
    SEQ_CASE(F_SUM) SEQ_CASE(F_AVG) SEQ_CASE(F_COUNT) SEQ_CASE(F_SQUARESUM) SEQ_CASE(F_MIN) SEQ_CASE(F_MAX)
    SEQ_CASE(F_DEV) SEQ_CASE(F_FIRST) SEQ_CASE(F_LAST) SEQ_CASE(F_DIFF) SEQ_CASE(F_MULT)
    default: return hipErrorInvalidValue;
  }
#undef SEQ_CASE
  return hipGetLastError();
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

// Owner merge of a group that straddles devices (multi.cpp): thread k folds the later devices'
// states of slot k into the owner's, in device order (= SpanGroup order).
__global__ __launch_bounds__(256) void k_state_fold(StateFoldParams p) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned char* b = p.state;
  if (k < p.K) {
    const int64_t i = p.g * p.K + k;
    PState S;
    S.a = reinterpret_cast<const double*>(b)[i];
    S.b = reinterpret_cast<const double*>(b + p.off_b)[i];
    S.n = reinterpret_cast<const uint32_t*>(b + p.off_n)[i];
    S.f = reinterpret_cast<const uint32_t*>(b + p.off_f)[i];
    for (int m = 0; m < p.n_mini; m++) {
      const unsigned char* x = p.mini + (int64_t)m * p.mini_stride;
      PState X;
      X.a = reinterpret_cast<const double*>(x)[k];
      X.b = reinterpret_cast<const double*>(x + 8 * p.K)[k];
      X.n = reinterpret_cast<const uint32_t*>(x + 16 * p.K)[k];
      X.f = reinterpret_cast<const uint32_t*>(x + 20 * p.K)[k];
      S = ps_merge(p.ga, S, X);
    }
    reinterpret_cast<double*>(b)[i] = S.a;
    reinterpret_cast<double*>(b + p.off_b)[i] = S.b;
    reinterpret_cast<uint32_t*>(b + p.off_n)[i] = S.n;
    reinterpret_cast<uint32_t*>(b + p.off_f)[i] = S.f;
  }
  if (k == 0) {
    uint32_t act = reinterpret_cast<const uint32_t*>(b + p.off_act)[p.g];
    for (int m = 0; m < p.n_mini; m++)
      act |= reinterpret_cast<const uint32_t*>(p.mini + (int64_t)m * p.mini_stride + 24 * p.K)[0];
    reinterpret_cast<uint32_t*>(b + p.off_act)[p.g] = act;
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
    synth_series(p, p.pos0 + pos, i, grp);   // global batch position of the shard's series
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
    synth_series(p, p.pos0 + pos, i, grp);
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

// ---- k_first_ts: each series' first datapoint at or after a seek point -------------------
// The general calendar plan (engine.cpp) anchors every span's Downsampler at
// previousInterval(first datapoint after the seek, src/core/Downsampler.java:336-350), so it
// needs that datapoint per series: rows with base in [ss, se), in order, qualifiers walked
// (2-byte second or 4-byte millisecond, Internal.java:621-810) until the first timestamp >= t0.
// One thread per series; INT64_MAX when the series has none.  Span.seekRow passes over a row
// whose last cell is before t0 (Span.java:360-380): for a row out of order (ROW_UNSORTED) that
// is not the last of the scan, its first cell at or past t0 does not count.
__global__ void k_first_ts(const RowDesc* __restrict__ rows, const int64_t* __restrict__ srp,
                           const uint8_t* __restrict__ qual, int64_t n, int64_t ss, int64_t se, int64_t t0,
                           int64_t* __restrict__ out) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  int64_t res = INT64_MAX;
  for (int64_t r = srp[s]; r < srp[s + 1] && res == INT64_MAX; r++) {
    const RowDesc d = rows[r];
    if ((int64_t)d.base < ss || (int64_t)d.base >= se) continue;
    if ((int64_t)d.base * 1000 + 4194304 <= t0) continue;   // every offset is < 2^22 ms
    const bool last_row = r + 1 >= srp[s + 1] || (int64_t)rows[r + 1].base >= se;
    const bool whole = (d.flags & ROW_UNSORTED) && !last_row;   // the last cell decides
    int64_t first = INT64_MAX, last = INT64_MIN;
    const uint8_t* q = qual + d.qoff;
    uint32_t pos = 0;
    for (uint32_t i = 0; i < d.ndp && pos < d.qlen; i++) {
      int64_t off;
      if ((q[pos] & 0xF0) == 0xF0) {
        const uint32_t w = ((uint32_t)q[pos] << 24) | ((uint32_t)q[pos + 1] << 16) | ((uint32_t)q[pos + 2] << 8) | q[pos + 3];
        off = (w & 0x0FFFFFC0u) >> 6;
        pos += 4;
      } else {
        off = (int64_t)((((uint32_t)q[pos] << 8) | q[pos + 1]) >> 4) * 1000;
        pos += 2;
      }
      const int64_t ts = (int64_t)d.base * 1000 + off;
      last = ts;
      if (ts >= t0 && first == INT64_MAX) {
        first = ts;
        if (!whole) break;
      }
    }
    if (!whole || last >= t0) res = first;
  }
  out[s] = res;
}

hipError_t launch_first_ts(const RowDesc* rows, const int64_t* srp, const uint8_t* qual, int64_t n, int64_t ss,
                           int64_t se, int64_t t0, int64_t* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_first_ts, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, rows, srp, qual, n, ss, se, t0, out);
  return hipGetLastError();
}

// The no-value pattern over a [series][K] contribution buffer before the downsampling pass
// writes the rows it has (GBs for the percentile / ordered group-by): 16-byte non-temporal
// stores from a grid sized to the chip (hipMemsetD32 reached 2.8 TB/s on config 3's 4.8 GB).
__global__ __launch_bounds__(256) void k_fill64(uint64_t* p, uint64_t v, int64_t n) {
  const int64_t n2 = n >> 1;
  typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
  u64x2* p2 = reinterpret_cast<u64x2*>(p);
  const u64x2 q = {v, v};
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride)
    __builtin_nontemporal_store(q, p2 + i);
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) p[n - 1] = v;
}

// Rows the sel_direct pass did not write (series with no row in the scan range): the no-value
// pattern, so the whole S x K buffer need not be filled beforehand.
__global__ __launch_bounds__(256) void k_fill_rows(uint64_t* p, const uint8_t* wr, int64_t n_series, int64_t K,
                                                   uint64_t v, const int64_t* gsp, int64_t G) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_series || wr[s]) return;
  if (!gsp) {
    for (int64_t k = 0; k < K; k++) p[s * K + k] = v;
    return;
  }
  // column layout: the series' group by binary search over gsp (ungrouped series have no column)
  if (s >= gsp[G]) return;
  int64_t lo = 0, hi = G;
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (gsp[mid] <= s) lo = mid; else hi = mid;
  }
  const int64_t g0 = gsp[lo], ng = gsp[lo + 1] - g0;
  for (int64_t k = 0; k < K; k++) p[g0 * K + k * ng + (s - g0)] = v;
}

hipError_t launch_fill_rows(uint64_t* p, const uint8_t* wr, int64_t n_series, int64_t K, uint64_t v, hipStream_t s,
                            const int64_t* gsp, int64_t G) {
  if (n_series <= 0 || K <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_fill_rows, dim3((unsigned)((n_series + 255) / 256)), dim3(256), 0, s, p, wr, n_series, K, v, gsp, G);
  return hipGetLastError();
}

hipError_t launch_fill64(uint64_t* p, uint64_t v, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(((n >> 1) + 255) / 256, 256 * 16));
  hipLaunchKernelGGL(k_fill64, dim3((unsigned)blocks), dim3(256), 0, s, p, v, n);
  return hipGetLastError();
}

// ---- launchers -------------------------------------------------------------------
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

int64_t fast_wave_lds(int64_t K, bool rate, bool part) { return align16(1024 + fast_slot_bytes(K, rate, part)); }   // + VL==0 value stage

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

// Host -> device copy by the GPU's own loads from page-locked host memory (mapped into the
// device's address space): the queue's copy engine ran the compaction upload at half the link
// rate on every call after the first (19 ms for 576 MB against 10 ms; blit copies: 10 ms, r05n /
// r05o profiles).  src and dst share their address modulo 16; 16-byte loads across the grid.
__global__ __launch_bounds__(256) void k_pull(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, size_t n) {
  const size_t head = (16 - ((uintptr_t)dst & 15)) & 15;
  const size_t h = head < n ? head : n;
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (size_t)gridDim.x * blockDim.x;
  if (tid < h) dst[tid] = src[tid];
  const size_t body = (n - h) >> 4;
  const uint4* s4 = reinterpret_cast<const uint4*>(src + h);
  uint4* d4 = reinterpret_cast<uint4*>(dst + h);
  for (size_t i = tid; i < body; i += nth) d4[i] = s4[i];
  const size_t t0 = h + (body << 4);
  if (t0 + tid < n) dst[t0 + tid] = src[t0 + tid];
}

hipError_t launch_pull(void* dst, const void* src, size_t n, hipStream_t s) {
  if (!n) return hipSuccess;
  const size_t units = n / 16 + 1;
  const unsigned blocks = (unsigned)std::min<size_t>(8192, std::max<size_t>(1, (units + 255) / 256));
  hipLaunchKernelGGL(k_pull, dim3(blocks), dim3(256), 0, s, static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), n);
  return hipGetLastError();
}

hipError_t launch_state_fold(const StateFoldParams& p, hipStream_t s) {
  hipLaunchKernelGGL(k_state_fold, dim3((unsigned)((p.K + 255) / 256)), dim3(256), 0, s, p);
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

// Rollup read path: Downsampler.next's rollup branches
// (src/core/Downsampler.java:165-221, FillingDownsampler.java:196-253) from two SUM
// downsamplings.  dense[s][k] holds Σsum of value series s (in datapoint order, as the
// reference's `sum += nextDoubleValue()`), dense[cmap[s]][k] Σcount of its count series; a
// bucket with datapoints becomes Σsum / Σcount (0 when Σcount is 0) for avg, Σcount for
// count.  The count series are never written (cmap of a count series is -1).
__global__ __launch_bounds__(256) void k_rollup_combine(double* __restrict__ dense, const uint8_t* __restrict__ pres,
                                                        const int64_t* __restrict__ cmap, int64_t n_series, int64_t K,
                                                        int avg) {
  const int64_t total = n_series * K;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = i / K;
    const int64_t cs = cmap[s];
    if (cs < 0 || !pres[i]) continue;
    const double sum = dense[i];
    const int64_t ci = cs * K + (i - s * K);
    const double count = pres[ci] ? dense[ci] : 0.0;   // a bucket the count series left empty holds no count
    dense[i] = avg ? (count == 0.0 ? 0.0 : sum / count) : count;
  }
}

hipError_t launch_rollup_combine(double* dense, const uint8_t* pres, const int64_t* cmap, int64_t n_series, int64_t K,
                                 int avg, hipStream_t s) {
  const int64_t total = n_series * K;
  if (total <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(k_rollup_combine, dim3((unsigned)blocks), dim3(256), 0, s, dense, pres, cmap, n_series, K, avg);
  return hipGetLastError();
}

}  // namespace tsdb
