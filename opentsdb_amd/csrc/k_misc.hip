// k_misc.hip -- row index, cross-tile group reduction, synthetic store and the
// per-function dispatch of libtsdbhip (the k_grid / k_fast instantiations live in
// k_grid.hip / k_fast.hip, compiled once per downsample function).
#include "kcommon.h"

namespace tsdb {

// ---- k_index: classify every row, validate it, certificate stats ---------------------
// Also writes val2: for 2-byte-qualifier rows, every integer value of 1 or 2 bytes as a
// little-endian int16 at val2 + qoff + 2 i (same offsets as the qualifiers), the layout the
// vle-integer class of k_short / k_fast reads.
__global__ __launch_bounds__(256) void k_index(const uint8_t* __restrict__ qual, const uint8_t* __restrict__ val,
                                               uint8_t* __restrict__ val2, RowDesc* __restrict__ rows, int64_t n_rows,
                                               int32_t* err) {
  const int lane = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = wave; r < n_rows; r += nwaves) {
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
                        int32_t* err, hipStream_t s) {
  if (n_rows == 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((n_rows + 3) / 4, 65536);
  hipLaunchKernelGGL(k_index, dim3((unsigned)blocks), dim3(256), 0, s, qual, val, val2, rows, n_rows, err);
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
