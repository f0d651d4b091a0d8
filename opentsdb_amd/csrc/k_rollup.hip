// k_rollup.hip -- rollup generation: the per-series downsampled
// buckets of one function (dense [series][slot] outputs of the NONE-aggregator query,
// engine.cpp) -> rollup cells [agg id][BE16 offset|flags] + value bytes.
//
// Two passes over the (series, slot) grid in batch series order: k_rollup_size writes a
// cell flag and the value length of every present bucket, two device-wide exclusive scans
// turn them into cell and byte offsets, k_rollup_write writes the cells.  The grid is
// 1 thread per (series, slot): a few bytes read and written per bucket, HBM-bound.
#include <hipcub/hipcub.hpp>

#include "engine.h"
#include "rollup_codec.h"
#include "../../include/tsdbhip.h"

namespace tsdb {

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
