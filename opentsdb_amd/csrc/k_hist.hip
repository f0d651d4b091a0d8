// k_hist.hip -- gfx950 kernels of the histogram path.
//
// Reference: TsdbQuery.HistogramGroupByAndAggregateCB (src/core/TsdbQuery.java:1061-1255) over
// HistogramSpans (src/core/HistogramSpan.java), HistogramDownsampler
// (src/core/HistogramDownsampler.java:64-397), HistogramAggregationIterator
// (src/core/HistogramAggregationIterator.java:91-313) and SimpleHistogram
// (src/core/SimpleHistogram.java:97-271).
//
//   k_hist_validate  thread per column: the codec's decode (Kryo 2.21 layout) -- a column that
//                    throws is dropped as SaltScanner.processRow drops it -- and every bucket key
//                    of a SimpleHistogram into the store's dictionary hash set
//   k_hist_slots     thread per span of the query: HistogramSpan.Iterator.seek, the
//                    HistogramDownsampler's interval walk (or the raw datapoints) and the
//                    aggregation iterator's per-span admission (first point >= start, stop at a
//                    zero timestamp / past end) -> each datapoint's output slot
//   k_hist_accum     wave of 64 consecutive datapoints: the columns are parsed in lock step (lane =
//                    datapoint, loop = bucket position), counts are summed over the lanes that
//                    hit the same (point, bucket) with a segmented wave scan and added once per
//                    run (64-bit atomics: SUM of longs is exact in any order)
//   k_hist_final     thread per (group, slot): SimpleHistogram.percentile / the long codec's
//                    data * p, bucket counts and presence of the emitted points
#include "hist.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>

namespace tsdb {

struct HWiden {
  __host__ __device__ int64_t operator()(uint32_t x) const { return (int64_t)x; }
};

namespace {

__device__ __forceinline__ uint32_t fcanon(uint32_t b) {   // Float.floatToIntBits
  return ((b & 0x7F800000u) == 0x7F800000u && (b & 0x007FFFFFu)) ? 0x7FC00000u : b;
}
__device__ __forceinline__ uint64_t hk_hash(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}
__device__ __forceinline__ uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
// Kryo Input.readLong(true): 7-bit groups, the 9th byte carries 8 bits; false = buffer underflow
__device__ __forceinline__ bool varlong(const uint8_t* v, uint64_t n, uint64_t& i, uint64_t& out) {
  uint64_t r = 0;
#pragma unroll 1
  for (int j = 0; j < 8; j++) {
    if (i >= n) return false;
    const uint32_t b = v[i++];
    r |= (uint64_t)(b & 0x7F) << (7 * j);
    if (!(b & 0x80)) { out = r; return true; }
  }
  if (i >= n) return false;
  r |= (uint64_t)v[i++] << 56;
  out = r;
  return true;
}

// SimpleHistogram.fromHistogram(raw, true) (:97-122): count and byte length of a valid column
__device__ bool simple_valid(const uint8_t* v, uint64_t n) {
  if (n < 6) return false;
  const int cnt = (int16_t)(((uint32_t)v[1] << 8) | v[2]);
  uint64_t i = 3, c;
#pragma unroll 1
  for (int j = 0; j < cnt; j++) {
    if (i + 8 > n) return false;
    i += 8;
    if (!varlong(v, n, i, c)) return false;
  }
  return varlong(v, n, i, c) && varlong(v, n, i, c);
}

__global__ void k_hist_validate(HistLoadParams p) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= p.n_cells) return;
  const uint64_t o = p.voff[c], n = p.voff[c + 1] - o;
  const uint8_t* v = p.val + o;
  uint8_t st = HC_DROP;
  if (n >= 1) {
    const int id = (int8_t)v[0];
    const uint8_t kind = id >= 0 ? p.codec[id] : 0;
    if (kind == HC_LONG) st = n >= 9 ? HC_LONG : HC_DROP;             // Bytes.getLong(raw, 1)
    else if (kind == HC_SIMPLE && simple_valid(v, n)) st = HC_SIMPLE;
  }
  p.status[c] = st;
  if (st != HC_SIMPLE) return;
  const int cnt = (int16_t)(((uint32_t)v[1] << 8) | v[2]);
  uint64_t i = 3, cv;
  uint64_t prev_ord = 0;
  bool sorted = true;   // keys in HistogramBucket.compareTo order, strictly (histogram() writes a TreeMap)
#pragma unroll 1
  for (int j = 0; j < cnt; j++) {
    const uint64_t key = ((uint64_t)fcanon(be32(v + i)) << 32) | fcanon(be32(v + i + 4));
    // Float.compare order of (lower, upper) as one unsigned key
    auto ford = [](uint32_t b) { return (b & 0x80000000u) ? ~b : (b | 0x80000000u); };
    const uint64_t ord = ((uint64_t)ford((uint32_t)(key >> 32)) << 32) | ford((uint32_t)key);
    if (j > 0 && ord <= prev_ord) sorted = false;
    prev_ord = ord;
    i += 8;
    varlong(v, n, i, cv);
    uint64_t slot = hk_hash(key) & (uint64_t)(HT_SIZE - 1);
#pragma unroll 1
    for (int64_t probe = 0;; probe++) {
      if (probe >= HT_SIZE) { atomicAdd(p.hcount, HK_MAX + 1); break; }
      const uint64_t cur = __hip_atomic_load(&p.hkey[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == key) break;
      if (cur == HK_EMPTY) {
        const unsigned long long prev =
            atomicCAS((unsigned long long*)&p.hkey[slot], (unsigned long long)HK_EMPTY, (unsigned long long)key);
        if (prev == HK_EMPTY) { atomicAdd(p.hcount, 1); break; }
        if (prev == key) break;
      }
      slot = (slot + 1) & (uint64_t)(HT_SIZE - 1);
    }
  }
  if (!sorted) p.status[c] = HC_SIMPLE | HC_UNSORTED;
}

__device__ __forceinline__ int32_t dict_index(const HistQueryParams& p, uint64_t key) {
  uint64_t slot = hk_hash(key) & (uint64_t)(HT_SIZE - 1);
#pragma unroll 1
  for (int64_t probe = 0; probe < HT_SIZE; probe++) {
    const uint64_t cur = p.hkey[slot];
    if (cur == key) return p.hidx[slot];
    if (cur == HK_EMPTY) return -1;
    slot = (slot + 1) & (uint64_t)(HT_SIZE - 1);
  }
  return -1;
}

__device__ __forceinline__ void set_err(int32_t* err, int code, int why) {
  if (atomicCAS(err, 0, code) == 0) err[1] = why;
}

// error reasons (err[1]) reported by the host
enum { WHY_SEEK = 1, WHY_NPE = 2, WHY_UNSORTED = 3, WHY_SLOT = 4, WHY_MIXED = 5, WHY_DICT = 6 };

// HistogramSpan.Iterator.seek (:525-532 with seekRow :417-437 and HistogramRowSeq.Iterator.seek
// :357-368): the position iteration continues from
__device__ int64_t span_seek(const HistQueryParams& p, int64_t rlo, int64_t rhi, int64_t target) {
  int64_t ri = rlo;
  for (int64_t r = rlo; r < rhi; r++) {
    const int64_t a = p.row_pos[r], b = p.row_pos[r + 1];
    if (b - a < 1 || p.pos_ts[b - 1] < target) ri++;
    else break;
  }
  if (ri == rhi) --ri;
  int64_t q = p.row_pos[ri];
  const int64_t e = p.row_pos[ri + 1];
  while (q < e && p.pos_ts[q] < target) ++q;
  return q;
}

__global__ void k_hist_slots(HistQueryParams p) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= p.n_spans) return;
  const int64_t rlo = p.sp_rlo[s], rhi = p.sp_rhi[s];
  const int64_t p0 = p.row_pos[rlo], p1 = p.row_pos[rhi];
  if (p1 <= p0) return;
  // HistogramSpanGroup.add (:187-203): a datapoint of the span in [start, end]
  int64_t first = p.pos_ts[p0], last = p.pos_ts[p1 - 1];
  if ((first & (int64_t)0xFFFFFFFF00000000LL) == 0) first *= 1000;
  if ((last & (int64_t)0xFFFFFFFF00000000LL) == 0) last *= 1000;
  if (!(first <= p.end && last >= p.start)) return;
  const int64_t g = p.sp_out[s];
  const int64_t target = p.ds == 1 ? (p.start + p.I - 1) - (p.start + p.I - 1) % p.I : (p.ds == 3 ? p.cal_seek : p.start);
  if (target & (int64_t)0xFFFFF00000000000LL) { set_err(p.err, -3 /* IAE */, WHY_SEEK); return; }
  int64_t q = span_seek(p, rlo, rhi, target);
  if (p.ds == 0) {
    // raw: every datapoint is an output of the span (HistogramSpan.Iterator)
    int64_t prev = INT64_MIN;
    for (bool firstout = true; q < p1; q++, firstout = false) {
      const int64_t ts = p.pos_ts[q];
      if (firstout && ts < p.start) return;   // ctor :141-151: the span ends
      if (ts == 0 || ts > p.end) return;      // endReached / never merged again
      if (ts <= prev) { set_err(p.err, -22, WHY_UNSORTED); return; }
      prev = ts;
      p.pos_key[q] = (g << 42) | (ts - p.start);
    }
    return;
  }
  if (p.ds == 2) {
    // "all" (:251-276): skip datapoints before the query start, stop at the first one at or past
    // the query end; one output whose timestamp() is the query start
    int64_t n = 0;
    int64_t r = q;
    for (; r < p1; r++) {
      const int64_t ts = p.pos_ts[r];
      if (ts < p.qs) continue;
      if (ts >= p.qe) break;
      n++;
    }
    if (n == 0) return;
    if (n >= 2 && !p.ds_sum) { set_err(p.err, -10, WHY_NPE); return; }
    if (p.qs < p.start || p.qs == 0 || p.qs > p.end) return;
    for (r = q; r < p1; r++) {
      const int64_t ts = p.pos_ts[r];
      if (ts < p.qs) continue;
      if (ts >= p.qe) break;
      p.pos_slot[r] = (int32_t)g;
    }
    return;
  }
  if (p.ds == 3) {
    // calendar (:219-248, 282-300, 309-331): intervals from previousInterval(the first datapoint
    // after the seek) stepped by the calendar unit -- the host's boundary run of this span's
    // anchor; outputs are keyed like raw datapoints and merged over the union of timestamps
    const int64_t* tab = p.cal_tab + p.sp_cal[2 * s];
    const int64_t nb = p.sp_cal[2 * s + 1];
    int64_t j = 0, prev = INT64_MIN;
    for (bool firstout = true; q < p1; firstout = false) {
      const int64_t a = p.pos_ts[q];
      while (j + 1 < nb && tab[j + 1] <= a) j++;
      const int64_t ots = tab[j];
      const int64_t tei = j + 1 < nb ? tab[j + 1] : INT64_MAX;
      int64_t e = q;
      while (e < p1 && p.pos_ts[e] < tei) e++;
      if (e - q >= 2 && !p.ds_sum) { set_err(p.err, -10, WHY_NPE); return; }
      if (firstout && ots < p.start) return;
      if (ots == 0 || ots > p.end) return;
      if (ots <= prev) { set_err(p.err, -22, WHY_UNSORTED); return; }
      prev = ots;
      for (int64_t r = q; r < e; r++) p.pos_key[r] = (g << 42) | (ots - p.start);
      q = e;
    }
    return;
  }
  // fixed interval (:242-244, 296-297, 334-349): the interval of the first datapoint not yet
  // consumed, every following datapoint below its end
  int64_t prev = INT64_MIN;
  for (bool firstout = true; q < p1; firstout = false) {
    const int64_t a = p.pos_ts[q];
    const int64_t tei = a - a % p.I + p.I;
    const int64_t ots = tei - p.I;
    int64_t e = q;
    while (e < p1 && p.pos_ts[e] < tei) e++;
    // the aggregation iterator pulls this interval (the HistogramDownsampler sums it now)
    if (e - q >= 2 && !p.ds_sum) { set_err(p.err, -10, WHY_NPE); return; }
    if (firstout && ots < p.start) return;
    if (ots == 0 || ots > p.end) return;
    if (ots <= prev) { set_err(p.err, -22, WHY_UNSORTED); return; }
    prev = ots;
    const int64_t k = (ots - p.B0) / p.I;
    if (ots < p.B0 || k >= p.K) { set_err(p.err, -22, WHY_SLOT); return; }
    const int32_t slot = (int32_t)(g * p.K + k);
    for (int64_t r = q; r < e; r++) p.pos_slot[r] = slot;
    q = e;
  }
}

// Raw group-by over spans some of which are out of time order (a row mixing second and
// millisecond qualifiers is iterated in column order: HistogramRowSeq does not sort).
// HistogramAggregationIterator (src/core/HistogramAggregationIterator.java:118-160 ctor, :240-292
// next) is then a greedy walk, not the union of timestamps: each step takes the smallest current
// timestamp t among the spans whose current one is neither 0 (endReached) nor past the end, sums
// every span's current histogram at t (the first such span's value aggregated with the others in
// span order -- integer bucket counts, order-free) and advances exactly those spans; a span can
// come back below t later.  One wave a group: lane l holds spans l, l + 64, ...; a step is a wave
// min, then the lanes holding it label their spans' current positions with the step and advance
// them.  The ctor's rules: HistogramSpanGroup.add's [start, end] overlap (k_hist_slots), the seek
// to the start, a first datapoint before the start ends the span.
__global__ void k_hist_walk(HistQueryParams p, const int64_t* gsp, int64_t G, int64_t* sp_q, int64_t* sp_ts) {
  const int64_t g = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (g >= G) return;
  const int lane = __lane_id();
  const int64_t a = gsp[g], b = gsp[g + 1];
  // ctor: the first datapoint of every span (0 = ended)
  for (int64_t s = a + lane; s < b; s += 64) {
    int64_t ts = 0, q = 0;
    const int64_t rlo = p.sp_rlo[s], rhi = p.sp_rhi[s];
    const int64_t p0 = p.row_pos[rlo], p1 = p.row_pos[rhi];
    if (p1 > p0) {
      int64_t first = p.pos_ts[p0], last = p.pos_ts[p1 - 1];
      if ((first & (int64_t)0xFFFFFFFF00000000LL) == 0) first *= 1000;
      if ((last & (int64_t)0xFFFFFFFF00000000LL) == 0) last *= 1000;
      if (first <= p.end && last >= p.start) {
        q = span_seek(p, rlo, rhi, p.start);
        if (q < p1 && p.pos_ts[q] >= p.start) ts = p.pos_ts[q];
      }
    }
    sp_q[s] = q;
    sp_ts[s] = ts;
  }
  __builtin_amdgcn_wave_barrier();
  __threadfence_block();
  for (int64_t step = 0;; step++) {
    int64_t m = INT64_MAX;
    for (int64_t s = a + lane; s < b; s += 64) {
      const int64_t t = sp_ts[s];
      if (t != 0 && t <= p.end && t < m) m = t;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      const int64_t o = __shfl_xor(m, d);
      m = o < m ? o : m;
    }
    if (m == INT64_MAX) break;
    for (int64_t s = a + lane; s < b; s += 64) {
      if (sp_ts[s] != m) continue;
      const int64_t q = sp_q[s];
      p.pos_key[q] = (g << 42) | step;
      const int64_t p1 = p.row_pos[p.sp_rhi[s]];
      sp_q[s] = q + 1;
      sp_ts[s] = q + 1 < p1 ? p.pos_ts[q + 1] : 0;   // (a datapoint at 0 ends the span, as endReached)
    }
  }
}

// k_hist_walk with a block a group: the group's spans one per thread slot (thread t holds spans
// t, t + blockDim, ... -- up to WALK_SPT of them, in registers), a step's minimum is a wave min then
// one LDS exchange between the block's waves (double-buffered: one barrier a step), and only the
// spans at the minimum touch memory.  k_hist_walk's wave walks every span's current timestamp
// in global memory twice a step: 44 ms for 4 groups of 5000 spans x 360 steps (profiles/r06af).
// Same steps, same labels.
#define WALK_SPT 8
__global__ __launch_bounds__(1024) void k_hist_walk_blk(HistQueryParams p, const int64_t* gsp) {
  const int64_t g = blockIdx.x;
  const int t = threadIdx.x, nt = blockDim.x, lane = __lane_id(), w = t >> 6, nw = nt >> 6;
  const int64_t a = gsp[g], b = gsp[g + 1];
  __shared__ int64_t red[2][16];
  int64_t ts[WALK_SPT], q[WALK_SPT], qe[WALK_SPT];
#pragma unroll
  for (int i = 0; i < WALK_SPT; i++) {
    const int64_t s = a + t + (int64_t)i * nt;
    ts[i] = 0;
    q[i] = 0;
    qe[i] = 0;
    if (s < b) {   // the ctor, as k_hist_walk
      const int64_t rlo = p.sp_rlo[s], rhi = p.sp_rhi[s];
      const int64_t p0 = p.row_pos[rlo], p1 = p.row_pos[rhi];
      qe[i] = p1;
      if (p1 > p0) {
        int64_t first = p.pos_ts[p0], last = p.pos_ts[p1 - 1];
        if ((first & (int64_t)0xFFFFFFFF00000000LL) == 0) first *= 1000;
        if ((last & (int64_t)0xFFFFFFFF00000000LL) == 0) last *= 1000;
        if (first <= p.end && last >= p.start) {
          q[i] = span_seek(p, rlo, rhi, p.start);
          if (q[i] < p1 && p.pos_ts[q[i]] >= p.start) ts[i] = p.pos_ts[q[i]];
        }
      }
    }
  }
  for (int64_t step = 0;; step++) {
    int64_t m = INT64_MAX;
#pragma unroll
    for (int i = 0; i < WALK_SPT; i++)
      if (ts[i] != 0 && ts[i] <= p.end && ts[i] < m) m = ts[i];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      const int64_t o = __shfl_xor(m, d);
      m = o < m ? o : m;
    }
    if (lane == 0) red[step & 1][w] = m;
    __syncthreads();
    m = INT64_MAX;
    for (int i = 0; i < nw; i++) {
      const int64_t o = red[step & 1][i];
      m = o < m ? o : m;
    }
    if (m == INT64_MAX) break;   // (block-uniform)
#pragma unroll
    for (int i = 0; i < WALK_SPT; i++) {
      if (ts[i] != m) continue;
      p.pos_key[q[i]] = (g << 42) | step;
      q[i]++;
      ts[i] = q[i] < qe[i] ? p.pos_ts[q[i]] : 0;   // (a datapoint at 0 ends the span, as endReached)
    }
  }
}

// segmented (by equal address) inclusive scan over the wave (runs of equal addr are contiguous
// lanes in the common case; equal addresses further apart only cost extra atomics); returns true
// on the run's last lane
template <class T, class Op>
__device__ __forceinline__ bool seg_scan(uint64_t addr, T& v, Op op) {
  const int lane = __lane_id();
  const uint64_t left = __shfl_up(addr, 1);
  const bool head = lane == 0 || left != addr;
  const uint64_t heads = __ballot(head);
  const uint64_t upto = heads & (lane == 63 ? ~0ull : ((2ull << lane) - 1));
  const int start = 63 - __builtin_clzll(upto);
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const T o = __shfl_up(v, d);
    if (lane - d >= start) v = op(v, o);
  }
  const uint64_t right = __shfl_down(addr, 1);
  return lane == 63 || right != addr;
}
struct OpAdd { __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return a + b; } };
struct OpOr { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a | b; } };

// byte sources of a column: the block's LDS stage or global memory
struct SrcLds {
  const uint8_t* b;
  __device__ __forceinline__ uint32_t at(uint64_t i) const { return b[i]; }
};
struct SrcGlobal {
  const uint8_t* b;
  __device__ __forceinline__ uint32_t at(uint64_t i) const { return b[i]; }
};
template <class S>
__device__ __forceinline__ uint32_t sbe32(const S& s, uint64_t i) {
  return (s.at(i) << 24) | (s.at(i + 1) << 16) | (s.at(i + 2) << 8) | s.at(i + 3);
}
template <class S>
__device__ __forceinline__ uint64_t svarlong(const S& s, uint64_t& i) {   // the column was validated at load
  uint64_t r = 0;
#pragma unroll 1
  for (int j = 0; j < 8; j++) {
    const uint32_t b = s.at(i++);
    r |= (uint64_t)(b & 0x7F) << (7 * j);
    if (!(b & 0x80)) return r;
  }
  return r | ((uint64_t)s.at(i++) << 56);
}

static constexpr int LDICT = 1024;   // LDS dictionary slots (dictionaries of at most LDICT / 2 buckets)
static constexpr int ATP = 128;      // positions per tile = threads per block
static constexpr int STAGE_W = 8192; // 32 KB of column bytes staged per tile

struct DictLds {
  const uint64_t* key;
  const int32_t* idx;
  uint32_t mask = LDICT - 1;   // slots - 1
  __device__ __forceinline__ int32_t find(uint64_t k) const {
    uint32_t slot = lds_dict_slot(k, mask);
#pragma unroll 1
    for (uint32_t probe = 0; probe <= mask; probe++) {
      const uint64_t cur = key[slot];
      if (cur == k) return idx[slot];
      if (cur == HK_EMPTY) return -1;
      slot = (slot + 1) & mask;
    }
    return -1;
  }
};
struct DictGlobal {
  const HistQueryParams* p;
  __device__ __forceinline__ int32_t find(uint64_t k) const { return dict_index(*p, k); }
};

// One column per lane (pt < 0: no column); the wave's lanes step through their buckets together.
// true when the bucket key recurs among the column's buckets [j + 1, cnt) (bytes from i on):
// TreeMap.put keeps the last count of a key (SimpleHistogram.fromHistogram :110-113)
template <class S>
__device__ bool key_recurs(const S& src, uint64_t i, int j, int cnt, uint64_t key) {
#pragma unroll 1
  for (int k = j + 1; k < cnt; k++) {
    const uint64_t kk = ((uint64_t)fcanon(sbe32(src, i)) << 32) | fcanon(sbe32(src, i + 4));
    i += 8;
    (void)svarlong(src, i);
    if (kk == key) return true;
  }
  return false;
}

template <class S, class Dict>
__device__ __forceinline__ void accum_columns(const HistQueryParams& p, int32_t pt, const S& src, uint64_t i0,
                                              uint8_t kind_st, const Dict& dict) {
  const uint8_t kind = kind_st & HC_KIND;
  const bool unsorted = (kind_st & HC_UNSORTED) != 0;
  int cnt = 0;
  uint64_t i = i0 + 3;
  if (pt >= 0 && kind == HC_SIMPLE) cnt = (int16_t)((src.at(i0 + 1) << 8) | src.at(i0 + 2));
  const uint64_t base = (uint64_t)(pt >= 0 ? pt : 0) * (uint64_t)p.C;
  {  // codec bits of the point, and the long codec's data (LongHistogramDataPointForTest.aggregate)
    uint32_t kb = pt >= 0 ? (kind == HC_SIMPLE ? 1u : 2u) : 0u;
    const uint64_t paddr = pt >= 0 ? (uint64_t)pt : ~0ull;
    if (seg_scan(paddr, kb, OpOr()) && pt >= 0) atomicOr(&p.pkind[pt], kb);
    uint64_t val = 0, addr = ~0ull;
    if (pt >= 0 && kind == HC_LONG) {
      for (int j = 1; j < 9; j++) val = (val << 8) | src.at(i0 + j);
      addr = base + p.C - 1;
    }
    if (seg_scan(addr, val, OpAdd()) && addr != ~0ull) atomicAdd((unsigned long long*)&p.acc[addr], (unsigned long long)val);
  }
  int maxc = cnt;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) maxc = max(maxc, __shfl_xor(maxc, d));
  // buckets in lock step (SimpleHistogram.aggregate :246-261: counts of equal keys add)
#pragma unroll 1
  for (int j = 0; j < maxc; j++) {
    uint64_t addr = ~0ull, val = 0;
    int32_t di = -1;
    if (j < cnt) {
      const uint64_t key = ((uint64_t)fcanon(sbe32(src, i)) << 32) | fcanon(sbe32(src, i + 4));
      i += 8;
      val = svarlong(src, i);
      if (unsorted && key_recurs(src, i, j, cnt, key)) val = 0;   // a later bucket's count replaces it
      di = dict.find(key);
      if (di < 0) set_err(p.err, -22, WHY_DICT);
      else addr = base + (uint64_t)di;
    }
    if (seg_scan(addr, val, OpAdd()) && addr != ~0ull && !HIST_SKIP_ADD(p))
      atomicAdd((unsigned long long*)&p.acc[addr], (unsigned long long)val);
    if (p.pres && di >= 0) atomicOr(&p.pres[(uint64_t)pt * p.W + (di >> 5)], 1u << (di & 31));
  }
  for (int u = 0; u < 2; u++) {   // underflow, overflow (:256-257)
    uint64_t addr = ~0ull, val = 0;
    if (pt >= 0 && kind == HC_SIMPLE) {
      val = svarlong(src, i);
      addr = base + (uint64_t)p.D + u;
    }
    if (seg_scan(addr, val, OpAdd()) && addr != ~0ull) atomicAdd((unsigned long long*)&p.acc[addr], (unsigned long long)val);
  }
}

// Persistent blocks over tiles of ATP consecutive positions.  A tile whose columns are
// consecutive in the store and fit STAGE_W words is staged into LDS with coalesced dword loads
// and parsed there; other tiles parse from global memory.  Small dictionaries live in LDS.
template <bool LDSDICT>
__global__ void __launch_bounds__(ATP) k_hist_accum(HistQueryParams p, int64_t n_pos, const uint64_t* lkey_g,
                                                    const int32_t* lidx_g) {
  __shared__ uint32_t stage[STAGE_W];
  __shared__ uint64_t lkey[LDSDICT ? LDICT : 1];
  __shared__ int32_t lidx[LDSDICT ? LDICT : 1];
  const int tid = threadIdx.x;
  if (LDSDICT) {
    for (int k = tid; k < LDICT; k += ATP) { lkey[k] = lkey_g[k]; lidx[k] = lidx_g[k]; }
  }
  const int64_t n_tiles = (n_pos + ATP - 1) / ATP;
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const int64_t p0 = tile * ATP, q = p0 + tid;
    const int64_t m = min((int64_t)ATP, n_pos - p0);
    const bool in = tid < m;
    int32_t pt = -1;
    if (in) pt = p.pos_point ? p.pos_point[q] : p.pos_slot[q];
    __syncthreads();   // the previous tile's stage is consumed (and the dictionary is loaded)
    if (!__syncthreads_or(pt >= 0)) continue;
    const int64_t c0 = p.pos_cell[p0];
    const int64_t c = in ? p.pos_cell[q] : c0 + tid;
    const bool contiguous = __syncthreads_and(c == c0 + tid);
    const uint64_t b0 = p.voff[c0], b1 = contiguous ? p.voff[c0 + m] : b0;
    const uint64_t w0 = b0 >> 2, w1 = (b1 + 3) >> 2;
    const bool staged = contiguous && (w1 - w0) <= (uint64_t)STAGE_W;
    const uint8_t kind = pt >= 0 ? p.pos_kind[q] : 0;
    if (staged) {
      const uint32_t* g = reinterpret_cast<const uint32_t*>(p.val) + w0;
      for (uint64_t w = tid; w < w1 - w0; w += ATP) stage[w] = g[w];
      __syncthreads();
      const SrcLds src{reinterpret_cast<const uint8_t*>(stage)};
      const uint64_t i0 = pt >= 0 ? p.voff[c] - (w0 << 2) : 0;
      if (LDSDICT) accum_columns(p, pt, src, i0, kind, DictLds{lkey, lidx});
      else accum_columns(p, pt, src, i0, kind, DictGlobal{&p});
    } else {
      const SrcGlobal src{p.val};
      const uint64_t i0 = pt >= 0 ? p.voff[c] : 0;
      if (LDSDICT) accum_columns(p, pt, src, i0, kind, DictLds{lkey, lidx});
      else accum_columns(p, pt, src, i0, kind, DictGlobal{&p});
    }
  }
}

__global__ void k_hist_flags(HistQueryParams p, uint32_t* flag) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= p.n_points) return;
  const uint32_t k = p.pkind[t];
  if (k == 3u) set_err(p.err, -3, WHY_MIXED);
  flag[t] = k ? 1u : 0u;
}

__global__ void k_hist_final(HistQueryParams p) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= p.n_points) return;
  const uint32_t kind = p.pkind[t];
  if (!kind) return;
  const int64_t o = p.pt_out[t];
  const uint64_t* a = p.acc + (uint64_t)t * p.C;
  p.out_ts[o] = p.pt_ts ? p.pt_ts[t] : p.B0 + (t % p.K) * p.I;
  p.out_group[o] = p.pt_group ? p.pt_group[t] : (int32_t)(t / p.K);
  p.out_kind[o] = kind == 1u ? HC_SIMPLE : HC_LONG;
  for (int j = 0; j < p.n_pct; j++) {
    const double perc = (double)p.pct[j];
    double r;
    if (kind == 2u) {
      r = (double)(int64_t)a[p.C - 1] * perc;   // LongHistogramDataPointForTest.percentile
    } else if (perc < 1.0 || perc > 100.0) {
      r = -1.0;
    } else {   // SimpleHistogram.percentile (:133-164): int counts, bucket midpoints as float
      int32_t sum = 0;
      for (int b = 0; b < p.D; b++) sum = (int32_t)((uint32_t)sum + (uint32_t)a[b]);
      int64_t running = 0;
      r = 0.0;
      for (int b = 0; b < p.D; b++) {
        running += (int32_t)(uint32_t)a[b];
        const double area = (double)running * 100.0 / (double)sum;
        if (area >= perc) {
          const float mid = (__uint_as_float(p.dict_lo[b]) + __uint_as_float(p.dict_up[b])) / 2;
          r = (double)mid;
          break;
        }
      }
    }
    p.out_pct[o * p.n_pct + j] = r;
  }
  if (p.out_count) {
    for (int b = 0; b < p.D + 2; b++) p.out_count[o * (p.D + 2) + b] = (int64_t)a[b];
    for (int b = 0; b < p.D; b++) p.out_present[o * p.D + b] = (p.pres[(uint64_t)t * p.W + (b >> 5)] >> (b & 31)) & 1u;
  }
}

// sparse mode: sorted (group << 42 | ts - start) keys -> union points
__global__ void k_hist_heads(const uint64_t* key, int64_t n, uint32_t* head) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  head[i] = key[i] != ~0ull && (i == 0 || key[i] != key[i - 1]) ? 1u : 0u;
}
__global__ void k_hist_points(const uint64_t* key, const uint32_t* pos, int64_t n, const int64_t* incl,
                              int64_t start, int32_t* pos_point, int64_t* pt_ts, int32_t* pt_group,
                              const int64_t* greedy_ts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || key[i] == ~0ull) return;
  const int64_t pt = incl[i + 1] - 1;   // inclusive count of heads up to i, minus one
  pos_point[pos[i]] = (int32_t)pt;
  if (i == 0 || key[i] != key[i - 1]) {
    pt_ts[pt] = greedy_ts ? greedy_ts[pos[i]] : start + (int64_t)(key[i] & ((1ull << 42) - 1));
    pt_group[pt] = (int32_t)(key[i] >> 42);
  }
}
__global__ void k_iota(uint32_t* v, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = (uint32_t)i;
}

// ---- bucket layouts (load) ------------------------------------------------------------------
// column c shares column c - 1's layout when both are sorted SimpleHistograms of the same bucket
// count whose key bytes are equal (the counts in between may differ in length)
__device__ bool same_keys(const uint8_t* a, uint64_t na, const uint8_t* b, uint64_t nb) {
  const int ca = (int16_t)(((uint32_t)a[1] << 8) | a[2]), cb = (int16_t)(((uint32_t)b[1] << 8) | b[2]);
  if (ca != cb) return false;
  uint64_t i = 3, k = 3, c;
#pragma unroll 1
  for (int j = 0; j < ca; j++) {
    for (int t = 0; t < 8; t++)
      if (a[i + t] != b[k + t]) return false;
    i += 8;
    k += 8;
    varlong(a, na, i, c);
    varlong(b, nb, k, c);
  }
  return true;
}
__global__ void k_hist_layhead(int64_t n, const uint64_t* voff, const uint8_t* val, const uint8_t* status, uint32_t* head) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const bool el = status[c] == HC_SIMPLE;   // (unsorted columns carry HC_UNSORTED: not eligible)
  bool h = false;
  if (el) {
    const uint64_t o = voff[c], l = voff[c + 1] - o;
    const int cnt = (int16_t)(((uint32_t)val[o + 1] << 8) | val[o + 2]);
    if (cnt < 0 || cnt > HIST_LAY_MAXB) h = false;
    else h = c == 0 || status[c - 1] != HC_SIMPLE || !same_keys(val + o, l, val + voff[c - 1], voff[c] - voff[c - 1]);
  }
  head[c] = h ? 1u : 0u;
}
__global__ void k_hist_laylid(int64_t n, const uint64_t* voff, const uint8_t* val, const uint8_t* status,
                              const uint32_t* head, const int64_t* excl, int32_t* col_lid, int32_t* lay_col) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  int32_t lid = -1;
  if (status[c] == HC_SIMPLE) {
    const uint64_t o = voff[c];
    const int cnt = (int16_t)(((uint32_t)val[o + 1] << 8) | val[o + 2]);
    // heads up to and including c, minus one: c's layout (a column past HIST_LAY_MAXB buckets has none)
    if (cnt >= 0 && cnt <= HIST_LAY_MAXB) lid = (int32_t)(excl[c + 1] - 1);
  }
  col_lid[c] = lid;
  if (head[c]) lay_col[lid] = (int32_t)c;
}
__global__ void k_hist_laydi(int64_t nl, const int32_t* lay_col, const int32_t* lay_off, const uint64_t* voff,
                             const uint8_t* val, const uint64_t* hkey, const int32_t* hidx, int32_t* lay_di) {
  const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= nl) return;
  const int64_t c = lay_col[l];
  const uint64_t o = voff[c], n = voff[c + 1] - o;
  const uint8_t* v = val + o;
  const int cnt = (int16_t)(((uint32_t)v[1] << 8) | v[2]);
  uint64_t i = 3, cv;
  for (int j = 0; j < cnt; j++) {
    const uint64_t key = ((uint64_t)fcanon(be32(v + i)) << 32) | fcanon(be32(v + i + 4));
    i += 8;
    varlong(v, n, i, cv);
    uint64_t slot = hk_hash(key) & (uint64_t)(HT_SIZE - 1);
    int32_t di = -1;
    for (int64_t probe = 0; probe < HT_SIZE; probe++) {
      const uint64_t cur = hkey[slot];
      if (cur == key) { di = hidx[slot]; break; }
      if (cur == HK_EMPTY) break;
      slot = (slot + 1) & (uint64_t)(HT_SIZE - 1);
    }
    lay_di[lay_off[l] + j] = di;
  }
}

// ---- windowed accumulation ---------------------------------------------------------------
// The datapoints in SpanGroup order (vpos: the present spans sorted by output group, each span's
// in-range positions), each block a contiguous chunk of them.  A group's spans all land on the
// group's points, so a block keeps a window of WS consecutive points' [C] counters in LDS, adds
// there with LDS atomics and flushes the window to the global accumulator (contiguous 64-bit
// atomics, one per nonzero counter) only when a tile's points leave it.  Columns are staged in
// LDS per run of consecutive cells (up to WRUNS runs a tile) and parsed with unaligned dword
// reads (bucket key, one-dword varints).

static constexpr int WRUNS = 8;

__global__ void k_hist_vlen(const int64_t* rlo, const int64_t* rhi, const int64_t* row_pos, int64_t n, uint32_t* len) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) len[i] = (uint32_t)(row_pos[rhi[i]] - row_pos[rlo[i]]);
}
__global__ void k_hist_vpos(const int64_t* rlo, const int64_t* row_pos, const int64_t* off, int32_t* vpos) {
  const int64_t sp = blockIdx.x;
  const int64_t p0 = row_pos[rlo[sp]], o = off[sp], n = off[sp + 1] - o;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) vpos[o + i] = (int32_t)(p0 + i);
}

// little-endian dword of the bytes [i, i + 4) of a byte stream held as aligned dwords
__device__ __forceinline__ uint32_t udw(const uint32_t* w, uint64_t i) {
  const uint64_t k = i >> 2;
  return __builtin_amdgcn_alignbyte(w[k + 1], w[k], (uint32_t)(i & 3));
}
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

struct SrcW {   // LDS stage or global bytes, read as unaligned dwords
  const uint32_t* w;
  __device__ __forceinline__ uint32_t at(uint64_t i) const { return (udw(w, i) & 0xFF); }
  __device__ __forceinline__ uint32_t dw(uint64_t i) const { return udw(w, i); }
};

// Kryo readLong(true) from one dword when the varint has at most 4 bytes; else byte by byte
__device__ __forceinline__ uint64_t wvarlong(const SrcW& s, uint64_t& i) {
  const uint32_t x = s.dw(i);
  const uint32_t m = ~x & 0x80808080u;
  if (m) {
    const uint32_t L = (__builtin_ctz(m) >> 3) + 1;
    uint32_t v = (x & 0x7Fu) | ((x >> 1) & 0x3F80u) | ((x >> 2) & 0x1FC000u) | ((x >> 3) & 0xFE00000u);
    v &= (L == 4) ? 0x0FFFFFFFu : ((1u << (7 * L)) - 1);
    i += L;
    return v;
  }
  return svarlong(s, i);
}
__device__ __forceinline__ uint64_t wkey(const SrcW& s, uint64_t i) {
  return ((uint64_t)fcanon(bswap32(s.dw(i))) << 32) | fcanon(bswap32(s.dw(i + 4)));
}

struct Window {
  uint64_t* acc;     // [WS * C]
  uint32_t* kind;    // [WS]
  uint32_t* pres;    // [WS * W]
};

__device__ __forceinline__ void w_add(const HistQueryParams& p, const Window& w, int32_t local, int32_t pt, int col,
                                      uint64_t v) {
  if (!v) return;
  if (local >= 0) atomicAdd((unsigned long long*)&w.acc[(uint32_t)local * (uint32_t)p.C + col], (unsigned long long)v);
  else atomicAdd((unsigned long long*)&p.acc[(uint64_t)pt * p.C + col], (unsigned long long)v);
}

__device__ void accum_column_w(const HistQueryParams& p, const Window& w, int32_t pt, int32_t local, const SrcW& src,
                               uint64_t i0, uint8_t kind_st, const DictLds& dict) {
  const uint8_t kind = kind_st & HC_KIND;
  const uint32_t kb = kind == HC_SIMPLE ? 1u : 2u;
  if (local >= 0) atomicOr(&w.kind[local], kb);
  else atomicOr(&p.pkind[pt], kb);
  if (kind == HC_LONG) {   // LongHistogramDataPointForTest.aggregate: the 8-byte data adds
    const uint64_t v = ((uint64_t)bswap32(src.dw(i0 + 1)) << 32) | bswap32(src.dw(i0 + 5));
    w_add(p, w, local, pt, p.C - 1, v);
    return;
  }
  const bool unsorted = (kind_st & HC_UNSORTED) != 0;
  const int cnt = (int16_t)((src.at(i0 + 1) << 8) | src.at(i0 + 2));
  uint64_t i = i0 + 3;
#pragma unroll 1
  for (int j = 0; j < cnt; j++) {   // SimpleHistogram.aggregate (:246-261): counts of equal keys add
    const uint64_t key = wkey(src, i);
    i += 8;
    uint64_t val = wvarlong(src, i);
    if (unsorted && key_recurs(src, i, j, cnt, key)) val = 0;   // a later bucket's count replaces it
    const int32_t di = dict.find(key);
    if (di < 0) {
      set_err(p.err, -22, WHY_DICT);
      continue;
    }
    if (!HIST_SKIP_ADD(p)) w_add(p, w, local, pt, di, val);
    if (p.pres) {
      if (local >= 0) atomicOr(&w.pres[(uint32_t)local * (uint32_t)p.W + (di >> 5)], 1u << (di & 31));
      else atomicOr(&p.pres[(uint64_t)pt * p.W + (di >> 5)], 1u << (di & 31));
    }
  }
  const uint64_t under = wvarlong(src, i);   // underflow, overflow (:256-257)
  const uint64_t over = wvarlong(src, i);
  w_add(p, w, local, pt, p.D, under);
  w_add(p, w, local, pt, p.D + 1, over);
}

// accum_column_w with the bucket loop software-pipelined: bucket j's dictionary probe is issued
// together with bucket j + 1's key and count dwords, so each bucket waits for one LDS round trip
// instead of two (the key / count reads of j + 1 do not depend on j's lookup)
__device__ void accum_column_wp(const HistQueryParams& p, const Window& w, int32_t pt, int32_t local, const SrcW& src,
                                uint64_t i0, uint8_t kind_st, const DictLds& dict, int32_t lid) {
  const uint8_t kind = kind_st & HC_KIND;
  if ((kind_st & HC_UNSORTED) || kind != HC_SIMPLE) {
    accum_column_w(p, w, pt, local, src, i0, kind_st, dict);
    return;
  }
  if (local >= 0) atomicOr(&w.kind[local], 1u);
  else atomicOr(&p.pkind[pt], 1u);
  const int cnt = (int16_t)((src.at(i0 + 1) << 8) | src.at(i0 + 2));
  uint64_t i = i0 + 3;
  if (lid >= 0) {
    // a known layout: the dictionary indices come from the layout table, the keys are skipped
    const int32_t* lt = p.lay_di + p.lay_off[lid];
    int32_t dis[HIST_LAY_MAXB];
#pragma unroll
    for (int j = 0; j < HIST_LAY_MAXB; j++) dis[j] = j < cnt ? lt[j] : 0;
#pragma unroll
    for (int j = 0; j < HIST_LAY_MAXB; j++) {
      if (j < cnt) {
        i += 8;
        const uint64_t val = wvarlong(src, i);
        const int32_t di = dis[j];
        if (di < 0) {
          set_err(p.err, -22, WHY_DICT);
          continue;
        }
        if (!HIST_SKIP_ADD(p)) w_add(p, w, local, pt, di, val);
        if (p.pres) {
          if (local >= 0) atomicOr(&w.pres[(uint32_t)local * (uint32_t)p.W + (di >> 5)], 1u << (di & 31));
          else atomicOr(&p.pres[(uint64_t)pt * p.W + (di >> 5)], 1u << (di & 31));
        }
      }
    }
    const uint64_t under = wvarlong(src, i);
    const uint64_t over = wvarlong(src, i);
    w_add(p, w, local, pt, p.D, under);
    w_add(p, w, local, pt, p.D + 1, over);
    return;
  }
  uint64_t key = 0, val = 0;
  if (cnt > 0) {
    key = wkey(src, i);
    i += 8;
    val = wvarlong(src, i);
  }
#pragma unroll 1
  for (int j = 0; j < cnt; j++) {
    const uint32_t slot = lds_dict_slot(key, dict.mask);
    const uint64_t cur = dict.key[slot];
    const int32_t cidx = dict.idx[slot];
    uint32_t x0 = 0, x1 = 0, xv = 0;
    const bool more = j + 1 < cnt;
    if (more) {
      x0 = src.dw(i);
      x1 = src.dw(i + 4);
      xv = src.dw(i + 8);
    }
    int32_t di = cur == key ? cidx : (cur == HK_EMPTY ? -1 : dict.find(key));
    if (di < 0) set_err(p.err, -22, WHY_DICT);
    else {
      if (!HIST_SKIP_ADD(p)) w_add(p, w, local, pt, di, val);
      if (p.pres) {
        if (local >= 0) atomicOr(&w.pres[(uint32_t)local * (uint32_t)p.W + (di >> 5)], 1u << (di & 31));
        else atomicOr(&p.pres[(uint64_t)pt * p.W + (di >> 5)], 1u << (di & 31));
      }
    }
    if (more) {
      key = ((uint64_t)fcanon(bswap32(x0)) << 32) | fcanon(bswap32(x1));
      i += 8;
      const uint32_t m = ~xv & 0x80808080u;
      if (m) {
        const uint32_t L = (__builtin_ctz(m) >> 3) + 1;
        uint32_t v = (xv & 0x7Fu) | ((xv >> 1) & 0x3F80u) | ((xv >> 2) & 0x1FC000u) | ((xv >> 3) & 0xFE00000u);
        v &= (L == 4) ? 0x0FFFFFFFu : ((1u << (7 * L)) - 1);
        val = v;
        i += L;
      } else {
        val = svarlong(src, i);
      }
    }
  }
  const uint64_t under = wvarlong(src, i);   // underflow, overflow (:256-257)
  const uint64_t over = wvarlong(src, i);
  w_add(p, w, local, pt, p.D, under);
  w_add(p, w, local, pt, p.D + 1, over);
}

// the window's counters to the global accumulator (points [wb, wb + WS)), zeroed for the next
__device__ void w_flush(const HistQueryParams& p, const Window& w, int64_t wb, int WS) {
  __syncthreads();
  const int64_t lim = (p.n_points - wb) * p.C;   // counters of real points
  const int nc = WS * p.C;
  uint64_t* g = p.acc + (uint64_t)wb * p.C;
  for (int e = threadIdx.x; e < nc; e += blockDim.x) {
    const uint64_t v = w.acc[e];
    if (v && e < lim) atomicAdd((unsigned long long*)&g[e], (unsigned long long)v);
    w.acc[e] = 0;
  }
  for (int e = threadIdx.x; e < WS; e += blockDim.x) {
    const uint32_t v = w.kind[e];
    if (v && wb + e < p.n_points) atomicOr(&p.pkind[wb + e], v);
    w.kind[e] = 0;
  }
  if (p.pres) {
    const int np = WS * p.W;
    for (int e = threadIdx.x; e < np; e += blockDim.x) {
      const uint32_t v = w.pres[e];
      if (v && wb + e / p.W < p.n_points) atomicOr(&p.pres[(uint64_t)wb * p.W + e], v);
      w.pres[e] = 0;
    }
  }
  __syncthreads();
}

// A position's column as k_hist_accw reads it: one coalesced 24-B load a lane instead of the
// vpos -> pos_point / pos_cell -> voff / col_lid chain (three dependent round trips a tile), so the
// next tile's entries are in flight while the current tile is staged and parsed.
struct HTIdx {
  uint64_t vo0;    // the column's value bytes [vo0, vo0 + len)
  uint32_t len;
  uint32_t kind;   // pos_kind
  int32_t pt;      // output point (-1: none)
  int32_t lid;     // layout id (-1: none)
};
static_assert(sizeof(HTIdx) == 24, "HTIdx layout");

__global__ void k_hist_tidx(HistQueryParams p, const int32_t* __restrict__ vpos, int64_t nvp, HTIdx* __restrict__ out) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= nvp) return;
  const int64_t q = vpos[v];
  const int64_t c = p.pos_cell[q];
  HTIdx x;
  x.vo0 = p.voff[c];
  x.len = (uint32_t)(p.voff[c + 1] - x.vo0);
  x.kind = p.pos_kind[q];
  x.pt = p.pos_point ? p.pos_point[q] : p.pos_slot[q];
  x.lid = p.col_lid ? p.col_lid[c] : -1;
  out[v] = x;
}

template <bool PIPE, int SU>
__global__ void __launch_bounds__(ATP) k_hist_accw(HistQueryParams p, const HTIdx* __restrict__ tix, int64_t nvp,
                                                   int64_t chunk, const uint64_t* lkey_g, const int32_t* lidx_g, int WS,
                                                   int LS) {
  extern __shared__ uint4 smem4[];   // (16-byte aligned: the stage takes 16-byte stores)
  uint64_t* smem64 = reinterpret_cast<uint64_t*>(smem4);
  uint32_t* stage = reinterpret_cast<uint32_t*>(smem64);                         // STAGE_W + 8 dwords
  uint64_t* lkey = smem64 + (STAGE_W + 8) / 2;                                    // LS (compact table)
  int32_t* lidx = reinterpret_cast<int32_t*>(lkey + LS);                          // LS
  uint64_t* wacc = reinterpret_cast<uint64_t*>(lidx + LS);                        // WS * C
  uint32_t* wkind = reinterpret_cast<uint32_t*>(wacc + (size_t)WS * p.C);        // WS
  uint32_t* wpres = wkind + WS;                                                   // WS * W
  __shared__ int32_t red[4];
  __shared__ int32_t wheads[2];
  __shared__ uint64_t run_b0[WRUNS], run_b1[WRUNS];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int k = tid; k < LS; k += ATP) { lkey[k] = lkey_g[k]; lidx[k] = lidx_g[k]; }
  const int nwin = WS * p.C;
  for (int e = tid; e < nwin; e += ATP) wacc[e] = 0;
  for (int e = tid; e < WS; e += ATP) wkind[e] = 0;
  if (p.pres) for (int e = tid; e < WS * p.W; e += ATP) wpres[e] = 0;
  const Window win{wacc, wkind, wpres};
  const DictLds dict{lkey, lidx, (uint32_t)(LS - 1)};
  const int64_t v0 = (int64_t)blockIdx.x * chunk, v1 = min(nvp, v0 + chunk);
  int64_t wb = -1;
  HTIdx nx{};
  if (v0 + tid < v1) nx = tix[v0 + tid];
  for (int64_t t0 = v0; t0 < v1; t0 += ATP) {
    const bool in = t0 + tid < v1;
    const HTIdx cur = nx;
    if (t0 + ATP + tid < v1) nx = tix[t0 + ATP + tid];   // the next tile's entries, in flight from here
    const int32_t pt = in ? cur.pt : -1;
    const uint64_t vo0 = cur.vo0, vend = cur.vo0 + cur.len;
    // the tile's point range
    int32_t mn = pt >= 0 ? pt : INT32_MAX, mx = pt;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      mn = min(mn, __shfl_xor(mn, d));
      mx = max(mx, __shfl_xor(mx, d));
    }
    __syncthreads();   // the previous tile's stage and descriptors are consumed
    if (lane == 0) { red[wv * 2] = mn; red[wv * 2 + 1] = mx; }
    // runs of contiguous column bytes (the stage plan)
    const uint64_t eprev = __shfl_up(vend, 1);
    const bool inprev = __shfl_up((int)in, 1) != 0;
    bool head = in && (lane == 0 || !inprev || vo0 != eprev);
    const uint64_t hb = __ballot(head);
    if (lane == 0) wheads[wv] = __popcll(hb);
    __syncthreads();
    mn = min(red[0], red[2]);
    mx = max(red[1], red[3]);
    if (mx < 0) continue;   // (block-uniform)
    if (wb < 0 || mn < wb || mx >= wb + WS) {
      if (wb >= 0) w_flush(p, win, wb, WS);
      wb = mn;
    }
    // every wave's lane 0 starts a run, so no run crosses a wave boundary
    const int nh0 = wheads[0], nruns = nh0 + wheads[1];
    const int rid = (wv ? nh0 : 0) + (int)__popcll(hb & ((1ull << lane) - 1)) - (head ? 0 : 1);
    const bool fit = nruns <= WRUNS;
    if (fit && in) {
      const uint64_t nxt_b = __shfl_down(vo0, 1);
      const bool nxt_in = __shfl_down((int)in, 1) != 0;
      const bool last = lane == 63 || !nxt_in || nxt_b != vend;
      if (head) run_b0[rid] = vo0;
      if (last) run_b1[rid] = vend;
    }
    __syncthreads();
    // run r's dwords [w0, w1) at LDS dword base
    uint64_t my_b0 = 0;
    uint32_t my_base = 0;
    bool staged = fit;
    if (fit) {
      // each run as whole 16-byte units (16-B aligned in HBM and in LDS)
      uint32_t base = 0;
      for (int r = 0; r < nruns; r++) {
        const uint64_t w0 = (run_b0[r] >> 2) & ~3ull, w1 = (((run_b1[r] + 3) >> 2) + 3) & ~3ull;
        if (r == rid) { my_b0 = w0; my_base = base; }
        base += (uint32_t)(w1 - w0);
      }
      staged = base <= (uint32_t)STAGE_W;
      if (staged) {
        uint32_t b = 0;
        for (int r = 0; r < nruns; r++) {
          const uint64_t w0 = (run_b0[r] >> 2) & ~3ull, w1 = (((run_b1[r] + 3) >> 2) + 3) & ~3ull;
          const uint4* g = reinterpret_cast<const uint4*>(p.val) + (w0 >> 2);
          uint4* st4 = reinterpret_cast<uint4*>(stage + b);
          const uint32_t n4 = (uint32_t)((w1 - w0) >> 2);
          // up to SU loads in flight per thread (SU 16: a whole 32 KB tile in one round trip), then
          // the stores
          for (uint32_t k0 = 0; k0 < n4; k0 += SU * ATP) {
            uint4 a[SU];
#pragma unroll
            for (int u = 0; u < SU; u++) {
              const uint32_t k = k0 + u * ATP + tid;
              if (k < n4) a[u] = g[k];
            }
#pragma unroll
            for (int u = 0; u < SU; u++) {
              const uint32_t k = k0 + u * ATP + tid;
              if (k < n4) st4[k] = a[u];
            }
          }
          b += (uint32_t)(w1 - w0);
        }
        __syncthreads();
      }
    }
    if (pt < 0) continue;
    const int32_t local = pt - wb < WS ? (int32_t)(pt - wb) : -1;
    const uint8_t kind = (uint8_t)cur.kind;
    if (staged) {
      const uint64_t i0 = (uint64_t)my_base * 4 + (vo0 - my_b0 * 4);
      if (PIPE) accum_column_wp(p, win, pt, local, SrcW{stage}, i0, kind, dict, cur.lid);
      else accum_column_w(p, win, pt, local, SrcW{stage}, i0, kind, dict);
    } else {
      accum_column_w(p, win, pt, local, SrcW{reinterpret_cast<const uint32_t*>(p.val)}, vo0, kind, dict);
    }
  }
  if (wb >= 0) w_flush(p, win, wb, WS);
}

}  // namespace

// exclusive scan of n flags into out[0 .. n] (out[n] = total)
hipError_t hist_scan(const uint32_t* flag, int64_t* out, int64_t n, void** tmp, size_t* tmp_bytes, hipStream_t s) {
  hipcub::TransformInputIterator<int64_t, HWiden, const uint32_t*> in(flag, HWiden());
  size_t need = 0;
  hipError_t e = hipcub::DeviceScan::InclusiveSum(nullptr, need, in, out + 1, (int)std::max<int64_t>(1, n), s);
  if (e != hipSuccess) return e;
  if (need > *tmp_bytes) {
    if (*tmp) (void)hipFree(*tmp);
    *tmp = nullptr;
    *tmp_bytes = 0;
    if ((e = hipMalloc(tmp, need)) != hipSuccess) return e;
    *tmp_bytes = need;
  }
  if ((e = hipMemsetAsync(out, 0, 8, s)) != hipSuccess) return e;
  if (n <= 0) return hipSuccess;
  return hipcub::DeviceScan::InclusiveSum(*tmp, need, in, out + 1, (int)n, s);
}

// sparse (no downsampling) union: sort the datapoints' (group, timestamp) keys, one point per
// distinct key; pos_point[position], pt_ts / pt_group[point]; returns the point count in *n_points
hipError_t hist_sparse(const HistQueryParams& p, int64_t n_pos, uint64_t* key2, uint32_t* pos, uint32_t* pos2,
                       uint32_t* head, int64_t* incl, int64_t* pt_ts, int32_t* pt_group, int64_t* n_points,
                       void** tmp, size_t* tmp_bytes, hipStream_t s) {
  hipError_t e;
  const unsigned nb = (unsigned)((n_pos + 255) / 256);
  hipLaunchKernelGGL(k_iota, dim3(nb), dim3(256), 0, s, pos, n_pos);
  size_t need = 0;
  if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, need, (const uint64_t*)p.pos_key, key2, pos, pos2, (int)n_pos, 0,
                                              64, s)) != hipSuccess)
    return e;
  if (need > *tmp_bytes) {
    if (*tmp) (void)hipFree(*tmp);
    *tmp = nullptr;
    *tmp_bytes = 0;
    if ((e = hipMalloc(tmp, need)) != hipSuccess) return e;
    *tmp_bytes = need;
  }
  if ((e = hipcub::DeviceRadixSort::SortPairs(*tmp, need, (const uint64_t*)p.pos_key, key2, pos, pos2, (int)n_pos, 0, 64,
                                              s)) != hipSuccess)
    return e;
  hipLaunchKernelGGL(k_hist_heads, dim3(nb), dim3(256), 0, s, key2, n_pos, head);
  if ((e = hist_scan(head, incl, n_pos, tmp, tmp_bytes, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_hist_points, dim3(nb), dim3(256), 0, s, key2, pos2, n_pos, incl, p.start,
                     const_cast<int32_t*>(p.pos_point), pt_ts, pt_group, p.greedy ? p.pos_ts : nullptr);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = hipMemcpyAsync(n_points, incl + n_pos, 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  return hipStreamSynchronize(s);
}

hipError_t hist_validate(const HistLoadParams& p, hipStream_t s) {
  if (p.n_cells <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_hist_validate, dim3((unsigned)((p.n_cells + 255) / 256)), dim3(256), 0, s, p);
  return hipGetLastError();
}
hipError_t hist_walk(const HistQueryParams& p, const int64_t* gsp, int64_t G, int64_t max_spans, int64_t* sp_q,
                     int64_t* sp_ts, hipStream_t s) {
  if (G <= 0) return hipSuccess;
  if (max_spans <= 1024 * WALK_SPT) {   // a block a group, the spans in registers
    const int64_t waves = std::max<int64_t>(1, (max_spans + 64 * WALK_SPT - 1) / (64 * WALK_SPT));
    hipLaunchKernelGGL(k_hist_walk_blk, dim3((unsigned)G), dim3((unsigned)(64 * waves)), 0, s, p, gsp);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_hist_walk, dim3((unsigned)((G + 3) / 4)), dim3(256), 0, s, p, gsp, G, sp_q, sp_ts);
  return hipGetLastError();
}
hipError_t hist_slots(const HistQueryParams& p, hipStream_t s) {
  if (p.n_spans <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_hist_slots, dim3((unsigned)((p.n_spans + 127) / 128)), dim3(128), 0, s, p);
  return hipGetLastError();
}
hipError_t hist_accum(const HistQueryParams& p, int64_t n_pos, const uint64_t* lkey, const int32_t* lidx, hipStream_t s) {
  if (n_pos <= 0) return hipSuccess;
  const int64_t tiles = (n_pos + ATP - 1) / ATP;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const unsigned grid = (unsigned)std::min<int64_t>(tiles, (int64_t)cus * 4);
  if (lkey) hipLaunchKernelGGL(k_hist_accum<true>, dim3(grid), dim3(ATP), 0, s, p, n_pos, lkey, lidx);
  else hipLaunchKernelGGL(k_hist_accum<false>, dim3(grid), dim3(ATP), 0, s, p, n_pos, lkey, lidx);
  return hipGetLastError();
}
hipError_t hist_vpos(const int64_t* rlo, const int64_t* rhi, const int64_t* row_pos, int64_t n_spans, uint32_t* len,
                     int64_t* off, int32_t* vpos, int64_t* nvp, void** tmp, size_t* tmp_bytes, hipStream_t s) {
  *nvp = 0;
  if (n_spans <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_hist_vlen, dim3((unsigned)((n_spans + 255) / 256)), dim3(256), 0, s, rlo, rhi, row_pos, n_spans, len);
  hipError_t e = hist_scan(len, off, n_spans, tmp, tmp_bytes, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_hist_vpos, dim3((unsigned)n_spans), dim3(256), 0, s, rlo, row_pos, off, vpos);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = hipMemcpyAsync(nvp, off + n_spans, 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  return hipStreamSynchronize(s);
}

int hist_window_points(const HistQueryParams& p, int lslots) {
  const int64_t fixed = (int64_t)(STAGE_W + 8) * 4 + (int64_t)lslots * 12 + 256;
  const int64_t per = (int64_t)p.C * 8 + 4 + (p.pres ? (int64_t)p.W * 4 : 0);
  // three blocks a CU when a 64-point window fits in HIST_WLDS, else two with 80 KB
  const int64_t budget = HIST_WLDS;
  int64_t ws = (budget - fixed) / per;
  if (ws < 64) ws = (80 * 1024 - fixed) / per;
  if (ws < 32) return 0;
  if (opt(OPT_HIST_WS) > 0) ws = std::min<int64_t>(ws, opt(OPT_HIST_WS));   // tests: tiny windows
  return (int)std::min<int64_t>(ws, 4096);
}

hipError_t hist_accum_window(const HistQueryParams& p, const int32_t* vpos, int64_t nvp, const uint64_t* lkey,
                             const int32_t* lidx, int lslots, void* tix_buf, hipStream_t s) {
  if (nvp <= 0) return hipSuccess;
  HTIdx* tix = reinterpret_cast<HTIdx*>(tix_buf);
  hipLaunchKernelGGL(k_hist_tidx, dim3((unsigned)((nvp + 255) / 256)), dim3(256), 0, s, p, vpos, nvp, tix);
  const int WS = hist_window_points(p, lslots);
  if (WS <= 0 || !lkey) return hipErrorInvalidValue;
  const size_t lds = (size_t)(STAGE_W + 8) * 4 + (size_t)lslots * 12 + (size_t)WS * p.C * 8 + (size_t)WS * 4 +
                     (p.pres ? (size_t)WS * p.W * 4 : 0);
  // the pipelined bucket loop with 4 staging loads in flight a thread.  r03o sweep of the
  // histogram bench query: 52 KB window + 4 in flight 2.60 ms; + 16 2.77; 80 KB 3.21 / 3.40; 160 KB
  // 5.08; the unpipelined loop lost as well (those variants are gone).  Round 6: the next
  // tile's stage units in registers during the parse measured slower (1.80 vs 1.54 ms,
  // profiles/r06as/): the parse, not the staging round trips, holds the tile
  const void* kf = reinterpret_cast<const void*>(&k_hist_accw<true, 4>);
  hipError_t e = hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t tiles = (nvp + ATP - 1) / ATP;
  const int64_t per_cu = std::max<int64_t>(1, std::min<int64_t>(4, (int64_t)(160 * 1024) / (int64_t)lds));
  const int64_t want = std::min<int64_t>(tiles, (int64_t)cus * per_cu);
  const int64_t chunk = ((tiles + want - 1) / want) * ATP;
  const unsigned grid = (unsigned)((nvp + chunk - 1) / chunk);
  hipLaunchKernelGGL((k_hist_accw<true, 4>), dim3(grid), dim3(ATP), lds, s, p, tix, nvp, chunk, lkey, lidx, WS, lslots);
  return hipGetLastError();
}
hipError_t hist_layout_index(int64_t n_cells, const uint64_t* voff, const uint8_t* val, const uint8_t* status,
                             uint32_t* head, int64_t* excl, int32_t* col_lid, int32_t* lay_col, int64_t* n_layouts,
                             void** tmp, size_t* tmp_bytes, hipStream_t s) {
  *n_layouts = 0;
  if (n_cells <= 0) return hipSuccess;
  const unsigned nb = (unsigned)((n_cells + 255) / 256);
  hipLaunchKernelGGL(k_hist_layhead, dim3(nb), dim3(256), 0, s, n_cells, voff, val, status, head);
  hipError_t e = hist_scan(head, excl, n_cells, tmp, tmp_bytes, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_hist_laylid, dim3(nb), dim3(256), 0, s, n_cells, voff, val, status, head, excl, col_lid, lay_col);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = hipMemcpyAsync(n_layouts, excl + n_cells, 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  return hipStreamSynchronize(s);
}
hipError_t hist_layout_di(int64_t n_layouts, const int32_t* lay_col, const int32_t* lay_off, const uint64_t* voff,
                          const uint8_t* val, const uint64_t* hkey, const int32_t* hidx, int32_t* lay_di, hipStream_t s) {
  if (n_layouts <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_hist_laydi, dim3((unsigned)((n_layouts + 255) / 256)), dim3(256), 0, s, n_layouts, lay_col, lay_off,
                     voff, val, hkey, hidx, lay_di);
  return hipGetLastError();
}
hipError_t hist_flags(const HistQueryParams& p, uint32_t* flag, hipStream_t s) {
  if (p.n_points <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_hist_flags, dim3((unsigned)((p.n_points + 255) / 256)), dim3(256), 0, s, p, flag);
  return hipGetLastError();
}
hipError_t hist_final(const HistQueryParams& p, hipStream_t s) {
  if (p.n_points <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_hist_final, dim3((unsigned)((p.n_points + 255) / 256)), dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace tsdb
