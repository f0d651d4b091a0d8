// Query-time compaction: what TSDB.compact(row) does to every row a
// query scans (SaltScanner.processRow :802-830 -> CompactionQueue.Compaction.compact
// :330-385), for every row at once.  The reference's per-row heap merge of column iterators
// (defaultMergeDataPoints :512-545 over ColumnDatapointIterator :63-205) becomes:
//   k_cmp_cols     one thread per column: its kind (datapoints / append / ignored), the 2-byte
//                  fixups (Internal.fixFloatingPointValue / fixQualifierFlags :535-591) and its
//                  datapoint count; errors recorded per row
//   k_cmp_explode  one thread per column: an entry per datapoint, keyed row << 22 | offset ms
//   radix sort     (stable: equal keys keep scan order -- column, then position)
//   k_cmp_dedup    one thread per run of equal keys: the heap's order at one offset is newest
//                  column first, so the kept datapoint is the newest column's; the others must
//                  hold the same bytes unless fix_duplicates (IllegalDataException); a later
//                  pair of the same append column replaces an earlier one
//                  (AppendDataPoints.parseKeyValue :110-240)
//   scans          kept qualifier / value bytes, kept and millisecond datapoints
//   k_cmp_rows     one thread per row: its compacted size and meta byte (buildCompactedColumn
//                  :547-566), or the single column as stored (noMergesOrFixups :311-328)
//   k_cmp_write    one thread per kept datapoint: its bytes at the row's destination
//   k_cmp_rowfix   one thread per row: stored single columns and meta bytes.
// The heap merge equals the sorted merge when every column's datapoints are in time order,
// which compactions write; a compacted column out of order is reported NOT_IMPLEMENTED.
// When every row of a chunk has at most 4096 datapoints (the common case: an hour row), the
// explode / sort / dedup / scans / write steps run instead per row in one block's LDS
// (k_cmp_row, below): no global entry arrays, no global radix sort.
#include "kcommon.h"

#include <hipcub/hipcub.hpp>

namespace tsdb {

namespace {

__device__ __forceinline__ bool cmp_in_ms(uint8_t b) { return (b & 0xF0) == 0xF0; }
__device__ __forceinline__ uint32_t cmp_be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
__device__ __forceinline__ uint32_t cmp_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
// Internal.getOffsetFromQualifier in ms (< 2^22 for both widths)
__device__ __forceinline__ uint32_t cmp_off(const uint8_t* q, int eq) {
  return eq == 4 ? ((cmp_be32(q) & 0x0FFFFFC0u) >> 6) : (cmp_be16(q) >> 4) * 1000u;
}
__device__ __forceinline__ void cmp_fail(int32_t* row_err, int64_t row, int32_t code) {
  atomicCAS(&row_err[row], 0, code);
}

// the row of every column: one wave a row, its lanes striding over the row's columns (coalesced
// stores; a thread a row wrote an hour row's 3600 entries one after the other)
__global__ __launch_bounds__(256) void k_cmp_colrow(CmpParams p) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= p.n_rows) return;
  const int64_t c1 = p.row_col_ptr[r + 1];
  for (int64_t c = p.row_col_ptr[r] + (threadIdx.x & 63); c < c1; c += 64) p.col_row[c] = (int32_t)r;
}

// Walk of a datapoint column (ColumnDatapointIterator.update / advance), shared by the count
// and the explode passes.  Returns false on a malformed column.
template <class F>
__device__ __forceinline__ bool walk_data(const uint8_t* q, int64_t ql, int64_t vlen, uint8_t fixed_flags, F&& f) {
  int64_t qi = 0, vi = 0;
  while (qi < ql && vi < vlen) {
    const int eq = cmp_in_ms(q[qi]) ? 4 : 2;
    if (qi + eq > ql) return false;                       // ArrayIndexOutOfBounds
    const uint8_t fl = ql == 2 ? fixed_flags : q[qi + eq - 1];
    const int evl = (fl & 7) + 1;
    if (vi + evl > vlen) return false;                    // value shorter than its qualifiers
    f(qi, vi, eq, evl, cmp_off(q + qi, eq));
    qi += eq;
    vi += evl;
  }
  return true;
}
template <class F>
__device__ __forceinline__ bool walk_append(const uint8_t* v, int64_t vl, F&& f) {
  int64_t idx = 0;
  while (idx < vl) {
    const int eq = cmp_in_ms(v[idx]) ? 4 : 2;
    if (idx + eq > vl) return false;
    const int evl = (v[idx + eq - 1] & 7) + 1;
    if (idx + eq + evl > vl) return false;
    f(idx, idx + eq, eq, evl, cmp_off(v + idx, eq));
    idx += eq + evl;
  }
  return true;
}

// column offsets: 64-bit, or (W32, the one-pass path when a chunk's blobs are under 4 GB) 32-bit
template <bool W32>
__device__ __forceinline__ uint64_t col_q(const CmpParams& p, int64_t c) {
  if constexpr (W32) return (uint64_t)p.col_qo32[c];
  else return p.col_qo[c];
}
template <bool W32>
__device__ __forceinline__ uint64_t col_v(const CmpParams& p, int64_t c) {
  if constexpr (W32) return (uint64_t)p.col_vo32[c];
  else return p.col_vo[c];
}

// One column: kind, fixups, datapoint count, errors.  Returns whether it joins the heap.  *qb /
// *vb: bounds of the compacted bytes it can contribute (a data column keeps its qualifier width
// and value bytes; an append column's qualifiers and values both come out of its value)
template <bool W32 = false>
__device__ __forceinline__ bool cmp_col(const CmpParams& p, int64_t c, int64_t row, int64_t* qb = nullptr,
                                        int64_t* vb = nullptr, int64_t* nout = nullptr, bool store = true,
                                        uint32_t* info_out = nullptr) {
  const uint64_t qo = col_q<W32>(p, c), vo = col_v<W32>(p, c);
  const int64_t ql = (int64_t)(col_q<W32>(p, c + 1) - qo), vl = (int64_t)(col_v<W32>(p, c + 1) - vo);
  const uint8_t* q = p.q + qo;
  const uint8_t* v = p.v + vo;
  uint32_t kind = CMP_IGNORE, info = 0;
  int64_t n = 0;
  int32_t err = 0;
  bool heap = false;
  if (ql & 1) {
    if (ql == 3 && q[0] == 0x05) {   // AppendDataPoints.APPEND_COLUMN_PREFIX
      kind = CMP_APPEND;
      if (!walk_append(v, vl, [&](int64_t, int64_t, int, int, uint32_t) { n++; })) err = TSDB_E_ILLEGAL_DATA;
      heap = n > 0;
    }
    // annotations, histograms, other prefixes: not datapoints
  } else if (ql > 0) {
    kind = CMP_DATA;
    heap = true;
    int64_t vstart = 0, vlen = vl;
    uint8_t ff = 0;
    bool fixed = false;
    if (ql == 2) {   // ColumnDatapointIterator.checkForFixup :74-89
      const uint8_t q1 = q[1];
      if ((q1 & 8) && (q1 & 7) == 3 && vl == 8) {
        if (v[0] | v[1] | v[2] | v[3]) err = TSDB_E_ILLEGAL_DATA;   // "first 4 bytes are expected to be zeros"
        vstart = 4;
        vlen = 4;
        fixed = true;
      }
      ff = (uint8_t)((q1 & ~7) | (uint8_t)(vlen - 1));
      if (ff != q1) fixed = true;
    }
    if (vlen == 0) err = TSDB_E_NOT_IMPLEMENTED;   // a datapoint column without a value
    uint32_t prev = 0;
    bool sorted = true;
    if (!err && !walk_data(q, ql, vlen, ff, [&](int64_t, int64_t, int, int, uint32_t t) {
          if (n > 0 && t < prev) sorted = false;
          prev = t;
          n++;
        }))
      err = TSDB_E_ILLEGAL_DATA;
    if (!err && !sorted) err = TSDB_E_NOT_IMPLEMENTED;   // a compacted column out of time order
    info = (vstart ? 4u : 0u) | (fixed ? 8u : 0u) | ((uint32_t)ff << 8);
  }
  if (err) {
    cmp_fail(p.row_err, row, err);
    n = 0;
  }
  if (store) {
    p.col_n[c] = n;
    p.col_info[c] = kind | info;
  }
  if (info_out) *info_out = kind | info;
  if (nout) *nout = n;
  if (qb) {
    *qb = n == 0 ? 0 : (kind == CMP_APPEND ? vl : ql);
    *vb = n == 0 ? 0 : (kind == CMP_APPEND ? vl : vl - ((info & 4) ? 4 : 0));
  }
  return heap;
}

__global__ __launch_bounds__(256) void k_cmp_cols(CmpParams p) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = c < p.n_cols;
  bool heap = false;
  const int64_t row = valid ? p.col_row[c] : -1;
  if (valid) heap = cmp_col(p, c, row);
  // per-row heap counts, aggregated per wave: a row's columns are consecutive, so a wave
  // covers few rows and each of them takes one atomic instead of one per column
  const int lane = (int)(threadIdx.x & 63);
  const int64_t prev_row = __shfl_up(row, 1);
  const bool leader = valid && (lane == 0 || prev_row != row);
  const uint64_t lead_mask = __ballot(leader);
  const uint64_t heap_mask = __ballot(valid && heap);
  if (leader) {
    const uint64_t after = lane == 63 ? 0ull : (lead_mask & ~((2ull << lane) - 1));
    const int end = after ? __builtin_ctzll(after) : 64;
    const uint64_t seg = (end == 64 ? ~0ull : ((1ull << end) - 1)) & ~((1ull << lane) - 1);
    const uint64_t hm = heap_mask & seg;
    if (hm) {
      atomicAdd(&p.row_heap[row], (int32_t)__popcll(hm));
      const int top = 63 - __builtin_clzll(hm);
      atomicMax((unsigned long long*)&p.row_one[row], (unsigned long long)(c - lane + top));
    }
  }
}

__global__ __launch_bounds__(256) void k_cmp_explode(CmpParams p) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= p.n_cols || p.col_n[c] == 0) return;
  const uint64_t row = (uint64_t)p.col_row[c];
  const uint64_t qo = p.col_qo[c], vo = p.col_vo[c];
  const int64_t ql = (int64_t)(p.col_qo[c + 1] - qo), vl = (int64_t)(p.col_vo[c + 1] - vo);
  const uint32_t info = p.col_info[c];
  int64_t e = p.col_off[c];
  auto put = [&](int64_t qpos, int64_t vpos, int, int, uint32_t t) {
    p.key[e] = (row << 22) | t;
    p.idx[e] = (uint32_t)e;
    p.ent_col[e] = (uint32_t)c;
    p.ent_qo[e] = (uint32_t)qpos;
    p.ent_vo[e] = (uint32_t)vpos;
    e++;
  };
  if ((info & 3) == CMP_APPEND) {
    walk_append(p.v + vo, vl, put);
  } else {
    const int64_t vstart = (info & 4) ? 4 : 0;
    walk_data(p.q + qo, ql, vl - vstart, (uint8_t)(info >> 8),
              [&](int64_t qi, int64_t vi, int eq, int evl, uint32_t t) { put(qi, vstart + vi, eq, evl, t); });
  }
}

// qualifier / value of entry e: pointers and lengths (fixups applied)
struct CmpEnt {
  const uint8_t* qp;
  const uint8_t* vp;
  int eq, evl;
  uint8_t fixed_q1;   // the replacement second qualifier byte (2-byte fixed columns), else 0
  bool fix;
};
__device__ __forceinline__ CmpEnt cmp_ent(const CmpParams& p, uint32_t e) {
  CmpEnt r;
  const uint32_t c = p.ent_col[e];
  const uint32_t info = p.col_info[c];
  const uint8_t* vb = p.v + p.col_vo[c];
  const int64_t ql = (int64_t)(p.col_qo[c + 1] - p.col_qo[c]);
  r.fix = false;
  r.fixed_q1 = 0;
  if ((info & 3) == CMP_APPEND) {
    r.qp = vb + p.ent_qo[e];
  } else {
    r.qp = p.q + p.col_qo[c] + p.ent_qo[e];
    if (ql == 2 && (info & 8)) { r.fix = true; r.fixed_q1 = (uint8_t)(info >> 8); }
  }
  r.eq = cmp_in_ms(r.qp[0]) ? 4 : 2;
  const uint8_t fl = r.fix ? r.fixed_q1 : r.qp[r.eq - 1];
  r.evl = (fl & 7) + 1;
  r.vp = vb + p.ent_vo[e];
  return r;
}

// ColumnDatapointIterator.getCellValueAsDouble (:201-211) of an entry: false where ByteBuffer would
// read past the value (a float of a length other than 4 / 8, an integer of 3, 5, 6 or 7 bytes)
__device__ __forceinline__ bool cmp_dval(const CmpEnt& e, double* out) {
  const uint8_t fl = e.fix ? e.fixed_q1 : e.qp[e.eq - 1];
  const uint8_t* v = e.vp;
  uint64_t b = 0;
  for (int i = 0; i < e.evl; i++) b = (b << 8) | v[i];
  if (fl & 8) {
    if (e.evl == 4) { *out = (double)__uint_as_float((uint32_t)b); return true; }
    if (e.evl == 8) { *out = __longlong_as_double((long long)b); return true; }
    return false;
  }
  if (e.evl == 1) *out = (double)(int8_t)b;
  else if (e.evl == 2) *out = (double)(int16_t)b;
  else if (e.evl == 4) *out = (double)(int32_t)b;
  else if (e.evl == 8) *out = (double)(int64_t)b;
  else return false;
  return true;
}

// the single column a row keeps as stored (noMergesOrFixups :311-328): no merge, no value read
__device__ __forceinline__ bool cmp_as_stored(const CmpParams& p, int64_t r) {
  if (p.row_heap[r] != 1) return false;
  const int64_t c = p.row_one[r];
  const uint32_t info = p.col_info[c];
  const int64_t ql = (int64_t)(p.col_qo[c + 1] - p.col_qo[c]);
  return (info & 3) == CMP_DATA && !(info & 8) && (ql == 2 || (ql == 4 && cmp_in_ms(p.q[p.col_qo[c]])));
}

// dtcsMergeDataPoints (CompactionQueue.java:508-547) over one run [i, j) of equal keys.  The heap
// visits the run newest column first (equal write timestamps: scan order); the head's value is
// replaced by each later one that is strictly greater (p.dtcs 1, use_max_value) / smaller (2).
// So the kept entry is the head when its value is NaN, else the first in heap order holding the
// extreme of the non-NaN values.  No duplicate exception.  The meta byte reads the kept
// column's isMilliseconds() after the run advanced it (:544-545): the resolution of the column's
// datapoint after its last one in the run (or of that one when it was the column's last); klen
// bit 1 carries that flag instead of the kept entry's own width.
__device__ void cmp_dedup_dtcs(const CmpParams& p, int64_t i, int64_t j, int64_t row) {
  const bool merged = !cmp_as_stored(p, row);
  auto superseded = [&](int64_t t) {
    const uint32_t c = p.ent_col[p.idx2[t]];
    return (p.col_info[c] & 3) == CMP_APPEND && t + 1 < j && p.ent_col[p.idx2[t + 1]] == c;
  };
  // heap rank of t over u: newer column, then scan order
  auto before = [&](int64_t t, int64_t u) {
    const int64_t a = p.col_ts ? p.col_ts[p.ent_col[p.idx2[t]]] : 0, b = p.col_ts ? p.col_ts[p.ent_col[p.idx2[u]]] : 0;
    return a != b ? a > b : t < u;
  };
  int64_t head = -1, best = -1;
  double ext = 0;
  bool any = false, bad = false;
  for (int64_t t = i; t < j; t++) {
    p.klen[t] = 0;
    if (superseded(t)) continue;
    double x = 0;
    if (!cmp_dval(cmp_ent(p, p.idx2[t]), &x)) { bad = true; continue; }
    if (head < 0 || before(t, head)) head = t;
    if (x != x) continue;
    if (!any || (p.dtcs == 1 ? x > ext : x < ext)) { ext = x; any = true; }
  }
  if (bad && merged) cmp_fail(p.row_err, row, TSDB_E_RUNTIME);   // BufferUnderflowException
  if (head < 0) return;
  double hv = 0;
  (void)cmp_dval(cmp_ent(p, p.idx2[head]), &hv);
  if (hv != hv || !any) {
    best = head;
  } else {
    for (int64_t t = i; t < j; t++) {
      if (superseded(t)) continue;
      double x = 0;
      if (!cmp_dval(cmp_ent(p, p.idx2[t]), &x) || !(x == ext)) continue;
      if (best < 0 || before(t, best)) best = t;
    }
  }
  const uint32_t e = p.idx2[best];
  const uint32_t c = p.ent_col[e];
  const CmpEnt kb = cmp_ent(p, e);
  // the kept column's last entry in the run, then its next datapoint
  int64_t last = best;
  for (int64_t t = i; t < j; t++)
    if (p.ent_col[p.idx2[t]] == c && p.ent_qo[p.idx2[t]] > p.ent_qo[p.idx2[last]]) last = t;
  const uint32_t el = p.idx2[last];
  const CmpEnt kl = cmp_ent(p, el);
  bool ms = kl.eq == 4;
  const uint32_t info = p.col_info[c];
  if ((info & 3) == CMP_APPEND) {
    // the parsed append column iterates its pairs by offset: the column's next entry in key order
    for (int64_t t = j; t < p.n_ent && (int64_t)(p.key2[t] >> 22) == row; t++)
      if (p.ent_col[p.idx2[t]] == c) {
        int64_t u = t;   // (the surviving pair of that offset: the column's last one there)
        while (u + 1 < p.n_ent && p.key2[u + 1] == p.key2[t] && p.ent_col[p.idx2[u + 1]] == c) u++;
        ms = cmp_ent(p, p.idx2[u]).eq == 4;
        break;
      }
  } else {
    const uint64_t qo = p.col_qo[c];
    const int64_t ql = (int64_t)(p.col_qo[c + 1] - qo);
    const int64_t vstart = (info & 4) ? 4 : 0;
    const int64_t vlen = (int64_t)(p.col_vo[c + 1] - p.col_vo[c]) - vstart;
    const int64_t qn = (int64_t)p.ent_qo[el] + kl.eq, vn = (int64_t)p.ent_vo[el] - vstart + kl.evl;
    if (qn < ql && vn < vlen) ms = cmp_in_ms(p.q[qo + qn]);
  }
  p.klen[best] = 1u | ((ms ? 1u : 0u) << 1) | ((uint32_t)kb.eq << 2) | ((uint32_t)kb.evl << 8);
}

__global__ __launch_bounds__(256) void k_cmp_dedup(CmpParams p) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n_ent) return;
  const uint64_t k = p.key2[i];
  if (i > 0 && p.key2[i - 1] == k) return;   // not the first of its run
  int64_t j = i + 1;
  while (j < p.n_ent && p.key2[j] == k) j++;
  const int64_t row = (int64_t)(k >> 22);
  if (p.dtcs) {
    cmp_dedup_dtcs(p, i, j, row);
    return;
  }
  // a pair an append column repeats later is replaced (TreeMap.put); the newest column wins
  auto superseded = [&](int64_t t) {
    const uint32_t c = p.ent_col[p.idx2[t]];
    return (p.col_info[c] & 3) == CMP_APPEND && t + 1 < j && p.ent_col[p.idx2[t + 1]] == c;
  };
  int64_t best = -1;
  int64_t best_ts = 0;
  for (int64_t t = i; t < j; t++) {
    if (superseded(t)) continue;
    const uint32_t c = p.ent_col[p.idx2[t]];
    const int64_t ts = p.col_ts ? p.col_ts[c] : 0;
    if (best < 0 || ts > best_ts) { best = t; best_ts = ts; }
  }
  const CmpEnt kb = cmp_ent(p, p.idx2[best]);
  for (int64_t t = i; t < j; t++) {
    if (t == best) {
      p.klen[t] = 1u | ((kb.eq == 4 ? 1u : 0u) << 1) | ((uint32_t)kb.eq << 2) | ((uint32_t)kb.evl << 8);
      continue;
    }
    p.klen[t] = 0;
    if (superseded(t) || p.fix_dup) continue;
    const CmpEnt o = cmp_ent(p, p.idx2[t]);   // getCopyOfCurrentValue vs the kept segment
    bool same = o.evl == kb.evl;
    for (int b = 0; same && b < o.evl; b++) same = o.vp[b] == kb.vp[b];
    if (!same) cmp_fail(p.row_err, row, TSDB_E_ILLEGAL_DATA);
  }
}

struct KeptField {
  int f;
  __host__ __device__ int64_t operator()(uint32_t x) const {
    return f == 0 ? (int64_t)((x >> 2) & 7) * (x & 1) : f == 1 ? (int64_t)(x >> 8) * (x & 1)
                  : f == 2 ? (int64_t)(x & 1) : (int64_t)((x >> 1) & 1);
  }
};

__device__ __forceinline__ int64_t lower_bound_u64(const uint64_t* a, int64_t n, uint64_t x) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (a[m] < x) lo = m + 1;
    else hi = m;
  }
  return lo;
}

__global__ __launch_bounds__(256) void k_cmp_rows(CmpParams p) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= p.n_rows) return;
  const int64_t lo = lower_bound_u64(p.key2, p.n_ent, (uint64_t)r << 22);
  const int64_t hi = lower_bound_u64(p.key2, p.n_ent, (uint64_t)(r + 1) << 22);
  p.row_lo[r] = lo;
  p.row_meta[r] = 0;
  p.row_q[r] = p.row_v[r] = 0;
  if (p.row_err[r] || p.row_heap[r] == 0) { p.row_state[r] = 0; return; }
  if (p.row_heap[r] == 1) {   // noMergesOrFixups: one 2-byte or one 4-byte ms column, no fixup
    const int64_t c = p.row_one[r];
    const uint32_t info = p.col_info[c];
    const int64_t ql = (int64_t)(p.col_qo[c + 1] - p.col_qo[c]);
    if ((info & 3) == CMP_DATA && !(info & 8) && (ql == 2 || (ql == 4 && cmp_in_ms(p.q[p.col_qo[c]])))) {
      p.row_state[r] = 2;
      p.row_q[r] = ql;
      p.row_v[r] = (int64_t)(p.col_vo[c + 1] - p.col_vo[c]);
      return;
    }
  }
  const int64_t cnt = p.sc[hi] - p.sc[lo];
  if (cnt == 0) { p.row_state[r] = 0; return; }
  const int64_t ms = p.sm[hi] - p.sm[lo];
  p.row_state[r] = 1;
  p.row_q[r] = p.sq[hi] - p.sq[lo];
  p.row_v[r] = p.sv[hi] - p.sv[lo] + (cnt > 1 ? 1 : 0);
  p.row_meta[r] = (ms > 0 && ms < cnt) ? 1 : 0;   // Const.MS_MIXED_COMPACT
}

__global__ __launch_bounds__(256) void k_cmp_write(CmpParams p) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n_ent || !(p.klen[i] & 1)) return;
  const int64_t r = (int64_t)(p.key2[i] >> 22);
  if (p.row_state[r] != 1 || p.row_dq[r] < 0) return;
  const int64_t lo = p.row_lo[r];
  const int64_t dq = p.row_dq[r] + (p.sq[i] - p.sq[lo]);
  const int64_t dv = p.row_dv[r] + (p.sv[i] - p.sv[lo]);
  const CmpEnt e = cmp_ent(p, p.idx2[i]);
  for (int b = 0; b < e.eq; b++) p.out_q[dq + b] = (e.fix && b == 1) ? e.fixed_q1 : e.qp[b];
  for (int b = 0; b < e.evl; b++) p.out_v[dv + b] = e.vp[b];
}

__global__ __launch_bounds__(256) void k_cmp_rowfix(CmpParams p) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= p.n_rows || p.row_dq[r] < 0) return;
  if (p.row_state[r] == 2) {
    const int64_t c = p.row_one[r];
    const uint8_t* qs = p.q + p.col_qo[c];
    const uint8_t* vs = p.v + p.col_vo[c];
    for (int64_t b = 0; b < p.row_q[r]; b++) p.out_q[p.row_dq[r] + b] = qs[b];
    for (int64_t b = 0; b < p.row_v[r]; b++) p.out_v[p.row_dv[r] + b] = vs[b];
  } else if (p.row_state[r] == 1) {
    const int64_t lo = p.row_lo[r];
    const int64_t hi = lower_bound_u64(p.key2, p.n_ent, (uint64_t)(r + 1) << 22);
    if (p.sc[hi] - p.sc[lo] > 1) p.out_v[p.row_dv[r] + p.row_v[r] - 1] = p.row_meta[r];
  }
}

inline unsigned blocks_of(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + 255) / 256); }

// exclusive scan into out[0 .. n] (n + 1 values) of f(klen[i])
hipError_t scan_field(const CmpParams& p, int f, int64_t* out, void* tmp, size_t& bytes, hipStream_t s) {
  hipcub::TransformInputIterator<int64_t, KeptField, const uint32_t*> in(p.klen, KeptField{f});
  if (!tmp) return hipcub::DeviceScan::InclusiveSum(nullptr, bytes, in, out + 1, (int)p.n_ent, s);
  hipError_t e = hipMemsetAsync(out, 0, 8, s);
  if (e != hipSuccess) return e;
  if (p.n_ent == 0) return hipSuccess;
  return hipcub::DeviceScan::InclusiveSum(tmp, bytes, in, out + 1, (int)p.n_ent, s);
}

}  // namespace

hipError_t cmp_analyze(CmpParams& p, void** tmp, size_t* tmp_bytes, hipStream_t s) {
  if (p.n_rows > 0) hipLaunchKernelGGL(k_cmp_colrow, dim3((unsigned)((p.n_rows + 3) / 4)), dim3(256), 0, s, p);
  if (p.n_cols > 0) hipLaunchKernelGGL(k_cmp_cols, dim3(blocks_of(p.n_cols)), dim3(256), 0, s, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // col_off = exclusive sum of col_n (n_cols + 1 values)
  size_t need = 0;
  e = hipcub::DeviceScan::InclusiveSum(nullptr, need, p.col_n, p.col_off + 1, (int)std::max<int64_t>(1, p.n_cols), s);
  if (e != hipSuccess) return e;
  if (need > *tmp_bytes) {
    if (*tmp) (void)hipFree(*tmp);
    *tmp = nullptr;
    *tmp_bytes = 0;
    e = hipMalloc(tmp, need);
    if (e != hipSuccess) return e;
    *tmp_bytes = need;
  }
  e = hipMemsetAsync(p.col_off, 0, 8, s);
  if (e != hipSuccess || p.n_cols == 0) return e;
  size_t b = *tmp_bytes;
  return hipcub::DeviceScan::InclusiveSum(*tmp, b, p.col_n, p.col_off + 1, (int)p.n_cols, s);
}

hipError_t cmp_entries(CmpParams& p, void** tmp, size_t* tmp_bytes, int end_bit, hipStream_t s) {
  hipError_t e;
  if (p.n_ent > 0) {
    hipLaunchKernelGGL(k_cmp_explode, dim3(blocks_of(p.n_cols)), dim3(256), 0, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  size_t need = 0, b = 0;
  e = hipcub::DeviceRadixSort::SortPairs(nullptr, b, p.key, p.key2, p.idx, p.idx2, (int)std::max<int64_t>(1, p.n_ent), 0,
                                         end_bit, s);
  if (e != hipSuccess) return e;
  need = b;
  for (int f = 0; f < 4; f++) {
    b = 0;
    if ((e = scan_field(p, f, p.sq, nullptr, b, s)) != hipSuccess) return e;
    need = std::max(need, b);
  }
  if (need > *tmp_bytes) {
    if (*tmp) (void)hipFree(*tmp);
    *tmp = nullptr;
    *tmp_bytes = 0;
    if ((e = hipMalloc(tmp, need)) != hipSuccess) return e;
    *tmp_bytes = need;
  }
  if (p.n_ent > 0) {
    b = *tmp_bytes;
    e = hipcub::DeviceRadixSort::SortPairs(*tmp, b, p.key, p.key2, p.idx, p.idx2, (int)p.n_ent, 0, end_bit, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_cmp_dedup, dim3(blocks_of(p.n_ent)), dim3(256), 0, s, p);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  int64_t* outs[4] = {p.sq, p.sv, p.sc, p.sm};
  for (int f = 0; f < 4; f++) {
    b = *tmp_bytes;
    if ((e = scan_field(p, f, outs[f], *tmp, b, s)) != hipSuccess) return e;
  }
  if (p.n_rows > 0) hipLaunchKernelGGL(k_cmp_rows, dim3(blocks_of(p.n_rows)), dim3(256), 0, s, p);
  return hipGetLastError();
}

// dst[i] = src[i] - base over n values; bad |= 1 when the values decrease or start below base
__global__ __launch_bounds__(256) void k_cmp_rebase(const uint64_t* src, uint64_t* dst, int64_t n, uint64_t base,
                                                    int32_t* bad, uint32_t* dst32) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t v = src[i];
  if (v < base || (i + 1 < n && src[i + 1] < v)) atomicOr(bad, 1);
  dst[i] = v - base;
  if (dst32) dst32[i] = (uint32_t)(v - base);   // (the caller checked the chunk's bytes fit 32 bits)
}

hipError_t cmp_rebase(const uint64_t* src, uint64_t* dst, int64_t n, uint64_t base, int32_t* bad, hipStream_t s,
                      uint32_t* dst32) {
  if (n > 0) hipLaunchKernelGGL(k_cmp_rebase, dim3(blocks_of(n)), dim3(256), 0, s, src, dst, n, base, bad, dst32);
  return hipGetLastError();
}

hipError_t cmp_write(const CmpParams& p, hipStream_t s) {
  if (p.n_ent > 0) hipLaunchKernelGGL(k_cmp_write, dim3(blocks_of(p.n_ent)), dim3(256), 0, s, p);
  if (p.n_rows > 0) hipLaunchKernelGGL(k_cmp_rowfix, dim3(blocks_of(p.n_rows)), dim3(256), 0, s, p);
  return hipGetLastError();
}

// ---- the per-row path ----------------------------------------------------------------------
// A scan row holds at most a few thousand datapoints (3600 a second-resolution hour), so one
// block takes a whole row.  Sizing pass (k_cmp_row): its columns' datapoints are exploded into
// LDS -- sort key (offset ms << 12 | entry; the entry ordinal keeps scan order among equal
// offsets, as the global sort's stability does) and everything later steps need (source
// offsets, lengths, fixup / append flags, column) -- bitonic-sorted there, deduplicated run by
// run (a run of one offset is the common case and touches no global memory; longer runs apply
// the heap's newest-column rule, append repeats and the duplicate check), prefix-summed; the
// row's sizes go to the host and its kept datapoints, in output order with their source and
// destination offsets, to a list (16 B each).  Write pass (k_cmp_rowwrite, after the host
// layout): one block per row streams its list and copies the bytes.
constexpr int CMP_ROW_CAP = 4096;   // datapoints per row (12 bits of the key)
constexpr int CMP_ROW_THREADS = 1024;
constexpr uint64_t CMP_KEPT = 1ULL << 62;   // in a sorted key: the datapoint is kept

__global__ __launch_bounds__(256) void k_cmp_rowmax(CmpParams p, uint32_t* out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t n = 0, nc = 0, span = 0;
  if (r < p.n_rows) {
    const int64_t c0 = p.row_col_ptr[r], c1 = p.row_col_ptr[r + 1];
    const int64_t e = p.col_off[c1] - p.col_off[c0];
    const uint64_t qs = p.col_qo[c1] - p.col_qo[c0], vs = p.col_vo[c1] - p.col_vo[c0];
    n = (uint32_t)min<int64_t>(e, 0xFFFFFFFFll);
    nc = (uint32_t)min<int64_t>(c1 - c0, 0xFFFFFFFFll);
    span = (uint32_t)min<uint64_t>(max(qs, vs), 0xFFFFFFFFull);
  }
  for (int o = 32; o > 0; o >>= 1) {
    n = max(n, (uint32_t)__shfl_xor((int)n, o));
    nc = max(nc, (uint32_t)__shfl_xor((int)nc, o));
    span = max(span, (uint32_t)__shfl_xor((int)span, o));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(&out[0], n);
    atomicMax(&out[1], nc);
    atomicMax(&out[2], span);
  }
}

// per-entry flags in LDS: bit0 ms (4-byte qualifier), bits1-3 value length - 1, bit4 the
// 2-byte qualifier's flags byte is fixed up, bit5 append column (qualifier inside the value)
__device__ __forceinline__ int em_eq(uint32_t em) { return (em & 1) ? 4 : 2; }
__device__ __forceinline__ int em_evl(uint32_t em) { return (int)((em >> 1) & 7) + 1; }

// block-wide exclusive scan of one int per thread (LDS scratch of >= 16 + 1 ints); returns
// the thread's offset, *total = the block's sum
__device__ __forceinline__ int block_excl_scan(int x, int* sh, int* total) {
  const int t = threadIdx.x;
  const int nw = (int)(blockDim.x >> 6);
  const int lane = t & 63;
  const int v = wave_incl_sum_dpp(x);   // inclusive wave scan (DPP: no LDS permutes)
  if (lane == 63) sh[t >> 6] = v;
  __syncthreads();
  int base = 0, all = 0;
  for (int w = 0; w < nw; w++) {
    const int sw = sh[w];
    base += w < (t >> 6) ? sw : 0;
    all += sw;
  }
  __syncthreads();
  *total = all;
  return base + v - x;
}

// two block-wide exclusive scans sharing one pair of barriers (LDS scratch >= 2 x 16 ints)
__device__ __forceinline__ int block_excl_scan2(int x, int y, int* sh, int* totx, int* oy, int* toty) {
  const int t = threadIdx.x;
  const int nw = (int)(blockDim.x >> 6);
  const int lane = t & 63;
  const int vx = wave_incl_sum_dpp(x), vy = wave_incl_sum_dpp(y);
  if (lane == 63) { sh[t >> 6] = vx; sh[16 + (t >> 6)] = vy; }
  __syncthreads();
  int bx = 0, ax = 0, by = 0, ay = 0;
  for (int w = 0; w < nw; w++) {
    const int sx = sh[w], sy = sh[16 + w];
    bx += w < (t >> 6) ? sx : 0;
    by += w < (t >> 6) ? sy : 0;
    ax += sx;
    ay += sy;
  }
  __syncthreads();
  *totx = ax;
  *toty = ay;
  *oy = by + vy - y;
  return bx + vx - x;
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t x, int m) {
  const int lo = __shfl_xor((int)(uint32_t)x, m, 64), hi = __shfl_xor((int)(uint32_t)(x >> 32), m, 64);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

// Bitonic sort of P = 1024 E keys by a 1024-thread block, thread t holding keys t E .. t E + E - 1
// in registers: partners within the thread are compare-exchanged in registers, within the wave
// through lane shuffles, and only distances of 64 E and more go through LDS (10 of the 78
// stages for 4096 keys, each a write / barrier / read / barrier).  Element i's new value is the
// min or the max of (i, i ^ j) as ((i & j) == 0) == ((i & k) == 0).
template <int E>
__device__ __forceinline__ void cmp_sort_block(uint64_t* key, int P) {
  const int t = threadIdx.x;
  uint64_t v[E];
#pragma unroll
  for (int e = 0; e < E; e++) v[e] = key[t * E + e];
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= 64 * E) {
        __syncthreads();
#pragma unroll
        for (int e = 0; e < E; e++) key[t * E + e] = v[e];
        __syncthreads();
#pragma unroll
        for (int e = 0; e < E; e++) {
          const int i = t * E + e;
          const uint64_t y = key[i ^ j];
          v[e] = (((i & j) == 0) == ((i & k) == 0)) ? (v[e] < y ? v[e] : y) : (v[e] > y ? v[e] : y);
        }
      } else if (j >= E) {
#pragma unroll
        for (int e = 0; e < E; e++) {
          const int i = t * E + e;
          const uint64_t y = shfl_xor_u64(v[e], j / E);
          v[e] = (((i & j) == 0) == ((i & k) == 0)) ? (v[e] < y ? v[e] : y) : (v[e] > y ? v[e] : y);
        }
      } else {
        // j < E: pairs inside the thread (static register indices)
#pragma unroll
        for (int e = 0; e < E; e++) {
          const int f = e ^ j;   // (j is 1 or 2 here; E <= 4)
          if (E >= 2 && j == 1 && (e & 1) == 0) {
            const bool up = ((t * E + e) & k) == 0;
            const uint64_t a = v[e], b = v[e + 1 < E ? e + 1 : e];
            const uint64_t lo = a < b ? a : b, hi = a < b ? b : a;
            v[e] = up ? lo : hi;
            v[e + 1 < E ? e + 1 : e] = up ? hi : lo;
          } else if (E >= 4 && j == 2 && (e & 2) == 0) {
            const bool up = ((t * E + e) & k) == 0;
            const uint64_t a = v[e], b = v[e + 2 < E ? e + 2 : e];
            const uint64_t lo = a < b ? a : b, hi = a < b ? b : a;
            v[e] = up ? lo : hi;
            v[e + 2 < E ? e + 2 : e] = up ? hi : lo;
          }
          (void)f;
        }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < E; e++) key[t * E + e] = v[e];
  __syncthreads();
}

// kept datapoint of a row, in output order (the write pass's input)
struct CmpKept {
  uint32_t qsrc;   // qualifier source, from the row's first column's qualifier (append: value) bytes
  uint32_t vsrc;   // value source, from the row's first column's value bytes
  uint32_t qdst;   // destination offset in the compacted qualifier << 8 | em
  uint32_t vdst;   // destination offset in the compacted value
};

__global__ __launch_bounds__(CMP_ROW_THREADS) void k_cmp_row(CmpParams p, CmpKept* klist, int P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  uint64_t* key = reinterpret_cast<uint64_t*>(sm);       // [P] sorted keys
  uint32_t* eq_src = reinterpret_cast<uint32_t*>(key + P);   // [P] by entry: qualifier source (row-relative)
  uint32_t* ev_src = eq_src + P;                         //          value source
  uint16_t* eem = reinterpret_cast<uint16_t*>(ev_src + P);   //          flags (em_*)
  uint16_t* ecol = eem + P;                              //          column - c0
  __shared__ int scan_sh[CMP_ROW_THREADS / 64];
  __shared__ int dup_err;   // a duplicate with different bytes in this row (the global flag may be stale in L1)
  const int64_t r = blockIdx.x;
  const int t = threadIdx.x;
  if (t == 0) dup_err = 0;
  // k_cmp_rows' verdicts that need no datapoint
  if (p.row_err[r] || p.row_heap[r] == 0) {
    if (t == 0) { p.row_state[r] = 0; p.row_q[r] = p.row_v[r] = 0; p.row_meta[r] = 0; p.row_lo[r] = 0; }
    return;
  }
  if (p.row_heap[r] == 1) {
    const int64_t c = p.row_one[r];
    const uint32_t info = p.col_info[c];
    const int64_t ql = (int64_t)(p.col_qo[c + 1] - p.col_qo[c]);
    if ((info & 3) == CMP_DATA && !(info & 8) && (ql == 2 || (ql == 4 && cmp_in_ms(p.q[p.col_qo[c]])))) {
      if (t == 0) {   // noMergesOrFixups: the single column as stored
        p.row_state[r] = 2;
        p.row_q[r] = ql;
        p.row_v[r] = (int64_t)(p.col_vo[c + 1] - p.col_vo[c]);
        p.row_meta[r] = 0;
        p.row_lo[r] = 0;
      }
      return;
    }
  }
  const int64_t c0 = p.row_col_ptr[r], c1 = p.row_col_ptr[r + 1];
  const int64_t e0 = p.col_off[c0];
  const int n = (int)(p.col_off[c1] - e0);
  const uint64_t qb = p.col_qo[c0], vb = p.col_vo[c0];
  const uint8_t* vrow = p.v + vb;
  // explode: one thread per column
  for (int64_t c = c0 + t; c < c1; c += CMP_ROW_THREADS) {
    const int64_t nc_ = p.col_n[c];
    if (nc_ == 0) continue;
    int e = (int)(p.col_off[c] - e0);
    const uint64_t qo = p.col_qo[c], vo = p.col_vo[c];
    const int64_t ql = (int64_t)(p.col_qo[c + 1] - qo), vl = (int64_t)(p.col_vo[c + 1] - vo);
    const uint32_t info = p.col_info[c];
    const bool app = (info & 3) == CMP_APPEND;
    const bool fix = !app && ql == 2 && (info & 8);
    const uint32_t qbase = (uint32_t)((app ? vo - vb : qo - qb));
    const uint32_t vbase = (uint32_t)(vo - vb);
    auto put = [&](int64_t qpos, int64_t vpos, int eq, int evl, uint32_t off) {
      key[e] = ((uint64_t)off << 12) | (uint64_t)e;
      eq_src[e] = qbase + (uint32_t)qpos;
      ev_src[e] = vbase + (uint32_t)vpos;
      eem[e] = (uint16_t)((eq == 4 ? 1u : 0u) | ((uint32_t)(evl - 1) << 1) | (fix ? 16u : 0u) | (app ? 32u : 0u));
      ecol[e] = (uint16_t)(c - c0);
      e++;
    };
    if (app) {
      walk_append(p.v + vo, vl, put);
    } else {
      const int64_t vstart = (info & 4) ? 4 : 0;
      walk_data(p.q + qo, ql, vl - vstart, (uint8_t)(info >> 8),
                [&](int64_t qi, int64_t vi, int eq, int evl, uint32_t off) { put(qi, vstart + vi, eq, evl, off); });
    }
  }
  for (int i = n + t; i < P; i += CMP_ROW_THREADS) key[i] = ~0ull >> 2;   // above every key, kept bit clear
  __syncthreads();
  // sort the P keys (unique: the entry ordinal is in the low bits) unless the columns came in
  // time order already -- an HBase scan returns a row's columns sorted by qualifier, which is
  // time order for second qualifiers
  int unsorted = 0;
  for (int i = t + 1; i < n; i += CMP_ROW_THREADS) unsorted |= key[i - 1] > key[i] ? 1 : 0;
  bool placed = false;
  if (__syncthreads_or(unsorted) && P == 4096) {
    // Columns out of time order whose datapoints all sit on distinct whole seconds (a second-
    // resolution hour row of single-datapoint columns): each entry goes straight to its second
    // -- a bitmap of the seconds (a second hit twice means duplicates: the sort below), the
    // entries by second in ecol's space (only runs of several datapoints read ecol), then one
    // block scan over the bitmap gives every entry its sorted position.  The same order the
    // sort gives: the keys are distinct, so the entry bits never decide.
    __shared__ uint32_t secmap[4096 / 32];
    __shared__ int place_fail;
    for (int i = t; i < 4096 / 32; i += CMP_ROW_THREADS) secmap[i] = 0;
    if (t == 0) place_fail = 0;
    __syncthreads();
    for (int i = t; i < n; i += CMP_ROW_THREADS) {
      const uint64_t off = key[i] >> 12;
      if (off % 1000u != 0 || off >= 4096000u) { place_fail = 1; continue; }
      const uint32_t sec = (uint32_t)(off / 1000u);
      const uint32_t bit = 1u << (sec & 31);
      if (atomicOr(&secmap[sec >> 5], bit) & bit) place_fail = 1;
    }
    __syncthreads();
    if (!place_fail) {
      uint16_t* by_sec = ecol;   // [4096]: the entry on each occupied second
      for (int i = t; i < n; i += CMP_ROW_THREADS) by_sec[(uint32_t)((key[i] >> 12) / 1000u)] = (uint16_t)i;
      const uint32_t bits = (secmap[t >> 3] >> ((t & 7) * 4)) & 0xFu;   // seconds 4t .. 4t + 3
      int total;
      int pos = block_excl_scan(__popc(bits), scan_sh, &total);   // (its barriers order the writes above)
#pragma unroll
      for (int j = 0; j < 4; j++) {
        if ((bits >> j) & 1u) {
          const uint32_t sec = 4u * (uint32_t)t + (uint32_t)j;
          key[pos++] = ((uint64_t)(sec * 1000u) << 12) | by_sec[sec];
        }
      }
      __syncthreads();
      placed = true;
    }
  }
  if (!placed && __syncthreads_or(unsorted)) {
    if (P == 4096) cmp_sort_block<4>(key, P);
    else if (P == 2048) cmp_sort_block<2>(key, P);
    else if (P == 1024) cmp_sort_block<1>(key, P);
    else {
      for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
          for (int i = t; i < P / 2; i += CMP_ROW_THREADS) {
            const int lo = ((i & ~(j - 1)) << 1) | (i & (j - 1));
            const int hi = lo + j;
            const uint64_t x = key[lo], y = key[hi];
            if ((x > y) == ((lo & k) == 0)) {
              key[lo] = y;
              key[hi] = x;
            }
          }
          __syncthreads();
        }
    }
  }
  // runs of one offset: a single datapoint is kept as is; of several, the newest column's
  // (k_cmp_dedup's rules)
  for (int i = t; i < n; i += CMP_ROW_THREADS) {
    const uint64_t off = key[i] >> 12;
    if (i > 0 && (key[i - 1] >> 12) == off) continue;
    int j = i + 1;
    while (j < n && (key[j] >> 12) == off) j++;
    if (j == i + 1) {
      key[i] |= CMP_KEPT;
      continue;
    }
    auto ent = [&](int s) { return (int)(key[s] & 4095); };
    auto superseded = [&](int s) {
      const int es = ent(s);
      return (eem[es] & 32) && s + 1 < j && ecol[ent(s + 1)] == ecol[es];
    };
    int best = -1;
    int64_t best_ts = 0;
    for (int s = i; s < j; s++) {
      if (superseded(s)) continue;
      const int64_t ts = p.col_ts ? p.col_ts[c0 + ecol[ent(s)]] : 0;
      if (best < 0 || ts > best_ts) { best = s; best_ts = ts; }
    }
    key[best] |= CMP_KEPT;
    if (p.fix_dup) continue;
    const int eb = ent(best);
    const int lb = em_evl(eem[eb]);
    const uint8_t* vk = vrow + ev_src[eb];
    for (int s = i; s < j; s++) {
      if (s == best || superseded(s)) continue;
      const int es = ent(s);   // getCopyOfCurrentValue vs the kept one
      bool same = em_evl(eem[es]) == lb;
      const uint8_t* vo = vrow + ev_src[es];
      for (int b = 0; same && b < lb; b++) same = vo[b] == vk[b];
      if (!same) {
        cmp_fail(p.row_err, r, TSDB_E_ILLEGAL_DATA);
        dup_err = 1;
      }
    }
  }
  __syncthreads();
  // each thread a contiguous run of m sorted positions: its kept bytes / datapoints, then the
  // block's exclusive offsets, then the thread's list records
  const int m = P / CMP_ROW_THREADS > 0 ? P / CMP_ROW_THREADS : 1;
  const int a0 = t * m, a1 = min(n, a0 + m);
  int sq = 0, sv = 0, sc = 0, sms = 0;
  for (int i = a0; i < a1; i++) {
    const uint64_t kk = key[i];
    if (!(kk & CMP_KEPT)) continue;
    const uint32_t em = eem[kk & 4095];
    sq += em_eq(em);
    sv += em_evl(em);
    sc++;
    sms += em & 1;
  }
  int tq, tv, tc, tm;
  int oq = block_excl_scan(sq, scan_sh, &tq);
  int ov = block_excl_scan(sv, scan_sh, &tv);
  int oc = block_excl_scan(sc, scan_sh, &tc);
  block_excl_scan(sms, scan_sh, &tm);
  if (dup_err) {
    if (t == 0) { p.row_state[r] = 0; p.row_q[r] = p.row_v[r] = 0; p.row_meta[r] = 0; p.row_lo[r] = 0; }
    return;
  }
  CmpKept* out = klist + e0;
  for (int i = a0; i < a1; i++) {
    const uint64_t kk = key[i];
    if (!(kk & CMP_KEPT)) continue;
    const int e = (int)(kk & 4095);
    const uint32_t em = eem[e];
    out[oc] = CmpKept{eq_src[e], ev_src[e], ((uint32_t)oq << 8) | em, (uint32_t)ov};
    oq += em_eq(em);
    ov += em_evl(em);
    oc++;
  }
  if (t == 0) {
    p.row_state[r] = tc ? 1 : 0;
    p.row_q[r] = tc ? tq : 0;
    p.row_v[r] = tc ? tv + (tc > 1 ? 1 : 0) : 0;
    p.row_meta[r] = (tm > 0 && tm < tc) ? 1 : 0;   // Const.MS_MIXED_COMPACT
    p.row_lo[r] = tc;                               // kept datapoints (list length)
  }
}

// The compacted cell of each row at the host's layout, from the sizing pass's list.  The row's
// source bytes (its columns' qualifiers and values, contiguous) are staged in LDS with dword
// loads when they fit, the cell is assembled in LDS byte by byte, and leaves in dwords (the
// destination rows are 16-byte aligned).  Rows whose sources do not fit read them from HBM.
__global__ __launch_bounds__(CMP_ROW_THREADS) void k_cmp_rowwrite(CmpParams p, const CmpKept* klist, int oq_cap,
                                                                  int ov_cap, int src_cap) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smw[];
  uint8_t* oq = reinterpret_cast<uint8_t*>(smw);
  uint8_t* ov = oq + oq_cap;
  uint32_t* srcw = reinterpret_cast<uint32_t*>(ov + ov_cap);
  const int64_t r = blockIdx.x;
  const int t = threadIdx.x;
  const int nt = CMP_ROW_THREADS;
  if (p.row_dq[r] < 0 || p.row_state[r] == 0) return;
  uint8_t* dq = p.out_q + p.row_dq[r];
  uint8_t* dv = p.out_v + p.row_dv[r];
  const int64_t c0 = p.row_col_ptr[r], c1 = p.row_col_ptr[r + 1];
  if (p.row_state[r] == 2) {   // the single column as stored (noMergesOrFixups)
    const int64_t c = p.row_one[r];
    const uint8_t* qs = p.q + p.col_qo[c];
    const uint8_t* vs = p.v + p.col_vo[c];
    for (int64_t b = t; b < p.row_q[r]; b += nt) dq[b] = qs[b];
    for (int64_t b = t; b < p.row_v[r]; b += nt) dv[b] = vs[b];
    return;
  }
  const uint64_t qb = p.col_qo[c0], vb = p.col_vo[c0];
  const uint64_t qspan = p.col_qo[c1] - qb, vspan = p.col_vo[c1] - vb;
  // dword windows over the sources: [qa, qa + 4 nqw) then [va, va + 4 nvw)
  const uint64_t qa = qb & ~3ull, va = vb & ~3ull;
  const int64_t nqw = (int64_t)((qb + qspan - qa + 3) / 4), nvw = (int64_t)((vb + vspan - va + 3) / 4);
  const bool staged = (nqw + nvw) * 4 <= src_cap;
  const int64_t nq = p.row_q[r], nv = p.row_v[r];
  const int64_t nqd = (nq + 3) / 4, nvd = (nv + 3) / 4;
  uint32_t* oqw = reinterpret_cast<uint32_t*>(oq);
  uint32_t* ovw = reinterpret_cast<uint32_t*>(ov);
  for (int64_t w = t; w < nqd; w += nt) oqw[w] = 0;
  for (int64_t w = t; w < nvd; w += nt) ovw[w] = 0;
  if (staged) {
    const uint32_t* gq = reinterpret_cast<const uint32_t*>(p.q + qa);
    const uint32_t* gv = reinterpret_cast<const uint32_t*>(p.v + va);
    for (int64_t w = t; w < nqw; w += nt) srcw[w] = gq[w];
    for (int64_t w = t; w < nvw; w += nt) srcw[nqw + w] = gv[w];
  }
  __syncthreads();
  const uint8_t* sq = staged ? reinterpret_cast<const uint8_t*>(srcw) + (qb - qa) : p.q + qb;
  const uint8_t* sv = staged ? reinterpret_cast<const uint8_t*>(srcw + nqw) + (vb - va) : p.v + vb;
  const CmpKept* list = klist + p.col_off[c0];
  const int64_t nk = p.row_lo[r];
  for (int64_t i = t; i < nk; i += nt) {
    const CmpKept k = list[i];
    const uint32_t em = k.qdst & 255;
    const int eq = em_eq(em), evl = em_evl(em);
    const uint8_t* qs = ((em & 32) ? sv : sq) + k.qsrc;
    uint8_t* qd = oq + (k.qdst >> 8);
    qd[0] = qs[0];
    qd[1] = (em & 16) ? (uint8_t)((qs[1] & 0xF8) | (evl - 1)) : qs[1];   // checkForFixup's flags
    if (eq == 4) {
      qd[2] = qs[2];
      qd[3] = qs[3];
    }
    const uint8_t* vs = sv + k.vsrc;
    uint8_t* vd = ov + k.vdst;
    for (int b = 0; b < evl; b++) vd[b] = vs[b];
  }
  __syncthreads();
  if (t == 0 && nk > 1) ov[nv - 1] = p.row_meta[r];
  __syncthreads();
  uint32_t* dqw = reinterpret_cast<uint32_t*>(dq);
  uint32_t* dvw = reinterpret_cast<uint32_t*>(dv);
  for (int64_t w = t; w < nqd; w += nt) dqw[w] = oqw[w];
  for (int64_t w = t; w < nvd; w += nt) dvw[w] = ovw[w];
}

// ---- the one-pass per-row path ------------------------------------------------------------
// The host lays every row out from k_cmp_cols' byte bounds before any datapoint is sorted, so the
// row kernel can write the compacted cell itself: no kept-datapoint list through HBM, no second
// read of the sources, no scan over the column counts (a block scan gives the row's entry
// offsets).  Same explode / order / dedup as k_cmp_row; the cell is assembled in the LDS the
// sort used and leaves in dwords.
__global__ __launch_bounds__(256) void k_cmp_rowmax2(CmpParams p, uint32_t* out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t n = 0, nc = 0;
  if (r < p.n_rows) {
    n = (uint32_t)min<int64_t>(p.row_n[r], 0xFFFFFFFFll);
    nc = (uint32_t)min<int64_t>(p.row_col_ptr[r + 1] - p.row_col_ptr[r], 0xFFFFFFFFll);
  }
  for (int o = 32; o > 0; o >>= 1) {
    n = max(n, (uint32_t)__shfl_xor((int)n, o));
    nc = max(nc, (uint32_t)__shfl_xor((int)nc, o));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(&out[0], n);
    atomicMax(&out[1], nc);
  }
}

// bytes [s, s + n) of src to dst (16-byte aligned) in dwords: each output dword from the two
// aligned source dwords it straddles
__device__ __forceinline__ void cmp_copy_to_aligned(uint8_t* dst, const uint8_t* src, int64_t n, int t, int nt) {
  const uintptr_t sa = (uintptr_t)src;
  const uint32_t* s4 = reinterpret_cast<const uint32_t*>(sa & ~(uintptr_t)3);
  const int sh = (int)(sa & 3) * 8;
  uint32_t* d4 = reinterpret_cast<uint32_t*>(dst);
  const int64_t nw = n >> 2;
  for (int64_t w = t; w < nw; w += nt) {
    const uint32_t lo = s4[w];
    const uint32_t hi = sh ? s4[w + 1] : 0u;   // (the sources carry 16 bytes of slack)
    d4[w] = sh ? ((lo >> sh) | (hi << (32 - sh))) : lo;
  }
  for (int64_t b = (nw << 2) + t; b < n; b += nt) dst[b] = src[b];
}

template <bool W32>
__global__ __launch_bounds__(CMP_ROW_THREADS) void k_cmp_rowone(CmpParams p, int P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  uint64_t* key = reinterpret_cast<uint64_t*>(sm);
  uint32_t* eq_src = reinterpret_cast<uint32_t*>(key + P);
  uint32_t* ev_src = eq_src + P;
  uint16_t* eem = reinterpret_cast<uint16_t*>(ev_src + P);
  uint16_t* ecol = eem + P;
  __shared__ int scan_sh[2 * CMP_ROW_THREADS / 64];
  __shared__ int dup_err;
  const int64_t r = blockIdx.x;
  const int t = threadIdx.x;
  if (t == 0) dup_err = 0;
  auto no_cell = [&]() {
    if (t == 0) { p.row_state[r] = 0; p.row_q[r] = p.row_v[r] = 0; p.row_meta[r] = 0; p.row_lo[r] = 0; }
  };
  if (p.row_err[r] || p.row_heap[r] == 0) { no_cell(); return; }
  if (p.row_heap[r] == 1) {
    const int64_t c = p.row_one[r];
    uint32_t info = 0;
    cmp_col<W32>(p, c, r, nullptr, nullptr, nullptr, false, &info);
    const int64_t ql = (int64_t)(col_q<W32>(p, c + 1) - col_q<W32>(p, c));
    if ((info & 3) == CMP_DATA && !(info & 8) && (ql == 2 || (ql == 4 && cmp_in_ms(p.q[col_q<W32>(p, c)])))) {
      const int64_t vl = (int64_t)(col_v<W32>(p, c + 1) - col_v<W32>(p, c));   // noMergesOrFixups: as stored
      if (ql > p.row_qb[r] || vl > p.row_vb[r]) {
        if (t == 0) cmp_fail(p.row_err, r, TSDB_E_ILLEGAL_STATE);
        no_cell();
        return;
      }
      cmp_copy_to_aligned(p.out_q + p.row_dq[r], p.q + col_q<W32>(p, c), ql, t, CMP_ROW_THREADS);
      cmp_copy_to_aligned(p.out_v + p.row_dv[r], p.v + col_v<W32>(p, c), vl, t, CMP_ROW_THREADS);
      if (t == 0) { p.row_state[r] = 2; p.row_q[r] = ql; p.row_v[r] = vl; p.row_meta[r] = 0; p.row_lo[r] = 0; }
      return;
    }
  }
  const int64_t c0 = p.row_col_ptr[r], c1 = p.row_col_ptr[r + 1];
  const uint64_t qb = col_q<W32>(p, c0), vb = col_v<W32>(p, c0);
  const uint8_t* qrow = p.q + qb;
  const uint8_t* vrow = p.v + vb;
  // Fast path: every column one datapoint with a 2-byte (second) qualifier, no two on one
  // second -- an hour row of single-datapoint cells.  Each column goes straight to its second (a
  // 4096-bit map and a second -> column map at the top of the LDS); one dual block scan over the
  // map gives the output positions; the cell is assembled as below.  No entry arrays, sort or
  // dedup.  Anything else (a compacted column, an append, ms qualifiers, a second hit twice)
  // falls through to the general path.
  if (P >= 2048 && c1 - c0 <= 4096) {
    __shared__ int fp_fail;
    uint16_t* scol = reinterpret_cast<uint16_t*>(sm + (size_t)P * 20 - 12800);   // [4096] column - c0, 0xFFFF none
    uint8_t* sinf = reinterpret_cast<uint8_t*>(scol + 4096);                      // [4096] fix | vstart | evl - 1
    if (t == 0) fp_fail = 0;
    for (int i = t; i < 2048; i += CMP_ROW_THREADS) reinterpret_cast<uint32_t*>(scol)[i] = 0xFFFFFFFFu;
    __syncthreads();
    // (no atomics: every column stores its index at its second, then checks it is still there --
    // a second two columns hit keeps one of them, and the other one sees it)
    uint32_t mysec[4];
    int nmine = 0;
    for (int64_t c = c0 + t; c < c1; c += CMP_ROW_THREADS) {
      int64_t nn = 0;
      uint32_t info = 0;
      cmp_col<W32>(p, c, r, nullptr, nullptr, &nn, false, &info);
      const int64_t ql = (int64_t)(col_q<W32>(p, c + 1) - col_q<W32>(p, c));
      if ((info & 3) != CMP_DATA || ql != 2 || nn != 1) { fp_fail = 1; continue; }
      const uint8_t* q = p.q + col_q<W32>(p, c);
      const uint32_t sec = (((uint32_t)q[0] << 8) | q[1]) >> 4;
      scol[sec] = (uint16_t)(c - c0);
      const uint32_t evl1 = (info >> 8) & 7;   // (the fixed flags byte's length)
      sinf[sec] = (uint8_t)(evl1 | ((info & 4) ? 8u : 0u) | ((info & 8) ? 16u : 0u));
      if (nmine < 4) mysec[nmine] = sec | ((uint32_t)(c - c0) << 12);
      nmine++;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; j++)
      if (j < nmine && scol[mysec[j] & 4095] != (uint16_t)(mysec[j] >> 12)) fp_fail = 1;   // a second hit twice
    __syncthreads();
    if (!fp_fail) {
      uint32_t bits = 0;   // seconds 4t .. 4t + 3 present
#pragma unroll
      for (int j = 0; j < 4; j++) bits |= (scol[4 * t + j] != 0xFFFFu ? 1u : 0u) << j;
      int sv = 0;
#pragma unroll
      for (int j = 0; j < 4; j++)
        if ((bits >> j) & 1u) sv += (sinf[4 * t + j] & 7) + 1;
      const int kc = __popc(bits);
      int tcn, tvb, ovb;
      const int ocn = block_excl_scan2(kc, sv, scan_sh, &tcn, &ovb, &tvb);
      const int tq = 2 * tcn, nv = tvb + (tcn > 1 ? 1 : 0);
      if (tq > p.row_qb[r] || tvb > p.row_vb[r]) {
        if (t == 0) cmp_fail(p.row_err, r, TSDB_E_ILLEGAL_STATE);
        no_cell();
        return;
      }
      uint8_t* oq = sm;
      uint8_t* ov = sm + ((tq + 15) & ~15);
      int q_at = 2 * ocn, v_at = ovb;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        if ((bits >> j) & 1u) {
          const uint32_t sec = 4u * (uint32_t)t + (uint32_t)j;
          const int64_t c = c0 + scol[sec];
          const uint32_t f = sinf[sec];
          const int evl = (int)(f & 7) + 1;
          const uint8_t* qs = p.q + col_q<W32>(p, c);
          const uint8_t* vs = p.v + col_v<W32>(p, c) + ((f & 8) ? 4 : 0);
          if (!(((uintptr_t)qs | (uintptr_t)(oq + q_at)) & 1)) {
            uint32_t w = *reinterpret_cast<const uint16_t*>(qs);
            if (f & 16) w = (w & 0x00FFu) | ((((w >> 8) & 0xF8u) | (uint32_t)(evl - 1)) << 8);   // checkForFixup's flags
            *reinterpret_cast<uint16_t*>(oq + q_at) = (uint16_t)w;
          } else {
            oq[q_at] = qs[0];
            oq[q_at + 1] = (f & 16) ? (uint8_t)((qs[1] & 0xF8) | (evl - 1)) : qs[1];
          }
          if ((evl == 8 || evl == 4) && !(((uintptr_t)vs | (uintptr_t)(ov + v_at)) & 3)) {
            *reinterpret_cast<uint32_t*>(ov + v_at) = *reinterpret_cast<const uint32_t*>(vs);
            if (evl == 8) *reinterpret_cast<uint32_t*>(ov + v_at + 4) = *reinterpret_cast<const uint32_t*>(vs + 4);
          } else {
            for (int b2 = 0; b2 < evl; b2++) ov[v_at + b2] = vs[b2];
          }
          q_at += 2;
          v_at += evl;
        }
      }
      const int nqd = (tq + 3) >> 2, nvd = (nv + 3) >> 2;
      if (kc > 0 && ocn + kc == tcn) {   // the last datapoint's thread: meta byte (seconds only: 0), padding
        if (tcn > 1) ov[nv - 1] = 0;
        for (int b2 = tq; b2 < nqd * 4; b2++) oq[b2] = 0;
        for (int b2 = nv; b2 < nvd * 4; b2++) ov[b2] = 0;
      }
      __syncthreads();
      const uint32_t* oqw = reinterpret_cast<const uint32_t*>(oq);
      const uint32_t* ovw = reinterpret_cast<const uint32_t*>(ov);
      uint32_t* dqw = reinterpret_cast<uint32_t*>(p.out_q + p.row_dq[r]);
      uint32_t* dvw = reinterpret_cast<uint32_t*>(p.out_v + p.row_dv[r]);
      for (int w = t; w < nqd; w += CMP_ROW_THREADS) dqw[w] = oqw[w];
      for (int w = t; w < nvd; w += CMP_ROW_THREADS) dvw[w] = ovw[w];
      if (t == 0) {
        p.row_state[r] = tcn ? 1 : 0;
        p.row_q[r] = tcn ? tq : 0;
        p.row_v[r] = tcn ? nv : 0;
        p.row_meta[r] = 0;
        p.row_lo[r] = tcn;
      }
      return;
    }
    __syncthreads();   // (the general path below reuses the LDS)
  }
  // explode, 4096 columns a round (4 consecutive a thread, in scan order): the entry offsets of a
  // round from one block scan of the threads' counts
  constexpr int CPT = 4;
  int n = 0;
  for (int64_t cr = c0; cr < c1; cr += CMP_ROW_THREADS * CPT) {
    const int64_t cb = cr + (int64_t)t * CPT;
    int ncs[CPT], sum = 0;
    uint32_t infos[CPT];
#pragma unroll
    for (int j = 0; j < CPT; j++) {
      int64_t nn = 0;
      infos[j] = 0;
      if (cb + j < c1) cmp_col<W32>(p, cb + j, r, nullptr, nullptr, &nn, false, &infos[j]);
      ncs[j] = (int)nn;
      sum += ncs[j];
    }
    int tot;
    int e = n + block_excl_scan(sum, scan_sh, &tot);
    n += tot;
#pragma unroll
    for (int j = 0; j < CPT; j++) {
      if (ncs[j] == 0) continue;
      const int64_t c = cb + j;
      const uint64_t qo = col_q<W32>(p, c), vo = col_v<W32>(p, c);
      const int64_t ql = (int64_t)(col_q<W32>(p, c + 1) - qo), vl = (int64_t)(col_v<W32>(p, c + 1) - vo);
      const uint32_t info = infos[j];
      const bool app = (info & 3) == CMP_APPEND;
      const bool fix = !app && ql == 2 && (info & 8);
      const uint32_t qbase = (uint32_t)((app ? vo - vb : qo - qb));
      const uint32_t vbase = (uint32_t)(vo - vb);
      auto put = [&](int64_t qpos, int64_t vpos, int eq, int evl, uint32_t off) {
        key[e] = ((uint64_t)off << 12) | (uint64_t)e;
        eq_src[e] = qbase + (uint32_t)qpos;
        ev_src[e] = vbase + (uint32_t)vpos;
        eem[e] = (uint16_t)((eq == 4 ? 1u : 0u) | ((uint32_t)(evl - 1) << 1) | (fix ? 16u : 0u) | (app ? 32u : 0u));
        ecol[e] = (uint16_t)(c - c0);
        e++;
      };
      if (app) {
        walk_append(p.v + vo, vl, put);
      } else {
        const int64_t vstart = (info & 4) ? 4 : 0;
        walk_data(p.q + qo, ql, vl - vstart, (uint8_t)(info >> 8),
                  [&](int64_t qi, int64_t vi, int eq, int evl, uint32_t off) { put(qi, vstart + vi, eq, evl, off); });
      }
    }
  }
  for (int i = n + t; i < P; i += CMP_ROW_THREADS) key[i] = ~0ull >> 2;
  __syncthreads();
  int unsorted = 0;
  for (int i = t + 1; i < n; i += CMP_ROW_THREADS) unsorted |= key[i - 1] > key[i] ? 1 : 0;
  bool placed = false;
  if (__syncthreads_or(unsorted) && P == 4096) {   // distinct whole seconds: placed by second (k_cmp_row)
    __shared__ uint32_t secmap[4096 / 32];
    __shared__ int place_fail;
    for (int i = t; i < 4096 / 32; i += CMP_ROW_THREADS) secmap[i] = 0;
    if (t == 0) place_fail = 0;
    __syncthreads();
    for (int i = t; i < n; i += CMP_ROW_THREADS) {
      const uint64_t off = key[i] >> 12;
      if (off % 1000u != 0 || off >= 4096000u) { place_fail = 1; continue; }
      const uint32_t sec = (uint32_t)(off / 1000u);
      const uint32_t bit = 1u << (sec & 31);
      if (atomicOr(&secmap[sec >> 5], bit) & bit) place_fail = 1;
    }
    __syncthreads();
    if (!place_fail) {
      uint16_t* by_sec = ecol;
      for (int i = t; i < n; i += CMP_ROW_THREADS) by_sec[(uint32_t)((key[i] >> 12) / 1000u)] = (uint16_t)i;
      const uint32_t bits = (secmap[t >> 3] >> ((t & 7) * 4)) & 0xFu;
      int total;
      int pos = block_excl_scan(__popc(bits), scan_sh, &total);
#pragma unroll
      for (int j = 0; j < 4; j++) {
        if ((bits >> j) & 1u) {
          const uint32_t sec = 4u * (uint32_t)t + (uint32_t)j;
          key[pos++] = ((uint64_t)(sec * 1000u) << 12) | by_sec[sec];
        }
      }
      __syncthreads();
      placed = true;
    }
  }
  if (!placed && __syncthreads_or(unsorted)) {
    if (P == 4096) cmp_sort_block<4>(key, P);
    else if (P == 2048) cmp_sort_block<2>(key, P);
    else if (P == 1024) cmp_sort_block<1>(key, P);
    else {
      for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
          for (int i = t; i < P / 2; i += CMP_ROW_THREADS) {
            const int lo = ((i & ~(j - 1)) << 1) | (i & (j - 1));
            const int hi = lo + j;
            const uint64_t x = key[lo], y = key[hi];
            if ((x > y) == ((lo & k) == 0)) {
              key[lo] = y;
              key[hi] = x;
            }
          }
          __syncthreads();
        }
    }
  }
  // runs of one offset (k_cmp_row's rules)
  for (int i = t; i < n; i += CMP_ROW_THREADS) {
    const uint64_t off = key[i] >> 12;
    if (i > 0 && (key[i - 1] >> 12) == off) continue;
    int j = i + 1;
    while (j < n && (key[j] >> 12) == off) j++;
    if (j == i + 1) {
      key[i] |= CMP_KEPT;
      continue;
    }
    auto ent = [&](int s) { return (int)(key[s] & 4095); };
    auto superseded = [&](int s) {
      const int es = ent(s);
      return (eem[es] & 32) && s + 1 < j && ecol[ent(s + 1)] == ecol[es];
    };
    int best = -1;
    int64_t best_ts = 0;
    for (int s = i; s < j; s++) {
      if (superseded(s)) continue;
      const int64_t ts = p.col_ts ? p.col_ts[c0 + ecol[ent(s)]] : 0;
      if (best < 0 || ts > best_ts) { best = s; best_ts = ts; }
    }
    key[best] |= CMP_KEPT;
    if (p.fix_dup) continue;
    const int eb = ent(best);
    const int lb = em_evl(eem[eb]);
    const uint8_t* vk = vrow + ev_src[eb];
    for (int s = i; s < j; s++) {
      if (s == best || superseded(s)) continue;
      const int es = ent(s);
      bool same = em_evl(eem[es]) == lb;
      const uint8_t* vo = vrow + ev_src[es];
      for (int b = 0; same && b < lb; b++) same = vo[b] == vk[b];
      if (!same) {
        cmp_fail(p.row_err, r, TSDB_E_ILLEGAL_DATA);
        dup_err = 1;
      }
    }
  }
  __syncthreads();
  // each thread m consecutive sorted positions (m <= 4): its kept entries into registers, two
  // block scans of packed sums (qualifier | value bytes, datapoints | ms datapoints)
  constexpr int MMAX = CMP_ROW_CAP / CMP_ROW_THREADS;
  const int m = P / CMP_ROW_THREADS > 0 ? P / CMP_ROW_THREADS : 1;
  const int a0 = t * m, a1 = min(n, a0 + m);
  uint32_t kq[MMAX], kv[MMAX], kem[MMAX];
  int kc = 0, sq = 0, sv = 0, sms = 0;
#pragma unroll
  for (int x = 0; x < MMAX; x++) {
    const int i = a0 + x;
    kq[x] = kv[x] = kem[x] = 0;
    if (x < m && i < a1) {
      const uint64_t kk = key[i];
      if (kk & CMP_KEPT) {
        const int e = (int)(kk & 4095);
        const uint32_t em = eem[e];
        kq[x] = eq_src[e];
        kv[x] = ev_src[e];
        kem[x] = em | 0x10000u;   // (bit 16: kept)
        sq += em_eq(em);
        sv += em_evl(em);
        kc++;
        sms += em & 1;
      }
    }
  }
  int tqv, tcm, ocm;
  const int oqv = block_excl_scan2((sq << 16) | sv, (kc << 16) | sms, scan_sh, &tqv, &ocm, &tcm);   // (sq <= 16384, sv <= 32768 a row)
  const int tq = tqv >> 16, tv = tqv & 0xFFFF, tc = tcm >> 16, tm = tcm & 0xFFFF;
  if (dup_err) { no_cell(); return; }
  if (tc == 0) { no_cell(); return; }
  const int nv = tv + (tc > 1 ? 1 : 0);   // + the meta byte
  if (tq > p.row_qb[r] || tv > p.row_vb[r]) {   // (the host's region is too small: cannot happen)
    if (t == 0) cmp_fail(p.row_err, r, TSDB_E_ILLEGAL_STATE);
    no_cell();
    return;
  }
  // the cell in LDS (the sort's space is free: every thread's entries are in registers)
  uint8_t* oq = sm;
  uint8_t* ov = sm + ((tq + 15) & ~15);
  const int nqd = (tq + 3) >> 2, nvd = (nv + 3) >> 2;
  uint32_t* oqw = reinterpret_cast<uint32_t*>(oq);
  uint32_t* ovw = reinterpret_cast<uint32_t*>(ov);
  const uint8_t meta = (tm > 0 && tm < tc) ? 1 : 0;   // Const.MS_MIXED_COMPACT
  // (no zero pass: the cell's bytes are each written once below; the thread holding the last kept
  // datapoint writes the meta byte and zeroes the rest of the last dwords)
  const bool last_owner = kc > 0 && (ocm >> 16) + kc == tc;
  int q_at = oqv >> 16, v_at = oqv & 0xFFFF;
#pragma unroll
  for (int x = 0; x < MMAX; x++) {
    if (kem[x] & 0x10000u) {
      const uint32_t em = kem[x];
      const int eq = em_eq(em), evl = em_evl(em);
      const uint8_t* qs = ((em & 32) ? vrow : qrow) + kq[x];
      uint8_t* qd = oq + q_at;
      if (eq == 2 && !(((uintptr_t)qs | (uintptr_t)qd) & 1)) {   // a 2-byte qualifier: one 16-bit move
        uint32_t w = *reinterpret_cast<const uint16_t*>(qs);   // (little-endian: byte 1 is the high half)
        if (em & 16) w = (w & 0x00FFu) | ((((w >> 8) & 0xF8u) | (uint32_t)(evl - 1)) << 8);   // checkForFixup's flags
        *reinterpret_cast<uint16_t*>(qd) = (uint16_t)w;
      } else {
        qd[0] = qs[0];
        qd[1] = (em & 16) ? (uint8_t)((qs[1] & 0xF8) | (evl - 1)) : qs[1];   // checkForFixup's flags
        if (eq == 4) {
          qd[2] = qs[2];
          qd[3] = qs[3];
        }
      }
      const uint8_t* vs = vrow + kv[x];
      uint8_t* vd = ov + v_at;
      if ((evl == 8 || evl == 4) && !(((uintptr_t)vs | (uintptr_t)vd) & 3)) {   // dword moves
        *reinterpret_cast<uint32_t*>(vd) = *reinterpret_cast<const uint32_t*>(vs);
        if (evl == 8) *reinterpret_cast<uint32_t*>(vd + 4) = *reinterpret_cast<const uint32_t*>(vs + 4);
      } else {
        for (int b = 0; b < evl; b++) vd[b] = vs[b];
      }
      q_at += eq;
      v_at += evl;
    }
  }
  if (last_owner) {
    if (tc > 1) ov[nv - 1] = meta;
    for (int b = tq; b < nqd * 4; b++) oq[b] = 0;
    for (int b = nv; b < nvd * 4; b++) ov[b] = 0;
  }
  __syncthreads();
  uint32_t* dqw = reinterpret_cast<uint32_t*>(p.out_q + p.row_dq[r]);
  uint32_t* dvw = reinterpret_cast<uint32_t*>(p.out_v + p.row_dv[r]);
  for (int w = t; w < nqd; w += CMP_ROW_THREADS) dqw[w] = oqw[w];
  for (int w = t; w < nvd; w += CMP_ROW_THREADS) dvw[w] = ovw[w];
  if (t == 0) {
    p.row_state[r] = 1;
    p.row_q[r] = tq;
    p.row_v[r] = nv;
    p.row_meta[r] = meta;
    p.row_lo[r] = tc;
  }
}

// k_cmp_cols for the one-pass path: one wave a row, its lanes striding over the row's columns
// (coalesced), the row's heap count / datapoints / byte bounds reduced in the wave and stored
// once -- no per-column row index, no atomics (k_cmp_cols' per-row atomics from every wave of a
// 3600-column row serialised in L2: 1.1 ms for 72M columns against 0.78 without the sums).
template <bool W32>
__global__ __launch_bounds__(256) void k_cmp_cols_rowwave(CmpParams p) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= p.n_rows) return;
  const int lane = (int)(threadIdx.x & 63);
  const int64_t c0 = p.row_col_ptr[r], c1 = p.row_col_ptr[r + 1];
  long long heap = 0, n = 0, qs = 0, vs = 0;
  int64_t top = -1;
  for (int64_t c = c0 + lane; c < c1; c += 64) {
    int64_t qb = 0, vb = 0, nc = 0;
    // (no per-column arrays: k_cmp_rowone recomputes a column's count and kind from its bytes,
    // cheaper than writing and re-reading 12 bytes a column)
    if (cmp_col<W32>(p, c, r, &qb, &vb, &nc, false)) { heap++; top = c; }
    n += nc;
    qs += qb;
    vs += vb;
  }
  heap = wave_sum64(heap);
  n = wave_sum64(n);
  qs = wave_sum64(qs);
  vs = wave_sum64(vs);
  long long t = (long long)top;
  for (int d = 32; d >= 1; d >>= 1) t = max(t, (long long)__shfl_xor(t, d, 64));
  if (lane == 0) {
    p.row_heap[r] = (int32_t)heap;
    p.row_one[r] = t < 0 ? 0 : (int64_t)t;
    p.row_n[r] = n;
    p.row_qb[r] = qs;
    p.row_vb[r] = vs;
  }
}

hipError_t cmp_cols_rows(const CmpParams& p, hipStream_t s) {
  if (p.n_rows > 0) {
    if (p.col_qo32) hipLaunchKernelGGL(k_cmp_cols_rowwave<true>, dim3((unsigned)((p.n_rows + 3) / 4)), dim3(256), 0, s, p);
    else hipLaunchKernelGGL(k_cmp_cols_rowwave<false>, dim3((unsigned)((p.n_rows + 3) / 4)), dim3(256), 0, s, p);
  }
  return hipGetLastError();
}


int cmp_onepass_cap(const CmpParams& p, uint32_t* scratch3, hipStream_t s, hipError_t* err) {
  *err = hipSuccess;
  if (p.n_rows <= 0) return 64;
  if ((*err = hipMemsetAsync(scratch3, 0, 12, s)) != hipSuccess) return 0;
  hipLaunchKernelGGL(k_cmp_rowmax2, dim3(blocks_of(p.n_rows)), dim3(256), 0, s, p, scratch3);
  uint32_t h[3] = {0, 0, 0};
  if ((*err = hipMemcpyAsync(h, scratch3, 12, hipMemcpyDeviceToHost, s)) != hipSuccess) return 0;
  if ((*err = hipStreamSynchronize(s)) != hipSuccess) return 0;
  if (h[0] > (uint32_t)CMP_ROW_CAP || h[1] > 65535u) return 0;
  int cap = 64;
  while (cap < (int)h[0]) cap <<= 1;
  return cap;
}

hipError_t cmp_rows_onepass(const CmpParams& p, int cap, hipStream_t s) {
  if (p.n_rows <= 0) return hipSuccess;
  // the sort's arrays (20 B an entry); the cell assembled in the same space needs <= 12 B an entry
  const size_t lds = (size_t)cap * 20;
  const void* kf = p.col_qo32 ? (const void*)k_cmp_rowone<true> : (const void*)k_cmp_rowone<false>;
  if (lds > 65536) {
    const hipError_t e = hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  if (p.col_qo32) hipLaunchKernelGGL(k_cmp_rowone<true>, dim3((unsigned)p.n_rows), dim3(CMP_ROW_THREADS), lds, s, p, cap);
  else hipLaunchKernelGGL(k_cmp_rowone<false>, dim3((unsigned)p.n_rows), dim3(CMP_ROW_THREADS), lds, s, p, cap);
  return hipGetLastError();
}

int cmp_row_cap(const CmpParams& p, uint32_t* scratch3, hipStream_t s, hipError_t* err, uint32_t* span) {
  *err = hipSuccess;
  if (p.n_rows <= 0) return 64;
  if ((*err = hipMemsetAsync(scratch3, 0, 12, s)) != hipSuccess) return 0;
  hipLaunchKernelGGL(k_cmp_rowmax, dim3(blocks_of(p.n_rows)), dim3(256), 0, s, p, scratch3);
  uint32_t h[3] = {0, 0, 0};
  if ((*err = hipMemcpyAsync(h, scratch3, 12, hipMemcpyDeviceToHost, s)) != hipSuccess) return 0;
  if ((*err = hipStreamSynchronize(s)) != hipSuccess) return 0;
  if (h[0] > (uint32_t)CMP_ROW_CAP || h[1] > 65535u || h[2] >= 0x7FFFFFFFu) return 0;
  *span = h[2];
  int cap = 64;
  while (cap < (int)h[0]) cap <<= 1;
  return cap;
}

hipError_t cmp_rows_fused(const CmpParams& p, void* klist, int cap, uint32_t span, bool write, hipStream_t s) {
  if (p.n_rows <= 0) return hipSuccess;
  if (write) {
    // output cell <= cap x (4 + 8) bytes + the meta byte; sources staged up to 96 KB a row
    const int oq_cap = cap * 4 + 16, ov_cap = cap * 8 + 16;
    const int src_cap = (int)std::min<uint64_t>((uint64_t)96 << 10, ((uint64_t)span * 2 + 64 + 15) & ~15ull);
    const size_t lds = (size_t)oq_cap + ov_cap + src_cap;
    const hipError_t e = hipFuncSetAttribute((const void*)k_cmp_rowwrite, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_cmp_rowwrite, dim3((unsigned)p.n_rows), dim3(CMP_ROW_THREADS), lds, s, p, (const CmpKept*)klist,
                       oq_cap, ov_cap, src_cap);
    return hipGetLastError();
  }
  const size_t lds = (size_t)cap * 20;
  if (lds > 65536) {
    const hipError_t e = hipFuncSetAttribute((const void*)k_cmp_row, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_cmp_row, dim3((unsigned)p.n_rows), dim3(CMP_ROW_THREADS), lds, s, p, (CmpKept*)klist, cap);
  return hipGetLastError();
}

}  // namespace tsdb
