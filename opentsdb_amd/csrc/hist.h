// hist.h -- internal declarations of the histogram path shared by the
// host side (hist.cpp) and the gfx950 kernels (k_hist.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "opts.h"

// the bucket-atomics skip of the profiling bits exists only in a -DTSDBHIP_KDBG build
#ifdef TSDBHIP_KDBG
#define HIST_SKIP_ADD(p) (((p).dbg & 1) != 0)
#else
#define HIST_SKIP_ADD(p) false
#endif

namespace tsdb {

// Bucket dictionary: open-addressing hash set of the store's bucket keys
// (canonical lower bits << 32 | canonical upper bits, Float.floatToIntBits canonical NaN).
static constexpr uint64_t HK_EMPTY = ~0ull;   // never a canonical key (0xFFFFFFFF is a non-canonical NaN)
static constexpr int HT_BITS = 16;             // 65536 slots: up to 32768 distinct buckets per store
static constexpr int64_t HT_SIZE = 1ll << HT_BITS;
static constexpr int HK_MAX = 1 << (HT_BITS - 1);

// per-column decode status (k_hist_validate)
enum : uint8_t { HC_DROP = 0, HC_SIMPLE = 1, HC_LONG = 2 };
// status bit: a SimpleHistogram column whose bucket keys are not strictly increasing (it may
// repeat a key: fromHistogram's TreeMap.put keeps the last count)
constexpr uint8_t HC_UNSORTED = 0x80;
constexpr uint8_t HC_KIND = 0x7F;

struct HistLoadParams {
  int64_t n_cells;
  const uint64_t* voff;      // [n_cells + 1]
  const uint8_t* val;
  const uint8_t* codec;      // [256] codec kind of each id
  uint8_t* status;           // [n_cells] HC_*
  uint64_t* hkey;            // [HT_SIZE]
  int32_t* hcount;           // distinct keys inserted (overflow: > HK_MAX)
};

// Query over the resident store.  Positions are the spans' datapoints in HistogramSpan
// iteration order (rows sorted by base time); pos_cell maps a position to its column.
struct HistQueryParams {
  // store
  const uint64_t* voff;
  const uint8_t* val;
  const int64_t* pos_cell;   // [n_pos]
  const int64_t* pos_ts;     // [n_pos] timestamp (ms)
  const uint8_t* pos_kind;   // [n_pos] HC_SIMPLE / HC_LONG
  const int64_t* row_pos;    // [n_rows + 1] positions of each (kept) row
  const uint64_t* hkey;      // dictionary hash table
  const int32_t* hidx;       // [HT_SIZE] dictionary index of each slot
  const uint32_t* dict_lo;   // [D] bucket bounds (float bits) in dictionary (TreeMap) order
  const uint32_t* dict_up;
  int32_t D;                 // dictionary size
  int32_t C;                 // accumulator columns: D buckets, underflow, overflow, long data
  // present spans of the query (one thread each in k_hist_slots)
  int64_t n_spans;
  const int64_t* sp_rlo;     // [n_spans] in-range kept rows [rlo, rhi)
  const int64_t* sp_rhi;
  const int32_t* sp_out;     // [n_spans] emitted group index
  // geometry (ms)
  int64_t start, end;        // HistogramSpanGroup start / end (scan bounds)
  int64_t qs, qe;            // query start / end ("all")
  int32_t ds;                // 0 none, 1 fixed interval, 2 all, 3 calendar (union of per-span intervals)
  int32_t ds_sum;            // the downsampling function is "sum"
  int64_t I;                 // interval
  int64_t B0;                // slot 0 timestamp (dense modes)
  int64_t K;                 // slots per group (dense modes)
  const int64_t* cal_tab;    // calendar: interval boundaries, one run per distinct span anchor
  const int64_t* sp_cal;     // calendar: [n_spans][2] first boundary of the span's run, boundaries in it
  int64_t cal_seek;          // calendar: HistogramDownsampler.seekInterval's target
  // outputs of k_hist_slots
  int32_t* pos_slot;         // [n_pos] slot (dense) or -1
  int64_t* pos_key;          // [n_pos] sparse mode: (group << 42 | ts - start) or -1; after the
                             // greedy walk (spans out of time order): (group << 42 | step)
  int32_t greedy;            // pos_key holds walk steps: a point's timestamp is its positions' pos_ts
  int32_t* err;              // [2]: first error code, reason
  // accumulation ([point][C] u64) -- point = group * K + slot (dense) or a union index (sparse)
  const int32_t* pos_point;  // sparse mode: [n_pos] point of each position, -1 excluded (null: dense)
  uint64_t* acc;
  uint32_t* pres;            // [point][W] bucket presence bits (null: not tracked)
  int32_t W;
  uint32_t* pkind;           // [point] codec bits (1 simple, 2 long)
  int64_t n_points;
  // finalisation
  int32_t n_pct;
  const float* pct;          // [n_pct]
  double* out_pct;           // [n_out * n_pct]
  const int64_t* pt_out;     // [n_points] exclusive scan of emitted points (n_points + 1)
  int64_t* out_ts;
  const int64_t* pt_ts;      // sparse mode: [n_points] timestamp of each point
  const int32_t* pt_group;   // sparse mode: [n_points] emitted group of each point
  int32_t* out_group;        // [n_out]
  uint8_t* out_kind;
  int64_t* out_count;        // [n_out * (D + 2)] (show_buckets)
  uint8_t* out_present;      // [n_out * D]
  const int32_t* col_lid;    // [n_cells] bucket layout of the column (-1: none), or null
  const int32_t* lay_off;    // [layouts] first entry of the layout's dictionary indices in lay_di
  const int32_t* lay_di;     // dictionary index of each bucket of each layout
  int32_t dbg;               // profiling bits (option DBG, a -DTSDBHIP_KDBG build only; results invalid): 1 skip the bucket atomics
};

hipError_t hist_validate(const HistLoadParams& p, hipStream_t s);
hipError_t hist_slots(const HistQueryParams& p, hipStream_t s);
// lkey / lidx: the dictionary as an LDICT-slot table for LDS (k_hist.hip), or null
hipError_t hist_accum(const HistQueryParams& p, int64_t n_pos, const uint64_t* lkey, const int32_t* lidx, hipStream_t s);
static constexpr int HIST_LDICT = 1024;
// slot of a bucket key in the LDS dictionary table (HIST_LDICT = 2^10 slots): two 32-bit
// multiplies instead of the global table's 64-bit mixer (host and device must agree)
__host__ __device__ inline uint32_t lds_dict_slot(uint64_t k, uint32_t mask = HIST_LDICT - 1) {
  const uint32_t h = ((uint32_t)(k >> 32) * 0x9E3779B1u) ^ ((uint32_t)k * 0x85EBCA77u);
  return (h ^ (h >> 16)) & mask;
}
// slots of k_hist_accw's compact LDS table for a D-bucket dictionary (load factor <= 1/2)
inline int hist_lds_slots(int D) {
  int n = 64;
  while (n < 2 * D) n <<= 1;
  return n;
}
static constexpr int64_t HIST_WLDS = 52 * 1024;   // LDS of a k_hist_accw block (three blocks per CU)
// the present spans' in-range positions in span order: vpos[off[i] .. off[i + 1]) = span i's
hipError_t hist_vpos(const int64_t* rlo, const int64_t* rhi, const int64_t* row_pos, int64_t n_spans, uint32_t* len,
                     int64_t* off, int32_t* vpos, int64_t* nvp, void** tmp, size_t* tmp_bytes, hipStream_t s);
// points of the k_hist_accw LDS window for this query (0: the counters do not fit, use hist_accum)
int hist_window_points(const HistQueryParams& p, int lslots);
// windowed accumulation over vpos (spans sorted by output group); needs the LDS dictionary
// tix_buf: nvp x 24 B of scratch (the positions' packed column entries, k_hist_tidx)
hipError_t hist_accum_window(const HistQueryParams& p, const int32_t* vpos, int64_t nvp, const uint64_t* lkey,
                             const int32_t* lidx, int lslots, void* tix_buf, hipStream_t s);
// Bucket layouts (load): a SimpleHistogram column with strictly increasing keys whose key bytes
// equal the previous column's shares its layout; col_lid[c] = the layout, lay_col[l] = its first
// column.  hist_layout_index writes col_lid / lay_col and returns the layout count;
// hist_layout_di fills lay_di[lay_off[l] + j] = the dictionary index of layout l's bucket j.
hipError_t hist_layout_index(int64_t n_cells, const uint64_t* voff, const uint8_t* val, const uint8_t* status,
                             uint32_t* head, int64_t* excl, int32_t* col_lid, int32_t* lay_col, int64_t* n_layouts,
                             void** tmp, size_t* tmp_bytes, hipStream_t s);
hipError_t hist_layout_di(int64_t n_layouts, const int32_t* lay_col, const int32_t* lay_off, const uint64_t* voff,
                          const uint8_t* val, const uint64_t* hkey, const int32_t* hidx, int32_t* lay_di, hipStream_t s);
static constexpr int HIST_LAY_MAXB = 32;   // layouts of more buckets take the keyed path
hipError_t hist_flags(const HistQueryParams& p, uint32_t* flag, hipStream_t s);   // [n_points] 1 = emitted
hipError_t hist_final(const HistQueryParams& p, hipStream_t s);
hipError_t hist_scan(const uint32_t* flag, int64_t* out, int64_t n, void** tmp, size_t* tmp_bytes, hipStream_t s);
// HistogramAggregationIterator.next()'s walk over raw spans some of which are out of time order
// (one wave a group; span state in sp_q / sp_ts, [n_spans] scratch); gsp[G + 1]: the group's spans
hipError_t hist_walk(const HistQueryParams& p, const int64_t* gsp, int64_t G, int64_t max_spans, int64_t* sp_q,
                     int64_t* sp_ts, hipStream_t s);
hipError_t hist_sparse(const HistQueryParams& p, int64_t n_pos, uint64_t* key2, uint32_t* pos, uint32_t* pos2,
                       uint32_t* head, int64_t* incl, int64_t* pt_ts, int32_t* pt_group, int64_t* n_points,
                       void** tmp, size_t* tmp_bytes, hipStream_t s);

}  // namespace tsdb
