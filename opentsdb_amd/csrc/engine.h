// engine.h -- internal declarations shared by the host side (engine.cpp) and the
// gfx950 kernels (kernels.hip) of libtsdbhip.  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>

#include "rollup_codec.h"
#include "opts.h"
#include <stdint.h>

namespace tsdb {

static constexpr int CH_ROWS = 512;   // k_fast chunk: datapoints per chunk (64 lanes x 8), = CH in kcommon.h

// One compacted cell (RowSeq) as laid out in HBM.  qoff/voff are 16-byte aligned.
struct RowDesc {
  uint64_t qoff;    // byte offset of the qualifiers in the qualifier blob
  uint64_t voff;    // byte offset of the values (incl. trailing meta byte) in the value blob
  uint32_t base;    // row base time, seconds
  uint32_t ndp;     // datapoints in the row
  uint32_t qlen;    // qualifier bytes
  uint32_t vlen;    // value bytes
  uint32_t flags;   // ROW_* below
  int32_t lsb;      // exactness certificate: min exponent of the least significant set bit
                    // over the row's non-zero finite values (INT32_MAX if none)
  double absmax;    // max |value| over the row (inf if any +-inf)
};
static_assert(sizeof(RowDesc) == 48, "RowDesc layout");

// RowDesc.flags
enum : uint32_t {
  ROW_QW_MASK = 0x7,        // 2 = all 2-byte (second) qualifiers, 4 = all 4-byte (ms), 0 = mixed
  ROW_VL_SHIFT = 8,         // uniform value length 1/2/4/8, 0 = variable (vle ints)
  ROW_VL_MASK = 0xF00,
  ROW_ERR = 0x10000,        // malformed cell (IllegalDataException when decoded)
  ROW_ALLF = 0x20000,       // every value is floating point
  ROW_NAN = 0x40000,        // some value is NaN
  ROW_NEGZ = 0x80000,       // some value is -0.0
  ROW_UNSORTED = 0x100000,  // datapoint offsets not strictly increasing
  ROW_SFIRST = 0x200000,    // first row of its series (set by the host at load)
  ROW_ALLI = 0x400000,      // every value is an integer
  ROW_VLE2 = 0x800000,      // every value is 1 or 2 bytes long
  ROW_NOCERT = 0x1000000,   // two of the row's values cannot add exactly (row_nocert): an order-free sum is ruled out
};

// The exactness certificate (n * absmax <= 2^(52 + lsb)) fails for any bucket of
// two or more of this row's values: sums over them must keep Java's order (k_grid's sequential path).
__host__ __device__ inline bool row_nocert(int lsb, double absmax) {
  if (lsb == INT32_MAX || absmax == 0.0) return false;
  return isinf(absmax) || 2.0 * absmax * (1.0 + 1e-12) > ldexp(1.0, 52 + lsb);
}

// A rollup value row with its lock-step count row, packed once per rollup batch (k_ro_pack) for
// k_ro_pairs: 24 B a pair where k_seq_rows_ro reads two 48-B RowDescs, the partner and the
// series of every row, count rows included.
struct RoPair {
  uint32_t base;    // the rows' base time (s)
  uint32_t qoff;    // value row: qualifier bytes offset
  uint32_t voff;    // value row: value bytes offset
  uint32_t cvoff;   // count row: value bytes offset
  uint32_t meta;    // ndp | log2 vl << 16 | log2 count vl << 18 | 4-byte qualifiers << 20 | RP_OK
  int32_t series;   // the value series (resident position)
};
static_assert(sizeof(RoPair) == 24, "RoPair layout");
// A run of RoPairs of one series that differ only by a constant step: the pair j rows into the
// run is base0 + j * bstep * 3600 s, qoff0 + j * qs * 16 bytes, ...  A rollup table's hour rows
// are such runs (one a series when every row holds the same cells), so the walk reads a 4-B run
// id a pair and one 32-B run for every series instead of 24 B a pair (k_ro_pairs / k_ro_rows).
struct RoRun {
  uint32_t first;   // the run's first pair
  uint32_t base0, qoff0, voff0, cvoff0;
  uint32_t meta;    // RoPair::meta, equal over the run
  int32_t series;
  uint32_t step;    // qs (7 bits) | vs << 7 (9 bits) | cvs << 16 (8 bits) | bstep << 24 (8 bits)
};
static_assert(sizeof(RoRun) == 32, "RoRun layout");
__host__ __device__ inline RoPair ro_run_pair(const RoRun& R, uint32_t i) {
  const uint32_t j = i - R.first;
  RoPair P;
  P.base = R.base0 + j * ((R.step >> 24) * 3600u);
  P.qoff = R.qoff0 + j * ((R.step & 0x7Fu) << 4);
  P.voff = R.voff0 + j * (((R.step >> 7) & 0x1FFu) << 4);
  P.cvoff = R.cvoff0 + j * (((R.step >> 16) & 0xFFu) << 4);
  P.meta = R.meta;
  P.series = R.series;
  return P;
}
enum : uint32_t {
  RP_OK = 0x80000000u,    // k_seq_rows_ro's premises hold for the pair
  RP_VOK = 0x40000000u,   // k_seq_rows' premises hold for the value row alone
};

// Per-tile partial group state, structure of arrays, [tile][K].
struct Partials {
  double* a;
  double* b;
  uint32_t* n;
  uint32_t* f;   // bit0 union (a real point of some series sits on this slot), bit1 has, >>2 count
};

enum : uint32_t { PF_UNION = 1u, PF_HAS = 2u };

enum : int32_t { MULTI_ON = 1, MULTI_DEV = 2 };
// Per-tile partial states of the fused multi-aggregator pass (GridParams.multi), [tile][K]:
// sum / avg (sum, nl), min (mn), max (mx), dev (mean, m2, nl), count (nz); f = union flags.
// Aggregator x reads them as Partials in k_reduce (the mapping is in engine.cpp run_multi_fused).
struct MultiPartials {
  double *sum, *mn, *mx, *mean, *m2;
  uint32_t *nl, *nz, *f;
};

// Kernel modes
enum : int { MODE_GRID = 0, MODE_ALL = 1, MODE_TABLE = 2 };   // TABLE: slot k = [bounds[k], bounds[k+1]) (calendar months / years)

// Group-aggregator classes (cross-series reduction)
enum : int {
  GA_SUM = 0, GA_AVG, GA_COUNT, GA_SQUARESUM, GA_MIN, GA_MAX, GA_DEV, GA_FIRST, GA_LAST,
  GA_DIFF, GA_MULT, GA_NONE
};
// Downsample function classes (per-bucket, per-series, sequential in time order)
enum : int {
  F_SUM = 0, F_AVG, F_COUNT, F_SQUARESUM, F_MIN, F_MAX, F_DEV, F_FIRST, F_LAST, F_DIFF, F_MULT,
  F_NUM,
  F_SEL = 100   // percentile / median: order statistics per bucket (k_pct.hip)
};

struct GridParams {
  // data
  const RowDesc* rows;
  const int64_t* series_row_ptr;
  const uint8_t* qual;
  const uint8_t* val;
  const uint8_t* val2;   // int16 copy of 1-2-byte integer values, at the row's qualifier offset
  // tiles: series [tile_begin[t], tile_end[t]) of group tile_group[t]
  const int64_t* tile_begin;
  const int64_t* tile_end;
  const int32_t* tile_group;
  int64_t n_tiles;
  int64_t n_launch;      // waves launched (list launches: the list's capacity); 0 = n_tiles
  // query geometry (ms unless noted)
  int64_t ss, se;        // scan bounds, seconds: rows with base in [ss, se)
  int64_t B0;            // timestamp of slot 0
  int64_t I;             // interval
  int64_t K;             // slots
  int64_t qs, qe;        // "all" bounds (raw query start/end)
  const int64_t* bounds; // MODE_TABLE: K + 1 slot boundaries (ms)
  int64_t seek_ms;       // MODE_TABLE: points before this are skipped (Downsampler.seekInterval)
  int64_t seek_any;      // the point every span's Downsampler seeks to (any mode; stream order, so_row_skip)
  int32_t skip0;         // MODE_TABLE: slot 0 lies before the SpanGroup start (a filled leading
                         // bucket): it feeds RateSpan but AggregationIterator drops it
  float rcpI;            // 1/I as float (slot division)
  int32_t mode;          // MODE_*
  int32_t ga;            // GA_*
  int32_t interp;        // TSDB_INTERP_*
  int32_t fill;          // TSDB_FILL_*
  int32_t rate, counter, drop;
  int64_t counter_max, reset_value;
  int32_t wave_lds;      // bytes of LDS per wave
  int32_t waves;         // waves per workgroup
  // slot arrays in global memory (large K): [tile][K]
  double* g_dense;
  uint8_t* g_pres;
  double* g_rate;
  // outputs
  Partials part;
  uint32_t* group_active;
  int32_t* err;          // first error code (atomicCAS from 0)
  // k_grid over a tile list (tiles k_fast handed back): tile = tile_list[i], i < *tile_list_n
  const int32_t* tile_list;
  const int32_t* tile_list_n;
  const int32_t* row_series;   // [n_rows] series of each row (k_seq_rows)
  uint32_t* redo_mark;         // [n_series] a series is on redo_list (k_seq_rows)
  const int32_t* ro_partner;   // [n_rows] rollup batch: a value row's count row (-1: a count row,
                               // -2: the count series does not mirror the value series' rows)
  const RoPair* ro_pairs;      // rollup batch: the packed value / count row pairs (k_ro_pairs)
  const RoRun* ro_runs;        // ... or the pairs as runs (ro_runs[ro_rid[i]] holds pair i)
  const uint32_t* ro_rid;
  // k_fast: geometry in "n-units" (seconds when every row has second qualifiers and the
  // interval / slot origin are whole seconds, else milliseconds) and the redo list
  int32_t unit_s;        // 1: n-units are seconds
  int32_t In;            // interval in n-units
  int64_t B0n;           // slot-0 timestamp in n-units
  double rcpn;           // 1/In rounded up (floor(n * rcpn) == n / In for 0 <= n < 2^50)
  int32_t* redo_list;
  int32_t* redo_n;
  // k_pct / k_emit: per-series bucket values computed before the group-by step
  int32_t sel_fn;        // TSDB_AGG_* of the percentile / median downsample function
  bool pct_vonly;        // k_pct_rows key kernel: rows certified at load, values read alone
  bool pct_v6;           // ... and no such row over 384 values: 6 values a lane
  int64_t n_series;
  double* pre_dense;     // [n_series][K]
  uint8_t* pre_pres;     // [n_series][K]
  int32_t shortk;        // k_fast launch runs k_short (1: one row per series) / k_rows (2: rows <= CH)
  int32_t oneb;          // streaming kernels: buckets of an hour or more -- try the one-bucket chunk fold
  int32_t win_w;         // k_hwin: slots a window (3600 s / interval; windows start on slot multiples of it)
  int32_t win_split;     // k_hwin: work items a tile (each a contiguous range of its windows); 0/1 = whole tiles
  int32_t short6;        // k_short, vle class: 6 datapoints a lane (rows of <= 384 points)
  // percentile / median as the group-by aggregator (k_emit_vals, k_sel_seg): the value of
  // span i of group g at slot k goes to sel_vals[(gsp[g] + i) * K + k] ([series][slot], the
  // span's K values contiguous); NaN = no contribution
  double* sel_vals;
  uint8_t* sel_uni;            // [G][K]: some series contributed with a real point (emit)
  uint8_t* sel_wr;             // [series] 1 = sel_direct wrote the series' row (null: rows pre-filled)
  const int64_t* group_series_ptr;   // [G + 1]
  // 1: the downsampling pass writes the contributions itself (kcommon.h sel_direct_out;
  // K <= 64, no rate)
  int32_t sel_direct;
  int32_t sel_cols;              // sel_direct into [gsp[g] * K + k * n_g + i] (contiguous (group, slot) columns)
  int32_t sel_stage;             // k_short + sel_cols: byte offset of an 8-series x K stage in the wave's LDS (0: none)
  // sampled window (k_short KR 5, kcommon.h sel_window_out): each (group, slot) column's window
  // [win_lo, win_hi] ([G][K]); the tile's values inside go to win_val ([tile][K][WIN_CAP], a
  // tile's whole column) and at the tile's end to the column's candidates (win_cand
  // [G][K][WIN_CCAP], at win_cur's cursor); the column's counts below | above << 32 in win_gcnt
  int32_t sel_win;
  int32_t win_stage;             // KR 5: byte offset of the wave's LDS stage of kept values (WIN_LDS a lane)
  const double* win_lo;
  const double* win_hi;
  double* win_val;
  unsigned long long* win_gcnt;
  uint32_t* win_cur;
  double* win_cand;
  // non-null: the grid kernels write every series' bucket values / presence here
  // ([series][K], before rate and fill) instead of its SpanGroup contributions
  double* dense_out;
  uint8_t* pres_out;
  // k_pct BIG pass: each of the n_launch waves owns big_cap values of big_scratch for buckets
  // of more than PCT_CAP values (big_cap >= the largest series' in-range datapoints)
  double* big_scratch;
  int64_t big_cap;
  // fused multi-aggregator pass (tsdbhip_run_multi): the register-partial kernels keep every
  // decomposable aggregator's state and write them to mp (K <= 64, no rate, LERP + count)
  int32_t multi;          // MULTI_ON | MULTI_DEV (the Welford state is kept only for a dev query)
  MultiPartials mp;
  int32_t dbg;           // k_short profiling switches (TSDBHIP_DBG, results invalid): 1 skip series end,
                         // 2 skip chunk fold, 8 consume loads, 16 stop after the descriptors, 32 load row 0 only
};

struct ReduceParams {
  Partials part;
  const int64_t* group_tile_ptr;  // [G+1]
  int64_t G, K;
  int32_t ga;
  double* out_val;                // [G][K]
  uint8_t* out_flag;              // [G][K] bit0 emit
  int32_t* err;
  Partials state;                 // non-null a: write the merged (unfinalised) state instead
  int32_t no_inf;                 // per-span pass feeding another aggregator: no +-Inf check
};

// Order statistic per (group, slot) (percentile / median group-by aggregator): segment
// (g, k) is vals[(gsp[g] + i) * K + k], i < gsp[g + 1] - gsp[g].
struct SelParams {
  const double* vals;             // [series][K], or (cols) [gsp[g] * K + k * n_g + i]
  int32_t cols;
  double* scratch;                // [sum n_g * K] key space for segments longer than SEL_CAP
  const uint8_t* uni;             // [G][K]
  const int64_t* group_series_ptr;
  int64_t G, K;
  int32_t fn;                     // TSDB_AGG_* (median / pXX / epXXrY)
  double* out_val;
  uint8_t* out_flag;
  int32_t* err;
};
static constexpr int SEL_CAP = 12288;   // values of one segment staged in LDS (96 KB)
static constexpr int WIN_CAP = 64;      // window values kept a (tile, slot) (k_short KR 5): a tile's whole column
static constexpr int WIN_LDS = 8;       // ... of which the first WIN_LDS a lane in LDS (no global store in the ring)
static constexpr int WIN_SCAP = 1024;   // sample values a column (k_win_bounds)
static constexpr int WIN_CCAP = 1024;   // window values a column (k_win_select)

// The sampled-window select (engine.cpp sel_window): the sample pass's values of each (group,
// slot) column (the sampled tiles' positions of the column layout) -> the window bounds; then
// the counts and window values of the main pass -> the order statistics.
struct WinParams {
  const double* vals;             // the column layout (sample pass)
  const uint8_t* wr;              // [series] written by the sample pass (other positions are stale)
  const int64_t* group_series_ptr;
  const int64_t* tile_begin;
  const int64_t* tile_end;
  const int32_t* samp_ptr;        // [G + 1] into samp_pos
  const int32_t* samp_pos;        // the sampled positions of each group (series - group's first, <= WIN_SCAP)
  const int64_t* group_tile_ptr;  // [G + 1] the group's tiles
  const uint8_t* uni;             // [G][K]
  double* lo;                     // [G][K]
  double* hi;
  const unsigned long long* gcnt; // [G][K] below | above << 32
  const uint32_t* cur;            // [G][K] values inside (the candidates' cursor)
  const double* cand;             // [G][K][WIN_CCAP] the values inside
  int64_t G, K;
  int32_t fn;
  double* out_val;
  uint8_t* out_flag;
  int32_t* err;
  int32_t* fail;                  // set when a column's window misses its ranks (the caller redoes the query)
};
hipError_t launch_win_bounds(const WinParams& p, hipStream_t s);
hipError_t launch_win_select(const WinParams& p, hipStream_t s);

// Ordered (TSDB_QF_ORDERED) reduction of the span values per (group, slot).
struct OrdParams {
  const double* vals;             // [series][K] as GridParams.sel_vals (fill pattern = no value)
  const uint8_t* uni;             // [G][K]
  const int64_t* group_series_ptr;
  int64_t G, K;
  int32_t ga;
  double* out_val;
  uint8_t* out_flag;
  int32_t* err;
};

// Rank-ordered merge of all-gathered per-rank partial buffers (tsdbhip_finalize).
struct RankMergeParams {
  const unsigned char* base;      // n_ranks consecutive buffers of `stride` bytes
  int64_t stride;
  int64_t off_b, off_n, off_f, off_act;   // byte offsets of the parts inside one buffer
  int32_t n_ranks;
  int64_t G, K;
  int32_t ga;
  double* out_val;
  uint8_t* out_flag;
  uint32_t* out_act;
  int32_t* err;
};

// Multi-device owner merge (multi.cpp): the partial states of group g (K slots) that n_mini later
// devices hold, gathered in device order as mini states ([a K f64 | b K f64 | n K u32 | f K u32 |
// act u32], mini_state_stride(K) bytes each, multi.h), folded into the owner's state of g in that order.
struct StateFoldParams {
  unsigned char* state;           // the owner's partials buffer (tsdbhip_partials layout)
  int64_t off_b, off_n, off_f, off_act;
  int64_t g, K;
  int32_t ga;
  const unsigned char* mini;
  int64_t mini_stride;
  int32_t n_mini;
};

// ---- raw path (no downsampling): AggregationIterator over the timestamp union ----
// A decoded datapoint: tsf = timestamp (ms) | RAW_FLOAT when the value bits are a double
// (AggregationIterator keeps exactly this FLAG_FLOAT encoding, src/core/AggregationIterator.java:112-118).
struct RawPt {
  int64_t tsf;
  uint64_t bits;
};
static constexpr int64_t RAW_FLOAT = (int64_t)0x8000000000000000ULL;
static constexpr int64_t RAW_TIME_MASK = 0x7FFFFFFFFFFFFFFFLL;
static constexpr int RAW_W = 8;                // 64-point windows per k_raw_eval wave
static constexpr int RAW_STRIP = 64 * RAW_W;   // union points per k_raw_eval wave
static constexpr int RAW_SEL_SPANS = 32;       // spans per k_raw_vals wave

struct RawParams {
  // decode
  const RowDesc* rows;
  const uint8_t* qual;
  const uint8_t* val;
  int64_t n_rows;
  const int64_t* row_pt_off;   // [n_rows] first point of the row, -1 outside the scan range
  RawPt* pts;                  // [n_pts]
  // series (resident, group-sorted order)
  int64_t n_series;
  const int64_t* sp_off;       // [n_series + 1] point range of each series
  int32_t* sp_n;               // [n_series] points (rate mode: kept rate points, compacted in place)
  // rate (RateSpan, src/core/RateSpan.java:121-180)
  int32_t rate, counter, drop;
  int64_t counter_max, reset_value;
  // union of timestamps, one chunk of groups [g0, g1) at a time
  int64_t start_ms, gran, W;   // bitmap origin, granularity (ms), words per group
  int64_t g0, g1;
  const int64_t* grp_ser;      // [G + 1] series range of each group
  uint32_t* bitmap;            // [(g1 - g0) * W]
  uint32_t* wbase;             // [(g1 - g0) * W] exclusive popcount prefix
  int32_t* U;                  // [g1 - g0] union size
  int32_t* rank;               // [n_pts] union points strictly before the point
  // evaluation
  const int64_t* out_off;      // [g1 - g0] chunk-relative output offset of each group
  const int32_t* strip_g;      // [n_strips] chunk-relative group
  const int32_t* strip_t;      // [n_strips] strip index inside the group (first union point t * RAW_STRIP)
  int64_t n_strips;
  const int64_t* cur_off;      // [g1 - g0] offset of the group's cursor table
  int32_t* cur;                // per group [strip][span]: counted points with rank < strip start
  int32_t ga, interp, do_long, do_double;
  int64_t* out_ts;
  uint64_t* out_bits;
  uint8_t* out_int;
  int32_t* err;
  // percentile / median group-by (k_raw_vals, k_raw_sel) over a batch of strips (strip_g /
  // strip_t point at the batch's first strip): span i's operand at point ua + j of batch
  // strip b sits at vals_off[b] + i * RAW_STRIP + j (span-major: the lanes of a wave coalesce)
  int32_t sel_fn;              // TSDB_AGG_* (median / pXX / epXXrY); 0 = not a selection query
  const int64_t* vals_off;     // [n_strips] of the batch
  int64_t* vals_l;             // runLong operands
  double* vals_d;              // runDouble operands (NaN = no value; runDouble skips NaNs)
  uint8_t* vals_p;             // 1 = the span has a long operand at the point
  // cells with unsorted datapoints (k_raw_merge instead of the bitmap union): the greedy
  // AggregationIterator walk gives every point its step; the evaluation then also meets points
  // on either end of a span's window and windows with x1 <= x0
  int32_t uns;
  int32_t lerp_fast;           // k_raw_eval: exact double LERP for strip-wide windows (lerpw_*)
  const int64_t* bnd_off;      // [g1 - g0] offset of each group's step timestamps in mts
  int64_t* mts;                // step timestamps, bnd_off layout (a group's points bound its steps)
  int32_t* m_pos;              // [n_series] next point of the span
  int64_t* m_head;             // [n_series] timestamp of that point (INT64_MAX: none)
  uint8_t* dz;                 // [points of the chunk] a long LERP divided by zero (k_raw_vals)
};

struct SynthParams {
  int64_t n_series, n_groups, n_rows_per_series, n_points;
  int64_t pos0;                  // global batch position of local series 0 (a shard of the store)
  int64_t start_ms, period_ms;
  int32_t value_kind, ms_qual;
  int64_t int_mod;
  uint64_t seed;
  const int64_t* grp_off;        // [G+1] batch position offsets of each group
  // per-row template (identical for every series): first point index, count, base time
  const int64_t* row_k0;
  const int32_t* row_n;
  const uint32_t* row_base;
  RowDesc* rows;                 // [n_series * R]
  uint8_t* qual;
  uint8_t* val;
  uint32_t* row_vbytes;          // pass 1 output (value bytes incl. meta)
  int32_t* group_id;             // [n_series] (batch order)
};

// rollup generation (k_rollup.hip); grid = n series (batch order) x K slots
struct RollupParams {
  const double* val;        // [G][K] downsampled bucket values (sorted series positions)
  const uint8_t* flag;      // [G][K] bucket present
  const int64_t* ord;       // [n series] sorted position of the i-th series in batch order
  const int64_t* orig;      // [G] batch index of sorted position
  const uint8_t* allint;    // [G] every datapoint of the series is an integer
  int64_t n, K, B0, I, start_ms, end_ms;
  RollupIv iv;
  int32_t agg_id;
  int32_t as_long_all;      // count: every value is a long
  uint32_t* cnt;            // [n] cell flag      -> coff
  uint32_t* vsz;            // [n] value length   -> voff
  const int64_t* coff;
  const uint64_t* voff;
  int32_t* o_series;
  uint32_t* o_base;
  uint8_t* o_qual;
  uint64_t* o_voff;
  uint8_t* o_val;
  int32_t* err;
};
// fused per-series reduction of every rollup function (k_rollup.hip): out[f * stride + s * K + k]
// for f = 0 sum, 1 count, 2 max, 3 min; pres[s * K + k] = the bucket has a datapoint
struct RollupAggParams {
  double* out;
  int64_t stride;           // n_series * K
  int64_t K;
  uint8_t* pres;
};
hipError_t launch_rollup_agg(const GridParams& p, const RollupAggParams& rp, hipStream_t s);
// each series' first datapoint >= t0 in rows with base in [ss, se) (INT64_MAX: none)
// ---- query-time compaction (k_compact.hip) ----------------------------
enum : uint32_t { CMP_IGNORE = 0, CMP_DATA = 1, CMP_APPEND = 2 };
struct CmpParams {
  // input: the scanner's rows, every column (KeyValue) of a row in scan order
  int64_t n_rows, n_cols;
  const int64_t* row_col_ptr;   // [n_rows + 1]
  const uint64_t* col_qo;       // [n_cols + 1] qualifier bytes of each column
  const uint64_t* col_vo;       // [n_cols + 1] value bytes
  const uint32_t* col_qo32;     // the same in 32 bits (one-pass path, blobs under 4 GB), else null
  const uint32_t* col_vo32;
  const int64_t* col_ts;        // [n_cols] KeyValue timestamps, or null (all equal)
  const uint8_t* q;
  const uint8_t* v;
  int32_t fix_dup;
  int32_t dtcs;                 // 0: defaultMergeDataPoints; 1 / 2: dtcsMergeDataPoints keeping the max / min
  // per column
  int32_t* col_row;             // [n_cols]
  int64_t* col_n;               // [n_cols] datapoints the column contributes
  int64_t* col_off;             // [n_cols + 1] their first entry
  uint32_t* col_info;           // kind | 4: value starts 4 bytes in | 8: fixed up | fixed flags byte << 8
  // per row
  int32_t* row_heap;            // columns in the compaction heap
  int64_t* row_one;             // one of them (the only one when row_heap == 1)
  int32_t* row_err;             // first error: TSDB_E_ILLEGAL_DATA or TSDB_E_NOT_IMPLEMENTED
  int64_t* row_n;               // one-pass path (k_cmp_cols_rowwave): datapoints of the row,
  int64_t* row_qb;              //   bounds of its compacted qualifier bytes
  int64_t* row_vb;              //   and value bytes (before the meta byte)
  // entries (one per datapoint of every column)
  int64_t n_ent;
  uint64_t* key;                // [n_ent] row << 22 | offset (ms), then sorted
  uint64_t* key2;
  uint32_t* idx;                // [n_ent] entry ordinal, sorted along
  uint32_t* idx2;
  uint32_t* ent_col;            // [n_ent] (by ordinal)
  uint32_t* ent_qo;             // qualifier position inside the column (append: inside its value)
  uint32_t* ent_vo;             // value position inside the column value
  uint32_t* klen;               // [n_ent] by sorted position: kept | ms << 1 | qlen << 2 | vlen << 8
  int64_t* sq;                  // [n_ent + 1] exclusive sums over sorted positions of kept qualifier bytes
  int64_t* sv;                  //   ... value bytes
  int64_t* sc;                  //   ... kept datapoints
  int64_t* sm;                  //   ... kept millisecond datapoints
  // per row results
  int64_t* row_lo;              // first sorted position of the row
  int64_t* row_q;               // compacted qualifier bytes
  int64_t* row_v;               // compacted value bytes (incl. the meta byte)
  int32_t* row_state;           // 0: no cell (compacted == null, or an error), 1: merged, 2: the column as stored
  uint8_t* row_meta;
  // output
  const int64_t* row_dq;        // [n_rows] destination of the row's qualifiers (-1: none)
  const int64_t* row_dv;
  uint8_t* out_q;
  uint8_t* out_v;
};
hipError_t cmp_analyze(CmpParams& p, void** tmp, size_t* tmp_bytes, hipStream_t s);   // through k_cmp_cols, col_off
hipError_t cmp_entries(CmpParams& p, void** tmp, size_t* tmp_bytes, int end_bit, hipStream_t s);   // explode, sort, dedup, scans, rows
hipError_t cmp_write(const CmpParams& p, hipStream_t s);
// The per-row path (k_cmp_row / k_cmp_rowwrite): every row's datapoints sorted and deduplicated
// by one block in LDS, the kept ones listed (16 B each, klist: n_ent entries) and written after
// the host layout.  cmp_row_cap: the largest row's datapoints / columns / bytes of the chunk
// (after cmp_analyze) -> the LDS capacity to launch with, 0 when a row does not fit.
// *span: the largest row's qualifier or value bytes (the write pass's LDS stage).
int cmp_row_cap(const CmpParams& p, uint32_t* scratch3, hipStream_t s, hipError_t* err, uint32_t* span);
hipError_t cmp_rows_fused(const CmpParams& p, void* klist, int cap, uint32_t span, bool write, hipStream_t s);
// One-pass per-row compaction (a chunk whose rows all fit a block): cmp_cols_rows = k_cmp_cols'
// analysis a wave per row, with the per-row heap count, datapoints and byte bounds (p.row_heap /
// row_one / row_n / row_qb / row_vb), no column offsets; cmp_onepass_cap = the LDS capacity (0: a
// row does not fit);
// cmp_rows_onepass = k_cmp_rowone: sort, deduplicate and write every row at p.row_dq / row_dv
// (laid out by the host from the bounds) in one kernel.
hipError_t cmp_cols_rows(const CmpParams& p, hipStream_t s);
int cmp_onepass_cap(const CmpParams& p, uint32_t* scratch3, hipStream_t s, hipError_t* err);
hipError_t cmp_rows_onepass(const CmpParams& p, int cap, hipStream_t s);
// dst = src - base over n offsets (a chunk of the scan, rebased); *bad |= 1 unless non-decreasing and >= base
hipError_t cmp_rebase(const uint64_t* src, uint64_t* dst, int64_t n, uint64_t base, int32_t* bad, hipStream_t s,
                      uint32_t* dst32 = nullptr);   // dst32: also a 32-bit copy (the one-pass path)

// rollup read path: value series buckets <- Σsum / Σcount (avg) or Σcount, from the SUM
// downsampling of each value series and of its count series (cmap[s], -1: none)
hipError_t launch_rollup_combine(double* dense, const uint8_t* pres, const int64_t* cmap, int64_t n_series, int64_t K,
                                 int avg, hipStream_t s);
hipError_t launch_first_ts(const RowDesc* rows, const int64_t* srp, const uint8_t* qual, int64_t n, int64_t ss,
                           int64_t se, int64_t t0, int64_t* out, hipStream_t s);
// n 8-byte words of `v` from p (16-byte aligned): 16-byte non-temporal stores
hipError_t launch_fill64(uint64_t* p, uint64_t v, int64_t n, hipStream_t s);
// the rows [series][K] of `p` whose wr flag is 0 filled with `v` (after a sel_direct pass)
hipError_t launch_fill_rows(uint64_t* p, const uint8_t* wr, int64_t n_series, int64_t K, uint64_t v, hipStream_t s,
                            const int64_t* gsp = nullptr, int64_t G = 0);   // gsp: the column layout
// streaming variant for one uniform row class (k_fast's premises + the sum certificate);
// series that break a premise go to p.redo_list for launch_rollup_agg (tile_list mode)
bool rollup_fast_supported(int qw, int vl);
int64_t rollup_fast_lds(int64_t K);
hipError_t launch_rollup_fast(const GridParams& p, const RollupAggParams& rp, int qw, int vl, hipStream_t s);
hipError_t launch_series_allint(const RowDesc* rows, const int64_t* srp, int64_t n, uint8_t* allint, hipStream_t s);
hipError_t launch_rollup_size(const RollupParams& p, hipStream_t s);
hipError_t launch_rollup_write(const RollupParams& p, hipStream_t s);
hipError_t rollup_scan(const uint32_t* cnt, int64_t* coff, const uint32_t* vsz, uint64_t* voff, int64_t n,
                       void** tmp, size_t* tmp_bytes, hipStream_t s);

// launchers (kernels.hip)
// k_index.hip: row classification (once per load).  index_classes: per-row class, class
// counts and class row lists; index_rows: the class kernels (+ the int16 copy of 1-2-byte
// integer values when val2 is non-null) and the sequential path for the rest (generic: every
// row sequentially -- test hook).
struct IndexBufs {
  uint8_t* hint;     // [n_rows] row class
  int32_t* list;     // [n_rows] rows by class
  uint32_t* cnt;     // [16] class counts / list cursors
};
struct IndexClasses {
  uint32_t cnt[16];
  uint32_t off[16];
  uint32_t vle_capable;   // rows of the 2-byte-qualifier integer classes (variable, 1-byte, 2-byte values)
  uint32_t listed;        // rows in the class lists (the class kernels')
  uint32_t short_rows;    // rows k_index_short takes (one chunk, 2-byte qualifiers, 4-byte or 1-2-byte values)
  bool short_done;        // index_fused: k_index_short has run (classification included)
};
hipError_t index_fused(const uint8_t* qual, const uint8_t* val, uint8_t* val2, RowDesc* rows, const IndexBufs& b,
                       int64_t n_rows, int32_t* err, IndexClasses* out, hipStream_t s);
hipError_t index_classes(const uint8_t* qual, const RowDesc* rows, const IndexBufs& b, int64_t n_rows,
                         IndexClasses* out, hipStream_t s);
hipError_t index_rows(const uint8_t* qual, const uint8_t* val, uint8_t* val2, RowDesc* rows, const IndexBufs& b,
                      const IndexClasses& k, int64_t n_rows, int32_t* err, bool generic, hipStream_t s);
// rows whose first datapoint is not after the series' earlier rows' datapoints: ROW_UNSORTED
hipError_t index_recede(RowDesc* rows, const int64_t* srp, const uint8_t* qual, int64_t n_series, hipStream_t s);
hipError_t launch_grid(const GridParams& p, int ds_function_class, hipStream_t s);
// k_fast: uniform float rows of one (qualifier width, value length) class; returns
// hipErrorNotSupported when no specialisation exists for (f, qw, vl)
bool fast_supported(int ds_function_class, int qw, int vl);
hipError_t launch_fast(const GridParams& p, int ds_function_class, int qw, int vl, hipStream_t s);
int64_t fast_wave_lds(int64_t K, bool rate, bool part = true);   // part = false: KR 0 with dense_out
hipError_t launch_reduce(const ReduceParams& p, hipStream_t s);
// percentile / median downsampling (k_pct.hip): bucket order statistics, then group-by
static constexpr int PCT_CAP = 4096;   // values per bucket sorted in LDS; larger buckets are radix-selected
// pass 0: every series; 1: the series k_pct_rows handed back (tile_list); 2: the large-bucket
// pass over redo_list (n = waves launched = p.n_launch)
hipError_t launch_pct(const GridParams& p, int pass, int64_t n, hipStream_t s);
bool pct_rows_supported(int qw, int vl);
hipError_t launch_pct_rows(const GridParams& p, int qw, int vl, hipStream_t s);
hipError_t launch_emit(const GridParams& p, hipStream_t s);
// sum / avg downsampling in Java's order, one series per thread, into [series][K] (k_misc.hip)
// sum / avg downsampling in Java's order, one row per thread, when every bucket lies inside one
// hour row; series that break the premise go to redo_list for k_seq_dense (k_misc.hip)
hipError_t launch_seq_rows(const GridParams& p, int f, double* dense, uint8_t* pres, int64_t n_rows, hipStream_t s);
// rollup avg / count: a value row with its lock-step count row, combined in place (k_misc.hip)
hipError_t launch_seq_rows_ro(const GridParams& p, int avg, double* dense, uint8_t* pres, const int64_t* cmap, int64_t n_rows,
                              hipStream_t s);
hipError_t launch_rollup_combine_list(double* dense, const uint8_t* pres, const int64_t* cmap, const int32_t* list,
                                      const int32_t* list_n, int64_t n_max, int64_t K, int avg, hipStream_t s);
hipError_t launch_seq_dense(const GridParams& p, int f, double* dense, uint8_t* pres, int64_t n_series, hipStream_t s,
                            bool uniform = false);   // uniform: every row of one width (k_seq_wave)
hipError_t launch_emit_vals(const GridParams& p, hipStream_t s);
hipError_t launch_sel_seg(const SelParams& p, hipStream_t s, int64_t maxn);
hipError_t launch_ordered(const OrdParams& p, hipStream_t s);
hipError_t launch_rank_merge(const RankMergeParams& p, hipStream_t s);
hipError_t launch_state_fold(const StateFoldParams& p, hipStream_t s);
hipError_t launch_pull(void* dst, const void* src, size_t n, hipStream_t s);   // device pointer of page-locked host src
// per-downsample-function instantiations (k_grid.hip / k_fast.hip, one object per F)
template <int F> hipError_t launch_grid_inst(const GridParams& p, hipStream_t s);
template <int F> hipError_t launch_fast_inst(const GridParams& p, int qw, int vl, hipStream_t s);
int64_t grid_wave_lds(int64_t K, bool rate, bool gslot);
hipError_t launch_synth_sizes(const SynthParams& p, hipStream_t s);
// raw path (k_raw.hip)
hipError_t launch_raw_decode(const RawParams& p, hipStream_t s);
hipError_t launch_raw_rate(const RawParams& p, hipStream_t s);
hipError_t launch_raw_union(const RawParams& p, int64_t s_begin, int64_t s_end, hipStream_t s);  // mark + scan
hipError_t launch_raw_rank(const RawParams& p, int64_t s_begin, int64_t s_end, hipStream_t s);   // rank + union ts
hipError_t launch_raw_cursor(const RawParams& p, int64_t s_begin, int64_t s_end, hipStream_t s);
hipError_t launch_raw_merge(const RawParams& p, hipStream_t s);      // unsorted cells: steps, ranks, U
hipError_t launch_raw_merge_ts(const RawParams& p, hipStream_t s);   // step timestamps -> out_ts
hipError_t launch_raw_dz_check(const RawParams& p, int64_t n_out, hipStream_t s);
hipError_t launch_raw_eval(const RawParams& p, hipStream_t s);
hipError_t launch_raw_vals(const RawParams& p, int64_t k_max, hipStream_t s);
hipError_t launch_raw_sel(const RawParams& p, int64_t k_max, hipStream_t s);
hipError_t launch_raw_top(const RawParams& p, int T, hipStream_t s);   // fused operands + selection (k_raw_eval.hip)
hipError_t launch_ro_pack(const RowDesc* rows, const int32_t* partner, const int32_t* vrows, const int32_t* vser,
                          const uint8_t* qual, int64_t n, RoPair* out, hipStream_t s);
hipError_t launch_ro_pairs(const GridParams& p, int avg, double* dense, uint8_t* pres, const int64_t* cmap, int64_t n,
                           hipStream_t s);
hipError_t launch_ro_rows(const GridParams& p, int f, double* dense, uint8_t* pres, int64_t n, hipStream_t s);
template <int GA> hipError_t launch_raw_eval_inst(const RawParams& p, hipStream_t s);   // k_raw_eval.hip
hipError_t launch_synth_write(const SynthParams& p, hipStream_t s);

}  // namespace tsdb
