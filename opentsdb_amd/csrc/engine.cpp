// engine.cpp -- host side of libtsdbhip: the C ABI (include/tsdbhip.h), the query
// planning the reference does on the host (scan bounds, downsample spec parsing,
// SpanGroup membership), HBM layout of the loaded Spans, and result assembly.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/tsdbhip.h"
#include "engine.h"
#include "multi.h"
#include "ksel.h"

using namespace tsdb;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define HIP_OK(expr)                                                                   \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      return fail(TSDB_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));      \
  } while (0)

const char* const AGG_NAMES[TSDB_AGG_COUNT_ALL] = {
    "sum", "pfsum", "min", "max", "avg", "median", "none", "mult", "dev", "diff",
    "zimsum", "mimmin", "mimmax", "squareSum", "count", "first", "last",
    "p999", "p99", "p95", "p90", "p75", "p50",
    "ep999r3", "ep99r3", "ep95r3", "ep90r3", "ep75r3", "ep50r3",
    "ep999r7", "ep99r7", "ep95r7", "ep90r7", "ep75r7", "ep50r7"};

int interp_of(int a) {  // Aggregators.java:47-173
  switch (a) {
    case TSDB_AGG_PFSUM: return TSDB_INTERP_PREV;
    case TSDB_AGG_NONE: case TSDB_AGG_ZIMSUM: case TSDB_AGG_SQUARESUM: case TSDB_AGG_COUNT:
    case TSDB_AGG_FIRST: case TSDB_AGG_LAST: return TSDB_INTERP_ZIM;
    case TSDB_AGG_MIMMIN: return TSDB_INTERP_MAX;
    case TSDB_AGG_MIMMAX: return TSDB_INTERP_MIN;
    default: return TSDB_INTERP_LERP;
  }
}

// group-aggregator class, -1 if not decomposable (median / percentiles)
int ga_of(int a) {
  switch (a) {
    case TSDB_AGG_SUM: case TSDB_AGG_PFSUM: case TSDB_AGG_ZIMSUM: return GA_SUM;
    case TSDB_AGG_AVG: return GA_AVG;
    case TSDB_AGG_COUNT: return GA_COUNT;
    case TSDB_AGG_SQUARESUM: return GA_SQUARESUM;
    case TSDB_AGG_MIN: case TSDB_AGG_MIMMIN: return GA_MIN;
    case TSDB_AGG_MAX: case TSDB_AGG_MIMMAX: return GA_MAX;
    case TSDB_AGG_DEV: return GA_DEV;
    case TSDB_AGG_FIRST: return GA_FIRST;
    case TSDB_AGG_LAST: return GA_LAST;
    case TSDB_AGG_DIFF: return GA_DIFF;
    case TSDB_AGG_MULT: return GA_MULT;
    case TSDB_AGG_NONE: return GA_NONE;
    default: return -1;
  }
}

int f_of(int a) {
  switch (a) {
    case TSDB_AGG_SUM: case TSDB_AGG_PFSUM: case TSDB_AGG_ZIMSUM: return F_SUM;
    case TSDB_AGG_AVG: return F_AVG;
    case TSDB_AGG_COUNT: return F_COUNT;
    case TSDB_AGG_SQUARESUM: return F_SQUARESUM;
    case TSDB_AGG_MIN: case TSDB_AGG_MIMMIN: return F_MIN;
    case TSDB_AGG_MAX: case TSDB_AGG_MIMMAX: return F_MAX;
    case TSDB_AGG_DEV: return F_DEV;
    case TSDB_AGG_FIRST: return F_FIRST;
    case TSDB_AGG_LAST: return F_LAST;
    case TSDB_AGG_DIFF: return F_DIFF;
    case TSDB_AGG_MULT: return F_MULT;
    default: return -1;
  }
}

inline int64_t align16(int64_t x) { return (x + 15) & ~(int64_t)15; }

// ---- calendar intervals (UTC) -----------------------------------------------------------
constexpr int64_t CAL_UNIT_MS[9] = {0, 1, 1000, 60000, 3600000, 86400000, 604800000, 2592000000LL, 31536000000LL};

int cal_unit_of(const std::string& d) {   // suffix of a parseDuration string (parse already checked it)
  if (d.size() >= 2 && (d.compare(d.size() - 2, 2, "ms") == 0)) return TSDB_CAL_MS;
  switch (d.empty() ? 0 : d.back()) {
    case 's': return TSDB_CAL_S;
    case 'm': return TSDB_CAL_M;
    case 'h': return TSDB_CAL_H;
    case 'd': return TSDB_CAL_D;
    case 'w': return TSDB_CAL_W;
    case 'n': return TSDB_CAL_N;
    case 'y': return TSDB_CAL_Y;
  }
  return TSDB_CAL_NONE;
}

inline int64_t floor_div(int64_t a, int64_t b) { int64_t q = a / b; if ((a % b) && ((a < 0) != (b < 0))) q--; return q; }

// A calendar interval whose DateTime.previousInterval grid (src/utils/DateTime.java:445-606)
// is one global sequence in UTC: width W ms, boundaries at O + j W.  ms / s / m / h intervals
// that divide the next unit start at the top of the second / minute / hour / day, which are
// multiples of W since the epoch; "1dc" steps days from midnight; "1wc" steps 7 days from
// Sunday (default US locale; 1970-01-04 was a Sunday, O = 3 days).  0 = not such an interval.
bool cal_grid(int unit, int64_t interval_ms, int64_t* W, int64_t* O) {
  if (unit < TSDB_CAL_MS || unit > TSDB_CAL_Y) return false;
  const int64_t n = interval_ms / CAL_UNIT_MS[unit];
  if (n < 1 || n * CAL_UNIT_MS[unit] != interval_ms) return false;
  bool ok = false;
  switch (unit) {
    case TSDB_CAL_MS: ok = 1000 % n == 0; break;
    case TSDB_CAL_S: case TSDB_CAL_M: ok = 60 % n == 0; break;
    case TSDB_CAL_H: ok = 24 % n == 0; break;
    case TSDB_CAL_D: case TSDB_CAL_W: ok = n == 1; break;
    default: ok = false;   // months / years: variable widths
  }
  if (!ok) return false;
  *W = interval_ms;
  *O = unit == TSDB_CAL_W ? 3 * 86400000LL : 0;
  return true;
}

// Month-based calendar intervals (UTC): n months (12 % n == 0) or 1 year, anchored at the
// top of the year (DateTime.previousInterval :580-588), so every span sees the same grid.
// Month index m = 12 * year + (month - 1) <-> first instant of that month (ms).
int64_t month_start_ms(int64_t m) {
  int64_t y = floor_div(m, 12);
  const int mo = (int)(m - y * 12) + 1;
  y -= mo <= 2;   // days_from_civil
  const int64_t era = floor_div(y, 400);
  const int64_t yoe = y - era * 400;
  const int64_t doy = (153 * (mo + (mo > 2 ? -3 : 9)) + 2) / 5;
  const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return (era * 146097 + doe - 719468) * 86400000LL;
}
int64_t month_of_ms(int64_t t) {   // month index containing t
  int64_t m = floor_div(floor_div(t, 86400000LL) * 4800, 146097) + 1970 * 12;   // estimate (days / 30.44)
  while (month_start_ms(m) > t) m--;
  while (month_start_ms(m + 1) <= t) m++;
  return m;
}
bool cal_months(int unit, int64_t interval_ms, int64_t* step_months) {
  if (unit == TSDB_CAL_N) {
    const int64_t n = interval_ms / CAL_UNIT_MS[TSDB_CAL_N];
    if (n < 1 || n * CAL_UNIT_MS[TSDB_CAL_N] != interval_ms || 12 % n) return false;
    *step_months = n;
    return true;
  }
  if (unit == TSDB_CAL_Y) {
    if (interval_ms != CAL_UNIT_MS[TSDB_CAL_Y]) return false;
    *step_months = 12;
    return true;
  }
  return false;
}

// ---- calendar intervals in a time zone (java.util.GregorianCalendar) ----------------------
// The host-side Calendar the general calendar plan runs (plan_query): DateTime.previousInterval
// (src/utils/DateTime.java:445-606) and Calendar.add in the zone of the query's tsdbhip_tz
// (UTC when none) -- ZoneInfo.getOffsets by instant, getOffsetsByWall when an instant is
// recomputed from local fields, GregorianCalendar.add's per-unit rules.
struct JZone {
  const tsdbhip_tz* z = nullptr;
  int32_t at(int64_t t) const {   // offset in effect at instant t
    if (!z || z->n <= 0) return z ? z->offset_ms[0] : 0;
    const int64_t* u = z->utc_ms;
    const int64_t i = std::upper_bound(u, u + z->n, t) - u;   // transitions at or before t
    return z->offset_ms[i];
  }
  int32_t by_wall(int64_t w) const {   // getTransitionIndex(WALL_TIME): gap -> old offset, overlap -> new
    if (!z || z->n <= 0) return z ? z->offset_ms[0] : 0;
    int lo = 0, hi = z->n - 1;
    while (lo <= hi) {
      const int mid = (lo + hi) >> 1;
      const int64_t mv = z->utc_ms[mid] + z->offset_ms[mid + 1];
      if (mv < w) lo = mid + 1;
      else if (mv > w) hi = mid - 1;
      else return z->offset_ms[mid + 1];
    }
    if (lo >= z->n) return z->offset_ms[z->n];
    return lo == 0 ? z->offset_ms[0] : z->offset_ms[lo];
  }
  int64_t from_wall(int64_t w) const { return w - by_wall(w); }
};

void civil_of_day(int64_t z, int64_t& y, int& m, int& d) {
  z += 719468;
  const int64_t era = floor_div(z, 146097);
  const int64_t doe = z - era * 146097;
  const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const int64_t mp = (5 * doy + 2) / 153;
  d = (int)(doy - (153 * mp + 2) / 5 + 1);
  m = (int)(mp < 10 ? mp + 3 : mp - 9);
  y = yoe + era * 400 + (m <= 2);
}
int64_t day_of_civil(int64_t y, int m, int d) { return floor_div(month_start_ms(y * 12 + m - 1), 86400000LL) + d - 1; }
int month_len(int64_t y, int m) {
  static const int md[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  const bool leap = (y % 4 == 0 && y % 100 != 0) || y % 400 == 0;
  return m == 2 ? 28 + (leap ? 1 : 0) : md[m - 1];
}

// Calendar.add(unit, n): ms / s / m / h absolute; days keep the local time of day and correct
// an offset change (keeping the date); months / years move the local date, pin the day of
// month and recompute the instant from the wall clock
int64_t jcal_add(const JZone& Z, int64_t t, int unit, int64_t n) {
  if (unit != TSDB_CAL_D && unit != TSDB_CAL_N && unit != TSDB_CAL_Y) return t + n * CAL_UNIT_MS[unit];
  const int64_t off = Z.at(t);
  const int64_t loc = t + off;
  int64_t fd = floor_div(loc, 86400000LL);
  const int64_t tod = loc - fd * 86400000LL;
  if (unit == TSDB_CAL_D) {
    fd += n;
    const int64_t t1 = fd * 86400000LL + tod - off;
    const int64_t diff = off - Z.at(t1);
    if (diff == 0) return t1;
    const int64_t t2 = t1 + diff;
    return floor_div(t2 + Z.at(t2), 86400000LL) != fd ? t1 : t2;
  }
  int64_t y;
  int m, d;
  civil_of_day(fd, y, m, d);
  int64_t mm = y * 12 + (m - 1) + (unit == TSDB_CAL_N ? n : 12 * n);
  y = floor_div(mm, 12);
  m = (int)(mm - y * 12) + 1;
  d = std::min(d, month_len(y, m));
  return Z.from_wall(day_of_civil(y, m, d) * 86400000LL + tod);
}
// one Downsampler step (weeks: interval * 7 days)
int64_t jcal_step(const JZone& Z, int64_t t, int unit, int64_t n, int sign) {
  if (unit == TSDB_CAL_W) return jcal_add(Z, t, TSDB_CAL_D, sign * n * 7);
  return jcal_add(Z, t, unit, sign * n);
}
// DateTime.previousInterval(ts, n, unit, tz) in two steps: jcal_top, the instant the set()
// calls produce (the top of the enclosing unit, shifted back for intervals longer than it) and
// the unit / count the walk steps by; then the walk from there to the last step <= ts.
bool jcal_top(const JZone& Z, int64_t ts, int64_t n, int unit, int64_t& c, int& uo, int64_t& io) {
  uo = unit;
  io = n;
  const int64_t loc = ts + Z.at(ts);
  const int64_t day = floor_div(loc, 86400000LL);
  const int64_t tod = loc - day * 86400000LL;
  int64_t y;
  int m, d;
  civil_of_day(day, y, m, d);
  switch (unit) {
    case TSDB_CAL_MS:
      if (1000 % n == 0) { c = Z.from_wall(loc - tod % 1000); if (n > 1000) c -= n; }
      else c = Z.from_wall(loc - tod % 60000);
      break;
    case TSDB_CAL_S:
      if (60 % n == 0) { c = Z.from_wall(loc - tod % 60000); if (n > 60) c -= n * 1000; }
      else c = Z.from_wall(loc - tod % 3600000);
      break;
    case TSDB_CAL_M:
      if (60 % n == 0) { c = Z.from_wall(loc - tod % 3600000); if (n > 60) c -= n * 60000; }
      else c = Z.from_wall(day * 86400000LL);
      break;
    case TSDB_CAL_H:
      if (24 % n == 0) { c = Z.from_wall(day * 86400000LL); if (n > 24) c -= n * 3600000LL; }
      else c = Z.from_wall(day_of_civil(y, m, 1) * 86400000LL);
      break;
    case TSDB_CAL_D:
      c = Z.from_wall(day_of_civil(y, n == 1 ? m : 1, 1) * 86400000LL);
      break;
    case TSDB_CAL_W: {
      // Sunday-first weeks, one minimal day in the first week (the default US locale;
      // 1970-01-04 was a Sunday)
      auto sunday_on_or_before = [](int64_t dd) { return dd - ((dd - 3) % 7 + 7) % 7; };
      if (2 % n == 0) {
        c = Z.from_wall(sunday_on_or_before(day) * 86400000LL);   // set(DAY_OF_WEEK, SUNDAY)
      } else {
        // set(MONTH, 0) then set(DAY_OF_WEEK, SUNDAY): GregorianCalendar resolves YEAR + MONTH +
        // WEEK_OF_MONTH (still ts's week of ITS month) + DAY_OF_WEEK, i.e. that week of January
        const int64_t wom = (day - sunday_on_or_before(day_of_civil(y, m, 1))) / 7 + 1;
        c = Z.from_wall((sunday_on_or_before(day_of_civil(y, 1, 1)) + 7 * (wom - 1)) * 86400000LL);
      }
      uo = TSDB_CAL_D;   // the walk steps 7 days whatever the interval
      io = 7;
      break;
    }
    default:   // months, years: from the top of the year
      c = Z.from_wall(day_of_civil(y, 1, 1) * 86400000LL);
      break;
  }
  return true;
}
bool jcal_prev(const JZone& Z, int64_t ts, int64_t n, int unit, int64_t& out) {
  int64_t c, io;
  int uo;
  if (!jcal_top(Z, ts, n, unit, c, uo, io)) return false;
  if (c != ts) {
    while (c <= ts) c = jcal_add(Z, c, uo, io);
    c = jcal_add(Z, c, uo, -io);
  }
  out = c;
  return true;
}

// bytes past the end of the qualifier / value blobs that kernels may read (never use):
// k_fast's vle class loads a 1 KB value window from each row start
constexpr int64_t BLOB_SLACK = 1024 + 64;

struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= n && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
    if (e == hipSuccess) n = bytes;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

// page-locked host staging (device -> host copies of dense results), grown on demand
struct HostBuf {
  void* p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= n && p) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipHostMalloc(&p, bytes ? bytes : 16, hipHostMallocDefault);
    if (e == hipSuccess) n = bytes;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
  }
};


}  // namespace

// One RollupSeq of a rollup batch (RollupSpan.addRow merges the cells of one row key):
// what the query-time scan needs of it.
struct RoSeqRow {
  int64_t base = 0;
  int64_t order = 0;            // scan order inside the series
  int32_t err = 0;              // RollupSeq.append's exception for these cells (thrown when scanned)
  std::string msg;
  bool verr = false;            // a value the extract functions reject (thrown when read)
  bool cerr = false;            // a count the extract functions reject (thrown by valueCount())
  int64_t npts = 0;             // datapoints the RollupIterator yields
  int64_t last_ts = 0;          // its last timestamp (ms)
  int64_t pp_ts = INT64_MAX;    // first value cell after which value / count cells stop pairing one
                                // to one (RollupIterator.seek walks them in lock step)
};

struct tsdbhip_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;   // result downloads overlapped with evaluation
  hipEvent_t ev[4] = {};
  hipEvent_t cev[9] = {};              // chunk-done events for copy_stream (+ timestamps final)
  std::mutex mu;
  // resident batch (series in group-sorted order)
  int64_t n_series = 0, n_rows = 0, n_groups = 0;
  int64_t max_series_rows = INT64_MAX; // most rows of one series in the resident batch (k_recede when > 1)
  uint64_t qual_bytes = 0, val_bytes = 0;
  DevBuf rows, srp, qual, val, gid;
  DevBuf val2;                         // int16 copy of vle-integer values (k_index), at qualifier offsets
  DevBuf hint, ilist, icnt;            // k_index scratch: row classes, rows by class, class counts
  std::vector<int64_t> h_srp;          // [n_series+1]
  std::vector<uint32_t> h_base;        // [n_rows]
  std::vector<uint32_t> h_ndp;         // [n_rows]
  std::vector<uint32_t> h_qlen, h_vlen;
  std::vector<uint32_t> h_flags;       // [n_rows] RowDesc.flags after k_index
  std::vector<int32_t> h_group;        // [n_series] group of sorted position
  std::vector<int64_t> h_orig;         // [n_series] original batch index of sorted position
  // tiles over groups
  std::vector<int64_t> tb, te, gtp;
  std::vector<int32_t> tg;
  DevBuf d_tb, d_te, d_tg, d_gtp;
  // tiles for the NONE aggregator (one series each)
  bool none_tiles_ready = false;
  DevBuf n_tb, n_te, n_tg, n_gtp;
  // scratch
  DevBuf pa, pb, pn, pf, out_val, out_flag, gact, err, g_dense, g_pres, g_rate, redo, redo_n, redo2, redo2_n;
  DevBuf xbuf, gbuf;
  DevBuf m_sum, m_mn, m_mx, m_mean, m_m2, m_nl, m_nz, m_f;   // fused multi-aggregator partials
  DevBuf pre_dense, pre_pres;         // percentile / median downsampling
  DevBuf row_ser, sr_list, sr_n, sr_mark;   // k_seq_rows: series of each row, handed-back series
  bool row_ser_valid = false;
  int64_t n_grouped = -1;              // series before the first ungrouped one, when every later one
                                       // is ungrouped (else n_series); -1 = not computed
  DevBuf big_scratch;                  // k_pct large buckets: per-wave overflow regions
  bool mdp_valid = false;              // series_max_dp() cache (invalidated by every load)
  bool ro_meta_valid = false;          // rollup ro_ord / ro_orig / ro_allint of the loaded batch
  bool lc_valid = false;               // local_counts() cache
  std::vector<int64_t> lc;
  // general calendar plan cache (plan_calendar): key, then its boundaries / seek point
  bool calc_valid = false;
  std::vector<int64_t> calc_key, calc_bounds;
  int64_t calc_seek = 0;
  bool calc_anchored = false;            // ... the spans' grids disagree: per-anchor sequences
  std::vector<int64_t> calc_anchors;
  std::vector<std::vector<int64_t>> calc_seqs;
  std::vector<int64_t> calc_fill;      // FillingDownsampler's calendar sequence of an anchored plan
  DevBuf first_ts;
  int64_t mdp_ss = 0, mdp_se = 0, mdp = 0;
  DevBuf sel_vals, sel_sorted, sel_uni, sel_gsp;   // percentile / median group-by
  DevBuf sel_wr;                                    // sel_direct: rows of sel_vals written
  // the sampled-window select (sel_window): window bounds [G][K], per (tile, slot) counts and
  // values, the fail flag, the sampled tiles (by group, and as class lists for run_device)
  DevBuf win_lo, win_hi, win_val, win_gcnt, win_cur, win_cand, win_fail, samp_tiles, samp_ptr, samp_tl, samp_tl_n;
  int64_t win_runs = 0, win_misses = 0;        // sel_window runs, and those that fell back to the full path (tests)
  const int32_t* tl_dev_override = nullptr;    // run_device: these class lists instead of d_tl / d_tl_n
  const int32_t* tln_dev_override = nullptr;
  DevBuf cal_bounds;                                // calendar month / year slot boundaries
  // raw path scratch
  DevBuf r_rowpt, r_spoff, r_spn, r_grp, r_pts, r_rank, r_bm, r_wb, r_U, r_ooff, r_sg, r_su, r_ots, r_obits, r_oint,
      r_coff, r_cur, r_voff, r_vl, r_vd, r_vp, r_bnd, r_mts, r_mpos, r_mhead, r_dz;                   // multi-GPU: this rank's partial states, gathered states
  // dominant uniform row class of the batch (k_fast specialisation), 0 = none
  int fast_qw = 0, fast_vl = 0;        // dominant k_fast row class (0 = none)
  int fast_qw2 = 0, fast_vl2 = 0;      // second class, chained over the first one's redo list
  int pct_qw = 0, pct_vl = 0;          // dominant uniform class of one-chunk rows (k_pct_rows)
  bool pct_vonly = false;              // every row of that class (4-byte values) all-float without NaN
                                       // or all-integer: the key kernel reads values only
  bool pct_v6 = false;                 // ... and none over 384 values (6 values a lane)
  // tile lists by k_fast row class (built at load): [class A / class B][walker / short /
  // rows], and the tiles of neither class (general kernel only).  Short = one row per series
  // of at most CH datapoints (k_short); rows = several rows per series, none over CH (k_rows).
  std::vector<int32_t> tl[2][3], tl_other;
  DevBuf d_tl, d_tl_n, r1a, r1b, r3a, r3b, r2, r_n;   // device copies; k_short / k_rows / k_fast redo lists
  DevBuf hw_mark;                                      // k_hwin: a tile is on the redo list (one word a tile)
  int64_t tl_off[7] = {};
  bool fast_used = false;
  HostBuf h_stage;   // collect(): the dense [G][K] values and flags, page-locked
  HostBuf h_small;   // collect(): the group activity flags, error code and hand-back count, page-locked
  HostBuf h_scal;    // d2h_small: 16 page-locked 8-byte slots for scalars read back
  void* small_dst[16] = {};
  int small_len[16] = {};
  int small_n = 0;
  void* up_stage[2] = {nullptr, nullptr};   // h2d: page-locked staging of pageable uploads (UP_CHUNK each)
  hipEvent_t up_ev[2] = {nullptr, nullptr};
  bool up_busy[2] = {false, false};
  const int32_t* redo_final = nullptr;   // device counter of the tiles k_fast handed to k_grid
  int64_t redo_other = 0;                // + tiles of neither row class (k_grid only)
  tsdbhip_timing timing{};
  double index_ms = 0;                   // k_index (+ val2 pass) of the last load
  double compact_ms = 0;                 // k_compact pipeline of the last tsdbhip_load_cells
  int64_t fused_n = 0;                   // queries of the fused multi-aggregator pass being collected
  // account() cache (invalidated by every load)
  bool acct_valid = false;
  bool seqd_valid = false;             // cached seq_dense_wanted answer for (seqd_ss, seqd_se)
  bool seqd_uniform = false;          // every row of the cached scan range has one qualifier width and value length
  bool seqd_ok = false, seqd_nocert = false, seqd_tiny = false;
  int64_t seqd_ss = 0, seqd_se = 0;
  int64_t acct_ss = 0, acct_se = 0, acct_dps = 0, acct_bytes = 0;
  bool acct_none = false;
  // rollup generation: scratch and the per-function cells of the last tsdbhip_rollup_run
  DevBuf ro_allint, ro_ord, ro_orig, ro_cnt, ro_vsz, ro_coff, ro_voff;
  DevBuf ro_agg, ro_pres;              // fused rollup pass: [4][series][K] values, [series][K] presence
  void* ro_tmp = nullptr;
  size_t ro_tmp_bytes = 0;
  struct RollupOut {
    DevBuf series, base, qual, voff, val;
    int64_t cells = 0;
    uint64_t bytes = 0;
  } ro_out[4];
  int ro_n = 0;
  // rollup read path (tsdbhip_load_rollup): the resident batch holds the value series (batch
  // positions [0, ro_nval), their groups) and, with count cells, one count series per value
  // series (positions ro_nval + s, no group), both re-rowed into hour rows
  bool ro_active = false, ro_counts = false;
  tsdbhip_rollup_interval ro_iv{};
  int64_t ro_nval = 0;
  std::vector<int64_t> ro_rp;          // [ro_nval + 1] -> ro_rows
  std::vector<RoSeqRow> ro_rows;
  std::vector<std::string> ro_unsup;   // per value series: why the engine does not run it ("" = runs)
  std::vector<int64_t> ro_res;         // batch position -> resident index
  DevBuf ro_cmap;                      // [n_series] resident index of a value series' count series (-1: none)
  DevBuf ro_partner;                   // [n_rows] a value row's lock-step count row (GridParams.ro_partner)
  DevBuf ro_pairs;                     // [ro_npairs] the packed value / count row pairs (k_ro_pairs)
  int64_t ro_npairs = 0;
  DevBuf ro_runs, ro_rid;              // ... or as runs: [ro_nruns] RoRun, [ro_npairs] run of each pair
  int64_t ro_nruns = 0;
  // query-time compaction (tsdbhip_load_cells): rows whose compaction failed, raised when a
  // query's scan range covers them (SaltScanner.processRow fails the scan)
  struct CmpErr { int64_t series, row; int64_t base; int32_t code; };
  std::vector<CmpErr> cmp_errs;
  void* cmp_tmp = nullptr;
  size_t cmp_tmp_bytes = 0;
  bool ro_scan_valid = false;          // scan-active value series of the last scan range
  // the last scan range whose rollup rows passed ro_scan's checks (a host walk over every row:
  // 4 ms a query for a 1M-series table; the store is immutable until the next load)
  bool ro_chk_valid = false, ro_chk_counts = false;
  int64_t ro_chk_ss = 0, ro_chk_se = 0, ro_chk_T = 0;
  int64_t ro_scan_ss = 0, ro_scan_se = 0;
  std::vector<uint8_t> ro_scan_act;    // [n_series] resident: rollup rows in the scan range
  std::vector<int32_t> ro_scan_gact;   // the groups holding such a series (with ro_scan_act)
  // histogram path (hist.cpp): the resident histogram store and its query scratch
  void* hist = nullptr;
  // multi-device context (multi.cpp, tsdbhip_init_devices): its devices' contexts; null on a
  // one-device context
  void* md = nullptr;
  bool none_orig = false;              // NONE result groups keyed by batch position (multi.cpp merges them)
};

// accessors for the histogram path's translation unit (hist.cpp)
namespace tsdb {
hipStream_t ctx_stream(tsdbhip_ctx* c) { return c->stream; }
int ctx_device(tsdbhip_ctx* c) { return c->device; }
std::mutex& ctx_mutex(tsdbhip_ctx* c) { return c->mu; }

// Scalars read back from the device go through page-locked slots of the context: a copy into
// pageable memory blocks in the runtime until the stream drains, and measured ~0.85 ms a call
// however little was left to run (profiles/r05ad/ro_api: rollup avg:1h-avg, 0.27 ms of kernels in
// a 0.99 ms call).  d2h_small queues the copy into a slot; sync_small synchronises the stream and
// hands the slots' values to their destinations.
int d2h_small(tsdbhip_ctx* c, void* dst, const void* src, size_t bytes, hipStream_t st) {
  if (bytes > 8 || c->small_n >= (int)(sizeof(c->small_dst) / sizeof(c->small_dst[0]))) {
    HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st));
    return 0;
  }
  HIP_OK(c->h_scal.ensure(8 * 16));
  char* slot = reinterpret_cast<char*>(c->h_scal.p) + 8 * c->small_n;
  HIP_OK(hipMemcpyAsync(slot, src, bytes, hipMemcpyDeviceToHost, st));
  c->small_dst[c->small_n] = dst;
  c->small_len[c->small_n] = (int)bytes;
  c->small_n++;
  return 0;
}
int sync_small(tsdbhip_ctx* c, hipStream_t st) {
  const hipError_t e = hipStreamSynchronize(st);
  for (int i = 0; i < c->small_n; i++)
    std::memcpy(c->small_dst[i], reinterpret_cast<char*>(c->h_scal.p) + 8 * i, (size_t)c->small_len[i]);
  c->small_n = 0;
  if (e != hipSuccess) return fail(TSDB_E_HIP, std::string("hipStreamSynchronize: ") + hipGetErrorString(e));
  return 0;
}

// The context's lock for an entry point; also drops d2h_small copies an earlier call left
// pending when it returned on an error between the copy and its sync_small.
struct CtxLock {
  std::lock_guard<std::mutex> g;
  explicit CtxLock(tsdbhip_ctx* c) : g(c->mu) { c->small_n = 0; }
};
void*& ctx_hist(tsdbhip_ctx* c) { return c->hist; }
int set_error(int code, const std::string& msg) { return fail(code, msg); }
void hist_release(void* h);
void*& ctx_md(tsdbhip_ctx* c) { return c->md; }
bool ctx_is_md(tsdbhip_ctx* c) { return c && c->md; }
void ctx_set_none_orig(tsdbhip_ctx* c, bool on) { c->none_orig = on; }
// DateTime.previousInterval and one Downsampler calendar step in a zone (null: UTC), for hist.cpp
bool cal_prev_tz(const tsdbhip_tz* z, int64_t ts, int64_t n, int unit, int64_t* out) {
  JZone Z;
  Z.z = z;
  return jcal_prev(Z, ts, n, unit, *out);
}
int64_t cal_step_tz(const tsdbhip_tz* z, int64_t t, int unit, int64_t n) {
  JZone Z;
  Z.z = z;
  return jcal_step(Z, t, unit, n, 1);
}
int64_t cal_unit_ms(int unit) { return unit >= 0 && unit < 9 ? CAL_UNIT_MS[unit] : 0; }
}  // namespace tsdb

// Entry points bound to one device's resident store refuse a multi-device context.
#define MD_REFUSE(c, fn)                                                                                   \
  if ((c) && (c)->md)                                                                                      \
  return fail(TSDB_E_NOT_IMPLEMENTED, fn " on a multi-device context (tsdbhip_init_devices): it is bound to " \
                                         "one device's resident store")

// ===========================================================================
// host logic restatements
// ===========================================================================
extern "C" int tsdbhip_abi_version(void) { return TSDBHIP_ABI_VERSION; }

// ---- developer options (opts.h): set through the C ABI only, never from the environment ----
namespace tsdb {
namespace {
// stored as value + 1 so that the zero-initialised table means "every option unset"
std::atomic<int64_t> g_opts[OPT_COUNT];
const char* const kOptNames[OPT_COUNT] = {
    "FAST", "SHORT", "ROWS", "HWIN", "SEQ", "SEQ_ROWS", "SEQ_WAVE", "INDEX_GENERIC", "CMP_CHUNK", "CMP_ROWS",
    "CMP_ONEPASS", "PCT_ROWS", "PCT_KEYS", "PCT_VONLY", "PCT_V6", "SEL_FUSED", "SEL_COLS", "SEL_WIN", "SEL_WAVE",
    "SEL_REG", "SELOPS", "RAW_LERPW", "RAW_SEL_TOP", "RAW_SEL_REG", "RO_FUSE", "RO_RUNS", "MULTI_FUSE", "EMIT_HALF", "HIST_WINDOW",
    "HIST_WS", "HIST_LAYOUT", "TRACE", "DBG"};
int opt_index(const char* name) {
  if (!name) return -1;
  for (int i = 0; i < OPT_COUNT; i++)
    if (std::strcmp(name, kOptNames[i]) == 0) return i;
  return -1;
}
}  // namespace
int64_t opt(Opt o) { return g_opts[o].load(std::memory_order_relaxed) - 1; }
}  // namespace tsdb

extern "C" int tsdbhip_set_option(const char* name, int64_t value) {
  const int i = tsdb::opt_index(name);
  if (i < 0) return fail(TSDB_E_ILLEGAL_ARGUMENT, std::string("unknown option: ") + (name ? name : "(null)"));
  if (value < -1) return fail(TSDB_E_ILLEGAL_ARGUMENT, "option values are >= 0 (-1 resets)");
  tsdb::g_opts[i].store(value + 1, std::memory_order_relaxed);
  return 0;
}

extern "C" int tsdbhip_get_option(const char* name, int64_t* value) {
  const int i = tsdb::opt_index(name);
  if (i < 0 || !value) return fail(TSDB_E_ILLEGAL_ARGUMENT, std::string("unknown option: ") + (name ? name : "(null)"));
  *value = tsdb::opt((tsdb::Opt)i);
  return 0;
}

namespace tsdb {
hipError_t h2d(tsdbhip_ctx* c, void* dst, const void* src, size_t n, hipStream_t st);   // (defined at the end)
}  // namespace tsdb

extern "C" int tsdbhip_host_alloc(uint64_t bytes, void** out) {
  if (!out) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  *out = nullptr;
  HIP_OK(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocPortable));
  return 0;
}

extern "C" void tsdbhip_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}
extern "C" const char* tsdbhip_last_error(void) { return g_last_error.c_str(); }

extern "C" int tsdbhip_aggregator_get(const char* name) {
  if (!name) return fail(TSDB_E_NO_SUCH_ELEMENT, "No such aggregator: null");
  for (int i = 0; i < TSDB_AGG_COUNT_ALL; i++)
    if (std::strcmp(AGG_NAMES[i], name) == 0) return i;
  return fail(TSDB_E_NO_SUCH_ELEMENT, std::string("No such aggregator: ") + name);
}

extern "C" int tsdbhip_aggregator_interpolation(int a) {
  if (a < 0 || a >= TSDB_AGG_COUNT_ALL) return fail(TSDB_E_ILLEGAL_ARGUMENT, "bad aggregator");
  return interp_of(a);
}

// DateTime.parseDuration (src/utils/DateTime.java:186-226)
extern "C" int tsdbhip_parse_duration(const char* duration, int64_t* out_ms) {
  if (!duration || !*duration) return fail(TSDB_E_ILLEGAL_ARGUMENT, "Invalid duration");
  const size_t len = std::strlen(duration);
  size_t unit = 0;
  while (std::isdigit((unsigned char)duration[unit])) {
    unit++;
    if (unit >= len) return fail(TSDB_E_ILLEGAL_ARGUMENT, std::string("Invalid duration, must have an integer and unit: ") + duration);
  }
  if (unit == 0 || unit > 18) return fail(TSDB_E_ILLEGAL_ARGUMENT, std::string("Invalid duration (number): ") + duration);
  const int64_t interval = std::stoll(std::string(duration, unit));
  if (interval <= 0) return fail(TSDB_E_ILLEGAL_ARGUMENT, std::string("Zero or negative duration: ") + duration);
  int64_t mult;
  switch (std::tolower((unsigned char)duration[len - 1])) {
    case 's':
      if (len >= 2 && duration[len - 2] == 'm') { *out_ms = interval; return 0; }
      mult = 1; break;
    case 'm': mult = 60; break;
    case 'h': mult = 3600; break;
    case 'd': mult = 86400; break;
    case 'w': mult = 604800; break;
    case 'n': mult = 2592000; break;
    case 'y': mult = 31536000; break;
    default: return fail(TSDB_E_ILLEGAL_ARGUMENT, std::string("Invalid duration (suffix): ") + duration);
  }
  mult *= 1000;
  if ((double)interval * (double)mult > 9223372036854775807.0)
    return fail(TSDB_E_ILLEGAL_ARGUMENT, std::string("Duration must be < Long.MAX_VALUE ms: ") + duration);
  *out_ms = interval * mult;
  return 0;
}

// new DownsamplingSpecification(String) (src/core/DownsamplingSpecification.java:116-191)
extern "C" int tsdbhip_parse_downsample(const char* spec, tsdbhip_query* q) {
  if (!spec) return fail(TSDB_E_ILLEGAL_ARGUMENT, "Downsampling specifier cannot be null");
  std::vector<std::string> parts;
  std::string cur;
  for (const char* c = spec; *c; c++) {
    if (*c == '-') { parts.push_back(cur); cur.clear(); } else cur += *c;
  }
  parts.push_back(cur);
  while (!parts.empty() && parts.back().empty()) parts.pop_back();
  if (parts.size() < 2)
    return fail(TSDB_E_ILLEGAL_ARGUMENT, std::string("Invalid downsampling specifier '") + spec + "': must provide at least interval and function");
  if (parts.size() > 3)
    return fail(TSDB_E_ILLEGAL_ARGUMENT, std::string("Invalid downsampling specifier '") + spec + "': must consist of interval, function, and optional fill policy");
  q->ds_all = 0;
  q->ds_calendar = 0;
  if (parts[0].find("all") != std::string::npos) {
    q->ds_interval_ms = 0;
    q->ds_all = 1;
  } else {
    std::string d = parts[0];
    const bool cal = !d.empty() && d.back() == 'c';
    if (cal) d.pop_back();
    int rc = tsdbhip_parse_duration(d.c_str(), &q->ds_interval_ms);
    if (rc) return rc;
    if (cal) q->ds_calendar = cal_unit_of(d);   // DateTime.unitsToCalendarType (src/utils/DateTime.java:616-640)
  }
  int f = -1;
  for (int i = 0; i < TSDB_AGG_COUNT_ALL; i++) if (parts[1] == AGG_NAMES[i]) f = i;
  if (f < 0) return fail(TSDB_E_ILLEGAL_ARGUMENT, "No such downsampling function: " + parts[1]);
  if (f == TSDB_AGG_NONE) return fail(TSDB_E_ILLEGAL_ARGUMENT, "cannot use the NONE aggregator for downsampling");
  q->ds_function = f;
  q->ds_fill = TSDB_FILL_NONE;
  if (parts.size() == 3) {
    static const char* const fills[5] = {"none", "zero", "nan", "null", "scalar"};
    int found = -1;
    for (int i = 0; i < 5; i++) if (strcasecmp(fills[i], parts[2].c_str()) == 0) found = i;
    if (found < 0) return fail(TSDB_E_ILLEGAL_ARGUMENT, "Unrecognized fill policy: " + parts[2]);
    q->ds_fill = found;
  }
  return 0;
}

// TsdbQuery.getScanStartTimeSeconds / getScanEndTimeSeconds (src/core/TsdbQuery.java:1506-1606)
extern "C" int tsdbhip_scan_bounds(const tsdbhip_query* q, int64_t* s_out, int64_t* e_out) {
  const bool ds = q->ds_function >= 0 && q->ds_interval_ms > 0;
  int64_t start = q->start_time;
  if ((start & (int64_t)0xFFFFFFFF00000000LL) != 0) start /= 1000;
  int64_t aligned = start;
  if (ds) aligned -= ((1000 * start) % q->ds_interval_ms) / 1000;
  const int64_t ta = aligned - (aligned % 3600);
  *s_out = ta > 0 ? ta : 0;
  int64_t end = q->end_time;
  if ((end & (int64_t)0xFFFFFFFF00000000LL) != 0) {
    end /= 1000;
    if (end - (end * 1000) < 1) end++;
  }
  if (ds) {
    const int64_t ia = end + (q->ds_interval_ms - (1000 * end) % q->ds_interval_ms) / 1000;
    const int64_t toff = ia % 3600;
    *e_out = toff == 0 ? ia : ia + (3600 - toff);
  } else {
    *e_out = end + (3600 - end % 3600);
  }
  return 0;
}

// ===========================================================================
// context
// ===========================================================================
extern "C" int tsdbhip_init(int device, tsdbhip_ctx** out) {
  if (!out) return fail(TSDB_E_ILLEGAL_ARGUMENT, "out is null");
  int ndev = 0;
  HIP_OK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(TSDB_E_HIP, "no such HIP device " + std::to_string(device));
  HIP_OK(hipSetDevice(device));
  auto* c = new tsdbhip_ctx();
  c->device = device;
  HIP_OK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  HIP_OK(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
  for (auto& e : c->ev) HIP_OK(hipEventCreate(&e));
  for (auto& e : c->cev) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_OK(c->err.ensure(16));
  *out = c;
  return 0;
}

static void release_batch(tsdbhip_ctx* c) {
  for (DevBuf* b : {&c->rows, &c->srp, &c->qual, &c->val, &c->val2, &c->hint, &c->ilist, &c->icnt, &c->gid, &c->d_tb, &c->d_te, &c->d_tg, &c->d_gtp,
                    &c->n_tb, &c->n_te, &c->n_tg, &c->n_gtp})
    b->release();
  c->none_tiles_ready = false;
  c->acct_valid = false;
  c->seqd_valid = false;
  c->row_ser_valid = false;
  c->n_grouped = -1;
  c->mdp_valid = false;
  c->ro_meta_valid = false;
  c->lc_valid = false;
  c->calc_valid = false;
  c->n_series = c->n_rows = c->n_groups = 0;
  c->max_series_rows = INT64_MAX;   // (unknown until a load sets it: k_recede runs)
  c->ro_active = c->ro_counts = false;
  c->ro_scan_valid = false;
  c->ro_chk_valid = false;
  c->ro_nval = 0;
  c->ro_rp.clear();
  c->ro_rows.clear();
  c->ro_unsup.clear();
  c->ro_res.clear();
  c->ro_cmap.release();
  c->ro_partner.release();
  c->ro_pairs.release();
  c->ro_npairs = 0;
  c->ro_runs.release();
  c->ro_rid.release();
  c->ro_nruns = 0;
  c->cmp_errs.clear();
  c->compact_ms = 0;
}

namespace tsdb {
// multi.cpp: the merge context's resident state reset (a load that is not a rollup load)
void ctx_drop_batch(tsdbhip_ctx* c) {
  CtxLock lk(c);
  release_batch(c);
}
int64_t ctx_n_series(tsdbhip_ctx* c) { return c->n_series; }   // resident series (count series too)
// the last tsdbhip_rollup_run's cells / value bytes per function (its output order)
int ctx_rollup_parts(tsdbhip_ctx* c, int64_t* cells, uint64_t* bytes) {
  for (int i = 0; i < c->ro_n; i++) {
    cells[i] = c->ro_out[i].cells;
    bytes[i] = c->ro_out[i].bytes;
  }
  return c->ro_n;
}
}  // namespace tsdb

extern "C" void tsdbhip_destroy(tsdbhip_ctx* c) {
  if (!c) return;
  if (c->md) { tsdb::md_destroy(c->md); c->md = nullptr; }
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  release_batch(c);
  for (DevBuf* b : {&c->pa, &c->pb, &c->pn, &c->pf, &c->out_val, &c->out_flag, &c->gact, &c->err, &c->g_dense,
                    &c->g_pres, &c->g_rate, &c->redo, &c->redo_n, &c->redo2, &c->redo2_n, &c->d_tl, &c->d_tl_n, &c->r1a, &c->r1b, &c->r3a, &c->r3b, &c->r2, &c->r_n, &c->xbuf, &c->gbuf, &c->r_rowpt,
                    &c->r_spoff, &c->r_spn, &c->r_grp, &c->r_pts, &c->r_rank, &c->r_bm, &c->r_wb, &c->r_U, &c->r_ooff,
                    &c->r_sg, &c->r_su, &c->r_ots, &c->r_obits, &c->r_oint, &c->r_coff, &c->r_cur, &c->r_voff, &c->r_vl, &c->r_vd, &c->r_vp, &c->pre_dense, &c->pre_pres,
                    &c->row_ser, &c->sr_list, &c->sr_n, &c->sr_mark,
                    &c->ro_allint, &c->ro_ord, &c->ro_orig, &c->ro_cnt, &c->ro_vsz, &c->ro_coff, &c->ro_voff,
                    &c->big_scratch, &c->ro_agg, &c->ro_pres})
    b->release();
  c->h_stage.release();
  c->h_small.release();
  c->h_scal.release();
  for (auto& o : c->ro_out)
    for (DevBuf* b : {&o.series, &o.base, &o.qual, &o.voff, &o.val}) b->release();
  if (c->ro_tmp) (void)hipFree(c->ro_tmp);
  if (c->cmp_tmp) (void)hipFree(c->cmp_tmp);
  tsdb::hist_release(c->hist);
  c->hist = nullptr;
  for (DevBuf* b : {&c->sel_vals, &c->sel_sorted, &c->sel_uni, &c->sel_gsp, &c->cal_bounds, &c->sel_wr, &c->first_ts,
                    &c->hw_mark, &c->m_sum, &c->m_mn, &c->m_mx, &c->m_mean, &c->m_m2, &c->m_nl, &c->m_nz, &c->m_f})
    b->release();
  for (int i = 0; i < 2; i++) {
    if (c->up_ev[i]) (void)hipEventDestroy(c->up_ev[i]);
    if (c->up_stage[i]) (void)hipHostFree(c->up_stage[i]);
  }
  for (auto& e : c->ev) if (e) (void)hipEventDestroy(e);
  for (auto& e : c->cev) if (e) (void)hipEventDestroy(e);
  if (c->copy_stream) { (void)hipStreamSynchronize(c->copy_stream); (void)hipStreamDestroy(c->copy_stream); }
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

extern "C" int tsdbhip_sync(tsdbhip_ctx* c) {
  if (!c) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null ctx");
  if (c->md) return tsdb::md_sync(c);
  HIP_OK(hipSetDevice(c->device));
  HIP_OK(hipStreamSynchronize(c->stream));
  return 0;
}

// Tiles: consecutive series of one group, at most T each.
static int build_tiles(tsdbhip_ctx* c) {
  const int64_t n = c->n_series;
  int64_t T = 64;
  // Keep enough waves in flight for small batches (8192 tiles).  TSDBHIP_TILE_MIN raises the tile
  // count for batches of heavy series (more than TSDBHIP_TILE_DP datapoints a tile): measured on
  // config 2 (1M series of 3600 dp), 62.5k tiles of 16 series instead of 15.6k of 64 gave k_fast
  // 3.79 vs 3.82 ms but k_reduce 0.13 vs 0.04 ms over 4x the partials -- a slower step
  // (profiles/r04e), so the default stays at 8192.
  int64_t min_tiles = 8192, tile_dp = 40000;
  int64_t dps = 0;
  for (int64_t r = 0; r < c->n_rows; r++) dps += c->h_ndp[r];
  const double dp_per_series = n ? (double)dps / (double)n : 0.0;
  while (T > 1 && ((n + T - 1) / T < 8192 || ((n + T - 1) / T < min_tiles && (double)T * dp_per_series > (double)tile_dp)))
    T >>= 1;
  c->tb.clear(); c->te.clear(); c->tg.clear();
  c->gtp.assign(c->n_groups + 1, 0);
  int64_t s = 0;
  for (int64_t g = 0; g < c->n_groups; g++) {
    c->gtp[g] = (int64_t)c->tb.size();
    int64_t e = s;
    while (e < n && c->h_group[e] == g) e++;
    for (int64_t a = s; a < e; a += T) {
      c->tb.push_back(a);
      c->te.push_back(std::min(e, a + T));
      c->tg.push_back((int32_t)g);
    }
    s = e;
  }
  c->gtp[c->n_groups] = (int64_t)c->tb.size();
  const size_t nt = c->tb.size();
  // per-tile k_fast class: every row of the tile in class A (or B); the kernels re-check
  for (auto& a : c->tl) for (auto& b : a) b.clear();
  c->tl_other.clear();
  auto row_class = [&](int64_t r, int qw, int vl) {
    const uint32_t f = c->h_flags[r];
    if (!qw) return false;
    if ((f & ROW_QW_MASK) != (uint32_t)qw || (f & (ROW_ERR | ROW_UNSORTED))) return false;
    if (vl == 0) return (f & ROW_ALLI) && (f & ROW_VLE2) && c->h_ndp[r] <= (uint32_t)CH_ROWS;
    return ((f & ROW_VL_MASK) >> ROW_VL_SHIFT) == (uint32_t)vl && (f & ROW_ALLF) && !(f & ROW_NAN);
  };
  for (size_t t = 0; t < nt; t++) {
    const int64_t r0 = c->h_srp[c->tb[t]], r1 = c->h_srp[c->te[t]];
    int cls = -1;
    for (int k = 0; k < 2 && cls < 0; k++) {
      const int qw = k ? c->fast_qw2 : c->fast_qw, vl = k ? c->fast_vl2 : c->fast_vl;
      bool all = r1 > r0;
      for (int64_t r = r0; r < r1 && all; r++) all = row_class(r, qw, vl);
      if (all) cls = k;
    }
    if (cls < 0) { c->tl_other.push_back((int32_t)t); continue; }
    bool chunk = true;   // every row one chunk
    for (int64_t r = r0; r < r1 && chunk; r++) chunk = c->h_ndp[r] <= (uint32_t)CH_ROWS;
    const bool shrt = chunk && r1 - r0 == c->te[t] - c->tb[t];
    c->tl[cls][shrt ? 1 : (chunk && c->te[t] - c->tb[t] <= 64) ? 2 : 0].push_back((int32_t)t);
  }
  {
    std::vector<int32_t> all, cnt;
    const std::vector<int32_t>* parts[7] = {&c->tl[0][0], &c->tl[0][1], &c->tl[0][2], &c->tl[1][0],
                                            &c->tl[1][1], &c->tl[1][2], &c->tl_other};
    for (int i = 0; i < 7; i++) {
      c->tl_off[i] = (int64_t)all.size();
      all.insert(all.end(), parts[i]->begin(), parts[i]->end());
      cnt.push_back((int32_t)parts[i]->size());
    }
    HIP_OK(c->d_tl.ensure(std::max<size_t>(1, all.size()) * 4));
    HIP_OK(c->d_tl_n.ensure(7 * 4));
    if (!all.empty()) HIP_OK(hipMemcpy(c->d_tl.p, all.data(), all.size() * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(c->d_tl_n.p, cnt.data(), 7 * 4, hipMemcpyHostToDevice));
  }
  HIP_OK(c->d_tb.ensure(nt * 8));
  HIP_OK(c->d_te.ensure(nt * 8));
  HIP_OK(c->d_tg.ensure(nt * 4));
  HIP_OK(c->d_gtp.ensure(c->gtp.size() * 8));
  if (nt) {
    HIP_OK(hipMemcpy(c->d_tb.p, c->tb.data(), nt * 8, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(c->d_te.p, c->te.data(), nt * 8, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(c->d_tg.p, c->tg.data(), nt * 4, hipMemcpyHostToDevice));
  }
  HIP_OK(hipMemcpy(c->d_gtp.p, c->gtp.data(), c->gtp.size() * 8, hipMemcpyHostToDevice));
  c->none_tiles_ready = false;
  return 0;
}

static int build_none_tiles(tsdbhip_ctx* c) {
  if (c->none_tiles_ready) return 0;
  const int64_t n = c->n_series;
  std::vector<int64_t> tb(n), te(n), gtp(n + 1);
  std::vector<int32_t> tg(n);
  for (int64_t i = 0; i < n; i++) { tb[i] = i; te[i] = i + 1; tg[i] = (int32_t)i; gtp[i] = i; }
  gtp[n] = n;
  HIP_OK(c->n_tb.ensure(n * 8 + 8));
  HIP_OK(c->n_te.ensure(n * 8 + 8));
  HIP_OK(c->n_tg.ensure(n * 4 + 4));
  HIP_OK(c->n_gtp.ensure((n + 1) * 8));
  if (n) {
    HIP_OK(hipMemcpy(c->n_tb.p, tb.data(), n * 8, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(c->n_te.p, te.data(), n * 8, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(c->n_tg.p, tg.data(), n * 4, hipMemcpyHostToDevice));
  }
  HIP_OK(hipMemcpy(c->n_gtp.p, gtp.data(), (n + 1) * 8, hipMemcpyHostToDevice));
  c->none_tiles_ready = true;
  return 0;
}

static int finish_load(tsdbhip_ctx* c, const std::vector<RowDesc>& rd) {
  // classify rows on the device, then fetch ndp for host-side accounting
  HIP_OK(hipMemsetAsync(c->err.p, 0, 4, c->stream));
  const bool generic = opt_is(OPT_INDEX_GENERIC, 1);   // test hook: sequential per-datapoint path
  HIP_OK(c->hint.ensure(std::max<int64_t>(1, c->n_rows)));
  HIP_OK(c->ilist.ensure(std::max<int64_t>(1, c->n_rows) * 4));
  HIP_OK(c->icnt.ensure(32 * 4));
  const IndexBufs ib{c->hint.as<uint8_t>(), c->ilist.as<int32_t>(), c->icnt.as<uint32_t>()};
  // the int16 copy of 1-2-byte integer values (val2, k_short / k_fast's vle rows) is written by
  // the class kernels of the 2-byte-qualifier integer classes, allocated when such rows exist
  c->val2.release();
  // val2 allocated up front when it fits beside the batch with room to spare: the short rows are
  // then indexed by the classifying pass itself (index_fused, no separate k_index_hint); else the
  // classes first, val2 only when some row can need it (a 216-GB store has no room for a spare 72)
  bool fused = false;
  if (!generic) {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && fr > c->qual_bytes + BLOB_SLACK + ((size_t)8 << 30)) {
      HIP_OK(c->val2.ensure(c->qual_bytes + BLOB_SLACK));
      fused = true;
    }
  }
  HIP_OK(hipEventRecord(c->ev[0], c->stream));
  IndexClasses ik;
  if (fused)
    HIP_OK(index_fused(c->qual.as<uint8_t>(), c->val.as<uint8_t>(), c->val2.as<uint8_t>(), c->rows.as<RowDesc>(), ib,
                       c->n_rows, c->err.as<int32_t>(), &ik, c->stream));
  else
    HIP_OK(index_classes(c->qual.as<uint8_t>(), c->rows.as<RowDesc>(), ib, c->n_rows, &ik, c->stream));
  HIP_OK(hipEventRecord(c->ev[2], c->stream));
  if (!fused && ik.vle_capable && !generic) HIP_OK(c->val2.ensure(c->qual_bytes + BLOB_SLACK));
  HIP_OK(hipEventRecord(c->ev[3], c->stream));   // (the allocation is not index time)
  HIP_OK(index_rows(c->qual.as<uint8_t>(), c->val.as<uint8_t>(), c->val2.as<uint8_t>(), c->rows.as<RowDesc>(), ib, ik,
                    c->n_rows, c->err.as<int32_t>(), generic, c->stream));
  if (c->max_series_rows > 1)   // (rows going back in time need two rows of one series)
    HIP_OK(index_recede(c->rows.as<RowDesc>(), c->srp.as<int64_t>(), c->qual.as<uint8_t>(), c->n_series, c->stream));
  HIP_OK(hipEventRecord(c->ev[1], c->stream));
  std::vector<RowDesc> back(c->n_rows);
  if (c->n_rows)
    HIP_OK(hipMemcpyAsync(back.data(), c->rows.p, c->n_rows * sizeof(RowDesc), hipMemcpyDeviceToHost, c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  float t_index = 0, t_val2 = 0, t_cls = 0;
  (void)hipEventElapsedTime(&t_cls, c->ev[0], c->ev[2]);
  (void)hipEventElapsedTime(&t_index, c->ev[3], c->ev[1]);
  t_index += t_cls;
  bool need_val2 = false;
  for (const RowDesc& d : back)
    if ((d.flags & (ROW_QW_MASK | ROW_ALLI | ROW_VLE2 | ROW_ERR)) == (2u | ROW_ALLI | ROW_VLE2)) { need_val2 = true; break; }
  if (!need_val2) {
    c->val2.release();
  } else if (generic) {   // test hook: the sequential path writes the copy in a second pass
    HIP_OK(c->val2.ensure(c->qual_bytes + BLOB_SLACK));
    HIP_OK(hipEventRecord(c->ev[2], c->stream));
    HIP_OK(index_rows(c->qual.as<uint8_t>(), c->val.as<uint8_t>(), c->val2.as<uint8_t>(), c->rows.as<RowDesc>(), ib,
                      ik, c->n_rows, c->err.as<int32_t>(), true, c->stream));
    HIP_OK(hipEventRecord(c->ev[3], c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    (void)hipEventElapsedTime(&t_val2, c->ev[2], c->ev[3]);
  }
  c->index_ms = (double)t_index + t_val2;
  (void)rd;
  c->h_ndp.resize(c->n_rows);
  c->h_base.resize(c->n_rows);
  c->h_qlen.resize(c->n_rows);
  c->h_vlen.resize(c->n_rows);
  c->h_flags.resize(c->n_rows);
  int64_t cls[2][2] = {{0, 0}, {0, 0}};   // [qw 2/4][vl 4/8] uniform float rows
  int64_t cls_vle = 0;                    // 2-byte qualifiers, 1-2 byte integers, one chunk
  int64_t cls_pct[2][9] = {};             // [qw 2/4][vl]: uniform sorted rows of <= 512 dp
  int64_t cls_vonly[2] = {};              // [qw 2/4]: those of 4-byte values, all-float without NaN or all-int
  uint32_t vonly_max[2] = {};             // [qw 2/4]: their longest row
  for (int64_t r = 0; r < c->n_rows; r++) {
    c->h_ndp[r] = back[r].ndp;
    c->h_base[r] = back[r].base;
    c->h_qlen[r] = back[r].qlen;
    c->h_vlen[r] = back[r].vlen;
    c->h_flags[r] = back[r].flags;
    const uint32_t f = back[r].flags;
    const uint32_t qw = f & ROW_QW_MASK, vl = (f & ROW_VL_MASK) >> ROW_VL_SHIFT;
    if ((f & ROW_ALLF) && !(f & (ROW_ERR | ROW_NAN | ROW_UNSORTED)) && (qw == 2 || qw == 4) && (vl == 4 || vl == 8))
      cls[qw == 4][vl == 8] += back[r].ndp;
    if ((f & ROW_ALLI) && (f & ROW_VLE2) && !(f & (ROW_ERR | ROW_UNSORTED)) && qw == 2 && back[r].ndp <= 512)
      cls_vle += back[r].ndp;
    if (!(f & (ROW_ERR | ROW_UNSORTED)) && (qw == 2 || qw == 4) && (vl == 1 || vl == 2 || vl == 4 || vl == 8) &&
        back[r].ndp <= 512)
      cls_pct[qw == 4][vl] += back[r].ndp;
    if (!(f & (ROW_ERR | ROW_UNSORTED)) && (qw == 2 || qw == 4) && vl == 4 && back[r].ndp <= 512 &&
        (((f & ROW_ALLF) && !(f & ROW_NAN)) || (f & ROW_ALLI))) {
      cls_vonly[qw == 4] += back[r].ndp;
      vonly_max[qw == 4] = std::max(vonly_max[qw == 4], back[r].ndp);
    }
  }
  // the two largest k_fast row classes by datapoints
  struct Cand { int64_t n; int qw, vl; };
  std::vector<Cand> cand = {{cls[0][0], 2, 4}, {cls[0][1], 2, 8}, {cls[1][0], 4, 4}, {cls[1][1], 4, 8}, {cls_vle, 2, 0}};
  std::stable_sort(cand.begin(), cand.end(), [](const Cand& x, const Cand& y) { return x.n > y.n; });
  c->fast_qw = c->fast_vl = c->fast_qw2 = c->fast_vl2 = 0;
  if (cand[0].n > 0) { c->fast_qw = cand[0].qw; c->fast_vl = cand[0].vl; }
  if (cand[1].n > 0) { c->fast_qw2 = cand[1].qw; c->fast_vl2 = cand[1].vl; }
  c->pct_qw = c->pct_vl = 0;
  int64_t best = 0;
  for (int a = 0; a < 2; a++)
    for (int v = 1; v <= 8; v++)
      if (cls_pct[a][v] > best) { best = cls_pct[a][v]; c->pct_qw = a ? 4 : 2; c->pct_vl = v; }
  c->pct_vonly = c->pct_vl == 4 && best > 0 && cls_vonly[c->pct_qw == 4] == best;
  c->pct_v6 = c->pct_vonly && vonly_max[c->pct_qw == 4] <= 384;
  // malformed rows are reported lazily, when a query reads them (as the reference does)
  return build_tiles(c);
}

// RowSeq.addRow (src/core/RowSeq.java:91-222): ordered merge of the remote cell into the
// local one by qualifier offset (Internal.compareQualifiers :511-519), the remote datapoint
// dropped on equal offsets, meta byte MS_MIXED_COMPACT if either side has it.  false: a
// malformed cell (left unmerged; k_index reports it).
static bool merge_cells(std::vector<uint8_t>& lq, std::vector<uint8_t>& lv, const uint8_t* rq, size_t rql,
                        const uint8_t* rv, size_t rvl) {
  auto qlen_at = [](const uint8_t* q, size_t i) -> size_t { return (q[i] & 0xF0) == 0xF0 ? 4 : 2; };
  auto off_at = [](const uint8_t* q, size_t i) -> int64_t {
    if ((q[i] & 0xF0) == 0xF0)
      return (int64_t)(((((uint32_t)q[i] << 24) | ((uint32_t)q[i + 1] << 16) | ((uint32_t)q[i + 2] << 8) | q[i + 3]) &
                        0x0FFFFFC0u) >> 6);
    return (int64_t)((((uint32_t)q[i] << 8) | q[i + 1]) >> 4) * 1000;
  };
  if (lv.empty() || rvl == 0) return false;
  const uint8_t* q0 = lq.data();
  const uint8_t* v0 = lv.data();
  // value bytes are located through the qualifiers; the last byte of each side is its meta
  // byte (for a single-datapoint cell, the value's own last byte -- as the reference reads it)
  const size_t ql = lq.size(), vl = lv.size(), rvl0 = rvl;
  std::vector<uint8_t> mq, mv;
  mq.reserve(ql + rql);
  mv.reserve(vl + rvl0 + 1);
  size_t li = 0, ri = 0, lvi = 0, rvi = 0;
  while (ri < rql || li < ql) {
    bool remote;
    if (ri >= rql) remote = false;
    else if (li >= ql) remote = true;
    else {
      if (ri + qlen_at(rq, ri) > rql || li + qlen_at(q0, li) > ql) return false;
      const int64_t a = off_at(rq, ri), b2 = off_at(q0, li);
      if (a == b2) {
        rvi += (rq[ri + qlen_at(rq, ri) - 1] & 7) + 1;
        ri += qlen_at(rq, ri);
        continue;
      }
      remote = a < b2;
    }
    const uint8_t* q = remote ? rq : q0;
    const uint8_t* v = remote ? rv : v0;
    size_t& qi = remote ? ri : li;
    size_t& vi = remote ? rvi : lvi;
    const size_t qn = qlen_at(q, qi);
    if (qi + qn > (remote ? rql : ql)) return false;
    const size_t vn = (q[qi + qn - 1] & 7) + 1;
    if (vi + vn > (remote ? rvl0 : vl)) return false;
    mq.insert(mq.end(), q + qi, q + qi + qn);
    mv.insert(mv.end(), v + vi, v + vi + vn);
    qi += qn;
    vi += vn;
  }
  mv.push_back(((v0[vl - 1] & 1) || (rv[rvl0 - 1] & 1)) ? 1 : 0);
  lq.swap(mq);
  lv.swap(mv);
  return true;
}

// Loads series cand[0 .. m) of the batch (all series when cand is null), in that order as the
// "batch order" of the resident store (NONE results are emitted in it); series are then stably
// sorted by group (SpanGroup membership, order inside a group kept).
// (the caller holds c->mu: tsdbhip_load_rollup sets its rollup state under the same lock)
static int load_body(tsdbhip_ctx* c, const tsdbhip_batch* b, const std::vector<int64_t>* cand) {
  HIP_OK(hipSetDevice(c->device));
  if (b->n_series < 0 || b->n_rows < 0) return fail(TSDB_E_ILLEGAL_ARGUMENT, "negative sizes");
  if (b->n_series > 0 && (!b->series_row_ptr || !b->group_id)) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null batch arrays");
  if (b->n_rows > 0 && (!b->row_base_time || !b->row_qual_off || !b->row_val_off || !b->qual || !b->val))
    return fail(TSDB_E_ILLEGAL_ARGUMENT, "null batch arrays");
  if (b->n_series > 0 && (b->series_row_ptr[0] != 0 || b->series_row_ptr[b->n_series] != b->n_rows))
    return fail(TSDB_E_ILLEGAL_ARGUMENT, "series_row_ptr does not cover the rows");
  release_batch(c);
  const int64_t m = cand ? (int64_t)cand->size() : b->n_series;
  auto ser = [&](int64_t v) { return cand ? (*cand)[v] : v; };   // virtual batch position -> batch series
  // stable order of series by group (SpanGroup membership; order inside a group kept).
  // Series without a group (group id -1: a group-by tag missing) stay resident after the last
  // group, in batch order, under the sentinel group n_groups: no group-by tile visits them,
  // but the NONE aggregator emits every span (TsdbQuery.java:940-961).
  std::vector<int64_t> order;   // virtual positions
  int32_t maxg = -1;
  for (int64_t v = 0; v < m; v++) {
    const int64_t s = ser(v);
    if (s < 0 || s >= b->n_series) return fail(TSDB_E_ILLEGAL_ARGUMENT, "series index out of range");
    if (b->series_row_ptr[s + 1] < b->series_row_ptr[s]) return fail(TSDB_E_ILLEGAL_ARGUMENT, "series_row_ptr not monotonic");
    order.push_back(v);
    maxg = std::max(maxg, b->group_id[s]);
  }
  auto key = [&](int64_t v) { const int32_t g = b->group_id[ser(v)]; return g < 0 ? INT32_MAX : g; };
  std::stable_sort(order.begin(), order.end(), [&](int64_t x, int64_t y) { return key(x) < key(y); });
  c->n_series = (int64_t)order.size();
  c->n_groups = maxg + 1;
  c->h_group.resize(c->n_series);
  c->h_orig = order;
  c->h_srp.assign(c->n_series + 1, 0);
  c->max_series_rows = 0;
  std::vector<RowDesc> rd;
  uint64_t qtot = 0, vtot = 0;
  for (int64_t i = 0; i < c->n_series; i++) {
    const int64_t s = ser(order[i]);
    c->h_group[i] = b->group_id[s] < 0 ? (int32_t)c->n_groups : b->group_id[s];
    for (int64_t r = b->series_row_ptr[s]; r < b->series_row_ptr[s + 1]; r++) {
      RowDesc d{};
      d.base = b->row_base_time[r];
      const uint64_t ql = b->row_qual_off[r + 1] - b->row_qual_off[r];
      const uint64_t vl = b->row_val_off[r + 1] - b->row_val_off[r];
      if (ql > 0xFFFFFFFFull || vl > 0xFFFFFFFFull) return fail(TSDB_E_ILLEGAL_ARGUMENT, "row too large");
      d.qlen = (uint32_t)ql;
      d.vlen = (uint32_t)vl;
      d.qoff = qtot;
      d.voff = vtot;
      qtot += align16(ql);
      vtot += align16(vl);
      rd.push_back(d);
    }
    c->h_srp[i + 1] = (int64_t)rd.size();
    c->max_series_rows = std::max<int64_t>(c->max_series_rows, c->h_srp[i + 1] - c->h_srp[i]);
  }
  // rows of a series must be in base-time order (Span.checkRowOrder): stable sort per series
  for (int64_t i = 0; i < c->n_series; i++) {
    std::stable_sort(rd.begin() + c->h_srp[i], rd.begin() + c->h_srp[i + 1],
                     [](const RowDesc& x, const RowDesc& y) { return x.base < y.base; });
    if (c->h_srp[i + 1] > c->h_srp[i]) rd[c->h_srp[i]].flags |= ROW_SFIRST;
  }
  c->n_rows = (int64_t)rd.size();
  c->qual_bytes = qtot;
  c->val_bytes = vtot;
  // staging: re-laid-out blobs
  // tail slack: k_fast's vle class reads a fixed 1 KB value window from every row start
  std::vector<uint8_t> hq(qtot + BLOB_SLACK, 0), hv(vtot + BLOB_SLACK, 0);
  {
    // copy rows in the order their offsets were assigned (before the per-series sort)
    uint64_t qo = 0, vo = 0;
    for (int64_t i = 0; i < c->n_series; i++) {
      const int64_t s = ser(order[i]);
      for (int64_t r = b->series_row_ptr[s]; r < b->series_row_ptr[s + 1]; r++) {
        const uint64_t ql = b->row_qual_off[r + 1] - b->row_qual_off[r];
        const uint64_t vl = b->row_val_off[r + 1] - b->row_val_off[r];
        std::memcpy(hq.data() + qo, b->qual + b->row_qual_off[r], ql);
        std::memcpy(hv.data() + vo, b->val + b->row_val_off[r], vl);
        qo += align16(ql);
        vo += align16(vl);
      }
    }
  }
  HIP_OK(c->rows.ensure(std::max<size_t>(1, rd.size()) * sizeof(RowDesc)));
  HIP_OK(c->srp.ensure((c->n_series + 1) * 8));
  HIP_OK(c->qual.ensure(hq.size()));
  HIP_OK(c->val.ensure(hv.size()));
  HIP_OK(c->gid.ensure(std::max<int64_t>(1, c->n_series) * 4));
  if (!rd.empty()) HIP_OK(hipMemcpy(c->rows.p, rd.data(), rd.size() * sizeof(RowDesc), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(c->srp.p, c->h_srp.data(), (c->n_series + 1) * 8, hipMemcpyHostToDevice));
  HIP_OK(h2d(c, c->qual.p, hq.data(), hq.size(), c->stream));   // (the GPU pulls staged chunks: see h2d)
  HIP_OK(h2d(c, c->val.p, hv.data(), hv.size(), c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  if (c->n_series) HIP_OK(hipMemcpy(c->gid.p, c->h_group.data(), c->n_series * 4, hipMemcpyHostToDevice));
  return finish_load(c, rd);
}

static int load_impl(tsdbhip_ctx* c, const tsdbhip_batch* b, const std::vector<int64_t>* cand = nullptr) {
  if (!c || !b) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  CtxLock lk(c);
  return load_body(c, b, cand);
}

// ---------------------------------------------------------------------------
// synthetic store in HBM (the MockBase-equivalent generator of BASELINE.md)
// ---------------------------------------------------------------------------

// Span.addRow (src/core/Span.java:177-220): several cells of one series with the same base
// time (salt-bucket duplicates) merge into one RowSeq (RowSeq.addRow).  Batches without such
// rows are loaded as given; otherwise the merged batch is built first.
static int load_with(tsdbhip_ctx* c, const tsdbhip_batch* b, const std::vector<int64_t>* cand) {
  if (!c || !b) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  bool dup = false;
  if (b->n_series > 0 && b->n_rows > 0 && b->series_row_ptr && b->row_base_time && b->row_qual_off &&
      b->row_val_off && b->qual && b->val) {
    std::vector<uint32_t> bases;
    for (int64_t s = 0; s < b->n_series && !dup; s++) {
      const int64_t r0 = b->series_row_ptr[s], r1 = b->series_row_ptr[s + 1];
      if (r1 - r0 < 2 || r0 < 0 || r1 > b->n_rows) continue;
      bases.assign(b->row_base_time + r0, b->row_base_time + r1);
      std::sort(bases.begin(), bases.end());
      dup = std::adjacent_find(bases.begin(), bases.end()) != bases.end();
    }
  }
  if (!dup) return load_impl(c, b, cand);
  std::vector<int64_t> srp(b->n_series + 1, 0);
  std::vector<uint32_t> base;
  std::vector<uint64_t> qoff{0}, voff{0};
  std::vector<uint8_t> qual, val;
  for (int64_t s = 0; s < b->n_series; s++) {
    std::vector<uint32_t> obase;
    std::vector<std::vector<uint8_t>> oq, ov;
    for (int64_t r = b->series_row_ptr[s]; r < b->series_row_ptr[s + 1]; r++) {
      const uint8_t* q = b->qual + b->row_qual_off[r];
      const uint8_t* v = b->val + b->row_val_off[r];
      const size_t ql = b->row_qual_off[r + 1] - b->row_qual_off[r], vl = b->row_val_off[r + 1] - b->row_val_off[r];
      size_t j = 0;
      while (j < obase.size() && obase[j] != b->row_base_time[r]) j++;
      if (j < obase.size()) {
        std::vector<uint8_t> mq = oq[j], mv = ov[j];
        if (merge_cells(mq, mv, q, ql, v, vl)) { oq[j].swap(mq); ov[j].swap(mv); continue; }
      }
      obase.push_back(b->row_base_time[r]);
      oq.emplace_back(q, q + ql);
      ov.emplace_back(v, v + vl);
    }
    for (size_t j = 0; j < obase.size(); j++) {
      base.push_back(obase[j]);
      qual.insert(qual.end(), oq[j].begin(), oq[j].end());
      val.insert(val.end(), ov[j].begin(), ov[j].end());
      qoff.push_back(qual.size());
      voff.push_back(val.size());
    }
    srp[s + 1] = (int64_t)base.size();
  }
  if (qual.empty()) qual.push_back(0);
  if (val.empty()) val.push_back(0);
  tsdbhip_batch m = *b;
  m.n_rows = (int64_t)base.size();
  m.series_row_ptr = srp.data();
  m.row_base_time = base.data();
  m.row_qual_off = qoff.data();
  m.row_val_off = voff.data();
  m.qual = qual.data();
  m.val = val.data();
  return load_impl(c, &m, cand);   // series indices are unchanged by the merge
}

extern "C" int tsdbhip_load(tsdbhip_ctx* c, const tsdbhip_batch* b) {
  if (c && c->md) return tsdb::md_load(c, b);
  return load_with(c, b, nullptr);
}

// ---- rollup read path ---------------------------------------------
// The host restates what the scan builds of a rollup table -- RollupSpan.addRow
// (src/rollup/RollupSpan.java:62-80), RollupSeq.append (src/rollup/RollupSeq.java:238-318)
// and the RollupIterator's sync (:521-555) -- and hands the device the datapoints the
// iterators yield: each value series (its cells decoded by the resident kernels as they are)
// and, with count cells, a count series of valueCount()s, both re-rowed into hour rows with
// 2-byte second qualifiers.  Every hour row holds the points of one rollup row (rollup row
// spans are whole hours), so the scan range picks the same points either way.
namespace {

struct RoCell {
  uint32_t q;
  const uint8_t* v;
};

int64_t ro_cell_len(uint32_t q) { return (q & 7) + 1; }   // Internal.getValueLengthFromQualifier

// valueCount() of a count cell (RollupSeq.java:661-675): the integer, or (long) of the float
bool ro_count_value(const RoCell& k, int64_t& out) {
  const uint8_t* p = k.v;
  auto be = [&](int n) { uint64_t x = 0; for (int i = 0; i < n; i++) x = (x << 8) | p[i]; return x; };
  if ((k.q & 0x8) == 0) {
    switch (k.q & 7) {
      case 7: out = (int64_t)be(8); return true;
      case 3: out = (int32_t)(uint32_t)be(4); return true;
      case 1: out = (int16_t)(uint16_t)be(2); return true;
      case 0: out = (int8_t)p[0]; return true;
      default: return false;
    }
  }
  double x;
  if ((k.q & 7) == 7) { const uint64_t u = be(8); std::memcpy(&x, &u, 8); }
  else if ((k.q & 7) == 3) { const uint32_t u = (uint32_t)be(4); float f; std::memcpy(&f, &u, 4); x = f; }
  else return false;
  out = x != x ? 0 : (x >= 9.2233720368547758e18 ? INT64_MAX : (x <= -9.2233720368547758e18 ? INT64_MIN : (int64_t)x));
  return true;
}

bool ro_value_ok(uint32_t q) {   // extractIntegerValue / extractFloatingPointValue accept these
  const uint32_t l = q & 7;
  return (q & 0x8) ? (l == 3 || l == 7) : (l == 0 || l == 1 || l == 3 || l == 7);
}

// Internal.vleEncodeLong
int vle_put(std::vector<uint8_t>& out, int64_t v) {
  int n = (v >= -128 && v <= 127) ? 1 : (v >= -32768 && v <= 32767) ? 2 : (v >= INT32_MIN && v <= INT32_MAX) ? 4 : 8;
  for (int i = n - 1; i >= 0; i--) out.push_back((uint8_t)((uint64_t)v >> (8 * i)));
  return n;
}
// The packed pairs as runs (RoRun): consecutive pairs of one series with equal meta whose base
// time and byte offsets advance by one constant step each.  Kept only when the runs and the
// per-pair run ids take less than the pairs (hour rows of equal shape: one run a series).
static int ro_build_runs(tsdbhip_ctx* c) {
  const int64_t n = c->ro_npairs;
  c->ro_nruns = 0;
  if (n <= 0 || opt_off(OPT_RO_RUNS)) return 0;
  std::vector<RoPair> hp(n);
  HIP_OK(hipMemcpy(hp.data(), c->ro_pairs.p, n * sizeof(RoPair), hipMemcpyDeviceToHost));
  std::vector<RoRun> runs;
  std::vector<uint32_t> rid(n);
  auto same = [](const RoPair& a, const RoPair& b) {
    return a.base == b.base && a.qoff == b.qoff && a.voff == b.voff && a.cvoff == b.cvoff && a.meta == b.meta &&
           a.series == b.series;
  };
  for (int64_t i = 0; i < n; i++) {
    const RoPair& P = hp[i];
    bool cont = false;
    if (!runs.empty()) {
      RoRun& R = runs.back();
      if (P.series == R.series && P.meta == R.meta) {
        if ((int64_t)i - R.first == 1) {   // the run's second pair sets its step
          const int64_t db = (int64_t)P.base - R.base0, dq = (int64_t)P.qoff - R.qoff0,
                        dv = (int64_t)P.voff - R.voff0, dc = (int64_t)P.cvoff - R.cvoff0;
          if (db > 0 && db % 3600 == 0 && db / 3600 < 256 && dq >= 0 && dq % 16 == 0 && dq / 16 < 128 && dv >= 0 &&
              dv % 16 == 0 && dv / 16 < 512 && dc >= 0 && dc % 16 == 0 && dc / 16 < 256) {
            R.step = (uint32_t)(dq / 16) | (uint32_t)(dv / 16) << 7 | (uint32_t)(dc / 16) << 16 | (uint32_t)(db / 3600) << 24;
            cont = same(ro_run_pair(R, (uint32_t)i), P);
            if (!cont) R.step = 0;
          }
        } else if ((int64_t)i - R.first > 1) {
          cont = same(ro_run_pair(R, (uint32_t)i), P);
        }
      }
    }
    if (!cont) runs.push_back(RoRun{(uint32_t)i, P.base, P.qoff, P.voff, P.cvoff, P.meta, P.series, 0u});
    rid[i] = (uint32_t)(runs.size() - 1);
  }
  const int64_t nr = (int64_t)runs.size();
  if (nr * (int64_t)sizeof(RoRun) + n * 4 >= n * (int64_t)sizeof(RoPair)) return 0;   // the pairs are smaller
  HIP_OK(c->ro_runs.ensure(nr * (int64_t)sizeof(RoRun)));
  HIP_OK(c->ro_rid.ensure(n * 4));
  HIP_OK(hipMemcpy(c->ro_runs.p, runs.data(), nr * sizeof(RoRun), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(c->ro_rid.p, rid.data(), n * 4, hipMemcpyHostToDevice));
  c->ro_pairs.release();
  c->ro_nruns = nr;
  return 0;
}


}  // namespace

extern "C" int tsdbhip_load_rollup(tsdbhip_ctx* c, const tsdbhip_rollup_batch* rb) {
  if (c && c->md) return tsdb::md_load_rollup(c, rb);
  if (!c || !rb) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  const tsdbhip_batch* b = &rb->cells;
  const bool cnt = rb->row_cqual_off != nullptr;
  if (cnt && (!rb->row_cval_off || !rb->cqual || !rb->cval)) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null count arrays");
  const tsdbhip_rollup_interval iv = rb->interval;
  if (iv.interval_s <= 0 || iv.intervals <= 0) return fail(TSDB_E_ILLEGAL_ARGUMENT, "bad rollup interval");
  const int64_t NS = b->n_series;
  if (NS < 0 || b->n_rows < 0) return fail(TSDB_E_ILLEGAL_ARGUMENT, "negative sizes");
  if (NS > 0 && (!b->series_row_ptr || !b->group_id)) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null batch arrays");
  if (b->n_rows > 0 && (!b->row_base_time || !b->row_qual_off || !b->row_val_off || !b->qual || !b->val))
    return fail(TSDB_E_ILLEGAL_ARGUMENT, "null batch arrays");
  if (NS > 0 && (b->series_row_ptr[0] != 0 || b->series_row_ptr[NS] != b->n_rows))
    return fail(TSDB_E_ILLEGAL_ARGUMENT, "series_row_ptr does not cover the rows");
  for (int64_t s = 0; s < NS; s++)
    if (b->series_row_ptr[s + 1] < b->series_row_ptr[s]) return fail(TSDB_E_ILLEGAL_ARGUMENT, "series_row_ptr not monotonic");
  for (int64_t r = 0; r < b->n_rows; r++) {
    if (b->row_qual_off[r + 1] < b->row_qual_off[r] || b->row_val_off[r + 1] < b->row_val_off[r] ||
        (cnt && (rb->row_cqual_off[r + 1] < rb->row_cqual_off[r] || rb->row_cval_off[r + 1] < rb->row_cval_off[r])))
      return fail(TSDB_E_ILLEGAL_ARGUMENT, "cell offsets not monotonic");
  }
  const int64_t iv_ms = (int64_t)iv.interval_s * 1000;
  // the converted batch: value series [0, NS), then (cnt) count series [NS, 2 NS)
  struct Out {
    std::vector<int64_t> srp{0};
    std::vector<uint32_t> base;
    std::vector<uint64_t> qo{0}, vo{0};
    std::vector<uint8_t> q, v;
  } ov, oc;
  std::vector<RoSeqRow> rows;
  std::vector<int64_t> rp{0};
  std::vector<std::string> unsup(NS);
  struct Pt { int64_t ts; RoCell v; int64_t n; };
  for (int64_t s = 0; s < NS; s++) {
    struct Seq {
      RoSeqRow info;
      std::vector<RoCell> vc, cc;
      int64_t lo = -1, lco = -1;
    };
    std::vector<Seq> seqs;
    for (int64_t r = b->series_row_ptr[s]; r < b->series_row_ptr[s + 1]; r++) {
      // RollupSpan.addRow: a row with the last row's key appends to that RollupSeq
      if (seqs.empty() || seqs.back().info.base != (int64_t)b->row_base_time[r]) {
        seqs.emplace_back();
        seqs.back().info.base = b->row_base_time[r];
        seqs.back().info.order = (int64_t)seqs.size() - 1;
      }
      Seq& sq = seqs.back();
      if (sq.info.err) continue;   // the scan throws at the first bad cell of this key
      // RollupSeq.append :238-318 per cell, value cells then count cells (qualifier order)
      for (int pass = 0; pass < (cnt ? 2 : 1) && !sq.info.err; pass++) {
        const bool isc = pass == 1;
        const uint64_t* qo = isc ? rb->row_cqual_off : b->row_qual_off;
        const uint64_t* vo = isc ? rb->row_cval_off : b->row_val_off;
        const uint8_t* qb = isc ? rb->cqual : b->qual;
        const uint8_t* vb = isc ? rb->cval : b->val;
        const int64_t ql = (int64_t)(qo[r + 1] - qo[r]), vl = (int64_t)(vo[r + 1] - vo[r]);
        if (ql % 2) { sq.info.err = TSDB_E_ILLEGAL_DATA; sq.info.msg = "rollup qualifiers are 2 bytes"; break; }
        int64_t vi = 0;
        for (int64_t i = 0; i < ql; i += 2) {
          const uint32_t q = ((uint32_t)qb[qo[r] + i] << 8) | qb[qo[r] + i + 1];
          const int64_t len = ro_cell_len(q);
          if (vi + len > vl) { sq.info.err = TSDB_E_ILLEGAL_DATA; sq.info.msg = "rollup value bytes shorter than the qualifiers say"; break; }
          const int64_t off = (int64_t)(q >> 4);
          int64_t& last = isc ? sq.lco : sq.lo;
          std::vector<RoCell>& cells = isc ? sq.cc : sq.vc;
          if (last > -1 && off <= last) {
            if (off == last && rb->fix_duplicates) {
              cells.pop_back();   // the later cell replaces the earlier one (equal write timestamps)
            } else {
              sq.info.err = isc ? TSDB_E_ILLEGAL_ARGUMENT : TSDB_E_ILLEGAL_DATA;
              sq.info.msg = std::string(isc ? "The count offset " : "The offset ") + std::to_string(off) +
                            " is <= the last offset " + std::to_string(last);
              break;
            }
          }
          last = off;
          cells.push_back({q, vb + vo[r] + vi});
          vi += len;
        }
        if (!sq.info.err && vi != vl) { sq.info.err = TSDB_E_ILLEGAL_DATA; sq.info.msg = "rollup value bytes longer than the qualifiers say"; }
      }
    }
    // Span.checkRowOrder: stable sort by base time; then each RollupIterator's datapoints
    std::vector<Seq*> sorted;
    for (auto& sq : seqs) sorted.push_back(&sq);
    std::stable_sort(sorted.begin(), sorted.end(), [](const Seq* x, const Seq* y) { return x->info.base < y->info.base; });
    std::vector<Pt> pts;
    for (size_t i = 0; i < sorted.size(); i++) {
      Seq& sq = *sorted[i];
      if (i > 0 && sorted[i - 1]->info.base == sq.info.base && unsup[s].empty())
        unsup[s] = "two RollupSeqs with one row key (cells of a key not adjacent in the batch)";
      if (sq.info.err) continue;
      int32_t basetime = 0;
      if (tsdbhip_rollup_basetime(sq.info.base, &iv, &basetime) || basetime != sq.info.base) {
        if (unsup[s].empty()) unsup[s] = "rollup row base time not on the table's row span";
        continue;
      }
      const int64_t nv = (int64_t)sq.vc.size(), nc = (int64_t)sq.cc.size();
      int64_t qi = 0, ci = 0;
      auto sync = [&]() {   // RollupIterator.sync :521-555
        while (qi < nv && ci < nc) {
          const int64_t a = sq.vc[qi].q >> 4, d = sq.cc[ci].q >> 4;
          if (a == d) return;
          if (a > d) ci++; else qi++;
        }
      };
      if (cnt) {
        sync();
        // lock-step pairing from the first matched pair (RollupIterator.seek walks both)
        for (int64_t k = 0; qi + k < nv; k++) {
          if (ci + k >= nc || (sq.vc[qi + k].q >> 4) != (sq.cc[ci + k].q >> 4)) {
            sq.info.pp_ts = sq.info.base * 1000 + (int64_t)(sq.vc[qi + k].q >> 4) * iv_ms;
            break;
          }
        }
      }
      for (;;) {
        if (cnt) sync();
        if (!(qi < nv && (!cnt || ci < nc))) break;
        const RoCell& v = sq.vc[qi++];
        int64_t n = 1;
        if (cnt && !ro_count_value(sq.cc[ci++], n)) sq.info.cerr = true;
        if (!ro_value_ok(v.q)) sq.info.verr = true;
        const int64_t ts = sq.info.base * 1000 + (int64_t)(v.q >> 4) * iv_ms;
        int32_t bt = 0;
        if ((tsdbhip_rollup_basetime(ts / 1000, &iv, &bt) || bt != sq.info.base) && unsup[s].empty())
          unsup[s] = "rollup offset beyond the row span";
        pts.push_back({ts, v, n});
        sq.info.npts++;
        sq.info.last_ts = ts;
      }
    }
    for (size_t i = 1; i < pts.size() && unsup[s].empty(); i++)
      if (pts[i].ts <= pts[i - 1].ts) unsup[s] = "rollup datapoints out of time order across rows";
    for (auto& sq : seqs) rows.push_back(sq.info);
    rp.push_back((int64_t)rows.size());
    if (!unsup[s].empty()) pts.clear();
    // hour rows: compacted cells (2-byte qualifiers, meta byte 0 after two or more points)
    for (size_t i = 0; i < pts.size();) {
      const int64_t hb = (pts[i].ts / 1000) - (pts[i].ts / 1000) % 3600;
      size_t j = i;
      while (j < pts.size() && pts[j].ts / 1000 - hb < 3600) j++;
      for (int side = 0; side < (cnt ? 2 : 1); side++) {
        Out& o = side ? oc : ov;
        o.base.push_back((uint32_t)hb);
        for (size_t k = i; k < j; k++) {
          const uint32_t off = (uint32_t)(pts[k].ts / 1000 - hb);
          uint32_t q;
          if (side == 0) {
            q = (off << 4) | (pts[k].v.q & 0xF);
            o.v.insert(o.v.end(), pts[k].v.v, pts[k].v.v + ro_cell_len(pts[k].v.q));
          } else {
            q = (off << 4) | (uint32_t)(vle_put(o.v, pts[k].n) - 1);
          }
          o.q.push_back((uint8_t)(q >> 8));
          o.q.push_back((uint8_t)q);
        }
        if (j - i > 1) o.v.push_back(0);
        o.qo.push_back(o.q.size());
        o.vo.push_back(o.v.size());
      }
      i = j;
    }
    ov.srp.push_back((int64_t)ov.base.size());
    if (cnt) oc.srp.push_back((int64_t)oc.base.size());
  }
  // one batch: the count series after the value series
  const int64_t nrv = (int64_t)ov.base.size();
  std::vector<int32_t> gid(b->group_id, b->group_id + NS);
  if (cnt) {
    for (size_t i = 1; i < oc.srp.size(); i++) ov.srp.push_back(nrv + oc.srp[i]);
    const uint64_t q0 = ov.q.size(), v0 = ov.v.size();
    ov.base.insert(ov.base.end(), oc.base.begin(), oc.base.end());
    for (size_t i = 1; i < oc.qo.size(); i++) { ov.qo.push_back(q0 + oc.qo[i]); ov.vo.push_back(v0 + oc.vo[i]); }
    ov.q.insert(ov.q.end(), oc.q.begin(), oc.q.end());
    ov.v.insert(ov.v.end(), oc.v.begin(), oc.v.end());
    gid.insert(gid.end(), NS, -1);
  }
  if (ov.q.empty()) ov.q.push_back(0);
  if (ov.v.empty()) ov.v.push_back(0);
  tsdbhip_batch m{};
  m.n_series = cnt ? 2 * NS : NS;
  m.series_row_ptr = ov.srp.data();
  m.n_rows = (int64_t)ov.base.size();
  m.row_base_time = ov.base.data();
  m.row_qual_off = ov.qo.data();
  m.row_val_off = ov.vo.data();
  m.qual = ov.q.data();
  m.val = ov.v.data();
  m.group_id = gid.data();
  CtxLock lk(c);   // the batch and its rollup state in one critical section
  int rc = load_body(c, &m, nullptr);
  if (rc) return rc;
  c->ro_active = true;
  c->ro_counts = cnt;
  c->ro_iv = iv;
  c->ro_nval = NS;
  c->ro_rp = std::move(rp);
  c->ro_rows = std::move(rows);
  c->ro_chk_valid = false;
  c->ro_unsup = std::move(unsup);
  c->ro_res.assign(c->n_series, -1);
  for (int64_t i = 0; i < c->n_series; i++) c->ro_res[c->h_orig[i]] = i;
  std::vector<int64_t> cmap(std::max<int64_t>(1, c->n_series), -1);
  if (cnt)
    for (int64_t s = 0; s < NS; s++) cmap[c->ro_res[s]] = c->ro_res[NS + s];
  HIP_OK(c->ro_cmap.ensure((int64_t)cmap.size() * 8));
  HIP_OK(hipMemcpy(c->ro_cmap.p, cmap.data(), cmap.size() * 8, hipMemcpyHostToDevice));
  if (cnt) {   // each value row's count row: the load wrote them in lock step
    std::vector<int32_t> partner(std::max<int64_t>(1, c->n_rows), -1);
    for (int64_t s = 0; s < c->n_series; s++) {
      const int64_t cs = cmap[s];
      if (cs < 0) continue;
      const int64_t n = c->h_srp[s + 1] - c->h_srp[s];
      const bool mirror = c->h_srp[cs + 1] - c->h_srp[cs] == n;
      for (int64_t k = 0; k < n; k++) partner[c->h_srp[s] + k] = mirror ? (int32_t)(c->h_srp[cs] + k) : -2;
    }
    HIP_OK(c->ro_partner.ensure((int64_t)partner.size() * 4));
    HIP_OK(hipMemcpy(c->ro_partner.p, partner.data(), partner.size() * 4, hipMemcpyHostToDevice));
  }
  // the value rows packed (with their count rows when the table has count cells): k_ro_pack,
  // for k_ro_pairs (avg / count downsampling) and k_ro_rows (the other functions)
  {
    std::vector<int32_t> vrows, vser;
    for (int64_t s = 0; s < c->n_series; s++) {
      if (c->h_orig[s] >= NS) continue;   // a count series
      for (int64_t r = c->h_srp[s]; r < c->h_srp[s + 1]; r++) {
        vrows.push_back((int32_t)r);
        vser.push_back((int32_t)s);
      }
    }
    c->ro_npairs = (int64_t)vrows.size();
    if (c->ro_npairs && c->n_rows < ((int64_t)1 << 31)) {
      DevBuf dv, ds;
      HIP_OK(dv.ensure(c->ro_npairs * 4));
      HIP_OK(ds.ensure(c->ro_npairs * 4));
      HIP_OK(hipMemcpy(dv.p, vrows.data(), c->ro_npairs * 4, hipMemcpyHostToDevice));
      HIP_OK(hipMemcpy(ds.p, vser.data(), c->ro_npairs * 4, hipMemcpyHostToDevice));
      HIP_OK(c->ro_pairs.ensure(c->ro_npairs * (int64_t)sizeof(RoPair)));
      HIP_OK(launch_ro_pack(c->rows.as<RowDesc>(), cnt ? c->ro_partner.as<int32_t>() : nullptr, dv.as<int32_t>(),
                            ds.as<int32_t>(), c->qual.as<uint8_t>(), c->ro_npairs, c->ro_pairs.as<RoPair>(), c->stream));
      const hipError_t e = hipStreamSynchronize(c->stream);
      dv.release();   // (DevBuf frees nothing on its own)
      ds.release();
      HIP_OK(e);
      int rc = ro_build_runs(c);
      if (rc) return rc;
    } else {
      c->ro_npairs = 0;
    }
  }
  return 0;
}

// ---- query-time compaction -----------------------------------------
// The scanner's rows before TSDB.compact: the device compacts every row (k_compact.hip), the
// host lays the compacted rows out as the resident batch (series by group, rows by base time,
// rows without a datapoint dropped as SaltScanner.processRow drops a null compaction).
extern "C" int tsdbhip_load_cells(tsdbhip_ctx* c, const tsdbhip_cell_batch* cb) {
  if (!c || !cb) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  if (c->md) return tsdb::md_load_cells(c, cb);
  const int64_t NS = cb->n_series, NR = cb->n_rows, NC = cb->n_cols;
  if (NS < 0 || NR < 0 || NC < 0) return fail(TSDB_E_ILLEGAL_ARGUMENT, "negative sizes");
  if (NS > 0 && (!cb->series_row_ptr || !cb->group_id)) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null batch arrays");
  if (NR > 0 && (!cb->row_base_time || !cb->row_col_ptr)) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null batch arrays");
  if (NC > 0 && (!cb->col_qual_off || !cb->col_val_off || !cb->qual || !cb->val))
    return fail(TSDB_E_ILLEGAL_ARGUMENT, "null batch arrays");
  if (NS > 0 && (cb->series_row_ptr[0] != 0 || cb->series_row_ptr[NS] != NR))
    return fail(TSDB_E_ILLEGAL_ARGUMENT, "series_row_ptr does not cover the rows");
  if (NR > 0 && (cb->row_col_ptr[0] != 0 || cb->row_col_ptr[NR] != NC))
    return fail(TSDB_E_ILLEGAL_ARGUMENT, "row_col_ptr does not cover the columns");
  for (int64_t s = 0; s < NS; s++)
    if (cb->series_row_ptr[s + 1] < cb->series_row_ptr[s]) return fail(TSDB_E_ILLEGAL_ARGUMENT, "series_row_ptr not monotonic");
  for (int64_t r = 0; r < NR; r++)
    if (cb->row_col_ptr[r + 1] < cb->row_col_ptr[r]) return fail(TSDB_E_ILLEGAL_ARGUMENT, "row_col_ptr not monotonic");
  if (NC > 0 && (cb->col_qual_off[0] != 0 || cb->col_val_off[0] != 0))
    return fail(TSDB_E_ILLEGAL_ARGUMENT, "column offsets must start at 0");
  // The scan in chunks of whole rows, each under 2^31 columns and 2^31 datapoints: a datapoint
  // takes at least 2 qualifier bytes, or 3 bytes of an append value, so a row holds at most
  // (qualifier + value bytes) / 2.  The column offsets are checked on the device chunk by chunk
  // (k_cmp_rebase), not here.  One chunk: one pass.  Several: the first pass sizes every row, the
  // host lays the batch out, and the second pass recomputes each chunk's entries and writes them.
  const int64_t kLim = ((int64_t)1 << 31) - 1;
  int64_t limit = kLim;
  if (opt(OPT_CMP_CHUNK) > 0) limit = opt(OPT_CMP_CHUNK);   // tests: force chunks
  std::vector<int64_t> cuts{0};
  {
    int64_t w = 0;
    for (int64_t r = 0; r < NR; r++) {
      const int64_t c0 = cb->row_col_ptr[r], c1 = cb->row_col_ptr[r + 1];
      int64_t wr = c1 - c0;
      if (c1 > c0) {
        const uint64_t q0 = cb->col_qual_off[c0], q1 = cb->col_qual_off[c1];
        const uint64_t v0 = cb->col_val_off[c0], v1 = cb->col_val_off[c1];
        if (q1 < q0 || v1 < v0) return fail(TSDB_E_ILLEGAL_ARGUMENT, "column offsets not monotonic");
        if (q1 - q0 + v1 - v0 >= (uint64_t)2 * kLim) wr = kLim;
        else wr = std::max<int64_t>(wr, (int64_t)((q1 - q0 + v1 - v0) / 2));
      }
      if (wr >= kLim) return fail(TSDB_E_NOT_IMPLEMENTED, "a row of more than 2^31 columns or datapoints");
      if (w + wr > limit && r > cuts.back()) {
        cuts.push_back(r);
        w = 0;
      }
      w += wr;
    }
    cuts.push_back(NR);
  }
  const int n_chunks = (int)cuts.size() - 1;
  // option TRACE = 1: host wall time of the call's phases on stderr (diagnostics only)
  const bool trace = opt_is(OPT_TRACE, 1);
  auto t_last = std::chrono::steady_clock::now();
  auto mark = [&](const char* what) {
    if (!trace) return;
    (void)hipStreamSynchronize(c->stream);
    const auto t = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[trace load_cells] %-14s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t - t_last).count());
    t_last = t;
  };
  mark("validate+plan");
  CtxLock lk(c);
  HIP_OK(hipSetDevice(c->device));
  release_batch(c);
  // device copies of one chunk of the scan and per-column / per-row scratch (freed at the end)
  DevBuf d_rcp, d_cqo, d_cvo, d_cts, d_q, d_v, d_crow, d_cn, d_coff, d_cinfo, d_rheap, d_rone, d_rerr;
  DevBuf d_key, d_key2, d_idx, d_idx2, d_ecol, d_eqo, d_evo, d_klen, d_sq, d_sv, d_sc, d_sm;
  DevBuf d_rlo, d_rq, d_rv, d_rstate, d_rmeta, d_rdq, d_rdv, d_raw, d_bad, d_rmax, d_klist, d_cq32, d_cv32;
  auto release_all = [&]() {
    for (DevBuf* b : {&d_rcp, &d_cqo, &d_cvo, &d_cts, &d_q, &d_v, &d_crow, &d_cn, &d_coff, &d_cinfo, &d_rheap, &d_rone,
                      &d_rerr, &d_key, &d_key2, &d_idx, &d_idx2, &d_ecol, &d_eqo, &d_evo, &d_klen, &d_sq, &d_sv,
                      &d_sc, &d_sm, &d_rlo, &d_rq, &d_rv, &d_rstate, &d_rmeta, &d_rdq, &d_rdv, &d_raw, &d_bad, &d_rmax, &d_klist, &d_cq32, &d_cv32})
      b->release();
  };
  struct Rel { std::function<void()> f; ~Rel() { f(); } } rel{release_all};
  const hipStream_t st = c->stream;
  const int64_t R1 = std::max<int64_t>(1, NR);
  std::vector<int64_t> rq(R1), rv(R1), rdq(R1, -1), rdv(R1, -1);
  std::vector<int32_t> rstate(R1), rerr(R1);
  CmpParams p{};
  p.fix_dup = cb->fix_duplicates ? 1 : 0;
  p.dtcs = cb->use_otsdb_timestamp ? (cb->use_max_value ? 1 : 2) : 0;
  // device spans; the uploads and the host layout between them are not counted.  A scan in several
  // chunks sizes every chunk, then recomputes each one before writing it: both passes count.
  double cmp_ms = 0;
  HIP_OK(d_bad.ensure(4));
  HIP_OK(d_rmax.ensure(16));
  // the per-row LDS path (k_cmp_row) when every row of a chunk fits one block; else the global
  // sort (option CMP_ROWS = 0 forces the latter)
  // (dtcsMergeDataPoints, a non-default configuration, is restated in k_cmp_dedup only)
  const bool rows_ok = !opt_off(OPT_CMP_ROWS) && !p.dtcs;
  std::vector<int> row_cap(n_chunks, 0);
  std::vector<uint32_t> row_span(n_chunks, 0);
  // upload, analyze and build the entries of chunk k; its rows' sizes and states to the host
  auto prepare = [&](int k) -> int {
    const int64_t r0 = cuts[k], r1 = cuts[k + 1], nr = r1 - r0;
    const int64_t c0 = NR ? cb->row_col_ptr[r0] : 0, c1 = NR ? cb->row_col_ptr[r1] : 0, nc = c1 - c0;
    const uint64_t qa = nc ? cb->col_qual_off[c0] : 0, qz = nc ? cb->col_qual_off[c1] : 0;
    const uint64_t va = nc ? cb->col_val_off[c0] : 0, vz = nc ? cb->col_val_off[c1] : 0;
    const int64_t r1c = std::max<int64_t>(1, nr), c1c = std::max<int64_t>(1, nc);
    HIP_OK(d_rcp.ensure((r1c + 1) * 8));
    HIP_OK(d_cqo.ensure((c1c + 1) * 8));
    HIP_OK(d_cvo.ensure((c1c + 1) * 8));
    HIP_OK(d_raw.ensure((std::max(r1c, c1c) + 1) * 8));
    HIP_OK(d_q.ensure(std::max<uint64_t>(16, qz - qa) + 16));   // (+16: dword reads past the last byte)
    HIP_OK(d_v.ensure(std::max<uint64_t>(16, vz - va) + 16));
    if (cb->col_timestamp) HIP_OK(d_cts.ensure(c1c * 8));
    HIP_OK(hipMemsetAsync(d_bad.p, 0, 4, st));
    if (nr) {
      HIP_OK(hipMemcpyAsync(d_raw.p, cb->row_col_ptr + r0, (nr + 1) * 8, hipMemcpyHostToDevice, st));
      HIP_OK(cmp_rebase(d_raw.as<uint64_t>(), d_rcp.as<uint64_t>(), nr + 1, (uint64_t)c0, d_bad.as<int32_t>(), st));
    }
    if (nc) {
      HIP_OK(h2d(c, d_raw.p, cb->col_qual_off + c0, (nc + 1) * 8, st));
      HIP_OK(cmp_rebase(d_raw.as<uint64_t>(), d_cqo.as<uint64_t>(), nc + 1, qa, d_bad.as<int32_t>(), st));
      HIP_OK(h2d(c, d_raw.p, cb->col_val_off + c0, (nc + 1) * 8, st));
      HIP_OK(cmp_rebase(d_raw.as<uint64_t>(), d_cvo.as<uint64_t>(), nc + 1, va, d_bad.as<int32_t>(), st));
      if (qz > qa) HIP_OK(h2d(c, d_q.p, cb->qual + qa, qz - qa, st));
      if (vz > va) HIP_OK(h2d(c, d_v.p, cb->val + va, vz - va, st));
      if (cb->col_timestamp) HIP_OK(h2d(c, d_cts.p, cb->col_timestamp + c0, nc * 8, st));
    }
    int32_t bad = 0;
    { int rc_ = d2h_small(c, &bad, d_bad.p, 4, st); if (rc_) return rc_; }
    { int rc_ = sync_small(c, st); if (rc_) return rc_; }
    if (bad) return fail(TSDB_E_ILLEGAL_ARGUMENT, "column offsets not monotonic");
    HIP_OK(d_crow.ensure(c1c * 4));
    HIP_OK(d_cn.ensure(c1c * 8));
    HIP_OK(d_coff.ensure((c1c + 1) * 8));
    HIP_OK(d_cinfo.ensure(c1c * 4));
    HIP_OK(d_rheap.ensure(r1c * 4));
    HIP_OK(d_rone.ensure(r1c * 8));
    HIP_OK(d_rerr.ensure(r1c * 4));
    HIP_OK(hipMemsetAsync(d_rheap.p, 0, r1c * 4, st));
    HIP_OK(hipMemsetAsync(d_rone.p, 0, r1c * 8, st));
    HIP_OK(hipMemsetAsync(d_rerr.p, 0, r1c * 4, st));
    p.n_rows = nr;
    p.n_cols = nc;
    p.row_col_ptr = d_rcp.as<int64_t>();
    p.col_qo = d_cqo.as<uint64_t>();
    p.col_vo = d_cvo.as<uint64_t>();
    p.col_ts = cb->col_timestamp ? d_cts.as<int64_t>() : nullptr;
    p.q = d_q.as<uint8_t>();
    p.v = d_v.as<uint8_t>();
    p.col_row = d_crow.as<int32_t>();
    p.col_n = d_cn.as<int64_t>();
    p.col_off = d_coff.as<int64_t>();
    p.col_info = d_cinfo.as<uint32_t>();
    p.row_heap = d_rheap.as<int32_t>();
    p.row_one = d_rone.as<int64_t>();
    p.row_err = d_rerr.as<int32_t>();
    HIP_OK(hipEventRecord(c->ev[0], st));
    HIP_OK(cmp_analyze(p, &c->cmp_tmp, &c->cmp_tmp_bytes, st));
    int64_t n_ent = 0;
    { int rc_ = d2h_small(c, &n_ent, p.col_off + nc, 8, st); if (rc_) return rc_; }
    { int rc_ = sync_small(c, st); if (rc_) return rc_; }
    if (n_ent >= kLim) return fail(TSDB_E_NOT_IMPLEMENTED, "more than 2^31 datapoints in one compaction chunk");
    p.n_ent = n_ent;
    HIP_OK(d_rq.ensure(r1c * 8));
    HIP_OK(d_rv.ensure(r1c * 8));
    HIP_OK(d_rstate.ensure(r1c * 4));
    HIP_OK(d_rmeta.ensure(r1c));
    p.row_q = d_rq.as<int64_t>();
    p.row_v = d_rv.as<int64_t>();
    p.row_state = d_rstate.as<int32_t>();
    p.row_meta = d_rmeta.as<uint8_t>();
    row_cap[k] = 0;
    if (rows_ok) {
      hipError_t he = hipSuccess;
      row_cap[k] = cmp_row_cap(p, d_rmax.as<uint32_t>(), st, &he, &row_span[k]);
      HIP_OK(he);
    }
    if (row_cap[k]) {
      HIP_OK(d_rlo.ensure(r1c * 8));
      HIP_OK(d_klist.ensure(std::max<int64_t>(1, n_ent) * 16));
      p.row_lo = d_rlo.as<int64_t>();
      HIP_OK(cmp_rows_fused(p, d_klist.p, row_cap[k], row_span[k], false, st));
    } else {
    const int64_t E1 = std::max<int64_t>(1, n_ent);
    HIP_OK(d_key.ensure(E1 * 8));
    HIP_OK(d_key2.ensure(E1 * 8));
    HIP_OK(d_idx.ensure(E1 * 4));
    HIP_OK(d_idx2.ensure(E1 * 4));
    HIP_OK(d_ecol.ensure(E1 * 4));
    HIP_OK(d_eqo.ensure(E1 * 4));
    HIP_OK(d_evo.ensure(E1 * 4));
    HIP_OK(d_klen.ensure(E1 * 4));
    for (DevBuf* b : {&d_sq, &d_sv, &d_sc, &d_sm}) HIP_OK(b->ensure((E1 + 1) * 8));
    HIP_OK(d_rlo.ensure(r1c * 8));
    p.key = d_key.as<uint64_t>();
    p.key2 = d_key2.as<uint64_t>();
    p.idx = d_idx.as<uint32_t>();
    p.idx2 = d_idx2.as<uint32_t>();
    p.ent_col = d_ecol.as<uint32_t>();
    p.ent_qo = d_eqo.as<uint32_t>();
    p.ent_vo = d_evo.as<uint32_t>();
    p.klen = d_klen.as<uint32_t>();
    p.sq = d_sq.as<int64_t>();
    p.sv = d_sv.as<int64_t>();
    p.sc = d_sc.as<int64_t>();
    p.sm = d_sm.as<int64_t>();
    p.row_lo = d_rlo.as<int64_t>();
    int rb = 1;
    while (((int64_t)1 << rb) <= nr) rb++;
    HIP_OK(cmp_entries(p, &c->cmp_tmp, &c->cmp_tmp_bytes, std::min(64, 22 + rb), st));
    }
    HIP_OK(hipEventRecord(c->ev[2], st));
    if (nr) {
      HIP_OK(hipMemcpyAsync(rq.data() + r0, p.row_q, nr * 8, hipMemcpyDeviceToHost, st));
      HIP_OK(hipMemcpyAsync(rv.data() + r0, p.row_v, nr * 8, hipMemcpyDeviceToHost, st));
      HIP_OK(hipMemcpyAsync(rstate.data() + r0, p.row_state, nr * 4, hipMemcpyDeviceToHost, st));
      HIP_OK(hipMemcpyAsync(rerr.data() + r0, p.row_err, nr * 4, hipMemcpyDeviceToHost, st));
    }
    HIP_OK(hipStreamSynchronize(st));
    float t = 0;
    (void)hipEventElapsedTime(&t, c->ev[0], c->ev[2]);
    cmp_ms += t;
    return 0;
  };
  // chunk k (prepared last) to the resident blob at the host's layout
  auto write = [&](int k) -> int {
    const int64_t r0 = cuts[k], nr = cuts[k + 1] - r0;
    HIP_OK(d_rdq.ensure(std::max<int64_t>(1, nr) * 8));
    HIP_OK(d_rdv.ensure(std::max<int64_t>(1, nr) * 8));
    if (nr) {
      HIP_OK(hipMemcpyAsync(d_rdq.p, rdq.data() + r0, nr * 8, hipMemcpyHostToDevice, st));
      HIP_OK(hipMemcpyAsync(d_rdv.p, rdv.data() + r0, nr * 8, hipMemcpyHostToDevice, st));
    }
    p.row_dq = d_rdq.as<int64_t>();
    p.row_dv = d_rdv.as<int64_t>();
    p.out_q = c->qual.as<uint8_t>();
    p.out_v = c->val.as<uint8_t>();
    HIP_OK(hipEventRecord(c->ev[3], st));
    if (row_cap[k]) HIP_OK(cmp_rows_fused(p, d_klist.p, row_cap[k], row_span[k], true, st));
    else HIP_OK(cmp_write(p, st));
    HIP_OK(hipEventRecord(c->ev[1], st));
    HIP_OK(hipStreamSynchronize(st));
    float t = 0;
    (void)hipEventElapsedTime(&t, c->ev[3], c->ev[1]);
    cmp_ms += t;
    return 0;
  };
  // resident layout: series stable-sorted by group, each series' kept rows by base time
  std::vector<int64_t> order(NS);
  int32_t maxg = -1;
  for (int64_t s = 0; s < NS; s++) { order[s] = s; maxg = std::max(maxg, cb->group_id[s]); }
  auto gkey = [&](int64_t s) { const int32_t g = cb->group_id[s]; return g < 0 ? INT32_MAX : g; };
  std::stable_sort(order.begin(), order.end(), [&](int64_t x, int64_t y) { return gkey(x) < gkey(y); });
  // One chunk whose rows all fit a block: the one-pass path.  k_cmp_cols sums every row's
  // datapoints and byte bounds; the host lays the rows out from the bounds (the layout below, with
  // each row's region reserved whether or not it keeps a cell); k_cmp_rowone compacts every row
  // straight into its region.  TSDBHIP_CMP_ONEPASS=0: the sizing pass + write pass below.
  uint64_t op_qtot = 0, op_vtot = 0;
  auto onepass = [&]() -> int {   // 0: compacted in place, 1: not taken (nothing kept), < 0: error
    const int64_t nr = NR, nc = NC;
    const uint64_t qz = nc ? cb->col_qual_off[nc] : 0, vz = nc ? cb->col_val_off[nc] : 0;
    const int64_t r1c = std::max<int64_t>(1, nr), c1c = std::max<int64_t>(1, nc);
    HIP_OK(d_rcp.ensure((r1c + 1) * 8));
    HIP_OK(d_cqo.ensure((c1c + 1) * 8));
    HIP_OK(d_cvo.ensure((c1c + 1) * 8));
    HIP_OK(d_q.ensure(std::max<uint64_t>(16, qz) + 16));
    HIP_OK(d_v.ensure(std::max<uint64_t>(16, vz) + 16));
    if (cb->col_timestamp) HIP_OK(d_cts.ensure(c1c * 8));
    HIP_OK(d_raw.ensure((std::max(r1c, c1c) + 1) * 8));
    HIP_OK(hipMemsetAsync(d_bad.p, 0, 4, st));
    if (nr) {   // (rebase 0: the monotonicity check; the offsets are used as given)
      HIP_OK(hipMemcpyAsync(d_raw.p, cb->row_col_ptr, (nr + 1) * 8, hipMemcpyHostToDevice, st));
      HIP_OK(cmp_rebase(d_raw.as<uint64_t>(), d_rcp.as<uint64_t>(), nr + 1, 0, d_bad.as<int32_t>(), st));
    }
    // 32-bit copies of the column offsets when the blobs are under 4 GB (written by the same
    // checking pass; the one-pass kernels read 4 bytes an offset instead of 8)
    mark("onepass alloc");
    const bool w32 = nc && qz < ((uint64_t)1 << 32) && vz < ((uint64_t)1 << 32);
    if (w32) {
      HIP_OK(d_cq32.ensure((c1c + 1) * 4));
      HIP_OK(d_cv32.ensure((c1c + 1) * 4));
    }
    if (nc) {
      HIP_OK(h2d(c, d_raw.p, cb->col_qual_off, (nc + 1) * 8, st));
      HIP_OK(cmp_rebase(d_raw.as<uint64_t>(), d_cqo.as<uint64_t>(), nc + 1, 0, d_bad.as<int32_t>(), st,
                        w32 ? d_cq32.as<uint32_t>() : nullptr));
      HIP_OK(h2d(c, d_raw.p, cb->col_val_off, (nc + 1) * 8, st));
      HIP_OK(cmp_rebase(d_raw.as<uint64_t>(), d_cvo.as<uint64_t>(), nc + 1, 0, d_bad.as<int32_t>(), st,
                        w32 ? d_cv32.as<uint32_t>() : nullptr));
      if (qz) HIP_OK(h2d(c, d_q.p, cb->qual, qz, st));
      if (vz) HIP_OK(h2d(c, d_v.p, cb->val, vz, st));
      if (cb->col_timestamp) HIP_OK(h2d(c, d_cts.p, cb->col_timestamp, nc * 8, st));
    }
    int32_t bad = 0;
    { int rc_ = d2h_small(c, &bad, d_bad.p, 4, st); if (rc_) return rc_; }
    { int rc_ = sync_small(c, st); if (rc_) return rc_; }
    mark("onepass H2D");
    if (bad) return fail(TSDB_E_ILLEGAL_ARGUMENT, "column offsets not monotonic");
    HIP_OK(d_crow.ensure(c1c * 4));
    HIP_OK(d_cn.ensure(c1c * 8));
    HIP_OK(d_cinfo.ensure(c1c * 4));
    for (DevBuf* b : {&d_rheap, &d_rerr}) HIP_OK(b->ensure(r1c * 4));
    for (DevBuf* b : {&d_rone, &d_rlo, &d_rq, &d_rv, &d_sq, &d_sv, &d_sc}) HIP_OK(b->ensure(r1c * 8));
    HIP_OK(d_rstate.ensure(r1c * 4));
    HIP_OK(d_rmeta.ensure(r1c));
    HIP_OK(hipMemsetAsync(d_rheap.p, 0, r1c * 4, st));
    HIP_OK(hipMemsetAsync(d_rone.p, 0, r1c * 8, st));
    HIP_OK(hipMemsetAsync(d_rerr.p, 0, r1c * 4, st));
    for (DevBuf* b : {&d_sq, &d_sv, &d_sc}) HIP_OK(hipMemsetAsync(b->p, 0, r1c * 8, st));
    p.n_rows = nr;
    p.n_cols = nc;
    p.row_col_ptr = d_rcp.as<int64_t>();
    p.col_qo = d_cqo.as<uint64_t>();
    p.col_vo = d_cvo.as<uint64_t>();
    p.col_qo32 = w32 ? d_cq32.as<uint32_t>() : nullptr;
    p.col_vo32 = w32 ? d_cv32.as<uint32_t>() : nullptr;
    p.col_ts = cb->col_timestamp ? d_cts.as<int64_t>() : nullptr;
    p.q = d_q.as<uint8_t>();
    p.v = d_v.as<uint8_t>();
    p.col_row = d_crow.as<int32_t>();
    p.col_n = d_cn.as<int64_t>();
    p.col_off = nullptr;
    p.col_info = d_cinfo.as<uint32_t>();
    p.row_heap = d_rheap.as<int32_t>();
    p.row_one = d_rone.as<int64_t>();
    p.row_err = d_rerr.as<int32_t>();
    p.row_n = d_sc.as<int64_t>();
    p.row_qb = d_sq.as<int64_t>();
    p.row_vb = d_sv.as<int64_t>();
    p.row_lo = d_rlo.as<int64_t>();
    p.row_q = d_rq.as<int64_t>();
    p.row_v = d_rv.as<int64_t>();
    p.row_state = d_rstate.as<int32_t>();
    p.row_meta = d_rmeta.as<uint8_t>();
    HIP_OK(hipEventRecord(c->ev[0], st));
    HIP_OK(cmp_cols_rows(p, st));
    HIP_OK(hipEventRecord(c->ev[2], st));
    hipError_t he = hipSuccess;
    const int cap = cmp_onepass_cap(p, d_rmax.as<uint32_t>(), st, &he);   // (synchronises)
    HIP_OK(he);
    mark("onepass cols");
    float t_cols = 0;
    (void)hipEventElapsedTime(&t_cols, c->ev[0], c->ev[2]);
    if (!cap) {
      p.row_n = p.row_qb = p.row_vb = nullptr;
      p.col_qo32 = p.col_vo32 = nullptr;
      return 1;
    }
    std::vector<int64_t> qbv(r1c, 0), vbv(r1c, 0);
    if (nr) {
      HIP_OK(hipMemcpyAsync(qbv.data(), p.row_qb, nr * 8, hipMemcpyDeviceToHost, st));
      HIP_OK(hipMemcpyAsync(vbv.data(), p.row_vb, nr * 8, hipMemcpyDeviceToHost, st));
    }
    HIP_OK(hipStreamSynchronize(st));
    // regions: series in resident order, each series' rows by base time; rows of one base time
    // (salt buckets) adjacent, with 16 more bytes for the merged cell's meta byte
    uint64_t qt = 0, vt = 0;
    for (int64_t i = 0; i < NS; i++) {
      const int64_t s = order[i];
      std::vector<int64_t> rows;
      for (int64_t r = cb->series_row_ptr[s]; r < cb->series_row_ptr[s + 1]; r++) rows.push_back(r);
      std::stable_sort(rows.begin(), rows.end(), [&](int64_t x, int64_t y) { return cb->row_base_time[x] < cb->row_base_time[y]; });
      for (size_t k0 = 0; k0 < rows.size();) {
        size_t k1 = k0 + 1;
        while (k1 < rows.size() && cb->row_base_time[rows[k1]] == cb->row_base_time[rows[k0]]) k1++;
        for (size_t k = k0; k < k1; k++) {
          const int64_t r = rows[k];
          rdq[r] = (int64_t)qt;
          rdv[r] = (int64_t)vt;
          qt += align16((uint64_t)qbv[r]);
          vt += align16((uint64_t)vbv[r] + 1);
        }
        if (k1 - k0 > 1) vt += 16;
        k0 = k1;
      }
    }
    op_qtot = qt;
    op_vtot = vt;
    mark("onepass layout");
    HIP_OK(c->qual.ensure(qt + BLOB_SLACK));
    HIP_OK(c->val.ensure(vt + BLOB_SLACK));
    HIP_OK(hipMemsetAsync(c->qual.p, 0, qt + BLOB_SLACK, st));
    HIP_OK(hipMemsetAsync(c->val.p, 0, vt + BLOB_SLACK, st));
    HIP_OK(d_rdq.ensure(r1c * 8));
    HIP_OK(d_rdv.ensure(r1c * 8));
    if (nr) {
      HIP_OK(hipMemcpyAsync(d_rdq.p, rdq.data(), nr * 8, hipMemcpyHostToDevice, st));
      HIP_OK(hipMemcpyAsync(d_rdv.p, rdv.data(), nr * 8, hipMemcpyHostToDevice, st));
    }
    p.row_dq = d_rdq.as<int64_t>();
    p.row_dv = d_rdv.as<int64_t>();
    p.out_q = c->qual.as<uint8_t>();
    p.out_v = c->val.as<uint8_t>();
    HIP_OK(hipEventRecord(c->ev[3], st));
    HIP_OK(cmp_rows_onepass(p, cap, st));
    HIP_OK(hipEventRecord(c->ev[1], st));
    if (nr) {
      HIP_OK(hipMemcpyAsync(rq.data(), p.row_q, nr * 8, hipMemcpyDeviceToHost, st));
      HIP_OK(hipMemcpyAsync(rv.data(), p.row_v, nr * 8, hipMemcpyDeviceToHost, st));
      HIP_OK(hipMemcpyAsync(rstate.data(), p.row_state, nr * 4, hipMemcpyDeviceToHost, st));
      HIP_OK(hipMemcpyAsync(rerr.data(), p.row_err, nr * 4, hipMemcpyDeviceToHost, st));
    }
    HIP_OK(hipStreamSynchronize(st));
    mark("onepass rows");
    float t_rows = 0;
    (void)hipEventElapsedTime(&t_rows, c->ev[3], c->ev[1]);
    cmp_ms = t_cols + t_rows;
    return 0;
  };
  int op = 1;
  {
    if (n_chunks == 1 && rows_ok && !opt_off(OPT_CMP_ONEPASS)) {
      op = onepass();
      if (op < 0) return op;
    }
  }
  if (op)
    for (int k = 0; k < n_chunks; k++)
      if (int rc = prepare(k)) return rc;
  mark("upload+entries");
  std::vector<tsdbhip_ctx::CmpErr> errs;
  std::vector<int64_t> srp(NS + 1, 0);
  std::vector<RowDesc> rd;
  std::vector<int32_t> hgroup(NS);
  // Rows of one series with the same base time (salt buckets): Span.addRow merges the second
  // compacted row into the first (RowSeq.addRow, src/core/Span.java:202-219).  Such rows are
  // compacted into consecutive slots of one region and merged there afterwards; the merged row
  // is never longer than the region (plus 16 bytes for a meta byte).
  struct SaltGroup { size_t rd_index; std::vector<int64_t> rows; };
  std::vector<SaltGroup> salt;
  uint64_t qtot = 0, vtot = 0;
  for (int64_t i = 0; i < NS; i++) {
    const int64_t s = order[i];
    hgroup[i] = cb->group_id[s] < 0 ? maxg + 1 : cb->group_id[s];
    std::vector<int64_t> rows;
    for (int64_t r = cb->series_row_ptr[s]; r < cb->series_row_ptr[s + 1]; r++) {
      if (rerr[r]) errs.push_back({s, r, (int64_t)cb->row_base_time[r], rerr[r]});
      else if (rstate[r] != 0) rows.push_back(r);
    }
    std::stable_sort(rows.begin(), rows.end(), [&](int64_t x, int64_t y) { return cb->row_base_time[x] < cb->row_base_time[y]; });
    for (size_t k0 = 0; k0 < rows.size();) {
      size_t k1 = k0 + 1;
      while (k1 < rows.size() && cb->row_base_time[rows[k1]] == cb->row_base_time[rows[k0]]) k1++;
      RowDesc d{};
      d.base = cb->row_base_time[rows[k0]];
      d.qoff = op ? qtot : (uint64_t)rdq[rows[k0]];   // (one-pass: the regions laid out before the kernel)
      d.voff = op ? vtot : (uint64_t)rdv[rows[k0]];
      uint64_t ql = 0, vl = 0;
      for (size_t k = k0; k < k1; k++) {
        const int64_t r = rows[k];
        if (rq[r] > 0xFFFFFFFFLL || rv[r] > 0xFFFFFFFFLL) return fail(TSDB_E_ILLEGAL_ARGUMENT, "row too large");
        if (op) {
          rdq[r] = (int64_t)qtot;
          rdv[r] = (int64_t)vtot;
          qtot += align16(rq[r]);
          vtot += align16(rv[r]);
        }
        ql += rq[r];
        vl += rv[r];
      }
      if (ql > 0xFFFFFFFFull || vl > 0xFFFFFFFFull) return fail(TSDB_E_ILLEGAL_ARGUMENT, "row too large");
      d.qlen = (uint32_t)rq[rows[k0]];
      d.vlen = (uint32_t)rv[rows[k0]];
      if (k1 - k0 > 1) {
        if (op) vtot += 16;   // the merged cell's meta byte (two single-datapoint cells become a compacted one)
        salt.push_back({rd.size(), std::vector<int64_t>(rows.begin() + k0, rows.begin() + k1)});
      }
      if (rd.size() == (size_t)srp[i]) d.flags |= ROW_SFIRST;
      rd.push_back(d);
      k0 = k1;
    }
    srp[i + 1] = (int64_t)rd.size();
  }
  std::sort(errs.begin(), errs.end(), [](const tsdbhip_ctx::CmpErr& a, const tsdbhip_ctx::CmpErr& b) {
    return a.series != b.series ? a.series < b.series : a.row < b.row;
  });
  // the compacted cells, written in place
  if (!op) {
    qtot = op_qtot;
    vtot = op_vtot;
  } else {
    HIP_OK(c->qual.ensure(qtot + BLOB_SLACK));
    HIP_OK(c->val.ensure(vtot + BLOB_SLACK));
    HIP_OK(hipMemsetAsync(c->qual.p, 0, qtot + BLOB_SLACK, c->stream));
    HIP_OK(hipMemsetAsync(c->val.p, 0, vtot + BLOB_SLACK, c->stream));
  }
  mark("host layout");
  if (!op) {
  } else if (n_chunks == 1) {
    if (int rc = write(0)) return rc;
  } else {
    for (int k = 0; k < n_chunks; k++) {
      if (int rc = prepare(k)) return rc;
      if (int rc = write(k)) return rc;
    }
  }
  for (const SaltGroup& sg : salt) {   // RowSeq.addRow of each later row, in scan order
    std::vector<uint8_t> lq, lv, q2, v2;
    bool ok = true;
    for (size_t k = 0; k < sg.rows.size() && ok; k++) {
      const int64_t r = sg.rows[k];
      std::vector<uint8_t>& tq = k ? q2 : lq;
      std::vector<uint8_t>& tv = k ? v2 : lv;
      tq.resize(rq[r]);
      tv.resize(rv[r]);
      if (rq[r]) HIP_OK(hipMemcpy(tq.data(), c->qual.as<uint8_t>() + rdq[r], rq[r], hipMemcpyDeviceToHost));
      if (rv[r]) HIP_OK(hipMemcpy(tv.data(), c->val.as<uint8_t>() + rdv[r], rv[r], hipMemcpyDeviceToHost));
      if (k) ok = merge_cells(lq, lv, q2.data(), q2.size(), v2.data(), v2.size());
    }
    if (!ok)
      return fail(TSDB_E_NOT_IMPLEMENTED, "salt-bucket rows of one series whose compacted cells do not merge (RowSeq.addRow)");
    RowDesc& d = rd[sg.rd_index];
    if (!lq.empty()) HIP_OK(hipMemcpy(c->qual.as<uint8_t>() + d.qoff, lq.data(), lq.size(), hipMemcpyHostToDevice));
    if (!lv.empty()) HIP_OK(hipMemcpy(c->val.as<uint8_t>() + d.voff, lv.data(), lv.size(), hipMemcpyHostToDevice));
    d.qlen = (uint32_t)lq.size();
    d.vlen = (uint32_t)lv.size();
  }
  // resident batch state (as load_impl)
  c->n_series = NS;
  c->n_groups = maxg + 1;
  c->h_group = hgroup;
  c->h_orig = order;
  c->h_srp = srp;
  c->max_series_rows = 0;
  for (int64_t s = 0; s < NS; s++) c->max_series_rows = std::max<int64_t>(c->max_series_rows, srp[s + 1] - srp[s]);
  c->n_rows = (int64_t)rd.size();
  c->qual_bytes = qtot;
  c->val_bytes = vtot;
  HIP_OK(c->rows.ensure(std::max<size_t>(1, rd.size()) * sizeof(RowDesc)));
  HIP_OK(c->srp.ensure((NS + 1) * 8));
  HIP_OK(c->gid.ensure(std::max<int64_t>(1, NS) * 4));
  if (!rd.empty()) HIP_OK(hipMemcpy(c->rows.p, rd.data(), rd.size() * sizeof(RowDesc), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(c->srp.p, srp.data(), (NS + 1) * 8, hipMemcpyHostToDevice));
  if (NS) HIP_OK(hipMemcpy(c->gid.p, hgroup.data(), NS * 4, hipMemcpyHostToDevice));
  mark("write+merge");
  const int rc = finish_load(c, rd);
  mark("finish_load");
  c->cmp_errs = std::move(errs);
  c->compact_ms = cmp_ms;
  return rc;
}

// ---- sharding a host batch over ranks ----------------------------------------
namespace {

// Contiguous byte-balanced split of n weights over `world` parts: bounds[r] = the first index
// whose cumulative weight reaches r / world of the total (numpy searchsorted 'left' over the
// cumulative sums), made monotone.
void balanced_bounds(const std::vector<double>& w, int world, int64_t* bounds) {
  const int64_t n = (int64_t)w.size();
  std::vector<double> cum(n + 1, 0.0);
  for (int64_t i = 0; i < n; i++) cum[i + 1] = cum[i] + w[i];
  const double total = cum[n];
  bounds[0] = 0;
  for (int r = 1; r < world; r++) {
    int64_t b;
    if (total > 0) b = std::lower_bound(cum.begin(), cum.end(), total * r / world) - cum.begin();
    else b = n * r / world;
    bounds[r] = std::max(b, bounds[r - 1]);
  }
  bounds[world] = n;
}

double series_bytes(const tsdbhip_batch* b, int64_t s) {
  const int64_t r0 = b->series_row_ptr[s], r1 = b->series_row_ptr[s + 1];
  return (double)(b->row_qual_off[r1] - b->row_qual_off[r0]) + (double)(b->row_val_off[r1] - b->row_val_off[r0]);
}

// kept series (group id >= 0) stably sorted by group: SpanGroup order
std::vector<int64_t> group_order(const tsdbhip_batch* b) {
  std::vector<int64_t> o;
  for (int64_t s = 0; s < b->n_series; s++) if (b->group_id[s] >= 0) o.push_back(s);
  std::stable_sort(o.begin(), o.end(), [&](int64_t x, int64_t y) { return b->group_id[x] < b->group_id[y]; });
  return o;
}

int check_batch_arrays(const tsdbhip_batch* b) {
  if (!b || b->n_series < 0) return fail(TSDB_E_ILLEGAL_ARGUMENT, "bad batch");
  if (b->n_series > 0 && (!b->series_row_ptr || !b->group_id || !b->row_qual_off || !b->row_val_off))
    return fail(TSDB_E_ILLEGAL_ARGUMENT, "null batch arrays");
  return 0;
}

}  // namespace

extern "C" int tsdbhip_shard_bounds(const tsdbhip_batch* b, int world, int mode, int64_t* bounds) {
  int rc = check_batch_arrays(b);
  if (rc) return rc;
  if (world < 1 || !bounds) return fail(TSDB_E_ILLEGAL_ARGUMENT, "world must be >= 1");
  std::vector<double> w;
  if (mode == TSDB_SHARD_SERIES) {
    for (int64_t s : group_order(b)) w.push_back(series_bytes(b, s));
  } else if (mode == TSDB_SHARD_GROUPS) {
    int32_t maxg = -1;
    for (int64_t s = 0; s < b->n_series; s++) maxg = std::max(maxg, b->group_id[s]);
    w.assign(maxg + 1, 0.0);
    for (int64_t s = 0; s < b->n_series; s++) if (b->group_id[s] >= 0) w[b->group_id[s]] += series_bytes(b, s);
  } else if (mode == TSDB_SHARD_SPANS) {
    for (int64_t s = 0; s < b->n_series; s++) w.push_back(series_bytes(b, s));   // every span (NONE)
  } else {
    return fail(TSDB_E_ILLEGAL_ARGUMENT, "bad shard mode");
  }
  balanced_bounds(w, world, bounds);
  return 0;
}

extern "C" int tsdbhip_load_shard(tsdbhip_ctx* c, const tsdbhip_batch* b, int mode, int64_t begin, int64_t end) {
  MD_REFUSE(c, "tsdbhip_load_shard");
  int rc = check_batch_arrays(b);
  if (rc) return rc;
  if (begin < 0 || end < begin) return fail(TSDB_E_ILLEGAL_ARGUMENT, "bad shard range");
  std::vector<int64_t> cand;
  if (mode == TSDB_SHARD_SERIES) {
    const std::vector<int64_t> o = group_order(b);
    if (end > (int64_t)o.size()) return fail(TSDB_E_ILLEGAL_ARGUMENT, "shard range past the series");
    cand.assign(o.begin() + begin, o.begin() + end);
  } else if (mode == TSDB_SHARD_GROUPS) {
    for (int64_t s : group_order(b)) if (b->group_id[s] >= begin && b->group_id[s] < end) cand.push_back(s);
  } else if (mode == TSDB_SHARD_SPANS) {
    if (end > b->n_series) return fail(TSDB_E_ILLEGAL_ARGUMENT, "shard range past the series");
    for (int64_t s = begin; s < end; s++) cand.push_back(s);
  } else {
    return fail(TSDB_E_ILLEGAL_ARGUMENT, "bad shard mode");
  }
  return load_with(c, b, &cand);
}

// Batch positions [p0, p1) of the synthetic store (series sorted by group; group g holds
// global series g, g + G, g + 2G, ...): one GPU's contiguous shard of the whole store.
static int synth_impl(tsdbhip_ctx* c, const tsdbhip_synth_spec* sp, int64_t p0, int64_t p1) {
  if (!c || !sp) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  CtxLock lk(c);
  HIP_OK(hipSetDevice(c->device));
  if (sp->n_series <= 0 || sp->n_points <= 0 || sp->period_ms <= 0 || sp->n_groups <= 0 || sp->start_s < 0)
    return fail(TSDB_E_ILLEGAL_ARGUMENT, "bad synth spec");
  if (p0 < 0 || p1 > sp->n_series || p0 >= p1) return fail(TSDB_E_ILLEGAL_ARGUMENT, "bad synth shard range");
  if (sp->value_kind != 0 && sp->int_mod <= 0) return fail(TSDB_E_ILLEGAL_ARGUMENT, "int_mod must be > 0");
  release_batch(c);
  const bool ms_qual = (sp->period_ms % 1000) != 0 || (sp->start_s * 1000) % 1000 != 0;
  const int qw = ms_qual ? 4 : 2;
  const int64_t start_ms = sp->start_s * 1000;
  // row template
  std::vector<int64_t> k0;
  std::vector<int32_t> rn;
  std::vector<uint32_t> rbase;
  for (int64_t k = 0; k < sp->n_points;) {
    const int64_t ts = start_ms + k * sp->period_ms;
    const int64_t base = (ts / 1000) - (ts / 1000) % 3600;
    int64_t e = k;
    while (e < sp->n_points && (start_ms + e * sp->period_ms) / 1000 - ((start_ms + e * sp->period_ms) / 1000) % 3600 == base) e++;
    k0.push_back(k);
    rn.push_back((int32_t)(e - k));
    rbase.push_back((uint32_t)base);
    k = e;
  }
  const int64_t R = (int64_t)k0.size();
  const int64_t SG = sp->n_series, G = sp->n_groups;   // the whole store
  const int64_t S = p1 - p0;                           // this shard
  std::vector<int64_t> grp_off(G + 1, 0);
  for (int64_t g = 0; g < G; g++) grp_off[g + 1] = grp_off[g] + SG / G + (g < SG % G ? 1 : 0);
  c->n_series = S;
  c->n_rows = S * R;
  c->n_groups = G;
  c->max_series_rows = S ? R : 0;
  // qualifier offsets (identical layout for every series)
  // row starts 16-byte aligned (a 128-B alignment moved k_hwin by 1 % and slowed k_rows / k_short by 3 %,
  // profiles/r05d)
  auto alignr = [](int64_t x) { return (x + 15) / 16 * 16; };
  std::vector<int64_t> rq(R);
  int64_t QS = 0;
  for (int64_t h = 0; h < R; h++) { rq[h] = QS; QS += alignr((int64_t)rn[h] * qw); }
  DevBuf d_k0, d_rn, d_rbase, d_goff, d_vbytes;
  HIP_OK(d_k0.ensure(R * 8));
  HIP_OK(d_rn.ensure(R * 4));
  HIP_OK(d_rbase.ensure(R * 4));
  HIP_OK(d_goff.ensure((G + 1) * 8));
  HIP_OK(hipMemcpy(d_k0.p, k0.data(), R * 8, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_rn.p, rn.data(), R * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_rbase.p, rbase.data(), R * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_goff.p, grp_off.data(), (G + 1) * 8, hipMemcpyHostToDevice));
  HIP_OK(c->gid.ensure(S * 4));
  SynthParams p{};
  p.n_series = S; p.n_groups = G; p.n_rows_per_series = R; p.n_points = sp->n_points; p.pos0 = p0;
  p.start_ms = start_ms; p.period_ms = sp->period_ms; p.value_kind = sp->value_kind; p.ms_qual = ms_qual;
  p.int_mod = sp->int_mod; p.seed = sp->seed;
  p.grp_off = d_goff.as<int64_t>(); p.row_k0 = d_k0.as<int64_t>(); p.row_n = d_rn.as<int32_t>();
  p.row_base = d_rbase.as<uint32_t>(); p.group_id = c->gid.as<int32_t>();
  // value bytes per row
  std::vector<uint32_t> vbytes;
  if (sp->value_kind == 0) {
    vbytes.resize(S * R);
    for (int64_t s = 0; s < S; s++)
      for (int64_t h = 0; h < R; h++) vbytes[s * R + h] = (uint32_t)(rn[h] * 4 + (rn[h] > 1 ? 1 : 0));
  } else {
    HIP_OK(d_vbytes.ensure(S * R * 4));
    p.row_vbytes = d_vbytes.as<uint32_t>();
    HIP_OK(launch_synth_sizes(p, c->stream));
    vbytes.resize(S * R);
    HIP_OK(hipMemcpyAsync(vbytes.data(), d_vbytes.p, S * R * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
  }
  std::vector<RowDesc> rd(S * R);
  uint64_t vtot = 0;
  for (int64_t s = 0; s < S; s++) {
    for (int64_t h = 0; h < R; h++) {
      RowDesc& d = rd[s * R + h];
      d.base = rbase[h];
      d.qoff = (uint64_t)(s * QS + rq[h]);
      d.qlen = (uint32_t)(rn[h] * qw);
      d.voff = vtot;
      d.vlen = vbytes[s * R + h];
      d.flags = h == 0 ? ROW_SFIRST : 0;
      vtot += alignr(d.vlen);
    }
  }
  c->qual_bytes = (uint64_t)(S * QS);
  c->val_bytes = vtot;
  HIP_OK(c->rows.ensure(rd.size() * sizeof(RowDesc)));
  HIP_OK(c->qual.ensure(c->qual_bytes + BLOB_SLACK));
  HIP_OK(c->val.ensure(c->val_bytes + BLOB_SLACK));
  HIP_OK(hipMemsetAsync(c->qual.p, 0, c->qual_bytes + BLOB_SLACK, c->stream));
  HIP_OK(hipMemsetAsync(c->val.p, 0, c->val_bytes + BLOB_SLACK, c->stream));
  HIP_OK(hipMemcpyAsync(c->rows.p, rd.data(), rd.size() * sizeof(RowDesc), hipMemcpyHostToDevice, c->stream));
  p.rows = c->rows.as<RowDesc>();
  p.qual = c->qual.as<uint8_t>();
  p.val = c->val.as<uint8_t>();
  HIP_OK(launch_synth_write(p, c->stream));
  c->h_srp.resize(S + 1);
  for (int64_t s = 0; s <= S; s++) c->h_srp[s] = s * R;
  HIP_OK(c->srp.ensure((S + 1) * 8));
  HIP_OK(hipMemcpyAsync(c->srp.p, c->h_srp.data(), (S + 1) * 8, hipMemcpyHostToDevice, c->stream));
  c->h_group.resize(S);
  c->h_orig.resize(S);
  for (int64_t g = 0; g < G; g++)
    for (int64_t i = std::max(grp_off[g], p0); i < std::min(grp_off[g + 1], p1); i++) c->h_group[i - p0] = (int32_t)g;
  std::iota(c->h_orig.begin(), c->h_orig.end(), 0);
  HIP_OK(hipStreamSynchronize(c->stream));
  return finish_load(c, rd);
}

extern "C" int tsdbhip_synth(tsdbhip_ctx* c, const tsdbhip_synth_spec* sp) {
  if (c && c->md) return tsdb::md_synth(c, sp);
  return synth_impl(c, sp, 0, sp ? sp->n_series : 0);
}

extern "C" int tsdbhip_synth_shard(tsdbhip_ctx* c, const tsdbhip_synth_spec* sp, int64_t pos_begin, int64_t pos_end) {
  MD_REFUSE(c, "tsdbhip_synth_shard");
  return synth_impl(c, sp, pos_begin, pos_end);
}

extern "C" int tsdbhip_batch_sizes(tsdbhip_ctx* c, int64_t* n_series, int64_t* n_rows, uint64_t* qual_bytes,
                                   uint64_t* val_bytes) {
  if (c && c->md) return tsdb::md_batch_sizes(c, n_series, n_rows, qual_bytes, val_bytes);
  if (c && c->ro_active) return fail(TSDB_E_NOT_IMPLEMENTED, "tsdbhip_batch_sizes over a rollup batch (tsdbhip_load_rollup)");
  if (!c) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null ctx");
  uint64_t q = 0, v = 0;
  for (int64_t r = 0; r < c->n_rows; r++) { q += c->h_qlen[r]; v += c->h_vlen[r]; }
  *n_series = c->n_series;
  *n_rows = c->n_rows;
  *qual_bytes = q;
  *val_bytes = v;
  return 0;
}

// Resident batch back to host in the tsdbhip_batch layout (series in resident order).
extern "C" int tsdbhip_batch_download(tsdbhip_ctx* c, int64_t* series_row_ptr, uint32_t* row_base_time,
                                      uint64_t* row_qual_off, uint64_t* row_val_off, uint8_t* qual, uint8_t* val,
                                      int32_t* group_id) {
  MD_REFUSE(c, "tsdbhip_batch_download");
  if (c && c->ro_active) return fail(TSDB_E_NOT_IMPLEMENTED, "tsdbhip_batch_download over a rollup batch (tsdbhip_load_rollup)");
  if (!c) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null ctx");
  CtxLock lk(c);
  HIP_OK(hipSetDevice(c->device));
  std::vector<RowDesc> rd(c->n_rows);
  if (c->n_rows) HIP_OK(hipMemcpy(rd.data(), c->rows.p, c->n_rows * sizeof(RowDesc), hipMemcpyDeviceToHost));
  std::vector<uint8_t> hq(c->qual.n), hv(c->val.n);
  HIP_OK(hipMemcpy(hq.data(), c->qual.p, c->qual.n, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(hv.data(), c->val.p, c->val.n, hipMemcpyDeviceToHost));
  uint64_t qo = 0, vo = 0;
  for (int64_t r = 0; r < c->n_rows; r++) {
    row_base_time[r] = rd[r].base;
    row_qual_off[r] = qo;
    row_val_off[r] = vo;
    std::memcpy(qual + qo, hq.data() + rd[r].qoff, rd[r].qlen);
    std::memcpy(val + vo, hv.data() + rd[r].voff, rd[r].vlen);
    qo += rd[r].qlen;
    vo += rd[r].vlen;
  }
  row_qual_off[c->n_rows] = qo;
  row_val_off[c->n_rows] = vo;
  for (int64_t s = 0; s <= c->n_series; s++) series_row_ptr[s] = c->h_srp[s];
  for (int64_t s = 0; s < c->n_series; s++) group_id[s] = c->h_group[s] >= c->n_groups ? -1 : c->h_group[s];
  return 0;
}

// Sizes of resident series positions [s0, s1) in the tsdbhip_batch layout.
extern "C" int tsdbhip_batch_range_sizes(tsdbhip_ctx* c, int64_t s0, int64_t s1, int64_t* n_rows, uint64_t* qual_bytes,
                                         uint64_t* val_bytes) {
  MD_REFUSE(c, "tsdbhip_batch_range_sizes");
  if (!c) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null ctx");
  if (c->ro_active) return fail(TSDB_E_NOT_IMPLEMENTED, "tsdbhip_batch_range_sizes over a rollup batch");
  CtxLock lk(c);
  if (s0 < 0 || s1 < s0 || s1 > c->n_series) return fail(TSDB_E_ILLEGAL_ARGUMENT, "series range out of bounds");
  const int64_t r0 = c->h_srp[s0], r1 = c->h_srp[s1];
  uint64_t q = 0, v = 0;
  for (int64_t r = r0; r < r1; r++) { q += c->h_qlen[r]; v += c->h_vlen[r]; }
  if (n_rows) *n_rows = r1 - r0;
  if (qual_bytes) *qual_bytes = q;
  if (val_bytes) *val_bytes = v;
  return 0;
}

// Resident series positions [s0, s1) back to host in the tsdbhip_batch layout (offsets from 0).
// Only the blob span those rows occupy crosses PCIe, so a slice of a store far larger than host
// memory can be checked.  Any output pointer may be null (that part is skipped).
extern "C" int tsdbhip_batch_download_range(tsdbhip_ctx* c, int64_t s0, int64_t s1, int64_t* series_row_ptr,
                                            uint32_t* row_base_time, uint64_t* row_qual_off, uint64_t* row_val_off,
                                            uint8_t* qual, uint8_t* val, int32_t* group_id) {
  MD_REFUSE(c, "tsdbhip_batch_download_range");
  if (!c) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null ctx");
  if (c->ro_active) return fail(TSDB_E_NOT_IMPLEMENTED, "tsdbhip_batch_download_range over a rollup batch");
  CtxLock lk(c);
  if (s0 < 0 || s1 < s0 || s1 > c->n_series) return fail(TSDB_E_ILLEGAL_ARGUMENT, "series range out of bounds");
  HIP_OK(hipSetDevice(c->device));
  const int64_t r0 = c->h_srp[s0], r1 = c->h_srp[s1], nr = r1 - r0;
  if (series_row_ptr)
    for (int64_t s = s0; s <= s1; s++) series_row_ptr[s - s0] = c->h_srp[s] - r0;
  if (group_id)
    for (int64_t s = s0; s < s1; s++) group_id[s - s0] = c->h_group[s] >= c->n_groups ? -1 : c->h_group[s];
  if (!row_base_time && !row_qual_off && !row_val_off && !qual && !val) return 0;
  std::vector<RowDesc> rd(nr);
  if (nr) HIP_OK(hipMemcpy(rd.data(), (const RowDesc*)c->rows.p + r0, nr * sizeof(RowDesc), hipMemcpyDeviceToHost));
  // the blob spans of the rows (rows of consecutive positions are laid out in order, but the
  // span is taken from the descriptors, whatever the layout)
  uint64_t qlo = UINT64_MAX, qhi = 0, vlo = UINT64_MAX, vhi = 0;
  for (const RowDesc& d : rd) {
    qlo = std::min<uint64_t>(qlo, d.qoff); qhi = std::max<uint64_t>(qhi, d.qoff + d.qlen);
    vlo = std::min<uint64_t>(vlo, d.voff); vhi = std::max<uint64_t>(vhi, d.voff + d.vlen);
  }
  std::vector<uint8_t> hq, hv;
  if (qual && qhi > qlo) {
    hq.resize(qhi - qlo);
    HIP_OK(hipMemcpy(hq.data(), (const uint8_t*)c->qual.p + qlo, qhi - qlo, hipMemcpyDeviceToHost));
  }
  if (val && vhi > vlo) {
    hv.resize(vhi - vlo);
    HIP_OK(hipMemcpy(hv.data(), (const uint8_t*)c->val.p + vlo, vhi - vlo, hipMemcpyDeviceToHost));
  }
  uint64_t qo = 0, vo = 0;
  for (int64_t i = 0; i < nr; i++) {
    const RowDesc& d = rd[i];
    if (row_base_time) row_base_time[i] = d.base;
    if (row_qual_off) row_qual_off[i] = qo;
    if (row_val_off) row_val_off[i] = vo;
    if (qual && d.qlen) std::memcpy(qual + qo, hq.data() + (d.qoff - qlo), d.qlen);
    if (val && d.vlen) std::memcpy(val + vo, hv.data() + (d.voff - vlo), d.vlen);
    qo += d.qlen;
    vo += d.vlen;
  }
  if (row_qual_off) row_qual_off[nr] = qo;
  if (row_val_off) row_val_off[nr] = vo;
  return 0;
}

// Test hook: sampled-window select runs and fall-backs (sel_window).
extern "C" int tsdbhip_debug_sel_window(tsdbhip_ctx* c, int64_t* runs, int64_t* misses) {
  MD_REFUSE(c, "tsdbhip_debug_sel_window");
  if (!c) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null ctx");
  CtxLock lk(c);
  if (runs) *runs = c->win_runs;
  if (misses) *misses = c->win_misses;
  return 0;
}

// Test hook: the per-row facts k_index derived (RowDesc.ndp / flags / lsb / absmax).
extern "C" int tsdbhip_debug_rows(tsdbhip_ctx* c, uint32_t* ndp, uint32_t* flags, int32_t* lsb, double* absmax) {
  MD_REFUSE(c, "tsdbhip_debug_rows");
  if (!c) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null ctx");
  CtxLock lk(c);
  HIP_OK(hipSetDevice(c->device));
  std::vector<RowDesc> rd(c->n_rows);
  if (c->n_rows) HIP_OK(hipMemcpy(rd.data(), c->rows.p, c->n_rows * sizeof(RowDesc), hipMemcpyDeviceToHost));
  for (int64_t r = 0; r < c->n_rows; r++) {
    if (ndp) ndp[r] = rd[r].ndp;
    if (flags) flags[r] = rd[r].flags;
    if (lsb) lsb[r] = rd[r].lsb;
    if (absmax) absmax[r] = rd[r].absmax;
  }
  return 0;
}

// ===========================================================================
// query execution
// ===========================================================================
namespace {

struct Plan {
  int ga = 0, f = 0, interp = 0;
  int mode = MODE_GRID;
  int64_t ss = 0, se = 0, B0 = 0, I = 1, K = 0;
  bool none = false;
  bool gslot = false;
  bool raw = false;   // no downsampling: AggregationIterator over the raw timestamp union
  int gsel = 0;       // TSDB_AGG_* when the group-by aggregator is a percentile / median (0: none)
  bool no_inf = false;   // per-span pass feeding the percentile group-by: no +-Inf check
  bool dense_out = false;   // grid kernels write per-series bucket values to pre_dense / pre_pres
  bool sel_direct = false;  // grid kernels write percentile group-by contributions (GridParams.sel_direct)
  std::vector<int64_t> bounds;   // MODE_TABLE: K + 1 calendar slot boundaries (ms)
  int64_t seek = 0;              // MODE_TABLE: first timestamp the spans' Downsamplers read
  bool ordered = false;          // TSDB_QF_ORDERED float reduction: run_ordered
  bool values_only = false;      // percentile downsampling pass without the group-by step
  bool emit_only = false;        // group-by step over bucket values already in pre_dense / pre_pres
  bool split2 = false;           // ... the second pass of a dense split (or after a rollup's staged pass): the first pass's timing stands
  bool seq_dense = false;        // sum / avg buckets in Java's order first (k_seq_dense), then the group-by step
  int ro_fuse = 0;               // rollup avg (1) / count (2) stage: value rows with their count rows (k_seq_rows_ro)
  bool sel_cols = false;         // sel_direct in the (group, slot) column layout
  bool sel_win = false;          // sel_direct through the sampled window (k_short KR 5, sel_window)
  bool multi = false;            // fused multi-aggregator pass (run_multi_fused): partials to c->mp*, no reduce
  bool multi_dev = false;        //   ... with the Welford state (a dev query among them)
  // calendar grids anchored per span that disagree (plan_calendar): each anchor's boundary
  // sequence; run_anchored downsamples every span on its own and aggregates over the union
  bool anchored = false;
  std::vector<int64_t> anchors;
  std::vector<std::vector<int64_t>> seqs;
  std::vector<int64_t> fillseq;   // anchored + fill: previousInterval(start) .. previousInterval(end)
};

bool is_sel_agg(int a) { return a == TSDB_AGG_MEDIAN || (a >= TSDB_AGG_P999 && a < TSDB_AGG_COUNT_ALL); }

// A calendar interval in a time zone, or one anchored per span (DateTime.previousInterval of the
// span's first datapoint: 7sc, 2dc, 5nc, 2wc, 2yc ...), as a MODE_TABLE slot table.  Every
// span's Downsampler seeks to the first boundary at or after the scan start
// (Downsampler.seekInterval :415-437), anchors at previousInterval(its first datapoint there)
// (:336-350) and steps by the interval (:388-406); a FillingDownsampler emits from
// previousInterval(start) to previousInterval(end) (FillingDownsampler.java:113-135).  The
// slots are the union of those boundary sequences, provided they agree where they overlap --
// always for days, weeks, n months (12 % n == 0) and years, which step on the local calendar,
// and for ms / s / m / h lattices when the zone's offsets in range are congruent modulo the
// step; otherwise the anchors come from each series' first datapoint (k_first_ts), and spans on
// grids that disagree run per anchor and aggregate over the union of their timestamps
// (run_anchored: the raw union evaluator, fills included).
// DateTime.previousInterval of every first datapoint f[i] (sorted; INT64_MAX = the series has
// none, anchor INT64_MAX).  Datapoints with the same jcal_top inside one step of that top's walk
// share its anchor, so the walk runs once per such step.
void anchors_of(const JZone& Z, int64_t n, int unit, const std::vector<int64_t>& f, std::vector<int64_t>& a) {
  a.assign(f.size(), INT64_MAX);
  int64_t top = INT64_MIN, lo = INT64_MAX, hi = INT64_MIN, cur = 0;
  for (size_t i = 0; i < f.size(); i++) {
    const int64_t t = f[i];
    if (t == INT64_MAX) break;
    int64_t tp, io;
    int uo;
    jcal_top(Z, t, n, unit, tp, uo, io);
    if (!(tp == top && t >= lo && t < hi)) {
      jcal_prev(Z, t, n, unit, cur);
      top = tp;
      lo = cur;
      hi = jcal_add(Z, cur, uo, io);
    }
    a[i] = cur;
  }
}

int plan_calendar(tsdbhip_ctx* c, const tsdbhip_query* q, Plan& P) {
  const int unit = q->ds_calendar;
  if (unit < TSDB_CAL_MS || unit > TSDB_CAL_Y) return fail(TSDB_E_ILLEGAL_ARGUMENT, "Unrecognized unit type");
  const int64_t n = q->ds_interval_ms / CAL_UNIT_MS[unit];
  if (n < 1 || n * CAL_UNIT_MS[unit] != q->ds_interval_ms || n > (1 << 30))
    return fail(TSDB_E_ILLEGAL_ARGUMENT, "calendar interval is not a whole number of units");
  const JZone Z{q->ds_tz};
  const int64_t S0 = P.ss * 1000, E0 = P.se * 1000;
  const bool fill = q->ds_fill != TSDB_FILL_NONE;
  // cache: the plan depends on the interval, the scan range, the fill, the zone and the batch
  std::vector<int64_t> key = {unit, n, S0, E0, fill ? 1 : 0, q->ds_tz ? 1 : 0,
                              q->ds_tz ? q->ds_tz->n : -1};
  if (q->ds_tz) {   // the whole table (a struct reused at the same address may hold another zone)
    uint64_t h = 1469598103934665603ULL;   // FNV-1a over the transitions and offsets
    auto mix = [&](uint64_t v) { for (int i = 0; i < 8; i++) { h ^= (v >> (8 * i)) & 0xFF; h *= 1099511628211ULL; } };
    for (int i = 0; i < q->ds_tz->n; i++) mix((uint64_t)q->ds_tz->utc_ms[i]);
    for (int i = 0; i <= q->ds_tz->n; i++) mix((uint64_t)(uint32_t)q->ds_tz->offset_ms[i]);
    key.push_back((int64_t)h);
  }
  if (c->calc_valid && c->calc_key == key) {
    P.bounds = c->calc_bounds;
  } else {
    int64_t a0;
    jcal_prev(Z, S0, n, unit, a0);
    const int64_t sc = a0 == S0 ? a0 : jcal_step(Z, a0, unit, n, 1);   // seekInterval(scan start)
    // zone-global grids: one boundary sequence whatever the anchor
    bool global = unit == TSDB_CAL_D ? n == 1 : unit == TSDB_CAL_W ? n == 1 : unit == TSDB_CAL_N ? 12 % n == 0
                  : unit == TSDB_CAL_Y ? n == 1 : false;
    if (unit == TSDB_CAL_MS || unit == TSDB_CAL_S || unit == TSDB_CAL_M || unit == TSDB_CAL_H) {
      const int64_t top = unit == TSDB_CAL_MS ? 1000 : unit == TSDB_CAL_H ? 24 : 60;
      if (top % n == 0) {
        global = true;
        const int64_t step = n * CAL_UNIT_MS[unit];
        const int32_t ref = Z.at(S0);
        if (q->ds_tz) {
          const tsdbhip_tz* z = q->ds_tz;
          for (int i = 0; i <= z->n && global; i++) {
            const int64_t from = i == 0 ? INT64_MIN : z->utc_ms[i - 1];
            const int64_t to = i == z->n ? INT64_MAX : z->utc_ms[i];
            if (to < S0 - 2 * 86400000LL || from > E0 + 2 * 86400000LL) continue;
            if (((int64_t)z->offset_ms[i] - ref) % step != 0) global = false;
          }
        }
      }
    }
    std::vector<int64_t> anchors;
    if (global) {
      anchors.push_back(sc);
    } else {
      // every series' first datapoint at or after the seek point (device), its anchor (host)
      const int64_t NS = c->n_series;
      std::vector<int64_t> f(std::max<int64_t>(1, NS));
      HIP_OK(c->first_ts.ensure(std::max<int64_t>(1, NS) * 8));
      HIP_OK(launch_first_ts(c->rows.as<RowDesc>(), c->srp.as<int64_t>(), c->qual.as<uint8_t>(), NS, P.ss, P.se, sc,
                             c->first_ts.as<int64_t>(), c->stream));
      if (NS) HIP_OK(hipMemcpyAsync(f.data(), c->first_ts.p, NS * 8, hipMemcpyDeviceToHost, c->stream));
      HIP_OK(hipStreamSynchronize(c->stream));
      f.resize(NS);
      std::sort(f.begin(), f.end());
      f.erase(std::unique(f.begin(), f.end()), f.end());
      anchors_of(Z, n, unit, f, anchors);
      anchors.erase(std::remove(anchors.begin(), anchors.end(), INT64_MAX), anchors.end());
      std::sort(anchors.begin(), anchors.end());
      anchors.erase(std::unique(anchors.begin(), anchors.end()), anchors.end());
    }
    // each anchor's boundary sequence through the first boundary >= the scan end
    std::vector<std::vector<int64_t>> seqs;
    std::vector<int64_t> T;
    for (int64_t a : anchors) {
      std::vector<int64_t> sq{a};
      while (sq.back() < E0) {
        sq.push_back(jcal_step(Z, sq.back(), unit, n, 1));
        if (sq.size() > 50000000) return fail(TSDB_E_ILLEGAL_ARGUMENT, "too many calendar buckets");
      }
      T.insert(T.end(), sq.begin(), sq.end());
      seqs.push_back(std::move(sq));
    }
    std::vector<int64_t> F;   // FillingDownsampler: previousInterval(start) .. previousInterval(end)
    if (fill) {
      int64_t f0, eC;
      jcal_prev(Z, S0, n, unit, f0);
      jcal_prev(Z, E0, n, unit, eC);
      if (eC == f0) eC = jcal_step(Z, eC, unit, n, 1);
      for (int64_t t = f0; t < eC; t = jcal_step(Z, t, unit, n, 1)) {
        F.push_back(t);
        if (F.size() > 50000000) return fail(TSDB_E_ILLEGAL_ARGUMENT, "too many calendar buckets");
      }
      F.push_back(eC);
      T.insert(T.end(), F.begin(), F.end());
    }
    std::sort(T.begin(), T.end());
    T.erase(std::unique(T.begin(), T.end()), T.end());
    // the sequences must coincide with the union wherever they run
    auto agrees = [&](const std::vector<int64_t>& sq) {
      const auto it = std::lower_bound(T.begin(), T.end(), sq.front());
      const size_t i0 = it - T.begin();
      if (i0 + sq.size() > T.size()) return false;
      for (size_t k = 0; k < sq.size(); k++) if (T[i0 + k] != sq[k]) return false;
      return true;
    };
    bool disagree = false;
    for (const auto& sq : seqs) disagree = disagree || !agrees(sq);
    // a fill over grids that disagree (with each other or with the FillingDownsampler's own
    // sequence): every span's filled output runs through the union evaluator (run_anchored)
    if (fill && !agrees(F)) disagree = true;
    P.bounds = fill && !disagree ? F : T;
    c->calc_key = key;
    c->calc_bounds = P.bounds;
    c->calc_seek = sc;
    c->calc_anchored = disagree;
    c->calc_anchors = disagree ? anchors : std::vector<int64_t>();
    c->calc_seqs = disagree ? seqs : std::vector<std::vector<int64_t>>();
    c->calc_fill = disagree && fill ? F : std::vector<int64_t>();
    c->calc_valid = true;
  }
  // spans on grids that disagree: their union of timestamps is no slot grid; run_anchored
  // downsamples each anchor's spans on its own sequence and aggregates over the union
  P.anchored = c->calc_anchored;
  if (P.anchored) {
    P.anchors = c->calc_anchors;
    P.seqs = c->calc_seqs;
    P.fillseq = c->calc_fill;
  }
  P.mode = MODE_TABLE;
  P.seek = c->calc_seek;
  P.I = q->ds_interval_ms;
  if (P.bounds.size() < 2) {
    P.bounds.assign(1, P.bounds.empty() ? S0 : P.bounds[0]);
    P.K = 0;
  } else {
    P.K = (int64_t)P.bounds.size() - 1;
  }
  P.B0 = P.bounds[0];
  return 0;
}

// TsdbQuery.getScanStartTimeSeconds :1515-1526 / getScanEndTimeSeconds :1562-1567 with a
// RollupQuery: the rollup row of the start (one further back for a rate), the row of the end
// plus one row span.
int rollup_scan_bounds(const tsdbhip_query* q, const tsdbhip_rollup_interval& iv, int64_t& ss, int64_t& se) {
  int64_t start = q->start_time;
  if ((start & (int64_t)0xFFFFFFFF00000000LL) != 0) start /= 1000;
  int32_t b = 0;
  int rc = tsdbhip_rollup_basetime(start, &iv, &b);
  if (rc) return rc;
  if (q->rate) {
    rc = tsdbhip_rollup_basetime((int64_t)b - 1, &iv, &b);
    if (rc) return rc;
  }
  ss = b;
  int64_t end = q->end_time;
  if ((end & (int64_t)0xFFFFFFFF00000000LL) != 0) {
    end /= 1000;
    if (end - (end * 1000) < 1) end++;
  }
  rc = tsdbhip_rollup_basetime(end + (int64_t)iv.interval_s * iv.intervals, &iv, &b);
  if (rc) return rc;
  se = b;
  return 0;
}

int scan_bounds_of(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t& ss, int64_t& se) {
  if (c->ro_active) return rollup_scan_bounds(q, c->ro_iv, ss, se);
  return tsdbhip_scan_bounds(q, &ss, &se);
}

// A row whose query-time compaction failed fails every query whose scan covers it
// (SaltScanner.processRow :825-830 closes the scanner with the exception), in scan order.
int cmp_scan_check(tsdbhip_ctx* c, const Plan& P) {
  for (const auto& e : c->cmp_errs)
    if (e.base >= P.ss && e.base < P.se)
      return fail(e.code, e.code == TSDB_E_NOT_IMPLEMENTED
                              ? "query-time compaction of a row this engine does not restate (a compacted cell out of "
                                "time order, or a datapoint column without a value)"
                              : "IllegalDataException in the query-time compaction of a row (duplicate timestamp with a "
                                "different value, or a corrupted cell)");
  return 0;
}

// The point every span's Downsampler seeks to (Downsampler.seekInterval :415-437; ds_all: the
// scan start), for the kernels' stream-order row skip (kcommon.h so_row_skip)
int64_t seek_point(const Plan& P) {
  return P.mode == MODE_ALL ? P.ss * 1000 : P.mode == MODE_TABLE ? P.seek : P.B0;
}

int plan_query(tsdbhip_ctx* c, const tsdbhip_query* q, Plan& P) {
  if (q->aggregator < 0 || q->aggregator >= TSDB_AGG_COUNT_ALL) return fail(TSDB_E_ILLEGAL_ARGUMENT, "bad aggregator");
  if (q->ds_function >= TSDB_AGG_COUNT_ALL) return fail(TSDB_E_ILLEGAL_ARGUMENT, "bad downsampling function");
  if (q->ds_function == TSDB_AGG_NONE) return fail(TSDB_E_ILLEGAL_ARGUMENT, "cannot use the NONE aggregator for downsampling");
  if (q->ds_function < 0) {
    P.raw = true;
    P.ga = ga_of(q->aggregator);
    if (P.ga < 0 && is_sel_agg(q->aggregator)) {
      P.gsel = q->aggregator;   // span operands per union point, then k_raw_sel
      P.ga = GA_NONE;           // placeholder: k_raw_eval does not run
    }
    if (P.ga < 0) return fail(TSDB_E_NOT_IMPLEMENTED, std::string("group-by aggregator not implemented yet: ") + AGG_NAMES[q->aggregator]);
    P.interp = interp_of(q->aggregator);
    P.none = q->aggregator == TSDB_AGG_NONE;
    { const int brc = scan_bounds_of(c, q, P.ss, P.se); if (brc) return brc; }
    return cmp_scan_check(c, P);
  }
  if (!q->ds_all && q->ds_interval_ms <= 0) return fail(TSDB_E_ILLEGAL_ARGUMENT, "interval not > 0");
  int64_t calW = 0, calO = 0, calM = 0;
  bool table = false, general = false;
  if (q->ds_calendar && !q->ds_all) {
    if (q->ds_tz) general = true;   // a time zone: the general calendar plan
    else if (cal_grid(q->ds_calendar, q->ds_interval_ms, &calW, &calO)) {}
    else if (cal_months(q->ds_calendar, q->ds_interval_ms, &calM)) table = true;
    else general = true;            // anchored per span
  }
  P.ga = ga_of(q->aggregator);
  P.f = f_of(q->ds_function);
  if (P.f < 0 && (q->ds_function == TSDB_AGG_MEDIAN || q->ds_function >= TSDB_AGG_P999)) P.f = F_SEL;
  if (P.ga < 0 && is_sel_agg(q->aggregator)) {
    P.gsel = q->aggregator;   // order statistics per (group, slot): run_sel_group
    P.ga = GA_NONE;           // placeholder: no partial state is built for these
  }
  if (P.ga < 0) return fail(TSDB_E_NOT_IMPLEMENTED, std::string("group-by aggregator not implemented yet: ") + AGG_NAMES[q->aggregator]);
  if (P.f < 0) return fail(TSDB_E_NOT_IMPLEMENTED, std::string("downsampling function not implemented yet: ") + AGG_NAMES[q->ds_function]);
  // TSDB_QF_ORDERED: float reductions in SpanGroup index order (bit-exact); the other
  // aggregators are already order-exact on the partials path
  P.ordered = (q->flags & TSDB_QF_ORDERED) && !P.gsel &&
              (P.ga == GA_SUM || P.ga == GA_AVG || P.ga == GA_SQUARESUM || P.ga == GA_DEV || P.ga == GA_MULT);
  P.interp = interp_of(q->aggregator);
  P.none = q->aggregator == TSDB_AGG_NONE;
  { const int brc = scan_bounds_of(c, q, P.ss, P.se); if (brc) return brc; }
  const int64_t S0 = P.ss * 1000, E0 = P.se * 1000;
  if (q->ds_all) {
    P.mode = MODE_ALL;
    P.I = 1;
    P.B0 = 0;
    P.K = 1;
  } else {
    P.mode = MODE_GRID;
    const int64_t I = q->ds_interval_ms;
    P.I = I;
    if (general) {
      const int rc = plan_calendar(c, q, P);
      if (rc) return rc;
    } else if (table) {
      // slot boundaries of the month grid: first slot = seekInterval(scan start) :420-432
      P.mode = MODE_TABLE;
      auto mprev = [&](int64_t t) {   // previousInterval: the n-month block of t, from January
        const int64_t m = month_of_ms(t);
        const int64_t y = floor_div(m, 12);
        return y * 12 + floor_div(m - y * 12, calM) * calM;
      };
      const int64_t f0 = mprev(S0);
      const int64_t m0 = month_start_ms(f0) == S0 ? f0 : f0 + calM;
      int64_t mbeg = m0, mend;   // first slot's month, first month index not covered
      if (q->ds_fill != TSDB_FILL_NONE) {
        // FillingDownsampler :113-135 emits from previousInterval(start); a leading block
        // before the seek point gets no points (fill value only)
        mbeg = f0;
        int64_t eC = mprev(E0);
        if (eC == f0) eC += calM;
        mend = eC;
      } else {
        mend = m0;
        while (month_start_ms(mend) < E0) mend += calM;
      }
      P.seek = month_start_ms(m0);
      P.bounds.clear();
      for (int64_t m = mbeg; m <= mend; m += calM) P.bounds.push_back(month_start_ms(m));
      if (P.bounds.size() < 2) { P.bounds.assign(1, month_start_ms(m0)); P.K = 0; }
      else P.K = (int64_t)P.bounds.size() - 1;
      P.B0 = P.bounds[0];
    } else if (q->ds_calendar) {
      // Downsampler.seekInterval :420-432 (previousInterval, next one if the seek time is
      // past it); FillingDownsampler ctor :113-135: buckets from previousInterval(start) to
      // previousInterval(end), one bucket when both are the same.
      auto cfloor = [&](int64_t t) { return calO + floor_div(t - calO, I) * I; };
      const int64_t f0 = cfloor(S0);
      P.B0 = f0 == S0 ? S0 : f0 + I;
      if (q->ds_fill != TSDB_FILL_NONE) {
        int64_t eC = cfloor(E0);
        if (eC == f0) eC += I;
        if (f0 < P.B0) {
          // a leading slot before the seek point (weeks): a boundary table whose slot 0
          // receives no points
          P.mode = MODE_TABLE;
          P.seek = P.B0;
          P.bounds.clear();
          for (int64_t t = f0; t <= eC; t += I) P.bounds.push_back(t);
          P.K = (int64_t)P.bounds.size() - 1;
          P.B0 = f0;
        } else {
          P.K = eC > P.B0 ? (eC - P.B0) / I : 0;
        }
      } else {
        P.K = E0 > P.B0 ? (E0 - P.B0 + I - 1) / I : 0;
      }
    } else {
      P.B0 = ((S0 + I - 1) / I) * I;  // Downsampler seek: first bucket fully after the scan start
      if (q->ds_fill != TSDB_FILL_NONE) {
        const int64_t aE = E0 - E0 % I;
        P.K = aE > P.B0 ? (aE - P.B0) / I : 0;
      } else {
        P.K = E0 > P.B0 ? (E0 - P.B0 + I - 1) / I : 0;
      }
    }
  }
  // slot arrays live in LDS when they fit next to 4 waves' worth of staging, else in HBM
  P.gslot = grid_wave_lds(P.K, q->rate != 0, false) > 40 * 1024;
  return cmp_scan_check(c, P);
}

// Largest number of datapoints one series holds in rows with base in [ss, se) (cached per
// scan range; the batch is resident).
int64_t series_max_dp(tsdbhip_ctx* c, int64_t ss, int64_t se) {
  if (c->mdp_valid && c->mdp_ss == ss && c->mdp_se == se) return c->mdp;
  int64_t m = 0;
  for (int64_t s = 0; s < c->n_series; s++) {
    int64_t n = 0;
    for (int64_t r = c->h_srp[s]; r < c->h_srp[s + 1]; r++)
      if ((int64_t)c->h_base[r] >= ss && (int64_t)c->h_base[r] < se) n += c->h_ndp[r];
    m = std::max(m, n);
  }
  c->mdp_valid = true;
  c->mdp_ss = ss;
  c->mdp_se = se;
  c->mdp = m;
  return m;
}

// The streaming kernels (k_short / k_fast) can take the query: fixed grid, a row class of the
// batch they are specialised for, their LDS slot budget.
// LDS a streaming-kernel wave takes: KR 0 writing the buckets to HBM (dense_out, K > 64 or rate)
// keeps no partials or rate values; the register-partial variants (KR != 0: K <= 64, no rate) keep
// their partials in registers (k_short's staged column variant then fits 4 waves a SIMD: 10.9 ->
// 9.5 KB a wave)
int64_t fast_lds_of(const tsdbhip_query* q, const Plan& P) {
  const bool rate = q->rate != 0;
  const bool kr = P.K <= 64 && !rate;
  const bool dense0 = P.dense_out && !kr;
  return fast_wave_lds(P.K, rate && !dense0, !dense0 && !kr);
}

bool fast_path_ok(tsdbhip_ctx* c, const tsdbhip_query* q, const Plan& P) {
  if (!(P.mode == MODE_GRID && c->fast_qw &&
        (fast_supported(P.f, c->fast_qw, c->fast_vl) || (c->fast_qw2 && fast_supported(P.f, c->fast_qw2, c->fast_vl2))) &&
        P.I <= (1LL << 29) && fast_lds_of(q, P) <= 32 * 1024 && P.K > 0))
    return false;
  return !opt_off(OPT_FAST);
}

// The series of every row, on the device (k_seq_rows), once per resident batch.
int ensure_row_series(tsdbhip_ctx* c) {
  if (c->row_ser_valid) return 0;
  std::vector<int32_t> rs(std::max<int64_t>(1, c->n_rows));
  for (int64_t s = 0; s < c->n_series; s++)
    for (int64_t r = c->h_srp[s]; r < c->h_srp[s + 1]; r++) rs[r] = (int32_t)s;
  HIP_OK(c->row_ser.ensure(rs.size() * 4));
  HIP_OK(hipMemcpy(c->row_ser.p, rs.data(), rs.size() * 4, hipMemcpyHostToDevice));
  c->row_ser_valid = true;
  return 0;
}

// Series a grouped query reads: the ungrouped ones (a rollup batch's count series, spans without
// a group) sort last and only NONE reads them, so the sequential kernels stop before them.
int64_t grouped_prefix(tsdbhip_ctx* c) {
  if (c->n_grouped >= 0) return c->n_grouped;
  int64_t n = 0;
  while (n < c->n_series && c->h_group[n] < c->n_groups) n++;
  for (int64_t i = n; i < c->n_series; i++)
    if (c->h_group[i] < c->n_groups) { n = c->n_series; break; }
  c->n_grouped = n;
  return n;
}

// k_seq_rows takes a sequential (Java-order) downsampling when the interval divides one hour
// and slot 0 is interval-aligned (then a bucket of an hour row aligned to the hour holds only
// that row's datapoints; the kernel checks the rows), over rows short enough that one thread a
// row beats k_seq_wave's wave a series (fewer than 64 datapoints a row on average).
bool seq_rows_ok(tsdbhip_ctx* c, const Plan& P) {
  if (opt_off(OPT_SEQ_ROWS)) return false;
  return P.mode == MODE_GRID && P.I > 0 && 3600000 % P.I == 0 && P.B0 % P.I == 0 && P.K > 0 && !c->seqd_uniform &&
         c->n_rows < ((int64_t)1 << 31);
}

// A grid query whose streaming-kernel LDS (the per-slot partials of K buckets) exceeds a wave's
// budget -- a day of 1m buckets: K = 1440 -- would run k_grid's general path with slot arrays in
// HBM (5 % of HBM on config 3's day, c3day_bench).  Split it instead: the streaming kernels write
// every series' buckets to HBM (dense_out, no partials in LDS), then the group-by step runs over
// them (emit_only: k_emit + k_reduce), as the percentile functions do.
// k_hwin takes the query: a fixed grid of K > 64 buckets dividing the hour with slot 0 on an
// hour (every hour row in one window of W = 1 h / interval <= 64 slots), no rate, an order-free
// function, and every tile of one streaming class with one-chunk rows.
int hwin_slots(tsdbhip_ctx* c, const tsdbhip_query* q, const Plan& P, bool for_multi = false) {
  if (opt_off(OPT_HWIN)) return 0;   // option HWIN: 0 never; 2 wherever it applies (A/B)
  if (opt_is(OPT_HWIN, 2)) for_multi = true;
  // (fill policies need every participating series' fill values in windows where it has no row:
  // left to the dense split)
  if (P.mode != MODE_GRID || q->rate || q->ds_fill != TSDB_FILL_NONE || P.K <= 64 || P.I <= 0 || 3600000 % P.I != 0 || 3600000 / P.I > 64 ||
      ((P.B0 % 3600000) + 3600000) % 3600000 != 0 || P.dense_out || P.emit_only || P.values_only || P.sel_direct ||
      P.seq_dense || P.raw || P.anchored || P.none || P.f == F_SEL || !c->fast_qw || !c->tl_other.empty())
    return 0;
  for (int cls = 0; cls < 2; cls++) {
    if (!c->tl[cls][0].empty()) return 0;
    if (c->tl[cls][1].empty() && c->tl[cls][2].empty()) continue;
    const int qw = cls ? c->fast_qw2 : c->fast_qw, vl = cls ? c->fast_vl2 : c->fast_vl;
    if (!qw || !fast_supported(P.f, qw, vl)) return 0;
  }
  if (opt_off(OPT_FAST)) return 0;
  // Every K > 64 that tiles the hour, since k_hwin runs a work item a (tile, window): 12 h of 1m
  // buckets (K = 720, whose slots fit the fused kernels' LDS) 50.6 ms through k_rows vs 11.4 ms
  // here, 10m buckets of a day (K = 144) 11.8 vs 11.3 ms (profiles/r05j/).  (Before the per-window
  // items, k_rows won at 10m: profiles/r04x.)  The fused multi-aggregator pass has no K > 64
  // variant of the other kernels either.
  (void)for_multi;
  return (int)(3600000 / P.I);
}

bool dense_split_wanted(tsdbhip_ctx* c, const tsdbhip_query* q, const Plan& P) {
  if (hwin_slots(c, q, P)) return false;   // (k_hwin needs no bucket store)
  if (P.dense_out || P.emit_only || P.values_only || P.sel_direct || P.multi || P.seq_dense || P.raw || P.anchored ||
      P.f == F_SEL || P.mode != MODE_GRID || P.K <= 64)
    return false;
  if (fast_wave_lds(P.K, q->rate != 0, true) <= 32 * 1024) return false;   // the fused pass fits
  Plan Pd = P;
  Pd.dense_out = true;
  if (!fast_path_ok(c, q, Pd)) return false;
  return (double)c->n_series * (double)P.K * 9.0 <= 64.0 * (1ull << 30);   // [series][K] values + presence
}

int run_device(tsdbhip_ctx* c, const tsdbhip_query* q, const Plan& P, int64_t G, bool do_reduce) {
  if (dense_split_wanted(c, q, P)) {
    Plan P1 = P;
    P1.dense_out = true;
    int rc = run_device(c, q, P1, G, false);
    if (rc) return rc;
    Plan P2 = P;
    P2.emit_only = true;
    P2.split2 = true;
    return run_device(c, q, P2, G, do_reduce);
  }
  const bool none = P.none;
  if (none) { int rc = build_none_tiles(c); if (rc) return rc; }
  const int64_t nt = none ? c->n_series : (int64_t)c->tb.size();
  const int64_t K = P.K;
  HIP_OK(c->pa.ensure(std::max<int64_t>(1, nt * K) * 8));
  HIP_OK(c->pb.ensure(std::max<int64_t>(1, nt * K) * 8));
  HIP_OK(c->pn.ensure(std::max<int64_t>(1, nt * K) * 4));
  HIP_OK(c->pf.ensure(std::max<int64_t>(1, nt * K) * 4));
  HIP_OK(c->out_val.ensure(std::max<int64_t>(1, G * K) * 8));
  HIP_OK(c->out_flag.ensure(std::max<int64_t>(1, G * K)));
  HIP_OK(c->gact.ensure(std::max<int64_t>(1, G) * 4));
  HIP_OK(hipMemsetAsync(c->gact.p, 0, std::max<int64_t>(1, G) * 4, c->stream));
  HIP_OK(hipMemsetAsync(c->err.p, 0, 4, c->stream));
  GridParams gp{};
  gp.rows = c->rows.as<RowDesc>();
  gp.series_row_ptr = c->srp.as<int64_t>();
  gp.qual = c->qual.as<uint8_t>();
  gp.val = c->val.as<uint8_t>();
  gp.val2 = c->val2.as<uint8_t>();
  gp.tile_begin = (none ? c->n_tb : c->d_tb).as<int64_t>();
  gp.tile_end = (none ? c->n_te : c->d_te).as<int64_t>();
  gp.tile_group = (none ? c->n_tg : c->d_tg).as<int32_t>();
  gp.n_tiles = nt;
  gp.ss = P.ss;
  gp.se = P.se;
  gp.B0 = P.B0;
  gp.I = P.I;
  gp.K = K;
  gp.qs = q->start_time;
  gp.qe = q->end_time;
  gp.rcpI = (float)(1.0 / (double)P.I);
  gp.mode = P.mode;
  gp.seek_any = seek_point(P);
  gp.ga = P.ga;
  gp.interp = P.interp;
  gp.fill = q->ds_fill;
  if (P.mode == MODE_TABLE) {
    HIP_OK(c->cal_bounds.ensure((int64_t)P.bounds.size() * 8));
    HIP_OK(hipMemcpyAsync(c->cal_bounds.p, P.bounds.data(), P.bounds.size() * 8, hipMemcpyHostToDevice, c->stream));
    gp.bounds = c->cal_bounds.as<int64_t>();
    gp.seek_ms = P.seek;
    gp.skip0 = P.bounds[0] < P.ss * 1000 ? 1 : 0;
  }
  gp.rate = q->rate;
  gp.counter = q->rate_counter;
  gp.drop = q->rate_drop_resets;
  gp.counter_max = q->rate_counter_max;
  gp.reset_value = q->rate_reset_value;
  gp.wave_lds = (int32_t)grid_wave_lds(K, q->rate != 0, P.gslot);
  int waves = (int)std::max<int64_t>(1, std::min<int64_t>(4, (64 * 1024) / gp.wave_lds));
  if (P.gslot) {
    HIP_OK(c->g_dense.ensure(std::max<int64_t>(1, nt * K) * 8));
    HIP_OK(c->g_pres.ensure(std::max<int64_t>(1, nt * K)));
    if (q->rate) HIP_OK(c->g_rate.ensure(std::max<int64_t>(1, nt * K) * 8));
    gp.g_dense = c->g_dense.as<double>();
    gp.g_pres = c->g_pres.as<uint8_t>();
    gp.g_rate = q->rate ? c->g_rate.as<double>() : nullptr;
  }
  gp.waves = waves;
  gp.part = Partials{c->pa.as<double>(), c->pb.as<double>(), c->pn.as<uint32_t>(), c->pf.as<uint32_t>()};
  gp.group_active = c->gact.as<uint32_t>();
  gp.err = c->err.as<int32_t>();
  if (P.multi) {   // fused multi-aggregator pass: every decomposable aggregator's tile partials
    const int64_t n = std::max<int64_t>(1, nt * K);
    HIP_OK(c->m_sum.ensure(n * 8));
    HIP_OK(c->m_mn.ensure(n * 8));
    HIP_OK(c->m_mx.ensure(n * 8));
    HIP_OK(c->m_mean.ensure(n * 8));
    HIP_OK(c->m_m2.ensure(n * 8));
    HIP_OK(c->m_nl.ensure(n * 4));
    HIP_OK(c->m_nz.ensure(n * 4));
    HIP_OK(c->m_f.ensure(n * 4));
    gp.multi = MULTI_ON | (P.multi_dev ? MULTI_DEV : 0);
    gp.mp = MultiPartials{c->m_sum.as<double>(), c->m_mn.as<double>(), c->m_mx.as<double>(), c->m_mean.as<double>(),
                          c->m_m2.as<double>(), c->m_nl.as<uint32_t>(), c->m_nz.as<uint32_t>(), c->m_f.as<uint32_t>()};
  }
#ifdef TSDBHIP_KDBG
  if (opt(OPT_DBG) > 0) gp.dbg = (int32_t)opt(OPT_DBG);   // profiling build only
#endif
  if (P.sel_direct) {   // buffers prepared by sel_values
    gp.sel_direct = 1;
    if (P.sel_win) {   // (sel_window)
      gp.sel_win = 1;
      gp.win_lo = c->win_lo.as<double>();
      gp.win_hi = c->win_hi.as<double>();
      gp.win_val = c->win_val.as<double>();
      gp.win_gcnt = c->win_gcnt.as<unsigned long long>();
      gp.win_cur = c->win_cur.as<uint32_t>();
      gp.win_cand = c->win_cand.as<double>();
    }
    gp.sel_cols = P.sel_cols ? 1 : 0;
    gp.sel_vals = c->sel_vals.as<double>();
    gp.sel_uni = c->sel_uni.as<uint8_t>();
    gp.sel_wr = c->sel_wr.as<uint8_t>();
    gp.group_series_ptr = c->sel_gsp.as<int64_t>();
  } else if (P.dense_out) {
    HIP_OK(c->pre_dense.ensure(std::max<int64_t>(1, c->n_series * K) * 8));
    HIP_OK(c->pre_pres.ensure(std::max<int64_t>(1, c->n_series * K)));
    HIP_OK(hipMemsetAsync(c->pre_pres.p, 0, std::max<int64_t>(1, c->n_series * K), c->stream));
    gp.dense_out = c->pre_dense.as<double>();
    gp.pres_out = c->pre_pres.as<uint8_t>();
  }

  if (P.f == F_SEL || P.emit_only || P.seq_dense) {
    // percentile / median: per-series bucket order statistics, then the group-by step
    // (emit_only: the group-by step alone, over buckets a previous pass left in pre_dense;
    // seq_dense: k_seq_dense leaves them there first)
    HIP_OK(c->pre_dense.ensure(std::max<int64_t>(1, c->n_series * K) * 8));
    HIP_OK(c->pre_pres.ensure(std::max<int64_t>(1, c->n_series * K)));
    if (P.seq_dense) {
      HIP_OK(hipEventRecord(c->ev[0], c->stream));
      HIP_OK(hipMemsetAsync(c->pre_pres.p, 0, std::max<int64_t>(1, c->n_series * K), c->stream));
      const int64_t ns = P.none ? c->n_series : grouped_prefix(c);   // series the query reads
      if (P.ro_fuse && seq_rows_ok(c, P)) {
        // rollup avg / count: a thread a value row with its count row, combined in place; the
        // handed-back series (value and count) through k_seq_dense, then combined
        int rc = ensure_row_series(c);
        if (rc) return rc;
        HIP_OK(c->sr_list.ensure(std::max<int64_t>(1, c->n_series) * 4));
        HIP_OK(c->sr_mark.ensure(std::max<int64_t>(1, c->n_series) * 4));
        HIP_OK(c->sr_n.ensure(16));
        HIP_OK(hipMemsetAsync(c->sr_mark.p, 0, std::max<int64_t>(1, c->n_series) * 4, c->stream));
        HIP_OK(hipMemsetAsync(c->sr_n.p, 0, 4, c->stream));
        GridParams rp = gp;
        rp.row_series = c->row_ser.as<int32_t>();
        rp.redo_list = c->sr_list.as<int32_t>();
        rp.redo_n = c->sr_n.as<int32_t>();
        rp.redo_mark = c->sr_mark.as<uint32_t>();
        rp.ro_partner = c->ro_partner.as<int32_t>();
        const int avg = P.ro_fuse == 1 ? 1 : 0;
        if (c->ro_npairs > 0) {
          rp.ro_pairs = c->ro_pairs.as<RoPair>();
          if (c->ro_nruns) {
            rp.ro_runs = c->ro_runs.as<RoRun>();
            rp.ro_rid = c->ro_rid.as<uint32_t>();
          }
          HIP_OK(launch_ro_pairs(rp, avg, c->pre_dense.as<double>(), c->pre_pres.as<uint8_t>(), c->ro_cmap.as<int64_t>(),
                                 c->ro_npairs, c->stream));
        } else {
          HIP_OK(launch_seq_rows_ro(rp, avg, c->pre_dense.as<double>(), c->pre_pres.as<uint8_t>(), c->ro_cmap.as<int64_t>(),
                                    c->n_rows, c->stream));
        }
        GridParams dp = gp;
        dp.tile_list = c->sr_list.as<int32_t>();
        dp.tile_list_n = c->sr_n.as<int32_t>();
        HIP_OK(launch_seq_dense(dp, F_SUM, c->pre_dense.as<double>(), c->pre_pres.as<uint8_t>(), c->n_series, c->stream,
                                false));
        HIP_OK(launch_rollup_combine_list(c->pre_dense.as<double>(), c->pre_pres.as<uint8_t>(), c->ro_cmap.as<int64_t>(),
                                          c->sr_list.as<int32_t>(), c->sr_n.as<int32_t>(), c->n_series, K, avg,
                                          c->stream));
      } else if (seq_rows_ok(c, P)) {
        // every bucket inside one hour row: a thread a row, then k_seq_dense over the series
        // whose rows broke that premise
        int rc = ensure_row_series(c);
        if (rc) return rc;
        HIP_OK(c->sr_list.ensure(std::max<int64_t>(1, c->n_series) * 4));
        HIP_OK(c->sr_mark.ensure(std::max<int64_t>(1, c->n_series) * 4));
        HIP_OK(c->sr_n.ensure(16));
        HIP_OK(hipMemsetAsync(c->sr_mark.p, 0, std::max<int64_t>(1, c->n_series) * 4, c->stream));
        HIP_OK(hipMemsetAsync(c->sr_n.p, 0, 4, c->stream));
        GridParams rp = gp;
        rp.row_series = c->row_ser.as<int32_t>();
        rp.redo_list = c->sr_list.as<int32_t>();
        rp.redo_n = c->sr_n.as<int32_t>();
        rp.redo_mark = c->sr_mark.as<uint32_t>();
        if (c->ro_active && c->ro_npairs > 0 && !P.none) {
          rp.ro_pairs = c->ro_pairs.as<RoPair>();   // a rollup batch's value rows, packed (k_ro_rows)
          if (c->ro_nruns) {
            rp.ro_runs = c->ro_runs.as<RoRun>();
            rp.ro_rid = c->ro_rid.as<uint32_t>();
          }
          HIP_OK(launch_ro_rows(rp, P.f, c->pre_dense.as<double>(), c->pre_pres.as<uint8_t>(), c->ro_npairs, c->stream));
        } else {
          HIP_OK(launch_seq_rows(rp, P.f, c->pre_dense.as<double>(), c->pre_pres.as<uint8_t>(), c->h_srp[ns], c->stream));
        }
        GridParams dp = gp;
        dp.tile_list = c->sr_list.as<int32_t>();
        dp.tile_list_n = c->sr_n.as<int32_t>();
        HIP_OK(launch_seq_dense(dp, P.f, c->pre_dense.as<double>(), c->pre_pres.as<uint8_t>(), ns, c->stream, false));
      } else {
        HIP_OK(launch_seq_dense(gp, P.f, c->pre_dense.as<double>(), c->pre_pres.as<uint8_t>(), ns, c->stream,
                                c->seqd_uniform));
      }
    }
    gp.sel_fn = q->ds_function;
    gp.n_series = c->n_series;
    gp.pre_dense = c->pre_dense.as<double>();
    gp.pre_pres = c->pre_pres.as<uint8_t>();
    const int64_t elds = align16(K * 8) * 2 + align16(K * 4) * 2 + (q->rate ? align16(K * 8) : 0);
    if (elds > 48 * 1024) {
      HIP_OK(c->g_dense.ensure(std::max<int64_t>(1, nt * K) * 8));
      if (q->rate) HIP_OK(c->g_rate.ensure(std::max<int64_t>(1, nt * K) * 8));
      gp.g_dense = c->g_dense.as<double>();
      gp.g_rate = q->rate ? c->g_rate.as<double>() : nullptr;
      gp.wave_lds = 16;
    } else {
      gp.g_dense = nullptr;
      gp.wave_lds = (int32_t)std::max<int64_t>(16, elds);
    }
    gp.waves = (int)std::max<int64_t>(1, std::min<int64_t>(4, (64 * 1024) / gp.wave_lds));
    if (!P.split2) c->fast_used = false;   // (split: ev[0] and the k_fast state of the first pass stand)
    if (!P.seq_dense && !P.split2) HIP_OK(hipEventRecord(c->ev[0], c->stream));
    if (!P.emit_only && !P.seq_dense) {
    HIP_OK(c->redo.ensure(std::max<int64_t>(1, c->n_series) * 4));
    HIP_OK(c->redo_n.ensure(16));
    HIP_OK(hipMemsetAsync(c->redo_n.p, 0, 4, c->stream));
    gp.redo_list = c->redo.as<int32_t>();
    gp.redo_n = c->redo_n.as<int32_t>();
    // Buckets inside rows (interval | 1 h): k_pct_rows, with k_pct over the series it hands
    // back; else k_pct over every series.  Its extraction covers statistics near the ends (p90
    // and up); 1 h buckets of 4-byte values go through its 32-bit key kernel, which ranks any
    // statistic (median, p50, p75 by a bitwise search).
    const int sel_i = (q->ds_function - TSDB_AGG_P999) % 6;
    const bool near_end = q->ds_function != TSDB_AGG_MEDIAN && sel_i <= 3;
    const bool keys = c->pct_vl == 4 && P.I == 3600000 && !opt_off(OPT_PCT_KEYS);
    const bool rows_path = P.mode == MODE_GRID && (near_end || keys) && P.I > 0 && 3600000 % P.I == 0 &&
                           P.B0 % P.I == 0 && pct_rows_supported(c->pct_qw, c->pct_vl) && !opt_off(OPT_PCT_ROWS);
    if (rows_path) {
      HIP_OK(c->redo2.ensure(std::max<int64_t>(1, c->n_series) * 4));
      HIP_OK(c->redo2_n.ensure(16));
      HIP_OK(hipMemsetAsync(c->redo2_n.p, 0, 4, c->stream));
      GridParams rp = gp;
      rp.redo_list = c->redo2.as<int32_t>();
      rp.redo_n = c->redo2_n.as<int32_t>();
      rp.pct_vonly = keys && c->pct_vonly && !opt_off(OPT_PCT_VONLY);
      rp.pct_v6 = rp.pct_vonly && c->pct_v6 && !opt_off(OPT_PCT_V6);
      HIP_OK(launch_pct_rows(rp, c->pct_qw, c->pct_vl, c->stream));
      int32_t nback = 0;
      { int rc_ = d2h_small(c, &nback, c->redo2_n.p, 4, c->stream); if (rc_) return rc_; }
      { int rc_ = sync_small(c, c->stream); if (rc_) return rc_; }
      gp.tile_list = c->redo2.as<int32_t>();
      gp.tile_list_n = c->redo2_n.as<int32_t>();
      HIP_OK(launch_pct(gp, 1, nback, c->stream));
    } else {
      HIP_OK(launch_pct(gp, 0, c->n_series, c->stream));
    }
    int32_t nbig = 0;   // series with a bucket of more than 512 values: the large-bucket pass
    { int rc_ = d2h_small(c, &nbig, c->redo_n.p, 4, c->stream); if (rc_) return rc_; }
    { int rc_ = sync_small(c, c->stream); if (rc_) return rc_; }
    if (nbig > 0) {
      // persistent waves, each with an overflow region as large as the largest series' in-range
      // datapoints (buckets above PCT_CAP values); at most ~2 GB of regions
      const int64_t cap = std::max<int64_t>(PCT_CAP + 1, series_max_dp(c, P.ss, P.se));
      int64_t nw = std::min<int64_t>({(int64_t)nbig, 4096, std::max<int64_t>(2, ((int64_t)2 << 30) / (cap * 8))});
      nw = (nw + 1) & ~(int64_t)1;
      HIP_OK(c->big_scratch.ensure(nw * cap * 8));
      gp.big_scratch = c->big_scratch.as<double>();
      gp.big_cap = cap;
      gp.n_launch = nw;
      HIP_OK(launch_pct(gp, 2, nw, c->stream));
    }
    }
    if (!P.gsel && !P.ordered && !P.values_only)
      HIP_OK(launch_emit(gp, c->stream));   // else the caller takes the bucket values
    HIP_OK(hipEventRecord(c->ev[1], c->stream));
  } else {
  // streaming kernel first (when the batch's row class and the query allow it), then the
  // general kernel over the tiles it handed back
  const int hwin = hwin_slots(c, q, P);
  const bool fast = hwin || fast_path_ok(c, q, P);
  if (P.multi && !fast) return fail(TSDB_E_NOT_IMPLEMENTED, "fused multi-aggregator pass without the streaming kernels");
  c->fast_used = fast;
  if (!P.split2) HIP_OK(hipEventRecord(c->ev[0], c->stream));   // (split2: an earlier pass's start stands)
  if (fast) {
    // Per row class (A, B): k_short over its one-row-series tiles, k_rows over its tiles of
    // one-chunk rows, k_fast over its other tiles and over what those two handed back; k_grid
    // over what k_fast handed back and over the tiles of neither class.  Lists by class are
    // built at load (no per-tile appends for class mismatches); only tiles that break a
    // premise at run time are appended.
    const bool use_short = !opt_off(OPT_SHORT);
    const bool use_rows = !opt_off(OPT_ROWS);
    const int32_t* dl = c->tl_dev_override ? c->tl_dev_override : c->d_tl.as<int32_t>();
    const int32_t* dn = c->tln_dev_override ? c->tln_dev_override : c->d_tl_n.as<int32_t>();
    HIP_OK(c->r1a.ensure(std::max<int64_t>(1, nt) * 4));
    HIP_OK(c->r1b.ensure(std::max<int64_t>(1, nt) * 4));
    HIP_OK(c->r3a.ensure(std::max<int64_t>(1, nt) * 4));
    HIP_OK(c->r3b.ensure(std::max<int64_t>(1, nt) * 4));
    HIP_OK(c->r2.ensure(std::max<int64_t>(1, nt) * 4));
    HIP_OK(c->r_n.ensure(32));
    HIP_OK(hipMemsetAsync(c->r_n.p, 0, 32, c->stream));
    int32_t* rn = c->r_n.as<int32_t>();   // [0] r1a, [1] r1b, [2] r2, [3] r3a, [4] r3b
    auto fast_launch = [&](int cls, int shortk, const int32_t* list, const int32_t* list_n, int64_t cap,
                           int32_t* out, int32_t* out_n) -> int {
      const int qw = cls ? c->fast_qw2 : c->fast_qw, vl = cls ? c->fast_vl2 : c->fast_vl;
      if (cap == 0 || !qw || !fast_supported(P.f, qw, vl)) return 1;   // not run: caller routes the list on
      GridParams fp = gp;
      fp.shortk = shortk;
      fp.unit_s = (qw == 2 && P.I % 1000 == 0 && P.B0 % 1000 == 0) ? 1 : 0;
      fp.In = (int32_t)(fp.unit_s ? P.I / 1000 : P.I);
      fp.B0n = fp.unit_s ? P.B0 / 1000 : P.B0;
      fp.rcpn = std::nextafter(1.0 / (double)fp.In, INFINITY);
      fp.oneb = P.I >= 3600000 ? 1 : 0;   // (an hour row's chunk in one bucket)
      fp.wave_lds = (int32_t)(shortk == 3 ? fast_wave_lds(hwin, false, false) : fast_lds_of(q, P));
      fp.win_w = hwin;
      if (shortk == 3) fp.redo_mark = c->hw_mark.as<uint32_t>();
      if (shortk == 3) {
        // k_hwin: one work item a (tile, hour window) -- a tile's 24 windows as one item left the
        // last round of the launch mostly idle; items of fewer windows measured 13.6 (whole tiles)
        // -> 12.6 (4) -> 12.2 (6) -> 11.9 (12) -> 11.4 ms (24) on config 3's day shard
        // (profiles/r05h/split*.jsonl).  TSDBHIP_HWIN_SPLIT: items a tile.
        const int nw = (int)((K + hwin - 1) / hwin);
        fp.win_split = nw;
      }
      fp.short6 = (shortk == 1 || shortk == 3) ? 1 : 0;
      if (shortk == 1 && fp.sel_direct && fp.sel_win) {   // k_short KR 5's stage of kept values
        fp.win_stage = fp.wave_lds;
        fp.wave_lds += (int32_t)align16(64 * WIN_LDS * 8);
      }
      if (shortk == 1 && fp.sel_direct && fp.sel_cols && !fp.sel_win && K <= 64) {   // k_short's column stage
        fp.sel_stage = fp.wave_lds;
        fp.wave_lds += (int32_t)align16(2 * 8 * K * 8);   // two stages of 8 series (k_short KR 4)

      }
      fp.waves = (int)std::max<int64_t>(1, std::min<int64_t>(4, (64 * 1024) / fp.wave_lds));
      fp.tile_list = list;
      fp.tile_list_n = list_n;
      fp.n_launch = cap;
      fp.redo_list = out;
      fp.redo_n = out_n;
      hipError_t e = launch_fast(fp, P.f, qw, vl, c->stream);
      if (e != hipSuccess) return fail(TSDB_E_HIP, std::string("launch_fast: ") + hipGetErrorString(e));
      return 0;
    };
    // lists that no fast kernel takes go to k_grid: collect them
    std::vector<std::pair<const int32_t*, std::pair<const int32_t*, int64_t>>> to_grid;
    int32_t* r1[2] = {c->r1a.as<int32_t>(), c->r1b.as<int32_t>()};
    int32_t* r3[2] = {c->r3a.as<int32_t>(), c->r3b.as<int32_t>()};
    int64_t routed = 0;   // tiles of host lists sent straight to k_grid
    if (none) {
      // NONE aggregator: one tile per series (not the group tiles the lists index) --
      // class A over every tile, class B over what A handed back
      int rc = fast_launch(0, 0, nullptr, nullptr, nt, r1[0], rn + 0);
      if (rc < 0) return rc;
      const bool a = rc == 0;
      rc = fast_launch(1, 0, a ? r1[0] : nullptr, a ? rn + 0 : nullptr, nt, c->r2.as<int32_t>(), rn + 2);
      if (rc < 0) return rc;
      if (rc == 1) {
        if (a) to_grid.push_back({r1[0], {rn + 0, nt}});
        else return fail(TSDB_E_HIP, "no fast class ran");   // unreachable: `fast` needs one
      }
    }
    for (int cls = 0; cls < 2 && !none; cls++) {
      const int64_t n0 = (int64_t)c->tl[cls][0].size(), n1 = (int64_t)c->tl[cls][1].size();
      const int64_t n2 = (int64_t)c->tl[cls][2].size();
      const int32_t* l0 = dl + c->tl_off[3 * cls];
      const int32_t* l1 = dl + c->tl_off[3 * cls + 1];
      const int32_t* l2 = dl + c->tl_off[3 * cls + 2];
      const int32_t* dn0 = dn + 3 * cls;
      const int32_t* dn1 = dn + 3 * cls + 1;
      const int32_t* dn2 = dn + 3 * cls + 2;
      int rc;
      if (hwin) {   // k_hwin over the one-chunk-row tiles (hwin_slots: no other tiles); k_grid takes what it hands back
        if (cls == 0) {   // (a tile's work items hand it back once: zeroed marks for both classes' launches)
          HIP_OK(c->hw_mark.ensure(std::max<int64_t>(1, nt) * 4));
          HIP_OK(hipMemsetAsync(c->hw_mark.p, 0, std::max<int64_t>(1, nt) * 4, c->stream));
        }
        for (int part = 1; part <= 2; part++) {
          const int64_t nn = part == 1 ? n1 : n2;
          if (!nn) continue;
          rc = fast_launch(cls, 3, part == 1 ? l1 : l2, part == 1 ? dn1 : dn2, nn, c->r2.as<int32_t>(), rn + 2);
          if (rc < 0) return rc;
          if (rc == 1) { to_grid.push_back({part == 1 ? l1 : l2, {part == 1 ? dn1 : dn2, nn}}); routed += nn; }
        }
        continue;
      }
      if (use_rows && n2) {
        rc = fast_launch(cls, 2, l2, dn2, n2, r3[cls], rn + 3 + cls);
        if (rc < 0) return rc;
        if (rc == 0) {
          rc = fast_launch(cls, 0, r3[cls], rn + 3 + cls, n2, c->r2.as<int32_t>(), rn + 2);
          if (rc < 0) return rc;
          if (rc == 1) to_grid.push_back({r3[cls], {rn + 3 + cls, n2}});
        } else {
          to_grid.push_back({l2, {dn2, n2}});
          routed += n2;
        }
      } else if (n2) {
        rc = fast_launch(cls, 0, l2, dn2, n2, c->r2.as<int32_t>(), rn + 2);
        if (rc < 0) return rc;
        if (rc == 1) { to_grid.push_back({l2, {dn2, n2}}); routed += n2; }
      }
      if (use_short && n1) {
        rc = fast_launch(cls, 1, l1, dn1, n1, r1[cls], rn + cls);
        if (rc < 0) return rc;
        if (rc == 0) {
          rc = fast_launch(cls, 0, r1[cls], rn + cls, n1, c->r2.as<int32_t>(), rn + 2);
          if (rc < 0) return rc;
          if (rc == 1) to_grid.push_back({r1[cls], {rn + cls, n1}});
        } else {
          to_grid.push_back({l1, {dn1, n1}});
          routed += n1;
        }
      } else if (n1) {
        rc = fast_launch(cls, 0, l1, dn1, n1, c->r2.as<int32_t>(), rn + 2);
        if (rc < 0) return rc;
        if (rc == 1) { to_grid.push_back({l1, {dn1, n1}}); routed += n1; }
      }
      if (n0) {
        rc = fast_launch(cls, 0, l0, dn0, n0, c->r2.as<int32_t>(), rn + 2);
        if (rc < 0) return rc;
        if (rc == 1) { to_grid.push_back({l0, {dn0, n0}}); routed += n0; }
      }
    }
    to_grid.push_back({c->r2.as<int32_t>(), {rn + 2, nt}});
    if (!none && !c->tl_other.empty()) to_grid.push_back({dl + c->tl_off[6], {dn + 6, (int64_t)c->tl_other.size()}});
    HIP_OK(hipEventRecord(c->ev[3], c->stream));
    for (auto& tg : to_grid) {
      if (P.multi) break;   // the caller checks that nothing was handed back (else separate passes)
      GridParams g2 = gp;
      g2.tile_list = tg.first;
      g2.tile_list_n = tg.second.first;
      g2.n_launch = tg.second.second;
      HIP_OK(launch_grid(g2, P.f, c->stream));
    }
    c->redo_final = rn + 2;
    c->redo_other = none ? 0 : (int64_t)c->tl_other.size() + routed;
  } else {
    HIP_OK(launch_grid(gp, P.f, c->stream));
  }
  HIP_OK(hipEventRecord(c->ev[1], c->stream));
  }
  if (do_reduce) {
    ReduceParams rp{};
    rp.part = gp.part;
    rp.group_tile_ptr = (none ? c->n_gtp : c->d_gtp).as<int64_t>();
    rp.G = G;
    rp.K = K;
    rp.ga = P.ga;
    rp.out_val = c->out_val.as<double>();
    rp.out_flag = c->out_flag.as<uint8_t>();
    rp.err = c->err.as<int32_t>();
    rp.no_inf = P.no_inf ? 1 : 0;
    HIP_OK(launch_reduce(rp, c->stream));
  }
  HIP_OK(hipEventRecord(c->ev[2], c->stream));
  return 0;
}

// Raw datapoints and algorithmic HBM bytes of the query:
//   per row in the scan range: qualifier bytes + value bytes (incl. the meta byte)
//                              + 4 B base time + 2 x 8 B CSR offsets;  per series: 4 B group id.
// Cached per scan range (the batch is resident; the loop is O(rows)).
void account(tsdbhip_ctx* c, const Plan& P) {
  if (c->acct_valid && c->acct_ss == P.ss && c->acct_se == P.se && c->acct_none == P.none) {
    c->timing.datapoints = c->acct_dps;
    c->timing.bytes = c->acct_bytes;
    return;
  }
  int64_t dps = 0, bytes = 0;
  for (int64_t s = 0; s < c->n_series; s++) {
    if (!P.none && c->h_group[s] >= c->n_groups) continue;   // ungrouped: only NONE reads it
    bytes += 4;
    for (int64_t r = c->h_srp[s]; r < c->h_srp[s + 1]; r++) {
      if ((int64_t)c->h_base[r] < P.ss || (int64_t)c->h_base[r] >= P.se) continue;
      dps += c->h_ndp[r];
      bytes += (int64_t)c->h_qlen[r] + c->h_vlen[r] + 4 + 16;
    }
  }
  c->acct_valid = true;
  c->acct_none = P.none;
  c->acct_ss = P.ss;
  c->acct_se = P.se;
  c->acct_dps = dps;
  c->acct_bytes = bytes;
  c->timing.datapoints = dps;
  c->timing.bytes = bytes;
}

// Result blocks.  Large results are device-to-host copies of up to GBs (the raw path writes
// the result arrays on the device): a D2H copy into pageable memory goes through a staging
// bounce at a fraction of the link rate, so blocks of >= 1 MB come from a process-wide pool of
// pinned (hipHostMalloc) blocks, returned to it by tsdbhip_result_free and reused by the next
// query instead of being pinned anew.  A header before the result records the block's origin.
struct ResultHeader {
  uint64_t magic;       // RESULT_MAGIC
  uint64_t capacity;    // block bytes (header included)
  uint64_t pinned;      // 1: from the pinned pool
  uint64_t pad;
};
constexpr uint64_t RESULT_MAGIC = 0x7473646268697052ULL;
constexpr size_t PINNED_MIN = 1 << 20;
constexpr size_t POOL_MAX = (size_t)8 << 30;   // bytes kept pinned while unused
constexpr size_t PIN_ASYNC_MIN = (size_t)64 << 20;   // blocks pinned by a helper thread instead of in the call

struct PinnedPool {
  std::mutex mu;
  std::vector<std::pair<size_t, void*>> free_blocks;   // (capacity, block)
  size_t held = 0;
  void* take(size_t bytes, size_t& cap) {
    {
      std::lock_guard<std::mutex> lk(mu);
      size_t best = SIZE_MAX;
      for (size_t i = 0; i < free_blocks.size(); i++)
        if (free_blocks[i].first >= bytes && (best == SIZE_MAX || free_blocks[i].first < free_blocks[best].first)) best = i;
      if (best != SIZE_MAX && free_blocks[best].first <= 4 * bytes + PINNED_MIN) {
        void* b = free_blocks[best].second;
        cap = free_blocks[best].first;
        held -= cap;
        free_blocks.erase(free_blocks.begin() + (long)best);
        return b;
      }
    }
    cap = PINNED_MIN;
    while (cap < bytes) cap <<= 1;
    if (cap >= PIN_ASYNC_MIN) {
      // pinning hundreds of MB takes ~0.5 ms a MB (a config-4 raw result, 570 MB: 250 ms in the
      // call): this result takes pageable memory, and a helper thread pins a block of its size
      // for the pool, so the following queries find one
      pin_async(cap);
      return nullptr;
    }
    void* b = nullptr;
    if (hipHostMalloc(&b, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
    return b;
  }
  void pin_async(size_t cap) {
    {
      std::lock_guard<std::mutex> lk(mu);
      if (pinning) return;   // one at a time
      pinning = true;
    }
    try {
      std::thread([this, cap] {
        void* b = nullptr;
        const bool ok = hipHostMalloc(&b, cap, hipHostMallocDefault) == hipSuccess;
        if (ok) give(b, cap);
        std::lock_guard<std::mutex> lk(mu);
        pinning = false;
      }).detach();
    } catch (const std::exception&) {
      std::lock_guard<std::mutex> lk(mu);
      pinning = false;
    }
  }
  bool pinning = false;
  void give(void* b, size_t cap) {
    std::lock_guard<std::mutex> lk(mu);
    while (held + cap > POOL_MAX && !free_blocks.empty()) {   // drop the oldest blocks
      (void)hipHostFree(free_blocks.front().second);
      held -= free_blocks.front().first;
      free_blocks.erase(free_blocks.begin());
    }
    if (cap > POOL_MAX) { (void)hipHostFree(b); return; }
    free_blocks.push_back({cap, b});
    held += cap;
  }
};
PinnedPool& pinned_pool() {
  static PinnedPool* pool = new PinnedPool();   // never destroyed: results may outlive every context
  return *pool;
}

void result_free(tsdbhip_result* r) {
  if (!r) return;
  auto* h = reinterpret_cast<ResultHeader*>(reinterpret_cast<char*>(r) - sizeof(ResultHeader));
  if (h->magic != RESULT_MAGIC) return;   // not ours
  h->magic = 0;
  if (h->pinned) pinned_pool().give(h, h->capacity);
  else std::free(h);
}

tsdbhip_result* make_result(int64_t n_groups, int64_t n_points) {
  const size_t bytes = sizeof(ResultHeader) + sizeof(tsdbhip_result) + (n_groups + 1) * 4 + (n_groups + 1) * 8 +
                       (n_points + 1) * 8 * 2 + (n_points + 1) + 64;
  // every array is fully written by the callers: no zero fill (results can be GBs)
  size_t cap = bytes;
  bool pinned = false;
  char* blk = nullptr;
  if (bytes >= PINNED_MIN) {
    blk = (char*)pinned_pool().take(bytes, cap);
    pinned = blk != nullptr;
  }
  if (!blk) {
    cap = bytes;
    blk = (char*)std::malloc(bytes);
  }
  if (!blk) return nullptr;
  auto* h = reinterpret_cast<ResultHeader*>(blk);
  h->magic = RESULT_MAGIC;
  h->capacity = cap;
  h->pinned = pinned ? 1 : 0;
  char* m = blk + sizeof(ResultHeader);
  std::memset(m, 0, sizeof(tsdbhip_result));
  auto* r = reinterpret_cast<tsdbhip_result*>(m);
  char* p = m + sizeof(tsdbhip_result);
  auto al8 = [&](char* x) { return (char*)(((uintptr_t)x + 7) & ~(uintptr_t)7); };
  p = al8(p);
  r->group_ptr = (const int64_t*)p; p += (n_groups + 1) * 8;
  r->ts_ms = (const int64_t*)p; p += (n_points + 1) * 8;
  r->value_bits = (const uint64_t*)p; p += (n_points + 1) * 8;
  r->group_id = (const int32_t*)p; p += (n_groups + 1) * 4;
  r->is_int = (const uint8_t*)p;
  r->n_groups = n_groups;
  return r;
}

// Persistent host helpers of the result assembly, one pool per process: a multi-device context
// assembles on every device worker at once, and spawning up to 8 threads per call there meant up
// to 64 thread creations a query (and a std::system_error across the C ABI when one failed).  One
// caller uses the pool at a time; a concurrent caller, or any caller when no helper thread could
// be created, runs its items inline.
class AssemblyPool {
 public:
  static AssemblyPool& get() {
    // never destroyed: a condition variable destroyed at exit while the detached helpers wait on
    // it blocks the exiting process (glibc pthread_cond_destroy)
    static AssemblyPool* p = new AssemblyPool();
    return *p;
  }
  // fn(t) for t in [0, nt) with t = 0 on the calling thread; false when the pool is busy
  bool run(int nt, const std::function<void(int)>& fn) {
    if (getpid() != pid_) return false;   // a forked child: the helpers live in the parent only
    std::unique_lock<std::mutex> call(call_mu_, std::try_to_lock);
    if (!call.owns_lock()) return false;
    nt = std::min<int>(nt, 1 + (int)th_.size());
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &fn;
      nt_ = nt;
      pending_ = nt - 1;
      gen_++;
    }
    cv_.notify_all();
    fn(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [this] { return pending_ == 0; });
    job_ = nullptr;
    return true;
  }
  int width() const { return 1 + (int)th_.size(); }

 private:
  AssemblyPool() : pid_(getpid()) {
    const int hw = std::max(1, std::min(8, (int)std::thread::hardware_concurrency()));
    try {
      for (int t = 1; t < hw; t++) th_.emplace_back([this, t] { loop(t); });
    } catch (const std::exception&) {   // fewer helpers (or none): run() narrows nt
    }
    for (auto& t : th_) t.detach();   // process lifetime (no join at static destruction)
  }
  void loop(int t) {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return gen_ != seen; });
      seen = gen_;
      if (t >= nt_) continue;
      const std::function<void(int)>* fn = job_;
      lk.unlock();
      (*fn)(t);
      lk.lock();
      if (--pending_ == 0) done_.notify_all();
    }
  }
  std::mutex call_mu_, mu_;
  std::condition_variable cv_, done_;
  std::vector<std::thread> th_;
  const std::function<void(int)>* job_ = nullptr;
  int nt_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  const pid_t pid_;
};

// n work items over up to 8 host threads when the work is large (a day of 1m buckets over 1000
// groups is 1.4M points: 1.6 ms single-threaded), else inline
template <class Fn>
void par_groups(int64_t n, int64_t work, Fn&& fn) {
  AssemblyPool& pool = AssemblyPool::get();
  const int64_t nt = work >= (1 << 18) ? std::min<int64_t>(pool.width(), n) : 1;
  if (nt > 1) {
    const std::function<void(int)> chunk = [&](int t) {
      for (int64_t i = t * n / nt; i < (t + 1) * n / nt; i++) fn(i);
    };
    if (pool.run((int)nt, chunk)) return;
  }
  for (int64_t i = 0; i < n; i++) fn(i);
}

int assemble(tsdbhip_ctx* c, const tsdbhip_query* q, const Plan& P, int64_t G, const double* val,
             const uint8_t* flag, const std::vector<uint32_t>& act, tsdbhip_result** out) {
  const int64_t K = P.K;
  // group emission order: batch group id order; NONE: span order (original series order)
  std::vector<std::pair<int64_t, int64_t>> groups;  // (result group id, row in dense output)
  if (P.none) {
    std::vector<std::pair<int64_t, int64_t>> tmp;
    for (int64_t g = 0; g < G; g++) if (act[g]) tmp.push_back({c->h_orig[g], g});
    std::sort(tmp.begin(), tmp.end());
    for (size_t i = 0; i < tmp.size(); i++) groups.push_back({c->none_orig ? tmp[i].first : (int64_t)i, tmp[i].second});
  } else {
    for (int64_t g = 0; g < G; g++) if (act[g]) groups.push_back({g, g});
  }
  const int64_t ng = (int64_t)groups.size();
  std::vector<int64_t> off(ng + 1, 0);
  par_groups(ng, ng * K, [&](int64_t i) {
    const uint8_t* f = flag + groups[i].second * K;
    int64_t n = 0;
    for (int64_t k = 0; k < K; k++) n += f[k] ? 1 : 0;
    off[i + 1] = n;
  });
  for (int64_t i = 0; i < ng; i++) off[i + 1] += off[i];
  tsdbhip_result* r = make_result(ng, off[ng]);
  if (!r) return fail(TSDB_E_NOMEM, "result allocation");
  auto* gptr = const_cast<int64_t*>(r->group_ptr);
  auto* gid = const_cast<int32_t*>(r->group_id);
  auto* ts = const_cast<int64_t*>(r->ts_ms);
  auto* vb = const_cast<uint64_t*>(r->value_bits);
  auto* isi = const_cast<uint8_t*>(r->is_int);
  par_groups(ng, off[ng], [&](int64_t i) {
    int64_t o = off[i];
    gptr[i] = o;
    gid[i] = (int32_t)groups[i].first;
    const int64_t row = groups[i].second;
    const uint8_t* f = flag + row * K;
    const double* v = val + row * K;
    if (off[i + 1] - o == K && P.mode != MODE_ALL && P.mode != MODE_TABLE) {   // every slot emitted: straight copies
      std::memcpy(&vb[o], v, K * 8);
      for (int64_t k = 0; k < K; k++) ts[o + k] = P.B0 + k * P.I;
      std::memset(&isi[o], 0, K);
      return;
    }
    for (int64_t k = 0; k < K; k++) {
      if (!f[k]) continue;
      // only points inside [start_time, end_time] of the SpanGroup are produced (x <= end_time)
      ts[o] = (P.mode == MODE_ALL) ? q->start_time : (P.mode == MODE_TABLE ? P.bounds[k] : P.B0 + k * P.I);
      std::memcpy(&vb[o], &v[k], 8);
      isi[o] = 0;   // downsampled values are always doubles (Downsampler.isInteger, :259-262)
      o++;
    }
  });
  gptr[ng] = off[ng];
  *out = r;
  return 0;
}

}  // namespace

namespace {

// Device timings of the last run (events recorded by run_device).
// Percentile / median as the group-by aggregator (downsampled queries):
//  1. every series' bucket values: k_pct for a percentile / median downsample function,
//     else a NONE-aggregator pass without rate (= each span's Downsampler output);
//  2. k_emit_vals: the SpanGroup contributions (rate, fill, LERP) per (series, slot);
//  3. k_sel_seg: runDouble's order statistic per (group, slot) by radix select.
// Group -> first value of its segments in the [g][k][i] layout: prefix of `counts`.
std::vector<int64_t> seg_ptr(const std::vector<int64_t>& counts) {
  std::vector<int64_t> gsp(counts.size() + 1, 0);
  for (size_t g = 0; g < counts.size(); g++) gsp[g + 1] = gsp[g] + counts[g];
  return gsp;
}

// local series per group id g < G (resident order is group-sorted); cached per loaded batch
const std::vector<int64_t>& local_counts(tsdbhip_ctx* c, int64_t G) {
  if (c->lc_valid && (int64_t)c->lc.size() == G) return c->lc;
  std::vector<int64_t>& n = c->lc;
  n.assign(G, 0);
  for (int64_t s = 0; s < c->n_series; s++)
    // ungrouped series carry the LOCAL sentinel group n_groups, which can be a real group id
    // of a wider (global) numbering: not one of its groups
    if (c->h_group[s] < c->n_groups && c->h_group[s] < G) n[c->h_group[s]]++;
  c->lc_valid = true;
  return n;
}

// Stages 1-2 of the percentile / median group-by: every local span's contribution to each
// (group, slot) into c->sel_vals ([series][K], NaN = none), c->sel_uni [G][K], c->gact [G].
// When the query allows it (no rate, K <= 64, not a percentile downsampling) the downsampling
// pass writes the contributions itself (GridParams.sel_direct): no bucket values round-trip
// through pre_dense and no k_emit_vals pass.
int sel_values(tsdbhip_ctx* c, const tsdbhip_query* q, const Plan& P, int64_t G, bool* cols_out = nullptr) {
  const int64_t S = c->n_series, K = P.K;
  if (S * K > 0x7FFFFFFFLL) return fail(TSDB_E_NOT_IMPLEMENTED, "percentile group-by over more than 2^31 (series, slot) values");
  if (P.f != F_SEL && !P.emit_only && !q->rate && K >= 1 && K <= 64 && !opt_off(OPT_SEL_FUSED)) {
    const std::vector<int64_t> gsp = seg_ptr(local_counts(c, G));
    HIP_OK(c->sel_gsp.ensure((G + 1) * 8));
    HIP_OK(c->sel_vals.ensure(std::max<int64_t>(1, S * K) * 8));
    HIP_OK(c->sel_uni.ensure(std::max<int64_t>(1, G * K)));
    HIP_OK(hipMemcpyAsync(c->sel_gsp.p, gsp.data(), (G + 1) * 8, hipMemcpyHostToDevice, c->stream));
    // a written-row flag per series, and the no-value pattern afterwards only into the rows
    // the pass did not write (config 3: 10 MB of flags instead of filling 4.8 GB up front)
    HIP_OK(c->sel_wr.ensure(std::max<int64_t>(1, S)));
    HIP_OK(hipMemsetAsync(c->sel_wr.p, 0, std::max<int64_t>(1, S), c->stream));
    HIP_OK(hipMemsetAsync(c->sel_uni.p, 0, std::max<int64_t>(1, G * K), c->stream));
    Plan P2;
    int rc = plan_query(c, q, P2);
    if (rc) return rc;
    P2.sel_direct = true;
    // the caller that selects right here takes contiguous (group, slot) columns
    P2.sel_cols = cols_out != nullptr && !opt_off(OPT_SEL_COLS);
    rc = run_device(c, q, P2, G, false);   // sets c->gact like the group-by pass
    if (rc) return rc;
    HIP_OK(launch_fill_rows(c->sel_vals.as<uint64_t>(), c->sel_wr.as<uint8_t>(), S, K, 0x7FF87FF87FF87FF8ULL, c->stream,
                            P2.sel_cols ? c->sel_gsp.as<int64_t>() : nullptr, G));
    if (cols_out) *cols_out = P2.sel_cols;
    HIP_OK(hipStreamSynchronize(c->stream));   // `gsp` leaves scope
    return 0;
  }
  HIP_OK(c->pre_dense.ensure(std::max<int64_t>(1, S * K) * 8));
  HIP_OK(c->pre_pres.ensure(std::max<int64_t>(1, S * K)));
  if (P.emit_only) {
    // the buckets are already in pre_dense / pre_pres: a rollup table's avg / count downsampling
    // (ro_stage: Σsum / Σcount per bucket, Downsampler.java:165-221)
  } else if (P.f == F_SEL) {
    int rc = run_device(c, q, P, G, false);   // k_pct -> pre_dense / pre_pres (no k_emit)
    if (rc) return rc;
  } else {
    // the grid kernels over the group tiles, each series' Downsampler output (no rate: the
    // SpanGroup step below applies it) written to pre_dense / pre_pres
    tsdbhip_query q2 = *q;
    q2.rate = 0;
    Plan P2;
    int rc = plan_query(c, &q2, P2);
    if (rc) return rc;
    P2.dense_out = true;
    rc = run_device(c, &q2, P2, G, false);
    if (rc) return rc;
  }
  const std::vector<int64_t> gsp = seg_ptr(local_counts(c, G));
  HIP_OK(c->sel_gsp.ensure((G + 1) * 8));
  HIP_OK(c->sel_vals.ensure(std::max<int64_t>(1, S * K) * 8));
  HIP_OK(c->sel_uni.ensure(std::max<int64_t>(1, G * K)));
  HIP_OK(c->gact.ensure(std::max<int64_t>(1, G) * 4));
  HIP_OK(hipMemcpyAsync(c->sel_gsp.p, gsp.data(), (G + 1) * 8, hipMemcpyHostToDevice, c->stream));
  HIP_OK(launch_fill64(c->sel_vals.as<uint64_t>(), 0x7FF87FF87FF87FF8ULL, S * K, c->stream));   // +NaN
  HIP_OK(hipMemsetAsync(c->sel_uni.p, 0, std::max<int64_t>(1, G * K), c->stream));
  HIP_OK(hipMemsetAsync(c->gact.p, 0, std::max<int64_t>(1, G) * 4, c->stream));
  const int64_t nt = (int64_t)c->tb.size();
  GridParams gp{};
  gp.rows = c->rows.as<RowDesc>();
  gp.series_row_ptr = c->srp.as<int64_t>();
  gp.tile_begin = c->d_tb.as<int64_t>();
  gp.tile_end = c->d_te.as<int64_t>();
  gp.tile_group = c->d_tg.as<int32_t>();
  gp.n_tiles = nt;
  gp.ss = P.ss;
  gp.se = P.se;
  gp.B0 = P.B0;
  gp.I = P.I;
  gp.K = K;
  gp.qs = q->start_time;
  gp.qe = q->end_time;
  gp.mode = P.mode;
  gp.seek_any = seek_point(P);
  gp.ga = P.ga;
  gp.interp = P.interp;
  gp.fill = q->ds_fill;
  if (P.mode == MODE_TABLE) {
    HIP_OK(c->cal_bounds.ensure((int64_t)P.bounds.size() * 8));
    HIP_OK(hipMemcpyAsync(c->cal_bounds.p, P.bounds.data(), P.bounds.size() * 8, hipMemcpyHostToDevice, c->stream));
    gp.bounds = c->cal_bounds.as<int64_t>();
    gp.seek_ms = P.seek;
    gp.skip0 = P.bounds[0] < P.ss * 1000 ? 1 : 0;
  }
  gp.rate = q->rate;
  gp.counter = q->rate_counter;
  gp.drop = q->rate_drop_resets;
  gp.counter_max = q->rate_counter_max;
  gp.reset_value = q->rate_reset_value;
  gp.pre_dense = c->pre_dense.as<double>();
  gp.pre_pres = c->pre_pres.as<uint8_t>();
  gp.sel_vals = c->sel_vals.as<double>();
  gp.sel_uni = c->sel_uni.as<uint8_t>();
  gp.group_series_ptr = c->sel_gsp.as<int64_t>();
  gp.group_active = c->gact.as<uint32_t>();
  gp.err = c->err.as<int32_t>();
  gp.wave_lds = q->rate ? (int32_t)align16(K * 8) : 16;
  if (gp.wave_lds > 48 * 1024) {
    HIP_OK(c->g_rate.ensure(std::max<int64_t>(1, nt * K) * 8));
    gp.g_rate = c->g_rate.as<double>();
    gp.wave_lds = 16;
  }
  gp.waves = (int)std::max<int64_t>(1, std::min<int64_t>(4, (64 * 1024) / gp.wave_lds));
  HIP_OK(launch_emit_vals(gp, c->stream));
  c->fast_used = false;
  return 0;
}

// Stage 3: the order statistic of every (group, slot) column of `vals` (device,
// [series][K] with counts[g] series in group g) -> c->out_val / c->out_flag [G][K].
int sel_select(tsdbhip_ctx* c, const Plan& P, int64_t G, double* vals, const std::vector<int64_t>& counts,
               const uint8_t* uni, bool cols = false) {
  const int64_t K = P.K;
  const std::vector<int64_t> gsp = seg_ptr(counts);
  int64_t maxn = 0;
  for (int64_t g = 0; g < G; g++) maxn = std::max(maxn, counts[g]);
  HIP_OK(c->sel_gsp.ensure((G + 1) * 8));
  HIP_OK(c->out_val.ensure(std::max<int64_t>(1, G * K) * 8));
  HIP_OK(c->out_flag.ensure(std::max<int64_t>(1, G * K)));
  if (maxn > SEL_CAP) HIP_OK(c->sel_sorted.ensure(std::max<int64_t>(1, gsp[G] * K) * 8));   // key space
  HIP_OK(hipMemcpyAsync(c->sel_gsp.p, gsp.data(), (G + 1) * 8, hipMemcpyHostToDevice, c->stream));
  SelParams sp{};
  sp.vals = vals;
  sp.cols = cols ? 1 : 0;
  sp.scratch = maxn > SEL_CAP ? c->sel_sorted.as<double>() : nullptr;
  sp.uni = uni;
  sp.group_series_ptr = c->sel_gsp.as<int64_t>();
  sp.G = G;
  sp.K = K;
  sp.fn = P.gsel;
  sp.out_val = c->out_val.as<double>();
  sp.out_flag = c->out_flag.as<uint8_t>();
  sp.err = c->err.as<int32_t>();
  HIP_OK(launch_sel_seg(sp, c->stream, maxn));
  return 0;
}

// The sampled window (percentile / median group-by over the streaming kernels' short tiles, §5.5):
//  1. the sample pass: k_short KR 4 over every stride-th tile of each group (the column layout at
//     those tiles' positions; ~max(640, n_g / 16) sampled series a group);
//  2. k_win_bounds: per (group, slot) column, a window [lo, hi] around the target ranks from the
//     sample (binomial margin);
//  3. the main pass: k_short KR 5 over every tile: each contribution counted below / above the
//     window, or kept; at the tile's end its counts go to the column's (atomics) and its kept
//     values to the column's candidates (a cursor, at most WIN_CCAP a column);
//  4. k_win_select: exact counts -> the ranks; where the window holds them, the select over the
//     kept values -- the full path's values and ranks, so its result.
// *done = false: the batch or query does not qualify, a tile was handed back, or a column's
// window missed (k_win_select's fail flag): the caller runs the full path.
// the quantile of a percentile function id (ksel.h pct_quantile)
double pct_quantile_host(int fn) {
  const int i = (fn - TSDB_AGG_P999) % 6;
  return i == 0 ? 99.9 : i == 1 ? 99.0 : i == 2 ? 95.0 : i == 3 ? 90.0 : i == 4 ? 75.0 : 50.0;
}

int sel_window(tsdbhip_ctx* c, const tsdbhip_query* q, const Plan& P, int64_t G, bool* done) {
  *done = false;
  if (opt_off(OPT_SEL_WIN)) return 0;   // option SEL_WIN: 0 never; 2 also for small groups (tests)
  const int64_t S = c->n_series, K = P.K;
  if (P.f == F_SEL || P.emit_only || q->rate || K < 1 || K > 64 || P.none || !P.gsel || G < 1) return 0;
  // ranks near the ends only (p90 and up): a window around the median keeps ~a quarter of the
  // values and measured slower than the full path (config 3 median:1m-avg 8.85 vs 7.24 ms)
  if (!(P.gsel != TSDB_AGG_MEDIAN && pct_quantile_host(P.gsel) >= 90.0) && !opt_is(OPT_SEL_WIN, 2)) return 0;
  if (!c->tl_other.empty()) return 0;
  int64_t nshort = 0;
  for (int cls = 0; cls < 2; cls++) {
    if (!c->tl[cls][0].empty() || !c->tl[cls][2].empty()) return 0;
    nshort += (int64_t)c->tl[cls][1].size();
  }
  if (nshort == 0 || nshort != (int64_t)c->tb.size()) return 0;
  const std::vector<int64_t> counts = local_counts(c, G);
  int64_t maxn = 0;
  for (int64_t g = 0; g < G; g++) maxn = std::max(maxn, counts[g]);
  if (maxn < 4096 && !opt_is(OPT_SEL_WIN, 2)) return 0;   // small groups: the full path is cheap
  Plan P2;
  int rc = plan_query(c, q, P2);
  if (rc) return rc;
  P2.sel_direct = true;
  P2.sel_cols = true;
  if (!fast_path_ok(c, q, P2)) return 0;
  // sampled tiles, by group and by class (a short tile is in one class list)
  const int64_t nt = (int64_t)c->tb.size();
  // every stride-th tile of a group, the stride set for ~max(640, n_g / 16) sampled series (at
  // most WIN_SCAP positions a group go to the bounds)
  // (groups whose window would keep more values than a column holds -- the window's width is
  // ~2 x (6 sd + 2) of ~WIN_SCAP sampled ranks: large groups, p95 / p90 -- would fall back every time)
  {
    const double f = pct_quantile_host(P.gsel) / 100.0;
    for (int64_t g = 0; g < G; g++) {
      const double ng = (double)counts[g];
      const double ns = std::min<double>(WIN_SCAP, std::max<double>(640.0, ng / 16.0));
      if (ng >= 64 && ng * 2.0 * (6.0 * std::sqrt(ns * f * (1.0 - f)) + 2.0) / ns > 0.7 * WIN_CCAP &&
          !opt_is(OPT_SEL_WIN, 2))
        return 0;
    }
  }
  std::vector<uint8_t> samp(nt, 0);
  std::vector<int32_t> sptr(G + 1, 0), spos;
  for (int64_t g = 0; g < G; g++) {
    sptr[g] = (int32_t)spos.size();
    const int64_t a = c->gtp[g], b = c->gtp[g + 1], ntg = b - a;
    if (ntg <= 0) continue;
    const int64_t g0 = c->tb[a], ng = c->te[b - 1] - g0;
    const int64_t target = std::min<int64_t>(WIN_SCAP, std::max<int64_t>(640, ng / 16));
    const int64_t stride = std::max<int64_t>(1, ng / std::max<int64_t>(1, target));
    int64_t kept = 0;
    for (int64_t t = a; t < b && kept < WIN_SCAP; t += stride) {
      samp[t] = 1;
      for (int64_t s = c->tb[t]; s < c->te[t] && kept < WIN_SCAP; s++, kept++) spos.push_back((int32_t)(s - g0));
    }
  }
  sptr[G] = (int32_t)spos.size();
  std::vector<int32_t> sl[2];
  for (int cls = 0; cls < 2; cls++)
    for (const int32_t t : c->tl[cls][1])
      if (samp[t]) sl[cls].push_back(t);
  std::vector<int32_t> all(sl[0]);
  all.insert(all.end(), sl[1].begin(), sl[1].end());
  const int32_t ncnt[7] = {0, (int32_t)sl[0].size(), 0, 0, (int32_t)sl[1].size(), 0, 0};
  HIP_OK(c->samp_tl.ensure(std::max<size_t>(1, all.size()) * 4));
  HIP_OK(c->samp_tl_n.ensure(8 * 4));
  HIP_OK(c->samp_tiles.ensure(std::max<size_t>(1, spos.size()) * 4));
  HIP_OK(c->samp_ptr.ensure((G + 1) * 4));
  if (!all.empty()) HIP_OK(hipMemcpyAsync(c->samp_tl.p, all.data(), all.size() * 4, hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipMemcpyAsync(c->samp_tl_n.p, ncnt, 7 * 4, hipMemcpyHostToDevice, c->stream));
  if (!spos.empty()) HIP_OK(hipMemcpyAsync(c->samp_tiles.p, spos.data(), spos.size() * 4, hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipMemcpyAsync(c->samp_ptr.p, sptr.data(), (G + 1) * 4, hipMemcpyHostToDevice, c->stream));
  // the sample pass's buffers (as sel_values)
  const std::vector<int64_t> gsp = seg_ptr(counts);
  HIP_OK(c->sel_gsp.ensure((G + 1) * 8));
  HIP_OK(c->sel_vals.ensure(std::max<int64_t>(1, S * K) * 8));
  HIP_OK(c->sel_uni.ensure(std::max<int64_t>(1, G * K)));
  HIP_OK(c->sel_wr.ensure(std::max<int64_t>(1, S)));
  HIP_OK(hipMemcpyAsync(c->sel_gsp.p, gsp.data(), (G + 1) * 8, hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipMemsetAsync(c->sel_wr.p, 0, std::max<int64_t>(1, S), c->stream));
  HIP_OK(hipMemsetAsync(c->sel_uni.p, 0, std::max<int64_t>(1, G * K), c->stream));
  {
    // run_device over the sampled tiles: the class lists swapped for the sample's
    std::vector<int32_t> keep[2][3], keep_other;
    int64_t keep_off[7];
    for (int cls = 0; cls < 2; cls++)
      for (int j = 0; j < 3; j++) keep[cls][j].swap(c->tl[cls][j]);
    keep_other.swap(c->tl_other);
    std::memcpy(keep_off, c->tl_off, sizeof(keep_off));
    c->tl[0][1] = sl[0];
    c->tl[1][1] = sl[1];
    const int64_t off[7] = {0, 0, (int64_t)sl[0].size(), (int64_t)sl[0].size(), (int64_t)sl[0].size(),
                            (int64_t)all.size(), (int64_t)all.size()};
    std::memcpy(c->tl_off, off, sizeof(off));
    c->tl_dev_override = c->samp_tl.as<int32_t>();
    c->tln_dev_override = c->samp_tl_n.as<int32_t>();
    rc = run_device(c, q, P2, G, false);
    c->tl_dev_override = nullptr;
    c->tln_dev_override = nullptr;
    for (int cls = 0; cls < 2; cls++)
      for (int j = 0; j < 3; j++) keep[cls][j].swap(c->tl[cls][j]);
    keep_other.swap(c->tl_other);
    std::memcpy(c->tl_off, keep_off, sizeof(keep_off));
    if (rc) return rc;
  }
  // the windows
  c->win_runs++;
  HIP_OK(c->win_lo.ensure(std::max<int64_t>(1, G * K) * 8));
  HIP_OK(c->win_hi.ensure(std::max<int64_t>(1, G * K) * 8));
  HIP_OK(c->win_val.ensure(std::max<int64_t>(1, nt * K * WIN_CAP) * 8));
  HIP_OK(c->win_gcnt.ensure(std::max<int64_t>(1, G * K) * 8));
  HIP_OK(c->win_cur.ensure(std::max<int64_t>(1, G * K) * 4));
  HIP_OK(c->win_cand.ensure(std::max<int64_t>(1, G * K * WIN_CCAP) * 8));
  HIP_OK(c->win_fail.ensure(16));
  HIP_OK(c->out_val.ensure(std::max<int64_t>(1, G * K) * 8));
  HIP_OK(c->out_flag.ensure(std::max<int64_t>(1, G * K)));
  WinParams wp{};
  wp.vals = c->sel_vals.as<double>();
  wp.wr = c->sel_wr.as<uint8_t>();
  wp.group_series_ptr = c->sel_gsp.as<int64_t>();
  wp.tile_begin = c->d_tb.as<int64_t>();
  wp.tile_end = c->d_te.as<int64_t>();
  wp.samp_ptr = c->samp_ptr.as<int32_t>();
  wp.samp_pos = c->samp_tiles.as<int32_t>();
  wp.group_tile_ptr = c->d_gtp.as<int64_t>();
  wp.uni = c->sel_uni.as<uint8_t>();
  wp.lo = c->win_lo.as<double>();
  wp.hi = c->win_hi.as<double>();
  wp.gcnt = c->win_gcnt.as<unsigned long long>();
  wp.cur = c->win_cur.as<uint32_t>();
  wp.cand = c->win_cand.as<double>();
  wp.G = G;
  wp.K = K;
  wp.fn = P.gsel;
  wp.out_val = c->out_val.as<double>();
  wp.out_flag = c->out_flag.as<uint8_t>();
  wp.err = c->err.as<int32_t>();
  wp.fail = c->win_fail.as<int32_t>();

  HIP_OK(launch_win_bounds(wp, c->stream));
  // the main pass (its union flags and activity afresh; the sample pass's start event stands)
  HIP_OK(hipMemsetAsync(c->sel_uni.p, 0, std::max<int64_t>(1, G * K), c->stream));
  HIP_OK(hipMemsetAsync(c->win_fail.p, 0, 4, c->stream));
  HIP_OK(hipMemsetAsync(c->win_gcnt.p, 0, std::max<int64_t>(1, G * K) * 8, c->stream));
  HIP_OK(hipMemsetAsync(c->win_cur.p, 0, std::max<int64_t>(1, G * K) * 4, c->stream));
  Plan P3 = P2;
  P3.sel_win = true;
  P3.split2 = true;
  rc = run_device(c, q, P3, G, false);
  if (rc) return rc;
  const int64_t routed = c->redo_other;
  HIP_OK(launch_win_select(wp, c->stream));
  int32_t fail = 0, hb0 = 0, hb1 = 0;
  {
    int rc_ = d2h_small(c, &fail, c->win_fail.p, 4, c->stream);
    if (!rc_) rc_ = d2h_small(c, &hb0, c->r_n.as<int32_t>() + 0, 4, c->stream);
    if (!rc_) rc_ = d2h_small(c, &hb1, c->r_n.as<int32_t>() + 1, 4, c->stream);
    if (!rc_) rc_ = sync_small(c, c->stream);
    if (rc_) return rc_;
  }
  // (a tile k_short handed back was re-run by k_fast, which writes the column layout, not windows)
  if (fail || hb0 || hb1 || routed) {
    c->win_misses++;
    return 0;
  }
  *done = true;
  return 0;
}

// Percentile / median as the group-by aggregator (downsampled queries):
//  1. every series' bucket values: k_pct for a percentile / median downsample function,
//     else a NONE-aggregator pass without rate (= each span's Downsampler output);
//  2. k_emit_vals: the SpanGroup contributions (rate, fill, LERP) per (series, slot);
//  3. k_sel_seg: runDouble's order statistic per (group, slot) by radix select.
int run_sel_group(tsdbhip_ctx* c, const tsdbhip_query* q, const Plan& P, int64_t G) {
  bool done = false;
  int rc = sel_window(c, q, P, G, &done);
  if (rc) return rc;
  if (!done) {
    bool cols = false;
    rc = sel_values(c, q, P, G, &cols);
    if (rc) return rc;
    rc = sel_select(c, P, G, c->sel_vals.as<double>(), local_counts(c, G), c->sel_uni.as<uint8_t>(), cols);
    if (rc) return rc;
  }
  HIP_OK(hipEventRecord(c->ev[1], c->stream));
  HIP_OK(hipEventRecord(c->ev[2], c->stream));
  return 0;
}

// TSDB_QF_ORDERED: the span values per (group, slot) as for the percentile group-by
// (stages 1-2), then k_ordered folds each (group, slot) over the group's spans in SpanGroup
// index order -- Aggregator.runDouble's operand sequence, so float sums are bit-exact.
int run_ordered(tsdbhip_ctx* c, const tsdbhip_query* q, const Plan& P, int64_t G) {
  int rc = sel_values(c, q, P, G);
  if (rc) return rc;
  HIP_OK(c->out_val.ensure(std::max<int64_t>(1, G * P.K) * 8));
  HIP_OK(c->out_flag.ensure(std::max<int64_t>(1, G * P.K)));
  OrdParams op{};
  op.vals = c->sel_vals.as<double>();
  op.uni = c->sel_uni.as<uint8_t>();
  op.group_series_ptr = c->sel_gsp.as<int64_t>();
  op.G = G;
  op.K = P.K;
  op.ga = P.ga;
  op.out_val = c->out_val.as<double>();
  op.out_flag = c->out_flag.as<uint8_t>();
  op.err = c->err.as<int32_t>();
  HIP_OK(launch_ordered(op, c->stream));
  HIP_OK(hipEventRecord(c->ev[1], c->stream));
  HIP_OK(hipEventRecord(c->ev[2], c->stream));
  return 0;
}

void record_timing(tsdbhip_ctx* c, const Plan& P, int32_t redo_n) {
  float t01 = 0, t12 = 0, t03 = 0;
  (void)hipEventElapsedTime(&t01, c->ev[0], c->ev[1]);
  (void)hipEventElapsedTime(&t12, c->ev[1], c->ev[2]);
  if (c->fast_used) (void)hipEventElapsedTime(&t03, c->ev[0], c->ev[3]);
  c->timing.decode_downsample_ms = t01;
  c->timing.group_reduce_ms = t12;
  c->timing.total_ms = t01 + t12;
  c->timing.fast_ms = t03;
  c->timing.tiles = P.none ? c->n_series : (int64_t)c->tb.size();
  c->timing.redo_tiles = c->fast_used ? redo_n + c->redo_other : c->timing.tiles;
  c->timing.fused_queries = c->fused_n;
  account(c, P);
}

// Dense [G][K] outputs on the device -> result (after the stream's work is queued).
void ro_activity(const tsdbhip_ctx* c, const Plan& P, int64_t G, std::vector<uint32_t>& act);

// TSDBHIP_TRACE=1: host wall time of a query's phases on stderr (diagnostics only)
struct PhaseTrace {
  bool on;
  const char* name;
  std::chrono::steady_clock::time_point t0, last;
  explicit PhaseTrace(const char* n) : on(opt_is(OPT_TRACE, 1)), name(n) {
    t0 = last = std::chrono::steady_clock::now();
  }
  void mark(const char* what) {
    if (!on) return;
    const auto t = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[trace %s] %-18s %8.3f ms  (total %8.3f)\n", name, what,
                 std::chrono::duration<double, std::milli>(t - last).count(),
                 std::chrono::duration<double, std::milli>(t - t0).count());
    last = t;
  }
};

// The group activity flags, the error code and the hand-back count of a query into page-locked
// memory kept by the context.  (A copy into pageable memory blocks in the runtime until the stream
// has drained, and measured ~0.85 ms a call however little was left to run: rollup avg:1h-avg,
// 0.27 ms of kernels in a 0.99 ms call, profiles/r05ad/ro_api.)
struct SmallD2H {
  uint32_t* act;
  int32_t* err;
  int32_t* redo;
};
int small_d2h(tsdbhip_ctx* c, int64_t G, bool redo, SmallD2H& o) {
  const int64_t g4 = (std::max<int64_t>(1, G) * 4 + 15) & ~(int64_t)15;
  HIP_OK(c->h_small.ensure(g4 + 16));
  char* b = reinterpret_cast<char*>(c->h_small.p);
  o.act = reinterpret_cast<uint32_t*>(b);
  o.err = reinterpret_cast<int32_t*>(b + g4);
  o.redo = o.err + 1;
  *o.err = 0;
  *o.redo = 0;
  if (G) HIP_OK(hipMemcpyAsync(o.act, c->gact.p, G * 4, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(hipMemcpyAsync(o.err, c->err.p, 4, hipMemcpyDeviceToHost, c->stream));
  if (redo) HIP_OK(hipMemcpyAsync(o.redo, c->redo_final, 4, hipMemcpyDeviceToHost, c->stream));
  return 0;
}

int collect(tsdbhip_ctx* c, const tsdbhip_query* q, const Plan& P, int64_t G, bool timed, tsdbhip_result** out,
            const void* d_val = nullptr, const void* d_flag = nullptr) {
  // the dense [G][K] rows land in page-locked staging kept by the context (no zero fill, DMA
  // at the link's rate; a day of 1m buckets over 1000 groups is 13 MB a query)
  const int64_t gk = G * P.K;
  HIP_OK(c->h_stage.ensure(std::max<int64_t>(16, gk * 9 + 16)));
  double* val = reinterpret_cast<double*>(c->h_stage.p);
  uint8_t* flag = reinterpret_cast<uint8_t*>(c->h_stage.p) + gk * 8;
  if (gk) {
    HIP_OK(hipMemcpyAsync(val, d_val ? d_val : c->out_val.p, gk * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipMemcpyAsync(flag, d_flag ? d_flag : c->out_flag.p, gk, hipMemcpyDeviceToHost, c->stream));
  }
  SmallD2H sm;
  int rc0 = small_d2h(c, G, timed && c->fast_used, sm);
  if (rc0) return rc0;
  PhaseTrace tr("collect");
  HIP_OK(hipStreamSynchronize(c->stream));
  std::vector<uint32_t> act(sm.act, sm.act + std::max<int64_t>(1, G));
  const int32_t err = *sm.err, redo_n = *sm.redo;
  tr.mark("device + d2h");
  if (timed) record_timing(c, P, redo_n);
  if (err) return fail(err, "error raised by the device path");
  if (P.mode == MODE_ALL) {
    // AggregationIterator ctor: the single "all" point is skipped unless start_time <= qs <= end_time
    const int64_t S0 = P.ss * 1000, E0 = P.se * 1000;
    if (q->start_time < S0 || q->start_time > E0) std::fill(flag, flag + gk, 0);
  }
  ro_activity(c, P, G, act);
  tr.mark("ro_activity");
  const int rc = assemble(c, q, P, G, val, flag, act, out);
  tr.mark("assemble");
  return rc;
}

}  // namespace

// ---------------------------------------------------------------------------
// raw path (k_raw.hip): no downsampling
// ---------------------------------------------------------------------------
namespace {


// Points handed to the raw evaluator instead of the resident rows' datapoints: each span's
// Downsampler output (run_anchored).  n[s] points of series s, consecutive in pts; live[s] = the
// span has rows in the scan range (its SpanGroup exists even when no bucket survives).
struct RawExt {
  std::vector<int32_t> n;
  std::vector<RawPt> pts;
  std::vector<uint8_t> live;
  bool sec = true;   // every timestamp a whole second
};

int run_raw(tsdbhip_ctx* c, const tsdbhip_query* q, const Plan& P, tsdbhip_result** out, const RawExt* ext = nullptr) {
  PhaseTrace tr("raw");
  const int64_t S = c->n_series;
  const int64_t start = P.ss * 1000, end = P.se * 1000;
  // points of every series inside the scan range (rows with base in [ss, se), Span order)
  std::vector<int64_t> row_pt(std::max<int64_t>(1, c->n_rows), -1), sp_off(S + 1, 0);
  std::vector<int32_t> sp_n(std::max<int64_t>(1, S), 0);
  bool all_s = true, any_int = false, any_float = false;
  bool uns = false;   // a cell with unsorted datapoints: k_raw_merge walks the greedy steps
  int64_t np = 0;
  for (int64_t s = 0; s < S; s++) {
    sp_off[s] = np;
    if (ext) {
      np += ext->n[s];
      sp_n[s] = ext->n[s];
      continue;
    }
    for (int64_t r = c->h_srp[s]; r < c->h_srp[s + 1]; r++) {
      if ((int64_t)c->h_base[r] < P.ss || (int64_t)c->h_base[r] >= P.se) continue;
      const uint32_t f = c->h_flags[r];
      if (f & ROW_UNSORTED) uns = true;
      if ((f & ROW_QW_MASK) != 2) all_s = false;
      if (f & ROW_ALLF) any_float = true;
      else { any_int = true; if (!(f & ROW_ALLI)) any_float = true; }
      row_pt[r] = np;
      np += c->h_ndp[r];
    }
    sp_n[s] = (int32_t)(np - sp_off[s]);
  }
  sp_off[S] = np;
  if (ext) {   // Downsampler outputs: doubles (Downsampler.isInteger :259-262)
    all_s = ext->sec;
    any_float = true;
  }
  // a span counts for its SpanGroup when it has points -- or, for Downsampler outputs, rows
  auto span_live = [&](int64_t s) { return ext ? ext->live[s] != 0 : sp_n[s] > 0; };
  // groups: dense batch groups, or one per span for NONE (TsdbQuery.java:941-962)
  std::vector<int64_t> grp_ser;
  std::vector<int64_t> gid_of;   // result group id of each group row
  if (P.none) {
    std::vector<std::pair<int64_t, int64_t>> tmp;
    for (int64_t s = 0; s < S; s++) if (span_live(s)) tmp.push_back({c->h_orig[s], s});
    std::sort(tmp.begin(), tmp.end());
    // NONE groups must be contiguous series ranges: one series each, in resident order
    grp_ser.resize(S + 1);
    for (int64_t s = 0; s <= S; s++) grp_ser[s] = s;
    gid_of.assign(S, -1);
    for (size_t i = 0; i < tmp.size(); i++) gid_of[tmp[i].second] = c->none_orig ? tmp[i].first : (int64_t)i;
  } else {
    grp_ser.assign(c->n_groups + 1, 0);
    for (int64_t g = 0, s = 0; g < c->n_groups; g++) {
      grp_ser[g] = s;
      while (s < S && c->h_group[s] == g) s++;
      grp_ser[g + 1] = s;
    }
  }
  const int64_t G = (int64_t)grp_ser.size() - 1;
  tr.mark("host spans");
  std::vector<uint8_t> act(std::max<int64_t>(1, G), 0);
  for (int64_t g = 0; g < G; g++)
    for (int64_t s = grp_ser[g]; s < grp_ser[g + 1]; s++) if (span_live(s)) { act[g] = 1; break; }
  // device arrays
  const int64_t R = std::max<int64_t>(1, c->n_rows);
  HIP_OK(c->r_rowpt.ensure(R * 8));
  HIP_OK(c->r_spoff.ensure((S + 1) * 8));
  HIP_OK(c->r_spn.ensure(std::max<int64_t>(1, S) * 4));
  HIP_OK(c->r_grp.ensure((G + 1) * 8));
  HIP_OK(c->r_pts.ensure(std::max<int64_t>(1, np) * sizeof(RawPt)));
  HIP_OK(c->r_rank.ensure(std::max<int64_t>(1, np) * 4));
  HIP_OK(hipMemcpyAsync(c->r_rowpt.p, row_pt.data(), R * 8, hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipMemcpyAsync(c->r_spoff.p, sp_off.data(), (S + 1) * 8, hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipMemcpyAsync(c->r_spn.p, sp_n.data(), std::max<int64_t>(1, S) * 4, hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipMemcpyAsync(c->r_grp.p, grp_ser.data(), (G + 1) * 8, hipMemcpyHostToDevice, c->stream));
  HIP_OK(hipMemsetAsync(c->err.p, 0, 4, c->stream));
  tr.mark("device arrays + H2D");
  RawParams rp{};
  rp.rows = c->rows.as<RowDesc>();
  rp.qual = c->qual.as<uint8_t>();
  rp.val = c->val.as<uint8_t>();
  rp.n_rows = c->n_rows;
  rp.row_pt_off = c->r_rowpt.as<int64_t>();
  rp.pts = c->r_pts.as<RawPt>();
  rp.n_series = S;
  rp.sp_off = c->r_spoff.as<int64_t>();
  rp.sp_n = c->r_spn.as<int32_t>();
  rp.rate = q->rate;
  rp.counter = q->rate_counter;
  rp.drop = q->rate_drop_resets;
  rp.counter_max = q->rate_counter_max;
  rp.reset_value = q->rate_reset_value;
  rp.start_ms = start;
  rp.gran = all_s ? 1000 : 1;
  const int64_t nbits = std::max<int64_t>(1, (end - start + rp.gran - 1) / rp.gran);
  rp.W = (nbits + 31) / 32;
  rp.grp_ser = c->r_grp.as<int64_t>();
  rp.rank = c->r_rank.as<int32_t>();
  rp.ga = P.ga;
  rp.interp = P.interp;
  rp.do_long = !q->rate && any_int;
  rp.do_double = q->rate || any_float;
  if (!rp.do_long && !rp.do_double) rp.do_double = 1;
  rp.err = c->err.as<int32_t>();
  rp.uns = uns ? 1 : 0;
  rp.lerp_fast = !opt_off(OPT_RAW_LERPW);
  if (uns) {
    HIP_OK(c->r_mts.ensure(std::max<int64_t>(1, np) * 8));
    HIP_OK(c->r_mpos.ensure(std::max<int64_t>(1, S) * 4));
    HIP_OK(c->r_mhead.ensure(std::max<int64_t>(1, S) * 8));
    HIP_OK(c->r_bnd.ensure((G + 1) * 8));
    rp.mts = c->r_mts.as<int64_t>();
    rp.m_pos = c->r_mpos.as<int32_t>();
    rp.m_head = c->r_mhead.as<int64_t>();
  }
  HIP_OK(hipEventRecord(c->ev[0], c->stream));
  if (ext) {
    if (np) HIP_OK(hipMemcpyAsync(rp.pts, ext->pts.data(), np * sizeof(RawPt), hipMemcpyHostToDevice, c->stream));
  } else {
    HIP_OK(launch_raw_decode(rp, c->stream));
  }
  tr.mark("decode launch");
  if (q->rate) {
    HIP_OK(launch_raw_rate(rp, c->stream));
    HIP_OK(hipMemcpyAsync(sp_n.data(), c->r_spn.p, std::max<int64_t>(1, S) * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
  }
  // group chunks whose timestamp bitmaps fit the budget
  const int64_t budget = (int64_t)2 << 30;
  // (the greedy merge keeps no bitmap: one chunk, its step timestamps bounded by the points)
  const int64_t per_chunk = uns ? std::max<int64_t>(1, G) : std::max<int64_t>(1, budget / (rp.W * 8));
  std::vector<int64_t> res_ts;
  std::vector<uint64_t> res_bits;
  std::vector<uint8_t> res_int;
  std::vector<int64_t> g_ptr(G + 1, 0);
  double eval_ms = 0.0;
  const bool direct = !P.none && per_chunk >= G;
  tsdbhip_result* direct_r = nullptr;
  // On an early return the copy stream may still be writing into direct_r's pinned block:
  // drain it before the block goes back to the pool.
  struct Guard {
    tsdbhip_result** r;
    hipStream_t cs;
    ~Guard() {
      if (*r) {
        (void)hipStreamSynchronize(cs);
        result_free(*r);
      }
    }
  } guard{&direct_r, c->copy_stream};
  if (direct) {
    // the result block, sized by the decoded points (every union point is one of them), is
    // allocated while the device decodes: a fresh pinned block of 100s of MB costs the host
    // longer than the evaluation itself
    int64_t nact = 0;
    for (int64_t g = 0; g < G; g++) nact += act[g];
    direct_r = make_result(nact, std::max<int64_t>(0, np));
    if (!direct_r) return fail(TSDB_E_NOMEM, "result allocation");
    tr.mark("result alloc");
  }
  for (int64_t g0 = 0; g0 < G; g0 += per_chunk) {
    const int64_t g1 = std::min(G, g0 + per_chunk);
    const int64_t ng = g1 - g0;
    rp.g0 = g0;
    rp.g1 = g1;
    HIP_OK(c->r_U.ensure(ng * 4));
    rp.U = c->r_U.as<int32_t>();
    std::vector<int64_t> bnd;   // greedy merge: each group's steps are bounded by its counted points
    if (uns) {
      bnd.assign(ng + 1, 0);
      const int first = q->rate ? 1 : 0;
      for (int64_t i = 0; i < ng; i++) {
        bnd[i + 1] = bnd[i];
        for (int64_t s = grp_ser[g0 + i]; s < grp_ser[g0 + i + 1]; s++) bnd[i + 1] += std::max(0, sp_n[s] - first);
      }
      HIP_OK(hipMemcpyAsync(c->r_bnd.p, bnd.data(), (ng + 1) * 8, hipMemcpyHostToDevice, c->stream));
      rp.bnd_off = c->r_bnd.as<int64_t>();
      HIP_OK(launch_raw_merge(rp, c->stream));
    } else {
      HIP_OK(c->r_bm.ensure(ng * rp.W * 4));
      HIP_OK(c->r_wb.ensure(ng * rp.W * 4));
      rp.bitmap = c->r_bm.as<uint32_t>();
      rp.wbase = c->r_wb.as<uint32_t>();
      HIP_OK(hipMemsetAsync(rp.bitmap, 0, ng * rp.W * 4, c->stream));
      HIP_OK(launch_raw_union(rp, grp_ser[g0], grp_ser[g1], c->stream));
    }
    std::vector<int32_t> U(ng);
    HIP_OK(hipMemcpyAsync(U.data(), rp.U, ng * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    tr.mark("decode+union");
    std::vector<int64_t> ooff(ng + 1, 0), coff(ng + 1, 0);
    std::vector<int32_t> sg, st;
    for (int64_t i = 0; i < ng; i++) {
      ooff[i + 1] = ooff[i] + U[i];
      const int64_t nst = (U[i] + RAW_STRIP - 1) / RAW_STRIP;
      for (int64_t t = 0; t < nst; t++) { sg.push_back((int32_t)i); st.push_back((int32_t)t); }
      coff[i + 1] = coff[i] + nst * (grp_ser[g0 + i + 1] - grp_ser[g0 + i]);
    }
    const int64_t nout = ooff[ng];
    const int64_t ns = (int64_t)sg.size();
    HIP_OK(c->r_ooff.ensure((ng + 1) * 8));
    HIP_OK(c->r_coff.ensure((ng + 1) * 8));
    HIP_OK(c->r_cur.ensure(std::max<int64_t>(1, coff[ng]) * 4));
    HIP_OK(c->r_sg.ensure(std::max<int64_t>(1, ns) * 4));
    HIP_OK(c->r_su.ensure(std::max<int64_t>(1, ns) * 4));
    HIP_OK(c->r_ots.ensure(std::max<int64_t>(1, nout) * 8));
    HIP_OK(c->r_obits.ensure(std::max<int64_t>(1, nout) * 8));
    HIP_OK(c->r_oint.ensure(std::max<int64_t>(1, nout)));
    HIP_OK(hipMemcpyAsync(c->r_ooff.p, ooff.data(), (ng + 1) * 8, hipMemcpyHostToDevice, c->stream));
    HIP_OK(hipMemcpyAsync(c->r_coff.p, coff.data(), (ng + 1) * 8, hipMemcpyHostToDevice, c->stream));
    if (ns) {
      HIP_OK(hipMemcpyAsync(c->r_sg.p, sg.data(), ns * 4, hipMemcpyHostToDevice, c->stream));
      HIP_OK(hipMemcpyAsync(c->r_su.p, st.data(), ns * 4, hipMemcpyHostToDevice, c->stream));
    }
    rp.out_off = c->r_ooff.as<int64_t>();
    rp.cur_off = c->r_coff.as<int64_t>();
    rp.cur = c->r_cur.as<int32_t>();
    rp.strip_g = c->r_sg.as<int32_t>();
    rp.strip_t = c->r_su.as<int32_t>();
    rp.n_strips = ns;
    rp.out_ts = c->r_ots.as<int64_t>();
    rp.out_bits = c->r_obits.as<uint64_t>();
    rp.out_int = c->r_oint.as<uint8_t>();
    if (uns) HIP_OK(launch_raw_merge_ts(rp, c->stream));
    else HIP_OK(launch_raw_rank(rp, grp_ser[g0], grp_ser[g1], c->stream));
    HIP_OK(launch_raw_cursor(rp, grp_ser[g0], grp_ser[g1], c->stream));
    // percentile / median with every rank asked for within 32 of the top (p90 ... p999 of
    // large groups, any rank of small ones): k_raw_top folds each span operand into its point's
    // top keys as it evaluates it -- no operand arrays
    int top_t = 0;
    if (P.gsel) {
      {
        int64_t k_all = 1;
        for (int64_t g = g0; g < g1; g++) k_all = std::max<int64_t>(k_all, grp_ser[g + 1] - grp_ser[g]);
        const int need = raw_top_need(P.gsel, k_all, 32);
        top_t = need <= 8 ? 8 : need <= 16 ? 16 : need <= 32 ? 32 : 0;
      }
    }
    if (top_t) {
      rp.sel_fn = P.gsel;
      HIP_OK(hipEventRecord(c->ev[3], c->stream));
      if (uns) {
        HIP_OK(c->r_dz.ensure(std::max<int64_t>(1, nout)));
        HIP_OK(hipMemsetAsync(c->r_dz.p, 0, std::max<int64_t>(1, nout), c->stream));
        rp.dz = c->r_dz.as<uint8_t>();
      }
      HIP_OK(launch_raw_top(rp, top_t, c->stream));
      if (uns) HIP_OK(launch_raw_dz_check(rp, nout, c->stream));
    } else if (P.gsel) {
      // percentile / median: every span operand of every union point, strip by strip
      // (RAW_STRIP points x the group's spans each), in batches of at most kSelOps operands
      int64_t kSelOps = (int64_t)1 << 28;
      if (opt(OPT_SELOPS) > 0) kSelOps = opt(OPT_SELOPS);   // tests: force batches
      std::vector<int64_t> soff(ns + 1, 0);
      for (int64_t t = 0; t < ns; t++) soff[t + 1] = soff[t] + (grp_ser[g0 + sg[t] + 1] - grp_ser[g0 + sg[t]]) * RAW_STRIP;
      // batches [bat[i], bat[i + 1]) of strips: at least one strip each, else <= kSelOps operands
      std::vector<int64_t> bat{0};
      int64_t nv_max = 1;
      for (int64_t s0 = 0; s0 < ns;) {
        int64_t s1 = s0 + 1;
        while (s1 < ns && soff[s1 + 1] - soff[s0] <= kSelOps) s1++;
        nv_max = std::max<int64_t>(nv_max, soff[s1] - soff[s0]);
        bat.push_back(s1);
        s0 = s1;
      }
      HIP_OK(c->r_voff.ensure(std::max<int64_t>(1, ns) * 8));
      HIP_OK(c->r_vl.ensure(nv_max * 8));
      HIP_OK(c->r_vd.ensure(nv_max * 8));
      HIP_OK(c->r_vp.ensure(nv_max));
      rp.sel_fn = P.gsel;
      rp.vals_l = c->r_vl.as<int64_t>();
      rp.vals_d = c->r_vd.as<double>();
      rp.vals_p = c->r_vp.as<uint8_t>();
      HIP_OK(hipEventRecord(c->ev[3], c->stream));
      // every strip's operand offset relative to its batch, uploaded once
      std::vector<int64_t> boff(std::max<int64_t>(1, ns), 0);
      for (size_t bi = 0; bi + 1 < bat.size(); bi++)
        for (int64_t t = bat[bi]; t < bat[bi + 1]; t++) boff[t] = soff[t] - soff[bat[bi]];
      HIP_OK(hipMemcpyAsync(c->r_voff.p, boff.data(), std::max<int64_t>(1, ns) * 8, hipMemcpyHostToDevice, c->stream));
      HIP_OK(hipStreamSynchronize(c->stream));   // `boff` leaves scope before the chunk's sync
      HIP_OK(hipMemsetAsync(rp.out_int, 1, std::max<int64_t>(1, nout), c->stream));   // isInteger until a double is seen
      if (uns) {
        HIP_OK(c->r_dz.ensure(std::max<int64_t>(1, nout)));
        HIP_OK(hipMemsetAsync(c->r_dz.p, 0, std::max<int64_t>(1, nout), c->stream));
        rp.dz = c->r_dz.as<uint8_t>();
      }
      for (size_t bi = 0; bi + 1 < bat.size(); bi++) {
        const int64_t s0 = bat[bi], s1 = bat[bi + 1];
        const int64_t nv = soff[s1] - soff[s0];
        HIP_OK(hipMemsetAsync(c->r_vp.p, 0, nv, c->stream));
        // NaN: no operand (only double points read r_vd; a long-only query never has one)
        if (rp.do_double) HIP_OK(hipMemsetAsync(c->r_vd.p, 0xFF, nv * 8, c->stream));
        RawParams bp = rp;
        bp.strip_g = rp.strip_g + s0;
        bp.strip_t = rp.strip_t + s0;
        bp.n_strips = s1 - s0;
        bp.vals_off = c->r_voff.as<int64_t>() + s0;
        int64_t k_max = 1;
        for (int64_t t = s0; t < s1; t++) k_max = std::max<int64_t>(k_max, grp_ser[g0 + sg[t] + 1] - grp_ser[g0 + sg[t]]);
        HIP_OK(launch_raw_vals(bp, k_max, c->stream));
        // k_raw_sel CONSUMES this batch's operand buffers: for groups above its LDS capacity it
        // builds the sort keys in place over r_vl / r_vd, so they hold keys, not operands,
        // afterwards.  Every batch is staged by launch_raw_vals right before its selection;
        // a second selection over the same batch would have to re-stage it.
        HIP_OK(launch_raw_sel(bp, k_max, c->stream));
      }
      if (uns) HIP_OK(launch_raw_dz_check(rp, nout, c->stream));
    } else if (!direct) {
      HIP_OK(hipEventRecord(c->ev[3], c->stream));
      HIP_OK(launch_raw_eval(rp, c->stream));
    }
    const size_t base = res_ts.size();
    if (direct) {
      // one chunk, groups emitted in batch order: device layout == result layout.  The strips
      // are evaluated in up to 8 launches split at group boundaries; each launch's output range
      // (its groups' union points, contiguous) downloads on copy_stream while the next one
      // runs, into a pinned result block
      if (!P.gsel) HIP_OK(hipEventRecord(c->ev[3], c->stream));
      // chunked only for the double-only evaluation: its strips are short (config 4 rate: the
      // download hides behind the next chunk, 36 -> 30 ms per step); the long LERP strips are
      // long-running waves that a launch split leaves idle at every chunk's tail (94 -> 188 ms)
      const int nch = (P.gsel || rp.do_long) ? 1 : (int)std::min<int64_t>(8, std::max<int64_t>(1, ns / 64));
      // the timestamps are final once k_raw_rank ran: their download overlaps the evaluation
      HIP_OK(hipEventRecord(c->cev[8], c->stream));
      if (nout) {
        HIP_OK(hipStreamWaitEvent(c->copy_stream, c->cev[8], 0));
        HIP_OK(hipMemcpyAsync(const_cast<int64_t*>(direct_r->ts_ms), rp.out_ts, nout * 8, hipMemcpyDeviceToHost,
                              c->copy_stream));
      }
      int64_t s_lo = 0;
      for (int ci = 0; ci < nch; ci++) {
        int64_t s_hi = ci + 1 == nch ? ns : std::max(s_lo, ns * (ci + 1) / nch);
        while (s_hi > s_lo && s_hi < ns && sg[s_hi] == sg[s_hi - 1]) s_hi++;   // end at a group boundary
        if (ci + 1 == nch) s_hi = ns;
        if (!P.gsel && s_hi > s_lo) {
          RawParams ep = rp;
          ep.strip_g = rp.strip_g + s_lo;
          ep.strip_t = rp.strip_t + s_lo;
          ep.n_strips = s_hi - s_lo;
          HIP_OK(launch_raw_eval(ep, c->stream));
        }
        // output points of groups [first group of the chunk, first group of the next chunk)
        const int64_t o0 = s_lo < ns ? ooff[sg[s_lo]] : nout;
        const int64_t o1 = s_hi < ns ? ooff[sg[s_hi]] : nout;
        HIP_OK(hipEventRecord(c->cev[ci], c->stream));
        if (o1 > o0) {
          HIP_OK(hipStreamWaitEvent(c->copy_stream, c->cev[ci], 0));
          HIP_OK(hipMemcpyAsync(const_cast<uint64_t*>(direct_r->value_bits) + o0, rp.out_bits + o0, (o1 - o0) * 8,
                                hipMemcpyDeviceToHost, c->copy_stream));
          HIP_OK(hipMemcpyAsync(const_cast<uint8_t*>(direct_r->is_int) + o0, rp.out_int + o0, o1 - o0,
                                hipMemcpyDeviceToHost, c->copy_stream));
        }
        s_lo = s_hi;
      }
      HIP_OK(hipEventRecord(c->ev[1], c->stream));
      HIP_OK(hipStreamSynchronize(c->stream));
      tr.mark("eval (device)");
      HIP_OK(hipStreamSynchronize(c->copy_stream));
      tr.mark("download tail");
    } else {
      HIP_OK(hipEventRecord(c->ev[1], c->stream));
      res_ts.resize(base + nout);
      res_bits.resize(base + nout);
      res_int.resize(base + nout);
      if (nout) {
        HIP_OK(hipMemcpyAsync(res_ts.data() + base, rp.out_ts, nout * 8, hipMemcpyDeviceToHost, c->stream));
        HIP_OK(hipMemcpyAsync(res_bits.data() + base, rp.out_bits, nout * 8, hipMemcpyDeviceToHost, c->stream));
        HIP_OK(hipMemcpyAsync(res_int.data() + base, rp.out_int, nout, hipMemcpyDeviceToHost, c->stream));
      }
    }
    HIP_OK(hipStreamSynchronize(c->stream));
    float te = 0;
    (void)hipEventElapsedTime(&te, c->ev[3], c->ev[1]);
    eval_ms += te;
    for (int64_t i = 0; i < ng; i++) g_ptr[g0 + i + 1] = (int64_t)base + ooff[i + 1];
  }
  int32_t err = 0;
  { int rc_ = d2h_small(c, &err, c->err.p, 4, c->stream); if (rc_) return rc_; }
  { int rc_ = sync_small(c, c->stream); if (rc_) return rc_; }
  float t01 = 0;
  (void)hipEventElapsedTime(&t01, c->ev[0], c->ev[1]);
  c->fast_used = false;
  c->timing.decode_downsample_ms = t01;
  c->timing.group_reduce_ms = eval_ms;
  c->timing.total_ms = t01;
  c->timing.fast_ms = 0;
  c->timing.tiles = G;
  c->timing.redo_tiles = 0;
  account(c, P);
  if (err) return fail(err, "error raised by the device path");
  if (direct && !direct_r) {   // no group chunk ran (an empty shard): an empty result
    direct_r = make_result(0, 0);
    if (!direct_r) return fail(TSDB_E_NOMEM, "result allocation");
  }
  tr.mark("finish");
  if (direct) {
    auto* gptr = const_cast<int64_t*>(direct_r->group_ptr);
    auto* gid = const_cast<int32_t*>(direct_r->group_id);
    int64_t i = 0;
    for (int64_t g = 0; g < G; g++) {
      if (!act[g]) continue;
      gid[i] = (int32_t)g;
      gptr[i] = g_ptr[g];
      i++;
    }
    gptr[i] = g_ptr[G];
    *out = direct_r;
    direct_r = nullptr;
    return 0;
  }
  // result: emitted groups in emission order
  std::vector<std::pair<int64_t, int64_t>> order;   // (result group id, group row)
  for (int64_t g = 0; g < G; g++) {
    if (!act[g]) continue;
    order.push_back({P.none ? gid_of[g] : g, g});
  }
  std::sort(order.begin(), order.end());
  int64_t npts = 0;
  for (auto& o : order) npts += g_ptr[o.second + 1] - g_ptr[o.second];
  tsdbhip_result* r = make_result((int64_t)order.size(), npts);
  if (!r) return fail(TSDB_E_NOMEM, "result allocation");
  auto* gptr = const_cast<int64_t*>(r->group_ptr);
  auto* gid = const_cast<int32_t*>(r->group_id);
  auto* ts = const_cast<int64_t*>(r->ts_ms);
  auto* vb = const_cast<uint64_t*>(r->value_bits);
  auto* isi = const_cast<uint8_t*>(r->is_int);
  int64_t o = 0;
  for (size_t i = 0; i < order.size(); i++) {
    const int64_t g = order[i].second;
    gptr[i] = o;
    gid[i] = (int32_t)order[i].first;
    const int64_t a = g_ptr[g], n = g_ptr[g + 1] - a;
    if (n) {
      std::memcpy(ts + o, res_ts.data() + a, n * 8);
      std::memcpy(vb + o, res_bits.data() + a, n * 8);
      std::memcpy(isi + o, res_int.data() + a, n);
    }
    o += n;
  }
  gptr[order.size()] = o;
  *out = r;
  return 0;
}

// Spans on calendar grids that disagree (per-span anchors: DateTime.previousInterval of each
// span's first datapoint, src/core/Downsampler.java:336-350, src/utils/DateTime.java:445-606).
// The reference's AggregationIterator interleaves the spans' Downsampler outputs over the union
// of their timestamps, interpolating the spans without a point there
// (src/core/AggregationIterator.java:500-797) -- the raw path's evaluation.  Each anchor's spans
// are downsampled on that anchor's boundary sequence (one MODE_TABLE pass per anchor, every
// series' bucket values in pre_dense / pre_pres), the buckets become the spans' points, and the
// raw union evaluator (k_raw_*) aggregates them: rate, LERP, percentile group-by and NONE as for
// raw datapoints.  Points before the SpanGroup start are dropped (AggregationIterator :416-441).
int run_anchored(tsdbhip_ctx* c, const tsdbhip_query* q, const Plan& P, tsdbhip_result** out) {
  const int64_t S = c->n_series;
  const int unit = q->ds_calendar;
  const int64_t n = q->ds_interval_ms / CAL_UNIT_MS[unit];
  const JZone Z{q->ds_tz};
  // every series' first datapoint at or after the seek point, and its anchor
  std::vector<int64_t> f(std::max<int64_t>(1, S), INT64_MAX);
  HIP_OK(c->first_ts.ensure(std::max<int64_t>(1, S) * 8));
  HIP_OK(launch_first_ts(c->rows.as<RowDesc>(), c->srp.as<int64_t>(), c->qual.as<uint8_t>(), S, P.ss, P.se, P.seek,
                         c->first_ts.as<int64_t>(), c->stream));
  if (S) HIP_OK(hipMemcpyAsync(f.data(), c->first_ts.p, S * 8, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  f.resize(S);
  std::vector<int64_t> fu(f);
  std::sort(fu.begin(), fu.end());
  fu.erase(std::unique(fu.begin(), fu.end()), fu.end());
  std::vector<int64_t> au;
  anchors_of(Z, n, unit, fu, au);
  std::vector<int32_t> cls(S, -1);
  for (int64_t s = 0; s < S; s++) {
    if (f[s] == INT64_MAX) continue;
    const int64_t a = au[std::lower_bound(fu.begin(), fu.end(), f[s]) - fu.begin()];
    const auto it = std::lower_bound(P.anchors.begin(), P.anchors.end(), a);
    if (it == P.anchors.end() || *it != a) return fail(TSDB_E_HIP, "calendar anchor of a series missing from the plan");
    cls[s] = (int32_t)(it - P.anchors.begin());
  }
  // the spans with rows in the scan range: their SpanGroups exist
  RawExt ext;
  ext.n.assign(S, 0);
  ext.live.assign(S, 0);
  for (int64_t s = 0; s < S; s++)
    for (int64_t r = c->h_srp[s]; r < c->h_srp[s + 1] && !ext.live[s]; r++)
      ext.live[s] = (int64_t)c->h_base[r] >= P.ss && (int64_t)c->h_base[r] < P.se;
  std::vector<std::vector<RawPt>> sp(S);
  const int64_t start = P.ss * 1000;
  const bool fill = q->ds_fill != TSDB_FILL_NONE;
  if (fill && q->ds_fill == TSDB_FILL_SCALAR) return fail(TSDB_E_RUNTIME, "unhandled fill policy");
  tsdbhip_query q2 = *q;
  q2.rate = 0;   // RateSpan wraps the Downsampler: the raw evaluator applies it to the buckets
  for (size_t k = 0; k < P.anchors.size(); k++) {
    const std::vector<int64_t>& sq = P.seqs[k];
    if (sq.size() < 2 || std::find(cls.begin(), cls.end(), (int32_t)k) == cls.end()) continue;
    Plan Pk = P;
    Pk.anchored = false;
    Pk.anchors.clear();
    Pk.seqs.clear();
    Pk.mode = MODE_TABLE;
    Pk.bounds = sq;
    Pk.K = (int64_t)sq.size() - 1;
    Pk.B0 = sq[0];
    Pk.none = true;   // one tile per series: ungrouped spans too
    Pk.gsel = 0;
    Pk.ordered = false;
    Pk.raw = false;
    Pk.gslot = grid_wave_lds(Pk.K, false, false) > 40 * 1024;
    if (P.f == F_SEL) Pk.values_only = true;
    else Pk.dense_out = true;
    int rc = run_device(c, &q2, Pk, S, false);
    if (rc) return rc;
    const int64_t K = Pk.K;
    std::vector<double> dense(std::max<int64_t>(1, S * K));
    std::vector<uint8_t> pres(std::max<int64_t>(1, S * K));
    int32_t err = 0;
    if (S * K) {
      HIP_OK(hipMemcpyAsync(dense.data(), c->pre_dense.p, S * K * 8, hipMemcpyDeviceToHost, c->stream));
      HIP_OK(hipMemcpyAsync(pres.data(), c->pre_pres.p, S * K, hipMemcpyDeviceToHost, c->stream));
    }
    { int rc_ = d2h_small(c, &err, c->err.p, 4, c->stream); if (rc_) return rc_; }
    { int rc_ = sync_small(c, c->stream); if (rc_) return rc_; }
    if (err) return fail(err, "error raised by the device path");
    for (int64_t s = 0; s < S; s++) {
      if (cls[s] != (int32_t)k) continue;
      for (int64_t j = 0; j < K; j++) {
        if (!pres[s * K + j] || (sq[j] < start && !fill)) continue;
        RawPt pt;
        pt.tsf = sq[j] | RAW_FLOAT;
        std::memcpy(&pt.bits, &dense[s * K + j], 8);
        sp[s].push_back(pt);
        if (sq[j] % 1000) ext.sec = false;
      }
    }
  }
  if (fill) {
    // FillingDownsampler.next (src/core/FillingDownsampler.java:172-301): one output per step of
    // its own calendar sequence, previousInterval(start) up to previousInterval(end) exclusive --
    // the span's bucket at exactly that timestamp (earlier buckets are consumed), else the fill
    // value; a span with rows in the scan but no bucket emits fills only
    const double fv = q->ds_fill == TSDB_FILL_ZERO ? 0.0 : std::numeric_limits<double>::quiet_NaN();
    uint64_t fbits;
    std::memcpy(&fbits, &fv, 8);
    const std::vector<int64_t>& F = P.fillseq;
    for (int64_t s = 0; s < S; s++) {
      std::vector<RawPt> out;
      if (ext.live[s]) {
        size_t b = 0;
        for (size_t i = 0; i + 1 < F.size(); i++) {
          const int64_t t = F[i];
          while (b < sp[s].size() && (sp[s][b].tsf & RAW_TIME_MASK) < t) b++;
          RawPt pt;
          pt.tsf = t | RAW_FLOAT;
          pt.bits = b < sp[s].size() && (sp[s][b].tsf & RAW_TIME_MASK) == t ? sp[s][b].bits : fbits;
          if (t < start) continue;
          out.push_back(pt);
          if (t % 1000) ext.sec = false;
        }
      }
      sp[s].swap(out);
    }
  }
  for (int64_t s = 0; s < S; s++) {
    ext.n[s] = (int32_t)sp[s].size();
    ext.pts.insert(ext.pts.end(), sp[s].begin(), sp[s].end());
  }
  return run_raw(c, q, P, out, &ext);
}

}  // namespace

namespace {

// The scan of a rollup query over the resident rollup batch: RollupSeq.append's exceptions
// (thrown while the spans are built, in scan order), reads the engine does not restate, and
// which value series the scan finds (cached per scan range).
int ro_scan(tsdbhip_ctx* c, const Plan& P, bool reads_counts) {
  const int64_t S0 = P.ss * 1000;
  const int64_t T = P.mode == MODE_TABLE ? P.seek : (P.mode == MODE_ALL ? S0 : P.B0);
  const bool checked = c->ro_chk_valid && c->ro_chk_ss == P.ss && c->ro_chk_se == P.se && c->ro_chk_T == T &&
                       (c->ro_chk_counts || !reads_counts);
  for (int64_t s = 0; s < c->ro_nval && !checked; s++) {
    const RoSeqRow* first_err = nullptr;
    bool in = false, verr = false, cerr = false;
    for (int64_t i = c->ro_rp[s]; i < c->ro_rp[s + 1]; i++) {
      const RoSeqRow& r = c->ro_rows[i];
      if (r.base < P.ss || r.base >= P.se) continue;
      in = true;
      if (r.err && (!first_err || r.order < first_err->order)) first_err = &r;
      verr |= r.verr;
      cerr |= r.cerr;
    }
    if (first_err) return fail(first_err->err, first_err->msg);
    if (!in) continue;
    // cells no HBase scan of a rollup table returns (a row key's cells arrive together, offsets stay
    // inside the row span): refused as data RollupSeq does not take (IllegalDataException,
    // RollupSeq.addRow src/rollup/RollupSeq.java:170-205), naming the case
    if (!c->ro_unsup[s].empty()) return fail(TSDB_E_ILLEGAL_DATA, "rollup span: " + c->ro_unsup[s]);
    if (verr) return fail(TSDB_E_ILLEGAL_DATA, "rollup value of a bad length");
    if (cerr && reads_counts) return fail(TSDB_E_ILLEGAL_DATA, "rollup count of a bad length");
  }
  // RollupIterator.seek walks value and count cells in lock step from the first pair: past a
  // cell where they stop pairing one to one its iteration differs from a fresh one's.  The
  // Downsampler seeks every span to its first bucket; a RollupSeq it seeks into past such a
  // cell is not restated.
  if (c->ro_counts && T > S0 && !checked) {
    for (int64_t s = 0; s < c->ro_nval; s++) {
      const RoSeqRow* pick = nullptr;   // Span.seekRow: first row (by base) whose last point >= T
      for (int64_t i = c->ro_rp[s]; i < c->ro_rp[s + 1]; i++) {
        const RoSeqRow& r = c->ro_rows[i];
        if (r.base < P.ss || r.base >= P.se || r.npts < 1 || r.last_ts < T) continue;
        if (!pick || r.base < pick->base) pick = &r;
      }
      if (pick && pick->pp_ts < T)
        return fail(TSDB_E_NOT_IMPLEMENTED, "rollup row whose value and count cells stop pairing before the seek point");
    }
  }
  if (!checked) {   // every check passed for this range (failures are not cached: they re-raise)
    c->ro_chk_valid = true;
    c->ro_chk_ss = P.ss;
    c->ro_chk_se = P.se;
    c->ro_chk_T = T;
    c->ro_chk_counts = reads_counts;
  }
  if (!(c->ro_scan_valid && c->ro_scan_ss == P.ss && c->ro_scan_se == P.se)) {
    c->ro_scan_act.assign(std::max<int64_t>(1, c->n_series), 0);
    for (int64_t s = 0; s < c->ro_nval; s++)
      for (int64_t i = c->ro_rp[s]; i < c->ro_rp[s + 1]; i++)
        if (c->ro_rows[i].base >= P.ss && c->ro_rows[i].base < P.se) { c->ro_scan_act[c->ro_res[s]] = 1; break; }
    // the groups those series belong to, once per scan range (not a pass over every series per query)
    std::vector<uint8_t> seen(std::max<int64_t>(1, c->n_groups), 0);
    c->ro_scan_gact.clear();
    for (int64_t i = 0; i < c->n_series; i++) {
      const int64_t g = c->h_group[i];
      if (c->ro_scan_act[i] && g < c->n_groups && !seen[g]) { seen[g] = 1; c->ro_scan_gact.push_back((int32_t)g); }
    }
    c->ro_scan_valid = true;
    c->ro_scan_ss = P.ss;
    c->ro_scan_se = P.se;
  }
  return 0;
}

// TsdbQuery.run with a RollupQuery (src/core/TsdbQuery.java:1665-1700 builds it from the
// downsampler; a count group-by aggregator sums).  Avg and count downsampling of a batch with
// count cells (Downsampler.java:165-221, FillingDownsampler.java:196-253):
//   1. every series' SUM downsampling (value series: Σsum per bucket, count series: Σcount)
//      into pre_dense, one NONE tile per series;
//   2. k_rollup_combine: each value series' buckets <- Σsum / Σcount (0 when Σcount is 0) or
//      Σcount;
//   3. the SpanGroup step (rate, fill, LERP, group-by) over those buckets (k_emit).
// Every other downsampling function reads only the value series: the ordinary pipeline.
// The query a rollup batch runs: a count group-by sums (the aggregator RollupQuery leaves).
tsdbhip_query ro_query(const tsdbhip_ctx* c, const tsdbhip_query* q) {
  tsdbhip_query r = *q;
  if (c->ro_active && r.aggregator == TSDB_AGG_COUNT) r.aggregator = TSDB_AGG_SUM;
  return r;
}

int ro_check(const tsdbhip_query* q) {
  if (q->ds_function < 0 || (!q->ds_all && q->ds_interval_ms <= 0))
    return fail(TSDB_E_ILLEGAL_ARGUMENT, "a rollup query needs a downsampling interval");
  if (q->ds_function == TSDB_AGG_DEV)
    return fail(TSDB_E_UNSUPPORTED, "Standard deviation over rolled up data is not supported at this time");
  return 0;
}

// The scan (ro_scan) and, for avg / count downsampling over count cells, steps 1-2 above: the
// query's group-by step then runs over pre_dense (P.emit_only).  q is the caller's query, qr
// ro_query(q), P planned from qr.
bool seq_dense_wanted(tsdbhip_ctx* c, const Plan& P);

int ro_stage(tsdbhip_ctx* c, const tsdbhip_query* q, const tsdbhip_query& qr, Plan& P) {
  const bool combine = c->ro_counts && (q->ds_function == TSDB_AGG_AVG || q->ds_function == TSDB_AGG_COUNT);
  int rc = ro_scan(c, P, combine);
  if (rc || !combine) return rc;
  // (a percentile / median group-by or TSDB_QF_ORDERED then takes these buckets as its span
  // values: sel_values skips its own downsampling pass under P.emit_only)
  tsdbhip_query q1 = qr;
  q1.ds_function = TSDB_AGG_SUM;
  q1.aggregator = TSDB_AGG_NONE;
  q1.rate = 0;
  q1.flags = 0;
  // the query's own slot grid and scan range (a rate query scans one row further back)
  Plan P1 = P;
  P1.f = f_of(TSDB_AGG_SUM);
  P1.ga = ga_of(TSDB_AGG_NONE);
  P1.interp = interp_of(TSDB_AGG_NONE);
  P1.none = true;
  P1.gsel = 0;
  P1.ordered = false;
  P1.gslot = grid_wave_lds(P.K, false, false) > 40 * 1024;
  bool fused = false;
  if (seq_dense_wanted(c, P1)) {   // sums that cannot add in any order: k_seq_dense, Java's order, one pass
    P1.seq_dense = true;
    P1.values_only = true;
    // value rows with their lock-step count rows in one pass (k_seq_rows_ro), combined in place
    if (seq_rows_ok(c, P1) && c->ro_partner.p && !opt_off(OPT_RO_FUSE)) {
      P1.ro_fuse = q->ds_function == TSDB_AGG_AVG ? 1 : 2;
      fused = true;
    }
  } else {
    P1.dense_out = true;
  }
  rc = run_device(c, &q1, P1, c->n_series, false);
  if (rc) return rc;
  if (!fused)
    HIP_OK(launch_rollup_combine(c->pre_dense.as<double>(), c->pre_pres.as<uint8_t>(), c->ro_cmap.as<int64_t>(),
                                 c->n_series, P.K, q->ds_function == TSDB_AGG_AVG ? 1 : 0, c->stream));
  P.emit_only = true;
  P.split2 = true;   // the query's device time starts with this pass (its ev[0] stands)
  return 0;
}

// rollup: a span the scan found is a SpanGroup member (or, NONE, its own SpanGroup) even when
// its RollupSeqs yield no datapoint; count series are no spans of the query
void ro_activity(const tsdbhip_ctx* c, const Plan& P, int64_t G, std::vector<uint32_t>& act) {
  if (!(c->ro_active && c->ro_scan_valid)) return;
  if (!P.none) {
    for (const int32_t g : c->ro_scan_gact)
      if (g < G) act[g] = 1;
    return;
  }
  for (int64_t i = 0; i < std::min<int64_t>(G, c->n_series); i++)
    act[i] = c->h_orig[i] < c->ro_nval ? (act[i] | c->ro_scan_act[i]) : 0;
}

// Sum / avg downsampling over a scan holding rows whose values cannot add exactly in any order
// (ROW_NOCERT): k_seq_dense computes every bucket in Java's order in one pass instead of the
// streaming kernels handing those tiles to k_grid's sequential re-walk.  Needs rows in time
// order throughout the scan (the cache is per scan range; the rows are resident).
// Also every other downsampling function over scans of tiny rows at scale (rollup tables read
// as hour rows of a few cells: the streaming kernels' per-row overhead dominates there).
bool seq_dense_wanted(tsdbhip_ctx* c, const Plan& P) {
  if (!(P.f >= F_SUM && P.f <= F_MULT) || P.raw || P.anchored || P.gsel || P.ordered || P.multi || P.emit_only ||
      P.dense_out || P.values_only || P.sel_direct)
    return false;
  if (opt_off(OPT_SEQ) || opt_off(OPT_FAST)) return false;   // tests: the k_grid path (the general path only)
  if (!(c->seqd_valid && c->seqd_ss == P.ss && c->seqd_se == P.se)) {
    bool any = false, ok = true, uni = true;
    int64_t rows = 0, dps = 0;
    for (int64_t r = 0; r < c->n_rows && ok; r++) {
      if ((int64_t)c->h_base[r] < P.ss || (int64_t)c->h_base[r] >= P.se) continue;
      const uint32_t f = c->h_flags[r];
      ok = !(f & ROW_UNSORTED);
      any = any || (f & ROW_NOCERT);
      const int qw = f & ROW_QW_MASK, vl = (f & ROW_VL_MASK) >> ROW_VL_SHIFT;
      uni = uni && (qw == 2 || qw == 4) && (vl == 1 || vl == 2 || vl == 4 || vl == 8);
      rows++;
      dps += c->h_ndp[r];
    }
    c->seqd_valid = true;
    c->seqd_ss = P.ss;
    c->seqd_se = P.se;
    c->seqd_ok = ok;
    c->seqd_nocert = any;
    c->seqd_tiny = rows >= 100000 && dps <= 8 * rows;
    // k_seq_wave walks a series' rows one after the other with the whole wave: worth it for long
    // rows only (a rollup table read as one-cell rows: 144 rows a series, 47 vs 3.9 ms)
    c->seqd_uniform = uni && dps >= 64 * rows;
  }
  if (!c->seqd_ok) return false;
  return (c->seqd_nocert && (P.f == F_SUM || P.f == F_AVG)) || c->seqd_tiny;
}

int run_rollup(tsdbhip_ctx* c, const tsdbhip_query* q, tsdbhip_result** out) {
  PhaseTrace tr("rollup");
  int rc = ro_check(q);
  if (rc) return rc;
  const tsdbhip_query qr = ro_query(c, q);
  Plan P;
  rc = plan_query(c, &qr, P);
  if (rc) return rc;
  tr.mark("plan");
  rc = ro_stage(c, q, qr, P);
  if (rc) return rc;
  tr.mark("scan + stage");
  const int64_t G = P.none ? c->n_series : c->n_groups;
  P.seq_dense = seq_dense_wanted(c, P);
  tr.mark("seq_dense_wanted");
  if (P.gsel || P.ordered) {
    rc = P.gsel ? run_sel_group(c, &qr, P, G) : run_ordered(c, &qr, P, G);
    if (rc) return rc;
    return collect(c, &qr, P, G, true, out);
  }
  rc = run_device(c, &qr, P, G, true);
  if (rc) return rc;
  tr.mark("device launches");
  return collect(c, &qr, P, G, true, out);
}

// The fused streaming pass of run_multi_fused / tsdbhip_run_partials_multi: every decomposable
// aggregator's tile partials in c->m_* (MultiPartials).  1: the queries or the batch do not
// qualify, or a tile broke a streaming premise (the caller runs the queries one by one).
int fused_pass(tsdbhip_ctx* c, const tsdbhip_query* qs, int n, Plan& P) {
  if (n < 2 || opt_off(OPT_MULTI_FUSE)) return 1;
  for (int i = 0; i < n; i++) {
    const int a = qs[i].aggregator;
    if (!(a == TSDB_AGG_SUM || a == TSDB_AGG_AVG || a == TSDB_AGG_MIN || a == TSDB_AGG_MAX || a == TSDB_AGG_DEV ||
          a == TSDB_AGG_COUNT) ||
        qs[i].rate || qs[i].flags)
      return 1;
  }
  tsdbhip_query q0 = qs[0];
  q0.aggregator = TSDB_AGG_SUM;   // LERP: the interpolation of every fused aggregator but count
  int rc = plan_query(c, &q0, P);
  if (rc) return rc;
  if (P.raw || P.none || P.gsel || P.f == F_SEL || !c->tl_other.empty()) return 1;
  // K <= 64: k_short / k_rows / k_fast (KR 2); K > 64 (a day of 1m buckets): k_hwin's MULTI variant
  if (!hwin_slots(c, &q0, P, true) && (P.K > 64 || !fast_path_ok(c, &q0, P))) return 1;
  for (int cls = 0; cls < 2; cls++) {
    if (c->tl[cls][0].empty() && c->tl[cls][1].empty() && c->tl[cls][2].empty()) continue;
    const int qw = cls ? c->fast_qw2 : c->fast_qw, vl = cls ? c->fast_vl2 : c->fast_vl;
    if (!qw || !fast_supported(P.f, qw, vl)) return 1;
  }
  P.multi = true;
  for (int i = 0; i < n; i++) P.multi_dev = P.multi_dev || qs[i].aggregator == TSDB_AGG_DEV;
  rc = run_device(c, &q0, P, c->n_groups, false);
  if (rc) return rc;
  int32_t handed_back = 0;
  { int rc_ = d2h_small(c, &handed_back, c->redo_final, 4, c->stream); if (rc_) return rc_; }
  { int rc_ = sync_small(c, c->stream); if (rc_) return rc_; }
  return handed_back ? 1 : 0;
}

// aggregator agg's view of the fused pass's tile partials (as k_reduce reads its own pass's)
Partials multi_view(tsdbhip_ctx* c, int agg) {
  switch (agg) {
    case TSDB_AGG_MIN: return Partials{c->m_mn.as<double>(), c->m_m2.as<double>(), c->m_nl.as<uint32_t>(), c->m_f.as<uint32_t>()};
    case TSDB_AGG_MAX: return Partials{c->m_mx.as<double>(), c->m_m2.as<double>(), c->m_nl.as<uint32_t>(), c->m_f.as<uint32_t>()};
    case TSDB_AGG_DEV: return Partials{c->m_mean.as<double>(), c->m_m2.as<double>(), c->m_nl.as<uint32_t>(), c->m_f.as<uint32_t>()};
    case TSDB_AGG_COUNT: return Partials{c->m_sum.as<double>(), c->m_m2.as<double>(), c->m_nz.as<uint32_t>(), c->m_f.as<uint32_t>()};
    default: return Partials{c->m_sum.as<double>(), c->m_m2.as<double>(), c->m_nl.as<uint32_t>(), c->m_f.as<uint32_t>()};
  }
}

// Several decomposable group-by aggregators over one cheap downsampling, fused: ONE streaming
// pass (k_short / k_fast / k_rows KR 2, or k_hwin's MULTI variant for K > 64) decodes and
// downsamples every series once and folds each series' SpanGroup contributions into the
// per-tile state of every aggregator at once (kcommon.h MultiReg: sum / avg, min, max, dev,
// count); then one k_reduce per query over its view of those states.  Each aggregator sees
// exactly the contributions -- in the same order -- that its own pass would feed it
// (AggregationIterator.nextDoubleValue :735-797 per span, per timestamp), so results are
// bit-identical to separate queries.  Returns 1 when the queries or the batch do not qualify
// (rate, other aggregators, flags, a row class the streaming kernels do not take) or when a
// tile broke a streaming premise at run time: the caller then runs the queries one by one.
int run_multi_fused(tsdbhip_ctx* c, const tsdbhip_query* qs, int n, tsdbhip_result** outs) {
  PhaseTrace tr("run_multi_fused");
  Plan P;
  int rc = fused_pass(c, qs, n, P);
  if (rc) return rc;
  tr.mark("fused pass (synchronised)");
  const int64_t G = c->n_groups, K = P.K;
  // one k_reduce per query over its view of the fused partials, into its own output rows
  const int64_t gk = std::max<int64_t>(1, G * K);
  HIP_OK(c->out_val.ensure(gk * 8 * n));
  HIP_OK(c->out_flag.ensure(gk * n));
  std::vector<Plan> plans(n);
  for (int i = 0; i < n; i++) {
    rc = plan_query(c, &qs[i], plans[i]);
    if (rc) return rc;
    const int ga = ga_of(qs[i].aggregator);
    ReduceParams rp{};
    rp.part = multi_view(c, qs[i].aggregator);
    rp.group_tile_ptr = c->d_gtp.as<int64_t>();
    rp.G = G;
    rp.K = K;
    rp.ga = ga;
    rp.out_val = c->out_val.as<double>() + i * gk;
    rp.out_flag = c->out_flag.as<uint8_t>() + i * gk;
    rp.err = c->err.as<int32_t>();
    HIP_OK(launch_reduce(rp, c->stream));
  }
  HIP_OK(hipEventRecord(c->ev[2], c->stream));
  // every query's dense rows in one copy each (collect() per query would sync n times), into the
  // context's page-locked staging (a day of 1m buckets over 1000 groups: 13 MB a query)
  HIP_OK(c->h_stage.ensure(std::max<int64_t>(16, gk * 9 * n + 16)));
  double* val = reinterpret_cast<double*>(c->h_stage.p);
  uint8_t* flag = reinterpret_cast<uint8_t*>(c->h_stage.p) + gk * 8 * n;
  HIP_OK(hipMemcpyAsync(val, c->out_val.p, gk * n * 8, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(hipMemcpyAsync(flag, c->out_flag.p, gk * n, hipMemcpyDeviceToHost, c->stream));
  SmallD2H sm;
  rc = small_d2h(c, G, true, sm);
  if (rc) return rc;
  HIP_OK(hipStreamSynchronize(c->stream));
  std::vector<uint32_t> act(sm.act, sm.act + std::max<int64_t>(1, G));
  const int32_t err = *sm.err, redo_n = *sm.redo;
  tr.mark("reduce x n + d2h");
  c->fused_n = n;
  record_timing(c, P, redo_n);
  c->fused_n = 0;
  if (err) return fail(err, "error raised by the device path");
  for (int i = 0; i < n; i++) {
    rc = assemble(c, &qs[i], plans[i], G, val + i * gk, flag + i * gk, act, &outs[i]);
    if (rc) return rc;
  }
  tr.mark("assemble x n");
  return 0;
}

}  // namespace

extern "C" int tsdbhip_run(tsdbhip_ctx* c, const tsdbhip_query* q, tsdbhip_result** out) {
  if (c && c->md) return tsdb::md_run(c, q, out);
  if (!c || !q || !out) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  CtxLock lk(c);
  *out = nullptr;
  HIP_OK(hipSetDevice(c->device));
  if (c->ro_active) return run_rollup(c, q, out);
  Plan P;
  int rc = plan_query(c, q, P);
  if (rc) return rc;
  const int64_t G = P.none ? c->n_series : c->n_groups;
  if (P.raw) return run_raw(c, q, P, out);
  if (P.anchored) return run_anchored(c, q, P, out);
  if (P.gsel || P.ordered) {
    rc = P.gsel ? run_sel_group(c, q, P, G) : run_ordered(c, q, P, G);
    if (rc) return rc;
    return collect(c, q, P, G, true, out);
  }
  P.seq_dense = seq_dense_wanted(c, P);
  rc = run_device(c, q, P, G, true);
  if (rc) return rc;
  return collect(c, q, P, G, true, out);
}

// Several group-by aggregators over one downsampling (a TSQuery with several sub-queries over
// one metric).  With a percentile / median downsampling function one bucket-selection pass
// leaves every series' buckets in pre_dense / pre_pres and each query runs only its SpanGroup
// step (k_emit + k_reduce) over them; with the cheap functions each query runs the fused
// streaming pass.  The queries must share the time range and the downsampling specification;
// rate, aggregator and flags may differ.
extern "C" int tsdbhip_run_multi(tsdbhip_ctx* c, const tsdbhip_query* qs, int n, tsdbhip_result** outs) {
  if (!c || !qs || !outs || n < 1) return fail(TSDB_E_ILLEGAL_ARGUMENT, "bad argument");
  for (int i = 0; i < n; i++) outs[i] = nullptr;
  // (checked before the multi-device dispatch too: every context refuses the same batches)
  for (int i = 1; i < n; i++) {
    const tsdbhip_query &a = qs[0], &b = qs[i];
    if (a.start_time != b.start_time || a.end_time != b.end_time || a.ds_function != b.ds_function ||
        a.ds_interval_ms != b.ds_interval_ms || a.ds_fill != b.ds_fill || a.ds_all != b.ds_all ||
        a.ds_calendar != b.ds_calendar)
      return fail(TSDB_E_ILLEGAL_ARGUMENT, "tsdbhip_run_multi: the queries must share the time range and downsampling");
  }
  if (c->md) return tsdb::md_run_multi(c, qs, n, outs);
  CtxLock lk(c);
  HIP_OK(hipSetDevice(c->device));
  if (c->ro_active) {
    // a rollup table: each query reads its own aggregate's cells (RollupQuery per sub-query,
    // TsdbQuery.java:1665-1700), so the queries run one after the other
    for (int i = 0; i < n; i++) {
      const int rc = run_rollup(c, &qs[i], &outs[i]);
      if (rc) {
        for (int j = 0; j < n; j++) { result_free(outs[j]); outs[j] = nullptr; }
        return rc;
      }
    }
    return 0;
  }
  const int64_t G = c->n_groups;
  tsdbhip_query q0 = qs[0];
  q0.rate = 0;
  q0.aggregator = TSDB_AGG_SUM;
  q0.flags = 0;
  Plan P0;
  int rc = plan_query(c, &q0, P0);
  if (rc) return rc;
  if (P0.raw) return fail(TSDB_E_NOT_IMPLEMENTED, "tsdbhip_run_multi needs a downsampling specification");
  if (P0.f != F_SEL || P0.anchored) {
    // Cheap downsampling functions: decomposable aggregators (sum, avg, min, max, dev, count)
    // share ONE streaming pass that keeps every aggregator's SpanGroup state (run_multi_fused);
    // otherwise each query runs its own fused pass, which beats a generic group-by step over
    // stored buckets (config 3, 5 aggregators: 22 ms as separate passes vs 35 ms sharing one).
    rc = run_multi_fused(c, qs, n, outs);
    if (rc <= 0) {
      if (rc) for (int j = 0; j < n; j++) { result_free(outs[j]); outs[j] = nullptr; }
      return rc;
    }
    for (int i = 0; i < n; i++) {
      Plan P;
      rc = plan_query(c, &qs[i], P);
      if (!rc) {
        if (P.raw) rc = fail(TSDB_E_ILLEGAL_ARGUMENT, "bad query");
        else if (P.anchored) { rc = run_anchored(c, &qs[i], P, &outs[i]); if (!rc) continue; }
        else if (P.gsel || P.ordered) rc = P.gsel ? run_sel_group(c, &qs[i], P, G) : run_ordered(c, &qs[i], P, G);
        else {
          P.seq_dense = seq_dense_wanted(c, P);   // as tsdbhip_run: sums that cannot add in any order
          rc = run_device(c, &qs[i], P, P.none ? c->n_series : G, true);
        }
        if (!rc) rc = collect(c, &qs[i], P, P.none ? c->n_series : G, true, &outs[i]);
      }
      if (rc) {
        for (int j = 0; j < n; j++) { result_free(outs[j]); outs[j] = nullptr; }
        return rc;
      }
    }
    return 0;
  }
  // percentile / median downsampling: its bucket selection dominates -- share it
  P0.values_only = true;
  rc = run_device(c, &q0, P0, G, false);
  if (rc) return rc;
  int32_t err = 0;
  { int rc_ = d2h_small(c, &err, c->err.p, 4, c->stream); if (rc_) return rc_; }
  { int rc_ = sync_small(c, c->stream); if (rc_) return rc_; }
  if (err) return fail(err, "error raised by the device path");
  for (int i = 0; i < n; i++) {
    Plan P;
    rc = plan_query(c, &qs[i], P);
    if (!rc) {
      if (P.gsel || P.ordered) {
        rc = P.gsel ? run_sel_group(c, &qs[i], P, G) : run_ordered(c, &qs[i], P, G);
        if (!rc) {   // those pipelines overwrote pre_dense: restore the shared buckets
          rc = collect(c, &qs[i], P, G, true, &outs[i]);
          if (!rc && i + 1 < n) rc = run_device(c, &q0, P0, G, false);
        }
      } else {
        P.emit_only = true;
        rc = run_device(c, &qs[i], P, G, true);
        if (!rc) rc = collect(c, &qs[i], P, G, true, &outs[i]);
      }
    }
    if (rc) {
      for (int j = 0; j < n; j++) { result_free(outs[j]); outs[j] = nullptr; }
      return rc;
    }
  }
  return 0;
}

extern "C" void tsdbhip_result_free(tsdbhip_result* r) { result_free(r); }

// result allocation for the expression functions' translation unit (expr.cpp)
namespace tsdb {
tsdbhip_result* new_result(int64_t n_groups, int64_t n_points) { return make_result(n_groups, n_points); }

// multi.cpp: series of a host batch (batch indices, any order) as a device's resident store
int load_series(tsdbhip_ctx* c, const tsdbhip_batch* b, const std::vector<int64_t>& series) {
  return load_with(c, b, &series);
}

// multi.cpp: how a query crosses devices -- partial states, span contributions (percentile /
// median group-by, TSDB_QF_ORDERED), a raw group-by, or the per-span NONE aggregator
int query_kind(tsdbhip_ctx* c, const tsdbhip_query* q, int* kind) {
  if (!q || !kind) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  Plan P;
  const int rc = plan_query(c, q, P);
  if (rc) return rc;
  *kind = P.none ? QK_NONE : P.raw ? QK_RAW : (P.gsel || P.ordered) ? QK_SEL : QK_PARTIALS;
  return 0;
}
}  // namespace tsdb

extern "C" int tsdbhip_last_timing(tsdbhip_ctx* c, tsdbhip_timing* out) {
  if (c && c->md) return tsdb::md_timing(c, out);
  if (!c || !out) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  *out = c->timing;
  out->index_ms = c->index_ms;
  out->compact_ms = c->compact_ms;
  return 0;
}

// ---------------------------------------------------------------------------
// multi-GPU partials: every rank reduces its shard to per-(group, slot) partial
// states; ranks all-gather them (RCCL) and each merges in rank order.
// ---------------------------------------------------------------------------
namespace {

struct PartLayout {
  int64_t off_b, off_n, off_f, off_act, bytes;
};

PartLayout part_layout(int64_t G, int64_t K) {
  PartLayout L;
  const int64_t n = G * K;
  L.off_b = align16(n * 8);
  L.off_n = L.off_b + align16(n * 8);
  L.off_f = L.off_n + align16(n * 4);
  L.off_act = L.off_f + align16(n * 4);
  L.bytes = L.off_act + align16(std::max<int64_t>(1, G) * 4);
  return L;
}

int plan_partials(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t n_groups_global, Plan& P) {
  int rc = plan_query(c, q, P);
  if (rc) return rc;
  if (P.none) return fail(TSDB_E_NOT_IMPLEMENTED, "NONE aggregator is per-span; it has no cross-rank exchange");
  if (P.raw) return fail(TSDB_E_NOT_IMPLEMENTED, "multi-GPU raw (union LERP) queries are not implemented yet");
  if (P.gsel) return fail(TSDB_E_NOT_IMPLEMENTED, "percentile / median group-by: use the tsdbhip_sel_* exchange");
  if (P.ordered) return fail(TSDB_E_NOT_IMPLEMENTED, "TSDB_QF_ORDERED across ranks: use the tsdbhip_sel_* exchange");
  if (P.anchored)
    return fail(TSDB_E_NOT_IMPLEMENTED, "calendar grids anchored per span that disagree across ranks: shard by group");
  if (n_groups_global < c->n_groups) return fail(TSDB_E_ILLEGAL_ARGUMENT, "n_groups_global smaller than the local groups");
  return 0;
}

}  // namespace

extern "C" int tsdbhip_partials_layout_get(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t n_groups_global,
                                           tsdbhip_partials_layout* out) {
  MD_REFUSE(c, "tsdbhip_partials_layout_get");
  if (!c || !q || !out) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  if (c->ro_active) { const int r = ro_check(q); if (r) return r; }
  const tsdbhip_query qr = ro_query(c, q);
  Plan P;
  int rc = plan_partials(c, &qr, n_groups_global, P);
  if (rc) return rc;
  out->n_groups = n_groups_global;
  out->n_slots = P.K;
  out->bytes = part_layout(n_groups_global, P.K).bytes;
  return 0;
}

namespace {
// tsdbhip_run_partials with c->mu held
int run_partials_locked(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t n_groups_global, void* partials) {
  HIP_OK(hipSetDevice(c->device));
  if (c->ro_active) { const int r = ro_check(q); if (r) return r; }
  const tsdbhip_query qr = ro_query(c, q);
  Plan P;
  int rc = plan_partials(c, &qr, n_groups_global, P);
  if (rc) return rc;
  if (c->ro_active) {   // a rollup shard: its scan and (avg / count over counts) the combine pass
    rc = ro_stage(c, q, qr, P);
    if (rc) return rc;
  }
  const int64_t G = n_groups_global, K = P.K;
  const PartLayout L = part_layout(G, K);
  rc = run_device(c, &qr, P, c->n_groups, false);
  if (rc) return rc;
  // merged per-(group, slot) states of this shard; groups this rank does not hold keep
  // the identity state (zero bytes except the min / max identities written below)
  HIP_OK(c->xbuf.ensure(L.bytes));
  unsigned char* xb = c->xbuf.as<unsigned char>();
  HIP_OK(hipMemsetAsync(xb, 0, L.bytes, c->stream));
  if (c->n_groups * K) {
    ReduceParams rp{};
    rp.part = Partials{c->pa.as<double>(), c->pb.as<double>(), c->pn.as<uint32_t>(), c->pf.as<uint32_t>()};
    rp.group_tile_ptr = c->d_gtp.as<int64_t>();
    rp.G = c->n_groups;
    rp.K = K;
    rp.ga = P.ga;
    rp.err = c->err.as<int32_t>();
    rp.state = Partials{reinterpret_cast<double*>(xb), reinterpret_cast<double*>(xb + L.off_b),
                        reinterpret_cast<uint32_t*>(xb + L.off_n), reinterpret_cast<uint32_t*>(xb + L.off_f)};
    HIP_OK(launch_reduce(rp, c->stream));
  }
  if (G > c->n_groups && (P.ga == GA_MIN || P.ga == GA_MAX)) {
    std::vector<double> ident((G - c->n_groups) * K, P.ga == GA_MIN ? INFINITY : -INFINITY);
    HIP_OK(hipMemcpyAsync(xb + c->n_groups * K * 8, ident.data(), ident.size() * 8, hipMemcpyHostToDevice, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
  }
  if (c->n_groups && c->ro_active) {   // + the groups of the spans the rollup scan found
    std::vector<uint32_t> act(c->n_groups);
    HIP_OK(hipMemcpyAsync(act.data(), c->gact.p, c->n_groups * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    ro_activity(c, P, c->n_groups, act);
    HIP_OK(hipMemcpyAsync(xb + L.off_act, act.data(), c->n_groups * 4, hipMemcpyHostToDevice, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
  } else if (c->n_groups) {
    HIP_OK(hipMemcpyAsync(xb + L.off_act, c->gact.p, c->n_groups * 4, hipMemcpyDeviceToDevice, c->stream));
  }
  HIP_OK(hipEventRecord(c->ev[2], c->stream));
  HIP_OK(hipMemcpyAsync(partials, xb, L.bytes, hipMemcpyDefault, c->stream));
  int32_t err = 0, redo_n = 0;
  { int rc_ = d2h_small(c, &err, c->err.p, 4, c->stream); if (rc_) return rc_; }
  if (c->fast_used) { int rc_ = d2h_small(c, &redo_n, c->redo_final, 4, c->stream); if (rc_) return rc_; }
  { int rc_ = sync_small(c, c->stream); if (rc_) return rc_; }
  record_timing(c, P, redo_n);
  if (err) return fail(err, "error raised by the device path");
  return 0;
}

// The fused pass's per-query partial states (tsdbhip_run_partials_multi): query i's merged
// (group, slot) states at partials + i * L.bytes.  1: not fusable (the caller loops).
int run_partials_fused(tsdbhip_ctx* c, const tsdbhip_query* qs, int n, int64_t n_groups_global, void* partials) {
  if (c->ro_active) return 1;   // (a rollup shard stages each aggregate's own cells)
  for (int i = 0; i < n; i++) {
    Plan Pi;
    const int rc = plan_partials(c, &qs[i], n_groups_global, Pi);
    if (rc) return rc;
  }
  Plan P;
  int rc = fused_pass(c, qs, n, P);
  if (rc) return rc;
  const int64_t G = n_groups_global, K = P.K, GL = c->n_groups;
  const PartLayout L = part_layout(G, K);
  HIP_OK(c->xbuf.ensure(L.bytes * n));
  unsigned char* xb0 = c->xbuf.as<unsigned char>();
  HIP_OK(hipMemsetAsync(xb0, 0, L.bytes * n, c->stream));
  std::vector<double> ident;
  for (int i = 0; i < n; i++) {
    unsigned char* xb = xb0 + (int64_t)i * L.bytes;
    const int ga = ga_of(qs[i].aggregator);
    if (GL * K) {
      ReduceParams rp{};
      rp.part = multi_view(c, qs[i].aggregator);
      rp.group_tile_ptr = c->d_gtp.as<int64_t>();
      rp.G = GL;
      rp.K = K;
      rp.ga = ga;
      rp.err = c->err.as<int32_t>();
      rp.state = Partials{reinterpret_cast<double*>(xb), reinterpret_cast<double*>(xb + L.off_b),
                          reinterpret_cast<uint32_t*>(xb + L.off_n), reinterpret_cast<uint32_t*>(xb + L.off_f)};
      HIP_OK(launch_reduce(rp, c->stream));
    }
    if (G > GL && (ga == GA_MIN || ga == GA_MAX)) {   // identity states of the groups this shard lacks
      ident.assign((G - GL) * K, ga == GA_MIN ? INFINITY : -INFINITY);
      HIP_OK(hipMemcpyAsync(xb + GL * K * 8, ident.data(), ident.size() * 8, hipMemcpyHostToDevice, c->stream));
      HIP_OK(hipStreamSynchronize(c->stream));
    }
    if (GL) HIP_OK(hipMemcpyAsync(xb + L.off_act, c->gact.p, GL * 4, hipMemcpyDeviceToDevice, c->stream));
  }
  HIP_OK(hipEventRecord(c->ev[2], c->stream));
  HIP_OK(hipMemcpyAsync(partials, xb0, L.bytes * n, hipMemcpyDefault, c->stream));
  int32_t err = 0, redo_n = 0;
  { int rc_ = d2h_small(c, &err, c->err.p, 4, c->stream); if (rc_) return rc_; }
  { int rc_ = d2h_small(c, &redo_n, c->redo_final, 4, c->stream); if (rc_) return rc_; }
  { int rc_ = sync_small(c, c->stream); if (rc_) return rc_; }
  c->fused_n = n;
  record_timing(c, P, redo_n);
  c->fused_n = 0;
  if (err) return fail(err, "error raised by the device path");
  return 0;
}
}  // namespace

extern "C" int tsdbhip_run_partials(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t n_groups_global, void* partials) {
  MD_REFUSE(c, "tsdbhip_run_partials");
  if (!c || !q || !partials) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  CtxLock lk(c);
  return run_partials_locked(c, q, n_groups_global, partials);
}

// Several queries' partial states from one fused streaming pass (a TSQuery's sub-queries over
// one metric on a rank's shard): as n tsdbhip_run_partials calls, query i's layout at
// partials + i * tsdbhip_partials_layout.bytes.
extern "C" int tsdbhip_run_partials_multi(tsdbhip_ctx* c, const tsdbhip_query* qs, int n, int64_t n_groups_global,
                                          void* partials) {
  MD_REFUSE(c, "tsdbhip_run_partials_multi");
  if (!c || !qs || !partials || n < 1) return fail(TSDB_E_ILLEGAL_ARGUMENT, "bad argument");
  for (int i = 1; i < n; i++) {
    const tsdbhip_query &a = qs[0], &b = qs[i];
    if (a.start_time != b.start_time || a.end_time != b.end_time || a.ds_function != b.ds_function ||
        a.ds_interval_ms != b.ds_interval_ms || a.ds_fill != b.ds_fill || a.ds_all != b.ds_all ||
        a.ds_calendar != b.ds_calendar)
      return fail(TSDB_E_ILLEGAL_ARGUMENT, "tsdbhip_run_partials_multi: the queries must share the time range and downsampling");
  }
  CtxLock lk(c);
  HIP_OK(hipSetDevice(c->device));
  int rc = run_partials_fused(c, qs, n, n_groups_global, partials);
  if (rc <= 0) return rc;
  tsdbhip_partials_layout L{};
  {
    const tsdbhip_query qr = ro_query(c, &qs[0]);
    Plan P;
    rc = plan_partials(c, &qr, n_groups_global, P);
    if (rc) return rc;
    L.bytes = part_layout(n_groups_global, P.K).bytes;
  }
  for (int i = 0; i < n; i++) {
    rc = run_partials_locked(c, &qs[i], n_groups_global, static_cast<unsigned char*>(partials) + (int64_t)i * L.bytes);
    if (rc) return rc;
  }
  return 0;
}

extern "C" int tsdbhip_finalize(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t n_groups_global, const void* partials,
                                int n_ranks, tsdbhip_result** out) {
  MD_REFUSE(c, "tsdbhip_finalize");
  if (!c || !q || !partials || !out || n_ranks < 1) return fail(TSDB_E_ILLEGAL_ARGUMENT, "bad argument");
  CtxLock lk(c);
  *out = nullptr;
  HIP_OK(hipSetDevice(c->device));
  if (c->ro_active) { const int r = ro_check(q); if (r) return r; }
  const tsdbhip_query qr0 = ro_query(c, q);
  q = &qr0;
  c->ro_scan_valid = false;   // the ranks' activity arrives in the partials (no local scan to add)
  Plan P;
  int rc = plan_partials(c, q, n_groups_global, P);
  if (rc) return rc;
  const int64_t G = n_groups_global, K = P.K;
  const PartLayout L = part_layout(G, K);
  HIP_OK(c->gbuf.ensure(L.bytes * n_ranks));
  HIP_OK(hipMemcpyAsync(c->gbuf.p, partials, L.bytes * n_ranks, hipMemcpyDefault, c->stream));
  HIP_OK(c->out_val.ensure(std::max<int64_t>(1, G * K) * 8));
  HIP_OK(c->out_flag.ensure(std::max<int64_t>(1, G * K)));
  HIP_OK(c->gact.ensure(std::max<int64_t>(1, G) * 4));
  HIP_OK(hipMemsetAsync(c->err.p, 0, 4, c->stream));
  RankMergeParams mp{};
  mp.base = c->gbuf.as<unsigned char>();
  mp.stride = L.bytes;
  mp.off_b = L.off_b;
  mp.off_n = L.off_n;
  mp.off_f = L.off_f;
  mp.off_act = L.off_act;
  mp.n_ranks = n_ranks;
  mp.G = G;
  mp.K = K;
  mp.ga = P.ga;
  mp.out_val = c->out_val.as<double>();
  mp.out_flag = c->out_flag.as<uint8_t>();
  mp.out_act = c->gact.as<uint32_t>();
  mp.err = c->err.as<int32_t>();
  HIP_OK(launch_rank_merge(mp, c->stream));
  return collect(c, q, P, G, false, out);
}

// ---------------------------------------------------------------------------
// multi-GPU percentile / median group-by: values go to the group's owning rank
// ---------------------------------------------------------------------------
namespace {

int plan_sel(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t n_groups_global, Plan& P) {
  int rc = plan_query(c, q, P);
  if (rc) return rc;
  if (!P.gsel && !P.ordered)
    return fail(TSDB_E_ILLEGAL_ARGUMENT, "not a percentile / median group-by or TSDB_QF_ORDERED query");
  if (P.anchored)
    return fail(TSDB_E_NOT_IMPLEMENTED, "calendar grids anchored per span that disagree across ranks: shard by group");
  if (n_groups_global < c->n_groups) return fail(TSDB_E_ILLEGAL_ARGUMENT, "n_groups_global smaller than the local groups");
  return 0;
}

// Stages 1-2 on this device: the local spans' contributions stay in c->sel_vals ([span][K] rows,
// groups in SpanGroup order, ungrouped spans last; room for `extra_rows` more rows), the emit
// flags in c->sel_uni; `a` = the groups' active flags on the host.  Caller holds c->mu.
int sel_values_stage(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t G, int64_t extra_rows, Plan& P,
                     std::vector<uint32_t>& a) {
  HIP_OK(hipSetDevice(c->device));
  if (c->ro_active) { const int r = ro_check(q); if (r) return r; }
  const tsdbhip_query qr = ro_query(c, q);
  int rc = plan_sel(c, &qr, G, P);
  if (rc) return rc;
  if (c->ro_active) {
    rc = ro_stage(c, q, qr, P);
    if (rc) return rc;
  }
  if (extra_rows > 0) HIP_OK(c->sel_vals.ensure((c->n_series + extra_rows) * P.K * 8));
  HIP_OK(hipMemsetAsync(c->err.p, 0, 4, c->stream));
  rc = sel_values(c, &qr, P, G);
  if (rc) return rc;
  a.assign(std::max<int64_t>(1, G), 0);
  if (G) HIP_OK(hipMemcpyAsync(a.data(), c->gact.p, G * 4, hipMemcpyDeviceToHost, c->stream));
  int32_t err = 0;
  { int rc_ = d2h_small(c, &err, c->err.p, 4, c->stream); if (rc_) return rc_; }
  { int rc_ = sync_small(c, c->stream); if (rc_) return rc_; }
  if (err) return fail(err, "error raised by the device path");
  ro_activity(c, P, G, a);
  return 0;
}

// Stages 3-4 on this device over rows already on it (`vals`, counts[g] rows per group) and the
// emit flags in c->sel_uni: the order statistic (or, TSDB_QF_ORDERED, the fold in row order)
// of every (group, slot) -> c->out_val / c->out_flag [G][K].  Caller holds c->mu.
int sel_select_stage(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t G, const double* vals,
                     const std::vector<int64_t>& cnt, Plan& P) {
  HIP_OK(hipSetDevice(c->device));
  if (c->ro_active) { const int r = ro_check(q); if (r) return r; }
  const tsdbhip_query qr0 = ro_query(c, q);
  int rc = plan_sel(c, &qr0, G, P);
  if (rc) return rc;
  const int64_t K = P.K;
  HIP_OK(hipMemsetAsync(c->err.p, 0, 4, c->stream));
  if (P.ordered) {   // the owner folds each (group, slot) over the ranks' spans in rank (= span) order
    const std::vector<int64_t> gsp = seg_ptr(cnt);
    HIP_OK(c->sel_gsp.ensure((G + 1) * 8));
    HIP_OK(c->out_val.ensure(std::max<int64_t>(1, G * K) * 8));
    HIP_OK(c->out_flag.ensure(std::max<int64_t>(1, G * K)));
    HIP_OK(hipMemcpyAsync(c->sel_gsp.p, gsp.data(), (G + 1) * 8, hipMemcpyHostToDevice, c->stream));
    OrdParams op{};
    op.vals = vals;
    op.uni = c->sel_uni.as<uint8_t>();
    op.group_series_ptr = c->sel_gsp.as<int64_t>();
    op.G = G;
    op.K = K;
    op.ga = P.ga;
    op.out_val = c->out_val.as<double>();
    op.out_flag = c->out_flag.as<uint8_t>();
    op.err = c->err.as<int32_t>();
    HIP_OK(launch_ordered(op, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));   // `gsp` leaves scope
  } else {
    rc = sel_select(c, P, G, const_cast<double*>(vals), cnt, c->sel_uni.as<uint8_t>());
    if (rc) return rc;
  }
  int32_t err = 0;
  { int rc_ = d2h_small(c, &err, c->err.p, 4, c->stream); if (rc_) return rc_; }
  { int rc_ = sync_small(c, c->stream); if (rc_) return rc_; }
  if (err) return fail(err, "error raised by the device path");
  return 0;
}

}  // namespace

namespace tsdb {
// multi.cpp, owner-routed percentile / ordered exchange: this device's span contributions left in
// place (*vals, on this device) with room for extra_rows more rows after the grouped ones;
// emit flags [G * K] and group activity [G] to the host.
int md_sel_values(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t G, int64_t extra_rows, double** vals,
                  int64_t* K, uint8_t* uni, uint32_t* act) {
  CtxLock lk(c);
  Plan P;
  std::vector<uint32_t> a;
  int rc = sel_values_stage(c, q, G, extra_rows, P, a);
  if (rc) return rc;
  if (G * P.K) HIP_OK(hipMemcpy(uni, c->sel_uni.p, G * P.K, hipMemcpyDeviceToHost));
  std::copy(a.begin(), a.begin() + G, act);
  *vals = c->sel_vals.as<double>();
  *K = P.K;
  return 0;
}

// ... and the owner's selection over rows on its device: out_val / out_flag [G][K] stay on it.
int md_sel_select(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t G, const double* vals, const int64_t* counts,
                  const uint8_t* uni, double** out_val, uint8_t** out_flag) {
  CtxLock lk(c);
  HIP_OK(hipSetDevice(c->device));
  Plan P;
  int rc = plan_sel(c, q, G, P);
  if (rc) return rc;
  HIP_OK(c->sel_uni.ensure(std::max<int64_t>(1, G * P.K)));
  if (G * P.K) HIP_OK(hipMemcpyAsync(c->sel_uni.p, uni, G * P.K, hipMemcpyHostToDevice, c->stream));
  rc = sel_select_stage(c, q, G, vals, std::vector<int64_t>(counts, counts + G), P);
  if (rc) return rc;
  *out_val = c->out_val.as<double>();
  *out_flag = c->out_flag.as<uint8_t>();
  return 0;
}

// multi.cpp, owner-routed partials: the byte offsets of a partials buffer's parts
void partials_offsets(int64_t G, int64_t K, int64_t* off_b, int64_t* off_n, int64_t* off_f, int64_t* off_act,
                      int64_t* bytes) {
  const PartLayout L = part_layout(G, K);
  *off_b = L.off_b;
  *off_n = L.off_n;
  *off_f = L.off_f;
  *off_act = L.off_act;
  *bytes = L.bytes;
}

// ... the owner's step: the states of group g_fold that n_mini later devices hold (mini_state
// layout, in device order) folded into its own state of g_fold (SpanGroup order continues
// across devices), then every group of its buffer finalised -- dense value / emit rows and
// activity in out_val / out_flag / out_act (device memory of this context).
int md_partials_finish(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t G, unsigned char* state, int64_t g_fold,
                       const unsigned char* mini, int n_mini, double* out_val, uint8_t* out_flag, uint32_t* out_act) {
  CtxLock lk(c);
  HIP_OK(hipSetDevice(c->device));
  if (c->ro_active) { const int r = ro_check(q); if (r) return r; }
  const tsdbhip_query qr = ro_query(c, q);
  Plan P;
  int rc = plan_partials(c, &qr, G, P);
  if (rc) return rc;
  const int64_t K = P.K;
  const PartLayout L = part_layout(G, K);
  HIP_OK(hipMemsetAsync(c->err.p, 0, 4, c->stream));
  if (n_mini > 0 && g_fold >= 0 && K > 0) {
    StateFoldParams fp{};
    fp.state = state;
    fp.off_b = L.off_b;
    fp.off_n = L.off_n;
    fp.off_f = L.off_f;
    fp.off_act = L.off_act;
    fp.g = g_fold;
    fp.K = K;
    fp.ga = P.ga;
    fp.mini = mini;
    fp.mini_stride = mini_state_stride(K);
    fp.n_mini = n_mini;
    HIP_OK(launch_state_fold(fp, c->stream));
  }
  RankMergeParams mp{};
  mp.base = state;
  mp.stride = L.bytes;
  mp.off_b = L.off_b;
  mp.off_n = L.off_n;
  mp.off_f = L.off_f;
  mp.off_act = L.off_act;
  mp.n_ranks = 1;
  mp.G = G;
  mp.K = K;
  mp.ga = P.ga;
  mp.out_val = out_val;
  mp.out_flag = out_flag;
  mp.out_act = out_act;
  mp.err = c->err.as<int32_t>();
  HIP_OK(launch_rank_merge(mp, c->stream));
  int32_t err = 0;
  { int rc_ = d2h_small(c, &err, c->err.p, 4, c->stream); if (rc_) return rc_; }
  { int rc_ = sync_small(c, c->stream); if (rc_) return rc_; }
  if (err) return fail(err, "error raised by the device path");
  return 0;
}

// local series per group id < G of the resident batch (multi.cpp: which groups straddle devices)
std::vector<int64_t> ctx_group_counts(tsdbhip_ctx* c, int64_t G) {
  CtxLock lk(c);
  return local_counts(c, G);
}

// resident positions [p0, p1) of group g (the resident order is group-sorted)
void ctx_group_range(tsdbhip_ctx* c, int64_t g, int64_t* p0, int64_t* p1) {
  CtxLock lk(c);
  *p0 = *p1 = 0;
  if (g < 0 || g >= c->n_groups) return;   // (the local sentinel n_groups marks ungrouped series)
  const auto lo = std::lower_bound(c->h_group.begin(), c->h_group.begin() + c->n_series, (int32_t)g);
  const auto hi = std::upper_bound(lo, c->h_group.begin() + c->n_series, (int32_t)g);
  *p0 = lo - c->h_group.begin();
  *p1 = hi - c->h_group.begin();
}
}  // namespace tsdb

extern "C" int tsdbhip_sel_layout(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t n_groups_global, int64_t* counts,
                                  int64_t* n_slots) {
  MD_REFUSE(c, "tsdbhip_sel_layout");
  if (!c || !q || !counts || !n_slots) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  if (c->ro_active) { const int r = ro_check(q); if (r) return r; }
  const tsdbhip_query qr = ro_query(c, q);
  Plan P;
  int rc = plan_sel(c, &qr, n_groups_global, P);
  if (rc) return rc;
  const std::vector<int64_t> n = local_counts(c, n_groups_global);
  for (int64_t g = 0; g < n_groups_global; g++) counts[g] = n[g];
  *n_slots = P.K;
  return 0;
}

extern "C" int tsdbhip_sel_run_values(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t n_groups_global, void* vals,
                                      void* uni, void* act) {
  MD_REFUSE(c, "tsdbhip_sel_run_values");
  if (!c || !q || !vals || !uni || !act) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  CtxLock lk(c);
  Plan P;
  std::vector<uint32_t> a;
  int rc = sel_values_stage(c, q, n_groups_global, 0, P, a);
  if (rc) return rc;
  const int64_t G = n_groups_global, K = P.K;
  int64_t n = 0;   // the grouped spans (ungrouped ones, and a rollup batch's count series, last)
  for (int64_t x : local_counts(c, G)) n += x * K;
  if (n) HIP_OK(hipMemcpyAsync(vals, c->sel_vals.p, n * 8, hipMemcpyDefault, c->stream));
  if (G * K) HIP_OK(hipMemcpyAsync(uni, c->sel_uni.p, G * K, hipMemcpyDefault, c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  if (G) HIP_OK(hipMemcpy(act, a.data(), G * 4, hipMemcpyDefault));
  return 0;
}

extern "C" int tsdbhip_sel_select(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t n_groups_global, const void* vals,
                                  const int64_t* counts, const void* uni, void* out_val, void* out_flag) {
  MD_REFUSE(c, "tsdbhip_sel_select");
  if (!c || !q || !counts || !uni || !out_val || !out_flag) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  CtxLock lk(c);
  HIP_OK(hipSetDevice(c->device));
  if (c->ro_active) { const int r = ro_check(q); if (r) return r; }
  const tsdbhip_query qr0 = ro_query(c, q);
  q = &qr0;
  Plan P;
  int rc = plan_sel(c, q, n_groups_global, P);
  if (rc) return rc;
  const int64_t G = n_groups_global, K = P.K;
  std::vector<int64_t> cnt(counts, counts + G);
  int64_t n = 0;
  for (int64_t g = 0; g < G; g++) {
    if (cnt[g] < 0) return fail(TSDB_E_ILLEGAL_ARGUMENT, "negative count");
    n += cnt[g] * K;
  }
  if (n && !vals) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null vals");
  HIP_OK(c->sel_vals.ensure(std::max<int64_t>(1, n) * 8));
  HIP_OK(c->sel_uni.ensure(std::max<int64_t>(1, G * K)));
  if (n) HIP_OK(hipMemcpyAsync(c->sel_vals.p, vals, n * 8, hipMemcpyDefault, c->stream));
  if (G * K) HIP_OK(hipMemcpyAsync(c->sel_uni.p, uni, G * K, hipMemcpyDefault, c->stream));
  rc = sel_select_stage(c, q, G, c->sel_vals.as<double>(), cnt, P);
  if (rc) return rc;
  if (G * K) {
    HIP_OK(hipMemcpyAsync(out_val, c->out_val.p, G * K * 8, hipMemcpyDefault, c->stream));
    HIP_OK(hipMemcpyAsync(out_flag, c->out_flag.p, G * K, hipMemcpyDefault, c->stream));
  }
  HIP_OK(hipStreamSynchronize(c->stream));
  return 0;
}

extern "C" int tsdbhip_assemble(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t n_groups_global, const void* val,
                                const void* flag, const void* act, tsdbhip_result** out) {
  MD_REFUSE(c, "tsdbhip_assemble");
  if (!c || !q || !val || !flag || !act || !out) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  CtxLock lk(c);
  *out = nullptr;
  HIP_OK(hipSetDevice(c->device));
  if (c->ro_active) { const int r = ro_check(q); if (r) return r; }
  const tsdbhip_query qr0 = ro_query(c, q);
  q = &qr0;
  Plan P;
  int rc = plan_query(c, q, P);
  if (rc) return rc;
  if (P.raw || P.none) return fail(TSDB_E_ILLEGAL_ARGUMENT, "assemble takes downsampled group-by queries");
  if (P.anchored) return fail(TSDB_E_NOT_IMPLEMENTED, "calendar grids anchored per span that disagree: no dense slot grid");
  const int64_t G = n_groups_global, K = P.K;
  HIP_OK(c->out_val.ensure(std::max<int64_t>(1, G * K) * 8));
  HIP_OK(c->out_flag.ensure(std::max<int64_t>(1, G * K)));
  HIP_OK(c->gact.ensure(std::max<int64_t>(1, G) * 4));
  HIP_OK(hipMemsetAsync(c->err.p, 0, 4, c->stream));
  if (G * K) {
    HIP_OK(hipMemcpyAsync(c->out_val.p, val, G * K * 8, hipMemcpyDefault, c->stream));
    HIP_OK(hipMemcpyAsync(c->out_flag.p, flag, G * K, hipMemcpyDefault, c->stream));
  }
  if (G) HIP_OK(hipMemcpyAsync(c->gact.p, act, G * 4, hipMemcpyDefault, c->stream));
  return collect(c, q, P, G, false, out);
}

namespace tsdb {
// multi.cpp's result step: nq queries' dense [G][K] rows gathered on this context's device (query
// i's values / flags at i * stride, its activity words at i * max(1, G)) -> nq results.  One copy
// of each array into the context's page-locked staging and one synchronisation for the whole
// query list, then the queries' host assembly side by side on the assembly pool.  Per query the
// same steps as tsdbhip_assemble + collect (rollup rewrite, "all" window check, activity, rows).
int md_assemble(tsdbhip_ctx* c, const tsdbhip_query* qs, int nq, int64_t G, int64_t stride, const void* val,
                const void* flag, const void* act, tsdbhip_result** outs) {
  if (!c || !qs || nq < 1 || !val || !flag || !act || !outs) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  CtxLock lk(c);
  PhaseTrace tr("md_assemble");
  for (int i = 0; i < nq; i++) outs[i] = nullptr;
  HIP_OK(hipSetDevice(c->device));
  std::vector<tsdbhip_query> qr(nq);
  std::vector<Plan> P(nq);
  for (int i = 0; i < nq; i++) {
    if (c->ro_active) { const int r = ro_check(&qs[i]); if (r) return r; }
    qr[i] = ro_query(c, &qs[i]);
    const int rc = plan_query(c, &qr[i], P[i]);
    if (rc) return rc;
    if (P[i].raw || P[i].none) return fail(TSDB_E_ILLEGAL_ARGUMENT, "assemble takes downsampled group-by queries");
    if (P[i].anchored) return fail(TSDB_E_NOT_IMPLEMENTED, "calendar grids anchored per span that disagree: no dense slot grid");
    if (G * P[i].K > stride) return fail(TSDB_E_ILLEGAL_ARGUMENT, "dense rows wider than the query stride");
  }
  tr.mark("plans");
  const int64_t ga = std::max<int64_t>(1, G);
  const int64_t vb = nq * stride * 8, fb = (nq * stride + 15) & ~(int64_t)15;
  HIP_OK(c->h_stage.ensure(std::max<int64_t>(16, vb + fb + nq * ga * 4)));
  double* hv = reinterpret_cast<double*>(c->h_stage.p);
  uint8_t* hf = reinterpret_cast<uint8_t*>(c->h_stage.p) + vb;
  uint32_t* ha = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(c->h_stage.p) + vb + fb);
  // query by query, each copy followed by its event: the host rows of query i are built while
  // the later queries' rows are still on the link
  std::vector<hipEvent_t> ev(nq, nullptr);
  int rc = 0;
  for (int i = 0; i < nq && !rc; i++) {
    if (stride) {
      if (hipMemcpyAsync(hv + i * stride, static_cast<const double*>(val) + i * stride, stride * 8, hipMemcpyDefault,
                         c->stream) != hipSuccess ||
          hipMemcpyAsync(hf + i * stride, static_cast<const uint8_t*>(flag) + i * stride, stride, hipMemcpyDefault,
                         c->stream) != hipSuccess)
        rc = fail(TSDB_E_HIP, "result rows to the host");
    }
    if (!rc && G && hipMemcpyAsync(ha + i * ga, static_cast<const uint32_t*>(act) + i * ga, ga * 4, hipMemcpyDefault,
                                   c->stream) != hipSuccess)
      rc = fail(TSDB_E_HIP, "result activity to the host");
    if (!rc && (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess ||
                hipEventRecord(ev[i], c->stream) != hipSuccess))
      rc = fail(TSDB_E_HIP, "result copy event");
  }
  if (rc) {
    (void)hipStreamSynchronize(c->stream);
    for (hipEvent_t e : ev) if (e) (void)hipEventDestroy(e);
    return rc;
  }
  tr.mark("d2h issued");
  // the queries in order, each query's rows over the assembly pool (assemble's own split) as soon
  // as its copy has landed (one thread a query left each thread ~1 ms of a 12 h x 1000-group
  // query's 12 MB of rows)
  std::vector<int> rcs(nq, 0);
  for (int64_t i = 0; i < nq; i++) {
    if (hipEventSynchronize(ev[i]) != hipSuccess) {
      rcs[i] = TSDB_E_HIP;
      break;
    }
    const Plan& Pi = P[i];
    uint8_t* f = hf + i * stride;
    if (Pi.mode == MODE_ALL) {   // as collect: the single "all" point only for start_time in the scan window
      const int64_t S0 = Pi.ss * 1000, E0 = Pi.se * 1000;
      if (qr[i].start_time < S0 || qr[i].start_time > E0) std::fill(f, f + G * Pi.K, 0);
    }
    std::vector<uint32_t> a(ha + i * ga, ha + i * ga + ga);
    ro_activity(c, Pi, G, a);
    rcs[i] = assemble(c, &qr[i], Pi, G, hv + i * stride, f, a, &outs[i]);
    if (rcs[i]) break;
  }
  tr.mark("host rows");
  for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  for (int i = 0; i < nq; i++)
    if (rcs[i]) {
      for (int j = 0; j < nq; j++) {
        result_free(outs[j]);
        outs[j] = nullptr;
      }
      return fail(rcs[i], rcs[i] == TSDB_E_HIP ? "result rows to the host" : "result allocation");
    }
  return 0;
}
}  // namespace tsdb

// ===========================================================================
// rollup codec and generation
// ===========================================================================
namespace {

RollupIv to_iv(const tsdbhip_rollup_interval* iv) {
  RollupIv r;
  r.interval_s = iv->interval_s;
  r.intervals = iv->intervals;
  r.units = iv->units;
  r.mult = iv->unit_multiplier;
  return r;
}

bool iv_valid(const tsdbhip_rollup_interval* iv) {
  return iv && iv->interval_s >= 1 && iv->intervals >= 1 &&
         (iv->units == 'h' || iv->units == 'd' || iv->units == 'n' || iv->units == 'y');
}

}  // namespace

// new RollupInterval(builder) + validateAndCompile (src/rollup/RollupInterval.java:62-103,169-235),
// with DateTime.getDurationUnits / getDurationInterval (src/utils/DateTime.java:237-284).
extern "C" int tsdbhip_rollup_interval_parse(const char* interval, const char* row_span, tsdbhip_rollup_interval* out) {
  if (!out) return fail(TSDB_E_ILLEGAL_ARGUMENT, "out is null");
  if (!row_span || !*row_span) return fail(TSDB_E_ILLEGAL_ARGUMENT, "Duration cannot be null or empty");
  size_t u = 0;
  const size_t n = std::strlen(row_span);
  while (u < n && std::isdigit((unsigned char)row_span[u])) u++;
  std::string units(row_span + u);
  for (auto& ch : units) ch = (char)std::tolower((unsigned char)ch);
  static const char* const ok[] = {"ms", "s", "m", "h", "d", "w", "n", "y"};
  bool valid = false;
  for (const char* o : ok) valid |= units == o;
  if (!valid) return fail(TSDB_E_ILLEGAL_ARGUMENT, "Invalid units in the duration: " + units);
  if (units.size() > 1) return fail(TSDB_E_ILLEGAL_ARGUMENT, "Milliseconds are not supported");
  if (std::strchr(row_span, '.')) return fail(TSDB_E_ILLEGAL_ARGUMENT, "Floating point intervals are not supported");
  if (u == 0 || u > 10) return fail(TSDB_E_ILLEGAL_ARGUMENT, std::string("Invalid duration (number): ") + row_span);
  const long long mult_ll = std::stoll(std::string(row_span, u));
  if (mult_ll > 2147483647LL) return fail(TSDB_E_ILLEGAL_ARGUMENT, std::string("Invalid duration (number): ") + row_span);
  const int32_t mult = (int32_t)mult_ll;
  if (mult <= 0) return fail(TSDB_E_ILLEGAL_ARGUMENT, std::string("Zero or negative duration: ") + row_span);
  const char un = units[0];
  if (un != 'h' && mult > 1) return fail(TSDB_E_ILLEGAL_ARGUMENT, "Multipliers are only usable with the 'h' unit");
  if (un == 'h' && mult > 1 && mult % 2 != 0) return fail(TSDB_E_ILLEGAL_ARGUMENT, "The multiplier must be 1 or an even value");
  if (!interval) return fail(TSDB_E_ILLEGAL_ARGUMENT, "interval is null");
  int64_t ms = 0;
  int rc = tsdbhip_parse_duration(interval, &ms);
  if (rc) return rc;
  const int32_t iv_s = (int32_t)(uint32_t)(uint64_t)(ms / 1000);   // Java (int) of a long
  if (iv_s < 1) return fail(TSDB_E_ILLEGAL_ARGUMENT, "Millisecond intervals are not supported");
  if (iv_s >= 2147483647) return fail(TSDB_E_ILLEGAL_ARGUMENT, "Interval is too big");
  int32_t num_span;
  switch (un) {
    case 'h': num_span = 3600; break;
    case 'd': num_span = 86400; break;
    case 'n': num_span = 86400 * 32; break;
    case 'y': num_span = 86400 * 366; break;
    default: return fail(TSDB_E_ILLEGAL_ARGUMENT, std::string("Unrecogznied span '") + un + "'");
  }
  num_span = (int32_t)((uint32_t)num_span * (uint32_t)mult);
  if (iv_s >= num_span) return fail(TSDB_E_ILLEGAL_ARGUMENT, "Interval is too large for the span");
  const int32_t intervals = num_span / iv_s;
  if (intervals > 7774) return fail(TSDB_E_ILLEGAL_ARGUMENT, "Too many intervals in the span");
  if (intervals < 12) return fail(TSDB_E_ILLEGAL_ARGUMENT, "Not enough intervals for the span");
  out->interval_s = iv_s;
  out->intervals = intervals;
  out->units = un;
  out->interval_units = interval[std::strlen(interval) - 1];
  out->unit_multiplier = (int16_t)std::min<int32_t>(mult, 32767);
  return 0;
}

extern "C" int tsdbhip_rollup_basetime(int64_t timestamp, const tsdbhip_rollup_interval* iv, int32_t* out) {
  if (!iv || !out) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  if (!rc_basetime(timestamp, to_iv(iv), *out))
    return fail(TSDB_E_ILLEGAL_ARGUMENT, "Not supporting negative timestamps / unrecognised span");
  return 0;
}

extern "C" int tsdbhip_rollup_qualifier(int64_t timestamp, int32_t basetime, int16_t flags, int32_t aggregator_id,
                                        const tsdbhip_rollup_interval* iv, uint8_t out[3]) {
  if (!iv || !out) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  if (iv->interval_s < 1) return fail(TSDB_E_ILLEGAL_ARGUMENT, "bad interval");
  if (!rc_qualifier(timestamp, basetime, flags, aggregator_id, to_iv(iv), out))
    return fail(TSDB_E_ILLEGAL_ARGUMENT, "Offset was greater than the configured intervals");
  return 0;
}

extern "C" int tsdbhip_rollup_run(tsdbhip_ctx* c, const tsdbhip_rollup_spec* sp, int64_t* n_cells, uint64_t* value_bytes) {
  if (c && c->md) return tsdb::md_rollup_run(c, sp, n_cells, value_bytes);
  if (c && c->ro_active) return fail(TSDB_E_NOT_IMPLEMENTED, "tsdbhip_rollup_run over a rollup batch (tsdbhip_load_rollup)");
  if (!c || !sp) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  if (!iv_valid(&sp->interval)) return fail(TSDB_E_ILLEGAL_ARGUMENT, "invalid rollup interval");
  if (sp->n_funcs < 1 || sp->n_funcs > 4) return fail(TSDB_E_ILLEGAL_ARGUMENT, "1..4 rollup functions");
  if (sp->start_s < 0 || sp->end_s <= sp->start_s) return fail(TSDB_E_ILLEGAL_ARGUMENT, "bad rollup time range");
  for (int i = 0; i < sp->n_funcs; i++) {
    const int f = sp->func[i];
    if (f != TSDB_AGG_SUM && f != TSDB_AGG_COUNT && f != TSDB_AGG_MAX && f != TSDB_AGG_MIN)
      return fail(TSDB_E_ILLEGAL_ARGUMENT, "rollup functions are sum, count, max and min");
  }
  CtxLock lk(c);
  HIP_OK(hipSetDevice(c->device));
  c->ro_n = 0;
  // the series with a group (ungrouped ones -- group id -1 -- sit after them and get no rollups)
  int64_t n = 0;
  while (n < c->n_series && c->h_group[n] < c->n_groups) n++;
  // batch order -> sorted position, and the per-series integer flag (once per loaded batch)
  if (!c->ro_meta_valid) {
    std::vector<int64_t> ord(n);
    std::iota(ord.begin(), ord.end(), 0);
    std::sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return c->h_orig[a] < c->h_orig[b]; });
    HIP_OK(c->ro_ord.ensure(std::max<int64_t>(1, n) * 8));
    HIP_OK(c->ro_orig.ensure(std::max<int64_t>(1, n) * 8));
    HIP_OK(c->ro_allint.ensure(std::max<int64_t>(1, n)));
    if (n) {
      HIP_OK(hipMemcpyAsync(c->ro_ord.p, ord.data(), n * 8, hipMemcpyHostToDevice, c->stream));
      HIP_OK(hipMemcpyAsync(c->ro_orig.p, c->h_orig.data(), n * 8, hipMemcpyHostToDevice, c->stream));
    }
    HIP_OK(launch_series_allint(c->rows.as<RowDesc>(), c->srp.as<int64_t>(), n, c->ro_allint.as<uint8_t>(), c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));   // `ord` leaves scope
    c->ro_meta_valid = true;
  }
  // Downsampler of every series at the rollup interval (fill none; the geometry of a NONE-
  // aggregator query): one fused pass reduces every bucket with sum, count, max and min
  tsdbhip_query q{};
  q.start_time = sp->start_s;
  q.end_time = sp->end_s - 1;
  q.aggregator = TSDB_AGG_NONE;
  q.ds_function = TSDB_AGG_SUM;
  q.ds_fill = TSDB_FILL_NONE;
  q.ds_interval_ms = (int64_t)sp->interval.interval_s * 1000;
  q.rate_counter_max = INT64_MAX;
  Plan P;
  {
    int rc = plan_query(c, &q, P);
    if (rc) return rc;
  }
  const int64_t NS = c->n_series;
  HIP_OK(c->ro_agg.ensure(std::max<int64_t>(1, 4 * NS * P.K) * 8));
  HIP_OK(c->ro_pres.ensure(std::max<int64_t>(1, NS * P.K)));
  HIP_OK(hipMemsetAsync(c->err.p, 0, 4, c->stream));
  HIP_OK(hipEventRecord(c->ev[0], c->stream));
  {
    GridParams gp{};
    gp.rows = c->rows.as<RowDesc>();
    gp.series_row_ptr = c->srp.as<int64_t>();
    gp.qual = c->qual.as<uint8_t>();
    gp.val = c->val.as<uint8_t>();
    gp.ss = P.ss;
    gp.se = P.se;
    gp.B0 = P.B0;
    gp.I = P.I;
    gp.K = P.K;
    gp.rcpI = (float)(1.0 / (double)P.I);
    gp.mode = MODE_GRID;
    gp.seek_any = P.B0;
    gp.n_series = n;
    gp.err = c->err.as<int32_t>();
    gp.val2 = c->val2.as<uint8_t>();
    RollupAggParams ap{};
    ap.out = c->ro_agg.as<double>();
    ap.stride = NS * P.K;
    ap.K = P.K;
    ap.pres = c->ro_pres.as<uint8_t>();
    // streaming kernel per row class (class A over every series, class B over what A handed
    // back), then the general kernel over the rest
    const bool fast = !opt_off(OPT_FAST) && c->fast_qw && n > 0 && P.I <= (1LL << 29) &&
                      rollup_fast_lds(P.K) <= 32 * 1024;
    const int32_t* list = nullptr;
    const int32_t* list_n = nullptr;
    if (fast) {
      HIP_OK(c->r1a.ensure(n * 4));
      HIP_OK(c->r2.ensure(n * 4));
      HIP_OK(c->r_n.ensure(16));
      HIP_OK(hipMemsetAsync(c->r_n.p, 0, 16, c->stream));
      int32_t* rn = c->r_n.as<int32_t>();
      int32_t* outs[2] = {c->r1a.as<int32_t>(), c->r2.as<int32_t>()};
      for (int cls = 0; cls < 2; cls++) {
        const int qw = cls ? c->fast_qw2 : c->fast_qw, vl = cls ? c->fast_vl2 : c->fast_vl;
        if (!qw || !rollup_fast_supported(qw, vl) || (cls == 1 && !list)) continue;
        GridParams fp = gp;
        fp.unit_s = (qw == 2 && P.I % 1000 == 0 && P.B0 % 1000 == 0) ? 1 : 0;
        fp.In = (int32_t)(fp.unit_s ? P.I / 1000 : P.I);
        fp.B0n = fp.unit_s ? P.B0 / 1000 : P.B0;
        fp.rcpn = std::nextafter(1.0 / (double)fp.In, INFINITY);
        fp.wave_lds = (int32_t)rollup_fast_lds(P.K);
        fp.waves = (int)std::max<int64_t>(1, std::min<int64_t>(4, (64 * 1024) / std::max<int64_t>(16, fp.wave_lds)));
        fp.tile_list = list;
        fp.tile_list_n = list_n;
        fp.n_launch = n;
        fp.redo_list = outs[cls];
        fp.redo_n = rn + cls;
        HIP_OK(launch_rollup_fast(fp, ap, qw, vl, c->stream));
        list = outs[cls];
        list_n = rn + cls;
      }
    }
    if (list) {
      gp.tile_list = list;
      gp.tile_list_n = list_n;
      gp.n_launch = std::min<int64_t>(n, 16384);
    }
    HIP_OK(launch_rollup_agg(gp, ap, c->stream));
  }
  HIP_OK(hipEventRecord(c->ev[1], c->stream));
  for (int fi = 0; fi < sp->n_funcs; fi++) {
    const int f = sp->func[fi];
    const int fslot = f == TSDB_AGG_SUM ? 0 : f == TSDB_AGG_COUNT ? 1 : f == TSDB_AGG_MAX ? 2 : 3;
    const int64_t NK = n * P.K;
    HIP_OK(c->ro_cnt.ensure(std::max<int64_t>(1, NK) * 4));
    HIP_OK(c->ro_vsz.ensure(std::max<int64_t>(1, NK) * 4));
    HIP_OK(c->ro_coff.ensure(std::max<int64_t>(1, NK) * 8));
    HIP_OK(c->ro_voff.ensure(std::max<int64_t>(1, NK) * 8));
    RollupParams rp{};
    rp.val = c->ro_agg.as<double>() + fslot * NS * P.K;
    rp.flag = c->ro_pres.as<uint8_t>();
    rp.ord = c->ro_ord.as<int64_t>();
    rp.orig = c->ro_orig.as<int64_t>();
    rp.allint = c->ro_allint.as<uint8_t>();
    rp.n = NK;
    rp.K = P.K;
    rp.B0 = P.B0;
    rp.I = P.I;
    rp.start_ms = sp->start_s * 1000;
    rp.end_ms = sp->end_s * 1000;
    rp.iv = to_iv(&sp->interval);
    rp.agg_id = sp->agg_id[fi];
    rp.as_long_all = sp->func[fi] == TSDB_AGG_COUNT;
    rp.cnt = c->ro_cnt.as<uint32_t>();
    rp.vsz = c->ro_vsz.as<uint32_t>();
    rp.coff = c->ro_coff.as<int64_t>();
    rp.voff = c->ro_voff.as<uint64_t>();
    rp.err = c->err.as<int32_t>();
    HIP_OK(launch_rollup_size(rp, c->stream));
    if (NK > 0x7FFFFFFFLL) return fail(TSDB_E_NOT_IMPLEMENTED, "more than 2^31 rollup buckets in one pass");
    if (NK) HIP_OK(rollup_scan(rp.cnt, c->ro_coff.as<int64_t>(), rp.vsz, c->ro_voff.as<uint64_t>(), NK, &c->ro_tmp,
                               &c->ro_tmp_bytes, c->stream));
    // totals = last offset + last element
    int64_t last_off = 0;
    uint64_t last_voff = 0;
    uint32_t last_c = 0, last_v = 0;
    int32_t err = 0;
    if (NK) {
      { int rc_ = d2h_small(c, &last_off, c->ro_coff.as<int64_t>() + NK - 1, 8, c->stream); if (rc_) return rc_; }
      { int rc_ = d2h_small(c, &last_voff, c->ro_voff.as<uint64_t>() + NK - 1, 8, c->stream); if (rc_) return rc_; }
      { int rc_ = d2h_small(c, &last_c, rp.cnt + NK - 1, 4, c->stream); if (rc_) return rc_; }
      { int rc_ = d2h_small(c, &last_v, rp.vsz + NK - 1, 4, c->stream); if (rc_) return rc_; }
    }
    { int rc_ = d2h_small(c, &err, c->err.p, 4, c->stream); if (rc_) return rc_; }
    { int rc_ = sync_small(c, c->stream); if (rc_) return rc_; }
    // an infinite bucket value trips AggregationIterator's Inf check (IllegalStateException)
    // in the NONE-aggregator pass; for a rollup it is addAggregatePoint's rejection
    if (err == TSDB_E_ILLEGAL_STATE) err = TSDB_E_ILLEGAL_ARGUMENT;
    if (err) return fail(err, "rollup generation: value or offset rejected (addAggregatePoint / buildRollupQualifier)");
    auto& o = c->ro_out[fi];
    o.cells = last_off + last_c;
    o.bytes = last_voff + last_v;
    HIP_OK(o.series.ensure(std::max<int64_t>(1, o.cells) * 4));
    HIP_OK(o.base.ensure(std::max<int64_t>(1, o.cells) * 4));
    HIP_OK(o.qual.ensure(std::max<int64_t>(1, o.cells) * 3));
    HIP_OK(o.voff.ensure((o.cells + 1) * 8));
    HIP_OK(o.val.ensure(std::max<uint64_t>(1, o.bytes)));
    rp.o_series = o.series.as<int32_t>();
    rp.o_base = o.base.as<uint32_t>();
    rp.o_qual = o.qual.as<uint8_t>();
    rp.o_voff = o.voff.as<uint64_t>();
    rp.o_val = o.val.as<uint8_t>();
    HIP_OK(launch_rollup_write(rp, c->stream));
    HIP_OK(hipMemcpyAsync(o.voff.as<uint64_t>() + o.cells, &o.bytes, 8, hipMemcpyHostToDevice, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    c->ro_n = fi + 1;
  }
  HIP_OK(hipEventRecord(c->ev[2], c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  {
    float t01 = 0, t02 = 0;
    (void)hipEventElapsedTime(&t01, c->ev[0], c->ev[1]);
    (void)hipEventElapsedTime(&t02, c->ev[0], c->ev[2]);
    c->timing.decode_downsample_ms = t01;   // the fused sum / count / max / min pass
    c->timing.group_reduce_ms = t02 - t01;  // cell sizing, scans and writes
    c->timing.total_ms = t02;
    c->timing.fast_ms = 0;
    account(c, P);
  }
  int64_t cells = 0;
  uint64_t bytes = 0;
  for (int i = 0; i < c->ro_n; i++) { cells += c->ro_out[i].cells; bytes += c->ro_out[i].bytes; }
  if (n_cells) *n_cells = cells;
  if (value_bytes) *value_bytes = bytes;
  return 0;
}

extern "C" int tsdbhip_rollup_download(tsdbhip_ctx* c, int32_t* series, uint32_t* base_time, uint8_t* qualifier,
                                       uint64_t* val_off, uint8_t* value) {
  if (c && c->md) return tsdb::md_rollup_download(c, series, base_time, qualifier, val_off, value);
  if (!c) return fail(TSDB_E_ILLEGAL_ARGUMENT, "null ctx");
  CtxLock lk(c);
  HIP_OK(hipSetDevice(c->device));
  int64_t cell0 = 0;
  uint64_t byte0 = 0;
  for (int i = 0; i < c->ro_n; i++) {
    const auto& o = c->ro_out[i];
    if (o.cells) {
      if (series) HIP_OK(hipMemcpy(series + cell0, o.series.p, o.cells * 4, hipMemcpyDeviceToHost));
      if (base_time) HIP_OK(hipMemcpy(base_time + cell0, o.base.p, o.cells * 4, hipMemcpyDeviceToHost));
      if (qualifier) HIP_OK(hipMemcpy(qualifier + 3 * cell0, o.qual.p, o.cells * 3, hipMemcpyDeviceToHost));
      if (val_off) {
        HIP_OK(hipMemcpy(val_off + cell0, o.voff.p, o.cells * 8, hipMemcpyDeviceToHost));
        for (int64_t k = 0; k < o.cells; k++) val_off[cell0 + k] += byte0;
      }
      if (value && o.bytes) HIP_OK(hipMemcpy(value + byte0, o.val.p, o.bytes, hipMemcpyDeviceToHost));
    }
    cell0 += o.cells;
    byte0 += o.bytes;
  }
  if (val_off) val_off[cell0] = byte0;
  return 0;
}

namespace tsdb {
// Host -> device upload of a scan's arrays (tsdbhip_load_cells).  The queue's copy engine ran these
// uploads at half the PCIe rate on every call after the first (576 MB in 19 ms against 10 ms; blit
// copies 10 ms: profiles/r05n, r05o), so the GPU pulls the bytes itself (k_pull, 16-byte loads
// over the device mapping of page-locked memory):
//   - page-locked sources (tsdbhip_host_alloc, registered memory): pulled directly;
//   - pageable sources: copied into two page-locked staging chunks of the context by the host's
//     assembly threads, each chunk pulled while the next one is copied (hipEvents order the reuse).
// Small or misaligned copies, and TSDBHIP_PULL=0, take hipMemcpyAsync.
constexpr size_t UP_CHUNK = (size_t)32 << 20;
hipError_t h2d(tsdbhip_ctx* c, void* dst, const void* src, size_t n, hipStream_t st) {
  if (n < ((size_t)1 << 20) || ((uintptr_t)dst & 15) != 0) return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, st);
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, src) == hipSuccess && a.type == hipMemoryTypeHost && a.devicePointer) {
    if ((((uintptr_t)src ^ (uintptr_t)dst) & 15) != 0) return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, st);
    const size_t off = a.hostPointer ? (size_t)((const char*)src - (const char*)a.hostPointer) : 0;
    return launch_pull(dst, (const char*)a.devicePointer + off, n, st);
  }
  (void)hipGetLastError();   // (pageable memory: no attributes)
  for (int i = 0; i < 2; i++) {
    if (!c->up_stage[i]) {
      hipError_t e = hipHostMalloc(&c->up_stage[i], UP_CHUNK, hipHostMallocDefault);
      if (e != hipSuccess) { c->up_stage[i] = nullptr; return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, st); }
      e = hipEventCreateWithFlags(&c->up_ev[i], hipEventDisableTiming);
      if (e != hipSuccess) return e;
    }
  }
  AssemblyPool& pool = AssemblyPool::get();
  const char* s8 = static_cast<const char*>(src);
  char* d8 = static_cast<char*>(dst);
  for (size_t off = 0, i = 0; off < n; off += UP_CHUNK, i++) {
    const int b = (int)(i & 1);
    const size_t len = std::min(UP_CHUNK, n - off);
    if (c->up_busy[b]) {
      const hipError_t e = hipEventSynchronize(c->up_ev[b]);
      if (e != hipSuccess) return e;
    }
    char* stage = static_cast<char*>(c->up_stage[b]);
    const int nt = len >= ((size_t)8 << 20) ? pool.width() : 1;
    const std::function<void(int)> part = [&](int t) {
      const size_t a0 = (len * t / nt) & ~(size_t)63, a1 = t + 1 == nt ? len : (len * (t + 1) / nt) & ~(size_t)63;
      std::memcpy(stage + a0, s8 + off + a0, a1 - a0);
    };
    if (nt <= 1 || !pool.run(nt, part)) std::memcpy(stage, s8 + off, len);
    hipError_t e = launch_pull(d8 + off, stage, len, st);   // (page-locked memory: the host pointer maps)
    if (e == hipSuccess) e = hipEventRecord(c->up_ev[b], st);
    if (e != hipSuccess) return e;
    c->up_busy[b] = true;
  }
  return hipSuccess;
}
}  // namespace tsdb
