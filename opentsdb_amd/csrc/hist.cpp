// hist.cpp -- host side of the histogram path: tsdbhip_load_histograms,
// tsdbhip_hist_run.  The kernels are in k_hist.hip.
//
// Reference: TsdbQuery.runHistogram -> HistogramGroupByAndAggregateCB
// (src/core/TsdbQuery.java:759-776, 1061-1287), SaltScanner's histogram rows
// (src/core/SaltScanner.java:734-800, 336-378) and HistogramSpan.addRow
// (src/core/HistogramSpan.java:280-328, HistogramRowSeq.addRow :66-105).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/tsdbhip.h"
#include "hist.h"

namespace tsdb {
hipStream_t ctx_stream(tsdbhip_ctx* c);
int ctx_device(tsdbhip_ctx* c);
std::mutex& ctx_mutex(tsdbhip_ctx* c);
void*& ctx_hist(tsdbhip_ctx* c);
int set_error(int code, const std::string& msg);
bool cal_prev_tz(const tsdbhip_tz* z, int64_t ts, int64_t n, int unit, int64_t* out);
int64_t cal_step_tz(const tsdbhip_tz* z, int64_t t, int unit, int64_t n);
int64_t cal_unit_ms(int unit);
void*& ctx_md(tsdbhip_ctx* c);
// multi.cpp: the histogram store of a multi-device context, whole groups per device
int md_load_histograms(tsdbhip_ctx* c, const tsdbhip_hist_batch* hb);
int md_hist_run(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t start, int64_t end, int64_t ss, int64_t se, int n_pct,
                const float* pct, int show_buckets, tsdbhip_hist_result** out);

namespace {

#define HOK(expr)                                                                           \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess) return set_error(TSDB_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

struct Buf {
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

// The resident histogram store.
struct HistStore {
  bool loaded = false;
  int64_t n_series = 0, n_cells = 0, n_pos = 0;
  Buf val, voff, codec, status, hkey, hcount, hidx, dlo, dup, lkey, lidx, lkey2, lidx2;
  int lslots = 64;                              // k_hist_accw's compact LDS dictionary table
  bool lds_dict = false;                        // the dictionary fits the LDS table of k_hist_accum
  Buf pos_cell, pos_ts, pos_kind, row_pos;
  Buf col_lid, lay_col, lay_off, lay_di;        // bucket layouts: dictionary indices without the keys
  int64_t n_layouts = 0;
  int32_t D = 0;
  int64_t max_ts = 0;                           // largest datapoint timestamp of the store (ms)
  std::vector<uint32_t> h_dlo, h_dup;           // dictionary bounds (float bits), TreeMap order
  std::vector<int64_t> sp_row;                  // [n_series + 1] kept rows of each span (base-time order)
  std::vector<int64_t> h_pos_ts, h_row_pos;     // host copies (calendar anchors are planned on the host)
  std::vector<uint32_t> row_base;               // [kept rows]
  std::vector<int32_t> group;                   // [n_series]
  // query scratch
  Buf q_rlo, q_rhi, q_out, q_slot, q_key, q_key2, q_pos, q_pos2, q_head, q_incl, q_point, q_ptts, q_ptgrp;
  Buf q_vlen, q_voff, q_vpos, q_tix;   // windowed accumulation: the spans' positions in output-group order, their entries
  Buf q_caltab, q_spcal;         // calendar downsampling: boundary runs per span anchor
  Buf q_gsp, q_spq, q_spts;      // greedy walk over spans out of time order (k_hist_walk)
  Buf acc, pres, pkind, flag, ptout, err, pct;
  Buf o_ts, o_grp, o_kind, o_pct, o_cnt, o_pres;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  void release() {
    for (Buf* b : {&val, &voff, &codec, &status, &hkey, &hcount, &hidx, &dlo, &dup, &lkey, &lidx, &lkey2, &lidx2, &pos_cell, &pos_ts, &pos_kind,
                   &row_pos, &col_lid, &lay_col, &lay_off, &lay_di, &q_rlo, &q_rhi, &q_out, &q_slot, &q_key, &q_key2, &q_pos, &q_pos2, &q_head, &q_incl,
                   &q_point, &q_ptts, &q_ptgrp, &q_vlen, &q_voff, &q_vpos, &q_tix, &q_caltab, &q_spcal, &q_gsp, &q_spq, &q_spts, &acc, &pres, &pkind, &flag, &ptout, &err, &pct, &o_ts, &o_grp,
                   &o_kind, &o_pct, &o_cnt, &o_pres})
      b->release();
    if (tmp) (void)hipFree(tmp);
    tmp = nullptr;
    tmp_bytes = 0;
  }
};

HistStore* store_of(tsdbhip_ctx* c) {
  void*& h = ctx_hist(c);
  if (!h) h = new HistStore();
  return static_cast<HistStore*>(h);
}

// Internal.getTimeStampFromNonDP (src/core/Internal.java:1059-1074); false: invalid qualifier
bool nondp_ts(int64_t base, const uint8_t* q, uint64_t ql, int64_t* out) {
  if (ql == 3) {
    const int32_t off = (int32_t)((uint32_t)(int32_t)(int8_t)q[1] << 8) | q[2];
    *out = (base + off) * 1000;
    return true;
  }
  if (ql == 5) {
    const int32_t off = (int32_t)(((uint32_t)q[1] << 24) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 8) | q[4]);
    *out = base * 1000 + off;
    return true;
  }
  return false;
}

inline uint32_t ford(uint32_t b) { return (b & 0x80000000u) ? ~b : (b | 0x80000000u); }   // Float.compare order

// One HistogramRowSeq while the span is assembled: its datapoints as (timestamp, column)
struct HRow {
  uint32_t base;
  std::vector<std::pair<int64_t, int64_t>> dp;
};

// HistogramRowSeq.addRow (:66-105): merge by timestamp, the local datapoint kept on a tie
void row_merge(HRow& local, const HRow& remote) {
  std::vector<std::pair<int64_t, int64_t>> out;
  out.reserve(local.dp.size() + remote.dp.size());
  size_t il = 0, ir = 0;
  while (il < local.dp.size() && ir < remote.dp.size()) {
    const int64_t sort = remote.dp[ir].first - local.dp[il].first;
    if (sort == 0) { out.push_back(local.dp[il++]); ir++; }
    else if (sort > 0) out.push_back(local.dp[il++]);
    else out.push_back(remote.dp[ir++]);
  }
  while (il < local.dp.size()) out.push_back(local.dp[il++]);
  while (ir < remote.dp.size()) out.push_back(remote.dp[ir++]);
  local.dp.swap(out);
}

struct HistResultOwner {
  tsdbhip_hist_result r{};
  std::vector<int32_t> gid;
  std::vector<int64_t> gptr, ts, cnt;
  std::vector<double> pct;
  std::vector<uint32_t> blo, bup;
  std::vector<uint8_t> pres, kind;
};

}  // namespace

void hist_release(void* h) {
  if (!h) return;
  auto* s = static_cast<HistStore*>(h);
  s->release();
  delete s;
}

}  // namespace tsdb

using namespace tsdb;

// On a multi-device context (tsdbhip_init_devices) the histogram spans are sharded by whole groups
// over the devices (multi.cpp md_load_histograms); every device's store is loaded here.
extern "C" int tsdbhip_load_histograms(tsdbhip_ctx* c, const tsdbhip_hist_batch* hb) {
  if (!c || !hb) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  if (ctx_md(c)) return md_load_histograms(c, hb);
  std::lock_guard<std::mutex> lk(ctx_mutex(c));
  HOK(hipSetDevice(ctx_device(c)));
  hipStream_t st = ctx_stream(c);
  HistStore* S = store_of(c);
  S->loaded = false;
  const int64_t NS = hb->n_series, NR = hb->n_rows, NC = hb->n_cells;
  if (NS < 0 || NR < 0 || NC < 0 || !hb->series_row_ptr || (NR && (!hb->row_base_time || !hb->row_cell_ptr)) ||
      (NC && (!hb->cell_qual_off || !hb->cell_val_off)) || (NS && !hb->group_id))
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "malformed histogram batch");
  if (hb->series_row_ptr[0] != 0 || hb->series_row_ptr[NS] != NR || (NR && (hb->row_cell_ptr[0] != 0 || hb->row_cell_ptr[NR] != NC)))
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "histogram batch offsets do not cover the rows / columns");
  if (NC >= ((int64_t)1 << 31)) return set_error(TSDB_E_NOT_IMPLEMENTED, "more than 2^31 histogram columns in one store");
  const uint64_t vbytes = NC ? hb->cell_val_off[NC] : 0;
  // 1. device: decode check of every column, bucket keys into the dictionary hash set
  HOK(S->val.ensure(vbytes + 64));   // (k_hist_accw stages whole 16-byte units past a column's end)
  HOK(S->voff.ensure((NC + 1) * 8));
  HOK(S->codec.ensure(256));
  HOK(S->status.ensure(NC + 1));
  HOK(S->hkey.ensure(HT_SIZE * 8));
  HOK(S->hcount.ensure(16));
  if (vbytes) HOK(hipMemcpyAsync(S->val.p, hb->val, vbytes, hipMemcpyHostToDevice, st));
  if (NC) HOK(hipMemcpyAsync(S->voff.p, hb->cell_val_off, (NC + 1) * 8, hipMemcpyHostToDevice, st));
  HOK(hipMemcpyAsync(S->codec.p, hb->codec, 256, hipMemcpyHostToDevice, st));
  HOK(hipMemsetAsync(S->hkey.p, 0xFF, HT_SIZE * 8, st));
  HOK(hipMemsetAsync(S->hcount.p, 0, 16, st));
  HistLoadParams lp{NC, S->voff.as<uint64_t>(), S->val.as<uint8_t>(), S->codec.as<uint8_t>(), S->status.as<uint8_t>(),
                    S->hkey.as<uint64_t>(), S->hcount.as<int32_t>()};
  HOK(hist_validate(lp, st));
  std::vector<uint8_t> status(NC);
  std::vector<uint64_t> hkey(HT_SIZE);
  int32_t hcount = 0;
  if (NC) HOK(hipMemcpyAsync(status.data(), S->status.p, NC, hipMemcpyDeviceToHost, st));
  HOK(hipMemcpyAsync(hkey.data(), S->hkey.p, HT_SIZE * 8, hipMemcpyDeviceToHost, st));
  HOK(hipMemcpyAsync(&hcount, S->hcount.p, 4, hipMemcpyDeviceToHost, st));
  HOK(hipStreamSynchronize(st));
  if (hcount > HK_MAX)
    return set_error(TSDB_E_NOT_IMPLEMENTED, "more than " + std::to_string(HK_MAX) + " distinct histogram buckets in one store");
  // 2. host: the dictionary in HistogramBucket order (Float.compare of lower, then upper)
  std::vector<int64_t> slots;
  for (int64_t i = 0; i < HT_SIZE; i++)
    if (hkey[i] != HK_EMPTY) slots.push_back(i);
  std::sort(slots.begin(), slots.end(), [&](int64_t a, int64_t b) {
    const uint32_t la = ford((uint32_t)(hkey[a] >> 32)), lb = ford((uint32_t)(hkey[b] >> 32));
    if (la != lb) return la < lb;
    return ford((uint32_t)hkey[a]) < ford((uint32_t)hkey[b]);
  });
  S->D = (int32_t)slots.size();
  std::vector<int32_t> hidx(HT_SIZE, -1);
  S->h_dlo.resize(S->D);
  S->h_dup.resize(S->D);
  for (int32_t d = 0; d < S->D; d++) {
    hidx[slots[d]] = d;
    S->h_dlo[d] = (uint32_t)(hkey[slots[d]] >> 32);
    S->h_dup[d] = (uint32_t)hkey[slots[d]];
  }
  HOK(S->hidx.ensure(HT_SIZE * 4));
  HOK(S->dlo.ensure(S->D * 4 + 4));
  HOK(S->dup.ensure(S->D * 4 + 4));
  HOK(hipMemcpyAsync(S->hidx.p, hidx.data(), HT_SIZE * 4, hipMemcpyHostToDevice, st));
  if (S->D) {
    HOK(hipMemcpyAsync(S->dlo.p, S->h_dlo.data(), S->D * 4, hipMemcpyHostToDevice, st));
    HOK(hipMemcpyAsync(S->dup.p, S->h_dup.data(), S->D * 4, hipMemcpyHostToDevice, st));
  }
  // the dictionary as the LDS hash table of k_hist_accum (same hash, HIST_LDICT slots)
  S->lds_dict = S->D <= HIST_LDICT / 2;
  if (S->lds_dict) {
    std::vector<uint64_t> lk(HIST_LDICT, HK_EMPTY);
    std::vector<int32_t> li(HIST_LDICT, -1);
    for (int32_t d = 0; d < S->D; d++) {
      const uint64_t key = ((uint64_t)S->h_dlo[d] << 32) | S->h_dup[d];
      uint32_t slot = lds_dict_slot(key);
      while (lk[slot] != HK_EMPTY) slot = (slot + 1) & (HIST_LDICT - 1);
      lk[slot] = key;
      li[slot] = d;
    }
    HOK(S->lkey.ensure(HIST_LDICT * 8));
    HOK(S->lidx.ensure(HIST_LDICT * 4));
    HOK(hipMemcpyAsync(S->lkey.p, lk.data(), HIST_LDICT * 8, hipMemcpyHostToDevice, st));
    HOK(hipMemcpyAsync(S->lidx.p, li.data(), HIST_LDICT * 4, hipMemcpyHostToDevice, st));
    // the compact table k_hist_accw keeps in LDS (its window takes the space the rest leaves)
    S->lslots = hist_lds_slots(S->D);
    std::vector<uint64_t> ck(S->lslots, HK_EMPTY);
    std::vector<int32_t> ci(S->lslots, -1);
    for (int32_t d = 0; d < S->D; d++) {
      const uint64_t key = ((uint64_t)S->h_dlo[d] << 32) | S->h_dup[d];
      uint32_t slot = lds_dict_slot(key, (uint32_t)S->lslots - 1);
      while (ck[slot] != HK_EMPTY) slot = (slot + 1) & (uint32_t)(S->lslots - 1);
      ck[slot] = key;
      ci[slot] = d;
    }
    HOK(S->lkey2.ensure(S->lslots * 8));
    HOK(S->lidx2.ensure(S->lslots * 4));
    HOK(hipMemcpyAsync(S->lkey2.p, ck.data(), S->lslots * 8, hipMemcpyHostToDevice, st));
    HOK(hipMemcpyAsync(S->lidx2.p, ci.data(), S->lslots * 4, hipMemcpyHostToDevice, st));
    HOK(hipStreamSynchronize(st));
  }
  // bucket layouts: runs of columns with the same key bytes share one row of dictionary indices
  {
    Buf head, excl;
    struct Rel { Buf* a; Buf* b; ~Rel() { a->release(); b->release(); } } rel{&head, &excl};
    HOK(head.ensure(NC * 4 + 4));
    HOK(excl.ensure(NC * 8 + 16));
    HOK(S->col_lid.ensure(NC * 4 + 4));
    HOK(S->lay_col.ensure(NC * 4 + 4));
    HOK(hist_layout_index(NC, S->voff.as<uint64_t>(), S->val.as<uint8_t>(), S->status.as<uint8_t>(), head.as<uint32_t>(),
                          excl.as<int64_t>(), S->col_lid.as<int32_t>(), S->lay_col.as<int32_t>(), &S->n_layouts, &S->tmp,
                          &S->tmp_bytes, st));
    const int64_t NL = S->n_layouts;
    std::vector<int32_t> lcol(std::max<int64_t>(1, NL)), loff(std::max<int64_t>(1, NL) + 1, 0);
    if (NL) HOK(hipMemcpyAsync(lcol.data(), S->lay_col.p, NL * 4, hipMemcpyDeviceToHost, st));
    HOK(hipStreamSynchronize(st));
    for (int64_t l = 0; l < NL; l++) {
      const uint8_t* v = hb->val + hb->cell_val_off[lcol[l]];
      loff[l + 1] = loff[l] + (int16_t)(((uint32_t)v[1] << 8) | v[2]);
    }
    HOK(S->lay_off.ensure((NL + 1) * 4));
    HOK(S->lay_di.ensure(std::max<int64_t>(1, loff[NL]) * 4));
    HOK(hipMemcpyAsync(S->lay_off.p, loff.data(), (NL + 1) * 4, hipMemcpyHostToDevice, st));
    HOK(hist_layout_di(NL, S->lay_col.as<int32_t>(), S->lay_off.as<int32_t>(), S->voff.as<uint64_t>(), S->val.as<uint8_t>(),
                       S->hkey.as<uint64_t>(), S->hidx.as<int32_t>(), S->lay_di.as<int32_t>(), st));
    HOK(hipStreamSynchronize(st));
  }
  // 3. host: spans (SaltScanner.processRow -> HistogramSpan.addRow, rows sorted by base time)
  std::vector<int64_t> pos_cell, pos_ts, row_pos{0};
  std::vector<uint8_t> pos_kind;
  S->sp_row.assign(1, 0);
  S->row_base.clear();
  S->group.assign(hb->group_id, hb->group_id + NS);
  pos_cell.reserve(NC);
  pos_ts.reserve(NC);
  pos_kind.reserve(NC);
  std::vector<HRow> rows;
  for (int64_t s = 0; s < NS; s++) {
    rows.clear();
    for (int64_t r = hb->series_row_ptr[s]; r < hb->series_row_ptr[s + 1]; r++) {
      HRow row{hb->row_base_time[r], {}};
      for (int64_t cc = hb->row_cell_ptr[r]; cc < hb->row_cell_ptr[r + 1]; cc++) {
        const uint64_t qo = hb->cell_qual_off[cc], ql = hb->cell_qual_off[cc + 1] - qo;
        if (ql < 1 || hb->qual[qo] != 0x06) continue;   // not a histogram column
        int64_t ts;
        if (!nondp_ts(row.base, hb->qual + qo, ql, &ts) || status[cc] == HC_DROP) continue;
        row.dp.emplace_back(ts, cc);
      }
      if (row.dp.empty()) continue;   // processRow adds no histogram row
      // HistogramSpan.addRow (:280-328)
      int64_t last_ts = 0;
      if (!rows.empty()) last_ts = rows.back().dp.back().first;
      bool merged = false;
      if (last_ts >= row.dp[0].first) {
        for (auto& rs : rows)
          if (rs.base == row.base) { row_merge(rs, row); merged = true; break; }
      }
      if (!merged) rows.push_back(std::move(row));
    }
    std::stable_sort(rows.begin(), rows.end(), [](const HRow& a, const HRow& b) { return a.base < b.base; });
    for (const auto& rw : rows) {
      for (const auto& d : rw.dp) {
        pos_ts.push_back(d.first);
        pos_cell.push_back(d.second);
        pos_kind.push_back(status[d.second]);
      }
      row_pos.push_back((int64_t)pos_ts.size());
      S->row_base.push_back(rw.base);
    }
    S->sp_row.push_back((int64_t)S->row_base.size());
  }
  S->n_series = NS;
  S->n_cells = NC;
  S->max_ts = pos_ts.empty() ? 0 : *std::max_element(pos_ts.begin(), pos_ts.end());
  S->n_pos = (int64_t)pos_ts.size();
  HOK(S->pos_cell.ensure(S->n_pos * 8 + 8));
  HOK(S->pos_ts.ensure(S->n_pos * 8 + 8));
  HOK(S->pos_kind.ensure(S->n_pos + 8));
  HOK(S->row_pos.ensure(row_pos.size() * 8));
  if (S->n_pos) {
    HOK(hipMemcpyAsync(S->pos_cell.p, pos_cell.data(), S->n_pos * 8, hipMemcpyHostToDevice, st));
    HOK(hipMemcpyAsync(S->pos_ts.p, pos_ts.data(), S->n_pos * 8, hipMemcpyHostToDevice, st));
    HOK(hipMemcpyAsync(S->pos_kind.p, pos_kind.data(), S->n_pos, hipMemcpyHostToDevice, st));
  }
  HOK(hipMemcpyAsync(S->row_pos.p, row_pos.data(), row_pos.size() * 8, hipMemcpyHostToDevice, st));
  HOK(hipStreamSynchronize(st));
  S->h_pos_ts.swap(pos_ts);
  S->h_row_pos.swap(row_pos);
  S->loaded = true;
  return 0;
}

namespace tsdb {
// start / end: HistogramSpanGroup bounds (ms); rows with base time in [row_lo, row_hi) are scanned
int hist_run(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t start, int64_t end, int64_t ss, int64_t se, int n_pct,
             const float* pct, int show_buckets, tsdbhip_hist_result** out) {
  if (!c || !q || !out || n_pct < 0 || (n_pct && !pct)) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  *out = nullptr;
  if (ctx_md(c)) return md_hist_run(c, q, start, end, ss, se, n_pct, pct, show_buckets, out);
  std::lock_guard<std::mutex> lk(ctx_mutex(c));
  HOK(hipSetDevice(ctx_device(c)));
  hipStream_t st = ctx_stream(c);
  HistStore* S = store_of(c);
  if (!S->loaded) return set_error(TSDB_E_ILLEGAL_STATE, "no histogram store loaded (tsdbhip_load_histograms)");
  int ds;
  if (q->ds_function < 0) ds = 0;
  else if (q->ds_all) ds = 2;
  else if (q->ds_calendar) ds = 3;
  else ds = 1;
  if (ds == 1 && q->ds_interval_ms <= 0) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "downsampling interval must be positive");
  // the spans the scan returns (rows with base in [ss, se)) and the groups they form
  const int64_t NS = S->n_series;
  ss = std::max<int64_t>(0, std::min<int64_t>(ss, (int64_t)UINT32_MAX + 1));
  se = std::max<int64_t>(0, std::min<int64_t>(se, (int64_t)UINT32_MAX + 1));
  std::vector<int64_t> rlo, rhi;
  std::vector<int32_t> sout, gid_of_out;
  const bool none = q->aggregator == TSDB_AGG_NONE;
  std::vector<int32_t> gmap;
  if (!none) {
    int32_t gmax = -1;
    for (int64_t s = 0; s < NS; s++) gmax = std::max(gmax, S->group[s]);
    gmap.assign((size_t)gmax + 1, -1);
  }
  std::vector<uint8_t> present(NS, 0);
  std::vector<int64_t> lo(NS), hi(NS);
  for (int64_t s = 0; s < NS; s++) {
    const auto b0 = S->row_base.begin() + S->sp_row[s], b1 = S->row_base.begin() + S->sp_row[s + 1];
    lo[s] = ss > (int64_t)UINT32_MAX ? S->sp_row[s + 1] : std::lower_bound(b0, b1, (uint32_t)ss) - S->row_base.begin();
    hi[s] = se > (int64_t)UINT32_MAX ? S->sp_row[s + 1] : std::lower_bound(b0, b1, (uint32_t)se) - S->row_base.begin();
    present[s] = lo[s] < hi[s];
    if (present[s] && !none && S->group[s] >= 0) gmap[S->group[s]] = 0;
  }
  if (!none) {
    int32_t e = 0;
    for (size_t g = 0; g < gmap.size(); g++)
      if (gmap[g] == 0) { gmap[g] = e++; gid_of_out.push_back((int32_t)g); }
  }
  for (int64_t s = 0; s < NS; s++) {
    if (!present[s]) continue;
    int32_t o;
    if (none) { o = (int32_t)gid_of_out.size(); gid_of_out.push_back((int32_t)s); }
    else if (S->group[s] < 0) continue;   // no matching group-by tag: dropped (TsdbQuery.java:1195-1200)
    else o = gmap[S->group[s]];
    rlo.push_back(lo[s]);
    rhi.push_back(hi[s]);
    sout.push_back(o);
  }
  if (!none && !sout.empty()) {   // spans by output group (stable): a group's datapoints become contiguous
    std::vector<int64_t> first(gid_of_out.size() + 1, 0);
    for (int32_t o : sout) first[o + 1]++;
    for (size_t g = 0; g < gid_of_out.size(); g++) first[g + 1] += first[g];
    std::vector<int64_t> r2(rlo.size()), h2(rhi.size());
    std::vector<int32_t> o2(sout.size());
    for (size_t i = 0; i < sout.size(); i++) {
      const int64_t k = first[sout[i]]++;
      r2[k] = rlo[i];
      h2[k] = rhi[i];
      o2[k] = sout[i];
    }
    rlo.swap(r2);
    rhi.swap(h2);
    sout.swap(o2);
  }
  const int64_t G = (int64_t)gid_of_out.size(), nsp = (int64_t)rlo.size();
  if (G >= ((int64_t)1 << 21)) return set_error(TSDB_E_NOT_IMPLEMENTED, "more than 2^21 histogram groups in one query");
  const int64_t NP = S->n_pos;
  HistQueryParams p{};
  p.voff = S->voff.as<uint64_t>();
  p.val = S->val.as<uint8_t>();
  p.pos_cell = S->pos_cell.as<int64_t>();
  p.pos_ts = S->pos_ts.as<int64_t>();
  p.pos_kind = S->pos_kind.as<uint8_t>();
  p.row_pos = S->row_pos.as<int64_t>();
  p.hkey = S->hkey.as<uint64_t>();
  p.hidx = S->hidx.as<int32_t>();
  if (!opt_off(OPT_HIST_LAYOUT) && S->n_layouts > 0) {
    p.col_lid = S->col_lid.as<int32_t>();   // (option HIST_LAYOUT = 0: every bucket through the keyed lookup)
    p.lay_off = S->lay_off.as<int32_t>();
    p.lay_di = S->lay_di.as<int32_t>();
  }
  p.dict_lo = S->dlo.as<uint32_t>();
  p.dict_up = S->dup.as<uint32_t>();
  p.D = S->D;
  p.C = S->D + 3;
  p.n_spans = nsp;
  p.start = start;
  p.end = end;
  p.qs = q->start_time;   // TsdbQuery.getStartTime(): as set (HistogramDownsampler "all" bounds)
  p.qe = q->end_time;
  p.ds = ds;
  p.ds_sum = q->ds_function == TSDB_AGG_SUM;
  p.I = ds == 1 ? q->ds_interval_ms : 0;
  if (ds == 1) {
    p.B0 = start >= 0 ? ((start + p.I - 1) / p.I) * p.I : start - start % p.I;
    // outputs lie in [B0, min(end, the interval of the store's last datapoint)]
    const int64_t top = std::min(end, S->max_ts - S->max_ts % p.I);
    p.K = top >= p.B0 ? (top - p.B0) / p.I + 1 : 0;
  } else if (ds == 2) {
    p.B0 = q->end_time;   // the clone's timestamp: HistogramDownsampler.timestamp field = the query end (:179-183, 334-345)
    p.K = 1;
  }
  if (ds == 3) {
    // HistogramDownsampler with a calendar interval: seekInterval's target (previousInterval of
    // the span group start, stepped once when the start is past it), then per span the intervals
    // from previousInterval(its first datapoint after the seek) -- one boundary run per distinct
    // anchor, reaching past the span's last datapoint
    const int unit = q->ds_calendar;
    const int64_t um = cal_unit_ms(unit);
    const int64_t n = um > 0 ? q->ds_interval_ms / um : 0;
    if (n < 1) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "Interval must be greater than zero");
    if (start < 0) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "Timestamp cannot be less than zero");
    const tsdbhip_tz* z = q->ds_tz;
    int64_t c = 0;
    cal_prev_tz(z, start, n, unit, &c);
    if (start > c) c = cal_step_tz(z, c, unit, n);
    p.cal_seek = c;
    const std::vector<int64_t>& rp = S->h_row_pos;
    const std::vector<int64_t>& pt = S->h_pos_ts;
    auto seek = [&](int64_t rl, int64_t rh, int64_t target) {   // k_hist.hip span_seek
      int64_t ri = rl;
      for (int64_t r = rl; r < rh; r++) {
        if (rp[r + 1] - rp[r] < 1 || pt[rp[r + 1] - 1] < target) ri++;
        else break;
      }
      if (ri == rh) --ri;
      int64_t qq = rp[ri];
      while (qq < rp[ri + 1] && pt[qq] < target) ++qq;
      return qq;
    };
    std::vector<int64_t> anchor(nsp, INT64_MIN);
    std::vector<std::pair<int64_t, int64_t>> need;   // (anchor, latest datapoint its run must pass)
    for (int64_t i = 0; i < nsp; i++) {
      const int64_t q0 = seek(rlo[i], rhi[i], c), p1 = rp[rhi[i]];
      if (q0 >= p1) continue;
      if (pt[q0] < 0) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "Timestamp cannot be less than zero");
      cal_prev_tz(z, pt[q0], n, unit, &anchor[i]);
      int64_t mx = pt[q0];
      for (int64_t k = q0; k < p1; k++) mx = std::max(mx, pt[k]);
      need.emplace_back(anchor[i], mx);
    }
    std::sort(need.begin(), need.end());
    std::vector<int64_t> tab, run_a, run_off, run_n;
    for (size_t k = 0; k < need.size();) {
      size_t k1 = k;
      int64_t reach = need[k].second;
      while (k1 < need.size() && need[k1].first == need[k].first) reach = std::max(reach, need[k1++].second);
      run_a.push_back(need[k].first);
      run_off.push_back((int64_t)tab.size());
      int64_t b = need[k].first;
      tab.push_back(b);
      while (b <= reach) {
        b = cal_step_tz(z, b, unit, n);
        tab.push_back(b);
        if (tab.size() > ((size_t)1 << 27))
          return set_error(TSDB_E_NOT_IMPLEMENTED, "more than 2^27 calendar intervals in one histogram query");
      }
      run_n.push_back((int64_t)tab.size() - run_off.back());
      k = k1;
    }
    std::vector<int64_t> spc(2 * std::max<int64_t>(1, nsp), 0);
    for (int64_t i = 0; i < nsp; i++) {
      if (anchor[i] == INT64_MIN) continue;
      const size_t r = std::lower_bound(run_a.begin(), run_a.end(), anchor[i]) - run_a.begin();
      spc[2 * i] = run_off[r];
      spc[2 * i + 1] = run_n[r];
    }
    if (tab.empty()) tab.push_back(0);
    HOK(S->q_caltab.ensure(tab.size() * 8));
    HOK(S->q_spcal.ensure(spc.size() * 8));
    HOK(hipMemcpyAsync(S->q_caltab.p, tab.data(), tab.size() * 8, hipMemcpyHostToDevice, st));
    HOK(hipMemcpyAsync(S->q_spcal.p, spc.data(), spc.size() * 8, hipMemcpyHostToDevice, st));
    HOK(hipStreamSynchronize(st));   // (tab / spc leave scope)
    p.cal_tab = S->q_caltab.as<int64_t>();
    p.sp_cal = S->q_spcal.as<int64_t>();
  }
  const bool sparse = ds == 0 || ds == 3;
  HOK(S->q_rlo.ensure(nsp * 8 + 8));
  HOK(S->q_rhi.ensure(nsp * 8 + 8));
  HOK(S->q_out.ensure(nsp * 4 + 4));
  HOK(S->err.ensure(16));
  if (nsp) {
    HOK(hipMemcpyAsync(S->q_rlo.p, rlo.data(), nsp * 8, hipMemcpyHostToDevice, st));
    HOK(hipMemcpyAsync(S->q_rhi.p, rhi.data(), nsp * 8, hipMemcpyHostToDevice, st));
    HOK(hipMemcpyAsync(S->q_out.p, sout.data(), nsp * 4, hipMemcpyHostToDevice, st));
  }
  HOK(hipMemsetAsync(S->err.p, 0, 16, st));
  p.sp_rlo = S->q_rlo.as<int64_t>();
  p.sp_rhi = S->q_rhi.as<int64_t>();
  p.sp_out = S->q_out.as<int32_t>();
  p.err = S->err.as<int32_t>();
  if (sparse) {
    if (NP >= ((int64_t)1 << 31)) return set_error(TSDB_E_NOT_IMPLEMENTED, "more than 2^31 histogram datapoints without downsampling");
    HOK(S->q_key.ensure(NP * 8 + 8));
    HOK(hipMemsetAsync(S->q_key.p, 0xFF, NP * 8 + 8, st));
    p.pos_key = S->q_key.as<int64_t>();
  } else {
    HOK(S->q_slot.ensure(NP * 4 + 4));
    HOK(hipMemsetAsync(S->q_slot.p, 0xFF, NP * 4 + 4, st));
    p.pos_slot = S->q_slot.as<int32_t>();
  }
  HOK(hist_slots(p, st));
  int32_t err[2] = {0, 0};
  HOK(hipMemcpyAsync(err, S->err.p, 8, hipMemcpyDeviceToHost, st));
  HOK(hipStreamSynchronize(st));
  if (ds == 0 && err[0] == TSDB_E_NOT_IMPLEMENTED && err[1] == 3 /* WHY_UNSORTED */) {
    // a span out of time order: the aggregation iterator's greedy walk labels the points instead
    // of the union of timestamps (k_hist_walk); spans of a group are consecutive in sp_*
    std::vector<int64_t> gsp(G + 1, 0);
    for (int32_t o : sout) gsp[o + 1]++;
    for (int64_t g = 0; g < G; g++) gsp[g + 1] += gsp[g];
    HOK(S->q_gsp.ensure((G + 1) * 8));
    HOK(S->q_spq.ensure(nsp * 8 + 8));
    HOK(S->q_spts.ensure(nsp * 8 + 8));
    HOK(hipMemcpyAsync(S->q_gsp.p, gsp.data(), (G + 1) * 8, hipMemcpyHostToDevice, st));
    HOK(hipMemsetAsync(S->q_key.p, 0xFF, NP * 8 + 8, st));
    HOK(hipMemsetAsync(S->err.p, 0, 16, st));
    int64_t max_spans = 0;
    for (int64_t g = 0; g < G; g++) max_spans = std::max(max_spans, gsp[g + 1] - gsp[g]);
    HOK(hist_walk(p, S->q_gsp.as<int64_t>(), G, max_spans, S->q_spq.as<int64_t>(), S->q_spts.as<int64_t>(), st));
    HOK(hipMemcpyAsync(err, S->err.p, 8, hipMemcpyDeviceToHost, st));
    HOK(hipStreamSynchronize(st));   // (gsp leaves scope)
    p.greedy = 1;
  }
  static const char* const WHY[] = {"", "invalid seek timestamp",
                                    "a histogram downsampling function other than sum aggregates two datapoints "
                                    "(HistogramAggregation null)",
                                    "histogram datapoints of a span out of time order", "internal: slot out of range",
                                    "histograms of two codecs aggregated", "internal: bucket missing from the dictionary"};
  auto why = [&](int w) { return std::string(w >= 0 && w <= 6 ? WHY[w] : "?"); };
  if (err[0]) return set_error(err[0], why(err[1]));
  int64_t n_points;
  if (sparse) {
    HOK(S->q_key2.ensure(NP * 8 + 8));
    HOK(S->q_pos.ensure(NP * 4 + 4));
    HOK(S->q_pos2.ensure(NP * 4 + 4));
    HOK(S->q_head.ensure(NP * 4 + 4));
    HOK(S->q_incl.ensure(NP * 8 + 16));
    HOK(S->q_point.ensure(NP * 4 + 4));
    HOK(S->q_ptts.ensure(NP * 8 + 8));
    HOK(S->q_ptgrp.ensure(NP * 4 + 4));
    HOK(hipMemsetAsync(S->q_point.p, 0xFF, NP * 4 + 4, st));
    p.pos_point = S->q_point.as<int32_t>();
    n_points = 0;
    if (NP)
      HOK(hist_sparse(p, NP, S->q_key2.as<uint64_t>(), S->q_pos.as<uint32_t>(), S->q_pos2.as<uint32_t>(),
                      S->q_head.as<uint32_t>(), S->q_incl.as<int64_t>(), S->q_ptts.as<int64_t>(), S->q_ptgrp.as<int32_t>(),
                      &n_points, &S->tmp, &S->tmp_bytes, st));
    p.pt_ts = S->q_ptts.as<int64_t>();
    p.pt_group = S->q_ptgrp.as<int32_t>();
  } else {
    n_points = G * p.K;
  }
  const double state = (double)n_points * (double)p.C * 8.0;
  if (state > 32e9) return set_error(TSDB_E_NOT_IMPLEMENTED, "more than 32 GB of histogram point state in one query");
  p.n_points = n_points;
  p.W = (S->D + 31) / 32;
  HOK(S->acc.ensure(n_points * p.C * 8 + 8));
  HOK(S->pkind.ensure(n_points * 4 + 4));
  HOK(hipMemsetAsync(S->acc.p, 0, n_points * p.C * 8 + 8, st));
  HOK(hipMemsetAsync(S->pkind.p, 0, n_points * 4 + 4, st));
  p.acc = S->acc.as<uint64_t>();
  p.pkind = S->pkind.as<uint32_t>();
  if (show_buckets && p.W) {
    HOK(S->pres.ensure(n_points * p.W * 4 + 4));
    HOK(hipMemsetAsync(S->pres.p, 0, n_points * p.W * 4 + 4, st));
    p.pres = S->pres.as<uint32_t>();
  }
#ifdef TSDBHIP_KDBG
  if (opt(OPT_DBG) > 0) p.dbg = (int32_t)opt(OPT_DBG);   // profiling build only (results invalid)
#endif
  // option HIST_WINDOW = 0 (tests): the per-column atomic kernel
  if (S->lds_dict && hist_window_points(p, S->lslots) > 0 && !opt_off(OPT_HIST_WINDOW)) {
    HOK(S->q_vlen.ensure(nsp * 4 + 4));
    HOK(S->q_voff.ensure(nsp * 8 + 16));
    HOK(S->q_vpos.ensure(NP * 4 + 4));
    int64_t nvp = 0;
    HOK(hist_vpos(S->q_rlo.as<int64_t>(), S->q_rhi.as<int64_t>(), S->row_pos.as<int64_t>(), nsp, S->q_vlen.as<uint32_t>(),
                  S->q_voff.as<int64_t>(), S->q_vpos.as<int32_t>(), &nvp, &S->tmp, &S->tmp_bytes, st));
    HOK(S->q_tix.ensure(nvp * 24 + 24));
    HOK(hist_accum_window(p, S->q_vpos.as<int32_t>(), nvp, S->lkey2.as<uint64_t>(), S->lidx2.as<int32_t>(), S->lslots,
                          S->q_tix.p, st));
  } else {
    HOK(hist_accum(p, NP, S->lds_dict ? S->lkey.as<uint64_t>() : nullptr, S->lds_dict ? S->lidx.as<int32_t>() : nullptr, st));
  }
  HOK(S->flag.ensure(n_points * 4 + 4));
  HOK(S->ptout.ensure(n_points * 8 + 16));
  HOK(hist_flags(p, S->flag.as<uint32_t>(), st));
  HOK(hist_scan(S->flag.as<uint32_t>(), S->ptout.as<int64_t>(), n_points, &S->tmp, &S->tmp_bytes, st));
  int64_t n_out = 0;
  HOK(hipMemcpyAsync(&n_out, S->ptout.as<int64_t>() + n_points, 8, hipMemcpyDeviceToHost, st));
  HOK(hipMemcpyAsync(err, S->err.p, 8, hipMemcpyDeviceToHost, st));
  HOK(hipStreamSynchronize(st));
  if (err[0]) return set_error(err[0], why(err[1]));
  p.pt_out = S->ptout.as<int64_t>();
  p.n_pct = n_pct;
  HOK(S->pct.ensure(n_pct * 4 + 4));
  if (n_pct) HOK(hipMemcpyAsync(S->pct.p, pct, n_pct * 4, hipMemcpyHostToDevice, st));
  p.pct = S->pct.as<float>();
  HOK(S->o_ts.ensure(n_out * 8 + 8));
  HOK(S->o_grp.ensure(n_out * 4 + 4));
  HOK(S->o_kind.ensure(n_out + 8));
  HOK(S->o_pct.ensure(n_out * n_pct * 8 + 8));
  p.out_ts = S->o_ts.as<int64_t>();
  p.out_group = S->o_grp.as<int32_t>();
  p.out_kind = S->o_kind.as<uint8_t>();
  p.out_pct = S->o_pct.as<double>();
  if (show_buckets) {
    HOK(S->o_cnt.ensure(n_out * (S->D + 2) * 8 + 8));
    HOK(S->o_pres.ensure(n_out * S->D + 8));
    p.out_count = S->o_cnt.as<int64_t>();
    p.out_present = S->o_pres.as<uint8_t>();
  }
  HOK(hist_final(p, st));
  auto* R = new HistResultOwner();
  R->ts.resize(n_out);
  std::vector<int32_t> ogrp(n_out);
  R->kind.resize(n_out);
  R->pct.resize((size_t)n_out * n_pct);
  if (n_out) {
    HOK(hipMemcpyAsync(R->ts.data(), S->o_ts.p, n_out * 8, hipMemcpyDeviceToHost, st));
    HOK(hipMemcpyAsync(ogrp.data(), S->o_grp.p, n_out * 4, hipMemcpyDeviceToHost, st));
    HOK(hipMemcpyAsync(R->kind.data(), S->o_kind.p, n_out, hipMemcpyDeviceToHost, st));
    if (n_pct) HOK(hipMemcpyAsync(R->pct.data(), S->o_pct.p, n_out * n_pct * 8, hipMemcpyDeviceToHost, st));
    if (show_buckets) {
      R->cnt.resize((size_t)n_out * (S->D + 2));
      R->pres.resize((size_t)n_out * S->D);
      HOK(hipMemcpyAsync(R->cnt.data(), S->o_cnt.p, n_out * (S->D + 2) * 8, hipMemcpyDeviceToHost, st));
      if (S->D) HOK(hipMemcpyAsync(R->pres.data(), S->o_pres.p, n_out * S->D, hipMemcpyDeviceToHost, st));
    }
  }
  const hipError_t se2 = hipStreamSynchronize(st);
  if (se2 != hipSuccess) { delete R; return set_error(TSDB_E_HIP, std::string("hist_run: ") + hipGetErrorString(se2)); }
  // every emitted group, with its (possibly empty) point range
  R->gid = gid_of_out;
  R->gptr.assign(G + 1, 0);
  for (int64_t o = 0; o < n_out; o++) R->gptr[ogrp[o] + 1]++;
  for (int64_t g = 0; g < G; g++) R->gptr[g + 1] += R->gptr[g];
  R->blo = S->h_dlo;
  R->bup = S->h_dup;
  tsdbhip_hist_result& r = R->r;
  r.n_groups = G;
  r.group_id = R->gid.data();
  r.group_ptr = R->gptr.data();
  r.ts_ms = R->ts.data();
  r.n_pct = n_pct;
  r.pct = R->pct.data();
  r.show_buckets = show_buckets ? 1 : 0;
  r.n_buckets = S->D;
  r.bucket_lower = R->blo.data();
  r.bucket_upper = R->bup.data();
  r.count = show_buckets ? R->cnt.data() : nullptr;
  r.present = show_buckets ? R->pres.data() : nullptr;
  r.codec = R->kind.data();
  *out = &R->r;
  return 0;
}

// The devices' results of one histogram query (multi-device context, whole groups per device) as
// the result of the whole store: the groups in group-id order ("none": the spans in batch order,
// span_of[d] maps device d's span index to the batch's), the bucket dictionary the union of the
// devices' (HistogramBucket order), each point's counts / presence moved to its buckets' places in
// it (a bucket of another device's store is absent from the point: count 0, not present).
int hist_merge(const std::vector<tsdbhip_hist_result*>& parts, const std::vector<const std::vector<int64_t>*>& span_of,
               bool none, tsdbhip_hist_result** out) {
  *out = nullptr;
  const size_t np = parts.size();
  if (!np) return set_error(TSDB_E_ILLEGAL_STATE, "no histogram store loaded (tsdbhip_load_histograms)");
  const int n_pct = parts[0]->n_pct, sb = parts[0]->show_buckets;
  auto ord = [](uint32_t lo, uint32_t up) { return ((uint64_t)ford(lo) << 32) | ford(up); };
  std::vector<uint64_t> keys;
  for (const tsdbhip_hist_result* r : parts)
    for (int32_t b = 0; b < r->n_buckets; b++) keys.push_back(ord(r->bucket_lower[b], r->bucket_upper[b]));
  std::sort(keys.begin(), keys.end());
  keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
  const int64_t D = (int64_t)keys.size();
  std::vector<std::vector<int32_t>> bmap(np);
  for (size_t i = 0; i < np; i++) {
    const tsdbhip_hist_result* r = parts[i];
    bmap[i].resize(r->n_buckets);
    for (int32_t b = 0; b < r->n_buckets; b++)
      bmap[i][b] = (int32_t)(std::lower_bound(keys.begin(), keys.end(), ord(r->bucket_lower[b], r->bucket_upper[b])) - keys.begin());
  }
  struct Ent { int64_t key; int32_t part; int64_t g; };
  std::vector<Ent> ents;
  for (size_t i = 0; i < np; i++)
    for (int64_t g = 0; g < parts[i]->n_groups; g++) {
      const int32_t id = parts[i]->group_id[g];
      ents.push_back({none ? (*span_of[i])[id] : (int64_t)id, (int32_t)i, g});
    }
  std::sort(ents.begin(), ents.end(), [](const Ent& a, const Ent& b) { return a.key < b.key; });
  auto* R = new HistResultOwner();
  const int64_t G = (int64_t)ents.size();
  R->gid.resize(G);
  R->gptr.assign(G + 1, 0);
  for (int64_t e = 0; e < G; e++) {
    const tsdbhip_hist_result* r = parts[ents[e].part];
    R->gid[e] = (int32_t)ents[e].key;
    R->gptr[e + 1] = R->gptr[e] + (r->group_ptr[ents[e].g + 1] - r->group_ptr[ents[e].g]);
  }
  const int64_t n_out = R->gptr[G];
  R->ts.resize(n_out);
  R->kind.resize(n_out);
  R->pct.resize((size_t)n_out * n_pct);
  if (sb) {
    R->cnt.assign((size_t)n_out * (D + 2), 0);
    R->pres.assign((size_t)n_out * D, 0);
  }
  for (int64_t e = 0; e < G; e++) {
    const tsdbhip_hist_result* r = parts[ents[e].part];
    const std::vector<int32_t>& bm = bmap[ents[e].part];
    const int64_t Dl = r->n_buckets;
    for (int64_t i = r->group_ptr[ents[e].g], o = R->gptr[e]; i < r->group_ptr[ents[e].g + 1]; i++, o++) {
      R->ts[o] = r->ts_ms[i];
      R->kind[o] = r->codec[i];
      for (int j = 0; j < n_pct; j++) R->pct[(size_t)o * n_pct + j] = r->pct[(size_t)i * n_pct + j];
      if (!sb) continue;
      for (int64_t b = 0; b < Dl; b++) {
        R->cnt[(size_t)o * (D + 2) + bm[b]] = r->count[(size_t)i * (Dl + 2) + b];
        R->pres[(size_t)o * D + bm[b]] = r->present[(size_t)i * Dl + b];
      }
      R->cnt[(size_t)o * (D + 2) + D] = r->count[(size_t)i * (Dl + 2) + Dl];           // underflow
      R->cnt[(size_t)o * (D + 2) + D + 1] = r->count[(size_t)i * (Dl + 2) + Dl + 1];   // overflow
    }
  }
  R->blo.resize(D);
  R->bup.resize(D);
  auto unord = [](uint32_t k) { return (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k; };   // inverse of ford
  for (int64_t b = 0; b < D; b++) {
    R->blo[b] = unord((uint32_t)(keys[b] >> 32));
    R->bup[b] = unord((uint32_t)keys[b]);
  }
  tsdbhip_hist_result& r = R->r;
  r.n_groups = G;
  r.group_id = R->gid.data();
  r.group_ptr = R->gptr.data();
  r.ts_ms = R->ts.data();
  r.n_pct = n_pct;
  r.pct = R->pct.data();
  r.show_buckets = sb;
  r.n_buckets = (int32_t)D;
  r.bucket_lower = R->blo.data();
  r.bucket_upper = R->bup.data();
  r.count = sb ? R->cnt.data() : nullptr;
  r.present = sb ? R->pres.data() : nullptr;
  r.codec = R->kind.data();
  *out = &R->r;
  return 0;
}
}  // namespace tsdb

extern "C" int tsdbhip_hist_run(tsdbhip_ctx* c, const tsdbhip_query* q, int n_pct, const float* pct, int show_buckets,
                                tsdbhip_hist_result** out) {
  int64_t ss, se;
  const int rc = q ? tsdbhip_scan_bounds(q, &ss, &se) : TSDB_E_ILLEGAL_ARGUMENT;
  if (rc) return rc == TSDB_E_ILLEGAL_ARGUMENT && !q ? set_error(rc, "null query") : rc;
  // HistogramSpanGroup start / end: the scan bounds in ms (TsdbQuery.java:1128-1138,
  // HistogramSpanGroup.java:119-122); the scan returns rows with base time in [ss, se)
  return hist_run(c, q, ss * 1000, se * 1000, ss, se, n_pct, pct, show_buckets, out);
}

extern "C" int tsdbhip_hist_run_range(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t start_ms, int64_t end_ms,
                                      int n_pct, const float* pct, int show_buckets, tsdbhip_hist_result** out) {
  return hist_run(c, q, start_ms, end_ms, 0, (int64_t)UINT32_MAX + 1, n_pct, pct, show_buckets, out);
}

extern "C" void tsdbhip_hist_result_free(tsdbhip_hist_result* r) {
  if (r) delete reinterpret_cast<HistResultOwner*>(r);
}
