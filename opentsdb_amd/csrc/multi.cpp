// One process, several GPUs behind one tsdbhip_ctx (include/tsdbhip.h, "multi-device context";
// SURVEY.md 8e).  The reference runs a query's whole scan in one TSD: TsdbQuery.run
// (src/core/TsdbQuery.java:800-870) feeds every span of a SpanGroup to one AggregationIterator
// (GroupByAndAggregateCB :927-1048).  A TSD JVM that owns all the GPUs of a node therefore wants
// ONE engine handle that spreads the spans of the query over them, not one process per GPU.
//
// A multi-device context holds one ordinary engine context (stream, scratch, resident shard)
// per device and a merge context on devices[0].  Loads split the batch by bytes:
//   GROUPS  whole SpanGroups per device -- every query runs locally, results concatenate;
//   SERIES  positions of the SpanGroup order -- the devices' partial states (or, for percentile /
//           median group-by and TSDB_QF_ORDERED, their span contributions) are gathered to
//           devices[0] over RCCL (send / recv, one rank per GPU, ncclCommInitAll) and merged in
//           device order, which continues SpanGroup order across devices.
// Every device runs on its own host thread; the gather is the only device-to-device traffic.
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <functional>
#include <mutex>
#include <numeric>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "multi.h"

namespace tsdb {
std::mutex& ctx_mutex(tsdbhip_ctx* c);
hipStream_t ctx_stream(tsdbhip_ctx* c);

namespace {

#define MOK(expr)                                                                            \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) return set_error(TSDB_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

// ---- RCCL, resolved at run time -----------------------------------------------------------
// librccl.so.1 is the copy already in the process when there is one (PyTorch's, same soname),
// else the system's: the library itself loads without RCCL, and a context whose devices repeat
// (several shards on one GPU) never needs it.
struct Rccl {
  bool ok = false;
  std::string why;
  decltype(&ncclCommInitAll) init_all = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGetErrorString) err_str = nullptr;
};

Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char* e = dlerror();
      r.why = e ? e : "dlopen failed";
      return;
    }
    r.init_all = reinterpret_cast<decltype(r.init_all)>(dlsym(h, "ncclCommInitAll"));
    r.destroy = reinterpret_cast<decltype(r.destroy)>(dlsym(h, "ncclCommDestroy"));
    r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
    r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
    r.send = reinterpret_cast<decltype(r.send)>(dlsym(h, "ncclSend"));
    r.recv = reinterpret_cast<decltype(r.recv)>(dlsym(h, "ncclRecv"));
    r.err_str = reinterpret_cast<decltype(r.err_str)>(dlsym(h, "ncclGetErrorString"));
    r.ok = r.init_all && r.destroy && r.group_start && r.group_end && r.send && r.recv && r.err_str;
    if (!r.ok) r.why = "librccl.so.1 lacks the send / recv API";
  });
  return r;
}

int rccl_fail(ncclResult_t e, const char* what) {
  return set_error(TSDB_E_HIP, std::string("RCCL ") + what + ": " + rccl().err_str(e));
}

// device buffer on one device of the context
struct Buf {
  int dev = 0;
  void* p = nullptr;
  size_t n = 0;
  int ensure(size_t bytes) {
    bytes = std::max<size_t>(bytes, 16);
    if (n >= bytes) return 0;
    release();
    MOK(hipSetDevice(dev));
    MOK(hipMalloc(&p, bytes));
    n = bytes;
    return 0;
  }
  void release() {
    if (p) {
      (void)hipSetDevice(dev);
      (void)hipFree(p);
    }
    p = nullptr;
    n = 0;
  }
};

struct MultiDev {
  std::vector<int> devices;
  std::vector<tsdbhip_ctx*> subs;       // one engine context per device (slot d = RCCL rank d)
  tsdbhip_ctx* root = nullptr;          // merge context on devices[0]
  int transport = TSDB_MD_COPY;
  std::vector<ncclComm_t> comms;
  int mode_req = TSDB_SHARD_AUTO;       // shard mode of the next load
  int mode = TSDB_SHARD_AUTO;           // shard mode of the resident batch (AUTO: nothing loaded)
  int64_t G = 0;                        // groups of the whole batch
  std::vector<char> live;               // the device holds series
  std::vector<std::vector<int64_t>> series;   // load: batch index of each resident virtual position
  std::vector<int64_t> pos0;            // synth: first batch position of each shard
  std::vector<Buf> xb;                  // per device: exchange source
  Buf gb, ov, of;                       // devices[0]: gathered exchange, merged values / flags
  tsdbhip_timing timing{};
};

MultiDev* md_of(tsdbhip_ctx* c) { return static_cast<MultiDev*>(ctx_md(c)); }

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// fn(d) for every live device (all devices when `all`), each on its own host thread; the error
// of the first failing device in device order is the call's.
int each_device(MultiDev* m, const std::function<int(int)>& fn, bool all = false) {
  const int n = (int)m->devices.size();
  std::vector<int> run;
  for (int d = 0; d < n; d++) if (all || m->live[d]) run.push_back(d);
  if (run.size() == 1) return fn(run[0]);
  std::vector<int> rc(n, 0);
  std::vector<std::string> msg(n);
  std::vector<std::thread> th;
  for (int d : run)
    th.emplace_back([&, d] {
      rc[d] = fn(d);
      if (rc[d]) msg[d] = tsdbhip_last_error();
    });
  for (auto& t : th) t.join();
  for (int d : run) if (rc[d]) return set_error(rc[d], msg[d]);
  return 0;
}

std::vector<int> live_devices(const MultiDev* m) {
  std::vector<int> v;
  for (int d = 0; d < (int)m->devices.size(); d++) if (m->live[d]) v.push_back(d);
  return v;
}

// Contiguous byte-balanced split of weights over n parts (tsdbhip_shard_bounds' rule).
std::vector<int64_t> split(const std::vector<double>& w, int n) {
  const int64_t N = (int64_t)w.size();
  std::vector<double> cum(N + 1, 0.0);
  for (int64_t i = 0; i < N; i++) cum[i + 1] = cum[i] + w[i];
  std::vector<int64_t> b(n + 1, 0);
  for (int r = 1; r < n; r++) {
    const int64_t x = cum[N] > 0 ? std::lower_bound(cum.begin(), cum.end(), cum[N] * r / n) - cum.begin() : N * r / n;
    b[r] = std::max(x, b[r - 1]);
  }
  b[n] = N;
  return b;
}

// The group-aligned split is used when its largest shard is within 10% of the byte balance.
bool groups_balanced(const std::vector<double>& gw, const std::vector<int64_t>& gb, int n) {
  double total = 0, worst = 0;
  for (double x : gw) total += x;
  for (int d = 0; d < n; d++) {
    double s = 0;
    for (int64_t g = gb[d]; g < gb[d + 1]; g++) s += gw[g];
    worst = std::max(worst, s);
  }
  return (int64_t)gw.size() >= n && worst <= 1.10 * total / n;
}

// Copies bytes[i] from src[i] (on devices[ds[i]]) to dst on devices[0], concatenated in the
// order of ds: RCCL send / recv to rank 0, or peer copies on the merge stream.
int gather(MultiDev* m, const std::vector<int>& ds, const std::vector<const void*>& src,
           const std::vector<size_t>& bytes, void* dst) {
  hipStream_t rs = ctx_stream(m->root);
  std::vector<size_t> off(ds.size() + 1, 0);
  for (size_t i = 0; i < ds.size(); i++) off[i + 1] = off[i] + bytes[i];
  if (m->transport == TSDB_MD_RCCL) {
    Rccl& R = rccl();
    ncclResult_t e = R.group_start();
    if (e != ncclSuccess) return rccl_fail(e, "ncclGroupStart");
    for (size_t i = 0; i < ds.size(); i++) {
      if (!bytes[i]) continue;
      const int d = ds[i];
      e = R.send(src[i], bytes[i], ncclUint8, 0, m->comms[d], d == 0 ? rs : ctx_stream(m->subs[d]));
      if (e == ncclSuccess) e = R.recv(static_cast<char*>(dst) + off[i], bytes[i], ncclUint8, d, m->comms[0], rs);
      if (e != ncclSuccess) {
        (void)R.group_end();
        return rccl_fail(e, "ncclSend / ncclRecv");
      }
    }
    e = R.group_end();
    if (e != ncclSuccess) return rccl_fail(e, "ncclGroupEnd");
    for (size_t i = 0; i < ds.size(); i++) {
      if (!bytes[i] || ds[i] == 0) continue;
      MOK(hipSetDevice(m->devices[ds[i]]));
      MOK(hipStreamSynchronize(ctx_stream(m->subs[ds[i]])));
    }
  } else {
    MOK(hipSetDevice(m->devices[0]));
    for (size_t i = 0; i < ds.size(); i++)
      if (bytes[i])
        MOK(hipMemcpyPeerAsync(static_cast<char*>(dst) + off[i], m->devices[0], src[i], m->devices[ds[i]], bytes[i], rs));
  }
  MOK(hipSetDevice(m->devices[0]));
  MOK(hipStreamSynchronize(rs));
  return 0;
}

int64_t batch_index(const MultiDev* m, int d, int64_t v) {
  return m->series.empty() ? m->pos0[d] + v : m->series[d][v];
}

// One result from the devices' results: groups in group id order (whole SpanGroups per device),
// or for NONE every span in batch order, renumbered (TsdbQuery.java:940-961).
int merge(MultiDev* m, const std::vector<tsdbhip_result*>& parts, bool none, tsdbhip_result** out) {
  struct E { int64_t key; int d; int64_t i; };
  std::vector<E> e;
  int64_t npts = 0;
  for (int d = 0; d < (int)parts.size(); d++) {
    const tsdbhip_result* r = parts[d];
    if (!r) continue;
    for (int64_t i = 0; i < r->n_groups; i++)
      e.push_back({none ? batch_index(m, d, r->group_id[i]) : (int64_t)r->group_id[i], d, i});
    npts += r->group_ptr[r->n_groups];
  }
  std::sort(e.begin(), e.end(), [](const E& a, const E& b) { return a.key < b.key; });
  tsdbhip_result* r = new_result((int64_t)e.size(), npts);
  if (!r) return set_error(TSDB_E_NOMEM, "result allocation");
  auto* gptr = const_cast<int64_t*>(r->group_ptr);
  auto* gid = const_cast<int32_t*>(r->group_id);
  auto* ts = const_cast<int64_t*>(r->ts_ms);
  auto* vb = const_cast<uint64_t*>(r->value_bits);
  auto* isi = const_cast<uint8_t*>(r->is_int);
  int64_t o = 0;
  for (size_t k = 0; k < e.size(); k++) {
    const tsdbhip_result* p = parts[e[k].d];
    const int64_t a = p->group_ptr[e[k].i], n = p->group_ptr[e[k].i + 1] - a;
    gptr[k] = o;
    gid[k] = none ? (int32_t)k : (int32_t)e[k].key;
    std::copy(p->ts_ms + a, p->ts_ms + a + n, ts + o);
    std::copy(p->value_bits + a, p->value_bits + a + n, vb + o);
    std::copy(p->is_int + a, p->is_int + a + n, isi + o);
    o += n;
  }
  gptr[e.size()] = o;
  *out = r;
  return 0;
}

void free_all(std::vector<tsdbhip_result*>& v) {
  for (auto*& r : v) {
    if (r) tsdbhip_result_free(r);
    r = nullptr;
  }
}

// Every device answers the query over its shard; the results merge.
int run_local(MultiDev* m, const tsdbhip_query* q, bool none, tsdbhip_result** out) {
  std::vector<tsdbhip_result*> parts(m->devices.size(), nullptr);
  int rc = each_device(m, [&](int d) { return tsdbhip_run(m->subs[d], q, &parts[d]); });
  const double t0 = now_ms();
  if (!rc) rc = merge(m, parts, none, out);
  m->timing.exchange_ms = now_ms() - t0;
  free_all(parts);
  return rc;
}

std::string per_span_calendar() {
  return "a calendar downsampling anchored per span (non-global grid) over a series-sharded multi-device context: "
         "load with tsdbhip_md_shard_mode(ctx, TSDB_SHARD_GROUPS)";
}

// Decomposable group-by over straddling groups: partial states per device -> gather -> merge in
// device order (tsdbhip_finalize on the merge context).
int run_partials_xchg(MultiDev* m, const tsdbhip_query* q, tsdbhip_result** out) {
  const std::vector<int> ds = live_devices(m);
  tsdbhip_partials_layout L{};
  int rc = tsdbhip_partials_layout_get(m->root, q, m->G, &L);
  if (rc) return rc;
  for (int d : ds) {
    tsdbhip_partials_layout Ld{};
    rc = tsdbhip_partials_layout_get(m->subs[d], q, m->G, &Ld);
    if (rc) return rc;
    if (Ld.bytes != L.bytes || Ld.n_slots != L.n_slots) return set_error(TSDB_E_NOT_IMPLEMENTED, per_span_calendar());
  }
  rc = each_device(m, [&](int d) {
    const int r = m->xb[d].ensure((size_t)L.bytes);
    return r ? r : tsdbhip_run_partials(m->subs[d], q, m->G, m->xb[d].p);
  });
  if (rc) return rc;
  const double t0 = now_ms();
  std::vector<const void*> src;
  std::vector<size_t> bytes;
  for (int d : ds) { src.push_back(m->xb[d].p); bytes.push_back((size_t)L.bytes); }
  rc = m->gb.ensure((size_t)L.bytes * ds.size());
  if (!rc) rc = gather(m, ds, src, bytes, m->gb.p);
  if (!rc) rc = tsdbhip_finalize(m->root, q, m->G, m->gb.p, (int)ds.size(), out);
  m->timing.exchange_ms = now_ms() - t0;
  return rc;
}

// Percentile / median group-by and TSDB_QF_ORDERED over straddling groups: every span's
// contributions are gathered to devices[0] in device (= SpanGroup) order, which selects / folds
// every (group, slot) there (tsdbhip_sel_select).
int run_sel_xchg(MultiDev* m, const tsdbhip_query* q, tsdbhip_result** out) {
  const std::vector<int> ds = live_devices(m);
  const int64_t G = m->G;
  int64_t K = 0;
  std::vector<int64_t> none_counts(std::max<int64_t>(1, G));
  int rc = tsdbhip_sel_layout(m->root, q, G, none_counts.data(), &K);
  if (rc) return rc;
  const int n = (int)m->devices.size();
  std::vector<std::vector<int64_t>> counts(n);
  std::vector<int64_t> n_series(n, 0);
  for (int d : ds) {
    counts[d].assign(std::max<int64_t>(1, G), 0);
    int64_t Kd = 0;
    rc = tsdbhip_sel_layout(m->subs[d], q, G, counts[d].data(), &Kd);
    if (rc) return rc;
    if (Kd != K) return set_error(TSDB_E_NOT_IMPLEMENTED, per_span_calendar());
    n_series[d] = ctx_n_series(m->subs[d]);
  }
  std::vector<std::vector<uint8_t>> uni(n);
  std::vector<std::vector<uint32_t>> act(n);
  for (int d : ds) {
    uni[d].assign(std::max<int64_t>(1, G * K), 0);
    act[d].assign(std::max<int64_t>(1, G), 0);
  }
  rc = each_device(m, [&](int d) {
    const int r = m->xb[d].ensure((size_t)(n_series[d] * K * 8));
    return r ? r : tsdbhip_sel_run_values(m->subs[d], q, G, m->xb[d].p, uni[d].data(), act[d].data());
  });
  if (rc) return rc;
  const double t0 = now_ms();
  std::vector<const void*> src;
  std::vector<size_t> bytes;
  std::vector<int64_t> total(std::max<int64_t>(1, G), 0);
  size_t all = 0;
  for (int d : ds) {
    int64_t nv = 0;
    for (int64_t g = 0; g < G; g++) { nv += counts[d][g]; total[g] += counts[d][g]; }
    src.push_back(m->xb[d].p);
    bytes.push_back((size_t)(nv * K * 8));   // the spans of groups (ungrouped spans come last)
    all += bytes.back();
  }
  std::vector<uint8_t> u(std::max<int64_t>(1, G * K), 0);
  std::vector<uint32_t> a(std::max<int64_t>(1, G), 0);
  for (int d : ds) {
    for (int64_t i = 0; i < G * K; i++) u[i] |= uni[d][i];
    for (int64_t g = 0; g < G; g++) a[g] |= act[d][g];
  }
  rc = m->gb.ensure(all);
  if (!rc) rc = gather(m, ds, src, bytes, m->gb.p);
  if (!rc) rc = m->ov.ensure((size_t)(G * K * 8));
  if (!rc) rc = m->of.ensure((size_t)(G * K));
  if (!rc) rc = tsdbhip_sel_select(m->root, q, G, m->gb.p, total.data(), u.data(), m->ov.p, m->of.p);
  if (!rc) rc = tsdbhip_assemble(m->root, q, G, m->ov.p, m->of.p, a.data(), out);
  m->timing.exchange_ms = now_ms() - t0;
  return rc;
}

int first_live(const MultiDev* m) {
  for (int d = 0; d < (int)m->devices.size(); d++) if (m->live[d]) return d;
  return 0;
}

int run_one(MultiDev* m, const tsdbhip_query* q, tsdbhip_result** out) {
  m->timing.exchange_ms = 0;
  if (m->mode == TSDB_SHARD_AUTO) return tsdbhip_run(m->root, q, out);   // nothing loaded: as one empty device
  int kind = 0;
  int rc = query_kind(m->subs[first_live(m)], q, &kind);
  if (rc) return rc;
  if (m->mode == TSDB_SHARD_GROUPS || kind == QK_NONE) return run_local(m, q, kind == QK_NONE, out);
  if (kind == QK_RAW)
    return set_error(TSDB_E_NOT_IMPLEMENTED, "a raw (no downsampling) group-by over a series-sharded multi-device context: "
                                             "load with tsdbhip_md_shard_mode(ctx, TSDB_SHARD_GROUPS)");
  return kind == QK_PARTIALS ? run_partials_xchg(m, q, out) : run_sel_xchg(m, q, out);
}

// Per-device stage times: maximum over the devices; counters: summed.
void device_timing(MultiDev* m, double wall_ms, bool fused) {
  tsdbhip_timing t{};
  int64_t fq = -1;
  for (int d : live_devices(m)) {
    tsdbhip_timing s{};
    if (tsdbhip_last_timing(m->subs[d], &s)) continue;
    t.decode_downsample_ms = std::max(t.decode_downsample_ms, s.decode_downsample_ms);
    t.group_reduce_ms = std::max(t.group_reduce_ms, s.group_reduce_ms);
    t.fast_ms = std::max(t.fast_ms, s.fast_ms);
    t.index_ms = std::max(t.index_ms, s.index_ms);
    t.compact_ms = std::max(t.compact_ms, s.compact_ms);
    t.datapoints += s.datapoints;
    t.bytes += s.bytes;
    t.tiles += s.tiles;
    t.redo_tiles += s.redo_tiles;
    fq = fq < 0 ? s.fused_queries : std::min(fq, s.fused_queries);
  }
  t.fused_queries = fused && fq > 0 ? fq : 0;
  t.total_ms = wall_ms;
  t.exchange_ms = m->timing.exchange_ms;
  m->timing = t;
}

}  // namespace

// ---- load -------------------------------------------------------------------------------
// The batch positions each device loads: whole SpanGroups (GROUPS) or a byte-balanced split of
// the SpanGroup order (SERIES); ungrouped series on the last device.  Sets m->live / mode state.
std::vector<std::vector<int64_t>> shard_series(MultiDev* m, const int32_t* gid, const std::vector<double>& w, int& mode,
                                               int64_t& G) {
  const int n = (int)m->devices.size();
  const int64_t S = (int64_t)w.size();
  int32_t maxg = -1;
  for (int64_t s = 0; s < S; s++) maxg = std::max(maxg, gid[s]);
  G = maxg + 1;
  std::vector<double> gw(G, 0.0);
  for (int64_t s = 0; s < S; s++) if (gid[s] >= 0) gw[gid[s]] += w[s];
  const std::vector<int64_t> gb = split(gw, n);
  mode = m->mode_req;
  if (mode == TSDB_SHARD_AUTO) mode = (n == 1 || groups_balanced(gw, gb, n)) ? TSDB_SHARD_GROUPS : TSDB_SHARD_SERIES;
  std::vector<std::vector<int64_t>> cand(n);
  if (mode == TSDB_SHARD_GROUPS) {
    std::vector<int32_t> owner(G, 0);
    for (int d = 0; d < n; d++)
      for (int64_t g = gb[d]; g < gb[d + 1]; g++) owner[g] = d;
    for (int64_t s = 0; s < S; s++) cand[gid[s] < 0 ? n - 1 : owner[gid[s]]].push_back(s);
  } else {
    std::vector<int64_t> order;   // kept series stably by group: the SpanGroup order
    for (int64_t s = 0; s < S; s++) if (gid[s] >= 0) order.push_back(s);
    std::stable_sort(order.begin(), order.end(), [&](int64_t x, int64_t y) { return gid[x] < gid[y]; });
    std::vector<double> ow(order.size());
    for (size_t i = 0; i < order.size(); i++) ow[i] = w[order[i]];
    const std::vector<int64_t> pb = split(ow, n);
    for (int d = 0; d < n; d++) cand[d].assign(order.begin() + pb[d], order.begin() + pb[d + 1]);
    for (int64_t s = 0; s < S; s++) if (gid[s] < 0) cand[n - 1].push_back(s);
  }
  m->mode = TSDB_SHARD_AUTO;
  m->series.clear();
  m->pos0.clear();
  m->live.assign(n, 0);
  bool any = false;
  for (int d = 0; d < n; d++) { m->live[d] = !cand[d].empty(); any = any || m->live[d]; }
  if (!any) m->live[0] = 1;   // an empty batch: device 0 holds it, as one device would
  return cand;
}

int md_load(tsdbhip_ctx* c, const tsdbhip_batch* b) {
  MultiDev* m = md_of(c);
  if (!b) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  if (b->n_series < 0 || b->n_rows < 0) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "negative sizes");
  if (b->n_series > 0 && (!b->series_row_ptr || !b->group_id || !b->row_qual_off || !b->row_val_off))
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null batch arrays");
  if (b->n_series > 0 && (b->series_row_ptr[0] != 0 || b->series_row_ptr[b->n_series] != b->n_rows))
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "series_row_ptr does not cover the rows");
  std::lock_guard<std::mutex> lk(ctx_mutex(c));
  const int64_t S = b->n_series;
  std::vector<double> w(S);
  for (int64_t s = 0; s < S; s++) {
    if (b->series_row_ptr[s + 1] < b->series_row_ptr[s]) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "series_row_ptr not monotonic");
    const int64_t r0 = b->series_row_ptr[s], r1 = b->series_row_ptr[s + 1];
    w[s] = (double)(b->row_qual_off[r1] - b->row_qual_off[r0]) + (double)(b->row_val_off[r1] - b->row_val_off[r0]);
  }
  int mode = 0;
  int64_t G = 0;
  const std::vector<std::vector<int64_t>> cand = shard_series(m, b->group_id, w, mode, G);
  ctx_drop_batch(m->root);   // (a rollup load before leaves rollup state on the merge context)
  const int rc = each_device(m, [&](int d) { return load_series(m->subs[d], b, cand[d]); });
  if (rc) {
    m->live.assign(m->devices.size(), 0);
    return rc;
  }
  m->mode = mode;
  m->G = G;
  m->series = cand;
  return 0;
}

// A rollup batch: each device loads the rollup spans of its series (value and count cells copied
// out of the caller's arrays); the merge context holds an empty rollup batch of the same table,
// so its plans (scan bounds of the rollup interval, count group-by as sum) match the devices'.
int md_load_rollup(tsdbhip_ctx* c, const tsdbhip_rollup_batch* rb) {
  MultiDev* m = md_of(c);
  if (!rb) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  const tsdbhip_batch* b = &rb->cells;
  const bool cnt = rb->row_cqual_off != nullptr;
  if (cnt && (!rb->row_cval_off || !rb->cqual || !rb->cval)) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null count arrays");
  if (b->n_series < 0 || b->n_rows < 0) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "negative sizes");
  if (b->n_series > 0 && (!b->series_row_ptr || !b->group_id)) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null batch arrays");
  if (b->n_rows > 0 && (!b->row_base_time || !b->row_qual_off || !b->row_val_off || !b->qual || !b->val))
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null batch arrays");
  if (b->n_series > 0 && (b->series_row_ptr[0] != 0 || b->series_row_ptr[b->n_series] != b->n_rows))
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "series_row_ptr does not cover the rows");
  const int64_t S = b->n_series;
  for (int64_t s = 0; s < S; s++)
    if (b->series_row_ptr[s + 1] < b->series_row_ptr[s]) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "series_row_ptr not monotonic");
  for (int64_t r = 0; r < b->n_rows; r++)
    if (b->row_qual_off[r + 1] < b->row_qual_off[r] || b->row_val_off[r + 1] < b->row_val_off[r] ||
        (cnt && (rb->row_cqual_off[r + 1] < rb->row_cqual_off[r] || rb->row_cval_off[r + 1] < rb->row_cval_off[r])))
      return set_error(TSDB_E_ILLEGAL_ARGUMENT, "cell offsets not monotonic");
  std::lock_guard<std::mutex> lk(ctx_mutex(c));
  std::vector<double> w(S);
  auto span = [](const uint64_t* o, int64_t r0, int64_t r1) { return (double)(o[r1] - o[r0]); };
  for (int64_t s = 0; s < S; s++) {
    const int64_t r0 = b->series_row_ptr[s], r1 = b->series_row_ptr[s + 1];
    w[s] = span(b->row_qual_off, r0, r1) + span(b->row_val_off, r0, r1) +
           (cnt ? span(rb->row_cqual_off, r0, r1) + span(rb->row_cval_off, r0, r1) : 0.0);
  }
  int mode = 0;
  int64_t G = 0;
  const std::vector<std::vector<int64_t>> cand = shard_series(m, b->group_id, w, mode, G);
  const int n = (int)m->devices.size();
  struct Sub {
    std::vector<int64_t> srp{0};
    std::vector<int32_t> gid;
    std::vector<uint32_t> base;
    std::vector<uint64_t> qo{0}, vo{0}, cqo{0}, cvo{0};
    std::vector<uint8_t> q, v, cq, cv;
    tsdbhip_rollup_batch rb{};
  };
  std::vector<Sub> sub(n);
  auto append = [](std::vector<uint8_t>& dst, std::vector<uint64_t>& off, const uint8_t* src, const uint64_t* o, int64_t r) {
    dst.insert(dst.end(), src + o[r], src + o[r + 1]);
    off.push_back(dst.size());
  };
  for (int d = 0; d < n; d++) {
    Sub& u = sub[d];
    for (int64_t s : cand[d]) {
      for (int64_t r = b->series_row_ptr[s]; r < b->series_row_ptr[s + 1]; r++) {
        u.base.push_back(b->row_base_time[r]);
        append(u.q, u.qo, b->qual, b->row_qual_off, r);
        append(u.v, u.vo, b->val, b->row_val_off, r);
        if (cnt) {
          append(u.cq, u.cqo, rb->cqual, rb->row_cqual_off, r);
          append(u.cv, u.cvo, rb->cval, rb->row_cval_off, r);
        }
      }
      u.srp.push_back((int64_t)u.base.size());
      u.gid.push_back(b->group_id[s]);
    }
    for (auto* x : {&u.q, &u.v, &u.cq, &u.cv}) if (x->empty()) x->push_back(0);
    if (u.gid.empty()) u.gid.push_back(-1);
    u.rb = *rb;
    u.rb.cells.n_series = (int64_t)cand[d].size();
    u.rb.cells.n_rows = (int64_t)u.base.size();
    u.rb.cells.series_row_ptr = u.srp.data();
    u.rb.cells.group_id = u.gid.data();
    u.rb.cells.row_base_time = u.base.empty() ? nullptr : u.base.data();
    u.rb.cells.row_qual_off = u.qo.data();
    u.rb.cells.row_val_off = u.vo.data();
    u.rb.cells.qual = u.q.data();
    u.rb.cells.val = u.v.data();
    u.rb.row_cqual_off = cnt ? u.cqo.data() : nullptr;
    u.rb.row_cval_off = cnt ? u.cvo.data() : nullptr;
    u.rb.cqual = cnt ? u.cq.data() : nullptr;
    u.rb.cval = cnt ? u.cv.data() : nullptr;
  }
  int rc = each_device(m, [&](int d) { return tsdbhip_load_rollup(m->subs[d], &sub[d].rb); });
  if (!rc) {   // the merge context: an empty batch of the same rollup table
    Sub e;
    e.q.push_back(0);
    e.rb = *rb;
    e.rb.cells = tsdbhip_batch{};
    e.rb.cells.series_row_ptr = e.srp.data();
    e.rb.cells.row_qual_off = e.qo.data();
    e.rb.cells.row_val_off = e.vo.data();
    e.rb.cells.qual = e.q.data();
    e.rb.cells.val = e.q.data();
    if (cnt) {
      e.rb.row_cqual_off = e.cqo.data();
      e.rb.row_cval_off = e.cvo.data();
      e.rb.cqual = e.rb.cval = e.q.data();
    }
    rc = tsdbhip_load_rollup(m->root, &e.rb);
  }
  if (rc) {
    m->live.assign(n, 0);
    return rc;
  }
  m->mode = mode;
  m->G = G;
  m->series = cand;
  return 0;
}

int md_synth(tsdbhip_ctx* c, const tsdbhip_synth_spec* sp) {
  MultiDev* m = md_of(c);
  if (!sp) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  if (sp->n_series <= 0 || sp->n_groups <= 0) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "bad synth spec");
  std::lock_guard<std::mutex> lk(ctx_mutex(c));
  const int n = (int)m->devices.size();
  const int64_t SG = sp->n_series, G = sp->n_groups;
  // group g holds batch positions [goff[g], goff[g + 1]) (tsdbhip_synth's layout)
  std::vector<int64_t> goff(G + 1, 0);
  std::vector<double> gw(G);
  for (int64_t g = 0; g < G; g++) {
    gw[g] = (double)(SG / G + (g < SG % G ? 1 : 0));
    goff[g + 1] = goff[g] + (int64_t)gw[g];
  }
  const std::vector<int64_t> gb = split(gw, n);
  int mode = m->mode_req;
  if (mode == TSDB_SHARD_AUTO) mode = (n == 1 || groups_balanced(gw, gb, n)) ? TSDB_SHARD_GROUPS : TSDB_SHARD_SERIES;
  std::vector<int64_t> p(n + 1);
  for (int d = 0; d <= n; d++) p[d] = mode == TSDB_SHARD_GROUPS ? goff[gb[d]] : SG * d / n;
  m->mode = TSDB_SHARD_AUTO;
  m->series.clear();
  m->live.assign(n, 0);
  for (int d = 0; d < n; d++) m->live[d] = p[d + 1] > p[d];
  ctx_drop_batch(m->root);
  const int rc = each_device(m, [&](int d) { return tsdbhip_synth_shard(m->subs[d], sp, p[d], p[d + 1]); });
  if (rc) {
    m->live.assign(n, 0);
    return rc;
  }
  m->pos0.assign(p.begin(), p.end() - 1);
  m->mode = mode;
  m->G = G;
  return 0;
}

// ---- queries ------------------------------------------------------------------------------
int md_run(tsdbhip_ctx* c, const tsdbhip_query* q, tsdbhip_result** out) {
  MultiDev* m = md_of(c);
  if (!q || !out) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  std::lock_guard<std::mutex> lk(ctx_mutex(c));
  *out = nullptr;
  const double t0 = now_ms();
  const int rc = run_one(m, q, out);
  if (!rc) device_timing(m, now_ms() - t0, false);
  return rc;
}

int md_run_multi(tsdbhip_ctx* c, const tsdbhip_query* qs, int n, tsdbhip_result** outs) {
  MultiDev* m = md_of(c);
  if (!qs || !outs || n < 1) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "bad argument");
  std::lock_guard<std::mutex> lk(ctx_mutex(c));
  for (int i = 0; i < n; i++) outs[i] = nullptr;
  const double t0 = now_ms();
  m->timing.exchange_ms = 0;
  int rc = 0;
  if (m->mode == TSDB_SHARD_GROUPS) {
    // whole SpanGroups per device: each device runs its own fused pass over the queries
    const int nd = (int)m->devices.size();
    std::vector<std::vector<tsdbhip_result*>> parts(nd, std::vector<tsdbhip_result*>(n, nullptr));
    rc = each_device(m, [&](int d) { return tsdbhip_run_multi(m->subs[d], qs, n, parts[d].data()); });
    const double t1 = now_ms();
    for (int i = 0; i < n && !rc; i++) {
      std::vector<tsdbhip_result*> pi(nd, nullptr);
      for (int d = 0; d < nd; d++) pi[d] = parts[d][i];
      rc = merge(m, pi, qs[i].aggregator == TSDB_AGG_NONE, &outs[i]);
    }
    m->timing.exchange_ms = now_ms() - t1;
    for (auto& p : parts) free_all(p);
  } else {
    for (int i = 0; i < n && !rc; i++) rc = run_one(m, &qs[i], &outs[i]);
  }
  if (rc) {
    for (int i = 0; i < n; i++) {
      if (outs[i]) tsdbhip_result_free(outs[i]);
      outs[i] = nullptr;
    }
    return rc;
  }
  device_timing(m, now_ms() - t0, m->mode == TSDB_SHARD_GROUPS);
  return 0;
}

int md_timing(tsdbhip_ctx* c, tsdbhip_timing* out) {
  if (!out) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  *out = md_of(c)->timing;
  return 0;
}

int md_sync(tsdbhip_ctx* c) {
  MultiDev* m = md_of(c);
  return each_device(m, [&](int d) { return tsdbhip_sync(m->subs[d]); }, true);
}

int md_batch_sizes(tsdbhip_ctx* c, int64_t* n_series, int64_t* n_rows, uint64_t* qual_bytes, uint64_t* val_bytes) {
  MultiDev* m = md_of(c);
  if (!n_series || !n_rows || !qual_bytes || !val_bytes) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  *n_series = *n_rows = 0;
  *qual_bytes = *val_bytes = 0;
  for (int d = 0; d < (int)m->devices.size(); d++) {
    if (!m->live.empty() && !m->live[d]) continue;
    int64_t ns = 0, nr = 0;
    uint64_t qb = 0, vb = 0;
    const int rc = tsdbhip_batch_sizes(m->subs[d], &ns, &nr, &qb, &vb);
    if (rc) return rc;
    *n_series += ns;
    *n_rows += nr;
    *qual_bytes += qb;
    *val_bytes += vb;
  }
  return 0;
}

void md_destroy(void* p) {
  auto* m = static_cast<MultiDev*>(p);
  if (!m) return;
  for (ncclComm_t cm : m->comms) if (cm) (void)rccl().destroy(cm);
  for (Buf& b : m->xb) b.release();
  m->gb.release();
  m->ov.release();
  m->of.release();
  for (tsdbhip_ctx* s : m->subs) tsdbhip_destroy(s);
  if (m->root) tsdbhip_destroy(m->root);
  delete m;
}

}  // namespace tsdb

using namespace tsdb;

extern "C" int tsdbhip_init_devices(const int* devices, int n_devices, int transport, tsdbhip_ctx** out) {
  if (!devices || n_devices < 1 || !out) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "bad argument");
  *out = nullptr;
  if (transport != TSDB_MD_AUTO && transport != TSDB_MD_COPY && transport != TSDB_MD_RCCL)
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "bad transport");
  int count = 0;
  MOK(hipGetDeviceCount(&count));
  for (int d = 0; d < n_devices; d++)
    if (devices[d] < 0 || devices[d] >= count)
      return set_error(TSDB_E_HIP, "no such HIP device " + std::to_string(devices[d]));
  const bool distinct = std::set<int>(devices, devices + n_devices).size() == (size_t)n_devices;
  if (transport == TSDB_MD_RCCL && !distinct)
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "RCCL needs distinct devices (one rank per GPU)");
  int tr = transport;
  if (tr == TSDB_MD_AUTO) tr = distinct && rccl().ok ? TSDB_MD_RCCL : TSDB_MD_COPY;
  if (tr == TSDB_MD_RCCL && !rccl().ok) return set_error(TSDB_E_HIP, "RCCL unavailable: " + rccl().why);
  tsdbhip_ctx* c = nullptr;
  int rc = tsdbhip_init(devices[0], &c);
  if (rc) return rc;
  auto* m = new MultiDev();
  ctx_md(c) = m;   // tsdbhip_destroy(c) releases it from here on
  m->devices.assign(devices, devices + n_devices);
  m->transport = tr;
  m->live.assign(n_devices, 0);
  for (int d = 0; d < n_devices && !rc; d++) {
    tsdbhip_ctx* s = nullptr;
    rc = tsdbhip_init(devices[d], &s);
    if (!rc) {
      ctx_set_none_orig(s, true);
      m->subs.push_back(s);
      m->xb.push_back(Buf{devices[d]});
    }
  }
  if (!rc) rc = tsdbhip_init(devices[0], &m->root);
  m->gb.dev = m->ov.dev = m->of.dev = devices[0];
  if (!rc && tr == TSDB_MD_RCCL) {
    m->comms.assign(n_devices, nullptr);
    const ncclResult_t e = rccl().init_all(m->comms.data(), n_devices, devices);
    if (e != ncclSuccess) {
      m->comms.clear();
      rc = rccl_fail(e, "ncclCommInitAll");
    }
  }
  if (rc) {
    const std::string msg = tsdbhip_last_error();
    tsdbhip_destroy(c);
    return set_error(rc, msg);
  }
  *out = c;
  return 0;
}

extern "C" int tsdbhip_md_shard_mode(tsdbhip_ctx* c, int mode) {
  if (!c || !md_of(c)) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "not a multi-device context (tsdbhip_init_devices)");
  if (mode != TSDB_SHARD_AUTO && mode != TSDB_SHARD_SERIES && mode != TSDB_SHARD_GROUPS)
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "shard mode must be TSDB_SHARD_AUTO, _SERIES or _GROUPS");
  std::lock_guard<std::mutex> lk(ctx_mutex(c));
  md_of(c)->mode_req = mode;
  return 0;
}

extern "C" int tsdbhip_md_info(tsdbhip_ctx* c, int* n_devices, int* transport, int* mode, int64_t* shard_series) {
  if (!c || !md_of(c)) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "not a multi-device context (tsdbhip_init_devices)");
  MultiDev* m = md_of(c);
  std::lock_guard<std::mutex> lk(ctx_mutex(c));
  if (n_devices) *n_devices = (int)m->devices.size();
  if (transport) *transport = m->transport;
  if (mode) *mode = m->mode;
  if (shard_series) {
    for (int d = 0; d < (int)m->devices.size(); d++) {
      shard_series[d] = 0;
      if (!m->live[d]) continue;
      if (!m->series.empty()) {   // loaded: the batch series the device holds
        shard_series[d] = (int64_t)m->series[d].size();
      } else {                    // synthesized
        int64_t ns = 0, nr = 0;
        uint64_t qb = 0, vb = 0;
        if (tsdbhip_batch_sizes(m->subs[d], &ns, &nr, &qb, &vb) == 0) shard_series[d] = ns;
      }
    }
  }
  return 0;
}
