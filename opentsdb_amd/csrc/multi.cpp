// One process, several GPUs behind one tsdbhip_ctx (include/tsdbhip.h, "multi-device context";
// SURVEY.md 8e).  The reference runs a query's whole scan in one TSD: TsdbQuery.run
// (src/core/TsdbQuery.java:800-870) feeds every span of a SpanGroup to one AggregationIterator
// (GroupByAndAggregateCB :927-1048).  A TSD JVM that owns all the GPUs of a node therefore wants
// ONE engine handle that spreads the spans of the query over them, not one process per GPU.
//
// A multi-device context holds one ordinary engine context (stream, scratch, resident shard)
// per device and a merge context on devices[0].  Loads split the batch by bytes:
//   GROUPS  whole SpanGroups per device -- every query runs locally, results concatenate;
//   SERIES  contiguous positions of the SpanGroup order, so a group may straddle devices:
//           - decomposable aggregators: the devices' partial states are gathered to devices[0]
//             and merged in device order, which continues SpanGroup order across devices;
//           - percentile / median group-by and TSDB_QF_ORDERED: group g is owned by the first
//             device holding one of its spans; only the straddling groups' span rows move (to
//             the owner, appended in device order), every owner selects its groups in place, and
//             the owners' dense (group, slot) rows go to devices[0];
//           - raw group-by (no downsampler): each straddling group is assembled once per load on
//             its owner (a side context holding the whole SpanGroup), so every group is evaluated
//             over all its spans in SpanGroup order on one device.
// Device-to-device bytes move over RCCL (grouped ncclSend / ncclRecv, one rank per GPU,
// ncclCommInitAll) or peer copies.  Every device runs on its own persistent host thread.
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cstring>
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
// The system's librccl.so.1 (built against the same HIP runtime as this library; PyTorch's wheel
// carries its own librccl.so and HIP runtime, which this does not bind).  Resolved at run time:
// the library itself loads without RCCL, and a context whose devices repeat (several shards on
// one GPU) never needs it.
struct Rccl {
  bool ok = false;
  std::string why;
  decltype(&ncclCommInitAll) init_all = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclCommCount) count = nullptr;
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
    r.count = reinterpret_cast<decltype(r.count)>(dlsym(h, "ncclCommCount"));
    r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
    r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
    r.send = reinterpret_cast<decltype(r.send)>(dlsym(h, "ncclSend"));
    r.recv = reinterpret_cast<decltype(r.recv)>(dlsym(h, "ncclRecv"));
    r.err_str = reinterpret_cast<decltype(r.err_str)>(dlsym(h, "ncclGetErrorString"));
    r.ok = r.init_all && r.destroy && r.count && r.group_start && r.group_end && r.send && r.recv && r.err_str;
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

// One persistent host thread per device slot but the first (slot 0's work runs on the calling
// thread): a query's per-device calls start without a thread creation each (8 x ~30 us).
class Workers {
 public:
  explicit Workers(int n) : slots_(n) {
    for (int i = 1; i < n; i++) th_.emplace_back([this, i] { loop(i); });
  }
  ~Workers() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // fn(i) for every i of idx at once; returns when all have finished.  Callers are serialized
  // (call_mu_): the slots and pending_ belong to one call at a time.
  void run(const std::vector<int>& idx, const std::function<void(int)>& fn) {
    std::lock_guard<std::mutex> call(call_mu_);
    // slot 0 (no worker of its own) runs here, or else the last slot of the set
    const int inline_i = std::find(idx.begin(), idx.end(), 0) != idx.end() ? 0 : idx.back();
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (int i : idx) {
        if (i == inline_i) continue;
        slots_[i].job = [&fn, i] { fn(i); };
        slots_[i].has = true;
        pending_++;
      }
    }
    cv_.notify_all();
    fn(inline_i);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [this] { return pending_ == 0; });
  }

 private:
  struct Slot {
    std::function<void()> job;
    bool has = false;
  };
  void loop(int i) {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || slots_[i].has; });
      if (!slots_[i].has) return;
      std::function<void()> job = std::move(slots_[i].job);
      lk.unlock();
      job();
      lk.lock();
      slots_[i].has = false;
      if (--pending_ == 0) done_.notify_all();
    }
  }
  std::mutex call_mu_, mu_;
  std::condition_variable cv_, done_;
  std::vector<Slot> slots_;
  std::vector<std::thread> th_;
  int pending_ = 0;
  bool stop_ = false;
};

struct MultiDev {
  std::vector<int> devices;
  std::vector<tsdbhip_ctx*> subs;       // one engine context per device (slot d = RCCL rank d)
  tsdbhip_ctx* root = nullptr;          // merge context on devices[0]
  int transport = TSDB_MD_COPY;
  std::vector<ncclComm_t> comms;
  Workers* pool = nullptr;
  int mode_req = TSDB_SHARD_AUTO;       // shard mode of the next load
  int mode = TSDB_SHARD_AUTO;           // shard mode of the resident batch (AUTO: nothing loaded)
  int64_t G = 0;                        // groups of the whole batch
  std::vector<char> live;               // the device holds series
  std::vector<std::vector<int64_t>> series;   // load: batch index of each resident virtual position
  std::vector<int64_t> pos0;            // synth: first batch position of each shard
  bool rollup = false;                  // the resident batch is a rollup table
  // raw group-by over SERIES shards: per owner device a side context holding the whole straddling
  // SpanGroups it owns, built at the first raw query after a load
  bool side_valid = false;
  std::vector<tsdbhip_ctx*> side;
  std::vector<char> straddle;           // [G] the group's spans sit on several devices
  std::vector<Buf> xb;                  // per device: exchange source (partial states)
  std::vector<Buf> mb;                  // per device: straddling groups' states from later devices
  std::vector<Buf> dv, df, da;          // per device: owned groups' dense values / emit flags / activity
  Buf ov, of, oa;                       // devices[0]: the owners' dense rows gathered
  // resident series of each group on each device, per load (owner-routed partials)
  bool gcnt_valid = false;
  std::vector<std::vector<int64_t>> gcnt;
  // stage wall times of the current call (tsdbhip_timing devices / xfer / select / assemble_ms)
  double t_dev = 0, t_xfer = 0, t_sel = 0, t_asm = 0;
  tsdbhip_timing timing{};
  std::vector<tsdbhip_timing> dev_timing;   // per device, last call
  double xfer_bytes = 0;                // device-to-device bytes of the last call
  // the last rollup generation: per device, per function, its cells / value bytes (on the device
  // until tsdbhip_rollup_download)
  bool ro_valid = false;
  int ro_nf = 0;
  std::vector<std::vector<int64_t>> ro_cells;
  std::vector<std::vector<uint64_t>> ro_bytes;
  // the histogram store (tsdbhip_load_histograms): whole groups per device; per device its spans'
  // batch indices, and the devices holding spans
  bool hist_loaded = false;
  std::vector<int> hist_devs;
  std::vector<std::vector<int64_t>> hist_series;
};

MultiDev* md_of(tsdbhip_ctx* c) { return static_cast<MultiDev*>(ctx_md(c)); }

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// fn(d) for every d of `run`, each on its device's worker; the error of the first failing device
// in device order is the call's.
int each_of(MultiDev* m, const std::vector<int>& run, const std::function<int(int)>& fn) {
  if (run.empty()) return 0;
  if (run.size() == 1) return fn(run[0]);
  const int n = (int)m->devices.size();
  std::vector<int> rc(n, 0);
  std::vector<std::string> msg(n);
  m->pool->run(run, [&](int d) {
    rc[d] = fn(d);
    if (rc[d]) msg[d] = tsdbhip_last_error();
  });
  for (int d : run) if (rc[d]) return set_error(rc[d], msg[d]);
  return 0;
}

// ... for every live device (all devices when `all`)
int each_device(MultiDev* m, const std::function<int(int)>& fn, bool all = false) {
  std::vector<int> run;
  for (int d = 0; d < (int)m->devices.size(); d++) if (all || m->live[d]) run.push_back(d);
  return each_of(m, run, fn);
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

// One device-to-device copy: bytes from slot `src` (device memory there) to slot `dst`.
struct Xfer {
  int src;
  const void* sp;
  int dst;
  void* dp;
  size_t n;
};

// Moves every piece: RCCL -- one grouped round of ncclSend / ncclRecv between the ranks, pieces
// within a device as copies on its stream; COPY -- peer copies on the destination's stream.
// Sources must be complete; returns when every destination holds its bytes.
int transfer_(MultiDev* m, const std::vector<Xfer>& xs);
int transfer(MultiDev* m, const std::vector<Xfer>& xs) {
  const double t0 = now_ms();
  const int rc = transfer_(m, xs);
  m->t_xfer += now_ms() - t0;
  return rc;
}
int transfer_(MultiDev* m, const std::vector<Xfer>& xs) {
  const int n = (int)m->devices.size();
  std::vector<char> used(n, 0);
  auto st = [&](int d) { return ctx_stream(m->subs[d]); };
  for (const Xfer& x : xs) {
    if (!x.n) continue;
    used[x.src] = used[x.dst] = 1;
    m->xfer_bytes += x.src != x.dst ? (double)x.n : 0.0;
  }
  if (m->transport == TSDB_MD_RCCL) {
    for (const Xfer& x : xs) {
      if (!x.n || x.src != x.dst) continue;
      MOK(hipSetDevice(m->devices[x.dst]));
      MOK(hipMemcpyAsync(x.dp, x.sp, x.n, hipMemcpyDeviceToDevice, st(x.dst)));
    }
    Rccl& R = rccl();
    ncclResult_t e = R.group_start();
    if (e != ncclSuccess) return rccl_fail(e, "ncclGroupStart");
    for (const Xfer& x : xs) {
      if (!x.n || x.src == x.dst) continue;
      // the same list drives both sides, so the pieces of every (src, dst) pair are posted in
      // the same order at the sender and at the receiver
      e = R.send(x.sp, x.n, ncclUint8, x.dst, m->comms[x.src], st(x.src));
      if (e == ncclSuccess) e = R.recv(x.dp, x.n, ncclUint8, x.src, m->comms[x.dst], st(x.dst));
      if (e != ncclSuccess) {
        (void)R.group_end();
        return rccl_fail(e, "ncclSend / ncclRecv");
      }
    }
    e = R.group_end();
    if (e != ncclSuccess) return rccl_fail(e, "ncclGroupEnd");
  } else {
    for (const Xfer& x : xs) {
      if (!x.n) continue;
      MOK(hipSetDevice(m->devices[x.dst]));
      MOK(hipMemcpyPeerAsync(x.dp, m->devices[x.dst], x.sp, m->devices[x.src], x.n, st(x.dst)));
    }
  }
  for (int d = 0; d < n; d++) {
    if (!used[d]) continue;
    MOK(hipSetDevice(m->devices[d]));
    MOK(hipStreamSynchronize(st(d)));
  }
  return 0;
}

int64_t batch_index(const MultiDev* m, int d, int64_t v) {
  return m->series.empty() ? m->pos0[d] + v : m->series[d][v];
}

// One result from the devices' results: groups in group id order (whole SpanGroups per device),
// or for NONE every span in batch order, renumbered (TsdbQuery.java:940-961).  parts[i] belongs
// to device slot i % n_devices; for i < n_skip the groups flagged in `skip` are left out (their
// answer comes from a later part).
int merge(MultiDev* m, const std::vector<tsdbhip_result*>& parts, bool none, tsdbhip_result** out,
          const std::vector<char>* skip = nullptr, size_t n_skip = 0) {
  struct E { int64_t key; int p; int64_t i; };
  const int nd = (int)m->devices.size();
  std::vector<E> e;
  int64_t npts = 0;
  for (int p = 0; p < (int)parts.size(); p++) {
    const tsdbhip_result* r = parts[p];
    if (!r) continue;
    for (int64_t i = 0; i < r->n_groups; i++) {
      const int64_t key = none ? batch_index(m, p % nd, r->group_id[i]) : (int64_t)r->group_id[i];
      if (skip && (size_t)p < n_skip && key >= 0 && key < (int64_t)skip->size() && (*skip)[key]) continue;
      e.push_back({key, p, i});
      npts += r->group_ptr[i + 1] - r->group_ptr[i];
    }
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
    const tsdbhip_result* p = parts[e[k].p];
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
  double t0 = now_ms();
  int rc = each_device(m, [&](int d) { return tsdbhip_run(m->subs[d], q, &parts[d]); });
  m->t_dev += now_ms() - t0;
  t0 = now_ms();
  if (!rc) rc = merge(m, parts, none, out);
  m->t_asm += now_ms() - t0;
  free_all(parts);
  return rc;
}

std::string per_span_calendar() {
  return "a calendar downsampling anchored per span (non-global grid) over a series-sharded multi-device context: "
         "load with tsdbhip_md_shard_mode(ctx, TSDB_SHARD_GROUPS)";
}

// Group ownership over SERIES shards: group g is owned by the first device holding one of its
// spans (a group without spans: the owner of the group before it, so owned ranges are
// contiguous).  Shards are contiguous in SpanGroup order, so a device's groups it does not own
// precede the ones it owns, and only its last owned group can continue on later devices.
struct Owners {
  std::vector<int> owner;                // [G]
  std::vector<int64_t> total;            // [G] spans over every device
  std::vector<int64_t> skip, rows;       // [n] spans of groups the device does not own (a prefix); all its spans
  std::vector<int64_t> last, extra;      // [n] its last owned group, and that group's spans on later devices
  std::vector<int64_t> ga, gb;           // [n] owned group range [ga, gb) (-1: owns none)
  std::vector<std::vector<int>> later;   // [n] the later devices holding spans of last[o], in device order
};

int owners_of(const MultiDev* m, const std::vector<int>& ds, const std::vector<std::vector<int64_t>>& cnt, Owners& O) {
  const int n = (int)m->devices.size();
  const int64_t G = m->G;
  O.owner.assign(std::max<int64_t>(1, G), ds[0]);
  O.total.assign(std::max<int64_t>(1, G), 0);
  for (int64_t g = 0, prev = ds[0]; g < G; g++) {
    int o = -1;
    for (int d : ds) {
      if (cnt[d][g] > 0 && o < 0) o = d;
      O.total[g] += cnt[d][g];
    }
    O.owner[g] = o < 0 ? (int)prev : o;
    prev = O.owner[g];
  }
  O.skip.assign(n, 0);
  O.rows.assign(n, 0);
  O.extra.assign(n, 0);
  O.last.assign(n, -1);
  O.ga.assign(n, -1);
  O.gb.assign(n, -1);
  O.later.assign(n, {});
  for (int d : ds) {
    bool owned_seen = false;
    for (int64_t g = 0; g < G; g++) {
      if (O.owner[g] == d) {
        if (O.ga[d] < 0) O.ga[d] = g;
        O.gb[d] = g + 1;
      }
      if (!cnt[d][g]) continue;
      O.rows[d] += cnt[d][g];
      if (O.owner[g] != d) {
        if (owned_seen) return set_error(TSDB_E_HIP, "multi-device exchange: shard not contiguous in SpanGroup order");
        O.skip[d] += cnt[d][g];
        continue;
      }
      if (O.last[d] >= 0 && O.total[O.last[d]] != cnt[d][O.last[d]])
        return set_error(TSDB_E_HIP, "multi-device exchange: a straddling group inside a shard");
      owned_seen = true;
      O.last[d] = g;
    }
    if (O.last[d] >= 0) {
      O.extra[d] = O.total[O.last[d]] - cnt[d][O.last[d]];
      for (int e : ds)
        if (e > d && cnt[e][O.last[d]] > 0) O.later[d].push_back(e);
    }
  }
  return 0;
}

// resident series of every group on every live device, once per load
const std::vector<std::vector<int64_t>>& group_counts(MultiDev* m) {
  if (!m->gcnt_valid) {
    m->gcnt.assign(m->devices.size(), {});
    for (int d : live_devices(m)) m->gcnt[d] = ctx_group_counts(m->subs[d], m->G);
    m->gcnt_valid = true;
  }
  return m->gcnt;
}

// Decomposable group-by over straddling groups (sum, count, min, max, avg, dev
// partials), owner-routed: every device reduces its shard to per-(group, slot) partial states
// (n queries from one fused pass when they share the downsampling, tsdbhip_run_partials_multi);
// only the straddling groups' K-slot states move, to their owners, which fold them in device
// order (= SpanGroup order, TsdbQuery.java:916-1049's one AggregationIterator per group) and
// finalise their groups in place; the owners' dense (group, slot) rows (G x K x 9 B a query)
// go to devices[0] for the result.  No device receives every device's G x K states.
int run_partials_owner(MultiDev* m, const tsdbhip_query* qs, int nq, tsdbhip_result** outs) {
  const std::vector<int> ds = live_devices(m);
  const int64_t G = m->G;
  tsdbhip_partials_layout L{};
  int rc = tsdbhip_partials_layout_get(m->root, &qs[0], G, &L);
  if (rc) return rc;
  for (int d : ds) {
    tsdbhip_partials_layout Ld{};
    rc = tsdbhip_partials_layout_get(m->subs[d], &qs[0], G, &Ld);
    if (rc) return rc;
    if (Ld.bytes != L.bytes || Ld.n_slots != L.n_slots) return set_error(TSDB_E_NOT_IMPLEMENTED, per_span_calendar());
  }
  const int64_t K = L.n_slots;
  int64_t off_b = 0, off_n = 0, off_f = 0, off_act = 0, bytes = 0;
  partials_offsets(G, K, &off_b, &off_n, &off_f, &off_act, &bytes);
  Owners O;
  rc = owners_of(m, ds, group_counts(m), O);
  if (rc) return rc;
  // 1. every device's partial states, nq queries' buffers back to back
  double t0 = now_ms();
  rc = each_device(m, [&](int d) {
    const int r = m->xb[d].ensure((size_t)L.bytes * nq);
    if (r) return r;
    return nq > 1 ? tsdbhip_run_partials_multi(m->subs[d], qs, nq, G, m->xb[d].p)
                  : tsdbhip_run_partials(m->subs[d], &qs[0], G, m->xb[d].p);
  });
  m->t_dev += now_ms() - t0;
  if (rc) return rc;
  // 2. the straddling groups' states to their owners (mini states, in device order)
  const int64_t ms = mini_state_stride(K);
  std::vector<Xfer> xs;
  for (int o : ds) {
    const int nm = (int)O.later[o].size();
    if (!nm) continue;
    rc = m->mb[o].ensure((size_t)(ms * nm * nq));
    if (rc) return rc;
    const int64_t g = O.last[o];
    for (int i = 0; i < nq; i++)
      for (int j = 0; j < nm; j++) {
        const int d = O.later[o][j];
        const char* src = static_cast<const char*>(m->xb[d].p) + (int64_t)i * L.bytes;
        char* dst = static_cast<char*>(m->mb[o].p) + ((int64_t)i * nm + j) * ms;
        xs.push_back({d, src + g * K * 8, o, dst, (size_t)(K * 8)});
        xs.push_back({d, src + off_b + g * K * 8, o, dst + 8 * K, (size_t)(K * 8)});
        xs.push_back({d, src + off_n + g * K * 4, o, dst + 16 * K, (size_t)(K * 4)});
        xs.push_back({d, src + off_f + g * K * 4, o, dst + 20 * K, (size_t)(K * 4)});
        xs.push_back({d, src + off_act + g * 4, o, dst + 24 * K, 4});
      }
  }
  rc = transfer(m, xs);
  if (rc) return rc;
  // 3. every owner folds its straddling group and finalises its groups: dense rows on the device
  std::vector<int> owners;
  for (int d : ds) if (O.ga[d] >= 0) owners.push_back(d);
  const int64_t gk = std::max<int64_t>(1, G * K);
  t0 = now_ms();
  rc = each_of(m, owners, [&](int o) {
    int r = m->dv[o].ensure((size_t)(gk * 8 * nq));
    if (!r) r = m->df[o].ensure((size_t)(gk * nq));
    if (!r) r = m->da[o].ensure((size_t)(std::max<int64_t>(1, G) * 4 * nq));
    for (int i = 0; i < nq && !r; i++)
      r = md_partials_finish(m->subs[o], &qs[i], G, static_cast<unsigned char*>(m->xb[o].p) + (int64_t)i * L.bytes,
                             O.last[o], static_cast<const unsigned char*>(m->mb[o].p) + (int64_t)i * O.later[o].size() * ms,
                             (int)O.later[o].size(), static_cast<double*>(m->dv[o].p) + i * gk,
                             static_cast<uint8_t*>(m->df[o].p) + i * gk,
                             static_cast<uint32_t*>(m->da[o].p) + i * std::max<int64_t>(1, G));
    return r;
  });
  m->t_sel += now_ms() - t0;
  if (rc) return rc;
  // 4. the owners' rows to devices[0]
  rc = m->ov.ensure((size_t)(gk * 8 * nq));
  if (!rc) rc = m->of.ensure((size_t)(gk * nq));
  if (!rc) rc = m->oa.ensure((size_t)(std::max<int64_t>(1, G) * 4 * nq));
  if (rc) return rc;
  std::vector<Xfer> ys;
  for (int i = 0; i < nq; i++)
    for (int o : owners) {
      const int64_t r0 = O.ga[o] * K, nr = (O.gb[o] - O.ga[o]) * K;
      const int64_t vo = i * gk + r0, ao = i * std::max<int64_t>(1, G) + O.ga[o];
      ys.push_back({o, static_cast<double*>(m->dv[o].p) + vo, 0, static_cast<double*>(m->ov.p) + vo, (size_t)(nr * 8)});
      ys.push_back({o, static_cast<uint8_t*>(m->df[o].p) + vo, 0, static_cast<uint8_t*>(m->of.p) + vo, (size_t)nr});
      ys.push_back({o, static_cast<uint32_t*>(m->da[o].p) + ao, 0, static_cast<uint32_t*>(m->oa.p) + ao,
                    (size_t)((O.gb[o] - O.ga[o]) * 4)});
    }
  rc = transfer(m, ys);
  if (rc) return rc;
  // 5. the results on the host: the query list's rows in one copy per array, assembled side by side
  t0 = now_ms();
  rc = md_assemble(m->root, qs, nq, G, gk, m->ov.p, m->of.p, m->oa.p, outs);
  m->t_asm += now_ms() - t0;
  return rc;
}

// Percentile / median group-by and TSDB_QF_ORDERED over straddling groups (the
// values of a non-decomposable aggregate go to the owning rank; Aggregators.java:657-708).
// Group g's owner is the first device holding one of its spans (Owners).  The straddling groups'
// rows are appended to their owner's rows in device order (= SpanGroup order), and each owner
// selects its groups over rows that never left it.  Traffic: the straddling groups' rows plus
// G * K * 9 B of results, instead of every span's contributions to devices[0].
int run_sel_xchg(MultiDev* m, const tsdbhip_query* q, tsdbhip_result** out) {
  const std::vector<int> ds = live_devices(m);
  const int n = (int)m->devices.size();
  const int64_t G = m->G;
  int64_t K = 0;
  int rc = 0;
  {
    std::vector<int64_t> none_counts(std::max<int64_t>(1, G));
    rc = tsdbhip_sel_layout(m->root, q, G, none_counts.data(), &K);   // the merge context's refusals
    if (rc) return rc;
  }
  std::vector<std::vector<int64_t>> cnt(n);
  for (int d : ds) {
    cnt[d].assign(std::max<int64_t>(1, G), 0);
    int64_t Kd = 0;
    rc = tsdbhip_sel_layout(m->subs[d], q, G, cnt[d].data(), &Kd);
    if (rc) return rc;
    if (Kd != K) return set_error(TSDB_E_NOT_IMPLEMENTED, per_span_calendar());
  }
  Owners O;
  rc = owners_of(m, ds, cnt, O);
  if (rc) return rc;
  std::vector<double*> vals(n, nullptr);
  std::vector<std::vector<uint8_t>> uni(n);
  std::vector<std::vector<uint32_t>> act(n);
  for (int d : ds) {
    uni[d].assign(std::max<int64_t>(1, G * K), 0);
    act[d].assign(std::max<int64_t>(1, G), 0);
  }
  double t0 = now_ms();
  rc = each_of(m, ds, [&](int d) {
    int64_t Kd = 0;
    return md_sel_values(m->subs[d], q, G, O.extra[d], &vals[d], &Kd, uni[d].data(), act[d].data());
  });
  m->t_dev += now_ms() - t0;
  if (rc) return rc;
  // 1. the straddling groups' rows to their owners, appended in device order
  std::vector<Xfer> xs;
  for (int o : ds) {
    if (O.last[o] < 0 || !O.extra[o]) continue;
    const int64_t g = O.last[o];
    int64_t at = O.rows[o];
    for (int d : O.later[o]) {
      int64_t pre = 0;   // rows before g on d
      for (int64_t h = 0; h < g; h++) pre += cnt[d][h];
      xs.push_back({d, vals[d] + pre * K, o, vals[o] + at * K, (size_t)(cnt[d][g] * K * 8)});
      at += cnt[d][g];
    }
  }
  rc = transfer(m, xs);
  if (rc) return rc;
  // 2. every owner selects its groups (the rows of groups it does not own are skipped).  Its emit
  // flags are its own, OR-ed with the later devices' flags of its straddling group (K bytes each);
  // group activity over every device (G words each)
  t0 = now_ms();
  std::vector<uint32_t> a(std::max<int64_t>(1, G), 0);
  for (int d : ds)
    for (int64_t g = 0; g < G; g++) a[g] |= act[d][g];
  std::vector<int> owners;
  std::vector<std::vector<int64_t>> oc(n);
  for (int d : ds) {
    if (O.ga[d] < 0) continue;
    owners.push_back(d);
    oc[d].assign(std::max<int64_t>(1, G), 0);
    for (int64_t g = O.ga[d]; g < O.gb[d]; g++) oc[d][g] = O.total[g];
    if (O.last[d] >= 0)
      for (int e : O.later[d])
        for (int64_t k = 0; k < K; k++) uni[d][O.last[d] * K + k] |= uni[e][O.last[d] * K + k];
  }
  std::vector<double*> ov(n, nullptr);
  std::vector<uint8_t*> of(n, nullptr);
  rc = each_of(m, owners, [&](int d) {
    return md_sel_select(m->subs[d], q, G, vals[d] + O.skip[d] * K, oc[d].data(), uni[d].data(), &ov[d], &of[d]);
  });
  m->t_sel += now_ms() - t0;
  // 3. the owners' dense rows to devices[0]
  if (!rc) rc = m->ov.ensure((size_t)(G * K * 8));
  if (!rc) rc = m->of.ensure((size_t)(G * K));
  if (rc) return rc;
  std::vector<Xfer> ys;
  for (int d : owners) {
    const int64_t r0 = O.ga[d] * K, nr = (O.gb[d] - O.ga[d]) * K;
    ys.push_back({d, ov[d] + r0, 0, static_cast<double*>(m->ov.p) + r0, (size_t)(nr * 8)});
    ys.push_back({d, of[d] + r0, 0, static_cast<uint8_t*>(m->of.p) + r0, (size_t)nr});
  }
  rc = transfer(m, ys);
  t0 = now_ms();
  if (!rc) rc = md_assemble(m->root, q, 1, G, G * K, m->ov.p, m->of.p, a.data(), out);
  m->t_asm += now_ms() - t0;
  return rc;
}

void drop_side(MultiDev* m) {
  for (tsdbhip_ctx*& s : m->side) {
    if (s) tsdbhip_destroy(s);
    s = nullptr;
  }
  m->side_valid = false;
  m->straddle.clear();
}

// Host batch assembled from resident ranges of the devices (tsdbhip_batch_download_range).
struct HostPieces {
  std::vector<int64_t> srp{0};
  std::vector<uint32_t> base;
  std::vector<uint64_t> qo{0}, vo{0};
  std::vector<uint8_t> q, v;
  std::vector<int32_t> gid;
  int add(tsdbhip_ctx* c, int64_t s0, int64_t s1) {
    if (s1 <= s0) return 0;
    int64_t nr = 0;
    uint64_t qb = 0, vb = 0;
    int rc = tsdbhip_batch_range_sizes(c, s0, s1, &nr, &qb, &vb);
    if (rc) return rc;
    std::vector<int64_t> p(s1 - s0 + 1);
    std::vector<uint32_t> b(std::max<int64_t>(1, nr));
    std::vector<uint64_t> po(nr + 1), pv(nr + 1);
    std::vector<uint8_t> pq(std::max<uint64_t>(1, qb)), pw(std::max<uint64_t>(1, vb));
    std::vector<int32_t> g(s1 - s0);
    rc = tsdbhip_batch_download_range(c, s0, s1, p.data(), b.data(), po.data(), pv.data(), pq.data(), pw.data(), g.data());
    if (rc) return rc;
    const int64_t r0 = (int64_t)base.size();
    const uint64_t q0 = q.size(), v0 = v.size();
    for (int64_t i = 1; i <= s1 - s0; i++) srp.push_back(r0 + p[i]);
    base.insert(base.end(), b.begin(), b.begin() + nr);
    for (int64_t r = 1; r <= nr; r++) {
      qo.push_back(q0 + po[r]);
      vo.push_back(v0 + pv[r]);
    }
    q.insert(q.end(), pq.begin(), pq.begin() + qb);
    v.insert(v.end(), pw.begin(), pw.begin() + vb);
    gid.insert(gid.end(), g.begin(), g.end());
    return 0;
  }
  tsdbhip_batch batch() {
    if (q.empty()) q.push_back(0);
    if (v.empty()) v.push_back(0);
    tsdbhip_batch b{};
    b.n_series = (int64_t)gid.size();
    b.n_rows = (int64_t)base.size();
    b.series_row_ptr = srp.data();
    b.row_base_time = base.empty() ? nullptr : base.data();
    b.row_qual_off = qo.data();
    b.row_val_off = vo.data();
    b.qual = q.data();
    b.val = v.data();
    b.group_id = gid.data();
    return b;
  }
};

// The side contexts of the raw path: every straddling group, whole, on its owner (the first
// device holding one of its spans), its spans in device order = SpanGroup order.
int build_side(MultiDev* m) {
  if (m->side_valid) return 0;
  drop_side(m);
  const int n = (int)m->devices.size();
  const int64_t G = m->G;
  const std::vector<int> ds = live_devices(m);
  std::vector<std::vector<int64_t>> cnt(n);
  for (int d : ds) cnt[d] = ctx_group_counts(m->subs[d], G);
  m->straddle.assign(std::max<int64_t>(1, G), 0);
  std::vector<std::vector<int64_t>> own(n);
  for (int64_t g = 0; g < G; g++) {
    int first = -1, held = 0;
    for (int d : ds)
      if (cnt[d][g] > 0) {
        if (first < 0) first = d;
        held++;
      }
    if (held >= 2) {
      m->straddle[g] = 1;
      own[first].push_back(g);
    }
  }
  m->side.assign(n, nullptr);
  for (int o = 0; o < n; o++) {
    if (own[o].empty()) continue;
    HostPieces h;
    for (int64_t g : own[o])
      for (int d : ds) {
        if (!cnt[d][g]) continue;
        int64_t p0 = 0, p1 = 0;
        ctx_group_range(m->subs[d], g, &p0, &p1);
        const int rc = h.add(m->subs[d], p0, p1);
        if (rc) return rc;
      }
    int rc = tsdbhip_init(m->devices[o], &m->side[o]);
    if (rc) return rc;
    const tsdbhip_batch b = h.batch();
    rc = tsdbhip_load(m->side[o], &b);
    if (rc) return rc;
  }
  m->side_valid = true;
  return 0;
}

// Raw group-by (no downsampler) over SERIES shards: every device answers its whole groups, the
// side contexts answer the straddling ones (AggregationIterator over all of a group's spans,
// :514-797, on one device, so float operands keep SpanGroup order).
int run_raw_series(MultiDev* m, const tsdbhip_query* q, tsdbhip_result** out) {
  int rc = build_side(m);
  if (rc) return rc;
  const int n = (int)m->devices.size();
  std::vector<tsdbhip_result*> parts(2 * n, nullptr);
  std::vector<int> run = live_devices(m);
  for (int d = 0; d < n; d++)
    if (m->side[d] && !m->live[d]) run.push_back(d);
  std::sort(run.begin(), run.end());
  double t0 = now_ms();
  rc = each_of(m, run, [&](int d) {
    int r = m->live[d] ? tsdbhip_run(m->subs[d], q, &parts[d]) : 0;
    if (!r && m->side[d]) r = tsdbhip_run(m->side[d], q, &parts[n + d]);
    return r;
  });
  m->t_dev += now_ms() - t0;
  t0 = now_ms();
  if (!rc) rc = merge(m, parts, false, out, &m->straddle, (size_t)n);
  m->t_asm += now_ms() - t0;
  free_all(parts);
  return rc;
}

int first_live(const MultiDev* m) {
  for (int d = 0; d < (int)m->devices.size(); d++) if (m->live[d]) return d;
  return 0;
}

int run_one(MultiDev* m, const tsdbhip_query* q, tsdbhip_result** out) {
  if (m->mode == TSDB_SHARD_AUTO) return tsdbhip_run(m->root, q, out);   // nothing loaded: as one empty device
  int kind = 0;
  int rc = query_kind(m->subs[first_live(m)], q, &kind);
  if (rc) return rc;
  if (m->mode == TSDB_SHARD_GROUPS || kind == QK_NONE) return run_local(m, q, kind == QK_NONE, out);
  if (kind == QK_RAW) return m->rollup ? run_local(m, q, false, out) : run_raw_series(m, q, out);
  return kind == QK_PARTIALS ? run_partials_owner(m, q, 1, out) : run_sel_xchg(m, q, out);
}

void reset_stages(MultiDev* m) {
  m->t_dev = m->t_xfer = m->t_sel = m->t_asm = 0;
  m->xfer_bytes = 0;
}

// Per-device stage times: maximum over the devices; counters: summed.
void device_timing(MultiDev* m, double wall_ms, bool fused) {
  tsdbhip_timing t{};
  int64_t fq = -1;
  m->dev_timing.assign(m->devices.size(), tsdbhip_timing{});
  for (int d : live_devices(m)) {
    tsdbhip_timing s{};
    if (tsdbhip_last_timing(m->subs[d], &s)) continue;
    m->dev_timing[d] = s;
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
  t.devices_ms = m->t_dev;
  t.xfer_ms = m->t_xfer;
  t.select_ms = m->t_sel;
  t.assemble_ms = m->t_asm;
  t.exchange_ms = m->t_xfer + m->t_sel + m->t_asm;
  m->timing = t;
}

// After a load: devices without series give up what they held before.
void drop_idle(MultiDev* m) {
  for (int d = 0; d < (int)m->devices.size(); d++)
    if (!m->live[d]) ctx_drop_batch(m->subs[d]);
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
  m->rollup = false;
  m->gcnt_valid = false;
  drop_side(m);
  m->live.assign(n, 0);
  bool any = false;
  for (int d = 0; d < n; d++) { m->live[d] = !cand[d].empty(); any = any || m->live[d]; }
  if (!any) m->live[0] = 1;   // an empty batch: device 0 holds it, as one device would
  return cand;
}

int md_load(tsdbhip_ctx* c, const tsdbhip_batch* b) {
  MultiDev* m = md_of(c);
  m->ro_valid = false;
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
  drop_idle(m);
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
  m->ro_valid = false;
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
  drop_idle(m);
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
  m->rollup = true;
  return 0;
}

int md_synth(tsdbhip_ctx* c, const tsdbhip_synth_spec* sp) {
  MultiDev* m = md_of(c);
  m->ro_valid = false;
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
  m->rollup = false;
  m->gcnt_valid = false;
  drop_side(m);
  m->live.assign(n, 0);
  for (int d = 0; d < n; d++) m->live[d] = p[d + 1] > p[d];
  ctx_drop_batch(m->root);
  drop_idle(m);
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


// A compaction scan (tsdbhip_load_cells): the scan's series split as md_load splits a batch (by
// their column bytes), each device compacting its series' rows (copied out of the caller's arrays)
// into its resident shard; compaction exceptions surface lazily from the device holding the row.
int md_load_cells(tsdbhip_ctx* c, const tsdbhip_cell_batch* cb) {
  MultiDev* m = md_of(c);
  m->ro_valid = false;
  const int64_t S = cb->n_series, NR = cb->n_rows, NC = cb->n_cols;
  if (S < 0 || NR < 0 || NC < 0) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "negative sizes");
  if (S > 0 && (!cb->series_row_ptr || !cb->group_id)) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null batch arrays");
  if (NR > 0 && (!cb->row_base_time || !cb->row_col_ptr)) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null batch arrays");
  if (NC > 0 && (!cb->col_qual_off || !cb->col_val_off || !cb->qual || !cb->val))
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null batch arrays");
  if (S > 0 && (cb->series_row_ptr[0] != 0 || cb->series_row_ptr[S] != NR))
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "series_row_ptr does not cover the rows");
  if (NR > 0 && (cb->row_col_ptr[0] != 0 || cb->row_col_ptr[NR] != NC))
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "row_col_ptr does not cover the columns");
  for (int64_t s = 0; s < S; s++)
    if (cb->series_row_ptr[s + 1] < cb->series_row_ptr[s]) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "series_row_ptr not monotonic");
  for (int64_t r = 0; r < NR; r++)
    if (cb->row_col_ptr[r + 1] < cb->row_col_ptr[r]) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "row_col_ptr not monotonic");
  for (int64_t k = 0; k < NC; k++)
    if (cb->col_qual_off[k + 1] < cb->col_qual_off[k] || cb->col_val_off[k + 1] < cb->col_val_off[k])
      return set_error(TSDB_E_ILLEGAL_ARGUMENT, "column offsets not monotonic");
  std::lock_guard<std::mutex> lk(ctx_mutex(c));
  std::vector<double> w(S);
  for (int64_t s = 0; s < S; s++) {
    const int64_t k0 = cb->row_col_ptr[cb->series_row_ptr[s]], k1 = cb->row_col_ptr[cb->series_row_ptr[s + 1]];
    w[s] = (double)(cb->col_qual_off[k1] - cb->col_qual_off[k0]) + (double)(cb->col_val_off[k1] - cb->col_val_off[k0]);
  }
  int mode = 0;
  int64_t G = 0;
  const std::vector<std::vector<int64_t>> cand = shard_series(m, cb->group_id, w, mode, G);
  const int n = (int)m->devices.size();
  struct Sub {
    std::vector<int64_t> srp{0}, rcp{0}, ts;
    std::vector<int32_t> gid;
    std::vector<uint32_t> base;
    std::vector<uint64_t> qo{0}, vo{0};
    std::vector<uint8_t> q, v;
    tsdbhip_cell_batch cb{};
  };
  std::vector<Sub> sub(n);
  for (int d = 0; d < n; d++) {
    Sub& u = sub[d];
    for (int64_t s : cand[d]) {
      for (int64_t r = cb->series_row_ptr[s]; r < cb->series_row_ptr[s + 1]; r++) {
        u.base.push_back(cb->row_base_time[r]);
        for (int64_t k = cb->row_col_ptr[r]; k < cb->row_col_ptr[r + 1]; k++) {
          u.q.insert(u.q.end(), cb->qual + cb->col_qual_off[k], cb->qual + cb->col_qual_off[k + 1]);
          u.v.insert(u.v.end(), cb->val + cb->col_val_off[k], cb->val + cb->col_val_off[k + 1]);
          u.qo.push_back(u.q.size());
          u.vo.push_back(u.v.size());
          if (cb->col_timestamp) u.ts.push_back(cb->col_timestamp[k]);
        }
        u.rcp.push_back((int64_t)u.qo.size() - 1);
      }
      u.srp.push_back((int64_t)u.base.size());
      u.gid.push_back(cb->group_id[s]);
    }
    for (auto* x : {&u.q, &u.v}) if (x->empty()) x->push_back(0);
    if (u.gid.empty()) u.gid.push_back(-1);
    u.cb = *cb;
    u.cb.n_series = (int64_t)cand[d].size();
    u.cb.series_row_ptr = u.srp.data();
    u.cb.n_rows = (int64_t)u.base.size();
    u.cb.row_base_time = u.base.empty() ? nullptr : u.base.data();
    u.cb.row_col_ptr = u.rcp.data();
    u.cb.n_cols = (int64_t)u.qo.size() - 1;
    u.cb.col_qual_off = u.qo.data();
    u.cb.col_val_off = u.vo.data();
    u.cb.col_timestamp = cb->col_timestamp ? (u.ts.empty() ? u.srp.data() : u.ts.data()) : nullptr;
    u.cb.qual = u.q.data();
    u.cb.val = u.v.data();
    u.cb.group_id = u.gid.data();
  }
  ctx_drop_batch(m->root);
  drop_idle(m);
  const int rc = each_device(m, [&](int d) { return tsdbhip_load_cells(m->subs[d], &sub[d].cb); });
  if (rc) {
    m->live.assign(n, 0);
    return rc;
  }
  m->mode = mode;
  m->G = G;
  m->series = cand;
  return 0;
}

// Rollup generation (tsdbhip_rollup_run): every device writes the rollup cells of its series
// (RollupUtils / TSDB.addAggregatePoint's cells, per series -- no exchange); the cells stay on the
// devices until tsdbhip_rollup_download puts them in the one-GPU order (function, batch series,
// time).  The spec checks are the one-GPU entry point's (each device applies them).
int md_rollup_run(tsdbhip_ctx* c, const tsdbhip_rollup_spec* sp, int64_t* n_cells, uint64_t* value_bytes) {
  MultiDev* m = md_of(c);
  if (!sp) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  std::lock_guard<std::mutex> lk(ctx_mutex(c));
  if (m->rollup) return set_error(TSDB_E_NOT_IMPLEMENTED, "tsdbhip_rollup_run over a rollup batch (tsdbhip_load_rollup)");
  const int n = (int)m->devices.size();
  reset_stages(m);
  const double t0 = now_ms();
  m->ro_valid = false;
  std::vector<int64_t> nc(n, 0);
  std::vector<uint64_t> nb(n, 0);
  const int rc = each_device(m, [&](int d) { return tsdbhip_rollup_run(m->subs[d], sp, &nc[d], &nb[d]); });
  m->t_dev += now_ms() - t0;
  if (rc) return rc;
  m->ro_nf = sp->n_funcs;
  m->ro_cells.assign(n, std::vector<int64_t>(4, 0));
  m->ro_bytes.assign(n, std::vector<uint64_t>(4, 0));
  int64_t cells = 0;
  uint64_t bytes = 0;
  for (int d = 0; d < n; d++) {
    if (!m->live[d]) continue;
    const int nf = ctx_rollup_parts(m->subs[d], m->ro_cells[d].data(), m->ro_bytes[d].data());
    if (nf != sp->n_funcs) return set_error(TSDB_E_HIP, "rollup function count differs on a device");
    cells += nc[d];
    bytes += nb[d];
  }
  m->ro_valid = true;
  if (n_cells) *n_cells = cells;
  if (value_bytes) *value_bytes = bytes;
  device_timing(m, now_ms() - t0, false);
  return 0;
}

int md_rollup_download(tsdbhip_ctx* c, int32_t* series, uint32_t* base_time, uint8_t* qualifier, uint64_t* val_off,
                       uint8_t* value) {
  MultiDev* m = md_of(c);
  std::lock_guard<std::mutex> lk(ctx_mutex(c));
  if (!m->ro_valid) return set_error(TSDB_E_ILLEGAL_STATE, "tsdbhip_rollup_download before tsdbhip_rollup_run");
  const int n = (int)m->devices.size();
  struct Part {
    std::vector<int32_t> ser;
    std::vector<uint32_t> base;
    std::vector<uint8_t> qual, val;
    std::vector<uint64_t> voff;
  };
  std::vector<Part> part(n);
  int rc = each_device(m, [&](int d) {
    Part& p = part[d];
    int64_t cells = 0;
    uint64_t bytes = 0;
    for (int i = 0; i < m->ro_nf; i++) { cells += m->ro_cells[d][i]; bytes += m->ro_bytes[d][i]; }
    p.ser.resize(std::max<int64_t>(1, cells));
    p.base.resize(std::max<int64_t>(1, cells));
    p.qual.resize(std::max<int64_t>(1, 3 * cells));
    p.voff.resize(cells + 1);
    p.val.resize(std::max<uint64_t>(1, bytes));
    return tsdbhip_rollup_download(m->subs[d], p.ser.data(), p.base.data(), p.qual.data(), p.voff.data(), p.val.data());
  });
  if (rc) return rc;
  // per function, the devices' runs of one series' cells, in global batch-series order (synth
  // shards and group shards are already in device order; loaded shards interleave batch indices)
  struct Run { int64_t g; int d; int64_t c0, c1; };
  int64_t out_c = 0;
  uint64_t out_b = 0;
  std::vector<int64_t> f0(n, 0);   // first cell of the current function on each device
  for (int i = 0; i < m->ro_nf; i++) {
    std::vector<Run> runs;
    for (int d = 0; d < n; d++) {
      if (!m->live[d]) continue;
      const Part& p = part[d];
      const int64_t a = f0[d], b = a + m->ro_cells[d][i];
      for (int64_t k = a; k < b;) {
        int64_t e = k + 1;
        while (e < b && p.ser[e] == p.ser[k]) e++;
        runs.push_back({batch_index(m, d, p.ser[k]), d, k, e});
        k = e;
      }
      f0[d] = b;
    }
    if (!m->series.empty())
      std::stable_sort(runs.begin(), runs.end(), [](const Run& x, const Run& y) { return x.g < y.g; });
    for (const Run& r : runs) {
      const Part& p = part[r.d];
      const int64_t k = r.c1 - r.c0;
      const uint64_t b0 = p.voff[r.c0], nbytes = p.voff[r.c1] - b0;
      if (series) for (int64_t j = 0; j < k; j++) series[out_c + j] = (int32_t)r.g;
      if (base_time) std::copy(p.base.begin() + r.c0, p.base.begin() + r.c1, base_time + out_c);
      if (qualifier) std::copy(p.qual.begin() + 3 * r.c0, p.qual.begin() + 3 * r.c1, qualifier + 3 * out_c);
      if (val_off) for (int64_t j = 0; j < k; j++) val_off[out_c + j] = out_b + (p.voff[r.c0 + j] - b0);
      if (value && nbytes) std::copy(p.val.begin() + b0, p.val.begin() + b0 + nbytes, value + out_b);
      out_c += k;
      out_b += nbytes;
    }
  }
  if (val_off) val_off[out_c] = out_b;
  return 0;
}

// ---- queries ------------------------------------------------------------------------------
int md_run(tsdbhip_ctx* c, const tsdbhip_query* q, tsdbhip_result** out) {
  MultiDev* m = md_of(c);
  if (!q || !out) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  std::lock_guard<std::mutex> lk(ctx_mutex(c));
  *out = nullptr;
  reset_stages(m);
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
  reset_stages(m);
  int rc = 0;
  bool fused = false;
  if (m->mode == TSDB_SHARD_GROUPS) {
    // whole SpanGroups per device: each device runs its own fused pass over the queries
    const int nd = (int)m->devices.size();
    std::vector<std::vector<tsdbhip_result*>> parts(nd, std::vector<tsdbhip_result*>(n, nullptr));
    double t1 = now_ms();
    rc = each_device(m, [&](int d) { return tsdbhip_run_multi(m->subs[d], qs, n, parts[d].data()); });
    m->t_dev += now_ms() - t1;
    t1 = now_ms();
    for (int i = 0; i < n && !rc; i++) {
      std::vector<tsdbhip_result*> pi(nd, nullptr);
      for (int d = 0; d < nd; d++) pi[d] = parts[d][i];
      rc = merge(m, pi, qs[i].aggregator == TSDB_AGG_NONE, &outs[i]);
    }
    m->t_asm += now_ms() - t1;
    for (auto& p : parts) free_all(p);
    fused = true;
  } else {
    // series shards: queries that all exchange partial states share one fused pass per device
    // (tsdbhip_run_partials_multi) and one owner-routed exchange; any other mix runs one by one
    bool all_partials = m->mode != TSDB_SHARD_AUTO && n > 1;
    for (int i = 0; i < n && all_partials && !rc; i++) {
      int kind = 0;
      rc = query_kind(m->subs[first_live(m)], &qs[i], &kind);
      all_partials = kind == QK_PARTIALS;
    }
    if (!rc && all_partials) {
      rc = run_partials_owner(m, qs, n, outs);
      fused = true;
    } else {
      for (int i = 0; i < n && !rc; i++) rc = run_one(m, &qs[i], &outs[i]);
    }
  }
  if (rc) {
    for (int i = 0; i < n; i++) {
      if (outs[i]) tsdbhip_result_free(outs[i]);
      outs[i] = nullptr;
    }
    return rc;
  }
  device_timing(m, now_ms() - t0, fused);
  return 0;
}

// Histogram spans over the devices: a HistogramSpanGroup is a sum over its
// spans' histograms (HistogramAggregationIterator, src/core/HistogramAggregationIterator.java:
// 91-287) with no cross-group state, so each device holds whole groups -- contiguous runs of
// group ids, balanced by column bytes -- and answers them as one GPU does; an ungrouped span
// (dropped by a group-by, its own group under "none") is a unit of its own.  hist_merge orders
// the devices' groups (or the spans, "none") as one context does and unions the bucket dictionary.
int md_load_histograms(tsdbhip_ctx* c, const tsdbhip_hist_batch* hb) {
  MultiDev* m = md_of(c);
  const int n = (int)m->devices.size();
  m->hist_loaded = false;
  m->hist_devs.clear();
  m->hist_series.assign(n, {});
  const int64_t NS = hb->n_series, NR = hb->n_rows, NC = hb->n_cells;
  if (NS < 0 || NR < 0 || NC < 0 || !hb->series_row_ptr || (NR && (!hb->row_base_time || !hb->row_cell_ptr)) ||
      (NC && (!hb->cell_qual_off || !hb->cell_val_off || !hb->qual || !hb->val)) || (NS && !hb->group_id))
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "malformed histogram batch");
  if (hb->series_row_ptr[0] != 0 || hb->series_row_ptr[NS] != NR || (NR && (hb->row_cell_ptr[0] != 0 || hb->row_cell_ptr[NR] != NC)))
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "histogram batch offsets do not cover the rows / columns");
  for (int64_t s = 0; s < NS; s++)
    if (hb->series_row_ptr[s + 1] < hb->series_row_ptr[s]) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "row offsets not monotonic");
  for (int64_t r = 0; r < NR; r++)
    if (hb->row_cell_ptr[r + 1] < hb->row_cell_ptr[r]) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "column offsets not monotonic");
  for (int64_t k = 0; k < NC; k++)
    if (hb->cell_qual_off[k + 1] < hb->cell_qual_off[k] || hb->cell_val_off[k + 1] < hb->cell_val_off[k])
      return set_error(TSDB_E_ILLEGAL_ARGUMENT, "column byte offsets not monotonic");
  // units: a group's spans, or one ungrouped span; in group-id order, ungrouped spans after
  std::vector<int64_t> order(NS);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
    const int32_t ga = hb->group_id[a], gb = hb->group_id[b];
    if ((ga < 0) != (gb < 0)) return gb < 0;
    return ga >= 0 && ga < gb;
  });
  auto sbytes = [&](int64_t s) {
    const int64_t c0 = hb->row_cell_ptr[hb->series_row_ptr[s]], c1 = hb->row_cell_ptr[hb->series_row_ptr[s + 1]];
    return (double)(hb->cell_val_off[c1] - hb->cell_val_off[c0] + hb->cell_qual_off[c1] - hb->cell_qual_off[c0]) + 1.0;
  };
  double total = 0;
  for (int64_t s = 0; s < NS; s++) total += sbytes(s);
  std::vector<int> dev_of(NS, 0);
  {
    double acc = 0;
    int d = 0;
    for (int64_t i = 0; i < NS;) {
      int64_t j = i + 1;   // the unit [i, j)
      const int32_t g = hb->group_id[order[i]];
      if (g >= 0)
        while (j < NS && hb->group_id[order[j]] == g) j++;
      double ub = 0;
      for (int64_t k = i; k < j; k++) ub += sbytes(order[k]);
      while (d < n - 1 && acc + ub / 2 > total * (d + 1) / n) d++;   // the unit's midpoint picks the device
      for (int64_t k = i; k < j; k++) dev_of[order[k]] = d;
      acc += ub;
      i = j;
    }
  }
  for (int64_t s = 0; s < NS; s++) m->hist_series[dev_of[s]].push_back(s);   // batch order on each device
  for (int d = 0; d < n; d++)
    if (!m->hist_series[d].empty() || (NS == 0 && d == 0)) m->hist_devs.push_back(d);
  // each device's sub-batch (the same codec table, group ids kept)
  struct Sub {
    std::vector<int64_t> srp{0}, rcp{0};
    std::vector<uint32_t> base;
    std::vector<uint64_t> qo{0}, vo{0};
    std::vector<uint8_t> q, v;
    std::vector<int32_t> gid;
  };
  std::vector<Sub> subs(n);
  for (int d : m->hist_devs) {
    Sub& u = subs[d];
    for (int64_t s : m->hist_series[d]) {
      for (int64_t r = hb->series_row_ptr[s]; r < hb->series_row_ptr[s + 1]; r++) {
        u.base.push_back(hb->row_base_time[r]);
        for (int64_t k = hb->row_cell_ptr[r]; k < hb->row_cell_ptr[r + 1]; k++) {
          u.q.insert(u.q.end(), hb->qual + hb->cell_qual_off[k], hb->qual + hb->cell_qual_off[k + 1]);
          u.v.insert(u.v.end(), hb->val + hb->cell_val_off[k], hb->val + hb->cell_val_off[k + 1]);
          u.qo.push_back(u.q.size());
          u.vo.push_back(u.v.size());
        }
        u.rcp.push_back((int64_t)u.qo.size() - 1);
      }
      u.srp.push_back((int64_t)u.base.size());
      u.gid.push_back(hb->group_id[s]);
    }
  }
  const int rc = each_of(m, m->hist_devs, [&](int d) {
    const Sub& u = subs[d];
    tsdbhip_hist_batch sb{};
    sb.n_series = (int64_t)u.gid.size();
    sb.series_row_ptr = u.srp.data();
    sb.n_rows = (int64_t)u.base.size();
    sb.row_base_time = u.base.data();
    sb.row_cell_ptr = u.rcp.data();
    sb.n_cells = (int64_t)u.qo.size() - 1;
    sb.cell_qual_off = u.qo.data();
    sb.cell_val_off = u.vo.data();
    sb.qual = u.q.data();
    sb.val = u.v.data();
    sb.group_id = u.gid.data();
    std::memcpy(sb.codec, hb->codec, sizeof(sb.codec));
    return tsdbhip_load_histograms(m->subs[d], &sb);
  });
  if (rc) return rc;
  m->hist_loaded = true;
  return 0;
}

int md_hist_run(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t start, int64_t end, int64_t ss, int64_t se, int n_pct,
                const float* pct, int show_buckets, tsdbhip_hist_result** out) {
  MultiDev* m = md_of(c);
  if (!m->hist_loaded) return set_error(TSDB_E_ILLEGAL_STATE, "no histogram store loaded (tsdbhip_load_histograms)");
  const int n = (int)m->devices.size();
  std::vector<tsdbhip_hist_result*> parts(n, nullptr);
  int rc = each_of(m, m->hist_devs, [&](int d) {
    return hist_run(m->subs[d], q, start, end, ss, se, n_pct, pct, show_buckets, &parts[d]);
  });
  if (!rc) {
    std::vector<tsdbhip_hist_result*> ps;
    std::vector<const std::vector<int64_t>*> span_of;
    for (int d : m->hist_devs) {
      ps.push_back(parts[d]);
      span_of.push_back(&m->hist_series[d]);
    }
    rc = hist_merge(ps, span_of, q->aggregator == TSDB_AGG_NONE, out);
  }
  for (tsdbhip_hist_result* p : parts) tsdbhip_hist_result_free(p);
  return rc;
}

int md_timing(tsdbhip_ctx* c, tsdbhip_timing* out) {
  if (!out) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  *out = md_of(c)->timing;
  return 0;
}

int md_sync(tsdbhip_ctx* c) {
  MultiDev* m = md_of(c);
  std::lock_guard<std::mutex> lk(ctx_mutex(c));
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
  delete m->pool;
  m->pool = nullptr;
  drop_side(m);
  for (ncclComm_t cm : m->comms) if (cm) (void)rccl().destroy(cm);
  for (auto* v : {&m->xb, &m->mb, &m->dv, &m->df, &m->da})
    for (Buf& b : *v) b.release();
  m->ov.release();
  m->of.release();
  m->oa.release();
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
      return set_error(TSDB_E_HIP, "no such HIP device " + std::to_string(devices[d]) + " (" +
                                       std::to_string(count) + " visible)");
  const bool distinct = std::set<int>(devices, devices + n_devices).size() == (size_t)n_devices;
  if (transport == TSDB_MD_RCCL && !distinct)
    return set_error(TSDB_E_ILLEGAL_ARGUMENT, "RCCL needs distinct devices (one rank per GPU)");
  int tr = transport;
  if (tr == TSDB_MD_AUTO) tr = distinct && n_devices > 1 && rccl().ok ? TSDB_MD_RCCL : TSDB_MD_COPY;
  if (tr == TSDB_MD_RCCL && !rccl().ok) return set_error(TSDB_E_HIP, "RCCL unavailable: " + rccl().why);
  tsdbhip_ctx* c = nullptr;
  int rc = tsdbhip_init(devices[0], &c);
  if (rc) return rc;
  auto* m = new MultiDev();
  ctx_md(c) = m;   // tsdbhip_destroy(c) releases it from here on
  m->devices.assign(devices, devices + n_devices);
  m->transport = tr;
  m->live.assign(n_devices, 0);
  m->pool = new Workers(n_devices);
  for (int d = 0; d < n_devices && !rc; d++) {
    tsdbhip_ctx* s = nullptr;
    rc = tsdbhip_init(devices[d], &s);
    if (!rc) {
      ctx_set_none_orig(s, true);
      m->subs.push_back(s);
      for (auto* v : {&m->xb, &m->mb, &m->dv, &m->df, &m->da}) v->push_back(Buf{devices[d]});
    }
  }
  if (!rc) rc = tsdbhip_init(devices[0], &m->root);
  m->ov.dev = m->of.dev = m->oa.dev = devices[0];
  // direct peer access between distinct devices (xGMI): peer copies and RCCL's P2P path use it
  if (!rc && distinct)
    for (int a = 0; a < n_devices; a++)
      for (int b = 0; b < n_devices; b++) {
        int can = 0;
        if (a == b || hipDeviceCanAccessPeer(&can, devices[a], devices[b]) != hipSuccess || !can) continue;
        (void)hipSetDevice(devices[a]);
        const hipError_t e = hipDeviceEnablePeerAccess(devices[b], 0);
        if (e != hipSuccess) (void)hipGetLastError();   // (already enabled by someone else: fine)
      }
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

extern "C" int tsdbhip_device_count(int* n) {
  if (!n) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "null argument");
  *n = 0;
  MOK(hipGetDeviceCount(n));
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
        shard_series[d] = ctx_n_series(m->subs[d]);
      }
    }
  }
  return 0;
}

extern "C" int tsdbhip_md_stats(tsdbhip_ctx* c, tsdbhip_timing* per_device, int* rccl_ranks, double* xfer_bytes) {
  if (!c || !md_of(c)) return set_error(TSDB_E_ILLEGAL_ARGUMENT, "not a multi-device context (tsdbhip_init_devices)");
  MultiDev* m = md_of(c);
  std::lock_guard<std::mutex> lk(ctx_mutex(c));
  if (per_device)
    for (size_t d = 0; d < m->devices.size(); d++)
      per_device[d] = d < m->dev_timing.size() ? m->dev_timing[d] : tsdbhip_timing{};
  if (rccl_ranks) {
    *rccl_ranks = 0;
    if (!m->comms.empty() && m->comms[0]) {
      int k = 0;
      const ncclResult_t e = rccl().count(m->comms[0], &k);
      if (e != ncclSuccess) return rccl_fail(e, "ncclCommCount");
      *rccl_ranks = k;
    }
  }
  if (xfer_bytes) *xfer_bytes = m->xfer_bytes;
  return 0;
}
