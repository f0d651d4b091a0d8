// Multi-device context (multi.cpp) <-> engine.cpp: the engine entry points hand a context made by
// tsdbhip_init_devices to these; multi.cpp drives its per-device contexts through the public API
// plus the few hooks below.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/tsdbhip.h"

namespace tsdb {
// engine.cpp
void*& ctx_md(tsdbhip_ctx* c);                     // the MultiDev of a multi-device context (or null)
void ctx_set_none_orig(tsdbhip_ctx* c, bool on);   // NONE results keyed by batch position, not renumbered
int load_series(tsdbhip_ctx* c, const tsdbhip_batch* b, const std::vector<int64_t>& series);
enum { QK_PARTIALS = 0, QK_SEL = 1, QK_RAW = 2, QK_NONE = 3 };
int query_kind(tsdbhip_ctx* c, const tsdbhip_query* q, int* kind);   // plan_query's verdict
int set_error(int code, const std::string& msg);
tsdbhip_result* new_result(int64_t n_groups, int64_t n_points);
void ctx_drop_batch(tsdbhip_ctx* c);               // release the resident batch (and rollup state)
int64_t ctx_n_series(tsdbhip_ctx* c);              // resident series, a rollup batch's count series too
int ctx_rollup_parts(tsdbhip_ctx* c, int64_t* cells, uint64_t* bytes);   // last rollup_run per function
std::vector<int64_t> ctx_group_counts(tsdbhip_ctx* c, int64_t G);   // resident series of each group id < G
void ctx_group_range(tsdbhip_ctx* c, int64_t g, int64_t* p0, int64_t* p1);   // resident positions of group g
// owner-routed percentile / ordered exchange: span contributions left on the device (room for
// extra_rows more rows), then the owner's selection over rows on its device
int md_sel_values(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t G, int64_t extra_rows, double** vals,
                  int64_t* K, uint8_t* uni, uint32_t* act);
int md_sel_select(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t G, const double* vals, const int64_t* counts,
                  const uint8_t* uni, double** out_val, uint8_t** out_flag);
// owner-routed partials (decomposable group-by over series shards): a partials buffer's part
// offsets, and the owner's fold of a straddling group + finalisation of its groups
// a straddling group's K-slot state as one device sends it to the owner:
// [a K f64 | b K f64 | n K u32 | f K u32 | act u32], 16-byte aligned
inline int64_t mini_state_stride(int64_t K) { return ((K * 24 + 4) + 15) & ~(int64_t)15; }
void partials_offsets(int64_t G, int64_t K, int64_t* off_b, int64_t* off_n, int64_t* off_f, int64_t* off_act,
                      int64_t* bytes);
int md_partials_finish(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t G, unsigned char* state, int64_t g_fold,
                       const unsigned char* mini, int n_mini, double* out_val, uint8_t* out_flag, uint32_t* out_act);
// nq queries' dense rows on the context's device (query i at i * stride values) -> nq results with
// one copy per array and one synchronisation
int md_assemble(tsdbhip_ctx* c, const tsdbhip_query* qs, int nq, int64_t G, int64_t stride, const void* val,
                const void* flag, const void* act, tsdbhip_result** outs);
// hist.cpp: one context's histogram query, and the devices' results merged into one
int hist_run(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t start, int64_t end, int64_t ss, int64_t se, int n_pct,
             const float* pct, int show_buckets, tsdbhip_hist_result** out);
int hist_merge(const std::vector<tsdbhip_hist_result*>& parts, const std::vector<const std::vector<int64_t>*>& span_of,
               bool none, tsdbhip_hist_result** out);
// multi.cpp
int md_load_histograms(tsdbhip_ctx* c, const tsdbhip_hist_batch* hb);
int md_hist_run(tsdbhip_ctx* c, const tsdbhip_query* q, int64_t start, int64_t end, int64_t ss, int64_t se, int n_pct,
                const float* pct, int show_buckets, tsdbhip_hist_result** out);
int md_load(tsdbhip_ctx* c, const tsdbhip_batch* b);
int md_synth(tsdbhip_ctx* c, const tsdbhip_synth_spec* sp);
int md_load_rollup(tsdbhip_ctx* c, const tsdbhip_rollup_batch* rb);
int md_load_cells(tsdbhip_ctx* c, const tsdbhip_cell_batch* cb);
int md_rollup_run(tsdbhip_ctx* c, const tsdbhip_rollup_spec* sp, int64_t* n_cells, uint64_t* value_bytes);
int md_rollup_download(tsdbhip_ctx* c, int32_t* series, uint32_t* base_time, uint8_t* qualifier, uint64_t* val_off,
                       uint8_t* value);
int md_run(tsdbhip_ctx* c, const tsdbhip_query* q, tsdbhip_result** out);
int md_run_multi(tsdbhip_ctx* c, const tsdbhip_query* qs, int n, tsdbhip_result** outs);
int md_timing(tsdbhip_ctx* c, tsdbhip_timing* out);
int md_sync(tsdbhip_ctx* c);
int md_batch_sizes(tsdbhip_ctx* c, int64_t* n_series, int64_t* n_rows, uint64_t* qual_bytes, uint64_t* val_bytes);
void md_destroy(void* md);
}  // namespace tsdb
