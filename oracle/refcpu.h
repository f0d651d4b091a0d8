/*
 * refcpu.h -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference
 * OpenTSDB 2.4 query-aggregation path, used as the parity oracle and as the CPU
 * baseline ("port").  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product (libtsdbhip) never links or calls it.
 *
 * The functions mirror the reference's iterator objects one for one so that the
 * reference's own unit tests (SeekableViewsForTest-driven) can be replayed:
 *   ref_view_array        <-> SeekableViewsForTest.MockSeekableView / DataPointGenerator
 *   ref_view_span         <-> Span.Iterator over RowSeq compacted cells
 *   ref_view_downsampler  <-> Downsampler / FillingDownsampler (Span.downsampler)
 *   ref_view_rate         <-> RateSpan
 *   ref_view_aggregate    <-> AggregationIterator
 *   ref_run_query         <-> TsdbQuery.run() from GroupByAndAggregateCB through
 *                             SpanGroup.iterator() for every group
 */
#ifndef REFCPU_H
#define REFCPU_H
#include <stdint.h>
#include "../include/tsdbhip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ref_view ref_view;

typedef struct {
  int64_t ts;
  int32_t is_int;
  int32_t bad;        /* nonzero: reading the value throws this TSDB_E_* code (lazy Java semantics) */
  int64_t lv;         /* longValue() when is_int */
  double dv;          /* doubleValue() when !is_int */
  int64_t cnt;        /* RollupSeq valueCount() (rollup spans; 1 without count cells) */
  int32_t cnt_bad;    /* nonzero: valueCount() throws this TSDB_E_* code */
  int32_t pad_;
} ref_dp;

const char* ref_last_error(void);

/* Views.  Every constructor returns NULL on error (ref_last_error()). */
ref_view* ref_view_array(const int64_t* ts, const int32_t* is_int, const int64_t* bits, int64_t n,
                         int generator_seek);
ref_view* ref_view_span(int64_t n_rows, const uint32_t* base_time, const uint64_t* qual_off,
                        const uint64_t* val_off, const uint8_t* qual, const uint8_t* val);
ref_view* ref_view_downsampler(ref_view* src, int32_t function, int64_t interval_ms, int32_t fill,
                               int32_t run_all, int64_t start_time, int64_t end_time,
                               int64_t query_start, int64_t query_end, int32_t calendar);
/* the same in a time zone (DownsamplingSpecification.setTimezone; NULL = UTC) */
ref_view* ref_view_downsampler_tz(ref_view* src, int32_t function, int64_t interval_ms, int32_t fill,
                                  int32_t run_all, int64_t start_time, int64_t end_time,
                                  int64_t query_start, int64_t query_end, int32_t calendar, const tsdbhip_tz* tz);
ref_view* ref_view_rate(ref_view* src, int32_t counter, int64_t counter_max, int64_t reset_value,
                        int32_t drop_resets);
ref_view* ref_view_aggregate(ref_view** srcs, int64_t n, int64_t start_time, int64_t end_time,
                             int32_t aggregator, int32_t interpolation, int32_t rate);
void ref_view_free(ref_view* v);

/* Iteration: 1/0 on success, <0 on exception. */
int ref_has_next(ref_view* v);
/* Drains v: writes up to cap points (ts, is_int, value bits).  Returns count or <0. */
int64_t ref_drain(ref_view* v, int64_t cap, int64_t* ts, int32_t* is_int, uint64_t* bits);
int ref_seek(ref_view* v, int64_t ts);

/* Aggregator.runLong / runDouble over a plain array (TestAggregators' Numbers). */
int ref_agg_run_long(int32_t aggregator, const int64_t* v, int64_t n, int64_t* out);
int ref_agg_run_double(int32_t aggregator, const double* v, int64_t n, double* out);

/* Host logic restatements (same contract as the tsdbhip_* helpers). */
int ref_parse_duration(const char* s, int64_t* out_ms);
int ref_parse_downsample(const char* spec, tsdbhip_query* q);
int ref_aggregator_get(const char* name);
int ref_scan_bounds(const tsdbhip_query* q, int64_t* s, int64_t* e);

/* End-to-end query (TsdbQuery.run). Result arrays are malloc'd; free with ref_result_free. */
typedef struct {
  int64_t n_groups;
  int32_t* group_id;
  int64_t* group_ptr;
  int64_t* ts_ms;
  uint64_t* value_bits;
  uint8_t* is_int;
  int64_t n_points;
} ref_result;
int ref_run_query(const tsdbhip_batch* b, const tsdbhip_query* q, ref_result** out);
/* Same, but groups processed by nthreads std threads (CPU baseline "parallel over groups"). */
int ref_run_query_mt(const tsdbhip_batch* b, const tsdbhip_query* q, int nthreads, ref_result** out);
void ref_result_free(ref_result* r);
/* TsdbQuery.run over a rollup table (RollupSpan / RollupSeq spans, the Downsampler's rollup
 * branches, rollup scan bounds); layout as tsdbhip_load_rollup. */
int ref_run_rollup_query(const tsdbhip_rollup_batch* rb, const tsdbhip_query* q, ref_result** out);
/* Compaction.compact() of one row's columns (query-time, no write-back): 1 + the compacted
 * cell (free both with ref_free), 0 = no datapoint, < 0 = TSDB_E_* */
int ref_compact_row(int64_t ncols, const uint8_t* const* quals, const int64_t* qlens, const uint8_t* const* vals,
                    const int64_t* vlens, const int64_t* col_ts, int fix_duplicates, int dtcs, uint8_t** out_q,
                    int64_t* out_qlen, uint8_t** out_v, int64_t* out_vlen);
void ref_free(void* p);
/* ---- histogram path (refhist.c) ----------------------------------
 * TsdbQuery.runHistogram over a tsdbhip_hist_batch: SaltScanner's histogram decode,
 * HistogramSpan / HistogramRowSeq, HistogramDownsampler, HistogramAggregationIterator,
 * SimpleHistogram and the two DataPoints adaptors.  Per emitted group: its points (ts), the
 * percentile series values pct[point * n_pct + j], and its bucket series (the first point's
 * getHistogramBucketsIfHas keys: type 0 underflow / 1 regular / 2 overflow, float bits) with
 * one long per point each: bk_val[bk_val_off[g] + series * n_points_g + i]. */
typedef struct {
  int64_t n_groups;
  int32_t* group_id;
  int64_t* group_ptr;
  int64_t* ts;
  int32_t n_pct;
  double* pct;
  int64_t* bk_ptr;        /* [n_groups + 1] bucket series of each group */
  int32_t* bk_type;
  uint32_t* bk_lo;
  uint32_t* bk_up;
  int64_t* bk_val_off;    /* [n_groups + 1] */
  int64_t* bk_val;
} ref_hist_result;
int ref_run_hist(const tsdbhip_hist_batch* hb, const tsdbhip_query* q, int n_pct, const float* pct,
                 int show_buckets, ref_hist_result** out);
/* HistogramAggregationIterator.create(spans, start_ms, end_ms, ...) over every row of the batch
 * (the reference's iterator-level tests; query start / end feed "all" only) */
int ref_run_hist_range(const tsdbhip_hist_batch* hb, const tsdbhip_query* q, int64_t start_ms, int64_t end_ms,
                       int n_pct, const float* pct, int show_buckets, ref_hist_result** out);
void ref_hist_result_free(ref_hist_result* r);
/* SimpleHistogram.percentile / the long codec's percentile of one decoded column value
 * (with the codec id byte); -1 = the column does not decode (it would be dropped). */
int ref_hist_value_percentile(const uint8_t* v, int64_t n, int kind, double p, double* out);
/* Calendar helpers of refcpu.c for refhist.c: DateTime.previousInterval and one Downsampler
 * calendar step (weeks: interval * 7 days); 0 or a TSDB_E_* code. */
int ref_cal_prev_ex(int64_t ts, int64_t n, int unit, const tsdbhip_tz* z, int64_t* out);
int ref_cal_step_ex(int64_t ts, int unit, int64_t n, const tsdbhip_tz* z, int64_t* out);

int ref_rollup_scan_bounds(const tsdbhip_query* q, const tsdbhip_rollup_interval* iv, int64_t* s_out, int64_t* e_out);

#ifdef __cplusplus
}
#endif
#endif
