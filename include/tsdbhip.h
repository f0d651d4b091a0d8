/*
 * tsdbhip.h -- C ABI of libtsdbhip, the MI355X (gfx950) engine for OpenTSDB's
 * query-time aggregation path.
 *
 * Drop-in boundary.  In the reference the path starts where storage I/O ends:
 *   TsdbQuery.GroupByAndAggregateCB.call(SortedMap<byte[],Span>) -> DataPoints[]
 *   (reference src/core/TsdbQuery.java:916-1049)
 * and is evaluated lazily by SpanGroup.iterator() -> AggregationIterator.create
 *   (src/core/SpanGroup.java:527-532, src/core/AggregationIterator.java:351-380).
 * The Java host keeps TsdbQuery/TSQuery, Aggregators.get, DownsamplingSpecification
 * and RateOptions unchanged; a GpuGroupByAndAggregateCB flattens
 * the scanned Spans into a tsdbhip_batch, calls tsdbhip_run and wraps the
 * tsdbhip_result arrays as DataPoints.
 *
 * Everything crossing this boundary is plain C: pointers, sizes, enums.  No torch,
 * no HIP types.  Functions return 0 on success or a negative TSDB_E_* code that maps
 * 1:1 to the Java exception the reference would throw; tsdbhip_last_error() gives the
 * message (thread-local).
 */
#ifndef TSDBHIP_H
#define TSDBHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TSDBHIP_ABI_VERSION 12

/* ---- error codes: one per Java exception on the path --------------------- */
enum {
  TSDB_OK = 0,
  TSDB_E_ILLEGAL_DATA = -2,      /* IllegalDataException  (src/core/RowSeq.java:242-265, Internal.java:307-321) */
  TSDB_E_ILLEGAL_ARGUMENT = -3,  /* IllegalArgumentException (DownsamplingSpecification.java:84-185, DateTime.java:186-226) */
  TSDB_E_ILLEGAL_STATE = -4,     /* IllegalStateException (AggregationIterator.java:640-643, RateSpan.java:129-134) */
  TSDB_E_UNSUPPORTED = -5,       /* UnsupportedOperationException (Downsampler.java:208-211) */
  TSDB_E_RUNTIME = -6,           /* RuntimeException "unhandled fill policy" (FillingDownsampler.java:273-274) */
  TSDB_E_NO_SUCH_ELEMENT = -7,   /* NoSuchElementException (Aggregators.get, iterators) */
  TSDB_E_ASSERTION = -8,         /* AssertionError (AggregationIterator.java:701-703,769-771) */
  TSDB_E_CLASS_CAST = -9,        /* ClassCastException */
  TSDB_E_NULL_POINTER = -10,     /* NullPointerException (a histogram downsampling function other than sum,
                                    DownsamplingSpecification.java:153-157 -> SimpleHistogramDataPointAdapter
                                    .mapAggregation) */
  TSDB_E_HIP = -20,              /* device/runtime failure (no reference counterpart) */
  TSDB_E_NOMEM = -21,
  TSDB_E_NOT_IMPLEMENTED = -22   /* valid reference query this engine does not run yet */
};

/* ---- Aggregators (src/core/Aggregators.java:47-203) ----------------------- */
enum {
  TSDB_AGG_SUM = 0, TSDB_AGG_PFSUM, TSDB_AGG_MIN, TSDB_AGG_MAX, TSDB_AGG_AVG,
  TSDB_AGG_MEDIAN, TSDB_AGG_NONE, TSDB_AGG_MULT, TSDB_AGG_DEV, TSDB_AGG_DIFF,
  TSDB_AGG_ZIMSUM, TSDB_AGG_MIMMIN, TSDB_AGG_MIMMAX, TSDB_AGG_SQUARESUM,
  TSDB_AGG_COUNT, TSDB_AGG_FIRST, TSDB_AGG_LAST,
  /* PercentileAgg (Aggregators.java:125-173), LEGACY estimation */
  TSDB_AGG_P999, TSDB_AGG_P99, TSDB_AGG_P95, TSDB_AGG_P90, TSDB_AGG_P75, TSDB_AGG_P50,
  /* R_3 estimation */
  TSDB_AGG_EP999R3, TSDB_AGG_EP99R3, TSDB_AGG_EP95R3, TSDB_AGG_EP90R3, TSDB_AGG_EP75R3, TSDB_AGG_EP50R3,
  /* R_7 estimation */
  TSDB_AGG_EP999R7, TSDB_AGG_EP99R7, TSDB_AGG_EP95R7, TSDB_AGG_EP90R7, TSDB_AGG_EP75R7, TSDB_AGG_EP50R7,
  TSDB_AGG_COUNT_ALL
};

/* Aggregators.Interpolation (src/core/Aggregators.java:38-44) */
enum { TSDB_INTERP_LERP = 0, TSDB_INTERP_ZIM, TSDB_INTERP_MAX, TSDB_INTERP_MIN, TSDB_INTERP_PREV };

/* FillPolicy (src/core/FillPolicy.java:22-28) */
enum { TSDB_FILL_NONE = 0, TSDB_FILL_ZERO, TSDB_FILL_NAN, TSDB_FILL_NULL, TSDB_FILL_SCALAR };

/* ---- Batch: the Spans found by TsdbQuery.findSpans, flattened to CSR ------
 * Series s owns rows [series_row_ptr[s], series_row_ptr[s+1]) sorted by base time
 * (Span.checkRowOrder, src/core/Span.java:387-392).  Row r is one compacted cell
 * (RowSeq, src/core/RowSeq.java:39-77): its qualifier bytes are
 * qual[row_qual_off[r] .. row_qual_off[r+1]) and its value bytes (including the
 * trailing meta byte written by CompactionQueue, src/core/CompactionQueue.java:594-612)
 * are val[row_val_off[r] .. row_val_off[r+1]).  Everything big-endian, byte-identical
 * to the HBase cells.  group_id[s] is the dense index of the series' SpanGroup in
 * ByteMap key order (TsdbQuery.java:987-1043); series are given in SpanCmp order.
 */
typedef struct {
  int64_t n_series;
  const int64_t* series_row_ptr;   /* [n_series + 1] */
  int64_t n_rows;
  const uint32_t* row_base_time;   /* [n_rows]   seconds (row key bytes, Internal.baseTime) */
  const uint64_t* row_qual_off;    /* [n_rows + 1] */
  const uint64_t* row_val_off;     /* [n_rows + 1] */
  const uint8_t* qual;             /* [row_qual_off[n_rows]] */
  const uint8_t* val;              /* [row_val_off[n_rows]] */
  const int32_t* group_id;         /* [n_series]; -1: no matching group-by tag -- dropped by group-by
                                      aggregators, still emitted by NONE (TsdbQuery.java:940-961) */
} tsdbhip_batch;

/* ---- Time zone of a calendar downsampling --------------------------------
 * DownsamplingSpecification.setTimezone (src/core/DownsamplingSpecification.java:199-207):
 * the zone's UTC offset history as a transition table that the host builds from its own
 * time-zone database (a JVM host: ZoneId.of(id).getRules() -- getTransitions(), plus
 * getTransitionRules() expanded over the query range), so that the engine reproduces
 * java.util.GregorianCalendar's arithmetic in that zone (ZoneInfo.getOffsets by UTC time,
 * getOffsetsByWall for local fields).  offset_ms[0] holds before utc_ms[0] and offset_ms[i + 1]
 * from utc_ms[i] on; the table must cover the query's time range.  The engine reads it during
 * tsdbhip_run only. */
typedef struct {
  int32_t n;                   /* transitions */
  const int64_t* utc_ms;       /* [n] ascending instants */
  const int32_t* offset_ms;    /* [n + 1] total offset (raw + DST), ms east of UTC */
} tsdbhip_tz;

/* ---- Query: TsdbQuery state that reaches the aggregation path ------------- */
typedef struct {
  int64_t start_time;        /* TsdbQuery.setStartTime: unix seconds or ms (TsdbQuery.java:262-289) */
  int64_t end_time;          /* TsdbQuery.setEndTime */
  int32_t aggregator;        /* TSDB_AGG_*: group-by aggregator */
  /* DownsamplingSpecification (src/core/DownsamplingSpecification.java:25-191) */
  int32_t ds_function;       /* TSDB_AGG_* or -1 for NO_DOWNSAMPLER */
  int32_t ds_fill;           /* TSDB_FILL_* */
  int32_t ds_all;            /* "0all-..." : one bucket over [query start, query end) */
  int32_t ds_calendar;       /* 'c' suffix: TSDB_CAL_* unit of the interval (0 = epoch-aligned); UTC */
  int64_t ds_interval_ms;
  /* RateOptions (src/core/RateOptions.java:27-97) */
  int32_t rate;
  int32_t rate_counter;
  int32_t rate_drop_resets;
  int32_t flags;             /* TSDB_QF_* */
  int64_t rate_counter_max;  /* default Long.MAX_VALUE */
  int64_t rate_reset_value;  /* default 0 */
  const tsdbhip_tz* ds_tz;   /* calendar time zone; NULL = UTC (the DownsamplingSpecification default) */
} tsdbhip_query;

/* Calendar units of a 'c' downsampling interval (DateTime.unitsToCalendarType,
 * src/utils/DateTime.java:616-640); the interval count is ds_interval_ms / the unit's
 * parseDuration length (ms 1, s 1e3, m 6e4, h 3.6e6, d 8.64e7, w 6.048e8, n 30 d, y 365 d).
 * The calendar is the query's zone (ds_tz; UTC when NULL, the DownsamplingSpecification
 * default).  UTC intervals whose grid is one global sequence -- ms (1000 % n == 0), s / m
 * (60 % n == 0), h (24 % n == 0), d (n == 1), w (n == 1, weeks from Sunday) -- run on a fixed
 * grid, n months (12 % n == 0) and 1 year on a slot boundary table.  Everything else (a time
 * zone, or an interval anchored per span: 7sc, 2dc, 5nc, 2wc, 3wc, 2yc ...) runs on the union
 * of the spans' boundary sequences, each anchored at previousInterval(the span's first
 * datapoint after the seek).  Spans whose sequences disagree run per anchor and aggregate over
 * the union of their timestamps; percentile / median downsampling runs over boundary tables as
 * well.  Refused (TSDB_E_NOT_IMPLEMENTED): the per-rank exchange entry points
 * (tsdbhip_run_partials / tsdbhip_sel_*) when the anchored grids disagree across ranks -- shard
 * such queries by group. */
enum {
  TSDB_CAL_NONE = 0, TSDB_CAL_MS, TSDB_CAL_S, TSDB_CAL_M, TSDB_CAL_H, TSDB_CAL_D, TSDB_CAL_W, TSDB_CAL_N, TSDB_CAL_Y
};

/* Query flags. */
#define TSDB_QF_ORDERED 0x1  /* cross-series float reductions in SpanGroup index order (bit-exact, slower;
                                across ranks through the tsdbhip_sel_* exchange, not run_partials) */

/* ---- Result: DataPoints[] (one entry per SpanGroup, in emission order) ----- */
typedef struct {
  int64_t n_groups;
  const int32_t* group_id;     /* [n_groups] batch group id of each emitted SpanGroup (-1..: raw span index for NONE) */
  const int64_t* group_ptr;    /* [n_groups + 1] point range of each group */
  const int64_t* ts_ms;        /* [n_points] DataPoint.timestamp() */
  const uint64_t* value_bits;  /* [n_points] longValue() or Double.doubleToRawLongBits(doubleValue()) */
  const uint8_t* is_int;       /* [n_points] DataPoint.isInteger() */
} tsdbhip_result;

/* Per-stage device timing of the last tsdbhip_run (hipEvents on the engine stream). */
typedef struct {
  double decode_downsample_ms;   /* fused decode + downsample + per-tile group partials */
  double group_reduce_ms;        /* cross-tile group reduction + emission */
  double total_ms;
  int64_t datapoints;            /* raw datapoints decoded */
  int64_t bytes;                 /* algorithmic HBM bytes: per row q+v+4+16, per series 4 */
  int64_t tiles;                 /* series tiles of the query */
  int64_t redo_tiles;            /* tiles the streaming kernel handed to the general kernel */
  double fast_ms;                /* streaming kernel (k_fast) alone; 0 when not used */
  double index_ms;               /* k_index of the last tsdbhip_load / tsdbhip_synth: row classification,
                                    validation, certificate stats (+ the int16 value copy of vle rows) */
  double compact_ms;             /* device compaction of the last tsdbhip_load_cells (k_compact pipeline) */
  int64_t fused_queries;         /* queries the last tsdbhip_run_multi answered from ONE fused streaming pass
                                    (0: separate passes, or not a run_multi) */
  double exchange_ms;            /* multi-device context: xfer_ms + select_ms + assemble_ms (host wall time) */
  /* multi-device context, host wall time of the call's stages (they sum to total_ms up to bookkeeping):
   * devices_ms   every device's own pass over its shard (in parallel; per-device kernel times in
   *              tsdbhip_md_stats), partial states / span values left on the devices;
   * xfer_ms      device-to-device moves (transfer(): RCCL send / recv or peer copies, to completion);
   * select_ms    owners' merge of straddling groups + finalisation, or their percentile selection;
   * assemble_ms  the result on the host from devices[0]'s dense rows (or the devices' results merged). */
  double devices_ms;
  double xfer_ms;
  double select_ms;
  double assemble_ms;
} tsdbhip_timing;

/* ---- library-level helpers (host logic of the reference, restated) ------- */
int tsdbhip_abi_version(void);
const char* tsdbhip_last_error(void);
/* Developer options (no reference counterpart): kernel-choice switches that the parity tests
 * use to force an alternative kernel onto the same data (the general kernel, a sequential path,
 * small compaction chunks, ...), by name without a prefix: FAST, SHORT, ROWS, HWIN, SEQ,
 * SEQ_ROWS, SEQ_WAVE, INDEX_GENERIC, CMP_CHUNK, CMP_ROWS, CMP_ONEPASS, PCT_ROWS, PCT_KEYS,
 * PCT_VONLY, PCT_V6, SEL_FUSED, SEL_COLS, SEL_WIN, SEL_WAVE, SEL_REG, SELOPS, RAW_LERPW,
 * RAW_SEL_TOP, RAW_SEL_REG, RO_FUSE, RO_RUNS, MULTI_FUSE, EMIT_HALF, HIST_WINDOW, HIST_WS, HIST_LAYOUT, TRACE, DBG
 * (opentsdb_amd/csrc/opts.h says what each value does).  Process-wide; -1 resets an option to
 * its production choice, which is every option's initial state.  The library reads no
 * environment variable: an inherited environment cannot change its kernels.  DBG is honoured
 * only by a -DTSDBHIP_KDBG profiling build.  Unknown names -> TSDB_E_ILLEGAL_ARGUMENT. */
int tsdbhip_set_option(const char* name, int64_t value);
int tsdbhip_get_option(const char* name, int64_t* value);
/* Aggregators.get(name) (src/core/Aggregators.java:222-228); returns id or TSDB_E_NO_SUCH_ELEMENT */
int tsdbhip_aggregator_get(const char* name);
/* Aggregator.interpolationMethod() */
int tsdbhip_aggregator_interpolation(int aggregator);
/* DateTime.parseDuration (src/utils/DateTime.java:186-226) */
int tsdbhip_parse_duration(const char* duration, int64_t* out_ms);
/* new DownsamplingSpecification(String) (src/core/DownsamplingSpecification.java:116-191);
 * fills the ds_* fields of q */
int tsdbhip_parse_downsample(const char* spec, tsdbhip_query* q);
/* TsdbQuery.getScanStartTimeSeconds / getScanEndTimeSeconds (src/core/TsdbQuery.java:1506-1606) */
int tsdbhip_scan_bounds(const tsdbhip_query* q, int64_t* scan_start_s, int64_t* scan_end_s);

/* ---- engine ------------------------------------------------------------- */
typedef struct tsdbhip_ctx tsdbhip_ctx;

/* One context on one GPU (hipSetDevice(device)).  Several GPUs: one process per GPU with one
 * context each (the partials / sel exchange below), or one multi-device context
 * (tsdbhip_init_devices). */
int tsdbhip_init(int device, tsdbhip_ctx** out);
void tsdbhip_destroy(tsdbhip_ctx* ctx);
/* Copy a host batch into HBM (re-laid out: rows 16-B aligned).  Replaces any previous batch. */
int tsdbhip_load(tsdbhip_ctx* ctx, const tsdbhip_batch* host_batch);
/* ---- sharding one query's spans over ranks -------------------------
 * Byte-balanced contiguous shards, one per rank; bounds[world + 1], rank r owns
 * [bounds[r], bounds[r + 1]) of:
 *   TSDB_SHARD_SERIES  positions in SpanGroup order (kept series stably sorted by group id):
 *                      a group may straddle ranks (tsdbhip_run_partials, tsdbhip_sel_*);
 *   TSDB_SHARD_GROUPS  group ids: whole SpanGroups per rank (raw queries, no downsampler);
 *   TSDB_SHARD_SPANS   series positions in batch order, every span (NONE aggregator: it
 *                      ignores group-by tags, so series with group id -1 count too).
 * tsdbhip_load_shard loads one such range of a host batch (tsdbhip_load semantics; for
 * SPANS the shard's batch order is kept, so NONE results concatenate in rank order). */
enum { TSDB_SHARD_SERIES = 0, TSDB_SHARD_GROUPS = 1, TSDB_SHARD_SPANS = 2 };
int tsdbhip_shard_bounds(const tsdbhip_batch* batch, int world, int mode, int64_t* bounds);
int tsdbhip_load_shard(tsdbhip_ctx* ctx, const tsdbhip_batch* batch, int mode, int64_t begin, int64_t end);
/* Synthetic MockBase-equivalent store generated directly in HBM (see tsdbhip_synth_spec). */
typedef struct {
  int64_t n_series;
  int64_t start_s;          /* first timestamp (seconds) */
  int64_t n_points;         /* datapoints per series */
  int64_t period_ms;        /* sampling period (>= 1000 and multiple of 1000 -> second qualifiers) */
  int32_t value_kind;       /* 0 = float32 50+10(u-0.5); 1 = int hash % int_mod; 2 = even series int, odd float32 */
  int32_t n_groups;         /* group_id = series % n_groups, series sorted by group */
  int64_t int_mod;
  uint64_t seed;
} tsdbhip_synth_spec;
int tsdbhip_synth(tsdbhip_ctx* ctx, const tsdbhip_synth_spec* spec);
/* Batch positions [pos_begin, pos_end) of that store (series in group order): one rank's
 * contiguous TSDB_SHARD_SERIES shard of the whole store, generated on its own GPU. */
int tsdbhip_synth_shard(tsdbhip_ctx* ctx, const tsdbhip_synth_spec* spec, int64_t pos_begin, int64_t pos_end);
/* Copy the resident batch back to host (for parity checks); host arrays sized by tsdbhip_batch_sizes. */
int tsdbhip_batch_sizes(tsdbhip_ctx* ctx, int64_t* n_series, int64_t* n_rows, uint64_t* qual_bytes, uint64_t* val_bytes);
int tsdbhip_batch_download(tsdbhip_ctx* ctx, int64_t* series_row_ptr, uint32_t* row_base_time,
                           uint64_t* row_qual_off, uint64_t* row_val_off, uint8_t* qual, uint8_t* val,
                           int32_t* group_id);
/* The same for resident series positions [s0, s1) only (offsets from 0; only the rows' blob span
 * is copied, so slices of a store larger than host memory can be checked).  Any output pointer
 * may be NULL: that part is skipped (e.g. group_id alone gives the resident group order). */
int tsdbhip_batch_range_sizes(tsdbhip_ctx* ctx, int64_t s0, int64_t s1, int64_t* n_rows, uint64_t* qual_bytes,
                              uint64_t* val_bytes);
int tsdbhip_batch_download_range(tsdbhip_ctx* ctx, int64_t s0, int64_t s1, int64_t* series_row_ptr,
                                 uint32_t* row_base_time, uint64_t* row_qual_off, uint64_t* row_val_off,
                                 uint8_t* qual, uint8_t* val, int32_t* group_id);

/* Run the query over the resident batch: TsdbQuery.run() from GroupByAndAggregateCB on. */
int tsdbhip_run(tsdbhip_ctx* ctx, const tsdbhip_query* q, tsdbhip_result** out);
/* n queries that share the time range and the downsampling specification (a TSQuery with
 * several sub-queries over one metric).  A percentile / median downsampling is computed once
 * and shared by the queries' group-by steps.  With a cheap downsampling function, decomposable
 * group-by aggregators (sum, avg, min, max, dev, count; no rate, no flags, <= 64 output slots)
 * share ONE fused streaming pass that keeps every aggregator's SpanGroup state -- results
 * bit-identical to separate tsdbhip_run calls (tsdbhip_timing.fused_queries = n); any other mix
 * runs one fused pass per query.  outs[i] as tsdbhip_run's result; on error none is returned. */
int tsdbhip_run_multi(tsdbhip_ctx* ctx, const tsdbhip_query* qs, int n, tsdbhip_result** outs);
void tsdbhip_result_free(tsdbhip_result* r);
int tsdbhip_last_timing(tsdbhip_ctx* ctx, tsdbhip_timing* out);

/* ---- multi-GPU (series sharded over ranks; one exchange step) --------------
 * One process per GPU, each with its own context and its own contiguous shard of the
 * group-sorted series.  A SpanGroup may straddle ranks.  Every rank reduces
 * its shard to one partial state per (group, output slot); the caller all-gathers the
 * per-rank buffers (RCCL ncclAllGather over xGMI) into n_ranks consecutive copies in rank
 * order, and tsdbhip_finalize merges them in rank order -- which is SpanGroup series order,
 * so first/last/diff/mult keep the reference's semantics -- and finalises the aggregator
 * (AggregationIterator.doubleValue / Aggregator.runDouble).  An all-gather rather than an
 * all-reduce because the merge is not an RCCL operator for dev (Chan merge of Welford
 * states), first/last/diff/mult (ordered), and because the buffer is small:
 * n_groups * n_slots * 24 B (config 2: 64 x 60 -> 92 KB per rank).
 *
 * Buffer layout of one rank (bytes = tsdbhip_partials_layout.bytes, 16-B aligned parts):
 *   double   a[n_groups * n_slots]    sum / min / max / mean / first / last / product
 *   double   b[n_groups * n_slots]    Welford M2 / last value (diff)
 *   uint32_t n[n_groups * n_slots]    non-NaN contributions
 *   uint32_t f[n_groups * n_slots]    bit0 union point, bit1 has-value, >>2 contributions
 *   uint32_t active[n_groups]         the group has a span in [scan start, scan end]
 * Index [g * n_slots + k]; slot k is timestamp B0 + k * interval (or the "all" bucket). */
typedef struct {
  int64_t n_groups;
  int64_t n_slots;
  int64_t bytes;             /* per rank */
} tsdbhip_partials_layout;
int tsdbhip_partials_layout_get(tsdbhip_ctx* ctx, const tsdbhip_query* q, int64_t n_groups_global,
                                tsdbhip_partials_layout* out);
/* Computes this shard's partial states into `partials` (device or host memory, layout above). */
int tsdbhip_run_partials(tsdbhip_ctx* ctx, const tsdbhip_query* q, int64_t n_groups_global, void* partials);
/* n queries sharing the time range and downsampling (a TSQuery's sub-queries over one metric,
 * TsdbQuery.java:916-1049 once per sub-query): query i's partial states at partials + i * bytes.
 * sum / avg / min / max / dev / count without rate come from ONE fused streaming pass over the
 * shard (bit-identical to n tsdbhip_run_partials calls); any other mix runs query by query. */
int tsdbhip_run_partials_multi(tsdbhip_ctx* ctx, const tsdbhip_query* qs, int n, int64_t n_groups_global,
                               void* partials);
/* Merges n_ranks rank-ordered partial buffers (device or host memory) and builds the result. */
int tsdbhip_finalize(tsdbhip_ctx* ctx, const tsdbhip_query* q, int64_t n_groups_global,
                     const void* partials, int n_ranks, tsdbhip_result** out);
/* ---- multi-GPU percentile / median group-by (non-decomposable) ---------------
 * PercentileAgg / Median have no mergeable partial state (src/core/Aggregators.java:397-431,
 * 657-708), so every span's value per (group, slot) travels to the group's owning rank
 * (SURVEY.md 8e).  Per query, on every rank:
 *   1. tsdbhip_sel_layout: counts[g] = local spans of group g (n_groups_global entries),
 *      n_slots = K;
 *   2. tsdbhip_sel_run_values: the local spans' contributions (Downsampler, RateSpan, fill,
 *      LERP -- what AggregationIterator hands runDouble) into
 *        double  vals[sum_g counts[g] * K]   [span][slot], spans group by group in SpanGroup
 *                                            order (a span's K values contiguous; +NaN = none)
 *        uint8_t uni[n_groups * K]           a real point of some span (emit flag)
 *        uint32_t act[n_groups]              the group has a span in the scan range;
 *   3. the caller moves each group's block ([counts[g]][K]) to its owner (all-to-all over
 *      RCCL), concatenates the ranks' blocks of a group span-wise, OR-reduces uni / act;
 *   4. tsdbhip_sel_select on the owner: same layout with the gathered counts, segments
 *      sorted and runDouble's order statistic taken -> dense out_val [n_groups * K] f64 and
 *      out_flag [n_groups * K] u8 (groups with count 0: NaN where uni is set);
 *   5. after the owners' rows are combined, tsdbhip_assemble builds the usual result.
 * All buffer pointers may be device or host memory. */
int tsdbhip_sel_layout(tsdbhip_ctx* ctx, const tsdbhip_query* q, int64_t n_groups_global, int64_t* counts,
                       int64_t* n_slots);
int tsdbhip_sel_run_values(tsdbhip_ctx* ctx, const tsdbhip_query* q, int64_t n_groups_global, void* vals,
                           void* uni, void* act);
int tsdbhip_sel_select(tsdbhip_ctx* ctx, const tsdbhip_query* q, int64_t n_groups_global, const void* vals,
                       const int64_t* counts, const void* uni, void* out_val, void* out_flag);
/* Result of a downsampled group-by from dense per-(group, slot) values, emit flags and
 * group-active flags (layouts as tsdbhip_sel_select / tsdbhip_sel_run_values). */
int tsdbhip_assemble(tsdbhip_ctx* ctx, const tsdbhip_query* q, int64_t n_groups_global, const void* val,
                     const void* flag, const void* act, tsdbhip_result** out);
/* ---- one process, several GPUs: a multi-device context ----------
 * For a host that drives every GPU from one process (the TSD JVM): tsdbhip_init_devices
 * returns ONE context over devices[0 .. n_devices) -- an engine context and HIP stream per
 * device plus a merge context on devices[0].  tsdbhip_load / tsdbhip_synth shard the batch over
 * the devices, tsdbhip_run / tsdbhip_run_multi run every shard on its own host thread and return
 * what a one-GPU context returns for the same batch:
 *   TSDB_SHARD_GROUPS  whole SpanGroups per device (byte-balanced ranges of group ids; series
 *                      without a group on the last device): every query type runs locally and
 *                      the results are concatenated in group order (NONE: in batch order) --
 *                      no device exchange, bit-identical to one GPU;
 *   TSDB_SHARD_SERIES  contiguous byte-balanced positions of the SpanGroup order (a group may
 *                      straddle devices): decomposable aggregators gather their partial states
 *                      to devices[0] (RCCL send / recv over xGMI, or peer copies) and merge them
 *                      in device order (tsdbhip_finalize); percentile / median group-by and
 *                      TSDB_QF_ORDERED route each group to its owner (the first device holding
 *                      one of its spans): only the straddling groups' span rows move, every owner
 *                      selects its groups in place, and the owners' G x K result rows go to
 *                      devices[0]; raw group-by queries (no downsampler) run every whole group
 *                      locally and each straddling group on its owner over a copy of all its
 *                      spans (built once per load), so results are bit-identical to one GPU.
 *                      VERIFICATION STATUS: the exchange has been tested over one GPU repeated
 *                      as 2-8 devices (peer copies) and a one-rank RCCL communicator only; the
 *                      rank-to-rank moves between DISTINCT GPUs (RCCL send / recv, peer copies
 *                      over xGMI) are unverified on hardware until tests/test_gpu_multidev.py::
 *                      test_distinct_devices has run on a multi-GPU node.
 * TSDB_SHARD_AUTO (default) picks GROUPS when the group-aligned split is within 10% of the byte
 * balance, else SERIES; tsdbhip_md_shard_mode sets the mode of the following loads.
 * transport: TSDB_MD_AUTO = RCCL (ncclCommInitAll) when two or more devices are all distinct,
 * device copies when a device repeats (several shards on one GPU); TSDB_MD_RCCL / TSDB_MD_COPY
 * force one.
 * Entry points bound to one device's resident store (load_shard, synth_shard, batch
 * downloads, the per-rank partials / sel exchange, debug_rows) return TSDB_E_NOT_IMPLEMENTED on
 * such a context.  tsdbhip_load_rollup shards a rollup batch and tsdbhip_load_cells a compaction
 * scan (each device compacts its series' rows) as tsdbhip_load shards a batch;
 * tsdbhip_rollup_run generates every device's series' rollup cells on that device and
 * tsdbhip_rollup_download returns them in the one-GPU order (function, batch series, time),
 * byte for byte the one-GPU cells.  tsdbhip_load_histograms shards the histogram spans by whole
 * groups over the devices (contiguous group-id runs balanced by column bytes; an ungrouped span is
 * a unit of its own) and tsdbhip_hist_run / _range answer on every device and merge: groups in
 * group-id order ("none": spans in batch order), the bucket dictionary the union of the devices'.
 * The expression functions run on devices[0].  tsdbhip_last_timing: per-device stage times are the maximum over
 * the devices, counters are summed, total_ms is the host wall time of the call and exchange_ms
 * its gather + merge part. */
enum { TSDB_SHARD_AUTO = -1 };
enum { TSDB_MD_AUTO = -1, TSDB_MD_COPY = 0, TSDB_MD_RCCL = 1 };
int tsdbhip_init_devices(const int* devices, int n_devices, int transport, tsdbhip_ctx** out);
/* HIP devices visible to this process (hipGetDeviceCount), for a host that sizes its device list
 * without initialising another runtime. */
int tsdbhip_device_count(int* n);
int tsdbhip_md_shard_mode(tsdbhip_ctx* ctx, int mode);
/* n_devices, transport in use, shard mode of the resident batch (TSDB_SHARD_AUTO before a load)
 * and, when shard_series is not NULL, the resident series of every device ([n_devices]). */
int tsdbhip_md_info(tsdbhip_ctx* ctx, int* n_devices, int* transport, int* mode, int64_t* shard_series);
/* The last tsdbhip_run / tsdbhip_run_multi on a multi-device context: per_device[d] = device d's
 * own timing record, n_devices entries or NULL, *rccl_ranks = ranks of the RCCL communicator
 * (ncclCommCount; 0 with device copies), *xfer_bytes = bytes moved between devices. */
int tsdbhip_md_stats(tsdbhip_ctx* ctx, tsdbhip_timing* per_device, int* rccl_ranks, double* xfer_bytes);
/* ---- rollup generation --------------------------------
 * RollupInterval (src/rollup/RollupInterval.java:62-240): `interval` e.g. "1h", `row_span`
 * e.g. "1d"; validateAndCompile's checks and arithmetic, IllegalArgumentException ->
 * TSDB_E_ILLEGAL_ARGUMENT. */
typedef struct {
  int32_t interval_s;        /* getIntervalSeconds() */
  int32_t intervals;         /* getIntervals(): span seconds / interval (12 .. 7774) */
  char units;                /* getUnits(): row span unit 'h' 'd' 'n' 'y' */
  char interval_units;       /* getIntervalUnits(): last character of the interval string */
  int16_t unit_multiplier;   /* getUnitMultiplier(): row span count */
} tsdbhip_rollup_interval;
int tsdbhip_rollup_interval_parse(const char* interval, const char* row_span, tsdbhip_rollup_interval* out);
/* RollupUtils.getRollupBasetime (src/rollup/RollupUtils.java:52-112); timestamp in s or ms. */
int tsdbhip_rollup_basetime(int64_t timestamp, const tsdbhip_rollup_interval* iv, int32_t* out);
/* RollupUtils.buildRollupQualifier (src/rollup/RollupUtils.java:143-171): 3 bytes
 * [aggregator id][BE16((offset_in_intervals << 4) | flags)]. */
int tsdbhip_rollup_qualifier(int64_t timestamp, int32_t basetime, int16_t flags, int32_t aggregator_id,
                             const tsdbhip_rollup_interval* iv, uint8_t out[3]);

/* Rollup generation over the resident batch.  The reference ingests rollups
 * (/api/rollup, src/tsd/RollupDataPointRpc.java:157-165 -> TSDB.addAggregatePoint,
 * src/core/TSDB.java:1322-1588) but never computes them; the engine computes them as the
 * Downsampler (fixed interval = the rollup interval, fill none) of every series with each
 * requested function, and writes each bucket as the cell addAggregatePoint would store:
 *   qualifier  buildRollupQualifier(bucket start, base, flags, agg_id[i], interval)
 *   row base   getRollupBasetime(bucket start, interval)
 *   value      count, and sum/min/max of a series whose every datapoint is an integer:
 *                vleEncodeLong((long) v)                        (flags = length - 1)
 *              otherwise a float32 when (float) v == v          (flags 0xB, Tags.fitsInFloat)
 *              else a float64                                   (flags 0xF)
 *              NaN / +-Inf -> TSDB_E_ILLEGAL_ARGUMENT (addAggregatePoint rejects them).
 * Buckets whose start lies in [start_s, end_s) are written.  Cells are ordered by
 * (function index i, batch series index, time).  Output stays on the device until
 * tsdbhip_rollup_download. */
typedef struct {
  tsdbhip_rollup_interval interval;
  int64_t start_s, end_s;
  int32_t n_funcs;           /* 1..4 */
  int32_t func[4];           /* TSDB_AGG_SUM / COUNT / MAX / MIN (any order) */
  int32_t agg_id[4];         /* RollupConfig id written in the qualifier (TestTsdbQueryRollup: sum 0, count 1, max 2, min 3) */
} tsdbhip_rollup_spec;
int tsdbhip_rollup_run(tsdbhip_ctx* ctx, const tsdbhip_rollup_spec* spec, int64_t* n_cells, uint64_t* value_bytes);
/* Copies the last rollup_run's cells to caller-allocated host arrays:
 * series[n_cells] (batch series index), base_time[n_cells], qualifier[3 * n_cells],
 * val_off[n_cells + 1], value[value_bytes]. */
int tsdbhip_rollup_download(tsdbhip_ctx* ctx, int32_t* series, uint32_t* base_time, uint8_t* qualifier,
                            uint64_t* val_off, uint8_t* value);

/* ---- rollup read path ----------------------------------
 * A query over a rollup table (TsdbQuery with a RollupQuery, src/core/TsdbQuery.java:1293-1362;
 * the rollup interval matched the downsampling interval).  The spans are RollupSpans of
 * RollupSeq rows (src/rollup/RollupSeq.java:52-740): per row the cells of the queried
 * aggregate, and -- when the group-by aggregator is avg or dev (RollupSeq.need_count) -- the
 * count cells.  Each cell: 2-byte rollup qualifier (offset << 4 | flags, the aggregator byte or
 * the old "sum:" string prefix stripped), value bytes (no meta byte).  A datapoint's timestamp
 * is base + offset * interval_s (RollupUtils.getTimestampFromRollupQualifier :178-235); with
 * counts the iterator yields only offsets present in both streams (RollupSeq.sync); offsets
 * must increase within a row (else IllegalDataException; a repeated offset keeps the later
 * cell when fix_duplicates).  The Downsampler then follows its rollup branches
 * (src/core/Downsampler.java:165-221, FillingDownsampler.java:196-253): an avg downsampling
 * of avg rollups is Σsum / Σcount per bucket (0 when Σcount is 0); count sums the counts;
 * the other functions run on the values.  Scan bounds are the rollup's
 * (TsdbQuery.getScanStart/EndTimeSeconds :1515-1526, 1562-1567). */
typedef struct {
  tsdbhip_batch cells;               /* the aggregate's cells, rows as above */
  const uint64_t* row_cqual_off;     /* [n_rows + 1] count cells per row, or NULL (no counts) */
  const uint64_t* row_cval_off;      /* [n_rows + 1] */
  const uint8_t* cqual;
  const uint8_t* cval;
  tsdbhip_rollup_interval interval;  /* the rollup table's interval */
  int32_t fix_duplicates;            /* tsd.storage.fix_duplicates */
} tsdbhip_rollup_batch;
/* Loads a rollup batch as the resident batch; tsdbhip_run then runs rollup queries over it
 * (downsampling required; tsdbhip_run_multi excluded).  A rank's rollup shard takes part in
 * the partials (tsdbhip_run_partials / finalize) and percentile (tsdbhip_sel_*) exchanges --
 * every rank plans a count group-by as sum -- and a multi-device context shards a rollup batch
 * like tsdbhip_load (value and count cells of a series stay together). */
int tsdbhip_load_rollup(tsdbhip_ctx* ctx, const tsdbhip_rollup_batch* rb);

/* ---- query-time compaction ----------------------------------
 * The scanner's rows before TSDB.compact (src/core/SaltScanner.java:734-870): every column
 * (KeyValue) of a row key in scan order -- single datapoints (2-byte or 4-byte ms qualifiers),
 * earlier compactions, append columns (qualifier 0x05 0x00 0x00) and annotations / other
 * odd-length qualifiers (skipped) -- with their HBase write timestamps.  Every row is compacted
 * on the GPU as CompactionQueue.Compaction.compact (src/core/CompactionQueue.java:330-566,
 * ColumnDatapointIterator.java:63-205, AppendDataPoints.java:110-240) returns it to a query:
 * datapoints merged by offset, the newest column's kept at a repeated offset (any other value
 * -> IllegalDataException unless fix_duplicates), 2-byte float and length fixups, the meta byte;
 * a single column needing no fixup as stored; rows without a datapoint dropped.  The compacted
 * rows become the resident batch; rows of one series with the same base time (one per salt
 * bucket) are compacted each and then merged in scan order as Span.addRow / RowSeq.addRow merge
 * them (src/core/Span.java:202-219).  Compaction exceptions are raised by the first query whose
 * scan range covers the row.  Scans of more than 2^31 columns or datapoints are compacted in
 * chunks of whole rows.  NOT_IMPLEMENTED: a row of more than 2^31 columns or datapoints, more
 * than 2^31 rows; per row, lazily: a compacted cell out of time order, a datapoint column with an empty
 * value.
 * use_otsdb_timestamp (Config.java:621, default false) switches the merge to dtcsMergeDataPoints
 * (CompactionQueue.java:500-547): at a repeated offset the datapoint with the greatest value
 * (use_max_value, Config.java:622, default true) or the smallest (false), by
 * ColumnDatapointIterator.getCellValueAsDouble, is kept -- the first in heap order (newest column
 * first) on a tie, the heap's head when its value is NaN -- with no duplicate exception; a merged
 * row holding a value that getCellValueAsDouble cannot read (a float of 1, 2, 3, 5, 6 or 7 bytes,
 * an integer of 3, 5, 6 or 7) raises TSDB_E_RUNTIME (BufferUnderflowException); the meta byte
 * follows the reference's isMilliseconds() read after the kept column advanced.  The HBase scan
 * time range that flag also sets (TsdbQuery.java:1401-1409) is the caller's scan.  Such batches
 * run the global-sort compaction path.
 * Documented approximation (parity unpinned): columns with EQUAL HBase write timestamps are taken
 * in scan order, here and in the oracle.  The reference's ColumnDatapointIterator.compareTo returns
 * 0 for them and java.util.PriorityQueue is not stable, so which of two such columns heads the heap
 * -- the one whose datapoint a DTCS tie keeps (int 5 vs float 5.0, a NaN head) -- is not defined by
 * the reference; give such columns distinct col_timestamp values for a defined answer. */
typedef struct {
  int64_t n_series;
  const int64_t* series_row_ptr;   /* [n_series + 1] */
  int64_t n_rows;
  const uint32_t* row_base_time;   /* [n_rows] */
  const int64_t* row_col_ptr;      /* [n_rows + 1] columns of each row */
  int64_t n_cols;
  const uint64_t* col_qual_off;    /* [n_cols + 1] from 0 */
  const uint64_t* col_val_off;     /* [n_cols + 1] from 0 */
  const int64_t* col_timestamp;    /* [n_cols] KeyValue.timestamp(), or NULL (equal: scan order decides) */
  const uint8_t* qual;
  const uint8_t* val;
  const int32_t* group_id;         /* [n_series] */
  int32_t fix_duplicates;          /* tsd.storage.fix_duplicates */
  int32_t use_otsdb_timestamp;     /* tsd.storage.use_otsdb_timestamp: dtcsMergeDataPoints */
  int32_t use_max_value;           /* tsd.storage.use_max_value (with use_otsdb_timestamp) */
} tsdbhip_cell_batch;
int tsdbhip_load_cells(tsdbhip_ctx* ctx, const tsdbhip_cell_batch* cb);

/* ---- histogram path ----------------------------------------
 * TsdbQuery.runHistogram (src/core/TsdbQuery.java:759-776, HistogramGroupByAndAggregateCB
 * :1061-1255): the scanner's histogram columns (qualifier prefix 0x06, Internal.getQualifier /
 * getTimeStampFromNonDP :1059-1074; value = [codec id][codec payload]) per row in column order,
 * decoded by the codec HistogramCodecManager maps the id to (src/core/HistogramCodecManager.java:
 * 148-206): SimpleHistogram (Kryo 2.21: BE16 bucket count, per bucket BE float lower / upper and a
 * varint count, varint underflow and overflow; src/core/SimpleHistogram.java:97-122) or the
 * reference's 8-byte long test codec (test/core/LongHistogramDataPointForTest.java).  A column
 * that fails to decode is dropped (SaltScanner.processRow :771-778), a row without a histogram
 * is not added.  Rows of a series become a HistogramSpan (addRow merge, :280-328); the spans of a
 * group are merged by HistogramAggregationIterator (:91-287: union of timestamps, SUM of the
 * histograms at equal timestamps, no interpolation) after the HistogramDownsampler (:28-403,
 * SUM inside each interval, fill policies ignored).  Each group yields one DataPoints per
 * requested percentile (HistogramDataPointsToDataPointsAdaptor: SimpleHistogram.percentile
 * :133-164, the long codec data * p) and, with show_buckets, one per bucket of its first point
 * (HistogramBucketDataPointsAdaptor).  Any group-by aggregator other than "none" is SUM
 * (TsdbQuery.java:1132); "none" emits every span as its own group. */
enum { TSDB_HCODEC_NONE = 0, TSDB_HCODEC_SIMPLE = 1, TSDB_HCODEC_LONG = 2 };
typedef struct {
  int64_t n_series;
  const int64_t* series_row_ptr;   /* [n_series + 1] rows of each span, scan order */
  int64_t n_rows;
  const uint32_t* row_base_time;   /* [n_rows] seconds */
  const int64_t* row_cell_ptr;     /* [n_rows + 1] histogram columns of each row, column order */
  int64_t n_cells;
  const uint64_t* cell_qual_off;   /* [n_cells + 1] from 0 */
  const uint64_t* cell_val_off;    /* [n_cells + 1] from 0 */
  const uint8_t* qual;
  const uint8_t* val;
  const int32_t* group_id;         /* [n_series] as tsdbhip_batch */
  uint8_t codec[256];              /* codec kind (TSDB_HCODEC_*) of each codec id */
} tsdbhip_hist_batch;
/* Loads histogram spans as the resident histogram store (replaces the previous one; the
 * numeric batch is unaffected). */
int tsdbhip_load_histograms(tsdbhip_ctx* ctx, const tsdbhip_hist_batch* hb);

/* Result of a histogram query, one entry per emitted HistogramSpanGroup (group order; for
 * "none" one per span in batch order, group_id = span index).  Points of group g are
 * [group_ptr[g], group_ptr[g + 1]).  pct[point * n_pct + j] = the j-th requested percentile.
 * With show_buckets: the bucket dictionary (every bucket of the store, TreeMap order of
 * HistogramBucket.compareTo: Float.compare of lower then upper bound; NaN bounds canonical), per
 * point count[point * (n_buckets + 2) + b] (b < n_buckets: the bucket's summed count, n_buckets:
 * underflow, n_buckets + 1: overflow) and present[point * n_buckets + b] (the bucket is in the
 * point's histogram); codec[point] = codec kind of the point's histogram (bucket series exist for
 * SimpleHistogram only).  The bucket series themselves (HistogramBucketDataPointsAdaptor:
 * the first point's buckets, each looked up in every point) are built by the host from these. */
typedef struct {
  int64_t n_groups;
  const int32_t* group_id;
  const int64_t* group_ptr;
  const int64_t* ts_ms;
  int32_t n_pct;
  const double* pct;
  int32_t show_buckets;
  int32_t n_buckets;
  const uint32_t* bucket_lower;    /* float bits */
  const uint32_t* bucket_upper;
  const int64_t* count;
  const uint8_t* present;
  const uint8_t* codec;
} tsdbhip_hist_result;
/* The query's start / end, aggregator and downsampling (ds_function is ignored: histograms are
 * always summed; -1 = no downsampling) as for tsdbhip_run; pct[n_pct] the percentiles
 * (TsdbQuery.setPercentiles, List<Float>).  Calendar downsampling (UTC, ds_tz, per-span anchors)
 * included.  Raw group-by over spans whose datapoints are not in time order (a row mixing second
 * and millisecond qualifiers is iterated in column order) follows HistogramAggregationIterator.next's
 * greedy walk (:240-292): repeated and receding timestamps, points merged only when current together.
 * NOT_IMPLEMENTED: more than 32 GB of per-point state, more than 32768 distinct buckets. */
int tsdbhip_hist_run(tsdbhip_ctx* ctx, const tsdbhip_query* q, int n_pct, const float* pct, int show_buckets,
                     tsdbhip_hist_result** out);
/* The same over every row of the store with the HistogramSpanGroup bounds given directly (ms):
 * HistogramAggregationIterator.create(spans, start_ms, end_ms, ...) as the reference's iterator
 * tests call it (test/core/TestHistogramAggregationIterator.java); the query's start / end only
 * bound "all" downsampling. */
int tsdbhip_hist_run_range(tsdbhip_ctx* ctx, const tsdbhip_query* q, int64_t start_ms, int64_t end_ms, int n_pct,
                           const float* pct, int show_buckets, tsdbhip_hist_result** out);
void tsdbhip_hist_result_free(tsdbhip_hist_result* r);

/* ---- expression functions over query results ----------------------
 * The graphite-style functions of src/query/expression/ (ExpressionFactory.java:41-63) run over
 * the DataPoints a query returned.  Input: n_series result series as flat arrays (series i owns
 * points [ptr[i], ptr[i + 1]) of ts / bits / is_int, the tsdbhip_result layout); output: a
 * tsdbhip_result with one group per output series (group_id = its index).
 *
 * tsdbhip_expr_map, one output series per input series:
 *   TSDB_EXPR_SCALE         Scale.scale (Scale.java:86-112): a long times an integral factor stays a
 *                           long ((long) factor * v, Java wrap), everything else factor * v as double
 *   TSDB_EXPR_ABSOLUTE      Absolute.abs (Absolute.java:64-83): Math.abs of the long or the double
 *   TSDB_EXPR_SHIFT         TimeShift.shift (TimeShift.java:121-141): ts + iparam ms, longValue()
 *                           (a double point raises ClassCastException, as MutableDataPoint does)
 *   TSDB_EXPR_MOVING_AVG    MovingAverage (MovingAverage.java:60-123, MovingAverageAggregator
 *                           :190-330) through a one-span AggregationIterator over [start, end]:
 *                           the mean of the last iparam non-NaN values (fparam = 0) or of the
 *                           points within iparam ms (fparam = 1, the first point 0), newest first
 * tsdbhip_expr_zip: ExpressionIterator (ExpressionIterator.java:282-318) as EDPtoDPS iterates it
 *   (EDPtoDPS.java:148-160): per joined set j the variables' series (set_series[j * n_vars + v],
 *   -1: the variable has no series with that set's tags) are read position by position, the
 *   timestamp is the smallest of the present series', a NaN value is the variable's fill value
 *   (TimeSyncedIterator's NumericFillPolicy, ZERO by default), an absent variable reads 0; a
 *   present series that ends before another raises RuntimeException ("No more elements",
 *   TimeSyncedIterator.java:152-160).  The expression is a postfix program over doubles (JEXL 2.1.1
 *   arithmetic on Doubles: + - * / % and negation, comparisons; a division or modulo by zero yields
 *   0.0, the lenient JEXL interpreter's answer -- TestExpressionIterator.aDivideByZeroWithTwoSeries). */
enum { TSDB_EXPR_SCALE = 0, TSDB_EXPR_ABSOLUTE, TSDB_EXPR_SHIFT, TSDB_EXPR_MOVING_AVG };
enum { TSDB_XOP_VAR = 0, TSDB_XOP_CONST, TSDB_XOP_ADD, TSDB_XOP_SUB, TSDB_XOP_MUL, TSDB_XOP_DIV, TSDB_XOP_MOD,
       TSDB_XOP_NEG,
       /* comparisons (JexlArithmetic.lessThan & co. on doubles): 1.0 / 0.0, as ExpressionIterator maps a
          Boolean result; NOT: negate(Boolean); IDIV / IMOD: the integer path of divide / mod (operands
          that are Integers or Booleans: truncating division, BigInteger.mod) */
       TSDB_XOP_LT, TSDB_XOP_GT, TSDB_XOP_LE, TSDB_XOP_GE, TSDB_XOP_EQ, TSDB_XOP_NE, TSDB_XOP_NOT, TSDB_XOP_IDIV,
       TSDB_XOP_IMOD };
typedef struct {
  int64_t n_series;
  const int64_t* ptr;          /* [n_series + 1] */
  const int64_t* ts_ms;
  const uint64_t* value_bits;  /* longValue() or doubleToRawLongBits(doubleValue()) */
  const uint8_t* is_int;
} tsdbhip_series_set;
int tsdbhip_expr_map(tsdbhip_ctx* ctx, int fn, double fparam, int64_t iparam, int64_t start_ms, int64_t end_ms,
                     const tsdbhip_series_set* in, tsdbhip_result** out);
/* program: n_ops (op, arg) pairs -- arg = variable index (TSDB_XOP_VAR) or constant index */
int tsdbhip_expr_zip(tsdbhip_ctx* ctx, const int32_t* program, int n_ops, const double* consts, int n_vars,
                     int64_t n_sets, const int32_t* set_series, const double* var_fill, const tsdbhip_series_set* in,
                     tsdbhip_result** out);

/* tsdbhip_expr_sync: ExpressionIterator.next(timestamp) as /api/query/exp serializes it
 * (src/tsd/QueryExecutor.java:668-708): the join iterator (UnionIterator / IntersectionIterator
 * .next(), UnionIterator.java:409-419, IntersectionIterator.java:215-223) steps every sub-query's
 * TimeSyncedIterator to the smallest next timestamp of its series (TimeSyncedIterator.java:125-158);
 * a series without a point at that step reads its variable's fill (var_fill[v], the sub-query's
 * NumericFillPolicy), as does a NaN value (ExpressionIterator.java:332-345); a variable without a
 * series in a joined set (UNION's fill_dp) reads absent_value (the union's fill, 0).  The steps are the
 * distinct timestamps of the series marked active (NULL: every series; IntersectionIterator nulls the
 * series it kicks out, :306-349), those in [start_ms, end_ms] are emitted: one output group per
 * joined set, one double per step.  The join itself (flattenTags keys, ByteMap order) is host logic
 * (opentsdb_amd/expression.py).  A series may repeat a timestamp: the step walk then steps it as
 * often as the series holding most copies of it, the j-th step reading each series' j-th copy (or
 * its fill).  A series out of time order (a decreasing timestamp) -> TSDB_E_NOT_IMPLEMENTED. */
int tsdbhip_expr_sync(tsdbhip_ctx* ctx, const int32_t* program, int n_ops, const double* consts, int n_vars,
                      int64_t n_sets, const int32_t* set_series, const double* var_fill, double absent_value,
                      const uint8_t* active, int64_t start_ms, int64_t end_ms, const tsdbhip_series_set* in,
                      tsdbhip_result** out);

/* highestMax / highestCurrent (HighestMax.java:37-150, HighestCurrent.java:37-151): the series
 * of `in` (every sub-query's group-bys, flattened in order; each sorted by time) run through one
 * AggregationIterator(start_ms, end_ms, LERP) with MaxCacheAggregator (HighestMax.java:182-292)
 * or MaxLatestAggregator (HighestCurrent.java:172-283).  Those keep the operands of each point
 * by POSITION among the spans that have a value, not by series.  The series are then ranked
 * by TopNSortingEntry (descending Double.compare, stable).  out_index (capacity in->n_series)
 * receives the indices into `in` of the min(topn, n) series returned, in order; *out_n their
 * count.  HighestCurrent drops series without points first, as the reference does.
 * topn < 1 -> TSDB_E_ILLEGAL_ARGUMENT (the host mirror parses the string parameter); series
 * but no point in [start_ms, end_ms] -> TSDB_E_NULL_POINTER (the reference sorts null entries);
 * a series out of time order -> TSDB_E_ILLEGAL_ARGUMENT. */
enum { TSDB_EXPR_HIGHEST_MAX = 4, TSDB_EXPR_HIGHEST_CURRENT = 5 };
int tsdbhip_expr_topn(tsdbhip_ctx* ctx, int fn, int32_t topn, int64_t start_ms, int64_t end_ms,
                      const tsdbhip_series_set* in, int32_t* out_index, int32_t* out_n);

/* Page-locked host memory for the buffers a caller hands to the load entry points
 * (tsdbhip_load, tsdbhip_load_cells, tsdbhip_load_histograms ...): their uploads are then DMA
 * transfers at the link's rate instead of staged copies of pageable memory.  A JVM caller wraps
 * the block in a direct ByteBuffer (JNI NewDirectByteBuffer) and assembles the scan into it.
 * No reference counterpart (the JVM's scan buffers). */
int tsdbhip_host_alloc(uint64_t bytes, void** out);
void tsdbhip_host_free(void* p);

/* Device synchronisation helper for host code that does not use HIP directly. */
int tsdbhip_sync(tsdbhip_ctx* ctx);

/* Test hook (no reference counterpart): the per-row facts k_index derived for the resident
 * batch, rows in resident order -- datapoints, RowDesc flags, exactness-certificate lsb and
 * max |value|.  Any pointer may be null. */
int tsdbhip_debug_rows(tsdbhip_ctx* ctx, uint32_t* ndp, uint32_t* flags, int32_t* lsb, double* absmax);

/* Test hook (no reference counterpart): how many percentile / median group-by queries took the
 * sampled-window select, and how many of those fell back to the full path (a window that missed
 * its ranks, a handed-back tile). */
int tsdbhip_debug_sel_window(tsdbhip_ctx* ctx, int64_t* runs, int64_t* misses);

#ifdef __cplusplus
}
#endif
#endif /* TSDBHIP_H */
