/*
 * refcpu.c -- TEST INFRASTRUCTURE ONLY (parity oracle + CPU baseline "port").
 *
 * Plain-C restatement of the OpenTSDB 2.4 query-time aggregation path, following
 * the reference iterator structure and evaluation order one for one (citations are
 * relative to the reference tree, /root/reference):
 *   RowSeq / Internal qualifier codec .... src/core/RowSeq.java, src/core/Internal.java
 *   Span.Iterator ........................ src/core/Span.java:355-479
 *   Downsampler / ValuesInInterval ....... src/core/Downsampler.java:118-512
 *   FillingDownsampler ................... src/core/FillingDownsampler.java:94-311
 *   RateSpan ............................. src/core/RateSpan.java:47-180
 *   AggregationIterator .................. src/core/AggregationIterator.java:395-797
 *   Aggregators .......................... src/core/Aggregators.java:231-852
 *   commons-math3 3.4.1 Percentile ....... (third_party/apache/include.mk:25, not vendored;
 *                                           restated from its published algorithm)
 *   SpanGroup / TsdbQuery ................ src/core/SpanGroup.java:257-341,527-532,
 *                                           src/core/TsdbQuery.java:916-1049,1506-1606
 * Build with -ffp-contract=off (Java never fuses multiply-add).  Java exceptions are
 * modelled with setjmp/longjmp and surface as TSDB_E_* codes.
 */
#define _GNU_SOURCE
#include "refcpu.h"

#include <math.h>
#include <pthread.h>
#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <ctype.h>

/* ------------------------------------------------------------------------ */
/* exceptions                                                                */
/* ------------------------------------------------------------------------ */
static __thread jmp_buf* g_jb = NULL;
static __thread char g_msg[512];
static __thread int g_code;

const char* ref_last_error(void) { return g_msg; }

static void jthrow(int code, const char* fmt, ...) __attribute__((noreturn));
static void jthrow(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_msg, sizeof g_msg, fmt, ap);
  va_end(ap);
  g_code = code;
  if (g_jb) longjmp(*g_jb, 1);
  fprintf(stderr, "refcpu: uncaught exception %d: %s\n", code, g_msg);
  abort();
}

/* TRY { ... } CATCH(code) { ... } -- nests. */
#define TRY                                       \
  {                                               \
    jmp_buf _jb;                                  \
    jmp_buf* _prev = g_jb;                        \
    g_jb = &_jb;                                  \
    if (setjmp(_jb) == 0) {
#define CATCH(var)                                \
    g_jb = _prev;                                 \
    } else {                                      \
      int var = g_code;                           \
      g_jb = _prev;
#define END_TRY }}

static void* xmalloc(size_t n) {
  void* p = malloc(n ? n : 1);
  if (!p) jthrow(TSDB_E_NOMEM, "out of memory");
  return p;
}
static void* xcalloc(size_t n, size_t m) {
  void* p = calloc(n ? n : 1, m ? m : 1);
  if (!p) jthrow(TSDB_E_NOMEM, "out of memory");
  return p;
}

/* ------------------------------------------------------------------------ */
/* Java arithmetic                                                           */
/* ------------------------------------------------------------------------ */
#define LONG_MAX_J INT64_MAX
#define LONG_MIN_J INT64_MIN
static inline int64_t jadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
static inline int64_t jsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
static inline int64_t jmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }
static inline int64_t jdiv(int64_t a, int64_t b) {
  if (b == 0) jthrow(TSDB_E_ILLEGAL_STATE, "ArithmeticException: / by zero");
  if (a == LONG_MIN_J && b == -1) return LONG_MIN_J;
  return a / b;
}
/* (long) of a double, JLS 5.1.3 */
static inline int64_t jd2l(double d) {
  if (isnan(d)) return 0;
  if (d >= 9223372036854775807.0) return LONG_MAX_J;
  if (d <= -9223372036854775808.0) return LONG_MIN_J;
  return (int64_t)d;
}
static inline uint64_t dbits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
static inline double bitsd(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }

/* ------------------------------------------------------------------------ */
/* DataPoint accessors (lazy value decode errors)                            */
/* ------------------------------------------------------------------------ */
static inline int64_t dp_long(const ref_dp* d) {
  if (d->bad) jthrow(d->bad, "bad value at ts=%lld", (long long)d->ts);
  if (!d->is_int) jthrow(TSDB_E_CLASS_CAST, "value is a double");
  return d->lv;
}
static inline double dp_double(const ref_dp* d) {
  if (d->bad) jthrow(d->bad, "bad value at ts=%lld", (long long)d->ts);
  if (d->is_int) jthrow(TSDB_E_CLASS_CAST, "value is a long");
  return d->dv;
}
static inline double dp_to_double(const ref_dp* d) {
  if (d->bad) jthrow(d->bad, "bad value at ts=%lld", (long long)d->ts);
  return d->is_int ? (double)d->lv : d->dv;
}
static inline ref_dp dp_of_long(int64_t ts, int64_t v) { ref_dp d = {ts, 1, 0, v, 0.0, 1, 0, 0}; return d; }
static inline ref_dp dp_of_double(int64_t ts, double v) { ref_dp d = {ts, 0, 0, 0, v, 1, 0, 0}; return d; }
/* MutableDataPoint.reset(DataPoint) reads the value eagerly (src/core/MutableDataPoint.java) */
static inline ref_dp dp_copy_eager(const ref_dp* d) {
  if (d->is_int) return dp_of_long(d->ts, dp_long(d));
  return dp_of_double(d->ts, dp_double(d));
}

/* ------------------------------------------------------------------------ */
/* views                                                                     */
/* ------------------------------------------------------------------------ */
typedef struct {
  int (*has_next)(ref_view*);
  ref_dp (*next)(ref_view*);
  void (*seek)(ref_view*, int64_t);
  void (*destroy)(ref_view*);
} view_vt;
struct ref_view { const view_vt* vt; };

static inline int v_has_next(ref_view* v) { return v->vt->has_next(v); }
static inline ref_dp v_next(ref_view* v) { return v->vt->next(v); }
static inline void v_seek(ref_view* v, int64_t t) { v->vt->seek(v, t); }

/* ---- values interface for Aggregator.runLong/runDouble ------------------ */
typedef struct {
  int (*has)(void*);
  int64_t (*nl)(void*);
  double (*nd)(void*);
  void* c;
} vals_t;

/* ======================================================================== */
/* Aggregators (src/core/Aggregators.java)                                   */
/* ======================================================================== */
static const char* const AGG_NAMES[TSDB_AGG_COUNT_ALL] = {
    "sum", "pfsum", "min", "max", "avg", "median", "none", "mult", "dev", "diff",
    "zimsum", "mimmin", "mimmax", "squareSum", "count", "first", "last",
    "p999", "p99", "p95", "p90", "p75", "p50",
    "ep999r3", "ep99r3", "ep95r3", "ep90r3", "ep75r3", "ep50r3",
    "ep999r7", "ep99r7", "ep95r7", "ep90r7", "ep75r7", "ep50r7"};

int ref_aggregator_get(const char* name) {
  for (int i = 0; i < TSDB_AGG_COUNT_ALL; i++)
    if (strcmp(AGG_NAMES[i], name) == 0) return i;
  snprintf(g_msg, sizeof g_msg, "No such aggregator: %s", name);
  return TSDB_E_NO_SUCH_ELEMENT;
}

/* Aggregators.java:47-173 */
static int agg_interp(int a) {
  switch (a) {
    case TSDB_AGG_PFSUM: return TSDB_INTERP_PREV;
    case TSDB_AGG_NONE: case TSDB_AGG_ZIMSUM: case TSDB_AGG_SQUARESUM: case TSDB_AGG_COUNT:
    case TSDB_AGG_FIRST: case TSDB_AGG_LAST: return TSDB_INTERP_ZIM;
    case TSDB_AGG_MIMMIN: return TSDB_INTERP_MAX;
    case TSDB_AGG_MIMMAX: return TSDB_INTERP_MIN;
    default: return TSDB_INTERP_LERP;
  }
}

static int is_percentile(int a) { return a >= TSDB_AGG_P999 && a <= TSDB_AGG_EP50R7; }
static double pct_value(int a) {
  static const double q[6] = {99.9, 99.0, 95.0, 90.0, 75.0, 50.0};
  return q[(a - TSDB_AGG_P999) % 6];
}
/* 0 = LEGACY (estimation null), 3 = R_3, 7 = R_7 */
static int pct_est(int a) { int b = (a - TSDB_AGG_P999) / 6; return b == 0 ? 0 : (b == 1 ? 3 : 7); }

static int cmp_double(const void* a, const void* b) {
  double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : (x > y ? 1 : 0);
}
/* Double.compareTo (Collections.sort of a List<Double>): -0.0 before 0.0 (NaNs are dropped) */
static int cmp_double_total(const void* a, const void* b) {
  double x = *(const double*)a, y = *(const double*)b;
  if (x < y) return -1;
  if (x > y) return 1;
  const int sx = signbit(x) != 0, sy = signbit(y) != 0;
  return sx == sy ? 0 : (sx ? -1 : 1);
}

/* commons-math3 3.4.1 Percentile.evaluate with EstimationType LEGACY / R_3 / R_7
 * (index() and the shared estimate()); NaNs already removed by the caller. */
static double percentile_eval(double* work, int64_t n, double quantile, int est) {
  if (n == 0) return NAN;
  if (n == 1) return work[0];
  qsort(work, (size_t)n, sizeof(double), cmp_double);
  const double p = quantile / 100.0;
  double pos;
  if (est == 3) {
    const double minLimit = 0.5 / (double)n;
    pos = (p <= minLimit) ? 0.0 : rint((double)n * p);
  } else if (est == 7) {
    pos = (p == 0.0) ? 0.0 : (p == 1.0 ? (double)n : 1.0 + (double)(n - 1) * p);
  } else {
    pos = (p == 0.0) ? 0.0 : (p == 1.0 ? (double)n : p * (double)(n + 1));
  }
  const double fpos = floor(pos);
  const int64_t intPos = (int64_t)fpos;
  const double dif = pos - fpos;
  if (pos < 1) return work[0];
  if (pos >= (double)n) return work[n - 1];
  const double lower = work[intPos - 1];
  const double upper = work[intPos];
  return lower + dif * (upper - lower);
}

typedef struct { double* a; int64_t n, cap; } dvec;
static void dvec_push(dvec* v, double x) {
  if (v->n == v->cap) {
    v->cap = v->cap ? v->cap * 2 : 16;
    double* na = (double*)realloc(v->a, (size_t)v->cap * sizeof(double));
    if (!na) jthrow(TSDB_E_NOMEM, "oom");
    v->a = na;
  }
  v->a[v->n++] = x;
}
typedef struct { int64_t* a; int64_t n, cap; } lvec;
static void lvec_push(lvec* v, int64_t x) {
  if (v->n == v->cap) {
    v->cap = v->cap ? v->cap * 2 : 16;
    int64_t* na = (int64_t*)realloc(v->a, (size_t)v->cap * sizeof(int64_t));
    if (!na) jthrow(TSDB_E_NOMEM, "oom");
    v->a = na;
  }
  v->a[v->n++] = x;
}
static int cmp_long(const void* a, const void* b) {
  int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
  return x < y ? -1 : (x > y ? 1 : 0);
}

static int64_t agg_run_long(int a, vals_t* v) {
  switch (a) {
    case TSDB_AGG_SUM: case TSDB_AGG_PFSUM: case TSDB_AGG_ZIMSUM: {  /* :237-243 */
      int64_t r = v->nl(v->c);
      while (v->has(v->c)) r = jadd(r, v->nl(v->c));
      return r;
    }
    case TSDB_AGG_SQUARESUM: {  /* :269-277 */
      int64_t x = v->nl(v->c);
      int64_t r = jmul(x, x);
      while (v->has(v->c)) { x = v->nl(v->c); r = jadd(r, jmul(x, x)); }
      return r;
    }
    case TSDB_AGG_MIN: case TSDB_AGG_MIMMIN: {  /* :303-312 */
      int64_t m = v->nl(v->c);
      while (v->has(v->c)) { int64_t x = v->nl(v->c); if (x < m) m = x; }
      return m;
    }
    case TSDB_AGG_MAX: case TSDB_AGG_MIMMAX: {  /* :337-346 */
      int64_t m = v->nl(v->c);
      while (v->has(v->c)) { int64_t x = v->nl(v->c); if (x > m) m = x; }
      return m;
    }
    case TSDB_AGG_AVG: {  /* :371-379 */
      int64_t r = v->nl(v->c);
      int32_t n = 1;
      while (v->has(v->c)) { r = jadd(r, v->nl(v->c)); n++; }
      return jdiv(r, n);
    }
    case TSDB_AGG_MEDIAN: {  /* :403-413 */
      lvec c = {0};
      while (v->has(v->c)) lvec_push(&c, v->nl(v->c));
      if (c.n == 0) { free(c.a); jthrow(TSDB_E_ILLEGAL_STATE, "Shouldn't be here without any data"); }
      qsort(c.a, (size_t)c.n, sizeof(int64_t), cmp_long);
      int64_t r = c.a[c.n / 2];
      free(c.a);
      return r;
    }
    case TSDB_AGG_NONE: {  /* :445-451 */
      int64_t x = v->nl(v->c);
      if (v->has(v->c)) jthrow(TSDB_E_ILLEGAL_DATA, "More than one value in aggregator");
      return x;
    }
    case TSDB_AGG_MULT: {  /* :470-476 */
      int64_t r = v->nl(v->c);
      while (v->has(v->c)) r = jmul(r, v->nl(v->c));
      return r;
    }
    case TSDB_AGG_DEV: {  /* :504-523 */
      double old_mean = (double)v->nl(v->c);
      if (!v->has(v->c)) return 0;
      int64_t n = 2;
      double new_mean = 0., M2 = 0.;
      do {
        const double x = (double)v->nl(v->c);
        new_mean = old_mean + (x - old_mean) / (double)n;
        M2 += (x - old_mean) * (x - new_mean);
        old_mean = new_mean;
        n++;
      } while (v->has(v->c));
      return jd2l(sqrt(M2 / (double)(n - 1)));
    }
    case TSDB_AGG_DIFF: {  /* :582-595 */
      int64_t first = v->nl(v->c);
      if (!v->has(v->c)) return 0;
      int64_t last = 0;
      do { last = v->nl(v->c); } while (v->has(v->c));
      return jsub(last, first);
    }
    case TSDB_AGG_COUNT: {  /* :626-633 */
      int64_t r = 0;
      while (v->has(v->c)) { v->nl(v->c); r++; }
      return r;
    }
    case TSDB_AGG_FIRST: {  /* :815-821 */
      int64_t x = v->nl(v->c);
      while (v->has(v->c)) v->nl(v->c);
      return x;
    }
    case TSDB_AGG_LAST: {  /* :837-843 */
      int64_t x = v->nl(v->c);
      while (v->has(v->c)) x = v->nl(v->c);
      return x;
    }
    default:
      if (is_percentile(a)) {  /* :675-686: runLong honours the estimation type */
        dvec c = {0};
        while (v->has(v->c)) dvec_push(&c, (double)v->nl(v->c));
        double r = percentile_eval(c.a, c.n, pct_value(a), pct_est(a));
        free(c.a);
        return jd2l(r);
      }
  }
  jthrow(TSDB_E_ILLEGAL_ARGUMENT, "bad aggregator %d", a);
}

static double agg_run_double(int a, vals_t* v) {
  switch (a) {
    case TSDB_AGG_SUM: case TSDB_AGG_PFSUM: case TSDB_AGG_ZIMSUM: {  /* :246-259 */
      double r = 0.;
      int64_t n = 0;
      while (v->has(v->c)) {
        const double x = v->nd(v->c);
        if (!isnan(x)) { r += x; ++n; }
      }
      return n == 0 ? NAN : r;
    }
    case TSDB_AGG_SQUARESUM: {  /* :280-293 */
      double r = 0.;
      int64_t n = 0;
      while (v->has(v->c)) {
        const double x = v->nd(v->c);
        if (!isnan(x)) { r += x * x; ++n; }
      }
      return n == 0 ? NAN : r;
    }
    case TSDB_AGG_MIN: case TSDB_AGG_MIMMIN: {  /* :315-327 */
      const double init = v->nd(v->c);
      double m = isnan(init) ? INFINITY : init;
      while (v->has(v->c)) {
        const double x = v->nd(v->c);
        if (!isnan(x) && x < m) m = x;
      }
      return m == INFINITY ? NAN : m;
    }
    case TSDB_AGG_MAX: case TSDB_AGG_MIMMAX: {  /* :349-361 */
      const double init = v->nd(v->c);
      double m = isnan(init) ? -INFINITY : init;
      while (v->has(v->c)) {
        const double x = v->nd(v->c);
        if (!isnan(x) && x > m) m = x;
      }
      return m == -INFINITY ? NAN : m;
    }
    case TSDB_AGG_AVG: {  /* :382-393 */
      double r = 0.;
      int32_t n = 0;
      while (v->has(v->c)) {
        const double x = v->nd(v->c);
        if (!isnan(x)) { r += x; n++; }
      }
      return n == 0 ? NAN : r / (double)n;
    }
    case TSDB_AGG_MEDIAN: {  /* :416-430 */
      dvec c = {0};
      while (v->has(v->c)) { const double x = v->nd(v->c); if (!isnan(x)) dvec_push(&c, x); }
      if (c.n == 0) { free(c.a); return NAN; }
      qsort(c.a, (size_t)c.n, sizeof(double), cmp_double_total);   /* Collections.sort :428 */
      double r = c.a[c.n / 2];
      free(c.a);
      return r;
    }
    case TSDB_AGG_NONE: {  /* :454-460 */
      const double x = v->nd(v->c);
      if (v->has(v->c)) jthrow(TSDB_E_ILLEGAL_DATA, "More than one value in aggregator");
      return x;
    }
    case TSDB_AGG_MULT: {  /* :479-485 */
      double r = v->nd(v->c);
      while (v->has(v->c)) r *= v->nd(v->c);
      return r;
    }
    case TSDB_AGG_DEV: {  /* :526-569 */
      double old_mean = v->nd(v->c);
      while (isnan(old_mean) && v->has(v->c)) old_mean = v->nd(v->c);
      if (isnan(old_mean)) return NAN;
      if (!v->has(v->c)) return 0.;
      int64_t n = 2;
      double new_mean = 0., M2 = 0.;
      do {
        const double x = v->nd(v->c);
        if (!isnan(x)) {
          new_mean = old_mean + (x - old_mean) / (double)n;
          M2 += (x - old_mean) * (x - new_mean);
          old_mean = new_mean;
          n++;
        }
      } while (v->has(v->c));
      return n == 2 ? 0. : sqrt(M2 / (double)(n - 1));
    }
    case TSDB_AGG_DIFF: {  /* :598-617 */
      double first = v->nd(v->c);
      while (isnan(first) && v->has(v->c)) first = v->nd(v->c);
      if (isnan(first)) return NAN;
      if (!v->has(v->c)) return 0.;
      double last = 0.;
      do { last = v->nd(v->c); } while (v->has(v->c));
      return last - first;
    }
    case TSDB_AGG_COUNT: {  /* :636-645 */
      double r = 0;
      while (v->has(v->c)) { const double x = v->nd(v->c); if (!isnan(x)) r++; }
      return r;
    }
    case TSDB_AGG_FIRST: {  /* :823-829 */
      const double x = v->nd(v->c);
      while (v->has(v->c)) v->nd(v->c);
      return x;
    }
    case TSDB_AGG_LAST: {  /* :845-851 */
      double x = v->nd(v->c);
      while (v->has(v->c)) x = v->nd(v->c);
      return x;
    }
    default:
      if (is_percentile(a)) {  /* :689-706: runDouble always LEGACY, NaNs skipped */
        dvec c = {0};
        while (v->has(v->c)) { const double x = v->nd(v->c); if (!isnan(x)) dvec_push(&c, x); }
        if (c.n == 0) { free(c.a); return NAN; }
        double r = percentile_eval(c.a, c.n, pct_value(a), 0);
        free(c.a);
        return r;
      }
  }
  jthrow(TSDB_E_ILLEGAL_ARGUMENT, "bad aggregator %d", a);
}

/* ---- plain arrays (TestAggregators.Numbers) ------------------------------ */
typedef struct { const int64_t* l; const double* d; int64_t n, i; } arr_vals;
static int av_has(void* c) { arr_vals* a = (arr_vals*)c; return a->i < a->n; }
static int64_t av_nl(void* c) {
  arr_vals* a = (arr_vals*)c;
  if (a->i >= a->n) jthrow(TSDB_E_NO_SUCH_ELEMENT, "ArrayIndexOutOfBounds");
  return a->l[a->i++];
}
static double av_nd(void* c) {
  arr_vals* a = (arr_vals*)c;
  if (a->i >= a->n) jthrow(TSDB_E_NO_SUCH_ELEMENT, "ArrayIndexOutOfBounds");
  return a->d[a->i++];
}

int ref_agg_run_long(int32_t aggregator, const int64_t* v, int64_t n, int64_t* out) {
  int rc = 0;
  TRY {
    arr_vals a = {v, NULL, n, 0};
    vals_t vv = {av_has, av_nl, av_nd, &a};
    *out = agg_run_long(aggregator, &vv);
  } CATCH(e) { rc = e; } END_TRY
  return rc;
}
int ref_agg_run_double(int32_t aggregator, const double* v, int64_t n, double* out) {
  int rc = 0;
  TRY {
    arr_vals a = {NULL, v, n, 0};
    vals_t vv = {av_has, av_nl, av_nd, &a};
    *out = agg_run_double(aggregator, &vv);
  } CATCH(e) { rc = e; } END_TRY
  return rc;
}

/* ======================================================================== */
/* ArrayView: SeekableViewsForTest.MockSeekableView / DataPointGenerator      */
/* ======================================================================== */
typedef struct {
  ref_view base;
  ref_dp* dps;
  int64_t n, idx;
  int gen;
} array_view;

static int av_has_next(ref_view* v) { array_view* a = (array_view*)v; return a->idx < a->n; }
static ref_dp av_next(ref_view* v) {
  array_view* a = (array_view*)v;
  if (a->idx >= a->n) jthrow(TSDB_E_NO_SUCH_ELEMENT, "no more values");
  return a->dps[a->idx++];
}
static void av_seek(ref_view* v, int64_t ts) {
  array_view* a = (array_view*)v;
  if (a->gen) {  /* DataPointGenerator.seek: forward only */
    while (a->idx < a->n && a->dps[a->idx].ts < ts) a->idx++;
  } else {       /* MockSeekableView.seek: rescans from 0 */
    for (a->idx = 0; a->idx < a->n; ++a->idx)
      if (a->dps[a->idx].ts >= ts) break;
  }
}
static void av_destroy(ref_view* v) { array_view* a = (array_view*)v; free(a->dps); free(a); }
static const view_vt ARRAY_VT = {av_has_next, av_next, av_seek, av_destroy};

ref_view* ref_view_array(const int64_t* ts, const int32_t* is_int, const int64_t* bits, int64_t n,
                         int generator_seek) {
  array_view* a = (array_view*)calloc(1, sizeof(array_view));
  if (!a) return NULL;
  a->base.vt = &ARRAY_VT;
  a->dps = (ref_dp*)calloc((size_t)(n ? n : 1), sizeof(ref_dp));
  a->n = n;
  a->gen = generator_seek;
  for (int64_t i = 0; i < n; i++) {
    a->dps[i].ts = ts[i];
    a->dps[i].is_int = is_int[i];
    if (is_int[i]) a->dps[i].lv = bits[i];
    else a->dps[i].dv = bitsd((uint64_t)bits[i]);
  }
  return &a->base;
}

/* ======================================================================== */
/* RowSeq + Span.Iterator                                                    */
/* ======================================================================== */
typedef struct {
  int64_t base;          /* seconds */
  const uint8_t* q;
  int64_t qlen;
  const uint8_t* v;
  int64_t vlen;
} rowseq;

static inline uint32_t be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
static inline uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
static inline uint64_t be64(const uint8_t* p) { return ((uint64_t)be32(p) << 32) | be32(p + 4); }
static inline int in_ms(uint8_t b) { return (b & 0xF0) == 0xF0; }  /* Internal.inMilliseconds :621 */

/* Internal.validateQualifier :885-892 + getOffsetFromQualifier :647-658 */
static int64_t row_ts_at_qual(const rowseq* r, int64_t off) {
  if (off < 0 || off >= r->qlen - 1) jthrow(TSDB_E_ILLEGAL_DATA, "Offset of [%lld] is out of bounds", (long long)off);
  if (in_ms(r->q[off])) {
    if (off + 4 > r->qlen) jthrow(TSDB_E_ILLEGAL_DATA, "ArrayIndexOutOfBounds in qualifier");
    return r->base * 1000 + (int64_t)((be32(r->q + off) & 0x0FFFFFC0u) >> 6);
  }
  return r->base * 1000 + (int64_t)(be16(r->q + off) >> 4) * 1000;
}

/* RowSeq.size() :338-356 (including the meta-byte quirk) */
static int64_t row_size(const rowseq* r) {
  if (r->vlen > 0 && (r->v[r->vlen - 1] & 1) == 1) {
    int64_t size = 0;
    for (int64_t i = 0; i < r->qlen; i += 2) {
      if (in_ms(r->q[i])) i += 2;
      size++;
    }
    return size;
  } else if (r->qlen > 0 && in_ms(r->q[0])) {
    return r->qlen / 4;
  }
  return r->qlen / 2;
}

/* RowSeq.timestamp(i) :395-420 */
static int64_t row_timestamp(const rowseq* r, int64_t i) {
  int64_t sz = row_size(r);
  if (i >= sz || i < 0) jthrow(TSDB_E_ILLEGAL_DATA, "IndexOutOfBounds %lld", (long long)i);
  if (r->vlen > 0 && (r->v[r->vlen - 1] & 1) == 1) {
    int64_t index = 0;
    for (int64_t idx = 0; idx < r->qlen; idx += 2) {
      if (i == index) return row_ts_at_qual(r, idx);
      if (in_ms(r->q[idx])) idx += 2;
      index++;
    }
    jthrow(TSDB_E_RUNTIME, "WTF timestamp for index");
  } else if (in_ms(r->q[0])) {
    return row_ts_at_qual(r, i * 4);
  }
  return row_ts_at_qual(r, i * 2);
}

typedef struct {
  const rowseq* r;
  int64_t qi, vi;
  uint32_t qualifier;
} row_it;

static inline int row_it_has(const row_it* it) { return it->qi < it->r->qlen; }

static void row_it_advance(row_it* it) {  /* shared body of next() and seek() */
  const rowseq* r = it->r;
  if (in_ms(r->q[it->qi])) {
    if (it->qi + 4 > r->qlen) jthrow(TSDB_E_ILLEGAL_DATA, "ArrayIndexOutOfBounds in qualifier");
    it->qualifier = be32(r->q + it->qi);
    it->qi += 4;
  } else {
    if (it->qi + 2 > r->qlen) jthrow(TSDB_E_ILLEGAL_DATA, "ArrayIndexOutOfBounds in qualifier");
    it->qualifier = be16(r->q + it->qi);
    it->qi += 2;
  }
  const uint32_t flags = it->qualifier & 0xFF;
  it->vi += (flags & 7) + 1;
}

/* RowSeq.Iterator.next() :552-568 + DataPoint accessors :605-639 */
static ref_dp row_it_next(row_it* it) {
  if (!row_it_has(it)) jthrow(TSDB_E_NO_SUCH_ELEMENT, "no more elements");
  row_it_advance(it);
  const rowseq* r = it->r;
  const uint32_t q = it->qualifier;
  ref_dp d;
  memset(&d, 0, sizeof d);
  if ((q & 0xF0000000u) == 0xF0000000u)
    d.ts = r->base * 1000 + (int64_t)((q & 0x0FFFFFC0u) >> 6);
  else
    d.ts = (r->base + (int64_t)((q & 0xFFFF) >> 4)) * 1000;
  d.is_int = (q & 0x8) == 0;
  const uint32_t flags = q & 0xFF;
  const int64_t vlen = (flags & 7) + 1;
  const int64_t at = it->vi - vlen;
  if (at < 0 || at + vlen > r->vlen) { d.bad = TSDB_E_ILLEGAL_DATA; return d; }
  const uint8_t* p = r->v + at;
  if (d.is_int) {  /* extractIntegerValue :233-245 */
    switch (flags & 7) {
      case 7: d.lv = (int64_t)be64(p); break;
      case 3: d.lv = (int32_t)be32(p); break;
      case 1: d.lv = (int16_t)be16(p); break;
      case 0: d.lv = (int8_t)p[0]; break;
      default: d.bad = TSDB_E_ILLEGAL_DATA;
    }
  } else {         /* extractFloatingPointValue :256-266 */
    switch (flags & 7) {
      case 7: d.dv = bitsd(be64(p)); break;
      case 3: { uint32_t u = be32(p); float f; memcpy(&f, &u, 4); d.dv = (double)f; break; }
      default: d.bad = TSDB_E_ILLEGAL_DATA;
    }
  }
  return d;
}

/* RowSeq.Iterator.seek :578-599 */
static void row_it_seek(row_it* it, int64_t ts) {
  if ((ts & (int64_t)0xFFFFF00000000000LL) != 0) jthrow(TSDB_E_ILLEGAL_ARGUMENT, "invalid timestamp: %lld", (long long)ts);
  it->qi = 0;
  it->vi = 0;
  while (it->qi < it->r->qlen && row_ts_at_qual(it->r, it->qi) < ts) row_it_advance(it);
}

typedef struct {
  ref_view base;
  rowseq* rows;
  int64_t nrows;
  int64_t row_index;
  row_it cur;
  uint8_t** owned;      /* merged cells (RowSeq.addRow) owned by the span */
  int64_t n_owned;
} span_view;

static int sv_has_next(ref_view* v) {  /* Span.Iterator.hasNext :421-435 */
  span_view* s = (span_view*)v;
  if (row_it_has(&s->cur)) return 1;
  while (s->row_index < s->nrows - 1) {
    s->row_index++;
    s->cur.r = &s->rows[s->row_index];
    s->cur.qi = s->cur.vi = 0;
    s->cur.qualifier = 0;
    if (row_it_has(&s->cur)) return 1;
  }
  return 0;
}
static ref_dp sv_next(ref_view* v) {  /* :438-452 */
  span_view* s = (span_view*)v;
  if (row_it_has(&s->cur)) return row_it_next(&s->cur);
  while (s->row_index < s->nrows - 1) {
    s->row_index++;
    s->cur.r = &s->rows[s->row_index];
    s->cur.qi = s->cur.vi = 0;
    s->cur.qualifier = 0;
    if (row_it_has(&s->cur)) return row_it_next(&s->cur);
  }
  jthrow(TSDB_E_NO_SUCH_ELEMENT, "no more elements");
}
static void sv_seek(ref_view* v, int64_t ts) {  /* :464-471 with seekRow :360-380 */
  span_view* s = (span_view*)v;
  int64_t ri = 0;
  for (int64_t i = 0; i < s->nrows; i++) {
    const int64_t sz = row_size(&s->rows[i]);
    if (sz < 1) ri++;
    else if (row_timestamp(&s->rows[i], sz - 1) < ts) ri++;
    else break;
  }
  if (ri == s->nrows) --ri;
  if (ri != s->row_index) {
    s->row_index = ri;
    s->cur.r = &s->rows[ri];
    s->cur.qi = s->cur.vi = 0;
  }
  row_it_seek(&s->cur, ts);
}
static void sv_destroy(ref_view* v) {
  span_view* s = (span_view*)v;
  for (int64_t i = 0; i < s->n_owned; i++) free(s->owned[i]);
  free(s->owned);
  free(s->rows);
  free(s);
}
static const view_vt SPAN_VT = {sv_has_next, sv_next, sv_seek, sv_destroy};

static int cmp_rowseq(const void* a, const void* b) {
  const rowseq* x = (const rowseq*)a;
  const rowseq* y = (const rowseq*)b;
  return x->base < y->base ? -1 : (x->base > y->base ? 1 : 0);
}

/* Internal.getQualifierLength :712-727 / getValueLengthFromQualifier :680-690 */
static int64_t qual_len_at(const uint8_t* q, int64_t i) { return in_ms(q[i]) ? 4 : 2; }
static int64_t val_len_at(const uint8_t* q, int64_t i) { return (q[i + qual_len_at(q, i) - 1] & 7) + 1; }
static int64_t qual_offset_ms(const uint8_t* q, int64_t i) {   /* getOffsetFromQualifier :647-658 */
  return in_ms(q[i]) ? (int64_t)((be32(q + i) & 0x0FFFFFC0u) >> 6) : (int64_t)(be16(q + i) >> 4) * 1000;
}

/* RowSeq.addRow :91-222: ordered merge of the remote cell into the local one by qualifier
 * offset (Internal.compareQualifiers :511-519); on equal offsets the remote datapoint is
 * dropped; the meta byte is MS_MIXED_COMPACT if either side has it. */
static void rowseq_merge(span_view* s, rowseq* local, const rowseq* remote) {
  const int64_t ql = local->qlen, rql = remote->qlen;
  uint8_t* mq = (uint8_t*)xcalloc((size_t)(ql + rql + 1), 1);
  uint8_t* mv = (uint8_t*)xcalloc((size_t)(local->vlen + remote->vlen + 1), 1);
  int64_t li = 0, ri = 0, mi = 0, lv = 0, rv = 0, mvi = 0;
  while (ri < rql || li < ql) {
    int take_remote;
    if (ri >= rql) take_remote = 0;
    else if (li >= ql) take_remote = 1;
    else {
      const int64_t a = qual_offset_ms(remote->q, ri), b = qual_offset_ms(local->q, li);
      if (a == b) {   /* duplicate: skip the remote one */
        rv += val_len_at(remote->q, ri);
        ri += qual_len_at(remote->q, ri);
        continue;
      }
      take_remote = a < b;
    }
    const uint8_t* q = take_remote ? remote->q : local->q;
    const uint8_t* v = take_remote ? remote->v : local->v;
    int64_t* qi = take_remote ? &ri : &li;
    int64_t* vi = take_remote ? &rv : &lv;
    const int64_t vl = val_len_at(q, *qi), qlen = qual_len_at(q, *qi);
    if (*vi + vl > (take_remote ? remote->vlen : local->vlen)) jthrow(TSDB_E_ILLEGAL_DATA, "value out of bounds in addRow");
    memcpy(mv + mvi, v + *vi, (size_t)vl);
    memcpy(mq + mi, q + *qi, (size_t)qlen);
    *vi += vl;
    mvi += vl;
    *qi += qlen;
    mi += qlen;
  }
  const uint8_t meta_l = local->vlen ? local->v[local->vlen - 1] : 0;
  const uint8_t meta_r = remote->vlen ? remote->v[remote->vlen - 1] : 0;
  mv[mvi] = ((meta_l & 1) || (meta_r & 1)) ? 1 : 0;   /* Const.MS_MIXED_COMPACT */
  s->owned = (uint8_t**)realloc(s->owned, (size_t)(s->n_owned + 2) * sizeof(uint8_t*));
  s->owned[s->n_owned++] = mq;
  s->owned[s->n_owned++] = mv;
  local->q = mq;
  local->qlen = mi;
  local->v = mv;
  local->vlen = mvi + 1;
}

static ref_view* make_span(int64_t n_rows, const uint32_t* base_time, const uint64_t* qual_off,
                           const uint64_t* val_off, const uint8_t* qual, const uint8_t* val,
                           const int64_t* row_ids) {
  span_view* s = (span_view*)xcalloc(1, sizeof(span_view));
  s->base.vt = &SPAN_VT;
  s->rows = (rowseq*)xcalloc((size_t)(n_rows ? n_rows : 1), sizeof(rowseq));
  s->nrows = 0;
  /* Span.addRow :177-220 in arrival order: a cell whose first timestamp is not after the
   * last row's last one merges into the row with the same key (same series, same base) */
  for (int64_t i = 0; i < n_rows; i++) {
    const int64_t r = row_ids ? row_ids[i] : i;
    rowseq nr;
    nr.base = base_time[r];
    nr.q = qual + qual_off[r];
    nr.qlen = (int64_t)(qual_off[r + 1] - qual_off[r]);
    nr.v = val + val_off[r];
    nr.vlen = (int64_t)(val_off[r + 1] - val_off[r]);
    if (s->nrows > 0) {
      const rowseq* last = &s->rows[s->nrows - 1];
      const int64_t last_ts = row_timestamp(last, row_size(last) - 1);
      if (last_ts >= row_timestamp(&nr, 0)) {
        int64_t j = 0;
        for (; j < s->nrows; j++) if (s->rows[j].base == nr.base) break;
        if (j < s->nrows) { rowseq_merge(s, &s->rows[j], &nr); continue; }
      }
    }
    s->rows[s->nrows++] = nr;
  }
  n_rows = s->nrows;
  /* Span.checkRowOrder: Collections.sort (stable) by base time */
  int sorted = 1;
  for (int64_t i = 1; i < n_rows; i++) if (s->rows[i].base < s->rows[i - 1].base) sorted = 0;
  if (!sorted) {
    /* insertion sort keeps it stable */
    for (int64_t i = 1; i < n_rows; i++) {
      rowseq t = s->rows[i];
      int64_t j = i - 1;
      while (j >= 0 && cmp_rowseq(&s->rows[j], &t) > 0) { s->rows[j + 1] = s->rows[j]; j--; }
      s->rows[j + 1] = t;
    }
  }
  s->row_index = 0;
  s->cur.r = &s->rows[0];
  return &s->base;
}

ref_view* ref_view_span(int64_t n_rows, const uint32_t* base_time, const uint64_t* qual_off,
                        const uint64_t* val_off, const uint8_t* qual, const uint8_t* val) {
  ref_view* r = NULL;
  TRY { r = make_span(n_rows, base_time, qual_off, val_off, qual, val, NULL); } CATCH(e) { (void)e; r = NULL; } END_TRY
  return r;
}

/* Span first / last timestamps (Span.timestamp(0), Span.timestamp(size-1), :279-285) */
static void span_first_last(span_view* s, int64_t* first, int64_t* last, int64_t* size) {
  int64_t total = 0;
  for (int64_t i = 0; i < s->nrows; i++) total += row_size(&s->rows[i]);
  *size = total;
  if (total == 0) return;
  /* getIdxOffsetFor(i) */
  int64_t idx = 0, off = 0;
  for (idx = 0; idx < s->nrows; idx++) { if (row_size(&s->rows[idx]) > 0) break; }
  *first = row_timestamp(&s->rows[idx], 0);
  int64_t want = total - 1;
  off = 0;
  for (idx = 0; idx < s->nrows; idx++) {
    const int64_t sz = row_size(&s->rows[idx]);
    if (off + sz > want) break;
    off += sz;
  }
  *last = row_timestamp(&s->rows[idx], want - off);
}

/* ======================================================================== */
/* Query-time compaction: CompactionQueue.Compaction (src/core/CompactionQueue.java:267-626,  */
/* default merge, no write-back), ColumnDatapointIterator (src/core/ColumnDatapointIterator    */
/* .java:63-205), AppendDataPoints.parseKeyValue (src/core/AppendDataPoints.java:110-240) and  */
/* the float / flag fixups (src/core/Internal.java:535-591).                                  */
/* ======================================================================== */
typedef struct {
  uint8_t* q;          /* (fixed) qualifier, owned */
  int64_t qlen;
  uint8_t* v;          /* (fixed) value, owned */
  int64_t vlen;
  int64_t ts;          /* KeyValue.timestamp() */
  int64_t order;       /* position in the row (tie-break of equal (offset, timestamp)) */
  int64_t qi, vi;      /* qualifier_offset, value_offset */
  int cur_qlen, cur_vlen, is_ms;
  int64_t cur_off;     /* current_timestamp_offset (ms) */
  int needs_fixup;
} cdi;

static int cdi_update(cdi* c) {   /* ColumnDatapointIterator.update :150-166 */
  if (c->qi >= c->qlen || c->vi >= c->vlen) return 0;
  if (in_ms(c->q[c->qi])) {
    if (c->qi + 4 > c->qlen) jthrow(TSDB_E_ILLEGAL_DATA, "ArrayIndexOutOfBounds in a compacted qualifier");
    c->cur_qlen = 4;
    c->is_ms = 1;
    c->cur_off = (int64_t)((be32(c->q + c->qi) & 0x0FFFFFC0u) >> 6);
  } else {
    c->cur_qlen = 2;
    c->is_ms = 0;
    c->cur_off = (int64_t)(be16(c->q + c->qi) >> 4) * 1000;
  }
  c->cur_vlen = (c->q[c->qi + c->cur_qlen - 1] & 7) + 1;
  return 1;
}
static int cdi_advance(cdi* c) {   /* :141-145 */
  c->qi += c->cur_qlen;
  c->vi += c->cur_vlen;
  return cdi_update(c);
}
/* heap order :181-189: offset ascending, column timestamp descending (the entry kept first);
 * equal pairs by position in the row (PriorityQueue leaves them unordered) */
static int cdi_less(const cdi* a, const cdi* b) {
  if (a->cur_off != b->cur_off) return a->cur_off < b->cur_off;
  if (a->ts != b->ts) return a->ts > b->ts;
  return a->order < b->order;
}

static void cdi_init(cdi* c, const uint8_t* q, int64_t qlen, const uint8_t* v, int64_t vlen, int64_t ts, int64_t order) {
  memset(c, 0, sizeof *c);
  c->q = (uint8_t*)xmalloc((size_t)(qlen ? qlen : 1));
  c->v = (uint8_t*)xmalloc((size_t)(vlen ? vlen : 1));
  if (qlen) memcpy(c->q, q, (size_t)qlen);
  if (vlen) memcpy(c->v, v, (size_t)vlen);
  c->qlen = qlen;
  c->vlen = vlen;
  c->ts = ts;
  c->order = order;
  if (qlen == 2) {   /* checkForFixup :74-89 (fixups predate compaction: 2-byte qualifiers only) */
    const uint8_t qual1 = c->q[1];
    if ((qual1 & 0x8) && (qual1 & 7) == 3 && c->vlen == 8) {   /* floatingPointValueToFix */
      if (c->v[0] || c->v[1] || c->v[2] || c->v[3])
        jthrow(TSDB_E_ILLEGAL_DATA, "Corrupted floating point value -- first 4 bytes are expected to be zeros");
      memmove(c->v, c->v + 4, 4);
      c->vlen = 4;
      c->needs_fixup = 1;
    }
    const uint8_t len_byte = (uint8_t)((qual1 & ~7) | (uint8_t)(c->vlen - 1));   /* fixQualifierFlags */
    if (len_byte != qual1) {
      c->q[1] = len_byte;
      c->needs_fixup = 1;
    }
  }
  cdi_update(c);
}

/* AppendDataPoints.parseKeyValue: the (qualifier, value) pairs of an append column, a later
 * pair replacing an earlier one of the same offset, sorted by offset */
static void parse_append(const uint8_t* v, int64_t vlen, uint8_t** oq, int64_t* oql, uint8_t** ov, int64_t* ovl) {
  typedef struct { int64_t delta; int64_t qo, ql, vo, vl; } apc;
  apc* cells = (apc*)xcalloc((size_t)(vlen + 1), sizeof(apc));
  int64_t n = 0, idx = 0;
  while (idx < vlen) {
    const int64_t ql = in_ms(v[idx]) ? 4 : 2;
    if (idx + ql > vlen) { free(cells); jthrow(TSDB_E_ILLEGAL_DATA, "Corrupted value: couldn't break down into individual values"); }
    const int64_t vl = (v[idx + ql - 1] & 7) + 1;
    if (idx + ql + vl > vlen) { free(cells); jthrow(TSDB_E_ILLEGAL_DATA, "Corrupted value: couldn't break down into individual values"); }
    const int64_t delta = ql == 4 ? (int64_t)((be32(v + idx) & 0x0FFFFFC0u) >> 6) : (int64_t)(be16(v + idx) >> 4) * 1000;
    int64_t j = 0;
    for (; j < n; j++) if (cells[j].delta == delta) break;
    cells[j].delta = delta;
    cells[j].qo = idx;
    cells[j].ql = ql;
    cells[j].vo = idx + ql;
    cells[j].vl = vl;
    if (j == n) n++;
    idx += ql + vl;
  }
  for (int64_t i = 1; i < n; i++) {   /* TreeMap order */
    apc t = cells[i];
    int64_t j = i - 1;
    while (j >= 0 && cells[j].delta > t.delta) { cells[j + 1] = cells[j]; j--; }
    cells[j + 1] = t;
  }
  int64_t tq = 0, tv = 0;
  for (int64_t i = 0; i < n; i++) { tq += cells[i].ql; tv += cells[i].vl; }
  *oq = (uint8_t*)xmalloc((size_t)(tq ? tq : 1));
  *ov = (uint8_t*)xmalloc((size_t)(tv ? tv : 1));
  int64_t a = 0, b = 0;
  for (int64_t i = 0; i < n; i++) {
    memcpy(*oq + a, v + cells[i].qo, (size_t)cells[i].ql);
    memcpy(*ov + b, v + cells[i].vo, (size_t)cells[i].vl);
    a += cells[i].ql;
    b += cells[i].vl;
  }
  *oql = tq;
  *ovl = tv;
  free(cells);
}

/* Compaction.compact() as TSDB.compact(row) returns it to a query (SaltScanner.processRow
 * :802-830).  Returns 1 with the compacted cell in out_q / out_v (malloc'd), 0 when the row
 * has no datapoint (compacted == null), or a negative TSDB_E_* code. */
/* ColumnDatapointIterator.getCellValueAsDouble :201-211 of the current datapoint (fixups applied):
 * ByteBuffer.getFloat / getDouble / get / getShort / getInt / getLong by its value length; a float of
 * a length other than 4 or 8, or an integer of 3, 5, 6 or 7 bytes, reads past the copy
 * (BufferUnderflowException, a RuntimeException) */
static int cdi_dval(const cdi* c, double* out) {
  const uint8_t* v = c->v + c->vi;
  const int64_t n = c->cur_vlen;
  if (c->q[c->qi + c->cur_qlen - 1] & 0x8) {   /* Internal.isFloat of the current qualifier */
    if (n == 4) {
      const uint32_t b = be32(v);
      float f;
      memcpy(&f, &b, 4);
      *out = (double)f;
      return 1;
    }
    if (n == 8) {
      const uint64_t b = ((uint64_t)be32(v) << 32) | be32(v + 4);
      memcpy(out, &b, 8);
      return 1;
    }
    return 0;
  }
  if (n == 1) *out = (double)(int8_t)v[0];
  else if (n == 2) *out = (double)(int16_t)be16(v);
  else if (n == 4) *out = (double)(int32_t)be32(v);
  else if (n == 8) *out = (double)(int64_t)(((uint64_t)be32(v) << 32) | be32(v + 4));
  else return 0;
  return 1;
}
#define DTCS_UNDERFLOW(c) \
  do { free(live); jthrow(TSDB_E_RUNTIME, "BufferUnderflowException: a %lld-byte value in getCellValueAsDouble", (long long)(c)->cur_vlen); } while (0)

/* dtcs: 0 = defaultMergeDataPoints; 1 / 2 = dtcsMergeDataPoints (tsd.storage.use_otsdb_timestamp)
 * keeping the max / the min value (tsd.storage.use_max_value true / false) */
int ref_compact_row(int64_t ncols, const uint8_t* const* quals, const int64_t* qlens, const uint8_t* const* vals,
                    const int64_t* vlens, const int64_t* col_ts, int fix_duplicates, int dtcs, uint8_t** out_q,
                    int64_t* out_qlen, uint8_t** out_v, int64_t* out_vlen) {
  cdi* volatile cols = NULL;
  volatile int64_t n = 0;
  volatile int rc = 0;
  *out_q = *out_v = NULL;
  *out_qlen = *out_vlen = 0;
  TRY {
    cols = (cdi*)xcalloc((size_t)(ncols ? ncols : 1), sizeof(cdi));
    int64_t first_dp = -1;    /* findFirstDatapointColumn :389-399 */
    int appended = 0;
    for (int64_t i = 0; i < ncols; i++) {   /* buildHeapProcessAnnotations :401-452 */
      const int64_t ql = qlens[i];
      if (ql & 1) {
        if (ql == 3 && quals[i][0] == 0x05) {   /* AppendDataPoints.APPEND_COLUMN_PREFIX */
          uint8_t *aq, *av;
          int64_t aql, avl;
          parse_append(vals[i], vlens[i], &aq, &aql, &av, &avl);
          cdi_init(&cols[n], aq, aql, av, avl, col_ts ? col_ts[i] : 0, i);
          free(aq);
          free(av);
          appended = 1;
          first_dp = n;
          if (cols[n].qlen > 0) n++;
          else { free(cols[n].q); free(cols[n].v); }
        }
        continue;   /* annotations, histograms, unknown prefixes */
      }
      if (first_dp < 0 && !appended) first_dp = n;
      cdi_init(&cols[n], quals[i], ql, vals[i], vlens[i], col_ts ? col_ts[i] : 0, i);
      if (cols[n].qlen > 0) n++;
      else { free(cols[n].q); free(cols[n].v); }
    }
    if (n == 0) {
      rc = 0;
    } else if (n == 1 && (cols[0].qlen == 2 || (cols[0].qlen == 4 && in_ms(cols[0].q[0]))) && !cols[0].needs_fixup) {
      /* noMergesOrFixups :311-328: the single column as stored (or as parsed from the append) */
      if (cols[0].vlen == 0) jthrow(TSDB_E_ILLEGAL_DATA, "empty value");
      *out_q = (uint8_t*)xmalloc((size_t)cols[0].qlen);
      *out_v = (uint8_t*)xmalloc((size_t)cols[0].vlen);
      memcpy(*out_q, cols[0].q, (size_t)cols[0].qlen);
      memcpy(*out_v, cols[0].v, (size_t)cols[0].vlen);
      *out_qlen = cols[0].qlen;
      *out_vlen = cols[0].vlen;
      rc = 1;
    } else {
      /* defaultMergeDataPoints :512-545 over the heap of columns */
      int64_t tq = 0, tv = 0;
      for (int64_t i = 0; i < n; i++) { tq += cols[i].qlen; tv += cols[i].vlen; }
      uint8_t* cq = (uint8_t*)xmalloc((size_t)tq + 1);
      uint8_t* cv = (uint8_t*)xmalloc((size_t)tv + 2);
      *out_q = cq;
      *out_v = cv;
      int64_t qo = 0, vo = 0, segs = 0, last_vo = 0, last_vl = 0, prev = -1;
      int ms_in_row = 0, s_in_row = 0;
      int* live = (int*)xcalloc((size_t)n, sizeof(int));
      for (int64_t i = 0; i < n; i++) live[i] = cols[i].vlen > 0 && cols[i].qi < cols[i].qlen;
      for (int64_t i = 0; i < n; i++)
        if (!live[i]) { free(live); jthrow(TSDB_E_ILLEGAL_DATA, "empty value"); }
      if (dtcs) {
        /* dtcsMergeDataPoints :508-547.  col1 = the heap's head; its value and position are taken
         * before it advances; every further column at the same offset (heap order: newest column
         * first) replaces it when its value is strictly greater (use_max_value) / smaller.  No
         * duplicate exception.  ms_in_row / s_in_row read the winner's isMilliseconds() AFTER it
         * advanced (:544-545): the resolution of its next datapoint, or of its last one. */
        for (;;) {
          int64_t best = -1;
          for (int64_t i = 0; i < n; i++)
            if (live[i] && (best < 0 || cdi_less(&cols[i], &cols[best]))) best = i;
          if (best < 0) break;
          cdi* c1 = &cols[best];
          if (c1->vi + c1->cur_vlen > c1->vlen) { free(live); jthrow(TSDB_E_ILLEGAL_DATA, "value shorter than its qualifiers"); }
          int64_t w = best, wqi = c1->qi, wvi = c1->vi, wql = c1->cur_qlen, wvl = c1->cur_vlen;
          const int64_t ts1 = c1->cur_off;
          double v1 = 0, v2 = 0;
          if (!cdi_dval(c1, &v1)) DTCS_UNDERFLOW(c1);
          live[best] = cdi_advance(c1);
          for (;;) {
            int64_t b2 = -1;
            for (int64_t i = 0; i < n; i++)
              if (live[i] && (b2 < 0 || cdi_less(&cols[i], &cols[b2]))) b2 = i;
            if (b2 < 0 || cols[b2].cur_off != ts1) break;
            cdi* c2 = &cols[b2];
            if (c2->vi + c2->cur_vlen > c2->vlen) { free(live); jthrow(TSDB_E_ILLEGAL_DATA, "value shorter than its qualifiers"); }
            if (!cdi_dval(c2, &v2)) DTCS_UNDERFLOW(c2);
            if ((dtcs == 1 && v2 > v1) || (dtcs != 1 && v1 > v2)) {
              w = b2; v1 = v2;
              wqi = c2->qi; wvi = c2->vi; wql = c2->cur_qlen; wvl = c2->cur_vlen;
            }
            live[b2] = cdi_advance(c2);
          }
          memcpy(cq + qo, cols[w].q + wqi, (size_t)wql);   /* writeToBuffersFromOffset */
          memcpy(cv + vo, cols[w].v + wvi, (size_t)wvl);
          qo += wql;
          vo += wvl;
          segs++;
          if (cols[w].is_ms) ms_in_row = 1; else s_in_row = 1;
        }
      }
      for (; !dtcs;) {
        int64_t best = -1;
        for (int64_t i = 0; i < n; i++)
          if (live[i] && (best < 0 || cdi_less(&cols[i], &cols[best]))) best = i;
        if (best < 0) break;
        cdi* c = &cols[best];
        if (c->vi + c->cur_vlen > c->vlen) { free(live); jthrow(TSDB_E_ILLEGAL_DATA, "value shorter than its qualifiers"); }
        if (c->cur_off == prev) {
          /* getCopyOfCurrentValue vs the last segment written */
          if (c->cur_vlen != last_vl || memcmp(c->v + c->vi, cv + last_vo, (size_t)last_vl) != 0) {
            if (!fix_duplicates) {
              free(live);
              jthrow(TSDB_E_ILLEGAL_DATA, "Duplicate timestamp for key, ms_offset=%lld; set tsd.storage.fix_duplicates=true",
                     (long long)c->cur_off);
            }
          }
        } else {
          prev = c->cur_off;
          memcpy(cq + qo, c->q + c->qi, (size_t)c->cur_qlen);   /* writeToBuffers */
          memcpy(cv + vo, c->v + c->vi, (size_t)c->cur_vlen);
          last_vo = vo;
          last_vl = c->cur_vlen;
          qo += c->cur_qlen;
          vo += c->cur_vlen;
          segs++;
          if (c->is_ms) ms_in_row = 1; else s_in_row = 1;
        }
        live[best] = cdi_advance(c);
      }
      free(live);
      if (segs > 1) cv[vo++] = (ms_in_row && s_in_row) ? 1 : 0;   /* buildCompactedColumn :547-566 */
      *out_qlen = qo;
      *out_vlen = vo;
      rc = 1;
    }
  } CATCH(e) {
    rc = e;
    free(*out_q);
    free(*out_v);
    *out_q = *out_v = NULL;
  } END_TRY
  if (cols) {
    for (int64_t i = 0; i < n; i++) { free(cols[i].q); free(cols[i].v); }
    free(cols);
  }
  return rc;
}
void ref_free(void* p) { free(p); }

/* ======================================================================== */
/* RollupSpan + RollupSeq (src/rollup/RollupSpan.java, src/rollup/RollupSeq.java) */
/* ======================================================================== */
/* A RollupSeq row: the queried aggregate's cells and (need_count) the count cells, each a
 * 2-byte rollup qualifier (offset << 4 | flags) and its value bytes. */
typedef struct { uint32_t q; const uint8_t* v; } ro_cell;
typedef struct {
  int64_t base;
  ro_cell* vc;
  int64_t nv, capv;
  ro_cell* cc;
  int64_t nc, capc;
  int64_t last_off, last_coff;   /* RollupSeq.last_offset / last_count_offset */
} ro_row;

static inline int64_t ro_off(uint32_t q) { return (int64_t)((q & 0xFFFF) >> 4); }
static int64_t cal_fdiv(int64_t a, int64_t b);
static int64_t days_from_civil(int64_t y, int m, int d);
static void civil_from_days(int64_t z, int64_t* y, int* m, int* d);

/* RollupSeq.append :238-318.  The batch carries no HBase write timestamps: a repeated offset
 * under fix_duplicates takes the "equal timestamps" branch (the later cell replaces the
 * earlier one, :257-266 / :290-299). */
static void ro_append(ro_row* r, uint32_t q, const uint8_t* v, int is_count, int fix_dup) {
  const int64_t off = ro_off(q);
  int64_t* last = is_count ? &r->last_coff : &r->last_off;
  if (*last > -1 && off <= *last) {
    if (off == *last && fix_dup) {
      if (is_count) r->nc--; else r->nv--;
    } else if (is_count) {
      jthrow(TSDB_E_ILLEGAL_ARGUMENT, "The count offset of %lld is <= the last offset %lld", (long long)off, (long long)*last);
    } else {
      jthrow(TSDB_E_ILLEGAL_DATA, "The offset of %lld is <= the last offset %lld", (long long)off, (long long)*last);
    }
  }
  *last = off;
  ro_cell** a = is_count ? &r->cc : &r->vc;
  int64_t* n = is_count ? &r->nc : &r->nv;
  int64_t* cap = is_count ? &r->capc : &r->capv;
  if (*n == *cap) {
    *cap = *cap ? *cap * 2 : 16;
    *a = (ro_cell*)realloc(*a, (size_t)*cap * sizeof(ro_cell));
    if (!*a) jthrow(TSDB_E_NOMEM, "oom");
  }
  (*a)[*n].q = q;
  (*a)[*n].v = v;
  (*n)++;
}

/* the cells of batch row r (2-byte qualifiers, values back to back) appended to `row` */
static void ro_append_cells(ro_row* row, const uint64_t* qoff, const uint64_t* voff, const uint8_t* qual,
                            const uint8_t* val, int64_t r, int is_count, int fix_dup) {
  const int64_t ql = (int64_t)(qoff[r + 1] - qoff[r]), vl = (int64_t)(voff[r + 1] - voff[r]);
  if (ql % 2) jthrow(TSDB_E_ILLEGAL_DATA, "rollup qualifiers are 2 bytes");
  int64_t vi = 0;
  for (int64_t i = 0; i < ql; i += 2) {
    const uint32_t q = be16(qual + qoff[r] + i);
    const int64_t len = (q & 7) + 1;   /* Internal.getValueLengthFromQualifier */
    if (vi + len > vl) jthrow(TSDB_E_ILLEGAL_DATA, "rollup value bytes shorter than the qualifiers say");
    ro_append(row, q, val + voff[r] + vi, is_count, fix_dup);
    vi += len;
  }
  if (vi != vl) jthrow(TSDB_E_ILLEGAL_DATA, "rollup value bytes longer than the qualifiers say");
}

typedef struct {
  ref_view base;
  ro_row* rows;
  int64_t nrows;
  int need_count;
  int64_t interval_ms;
  int64_t row_index;
  int64_t qi, ci;   /* RollupIterator.qual_index / count_qual_index, in cells */
} ro_span;

/* RollupIterator.sync :521-555 */
static void ro_sync(const ro_row* r, int64_t* qi, int64_t* ci) {
  while (*qi < r->nv && *ci < r->nc) {
    const int64_t a = ro_off(r->vc[*qi].q), b = ro_off(r->cc[*ci].q);
    if (a == b) return;
    if (a > b) (*ci)++;
    else (*qi)++;
  }
}
/* RollupIterator.hasNext :512-519 */
static int ro_row_has(const ro_row* r, int need_count, int64_t* qi, int64_t* ci) {
  if (!need_count) return *qi < r->nv;
  ro_sync(r, qi, ci);
  return *qi < r->nv && *ci < r->nc;
}
static inline int64_t ro_ts(const ro_span* s, const ro_row* r, uint32_t q) {  /* getTimestampFromRollupQualifier :193-197 */
  return r->base * 1000 + ro_off(q) * s->interval_ms;
}
/* RollupIterator.next :557-572 and the DataPoint accessors :641-700 */
static ref_dp ro_row_next(ro_span* s, const ro_row* r) {
  if (!ro_row_has(r, s->need_count, &s->qi, &s->ci)) jthrow(TSDB_E_NO_SUCH_ELEMENT, "no more elements");
  const ro_cell* c = &r->vc[s->qi++];
  ref_dp d;
  memset(&d, 0, sizeof d);
  d.ts = ro_ts(s, r, c->q);
  d.is_int = (c->q & 0x8) == 0;
  const uint8_t* p = c->v;
  if (d.is_int) {   /* Internal.extractIntegerValue */
    switch (c->q & 7) {
      case 7: d.lv = (int64_t)be64(p); break;
      case 3: d.lv = (int32_t)be32(p); break;
      case 1: d.lv = (int16_t)be16(p); break;
      case 0: d.lv = (int8_t)p[0]; break;
      default: d.bad = TSDB_E_ILLEGAL_DATA;
    }
  } else {          /* Internal.extractFloatingPointValue */
    switch (c->q & 7) {
      case 7: d.dv = bitsd(be64(p)); break;
      case 3: { uint32_t u = be32(p); float f; memcpy(&f, &u, 4); d.dv = (double)f; break; }
      default: d.bad = TSDB_E_ILLEGAL_DATA;
    }
  }
  d.cnt = 1;   /* valueCount() without count cells */
  if (s->need_count) {
    const ro_cell* k = &r->cc[s->ci++];
    const uint8_t* kp = k->v;
    if ((k->q & 0x8) == 0) {
      switch (k->q & 7) {
        case 7: d.cnt = (int64_t)be64(kp); break;
        case 3: d.cnt = (int32_t)be32(kp); break;
        case 1: d.cnt = (int16_t)be16(kp); break;
        case 0: d.cnt = (int8_t)kp[0]; break;
        default: d.cnt_bad = TSDB_E_ILLEGAL_DATA;
      }
    } else {        /* (long) of the float count */
      double x;
      switch (k->q & 7) {
        case 7: x = bitsd(be64(kp)); break;
        case 3: { uint32_t u = be32(kp); float f; memcpy(&f, &u, 4); x = (double)f; break; }
        default: x = 0; d.cnt_bad = TSDB_E_ILLEGAL_DATA;
      }
      /* Java's (long) of a double: NaN -> 0, saturating */
      d.cnt = x != x ? 0 : (x >= 9.2233720368547758e18 ? INT64_MAX : (x <= -9.2233720368547758e18 ? INT64_MIN : (int64_t)x));
    }
  }
  return d;
}
/* RollupIterator.seek :578-609: reset, then walk the value cells with the count cells in
 * lock step (not re-synced during the walk) */
static void ro_row_seek(ro_span* s, const ro_row* r, int64_t ts) {
  if ((ts & (int64_t)0xFFFFFFFF00000000LL) == 0) ts *= 1000;
  s->qi = s->ci = 0;
  if (!ro_row_has(r, s->need_count, &s->qi, &s->ci)) return;
  while (s->qi < r->nv && ro_ts(s, r, r->vc[s->qi].q) < ts) {
    s->qi++;
    if (s->need_count) s->ci++;
  }
}
/* RollupSeq.size() / timestamp(size - 1) (:420-470): datapoints a fresh iterator yields */
static int64_t ro_row_size(const ro_span* s, const ro_row* r, int64_t* last_ts, int64_t* first_ts) {
  int64_t qi = 0, ci = 0, n = 0;
  while (ro_row_has(r, s->need_count, &qi, &ci)) {
    const int64_t t = ro_ts(s, r, r->vc[qi].q);
    if (n == 0 && first_ts) *first_ts = t;
    if (last_ts) *last_ts = t;
    qi++;
    if (s->need_count) ci++;
    n++;
  }
  return n;
}
static void ro_new_row_it(ro_span* s) {   /* RollupIterator() :507-510 */
  s->qi = s->ci = 0;
  if (s->need_count && s->nrows) ro_sync(&s->rows[s->row_index], &s->qi, &s->ci);
}
static int ros_has_next(ref_view* v) {  /* Span.Iterator.hasNext :421-435 */
  ro_span* s = (ro_span*)v;
  if (s->nrows == 0) return 0;
  if (ro_row_has(&s->rows[s->row_index], s->need_count, &s->qi, &s->ci)) return 1;
  while (s->row_index < s->nrows - 1) {
    s->row_index++;
    ro_new_row_it(s);
    if (ro_row_has(&s->rows[s->row_index], s->need_count, &s->qi, &s->ci)) return 1;
  }
  return 0;
}
static ref_dp ros_next(ref_view* v) {  /* :438-452 */
  ro_span* s = (ro_span*)v;
  if (s->nrows && ro_row_has(&s->rows[s->row_index], s->need_count, &s->qi, &s->ci))
    return ro_row_next(s, &s->rows[s->row_index]);
  while (s->row_index < s->nrows - 1) {
    s->row_index++;
    ro_new_row_it(s);
    if (ro_row_has(&s->rows[s->row_index], s->need_count, &s->qi, &s->ci)) return ro_row_next(s, &s->rows[s->row_index]);
  }
  jthrow(TSDB_E_NO_SUCH_ELEMENT, "no more elements");
}
static void ros_seek(ref_view* v, int64_t ts) {  /* :464-471 with seekRow :360-380 */
  ro_span* s = (ro_span*)v;
  if (s->nrows == 0) return;
  int64_t ri = 0;
  for (int64_t i = 0; i < s->nrows; i++) {
    int64_t last = 0;
    const int64_t sz = ro_row_size(s, &s->rows[i], &last, NULL);
    if (sz < 1) ri++;
    else if (last < ts) ri++;
    else break;
  }
  if (ri == s->nrows) --ri;
  if (ri != s->row_index) {
    s->row_index = ri;
    ro_new_row_it(s);
  }
  ro_row_seek(s, &s->rows[s->row_index], ts);
}
static void ro_rows_free(ro_row* rows, int64_t n) {
  for (int64_t i = 0; i < n; i++) { free(rows[i].vc); free(rows[i].cc); }
  free(rows);
}
static void ros_destroy(ref_view* v) {
  ro_span* s = (ro_span*)v;
  ro_rows_free(s->rows, s->nrows);
  free(s);
}
static const view_vt ROLLUP_SPAN_VT = {ros_has_next, ros_next, ros_seek, ros_destroy};

/* RollupSpan.addRow :62-80 over the span's rows in scan order (a row with the last row's key
 * appends its cells to that RollupSeq, RollupSeq.addRow :170-205), then Span.checkRowOrder's
 * stable sort by base time.  Throws as RollupSeq.append does. */
static ref_view* make_rollup_span(const tsdbhip_rollup_batch* rb, const int64_t* row_ids, int64_t n_rows) {
  const tsdbhip_batch* b = &rb->cells;
  ro_span* s = (ro_span*)xcalloc(1, sizeof(ro_span));
  s->base.vt = &ROLLUP_SPAN_VT;
  s->need_count = rb->row_cqual_off != NULL;
  s->interval_ms = (int64_t)rb->interval.interval_s * 1000;
  s->rows = (ro_row*)xcalloc((size_t)(n_rows ? n_rows : 1), sizeof(ro_row));
  volatile int err = 0;
  TRY {
    for (int64_t i = 0; i < n_rows; i++) {
      const int64_t r = row_ids[i];
      ro_row* row;
      if (s->nrows > 0 && s->rows[s->nrows - 1].base == (int64_t)b->row_base_time[r]) {
        row = &s->rows[s->nrows - 1];
      } else {
        row = &s->rows[s->nrows++];
        row->base = b->row_base_time[r];
        row->last_off = row->last_coff = -1;
      }
      ro_append_cells(row, b->row_qual_off, b->row_val_off, b->qual, b->val, r, 0, rb->fix_duplicates);
      if (s->need_count) ro_append_cells(row, rb->row_cqual_off, rb->row_cval_off, rb->cqual, rb->cval, r, 1, rb->fix_duplicates);
    }
  } CATCH(e) { err = e; } END_TRY
  if (err) {
    ro_rows_free(s->rows, s->nrows);
    free(s);
    jthrow(err, "%s", g_msg);
  }
  for (int64_t i = 1; i < s->nrows; i++) {   /* stable insertion sort by base */
    ro_row t = s->rows[i];
    int64_t j = i - 1;
    while (j >= 0 && s->rows[j].base > t.base) { s->rows[j + 1] = s->rows[j]; j--; }
    s->rows[j + 1] = t;
  }
  s->row_index = 0;
  ro_new_row_it(s);
  return &s->base;
}

/* Span.size() / timestamp(0) / timestamp(size - 1) of a rollup span */
static void rollup_span_first_last(ro_span* s, int64_t* first, int64_t* last, int64_t* size) {
  int64_t total = 0, f = 0, l = 0;
  for (int64_t i = 0; i < s->nrows; i++) {
    int64_t fi = 0, li = 0;
    const int64_t n = ro_row_size(s, &s->rows[i], &li, &fi);
    if (n == 0) continue;
    if (total == 0) f = fi;
    l = li;
    total += n;
  }
  *size = total;
  *first = f;
  *last = l;
}

/* RollupUtils.getRollupBasetime :52-112 (int result) */
static int64_t ro_basetime(int64_t ts, const tsdbhip_rollup_interval* iv) {
  if (ts < 0) jthrow(TSDB_E_ILLEGAL_ARGUMENT, "Not supporting negative timestamps at this time: %lld", (long long)ts);
  if (iv->units == 'h') {
    const int64_t modulo = iv->unit_multiplier > 1 ? (int64_t)iv->unit_multiplier * 3600 : 3600;
    const int64_t t = (ts & (int64_t)0xFFFFFFFF00000000LL) ? ts / 1000 : ts;
    return (int32_t)(uint32_t)(t - t % modulo);
  }
  const int64_t ms = (ts & (int64_t)0xFFFFFFFF00000000LL) ? ts : ts * 1000;
  const int64_t day = cal_fdiv(ms, 86400000LL);
  const int64_t msod = ms - day * 86400000LL;
  int64_t y;
  int m, d;
  civil_from_days(day, &y, &m, &d);
  int64_t z;
  switch (iv->units) {
    case 'd': z = day; break;
    case 'n': z = days_from_civil(y, m, 1); break;
    case 'y': z = days_from_civil(y, 1, 1); break;
    default: jthrow(TSDB_E_ILLEGAL_ARGUMENT, "Unrecogznied span");
  }
  /* HOUR_OF_DAY / MINUTE / SECOND zeroed, the milliseconds kept, then / 1000 */
  return (int32_t)(uint32_t)((z * 86400000LL + msod % 1000) / 1000);
}

/* ======================================================================== */
/* UTC calendar (java.util.GregorianCalendar in the UTC zone, default US locale: weeks   */
/* start on Sunday) -- the arithmetic DateTime.previousInterval and the calendar          */
/* Downsampler / FillingDownsampler use (src/utils/DateTime.java:445-606,                 */
/* src/core/Downsampler.java:131-147,336-350,390-400,420-432,446-447,                     */
/* src/core/FillingDownsampler.java:113-135,280-286).                                     */
/* ======================================================================== */
static const int64_t CAL_UNIT_MS[9] = {0, 1, 1000, 60000, 3600000, 86400000, 604800000, 2592000000LL, 31536000000LL};

static int cal_unit_of(const char* dur) {  /* suffix of a parseDuration string */
  size_t l = strlen(dur);
  if (l >= 2 && strcasecmp(dur + l - 2, "ms") == 0) return TSDB_CAL_MS;
  if (l == 0) return 0;
  switch (dur[l - 1]) {
    case 's': return TSDB_CAL_S;
    case 'm': return TSDB_CAL_M;
    case 'h': return TSDB_CAL_H;
    case 'd': return TSDB_CAL_D;
    case 'w': return TSDB_CAL_W;
    case 'n': return TSDB_CAL_N;
    case 'y': return TSDB_CAL_Y;
  }
  return 0;
}

static int64_t cal_fdiv(int64_t a, int64_t b) { int64_t q = a / b; if ((a % b) && ((a < 0) != (b < 0))) q--; return q; }
/* days since 1970-01-01 of a proleptic Gregorian civil date, and back */
static int64_t days_from_civil(int64_t y, int m, int d) {
  y -= m <= 2;
  const int64_t era = cal_fdiv(y, 400);
  const int64_t yoe = y - era * 400;
  const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}
static void civil_from_days(int64_t z, int64_t* y, int* m, int* d) {
  z += 719468;
  const int64_t era = cal_fdiv(z, 146097);
  const int64_t doe = z - era * 146097;
  const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const int64_t mp = (5 * doy + 2) / 153;
  *d = (int)(doy - (153 * mp + 2) / 5 + 1);
  *m = (int)(mp < 10 ? mp + 3 : mp - 9);
  *y = yoe + era * 400 + (*m <= 2);
}
static int month_days(int64_t y, int m) {
  static const int md[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  const int leap = (y % 4 == 0 && y % 100 != 0) || y % 400 == 0;
  return m == 2 ? 28 + leap : md[m - 1];
}
/* ---- time zone (ZoneInfo restated over the host's tsdbhip_tz table) ------- */
/* ZoneInfo.getOffsets(date, UTC_TIME): the offset of the last transition at or before t */
static int32_t tz_off_utc(const tsdbhip_tz* z, int64_t t) {
  if (!z) return 0;
  int lo = 0, hi = z->n - 1, idx = -1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    if (z->utc_ms[mid] <= t) { idx = mid; lo = mid + 1; }
    else hi = mid - 1;
  }
  return z->offset_ms[idx + 1];
}
/* ZoneInfo.getOffsetsByWall (getTransitionIndex with WALL_TIME): a transition's wall time is
 * its instant plus the offset that starts there; a wall time in a spring-forward gap takes
 * the old offset, one in a fall-back overlap the new one */
static int32_t tz_off_wall(const tsdbhip_tz* z, int64_t w) {
  if (!z) return 0;
  int lo = 0, hi = z->n - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    const int64_t mv = z->utc_ms[mid] + z->offset_ms[mid + 1];
    if (mv < w) lo = mid + 1;
    else if (mv > w) hi = mid - 1;
    else return z->offset_ms[mid + 1];
  }
  if (lo >= z->n) return z->offset_ms[z->n];
  return lo - 1 < 0 ? z->offset_ms[0] : z->offset_ms[lo];
}
/* GregorianCalendar.computeTime from local wall-clock fields */
static int64_t tz_from_wall(const tsdbhip_tz* z, int64_t w) { return w - tz_off_wall(z, w); }

/* GregorianCalendar.add(unit, n) in zone z: ms / s / m / h add absolute milliseconds;
 * days keep the local time of day and re-adjust for an offset change (the previous instant if
 * the adjustment changes the date); months / years move the local date, pin the day of month
 * and recompute the instant from the wall-clock fields */
static int64_t cal_add(int64_t ts, int unit, int64_t n, const tsdbhip_tz* z) {
  if (unit != TSDB_CAL_N && unit != TSDB_CAL_Y && unit != TSDB_CAL_D) return ts + n * CAL_UNIT_MS[unit];
  const int64_t off = tz_off_utc(z, ts);
  const int64_t loc = ts + off;
  int64_t fd = cal_fdiv(loc, 86400000);
  const int64_t tod = loc - fd * 86400000;
  if (unit == TSDB_CAL_D) {
    fd += n;
    const int64_t t1 = fd * 86400000 + tod - off;
    const int64_t diff = off - tz_off_utc(z, t1);
    if (diff == 0) return t1;
    const int64_t t2 = t1 + diff;
    return cal_fdiv(t2 + tz_off_utc(z, t2), 86400000) != fd ? t1 : t2;
  }
  int64_t y; int m, d;
  civil_from_days(fd, &y, &m, &d);
  if (unit == TSDB_CAL_N) {
    const int64_t mm = y * 12 + (m - 1) + n;
    y = cal_fdiv(mm, 12);
    m = (int)(mm - y * 12) + 1;
  } else {
    y += n;
  }
  const int ml = month_days(y, m);
  if (d > ml) d = ml;   /* add() pins the day of month */
  return tz_from_wall(z, days_from_civil(y, m, d) * 86400000 + tod);
}
/* one Downsampler step: interval units, or interval * WEEK_LENGTH days for weeks */
static int64_t cal_step(int64_t ts, int unit, int64_t n, int sign, const tsdbhip_tz* z) {
  if (unit == TSDB_CAL_W) return cal_add(ts, TSDB_CAL_D, sign * n * 7, z);
  return cal_add(ts, unit, sign * n, z);
}
/* DateTime.previousInterval(ts, interval, unit, tz) :445-606: the set() calls zero local
 * fields (the instant is recomputed from the wall clock), the adds run in zone z */
static int64_t cal_prev(int64_t ts, int64_t n, int unit, const tsdbhip_tz* z) {
  if (ts < 0) jthrow(TSDB_E_ILLEGAL_ARGUMENT, "Timestamp cannot be less than zero");
  if (n < 1) jthrow(TSDB_E_ILLEGAL_ARGUMENT, "Interval must be greater than zero");
  int uo = unit;
  int64_t io = n;
  const int64_t loc = ts + tz_off_utc(z, ts);
  const int64_t day = cal_fdiv(loc, 86400000);
  const int64_t tod = loc - day * 86400000;
  int64_t y; int m, d;
  civil_from_days(day, &y, &m, &d);
  int64_t c;
  switch (unit) {
    case TSDB_CAL_MS:
      if (1000 % n == 0) { c = tz_from_wall(z, loc - tod % 1000); if (n > 1000) c -= n; }
      else c = tz_from_wall(z, loc - tod % 60000);
      break;
    case TSDB_CAL_S:
      if (60 % n == 0) { c = tz_from_wall(z, loc - tod % 60000); if (n > 60) c -= n * 1000; }
      else c = tz_from_wall(z, loc - tod % 3600000);
      break;
    case TSDB_CAL_M:
      if (60 % n == 0) { c = tz_from_wall(z, loc - tod % 3600000); if (n > 60) c -= n * 60000; }
      else c = tz_from_wall(z, day * 86400000);
      break;
    case TSDB_CAL_H:
      if (24 % n == 0) { c = tz_from_wall(z, day * 86400000); if (n > 24) c -= n * 3600000; }
      else c = tz_from_wall(z, days_from_civil(y, m, 1) * 86400000);
      break;
    case TSDB_CAL_D:
      if (n == 1) c = tz_from_wall(z, days_from_civil(y, m, 1) * 86400000);
      else c = tz_from_wall(z, days_from_civil(y, 1, 1) * 86400000);
      break;
    case TSDB_CAL_W:
      if (2 % n == 0) {
        /* set(DAY_OF_WEEK, SUNDAY): the Sunday of the Sunday-first week (1970-01-04 was one) */
        const int64_t dow = ((day - 3) % 7 + 7) % 7;
        c = tz_from_wall(z, (day - dow) * 86400000);
      } else {
        /* set(MONTH, 0) then set(DAY_OF_WEEK, SUNDAY): GregorianCalendar.computeTime resolves
         * YEAR + MONTH + WEEK_OF_MONTH + DAY_OF_WEEK (Calendar.selectFields: the WEEK_OF_MONTH
         * pattern carries the newest stamp, DAY_OF_WEEK's).  WEEK_OF_MONTH is still the computed
         * week of ts in its own month (getWeekNumber, minimal days 1): week w of January. */
        const int64_t dow1 = ((days_from_civil(y, m, 1) - 3) % 7 + 7) % 7;
        const int64_t wom = (day - (days_from_civil(y, m, 1) - dow1)) / 7 + 1;
        const int64_t j1 = days_from_civil(y, 1, 1);
        const int64_t jdow = ((j1 - 3) % 7 + 7) % 7;
        c = tz_from_wall(z, (j1 - jdow + 7 * (wom - 1)) * 86400000);
      }
      uo = TSDB_CAL_D;   /* the loop steps 7 days whatever the interval */
      io = 7;
      break;
    default:   /* MONTH, YEAR: from the top of the year */
      c = tz_from_wall(z, days_from_civil(y, 1, 1) * 86400000);
      break;
  }
  if (c == ts) return c;
  while (c <= ts) c = cal_add(c, uo, io, z);
  return cal_add(c, uo, -io, z);
}

int ref_cal_prev_ex(int64_t ts, int64_t n, int unit, const tsdbhip_tz* z, int64_t* out) {
  int rc = 0;
  TRY { *out = cal_prev(ts, n, unit, z); }
  CATCH(code) { rc = code; }
  END_TRY
  return rc;
}
int ref_cal_step_ex(int64_t ts, int unit, int64_t n, const tsdbhip_tz* z, int64_t* out) {
  int rc = 0;
  TRY { *out = cal_step(ts, unit, n, 1, z); }
  CATCH(code) { rc = code; }
  END_TRY
  return rc;
}

/* ======================================================================== */
/* Downsampler / FillingDownsampler                                          */
/* ======================================================================== */
typedef struct {
  ref_view base;
  ref_view* src;
  int32_t fn;
  int64_t interval;
  int32_t fill;
  int32_t run_all;
  int64_t qs, qe;
  int filling;
  int64_t timestamp;      /* Downsampler.timestamp (also FillingDownsampler's expected ts) */
  double value;
  int64_t end_timestamp;  /* FillingDownsampler */
  /* ValuesInInterval */
  int64_t tei;
  int has_src;
  ref_dp next_dp;
  int next_dp_null;
  int initialized;
  /* useCalendar: unit, interval count, Downsampler.previous_calendar / next_calendar, and
   * FillingDownsampler's own previous_calendar / next_calendar (FillingDownsampler.java:38-41) */
  int cal;
  int64_t cal_n;
  const tsdbhip_tz* tz;   /* DownsamplingSpecification.getTimezone (NULL = UTC) */
  int32_t rollup_agg;     /* RollupQuery.getRollupAgg (-1: not a rollup query) */
  int64_t prev_cal, next_cal;
  int64_t fprev_cal, fnext_cal;
} ds_view;

static inline int64_t ds_align(ds_view* d, int64_t t) { return t - (t % d->interval); }

static void viv_move_to_next_value(ds_view* d) {  /* :357-382 */
  if (v_has_next(d->src)) {
    d->has_src = 1;
    if (d->run_all) {
      while (v_has_next(d->src)) {
        d->next_dp = v_next(d->src);
        d->next_dp_null = 0;
        if (d->next_dp.ts < d->qs) { d->next_dp_null = 1; continue; }
        if (d->next_dp.ts >= d->qe) d->has_src = 0;
        break;
      }
      if (d->next_dp_null) d->has_src = 0;
    } else {
      d->next_dp = v_next(d->src);
      d->next_dp_null = 0;
    }
  } else {
    d->has_src = 0;
  }
}
static void viv_init(ds_view* d) {  /* :327-354 */
  if (!d->initialized) {
    d->initialized = 1;
    if (v_has_next(d->src)) {
      viv_move_to_next_value(d);
      if (!d->run_all) {
        if (d->cal) {
          d->prev_cal = cal_prev(d->next_dp.ts, d->cal_n, d->cal, d->tz);
          d->next_cal = cal_step(d->prev_cal, d->cal, d->cal_n, 1, d->tz);
          d->tei = d->next_cal;
        } else {
          d->tei = ds_align(d, d->next_dp.ts) + d->interval;
        }
      }
    }
  }
}
static void viv_reset_end(ds_view* d) {  /* :388-406 */
  if (d->has_src && !d->run_all) {
    if (d->cal) {
      while (d->next_dp.ts >= d->tei) {
        d->prev_cal = cal_step(d->prev_cal, d->cal, d->cal_n, 1, d->tz);
        d->next_cal = cal_step(d->next_cal, d->cal, d->cal_n, 1, d->tz);
        d->tei = d->next_cal;
      }
    } else {
      d->tei = ds_align(d, d->next_dp.ts) + d->interval;
    }
  }
}
static void viv_move_to_next_interval(ds_view* d) { viv_init(d); viv_reset_end(d); }
static void viv_seek(ds_view* d, int64_t ts) {  /* :415-437 */
  if (d->run_all) {
    v_seek(d->src, ts);
  } else if (d->cal) {
    int64_t sc = cal_prev(ts, d->cal_n, d->cal, d->tz);
    if (ts > sc) sc = cal_step(sc, d->cal, d->cal_n, 1, d->tz);
    v_seek(d->src, sc);
  } else {
    v_seek(d->src, ds_align(d, ts + d->interval - 1));
  }
  d->initialized = 0;
}
static int64_t viv_interval_ts(ds_view* d) {  /* :440-452 */
  if (d->run_all) return d->tei;
  if (d->cal) return d->prev_cal;
  return ds_align(d, d->tei - d->interval);
}
static int viv_has(void* c) {  /* :464-471 */
  ds_view* d = (ds_view*)c;
  viv_init(d);
  if (d->run_all) return d->has_src;
  return d->has_src && d->next_dp.ts < d->tei;
}
static double viv_nd(void* c) {  /* :474-482 */
  ds_view* d = (ds_view*)c;
  if (viv_has(c)) {
    const double v = dp_to_double(&d->next_dp);
    viv_move_to_next_value(d);
    return v;
  }
  jthrow(TSDB_E_NO_SUCH_ELEMENT, "no more values in interval of %lld", (long long)d->tei);
}
static int64_t viv_nl(void* c) { (void)c; jthrow(TSDB_E_CLASS_CAST, "ValuesInInterval is Doubles only"); }

/* Downsampler.next :165-221 / FillingDownsampler.next :196-253: the bucket value, with the
 * rollup branches -- avg rollups: avg downsampling is Σsum / Σcount (0 when the count is 0),
 * any other function runs on each point's sum / count; count downsampling of a rollup sums
 * valueCount() (consuming the values) */
static int64_t ds_value_count(ds_view* d) {   /* ValuesInInterval.nextValueCount :484-493 */
  if (!viv_has(d)) jthrow(TSDB_E_NO_SUCH_ELEMENT, "no more values in interval");
  if (d->next_dp.cnt_bad) jthrow(d->next_dp.cnt_bad, "bad count value");
  return d->next_dp.cnt;
}
static double ds_bucket_value(ds_view* d, vals_t* vv) {
  if (d->rollup_agg == TSDB_AGG_AVG) {
    if (d->fn == TSDB_AGG_AVG) {
      double sum = 0;
      int64_t count = 0;
      while (viv_has(d)) {
        count += ds_value_count(d);
        sum += viv_nd(d);
      }
      return count == 0 ? 0.0 : sum / (double)count;
    }
    double* acc = NULL;
    int64_t n = 0, cap = 0;
    while (viv_has(d)) {
      const int64_t count = ds_value_count(d);
      const double sum = viv_nd(d);
      if (n == cap) {
        cap = cap ? cap * 2 : 64;
        acc = (double*)realloc(acc, (size_t)cap * 8);
        if (!acc) jthrow(TSDB_E_NOMEM, "oom");
      }
      acc[n++] = count == 0 ? 0.0 : sum / (double)count;
    }
    arr_vals a = {NULL, acc, n, 0};
    vals_t av = {av_has, av_nl, av_nd, &a};
    volatile double r = 0;
    volatile int err = 0;
    TRY { r = agg_run_double(d->fn, &av); } CATCH(e) { err = e; } END_TRY
    free(acc);
    if (err) jthrow(err, "%s", g_msg);
    return r;
  }
  if (d->rollup_agg == TSDB_AGG_DEV)
    jthrow(TSDB_E_UNSUPPORTED, "Standard deviation over rolled up data is not supported at this time");
  if (d->rollup_agg >= 0 && d->fn == TSDB_AGG_COUNT) {
    double count = 0;
    while (viv_has(d)) {
      count += (double)ds_value_count(d);
      viv_nd(d);
    }
    return count;
  }
  return agg_run_double(d->fn, vv);
}

static int ds_has_next(ref_view* v) {
  ds_view* d = (ds_view*)v;
  if (!d->filling) return viv_has(d);                 /* Downsampler.hasNext :155-157 */
  if (d->run_all) return viv_has(d);                  /* FillingDownsampler.hasNext :153-161 */
  return d->timestamp < d->end_timestamp;
}

static ref_dp ds_next(ref_view* v) {
  ds_view* d = (ds_view*)v;
  vals_t vv = {viv_has, viv_nl, viv_nd, d};
  if (!d->filling) {  /* Downsampler.next :163-231 (rollup branches not reachable) */
    if (!viv_has(d)) jthrow(TSDB_E_NO_SUCH_ELEMENT, "no more data points");
    d->value = ds_bucket_value(d, &vv);
    d->timestamp = viv_interval_ts(d);
    viv_move_to_next_interval(d);
    return dp_of_double(d->run_all ? d->qs : d->timestamp, d->value);
  }
  /* FillingDownsampler.next :172-301 */
  if (!ds_has_next(v)) jthrow(TSDB_E_NO_SUCH_ELEMENT, "no more data points");
  viv_init(d);
  int64_t actual = viv_has(d) ? viv_interval_ts(d) : LONG_MAX_J;
  while (!d->run_all && viv_has(d) && actual < d->timestamp) {
    agg_run_double(d->fn, &vv);
    viv_move_to_next_interval(d);
    actual = viv_interval_ts(d);
  }
  if (d->run_all || actual == d->timestamp) {
    d->value = ds_bucket_value(d, &vv);
    viv_move_to_next_interval(d);
  } else {
    switch (d->fill) {
      case TSDB_FILL_NAN: case TSDB_FILL_NULL: d->value = NAN; break;
      case TSDB_FILL_ZERO: d->value = 0.0; break;
      default: jthrow(TSDB_E_RUNTIME, "unhandled fill policy");
    }
  }
  if (d->run_all) return dp_of_double(d->qs, d->value);
  if (d->cal) {   /* advance :280-286; timestamp() = previous_calendar :304-311 */
    d->fprev_cal = cal_step(d->fprev_cal, d->cal, d->cal_n, 1, d->tz);
    d->fnext_cal = cal_step(d->fnext_cal, d->cal, d->cal_n, 1, d->tz);
    d->timestamp = d->fnext_cal;
    return dp_of_double(d->fprev_cal, d->value);
  }
  d->timestamp += d->interval;
  return dp_of_double(d->timestamp - d->interval, d->value);
}
static void ds_seek(ref_view* v, int64_t ts) { viv_seek((ds_view*)v, ts); }
static void ds_destroy(ref_view* v) { ds_view* d = (ds_view*)v; ref_view_free(d->src); free(d); }
static const view_vt DS_VT = {ds_has_next, ds_next, ds_seek, ds_destroy};

static ref_view* make_downsampler(ref_view* src, int32_t function, int64_t interval_ms, int32_t fill,
                                  int32_t run_all, int64_t start_time, int64_t end_time,
                                  int64_t query_start, int64_t query_end, int32_t calendar,
                                  const tsdbhip_tz* tz) {
  if (function == TSDB_AGG_NONE) jthrow(TSDB_E_ILLEGAL_ARGUMENT, "cannot use the NONE aggregator for downsampling");
  if (!run_all && interval_ms <= 0) jthrow(TSDB_E_ILLEGAL_ARGUMENT, "interval not > 0");
  ds_view* d = (ds_view*)xcalloc(1, sizeof(ds_view));
  d->base.vt = &DS_VT;
  d->src = src;
  d->fn = function;
  d->tz = tz;
  d->rollup_agg = -1;
  d->interval = interval_ms;
  d->fill = fill;
  d->run_all = run_all;
  d->qs = query_start;
  d->qe = query_end;
  d->filling = fill != TSDB_FILL_NONE;   /* Span.downsampler :545-560 */
  d->next_dp_null = 1;
  d->tei = run_all ? query_end : interval_ms;  /* ValuesInInterval() :318-324 */
  if (calendar && !run_all) {   /* Downsampler ctor :131-142 */
    if (calendar < TSDB_CAL_MS || calendar > TSDB_CAL_Y) jthrow(TSDB_E_ILLEGAL_ARGUMENT, "Unrecognized unit type");
    d->cal = calendar;
    d->cal_n = interval_ms / CAL_UNIT_MS[calendar];
  }
  if (d->filling) {
    if (run_all) {
      d->timestamp = start_time;
      d->end_timestamp = end_time;
    } else if (d->cal) {   /* FillingDownsampler ctor :113-135 */
      d->fnext_cal = cal_prev(start_time, d->cal_n, d->cal, d->tz);
      d->fprev_cal = cal_step(d->fnext_cal, d->cal, d->cal_n, -1, d->tz);
      int64_t end_cal = cal_prev(end_time, d->cal_n, d->cal, d->tz);
      if (end_cal == d->fnext_cal) end_cal = cal_step(end_cal, d->cal, d->cal_n, 1, d->tz);
      d->timestamp = d->fnext_cal;
      d->end_timestamp = end_cal;
    } else {
      d->timestamp = ds_align(d, start_time);
      d->end_timestamp = ds_align(d, end_time);
    }
  }
  return &d->base;
}

ref_view* ref_view_downsampler_tz(ref_view* src, int32_t function, int64_t interval_ms, int32_t fill,
                                  int32_t run_all, int64_t start_time, int64_t end_time,
                                  int64_t query_start, int64_t query_end, int32_t calendar, const tsdbhip_tz* tz) {
  ref_view* r = NULL;
  TRY { r = make_downsampler(src, function, interval_ms, fill, run_all, start_time, end_time, query_start, query_end, calendar, tz); }
  CATCH(e) { (void)e; r = NULL; } END_TRY
  return r;
}
ref_view* ref_view_downsampler(ref_view* src, int32_t function, int64_t interval_ms, int32_t fill,
                               int32_t run_all, int64_t start_time, int64_t end_time,
                               int64_t query_start, int64_t query_end, int32_t calendar) {
  return ref_view_downsampler_tz(src, function, interval_ms, fill, run_all, start_time, end_time, query_start,
                                 query_end, calendar, NULL);
}

/* ======================================================================== */
/* RateSpan                                                                  */
/* ======================================================================== */
typedef struct {
  ref_view base;
  ref_view* src;
  int32_t counter, drop;
  int64_t counter_max, reset_value;
  ref_dp next_data, next_rate, prev_rate;
  int initialized;
} rate_view;

static void rate_populate(rate_view* r) {  /* :121-180; the drop-resets recursion as a loop */
  for (;;) {
    if (!v_has_next(r->src)) {
      r->next_rate = dp_of_long(LONG_MAX_J, 0);
      return;
    }
    const ref_dp prev = r->next_data;
    ref_dp nd = v_next(r->src);
    r->next_data = dp_copy_eager(&nd);
    const ref_dp* next = &r->next_data;
    const int64_t t0 = prev.ts, t1 = next->ts;
    if (t1 <= t0) jthrow(TSDB_E_ILLEGAL_STATE, "Next timestamp (%lld) is supposed to be strictly greater than the previous one (%lld)", (long long)t1, (long long)t0);
    const double dt = (double)(t1 - t0) / 1000.0;
    double diff;
    if (prev.is_int && next->is_int) diff = (double)jsub(next->lv, prev.lv);
    else diff = dp_to_double(next) - dp_to_double(&prev);
    if (r->counter && diff < 0) {
      if (r->drop) continue;
      if (prev.is_int && next->is_int) diff = (double)jadd(jsub(r->counter_max, prev.lv), next->lv);
      else diff = (double)r->counter_max - dp_to_double(&prev) + dp_to_double(next);
      const double rate = diff / dt;
      if (r->reset_value > 0 && rate > (double)r->reset_value) r->next_rate = dp_of_double(next->ts, 0.0);
      else r->next_rate = dp_of_double(next->ts, rate);
    } else {
      r->next_rate = dp_of_double(next->ts, diff / dt);
    }
    return;
  }
}
static void rate_init(rate_view* r) {  /* :103-116 */
  if (!r->initialized) {
    r->initialized = 1;
    r->next_data = dp_of_long(0, 0);
    rate_populate(r);
  }
}
static int rv_has_next(ref_view* v) { rate_view* r = (rate_view*)v; rate_init(r); return r->next_rate.ts != LONG_MAX_J; }
static ref_dp rv_next(ref_view* v) {
  rate_view* r = (rate_view*)v;
  rate_init(r);
  if (!rv_has_next(v)) jthrow(TSDB_E_NO_SUCH_ELEMENT, "no more values");
  r->prev_rate = r->next_rate;
  rate_populate(r);
  return r->prev_rate;
}
static void rv_seek(ref_view* v, int64_t ts) { rate_view* r = (rate_view*)v; v_seek(r->src, ts); r->initialized = 0; }
static void rv_destroy(ref_view* v) { rate_view* r = (rate_view*)v; ref_view_free(r->src); free(r); }
static const view_vt RATE_VT = {rv_has_next, rv_next, rv_seek, rv_destroy};

ref_view* ref_view_rate(ref_view* src, int32_t counter, int64_t counter_max, int64_t reset_value,
                        int32_t drop_resets) {
  rate_view* r = (rate_view*)calloc(1, sizeof(rate_view));
  if (!r) return NULL;
  r->base.vt = &RATE_VT;
  r->src = src;
  r->counter = counter;
  r->counter_max = counter_max;
  r->reset_value = reset_value;
  r->drop = drop_resets;
  return &r->base;
}

/* ======================================================================== */
/* AggregationIterator                                                       */
/* ======================================================================== */
#define FLAG_FLOAT ((int64_t)0x8000000000000000ULL)
#define TIME_MASK ((int64_t)0x7FFFFFFFFFFFFFFFLL)
#define MILLISECOND_MASK ((int64_t)0xFFFFF00000000000ULL)

typedef struct {
  ref_view base;
  ref_view** its;
  ref_view** owned;
  int64_t k;
  int64_t start, end;
  int32_t agg, interp, rate;
  int64_t* ts;
  int64_t* vals;
  int64_t current, pos;
  ref_dp out;   /* heap-resident: survives longjmp */
} agg_view;

static void ai_end_reached(agg_view* a, int64_t i) { a->ts[a->k + i] = TIME_MASK; a->its[i] = NULL; }
static void ai_put(agg_view* a, int64_t i, const ref_dp* dp) {  /* :482-494 */
  a->ts[i] = dp->ts;
  if (dp->is_int) {
    a->vals[i] = dp_long(dp);
  } else {
    a->vals[i] = (int64_t)dbits(dp_double(dp));
    a->ts[i] |= FLAG_FLOAT;
  }
}
static void ai_move_to_next(agg_view* a, int64_t i) {  /* :573-588 */
  const int64_t nx = a->k + i;
  a->ts[i] = a->ts[nx];
  a->vals[i] = a->vals[nx];
  ref_view* it = a->its[i];
  if (!it) jthrow(TSDB_E_ILLEGAL_STATE, "NullPointerException: iterator %lld already ended", (long long)i);
  if (v_has_next(it)) {
    ref_dp d = v_next(it);
    ai_put(a, nx, &d);
  } else {
    ai_end_reached(a, i);
  }
}
static int ai_has_next(ref_view* v) {  /* :500-512 */
  agg_view* a = (agg_view*)v;
  for (int64_t i = 0; i < a->k; i++)
    if ((a->ts[a->k + i] & TIME_MASK) <= a->end) return 1;
  return 0;
}
static int ai_is_integer(agg_view* a) {  /* :612-625 */
  if (a->rate) return 0;
  for (int64_t i = 2 * a->k - 1; i >= 0; i--)
    if ((a->ts[i] & FLAG_FLOAT) == FLAG_FLOAT) return 0;
  return 1;
}
static int ai_has_next_value_upd(agg_view* a, int upd) {  /* :667-680 */
  for (int64_t i = a->pos + 1; i < a->k; i++) {
    if (a->ts[i] != 0) {
      if (upd) a->pos = i;
      return 1;
    }
  }
  return 0;
}
static int ai_has_value(void* c) { return ai_has_next_value_upd((agg_view*)c, 0); }
static int64_t ai_next_long(void* c) {  /* :682-729 */
  agg_view* a = (agg_view*)c;
  if (!ai_has_next_value_upd(a, 1)) jthrow(TSDB_E_NO_SUCH_ELEMENT, "no more longs");
  const int64_t pos = a->pos;
  const int64_t y0 = a->vals[pos];
  if (a->rate) jthrow(TSDB_E_ASSERTION, "Should not be here, impossible!");
  if (a->current == pos) return y0;
  const int64_t x = a->ts[a->current] & TIME_MASK;
  const int64_t x0 = a->ts[pos] & TIME_MASK;
  if (x == x0) return y0;
  const int64_t y1 = a->vals[pos + a->k];
  const int64_t x1 = a->ts[pos + a->k] & TIME_MASK;
  if (x == x1) return y1;
  if ((x1 & MILLISECOND_MASK) != 0) jthrow(TSDB_E_ASSERTION, "x1=%lld", (long long)x1);
  switch (a->interp) {
    case TSDB_INTERP_LERP: return jadd(y0, jdiv(jmul(jsub(x, x0), jsub(y1, y0)), jsub(x1, x0)));
    case TSDB_INTERP_ZIM: return 0;
    case TSDB_INTERP_MAX: return LONG_MAX_J;
    case TSDB_INTERP_MIN: return LONG_MIN_J;
    case TSDB_INTERP_PREV: return y0;
  }
  jthrow(TSDB_E_ILLEGAL_DATA, "Invalid interpolation somehow??");
}
static double ai_next_double(void* c) {  /* :735-797 */
  agg_view* a = (agg_view*)c;
  if (!ai_has_next_value_upd(a, 1)) jthrow(TSDB_E_NO_SUCH_ELEMENT, "no more doubles");
  const int64_t pos = a->pos;
  const double y0 = (a->ts[pos] & FLAG_FLOAT) == FLAG_FLOAT ? bitsd((uint64_t)a->vals[pos]) : (double)a->vals[pos];
  if (a->current == pos) return y0;
  if (a->rate) return y0;
  const int64_t x = a->ts[a->current] & TIME_MASK;
  const int64_t x0 = a->ts[pos] & TIME_MASK;
  if (x == x0) return y0;
  const int64_t nx = pos + a->k;
  const double y1 = (a->ts[nx] & FLAG_FLOAT) == FLAG_FLOAT ? bitsd((uint64_t)a->vals[nx]) : (double)a->vals[nx];
  const int64_t x1 = a->ts[nx] & TIME_MASK;
  if (x == x1) return y1;
  if ((x1 & MILLISECOND_MASK) != 0) jthrow(TSDB_E_ASSERTION, "x1=%lld", (long long)x1);
  switch (a->interp) {
    case TSDB_INTERP_LERP: return y0 + (double)(x - x0) * (y1 - y0) / (double)(x1 - x0);
    case TSDB_INTERP_ZIM: return 0;
    case TSDB_INTERP_MAX: return 1.7976931348623157e308;   /* Double.MAX_VALUE */
    case TSDB_INTERP_MIN: return 4.9e-324;                /* Double.MIN_VALUE */
    case TSDB_INTERP_PREV: return y0;
  }
  jthrow(TSDB_E_ILLEGAL_DATA, "Invalid interpolation somehow??");
}

static ref_dp ai_next(ref_view* v) {  /* :514-567, then the DataPoint view of the result */
  agg_view* a = (agg_view*)v;
  const int64_t k = a->k;
  int64_t min_ts = LONG_MAX_J;
  for (int64_t i = a->current; i < k; i++)
    if (a->ts[i + k] == TIME_MASK) a->ts[i] = 0;
  a->current = -1;
  int multiple = 0;
  for (int64_t i = 0; i < k; i++) {
    const int64_t t = a->ts[k + i] & TIME_MASK;
    if (t <= a->end) {
      if (t < min_ts) { min_ts = t; a->current = i; multiple = 0; }
      else if (t == min_ts) multiple = 1;
    }
  }
  if (a->current < 0) jthrow(TSDB_E_NO_SUCH_ELEMENT, "no more elements");
  ai_move_to_next(a, a->current);
  if (multiple) {
    for (int64_t i = a->current + 1; i < k; i++)
      if ((a->ts[k + i] & TIME_MASK) == min_ts) ai_move_to_next(a, i);
  }
  /* DataPoint: timestamp() :608, isInteger() :612, longValue() :627, doubleValue() :635 */
  memset(&a->out, 0, sizeof a->out);
  a->out.ts = a->ts[a->current] & TIME_MASK;
  a->out.is_int = ai_is_integer(a);
  vals_t vv = {ai_has_value, ai_next_long, ai_next_double, a};
  TRY {
    a->pos = -1;
    if (a->out.is_int) {
      a->out.lv = agg_run_long(a->agg, &vv);
    } else {
      a->out.dv = agg_run_double(a->agg, &vv);
      if (isinf(a->out.dv)) jthrow(TSDB_E_ILLEGAL_STATE, "Got Infinity: %g", a->out.dv);
    }
  } CATCH(e) { a->out.bad = e; } END_TRY
  return a->out;
}
static void ai_seek(ref_view* v, int64_t ts) {  /* :598-602 */
  agg_view* a = (agg_view*)v;
  for (int64_t i = 0; i < a->k; i++) if (a->its[i]) v_seek(a->its[i], ts);
}
static void ai_destroy(ref_view* v) {
  agg_view* a = (agg_view*)v;
  for (int64_t i = 0; i < a->k; i++) ref_view_free(a->owned[i]);
  free(a->owned); free(a->its); free(a->ts); free(a->vals); free(a);
}
static const view_vt AGG_VT = {ai_has_next, ai_next, ai_seek, ai_destroy};

/* Constructor :395-465, in two steps so that an exception thrown while priming the spans
 * (the second step) finds the object already owned by the caller: agg_new takes ownership of
 * the spans and cannot throw. */
static agg_view* agg_new(ref_view** srcs, int64_t n, int64_t start_time, int64_t end_time,
                         int32_t aggregator, int32_t interpolation, int32_t rate) {
  agg_view* a = (agg_view*)xcalloc(1, sizeof(agg_view));
  a->base.vt = &AGG_VT;
  a->k = n;
  a->its = (ref_view**)xcalloc((size_t)n, sizeof(ref_view*));
  a->owned = (ref_view**)xcalloc((size_t)n, sizeof(ref_view*));
  a->ts = (int64_t*)xcalloc((size_t)(2 * n), sizeof(int64_t));
  a->vals = (int64_t*)xcalloc((size_t)(2 * n), sizeof(int64_t));
  a->start = start_time;
  a->end = end_time;
  a->agg = aggregator;
  a->interp = interpolation;
  a->rate = rate;
  a->current = 0;
  for (int64_t i = 0; i < n; i++) { a->its[i] = srcs[i]; a->owned[i] = srcs[i]; }
  return a;
}

static void agg_start(agg_view* a) {
  const int64_t n = a->k, start_time = a->start;
  for (int64_t i = 0; i < n; i++) {
    ref_view* it = a->its[i];
    v_seek(it, start_time);
    if (!v_has_next(it)) { ai_end_reached(a, i); continue; }
    ref_dp d = v_next(it);
    if (d.ts >= start_time) {
      ai_put(a, n + i, &d);
    } else {
      int null_dp = 0;
      while (!null_dp && d.ts < start_time) {
        if (v_has_next(it)) d = v_next(it);
        else null_dp = 1;
      }
      if (null_dp) { ai_end_reached(a, i); continue; }
      ai_put(a, n + i, &d);
    }
    if (a->rate) {
      if (v_has_next(it)) ai_move_to_next(a, i);
      else ai_end_reached(a, i);
    }
  }
}

ref_view* ref_view_aggregate(ref_view** srcs, int64_t n, int64_t start_time, int64_t end_time,
                             int32_t aggregator, int32_t interpolation, int32_t rate) {
  agg_view* a = agg_new(srcs, n, start_time, end_time, aggregator, interpolation, rate);
  volatile int failed = 0;
  TRY { agg_start(a); }
  CATCH(e) { (void)e; failed = 1; } END_TRY
  if (failed) { ai_destroy(&a->base); return NULL; }   /* the spans were handed over: freed with it */
  return &a->base;
}

void ref_view_free(ref_view* v) { if (v) v->vt->destroy(v); }

int ref_has_next(ref_view* v) {
  int rc = 0;
  TRY { rc = v_has_next(v); } CATCH(e) { rc = e; } END_TRY
  return rc;
}
int ref_seek(ref_view* v, int64_t ts) {
  int rc = 0;
  TRY { v_seek(v, ts); } CATCH(e) { rc = e; } END_TRY
  return rc;
}

/* Drains the view the way a consumer does: for (DataPoint dp : dps) { dp.timestamp();
 * isInteger() ? longValue() : doubleValue(); } */
int64_t ref_drain(ref_view* v, int64_t cap, int64_t* ts, int32_t* is_int, uint64_t* bits) {
  volatile int64_t n = 0;
  volatile int64_t rc = 0;
  TRY {
    while (v_has_next(v)) {
      ref_dp d = v_next(v);
      int64_t lv = 0; double dv = 0;
      if (d.is_int) lv = dp_long(&d); else dv = dp_double(&d);
      if (n < cap) {
        ts[n] = d.ts;
        is_int[n] = d.is_int;
        bits[n] = d.is_int ? (uint64_t)lv : dbits(dv);
      }
      n++;
    }
    rc = n;
  } CATCH(e) { rc = e; } END_TRY
  return rc;
}

/* ======================================================================== */
/* host logic: parseDuration, DownsamplingSpecification, scan bounds         */
/* ======================================================================== */
int ref_parse_duration(const char* duration, int64_t* out) {  /* DateTime.java:186-226 */
  size_t len = strlen(duration);
  size_t unit = 0;
  if (len == 0) { snprintf(g_msg, sizeof g_msg, "Invalid duration"); return TSDB_E_ILLEGAL_ARGUMENT; }
  while (isdigit((unsigned char)duration[unit])) {
    unit++;
    if (unit >= len) { snprintf(g_msg, sizeof g_msg, "Invalid duration, must have an integer and unit: %s", duration); return TSDB_E_ILLEGAL_ARGUMENT; }
  }
  if (unit == 0 || unit > 18) { snprintf(g_msg, sizeof g_msg, "Invalid duration (number): %s", duration); return TSDB_E_ILLEGAL_ARGUMENT; }
  char num[32];
  memcpy(num, duration, unit);
  num[unit] = 0;
  int64_t interval = strtoll(num, NULL, 10);
  if (interval <= 0) { snprintf(g_msg, sizeof g_msg, "Zero or negative duration: %s", duration); return TSDB_E_ILLEGAL_ARGUMENT; }
  int64_t mult;
  switch (tolower((unsigned char)duration[len - 1])) {
    case 's':
      if (len >= 2 && duration[len - 2] == 'm') { *out = interval; return 0; }
      mult = 1; break;
    case 'm': mult = 60; break;
    case 'h': mult = 3600; break;
    case 'd': mult = 3600 * 24; break;
    case 'w': mult = 3600 * 24 * 7; break;
    case 'n': mult = 3600 * 24 * 30; break;
    case 'y': mult = 3600LL * 24 * 365; break;
    default: snprintf(g_msg, sizeof g_msg, "Invalid duration (suffix): %s", duration); return TSDB_E_ILLEGAL_ARGUMENT;
  }
  mult *= 1000;
  if ((double)interval * (double)mult > 9223372036854775807.0) {
    snprintf(g_msg, sizeof g_msg, "Duration must be < Long.MAX_VALUE ms: %s", duration);
    return TSDB_E_ILLEGAL_ARGUMENT;
  }
  *out = interval * mult;
  return 0;
}

/* new DownsamplingSpecification(String) :116-191 */
int ref_parse_downsample(const char* spec, tsdbhip_query* q) {
  char buf[256];
  if (!spec || strlen(spec) >= sizeof buf) { snprintf(g_msg, sizeof g_msg, "Downsampling specifier cannot be null"); return TSDB_E_ILLEGAL_ARGUMENT; }
  strcpy(buf, spec);
  char* parts[8];
  int np = 0;
  /* String.split("-") drops trailing empty strings */
  char* p = buf;
  for (;;) {
    char* d = strchr(p, '-');
    if (np < 8) parts[np++] = p;
    if (!d) break;
    *d = 0;
    p = d + 1;
  }
  while (np > 0 && parts[np - 1][0] == 0) np--;
  if (np < 2) { snprintf(g_msg, sizeof g_msg, "Invalid downsampling specifier '%s': must provide at least interval and function", spec); return TSDB_E_ILLEGAL_ARGUMENT; }
  if (np > 3) { snprintf(g_msg, sizeof g_msg, "Invalid downsampling specifier '%s': must consist of interval, function, and optional fill policy", spec); return TSDB_E_ILLEGAL_ARGUMENT; }
  q->ds_all = 0;
  q->ds_calendar = 0;
  if (strstr(parts[0], "all")) {
    q->ds_interval_ms = 0;
    q->ds_all = 1;
  } else {
    size_t l = strlen(parts[0]);
    int cal = 0;
    if (l > 0 && parts[0][l - 1] == 'c') {
      parts[0][l - 1] = 0;
      cal = 1;
    }
    int rc = ref_parse_duration(parts[0], &q->ds_interval_ms);
    if (rc) return rc;
    if (cal) {
      q->ds_calendar = cal_unit_of(parts[0]);   /* DateTime.unitsToCalendarType :616-640 */
      if (!q->ds_calendar) { snprintf(g_msg, sizeof g_msg, "Unrecognized unit type: %s", parts[0]); return TSDB_E_ILLEGAL_ARGUMENT; }
    }
  }
  int f = ref_aggregator_get(parts[1]);
  if (f < 0) { snprintf(g_msg, sizeof g_msg, "No such downsampling function: %s", parts[1]); return TSDB_E_ILLEGAL_ARGUMENT; }
  if (f == TSDB_AGG_NONE) { snprintf(g_msg, sizeof g_msg, "cannot use the NONE aggregator for downsampling"); return TSDB_E_ILLEGAL_ARGUMENT; }
  q->ds_function = f;
  q->ds_fill = TSDB_FILL_NONE;
  if (np == 3) {
    static const char* const fills[5] = {"none", "zero", "nan", "null", "scalar"};
    int found = -1;
    for (int i = 0; i < 5; i++) if (strcasecmp(fills[i], parts[2]) == 0) found = i;
    if (found < 0) { snprintf(g_msg, sizeof g_msg, "Unrecognized fill policy: %s", parts[2]); return TSDB_E_ILLEGAL_ARGUMENT; }
    q->ds_fill = found;
  }
  return 0;
}

static int has_downsampler(const tsdbhip_query* q) { return q->ds_function >= 0; }

/* TsdbQuery.getScanStartTimeSeconds :1506-1546, getScanEndTimeSeconds :1548-1606 (no rollups) */
int ref_scan_bounds(const tsdbhip_query* q, int64_t* s_out, int64_t* e_out) {
  int64_t start = q->start_time;
  if ((start & (int64_t)0xFFFFFFFF00000000LL) != 0) start /= 1000;
  int64_t aligned = start;
  if (has_downsampler(q) && q->ds_interval_ms > 0) {
    const int64_t off = (1000 * start) % q->ds_interval_ms;
    aligned -= off / 1000;
  }
  const int64_t ts_aligned = aligned - (aligned % 3600);
  *s_out = ts_aligned > 0 ? ts_aligned : 0;

  int64_t end = q->end_time;
  if ((end & (int64_t)0xFFFFFFFF00000000LL) != 0) {
    end /= 1000;
    if (end - (end * 1000) < 1) end++;
  }
  if (has_downsampler(q) && q->ds_interval_ms > 0) {
    const int64_t off = (1000 * end) % q->ds_interval_ms;
    const int64_t ia = end + (q->ds_interval_ms - off) / 1000;
    const int64_t toff = ia % 3600;
    *e_out = toff == 0 ? ia : ia + (3600 - toff);
  } else {
    const int64_t toff = end % 3600;
    *e_out = end + (3600 - toff);
  }
  return 0;
}

/* ======================================================================== */
/* End-to-end query: TsdbQuery.run() -> SpanGroup[] -> iteration             */
/* ======================================================================== */
typedef struct {
  int64_t* row_ids;   /* rows of the span inside the scan range */
  int64_t nrows;
  int32_t group;
} span_desc;

typedef struct {
  int32_t group_id;
  int64_t* spans;     /* indices into span_desc */
  int64_t nspans;
  /* output */
  int64_t n, cap;
  int64_t* ts;
  uint64_t* bits;
  uint8_t* is_int;
  int err;
  char msg[512];
} group_job;

static void job_push(group_job* g, int64_t ts, int is_int, uint64_t bits) {
  if (g->n == g->cap) {
    g->cap = g->cap ? g->cap * 2 : 64;
    g->ts = (int64_t*)realloc(g->ts, (size_t)g->cap * 8);
    g->bits = (uint64_t*)realloc(g->bits, (size_t)g->cap * 8);
    g->is_int = (uint8_t*)realloc(g->is_int, (size_t)g->cap);
    if (!g->ts || !g->bits || !g->is_int) jthrow(TSDB_E_NOMEM, "oom");
  }
  g->ts[g->n] = ts;
  g->bits[g->n] = bits;
  g->is_int[g->n] = (uint8_t)is_int;
  g->n++;
}

typedef struct {
  const tsdbhip_batch* b;
  const tsdbhip_query* q;
  span_desc* spans;
  int64_t scan_start_ms, scan_end_ms;
  const tsdbhip_rollup_batch* rb;   /* rollup query: RollupSpans over these cells */
} query_env;

/* RollupQuery ctor :69-80: zimsum / mimmax / mimmin read the sum / max / min columns */
static int32_t rollup_agg_of(int32_t f) {
  return f == TSDB_AGG_ZIMSUM ? TSDB_AGG_SUM : f == TSDB_AGG_MIMMAX ? TSDB_AGG_MAX : f == TSDB_AGG_MIMMIN ? TSDB_AGG_MIN : f;
}

/* SpanGroup.iterator() :527 -> AggregationIterator.create :351-380 -> drain */
static void run_group(const query_env* env, group_job* g) {
  const tsdbhip_batch* b = env->b;
  const tsdbhip_query* q = env->q;
  ref_view** its = (ref_view**)xcalloc((size_t)(g->nspans ? g->nspans : 1), sizeof(ref_view*));
  volatile int64_t k = 0;
  ref_view* volatile ai = NULL;
  TRY {
    for (int64_t i = 0; i < g->nspans; i++) {
      span_desc* sd = &env->spans[g->spans[i]];
      ref_view* it;
      int64_t first = 0, last = 0, size = 0;
      if (env->rb) {
        it = make_rollup_span(env->rb, sd->row_ids, sd->nrows);
        rollup_span_first_last((ro_span*)it, &first, &last, &size);
      } else {
        it = make_span(sd->nrows, b->row_base_time, b->row_qual_off, b->row_val_off, b->qual, b->val, sd->row_ids);
        span_first_last((span_view*)it, &first, &last, &size);
      }
      /* SpanGroup.add :324-339: admit only spans overlapping [start, end] */
      if (size == 0 || !(first <= env->scan_end_ms && last >= env->scan_start_ms)) { ref_view_free(it); continue; }
      if (has_downsampler(q)) {
        it = make_downsampler(it, q->ds_function, q->ds_interval_ms, q->ds_fill, q->ds_all,
                              env->scan_start_ms, env->scan_end_ms, q->start_time, q->end_time, q->ds_calendar,
                              q->ds_tz);
        if (env->rb) ((ds_view*)it)->rollup_agg = rollup_agg_of(q->ds_function);   /* Span.downsampler's rollup_query */
      }
      if (q->rate) it = ref_view_rate(it, q->rate_counter, q->rate_counter_max, q->rate_reset_value, q->rate_drop_resets);
      its[k++] = it;
    }
    agg_view* na = agg_new(its, k, env->scan_start_ms, env->scan_end_ms, q->aggregator, agg_interp(q->aggregator), q->rate);
    ai = &na->base;
    k = 0;  /* ownership moved */
    agg_start(na);
    while (v_has_next(ai)) {
      ref_dp d = v_next(ai);
      if (d.is_int) job_push(g, d.ts, 1, (uint64_t)dp_long(&d));
      else job_push(g, d.ts, 0, dbits(dp_double(&d)));
    }
  } CATCH(e) {
    g->err = e;
    snprintf(g->msg, sizeof g->msg, "%s", g_msg);
  } END_TRY
  for (int64_t i = 0; i < k; i++) ref_view_free(its[i]);
  ref_view_free(ai);
  free(its);
}

typedef struct {
  const query_env* env;
  group_job* jobs;
  int64_t njobs;
  int64_t next;
  pthread_mutex_t mu;
} pool_t;

static void* pool_worker(void* arg) {
  pool_t* p = (pool_t*)arg;
  for (;;) {
    pthread_mutex_lock(&p->mu);
    int64_t j = p->next++;
    pthread_mutex_unlock(&p->mu);
    if (j >= p->njobs) break;
    run_group(p->env, &p->jobs[j]);
  }
  return NULL;
}

/* TsdbQuery.getScanStartTimeSeconds :1515-1526 / getScanEndTimeSeconds :1562-1567 with a
 * rollup query */
static void rollup_scan_bounds(const tsdbhip_query* q, const tsdbhip_rollup_interval* iv, int64_t* s_out, int64_t* e_out) {
  int64_t start = q->start_time;
  if ((start & (int64_t)0xFFFFFFFF00000000LL) != 0) start /= 1000;
  int64_t base = ro_basetime(start, iv);
  if (q->rate) base = ro_basetime(base - 1, iv);   /* one row back for the first rate */
  *s_out = base;
  int64_t end = q->end_time;
  if ((end & (int64_t)0xFFFFFFFF00000000LL) != 0) {
    end /= 1000;
    if (end - (end * 1000) < 1) end++;
  }
  *e_out = ro_basetime(end + (int64_t)iv->interval_s * iv->intervals, iv);
}

static int run_query_impl(const tsdbhip_batch* b, const tsdbhip_query* q0, int nthreads, ref_result** out,
                          const tsdbhip_rollup_batch* rb) {
  volatile int rc = 0;
  span_desc* volatile spans = NULL;
  group_job* volatile jobs = NULL;
  volatile int64_t njobs = 0, nspans = 0;
  *out = NULL;
  tsdbhip_query qr = *q0;
  const tsdbhip_query* q = &qr;
  TRY {
    if (has_downsampler(q)) {
      if (q->ds_function == TSDB_AGG_NONE) jthrow(TSDB_E_ILLEGAL_ARGUMENT, "cannot use the NONE aggregator for downsampling");
    }
    int64_t ss, se;
    if (rb) {
      /* TsdbQuery.transformDownSamplerToRollupQuery :1665-1700: a rollup query exists only
       * with a downsampler; a count group-by sums the rolled-up counts */
      if (!has_downsampler(q) || (!q->ds_all && q->ds_interval_ms <= 0))
        jthrow(TSDB_E_ILLEGAL_ARGUMENT, "a rollup query needs a downsampling interval");
      if (qr.aggregator == TSDB_AGG_COUNT) qr.aggregator = TSDB_AGG_SUM;
      rollup_scan_bounds(q, &rb->interval, &ss, &se);
    } else {
      ref_scan_bounds(q, &ss, &se);
    }
    /* SpanGroup ctor :270-273: seconds -> ms */
    query_env env = {b, q, NULL, ss * 1000, se * 1000, rb};
    /* findSpans: rows with base_time in [scan_start, scan_end) (QueryUtil.getMetricScanner) */
    spans = (span_desc*)xcalloc((size_t)(b->n_series ? b->n_series : 1), sizeof(span_desc));
    for (int64_t s = 0; s < b->n_series; s++) {
      const int64_t r0 = b->series_row_ptr[s], r1 = b->series_row_ptr[s + 1];
      int64_t cnt = 0;
      for (int64_t r = r0; r < r1; r++)
        if ((int64_t)b->row_base_time[r] >= ss && (int64_t)b->row_base_time[r] < se) cnt++;
      if (cnt == 0) continue;
      span_desc* sd = &spans[nspans++];
      sd->row_ids = (int64_t*)xmalloc((size_t)cnt * 8);
      sd->nrows = 0;
      for (int64_t r = r0; r < r1; r++)
        if ((int64_t)b->row_base_time[r] >= ss && (int64_t)b->row_base_time[r] < se) sd->row_ids[sd->nrows++] = r;
      sd->group = b->group_id ? b->group_id[s] : 0;
      if (rb) {   /* the scan builds every RollupSeq: RollupSeq.append throws here, in scan order */
        ref_view* t = make_rollup_span(rb, sd->row_ids, sd->nrows);
        ref_view_free(t);
      }
    }
    env.spans = spans;
    if (q->aggregator == TSDB_AGG_NONE) {  /* TsdbQuery.java:941-962: one SpanGroup per span */
      jobs = (group_job*)xcalloc((size_t)(nspans ? nspans : 1), sizeof(group_job));
      for (int64_t i = 0; i < nspans; i++) {
        jobs[njobs].group_id = (int32_t)i;
        jobs[njobs].spans = (int64_t*)xmalloc(8);
        jobs[njobs].spans[0] = i;
        jobs[njobs].nspans = 1;
        njobs++;
      }
    } else {
      int32_t maxg = -1;
      for (int64_t i = 0; i < nspans; i++) if (spans[i].group > maxg) maxg = spans[i].group;
      int64_t* cnt = (int64_t*)xcalloc((size_t)(maxg + 2), 8);
      for (int64_t i = 0; i < nspans; i++) if (spans[i].group >= 0) cnt[spans[i].group]++;
      jobs = (group_job*)xcalloc((size_t)(maxg + 2), sizeof(group_job));
      int64_t* slot = (int64_t*)xcalloc((size_t)(maxg + 2), 8);
      for (int32_t gi = 0; gi <= maxg; gi++) {
        if (cnt[gi] == 0) { slot[gi] = -1; continue; }
        slot[gi] = njobs;
        jobs[njobs].group_id = gi;
        jobs[njobs].spans = (int64_t*)xmalloc((size_t)cnt[gi] * 8);
        njobs++;
      }
      for (int64_t i = 0; i < nspans; i++) {
        if (spans[i].group < 0) continue;
        group_job* g = &jobs[slot[spans[i].group]];
        g->spans[g->nspans++] = i;
      }
      free(cnt);
      free(slot);
    }
    if (nthreads <= 1 || njobs <= 1) {
      for (int64_t j = 0; j < njobs; j++) run_group(&env, &jobs[j]);
    } else {
      pool_t pool = {&env, jobs, njobs, 0, PTHREAD_MUTEX_INITIALIZER};
      pthread_t th[256];
      int nt = nthreads > 256 ? 256 : nthreads;
      for (int t = 0; t < nt; t++) pthread_create(&th[t], NULL, pool_worker, &pool);
      for (int t = 0; t < nt; t++) pthread_join(th[t], NULL);
    }
    for (int64_t j = 0; j < njobs; j++) {
      if (jobs[j].err) {
        snprintf(g_msg, sizeof g_msg, "%s", jobs[j].msg);
        jthrow(jobs[j].err, "%s", jobs[j].msg);
      }
    }
    ref_result* r = (ref_result*)xcalloc(1, sizeof(ref_result));
    r->n_groups = njobs;
    int64_t tot = 0;
    for (int64_t j = 0; j < njobs; j++) tot += jobs[j].n;
    r->n_points = tot;
    r->group_id = (int32_t*)xcalloc((size_t)(njobs ? njobs : 1), 4);
    r->group_ptr = (int64_t*)xcalloc((size_t)njobs + 1, 8);
    r->ts_ms = (int64_t*)xcalloc((size_t)(tot ? tot : 1), 8);
    r->value_bits = (uint64_t*)xcalloc((size_t)(tot ? tot : 1), 8);
    r->is_int = (uint8_t*)xcalloc((size_t)(tot ? tot : 1), 1);
    int64_t o = 0;
    for (int64_t j = 0; j < njobs; j++) {
      r->group_id[j] = jobs[j].group_id;
      r->group_ptr[j] = o;
      if (jobs[j].n) {
        memcpy(r->ts_ms + o, jobs[j].ts, (size_t)jobs[j].n * 8);
        memcpy(r->value_bits + o, jobs[j].bits, (size_t)jobs[j].n * 8);
        memcpy(r->is_int + o, jobs[j].is_int, (size_t)jobs[j].n);
      }
      o += jobs[j].n;
    }
    r->group_ptr[njobs] = o;
    *out = r;
  } CATCH(e) { rc = e; } END_TRY
  for (int64_t i = 0; i < nspans; i++) free(spans[i].row_ids);
  free(spans);
  for (int64_t j = 0; j < njobs; j++) { free(jobs[j].spans); free(jobs[j].ts); free(jobs[j].bits); free(jobs[j].is_int); }
  free(jobs);
  return rc;
}

int ref_run_query(const tsdbhip_batch* b, const tsdbhip_query* q, ref_result** out) {
  return run_query_impl(b, q, 1, out, NULL);
}
int ref_run_query_mt(const tsdbhip_batch* b, const tsdbhip_query* q, int nthreads, ref_result** out) {
  return run_query_impl(b, q, nthreads, out, NULL);
}
int ref_run_rollup_query(const tsdbhip_rollup_batch* rb, const tsdbhip_query* q, ref_result** out) {
  if (!rb || !q || !out) return TSDB_E_ILLEGAL_ARGUMENT;
  return run_query_impl(&rb->cells, q, 1, out, rb);
}
int ref_rollup_scan_bounds(const tsdbhip_query* q, const tsdbhip_rollup_interval* iv, int64_t* s_out, int64_t* e_out) {
  volatile int rc = 0;
  TRY { rollup_scan_bounds(q, iv, s_out, e_out); } CATCH(e) { rc = e; } END_TRY
  return rc;
}
void ref_result_free(ref_result* r) {
  if (!r) return;
  free(r->group_id); free(r->group_ptr); free(r->ts_ms); free(r->value_bits); free(r->is_int); free(r);
}
