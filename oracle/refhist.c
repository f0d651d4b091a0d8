/*
 * refhist.c -- TEST INFRASTRUCTURE ONLY (parity oracle of the histogram path).
 *
 * Plain-C restatement of OpenTSDB 2.4's histogram query path, object for object (citations
 * relative to the reference tree):
 *   histogram column decode .......... src/core/SaltScanner.java:734-800 (decode failures drop
 *                                      the column), src/core/Internal.java:1059-1104
 *   Kryo 2.21.1 Input ................ third_party/kryo/include.mk:16 (not vendored; restated:
 *                                      readShort / readFloat big-endian, readLong(true) varint of
 *                                      7-bit groups, the 9th byte carrying 8 bits; buffer underflow
 *                                      throws)
 *   SimpleHistogram .................. src/core/SimpleHistogram.java:97-271
 *   LongHistogramDataPointForTest .... test/core/LongHistogramDataPointForTest.java (codec of the
 *                                      reference's histogram query tests)
 *   HistogramDataPoint.HistogramBucket src/core/HistogramDataPoint.java:83-185 (equals/compareTo)
 *   SimpleHistogramDataPointAdapter .. src/core/SimpleHistogramDataPointAdapter.java:60-139
 *   HistogramRowSeq / HistogramSpan .. src/core/HistogramRowSeq.java:56-388,
 *                                      src/core/HistogramSpan.java:280-541
 *   HistogramDownsampler ............. src/core/HistogramDownsampler.java:64-397
 *   HistogramAggregationIterator ..... src/core/HistogramAggregationIterator.java:91-313
 *   HistogramSpanGroup ............... src/core/HistogramSpanGroup.java:110-205,347-350
 *   TsdbQuery (histogram callback) ... src/core/TsdbQuery.java:1061-1287
 *   adaptors ......................... src/core/HistogramDataPointsToDataPointsAdaptor.java,
 *                                      src/core/HistogramBucketDataPointsAdaptor.java
 *   java.util.TreeMap ................ red-black put / getEntry (JDK 8), restated so that the
 *                                      bucket adaptor's lookups follow HistogramBucket.compareTo,
 *                                      which is inconsistent between REGULAR and UNDER/OVERFLOW keys
 * Only tests/ load this (through librefcpu.so).
 */
#define _GNU_SOURCE
#include "refcpu.h"

#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---- exceptions (local to this file) ------------------------------------------------- */
static __thread jmp_buf* h_jb = NULL;
static __thread int h_code;
static __thread char h_msg[256];

static void hthrow(int code, const char* fmt, ...) __attribute__((noreturn));
static void hthrow(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(h_msg, sizeof h_msg, fmt, ap);
  va_end(ap);
  h_code = code;
  if (h_jb) longjmp(*h_jb, 1);
  fprintf(stderr, "refhist: uncaught exception %d: %s\n", code, h_msg);
  abort();
}
static void* hx(void* p) {
  if (!p) hthrow(TSDB_E_NOMEM, "out of memory");
  return p;
}
static void* hmalloc_(size_t n) { return hx(malloc(n ? n : 1)); }
#define HMALLOC(n) hmalloc_(n)
#define HCALLOC(n, m) hx(calloc((n) ? (n) : 1, (m) ? (m) : 1))

/* ---- Float.compare / HistogramBucket ------------------------------------------------- */
static inline float f_of(uint32_t b) { float f; memcpy(&f, &b, 4); return f; }
static inline uint32_t f_canon(uint32_t b) {   /* Float.floatToIntBits */
  return ((b & 0x7F800000u) == 0x7F800000u && (b & 0x007FFFFFu)) ? 0x7FC00000u : b;
}
static int fcmp(uint32_t a, uint32_t b) {   /* Float.compare(a, b) */
  const float x = f_of(a), y = f_of(b);
  if (x < y) return -1;
  if (x > y) return 1;
  const int32_t ia = (int32_t)f_canon(a), ib = (int32_t)f_canon(b);
  return ia == ib ? 0 : (ia < ib ? -1 : 1);
}
enum { BK_UNDER = 0, BK_REG = 1, BK_OVER = 2 };
typedef struct { int type; uint32_t lo, up; } hbucket;
static int bk_equals(const hbucket* a, const hbucket* b) {   /* HistogramBucket.equals :117-144 */
  if (a->type != b->type) return 0;
  if (a->type != BK_REG) return 1;
  return fcmp(a->lo, b->lo) == 0 && fcmp(a->up, b->up) == 0;
}
static int bk_compare(const hbucket* a, const hbucket* b) {   /* compareTo :146-165 */
  if (bk_equals(a, b)) return 0;
  if (a->type == BK_UNDER) return -1;
  if (a->type == BK_REG) {
    const int c = fcmp(a->lo, b->lo);
    return c ? c : fcmp(a->up, b->up);
  }
  return 1;
}

/* ---- java.util.TreeMap (red-black), only what the bucket adaptor needs ----------------- */
typedef struct tm_node {
  hbucket key;
  int64_t val;
  struct tm_node *l, *r, *p;
  int black;
} tm_node;
typedef struct { tm_node* root; tm_node* pool; int n, cap; } treemap;
static tm_node* tm_par(tm_node* x) { return x ? x->p : NULL; }
static tm_node* tm_left(tm_node* x) { return x ? x->l : NULL; }
static tm_node* tm_right(tm_node* x) { return x ? x->r : NULL; }
static int tm_black(tm_node* x) { return x ? x->black : 1; }
static void tm_set(tm_node* x, int black) { if (x) x->black = black; }
static void tm_rotl(treemap* t, tm_node* p) {
  if (!p) return;
  tm_node* r = p->r;
  p->r = r->l;
  if (r->l) r->l->p = p;
  r->p = p->p;
  if (!p->p) t->root = r;
  else if (p->p->l == p) p->p->l = r;
  else p->p->r = r;
  r->l = p;
  p->p = r;
}
static void tm_rotr(treemap* t, tm_node* p) {
  if (!p) return;
  tm_node* l = p->l;
  p->l = l->r;
  if (l->r) l->r->p = p;
  l->p = p->p;
  if (!p->p) t->root = l;
  else if (p->p->r == p) p->p->r = l;
  else p->p->l = l;
  l->r = p;
  p->p = l;
}
static void tm_fix(treemap* t, tm_node* x) {   /* TreeMap.fixAfterInsertion */
  x->black = 0;
  while (x && x != t->root && !x->p->black) {
    if (tm_par(x) == tm_left(tm_par(tm_par(x)))) {
      tm_node* y = tm_right(tm_par(tm_par(x)));
      if (!tm_black(y)) {
        tm_set(tm_par(x), 1); tm_set(y, 1); tm_set(tm_par(tm_par(x)), 0);
        x = tm_par(tm_par(x));
      } else {
        if (x == tm_right(tm_par(x))) { x = tm_par(x); tm_rotl(t, x); }
        tm_set(tm_par(x), 1); tm_set(tm_par(tm_par(x)), 0);
        tm_rotr(t, tm_par(tm_par(x)));
      }
    } else {
      tm_node* y = tm_left(tm_par(tm_par(x)));
      if (!tm_black(y)) {
        tm_set(tm_par(x), 1); tm_set(y, 1); tm_set(tm_par(tm_par(x)), 0);
        x = tm_par(tm_par(x));
      } else {
        if (x == tm_left(tm_par(x))) { x = tm_par(x); tm_rotr(t, x); }
        tm_set(tm_par(x), 1); tm_set(tm_par(tm_par(x)), 0);
        tm_rotl(t, tm_par(tm_par(x)));
      }
    }
  }
  t->root->black = 1;
}
static void tm_put(treemap* t, hbucket k, int64_t v) {   /* TreeMap.put (the new key's compareTo) */
  tm_node* par = NULL;
  int c = 0;
  for (tm_node* x = t->root; x;) {
    par = x;
    c = bk_compare(&k, &x->key);
    if (c < 0) x = x->l;
    else if (c > 0) x = x->r;
    else { x->val = v; return; }
  }
  tm_node* e = &t->pool[t->n++];
  memset(e, 0, sizeof *e);
  e->key = k;
  e->val = v;
  e->p = par;
  if (!par) { t->root = e; e->black = 1; return; }
  if (c < 0) par->l = e; else par->r = e;
  tm_fix(t, e);
}
static tm_node* tm_get(const treemap* t, const hbucket* k) {   /* TreeMap.getEntry */
  for (tm_node* x = t->root; x;) {
    const int c = bk_compare(k, &x->key);
    if (c < 0) x = x->l;
    else if (c > 0) x = x->r;
    else return x;
  }
  return NULL;
}

/* ---- histogram values ------------------------------------------------------------------ */
typedef struct { uint32_t lo, up; int64_t cnt; } hreg;   /* a REGULAR bucket and its count */
typedef struct {
  int kind;          /* TSDB_HCODEC_SIMPLE / _LONG */
  int64_t ts;        /* timestamp() */
  int64_t cts;       /* the timestamp clone() gives (HistogramDownsampler.clone uses its timestamp
                        field, not timestamp(): they differ for "all", :96-101,179-183) */
  hreg* b;           /* SimpleHistogram.buckets (TreeMap of REGULAR keys: consistent order) */
  int nb, cap;
  int64_t under, over;
  int64_t data;      /* LongHistogramDataPointForTest.data */
} hval;

static void hv_free(hval* h) { free(h->b); h->b = NULL; h->nb = h->cap = 0; }
static void hv_clone(hval* dst, const hval* src, int64_t ts) {   /* clone / cloneAndSetTimestamp */
  *dst = *src;
  dst->ts = dst->cts = ts;
  dst->b = (hreg*)HMALLOC(sizeof(hreg) * (size_t)(src->cap > 0 ? src->cap : 1));
  if (src->nb) memcpy(dst->b, src->b, sizeof(hreg) * (size_t)src->nb);
}
static int reg_cmp(uint32_t lo, uint32_t up, const hreg* b) {
  const int c = fcmp(lo, b->lo);
  return c ? c : fcmp(up, b->up);
}
static int hv_find(const hval* h, uint32_t lo, uint32_t up, int* at) {
  int a = 0, z = h->nb;
  while (a < z) {
    const int m = (a + z) / 2;
    const int c = reg_cmp(lo, up, &h->b[m]);
    if (c == 0) { *at = m; return 1; }
    if (c < 0) z = m; else a = m + 1;
  }
  *at = a;
  return 0;
}
static void hv_put(hval* h, uint32_t lo, uint32_t up, int64_t cnt) {   /* addBucket / buckets.put */
  int at;
  if (hv_find(h, lo, up, &at)) { h->b[at].cnt = cnt; return; }   /* TreeMap keeps the first key */
  if (h->nb == h->cap) {
    h->cap = h->cap ? 2 * h->cap : 8;
    h->b = (hreg*)hx(realloc(h->b, sizeof(hreg) * (size_t)h->cap));
  }
  memmove(h->b + at + 1, h->b + at, sizeof(hreg) * (size_t)(h->nb - at));
  h->b[at].lo = lo; h->b[at].up = up; h->b[at].cnt = cnt;
  h->nb++;
}
static int64_t jadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }

/* SimpleHistogramDataPointAdapter.aggregate -> SimpleHistogram.aggregate (:246-261) or
 * LongHistogramDataPointForTest.aggregate */
static void hv_aggregate(hval* h, const hval* o) {
  if (h->kind == TSDB_HCODEC_SIMPLE) {
    if (o->kind != TSDB_HCODEC_SIMPLE) hthrow(TSDB_E_CLASS_CAST, "not a SimpleHistogram");
    for (int i = 0; i < o->nb; i++) {
      int at;
      const int64_t cur = hv_find(h, o->b[i].lo, o->b[i].up, &at) ? h->b[at].cnt : 0;
      hv_put(h, o->b[i].lo, o->b[i].up, jadd(cur, o->b[i].cnt));
    }
    h->over = jadd(o->over, h->over);
    h->under = jadd(o->under, h->under);
  } else {
    if (o->kind != TSDB_HCODEC_LONG)
      hthrow(TSDB_E_ILLEGAL_ARGUMENT, "The object must be an instance of the LongHistogramDataPointForTest");
    h->data = jadd(h->data, o->data);
  }
}

/* SimpleHistogram.percentile (:133-164) / LongHistogramDataPointForTest.percentile */
static double hv_percentile(const hval* h, double perc) {
  if (h->kind == TSDB_HCODEC_LONG) return (double)h->data * perc;
  if (perc < 1.0 || perc > 100.0) return -1.0;
  int32_t sum = 0;
  for (int i = 0; i < h->nb; i++) sum = (int32_t)((uint32_t)sum + (uint32_t)(int32_t)h->b[i].cnt);
  int64_t running = 0;
  for (int i = 0; i < h->nb; i++) {
    running += (int32_t)h->b[i].cnt;
    const double area = (double)running * 100.0 / (double)sum;
    if (area >= perc) {
      const float mid = (f_of(h->b[i].lo) + f_of(h->b[i].up)) / 2;
      return (double)mid;
    }
  }
  return 0.0;
}

/* ---- Kryo 2.21 Input over one value ------------------------------------------------------ */
typedef struct { const uint8_t* p; int64_t n, i; } kin;
static int k_u8(kin* k, uint8_t* b) { if (k->i >= k->n) return -1; *b = k->p[k->i++]; return 0; }
static int k_short(kin* k, int* out) {
  uint8_t a, b;
  if (k_u8(k, &a) || k_u8(k, &b)) return -1;
  *out = (int16_t)(((uint16_t)a << 8) | b);
  return 0;
}
static int k_int(kin* k, uint32_t* out) {
  uint32_t v = 0;
  for (int j = 0; j < 4; j++) { uint8_t b; if (k_u8(k, &b)) return -1; v = (v << 8) | b; }
  *out = v;
  return 0;
}
static int k_varlong(kin* k, int64_t* out) {   /* Input.readLong(true) */
  uint64_t r = 0;
  uint8_t b;
  for (int j = 0; j < 8; j++) {
    if (k_u8(k, &b)) return -1;
    r |= (uint64_t)(b & 0x7F) << (7 * j);
    if (!(b & 0x80)) { *out = (int64_t)r; return 0; }
  }
  if (k_u8(k, &b)) return -1;
  r |= (uint64_t)b << 56;
  *out = (int64_t)r;
  return 0;
}

/* HistogramCodecManager.decode(value[0], value, true); 0 ok, -1 = the column is dropped */
static int hv_decode(const uint8_t* v, int64_t n, const uint8_t* codec, hval* out) {
  memset(out, 0, sizeof *out);
  if (n < 1) return -1;                           /* value[0] */
  const int id = (int)(int8_t)v[0];
  if (id < 0 || !codec[id]) return -1;            /* "No codec found mapped to ID" */
  out->kind = codec[id];
  if (out->kind == TSDB_HCODEC_LONG) {
    if (n < 9) return -1;                         /* Bytes.getLong(raw, 1) */
    uint64_t d = 0;
    for (int j = 1; j < 9; j++) d = (d << 8) | v[j];
    out->data = (int64_t)d;
    return 0;
  }
  if (n < 6) return -1;                           /* fromHistogram :98-101 */
  kin k = {v, n, 1};
  int cnt;
  if (k_short(&k, &cnt)) return -1;
  for (int i = 0; i < cnt; i++) {
    uint32_t lo, up;
    int64_t c;
    if (k_int(&k, &lo) || k_int(&k, &up) || k_varlong(&k, &c)) { hv_free(out); return -1; }
    hv_put(out, lo, up, c);
  }
  if (k_varlong(&k, &out->under) || k_varlong(&k, &out->over)) { hv_free(out); return -1; }
  return 0;
}

int ref_hist_value_percentile(const uint8_t* v, int64_t n, int kind, double p, double* out) {
  uint8_t codec[256] = {0};
  if (n >= 1 && (int8_t)v[0] >= 0) codec[v[0]] = (uint8_t)kind;
  hval h;
  if (hv_decode(v, n, codec, &h)) return -1;
  *out = hv_percentile(&h, p);
  hv_free(&h);
  return 0;
}

/* ---- HistogramRowSeq / HistogramSpan --------------------------------------------------- */
typedef struct { int64_t base; hval* dp; int n; } hrow;
typedef struct { hrow* rows; int nr, cap; } hspan;

/* Internal.getTimeStampFromNonDP (:1059-1074); 0 ok, -1 = invalid qualifier */
static int nondp_ts(int64_t base, const uint8_t* q, int64_t ql, int64_t* out) {
  if (ql == 3) {
    const int32_t off = (int32_t)((uint32_t)(int32_t)(int8_t)q[1] << 8) | q[2];
    *out = (base + off) * 1000;
    return 0;
  }
  if (ql == 5) {
    const int32_t off = (int32_t)(((uint32_t)q[1] << 24) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 8) | q[4]);
    *out = base * 1000 + off;
    return 0;
  }
  return -1;
}

static void row_merge(hrow* local, const hrow* remote) {   /* HistogramRowSeq.addRow :66-105 */
  hval* out = (hval*)HMALLOC(sizeof(hval) * (size_t)(local->n + remote->n));
  int il = 0, ir = 0, n = 0;
  while (il < local->n && ir < remote->n) {
    const int64_t sort = remote->dp[ir].ts - local->dp[il].ts;
    if (sort == 0) { out[n++] = local->dp[il++]; hv_free(&remote->dp[ir++]); }
    else if (sort > 0) out[n++] = local->dp[il++];
    else out[n++] = remote->dp[ir++];
  }
  while (il < local->n) out[n++] = local->dp[il++];
  while (ir < remote->n) out[n++] = remote->dp[ir++];
  free(local->dp);
  free(remote->dp);
  local->dp = out;
  local->n = n;
}

static void span_add_row(hspan* s, int64_t base, hval* dps, int n) {   /* HistogramSpan.addRow :280-328 */
  int64_t last_ts = 0;
  if (s->nr) {
    const hrow* last = &s->rows[s->nr - 1];
    last_ts = last->dp[last->n - 1].ts;
  }
  hrow r = {base, dps, n};
  if (last_ts >= r.dp[0].ts) {
    for (int i = 0; i < s->nr; i++)
      if (s->rows[i].base == base) { row_merge(&s->rows[i], &r); return; }
  }
  if (s->nr == s->cap) {
    s->cap = s->cap ? 2 * s->cap : 4;
    s->rows = (hrow*)hx(realloc(s->rows, sizeof(hrow) * (size_t)s->cap));
  }
  s->rows[s->nr++] = r;
}
static void span_sort(hspan* s) {   /* checkRowOrder: Collections.sort (stable) by base time */
  for (int i = 1; i < s->nr; i++) {
    hrow x = s->rows[i];
    int j = i - 1;
    while (j >= 0 && s->rows[j].base > x.base) { s->rows[j + 1] = s->rows[j]; j--; }
    s->rows[j + 1] = x;
  }
}
static int64_t span_size(const hspan* s) { int64_t n = 0; for (int i = 0; i < s->nr; i++) n += s->rows[i].n; return n; }
static int64_t span_ts(const hspan* s, int64_t i) {   /* timestamp(i) */
  for (int r = 0; r < s->nr; r++) {
    if (i < s->rows[r].n) return s->rows[r].dp[i].ts;
    i -= s->rows[r].n;
  }
  hthrow(TSDB_E_ILLEGAL_STATE, "index out of bounds");
}
static void span_free(hspan* s) {
  for (int r = 0; r < s->nr; r++) {
    for (int i = 0; i < s->rows[r].n; i++) hv_free(&s->rows[r].dp[i]);
    free(s->rows[r].dp);
  }
  free(s->rows);
}

/* ---- seekable views -------------------------------------------------------------------- */
typedef struct hview hview;
struct hview {
  int (*has_next)(hview*);
  const hval* (*next)(hview*);   /* the current data point (valid until the next call) */
  void (*seek)(hview*, int64_t);
  void (*destroy)(hview*);
};

typedef struct {   /* HistogramSpan.Iterator :461-541 */
  hview v;
  const hspan* s;
  int row_index;
  int next_index;   /* HistogramRowSeq.Iterator of rows[row_index] */
} span_it;
static int si_has(hview* v) {
  span_it* it = (span_it*)v;
  if (it->next_index < it->s->rows[it->row_index].n) return 1;
  while (it->row_index < it->s->nr - 1) {
    it->row_index++;
    it->next_index = 0;
    if (it->s->rows[it->row_index].n > 0) return 1;
  }
  return 0;
}
static const hval* si_next(hview* v) {
  span_it* it = (span_it*)v;
  if (!si_has(v)) hthrow(TSDB_E_NO_SUCH_ELEMENT, "no more elements");
  return &it->s->rows[it->row_index].dp[it->next_index++];
}
static void si_seek(hview* v, int64_t ts) {
  span_it* it = (span_it*)v;
  /* seekRow :417-437 */
  int ri = 0;
  for (int i = 0; i < it->s->nr; i++) {
    const hrow* r = &it->s->rows[i];
    if (r->n < 1) ri++;
    else if (r->dp[r->n - 1].ts < ts) ri++;
    else break;
  }
  if (ri == it->s->nr) --ri;
  it->row_index = ri;
  /* HistogramRowSeq.Iterator.seek :357-368 */
  if (ts & (int64_t)0xFFFFF00000000000LL) hthrow(TSDB_E_ILLEGAL_ARGUMENT, "invalid timestamp: %lld", (long long)ts);
  const hrow* r = &it->s->rows[ri];
  int ni = 0;
  while (ni < r->n && r->dp[ni].ts < ts) ++ni;
  it->next_index = ni;
}
static void si_destroy(hview* v) { free(v); }
static hview* span_iterator(const hspan* s) {
  span_it* it = (span_it*)HCALLOC(1, sizeof *it);
  it->v.has_next = si_has; it->v.next = si_next; it->v.seek = si_seek; it->v.destroy = si_destroy;
  it->s = s;
  return &it->v;
}

typedef struct {   /* HistogramDownsampler :28-397 */
  hview v;
  hview* src;
  int64_t interval_ms;
  int cal_unit;      /* 0: fixed interval */
  int64_t cal_n;
  const tsdbhip_tz* tz;
  int run_all;
  int hist_sum;      /* the downsampling function is "sum" */
  int64_t qs, qe;
  int64_t timestamp;
  hval value;
  int has_value;
  /* ValuesInInterval */
  int64_t prev_cal, next_cal;
  int64_t tei;
  int has_src;
  hval next_dp;      /* a clone of the source's last data point */
  int next_dp_set;
  int initialized;
} hds;
static int64_t hds_align(hds* d, int64_t t) { return t - (t % d->interval_ms); }
static void cal_prev_or_throw(int64_t ts, int64_t n, int unit, const tsdbhip_tz* z, int64_t* out) {
  const int rc = ref_cal_prev_ex(ts, n, unit, z, out);
  if (rc) hthrow(rc, "DateTime.previousInterval");
}
static void cal_step_or_throw(int64_t ts, int unit, int64_t n, const tsdbhip_tz* z, int64_t* out) {
  const int rc = ref_cal_step_ex(ts, unit, n, z, out);
  if (rc) hthrow(rc, "Calendar.add");
}
static void viv_take(hds* d, const hval* src) {
  if (d->next_dp_set) hv_free(&d->next_dp);
  hv_clone(&d->next_dp, src, src->ts);
  d->next_dp_set = 1;
}
static void viv_drop(hds* d) { if (d->next_dp_set) hv_free(&d->next_dp); d->next_dp_set = 0; }
static void viv_move_to_next_value(hds* d) {   /* :251-276 */
  if (d->src->has_next(d->src)) {
    d->has_src = 1;
    if (d->run_all) {
      while (d->src->has_next(d->src)) {
        viv_take(d, d->src->next(d->src));
        if (d->next_dp.ts < d->qs) { viv_drop(d); continue; }
        if (d->next_dp.ts >= d->qe) d->has_src = 0;
        break;
      }
      if (!d->next_dp_set) d->has_src = 0;
    } else {
      viv_take(d, d->src->next(d->src));
    }
  } else {
    d->has_src = 0;
  }
}
static void viv_init(hds* d) {   /* initializeIfNotDone :219-248 */
  if (d->initialized) return;
  d->initialized = 1;
  if (d->src->has_next(d->src)) {
    viv_move_to_next_value(d);
    if (!d->run_all) {
      if (d->cal_unit) {
        cal_prev_or_throw(d->next_dp.ts, d->cal_n, d->cal_unit, d->tz, &d->prev_cal);
        d->next_cal = d->prev_cal;
        cal_step_or_throw(d->next_cal, d->cal_unit, d->cal_n, d->tz, &d->next_cal);
        d->tei = d->next_cal;
      } else {
        d->tei = hds_align(d, d->next_dp.ts) + d->interval_ms;
      }
    }
  }
}
static void viv_reset_end(hds* d) {   /* resetEndOfInterval :282-300 */
  if (d->has_src && !d->run_all) {
    if (d->cal_unit) {
      while (d->next_dp.ts >= d->tei) {
        cal_step_or_throw(d->prev_cal, d->cal_unit, d->cal_n, d->tz, &d->prev_cal);
        cal_step_or_throw(d->next_cal, d->cal_unit, d->cal_n, d->tz, &d->next_cal);
        d->tei = d->next_cal;
      }
    } else {
      d->tei = hds_align(d, d->next_dp.ts) + d->interval_ms;
    }
  }
}
static int viv_has_next_value(hds* d) {   /* :352-360 */
  viv_init(d);
  if (d->run_all) return d->has_src;
  return d->has_src && d->next_dp.ts < d->tei;
}
static void viv_next_value(hds* d, hval* out) {   /* nextHistogramValue :362-377 (a clone) */
  if (!viv_has_next_value(d) || !d->next_dp_set) hthrow(TSDB_E_NO_SUCH_ELEMENT, "no more values in interval");
  hv_clone(out, &d->next_dp, d->next_dp.ts);
  viv_move_to_next_value(d);
}
static int64_t viv_interval_ts(hds* d) {   /* getIntervalTimestamp :334-345 */
  if (d->run_all) return d->tei;
  if (d->cal_unit) return d->prev_cal;
  return hds_align(d, d->tei - d->interval_ms);
}
static int hds_has(hview* v) { return viv_has_next_value((hds*)v); }
static const hval* hds_next(hview* v) {   /* next :133-149 */
  hds* d = (hds*)v;
  if (!viv_has_next_value(d)) hthrow(TSDB_E_NO_SUCH_ELEMENT, "no more data points");
  if (d->has_value) hv_free(&d->value);
  viv_next_value(d, &d->value);
  d->has_value = 1;
  while (viv_has_next_value(d)) {
    hval o;
    viv_next_value(d, &o);
    /* specification.getHistogramAggregation() is null unless the function is "sum"
     * (DownsamplingSpecification.java:153-157): the adapter's mapAggregation switch throws */
    if (!d->hist_sum) { hv_free(&o); hthrow(TSDB_E_NULL_POINTER, "null HistogramAggregation"); }
    hv_aggregate(&d->value, &o);
    hv_free(&o);
  }
  d->timestamp = viv_interval_ts(d);
  viv_init(d);          /* moveToNextInterval */
  viv_reset_end(d);
  /* timestamp() :96-101 ("all": the query start) is what the aggregation iterator orders by;
   * its clone() carries the timestamp field (for "all" the query end) */
  d->value.ts = d->run_all ? d->qs : d->timestamp;
  d->value.cts = d->timestamp;
  return &d->value;
}
static void hds_seek(hview* v, int64_t ts) {   /* seekInterval :309-331 */
  hds* d = (hds*)v;
  if (d->run_all) {
    d->src->seek(d->src, ts);
  } else if (d->cal_unit) {
    int64_t c;
    cal_prev_or_throw(ts, d->cal_n, d->cal_unit, d->tz, &c);
    if (ts > c) cal_step_or_throw(c, d->cal_unit, d->cal_n, d->tz, &c);
    d->src->seek(d->src, c);
  } else {
    d->src->seek(d->src, hds_align(d, ts + d->interval_ms - 1));
  }
  d->initialized = 0;
}
static void hds_destroy(hview* v) {
  hds* d = (hds*)v;
  if (d->has_value) hv_free(&d->value);
  viv_drop(d);
  d->src->destroy(d->src);
  free(d);
}

/* ---- HistogramAggregationIterator --------------------------------------------------------- */
typedef struct {
  int n;
  hview** its;
  int64_t* ts;
  hval* vals;
  int* has_val;
  int64_t start, end;
  hval value;
  int has_value;
} hagg;
static void hagg_put(hagg* a, int i, const hval* dp) {   /* putDataPoint :178-181 */
  a->ts[i] = dp->ts;
  if (a->has_val[i]) hv_free(&a->vals[i]);
  hv_clone(&a->vals[i], dp, dp->cts);
  a->has_val[i] = 1;
}
static void hagg_end(hagg* a, int i) {   /* endReached :167-170 */
  a->ts[i] = 0;
  if (a->its[i]) a->its[i]->destroy(a->its[i]);
  a->its[i] = NULL;
}
static void hagg_move(hagg* a, int i) {   /* moveToNext :294-301 */
  hview* it = a->its[i];
  if (it->has_next(it)) hagg_put(a, i, it->next(it));
  else hagg_end(a, i);
}
static void hagg_init(hagg* a) {   /* ctor :115-160 */
  for (int i = 0; i < a->n; i++) {
    hview* it = a->its[i];
    it->seek(it, a->start);
    if (!it->has_next(it)) { hagg_end(a, i); continue; }
    const hval* dp = it->next(it);
    if (dp->ts >= a->start) hagg_put(a, i, dp);
    else hagg_end(a, i);
  }
}
static int hagg_has(hagg* a) {   /* :229-237 */
  for (int i = 0; i < a->n; i++)
    if (a->ts[i] != 0 && a->ts[i] <= a->end) return 1;
  return 0;
}
static const hval* hagg_next(hagg* a) {   /* :240-287 */
  if (!hagg_has(a)) hthrow(TSDB_E_NO_SUCH_ELEMENT, "no more elements");
  int64_t min_ts = INT64_MAX;
  int first = -1, multiple = 0;
  for (int i = 0; i < a->n; i++) {
    if (a->ts[i] == 0 || a->ts[i] > a->end) continue;
    if (a->ts[i] < min_ts) { min_ts = a->ts[i]; first = i; multiple = 0; }
    else if (a->ts[i] == min_ts) multiple = 1;
  }
  if (first < 0) hthrow(TSDB_E_NO_SUCH_ELEMENT, "no more elements");
  if (a->has_value) hv_free(&a->value);
  a->value = a->vals[first];   /* this.value = values[first] (the object; putDataPoint replaces the slot) */
  a->has_val[first] = 0;
  a->has_value = 1;
  if (multiple) {
    for (int i = first + 1; i < a->n; i++) {
      if (a->ts[i] == min_ts) {
        hv_aggregate(&a->value, &a->vals[i]);
        hagg_move(a, i);
      }
    }
  }
  hagg_move(a, first);
  return &a->value;
}
static void hagg_free(hagg* a) {
  for (int i = 0; i < a->n; i++) {
    if (a->its[i]) a->its[i]->destroy(a->its[i]);
    if (a->has_val[i]) hv_free(&a->vals[i]);
  }
  if (a->has_value) hv_free(&a->value);
  free(a->its); free(a->ts); free(a->vals); free(a->has_val);
}

/* ---- the query ------------------------------------------------------------------------- */
typedef struct { void* p; int64_t n, cap; size_t el; } dvec;
static void* dv_push(dvec* v, int64_t k) {   /* room for k more elements; returns the first */
  if (v->n + k > v->cap) {
    int64_t nc = v->cap ? v->cap : 16;
    while (nc < v->n + k) nc *= 2;
    v->p = hx(realloc(v->p, v->el * (size_t)nc));
    v->cap = nc;
  }
  void* at = (char*)v->p + v->el * (size_t)v->n;
  v->n += k;
  return at;
}
typedef struct {
  dvec ts, pct, gid, gptr, bkptr, bkt, bklo, bkup, bvoff, bv;
} hout;
static void hout_init(hout* o) {
  memset(o, 0, sizeof *o);
  o->ts.el = 8; o->pct.el = 8; o->gid.el = 4; o->gptr.el = 8; o->bkptr.el = 8; o->bkt.el = 4; o->bklo.el = 4;
  o->bkup.el = 4; o->bvoff.el = 8; o->bv.el = 8;
  *(int64_t*)dv_push(&o->gptr, 1) = 0;
  *(int64_t*)dv_push(&o->bkptr, 1) = 0;
  *(int64_t*)dv_push(&o->bvoff, 1) = 0;
}

/* the bucket map of a point: getHistogramBucketsIfHas (:110-135 of the adapter) */
static void bucket_map(const hval* h, treemap* t) {
  t->root = NULL;
  t->n = 0;
  if (t->cap < h->nb + 2) {
    t->cap = h->nb + 2;
    t->pool = (tm_node*)hx(realloc(t->pool, sizeof(tm_node) * (size_t)t->cap));
  }
  for (int i = 0; i < h->nb; i++) { hbucket k = {BK_REG, h->b[i].lo, h->b[i].up}; tm_put(t, k, h->b[i].cnt); }
  hbucket u = {BK_UNDER, 0, 0}, o = {BK_OVER, 0, 0};
  tm_put(t, u, h->under);
  tm_put(t, o, h->over);
}
static void tm_inorder(const tm_node* x, hbucket* out, int* n) {
  if (!x) return;
  tm_inorder(x->l, out, n);
  out[(*n)++] = x->key;
  tm_inorder(x->r, out, n);
}

/* One HistogramSpanGroup: its spans, drained through the aggregation iterator. */
static void run_group(int32_t gid, hspan** spans, int ns, const tsdbhip_query* q, int64_t ss_ms, int64_t se_ms,
                      int n_pct, const float* pct, int show_buckets, hout* o) {
  /* HistogramSpanGroup.add (:160-205): spans with a data point in [start, end] */
  hspan** kept = (hspan**)HMALLOC(sizeof(hspan*) * (size_t)(ns ? ns : 1));
  int nk = 0;
  for (int i = 0; i < ns; i++) {
    const int64_t sz = span_size(spans[i]);
    if (sz == 0) continue;
    int64_t first = span_ts(spans[i], 0), last = span_ts(spans[i], sz - 1);
    if ((first & (int64_t)0xFFFFFFFF00000000LL) == 0) first *= 1000;
    if ((last & (int64_t)0xFFFFFFFF00000000LL) == 0) last *= 1000;
    if (first <= se_ms && last >= ss_ms) kept[nk++] = spans[i];
  }
  hagg a;
  memset(&a, 0, sizeof a);
  a.n = nk;
  a.its = (hview**)HCALLOC((size_t)nk, sizeof(hview*));
  a.ts = (int64_t*)HCALLOC((size_t)nk, sizeof(int64_t));
  a.vals = (hval*)HCALLOC((size_t)nk, sizeof(hval));
  a.has_val = (int*)HCALLOC((size_t)nk, sizeof(int));
  a.start = ss_ms;
  a.end = se_ms;
  for (int i = 0; i < nk; i++) {   /* HistogramAggregationIterator.create :91-113 */
    hview* it = span_iterator(kept[i]);
    if (q->ds_function >= 0) {
      hds* d = (hds*)HCALLOC(1, sizeof *d);
      d->v.has_next = hds_has; d->v.next = hds_next; d->v.seek = hds_seek; d->v.destroy = hds_destroy;
      d->src = it;
      d->run_all = q->ds_all;
      d->hist_sum = q->ds_function == TSDB_AGG_SUM;
      d->interval_ms = q->ds_interval_ms;
      d->qs = q->start_time;   /* TsdbQuery.getStartTime(): as set (s or ms), TsdbQuery.java:1093-1094 */
      d->qe = q->end_time;
      if (q->ds_calendar && !q->ds_all) {
        static const int64_t U[9] = {0, 1, 1000, 60000, 3600000, 86400000, 604800000, 2592000000LL, 31536000000LL};
        d->cal_unit = q->ds_calendar;
        d->cal_n = q->ds_interval_ms / U[q->ds_calendar];
        d->tz = q->ds_tz;
      }
      if (!d->run_all) d->tei = d->cal_unit ? INT64_MIN : d->interval_ms;   /* ValuesInInterval() :210-216 */
      else d->tei = d->qe;
      it = &d->v;
    }
    a.its[i] = it;
  }
  /* emit the group: drain the iterator once (every adaptor iterates the same sequence) */
  *(int32_t*)dv_push(&o->gid, 1) = gid;
  treemap tm = {0};
  hbucket* first_keys = NULL;
  int nfirst = 0;
  dvec* bkv = NULL;   /* per bucket series: values */
  int first = 1;
  hagg_init(&a);
  while (hagg_has(&a)) {
    const hval* h = hagg_next(&a);
    *(int64_t*)dv_push(&o->ts, 1) = h->ts;
    double* pv = n_pct ? (double*)dv_push(&o->pct, n_pct) : NULL;
    for (int j = 0; j < n_pct; j++) pv[j] = hv_percentile(h, (double)pct[j]);
    if (show_buckets) {
      if (first && h->kind == TSDB_HCODEC_SIMPLE) {   /* generateHistogramBucketDataPoints :1268-1287 */
        bucket_map(h, &tm);
        first_keys = (hbucket*)HMALLOC(sizeof(hbucket) * (size_t)tm.n);
        tm_inorder(tm.root, first_keys, &nfirst);
        bkv = (dvec*)HCALLOC((size_t)nfirst, sizeof(dvec));
        for (int b = 0; b < nfirst; b++) bkv[b].el = 8;
      }
      if (nfirst) {   /* HistogramBucketDataPointsAdaptor.Iterator.next: containsKey / get */
        if (h->kind == TSDB_HCODEC_SIMPLE) bucket_map(h, &tm);
        for (int b = 0; b < nfirst; b++) {
          int64_t val = 0;
          if (h->kind == TSDB_HCODEC_SIMPLE) {
            const tm_node* e = tm_get(&tm, &first_keys[b]);
            if (e) val = e->val;
          }
          *(int64_t*)dv_push(&bkv[b], 1) = val;
        }
      }
    }
    first = 0;
  }
  *(int64_t*)dv_push(&o->gptr, 1) = o->ts.n;
  for (int b = 0; b < nfirst; b++) {
    *(int32_t*)dv_push(&o->bkt, 1) = first_keys[b].type;
    *(uint32_t*)dv_push(&o->bklo, 1) = first_keys[b].lo;
    *(uint32_t*)dv_push(&o->bkup, 1) = first_keys[b].up;
    if (bkv[b].n) memcpy(dv_push(&o->bv, bkv[b].n), bkv[b].p, 8 * (size_t)bkv[b].n);
    free(bkv[b].p);
  }
  *(int64_t*)dv_push(&o->bkptr, 1) = o->bkt.n;
  *(int64_t*)dv_push(&o->bvoff, 1) = o->bv.n;
  free(bkv);
  free(first_keys);
  free(tm.pool);
  hagg_free(&a);
  free(kept);
}

static void hout_free(hout* o) {
  dvec* all[] = {&o->ts, &o->pct, &o->gid, &o->gptr, &o->bkptr, &o->bkt, &o->bklo, &o->bkup, &o->bvoff, &o->bv};
  for (size_t i = 0; i < sizeof all / sizeof *all; i++) free(all[i]->p);
}
static int run_hist(const tsdbhip_hist_batch* hb, const tsdbhip_query* q, int64_t ss_ms, int64_t se_ms,
                    int64_t row_lo, int64_t row_hi, int n_pct, const float* pct, int show_buckets,
                    ref_hist_result** out) {
  *out = NULL;
  int rc = 0;
  const int64_t S = hb->n_series;
  hspan* spans = (hspan*)calloc((size_t)(S ? S : 1), sizeof(hspan));
  hout o;
  hout_init(&o);
  jmp_buf jb;
  jmp_buf* prev = h_jb;
  h_jb = &jb;
  if (setjmp(jb) == 0) {
    /* the scan: rows with base time in [scan start, scan end), columns decoded, spans built
     * (SaltScanner.processRow / mergeHistogramDataPoints :336-378) */
    for (int64_t s = 0; s < S; s++) {
      for (int64_t r = hb->series_row_ptr[s]; r < hb->series_row_ptr[s + 1]; r++) {
        const int64_t base = hb->row_base_time[r];
        if (base < row_lo || base >= row_hi) continue;
        const int64_t c0 = hb->row_cell_ptr[r], c1 = hb->row_cell_ptr[r + 1];
        hval* dps = (hval*)HCALLOC((size_t)(c1 - c0), sizeof(hval));
        int n = 0;
        for (int64_t c = c0; c < c1; c++) {
          const uint8_t* qp = hb->qual + hb->cell_qual_off[c];
          const int64_t ql = (int64_t)(hb->cell_qual_off[c + 1] - hb->cell_qual_off[c]);
          if (ql < 1 || qp[0] != 0x06) continue;   /* not a histogram column */
          int64_t ts;
          if (nondp_ts(base, qp, ql, &ts)) continue;
          if (hv_decode(hb->val + hb->cell_val_off[c], (int64_t)(hb->cell_val_off[c + 1] - hb->cell_val_off[c]),
                        hb->codec, &dps[n]))
            continue;
          dps[n].ts = dps[n].cts = ts;
          n++;
        }
        if (n == 0) { free(dps); continue; }
        span_add_row(&spans[s], base, dps, n);
      }
      span_sort(&spans[s]);
    }
    if (q->aggregator == TSDB_AGG_NONE) {   /* :1085-1123: every span its own group */
      for (int64_t s = 0; s < S; s++) {
        if (!spans[s].nr) continue;
        hspan* one = &spans[s];
        run_group((int32_t)s, &one, 1, q, ss_ms, se_ms, n_pct, pct, show_buckets, &o);
      }
    } else {
      int32_t G = -1;
      for (int64_t s = 0; s < S; s++)
        if (spans[s].nr && hb->group_id[s] > G) G = hb->group_id[s];
      hspan** members = (hspan**)HMALLOC(sizeof(hspan*) * (size_t)(S ? S : 1));
      for (int32_t g = 0; g <= G; g++) {
        int nm = 0;
        for (int64_t s = 0; s < S; s++)
          if (spans[s].nr && hb->group_id[s] == g) members[nm++] = &spans[s];
        if (nm) run_group(g, members, nm, q, ss_ms, se_ms, n_pct, pct, show_buckets, &o);
      }
      free(members);
    }
  } else {
    rc = h_code;
  }
  h_jb = prev;
  for (int64_t s = 0; s < S; s++) span_free(&spans[s]);
  free(spans);
  if (rc) { hout_free(&o); return rc; }
  ref_hist_result* r = (ref_hist_result*)calloc(1, sizeof *r);
  dvec* all[] = {&o.ts, &o.pct, &o.gid, &o.gptr, &o.bkptr, &o.bkt, &o.bklo, &o.bkup, &o.bvoff, &o.bv};
  for (size_t i = 0; i < sizeof all / sizeof *all; i++)
    if (!all[i]->p) all[i]->p = calloc(1, 8);
  r->n_groups = o.gid.n;
  r->group_id = (int32_t*)o.gid.p;
  r->group_ptr = (int64_t*)o.gptr.p;
  r->ts = (int64_t*)o.ts.p;
  r->n_pct = n_pct;
  r->pct = (double*)o.pct.p;
  r->bk_ptr = (int64_t*)o.bkptr.p;
  r->bk_type = (int32_t*)o.bkt.p;
  r->bk_lo = (uint32_t*)o.bklo.p;
  r->bk_up = (uint32_t*)o.bkup.p;
  r->bk_val_off = (int64_t*)o.bvoff.p;
  r->bk_val = (int64_t*)o.bv.p;
  *out = r;
  return 0;
}

int ref_run_hist(const tsdbhip_hist_batch* hb, const tsdbhip_query* q, int n_pct, const float* pct,
                 int show_buckets, ref_hist_result** out) {
  int64_t ss, se;
  const int rc = ref_scan_bounds(q, &ss, &se);
  if (rc) return rc;
  /* the scan returns rows with base time in [scan start, scan end); HistogramSpanGroup's bounds are
   * the scan bounds in ms (TsdbQuery.java:1128-1138, HistogramSpanGroup.java:119-122) */
  return run_hist(hb, q, ss * 1000, se * 1000, ss, se, n_pct, pct, show_buckets, out);
}

int ref_run_hist_range(const tsdbhip_hist_batch* hb, const tsdbhip_query* q, int64_t start_ms, int64_t end_ms,
                       int n_pct, const float* pct, int show_buckets, ref_hist_result** out) {
  return run_hist(hb, q, start_ms, end_ms, INT64_MIN, INT64_MAX, n_pct, pct, show_buckets, out);
}

void ref_hist_result_free(ref_hist_result* r) {
  if (!r) return;
  free(r->group_id); free(r->group_ptr); free(r->ts); free(r->pct); free(r->bk_ptr); free(r->bk_type);
  free(r->bk_lo); free(r->bk_up); free(r->bk_val_off); free(r->bk_val);
  free(r);
}
