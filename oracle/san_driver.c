/*
 * san_driver.c -- TEST INFRASTRUCTURE ONLY.  Sanitizer driver for the CPU oracle: built with
 * -fsanitize=address,undefined together with refcpu.c (make -C oracle san), it runs the oracle
 * over synthetic compacted cells of every row shape the reference reads (2-byte second and
 * 4-byte millisecond qualifiers, vle integers of 1/2/4/8 bytes, float32/float64, NaN values,
 * duplicate and out-of-order timestamps, a malformed value length) through a matrix of
 * aggregators x downsamplers x fill policies x rate options, single- and multi-threaded.
 * The CPU pytest suite runs against the UBSan build of the shared library
 * (TSDB_ORACLE_LIB=oracle/build/librefcpu_ubsan.so); ASan needs its runtime first in the
 * process, so the ASan leg is this stand-alone executable.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "refcpu.h"

typedef struct {
  uint8_t* p;
  size_t n, cap;
} Buf;

static void put(Buf* b, const void* src, size_t n) {
  if (b->n + n > b->cap) {
    b->cap = (b->n + n) * 2 + 64;
    b->p = (uint8_t*)realloc(b->p, b->cap);
  }
  memcpy(b->p + b->n, src, n);
  b->n += n;
}

static void put_be(Buf* b, uint64_t v, int len) {
  uint8_t t[8];
  for (int i = 0; i < len; i++) t[i] = (uint8_t)(v >> (8 * (len - 1 - i)));
  put(b, t, (size_t)len);
}

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t next(void) {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return rng;
}

/* one datapoint: qualifier + value (Internal.java:621-810, RowSeq.java:233-266) */
static void emit_point(Buf* q, Buf* v, int ms_qual, uint32_t off, int kind, int bad) {
  int len;
  int fl;
  uint64_t bits;
  switch (kind) {
    case 0: len = 1; fl = 0; bits = (uint64_t)(int64_t)(int8_t)(next() % 200); break;
    case 1: len = 2; fl = 0; bits = (uint64_t)(int64_t)(int16_t)(next() % 60000); break;
    case 2: len = 4; fl = 0; bits = (uint64_t)(uint32_t)(int32_t)(next() % 2000000); break;
    case 3: len = 8; fl = 0; bits = next() % 4000000000ull; break;
    case 4: {
      float f = (float)((double)(next() % 100000) / 7.0);
      if (next() % 50 == 0) f = NAN;
      uint32_t u;
      memcpy(&u, &f, 4);
      len = 4; fl = 0x8; bits = u;
      break;
    }
    default: {
      double d = (double)(next() % 1000000) / 3.0 - 1000.0;
      if (next() % 50 == 0) d = NAN;
      memcpy(&bits, &d, 8);
      len = 8; fl = 0x8;
      break;
    }
  }
  const int lcode = bad ? 2 : len - 1;   /* a 3-byte length: IllegalDataException on read */
  if (ms_qual) put_be(q, 0xF0000000u | ((uint64_t)off << 6) | (uint64_t)(fl | lcode), 4);
  else put_be(q, ((uint64_t)off << 4) | (uint64_t)(fl | lcode), 2);
  put_be(v, bits, len);
}

typedef struct {
  int64_t n_series, n_rows;
  int64_t* srp;
  uint32_t* base;
  uint64_t *qoff, *voff;
  Buf q, v;
  int32_t* gid;
} Batch;

static void make_batch(Batch* B, int64_t n_series, int rows_per, int pts, uint32_t t0, int with_bad) {
  memset(B, 0, sizeof(*B));
  B->n_series = n_series;
  B->n_rows = n_series * rows_per;
  B->srp = (int64_t*)calloc((size_t)n_series + 1, 8);
  B->base = (uint32_t*)calloc((size_t)B->n_rows, 4);
  B->qoff = (uint64_t*)calloc((size_t)B->n_rows + 1, 8);
  B->voff = (uint64_t*)calloc((size_t)B->n_rows + 1, 8);
  B->gid = (int32_t*)calloc((size_t)n_series, 4);
  int64_t r = 0;
  for (int64_t s = 0; s < n_series; s++) {
    B->srp[s] = r;
    B->gid[s] = (s % 5 == 4) ? -1 : (int32_t)(s % 3);
    for (int k = 0; k < rows_per; k++, r++) {
      B->base[r] = t0 + (uint32_t)k * 3600u;
      B->qoff[r] = B->q.n;
      B->voff[r] = B->v.n;
      const int shape = (int)((s + k) % 4);   /* 0 s-quals, 1 ms-quals, 2 mixed, 3 mixed kinds */
      const int kind0 = (int)(next() % 6);
      uint32_t prev_ms = 0;
      for (int i = 0; i < pts; i++) {
        int ms = shape == 1 || (shape == 2 && (i & 1));
        uint32_t off_ms = (uint32_t)(i * (3600000 / pts)) + (uint32_t)(next() % 7) * 1000u;
        if (off_ms <= prev_ms && i) off_ms = prev_ms + 1000;   /* strictly increasing */
        if (off_ms >= 3600000u) break;
        prev_ms = off_ms;
        const int kind = shape == 3 ? (int)(next() % 6) : kind0;
        const int bad = with_bad && s == 1 && k == 0 && i == 3;
        if (ms) emit_point(&B->q, &B->v, 1, off_ms, kind, bad);
        else emit_point(&B->q, &B->v, 0, off_ms / 1000u, kind, bad);
      }
      const uint8_t meta = 0;
      put(&B->v, &meta, 1);
    }
  }
  B->srp[n_series] = r;
  B->qoff[r] = B->q.n;
  B->voff[r] = B->v.n;
}

static void free_batch(Batch* B) {
  free(B->srp);
  free(B->base);
  free(B->qoff);
  free(B->voff);
  free(B->gid);
  free(B->q.p);
  free(B->v.p);
}

static long runs = 0, errors = 0;

static void run(const Batch* B, const tsdbhip_query* q) {
  tsdbhip_batch b = {B->n_series, B->srp, B->n_rows, B->base, B->qoff, B->voff, B->q.p, B->v.p, B->gid};
  ref_result* r = NULL;
  int rc = ref_run_query(&b, q, &r);
  runs++;
  if (rc) errors++;
  else ref_result_free(r);
  r = NULL;
  rc = ref_run_query_mt(&b, q, 3, &r);
  runs++;
  if (rc) errors++;
  else ref_result_free(r);
}

int main(void) {
  const uint32_t t0 = 1356998400u;
  Batch B, Bad;
  make_batch(&B, 12, 3, 97, t0, 0);
  make_batch(&Bad, 4, 2, 40, t0, 1);
  const int aggs[] = {TSDB_AGG_SUM, TSDB_AGG_PFSUM, TSDB_AGG_MIN, TSDB_AGG_MAX, TSDB_AGG_AVG, TSDB_AGG_MEDIAN,
                      TSDB_AGG_NONE, TSDB_AGG_MULT, TSDB_AGG_DEV, TSDB_AGG_DIFF, TSDB_AGG_ZIMSUM, TSDB_AGG_MIMMIN,
                      TSDB_AGG_MIMMAX, TSDB_AGG_SQUARESUM, TSDB_AGG_COUNT, TSDB_AGG_FIRST, TSDB_AGG_LAST,
                      TSDB_AGG_P99, TSDB_AGG_EP95R3, TSDB_AGG_EP50R7};
  const char* ds[] = {NULL, "1m-sum", "10m-avg", "1h-p95", "30s-count-zero", "1m-max-nan", "2m-dev-null",
                      "0all-sum", "1h-median", "10m-first", "1dc-sum", "1nc-avg", "15m-ep99r7", "1m-squareSum"};
  for (size_t a = 0; a < sizeof(aggs) / sizeof(aggs[0]); a++) {
    for (size_t d = 0; d < sizeof(ds) / sizeof(ds[0]); d++) {
      for (int rate = 0; rate < 3; rate++) {
        tsdbhip_query q;
        memset(&q, 0, sizeof(q));
        q.ds_function = -1;
        if (ds[d] && ref_parse_downsample(ds[d], &q)) {
          fprintf(stderr, "parse %s: %s\n", ds[d], ref_last_error());
          return 2;
        }
        q.start_time = t0 + 60;
        q.end_time = t0 + 3 * 3600 - 61;
        q.aggregator = aggs[a];
        q.rate = rate > 0;
        q.rate_counter = rate == 2;
        q.rate_drop_resets = rate == 2 && (a & 1);
        q.rate_counter_max = rate == 2 ? 70000 : INT64_MAX;
        q.rate_reset_value = rate == 2 ? 100 : 0;
        run(&B, &q);
        if (d < 3) run(&Bad, &q);
      }
    }
  }
  /* Aggregator.run* over plain arrays, including empty and NaN inputs */
  double dv[64];
  int64_t lv[64];
  for (int i = 0; i < 64; i++) {
    dv[i] = (i % 9 == 0) ? NAN : (double)i * 1.5 - 20.0;
    lv[i] = (int64_t)i * 3 - 50;
  }
  for (size_t a = 0; a < sizeof(aggs) / sizeof(aggs[0]); a++) {
    for (int n = 0; n <= 64; n += 7) {
      double od;
      int64_t ol;
      (void)ref_agg_run_double(aggs[a], dv, n, &od);
      (void)ref_agg_run_long(aggs[a], lv, n, &ol);
    }
  }
  /* parse helpers on odd strings */
  const char* odd[] = {"", "1", "m", "0m-sum", "-1m-sum", "1x-sum", "1m-sum-bogus", "99999999999999999999y-sum",
                       "1m-p999-zero", "all-sum", "1m-sum-", "1mc-sum", "7sc-sum", "2wc-max"};
  for (size_t i = 0; i < sizeof(odd) / sizeof(odd[0]); i++) {
    tsdbhip_query q;
    int64_t ms;
    memset(&q, 0, sizeof(q));
    (void)ref_parse_downsample(odd[i], &q);
    (void)ref_parse_duration(odd[i], &ms);
    (void)ref_aggregator_get(odd[i]);
  }
  free_batch(&B);
  free_batch(&Bad);
  printf("san_driver: %ld oracle queries (%ld raised a TSDB_E_* error as the reference would), clean\n", runs,
         errors);
  return 0;
}
