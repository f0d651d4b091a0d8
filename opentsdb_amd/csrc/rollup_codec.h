// rollup_codec.h -- the rollup cell codec, shared by the host ABI functions and the
// generation kernels (k_rollup.hip).  Java int arithmetic (32-bit wrap, truncating
// division) is restated explicitly.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace tsdb {

constexpr int64_t RC_SECOND_MASK = (int64_t)0xFFFFFFFF00000000ULL;   // Const.SECOND_MASK

struct RollupIv {
  int32_t interval_s;
  int32_t intervals;
  char units;
  int32_t mult;
};

__host__ __device__ inline int32_t jint(int64_t x) { return (int32_t)(uint32_t)(uint64_t)x; }

// days since 1970-01-01 -> (year, month 1..12); proleptic Gregorian, which is what
// java.util.GregorianCalendar uses for every date after 1582.
__host__ __device__ inline void rc_civil(int64_t days, int64_t& y, int& m) {
  const int64_t z = days + 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const int64_t doe = z - era * 146097;
  const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const int64_t mp = (5 * doy + 2) / 153;
  m = (int)(mp < 10 ? mp + 3 : mp - 9);
  y = yoe + era * 400 + (m <= 2 ? 1 : 0);
}

__host__ __device__ inline int64_t rc_days_from_civil(int64_t y, int m, int d) {
  y -= m <= 2 ? 1 : 0;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const int64_t yoe = y - era * 400;
  const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}

// RollupUtils.getRollupBasetime (src/rollup/RollupUtils.java:52-112).  Returns false for
// IllegalArgumentException (negative timestamp, unknown span).
__host__ __device__ inline bool rc_basetime(int64_t ts, const RollupIv& iv, int32_t& out) {
  if (ts < 0) return false;
  if (iv.units == 'h') {
    const int64_t modulo = iv.mult > 1 ? (int64_t)iv.mult * 3600 : 3600;   // Const.MAX_TIMESPAN
    if ((ts & RC_SECOND_MASK) != 0) {
      const int64_t s = ts / 1000;
      out = jint(s - s % modulo);
    } else {
      out = jint(ts - ts % modulo);
    }
    return true;
  }
  const int64_t ms = (ts & RC_SECOND_MASK) != 0 ? ts : ts * 1000;
  const int64_t days = ms / 86400000;   // UTC calendar; HOUR/MINUTE/SECOND zeroed (ms kept, truncated below)
  const int64_t rem_ms = ms % 86400000 % 1000;
  int64_t day0;
  if (iv.units == 'd') {
    day0 = days;
  } else if (iv.units == 'n' || iv.units == 'y') {
    int64_t y;
    int m;
    rc_civil(days, y, m);
    day0 = rc_days_from_civil(y, iv.units == 'n' ? m : 1, 1);
  } else {
    return false;
  }
  out = jint((day0 * 86400000 + rem_ms) / 1000);
  return true;
}

// RollupUtils.buildRollupQualifier (src/rollup/RollupUtils.java:143-171).  Returns false
// for IllegalArgumentException (offset >= intervals).
__host__ __device__ inline bool rc_qualifier(int64_t ts, int32_t base, int16_t flags, int32_t agg_id,
                                             const RollupIv& iv, uint8_t q[3]) {
  const int32_t tsec = jint((ts & RC_SECOND_MASK) != 0 ? ts / 1000 : ts);
  int32_t off = (int32_t)((uint32_t)tsec - (uint32_t)base) / iv.interval_s;
  if (off >= iv.intervals) return false;
  off = (int32_t)((uint32_t)off << 4) | (int32_t)flags;
  q[0] = (uint8_t)agg_id;
  q[1] = (uint8_t)((uint32_t)off >> 8);
  q[2] = (uint8_t)off;
  return true;
}

// TSDB.addAggregatePoint value encodings (src/core/TSDB.java:1322-1438):
// vleEncodeLong (src/core/Internal.java:963-973) -> flags = length - 1.
__host__ __device__ inline int rc_vle_len(int64_t v) {
  if (v == (int8_t)v) return 1;
  if (v == (int16_t)v) return 2;
  if (v == (int32_t)v) return 4;
  return 8;
}

// Java (long) of a double: truncation, saturating, NaN -> 0.
__host__ __device__ inline int64_t rc_d2l(double v) {
  if (v != v) return 0;
  if (v >= 9223372036854775807.0) return INT64_MAX;
  if (v <= -9223372036854775808.0) return INT64_MIN;
  return (int64_t)v;
}

// Value of a rollup cell: returns the encoded length (1/2/4/8), the qualifier flags and
// the big-endian bytes in `be` (the low `len` bytes, most significant first), or 0 when
// addAggregatePoint would reject the value (NaN / infinite float).
__host__ __device__ inline int rc_value(double v, bool as_long, int16_t& flags, uint64_t& be) {
  if (as_long) {
    const int64_t l = rc_d2l(v);
    const int len = rc_vle_len(l);
    flags = (int16_t)(len - 1);
    be = (uint64_t)l;
    return len;
  }
  if (v != v || v == INFINITY || v == -INFINITY) return 0;
  const float f = (float)v;
  if ((double)f == v) {   // Tags.fitsInFloat (src/core/Tags.java:853-858)
    union { float f; uint32_t u; } c;
    c.f = f;
    flags = 0x8 | 0x3;
    be = c.u;
    return 4;
  }
  union { double d; uint64_t u; } c;
  c.d = v;
  flags = 0x8 | 0x7;
  be = c.u;
  return 8;
}

}  // namespace tsdb
