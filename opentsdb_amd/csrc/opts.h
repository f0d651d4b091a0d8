// Developer options of libtsdbhip: kernel-choice switches for the parity tests (force the
// general kernel, a sequential path, small chunks ...) and for A/B measurements.
//
// The library reads NO environment variable.  An option changes only when a caller sets it
// through tsdbhip_set_option (include/tsdbhip.h); every option starts unset (-1), which is the
// production choice.  Options are process-wide, like the code objects they pick between.
#pragma once
#include <cstdint>

namespace tsdb {

enum Opt : int {
  OPT_FAST,           // 0: every tile through the general kernel k_grid
  OPT_SHORT,          // 0: no k_short (one-row series take k_fast)
  OPT_ROWS,           // 0: no k_rows (one-chunk rows take the k_fast row walker)
  OPT_HWIN,           // 0: no k_hwin (K > 64 through the dense split); 2: also for the fused multi pass
  OPT_SEQ,            // 0: no sequential dense kernels (full-mantissa sums through k_grid)
  OPT_SEQ_ROWS,       // 0: no k_seq_rows (k_seq_dense instead)
  OPT_SEQ_WAVE,       // 0: k_seq_dense (a series a lane) instead of k_seq_wave
  OPT_INDEX_GENERIC,  // 1: the sequential per-datapoint index path for every row
  OPT_CMP_CHUNK,      // > 0: compaction chunks of at most this many columns / datapoints
  OPT_CMP_ROWS,       // 0: the global-sort compaction pipeline instead of the per-row one
  OPT_CMP_ONEPASS,    // 0: the two-pass per-row compaction
  OPT_PCT_ROWS,       // 0: percentile downsampling without k_pct_rows
  OPT_PCT_KEYS,       // 0: no 32-bit key kernel for 1 h percentile buckets
  OPT_PCT_VONLY,      // 0: key rows read qualifiers too
  OPT_PCT_V6,         // 0: values-only key rows without the 6-point lanes
  OPT_SEL_FUSED,      // 0: percentile group-by contributions through pre_dense + k_emit_vals
  OPT_SEL_COLS,       // 0: contributions row by row instead of contiguous (group, slot) columns
  OPT_SEL_WIN,        // 0: never the sampled window; 2: also for small groups and mid ranks
  OPT_SEL_WAVE,       // 0: columns of <= 2048 values through k_sel_reg instead of k_sel_wave
  OPT_SEL_REG,        // 0: the LDS k_sel_seg for every column
  OPT_SELOPS,         // > 0: raw percentile batches of at most this many operands
  OPT_RAW_LERPW,      // 0: the general 64-bit raw LERP (no strip-wide windows)
  OPT_RAW_SEL_TOP,    // 0: raw percentiles through the per-point kernels
  OPT_RAW_SEL_REG,    // 0: the LDS-staged raw percentile kernel
  OPT_RO_FUSE,        // 0: rollup avg / count in two passes
  OPT_RO_RUNS,        // 0: rollup pairs read packed, not as runs
  OPT_MULTI_FUSE,     // 0: tsdbhip_run_multi query by query
  OPT_EMIT_HALF,      // 0: no two-series-a-step group-by over stored buckets (k_emit_reg2, K <= 32)
  OPT_HIST_WINDOW,    // 0: the per-column atomic histogram kernel
  OPT_HIST_WS,        // > 0: histogram windows of at most this many points
  OPT_HIST_LAYOUT,    // 0: every histogram bucket through the keyed lookup
  OPT_TRACE,          // 1: host wall time of load / query phases on stderr
  OPT_DBG,            // profiling bits (results invalid); honoured only by a -DTSDBHIP_KDBG build
  OPT_COUNT
};

// -1 when unset
int64_t opt(Opt o);
inline bool opt_is(Opt o, int64_t v) { return opt(o) == v; }
inline bool opt_off(Opt o) { return opt(o) == 0; }

}  // namespace tsdb
