// plan.cpp — segment planning on the host (C++), bit-exact with the reference.
//
// The reference planner is Python float (IEEE double) and int arithmetic.  Every
// function here follows the reference statement by statement, including
// Python's min()/max() tie rules (min/max return the FIRST argument unless the
// second compares strictly smaller/larger), so results match bit for bit:
//   plan_segments              utils/video_segmenter.py:42-83
//   _estimate_segments         utils/budget_planner.py:43-53
//   _estimate_calls            utils/budget_planner.py:56-70
//   plan_segments_with_budget  utils/budget_planner.py:73-194
// Python bigints become int64 here; a result that would leave int64 returns
// VTS_E_RANGE instead of silently wrapping.
#include <cmath>
#include <cstring>
#include <limits>

#include "common.h"

namespace vts {

std::string &last_error() {
  static thread_local std::string msg;
  return msg;
}

namespace {

// Python builtins max(a, b) / min(a, b) on two floats.
inline double py_max(double a, double b) { return (b > a) ? b : a; }
inline double py_min(double a, double b) { return (b < a) ? b : a; }
inline int64_t py_max_i(int64_t a, int64_t b) { return (b > a) ? b : a; }
inline int64_t py_min_i(int64_t a, int64_t b) { return (b < a) ? b : a; }

// int(math.ceil(x)) with Python's exceptions.
int py_ceil_int(double x, int64_t *out) {
  if (std::isnan(x)) return fail(VTS_E_VALUE, "cannot convert float NaN to integer");
  if (std::isinf(x)) return fail(VTS_E_OVERFLOW, "cannot convert float infinity to integer");
  double c = std::ceil(x);
  // int64 range is [-2^63, 2^63); 2^63 itself is exactly representable.
  if (c >= 9223372036854775808.0 || c < -9223372036854775808.0)
    return fail(VTS_E_RANGE, "integer %g outside int64", c);
  *out = static_cast<int64_t>(c);
  return VTS_OK;
}

inline int add_i(int64_t a, int64_t b, int64_t *out) {
  if (__builtin_add_overflow(a, b, out)) return fail(VTS_E_RANGE, "int64 overflow");
  return VTS_OK;
}
inline int sub_i(int64_t a, int64_t b, int64_t *out) {
  if (__builtin_sub_overflow(a, b, out)) return fail(VTS_E_RANGE, "int64 overflow");
  return VTS_OK;
}
inline int mul_i(int64_t a, int64_t b, int64_t *out) {
  if (__builtin_mul_overflow(a, b, out)) return fail(VTS_E_RANGE, "int64 overflow");
  return VTS_OK;
}

// Python a // b on ints (floor division).
int py_floordiv(int64_t a, int64_t b, int64_t *out) {
  if (b == 0) return fail(VTS_E_ZERODIV, "integer division or modulo by zero");
  if (a == std::numeric_limits<int64_t>::min() && b == -1)
    return fail(VTS_E_RANGE, "int64 overflow");
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  *out = q;
  return VTS_OK;
}

// Python `float <= int` / `float < int` for ints within +-2^53 (exact there).
inline double as_f(int64_t v) { return static_cast<double>(v); }

// _estimate_segments (budget_planner.py:43-53)
int estimate_segments(double duration, int64_t segment_duration, int64_t overlap,
                      int64_t *out) {
  if (duration <= 0) {
    *out = 0;
    return VTS_OK;
  }
  segment_duration = py_max_i(segment_duration, 1);
  overlap = py_max_i(py_min_i(overlap, segment_duration - 1), 0);
  if (duration <= as_f(segment_duration)) {
    *out = 1;
    return VTS_OK;
  }
  int64_t stride = segment_duration - overlap;
  if (stride <= 0) stride = 1;
  int64_t c = 0;
  VTS_TRY(py_ceil_int((duration - as_f(segment_duration)) / as_f(stride), &c));
  return add_i(c, 1, out);
}

// _estimate_calls (budget_planner.py:56-70)
int estimate_calls(int64_t num_segments, int64_t max_continuations,
                   int64_t retry_buffer, int64_t extra_calls, int64_t *out) {
  if (num_segments <= 0) {
    *out = 0;
    return VTS_OK;
  }
  int64_t t = 0, prod = 0;
  VTS_TRY(add_i(num_segments, 1, &t));
  VTS_TRY(add_i(t, extra_calls, &t));
  VTS_TRY(mul_i(num_segments, max_continuations, &prod));
  VTS_TRY(add_i(t, prod, &t));
  VTS_TRY(add_i(t, retry_buffer, &t));
  *out = t;
  return VTS_OK;
}

void zero_plan(vts_plan *p, int64_t available, int64_t hard) {
  std::memset(p, 0, sizeof *p);
  p->available_calls = available;
  p->hard_max_calls = hard;
  p->fits_budget = 0;
}

// ceil(duration / n) for the budget loop, int64 n > 0.
int ceil_div_f(double duration, int64_t n, int64_t *out) {
  return py_ceil_int(duration / as_f(n), out);
}

}  // namespace
}  // namespace vts

using namespace vts;

extern "C" int vts_plan_segments(double duration, double segment_seconds,
                                 double overlap_seconds, vts_segment *out,
                                 int64_t cap, int64_t *n_out) {
  clear_error();
  if (!n_out) return fail(VTS_E_INVALID, "n_out is NULL");
  *n_out = 0;
  // video_segmenter.py:45-46
  if (duration <= 0 || segment_seconds <= 0) return VTS_OK;
  // Guard inputs on which the reference `while` never ends or would build an
  // absurd list (it terminates only when cursor stops being < duration).
  if (std::isinf(duration) && duration > 0 && std::isfinite(segment_seconds))
    return fail(VTS_E_NONTERMINATING, "duration is +inf: reference loop never ends");
  if (std::isfinite(duration) && std::isfinite(segment_seconds) &&
      duration / segment_seconds > 4.0e9)
    return fail(VTS_E_RANGE, "more than 4e9 segments");

  const double overlap = py_max(0.0, overlap_seconds);  // :48
  double cursor = 0.0;                                  // :50
  int64_t segment_id = 0;                               // :51
  int64_t n = 0;
  while (cursor < duration) {                           // :53
    const double core_start = cursor;                   // :54
    const double cand = cursor + segment_seconds;
    const double core_end = py_min(cand, duration);     // :55
    const bool eff_end_is_dur = (duration < cand);  // min() returned `duration`
    double extract_start;
    if (core_start == 0) {                              // :57-60
      extract_start = 0.0;
    } else {
      extract_start = py_max(0.0, core_start - overlap);
    }
    double extract_end;
    bool end_is_dur;
    if (core_end >= duration) {                         // :62-65
      extract_end = duration;
      end_is_dur = true;
    } else {
      const double widened = core_end + overlap;
      extract_end = py_min(duration, widened);
      end_is_dur = !(widened < duration);
    }
    if (extract_end <= extract_start) break;            // :67-68
    if (out && n < cap) {
      vts_segment &s = out[n];
      s.segment_id = segment_id;
      s.start = extract_start;
      s.end = extract_end;
      s.effective_start = core_start;
      s.effective_end = core_end;
      s.flags = (end_is_dur ? 1 : 0) | (eff_end_is_dur ? 2 : 0);
    }
    ++n;
    ++segment_id;                                       // :80
    if (core_end == cursor)                             // no progress: endless
      return fail(VTS_E_NONTERMINATING,
                  "cursor stops advancing at %.17g: reference loop never ends", cursor);
    cursor = core_end;                                  // :81
  }
  *n_out = n;
  if (n > 0 && (!out || n > cap))
    return fail(VTS_E_CAPACITY, "need %lld segments", static_cast<long long>(n));
  return VTS_OK;
}

extern "C" int vts_plan_with_budget(double duration, const vts_budget_cfg *cfg,
                                    int64_t current_api_count, vts_plan *out) {
  clear_error();
  if (!cfg || !out) return fail(VTS_E_INVALID, "NULL argument");
  const int64_t default_segment = cfg->default_segment_seconds;
  int64_t overlap = cfg->overlap_seconds;
  const int64_t min_segment = cfg->min_segment_seconds;
  const int64_t hard_max_calls = cfg->hard_max_api_calls;
  const int64_t max_continuations = cfg->max_continuations;
  const int64_t retry_buffer = cfg->retry_times;
  const bool consolidate_enabled = cfg->consolidate != 0;

  duration = py_max(duration, 0.0);  // :104 max(float(duration), 0.0)
  int64_t available_calls = 0;
  VTS_TRY(sub_i(hard_max_calls, current_api_count, &available_calls));
  available_calls = py_max_i(available_calls, 0);  // :105

  if (duration <= 0 || available_calls == 0) {  // :107-116
    zero_plan(out, available_calls, hard_max_calls);
    return VTS_OK;
  }

  int64_t segment_duration = 0;
  if (cfg->has_threshold && duration < cfg->duration_threshold_seconds) {  // :125-427
    int64_t c = 0;
    VTS_TRY(py_ceil_int(duration, &c));
    segment_duration = py_max_i(c, 1);
    overlap = 0;
  } else {
    segment_duration = py_max_i(py_max_i(default_segment, min_segment), 1);  // :129
    int64_t sm1 = 0;
    VTS_TRY(sub_i(segment_duration, 1, &sm1));
    overlap = py_max_i(py_min_i(overlap, sm1), 0);
  }

  int64_t num_segments = 0, estimated_calls = 0;
  const int64_t extra_calls = consolidate_enabled ? 1 : 0;  // :133
  VTS_TRY(estimate_segments(duration, segment_duration, overlap, &num_segments));
  VTS_TRY(estimate_calls(num_segments, max_continuations, retry_buffer, extra_calls,
                         &estimated_calls));

  if (estimated_calls > available_calls) {  // :138-143
    overlap = 0;
    VTS_TRY(estimate_segments(duration, segment_duration, overlap, &num_segments));
    VTS_TRY(estimate_calls(num_segments, max_continuations, retry_buffer, extra_calls,
                           &estimated_calls));
  }

  if (estimated_calls > available_calls && available_calls > 0) {  // :145
    int64_t per_segment_calls = 0, overhead_calls = 0, max_segments = 0, num = 0;
    VTS_TRY(add_i(1, max_continuations, &per_segment_calls));
    VTS_TRY(add_i(1, extra_calls, &overhead_calls));
    VTS_TRY(add_i(overhead_calls, retry_buffer, &overhead_calls));
    VTS_TRY(sub_i(available_calls, overhead_calls, &num));
    VTS_TRY(py_floordiv(num, per_segment_calls, &max_segments));
    if (max_segments < 1) {  // :149-158
      zero_plan(out, available_calls, hard_max_calls);
      return VTS_OK;
    }
    max_segments = py_max_i(max_segments, 1);  // :160
    int64_t c = 0;
    VTS_TRY(ceil_div_f(duration, max_segments, &c));
    segment_duration = py_max_i(py_max_i(c, min_segment), 1);  // :161
    overlap = 0;
    VTS_TRY(estimate_segments(duration, segment_duration, overlap, &num_segments));
    VTS_TRY(estimate_calls(num_segments, max_continuations, retry_buffer, extra_calls,
                           &estimated_calls));
    while (estimated_calls > available_calls && max_segments > 1) {  // :168-176
      max_segments -= 1;
      VTS_TRY(ceil_div_f(duration, max_segments, &c));
      segment_duration = py_max_i(py_max_i(c, min_segment), 1);
      VTS_TRY(estimate_segments(duration, segment_duration, overlap, &num_segments));
      VTS_TRY(estimate_calls(num_segments, max_continuations, retry_buffer, extra_calls,
                             &estimated_calls));
    }
    if (estimated_calls > available_calls) {  // :178-187
      zero_plan(out, available_calls, hard_max_calls);
      return VTS_OK;
    }
  }

  out->segment_duration = segment_duration;  // :189-198
  out->overlap = overlap;
  out->num_segments = num_segments;
  out->estimated_calls = estimated_calls;
  out->available_calls = available_calls;
  out->hard_max_calls = hard_max_calls;
  out->fits_budget = estimated_calls <= available_calls ? 1 : 0;
  out->_pad = 0;
  return VTS_OK;
}

// ---------------------------------------------------------------------------
// Segment time -> frame index, exact rational comparison pts/timescale >= t.
// ---------------------------------------------------------------------------
namespace vts {

// Smallest integer q with q >= t * ts (exact), saturated to int64 bounds.
// Returns +1/-1 in *sat when the exact value is above/below the int64 range.
int64_t ceil_ticks(double t, int64_t ts, int *sat) {
  *sat = 0;
  if (t == 0.0) return 0;
  int exp = 0;
  double f = std::frexp(t, &exp);  // t = f * 2^exp, 0.5 <= |f| < 1
  // m = f * 2^53 is an exact integer; t = m * 2^(exp-53)
  const int64_t m = static_cast<int64_t>(std::ldexp(f, 53));
  int e = exp - 53;
  __int128 p = static_cast<__int128>(m) * ts;  // |p| < 2^53 * 2^63 = 2^116
  const __int128 lim = static_cast<__int128>(1) << 63;
  if (e >= 0) {
    if (e > 10) {  // |p| >= 2^52 (m normalised), ts >= 1: p << 11 >= 2^63
      *sat = p > 0 ? 1 : -1;
      return p > 0 ? INT64_MAX : INT64_MIN;
    }
    p <<= e;
    if (p >= lim) { *sat = 1; return INT64_MAX; }
    if (p < -lim) { *sat = -1; return INT64_MIN; }
    return static_cast<int64_t>(p);
  }
  const int sh = -e;
  if (sh >= 120) return p > 0 ? 1 : 0;  // |p| < 2^116: quotient in (-1, 1)
  // ceil(p / 2^sh) = -floor(-p / 2^sh); arithmetic shift is floor division.
  __int128 q = -((-p) >> sh);
  if (q >= lim) { *sat = 1; return INT64_MAX; }
  if (q < -lim) { *sat = -1; return INT64_MIN; }
  return static_cast<int64_t>(q);
}

}  // namespace vts

extern "C" int vts_boundary_frames_pts(const int64_t *pts, int64_t n_frames,
                                       int64_t timescale, const double *times,
                                       int64_t ntimes, int64_t *frame_idx) {
  clear_error();
  if ((n_frames > 0 && !pts) || (ntimes > 0 && (!times || !frame_idx)) ||
      n_frames < 0 || ntimes < 0)
    return fail(VTS_E_INVALID, "bad arguments");
  if (timescale <= 0) return fail(VTS_E_INVALID, "timescale must be > 0");
  for (int64_t i = 0; i < ntimes; ++i) {
    const double t = times[i];
    int64_t idx;
    if (std::isnan(t) || t == INFINITY) {
      idx = n_frames;
    } else if (t == -INFINITY) {
      idx = 0;
    } else {
      int sat = 0;
      const int64_t thr = vts::ceil_ticks(t, timescale, &sat);
      if (sat > 0) {
        idx = n_frames;
      } else if (sat < 0) {
        idx = 0;
      } else {
        int64_t lo = 0, hi = n_frames;  // lower_bound(pts, thr)
        while (lo < hi) {
          const int64_t mid = lo + (hi - lo) / 2;
          if (pts[mid] < thr) lo = mid + 1; else hi = mid;
        }
        idx = lo;
      }
    }
    frame_idx[i] = idx;
  }
  return VTS_OK;
}

extern "C" const char *vts_last_error(void) { return vts::last_error().c_str(); }
extern "C" int vts_abi_version(void) { return VTS_ABI_VERSION; }
