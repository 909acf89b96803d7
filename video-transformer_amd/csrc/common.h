// common.h — shared host-side helpers of libvtseg (error string, status).
#pragma once
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "vtseg.h"

namespace vts {

// Thread-local message of the calling thread's last failure (vts_last_error).
std::string &last_error();

// Record `code` with a printf-style message and return it.
inline int fail(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  last_error() = buf;
  return code;
}

inline void clear_error() { last_error().clear(); }

// Smallest integer q with q >= t * ts, computed exactly from the double's
// binary value; *sat = +1 / -1 when that integer is above / below int64.
int64_t ceil_ticks(double t, int64_t ts, int *sat);

}  // namespace vts

#define VTS_TRY(expr)                 \
  do {                                \
    int _vts_rc = (expr);             \
    if (_vts_rc != VTS_OK) return _vts_rc; \
  } while (0)
