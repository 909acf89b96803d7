// manifest.cpp — the segment manifest as JSON text, byte-identical to the
// reference's create_manifest + save_manifest
// (src/utils/video_segmenter.py:170-218: json.dumps(manifest, indent=2,
// ensure_ascii=True)), so a batch driver can plan and persist without Python
// and either implementation can resume the other's manifest.
//
// Python semantics restated here:
//   * float repr (json's float.__repr__): the shortest digits that round-trip
//     (std::to_chars), fixed notation for 1e-4 <= |x| < 1e16 with a ".0" on
//     integral values, else d[.ddd]e±XX; NaN / Infinity / -Infinity;
//   * ints (the caller's own int objects: SegmentPlan fields, an int duration
//     that min() hands back) are passed as their decimal repr and copied;
//   * ensure_ascii string escaping: \" \\ \n \r \t \b \f, other controls and
//     all non-ASCII as \uXXXX (UTF-16 surrogate pairs above U+FFFF);
//   * file_path = str(segment_dir / f"segment_{id:04d}.mp4").
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"
#include "vtseg.h"

namespace vts {
namespace {

void py_float_repr(double x, std::string &o) {
  if (std::isnan(x)) {
    o += "NaN";
    return;
  }
  if (std::isinf(x)) {
    o += x < 0 ? "-Infinity" : "Infinity";
    return;
  }
  if (std::signbit(x)) {
    o += '-';
    x = -x;
  }
  if (x == 0.0) {
    o += "0.0";
    return;
  }
  char buf[64];
  const auto r = std::to_chars(buf, buf + sizeof buf, x, std::chars_format::scientific);
  const std::string sci(buf, r.ptr);
  const size_t e = sci.find('e');
  std::string digits;
  for (size_t i = 0; i < e; ++i)
    if (sci[i] != '.') digits += sci[i];
  const int exp10 = std::atoi(sci.c_str() + e + 1);
  const int decpt = exp10 + 1;  // value = 0.DIGITS x 10^decpt
  const int nd = static_cast<int>(digits.size());
  if (decpt <= -4 || decpt > 16) {  // Python's 'r' rule (pystrtod.c format_float_short)
    o += digits[0];
    if (nd > 1) {
      o += '.';
      o.append(digits, 1, std::string::npos);
    }
    char eb[16];
    std::snprintf(eb, sizeof eb, "e%+.02d", decpt - 1);
    o += eb;
  } else if (decpt <= 0) {
    o += "0.";
    o.append(static_cast<size_t>(-decpt), '0');
    o += digits;
  } else if (decpt >= nd) {
    o += digits;
    o.append(static_cast<size_t>(decpt - nd), '0');
    o += ".0";
  } else {
    o.append(digits, 0, static_cast<size_t>(decpt));
    o += '.';
    o.append(digits, static_cast<size_t>(decpt), std::string::npos);
  }
}

void u_escape(uint32_t cp, std::string &o) {
  char b[8];
  std::snprintf(b, sizeof b, "\\u%04x", cp);
  o += b;
}

// JSON string with ensure_ascii; false on invalid UTF-8
bool json_string(const char *s, std::string &o) {
  o += '"';
  const auto *p = reinterpret_cast<const unsigned char *>(s);
  while (*p) {
    uint32_t c = *p;
    int extra = 0;
    if (c < 0x80) {
      switch (c) {
        case '"': o += "\\\""; break;
        case '\\': o += "\\\\"; break;
        case '\n': o += "\\n"; break;
        case '\r': o += "\\r"; break;
        case '\t': o += "\\t"; break;
        case '\b': o += "\\b"; break;
        case '\f': o += "\\f"; break;
        default:
          if (c < 0x20 || c == 0x7f) u_escape(c, o);  // outside ' '..'~'
          else o += static_cast<char>(c);
      }
      ++p;
      continue;
    }
    if ((c & 0xe0) == 0xc0) { c &= 0x1f; extra = 1; }
    else if ((c & 0xf0) == 0xe0) { c &= 0x0f; extra = 2; }
    else if ((c & 0xf8) == 0xf0) { c &= 0x07; extra = 3; }
    else return false;
    ++p;
    for (int i = 0; i < extra; ++i, ++p) {
      if ((*p & 0xc0) != 0x80) return false;
      c = (c << 6) | (*p & 0x3f);
    }
    if ((extra == 1 && c < 0x80) || (extra == 2 && c < 0x800) || (extra == 3 && c < 0x10000) ||
        c > 0x10ffff || (c >= 0xd800 && c <= 0xdfff))
      return false;
    if (c >= 0x10000) {
      c -= 0x10000;
      u_escape(0xd800 + (c >> 10), o);
      u_escape(0xdc00 + (c & 0x3ff), o);
    } else {
      u_escape(c, o);
    }
  }
  o += '"';
  return true;
}

void number(double x, const char *int_repr, std::string &o) {
  if (int_repr) o += int_repr; else py_float_repr(x, o);
}

}  // namespace
}  // namespace vts

using namespace vts;

extern "C" int vts_manifest_json(const vts_manifest_args *a, char *out, int64_t cap, int64_t *len) {
  clear_error();
  if (!a || !len || !a->video_id || !a->segment_dir || !a->created_at)
    return fail(VTS_E_INVALID, "NULL argument");
  // plan_segments(duration, segment_seconds, overlap_seconds)
  int64_t n = 0;
  int rc = vts_plan_segments(a->duration, a->segment_seconds, a->overlap_seconds, nullptr, 0, &n);
  if (rc != VTS_OK && rc != VTS_E_CAPACITY) return rc;
  std::vector<vts_segment> segs(static_cast<size_t>(n));
  if (n > 0) {
    rc = vts_plan_segments(a->duration, a->segment_seconds, a->overlap_seconds, segs.data(), n, &n);
    if (rc != VTS_OK) return rc;
  }
  clear_error();
  std::string o;
  o.reserve(256 + 400 * static_cast<size_t>(n));
  o += "{\n  \"version\": 1,\n  \"video_id\": ";
  if (!json_string(a->video_id, o)) return fail(VTS_E_INVALID, "video_id is not valid UTF-8");
  o += ",\n  \"created_at\": ";
  if (!json_string(a->created_at, o)) return fail(VTS_E_INVALID, "created_at is not valid UTF-8");
  o += ",\n  \"segment_seconds\": ";
  number(a->segment_seconds, a->segment_seconds_int, o);
  o += ",\n  \"overlap_seconds\": ";
  number(a->overlap_seconds, a->overlap_seconds_int, o);
  o += ",\n  \"segments\": [";
  std::string dir = a->segment_dir;
  for (int64_t i = 0; i < n; ++i) {
    const vts_segment &g = segs[static_cast<size_t>(i)];
    o += i ? ",\n    {\n      \"id\": " : "\n    {\n      \"id\": ";
    o += std::to_string(g.segment_id);
    o += ",\n      \"start\": ";
    py_float_repr(g.start, o);
    o += ",\n      \"end\": ";
    number(g.end, (g.flags & 1) ? a->duration_int : nullptr, o);
    o += ",\n      \"effective_start\": ";
    py_float_repr(g.effective_start, o);
    o += ",\n      \"effective_end\": ";
    number(g.effective_end, (g.flags & 2) ? a->duration_int : nullptr, o);
    o += ",\n      \"file_path\": ";
    char name[48];
    std::snprintf(name, sizeof name, "segment_%04lld.mp4", static_cast<long long>(g.segment_id));
    std::string path = dir;
    if (path.empty()) path = ".";  // str(Path("") / name) == name
    if (path == ".") path = name; else path += (path.back() == '/' ? "" : "/") + std::string(name);
    if (!json_string(path.c_str(), o)) return fail(VTS_E_INVALID, "segment_dir is not valid UTF-8");
    o += ",\n      \"status\": \"pending\",\n      \"attempts\": 0,\n      \"error\": null\n    }";
  }
  o += n ? "\n  ]\n}" : "]\n}";
  *len = static_cast<int64_t>(o.size());
  if (!out || cap < *len) return fail(VTS_E_CAPACITY, "need %lld bytes", static_cast<long long>(*len));
  std::memcpy(out, o.data(), o.size());
  return VTS_OK;
}
