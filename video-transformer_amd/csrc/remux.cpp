// remux.cpp — native MP4 stream copy of a time range (the reference's
// `ffmpeg -ss S -i IN -t D -movflags +faststart -c copy OUT`,
// src/utils/video_segmenter.py:118-136), for ISO-BMFF inputs.
//
// Codec-agnostic: sample descriptions (stsd), handler boxes and sample bytes
// are copied verbatim; only the sample tables are rebuilt.  Per track:
//   first sample = last sync sample whose presentation time <= start
//                  (the keyframe at or before S, as a stream-copy seek does);
//   last sample  = last sample (decode order) whose presentation time < end;
//   output timestamps start at 0 with an edit list whose media_time makes
//   presentation start at S, and whose duration is the kept span inside
//   [S, end);
//   layout is ftyp, moov, mdat (+faststart: moov before the media data).
// Exact ffmpeg byte parity is unpinned (no ffmpeg in this image); the tests
// check that the cut decodes to exactly the source frames it claims.
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"
#include "mp4.h"

namespace vts {
namespace {

void put32(std::vector<uint8_t> &v, uint32_t x) {
  v.push_back(uint8_t(x >> 24));
  v.push_back(uint8_t(x >> 16));
  v.push_back(uint8_t(x >> 8));
  v.push_back(uint8_t(x));
}
void put16(std::vector<uint8_t> &v, uint32_t x) {
  v.push_back(uint8_t(x >> 8));
  v.push_back(uint8_t(x));
}
void put64(std::vector<uint8_t> &v, uint64_t x) {
  put32(v, uint32_t(x >> 32));
  put32(v, uint32_t(x));
}
void putfour(std::vector<uint8_t> &v, const char *s) { v.insert(v.end(), s, s + 4); }

struct BoxW {
  std::vector<uint8_t> &v;
  size_t start;
  BoxW(std::vector<uint8_t> &vec, const char *type) : v(vec), start(vec.size()) {
    put32(v, 0);
    putfour(v, type);
  }
  ~BoxW() {
    const uint32_t sz = static_cast<uint32_t>(v.size() - start);
    v[start] = uint8_t(sz >> 24);
    v[start + 1] = uint8_t(sz >> 16);
    v[start + 2] = uint8_t(sz >> 8);
    v[start + 3] = uint8_t(sz);
  }
};

void put_matrix(std::vector<uint8_t> &v) {
  const uint32_t m[9] = {0x00010000, 0, 0, 0, 0x00010000, 0, 0, 0, 0x40000000};
  for (uint32_t x : m) put32(v, x);
}

struct Cut {
  const Mp4VideoTrack *t = nullptr;
  int src = 0;                          // input file the samples come from
  int64_t first = 0, last = -1;         // decode-order sample range [first, last]
  std::vector<int64_t> delta;           // per kept sample
  int64_t media_time = 0;               // edit list, track timescale
  int64_t edit_duration_ms = 0;         // movie timescale (1000)
  int64_t track_duration = 0;           // sum of kept deltas
  std::vector<int64_t> out_offset;      // file offsets in the output
};

// floor(t * ts) exactly
int64_t floor_ticks(double t, int64_t ts, int *sat) {
  const int64_t c = ceil_ticks(-t, ts, sat);
  *sat = -*sat;
  return (c == INT64_MIN) ? INT64_MAX : -c;
}

std::string plan_cut(const Mp4VideoTrack &t, double start, double end, Cut *c) {
  const int64_t n = static_cast<int64_t>(t.size.size());
  if (n == 0 || t.timescale <= 0) return "empty track";
  int64_t shift = 0;
  for (const EditEntry &e : t.edits)
    if (e.media_time >= 0) {
      shift = e.media_time;
      break;
    }
  std::vector<int64_t> pts(static_cast<size_t>(n)), dur(static_cast<size_t>(n));
  for (int64_t i = 0; i < n; ++i) {
    pts[i] = t.dts[i] + t.cts_offset[i] - shift;
    dur[i] = (i + 1 < n) ? t.dts[i + 1] - t.dts[i] : std::max<int64_t>(t.duration - t.dts[i], 0);
  }
  if (n > 1 && dur[n - 1] == 0) dur[n - 1] = dur[n - 2];
  int sat = 0;
  const int64_t s_floor = floor_ticks(start, t.timescale, &sat);
  const int64_t s_ticks = sat > 0 ? INT64_MAX : (sat < 0 ? INT64_MIN : s_floor);
  const int64_t e_ceil = ceil_ticks(end, t.timescale, &sat);
  const int64_t e_ticks = sat > 0 ? INT64_MAX : (sat < 0 ? INT64_MIN : e_ceil);
  // first: last sync sample with pts <= start (else the first sync sample)
  int64_t first = -1;
  for (int64_t i = 0; i < n; ++i)
    if (t.sync[i] && pts[i] <= s_ticks) first = i;
  if (first < 0)
    for (int64_t i = 0; i < n; ++i)
      if (t.sync[i]) {
        first = i;
        break;
      }
  if (first < 0) return "no sync sample";
  int64_t last = -1;
  for (int64_t i = first; i < n; ++i)
    if (pts[i] < e_ticks) last = i;
  if (last < first) return "no samples in range";
  c->t = &t;
  c->first = first;
  c->last = last;
  c->delta.assign(dur.begin() + first, dur.begin() + last + 1);
  c->track_duration = 0;
  int64_t pres_end = INT64_MIN;
  for (int64_t i = first; i <= last; ++i) {
    c->track_duration += dur[i];
    pres_end = std::max(pres_end, pts[i] + dur[i]);
  }
  // output composition time of input presentation time p: p + shift - dts[first]
  const int64_t base = t.dts[first];
  const int64_t pres_start = std::max(s_ticks, pts[first]);  // S, or later if no earlier frame
  c->media_time = std::max<int64_t>(0, pres_start + shift - base);
  const int64_t span = std::min(pres_end, e_ticks) - pres_start;
  if (span <= 0) return "range starts after the last frame";
  c->edit_duration_ms = (span * 1000 + t.timescale / 2) / t.timescale;
  return "";
}

void write_trak(std::vector<uint8_t> &v, const Cut &c, uint32_t track_id) {
  const Mp4VideoTrack &t = *c.t;
  const int64_t ns = c.last - c.first + 1;
  BoxW trak(v, "trak");
  {
    BoxW tkhd(v, "tkhd");
    v.push_back(1);
    v.push_back(0); v.push_back(0); v.push_back(3);
    put64(v, 0); put64(v, 0);
    put32(v, track_id);
    put32(v, 0);
    put64(v, static_cast<uint64_t>(c.edit_duration_ms));
    put32(v, 0); put32(v, 0);
    put16(v, 0); put16(v, 0);
    put16(v, static_cast<uint16_t>(t.volume));
    put16(v, 0);
    put_matrix(v);
    put32(v, static_cast<uint32_t>(t.tkhd_width) << 16);
    put32(v, static_cast<uint32_t>(t.tkhd_height) << 16);
  }
  {
    BoxW edts(v, "edts");
    BoxW elst(v, "elst");
    v.push_back(1);
    v.push_back(0); v.push_back(0); v.push_back(0);
    put32(v, 1);
    put64(v, static_cast<uint64_t>(c.edit_duration_ms));
    put64(v, static_cast<uint64_t>(c.media_time));
    put16(v, 1); put16(v, 0);  // media_rate 1.0
  }
  BoxW mdia(v, "mdia");
  {
    BoxW mdhd(v, "mdhd");
    v.push_back(1);
    v.push_back(0); v.push_back(0); v.push_back(0);
    put64(v, 0); put64(v, 0);
    put32(v, static_cast<uint32_t>(t.timescale));
    put64(v, static_cast<uint64_t>(c.track_duration));
    put16(v, t.language);
    put16(v, 0);
  }
  v.insert(v.end(), t.hdlr.begin(), t.hdlr.end());
  BoxW minf(v, "minf");
  if (!t.media_header.empty()) {
    v.insert(v.end(), t.media_header.begin(), t.media_header.end());
  } else {
    BoxW nmhd(v, "nmhd");
    put32(v, 0);
  }
  {
    BoxW dinf(v, "dinf");
    BoxW dref(v, "dref");
    put32(v, 0);
    put32(v, 1);
    BoxW url(v, "url ");
    put32(v, 1);
  }
  BoxW stbl(v, "stbl");
  v.insert(v.end(), t.stsd.begin(), t.stsd.end());
  {
    BoxW stts(v, "stts");
    put32(v, 0);
    std::vector<std::pair<uint32_t, uint32_t>> runs;
    for (int64_t d : c.delta) {
      if (!runs.empty() && runs.back().second == static_cast<uint32_t>(d)) ++runs.back().first;
      else runs.emplace_back(1u, static_cast<uint32_t>(d));
    }
    put32(v, static_cast<uint32_t>(runs.size()));
    for (auto &r : runs) {
      put32(v, r.first);
      put32(v, r.second);
    }
  }
  if (t.has_ctts) {
    BoxW ctts(v, "ctts");
    bool neg = false;
    for (int64_t i = c.first; i <= c.last; ++i) neg |= t.cts_offset[i] < 0;
    v.push_back(neg ? 1 : 0);
    v.push_back(0); v.push_back(0); v.push_back(0);
    std::vector<std::pair<uint32_t, int32_t>> runs;
    for (int64_t i = c.first; i <= c.last; ++i) {
      if (!runs.empty() && runs.back().second == t.cts_offset[i]) ++runs.back().first;
      else runs.emplace_back(1u, t.cts_offset[i]);
    }
    put32(v, static_cast<uint32_t>(runs.size()));
    for (auto &r : runs) {
      put32(v, r.first);
      put32(v, static_cast<uint32_t>(r.second));
    }
  }
  if (t.has_stss) {
    BoxW stss(v, "stss");
    put32(v, 0);
    std::vector<uint32_t> idx;
    for (int64_t i = c.first; i <= c.last; ++i)
      if (t.sync[i]) idx.push_back(static_cast<uint32_t>(i - c.first + 1));
    put32(v, static_cast<uint32_t>(idx.size()));
    for (uint32_t x : idx) put32(v, x);
  }
  {
    BoxW stsc(v, "stsc");
    put32(v, 0);
    put32(v, 1);
    put32(v, 1); put32(v, 1); put32(v, 1);
  }
  {
    BoxW stsz(v, "stsz");
    put32(v, 0);
    put32(v, 0);
    put32(v, static_cast<uint32_t>(ns));
    for (int64_t i = c.first; i <= c.last; ++i) put32(v, t.size[i]);
  }
  {
    BoxW co64(v, "co64");
    put32(v, 0);
    put32(v, static_cast<uint32_t>(ns));
    for (int64_t o : c.out_offset) put64(v, static_cast<uint64_t>(o));
  }
}

std::vector<uint8_t> build_moov(std::vector<Cut> &cuts) {
  std::vector<uint8_t> v;
  BoxW moov(v, "moov");
  int64_t dur = 0;
  for (const Cut &c : cuts) dur = std::max(dur, c.edit_duration_ms);
  {
    BoxW mvhd(v, "mvhd");
    v.push_back(1);
    v.push_back(0); v.push_back(0); v.push_back(0);
    put64(v, 0); put64(v, 0);
    put32(v, 1000);
    put64(v, static_cast<uint64_t>(dur));
    put32(v, 0x00010000);
    put16(v, 0x0100);
    put16(v, 0); put32(v, 0); put32(v, 0);
    put_matrix(v);
    for (int i = 0; i < 6; ++i) put32(v, 0);
    put32(v, static_cast<uint32_t>(cuts.size() + 1));
  }
  uint32_t id = 1;
  for (Cut &c : cuts) write_trak(v, c, id++);
  return v;
}

}  // namespace

namespace {

// ftyp, moov, mdat of `cuts` (samples read from srcs[cut.src]) into out_path.
std::string write_cuts(std::vector<Cut> &cuts, const char *const *srcs, int n_src,
                       const char *out_path) {
  std::vector<uint8_t> ftyp;
  {
    BoxW b(ftyp, "ftyp");
    putfour(ftyp, "isom");
    put32(ftyp, 0x200);
    putfour(ftyp, "isom");
    putfour(ftyp, "iso2");
    putfour(ftyp, "mp41");
  }
  // offsets are relative until the moov size is known; co64 keeps it fixed
  int64_t rel = 0;
  for (Cut &c : cuts) {
    c.out_offset.clear();
    for (int64_t i = c.first; i <= c.last; ++i) {
      c.out_offset.push_back(rel);
      rel += c.t->size[i];
    }
  }
  const size_t moov_size = build_moov(cuts).size();
  const int64_t data_start = static_cast<int64_t>(ftyp.size() + moov_size) + 16;
  for (Cut &c : cuts)
    for (int64_t &o : c.out_offset) o += data_start;
  const std::vector<uint8_t> moov = build_moov(cuts);
  if (moov.size() != moov_size) return "internal: moov size changed";

  std::vector<int> in(static_cast<size_t>(n_src), -1);
  for (int k = 0; k < n_src; ++k) {
    in[k] = ::open(srcs[k], O_RDONLY | O_CLOEXEC);
    if (in[k] < 0) {
      for (int j = 0; j < k; ++j) ::close(in[j]);
      return std::string("cannot open ") + srcs[k];
    }
  }
  FILE *out = std::fopen(out_path, "wb");
  if (!out) {
    for (int fd : in) ::close(fd);
    return std::string("cannot create ") + out_path;
  }
  bool ok = std::fwrite(ftyp.data(), 1, ftyp.size(), out) == ftyp.size() &&
            std::fwrite(moov.data(), 1, moov.size(), out) == moov.size();
  std::vector<uint8_t> hdr;
  put32(hdr, 1);
  putfour(hdr, "mdat");
  put64(hdr, static_cast<uint64_t>(rel + 16));
  ok = ok && std::fwrite(hdr.data(), 1, hdr.size(), out) == hdr.size();
  std::vector<uint8_t> buf;
  for (const Cut &c : cuts)
    for (int64_t i = c.first; ok && i <= c.last; ++i) {
      const size_t n = c.t->size[i];
      buf.resize(n);
      size_t got = 0;
      while (got < n) {
        const ssize_t r = ::pread(in[c.src], buf.data() + got, n - got,
                                  c.t->offset[i] + static_cast<int64_t>(got));
        if (r <= 0) break;
        got += static_cast<size_t>(r);
      }
      ok = (got == n) && std::fwrite(buf.data(), 1, n, out) == n;
    }
  for (int fd : in) ::close(fd);
  if (std::fclose(out) != 0) ok = false;
  if (!ok) {
    std::remove(out_path);
    return "I/O error while copying samples";
  }
  return "";
}

}  // namespace

std::string mp4_add_tracks(const char *video_path, const char *src_path, const char *out_path) {
  Mp4Info a, b;
  std::string e = mp4_parse_file(video_path, &a);
  if (!e.empty()) return e;
  e = mp4_parse_file(src_path, &b);
  if (!e.empty()) return e;
  const double inf = 1e300;  // finite: ceil_ticks saturates it (frexp of inf is not a number)
  std::vector<Cut> cuts;
  for (const Mp4VideoTrack &t : a.tracks) {
    Cut c;
    e = plan_cut(t, 0.0, inf, &c);
    if (!e.empty()) return e;
    cuts.push_back(std::move(c));
  }
  for (const Mp4VideoTrack &t : b.tracks) {
    if (t.handler == 0x76696465u) continue;  // 'vide': the new video replaces it
    Cut c;
    if (!plan_cut(t, 0.0, inf, &c).empty()) continue;  // an empty track is dropped
    c.src = 1;
    cuts.push_back(std::move(c));
  }
  const char *srcs[2] = {video_path, src_path};
  return write_cuts(cuts, srcs, 2, out_path);
}

std::string mp4_remux_segment(const char *in_path, double start, double end,
                              const char *out_path) {
  if (!(end - start > 0)) return "empty time range";
  Mp4Info mp4;
  std::string e = mp4_parse_file(in_path, &mp4);
  if (!e.empty()) return e;
  if (mp4.video.empty()) return "no video track";
  std::vector<Cut> cuts;
  for (const Mp4VideoTrack &t : mp4.tracks) {
    Cut c;
    e = plan_cut(t, start, end, &c);
    if (!e.empty()) {
      if (t.track_id == mp4.video.front().track_id) return e;  // the video track must cut
      continue;  // a secondary track with nothing in range is dropped
    }
    cuts.push_back(std::move(c));
  }
  if (cuts.empty()) return "nothing to copy";
  const char *srcs[1] = {in_path};
  return write_cuts(cuts, srcs, 1, out_path);
}

}  // namespace vts

extern "C" int vts_extract_segment(const char *in_path, double start, double end,
                                   const char *out_path) {
  vts::clear_error();
  if (!in_path || !out_path) return vts::fail(VTS_E_INVALID, "NULL path");
  const std::string e = vts::mp4_remux_segment(in_path, start, end, out_path);
  if (!e.empty()) return vts::fail(VTS_E_FORMAT, "%s", e.c_str());
  return VTS_OK;
}

extern "C" int vts_add_tracks(const char *video_path, const char *src_path, const char *out_path) {
  vts::clear_error();
  if (!video_path || !src_path || !out_path) return vts::fail(VTS_E_INVALID, "NULL path");
  const std::string e = vts::mp4_add_tracks(video_path, src_path, out_path);
  if (!e.empty()) return vts::fail(VTS_E_FORMAT, "%s", e.c_str());
  return VTS_OK;
}
