// Sanitizer harness of the host code that reads untrusted files — the MP4
// reader (mp4.cpp), the probe (probe.cpp), the slice-header scheduler
// (h264_sched.cpp, h264.cpp), the stream-copy cutter (remux.cpp) — and, through
// full_host.cpp's fh_decode, of the very parser / derivation /
// reconstruction code the device runs (parse_full.h, parse_cabac.h,
// derive_full.h, recon_full.h).  TEST INFRASTRUCTURE: tests/test_fuzz_host.py
// builds it with -fsanitize=address,undefined and feeds it truncated and
// bit-flipped files in a child process; every call must come back with a
// status (never crash, never trip a sanitizer).
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "h264.h"
#include "h264_sched.h"
#include "mp4.h"
#include "vtseg.h"

using namespace vts;

// the open path's host half: container, parameter sets, stream facts, every
// slice header and the reference bookkeeping (what vts_open does before it
// touches the device); 0 or -1 with the reason in err
extern "C" int fz_schedule(const char *path, char *err, int err_cap) {
  auto bad = [&](const std::string &m) {
    std::snprintf(err, static_cast<size_t>(err_cap), "%s", m.c_str());
    return -1;
  };
  Mp4Info mp4;
  std::string e = mp4_parse_file(path, &mp4);
  if (!e.empty()) return bad(e);
  if (mp4.video.empty()) return bad("no video track");
  const Mp4VideoTrack &t = mp4.video.front();
  if (t.sps.empty() || t.pps.empty()) return bad("no parameter sets");
  Sps sps;
  Pps pps;
  e = parse_sps(t.sps[0].data(), t.sps[0].size(), &sps);
  if (e.empty()) e = parse_pps(t.pps[0].data(), t.pps[0].size(), &pps);
  if (!e.empty()) return bad(e);
  SchedStream facts;
  e = sched_stream_facts(t.sps[0], t.pps[0], sps, pps, &facts);
  if (!e.empty()) return bad(e);
  std::vector<uint8_t> es;
  std::vector<int64_t> off;
  FILE *f = std::fopen(path, "rb");
  if (!f) return bad("open");
  for (size_t i = 0; i < t.size.size(); ++i) {
    off.push_back(static_cast<int64_t>(es.size()));
    const size_t n0 = es.size();
    if (t.size[i] > (64u << 20)) {
      std::fclose(f);
      return bad("sample too large");
    }
    es.resize(n0 + t.size[i]);
    if (fseeko(f, t.offset[i], SEEK_SET) != 0 || std::fread(es.data() + n0, 1, t.size[i], f) != t.size[i]) {
      std::fclose(f);
      return bad("read");
    }
  }
  std::fclose(f);
  es.resize(es.size() + 64, 0);
  std::vector<SchedFrame> frames;
  std::vector<SchedSlice> slices;
  e = sched_build(sps, pps, es.data(), off, t.size, t.nal_length_size, &frames, &slices);
  if (!e.empty()) return bad(e);
  return 0;
}
