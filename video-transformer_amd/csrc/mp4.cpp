// mp4.cpp — ISO/IEC 14496-12 box parsing (moov only) and a streaming writer.
#include "mp4.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <memory>

namespace vts {

namespace {

struct Source {
  virtual ~Source() = default;
  virtual bool read(int64_t off, void *dst, size_t n) const = 0;
  virtual int64_t size() const = 0;
};

struct FileSource final : Source {
  int fd = -1;
  int64_t sz = 0;
  ~FileSource() override {
    if (fd >= 0) ::close(fd);
  }
  bool read(int64_t off, void *dst, size_t n) const override {
    if (off < 0 || off + static_cast<int64_t>(n) > sz) return false;
    uint8_t *p = static_cast<uint8_t *>(dst);
    while (n > 0) {
      const ssize_t r = ::pread(fd, p, n, off);
      if (r <= 0) return false;
      p += r;
      off += r;
      n -= static_cast<size_t>(r);
    }
    return true;
  }
  int64_t size() const override { return sz; }
};

struct MemSource final : Source {
  const uint8_t *p = nullptr;
  int64_t sz = 0;
  bool read(int64_t off, void *dst, size_t n) const override {
    if (off < 0 || off + static_cast<int64_t>(n) > sz) return false;
    std::memcpy(dst, p + off, n);
    return true;
  }
  int64_t size() const override { return sz; }
};

inline uint32_t rd32(const uint8_t *p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3];
}
inline uint64_t rd64(const uint8_t *p) { return (uint64_t(rd32(p)) << 32) | rd32(p + 4); }
inline uint16_t rd16(const uint8_t *p) { return uint16_t((p[0] << 8) | p[1]); }

inline uint32_t fourcc(const char *s) {
  return (uint32_t(uint8_t(s[0])) << 24) | (uint32_t(uint8_t(s[1])) << 16) |
         (uint32_t(uint8_t(s[2])) << 8) | uint32_t(uint8_t(s[3]));
}

// A view over a box payload held in memory (moov is read whole).
struct Box {
  uint32_t type = 0;
  const uint8_t *p = nullptr;  // payload
  size_t n = 0;
};

// Iterate child boxes of a payload.
bool next_box(const uint8_t *&cur, const uint8_t *end, Box *b) {
  if (end - cur < 8) return false;
  uint64_t size = rd32(cur);
  b->type = rd32(cur + 4);
  size_t hdr = 8;
  if (size == 1) {
    if (end - cur < 16) return false;
    size = rd64(cur + 8);
    hdr = 16;
  } else if (size == 0) {
    size = static_cast<uint64_t>(end - cur);
  }
  if (size < hdr || size > static_cast<uint64_t>(end - cur)) return false;
  b->p = cur + hdr;
  b->n = static_cast<size_t>(size - hdr);
  cur += size;
  return true;
}

bool find_child(const Box &parent, uint32_t type, Box *out, size_t skip = 0) {
  const uint8_t *cur = parent.p + skip, *end = parent.p + parent.n;
  Box b;
  while (next_box(cur, end, &b))
    if (b.type == type) {
      *out = b;
      return true;
    }
  return false;
}

std::string parse_avcc(const uint8_t *p, size_t n, Mp4VideoTrack *t) {
  if (n < 7 || p[0] != 1) return "bad avcC";
  t->nal_length_size = (p[4] & 3) + 1;
  size_t pos = 5;
  const int nsps = p[pos++] & 0x1f;
  for (int i = 0; i < nsps; ++i) {
    if (pos + 2 > n) return "bad avcC sps";
    const size_t len = rd16(p + pos);
    pos += 2;
    if (pos + len > n) return "bad avcC sps";
    t->sps.emplace_back(p + pos, p + pos + len);
    pos += len;
  }
  if (pos + 1 > n) return "bad avcC";
  const int npps = p[pos++];
  for (int i = 0; i < npps; ++i) {
    if (pos + 2 > n) return "bad avcC pps";
    const size_t len = rd16(p + pos);
    pos += 2;
    if (pos + len > n) return "bad avcC pps";
    t->pps.emplace_back(p + pos, p + pos + len);
    pos += len;
  }
  return "";
}

std::string parse_stbl(const Box &stbl, Mp4VideoTrack *t) {
  Box b;
  // stsd -> first sample entry
  if (!find_child(stbl, fourcc("stsd"), &b) || b.n < 16) return "missing stsd";
  t->stsd.assign(b.p - 8, b.p + b.n);  // 32-bit size header (box < 4 GiB)
  {
    const uint8_t *cur = b.p + 8, *end = b.p + b.n;
    Box entry;
    if (!next_box(cur, end, &entry)) return "bad stsd";
    t->codec.assign(reinterpret_cast<const char *>(b.p + 8 + 4), 4);
    // VisualSampleEntry: 6 reserved + 2 dref + 16 + 2 w + 2 h + 50 = 78 bytes
    if (entry.type == fourcc("avc1") || entry.type == fourcc("avc3")) {
      if (entry.n < 78) return "bad avc1";
      Box avcc;
      if (!find_child(entry, fourcc("avcC"), &avcc, 78)) return "missing avcC";
      const std::string e = parse_avcc(avcc.p, avcc.n, t);
      if (!e.empty()) return e;
    }
  }
  // stsz
  if (!find_child(stbl, fourcc("stsz"), &b) || b.n < 12) return "missing stsz";
  const uint32_t uni = rd32(b.p + 4), count = rd32(b.p + 8);
  if (uni == 0 && b.n < 12 + size_t(count) * 4) return "truncated stsz";
  t->size.resize(count);
  for (uint32_t i = 0; i < count; ++i) t->size[i] = uni ? uni : rd32(b.p + 12 + 4 * size_t(i));
  // chunk offsets
  std::vector<int64_t> chunks;
  if (find_child(stbl, fourcc("stco"), &b) && b.n >= 8) {
    const uint32_t nc = rd32(b.p + 4);
    if (b.n < 8 + size_t(nc) * 4) return "truncated stco";
    chunks.resize(nc);
    for (uint32_t i = 0; i < nc; ++i) chunks[i] = rd32(b.p + 8 + 4 * size_t(i));
  } else if (find_child(stbl, fourcc("co64"), &b) && b.n >= 8) {
    const uint32_t nc = rd32(b.p + 4);
    if (b.n < 8 + size_t(nc) * 8) return "truncated co64";
    chunks.resize(nc);
    for (uint32_t i = 0; i < nc; ++i) chunks[i] = static_cast<int64_t>(rd64(b.p + 8 + 8 * size_t(i)));
  } else {
    return "missing stco/co64";
  }
  // stsc -> sample offsets
  if (!find_child(stbl, fourcc("stsc"), &b) || b.n < 8) return "missing stsc";
  {
    const uint32_t ne = rd32(b.p + 4);
    if (b.n < 8 + size_t(ne) * 12) return "truncated stsc";
    t->offset.resize(count);
    uint32_t s = 0;
    for (uint32_t e = 0; e < ne && s < count; ++e) {
      const uint32_t first = rd32(b.p + 8 + 12 * size_t(e));
      const uint32_t spc = rd32(b.p + 8 + 12 * size_t(e) + 4);
      const uint32_t last = (e + 1 < ne) ? rd32(b.p + 8 + 12 * size_t(e + 1)) : uint32_t(chunks.size() + 1);
      if (first == 0 || last < first) return "bad stsc";
      for (uint32_t c = first; c < last && s < count; ++c) {
        if (c - 1 >= chunks.size()) return "stsc references missing chunk";
        int64_t off = chunks[c - 1];
        for (uint32_t k = 0; k < spc && s < count; ++k) {
          t->offset[s] = off;
          off += t->size[s];
          ++s;
        }
      }
    }
    if (s != count) return "stsc does not cover all samples";
  }
  // stts -> dts
  if (!find_child(stbl, fourcc("stts"), &b) || b.n < 8) return "missing stts";
  {
    const uint32_t ne = rd32(b.p + 4);
    if (b.n < 8 + size_t(ne) * 8) return "truncated stts";
    t->dts.resize(count);
    uint32_t s = 0;
    int64_t d = 0;
    for (uint32_t e = 0; e < ne && s < count; ++e) {
      const uint32_t cnt = rd32(b.p + 8 + 8 * size_t(e));
      const uint32_t delta = rd32(b.p + 8 + 8 * size_t(e) + 4);
      for (uint32_t k = 0; k < cnt && s < count; ++k) {
        t->dts[s++] = d;
        d += delta;
      }
    }
    for (; s < count; ++s) t->dts[s] = d;
  }
  // ctts
  t->cts_offset.assign(count, 0);
  if (find_child(stbl, fourcc("ctts"), &b) && b.n >= 8) {
    t->has_ctts = true;
    const uint32_t ne = rd32(b.p + 4);
    if (b.n < 8 + size_t(ne) * 8) return "truncated ctts";
    uint32_t s = 0;
    for (uint32_t e = 0; e < ne && s < count; ++e) {
      const uint32_t cnt = rd32(b.p + 8 + 8 * size_t(e));
      const int32_t off = static_cast<int32_t>(rd32(b.p + 8 + 8 * size_t(e) + 4));
      for (uint32_t k = 0; k < cnt && s < count; ++k) t->cts_offset[s++] = off;
    }
  }
  // stss
  if (find_child(stbl, fourcc("stss"), &b) && b.n >= 8) {
    t->has_stss = true;
    t->sync.assign(count, 0);
    const uint32_t ne = rd32(b.p + 4);
    if (b.n < 8 + size_t(ne) * 4) return "truncated stss";
    for (uint32_t e = 0; e < ne; ++e) {
      const uint32_t idx = rd32(b.p + 8 + 4 * size_t(e));
      if (idx >= 1 && idx <= count) t->sync[idx - 1] = 1;
    }
  } else {
    t->sync.assign(count, 1);
  }
  return "";
}

std::string parse_trak(const Box &trak, Mp4Info *info) {
  Box mdia, hdlr, mdhd, minf, stbl, tkhd;
  if (!find_child(trak, fourcc("mdia"), &mdia)) return "";
  if (!find_child(mdia, fourcc("hdlr"), &hdlr) || hdlr.n < 12) return "";
  Mp4VideoTrack t;
  t.handler = rd32(hdlr.p + 8);
  t.hdlr.assign(hdlr.p - 8, hdlr.p + hdlr.n);
  if (find_child(trak, fourcc("tkhd"), &tkhd) && tkhd.n >= 84) {
    const int v = tkhd.p[0];
    // version/flags, times, track_ID, reserved, duration
    const size_t base = (v == 1) ? 36 : 24;
    t.track_id = rd32(tkhd.p + (v == 1 ? 20 : 12));
    t.volume = static_cast<int16_t>(rd16(tkhd.p + base + 8 + 2 + 2));
    // reserved[2], layer, alternate_group, volume, reserved, matrix[9]
    const size_t wpos = base + 8 + 2 + 2 + 2 + 2 + 36;
    if (tkhd.n >= wpos + 8) {
      t.tkhd_width = static_cast<int>(rd32(tkhd.p + wpos) >> 16);
      t.tkhd_height = static_cast<int>(rd32(tkhd.p + wpos + 4) >> 16);
    }
  }
  if (!find_child(mdia, fourcc("mdhd"), &mdhd) || mdhd.n < 24) return "bad mdhd";
  if (mdhd.p[0] == 1) {
    if (mdhd.n < 36) return "bad mdhd";
    t.timescale = rd32(mdhd.p + 20);
    t.duration = static_cast<int64_t>(rd64(mdhd.p + 24));
  } else {
    t.timescale = rd32(mdhd.p + 12);
    t.duration = rd32(mdhd.p + 16);
  }
  t.language = rd16(mdhd.p + (mdhd.p[0] == 1 ? 32 : 20));
  Box edts, elst;
  if (find_child(trak, fourcc("edts"), &edts) && find_child(edts, fourcc("elst"), &elst) &&
      elst.n >= 8) {
    const int v = elst.p[0];
    const uint32_t ne = rd32(elst.p + 4);
    const size_t esz = (v == 1) ? 20 : 12;
    if (elst.n < 8 + ne * esz) return "truncated elst";
    for (uint32_t i = 0; i < ne; ++i) {
      const uint8_t *e = elst.p + 8 + i * esz;
      EditEntry ed;
      if (v == 1) {
        ed.segment_duration = static_cast<int64_t>(rd64(e));
        ed.media_time = static_cast<int64_t>(rd64(e + 8));
      } else {
        ed.segment_duration = rd32(e);
        ed.media_time = static_cast<int32_t>(rd32(e + 4));
      }
      t.edits.push_back(ed);
    }
  }
  if (!find_child(mdia, fourcc("minf"), &minf) || !find_child(minf, fourcc("stbl"), &stbl))
    return "missing stbl";
  for (const char *mh : {"vmhd", "smhd", "nmhd", "sthd", "hmhd"}) {
    Box h;
    if (find_child(minf, fourcc(mh), &h)) {
      t.media_header.assign(h.p - 8, h.p + h.n);
      break;
    }
  }
  const std::string e = parse_stbl(stbl, &t);
  if (!e.empty()) return e;
  info->tracks.push_back(t);
  if (t.handler == fourcc("vide")) info->video.push_back(std::move(t));
  return "";
}

// ISO/IEC 14496-12 §8.8: the samples of the movie fragments appended to the
// tracks' tables.  trex gives each track's defaults, tfhd a fragment's
// (track, base data offset, defaults), tfdt its first decode time, trun its
// samples (duration, size, flags, composition offset, each present or
// defaulted; data_offset from the base, else on from the previous run).
// Sync = sample_is_non_sync_sample (flags bit 16) clear.
struct Moof {
  int64_t start;                 // file offset of the moof box
  std::vector<uint8_t> payload;
};
struct Trex {
  uint32_t duration = 0, size = 0, flags = 0;
};

std::string apply_fragments(const Box &moov, const std::vector<Moof> &moofs, Mp4Info *info) {
  std::vector<std::pair<uint32_t, Trex>> trex;
  Box mvex;
  if (find_child(moov, fourcc("mvex"), &mvex)) {
    const uint8_t *cur = mvex.p, *end = mvex.p + mvex.n;
    Box b;
    while (next_box(cur, end, &b)) {
      if (b.type == fourcc("trex") && b.n >= 24) {
        Trex t;
        t.duration = rd32(b.p + 12);
        t.size = rd32(b.p + 16);
        t.flags = rd32(b.p + 20);
        trex.emplace_back(rd32(b.p + 4), t);
      } else if (b.type == fourcc("mehd") && b.n >= 8) {
        info->fragment_duration = b.p[0] == 1 ? (b.n >= 12 ? static_cast<int64_t>(rd64(b.p + 4)) : 0) : rd32(b.p + 4);
      }
    }
  }
  auto track_of = [&](uint32_t id) -> Mp4VideoTrack * {
    for (Mp4VideoTrack &t : info->tracks)
      if (t.track_id == id) return &t;
    return nullptr;
  };
  std::vector<int64_t> next_dts(info->tracks.size(), -1);  // decode time after each track's last sample
  for (size_t k = 0; k < info->tracks.size(); ++k) {
    const Mp4VideoTrack &t = info->tracks[k];
    if (!t.dts.empty()) next_dts[k] = t.dts.back();  // (the moov's last sample's duration is unknown here)
  }
  for (const Moof &mf : moofs) {
    Box root{fourcc("moof"), mf.payload.data(), mf.payload.size()};
    const uint8_t *cur = root.p, *end = root.p + root.n;
    Box traf;
    int64_t prev_end = mf.start;  // base of a traf without an explicit / moof base: the previous traf's data end
    bool first_traf = true;
    while (next_box(cur, end, &traf)) {
      if (traf.type != fourcc("traf")) continue;
      Box tfhd;
      if (!find_child(traf, fourcc("tfhd"), &tfhd) || tfhd.n < 8) return "traf without tfhd";
      const uint32_t tf = rd32(tfhd.p) & 0xffffff, id = rd32(tfhd.p + 4);
      Mp4VideoTrack *t = track_of(id);
      if (!t) return "movie fragment of an unknown track";
      const size_t ti = static_cast<size_t>(t - info->tracks.data());
      Trex d;
      for (const auto &x : trex)
        if (x.first == id) d = x.second;
      size_t q = 8;
      int64_t base;
      auto need = [&](size_t n) { return q + n <= tfhd.n; };
      if (tf & 0x1) {
        if (!need(8)) return "truncated tfhd";
        base = static_cast<int64_t>(rd64(tfhd.p + q));
        q += 8;
      } else {
        base = (tf & 0x20000) || first_traf ? mf.start : prev_end;
      }
      if (tf & 0x2) q += 4;  // sample_description_index
      if (tf & 0x8) {
        if (!need(4)) return "truncated tfhd";
        d.duration = rd32(tfhd.p + q);
        q += 4;
      }
      if (tf & 0x10) {
        if (!need(4)) return "truncated tfhd";
        d.size = rd32(tfhd.p + q);
        q += 4;
      }
      if (tf & 0x20) {
        if (!need(4)) return "truncated tfhd";
        d.flags = rd32(tfhd.p + q);
        q += 4;
      }
      Box tfdt;
      int64_t dts = next_dts[ti] < 0 ? 0 : next_dts[ti];
      if (find_child(traf, fourcc("tfdt"), &tfdt) && tfdt.n >= 8)
        dts = tfdt.p[0] == 1 ? (tfdt.n >= 12 ? static_cast<int64_t>(rd64(tfdt.p + 4)) : dts) : rd32(tfdt.p + 4);
      int64_t pos = base;
      const uint8_t *tc = traf.p, *te = traf.p + traf.n;
      Box trun;
      while (next_box(tc, te, &trun)) {
        if (trun.type != fourcc("trun")) continue;
        if (trun.n < 8) return "truncated trun";
        const int ver = trun.p[0];
        const uint32_t rf = rd32(trun.p) & 0xffffff, count = rd32(trun.p + 4);
        size_t r = 8;
        if (rf & 0x1) {
          if (r + 4 > trun.n) return "truncated trun";
          pos = base + static_cast<int32_t>(rd32(trun.p + r));
          r += 4;
        }
        uint32_t first_flags = 0;
        const bool has_first = (rf & 0x4) != 0;
        if (has_first) {
          if (r + 4 > trun.n) return "truncated trun";
          first_flags = rd32(trun.p + r);
          r += 4;
        }
        const size_t per = 4u * (((rf >> 8) & 1) + ((rf >> 9) & 1) + ((rf >> 10) & 1) + ((rf >> 11) & 1));
        if (r + per * count > trun.n) return "truncated trun";
        for (uint32_t i = 0; i < count; ++i) {
          uint32_t dur = d.duration, sz = d.size, fl = (i == 0 && has_first) ? first_flags : d.flags;
          int32_t cto = 0;
          if (rf & 0x100) { dur = rd32(trun.p + r); r += 4; }
          if (rf & 0x200) { sz = rd32(trun.p + r); r += 4; }
          if (rf & 0x400) { fl = rd32(trun.p + r); r += 4; }
          if (rf & 0x800) {
            const uint32_t c = rd32(trun.p + r);
            cto = ver == 0 && c > 0x7fffffffu ? 0x7fffffff : static_cast<int32_t>(c);
            r += 4;
          }
          if (pos < 0 || pos + static_cast<int64_t>(sz) > info->file_size) return "fragment sample outside the file";
          t->offset.push_back(pos);
          t->size.push_back(sz);
          t->dts.push_back(dts);
          t->cts_offset.push_back(cto);
          t->sync.push_back(((fl >> 16) & 1) ? 0 : 1);
          if (cto) t->has_ctts = true;
          pos += sz;
          dts += dur;
        }
      }
      t->has_stss = true;  // every fragment sample's sync flag is explicit
      next_dts[ti] = dts;
      prev_end = pos;
      first_traf = false;
    }
  }
  // the track's media duration: its fragments' end (track timescale)
  for (size_t k = 0; k < info->tracks.size(); ++k)
    if (next_dts[k] > info->tracks[k].duration && !moofs.empty()) info->tracks[k].duration = next_dts[k];
  info->video.clear();
  for (const Mp4VideoTrack &t : info->tracks)
    if (t.handler == fourcc("vide")) info->video.push_back(t);
  return "";
}

std::string parse_source(const Source &src, Mp4Info *info) {
  *info = Mp4Info{};
  info->file_size = src.size();
  int64_t pos = 0;
  std::vector<uint8_t> moov;
  std::vector<Moof> moofs;
  bool have_moov = false;
  while (pos + 8 <= src.size()) {
    uint8_t h[16];
    if (!src.read(pos, h, 8)) return "read error";
    uint64_t size = rd32(h);
    const uint32_t type = rd32(h + 4);
    int64_t hdr = 8;
    if (size == 1) {
      if (!src.read(pos + 8, h + 8, 8)) return "read error";
      size = rd64(h + 8);
      hdr = 16;
    } else if (size == 0) {
      size = static_cast<uint64_t>(src.size() - pos);
    }
    if (size < static_cast<uint64_t>(hdr) || pos + static_cast<int64_t>(size) > src.size()) {
      if (have_moov) break;  // trailing garbage after a complete moov
      return "truncated or corrupt box";
    }
    if (type == fourcc("moov")) {
      if (size > (1ull << 31)) return "moov too large";
      moov.resize(static_cast<size_t>(size - hdr));
      if (!src.read(pos + hdr, moov.data(), moov.size())) return "read error";
      have_moov = true;
    } else if (type == fourcc("moof")) {
      info->fragmented = true;
      if (size > (64ull << 20)) return "moof too large";
      Moof m;
      m.start = pos;
      m.payload.resize(static_cast<size_t>(size - hdr));
      if (!src.read(pos + hdr, m.payload.data(), m.payload.size())) return "read error";
      moofs.push_back(std::move(m));
    }
    pos += static_cast<int64_t>(size);
  }
  if (!have_moov) return "no moov box (not an MP4/ISO-BMFF file)";
  Box root{fourcc("moov"), moov.data(), moov.size()};
  Box mvhd, mvex;
  if (find_child(root, fourcc("mvhd"), &mvhd) && mvhd.n >= 20) {
    info->has_mvhd = true;
    if (mvhd.p[0] == 1) {
      if (mvhd.n < 32) return "bad mvhd";
      info->movie_timescale = rd32(mvhd.p + 20);
      info->movie_duration = static_cast<int64_t>(rd64(mvhd.p + 24));
    } else {
      info->movie_timescale = rd32(mvhd.p + 12);
      info->movie_duration = rd32(mvhd.p + 16);
    }
  }
  if (find_child(root, fourcc("mvex"), &mvex)) info->fragmented = true;
  const uint8_t *cur = root.p, *end = root.p + root.n;
  Box b;
  while (next_box(cur, end, &b)) {
    if (b.type == fourcc("trak")) {
      const std::string e = parse_trak(b, info);
      if (!e.empty()) return e;
    }
  }
  if (info->fragmented) return apply_fragments(root, moofs, info);
  return "";
}

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

// Box builder: begin() reserves the size field, end() patches it.
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

}  // namespace

std::string mp4_parse_file(const char *path, Mp4Info *out) {
  FileSource src;
  src.fd = ::open(path, O_RDONLY | O_CLOEXEC);
  if (src.fd < 0) return std::string("cannot open ") + path + ": " + std::strerror(errno);
  struct stat st;
  if (::fstat(src.fd, &st) != 0) return "stat failed";
  if (!S_ISREG(st.st_mode)) return "not a regular file";
  src.sz = st.st_size;
  return parse_source(src, out);
}

std::string mp4_parse_memory(const uint8_t *data, int64_t size, Mp4Info *out) {
  MemSource src;
  src.p = data;
  src.sz = size;
  return parse_source(src, out);
}

int64_t mvhd_duration_us(const Mp4Info &info) {
  int64_t ts = info.movie_timescale;
  if (ts <= 0) ts = 1;
  const __int128 a = info.movie_duration;
  // av_rescale_rnd(a, 1000000, ts, AV_ROUND_NEAR_INF)
  const __int128 num = a * 1000000;
  const __int128 half = ts / 2;
  const __int128 q = (num >= 0) ? (num + half) / ts : -((-num + half) / ts);
  return static_cast<int64_t>(q);
}

int64_t container_duration_us(const Mp4Info &info) {
  if (!info.has_mvhd) return -1;
  if (info.movie_duration > 0 || !info.fragmented) return mvhd_duration_us(info);
  int64_t best = -1;
  for (const Mp4VideoTrack &t : info.tracks) {
    if (t.dts.empty()) continue;
    Mp4Info one;  // the track's own timescale through the same rounding
    one.movie_timescale = t.timescale;
    one.movie_duration = t.duration - t.dts.front();
    best = std::max(best, mvhd_duration_us(one));
  }
  return best;
}

// ------------------------------------------------------------------ writer

Mp4Writer::~Mp4Writer() {
  if (f_) std::fclose(f_);
}

std::string Mp4Writer::open(const char *path) {
  f_ = std::fopen(path, "wb");
  if (!f_) return std::string("cannot create ") + path + ": " + std::strerror(errno);
  std::setvbuf(f_, nullptr, _IOFBF, 4 << 20);  // samples are small: 4 MiB writes
  std::vector<uint8_t> v;
  {
    BoxW ftyp(v, "ftyp");
    putfour(v, "isom");
    put32(v, 0x200);
    putfour(v, "isom");
    putfour(v, "iso2");
    putfour(v, "avc1");
    putfour(v, "mp41");
  }
  mdat_start_ = static_cast<int64_t>(v.size());
  put32(v, 1);  // 64-bit size follows
  putfour(v, "mdat");
  put64(v, 0);  // patched in finish()
  if (std::fwrite(v.data(), 1, v.size(), f_) != v.size()) return "write error";
  pos_ = static_cast<int64_t>(v.size());
  return "";
}

std::string Mp4Writer::add_sample(const uint8_t *data, size_t n, bool sync, uint32_t cts_frames) {
  if (!f_) return "writer not open";
  if (n > 0xffffffffu) return "sample too large";
  if (std::fwrite(data, 1, n, f_) != n) return "write error";
  cts_.push_back(cts_frames);
  any_cts_ |= cts_frames != 0;
  offsets_.push_back(pos_);
  sizes_.push_back(static_cast<uint32_t>(n));
  if (sync) sync_.push_back(static_cast<uint32_t>(sizes_.size()));
  pos_ += static_cast<int64_t>(n);
  return "";
}

std::string Mp4Writer::append(const uint8_t *data, size_t n, int64_t *offset) {
  if (!f_) return "writer not open";
  if (n && std::fwrite(data, 1, n, f_) != n) return "write error";
  *offset = pos_;
  pos_ += static_cast<int64_t>(n);
  return "";
}

std::string Mp4Writer::add_sample_at(int64_t offset, size_t n, bool sync) {
  if (!f_) return "writer not open";
  if (n > 0xffffffffu) return "sample too large";
  if (offset < mdat_start_ || offset + static_cast<int64_t>(n) > pos_) return "sample outside mdat";
  cts_.push_back(0);
  offsets_.push_back(offset);
  sizes_.push_back(static_cast<uint32_t>(n));
  if (sync) sync_.push_back(static_cast<uint32_t>(sizes_.size()));
  return "";
}

std::string Mp4Writer::finish(int width, int height, int64_t track_timescale,
                              int64_t sample_delta, const std::vector<uint8_t> &sps,
                              const std::vector<uint8_t> &pps) {
  if (!f_) return "writer not open";
  const uint64_t nsamp = sizes_.size();
  const uint64_t track_dur = nsamp * static_cast<uint64_t>(sample_delta);
  const uint64_t movie_ts = 1000;
  // movie duration in ms, rounded to nearest
  const uint64_t movie_dur =
      (track_dur * movie_ts + static_cast<uint64_t>(track_timescale) / 2) /
      static_cast<uint64_t>(track_timescale);
  std::vector<uint8_t> v;
  {
    BoxW moov(v, "moov");
    {
      BoxW mvhd(v, "mvhd");
      v.push_back(1);  // version 1: 64-bit times
      v.push_back(0); v.push_back(0); v.push_back(0);
      put64(v, 0); put64(v, 0);
      put32(v, static_cast<uint32_t>(movie_ts));
      put64(v, movie_dur);
      put32(v, 0x00010000);  // rate
      put16(v, 0x0100);      // volume
      put16(v, 0); put32(v, 0); put32(v, 0);
      put_matrix(v);
      for (int i = 0; i < 6; ++i) put32(v, 0);
      put32(v, 2);  // next_track_ID
    }
    {
      BoxW trak(v, "trak");
      {
        BoxW tkhd(v, "tkhd");
        v.push_back(1);
        v.push_back(0); v.push_back(0); v.push_back(3);  // enabled | in_movie
        put64(v, 0); put64(v, 0);
        put32(v, 1);  // track_ID
        put32(v, 0);
        put64(v, movie_dur);
        put32(v, 0); put32(v, 0);
        put16(v, 0); put16(v, 0); put16(v, 0); put16(v, 0);
        put_matrix(v);
        put32(v, static_cast<uint32_t>(width) << 16);
        put32(v, static_cast<uint32_t>(height) << 16);
      }
      {
        BoxW mdia(v, "mdia");
        {
          BoxW mdhd(v, "mdhd");
          v.push_back(1);
          v.push_back(0); v.push_back(0); v.push_back(0);
          put64(v, 0); put64(v, 0);
          put32(v, static_cast<uint32_t>(track_timescale));
          put64(v, track_dur);
          put16(v, 0x55c4);  // "und"
          put16(v, 0);
        }
        {
          BoxW hdlr(v, "hdlr");
          put32(v, 0); put32(v, 0);
          putfour(v, "vide");
          put32(v, 0); put32(v, 0); put32(v, 0);
          const char name[] = "VideoHandler";
          v.insert(v.end(), name, name + sizeof name);
        }
        {
          BoxW minf(v, "minf");
          {
            BoxW vmhd(v, "vmhd");
            put32(v, 1);
            put16(v, 0); put16(v, 0); put16(v, 0); put16(v, 0);
          }
          {
            BoxW dinf(v, "dinf");
            BoxW dref(v, "dref");
            put32(v, 0);
            put32(v, 1);
            BoxW url(v, "url ");
            put32(v, 1);
          }
          {
            BoxW stbl(v, "stbl");
            {
              BoxW stsd(v, "stsd");
              put32(v, 0);
              put32(v, 1);
              BoxW avc1(v, "avc1");
              for (int i = 0; i < 6; ++i) v.push_back(0);
              put16(v, 1);  // data_reference_index
              for (int i = 0; i < 16; ++i) v.push_back(0);
              put16(v, static_cast<uint32_t>(width));
              put16(v, static_cast<uint32_t>(height));
              put32(v, 0x00480000); put32(v, 0x00480000);
              put32(v, 0);
              put16(v, 1);  // frame_count
              uint8_t comp[32] = {0};
              const char cname[] = "vtseg synthetic";
              comp[0] = sizeof cname - 1;
              std::memcpy(comp + 1, cname, sizeof cname - 1);
              v.insert(v.end(), comp, comp + 32);
              put16(v, 0x18);
              put16(v, 0xffff);
              BoxW avcc(v, "avcC");
              v.push_back(1);
              v.push_back(sps.size() > 1 ? sps[1] : 66);
              v.push_back(sps.size() > 2 ? sps[2] : 0);
              v.push_back(sps.size() > 3 ? sps[3] : 30);
              v.push_back(0xfc | 3);  // 4-byte NAL lengths
              v.push_back(0xe0 | 1);
              put16(v, static_cast<uint32_t>(sps.size()));
              v.insert(v.end(), sps.begin(), sps.end());
              v.push_back(1);
              put16(v, static_cast<uint32_t>(pps.size()));
              v.insert(v.end(), pps.begin(), pps.end());
            }
            {
              BoxW stts(v, "stts");
              put32(v, 0);
              put32(v, 1);
              put32(v, static_cast<uint32_t>(nsamp));
              put32(v, static_cast<uint32_t>(sample_delta));
            }
            if (any_cts_) {  // composition offsets, run-length coded (version 0)
              std::vector<std::pair<uint32_t, uint32_t>> runs;
              for (uint32_t c : cts_) {
                const uint32_t o = c * static_cast<uint32_t>(sample_delta);
                if (!runs.empty() && runs.back().second == o) ++runs.back().first;
                else runs.emplace_back(1u, o);
              }
              BoxW ctts(v, "ctts");
              put32(v, 0);
              put32(v, static_cast<uint32_t>(runs.size()));
              for (const auto &r : runs) {
                put32(v, r.first);
                put32(v, r.second);
              }
            }
            if (sync_.size() != nsamp) {
              BoxW stss(v, "stss");
              put32(v, 0);
              put32(v, static_cast<uint32_t>(sync_.size()));
              for (uint32_t s : sync_) put32(v, s);
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
              put32(v, static_cast<uint32_t>(nsamp));
              for (uint32_t s : sizes_) put32(v, s);
            }
            {
              BoxW co64(v, "co64");
              put32(v, 0);
              put32(v, static_cast<uint32_t>(nsamp));
              for (int64_t o : offsets_) put64(v, static_cast<uint64_t>(o));
            }
          }
        }
      }
    }
  }
  if (std::fwrite(v.data(), 1, v.size(), f_) != v.size()) return "write error";
  const int64_t mdat_size = pos_ - mdat_start_;
  std::vector<uint8_t> sz;
  put64(sz, static_cast<uint64_t>(mdat_size));
  if (std::fseek(f_, static_cast<long>(mdat_start_ + 8), SEEK_SET) != 0) return "seek error";
  if (std::fwrite(sz.data(), 1, 8, f_) != 8) return "write error";
  pos_ += static_cast<int64_t>(v.size());
  const int rc = std::fclose(f_);
  f_ = nullptr;
  if (rc != 0) return "close error";
  return "";
}

}  // namespace vts
