// CPU harness of the general device decoder: the product's host scheduler
// (h264_sched.cpp) and the very per-slice parser / per-picture derivation /
// per-macroblock reconstruction and deblocking code the GPU kernels run
// (parse_full.h, parse_cabac.h, derive_full.h, recon_full.h), driven in the
// kernels' order — inter macroblocks first,
// intra macroblocks and deblocking along the x + 2y wavefront — on host
// memory.  TEST INFRASTRUCTURE (tests/test_full_host.py compares it with the
// oracle); the product never runs the decoder on the CPU.
#include <algorithm>
#include <barrier>
#include <cstdio>
#include <thread>
#include <cstring>
#include <string>
#include <vector>

// -DVTS_STATS: count the parser's trace points (VTS_PARSE_TRACE: 0 macroblock,
// 1 context-coded bin, 2 bypass bin, 3 terminate bin) for fh_stats()
#ifdef VTS_STATS
static unsigned long long g_trace[32];
#define VTS_PARSE_TRACE(k) (++g_trace[(k)])
extern "C" void fh_stats(unsigned long long *out) {
  for (int i = 0; i < 8; ++i) out[i] = g_trace[i];
}
#endif
#include "h264.h"
#include "h264_full.h"
#include "h264_sched.h"
#include "mp4.h"
#include "parse_cabac.h"
#include "parse_full.h"
#include "derive_full.h"
#include "recon_full.h"
#include "intra_lanes.h"

using namespace vts;

// flags bit 2: intra macroblocks through the device's lane-parallel code
// (intra_lanes.h, h264_intra_v2), 32 host threads playing the 32 lanes
namespace {
struct HostGroup {
  std::barrier<> bar{32};
  int buf[32];
};
struct HostLanes {
  int t;
  HostGroup *g;
  void sync() const { g->bar.arrive_and_wait(); }
  int red16(int v) const {
    g->bar.arrive_and_wait();
    g->buf[t] = v;
    g->bar.arrive_and_wait();
    int s = 0;
    for (int i = 0; i < 16; ++i) s += g->buf[(t & 16) + i];
    g->bar.arrive_and_wait();
    return s;
  }
  void amax(int *p, int v) const { *p = std::max(*p, v); }  // one macroblock at a time on the host
  int bcast(int v, int l) const {
    g->bar.arrive_and_wait();
    g->buf[t] = v;
    g->bar.arrive_and_wait();
    const int r = g->buf[l];
    g->bar.arrive_and_wait();
    return r;
  }
};
// one picture's intra macroblocks level by level (the kernel's order; one
// macroblock at a time), line buffers as the kernel's LDS
void intra_lanes_picture(const i2::I2Ctx &ctx, const uint16_t *lv) {
  const int nmb = ctx.mbw * ctx.mbh;
  std::vector<std::pair<int, int>> order;  // (level, mb)
  for (int i = 0; i < nmb; ++i)
    if (lv[i] != kNoLevel) order.emplace_back(lv[i], i);
  std::stable_sort(order.begin(), order.end());
  std::vector<i2::I2Line> lines(static_cast<size_t>(ctx.mbw + ctx.mbh));
  for (auto &l : lines) l.tag = l.claim = -2;
  i2::I2Line *lcol = lines.data(), *lrow = lines.data() + ctx.mbw;
  uint8_t off4[9 * 16], off8[9 * 64];
  for (int i = 0; i < 9 * 16; ++i) off4[i] = static_cast<uint8_t>(i2::i2_intra4_off(i >> 4, i & 3, (i >> 2) & 3));
  for (int i = 0; i < 9 * 64; ++i) off8[i] = static_cast<uint8_t>(i2::i2_intra8_off(i >> 6, i & 7, (i >> 3) & 7));
  auto *T = new i2::I2Tile;
  HostGroup grp;
  std::vector<std::thread> th;
  for (int t = 0; t < 32; ++t)
    th.emplace_back([&, t]() {
      const HostLanes L{t, &grp};
      i2::I2NoProf np;
      // every macroblock's prefetch before any reconstruction: the kernel
      // prefetches a level ahead, so the border samples of neighbours this
      // launch reconstructs may predate them (part 1 must not use those)
      std::vector<i2::I2Pre> pre(order.size());
      for (size_t k = 0; k < order.size(); ++k) pre[k] = i2::i2_prefetch(ctx, order[k].second, t);
      L.sync();
      for (size_t k = 0; k < order.size(); ++k) {
        const auto &o = order[k];
        i2::intra2_prepare(ctx, o.second, pre[k], L, *T, lcol, lrow, np);
        L.sync();
        i2::intra2_finish(ctx, L, *T, lcol, lrow, off4, off8, np);
        L.sync();
      }
    });
  for (auto &x : th) x.join();
  delete T;
}
}  // namespace

// LevelScale4x4 / 8x8 the product derives from a file's SPS / PPS
// (sched_stream_facts, 8.5.9): ls4 = 6 x 6 x 16, ls8 = 2 x 6 x 64 int32
extern "C" int fh_scale(const char *path, int32_t *ls4, int32_t *ls8, int *flags, char *err, int err_cap) {
  auto bad = [&](const std::string &m) {
    std::snprintf(err, static_cast<size_t>(err_cap), "%s", m.c_str());
    return -1;
  };
  Mp4Info mp4;
  std::string e = mp4_parse_file(path, &mp4);
  if (!e.empty()) return bad(e);
  if (mp4.video.empty() || mp4.video.front().sps.empty() || mp4.video.front().pps.empty())
    return bad("no video track / parameter sets");
  const Mp4VideoTrack &t = mp4.video.front();
  Sps sps;
  Pps pps;
  e = parse_sps(t.sps[0].data(), t.sps[0].size(), &sps);
  if (e.empty()) e = parse_pps(t.pps[0].data(), t.pps[0].size(), &pps);
  SchedStream facts;
  if (e.empty()) e = sched_stream_facts(t.sps[0], t.pps[0], sps, pps, &facts);
  if (!e.empty()) return bad(e);
  std::memcpy(ls4, facts.scale.ls4, sizeof facts.scale.ls4);
  std::memcpy(ls8, facts.scale.ls8, sizeof facts.scale.ls8);
  flags[0] = facts.seq_scaling;
  flags[1] = facts.pic_scaling;
  return 0;
}

extern "C" int fh_decode(const char *path, int flags, uint8_t *out, int64_t out_cap, int64_t *n_out,
                         int *w_out, int *h_out, char *err, int err_cap) {
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
  if (!e.empty()) return bad("SPS: " + e);
  e = parse_pps(t.pps[0].data(), t.pps[0].size(), &pps);
  if (!e.empty()) return bad("PPS: " + e);
  SchedStream facts;
  e = sched_stream_facts(t.sps[0], t.pps[0], sps, pps, &facts);
  if (!e.empty()) return bad(e);
  // elementary stream: samples back to back
  std::vector<uint8_t> es;
  std::vector<int64_t> off;
  FILE *f = std::fopen(path, "rb");
  if (!f) return bad("open");
  for (size_t i = 0; i < t.size.size(); ++i) {
    off.push_back(static_cast<int64_t>(es.size()));
    const size_t n0 = es.size();
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
  const int n = static_cast<int>(frames.size());
  // presentation order: rank of dts + composition offset
  std::vector<int> disp(static_cast<size_t>(n));
  {
    std::vector<int> ord(static_cast<size_t>(n));
    for (int i = 0; i < n; ++i) ord[static_cast<size_t>(i)] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) {
      return t.dts[static_cast<size_t>(a)] + t.cts_offset[static_cast<size_t>(a)] <
             t.dts[static_cast<size_t>(b)] + t.cts_offset[static_cast<size_t>(b)];
    });
    for (int i = 0; i < n; ++i) disp[static_cast<size_t>(ord[static_cast<size_t>(i)])] = i;
  }
  const int mbw = sps.mb_width, mbh = sps.mb_height, nmb = mbw * mbh;
  const int pitch = mbw * 16, ch = mbh * 16;
  const int64_t stride = static_cast<int64_t>(pitch) * ch * 3 / 2;
  const int W = sps.width(), H = sps.height();
  *w_out = W;
  *h_out = H;
  *n_out = n;
  if (out_cap < static_cast<int64_t>(n) * W * H * 3 / 2) return bad("output too small");
  std::vector<uint8_t> surf(static_cast<size_t>(stride) * n + 64, 0);
  std::vector<MbRec> recs(static_cast<size_t>(nmb) * n);
  std::vector<uint16_t> ilvl(static_cast<size_t>(nmb) * n);
  std::vector<FullSlice> fs(slices.size());
  std::vector<SliceExt> exts;
  bool bframes = false;
  for (const SchedFrame &fr : frames) bframes |= fr.has_b;
  std::vector<MbRecB> recs1(bframes ? static_cast<size_t>(nmb) * n : 0);
  uint32_t arena_blocks = 0;
  for (size_t i = 0; i < slices.size(); ++i) {
    const SchedSlice &s = slices[i];
    FullSlice &d = fs[i];
    std::memset(&d, 0, sizeof d);
    d.nal_offset = s.nal_offset;
    d.nal_size = s.nal_size;
    d.slot = static_cast<int32_t>(s.frame);
    d.first_mb = s.first_mb;
    d.data_byte = s.data_byte;
    d.data_bit = s.data_bit;
    d.is_p = s.is_p;
    d.qp = s.qp;
    d.num_ref = s.num_ref;
    d.dbk_idc = s.dbk_idc;
    d.dbk_a = s.dbk_a;
    d.dbk_b = s.dbk_b;
    const int64_t cap = pps.entropy_coding_mode ? 27ll * s.n_mbs : std::min<int64_t>(27ll * s.n_mbs, 3ll * s.nal_size + 27);
    d.arena = arena_blocks;
    d.arena_cap = static_cast<uint32_t>(cap);
    arena_blocks += static_cast<uint32_t>(cap);
    for (int r = 0; r < 32; ++r) d.ref_slot[r] = static_cast<int16_t>(s.ref[r] >= 0 ? s.ref[r] : -1);
    d.ext = -1;
    if (s.needs_ext()) {
      SliceExt x;
      std::memset(&x, 0, sizeof x);
      x.num_ref1 = s.num_ref1;
      x.direct_spatial = s.direct_spatial;
      x.wmode = s.wmode;
      x.lwd = s.lwd;
      x.cwd = s.cwd;
      x.col_short = s.col_short;
      x.poc = s.poc;
      x.lt0 = s.lt0;
      x.lt1 = s.lt1;
      for (int r = 0; r < 32; ++r) {
        x.ref_slot1[r] = static_cast<int16_t>(s.ref1[r] >= 0 ? s.ref1[r] : -1);
        x.poc0[r] = s.poc0[r];
        x.poc1[r] = s.poc1[r];
      }
      std::memcpy(x.w, s.w, sizeof x.w);
      d.ext = static_cast<int32_t>(exts.size());
      exts.push_back(x);
    }
  }
  // CABAC: the session's window arena (session_full.hip cabac_window_blocks)
  if (pps.entropy_coding_mode) arena_blocks += arena_blocks / 8 + kArenaChunk * static_cast<uint32_t>(slices.size());
  std::vector<int16_t> arena(static_cast<size_t>(arena_blocks) * 16 + 16);
  // the kernel's LDS holds whatever the CU's last workgroup left there: the
  // harness fills it with a poison byte, never zeros
  auto poisoned_lds = [&]() {
    std::vector<uint64_t> lds((full::syn_lds_bytes(mbw) + 7) / 8);
    std::memset(lds.data(), 0xA5, lds.size() * sizeof(uint64_t));
    return lds;
  };
  FullParams P{};
  P.mb_width = mbw;
  P.mb_height = mbh;
  P.cip = pps.constrained_intra_pred;
  P.cqp_off = pps.chroma_qp_index_offset;
  P.cqp_off2 = facts.cqp_off2;
  P.cabac = pps.entropy_coding_mode;
  P.t8mode = facts.transform_8x8;
  P.scaled = facts.seq_scaling || facts.pic_scaling;
  P.bframes = bframes;
  P.has_ext = exts.empty() ? 0 : 1;
  P.direct8x8 = sps.direct_8x8_inference;
  const uint32_t epoch = 7;
  // CABAC: the window arena's block counter (kArenaChunk at a time; the
  // host decodes the whole stream as one window).  flags bit 3: the arena cut
  // to exactly what the slices ask for — a first parse of every slice counts
  // the blocks handed out, the decode below runs with that capacity (the same
  // requests in the same order on the host), then a canary region after it
  // must be untouched (no store past the blocks handed out)
  constexpr int16_t kCanary = 0x5a5b;
  uint32_t arena_top = 0, arena_cap = arena_blocks;
  if ((flags & 8) && pps.entropy_coding_mode) {
    for (int fi = 0; fi < n; ++fi) {
      const SchedFrame &fr = frames[static_cast<size_t>(fi)];
      for (int64_t si = fr.s0; si < fr.s0 + fr.ns; ++si) {
        const FullSlice &fsl = fs[static_cast<size_t>(si)];
        const SliceExt *x = fsl.ext >= 0 ? &exts[static_cast<size_t>(fsl.ext)] : nullptr;
        std::vector<uint8_t> rbsp(static_cast<size_t>(fsl.nal_size) + 128, 0);
        const int32_t rlen = full::unescape_nal(es.data() + fsl.nal_offset + 1, fsl.nal_size - 1, rbsp.data());
        std::vector<uint64_t> lds = poisoned_lds();
        const uint32_t e = full::parse_slice_cabac(
            rbsp.data(), rlen, fsl, static_cast<uint32_t>(si), P, recs.data() + static_cast<size_t>(fi) * nmb,
            bframes ? recs1.data() + static_cast<size_t>(fi) * nmb : nullptr, x, arena.data(), &arena_top, arena_cap,
            epoch, reinterpret_cast<full::SynScratch *>(lds.data()));
        if (e) return bad("counting parse: " + describe_decode_error(e));
      }
    }
    arena_cap = arena_top;
    arena_top = 0;
    arena.assign(static_cast<size_t>(arena_cap) * 16 + 16 * 16, kCanary);
  }
  for (int fi = 0; fi < n; ++fi) {
    const SchedFrame &fr = frames[static_cast<size_t>(fi)];
    MbRec *fr_recs = recs.data() + static_cast<size_t>(fi) * nmb;
    uint32_t errs = 0;
    MbRecB *fr_recs1 = bframes ? recs1.data() + static_cast<size_t>(fi) * nmb : nullptr;
    uint16_t *fr_ilvl = ilvl.data() + static_cast<size_t>(fi) * nmb;
    for (int64_t si = fr.s0; si < fr.s0 + fr.ns; ++si) {
      const FullSlice &fsl = fs[static_cast<size_t>(si)];
      const SliceExt *x = fsl.ext >= 0 ? &exts[static_cast<size_t>(fsl.ext)] : nullptr;
      // the device's nal_unescape, serially: the payload's RBSP (+ zero padding)
      std::vector<uint8_t> rbsp(static_cast<size_t>(fsl.nal_size) + 128, 0);
      const int32_t rlen = full::unescape_nal(es.data() + fsl.nal_offset + 1, fsl.nal_size - 1, rbsp.data());
      if (P.cabac) {
        // the kernel's LDS: scratch + one SynEdge per macroblock column
        std::vector<uint64_t> lds = poisoned_lds();
        errs |= full::parse_slice_cabac(rbsp.data(), rlen, fsl, static_cast<uint32_t>(si), P, fr_recs, fr_recs1, x,
                                        arena.data(), &arena_top, arena_cap, epoch,
                                        reinterpret_cast<full::SynScratch *>(lds.data()));
      } else {
        full::FullScratch sc;
        full::BCtx bc{};
        bc.recs1 = fr_recs1;
        bc.x = x;
        if (fsl.is_p == kSliceB) {
          const int col = exts[static_cast<size_t>(fsl.ext)].ref_slot1[0];
          bc.col = recs.data() + static_cast<size_t>(col) * nmb;
          bc.col1 = recs1.data() + static_cast<size_t>(col) * nmb;
        }
        errs |= full::parse_slice_full(rbsp.data(), rlen, fsl, static_cast<uint32_t>(si), P, fr_recs, fr_ilvl,
                                       arena.data(), epoch, &sc, bc);
      }
    }
    if (errs) return bad("frame " + std::to_string(fi) + ": parse: " + describe_decode_error(errs));
    if (P.cabac) {
      // h264_derive's per-macroblock work in raster order (every neighbour
      // precedes), the colocated pictures derived earlier (decoding order)
      full::DeriveCtx dc{};
      dc.recs = fr_recs;
      dc.recs1 = fr_recs1;
      dc.ilvl = fr_ilvl;
      dc.ring = recs.data();
      dc.ring1 = bframes ? recs1.data() : nullptr;
      dc.slices = fs.data();
      dc.exts = exts.data();
      dc.mbw = mbw;
      dc.mbh = mbh;
      dc.epoch = epoch;
      dc.cip = P.cip;
      dc.direct8x8 = P.direct8x8;
      dc.bframes = P.bframes;
      dc.col = -2;  // the colocated picture the frame's B slices share, else -1 (per macroblock)
      for (int64_t si = fr.s0; si < fr.s0 + fr.ns; ++si) {
        const FullSlice &fsl = fs[static_cast<size_t>(si)];
        if (fsl.is_p != kSliceB) continue;
        const int cs = exts[static_cast<size_t>(fsl.ext)].ref_slot1[0];
        dc.col = (dc.col == -2 || dc.col == cs) ? cs : -1;
      }
      if (dc.col < 0) dc.col = -1;
      std::vector<full::DEdge> er(static_cast<size_t>(nmb)), eb(static_cast<size_t>(nmb));
      full::DWork w;
      for (int a = 0; a < nmb; ++a) {
        const int x = a % mbw, y = a / mbw;
        const full::DEdge *A = x > 0 ? &er[static_cast<size_t>(a - 1)] : nullptr;
        const full::DEdge *B = y > 0 ? &eb[static_cast<size_t>(a - mbw)] : nullptr;
        const full::DEdge *C = y > 0 && x + 1 < mbw ? &eb[static_cast<size_t>(a - mbw + 1)] : nullptr;
        const full::DEdge *D = y > 0 && x > 0 ? &eb[static_cast<size_t>(a - mbw - 1)] : nullptr;
        full::DIn in;
        full::derive_load(dc, a, in);
        errs |= full::derive_mb(dc, a, in, A, B, C, D, w, &er[static_cast<size_t>(a)], &eb[static_cast<size_t>(a)]);
      }
      if (errs) return bad("frame " + std::to_string(fi) + ": derive: " + describe_decode_error(errs));
    }
    full::ReconCtx c{};
    c.recs = fr_recs;
    c.recs1 = bframes ? recs1.data() + static_cast<size_t>(fi) * nmb : nullptr;
    c.exts = exts.data();
    c.arena = arena.data();
    c.slices = fs.data();
    c.surf = surf.data();
    c.frame_stride = stride;
    c.pitch = pitch;
    c.uv_off = static_cast<int64_t>(pitch) * ch;
    c.mbw = mbw;
    c.mbh = mbh;
    c.cip = P.cip;
    c.cqp_off = P.cqp_off;
    c.cqp_off2 = P.cqp_off2;
    c.epoch = epoch;
    c.sct = &facts.scale;
    // kernel order: inter macroblocks, then intra ones along t = x + 2y
    for (int a = 0; a < nmb; ++a) {
      const MbRec &m = fr_recs[a];
      if (m.epoch != epoch) return bad("frame " + std::to_string(fi) + ": missing macroblock");
      if (m.type == kMbInter || m.type == kMbSkip) {
        full::MbRecon r(c, fi, a, m);
        r.run();
        if (r.err) return bad("recon: " + describe_decode_error(r.err));
      }
    }
    if (flags & 2) {
      i2::I2Ctx ic{};
      ic.recs = fr_recs;
      ic.arena = arena.data();
      ic.Y = surf.data() + static_cast<int64_t>(fi) * stride;
      ic.uv_off = static_cast<int64_t>(pitch) * ch;
      ic.pitch = pitch;
      ic.mbw = mbw;
      ic.mbh = mbh;
      ic.epoch = epoch;
      ic.cip = P.cip;
      ic.cqp_off = P.cqp_off;
      ic.cqp_off2 = P.cqp_off2;
      ic.scaled = P.scaled;
      ic.sct = &facts.scale;
      // I_PCM is written by the inter pass on the device; the rest by levels
      for (int a = 0; a < nmb; ++a)
        if (fr_recs[a].type == kMbPcm) {
          full::MbRecon r(c, fi, a, fr_recs[a]);
          r.run();
        }
      intra_lanes_picture(ic, ilvl.data() + static_cast<size_t>(fi) * nmb);
    } else {
    for (int tt = 0; tt < mbw + 2 * mbh; ++tt)
      for (int y = 0; y < mbh; ++y) {
        const int x = tt - 2 * y;
        if (x < 0 || x >= mbw) continue;
        const MbRec &m = fr_recs[y * mbw + x];
        if (m.type == kMbInter || m.type == kMbSkip) continue;
        full::MbRecon r(c, fi, y * mbw + x, m);
        r.run();
        if (r.err) return bad("recon: " + describe_decode_error(r.err));
      }
    }
    if (!(flags & 1))
      for (int tt = 0; tt < mbw + 2 * mbh; ++tt)
        for (int y = 0; y < mbh; ++y) {
          const int x = tt - 2 * y;
          if (x >= 0 && x < mbw) full::deblock_mb(c, fi, y * mbw + x);
        }
    // display-size NV12 (crop right / bottom), in presentation order
    uint8_t *o = out + static_cast<int64_t>(disp[static_cast<size_t>(fi)]) * W * H * 3 / 2;
    const uint8_t *Y = surf.data() + static_cast<int64_t>(fi) * stride;
    for (int y = 0; y < H; ++y) std::memcpy(o + static_cast<int64_t>(y) * W, Y + static_cast<int64_t>(y) * pitch, W);
    for (int y = 0; y < H / 2; ++y)
      std::memcpy(o + static_cast<int64_t>(W) * H + static_cast<int64_t>(y) * W,
                  Y + static_cast<int64_t>(pitch) * ch + static_cast<int64_t>(y) * pitch, W);
  }
  if ((flags & 8) && pps.entropy_coding_mode)
    for (size_t k = static_cast<size_t>(arena_cap) * 16; k < arena.size(); ++k)
      if (arena[k] != kCanary) return bad("a slice stored past the blocks handed out");
  return 0;
}
