// session_full.hip — the general decoder's schedule and run loop (vts_ctx with
// general = true).  DESIGN.md §5b.
//
// Open: every slice header is parsed on the host (h264_sched.cpp), which also
// keeps the reference picture bookkeeping, so each slice reaches the device
// with its RefPicList0 as ring slots.  A picture's level is one more than the
// highest level among the pictures its lists may name; windows hold whole
// runs of pictures that start at an intra picture no later picture predicts
// across (as in the subset path), sized to a ring budget of decoded surfaces,
// macroblock records and coefficient arena.
// Run, per window (two rings, decode of window i+1 overlapping scoring of
// window i): the slice parse (+ h264_derive for CABAC), then per level and
// GOP group the inter, intra and deblocking launches over that level's
// pictures (recon_full_launch; the level's bS on a paced side stream), then
// scoring: per level thumb_pics + the window's thumb_sad when surfaces are
// recycled (keep_frames 0), else score.hip's pass over the finished pictures.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"
#include "decode.h"
#include "decode_full.h"
#include "h264_sched.h"
#include "session.h"

namespace vts {
namespace {

// Coefficient blocks a slice may store.  CAVLC: a stored block costs >= 3
// bits, and each slice gets that bound as its own range.  CABAC: every stored
// 4x4 block holds a non-zero level, whose sign is one bypass bin = one bit the
// arithmetic decoder reads (an 8x8 block stores four 4x4 blocks per such bit),
// so 32 x the NAL bytes is a bound too — ~37x what real CABAC streams store
// (x264-like content: ~0.9 blocks per byte); the window's arena is sized from
// `per_byte` blocks per byte instead (cabac_window_blocks) and grows when a run
// overflows it.  Either way never more than the 27 blocks a macroblock holds.
// (per_byte_q4: quarter blocks per byte)
int64_t slice_arena_cap(bool cabac, int64_t n_mbs, int64_t nal_size, int64_t per_byte_q4) {
  const int64_t per_mb = static_cast<int64_t>(kMbMaxBlocks) * n_mbs;
  if (!cabac) return std::min<int64_t>(per_mb, 3ll * nal_size + 27);
  return std::min<int64_t>(per_mb, per_byte_q4 * nal_size / 4 + 64);
}
// CABAC: a window's arena for `blocks` stored blocks over `n_slices` slices:
// each slice leaves its last chunk partly unused and a chunk switch abandons
// fewer than kMbMaxBlocks of kArenaChunk (< 1/9)
int64_t cabac_window_blocks(int64_t blocks, int64_t n_slices) {
  return blocks + blocks / 8 + static_cast<int64_t>(kArenaChunk) * n_slices;
}

// per ring: parse throughput grows with the slices per launch, and every
// window runs its own chain of reconstruction levels, so one window per
// 10-min 720p CABAC video (~104 GB: the arena reserves 27 blocks per
// macroblock) while HBM allows it (avail / 2 below)
constexpr int64_t kWindowBytes = 128ll << 30;
constexpr int64_t kMinRingBytes = 1ll << 30;

}  // namespace

bool general_by_headers(const vts_ctx *c) {
  if (c->pps.entropy_coding_mode) return true;  // CABAC
  // a High-profile PPS tail (8x8 transform, scaling lists, a Cr QP offset the
  // subset kernels' deblocking gate does not see): ADVICE r03
  if (c->pps.has_tail) return true;
  if (c->pps.weighted_pred || c->pps.weighted_bipred_idc) return true;
  if (c->sps.max_num_ref_frames > 1 || c->pps.num_ref_idx_l0_default_active > 1) return true;
  return !c->pps.deblocking_filter_control_present;  // deblocking on, offsets 0
}

bool wants_general(const vts_ctx *c, const uint8_t *es, const std::vector<int64_t> &es_off,
                   const std::vector<uint32_t> &sizes, int nal_length_size) {
  if (general_by_headers(c)) return true;
  // the first pictures' slice headers: an active deblocking filter or several references
  const size_t n = std::min<size_t>(sizes.size(), 3);
  std::vector<int64_t> off(es_off.begin(), es_off.begin() + static_cast<int64_t>(n));
  std::vector<uint32_t> sz(sizes.begin(), sizes.begin() + static_cast<int64_t>(n));
  std::vector<SchedFrame> frames;
  std::vector<SchedSlice> slices;
  if (!sched_build(c->sps, c->pps, es, off, sz, nal_length_size, &frames, &slices).empty()) return true;
  // 8.7.2.2: an edge is filtered only where indexA = qPav + filterOffsetA >= 16
  // (alpha is 0 below).  Chroma edges use QPc of QPY + chroma_qp_index_offset;
  // QPc(x) = x below 30 and >= 29 from there, so x + offset >= 16 is exact
  // for the slice's QPY (I_PCM's QPY 0 only lowers qPav).
  const int cqp = std::max(0, c->pps.chroma_qp_index_offset);
  for (const SchedSlice &s : slices)
    if ((s.dbk_idc != 1 && s.qp + cqp + s.dbk_a >= 16) || (s.is_p && s.num_ref > 1)) return true;
  return false;
}

int build_general(vts_ctx *c, const uint8_t *es, const std::vector<int64_t> &es_off,
                  const std::vector<uint32_t> &sizes, int nal_length_size, const std::vector<uint8_t> &sps_nal,
                  const std::vector<uint8_t> &pps_nal) {
  SchedStream facts;
  std::string e = sched_stream_facts(sps_nal, pps_nal, c->sps, c->pps, &facts);
  if (!e.empty()) return fail(VTS_E_UNSUPPORTED, "%s", e.c_str());
  if (c->sps.crop_left || c->sps.crop_top) return fail(VTS_E_UNSUPPORTED, "left/top cropping is not supported");
  std::vector<SchedFrame> frames;
  std::vector<SchedSlice> slices;
  e = sched_build(c->sps, c->pps, es, es_off, sizes, nal_length_size, &frames, &slices);
  if (!e.empty()) return fail(VTS_E_UNSUPPORTED, "%s", e.c_str());
  c->general = true;
  c->fused = false;
  c->fprm = FullParams{};
  c->fprm.mb_width = c->sps.mb_width;
  c->fprm.mb_height = c->sps.mb_height;
  c->fprm.cip = c->pps.constrained_intra_pred;
  c->fprm.cqp_off = c->pps.chroma_qp_index_offset;
  c->fprm.cqp_off2 = facts.cqp_off2;
  c->fprm.cabac = c->pps.entropy_coding_mode;
  c->fprm.t8mode = facts.transform_8x8;
  c->fprm.scaled = facts.seq_scaling || facts.pic_scaling;
  c->scale_tab = facts.scale;
  for (const SchedFrame &fr : frames) c->fprm.bframes |= fr.has_b ? 1 : 0;
  c->fprm.direct8x8 = c->sps.direct_8x8_inference;
  const int64_t n = c->n_frames;
  const std::vector<int64_t> &disp = c->disp;  // presentation rank per sample
  const int64_t nmb = static_cast<int64_t>(c->sps.mb_width) * c->sps.mb_height;

  // levels and clean window starts
  std::vector<int64_t> level(static_cast<size_t>(n), 0), minref(static_cast<size_t>(n), n);
  for (int64_t f = 0; f < n; ++f) {
    const SchedFrame &fr = frames[static_cast<size_t>(f)];
    int64_t l = 0;
    for (int64_t r : fr.refs) {
      l = std::max(l, level[static_cast<size_t>(r)] + 1);
      minref[static_cast<size_t>(f)] = std::min(minref[static_cast<size_t>(f)], r);
    }
    level[static_cast<size_t>(f)] = l;
  }
  // clean[x]: an intra picture no later picture predicts across, before which
  // exactly the pictures [0, x) of the presentation order are decoded (so a
  // window is the same range of frames in decode and presentation order)
  std::vector<uint8_t> clean(static_cast<size_t>(n), 0);
  {
    int64_t m = n;
    for (int64_t x = n - 1; x >= 0; --x) {
      m = std::min(m, minref[static_cast<size_t>(x)]);
      clean[static_cast<size_t>(x)] = frames[static_cast<size_t>(x)].intra && m >= x;
    }
    int64_t mx = -1;
    for (int64_t x = 0; x < n; ++x) {
      if (mx != x - 1) clean[static_cast<size_t>(x)] = 0;
      mx = std::max(mx, disp[static_cast<size_t>(x)]);
    }
  }
  // parse order: a B picture's direct prediction reads its colocated
  // picture's records, so it parses one launch after that picture's
  std::vector<int32_t> plevel(static_cast<size_t>(n), 0);
  for (int64_t f = 0; f < n; ++f)
    for (int64_t col : frames[static_cast<size_t>(f)].cols)
      plevel[static_cast<size_t>(f)] = std::max(plevel[static_cast<size_t>(f)], plevel[static_cast<size_t>(col)] + 1);
  // coefficient blocks each slice may need (slice_arena_cap): CAVLC its
  // range, CABAC its share of the window's arena estimate
  c->arena_q4 = 3;  // 0.75 blocks per byte
  if (const char *ev = std::getenv("VTS_ARENA_PER_BYTE")) c->arena_q4 = 4 * std::max(0, std::atoi(ev));
  std::vector<int64_t> cap(slices.size());
  int64_t cap_total = 0;
  for (size_t i = 0; i < slices.size(); ++i) {
    cap[i] = slice_arena_cap(c->pps.entropy_coding_mode, slices[i].n_mbs, slices[i].nal_size, c->arena_q4);
    cap_total += cap[i];
  }
  // windows
  const int64_t tw_f = static_cast<int64_t>(c->width / c->k) * (c->height / c->k);
  const int64_t per_frame = c->frame_stride +
                            nmb * static_cast<int64_t>(sizeof(MbRec) + sizeof(uint16_t) + sizeof(DbkInfo) +
                                                       (c->fprm.bframes ? sizeof(MbRecB) : 0)) +
                            score_workspace_bytes(c->width, c->height, c->k, 1) +
                            32 * ((cap_total + n - 1) / std::max<int64_t>(1, n));
  size_t free_b = 0, total_b = 0;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(vts::dmem_free(&free_b, &total_b));
  // whole-video buffers: the elementary stream and its RBSP copy (d_rbsp,
  // same size), per-frame scoring outputs, the slice table with its RBSP
  // lengths and parse order, the per-picture parse counters, 1 GiB of slack
  const int64_t whole = 2 * c->es_bytes + n * (3 * tw_f + 1024 + 12 + 2 * 4) +
                        static_cast<int64_t>(slices.size()) *
                            static_cast<int64_t>(sizeof(FullSlice) + 2 * sizeof(int64_t) + 2 * sizeof(int32_t)) +
                        (1ll << 30);
  const int64_t avail = std::max<int64_t>(0, static_cast<int64_t>(free_b) - whole);
  const int64_t ring_budget = std::min(kWindowBytes, std::max(kMinRingBytes, avail / 4));
  int64_t wcap;
  if (c->params.window_frames > 0) wcap = c->params.window_frames;
  else if (n * per_frame <= std::min(kWindowBytes, avail / 2)) wcap = n;
  else wcap = std::max<int64_t>(1, ring_budget / per_frame);
  // ring slots are int16 (FullSlice.slot / ref_slot, MbRec ref slots, level
  // lists); VTS_WINDOW_SLOT_CAP lowers the cap (tests of the refusal below)
  int64_t slot_cap = 32767;
  if (const char *sc = std::getenv("VTS_WINDOW_SLOT_CAP")) slot_cap = std::max<int64_t>(1, std::min<int64_t>(32767, std::atoll(sc)));
  wcap = std::min<int64_t>(wcap, slot_cap);
  auto next_clean = [&](int64_t x) {
    while (x < n && !clean[static_cast<size_t>(x)]) ++x;
    return x;
  };
  c->windows.clear();
  for (int64_t f = 0; f < n;) {
    Window w;
    w.f0 = f;
    int64_t end = next_clean(f + 1);
    while (end < n) {
      const int64_t nxt = next_clean(end + 1);
      if (nxt - f > wcap) break;
      end = nxt;
    }
    w.f1 = end;
    // a window always reaches the next clean picture, so clean pictures
    // further apart than the slot range (one IDR then an endless GOP, intra
    // refresh, long open GOPs) cannot be windowed: refuse, never wrap a slot
    if (w.f1 - w.f0 > slot_cap)
      return fail(VTS_E_UNSUPPORTED,
                  "frames %lld..%lld hold no clean intra picture to start a window at (%lld frames > %lld ring slots)",
                  (long long)w.f0, (long long)w.f1 - 1, (long long)(w.f1 - w.f0), (long long)slot_cap);
    c->windows.push_back(w);
    f = end;
  }
  c->ring_frames = 0;
  for (const Window &w : c->windows) c->ring_frames = std::max(c->ring_frames, w.f1 - w.f0);
  c->n_rings = (c->windows.size() > 1 && c->params.n_streams >= 2) ? 2 : 1;

  // per window: device slices (window-relative slots and arena), level lists
  c->fslices.clear();
  c->fslice_nmbs.clear();
  c->exts.clear();
  c->porder.clear();
  c->porder_m.clear();
  c->pneed.clear();
  c->dslots.clear();
  c->level_frames.clear();
  c->arena_blocks = 0;
  c->arena_bound = 0;
  c->arena_reruns = 0;
  // recycled surfaces: only where no caller reads a decoded frame back (no
  // keep_frames, no transcode yet); VTS_SURF_POOL=0 keeps one surface per slot
  {
    const char *sp = std::getenv("VTS_SURF_POOL");
    c->surf_pool = c->params.keep_frames == 0 && !c->small.on && !(sp && std::atoi(sp) == 0);
  }
  c->surf_of.assign(static_cast<size_t>(c->surf_pool ? n : 0), 0);
  c->surf_count = 0;
  for (Window &w : c->windows) {
    w.fs0 = static_cast<int64_t>(c->fslices.size());
    int64_t arena = 0, abound = 0, maxl = 0;
    int32_t maxp = 0;
    for (int64_t f = w.f0; f < w.f1; ++f) maxp = std::max(maxp, plevel[static_cast<size_t>(f)]);
    w.plv_end.clear();
    auto slot_of = [&](int64_t f) { return static_cast<int16_t>(disp[static_cast<size_t>(f)] - w.f0); };
    for (int32_t pl = 0; pl <= maxp; ++pl) {
    for (int64_t f = w.f0; f < w.f1; ++f) {
      if (plevel[static_cast<size_t>(f)] != pl) continue;
      const SchedFrame &fr = frames[static_cast<size_t>(f)];
      maxl = std::max(maxl, level[static_cast<size_t>(f)]);
      for (int64_t si = fr.s0; si < fr.s0 + fr.ns; ++si) {
        const SchedSlice &s = slices[static_cast<size_t>(si)];
        FullSlice d{};
        d.nal_offset = s.nal_offset;
        d.nal_size = s.nal_size;
        d.slot = slot_of(f);
        d.first_mb = s.first_mb;
        d.data_byte = s.data_byte;
        d.data_bit = s.data_bit;
        d.is_p = s.is_p;
        d.qp = s.qp;
        d.num_ref = s.num_ref;
        d.dbk_idc = s.dbk_idc;
        d.dbk_a = s.dbk_a;
        d.dbk_b = s.dbk_b;
        if (!c->fprm.cabac) {
          d.arena = static_cast<uint32_t>(arena);
          d.arena_cap = static_cast<uint32_t>(cap[static_cast<size_t>(si)]);
        }
        arena += cap[static_cast<size_t>(si)];
        abound += slice_arena_cap(true, s.n_mbs, s.nal_size, 4 * 32);
        c->fslice_nmbs.push_back(static_cast<int32_t>(s.n_mbs));
        d.ext = -1;
        for (int i = 0; i < 32; ++i) {
          const int64_t r = s.ref[i];
          if (r >= 0 && (r < w.f0 || r >= f)) return fail(VTS_E_UNSUPPORTED, "reference crosses a window boundary");
          d.ref_slot[i] = r >= 0 ? slot_of(r) : static_cast<int16_t>(-1);
        }
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
          for (int i = 0; i < 32; ++i) {
            const int64_t r = s.ref1[i];
            if (r >= 0 && (r < w.f0 || r >= f)) return fail(VTS_E_UNSUPPORTED, "reference crosses a window boundary");
            x.ref_slot1[i] = r >= 0 ? slot_of(r) : static_cast<int16_t>(-1);
            x.poc0[i] = s.poc0[i];
            x.poc1[i] = s.poc1[i];
          }
          std::memcpy(x.w, s.w, sizeof x.w);
          // the slices of a picture share one record
          if (c->exts.empty() || std::memcmp(&c->exts.back(), &x, sizeof x) != 0) c->exts.push_back(x);
          d.ext = static_cast<int32_t>(c->exts.size()) - 1;
        }
        c->fslices.push_back(d);
      }
    }
    w.plv_end.push_back(static_cast<int32_t>(static_cast<int64_t>(c->fslices.size()) - w.fs0));
    // workgroups are dispatched in index order and a slice's wave runs for
    // time ~ its size: the largest slices first, so the launch does not end
    // on a few long waves running alone
    const int64_t l0 = static_cast<int64_t>(c->porder.size()), b = w.fs0 + (pl ? w.plv_end[pl - 1] : 0);
    for (int64_t k = b; k < static_cast<int64_t>(c->fslices.size()); ++k) c->porder.push_back(static_cast<int32_t>(k - b));
    std::stable_sort(c->porder.begin() + l0, c->porder.end(), [&](int32_t x, int32_t y) {
      return c->fslices[static_cast<size_t>(b + x)].nal_size > c->fslices[static_cast<size_t>(b + y)].nal_size;
    });
    }
    // merged parse launch (window-relative): CAVLC, the levels' orders back
    // to back (a B slice waits for its colocated picture's slices, which
    // therefore come first); CABAC, every slice of the window longest first
    // (its slices are independent: h264_derive does the colocated reads)
    // (CABAC) late[slot]: the picture has one of the window's long slices, or
    // its colocated picture is late — its derivation waits for the long parse
    std::vector<uint8_t> late(static_cast<size_t>(w.f1 - w.f0), 0);
    w.plong = 0;
    if (c->fprm.cabac) {
      const int64_t nws = static_cast<int64_t>(c->fslices.size()) - w.fs0;
      const size_t o0 = c->porder_m.size();
      for (int64_t k = 0; k < nws; ++k) c->porder_m.push_back(static_cast<int32_t>(k));
      std::stable_sort(c->porder_m.begin() + static_cast<int64_t>(o0), c->porder_m.end(), [&](int32_t a, int32_t b) {
        return c->fslices[static_cast<size_t>(w.fs0 + a)].nal_size > c->fslices[static_cast<size_t>(w.fs0 + b)].nal_size;
      });
      // The launch ends on its longest slices (an x264 stream's intra
      // pictures: one wave's serial bin chain each, several times the others'
      // time).  Those of at least a quarter of the longest's size parse in a
      // launch of their own when they are at most 1/8 of the window's slices;
      // the rest parse beside them, and every picture that needs none of them
      // (its slices all short, its colocated pictures early) is derived
      // while the long ones still parse.
      // (VTS_PARSE_SPLIT=0: one launch; 2, a test mode: the longest eighth,
      // whatever the sizes)
      const char *ps = std::getenv("VTS_PARSE_SPLIT");
      c->parse_split = ps ? std::min(std::max(std::atoi(ps), 0), 2) : 1;
      if (c->parse_split && nws > 1) {
        auto size_at = [&](int64_t k) { return c->fslices[static_cast<size_t>(w.fs0 + c->porder_m[o0 + static_cast<size_t>(k)])].nal_size; };
        const int64_t mx = size_at(0);
        int64_t k = 0;
        while (k < nws && 4 * static_cast<int64_t>(size_at(k)) >= mx) ++k;
        if (c->parse_split == 2) k = std::max<int64_t>(1, nws / 8);
        if (k < nws && 8 * k <= nws) {
          w.plong = static_cast<int32_t>(k);
          for (int64_t j = 0; j < k; ++j)
            late[static_cast<size_t>(c->fslices[static_cast<size_t>(w.fs0 + c->porder_m[o0 + static_cast<size_t>(j)])].slot)] = 1;
        }
      }
    } else {
      for (size_t j = 0; j < w.plv_end.size(); ++j) {
        const int32_t b0 = j ? w.plv_end[j - 1] : 0;
        for (int32_t k = b0; k < w.plv_end[j]; ++k)
          c->porder_m.push_back(b0 + c->porder[static_cast<size_t>(w.fs0 + k)]);
      }
    }
    // h264_derive launches (CABAC): the window's pictures by parse level, so a
    // B picture's colocated picture is complete before it
    // (with the colocated slot its B slices share, so each macroblock's
    // colocated words load with its own, or -1)
    w.ds0 = static_cast<int64_t>(c->dslots.size());
    w.dlv_end.clear();
    w.dlv_early.clear();
    for (int32_t pl = 0; pl <= maxp; ++pl) {
      std::vector<int2> early, lat;
      for (int64_t f = w.f0; f < w.f1; ++f) {
        if (plevel[static_cast<size_t>(f)] != pl) continue;
        const SchedFrame &fr = frames[static_cast<size_t>(f)];
        int64_t col = -2;  // -2: no B slice yet
        for (int64_t si = fr.s0; si < fr.s0 + fr.ns; ++si) {
          const SchedSlice &sl = slices[static_cast<size_t>(si)];
          if (sl.is_p != kSliceB) continue;
          const int64_t cs = sl.ref1[0] >= 0 ? disp[static_cast<size_t>(sl.ref1[0])] - w.f0 : -1;
          col = (col == -2 || col == cs) ? cs : -1;
        }
        const int16_t sf = slot_of(f);
        for (int64_t cf : fr.cols) {  // (colocated pictures: lower parse levels, flags final)
          const int64_t cslot = disp[static_cast<size_t>(cf)] - w.f0;
          if (cslot < 0 || cslot >= w.f1 - w.f0 || late[static_cast<size_t>(cslot)]) late[static_cast<size_t>(sf)] = 1;
        }
        (late[static_cast<size_t>(sf)] ? lat : early).push_back(make_int2(sf, static_cast<int32_t>(col < 0 ? -1 : col)));
      }
      c->dslots.insert(c->dslots.end(), early.begin(), early.end());
      c->dslots.insert(c->dslots.end(), lat.begin(), lat.end());
      w.dlv_early.push_back(static_cast<int32_t>(early.size()));
      w.dlv_end.push_back(static_cast<int32_t>(static_cast<int64_t>(c->dslots.size()) - w.ds0));
    }
    w.pn0 = static_cast<int64_t>(c->pneed.size());
    c->pneed.resize(c->pneed.size() + static_cast<size_t>(w.f1 - w.f0), 0);
    for (int64_t k = w.fs0; k < static_cast<int64_t>(c->fslices.size()); ++k)
      ++c->pneed[static_cast<size_t>(w.pn0 + c->fslices[static_cast<size_t>(k)].slot)];
    c->fprm.has_ext = c->exts.empty() ? 0 : 1;
    w.fs1 = static_cast<int64_t>(c->fslices.size());
    if (c->fprm.cabac) {
      // (VTS_ARENA_PER_BYTE=0: one chunk, the tests' way to make every run
      // outgrow its first arena)
      arena = c->arena_q4 == 0 ? static_cast<int64_t>(kArenaChunk) : cabac_window_blocks(arena, w.fs1 - w.fs0);
      abound = cabac_window_blocks(abound, w.fs1 - w.fs0);
      // the chunk counter and block indices are 32-bit: the bound stays below
      // 2^32 with a chunk per slice of headroom for requests past the end
      const int64_t lim = 0xffffffffll - static_cast<int64_t>(kArenaChunk) * (w.fs1 - w.fs0 + 1);
      if (arena > lim) return fail(VTS_E_UNSUPPORTED, "window coefficient arena beyond 32-bit indices");
      c->arena_bound = std::max(c->arena_bound, std::min(abound, lim));
    } else if (arena > 0xffffffffll) {
      return fail(VTS_E_UNSUPPORTED, "window coefficient arena beyond 32-bit indices");
    }
    c->arena_blocks = std::max(c->arena_blocks, arena);
    // two interleaved groups of GOPs reconstruct on two streams: a level's
    // pictures are one workgroup each, and two unsynchronised level sequences
    // pack the compute units better than one whose every level is a whole
    // number of rounds.  A GOP here is a run of pictures that no later picture
    // of the window predicts across, so a group never reads the other's pictures.
    const int64_t wn = w.f1 - w.f0;
    std::vector<uint8_t> fg(static_cast<size_t>(wn), 0);
    int ngrp = 1;
    if (c->general_groups > 1) {
      std::vector<uint8_t> split(static_cast<size_t>(wn), 0);
      int64_t m = w.f1;
      for (int64_t x = w.f1 - 1; x >= w.f0; --x) {
        m = std::min(m, minref[static_cast<size_t>(x)]);
        split[static_cast<size_t>(x - w.f0)] = m >= x;
      }
      int64_t seg = -1;
      for (int64_t x = 0; x < wn; ++x) {
        if (split[static_cast<size_t>(x)]) ++seg;
        fg[static_cast<size_t>(x)] = static_cast<uint8_t>(seg % c->general_groups);
      }
      ngrp = static_cast<int>(std::min<int64_t>(c->general_groups, seg + 1));
    }
    w.grp.clear();
    for (int g = 0; g < ngrp; ++g) {
      if (g) w.grp.push_back(static_cast<int32_t>(w.lvl_off.size()));
      std::vector<std::vector<int4>> lv(static_cast<size_t>(maxl + 1));
      for (int64_t f = w.f0; f < w.f1; ++f)
        if (fg[static_cast<size_t>(f - w.f0)] == g)
          lv[static_cast<size_t>(level[static_cast<size_t>(f)])].push_back(make_int4(slot_of(f), 0, 0, 0));
      for (auto &l : lv) {
        if (l.empty()) continue;
        w.lvl_off.push_back(static_cast<int64_t>(c->level_frames.size()));
        w.lvl_cnt.push_back(static_cast<int32_t>(l.size()));
        c->level_frames.insert(c->level_frames.end(), l.begin(), l.end());
      }
    }
    if (c->surf_pool) {
      // j: a picture's launch index in its group.  A surface is free for the
      // group's launches after max(last reader's j, own j): its readers and
      // its thumbnails (thumb_pics right after each level launch) ran earlier
      // on the group's stream.  Each group its own pool: the groups' launches
      // are not ordered against each other.
      std::vector<int32_t> jof(static_cast<size_t>(wn), 0), last(static_cast<size_t>(wn), -1);
      const size_t nl = w.lvl_off.size();
      std::vector<size_t> glo(static_cast<size_t>(ngrp) + 1, nl);
      glo[0] = 0;
      for (int g = 1; g < ngrp; ++g) glo[static_cast<size_t>(g)] = static_cast<size_t>(w.grp[static_cast<size_t>(g - 1)]);
      for (int g = 0; g < ngrp; ++g)
        for (size_t l = glo[static_cast<size_t>(g)]; l < glo[static_cast<size_t>(g) + 1]; ++l)
          for (int32_t i = 0; i < w.lvl_cnt[l]; ++i)
            jof[static_cast<size_t>(c->level_frames[static_cast<size_t>(w.lvl_off[l] + i)].x)] =
                static_cast<int32_t>(l - glo[static_cast<size_t>(g)]);
      for (int64_t f = w.f0; f < w.f1; ++f)
        for (int64_t rf : frames[static_cast<size_t>(f)].refs) {
          int32_t &lr = last[static_cast<size_t>(slot_of(rf))];
          lr = std::max(lr, jof[static_cast<size_t>(slot_of(f))]);
        }
      int64_t base = 0;
      for (int g = 0; g < ngrp; ++g) {
        const size_t l0 = glo[static_cast<size_t>(g)], l1 = glo[static_cast<size_t>(g) + 1];
        std::vector<std::vector<int32_t>> freed(l1 - l0);
        std::vector<int32_t> pool;
        int32_t made = 0;
        for (size_t l = l0; l < l1; ++l) {
          const size_t j = l - l0;
          if (j > 0) {
            for (int32_t s : freed[j - 1]) pool.push_back(s);
            freed[j - 1].clear();
          }
          for (int32_t i = 0; i < w.lvl_cnt[l]; ++i) {
            const int32_t slot = c->level_frames[static_cast<size_t>(w.lvl_off[l] + i)].x;
            int32_t s;
            if (pool.empty()) s = made++;
            else {
              s = pool.back();
              pool.pop_back();
            }
            c->surf_of[static_cast<size_t>(w.f0 + slot)] = static_cast<int32_t>(base + s);
            const size_t fa = static_cast<size_t>(std::max<int64_t>(last[static_cast<size_t>(slot)], static_cast<int64_t>(j)));
            if (fa < freed.size()) freed[fa].push_back(s);
          }
        }
        base += made;
      }
      c->surf_count = std::max(c->surf_count, base);
    }
  }
  // Deblocking descriptors (h264_bs_full -> h264_deblock_plane) live in a
  // ring of two level slots per GOP group: level l + 1's bS is derived while
  // level l deblocks, and level l + 2's only after level l + 1's inter launch,
  // which follows level l's deblocking on the group's stream (run_general).
  // Slot (2 g + (j & 1)) x the most pictures of a level, j the level's index
  // in its group; int4.y of each level entry is its picture's descriptor slot.
  // (When that ring would not be smaller than one slot per picture — few,
  // wide levels, e.g. all-intra — each picture keeps its own slot.)
  int64_t maxcnt = 1, maxg = 1;
  for (const Window &w : c->windows) {
    for (int32_t n2 : w.lvl_cnt) maxcnt = std::max<int64_t>(maxcnt, n2);
    maxg = std::max<int64_t>(maxg, 1 + static_cast<int64_t>(w.grp.size()));
  }
  if (2 * maxg * maxcnt >= c->ring_frames) {
    for (int4 &f : c->level_frames) f.y = f.x;
    c->dbk_pics = c->ring_frames;
    return VTS_OK;
  }
  for (const Window &w : c->windows) {
    int g = 0;
    size_t lo = 0;
    for (size_t l = 0; l < w.lvl_off.size(); ++l) {
      while (g < static_cast<int>(w.grp.size()) && l >= static_cast<size_t>(w.grp[static_cast<size_t>(g)])) {
        lo = static_cast<size_t>(w.grp[static_cast<size_t>(g)]);
        ++g;
      }
      const int64_t base = (2 * g + static_cast<int64_t>((l - lo) & 1)) * maxcnt;
      for (int32_t i = 0; i < w.lvl_cnt[l]; ++i)
        c->level_frames[static_cast<size_t>(w.lvl_off[l] + i)].y = static_cast<int32_t>(base + i);
    }
  }
  c->dbk_pics = 2 * maxg * maxcnt;
  return VTS_OK;
}

int run_general(vts_ctx *c) {
  VTS_TRY(submit_general(c));
  c->pending = true;
  return finish_all(c);
}

int submit_general(vts_ctx *c) {
  HIP_TRY(hipSetDevice(c->device));
  if (c->surf_pool && c->small.on) {
    // a transcode (after open) reads every decoded frame of a window: one
    // surface per window slot from now on
    HIP_TRY(hipDeviceSynchronize());
    for (int r = 0; r < c->n_rings; ++r) {
      vts::dfree(c->d_surf[r]);
      c->d_surf[r] = nullptr;
      HIP_TRY(vts::dmalloc(&c->d_surf[r], static_cast<size_t>(c->ring_frames * c->frame_stride + 256)));  // + kPad (session.hip)
    }
    c->surf_pool = false;
  }
  if (!c->h_err) HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&c->h_err), sizeof(uint32_t)));
  HIP_TRY(hipMemsetAsync(c->d_err, 0, sizeof(uint32_t), c->s_dec));
  HIP_TRY(hipEventRecord(c->ev_start, c->s_dec));
  HIP_TRY(hipStreamWaitEvent(c->s_score, c->ev_start, 0));
  HIP_TRY(hipStreamWaitEvent(c->s_parse, c->ev_start, 0));
  hipStream_t sd = c->s_dec;
  // slice parsing runs on its own stream one window ahead: window i + 1 parses
  // (thousands of one-lane waves) while window i reconstructs (one workgroup per
  // picture of a level, which leaves most compute units idle)
  hipStream_t sp = c->s_parse;
  hipStream_t ss = (c->params.n_streams >= 2 && c->windows.size() > 1) ? c->s_score : c->s_dec;
  // the paced bS launches: on the score stream when scoring is not on it (one
  // window, or one stream); with several windows scored on s_score, on a
  // group stream of their own (else window i + 1's bS, and with it its first
  // level, would queue behind window i's scoring; VTS_BS_STREAM=0:
  // the score stream regardless)
  hipStream_t sbs = c->s_score;
  if (ss == c->s_score && c->general_groups < vts_ctx::kMaxGroups) {
    const char *e = std::getenv("VTS_BS_STREAM");
    if (!e || std::atoi(e) != 0) sbs = c->s_grp[vts_ctx::kMaxGroups - 2];
  }
  const int64_t nmb = static_cast<int64_t>(c->sps.mb_width) * c->sps.mb_height;
  const size_t nw = c->windows.size();
  for (size_t wi = 0; wi < nw; ++wi) {
    const Window &w = c->windows[wi];
    const int r = static_cast<int>(wi % c->n_rings);
    hipEvent_t *E = &c->ev[wi * 6];
    if (wi >= static_cast<size_t>(c->n_rings)) {  // ring r: the window before has been scored
      HIP_TRY(hipStreamWaitEvent(sp, c->ev[(wi - c->n_rings) * 6 + 4], 0));
      HIP_TRY(hipStreamWaitEvent(sd, c->ev[(wi - c->n_rings) * 6 + 4], 0));
    }
    const int ng = 1 + static_cast<int>(w.grp.size());
    const int64_t run = c->run_no++;
    const uint32_t epoch = 1u + static_cast<uint32_t>(run % 0x7fffffff);
    if (c->ring_cleared_at[r] < 0) {  // records of another run read as absent (their epoch)
      HIP_TRY(hipMemsetAsync(c->d_recs[r], 0, static_cast<size_t>(c->ring_frames * nmb) * sizeof(MbRec), sp));
      c->ring_cleared_at[r] = run;
    }
    HIP_TRY(hipEventRecord(E[0], sp));
    FullParseArgs pa{};
    pa.rbsp = c->d_rbsp;
    pa.epoch = epoch;
    pa.recs = c->d_recs[r];
    pa.recs1 = c->d_recs1[r];
    pa.exts = c->d_exts;
    pa.ilvl = c->d_ilvl[r];
    pa.arena = c->d_arena[r];
    pa.err = c->d_err;
    pa.P = c->fprm;
    if (c->fprm.cabac) {
      pa.arena_top = c->d_arena_top + wi;
      pa.arena_blocks = static_cast<uint32_t>(c->arena_blocks);
      HIP_TRY(hipMemsetAsync(pa.arena_top, 0, sizeof(uint32_t), sp));
      // syntax records of every slice (no waits), then the per-picture
      // derivation by parse level
      pa.slices = c->d_fslices + w.fs0;
      pa.rbsp_len = c->d_rbsp_len + w.fs0;
      pa.n_slices = static_cast<int32_t>(w.fs1 - w.fs0);
      pa.slice0 = 0;
      pa.order = c->d_porder_m + w.fs0;
      pa.pdone = nullptr;
      pa.pneed = nullptr;
      DeriveArgs da{};
      da.recs = c->d_recs[r];
      da.recs1 = c->d_recs1[r];
      da.ilvl = c->d_ilvl[r];
      da.slices = c->d_fslices + w.fs0;
      da.exts = c->d_exts;
      da.err = c->d_err;
      da.epoch = epoch;
      da.P = c->fprm;
      // the long slices on the parse stream; the others, then the early
      // pictures' derivation, on a stream with a hardware queue of its own
      // (HIP puts plain streams on its few queues in turn, and two streams on
      // one queue run one after the other: the short launch would wait for
      // the long one): a session on CU-masked streams (own queues) uses its
      // third GOP group's, idle at two groups; one on plain streams makes one
      // (each stream on a queue of its own was measured: four content
      // sessions through plan_batch 2.34x -> 2.72x one session's step, the
      // process's queues being time-sliced)
      const bool own_q = c->stream_kind == 1 && c->general_groups <= 2;
      if (w.plong > 0 && !own_q && !c->s_px) {
        int cus = 0;
        HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
        std::vector<uint32_t> mask(static_cast<size_t>((cus + 31) / 32), 0u);
        for (int i = 0; i < cus; ++i) mask[static_cast<size_t>(i >> 5)] |= 1u << (i & 31);
        HIP_TRY(hipExtStreamCreateWithCUMask(&c->s_px, static_cast<uint32_t>(mask.size()), mask.data()));
      }
      hipStream_t sx = w.plong > 0 ? (own_q ? c->s_grp[1] : c->s_px) : nullptr;
      if (sx) {
        if (c->ev_px.size() < 2 * nw) {
          const size_t n0 = c->ev_px.size();
          c->ev_px.resize(2 * nw, nullptr);
          for (size_t k = n0; k < c->ev_px.size(); ++k) HIP_TRY(hipEventCreateWithFlags(&c->ev_px[k], hipEventDisableTiming));
        }
        HIP_TRY(hipEventRecord(c->ev_px[2 * wi], sp));  // the ring's records and the arena counter are reset
        HIP_TRY(hipStreamWaitEvent(sx, c->ev_px[2 * wi], 0));
        pa.n_slices = w.plong;
        FullParseArgs ps = pa;
        ps.order = c->d_porder_m + w.fs0 + w.plong;
        ps.n_slices = static_cast<int32_t>(w.fs1 - w.fs0) - w.plong;
        VTS_TRY(parse_full_launch(pa, sp));
        // the long slices' waves are the window's critical path: their launch
        // is dispatched before the short one's thousands of waves fill the
        // compute units (two queues' launches start in either order; without
        // this the content parse measured 130 or 157 ms run to run)
        VTS_TRY(delay_launch(50, sx));
        VTS_TRY(parse_full_launch(ps, sx));
        for (size_t j = 0; j < w.dlv_end.size(); ++j) {
          const int32_t b0 = j ? w.dlv_end[j - 1] : 0;
          da.pics = c->d_dslots + w.ds0 + b0;
          VTS_TRY(derive_launch(da, w.dlv_early[j], sx));
        }
        HIP_TRY(hipEventRecord(c->ev_px[2 * wi + 1], sx));
        HIP_TRY(hipStreamWaitEvent(sp, c->ev_px[2 * wi + 1], 0));
        for (size_t j = 0; j < w.dlv_end.size(); ++j) {
          const int32_t b0 = (j ? w.dlv_end[j - 1] : 0) + w.dlv_early[j];
          da.pics = c->d_dslots + w.ds0 + b0;
          VTS_TRY(derive_launch(da, w.dlv_end[j] - b0, sp));
        }
      } else {
        VTS_TRY(parse_full_launch(pa, sp));
        for (size_t j = 0; j < w.dlv_end.size(); ++j) {
          const int32_t b0 = j ? w.dlv_end[j - 1] : 0;
          da.pics = c->d_dslots + w.ds0 + b0;
          VTS_TRY(derive_launch(da, w.dlv_end[j] - b0, sp));
        }
      }
    } else if (c->parse_merged && w.plv_end.size() > 1) {
      // one launch: B slices wait for their colocated pictures' slices, which
      // come first in the order, so the launch ends on a full machine instead
      // of once per colocated level on its longest slices alone
      HIP_TRY(hipMemsetAsync(c->d_pdone[r], 0, sizeof(uint32_t) * static_cast<size_t>(w.f1 - w.f0), sp));
      pa.slices = c->d_fslices + w.fs0;
      pa.rbsp_len = c->d_rbsp_len + w.fs0;
      pa.n_slices = static_cast<int32_t>(w.fs1 - w.fs0);
      pa.slice0 = 0;
      pa.order = c->d_porder_m + w.fs0;
      pa.pdone = c->d_pdone[r];
      pa.pneed = c->d_pneed + w.pn0;
      VTS_TRY(parse_full_launch(pa, sp));
    } else {
      for (size_t j = 0; j < w.plv_end.size(); ++j) {  // B pictures after their colocated pictures
        const int32_t b0 = j ? w.plv_end[j - 1] : 0;
        pa.slices = c->d_fslices + w.fs0 + b0;
        pa.rbsp_len = c->d_rbsp_len + w.fs0 + b0;
        pa.n_slices = w.plv_end[j] - b0;
        pa.slice0 = b0;
        pa.order = c->d_porder + w.fs0 + b0;
        VTS_TRY(parse_full_launch(pa, sp));
      }
    }
    HIP_TRY(hipEventRecord(E[1], sp));
    HIP_TRY(hipStreamWaitEvent(sd, E[1], 0));
    HIP_TRY(hipEventRecord(E[5], sd));
    FullReconArgs ra{};
    ra.recs = c->d_recs[r];
    ra.recs1 = c->d_recs1[r];
    ra.exts = c->d_exts;
    ra.ilvl = c->d_ilvl[r];
    ra.dbk = c->d_dbk[r];
    ra.arena = c->d_arena[r];
    ra.slices = c->d_fslices + w.fs0;
    ra.surf = c->d_surf[r];
    ra.surf_of = c->surf_pool ? c->d_surf_of + w.f0 : nullptr;
    ra.frame_stride = c->frame_stride;
    ra.uv_off = static_cast<int64_t>(c->pitch) * c->coded_h;
    ra.pitch = c->pitch;
    ra.epoch = epoch;
    ra.deblock = 1;
    ra.intra_kernel = c->intra_kernel;
    ra.err = c->d_err;
    ra.sct = c->d_scale;
    ra.P = c->fprm;
    {
      // bS needs only the parse's records: one launch per level on the score
      // stream, paced by the chain (level l + 1's after level l's inter launch),
      // beside the intra and deblocking launches that leave most compute units
      // idle.  (Measured and dropped, DESIGN.md §9: one window-wide launch at the
      // head of the chain that both GOP groups waited for; bS inside each inter
      // launch.)
      const bool paced = !w.lvl_off.empty();
      auto bs_level = [&](size_t l, hipStream_t s) {
        ra.frames = c->d_levels + w.lvl_off[l];
        return bs_full_launch(ra, w.lvl_cnt[l], s);
      };
      if (c->surf_pool)  // thumb_pics' bands add into the window's histograms
        HIP_TRY(hipMemsetAsync(c->d_hist + w.f0 * 256, 0, sizeof(uint32_t) * 256 * static_cast<size_t>(w.f1 - w.f0), sd));
      if (ng > 1) {  // groups >= 1 on their own streams, after the parse
        HIP_TRY(hipEventRecord(c->ev_grp[0], sd));
        for (int g = 1; g < ng; ++g) HIP_TRY(hipStreamWaitEvent(c->s_grp[g - 1], c->ev_grp[0], 0));
      }
      // the groups' level launches, interleaved (j-th level of every group, then
      // the next): the score stream derives level j + 1's bS while
      // group g runs level j's intra and deblocking launches (compute units the
      // one-workgroup-per-picture kernels leave idle), and level j + 1 waits for it
      // (one side stream for every group: the groups' bS on separate streams,
      // odd groups' on the parse stream, measured slower — 188 -> 201 ms on the
      // content stream, that stream sharing a hardware queue with a group's,
      // profiles/r04t_bs_paced_split_ab.json)
      auto sb_of = [&](int) { return sbs; };
      // recycled surfaces: each level's thumbnails right after its
      // reconstruction, on the group's stream (the liveness plan's promise)
      PicThumbArgs ta{};
      if (c->surf_pool) {
        const int rb = c->k == 6 ? 48 : 16;
        ta.surf = c->d_surf[r];
        ta.frame_stride = c->frame_stride;
        ta.surf_of = c->d_surf_of + w.f0;
        ta.w = c->width / c->k;
        ta.h = c->height / c->k;
        ta.pitch = c->pitch;
        ta.uv_row_offset = c->coded_h;
        ta.chunks_per_row = c->width / rb;
        ta.n_chunks = ta.chunks_per_row * ta.h;
        ta.f0 = w.f0;
        ta.thumb = c->d_thumb[r];
        ta.rgb = c->d_rgb;
        ta.hist = c->d_hist;
      }
      std::vector<size_t> lo(static_cast<size_t>(ng)), hi(static_cast<size_t>(ng));
      size_t jmax = 0;
      for (int g = 0; g < ng; ++g) {
        lo[static_cast<size_t>(g)] = g ? static_cast<size_t>(w.grp[static_cast<size_t>(g - 1)]) : 0;
        hi[static_cast<size_t>(g)] = g + 1 < ng ? static_cast<size_t>(w.grp[static_cast<size_t>(g)]) : w.lvl_off.size();
        jmax = std::max(jmax, hi[static_cast<size_t>(g)] - lo[static_cast<size_t>(g)]);
      }
      if (paced) {
        if (c->ev_bs.size() < 2 * w.lvl_off.size()) {
          const size_t n0 = c->ev_bs.size();
          c->ev_bs.resize(2 * w.lvl_off.size(), nullptr);
          for (size_t k = n0; k < c->ev_bs.size(); ++k) HIP_TRY(hipEventCreateWithFlags(&c->ev_bs[k], hipEventDisableTiming));
        }
        HIP_TRY(hipStreamWaitEvent(sbs, E[1], 0));
        for (int g = 0; g < ng; ++g) {  // every group's first level
          if (lo[static_cast<size_t>(g)] >= hi[static_cast<size_t>(g)]) continue;
          VTS_TRY(bs_level(lo[static_cast<size_t>(g)], sb_of(g)));
          HIP_TRY(hipEventRecord(c->ev_bs[2 * lo[static_cast<size_t>(g)]], sb_of(g)));
        }
      }
      for (size_t jj = 0; jj < jmax; ++jj)
        for (int g = 0; g < ng; ++g) {
          const size_t l = lo[static_cast<size_t>(g)] + jj;
          if (l >= hi[static_cast<size_t>(g)]) continue;
          hipStream_t s = g ? c->s_grp[g - 1] : sd;
          if (paced) HIP_TRY(hipStreamWaitEvent(s, c->ev_bs[2 * l], 0));
          ra.frames = c->d_levels + w.lvl_off[l];
          const bool next = paced && l + 1 < hi[static_cast<size_t>(g)];
          VTS_TRY(recon_full_launch(ra, w.lvl_cnt[l], s, next ? c->ev_bs[2 * l + 1] : nullptr));
          if (c->surf_pool) {
            ta.pics = c->d_levels + w.lvl_off[l];
            ta.n_pics = w.lvl_cnt[l];
            VTS_TRY(thumb_pics_launch(ta, c->k, s));
          }
          if (next) {
            HIP_TRY(hipStreamWaitEvent(sb_of(g), c->ev_bs[2 * l + 1], 0));
            VTS_TRY(bs_level(l + 1, sb_of(g)));
            HIP_TRY(hipEventRecord(c->ev_bs[2 * (l + 1)], sb_of(g)));
          }
        }
      for (int g = 1; g < ng; ++g) {
        HIP_TRY(hipEventRecord(c->ev_grp[g - 1], c->s_grp[g - 1]));
        HIP_TRY(hipStreamWaitEvent(sd, c->ev_grp[g - 1], 0));
      }
    }
    if (c->small.on) VTS_TRY(small_window(c, r, w.f0, w.f1, sd));
    HIP_TRY(hipEventRecord(E[2], sd));
    HIP_TRY(hipStreamWaitEvent(ss, E[2], 0));
    HIP_TRY(hipEventRecord(E[3], ss));
    if (c->surf_pool) {  // SAD and score from the thumbnail ring
      ThumbSadArgs t{};
      t.thumb = c->d_thumb[r];
      t.prev_luma = wi > 0 ? c->d_last[(wi - 1) & 1] : nullptr;
      t.last_luma = c->d_last[wi & 1];
      t.frame0 = w.f0;
      t.n_frames = w.f1 - w.f0;
      t.w = c->width / c->k;
      t.h = c->height / c->k;
      t.sad = c->d_sad;
      t.score = c->d_score;
      VTS_TRY(thumb_sad_launch(t, ss));
      HIP_TRY(hipEventRecord(E[4], ss));
      continue;
    }
    vts_score_desc d{};
    d.nv12 = c->d_surf[r];
    d.frame_stride = c->frame_stride;
    d.n_frames = w.f1 - w.f0;
    d.width = c->width;
    d.height = c->height;
    d.pitch = c->pitch;
    d.uv_row_offset = c->coded_h;
    d.k = c->k;
    d.rgb = c->d_rgb + 3 * c->thumb_px * w.f0;
    d.hist = c->d_hist + w.f0 * 256;
    d.sad = c->d_sad + w.f0;
    d.score = c->d_score + w.f0;
    d.prev_luma = wi > 0 ? c->d_last[(wi - 1) & 1] : nullptr;
    d.last_luma = c->d_last[wi & 1];
    d.workspace = c->d_ws[r];
    d.workspace_bytes = c->ws_bytes;
    VTS_TRY(score_launch(&d, ss));
    HIP_TRY(hipEventRecord(E[4], ss));
  }
  HIP_TRY(hipStreamWaitEvent(sd, c->ev[(nw - 1) * 6 + 4], 0));
  HIP_TRY(hipMemcpyAsync(c->h_err, c->d_err, sizeof(uint32_t), hipMemcpyDeviceToHost, sd));
  HIP_TRY(hipEventRecord(c->ev_end, sd));
  return VTS_OK;
}

int finish_general(vts_ctx *c) {
  const size_t nw = c->windows.size();
  HIP_TRY(hipEventSynchronize(c->ev_end));
  const uint32_t err = *c->h_err;
  float ms = 0;
  HIP_TRY(hipEventElapsedTime(&ms, c->ev_start, c->ev_end));
  c->timings[0] = ms;
  c->timings[1] = c->timings[2] = c->timings[3] = 0;
  for (size_t wi = 0; wi < nw; ++wi) {
    hipEvent_t *E = &c->ev[wi * 6];
    float a = 0, b = 0, s = 0;
    HIP_TRY(hipEventElapsedTime(&a, E[0], E[1]));
    HIP_TRY(hipEventElapsedTime(&b, E[5], E[2]));
    HIP_TRY(hipEventElapsedTime(&s, E[3], E[4]));
    c->timings[1] += a;
    c->timings[2] += b;
    c->timings[3] += s;
  }
  c->last_window_done = static_cast<int64_t>(nw) - 1;
  if ((err & DEC_E_ARENA) && c->fprm.cabac && c->arena_blocks < c->arena_bound) {
    // a window's slices asked for more coefficient blocks than its arena
    // holds: the largest request (the counters keep counting past the end)
    // with a quarter more, at least twice the arena, at most the bound; the
    // run again
    std::vector<uint32_t> top(nw);
    HIP_TRY(hipMemcpy(top.data(), c->d_arena_top, sizeof(uint32_t) * nw, hipMemcpyDeviceToHost));
    const int64_t need = *std::max_element(top.begin(), top.end());
    c->arena_blocks = std::min(c->arena_bound, std::max(2 * c->arena_blocks, need + need / 4));
    ++c->arena_reruns;
    for (int r = 0; r < c->n_rings; ++r) {
      vts::dfree(c->d_arena[r]);
      c->d_arena[r] = nullptr;
      HIP_TRY(vts::dmalloc(&c->d_arena[r], static_cast<size_t>(std::max<int64_t>(1, c->arena_blocks)) * 32 + 256));  // + kPad (session.hip)
    }
    return run_all(c);
  }
  if (err) {
    c->have_results = false;
    return fail(VTS_E_DECODE, "device decoder: %s", describe_decode_error(err).c_str());
  }
  c->have_results = true;
  c->host_scores.clear();
  return VTS_OK;
}

}  // namespace vts
