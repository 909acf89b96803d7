// synth.cpp — deterministic synthetic H.264 (Constrained Baseline) in MP4.
//
// The reference's only synthetic clip is `ffmpeg -f lavfi -i color=...`
// (tests/test_video_segmenter.py:147-178); there is no ffmpeg in this image,
// so the build writes its own streams whose decoded pixels are known exactly:
//   * IDR pictures: every macroblock I_PCM (raw samples, lossless);
//   * P pictures: P_L0_16x16 with an integer (even) luma motion vector and
//     coded_block_pattern 0, P_Skip where the motion is zero, and a sprinkle
//     of I_PCM macroblocks;
//   * CAVLC, one reference frame, deblocking disabled in every slice,
//     pic_order_cnt_type 2 (output order = decode order);
//   * scene cuts every U[cut_min, cut_max] seconds (a new random texture, IDR)
//     and an IDR refresh at least every gop_max seconds.
// The encoder keeps its own reconstruction (the exact decoder output), which
// is what a refresh IDR re-encodes and what `vts_synth_info` hashes.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "bitstream.h"
#include "common.h"
#include "mp4.h"
#include "synth.h"

namespace vts {
namespace {

inline uint8_t clamp_sample(int v) {  // I_PCM samples kept >= 1 (no 00 00 in PCM data)
  return static_cast<uint8_t>(v < 1 ? 1 : (v > 255 ? 255 : v));
}

struct Picture {
  int w = 0, h = 0;  // coded size (luma)
  std::vector<uint8_t> y, u, v;
  void alloc(int cw, int ch) {
    w = cw;
    h = ch;
    y.assign(size_t(w) * h, 0);
    u.assign(size_t(w / 2) * (h / 2), 128);
    v.assign(size_t(w / 2) * (h / 2), 128);
  }
};

void fill_texture(Picture &p, Pcg32 &rng, bool zero_runs) {
  synth_texture(p.y.data(), p.u.data(), p.v.data(), p.w, p.h, rng, zero_runs);
}

struct MbInfo {
  bool intra = false;
  int mvx = 0, mvy = 0;  // quarter-pel
};

inline int median3(int a, int b, int c) {
  return std::max(std::min(a, b), std::min(std::max(a, b), c));
}

// ITU-T H.264 8.4.1.3 (16x16 partition) and 8.4.1.1 (P_Skip).
struct MvPred {
  const std::vector<MbInfo> *mb;
  int mbw;
  int slice_first;
  struct N {
    bool avail;
    int ref;  // -1 unavailable or intra
    int mvx, mvy;
  };
  N get(int addr, bool exists) const {
    N n{false, -1, 0, 0};
    if (!exists || addr < slice_first) return n;
    n.avail = true;
    const MbInfo &m = (*mb)[size_t(addr)];
    if (!m.intra) {
      n.ref = 0;
      n.mvx = m.mvx;
      n.mvy = m.mvy;
    }
    return n;
  }
  void neighbours(int addr, N *a, N *b, N *c) const {
    const int x = addr % mbw, y = addr / mbw;
    *a = get(addr - 1, x > 0);
    *b = get(addr - mbw, y > 0);
    *c = get(addr - mbw + 1, y > 0 && x < mbw - 1);
    if (!c->avail) *c = get(addr - mbw - 1, y > 0 && x > 0);
  }
  void pred16x16(int addr, int *px, int *py) const {
    N a, b, c;
    neighbours(addr, &a, &b, &c);
    if (!b.avail && !c.avail && a.avail) b = c = a;
    const int match = (a.ref == 0) + (b.ref == 0) + (c.ref == 0);
    if (match == 1) {
      const N &m = (a.ref == 0) ? a : (b.ref == 0) ? b : c;
      *px = m.mvx;
      *py = m.mvy;
    } else {
      *px = median3(a.mvx, b.mvx, c.mvx);
      *py = median3(a.mvy, b.mvy, c.mvy);
    }
  }
  void pskip(int addr, int *px, int *py) const {
    const int x = addr % mbw, y = addr / mbw;
    const N a = get(addr - 1, x > 0), b = get(addr - mbw, y > 0);
    if (!a.avail || !b.avail || (a.ref == 0 && a.mvx == 0 && a.mvy == 0) ||
        (b.ref == 0 && b.mvx == 0 && b.mvy == 0)) {
      *px = *py = 0;
      return;
    }
    pred16x16(addr, px, py);
  }
};

inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Motion compensation of the whole picture with one motion vector (quarter-pel
// units, integer-pel luma: a multiple of 4) and 1/8-pel chroma (8.4.2.2.2),
// edge-clamped: every macroblock of a P picture predicts with the frame's pan.
void mc_frame(const Picture &ref, Picture &dst, int mvx, int mvy) {
  const int ix = mvx >> 2, iy = mvy >> 2;
  const int cw = ref.w / 2, ch = ref.h / 2;
  const int fx = mvx & 7, fy = mvy & 7, cix = mvx >> 3, ciy = mvy >> 3;
  auto row = [](const uint8_t *s, uint8_t *d, int w, int dx) {
    // d[x] = s[clamp(x + dx, 0, w - 1)]
    const int a = std::min(w, std::max(0, -dx)), b = std::max(a, std::min(w, w - dx));
    std::memset(d, s[0], static_cast<size_t>(a));
    if (b > a) std::memcpy(d + a, s + a + dx, static_cast<size_t>(b - a));
    std::memset(d + b, s[w - 1], static_cast<size_t>(w - b));
  };
  for (int y = 0; y < ref.h; ++y)
    row(&ref.y[size_t(clampi(y + iy, 0, ref.h - 1)) * ref.w], &dst.y[size_t(y) * dst.w], ref.w, ix);
  if (fx == 0 && fy == 0) {
    for (int y = 0; y < ch; ++y) {
      const size_t sr = size_t(clampi(y + ciy, 0, ch - 1)) * cw;
      row(&ref.u[sr], &dst.u[size_t(y) * cw], cw, cix);
      row(&ref.v[sr], &dst.v[size_t(y) * cw], cw, cix);
    }
    return;
  }
  for (int yy = 0; yy < ch; ++yy)
    for (int xx = 0; xx < cw; ++xx) {
      const int xa = clampi(xx + cix, 0, cw - 1), xb = clampi(xx + cix + 1, 0, cw - 1);
      const int ya = clampi(yy + ciy, 0, ch - 1), yb = clampi(yy + ciy + 1, 0, ch - 1);
      for (int pl = 0; pl < 2; ++pl) {
        const std::vector<uint8_t> &s = pl ? ref.v : ref.u;
        std::vector<uint8_t> &d = pl ? dst.v : dst.u;
        const int A = s[size_t(ya) * cw + xa], B = s[size_t(ya) * cw + xb];
        const int C = s[size_t(yb) * cw + xa], D = s[size_t(yb) * cw + xb];
        d[size_t(yy) * cw + xx] = static_cast<uint8_t>(
            ((8 - fx) * (8 - fy) * A + fx * (8 - fy) * B + (8 - fx) * fy * C + fx * fy * D + 32) >> 6);
      }
    }
}

void put_pcm(BitWriter &bw, const Picture &p, int mbx, int mby) {
  bw.align_zero();  // pcm_alignment_zero_bit
  uint8_t buf[384];
  int k = 0;
  for (int yy = 0; yy < 16; ++yy)
    for (int xx = 0; xx < 16; ++xx) buf[k++] = p.y[size_t(mby * 16 + yy) * p.w + mbx * 16 + xx];
  const int cw = p.w / 2;
  for (int pl = 0; pl < 2; ++pl)
    for (int yy = 0; yy < 8; ++yy)
      for (int xx = 0; xx < 8; ++xx)
        buf[k++] = (pl ? p.v : p.u)[size_t(mby * 8 + yy) * cw + mbx * 8 + xx];
  bw.bytes(buf, 384);
}

void fill_sparkle(Picture &p, int mbx, int mby, Pcg32 &rng) {
  const int base = 20 + static_cast<int>(rng.below(216));
  for (int yy = 0; yy < 16; ++yy)
    for (int xx = 0; xx < 16; ++xx)
      p.y[size_t(mby * 16 + yy) * p.w + mbx * 16 + xx] =
          clamp_sample(base + static_cast<int>(rng.below(9)) - 4);
  const int cu = 60 + static_cast<int>(rng.below(136)), cv = 60 + static_cast<int>(rng.below(136));
  const int cw = p.w / 2;
  for (int yy = 0; yy < 8; ++yy)
    for (int xx = 0; xx < 8; ++xx) {
      p.u[size_t(mby * 8 + yy) * cw + mbx * 8 + xx] = clamp_sample(cu);
      p.v[size_t(mby * 8 + yy) * cw + mbx * 8 + xx] = clamp_sample(cv);
    }
}

}  // namespace

// Smooth value-noise texture: two octaves of bilinear random grids + noise.
void synth_texture(uint8_t *py, uint8_t *pu, uint8_t *pv, int pw, int ph, Pcg32 &rng, bool zero_runs) {
  auto plane = [&](uint8_t *dst, int w, int h, int cell, int lo, int hi, int noise) {
    const int gw = w / cell + 2, gh = h / cell + 2;
    std::vector<int> g(size_t(gw) * gh), g2(size_t(gw * 4 + 2) * (gh * 4 + 2));
    for (auto &x : g) x = lo + static_cast<int>(rng.below(static_cast<uint32_t>(hi - lo)));
    const int c2 = cell / 4 > 0 ? cell / 4 : 1;
    const int g2w = w / c2 + 2, g2h = h / c2 + 2;
    g2.assign(size_t(g2w) * g2h, 0);
    for (auto &x : g2) x = static_cast<int>(rng.below(41)) - 20;
    for (int yy = 0; yy < h; ++yy) {
      const int gy = yy / cell, fy = yy % cell;
      const int hy = yy / c2, ey = yy % c2;
      for (int xx = 0; xx < w; ++xx) {
        const int gx = xx / cell, fx = xx % cell;
        const int a = g[size_t(gy) * gw + gx], b = g[size_t(gy) * gw + gx + 1];
        const int c = g[size_t(gy + 1) * gw + gx], d = g[size_t(gy + 1) * gw + gx + 1];
        const int top = a * (cell - fx) + b * fx, bot = c * (cell - fx) + d * fx;
        int val = (top * (cell - fy) + bot * fy) / (cell * cell);
        const int hx = xx / c2, ex = xx % c2;
        const int a2 = g2[size_t(hy) * g2w + hx], b2 = g2[size_t(hy) * g2w + hx + 1];
        const int c2v = g2[size_t(hy + 1) * g2w + hx], d2 = g2[size_t(hy + 1) * g2w + hx + 1];
        const int top2 = a2 * (c2 - ex) + b2 * ex, bot2 = c2v * (c2 - ex) + d2 * ex;
        val += (top2 * (c2 - ey) + bot2 * ey) / (c2 * c2);
        if (noise) val += static_cast<int>(rng.below(static_cast<uint32_t>(2 * noise + 1))) - noise;
        dst[size_t(yy) * w + xx] = clamp_sample(val);
      }
    }
  };
  plane(py, pw, ph, 64, 24, 232, 3);
  if (zero_runs)  // 4 zero samples every 97 px on every 16th row: 00 00 00 00
    for (int yy = 0; yy < ph; yy += 16)
      for (int xx = 0; xx + 4 <= pw; xx += 97) std::memset(&py[size_t(yy) * pw + xx], 0, 4);
  plane(pu, pw / 2, ph / 2, 32, 72, 184, 1);
  plane(pv, pw / 2, ph / 2, 32, 72, 184, 1);
}

void append_nal(std::vector<uint8_t> &sample, uint8_t header, std::vector<uint8_t> &rbsp) {
  std::vector<uint8_t> nal;
  nal.reserve(rbsp.size() + rbsp.size() / 64 + 8);
  nal.push_back(header);
  append_ebsp(nal, rbsp.data(), rbsp.size());
  const uint32_t n = static_cast<uint32_t>(nal.size());
  sample.push_back(uint8_t(n >> 24));
  sample.push_back(uint8_t(n >> 16));
  sample.push_back(uint8_t(n >> 8));
  sample.push_back(uint8_t(n));
  sample.insert(sample.end(), nal.begin(), nal.end());
}

// Smallest level whose MaxFS / MaxMBPS (Table A-1) admit the stream.
int h264_pick_level(int mbs, double mbps) {
  struct L { int idc, max_fs; double max_mbps; };
  static const L t[] = {{30, 1620, 40500}, {31, 3600, 108000}, {32, 5120, 216000},
                        {40, 8192, 245760}, {42, 8704, 522240}, {50, 22080, 589824},
                        {51, 36864, 983040}, {52, 36864, 2073600}};
  for (const L &l : t)
    if (mbs <= l.max_fs && mbps <= l.max_mbps) return l.idc;
  return 52;
}

// Build the SPS/PPS RBSPs for the stream (also used by tests via the file).
void make_sps_pps(int mbw, int mbh, int crop_r, int crop_b, int level,
                         std::vector<uint8_t> *sps_nal, std::vector<uint8_t> *pps_nal,
                         int chroma_qp_index_offset) {
  BitWriter s;
  s.u(8, 66);        // profile_idc: Baseline
  s.u(8, 0xC0);      // constraint_set0 + set1: Constrained Baseline
  s.u(8, static_cast<uint32_t>(level));
  s.ue(0);           // seq_parameter_set_id
  s.ue(12);          // log2_max_frame_num_minus4 -> 16 bits
  s.ue(2);           // pic_order_cnt_type 2
  s.ue(1);           // max_num_ref_frames
  s.u(1, 0);         // gaps_in_frame_num_value_allowed_flag
  s.ue(static_cast<uint32_t>(mbw - 1));
  s.ue(static_cast<uint32_t>(mbh - 1));
  s.u(1, 1);         // frame_mbs_only_flag
  s.u(1, 1);         // direct_8x8_inference_flag
  if (crop_r || crop_b) {
    s.u(1, 1);
    s.ue(0);
    s.ue(static_cast<uint32_t>(crop_r / 2));
    s.ue(0);
    s.ue(static_cast<uint32_t>(crop_b / 2));
  } else {
    s.u(1, 0);
  }
  s.u(1, 0);         // vui_parameters_present_flag
  s.trailing();
  sps_nal->clear();
  sps_nal->push_back(0x67);  // nal_ref_idc 3, type 7
  append_ebsp(*sps_nal, s.data().data(), s.data().size());

  BitWriter p;
  p.ue(0);           // pic_parameter_set_id
  p.ue(0);           // seq_parameter_set_id
  p.u(1, 0);         // entropy_coding_mode_flag: CAVLC
  p.u(1, 0);         // bottom_field_pic_order_in_frame_present_flag
  p.ue(0);           // num_slice_groups_minus1
  p.ue(0);           // num_ref_idx_l0_default_active_minus1
  p.ue(0);           // num_ref_idx_l1_default_active_minus1
  p.u(1, 0);         // weighted_pred_flag
  p.u(2, 0);         // weighted_bipred_idc
  p.se(0);           // pic_init_qp_minus26
  p.se(0);           // pic_init_qs_minus26
  p.se(chroma_qp_index_offset);
  p.u(1, 1);         // deblocking_filter_control_present_flag
  p.u(1, 0);         // constrained_intra_pred_flag
  p.u(1, 0);         // redundant_pic_cnt_present_flag
  p.trailing();
  pps_nal->clear();
  pps_nal->push_back(0x68);
  append_ebsp(*pps_nal, p.data().data(), p.data().size());
}

}  // namespace vts

using namespace vts;

namespace vts {
namespace {

void encode_chunk(const vts_synth_params &P, SynthChunk *ck) {
  const bool odd_pans = (P.edge_cases & 2) != 0;
  const int mbw = (P.width + 15) / 16, mbh = (P.height + 15) / 16;
  const int cw = mbw * 16, ch = mbh * 16;
  const double fps = double(P.fps_num) / P.fps_den;
  Pcg32 rng(ck->seed);
  Pcg32 tex_rng(ck->seed ^ 0x9e3779b97f4a7c15ull, 0x7e47);
  Picture cur, ref;
  cur.alloc(cw, ch);
  ref.alloc(cw, ch);
  std::vector<MbInfo> mbinfo(size_t(mbw) * mbh);
  const int gop_max = std::max(1, static_cast<int>(std::floor(P.gop_max_s * fps)));
  auto scene_len = [&]() {
    const double lo = std::max(P.cut_min_s, 1.0 / fps), hi = std::max(P.cut_max_s, lo);
    return std::max<int64_t>(1, static_cast<int64_t>(std::llround((lo + (hi - lo) * rng.uniform()) * fps)));
  };
  int64_t next_cut = scene_len();
  int64_t since_idr = 0;
  int frame_num = 0, idr_pic_id = ck->idr_id_base;
  // edge case bit 3: refresh pictures (not scene cuts) are written as
  // non-reference, non-IDR I pictures; the P picture after one predicts from
  // the reference picture before it
  const bool nonref_refresh = (P.edge_cases & 8) != 0;
  // edge case bit 9: deblocking on, active on chroma edges only: QPY 3,
  // chroma_qp_index_offset 12, filter offsets +12.  Luma indexA <= 3 + 12 <
  // 16 everywhere; chroma qPav reaches QPc(0 + 12) = 12 on I_PCM edges (bS 3 /
  // 4), indexA 24.  A subset decoder must refuse it; the writer's own
  // pictures are unfiltered.
  const bool chroma_dbk = (P.edge_cases & 512) != 0;
  auto qp_dbk = [&](BitWriter &bw) {
    if (chroma_dbk) {
      bw.se(-23);  // slice_qp_delta: QPY 3
      bw.ue(0);    // disable_deblocking_filter_idc
      bw.se(6);    // slice_alpha_c0_offset_div2
      bw.se(6);    // slice_beta_offset_div2
    } else {
      bw.se(0);    // slice_qp_delta
      bw.ue(1);    // disable_deblocking_filter_idc
    }
  };
  bool prev_was_ref = true;
  int vx = 0, vy = 0;  // luma pixels per frame (even unless odd_pans)
  const int spr = P.slices_per_row;
  const int slice_mbs = spr > 0 ? (mbw + spr - 1) / spr : mbw * mbh;
  std::vector<uint8_t> sample;

  for (int64_t f = 0; f < ck->nf; ++f) {
    const int64_t gf = ck->f0 + f;  // frame index in the whole stream
    const bool cut = (f == 0) || (f == next_cut);
    if (f == next_cut) next_cut = f + scene_len();
    if (cut && gf > 0) ck->cuts.push_back(gf);
    if (f % P.fps_num == 0 || cut) {  // new velocity about once a second
      if (odd_pans) {
        const int m = P.max_motion;
        vx = static_cast<int>(rng.below(2 * m + 1)) - m;
        vy = static_cast<int>(rng.below(2 * m + 1)) - m;
      } else {
        const int m = P.max_motion / 2;
        vx = 2 * (static_cast<int>(rng.below(2 * m + 1)) - m);
        vy = 2 * (static_cast<int>(rng.below(2 * m + 1)) - m);
      }
      if (rng.below(4) == 0) vx = vy = 0;  // static stretches -> P_Skip runs
    }
    const bool idr = cut || since_idr >= gop_max;
    const bool nonref_i = idr && !cut && nonref_refresh;
    if (prev_was_ref) std::swap(cur, ref);  // ref = the latest reference reconstruction
    if (cut) {
      fill_texture(cur, tex_rng, (P.edge_cases & 1) != 0);
    } else {
      // refresh IDR: the panned previous picture re-coded as I_PCM; P picture:
      // every macroblock predicts with the frame's pan (sparkles overwrite
      // theirs below)
      mc_frame(ref, cur, 4 * vx, 4 * vy);
    }
    sample.clear();
    if (idr) {
      frame_num = nonref_i ? (frame_num + 1) & 0xffff : 0;
      for (int first = 0; first < mbw * mbh;) {
        const int row_end = (spr > 0) ? ((first / mbw) + 1) * mbw : mbw * mbh;
        const int last = std::min(first + slice_mbs, row_end);
        BitWriter bw;
        bw.ue(static_cast<uint32_t>(first));  // first_mb_in_slice
        bw.ue(7);                             // slice_type: I (all slices)
        bw.ue(0);                             // pic_parameter_set_id
        bw.u(16, static_cast<uint32_t>(frame_num));
        if (!nonref_i) {
          bw.ue(static_cast<uint32_t>(idr_pic_id));
          bw.u(1, 0);                         // no_output_of_prior_pics_flag
          bw.u(1, 0);                         // long_term_reference_flag
        }                                     // (nal_ref_idc 0: no dec_ref_pic_marking)
        qp_dbk(bw);
        for (int a = first; a < last; ++a) {
          bw.ue(25);  // mb_type I_PCM
          put_pcm(bw, cur, a % mbw, a / mbw);
          mbinfo[size_t(a)] = MbInfo{true, 0, 0};
        }
        bw.trailing();
        append_nal(sample, nonref_i ? 0x01 : 0x65, bw.data());  // non-ref non-IDR / nal_ref_idc 3 IDR
        first = last;
      }
      if (!nonref_i) {
        idr_pic_id ^= 1;
        ++ck->n_idr;
      }
      since_idr = 1;
    } else {
      // a non-reference picture does not advance frame_num (7.4.3)
      if (prev_was_ref) frame_num = (frame_num + 1) & 0xffff;
      // decide macroblocks, reconstruct, then write slices
      for (int first = 0; first < mbw * mbh;) {
        const int row_end = (spr > 0) ? ((first / mbw) + 1) * mbw : mbw * mbh;
        const int last = std::min(first + slice_mbs, row_end);
        MvPred pred{&mbinfo, mbw, first};
        BitWriter bw;
        bw.ue(static_cast<uint32_t>(first));
        bw.ue(5);                             // slice_type: P (all slices)
        bw.ue(0);
        bw.u(16, static_cast<uint32_t>(frame_num));
        bw.u(1, 0);                           // num_ref_idx_active_override_flag
        bw.u(1, 0);                           // ref_pic_list_modification_flag_l0
        bw.u(1, 0);                           // adaptive_ref_pic_marking_mode_flag
        qp_dbk(bw);
        uint32_t skip_run = 0;
        for (int a = first; a < last; ++a) {
          const int mx = a % mbw, my = a / mbw;
          const bool sparkle = rng.below(256) == 0;
          if (sparkle) {
            bw.ue(skip_run);
            skip_run = 0;
            bw.ue(30);  // I_PCM in a P slice (5 + 25)
            fill_sparkle(cur, mx, my, rng);
            put_pcm(bw, cur, mx, my);
            mbinfo[size_t(a)] = MbInfo{true, 0, 0};
            continue;
          }
          const int mvx = 4 * vx, mvy = 4 * vy;
          int sx, sy;
          pred.pskip(a, &sx, &sy);
          if (sx == mvx && sy == mvy) {
            ++skip_run;
          } else {
            int px, py;
            pred.pred16x16(a, &px, &py);
            bw.ue(skip_run);
            skip_run = 0;
            bw.ue(0);  // P_L0_16x16
            bw.se(mvx - px);
            bw.se(mvy - py);
            bw.ue(0);  // coded_block_pattern 0 (inter mapping codeNum 0)
          }
          mbinfo[size_t(a)] = MbInfo{false, mvx, mvy};  // samples: mc_frame above
        }
        if (skip_run) bw.ue(skip_run);
        bw.trailing();
        // edge case bit 2: the last picture loses the slice holding macroblock
        // row 1 (a decoder must report the macroblocks as missing)
        const bool drop = (P.edge_cases & 4) && gf == P.n_frames - 1 && first <= mbw && mbw < last;
        if (!drop) append_nal(sample, 0x41, bw.data());  // nal_ref_idc 2, non-IDR
        first = last;
      }
      ++since_idr;
    }
    if (P.hash_frames) {  // display-size NV12 of the reconstruction
      uint64_t h = 0, j = 0;
      for (int yy = 0; yy < P.height; ++yy)
        for (int xx = 0; xx < P.width; ++xx, ++j)
          h += uint64_t(cur.y[size_t(yy) * cw + xx]) * ((j % 65521) + 1);
      for (int yy = 0; yy < P.height / 2; ++yy)
        for (int xx = 0; xx < P.width / 2; ++xx) {
          h += uint64_t(cur.u[size_t(yy) * (cw / 2) + xx]) * ((j % 65521) + 1);
          ++j;
          h += uint64_t(cur.v[size_t(yy) * (cw / 2) + xx]) * ((j % 65521) + 1);
          ++j;
        }
      ck->recon_hash += h * uint64_t(gf + 1);
    }
    prev_was_ref = !nonref_i;
    ck->data.insert(ck->data.end(), sample.begin(), sample.end());
    ck->size.push_back(static_cast<uint32_t>(sample.size()));
    ck->sync.push_back(idr && !nonref_i ? 1 : 0);
  }
}

}  // namespace
}  // namespace vts

extern "C" int vts_synth_write(const char *path, const vts_synth_params *prm,
                               vts_synth_info *info, int64_t *cut_frames, int64_t cap) {
  clear_error();
  if (!path || !prm) return fail(VTS_E_INVALID, "NULL argument");
  const vts_synth_params &P = *prm;
  if (P.width < 16 || P.height < 16 || (P.width & 1) || (P.height & 1) ||
      P.width > 8192 || P.height > 8192)
    return fail(VTS_E_INVALID, "bad size %dx%d", P.width, P.height);
  if (P.fps_num <= 0 || P.fps_den <= 0 || P.n_frames <= 0)
    return fail(VTS_E_INVALID, "bad frame rate or frame count");
  const bool odd_pans = (P.edge_cases & 2) != 0;
  if (P.coding != 0 && P.coding != 1) return fail(VTS_E_INVALID, "coding must be 0 or 1");
  if (P.max_motion < 0 || ((P.max_motion & 1) && !odd_pans && P.coding == 0) || P.max_motion > 64)
    return fail(VTS_E_INVALID, "max_motion must be even, 0..64 (odd needs edge_cases bit 1)");
  const int mbw = (P.width + 15) / 16, mbh = (P.height + 15) / 16;
  const int cw = mbw * 16, ch = mbh * 16;
  const double fps = double(P.fps_num) / P.fps_den;
  const int level = h264_pick_level(mbw * mbh, mbw * mbh * fps);
  std::vector<uint8_t> sps, pps;
  if (P.coding == 1) make_sps_pps_full(P, level, &sps, &pps);
  else make_sps_pps(mbw, mbh, cw - P.width, ch - P.height, level, &sps, &pps, (P.edge_cases & 512) ? 12 : 0);

  Mp4Writer mw;
  std::string e = mw.open(path);
  if (!e.empty()) return fail(VTS_E_IO, "%s", e.c_str());

  // Chunks of frames coded independently on host threads (auto: one per 18 000
  // frames, i.e. 10 min at 30 fps), then written in order.
  // (full syntax: one run per 1 800 frames; its writer is ~10x slower per frame)
  const int64_t per_chunk = P.coding == 1 ? 1800 : 18000;
  int64_t n_chunks = P.chunks > 0 ? P.chunks : (P.n_frames + per_chunk - 1) / per_chunk;
  n_chunks = std::max<int64_t>(1, std::min<int64_t>(n_chunks, std::min<int64_t>(P.n_frames, 16384)));
  std::vector<SynthChunk> chunks(static_cast<size_t>(n_chunks));
  for (int64_t k = 0; k < n_chunks; ++k) {
    SynthChunk &c = chunks[static_cast<size_t>(k)];
    c.f0 = P.n_frames * k / n_chunks;
    c.nf = P.n_frames * (k + 1) / n_chunks - c.f0;
    c.seed = P.seed + static_cast<uint64_t>(k) * 0xd1b54a32d192ed03ull;
    c.idr_id_base = static_cast<int>(2 * k);
  }
  {
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int64_t nthreads = std::min<int64_t>(n_chunks, std::min<unsigned>(hw, 16u));
    std::atomic<int64_t> next{0};
    auto worker = [&]() {
      for (int64_t k; (k = next.fetch_add(1)) < n_chunks;) {
        SynthChunk *ck = &chunks[static_cast<size_t>(k)];
        if (P.coding == 1) encode_chunk_full(P, ck);
        else encode_chunk(P, ck);
      }
    };
    std::vector<std::thread> pool;
    for (int64_t t = 1; t < nthreads; ++t) pool.emplace_back(worker);
    worker();
    for (std::thread &t : pool) t.join();
  }
  int64_t n_idr = 0, n_cuts = 0;
  uint64_t recon_hash = 0;
  for (const SynthChunk &c : chunks)
    if (!c.error.empty()) return fail(VTS_E_INVALID, "%s", c.error.c_str());
  for (const SynthChunk &c : chunks) {
    size_t pos = 0;
    for (size_t i = 0; i < c.size.size(); ++i) {
      e = mw.add_sample(c.data.data() + pos, c.size[i], c.sync[i] != 0, c.cts.empty() ? 0u : c.cts[i]);
      if (!e.empty()) return fail(VTS_E_IO, "%s", e.c_str());
      pos += c.size[i];
    }
    for (int64_t cf : c.cuts) {
      if (cut_frames && n_cuts < cap) cut_frames[n_cuts] = cf;
      ++n_cuts;
    }
    n_idr += c.n_idr;
    recon_hash += c.recon_hash;
  }
  const int64_t ts = int64_t(P.fps_num) * 1000;
  e = mw.finish(P.width, P.height, ts, int64_t(P.fps_den) * 1000, sps, pps);
  if (!e.empty()) return fail(VTS_E_IO, "%s", e.c_str());
  if (info) {
    info->bytes_written = mw.bytes_written();
    info->n_idr = n_idr;
    info->n_cuts = n_cuts;
    info->timescale = ts;
    info->recon_hash = recon_hash;
  }
  return VTS_OK;
}
