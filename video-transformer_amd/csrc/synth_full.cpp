// synth_full.cpp — synthetic H.264 streams with the full CAVLC I/P syntax
// (vts_synth_params.coding = 1): the input the general device decoder
// (decode_full.hip) is tested and benchmarked on.
//
// The writer makes syntax decisions from a seeded PCG32 stream and codes them
// exactly; it never reconstructs pixels (the decoders define the pictures).
// What it must know to write valid syntax it derives the way a decoder does:
// neighbour availability (6.4.8 / 6.4.12), Intra_4x4 mode prediction
// (8.3.1.1), the nC context of every coeff_token (9.2.1) and motion vector
// prediction (8.4.1.3, P_Skip 8.4.1.1), so that motion vectors land on the
// pan it wants and intra modes only use available samples.
//
// Per picture: IDR at scene cuts and every gop_max seconds; P pictures with
// ~1/10 non-reference; up to 3 reference frames (sliding window), an active
// count chosen per picture (num_ref_idx_active_override) and an occasional
// ref_pic_list_modification; frame_num wraps at 16.  Per slice: QP, the
// deblocking filter (idc 0 mostly, 2 or 1 sometimes, random offsets).  Per
// macroblock (P): P_Skip ~45%, P_L0_16x16 / 16x8 / 8x16 / P_8x8 (sub 8x8 / 8x4
// / 4x8 / 4x4) / P_8x8ref0 with quarter-sample motion around the pan,
// intra ~8%; (I): Intra_4x4 ~60% with random valid modes, Intra_16x16 ~38%,
// I_PCM ~1%.  Residuals: random coded_block_pattern, mb_qp_delta, 4x4 blocks
// of 0..16 coefficients mostly +-1 with escapes up to |2000|.
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "bitstream.h"
#include "common.h"
#include "h264.h"
#include "h264_tables.h"
#include "synth.h"

namespace vts {
namespace {

using namespace h264;

constexpr int kLog2MaxFrameNum = 4;  // frame_num wraps at 16: exercises FrameNumWrap
constexpr int kMaxRefs = 3;
constexpr int kPpsRefDefault = 2;    // num_ref_idx_l0_default_active

struct GMb {
  int type = 0;   // 0 inter, 1 I_NxN, 2 I_16x16, 3 I_PCM, 4 P_Skip
  int slice = -1;
  int i4[16];     // Intra4x4PredMode, raster 4x4 blocks
  int nz[16];     // total_coeff, raster luma 4x4 blocks
  int nzc[2][4];  // chroma AC total_coeff
  int ref[16];
  int mv[16][2];
};

struct Loc {
  int mb = -1, xw = 0, yw = 0;
};

inline int imin(int a, int b) { return a < b ? a : b; }
inline int median3(int a, int b, int c) { return std::max(std::min(a, b), std::min(std::max(a, b), c)); }

class FullWriter {
 public:
  FullWriter(const vts_synth_params &P, SynthChunk *ck)
      : P_(P), ck_(ck), rng_(ck->seed, 0xf011), mbw_((P.width + 15) / 16), mbh_((P.height + 15) / 16) {
    nmb_ = mbw_ * mbh_;
    mb_.resize(static_cast<size_t>(nmb_));
    cip_ = (P.edge_cases & 16) != 0;
  }
  void run();

 private:
  const vts_synth_params &P_;
  SynthChunk *ck_;
  Pcg32 rng_;
  int mbw_, mbh_, nmb_;
  bool cip_;
  std::vector<GMb> mb_;
  BitWriter *bw_ = nullptr;
  int nref_ = 0;      // active references of the current P slice
  int qp_ = 26;       // QPY of the previous macroblock (mb_qp_delta base)

  bool intra(int n) const { return mb_[n].type >= 1 && mb_[n].type <= 3; }
  // 6.4.12 with 6.4.8 availability (same slice, lower address)
  Loc loc(int cur, int xN, int yN, int maxW) const {
    Loc r;
    const int mx = cur % mbw_;
    int n = -1;
    if (yN > maxW - 1) return r;
    if (xN < 0 && yN < 0) n = mx > 0 ? cur - mbw_ - 1 : -1;
    else if (xN < 0) n = mx > 0 ? cur - 1 : -1;
    else if (xN < maxW && yN < 0) n = cur - mbw_;
    else if (xN < maxW) n = cur;
    else if (yN < 0) n = mx < mbw_ - 1 ? cur - mbw_ + 1 : -1;
    else return r;
    if (n < 0 || n >= nmb_) return r;
    if (n != cur && (n > cur || mb_[n].slice != mb_[cur].slice)) return r;
    r.mb = n;
    r.xw = (xN + maxW) % maxW;
    r.yw = (yN + maxW) % maxW;
    return r;
  }
  bool intra_ok(int n) const { return n >= 0 && (!cip_ || intra(n)); }

  int nc(int cur, int bx, int by, bool chroma, int plane) const {
    const int maxW = chroma ? 8 : 16;
    const Loc a = loc(cur, bx * 4 - 1, by * 4, maxW), b = loc(cur, bx * 4, by * 4 - 1, maxW);
    auto val = [&](const Loc &l) {
      const GMb &m = mb_[l.mb];
      if (m.type == 4) return 0;
      if (m.type == 3) return 16;
      return chroma ? m.nzc[plane][(l.yw / 4) * 2 + l.xw / 4] : m.nz[(l.yw / 4) * 4 + l.xw / 4];
    };
    if (a.mb >= 0 && b.mb >= 0) return (val(a) + val(b) + 1) >> 1;
    if (a.mb >= 0) return val(a);
    if (b.mb >= 0) return val(b);
    return 0;
  }

  // --- motion vector prediction (8.4.1.3)
  struct Nb {
    bool avail = false;
    int ref = -1, mvx = 0, mvy = 0;
  };
  Nb nbmv(int cur, int xN, int yN, int done) const {
    Nb r;
    const Loc l = loc(cur, xN, yN, 16);
    if (l.mb < 0) return r;
    const int blk = (l.yw / 4) * 4 + l.xw / 4;
    if (l.mb == cur && !((done >> blk) & 1)) return r;
    r.avail = true;
    const GMb &m = mb_[l.mb];
    if (m.type >= 1 && m.type <= 3) return r;
    r.ref = m.ref[blk];
    r.mvx = m.mv[blk][0];
    r.mvy = m.mv[blk][1];
    return r;
  }
  void mvpred(int cur, int x0, int y0, int w, int h, int ref, int done, int *px, int *py) const {
    Nb a = nbmv(cur, x0 - 1, y0, done), b = nbmv(cur, x0, y0 - 1, done), c = nbmv(cur, x0 + w, y0 - 1, done);
    if (!c.avail) c = nbmv(cur, x0 - 1, y0 - 1, done);
    if (w == 16 && h == 8) {
      if (y0 == 0 && b.ref == ref) { *px = b.mvx; *py = b.mvy; return; }
      if (y0 == 8 && a.ref == ref) { *px = a.mvx; *py = a.mvy; return; }
    } else if (w == 8 && h == 16) {
      if (x0 == 0 && a.ref == ref) { *px = a.mvx; *py = a.mvy; return; }
      if (x0 == 8 && c.ref == ref) { *px = c.mvx; *py = c.mvy; return; }
    }
    if (!b.avail && !c.avail && a.avail) b = c = a;
    const int match = (a.ref == ref) + (b.ref == ref) + (c.ref == ref);
    if (match == 1) {
      const Nb &m = a.ref == ref ? a : (b.ref == ref ? b : c);
      *px = m.mvx;
      *py = m.mvy;
    } else {
      *px = median3(a.mvx, b.mvx, c.mvx);
      *py = median3(a.mvy, b.mvy, c.mvy);
    }
  }
  void skipmv(int cur, int *px, int *py) const {
    *px = *py = 0;
    const Loc la = loc(cur, -1, 0, 16), lb = loc(cur, 0, -1, 16);
    const Nb a = nbmv(cur, -1, 0, 0), b = nbmv(cur, 0, -1, 0);
    if (la.mb < 0 || lb.mb < 0 || (a.ref == 0 && a.mvx == 0 && a.mvy == 0) ||
        (b.ref == 0 && b.mvx == 0 && b.mvy == 0))
      return;
    mvpred(cur, 0, 0, 16, 16, 0, 0, px, py);
  }

  // --- CAVLC residual_block writer (inverse of 9.2); coef in scan order
  int write_block(const int *coef, int start, int end, int maxNum, int nC) {
    BitWriter &bw = *bw_;
    int pos[16], lev[16], tc = 0;
    for (int i = end; i >= start; --i)
      if (coef[i]) {
        pos[tc] = i;
        lev[tc++] = coef[i];
      }
    int t1 = 0;
    while (t1 < tc && t1 < 3 && (lev[t1] == 1 || lev[t1] == -1)) ++t1;
    if (nC >= 8) {
      bw.u(6, tc == 0 ? 3u : static_cast<uint32_t>(((tc - 1) << 2) | t1));
    } else {
      const int col = nC == -1 ? 3 : (nC < 2 ? 0 : (nC < 4 ? 1 : 2));
      bw.u(kCoeffTokenLen[col][tc][t1], kCoeffTokenCode[col][tc][t1]);
    }
    if (tc == 0) return 0;
    for (int i = 0; i < t1; ++i) bw.bit(lev[i] < 0 ? 1 : 0);
    int sl = (tc > 10 && t1 < 3) ? 1 : 0;
    for (int i = t1; i < tc; ++i) {
      const int level = lev[i];
      int code = level > 0 ? 2 * level - 2 : -2 * level - 1;
      if (i == t1 && t1 < 3) code -= 2;
      int prefix, suffix = 0, ssize = 0;
      if (sl == 0) {
        if (code < 14) prefix = code;
        else if (code < 30) { prefix = 14; suffix = code - 14; ssize = 4; }
        else { prefix = 15; suffix = code - 30; ssize = 12; }
      } else {
        if (code < (15 << sl)) { prefix = code >> sl; suffix = code & ((1 << sl) - 1); ssize = sl; }
        else { prefix = 15; suffix = code - (15 << sl); ssize = 12; }
      }
      for (int z = 0; z < prefix; ++z) bw.bit(0);
      bw.bit(1);
      if (ssize) bw.u(ssize, static_cast<uint32_t>(suffix));
      if (sl == 0) sl = 1;
      if (std::abs(level) > (3 << (sl - 1)) && sl < 6) ++sl;
    }
    int zeros = pos[0] - start + 1 - tc;
    if (tc < end - start + 1) {
      if (maxNum == 4) bw.u(kTotalZerosDcLen[tc - 1][zeros], kTotalZerosDcCode[tc - 1][zeros]);
      else bw.u(kTotalZerosLen[tc - 1][zeros], kTotalZerosCode[tc - 1][zeros]);
    }
    for (int i = 0; i < tc - 1 && zeros > 0; ++i) {
      const int run = pos[i] - pos[i + 1] - 1;
      const int row = imin(zeros, 7) - 1;
      bw.u(kRunBeforeLen[row][run], kRunBeforeCode[row][run]);
      zeros -= run;
    }
    return tc;
  }

  int rand_level() {
    const uint32_t r = rng_.below(1000);
    int mag;
    if (r < 600) mag = 1;
    else if (r < 850) mag = 2 + static_cast<int>(rng_.below(2));
    else if (r < 970) mag = 4 + static_cast<int>(rng_.below(12));
    else if (r < 997) mag = 16 + static_cast<int>(rng_.below(285));
    else mag = 300 + static_cast<int>(rng_.below(1701));
    return rng_.below(2) ? -mag : mag;
  }
  // coefficients of one block (scan order, [start, end]); p_zero: all-zero chance
  void rand_block(int *coef, int start, int end, int p_zero_pct) {
    for (int i = 0; i < 16; ++i) coef[i] = 0;
    if (static_cast<int>(rng_.below(100)) < p_zero_pct) return;
    const int n = end - start + 1;
    int tc = 1;
    while (tc < n && rng_.below(100) < 45) ++tc;
    for (int k = 0; k < tc; ++k) {
      // low frequencies first: a geometric pick of the position
      int p = 0;
      while (p < n - 1 && rng_.below(100) < 55) ++p;
      while (coef[start + p] && p < n - 1) ++p;
      if (coef[start + p]) {
        p = 0;
        while (p < n && coef[start + p]) ++p;
        if (p >= n) break;
      }
      coef[start + p] = rand_level();
    }
  }

  void write_residual(int cur, int cbp, bool i16) {
    GMb &m = mb_[cur];
    int coef[16];
    if (i16) {
      rand_block(coef, 0, 15, 30);
      write_block(coef, 0, 15, 16, nc(cur, 0, 0, false, 0));
    }
    for (int k8 = 0; k8 < 4; ++k8)
      for (int k4 = 0; k4 < 4; ++k4) {
        const int blk = k8 * 4 + k4, bx = kBlkX[blk], by = kBlkY[blk];
        if (!((cbp >> k8) & 1)) continue;
        const int n = nc(cur, bx, by, false, 0);
        int tc;
        if (i16) {
          rand_block(coef, 0, 14, 35);
          tc = write_block(coef, 0, 14, 15, n);
        } else {
          rand_block(coef, 0, 15, 30);
          tc = write_block(coef, 0, 15, 16, n);
        }
        m.nz[by * 4 + bx] = tc;
      }
    if (cbp >> 4)
      for (int pl = 0; pl < 2; ++pl) {
        rand_block(coef, 0, 3, 20);
        write_block(coef, 0, 3, 4, -1);
      }
    if ((cbp >> 4) & 2)
      for (int pl = 0; pl < 2; ++pl)
        for (int k = 0; k < 4; ++k) {
          const int n = nc(cur, k & 1, k >> 1, true, pl);
          rand_block(coef, 0, 14, 40);
          m.nzc[pl][k] = write_block(coef, 0, 14, 15, n);
        }
  }

  void write_qp_delta() {
    int dq = 0;
    if (rng_.below(5) == 0) dq = static_cast<int>(rng_.below(9)) - 4;
    if (qp_ + dq < 12 || qp_ + dq > 44) dq = -dq;
    bw_->se(dq);
    qp_ += dq;
  }

  // valid intra modes
  void write_intra(int cur, bool in_p) {
    GMb &m = mb_[cur];
    const uint32_t r = rng_.below(1000);
    const Loc A = loc(cur, -1, 0, 16), B = loc(cur, 0, -1, 16), D = loc(cur, -1, -1, 16);
    const bool la = intra_ok(A.mb), ta = intra_ok(B.mb), ca = intra_ok(D.mb);
    auto chroma_mode = [&]() {
      int modes[4], n = 0;
      modes[n++] = 0;
      if (la) modes[n++] = 1;
      if (ta) modes[n++] = 2;
      if (la && ta && ca) modes[n++] = 3;
      return modes[rng_.below(static_cast<uint32_t>(n))];
    };
    if (r < 10) {  // I_PCM
      m.type = 3;
      bw_->ue(in_p ? 30 : 25);
      bw_->align_zero();
      uint8_t buf[384];
      for (uint8_t &x : buf) x = static_cast<uint8_t>(rng_.below(256));
      bw_->bytes(buf, 384);
      for (int i = 0; i < 16; ++i) m.nz[i] = 16;
      for (int i = 0; i < 4; ++i) m.nzc[0][i] = m.nzc[1][i] = 16;
      return;
    }
    if (r < 600) {  // I_NxN
      m.type = 1;
      bw_->ue(in_p ? 5 : 0);
      for (int k = 0; k < 16; ++k) {
        const int bx = kBlkX[k], by = kBlkY[k];
        // availability of top / left / top-left samples of this block
        auto av = [&](int xN, int yN) {
          const Loc l = loc(cur, xN, yN, 16);
          return intra_ok(l.mb);  // inside the MB: left/top/top-left blocks precede in order
        };
        const bool t = av(bx * 4, by * 4 - 1), l = av(bx * 4 - 1, by * 4), tl = av(bx * 4 - 1, by * 4 - 1);
        int modes[9], n = 0;
        modes[n++] = 2;
        if (t) { modes[n++] = 0; modes[n++] = 3; modes[n++] = 7; }
        if (l) { modes[n++] = 1; modes[n++] = 8; }
        if (t && l && tl) { modes[n++] = 4; modes[n++] = 5; modes[n++] = 6; }
        // predicted mode (8.3.1.1)
        const Loc LA = loc(cur, bx * 4 - 1, by * 4, 16), LB = loc(cur, bx * 4, by * 4 - 1, 16);
        int pred;
        if (LA.mb < 0 || LB.mb < 0 || (cip_ && !intra(LA.mb)) || (cip_ && !intra(LB.mb))) {
          pred = 2;
        } else {
          const GMb &ma = mb_[LA.mb], &mb = mb_[LB.mb];
          const int a = ma.type == 1 ? ma.i4[(LA.yw / 4) * 4 + LA.xw / 4] : 2;
          const int b = mb.type == 1 ? mb.i4[(LB.yw / 4) * 4 + LB.xw / 4] : 2;
          pred = imin(a, b);
        }
        bool pred_ok = false;
        for (int i = 0; i < n; ++i) pred_ok |= modes[i] == pred;
        const int mode = (pred_ok && rng_.below(2)) ? pred : modes[rng_.below(static_cast<uint32_t>(n))];
        if (mode == pred) {
          bw_->bit(1);
        } else {
          bw_->bit(0);
          bw_->u(3, static_cast<uint32_t>(mode < pred ? mode : mode - 1));
        }
        m.i4[by * 4 + bx] = mode;
      }
      bw_->ue(static_cast<uint32_t>(chroma_mode()));
      const int cbp = static_cast<int>(rng_.below(16)) | (static_cast<int>(rng_.below(3)) << 4);
      int code = 0;
      while (kCbpIntra[code] != cbp) ++code;
      bw_->ue(static_cast<uint32_t>(code));
      if (cbp) write_qp_delta();
      write_residual(cur, cbp, false);
      return;
    }
    // I_16x16
    m.type = 2;
    int modes[4], n = 0;
    modes[n++] = 2;
    if (ta) modes[n++] = 0;
    if (la) modes[n++] = 1;
    if (la && ta && ca) modes[n++] = 3;
    const int pm = modes[rng_.below(static_cast<uint32_t>(n))];
    const int cc = static_cast<int>(rng_.below(3)), lum = rng_.below(2) ? 15 : 0;
    bw_->ue(static_cast<uint32_t>((in_p ? 5 : 0) + 1 + pm + 4 * cc + (lum ? 12 : 0)));
    bw_->ue(static_cast<uint32_t>(chroma_mode()));
    write_qp_delta();
    write_residual(cur, (cc << 4) | lum, true);
  }

  void write_inter(int cur, int pan_x, int pan_y) {
    GMb &m = mb_[cur];
    m.type = 0;
    const uint32_t r = rng_.below(1000);
    int mb_type = r < 640 ? 0 : (r < 760 ? 1 : (r < 880 ? 2 : (r < 980 ? 3 : 4)));
    if (mb_type == 4 && nref_ < 1) mb_type = 3;
    bw_->ue(static_cast<uint32_t>(mb_type));
    const int nparts = mb_type == 0 ? 1 : (mb_type <= 2 ? 2 : 4);
    int sub[4] = {0, 0, 0, 0}, refs[4] = {0, 0, 0, 0};
    if (mb_type >= 3)
      for (int k = 0; k < 4; ++k) {
        sub[k] = static_cast<int>(rng_.below(4));
        bw_->ue(static_cast<uint32_t>(sub[k]));
      }
    if (mb_type != 4 && nref_ > 1)
      for (int k = 0; k < nparts; ++k) {
        refs[k] = rng_.below(4) ? 0 : static_cast<int>(rng_.below(static_cast<uint32_t>(nref_)));
        if (nref_ == 2) bw_->bit(refs[k] ? 0 : 1);  // te(v), range 1
        else bw_->ue(static_cast<uint32_t>(refs[k]));
      }
    int done = 0;
    for (int k = 0; k < nparts; ++k) {
      int nsub = 1, pw, ph, x0, y0;
      if (mb_type == 0) { pw = ph = 16; x0 = y0 = 0; }
      else if (mb_type == 1) { pw = 16; ph = 8; x0 = 0; y0 = 8 * k; }
      else if (mb_type == 2) { pw = 8; ph = 16; x0 = 8 * k; y0 = 0; }
      else {
        x0 = 8 * (k & 1);
        y0 = 8 * (k >> 1);
        nsub = sub[k] == 0 ? 1 : (sub[k] == 3 ? 4 : 2);
        pw = (sub[k] == 0 || sub[k] == 1) ? 8 : 4;
        ph = (sub[k] == 0 || sub[k] == 2) ? 8 : 4;
      }
      for (int s = 0; s < nsub; ++s) {
        int sx = x0, sy = y0;
        if (mb_type >= 3) {
          if (sub[k] == 1) sy += 4 * s;
          else if (sub[k] == 2) sx += 4 * s;
          else if (sub[k] == 3) { sx += 4 * (s & 1); sy += 4 * (s >> 1); }
        }
        int px, py;
        mvpred(cur, sx, sy, pw, ph, refs[k], done, &px, &py);
        const int tx = (refs[k] + 1) * pan_x + static_cast<int>(rng_.below(13)) - 6;
        const int ty = (refs[k] + 1) * pan_y + static_cast<int>(rng_.below(13)) - 6;
        bw_->se(tx - px);
        bw_->se(ty - py);
        for (int yy = sy / 4; yy < (sy + ph) / 4; ++yy)
          for (int xx = sx / 4; xx < (sx + pw) / 4; ++xx) {
            const int blk = yy * 4 + xx;
            m.ref[blk] = refs[k];
            m.mv[blk][0] = tx;
            m.mv[blk][1] = ty;
            done |= 1 << blk;
          }
      }
    }
    int cbp = 0;
    for (int k8 = 0; k8 < 4; ++k8)
      if (rng_.below(100) < 35) cbp |= 1 << k8;
    const uint32_t cr = rng_.below(100);
    cbp |= (cr < 60 ? 0 : (cr < 85 ? 1 : 2)) << 4;
    int code = 0;
    while (kCbpInter[code] != cbp) ++code;
    bw_->ue(static_cast<uint32_t>(code));
    if (cbp) write_qp_delta();
    write_residual(cur, cbp, false);
  }

  void reset_mb(int a, int slice) {
    GMb &m = mb_[static_cast<size_t>(a)];
    m = GMb{};
    m.slice = slice;
    for (int i = 0; i < 16; ++i) {
      m.i4[i] = 2;
      m.nz[i] = 0;
      m.ref[i] = -1;
      m.mv[i][0] = m.mv[i][1] = 0;
    }
    for (int i = 0; i < 4; ++i) m.nzc[0][i] = m.nzc[1][i] = 0;
  }

  void write_slice_data(int first, int last, int slice, bool is_p, int pan_x, int pan_y) {
    uint32_t skip_run = 0;
    for (int a = first; a < last; ++a) {
      reset_mb(a, slice);
      if (is_p) {
        const uint32_t r = rng_.below(1000);
        if (r < 450) {  // P_Skip
          GMb &m = mb_[static_cast<size_t>(a)];
          m.type = 4;
          int px, py;
          skipmv(a, &px, &py);
          for (int i = 0; i < 16; ++i) {
            m.ref[i] = 0;
            m.mv[i][0] = px;
            m.mv[i][1] = py;
          }
          ++skip_run;
          continue;
        }
        bw_->ue(skip_run);
        skip_run = 0;
        if (r < 920) write_inter(a, pan_x, pan_y);
        else write_intra(a, true);
      } else {
        write_intra(a, false);
      }
    }
    if (is_p && skip_run) bw_->ue(skip_run);
  }

};

void FullWriter::run() {
  const double fps = double(P_.fps_num) / P_.fps_den;
  const int gop_max = std::max(1, static_cast<int>(P_.gop_max_s * fps));
  auto scene_len = [&]() {
    const double lo = std::max(P_.cut_min_s, 1.0 / fps), hi = std::max(P_.cut_max_s, lo);
    return std::max<int64_t>(1, static_cast<int64_t>((lo + (hi - lo) * rng_.uniform()) * fps + 0.5));
  };
  int64_t next_cut = scene_len(), since_idr = 0;
  int frame_num = 0, prev_ref_fn = 0, refs = 0, idr_id = ck_->idr_id_base;
  bool prev_ref = true;
  int pan_x = 0, pan_y = 0;  // quarter-sample motion per frame
  const int spr = P_.slices_per_row;
  const int slice_mbs = spr > 0 ? (mbw_ + spr - 1) / spr : nmb_;
  std::vector<uint8_t> sample;
  for (int64_t f = 0; f < ck_->nf; ++f) {
    const int64_t gf = ck_->f0 + f;
    const bool cut = f == 0 || f == next_cut;
    if (f == next_cut) next_cut = f + scene_len();
    if (cut && gf > 0) ck_->cuts.push_back(gf);
    if (f % P_.fps_num == 0 || cut) {
      const int m = 4 * P_.max_motion;
      pan_x = static_cast<int>(rng_.below(static_cast<uint32_t>(2 * m + 1))) - m;
      pan_y = static_cast<int>(rng_.below(static_cast<uint32_t>(2 * m + 1))) - m;
      if (rng_.below(4) == 0) pan_x = pan_y = 0;
    }
    const bool idr = cut || since_idr >= gop_max;
    // a non-reference P picture now and then (never two in a row: POC type 2)
    const bool nonref = !idr && prev_ref && rng_.below(10) == 0;
    if (idr) {
      frame_num = 0;
      refs = 0;
    } else {
      frame_num = (prev_ref_fn + 1) & ((1 << kLog2MaxFrameNum) - 1);
    }
    const int slice_type = idr ? (rng_.below(2) ? 7 : 2) : (rng_.below(2) ? 5 : 0);
    const int pic_qp = 20 + static_cast<int>(rng_.below(17));
    const int nref = idr ? 0 : 1 + static_cast<int>(rng_.below(static_cast<uint32_t>(refs)));
    sample.clear();
    int slice = 0;
    for (int first = 0; first < nmb_; ++slice) {
      const int row_end = spr > 0 ? ((first / mbw_) + 1) * mbw_ : nmb_;
      const int last = std::min(first + slice_mbs, row_end);
      BitWriter bw;
      bw_ = &bw;
      bw.ue(static_cast<uint32_t>(first));
      bw.ue(static_cast<uint32_t>(slice_type));
      bw.ue(0);
      bw.u(kLog2MaxFrameNum, static_cast<uint32_t>(frame_num));
      if (idr) bw.ue(static_cast<uint32_t>(idr_id));
      if (!idr) {
        nref_ = nref;
        if (nref != kPpsRefDefault) {
          bw.u(1, 1);
          bw.ue(static_cast<uint32_t>(nref - 1));
        } else {
          bw.u(1, 0);
        }
        // ref_pic_list_modification: now and then move an older reference first
        if (refs >= 2 && rng_.below(20) == 0) {
          bw.u(1, 1);
          const int k = 1 + static_cast<int>(rng_.below(static_cast<uint32_t>(refs - 1)));
          bw.ue(0);                              // subtract from the predicted picNum
          bw.ue(static_cast<uint32_t>(k));       // abs_diff_pic_num_minus1: PicNum = CurrPicNum - 1 - k
          bw.ue(3);
        } else {
          bw.u(1, 0);
        }
      }
      if (!nonref) {  // dec_ref_pic_marking
        if (idr) { bw.u(1, 0); bw.u(1, 0); }
        else bw.u(1, 0);
      }
      qp_ = pic_qp;
      bw.se(pic_qp - 26);
      const uint32_t dr = rng_.below(20);
      const int didc = dr < 16 ? 0 : (dr < 18 ? 2 : 1);
      bw.ue(static_cast<uint32_t>(didc));
      if (didc != 1) {
        bw.se(static_cast<int>(rng_.below(7)) - 3);
        bw.se(static_cast<int>(rng_.below(7)) - 3);
      }
      write_slice_data(first, last, slice, !idr, pan_x, pan_y);
      bw.trailing();
      append_nal(sample, idr ? 0x65 : (nonref ? 0x01 : 0x41), bw.data());
      first = last;
    }
    bw_ = nullptr;
    if (idr) {
      idr_id ^= 1;
      ++ck_->n_idr;
      since_idr = 1;
    } else {
      ++since_idr;
    }
    if (!nonref) {
      refs = std::min(refs + 1, kMaxRefs);
      prev_ref_fn = frame_num;
    }
    prev_ref = !nonref;
    ck_->data.insert(ck_->data.end(), sample.begin(), sample.end());
    ck_->size.push_back(static_cast<uint32_t>(sample.size()));
    ck_->sync.push_back(idr ? 1 : 0);
  }
}

}  // namespace

void encode_chunk_full(const vts_synth_params &P, SynthChunk *ck) {
  FullWriter w(P, ck);
  w.run();
}

// Constrained Baseline SPS / PPS of the full-syntax streams: 3 reference
// frames, frame_num wrapping at 16, POC type 2, deblocking control present,
// two active references by default, chroma QP offset from the seed.
void make_sps_pps_full(const vts_synth_params &P, int level, std::vector<uint8_t> *sps_nal,
                       std::vector<uint8_t> *pps_nal) {
  const int mbw = (P.width + 15) / 16, mbh = (P.height + 15) / 16;
  const int crop_r = mbw * 16 - P.width, crop_b = mbh * 16 - P.height;
  BitWriter s;
  s.u(8, 66);
  s.u(8, 0xC0);
  s.u(8, static_cast<uint32_t>(level));
  s.ue(0);
  s.ue(kLog2MaxFrameNum - 4);
  s.ue(2);
  s.ue(kMaxRefs);
  s.u(1, 0);
  s.ue(static_cast<uint32_t>(mbw - 1));
  s.ue(static_cast<uint32_t>(mbh - 1));
  s.u(1, 1);
  s.u(1, 1);
  if (crop_r || crop_b) {
    s.u(1, 1);
    s.ue(0);
    s.ue(static_cast<uint32_t>(crop_r / 2));
    s.ue(0);
    s.ue(static_cast<uint32_t>(crop_b / 2));
  } else {
    s.u(1, 0);
  }
  s.u(1, 0);
  s.trailing();
  sps_nal->clear();
  sps_nal->push_back(0x67);
  append_ebsp(*sps_nal, s.data().data(), s.data().size());
  BitWriter p;
  p.ue(0);
  p.ue(0);
  p.u(1, 0);                                   // CAVLC
  p.u(1, 0);
  p.ue(0);
  p.ue(kPpsRefDefault - 1);
  p.ue(0);
  p.u(1, 0);
  p.u(2, 0);
  p.se(0);                                     // pic_init_qp 26
  p.se(0);
  p.se(static_cast<int>(P.seed % 5) - 2);      // chroma_qp_index_offset
  p.u(1, 1);                                   // deblocking_filter_control_present_flag
  p.u(1, (P.edge_cases & 16) ? 1 : 0);         // constrained_intra_pred_flag
  p.u(1, 0);
  p.trailing();
  pps_nal->clear();
  pps_nal->push_back(0x68);
  append_ebsp(*pps_nal, p.data().data(), p.data().size());
}

}  // namespace vts
