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
//
// CABAC (edge_cases bit 10, Main / High profile): the same decisions written
// through the arithmetic coder of 9.3.4 with cabac_init_idc 0: every syntax
// element's binarization (9.3.2) and context selection (9.3.3.1), which the
// writer derives from its own neighbour records the way a decoder does
// (mb_skip_flag, mb_type, sub_mb_type, ref_idx, mvd, coded_block_pattern,
// mb_qp_delta, intra modes, coded_block_flag, significance maps, levels,
// end_of_slice_flag, I_PCM with the engine flushed and restarted).  With
// bit 11 (High profile, transform_8x8_mode_flag) Intra_NxN macroblocks are
// Intra_8x8 half the time and inter macroblocks without sub-8x8 partitions
// use the 8x8 transform half the time (8x8 blocks of up to 64 levels).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "bitstream.h"
#include "common.h"
#include "h264.h"
#include "h264_cabac_tables.h"
#include "h264_tables.h"
#include "synth.h"
#include "synth_content.h"
#include "recon_full.h"

namespace vts {
namespace {

using namespace h264;

constexpr int kLog2MaxFrameNum = 4;  // frame_num wraps at 16: exercises FrameNumWrap
constexpr int kMaxRefs = 3;
constexpr int kPpsRefDefault = 2;    // num_ref_idx_l0_default_active

struct GMb {
  int type = 0;   // 0 inter, 1 I_NxN, 2 I_16x16, 3 I_PCM, 4 P_Skip / B_Skip
  int slice = -1;
  int i4[16];     // Intra4x4PredMode, raster 4x4 blocks (Intra8x8PredMode repeated over its 4)
  int nz[16];     // total_coeff, raster luma 4x4 blocks
  int nzc[2][4];  // chroma AC total_coeff
  int ref[2][16];  // refIdxLX per raster 4x4 block (-1: list unused)
  int mv[2][16][2];
  int refd[2][16]; // display index of the picture refIdxLX names (B mode)
  // CABAC context facts (9.3.3.1.1)
  int cbp = 0;        // coded_block_pattern (I_16x16: the one its mb_type implies)
  int cmode = 0;      // intra_chroma_pred_mode
  bool t8 = false;    // transform_size_8x8_flag
  bool d16 = false;   // B_Skip / B_Direct_16x16
  int dmask = 0;      // 8x8 quarters predicted in direct mode
  uint32_t cbf = 0;   // coded_block_flag: bit 0 Intra16x16 DC, 1 + raster luma 4x4,
                      // 17 + plane chroma DC, 19 + 4 * plane + raster chroma AC
  int mvda[2][16][2]; // |mvd_lX| per raster 4x4 block (0: none written)
};

// CABAC arithmetic encoder (9.3.4) writing into a BitWriter; context
// variables initialised per 9.3.1.1 from the I column or cabac_init_idc 0.
const int8_t kInitI[VTS_CABAC_NCTX][2] = VTS_CABAC_INIT_I_DATA;
const int8_t kInitP[VTS_CABAC_NCTX][2] = VTS_CABAC_INIT_P0_DATA;
const uint8_t kRangeLps[64][4] = VTS_CABAC_RANGE_LPS_DATA;
const uint8_t kTransLps[64] = VTS_CABAC_TRANS_LPS_DATA;
const uint8_t kSig8[63] = VTS_SIG8x8_DATA;
const uint8_t kLast8[63] = VTS_LAST8x8_DATA;

class CabacEnc {
 public:
  void init(BitWriter *bw, bool is_i, int qp) {  // 9.3.1.1 + 9.3.4.1
    bw_ = bw;
    const int q = std::clamp(qp, 0, 51);
    for (int i = 0; i < VTS_CABAC_NCTX; ++i) {
      const int m = is_i ? kInitI[i][0] : kInitP[i][0], n = is_i ? kInitI[i][1] : kInitP[i][1];
      const int pre = std::clamp(((m * q) >> 4) + n, 1, 126);
      st_[i] = static_cast<uint8_t>(pre <= 63 ? (63 - pre) << 1 : ((pre - 64) << 1) | 1);
    }
    start();
  }
  void start() {  // InitEncoder
    low_ = 0;
    range_ = 510;
    first_ = true;
    outstanding_ = 0;
  }
  void enc(int ctx, int bin) {  // EncodeDecision
    const int s = st_[ctx], ps = s >> 1, mps = s & 1;
    const uint32_t lps = kRangeLps[ps][(range_ >> 6) & 3];
    range_ -= lps;
    if (bin != mps) {
      low_ += range_;
      range_ = lps;
      st_[ctx] = static_cast<uint8_t>((kTransLps[ps] << 1) | (ps == 0 ? 1 - mps : mps));
    } else {
      st_[ctx] = static_cast<uint8_t>((std::min(ps + 1, 62) << 1) | mps);
    }
    renorm();
  }
  void bypass(int bin) {  // EncodeBypass
    low_ <<= 1;
    if (bin) low_ += range_;
    if (low_ >= 1024) {
      put(1);
      low_ -= 1024;
    } else if (low_ < 512) {
      put(0);
    } else {
      low_ -= 512;
      ++outstanding_;
    }
  }
  void term(int bin) {  // EncodeTerminate; 1 flushes (the last bit written is the stop / final bit)
    range_ -= 2;
    if (bin) {
      low_ += range_;
      range_ = 2;  // EncodeFlush
      renorm();
      put((low_ >> 9) & 1);
      bw_->bit((low_ >> 8) & 1);
      bw_->bit(1);
    } else {
      renorm();
    }
  }
  void ueg(int v, int k) {  // k-th order Exp-Golomb suffix, bypass (9.3.2.3)
    while (v >= (1 << k)) {
      bypass(1);
      v -= 1 << k;
      ++k;
    }
    bypass(0);
    while (k--) bypass((v >> k) & 1);
  }

 private:
  void put(int b) {
    if (first_) first_ = false;
    else bw_->bit(static_cast<uint32_t>(b));
    for (; outstanding_ > 0; --outstanding_) bw_->bit(static_cast<uint32_t>(1 - b));
  }
  void renorm() {
    while (range_ < 256) {
      if (low_ < 256) {
        put(0);
      } else if (low_ >= 512) {
        low_ -= 512;
        put(1);
      } else {
        low_ -= 256;
        ++outstanding_;
      }
      range_ <<= 1;
      low_ <<= 1;
    }
  }
  BitWriter *bw_ = nullptr;
  uint32_t low_ = 0, range_ = 510;
  bool first_ = true;
  int outstanding_ = 0;
  uint8_t st_[VTS_CABAC_NCTX];
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
    cabac_ = (P.edge_cases & 1024) != 0;
    t8mode_ = cabac_ && (P.edge_cases & 2048) != 0;
    content_ = (P.edge_cases & 16384) != 0;
    // the PPS's chroma QP offsets (make_sps_pps_full)
    cqp_[0] = static_cast<int>(P.seed % 5) - 2;
    cqp_[1] = (t8mode_ || (P.edge_cases & 8192)) ? static_cast<int>(P.seed % 3) - 1 : cqp_[0];
    tex_rng_ = Pcg32(ck->seed ^ 0x9e3779b97f4a7c15ull, 0x7e47);
  }
  void run();
  void run_b();

 private:
  const vts_synth_params &P_;
  SynthChunk *ck_;
  Pcg32 rng_;
  int mbw_, mbh_, nmb_;
  bool cip_;
  bool cabac_ = false, t8mode_ = false;
  CabacEnc cab_;
  bool qpd_prev_ = false, qpd_cur_ = false;  // mb_qp_delta != 0 of the previous / current macroblock
  int cref_[2][4];                          // ref_idx_lX of the current macroblock's quarters written so far
  int cmvd_[2][16][2];                      // |mvd_lX| of the current macroblock written so far
  std::vector<GMb> mb_;
  BitWriter *bw_ = nullptr;
  int nref_ = 0;      // active references of the current P slice
  int qp_ = 26;       // QPY of the previous macroblock (mb_qp_delta base)
  // B mode (edge_cases bit 5): display index of each RefPicListX entry, the
  // current picture's display index / POC, and the pictures' motion fields
  bool bmode_ = false;
  int weighted_ = 0;  // weighted_bipred_idc
  int lst_[2][33] = {};
  int nlst_[2] = {0, 0};
  int cur_d_ = 0, cur_poc_ = 0;
  bool spatial_ = true;
  struct RefPic {
    int d, poc, fn;
    std::vector<GMb> mbs;
    std::vector<uint8_t> rec;  // content mode: the deblocked reconstruction (NV12)
  };
  std::vector<RefPic> dpb_;
  const RefPic *col_ = nullptr;   // RefPicList1[0]
  const RefPic *pic_of(int d) const {
    for (const RefPic &r : dpb_)
      if (r.d == d) return &r;
    return nullptr;
  }

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
  Nb nbmv(int cur, int xN, int yN, int done, int lx = 0) const {
    Nb r;
    const Loc l = loc(cur, xN, yN, 16);
    if (l.mb < 0) return r;
    const int blk = (l.yw / 4) * 4 + l.xw / 4;
    if (l.mb == cur && !((done >> blk) & 1)) return r;
    r.avail = true;
    const GMb &m = mb_[l.mb];
    if (m.type >= 1 && m.type <= 3) return r;
    r.ref = m.ref[lx][blk];
    if (r.ref < 0) return r;
    r.mvx = m.mv[lx][blk][0];
    r.mvy = m.mv[lx][blk][1];
    return r;
  }
  void mvpred(int cur, int x0, int y0, int w, int h, int ref, int done, int *px, int *py, int l = 0) const {
    Nb a = nbmv(cur, x0 - 1, y0, done, l), b = nbmv(cur, x0, y0 - 1, done, l), c = nbmv(cur, x0 + w, y0 - 1, done, l);
    if (!c.avail) c = nbmv(cur, x0 - 1, y0 - 1, done, l);
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

  // CABAC residual_block (7.3.5.3.3, 9.3.2.3 / 9.3.3.1.3): coef[0, maxNum) in
  // scan order; cat = ctxBlockCat (5: an 8x8 block, which has no
  // coded_block_flag and at least one non-zero level).  Returns the count of
  // non-zero levels.
  int cab_block(const int *coef, int maxNum, int cat, int cbf_inc) {
    static const int kCbfOff[5] = {0, 4, 8, 12, 16}, kSigOff[5] = {0, 15, 29, 44, 47};
    static const int kAbsOff[5] = {0, 10, 20, 30, 39};
    int last = -1, n = 0;
    for (int i = 0; i < maxNum; ++i)
      if (coef[i]) {
        last = i;
        ++n;
      }
    if (cat != 5) {
      cab_.enc(85 + kCbfOff[cat] + cbf_inc, last >= 0);
      if (last < 0) return 0;
    }
    for (int i = 0; i < maxNum - 1; ++i) {
      const int inc = cat == 3 ? std::min(i, 2) : i;
      const int sig = coef[i] != 0;
      cab_.enc(cat == 5 ? 402 + kSig8[i] : 105 + kSigOff[cat] + inc, sig);
      if (sig) {
        cab_.enc(cat == 5 ? 417 + kLast8[i] : 166 + kSigOff[cat] + inc, i == last);
        if (i == last) break;
      }
    }
    int eq1 = 0, gt1 = 0;
    const int base = cat == 5 ? 426 : 227 + kAbsOff[cat];
    for (int i = last; i >= 0; --i) {
      if (!coef[i]) continue;
      const int a = std::abs(coef[i]) - 1;  // coeff_abs_level_minus1: TU prefix cMax 14 + UEG0
      cab_.enc(base + (gt1 ? 0 : std::min(4, 1 + eq1)), a > 0);
      if (a > 0) {
        const int inc = 5 + std::min(4 - (cat == 3 ? 1 : 0), gt1);
        for (int k = 1; k < 14; ++k) {
          cab_.enc(base + inc, k < a);
          if (k >= a) break;
        }
        if (a >= 14) cab_.ueg(a - 14, 0);
      }
      cab_.bypass(coef[i] < 0);
      if (a == 0) ++eq1;
      else ++gt1;
    }
    return n;
  }
  // condTermFlagN of coded_block_flag (9.3.3.1.1.9); n: the neighbour
  // macroblock (-1 unavailable), tb: transBlockN is available
  int cbf_cond(int n, bool intra, bool tb, int bit) const {
    if (n < 0) return intra ? 1 : 0;
    const GMb &m = mb_[static_cast<size_t>(n)];
    if (m.type == 3) return 1;
    if (!tb || m.type == 4) return 0;
    return static_cast<int>((m.cbf >> bit) & 1u);
  }
  int cbf_inc_dc(int cur) const {
    const int a = nb_a(cur), b = nb_b(cur);
    return cbf_cond(a, true, a >= 0 && mb_[static_cast<size_t>(a)].type == 2, 0) +
           2 * cbf_cond(b, true, b >= 0 && mb_[static_cast<size_t>(b)].type == 2, 0);
  }
  int cbf_inc_luma(int cur, int bx, int by, bool intra) const {
    int inc = 0;
    for (int nb = 0; nb < 2; ++nb) {
      const Loc l = loc(cur, nb ? bx * 4 : bx * 4 - 1, nb ? by * 4 - 1 : by * 4, 16);
      bool tb = false;
      int bit = 0;
      if (l.mb >= 0) {
        tb = (mb_[static_cast<size_t>(l.mb)].cbp >> ((l.yw / 8) * 2 + l.xw / 8)) & 1;
        bit = 1 + (l.yw / 4) * 4 + l.xw / 4;
      }
      inc += cbf_cond(l.mb, intra, tb, bit) << nb;
    }
    return inc;
  }
  int cbf_inc_chroma(int cur, int pl, int blk, bool dc, bool intra) const {
    const int x = dc ? 0 : (blk & 1) * 4, y = dc ? 0 : (blk >> 1) * 4;
    int inc = 0;
    for (int nb = 0; nb < 2; ++nb) {
      const Loc l = loc(cur, nb ? x : x - 1, nb ? y - 1 : y, 8);
      bool tb = false;
      int bit = 0;
      if (l.mb >= 0) {
        const int cc = mb_[static_cast<size_t>(l.mb)].cbp >> 4;
        tb = dc ? cc != 0 : cc == 2;
        bit = dc ? 17 + pl : 19 + 4 * pl + (l.yw / 4) * 2 + l.xw / 4;
      }
      inc += cbf_cond(l.mb, intra, tb, bit) << nb;
    }
    return inc;
  }
  // 64 levels of an 8x8 block in scan order, at least one non-zero
  void rand_block8(int *coef) {
    for (int i = 0; i < 64; ++i) coef[i] = 0;
    int tc = 1;
    while (tc < 64 && rng_.below(100) < 70) ++tc;
    for (int k = 0; k < tc; ++k) {
      int p = 0;
      while (p < 63 && rng_.below(100) < 80) ++p;
      while (p < 63 && coef[p]) ++p;
      if (coef[p]) {
        p = 0;
        while (p < 64 && coef[p]) ++p;
        if (p >= 64) break;
      }
      coef[p] = rand_level();
    }
  }

  // L: the content mode's levels (else random ones)
  void write_residual(int cur, int cbp, bool i16, const content::Levels *L = nullptr) {
    GMb &m = mb_[static_cast<size_t>(cur)];
    const bool intra = m.type == 1 || m.type == 2;
    int coef[64];
    auto put = [&](const int *src, int n) { std::memcpy(coef, src, sizeof(int) * static_cast<size_t>(n)); };
    if (i16) {
      if (L) put(L->dc16, 16);
      else rand_block(coef, 0, 15, 30);
      if (cabac_) {
        if (cab_block(coef, 16, 0, cbf_inc_dc(cur))) m.cbf |= 1u;
      } else {
        write_block(coef, 0, 15, 16, nc(cur, 0, 0, false, 0));
      }
    }
    for (int k8 = 0; k8 < 4; ++k8) {
      if (!((cbp >> k8) & 1)) continue;
      if (m.t8) {  // CABAC only (the decoders refuse CAVLC 8x8 streams)
        if (L) put(L->l8[k8], 64);
        else rand_block8(coef);
        const int tc = cab_block(coef, 64, 5, 0);
        for (int j = 0; j < 4; ++j) {
          const int blk = k8 * 4 + j, r = kBlkY[blk] * 4 + kBlkX[blk];
          m.nz[r] = tc;
          m.cbf |= 1u << (1 + r);
        }
        continue;
      }
      for (int k4 = 0; k4 < 4; ++k4) {
        const int blk = k8 * 4 + k4, bx = kBlkX[blk], by = kBlkY[blk], r = by * 4 + bx;
        int tc;
        if (L) put(L->l4[r], 16);
        if (cabac_) {
          if (!L) {
            if (i16) rand_block(coef, 0, 14, 35);
            else rand_block(coef, 0, 15, 30);
          }
          tc = cab_block(coef, i16 ? 15 : 16, i16 ? 1 : 2, cbf_inc_luma(cur, bx, by, intra));
        } else {
          const int n = nc(cur, bx, by, false, 0);
          if (i16) {
            if (!L) rand_block(coef, 0, 14, 35);
            tc = write_block(coef, 0, 14, 15, n);
          } else {
            if (!L) rand_block(coef, 0, 15, 30);
            tc = write_block(coef, 0, 15, 16, n);
          }
        }
        m.nz[r] = tc;
        if (tc) m.cbf |= 1u << (1 + r);
      }
    }
    if (cbp >> 4)
      for (int pl = 0; pl < 2; ++pl) {
        if (L) {
          for (int i = 0; i < 16; ++i) coef[i] = i < 4 ? L->cdc[pl][i] : 0;
        } else {
          rand_block(coef, 0, 3, 20);
        }
        if (cabac_) {
          if (cab_block(coef, 4, 3, cbf_inc_chroma(cur, pl, 0, true, intra))) m.cbf |= 1u << (17 + pl);
        } else {
          write_block(coef, 0, 3, 4, -1);
        }
      }
    if ((cbp >> 4) & 2)
      for (int pl = 0; pl < 2; ++pl)
        for (int k = 0; k < 4; ++k) {
          int tc;
          if (L) put(L->cac[pl][k], 15);
          if (cabac_) {
            if (!L) rand_block(coef, 0, 14, 40);
            tc = cab_block(coef, 15, 4, cbf_inc_chroma(cur, pl, k, false, intra));
          } else {
            const int n = nc(cur, k & 1, k >> 1, true, pl);
            if (!L) rand_block(coef, 0, 14, 40);
            tc = write_block(coef, 0, 14, 15, n);
          }
          m.nzc[pl][k] = tc;
          if (tc) m.cbf |= 1u << (19 + 4 * pl + k);
        }
  }

  void write_qp_delta() {
    int dq = 0;
    if (!content_ && rng_.below(5) == 0) dq = static_cast<int>(rng_.below(9)) - 4;
    if (qp_ + dq < 12 || qp_ + dq > 44) dq = -dq;
    if (cabac_) {  // U binarization of the se() mapping; bin 0's context: the previous macroblock's delta
      const int k = dq > 0 ? 2 * dq - 1 : -2 * dq;
      cab_.enc(60 + (qpd_prev_ ? 1 : 0), k > 0);
      if (k > 0) {
        cab_.enc(62, k > 1);
        if (k > 1) {
          for (int i = 2; i < k; ++i) cab_.enc(63, 1);
          cab_.enc(63, 0);
        }
      }
      qpd_cur_ = dq != 0;
    } else {
      bw_->se(dq);
    }
    qp_ += dq;
  }

  // ------------------------------------------- syntax elements (CAVLC / CABAC)
  int nb_a(int cur) const { return loc(cur, -1, 0, 16).mb; }
  int nb_b(int cur) const { return loc(cur, 0, -1, 16).mb; }
  // mb_type of an intra macroblock: v 0 I_NxN, 1..24 I_16x16, 25 I_PCM;
  // base 0 (I slice), 5 (P), 23 (B): Table 9-36 after the slice's prefix
  void put_i_type(int cur, int v, int base) {
    if (!cabac_) {
      bw_->ue(static_cast<uint32_t>(base + v));
      return;
    }
    int sfx = 0, inc0 = 0;
    if (base == 0) {
      const int a = nb_a(cur), b = nb_b(cur);
      inc0 = (a >= 0 && mb_[static_cast<size_t>(a)].type != 1) + (b >= 0 && mb_[static_cast<size_t>(b)].type != 1);
    } else if (base == 5) {
      cab_.enc(14, 1);
      sfx = 17;
    } else {
      put_b_type(cur, 23);
      sfx = 32;
    }
    cab_.enc(sfx ? sfx : 3 + inc0, v != 0);
    if (v == 0) return;
    cab_.term(v == 25);
    if (v == 25) return;  // I_PCM: the caller aligns, writes the samples, restarts the engine
    const int cc = ((v - 1) / 4) % 3, pm = (v - 1) % 4;
    cab_.enc(sfx ? sfx + 1 : 6, v >= 13);
    cab_.enc(sfx ? sfx + 2 : 7, cc != 0);
    if (cc) cab_.enc(sfx ? sfx + 2 : 8, cc == 2);
    cab_.enc(sfx ? sfx + 3 : 9, pm >> 1);
    cab_.enc(sfx ? sfx + 3 : 10, pm & 1);
  }
  // P inter mb_type 0..3 (Table 9-37 P rows; P_8x8ref0 does not exist in CABAC)
  void put_p_type(int t) {
    if (!cabac_) {
      bw_->ue(static_cast<uint32_t>(t));
      return;
    }
    cab_.enc(14, 0);
    if (t == 0 || t == 3) {
      cab_.enc(15, 0);
      cab_.enc(16, t == 3);
    } else {
      cab_.enc(15, 1);
      cab_.enc(17, t == 1);
    }
  }
  void put_p_sub(int v) {
    if (!cabac_) {
      bw_->ue(static_cast<uint32_t>(v));
      return;
    }
    cab_.enc(21, v == 0);
    if (v == 0) return;
    cab_.enc(22, v >= 2);
    if (v >= 2) cab_.enc(23, v == 2);
  }
  // B mb_type t 0..22, 23 = the intra prefix (Table 9-37 B rows, ctxIdx 27..35)
  void put_b_type(int cur, int t) {
    if (!cabac_) {
      bw_->ue(static_cast<uint32_t>(t));
      return;
    }
    const int a = nb_a(cur), b = nb_b(cur);
    cab_.enc(27 + (a >= 0 && !mb_[static_cast<size_t>(a)].d16) + (b >= 0 && !mb_[static_cast<size_t>(b)].d16), t != 0);
    if (t == 0) return;
    if (t <= 2) {
      cab_.enc(30, 0);
      cab_.enc(32, t - 1);
      return;
    }
    cab_.enc(30, 1);
    int bits, extra = -1;
    if (t <= 10) bits = t - 3;
    else if (t == 11) bits = 14;
    else if (t == 22) bits = 15;
    else if (t == 23) bits = 13;
    else {
      bits = (t + 4) >> 1;
      extra = (t + 4) & 1;
    }
    cab_.enc(31, (bits >> 3) & 1);
    cab_.enc(32, (bits >> 2) & 1);
    cab_.enc(32, (bits >> 1) & 1);
    cab_.enc(32, bits & 1);
    if (extra >= 0) cab_.enc(32, extra);
  }
  void put_b_sub(int v) {
    if (!cabac_) {
      bw_->ue(static_cast<uint32_t>(v));
      return;
    }
    cab_.enc(36, v != 0);
    if (v == 0) return;
    if (v <= 2) {
      cab_.enc(37, 0);
      cab_.enc(39, v - 1);
      return;
    }
    cab_.enc(37, 1);
    if (v <= 6) {
      cab_.enc(38, 0);
      cab_.enc(39, (v - 3) >> 1);
      cab_.enc(39, (v - 3) & 1);
    } else if (v <= 10) {
      cab_.enc(38, 1);
      cab_.enc(39, 0);
      cab_.enc(39, (v - 7) >> 1);
      cab_.enc(39, (v - 7) & 1);
    } else {
      cab_.enc(38, 1);
      cab_.enc(39, 1);
      cab_.enc(39, v - 11);
    }
  }
  // condTermFlagN of ref_idx_lX (9.3.3.1.1.6)
  int ref_cond(int cur, int xN, int yN, int l) const {
    const Loc L = loc(cur, xN, yN, 16);
    if (L.mb < 0) return 0;
    const int p8 = (L.yw / 8) * 2 + L.xw / 8;
    const GMb &m = mb_[static_cast<size_t>(L.mb)];
    if ((m.dmask >> p8) & 1) return 0;
    if (L.mb == cur) return cref_[l][p8] > 0;
    if (m.type != 0) return 0;
    return m.ref[l][(L.yw / 4) * 4 + L.xw / 4] > 0;
  }
  // ref_idx_lX of the partition at (x0, y0), w8 x h8 quarters
  void put_ref(int cur, int x0, int y0, int w8, int h8, int l, int v, int nref) {
    if (!cabac_) {
      if (nref == 2) bw_->bit(v ? 0 : 1);  // te(v), range 1
      else bw_->ue(static_cast<uint32_t>(v));
    } else {
      cab_.enc(54 + ref_cond(cur, x0 - 1, y0, l) + 2 * ref_cond(cur, x0, y0 - 1, l), v > 0);
      if (v > 0) {
        cab_.enc(58, v > 1);
        if (v > 1) {
          for (int i = 2; i < v; ++i) cab_.enc(59, 1);
          cab_.enc(59, 0);
        }
      }
    }
    for (int qy = 0; qy < h8; ++qy)
      for (int qx = 0; qx < w8; ++qx) cref_[l][(y0 / 8 + qy) * 2 + x0 / 8 + qx] = v;
  }
  int mvd_abs_at(int cur, int xN, int yN, int comp, int l) const {
    const Loc L = loc(cur, xN, yN, 16);
    if (L.mb < 0) return 0;
    const int blk = (L.yw / 4) * 4 + L.xw / 4;
    if (L.mb == cur) return cmvd_[l][blk][comp];
    const GMb &m = mb_[static_cast<size_t>(L.mb)];
    return m.type == 0 ? m.mvda[l][blk][comp] : 0;
  }
  void cab_mvd(int base, int sum, int v) {  // UEG3, signedValFlag 1, uCoff 9 (9.3.2.3)
    static const int kInc[8] = {3, 4, 5, 6, 6, 6, 6, 6};
    const int a = std::abs(v);
    cab_.enc(base + (sum < 3 ? 0 : (sum > 32 ? 2 : 1)), a > 0);
    if (a == 0) return;
    for (int k = 1; k < 9; ++k) {
      cab_.enc(base + kInc[k - 1], k < a);
      if (k >= a) break;
    }
    if (a >= 9) cab_.ueg(a - 9, 3);
    cab_.bypass(v < 0);
  }
  // mvd_lX of the (sub-)partition at (sx, sy), pw x ph
  void put_mvd(int cur, int sx, int sy, int pw, int ph, int l, int dx, int dy) {
    if (!cabac_) {
      bw_->se(dx);
      bw_->se(dy);
    } else {
      cab_mvd(40, mvd_abs_at(cur, sx - 1, sy, 0, l) + mvd_abs_at(cur, sx, sy - 1, 0, l), dx);
      cab_mvd(47, mvd_abs_at(cur, sx - 1, sy, 1, l) + mvd_abs_at(cur, sx, sy - 1, 1, l), dy);
    }
    for (int yy = sy / 4; yy < (sy + ph) / 4; ++yy)
      for (int xx = sx / 4; xx < (sx + pw) / 4; ++xx) {
        cmvd_[l][yy * 4 + xx][0] = std::abs(dx);
        cmvd_[l][yy * 4 + xx][1] = std::abs(dy);
      }
  }
  void put_pred_mode(bool use_pred, int rem) {  // prev_intraNxN_pred_mode_flag / rem_intraNxN_pred_mode
    if (!cabac_) {
      bw_->bit(use_pred ? 1 : 0);
      if (!use_pred) bw_->u(3, static_cast<uint32_t>(rem));
      return;
    }
    cab_.enc(68, use_pred);
    if (!use_pred)
      for (int i = 0; i < 3; ++i) cab_.enc(69, (rem >> i) & 1);
  }
  void put_chroma_mode(int cur, int cm) {
    mb_[static_cast<size_t>(cur)].cmode = cm;
    if (!cabac_) {
      bw_->ue(static_cast<uint32_t>(cm));
      return;
    }
    int inc = 0;
    for (const int n : {nb_a(cur), nb_b(cur)})
      if (n >= 0) {
        const GMb &m = mb_[static_cast<size_t>(n)];
        inc += (m.type == 1 || m.type == 2) && m.cmode != 0;
      }
    cab_.enc(64 + inc, cm > 0);
    if (cm > 0) {
      cab_.enc(67, cm > 1);
      if (cm > 1) cab_.enc(67, cm > 2);
    }
  }
  void put_cbp(int cur, int cbp, bool intra) {
    GMb &m = mb_[static_cast<size_t>(cur)];
    if (!cabac_) {
      const uint8_t *t = intra ? kCbpIntra : kCbpInter;
      int code = 0;
      while (t[code] != cbp) ++code;
      bw_->ue(static_cast<uint32_t>(code));
      m.cbp = cbp;
      return;
    }
    int sofar = 0;  // 9.3.3.1.1.4: the current macroblock's bins already coded
    for (int b8 = 0; b8 < 4; ++b8) {
      const int bx = (b8 & 1) * 8, by = (b8 >> 1) * 8;
      int cond[2];
      for (int nb = 0; nb < 2; ++nb) {
        const Loc l = loc(cur, nb ? bx : bx - 1, nb ? by - 1 : by, 16);
        const int b8n = (l.yw / 8) * 2 + l.xw / 8;
        if (l.mb < 0) {
          cond[nb] = 0;
        } else if (l.mb == cur) {
          cond[nb] = ((sofar >> b8n) & 1) ? 0 : 1;
        } else {
          const GMb &n = mb_[static_cast<size_t>(l.mb)];
          cond[nb] = n.type == 3 ? 0 : (n.type == 4 ? 1 : (((n.cbp >> b8n) & 1) ? 0 : 1));
        }
      }
      const int bit = (cbp >> b8) & 1;
      cab_.enc(73 + cond[0] + 2 * cond[1], bit);
      sofar |= bit << b8;
    }
    int ca[2] = {0, 0}, c2[2] = {0, 0};
    const int nbs[2] = {nb_a(cur), nb_b(cur)};
    for (int i = 0; i < 2; ++i) {
      if (nbs[i] < 0) continue;
      const GMb &n = mb_[static_cast<size_t>(nbs[i])];
      const int cc = n.type == 3 ? 2 : (n.type == 4 ? 0 : n.cbp >> 4);
      ca[i] = cc != 0;
      c2[i] = cc == 2;
    }
    const int cc = cbp >> 4;
    cab_.enc(77 + ca[0] + 2 * ca[1], cc != 0);
    if (cc) cab_.enc(81 + c2[0] + 2 * c2[1], cc == 2);
    m.cbp = cbp;
  }
  void put_t8(int cur, bool t8) {  // transform_size_8x8_flag (CABAC streams only)
    mb_[static_cast<size_t>(cur)].t8 = t8;
    const int a = nb_a(cur), b = nb_b(cur);
    cab_.enc(399 + (a >= 0 && mb_[static_cast<size_t>(a)].t8) + (b >= 0 && mb_[static_cast<size_t>(b)].t8), t8);
  }
  void put_skip(int cur, bool skip, bool b_slice) {  // mb_skip_flag
    const int a = nb_a(cur), b = nb_b(cur);
    cab_.enc((b_slice ? 24 : 11) + (a >= 0 && mb_[static_cast<size_t>(a)].type != 4) +
                 (b >= 0 && mb_[static_cast<size_t>(b)].type != 4),
             skip);
  }
  void begin_mb(int a, int slice) {
    reset_mb(a, slice);
    qpd_prev_ = qpd_cur_;
    qpd_cur_ = false;
    for (int l = 0; l < 2; ++l) {
      for (int k = 0; k < 4; ++k) cref_[l][k] = -1;
      for (int k = 0; k < 16; ++k) cmvd_[l][k][0] = cmvd_[l][k][1] = 0;
    }
  }
  void end_mb(int a, int last) {
    GMb &m = mb_[static_cast<size_t>(a)];
    if (m.type == 0) std::memcpy(m.mvda, cmvd_, sizeof m.mvda);
    if (cabac_) cab_.term(a == last - 1);  // end_of_slice_flag
  }

  // valid intra modes
  void write_intra(int cur, bool in_p, int base_b = -1) {
    const int base = base_b >= 0 ? base_b : (in_p ? 5 : 0);
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
      m.cbp = 0x2f;
      put_i_type(cur, 25, base);  // CABAC: the terminate bin 1 flushed the engine
      bw_->align_zero();
      uint8_t buf[384];
      for (uint8_t &x : buf) x = static_cast<uint8_t>(rng_.below(256));
      bw_->bytes(buf, 384);
      for (int i = 0; i < 16; ++i) m.nz[i] = 16;
      for (int i = 0; i < 4; ++i) m.nzc[0][i] = m.nzc[1][i] = 16;
      if (cabac_) cab_.start();   // 9.3.1.2 after pcm_sample data
      return;
    }
    if (r < 600) {  // I_NxN (Intra_8x8 with transform_size_8x8_flag)
      m.type = 1;
      put_i_type(cur, 0, base);
      const bool t8 = t8mode_ && rng_.below(2) != 0;
      if (t8mode_) put_t8(cur, t8);
      const int nblk = t8 ? 4 : 16, bs = t8 ? 8 : 4;
      for (int k = 0; k < nblk; ++k) {
        const int bx = t8 ? (k & 1) * 2 : kBlkX[k], by = t8 ? (k >> 1) * 2 : kBlkY[k];
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
        put_pred_mode(mode == pred, mode < pred ? mode : mode - 1);
        // Intra8x8PredMode is kept on each of its 4x4 blocks: the 8.3.1.1 /
        // 8.3.2.1 neighbour lookups then read the block at the sample position
        for (int yy = 0; yy < bs / 4; ++yy)
          for (int xx = 0; xx < bs / 4; ++xx) m.i4[(by + yy) * 4 + bx + xx] = mode;
      }
      put_chroma_mode(cur, chroma_mode());
      const int cbp = static_cast<int>(rng_.below(16)) | (static_cast<int>(rng_.below(3)) << 4);
      put_cbp(cur, cbp, true);
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
    m.cbp = (cc << 4) | lum;
    put_i_type(cur, 1 + pm + 4 * cc + (lum ? 12 : 0), base);
    put_chroma_mode(cur, chroma_mode());
    write_qp_delta();
    write_residual(cur, (cc << 4) | lum, true);
  }

  void write_inter(int cur, int pan_x, int pan_y) {
    GMb &m = mb_[cur];
    m.type = 0;
    const uint32_t r = rng_.below(1000);
    int mb_type = r < 640 ? 0 : (r < 760 ? 1 : (r < 880 ? 2 : (r < 980 ? 3 : 4)));
    if (mb_type == 4 && (nref_ < 1 || cabac_)) mb_type = 3;  // no P_8x8ref0 in CABAC
    put_p_type(mb_type);
    const int nparts = mb_type == 0 ? 1 : (mb_type <= 2 ? 2 : 4);
    int sub[4] = {0, 0, 0, 0}, refs[4] = {0, 0, 0, 0};
    bool small = false;
    if (mb_type >= 3)
      for (int k = 0; k < 4; ++k) {
        sub[k] = static_cast<int>(rng_.below(4));
        small |= sub[k] != 0;
        put_p_sub(sub[k]);
      }
    if (mb_type != 4 && nref_ > 1)
      for (int k = 0; k < nparts; ++k) {
        refs[k] = rng_.below(4) ? 0 : static_cast<int>(rng_.below(static_cast<uint32_t>(nref_)));
        const int x0 = (mb_type == 2 || mb_type == 3) ? 8 * (k & 1) : 0;
        const int y0 = mb_type == 1 ? 8 * k : (mb_type == 3 ? 8 * (k >> 1) : 0);
        put_ref(cur, x0, y0, (mb_type == 0 || mb_type == 1) ? 2 : 1, (mb_type == 0 || mb_type == 2) ? 2 : 1, 0,
                refs[k], nref_);
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
        const int dist = bmode_ ? cur_d_ - lst_[0][refs[k]] : refs[k] + 1;
        const int tx = dist * pan_x + static_cast<int>(rng_.below(13)) - 6;
        const int ty = dist * pan_y + static_cast<int>(rng_.below(13)) - 6;
        put_mvd(cur, sx, sy, pw, ph, 0, tx - px, ty - py);
        for (int yy = sy / 4; yy < (sy + ph) / 4; ++yy)
          for (int xx = sx / 4; xx < (sx + pw) / 4; ++xx) {
            const int blk = yy * 4 + xx;
            m.ref[0][blk] = refs[k];
            m.mv[0][blk][0] = tx;
            m.mv[0][blk][1] = ty;
            m.refd[0][blk] = lst_[0][refs[k]];
            done |= 1 << blk;
          }
      }
    }
    int cbp = 0;
    for (int k8 = 0; k8 < 4; ++k8)
      if (rng_.below(100) < 35) cbp |= 1 << k8;
    const uint32_t cr = rng_.below(100);
    cbp |= (cr < 60 ? 0 : (cr < 85 ? 1 : 2)) << 4;
    put_cbp(cur, cbp, false);
    if (t8mode_ && (cbp & 15) && !small) put_t8(cur, rng_.below(2) != 0);
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
      for (int l = 0; l < 2; ++l) {
        m.ref[l][i] = -1;
        m.refd[l][i] = -1;
        m.mv[l][i][0] = m.mv[l][i][1] = 0;
        m.mvda[l][i][0] = m.mvda[l][i][1] = 0;
      }
    }
    for (int i = 0; i < 4; ++i) m.nzc[0][i] = m.nzc[1][i] = 0;
  }

  // slice_data(): CAVLC mb_skip_run, or CABAC mb_skip_flag + end_of_slice_flag
  void write_slice_data(int first, int last, int slice, bool is_p, int pan_x, int pan_y) {
    uint32_t skip_run = 0;
    qpd_cur_ = false;
    for (int a = first; a < last; ++a) {
      begin_mb(a, slice);
      if (content_ && !is_p) {
        content_intra(a, 0);
        end_mb(a, last);
        continue;
      }
      if (is_p) {
        const bool cskip = content_ && content_p_decide(a);
        if (cskip) {
          if (cabac_) put_skip(a, true, false);
          else ++skip_run;
          end_mb(a, last);
          continue;
        }
        const uint32_t r = content_ ? 999 : rng_.below(1000);
        if (r < 450) {  // P_Skip
          GMb &m = mb_[static_cast<size_t>(a)];
          m.type = 4;
          int px, py;
          skipmv(a, &px, &py);
          for (int i = 0; i < 16; ++i) {
            m.ref[0][i] = 0;
            m.mv[0][i][0] = px;
            m.mv[0][i][1] = py;
            m.refd[0][i] = lst_[0][0];
          }
          if (cabac_) put_skip(a, true, false);
          else ++skip_run;
          end_mb(a, last);
          continue;
        }
        if (cabac_) {
          put_skip(a, false, false);
        } else {
          bw_->ue(skip_run);
          skip_run = 0;
        }
        if (content_) content_p_write(a);
        else if (r < 920) write_inter(a, pan_x, pan_y);
        else write_intra(a, true);
      } else {
        write_intra(a, false);
      }
      end_mb(a, last);
    }
    if (!cabac_ && is_p && skip_run) bw_->ue(skip_run);
  }


  // ---------------------------------------------------------------- B mode
  static int min_pos(int x, int y) { return (x >= 0 && y >= 0) ? std::min(x, y) : std::max(x, y); }
  void set_b(GMb &m, int l, int blk, int ref, int mvx, int mvy) {
    m.ref[l][blk] = ref;
    m.refd[l][blk] = ref >= 0 ? lst_[l][ref] : -1;
    m.mv[l][blk][0] = ref >= 0 ? mvx : 0;
    m.mv[l][blk][1] = ref >= 0 ? mvy : 0;
  }
  // 8.4.1.2 direct prediction of the blocks in mask (as the decoder derives it)
  void direct(int cur, int mask) {
    GMb &m = mb_[static_cast<size_t>(cur)];
    int ref[2] = {-1, -1}, mvp[2][2] = {{0, 0}, {0, 0}};
    bool zero = false;
    if (spatial_) {
      for (int l = 0; l < 2; ++l) {
        Nb a = nbmv(cur, -1, 0, 0, l), b = nbmv(cur, 0, -1, 0, l), c = nbmv(cur, 16, -1, 0, l);
        if (!c.avail) c = nbmv(cur, -1, -1, 0, l);
        ref[l] = min_pos(a.ref, min_pos(b.ref, c.ref));
      }
      if (ref[0] < 0 && ref[1] < 0) {
        ref[0] = ref[1] = 0;
        zero = true;
      }
      for (int l = 0; l < 2; ++l)
        if (ref[l] >= 0 && !zero) mvpred(cur, 0, 0, 16, 16, ref[l], 0, &mvp[l][0], &mvp[l][1], l);
    }
    for (int blk = 0; blk < 16; ++blk) {
      if (!((mask >> blk) & 1)) continue;
      const int cb = ((blk >> 3) * 3) * 4 + ((blk & 3) >> 1) * 3;  // direct_8x8_inference
      const GMb &cm = col_->mbs[static_cast<size_t>(cur)];
      const bool cintra = cm.type >= 1 && cm.type <= 3;
      const int cl = cm.ref[0][cb] >= 0 ? 0 : 1;
      const int rcol = cintra ? -1 : cm.ref[cl][cb];
      const int mcx = rcol < 0 ? 0 : cm.mv[cl][cb][0], mcy = rcol < 0 ? 0 : cm.mv[cl][cb][1];
      if (spatial_) {
        const bool cz = rcol == 0 && mcx >= -1 && mcx <= 1 && mcy >= -1 && mcy <= 1;
        for (int l = 0; l < 2; ++l) {
          const bool z = zero || ref[l] < 0 || (ref[l] == 0 && cz);
          set_b(m, l, blk, ref[l], z ? 0 : mvp[l][0], z ? 0 : mvp[l][1]);
        }
      } else {
        int r0 = 0;
        if (rcol >= 0) {
          const int dref = cm.refd[cl][cb];
          r0 = -1;
          for (int i = 0; i < nlst_[0] && r0 < 0; ++i)
            if (lst_[0][i] == dref) r0 = i;
          if (r0 < 0) r0 = 0;  // run_b only picks temporal when every colocated reference is listed
        }
        const RefPic *p0 = pic_of(lst_[0][r0]), *p1 = col_;
        const int tb = std::clamp(cur_poc_ - p0->poc, -128, 127), td = std::clamp(p1->poc - p0->poc, -128, 127);
        int m0x = mcx, m0y = mcy, m1x = 0, m1y = 0;
        if (td != 0) {
          const int tx = (16384 + std::abs(td / 2)) / td;
          const int dsf = std::clamp((tb * tx + 32) >> 6, -1024, 1023);
          m0x = (dsf * mcx + 128) >> 8;
          m0y = (dsf * mcy + 128) >> 8;
          m1x = m0x - mcx;
          m1y = m0y - mcy;
        }
        set_b(m, 0, blk, r0, m0x, m0y);
        set_b(m, 1, blk, 0, m1x, m1y);
      }
    }
  }

  // B macroblock (inter): mb_type, sub types, ref_idx_l0/l1, mvd_l0/l1, cbp, residual
  void write_b_inter(int cur, int pan_x, int pan_y) {
    GMb &m = mb_[static_cast<size_t>(cur)];
    m.type = 0;
    static const uint8_t kPart[22][2] = {{0, 0}, {1, 0}, {2, 0}, {3, 0}, {1, 1}, {1, 1}, {2, 2}, {2, 2},
                                         {1, 2}, {1, 2}, {2, 1}, {2, 1}, {1, 3}, {1, 3}, {2, 3}, {2, 3},
                                         {3, 1}, {3, 1}, {3, 2}, {3, 2}, {3, 3}, {3, 3}};
    static const uint8_t kSub[13][2] = {{0, 0}, {1, 0}, {2, 0}, {3, 0}, {1, 1}, {1, 2}, {2, 1},
                                        {2, 2}, {3, 1}, {3, 2}, {1, 3}, {2, 3}, {3, 3}};
    const uint32_t r = rng_.below(100);
    int mb_type;
    if (r < 5) mb_type = 0;
    else if (r < 60) mb_type = 1 + static_cast<int>(rng_.below(3));
    else if (r < 85) mb_type = 4 + static_cast<int>(rng_.below(18));
    else mb_type = 22;
    put_b_type(cur, mb_type);
    int shape, pm[4] = {1, 1, 1, 1}, ssh[4] = {0, 0, 0, 0}, subv[4] = {0, 0, 0, 0};
    if (mb_type == 0) { shape = 0; pm[0] = 0; m.d16 = true; }
    else if (mb_type <= 3) { shape = 0; pm[0] = mb_type; }
    else if (mb_type < 22) { shape = (mb_type & 1) ? 2 : 1; pm[0] = kPart[mb_type][0]; pm[1] = kPart[mb_type][1]; }
    else shape = 3;
    const int nparts = shape == 0 ? 1 : (shape < 3 ? 2 : 4);
    if (shape == 3)
      for (int k = 0; k < 4; ++k) {
        subv[k] = static_cast<int>(rng_.below(13));
        pm[k] = kSub[subv[k]][0];
        ssh[k] = kSub[subv[k]][1];
      }
    // direct-predicted quarters (ref_idx contexts treat them as refIdx 0);
    // sub-8x8 partitions rule out the 8x8 transform (direct ones do not:
    // direct_8x8_inference_flag is 1)
    bool small = false;
    for (int k = 0; k < (shape == 3 ? 4 : 0); ++k) {
      if (pm[k] == 0) m.dmask |= 1 << k;
      else small |= ssh[k] != 0;
    }
    if (mb_type == 0) m.dmask = 0xf;
    int refs[2][4];
    for (int l = 0; l < 2; ++l)
      for (int k = 0; k < 4; ++k)
        refs[l][k] = ((pm[k] >> l) & 1) ? (rng_.below(4) ? 0 : static_cast<int>(rng_.below(static_cast<uint32_t>(nlst_[l])))) : -1;
    // motion in derivation order; mvds kept for the syntax order
    int mvd[2][4][4][2] = {};
    int done = 0;
    for (int k = 0; k < nparts; ++k) {
      int nsub = 1, pw, ph, x0, y0;
      if (shape == 0) { pw = ph = 16; x0 = y0 = 0; }
      else if (shape == 1) { pw = 16; ph = 8; x0 = 0; y0 = 8 * k; }
      else if (shape == 2) { pw = 8; ph = 16; x0 = 8 * k; y0 = 0; }
      else {
        x0 = 8 * (k & 1);
        y0 = 8 * (k >> 1);
        nsub = ssh[k] == 0 ? 1 : (ssh[k] == 3 ? 4 : 2);
        pw = (ssh[k] == 0 || ssh[k] == 1) ? 8 : 4;
        ph = (ssh[k] == 0 || ssh[k] == 2) ? 8 : 4;
      }
      if (pm[k] == 0) {
        int bm = 0;
        for (int yy = y0 / 4; yy < (y0 + ph) / 4; ++yy)
          for (int xx = x0 / 4; xx < (x0 + pw) / 4; ++xx) bm |= 1 << (yy * 4 + xx);
        direct(cur, bm);
        done |= bm;
        continue;
      }
      for (int q = 0; q < nsub; ++q) {
        int sx = x0, sy = y0;
        if (shape == 3) {
          if (ssh[k] == 1) sy += 4 * q;
          else if (ssh[k] == 2) sx += 4 * q;
          else if (ssh[k] == 3) { sx += 4 * (q & 1); sy += 4 * (q >> 1); }
        }
        for (int l = 0; l < 2; ++l) {
          int tx = 0, ty = 0;
          if (refs[l][k] >= 0) {
            int px, py;
            mvpred(cur, sx, sy, pw, ph, refs[l][k], done, &px, &py, l);
            const int dist = cur_d_ - lst_[l][refs[l][k]];
            tx = dist * pan_x + static_cast<int>(rng_.below(13)) - 6;
            ty = dist * pan_y + static_cast<int>(rng_.below(13)) - 6;
            mvd[l][k][q][0] = tx - px;
            mvd[l][k][q][1] = ty - py;
          }
          for (int yy = sy / 4; yy < (sy + ph) / 4; ++yy)
            for (int xx = sx / 4; xx < (sx + pw) / 4; ++xx) set_b(m, l, yy * 4 + xx, refs[l][k], tx, ty);
        }
        for (int yy = sy / 4; yy < (sy + ph) / 4; ++yy)
          for (int xx = sx / 4; xx < (sx + pw) / 4; ++xx) done |= 1 << (yy * 4 + xx);
      }
    }
    // syntax order (7.3.5.1 / 7.3.5.2)
    if (shape == 3)
      for (int k = 0; k < 4; ++k) put_b_sub(subv[k]);
    auto part = [&](int k, int *x0, int *y0, int *pw, int *ph) {
      if (shape == 0) { *pw = *ph = 16; *x0 = *y0 = 0; }
      else if (shape == 1) { *pw = 16; *ph = 8; *x0 = 0; *y0 = 8 * k; }
      else if (shape == 2) { *pw = 8; *ph = 16; *x0 = 8 * k; *y0 = 0; }
      else { *pw = *ph = 8; *x0 = 8 * (k & 1); *y0 = 8 * (k >> 1); }
    };
    for (int l = 0; l < 2; ++l)
      for (int k = 0; k < nparts; ++k) {
        if (refs[l][k] < 0 || nlst_[l] < 2) continue;
        int x0, y0, pw, ph;
        part(k, &x0, &y0, &pw, &ph);
        put_ref(cur, x0, y0, pw / 8, ph / 8, l, refs[l][k], nlst_[l]);
      }
    for (int l = 0; l < 2; ++l)
      for (int k = 0; k < nparts; ++k) {
        if (refs[l][k] < 0) continue;
        int x0, y0, pw, ph;
        part(k, &x0, &y0, &pw, &ph);
        const int nsub = shape < 3 ? 1 : (ssh[k] == 0 ? 1 : (ssh[k] == 3 ? 4 : 2));
        if (shape == 3) {
          pw = (ssh[k] == 0 || ssh[k] == 1) ? 8 : 4;
          ph = (ssh[k] == 0 || ssh[k] == 2) ? 8 : 4;
        }
        for (int q = 0; q < nsub; ++q) {
          int sx = x0, sy = y0;
          if (shape == 3) {
            if (ssh[k] == 1) sy += 4 * q;
            else if (ssh[k] == 2) sx += 4 * q;
            else if (ssh[k] == 3) { sx += 4 * (q & 1); sy += 4 * (q >> 1); }
          }
          put_mvd(cur, sx, sy, pw, ph, l, mvd[l][k][q][0], mvd[l][k][q][1]);
        }
      }
    int cbp = 0;
    for (int k8 = 0; k8 < 4; ++k8)
      if (rng_.below(100) < 30) cbp |= 1 << k8;
    const uint32_t cr = rng_.below(100);
    cbp |= (cr < 60 ? 0 : (cr < 85 ? 1 : 2)) << 4;
    put_cbp(cur, cbp, false);
    if (t8mode_ && (cbp & 15) && !small) put_t8(cur, rng_.below(2) != 0);
    if (cbp) write_qp_delta();
    write_residual(cur, cbp, false);
  }

  void write_slice_data_b(int first, int last, int slice, int pan_x, int pan_y) {
    uint32_t skip_run = 0;
    qpd_cur_ = false;
    for (int a = first; a < last; ++a) {
      begin_mb(a, slice);
      if (content_) {
        if (content_b_decide(a)) {
          if (cabac_) put_skip(a, true, true);
          else ++skip_run;
        } else {
          if (cabac_) {
            put_skip(a, false, true);
          } else {
            bw_->ue(skip_run);
            skip_run = 0;
          }
          content_b_write(a);
        }
        end_mb(a, last);
        continue;
      }
      const uint32_t r = rng_.below(1000);
      if (r < 350) {  // B_Skip
        GMb &m = mb_[static_cast<size_t>(a)];
        m.type = 4;
        m.d16 = true;
        m.dmask = 0xf;
        direct(a, 0xffff);
        if (cabac_) put_skip(a, true, true);
        else ++skip_run;
        end_mb(a, last);
        continue;
      }
      if (cabac_) {
        put_skip(a, false, true);
      } else {
        bw_->ue(skip_run);
        skip_run = 0;
      }
      if (r < 950) write_b_inter(a, pan_x, pan_y);
      else write_intra_b(a);
      end_mb(a, last);
    }
    if (!cabac_ && skip_run) bw_->ue(skip_run);
  }
  void write_intra_b(int a) { write_intra(a, true, 23); }


  // ------------------------------------------------------- content mode
  // (edge_cases bit 14, synth_content.h): decisions by SAD against the source,
  // predictions from the writer's own reconstruction (closed loop)
  bool content_ = false;
  int cqp_[2] = {0, 0};                    // chroma_qp_index_offset, second_chroma_qp_index_offset
  std::vector<content::Scene> scenes_;
  std::vector<int> scene_of_, offx_, offy_;  // per display frame of the chunk: scene, background pan offset
  std::vector<std::pair<int, content::Frame>> srcs_;  // rendered sources by display frame
  Pcg32 tex_rng_{0x7e47};
  std::vector<uint8_t> rec_;               // the current picture's reconstruction (NV12, coded size)
  std::vector<MbRec> mrec_;                // ... its macroblocks in decoder form (deblocking)
  std::vector<MbRecB> mrec1_;
  int W() const { return mbw_ * 16; }
  int H() const { return mbh_ * 16; }
  int qpc(int pl) const { return h264::kQpc[std::clamp(qp_ + cqp_[pl], 0, 51)]; }
  const content::Frame &src(int d) {
    for (auto &e : srcs_)
      if (e.first == d) return e.second;
    srcs_.emplace_back(d, content::Frame{});
    content::Frame &f = srcs_.back().second;
    f.alloc(W(), H());
    content::render(scenes_[static_cast<size_t>(scene_of_[static_cast<size_t>(d)])], d, offx_[static_cast<size_t>(d)],
                    offy_[static_cast<size_t>(d)], &f);
    return f;
  }
  // keep the sources of the current picture and the DPB
  void prune_sources() {
    std::vector<std::pair<int, content::Frame>> keep;
    for (auto &e : srcs_) {
      bool k = e.first == cur_d_;
      for (const RefPic &r : dpb_) k |= r.d == e.first;
      if (k) keep.push_back(std::move(e));
    }
    srcs_.swap(keep);
  }
  const uint8_t *rec_of(int d) const { return pic_of(d)->rec.data(); }
  // 8.4.2.2 for whole-pel even motion from a reconstruction (clamped samples)
  void predict_rec(const uint8_t *R, int mbx, int mby, int mvx, int mvy, content::MbPix *p) const {
    const int w = W(), h = H(), dx = mvx >> 2, dy = mvy >> 2;
    const uint8_t *UV = R + static_cast<size_t>(w) * h;
    for (int y = 0; y < 16; ++y) {
      const int yy = content::clampi(mby * 16 + y + dy, 0, h - 1);
      for (int x = 0; x < 16; ++x) p->y[y * 16 + x] = R[size_t(yy) * w + content::clampi(mbx * 16 + x + dx, 0, w - 1)];
    }
    for (int y = 0; y < 8; ++y) {
      const int yy = content::clampi(mby * 8 + y + dy / 2, 0, h / 2 - 1);
      for (int x = 0; x < 8; ++x) {
        const size_t o = size_t(yy) * w + 2 * content::clampi(mbx * 8 + x + dx / 2, 0, w / 2 - 1);
        p->c[0][y * 8 + x] = UV[o];
        p->c[1][y * 8 + x] = UV[o + 1];
      }
    }
  }
  // best whole-pel motion (quarter-sample units) of macroblock a from display
  // frame r: the background's pan, a sprite's motion, or none
  int best_mv(int a, int r, int *mvx, int *mvy, content::MbPix *pred) {
    const int mx = a % mbw_, my = a / mbw_;
    const content::Scene &sc = scenes_[static_cast<size_t>(scene_of_[static_cast<size_t>(cur_d_)])];
    content::MbPix cur, p;
    content::source_mb(src(cur_d_), mx, my, &cur);
    const uint8_t *R = rec_of(r);
    int cand[8][2], n = 0;
    cand[n][0] = 4 * (offx_[static_cast<size_t>(cur_d_)] - offx_[static_cast<size_t>(r)]);
    cand[n][1] = 4 * (offy_[static_cast<size_t>(cur_d_)] - offy_[static_cast<size_t>(r)]);
    ++n;
    cand[n][0] = cand[n][1] = 0;
    ++n;
    for (int k = 0; k < static_cast<int>(sc.spr.size()) && n < 8; ++k) {
      int cx, cy, rx, ry;
      content::sprite_pos(sc, k, cur_d_, &cx, &cy);
      content::sprite_pos(sc, k, r, &rx, &ry);
      const content::Sprite &sp = sc.spr[static_cast<size_t>(k)];
      const int px = content::wrapi(cx, W()), py = content::wrapi(cy, H());
      if (px > mx * 16 + 15 || px + sp.tex.w <= mx * 16 || py > my * 16 + 15 || py + sp.tex.h <= my * 16) continue;
      cand[n][0] = 4 * (rx - cx);
      cand[n][1] = 4 * (ry - cy);
      ++n;
    }
    int best = 1 << 30;
    for (int i = 0; i < n; ++i) {
      predict_rec(R, mx, my, cand[i][0], cand[i][1], &p);
      const int sd = content::sad_all(cur, p);
      if (sd < best) {
        best = sd;
        *mvx = cand[i][0];
        *mvy = cand[i][1];
        *pred = p;
      }
    }
    return best;
  }
  // 8.4.2.3.1 implicit bi-prediction weights of RefPicList0[r0] / RefPicList1[r1]
  void implicit_w(int r0, int r1, int *w0, int *w1) const {
    *w0 = *w1 = 32;
    const RefPic *p0 = pic_of(lst_[0][r0]), *p1 = pic_of(lst_[1][r1]);
    if (!p0 || !p1) return;
    const int tb = std::clamp(cur_poc_ - p0->poc, -128, 127), td = std::clamp(p1->poc - p0->poc, -128, 127);
    if (td == 0) return;
    const int tx = (16384 + std::abs(td / 2)) / td;
    const int dsf = std::clamp((tb * tx + 32) >> 6, -1024, 1023);
    if ((dsf >> 2) < -64 || (dsf >> 2) > 128) return;
    *w0 = 64 - (dsf >> 2);
    *w1 = dsf >> 2;
  }
  static int bipred(int p0, int p1, int w0, int w1, bool implicit) {
    return implicit ? std::clamp((p0 * w0 + p1 * w1 + 32) >> 6, 0, 255) : (p0 + p1 + 1) >> 1;
  }
  // prediction of macroblock a from its GMb's per-block references / motion
  // (skip and direct modes); false when a motion vector is not whole-pel even
  bool pred_from_mb(int a, content::MbPix *out) {
    const GMb &m = mb_[static_cast<size_t>(a)];
    const int mx = a % mbw_, my = a / mbw_;
    // one prediction per distinct (list, reference, motion): direct
    // modes mostly give the whole macroblock one
    content::MbPix pl[2];
    int have[2][3] = {{-1, 0, 0}, {-1, 0, 0}};
    for (int b = 0; b < 16; ++b) {
      const int rr[2] = {m.ref[0][b], m.ref[1][b]};
      for (int l = 0; l < 2; ++l) {
        if (rr[l] < 0) continue;
        if ((m.mv[l][b][0] & 7) || (m.mv[l][b][1] & 7)) return false;
        if (have[l][0] != rr[l] || have[l][1] != m.mv[l][b][0] || have[l][2] != m.mv[l][b][1]) {
          predict_rec(rec_of(lst_[l][rr[l]]), mx, my, m.mv[l][b][0], m.mv[l][b][1], &pl[l]);
          have[l][0] = rr[l];
          have[l][1] = m.mv[l][b][0];
          have[l][2] = m.mv[l][b][1];
        }
      }
      if (rr[0] < 0 && rr[1] < 0) return false;
      const bool bi = rr[0] >= 0 && rr[1] >= 0;
      int w0 = 32, w1 = 32;
      if (bi && weighted_ == 2) implicit_w(rr[0], rr[1], &w0, &w1);
      const int bx = (b & 3) * 4, by = (b >> 2) * 4;
      const content::MbPix &one = pl[rr[0] >= 0 ? 0 : 1];
      for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) {
          const int i = (by + y) * 16 + bx + x;
          out->y[i] = bi ? bipred(pl[0].y[i], pl[1].y[i], w0, w1, weighted_ == 2) : one.y[i];
        }
      for (int c = 0; c < 2; ++c)
        for (int y = 0; y < 2; ++y)
          for (int x = 0; x < 2; ++x) {
            const int i = (by / 2 + y) * 8 + bx / 2 + x;
            out->c[c][i] = bi ? bipred(pl[0].c[c][i], pl[1].c[c][i], w0, w1, weighted_ == 2) : one.c[c][i];
          }
    }
    return true;
  }

  // ---- reconstruction (8.5 with Flat_16 scaling; recon_full.h's transforms)
  static void ls4_flat(int qp, int32_t *ls) {
    for (int k = 0; k < 16; ++k) ls[k] = full::level_scale(qp % 6, k >> 2, k & 3);
  }
  void put_luma_blk(int a, int x0, int y0, int n, const int *pred16, const int *res) {
    const int w = W(), mx = a % mbw_, my = a / mbw_;
    for (int y = 0; y < n; ++y)
      for (int x = 0; x < n; ++x) {
        const int i = (y0 + y) * 16 + x0 + x;
        rec_[size_t(my * 16 + y0 + y) * w + mx * 16 + x0 + x] = static_cast<uint8_t>(std::clamp(pred16[i] + res[y * n + x], 0, 255));
      }
  }
  // luma 4x4 block b (raster) of a non-Intra_16x16 macroblock from its scan-order levels
  void recon_luma4(int a, int b, const int *lev, const int *pred16) {
    static const uint8_t kZ4[16] = VTS_ZZ_DATA;
    int cf[16] = {}, res[16], any = 0;
    int32_t ls[16];
    for (int s = 0; s < 16; ++s) any |= cf[kZ4[s]] = lev[s];
    if (!any) {  // no residual
      std::memset(res, 0, sizeof res);
      put_luma_blk(a, (b & 3) * 4, (b >> 2) * 4, 4, pred16, res);
      return;
    }
    ls4_flat(qp_, ls);
    full::scale_idct4(cf, qp_, ls, false, res);
    put_luma_blk(a, (b & 3) * 4, (b >> 2) * 4, 4, pred16, res);
  }
  void recon_luma(int a, const content::MbPix &pred, const content::Levels &L, bool i16, bool t8) {
    static const uint8_t kZ4[16] = VTS_ZZ_DATA;
    static const uint8_t kZ8[64] = VTS_ZZ8_DATA;
    static const uint8_t kN8[6][6] = VTS_NORM8_DATA;
    if (t8) {
      int32_t ls8[64];
      for (int k = 0; k < 64; ++k) ls8[k] = 16 * kN8[qp_ % 6][vts_norm8_class(k >> 3, k & 7)];
      for (int b8 = 0; b8 < 4; ++b8) {
        int cf[64] = {}, r8[64];
        for (int s = 0; s < 64; ++s) cf[kZ8[s]] = L.l8[b8][s];
        full::scale_idct8(cf, qp_, ls8, r8);
        put_luma_blk(a, (b8 & 1) * 8, (b8 >> 1) * 8, 8, pred.y, r8);
      }
      return;
    }
    if (!i16) {
      for (int b = 0; b < 16; ++b) recon_luma4(a, b, L.l4[b], pred.y);
      return;
    }
    // 8.5.10: Intra16x16 DC, Hadamard + scaling
    int c[16] = {}, t[16], dcy[16];
    for (int s = 0; s < 16; ++s) c[kZ4[s]] = L.dc16[s];
    for (int i = 0; i < 4; ++i) {
      const int a0 = c[i * 4], a1 = c[i * 4 + 1], a2 = c[i * 4 + 2], a3 = c[i * 4 + 3];
      t[i * 4] = a0 + a1 + a2 + a3;
      t[i * 4 + 1] = a0 + a1 - a2 - a3;
      t[i * 4 + 2] = a0 - a1 - a2 + a3;
      t[i * 4 + 3] = a0 - a1 + a2 - a3;
    }
    const int ls0 = full::level_scale(qp_ % 6, 0, 0);
    for (int j = 0; j < 4; ++j) {
      const int a0 = t[j], a1 = t[4 + j], a2 = t[8 + j], a3 = t[12 + j];
      const int f[4] = {a0 + a1 + a2 + a3, a0 + a1 - a2 - a3, a0 - a1 - a2 + a3, a0 - a1 + a2 - a3};
      for (int i = 0; i < 4; ++i)
        dcy[i * 4 + j] = qp_ >= 36 ? (f[i] * ls0) << (qp_ / 6 - 6) : (f[i] * ls0 + (1 << (5 - qp_ / 6))) >> (6 - qp_ / 6);
    }
    int32_t ls[16];
    ls4_flat(qp_, ls);
    for (int b = 0; b < 16; ++b) {
      int cf[16] = {}, res[16];
      for (int s = 1; s < 16; ++s) cf[kZ4[s]] = L.l4[b][s - 1];
      cf[0] = dcy[b];
      full::scale_idct4(cf, qp_, ls, true, res);
      put_luma_blk(a, (b & 3) * 4, (b >> 2) * 4, 4, pred.y, res);
    }
  }
  void recon_chroma(int a, const content::MbPix &pred, const content::Levels &L) {
    static const uint8_t kZ4[16] = VTS_ZZ_DATA;
    const int w = W(), mx = a % mbw_, my = a / mbw_;
    uint8_t *UV = rec_.data() + static_cast<size_t>(w) * H();
    for (int pl = 0; pl < 2; ++pl) {
      const int q = qpc(pl);
      const int c0 = L.cdc[pl][0], c1 = L.cdc[pl][1], c2 = L.cdc[pl][2], c3 = L.cdc[pl][3];
      const int f[4] = {c0 + c1 + c2 + c3, c0 - c1 + c2 - c3, c0 + c1 - c2 - c3, c0 - c1 - c2 + c3};
      int32_t ls[16];
      ls4_flat(q, ls);
      for (int k = 0; k < 4; ++k) {
        int cf[16] = {}, r[16], any = 0;
        for (int s = 1; s < 16; ++s) any |= cf[kZ4[s]] = L.cac[pl][k][s - 1];
        cf[0] = ((f[k] * ls[0]) << (q / 6)) >> 5;  // 8.5.11.2
        if (any | cf[0]) full::scale_idct4(cf, q, ls, true, r);
        else std::memset(r, 0, sizeof r);
        const int bx = (k & 1) * 4, by = (k >> 1) * 4;
        for (int y = 0; y < 4; ++y)
          for (int x = 0; x < 4; ++x)
            UV[size_t(my * 8 + by + y) * w + 2 * (mx * 8 + bx + x) + pl] =
                static_cast<uint8_t>(std::clamp(pred.c[pl][(by + y) * 8 + bx + x] + r[y * 4 + x], 0, 255));
      }
    }
  }
  // the decoder-form record of macroblock a (deblocking's bS inputs)
  void set_rec(int a, int type, bool t8, const content::Levels *L) {
    const GMb &m = mb_[static_cast<size_t>(a)];
    MbRec &r = mrec_[static_cast<size_t>(a)];
    MbRecB &r1 = mrec1_[static_cast<size_t>(a)];
    r = MbRec{};
    r1 = MbRecB{};
    r.slice = static_cast<uint32_t>(m.slice);
    r.type = static_cast<uint8_t>(type);
    r.qp = static_cast<uint8_t>(qp_);
    r.modes = t8 ? kModeT8 : 0;
    for (int k = 0; k < 4; ++k) r.ref_slot[k] = r1.ref_slot1[k] = -1;
    if (L)
      for (int b = 0; b < 16; ++b) {
        int n = 0;
        if (t8) {
          const int b8 = (b >> 3) * 2 + ((b & 3) >> 1);
          for (int v : L->l8[b8]) n += v != 0;
        } else {
          for (int v : L->l4[b]) n += v != 0;
        }
        r.nz[b] = static_cast<uint8_t>(std::min(n, 255));
      }
    if (type != kMbInter && type != kMbSkip) return;
    for (int b = 0; b < 16; ++b) {
      const int p8 = (b >> 3) * 2 + ((b & 3) >> 1);
      if (m.ref[0][b] >= 0) {
        r.ref_slot[p8] = static_cast<int16_t>(m.refd[0][b]);
        r.mv[b][0] = static_cast<int16_t>(m.mv[0][b][0]);
        r.mv[b][1] = static_cast<int16_t>(m.mv[0][b][1]);
      }
      if (m.ref[1][b] >= 0) {
        r1.ref_slot1[p8] = static_cast<int16_t>(m.refd[1][b]);
        r1.mv1[b][0] = static_cast<int16_t>(m.mv[1][b][0]);
        r1.mv1[b][1] = static_cast<int16_t>(m.mv[1][b][1]);
      }
    }
  }
  // after the picture's last macroblock: the deblocking filter (8.7), in
  // macroblock order as a decoder runs it
  void deblock_picture(int didc, int off_a, int off_b) {
    std::vector<FullSlice> sl(static_cast<size_t>(mb_.back().slice + 1));
    for (FullSlice &f : sl) {
      f = FullSlice{};
      f.dbk_idc = didc;
      f.dbk_a = off_a;
      f.dbk_b = off_b;
    }
    full::ReconCtx c{};
    c.recs = mrec_.data();
    c.recs1 = bmode_ ? mrec1_.data() : nullptr;
    c.slices = sl.data();
    c.surf = rec_.data();
    c.frame_stride = 0;
    c.pitch = W();
    c.uv_off = static_cast<int64_t>(W()) * H();
    c.mbw = mbw_;
    c.mbh = mbh_;
    c.cqp_off = cqp_[0];
    c.cqp_off2 = cqp_[1];
    // a macroblock whose edges all have bS 0 (inter, no levels, one motion
    // equal to its left and top neighbours') is left alone
    auto plain = [&](int a) {
      const MbRec &r = mrec_[static_cast<size_t>(a)];
      const MbRecB &r1 = mrec1_[static_cast<size_t>(a)];
      if (r.type != kMbInter && r.type != kMbSkip) return false;
      for (int b = 0; b < 16; ++b)
        if (r.nz[b] || r.mv[b][0] != r.mv[0][0] || r.mv[b][1] != r.mv[0][1] || r1.mv1[b][0] != r1.mv1[0][0] ||
            r1.mv1[b][1] != r1.mv1[0][1])
          return false;
      for (int k = 1; k < 4; ++k)
        if (r.ref_slot[k] != r.ref_slot[0] || r1.ref_slot1[k] != r1.ref_slot1[0]) return false;
      return true;
    };
    auto same = [&](int a, int n) {
      const MbRec &p = mrec_[static_cast<size_t>(a)], &q = mrec_[static_cast<size_t>(n)];
      const MbRecB &p1 = mrec1_[static_cast<size_t>(a)], &q1 = mrec1_[static_cast<size_t>(n)];
      return p.ref_slot[0] == q.ref_slot[0] && p1.ref_slot1[0] == q1.ref_slot1[0] && p.mv[0][0] == q.mv[0][0] &&
             p.mv[0][1] == q.mv[0][1] && p1.mv1[0][0] == q1.mv1[0][0] && p1.mv1[0][1] == q1.mv1[0][1];
    };
    std::vector<uint8_t> pl(static_cast<size_t>(nmb_));
    for (int a = 0; a < nmb_; ++a) pl[static_cast<size_t>(a)] = plain(a);
    for (int a = 0; a < nmb_; ++a) {
      const int mx = a % mbw_;
      if (pl[static_cast<size_t>(a)] && (mx == 0 || (pl[static_cast<size_t>(a - 1)] && same(a, a - 1))) &&
          (a < mbw_ || (pl[static_cast<size_t>(a - mbw_)] && same(a, a - mbw_))))
        continue;
      full::deblock_mb(c, 0, a);
    }
  }

  // quantise src - pred for an inter macroblock; t8 chosen by fewer levels
  int quant_inter(const content::MbPix &cur, const content::MbPix &pred, bool allow_t8, content::Levels *L, bool *t8) {
    const double dz = 1.0 / 6.0;
    int cbp = content::quant_luma(cur, pred, qp_, dz, false, false, L);
    *t8 = false;
    if (allow_t8 && t8mode_ && (cbp & 15)) {
      content::Levels L8 = *L;
      const int cbp8 = content::quant_luma(cur, pred, qp_, dz, false, true, &L8);
      if (content::nonzero(L8) < content::nonzero(*L)) {
        *L = L8;
        cbp = cbp8;
        *t8 = cbp != 0;
      }
    }
    return cbp | (content::quant_chroma(cur, pred, qpc(0), qpc(1), dz, L) << 4);
  }
  // the rest of an inter macroblock after its motion syntax: cbp, transform
  // size, mb_qp_delta, residual; then its reconstruction
  void put_inter_residual(int a, int cbp, bool t8, const content::Levels &L, const content::MbPix &pred) {
    put_cbp(a, cbp, false);
    if (t8mode_ && (cbp & 15)) put_t8(a, t8);
    if (cbp) write_qp_delta();
    write_residual(a, cbp, false, &L);
    recon_luma(a, pred, L, false, t8);
    recon_chroma(a, pred, L);
    set_rec(a, kMbInter, t8, &L);
  }
  void put_skipped(int a, const content::MbPix &pred) {
    content::Levels L{};
    recon_luma(a, pred, L, false, false);
    recon_chroma(a, pred, L);
    set_rec(a, kMbSkip, false, nullptr);
  }
  int intra_sad_est(int a) {  // flat-prediction SAD of the source, the inter / intra switch
    const int mx = a % mbw_, my = a / mbw_;
    content::MbPix cur;
    content::source_mb(src(cur_d_), mx, my, &cur);
    int sum = 0;
    for (int v : cur.y) sum += v;
    const int dc = (sum + 128) >> 8;
    int sd = 0;
    for (int v : cur.y) sd += std::abs(v - dc);
    return sd;
  }

  // content P macroblock; returns true for P_Skip (GMb and reconstruction
  // done, nothing written)
  bool content_p_decide(int a) {
    const int mx = a % mbw_, my = a / mbw_;
    int px, py;
    skipmv(a, &px, &py);
    if ((px & 7) || (py & 7)) return false;
    content::MbPix cur, ps;
    content::source_mb(src(cur_d_), mx, my, &cur);
    predict_rec(rec_of(lst_[0][0]), mx, my, px, py, &ps);
    content::Levels L;
    bool t8;
    if (quant_inter(cur, ps, false, &L, &t8)) return false;
    GMb &m = mb_[static_cast<size_t>(a)];
    m.type = 4;
    for (int i = 0; i < 16; ++i) {
      m.ref[0][i] = 0;
      m.mv[0][i][0] = px;
      m.mv[0][i][1] = py;
      m.refd[0][i] = lst_[0][0];
    }
    put_skipped(a, ps);
    return true;
  }
  void content_p_write(int a) {
    const int mx = a % mbw_, my = a / mbw_;
    content::MbPix cur, pred;
    content::source_mb(src(cur_d_), mx, my, &cur);
    int tx = 0, ty = 0;
    const int sd = best_mv(a, lst_[0][0], &tx, &ty, &pred);
    if (sd > 4096 && 2 * intra_sad_est(a) < sd) {
      content_intra(a, 5);
      return;
    }
    GMb &m = mb_[static_cast<size_t>(a)];
    m.type = 0;
    put_p_type(0);
    if (nref_ > 1) put_ref(a, 0, 0, 2, 2, 0, 0, nref_);
    int px, py;
    mvpred(a, 0, 0, 16, 16, 0, 0, &px, &py);
    put_mvd(a, 0, 0, 16, 16, 0, tx - px, ty - py);
    for (int b = 0; b < 16; ++b) {
      m.ref[0][b] = 0;
      m.mv[0][b][0] = tx;
      m.mv[0][b][1] = ty;
      m.refd[0][b] = lst_[0][0];
    }
    content::Levels L;
    bool t8;
    const int cbp = quant_inter(cur, pred, true, &L, &t8);
    put_inter_residual(a, cbp, t8, L, pred);
  }

  // content B macroblock; returns true for B_Skip (GMb and reconstruction
  // done, nothing written)
  bool content_b_decide(int a) {
    const int mx = a % mbw_, my = a / mbw_;
    GMb &m = mb_[static_cast<size_t>(a)];
    m.type = 4;
    m.d16 = true;
    m.dmask = 0xf;
    direct(a, 0xffff);
    content::MbPix cur, pd;
    content::source_mb(src(cur_d_), mx, my, &cur);
    if (pred_from_mb(a, &pd)) {
      content::Levels L;
      bool t8;
      if (!quant_inter(cur, pd, false, &L, &t8)) {
        put_skipped(a, pd);
        return true;
      }
    }
    reset_mb(a, m.slice);
    return false;
  }
  void content_b_write(int a) {
    const int mx = a % mbw_, my = a / mbw_;
    GMb &m = mb_[static_cast<size_t>(a)];
    const int slice = m.slice;
    content::MbPix cur, pd, p0, p1, pb;
    content::source_mb(src(cur_d_), mx, my, &cur);
    // direct with residual
    m.type = 0;
    m.d16 = true;
    m.dmask = 0xf;
    direct(a, 0xffff);
    const bool dok = pred_from_mb(a, &pd);
    const int sdd = dok ? content::sad_all(cur, pd) : (1 << 30);
    reset_mb(a, slice);
    int mv[2][2] = {{0, 0}, {0, 0}};
    const int s0 = best_mv(a, lst_[0][0], &mv[0][0], &mv[0][1], &p0);
    const int s1 = best_mv(a, lst_[1][0], &mv[1][0], &mv[1][1], &p1);
    int w0 = 32, w1 = 32;
    if (weighted_ == 2) implicit_w(0, 0, &w0, &w1);
    for (int i = 0; i < 256; ++i) pb.y[i] = bipred(p0.y[i], p1.y[i], w0, w1, weighted_ == 2);
    for (int c = 0; c < 2; ++c)
      for (int i = 0; i < 64; ++i) pb.c[c][i] = bipred(p0.c[c][i], p1.c[c][i], w0, w1, weighted_ == 2);
    const int sb = content::sad_all(cur, pb);
    // mb_type 0 direct, 1 L0, 2 L1, 3 Bi (16x16); direct gets a small bias
    int t = 0, best = sdd - 64;
    if (s0 < best) { t = 1; best = s0; }
    if (s1 < best) { t = 2; best = s1; }
    if (sb < best) { t = 3; best = sb; }
    if (best > 4096 && 2 * intra_sad_est(a) < best) {
      content_intra(a, 23);
      return;
    }
    const content::MbPix &pred = t == 0 ? pd : (t == 1 ? p0 : (t == 2 ? p1 : pb));
    put_b_type(a, t);
    m.type = 0;
    if (t == 0) {
      m.d16 = true;
      m.dmask = 0xf;
      direct(a, 0xffff);
    } else {
      const bool use[2] = {t == 1 || t == 3, t == 2 || t == 3};
      for (int l = 0; l < 2; ++l)
        if (use[l] && nlst_[l] >= 2) put_ref(a, 0, 0, 2, 2, l, 0, nlst_[l]);
      int mvd[2][2] = {{0, 0}, {0, 0}};
      for (int l = 0; l < 2; ++l) {
        if (!use[l]) continue;
        int px, py;
        mvpred(a, 0, 0, 16, 16, 0, 0, &px, &py, l);
        mvd[l][0] = mv[l][0] - px;
        mvd[l][1] = mv[l][1] - py;
      }
      for (int l = 0; l < 2; ++l)
        for (int b = 0; b < 16; ++b) set_b(m, l, b, use[l] ? 0 : -1, mv[l][0], mv[l][1]);
      for (int l = 0; l < 2; ++l)
        if (use[l]) put_mvd(a, 0, 0, 16, 16, l, mvd[l][0], mvd[l][1]);
    }
    content::Levels L;
    bool t8;
    const int cbp = quant_inter(cur, pred, true, &L, &t8);
    put_inter_residual(a, cbp, t8, L, pred);
  }

  // content intra macroblock (base: mb_type offset 0 I, 5 P, 23 B):
  // Intra_16x16 (V / H / DC / plane) or Intra_4x4 (V / H / DC), predicted
  // from the reconstruction's neighbouring samples, chosen by SAD
  void content_intra(int a, int base) {
    static const uint8_t kZ4[16] = VTS_ZZ_DATA;
    GMb &m = mb_[static_cast<size_t>(a)];
    const int mx = a % mbw_, my = a / mbw_, w = W();
    uint8_t *UV = rec_.data() + static_cast<size_t>(w) * H();
    content::MbPix cur;
    content::source_mb(src(cur_d_), mx, my, &cur);
    const Loc A = loc(a, -1, 0, 16), B = loc(a, 0, -1, 16), D = loc(a, -1, -1, 16);
    const bool la = intra_ok(A.mb), ta = intra_ok(B.mb), ca = intra_ok(D.mb);
    auto ys = [&](int x, int y) { return static_cast<int>(rec_[size_t(y) * w + x]); };
    const int x0 = mx * 16, y0 = my * 16;
    m.type = 1;  // intra for the availability of the macroblock's own blocks
    // ---- Intra_16x16 (8.3.3), from the samples around the macroblock
    content::MbPix p16[4];
    const bool ok16[4] = {ta, la, true, la && ta && ca};
    int st = 0, sl = 0;
    for (int i = 0; i < 16; ++i) {
      if (ta) st += ys(x0 + i, y0 - 1);
      if (la) sl += ys(x0 - 1, y0 + i);
    }
    const int dc = (ta && la) ? (st + sl + 16) >> 5 : (ta ? (st + 8) >> 4 : (la ? (sl + 8) >> 4 : 128));
    int hp = 0, vp = 0, pa = 0;
    if (ok16[3]) {
      for (int k = 0; k < 8; ++k) {
        hp += (k + 1) * (ys(x0 + 8 + k, y0 - 1) - ys(x0 + 6 - k, y0 - 1));
        vp += (k + 1) * (ys(x0 - 1, y0 + 8 + k) - ys(x0 - 1, y0 + 6 - k));
      }
      pa = 16 * (ys(x0 - 1, y0 + 15) + ys(x0 + 15, y0 - 1));
    }
    const int pb = (5 * hp + 32) >> 6, pc = (5 * vp + 32) >> 6;
    for (int y = 0; y < 16; ++y)
      for (int x = 0; x < 16; ++x) {
        const int i = y * 16 + x;
        p16[0].y[i] = ta ? ys(x0 + x, y0 - 1) : 0;
        p16[1].y[i] = la ? ys(x0 - 1, y0 + y) : 0;
        p16[2].y[i] = dc;
        p16[3].y[i] = std::clamp((pa + pb * (x - 7) + pc * (y - 7) + 16) >> 5, 0, 255);
      }
    int pm = 2, s16 = 1 << 30;
    for (int k = 0; k < 4; ++k) {
      if (!ok16[k]) continue;
      const int sd = content::sad_luma(cur, p16[k]);
      if (sd < s16) {
        s16 = sd;
        pm = k;
      }
    }
    // ---- Intra_4x4 (8.3.1.2 modes 0 / 1 / 2), blocks in decoding order, each
    // reconstructed before the next predicts from it (into rec_: Intra_16x16
    // reads only samples outside the macroblock)
    content::Levels L{};
    content::MbPix p4;
    int mode4[16], s4 = 0;
    for (int k = 0; k < 16; ++k) {
      const int bx = kBlkX[k], by = kBlkY[k], r = by * 4 + bx;
      const bool t = intra_ok(loc(a, bx * 4, by * 4 - 1, 16).mb), l = intra_ok(loc(a, bx * 4 - 1, by * 4, 16).mb);
      const int X = x0 + bx * 4, Y = y0 + by * 4;
      int cand[3][16], sums[2] = {0, 0};
      for (int i = 0; i < 4; ++i) {
        if (t) sums[0] += ys(X + i, Y - 1);
        if (l) sums[1] += ys(X - 1, Y + i);
      }
      const int d4 = (t && l) ? (sums[0] + sums[1] + 4) >> 3 : (t ? (sums[0] + 2) >> 2 : (l ? (sums[1] + 2) >> 2 : 128));
      for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) {
          cand[0][y * 4 + x] = t ? ys(X + x, Y - 1) : 0;
          cand[1][y * 4 + x] = l ? ys(X - 1, Y + y) : 0;
          cand[2][y * 4 + x] = d4;
        }
      int bm = 2, bs = 1 << 30;
      for (int md = 0; md < 3; ++md) {
        if ((md == 0 && !t) || (md == 1 && !l)) continue;
        int sd = 0;
        for (int y = 0; y < 4; ++y)
          for (int x = 0; x < 4; ++x) sd += std::abs(cur.y[(by * 4 + y) * 16 + bx * 4 + x] - cand[md][y * 4 + x]);
        if (sd < bs) {
          bs = sd;
          bm = md;
        }
      }
      mode4[k] = bm;
      s4 += bs;
      int xres[16], lv[16];
      for (int y = 0; y < 4; ++y)
        for (int x = 0; x < 4; ++x) {
          p4.y[(by * 4 + y) * 16 + bx * 4 + x] = cand[bm][y * 4 + x];
          xres[y * 4 + x] = cur.y[(by * 4 + y) * 16 + bx * 4 + x] - cand[bm][y * 4 + x];
        }
      content::quant4(xres, qp_, 1.0 / 3.0, lv);
      for (int s = 0; s < 16; ++s) L.l4[r][s] = lv[kZ4[s]];
      recon_luma4(a, r, L.l4[r], p4.y);
    }
    const bool use4 = s4 + 256 < s16;
    // ---- chroma (8.3.4): DC / horizontal / vertical
    auto cs = [&](int pl, int x, int y) { return static_cast<int>(UV[size_t(y) * w + 2 * x + pl]); };
    const int cx0 = mx * 8, cy0 = my * 8;
    content::MbPix pcm[3];
    for (int pl = 0; pl < 2; ++pl)
      for (int k = 0; k < 4; ++k) {
        const int xo = (k & 1) * 4, yo = (k >> 1) * 4;
        int stc = 0, slc = 0;
        for (int i = 0; i < 4; ++i) {
          if (ta) stc += cs(pl, cx0 + xo + i, cy0 - 1);
          if (la) slc += cs(pl, cx0 - 1, cy0 + yo + i);
        }
        int v;
        if ((xo == 0 && yo == 0) || (xo && yo)) {
          v = (ta && la) ? (stc + slc + 4) >> 3 : (la ? (slc + 2) >> 2 : (ta ? (stc + 2) >> 2 : 128));
        } else if (xo) {
          v = ta ? (stc + 2) >> 2 : (la ? (slc + 2) >> 2 : 128);
        } else {
          v = la ? (slc + 2) >> 2 : (ta ? (stc + 2) >> 2 : 128);
        }
        for (int y = 0; y < 4; ++y)
          for (int x = 0; x < 4; ++x) {
            const int i = (yo + y) * 8 + xo + x;
            pcm[0].c[pl][i] = v;
            pcm[1].c[pl][i] = la ? cs(pl, cx0 - 1, cy0 + yo + y) : 0;
            pcm[2].c[pl][i] = ta ? cs(pl, cx0 + xo + x, cy0 - 1) : 0;
          }
      }
    int cm = 0, scm = 1 << 30;
    for (int k = 0; k < 3; ++k) {
      if ((k == 1 && !la) || (k == 2 && !ta)) continue;
      int sd = 0;
      for (int pl = 0; pl < 2; ++pl)
        for (int i = 0; i < 64; ++i) sd += std::abs(cur.c[pl][i] - pcm[k].c[pl][i]);
      if (sd < scm) {
        scm = sd;
        cm = k;
      }
    }
    content::MbPix pred = use4 ? p4 : p16[pm];
    std::memcpy(pred.c, pcm[cm].c, sizeof pred.c);
    const int cc = content::quant_chroma(cur, pred, qpc(0), qpc(1), 1.0 / 3.0, &L);
    if (use4) {
      int cbp = cc << 4;
      for (int b = 0; b < 16; ++b)
        for (int v : L.l4[b])
          if (v) cbp |= 1 << ((b >> 3) * 2 + ((b & 3) >> 1));
      put_i_type(a, 0, base);
      if (t8mode_) put_t8(a, false);
      for (int k = 0; k < 16; ++k) {
        const int bx = kBlkX[k], by = kBlkY[k];
        const Loc LA = loc(a, bx * 4 - 1, by * 4, 16), LB = loc(a, bx * 4, by * 4 - 1, 16);
        int pred_m = 2;
        if (!(LA.mb < 0 || LB.mb < 0 || (cip_ && !intra(LA.mb)) || (cip_ && !intra(LB.mb)))) {
          const GMb &ma = mb_[static_cast<size_t>(LA.mb)], &mb = mb_[static_cast<size_t>(LB.mb)];
          const int pa4 = ma.type == 1 ? ma.i4[(LA.yw / 4) * 4 + LA.xw / 4] : 2;
          const int pb4 = mb.type == 1 ? mb.i4[(LB.yw / 4) * 4 + LB.xw / 4] : 2;
          pred_m = imin(pa4, pb4);
        }
        const int md = mode4[k];
        put_pred_mode(md == pred_m, md < pred_m ? md : md - 1);
        m.i4[by * 4 + bx] = md;
      }
      put_chroma_mode(a, cm);
      put_cbp(a, cbp, true);
      if (cbp) write_qp_delta();
      write_residual(a, cbp, false, &L);
      recon_chroma(a, pred, L);
      set_rec(a, kMbI4x4, false, &L);
      return;
    }
    m.type = 2;
    for (int i = 0; i < 16; ++i) m.i4[i] = 2;
    const int lum = content::quant_luma(cur, pred, qp_, 1.0 / 3.0, true, false, &L);
    const int cbp = lum | (cc << 4);
    m.cbp = cbp;
    put_i_type(a, 1 + pm + 4 * cc + (lum ? 12 : 0), base);
    put_chroma_mode(a, cm);
    write_qp_delta();
    write_residual(a, cbp, true, &L);
    recon_luma(a, pred, L, true, false);
    recon_chroma(a, pred, L);
    set_rec(a, kMbI16, false, &L);
  }

  // 8.2.4.2.3 list initialisation (no modification) from the writer's DPB
  void b_lists() {
    std::vector<const RefPic *> st;
    for (const RefPic &r : dpb_) st.push_back(&r);
    std::sort(st.begin(), st.end(), [](const RefPic *a, const RefPic *b) { return a->poc < b->poc; });
    std::vector<int> l0, l1;
    for (int i = static_cast<int>(st.size()) - 1; i >= 0; --i) if (st[i]->poc < cur_poc_) l0.push_back(st[i]->d);
    for (const RefPic *r : st) if (r->poc > cur_poc_) l0.push_back(r->d);
    for (const RefPic *r : st) if (r->poc > cur_poc_) l1.push_back(r->d);
    for (int i = static_cast<int>(st.size()) - 1; i >= 0; --i) if (st[i]->poc < cur_poc_) l1.push_back(st[i]->d);
    if (l1.size() > 1 && l0 == l1) std::swap(l1[0], l1[1]);
    for (size_t i = 0; i < l0.size(); ++i) lst_[0][i] = l0[i];
    for (size_t i = 0; i < l1.size(); ++i) lst_[1][i] = l1[i];
    nlst_[0] = static_cast<int>(l0.size());
    nlst_[1] = static_cast<int>(l1.size());
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
      if (cabac_ && !idr) bw.ue(0);  // cabac_init_idc
      qp_ = pic_qp;
      bw.se(pic_qp - 26);
      const uint32_t dr = rng_.below(20);
      const int didc = dr < 16 ? 0 : (dr < 18 ? 2 : 1);
      bw.ue(static_cast<uint32_t>(didc));
      if (didc != 1) {
        bw.se(static_cast<int>(rng_.below(7)) - 3);
        bw.se(static_cast<int>(rng_.below(7)) - 3);
      }
      if (cabac_) {  // cabac_alignment_one_bit, then 9.3.1 initialisation
        while (!bw.aligned()) bw.bit(1);
        cab_.init(&bw, idr, pic_qp);
      }
      write_slice_data(first, last, slice, !idr, pan_x, pan_y);
      if (cabac_) bw.align_zero();  // the flush wrote the rbsp_stop_one_bit
      else bw.trailing();
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


// B mode (edge_cases bit 5): mini-GOPs of 1..4 display frames coded anchor
// first (P, reference), then the B pictures between (the middle one of three a
// reference picture half the time: a B-picture colocated for the others), POC
// type 0 (2 x display distance from the IDR, 6-bit lsb so it wraps), list
// initialisation by POC, spatial or (bit 8) temporal direct prediction,
// explicit (bit 6) or implicit (bit 7) weighted prediction.  The MP4 carries
// composition offsets (display = decode position + 2 - reorder).
void FullWriter::run_b() {
  bmode_ = true;
  const int ec = P_.edge_cases;
  const double fps = double(P_.fps_num) / P_.fps_den;
  const int gop_max = std::max(1, static_cast<int>(P_.gop_max_s * fps));
  auto scene_len = [&]() {
    const double lo = std::max(P_.cut_min_s, 1.0 / fps), hi = std::max(P_.cut_max_s, lo);
    return std::max<int64_t>(1, static_cast<int64_t>((lo + (hi - lo) * rng_.uniform()) * fps + 0.5));
  };
  const int64_t nf = ck_->nf;
  std::vector<uint8_t> cut(static_cast<size_t>(nf), 0);
  std::vector<int> pxs(static_cast<size_t>(nf)), pys(static_cast<size_t>(nf));
  weighted_ = (ec & 64) ? 1 : ((ec & 128) ? 2 : 0);
  if (content_) {
    scene_of_.assign(static_cast<size_t>(nf), 0);
    offx_.assign(static_cast<size_t>(nf), 0);
    offy_.assign(static_cast<size_t>(nf), 0);
  }
  {
    int64_t next_cut = scene_len();
    int pan_x = 0, pan_y = 0;
    for (int64_t f = 0; f < nf; ++f) {
      const bool c = f == 0 || f == next_cut;
      if (f == next_cut) next_cut = f + scene_len();
      cut[static_cast<size_t>(f)] = c;
      if (c && ck_->f0 + f > 0) ck_->cuts.push_back(ck_->f0 + f);
      if (f % P_.fps_num == 0 || c) {
        if (content_) {  // whole-pel even pans (luma samples per frame x 4)
          const int h = P_.max_motion / 2;
          pan_x = 8 * (static_cast<int>(rng_.below(static_cast<uint32_t>(2 * h + 1))) - h);
          pan_y = 8 * (static_cast<int>(rng_.below(static_cast<uint32_t>(2 * h + 1))) - h);
        } else {
          const int m = 4 * P_.max_motion;
          pan_x = static_cast<int>(rng_.below(static_cast<uint32_t>(2 * m + 1))) - m;
          pan_y = static_cast<int>(rng_.below(static_cast<uint32_t>(2 * m + 1))) - m;
        }
        if (rng_.below(4) == 0) pan_x = pan_y = 0;
      }
      pxs[static_cast<size_t>(f)] = pan_x;
      pys[static_cast<size_t>(f)] = pan_y;
      if (content_) {
        const size_t u = static_cast<size_t>(f);
        if (c) {
          scenes_.emplace_back();
          content::make_scene(&scenes_.back(), f, mbw_ * 16, mbh_ * 16, P_.max_motion, tex_rng_);
          offx_[u] = offy_[u] = 0;
        } else {
          offx_[u] = offx_[u - 1] + pan_x / 4;
          offy_[u] = offy_[u - 1] + pan_y / 4;
        }
        scene_of_[u] = static_cast<int>(scenes_.size()) - 1;
      }
    }
  }
  struct Pic {
    int64_t d;
    int kind;  // 0 IDR, 1 P, 2 B
    bool ref;
  };
  std::vector<Pic> order;
  {
    int64_t d = 0, since_idr = 0;
    while (d < nf) {
      if (cut[static_cast<size_t>(d)] || since_idr >= gop_max) {
        order.push_back({d, 0, true});
        since_idr = 1;
        ++d;
        continue;
      }
      int64_t lim = d;
      while (lim < nf && !cut[static_cast<size_t>(lim)] && since_idr + (lim - d) < gop_max) ++lim;
      const int64_t g = std::min<int64_t>(1 + rng_.below(4), lim - d);
      const int64_t a = d + g - 1;
      order.push_back({a, 1, true});
      if (g >= 4 && rng_.below(2)) {
        const int64_t mid = d + (g - 1) / 2;
        order.push_back({mid, 2, true});
        for (int64_t x = d; x < a; ++x)
          if (x != mid) order.push_back({x, 2, false});
      } else {
        for (int64_t x = d; x < a; ++x) order.push_back({x, 2, rng_.below(8) == 0});
      }
      since_idr += g;
      d = a + 1;
    }
  }
  const int spr = P_.slices_per_row;
  const int slice_mbs = spr > 0 ? (mbw_ + spr - 1) / spr : nmb_;
  int frame_num = 0, prev_ref_fn = 0, idr_id = ck_->idr_id_base;
  int64_t d_idr = 0;
  std::vector<uint8_t> sample;
  for (size_t p = 0; p < order.size(); ++p) {
    const Pic &pc = order[p];
    const bool idr = pc.kind == 0, is_b = pc.kind == 2;
    cur_d_ = static_cast<int>(pc.d);
    if (idr) {
      frame_num = 0;
      dpb_.clear();
      d_idr = pc.d;
    } else {
      frame_num = (prev_ref_fn + 1) & ((1 << kLog2MaxFrameNum) - 1);
    }
    cur_poc_ = static_cast<int>(2 * (pc.d - d_idr));
    // reference lists (no modification in B mode)
    if (is_b) {
      b_lists();
    } else {
      std::vector<const RefPic *> st;
      for (const RefPic &r : dpb_) st.push_back(&r);
      auto wrap = [&](const RefPic *r) { return r->fn > frame_num ? r->fn - (1 << kLog2MaxFrameNum) : r->fn; };
      std::stable_sort(st.begin(), st.end(), [&](const RefPic *a, const RefPic *b) { return wrap(a) > wrap(b); });
      for (size_t i = 0; i < st.size(); ++i) lst_[0][i] = st[i]->d;
      nlst_[0] = static_cast<int>(st.size());
      nlst_[1] = 0;
    }
    if (!idr) {
      nlst_[0] = 1 + static_cast<int>(rng_.below(static_cast<uint32_t>(nlst_[0])));
      if (is_b) nlst_[1] = 1 + static_cast<int>(rng_.below(static_cast<uint32_t>(nlst_[1])));
    }
    col_ = is_b ? pic_of(lst_[1][0]) : nullptr;
    spatial_ = true;
    if (is_b && (ec & 256) && !content_ && rng_.below(2)) {
      // temporal direct only when every colocated reference is in RefPicList0
      bool ok = true;
      for (const GMb &cm : col_->mbs)
        for (int b = 0; b < 16 && ok; ++b)
          for (int l = 0; l < 2; ++l) {
            if (cm.ref[l][b] < 0 || (cm.type >= 1 && cm.type <= 3)) continue;
            bool found = false;
            for (int i = 0; i < nlst_[0]; ++i) found |= lst_[0][i] == cm.refd[l][b];
            ok &= found;
          }
      spatial_ = !ok;
    }
    const int slice_type = idr ? (rng_.below(2) ? 7 : 2) : (is_b ? (rng_.below(2) ? 6 : 1) : (rng_.below(2) ? 5 : 0));
    // content: x264-like QP offsets between I, P, reference B and B pictures
    const int pic_qp = content_ ? (idr ? 24 : (is_b ? (pc.ref ? 27 : 28) : 26)) : 20 + static_cast<int>(rng_.below(17));
    const bool wp = !idr && (ec & 64) != 0;   // explicit weights (weighted_pred_flag / weighted_bipred_idc 1)
    sample.clear();
    int slice = 0;
    if (content_) {
      rec_.assign(static_cast<size_t>(W()) * H() * 3 / 2, 0);
      mrec_.assign(static_cast<size_t>(nmb_), MbRec{});
      mrec1_.assign(static_cast<size_t>(nmb_), MbRecB{});
    }
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
      bw.u(6, static_cast<uint32_t>(cur_poc_ & 63));  // pic_order_cnt_lsb
      if (is_b) bw.u(1, spatial_ ? 1 : 0);
      if (!idr) {
        nref_ = nlst_[0];
        bw.u(1, 1);  // num_ref_idx_active_override_flag
        bw.ue(static_cast<uint32_t>(nlst_[0] - 1));
        if (is_b) bw.ue(static_cast<uint32_t>(nlst_[1] - 1));
        bw.u(1, 0);  // ref_pic_list_modification_flag_l0
        if (is_b) bw.u(1, 0);
      }
      if (wp) {  // pred_weight_table (7.3.3.2)
        const int lwd = static_cast<int>(rng_.below(7)), cwd = static_cast<int>(rng_.below(7));
        bw.ue(static_cast<uint32_t>(lwd));
        bw.ue(static_cast<uint32_t>(cwd));
        for (int l = 0; l < 1 + is_b; ++l)
          for (int i = 0; i < nlst_[l]; ++i) {
            if (rng_.below(3)) {
              bw.u(1, 1);
              bw.se((1 << lwd) + static_cast<int>(rng_.below(17)) - 8);
              bw.se(static_cast<int>(rng_.below(21)) - 10);
            } else {
              bw.u(1, 0);
            }
            if (rng_.below(2)) {
              bw.u(1, 1);
              for (int j = 0; j < 2; ++j) {
                bw.se((1 << cwd) + static_cast<int>(rng_.below(9)) - 4);
                bw.se(static_cast<int>(rng_.below(11)) - 5);
              }
            } else {
              bw.u(1, 0);
            }
          }
      }
      if (pc.ref) {  // dec_ref_pic_marking
        if (idr) { bw.u(1, 0); bw.u(1, 0); }
        else bw.u(1, 0);
      }
      if (cabac_ && !idr) bw.ue(0);  // cabac_init_idc
      qp_ = pic_qp;
      bw.se(pic_qp - 26);
      const uint32_t dr = content_ ? 0u : rng_.below(20);
      const int didc = dr < 16 ? 0 : (dr < 18 ? 2 : 1);
      bw.ue(static_cast<uint32_t>(didc));
      if (didc != 1) {
        bw.se(content_ ? 0 : static_cast<int>(rng_.below(7)) - 3);
        bw.se(content_ ? 0 : static_cast<int>(rng_.below(7)) - 3);
      }
      if (cabac_) {
        while (!bw.aligned()) bw.bit(1);
        cab_.init(&bw, idr, pic_qp);
      }
      const int pxn = pxs[static_cast<size_t>(pc.d)], pyn = pys[static_cast<size_t>(pc.d)];
      if (is_b) write_slice_data_b(first, last, slice, pxn, pyn);
      else write_slice_data(first, last, slice, !idr, pxn, pyn);
      if (cabac_) bw.align_zero();
      else bw.trailing();
      append_nal(sample, idr ? 0x65 : (pc.ref ? 0x41 : 0x01), bw.data());
      first = last;
    }
    bw_ = nullptr;
    if (content_) {
      deblock_picture(0, 0, 0);  // every content slice: idc 0, offsets 0
      if (P_.hash_frames) {      // display-size NV12 of the reconstruction (= a decoder's output)
        uint64_t h = 0, j = 0;
        const int w = W();
        for (int yy = 0; yy < P_.height; ++yy)
          for (int xx = 0; xx < P_.width; ++xx, ++j) h += uint64_t(rec_[size_t(yy) * w + xx]) * ((j % 65521) + 1);
        const uint8_t *UV = rec_.data() + static_cast<size_t>(w) * H();
        for (int yy = 0; yy < P_.height / 2; ++yy)
          for (int xx = 0; xx < P_.width; ++xx, ++j) h += uint64_t(UV[size_t(yy) * w + xx]) * ((j % 65521) + 1);
        ck_->recon_hash += h * uint64_t(ck_->f0 + cur_d_ + 1);
      }
    }
    if (idr) {
      idr_id ^= 1;
      ++ck_->n_idr;
    }
    if (pc.ref) {
      if (static_cast<int>(dpb_.size()) >= kMaxRefs) {  // sliding window (8.2.5.3)
        size_t o = 0;
        auto wrap = [&](const RefPic &r) { return r.fn > frame_num ? r.fn - (1 << kLog2MaxFrameNum) : r.fn; };
        for (size_t i = 1; i < dpb_.size(); ++i)
          if (wrap(dpb_[i]) < wrap(dpb_[o])) o = i;
        dpb_.erase(dpb_.begin() + static_cast<int64_t>(o));
      }
      dpb_.push_back(RefPic{cur_d_, cur_poc_, frame_num, mb_, content_ ? rec_ : std::vector<uint8_t>{}});
      prev_ref_fn = frame_num;
    }
    if (content_) prune_sources();
    ck_->data.insert(ck_->data.end(), sample.begin(), sample.end());
    ck_->size.push_back(static_cast<uint32_t>(sample.size()));
    ck_->sync.push_back(idr ? 1 : 0);
    ck_->cts.push_back(static_cast<uint32_t>(pc.d - static_cast<int64_t>(p) + 2));
    if (const char *dump = std::getenv("VTS_SYNTH_MVDUMP")) {  // debugging aid (see the oracle's FO_MVDUMP)
      if (FILE *df = std::fopen(dump, "a")) {
        for (int a = 0; a < nmb_; ++a)
          for (int k = 0; k < 16; ++k)
            for (int l = 0; l < 2; ++l) {
              const GMb &m = mb_[static_cast<size_t>(a)];
              const bool in = m.type >= 1 && m.type <= 3;
              const int r = in ? -1 : m.ref[l][k];
              std::fprintf(df, "%lld %d %d %d %d %d %d\n", static_cast<long long>(ck_->f0 + static_cast<int64_t>(p)), a,
                           k, l, r, r >= 0 ? m.mv[l][k][0] : 0, r >= 0 ? m.mv[l][k][1] : 0);
            }
        std::fclose(df);
      }
    }
  }
}

}  // namespace

void encode_chunk_full(const vts_synth_params &P, SynthChunk *ck) {
  if ((P.edge_cases & 16384) && (!(P.edge_cases & 32) || (P.edge_cases & (64 | 256 | 16)))) {
    ck->error = "content mode (edge_cases bit 14) needs B mode (bit 5) without explicit weights, temporal direct "
                "or constrained intra";
    return;
  }
  FullWriter w(P, ck);
  if (P.edge_cases & 32) w.run_b();
  else w.run();
}

// Constrained Baseline SPS / PPS of the full-syntax streams: 3 reference
// frames, frame_num wrapping at 16, POC type 2, deblocking control present,
// two active references by default, chroma QP offset from the seed.

// 7.3.2.1.1.1 scaling_list() for lists 0..n-1 (16 values each for 0..5, 64
// for 6, 7), each chosen from the seed: absent (the fall-back rules apply),
// useDefaultScalingMatrixFlag, a list that ends early (nextScale 0: the rest
// repeat the last value) or a full list of values 4..64
void write_scaling_lists(BitWriter &w, int n, uint64_t seed) {
  uint64_t x = seed * 0x9E3779B97F4A7C15ull + 0x2545F4914F6CDD1Dull;
  auto rnd = [&](uint32_t m) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return static_cast<uint32_t>(x % m);
  };
  for (int i = 0; i < n; ++i) {
    const uint32_t kind = rnd(4);  // 0 absent, 1 default, 2 early end, 3 full
    w.u(1, kind ? 1 : 0);          // scaling_list_present_flag
    if (!kind) continue;
    if (kind == 1) {
      w.se(-8);  // nextScale 0 at j = 0
      continue;
    }
    const int size = i < 6 ? 16 : 64;
    const int stop = kind == 2 ? 1 + static_cast<int>(rnd(static_cast<uint32_t>(size - 1))) : size;
    int last = 8;
    for (int j = 0; j < stop; ++j) {
      const int next = 4 + static_cast<int>(rnd(61));
      int delta = next - last;
      if (delta > 127) delta -= 256;
      if (delta < -128) delta += 256;
      w.se(delta);
      last = next;
    }
    if (stop < size) w.se(-last);  // nextScale 0: the remaining entries repeat the last
  }
}
void make_sps_pps_full(const vts_synth_params &P, int level, std::vector<uint8_t> *sps_nal,
                       std::vector<uint8_t> *pps_nal) {
  const int mbw = (P.width + 15) / 16, mbh = (P.height + 15) / 16;
  const int crop_r = mbw * 16 - P.width, crop_b = mbh * 16 - P.height;
  const bool bm = (P.edge_cases & 32) != 0;
  const bool cabac = (P.edge_cases & 1024) != 0, t8 = cabac && (P.edge_cases & 2048) != 0;
  // bits 12 / 13: scaling matrices in the SPS / the PPS (High profile)
  const bool sps_scale = (P.edge_cases & 4096) != 0, pps_scale = (P.edge_cases & 8192) != 0;
  const int profile = (t8 || sps_scale || pps_scale) ? 100 : ((bm || cabac) ? 77 : 66);  // High / Main / Constrained Baseline
  BitWriter s;
  s.u(8, static_cast<uint32_t>(profile));
  s.u(8, profile == 66 ? 0xC0 : 0x00);
  s.u(8, static_cast<uint32_t>(level));
  s.ue(0);
  if (profile == 100) {
    s.ue(1);    // chroma_format_idc 4:2:0
    s.ue(0);    // bit_depth_luma_minus8
    s.ue(0);    // bit_depth_chroma_minus8
    s.u(1, 0);  // qpprime_y_zero_transform_bypass_flag
    s.u(1, sps_scale ? 1 : 0);  // seq_scaling_matrix_present_flag
    if (sps_scale) write_scaling_lists(s, 8, P.seed * 2 + 1);
  }
  s.ue(kLog2MaxFrameNum - 4);
  if (bm) {
    s.ue(0);  // pic_order_cnt_type 0
    s.ue(2);  // log2_max_pic_order_cnt_lsb_minus4: 6-bit lsb
  } else {
    s.ue(2);
  }
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
  p.u(1, cabac ? 1 : 0);                       // entropy_coding_mode_flag
  p.u(1, 0);
  p.ue(0);
  p.ue(kPpsRefDefault - 1);
  p.ue(0);
  p.u(1, (bm && (P.edge_cases & 64)) ? 1 : 0);                           // weighted_pred_flag
  p.u(2, !bm ? 0u : ((P.edge_cases & 64) ? 1u : ((P.edge_cases & 128) ? 2u : 0u)));  // weighted_bipred_idc
  p.se(0);                                     // pic_init_qp 26
  p.se(0);
  p.se(static_cast<int>(P.seed % 5) - 2);      // chroma_qp_index_offset
  p.u(1, 1);                                   // deblocking_filter_control_present_flag
  p.u(1, (P.edge_cases & 16) ? 1 : 0);         // constrained_intra_pred_flag
  p.u(1, 0);
  if (t8 || pps_scale) {
    p.u(1, t8 ? 1 : 0);                        // transform_8x8_mode_flag
    p.u(1, pps_scale ? 1 : 0);                 // pic_scaling_matrix_present_flag
    if (pps_scale) write_scaling_lists(p, 6 + (t8 ? 2 : 0), P.seed * 2 + 2);
    p.se(static_cast<int>(P.seed % 3) - 1);    // second_chroma_qp_index_offset
  }
  p.trailing();
  pps_nal->clear();
  pps_nal->push_back(0x68);
  append_ebsp(*pps_nal, p.data().data(), p.data().size());
}

}  // namespace vts
