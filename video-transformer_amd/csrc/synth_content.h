// synth_content.h — the content mode of the full-syntax writer
// (vts_synth_params.edge_cases bit 14; synth_full.cpp).  The noise streams
// make every syntax decision from a random stream; a content stream codes
// pictures: textured scenes with planted cuts (a new texture, an IDR), a
// panning background and a few textured sprites moving on their own, coded
// with mode decisions (skip / direct / 16x16 motion / intra) by SAD and
// residuals quantised from the source's prediction error.
//
// Closed loop: the writer reconstructs every macroblock the way a decoder does
// (whole-pel motion, implicit bi-prediction weights, the intra modes it uses,
// the decoder's own scaling + inverse transforms and deblocking filter from
// recon_full.h) and predicts from that reconstruction, so the decoded pictures
// follow the source within the quantisation error and do not drift.  Motion
// is whole-pel and even (chroma whole-pel too).
//
// Quantisation inverts the decoder's own scaling + inverse transforms
// (8.5.10 - 8.5.13, flat scaling lists): the transforms' basis rows are
// orthogonal, so the level of coefficient (i, j) that best reproduces a
// residual X is 64 (M X M^T)_ij / (n_i n_j s_ij) (M the inverse transform's
// basis rows, n their squared norms, s_ij the decoder's scale per level),
// rounded with the usual dead zone (1/3 intra, 1/6 inter).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "h264_cabac_tables.h"
#include "h264_tables.h"
#include "synth.h"

namespace vts {
namespace content {

struct Frame {  // coded size; chroma planes w/2 x h/2
  int w = 0, h = 0;
  std::vector<uint8_t> y, u, v;
  void alloc(int cw, int ch) {
    w = cw;
    h = ch;
    y.assign(size_t(w) * h, 0);
    u.assign(size_t(w / 2) * (h / 2), 128);
    v.assign(size_t(w / 2) * (h / 2), 128);
  }
};

inline int wrapi(int v, int n) {
  v %= n;
  return v < 0 ? v + n : v;
}
inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

struct Sprite {
  int x0, y0;  // top-left at the scene's first frame (luma, even)
  int vx, vy;  // luma samples per frame (even)
  Frame tex;
};
struct Scene {
  int64_t d0 = 0;  // first display frame
  Frame bg;
  std::vector<Sprite> spr;
};

inline void make_scene(Scene *s, int64_t d0, int w, int h, int max_motion, Pcg32 &rng) {
  s->d0 = d0;
  s->bg.alloc(w, h);
  synth_texture(s->bg.y.data(), s->bg.u.data(), s->bg.v.data(), w, h, rng, false);
  s->spr.clear();
  const int n = 2 + static_cast<int>(rng.below(4));
  const int m = std::max(1, max_motion / 2);
  for (int k = 0; k < n; ++k) {
    Sprite sp;
    const int sw = 2 * (24 + static_cast<int>(rng.below(57))), sh = 2 * (24 + static_cast<int>(rng.below(57)));
    sp.x0 = 2 * static_cast<int>(rng.below(static_cast<uint32_t>(w / 2)));
    sp.y0 = 2 * static_cast<int>(rng.below(static_cast<uint32_t>(h / 2)));
    sp.vx = 2 * (static_cast<int>(rng.below(static_cast<uint32_t>(2 * m + 1))) - m);
    sp.vy = 2 * (static_cast<int>(rng.below(static_cast<uint32_t>(2 * m + 1))) - m);
    sp.tex.alloc(sw, sh);
    synth_texture(sp.tex.y.data(), sp.tex.u.data(), sp.tex.v.data(), sw, sh, rng, false);
    s->spr.push_back(std::move(sp));
  }
}

// the source picture of display frame d: the background shifted by the
// scene's accumulated pan (ox, oy) (wrapping), the sprites on top (wrapping)
inline void render(const Scene &s, int64_t d, int ox, int oy, Frame *f) {
  const int w = f->w, h = f->h, cw = w / 2, ch = h / 2;
  for (int y = 0; y < h; ++y) {
    const uint8_t *src = &s.bg.y[size_t(wrapi(y + oy, h)) * w];
    uint8_t *dst = &f->y[size_t(y) * w];
    const int x0 = wrapi(ox, w);
    std::memcpy(dst, src + x0, size_t(w - x0));
    std::memcpy(dst + (w - x0), src, size_t(x0));
  }
  for (int pl = 0; pl < 2; ++pl) {
    const std::vector<uint8_t> &sp = pl ? s.bg.v : s.bg.u;
    std::vector<uint8_t> &dp = pl ? f->v : f->u;
    const int x0 = wrapi(ox / 2, cw);
    for (int y = 0; y < ch; ++y) {
      const uint8_t *src = &sp[size_t(wrapi(y + oy / 2, ch)) * cw];
      uint8_t *dst = &dp[size_t(y) * cw];
      std::memcpy(dst, src + x0, size_t(cw - x0));
      std::memcpy(dst + (cw - x0), src, size_t(x0));
    }
  }
  const int64_t t = d - s.d0;
  for (const Sprite &sp : s.spr) {
    const int px = wrapi(static_cast<int>(sp.x0 + sp.vx * t), w), py = wrapi(static_cast<int>(sp.y0 + sp.vy * t), h);
    for (int y = 0; y < sp.tex.h; ++y) {
      const int yy = wrapi(py + y, h);
      for (int x = 0; x < sp.tex.w; ++x) f->y[size_t(yy) * w + wrapi(px + x, w)] = sp.tex.y[size_t(y) * sp.tex.w + x];
    }
    for (int y = 0; y < sp.tex.h / 2; ++y) {
      const int yy = wrapi(py / 2 + y, ch);
      for (int x = 0; x < sp.tex.w / 2; ++x) {
        const int xx = wrapi(px / 2 + x, cw);
        f->u[size_t(yy) * cw + xx] = sp.tex.u[size_t(y) * (sp.tex.w / 2) + x];
        f->v[size_t(yy) * cw + xx] = sp.tex.v[size_t(y) * (sp.tex.w / 2) + x];
      }
    }
  }
}

// Sprite k's luma position at display frame d (unwrapped)
inline void sprite_pos(const Scene &s, int k, int64_t d, int *x, int *y) {
  const Sprite &sp = s.spr[static_cast<size_t>(k)];
  *x = static_cast<int>(sp.x0 + sp.vx * (d - s.d0));
  *y = static_cast<int>(sp.y0 + sp.vy * (d - s.d0));
}

// Macroblock-sized samples: luma 16 x 16, Cb / Cr 8 x 8
struct MbPix {
  int y[256], c[2][64];
};

// 8.4.2.2 for whole-pel even luma motion (quarter-sample units, multiples of
// 8): reference samples at clamped coordinates, chroma at half the offset
inline void predict(const Frame &r, int mbx, int mby, int mvx, int mvy, MbPix *p) {
  const int dx = mvx >> 2, dy = mvy >> 2, cw = r.w / 2, ch = r.h / 2;
  for (int y = 0; y < 16; ++y) {
    const int yy = clampi(mby * 16 + y + dy, 0, r.h - 1);
    for (int x = 0; x < 16; ++x) p->y[y * 16 + x] = r.y[size_t(yy) * r.w + clampi(mbx * 16 + x + dx, 0, r.w - 1)];
  }
  for (int y = 0; y < 8; ++y) {
    const int yy = clampi(mby * 8 + y + dy / 2, 0, ch - 1);
    for (int x = 0; x < 8; ++x) {
      const size_t o = size_t(yy) * cw + clampi(mbx * 8 + x + dx / 2, 0, cw - 1);
      p->c[0][y * 8 + x] = r.u[o];
      p->c[1][y * 8 + x] = r.v[o];
    }
  }
}
inline void source_mb(const Frame &f, int mbx, int mby, MbPix *p) { predict(f, mbx, mby, 0, 0, p); }

inline int sad_luma(const MbPix &a, const MbPix &b) {
  int s = 0;
  for (int i = 0; i < 256; ++i) s += std::abs(a.y[i] - b.y[i]);
  return s;
}
inline int sad_all(const MbPix &a, const MbPix &b) {
  int s = sad_luma(a, b);
  for (int pl = 0; pl < 2; ++pl)
    for (int i = 0; i < 64; ++i) s += std::abs(a.c[pl][i] - b.c[pl][i]);
  return s;
}

// ------------------------------------------------------------ quantisation
struct Levels {
  int dc16[16];       // Intra16x16DCLevel, scan order
  int l4[16][16];     // luma 4x4 blocks by raster index, scan order (Intra_16x16: AC, scan 1..15 at 0..14)
  int l8[4][64];      // luma 8x8 blocks (raster), scan order
  int cdc[2][4];      // chroma DC, c0..c3
  int cac[2][4][15];  // chroma AC by raster 4x4 block, scan 1..15
};

struct Basis {
  double m4[4][4], n4[4], m8[8][8], n8[8];
  Basis() {
    const double r4[4][4] = {{1, 1, 1, 1}, {1, 0.5, -0.5, -1}, {1, -1, -1, 1}, {0.5, -1, 1, -0.5}};
    for (int i = 0; i < 4; ++i) {
      n4[i] = 0;
      for (int j = 0; j < 4; ++j) {
        m4[i][j] = r4[i][j];
        n4[i] += r4[i][j] * r4[i][j];
      }
    }
    // rows of the 8x8 inverse transform (8.5.13.2): the butterfly of one
    // unit coefficient, >> 1 / >> 2 taken as exact halves / quarters
    for (int j = 0; j < 8; ++j) {
      double v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      v[j] = 1;
      const double a0 = v[0] + v[4], a4 = v[0] - v[4], a2 = v[2] * 0.5 - v[6], a6 = v[2] + v[6] * 0.5;
      const double b0 = a0 + a6, b2 = a4 + a2, b4 = a4 - a2, b6 = a0 - a6;
      const double a1 = -v[3] + v[5] - v[7] - v[7] * 0.5, a3 = v[1] + v[7] - v[3] - v[3] * 0.5;
      const double a5 = -v[1] + v[7] + v[5] + v[5] * 0.5, a7 = v[3] + v[5] + v[1] + v[1] * 0.5;
      const double b1 = a1 + a7 * 0.25, b7 = a7 - a1 * 0.25, b3 = a3 + a5 * 0.25, b5 = a3 * 0.25 - a5;
      const double o[8] = {b0 + b7, b2 + b5, b4 + b3, b6 + b1, b6 - b1, b4 - b3, b2 - b5, b0 - b7};
      n8[j] = 0;
      for (int k = 0; k < 8; ++k) {
        m8[j][k] = o[k];
        n8[j] += o[k] * o[k];
      }
    }
  }
};
inline const Basis &basis() {
  static const Basis b;
  return b;
}

inline int deadzone(double l, double dz) {
  const int a = static_cast<int>(std::fabs(l) + dz);  // floor of a non-negative value
  const int c = std::min(a, 2047);
  return l < 0 ? -c : c;
}
inline double pow2(int e) { return std::ldexp(1.0, e); }

// 4x4 block x (raster) at qp -> levels in raster order.  The basis rows
// are the forward core transform's rows Cf scaled by c = (1, 1/2, 1, 1/2), so
// (M X M^T)_ij = c_i c_j (Cf X Cf^T)_ij: integer butterflies, then one factor
// per position and qp
struct Quant4Tab {
  double k[52][16];    // 64 c_i c_j / (n_i n_j s_ij)
  double kmax[52];     // max over (i, j) of k_ij max|Cf_i| max|Cf_j|: |level| <= kmax sum |x|
  Quant4Tab() {
    const double c[4] = {1, 0.5, 1, 0.5}, n[4] = {4, 2.5, 4, 2.5};
    for (int qp = 0; qp < 52; ++qp) {
      kmax[qp] = 0;
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
          const int cls = (!(i & 1) && !(j & 1)) ? 0 : (((i & 1) && (j & 1)) ? 1 : 2);
          const double sij = h264::kNormV[qp % 6][cls] * std::ldexp(1.0, qp / 6);
          k[qp][i * 4 + j] = 64.0 * c[i] * c[j] / (n[i] * n[j] * sij);
          kmax[qp] = std::max(kmax[qp], k[qp][i * 4 + j] * (1 + (i & 1)) * (1 + (j & 1)));
        }
    }
  }
};
inline const Quant4Tab &quant4_tab() {
  static const Quant4Tab t;
  return t;
}
inline void quant4(const int *x, int qp, double dz, int *lev) {
  const Quant4Tab &T = quant4_tab();
  int sa = 0;
  for (int i = 0; i < 16; ++i) sa += std::abs(x[i]);
  // below the dead zone everywhere -> all zero
  if (sa * T.kmax[qp] + dz < 1.0) {
    std::memset(lev, 0, 16 * sizeof(int));
    return;
  }
  int t[16], w[16];
  for (int i = 0; i < 4; ++i) {
    const int a = x[i * 4], b = x[i * 4 + 1], c = x[i * 4 + 2], d = x[i * 4 + 3];
    t[i * 4] = a + b + c + d;
    t[i * 4 + 1] = 2 * a + b - c - 2 * d;
    t[i * 4 + 2] = a - b - c + d;
    t[i * 4 + 3] = a - 2 * b + 2 * c - d;
  }
  for (int j = 0; j < 4; ++j) {
    const int a = t[j], b = t[4 + j], c = t[8 + j], d = t[12 + j];
    w[j] = a + b + c + d;
    w[4 + j] = 2 * a + b - c - 2 * d;
    w[8 + j] = a - b - c + d;
    w[12 + j] = a - 2 * b + 2 * c - d;
  }
  // w = Cf X Cf^T, raster (row i = vertical frequency)
  for (int k = 0; k < 16; ++k) lev[k] = deadzone(w[k] * T.k[qp][k], dz);
}

// 8x8 block x (raster) -> levels in raster order
inline void quant8(const int *x, int qp, double dz, int *lev) {
  static const uint8_t kN8[6][6] = VTS_NORM8_DATA;
  int any = 0;
  for (int i = 0; i < 64; ++i) any |= x[i];
  if (!any) {
    std::memset(lev, 0, 64 * sizeof(int));
    return;
  }
  const Basis &B = basis();
  double t[8][8];
  for (int i = 0; i < 8; ++i)
    for (int c = 0; c < 8; ++c) {
      double s = 0;
      for (int r = 0; r < 8; ++r) s += B.m8[i][r] * x[r * 8 + c];
      t[i][c] = s;
    }
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) {
      double w = 0;
      for (int c = 0; c < 8; ++c) w += t[i][c] * B.m8[j][c];
      const double s = kN8[qp % 6][vts_norm8_class(i, j)] * pow2(qp / 6) / 4.0;
      lev[i * 8 + j] = deadzone(64.0 * w / (B.n8[i] * B.n8[j] * s), dz);
    }
}

// Quantise a macroblock's luma residual (source - prediction).  i16:
// Intra_16x16 (DC through 8.5.10's Hadamard, AC at scan 1..15); t8: 8x8
// transforms.  Returns the luma bits of coded_block_pattern (Intra_16x16: 0
// or 15, AC anywhere).
inline int quant_luma(const MbPix &src, const MbPix &pred, int qp, double dz, bool i16, bool t8, Levels *L) {
  static const uint8_t kZ4[16] = VTS_ZZ_DATA;
  static const uint8_t kZ8[64] = VTS_ZZ8_DATA;
  int res[256], any = 0;
  for (int i = 0; i < 256; ++i) any |= res[i] = src.y[i] - pred.y[i];
  std::memset(L->dc16, 0, sizeof L->dc16);
  std::memset(L->l4, 0, sizeof L->l4);
  std::memset(L->l8, 0, sizeof L->l8);
  if (!any) return 0;  // an exact prediction
  int cbp = 0;
  if (t8) {
    for (int b8 = 0; b8 < 4; ++b8) {
      int x[64], lv[64];
      for (int y = 0; y < 8; ++y)
        for (int xx = 0; xx < 8; ++xx) x[y * 8 + xx] = res[((b8 >> 1) * 8 + y) * 16 + (b8 & 1) * 8 + xx];
      quant8(x, qp, dz, lv);
      bool nz = false;
      for (int s = 0; s < 64; ++s) {
        L->l8[b8][s] = lv[kZ8[s]];
        nz |= lv[kZ8[s]] != 0;
      }
      if (nz) cbp |= 1 << b8;
    }
    return cbp;
  }
  double mu[16];
  for (int b = 0; b < 16; ++b) {
    int x[16], lv[16];
    double sum = 0;
    for (int y = 0; y < 4; ++y)
      for (int xx = 0; xx < 4; ++xx) {
        x[y * 4 + xx] = res[((b >> 2) * 4 + y) * 16 + (b & 3) * 4 + xx];
        sum += x[y * 4 + xx];
      }
    mu[b] = sum / 16.0;
    quant4(x, qp, dz, lv);
    bool nz = false;
    for (int s = i16 ? 1 : 0; s < 16; ++s) {
      L->l4[b][s - (i16 ? 1 : 0)] = lv[kZ4[s]];
      nz |= lv[kZ4[s]] != 0;
    }
    if (nz) cbp |= 1 << ((b >> 3) * 2 + ((b & 3) >> 1));
  }
  if (!i16) return cbp;
  // f = 256 mu / (normAdjust(m, 0) 2^(qp / 6)); c = H f H / 16
  const double sc = 256.0 / (h264::kNormV[qp % 6][0] * pow2(qp / 6));
  static const int H[4][4] = {{1, 1, 1, 1}, {1, 1, -1, -1}, {1, -1, -1, 1}, {1, -1, 1, -1}};
  double t[16];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      double s = 0;
      for (int k = 0; k < 4; ++k) s += H[i][k] * mu[k * 4 + j] * sc;
      t[i * 4 + j] = s;
    }
  for (int q = 0; q < 16; ++q) {
    const int i = kZ4[q] >> 2, j = kZ4[q] & 3;
    double s = 0;
    for (int k = 0; k < 4; ++k) s += t[i * 4 + k] * H[k][j];
    L->dc16[q] = deadzone(s / 16.0, dz);
  }
  return cbp ? 15 : 0;
}

// Quantise the chroma residual; returns the chroma part of
// coded_block_pattern (0, 1 DC only, 2 AC)
inline int quant_chroma(const MbPix &src, const MbPix &pred, int qpc0, int qpc1, double dz, Levels *L) {
  static const uint8_t kZ4[16] = VTS_ZZ_DATA;
  std::memset(L->cdc, 0, sizeof L->cdc);
  std::memset(L->cac, 0, sizeof L->cac);
  int cc = 0;
  for (int pl = 0; pl < 2; ++pl) {
    const int q = pl ? qpc1 : qpc0;
    double mu[4];
    for (int k = 0; k < 4; ++k) {
      int x[16], lv[16];
      double sum = 0;
      for (int y = 0; y < 4; ++y)
        for (int xx = 0; xx < 4; ++xx) {
          const int i = ((k >> 1) * 4 + y) * 8 + (k & 1) * 4 + xx;
          x[y * 4 + xx] = src.c[pl][i] - pred.c[pl][i];
          sum += x[y * 4 + xx];
        }
      mu[k] = sum / 16.0;
      quant4(x, q, dz, lv);
      for (int s = 1; s < 16; ++s) {
        L->cac[pl][k][s - 1] = lv[kZ4[s]];
        if (lv[kZ4[s]]) cc = 2;
      }
    }
    // f = 128 mu / (normAdjust(m, 0) 2^(qpc / 6)); c = H2 f H2 / 4
    const double sc = 128.0 / (h264::kNormV[q % 6][0] * pow2(q / 6));
    const double f0 = mu[0] * sc, f1 = mu[1] * sc, f2 = mu[2] * sc, f3 = mu[3] * sc;
    const double c[4] = {(f0 + f1 + f2 + f3) / 4, (f0 - f1 + f2 - f3) / 4, (f0 + f1 - f2 - f3) / 4,
                         (f0 - f1 - f2 + f3) / 4};
    for (int k = 0; k < 4; ++k) {
      L->cdc[pl][k] = deadzone(c[k], dz);
      if (L->cdc[pl][k] && !cc) cc = 1;
    }
  }
  if (cc < 2) std::memset(L->cac, 0, sizeof L->cac);
  return cc;
}

inline int nonzero(const Levels &L) {
  int n = 0;
  for (int v : L.dc16) n += v != 0;
  for (auto &b : L.l4)
    for (int v : b) n += v != 0;
  for (auto &b : L.l8)
    for (int v : b) n += v != 0;
  return n;
}

}  // namespace content
}  // namespace vts
