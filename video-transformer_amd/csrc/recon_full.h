// recon_full.h — per-macroblock reconstruction and deblocking of the general
// device decoder, written once for the device kernels (decode_full.hip: one
// lane per macroblock, intra macroblocks and deblocking in wavefront order)
// and the CPU harness (tests/native/full_host.cpp).
//
// Pictures are NV12 in the decode ring: luma rows of `pitch` bytes, the
// interleaved Cb/Cr plane at + uv_off.  Clauses: 8.3 intra prediction, 8.4.2
// inter prediction (6-tap / bilinear interpolation on clamped reference
// windows), 8.5 scaling and transforms, 8.7 deblocking.
#pragma once
#include <cstdint>

#include "h264.h"
#include "h264_full.h"
#include "h264_tables.h"
#include "h264_cabac_tables.h"
#include "parse_full.h"

namespace vts {
namespace full {

#if defined(__HIPCC__)
#define kNv h264::kdNormV
#define kQpcT h264::kdQpc
#define kAl h264::kdAlpha
#define kBe h264::kdBeta
#define kTc h264::kdTc0
#else
static const uint8_t (*const kNv)[3] = h264::kNormV;
static const uint8_t *const kQpcT = h264::kQpc;
static const uint8_t *const kAl = h264::kAlpha;
static const uint8_t *const kBe = h264::kBeta;
static const uint8_t (*const kTc)[3] = h264::kTc0;
#endif

VTS_HD VTS_INLINE int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
VTS_HD VTS_INLINE int clip1(int v) { return clip3(0, 255, v); }
VTS_HD VTS_INLINE int iabs(int v) { return v < 0 ? -v : v; }
VTS_HD VTS_INLINE int qpc_of(int qpy, int off) { return kQpcT[clip3(0, 51, qpy + off)]; }
VTS_HD VTS_INLINE int level_scale(int m, int i, int j) {
  const int k = (!(i & 1) && !(j & 1)) ? 0 : (((i & 1) && (j & 1)) ? 1 : 2);
  return 16 * kNv[m][k];
}

// 8.4.2.3 weighted sample prediction of one block, reduced to one form per
// colour component c (0 Y, 1 Cb, 2 Cr): bi-predicted
//   Clip1(((p0 w0 + p1 w1 + 2^lwd) >> (lwd + 1)) + o)
// (explicit: the table's weights, o = (o0 + o1 + 1) >> 1; implicit 8.4.2.3.1:
// lwd 5, o 0; default: w 1, lwd 0), single list
//   Clip1(((p w0 + round) >> lwd) + o), round = 2^(lwd - 1) for lwd >= 1
// (default: w 1, lwd 0, o 0).
struct Wp {
  bool both;
  int lwd[3], w0[3], w1[3], o[3];
};
// r0 / r1: refIdxL0 / L1 (< 0: list unused); x null: default prediction
VTS_HD VTS_INLINE Wp wp_make(const SliceExt *x, int r0, int r1) {
  Wp W;
  W.both = r0 >= 0 && r1 >= 0;
  const int mode = x ? x->wmode : 0;
  int iw0 = 32, iw1 = 32;
  if (mode == 2 && W.both) {
    const int tb = clip3(-128, 127, x->poc - x->poc0[r0 & 31]), td = clip3(-128, 127, x->poc1[r1 & 31] - x->poc0[r0 & 31]);
    if (td != 0 && !((x->lt0 >> (r0 & 31)) & 1u) && !((x->lt1 >> (r1 & 31)) & 1u)) {
      const int tx = (16384 + iabs(td / 2)) / td;
      const int dsf = clip3(-1024, 1023, (tb * tx + 32) >> 6);
      if ((dsf >> 2) >= -64 && (dsf >> 2) <= 128) {
        iw0 = 64 - (dsf >> 2);
        iw1 = dsf >> 2;
      }
    }
  }
  for (int c = 0; c < 3; ++c) {
    if (mode == 1) {
      W.lwd[c] = c ? x->cwd : x->lwd;
      const int wa = r0 >= 0 ? x->w[0][r0 & 31][2 * c] : 0, oa = r0 >= 0 ? x->w[0][r0 & 31][2 * c + 1] : 0;
      const int wb = r1 >= 0 ? x->w[1][r1 & 31][2 * c] : 0, ob = r1 >= 0 ? x->w[1][r1 & 31][2 * c + 1] : 0;
      W.w0[c] = W.both || r0 >= 0 ? wa : wb;
      W.w1[c] = wb;
      W.o[c] = W.both ? (oa + ob + 1) >> 1 : (r0 >= 0 ? oa : ob);
    } else {
      W.lwd[c] = mode == 2 && W.both ? 5 : 0;
      W.w0[c] = mode == 2 && W.both ? iw0 : 1;
      W.w1[c] = mode == 2 && W.both ? iw1 : 1;
      W.o[c] = 0;
    }
  }
  return W;
}
// p: the used list's prediction when only one list is used
VTS_HD VTS_INLINE int wp_apply(const Wp &W, int c, int p0, int p1) {
  const int l = W.lwd[c];
  if (W.both) return clip1(((p0 * W.w0[c] + p1 * W.w1[c] + (1 << l)) >> (l + 1)) + W.o[c]);
  return clip1(((p0 * W.w0[c] + (l ? 1 << (l - 1) : 0)) >> l) + W.o[c]);
}

struct ReconCtx {
  const MbRec *recs;        // this frame's records
  const MbRecB *recs1;      // ... their list-1 halves (streams with B slices), else null
  const SliceExt *exts;     // the window's SliceExt records
  const int16_t *arena;
  const FullSlice *slices;  // window slices
  uint8_t *surf;            // ring base
  int64_t frame_stride;
  int32_t pitch;            // luma and UV row bytes
  int64_t uv_off;           // UV plane offset in a frame
  int32_t mbw, mbh;
  int32_t cip, cqp_off, cqp_off2;
  uint32_t epoch;
  const ScaleTab *sct;      // LevelScale4x4 / 8x8 (8.5.9)
};

// 8.5.12: scaling + 4x4 inverse transform; c raster (row i, col j); ls =
// LevelScale4x4(qP % 6, raster) of the block's list; dc_done: c[0] is an
// already scaled DC; r receives the residual
VTS_HD inline void scale_idct4(const int *c, int qp, const int32_t *ls, bool dc_done, int *r) {
  int d[16];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      const int k = i * 4 + j;
      if (k == 0 && dc_done) {
        d[0] = c[0];
        continue;
      }
      d[k] = qp >= 24 ? (c[k] * ls[k]) << (qp / 6 - 4) : (c[k] * ls[k] + (1 << (3 - qp / 6))) >> (4 - qp / 6);
    }
  int f[16];
  for (int i = 0; i < 4; ++i) {
    const int e0 = d[i * 4] + d[i * 4 + 2], e1 = d[i * 4] - d[i * 4 + 2];
    const int e2 = (d[i * 4 + 1] >> 1) - d[i * 4 + 3], e3 = d[i * 4 + 1] + (d[i * 4 + 3] >> 1);
    f[i * 4] = e0 + e3;
    f[i * 4 + 1] = e1 + e2;
    f[i * 4 + 2] = e1 - e2;
    f[i * 4 + 3] = e0 - e3;
  }
  for (int j = 0; j < 4; ++j) {
    const int g0 = f[j] + f[8 + j], g1 = f[j] - f[8 + j];
    const int g2 = (f[4 + j] >> 1) - f[12 + j], g3 = f[4 + j] + (f[12 + j] >> 1);
    r[j] = (g0 + g3 + 32) >> 6;
    r[4 + j] = (g1 + g2 + 32) >> 6;
    r[8 + j] = (g1 - g2 + 32) >> 6;
    r[12 + j] = (g0 - g3 + 32) >> 6;
  }
}

// the same with Flat_16 (the upload encoder's own reconstruction)
VTS_HD inline void scale_idct4(const int *c, int qp, bool dc_done, int *r) {
  int32_t ls[16];
  for (int k = 0; k < 16; ++k) ls[k] = level_scale(qp % 6, k >> 2, k & 3);
  scale_idct4(c, qp, ls, dc_done, r);
}

// 8.5.13: scaling + 8x8 inverse transform; c raster 8x8; ls8 = LevelScale8x8(qP % 6,
// raster) of the block's list; r receives the residual
#if defined(__HIPCC__)
__device__ __constant__ static const uint8_t kNorm8[6][6] = VTS_NORM8_DATA;
#else
static const uint8_t kNorm8[6][6] = VTS_NORM8_DATA;
#endif
VTS_HD inline void scale_idct8(const int *c, int qp, const int32_t *ls8, int *r) {
  int d[64], g[64];
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) {
      const int k = i * 8 + j, ls = ls8[k];
      d[k] = qp >= 36 ? (c[k] * ls) << (qp / 6 - 6) : (c[k] * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
    }
  for (int pass = 0; pass < 2; ++pass)
    for (int u = 0; u < 8; ++u) {
      int v[8], o[8];
      for (int k = 0; k < 8; ++k) v[k] = pass == 0 ? d[u * 8 + k] : g[k * 8 + u];
      const int a0 = v[0] + v[4], a4 = v[0] - v[4], a2 = (v[2] >> 1) - v[6], a6 = v[2] + (v[6] >> 1);
      const int b0 = a0 + a6, b2 = a4 + a2, b4 = a4 - a2, b6 = a0 - a6;
      const int a1 = -v[3] + v[5] - v[7] - (v[7] >> 1), a3 = v[1] + v[7] - v[3] - (v[3] >> 1);
      const int a5 = -v[1] + v[7] + v[5] + (v[5] >> 1), a7 = v[3] + v[5] + v[1] + (v[1] >> 1);
      const int b1 = a1 + (a7 >> 2), b7 = a7 - (a1 >> 2), b3 = a3 + (a5 >> 2), b5 = (a3 >> 2) - a5;
      o[0] = b0 + b7; o[1] = b2 + b5; o[2] = b4 + b3; o[3] = b6 + b1;
      o[4] = b6 - b1; o[5] = b4 - b3; o[6] = b2 - b5; o[7] = b0 - b7;
      for (int k = 0; k < 8; ++k) {
        if (pass == 0) g[u * 8 + k] = o[k];
        else r[k * 8 + u] = (o[k] + 32) >> 6;
      }
    }
}

VTS_HD VTS_INLINE int tap6(int a, int b, int c, int d, int e, int f) {
  return a - 5 * b + 20 * c + 20 * d - 5 * e + f;
}

struct MbRecon {
  const ReconCtx &c;
  int slot, mb, mx, my;
  const MbRec &m;
  uint8_t *Y;   // frame luma
  uint8_t *UV;  // frame interleaved chroma
  uint32_t err = 0;

  VTS_HD MbRecon(const ReconCtx &ctx, int s, int a, const MbRec &rec)
      : c(ctx), slot(s), mb(a), mx(a % ctx.mbw), my(a / ctx.mbw), m(rec) {
    Y = c.surf + static_cast<int64_t>(slot) * c.frame_stride;
    UV = Y + c.uv_off;
  }

  // block index in the arena of stored-block bit `bit`, -1 if not stored
  VTS_HD VTS_INLINE int64_t block_of(uint32_t bit) const {
    if (!((m.blocks >> bit) & 1u)) return -1;
    return static_cast<int64_t>(m.coef) + __builtin_popcount(m.blocks & ((1u << bit) - 1u));
  }
  VTS_HD VTS_INLINE void load_block8(int b8, int *cf) const {  // 4 consecutive blocks = raster 8x8
    const int64_t b = block_of(kBlkLuma0 + 4 * b8);
    for (int i = 0; i < 64; ++i) cf[i] = b < 0 ? 0 : c.arena[16 * b + i];
  }
  VTS_HD VTS_INLINE void load_block(uint32_t bit, int *cf) const {
    const int64_t b = block_of(bit);
    for (int i = 0; i < 16; ++i) cf[i] = b < 0 ? 0 : c.arena[16 * b + i];
  }

  // neighbour macroblock available for intra prediction (6.4.8, CIP)
  VTS_HD VTS_INLINE bool intra_nb(int n) const {
    if (n < 0) return false;
    const MbRec &r = c.recs[n];
    if (r.epoch != c.epoch || r.slice != m.slice) return false;
    if (c.cip && (r.type == kMbInter || r.type == kMbSkip)) return false;
    return true;
  }
  VTS_HD VTS_INLINE int nb_addr(int dx, int dy) const {  // dx, dy in {-1, 0, 1} macroblocks
    const int x = mx + dx, y = my + dy;
    if (x < 0 || x >= c.mbw || y < 0) return -1;
    return y * c.mbw + x;
  }

  VTS_HD VTS_INLINE int ly(int x, int y) const { return Y[static_cast<int64_t>(y) * c.pitch + x]; }
  VTS_HD VTS_INLINE int lc(int pl, int x, int y) const { return UV[static_cast<int64_t>(y) * c.pitch + 2 * x + pl]; }

  // ---- inter (8.4.2.2, weighted 8.4.2.3): both lists' predictions of the
  // block, combined into pred_y / pred_c
  VTS_HD void inter_block(int b) {
    const int p8 = (b >> 3) * 2 + ((b & 3) >> 1);
    const int r0 = m.ref_slot[p8] >= 0 ? m.ref[p8] : -1;
    const MbRecB *m1 = c.recs1 ? &c.recs1[mb] : nullptr;
    const int r1 = m1 && m1->ref_slot1[p8] >= 0 ? m1->ref1[p8] : -1;
    uint8_t ty[2][16] = {}, tc[2][2][4] = {};
    if (r0 >= 0) pred_list(b, m.ref_slot[p8], m.mv[b][0], m.mv[b][1], ty[0], tc[0]);
    if (r1 >= 0) pred_list(b, m1->ref_slot1[p8], m1->mv1[b][0], m1->mv1[b][1], ty[1], tc[1]);
    const FullSlice &sl = c.slices[m.slice];
    const Wp W = wp_make(sl.ext >= 0 ? &c.exts[sl.ext] : nullptr, r0, r1);
    const int u = r0 >= 0 ? 0 : 1;  // the list a single-list block uses
    const int bx = (b & 3) * 4, by = (b >> 2) * 4;
    for (int i = 0; i < 16; ++i)
      pred_y[(by + i / 4) * 16 + bx + i % 4] = static_cast<uint8_t>(wp_apply(W, 0, ty[u][i], ty[1][i]));
    for (int pl = 0; pl < 2; ++pl)
      for (int i = 0; i < 4; ++i)
        pred_c[pl][(by / 2 + i / 2) * 8 + bx / 2 + i % 2] =
            static_cast<uint8_t>(wp_apply(W, 1 + pl, tc[u][pl][i], tc[1][pl][i]));
  }
  // one list's 4x4 luma + 2x2 Cb / Cr prediction of raster block b from the picture in ring slot rs
  VTS_HD void pred_list(int b, int rs, int mvx, int mvy, uint8_t *oy, uint8_t (*oc)[4]) {
    const uint8_t *R = c.surf + static_cast<int64_t>(rs) * c.frame_stride;
    const uint8_t *RUV = R + c.uv_off;
    const int W = c.mbw * 16, H = c.mbh * 16;
    const int bx = mx * 16 + (b & 3) * 4, by = my * 16 + (b >> 2) * 4;
    const int xi = bx + (mvx >> 2), yi = by + (mvy >> 2), xf = mvx & 3, yf = mvy & 3;
    uint8_t w[9][9];
    for (int r = 0; r < 9; ++r) {
      const int yy = clip3(0, H - 1, yi - 2 + r);
      for (int q = 0; q < 9; ++q) w[r][q] = R[static_cast<int64_t>(yy) * c.pitch + clip3(0, W - 1, xi - 2 + q)];
    }
    for (int y = 0; y < 4; ++y)
      for (int x = 0; x < 4; ++x) {
        const int G = w[y + 2][x + 2];
        int v;
        if (!xf && !yf) {
          v = G;
        } else {
          const int b1 = tap6(w[y + 2][x], w[y + 2][x + 1], w[y + 2][x + 2], w[y + 2][x + 3], w[y + 2][x + 4], w[y + 2][x + 5]);
          const int h1 = tap6(w[y][x + 2], w[y + 1][x + 2], w[y + 2][x + 2], w[y + 3][x + 2], w[y + 4][x + 2], w[y + 5][x + 2]);
          const int s1 = tap6(w[y + 3][x], w[y + 3][x + 1], w[y + 3][x + 2], w[y + 3][x + 3], w[y + 3][x + 4], w[y + 3][x + 5]);
          const int m1 = tap6(w[y][x + 3], w[y + 1][x + 3], w[y + 2][x + 3], w[y + 3][x + 3], w[y + 4][x + 3], w[y + 5][x + 3]);
          const int bb = clip1((b1 + 16) >> 5), hh = clip1((h1 + 16) >> 5);
          const int ss = clip1((s1 + 16) >> 5), mm = clip1((m1 + 16) >> 5);
          int jj = 0;
          if ((xf | yf) & 1 ? (xf == 2 || yf == 2) : (xf == 2 && yf == 2)) {
            int hr[6];
            for (int k = 0; k < 6; ++k)
              hr[k] = tap6(w[y + k][x], w[y + k][x + 1], w[y + k][x + 2], w[y + k][x + 3], w[y + k][x + 4], w[y + k][x + 5]);
            jj = clip1((tap6(hr[0], hr[1], hr[2], hr[3], hr[4], hr[5]) + 512) >> 10);
          }
          const int Hs = w[y + 2][x + 3], Ms = w[y + 3][x + 2];
          switch (yf * 4 + xf) {
            case 1: v = (G + bb + 1) >> 1; break;
            case 2: v = bb; break;
            case 3: v = (Hs + bb + 1) >> 1; break;
            case 4: v = (G + hh + 1) >> 1; break;
            case 5: v = (bb + hh + 1) >> 1; break;
            case 6: v = (bb + jj + 1) >> 1; break;
            case 7: v = (bb + mm + 1) >> 1; break;
            case 8: v = hh; break;
            case 9: v = (hh + jj + 1) >> 1; break;
            case 10: v = jj; break;
            case 11: v = (jj + mm + 1) >> 1; break;
            case 12: v = (Ms + hh + 1) >> 1; break;
            case 13: v = (hh + ss + 1) >> 1; break;
            case 14: v = (jj + ss + 1) >> 1; break;
            default: v = (mm + ss + 1) >> 1; break;
          }
        }
        oy[y * 4 + x] = static_cast<uint8_t>(v);
      }
    // chroma 2x2 (8.4.2.2.2)
    const int cw = W / 2, ch = H / 2;
    const int cfx = mvx & 7, cfy = mvy & 7;
    const int cx0 = bx / 2 + (mvx >> 3), cy0 = by / 2 + (mvy >> 3);
    for (int y = 0; y < 2; ++y)
      for (int x = 0; x < 2; ++x) {
        const int xa = clip3(0, cw - 1, cx0 + x), xb = clip3(0, cw - 1, cx0 + x + 1);
        const int ya = clip3(0, ch - 1, cy0 + y), yb = clip3(0, ch - 1, cy0 + y + 1);
        for (int pl = 0; pl < 2; ++pl) {
          const int A = RUV[static_cast<int64_t>(ya) * c.pitch + 2 * xa + pl];
          const int B = RUV[static_cast<int64_t>(ya) * c.pitch + 2 * xb + pl];
          const int C = RUV[static_cast<int64_t>(yb) * c.pitch + 2 * xa + pl];
          const int D = RUV[static_cast<int64_t>(yb) * c.pitch + 2 * xb + pl];
          const int v = ((8 - cfx) * (8 - cfy) * A + cfx * (8 - cfy) * B + (8 - cfx) * cfy * C + cfx * cfy * D + 32) >> 6;
          oc[pl][y * 2 + x] = static_cast<uint8_t>(v);
        }
      }
  }

  uint8_t pred_y[256];
  uint8_t pred_c[2][64];

  // ---- Intra_4x4 (8.3.1.2) for luma4x4BlkIdx k, reading the picture
  VTS_HD void intra4x4(int k, int mode, uint32_t done) {
    const int bx = blk_x(k), by = blk_y(k);
    const int x0 = mx * 16 + bx * 4, y0 = my * 16 + by * 4;
    // availability of p[x,-1] (x=0..3 and 4..7), p[-1,y], p[-1,-1]
    auto avail = [&](int xN, int yN) -> bool {  // MB-relative luma location
      int dx = xN < 0 ? -1 : (xN > 15 ? 1 : 0), dy = yN < 0 ? -1 : 0;
      if (yN > 15 || (xN > 15 && yN >= 0)) return false;
      if (dx == 0 && dy == 0) {
        const int r = (yN / 4) * 4 + xN / 4;
        return (done >> r) & 1u;
      }
      return intra_nb(nb_addr(dx, dy));
    };
    const bool top = avail(bx * 4, by * 4 - 1);
    const bool tr = avail(bx * 4 + 4, by * 4 - 1);
    const bool left = avail(bx * 4 - 1, by * 4);
    const bool tl = avail(bx * 4 - 1, by * 4 - 1);
    int T[9], L[5];  // T[0] = L[0] = p[-1,-1]; T[1+x], L[1+y]
    T[0] = L[0] = tl ? ly(x0 - 1, y0 - 1) : 0;
    for (int x = 0; x < 4; ++x) T[1 + x] = top ? ly(x0 + x, y0 - 1) : 0;
    for (int x = 4; x < 8; ++x) T[1 + x] = tr ? ly(x0 + x, y0 - 1) : T[4];
    for (int y = 0; y < 4; ++y) L[1 + y] = left ? ly(x0 - 1, y0 + y) : 0;
#define PT(x) T[1 + (x)]
#define PL(y) L[1 + (y)]
    for (int y = 0; y < 4; ++y)
      for (int x = 0; x < 4; ++x) {
        int v;
        switch (mode) {
          case 0: v = PT(x); break;
          case 1: v = PL(y); break;
          case 2:
            if (top && left) v = (PT(0) + PT(1) + PT(2) + PT(3) + PL(0) + PL(1) + PL(2) + PL(3) + 4) >> 3;
            else if (left) v = (PL(0) + PL(1) + PL(2) + PL(3) + 2) >> 2;
            else if (top) v = (PT(0) + PT(1) + PT(2) + PT(3) + 2) >> 2;
            else v = 128;
            break;
          case 3:
            v = (x == 3 && y == 3) ? (PT(6) + 3 * PT(7) + 2) >> 2
                                   : (PT(x + y) + 2 * PT(x + y + 1) + PT(x + y + 2) + 2) >> 2;
            break;
          case 4:
            if (x > y) v = (PT(x - y - 2) + 2 * PT(x - y - 1) + PT(x - y) + 2) >> 2;
            else if (x < y) v = (PL(y - x - 2) + 2 * PL(y - x - 1) + PL(y - x) + 2) >> 2;
            else v = (PT(0) + 2 * PT(-1) + PL(0) + 2) >> 2;
            break;
          case 5: {
            const int z = 2 * x - y;
            if (z >= 0 && !(z & 1)) v = (PT(x - (y >> 1) - 1) + PT(x - (y >> 1)) + 1) >> 1;
            else if (z >= 0) v = (PT(x - (y >> 1) - 2) + 2 * PT(x - (y >> 1) - 1) + PT(x - (y >> 1)) + 2) >> 2;
            else if (z == -1) v = (PL(0) + 2 * PL(-1) + PT(0) + 2) >> 2;
            else v = (PL(y - 1) + 2 * PL(y - 2) + PL(y - 3) + 2) >> 2;
            break;
          }
          case 6: {
            const int z = 2 * y - x;
            if (z >= 0 && !(z & 1)) v = (PL(y - (x >> 1) - 1) + PL(y - (x >> 1)) + 1) >> 1;
            else if (z >= 0) v = (PL(y - (x >> 1) - 2) + 2 * PL(y - (x >> 1) - 1) + PL(y - (x >> 1)) + 2) >> 2;
            else if (z == -1) v = (PL(0) + 2 * PL(-1) + PT(0) + 2) >> 2;
            else v = (PT(x - 1) + 2 * PT(x - 2) + PT(x - 3) + 2) >> 2;
            break;
          }
          case 7:
            v = (y & 1) ? (PT(x + (y >> 1)) + 2 * PT(x + (y >> 1) + 1) + PT(x + (y >> 1) + 2) + 2) >> 2
                        : (PT(x + (y >> 1)) + PT(x + (y >> 1) + 1) + 1) >> 1;
            break;
          default: {
            const int z = x + 2 * y;
            if (z == 0 || z == 2 || z == 4) v = (PL(y + (x >> 1)) + PL(y + (x >> 1) + 1) + 1) >> 1;
            else if (z == 1 || z == 3) v = (PL(y + (x >> 1)) + 2 * PL(y + (x >> 1) + 1) + PL(y + (x >> 1) + 2) + 2) >> 2;
            else if (z == 5) v = (PL(2) + 3 * PL(3) + 2) >> 2;
            else v = PL(3);
            break;
          }
        }
        pred_y[(by * 4 + y) * 16 + bx * 4 + x] = static_cast<uint8_t>(v);
      }
#undef PT
#undef PL
  }

  // ---- Intra_8x8 (8.3.2) of raster 8x8 block b8, reference samples filtered
  VTS_HD void intra8x8(int b8, int mode, uint32_t done) {
    const int xo = (b8 & 1) * 8, yo = (b8 >> 1) * 8, x0 = mx * 16 + xo, y0 = my * 16 + yo;
    auto avail = [&](int xN, int yN) -> bool {  // MB-relative luma location
      const int dx = xN < 0 ? -1 : (xN > 15 ? 1 : 0), dy = yN < 0 ? -1 : 0;
      if (yN > 15 || (xN > 15 && yN >= 0)) return false;
      if (dx == 0 && dy == 0) return (done >> ((yN / 4) * 4 + xN / 4)) & 1u;
      return intra_nb(nb_addr(dx, dy));
    };
    int P_[25];  // 0 = p[-1,-1], 1 + x = p[x,-1] (x 0..15), 17 + y = p[-1,y]
    const bool tl = avail(xo - 1, yo - 1), top = avail(xo, yo - 1), left = avail(xo - 1, yo);
    bool tr = avail(xo + 8, yo - 1);
    P_[0] = tl ? ly(x0 - 1, y0 - 1) : 0;
    for (int x = 0; x < 16; ++x) P_[1 + x] = (x < 8 ? top : tr) ? ly(x0 + x, y0 - 1) : 0;
    if (!tr && top)
      for (int x = 8; x < 16; ++x) P_[1 + x] = P_[8];
    for (int y = 0; y < 8; ++y) P_[17 + y] = left ? ly(x0 - 1, y0 + y) : 0;
    int T[17] = {0}, L[8] = {0};
    if (top) {
      T[1] = tl ? (P_[0] + 2 * P_[1] + P_[2] + 2) >> 2 : (3 * P_[1] + P_[2] + 2) >> 2;
      for (int x = 1; x < 15; ++x) T[1 + x] = (P_[x] + 2 * P_[1 + x] + P_[2 + x] + 2) >> 2;
      T[16] = (P_[15] + 3 * P_[16] + 2) >> 2;
    }
    if (tl) {
      if (top && left) T[0] = (P_[1] + 2 * P_[0] + P_[17] + 2) >> 2;
      else if (top) T[0] = (3 * P_[0] + P_[1] + 2) >> 2;
      else if (left) T[0] = (3 * P_[0] + P_[17] + 2) >> 2;
      else T[0] = P_[0];
    }
    if (left) {
      L[0] = tl ? (P_[0] + 2 * P_[17] + P_[18] + 2) >> 2 : (3 * P_[17] + P_[18] + 2) >> 2;
      for (int y = 1; y < 7; ++y) L[y] = (P_[16 + y] + 2 * P_[17 + y] + P_[18 + y] + 2) >> 2;
      L[7] = (P_[23] + 3 * P_[24] + 2) >> 2;
    }
#define PT(x) T[1 + (x)]
#define PL(y) ((y) < 0 ? T[0] : L[(y)])
    for (int y = 0; y < 8; ++y)
      for (int x = 0; x < 8; ++x) {
        int v = 128;
        switch (mode) {
          case 0: v = PT(x); break;
          case 1: v = PL(y); break;
          case 2: {
            int st = 0, sl = 0;
            for (int i = 0; i < 8; ++i) {
              st += PT(i);
              sl += L[i];
            }
            if (top && left) v = (st + sl + 8) >> 4;
            else if (left) v = (sl + 4) >> 3;
            else if (top) v = (st + 4) >> 3;
            break;
          }
          case 3:
            v = (x == 7 && y == 7) ? (PT(14) + 3 * PT(15) + 2) >> 2 : (PT(x + y) + 2 * PT(x + y + 1) + PT(x + y + 2) + 2) >> 2;
            break;
          case 4:
            if (x > y) v = (PT(x - y - 2) + 2 * PT(x - y - 1) + PT(x - y) + 2) >> 2;
            else if (x < y) v = (PL(y - x - 2) + 2 * PL(y - x - 1) + PL(y - x) + 2) >> 2;
            else v = (PT(0) + 2 * PT(-1) + PL(0) + 2) >> 2;
            break;
          case 5: {
            const int z = 2 * x - y;
            if (z >= 0 && !(z & 1)) v = (PT(x - (y >> 1) - 1) + PT(x - (y >> 1)) + 1) >> 1;
            else if (z >= 0) v = (PT(x - (y >> 1) - 2) + 2 * PT(x - (y >> 1) - 1) + PT(x - (y >> 1)) + 2) >> 2;
            else if (z == -1) v = (PL(0) + 2 * PL(-1) + PT(0) + 2) >> 2;
            else v = (PL(y - 2 * x - 1) + 2 * PL(y - 2 * x - 2) + PL(y - 2 * x - 3) + 2) >> 2;
            break;
          }
          case 6: {
            const int z = 2 * y - x;
            if (z >= 0 && !(z & 1)) v = (PL(y - (x >> 1) - 1) + PL(y - (x >> 1)) + 1) >> 1;
            else if (z >= 0) v = (PL(y - (x >> 1) - 2) + 2 * PL(y - (x >> 1) - 1) + PL(y - (x >> 1)) + 2) >> 2;
            else if (z == -1) v = (PL(0) + 2 * PL(-1) + PT(0) + 2) >> 2;
            else v = (PT(x - 2 * y - 1) + 2 * PT(x - 2 * y - 2) + PT(x - 2 * y - 3) + 2) >> 2;
            break;
          }
          case 7:
            v = !(y & 1) ? (PT(x + (y >> 1)) + PT(x + (y >> 1) + 1) + 1) >> 1
                         : (PT(x + (y >> 1)) + 2 * PT(x + (y >> 1) + 1) + PT(x + (y >> 1) + 2) + 2) >> 2;
            break;
          default: {
            const int z = x + 2 * y;
            if (z < 13 && !(z & 1)) v = (PL(y + (x >> 1)) + PL(y + (x >> 1) + 1) + 1) >> 1;
            else if (z < 13) v = (PL(y + (x >> 1)) + 2 * PL(y + (x >> 1) + 1) + PL(y + (x >> 1) + 2) + 2) >> 2;
            else if (z == 13) v = (PL(6) + 3 * PL(7) + 2) >> 2;
            else v = PL(7);
            break;
          }
        }
        pred_y[(yo + y) * 16 + xo + x] = static_cast<uint8_t>(v);
      }
#undef PT
#undef PL
  }
  VTS_HD void put_luma8(int b8, const int *res) {
    const int bx = (b8 & 1) * 8, by = (b8 >> 1) * 8;
    uint8_t *d = Y + static_cast<int64_t>(my * 16 + by) * c.pitch + mx * 16 + bx;
    for (int y = 0; y < 8; ++y)
      for (int x = 0; x < 8; ++x)
        d[static_cast<int64_t>(y) * c.pitch + x] = static_cast<uint8_t>(clip1(pred_y[(by + y) * 16 + bx + x] + res[y * 8 + x]));
  }

  // ---- Intra_16x16 (8.3.3) and chroma (8.3.4) predictions
  VTS_HD void intra16(int mode) {
    const bool la = intra_nb(nb_addr(-1, 0)), ta = intra_nb(nb_addr(0, -1)), ca = intra_nb(nb_addr(-1, -1));
    const int x0 = mx * 16, y0 = my * 16;
    int T[17], L[17];
    T[0] = L[0] = ca ? ly(x0 - 1, y0 - 1) : 0;
    for (int i = 0; i < 16; ++i) {
      T[1 + i] = ta ? ly(x0 + i, y0 - 1) : 0;
      L[1 + i] = la ? ly(x0 - 1, y0 + i) : 0;
    }
    int dc = 128, a = 0, b = 0, cc = 0;
    if (mode == 2) {
      int st = 0, sl = 0;
      for (int i = 0; i < 16; ++i) {
        st += T[1 + i];
        sl += L[1 + i];
      }
      dc = (ta && la) ? (st + sl + 16) >> 5 : (la ? (sl + 8) >> 4 : (ta ? (st + 8) >> 4 : 128));
    } else if (mode == 3) {
      int Hh = 0, Vv = 0;
      for (int i = 0; i < 8; ++i) {
        Hh += (i + 1) * (T[1 + 8 + i] - T[1 + 6 - i]);
        Vv += (i + 1) * (L[1 + 8 + i] - L[1 + 6 - i]);
      }
      a = 16 * (L[16] + T[16]);
      b = (5 * Hh + 32) >> 6;
      cc = (5 * Vv + 32) >> 6;
    }
    for (int y = 0; y < 16; ++y)
      for (int x = 0; x < 16; ++x) {
        int v;
        if (mode == 0) v = T[1 + x];
        else if (mode == 1) v = L[1 + y];
        else if (mode == 2) v = dc;
        else v = clip1((a + b * (x - 7) + cc * (y - 7) + 16) >> 5);
        pred_y[y * 16 + x] = static_cast<uint8_t>(v);
      }
  }
  VTS_HD void intra_chroma(int mode) {
    const bool la = intra_nb(nb_addr(-1, 0)), ta = intra_nb(nb_addr(0, -1)), ca = intra_nb(nb_addr(-1, -1));
    const int x0 = mx * 8, y0 = my * 8;
    for (int pl = 0; pl < 2; ++pl) {
      int T[9], L[9];
      T[0] = L[0] = ca ? lc(pl, x0 - 1, y0 - 1) : 0;
      for (int i = 0; i < 8; ++i) {
        T[1 + i] = ta ? lc(pl, x0 + i, y0 - 1) : 0;
        L[1 + i] = la ? lc(pl, x0 - 1, y0 + i) : 0;
      }
      int a = 0, b = 0, cc = 0;
      if (mode == 3) {
        int Hh = 0, Vv = 0;
        for (int i = 0; i < 4; ++i) {
          Hh += (i + 1) * (T[1 + 4 + i] - T[1 + 2 - i]);
          Vv += (i + 1) * (L[1 + 4 + i] - L[1 + 2 - i]);
        }
        a = 16 * (L[8] + T[8]);
        b = (34 * Hh + 32) >> 6;
        cc = (34 * Vv + 32) >> 6;
      }
      for (int y = 0; y < 8; ++y)
        for (int x = 0; x < 8; ++x) {
          int v = 128;
          if (mode == 0) {
            const int xo = x & 4, yo = y & 4;
            int st = 0, sl = 0;
            for (int i = 0; i < 4; ++i) {
              st += T[1 + xo + i];
              sl += L[1 + yo + i];
            }
            if ((xo == 0 && yo == 0) || (xo && yo)) {
              if (ta && la) v = (st + sl + 4) >> 3;
              else if (la) v = (sl + 2) >> 2;
              else if (ta) v = (st + 2) >> 2;
            } else if (xo) {
              if (ta) v = (st + 2) >> 2;
              else if (la) v = (sl + 2) >> 2;
            } else {
              if (la) v = (sl + 2) >> 2;
              else if (ta) v = (st + 2) >> 2;
            }
          } else if (mode == 1) {
            v = L[1 + y];
          } else if (mode == 2) {
            v = T[1 + x];
          } else {
            v = clip1((a + b * (x - 3) + cc * (y - 3) + 16) >> 5);
          }
          pred_c[pl][y * 8 + x] = static_cast<uint8_t>(v);
        }
    }
  }

  // write luma 4x4 block (raster b) = clip(pred + residual)
  VTS_HD VTS_INLINE void put_luma(int b, const int *res) {
    const int bx = (b & 3) * 4, by = (b >> 2) * 4;
    uint8_t *d = Y + static_cast<int64_t>(my * 16 + by) * c.pitch + mx * 16 + bx;
    for (int y = 0; y < 4; ++y)
      for (int x = 0; x < 4; ++x) d[static_cast<int64_t>(y) * c.pitch + x] = static_cast<uint8_t>(clip1(pred_y[(by + y) * 16 + bx + x] + res[y * 4 + x]));
  }

  VTS_HD void luma_residual_block(int b, int qp, bool i16, const int *dcy, int *res) {
    int cf[16];
    const int k = ((b >> 3) << 3) | (((b & 3) >> 1) << 2) | (((b >> 2) & 1) << 1) | (b & 1);  // luma4x4BlkIdx
    load_block(kBlkLuma0 + k, cf);
    if (i16) cf[0] = dcy[b];
    scale_idct4(cf, qp, c.sct->ls4[scale_list4(m.type != kMbInter && m.type != kMbSkip, 0)][qp % 6], i16, res);
  }

  VTS_HD void chroma_residual(int qpy) {
    for (int pl = 0; pl < 2; ++pl) {
      const int qpc = qpc_of(qpy, pl ? c.cqp_off2 : c.cqp_off);
      int dcl[16];
      load_block(kBlkChromaDc0 + pl, dcl);
      const int c0 = dcl[0], c1 = dcl[1], c2 = dcl[2], c3 = dcl[3];
      const int f[4] = {c0 + c1 + c2 + c3, c0 - c1 + c2 - c3, c0 + c1 - c2 - c3, c0 - c1 - c2 + c3};
      const int32_t *lsc = c.sct->ls4[scale_list4(m.type != kMbInter && m.type != kMbSkip, 1 + pl)][qpc % 6];
      for (int k = 0; k < 4; ++k) {
        int cf[16], r[16];
        load_block(kBlkChromaAc0 + 4 * pl + k, cf);
        cf[0] = ((f[k] * lsc[0]) << (qpc / 6)) >> 5;  // 8.5.11.2
        scale_idct4(cf, qpc, lsc, true, r);
        const int bx = (k & 1) * 4, by = (k >> 1) * 4;
        for (int y = 0; y < 4; ++y)
          for (int x = 0; x < 4; ++x)
            UV[static_cast<int64_t>(my * 8 + by + y) * c.pitch + 2 * (mx * 8 + bx + x) + pl] =
                static_cast<uint8_t>(clip1(pred_c[pl][(by + y) * 8 + bx + x] + r[y * 4 + x]));
      }
    }
  }

  VTS_HD void run() {
    if (m.epoch != c.epoch) {
      err |= DEC_E_MISSING_MB;
      return;
    }
    const int qp = m.qp;
    if (m.type == kMbPcm) {
      const int16_t *s = c.arena + 16 * static_cast<int64_t>(m.coef);
      const uint8_t *b = reinterpret_cast<const uint8_t *>(s);
      for (int y = 0; y < 16; ++y)
        for (int x = 0; x < 16; ++x) Y[static_cast<int64_t>(my * 16 + y) * c.pitch + mx * 16 + x] = b[y * 16 + x];
      for (int pl = 0; pl < 2; ++pl)
        for (int y = 0; y < 8; ++y)
          for (int x = 0; x < 8; ++x)
            UV[static_cast<int64_t>(my * 8 + y) * c.pitch + 2 * (mx * 8 + x) + pl] = b[256 + 64 * pl + y * 8 + x];
      return;
    }
    int res[16];
    const int dummy_dc[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (m.type == kMbInter || m.type == kMbSkip) {
      for (int b = 0; b < 16; ++b) {
        const int p8 = (b >> 3) * 2 + ((b & 3) >> 1);
        const int rs = m.ref_slot[p8] >= 0 ? m.ref_slot[p8] : (c.recs1 ? c.recs1[mb].ref_slot1[p8] : -1);
        if (rs < 0) {
          err |= DEC_E_NO_REF;
          return;
        }
        inter_block(b);
      }
      if (m.modes & kModeT8) {
        for (int b8 = 0; b8 < 4; ++b8) {
          int cf[64], r8[64];
          load_block8(b8, cf);
          scale_idct8(cf, qp, c.sct->ls8[1][qp % 6], r8);
          put_luma8(b8, r8);
        }
      } else {
        for (int b = 0; b < 16; ++b) {
          luma_residual_block(b, qp, false, dummy_dc, res);
          put_luma(b, res);
        }
      }
    } else if (m.type == kMbI4x4 && (m.modes & kModeT8)) {
      uint32_t done = 0;
      for (int b8 = 0; b8 < 4; ++b8) {
        const int r = (b8 >> 1) * 8 + (b8 & 1) * 2;
        intra8x8(b8, (m.i4[r >> 1] >> ((r & 1) * 4)) & 15, done);
        int cf[64], r8[64];
        load_block8(b8, cf);
        scale_idct8(cf, qp, c.sct->ls8[0][qp % 6], r8);
        put_luma8(b8, r8);
        done |= (1u << r) | (1u << (r + 1)) | (1u << (r + 4)) | (1u << (r + 5));
      }
    } else if (m.type == kMbI4x4) {
      uint32_t done = 0;
      for (int k = 0; k < 16; ++k) {
        const int b = blk_y(k) * 4 + blk_x(k);
        intra4x4(k, (m.i4[b >> 1] >> ((b & 1) * 4)) & 15, done);
        luma_residual_block(b, qp, false, dummy_dc, res);
        put_luma(b, res);
        done |= 1u << b;
      }
    } else {
      intra16(m.modes & 3);
      // 8.5.10: Intra16x16 DC, Hadamard + scaling
      int dcl[16], t[16], dcy[16];
      load_block(kBlkI16Dc, dcl);
      for (int i = 0; i < 4; ++i) {
        const int a0 = dcl[i * 4], a1 = dcl[i * 4 + 1], a2 = dcl[i * 4 + 2], a3 = dcl[i * 4 + 3];
        t[i * 4] = a0 + a1 + a2 + a3;
        t[i * 4 + 1] = a0 + a1 - a2 - a3;
        t[i * 4 + 2] = a0 - a1 - a2 + a3;
        t[i * 4 + 3] = a0 - a1 + a2 - a3;
      }
      const int ls = c.sct->ls4[0][qp % 6][0];  // LevelScale4x4(qP % 6, 0, 0) of Intra Y
      for (int j = 0; j < 4; ++j) {
        const int a0 = t[j], a1 = t[4 + j], a2 = t[8 + j], a3 = t[12 + j];
        const int f[4] = {a0 + a1 + a2 + a3, a0 + a1 - a2 - a3, a0 - a1 - a2 + a3, a0 - a1 + a2 - a3};
        for (int i = 0; i < 4; ++i)
          dcy[i * 4 + j] = qp >= 36 ? (f[i] * ls) << (qp / 6 - 6) : (f[i] * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
      }
      for (int b = 0; b < 16; ++b) {
        luma_residual_block(b, qp, true, dcy, res);
        put_luma(b, res);
      }
    }
    if (m.type != kMbInter && m.type != kMbSkip) intra_chroma((m.modes >> 2) & 3);
    chroma_residual(qp);
  }
};

// ---------------------------------------------------------- deblocking (8.7)
VTS_HD VTS_INLINE bool mb_is_intra(const MbRec &r) { return r.type == kMbI4x4 || r.type == kMbI16 || r.type == kMbPcm; }

VTS_HD VTS_INLINE bool mv_far(int ax, int ay, int bx, int by) { return iabs(ax - bx) >= 4 || iabs(ay - by) >= 4; }

// bS 1 / 0 from the motion of two inter blocks (8.7.2.1, mixedModeEdgeFlag 0):
// reference pictures compared as pictures (ring slots, -1 = list unused) and
// as the set a bi-predicted block uses; mv X = (x, y) of list X
VTS_HD VTS_INLINE int bs_motion(int p0, int p1, int pm0x, int pm0y, int pm1x, int pm1y, int q0, int q1, int qm0x,
                                int qm0y, int qm1x, int qm1y) {
  const int np = (p0 >= 0) + (p1 >= 0), nq = (q0 >= 0) + (q1 >= 0);
  if (np != nq) return 1;
  if (np == 1) {
    const bool lp = p0 < 0, lq = q0 < 0;
    if ((lp ? p1 : p0) != (lq ? q1 : q0)) return 1;
    return mv_far(lp ? pm1x : pm0x, lp ? pm1y : pm0y, lq ? qm1x : qm0x, lq ? qm1y : qm0y);
  }
  if (!((p0 == q0 && p1 == q1) || (p0 == q1 && p1 == q0))) return 1;
  const bool same = mv_far(pm0x, pm0y, qm0x, qm0y) || mv_far(pm1x, pm1y, qm1x, qm1y);
  const bool cross = mv_far(pm0x, pm0y, qm1x, qm1y) || mv_far(pm1x, pm1y, qm0x, qm0y);
  if (p0 != p1) return p0 == q0 ? same : cross;
  return same && cross;
}

VTS_HD VTS_INLINE int bs_of(const MbRec &p, const MbRecB *p1, int bp, const MbRec &q, const MbRecB *q1, int bq,
                            bool mb_edge) {
  if (mb_is_intra(p) || mb_is_intra(q)) return mb_edge ? 4 : 3;
  if (p.nz[bp] || q.nz[bq]) return 2;
  const int p8 = (bp >> 3) * 2 + ((bp & 3) >> 1), q8 = (bq >> 3) * 2 + ((bq & 3) >> 1);
  if (!p1) {  // P pictures: one list
    if (p.ref_slot[p8] != q.ref_slot[q8]) return 1;
    return mv_far(p.mv[bp][0], p.mv[bp][1], q.mv[bq][0], q.mv[bq][1]);
  }
  return bs_motion(p.ref_slot[p8], p1->ref_slot1[p8], p.mv[bp][0], p.mv[bp][1], p1->mv1[bp][0], p1->mv1[bp][1],
                   q.ref_slot[q8], q1->ref_slot1[q8], q.mv[bq][0], q.mv[bq][1], q1->mv1[bq][0], q1->mv1[bq][1]);
}

// one line across an edge: s[k * step], k = -4..3 (p3..q3)
VTS_HD VTS_INLINE void filter_line(uint8_t *s, int64_t step, int bS, bool chroma, int iA, int alpha, int beta) {
  const int p0 = s[-step], p1 = s[-2 * step], q0 = s[0], q1 = s[step];
  if (!(bS > 0 && iabs(p0 - q0) < alpha && iabs(p1 - p0) < beta && iabs(q1 - q0) < beta)) return;
  if (bS < 4) {
    const int tc0 = kTc[iA][bS - 1];
    if (chroma) {
      const int tc = tc0 + 1;
      const int delta = clip3(-tc, tc, (((q0 - p0) << 2) + (p1 - q1) + 4) >> 3);
      s[-step] = static_cast<uint8_t>(clip1(p0 + delta));
      s[0] = static_cast<uint8_t>(clip1(q0 - delta));
      return;
    }
    const int p2 = s[-3 * step], q2 = s[2 * step];
    const int ap = iabs(p2 - p0), aq = iabs(q2 - q0);
    const int tc = tc0 + (ap < beta) + (aq < beta);
    const int delta = clip3(-tc, tc, (((q0 - p0) << 2) + (p1 - q1) + 4) >> 3);
    s[-step] = static_cast<uint8_t>(clip1(p0 + delta));
    s[0] = static_cast<uint8_t>(clip1(q0 - delta));
    if (ap < beta) s[-2 * step] = static_cast<uint8_t>(p1 + clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1));
    if (aq < beta) s[step] = static_cast<uint8_t>(q1 + clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1));
    return;
  }
  if (chroma) {
    s[-step] = static_cast<uint8_t>((2 * p1 + p0 + q1 + 2) >> 2);
    s[0] = static_cast<uint8_t>((2 * q1 + q0 + p1 + 2) >> 2);
    return;
  }
  const int p2 = s[-3 * step], q2 = s[2 * step], p3 = s[-4 * step], q3 = s[3 * step];
  const int ap = iabs(p2 - p0), aq = iabs(q2 - q0);
  const bool small = iabs(p0 - q0) < ((alpha >> 2) + 2);
  if (ap < beta && small) {
    s[-step] = static_cast<uint8_t>((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
    s[-2 * step] = static_cast<uint8_t>((p2 + p1 + p0 + q0 + 2) >> 2);
    s[-3 * step] = static_cast<uint8_t>((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
  } else {
    s[-step] = static_cast<uint8_t>((2 * p1 + p0 + q1 + 2) >> 2);
  }
  if (aq < beta && small) {
    s[0] = static_cast<uint8_t>((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
    s[step] = static_cast<uint8_t>((p0 + q0 + q1 + q2 + 2) >> 2);
    s[2 * step] = static_cast<uint8_t>((2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3);
  } else {
    s[0] = static_cast<uint8_t>((2 * q1 + q0 + p1 + 2) >> 2);
  }
}

// Deblock macroblock `a` of the frame in `slot` (all of its edges, 8.7)
VTS_HD inline void deblock_mb(const ReconCtx &c, int slot, int a) {
  const MbRec &q = c.recs[a];
  const FullSlice &sd = c.slices[q.slice];
  if (sd.dbk_idc == 1) return;
  const int mx = a % c.mbw, my = a / c.mbw;
  bool left = mx > 0, top = my > 0;
  if (sd.dbk_idc == 2) {
    if (left && c.recs[a - 1].slice != q.slice) left = false;
    if (top && c.recs[a - c.mbw].slice != q.slice) top = false;
  }
  uint8_t *Y = c.surf + static_cast<int64_t>(slot) * c.frame_stride;
  uint8_t *UV = Y + c.uv_off;
  const bool t8 = (q.modes & kModeT8) != 0;
  for (int dir = 0; dir < 2; ++dir)
    for (int e = 0; e < 4; ++e) {
      if (e == 0 && !(dir ? top : left)) continue;
      const int pa = e == 0 ? (dir ? a - c.mbw : a - 1) : a;
      const MbRec &p = c.recs[pa];
      const MbRecB *p1 = c.recs1 ? &c.recs1[pa] : nullptr, *q1 = c.recs1 ? &c.recs1[a] : nullptr;
      const int qpp = p.type == kMbPcm ? 0 : p.qp, qpq = q.type == kMbPcm ? 0 : q.qp;
      {
        const int qpav = (qpp + qpq + 1) >> 1;
        const int iA = clip3(0, 51, qpav + sd.dbk_a), iB = clip3(0, 51, qpav + sd.dbk_b);
        const int alpha = kAl[iA], beta = kBe[iB];
        if (alpha && beta && !(t8 && (e & 1)))  // 8x8 transform: no 4-sample internal luma edges
          for (int k = 0; k < 16; ++k) {
            const int xq = dir ? k : 4 * e, yq = dir ? 4 * e : k;
            const int xp = dir ? xq : (xq + 15) & 15, yp = dir ? (yq + 15) & 15 : yq;
            const int bS = bs_of(p, p1, (yp >> 2) * 4 + (xp >> 2), q, q1, (yq >> 2) * 4 + (xq >> 2), e == 0);
            uint8_t *s = Y + static_cast<int64_t>(my * 16 + yq) * c.pitch + mx * 16 + xq;
            filter_line(s, dir ? c.pitch : 1, bS, false, iA, alpha, beta);
          }
      }
      if (e == 0 || e == 2)
        for (int pl = 0; pl < 2; ++pl) {
          const int off = pl ? c.cqp_off2 : c.cqp_off;
          const int qpav = (qpc_of(qpp, off) + qpc_of(qpq, off) + 1) >> 1;
          const int iA = clip3(0, 51, qpav + sd.dbk_a), iB = clip3(0, 51, qpav + sd.dbk_b);
          const int alpha = kAl[iA], beta = kBe[iB];
          if (!alpha || !beta) continue;
          for (int k = 0; k < 8; ++k) {
            const int xq = dir ? 2 * k : 4 * e, yq = dir ? 4 * e : 2 * k;
            const int xp = dir ? xq : (xq + 15) & 15, yp = dir ? (yq + 15) & 15 : yq;
            const int bS = bs_of(p, p1, (yp >> 2) * 4 + (xp >> 2), q, q1, (yq >> 2) * 4 + (xq >> 2), e == 0);
            const int cx = dir ? k : 2 * e, cy = dir ? 2 * e : k;
            uint8_t *s = UV + static_cast<int64_t>(my * 8 + cy) * c.pitch + 2 * (mx * 8 + cx) + pl;
            filter_line(s, dir ? c.pitch : 2, bS, true, iA, alpha, beta);
          }
        }
    }
}

}  // namespace full
}  // namespace vts
