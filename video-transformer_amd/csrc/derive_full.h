// derive_full.h — what the general decoder's CABAC path derives per picture
// after the syntax parse (parse_cabac.h), host + device code: the kernel
// h264_derive (decode_full.hip) runs it as a wavefront, one lane per
// macroblock row, rows two macroblocks apart (a macroblock's A, B, C, D
// neighbours are final before it starts); the CPU harness
// (tests/native/full_host.cpp) runs the same derive_load + derive_mb in
// raster order.
//
// Per macroblock, completing the syntax record in place (MbRec / MbRecB
// exactly as the standard's decoding process defines them):
//   * motion (8.4.1): P_Skip (8.4.1.1), direct prediction, spatial or
//     temporal, from the colocated picture's final records (8.4.1.2), and
//     mvp + mvd per (sub-)partition in decoding order (8.4.1.3), both lists;
//     ref / ref_slot per 8x8 quadrant and mv per 4x4 block, list 1 in MbRecB;
//   * Intra4x4PredMode / Intra8x8PredMode from prev / rem and the neighbours'
//     modes (8.3.1.1, 8.3.2.1; constrained_intra_pred), into i4;
//   * the intra dependency level (1 + the highest level among the
//     intra-predicted neighbours A, B, C, D of the same slice, else 0;
//     kNoLevel when not intra-predicted), which orders h264_intra_v2.
// Neighbours cross macroblock edges as DEdge records (a macroblock's right
// column / bottom row), never as re-read global records.  Every global word a
// macroblock needs except its mvds (inter partitions only) is loaded at once
// by derive_load, before any is used (DIn), so a wavefront step costs one
// memory round trip, not one per 4x4 block.
#pragma once
#include <cstdint>

#include "parse_full.h"

namespace vts {
namespace full {

// a macroblock's facts along its right column (raster 3, 7, 11, 15) or
// bottom row (raster 12..15), index k in order
struct DEdge {
  uint32_t mv[2][4];  // motion of the edge blocks [list][k] (x | y << 16; 0 for intra / unused list)
  int8_t ref[2][4];   // refIdxLX of the edge blocks (-1: intra / list unused)
  uint8_t im[4];      // Intra4x4PredMode of the edge blocks (I_NxN; 2 otherwise)
  uint32_t slice;     // MbRec.slice
  uint16_t lvl;       // intra dependency level (kNoLevel: not intra-predicted)
  uint8_t type;       // kMb*
  uint8_t ok;         // parsed in this run (MbRec.epoch)
};
static_assert(sizeof(DEdge) == 52, "DEdge layout");

// the current macroblock's derived motion and modes (per lane; LDS on the
// device: indexed at run time)
struct DWork {
  uint32_t mv[2][16];  // [list][raster 4x4]
  int8_t ref[2][4];    // [list][8x8]
  uint8_t im[16];      // Intra4x4PredMode per raster 4x4 (Intra_8x8: the 8x8's mode in its four)
};

struct DeriveCtx {
  MbRec *recs;               // the picture's records
  MbRecB *recs1;             // ... list-1 halves (streams with B slices), else null
  uint16_t *ilvl;            // the picture's intra dependency levels
  const MbRec *ring;         // the window's records: colocated pictures by slot
  const MbRecB *ring1;
  const FullSlice *slices;   // the window's slices (MbRec.slice)
  const SliceExt *exts;      // the window's SliceExt records
  int mbw, mbh;
  uint32_t epoch;
  int cip, direct8x8, bframes;
  int col;                   // the colocated picture's slot when every B slice of the picture names
                             // the same RefPicList1[0] (else -1: read per macroblock)
};

// The record words derive_mb reads, loaded together (derive_load)
struct DIn {
  uint32_t w0, w1, w4, w5, w8, w9;  // MbRec: epoch, slice, type | qp << 8 | cbp << 16 | modes << 24,
                                    // ref[4], i4[0..3], i4[4..7]
  uint32_t b0, b3;                  // MbRecB: ref1[4], direct (byte 0)
  // the colocated macroblock (c.col >= 0): MbRec words 5..7 (ref, ref_slot),
  // MbRecB words 0..2 (ref1, ref_slot1), the motion of its corner blocks 0,
  // 3, 12, 15 (direct_8x8_inference: the quadrants' colocated blocks; without
  // it direct_pred reads every block from the record); named fields, not
  // arrays, so they stay in registers
  uint32_t c5, c6, c7, d0, d1, d2;
  uint32_t cm0, cm3, cm12, cm15, cn0, cn3, cn12, cn15;
  const uint32_t *cw, *cb;  // the colocated records (MbRec, MbRecB) as words
};

VTS_HD VTS_INLINE uint32_t mv_pack(int x, int y) {
  return static_cast<uint32_t>(static_cast<uint16_t>(x)) | (static_cast<uint32_t>(static_cast<uint16_t>(y)) << 16);
}
VTS_HD VTS_INLINE int mv_x(uint32_t v) { return static_cast<int16_t>(v & 0xffffu); }
VTS_HD VTS_INLINE int mv_y(uint32_t v) { return static_cast<int16_t>(v >> 16); }
VTS_HD VTS_INLINE int p8_of(int b) { return (b >> 3) * 2 + ((b & 3) >> 1); }
VTS_HD VTS_INLINE int sbyte(uint32_t w, int i) { return static_cast<int8_t>((w >> (8 * i)) & 255u); }
VTS_HD VTS_INLINE int shalf(uint32_t lo, uint32_t hi, int i) {
  return static_cast<int16_t>(((i < 2 ? lo : hi) >> (16 * (i & 1))) & 0xffffu);
}

// colocated words of macroblock addr in picture slot col
VTS_HD VTS_INLINE void derive_load_col(const DeriveCtx &c, int addr, int col, DIn &in) {
  const int64_t nmb = static_cast<int64_t>(c.mbw) * c.mbh;
  const uint32_t *cw = reinterpret_cast<const uint32_t *>(c.ring + col * nmb + addr);
  const uint32_t *cb = reinterpret_cast<const uint32_t *>(c.ring1 + col * nmb + addr);
  in.cw = cw;
  in.cb = cb;
  in.c5 = cw[5];
  in.c6 = cw[6];
  in.c7 = cw[7];
  in.d0 = cb[0];
  in.d1 = cb[1];
  in.d2 = cb[2];
  in.cm0 = cw[16];
  in.cm3 = cw[19];
  in.cm12 = cw[28];
  in.cm15 = cw[31];
  in.cn0 = cb[16];
  in.cn3 = cb[19];
  in.cn12 = cb[28];
  in.cn15 = cb[31];
}
VTS_HD VTS_INLINE void derive_load(const DeriveCtx &c, int addr, DIn &in) {
  const uint32_t *w = reinterpret_cast<const uint32_t *>(c.recs + addr);
  in.w0 = w[0];
  in.w1 = w[1];
  in.w4 = w[4];
  in.w5 = w[5];
  in.w8 = w[8];
  in.w9 = w[9];
  in.b0 = in.b3 = 0;
  if (c.bframes) {
    const uint32_t *b = reinterpret_cast<const uint32_t *>(c.recs1 + addr);
    in.b0 = b[0];
    in.b3 = b[3];
  }
  if (c.col >= 0) derive_load_col(c, addr, c.col, in);
}

struct Deriver {
  const DeriveCtx &c;
  const DEdge *A, *B, *C, *D;  // available neighbours (same slice, parsed), else null
  DWork &w;
  const FullSlice &s;
  const SliceExt *x;
  uint32_t err;

  struct Mv {
    bool avail;
    int ref, x, y;
  };
  // list l's motion of the neighbouring 4x4 block at luma (xN, yN) relative
  // to the macroblock; inside it the blocks in `done` (8.4.1.3.2)
  VTS_HD VTS_INLINE Mv nb_mv(int xN, int yN, uint32_t done, int l) const {
    if (xN >= 0 && xN < 16 && yN >= 0) {
      const int b = (yN >> 2) * 4 + (xN >> 2);
      if (yN > 15 || !((done >> b) & 1u)) return Mv{false, -1, 0, 0};
      const uint32_t v = w.mv[l][b];
      return Mv{true, w.ref[l][p8_of(b)], mv_x(v), mv_y(v)};
    }
    if (yN >= 0 && xN >= 16) return Mv{false, -1, 0, 0};
    const DEdge *e;
    int k;
    if (yN < 0) {
      if (xN < 0) { e = D; k = 3; }
      else if (xN < 16) { e = B; k = xN >> 2; }
      else { e = C; k = 0; }
    } else {
      e = A;
      k = yN >> 2;
    }
    if (!e) return Mv{false, -1, 0, 0};
    const uint32_t v = e->mv[l][k];
    return Mv{true, e->ref[l][k], mv_x(v), mv_y(v)};
  }
  VTS_HD VTS_INLINE void mv_pred(int x0, int y0, int pw, int ph, int ref, uint32_t done, int *px, int *py, int l) const {
    const Mv a = nb_mv(x0 - 1, y0, done, l);
    Mv b = nb_mv(x0, y0 - 1, done, l);
    Mv cc = nb_mv(x0 + pw, y0 - 1, done, l);
    if (!cc.avail) cc = nb_mv(x0 - 1, y0 - 1, done, l);
    if (pw == 16 && ph == 8) {
      if (y0 == 0 && b.ref == ref) { *px = b.x; *py = b.y; return; }
      if (y0 == 8 && a.ref == ref) { *px = a.x; *py = a.y; return; }
    } else if (pw == 8 && ph == 16) {
      if (x0 == 0 && a.ref == ref) { *px = a.x; *py = a.y; return; }
      if (x0 == 8 && cc.ref == ref) { *px = cc.x; *py = cc.y; return; }
    }
    if (!b.avail && !cc.avail && a.avail) {
      b = a;
      cc = a;
    }
    const int match = (a.ref == ref) + (b.ref == ref) + (cc.ref == ref);
    if (match == 1) {  // values selected, not addresses (an address select puts the Mvs in scratch)
      *px = a.ref == ref ? a.x : (b.ref == ref ? b.x : cc.x);
      *py = a.ref == ref ? a.y : (b.ref == ref ? b.y : cc.y);
    } else {
      *px = median3(a.x, b.x, cc.x);
      *py = median3(a.y, b.y, cc.y);
    }
  }
  VTS_HD VTS_INLINE void set_motion(int b, int l, int ref, int mx, int my) {
    w.mv[l][b] = ref >= 0 ? mv_pack(mx, my) : 0u;
    w.ref[l][p8_of(b)] = static_cast<int8_t>(ref);
  }

  // 8.4.1.2: direct prediction of the 8x8 quadrants in `qmask` from the
  // colocated macroblock's words (in)
  VTS_HD VTS_INLINE void direct_pred(uint32_t qmask, const DIn &in) {
    int ref0 = -1, ref1 = -1, mp0x = 0, mp0y = 0, mp1x = 0, mp1y = 0;
    bool zero = false;
    const bool spatial = x->direct_spatial != 0;
    if (spatial) {
      int rf0 = -1, rf1 = -1;
#pragma unroll
      for (int l = 0; l < 2; ++l) {
        const Mv a = nb_mv(-1, 0, 0, l), b = nb_mv(0, -1, 0, l);
        Mv cc = nb_mv(16, -1, 0, l);
        if (!cc.avail) cc = nb_mv(-1, -1, 0, l);
        const int r = min_positive(a.ref, min_positive(b.ref, cc.ref));
        if (l) rf1 = r;
        else rf0 = r;
      }
      ref0 = rf0;
      ref1 = rf1;
      if (ref0 < 0 && ref1 < 0) {
        ref0 = ref1 = 0;
        zero = true;
      }
      if (!zero) {
        if (ref0 >= 0) mv_pred(0, 0, 16, 16, ref0, 0, &mp0x, &mp0y, 0);
        if (ref1 >= 0) mv_pred(0, 0, 16, 16, ref1, 0, &mp1x, &mp1y, 1);
      }
    }
    for (int blk = 0; blk < 16; ++blk) {
      const int q = p8_of(blk);
      if (!((qmask >> q) & 1u)) continue;
      const int cref = sbyte(in.c5, q), cref1 = sbyte(in.d0, q);
      const bool use0 = cref >= 0;
      const int ref_col = use0 ? cref : cref1;  // -1: intra
      // the colocated block: with direct_8x8_inference the quadrant's corner
      // block (in registers), else block blk itself (from the record)
      uint32_t cmv;
      if (c.direct8x8) {
        const uint32_t c0 = use0 ? in.cm0 : in.cn0, c3 = use0 ? in.cm3 : in.cn3;
        const uint32_t c12 = use0 ? in.cm12 : in.cn12, c15 = use0 ? in.cm15 : in.cn15;
        cmv = q == 0 ? c0 : (q == 1 ? c3 : (q == 2 ? c12 : c15));
      } else {
        cmv = use0 ? in.cw[16 + blk] : in.cb[16 + blk];
      }
      const int mcx = ref_col < 0 ? 0 : mv_x(cmv), mcy = ref_col < 0 ? 0 : mv_y(cmv);
      if (spatial) {
        const bool col_zero = x->col_short && ref_col == 0 && mcx >= -1 && mcx <= 1 && mcy >= -1 && mcy <= 1;
        const bool z0 = zero || ref0 < 0 || (ref0 == 0 && col_zero);
        const bool z1 = zero || ref1 < 0 || (ref1 == 0 && col_zero);
        set_motion(blk, 0, ref0, z0 ? 0 : mp0x, z0 ? 0 : mp0y);
        set_motion(blk, 1, ref1, z1 ? 0 : mp1x, z1 ? 0 : mp1y);
      } else {
        int r0 = 0;
        if (ref_col >= 0) {  // the lowest list-0 index naming the colocated block's reference picture
          const int slot = use0 ? shalf(in.c6, in.c7, q) : shalf(in.d1, in.d2, q);
          r0 = -1;
          for (int i = s.num_ref - 1; i >= 0; --i)
            if (s.ref_slot[i] == slot) r0 = i;
          if (r0 < 0) {
            err |= DEC_E_NO_REF;
            r0 = 0;
          }
        }
        int m0x = mcx, m0y = mcy, m1x = 0, m1y = 0;
        const int tb = clip3i(-128, 127, x->poc - x->poc0[r0]), td = clip3i(-128, 127, x->poc1[0] - x->poc0[r0]);
        if (!((x->lt0 >> r0) & 1u) && td != 0) {
          const int tx = (16384 + (td < 0 ? -td : td) / 2) / td;
          const int dsf = clip3i(-1024, 1023, (tb * tx + 32) >> 6);
          m0x = (dsf * mcx + 128) >> 8;
          m0y = (dsf * mcy + 128) >> 8;
          m1x = m0x - mcx;
          m1y = m0y - mcy;
        }
        set_motion(blk, 0, r0, m0x, m0y);
        set_motion(blk, 1, 0, m1x, m1y);
      }
    }
  }

  // mvp + mvd per (sub-)partition in decoding order; partitions of prediction
  // 0 (B_8x8 direct) by direct_pred.  The mvds are read from the record here
  // (the sub-partition's first block holds them).
  VTS_HD VTS_INLINE void partitions(int addr, const DIn &in) {
    const int shape = static_cast<int>(in.w8 & 3u);
    const uint32_t pms = (in.w8 >> 8) & 255u, subs = (in.w8 >> 16) & 255u;
    const int nparts = shape == 0 ? 1 : (shape < 3 ? 2 : 4);
    const uint32_t *mvd0 = reinterpret_cast<const uint32_t *>(c.recs + addr) + 16;
    const uint32_t *mvd1 = c.bframes ? reinterpret_cast<const uint32_t *>(c.recs1 + addr) + 16 : nullptr;
    uint32_t done = 0;
    for (int k = 0; k < nparts; ++k) {
      const int pm = static_cast<int>((pms >> (2 * k)) & 3u), sub = static_cast<int>((subs >> (2 * k)) & 3u);
      int nsub = 1, pw, ph, x0, y0;
      if (shape == 0) { pw = ph = 16; x0 = y0 = 0; }
      else if (shape == 1) { pw = 16; ph = 8; x0 = 0; y0 = 8 * k; }
      else if (shape == 2) { pw = 8; ph = 16; x0 = 8 * k; y0 = 0; }
      else {
        x0 = 8 * (k & 1);
        y0 = 8 * (k >> 1);
        nsub = sub == 0 ? 1 : (sub == 3 ? 4 : 2);
        pw = (sub == 0 || sub == 1) ? 8 : 4;
        ph = (sub == 0 || sub == 2) ? 8 : 4;
      }
      const int q8 = (y0 / 8) * 2 + x0 / 8;
      if (pm == 0) {  // B_8x8 direct quadrant
        direct_pred(1u << q8, in);
        done |= 0x33u << ((y0 / 4) * 4 + x0 / 4);
        continue;
      }
      const int r0 = (pm & 1) ? sbyte(in.w5, q8) : -1, r1 = (pm & 2) ? sbyte(in.b0, q8) : -1;
      for (int q = 0; q < nsub; ++q) {
        int sx = x0, sy = y0;
        if (shape == 3) {
          if (sub == 1) sy += 4 * q;
          else if (sub == 2) sx += 4 * q;
          else if (sub == 3) { sx += 4 * (q & 1); sy += 4 * (q >> 1); }
        }
        const int b0 = (sy / 4) * 4 + sx / 4;
        const uint32_t d0 = (pm & 1) ? mvd0[b0] : 0u, d1 = (pm & 2) ? mvd1[b0] : 0u;
        int v0x = 0, v0y = 0, v1x = 0, v1y = 0;
        if (pm & 1) {
          int px, py;
          mv_pred(sx, sy, pw, ph, r0, done, &px, &py, 0);
          v0x = px + mv_x(d0);
          v0y = py + mv_y(d0);
        }
        if (pm & 2) {
          int px, py;
          mv_pred(sx, sy, pw, ph, r1, done, &px, &py, 1);
          v1x = px + mv_x(d1);
          v1y = py + mv_y(d1);
        }
        if (v0x < -32768 || v0x > 32767 || v0y < -32768 || v0y > 32767 || v1x < -32768 || v1x > 32767 ||
            v1y < -32768 || v1y > 32767)
          err |= DEC_E_SYNTAX;
        const uint32_t bm = blk_mask(sx, sy, pw, ph);
        for (int b = 0; b < 16; ++b)
          if ((bm >> b) & 1u) {
            set_motion(b, 0, r0, v0x, v0y);
            set_motion(b, 1, r1, v1x, v1y);
          }
        done |= bm;
      }
    }
  }

  // Intra4x4PredMode / Intra8x8PredMode predictor of the block at (x0, y0)
  // (8.3.1.1 / 8.3.2.1; frame macroblocks: the neighbouring 4x4 block is the
  // one the standard names for both block sizes)
  VTS_HD VTS_INLINE int mode_pred(int x0, int y0) const {
    if ((x0 == 0 && !A) || (y0 == 0 && !B)) return 2;
    const int ta = x0 ? static_cast<int>(kMbI4x4) : A->type, tb = y0 ? static_cast<int>(kMbI4x4) : B->type;
    if (c.cip && (ta == kMbInter || ta == kMbSkip || tb == kMbInter || tb == kMbSkip)) return 2;
    const int ma = ta != kMbI4x4 ? 2 : (x0 ? w.im[(y0 / 4) * 4 + x0 / 4 - 1] : A->im[y0 / 4]);
    const int mb = tb != kMbI4x4 ? 2 : (y0 ? w.im[(y0 / 4 - 1) * 4 + x0 / 4] : B->im[x0 / 4]);
    return vts_min(ma, mb);
  }
};

// The neighbours (A left, B above, C above-right, D above-left) whose samples
// an intra macroblock's prediction reads (8.3.1.2 Intra_4x4 by block and
// mode, 8.3.2.2 Intra_8x8 with its reference filtering, 8.3.3 Intra_16x16,
// 8.3.4 chroma).  Its reconstruction waits only for those of them this launch
// reconstructs; the others' samples, if loaded, go unused.  Intra 4x4 / 8x8
// modes: 0 V, 1 H, 2 DC, 3 diagonal down-left, 4 down-right, 5 vertical-
// right, 6 horizontal-down, 7 vertical-left, 8 horizontal-up.
constexpr uint32_t kUseA = 1, kUseB = 2, kUseC = 4, kUseD = 8;
VTS_HD VTS_INLINE uint32_t intra_uses(int ty, int modes, const uint8_t *im) {
  const int cm = (modes >> 2) & 3;  // chroma: DC, horizontal, vertical, plane
  uint32_t u = cm == 0 ? kUseA | kUseB : (cm == 1 ? kUseA : (cm == 2 ? kUseB : kUseA | kUseB | kUseD));
  if (ty == kMbI16) {
    const int m = modes & 3;  // vertical, horizontal, DC, plane
    return u | (m == 0 ? kUseB : (m == 1 ? kUseA : (m == 2 ? kUseA | kUseB : kUseA | kUseB | kUseD)));
  }
  auto top = [](int md) { return md != 1 && md != 8; };
  auto left = [](int md) { return md == 1 || md == 2 || md == 4 || md == 5 || md == 6 || md == 8; };
  if (modes & kModeT8) {
    // the filtered reference samples next to a used edge read its corner
    // neighbours too: block 0 top B + D, left A + D; block 1 top B + C,
    // left B (its p[-1, -1]); block 2 either A; block 3 none
    const int m0 = im[0], m1 = im[2], m2 = im[8];
    if (top(m0)) u |= kUseB | kUseD;
    if (left(m0)) u |= kUseA | kUseD;
    if (top(m1)) u |= kUseB | kUseC;
    if (left(m1)) u |= kUseB;
    if (top(m2) || left(m2)) u |= kUseA;
    return u;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {  // 4x4 blocks in raster order
    const int md = im[r], bx = r & 3, by = r >> 2;
    const bool tl = md == 4 || md == 5 || md == 6, tr = md == 3 || md == 7;
    if (by == 0 && top(md)) u |= kUseB;
    if (bx == 0 && left(md)) u |= kUseA;
    if (tl) u |= bx == 0 ? (by == 0 ? kUseD : kUseA) : (by == 0 ? kUseB : 0u);
    if (tr && by == 0) u |= bx == 3 ? kUseC : kUseB;
  }
  return u;
}

// Derive macroblock `addr` from its words `in` (derive_load) and its
// neighbours' edges A, B, C, D (null when outside the picture; another slice
// or an unparsed macroblock is dropped here), write the record's derived
// fields and ilvl, and return its right / bottom edges (written last: right
// may be the storage A came from).  DEC_E_* bits.
VTS_HD VTS_INLINE uint32_t derive_mb(const DeriveCtx &c, int addr, DIn &in, const DEdge *A, const DEdge *B,
                                     const DEdge *C, const DEdge *D, DWork &w, DEdge *right, DEdge *bottom) {
  if (in.w0 != c.epoch) {  // not parsed (a slice is missing): no neighbour of anyone
    right->ok = bottom->ok = 0;
    c.ilvl[addr] = kNoLevel;
    return DEC_E_MISSING_MB;
  }
  const uint32_t slice = in.w1;
  if (A && !(A->ok && A->slice == slice)) A = nullptr;
  if (B && !(B->ok && B->slice == slice)) B = nullptr;
  if (C && !(C->ok && C->slice == slice)) C = nullptr;
  if (D && !(D->ok && D->slice == slice)) D = nullptr;
  const FullSlice &s = c.slices[slice];
  Deriver d{c, A, B, C, D, w, s, s.ext >= 0 ? &c.exts[s.ext] : nullptr, 0u};
  const int ty = static_cast<int>(in.w4 & 255u);
  const int modes = static_cast<int>(in.w4 >> 24);
#pragma unroll
  for (int b = 0; b < 16; ++b) {
    w.mv[0][b] = 0;
    w.mv[1][b] = 0;
    w.im[b] = 2;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) w.ref[0][q] = w.ref[1][q] = -1;
  uint16_t lvl = kNoLevel;
  MbRec &m = c.recs[addr];
  if (ty == kMbInter || ty == kMbSkip) {
    const bool is_b = s.is_p == kSliceB;
    if (is_b && (!d.x || !c.bframes)) {
      d.err |= DEC_E_NO_REF;
    } else if (ty == kMbSkip && !is_b) {  // P_Skip (8.4.1.1)
      const Deriver::Mv a = d.nb_mv(-1, 0, 0, 0), b = d.nb_mv(0, -1, 0, 0);
      int px = 0, py = 0;
      if (!(!A || !B || (a.ref == 0 && a.x == 0 && a.y == 0) || (b.ref == 0 && b.x == 0 && b.y == 0)))
        d.mv_pred(0, 0, 16, 16, 0, 0, &px, &py, 0);
      if (s.ref_slot[0] < 0) d.err |= DEC_E_NO_REF;
#pragma unroll
      for (int blk = 0; blk < 16; ++blk) d.set_motion(blk, 0, 0, px, py);
    } else {
      if (is_b && c.col < 0) derive_load_col(c, addr, d.x->ref_slot1[0], in);  // the slice's own colocated picture
      if (is_b && (in.b3 & kDirect16)) d.direct_pred(15u, in);  // B_Skip, B_Direct_16x16
      else d.partitions(addr, in);
    }
    // the record's motion: final references, slots, vectors
    int8_t r0[4];
    int16_t sl0[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      r0[q] = w.ref[0][q];
      sl0[q] = r0[q] >= 0 ? s.ref_slot[r0[q] & 31] : static_cast<int16_t>(-1);
    }
    uint32_t *mw = reinterpret_cast<uint32_t *>(&m);
    mw[5] = static_cast<uint32_t>(static_cast<uint8_t>(r0[0])) | (static_cast<uint32_t>(static_cast<uint8_t>(r0[1])) << 8) |
            (static_cast<uint32_t>(static_cast<uint8_t>(r0[2])) << 16) | (static_cast<uint32_t>(static_cast<uint8_t>(r0[3])) << 24);
    mw[6] = static_cast<uint32_t>(static_cast<uint16_t>(sl0[0])) | (static_cast<uint32_t>(static_cast<uint16_t>(sl0[1])) << 16);
    mw[7] = static_cast<uint32_t>(static_cast<uint16_t>(sl0[2])) | (static_cast<uint32_t>(static_cast<uint16_t>(sl0[3])) << 16);
#pragma unroll
    for (int b = 0; b < 16; ++b) mw[16 + b] = w.mv[0][b];
    if (c.bframes) {
      int8_t r1[4];
      int16_t sl1[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        r1[q] = w.ref[1][q];
        sl1[q] = r1[q] >= 0 && d.x ? d.x->ref_slot1[r1[q] & 31] : static_cast<int16_t>(-1);
      }
      uint32_t *bw = reinterpret_cast<uint32_t *>(&c.recs1[addr]);
      bw[0] = static_cast<uint32_t>(static_cast<uint8_t>(r1[0])) | (static_cast<uint32_t>(static_cast<uint8_t>(r1[1])) << 8) |
              (static_cast<uint32_t>(static_cast<uint8_t>(r1[2])) << 16) | (static_cast<uint32_t>(static_cast<uint8_t>(r1[3])) << 24);
      bw[1] = static_cast<uint32_t>(static_cast<uint16_t>(sl1[0])) | (static_cast<uint32_t>(static_cast<uint16_t>(sl1[1])) << 16);
      bw[2] = static_cast<uint32_t>(static_cast<uint16_t>(sl1[2])) | (static_cast<uint32_t>(static_cast<uint16_t>(sl1[3])) << 16);
#pragma unroll
      for (int b = 0; b < 16; ++b) bw[16 + b] = w.mv[1][b];
    }
  } else if (ty == kMbI4x4 || ty == kMbI16) {
    if (ty == kMbI4x4) {
      const bool t8 = (modes & kModeT8) != 0;
      const int nb = t8 ? 4 : 16;
      for (int i = 0; i < nb; ++i) {
        const int x0 = t8 ? (i & 1) * 8 : blk_x(i) * 4, y0 = t8 ? (i >> 1) * 8 : blk_y(i) * 4;
        const int r = (y0 / 4) * 4 + x0 / 4;
        const int syn = static_cast<int>(((r < 8 ? in.w8 : in.w9) >> (4 * (r & 7))) & 15u);
        const int pm = d.mode_pred(x0, y0);
        const int mode = (syn & 8) ? pm : (syn < pm ? syn : syn + 1);
        w.im[r] = static_cast<uint8_t>(mode);
        if (t8) {
          w.im[r + 1] = static_cast<uint8_t>(mode);
          w.im[r + 4] = static_cast<uint8_t>(mode);
          w.im[r + 5] = static_cast<uint8_t>(mode);
        }
      }
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        lo |= static_cast<uint32_t>(w.im[b]) << (4 * b);
        hi |= static_cast<uint32_t>(w.im[8 + b]) << (4 * b);
      }
      uint32_t *mw = reinterpret_cast<uint32_t *>(&m);
      mw[8] = lo;
      mw[9] = hi;
    }
    // only the intra neighbours whose samples it predicts from order it
    const uint32_t use = intra_uses(ty, modes, w.im);
    int l = 0;
    if ((use & kUseA) && A && A->lvl != kNoLevel) l = vts_max(l, A->lvl + 1);
    if ((use & kUseB) && B && B->lvl != kNoLevel) l = vts_max(l, B->lvl + 1);
    if ((use & kUseC) && C && C->lvl != kNoLevel) l = vts_max(l, C->lvl + 1);
    if ((use & kUseD) && D && D->lvl != kNoLevel) l = vts_max(l, D->lvl + 1);
    lvl = static_cast<uint16_t>(l);
  }
  c.ilvl[addr] = lvl;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int br = 4 * k + 3, bb = 12 + k;
#pragma unroll
    for (int l = 0; l < 2; ++l) {
      right->mv[l][k] = w.mv[l][br];
      right->ref[l][k] = w.ref[l][p8_of(br)];
      bottom->mv[l][k] = w.mv[l][bb];
      bottom->ref[l][k] = w.ref[l][p8_of(bb)];
    }
    right->im[k] = w.im[br];
    bottom->im[k] = w.im[bb];
  }
  right->slice = bottom->slice = slice;
  right->lvl = bottom->lvl = lvl;
  right->type = bottom->type = static_cast<uint8_t>(ty);
  right->ok = bottom->ok = 1;
  return d.err;
}

}  // namespace full
}  // namespace vts
