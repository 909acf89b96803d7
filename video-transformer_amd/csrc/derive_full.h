// derive_full.h — what the general decoder's CABAC path derives per picture
// after the syntax parse (parse_cabac.h), host + device code: the kernel
// h264_derive (decode_full.hip) runs it as a wavefront, one lane per
// macroblock row, rows two macroblocks apart (a macroblock's A, B, C, D
// neighbours are final before it starts); the CPU harness
// (tests/native/full_host.cpp) runs the same derive_mb in raster order.
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
// column / bottom row), never as re-read global records.
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
};

VTS_HD VTS_INLINE uint32_t mv_pack(int x, int y) {
  return static_cast<uint32_t>(static_cast<uint16_t>(x)) | (static_cast<uint32_t>(static_cast<uint16_t>(y)) << 16);
}
VTS_HD VTS_INLINE int mv_x(uint32_t v) { return static_cast<int16_t>(v & 0xffffu); }
VTS_HD VTS_INLINE int mv_y(uint32_t v) { return static_cast<int16_t>(v >> 16); }
VTS_HD VTS_INLINE int p8_of(int b) { return (b >> 3) * 2 + ((b & 3) >> 1); }

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
    if (match == 1) {
      const Mv &m = a.ref == ref ? a : (b.ref == ref ? b : cc);
      *px = m.x;
      *py = m.y;
    } else {
      *px = median3(a.x, b.x, cc.x);
      *py = median3(a.y, b.y, cc.y);
    }
  }
  VTS_HD VTS_INLINE void set_motion(int b, int l, int ref, int mx, int my) {
    w.mv[l][b] = ref >= 0 ? mv_pack(mx, my) : 0u;
    w.ref[l][p8_of(b)] = static_cast<int8_t>(ref);
  }

  // 8.4.1.2: direct prediction of the raster 4x4 blocks in `mask`
  VTS_HD VTS_INLINE void direct_pred(int addr, uint32_t mask) {
    const int64_t nmb = static_cast<int64_t>(c.mbw) * c.mbh;
    const int col = x->ref_slot1[0];  // RefPicList1[0], derived before this picture
    const MbRec &cm = c.ring[col * nmb + addr];
    const MbRecB &cm1 = c.ring1[col * nmb + addr];
    int ref0 = -1, ref1 = -1, mp[2][2] = {{0, 0}, {0, 0}};
    bool zero = false;
    if (x->direct_spatial) {
      int rf[2];
#pragma unroll
      for (int l = 0; l < 2; ++l) {
        const Mv a = nb_mv(-1, 0, 0, l), b = nb_mv(0, -1, 0, l);
        Mv cc = nb_mv(16, -1, 0, l);
        if (!cc.avail) cc = nb_mv(-1, -1, 0, l);
        rf[l] = min_positive(a.ref, min_positive(b.ref, cc.ref));
      }
      ref0 = rf[0];
      ref1 = rf[1];
      if (ref0 < 0 && ref1 < 0) {
        ref0 = ref1 = 0;
        zero = true;
      }
      if (!zero) {
        if (ref0 >= 0) mv_pred(0, 0, 16, 16, ref0, 0, &mp[0][0], &mp[0][1], 0);
        if (ref1 >= 0) mv_pred(0, 0, 16, 16, ref1, 0, &mp[1][0], &mp[1][1], 1);
      }
    }
    for (int blk = 0; blk < 16; ++blk) {
      if (!((mask >> blk) & 1u)) continue;
      const int cb = c.direct8x8 ? ((blk >> 3) * 3) * 4 + ((blk & 3) >> 1) * 3 : blk;
      const int c8 = p8_of(cb);
      const bool use0 = cm.ref[c8] >= 0;
      const int ref_col = use0 ? cm.ref[c8] : cm1.ref1[c8];  // -1: intra
      const int mcx = ref_col < 0 ? 0 : (use0 ? cm.mv[cb][0] : cm1.mv1[cb][0]);
      const int mcy = ref_col < 0 ? 0 : (use0 ? cm.mv[cb][1] : cm1.mv1[cb][1]);
      if (x->direct_spatial) {
        const bool col_zero = x->col_short && ref_col == 0 && mcx >= -1 && mcx <= 1 && mcy >= -1 && mcy <= 1;
        const bool z0 = zero || ref0 < 0 || (ref0 == 0 && col_zero);
        const bool z1 = zero || ref1 < 0 || (ref1 == 0 && col_zero);
        set_motion(blk, 0, ref0, z0 ? 0 : mp[0][0], z0 ? 0 : mp[0][1]);
        set_motion(blk, 1, ref1, z1 ? 0 : mp[1][0], z1 ? 0 : mp[1][1]);
      } else {
        int r0 = 0;
        if (ref_col >= 0) {  // the lowest list-0 index naming the colocated block's reference picture
          const int slot = use0 ? cm.ref_slot[c8] : cm1.ref_slot1[c8];
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
  // 0 (B_8x8 direct) by direct_pred
  VTS_HD VTS_INLINE void partitions(int addr, const MbRec &m, const MbRecB *m1) {
    const int shape = m.i4[0] & 3;
    const int nparts = shape == 0 ? 1 : (shape < 3 ? 2 : 4);
    uint32_t done = 0;
    for (int k = 0; k < nparts; ++k) {
      const int pm = (m.i4[1] >> (2 * k)) & 3, sub = (m.i4[2] >> (2 * k)) & 3;
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
      if (pm == 0) {  // B_8x8 direct quadrant
        const uint32_t bm = 0x33u << ((y0 / 4) * 4 + x0 / 4);
        direct_pred(addr, bm);
        done |= bm;
        continue;
      }
      const int q8 = (y0 / 8) * 2 + x0 / 8;
      const int r0 = (pm & 1) ? m.ref[q8] : -1, r1 = (pm & 2) ? m1->ref1[q8] : -1;
      for (int q = 0; q < nsub; ++q) {
        int sx = x0, sy = y0;
        if (shape == 3) {
          if (sub == 1) sy += 4 * q;
          else if (sub == 2) sx += 4 * q;
          else if (sub == 3) { sx += 4 * (q & 1); sy += 4 * (q >> 1); }
        }
        const int b0 = (sy / 4) * 4 + sx / 4;  // the sub-partition's first block holds its mvd
        int v[2][2] = {{0, 0}, {0, 0}};
#pragma unroll
        for (int l = 0; l < 2; ++l) {
          if (!((pm >> l) & 1)) continue;
          int px, py;
          mv_pred(sx, sy, pw, ph, l ? r1 : r0, done, &px, &py, l);
          v[l][0] = px + (l ? m1->mv1[b0][0] : m.mv[b0][0]);
          v[l][1] = py + (l ? m1->mv1[b0][1] : m.mv[b0][1]);
          if (v[l][0] < -32768 || v[l][0] > 32767 || v[l][1] < -32768 || v[l][1] > 32767) err |= DEC_E_SYNTAX;
        }
        const uint32_t bm = blk_mask(sx, sy, pw, ph);
        for (int b = 0; b < 16; ++b)
          if ((bm >> b) & 1u) {
            set_motion(b, 0, r0, v[0][0], v[0][1]);
            set_motion(b, 1, r1, v[1][0], v[1][1]);
          }
        done |= bm;
      }
    }
  }

  // Intra4x4PredMode / Intra8x8PredMode predictor of the block at (x0, y0)
  // (8.3.1.1 / 8.3.2.1; frame macroblocks: the neighbouring 4x4 block is the
  // one the standard names for both block sizes)
  VTS_HD VTS_INLINE int mode_pred(int x0, int y0, int ty_cur) const {
    const DEdge *ea = x0 == 0 ? A : nullptr, *eb = y0 == 0 ? B : nullptr;
    if ((x0 == 0 && !A) || (y0 == 0 && !B)) return 2;
    const int ta = x0 ? ty_cur : ea->type, tb = y0 ? ty_cur : eb->type;
    if (c.cip && (ta == kMbInter || ta == kMbSkip || tb == kMbInter || tb == kMbSkip)) return 2;
    const int ma = ta != kMbI4x4 ? 2 : (x0 ? w.im[(y0 / 4) * 4 + x0 / 4 - 1] : ea->im[y0 / 4]);
    const int mb = tb != kMbI4x4 ? 2 : (y0 ? w.im[(y0 / 4 - 1) * 4 + x0 / 4] : eb->im[x0 / 4]);
    return vts_min(ma, mb);
  }
};

// Derive macroblock `addr` (its neighbours' edges A, B, C, D: null when
// outside the picture, in another slice or not parsed), write the record's
// derived fields and ilvl, and return its right / bottom edges.  DEC_E_* bits.
VTS_HD VTS_INLINE uint32_t derive_mb(const DeriveCtx &c, int addr, const DEdge *A, const DEdge *B, const DEdge *C,
                                     const DEdge *D, DWork &w, DEdge *right, DEdge *bottom) {
  MbRec &m = c.recs[addr];
  MbRecB *m1 = c.bframes ? &c.recs1[addr] : nullptr;
  if (m.epoch != c.epoch) {  // not parsed (a slice is missing): no neighbour of anyone
    right->ok = bottom->ok = 0;
    c.ilvl[addr] = kNoLevel;
    return DEC_E_MISSING_MB;
  }
  const uint32_t slice = m.slice;
  auto same = [&](const DEdge *e) -> const DEdge * { return (e && e->ok && e->slice == slice) ? e : nullptr; };
  A = same(A);
  B = same(B);
  C = same(C);
  D = same(D);
  const FullSlice &s = c.slices[slice];
  Deriver d{c, A, B, C, D, w, s, s.ext >= 0 ? &c.exts[s.ext] : nullptr, 0u};
  const int ty = m.type;
  for (int l = 0; l < 2; ++l) {
    for (int b = 0; b < 16; ++b) w.mv[l][b] = 0;
    for (int q = 0; q < 4; ++q) w.ref[l][q] = -1;
  }
  for (int b = 0; b < 16; ++b) w.im[b] = 2;
  uint16_t lvl = kNoLevel;
  if (ty == kMbInter || ty == kMbSkip) {
    const bool is_b = s.is_p == kSliceB;
    if (is_b && (!d.x || !m1)) {
      d.err |= DEC_E_NO_REF;
    } else if (ty == kMbSkip && !is_b) {  // P_Skip (8.4.1.1)
      const Deriver::Mv a = d.nb_mv(-1, 0, 0, 0), b = d.nb_mv(0, -1, 0, 0);
      int px = 0, py = 0;
      if (!(!A || !B || (a.ref == 0 && a.x == 0 && a.y == 0) || (b.ref == 0 && b.x == 0 && b.y == 0)))
        d.mv_pred(0, 0, 16, 16, 0, 0, &px, &py, 0);
      if (s.ref_slot[0] < 0) d.err |= DEC_E_NO_REF;
      for (int blk = 0; blk < 16; ++blk) d.set_motion(blk, 0, 0, px, py);
    } else if (is_b && (m1->direct & kDirect16)) {  // B_Skip, B_Direct_16x16
      d.direct_pred(addr, 0xffffu);
    } else {
      d.partitions(addr, m, m1);
    }
    // the record's motion: final references, slots, vectors
    for (int q = 0; q < 4; ++q) {
      const int r0 = w.ref[0][q];
      m.ref[q] = static_cast<int8_t>(r0);
      m.ref_slot[q] = r0 >= 0 ? s.ref_slot[r0 & 31] : static_cast<int16_t>(-1);
    }
    for (int b = 0; b < 16; ++b) {
      m.mv[b][0] = static_cast<int16_t>(mv_x(w.mv[0][b]));
      m.mv[b][1] = static_cast<int16_t>(mv_y(w.mv[0][b]));
    }
    if (m1) {
      for (int q = 0; q < 4; ++q) {
        const int r1 = w.ref[1][q];
        m1->ref1[q] = static_cast<int8_t>(r1);
        m1->ref_slot1[q] = r1 >= 0 && d.x ? d.x->ref_slot1[r1 & 31] : static_cast<int16_t>(-1);
      }
      for (int b = 0; b < 16; ++b) {
        m1->mv1[b][0] = static_cast<int16_t>(mv_x(w.mv[1][b]));
        m1->mv1[b][1] = static_cast<int16_t>(mv_y(w.mv[1][b]));
      }
    }
  } else if (ty == kMbI4x4 || ty == kMbI16) {
    if (ty == kMbI4x4) {
      const bool t8 = (m.modes & kModeT8) != 0;
      const int nb = t8 ? 4 : 16;
      for (int i = 0; i < nb; ++i) {
        const int x0 = t8 ? (i & 1) * 8 : blk_x(i) * 4, y0 = t8 ? (i >> 1) * 8 : blk_y(i) * 4;
        const int r = (y0 / 4) * 4 + x0 / 4;
        const int syn = (m.i4[r >> 1] >> ((r & 1) * 4)) & 15;
        const int pm = d.mode_pred(x0, y0, ty);
        const int mode = (syn & 8) ? pm : (syn < pm ? syn : syn + 1);
        w.im[r] = static_cast<uint8_t>(mode);
        if (t8) {
          w.im[r + 1] = static_cast<uint8_t>(mode);
          w.im[r + 4] = static_cast<uint8_t>(mode);
          w.im[r + 5] = static_cast<uint8_t>(mode);
        }
      }
      for (int j = 0; j < 8; ++j) m.i4[j] = static_cast<uint8_t>(w.im[2 * j] | (w.im[2 * j + 1] << 4));
    }
    int l = 0;
    const DEdge *nb[4] = {A, B, C, D};
    for (int i = 0; i < 4; ++i)
      if (nb[i] && nb[i]->lvl != kNoLevel) l = vts_max(l, nb[i]->lvl + 1);
    lvl = static_cast<uint16_t>(l);
  }
  c.ilvl[addr] = lvl;
  for (int k = 0; k < 4; ++k) {
    const int br = 4 * k + 3, bb = 12 + k;
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
