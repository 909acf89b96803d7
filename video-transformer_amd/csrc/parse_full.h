// parse_full.h — CAVLC slice_data() parser of the general device decoder
// (h264_parse_full in decode_full.hip runs one lane of it per slice; the CPU
// harness tests/native/full_host.cpp compiles the same code for the host).
//
// The host has already parsed the slice header (h264_sched.cpp) and hands
// over where slice_data() starts, the slice QP and RefPicList0 as ring slots.
// Per macroblock the lane derives everything later stages need and the
// standard derives from syntax alone — Intra_4x4 modes (8.3.1.1), motion
// vectors (8.4.1.3, P_Skip 8.4.1.1), QPY, total_coeff — and writes one MbRec
// plus its non-zero coefficient blocks (raster order, int16) into the slice's
// reserved arena range.  Errors come back as DEC_E_* bits.
#pragma once
#include <cstdint>

#include "h264.h"
#include "h264_full.h"
#include "h264_tables.h"
#include "parse_slice.h"  // WinBits, VTS_HD, VTS_INLINE

#ifndef VTS_PARSE_TRACE
#define VTS_PARSE_TRACE(...)
#endif

namespace vts {
namespace full {

// ---------------------------------------------------- VLC lookup tables
// coeff_token: [class][leading zeros 0..15][3 bits after the first 1] ->
// len | TotalCoeff << 5 | TrailingOnes << 10; 0 = no code.  (Chroma DC's
// all-zero 7-bit code for TotalCoeff 4 / T1 3 is handled by the reader.)
struct CtLut {
  uint16_t v[4][16][8];
};
constexpr CtLut make_ct_lut() {
  CtLut t{};
  const uint8_t len[4][17][4] = VTS_CT_LEN_DATA;
  const uint8_t code[4][17][4] = VTS_CT_CODE_DATA;
  for (int c = 0; c < 4; ++c)
    for (int tc = 0; tc < 17; ++tc)
      for (int t1 = 0; t1 < 4; ++t1) {
        const int l = len[c][tc][t1];
        if (l == 0) continue;
        const unsigned v = code[c][tc][t1];
        int lz = 0;
        while (lz < l && !((v >> (l - 1 - lz)) & 1u)) ++lz;
        if (lz == l) continue;  // all zeros (chroma DC 0000000)
        const int rest = l - lz - 1;  // bits after the first 1 (<= 3)
        const unsigned suffix = v & ((1u << rest) - 1u);
        for (unsigned s = 0; s < 8; ++s)
          if ((s >> (3 - rest)) == suffix)
            t.v[c][lz][s] = static_cast<uint16_t>(l | (tc << 5) | (t1 << 10));
      }
  return t;
}
// total_zeros (4x4): [TotalCoeff - 1][next 9 bits] -> total_zeros | len << 4
struct TzLut {
  uint8_t v[15][512];
  uint8_t dc[3][8];  // chroma DC: [TotalCoeff - 1][next 3 bits]
};
constexpr TzLut make_tz_lut() {
  TzLut t{};
  const uint8_t len[15][16] = VTS_TZ_LEN_DATA;
  const uint8_t code[15][16] = VTS_TZ_CODE_DATA;
  for (int tc = 0; tc < 15; ++tc)
    for (int z = 0; z < 16; ++z) {
      const int l = len[tc][z];
      if (l == 0) continue;
      for (unsigned s = 0; s < 512; ++s)
        if ((s >> (9 - l)) == code[tc][z]) t.v[tc][s] = static_cast<uint8_t>(z | (l << 4));
    }
  const uint8_t dlen[3][4] = VTS_TZC_LEN_DATA;
  const uint8_t dcode[3][4] = VTS_TZC_CODE_DATA;
  for (int tc = 0; tc < 3; ++tc)
    for (int z = 0; z < 4; ++z) {
      const int l = dlen[tc][z];
      if (l == 0) continue;
      for (unsigned s = 0; s < 8; ++s)
        if ((s >> (3 - l)) == dcode[tc][z]) t.dc[tc][s] = static_cast<uint8_t>(z | (l << 4));
    }
  return t;
}
// run_before for zerosLeft 1..6: [zerosLeft - 1][next 3 bits] -> run | len << 4
// (zerosLeft > 6: 3-bit codes 111..001 = runs 0..6, then 0001.. = 7.. by count)
struct RbLut {
  uint8_t v[6][8];
};
constexpr RbLut make_rb_lut() {
  RbLut t{};
  const uint8_t len[7][15] = VTS_RB_LEN_DATA;
  const uint8_t code[7][15] = VTS_RB_CODE_DATA;
  for (int r = 0; r < 6; ++r)
    for (int z = 0; z < 15; ++z) {
      const int l = len[r][z];
      if (l == 0) continue;
      for (unsigned s = 0; s < 8; ++s)
        if ((s >> (3 - l)) == code[r][z]) t.v[r][s] = static_cast<uint8_t>(z | (l << 4));
    }
  return t;
}

#if defined(__HIPCC__)
__device__ __constant__ static const CtLut kCtLut = make_ct_lut();
__device__ __constant__ static const TzLut kTzLut = make_tz_lut();
__device__ __constant__ static const RbLut kRbLut = make_rb_lut();
#define kZz h264::kdZigzag4x4
#define kCbpI h264::kdCbpIntra
#define kCbpP h264::kdCbpInter
#else
static const CtLut kCtLut = make_ct_lut();
static const TzLut kTzLut = make_tz_lut();
static const RbLut kRbLut = make_rb_lut();
static const uint8_t *const kZz = h264::kZigzag4x4;
static const uint8_t *const kCbpI = h264::kCbpIntra;
static const uint8_t *const kCbpP = h264::kCbpInter;
#endif

// luma4x4BlkIdx <-> raster 4x4 block
VTS_HD VTS_INLINE int blk_x(int k) { return ((k >> 2) & 1) * 2 + (k & 1); }
VTS_HD VTS_INLINE int blk_y(int k) { return ((k >> 3) & 1) * 2 + ((k >> 1) & 1); }

// Per-lane scratch (LDS on the device).
struct FullScratch {
  MbRec cur;              // the macroblock being parsed
  int16_t blk[16];        // coefficient block being decoded (raster)
  uint32_t cache[6];      // WinBits byte cache
};

struct Parser {
  WinBits br;
  const FullSlice *s;
  const FullParams *P;
  MbRec *recs;            // the frame's records (global)
  uint16_t *ilvl;         // the frame's intra dependency levels (kNoLevel: not intra-predicted)
  int16_t *arena;         // window coefficient arena, 16 int16 per block
  FullScratch *sc;
  uint32_t used;          // blocks stored so far in the slice
  uint32_t slice_index;
  uint32_t epoch;
  int mbw;
  int first_mb;
  uint32_t err;

  // --- neighbour access (6.4.12): mb -1 unavailable, -2 the current MB
  VTS_HD VTS_INLINE int nb_mb(int cur, int xN, int yN, int maxW, int *xw, int *yw) const {
    if (yN > maxW - 1) return -1;
    const int mx = cur % mbw;
    int n;
    const bool top_row = cur < mbw;  // nothing above the picture
    if (xN < 0 && yN < 0) n = (mx > 0 && !top_row) ? cur - mbw - 1 : -1;
    else if (xN < 0) n = mx > 0 ? cur - 1 : -1;
    else if (xN < maxW && yN < 0) n = top_row ? -1 : cur - mbw;
    else if (xN < maxW) n = -2;  // the current macroblock
    else if (yN < 0) n = (mx < mbw - 1 && !top_row) ? cur - mbw + 1 : -1;
    else return -1;
    if (n >= 0 && n < first_mb) n = -1;  // another slice (slices are contiguous in decoding order)
    *xw = (xN + maxW) % maxW;
    *yw = (yN + maxW) % maxW;
    return n;
  }
  VTS_HD VTS_INLINE const MbRec &rec(int n) const { return n == -2 ? sc->cur : recs[n]; }

  // 9.2.1 nC
  VTS_HD int nc_of(int cur, int bx, int by, bool chroma, int plane) const {
    const int maxW = chroma ? 8 : 16;
    int xa, ya, xb, yb;
    const int a = nb_mb(cur, bx * 4 - 1, by * 4, maxW, &xa, &ya);
    const int b = nb_mb(cur, bx * 4, by * 4 - 1, maxW, &xb, &yb);
    int na = 0, nbv = 0;
    if (a != -1) {
      const MbRec &m = rec(a);
      na = m.type == kMbSkip ? 0 : (m.type == kMbPcm ? 16 : (chroma ? m.nzc[plane * 4 + (ya / 4) * 2 + xa / 4]
                                                                      : m.nz[(ya / 4) * 4 + xa / 4]));
    }
    if (b != -1) {
      const MbRec &m = rec(b);
      nbv = m.type == kMbSkip ? 0 : (m.type == kMbPcm ? 16 : (chroma ? m.nzc[plane * 4 + (yb / 4) * 2 + xb / 4]
                                                                       : m.nz[(yb / 4) * 4 + xb / 4]));
    }
    if (a != -1 && b != -1) return (na + nbv + 1) >> 1;
    if (a != -1) return na;
    if (b != -1) return nbv;
    return 0;
  }

  // residual_block_cavlc into sc->blk (raster, coefficient list index k ->
  // zig-zag position k + start_pos); returns TotalCoeff or -1
  VTS_HD int residual_block(int nC, int maxNum, int start_pos) {
    for (int i = 0; i < 16; ++i) sc->blk[i] = 0;
    int tc, t1;
    br.ensure(32);
    const uint32_t peek = static_cast<uint32_t>(br.win >> 32);
    if (nC >= 8) {
      const uint32_t v = peek >> 26;
      br.skip(6);
      if (v == 3) {
        tc = 0;
        t1 = 0;
      } else {
        tc = static_cast<int>(v >> 2) + 1;
        t1 = static_cast<int>(v & 3);
        if (t1 > tc) return -1;
      }
    } else {
      const int col = nC == -1 ? 3 : (nC < 2 ? 0 : (nC < 4 ? 1 : 2));
      const int lz = peek ? __builtin_clz(peek) : 32;
      if (col == 3 && lz >= 7) {  // 0000000: TotalCoeff 4, TrailingOnes 3
        br.skip(7);
        tc = 4;
        t1 = 3;
      } else {
        if (lz > 15) return -1;
        const uint32_t s3 = (peek << (lz + 1)) >> 29;
        const uint16_t e = kCtLut.v[col][lz][s3];
        if (!e) return -1;
        br.skip(e & 31);
        tc = (e >> 5) & 31;
        t1 = e >> 10;
      }
    }
    if (tc > maxNum) return -1;
    if (tc == 0) return 0;
    int level[16];
    int suffix_len = (tc > 10 && t1 < 3) ? 1 : 0;
    for (int i = 0; i < tc; ++i) {
      if (i < t1) {
        level[i] = br.bit() ? -1 : 1;
        continue;
      }
      br.ensure(32);
      const uint32_t p = static_cast<uint32_t>(br.win >> 32);
      if (!p) return -1;
      const int prefix = __builtin_clz(p);
      if (prefix > 15) return -1;  // level_prefix > 15: not in these profiles
      br.skip(prefix + 1);
      int code = (vts_min(15, prefix) << suffix_len);
      const int size = (prefix == 14 && suffix_len == 0) ? 4 : (prefix >= 15 ? prefix - 3 : suffix_len);
      if (size > 0) code += static_cast<int>(br.bits(size));
      if (prefix >= 15 && suffix_len == 0) code += 15;
      if (i == t1 && t1 < 3) code += 2;
      level[i] = (code % 2 == 0) ? (code + 2) >> 1 : (-code - 1) >> 1;
      if (suffix_len == 0) suffix_len = 1;
      const int mag = level[i] < 0 ? -level[i] : level[i];
      if (mag > (3 << (suffix_len - 1)) && suffix_len < 6) ++suffix_len;
    }
    int zeros = 0;
    if (tc < maxNum) {
      br.ensure(16);
      const uint32_t p = static_cast<uint32_t>(br.win >> 32);
      uint8_t e;
      if (maxNum == 4) e = kTzLut.dc[tc - 1][p >> 29];
      else e = kTzLut.v[tc - 1][p >> 23];
      if (!e) return -1;
      br.skip(e >> 4);
      zeros = e & 15;
    }
    int pos = zeros + tc - 1;  // list index of the highest coefficient
    for (int i = 0; i < tc; ++i) {
      if (pos < 0) return -1;
      sc->blk[kZz[pos + start_pos]] = static_cast<int16_t>(level[i]);
      if (i == tc - 1) break;
      int run = 0;
      if (zeros > 0) {
        br.ensure(16);
        const uint32_t p = static_cast<uint32_t>(br.win >> 32);
        if (zeros <= 6) {
          const uint8_t e = kRbLut.v[zeros - 1][p >> 29];
          if (!e) return -1;
          br.skip(e >> 4);
          run = e & 15;
        } else {
          const int lz = p ? __builtin_clz(p) : 32;
          if (lz < 3) {
            run = 7 - static_cast<int>(p >> 29);
            br.skip(3);
          } else {
            if (lz > 10) return -1;
            run = lz + 4;
            br.skip(lz + 1);
          }
        }
        if (run > zeros) return -1;
        zeros -= run;
      }
      pos -= run + 1;
    }
    return tc;
  }

  // store sc->blk as the next arena block; bit = kBlk* index
  VTS_HD VTS_INLINE bool store_block(uint32_t bit) {
    if (used >= s->arena_cap) return false;
    int16_t *dst = arena + 16 * static_cast<int64_t>(s->arena + used);
#if defined(__HIPCC__)
    uint4 *d4 = reinterpret_cast<uint4 *>(dst);
    const uint4 *s4 = reinterpret_cast<const uint4 *>(sc->blk);
    d4[0] = s4[0];
    d4[1] = s4[1];
#else
    for (int i = 0; i < 16; ++i) dst[i] = sc->blk[i];
#endif
    if (sc->cur.blocks == 0) sc->cur.coef = s->arena + used;
    sc->cur.blocks |= 1u << bit;
    ++used;
    return true;
  }

  // --- motion vector prediction (8.4.1.3)
  struct Mv {
    bool avail;
    int ref, x, y;
  };
  VTS_HD Mv nb_mv(int cur, int xN, int yN, uint32_t done) const {
    Mv r{false, -1, 0, 0};
    int xw, yw;
    const int n = nb_mb(cur, xN, yN, 16, &xw, &yw);
    if (n == -1) return r;
    const int b = (yw / 4) * 4 + xw / 4;
    if (n == -2 && !((done >> b) & 1u)) return r;
    r.avail = true;
    const MbRec &m = rec(n);
    if (m.type != kMbInter && m.type != kMbSkip) return r;
    r.ref = m.ref[(b >> 3) * 2 + ((b & 3) >> 1)];
    r.x = m.mv[b][0];
    r.y = m.mv[b][1];
    return r;
  }
  VTS_HD void mv_pred(int cur, int x0, int y0, int w, int h, int ref, uint32_t done, int *px, int *py) const {
    const Mv A = nb_mv(cur, x0 - 1, y0, done);
    Mv B = nb_mv(cur, x0, y0 - 1, done);
    Mv C = nb_mv(cur, x0 + w, y0 - 1, done);
    if (!C.avail) C = nb_mv(cur, x0 - 1, y0 - 1, done);
    if (w == 16 && h == 8) {
      if (y0 == 0 && B.ref == ref) { *px = B.x; *py = B.y; return; }
      if (y0 == 8 && A.ref == ref) { *px = A.x; *py = A.y; return; }
    } else if (w == 8 && h == 16) {
      if (x0 == 0 && A.ref == ref) { *px = A.x; *py = A.y; return; }
      if (x0 == 8 && C.ref == ref) { *px = C.x; *py = C.y; return; }
    }
    if (!B.avail && !C.avail && A.avail) {
      B = A;
      C = A;
    }
    const int match = (A.ref == ref) + (B.ref == ref) + (C.ref == ref);
    if (match == 1) {
      const Mv &m = A.ref == ref ? A : (B.ref == ref ? B : C);
      *px = m.x;
      *py = m.y;
    } else {
      *px = median3(A.x, B.x, C.x);
      *py = median3(A.y, B.y, C.y);
    }
  }

  VTS_HD VTS_INLINE void begin_mb(int addr) {
    MbRec &m = sc->cur;
    m.epoch = epoch;
    m.slice = slice_index;
    m.coef = 0;
    m.blocks = 0;
    m.type = 0;
    m.cbp = 0;
    m.modes = 0;
    for (int i = 0; i < 4; ++i) {
      m.ref[i] = -1;
      m.ref_slot[i] = -1;
    }
    for (int i = 0; i < 8; ++i) m.i4[i] = 0x22;  // DC
    for (int i = 0; i < 16; ++i) {
      m.nz[i] = 0;
      m.mv[i][0] = m.mv[i][1] = 0;
    }
    for (int i = 0; i < 8; ++i) m.nzc[i] = 0;
    (void)addr;
  }
  VTS_HD VTS_INLINE void end_mb(int addr) {
    // intra dependency level: 1 + the highest level among the intra-predicted
    // neighbours A, B, C, D the prediction may read (same slice), else 0; the
    // reconstruction runs the levels in order (h264_intra_full)
    uint16_t lv = kNoLevel;
    if (sc->cur.type == kMbI4x4 || sc->cur.type == kMbI16) {
      int l = 0, xw, yw;
      const int nbx[4] = {-1, 0, 16, -1}, nby[4] = {0, -1, -1, -1};
      for (int i = 0; i < 4; ++i) {
        const int n = nb_mb(addr, nbx[i], nby[i], 16, &xw, &yw);
        if (n >= 0 && ilvl[n] != kNoLevel) l = vts_max(l, ilvl[n] + 1);
      }
      lv = static_cast<uint16_t>(l);
    }
    ilvl[addr] = lv;
#if defined(__HIPCC__)
    uint4 *d = reinterpret_cast<uint4 *>(&recs[addr]);
    const uint4 *s4 = reinterpret_cast<const uint4 *>(&sc->cur);
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = s4[i];
#else
    recs[addr] = sc->cur;
#endif
  }

  VTS_HD VTS_INLINE void set_motion(int b, int ref, int mvx, int mvy) {
    sc->cur.mv[b][0] = static_cast<int16_t>(mvx);
    sc->cur.mv[b][1] = static_cast<int16_t>(mvy);
    const int p8 = (b >> 3) * 2 + ((b & 3) >> 1);
    sc->cur.ref[p8] = static_cast<int8_t>(ref);
    sc->cur.ref_slot[p8] = s->ref_slot[ref & 31];
  }

  VTS_HD void skip_mb(int addr, int qp) {
    begin_mb(addr);
    MbRec &m = sc->cur;
    m.type = kMbSkip;
    m.qp = static_cast<uint8_t>(qp);
    int xw, yw;
    const int a = nb_mb(addr, -1, 0, 16, &xw, &yw), b = nb_mb(addr, 0, -1, 16, &xw, &yw);
    const Mv A = nb_mv(addr, -1, 0, 0), B = nb_mv(addr, 0, -1, 0);
    int px = 0, py = 0;
    if (!(a == -1 || b == -1 || (A.ref == 0 && A.x == 0 && A.y == 0) || (B.ref == 0 && B.x == 0 && B.y == 0)))
      mv_pred(addr, 0, 0, 16, 16, 0, 0, &px, &py);
    if (s->ref_slot[0] < 0) err |= DEC_E_NO_REF;
    for (int i = 0; i < 16; ++i) set_motion(i, 0, px, py);
    end_mb(addr);
  }

  // macroblock_layer(); returns false to stop the slice
  VTS_HD bool mb_layer(int addr, int *qp) {
    begin_mb(addr);
    MbRec &m = sc->cur;
    const int mb_type = static_cast<int>(br.ue());
    const int itype = s->is_p ? mb_type - 5 : mb_type;  // < 0: inter
    if (mb_type > (s->is_p ? 30 : 25)) {
      err |= DEC_E_SYNTAX;
      return false;
    }
    if (itype == 25) {  // I_PCM: samples through the RBSP reader (EPBs dropped)
      m.type = kMbPcm;
      m.qp = static_cast<uint8_t>(*qp);
      br.align();
      for (int j = 0; j < 16; ++j) m.nz[j] = 16;
      for (int j = 0; j < 8; ++j) m.nzc[j] = 16;
      for (int k = 0; k < 12; ++k) {
        for (int i = 0; i < 16; ++i) {
          const uint32_t lo = br.bits(8), hi = br.bits(8);
          sc->blk[i] = static_cast<int16_t>(lo | (hi << 8));
        }
        if (!store_block(k)) {
          err |= DEC_E_SYNTAX;
          return false;
        }
      }
      m.blocks = 0;  // PCM samples: kPcmBlocks from coef, not a kBlk mask
      end_mb(addr);
      return true;
    }
    int cbp = 0;
    bool i16 = false;
    if (itype == 0) {  // I_NxN
      m.type = kMbI4x4;
      int prev[16], rem[16];
      for (int k = 0; k < 16; ++k) {
        prev[k] = static_cast<int>(br.bit());
        rem[k] = prev[k] ? 0 : static_cast<int>(br.bits(3));
      }
      for (int k = 0; k < 16; ++k) {
        const int bx = blk_x(k), by = blk_y(k);
        int xa, ya, xb, yb;
        const int a = nb_mb(addr, bx * 4 - 1, by * 4, 16, &xa, &ya);
        const int b = nb_mb(addr, bx * 4, by * 4 - 1, 16, &xb, &yb);
        int pred = 2;
        bool dcf = a == -1 || b == -1;
        if (!dcf && P->cip) {
          const int ta = rec(a).type, tb = rec(b).type;
          dcf = ta == kMbInter || ta == kMbSkip || tb == kMbInter || tb == kMbSkip;
        }
        if (!dcf) {
          const MbRec &ma = rec(a), &mbb = rec(b);
          const int ra = (ya / 4) * 4 + xa / 4, rb = (yb / 4) * 4 + xb / 4;
          const int ma_mode = ma.type == kMbI4x4 ? (ma.i4[ra >> 1] >> ((ra & 1) * 4)) & 15 : 2;
          const int mb_mode = mbb.type == kMbI4x4 ? (mbb.i4[rb >> 1] >> ((rb & 1) * 4)) & 15 : 2;
          pred = vts_min(ma_mode, mb_mode);
        }
        const int mode = prev[k] ? pred : (rem[k] < pred ? rem[k] : rem[k] + 1);
        const int r = by * 4 + bx;
        m.i4[r >> 1] = static_cast<uint8_t>((m.i4[r >> 1] & (0xf0 >> ((r & 1) * 4))) | (mode << ((r & 1) * 4)));
      }
      const uint32_t cm = br.ue();
      if (cm > 3) err |= DEC_E_SYNTAX;
      m.modes = static_cast<uint8_t>((cm & 3) << 2);
    } else if (itype > 0) {  // I_16x16
      m.type = kMbI16;
      i16 = true;
      const int pm = (itype - 1) % 4;
      cbp = ((((itype - 1) / 4) % 3) << 4) | (itype >= 13 ? 15 : 0);
      const uint32_t cm = br.ue();
      if (cm > 3) err |= DEC_E_SYNTAX;
      m.modes = static_cast<uint8_t>(pm | ((cm & 3) << 2));
    } else {  // inter
      m.type = kMbInter;
      const int nparts = mb_type == 0 ? 1 : (mb_type <= 2 ? 2 : 4);
      int sub[4] = {0, 0, 0, 0}, refs[4] = {0, 0, 0, 0};
      if (mb_type >= 3)
        for (int k = 0; k < 4; ++k) {
          sub[k] = static_cast<int>(br.ue());
          if (sub[k] > 3) {
            err |= DEC_E_SYNTAX;
            return false;
          }
        }
      const int nref = s->num_ref;
      if (mb_type != 4 && nref > 1)
        for (int k = 0; k < nparts; ++k) refs[k] = nref == 2 ? static_cast<int>(!br.bit()) : static_cast<int>(br.ue());
      for (int k = 0; k < nparts; ++k)
        if (refs[k] >= nref || s->ref_slot[refs[k] & 31] < 0) {
          err |= DEC_E_NO_REF;
          return false;
        }
      uint32_t done = 0;
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
        for (int q = 0; q < nsub; ++q) {
          int sx = x0, sy = y0;
          if (mb_type >= 3) {
            if (sub[k] == 1) sy += 4 * q;
            else if (sub[k] == 2) sx += 4 * q;
            else if (sub[k] == 3) { sx += 4 * (q & 1); sy += 4 * (q >> 1); }
          }
          const int dx = br.se(), dy = br.se();
          int px, py;
          mv_pred(addr, sx, sy, pw, ph, refs[k], done, &px, &py);
          const int vx = px + dx, vy = py + dy;
          if (vx < -32768 || vx > 32767 || vy < -32768 || vy > 32767) {
            err |= DEC_E_SYNTAX;
            return false;
          }
          for (int yy = sy / 4; yy < (sy + ph) / 4; ++yy)
            for (int xx = sx / 4; xx < (sx + pw) / 4; ++xx) {
              set_motion(yy * 4 + xx, refs[k], vx, vy);
              done |= 1u << (yy * 4 + xx);
            }
        }
      }
    }
    if (!i16) {
      const uint32_t code = br.ue();
      if (code > 47) {
        err |= DEC_E_SYNTAX;
        return false;
      }
      cbp = m.type == kMbI4x4 ? kCbpI[code] : kCbpP[code];
    }
    m.cbp = static_cast<uint8_t>(cbp);
    if (cbp || i16) {
      const int dq = br.se();
      if (dq < -26 || dq > 25) {
        err |= DEC_E_SYNTAX;
        return false;
      }
      *qp = (*qp + dq + 52) % 52;
    }
    m.qp = static_cast<uint8_t>(*qp);
    // ---- residual (7.3.5.3)
    if (i16) {
      const int tc = residual_block(nc_of(addr, 0, 0, false, 0), 16, 0);
      VTS_PARSE_TRACE("  i16 dc tc %d bits %d\n", tc, br.consumed());
      if (tc < 0) { err |= DEC_E_SYNTAX; return false; }
      if (tc > 0 && !store_block(kBlkI16Dc)) { err |= DEC_E_SYNTAX; return false; }
    }
    for (int k = 0; k < 16; ++k) {
      if (!((cbp >> (k >> 2)) & 1)) continue;
      const int bx = blk_x(k), by = blk_y(k);
      const int n = nc_of(addr, bx, by, false, 0);
      const int tc = i16 ? residual_block(n, 15, 1) : residual_block(n, 16, 0);
      VTS_PARSE_TRACE("  luma blk %d nC %d tc %d bits %d\n", k, n, tc, br.consumed());
      if (tc < 0) { err |= DEC_E_SYNTAX; return false; }
      m.nz[by * 4 + bx] = static_cast<uint8_t>(tc);
      if (tc > 0 && !store_block(kBlkLuma0 + k)) { err |= DEC_E_SYNTAX; return false; }
    }
    if (cbp >> 4) {
      for (int pl = 0; pl < 2; ++pl) {
        const int tc = residual_block(-1, 4, 0);
        VTS_PARSE_TRACE("  chroma dc %d tc %d bits %d\n", pl, tc, br.consumed());
        if (tc < 0) { err |= DEC_E_SYNTAX; return false; }
        if (tc > 0) {
          // chroma DC levels in list order (not zig-zag): undo the scan
          int16_t lv[4];
          for (int i = 0; i < 4; ++i) lv[i] = sc->blk[kZz[i]];
          for (int i = 0; i < 16; ++i) sc->blk[i] = i < 4 ? lv[i] : 0;
          if (!store_block(kBlkChromaDc0 + pl)) { err |= DEC_E_SYNTAX; return false; }
        }
      }
    }
    if ((cbp >> 4) & 2) {
      for (int pl = 0; pl < 2; ++pl)
        for (int k = 0; k < 4; ++k) {
          const int n = nc_of(addr, k & 1, k >> 1, true, pl);
          const int tc = residual_block(n, 15, 1);
          VTS_PARSE_TRACE("  chroma ac %d %d nC %d tc %d bits %d\n", pl, k, n, tc, br.consumed());
          if (tc < 0) { err |= DEC_E_SYNTAX; return false; }
          m.nzc[pl * 4 + k] = static_cast<uint8_t>(tc);
          if (tc > 0 && !store_block(kBlkChromaAc0 + 4 * pl + k)) { err |= DEC_E_SYNTAX; return false; }
        }
    }
    if (br.err || br.overrun()) {
      err |= DEC_E_SYNTAX;
      return false;
    }
    end_mb(addr);
    return true;
  }
};

// Parse slice `s` (window slice index si) into recs (the frame's records) and
// the arena.  Returns DEC_E_* bits.
VTS_HD inline uint32_t parse_slice_full(const uint8_t *es, const FullSlice &s, uint32_t si, const FullParams &P,
                                        MbRec *frame_recs, uint16_t *frame_ilvl, int16_t *arena, uint32_t epoch,
                                        FullScratch *sc) {
  const uint8_t *nal = es + s.nal_offset;
  Parser p;
  p.s = &s;
  p.P = &P;
  p.recs = frame_recs;
  p.ilvl = frame_ilvl;
  p.arena = arena;
  p.sc = sc;
  p.used = 0;
  p.slice_index = si;
  p.epoch = epoch;
  p.mbw = P.mb_width;
  p.first_mb = s.first_mb;
  p.err = 0;
  const int nmb = P.mb_width * P.mb_height;
  int32_t last = s.nal_size - 1;
  while (last > 0 && nal[last] == 0) --last;
  if (last <= 0) return DEC_E_SYNTAX;
  const int tz = __builtin_ctz(static_cast<uint32_t>(nal[last]));
  const int32_t stop_byte = last - 1;
  const int64_t stop_bit = int64_t(stop_byte) * 8 + (7 - tz);
  p.br.init(nal + 1, s.nal_offset + 1, s.nal_size - 1, sc->cache);
  p.br.reset_at(s.data_byte, s.data_bit & ~7);
  p.br.ensure(8);
  p.br.skip(s.data_bit & 7);
  int addr = s.first_mb, qp = s.qp;
  bool more = true;
  while (more) {
    if (addr >= nmb) {
      p.err |= DEC_E_SYNTAX;
      break;
    }
    if (s.is_p) {
      const int run = static_cast<int>(p.br.ue());
      if (p.br.err || addr + run > nmb) {
        p.err |= DEC_E_SYNTAX;
        break;
      }
      for (int i = 0; i < run; ++i, ++addr) p.skip_mb(addr, qp);
      if (run > 0) {
        more = p.br.more(stop_byte, stop_bit);
        if (!more) break;
      }
      if (addr >= nmb) {
        p.err |= DEC_E_SYNTAX;
        break;
      }
    }
    const bool ok = p.mb_layer(addr, &qp);
    VTS_PARSE_TRACE("mb %d type %d cbp %d qp %d bits %d err %u\n", addr, p.sc->cur.type, p.sc->cur.cbp, qp,
                    p.br.consumed(), p.err);
    if (!ok) break;
    ++addr;
    more = p.br.more(stop_byte, stop_bit);
  }
  if (!p.err && (p.br.err || p.br.overrun() || p.br.consumed() != stop_bit - 8ll * p.br.epb)) p.err |= DEC_E_SYNTAX;
  return p.err;
}

}  // namespace full
}  // namespace vts
