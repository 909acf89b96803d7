// intra_lanes.h — lane-parallel intra reconstruction of one macroblock
// (h264_intra_v2 in decode_full.hip), written once for the device, where the
// macroblock's 32 lanes are half a wave, and for the CPU harness
// (tests/native/full_host.cpp), where 32 host threads play the lanes.  The
// lane primitives come from the Lanes policy: t (the lane, 0..31), sync()
// (the lanes' LDS writes visible to each other), red16(v) (sum over the
// lane's aligned group of 16) and bcast(v, l) (lane l's v).  DESIGN.md §5b.
//
// Work per macroblock (the kernel's comment has the why):
//  * residuals first, in two passes through the tile (rows, then columns);
//  * the neighbourhood: availability (6.4.11.1), border samples from the LDS
//    line buffers (neighbours this launch reconstructed) or from HBM;
//  * Intra_16x16 (8 samples per lane), Intra_8x8 (per 8x8 block: filtered
//    reference samples, derived arrays, 2 samples per lane), Intra_4x4 (10
//    steps of one or two 4x4 blocks, 16 lanes each), chroma (4 per lane);
//  * the macroblock to HBM as whole rows, its bottom row and right column to
//    the line buffers.
#pragma once
#include <cstdint>
#include <cstring>

#include "h264_cabac_tables.h"
#include "h264_full.h"
#include "recon_full.h"

#if defined(__HIPCC__)
#define VTS_I2 __host__ __device__ inline __attribute__((always_inline))
#else
#define VTS_I2 inline __attribute__((always_inline))
#endif

namespace vts {
namespace i2 {

struct I2V2 {
  uint32_t x, y;
};
struct I2V4 {
  uint32_t x, y, z, w;
};
// wide loads / stores (dwordx2 / x4 on the device; memcpy on the host)
VTS_I2 I2V2 i2_ld2(const void *p) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint2 u = *reinterpret_cast<const uint2 *>(p);
  return I2V2{u.x, u.y};
#else
  I2V2 v;
  std::memcpy(&v, p, sizeof v);
  return v;
#endif
}
VTS_I2 I2V4 i2_ld4(const void *p) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint4 u = *reinterpret_cast<const uint4 *>(p);
  return I2V4{u.x, u.y, u.z, u.w};
#else
  I2V4 v;
  std::memcpy(&v, p, sizeof v);
  return v;
#endif
}
VTS_I2 void i2_st4(void *p, const I2V4 &v) {
#if defined(__HIP_DEVICE_COMPILE__)
  *reinterpret_cast<uint4 *>(p) = make_uint4(v.x, v.y, v.z, v.w);
#else
  std::memcpy(p, &v, sizeof v);
#endif
}
VTS_I2 int i2_min(int a, int b) { return a < b ? a : b; }
VTS_I2 int i2_max(int a, int b) { return a > b ? a : b; }
VTS_I2 int64_t i2_max(int64_t a, int64_t b) { return a > b ? a : b; }
VTS_I2 int i2_c255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
VTS_I2 uint32_t i2_pack4(int a, int b, int c, int d) {
  return static_cast<uint32_t>(a) | (static_cast<uint32_t>(b) << 8) | (static_cast<uint32_t>(c) << 16) |
         (static_cast<uint32_t>(d) << 24);
}
// luma4x4BlkIdx of raster 4x4 block b
VTS_I2 int i2_blkidx(int b) { return ((b >> 3) << 3) | (((b & 3) >> 1) << 2) | (((b >> 2) & 1) << 1) | (b & 1); }
// arena block of stored-block bit `bit` of a macroblock, -1 if absent
VTS_I2 int64_t i2_stored(uint32_t blocks, uint32_t coef, uint32_t bit) {
  if (!((blocks >> bit) & 1u)) return -1;
  return static_cast<int64_t>(coef) + __builtin_popcount(blocks & ((1u << bit) - 1u));
}
VTS_I2 void i2_coefs(const int16_t *arena, int64_t blk, int *cf) {
  if (blk < 0) {
    for (int i = 0; i < 16; ++i) cf[i] = 0;
    return;
  }
  const I2V4 u0 = i2_ld4(arena + 16 * blk), u1 = i2_ld4(arena + 16 * blk + 8);
  const uint32_t w[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
  for (int i = 0; i < 8; ++i) {
    cf[2 * i] = static_cast<int16_t>(w[i] & 0xffff);
    cf[2 * i + 1] = static_cast<int16_t>(w[i] >> 16);
  }
}
// 8.5.12.1 chroma DC of chroma block ck: 2x2 Hadamard of the plane's DC levels, scaled
VTS_I2 int i2_chroma_dc(const int16_t *arena, uint32_t blocks, uint32_t coef, int pl, int ck, int qpc,
                        const int32_t *ls) {
  const int64_t blk = i2_stored(blocks, coef, kBlkChromaDc0 + pl);
  if (blk < 0) return 0;
  const I2V2 u = i2_ld2(arena + 16 * blk);
  const int c0 = static_cast<int16_t>(u.x & 0xffff), c1 = static_cast<int16_t>(u.x >> 16);
  const int c2 = static_cast<int16_t>(u.y & 0xffff), c3 = static_cast<int16_t>(u.y >> 16);
  const int f = ck == 0 ? c0 + c1 + c2 + c3 : ck == 1 ? c0 - c1 + c2 - c3 : ck == 2 ? c0 + c1 - c2 - c3 : c0 - c1 - c2 + c3;
  return ((f * ls[0]) << (qpc / 6)) >> 5;
}
// Every Intra_4x4 mode (8.3.1.2.1-9) reads each predicted sample as one entry
// of the block's array [E (0..14), F (16 + k), A (32 + k), DC (47)]: its
// offset for (mode, x, y)
VTS_I2 int i2_intra4_off(int mode, int x, int y) {
  switch (mode) {
    case 0: return 1 + 5 + x;
    case 1: return 1 + 3 - y;
    case 2: return 47;
    case 3: return 16 + 6 + x + y;
    case 4: return 16 + 4 + x - y;
    case 5: {
      const int z = 2 * x - y;
      if (z >= 0) return ((z & 1) ? 16 : 32) + 4 + x - (y >> 1);
      return z == -1 ? 16 + 4 : 16 + 5 - y;
    }
    case 6: {
      const int z = 2 * y - x;
      if (z >= 0) return (z & 1) ? 16 + 4 - y + (x >> 1) : 32 + 3 - y + (x >> 1);
      return z == -1 ? 16 + 4 : 16 + 3 + x;
    }
    case 7: return (y & 1) ? 16 + 6 + x + (y >> 1) : 32 + 5 + x + (y >> 1);
    default: {
      const int z = x + 2 * y;
      if (z > 5) return 1;
      if (z == 5) return 16;
      return ((z & 1) ? 16 : 32) + 2 - y - (x >> 1);
    }
  }
}
// the same for Intra_8x8 (8.3.2.2.2-10) into [E (0..26), F (32 + k), A (64 + k), DC (88)]
VTS_I2 int i2_intra8_off(int mode, int x, int y) {
  switch (mode) {
    case 0: return 1 + 9 + x;
    case 1: return 1 + 7 - y;
    case 2: return 88;
    case 3: return 32 + 10 + x + y;
    case 4: return 32 + 8 + x - y;
    case 5: {
      const int z = 2 * x - y;
      if (z >= 0) return ((z & 1) ? 32 : 64) + 8 + x - (y >> 1);
      return z == -1 ? 32 + 8 : 32 + 9 + 2 * x - y;
    }
    case 6: {
      const int z = 2 * y - x;
      if (z >= 0) return (z & 1) ? 32 + 8 - y + (x >> 1) : 64 + 7 - y + (x >> 1);
      return z == -1 ? 32 + 8 : 32 + 7 + x - 2 * y;
    }
    case 7: return (y & 1) ? 32 + 10 + x + (y >> 1) : 64 + 9 + x + (y >> 1);
    default: {
      const int z = x + 2 * y;
      if (z > 13) return 1;
      if (z == 13) return 32;
      return ((z & 1) ? 32 : 64) + 6 - y - (x >> 1);
    }
  }
}

// MbRec header words (the first 32 bytes)
struct I2Hdr {
  uint32_t epoch, slice, coef, blocks;
  int type, qp, cbp, modes;
};
VTS_I2 I2Hdr i2_hdr(const MbRec *m) {
  const I2V4 a = i2_ld4(m), b = i2_ld4(reinterpret_cast<const uint8_t *>(m) + 16);
  I2Hdr h;
  h.epoch = a.x;
  h.slice = a.y;
  h.coef = a.z;
  h.blocks = a.w;
  h.type = static_cast<int>(b.x & 255);
  h.qp = static_cast<int>((b.x >> 8) & 255);
  h.cbp = static_cast<int>((b.x >> 16) & 255);
  h.modes = static_cast<int>(b.x >> 24);
  return h;
}

// what one picture's intra reconstruction reads
struct I2Ctx {
  const MbRec *recs;    // the picture's macroblock records
  const int16_t *arena; // coefficient arena
  uint8_t *Y;           // the picture's luma plane; chroma (NV12) at Y + uv_off
  int64_t uv_off;
  int pitch, mbw, mbh;
  uint32_t epoch;
  int cip, cqp_off, cqp_off2, scaled;
  const ScaleTab *sct;  // LevelScale4x4 / 8x8 (8.5.9)
};
struct I2NoProf {
  VTS_I2 void mark(int) {}
};

// 8.5.13's 1-D 8-point inverse transform
VTS_I2 void idct8_1d(const int (&v)[8], int (&o)[8]) {
  const int a0 = v[0] + v[4], a4 = v[0] - v[4], a2 = (v[2] >> 1) - v[6], a6 = v[2] + (v[6] >> 1);
  const int b0 = a0 + a6, b2 = a4 + a2, b4 = a4 - a2, b6 = a0 - a6;
  const int a1 = -v[3] + v[5] - v[7] - (v[7] >> 1), a3 = v[1] + v[7] - v[3] - (v[3] >> 1);
  const int a5 = -v[1] + v[7] + v[5] + (v[5] >> 1), a7 = v[3] + v[5] + v[1] + (v[1] >> 1);
  const int b1 = a1 + (a7 >> 2), b7 = a7 - (a1 >> 2), b3 = a3 + (a5 >> 2), b5 = (a3 >> 2) - a5;
  o[0] = b0 + b7;
  o[1] = b2 + b5;
  o[2] = b4 + b3;
  o[3] = b6 + b1;
  o[4] = b6 - b1;
  o[5] = b4 - b3;
  o[6] = b2 - b5;
  o[7] = b0 - b7;
}
struct alignas(16) I2Tile {
  int32_t lres[16][16];  // luma residual, raster (row-pass intermediates first)
  int32_t cres[2][8][8]; // chroma residual per plane
  int32_t dc16[16];      // Intra_16x16: each block's scaled DC
  uint8_t y[17][28];     // luma rows -1..15 (index + 1) x cols -4..23 (index + 4)
  uint8_t c[2][9][12];   // per plane: chroma rows -1..7 (index + 1) x cols -1..7 (index + 1)
  uint8_t e4[2][16];     // Intra_4x4: per block slot E[0..14], DC at 15
  uint8_t p8[96];        // Intra_8x8: E at 0..26, F(k) at 32 + k, A(k) at 64 + k, DC at 88
  int32_t meta[8];       // part 1 -> part 2: macroblock, type | modes << 8, A..D, Intra_NxN mode words
};
// Intra_4x4 block steps: the raster blocks of step s (bx + 2 by = s), -1 none
VTS_I2 int i4_step_blk(int s, int slot) {
  // step:   0  1  2    3    4    5    6     7     8   9
  // slot 0: 0  1  2    3    6    7    10    11    14  15
  // slot 1: -  -  4    5    8    9    12    13    -   -
  const uint64_t s0 = 0xFEBA763210ull;  // nibble s
  const uint64_t s1 = 0x00DC985400ull;
  if (slot == 0) return static_cast<int>((s0 >> (4 * s)) & 15);
  return (s >= 2 && s <= 7) ? static_cast<int>((s1 >> (4 * s)) & 15) : -1;
}

// LDS line buffers, tagged with the macroblock that wrote them: a macroblock's
// bottom row in its column's entry, its right column in its row's entry.
// Levels follow the real dependencies (slice boundaries, inter neighbours),
// not a fixed wavefront, so an entry may hold another macroblock than the
// neighbour: a reader checks the tag and takes HBM instead (written a level
// earlier: visible after the level barrier).
struct alignas(16) I2Line {
  int32_t tag;    // the writer's row (column entry) / column (row entry); -2 none
  int32_t claim;  // the largest writer of the entry so far: only it writes (a round may hold
                  // several macroblocks of one column or row: isolated intra ones, level 0)
  int32_t _p[2];
  uint8_t y[16];  // luma: the bottom row (column entry) / the right column (row entry)
  uint8_t c[16];  // chroma: interleaved bottom row / right column (Cb, Cr of rows 0..7)
};

// What part 1 reads from HBM that no reconstruction of this launch changes:
// the macroblock's header and Intra_NxN mode words, its neighbours' headers,
// and the border samples as HBM holds them (final for inter / I_PCM
// neighbours; a neighbour this launch reconstructs comes from the line entries,
// or is re-read in part 1 when its entry was overwritten).  The kernel loads
// the next macroblock's at the end of part 2, so the loads cross the barrier
// in flight and part 1 waits only for the coefficients.
struct I2Pre {
  I2Hdr h;
  uint32_t i4w0, i4w1;
  I2V2 hA, hB, hC, hD;
  uint32_t tA, tB, tC, tD;
  uint32_t gTop, gCl, gCt;
  uint32_t gLeft;
};
// lane t: row -1 dword t (t < 7, cols -4 + 4t), col -1 of row t - 8 (8..23),
// chroma col -1 dword of row t - 24 (24..31), chroma row -1 dword t (t < 5)
VTS_I2 const uint8_t *i2_top_at(const I2Ctx &a, int mb, int t) {
  const int mx = mb % a.mbw, my = mb / a.mbw;
  const int64_t yrow0 = static_cast<int64_t>(my * 16) * a.pitch + mx * 16;
  const int64_t up = my > 0 ? yrow0 - a.pitch : yrow0;
  return a.Y + i2_max(up - 4 + 4 * i2_min(t, 6), static_cast<int64_t>(0));
}
VTS_I2 const uint8_t *i2_left_at(const I2Ctx &a, int mb, int t) {
  const int mx = mb % a.mbw, my = mb / a.mbw;
  const int64_t yrow0 = static_cast<int64_t>(my * 16) * a.pitch + mx * 16;
  return a.Y + i2_max(yrow0 + static_cast<int64_t>(i2_min(i2_max(t - 8, 0), 15)) * a.pitch - 1, static_cast<int64_t>(0));
}
VTS_I2 const uint8_t *i2_cleft_at(const I2Ctx &a, int mb, int t) {
  const int mx = mb % a.mbw, my = mb / a.mbw;
  const int64_t crow0 = static_cast<int64_t>(my * 8) * a.pitch + mx * 16;
  return a.Y + a.uv_off + crow0 + static_cast<int64_t>(i2_min(i2_max(t - 24, 0), 7)) * a.pitch - 4;
}
VTS_I2 const uint8_t *i2_ctop_at(const I2Ctx &a, int mb, int t) {
  const int mx = mb % a.mbw, my = mb / a.mbw;
  const int64_t crow0 = static_cast<int64_t>(my * 8) * a.pitch + mx * 16;
  return a.Y + a.uv_off + crow0 - a.pitch - 4 + 4 * i2_min(t, 4);
}
VTS_I2 I2Pre i2_prefetch(const I2Ctx &a, int mb, int t) {
  const int mbw = a.mbw, mx = mb % mbw, my = mb / mbw;
  const MbRec *frecs = a.recs, *rec = a.recs + mb;
  I2Pre p;
  p.h = i2_hdr(rec);
  p.i4w0 = reinterpret_cast<const uint32_t *>(rec)[8];
  p.i4w1 = reinterpret_cast<const uint32_t *>(rec)[9];
  const int nA = mx > 0 ? mb - 1 : mb, nB = my > 0 ? mb - mbw : mb;
  const int nC = my > 0 && mx < mbw - 1 ? mb - mbw + 1 : mb, nD = mx > 0 && my > 0 ? mb - mbw - 1 : mb;
  p.hA = i2_ld2(frecs + nA);
  p.hB = i2_ld2(frecs + nB);
  p.hC = i2_ld2(frecs + nC);
  p.hD = i2_ld2(frecs + nD);
  p.tA = reinterpret_cast<const uint32_t *>(frecs + nA)[4];
  p.tB = reinterpret_cast<const uint32_t *>(frecs + nB)[4];
  p.tC = reinterpret_cast<const uint32_t *>(frecs + nC)[4];
  p.tD = reinterpret_cast<const uint32_t *>(frecs + nD)[4];
  p.gTop = *reinterpret_cast<const uint32_t *>(i2_top_at(a, mb, t));
  p.gLeft = *i2_left_at(a, mb, t);
  p.gCl = *reinterpret_cast<const uint32_t *>(i2_cleft_at(a, mb, t));
  p.gCt = *reinterpret_cast<const uint32_t *>(i2_ctop_at(a, mb, t));
  return p;
}

// Part 1, reads only: the macroblock's neighbourhood and its residuals into
// its tile.  Part 2 (intra2_finish) predicts, reconstructs and writes.  The
// kernel runs part 1 of a round of macroblocks, a workgroup barrier, part 2,
// a barrier: no line-buffer entry is read while another lane writes it.
template <class Lanes, class Prof>
VTS_HD VTS_INLINE void intra2_prepare(const I2Ctx &a, int mb, const I2Pre &pre, const Lanes &L, I2Tile &T,
                                      const I2Line *lcol, const I2Line *lrow, Prof &rp_) {
  const int t = L.t;
  const int mbw = a.mbw;
  const I2Hdr h = pre.h;
  const int mx = mb % mbw, my = mb / mbw;
  const int qp = h.qp;
  const bool i16 = h.type == kMbI16, t8 = !i16 && (h.modes & kModeT8);
  const uint32_t i4w0 = pre.i4w0, i4w1 = pre.i4w1;
  const I2V2 hA = pre.hA, hB = pre.hB, hC = pre.hC, hD = pre.hD;
  const uint32_t tA = pre.tA, tB = pre.tB, tC = pre.tC, tD = pre.tD;
  // ---- neighbourhood: availability (6.4.11.1, constrained_intra_pred), then
  // the border samples from the line buffers (neighbours this launch
  // reconstructed) or HBM (the others); unavailable samples read as 0
  auto nb_ok = [&](bool exists, I2V2 u, uint32_t ty) -> bool {
    if (!exists || u.x != a.epoch || u.y != h.slice) return false;
    if (a.cip && ((ty & 255) == kMbInter || (ty & 255) == kMbSkip)) return false;
    return true;
  };
  auto mine = [](uint32_t ty) { return (ty & 255) == kMbI4x4 || (ty & 255) == kMbI16; };
  const bool A = nb_ok(mx > 0, hA, tA), B = nb_ok(my > 0, hB, tB);
  const bool C = nb_ok(my > 0 && mx < mbw - 1, hC, tC), D = nb_ok(mx > 0 && my > 0, hD, tD);
  // the tagged line entries this macroblock's neighbours would have written
  const I2Line &lB = lcol[mx], &lC = lcol[i2_min(mx + 1, mbw - 1)], &lD = lcol[i2_max(mx - 1, 0)];
  const I2Line &lA = lrow[my];
  const bool mB = B && mine(tB) && lB.tag == my - 1, mC = C && mine(tC) && lC.tag == my - 1;
  const bool mD = D && mine(tD) && lD.tag == my - 1, mA = A && mine(tA) && lA.tag == mx - 1;
  // a neighbour this launch reconstructed whose entry another macroblock took
  // over: its samples from HBM now (the prefetched ones predate them)
  const bool sD = D && mine(tD) && !mD, sB = B && mine(tB) && !mB, sC = C && mine(tC) && !mC, sA = A && mine(tA) && !mA;
  const uint32_t gTop = (t == 0 ? sD : (t < 5 ? sB : sC)) ? *reinterpret_cast<const uint32_t *>(i2_top_at(a, mb, t)) : pre.gTop;
  const uint8_t gLeft = sA ? *i2_left_at(a, mb, t) : static_cast<uint8_t>(pre.gLeft);
  const uint32_t gCl = sA ? *reinterpret_cast<const uint32_t *>(i2_cleft_at(a, mb, t)) : pre.gCl;
  const uint32_t gCt = (t == 0 ? sD : sB) ? *reinterpret_cast<const uint32_t *>(i2_ctop_at(a, mb, t)) : pre.gCt;
  if (t < 7) {  // row -1 dword t: cols -4 + 4t .. -1 + 4t (D | B | C)
    const bool ok = t == 0 ? D : (t < 5 ? B : C);
    uint32_t v = gTop;
    if (t == 0 && mD) v = *reinterpret_cast<const uint32_t *>(&lD.y[12]);
    if (t >= 1 && t < 5 && mB) v = *reinterpret_cast<const uint32_t *>(&lB.y[4 * (t - 1)]);
    if (t >= 5 && mC) v = *reinterpret_cast<const uint32_t *>(&lC.y[4 * (t - 5)]);
    *reinterpret_cast<uint32_t *>(&T.y[0][4 * t]) = ok ? v : 0u;
  }
  if (t >= 8 && t < 24) {
    const int r = t - 8;
    T.y[1 + r][3] = A ? (mA ? lA.y[r] : gLeft) : 0;
  }
  if (t >= 24) {  // chroma col -1, row t - 24: bytes 2, 3 of the dword (Cb, Cr of col -1)
    const int r = t - 24;
    const uint32_t v = mA ? (static_cast<uint32_t>(lA.c[2 * r]) << 16) | (static_cast<uint32_t>(lA.c[2 * r + 1]) << 24) : gCl;
    T.c[0][1 + r][0] = A ? (v >> 16) & 255 : 0;
    T.c[1][1 + r][0] = A ? v >> 24 : 0;
  }
  if (t < 5) {  // chroma row -1 dword t: interleaved bytes -4 + 4t (t = 0: D's col -1, else B)
    const bool ok = t == 0 ? D : B;
    uint32_t v0 = gCt;
    if (t == 0 && mD) v0 = *reinterpret_cast<const uint32_t *>(&lD.c[12]);
    if (t >= 1 && mB) v0 = *reinterpret_cast<const uint32_t *>(&lB.c[4 * (t - 1)]);
    const uint32_t v = ok ? v0 : 0u;
    if (t == 0) {
      T.c[0][0][0] = (v >> 16) & 255;
      T.c[1][0][0] = v >> 24;
    } else {
      const int c0 = 2 * (t - 1);
      T.c[0][0][1 + c0] = v & 255;
      T.c[1][0][1 + c0] = (v >> 8) & 255;
      T.c[0][0][2 + c0] = (v >> 16) & 255;
      T.c[1][0][2 + c0] = v >> 24;
    }
  }
  // ---- residuals (8.5.12 / 8.5.13), in two passes through the tile so no lane
  // holds a whole block: pass 1 scales and transforms rows (luma: 4x4 rows two
  // per lane, or 8x8 rows one per lane; chroma: one 4x4 row per lane), pass 2
  // the columns, in place (int32: a stream outside the standard's range still
  // decodes exactly like the oracle)
  {
    const int32_t *ls4 = a.sct->ls4[0][qp % 6];
    if (i16 && t < 16) {  // 8.5.10: block t's entry of the Hadamard-transformed DC levels, scaled
      const int bx = t & 3, by = t >> 2;
      int dcl[16];
      i2_coefs(a.arena, i2_stored(h.blocks, h.coef, kBlkI16Dc), dcl);
      int f = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // row transform of DC row k at column bx; the column signs for row by
        const int a0 = dcl[k * 4], a1 = dcl[k * 4 + 1], a2 = dcl[k * 4 + 2], a3 = dcl[k * 4 + 3];
        const int rk = bx == 0 ? a0 + a1 + a2 + a3 : (bx == 1 ? a0 + a1 - a2 - a3 : (bx == 2 ? a0 - a1 - a2 + a3 : a0 - a1 + a2 - a3));
        const bool pos = k == 0 || (k == 1 ? by <= 1 : (k == 2 ? (by == 0 || by == 3) : (by == 0 || by == 2)));
        f += pos ? rk : -rk;
      }
      const int ls = ls4[0], sh = qp / 6;
      T.dc16[t] = qp >= 36 ? (f * ls) << (sh - 6) : (f * ls + (1 << (5 - sh))) >> (6 - sh);
    }
    L.sync();
    if (t8) {
      const int b8 = t >> 3, i = t & 7;
      const int64_t lb = i2_stored(h.blocks, h.coef, kBlkLuma0 + 4 * b8);
      const int32_t *ls8 = a.scaled ? a.sct->ls8[0][qp % 6] : nullptr;
      int v[8];
      if (lb >= 0) {
        const I2V4 u = i2_ld4(a.arena + 16 * lb + 8 * i);
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
        const int sh = qp / 6;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int c = static_cast<int16_t>((w[j >> 1] >> ((j & 1) * 16)) & 0xffff);
          const int ls = ls8 ? ls8[i * 8 + j] : 16 * full::kNorm8[qp % 6][vts_norm8_class(i, j)];
          v[j] = qp >= 36 ? (c * ls) << (sh - 6) : (c * ls + (1 << (5 - sh))) >> (6 - sh);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0;
      }
      int o[8];
      idct8_1d(v, o);
      int32_t *dst = &T.lres[(b8 >> 1) * 8 + i][(b8 & 1) * 8];
#pragma unroll
      for (int j = 0; j < 8; ++j) dst[j] = o[j];
    } else {
      const int b = t >> 1, bx = b & 3, by = b >> 2;
      const int64_t lb = i2_stored(h.blocks, h.coef, kBlkLuma0 + i2_blkidx(b));
      const int sh = qp / 6;
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        const int i = (t & 1) * 2 + rr;  // row of the block
        int c[4] = {0, 0, 0, 0};
        if (lb >= 0) {
          const I2V2 u = i2_ld2(a.arena + 16 * lb + 4 * i);
          c[0] = static_cast<int16_t>(u.x & 0xffff);
          c[1] = static_cast<int16_t>(u.x >> 16);
          c[2] = static_cast<int16_t>(u.y & 0xffff);
          c[3] = static_cast<int16_t>(u.y >> 16);
        }
        int d[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          d[j] = qp >= 24 ? (c[j] * ls4[i * 4 + j]) << (sh - 4) : (c[j] * ls4[i * 4 + j] + (1 << (3 - sh))) >> (4 - sh);
        if (i16 && i == 0) d[0] = T.dc16[b];
        const int e0 = d[0] + d[2], e1 = d[0] - d[2], e2 = (d[1] >> 1) - d[3], e3 = d[1] + (d[3] >> 1);
        int32_t *dst = &T.lres[by * 4 + i][bx * 4];
        dst[0] = e0 + e3;
        dst[1] = e1 + e2;
        dst[2] = e1 - e2;
        dst[3] = e0 - e3;
      }
    }
    {  // chroma row: plane t >> 4, block (t >> 2) & 3, row t & 3
      const int pl = t >> 4, ck = (t >> 2) & 3, i = t & 3;
      const int qpc = full::qpc_of(qp, pl ? a.cqp_off2 : a.cqp_off);
      const int32_t *lsc = a.sct->ls4[1 + pl][qpc % 6];
      const int64_t cb = i2_stored(h.blocks, h.coef, kBlkChromaAc0 + 4 * pl + ck);
      const int sh = qpc / 6;
      int c[4] = {0, 0, 0, 0};
      if (cb >= 0) {
        const I2V2 u = i2_ld2(a.arena + 16 * cb + 4 * i);
        c[0] = static_cast<int16_t>(u.x & 0xffff);
        c[1] = static_cast<int16_t>(u.x >> 16);
        c[2] = static_cast<int16_t>(u.y & 0xffff);
        c[3] = static_cast<int16_t>(u.y >> 16);
      }
      int d[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        d[j] = qpc >= 24 ? (c[j] * lsc[i * 4 + j]) << (sh - 4) : (c[j] * lsc[i * 4 + j] + (1 << (3 - sh))) >> (4 - sh);
      if (i == 0) d[0] = i2_chroma_dc(a.arena, h.blocks, h.coef, pl, ck, qpc, lsc);
      const int e0 = d[0] + d[2], e1 = d[0] - d[2], e2 = (d[1] >> 1) - d[3], e3 = d[1] + (d[3] >> 1);
      int32_t *dst = &T.cres[pl][(ck >> 1) * 4 + i][(ck & 1) * 4];
      dst[0] = e0 + e3;
      dst[1] = e1 + e2;
      dst[2] = e1 - e2;
      dst[3] = e0 - e3;
    }
    L.sync();
    if (t8) {  // column t: 8x8 block t >> 3, column t & 7
      const int b8 = t >> 3, j = t & 7, r0 = (b8 >> 1) * 8, c0 = (b8 & 1) * 8 + j;
      int v[8], o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = T.lres[r0 + i][c0];
      idct8_1d(v, o);
#pragma unroll
      for (int i = 0; i < 8; ++i) T.lres[r0 + i][c0] = (o[i] + 32) >> 6;
    } else {  // columns 2t, 2t + 1 of the 64 4x4 columns (block b = t >> 1)
      const int b = t >> 1, r0 = (b >> 2) * 4;
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        const int col = (b & 3) * 4 + (t & 1) * 2 + cc;
        const int f0 = T.lres[r0][col], f1 = T.lres[r0 + 1][col], f2 = T.lres[r0 + 2][col], f3 = T.lres[r0 + 3][col];
        const int g0 = f0 + f2, g1 = f0 - f2, g2 = (f1 >> 1) - f3, g3 = f1 + (f3 >> 1);
        T.lres[r0][col] = (g0 + g3 + 32) >> 6;
        T.lres[r0 + 1][col] = (g1 + g2 + 32) >> 6;
        T.lres[r0 + 2][col] = (g1 - g2 + 32) >> 6;
        T.lres[r0 + 3][col] = (g0 - g3 + 32) >> 6;
      }
    }
    {  // chroma column t: plane t >> 4, block (t >> 2) & 3, column t & 3
      const int pl = t >> 4, ck = (t >> 2) & 3, r0 = (ck >> 1) * 4, col = (ck & 1) * 4 + (t & 3);
      int32_t(*C)[8] = T.cres[pl];
      const int f0 = C[r0][col], f1 = C[r0 + 1][col], f2 = C[r0 + 2][col], f3 = C[r0 + 3][col];
      const int g0 = f0 + f2, g1 = f0 - f2, g2 = (f1 >> 1) - f3, g3 = f1 + (f3 >> 1);
      C[r0][col] = (g0 + g3 + 32) >> 6;
      C[r0 + 1][col] = (g1 + g2 + 32) >> 6;
      C[r0 + 2][col] = (g1 - g2 + 32) >> 6;
      C[r0 + 3][col] = (g0 - g3 + 32) >> 6;
    }
  }
  if (t == 0) {  // claim this macroblock's entries (part 2 writes those it still holds)
    L.amax(&const_cast<I2Line *>(lcol)[mx].claim, my);
    L.amax(&const_cast<I2Line *>(lrow)[my].claim, mx);
  }
  if (t == 31) {  // what part 2 needs of the header and the neighbourhood
    T.meta[0] = mb;
    T.meta[1] = h.type | (h.modes << 8) | (h.qp << 16);
    T.meta[2] = (A ? 1 : 0) | (B ? 2 : 0) | (C ? 4 : 0) | (D ? 8 : 0);
    T.meta[3] = static_cast<int32_t>(i4w0);
    T.meta[4] = static_cast<int32_t>(i4w1);
  }
  L.sync();
  rp_.mark(3);
}

template <class Lanes, class Prof>
VTS_HD VTS_INLINE void intra2_finish(const I2Ctx &a, const Lanes &L, I2Tile &T, I2Line *lcol, I2Line *lrow,
                                     const uint8_t *s_off4, const uint8_t *s_off8, Prof &rp_) {
  const int t = L.t;
  const int mb = T.meta[0], mbw = a.mbw, pitch = a.pitch;
  const int mx = mb % mbw, my = mb / mbw;
  const int type = T.meta[1] & 255, modes = (T.meta[1] >> 8) & 255;
  const bool A = T.meta[2] & 1, B = (T.meta[2] >> 1) & 1, C = (T.meta[2] >> 2) & 1, D = (T.meta[2] >> 3) & 1;
  const uint32_t i4w0 = static_cast<uint32_t>(T.meta[3]), i4w1 = static_cast<uint32_t>(T.meta[4]);
  const bool i16 = type == kMbI16, t8 = !i16 && (modes & kModeT8);
  uint8_t *Y = a.Y;
  uint8_t *UV = Y + a.uv_off;
  const int64_t yrow0 = static_cast<int64_t>(my * 16) * pitch + mx * 16;
  const int64_t crow0 = static_cast<int64_t>(my * 8) * pitch + mx * 16;
  (void)C;
  // ---- luma prediction + reconstruction into the tile
  if (i16) {
    const int mode = modes & 3;
    // sums: lanes 0..15 the top row sample t / plane term, 16..31 the left column
    const int k = t & 15;
    const int vt = t < 16 ? T.y[0][4 + k] : T.y[1 + k][3];
    const int s = L.red16(vt);
    const int pt = k < 8 ? (k + 1) * (t < 16 ? T.y[0][4 + 8 + k] - T.y[0][4 + 6 - k] : T.y[1 + 8 + k][3] - T.y[1 + 6 - k][3]) : 0;
    const int ps = L.red16(pt);
    const int st = L.bcast(s, 0), sl = L.bcast(s, 16);
    const int Hh = L.bcast(ps, 0), Vv = L.bcast(ps, 16);
    const int dc = (A && B) ? (st + sl + 16) >> 5 : (A ? (sl + 8) >> 4 : (B ? (st + 8) >> 4 : 128));
    const int aa = 16 * (T.y[16][3] + T.y[0][19]), bb = (5 * Hh + 32) >> 6, cc = (5 * Vv + 32) >> 6;
    const int r = t >> 1, c0 = (t & 1) * 8;
    const int left = T.y[1 + r][3];
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      const int c = c0 + x;
      const int p = mode == 0 ? T.y[0][4 + c] : (mode == 1 ? left : (mode == 2 ? dc : i2_c255((aa + bb * (c - 7) + cc * (r - 7) + 16) >> 5)));
      T.y[1 + r][4 + c] = static_cast<uint8_t>(i2_c255(p + T.lres[r][c]));
    }
    L.sync();
  } else if (t8) {
#pragma unroll 1
    for (int b8 = 0; b8 < 4; ++b8) {
      const int xo = (b8 & 1) * 8, yo = (b8 >> 1) * 8;
      const int r8 = (b8 >> 1) * 8 + (b8 & 1) * 2;
      const uint32_t i4w = (r8 >> 3) ? i4w1 : i4w0;
      const int m8 = (i4w >> (((r8 >> 1) & 3) * 8 + (r8 & 1) * 4)) & 15;
      const bool top = yo > 0 || B, left = xo > 0 || A;
      const bool tl = (xo > 0 && yo > 0) || (yo == 0 && xo > 0 ? B : (xo == 0 && yo > 0 ? A : D));
      const bool tr = b8 == 0 ? B : (b8 == 1 ? C : b8 == 2);
      const int ty = yo, tx = 4 + xo;
      // raw reference samples P(k): 0 = p[-1,-1], 1 + x = p[x,-1], 17 + y = p[-1,y]
      auto P = [&](int k) -> int {
        if (k == 0) return tl ? T.y[ty][tx - 1] : 0;
        if (k <= 8) return top ? T.y[ty][tx + k - 1] : 0;
        if (k <= 16) return tr ? T.y[ty][tx + k - 1] : (top ? T.y[ty][tx + 7] : 0);
        return left ? T.y[ty + k - 16][tx - 1] : 0;
      };
      // 8.3.2.2.1 filtered samples, lane t: E[t] (t < 27); E[1 + j] = L'[7 - j],
      // E[9] = T'[0] (p'[-1,-1]), E[10 + i] = T'[1 + i], E[0] = E[1], E[26] = E[25]
      if (t < 27) {
        int v = 0;
        if (t <= 8) {
          const int y = t == 0 ? 7 : 8 - t;  // L'[y]
          if (!left) v = 0;
          else if (y == 0) v = tl ? (P(0) + 2 * P(17) + P(18) + 2) >> 2 : (3 * P(17) + P(18) + 2) >> 2;
          else if (y == 7) v = (P(23) + 3 * P(24) + 2) >> 2;
          else v = (P(16 + y) + 2 * P(17 + y) + P(18 + y) + 2) >> 2;
        } else if (t == 9) {
          if (!tl) v = 0;
          else if (top && left) v = (P(1) + 2 * P(0) + P(17) + 2) >> 2;
          else if (top) v = (3 * P(0) + P(1) + 2) >> 2;
          else if (left) v = (3 * P(0) + P(17) + 2) >> 2;
          else v = P(0);
        } else {
          const int i = i2_min(t - 10, 15);  // T'[1 + i]
          if (!top) v = 0;
          else if (i == 0) v = tl ? (P(0) + 2 * P(1) + P(2) + 2) >> 2 : (3 * P(1) + P(2) + 2) >> 2;
          else if (i == 15) v = (P(15) + 3 * P(16) + 2) >> 2;
          else v = (P(i) + 2 * P(1 + i) + P(2 + i) + 2) >> 2;
        }
        T.p8[t] = static_cast<uint8_t>(v);
      }
      L.sync();
      // F(k) = 3-tap of E, A(k) = mean of E[k + 1], E[k + 2]; DC (lane 31)
      {
        const uint8_t *e = T.p8;
        if (t < 25) T.p8[32 + t] = static_cast<uint8_t>((e[t] + 2 * e[t + 1] + e[t + 2] + 2) >> 2);
        if (t < 24) T.p8[64 + t] = static_cast<uint8_t>((e[1 + t] + e[2 + t] + 1) >> 1);
        if (t == 31) {
          int st = 0, sl = 0;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            st += e[10 + i];
            sl += e[1 + i];
          }
          T.p8[88] = static_cast<uint8_t>((top && left) ? (st + sl + 8) >> 4 : (left ? (sl + 4) >> 3 : (top ? (st + 4) >> 3 : 128)));
        }
      }
      L.sync();
      {
        const uint8_t *offs = s_off8 + 64 * i2_min(m8, 8);  // > 8: not a mode (as mode 8)
        const int x = t & 7;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int y = (t >> 3) + 4 * hh;
          T.y[1 + yo + y][4 + xo + x] = static_cast<uint8_t>(i2_c255(T.p8[offs[y * 8 + x]] + T.lres[yo + y][xo + x]));
        }
      }
      L.sync();
    }
  } else {
    const int bs = t >> 4, p = t & 15;
#pragma unroll 1
    for (int s = 0; s <= 9; ++s) {
      const int blk = i4_step_blk(s, bs);
      const int bx = blk & 3, by = blk >> 2;
      const uint32_t i4w = blk >= 8 ? i4w1 : i4w0;
      const int m4 = blk >= 0 ? (i4w >> (((blk >> 1) & 3) * 8 + (blk & 1) * 4)) & 15 : 0;
      const bool top = by > 0 || B, left = bx > 0 || A;
      const bool tl = (bx > 0 && by > 0) || (by == 0 && bx > 0 ? B : (bx == 0 && by > 0 ? A : D));
      const bool tr = by == 0 ? (bx < 3 ? B : C) : (bx < 3 && i2_blkidx((by - 1) * 4 + bx + 1) < i2_blkidx(blk));
      const int ty = by * 4, tx = 4 + bx * 4;
      if (blk >= 0) {  // E[p] (p < 15) / DC (p = 15)
        int v;
        if (p <= 4) {
          const int y = p <= 1 ? 3 : 4 - p;  // E[0] = E[1] = L[4] = p[-1,3]; E[2..4] = p[-1, 2..0]
          v = left ? T.y[ty + 1 + y][tx - 1] : 0;
        } else if (p == 5) {
          v = tl ? T.y[ty][tx - 1] : 0;
        } else if (p < 15) {
          const int x = i2_min(p - 6, 7);  // E[6 + x] = p[x,-1]; E[14] = E[13]
          if (x < 4) v = top ? T.y[ty][tx + x] : 0;
          else v = tr ? T.y[ty][tx + x] : (top ? T.y[ty][tx + 3] : 0);
        } else {
          int st = 0, sl = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            st += T.y[ty][tx + i];
            sl += T.y[ty + 1 + i][tx - 1];
          }
          v = (top && left) ? (st + sl + 4) >> 3 : (left ? (sl + 2) >> 2 : (top ? (st + 2) >> 2 : 128));
        }
        T.e4[bs][p] = static_cast<uint8_t>(v);
      }
      L.sync();
      if (blk >= 0) {
        const int x = p & 3, y = p >> 2;
        const int idx = s_off4[16 * i2_min(m4, 8) + p];  // > 8: not a mode (as mode 8)
        const uint8_t *e = T.e4[bs];
        const int k = idx >= 32 ? idx - 32 : (idx >= 16 ? idx - 16 : idx);
        const int e0 = e[i2_min(k, 15)], e1 = e[i2_min(k + 1, 15)], e2 = e[i2_min(k + 2, 15)];
        const int v = idx < 16 ? e0 : (idx < 32 ? (e0 + 2 * e1 + e2 + 2) >> 2 : (idx < 47 ? (e1 + e2 + 1) >> 1 : e[15]));
        T.y[ty + 1 + y][tx + x] = static_cast<uint8_t>(i2_c255(v + T.lres[by * 4 + y][bx * 4 + x]));
      }
      L.sync();
    }
  }
  rp_.mark(4);
  // ---- chroma (8.3.4): lane t = plane t >> 4, 4x4 block (t >> 2) & 3, row t & 3
  {
    const int pl = t >> 4, ck = (t >> 2) & 3, yy = t & 3, ox = (ck & 1) * 4, oy = (ck >> 1) * 4;
    const int cm = (modes >> 2) & 3;
    const uint8_t(*Cp)[12] = T.c[pl];  // Cp[0][1 + x] = p[x,-1], Cp[1 + y][0] = p[-1,y], Cp[0][0] = p[-1,-1]
    int v[4];
    if (cm == 0) {
      int st = 0, sl = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        st += Cp[0][1 + ox + i];
        sl += Cp[1 + oy + i][0];
      }
      int dc = 128;
      if ((ox == 0 && oy == 0) || (ox && oy)) {
        if (B && A) dc = (st + sl + 4) >> 3;
        else if (A) dc = (sl + 2) >> 2;
        else if (B) dc = (st + 2) >> 2;
      } else if (ox) {
        if (B) dc = (st + 2) >> 2;
        else if (A) dc = (sl + 2) >> 2;
      } else {
        if (A) dc = (sl + 2) >> 2;
        else if (B) dc = (st + 2) >> 2;
      }
#pragma unroll
      for (int x = 0; x < 4; ++x) v[x] = dc;
    } else if (cm == 1) {
#pragma unroll
      for (int x = 0; x < 4; ++x) v[x] = Cp[1 + oy + yy][0];
    } else if (cm == 2) {
#pragma unroll
      for (int x = 0; x < 4; ++x) v[x] = Cp[0][1 + ox + x];
    } else {
      int Hh = 0, Vv = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        Hh += (i + 1) * (Cp[0][1 + 4 + i] - Cp[0][1 + 2 - i]);
        Vv += (i + 1) * (Cp[1 + 4 + i][0] - (2 - i >= 0 ? Cp[1 + 2 - i][0] : Cp[0][0]));
      }
      const int aa = 16 * (Cp[8][0] + Cp[0][8]);
      const int bb = (34 * Hh + 32) >> 6, cc = (34 * Vv + 32) >> 6;
#pragma unroll
      for (int x = 0; x < 4; ++x) v[x] = i2_c255((aa + bb * (ox + x - 3) + cc * (oy + yy - 3) + 16) >> 5);
    }
    L.sync();  // every border read before the samples overwrite the tile's inside
#pragma unroll
    for (int x = 0; x < 4; ++x)
      T.c[pl][1 + oy + yy][1 + ox + x] = static_cast<uint8_t>(i2_c255(v[x] + T.cres[pl][oy + yy][ox + x]));
  }
  L.sync();
  rp_.mark(5);
  // ---- the macroblock to HBM (whole rows) and its bottom row / right column
  // to the line buffers
  I2Line &lme = lcol[mx], &rme = lrow[my];
  const bool wcol = lme.claim == my, wrow = rme.claim == mx;  // the only writer of the entry this round
  if (t < 16) {
    const uint8_t *src = &T.y[1 + t][4];
    const I2V4 row = i2_ld4(src);
    i2_st4(Y + yrow0 + static_cast<int64_t>(t) * pitch, row);
    if (t == 15 && wcol) i2_st4(lme.y, row);
    if (wrow) rme.y[t] = src[15];
  } else if (t < 24) {
    const int r = t - 16;
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      w[i] = i2_pack4(T.c[0][1 + r][1 + 2 * i], T.c[1][1 + r][1 + 2 * i], T.c[0][1 + r][2 + 2 * i], T.c[1][1 + r][2 + 2 * i]);
    const I2V4 row = {w[0], w[1], w[2], w[3]};
    i2_st4(UV + crow0 + static_cast<int64_t>(r) * pitch, row);
    if (r == 7 && wcol) i2_st4(lme.c, row);
    if (wrow) {
      rme.c[2 * r] = T.c[0][1 + r][8];
      rme.c[2 * r + 1] = T.c[1][1 + r][8];
    }
  } else if (t == 24) {
    if (wcol) lme.tag = my;
    if (wrow) rme.tag = mx;
  }
  L.sync();
}


}  // namespace i2
}  // namespace vts
