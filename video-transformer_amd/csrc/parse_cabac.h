// parse_cabac.h — CABAC slice_data() parser of the general device decoder
// (ITU-T H.264 9.3): High-profile I, P and B slices with 8x8 transforms.  The
// kernel (h264_parse_full) runs one slice per single-lane wave, so the whole
// arithmetic decoder is wave-uniform scalar code; the CPU harness compiles the
// same header.  It produces exactly what the CAVLC parser produces (MbRec,
// coefficient blocks, intra dependency level) plus, for the reconstruction,
// transform_size_8x8_flag (MbRec.modes bit 4) and 8x8 coefficient blocks.
//
// Context states and the engine's tables live in lane tables (LaneTab: the
// idle lanes of a few VGPRs, read and written with v_readlane / v_writelane),
// so a bin costs no memory access.  The
// neighbour facts CABAC's context selection needs come through the CAVLC
// parser's LDS neighbour copies: coded_block_flag bits in the (CAVLC-only)
// nzc bytes, clamped |mvd| of inter macroblocks' bottom rows in their i4
// bytes, the neighbourhood's |mvd| in FullScratch.mvx.
#pragma once
#include <cstdint>
#include <type_traits>

#include "h264_cabac_tables.h"
#include "parse_full.h"

namespace vts {
namespace full {

#if defined(__HIPCC__)
#define VTS_CTAB __device__ __constant__ static const
#else
#define VTS_CTAB static const
#endif
VTS_CTAB int8_t kCabInitI[VTS_CABAC_NCTX][2] = VTS_CABAC_INIT_I_DATA;
VTS_CTAB int8_t kCabInitP[VTS_CABAC_NCTX][2] = VTS_CABAC_INIT_P0_DATA;
#undef VTS_CTAB

// The engine's tables as 64 dwords each, loaded into lane tables (LaneTab) at
// slice start: rangeTabLPS[pStateIdx][0..3] in bytes 0..3; the next state
// byte (pStateIdx << 1 | valMPS-switch, to be XORed with valMPS) after an LPS
// (transIdxLPS, switching valMPS at state 0) in byte 0 and after an MPS
// (transIdxMPS) in byte 1; the 8x8 block's significant / last ctxIdxInc
// (Table 9-43, frame) and zig-zag position of coefficient i in bytes 0 / 1 / 2
struct CabLanes {
  uint32_t lps[64], trans[64], s8[64];
};
constexpr CabLanes make_cab_lanes() {
  CabLanes t{};
  const uint8_t r[64][4] = VTS_CABAC_RANGE_LPS_DATA;
  const uint8_t tr[64] = VTS_CABAC_TRANS_LPS_DATA;
  const uint8_t sig[63] = VTS_SIG8x8_DATA;
  const uint8_t last[63] = VTS_LAST8x8_DATA;
  const uint8_t zz[64] = VTS_ZZ8_DATA;
  for (int i = 0; i < 64; ++i) {
    t.lps[i] = r[i][0] | (uint32_t(r[i][1]) << 8) | (uint32_t(r[i][2]) << 16) | (uint32_t(r[i][3]) << 24);
    t.trans[i] = (uint32_t(tr[i]) << 1) | (i == 0 ? 1u : 0u) | (uint32_t(i < 62 ? i + 1 : 62) << 9);
    t.s8[i] = (i < 63 ? sig[i] | (uint32_t(last[i]) << 8) : 0u) | (uint32_t(zz[i]) << 16);
  }
  return t;
}
#if defined(__HIPCC__)
__device__ __constant__ static const CabLanes kCabLanes = make_cab_lanes();
#else
static const CabLanes kCabLanes = make_cab_lanes();
#endif
// per-category ctxIdxOffset parts (ctxBlockCat 0..4) as byte fields of one constant
VTS_HD VTS_INLINE int cbf_off(int cat) { return static_cast<int>((0x100C080400ull >> (8 * cat)) & 255u); }
VTS_HD VTS_INLINE int sig_off(int cat) { return static_cast<int>((0x2F2C1D0F00ull >> (8 * cat)) & 255u); }
VTS_HD VTS_INLINE int abs_off(int cat) { return static_cast<int>((0x271E140A00ull >> (8 * cat)) & 255u); }

// The engine's codIRange / codIOffset live in VGPRs: an opaque move makes
// them divergent, so their arithmetic issues on the vector ALUs (four per
// compute unit) instead of the one scalar unit that every wave of the compute
// unit shares, which the parser saturates; a decision's outcome, next state
// and renormalisation shift come back to the scalar side by readfirstlane
// (CABAC B parse -4 % same-box, profiles/r03_cabac_vgpr_engine_ab.txt;
// VTS_EXP_SENGINE keeps the scalar engine)
#if defined(__HIP_DEVICE_COMPILE__) && !defined(VTS_EXP_SENGINE)
__device__ __forceinline__ uint32_t vts_in_vgpr(uint32_t x) {
  uint32_t r;
  asm("; engine state in a VGPR" : "=v"(r) : "0"(x));
  return r;
}
#define VTS_EV(x) vts_in_vgpr(x)
#define VTS_EU(x) static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(x)))
#else
#define VTS_EV(x) (x)
#define VTS_EU(x) (x)
#endif

struct CabacParser : Parser {
  // The engine (9.3.1.2, 9.3.3.2) with codIOffset scaled: val holds the 9-bit
  // codIOffset in bits 31..23 and the next `la` bitstream bits below it, so
  // renormalisation is a shift of val and the bit reader is touched once per
  // 16 bits (la < 8 -> 16 more), not per bin.  codIOffset >= codIRange is
  // val >= codIRange << 23.
  uint32_t range, val;
  int32_t la;
  bool prev_qpd;  // the previous macroblock of the slice has mb_qp_delta != 0
  // context states (pStateIdx << 1 | valMPS), four per dword.  The residual
  // contexts of 4x4 blocks (ctxIdx 85..275) fill st[0] (slot c - 85); all
  // others (0..84, and 399..459 at 85..145) st[1], so every decode's table is
  // known at compile time (slot q: lane q >> 2, byte q & 3)
  LaneTab st[2];
  static VTS_HD VTS_INLINE int ctx_tab(int c) { return (c >= 85 && c <= 275) ? 0 : 1; }
  static VTS_HD VTS_INLINE int ctx_slot(int c) { return c >= 399 ? c - 314 : (c >= 85 ? c - 85 : c); }
  LaneTab lps, trn, s8;  // kCabLanes

  // ---------------------------------------------- arithmetic decoder (9.3.3.2)
  VTS_HD VTS_INLINE void cab_start() {  // 9.3.1.2: codIOffset = read_bits(9)
    range = VTS_EV(510u);
    val = VTS_EV(br.bits(32));
    la = 23;
  }
  // bits the engine has consumed (9.3.1.2's 9 + every renormalisation shift)
  VTS_HD VTS_INLINE int32_t cab_consumed() const { return br.consumed() - la; }
  VTS_HD VTS_INLINE void cab_fill() {
    if (la < 8) {
      val |= br.bits(16) << (7 - la);
      la += 16;
    }
  }
  VTS_HD VTS_INLINE void cab_tables() {
    for (int i = 0; i < 64; ++i) {
      lps.set(i, kCabLanes.lps[i]);
      trn.set(i, kCabLanes.trans[i]);
      s8.set(i, kCabLanes.s8[i]);
    }
  }
  VTS_HD VTS_INLINE void cab_init(bool is_i, int qp) {  // 9.3.1.1
    const int q = qp < 0 ? 0 : (qp > 51 ? 51 : qp);
    for (int t = 0; t < 2; ++t)
      for (int w = 0; w < 64; ++w) {
        uint32_t word = 0;
        for (int b = 0; b < 4; ++b) {
          const int slot = 4 * w + b;
          // the ctxIdx of this slot (the inverse of ctx_slot); unused slots stay 0
          const int i = t == 0 ? (slot <= 190 ? slot + 85 : -1) : (slot < 85 ? slot : (slot <= 145 ? slot + 314 : -1));
          if (i < 0) continue;
          const int m = is_i ? kCabInitI[i][0] : kCabInitP[i][0], n = is_i ? kCabInitI[i][1] : kCabInitP[i][1];
          int pre = ((m * q) >> 4) + n;
          pre = pre < 1 ? 1 : (pre > 126 ? 126 : pre);
          word |= static_cast<uint32_t>(pre <= 63 ? (63 - pre) << 1 : ((pre - 64) << 1) | 1) << (8 * b);
        }
        st[t].set(w, word);
      }
  }
  VTS_HD VTS_INLINE uint32_t dec(int ctx) {  // DecodeDecision
    VTS_PARSE_TRACE(1);
    const int q = ctx_slot(ctx);
    const uint32_t ln = static_cast<uint32_t>(q >> 2) & 63u, sh = static_cast<uint32_t>(q & 3) * 8u;
    // which of the two lane tables: folded where it is a constant (every call
    // site), else both are read and written with selects (no branch)
    const bool fixed = __builtin_constant_p(ctx_tab(ctx)), hi = ctx_tab(ctx) != 0;
    const uint32_t wa = fixed && hi ? 0u : st[0].get(ln), wb = fixed && !hi ? 0u : st[1].get(ln);
    const uint32_t word = hi ? wb : wa;
    const uint32_t s = (word >> sh) & 127u, ps = s >> 1, mps = s & 1u;
    const uint32_t lpsr = (lps.get(ps) >> ((range >> 3) & 24u)) & 255u;
    const uint32_t tw = trn.get(ps);  // read on both paths: no branch
    range -= lpsr;
    const uint32_t rs = range << 23;
    const bool lpsb = val >= rs;
    const uint32_t bin = mps ^ (lpsb ? 1u : 0u);
    const uint32_t ns = VTS_EU(((tw >> (lpsb ? 0u : 8u)) & 127u) ^ mps);
    val -= lpsb ? rs : 0u;
    range = lpsb ? lpsr : range;
    const uint32_t nw = (word & ~(255u << sh)) | (ns << sh);
    if (fixed) {
      if (hi) st[1].set(ln, nw);
      else st[0].set(ln, nw);
    } else {
      st[0].set(ln, hi ? wa : nw);
      st[1].set(ln, hi ? nw : wb);
    }
    const int n = static_cast<int>(VTS_EU(__builtin_clz(range) - 23));  // RenormD as one shift (0..6)
    range <<= n;
    val <<= n;
    la -= n;
    cab_fill();
    return VTS_EU(bin);
  }
  VTS_HD VTS_INLINE uint32_t bypass() {  // DecodeBypass
    VTS_PARSE_TRACE(2);
    // the doubled codIOffset needs 10 bits: its top bit leaves val, and then
    // the offset is >= codIRange whatever val holds (val - rs wraps to the
    // right difference)
    const uint32_t top = val >> 31;
    val <<= 1;
    --la;
    cab_fill();
    const uint32_t rs = range << 23;
    if (VTS_EU((top || val >= rs) ? 1u : 0u)) {
      val -= rs;
      return 1;
    }
    return 0;
  }
  VTS_HD VTS_INLINE uint32_t term() {  // DecodeTerminate: 1 ends parsing, no renormalisation
    VTS_PARSE_TRACE(3);
    range -= 2;
    if (VTS_EU(val >= (range << 23) ? 1u : 0u)) return 1;
    if (VTS_EU(range < 256 ? 1u : 0u)) {
      range <<= 1;
      val <<= 1;
      --la;
      cab_fill();
    }
    return 0;
  }

  // ------------------------------------------------------ neighbour facts
  VTS_HD VTS_INLINE uint32_t cbf_of(const MbRec &m) const {
    return static_cast<uint32_t>(m.nzc[0]) | (static_cast<uint32_t>(m.nzc[1]) << 8) |
           (static_cast<uint32_t>(m.nzc[2]) << 16) | (static_cast<uint32_t>(m.nzc[3]) << 24);
  }
  VTS_HD VTS_INLINE void set_cbf(uint32_t bit) {
    MbRec &m = cur();
    m.nzc[bit >> 3] = static_cast<uint8_t>(m.nzc[bit >> 3] | (1u << (bit & 7)));
  }
  VTS_HD VTS_INLINE bool avail_not(int n, int type) const { return n != -1 && rec(n).type != type; }
  // condTermFlagN of coded_block_flag (9.3.3.1.1.9)
  VTS_HD VTS_INLINE int cbf_cond(int n, bool cur_intra, bool tb, uint32_t bit) const {
    if (n == -1) return cur_intra ? 1 : 0;
    const MbRec &m = rec(n);
    if (m.type == kMbPcm) return 1;
    if (!tb || m.type == kMbSkip) return 0;
    return static_cast<int>((cbf_of(m) >> bit) & 1u);
  }
  VTS_HD VTS_INLINE int cbf_luma_inc(int addr, int bx, int by, bool intra) const {
    int inc = 0;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      int xw = 0, yw = 0;
      const int n = nb_mb(addr, nb ? bx * 4 : bx * 4 - 1, nb ? by * 4 - 1 : by * 4, 16, &xw, &yw);
      bool tb = false;
      uint32_t bit = 0;
      if (n != -1) {
        tb = (rec(n).cbp >> ((yw / 8) * 2 + xw / 8)) & 1;
        bit = 1u + static_cast<uint32_t>((yw / 4) * 4 + xw / 4);
      }
      inc += cbf_cond(n, intra, tb, bit) << nb;
    }
    return inc;
  }
  VTS_HD VTS_INLINE int cbf_chroma_inc(int addr, int pl, int blk, bool dc, bool intra) const {
    int inc = 0;
    const int x = dc ? 0 : (blk & 1) * 4, y = dc ? 0 : (blk >> 1) * 4;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      int xw = 0, yw = 0;
      const int n = nb_mb(addr, nb ? x : x - 1, nb ? y - 1 : y, 8, &xw, &yw);
      bool tb = false;
      uint32_t bit = 0;
      if (n != -1) {
        const int cc = rec(n).cbp >> 4;
        tb = dc ? cc != 0 : cc == 2;
        bit = dc ? 17u + static_cast<uint32_t>(pl) : 19u + static_cast<uint32_t>(4 * pl + (yw / 4) * 2 + xw / 4);
      }
      inc += cbf_cond(n, intra, tb, bit) << nb;
    }
    return inc;
  }
  // Min(|mvd_lX|, 33) at luma (xN, yN) of the current macroblock's
  // neighbourhood (skipped, intra and direct blocks carry 0)
  // (xN, yN in -1..15: A and B neighbours only; mvd_border filled the edges)
  VTS_HD VTS_INLINE int mvd_at(int addr, int xN, int yN, int comp, int l = 0) const {
    return sc->mvx[l][(yN >> 2) + 1][(xN >> 2) + 1][comp];
  }
  // a new macroblock's mvx: the left column takes the previous macroblock's
  // right column (when it is the left neighbour A), the top row the bottom-row
  // |mvd| the macroblock above kept in its record (inter only), the inside 0;
  // one cell per lane (every read is issued before any write)
  VTS_HD VTS_INLINE void mvd_border(int A, int B) {
    const bool top_inter = B != -1 && rec(B).type == kMbInter;
    const MbRec *tb = top_inter ? &rec(B) : nullptr;
    const MbRecB *tb1 = top_inter && bframes ? &rec1(B) : nullptr;
#if defined(__HIP_DEVICE_COMPILE__)
    VTS_LANES(50, i) {
      const int l = i / 25, r = (i % 25) / 5, c = i % 5;
      uint8_t v0 = 0, v1 = 0;
      if (r > 0 && c == 0) {
        if (A != -1) {
          v0 = sc->mvx[l][r][4][0];
          v1 = sc->mvx[l][r][4][1];
        }
      } else if (r == 0 && c > 0 && tb) {
        const uint8_t *src = l ? (tb1 ? tb1->mvd1 : nullptr) : tb->i4;
        if (src) {
          v0 = src[2 * (c - 1)];
          v1 = src[2 * (c - 1) + 1];
        }
      }
      asm volatile("" ::: "memory");  // every lane's read before any lane's write
      sc->mvx[l][r][c][0] = v0;
      sc->mvx[l][r][c][1] = v1;
    }
#else
    // host: the lanes' reads all precede their writes on the device; serially,
    // compute the cells first
    uint8_t nv[2][5][5][2] = {};
    for (int l = 0; l < 2; ++l)
      for (int r = 1; r < 5; ++r)
        if (A != -1) {
          nv[l][r][0][0] = sc->mvx[l][r][4][0];
          nv[l][r][0][1] = sc->mvx[l][r][4][1];
        }
    if (tb)
      for (int c = 1; c < 5; ++c) {
        nv[0][0][c][0] = tb->i4[2 * (c - 1)];
        nv[0][0][c][1] = tb->i4[2 * (c - 1) + 1];
        if (tb1) {
          nv[1][0][c][0] = tb1->mvd1[2 * (c - 1)];
          nv[1][0][c][1] = tb1->mvd1[2 * (c - 1) + 1];
        }
      }
    for (int l = 0; l < 2; ++l)
      for (int r = 0; r < 5; ++r)
        for (int c = 0; c < 5; ++c) {
          sc->mvx[l][r][c][0] = nv[l][r][c][0];
          sc->mvx[l][r][c][1] = nv[l][r][c][1];
        }
#endif
  }
  // condTermFlagN of ref_idx_lX (9.3.3.1.1.6): refIdxLX > 0 of an inter
  // neighbour that is neither skipped nor predicted in direct mode
  // (xN, yN in -1..15, A and B neighbours: the left / top macroblocks' flags
  // come from refb, which mvd_border filled)
  VTS_HD VTS_INLINE int ref_gt0_at(int addr, int xN, int yN, int l = 0) const {
    if (xN < 0) return static_cast<int>((refb >> (8 * l + (yN >> 3))) & 1u);
    if (yN < 0) return static_cast<int>((refb >> (8 * l + 4 + (xN >> 3))) & 1u);
    const MbRec &m = cur();
    const int p8 = (yN >> 3) * 2 + (xN >> 3);
    if (bframes && ((cur1().direct >> p8) & 1)) return 0;
    return (l ? cur1().ref1[p8] : m.ref[p8]) > 0 ? 1 : 0;
  }
  // refb bit 8 l + k: refIdxLX > 0 of the left neighbour's 8x8 row k (k 0, 1)
  // and bit 8 l + 4 + k of the top neighbour's 8x8 column k (inter, neither
  // skipped nor direct; 0 where unavailable)
  uint32_t refb;
  VTS_HD VTS_INLINE void ref_border(int A, int B) {
    uint32_t f = 0;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int n = nb ? B : A;
      if (n == -1 || rec(n).type != kMbInter) continue;
      const MbRec &m = rec(n);
      const MbRecB *m1 = bframes ? &rec1(n) : nullptr;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int p8 = nb ? 2 + k : 2 * k + 1;  // top: bottom 8x8 row; left: right 8x8 column
        if (m1 && ((m1->direct >> p8) & 1)) continue;
        f |= (m.ref[p8] > 0 ? 1u : 0u) << (4 * nb + k);
        if (m1) f |= (m1->ref1[p8] > 0 ? 1u : 0u) << (8 + 4 * nb + k);
      }
    }
    refb = f;
  }
  // Intra NxN mode predictor (8.3.1.1 / 8.3.2.1) of the block at (x0, y0)
  VTS_HD VTS_INLINE int mode_pred(int addr, int x0, int y0, bool is8) const {
    int xa = 0, ya = 0, xb = 0, yb = 0;
    const int a = nb_mb(addr, x0 - 1, y0, 16, &xa, &ya), b = nb_mb(addr, x0, y0 - 1, 16, &xb, &yb);
    if (a == -1 || b == -1) return 2;
    const MbRec &ma = rec(a), &mb = rec(b);
    if (cip && (ma.type == kMbInter || ma.type == kMbSkip || mb.type == kMbInter || mb.type == kMbSkip)) return 2;
    int md[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const MbRec &m = i ? mb : ma;
      const int xw = i ? xb : xa, yw = i ? yb : ya;
      if (m.type != kMbI4x4) {
        md[i] = 2;
        continue;
      }
      int r = (yw / 4) * 4 + xw / 4;
      if (is8 && !(m.modes & kModeT8)) {  // Intra4x4PredMode[luma8x8BlkIdxN * 4 + (A ? 1 : 2)]
        const int k = ((yw / 8) * 2 + xw / 8) * 4 + (i ? 2 : 1);
        r = blk_y(k) * 4 + blk_x(k);
      }
      md[i] = (m.i4[r >> 1] >> ((r & 1) * 4)) & 15;
    }
    return vts_min(md[0], md[1]);
  }
  VTS_HD VTS_INLINE void set_i4(int r, int mode) {
    MbRec &m = cur();
    m.i4[r >> 1] = static_cast<uint8_t>((m.i4[r >> 1] & (0xf0 >> ((r & 1) * 4))) | (mode << ((r & 1) * 4)));
  }

  // ------------------------------------------------------- syntax elements
  // mb_type of an I macroblock (Table 9-36): I slice prefix at ctxIdx 3, or
  // the suffix of a P (ctxIdxOffset sfx 17) or B (32) slice's intra mb_type; 0..25
  VTS_HD VTS_INLINE int i_type(int sfx, int inc0) {
    if (!dec(sfx ? sfx : 3 + inc0)) return 0;
    if (term()) return 25;
    const int luma = static_cast<int>(dec(sfx ? sfx + 1 : 6));
    int chroma = static_cast<int>(dec(sfx ? sfx + 2 : 7));
    if (chroma) chroma += static_cast<int>(dec(sfx ? sfx + 2 : 8));
    int pm = static_cast<int>(dec(sfx ? sfx + 3 : 9)) << 1;
    pm |= static_cast<int>(dec(sfx ? sfx + 3 : 10));
    return 1 + pm + 4 * chroma + 12 * luma;
  }
  // B mb_type (Table 9-37 binarization, ctxIdx 27..35 per Table 9-39): 0..22,
  // or 23 + the intra suffix's mb_type
  VTS_HD VTS_INLINE int b_type(int inc0) {
    if (!dec(27 + inc0)) return 0;                                       // B_Direct_16x16
    if (!dec(27 + 3)) return 1 + static_cast<int>(dec(27 + 5));           // B_L0 / B_L1_16x16
    int bits = static_cast<int>(dec(27 + 4)) << 3;
    bits |= static_cast<int>(dec(27 + 5)) << 2;
    bits |= static_cast<int>(dec(27 + 5)) << 1;
    bits |= static_cast<int>(dec(27 + 5));
    if (bits < 8) return bits + 3;
    if (bits == 13) return 23 + i_type(32, 0);
    if (bits == 14) return 11;
    if (bits == 15) return 22;                                           // B_8x8
    bits = (bits << 1) | static_cast<int>(dec(27 + 5));
    return bits - 4;
  }
  // B sub_mb_type (Table 9-38, ctxIdx 36..39): 0..12
  VTS_HD VTS_INLINE int b_sub() {
    if (!dec(36)) return 0;
    if (!dec(37)) return 1 + static_cast<int>(dec(39));
    int t = 3;
    if (dec(38)) {
      if (dec(39)) return 11 + static_cast<int>(dec(39));
      t += 4;
    }
    t += 2 * static_cast<int>(dec(39));
    t += static_cast<int>(dec(39));
    return t;
  }
  // ref_idx_lX (U binarization, ctxIdx 54..59)
  VTS_HD VTS_INLINE int ref_idx(int addr, int x0, int y0, int l) {
    int v = 0;
    if (dec(54 + ref_gt0_at(addr, x0 - 1, y0, l) + 2 * ref_gt0_at(addr, x0, y0 - 1, l))) {
      v = 1;
      if (dec(58)) {
        v = 2;
        while (dec(59))
          if (++v > 32) break;
      }
    }
    return v;
  }
  // mb_pred / sub_mb_pred of a B macroblock (7.3.5.1-2): mb_type 0..22;
  // *small: a partition below 8x8 (or a direct one without
  // direct_8x8_inference) rules out transform_size_8x8_flag
  VTS_HD VTS_INLINE bool b_inter_cabac(int addr, int mb_type, bool *small) {
    uint8_t *pm = sc->pm;
    int8_t *sub = sc->sub, *r0 = sc->refs, *r1 = sc->refs1;
    for (int k = 0; k < 4; ++k) {
      pm[k] = 0;
      sub[k] = 0;
      r0[k] = r1[k] = -1;
    }
    if (mb_type == 0) {  // B_Direct_16x16
      VTS_PARSE_TRACE(6);
      cur1().direct = 0x0f | kDirect16;
      if (!direct8x8) *small = true;
      direct_pred(addr, 0xffffu);
      return !err;
    }
    int shape;
    if (mb_type <= 3) {
      shape = 0;
      pm[0] = static_cast<uint8_t>(mb_type);
    } else if (mb_type < 22) {
      shape = (mb_type & 1) ? 2 : 1;
      pm[0] = kBPart[mb_type] & 3;
      pm[1] = kBPart[mb_type] >> 2;
    } else {
      shape = 3;
      for (int k = 0; k < 4; ++k) {
        const int v = b_sub();
        pm[k] = kBSub[v] & 3;
        sub[k] = static_cast<int8_t>(kBSub[v] >> 2);
        if (pm[k] == 0) {
          cur1().direct |= static_cast<uint8_t>(1u << k);
          if (!direct8x8) *small = true;
        } else if (sub[k]) {
          *small = true;
        }
      }
    }
    const int nparts = shape == 0 ? 1 : (shape < 3 ? 2 : 4);
    MbRec &m = cur();
    MbRecB &m1 = cur1();
    for (int l = 0; l < 2; ++l) {
      const int nref = l ? bc.x->num_ref1 : s->num_ref;
      int8_t *rr = l ? r1 : r0;
      for (int k = 0; k < nparts; ++k) {
        if (!((pm[k] >> l) & 1)) continue;
        const int x0 = (shape == 2 || shape == 3) ? 8 * (k & 1) : 0;
        const int y0 = shape == 1 ? 8 * k : (shape == 3 ? 8 * (k >> 1) : 0);
        const int v = nref > 1 ? ref_idx(addr, x0, y0, l) : 0;
        if (v >= nref || (l ? bc.x->ref_slot1[v & 31] : s->ref_slot[v & 31]) < 0) {
          err |= DEC_E_NO_REF;
          return false;
        }
        rr[k] = static_cast<int8_t>(v);
        // the partition's 8x8 quarters carry the index for later contexts
        const int pw = (shape == 0 || shape == 1) ? 2 : 1, ph = (shape == 0 || shape == 2) ? 2 : 1;
        for (int qy = 0; qy < ph; ++qy)
          for (int qx = 0; qx < pw; ++qx) {
            const int q8 = (y0 / 8 + qy) * 2 + x0 / 8 + qx;
            if (l) m1.ref1[q8] = static_cast<int8_t>(v);
            else m.ref[q8] = static_cast<int8_t>(v);
          }
      }
    }
    for (int l = 0; l < 2; ++l)
      for (int k = 0; k < nparts; ++k) {
        if (!((pm[k] >> l) & 1)) continue;
        int nsub = 1, pw, ph, x0, y0;
        if (shape == 0) { pw = ph = 16; x0 = y0 = 0; }
        else if (shape == 1) { pw = 16; ph = 8; x0 = 0; y0 = 8 * k; }
        else if (shape == 2) { pw = 8; ph = 16; x0 = 8 * k; y0 = 0; }
        else {
          x0 = 8 * (k & 1);
          y0 = 8 * (k >> 1);
          nsub = sub[k] == 0 ? 1 : (sub[k] == 3 ? 4 : 2);
          pw = (sub[k] == 0 || sub[k] == 1) ? 8 : 4;
          ph = (sub[k] == 0 || sub[k] == 2) ? 8 : 4;
        }
        for (int q = 0; q < nsub; ++q) {
          int sx = x0, sy = y0;
          if (shape == 3) {
            if (sub[k] == 1) sy += 4 * q;
            else if (sub[k] == 2) sx += 4 * q;
            else if (sub[k] == 3) { sx += 4 * (q & 1); sy += 4 * (q >> 1); }
          }
          const int dx = mvd(40, mvd_at(addr, sx - 1, sy, 0, l) + mvd_at(addr, sx, sy - 1, 0, l));
          const int dy = mvd(47, mvd_at(addr, sx - 1, sy, 1, l) + mvd_at(addr, sx, sy - 1, 1, l));
          sc->mvd[l][4 * k + q][0] = dx;
          sc->mvd[l][4 * k + q][1] = dy;
          const uint8_t ax = static_cast<uint8_t>(vts_min(dx < 0 ? -dx : dx, 33));
          const uint8_t ay = static_cast<uint8_t>(vts_min(dy < 0 ? -dy : dy, 33));
          const uint32_t bm = blk_mask(sx, sy, pw, ph);
          VTS_LANES(16, b) if ((bm >> b) & 1u) {
            sc->mvx[l][1 + (b >> 2)][1 + (b & 3)][0] = ax;
            sc->mvx[l][1 + (b >> 2)][1 + (b & 3)][1] = ay;
          }
        }
      }
    // the references the parse recorded are set again by the motion below
    for (int k = 0; k < 4; ++k) {
      m.ref[k] = -1;
      m1.ref1[k] = -1;
    }
    return b_motion(addr, shape);
  }
  VTS_HD VTS_INLINE int mvd(int base, int sum) {  // U prefix cMax 9 + UEG3 + sign
    if (!dec(base + (sum < 3 ? 0 : (sum > 32 ? 2 : 1)))) return 0;
    int v = 1;
    while (v < 9 && dec(base + vts_min(v + 2, 6))) ++v;  // ctxIdxInc 3, 4, 5, 6, 6, ...
    if (v >= 9) {
      int k = 3;
      while (bypass()) {
        v += 1 << k;
        if (++k > 24) {
          err |= DEC_E_SYNTAX;
          return 0;
        }
      }
      while (k--) v += static_cast<int>(bypass()) << k;
    }
    return bypass() ? -v : v;
  }
  // residual_block_cabac (7.3.5.3.3): each level goes straight to its raster
  // position in dst, which the caller has zeroed (4x4 blocks: zig-zag position
  // of coefficient start + i; 8x8: the 8x8 zig-zag; chroma DC: list order);
  // count of non-zero levels (0: coded_block_flag 0), -1 on error.  kT8: an
  // 8x8 block (ctxBlockCat 5, contexts 402..459); else cat 0..4 (85..275)
  template <bool kT8>
  VTS_HD VTS_INLINE int residual_t(int cat, int cbf_inc, int maxNum, int16_t *dst, int start) {
    typedef typename std::conditional<kT8, uint64_t, uint32_t>::type Mask;
    if (!kT8 && !dec(85 + cbf_off(cat) + cbf_inc)) return 0;
    Mask sig = 0;
    int numc = maxNum;
    const int sig_base = kT8 ? 402 : 105 + sig_off(cat), last_base = kT8 ? 417 : 166 + sig_off(cat);
    for (int i = 0; i < numc - 1; ++i) {
      int inc_s, inc_l;
      if (kT8) {
        const uint32_t e = s8.get(static_cast<uint32_t>(i));
        inc_s = static_cast<int>(e & 255u);
        inc_l = static_cast<int>((e >> 8) & 255u);
      } else {
        inc_s = inc_l = cat == 3 ? vts_min(i, 2) : i;
      }
      if (dec(kT8 ? 402 + (inc_s & 15) : vts_min(sig_base + inc_s, 165))) {
        sig |= Mask(1) << i;
        if (dec(kT8 ? 417 + (inc_l & 15) : vts_min(last_base + inc_l, 226))) {
          numc = i + 1;
          break;
        }
      }
    }
    (void)sig_base;
    (void)last_base;
    sig |= Mask(1) << (numc - 1);
    int eq1 = 0, gt1 = 0, n = 0;
    const int base = kT8 ? 426 : 227 + abs_off(cat);
    while (sig) {  // the significant coefficients, highest first
      const int i = kT8 ? 63 - static_cast<int>(__builtin_clzll(static_cast<uint64_t>(sig)))
                        : 31 - static_cast<int>(__builtin_clz(static_cast<uint32_t>(sig)));
      sig &= ~(Mask(1) << i);
      int v = 0;
      if (dec(base + (gt1 ? 0 : vts_min(4, 1 + eq1)))) {
        v = 1;
        const int inc = 5 + vts_min(4 - (cat == 3 ? 1 : 0), gt1);
        while (v < 14 && dec(base + inc)) ++v;
        if (v >= 14) {  // UEG0 suffix
          int k = 0;
          while (bypass()) {
            v += 1 << k;
            if (++k > 24) return -1;
          }
          while (k--) v += static_cast<int>(bypass()) << k;
        }
      }
      int lvl = v + 1;
      if (bypass()) lvl = -lvl;
      if (lvl > 32767 || lvl < -32768) return -1;
      const int pos = kT8 ? static_cast<int>((s8.get(static_cast<uint32_t>(i)) >> 16) & 63u)
                          : (cat == 3 ? i : zz4(i + start));
      dst[pos] = static_cast<int16_t>(lvl);
      if (v == 0) ++eq1;
      else ++gt1;
      ++n;
    }
    return n;
  }

  // ------------------------------------------------------ macroblock_layer
  // (begin_mb done by the caller); returns false to stop the slice
  VTS_HD VTS_INLINE bool mb_cabac(int addr, int *qp) {
    VTS_PROF(2);
    MbRec &m = cur();
    int xw, yw;
    const int A = nb_mb(addr, -1, 0, 16, &xw, &yw), B = nb_mb(addr, 0, -1, 16, &xw, &yw);
    int itype, mb_type = 0;
    if (s->is_p == kSliceB) {
      const int t = b_type((A != -1 && !(rec1(A).direct & kDirect16) ? 1 : 0) +
                           (B != -1 && !(rec1(B).direct & kDirect16) ? 1 : 0));
      itype = t >= 23 ? t - 23 : -1;
      mb_type = t;
    } else if (s->is_p) {
      if (dec(14)) {
        itype = i_type(17, 0);
      } else {
        itype = -1;
        if (!dec(15)) mb_type = dec(16) ? 3 : 0;
        else mb_type = dec(17) ? 1 : 2;
      }
    } else {
      itype = i_type(0, (avail_not(A, kMbI4x4) ? 1 : 0) + (avail_not(B, kMbI4x4) ? 1 : 0));
    }
    if (itype == 25) {  // I_PCM: alignment, 384 samples through the RBSP reader, engine restart
      m.type = kMbPcm;
      m.qp = static_cast<uint8_t>(*qp);
      br.reset_at(cab_consumed());  // the engine's lookahead goes back to the bit reader
      br.align();
      for (int j = 0; j < 16; ++j) m.nz[j] = 16;
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
      m.blocks = 0;
      prev_qpd = false;
      cab_start();
      return !br.err;
    }
    int cbp = 0;
    bool small = false;
    if (itype == 0) {  // I_NxN
      m.type = kMbI4x4;
      bool t8 = false;
      if (P_t8mode) {
        const int inc = (A != -1 && (rec(A).modes & kModeT8) ? 1 : 0) + (B != -1 && (rec(B).modes & kModeT8) ? 1 : 0);
        t8 = dec(399 + inc) != 0;
      }
      const int nb = t8 ? 4 : 16;
      if (t8) m.modes = kModeT8;
      uint8_t *pflag = sc->prev, *rem = sc->rem;
      for (int i = 0; i < nb; ++i) {
        pflag[i] = static_cast<uint8_t>(dec(68));
        if (!pflag[i]) {
          uint32_t r = dec(69);
          r |= dec(69) << 1;
          r |= dec(69) << 2;
          rem[i] = static_cast<uint8_t>(r);
        }
      }
      for (int i = 0; i < nb; ++i) {
        const int x0 = t8 ? (i & 1) * 8 : blk_x(i) * 4, y0 = t8 ? (i >> 1) * 8 : blk_y(i) * 4;
        const int pm = mode_pred(addr, x0, y0, t8);
        const int mode = pflag[i] ? pm : (rem[i] < pm ? rem[i] : rem[i] + 1);
        const int r = (y0 / 4) * 4 + x0 / 4;
        set_i4(r, mode);
        if (t8) {
          set_i4(r + 1, mode);
          set_i4(r + 4, mode);
          set_i4(r + 5, mode);
        }
      }
    } else if (itype > 0) {  // I_16x16
      m.type = kMbI16;
      cbp = ((((itype - 1) / 4) % 3) << 4) | (itype >= 13 ? 15 : 0);
      m.modes = static_cast<uint8_t>((itype - 1) % 4);
    } else if (s->is_p == kSliceB) {  // Table 7-14
      m.type = kMbInter;
      VTS_PROF(3);
      if (!b_inter_cabac(addr, mb_type, &small)) return false;
    } else {  // inter (Table 7-13)
      VTS_PROF(3);
      m.type = kMbInter;
      const int nparts = mb_type == 0 ? 1 : (mb_type <= 2 ? 2 : 4);
      int8_t *sub = sc->sub, *refs = sc->refs;
      for (int k = 0; k < 4; ++k) sub[k] = refs[k] = 0;
      if (mb_type == 3)
        for (int k = 0; k < 4; ++k) {
          int v;
          if (dec(21)) v = 0;
          else if (!dec(22)) v = 1;
          else v = dec(23) ? 2 : 3;
          sub[k] = static_cast<int8_t>(v);
          if (v) small = true;
        }
      const int nref = s->num_ref;
      for (int k = 0; k < nparts; ++k) {
        const int x0 = (mb_type == 2 || mb_type == 3) ? 8 * (k & 1) : 0;
        const int y0 = mb_type == 1 ? 8 * k : (mb_type == 3 ? 8 * (k >> 1) : 0);
        int v = 0;
        if (nref > 1) v = ref_idx(addr, x0, y0, 0);
        if (v >= nref || s->ref_slot[v & 31] < 0) {
          err |= DEC_E_NO_REF;
          return false;
        }
        refs[k] = static_cast<int8_t>(v);
        // the partition's 8x8 quarters carry the index for later contexts
        const int pw = (mb_type == 0 || mb_type == 1) ? 2 : 1, ph = (mb_type == 0 || mb_type == 2) ? 2 : 1;
        for (int qy = 0; qy < ph; ++qy)
          for (int qx = 0; qx < pw; ++qx) m.ref[(y0 / 8 + qy) * 2 + x0 / 8 + qx] = static_cast<int8_t>(v);
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
          if (mb_type == 3) {
            if (sub[k] == 1) sy += 4 * q;
            else if (sub[k] == 2) sx += 4 * q;
            else if (sub[k] == 3) { sx += 4 * (q & 1); sy += 4 * (q >> 1); }
          }
          const int dx = mvd(40, mvd_at(addr, sx - 1, sy, 0) + mvd_at(addr, sx, sy - 1, 0));
          const int dy = mvd(47, mvd_at(addr, sx - 1, sy, 1) + mvd_at(addr, sx, sy - 1, 1));
          int px, py;
          mv_pred(addr, sx, sy, pw, ph, refs[k], done, &px, &py);
          const int vx = px + dx, vy = py + dy;
          if (vx < -32768 || vx > 32767 || vy < -32768 || vy > 32767) {
            err |= DEC_E_SYNTAX;
            return false;
          }
          const uint8_t ax = static_cast<uint8_t>(vts_min(dx < 0 ? -dx : dx, 33));
          const uint8_t ay = static_cast<uint8_t>(vts_min(dy < 0 ? -dy : dy, 33));
          const uint32_t bm = blk_mask(sx, sy, pw, ph);
          const int rk = refs[k];
          VTS_LANES(16, b) if ((bm >> b) & 1u) {
            set_motion(b, rk, vx, vy);
            sc->mvx[0][1 + (b >> 2)][1 + (b & 3)][0] = ax;
            sc->mvx[0][1 + (b >> 2)][1 + (b & 3)][1] = ay;
          }
          done |= bm;
        }
      }
    }
    VTS_PROF(2);
    if (m.type == kMbI4x4 || m.type == kMbI16) {  // intra_chroma_pred_mode, TU cMax 3
      int inc = 0;
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const int n = nb ? B : A;
        if (n == -1) continue;
        const MbRec &r = rec(n);
        inc += ((r.type == kMbI4x4 || r.type == kMbI16) && ((r.modes >> 2) & 3)) ? 1 : 0;
      }
      int cm = 0;
      if (dec(64 + inc)) {
        cm = 1;
        if (dec(67)) {
          cm = 2;
          if (dec(67)) cm = 3;
        }
      }
      m.modes = static_cast<uint8_t>(m.modes | (cm << 2));
    }
    VTS_PROF(4);
    if (m.type != kMbI16) {  // coded_block_pattern (9.3.3.1.1.4)
      for (int b8 = 0; b8 < 4; ++b8) {
        const int bx = (b8 & 1) * 8, by = (b8 >> 1) * 8;
        int cond[2];
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
          int x2 = 0, y2 = 0;
          const int n = nb_mb(addr, nb ? bx : bx - 1, nb ? by - 1 : by, 16, &x2, &y2);
          const int b8n = (y2 / 8) * 2 + x2 / 8;
          if (n == -1) cond[nb] = 0;
          else if (n == -2) cond[nb] = ((cbp >> b8n) & 1) ? 0 : 1;
          else {
            const MbRec &r = rec(n);
            cond[nb] = r.type == kMbPcm ? 0 : (r.type == kMbSkip ? 1 : (((r.cbp >> b8n) & 1) ? 0 : 1));
          }
        }
        cbp |= static_cast<int>(dec(73 + cond[0] + 2 * cond[1])) << b8;
      }
      int ca[2] = {0, 0}, c2[2] = {0, 0};
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const int n = nb ? B : A;
        if (n == -1) continue;
        const MbRec &r = rec(n);
        const int cc = r.type == kMbPcm ? 2 : (r.type == kMbSkip ? 0 : r.cbp >> 4);
        ca[nb] = cc != 0;
        c2[nb] = cc == 2;
      }
      if (dec(77 + ca[0] + 2 * ca[1])) cbp |= (1 + static_cast<int>(dec(81 + c2[0] + 2 * c2[1]))) << 4;
    }
    m.cbp = static_cast<uint8_t>(cbp);
    if (m.type == kMbInter && (cbp & 15) && P_t8mode && !small) {
      const int inc = (A != -1 && (rec(A).modes & kModeT8) ? 1 : 0) + (B != -1 && (rec(B).modes & kModeT8) ? 1 : 0);
      if (dec(399 + inc)) m.modes = static_cast<uint8_t>(m.modes | kModeT8);
    }
    bool qpd = false;
    if (cbp || m.type == kMbI16) {  // mb_qp_delta: U of the se() mapping
      int k = 0;
      if (dec(60 + (prev_qpd ? 1 : 0))) {
        k = 1;
        if (dec(62)) {
          k = 2;
          while (dec(63))
            if (++k > 104) {
              err |= DEC_E_SYNTAX;
              return false;
            }
        }
      }
      const int dq = (k & 1) ? (k + 1) / 2 : -(k / 2);
      if (dq < -26 || dq > 25) {
        err |= DEC_E_SYNTAX;
        return false;
      }
      *qp = (*qp + dq + 52) % 52;
      qpd = dq != 0;
    }
    prev_qpd = qpd;
    m.qp = static_cast<uint8_t>(*qp);
    // ---- residual (7.3.5.3), blocks in bitstream order
    const bool intra = m.type == kMbI4x4 || m.type == kMbI16;
    const bool t8 = (m.modes & kModeT8) != 0;
    // the blocks present, in bitstream order = kBlk* bit order; an 8x8 block
    // is its quarter's first 4x4 bit.  One residual() site for all of them.
    // condTermFlagN (9.3.3.1.1.9) of the luma 4x4 blocks on the macroblock's
    // left / top edge, from the neighbours' records once: bits 0-3 = A of
    // rows 0-3, bits 4-7 = B of columns 0-3; inside the macroblock the
    // neighbour's flag is its coded_block_flag (cbfc)
    uint32_t nbl = 0, cbfc = 0;
    if ((cbp & 15) && !t8) {
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const int n = nb ? B : A;
        uint32_t f = 0;
        if (n == -1) {
          f = intra ? 15u : 0u;
        } else {
          const MbRec &r = rec(n);
          if (r.type == kMbPcm) {
            f = 15u;
          } else if (r.type != kMbSkip) {
            const uint32_t cb = cbf_of(r);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              // A: row k, right column (raster 4k + 3) in 8x8 (k / 2) * 2 + 1;
              // B: column k, bottom row (raster 12 + k) in 8x8 2 + k / 2
              const int b8 = nb ? 2 + (k >> 1) : (k >> 1) * 2 + 1, rr = nb ? 12 + k : 4 * k + 3;
              f |= (((r.cbp >> b8) & 1) ? (cb >> (1 + rr)) & 1u : 0u) << k;
            }
          }
        }
        nbl |= f << (4 * nb);
      }
    }
    uint32_t todo = m.type == kMbI16 ? 1u << kBlkI16Dc : 0u;
    for (int q = 0; q < 4; ++q)
      if ((cbp >> q) & 1) todo |= (t8 ? 1u : 15u) << (kBlkLuma0 + 4 * q);
    if (cbp >> 4) todo |= 3u << kBlkChromaDc0;
    if ((cbp >> 4) == 2) todo |= 255u << kBlkChromaAc0;
    VTS_PROF(5);
    while (todo) {
      const uint32_t bt = static_cast<uint32_t>(__builtin_ctz(todo));
      todo &= todo - 1u;
      int cat, inc = 0, maxNum = 16, start = 0, r = 0;
      int16_t *dst = sc->blk;
      if (bt == kBlkI16Dc) {
        cat = 0;
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
          const int n = nb ? B : A;
          inc += cbf_cond(n, true, n != -1 && rec(n).type == kMbI16, 0) << nb;
        }
      } else if (bt < kBlkChromaDc0) {
        const int k = static_cast<int>(bt) - kBlkLuma0, bx = blk_x(k), by = blk_y(k);
        r = by * 4 + bx;
        if (t8) {
          cat = 5;
          maxNum = 64;
          dst = sc->blk8;
        } else {
          cat = m.type == kMbI16 ? 1 : 2;
          if (cat == 1) {
            maxNum = 15;
            start = 1;
          }
          const uint32_t ca = bx ? (cbfc >> (r - 1)) & 1u : (nbl >> by) & 1u;
          const uint32_t cb = by ? (cbfc >> (r - 4)) & 1u : (nbl >> (4 + bx)) & 1u;
          inc = static_cast<int>(ca + 2 * cb);
        }
      } else if (bt < kBlkChromaAc0) {
        cat = 3;
        maxNum = 4;
        inc = cbf_chroma_inc(addr, static_cast<int>(bt) - kBlkChromaDc0, 0, true, intra);
      } else {
        const int j = static_cast<int>(bt) - kBlkChromaAc0;
        cat = 4;
        maxNum = 15;
        start = 1;
        inc = cbf_chroma_inc(addr, j >> 2, j & 3, false, intra);
      }
      zero16x(dst, cat == 5 ? 64 : 16);
      const int nc = cat == 5 ? residual_t<true>(5, 0, 64, dst, 0) : residual_t<false>(cat, inc, maxNum, dst, start);
      if (nc < 0) { err |= DEC_E_SYNTAX; return false; }
      if (cat == 5) {  // the quarter's 4 blocks: raster 8x8 rows 2j, 2j + 1
        const int rs[4] = {r, r + 1, r + 4, r + 5};
        for (int j = 0; j < 4; ++j) {
          m.nz[rs[j]] = static_cast<uint8_t>(nc > 255 ? 255 : nc);
          set_cbf(1u + static_cast<uint32_t>(rs[j]));
        }
        if (nc)
          for (int j = 0; j < 4; ++j)
            if (!store_block(bt + j, sc->blk8 + 16 * j)) { err |= DEC_E_SYNTAX; return false; }
        continue;
      }
      if (cat == 1 || cat == 2) {
        m.nz[r] = static_cast<uint8_t>(nc);
        cbfc |= (nc ? 1u : 0u) << r;
      }
      if (nc) {
        set_cbf(bt == kBlkI16Dc ? 0u : (cat <= 2 ? 1u + static_cast<uint32_t>(r) : bt));
        if (!store_block(bt)) { err |= DEC_E_SYNTAX; return false; }
      }
    }
    VTS_PROF(6);
    if (br.err || cab_consumed() > 8 * br.size) {
      err |= DEC_E_SYNTAX;
      return false;
    }
    return true;
  }

  // after a macroblock: its clamped |mvd| for the neighbours below / right
  VTS_HD VTS_INLINE void finish_mvd() {
    MbRec &m = cur();
    if (m.type == kMbInter)
      for (int x = 0; x < 4; ++x) {
        m.i4[2 * x] = sc->mvx[0][4][1 + x][0];
        m.i4[2 * x + 1] = sc->mvx[0][4][1 + x][1];
      }
    if (bframes) {
      MbRecB &m1 = cur1();
      for (int x = 0; x < 4; ++x) {
        m1.mvd1[2 * x] = sc->mvx[1][4][1 + x][0];
        m1.mvd1[2 * x + 1] = sc->mvx[1][4][1 + x][1];
      }
    }
  }

  bool P_t8mode;
};

// Parse CABAC slice `s` (window slice index si) from its RBSP (rbsp_len
// bytes, emulation-prevention bytes removed).  Returns DEC_E_* bits.
VTS_HD VTS_INLINE uint32_t parse_slice_cabac(const uint8_t *rbsp, int32_t rbsp_len, const FullSlice &s, uint32_t si,
                                         const FullParams P, MbRec *frame_recs, uint16_t *frame_ilvl, int16_t *arena,
                                         uint32_t epoch, FullScratch *sc, const BCtx &bc) {
  CabacParser p;
  p.bc = bc;
  p.bframes = P.bframes;
  p.direct8x8 = P.direct8x8;
  if (s.is_p == kSliceB && (!bc.x || !bc.col || !P.bframes)) return DEC_E_NO_REF;
  p.s = &s;
  p.cip = P.cip;
  p.P_t8mode = P.t8mode != 0;
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
  p.cur_addr = -2;
  p.cs = 0;
  p.tslots = 0;
  p.lvl_prev = kNoLevel;
  p.pf_col = -1;
#if defined(__HIP_DEVICE_COMPILE__)
  p.pf_col2 = -1;
#endif
  p.todo = 0;
  p.cur_i16 = false;
  p.prev_qpd = false;
  const int nmb = P.mb_width * P.mb_height;
  // the RBSP stop bit, past any trailing cabac_zero_words (zero bytes once
  // their emulation-prevention bytes are gone)
  int32_t last = rbsp_len - 1;
  while (last >= 0 && rbsp[last] == 0) --last;
  if (last < 0) return DEC_E_SYNTAX;
  const int64_t stop_bit = int64_t(last) * 8 + (7 - __builtin_ctz(static_cast<uint32_t>(rbsp[last])));
  p.br.init(rbsp, rbsp_len, sc->cache);
  p.refresh_lane();
  p.br.reset_at(s.data_bit);
  // cabac_alignment_one_bit
  while (p.br.consumed() & 7)
    if (!p.br.bit()) return DEC_E_SYNTAX;
  VTS_PROF_START(p);
  p.cab_tables();
  p.cab_init(!s.is_p, s.qp);
  p.cab_start();
  int addr = s.first_mb, qp = s.qp;
  for (;;) {
    if (addr >= nmb) {
      p.err |= DEC_E_SYNTAX;
      break;
    }
    p.refresh_lane();
    VTS_PROF_P(p, 1);
    p.begin_mb(addr);
    VTS_PROF_P(p, 2);
    bool ok = true, skip = false;
    if (s.is_p) {
      int xw, yw;
      const int A = p.nb_mb(addr, -1, 0, 16, &xw, &yw), B = p.nb_mb(addr, 0, -1, 16, &xw, &yw);
      p.mvd_border(A, B);
      p.ref_border(A, B);
      p.mv_border(addr);
      skip = p.dec((s.is_p == kSliceB ? 24 : 11) + (p.avail_not(A, kMbSkip) ? 1 : 0) +
                   (p.avail_not(B, kMbSkip) ? 1 : 0)) != 0;
    }
    if (skip) {
      VTS_PARSE_TRACE(s.is_p == kSliceB ? 4 : 5);
      VTS_PROF_P(p, 3);
      if (s.is_p == kSliceB) p.b_skip_body(addr, qp);
      else p.skip_body(addr, qp);
      p.prev_qpd = false;
    } else {
      ok = p.mb_cabac(addr, &qp);  // one inlined copy for every slice type
    }
    if (!ok || p.err) break;
    VTS_PROF_P(p, 6);
    p.finish_mvd();
    p.end_mb(addr);
    ++addr;
    if (p.term()) break;  // end_of_slice_flag
  }
  VTS_PROF_P(p, 7);
  VTS_PROF_FLUSH(p);
  // the arithmetic decoder has read through the stop bit
  if (!p.err && (p.br.err || p.cab_consumed() != stop_bit + 1)) p.err |= DEC_E_SYNTAX;
  return p.err;
}

}  // namespace full
}  // namespace vts
