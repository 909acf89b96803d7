// parse_cabac.h — CABAC slice_data() SYNTAX parser of the general device
// decoder (ITU-T H.264 9.3): High-profile I, P and B slices with 8x8
// transforms.  The kernel (h264_parse_full_cabac) runs one slice per wave;
// the whole arithmetic decoder is wave-uniform scalar code, and the CPU
// harness compiles the same header.
//
// The serial per-slice wave decodes bins and nothing else: the syntax
// elements, the coefficient blocks, and the few neighbour facts CABAC's
// context selection reads (9.3.3.1.1: mb types, cbp, coded_block_flag bits,
// |mvd|, refIdx > 0, transform / chroma-mode flags of the macroblocks to the
// left and above).  Those facts cross macroblock edges as 20-byte SynEdge
// records in LDS: the left one from the previous macroblock, the top ones in
// a per-column row of the wave's LDS that the slice itself fills — no record
// of another macroblock is ever read back from global memory.  Everything
// the standard derives from syntax plus decoded neighbours — motion-vector
// prediction (8.4.1.3), P_Skip (8.4.1.1), direct prediction (8.4.1.2),
// Intra4x4 / 8x8 prediction modes (8.3.1.1 / 8.3.2.1), reference slots, the
// intra dependency level — is left to the per-picture wavefront kernel
// h264_derive (derive_full.h), so a B slice no longer waits for its
// colocated picture's parse either.
//
// What the parse writes per macroblock, in the MbRec / MbRecB layout that
// h264_derive completes in place (the "syntax record"):
//   type, qp, cbp, modes, coef / blocks, nz, nzc (coded_block_flag bits) —
//     final;
//   ref[4] / ref1[4]: ref_idx_l0 / l1 per 8x8 quadrant as coded (-1 where the
//     partition does not use the list; direct quadrants -1); direct (MbRecB);
//   mv[16] / mv1[16]: mvd_l0 / l1 of the (sub-)partition covering each 4x4
//     block (0 for skipped / direct / intra blocks);
//   i4[8]: I_NxN — per 4x4 block (Intra_8x8: at the 8x8's top-left 4x4) the
//     nibble 8 | 0 for prev_intra_pred_mode_flag = 1, else rem_intra_pred_mode;
//     inter — i4[0] the partition shape (0 16x16, 1 16x8, 2 8x16, 3 8x8),
//     i4[1] the partitions' prediction (2 bits each: 0 direct, 1 L0, 2 L1,
//     3 Bi), i4[2] the sub-partition shapes (2 bits per 8x8: 0 8x8, 1 8x4,
//     2 4x8, 3 4x4).
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
// (CABAC B parse -4 % same-box, profiles/r03_cabac_vgpr_engine_ab.txt)
#if defined(__HIP_DEVICE_COMPILE__)
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

// ------------------------------------------------------- neighbour facts
// What the macroblock to the right (its left edge) or below (its top edge)
// reads of a macroblock for context selection, as bit fields of SynEdge::f.
// "Along the edge" = the 4x4 blocks / 8x8 quadrants touching it: the right
// column (raster 3, 7, 11, 15; quadrants 1, 3; chroma blocks 1, 3) or the
// bottom row (raster 12..15; quadrants 2, 3; chroma blocks 2, 3), index k in
// order.  I_PCM is stored as cbp luma 15 / chroma 2 and every
// coded_block_flag set, which gives exactly the standard's I_PCM rules below.
enum : uint32_t {
  kEType = 7u,          // bits 0-2: kMb* type
  kECbpSh = 3,          // bits 3-8: coded_block_pattern
  kET8 = 1u << 9,       // transform_size_8x8_flag
  kEChroma = 1u << 10,  // I_NxN / Intra_16x16 with intra_chroma_pred_mode != 0
  kEDirect16 = 1u << 11,  // B_Skip / B_Direct_16x16
  kERefSh = 12,         // bits 12 + 2 l + k: refIdxLX > 0 of edge quadrant k (explicitly coded only)
  kECbfSh = 16,         // bits 16 + k: luma 4x4 coded_block_flag along the edge
  kECbfDc = 1u << 20,   // Intra16x16DCLevel coded_block_flag
  kECdcSh = 21,         // bits 21 + iCbCr: chroma DC coded_block_flag
  kECacSh = 23,         // bits 23 + 2 iCbCr + k: chroma AC coded_block_flag along the edge
};
struct SynEdge {
  uint32_t f;
  uint8_t mvd[2][4][2];  // Min(|mvd_lX|, 33) of the edge's 4x4 blocks [list][k][component]
};
static_assert(sizeof(SynEdge) == 20, "SynEdge layout");

// Per-wave scratch (LDS on the device); SynEdge top[mb_width] follows it.
struct SynScratch {
  MbRec m;                      // the macroblock being parsed (its syntax record)
  MbRecB m1;                    // ... its list-1 half (streams with B slices)
  alignas(16) int16_t blk[16];  // coefficient block being decoded (raster)
  alignas(16) int16_t blk8[64]; // 8x8 block being decoded (raster)
  uint32_t cache[kCacheWords];  // bit reader
  // Min(|mvd_lX|, 33) around the current macroblock, per list: [row][col],
  // row 0 = the bottom row of the macroblock above, col 0 = the right column
  // of the one to the left (0 where unavailable / not coded), rows and cols
  // 1..4 = the current macroblock's 4x4 blocks
  uint8_t mvx[2][5][5][2];
  SynEdge left;                 // the previous macroblock's right edge
};
VTS_HD VTS_INLINE size_t syn_lds_bytes(int mb_width) {
  return (sizeof(SynScratch) + 15) / 16 * 16 + sizeof(SynEdge) * static_cast<size_t>(mb_width);
}

struct CabacSyn {
  RbspBitsT<kCacheWords> br;
  const FullSlice *s;     // global (the ref_slot table is indexed at run time)
  const SliceExt *x;      // B slices: the slice's SliceExt
  MbRec *recs;            // the frame's records (global)
  MbRecB *recs1;          // ... list-1 halves (streams with B slices), else null
  int16_t *arena;         // window coefficient arena, 16 int16 per block
  SynScratch *sc;
  SynEdge *top;           // per macroblock column: the bottom edge of the slice's last macroblock there
  uint32_t *arena_top;    // the window's counter of blocks handed out (kArenaChunk at a time)
  uint32_t arena_blocks;  // the window arena's capacity in blocks
  uint32_t blk_at, blk_end;  // the slice's current chunk: next free block, end
  uint32_t slice_index;
  uint32_t epoch;
  int mbw;
  int first_mb;
  uint32_t err;
  bool bframes;           // write the list-1 halves
  bool direct8x8;         // direct_8x8_inference_flag
  bool t8mode;            // transform_8x8_mode_flag
  bool prev_qpd;          // the previous macroblock of the slice has mb_qp_delta != 0
  // the current macroblock's neighbours A (left) and B (above): their edge
  // facts (0 when unavailable) and availability
  uint32_t fa, fb;
  bool av_a, av_b;
  // The engine (9.3.1.2, 9.3.3.2) with codIOffset scaled: val holds the 9-bit
  // codIOffset in bits 31..23 and the next `la` bitstream bits below it, so
  // renormalisation is a shift of val and the bit reader is touched once per
  // 16 bits (la < 8 -> 16 more), not per bin.  codIOffset >= codIRange is
  // val >= codIRange << 23.
  uint32_t range, val;
  int32_t la;
  // context states (pStateIdx << 1 | valMPS), four per dword.  The residual
  // contexts of 4x4 blocks (ctxIdx 85..275) fill st[0] (slot c - 85); all
  // others (0..84, and 399..459 at 85..145) st[1], so every decode's table is
  // known at compile time (slot q: lane q >> 2, byte q & 3)
  LaneTab st[2];
  LaneTab lps, trn, s8;  // kCabLanes
#if defined(__HIP_DEVICE_COMPILE__)
  // the lane index, re-read opaquely at every macroblock (refresh_lane): what
  // derives from it is computed per macroblock instead of hoisted out of the
  // macroblock loop and spilled
  int lane_;
  __device__ VTS_INLINE void refresh_lane() {
    lane_ = static_cast<int>(threadIdx.x);
    asm volatile("" : "+v"(lane_));
  }
#else
  void refresh_lane() {}
#endif
  static VTS_HD VTS_INLINE int ctx_tab(int c) { return (c >= 85 && c <= 275) ? 0 : 1; }
  static VTS_HD VTS_INLINE int ctx_slot(int c) { return c >= 399 ? c - 314 : (c >= 85 ? c - 85 : c); }

  // ---------------------------------------------- arithmetic decoder (9.3.3.2)
  VTS_HD VTS_INLINE void cab_start() {  // 9.3.1.2: codIOffset = read_bits(9)
    range = VTS_EV(510u);
    val = VTS_EV(br.bits(32));
    la = 23;
  }
  // bits the engine has consumed (9.3.1.2's 9 + every renormalisation shift)
  VTS_HD VTS_INLINE int32_t cab_consumed() const { return br.consumed() - la; }
  VTS_HD VTS_INLINE void cab_fill() {
    if (VTS_UNLIKELY(la < 8)) {
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
  // DecodeDecision on slot q of lane table kTab (ctx_slot / ctx_tab): the
  // table known at compile time, so only its lane is read and written
  template <int kTab>
  VTS_HD VTS_INLINE uint32_t dec_slot(uint32_t q) {
    VTS_PARSE_TRACE(1);
    const uint32_t ln = (q >> 2) & 63u, sh = (q & 3u) * 8u;
    const uint32_t word = st[kTab].get(ln);
    const uint32_t s = (word >> sh) & 127u, ps = s >> 1, mps = s & 1u;
    const uint32_t lpsr = (lps.get(ps) >> ((range >> 3) & 24u)) & 255u;
    const uint32_t tw = trn.get(ps);  // read on both paths: no branch
    range -= lpsr;
    const uint32_t rs = range << 23;
    // (the LPS test as a scalar condition from the compare's lane mask, with
    // bin and next state on the scalar unit: all-intra / content parse -2 %,
    // noise +5 %: the scalar unit is what many parse waves share;
    // profiles/r06o_cabac_uniform_decision_ab.json.  One state per dword in
    // six lane tables, no byte fields: bit-exact on the CPU harness, the
    // device parse of the real clip desynchronised; not kept)
    const bool lpsb = val >= rs;
    const uint32_t bin = mps ^ (lpsb ? 1u : 0u);
    const uint32_t ns = VTS_EU(((tw >> (lpsb ? 0u : 8u)) & 127u) ^ mps);
    val -= lpsb ? rs : 0u;
    range = lpsb ? lpsr : range;
    st[kTab].set(ln, (word & ~(255u << sh)) | (ns << sh));
    const int n = static_cast<int>(VTS_EU(__builtin_clz(range) - 23));  // RenormD as one shift (0..6)
    range <<= n;
    val <<= n;
    la -= n;
    cab_fill();
    VTS_PARSE_TRACE(10);
    return VTS_EU(bin);
  }
  VTS_HD VTS_INLINE uint32_t dec(int ctx) {  // DecodeDecision
    // which of the two lane tables: folded where it is a constant (every call
    // site but the residual loops, which call dec_slot), else both are read
    // and written with selects (no branch)
    if (__builtin_constant_p(ctx_tab(ctx)))
      return ctx_tab(ctx) ? dec_slot<1>(static_cast<uint32_t>(ctx_slot(ctx)))
                          : dec_slot<0>(static_cast<uint32_t>(ctx_slot(ctx)));
    VTS_PARSE_TRACE(1);
    const int q = ctx_slot(ctx);
    const uint32_t ln = static_cast<uint32_t>(q >> 2) & 63u, sh = static_cast<uint32_t>(q & 3) * 8u;
    const bool hi = ctx_tab(ctx) != 0;
    const uint32_t wa = st[0].get(ln), wb = st[1].get(ln);
    const uint32_t word = hi ? wb : wa;
    const uint32_t s = (word >> sh) & 127u, ps = s >> 1, mps = s & 1u;
    const uint32_t lpsr = (lps.get(ps) >> ((range >> 3) & 24u)) & 255u;
    const uint32_t tw = trn.get(ps);
    range -= lpsr;
    const uint32_t rs = range << 23;
    const bool lpsb = val >= rs;
    const uint32_t bin = mps ^ (lpsb ? 1u : 0u);
    const uint32_t ns = VTS_EU(((tw >> (lpsb ? 0u : 8u)) & 127u) ^ mps);
    val -= lpsb ? rs : 0u;
    range = lpsb ? lpsr : range;
    const uint32_t nw = (word & ~(255u << sh)) | (ns << sh);
    st[0].set(ln, hi ? wa : nw);
    st[1].set(ln, hi ? nw : wb);
    const int n = static_cast<int>(VTS_EU(__builtin_clz(range) - 23));
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
    const uint32_t top_bit = val >> 31;
    val <<= 1;
    --la;
    cab_fill();
    const uint32_t rs = range << 23;
    const uint32_t b = VTS_EU((top_bit || val >= rs) ? 1u : 0u);  // no branch: the bin selects
    val -= b ? rs : 0u;
    VTS_PARSE_TRACE(11);
    return b;
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

  // ------------------------------------------------------ macroblock frame
  VTS_HD VTS_INLINE MbRec &cur() const { return sc->m; }
  VTS_HD VTS_INLINE MbRecB &cur1() const { return sc->m1; }
  VTS_HD VTS_INLINE static int etype(uint32_t f) { return static_cast<int>(f & kEType); }
  VTS_HD VTS_INLINE static int ecbp(uint32_t f) { return static_cast<int>((f >> kECbpSh) & 63u); }

  // a new macroblock: its neighbours' availability and edge facts
  VTS_HD VTS_INLINE void begin_mb(int addr) {
    VTS_PARSE_TRACE(0);
    const int xcol = addr % mbw;
    av_a = xcol > 0 && addr - 1 >= first_mb;
    av_b = addr - mbw >= first_mb;
    fa = av_a ? sc->left.f : 0u;
    fb = av_b ? top[xcol].f : 0u;
  }
  // a skipped macroblock (P_Skip / B_Skip): its record and both edges are
  // constants but for the QP, so they go out from registers, one 16-byte
  // piece (record) or dword (edges) per lane, without a record image
  VTS_HD VTS_INLINE void emit_skip(int addr, int qp, bool is_b) {
    const uint32_t w4 = kMbSkip | (static_cast<uint32_t>(qp) << 8);
    const uint32_t ef = kMbSkip | (is_b ? kEDirect16 : 0u);
    SynEdge *te = &top[addr % mbw];
    (void)w4;
#if defined(__HIP_DEVICE_COMPILE__)
    VTS_LANES(26, l) {
      if (l < 16) {
        u32x4 v = {0u, 0u, 0u, 0u};
        if (l == 0) v = u32x4{epoch, slice_index, 0u, 0u};
        else if (l == 1) v = u32x4{w4, ~0u, ~0u, ~0u};
        else if (l == 2) v = u32x4{0x22222222u, 0x22222222u, 0u, 0u};
        else if (l == 8) v = u32x4{~0u, ~0u, ~0u, is_b ? 0x1fu : 0u};
        if (l < 8) reinterpret_cast<u32x4 *>(&recs[addr])[l] = v;
        else if (bframes && (l < 10 || l >= 12)) reinterpret_cast<u32x4 *>(&recs1[addr])[l - 8] = v;
      } else {
        // the edges: dword 0 the flags, 1..4 the (zero) |mvd| bytes
        const int e = l - 16, k = e % 5;
        uint32_t *dst = reinterpret_cast<uint32_t *>(e < 5 ? &sc->left : te);
        dst[k] = k == 0 ? ef : 0u;
      }
    }
#else
    MbRec m{};
    m.epoch = epoch;
    m.slice = slice_index;
    m.type = kMbSkip;
    m.qp = static_cast<uint8_t>(qp);
    for (int i = 0; i < 4; ++i) {
      m.ref[i] = -1;
      m.ref_slot[i] = -1;
    }
    for (int i = 0; i < 8; ++i) m.i4[i] = 0x22;
    recs[addr] = m;
    if (bframes) {
      MbRecB m1{};
      for (int i = 0; i < 4; ++i) {
        m1.ref1[i] = -1;
        m1.ref_slot1[i] = -1;
      }
      m1.direct = is_b ? 0x0f | kDirect16 : 0;
      recs1[addr] = m1;
    }
    SynEdge e{};
    e.f = ef;
    sc->left = e;
    *te = e;
#endif
  }
  // a coded macroblock: the record image reset, the |mvd| grid's borders from
  // the neighbours' edges (one cell per lane)
  VTS_HD VTS_INLINE void init_mb(int addr) {
    VTS_PARSE_TRACE(9);
    const int xcol = addr % mbw;
#if defined(__HIP_DEVICE_COMPILE__)
    // the record's initial dwords, one per lane: epoch, slice, 0 coef / blocks
    // / type..modes, ref -1, ref_slot -1, i4 DC (2), then zeros; list 1: ref1
    // -1, ref_slot1 -1, then zeros
    VTS_LANES(64, l) {
      if (l < 32) {
        const uint32_t v = l == 0 ? epoch : (l == 1 ? slice_index : ((l >= 5 && l <= 7) ? ~0u : ((l == 8 || l == 9) ? 0x22222222u : 0u)));
        reinterpret_cast<uint32_t *>(&cur())[l] = v;
      } else if (bframes) {
        reinterpret_cast<uint32_t *>(&cur1())[l - 32] = l - 32 < 3 ? ~0u : 0u;
      }
    }
    const SynEdge *te = &top[xcol];
    VTS_LANES(50, i) {
      const int l = i / 25, r = (i % 25) / 5, c = i % 5;
      uint8_t v0 = 0, v1 = 0;
      if (r > 0 && c == 0 && av_a) {
        v0 = sc->left.mvd[l][r - 1][0];
        v1 = sc->left.mvd[l][r - 1][1];
      } else if (r == 0 && c > 0 && av_b) {
        v0 = te->mvd[l][c - 1][0];
        v1 = te->mvd[l][c - 1][1];
      }
      sc->mvx[l][r][c][0] = v0;
      sc->mvx[l][r][c][1] = v1;
    }
#else
    MbRec &m = cur();
    m.epoch = epoch;
    m.slice = slice_index;
    m.coef = 0;
    m.blocks = 0;
    m.type = 0;
    m.qp = 0;
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
    if (bframes) {
      MbRecB &m1 = cur1();
      for (int i = 0; i < 4; ++i) {
        m1.ref1[i] = -1;
        m1.ref_slot1[i] = -1;
      }
      m1.direct = 0;
      for (int i = 0; i < 3; ++i) m1._p[i] = 0;
      for (int i = 0; i < 8; ++i) m1.mvd1[i] = 0;
      for (int i = 0; i < 40; ++i) m1._q[i] = 0;
      for (int i = 0; i < 16; ++i) m1.mv1[i][0] = m1.mv1[i][1] = 0;
    }
    for (int l = 0; l < 2; ++l)
      for (int r = 0; r < 5; ++r)
        for (int c = 0; c < 5; ++c)
          for (int k = 0; k < 2; ++k) {
            uint8_t v = 0;
            if (r > 0 && c == 0 && av_a) v = sc->left.mvd[l][r - 1][k];
            else if (r == 0 && c > 0 && av_b) v = top[xcol].mvd[l][c - 1][k];
            sc->mvx[l][r][c][k] = v;
          }
#endif
  }

  // the current macroblock's edge flags (right: true = its right edge for
  // the next macroblock, false = its bottom edge for the one below)
  VTS_HD VTS_INLINE uint32_t edge_flags(bool right) const {
    const MbRec &m = cur();
    const int ty = m.type;
    uint32_t f = static_cast<uint32_t>(ty);
    const bool pcm = ty == kMbPcm;
    const uint32_t cbp = pcm ? 0x2fu : m.cbp;
    f |= cbp << kECbpSh;
    if (m.modes & kModeT8) f |= kET8;
    if ((ty == kMbI4x4 || ty == kMbI16) && ((m.modes >> 2) & 3)) f |= kEChroma;
    const uint8_t dir = bframes ? cur1().direct : 0;
    if (dir & kDirect16) f |= kEDirect16;
    const uint32_t cbf = static_cast<uint32_t>(m.nzc[0]) | (static_cast<uint32_t>(m.nzc[1]) << 8) |
                         (static_cast<uint32_t>(m.nzc[2]) << 16) | (static_cast<uint32_t>(m.nzc[3]) << 24);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int rr = right ? 4 * k + 3 : 12 + k;  // raster luma block along the edge
      if (pcm || ((cbf >> (1 + rr)) & 1u)) f |= 1u << (kECbfSh + k);
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int p8 = right ? 2 * k + 1 : 2 + k;
      if (ty == kMbInter && !((dir >> p8) & 1)) {
        if (m.ref[p8] > 0) f |= 1u << (kERefSh + k);
        if (bframes && cur1().ref1[p8] > 0) f |= 1u << (kERefSh + 2 + k);
      }
      const int cb = right ? 2 * k + 1 : 2 + k;  // chroma 4x4 block along the edge
#pragma unroll
      for (int pl = 0; pl < 2; ++pl)
        if (pcm || ((cbf >> (kBlkChromaAc0 + 4 * pl + cb)) & 1u)) f |= 1u << (kECacSh + 2 * pl + k);
    }
    if (pcm || (cbf & 1u)) f |= kECbfDc;
#pragma unroll
    for (int pl = 0; pl < 2; ++pl)
      if (pcm || ((cbf >> (kBlkChromaDc0 + pl)) & 1u)) f |= 1u << (kECdcSh + pl);
    return f;
  }
  // after a coded macroblock: its record to global memory (16 bytes per
  // lane), its edges for the neighbours to the right and below (the flags
  // scalar, the |mvd| bytes one per lane)
  VTS_HD VTS_INLINE void end_mb(int addr) {
    VTS_PARSE_TRACE(8);
    const uint32_t fr = edge_flags(true), fbm = edge_flags(false);
    SynEdge *te = &top[addr % mbw];
#if defined(__HIP_DEVICE_COMPILE__)
    VTS_LANES(64, l) {
      if (l < 16) {
        if (l < 8) reinterpret_cast<u32x4 *>(&recs[addr])[l] = reinterpret_cast<const u32x4 *>(&cur())[l];
        else if (bframes && (l < 10 || l >= 12))
          reinterpret_cast<u32x4 *>(&recs1[addr])[l - 8] = reinterpret_cast<const u32x4 *>(&cur1())[l - 8];
      } else if (l < 48) {
        // byte (list, k, component) of the right (lanes 16..31) / bottom (32..47) edge
        const int e = l - 16, bot = e >> 4, li = (e >> 3) & 1, k = (e >> 1) & 3, cc = e & 1;
        const uint8_t v = bot ? sc->mvx[li][4][1 + k][cc] : sc->mvx[li][1 + k][4][cc];
        (bot ? te : &sc->left)->mvd[li][k][cc] = v;
      }
    }
#else
    recs[addr] = cur();
    if (bframes) recs1[addr] = cur1();
    for (int li = 0; li < 2; ++li)
      for (int k = 0; k < 4; ++k)
        for (int cc = 0; cc < 2; ++cc) {
          sc->left.mvd[li][k][cc] = sc->mvx[li][1 + k][4][cc];
          te->mvd[li][k][cc] = sc->mvx[li][4][1 + k][cc];
        }
#endif
    sc->left.f = fr;
    te->f = fbm;
  }

  // room for n blocks of one macroblock in the slice's current chunk, else a
  // new chunk from the window's counter (one lane adds; the wave reads lane
  // 0's result); false (DEC_E_ARENA) when the window arena is exhausted —
  // the counter keeps counting, so the host sees what the window asked for
  VTS_HD VTS_INLINE bool reserve(uint32_t n) {
    if (blk_end - blk_at >= n) return true;
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t b = 0;
    if (lane_ == 0) b = atomicAdd(arena_top, kArenaChunk);
    b = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(b)));
#else
    const uint32_t b = __atomic_fetch_add(arena_top, kArenaChunk, __ATOMIC_RELAXED);
#endif
    if (b > arena_blocks - kArenaChunk || arena_blocks < kArenaChunk) {
      err |= DEC_E_ARENA;
      return false;
    }
    blk_at = b;
    blk_end = b + kArenaChunk;
    return true;
  }
  // store sc->blk (or src) as the next arena block; bit = kBlk* index (the
  // macroblock reserved its room first)
  VTS_HD VTS_INLINE void store_block(uint32_t bit, const int16_t *src) {
    VTS_PARSE_TRACE(7);
    int16_t *dst = arena + 16 * static_cast<int64_t>(blk_at);
#if defined(__HIPCC__)
    u32x4 *d4 = reinterpret_cast<u32x4 *>(dst);
    const u32x4 *s4 = reinterpret_cast<const u32x4 *>(src);
    d4[0] = s4[0];
    d4[1] = s4[1];
#else
    for (int i = 0; i < 16; ++i) dst[i] = src[i];
#endif
    if (cur().blocks == 0) cur().coef = blk_at;
    cur().blocks |= 1u << bit;
    ++blk_at;
  }
  // The block being decoded by residual_t: on the device coefficient j
  // (raster position; an 8x8 block's 64 in raster order, its four stored
  // blocks lanes 16k..16k+15) lives in lane j of cv, so a level is one select
  // and the store one 2-byte write per lane, with no LDS round trip (the
  // scratch copy, sc->blk / blk8, stays the host's, and I_PCM's)
#if defined(__HIP_DEVICE_COMPILE__)
  int32_t cv;
  VTS_HD VTS_INLINE void coef_clear(int16_t *, int) { cv = 0; }
  VTS_HD VTS_INLINE void coef_set(int16_t *, int pos, int v) { cv = lane_ == pos ? v : cv; }
#else
  VTS_HD VTS_INLINE void coef_clear(int16_t *dst, int n) { zero16x(dst, n); }
  VTS_HD VTS_INLINE void coef_set(int16_t *dst, int pos, int v) { dst[pos] = static_cast<int16_t>(v); }
#endif
  // store nblk (1 or 4) consecutive blocks of the decoded block as the next
  // arena blocks; bit = the first's kBlk* index (room reserved by the caller)
  VTS_HD VTS_INLINE void store_coefs(uint32_t bit, int nblk, const int16_t *src) {
    VTS_PARSE_TRACE(7);
    int16_t *dst = arena + 16 * static_cast<int64_t>(blk_at);
#if defined(__HIP_DEVICE_COMPILE__)
    (void)src;
    if (lane_ < 16 * nblk) dst[lane_] = static_cast<int16_t>(cv);
#else
    for (int i = 0; i < 16 * nblk; ++i) dst[i] = src[i];
#endif
    MbRec &m = cur();
    if (m.blocks == 0) m.coef = blk_at;
    m.blocks |= ((1u << nblk) - 1u) << bit;
    blk_at += static_cast<uint32_t>(nblk);
  }
  VTS_HD VTS_INLINE void set_cbf(uint32_t bit) {
    MbRec &m = cur();
    m.nzc[bit >> 3] = static_cast<uint8_t>(m.nzc[bit >> 3] | (1u << (bit & 7)));
  }

  // condTermFlagN of ref_idx_lX (9.3.3.1.1.6): refIdxLX > 0 of an inter
  // neighbour partition that is neither skipped nor predicted in direct mode
  // (xN, yN in -1..15: A and B neighbours only)
  VTS_HD VTS_INLINE int ref_gt0_at(int xN, int yN, int l) const {
    if (xN < 0) return static_cast<int>((fa >> (kERefSh + 2 * l + (yN >> 3))) & 1u);
    if (yN < 0) return static_cast<int>((fb >> (kERefSh + 2 * l + (xN >> 3))) & 1u);
    const int p8 = (yN >> 3) * 2 + (xN >> 3);
    if (bframes && ((cur1().direct >> p8) & 1)) return 0;
    return (l ? cur1().ref1[p8] : cur().ref[p8]) > 0 ? 1 : 0;
  }
  VTS_HD VTS_INLINE int mvd_at(int xN, int yN, int comp, int l) const {
    return sc->mvx[l][(yN >> 2) + 1][(xN >> 2) + 1][comp];
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
  VTS_HD VTS_INLINE int ref_idx(int x0, int y0, int l) {
    int v = 0;
    if (dec(54 + ref_gt0_at(x0 - 1, y0, l) + 2 * ref_gt0_at(x0, y0 - 1, l))) {
      v = 1;
      if (dec(58)) {
        v = 2;
        while (dec(59))
          if (++v > 32) break;
      }
    }
    return v;
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

  // mb_pred / sub_mb_pred of an inter macroblock (7.3.5.1-2) as syntax:
  // shape 0..3 (16x16, 16x8, 8x16, 8x8), pm[k] the prediction of partition k
  // (bit 0 L0, bit 1 L1; 0 direct), sub[k] the sub-partition shape of 8x8 k.
  // ref_idx into ref / ref1 per quadrant, mvd into mv / mv1 per 4x4 block and
  // into the |mvd| grid.  false (err set) on a reference index outside the list.
  VTS_HD VTS_INLINE bool inter_syntax(int shape, const uint8_t (&pm)[4], const uint8_t (&sub)[4]) {
    const int nparts = shape == 0 ? 1 : (shape < 3 ? 2 : 4);
    MbRec &m = cur();
    MbRecB &m1 = cur1();
    for (int l = 0; l < 2; ++l) {
      const int nref = l ? (x ? x->num_ref1 : 0) : s->num_ref;
      for (int k = 0; k < nparts; ++k) {
        if (!((pm[k] >> l) & 1)) continue;
        const int x0 = (shape == 2 || shape == 3) ? 8 * (k & 1) : 0;
        const int y0 = shape == 1 ? 8 * k : (shape == 3 ? 8 * (k >> 1) : 0);
        const int v = nref > 1 ? ref_idx(x0, y0, l) : 0;
        if (v >= nref || (l ? x->ref_slot1[v & 31] : s->ref_slot[v & 31]) < 0) {
          err |= DEC_E_NO_REF;
          return false;
        }
        // the partition's 8x8 quarters carry the index (later contexts, h264_derive)
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
          const int dx = mvd(40, mvd_at(sx - 1, sy, 0, l) + mvd_at(sx, sy - 1, 0, l));
          const int dy = mvd(47, mvd_at(sx - 1, sy, 1, l) + mvd_at(sx, sy - 1, 1, l));
          const uint8_t ax = static_cast<uint8_t>(vts_min(dx < 0 ? -dx : dx, 33));
          const uint8_t ay = static_cast<uint8_t>(vts_min(dy < 0 ? -dy : dy, 33));
          const uint32_t bm = blk_mask(sx, sy, pw, ph);
          // mvd_lX lies in [-8192, 8191.75] samples (Annex A): the record's int16
          if (dx < -32768 || dx > 32767 || dy < -32768 || dy > 32767) {
            err |= DEC_E_SYNTAX;
            return false;
          }
          const int16_t cx = static_cast<int16_t>(dx), cy = static_cast<int16_t>(dy);
          VTS_LANES(16, b) if ((bm >> b) & 1u) {
            sc->mvx[l][1 + (b >> 2)][1 + (b & 3)][0] = ax;
            sc->mvx[l][1 + (b >> 2)][1 + (b & 3)][1] = ay;
            if (l) {
              m1.mv1[b][0] = cx;
              m1.mv1[b][1] = cy;
            } else {
              m.mv[b][0] = cx;
              m.mv[b][1] = cy;
            }
          }
        }
      }
    m.i4[0] = static_cast<uint8_t>(shape);
    m.i4[1] = static_cast<uint8_t>(pm[0] | (pm[1] << 2) | (pm[2] << 4) | (pm[3] << 6));
    m.i4[2] = static_cast<uint8_t>(sub[0] | (sub[1] << 2) | (sub[2] << 4) | (sub[3] << 6));
    return !err;
  }

  // residual_block_cabac (7.3.5.3.3): each level goes straight to its raster
  // position in dst, which the caller has zeroed (4x4 blocks: zig-zag position
  // of coefficient start + i; 8x8: the 8x8 zig-zag; chroma DC: list order);
  // count of non-zero levels (0: coded_block_flag 0), -1 on error.  kT8: an
  // 8x8 block (ctxBlockCat 5, contexts 402..459); else cat 0..4 (85..275)
  template <bool kT8>
  VTS_HD VTS_INLINE int residual_t(int cat, int cbf_inc, int maxNum, int16_t *dst, int start) {
    typedef typename std::conditional<kT8, uint64_t, uint32_t>::type Mask;
    // every context of a 4x4 block (ctxIdx 85..275) lies in lane table 0 at
    // slot ctxIdx - 85, every one of an 8x8 block (402..459) in table 1 at
    // ctxIdx - 314: the slots from their bases, no table select per bin
    constexpr int kTab = kT8 ? 1 : 0;
    VTS_PARSE_TRACE(13);
    if (!kT8 && !dec_slot<0>(static_cast<uint32_t>(cbf_off(cat) + cbf_inc))) return 0;
    Mask sig = 0;
    int numc = maxNum;
    const int sig_q = kT8 ? 402 - 314 : 105 - 85 + sig_off(cat), last_q = kT8 ? 417 - 314 : 166 - 85 + sig_off(cat);
    for (int i = 0; i < numc - 1; ++i) {
      int qs, ql;
      if (kT8) {
        const uint32_t e = s8.get(static_cast<uint32_t>(i));
        qs = sig_q + static_cast<int>(e & 15u);
        ql = last_q + static_cast<int>((e >> 8) & 15u);
      } else {
        // ctxIdxInc = i: Min(i, 2) of chroma DC (cat 3) is i too, its i <= 2
        // (4 levels); the largest slots are 80 / 141 (cat 4, i = 13)
        qs = sig_q + i;
        ql = last_q + i;
      }
      if (dec_slot<kTab>(static_cast<uint32_t>(qs))) {
        sig |= Mask(1) << i;
        if (dec_slot<kTab>(static_cast<uint32_t>(ql))) {
          numc = i + 1;
          break;
        }
      }
    }
    sig |= Mask(1) << (numc - 1);
    VTS_PARSE_TRACE(14);
    int eq1 = 0, gt1 = 0, n = 0;
    const int base = kT8 ? 426 - 314 : 227 - 85 + abs_off(cat);
    while (sig) {  // the significant coefficients, highest first
      const int i = kT8 ? 63 - static_cast<int>(__builtin_clzll(static_cast<uint64_t>(sig)))
                        : 31 - static_cast<int>(__builtin_clz(static_cast<uint32_t>(sig)));
      sig &= ~(Mask(1) << i);
      int v = 0;
      if (dec_slot<kTab>(static_cast<uint32_t>(base + (gt1 ? 0 : vts_min(4, 1 + eq1))))) {
        v = 1;
        const uint32_t qg = static_cast<uint32_t>(base + 5 + vts_min(4 - (cat == 3 ? 1 : 0), gt1));
        while (v < 14 && dec_slot<kTab>(qg)) ++v;
        if (VTS_UNLIKELY(v >= 14)) {  // UEG0 suffix
          int k = 0;
          while (bypass()) {
            v += 1 << k;
            if (++k > 24) return -1;
          }
          while (k--) v += static_cast<int>(bypass()) << k;
        }
      }
      const int mag = v + 1;
      const int lvl = bypass() ? -mag : mag;
      if (VTS_UNLIKELY(mag > 32768 || lvl > 32767)) return -1;
      const int pos = kT8 ? static_cast<int>((s8.get(static_cast<uint32_t>(i)) >> 16) & 63u)
                          : (cat == 3 ? i : zz4(i + start));
      coef_set(dst, pos, lvl);
      if (v == 0) ++eq1;
      else ++gt1;
      ++n;
    }
    return n;
  }

  // ------------------------------------------------------ macroblock_layer
  // (begin_mb done by the caller); returns false to stop the slice
  VTS_HD VTS_INLINE bool mb_cabac(int *qp) {
    MbRec &m = cur();
    const bool is_b = s->is_p == kSliceB;
    int itype, mb_type = 0;
    if (is_b) {
      const int t = b_type((av_a && !(fa & kEDirect16) ? 1 : 0) + (av_b && !(fb & kEDirect16) ? 1 : 0));
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
      itype = i_type(0, (av_a && etype(fa) != kMbI4x4 ? 1 : 0) + (av_b && etype(fb) != kMbI4x4 ? 1 : 0));
    }
    if (itype == 25) {  // I_PCM: alignment, 384 samples through the RBSP reader, engine restart
      m.type = kMbPcm;
      m.qp = static_cast<uint8_t>(*qp);
      br.reset_at(cab_consumed());  // the engine's lookahead goes back to the bit reader
      br.align();
      for (int j = 0; j < 16; ++j) m.nz[j] = 16;
      if (!reserve(kPcmBlocks)) return false;
      for (int k = 0; k < 12; ++k) {
        for (int i = 0; i < 16; ++i) {
          const uint32_t lo = br.bits(8), hi = br.bits(8);
          sc->blk[i] = static_cast<int16_t>(lo | (hi << 8));
        }
        store_block(k, sc->blk);
      }
      m.blocks = 0;
      prev_qpd = false;
      cab_start();
      return !br.err;
    }
    int cbp = 0;
    bool small = false;
    if (itype == 0) {  // I_NxN: the modes' syntax (h264_derive predicts them)
      m.type = kMbI4x4;
      bool t8 = false;
      if (t8mode) t8 = dec(399 + ((fa & kET8) ? 1 : 0) + ((fb & kET8) ? 1 : 0)) != 0;
      const int nb = t8 ? 4 : 16;
      if (t8) m.modes = kModeT8;
      for (int i = 0; i < nb; ++i) {
        uint32_t v = 8;
        if (!dec(68)) {
          v = dec(69);
          v |= dec(69) << 1;
          v |= dec(69) << 2;
        }
        const int r = t8 ? (i >> 1) * 8 + (i & 1) * 2 : blk_y(i) * 4 + blk_x(i);
        m.i4[r >> 1] = static_cast<uint8_t>((m.i4[r >> 1] & (0xf0 >> ((r & 1) * 4))) | (v << ((r & 1) * 4)));
      }
    } else if (itype > 0) {  // I_16x16
      m.type = kMbI16;
      cbp = ((((itype - 1) / 4) % 3) << 4) | (itype >= 13 ? 15 : 0);
      m.modes = static_cast<uint8_t>((itype - 1) % 4);
    } else {  // inter (Tables 7-13, 7-14, 7-17, 7-18)
      m.type = kMbInter;
      uint8_t pm[4] = {0, 0, 0, 0}, sub[4] = {0, 0, 0, 0};
      int shape;
      if (is_b) {
        if (mb_type == 0) {  // B_Direct_16x16
          VTS_PARSE_TRACE(6);
          cur1().direct = 0x0f | kDirect16;
          if (!direct8x8) small = true;
          shape = -1;
        } else if (mb_type <= 3) {
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
            sub[k] = static_cast<uint8_t>(kBSub[v] >> 2);
            if (pm[k] == 0) {
              cur1().direct |= static_cast<uint8_t>(1u << k);
              if (!direct8x8) small = true;
            } else if (sub[k]) {
              small = true;
            }
          }
        }
      } else {
        shape = mb_type;
        for (int k = 0; k < 4; ++k) pm[k] = 1;
        if (mb_type == 3)
          for (int k = 0; k < 4; ++k) {
            int v;
            if (dec(21)) v = 0;
            else if (!dec(22)) v = 1;
            else v = dec(23) ? 2 : 3;
            sub[k] = static_cast<uint8_t>(v);
            if (v) small = true;
          }
      }
      if (shape >= 0 && !inter_syntax(shape, pm, sub)) return false;
    }
    if (m.type == kMbI4x4 || m.type == kMbI16) {  // intra_chroma_pred_mode, TU cMax 3
      int cm = 0;
      if (dec(64 + ((fa & kEChroma) ? 1 : 0) + ((fb & kEChroma) ? 1 : 0))) {
        cm = 1;
        if (dec(67)) {
          cm = 2;
          if (dec(67)) cm = 3;
        }
      }
      m.modes = static_cast<uint8_t>(m.modes | (cm << 2));
    }
    if (m.type != kMbI16) {  // coded_block_pattern (9.3.3.1.1.4)
      const int ca_cbp = ecbp(fa), cb_cbp = ecbp(fb);
      for (int b8 = 0; b8 < 4; ++b8) {
        // A: the left 8x8 (inside, or the left macroblock's right column);
        // B: the 8x8 above (inside, or the top macroblock's bottom row)
        const int condA = (b8 & 1) ? !((cbp >> (b8 - 1)) & 1) : (av_a ? !((ca_cbp >> (b8 + 1)) & 1) : 0);
        const int condB = (b8 & 2) ? !((cbp >> (b8 - 2)) & 1) : (av_b ? !((cb_cbp >> (b8 + 2)) & 1) : 0);
        cbp |= static_cast<int>(dec(73 + condA + 2 * condB)) << b8;
      }
      const int ccA = av_a ? ca_cbp >> 4 : 0, ccB = av_b ? cb_cbp >> 4 : 0;
      if (dec(77 + (ccA != 0) + 2 * (ccB != 0))) cbp |= (1 + static_cast<int>(dec(81 + (ccA == 2) + 2 * (ccB == 2)))) << 4;
    }
    m.cbp = static_cast<uint8_t>(cbp);
    if (m.type == kMbInter && (cbp & 15) && t8mode && !small) {
      if (dec(399 + ((fa & kET8) ? 1 : 0) + ((fb & kET8) ? 1 : 0))) m.modes = static_cast<uint8_t>(m.modes | kModeT8);
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
    VTS_PARSE_TRACE(12);
    const bool intra = m.type == kMbI4x4 || m.type == kMbI16;
    const bool t8 = (m.modes & kModeT8) != 0;
    // condTermFlagN (9.3.3.1.1.9) of coded_block_flag across the edges: an
    // unavailable neighbour counts as the current macroblock's intra-ness
    const uint32_t un = intra ? 0xffffffffu : 0u;
    const uint32_t ea = av_a ? fa : un, eb = av_b ? fb : un;
    uint32_t cbfc = 0;  // inside the macroblock: the luma 4x4 blocks' coded_block_flag, raster
    uint32_t todo = m.type == kMbI16 ? 1u << kBlkI16Dc : 0u;
    for (int q = 0; q < 4; ++q)
      if ((cbp >> q) & 1) todo |= (t8 ? 1u : 15u) << (kBlkLuma0 + 4 * q);
    if (cbp >> 4) todo |= 3u << kBlkChromaDc0;
    if ((cbp >> 4) == 2) todo |= 255u << kBlkChromaAc0;
    if (todo && !reserve(kMbMaxBlocks)) return false;
    while (todo) {
      const uint32_t bt = static_cast<uint32_t>(__builtin_ctz(todo));
      todo &= todo - 1u;
      int cat, inc = 0, maxNum = 16, start = 0, r = 0;
      int16_t *dst = sc->blk;
      if (bt == kBlkI16Dc) {
        // an available neighbour's Intra16x16DCLevel flag (I_PCM: 1, other types 0)
        cat = 0;
        inc = static_cast<int>(((av_a ? fa : ~0u) & kECbfDc) ? 1 : 0) + 2 * static_cast<int>(((av_b ? fb : ~0u) & kECbfDc) ? 1 : 0);
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
          const uint32_t ca = bx ? (cbfc >> (r - 1)) & 1u : (ea >> (kECbfSh + by)) & 1u;
          const uint32_t cb = by ? (cbfc >> (r - 4)) & 1u : (eb >> (kECbfSh + bx)) & 1u;
          inc = static_cast<int>(ca + 2 * cb);
        }
      } else if (bt < kBlkChromaAc0) {
        cat = 3;
        maxNum = 4;
        const int pl = static_cast<int>(bt) - kBlkChromaDc0;
        inc = static_cast<int>((ea >> (kECdcSh + pl)) & 1u) + 2 * static_cast<int>((eb >> (kECdcSh + pl)) & 1u);
      } else {
        const int j = static_cast<int>(bt) - kBlkChromaAc0, pl = j >> 2, cx = j & 1, cy = (j >> 1) & 1;
        cat = 4;
        maxNum = 15;
        start = 1;
        const uint32_t cbf = static_cast<uint32_t>(m.nzc[2]) | (static_cast<uint32_t>(m.nzc[3]) << 8);  // bits 16..31
        const uint32_t ca = cx ? (cbf >> (kBlkChromaAc0 - 16 + 4 * pl + cy * 2)) & 1u : (ea >> (kECacSh + 2 * pl + cy)) & 1u;
        const uint32_t cb = cy ? (cbf >> (kBlkChromaAc0 - 16 + 4 * pl + cx)) & 1u : (eb >> (kECacSh + 2 * pl + cx)) & 1u;
        inc = static_cast<int>(ca + 2 * cb);
      }
      coef_clear(dst, cat == 5 ? 64 : 16);
      const int nc = cat == 5 ? residual_t<true>(5, 0, 64, dst, 0) : residual_t<false>(cat, inc, maxNum, dst, start);
      if (nc < 0) { err |= DEC_E_SYNTAX; return false; }
      if (cat == 5) {  // the quarter's 4 blocks: raster 8x8 rows 2j, 2j + 1
        const int rs[4] = {r, r + 1, r + 4, r + 5};
        for (int j = 0; j < 4; ++j) {
          m.nz[rs[j]] = static_cast<uint8_t>(nc > 255 ? 255 : nc);
          set_cbf(1u + static_cast<uint32_t>(rs[j]));
        }
        if (nc) store_coefs(bt, 4, sc->blk8);
        continue;
      }
      if (cat == 1 || cat == 2) {
        m.nz[r] = static_cast<uint8_t>(nc);
        cbfc |= (nc ? 1u : 0u) << r;
      }
      if (nc) {
        set_cbf(bt == kBlkI16Dc ? 0u : (cat <= 2 ? 1u + static_cast<uint32_t>(r) : bt));
        store_coefs(bt, 1, sc->blk);
      }
    }
    if (br.err || cab_consumed() > 8 * br.size) {
      err |= DEC_E_SYNTAX;
      return false;
    }
    return true;
  }
};

// Parse CABAC slice `s` (window slice index si) from its RBSP (rbsp_len
// bytes, emulation-prevention bytes removed) into syntax records (above);
// sc is the wave's scratch with SynEdge[P.mb_width] behind it.  Returns
// DEC_E_* bits.
VTS_HD VTS_INLINE uint32_t parse_slice_cabac(const uint8_t *rbsp, int32_t rbsp_len, const FullSlice &s, uint32_t si,
                                             const FullParams P, MbRec *frame_recs, MbRecB *frame_recs1,
                                             const SliceExt *x, int16_t *arena, uint32_t *arena_top,
                                             uint32_t arena_blocks, uint32_t epoch, SynScratch *sc) {
  CabacSyn p;
  p.bframes = P.bframes != 0;
  p.direct8x8 = P.direct8x8 != 0;
  p.t8mode = P.t8mode != 0;
  if (s.is_p == kSliceB && (!x || !P.bframes)) return DEC_E_NO_REF;
  p.s = &s;
  p.x = x;
  p.recs = frame_recs;
  p.recs1 = frame_recs1;
  p.arena = arena;
  p.sc = sc;
  p.top = reinterpret_cast<SynEdge *>(reinterpret_cast<uint8_t *>(sc) + (sizeof(SynScratch) + 15) / 16 * 16);
  p.arena_top = arena_top;
  p.arena_blocks = arena_blocks;
  p.blk_at = p.blk_end = 0;
  p.slice_index = si;
  p.epoch = epoch;
  p.mbw = P.mb_width;
  p.first_mb = s.first_mb;
  p.err = 0;
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
  p.cab_tables();
  p.cab_init(!s.is_p, s.qp);
  p.cab_start();
  VTS_PARSE_TRACE(15);
  int addr = s.first_mb, qp = s.qp;
  for (;;) {
    if (addr >= nmb) {
      p.err |= DEC_E_SYNTAX;
      break;
    }
    p.refresh_lane();
    p.begin_mb(addr);
    bool skip = false;
    if (s.is_p)
      skip = p.dec((s.is_p == kSliceB ? 24 : 11) + (p.av_a && CabacSyn::etype(p.fa) != kMbSkip ? 1 : 0) +
                   (p.av_b && CabacSyn::etype(p.fb) != kMbSkip ? 1 : 0)) != 0;
    if (skip) {
      VTS_PARSE_TRACE(s.is_p == kSliceB ? 4 : 5);
      p.emit_skip(addr, qp, s.is_p == kSliceB);
      p.prev_qpd = false;
    } else {
      p.init_mb(addr);
      if (!p.mb_cabac(&qp) || p.err) break;  // one inlined copy for every slice type
      p.end_mb(addr);
    }
    ++addr;
    if (p.term()) break;  // end_of_slice_flag
  }
  // the arithmetic decoder has read through the stop bit
  if (!p.err && (p.br.err || p.cab_consumed() != stop_bit + 1)) p.err |= DEC_E_SYNTAX;
  VTS_PARSE_TRACE(16);
  return p.err;
}

}  // namespace full
}  // namespace vts
