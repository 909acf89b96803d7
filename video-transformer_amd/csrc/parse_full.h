// parse_full.h — CAVLC slice_data() parser of the general device decoder
// (h264_parse_full in decode_full.hip runs one lane of it per slice; the CPU
// harness tests/native/full_host.cpp compiles the same code for the host).
//
// The host has already parsed the slice header (h264_sched.cpp) and hands
// over where slice_data() starts, the slice QP and RefPicList0 / 1 as ring
// slots.  Per macroblock the lane derives everything later stages need and the
// standard derives from syntax alone — Intra_4x4 modes (8.3.1.1), motion
// vectors (8.4.1.3, P_Skip 8.4.1.1, B direct prediction 8.4.1.2 from the
// colocated picture's records), QPY, total_coeff — and writes one MbRec (+ an
// MbRecB with the list-1 motion in streams with B slices) plus its non-zero
// coefficient blocks (raster order, int16) into the slice's reserved arena
// range.  Errors come back as DEC_E_* bits.
#pragma once
#include <cstdint>

#include "h264.h"
#include "h264_full.h"
#include "h264_tables.h"
#include "h264_cabac_tables.h"
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

// Table 7-14: prediction of the two partitions of B mb_type 1..21 (1 Pred_L0,
// 2 Pred_L1, 3 BiPred), as pm0 | pm1 << 2; Table 7-18: B sub_mb_type ->
// prediction (0 direct) | shape << 2 (0 8x8, 1 8x4, 2 4x8, 3 4x4)
#if defined(__HIPCC__)
__device__ __constant__ static const uint8_t kBPart[22] = {
#else
static const uint8_t kBPart[22] = {
#endif
    0, 1, 2, 3, 5, 5, 10, 10, 9, 9, 6, 6, 13, 13, 14, 14, 7, 7, 11, 11, 15, 15};
#if defined(__HIPCC__)
__device__ __constant__ static const uint8_t kBSub[13] = {
#else
static const uint8_t kBSub[13] = {
#endif
    0, 1, 2, 3, 5, 9, 6, 10, 7, 11, 13, 14, 15};

// What a B slice adds to the parse (null / zero otherwise)
struct BCtx {
  MbRecB *recs1;          // the frame's list-1 records (streams with B slices)
  const MbRec *col;       // the colocated picture's records (RefPicList1[0], B slices)
  const MbRecB *col1;
  const SliceExt *x;      // the slice's SliceExt (B slices, weighted P slices)
};

VTS_HD VTS_INLINE int clip3i(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
// MinPositive (8.4.1.2.2)
VTS_HD VTS_INLINE int min_positive(int x, int y) { return (x >= 0 && y >= 0) ? (x < y ? x : y) : (x > y ? x : y); }

// zero n (a multiple of 8) int16 in 16-byte stores (LDS on the device)
VTS_HD VTS_INLINE void zero16x(int16_t *p, int n) {
  for (int i = 0; i < n; i += 8) {
    int16_t *q = p + i;
#if defined(__HIPCC__)
    typedef uint32_t z4 __attribute__((ext_vector_type(4)));
    *reinterpret_cast<z4 *>(q) = z4{0, 0, 0, 0};
#else
    for (int k = 0; k < 8; ++k) q[k] = 0;
#endif
  }
}

// 64 dwords the single parse lane indexes at run time without a memory access:
// on the device the lanes of one VGPR (v_readlane / v_writelane with the lane
// in an SGPR; the kernel runs one lane per wave, so the other 63 lanes of every
// VGPR are free storage), on the host an array.  A byte table read this way
// costs one VALU instruction instead of a dependent global load (the __constant__
// byte tables compile to global_load_ubyte through the GOT).
#if defined(__HIP_DEVICE_COMPILE__)
// the intrinsic behind v_writelane_b32 (this compiler has no builtin for it)
extern "C" __device__ int vts_writelane(int value, int lane, int old) __asm("llvm.amdgcn.writelane");
#endif
struct LaneTab {
#if defined(__HIP_DEVICE_COMPILE__)
  // seeded with the lane id: the value must be divergent (a VGPR), or the
  // compiler treats the all-uniform writelane chain as one uniform value and
  // folds every readlane of it to that value
  uint32_t v = __builtin_amdgcn_mbcnt_lo(~0u, 0u);
  __device__ VTS_INLINE uint32_t get(uint32_t i) const {
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), static_cast<int>(i)));
  }
  __device__ VTS_INLINE void set(uint32_t i, uint32_t x) {
    v = static_cast<uint32_t>(vts_writelane(static_cast<int>(x), static_cast<int>(i), static_cast<int>(v)));
  }
#else
  uint32_t v[64];
  uint32_t get(uint32_t i) const { return v[i & 63]; }
  void set(uint32_t i, uint32_t x) { v[i & 63] = x; }
#endif
};

// ------------------------------------------------------------ RBSP bits
// 7.4.1: byte j of a NAL payload (after the header byte) is an
// emulation_prevention_three_byte iff it is 0x03 after two zero payload bytes
// (00 00 03 00 00 03 holds two: an EPB resets the zero count, and the two
// zeros before the second one are bytes 3 and 4).  The device removes them
// once per session (nal_unescape in decode_full.hip, one workgroup per slice
// NAL); this is the same rule, serially (the CPU harness).
VTS_HD VTS_INLINE bool is_epb(const uint8_t *p, int32_t j) { return j >= 2 && p[j] == 3 && p[j - 1] == 0 && p[j - 2] == 0; }
VTS_HD VTS_INLINE int32_t unescape_nal(const uint8_t *in, int32_t n, uint8_t *out) {
  int32_t o = 0;
  for (int32_t j = 0; j < n; ++j)
    if (!is_epb(in, j)) out[o++] = in[j];
  return o;
}

// The general parsers' bit reader: a left-aligned 64-bit window over an
// RBSP (no emulation-prevention bytes left, so a refill is one 4-byte append)
// filled from kW - 1 cached payload dwords in per-lane scratch (LDS on the
// device).  Bits past the RBSP read as zeros and make overrun() true.
template <int kW>
struct RbspBitsT {
  const uint8_t *base;   // first RBSP byte of the payload
  uint64_t win;          // next bits, MSB first
  int32_t nb;            // valid bits in win
  int32_t fill;          // bits appended to the window so far (incl. zero padding)
  int32_t size;          // RBSP bytes
  int32_t pos;           // next byte to append
  int32_t cache_at;      // payload index of cache[0] (multiple of 4 (kW - 1)), -1 none
  uint32_t *cache;       // kW dwords from cache_at (per-lane scratch)
  bool err;

  VTS_HD VTS_INLINE void init(const uint8_t *p, int32_t n, uint32_t *scratch) {
    cache = scratch;
    base = p;
    size = n;
    win = 0;
    nb = fill = pos = 0;
    cache_at = -1;
    err = false;
  }
  // 4 payload bytes at i, little endian (reads past the payload stay inside
  // the padded buffer)
  VTS_HD VTS_INLINE uint32_t load4(int32_t i) {
    constexpr int32_t kBlk = 4 * (kW - 1);
    const int32_t blk = i - (i % kBlk);
    if (VTS_UNLIKELY(blk != cache_at)) {
      const uint8_t *pb = base + blk;
      const int sh = static_cast<int>(reinterpret_cast<uintptr_t>(pb) & 3);
      // plain loads from a base the compiler can see is dword aligned, all in
      // flight together
      const uint32_t *w = reinterpret_cast<const uint32_t *>(reinterpret_cast<uintptr_t>(pb) & ~uintptr_t(3));
      uint32_t t[kW + 1];
#pragma unroll
      for (int k = 0; k <= kW; ++k) t[k] = w[k];
#pragma unroll
      for (int k = 0; k < kW; ++k) cache[k] = sh ? vts_alignbyte(t[k + 1], t[k], sh) : t[k];
      cache_at = blk;
    }
    const int32_t o = i - blk, q = o >> 2, r = o & 3;
    return vts_alignbyte(cache[q + 1], cache[q], r);
  }
  VTS_HD VTS_INLINE void refill() {  // requires nb <= 32
    uint32_t v = load4(pos);
    const int32_t left = size - pos;
    if (left < 4) v = left <= 0 ? 0u : v & (0xffffffffu >> (8 * (4 - left)));
    win |= static_cast<uint64_t>(__builtin_bswap32(v)) << (32 - nb);
    nb += 32;
    fill += 32;
    pos += 4;
  }
  VTS_HD VTS_INLINE void ensure(int n) {  // n <= 32
    if (VTS_UNLIKELY(nb < n)) refill();
  }
  VTS_HD VTS_INLINE void skip(int n) {  // n < 64, n <= nb
    win <<= n;
    nb -= n;
  }
  VTS_HD VTS_INLINE uint32_t bits(int n) {  // n <= 32
    if (n == 0) return 0;
    ensure(n);
    const uint32_t v = static_cast<uint32_t>(win >> (64 - n));
    skip(n);
    return v;
  }
  VTS_HD VTS_INLINE uint32_t bit() { return bits(1); }
  VTS_HD VTS_INLINE uint32_t ue() {
    ensure(32);
    const uint32_t p = static_cast<uint32_t>(win >> 32);
    if (p == 0) {  // more than 31 leading zeros
      err = true;
      return 0;
    }
    const int lz = __builtin_clz(p);
    if (lz < 16) {
      const int len = 2 * lz + 1;
      skip(len);
      return (p >> (32 - len)) - 1u;
    }
    skip(lz + 1);
    return ((1u << lz) - 1u) + bits(lz);
  }
  VTS_HD VTS_INLINE int32_t se() {
    const uint32_t k = ue();
    return (k & 1u) ? static_cast<int32_t>((k + 1) >> 1) : -static_cast<int32_t>(k >> 1);
  }
  VTS_HD VTS_INLINE int32_t consumed() const { return fill - nb; }  // RBSP bit index
  VTS_HD VTS_INLINE void align() { skip(nb & 7); }                  // fill is a multiple of 8
  VTS_HD VTS_INLINE bool overrun() const { return consumed() > 8 * size; }
  // more_rbsp_data(): the next bit lies before the stop bit (RBSP bit index)
  VTS_HD VTS_INLINE bool more(int64_t stop_bit) const { return consumed() < stop_bit; }
  // drop the window and continue at RBSP bit rb
  VTS_HD VTS_INLINE void reset_at(int32_t rb) {
    pos = rb >> 3;
    if (pos > size) err = true;
    win = 0;
    nb = 0;
    fill = pos * 8;
    ensure(8);
    skip(rb & 7);
  }
};

// Per-element work of a macroblock (its 16 blocks, its record's 32 dwords) on
// the wave's lanes: on the device the lanes l < n run the body once each (the
// parse waves have 64 lanes, all running the same uniform parse), on the host
// a loop.  Bodies are independent per l (no continue / break, no state carried
// between elements); a per-lane condition comes back uniform through vts_any.
#if defined(__HIP_DEVICE_COMPILE__)
#define VTS_LANES(n, l) if (const int l = lane_; l < (n))
__device__ VTS_INLINE bool vts_any(bool b) { return __ballot(b) != 0; }
#else
#define VTS_LANES(n, l) for (int l = 0; l < (n); ++l)
inline bool vts_any(bool b) { return b; }
#endif

// zig-zag position of coefficient i of a 4x4 block (8.5.6): 4-bit fields of one constant
VTS_HD VTS_INLINE int zz4(int i) { return static_cast<int>((0xFEB7ADC963258410ull >> (4 * i)) & 15u); }

// luma4x4BlkIdx <-> raster 4x4 block
VTS_HD VTS_INLINE int blk_x(int k) { return ((k >> 2) & 1) * 2 + (k & 1); }
VTS_HD VTS_INLINE int blk_y(int k) { return ((k >> 3) & 1) * 2 + ((k >> 1) & 1); }
// raster 4x4 blocks (bit y * 4 + x) of the luma rectangle (x0, y0, w, h)
VTS_HD VTS_INLINE uint32_t blk_mask(int x0, int y0, int w, int h) {
  const uint32_t cols = ((1u << (w >> 2)) - 1u) << (x0 >> 2), rows = 0x1111u & ((1u << (4 * (h >> 2))) - 1u);
  return (cols * rows) << (4 * (y0 >> 2));
}

// Per-lane scratch (LDS on the device): everything the parser indexes at run
// time lives here, so nothing spills to scratch memory, and the neighbours a
// macroblock reads are LDS copies instead of global records.
constexpr int kCacheWords = 17;  // bit reader: 64-byte blocks
struct FullScratch {
  MbRec mb[2];            // the macroblock being parsed and the previous one (left neighbour)
  MbRec top[3];           // row above, columns x-1, x, x+1 at slot column % 3: bytes 16..63 and
                          // 112..127 of the record (type, refs, modes, nz, bottom motion),
                          // word 0 = its intra dependency level
  alignas(16) int16_t blk[16];  // coefficient block being decoded (raster)
  int32_t lev[16];        // its levels in decoding order
  uint32_t cache[kCacheWords];
  uint8_t prev[16], rem[16];  // Intra4x4 prev_intra4x4_pred_mode_flag / rem_intra4x4_pred_mode
  int8_t sub[4], refs[4];     // sub_mb_type / ref_idx_l0 of the partitions
  int8_t refs1[4];            // B: ref_idx_l1 of the partitions
  uint8_t pm[4];              // B: prediction of the partitions (0 direct, 1 L0, 2 L1, 3 Bi)
  int32_t mvd[2][16][2];      // B: mvd_lX of partition k, sub-partition q at [X][4 k + q]
  MbRecB mb1[2];              // list-1 halves of mb[2] (streams with B slices)
  MbRecB top1[3];             // ... of top[3]: bytes 0..31 and 112..127
  // CABAC (parse_cabac.h)
  alignas(16) int16_t blk8[64]; // 8x8 block being decoded (raster)
  // the motion around the current macroblock, per list, for 8.4.1.3's A / B
  // / C / D (mv_border): entries 0..3 = the left neighbour's right column
  // (rows 0..3), 4..7 = the top neighbour's bottom row, 8 = C (top-right),
  // 9 = D (top-left); ref -2 = unavailable, -1 = intra / list unused
  uint32_t nbmv[2][10];
  int8_t nbref[2][10];
  // Min(|mvd_lX|, 33) around the current macroblock, per list: [row][col]
  // with row 0 = the bottom row of the macroblock above, col 0 = the right
  // column of the one to the left (0 where unavailable / not inter), rows and
  // cols 1..4 = the current macroblock's 4x4 blocks
  uint8_t mvx[2][5][5][2];
};

typedef uint32_t u32x4 __attribute__((vector_size(16)));  // SROA-friendly (uint4 copies are memmoves)
// the parts of a row-above record the parser reads (record bytes 16..63, 112..127)
struct TopCtx {
  u32x4 v0, v1, v2, v3;
  uint32_t lvl;
};

struct Parser {
  RbspBitsT<kCacheWords> br;
  const FullSlice *s;     // global (the ref_slot table is indexed at run time)
  int cip;                // constrained_intra_pred_flag
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
  int cur_addr;           // macroblock being parsed
  int cs;                 // sc->mb[cs] = current, sc->mb[cs ^ 1] = previous
  int tslots;             // sc->top slots of D, B, C in bits 0-1, 2-3, 4-5 (one field: a ?:
                          // between three fields becomes a select of their addresses)
  uint16_t lvl_prev;      // intra dependency level of the previous macroblock
  // row above, column pf_col: prefetched during the previous macroblock
  int pf_col;
#if defined(__HIP_DEVICE_COMPILE__)
  // the lane index, re-read opaquely at every macroblock (refresh_lane): what
  // derives from it is computed per macroblock instead of hoisted out of the
  // macroblock loop and spilled (each reload waited for every load in flight)
  int lane_;
  __device__ VTS_INLINE void refresh_lane() {
    lane_ = static_cast<int>(threadIdx.x);
    asm volatile("" : "+v"(lane_));
  }
  u32x4 pfl;              // lane p < 8: piece p of the prefetched column (piece_load)
  u32x4 pfl2;             // ... and of column pf_col + 1 (two columns in flight)
  int pf_col2;
#else
  void refresh_lane() {}
  TopCtx pf;
  u32x4 pf1[3];           // the prefetched column's list-1 context (bframes)
#endif
  BCtx bc;
  int bframes;            // write / read the list-1 records
  int direct8x8;          // direct_8x8_inference_flag
  uint32_t todo;          // residual blocks of the current macroblock still to decode (kBlk* bits)
  bool cur_i16;           // the current macroblock is Intra_16x16

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
  VTS_HD VTS_INLINE MbRec &cur() const { return sc->mb[cs]; }
  VTS_HD VTS_INLINE const MbRec &rec(int n) const {
    if (n == -2) return sc->mb[cs];
    if (n == cur_addr - 1) return sc->mb[cs ^ 1];
    const int d = n - (cur_addr - mbw);  // -1, 0, 1: D, B, C
    return sc->top[(tslots >> (2 * (d + 1))) & 3];
  }
  VTS_HD VTS_INLINE MbRecB &cur1() const { return sc->mb1[cs]; }
  VTS_HD VTS_INLINE const MbRecB &rec1(int n) const {
    if (n == -2) return sc->mb1[cs];
    if (n == cur_addr - 1) return sc->mb1[cs ^ 1];
    const int d = n - (cur_addr - mbw);
    return sc->top1[(tslots >> (2 * (d + 1))) & 3];
  }
  VTS_HD VTS_INLINE int level_of(int n) const {
    if (n == cur_addr - 1) return lvl_prev;
    return static_cast<int>(rec(n).epoch);
  }

  // --- row-above contexts (global record -> LDS slot)
  VTS_HD VTS_INLINE TopCtx top_load(int col) const {
    const int n = cur_addr - mbw + (col - cur_addr % mbw);
    const u32x4 *g = reinterpret_cast<const u32x4 *>(recs + n);
    TopCtx t;
    t.v0 = g[1];
    t.v1 = g[2];
    t.v2 = g[3];
    t.v3 = g[7];
    t.lvl = ilvl[n];
    return t;
  }
  VTS_HD VTS_INLINE void top_store(int col, TopCtx t) const {
    u32x4 *d = reinterpret_cast<u32x4 *>(&sc->top[col % 3]);
    d[1] = t.v0;
    d[2] = t.v1;
    d[3] = t.v2;
    d[7] = t.v3;
    sc->top[col % 3].epoch = t.lvl;
  }
  VTS_HD VTS_INLINE void top_load1(int col, u32x4 (&v)[3]) const {
    const int n = cur_addr - mbw + (col - cur_addr % mbw);
    const u32x4 *g = reinterpret_cast<const u32x4 *>(bc.recs1 + n);
    v[0] = g[0];
    v[1] = g[1];
    v[2] = g[7];
  }
  VTS_HD VTS_INLINE void top_store1(int col, const u32x4 (&v)[3]) const {
    u32x4 *d = reinterpret_cast<u32x4 *>(&sc->top1[col % 3]);
    d[0] = v[0];
    d[1] = v[1];
    d[7] = v[2];
  }
  VTS_HD VTS_INLINE void top_sync(int col) const {
    top_store(col, top_load(col));
    if (bframes) {
      u32x4 v[3];
      top_load1(col, v);
      top_store1(col, v);
    }
  }
#if defined(__HIP_DEVICE_COMPILE__)
  // the same context on the lanes: lane p < 8 moves piece p (record u32x4 1,
  // 2, 3, 7; the intra level; list-1 record u32x4 0, 1, 7), so the prefetch
  // lives in one VGPR quad per lane instead of 29 scalar registers
  __device__ VTS_INLINE u32x4 piece_load(int col) const {
    const int l = lane_;
    const int n = cur_addr - mbw + (col - cur_addr % mbw);
    u32x4 v = {0u, 0u, 0u, 0u};
    if (l < 4) v = reinterpret_cast<const u32x4 *>(recs + n)[l == 3 ? 7 : l + 1];
    else if (l == 4) v[0] = ilvl[n];
    else if (l < 8 && bframes) v = reinterpret_cast<const u32x4 *>(bc.recs1 + n)[l == 7 ? 7 : l - 5];
    return v;
  }
  __device__ VTS_INLINE void piece_store(int col, u32x4 v) const {
    const int l = lane_;
    if (l < 4) reinterpret_cast<u32x4 *>(&sc->top[col % 3])[l == 3 ? 7 : l + 1] = v;
    else if (l == 4) sc->top[col % 3].epoch = v[0];
    else if (l < 8 && bframes) reinterpret_cast<u32x4 *>(&sc->top1[col % 3])[l == 7 ? 7 : l - 5] = v;
  }
#endif
  // a new macroblock: the previous one becomes the left neighbour; the row
  // above rotates through the three slots, its next column loading one
  // macroblock ahead
  VTS_HD VTS_INLINE void advance(int addr) {
    const bool cont = addr > first_mb && addr == cur_addr + 1 && addr % mbw != 0;
    cs ^= 1;
    cur_addr = addr;
    const int x = addr % mbw, y = addr / mbw;
    tslots = ((x + 2) % 3) | ((x % 3) << 2) | (((x + 1) % 3) << 4);
#if defined(__HIP_DEVICE_COMPILE__)
    // two columns in flight: a skipped macroblock parses in less time than a
    // global load takes, so a load issued one macroblock ahead still stalled
    if (y > 0) {
      if (!cont) {
        if (x > 0) piece_store(x - 1, piece_load(x - 1));
        piece_store(x, piece_load(x));
      }
      if (x + 1 < mbw) {
        if (pf_col != x + 1) pfl = piece_load(x + 1);
        piece_store(x + 1, pfl);
      }
      pf_col = -1;
      if (x + 2 < mbw) {
        if (pf_col2 == x + 2) pfl = pfl2;
        else pfl = piece_load(x + 2);
        pf_col = x + 2;
      }
      pf_col2 = -1;
      if (x + 3 < mbw) {
        pfl2 = piece_load(x + 3);
        pf_col2 = x + 3;
      }
    }
#else
    if (y > 0) {
      if (!cont) {
        if (x > 0) top_sync(x - 1);
        top_sync(x);
      }
      if (x + 1 < mbw) {
        if (pf_col != x + 1) {
          pf = top_load(x + 1);
          if (bframes) top_load1(x + 1, pf1);
        }
        top_store(x + 1, pf);
        if (bframes) top_store1(x + 1, pf1);
      }
      pf_col = -1;
      if (x + 2 < mbw) {
        pf = top_load(x + 2);
        if (bframes) top_load1(x + 2, pf1);
        pf_col = x + 2;
      }
    }
#endif
  }

  // 9.2.1 nC
  VTS_HD VTS_INLINE int nc_of(int cur, int bx, int by, bool chroma, int plane) const {
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
  VTS_HD VTS_INLINE int residual_block(int nC, int maxNum, int start_pos) {
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
    zero16x(sc->blk, 16);
    int32_t *level = sc->lev;
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
      if (zeros + tc > maxNum) return -1;  // total_zeros beyond the block (a corrupt slice)
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
  VTS_HD VTS_INLINE bool store_block(uint32_t bit) { return store_block(bit, sc->blk); }
  VTS_HD VTS_INLINE bool store_block(uint32_t bit, const int16_t *src) {
    VTS_PARSE_TRACE(7);
    if (used >= s->arena_cap) return false;
    int16_t *dst = arena + 16 * static_cast<int64_t>(s->arena + used);
#if defined(__HIPCC__)
    u32x4 *d4 = reinterpret_cast<u32x4 *>(dst);
    const u32x4 *s4 = reinterpret_cast<const u32x4 *>(src);
    d4[0] = s4[0];
    d4[1] = s4[1];
#else
    for (int i = 0; i < 16; ++i) dst[i] = src[i];
#endif
    if (cur().blocks == 0) cur().coef = s->arena + used;
    cur().blocks |= 1u << bit;
    ++used;
    return true;
  }

  // --- motion vector prediction (8.4.1.3)
  struct Mv {
    bool avail;
    int ref, x, y;
  };
  // the neighbours' motion of a new macroblock (P / B slices), once: one
  // entry (list, position) per lane
  VTS_HD VTS_INLINE void mv_border(int addr) {
    VTS_LANES(20, i) {
      const int l = i / 10, e = i % 10;
      const int xN = e < 4 ? -1 : (e < 8 ? 4 * (e - 4) : (e == 8 ? 16 : -1)), yN = e < 4 ? 4 * e : -1;
      int xw = 0, yw = 0;
      const int n = nb_mb(addr, xN, yN, 16, &xw, &yw);
      int8_t r = -2;
      uint32_t mv = 0;
      if (n != -1) {
        const MbRec &m = rec(n);
        r = -1;
        if (m.type == kMbInter || m.type == kMbSkip) {
          const int b = (yw / 4) * 4 + xw / 4, p8 = (b >> 3) * 2 + ((b & 3) >> 1);
          if (l) {
            const MbRecB &m1 = rec1(n);
            r = m1.ref1[p8];
            mv = static_cast<uint16_t>(m1.mv1[b][0]) | (static_cast<uint32_t>(static_cast<uint16_t>(m1.mv1[b][1])) << 16);
          } else {
            r = m.ref[p8];
            mv = static_cast<uint16_t>(m.mv[b][0]) | (static_cast<uint32_t>(static_cast<uint16_t>(m.mv[b][1])) << 16);
          }
        }
      }
      sc->nbref[l][e] = r;
      sc->nbmv[l][e] = mv;
    }
  }
  // list l's motion of the neighbouring 4x4 block (ref -1: unavailable, intra
  // or list l unused, with a zero vector); outside the macroblock from
  // mv_border's entries
  VTS_HD VTS_INLINE Mv nb_mv(int cur, int xN, int yN, uint32_t done, int l = 0) const {
    if (xN >= 0 && xN < 16 && yN >= 0) {  // inside: blocks already decoded
      Mv r{false, -1, 0, 0};
      const int b = (yN >> 2) * 4 + (xN >> 2);
      if (yN > 15 || !((done >> b) & 1u)) return r;
      r.avail = true;
      const int p8 = (b >> 3) * 2 + ((b & 3) >> 1);
      if (l) {
        const MbRecB &m1 = sc->mb1[cs];
        r.ref = m1.ref1[p8];
        r.x = m1.mv1[b][0];
        r.y = m1.mv1[b][1];
      } else {
        const MbRec &m = sc->mb[cs];
        r.ref = m.ref[p8];
        r.x = m.mv[b][0];
        r.y = m.mv[b][1];
      }
      return r;
    }
    if (yN >= 0 && xN >= 16) return Mv{false, -1, 0, 0};
    const int e = yN < 0 ? (xN < 0 ? 9 : (xN < 16 ? 4 + (xN >> 2) : 8)) : (yN >> 2);
    const int ref = sc->nbref[l][e];
    if (ref == -2) return Mv{false, -1, 0, 0};
    const uint32_t mv = sc->nbmv[l][e];
    return Mv{true, ref, static_cast<int16_t>(mv & 0xffff), static_cast<int16_t>(mv >> 16)};
  }
  VTS_HD VTS_INLINE Mv nb_mv_generic(int cur, int xN, int yN, uint32_t done, int l = 0) const {
    Mv r{false, -1, 0, 0};
    int xw, yw;
    const int n = nb_mb(cur, xN, yN, 16, &xw, &yw);
    if (n == -1) return r;
    const int b = (yw / 4) * 4 + xw / 4;
    if (n == -2 && !((done >> b) & 1u)) return r;
    r.avail = true;
    const MbRec &m = rec(n);
    if (m.type != kMbInter && m.type != kMbSkip) return r;
    const int p8 = (b >> 3) * 2 + ((b & 3) >> 1);
    if (l) {
      const MbRecB &m1 = rec1(n);
      r.ref = m1.ref1[p8];
      r.x = m1.mv1[b][0];
      r.y = m1.mv1[b][1];
    } else {
      r.ref = m.ref[p8];
      r.x = m.mv[b][0];
      r.y = m.mv[b][1];
    }
    return r;
  }
  VTS_HD VTS_INLINE void mv_pred(int cur, int x0, int y0, int w, int h, int ref, uint32_t done, int *px, int *py,
                                 int l = 0) const {
    const Mv A = nb_mv(cur, x0 - 1, y0, done, l);
    Mv B = nb_mv(cur, x0, y0 - 1, done, l);
    Mv C = nb_mv(cur, x0 + w, y0 - 1, done, l);
    if (!C.avail) C = nb_mv(cur, x0 - 1, y0 - 1, done, l);
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
    VTS_PARSE_TRACE(0);
    advance(addr);
#if defined(__HIP_DEVICE_COMPILE__)
    // the records' initial dwords, one per lane: epoch, slice, 0 coef / blocks /
    // type..modes, ref -1, ref_slot -1, i4 DC (2), then zeros; list 1: ref1 -1,
    // ref_slot1 -1, then zeros
    VTS_LANES(64, l) {
      if (l < 32) {
        const uint32_t v = l == 0 ? epoch : (l == 1 ? slice_index : ((l >= 5 && l <= 7) ? ~0u : ((l == 8 || l == 9) ? 0x22222222u : 0u)));
        reinterpret_cast<uint32_t *>(&cur())[l] = v;
      } else if (bframes) {
        reinterpret_cast<uint32_t *>(&cur1())[l - 32] = l - 32 < 3 ? ~0u : 0u;
      }
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
#endif
  }
  VTS_HD VTS_INLINE void end_mb(int addr) {
    // intra dependency level: 1 + the highest level among the intra-predicted
    // neighbours A, B, C, D the prediction may read (same slice), else 0; the
    // reconstruction runs the levels in order (h264_intra_full)
    uint16_t lv = kNoLevel;
    const MbRec &c = cur();
    if (c.type == kMbI4x4 || c.type == kMbI16) {
      int l = 0, xw, yw;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int n = nb_mb(addr, i == 2 ? 16 : (i == 1 ? 0 : -1), i == 0 ? 0 : -1, 16, &xw, &yw);
        if (n >= 0) {
          const int ln = level_of(n);
          if (ln != kNoLevel) l = vts_max(l, ln + 1);
        }
      }
      lv = static_cast<uint16_t>(l);
    }
    ilvl[addr] = lv;
    lvl_prev = lv;
#if defined(__HIP_DEVICE_COMPILE__)
    // the records to global memory, 16 bytes per lane (list 1: its u32x4 2, 3 are padding)
    VTS_LANES(16, l) {
      if (l < 8) reinterpret_cast<u32x4 *>(&recs[addr])[l] = reinterpret_cast<const u32x4 *>(&cur())[l];
      else if (bframes && (l < 10 || l >= 12))
        reinterpret_cast<u32x4 *>(&bc.recs1[addr])[l - 8] = reinterpret_cast<const u32x4 *>(&cur1())[l - 8];
    }
#else
    recs[addr] = cur();
    if (bframes) bc.recs1[addr] = cur1();
#endif
  }

  VTS_HD VTS_INLINE void set_motion(int b, int ref, int mvx, int mvy) {
    cur().mv[b][0] = static_cast<int16_t>(ref >= 0 ? mvx : 0);
    cur().mv[b][1] = static_cast<int16_t>(ref >= 0 ? mvy : 0);
    const int p8 = (b >> 3) * 2 + ((b & 3) >> 1);
    cur().ref[p8] = static_cast<int8_t>(ref);
    cur().ref_slot[p8] = ref >= 0 ? s->ref_slot[ref & 31] : static_cast<int16_t>(-1);
  }
  VTS_HD VTS_INLINE void set_motion1(int b, int ref, int mvx, int mvy) {
    MbRecB &m1 = cur1();
    m1.mv1[b][0] = static_cast<int16_t>(ref >= 0 ? mvx : 0);
    m1.mv1[b][1] = static_cast<int16_t>(ref >= 0 ? mvy : 0);
    const int p8 = (b >> 3) * 2 + ((b & 3) >> 1);
    m1.ref1[p8] = static_cast<int8_t>(ref);
    m1.ref_slot1[p8] = ref >= 0 ? bc.x->ref_slot1[ref & 31] : static_cast<int16_t>(-1);
  }

  // 8.4.1.2: direct prediction of the raster 4x4 blocks in `mask` from the
  // colocated picture's records (8.4.1.2.1) — spatial (8.4.1.2.2) or temporal
  // (8.4.1.2.3)
  VTS_HD VTS_INLINE void direct_pred(int addr, uint32_t mask) {
    const SliceExt &x = *bc.x;
    const MbRec &cm = bc.col[addr];
    const MbRecB &cm1 = bc.col1[addr];
#if defined(__HIP_DEVICE_COMPILE__)
    // the colocated block's motion (global memory) requested before the
    // neighbours' (LDS) so its latency overlaps the spatial predictor
    const int lb = lane_ & 15;
    const int lcb = direct8x8 ? ((lb >> 3) * 3) * 4 + ((lb & 3) >> 1) * 3 : lb;
    const int lc8 = (lcb >> 3) * 2 + ((lcb & 3) >> 1);
    const int8_t c_ref0 = cm.ref[lc8], c_ref1 = cm1.ref1[lc8];
    const uint32_t c_mv0 = reinterpret_cast<const uint32_t *>(cm.mv)[lcb];
    const uint32_t c_mv1 = reinterpret_cast<const uint32_t *>(cm1.mv1)[lcb];
    const int16_t c_slot0 = cm.ref_slot[lc8], c_slot1 = cm1.ref_slot1[lc8];
#endif
    int ref0 = -1, ref1 = -1, mp[2][2] = {{0, 0}, {0, 0}};
    bool zero = false;
    if (x.direct_spatial) {
      int rf[2];
#pragma unroll
      for (int l = 0; l < 2; ++l) {
        const Mv A = nb_mv(addr, -1, 0, 0, l), B = nb_mv(addr, 0, -1, 0, l);
        Mv C = nb_mv(addr, 16, -1, 0, l);
        if (!C.avail) C = nb_mv(addr, -1, -1, 0, l);
        rf[l] = min_positive(A.ref, min_positive(B.ref, C.ref));
      }
      ref0 = rf[0];
      ref1 = rf[1];
      if (ref0 < 0 && ref1 < 0) {
        ref0 = ref1 = 0;
        zero = true;
      }
      if (!zero) {
        if (ref0 >= 0) mv_pred(addr, 0, 0, 16, 16, ref0, 0, &mp[0][0], &mp[0][1], 0);
        if (ref1 >= 0) mv_pred(addr, 0, 0, 16, 16, ref1, 0, &mp[1][0], &mp[1][1], 1);
      }
    }
    bool bad = false;  // temporal: the colocated reference is not in RefPicList0
    VTS_LANES(16, blk) if ((mask >> blk) & 1u) {
#if defined(__HIP_DEVICE_COMPILE__)
      const bool use0 = c_ref0 >= 0;
      const int ref_col = use0 ? c_ref0 : c_ref1;  // -1: intra
      const uint32_t cmv = use0 ? c_mv0 : c_mv1;
      const int mcx = ref_col < 0 ? 0 : static_cast<int16_t>(cmv & 0xffff);
      const int mcy = ref_col < 0 ? 0 : static_cast<int16_t>(cmv >> 16);
#else
      const int cb = direct8x8 ? ((blk >> 3) * 3) * 4 + ((blk & 3) >> 1) * 3 : blk;
      const int c8 = (cb >> 3) * 2 + ((cb & 3) >> 1);
      const bool use0 = cm.ref[c8] >= 0;
      const int ref_col = use0 ? cm.ref[c8] : cm1.ref1[c8];  // -1: intra
      const int mcx = ref_col < 0 ? 0 : (use0 ? cm.mv[cb][0] : cm1.mv1[cb][0]);
      const int mcy = ref_col < 0 ? 0 : (use0 ? cm.mv[cb][1] : cm1.mv1[cb][1]);
#endif
      if (x.direct_spatial) {
        const bool col_zero = x.col_short && ref_col == 0 && mcx >= -1 && mcx <= 1 && mcy >= -1 && mcy <= 1;
        const bool z0 = zero || ref0 < 0 || (ref0 == 0 && col_zero);
        const bool z1 = zero || ref1 < 0 || (ref1 == 0 && col_zero);
        set_motion(blk, ref0, z0 ? 0 : mp[0][0], z0 ? 0 : mp[0][1]);
        set_motion1(blk, ref1, z1 ? 0 : mp[1][0], z1 ? 0 : mp[1][1]);
      } else {
        int r0 = 0;
        if (ref_col >= 0) {  // the lowest list-0 index naming the colocated block's reference picture
#if defined(__HIP_DEVICE_COMPILE__)
          const int slot = use0 ? c_slot0 : c_slot1;
#else
          const int slot = use0 ? cm.ref_slot[c8] : cm1.ref_slot1[c8];
#endif
          r0 = -1;
          for (int i = s->num_ref - 1; i >= 0; --i)
            if (s->ref_slot[i] == slot) r0 = i;
          if (r0 < 0) {
            bad = true;
            r0 = 0;
          }
        }
        int m0x = mcx, m0y = mcy, m1x = 0, m1y = 0;
        const int tb = clip3i(-128, 127, x.poc - x.poc0[r0]), td = clip3i(-128, 127, x.poc1[0] - x.poc0[r0]);
        if (!((x.lt0 >> r0) & 1u) && td != 0) {
          const int tx = (16384 + (td < 0 ? -td : td) / 2) / td;
          const int dsf = clip3i(-1024, 1023, (tb * tx + 32) >> 6);
          m0x = (dsf * mcx + 128) >> 8;
          m0y = (dsf * mcy + 128) >> 8;
          m1x = m0x - mcx;
          m1y = m0y - mcy;
        }
        set_motion(blk, r0, m0x, m0y);
        set_motion1(blk, 0, m1x, m1y);
      }
    }
    if (vts_any(bad)) err |= DEC_E_NO_REF;
  }

  VTS_HD VTS_INLINE void skip_mb(int addr, int qp) {
    begin_mb(addr);
    mv_border(addr);
    if (s->is_p == kSliceB) b_skip_body(addr, qp);
    else skip_body(addr, qp);
  }
  // B_Skip (8.4.1.2) of the macroblock begin_mb has started
  VTS_HD VTS_INLINE void b_skip_body(int addr, int qp) {
    cur().type = kMbSkip;
    cur().qp = static_cast<uint8_t>(qp);
    cur1().direct = 0x0f | kDirect16;
    direct_pred(addr, 0xffffu);
  }
  // P_Skip (8.4.1.1) of the macroblock begin_mb has started
  VTS_HD VTS_INLINE void skip_body(int addr, int qp) {
    MbRec &m = cur();
    m.type = kMbSkip;
    m.qp = static_cast<uint8_t>(qp);
    int xw, yw;
    const int a = nb_mb(addr, -1, 0, 16, &xw, &yw), b = nb_mb(addr, 0, -1, 16, &xw, &yw);
    const Mv A = nb_mv(addr, -1, 0, 0), B = nb_mv(addr, 0, -1, 0);
    int px = 0, py = 0;
    if (!(a == -1 || b == -1 || (A.ref == 0 && A.x == 0 && A.y == 0) || (B.ref == 0 && B.x == 0 && B.y == 0)))
      mv_pred(addr, 0, 0, 16, 16, 0, 0, &px, &py);
    if (s->ref_slot[0] < 0) err |= DEC_E_NO_REF;
    VTS_LANES(16, i) set_motion(i, 0, px, py);
  }

  // mb_pred / sub_mb_pred of a B macroblock (7.3.5.1-2, Tables 7-14, 7-18)
  // and its motion: partitions in order, list 0 before list 1 of each
  // (sub-)partition, direct partitions by 8.4.1.2 in place
  VTS_HD VTS_INLINE bool b_inter(int addr, int mb_type) {
    uint8_t *pm = sc->pm;
    int8_t *sub = sc->sub, *r0 = sc->refs, *r1 = sc->refs1;
    int shape;
    for (int k = 0; k < 4; ++k) {
      pm[k] = 0;
      sub[k] = 0;
      r0[k] = r1[k] = -1;
    }
    if (mb_type == 0) {  // B_Direct_16x16
      cur1().direct = 0x0f | kDirect16;
      direct_pred(addr, 0xffffu);
      return true;
    }
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
        const uint32_t v = br.ue();
        if (v > 12) {
          err |= DEC_E_SYNTAX;
          return false;
        }
        pm[k] = kBSub[v] & 3;
        sub[k] = static_cast<int8_t>(kBSub[v] >> 2);
      }
    }
    const int nparts = shape == 0 ? 1 : (shape < 3 ? 2 : 4);
    for (int l = 0; l < 2; ++l) {
      const int nref = l ? bc.x->num_ref1 : s->num_ref;
      int8_t *rr = l ? r1 : r0;
      for (int k = 0; k < nparts; ++k) {
        if (!((pm[k] >> l) & 1)) continue;
        const uint32_t rv = nref > 1 ? (nref == 2 ? static_cast<uint32_t>(!br.bit()) : br.ue()) : 0u;
        if (rv >= static_cast<uint32_t>(nref) || (l ? bc.x->ref_slot1[rv & 31] : s->ref_slot[rv & 31]) < 0) {
          err |= DEC_E_NO_REF;
          return false;
        }
        rr[k] = static_cast<int8_t>(rv);
      }
    }
    for (int l = 0; l < 2; ++l)
      for (int k = 0; k < nparts; ++k) {
        if (!((pm[k] >> l) & 1)) continue;
        const int nsub = shape < 3 ? 1 : (sub[k] == 0 ? 1 : (sub[k] == 3 ? 4 : 2));
        for (int q = 0; q < nsub; ++q) {
          sc->mvd[l][4 * k + q][0] = br.se();
          sc->mvd[l][4 * k + q][1] = br.se();
        }
      }
    for (int k = 0; k < 4; ++k)
      if (shape == 3 && pm[k] == 0) cur1().direct |= static_cast<uint8_t>(1u << k);
    return b_motion(addr, shape);
  }

  // the motion of a B macroblock from sc->pm / sub / refs / refs1 / mvd:
  // partitions in order, list 0 before list 1 of each (sub-)partition, direct
  // quadrants by 8.4.1.2 in place
  VTS_HD VTS_INLINE bool b_motion(int addr, int shape) {
    const uint8_t *pm = sc->pm;
    const int8_t *sub = sc->sub, *r0 = sc->refs, *r1 = sc->refs1;
    const int nparts = shape == 0 ? 1 : (shape < 3 ? 2 : 4);
    uint32_t done = 0;
    for (int k = 0; k < nparts; ++k) {
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
      if (pm[k] == 0) {  // B_Direct_8x8
        const uint32_t bm = 0x33u << ((y0 / 4) * 4 + x0 / 4);
        direct_pred(addr, bm);
        if (err) return false;
        done |= bm;
        continue;
      }
      for (int q = 0; q < nsub; ++q) {
        int sx = x0, sy = y0;
        if (shape == 3) {
          if (sub[k] == 1) sy += 4 * q;
          else if (sub[k] == 2) sx += 4 * q;
          else if (sub[k] == 3) { sx += 4 * (q & 1); sy += 4 * (q >> 1); }
        }
        int v[2][2] = {{0, 0}, {0, 0}};
#pragma unroll
        for (int l = 0; l < 2; ++l) {
          if (!((pm[k] >> l) & 1)) continue;
          int px, py;
          mv_pred(addr, sx, sy, pw, ph, l ? r1[k] : r0[k], done, &px, &py, l);
          v[l][0] = px + sc->mvd[l][4 * k + q][0];
          v[l][1] = py + sc->mvd[l][4 * k + q][1];
          if (v[l][0] < -32768 || v[l][0] > 32767 || v[l][1] < -32768 || v[l][1] > 32767) {
            err |= DEC_E_SYNTAX;
            return false;
          }
        }
        const uint32_t bm = blk_mask(sx, sy, pw, ph);
        const int ra = (pm[k] & 1) ? r0[k] : -1, rb = (pm[k] & 2) ? r1[k] : -1;
        VTS_LANES(16, b) if ((bm >> b) & 1u) {
          set_motion(b, ra, v[0][0], v[0][1]);
          set_motion1(b, rb, v[1][0], v[1][1]);
        }
        done |= bm;
      }
    }
    return true;
  }

  // macroblock_layer(); returns false to stop the slice
  VTS_HD VTS_INLINE bool mb_layer(int addr, int *qp) {
    begin_mb(addr);
    if (s->is_p) mv_border(addr);
    MbRec &m = cur();
    const int mb_type = static_cast<int>(br.ue());
    const int intra0 = s->is_p == kSliceB ? 23 : (s->is_p ? 5 : 0);  // Tables 7-11, 7-13, 7-14
    const int itype = mb_type - intra0;  // < 0: inter
    if (mb_type > intra0 + 25) {
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
      todo = 0;
      return true;
    }
    int cbp = 0;
    bool i16 = false;
    if (itype == 0) {  // I_NxN
      m.type = kMbI4x4;
      uint8_t *prev = sc->prev, *rem = sc->rem;
      for (int k = 0; k < 16; ++k) {
        prev[k] = static_cast<uint8_t>(br.bit());
        rem[k] = prev[k] ? 0 : static_cast<uint8_t>(br.bits(3));
      }
      for (int k = 0; k < 16; ++k) {
        const int bx = blk_x(k), by = blk_y(k);
        int xa, ya, xb, yb;
        const int a = nb_mb(addr, bx * 4 - 1, by * 4, 16, &xa, &ya);
        const int b = nb_mb(addr, bx * 4, by * 4 - 1, 16, &xb, &yb);
        int pred = 2;
        bool dcf = a == -1 || b == -1;
        if (!dcf && cip) {
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
    } else if (s->is_p == kSliceB) {
      m.type = kMbInter;
      if (!b_inter(addr, mb_type)) return false;
    } else {  // inter
      m.type = kMbInter;
      const int nparts = mb_type == 0 ? 1 : (mb_type <= 2 ? 2 : 4);
      int8_t *sub = sc->sub, *refs = sc->refs;
      for (int k = 0; k < 4; ++k) sub[k] = refs[k] = 0;
      if (mb_type >= 3)
        for (int k = 0; k < 4; ++k) {
          const uint32_t sv = br.ue();
          sub[k] = static_cast<int8_t>(sv & 7);
          if (sv > 3) {
            err |= DEC_E_SYNTAX;
            return false;
          }
        }
      const int nref = s->num_ref;
      if (mb_type != 4 && nref > 1)
        for (int k = 0; k < nparts; ++k) {
          const uint32_t rv = nref == 2 ? static_cast<uint32_t>(!br.bit()) : br.ue();
          refs[k] = static_cast<int8_t>(rv > 127 ? 127 : rv);
        }
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
          const uint32_t bm = blk_mask(sx, sy, pw, ph);
          const int rk = refs[k];
          VTS_LANES(16, b) if ((bm >> b) & 1u) set_motion(b, rk, vx, vy);
          done |= bm;
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
    // residual blocks (7.3.5.3), in bitstream order = kBlk* bit order; they are
    // decoded one per step of the slice loop (block_step)
    uint32_t t = 0;
    if (i16) t |= 1u << kBlkI16Dc;
    for (int q = 0; q < 4; ++q)
      if ((cbp >> q) & 1) t |= 15u << (kBlkLuma0 + 4 * q);
    if (cbp >> 4) t |= 3u << kBlkChromaDc0;
    if ((cbp >> 4) & 2) t |= 255u << kBlkChromaAc0;
    todo = t;
    cur_i16 = i16;
    if (br.err || br.overrun()) {
      err |= DEC_E_SYNTAX;
      return false;
    }
    return true;
  }

  // one residual block of the current macroblock (the lowest bit of todo);
  // returns false to stop the slice
  VTS_HD VTS_INLINE bool block_step(int addr) {
    const uint32_t bt = static_cast<uint32_t>(__builtin_ctz(todo));
    todo &= todo - 1u;
    MbRec &m = cur();
    int nC = -1, maxNum = 15, start = 1;
    const bool luma = bt < kBlkChromaDc0, chroma_ac = bt >= kBlkChromaAc0;
    const int k = bt >= kBlkLuma0 && luma ? static_cast<int>(bt) - kBlkLuma0 : 0;
    const int j = chroma_ac ? static_cast<int>(bt) - kBlkChromaAc0 : 0;
    if (luma) {
      nC = nc_of(addr, blk_x(k), blk_y(k), false, 0);
      if (bt == kBlkI16Dc || !cur_i16) {
        maxNum = 16;
        start = 0;
      }
    } else if (chroma_ac) {
      nC = nc_of(addr, j & 3 & 1, (j & 3) >> 1, true, j >> 2);
    } else {
      maxNum = 4;
      start = 0;
    }
    const int tc = residual_block(nC, maxNum, start);
    if (tc < 0 || br.err) {
      err |= DEC_E_SYNTAX;
      return false;
    }
    if (bt >= kBlkLuma0 && luma) m.nz[blk_y(k) * 4 + blk_x(k)] = static_cast<uint8_t>(tc);
    if (chroma_ac) m.nzc[j] = static_cast<uint8_t>(tc);
    if (tc > 0) {
      if (!luma && !chroma_ac) {  // chroma DC levels in list order (not zig-zag): undo the scan
        int16_t lv[4];
        for (int i = 0; i < 4; ++i) lv[i] = sc->blk[kZz[i]];
        for (int i = 0; i < 16; ++i) sc->blk[i] = i < 4 ? lv[i] : 0;
      }
      if (!store_block(bt)) {
        err |= DEC_E_SYNTAX;
        return false;
      }
    }
    return true;
  }
};

// Parse slice `s` (window slice index si) into recs (the frame's records) and
// the arena.  rbsp = the slice NAL's payload with its emulation-prevention
// bytes removed (rbsp_len bytes).  Returns DEC_E_* bits.
VTS_HD VTS_INLINE uint32_t parse_slice_full(const uint8_t *rbsp, int32_t rbsp_len, const FullSlice &s, uint32_t si,
                                        const FullParams P, MbRec *frame_recs, uint16_t *frame_ilvl, int16_t *arena,
                                        uint32_t epoch, FullScratch *sc, const BCtx &bc) {
  Parser p;
  p.s = &s;
  p.cip = P.cip;
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
  p.bc = bc;
  p.bframes = P.bframes;
  p.direct8x8 = P.direct8x8;
  const int nmb = P.mb_width * P.mb_height;
  if (s.is_p == kSliceB && (!bc.x || !bc.col || !P.bframes)) return DEC_E_NO_REF;
  int32_t last = rbsp_len - 1;  // the stop bit's byte
  while (last >= 0 && rbsp[last] == 0) --last;
  if (last < 0) return DEC_E_SYNTAX;
  const int64_t stop_bit = int64_t(last) * 8 + (7 - __builtin_ctz(static_cast<uint32_t>(rbsp[last])));
  p.br.init(rbsp, rbsp_len, sc->cache);
  p.refresh_lane();
  p.br.reset_at(s.data_bit);
  p.todo = 0;
  p.cur_i16 = false;
  // slice_data() as a state machine whose every iteration does one small step
  // (a skipped macroblock, a macroblock header, or one residual block), so the
  // lanes of a wave - each parsing its own slice - meet again in the same
  // code at every iteration instead of serialising whole macroblocks
  enum { kRun, kSkip, kHeader, kBlock };
  int addr = s.first_mb, qp = s.qp, run = 0;
  int state = s.is_p ? kRun : kHeader;
  if (addr >= nmb) p.err |= DEC_E_SYNTAX;
  while (!p.err) {
    p.refresh_lane();
    bool finish = false;  // the current macroblock is complete
    if (state == kBlock) {
      if (!p.block_step(addr)) break;
      finish = p.todo == 0;
    } else if (state == kRun) {
      run = static_cast<int>(p.br.ue());
      if (p.br.err || addr + run > nmb) {
        p.err |= DEC_E_SYNTAX;
        break;
      }
      state = run > 0 ? kSkip : kHeader;
      if (state == kHeader && addr >= nmb) {
        p.err |= DEC_E_SYNTAX;
        break;
      }
    } else if (state == kSkip) {
      p.skip_mb(addr, qp);
      p.end_mb(addr);
      ++addr;
      if (--run == 0) {
        if (!p.br.more(stop_bit)) break;
        if (addr >= nmb) {
          p.err |= DEC_E_SYNTAX;
          break;
        }
        state = kHeader;
      }
    } else {
      if (!p.mb_layer(addr, &qp)) break;
      state = kBlock;
      finish = p.todo == 0;
    }
    if (finish) {
      p.end_mb(addr);
      ++addr;
      if (!p.br.more(stop_bit)) break;
      if (addr >= nmb) {
        p.err |= DEC_E_SYNTAX;
        break;
      }
      state = s.is_p ? kRun : kHeader;
    }
  }
  if (!p.err && (p.br.err || p.br.overrun() || p.br.consumed() != stop_bit)) p.err |= DEC_E_SYNTAX;
  return p.err;
}

}  // namespace full
}  // namespace vts
