// decode_full.hip — kernels of the general H.264 decoder (CAVLC I/P: intra
// 4x4 / 16x16 / chroma prediction, residuals, quarter-sample motion over up to
// 16 references, the deblocking filter).  DESIGN.md §5b.
//
//   h264_parse_full   one wave per slice: slice_data() -> MbRec + coefficient
//                     blocks + intra dependency level (CAVLC, parse_full.h)
//   h264_parse_full_cabac  one wave per slice: CABAC slice_data() -> syntax
//                     records + coefficient blocks (parse_cabac.h)
//   h264_derive       one workgroup per picture, one lane per macroblock row
//                     on the x + 2y wavefront: motion, intra modes and
//                     levels from the syntax records (derive_full.h)
//   h264_inter_full   one lane per 4x4 luma block (+ its 2x2 Cb/Cr) of every
//                     inter / skip / I_PCM macroblock of every picture of the
//                     level: 6-tap / bilinear prediction from dword windows,
//                     residual, one dword store per row
//   h264_intra_full   one workgroup per picture: the intra-predicted
//                     macroblocks by dependency level (the parser's level =
//                     1 + the highest level among the intra neighbours it
//                     reads; an all-intra picture gives the x + 2y wavefront),
//                     16 lanes per macroblock, its borders and 4x4 blocks in LDS
//   h264_bs_full      16 lanes per macroblock: bS of every edge + the edge
//                     filter parameters into a 96-byte descriptor
//   h264_deblock_plane one workgroup per (picture, plane), 16 lanes per
//                     macroblock row, the rows two macroblocks apart (8.7's
//                     raster order as a wavefront), rows above through LDS
// Per-macroblock arithmetic (transforms, interpolation, intra modes, edge
// filters) follows the same clauses as recon_full.h, which the CPU harness
// runs against the oracle.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "common.h"
#include "decode_full.h"
#if !defined(__HIP_DEVICE_COMPILE__)
#endif
#include "parse_cabac.h"
#include "parse_full.h"
#include "derive_full.h"
#include "recon_full.h"
#include "intra_lanes.h"

namespace vts {
namespace {

constexpr int kInterThreads = 256;   // 16 macroblocks x 16 blocks
#ifndef VTS_INTRA_THREADS
#define VTS_INTRA_THREADS 512
#endif
#ifndef VTS_DBK_THREADS
#define VTS_DBK_THREADS 1024
#endif
constexpr int kIntraThreads = VTS_INTRA_THREADS;  // 512: 32 macroblocks in flight (2 waves per SIMD, <= 256 VGPRs)
constexpr int kIntraSlots = kIntraThreads / 16;
constexpr int kIntraLevels = 512;  // intra dependency levels bucketed in LDS (more: one scan per level)
constexpr int kDbkThreads = VTS_DBK_THREADS;      // 1024: 16 waves = 16 row pairs in flight
constexpr int kDbkWaves = kDbkThreads / 64;
// (a 256-thread build, 16 rows in flight, hung on the noise stream: its ring
// hand-off between waves needs more rows in flight than one pass of 4 waves;
// 512 ran, no faster: profiles/r06ar_*)
static_assert(kDbkThreads >= 512 && kDbkThreads <= 1024 && kDbkThreads % 64 == 0, "deblocking workgroup size");
// experiment hook: per-workgroup start / end of the one-workgroup-per-picture
// kernels (tools/exp/wg_trace.h); nothing in the product build
#ifndef VTS_WG_TRACE
#define VTS_WG_TRACE(kernel, end, key) ((void)0)
#endif

// One slice per wave: every value of the parse is
// wave-uniform, so control flow never diverges and the integer work can go to
// the scalar unit; the parallelism is the window's slices (thousands of waves).
// 4 waves per SIMD.  Since the CABAC engine's arithmetic moved to the vector
// ALUs, 5 (<= 102 VGPRs, a few spilled) times faster: parse -6.5 % CABAC,
// -8.7 % CAVLC (3: +13 %; profiles/r03_parse_waves_ab.txt); it becomes the
// default once the GPU parity suite has run on a 5-wave build
// (-DVTS_PARSE_WAVES=5 builds it)
#ifndef VTS_PARSE_WAVES
#define VTS_PARSE_WAVES 5
#endif
// The entropy mode is per stream, so each mode is its own kernel: a wave only
// ever runs one parser's code, and each fits the instruction cache better.
// CAVLC (parse_full.h) derives motion, modes and levels inline and a B slice
// waits for its colocated picture's records; CABAC (parse_cabac.h) writes
// syntax records only, completed per picture by h264_derive, so its slices
// are independent.
__device__ __forceinline__ void parse_one_cavlc(const FullParseArgs &a, full::FullScratch *scratch) {
  const int i = a.order ? a.order[blockIdx.x] : static_cast<int>(blockIdx.x);
  const FullSlice &s = a.slices[i];
  const FullParams P = a.P;
  const int64_t nmb = static_cast<int64_t>(P.mb_width) * P.mb_height;
  full::BCtx bc{};
  if (P.bframes) bc.recs1 = a.recs1 + s.slot * nmb;
  if (s.ext >= 0) bc.x = a.exts + s.ext;
  if (s.is_p == kSliceB && bc.x) {  // colocated picture: RefPicList1[0], parsed earlier
    const int col = bc.x->ref_slot1[0];
    bc.col = a.recs + col * nmb;
    bc.col1 = a.recs1 + col * nmb;
    if (a.pdone) {
      // merged launch: the colocated picture's slices have lower workgroup
      // indices (dispatched first on every XCD), so this wait ends; bounded
      // anyway (~3 s), then DEC_E_COL_WAIT fails the run (the slice's direct
      // prediction would read a partly written colocated record)
      const uint32_t need = static_cast<uint32_t>(a.pneed[col]);
      uint32_t spins = 0;
      while (__hip_atomic_load(&a.pdone[col], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
        if (++spins > (1u << 25)) {
          atomicOr(a.err, static_cast<uint32_t>(DEC_E_COL_WAIT));
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the colocated records, across XCD L2s
    }
  }
  const uint32_t e = full::parse_slice_full(a.rbsp + s.nal_offset + 1, a.rbsp_len[i], s,
                                            static_cast<uint32_t>(a.slice0 + i), P, a.recs + s.slot * nmb,
                                            a.ilvl + s.slot * nmb, a.arena, a.epoch, scratch, bc);
  if (e) atomicOr(a.err, e);
  if (a.pdone) {  // this slice's records are out (every path, errors included)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (threadIdx.x == 0) __hip_atomic_fetch_add(&a.pdone[s.slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// A wave of 64 lanes that all run the same (uniform) parse: the parser's state
// is scalar, and full EXEC keeps the lane tables (LaneTab, parse_full.h) whole
// through every VGPR copy the compiler makes (a copy under a one-lane EXEC
// would move lane 0 only).  Stores of the same value to the same address from
// every lane coalesce into one.
__global__ void __launch_bounds__(64)
__attribute__((amdgpu_waves_per_eu(VTS_PARSE_WAVES, VTS_PARSE_WAVES))) h264_parse_full(FullParseArgs a) {
  __shared__ full::FullScratch scratch;
  parse_one_cavlc(a, &scratch);
}
// dynamic LDS: full::syn_lds_bytes(mb_width) (SynScratch + the row of top
// edges)
__global__ void __launch_bounds__(64)
__attribute__((amdgpu_waves_per_eu(VTS_PARSE_WAVES, VTS_PARSE_WAVES))) h264_parse_full_cabac(FullParseArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t syn_lds[];
  const int i = a.order ? a.order[blockIdx.x] : static_cast<int>(blockIdx.x);
  const FullSlice &s = a.slices[i];
  const FullParams P = a.P;
  const int64_t nmb = static_cast<int64_t>(P.mb_width) * P.mb_height;
  const uint32_t e = full::parse_slice_cabac(a.rbsp + s.nal_offset + 1, a.rbsp_len[i], s,
                                             static_cast<uint32_t>(a.slice0 + i), P, a.recs + s.slot * nmb,
                                             P.bframes ? a.recs1 + s.slot * nmb : nullptr,
                                             s.ext >= 0 ? a.exts + s.ext : nullptr, a.arena, a.arena_top,
                                             a.arena_blocks, a.epoch, reinterpret_cast<full::SynScratch *>(syn_lds));
  if (e) atomicOr(a.err, e);
}

// One workgroup per picture, one lane per macroblock row: at step t row y
// derives macroblock x = t - 2y (derive_full.h), so the row above has
// finished x - 1, x and x + 1 (its bottom edges in an LDS ring of four
// columns per row) and the lane's own previous macroblock is its left edge;
// a barrier per step.  Dynamic LDS: derive_lds_bytes.
__global__ void __launch_bounds__(256) h264_derive(DeriveArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t dlds[];
  const int mbw = a.P.mb_width, mbh = a.P.mb_height;
  const int64_t nmb = static_cast<int64_t>(mbw) * mbh;
  const int2 pic = a.pics[blockIdx.x];
  const int slot = pic.x;
  full::DWork *work = reinterpret_cast<full::DWork *>(dlds);                   // [blockDim]
  full::DEdge *ring = reinterpret_cast<full::DEdge *>(work + blockDim.x);      // [mbh][4]
  full::DEdge *left = ring + 4 * mbh;                                          // [mbh]
  full::DeriveCtx c;
  c.recs = a.recs + slot * nmb;
  c.recs1 = a.P.bframes ? a.recs1 + slot * nmb : nullptr;
  c.ilvl = a.ilvl + slot * nmb;
  c.ring = a.recs;
  c.ring1 = a.recs1;
  c.slices = a.slices;
  c.exts = a.exts;
  c.mbw = mbw;
  c.mbh = mbh;
  c.epoch = a.epoch;
  c.cip = a.P.cip;
  c.direct8x8 = a.P.direct8x8;
  c.bframes = a.P.bframes;
  c.col = pic.y;
  const int y = static_cast<int>(threadIdx.x);
  uint32_t err = 0;
  const int steps = mbw + 2 * (mbh - 1);
  full::DIn nxt;  // the lane's next macroblock's words, loaded one step ahead
  for (int t = 0; t < steps; ++t) {
    const int x = t - 2 * y;
    if (y < mbh && x >= 0 && x < mbw) {
      full::DIn in;
      if (x == 0) full::derive_load(c, y * mbw, in);
      else in = nxt;
      if (x + 1 < mbw) full::derive_load(c, y * mbw + x + 1, nxt);
      const full::DEdge *A = x > 0 ? &left[y] : nullptr;
      const full::DEdge *B = y > 0 ? &ring[4 * (y - 1) + (x & 3)] : nullptr;
      const full::DEdge *C = y > 0 && x + 1 < mbw ? &ring[4 * (y - 1) + ((x + 1) & 3)] : nullptr;
      const full::DEdge *D = y > 0 && x > 0 ? &ring[4 * (y - 1) + ((x - 1) & 3)] : nullptr;
      // the right edge replaces the left one (derive_mb writes its edges last)
      err |= full::derive_mb(c, y * mbw + x, in, A, B, C, D, work[y], &left[y], &ring[4 * y + (x & 3)]);
    }
    __syncthreads();
  }
  if (err) atomicOr(a.err, err);
}

// 7.4.1: one workgroup per slice NAL, 256 payload bytes per step; a byte is
// an emulation-prevention byte by full::is_epb (a local rule), its output
// index is its own minus the EPBs before it (wave ballots + a 4-entry scan)
constexpr int kUnescThreads = 256;
__global__ void __launch_bounds__(kUnescThreads) nal_unescape(const uint8_t *es, uint8_t *rbsp, const FullSlice *sl,
                                                              int32_t *lens) {
  __shared__ int wcnt[kUnescThreads / 64];
  const FullSlice &s = sl[blockIdx.x];
  const uint8_t *in = es + s.nal_offset + 1;
  uint8_t *out = rbsp + s.nal_offset + 1;
  const int32_t n = s.nal_size - 1;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int32_t removed = 0;
  for (int32_t c0 = 0; c0 < n; c0 += kUnescThreads) {
    const int32_t j = c0 + static_cast<int32_t>(threadIdx.x);
    const bool in_range = j < n;
    const uint8_t b = in_range ? in[j] : 0;
    const bool epb = in_range && full::is_epb(in, j);
    const uint64_t m = __ballot(epb);
    if (lane == 0) wcnt[w] = __popcll(m);
    __syncthreads();
    int before = removed + __popcll(m & ((1ull << lane) - 1ull)), total = 0;
#pragma unroll
    for (int k = 0; k < kUnescThreads / 64; ++k) {
      before += k < w ? wcnt[k] : 0;
      total += wcnt[k];
    }
    if (in_range && !epb) out[j - before] = b;
    __syncthreads();
    removed += total;
  }
  if (threadIdx.x == 0) lens[blockIdx.x] = n - removed;
}

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ int c255(int v) { return min(max(v, 0), 255); }
__device__ __forceinline__ int t6(int a, int b, int c, int d, int e, int f) {
  return a - 5 * b + 20 * c + 20 * d - 5 * e + f;
}
template <int N>
__device__ __forceinline__ int px(const uint32_t (&w)[9][N], int r, int c) {
  return (w[r][c >> 2] >> ((c & 3) * 8)) & 255;
}
__device__ __forceinline__ uint32_t pack4(int a, int b, int c, int d) {
  return static_cast<uint32_t>(a) | (static_cast<uint32_t>(b) << 8) | (static_cast<uint32_t>(c) << 16) |
         (static_cast<uint32_t>(d) << 24);
}
// luma4x4BlkIdx of raster 4x4 block b
__device__ __forceinline__ int blkidx(int b) {
  return ((b >> 3) << 3) | (((b & 3) >> 1) << 2) | (((b >> 2) & 1) << 1) | (b & 1);
}
// arena block of stored-block bit `bit` of a macroblock, -1 if absent
__device__ __forceinline__ int64_t stored(uint32_t blocks, uint32_t coef, uint32_t bit) {
  if (!((blocks >> bit) & 1u)) return -1;
  return static_cast<int64_t>(coef) + __builtin_popcount(blocks & ((1u << bit) - 1u));
}
__device__ __forceinline__ void load_coefs(const int16_t *arena, int64_t blk, int *cf) {
  if (blk < 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) cf[i] = 0;
    return;
  }
  const uint4 *p = reinterpret_cast<const uint4 *>(arena + 16 * blk);
  const uint4 u0 = p[0], u1 = p[1];
  const uint32_t w[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    cf[2 * i] = static_cast<int16_t>(w[i] & 0xffff);
    cf[2 * i + 1] = static_cast<int16_t>(w[i] >> 16);
  }
}

// 9x9 luma window w[r][c] = R[clampY(ys + r)][clampX(xs + c)], 3 packed dwords per row
__device__ __forceinline__ void load_win9(const uint8_t *R, int pitch, int W, int H, int xs, int ys,
                                          uint32_t (&w)[9][3]) {
  if (xs >= 0 && xs + 8 < W && ys >= 0 && ys + 8 < H) {
    const int sh = xs & 3;
    const uint8_t *p = R + static_cast<int64_t>(ys) * pitch + (xs & ~3);
#pragma unroll
    for (int r = 0; r < 9; ++r) {
      const uint32_t *q = reinterpret_cast<const uint32_t *>(p + static_cast<int64_t>(r) * pitch);
      const uint32_t d0 = q[0], d1 = q[1], d2 = q[2];
      w[r][0] = __builtin_amdgcn_alignbyte(d1, d0, sh);
      w[r][1] = __builtin_amdgcn_alignbyte(d2, d1, sh);
      w[r][2] = d2 >> (8 * sh);
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    const uint8_t *row = R + static_cast<int64_t>(min(max(ys + r, 0), H - 1)) * pitch;
    uint32_t v[3] = {0, 0, 0};
#pragma unroll
    for (int c = 0; c < 9; ++c) v[c >> 2] |= static_cast<uint32_t>(row[min(max(xs + c, 0), W - 1)]) << ((c & 3) * 8);
    w[r][0] = v[0];
    w[r][1] = v[1];
    w[r][2] = v[2];
  }
}

// 8.4.2.2.1 with one instruction stream for every fractional offset: every
// intermediate a 4x4 block can need (the 6-tap rows 0..8 for j, b / s, the
// 6-tap columns for h / m) computed once, the sample chosen by selects, so a
// wave whose lanes sit at different offsets runs no branch bodies one after
// another (profiles/r03_luma_unified_ab.txt); integer motion keeps its copy
__device__ __forceinline__ void luma_pred4(const uint32_t (&w)[9][3], int xf, int yf, int (&v)[16]) {
  if (!(xf | yf)) {
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int x = 0; x < 4; ++x) v[y * 4 + x] = px(w, y + 2, x + 2);
    return;
  }
  // one output row at a time, so only six rows of horizontal intermediates
  // (and the row's vertical ones) are live at once: 6-tap row r is made just
  // before output row r - 5 first needs it
  int hr[9][4];
  auto hrow = [&](int r) {
#pragma unroll
    for (int x = 0; x < 4; ++x) hr[r][x] = t6(px(w, r, x), px(w, r, x + 1), px(w, r, x + 2), px(w, r, x + 3), px(w, r, x + 4), px(w, r, x + 5));
  };
#pragma unroll
  for (int r = 0; r < 5; ++r) hrow(r);
  const bool x0 = xf == 0, y0 = yf == 0, x2 = xf == 2, y2 = yf == 2, x3 = xf == 3, y3 = yf == 3;
#pragma unroll
  for (int y = 0; y < 4; ++y) {
    hrow(y + 5);
    int vt[5];
#pragma unroll
    for (int c = 0; c < 5; ++c) vt[c] = t6(px(w, y, c + 2), px(w, y + 1, c + 2), px(w, y + 2, c + 2), px(w, y + 3, c + 2), px(w, y + 4, c + 2), px(w, y + 5, c + 2));
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int b = c255((hr[y + 2][x] + 16) >> 5), s_ = c255((hr[y + 3][x] + 16) >> 5);
      const int h = c255((vt[x] + 16) >> 5), m = c255((vt[x + 1] + 16) >> 5);
      const int j = c255((t6(hr[y][x], hr[y + 1][x], hr[y + 2][x], hr[y + 3][x], hr[y + 4][x], hr[y + 5][x]) + 512) >> 10);
      const int G = px(w, y + 2, x + 2), G1 = px(w, y + 2, x + 3), G2 = px(w, y + 3, x + 2);
      const int bs = y3 ? s_ : b, hm = x3 ? m : h;
      int P, Q;
      bool full;
      if (x0) {
        P = h;
        Q = y3 ? G2 : G;
        full = y2;
      } else if (y0) {
        P = b;
        Q = x3 ? G1 : G;
        full = x2;
      } else if (x2 || y2) {
        P = j;
        Q = x2 ? bs : hm;
        full = x2 && y2;
      } else {
        P = bs;
        Q = hm;
        full = false;
      }
      v[y * 4 + x] = full ? P : (P + Q + 1) >> 1;
    }
  }
}

// 8.5.12.1 chroma DC of chroma block ck: 2x2 Hadamard of the plane's DC levels, scaled
__device__ __forceinline__ int chroma_dc(const int16_t *arena, uint32_t blocks, uint32_t coef, int pl, int ck,
                                         int qpc, const int32_t *ls) {
  const int64_t blk = stored(blocks, coef, kBlkChromaDc0 + pl);
  if (blk < 0) return 0;
  const uint2 u = *reinterpret_cast<const uint2 *>(arena + 16 * blk);
  const int c0 = static_cast<int16_t>(u.x & 0xffff), c1 = static_cast<int16_t>(u.x >> 16);
  const int c2 = static_cast<int16_t>(u.y & 0xffff), c3 = static_cast<int16_t>(u.y >> 16);
  const int f = ck == 0 ? c0 + c1 + c2 + c3 : ck == 1 ? c0 - c1 + c2 - c3 : ck == 2 ? c0 + c1 - c2 - c3 : c0 - c1 - c2 + c3;
  return ((f * ls[0]) << (qpc / 6)) >> 5;
}
// chroma residual of one 4x4 chroma block of plane pl
// (ls: LevelScale4x4(qPc % 6, .) of the plane's list, 8.5.9)
__device__ __forceinline__ void chroma_res(const int16_t *arena, uint32_t blocks, uint32_t coef, int pl, int ck,
                                           int qpc, const int32_t *ls, int (&r)[16]) {
  int cf[16];
  load_coefs(arena, stored(blocks, coef, kBlkChromaAc0 + 4 * pl + ck), cf);
  cf[0] = chroma_dc(arena, blocks, coef, pl, ck, qpc, ls);
  full::scale_idct4(cf, qpc, ls, true, r);
}
// LevelScale4x4(qP % 6, .) of a 4x4 block of plane pl (0 Y) in an intra or
// inter macroblock: the stream's table (flat values without scaling matrices)
__device__ __forceinline__ const int32_t *ls4_of(const FullReconArgs &a, bool intra, int pl, int qp) {
  return a.sct->ls4[scale_list4(intra, pl)][qp % 6];
}

// 8.5.13 for one 4x4 quarter (qx, qy) of an 8x8 block stored as raster rows
// in the arena (4 consecutive blocks): all 8 rows transformed, then this
// quarter's 4 columns
// (ls8: LevelScale8x8(qP % 6, .) of the list when the stream has scaling
// matrices, else null: Flat_16 from normAdjust8x8's six values)
__device__ __forceinline__ void idct8_quarter(const int16_t *arena, int64_t blk, int qp, int qx, int qy,
                                              const int32_t *ls8, int (&res)[16]) {
  int n8[6];
#pragma unroll
  for (int c = 0; c < 6; ++c) n8[c] = 16 * full::kNorm8[qp % 6][c];
  const int sh = qp / 6;
  int t[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint4 u = *reinterpret_cast<const uint4 *>(arena + 16 * blk + 8 * i);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
    int v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = static_cast<int16_t>((w[j >> 1] >> ((j & 1) * 16)) & 0xffff);
      const int ls = ls8 ? ls8[i * 8 + j] : n8[vts_norm8_class(i, j)];
      v[j] = qp >= 36 ? (c * ls) << (sh - 6) : (c * ls + (1 << (5 - sh))) >> (6 - sh);
    }
    const int a0 = v[0] + v[4], a4 = v[0] - v[4], a2 = (v[2] >> 1) - v[6], a6 = v[2] + (v[6] >> 1);
    const int b0 = a0 + a6, b2 = a4 + a2, b4 = a4 - a2, b6 = a0 - a6;
    const int a1 = -v[3] + v[5] - v[7] - (v[7] >> 1), a3 = v[1] + v[7] - v[3] - (v[3] >> 1);
    const int a5 = -v[1] + v[7] + v[5] + (v[5] >> 1), a7 = v[3] + v[5] + v[1] + (v[1] >> 1);
    const int b1 = a1 + (a7 >> 2), b7 = a7 - (a1 >> 2), b3 = a3 + (a5 >> 2), b5 = (a3 >> 2) - a5;
    const int o[8] = {b0 + b7, b2 + b5, b4 + b3, b6 + b1, b6 - b1, b4 - b3, b2 - b5, b0 - b7};
#pragma unroll
    for (int k = 0; k < 4; ++k) t[i][k] = qx ? o[4 + k] : o[k];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int a0 = t[0][k] + t[4][k], a4 = t[0][k] - t[4][k], a2 = (t[2][k] >> 1) - t[6][k], a6 = t[2][k] + (t[6][k] >> 1);
    const int b0 = a0 + a6, b2 = a4 + a2, b4 = a4 - a2, b6 = a0 - a6;
    const int a1 = -t[3][k] + t[5][k] - t[7][k] - (t[7][k] >> 1), a3 = t[1][k] + t[7][k] - t[3][k] - (t[3][k] >> 1);
    const int a5 = -t[1][k] + t[7][k] + t[5][k] + (t[5][k] >> 1), a7 = t[3][k] + t[5][k] + t[1][k] + (t[1][k] >> 1);
    const int b1 = a1 + (a7 >> 2), b7 = a7 - (a1 >> 2), b3 = a3 + (a5 >> 2), b5 = (a3 >> 2) - a5;
    const int o[8] = {b0 + b7, b2 + b5, b4 + b3, b6 + b1, b6 - b1, b4 - b3, b2 - b5, b0 - b7};
#pragma unroll
    for (int r = 0; r < 4; ++r) res[r * 4 + k] = ((qy ? o[4 + r] : o[r]) + 32) >> 6;
  }
}

// MbRec header words (the first 32 bytes)
struct MbHdr {
  uint32_t epoch, slice, coef, blocks;
  int type, qp, cbp, modes;
  uint32_t refs;            // ref[4] bytes
  int16_t ref_slot[4];
};
__device__ __forceinline__ MbHdr load_hdr(const MbRec *m) {
  const uint4 *p = reinterpret_cast<const uint4 *>(m);
  const uint4 a = p[0], b = p[1];
  MbHdr h;
  h.epoch = a.x;
  h.slice = a.y;
  h.coef = a.z;
  h.blocks = a.w;
  h.type = b.x & 255;
  h.qp = (b.x >> 8) & 255;
  h.cbp = (b.x >> 16) & 255;
  h.modes = b.x >> 24;
  h.refs = b.y;
  h.ref_slot[0] = static_cast<int16_t>(b.z & 0xffff);
  h.ref_slot[1] = static_cast<int16_t>(b.z >> 16);
  h.ref_slot[2] = static_cast<int16_t>(b.w & 0xffff);
  h.ref_slot[3] = static_cast<int16_t>(b.w >> 16);
  return h;
}

// The NV12 surface of window slot `slot`: the slot itself, or the surface the
// host's liveness plan gave it (FullReconArgs::surf_of, recycled surfaces)
__device__ __forceinline__ uint8_t *surf_at(const FullReconArgs &a, int slot) {
  const int s = (a.surf_of && slot >= 0) ? a.surf_of[slot] : slot;
  return a.surf + static_cast<int64_t>(s) * a.frame_stride;
}

// one list's prediction of a 4x4 luma block at (x0, y0) and its 2x2 Cb / Cr at
// (cx, cy) from the picture in ring slot rs, motion mvw = mvx | mvy << 16
// (8.4.2.2.1 luma 6-tap, 8.4.2.2.2 chroma bilinear; windows edge-clamped).
// The results are packed bytes (pvp: one dword per row; cpp: Cb, Cr dwords
// of 2x2 samples, raster) and the chroma window is loaded only after the luma
// prediction: 155 -> 128 VGPRs in h264_inter_full, occupancy 3 -> 4 waves
// per SIMD (profiles/r05af_inter_packed_ab.json)
__device__ __forceinline__ void pred_ref(const FullReconArgs &a, int rs, uint32_t mvw, int x0, int y0, int cx,
                                            int cy, int W, int H, uint32_t (&pvp)[4], uint32_t (&cpp)[2]) {
  const int mvx = static_cast<int16_t>(mvw & 0xffff), mvy = static_cast<int16_t>(mvw >> 16);
  const int pitch = a.pitch;
  const uint8_t *R = surf_at(a, rs);
  {
    uint32_t w[9][3];
    load_win9(R, pitch, W, H, x0 + (mvx >> 2) - 2, y0 + (mvy >> 2) - 2, w);
    int pv[16];
    luma_pred4(w, mvx & 3, mvy & 3, pv);
#pragma unroll
    for (int r = 0; r < 4; ++r) pvp[r] = pack4(pv[r * 4], pv[r * 4 + 1], pv[r * 4 + 2], pv[r * 4 + 3]);
  }
  asm volatile("" ::: "memory");  // the chroma window's loads after the luma prediction
  const int CW = W / 2, CH = H / 2;
  const int cx0 = cx + (mvx >> 3), cy0 = cy + (mvy >> 3);
  const uint8_t *RUV = R + a.uv_off;
  uint32_t cwn[3][2];
  if (cx0 >= 0 && cx0 + 2 < CW && cy0 >= 0 && cy0 + 2 < CH) {
    const int o = 2 * cx0, sh = o & 3;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const uint32_t *q = reinterpret_cast<const uint32_t *>(RUV + static_cast<int64_t>(cy0 + r) * pitch + (o & ~3));
      const uint32_t d0 = q[0], d1 = q[1];
      cwn[r][0] = __builtin_amdgcn_alignbyte(d1, d0, sh);
      cwn[r][1] = d1 >> (8 * sh);
    }
  } else {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const uint8_t *row = RUV + static_cast<int64_t>(min(max(cy0 + r, 0), CH - 1)) * pitch;
      uint32_t v[2] = {0, 0};
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int xx = 2 * min(max(cx0 + c, 0), CW - 1);
        v[(2 * c) >> 2] |= static_cast<uint32_t>(row[xx]) << (((2 * c) & 3) * 8);
        v[(2 * c + 1) >> 2] |= static_cast<uint32_t>(row[xx + 1]) << (((2 * c + 1) & 3) * 8);
      }
      cwn[r][0] = v[0];
      cwn[r][1] = v[1];
    }
  }
  const int fx = mvx & 7, fy = mvy & 7;
  auto cpx = [&](int r, int i) { return static_cast<int>((cwn[r][i >> 2] >> ((i & 3) * 8)) & 255); };
#pragma unroll
  for (int pl = 0; pl < 2; ++pl) {
    int c4[4];
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const int A = cpx(y, 2 * x + pl), B = cpx(y, 2 * x + 2 + pl);
        const int C = cpx(y + 1, 2 * x + pl), D = cpx(y + 1, 2 * x + 2 + pl);
        c4[y * 2 + x] = ((8 - fx) * (8 - fy) * A + fx * (8 - fy) * B + (8 - fx) * fy * C + fx * fy * D + 32) >> 6;
      }
    cpp[pl] = pack4(c4[0], c4[1], c4[2], c4[3]);
  }
}
__device__ __forceinline__ int pk_at(const uint32_t *v, int i) { return static_cast<int>((v[i >> 2] >> ((i & 3) * 8)) & 255u); }

// ------------------------------------------------------- inter / I_PCM blocks
// lane = (macroblock, raster 4x4 block b)
__device__ __forceinline__ void inter_mb(const FullReconArgs &a, int slot, int mb, int b) {
  const int mbw = a.P.mb_width, mbh = a.P.mb_height, nmb = mbw * mbh;
  if (mb >= nmb) return;
  const MbRec *rec = a.recs + static_cast<int64_t>(slot) * nmb + mb;
  const MbHdr h = load_hdr(rec);
  if (h.epoch != a.epoch) {
    if (b == 0) atomicOr(a.err, static_cast<uint32_t>(DEC_E_MISSING_MB));
    return;
  }
  if (h.type == kMbI4x4 || h.type == kMbI16) return;  // h264_intra_full
  const int mx = mb % mbw, my = mb / mbw, bx = b & 3, by = b >> 2;
  uint8_t *Y = surf_at(a, slot);
  uint8_t *UV = Y + a.uv_off;
  const int x0 = mx * 16 + bx * 4, y0 = my * 16 + by * 4;
  const int cx = mx * 8 + bx * 2, cy = my * 8 + by * 2;
  const int pitch = a.pitch;
  if (h.type == kMbPcm) {
    const uint8_t *pcm = reinterpret_cast<const uint8_t *>(a.arena + 16 * static_cast<int64_t>(h.coef));
#pragma unroll
    for (int r = 0; r < 4; ++r)
      *reinterpret_cast<uint32_t *>(Y + static_cast<int64_t>(y0 + r) * pitch + x0) =
          *reinterpret_cast<const uint32_t *>(pcm + (by * 4 + r) * 16 + bx * 4);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int o = (by * 2 + r) * 8 + bx * 2;
      *reinterpret_cast<uint32_t *>(UV + static_cast<int64_t>(cy + r) * pitch + 2 * cx) =
          pack4(pcm[256 + o], pcm[320 + o], pcm[256 + o + 1], pcm[320 + o + 1]);
    }
    return;
  }
  const int p8 = (b >> 3) * 2 + ((b & 3) >> 1);
  const int rs0 = h.ref_slot[p8];
  const uint32_t mvw = reinterpret_cast<const uint32_t *>(rec)[16 + b];
  int rs1 = -1, r1 = -1;
  uint32_t mvw1 = 0;
  if (a.P.bframes) {
    const uint32_t *q = reinterpret_cast<const uint32_t *>(a.recs1 + static_cast<int64_t>(slot) * nmb + mb);
    const uint32_t w0 = q[0], wsl = q[1 + (p8 >> 1)];
    mvw1 = q[16 + b];
    r1 = static_cast<int8_t>((w0 >> (8 * p8)) & 255);
    rs1 = static_cast<int16_t>((wsl >> (16 * (p8 & 1))) & 0xffff);
    if (rs1 < 0) r1 = -1;
  }
  const int r0 = rs0 >= 0 ? static_cast<int8_t>((h.refs >> (8 * p8)) & 255) : -1;
  if (rs0 < 0 && rs1 < 0) {
    atomicOr(a.err, static_cast<uint32_t>(DEC_E_NO_REF));
    return;
  }
  const int W = mbw * 16, H = mbh * 16;
  uint32_t pvp[4], cpp[2];
  pred_ref(a, rs0 >= 0 ? rs0 : rs1, rs0 >= 0 ? mvw : mvw1, x0, y0, cx, cy, W, H, pvp, cpp);
  const int ext = a.P.has_ext ? a.slices[h.slice].ext : -1;
  if (rs1 >= 0 || ext >= 0) {  // bi-prediction / weighted prediction (8.4.2.3)
    const full::Wp Wt = full::wp_make(ext >= 0 ? a.exts + ext : nullptr, r0, r1);
    uint32_t pvp1[4] = {0, 0, 0, 0}, cpp1[2] = {0, 0};
    if (rs0 >= 0 && rs1 >= 0) pred_ref(a, rs1, mvw1, x0, y0, cx, cy, W, H, pvp1, cpp1);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      pvp[r] = pack4(full::wp_apply(Wt, 0, pk_at(pvp, r * 4), Wt.both ? pk_at(pvp1, r * 4) : 0),
                     full::wp_apply(Wt, 0, pk_at(pvp, r * 4 + 1), Wt.both ? pk_at(pvp1, r * 4 + 1) : 0),
                     full::wp_apply(Wt, 0, pk_at(pvp, r * 4 + 2), Wt.both ? pk_at(pvp1, r * 4 + 2) : 0),
                     full::wp_apply(Wt, 0, pk_at(pvp, r * 4 + 3), Wt.both ? pk_at(pvp1, r * 4 + 3) : 0));
#pragma unroll
    for (int pl = 0; pl < 2; ++pl) {
      const uint32_t c0 = cpp[pl], c1 = cpp1[pl];
      auto cb = [](uint32_t v, int i) { return static_cast<int>((v >> (8 * i)) & 255u); };
      cpp[pl] = pack4(full::wp_apply(Wt, 1 + pl, cb(c0, 0), Wt.both ? cb(c1, 0) : 0),
                      full::wp_apply(Wt, 1 + pl, cb(c0, 1), Wt.both ? cb(c1, 1) : 0),
                      full::wp_apply(Wt, 1 + pl, cb(c0, 2), Wt.both ? cb(c1, 2) : 0),
                      full::wp_apply(Wt, 1 + pl, cb(c0, 3), Wt.both ? cb(c1, 3) : 0));
    }
  }
  int pv[16], cpred[2][4];
#pragma unroll
  for (int i = 0; i < 16; ++i) pv[i] = pk_at(pvp, i);
#pragma unroll
  for (int pl = 0; pl < 2; ++pl)
#pragma unroll
    for (int i = 0; i < 4; ++i) cpred[pl][i] = static_cast<int>((cpp[pl] >> (8 * i)) & 255u);
  // luma residual
  int res[16];
  const bool t8 = (h.modes & kModeT8) != 0;
  const int64_t lb = stored(h.blocks, h.coef, t8 ? kBlkLuma0 + 4 * ((by >> 1) * 2 + (bx >> 1)) : kBlkLuma0 + blkidx(b));
  if (lb >= 0 && t8) {
    idct8_quarter(a.arena, lb, h.qp, bx & 1, by & 1, a.P.scaled ? a.sct->ls8[1][h.qp % 6] : nullptr, res);
  } else if (lb >= 0) {
    int cf[16];
    load_coefs(a.arena, lb, cf);
    full::scale_idct4(cf, h.qp, ls4_of(a, false, 0, h.qp), false, res);
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) res[i] = 0;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
    *reinterpret_cast<uint32_t *>(Y + static_cast<int64_t>(y0 + r) * pitch + x0) =
        pack4(c255(pv[r * 4] + res[r * 4]), c255(pv[r * 4 + 1] + res[r * 4 + 1]), c255(pv[r * 4 + 2] + res[r * 4 + 2]),
              c255(pv[r * 4 + 3] + res[r * 4 + 3]));
  // chroma residual
  if (h.cbp >> 4) {
    const int ck = ((by >> 1) << 1) | (bx >> 1), sx = (bx & 1) * 2, sy = (by & 1) * 2;
#pragma unroll
    for (int pl = 0; pl < 2; ++pl) {
      int r[16];
      const int qpc = full::qpc_of(h.qp, pl ? a.P.cqp_off2 : a.P.cqp_off);
      chroma_res(a.arena, h.blocks, h.coef, pl, ck, qpc, ls4_of(a, false, 1 + pl, qpc), r);
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int x = 0; x < 2; ++x) cpred[pl][y * 2 + x] = c255(cpred[pl][y * 2 + x] + r[(sy + y) * 4 + sx + x]);
    }
  }
#pragma unroll
  for (int y = 0; y < 2; ++y)
    *reinterpret_cast<uint32_t *>(UV + static_cast<int64_t>(cy + y) * pitch + 2 * cx) =
        pack4(cpred[0][y * 2], cpred[1][y * 2], cpred[0][y * 2 + 1], cpred[1][y * 2 + 1]);
}
// grid (ceil(nmb / 16), pictures of the level)
// occupancy 4: 128 VGPRs, two spilled (measured faster than 3 waves without
// spills: content / noise reconstruction -2 % / -5 %, profiles/r05af)
__global__ void __launch_bounds__(kInterThreads, 4) h264_inter_full(FullReconArgs a) {
  inter_mb(a, a.frames[blockIdx.y].x, blockIdx.x * 16 + (threadIdx.x >> 4), threadIdx.x & 15);
}

// ------------------------------------------------------------ intra blocks
struct alignas(16) IntraTile {  // dword / 16-byte members first, so every wide LDS access is aligned
  uint8_t cout[8][16]; // reconstructed chroma rows, interleaved
  // Intra_8x8: the filtered reference samples p' as E (E[0..7] = p'[-1,7..0],
  // E[8] = p'[-1,-1], E[9..24] = p'[0..15,-1]) at 1..25 (0 and 26 repeat the
  // ends), F(k) at 32 + k, A(k) at 64 + k (as pe below), DC at 88
  uint8_t p8[96];
  // Intra_4x4, per lane: the block's reference samples E (E[0..3] = p[-1,3..0],
  // E[4] = p[-1,-1], E[5..12] = p[0..7,-1]) at 1..13 (0 and 14 repeat the
  // ends), their 3-tap filter F(k) = (E[k-1] + 2E[k] + E[k+1] + 2) >> 2 at
  // 16 + k, 2-tap mean A(k) = (E[k] + E[k+1] + 1) >> 1 at 32 + k, DC at 47
  uint8_t pe[16][48];
  uint8_t y[17][28];   // luma rows -1..15 (index + 1) x cols -4..23 (index + 4)
  uint8_t ct[2][9];    // chroma row -1, cols -1..7 (index + 1), per plane
  uint8_t cl[2][8];    // chroma col -1, rows 0..7
};
// Every Intra_4x4 mode (8.3.1.2.1-9) reads each predicted sample as one entry
// of IntraTile::pe: its offset for (mode, x, y), built by the formulas below
// once per workgroup, so lanes whose blocks use different modes run one
// instruction stream (a per-lane switch ran the modes' bodies one after another)
__device__ __forceinline__ int intra4_off(int mode, int x, int y) {
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
// the same for Intra_8x8 (8.3.2.2.2-10) into IntraTile::p8
__device__ __forceinline__ int intra8_off(int mode, int x, int y) {
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

__device__ __forceinline__ void lane_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// one intra-predicted macroblock with 16 lanes (lane = raster 4x4 block b)
// (inlined at its one call site: a non-inlined call takes the kernel
// arguments' address, which copies them to scratch and turns every field read
// into a scratch load)
__device__ __forceinline__ void intra_mb(const FullReconArgs &a, int slot, int mb, int b, IntraTile &t,
                                         const uint8_t *s_off4, const uint8_t *s_off8) {
  const int mbw = a.P.mb_width, nmb = mbw * a.P.mb_height;
  const MbRec *frecs = a.recs + static_cast<int64_t>(slot) * nmb;
  const MbRec *rec = frecs + mb;
  const MbHdr h = load_hdr(rec);
  const int mx = mb % mbw, my = mb / mbw, bx = b & 3, by = b >> 2;
  const int pitch = a.pitch;
  uint8_t *Y = surf_at(a, slot);
  uint8_t *UV = Y + a.uv_off;
  // Every load of the neighbourhood is issued at once, unconditionally, from
  // clamped addresses (a neighbour's header, this lane's border samples), and
  // the availability decides afterwards which values count: conditional
  // loads each waited for the one before (header -> availability -> samples)
  const int nA = mx > 0 ? mb - 1 : mb, nB = my > 0 ? mb - mbw : mb;
  const int nC = my > 0 && mx < mbw - 1 ? mb - mbw + 1 : mb, nD = mx > 0 && my > 0 ? mb - mbw - 1 : mb;
  const uint2 hA = *reinterpret_cast<const uint2 *>(frecs + nA), hB = *reinterpret_cast<const uint2 *>(frecs + nB);
  const uint2 hC = *reinterpret_cast<const uint2 *>(frecs + nC), hD = *reinterpret_cast<const uint2 *>(frecs + nD);
  const uint32_t tA = reinterpret_cast<const uint32_t *>(frecs + nA)[4], tB = reinterpret_cast<const uint32_t *>(frecs + nB)[4];
  const uint32_t tC = reinterpret_cast<const uint32_t *>(frecs + nC)[4], tD = reinterpret_cast<const uint32_t *>(frecs + nD)[4];
  const int64_t yrow0 = static_cast<int64_t>(my * 16) * pitch + mx * 16;
  const int64_t crow0 = static_cast<int64_t>(my * 8) * pitch + mx * 16;
  // row -1 (b < 7: cols -4 + 4b), col -1 (row b), chroma col -1 (b < 8: row b), chroma row -1 (8 <= b < 13)
  const int64_t up = my > 0 ? yrow0 - pitch : yrow0;
  const uint32_t vTop = *reinterpret_cast<const uint32_t *>(Y + max(up - 4 + 4 * min(b, 6), static_cast<int64_t>(0)));
  const uint8_t vLeft = Y[max(yrow0 + static_cast<int64_t>(b) * pitch - 1, static_cast<int64_t>(0))];
  const uint32_t vCl = *reinterpret_cast<const uint32_t *>(UV + crow0 + static_cast<int64_t>(min(b, 7)) * pitch - 4);
  const uint32_t vCt = *reinterpret_cast<const uint32_t *>(UV + crow0 - pitch - 4 + 4 * min(max(b - 8, 0), 4));
  auto nb_ok = [&](bool exists, uint2 u, uint32_t ty) -> bool {
    if (!exists || u.x != a.epoch || u.y != h.slice) return false;
    if (a.P.cip && ((ty & 255) == kMbInter || (ty & 255) == kMbSkip)) return false;
    return true;
  };
  const bool A = nb_ok(mx > 0, hA, tA);
  const bool B = nb_ok(my > 0, hB, tB);
  const bool C = nb_ok(my > 0 && mx < mbw - 1, hC, tC);
  const bool D = nb_ok(mx > 0 && my > 0, hD, tD);
  // borders into the tile; unavailable neighbours read as 0 (as the oracle;
  // conforming streams never use them)
  if (b < 7) {
    const bool need = b == 0 ? D : (b < 5 ? B : C);
    *reinterpret_cast<uint32_t *>(&t.y[0][4 * b]) = need ? vTop : 0u;
  }
  t.y[1 + b][3] = A ? vLeft : 0;
  if (b < 8) {
    const uint32_t v = A ? vCl : 0u;
    t.cl[0][b] = (v >> 16) & 255;
    t.cl[1][b] = v >> 24;
  }
  if (b >= 8 && b < 13) {
    const int i = b - 8;  // dword i of chroma row -1, interleaved bytes -4 + 4i
    {
      const uint32_t v = (i == 0 ? D : B) ? vCt : 0u;
      if (i == 0) {
        t.ct[0][0] = (v >> 16) & 255;
        t.ct[1][0] = v >> 24;
      } else {
        const int c0 = 2 * (i - 1);
        t.ct[0][1 + c0] = v & 255;
        t.ct[1][1 + c0] = (v >> 8) & 255;
        t.ct[0][2 + c0] = (v >> 16) & 255;
        t.ct[1][2 + c0] = v >> 24;
      }
    }
  }
  lane_sync();
  const int qp = h.qp;
  if (h.type == kMbI16) {
    const int mode = h.modes & 3;
    int v[16];
    if (mode == 0) {
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int x = 0; x < 4; ++x) v[y * 4 + x] = t.y[0][4 + bx * 4 + x];
    } else if (mode == 1) {
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int x = 0; x < 4; ++x) v[y * 4 + x] = t.y[1 + by * 4 + y][3];
    } else if (mode == 2) {
      int st = 0, sl = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        st += t.y[0][4 + i];
        sl += t.y[1 + i][3];
      }
      const int dc = (A && B) ? (st + sl + 16) >> 5 : (A ? (sl + 8) >> 4 : (B ? (st + 8) >> 4 : 128));
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = dc;
    } else {
      int Hh = 0, Vv = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        Hh += (i + 1) * (t.y[0][4 + 8 + i] - t.y[0][4 + 6 - i]);
        Vv += (i + 1) * (t.y[1 + 8 + i][3] - t.y[1 + 6 - i][3]);  // row -1 is t.y[0][3]
      }
      const int aa = 16 * (t.y[16][3] + t.y[0][19]);
      const int bb = (5 * Hh + 32) >> 6, cc = (5 * Vv + 32) >> 6;
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int x = 0; x < 4; ++x) v[y * 4 + x] = c255((aa + bb * (bx * 4 + x - 7) + cc * (by * 4 + y - 7) + 16) >> 5);
    }
    // 8.5.10 DC: Hadamard of the 16 DC levels (raster), scaled; this block's entry
    int dcl[16];
    load_coefs(a.arena, stored(h.blocks, h.coef, kBlkI16Dc), dcl);
    int tr[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int a0 = dcl[i * 4], a1 = dcl[i * 4 + 1], a2 = dcl[i * 4 + 2], a3 = dcl[i * 4 + 3];
      tr[i * 4] = a0 + a1 + a2 + a3;
      tr[i * 4 + 1] = a0 + a1 - a2 - a3;
      tr[i * 4 + 2] = a0 - a1 - a2 + a3;
      tr[i * 4 + 3] = a0 - a1 + a2 - a3;
    }
    const int a0 = tr[bx], a1 = tr[4 + bx], a2 = tr[8 + bx], a3 = tr[12 + bx];
    const int f = by == 0 ? a0 + a1 + a2 + a3 : by == 1 ? a0 + a1 - a2 - a3 : by == 2 ? a0 - a1 - a2 + a3 : a0 - a1 + a2 - a3;
    const int32_t *ls4 = ls4_of(a, true, 0, qp);
    const int ls = ls4[0];  // 8.5.10: LevelScale4x4(qP % 6, 0, 0) of Intra Y
    int cf[16], res[16];
    load_coefs(a.arena, stored(h.blocks, h.coef, kBlkLuma0 + blkidx(b)), cf);
    cf[0] = qp >= 36 ? (f * ls) << (qp / 6 - 6) : (f * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
    full::scale_idct4(cf, qp, ls4, true, res);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      *reinterpret_cast<uint32_t *>(Y + yrow0 + static_cast<int64_t>(by * 4 + r) * pitch + bx * 4) =
          pack4(c255(v[r * 4] + res[r * 4]), c255(v[r * 4 + 1] + res[r * 4 + 1]), c255(v[r * 4 + 2] + res[r * 4 + 2]),
                c255(v[r * 4 + 3] + res[r * 4 + 3]));
  } else if (h.modes & kModeT8) {
    // Intra_8x8 (8.3.2): the 8x8 blocks in order, one step each; the 4 lanes
    // of a block each predict and reconstruct one 4x4 quarter from the
    // filtered reference samples (every lane filters them itself)
    const int b8 = (by >> 1) * 2 + (bx >> 1), qx = bx & 1, qy = by & 1;
    const int xo = (b8 & 1) * 8, yo = (b8 >> 1) * 8;
    const int r8 = (b8 >> 1) * 8 + (b8 & 1) * 2;
    const uint32_t i4w = reinterpret_cast<const uint32_t *>(rec)[8 + (r8 >> 3)];
    const int m8 = (i4w >> (((r8 >> 1) & 3) * 8 + (r8 & 1) * 4)) & 15;
    const bool top = yo > 0 || B, left = xo > 0 || A;
    const bool tl = (xo > 0 && yo > 0) || (yo == 0 && xo > 0 ? B : (xo == 0 && yo > 0 ? A : D));
    const bool tr = b8 == 0 ? B : (b8 == 1 ? C : b8 == 2);
    const int64_t lb = stored(h.blocks, h.coef, kBlkLuma0 + 4 * b8);
    for (int s = 0; s < 4; ++s) {
      if (s == b8 && qx == 0 && qy == 0) {  // the block's first lane filters the reference samples
        const int ty = yo, tx = 4 + xo;  // tile row of p[., -1], col of p[0, .]
        int P_[25];  // 0 = p[-1,-1], 1 + x = p[x,-1], 17 + y = p[-1,y]
        P_[0] = tl ? t.y[ty][tx - 1] : 0;
#pragma unroll
        for (int x = 0; x < 8; ++x) P_[1 + x] = top ? t.y[ty][tx + x] : 0;
#pragma unroll
        for (int x = 8; x < 16; ++x) P_[1 + x] = tr ? t.y[ty][tx + x] : P_[8];
#pragma unroll
        for (int y = 0; y < 8; ++y) P_[17 + y] = left ? t.y[ty + 1 + y][tx - 1] : 0;
        int T[17], L[8];
#pragma unroll
        for (int i = 0; i < 17; ++i) T[i] = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) L[i] = 0;
        if (top) {
          T[1] = tl ? (P_[0] + 2 * P_[1] + P_[2] + 2) >> 2 : (3 * P_[1] + P_[2] + 2) >> 2;
#pragma unroll
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
#pragma unroll
          for (int y = 1; y < 7; ++y) L[y] = (P_[16 + y] + 2 * P_[17 + y] + P_[18 + y] + 2) >> 2;
          L[7] = (P_[23] + 3 * P_[24] + 2) >> 2;
        }
        int e[27];
#pragma unroll
        for (int k = 0; k < 8; ++k) e[1 + k] = L[7 - k];
        e[0] = e[1];
        e[9] = T[0];
#pragma unroll
        for (int i = 0; i < 16; ++i) e[10 + i] = T[1 + i];
        e[26] = e[25];
        int st = 0, sl = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          st += T[1 + i];
          sl += L[i];
        }
        int pv[96];
#pragma unroll
        for (int i = 0; i < 96; ++i) pv[i] = 0;
#pragma unroll
        for (int i = 0; i < 27; ++i) pv[i] = e[i];
#pragma unroll
        for (int k = 0; k < 25; ++k) pv[32 + k] = (e[k] + 2 * e[k + 1] + e[k + 2] + 2) >> 2;
#pragma unroll
        for (int k = 0; k < 24; ++k) pv[64 + k] = (e[1 + k] + e[2 + k] + 1) >> 1;
        pv[88] = (top && left) ? (st + sl + 8) >> 4 : (left ? (sl + 4) >> 3 : (top ? (st + 4) >> 3 : 128));
#pragma unroll
        for (int i = 0; i < 24; ++i)
          *reinterpret_cast<uint32_t *>(t.p8 + 4 * i) = pack4(pv[4 * i], pv[4 * i + 1], pv[4 * i + 2], pv[4 * i + 3]);
      }
      lane_sync();
      if (s == b8) {
        int res[16];
        if (lb >= 0) idct8_quarter(a.arena, lb, qp, qx, qy, a.P.scaled ? a.sct->ls8[0][qp % 6] : nullptr, res);
        else
#pragma unroll
          for (int i = 0; i < 16; ++i) res[i] = 0;
        const uint8_t *offs = s_off8 + 64 * min(m8, 8);  // > 8: not a mode (as mode 8)
#pragma unroll
        for (int yy = 0; yy < 4; ++yy) {
          const uint32_t ow = *reinterpret_cast<const uint32_t *>(offs + (qy * 4 + yy) * 8 + qx * 4);
          int o[4];
#pragma unroll
          for (int xx = 0; xx < 4; ++xx) o[xx] = c255(t.p8[(ow >> (8 * xx)) & 255] + res[yy * 4 + xx]);
          const uint32_t w4 = pack4(o[0], o[1], o[2], o[3]);
          *reinterpret_cast<uint32_t *>(&t.y[1 + by * 4 + yy][4 + bx * 4]) = w4;
          *reinterpret_cast<uint32_t *>(Y + yrow0 + static_cast<int64_t>(by * 4 + yy) * pitch + bx * 4) = w4;
        }
      }
      lane_sync();
    }
  } else {
    // Intra_4x4: block (bx, by) at step bx + 2 by; its left / top / top-left /
    // top-right blocks (earlier in luma4x4BlkIdx order) are done one or more steps before
    const int k = blkidx(b);
    const uint32_t i4w = reinterpret_cast<const uint32_t *>(rec)[8 + (b >> 3)];
    const int m4 = (i4w >> (((b >> 1) & 3) * 8 + (b & 1) * 4)) & 15;
    const bool top = by > 0 || B;
    const bool left = bx > 0 || A;
    const bool tl = (bx > 0 && by > 0) || (by == 0 && bx > 0 ? B : (bx == 0 && by > 0 ? A : D));
    bool tr;
    if (by == 0) tr = bx < 3 ? B : C;
    else tr = bx < 3 && blkidx((by - 1) * 4 + bx + 1) < k;
    int cf[16], res[16];
    load_coefs(a.arena, stored(h.blocks, h.coef, kBlkLuma0 + k), cf);
    full::scale_idct4(cf, qp, ls4_of(a, true, 0, qp), false, res);
    const int step = bx + 2 * by;
    for (int s = 0; s <= 9; ++s) {
      if (s == step) {
        const int ty = by * 4, tx = 4 + bx * 4;  // tile row of p[., -1] and col of p[0, .]
        int T[9], L[5];
        T[0] = L[0] = tl ? t.y[ty][tx - 1] : 0;
#pragma unroll
        for (int x = 0; x < 4; ++x) T[1 + x] = top ? t.y[ty][tx + x] : 0;
#pragma unroll
        for (int x = 4; x < 8; ++x) T[1 + x] = tr ? t.y[ty][tx + x] : T[4];
#pragma unroll
        for (int y = 0; y < 4; ++y) L[1 + y] = left ? t.y[ty + 1 + y][tx - 1] : 0;
        int e[15];  // pe[0..14]
        e[0] = e[1] = L[4];
        e[2] = L[3];
        e[3] = L[2];
        e[4] = L[1];
        e[5] = T[0];
#pragma unroll
        for (int x = 0; x < 8; ++x) e[6 + x] = T[1 + x];
        e[14] = e[13];
        int dc;
        if (top && left) dc = (T[1] + T[2] + T[3] + T[4] + L[1] + L[2] + L[3] + L[4] + 4) >> 3;
        else if (left) dc = (L[1] + L[2] + L[3] + L[4] + 2) >> 2;
        else if (top) dc = (T[1] + T[2] + T[3] + T[4] + 2) >> 2;
        else dc = 128;
        int pv[48];
#pragma unroll
        for (int i = 0; i < 48; ++i) pv[i] = 0;
#pragma unroll
        for (int i = 0; i < 15; ++i) pv[i] = e[i];
#pragma unroll
        for (int k = 0; k < 13; ++k) pv[16 + k] = (e[k] + 2 * e[k + 1] + e[k + 2] + 2) >> 2;
#pragma unroll
        for (int k = 0; k < 12; ++k) pv[32 + k] = (e[1 + k] + e[2 + k] + 1) >> 1;
        pv[47] = dc;
        uint8_t *pe = t.pe[b];
#pragma unroll
        for (int i = 0; i < 12; ++i)
          *reinterpret_cast<uint32_t *>(pe + 4 * i) = pack4(pv[4 * i], pv[4 * i + 1], pv[4 * i + 2], pv[4 * i + 3]);
        const uint32_t *offw = reinterpret_cast<const uint32_t *>(s_off4 + 16 * min(m4, 8));  // > 8: not a mode (as mode 8)
        int o[16];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t ow = offw[r];
#pragma unroll
          for (int x = 0; x < 4; ++x) o[r * 4 + x] = c255(pe[(ow >> (8 * x)) & 255] + res[r * 4 + x]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t w4 = pack4(o[r * 4], o[r * 4 + 1], o[r * 4 + 2], o[r * 4 + 3]);
          *reinterpret_cast<uint32_t *>(&t.y[ty + 1 + r][tx]) = w4;
          *reinterpret_cast<uint32_t *>(Y + yrow0 + static_cast<int64_t>(by * 4 + r) * pitch + bx * 4) = w4;
        }
      }
      lane_sync();
    }
  }
  // chroma (8.3.4): lanes 0..7 = (plane, 4x4 block)
  if (b < 8) {
    const int pl = b >> 2, ck = b & 3, ox = (ck & 1) * 4, oy = (ck >> 1) * 4;
    const int cm = (h.modes >> 2) & 3;
    const uint8_t *T = t.ct[pl];  // T[0] = p[-1,-1], T[1 + x]
    const uint8_t *L = t.cl[pl];  // L[y]
    int v[16];
    if (cm == 0) {
      int st = 0, sl = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        st += T[1 + ox + i];
        sl += L[oy + i];
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
      for (int i = 0; i < 16; ++i) v[i] = dc;
    } else if (cm == 1) {
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int x = 0; x < 4; ++x) v[y * 4 + x] = L[oy + y];
    } else if (cm == 2) {
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int x = 0; x < 4; ++x) v[y * 4 + x] = T[1 + ox + x];
    } else {
      int Hh = 0, Vv = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        Hh += (i + 1) * (T[1 + 4 + i] - T[1 + 2 - i]);
        Vv += (i + 1) * ((4 + i < 8 ? L[4 + i] : 0) - (2 - i >= 0 ? L[2 - i] : T[0]));
      }
      const int aa = 16 * (L[7] + T[8]);
      const int bb = (34 * Hh + 32) >> 6, cc = (34 * Vv + 32) >> 6;
#pragma unroll
      for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int x = 0; x < 4; ++x) v[y * 4 + x] = c255((aa + bb * (ox + x - 3) + cc * (oy + y - 3) + 16) >> 5);
    }
    int r[16];
    const int qpc = full::qpc_of(qp, pl ? a.P.cqp_off2 : a.P.cqp_off);
    chroma_res(a.arena, h.blocks, h.coef, pl, ck, qpc, ls4_of(a, true, 1 + pl, qpc), r);
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
      for (int x = 0; x < 4; ++x) t.cout[oy + y][2 * (ox + x) + pl] = static_cast<uint8_t>(c255(v[y * 4 + x] + r[y * 4 + x]));
  }
  lane_sync();
  if (b < 8) {
    const uint4 row = *reinterpret_cast<const uint4 *>(&t.cout[b][0]);
    *reinterpret_cast<uint4 *>(UV + crow0 + static_cast<int64_t>(b) * pitch) = row;
  }
  lane_sync();
}

// grid: pictures of the level; the intra-predicted macroblocks by dependency level
__global__ void __launch_bounds__(kIntraThreads) h264_intra_full(FullReconArgs a) {
  extern __shared__ uint16_t s_list[];  // nmb entries
  __shared__ IntraTile tiles[kIntraSlots];
  __shared__ int s_max, s_cnt;
  __shared__ int s_lvl[kIntraLevels + 1], s_fill[kIntraLevels];
  __shared__ __attribute__((aligned(4))) uint8_t s_off4[9 * 16];
  __shared__ __attribute__((aligned(4))) uint8_t s_off8[9 * 64];
  const int nmb = a.P.mb_width * a.P.mb_height;
  const int slot = a.frames[blockIdx.x].x;
  const uint16_t *lv = a.ilvl + static_cast<int64_t>(slot) * nmb;
  const int tid = threadIdx.x;
  if (tid == 0) s_max = -1;
  if (tid < 9 * 16) s_off4[tid] = static_cast<uint8_t>(intra4_off(tid >> 4, tid & 3, (tid >> 2) & 3));
  for (int i = tid; i < 9 * 64; i += kIntraThreads) s_off8[i] = static_cast<uint8_t>(intra8_off(i >> 6, i & 7, (i >> 3) & 7));
  __syncthreads();
  int m = -1;
  for (int i = tid; i < nmb; i += kIntraThreads) {
    const int v = lv[i];
    if (v != kNoLevel) m = max(m, v);
  }
  if (m >= 0) atomicMax(&s_max, m);
  __syncthreads();
  const int maxl = __builtin_amdgcn_readfirstlane(s_max);  // uniform: the loops below hold barriers
  const int ms = tid >> 4, b = tid & 15;
  const bool bucketed = maxl < kIntraLevels;
  if (bucketed) {
    // the picture's intra macroblocks bucketed by level once (a counting
    // sort in LDS), then the levels in order: an all-intra picture has
    // ~mbw + 2 mbh levels, and a scan of every level per level cost more
    // than its reconstruction
    for (int i = tid; i <= maxl + 1; i += kIntraThreads) s_lvl[i] = 0;
    __syncthreads();
    for (int i = tid; i < nmb; i += kIntraThreads) {
      const int v = lv[i];
      if (v != kNoLevel) atomicAdd(&s_lvl[v + 1], 1);
    }
    __syncthreads();
    if (tid == 0)  // s_lvl[l] = first list entry of level l (exclusive scan)
      for (int l = 1; l <= maxl + 1; ++l) s_lvl[l] += s_lvl[l - 1];
    __syncthreads();
    for (int i = tid; i <= maxl; i += kIntraThreads) s_fill[i] = s_lvl[i];
    __syncthreads();
    for (int i = tid; i < nmb; i += kIntraThreads) {
      const int v = lv[i];
      if (v != kNoLevel) s_list[atomicAdd(&s_fill[v], 1)] = static_cast<uint16_t>(i);
    }
    __syncthreads();
  }
  for (int l = 0; l <= maxl; ++l) {
    int j0, j1;
    if (bucketed) {
      j0 = __builtin_amdgcn_readfirstlane(s_lvl[l]);
      j1 = __builtin_amdgcn_readfirstlane(s_lvl[l + 1]);
    } else {  // more levels than buckets: this level's macroblocks by a scan
      if (tid == 0) s_cnt = 0;
      __syncthreads();
      for (int i = tid; i < nmb; i += kIntraThreads)
        if (lv[i] == l) s_list[atomicAdd(&s_cnt, 1)] = static_cast<uint16_t>(i);
      __syncthreads();
      j0 = 0;
      j1 = __builtin_amdgcn_readfirstlane(s_cnt);
    }
    for (int j = j0 + ms; j < j1; j += kIntraSlots) {
      intra_mb(a, slot, s_list[j], b, tiles[ms], s_off4, s_off8);
    }
    __syncthreads();
  }
}

// ---- intra, lane-parallel (default; VTS_INTRA=1 runs h264_intra_full)
// The same dependency levels as h264_intra_full (the x + 2y wavefront of an
// all-intra picture), with the work inside a macroblock spread over 32 lanes
// by sample instead of by 4x4 block, and the neighbourhood kept in LDS:
//  * 32 lanes (half a wave) per macroblock, 32 macroblocks in flight;
//  * the residual of every block is computed first, lane per block, into the
//    macroblock's tile (it needs no neighbour);
//  * prediction by sample: Intra_4x4 runs its 10 block steps (bx + 2 by) with
//    the step's one or two blocks as 16 lanes each (the lanes build the
//    block's reference-sample array E, then each predicts its sample from E
//    by the (mode, x, y) offset table); Intra_8x8 its 4 blocks with the
//    filtered reference samples and their derived arrays built by lanes in
//    parallel; Intra_16x16 and chroma 8 / 4 samples per lane, sums by
//    cross-lane reduction;
//  * the samples a later level reads (each macroblock's bottom row and right
//    column, luma and chroma) go to LDS line buffers (bottom rows by macroblock
//    row parity, right columns per row), so a macroblock reads intra
//    neighbours from LDS after the level barrier and only inter / I_PCM
//    neighbours (final before this launch) from HBM, from loads issued with
//    its record loads;
//  * the macroblock leaves as whole rows at the end (dword stores).
// h264_intra_full spent ~62 k cycles per macroblock step per wave and ~41 k
// per wave at the level barrier (profiles/r04c_recon_sections_dbk2.json).
constexpr int kI2Threads = 1024;
constexpr int kI2Groups = kI2Threads / 32;
using i2::I2Tile;
// the macroblock's 32 lanes are half a wave
struct DevLanes {
  int t;
  __device__ __forceinline__ void sync() const { lane_sync(); }
  __device__ __forceinline__ int red16(int v) const {
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) v += __shfl_xor(v, m, 16);
    return v;
  }
  __device__ __forceinline__ int bcast(int v, int l) const { return __shfl(v, static_cast<int>(threadIdx.x & 32) + l); }
  __device__ __forceinline__ void amax(int *p, int v) const { atomicMax(p, v); }
};

// The intra phase's LDS: the groups' tiles, the level buckets and offset
// tables, then (dynamic) the tagged line entries (one per macroblock column
// and row, i2::I2Line), the level lists and the round table (2 B per
// macroblock each)
struct I2Lds {
  I2Tile tiles[kI2Groups];
  int s_max, s_cnt;
  int s_lvl[kIntraLevels + 1], s_fill[kIntraLevels];
  uint8_t s_off4[9 * 16];
  uint8_t s_off8[9 * 64];
};
__host__ __device__ constexpr size_t i2_lds_bytes(int mbw, int mbh) {
  return (sizeof(I2Lds) + 15) / 16 * 16 + sizeof(i2::I2Line) * static_cast<size_t>(mbw + mbh) +
         4 * static_cast<size_t>(mbw) * static_cast<size_t>(mbh);
}
__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = min(v, __shfl_xor(v, off, 64));
  return v;
}
// one picture's intra macroblocks by dependency level (1024 threads)
__device__ __forceinline__ void intra_v2_picture(const FullReconArgs &a, int slot, uint8_t *lds) {
  I2Lds &L0 = *reinterpret_cast<I2Lds *>(lds);
  I2Tile *tiles = L0.tiles;
  int &s_max = L0.s_max, &s_cnt = L0.s_cnt;
  int *s_lvl = L0.s_lvl, *s_fill = L0.s_fill;
  uint8_t *s_off4 = L0.s_off4, *s_off8 = L0.s_off8;
  uint8_t *s_dyn = lds + (sizeof(I2Lds) + 15) / 16 * 16;
  const int mbw = a.P.mb_width, mbh = a.P.mb_height, nmb = mbw * mbh;
  const int pitch = a.pitch;
  i2::I2Line *lcol = reinterpret_cast<i2::I2Line *>(s_dyn), *lrow = lcol + mbw;
  uint16_t *s_list = reinterpret_cast<uint16_t *>(lrow + mbh);
  uint16_t *s_rnd = s_list + nmb;  // per macroblock: its level, then 0x8000 | its round
  for (int i = threadIdx.x; i < mbw + mbh; i += kI2Threads) {
    lcol[i].tag = -2;
    lcol[i].claim = -2;
  }
  const uint16_t *lv = a.ilvl + static_cast<int64_t>(slot) * nmb;
  const int tid = threadIdx.x;
  if (tid == 0) s_max = -1;
  if (tid < 9 * 16) s_off4[tid] = static_cast<uint8_t>(intra4_off(tid >> 4, tid & 3, (tid >> 2) & 3));
  for (int i = tid; i < 9 * 64; i += kI2Threads) s_off8[i] = static_cast<uint8_t>(intra8_off(i >> 6, i & 7, (i >> 3) & 7));
  __syncthreads();
  int m = -1;
  for (int i = tid; i < nmb; i += kI2Threads) {
    const int v = lv[i];
    if (v != kNoLevel) m = max(m, v);
  }
  if (m >= 0) atomicMax(&s_max, m);
  __syncthreads();
  int maxl = __builtin_amdgcn_readfirstlane(s_max);  // uniform: the loops below hold barriers
  const int g = tid >> 5;
  const DevLanes lanes0{tid & 31};
  i2::I2NoProf rp_;
  i2::I2Ctx ctx;
  ctx.recs = a.recs + static_cast<int64_t>(slot) * nmb;
  ctx.arena = a.arena;
  ctx.Y = surf_at(a, slot);
  ctx.uv_off = a.uv_off;
  ctx.pitch = pitch;
  ctx.mbw = a.P.mb_width;
  ctx.mbh = mbh;
  ctx.epoch = a.epoch;
  ctx.cip = a.P.cip;
  ctx.cqp_off = a.P.cqp_off;
  ctx.cqp_off2 = a.P.cqp_off2;
  ctx.scaled = a.P.scaled;
  ctx.sct = a.sct;
  const bool bucketed = maxl < kIntraLevels;
  if (bucketed) {  // the intra macroblocks bucketed by level (counting sort), as h264_intra_full
    for (int i = tid; i <= maxl + 1; i += kI2Threads) s_lvl[i] = 0;
    __syncthreads();
    for (int i = tid; i < nmb; i += kI2Threads) {
      const int v = lv[i];
      if (v != kNoLevel) atomicAdd(&s_lvl[v + 1], 1);
    }
    __syncthreads();
    if (tid == 0)
      for (int l = 1; l <= maxl + 1; ++l) s_lvl[l] += s_lvl[l - 1];
    __syncthreads();
    for (int i = tid; i <= maxl; i += kI2Threads) s_fill[i] = s_lvl[i];
    __syncthreads();
    for (int i = tid; i < nmb; i += kI2Threads) {
      const int v = lv[i];
      if (v != kNoLevel) s_list[atomicAdd(&s_fill[v], 1)] = static_cast<uint16_t>(i);
      s_rnd[i] = static_cast<uint16_t>(v == kNoLevel ? 0x7fff : v);
    }
    if (tid == 0) {
      int widest = 0;
      for (int l = 0; l <= maxl; ++l) widest = max(widest, s_lvl[l + 1] - s_lvl[l]);
      s_cnt = widest;
    }
    __syncthreads();
    // Rounds instead of levels where a level holds more macroblocks than a
    // round (an x + 2y diagonal of 33..40 at 720p took two rounds): each
    // macroblock in the earliest round after its intra neighbours' (A, B, C,
    // D at lower levels: a superset of what it predicts from) with room.  An
    // all-intra 720p picture: 208 -> 175 rounds (1080p 380 -> 317).  The
    // line entries' tags make any such order safe (a neighbour whose entry
    // was taken over is read from HBM).  Wave 0 assigns, level by level.
    if (__builtin_amdgcn_readfirstlane(s_cnt) > kI2Groups) {
      for (int i = tid; i < kIntraLevels; i += kI2Threads) s_fill[i] = 0;  // per round: macroblocks
      __syncthreads();
      if (tid < 64) {
        int rmax = -1;
        bool over = false;
        for (int l = 0; l <= maxl && !over; ++l) {
          const int j0 = __builtin_amdgcn_readfirstlane(s_lvl[l]), j1 = __builtin_amdgcn_readfirstlane(s_lvl[l + 1]);
          for (int c0 = j0; c0 < j1 && !over; c0 += 64) {
            const int i = c0 + tid;
            const bool valid = i < j1;
            int r0 = 0, mb = 0;
            if (valid) {
              mb = s_list[i];
              const int mx = mb % mbw, my = mb / mbw;
              auto dep = [&](bool ok, int n) {
                if (ok) {
                  const int e = s_rnd[n];
                  if (e & 0x8000) r0 = max(r0, (e & 0x7fff) + 1);  // assigned: a lower level
                }
              };
              dep(mx > 0, mb - 1);
              dep(my > 0, mb - mbw);
              dep(my > 0 && mx + 1 < mbw, mb - mbw + 1);
              dep(my > 0 && mx > 0, mb - mbw - 1);
            }
            bool un = valid;
            int r = wave_min(un ? r0 : 0x7fffffff);
            while (__ballot(un) != 0) {
              if (r >= kIntraLevels) {
                over = true;
                break;
              }
              const uint64_t el = __ballot(un && r0 <= r);
              if (el == 0) {
                r = wave_min(un ? r0 : 0x7fffffff);
                continue;
              }
              const int fill = s_fill[r];
              const int room = kI2Groups - fill;
              const int before = __popcll(el & ((1ull << tid) - 1ull));
              if (un && r0 <= r && before < room) {
                s_rnd[mb] = static_cast<uint16_t>(0x8000 | r);
                un = false;
              }
              const int taken = min(room, __popcll(el));
              s_fill[r] = fill + taken;  // every lane the same value
              if (taken > 0) rmax = max(rmax, r);
              ++r;
            }
          }
        }
        if (tid == 0) s_cnt = over ? -1 : rmax;
      }
      __syncthreads();
      const int nr = __builtin_amdgcn_readfirstlane(s_cnt) + 1;
      if (nr > 0) {  // the lists by round (else they stay by level)
        if (tid == 0) {
          s_lvl[0] = 0;
          for (int r = 0; r < nr; ++r) s_lvl[r + 1] = s_lvl[r] + s_fill[r];
        }
        __syncthreads();
        for (int i = tid; i < nr; i += kI2Threads) s_fill[i] = s_lvl[i];
        __syncthreads();
        for (int i = tid; i < nmb; i += kI2Threads) {
          const int e = s_rnd[i];
          if (e & 0x8000) s_list[atomicAdd(&s_fill[e & 0x7fff], 1)] = static_cast<uint16_t>(i);
        }
        maxl = nr - 1;
        __syncthreads();
      }
    }
  }
  // the group processes s_lvl[l] + g + 32 k of every level l, in order: its
  // first macroblock at level l0 or later (-1: none)
  auto first_at = [&](int l0) -> int {
    for (int l = l0; l <= maxl; ++l)
      if (s_lvl[l] + g < s_lvl[l + 1]) return s_lvl[l] + g;
    return -1;
  };
  i2::I2Pre pre{};
  bool pv = false;  // pre holds the group's next macroblock
  if (bucketed) {
    const int jf = first_at(0);
    pv = jf >= 0;
    if (pv) pre = i2::i2_prefetch(ctx, s_list[jf], lanes0.t);
  }
  for (int l = 0; l <= maxl; ++l) {
    int j0, j1;
    if (bucketed) {
      j0 = __builtin_amdgcn_readfirstlane(s_lvl[l]);
      j1 = __builtin_amdgcn_readfirstlane(s_lvl[l + 1]);
    } else {
      if (tid == 0) s_cnt = 0;
      __syncthreads();
      for (int i = tid; i < nmb; i += kI2Threads)
        if (lv[i] == l) s_list[atomicAdd(&s_cnt, 1)] = static_cast<uint16_t>(i);
      __syncthreads();
      j0 = 0;
      j1 = __builtin_amdgcn_readfirstlane(s_cnt);
    }
    // rounds of 32 macroblocks: every group's reads (part 1), barrier, every
    // group's reconstruction and writes (part 2), the group's next
    // macroblock's records and border loads issued (in flight across the
    // barrier), barrier
    for (int base = j0; base < j1; base += kI2Groups) {
      const int j = base + g;
      // the lane index made opaque each round: what derives from it (lane
      // masks and addresses) is recomputed per round instead of hoisted out
      // of the loop and spilled, whose reloads waited for every load in flight
      DevLanes lanes = lanes0;
      asm volatile("" : "+v"(lanes.t));
      if (j < j1) {
        if (!pv) pre = i2::i2_prefetch(ctx, s_list[j], lanes.t);
        i2::intra2_prepare(ctx, s_list[j], pre, lanes, tiles[g], lcol, lrow, rp_);
      } else {
        // no macroblock this round: drop the prefetch (re-issued when the
        // group has work again) rather than keep its registers across part 2
        pre = i2::I2Pre{};
        pv = false;
      }
      __syncthreads();
      if (j < j1) {
        i2::intra2_finish(ctx, lanes, tiles[g], lcol, lrow, s_off4, s_off8, rp_);
        const int jn = !bucketed ? -1 : (j + kI2Groups < j1 ? j + kI2Groups : first_at(l + 1));
        pv = jn >= 0;
        if (pv) pre = i2::i2_prefetch(ctx, s_list[jn], lanes.t);
      }
      __syncthreads();
    }
  }
}
// grid: pictures of the level; dynamic LDS: i2_lds_bytes
__global__ void __launch_bounds__(kI2Threads) h264_intra_v2(FullReconArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t s_i2[];
  VTS_WG_TRACE(1, 0, a.frames);
  intra_v2_picture(a, a.frames[blockIdx.x].x, s_i2);
  VTS_WG_TRACE(1, 1, a.frames);
}

// --------------------------------------------------------------- deblocking
__device__ __forceinline__ bool is_intra_t(int ty) { return ty == kMbI4x4 || ty == kMbI16 || ty == kMbPcm; }

// bS between 4x4 blocks bp of P and bq of Q (8.7.2.1, frames); P1 / Q1: their
// list-1 halves in streams with B slices, else null
__device__ __forceinline__ int bs_dev(const MbRec *P, const MbRecB *P1, int bp, const MbRec *Q, const MbRecB *Q1, int bq,
                                      int tp, int tq, bool mbe) {
  if (is_intra_t(tp) || is_intra_t(tq)) return mbe ? 4 : 3;
  if (P->nz[bp] || Q->nz[bq]) return 2;
  const int p8 = (bp >> 3) * 2 + ((bp & 3) >> 1), q8 = (bq >> 3) * 2 + ((bq & 3) >> 1);
  const uint32_t mp = reinterpret_cast<const uint32_t *>(P)[16 + bp], mq = reinterpret_cast<const uint32_t *>(Q)[16 + bq];
  if (P1) {
    const uint32_t mp1 = reinterpret_cast<const uint32_t *>(P1)[16 + bp], mq1 = reinterpret_cast<const uint32_t *>(Q1)[16 + bq];
    return full::bs_motion(P->ref_slot[p8], P1->ref_slot1[p8], static_cast<int16_t>(mp & 0xffff), static_cast<int16_t>(mp >> 16),
                           static_cast<int16_t>(mp1 & 0xffff), static_cast<int16_t>(mp1 >> 16), Q->ref_slot[q8],
                           Q1->ref_slot1[q8], static_cast<int16_t>(mq & 0xffff), static_cast<int16_t>(mq >> 16),
                           static_cast<int16_t>(mq1 & 0xffff), static_cast<int16_t>(mq1 >> 16));
  }
  if (P->ref_slot[p8] != Q->ref_slot[q8]) return 1;
  const int dx = static_cast<int16_t>(mp & 0xffff) - static_cast<int16_t>(mq & 0xffff);
  const int dy = static_cast<int16_t>(mp >> 16) - static_cast<int16_t>(mq >> 16);
  return (dx >= 4 || dx <= -4 || dy >= 4 || dy <= -4) ? 1 : 0;
}

// the packed parameters of an edge whose average QP is qpav (DbkInfo::lv)
__device__ __forceinline__ uint32_t edge_word(int qpav, int fa, int fb) {
  const int ia = min(max(qpav + fa, 0), 51), ib = min(max(qpav + fb, 0), 51);
  const uint32_t alpha = kAl[ia], beta = kBe[ib];
  if (!alpha || !beta) return 0u;
  return alpha | beta << 8 | static_cast<uint32_t>(kTc[ia][0]) << 16 | static_cast<uint32_t>(kTc[ia][1]) << 21 |
         static_cast<uint32_t>(kTc[ia][2]) << 26;
}

// grid (ceil(nmb / 16), pictures): 16 lanes per macroblock, lane = raster
// 4x4 block b, which derives the bS of the vertical edge on its left and of
// the horizontal edge above it (8.7.2.1); the macroblock's 32 nibbles meet in
// an OR butterfly over its 16 lanes, so the wavefront below reads one 32-byte
// descriptor per macroblock.  (A lane per macroblock walking all 32 edges
// made every load a strided 4-byte gather.)
__device__ void bs_mb(const FullReconArgs &a, int slot, int di, int mb, int b) {
  const int mbw = a.P.mb_width, nmb = mbw * a.P.mb_height;
  const bool ok = mb < nmb;
  const int mbc = ok ? mb : nmb - 1;  // tail lanes: a valid macroblock, result unused (the butterfly needs them)
  const MbRec *Q = a.recs + static_cast<int64_t>(slot) * nmb + mbc;
  const MbRecB *Q1 = a.P.bframes ? a.recs1 + static_cast<int64_t>(slot) * nmb + mbc : nullptr;
  const MbHdr hq = load_hdr(Q);
  const FullSlice &sd = a.slices[hq.slice];
  const int x = mbc % mbw, y = mbc / mbw, bx = b & 3, by = b >> 2;
  const int idc = sd.dbk_idc, tq = hq.type;
  uint32_t w[4] = {0, 0, 0, 0};
  int qpl = 0, qpt = 0;
  if (idc != 1) {
    const MbRec *PL = Q - 1, *PT = Q - mbw;
    bool fl = x > 0, ft = y > 0;
    int tl = 0, tt = 0;
    if (fl) {
      const MbHdr h = load_hdr(PL);
      if (idc == 2 && h.slice != hq.slice) fl = false;
      tl = h.type;
      qpl = tl == kMbPcm ? 0 : h.qp;
    }
    if (ft) {
      const MbHdr h = load_hdr(PT);
      if (idc == 2 && h.slice != hq.slice) ft = false;
      tt = h.type;
      qpt = tt == kMbPcm ? 0 : h.qp;
    }
    const bool t8 = (hq.modes & kModeT8) != 0;
#pragma unroll
    for (int dir = 0; dir < 2; ++dir) {
      const int e = dir ? by : bx, seg = dir ? bx : by;
      if (e == 0 && !(dir ? ft : fl)) continue;
      if (t8 && (e & 1)) continue;  // 8x8 transform: no 4-sample internal luma edges (chroma uses e = 0, 2)
      const MbRec *Pm = e ? Q : (dir ? PT : PL);
      const MbRecB *Pm1 = Q1 ? Q1 - (e ? 0 : (dir ? mbw : 1)) : nullptr;
      const int tp = e ? tq : (dir ? tt : tl);
      const int bp = dir ? (e ? b - 4 : 12 + seg) : (e ? b - 1 : seg * 4 + 3);
      const int bS = bs_dev(Pm, Pm1, bp, Q, Q1, b, tp, tq, e == 0);
      w[dir * 2 + (e >> 1)] |= static_cast<uint32_t>(bS) << (((e & 1) * 4 + seg) * 4);
    }
  }
#pragma unroll
  for (int m = 1; m < 16; m <<= 1)
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] |= static_cast<uint32_t>(__shfl_xor(static_cast<int>(w[i]), m, 16));
  if (!ok || b > 5) return;
  DbkInfo *o = a.dbk + static_cast<int64_t>(di) * nmb + mb;
  const int qpq = tq == kMbPcm ? 0 : hq.qp;
  if (b == 0) {
    reinterpret_cast<uint4 *>(o)[0] = make_uint4(w[0], w[1], w[2], w[3]);
  } else if (b == 1) {
    const uint32_t qp = static_cast<uint32_t>(qpq) | (static_cast<uint32_t>(qpl) << 8) |
                        (static_cast<uint32_t>(qpt) << 16) | (idc == 1 ? 1u << 24 : 0u);
    reinterpret_cast<uint4 *>(o)[1] = make_uint4(qp, static_cast<uint32_t>(sd.dbk_a), static_cast<uint32_t>(sd.dbk_b), 0u);
  } else {
    // edge parameter words: lanes 2 / 3 luma vertical / horizontal, 4 / 5 chroma
    const bool horiz = (b & 1) != 0;
    const int qpp = horiz ? qpt : qpl;  // the macroblock across edge 0
    uint32_t e4[4];
    if (b < 4) {
#pragma unroll
      for (int e = 0; e < 4; ++e) e4[e] = edge_word(e ? qpq : (qpp + qpq + 1) >> 1, sd.dbk_a, sd.dbk_b);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int off = (k & 1) ? a.P.cqp_off2 : a.P.cqp_off;
        const int cq = full::qpc_of(qpq, off);
        e4[k] = edge_word(k < 2 ? (full::qpc_of(qpp, off) + cq + 1) >> 1 : cq, sd.dbk_a, sd.dbk_b);
      }
    }
    reinterpret_cast<uint4 *>(o)[b] = make_uint4(e4[0], e4[1], e4[2], e4[3]);
  }
}
__global__ void __launch_bounds__(256) h264_bs_full(FullReconArgs a) {
  const int4 f = a.frames[blockIdx.y];
  bs_mb(a, f.x, f.y, blockIdx.x * 16 + (threadIdx.x >> 4), threadIdx.x & 15);
}


__device__ __forceinline__ uint32_t u4_at(const uint4 &v, int i) {
  return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}

// Luma and chroma edges in one instruction stream (8.7.2.3 / 8.7.2.4): s =
// p3 p2 p1 p0 q0 q1 q2 q3.  A chroma lane holds p1 p0 q0 q1 at s[2..5]; with
// ap / aq < beta forced false it takes exactly the chroma filter (tC = tC0 +
// 1, only p0 / q0 change, bS 4: p0' = (2 p1 + p0 + q1 + 2) >> 2), so a wave
// whose lanes mix luma and chroma runs one filter, not both
// The p and q sides of the edge sit in the two 16-bit halves of one register
// (p low, q high): the standard's p-side and q-side formulas mirror each
// other, so one packed instruction computes both (v_pk_* on gfx950), with the
// half-swapped registers (q, p) for the mirrored terms (round 5: content /
// noise reconstruction -3 % / -2 %, 103 -> 85 VGPRs, bit-exact;
// profiles/r05u_deblock_packed_filter_ab.json).
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
typedef int16_t i16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 pk_swap(u16x2 v) { return u16x2{v.y, v.x}; }
__device__ __forceinline__ u16x2 pk_pair(int p, int q) {
  return u16x2{static_cast<uint16_t>(p), static_cast<uint16_t>(q)};
}
__device__ __forceinline__ i16x2 pk_abs(i16x2 v) { return __builtin_elementwise_max(v, -v); }
__device__ __forceinline__ void filt_pk(int (&s)[8], int bS, uint32_t w, bool chroma) {
  const int alpha = w & 255, beta = (w >> 8) & 255;
  const u16x2 A = pk_pair(s[3], s[4]), B = pk_pair(s[2], s[5]), C = pk_pair(s[1], s[6]), D = pk_pair(s[0], s[7]);
  const u16x2 As = pk_swap(A), Bs = pk_swap(B);
  const i16x2 d1 = pk_abs(__builtin_bit_cast(i16x2, B) - __builtin_bit_cast(i16x2, A));
  const int d0 = abs(s[3] - s[4]);
  if (!(d0 < alpha && d1.x < beta && d1.y < beta)) return;
  const i16x2 d2 = pk_abs(__builtin_bit_cast(i16x2, C) - __builtin_bit_cast(i16x2, A));
  const bool apb = !chroma && d2.x < beta, aqb = !chroma && d2.y < beta;
  u16x2 nA, nB = B, nC = C;
  if (bS < 4) {
    const int tc0 = (w >> (11 + 5 * bS)) & 31;
    const int tc = tc0 + (chroma ? 1 : static_cast<int>(apb) + static_cast<int>(aqb));
    const int delta = min(max((((s[4] - s[3]) << 2) + (s[2] - s[5]) + 4) >> 3, -tc), tc);
    const i16x2 a2 = __builtin_bit_cast(i16x2, A) + i16x2{static_cast<int16_t>(delta), static_cast<int16_t>(-delta)};
    nA = __builtin_bit_cast(u16x2, __builtin_elementwise_min(__builtin_elementwise_max(a2, i16x2{0, 0}), i16x2{255, 255}));
    const u16x2 avg = (A + As + u16x2{1, 1}) >> 1;  // (p0 + q0 + 1) >> 1 in both halves
    i16x2 h = (__builtin_bit_cast(i16x2, C + avg) - __builtin_bit_cast(i16x2, B << 1)) >> 1;
    const int16_t t0 = static_cast<int16_t>(tc0);
    h = __builtin_elementwise_min(__builtin_elementwise_max(h, i16x2{static_cast<int16_t>(-t0), static_cast<int16_t>(-t0)}),
                                  i16x2{t0, t0});
    const u16x2 b2 = B + __builtin_bit_cast(u16x2, h);
    nB = u16x2{apb ? b2.x : B.x, aqb ? b2.y : B.y};
  } else {
    const bool small = d0 < ((alpha >> 2) + 2);
    const u16x2 s0 = (C + (B << 1) + (A << 1) + (As << 1) + Bs + u16x2{4, 4}) >> 3;
    const u16x2 s1 = (C + B + A + As + u16x2{2, 2}) >> 2;
    const u16x2 s2 = ((D << 1) + C + (C << 1) + B + A + As + u16x2{4, 4}) >> 3;
    const u16x2 w0 = ((B << 1) + A + Bs + u16x2{2, 2}) >> 2;
    const bool sp = apb && small, sq = aqb && small;
    nA = u16x2{sp ? s0.x : w0.x, sq ? s0.y : w0.y};
    nB = u16x2{sp ? s1.x : B.x, sq ? s1.y : B.y};
    nC = u16x2{sp ? s2.x : C.x, sq ? s2.y : C.y};
  }
  s[3] = nA.x;
  s[4] = nA.y;
  s[2] = nB.x;
  s[5] = nB.y;
  s[1] = nC.x;
  s[6] = nC.y;
}

// vertical pass: a chroma lane's interleaved row (Cb Cr pairs from x = -2)
// reordered so that slot s = (edge 2 (s >> 1), plane s & 1) has p1 p0 q0 q1
// at u[4 s + 2 .. 4 s + 5]: u[j] = r[kDbkCPerm[j]], r[i] = u[kDbkCInv[i]]
__device__ __constant__ static const uint8_t kDbkCPerm[20] = {18, 19, 0, 2, 4, 6, 1, 3, 5, 7,
                                                             8, 10, 12, 14, 9, 11, 13, 15, 16, 17};
__device__ __constant__ static const uint8_t kDbkCInv[20] = {2, 6, 3, 7, 4, 8, 5, 9, 10, 14,
                                                            11, 15, 12, 16, 13, 17, 18, 19, 0, 1};
// horizontal pass: chroma row of u index j (p1 p0 q0 q1 of chroma edges 0 / 4
// at u[2..5] / u[10..13], rows 6, 7 at u[14], u[15]); -1: none
constexpr int dbk_hrow(int j) {
  return (j >= 2 && j <= 5) ? j - 2 : ((j >= 10 && j <= 13) ? j - 6 : (j == 14 ? 8 : (j == 15 ? 9 : -1)));
}

}  // namespace


int nal_unescape_launch(const uint8_t *es, uint8_t *rbsp, const FullSlice *slices, int32_t n_slices,
                        int32_t *rbsp_len, hipStream_t s) {
  if (n_slices <= 0) return VTS_OK;
  hipLaunchKernelGGL(nal_unescape, dim3(n_slices), dim3(kUnescThreads), 0, s, es, rbsp, slices, rbsp_len);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(VTS_E_HIP, "nal_unescape launch: %s", hipGetErrorString(e));
  return VTS_OK;
}

int parse_full_launch(const FullParseArgs &a, hipStream_t s) {
  if (a.n_slices <= 0) return VTS_OK;
  if (a.P.cabac) {
    const size_t lds = full::syn_lds_bytes(a.P.mb_width);
    if (lds > 60 * 1024) return fail(VTS_E_UNSUPPORTED, "picture wider than the CABAC parser's LDS row allows");
    if (!a.arena_top) return fail(VTS_E_INVALID, "CABAC parse launch without its arena counter");
    hipLaunchKernelGGL(h264_parse_full_cabac, dim3(a.n_slices), dim3(64), lds, s, a);
  } else {
    hipLaunchKernelGGL(h264_parse_full, dim3(a.n_slices), dim3(64), 0, s, a);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(VTS_E_HIP, "h264_parse_full launch: %s", hipGetErrorString(e));
  return VTS_OK;
}

size_t derive_lds_bytes(int mb_height) {
  const int threads = 64 * ((mb_height + 63) / 64);
  return sizeof(full::DWork) * static_cast<size_t>(threads) + sizeof(full::DEdge) * 5 * static_cast<size_t>(mb_height);
}

// one wave that returns after `us` microseconds (the 100 MHz real-time
// counter): what a stream runs before a launch that must not be dispatched
// ahead of another queue's
__global__ void __launch_bounds__(64) stream_delay(uint32_t us) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime(), n = 100ull * us;
  while (__builtin_amdgcn_s_memrealtime() - t0 < n) __builtin_amdgcn_s_sleep(8);
}
int delay_launch(uint32_t us, hipStream_t s) {
  hipLaunchKernelGGL(stream_delay, dim3(1), dim3(64), 0, s, us);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(VTS_E_HIP, "stream_delay launch: %s", hipGetErrorString(e));
  return VTS_OK;
}

int derive_launch(const DeriveArgs &a, int n_pictures, hipStream_t s) {
  if (n_pictures <= 0) return VTS_OK;
  if (a.P.mb_height > 256) return fail(VTS_E_UNSUPPORTED, "picture taller than 256 macroblock rows (h264_derive)");
  const int threads = 64 * ((a.P.mb_height + 63) / 64);
  hipLaunchKernelGGL(h264_derive, dim3(n_pictures), dim3(threads), derive_lds_bytes(a.P.mb_height), s, a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(VTS_E_HIP, "h264_derive launch: %s", hipGetErrorString(e));
  return VTS_OK;
}

// ------------------------------------------------ deblocking by plane
// Luma and chroma deblock independently (they share only the bS words), and
// each needs 16 lanes per macroblock row instead of 32: one workgroup per
// (picture, plane) holds kDpGroups = 64 macroblock rows in flight (16 waves x
// 4 groups of 16 lanes), so a 720p / 1080p picture is one pass of the
// wavefront.  Per plane and step: rows above from an LDS ring (the rows a
// macroblock's top edge needs pass from row to row in LDS, never through
// HBM), vertical pass (lane = sample row),
// horizontal pass (lane = sample column), write-back (rows the row below
// finishes excepted), ring lines for the row below; the four rows of a wave
// run in lockstep two macroblocks apart, a wave's first row waits for the
// previous wave's last through prog[].
constexpr int kDpGroups = kDbkThreads / 16;
constexpr int kDpRingCols = 16;
struct DpTileY {
  uint8_t s[20][20];  // rows -4..15 x cols -4..15
};
struct DpTileC {
  uint8_t s[10][20];  // chroma rows -2..7 x interleaved bytes -4..15
};
struct DpLineY {
  uint8_t s[4][16];  // rows 12..15
};
struct DpLineC {
  uint8_t s[2][16];  // chroma rows 6..7
};
constexpr size_t kDpLdsY = sizeof(DpTileY) * kDpGroups + sizeof(DpLineY) * kDpGroups * kDpRingCols;
constexpr size_t kDpLdsC = sizeof(DpTileC) * kDpGroups + sizeof(DpLineC) * kDpGroups * kDpRingCols;
constexpr size_t kDpLds = kDpLdsY > kDpLdsC ? kDpLdsY : kDpLdsC;

// (A row one macroblock behind the row above instead of two was bit-exact
// and no faster)
template <bool kLuma>
__device__ __forceinline__ void dp_plane(const FullReconArgs &a, int slot, int di, uint8_t *lds, int *prog) {
  using Tile = typename std::conditional<kLuma, DpTileY, DpTileC>::type;
  using Line = typename std::conditional<kLuma, DpLineY, DpLineC>::type;
  Tile *tiles = reinterpret_cast<Tile *>(lds);
  Line(*ring)[kDpRingCols] = reinterpret_cast<Line(*)[kDpRingCols]>(lds + sizeof(Tile) * kDpGroups);
  const int mbw = a.P.mb_width, mbh = a.P.mb_height, nmb = mbw * mbh;
  const DbkInfo *fdbk = a.dbk + static_cast<int64_t>(di) * nmb;
  uint8_t *Y = surf_at(a, slot);
  const uint32_t uvo = static_cast<uint32_t>(a.uv_off);
  auto at = [Y](uint32_t o) { return Y + static_cast<uint64_t>(o); };
  const int pitch = a.pitch;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = lane >> 4, l = lane & 15;
  constexpr int kRows = kLuma ? 16 : 8;  // sample rows of a macroblock
  constexpr int kTop = kLuma ? 4 : 2;     // tile rows above the macroblock (kept in the ring lines)
  const bool lrow = l < kRows;           // vertical pass / write-back lane
  const int row = kLuma ? l : min(l, 7);
  Tile &t = tiles[wave * 4 + grp];
  constexpr int vq = kLuma ? 2 : 4, hq = kLuma ? 3 : 5;
  for (int p = wave; 4 * p < mbh; p += kDbkWaves) {
    const int y = 4 * p + grp;
    const bool row_ok = y < mbh;
    const int ya = row_ok ? y : mbh - 1;
    const bool last_row = y == mbh - 1;
    const int rs = y % kDpGroups, rsa = (y + kDpGroups - 1) % kDpGroups;
    const uint32_t rowo = kLuma ? static_cast<uint32_t>((ya * 16 + row) * pitch)
                                : uvo + static_cast<uint32_t>((ya * 8 + row) * pitch);
    const DbkInfo *const drow = fdbk + ya * mbw;
    // this row's ring slot was the row kDpGroups above's: its consumer must be done
    if (row_ok && y - kDpGroups >= 0) {
      while (__hip_atomic_load(&prog[y - kDpGroups + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < mbw + 1)
        __builtin_amdgcn_s_sleep(1);
    }
    uint32_t left = 0;   // carried cols 12..15 of the previous macroblock (this lane's row)
    bool ldirty = false;  // ... and they differ from what HBM holds (that macroblock was filtered)
    const uint4 *dq = reinterpret_cast<const uint4 *>(drow);
    uint4 nbs = dq[0], nv = dq[vq], nh = dq[hq];
    uint4 npx = *reinterpret_cast<const uint4 *>(at(rowo));
    constexpr int kLag = 2;
    for (int it = 0; it < mbw + 3 * kLag; ++it) {
      const int x = it - kLag * grp;
      const bool act = row_ok && x >= 0 && x < mbw;
      const uint4 bsw = nbs, pv = nv, ph = nh, q4 = npx;
      {
        const int xn = min(max(x + 1, 0), mbw - 1);
        const uint4 *dn = reinterpret_cast<const uint4 *>(drow + xn);
        nbs = dn[0];
        nv = dn[vq];
        nh = dn[hq];
        npx = *reinterpret_cast<const uint4 *>(at(rowo + static_cast<uint32_t>(xn * 16)));
      }
      // a wave's first row waits for the previous wave's last row; its last
      // row waits until it may overwrite ring column x (the next wave's first
      // row read column x - kDpRingCols)
      if (act) {
        const int need_up = (grp == 0 && y > 0) ? (x + 1 < mbw ? x + 2 : mbw + 1) : -(1 << 30);
        const int need_dn = (grp == 3 && y + 1 < mbh) ? x - kDpRingCols + 1 : -(1 << 30);
        const int *pu = &prog[y > 0 ? y - 1 : 0], *pd = &prog[y + 1 < mbh ? y + 1 : y];
        while (__hip_atomic_load(pu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need_up ||
               __hip_atomic_load(pd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need_dn)
          __builtin_amdgcn_s_sleep(1);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      const bool still = (bsw.x | bsw.y | bsw.z | bsw.w) == 0u;
      constexpr int kAbove = kLuma ? 4 : 2;  // rows above from the ring
      auto load_above = [&]() {
        if (act && l < kAbove && y > 0) {
          const Line &L = ring[rsa][x & (kDpRingCols - 1)];
          *reinterpret_cast<uint4 *>(&t.s[l][4]) = *reinterpret_cast<const uint4 *>(&L.s[l][0]);
        }
      };
      load_above();
      // ---- vertical edges: lane = sample row
      if (act && lrow && !still) {
        const uint32_t wv[5] = {x > 0 ? left : 0u, q4.x, q4.y, q4.z, q4.w};
        int r[20], u[20];
#pragma unroll
        for (int i = 0; i < 20; ++i) r[i] = (wv[i >> 2] >> ((i & 3) * 8)) & 255;
#pragma unroll
        for (int j = 0; j < 20; ++j) u[j] = kLuma ? r[j] : r[kDbkCPerm[j]];
        const int seg = kLuma ? row >> 2 : row >> 1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int bS = (u4_at(bsw, e >> 1) >> (((kLuma ? (e & 1) : 0) * 4 + seg) * 4)) & 15;
          if (!bS) continue;
          int s8[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) s8[i] = u[4 * e + i];
          filt_pk(s8, bS, u4_at(pv, e), !kLuma);
#pragma unroll
          for (int i = 0; i < 8; ++i) u[4 * e + i] = s8[i];
        }
#pragma unroll
        for (int i = 0; i < 20; ++i) r[i] = kLuma ? u[i] : u[kDbkCInv[i]];
        uint8_t *dst = &t.s[kTop + row][0];
#pragma unroll
        for (int i = 0; i < 5; ++i)
          *reinterpret_cast<uint32_t *>(dst + 4 * i) = pack4(r[4 * i], r[4 * i + 1], r[4 * i + 2], r[4 * i + 3]);
      }
      lane_sync();
      // ---- horizontal edges: lane = sample column (chroma: interleaved byte column)
      if (act && !still) {
        const int pl = l & 1, seg = l >> 2;
        int u[20];
        if constexpr (kLuma) {
          const uint8_t *col = &t.s[0][4 + l];
#pragma unroll
          for (int i = 0; i < 20; ++i) u[i] = col[i * 20];
        } else {
          const uint8_t *col = &t.s[0][4 + l];
#pragma unroll
          for (int i = 0; i < 20; ++i) {
            const int cr = dbk_hrow(i);
            u[i] = cr >= 0 ? col[cr * 20] : 0;
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          int bS = (u4_at(bsw, 2 + (e >> 1)) >> (((kLuma ? (e & 1) : 0) * 4 + seg) * 4)) & 15;
          if (!kLuma && (e & 1)) bS = 0;
          if (!bS) continue;
          int s8[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) s8[i] = u[4 * e + i];
          filt_pk(s8, bS, u4_at(ph, kLuma ? e : e + pl), !kLuma);
#pragma unroll
          for (int i = 0; i < 8; ++i) u[4 * e + i] = s8[i];
        }
        if constexpr (kLuma) {
          uint8_t *col = &t.s[0][4 + l];
#pragma unroll
          for (int i = 1; i < 20; ++i) col[i * 20] = static_cast<uint8_t>(u[i]);
        } else {
          uint8_t *col = &t.s[0][4 + l];
#pragma unroll
          for (int i = 1; i < 20; ++i) {
            const int cr = dbk_hrow(i);
            if (cr >= 1) col[cr * 20] = static_cast<uint8_t>(u[i]);
          }
        }
      }
      lane_sync();
      // ---- write back: this macroblock's rows shifted 4 bytes left except the
      // ones the row below finishes (luma 13..15, chroma 7), the ring lines for
      // the row below, the rows above that this macroblock's top edge finished
      if (act) {
        if (lrow) {
          uint32_t w0, w1, w2, w3;
          if (still) {
            w0 = left;
            w1 = q4.x;
            w2 = q4.y;
            w3 = q4.z;
            left = q4.w;
          } else {
            const uint8_t *src = &t.s[kTop + row][0];
            w0 = *reinterpret_cast<const uint32_t *>(src);
            w1 = *reinterpret_cast<const uint32_t *>(src + 4);
            w2 = *reinterpret_cast<const uint32_t *>(src + 8);
            w3 = *reinterpret_cast<const uint32_t *>(src + 12);
            left = *reinterpret_cast<const uint32_t *>(src + 16);
          }
          // a still macroblock's own samples are what HBM holds (only this
          // step writes its rows 0..12 / 0..6): stored are the left
          // neighbour's last columns when that one was filtered
          if (last_row || row < (kLuma ? 13 : 7)) {
            uint8_t *dst = at(rowo + static_cast<uint32_t>(x * 16));
            if (x > 0 && (!still || ldirty)) *reinterpret_cast<uint32_t *>(dst - 4) = w0;
            if (!still) {
              *reinterpret_cast<uint32_t *>(dst) = w1;
              *reinterpret_cast<uint32_t *>(dst + 4) = w2;
              *reinterpret_cast<uint32_t *>(dst + 8) = w3;
              if (x == mbw - 1) *reinterpret_cast<uint32_t *>(dst + 12) = left;
            }
          }
          ldirty = !still;
          const int lr = row - (kRows - kTop);  // ring line of this lane's row (luma 12..15, chroma 6..7)
          if (!last_row && lr >= 0) {
            Line &C = ring[rs][x & (kDpRingCols - 1)];
            uint8_t *cur = &C.s[lr][0];
            if (x > 0) *reinterpret_cast<uint32_t *>(&ring[rs][(x - 1) & (kDpRingCols - 1)].s[lr][12]) = w0;
            *reinterpret_cast<uint32_t *>(cur) = w1;
            *reinterpret_cast<uint32_t *>(cur + 4) = w2;
            *reinterpret_cast<uint32_t *>(cur + 8) = w3;
            if (x == mbw - 1) *reinterpret_cast<uint32_t *>(cur + 12) = left;
          }
        }
        // luma rows -3..-1 / chroma row -1 of the macroblock above (lane index
        // opaque: the offsets computed per step, not kept per row)
        if (l < (kLuma ? 3 : 1) && y > 0) {
          int lo = lane;
          asm volatile("" : "+v"(lo));
          const int i = lo & 15, g = lo >> 4, yy = min(4 * p + g, mbh - 1);
          const Tile &tt = tiles[__builtin_amdgcn_readfirstlane(wave) * 4 + g];
          // luma: tile row 1 + i (rows -3..-1); chroma: tile row 1 (row -1)
          const uint4 v = *reinterpret_cast<const uint4 *>(&tt.s[1 + i][4]);
          const uint32_t o = kLuma ? static_cast<uint32_t>((yy * 16 + i - 3) * pitch)
                                   : uvo + static_cast<uint32_t>((yy * 8 - 1) * pitch);
          *reinterpret_cast<uint4 *>(at(o + static_cast<uint32_t>(x * 16))) = v;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      if (act && l == 0) {
        __hip_atomic_store(&prog[y], x + 1 < mbw ? x + 1 : mbw + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
}
// grid: 2 x pictures of the level (even blocks luma, odd chroma)
__global__ void __launch_bounds__(kDbkThreads) h264_deblock_plane(FullReconArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kDpLds];
  __shared__ int prog[1024];  // per macroblock row: macroblocks finished (mbw + 1: row flushed)
  VTS_WG_TRACE(0, 0, a.frames);
  for (int i = threadIdx.x; i < a.P.mb_height; i += kDbkThreads) prog[i] = 0;
  __syncthreads();
  const int4 f = a.frames[blockIdx.x >> 1];
  if ((blockIdx.x & 1) == 0) dp_plane<true>(a, f.x, f.y, lds, prog);
  else dp_plane<false>(a, f.x, f.y, lds, prog);
  VTS_WG_TRACE(0, 1, a.frames);
}

int bs_full_launch(const FullReconArgs &a, int n_frames, hipStream_t s) {
  if (n_frames <= 0) return VTS_OK;
  if (n_frames > 65535) return fail(VTS_E_UNSUPPORTED, "more than 65535 pictures in one bS launch");
  const int nmb = a.P.mb_width * a.P.mb_height;
  hipLaunchKernelGGL(h264_bs_full, dim3((nmb + 15) / 16, n_frames), dim3(256), 0, s, a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(VTS_E_HIP, "h264_bs_full launch: %s", hipGetErrorString(e));
  return VTS_OK;
}

int recon_full_launch(const FullReconArgs &a, int n_frames, hipStream_t s, hipEvent_t after_inter) {
  if (n_frames <= 0) return VTS_OK;
  const int nmb = a.P.mb_width * a.P.mb_height;
  if (a.P.mb_height > 1024) return fail(VTS_E_UNSUPPORTED, "picture taller than 1024 macroblock rows");
  if (n_frames > 65535) return fail(VTS_E_UNSUPPORTED, "more than 65535 pictures in one level launch");
  hipLaunchKernelGGL(h264_inter_full, dim3((nmb + 15) / 16, n_frames), dim3(kInterThreads), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(VTS_E_HIP, "h264_inter_full launch: %s", hipGetErrorString(e));
  if (after_inter && hipEventRecord(after_inter, s) != hipSuccess) return fail(VTS_E_HIP, "hipEventRecord after h264_inter_full");
  // lane-parallel intra (default) while its LDS fits, else the by-block kernel
  const size_t i2_lds = i2_lds_bytes(a.P.mb_width, a.P.mb_height);
  if (a.intra_kernel != 1 && i2_lds <= 160 * 1024) {
    hipLaunchKernelGGL(h264_intra_v2, dim3(n_frames), dim3(kI2Threads), i2_lds, s, a);
    e = hipGetLastError();
    if (e != hipSuccess) return fail(VTS_E_HIP, "h264_intra_v2 launch: %s", hipGetErrorString(e));
  } else {
    hipLaunchKernelGGL(h264_intra_full, dim3(n_frames), dim3(kIntraThreads), sizeof(uint16_t) * nmb, s, a);
    e = hipGetLastError();
    if (e != hipSuccess) return fail(VTS_E_HIP, "h264_intra_full launch: %s", hipGetErrorString(e));
  }
  if (a.deblock) {
    hipLaunchKernelGGL(h264_deblock_plane, dim3(2 * n_frames), dim3(kDbkThreads), 0, s, a);
    e = hipGetLastError();
    if (e != hipSuccess) return fail(VTS_E_HIP, "h264_deblock_plane launch: %s", hipGetErrorString(e));
  }
  return VTS_OK;
}

}  // namespace vts
