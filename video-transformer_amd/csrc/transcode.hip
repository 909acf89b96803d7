// transcode.hip — vts_transcode: the 360p upload transcode on the device
// (replaces the pixel work of the reference's
// ContentAnalyzer._compress_video_for_upload, content_analyzer.py:167-236,
// `ffmpeg -vf scale=-2:360 -c:v libx264 -crf 28`).  DESIGN.md §11.
//
// Pipeline, all device work after the one decode:
//   1. the session's decode + score run (run_all), with `small_window`
//      downscaling every window's frames (area filter, NV12 -> NV12 at
//      (w, 360), coded 16-aligned) into a whole-video store while they sit
//      in the decode ring;
//   2. GOP plan on the host: IDR at frame 0 and every `keyint` frames (and,
//      opt-in, at every scene cut from the scores);
//   3. per GOP position j ("level", every GOP at once, as the decoder's
//      reconstruct levels): `enc_search` — one wave per macroblock, full
//      integer motion search in LDS against the previous reconstruction,
//      decision inter / I_PCM, reconstruction written (the next level's
//      reference); then per chunk of 16 levels on a second stream:
//      `enc_write` — one lane per slice (macroblock row) writes the CAVLC
//      slice NAL with emulation prevention into a fixed-capacity staging slot,
//      leaving I_PCM payloads as gaps; `enc_scan` — device offsets;
//      `enc_gather` + `enc_pcm` — packed output, one D2H copy per chunk;
//   4. host: MP4 mux (Mp4Writer) in display order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <memory>
#include <numeric>
#include <string>
#include <vector>

#include "mp4.h"
#include "recon_full.h"
#include "session.h"

namespace vts {
namespace {

constexpr uint32_t kPcmCmd = 0x80008000u;  // (mvx, mvy) = (-32768, -32768): never a motion
constexpr int kMaxTaps = 16;
constexpr int kMaxRange = 16;
constexpr int kWinPitch = 16 + 2 * kMaxRange + 4;  // LDS window row pitch (bytes)

// ----------------------------------------------------------- downscale
// Area filter, per axis: destination o covers source footprint [o n, (o+1) n)
// in units of 1/m; source i covers [i m, (i+1) m).  Tap table entry o =
// [i0, w_0 .. w_{K-1}] (weights / gcd(n, m)); outputs past the display size
// (coded padding) repeat the last display entry.
struct DsArgs {
  const uint8_t *src;      // ring surface of the window's first frame
  int64_t src_stride;
  int32_t pitch, uv_rows;  // UV plane at pitch * uv_rows
  int32_t sw, sh;          // source display size
  uint8_t *dst;            // small store, the window's first frame
  int64_t dst_stride;
  int32_t cw, ch;          // destination coded size
  const int32_t *tx, *ty, *tcx, *tcy;
  int32_t kx, ky, kcx, kcy;
  int32_t tl, tc;          // normalisers (product of the axes' n / gcd)
  int64_t n_frames;
};

__device__ __forceinline__ uint32_t area_px(const uint8_t *p, int pitch, int step, const int32_t *ex,
                                            int kx, const int32_t *ey, int ky, int nx, int ny, int t) {
  uint32_t sum = 0;
  const int x0 = ex[0], y0 = ey[0];
  for (int j = 0; j < ky; ++j) {
    const uint32_t wy = static_cast<uint32_t>(ey[1 + j]);
    if (!wy) continue;
    const uint8_t *row = p + static_cast<int64_t>(min(y0 + j, ny - 1)) * pitch;
    uint32_t s = 0;
    for (int i = 0; i < kx; ++i) s += static_cast<uint32_t>(ex[1 + i]) * row[min(x0 + i, nx - 1) * step];
    sum += wy * s;
  }
  const uint32_t v = (sum + static_cast<uint32_t>(t) / 2) / static_cast<uint32_t>(t);
  return v < 1 ? 1u : v;
}

// Integer ratio K on both axes (720p -> 360p: 2, 1080p -> 360p: 3): four
// outputs from K rows of 4K contiguous bytes, dword loads; luma and NV12
// chroma (4 bytes U0 V0 U1 V1 from 2K source pairs) share the addressing.
template <int K>
__device__ __forceinline__ uint32_t box4(const uint8_t *p, int pitch, bool chroma) {
  uint32_t acc[4] = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint32_t *r = reinterpret_cast<const uint32_t *>(p + static_cast<int64_t>(j) * pitch);
#pragma unroll
    for (int w = 0; w < K; ++w) {
      const uint32_t v = r[w];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int byte = 4 * w + b;  // 0 .. 4K-1
        // luma: output byte / K; chroma: pair byte / 2 -> output pair (pair / K), plane byte & 1
        const int q = chroma ? 2 * ((byte >> 1) / K) + (byte & 1) : byte / K;
        acc[q] += (v >> (8 * b)) & 255u;
      }
    }
  }
  uint32_t out = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t m = (acc[q] + K * K / 2) / (K * K);
    out |= (m < 1 ? 1u : m) << (8 * q);
  }
  return out;
}

template <int K>
__global__ void __launch_bounds__(256) downscale_nv12(DsArgs a) {
  const int groups = a.cw / 4;
  const int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  const int rows = a.ch + a.ch / 2;
  if (t >= static_cast<int64_t>(groups) * rows) return;
  const int64_t f = blockIdx.y;
  const int g = static_cast<int>(t % groups), row = static_cast<int>(t / groups);
  const uint8_t *src = a.src + f * a.src_stride;
  uint8_t *dst = a.dst + f * a.dst_stride;
  if constexpr (K > 0) {
    const int dw = a.sw / K, dh = a.sh / K;  // output display size
    if (row < dh && 4 * g + 3 < dw) {
      *reinterpret_cast<uint32_t *>(dst + static_cast<int64_t>(row) * a.cw + 4 * g) =
          box4<K>(src + static_cast<int64_t>(K * row) * a.pitch + 4 * K * g, a.pitch, false);
      return;
    }
    if (row >= a.ch && row - a.ch < dh / 2 && 4 * g + 3 < dw) {
      const int cy = row - a.ch;
      const uint8_t *uv = src + static_cast<int64_t>(a.pitch) * a.uv_rows;
      *reinterpret_cast<uint32_t *>(dst + static_cast<int64_t>(a.cw) * a.ch + static_cast<int64_t>(cy) * a.cw +
                                    4 * g) = box4<K>(uv + static_cast<int64_t>(K * cy) * a.pitch + 4 * K * g, a.pitch, true);
      return;
    }
  }
  uint32_t out = 0;
  if (row < a.ch) {
    const int32_t *ey = a.ty + static_cast<int64_t>(row) * (1 + a.ky);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int32_t *ex = a.tx + static_cast<int64_t>(4 * g + q) * (1 + a.kx);
      out |= area_px(src, a.pitch, 1, ex, a.kx, ey, a.ky, a.sw, a.sh, a.tl) << (8 * q);
    }
    *reinterpret_cast<uint32_t *>(dst + static_cast<int64_t>(row) * a.cw + 4 * g) = out;
  } else {
    const int cy = row - a.ch;
    const uint8_t *uv = src + static_cast<int64_t>(a.pitch) * a.uv_rows;
    const int32_t *ey = a.tcy + static_cast<int64_t>(cy) * (1 + a.kcy);
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // bytes U0 V0 U1 V1 of chroma columns 2g, 2g+1
      const int32_t *ex = a.tcx + static_cast<int64_t>(2 * g + (q >> 1)) * (1 + a.kcx);
      out |= area_px(uv + (q & 1), a.pitch, 2, ex, a.kcx, ey, a.kcy, a.sw / 2, a.sh / 2, a.tc) << (8 * q);
    }
    *reinterpret_cast<uint32_t *>(dst + static_cast<int64_t>(a.cw) * a.ch + static_cast<int64_t>(cy) * a.cw +
                                  4 * g) = out;
  }
}

// ------------------------------------------------------ residual coding
// Quantised residual of P_L0_16x16 macroblocks: the forward
// core transform W = Cf X Cf^T, levels sign(W) min(2047, (|W| MF + f) >>
// qbits) with qbits = 15 + qp / 6 and f = 2^qbits / 6 (chroma DC through the
// 2x2 Hadamard at qbits + 1 and 2f), the decoder's own scaling + inverse
// transform (full::scale_idct4) for the reconstruction, and CAVLC
// residual_block (9.2) for the bits.  Restated in oracle/transcode_oracle.c.
constexpr int kCoefPerMb = 384;  // luma 16 x 16 by luma4x4BlkIdx, Cb / Cr DC 2 x 4, Cb / Cr AC 8 x 15 (scan order)
constexpr int kPcmBits = 3072;   // I_PCM payload: a residual bounded above it is not worth coding
__device__ __constant__ static const uint8_t kCtLen[4][17][4] = VTS_CT_LEN_DATA;
__device__ __constant__ static const uint8_t kCtCode[4][17][4] = VTS_CT_CODE_DATA;
__device__ __constant__ static const uint8_t kTzLen[15][16] = VTS_TZ_LEN_DATA;
__device__ __constant__ static const uint8_t kTzCode[15][16] = VTS_TZ_CODE_DATA;
__device__ __constant__ static const uint8_t kTzcLen[3][4] = VTS_TZC_LEN_DATA;
__device__ __constant__ static const uint8_t kTzcCode[3][4] = VTS_TZC_CODE_DATA;
__device__ __constant__ static const uint8_t kRbLen[7][15] = VTS_RB_LEN_DATA;
__device__ __constant__ static const uint8_t kRbCode[7][15] = VTS_RB_CODE_DATA;
__device__ __constant__ static const uint8_t kZz4[16] = VTS_ZZ_DATA;
__device__ __constant__ static const uint8_t kCbpInterTab[48] = VTS_CBPP_DATA;
__device__ __constant__ static const uint8_t kQpcTab[52] = VTS_QPC_DATA;
__device__ __constant__ static const uint8_t kBlkXd[16] = {0, 1, 0, 1, 2, 3, 2, 3, 0, 1, 0, 1, 2, 3, 2, 3};
__device__ __constant__ static const uint8_t kBlkYd[16] = {0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3};
__device__ __constant__ static const int kMf[6][3] = {{13107, 5243, 8066}, {11916, 4660, 7490}, {10082, 4194, 6554},
                                                      {9362, 3647, 5825},  {8192, 3355, 5243},  {7282, 2893, 4559}};

__device__ __forceinline__ int pos_class(int i, int j) { return (!(i & 1) && !(j & 1)) ? 0 : ((i & 1) && (j & 1) ? 1 : 2); }
__device__ __forceinline__ void fwd4(const int *x, int *w) {  // W = Cf X Cf^T, raster
  int t[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int a = x[i * 4], b = x[i * 4 + 1], c = x[i * 4 + 2], d = x[i * 4 + 3];
    t[i * 4] = a + b + c + d;
    t[i * 4 + 1] = 2 * a + b - c - 2 * d;
    t[i * 4 + 2] = a - b - c + d;
    t[i * 4 + 3] = a - 2 * b + 2 * c - d;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int a = t[j], b = t[4 + j], c = t[8 + j], d = t[12 + j];
    w[j] = a + b + c + d;
    w[4 + j] = 2 * a + b - c - 2 * d;
    w[8 + j] = a - b - c + d;
    w[12 + j] = a - 2 * b + 2 * c - d;
  }
}
__device__ __forceinline__ int quant1(int w, int mf, int qbits, int64_t f) {
  const int64_t z = min(static_cast<int64_t>(2047), (static_cast<int64_t>(abs(w)) * mf + f) >> qbits);
  return w < 0 ? -static_cast<int>(z) : static_cast<int>(z);
}

// bits of residual_block_cavlc (7.3.5.3.2, 9.2) of levels lv[0, maxNum) in
// scan order with nC (-1: chroma DC); nC < -1: an upper bound (coeff_token
// taken as the longest code over the nC classes and the 6-bit FLC).  With o,
// the block is also written.
struct NalOut;
template <bool kWrite>
__device__ int cavlc_block(NalOut *o, const int *lv, int maxNum, int nC);

// ------------------------------------------------------ motion search
struct SearchArgs {
  const int4 *ent;      // per frame of the level: (frame, ref slot or -1 = small[frame-1], dst slot, 0)
  const uint8_t *small;
  int64_t stride;
  uint8_t *recon;       // [slot]
  uint32_t *cmd;        // [entry][mb]
  uint8_t *cbp;         // [entry][mb] coded_block_pattern (residual coding)
  int16_t *coef;        // [entry][mb][kCoefPerMb] levels (this level's ring slot)
  int32_t cw, ch, mbw, nmb;
  int32_t range, max_sad;
  int32_t qp, _pad;     // qp >= 1: residual coding at that QP
};

__device__ __forceinline__ uint32_t u32_at(const uint8_t *lds_row, int off) {  // 4 bytes at any offset
  const uint32_t *p = reinterpret_cast<const uint32_t *>(lds_row + (off & ~3));
  return __builtin_amdgcn_alignbyte(p[1], p[0], off & 3);  // byte shift
}

// One wave per macroblock: the reference window (16 + 2R)^2 and the source
// block go to LDS; each lane takes candidates c = lane, lane + 64, ...;
// (least luma SAD, candidate index) is a 64-bit min over the wave.
#ifndef VTS_SEARCH_WAVES
#define VTS_SEARCH_WAVES 0
#endif
#ifndef VTS_SEARCH_UV_LDS
#define VTS_SEARCH_UV_LDS 0  // 1: chroma reference window staged in LDS (measured slower: 45 vs 37 ms)
#endif
#ifndef VTS_SEARCH_SRC_LDS
#define VTS_SEARCH_SRC_LDS 1  // source rows read from LDS per use, rolled row loop: 47 VGPRs (vs 163), 33 vs 37 ms
#endif
#if VTS_SEARCH_WAVES
#define VTS_SEARCH_OCC __attribute__((amdgpu_waves_per_eu(VTS_SEARCH_WAVES)))
#else
#define VTS_SEARCH_OCC
#endif
constexpr int kUvPitch = 8 + 2 * kMaxRange + 2;  // chroma window row pitch (Cb|Cr pairs)

template <int RT>  // compile-time search range (register-blocked path), 0 = any range
__global__ void __launch_bounds__(64) VTS_SEARCH_OCC enc_search(SearchArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t win[(16 + 2 * kMaxRange) * kWinPitch];
  __shared__ __attribute__((aligned(16))) uint32_t srcy[64];
  __shared__ uint16_t winuv[kUvPitch * kUvPitch];
  const int lane = threadIdx.x;
  const int64_t e = blockIdx.x / a.nmb;
  const int mb = static_cast<int>(blockIdx.x % a.nmb);
  const int mx = mb % a.mbw, my = mb / a.mbw;
  const int4 en = a.ent[e];
  const uint8_t *src = a.small + static_cast<int64_t>(en.x) * a.stride;
  const uint8_t *ref = en.y < 0 ? a.small + static_cast<int64_t>(en.x - 1) * a.stride
                                : a.recon + static_cast<int64_t>(en.y) * a.stride;
  uint8_t *dst = a.recon + static_cast<int64_t>(en.z) * a.stride;
  const int R = a.range, side = 2 * R + 1, wsz = 16 + 2 * R;
  const int x0 = mx * 16 - R, y0 = my * 16 - R;
  // source luma: lane -> row lane / 4, 4 bytes
  srcy[lane] = *reinterpret_cast<const uint32_t *>(src + static_cast<int64_t>(my * 16 + (lane >> 2)) * a.cw +
                                                   mx * 16 + 4 * (lane & 3));
  {
    // window rows of W4 dwords (one division per lane, then carry stepping);
    // a dword wholly inside the picture row and aligned (R % 4 == 0) is one
    // load, else 4 edge-clamped byte loads
    const int W4 = (wsz + 3) >> 2, total = wsz * W4;
    int r = lane / W4, cd = lane - r * W4;
    const int dr = 64 / W4, dc = 64 - dr * W4;
    for (int k = lane; k < total; k += 64) {
      const uint8_t *rowp = ref + static_cast<int64_t>(min(max(y0 + r, 0), a.ch - 1)) * a.cw;
      const int sx = x0 + 4 * cd;
      uint32_t v;
      if (sx >= 0 && sx + 3 < a.cw && !(sx & 3)) {
        v = *reinterpret_cast<const uint32_t *>(rowp + sx);
      } else {
        v = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) v |= static_cast<uint32_t>(rowp[min(max(sx + q, 0), a.cw - 1)]) << (8 * q);
      }
      *reinterpret_cast<uint32_t *>(win + r * kWinPitch + 4 * cd) = v;
      r += dr;
      cd += dc;
      if (cd >= W4) {
        cd -= W4;
        ++r;
      }
    }
  }
  // edge-clamped chroma window (Cb|Cr pairs) covering every candidate's
  // 8.4.2.2.2 taps: origin (mx 8, my 8) - ceil(R/2), 8 + R + 2 pairs square;
  // loaded beside the luma window so the epilogue reads LDS, not HBM
  const int cwn = 8 + R + 2, cox = mx * 8 - ((R + 1) >> 1), coy = my * 8 - ((R + 1) >> 1);
  const int ccw = a.cw / 2, cch = a.ch / 2;
  const uint8_t *ruv = ref + static_cast<int64_t>(a.cw) * a.ch;
  for (int i = lane; VTS_SEARCH_UV_LDS && i < cwn * cwn; i += 64) {
    const int yy = i / cwn, xx = i - yy * cwn;
    const int sy = min(max(coy + yy, 0), cch - 1), sx = min(max(cox + xx, 0), ccw - 1);
    winuv[yy * kUvPitch + xx] = *reinterpret_cast<const uint16_t *>(ruv + static_cast<int64_t>(sy) * a.cw + 2 * sx);
  }
  __syncthreads();
  const int ncand = side * side, center = R * side + R;
  uint64_t best = ~0ull;
  if constexpr (RT > 0) {
    // Register blocking: lane (gx, gy) owns the G candidates dx = gx - R,
    // dy in [gy G, gy G + G) - R.  Each of their 16 + G - 1 window rows is
    // read from LDS once (5 dwords, 4 byte-aligns) and SAD'd against every
    // source row (held in VGPRs) it meets: ~4.6x fewer LDS reads and ~2x
    // fewer VALU instructions than one candidate per pass.
    constexpr int SIDE = 2 * RT + 1, NG = 64 / SIDE, G = (SIDE + NG - 1) / NG;
    const int gx = lane % SIDE, gy = lane / SIDE, dy0 = gy * G;
    if (gy < NG && dy0 < SIDE) {
#if !VTS_SEARCH_SRC_LDS
      uint32_t sv[64];
#pragma unroll
      for (int i = 0; i < 64; ++i) sv[i] = srcy[i];
#endif
      uint32_t acc[G];
#pragma unroll
      for (int g = 0; g < G; ++g) acc[g] = 0;
      const int sh = gx & 3;
      const uint32_t *wb = reinterpret_cast<const uint32_t *>(win + dy0 * kWinPitch + (gx & ~3));
#if VTS_SEARCH_SRC_LDS
#pragma unroll 2
#else
#pragma unroll
#endif
      for (int w = 0; w < 16 + G - 1; ++w) {
        const uint32_t *wr = wb + w * (kWinPitch / 4);
        const uint32_t w0 = wr[0], w1 = wr[1], w2 = wr[2], w3 = wr[3], w4 = wr[4];
        const uint32_t r0 = __builtin_amdgcn_alignbyte(w1, w0, sh), r1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
        const uint32_t r2 = __builtin_amdgcn_alignbyte(w3, w2, sh), r3 = __builtin_amdgcn_alignbyte(w4, w3, sh);
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const int yy = w - g;
          if (yy >= 0 && yy < 16) {
#if VTS_SEARCH_SRC_LDS
            const uint4 q = reinterpret_cast<const uint4 *>(srcy)[yy];  // broadcast read
            const uint32_t s0 = q.x, s1 = q.y, s2 = q.z, s3 = q.w;
#else
            const uint32_t s0 = sv[4 * yy], s1 = sv[4 * yy + 1], s2 = sv[4 * yy + 2], s3 = sv[4 * yy + 3];
#endif
            acc[g] = __builtin_amdgcn_sad_u8(r0, s0, acc[g]);
            acc[g] = __builtin_amdgcn_sad_u8(r1, s1, acc[g]);
            acc[g] = __builtin_amdgcn_sad_u8(r2, s2, acc[g]);
            acc[g] = __builtin_amdgcn_sad_u8(r3, s3, acc[g]);
          }
        }
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int dyi = dy0 + g;
        if (dyi < SIDE) {
          const int r = dyi * SIDE + gx;
          const int c = r == center ? 0 : (r < center ? r + 1 : r);
          const uint64_t key = (static_cast<uint64_t>(acc[g]) << 32) | static_cast<uint32_t>(c);
          best = key < best ? key : best;
        }
      }
    }
  } else {
    for (int c = lane; c < ncand; c += 64) {
      const int r = c == 0 ? center : (c - 1 < center ? c - 1 : c);
      const int dy = r / side - R, dx = r % side - R;
      uint32_t s = 0;  // the window holds edge-clamped samples: every candidate is valid
      const int ox = dx + R, sh = ox & 3;
      // per row: the 5 dwords covering the 16 candidate bytes, 4 byte-aligns,
      // the source row as one 16-byte broadcast read, 4 v_sad_u8
      const uint32_t *wr = reinterpret_cast<const uint32_t *>(win + (dy + R) * kWinPitch + (ox & ~3));
      const uint4 *sr = reinterpret_cast<const uint4 *>(srcy);
  #pragma unroll 4
      for (int yy = 0; yy < 16; ++yy) {
        const uint32_t *w = wr + yy * (kWinPitch / 4);
        const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
        const uint4 sv = sr[yy];
        s = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w1, w0, sh), sv.x, s);
        s = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w2, w1, sh), sv.y, s);
        s = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w3, w2, sh), sv.z, s);
        s = __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w4, w3, sh), sv.w, s);
      }
      const uint64_t key = (static_cast<uint64_t>(s) << 32) | static_cast<uint32_t>(c);
      best = key < best ? key : best;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t o = __shfl_xor(best, off);
    best = o < best ? o : best;
  }
  const int c = static_cast<int>(best & 0xffffffffu);
  const int r = c == 0 ? center : (c - 1 < center ? c - 1 : c);
  const int dy = r / side - R, dx = r % side - R;
  // prediction and cost: lane -> 4 luma samples (row lane/4) and one chroma pair
  const int ly = lane >> 2, lx = 4 * (lane & 3);
  const uint32_t py = u32_at(win + (dy + R + ly) * kWinPitch, dx + R + lx);
  const uint32_t sy4 = srcy[lane];
  uint32_t cost = __builtin_amdgcn_sad_u8(py, sy4, 0);
  const int ci = lane & 7, cj = lane >> 3;
  const int mvx = 4 * dx, mvy = 4 * dy, fx = mvx & 7, fy = mvy & 7;
  // window coordinates of taps (xi, yi) and (xi + 1, yi + 1); the window holds
  // the clamped samples, so this equals the decoder's per-tap clamping
#if VTS_SEARCH_UV_LDS
  const int wx = ci + (mvx >> 3) + ((R + 1) >> 1), wy = cj + (mvy >> 3) + ((R + 1) >> 1);
  const uint16_t A = winuv[wy * kUvPitch + wx], B = winuv[wy * kUvPitch + wx + 1];
  const uint16_t Cc = winuv[(wy + 1) * kUvPitch + wx], D = winuv[(wy + 1) * kUvPitch + wx + 1];
#else
  const int xi = mx * 8 + ci + (mvx >> 3), yi = my * 8 + cj + (mvy >> 3);
  const int xa = min(max(xi, 0), ccw - 1), xb = min(max(xi + 1, 0), ccw - 1);
  const int ya = min(max(yi, 0), cch - 1), yb = min(max(yi + 1, 0), cch - 1);
  const uint16_t A = *reinterpret_cast<const uint16_t *>(ruv + static_cast<int64_t>(ya) * a.cw + 2 * xa);
  const uint16_t B = *reinterpret_cast<const uint16_t *>(ruv + static_cast<int64_t>(ya) * a.cw + 2 * xb);
  const uint16_t Cc = *reinterpret_cast<const uint16_t *>(ruv + static_cast<int64_t>(yb) * a.cw + 2 * xa);
  const uint16_t D = *reinterpret_cast<const uint16_t *>(ruv + static_cast<int64_t>(yb) * a.cw + 2 * xb);
#endif
  const int wa = (8 - fx) * (8 - fy), wb = fx * (8 - fy), wc = (8 - fx) * fy, wd = fx * fy;
  const int pu = (wa * (A & 255) + wb * (B & 255) + wc * (Cc & 255) + wd * (D & 255) + 32) >> 6;
  const int pv = (wa * (A >> 8) + wb * (B >> 8) + wc * (Cc >> 8) + wd * (D >> 8) + 32) >> 6;
  const int64_t co = static_cast<int64_t>(a.cw) * a.ch + static_cast<int64_t>(my * 8 + cj) * a.cw + 2 * (mx * 8 + ci);
  const uint16_t suv = *reinterpret_cast<const uint16_t *>(src + co);
  cost += static_cast<uint32_t>(abs(pu - (suv & 255)) + abs(pv - (suv >> 8)));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) cost += __shfl_xor(cost, off);
  const int64_t lo = static_cast<int64_t>(my * 16 + ly) * a.cw + mx * 16 + lx;
  const uint32_t mvw =
      static_cast<uint32_t>(static_cast<uint16_t>(mvx)) | (static_cast<uint32_t>(static_cast<uint16_t>(mvy)) << 16);
  if (a.qp < 1 || a.max_sad < 0) {  // no residual: inter within max_sad, else I_PCM
    const bool inter = a.max_sad >= 0 && cost <= static_cast<uint32_t>(a.max_sad);
    *reinterpret_cast<uint32_t *>(dst + lo) = inter ? py : sy4;
    *reinterpret_cast<uint16_t *>(dst + co) = inter ? static_cast<uint16_t>(pu | (pv << 8)) : suv;
    if (lane == 0) {
      a.cmd[e * a.nmb + mb] = inter ? mvw : kPcmCmd;
      if (a.cbp) a.cbp[e * a.nmb + mb] = 0;
    }
    return;
  }
  // ---- residual coding: lanes 0..15 the luma blocks (luma4x4BlkIdx), 16..23
  // the chroma blocks (Cb 0..3, Cr 0..3), 24 / 25 the chroma DC blocks
  __shared__ uint32_t predy[64], recy[64];
  __shared__ uint16_t predc[64], srcc[64];
  __shared__ uint8_t recc[2][64];
  __shared__ int dcw[2][4], dcl[2][4];
  predy[lane] = py;
  predc[lane] = static_cast<uint16_t>(pu | (pv << 8));
  srcc[lane] = suv;
  __syncthreads();
  const int qp = a.qp, qpc = kQpcTab[qp];
  const int qbits = 15 + qp / 6, cqb = 15 + qpc / 6;
  const int64_t f = (int64_t(1) << qbits) / 6, cf = (int64_t(1) << cqb) / 6;
  int lv[16], z[16], nzb = 0, bits = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) lv[i] = z[i] = 0;
  if (lane < 16) {
    const int bx = kBlkXd[lane], by = kBlkYd[lane];
    int x[16], w[16];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t sv = srcy[(by * 4 + r) * 4 + bx], pv4 = predy[(by * 4 + r) * 4 + bx];
#pragma unroll
      for (int c = 0; c < 4; ++c) x[r * 4 + c] = static_cast<int>((sv >> (8 * c)) & 255) - static_cast<int>((pv4 >> (8 * c)) & 255);
    }
    fwd4(x, w);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      z[q] = quant1(w[q], kMf[qp % 6][pos_class(q >> 2, q & 3)], qbits, f);
      nzb |= z[q] != 0;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) lv[q] = z[kZz4[q]];
    int res[16];
    full::scale_idct4(z, qp, false, res);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t pv4 = predy[(by * 4 + r) * 4 + bx];
      uint32_t o = 0;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        o |= static_cast<uint32_t>(min(max(static_cast<int>((pv4 >> (8 * c)) & 255) + res[r * 4 + c], 0), 255)) << (8 * c);
      recy[(by * 4 + r) * 4 + bx] = o;
    }
    bits = cavlc_block<false>(nullptr, lv, 16, -2);
  } else if (lane < 24) {
    const int pl = (lane - 16) >> 2, k = (lane - 16) & 3, bx = (k & 1) * 4, by = (k >> 1) * 4;
    int x[16], w[16];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int i = (by + r) * 8 + bx + c;
        x[r * 4 + c] = static_cast<int>((srcc[i] >> (8 * pl)) & 255) - static_cast<int>((predc[i] >> (8 * pl)) & 255);
      }
    fwd4(x, w);
    dcw[pl][k] = w[0];
#pragma unroll
    for (int q = 1; q < 16; ++q) {
      z[q] = quant1(w[q], kMf[qpc % 6][pos_class(q >> 2, q & 3)], cqb, cf);
      nzb |= z[q] != 0;
    }
#pragma unroll
    for (int q = 1; q < 16; ++q) lv[q - 1] = z[kZz4[q]];
  }
  __syncthreads();
  if (lane == 16 || lane == 17) {  // chroma DC: 2x2 Hadamard, quantised at (qbits + 1, 2f)
    const int pl = lane - 16;
    const int c0 = dcw[pl][0], c1 = dcw[pl][1], c2 = dcw[pl][2], c3 = dcw[pl][3];
    const int fd[4] = {c0 + c1 + c2 + c3, c0 - c1 + c2 - c3, c0 + c1 - c2 - c3, c0 - c1 - c2 + c3};
#pragma unroll
    for (int k = 0; k < 4; ++k) dcl[pl][k] = quant1(fd[k], kMf[qpc % 6][0], cqb + 1, 2 * cf);
  }
  __syncthreads();
  const uint64_t nzm = __ballot(nzb);
  int cbp = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if ((nzm >> (4 * q)) & 15u) cbp |= 1 << q;
  bool dcnz = false;
#pragma unroll
  for (int k = 0; k < 8; ++k) dcnz |= dcl[k >> 2][k & 3] != 0;
  const int cc = ((nzm >> 16) & 0xffu) ? 2 : (dcnz ? 1 : 0);
  cbp |= cc << 4;
  int contrib = 0;  // this lane's share of the residual's CAVLC bound
  if (lane < 16) {
    contrib = ((cbp >> (lane >> 2)) & 1) ? bits : 0;
  } else if (lane < 24) {
    contrib = cc == 2 ? cavlc_block<false>(nullptr, lv, 15, -2) : 0;
  } else if (lane < 26 && cc) {
    const int d4[4] = {dcl[lane - 24][0], dcl[lane - 24][1], dcl[lane - 24][2], dcl[lane - 24][3]};
    contrib = cavlc_block<false>(nullptr, d4, 4, -1);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) contrib += __shfl_xor(contrib, off);
  const bool inter = contrib <= kPcmBits;
  if (lane >= 16 && lane < 24) {  // chroma reconstruction (8.5.11 DC, then 8.5.12)
    const int pl = (lane - 16) >> 2, k = (lane - 16) & 3, bx = (k & 1) * 4, by = (k >> 1) * 4;
    const int *c = dcl[pl];
    const int F = k == 0 ? c[0] + c[1] + c[2] + c[3]
                         : (k == 1 ? c[0] - c[1] + c[2] - c[3] : (k == 2 ? c[0] + c[1] - c[2] - c[3] : c[0] - c[1] - c[2] + c[3]));
    int co[16], res[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) co[q] = cc == 2 ? z[q] : 0;
    co[0] = ((F * full::level_scale(qpc % 6, 0, 0)) << (qpc / 6)) >> 5;
    full::scale_idct4(co, qpc, true, res);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int cx = 0; cx < 4; ++cx) {
        const int i = (by + r) * 8 + bx + cx;
        recc[pl][i] = static_cast<uint8_t>(min(max(static_cast<int>((predc[i] >> (8 * pl)) & 255) + res[r * 4 + cx], 0), 255));
      }
  }
  __syncthreads();
  *reinterpret_cast<uint32_t *>(dst + lo) = inter ? recy[lane] : sy4;
  *reinterpret_cast<uint16_t *>(dst + co) =
      inter ? static_cast<uint16_t>(recc[0][lane] | (recc[1][lane] << 8)) : suv;
  if (inter && cbp) {  // the levels the slice writer codes
    int16_t *cp = a.coef + (e * a.nmb + mb) * kCoefPerMb;
    if (lane < 16) {
#pragma unroll
      for (int q = 0; q < 16; ++q) cp[16 * lane + q] = static_cast<int16_t>(lv[q]);
    } else if (lane < 24) {
#pragma unroll
      for (int q = 0; q < 15; ++q) cp[264 + 15 * (lane - 16) + q] = static_cast<int16_t>(lv[q]);
    } else if (lane < 26) {
#pragma unroll
      for (int q = 0; q < 4; ++q) cp[256 + 4 * (lane - 24) + q] = static_cast<int16_t>(dcl[lane - 24][q]);
    }
  }
  if (lane == 0) {
    a.cmd[e * a.nmb + mb] = inter ? mvw : kPcmCmd;
    a.cbp[e * a.nmb + mb] = static_cast<uint8_t>(inter ? cbp : 0);
  }
}

// ------------------------------------------------------ slice writer
struct WriteArgs {
  const int4 *ent;      // per frame of the level: (frame, GOP position j, IDR parity, index within its level)
  const uint32_t *cmd;  // [entry][mb] (P levels)
  const uint8_t *cbp;   // [entry][mb] coded_block_pattern
  const int16_t *coef;  // level ring: [ring slot][index within level][mb][kCoefPerMb]
  int64_t coef_per_level;  // entries a ring slot holds
  int32_t ring, qp;     // ring slots (levels); qp >= 1: residual coding (slice_qp_delta = qp - 26)
  const uint8_t *small;
  int64_t stride;
  int32_t cw, ch, mbw, mbh;
  uint8_t *staging;     // [slice][cap]
  int64_t cap;
  int32_t *sizes;       // [slice] bytes incl. the 4-byte length prefix
  unsigned long long *stats;  // pcm, inter, skip
  uint32_t *err;
  uint4 *jobs;          // I_PCM payloads left for enc_pcm: (slice, byte offset in the slot, mx, 0)
  uint32_t *n_jobs;
  int32_t n_slices;
  int32_t _pad;
};

// RBSP bits -> EBSP bytes (emulation prevention) into a staging slot, four
// bytes per (aligned) dword store.
struct NalOut {
  uint32_t *w;          // slot payload (slot + 4), 4-byte aligned
  int64_t cap, n;       // bytes
  uint32_t cur;         // the bytes of the word being filled
  uint64_t acc;
  int nacc, zeros;
  bool over;
  __device__ void put(uint32_t b) {
    cur |= b << (8 * (n & 3));
    if (!(++n & 3)) {
      if (n <= cap) w[(n >> 2) - 1] = cur;
      else over = true;
      cur = 0;
    }
  }
  __device__ void flush() {  // the partial word (its tail bytes are don't-care)
    if (n & 3) {
      if (n <= cap) w[n >> 2] = cur;
      else over = true;
    }
  }
  __device__ void byte(uint32_t b) {
    if (zeros >= 2 && b <= 3) {
      put(3);
      zeros = 0;
    }
    put(b);
    zeros = b ? 0 : zeros + 1;
  }
  __device__ void bits(int k, uint32_t v) {  // k <= 32
    acc = (acc << k) | v;
    nacc += k;
    while (nacc >= 8) {
      nacc -= 8;
      byte(static_cast<uint32_t>(acc >> nacc) & 0xffu);
    }
  }
  __device__ void ue(uint32_t v) {
    const uint32_t x = v + 1;
    const int len = 31 - __builtin_clz(x);
    if (len) bits(len, 0);
    bits(len + 1, x);
  }
  __device__ void se(int v) { ue(v > 0 ? static_cast<uint32_t>(2 * v - 1) : static_cast<uint32_t>(-2 * v)); }
  __device__ void align() {
    if (nacc) bits(8 - nacc, 0);
  }
};

template <bool kWrite>
__device__ int cavlc_block(NalOut *o, const int *lv, int maxNum, int nC) {
  int tc = 0, t1 = 0, top = -1;
  bool open = true;
#pragma unroll
  for (int i = 15; i >= 0; --i) {
    const int v = i < maxNum ? lv[i] : 0;
    if (!v) continue;
    if (top < 0) top = i;
    ++tc;
    if (open && t1 < 3 && (v == 1 || v == -1)) ++t1;
    else open = false;
  }
  int bits;
  if (nC < -1) {  // the bound: the longest coeff_token over nC classes 0..2 and the FLC
    bits = max(6, max(static_cast<int>(kCtLen[0][tc][t1]), max(static_cast<int>(kCtLen[1][tc][t1]),
                                                              static_cast<int>(kCtLen[2][tc][t1]))));
  } else if (nC >= 8) {
    bits = 6;
    if (kWrite) o->bits(6, tc == 0 ? 3u : static_cast<uint32_t>(((tc - 1) << 2) | t1));
  } else {
    const int col = nC == -1 ? 3 : (nC < 2 ? 0 : (nC < 4 ? 1 : 2));
    bits = kCtLen[col][tc][t1];
    if (kWrite) o->bits(bits, kCtCode[col][tc][t1]);
  }
  if (tc == 0) return bits;
  int k = 0, sl = (tc > 10 && t1 < 3) ? 1 : 0;
#pragma unroll
  for (int i = 15; i >= 0; --i) {  // trailing ones' signs, then levels (9.2.2.1 inverted)
    const int v = i < maxNum ? lv[i] : 0;
    if (!v) continue;
    if (k < t1) {
      ++bits;
      if (kWrite) o->bits(1, v < 0 ? 1u : 0u);
    } else {
      int code = v > 0 ? 2 * v - 2 : -2 * v - 1;
      if (k == t1 && t1 < 3) code -= 2;
      int prefix, suffix = 0, ssize = 0;
      if (sl == 0) {
        if (code < 14) prefix = code;
        else if (code < 30) { prefix = 14; suffix = code - 14; ssize = 4; }
        else { prefix = 15; suffix = code - 30; ssize = 12; }
      } else if (code < (15 << sl)) {
        prefix = code >> sl;
        suffix = code & ((1 << sl) - 1);
        ssize = sl;
      } else {
        prefix = 15;
        suffix = code - (15 << sl);
        ssize = 12;
      }
      bits += prefix + 1 + ssize;
      if (kWrite) {
        o->bits(prefix + 1, 1u);
        if (ssize) o->bits(ssize, static_cast<uint32_t>(suffix));
      }
      if (sl == 0) sl = 1;
      if (abs(v) > (3 << (sl - 1)) && sl < 6) ++sl;
    }
    ++k;
  }
  int zl = top + 1 - tc;  // total_zeros
  if (tc < maxNum) {
    const int len = maxNum == 4 ? kTzcLen[tc - 1][zl] : kTzLen[tc - 1][zl];
    bits += len;
    if (kWrite) o->bits(len, maxNum == 4 ? kTzcCode[tc - 1][zl] : kTzCode[tc - 1][zl]);
  }
  int prev = -1;
#pragma unroll
  for (int i = 15; i >= 0; --i) {  // run_before of every coefficient but the lowest
    const int v = i < maxNum ? lv[i] : 0;
    if (!v) continue;
    if (prev >= 0 && zl > 0) {
      const int run = prev - i - 1, row = min(zl, 7) - 1;
      bits += kRbLen[row][run];
      if (kWrite) o->bits(kRbLen[row][run], kRbCode[row][run]);
      zl -= run;
    }
    prev = i;
  }
  return bits;
}

// residual() of an inter macroblock (7.3.5.3): cp the levels, cnz / cnzc
// receive the blocks' total_coeff; lnz / lnzc the left macroblock's right
// column (-1: unavailable; the macroblock above is another slice)
__device__ void put_residual(NalOut &o, const int16_t *cp, int cbp, const int *lnz, const int (*lnzc)[2], int *cnz,
                             int (*cnzc)[4]) {
  for (int i = 0; i < 16; ++i) cnz[i] = 0;
  for (int i = 0; i < 4; ++i) cnzc[0][i] = cnzc[1][i] = 0;
  int lv[16];
  for (int k = 0; k < 16; ++k) {
    if (!((cbp >> (k >> 2)) & 1)) continue;
    const int bx = kBlkXd[k], by = kBlkYd[k];
    const int na = bx ? cnz[by * 4 + bx - 1] : lnz[by], nb = by ? cnz[(by - 1) * 4 + bx] : -1;
    const int nC = (na >= 0 && nb >= 0) ? (na + nb + 1) >> 1 : (na >= 0 ? na : (nb >= 0 ? nb : 0));
    int tc = 0;
    for (int q = 0; q < 16; ++q) {
      lv[q] = cp[16 * k + q];
      tc += lv[q] != 0;
    }
    cavlc_block<true>(&o, lv, 16, nC);
    cnz[by * 4 + bx] = tc;
  }
  if (cbp >> 4)
    for (int pl = 0; pl < 2; ++pl) {
      for (int q = 0; q < 4; ++q) lv[q] = cp[256 + 4 * pl + q];
      cavlc_block<true>(&o, lv, 4, -1);
    }
  if ((cbp >> 4) == 2)
    for (int pl = 0; pl < 2; ++pl)
      for (int k = 0; k < 4; ++k) {
        const int bx = k & 1, by = k >> 1;
        const int na = bx ? cnzc[pl][by * 2] : lnzc[pl][by], nb = by ? cnzc[pl][bx] : -1;
        const int nC = (na >= 0 && nb >= 0) ? (na + nb + 1) >> 1 : (na >= 0 ? na : (nb >= 0 ? nb : 0));
        int tc = 0;
        for (int q = 0; q < 15; ++q) {
          lv[q] = cp[264 + 60 * pl + 15 * k + q];
          tc += lv[q] != 0;
        }
        cavlc_block<true>(&o, lv, 15, nC);
        cnzc[pl][k] = tc;
      }
}

// I_PCM: pcm_alignment_zero_bits, then 384 sample bytes that enc_pcm fills in
// later (the gap's bytes in the partial words either side are don't-care
// here: enc_pcm runs after enc_gather).  The samples are >= 1 (downscale
// clamp), and the byte before them holds mb_type's last 1 bits, so no
// emulation prevention byte can fall in or next to them and the zero-run
// state after them is 0.
__device__ void pcm_gap(NalOut &o, uint4 *job, int s, int mx) {
  o.align();
  o.flush();
  *job = make_uint4(static_cast<uint32_t>(s), static_cast<uint32_t>(4 + o.n), static_cast<uint32_t>(mx), 0);
  o.n += 384;  // a multiple of 4: the word phase is unchanged
  o.cur = 0;
  if (o.n > o.cap) o.over = true;
  o.zeros = 0;
}

__global__ void __launch_bounds__(64) enc_write(WriteArgs a) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.n_slices) return;
  const int e = s / a.mbh, row = s % a.mbh;
  const int4 en = a.ent[e];
  const bool idr = en.y == 0;  // GOP position 0
  uint8_t *slot = a.staging + static_cast<int64_t>(s) * a.cap;
  NalOut o{reinterpret_cast<uint32_t *>(slot + 4), a.cap - 4, 0, 0, 0, 0, 0, false};
  o.put(idr ? 0x65 : 0x41);  // nal_ref_idc 3 IDR / 2 non-IDR; every picture is a reference
  o.ue(static_cast<uint32_t>(row * a.mbw));  // first_mb_in_slice
  o.ue(idr ? 7 : 5);                       // slice_type I / P (all slices of the picture)
  o.ue(0);                                   // pic_parameter_set_id
  o.bits(16, static_cast<uint32_t>(en.y) & 0xffffu);  // frame_num (16 bits)
  if (idr) {
    o.ue(static_cast<uint32_t>(en.z));       // idr_pic_id
    o.bits(2, 0);                            // no_output_of_prior_pics, long_term_reference
  } else {
    o.bits(3, 0);  // num_ref_idx_active_override, ref_pic_list_modification_l0, adaptive_ref_pic_marking
  }
  o.se(a.qp >= 1 ? a.qp - 26 : 0);  // slice_qp_delta: SliceQPY = the residual's QP (pic_init_qp 26)
  o.ue(1);  // disable_deblocking_filter_idc
  unsigned long long npcm = 0, ninter = 0, nskip = 0;
  uint32_t skip = 0;
  bool a_ok = false;
  int amx = 0, amy = 0;
  const uint32_t *cmd = a.cmd + static_cast<int64_t>(e) * a.mbw * a.mbh + static_cast<int64_t>(row) * a.mbw;
  const uint8_t *cbpr = a.cbp + static_cast<int64_t>(e) * a.mbw * a.mbh + static_cast<int64_t>(row) * a.mbw;
  const int16_t *coef_row =
      a.coef + ((static_cast<int64_t>(en.y % a.ring) * a.coef_per_level + en.w) * a.mbh + row) * a.mbw * kCoefPerMb;
  // total_coeff of the left macroblock's right column for nC (9.2.1); -1 none
  int lnz[4] = {-1, -1, -1, -1}, lnzc[2][2] = {{-1, -1}, {-1, -1}}, cnz[16], cnzc[2][4];
  // reserve this slice's I_PCM jobs
  uint32_t njob = 0;
  if (idr) {
    njob = static_cast<uint32_t>(a.mbw);
  } else {
    for (int mx = 0; mx < a.mbw; ++mx) njob += cmd[mx] == kPcmCmd;
  }
  uint4 *job = a.jobs + (njob ? atomicAdd(a.n_jobs, njob) : 0u);
  for (int mx = 0; mx < a.mbw; ++mx) {
    if (idr) {
      o.ue(25);
      pcm_gap(o, job++, s, mx);
      ++npcm;
      continue;
    }
    const uint32_t c = cmd[mx];
    if (c == kPcmCmd) {
      o.ue(skip);
      skip = 0;
      o.ue(30);  // I_PCM in a P slice
      pcm_gap(o, job++, s, mx);
      a_ok = false;
      ++npcm;
      for (int i = 0; i < 4; ++i) lnz[i] = 16;
      lnzc[0][0] = lnzc[0][1] = lnzc[1][0] = lnzc[1][1] = 16;
      continue;
    }
    const int mvx = static_cast<int16_t>(c & 0xffffu), mvy = static_cast<int16_t>(c >> 16);
    const int cbp = cbpr[mx];
    if (mvx == 0 && mvy == 0 && cbp == 0) {  // P_Skip (neighbour B lies in another slice: skip motion is 0)
      ++skip;
      ++nskip;
      for (int i = 0; i < 4; ++i) lnz[i] = 0;
      lnzc[0][0] = lnzc[0][1] = lnzc[1][0] = lnzc[1][1] = 0;
    } else {
      const int px = a_ok ? amx : 0, py = a_ok ? amy : 0;  // 8.4.1.3, A the only neighbour
      o.ue(skip);
      skip = 0;
      o.ue(0);  // P_L0_16x16
      o.se(mvx - px);
      o.se(mvy - py);
      int code = 0;
      while (kCbpInterTab[code] != cbp) ++code;
      o.ue(static_cast<uint32_t>(code));  // coded_block_pattern me(v)
      if (cbp) {
        o.se(0);  // mb_qp_delta
        put_residual(o, coef_row + static_cast<int64_t>(mx) * kCoefPerMb, cbp, lnz, lnzc, cnz, cnzc);
      } else {
        for (int i = 0; i < 16; ++i) cnz[i] = 0;
        for (int i = 0; i < 4; ++i) cnzc[0][i] = cnzc[1][i] = 0;
      }
      for (int i = 0; i < 4; ++i) lnz[i] = cnz[i * 4 + 3];
      for (int pl = 0; pl < 2; ++pl) {
        lnzc[pl][0] = cnzc[pl][1];
        lnzc[pl][1] = cnzc[pl][3];
      }
      ++ninter;
    }
    a_ok = true;
    amx = mvx;
    amy = mvy;
  }
  if (skip) o.ue(skip);
  o.bits(1, 1);  // rbsp_stop_one_bit
  o.align();
  o.flush();
  const int64_t len = o.n;
  if (o.over) {
    atomicOr(a.err, 1u);
    a.sizes[s] = 0;
    return;
  }
  *reinterpret_cast<uint32_t *>(slot) = __builtin_bswap32(static_cast<uint32_t>(len));  // big-endian length
  a.sizes[s] = static_cast<int32_t>(len + 4);
  atomicAdd(&a.stats[0], npcm);
  atomicAdd(&a.stats[1], ninter);
  atomicAdd(&a.stats[2], nskip);
}

// Slice offsets of one level on the device: offs[s] = running output total +
// exclusive scan of the slice sizes (one 1024-thread workgroup), each frame's
// (offset, size), and the running total advanced.  No host round trip.
__global__ void __launch_bounds__(1024) enc_scan(const int32_t *sizes, int ns, const int4 *ent, int mbh,
                                                 int64_t *offs, int64_t *total, int64_t *fr_off,
                                                 int64_t *fr_size) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x;
  const int per = (ns + 1023) / 1024;
  const int b0 = min(ns, t * per), b1 = min(ns, b0 + per);
  const int64_t base = *total;
  int64_t sum = 0;
  for (int i = b0; i < b1; ++i) sum += sizes[i];
  part[t] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {  // inclusive scan of the partial sums
    const int64_t v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int64_t run = base + part[t] - sum;
  for (int i = b0; i < b1; ++i) {
    offs[i] = run;
    run += sizes[i];
  }
  __syncthreads();
  const int64_t end = base + part[1023];
  const int ne = ns / mbh;
  for (int e = t; e < ne; e += 1024) {
    const int64_t o = offs[static_cast<int64_t>(e) * mbh];
    fr_off[ent[e].x] = o;
    fr_size[ent[e].x] = (e + 1 < ne ? offs[static_cast<int64_t>(e + 1) * mbh] : end) - o;
  }
  if (t == 0) *total = end;
}

// one workgroup per slice: staging slot -> the chunk arena (offsets are
// absolute; the arena starts at *base)
__global__ void __launch_bounds__(256) enc_gather(const uint8_t *staging, int64_t cap, const int32_t *sizes,
                                                  const int64_t *offs, const int64_t *base, uint8_t *out) {
  const int s = blockIdx.x;
  const uint8_t *p = staging + static_cast<int64_t>(s) * cap;
  uint8_t *q = out + (offs[s] - *base);
  const int n = sizes[s];
  for (int i = threadIdx.x; i < n; i += 256) q[i] = p[i];
}

// I_PCM payloads: one wave per job, 6 bytes per lane, straight into the
// packed level output (after enc_gather): luma 16x16, then Cb 8x8, Cr 8x8
// (7.3.5) from the NV12 source.
__global__ void __launch_bounds__(64) enc_pcm(const uint4 *jobs, const uint32_t *n_jobs, const int4 *ent,
                                              const uint8_t *small, int64_t stride, int32_t cw, int32_t ch,
                                              int32_t mbh, const int64_t *offs, const int64_t *base,
                                              uint8_t *out) {
  const uint32_t n = *n_jobs;
  const int64_t b = *base;
  for (uint32_t j = blockIdx.x; j < n; j += gridDim.x) {
    const uint4 jb = jobs[j];
    const int s = static_cast<int>(jb.x), mx = static_cast<int>(jb.z);
    const int e = s / mbh, my = s % mbh;
    const uint8_t *src = small + static_cast<int64_t>(ent[e].x) * stride;
    const uint8_t *uv = src + static_cast<int64_t>(cw) * ch;
    uint8_t *dst = out + (offs[s] - b) + jb.y;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const int b = 6 * static_cast<int>(threadIdx.x) + q;
      uint8_t v;
      if (b < 256) {
        v = src[static_cast<int64_t>(my * 16 + (b >> 4)) * cw + mx * 16 + (b & 15)];
      } else {
        const int i = (b - 256) & 63, pl = (b - 256) >> 6;
        v = uv[static_cast<int64_t>(my * 8 + (i >> 3)) * cw + 2 * (mx * 8 + (i & 7)) + pl];
      }
      dst[b] = v;
    }
  }
}

// ------------------------------------------------------------ host
int64_t gcd64(int64_t a, int64_t b) {
  while (b) {
    const int64_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}

// tap table for n source -> m destination samples over `coded` outputs
std::vector<int32_t> area_taps(int64_t n, int64_t m, int coded, int *k_out, int32_t *t_out) {
  const int64_t g = gcd64(n, m);
  int k = 1;
  for (int64_t o = 0; o < m; ++o) {
    const int64_t i0 = o * n / m, i1 = ((o + 1) * n + m - 1) / m;
    k = std::max<int>(k, static_cast<int>(i1 - i0));
  }
  std::vector<int32_t> t(static_cast<size_t>(coded) * (1 + k), 0);
  for (int x = 0; x < coded; ++x) {
    const int64_t o = std::min<int64_t>(x, m - 1);
    const int64_t i0 = o * n / m;
    int32_t *e = &t[static_cast<size_t>(x) * (1 + k)];
    e[0] = static_cast<int32_t>(i0);
    for (int i = 0; i < k; ++i) {
      const int64_t si = i0 + i;
      const int64_t lo = std::max(o * n, si * m), hi = std::min((o + 1) * n, (si + 1) * m);
      e[1 + i] = (si < n && hi > lo) ? static_cast<int32_t>((hi - lo) / g) : 0;
    }
  }
  *k_out = k;
  *t_out = static_cast<int32_t>(n / g);
  return t;
}

template <class T>
int dev_alloc(T **p, size_t n) {
  HIP_TRY(vts::dmalloc(reinterpret_cast<void **>(p), std::max<size_t>(1, n) * sizeof(T)));
  return VTS_OK;
}

// Transcode scratch, freed on every exit path.  vts::dfree hands a range
// straight back to the process-wide cache (no implicit device synchronisation
// as with hipFree), so the streams whose kernels may still use the buffers
// are drained first: an early return after the searches were queued must not
// let a later allocation reuse memory those kernels still write.
struct DevBufs {
  std::vector<void *> ptrs;
  std::vector<hipStream_t> streams;  // synchronised before anything is freed
  template <class T>
  int get(T **p, size_t n) {
    VTS_TRY(dev_alloc(p, n));
    ptrs.push_back(*p);
    return VTS_OK;
  }
  ~DevBufs() {
    for (hipStream_t s : streams) (void)hipStreamSynchronize(s);
    for (void *p : ptrs) vts::dfree(p);
  }
};

int setup_small(vts_ctx *c, int sh) {
  SmallStore &S = c->small;
  const int W = c->width, H = c->height;
  const int sw = static_cast<int>((static_cast<int64_t>(sh) * W + H) / (2 * static_cast<int64_t>(H))) * 2;
  if (sw < 2) return fail(VTS_E_INVALID, "output width %d from %dx%d at height %d", sw, W, H, sh);
  if (S.d && S.w == sw && S.h == sh) return VTS_OK;
  if (S.d) vts::dfree(S.d);
  if (S.d_taps) vts::dfree(S.d_taps);
  S = SmallStore{};
  S.w = sw;
  S.h = sh;
  S.cw = (sw + 15) & ~15;
  S.ch = (sh + 15) & ~15;
  S.stride = (static_cast<int64_t>(S.cw) * S.ch * 3 / 2 + 255) & ~int64_t(255);
  int32_t tl_x, tl_y, tc_x, tc_y;
  const auto tx = area_taps(W, sw, S.cw, &S.taps_x, &tl_x);
  const auto ty = area_taps(H, sh, S.ch, &S.taps_y, &tl_y);
  const auto tcx = area_taps(W / 2, sw / 2, S.cw / 2, &S.taps_cx, &tc_x);
  const auto tcy = area_taps(H / 2, sh / 2, S.ch / 2, &S.taps_cy, &tc_y);
  if (std::max({S.taps_x, S.taps_y, S.taps_cx, S.taps_cy}) > kMaxTaps)
    return fail(VTS_E_UNSUPPORTED, "downscale ratio %dx%d -> %dx%d needs more than %d taps", W, H, sw, sh,
                kMaxTaps);
  if (static_cast<int64_t>(tl_x) * tl_y * 255 > 0x7fffffffll || static_cast<int64_t>(tc_x) * tc_y * 255 > 0x7fffffffll)
    return fail(VTS_E_UNSUPPORTED, "downscale ratio %dx%d -> %dx%d overflows 32-bit sums", W, H, sw, sh);
  S.tl = tl_x * tl_y;
  S.tc = tc_x * tc_y;
  std::vector<int32_t> all;
  S.off[0] = 0;
  for (const auto *v : {&tx, &ty, &tcx, &tcy}) {
    all.insert(all.end(), v->begin(), v->end());
  }
  S.off[1] = static_cast<int64_t>(tx.size());
  S.off[2] = S.off[1] + static_cast<int64_t>(ty.size());
  S.off[3] = S.off[2] + static_cast<int64_t>(tcx.size());
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(vts::dmalloc(&S.d_taps, all.size() * sizeof(int32_t)));
  HIP_TRY(hipMemcpy(S.d_taps, all.data(), all.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  const size_t bytes = static_cast<size_t>(S.stride * c->n_frames + 256);
  if (vts::dmalloc(&S.d, bytes) != hipSuccess) {
    (void)hipGetLastError();
    S.d = nullptr;
    return fail(VTS_E_HIP, "cannot allocate %.1f GiB for the %dx%d frames", bytes / 1073741824.0, sw, sh);
  }
  return VTS_OK;
}

}  // namespace

int small_window(vts_ctx *c, int ring, int64_t f0, int64_t f1, hipStream_t s) {
  const SmallStore &S = c->small;
  DsArgs a{};
  a.src = c->d_surf[ring];
  a.src_stride = c->frame_stride;
  a.pitch = c->pitch;
  a.uv_rows = c->coded_h;
  a.sw = c->width;
  a.sh = c->height;
  a.dst = S.d + f0 * S.stride;
  a.dst_stride = S.stride;
  a.cw = S.cw;
  a.ch = S.ch;
  a.tx = S.d_taps + S.off[0];
  a.ty = S.d_taps + S.off[1];
  a.tcx = S.d_taps + S.off[2];
  a.tcy = S.d_taps + S.off[3];
  a.kx = S.taps_x;
  a.ky = S.taps_y;
  a.kcx = S.taps_cx;
  a.kcy = S.taps_cy;
  a.tl = S.tl;
  a.tc = S.tc;
  a.n_frames = f1 - f0;
  const int64_t threads = static_cast<int64_t>(S.cw / 4) * (S.ch + S.ch / 2);
  // integer ratio on both axes (equal): the dword box path; else the tap tables
  const int W = c->width, H = c->height;
  const int k = (W % S.w == 0 && H % S.h == 0 && W / S.w == H / S.h) ? W / S.w : 0;
  for (int64_t g0 = 0; g0 < f1 - f0; g0 += 65535) {  // grid.y <= 65535 frames per launch
    DsArgs b = a;
    b.src = a.src + g0 * a.src_stride;
    b.dst = a.dst + g0 * a.dst_stride;
    b.n_frames = std::min<int64_t>(65535, f1 - f0 - g0);
    const dim3 grid(static_cast<unsigned>((threads + 255) / 256), static_cast<unsigned>(b.n_frames));
    switch (k) {
      case 2: hipLaunchKernelGGL(downscale_nv12<2>, grid, dim3(256), 0, s, b); break;
      case 3: hipLaunchKernelGGL(downscale_nv12<3>, grid, dim3(256), 0, s, b); break;
      case 4: hipLaunchKernelGGL(downscale_nv12<4>, grid, dim3(256), 0, s, b); break;
      default: hipLaunchKernelGGL(downscale_nv12<0>, grid, dim3(256), 0, s, b); break;
    }
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(VTS_E_HIP, "downscale_nv12 launch: %s", hipGetErrorString(e));
  return VTS_OK;
}

}  // namespace vts

using namespace vts;

extern "C" int vts_transcode(vts_ctx *c, const char *out_path, const vts_transcode_params *pin,
                             vts_transcode_info *info) {
  clear_error();
  if (!c || !out_path) return fail(VTS_E_INVALID, "NULL argument");
  using clk = std::chrono::steady_clock;
  vts_transcode_params p{};
  if (pin) p = *pin;
  const int sh = p.height > 0 ? p.height : 360;
  const int R = p.search_range == 0 ? 8 : std::max(0, p.search_range);
  const int T = p.max_mb_sad == 0 ? 1536 : p.max_mb_sad;
  const int qp = p.qp == 0 ? 28 : (p.qp < 0 ? 0 : p.qp);  // 0: no residual coding (the round-2 encoder)
  if (qp > 51) return fail(VTS_E_INVALID, "qp %d > 51", qp);
  const int keyint = p.keyint > 0 ? p.keyint : 250;
  const float thr = p.cut_threshold > 0 ? p.cut_threshold : c->params.cut_threshold;
  if ((sh & 1) || sh < 16 || sh > c->height)
    return fail(VTS_E_INVALID, "output height %d: even, 16 .. source height %d", sh, c->height);
  if (R > kMaxRange) return fail(VTS_E_INVALID, "search_range %d > %d", R, kMaxRange);
  // constant frame rate (the writer's stts is one entry)
  const int64_t n = c->n_frames;
  int64_t delta = n > 1 ? c->pts[1] - c->pts[0] : std::max<int64_t>(1, c->info.track_timescale / 30);
  for (int64_t i = 1; i < n; ++i)
    if (c->pts[i] - c->pts[i - 1] != delta)
      return fail(VTS_E_UNSUPPORTED, "variable frame rate (frame %lld) is not transcoded",
                  static_cast<long long>(i));
  HIP_TRY(hipSetDevice(c->device));
  VTS_TRY(setup_small(c, sh));
  const SmallStore &S = c->small;
  const int mbw = S.cw / 16, mbh = S.ch / 16, nmb = mbw * mbh;
  double ms[4] = {0, 0, 0, 0};

  // 1. decode + score + downscale
  auto t0 = clk::now();
  c->small.on = true;
  const int rc = run_all(c);
  c->small.on = false;
  VTS_TRY(rc);
  VTS_TRY(fetch_scores(c));
  ms[0] = std::chrono::duration<double, std::milli>(clk::now() - t0).count();

  // 2. GOPs: IDR at frame 0, at cuts, every keyint frames
  std::vector<int64_t> gop_start;
  for (int64_t f = 0; f < n; ++f)
    if (f == 0 || (p.idr_at_cuts && c->host_scores[f] > thr) || f - gop_start.back() >= keyint)
      gop_start.push_back(f);
  const int64_t ngop = static_cast<int64_t>(gop_start.size());
  std::vector<int64_t> gop_len(static_cast<size_t>(ngop));
  int64_t maxlen = 0;
  for (int64_t g = 0; g < ngop; ++g) {
    gop_len[g] = (g + 1 < ngop ? gop_start[g + 1] : n) - gop_start[g];
    maxlen = std::max(maxlen, gop_len[g]);
  }
  // per level j: search entries (frame, ref slot, dst slot) and write entries (frame, j, idr parity)
  std::vector<int4> sent, went;
  std::vector<int64_t> lvl_off(static_cast<size_t>(maxlen) + 1, 0);
  for (int64_t j = 0; j < maxlen; ++j) {
    lvl_off[j] = static_cast<int64_t>(went.size());
    for (int64_t g = 0; g < ngop; ++g) {
      if (gop_len[g] <= j) continue;
      const int f = static_cast<int>(gop_start[g] + j);
      sent.push_back(make_int4(f, j == 1 ? -1 : static_cast<int>(2 * g + ((j - 1) & 1)), static_cast<int>(2 * g + (j & 1)), 0));
      went.push_back(make_int4(f, static_cast<int>(j), static_cast<int>(g & 1),
                               static_cast<int>(static_cast<int64_t>(went.size()) - lvl_off[j])));
    }
  }
  lvl_off[maxlen] = static_cast<int64_t>(went.size());

  // 3. device encode, level by level
  // staging slot per slice: an I_PCM macroblock is < 400 bytes, and so is an
  // inter one (its residual is coded only under a 3072-bit bound); the rest
  // is headroom for emulation prevention bytes in residual data
  const int64_t cap = ((64 + static_cast<int64_t>(mbw) * 600) + 255) & ~int64_t(255);
  DevBufs B;
  int4 *d_sent, *d_went;
  uint8_t *d_recon, *d_stage, *d_out;
  uint32_t *d_cmd, *d_err;
  int32_t *d_sizes;
  int64_t *d_offs;
  unsigned long long *d_stats;
  VTS_TRY(B.get(&d_sent, sent.size()));
  VTS_TRY(B.get(&d_went, went.size()));
  VTS_TRY(B.get(&d_recon, static_cast<size_t>(2 * ngop * S.stride + 256)));
  VTS_TRY(B.get(&d_cmd, static_cast<size_t>(went.size()) * nmb));  // every frame: searches run ahead
  uint8_t *d_cbp;
  VTS_TRY(B.get(&d_cbp, static_cast<size_t>(went.size()) * nmb));
  // residual levels: a ring of kRing levels (the searches run at most kRing
  // levels ahead of the slice writing that reads them)
  constexpr int64_t kRing = 32;
  int16_t *d_coef = nullptr;
  if (qp >= 1) VTS_TRY(B.get(&d_coef, static_cast<size_t>(kRing * ngop * nmb * kCoefPerMb)));
  constexpr int64_t kChunkLevels = 16;  // levels written and drained together
  int64_t max_chunk = 0;                 // entries of the largest chunk
  for (int64_t j0 = 0; j0 < maxlen; j0 += kChunkLevels)
    max_chunk = std::max(max_chunk, lvl_off[std::min(maxlen, j0 + kChunkLevels)] - lvl_off[j0]);
  VTS_TRY(B.get(&d_stage, static_cast<size_t>(max_chunk * mbh * cap)));
  VTS_TRY(B.get(&d_out, static_cast<size_t>(max_chunk * mbh * cap)));
  int64_t *d_total, *d_base, *d_fr;
  VTS_TRY(B.get(&d_total, 1));
  VTS_TRY(B.get(&d_base, 1));
  VTS_TRY(B.get(&d_fr, static_cast<size_t>(2 * n)));  // per frame: absolute offset, size
  VTS_TRY(B.get(&d_sizes, static_cast<size_t>(max_chunk * mbh)));
  VTS_TRY(B.get(&d_offs, static_cast<size_t>(max_chunk * mbh)));
  VTS_TRY(B.get(&d_stats, 3));
  VTS_TRY(B.get(&d_err, 1));
  uint4 *d_jobs;
  uint32_t *d_njobs;
  VTS_TRY(B.get(&d_jobs, static_cast<size_t>(max_chunk * nmb)));
  VTS_TRY(B.get(&d_njobs, 1));
  // Two streams: every level's motion search is enqueued up front on s1
  // (level j needs only level j-1's reconstruction); the slice writing of a
  // chunk of 16 levels (write, device offset scan, gather, I_PCM payloads,
  // drain to the host) runs on s2 behind the chunk's last search event,
  // overlapping the searches of later chunks.
  hipStream_t s1 = c->s_dec, s2 = c->s_score;
  B.streams = {s1, s2};
  HIP_TRY(hipMemcpy(d_sent, sent.data(), sent.size() * sizeof(int4), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(d_went, went.data(), went.size() * sizeof(int4), hipMemcpyHostToDevice));
  HIP_TRY(hipMemsetAsync(d_stats, 0, 3 * sizeof(unsigned long long), s2));
  HIP_TRY(hipMemsetAsync(d_err, 0, sizeof(uint32_t), s2));
  const int64_t nchunks = (maxlen + kChunkLevels - 1) / kChunkLevels;
  std::vector<hipEvent_t> ev(static_cast<size_t>(maxlen + 5 + nchunks), nullptr);
  struct EvGuard {
    std::vector<hipEvent_t> &v;
    ~EvGuard() {
      for (hipEvent_t e : v)
        if (e) (void)hipEventDestroy(e);
    }
  } ev_guard{ev};
  for (auto &e : ev) HIP_TRY(hipEventCreate(&e));
  hipEvent_t es0 = ev[maxlen], es1 = ev[maxlen + 1], ew0 = ev[maxlen + 2], ew1 = ev[maxlen + 3];
  hipEvent_t *wev = &ev[maxlen + 5];  // per chunk: its slices written (its ring slots free again)
  HIP_TRY(hipEventRecord(es0, s1));
  int64_t next_search = 1;
  bool searches_done = false;
  // enqueue the searches of levels < upto; level j reuses the ring slot of
  // level j - kRing, whose chunk's slice writing must have finished
  auto enqueue_searches = [&](int64_t upto) -> int {
    for (; next_search < std::min(maxlen, upto); ++next_search) {
      const int64_t j = next_search;
      if (qp >= 1 && j >= kRing) HIP_TRY(hipStreamWaitEvent(s1, wev[(j - kRing) / kChunkLevels], 0));
      const int64_t ne = lvl_off[j + 1] - lvl_off[j];
      SearchArgs sa{};
      sa.ent = d_sent + lvl_off[j];
      sa.small = S.d;
      sa.stride = S.stride;
      sa.recon = d_recon;
      sa.cmd = d_cmd + lvl_off[j] * nmb;
      sa.cbp = d_cbp + lvl_off[j] * nmb;
      sa.coef = d_coef ? d_coef + (j % kRing) * ngop * nmb * kCoefPerMb : nullptr;
      sa.cw = S.cw;
      sa.ch = S.ch;
      sa.mbw = mbw;
      sa.nmb = nmb;
      sa.range = R;
      sa.max_sad = T;
      sa.qp = qp;
      const dim3 grid(static_cast<unsigned>(ne * nmb));
      switch (R) {
        case 4: hipLaunchKernelGGL(enc_search<4>, grid, dim3(64), 0, s1, sa); break;
        case 8: hipLaunchKernelGGL(enc_search<8>, grid, dim3(64), 0, s1, sa); break;
        case 16: hipLaunchKernelGGL(enc_search<16>, grid, dim3(64), 0, s1, sa); break;
        default: hipLaunchKernelGGL(enc_search<0>, grid, dim3(64), 0, s1, sa); break;
      }
      HIP_TRY(hipEventRecord(ev[j], s1));
    }
    if (next_search >= maxlen && !searches_done) {
      HIP_TRY(hipEventRecord(es1, s1));
      searches_done = true;
    }
    return VTS_OK;
  };
  VTS_TRY(enqueue_searches(qp >= 1 ? kRing : maxlen));
  HIP_TRY(hipGetLastError());
  // Output drained to the host every chunk (absolute bytes [chunk_start[c],
  // chunk_start[c+1])) and appended to the MP4's mdat while the GPU works on
  // the next chunk; the sample table (display order) points into mdat.
  Mp4Writer mw;
  std::string e = mw.open(out_path);
  if (!e.empty()) return fail(VTS_E_IO, "%s: %s", out_path, e.c_str());
  std::vector<std::unique_ptr<uint8_t[]>> host;
  std::vector<int64_t> chunk_start{0}, chunk_file;  // chunk c's file offset
  hipEvent_t ev_d2h = ev[maxlen + 4];              // reused: the last chunk's D2H
  bool pending = false;                            // a chunk's D2H not yet written out
  double mux_ms = 0;
  auto write_pending = [&]() -> int {
    if (!pending) return VTS_OK;
    HIP_TRY(hipEventSynchronize(ev_d2h));
    const auto tw = clk::now();
    const size_t c = host.size() - 1;
    int64_t off = 0;
    const std::string we = mw.append(host[c].get(), static_cast<size_t>(chunk_start[c + 1] - chunk_start[c]), &off);
    if (!we.empty()) return fail(VTS_E_IO, "%s: %s", out_path, we.c_str());
    chunk_file.push_back(off);
    host[c].reset();
    pending = false;
    mux_ms += std::chrono::duration<double, std::milli>(clk::now() - tw).count();
    return VTS_OK;
  };
  int status = VTS_OK;
  HIP_TRY(hipMemsetAsync(d_total, 0, sizeof(int64_t), s2));
  HIP_TRY(hipEventRecord(ew0, s2));
  for (int64_t j0 = 0; j0 < maxlen && status == VTS_OK; j0 += kChunkLevels) {
    // one chunk of levels = one contiguous run of entries: written, scanned,
    // gathered and drained together (wide launches instead of one per level)
    const int64_t j1 = std::min(maxlen, j0 + kChunkLevels);
    const int64_t e0 = lvl_off[j0], ne = lvl_off[j1] - e0;
    const int ns = static_cast<int>(ne * mbh);
    if (j1 - 1 > 0) HIP_TRY(hipStreamWaitEvent(s2, ev[j1 - 1], 0));  // searches run in level order
    HIP_TRY(hipMemcpyAsync(d_base, d_total, sizeof(int64_t), hipMemcpyDeviceToDevice, s2));
    HIP_TRY(hipMemsetAsync(d_njobs, 0, sizeof(uint32_t), s2));
    WriteArgs wa{};
    wa.ent = d_went + e0;
    wa.cmd = d_cmd + e0 * nmb;
    wa.cbp = d_cbp + e0 * nmb;
    wa.coef = d_coef;
    wa.coef_per_level = ngop;
    wa.ring = static_cast<int32_t>(kRing);
    wa.qp = qp;
    wa.small = S.d;
    wa.stride = S.stride;
    wa.cw = S.cw;
    wa.ch = S.ch;
    wa.mbw = mbw;
    wa.mbh = mbh;
    wa.staging = d_stage;
    wa.cap = cap;
    wa.sizes = d_sizes;
    wa.stats = d_stats;
    wa.err = d_err;
    wa.jobs = d_jobs;
    wa.n_jobs = d_njobs;
    wa.n_slices = ns;
    hipLaunchKernelGGL(enc_write, dim3(static_cast<unsigned>((ns + 63) / 64)), dim3(64), 0, s2, wa);
    HIP_TRY(hipEventRecord(wev[j0 / kChunkLevels], s2));
    VTS_TRY(enqueue_searches(j1 + kRing));  // the ring slots of this chunk's levels are free once it is written
    hipLaunchKernelGGL(enc_scan, dim3(1), dim3(1024), 0, s2, d_sizes, ns, d_went + e0, mbh, d_offs, d_total,
                       d_fr, d_fr + n);
    hipLaunchKernelGGL(enc_gather, dim3(static_cast<unsigned>(ns)), dim3(256), 0, s2, d_stage, cap, d_sizes, d_offs,
                       d_base, d_out);
    hipLaunchKernelGGL(enc_pcm, dim3(static_cast<unsigned>(std::min<int64_t>(16384, ne * nmb))), dim3(64), 0, s2,
                       d_jobs, d_njobs, d_went + e0, S.d, S.stride, S.cw, S.ch, mbh, d_offs, d_base, d_out);
    const hipError_t he = hipGetLastError();
    if (he != hipSuccess) {
      status = fail(VTS_E_HIP, "encoder launch: %s", hipGetErrorString(he));
      break;
    }
    if (status != VTS_OK) break;
    int64_t tot = 0;
    if (hipMemcpyAsync(&tot, d_total, sizeof tot, hipMemcpyDeviceToHost, s2) != hipSuccess) {
      status = fail(VTS_E_HIP, "encoder levels %lld.. failed", static_cast<long long>(j0));
      break;
    }
    status = write_pending();  // the previous chunk, while this one runs
    if (status != VTS_OK) break;
    if (hipStreamSynchronize(s2) != hipSuccess) {
      status = fail(VTS_E_HIP, "encoder levels %lld.. failed", static_cast<long long>(j0));
      break;
    }
    const int64_t bytes = tot - chunk_start.back();
    host.emplace_back(new uint8_t[static_cast<size_t>(std::max<int64_t>(bytes, 1))]);
    HIP_TRY(hipMemcpyAsync(host.back().get(), d_out, static_cast<size_t>(bytes), hipMemcpyDeviceToHost, s2));
    HIP_TRY(hipEventRecord(ev_d2h, s2));
    pending = true;
    chunk_start.push_back(tot);
  }
  if (status == VTS_OK) status = write_pending();
  std::vector<int64_t> fr(static_cast<size_t>(2 * n), 0);
  if (status == VTS_OK)
    HIP_TRY(hipMemcpyAsync(fr.data(), d_fr, sizeof(int64_t) * 2 * n, hipMemcpyDeviceToHost, s2));
  HIP_TRY(hipEventRecord(ew1, s2));
  if (hipStreamSynchronize(s2) != hipSuccess || hipStreamSynchronize(s1) != hipSuccess)
    status = status ? status : fail(VTS_E_HIP, "encoder failed");
  if (status == VTS_OK) {
    float a_ms = 0, b_ms = 0;
    (void)hipEventElapsedTime(&a_ms, es0, es1);
    (void)hipEventElapsedTime(&b_ms, ew0, ew1);
    ms[1] = a_ms;
    ms[2] = b_ms;
  }
  VTS_TRY(status);
  uint32_t err = 0;
  unsigned long long st[3] = {0, 0, 0};
  HIP_TRY(hipMemcpy(&err, d_err, sizeof err, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(st, d_stats, sizeof st, hipMemcpyDeviceToHost));
  if (err) return fail(VTS_E_CAPACITY, "a slice exceeded its %lld-byte staging slot", static_cast<long long>(cap));

  // 4. MP4 sample table (display order) over the mdat written above
  t0 = clk::now();
  std::vector<uint8_t> sps, pps;
  const double fps = static_cast<double>(c->info.track_timescale) / static_cast<double>(delta);
  make_sps_pps(mbw, mbh, S.cw - S.w, S.ch - S.h, h264_pick_level(nmb, nmb * fps), &sps, &pps);
  std::vector<uint8_t> is_idr(static_cast<size_t>(n), 0);
  for (int64_t f : gop_start) is_idr[f] = 1;
  for (int64_t f = 0; f < n && e.empty(); ++f) {
    const int64_t off = fr[f], size = fr[n + f];
    const size_t ci = static_cast<size_t>(std::upper_bound(chunk_start.begin(), chunk_start.end(), off) -
                                          chunk_start.begin()) - 1;
    if (ci >= chunk_file.size() || off + size > chunk_start[ci + 1])
      return fail(VTS_E_HIP, "frame %lld: output bookkeeping mismatch", static_cast<long long>(f));
    e = mw.add_sample_at(chunk_file[ci] + (off - chunk_start[ci]), static_cast<size_t>(size), is_idr[f] != 0);
  }
  if (e.empty()) e = mw.finish(S.w, S.h, c->info.track_timescale, delta, sps, pps);
  if (!e.empty()) return fail(VTS_E_IO, "%s: %s", out_path, e.c_str());
  ms[3] = mux_ms + std::chrono::duration<double, std::milli>(clk::now() - t0).count();
  if (info) {
    std::memset(info, 0, sizeof *info);
    info->width = S.w;
    info->height = S.h;
    info->n_frames = n;
    info->n_idr = ngop;
    info->pcm_mbs = static_cast<int64_t>(st[0]);
    info->inter_mbs = static_cast<int64_t>(st[1]);
    info->skip_mbs = static_cast<int64_t>(st[2]);
    info->bytes_written = mw.bytes_written();
    for (int i = 0; i < 4; ++i) info->ms[i] = ms[i];
  }
  return VTS_OK;
}
