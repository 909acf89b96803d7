// score.hip — per-frame scene scoring of NV12 surfaces on gfx950 (MI355X).
//
// No reference counterpart (the reference never decodes pixels for scoring);
// the definition below is the contract checked bit-exactly against
// oracle/vtseg_oracle.c:score_frames().
//
// One fused pass per frame, HBM-bound (no MFMA — this is a pixel reduction):
//   Y' = box mean of k x k luma, U'/V' = box mean of (k/2)x(k/2) chroma,
//   RGB = BT.709 limited-range fixed point of (Y',U',V'),
//   hist[256] of Y', SAD = sum |Y'_t - Y'_{t-1}|, score = sad / (w*h*255).
//
// Work decomposition (DESIGN.md §Score kernel):
//   * a workgroup of 1024 threads (16 waves) owns a TEMPORAL RUN of
//     consecutive frames; each thread owns a fixed set of "chunks" (G
//     thumbnail pixels = G*k bytes of each of k luma rows and k/2 UV rows), so
//     its previous-frame thumbnail luma sits in LDS at a thread-private slot —
//     SAD needs no second read of the previous frame;
//   * loads are 16 B per lane, consecutive lanes on consecutive chunks:
//     every load instruction covers 1 KiB of contiguous row bytes;
//   * byte sums use v_sad_u8 (|a-0| summed over 4 packed bytes), the frame
//     SAD uses v_sad_u8 on packed thumbnail luma, 4 pixels per instruction;
//   * the histogram is one LDS array per workgroup (ds_add_u32), written back
//     with plain stores once per frame — no global atomics, deterministic;
//   * the first frame of each run (other than run 0) gets its SAD from a tiny
//     seam kernel that compares the run's head thumbnail with the previous
//     run's tail thumbnail.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "common.h"
#include "decode.h"
#include "pixel.h"

namespace vts {
namespace {

constexpr int kThreads = 1024;
constexpr int kMaxRuns = 512;  // 256 CUs x 2 resident 1024-thread workgroups

template <int K>
struct Geo {
  static constexpr int kRowBytes = (K == 6) ? 48 : 16;   // bytes per row per chunk
  static constexpr int kWords = kRowBytes / 4;
  static constexpr int kG = kRowBytes / K;               // thumbnail px per chunk
  static constexpr int kH = K / 2;                       // chroma rows per box
  static constexpr uint32_t kYDiv = K * K;
  static constexpr uint32_t kCDiv = kH * kH;
};

// Sum of bytes [b0, b1) of the word array w (compile-time bounds).
template <int B0, int B1, int MASKSTEP = 1>
__device__ __forceinline__ uint32_t byte_sum(const uint32_t *w, uint32_t acc) {
#pragma unroll
  for (int wi = B0 / 4; wi <= (B1 - 1) / 4; ++wi) {
    uint32_t m = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int idx = wi * 4 + b;
      if (idx >= B0 && idx < B1 && ((idx - B0) % MASKSTEP) == 0) m |= 0xffu << (8 * b);
    }
    acc = sad_u8(w[wi] & m, 0u, acc);
  }
  return acc;
}

// Load kRowBytes of one row at `p` (16-byte aligned) as words.
template <int NW>
__device__ __forceinline__ void load_row(const uint8_t *p, uint32_t *w) {
#pragma unroll
  for (int i = 0; i < NW / 4; ++i) {
    const uint4 v = *reinterpret_cast<const uint4 *>(p + 16 * i);
    w[4 * i + 0] = v.x;
    w[4 * i + 1] = v.y;
    w[4 * i + 2] = v.z;
    w[4 * i + 3] = v.w;
  }
}

// One chunk of a thumbnail (G pixels of thumbnail row ty, from byte column
// col): luma box means yq and packed RGB (r | g << 8 | b << 16), each pixel
// counted into the LDS histogram as it is made; thumb_pics' form of
// score_runs' inner loop (kept inline there: sharing this function cost
// score_runs<6> 36 VGPRs and spills)
template <int K>
__device__ __forceinline__ void thumb_chunk(const uint8_t *yplane, const uint8_t *uvplane, int pitch, int ty,
                                            int64_t col, uint32_t *lds_hist, uint32_t (&yq)[Geo<K>::kG],
                                            uint32_t (&rgb24)[Geo<K>::kG]) {
  using G = Geo<K>;
  // --- luma box sums: G pixels, K rows
  uint32_t ys[G::kG];
#pragma unroll
  for (int p = 0; p < G::kG; ++p) ys[p] = 0;
#pragma unroll
  for (int r = 0; r < K; ++r) {
    uint32_t w[G::kWords];
    load_row<G::kWords>(yplane + static_cast<int64_t>(ty * K + r) * pitch + col, w);
#pragma unroll
    for (int p = 0; p < G::kG; ++p) {
      if constexpr (K == 6) {
        // compile-time byte ranges [6p, 6p+6)
        switch (p) {
          case 0: ys[0] = byte_sum<0, 6>(w, ys[0]); break;
          case 1: ys[1] = byte_sum<6, 12>(w, ys[1]); break;
          case 2: ys[2] = byte_sum<12, 18>(w, ys[2]); break;
          case 3: ys[3] = byte_sum<18, 24>(w, ys[3]); break;
          case 4: ys[4] = byte_sum<24, 30>(w, ys[4]); break;
          case 5: ys[5] = byte_sum<30, 36>(w, ys[5]); break;
          case 6: ys[6] = byte_sum<36, 42>(w, ys[6]); break;
          default: ys[7] = byte_sum<42, 48>(w, ys[7]); break;
        }
      } else if constexpr (K == 2) {
        ys[p] = sad_u8(w[p / 2] & ((p & 1) ? 0xffff0000u : 0x0000ffffu), 0u, ys[p]);
      } else if constexpr (K == 4) {
        ys[p] = sad_u8(w[p], 0u, ys[p]);
      } else {  // K == 8
        ys[p] = sad_u8(w[2 * p + 1], 0u, sad_u8(w[2 * p], 0u, ys[p]));
      }
    }
  }
  // --- chroma box sums: interleaved UV, K/2 rows, same byte columns
  uint32_t us[G::kG], vs[G::kG];
#pragma unroll
  for (int p = 0; p < G::kG; ++p) us[p] = vs[p] = 0;
#pragma unroll
  for (int r = 0; r < G::kH; ++r) {
    uint32_t w[G::kWords];
    load_row<G::kWords>(uvplane + static_cast<int64_t>(ty * G::kH + r) * pitch + col, w);
#pragma unroll
    for (int p = 0; p < G::kG; ++p) {
      if constexpr (K == 6) {
        switch (p) {
          case 0: us[0] = byte_sum<0, 6, 2>(w, us[0]); vs[0] = byte_sum<1, 6, 2>(w, vs[0]); break;
          case 1: us[1] = byte_sum<6, 12, 2>(w, us[1]); vs[1] = byte_sum<7, 12, 2>(w, vs[1]); break;
          case 2: us[2] = byte_sum<12, 18, 2>(w, us[2]); vs[2] = byte_sum<13, 18, 2>(w, vs[2]); break;
          case 3: us[3] = byte_sum<18, 24, 2>(w, us[3]); vs[3] = byte_sum<19, 24, 2>(w, vs[3]); break;
          case 4: us[4] = byte_sum<24, 30, 2>(w, us[4]); vs[4] = byte_sum<25, 30, 2>(w, vs[4]); break;
          case 5: us[5] = byte_sum<30, 36, 2>(w, us[5]); vs[5] = byte_sum<31, 36, 2>(w, vs[5]); break;
          case 6: us[6] = byte_sum<36, 42, 2>(w, us[6]); vs[6] = byte_sum<37, 42, 2>(w, vs[6]); break;
          default: us[7] = byte_sum<42, 48, 2>(w, us[7]); vs[7] = byte_sum<43, 48, 2>(w, vs[7]); break;
        }
      } else if constexpr (K == 2) {
        // one UV pair per thumbnail px: bytes 2p, 2p+1
        const uint32_t word = w[p / 2] >> ((p & 1) * 16);
        us[p] += word & 0xffu;
        vs[p] += (word >> 8) & 0xffu;
      } else if constexpr (K == 4) {
        us[p] = sad_u8(w[p] & 0x00ff00ffu, 0u, us[p]);
        vs[p] = sad_u8((w[p] >> 8) & 0x00ff00ffu, 0u, vs[p]);
      } else {  // K == 8: 4 UV pairs = 8 bytes = 2 words
        us[p] = sad_u8(w[2 * p + 1] & 0x00ff00ffu, 0u, sad_u8(w[2 * p] & 0x00ff00ffu, 0u, us[p]));
        vs[p] = sad_u8((w[2 * p + 1] >> 8) & 0x00ff00ffu, 0u,
                       sad_u8((w[2 * p] >> 8) & 0x00ff00ffu, 0u, vs[p]));
      }
    }
  }
  // --- thumbnail pixels: round, convert, histogram
#pragma unroll
  for (int p = 0; p < G::kG; ++p) {
    const uint32_t y = (ys[p] + G::kYDiv / 2) / G::kYDiv;
    const uint32_t u = (us[p] + G::kCDiv / 2) / G::kCDiv;
    const uint32_t v = (vs[p] + G::kCDiv / 2) / G::kCDiv;
    yq[p] = y;
    rgb24[p] = bt709_rgb24(y, u, v);
    atomicAdd(&lds_hist[y], 1u);
  }
}

struct RunArgs {
  const uint8_t *nv12;
  int64_t frame_stride;
  int64_t n_frames;
  int32_t w, h;            // thumbnail size
  int32_t pitch, uv_row_offset;
  int32_t chunks_per_row;  // w / G
  int32_t n_chunks;        // chunks_per_row * h
  int32_t n_runs;
  int32_t has_prev;
  uint8_t *rgb;
  uint32_t *hist;
  uint64_t *sad;
  float *score;
  const uint8_t *prev_luma;
  uint8_t *last_luma;
  uint8_t *head;           // n_runs * w*h
  uint8_t *tail;           // n_runs * w*h
};

template <int K>
__global__ void __launch_bounds__(kThreads, 2) score_runs(RunArgs a) {
  using G = Geo<K>;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t *lds_hist = reinterpret_cast<uint32_t *>(smem);             // 256
  uint32_t *lds_red = reinterpret_cast<uint32_t *>(smem + 1024);       // 16 waves
  uint8_t *lds_prev = smem + 1024 + 64;                                // w*h bytes

  const int tid = threadIdx.x;
  const int run = blockIdx.x;
  const int64_t f0 = (a.n_frames * run) / a.n_runs;
  const int64_t f1 = (a.n_frames * (run + 1)) / a.n_runs;
  const int64_t npx = static_cast<int64_t>(a.w) * a.h;
  const double denom = static_cast<double>(npx) * 255.0;

  for (int i = tid; i < 256; i += kThreads) lds_hist[i] = 0;
  // Run 0 may be seeded with the previous batch's last thumbnail.
  const bool seeded = (run == 0) && a.has_prev;
  if (seeded)
    for (int64_t i = tid; i < npx; i += kThreads) lds_prev[i] = a.prev_luma[i];
  __syncthreads();

  for (int64_t f = f0; f < f1; ++f) {
    const uint8_t *yplane = a.nv12 + f * a.frame_stride;
    const uint8_t *uvplane = yplane + static_cast<int64_t>(a.pitch) * a.uv_row_offset;
    const bool have_prev = (f > f0) || seeded;
    uint32_t sad = 0;
    for (int c = tid; c < a.n_chunks; c += kThreads) {
      const int ty = c / a.chunks_per_row;
      const int tx = c - ty * a.chunks_per_row;
      const int64_t col = static_cast<int64_t>(tx) * G::kRowBytes;
      // --- luma box sums: G pixels, K rows
      uint32_t ys[G::kG];
#pragma unroll
      for (int p = 0; p < G::kG; ++p) ys[p] = 0;
#pragma unroll
      for (int r = 0; r < K; ++r) {
        uint32_t w[G::kWords];
        load_row<G::kWords>(yplane + static_cast<int64_t>(ty * K + r) * a.pitch + col, w);
#pragma unroll
        for (int p = 0; p < G::kG; ++p) {
          if constexpr (K == 6) {
            // compile-time byte ranges [6p, 6p+6)
            switch (p) {
              case 0: ys[0] = byte_sum<0, 6>(w, ys[0]); break;
              case 1: ys[1] = byte_sum<6, 12>(w, ys[1]); break;
              case 2: ys[2] = byte_sum<12, 18>(w, ys[2]); break;
              case 3: ys[3] = byte_sum<18, 24>(w, ys[3]); break;
              case 4: ys[4] = byte_sum<24, 30>(w, ys[4]); break;
              case 5: ys[5] = byte_sum<30, 36>(w, ys[5]); break;
              case 6: ys[6] = byte_sum<36, 42>(w, ys[6]); break;
              default: ys[7] = byte_sum<42, 48>(w, ys[7]); break;
            }
          } else if constexpr (K == 2) {
            ys[p] = sad_u8(w[p / 2] & ((p & 1) ? 0xffff0000u : 0x0000ffffu), 0u, ys[p]);
          } else if constexpr (K == 4) {
            ys[p] = sad_u8(w[p], 0u, ys[p]);
          } else {  // K == 8
            ys[p] = sad_u8(w[2 * p + 1], 0u, sad_u8(w[2 * p], 0u, ys[p]));
          }
        }
      }
      // --- chroma box sums: interleaved UV, K/2 rows, same byte columns
      uint32_t us[G::kG], vs[G::kG];
#pragma unroll
      for (int p = 0; p < G::kG; ++p) us[p] = vs[p] = 0;
#pragma unroll
      for (int r = 0; r < G::kH; ++r) {
        uint32_t w[G::kWords];
        load_row<G::kWords>(uvplane + static_cast<int64_t>(ty * G::kH + r) * a.pitch + col, w);
#pragma unroll
        for (int p = 0; p < G::kG; ++p) {
          if constexpr (K == 6) {
            switch (p) {
              case 0: us[0] = byte_sum<0, 6, 2>(w, us[0]); vs[0] = byte_sum<1, 6, 2>(w, vs[0]); break;
              case 1: us[1] = byte_sum<6, 12, 2>(w, us[1]); vs[1] = byte_sum<7, 12, 2>(w, vs[1]); break;
              case 2: us[2] = byte_sum<12, 18, 2>(w, us[2]); vs[2] = byte_sum<13, 18, 2>(w, vs[2]); break;
              case 3: us[3] = byte_sum<18, 24, 2>(w, us[3]); vs[3] = byte_sum<19, 24, 2>(w, vs[3]); break;
              case 4: us[4] = byte_sum<24, 30, 2>(w, us[4]); vs[4] = byte_sum<25, 30, 2>(w, vs[4]); break;
              case 5: us[5] = byte_sum<30, 36, 2>(w, us[5]); vs[5] = byte_sum<31, 36, 2>(w, vs[5]); break;
              case 6: us[6] = byte_sum<36, 42, 2>(w, us[6]); vs[6] = byte_sum<37, 42, 2>(w, vs[6]); break;
              default: us[7] = byte_sum<42, 48, 2>(w, us[7]); vs[7] = byte_sum<43, 48, 2>(w, vs[7]); break;
            }
          } else if constexpr (K == 2) {
            // one UV pair per thumbnail px: bytes 2p, 2p+1
            const uint32_t word = w[p / 2] >> ((p & 1) * 16);
            us[p] += word & 0xffu;
            vs[p] += (word >> 8) & 0xffu;
          } else if constexpr (K == 4) {
            us[p] = sad_u8(w[p] & 0x00ff00ffu, 0u, us[p]);
            vs[p] = sad_u8((w[p] >> 8) & 0x00ff00ffu, 0u, vs[p]);
          } else {  // K == 8: 4 UV pairs = 8 bytes = 2 words
            us[p] = sad_u8(w[2 * p + 1] & 0x00ff00ffu, 0u, sad_u8(w[2 * p] & 0x00ff00ffu, 0u, us[p]));
            vs[p] = sad_u8((w[2 * p + 1] >> 8) & 0x00ff00ffu, 0u,
                           sad_u8((w[2 * p] >> 8) & 0x00ff00ffu, 0u, vs[p]));
          }
        }
      }
      // --- thumbnail pixels: round, convert, histogram
      uint32_t yq[G::kG];
      uint32_t rgb24[G::kG];  // r | g << 8 | b << 16
#pragma unroll
      for (int p = 0; p < G::kG; ++p) {
        const uint32_t y = (ys[p] + G::kYDiv / 2) / G::kYDiv;
        const uint32_t u = (us[p] + G::kCDiv / 2) / G::kCDiv;
        const uint32_t v = (vs[p] + G::kCDiv / 2) / G::kCDiv;
        yq[p] = y;
        rgb24[p] = bt709_rgb24(y, u, v);
        atomicAdd(&lds_hist[y], 1u);
      }
      // --- SAD against the previous frame's thumbnail (thread-private LDS slot)
      const int64_t tpx = static_cast<int64_t>(ty) * a.w + static_cast<int64_t>(tx) * G::kG;
      uint32_t packed[(G::kG + 3) / 4];
#pragma unroll
      for (int q = 0; q < (G::kG + 3) / 4; ++q) {
        uint32_t word = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b)
          if (4 * q + b < G::kG) word |= yq[4 * q + b] << (8 * b);
        packed[q] = word;
      }
      if constexpr (G::kG >= 4) {
        uint32_t *slot = reinterpret_cast<uint32_t *>(lds_prev + tpx);
#pragma unroll
        for (int q = 0; q < G::kG / 4; ++q) {
          if (have_prev) sad = sad_u8(packed[q], slot[q], sad);
          slot[q] = packed[q];
        }
      } else {  // G == 2 (K == 8): 16-bit slot
        uint16_t *slot = reinterpret_cast<uint16_t *>(lds_prev + tpx);
        if (have_prev) sad = sad_u8(packed[0], static_cast<uint32_t>(*slot), sad);
        *slot = static_cast<uint16_t>(packed[0]);
      }
      // --- stores: RGB thumbnail, run head / tail thumbnails
      if (a.rgb) {
        uint8_t *dst = a.rgb + f * npx * 3 + tpx * 3;
        store_rgb<G::kG>(dst, rgb24);
      }
      if (f == f0 && !seeded) {
        uint8_t *dst = a.head + static_cast<int64_t>(run) * npx + tpx;
#pragma unroll
        for (int p = 0; p < G::kG; ++p) dst[p] = static_cast<uint8_t>(yq[p]);
      }
      if (f == f1 - 1) {
        uint8_t *dst = (run == a.n_runs - 1 && a.last_luma)
                           ? a.last_luma + tpx
                           : a.tail + static_cast<int64_t>(run) * npx + tpx;
#pragma unroll
        for (int p = 0; p < G::kG; ++p) dst[p] = static_cast<uint8_t>(yq[p]);
      }
    }
    // --- per-frame reductions
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) sad += __shfl_xor(sad, off, 64);
    if ((tid & 63) == 0) lds_red[tid >> 6] = sad;
    __syncthreads();
    if (a.hist && tid < 256) a.hist[f * 256 + tid] = lds_hist[tid];
    if (tid < 256) lds_hist[tid] = 0;
    if (tid == 0) {
      uint64_t total = 0;
      for (int wv = 0; wv < kThreads / 64; ++wv) total += lds_red[wv];
      if (have_prev) {
        a.sad[f] = total;
        a.score[f] = static_cast<float>(static_cast<double>(total) / denom);
      } else if (run == 0) {  // very first frame, nothing to compare
        a.sad[f] = 0;
        a.score[f] = 0.0f;
      }
    }
    __syncthreads();
  }
}

// SAD of run r's head thumbnail against run r-1's tail thumbnail.
__global__ void __launch_bounds__(256) score_seams(RunArgs a) {
  const int run = blockIdx.x + 1;
  const int64_t f0 = (a.n_frames * run) / a.n_runs;
  const int64_t npx = static_cast<int64_t>(a.w) * a.h;
  const uint8_t *head = a.head + static_cast<int64_t>(run) * npx;
  const uint8_t *tail = a.tail + static_cast<int64_t>(run - 1) * npx;
  uint32_t s = 0;
  // npx is a multiple of 4 (w divisible by G >= 2, h even), buffers 4-aligned
  const int64_t nw = npx / 4;
  for (int64_t i = threadIdx.x; i < nw; i += blockDim.x)
    s = sad_u8(reinterpret_cast<const uint32_t *>(head)[i],
               reinterpret_cast<const uint32_t *>(tail)[i], s);
  for (int64_t i = nw * 4 + threadIdx.x; i < npx; i += blockDim.x) {
    const int d = static_cast<int>(head[i]) - static_cast<int>(tail[i]);
    s += static_cast<uint32_t>(d < 0 ? -d : d);
  }
  __shared__ uint32_t red[4];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t total = uint64_t(red[0]) + red[1] + red[2] + red[3];
    a.sad[f0] = total;
    a.score[f0] = static_cast<float>(static_cast<double>(total) /
                                     (static_cast<double>(npx) * 255.0));
  }
}

// Thumbnails of a list of pictures (one reconstruction level of the general
// decoder, so a surface can be reused once its level is thumbnailed): luma
// thumbnail into the window's thumbnail ring, RGB, histogram by frame.  The
// launch sits on the level chain, so each picture is split over
// blockIdx.y bands of thumbnail rows (a chunk per thread, not one
// workgroup's long loop); a band adds its LDS histogram into the frame's
// (zeroed per window, integer adds: deterministic).  thumb_sad then scores the
// window from the ring.
constexpr int kThumbThreads = 256;
template <int K>
__global__ void __launch_bounds__(kThumbThreads) thumb_pics(PicThumbArgs a) {
  using G = Geo<K>;
  __shared__ uint32_t lds_hist[256];
  const int tid = threadIdx.x;
  const int slot = a.pics[blockIdx.x].x;
  const int64_t f = a.f0 + slot;
  const uint8_t *yplane = a.surf + static_cast<int64_t>(a.surf_of ? a.surf_of[slot] : slot) * a.frame_stride;
  const uint8_t *uvplane = yplane + static_cast<int64_t>(a.pitch) * a.uv_row_offset;
  const int64_t npx = static_cast<int64_t>(a.w) * a.h;
  lds_hist[tid] = 0;
  __syncthreads();
  uint8_t *thumb = a.thumb + static_cast<int64_t>(slot) * npx;
  const int r0 = static_cast<int>((static_cast<int64_t>(a.h) * blockIdx.y) / gridDim.y);
  const int r1 = static_cast<int>((static_cast<int64_t>(a.h) * (blockIdx.y + 1)) / gridDim.y);
  for (int c = r0 * a.chunks_per_row + tid; c < r1 * a.chunks_per_row; c += kThumbThreads) {
    const int ty = c / a.chunks_per_row;
    const int tx = c - ty * a.chunks_per_row;
    uint32_t yq[G::kG], rgb24[G::kG];
    thumb_chunk<K>(yplane, uvplane, a.pitch, ty, static_cast<int64_t>(tx) * G::kRowBytes, lds_hist, yq, rgb24);
    const int64_t tpx = static_cast<int64_t>(ty) * a.w + static_cast<int64_t>(tx) * G::kG;
    if constexpr (G::kG >= 4) {
#pragma unroll
      for (int q = 0; q < G::kG / 4; ++q)
        reinterpret_cast<uint32_t *>(thumb + tpx)[q] = yq[4 * q] | yq[4 * q + 1] << 8 | yq[4 * q + 2] << 16 | yq[4 * q + 3] << 24;
    } else {
      *reinterpret_cast<uint16_t *>(thumb + tpx) = static_cast<uint16_t>(yq[0] | yq[1] << 8);
    }
    if (a.rgb) store_rgb<G::kG>(a.rgb + f * npx * 3 + tpx * 3, rgb24);
  }
  __syncthreads();
  if (a.hist && lds_hist[tid]) atomicAdd(&a.hist[f * 256 + tid], lds_hist[tid]);
}

int row_bytes_for(int k) { return k == 6 ? 48 : 16; }

}  // namespace

int64_t score_workspace_bytes(int32_t width, int32_t height, int32_t k, int64_t n_frames) {
  if (k <= 0) return 0;
  const int64_t npx = static_cast<int64_t>(width / k) * (height / k);
  const int64_t runs = n_frames < kMaxRuns ? (n_frames > 0 ? n_frames : 1) : kMaxRuns;
  return 2 * runs * npx + 256;
}

int score_launch(const vts_score_desc *d, hipStream_t stream) {
  if (!d) return fail(VTS_E_INVALID, "desc is NULL");
  const int k = d->k;
  if (k != 2 && k != 4 && k != 6 && k != 8) return fail(VTS_E_INVALID, "k must be 2, 4, 6 or 8");
  if (d->width <= 0 || d->height <= 0 || d->width % k || d->height % k)
    return fail(VTS_E_INVALID, "width/height (%d x %d) must be positive multiples of k=%d",
                d->width, d->height, k);
  const int rb = row_bytes_for(k);
  if (d->width % rb)
    return fail(VTS_E_INVALID, "width %d must be a multiple of %d for k=%d", d->width, rb, k);
  if (d->pitch < d->width || d->pitch % 16)
    return fail(VTS_E_INVALID, "pitch must be >= width and a multiple of 16");
  if (d->uv_row_offset < d->height) return fail(VTS_E_INVALID, "uv_row_offset < height");
  if (d->frame_stride % 16 ||
      d->frame_stride < static_cast<int64_t>(d->pitch) * (d->uv_row_offset + d->height / 2))
    return fail(VTS_E_INVALID, "frame_stride too small or not 16-aligned");
  if (!d->nv12 || !d->sad || !d->score) return fail(VTS_E_INVALID, "NULL nv12/sad/score");
  if (reinterpret_cast<uintptr_t>(d->nv12) % 16) return fail(VTS_E_INVALID, "nv12 not 16-aligned");
  if (!d->workspace || reinterpret_cast<uintptr_t>(d->workspace) % 16)
    return fail(VTS_E_INVALID, "workspace NULL or not 16-aligned");
  if (d->rgb && reinterpret_cast<uintptr_t>(d->rgb) % 4)
    return fail(VTS_E_INVALID, "rgb not 4-aligned");
  if (d->n_frames < 0) return fail(VTS_E_INVALID, "n_frames < 0");
  if (d->n_frames == 0) return VTS_OK;
  const int w = d->width / k, h = d->height / k;
  const int64_t npx = static_cast<int64_t>(w) * h;
  const size_t lds = 1024 + 64 + static_cast<size_t>((npx + 15) & ~int64_t(15));
  if (lds > 160 * 1024)
    return fail(VTS_E_INVALID, "thumbnail %dx%d too large for LDS; use a larger k", w, h);
  const int64_t need = score_workspace_bytes(d->width, d->height, k, d->n_frames);
  if (!d->workspace || d->workspace_bytes < need)
    return fail(VTS_E_INVALID, "workspace needs %lld bytes", static_cast<long long>(need));

  RunArgs a{};
  a.nv12 = d->nv12;
  a.frame_stride = d->frame_stride;
  a.n_frames = d->n_frames;
  a.w = w;
  a.h = h;
  a.pitch = d->pitch;
  a.uv_row_offset = d->uv_row_offset;
  a.chunks_per_row = d->width / rb;
  a.n_chunks = a.chunks_per_row * h;
  a.n_runs = static_cast<int32_t>(d->n_frames < kMaxRuns ? d->n_frames : kMaxRuns);
  a.has_prev = d->prev_luma ? 1 : 0;
  a.rgb = d->rgb;
  a.hist = d->hist;
  a.sad = d->sad;
  a.score = d->score;
  a.prev_luma = d->prev_luma;
  a.last_luma = d->last_luma;
  // head / tail thumbnails: n_runs slots of npx bytes each (npx % 4 == 0)
  a.head = d->workspace;
  a.tail = d->workspace + static_cast<int64_t>(a.n_runs) * npx;

  hipError_t e;
  switch (k) {
    case 2: hipLaunchKernelGGL(score_runs<2>, dim3(a.n_runs), dim3(kThreads), lds, stream, a); break;
    case 4: hipLaunchKernelGGL(score_runs<4>, dim3(a.n_runs), dim3(kThreads), lds, stream, a); break;
    case 6: hipLaunchKernelGGL(score_runs<6>, dim3(a.n_runs), dim3(kThreads), lds, stream, a); break;
    default: hipLaunchKernelGGL(score_runs<8>, dim3(a.n_runs), dim3(kThreads), lds, stream, a); break;
  }
  e = hipGetLastError();
  if (e != hipSuccess) return fail(VTS_E_HIP, "score_runs launch: %s", hipGetErrorString(e));
  if (a.n_runs > 1) {
    hipLaunchKernelGGL(score_seams, dim3(a.n_runs - 1), dim3(256), 0, stream, a);
    e = hipGetLastError();
    if (e != hipSuccess) return fail(VTS_E_HIP, "score_seams launch: %s", hipGetErrorString(e));
  }
  return VTS_OK;
}

int thumb_pics_launch(const PicThumbArgs &a, int k, hipStream_t s) {
  if (a.n_pics <= 0) return VTS_OK;
  if (a.w * k > a.pitch || a.chunks_per_row * row_bytes_for(k) != a.w * k || a.n_chunks != a.chunks_per_row * a.h)
    return fail(VTS_E_INVALID, "thumb_pics: thumbnail geometry does not match k=%d", k);
  // bands of rows: one chunk per thread (VTS_THUMB_CHUNKS; 1 / 2 / 4 / 8
  // measured, 1 the shortest level chain: profiles/r05am_thumb_bands_ab.json)
  static const int per_thread = [] {
    const char *e = std::getenv("VTS_THUMB_CHUNKS");
    return e ? std::max(1, std::atoi(e)) : 1;
  }();
  const int bands = std::max(1, std::min(a.h, (a.n_chunks + per_thread * kThumbThreads - 1) / (per_thread * kThumbThreads)));
  const dim3 grid(static_cast<unsigned>(a.n_pics), static_cast<unsigned>(bands));
  switch (k) {
    case 2: hipLaunchKernelGGL(thumb_pics<2>, grid, dim3(kThumbThreads), 0, s, a); break;
    case 4: hipLaunchKernelGGL(thumb_pics<4>, grid, dim3(kThumbThreads), 0, s, a); break;
    case 6: hipLaunchKernelGGL(thumb_pics<6>, grid, dim3(kThumbThreads), 0, s, a); break;
    case 8: hipLaunchKernelGGL(thumb_pics<8>, grid, dim3(kThumbThreads), 0, s, a); break;
    default: return fail(VTS_E_INVALID, "thumb_pics: k must be 2, 4, 6 or 8");
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(VTS_E_HIP, "thumb_pics launch: %s", hipGetErrorString(e));
  return VTS_OK;
}

}  // namespace vts

extern "C" int64_t vts_score_workspace_bytes(int32_t width, int32_t height, int32_t k,
                                             int64_t n_frames) {
  return vts::score_workspace_bytes(width, height, k, n_frames);
}

extern "C" int vts_score_nv12_dev(const vts_score_desc *desc, void *hip_stream) {
  vts::clear_error();
  return vts::score_launch(desc, static_cast<hipStream_t>(hip_stream));
}
