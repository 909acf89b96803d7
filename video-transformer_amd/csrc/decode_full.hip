// decode_full.hip — kernels of the general H.264 decoder (CAVLC I/P: intra
// 4x4 / 16x16 / chroma prediction, residuals, quarter-sample motion over up to
// 16 references, the deblocking filter).  DESIGN.md §5b.
//
//   h264_parse_full   one lane per slice: slice_data() -> MbRec + coefficient
//                     blocks (parse_full.h)
//   h264_recon_full   one workgroup per picture of a level launch: every inter
//                     macroblock in parallel (one lane each), then the intra
//                     macroblocks along the t = x + 2y wavefront (left, top,
//                     top-right neighbours are done one step earlier), a
//                     workgroup barrier per step (recon_full.h MbRecon)
//   h264_deblock_full one workgroup per picture: macroblocks along the same
//                     wavefront, which orders every pair of overlapping edge
//                     filters as the standard's raster order does (8.7)
// The per-macroblock code is shared with the CPU harness that is checked
// against the oracle (tests/test_full_host.py).
#include <hip/hip_runtime.h>

#include "common.h"
#include "decode_full.h"
#include "parse_full.h"
#include "recon_full.h"

namespace vts {
namespace {

constexpr int kParseLanes = 64;
constexpr int kReconThreads = 256;
constexpr int kDeblockThreads = 64;

__global__ void __launch_bounds__(kParseLanes) h264_parse_full(FullParseArgs a) {
  __shared__ full::FullScratch scratch[kParseLanes];
  const int i = blockIdx.x * kParseLanes + threadIdx.x;
  if (i >= a.n_slices) return;
  const FullSlice s = a.slices[i];
  const int64_t nmb = static_cast<int64_t>(a.P.mb_width) * a.P.mb_height;
  const uint32_t e = full::parse_slice_full(a.es, s, static_cast<uint32_t>(a.slice0 + i), a.P,
                                            a.recs + s.slot * nmb, a.arena, a.epoch, &scratch[threadIdx.x]);
  if (e) atomicOr(a.err, e);
}

__device__ full::ReconCtx make_ctx(const FullReconArgs &a, int slot) {
  full::ReconCtx c{};
  const int64_t nmb = static_cast<int64_t>(a.P.mb_width) * a.P.mb_height;
  c.recs = a.recs + slot * nmb;
  c.arena = a.arena;
  c.slices = a.slices;
  c.surf = a.surf;
  c.frame_stride = a.frame_stride;
  c.pitch = a.pitch;
  c.uv_off = a.uv_off;
  c.mbw = a.P.mb_width;
  c.mbh = a.P.mb_height;
  c.cip = a.P.cip;
  c.cqp_off = a.P.cqp_off;
  c.cqp_off2 = a.P.cqp_off2;
  c.epoch = a.epoch;
  return c;
}

__global__ void __launch_bounds__(kReconThreads) h264_recon_full(FullReconArgs a) {
  const int slot = a.frames[blockIdx.x].x;
  const full::ReconCtx c = make_ctx(a, slot);
  const int mbw = c.mbw, mbh = c.mbh, nmb = mbw * mbh;
  uint32_t err = 0;
  // inter macroblocks: independent of each other
  for (int mb = threadIdx.x; mb < nmb; mb += kReconThreads) {
    const MbRec &m = c.recs[mb];
    if (m.epoch != c.epoch) {
      err |= DEC_E_MISSING_MB;
      continue;
    }
    if (m.type == kMbInter || m.type == kMbSkip) {
      full::MbRecon r(c, slot, mb, m);
      r.run();
      err |= r.err;
    }
  }
  __syncthreads();
  // intra macroblocks along the wavefront t = x + 2y
  const int steps = mbw + 2 * (mbh - 1);
  for (int t = 0; t < steps; ++t) {
    for (int y = threadIdx.x; y < mbh; y += kReconThreads) {
      const int x = t - 2 * y;
      if (x < 0 || x >= mbw) continue;
      const MbRec &m = c.recs[y * mbw + x];
      if (m.epoch != c.epoch || m.type == kMbInter || m.type == kMbSkip) continue;
      full::MbRecon r(c, slot, y * mbw + x, m);
      r.run();
      err |= r.err;
    }
    __syncthreads();
  }
  if (err) atomicOr(a.err, err);
}

__global__ void __launch_bounds__(kDeblockThreads) h264_deblock_full(FullReconArgs a) {
  const int slot = a.frames[blockIdx.x].x;
  const full::ReconCtx c = make_ctx(a, slot);
  const int mbw = c.mbw, mbh = c.mbh;
  const int steps = mbw + 2 * (mbh - 1);
  for (int t = 0; t < steps; ++t) {
    for (int y = threadIdx.x; y < mbh; y += kDeblockThreads) {
      const int x = t - 2 * y;
      if (x >= 0 && x < mbw) full::deblock_mb(c, slot, y * mbw + x);
    }
    __syncthreads();
  }
}

}  // namespace

int parse_full_launch(const FullParseArgs &a, hipStream_t s) {
  if (a.n_slices <= 0) return VTS_OK;
  hipLaunchKernelGGL(h264_parse_full, dim3((a.n_slices + kParseLanes - 1) / kParseLanes), dim3(kParseLanes), 0, s, a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(VTS_E_HIP, "h264_parse_full launch: %s", hipGetErrorString(e));
  return VTS_OK;
}

int recon_full_launch(const FullReconArgs &a, int n_frames, hipStream_t s) {
  if (n_frames <= 0) return VTS_OK;
  hipLaunchKernelGGL(h264_recon_full, dim3(n_frames), dim3(kReconThreads), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(VTS_E_HIP, "h264_recon_full launch: %s", hipGetErrorString(e));
  if (a.deblock) {
    hipLaunchKernelGGL(h264_deblock_full, dim3(n_frames), dim3(kDeblockThreads), 0, s, a);
    e = hipGetLastError();
    if (e != hipSuccess) return fail(VTS_E_HIP, "h264_deblock_full launch: %s", hipGetErrorString(e));
  }
  return VTS_OK;
}

}  // namespace vts
