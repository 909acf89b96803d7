// decode.hip — device-side H.264 decode of the supported subset (gfx950).
//
// rocDecode/VCN is not available in this image or on the GPU pool (no
// librocdecode.so, no libva), so the decode that feeds the scorer is done by
// hand-written HIP kernels on the shader array:
//
//   h264_parse      one LANE per slice NAL: slice header + CAVLC macroblock
//                   layer (mb_skip_run, mb_type, mvd, coded_block_pattern,
//                   I_PCM alignment), motion-vector prediction (8.4.1.3,
//                   8.4.1.1).  Slices are independent, so a window of N
//                   frames x S slices runs N*S lanes at once.  Output: one
//                   64-bit command per macroblock (see h264.h MB_PCM/MB_INTER).
//   h264_recon      one WORKGROUP per macroblock row of a frame: turns the
//                   commands into NV12 samples — I_PCM copy (planar Cb/Cr
//                   interleaved into NV12 in registers) or motion-compensated
//                   copy from the reference picture (integer-pel luma, 1/8-pel
//                   bilinear chroma, edge clamping, 8.4.2.2).  Each lane writes
//                   one aligned 16-byte chunk; consecutive lanes write
//                   consecutive chunks of a row.  A launch covers every frame
//                   at the same distance from its IDR (GOP-parallel).
//
// Anything outside the subset sets a bit in a device error word that the
// host checks after every window (DEC_E_* in h264.h) — never a silent skip.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.h"
#include "decode.h"
#include "h264.h"
#include "parse_slice.h"
#include "pixel.h"

namespace vts {
namespace {

#ifndef VTS_PARSE_WAVES
#define VTS_PARSE_WAVES 0
#endif
#if VTS_PARSE_WAVES
#define VTS_PARSE_OCC __attribute__((amdgpu_waves_per_eu(VTS_PARSE_WAVES)))
#else
#define VTS_PARSE_OCC
#endif
// one lane per slice NAL
__global__ void __launch_bounds__(64) VTS_PARSE_OCC h264_parse(ParseArgs a) {
  __shared__ ParseScratch scratch[64];
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.n_slices) return;
  const SliceDesc sd = a.slices[s];
  const uint32_t errs = parse_slice(a.es, sd.nal_offset, sd.nal_size, sd.slot, sd.ref_slot, a.prm, a.cmd,
                                    &scratch[threadIdx.x], a.epoch);
  if (errs) atomicOr(a.err, errs);
}

// --------------------------------------------------------- reconstruction
// 16 bytes at any byte address: two aligned 16-byte loads (both coalesced
// across lanes) and a funnel shift in registers.  Reads up to 15 bytes past
// the 16 requested (buffers carry >= 32 bytes of padding).
__device__ __forceinline__ uint4 load16_any(const uint8_t *p) {
  const int sh = static_cast<int>(reinterpret_cast<uintptr_t>(p) & 15);
  const uint4 *q = reinterpret_cast<const uint4 *>(p - sh);  // stays a global pointer
  const uint4 lo = q[0];
  if (sh == 0) return lo;
  const uint4 hi = q[1];
  const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  const int qd = sh >> 2, r = sh & 3;
  uint32_t s[5];
#pragma unroll
  for (int i = 0; i < 5; ++i)
    s[i] = (qd == 0) ? w[i] : (qd == 1) ? w[i + 1] : (qd == 2) ? w[i + 2] : w[i + 3 < 8 ? i + 3 : 7];
  return make_uint4(__builtin_amdgcn_alignbyte(s[1], s[0], r), __builtin_amdgcn_alignbyte(s[2], s[1], r),
                    __builtin_amdgcn_alignbyte(s[3], s[2], r), __builtin_amdgcn_alignbyte(s[4], s[3], r));
}

__device__ __forceinline__ uint32_t has_zero_byte(uint32_t v) {
  return (v - 0x01010101u) & ~v & 0x80808080u;
}

// Emulation-prevention bytes (00 00 03) whose 03 lies inside the I_PCM sample
// span [pcm, pcm + 384) would make the recorded offsets wrong.  Checked only
// for chunks that contain a zero byte (a pattern needs two zeros).
__device__ bool epb_in_pcm(const uint8_t *chunk, int n, const uint8_t *pcm) {
  for (int j = -2; j < n; ++j) {
    const uint8_t *t = chunk + j;
    if (t + 2 < pcm || t + 2 >= pcm + 384) continue;
    if (t[0] == 0 && t[1] == 0 && t[2] == 3) return true;
  }
  return false;
}

// DEC_E_EPB_IN_PCM if an emulation-prevention byte falls inside the rows
// of group q (kk luma rows, hk chroma rows of each plane) of an I_PCM block.
__device__ __noinline__ uint32_t pcm_rows_epb(const uint8_t *pcm, int q, int kk, int hk) {
  bool bad = false;
  for (int i = 0; i < kk; ++i) bad |= epb_in_pcm(pcm + 16 * (q * kk + i), 16, pcm);
  for (int i = 0; i < hk; ++i)
    bad |= epb_in_pcm(pcm + 256 + 8 * (q * hk + i), 8, pcm) || epb_in_pcm(pcm + 320 + 8 * (q * hk + i), 8, pcm);
  return bad ? DEC_E_EPB_IN_PCM : 0u;
}

// interleave 8 Cb and 8 Cr bytes into 16 NV12 bytes (u0 v0 u1 v1 ...)
__device__ __forceinline__ uint4 interleave_uv(uint32_t u0, uint32_t u1, uint32_t v0, uint32_t v1) {
  // v_perm_b32 selector: bytes of {src0, src1} = {hi word, lo word}
  return make_uint4(__builtin_amdgcn_perm(v0, u0, 0x05010400u), __builtin_amdgcn_perm(v0, u0, 0x07030602u),
                    __builtin_amdgcn_perm(v1, u1, 0x05010400u), __builtin_amdgcn_perm(v1, u1, 0x07030602u));
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

constexpr int kReconThreads = 256;

#ifndef VTS_NT_LOAD
#define VTS_NT_LOAD 0
#endif
#ifndef VTS_NT_STORE
#define VTS_NT_STORE 1
#endif
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 16-byte row load / store of the fused kernel's streams.  Output rows are
// stored nontemporal (3-5% faster per launch, profiles/r01_variants.txt);
// nontemporal reference loads measured 8% slower and stay off.
__device__ __forceinline__ uint4 ld_row(const uint4 *p) {
#if VTS_NT_LOAD
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
#else
  return *p;
#endif
}
__device__ __forceinline__ void st_row(uint8_t *p, const uint4 v) {
#if VTS_NT_STORE
  __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4 *>(p));
#else
  *reinterpret_cast<uint4 *>(p) = v;
#endif
}

struct FrameRefs {
  const uint8_t *es;
  const uint8_t *ref, *ref_uv;  // reference picture (nullptr for none)
  int W, H, CW, CH;
  int64_t pitch;
};

// The 16 output bytes of row r (0..15 luma, 16..23 chroma NV12) of macroblock
// (m, mby) whose command is c.  errs collects DEC_E_* bits.
// General (slow) path: sub-pel chroma, edge clamping, error cases.  Inlined:
// as an out-of-line call it made every wave of the fused kernel set up
// scratch and the whole decode measured 25% slower.
__device__ __forceinline__ uint4 fetch_row(const FrameRefs &F, uint64_t c, int r, int m, int mby,
                                           uint32_t &errs) {
  const uint32_t kind = static_cast<uint32_t>(c >> 62);
  const int mvx = static_cast<int16_t>(c & 0xffff), mvy = static_cast<int16_t>((c >> 16) & 0xffff);
  uint4 out = make_uint4(0, 0, 0, 0);
  if (kind == 0 || (kind == 2 && !F.ref)) {
    errs |= (kind == 0) ? DEC_E_MISSING_MB : DEC_E_NO_REF;
  } else if (r < 16) {
    if (kind == 1) {
      const uint8_t *pcm = F.es + static_cast<int64_t>(c & 0xffffffffffffull);
      const uint8_t *src = pcm + 16 * r;
      out = load16_any(src);
      if ((has_zero_byte(out.x) | has_zero_byte(out.y) | has_zero_byte(out.z) | has_zero_byte(out.w)) &&
          epb_in_pcm(src, 16, pcm))
        errs |= DEC_E_EPB_IN_PCM;
    } else {
      const int sy = clampi(mby * 16 + r + (mvy >> 2), 0, F.H - 1);
      const int sx = m * 16 + (mvx >> 2);
      const uint8_t *row = F.ref + sy * F.pitch;
      if (sx >= 0 && sx + 15 <= F.W - 1) {
        out = load16_any(row + sx);
      } else {
        uint64_t lo8 = 0, hi8 = 0;  // rolled: this path is rare, keep its registers few
#pragma unroll 1
        for (int b = 0; b < 16; ++b) {
          const uint64_t v = row[clampi(sx + b, 0, F.W - 1)];
          if (b < 8) lo8 |= v << (8 * b); else hi8 |= v << (8 * (b - 8));
        }
        out = make_uint4(uint32_t(lo8), uint32_t(lo8 >> 32), uint32_t(hi8), uint32_t(hi8 >> 32));
      }
    }
  } else {
    const int cr = r - 16;
    if (kind == 1) {
      const uint8_t *pcm = F.es + static_cast<int64_t>(c & 0xffffffffffffull);
      const uint4 u = load16_any(pcm + 256 + 8 * cr);  // first 8 bytes used
      const uint4 v = load16_any(pcm + 320 + 8 * cr);
      out = interleave_uv(u.x, u.y, v.x, v.y);
      if ((has_zero_byte(u.x) | has_zero_byte(u.y) | has_zero_byte(v.x) | has_zero_byte(v.y)) &&
          (epb_in_pcm(pcm + 256 + 8 * cr, 8, pcm) || epb_in_pcm(pcm + 320 + 8 * cr, 8, pcm)))
        errs |= DEC_E_EPB_IN_PCM;
    } else {
      const int fx = mvx & 7, fy = mvy & 7;
      const int cx = m * 8 + (mvx >> 3), cy = mby * 8 + cr + (mvy >> 3);
      if (fx == 0 && fy == 0) {
        const uint8_t *row = F.ref_uv + clampi(cy, 0, F.CH - 1) * F.pitch;
        if (cx >= 0 && cx + 7 <= F.CW - 1) {
          out = load16_any(row + 2 * cx);
        } else {
          uint64_t lo8 = 0, hi8 = 0;
#pragma unroll 1
          for (int b = 0; b < 8; ++b) {
            const int sx = clampi(cx + b, 0, F.CW - 1);
            const uint64_t v = uint64_t(row[2 * sx]) | (uint64_t(row[2 * sx + 1]) << 8);
            if (b < 4) lo8 |= v << (16 * b); else hi8 |= v << (16 * (b - 4));
          }
          out = make_uint4(uint32_t(lo8), uint32_t(lo8 >> 32), uint32_t(hi8), uint32_t(hi8 >> 32));
        }
      } else {
        const uint8_t *ra = F.ref_uv + clampi(cy, 0, F.CH - 1) * F.pitch;
        const uint8_t *rb = F.ref_uv + clampi(cy + 1, 0, F.CH - 1) * F.pitch;
        uint64_t lo8 = 0, hi8 = 0;
#pragma unroll 1
        for (int b = 0; b < 8; ++b) {
          const int xa = clampi(cx + b, 0, F.CW - 1), xb = clampi(cx + b + 1, 0, F.CW - 1);
          uint64_t pair = 0;
#pragma unroll
          for (int pl = 0; pl < 2; ++pl) {
            const int A = ra[2 * xa + pl], B = ra[2 * xb + pl], C = rb[2 * xa + pl], D = rb[2 * xb + pl];
            const uint64_t v = static_cast<uint64_t>(
                ((8 - fx) * (8 - fy) * A + fx * (8 - fy) * B + (8 - fx) * fy * C + fx * fy * D + 32) >> 6);
            pair |= v << (8 * pl);
          }
          if (b < 4) lo8 |= pair << (16 * b); else hi8 |= pair << (16 * (b - 4));
        }
        out = make_uint4(uint32_t(lo8), uint32_t(lo8 >> 32), uint32_t(hi8), uint32_t(hi8 >> 32));
      }
    }
  }
  return out;
}

// A command of this run (epoch bits stripped), or 0 (= absent) for one left
// in the ring by an earlier run.
__device__ __forceinline__ uint64_t current_cmd(uint64_t c, uint32_t epoch) {
  return ((c & kCmdEpochMask) >> kCmdEpochShift) == epoch ? (c & ~kCmdEpochMask) : 0;
}

__device__ __forceinline__ FrameRefs frame_refs(const ReconArgs &a, int ref_slot) {
  FrameRefs F;
  F.es = a.es;
  F.W = a.mb_width * 16;
  F.H = a.mb_height * 16;
  F.CW = F.W / 2;
  F.CH = F.H / 2;
  F.pitch = a.pitch;
  F.ref = ref_slot >= 0 ? a.surf + static_cast<int64_t>(ref_slot) * a.frame_stride : nullptr;
  F.ref_uv = F.ref ? F.ref + F.pitch * F.H : nullptr;
  return F;
}

// ---------------------------------------------- fast-path row source
// One output row (16 bytes: luma row rin of the macroblock, or NV12 chroma
// row rin) of an I_PCM or integer-pel-chroma inter macroblock, as a pair of
// aligned loads issued now (issue_row) and a funnel shift done once they land
// (finish_row).  shf = byte shift | mode << 8: mode 1/2 = left/right picture
// edge (the edge-most aligned chunk against the replicated edge sample),
// I_PCM chroma rows are 8-byte pairs of the planar Cb and Cr rows.
__device__ __forceinline__ bool fast_cmd(const FrameRefs &F, uint64_t c) {
  const uint32_t kind = static_cast<uint32_t>(c >> 62);
  const int mvx = static_cast<int16_t>(c & 0xffff), mvy = static_cast<int16_t>((c >> 16) & 0xffff);
  return kind == 1 || (kind == 2 && F.ref && ((mvx | mvy) & 7) == 0);
}

__device__ __forceinline__ void issue_row(const FrameRefs &F, const uint8_t *pcmb, bool pcm, bool chroma,
                                          int rin, int m, int mby, int mvx, int mvy, uint4 &lo, uint4 &hi,
                                          int &shf) {
  if (pcm && chroma) {
    const uint8_t *pu = pcmb + 256 + 8 * rin;  // Cr row is 64 B on
    const int sh = static_cast<int>(reinterpret_cast<uintptr_t>(pu) & 7);
    const uint2 *au = reinterpret_cast<const uint2 *>(pu - sh);
    const uint2 u0 = au[0], u1 = au[1], v0 = au[8], v1 = au[9];
    shf = sh;
    lo = make_uint4(u0.x, u0.y, u1.x, u1.y);
    hi = make_uint4(v0.x, v0.y, v1.x, v1.y);
  } else {
    const uint4 *pa;
    int sh;
    if (pcm) {
      const uint8_t *p = pcmb + 16 * rin;
      sh = static_cast<int>(reinterpret_cast<uintptr_t>(p) & 15);
      pa = reinterpret_cast<const uint4 *>(p - sh);
    } else {
      // row start (16-byte aligned: pitch and W are multiples of 16)
      const uint8_t *row = chroma ? F.ref_uv + clampi(mby * 8 + rin + (mvy >> 3), 0, F.CH - 1) * F.pitch
                                  : F.ref + clampi(mby * 16 + rin + (mvy >> 2), 0, F.H - 1) * F.pitch;
      const int x0 = chroma ? 2 * (m * 8 + (mvx >> 3)) : m * 16 + (mvx >> 2);  // NV12 rows are W bytes
      if (x0 < 0) {                  // left edge: [fill x16][row 0..15]
        pa = reinterpret_cast<const uint4 *>(row);
        sh = (x0 > -16 ? 16 + x0 : 0) | (1 << 8);
      } else if (x0 > F.W - 16) {    // right edge: [row W-16..W-1][fill x16]
        pa = reinterpret_cast<const uint4 *>(row + F.W - 16);
        sh = min(x0 - (F.W - 16), 16) | (2 << 8);
      } else {
        const uint8_t *p = row + x0;
        // pointer arithmetic (not an integer round trip) keeps the global
        // address space, so these are global_load_dwordx4, not flat loads
        sh = static_cast<int>(reinterpret_cast<uintptr_t>(p) & 15);
        pa = reinterpret_cast<const uint4 *>(p - sh);
      }
    }
    shf = sh;
    lo = ld_row(pa);
    hi = ld_row(sh >> 8 ? pa : pa + 1);
  }
}

// zero collects has_zero_byte of I_PCM samples (pcm): any zero byte means a
// possible emulation-prevention pattern, checked exactly by the caller.
__device__ __forceinline__ uint4 finish_row(bool chroma, bool pcm, uint4 lo, uint4 hi, int shf, uint32_t &zero) {
  if (pcm && chroma) {
    const int sh = shf & 7, qd = sh >> 2, r = sh & 3;
    const uint32_t a0 = qd ? lo.y : lo.x, a1 = qd ? lo.z : lo.y, a2 = qd ? lo.w : lo.z;
    const uint32_t b0 = qd ? hi.y : hi.x, b1 = qd ? hi.z : hi.y, b2 = qd ? hi.w : hi.z;
    const uint32_t ux = __builtin_amdgcn_alignbyte(a1, a0, r), uy = __builtin_amdgcn_alignbyte(a2, a1, r);
    const uint32_t vx = __builtin_amdgcn_alignbyte(b1, b0, r), vy = __builtin_amdgcn_alignbyte(b2, b1, r);
    zero |= has_zero_byte(ux) | has_zero_byte(uy) | has_zero_byte(vx) | has_zero_byte(vy);
    return interleave_uv(ux, uy, vx, vy);
  }
  if (!pcm && (shf >> 8)) {
    // replicate the edge sample (a byte for luma, a Cb/Cr pair for NV12)
    if ((shf >> 8) == 1) {
      const uint32_t f = chroma ? (hi.x & 0xffffu) * 0x00010001u : (hi.x & 0xffu) * 0x01010101u;
      lo = make_uint4(f, f, f, f);
    } else {
      const uint32_t g = chroma ? (lo.w >> 16) * 0x00010001u : (lo.w >> 24) * 0x01010101u;
      hi = make_uint4(g, g, g, g);
      if ((shf & 0xff) == 16) lo = hi;
    }
    shf &= 15;
  }
  const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  const int qd = (shf >> 2) & 3, r = shf & 3;
  uint32_t t[5];
#pragma unroll
  for (int j = 0; j < 5; ++j)
    t[j] = (qd == 0) ? w[j] : (qd == 1) ? w[j + 1] : (qd == 2) ? w[j + 2] : w[j + 3 < 8 ? j + 3 : 7];
  const uint4 v = make_uint4(__builtin_amdgcn_alignbyte(t[1], t[0], r), __builtin_amdgcn_alignbyte(t[2], t[1], r),
                             __builtin_amdgcn_alignbyte(t[3], t[2], r), __builtin_amdgcn_alignbyte(t[4], t[3], r));
  if (pcm) zero |= has_zero_byte(v.x) | has_zero_byte(v.y) | has_zero_byte(v.z) | has_zero_byte(v.w);
  return v;
}

// Row source in at most 6 dwords (h264_recon_score6b, whose 9 rows are all
// in flight at once): a 16-byte load at 4-byte alignment plus the dword after
// it (interior and I_PCM luma rows: 5 dwords instead of two aligned 16-byte
// loads' 8), the aligned 16 bytes at a picture edge (4 dwords; the fill comes
// from them), or the Cb and Cr 8-byte runs of an I_PCM chroma row (3 + 3).
// shf = byte shift | mode << 8: 0 funnel, 1 / 2 left / right edge, 3 I_PCM
// chroma.
typedef uint4 uint4_a4 __attribute__((aligned(4)));
typedef uint32_t u32x3_a4 __attribute__((ext_vector_type(3), aligned(4)));
struct Row6 {
  uint32_t w0, w1, w2, w3, w4, w5;
  int shf;
};
__device__ __forceinline__ void issue_row6(const FrameRefs &F, const uint8_t *pcmb, bool pcm, bool chroma, int rin,
                                           int m, int mby, int mvx, int mvy, Row6 &o) {
  if (pcm && chroma) {
    const uint8_t *pu = pcmb + 256 + 8 * rin;  // Cr row is 64 B on
    const int sh = static_cast<int>(reinterpret_cast<uintptr_t>(pu) & 3);
    const u32x3_a4 a = *reinterpret_cast<const u32x3_a4 *>(pu - sh);
    const u32x3_a4 b = *reinterpret_cast<const u32x3_a4 *>(pu + 64 - sh);
    o.w0 = a.x, o.w1 = a.y, o.w2 = a.z, o.w3 = b.x, o.w4 = b.y, o.w5 = b.z;
    o.shf = sh | (3 << 8);
    return;
  }
  const uint8_t *p;
  int mode = 0, esh = 0;
  if (pcm) {
    p = pcmb + 16 * rin;
  } else {
    const uint8_t *row = chroma ? F.ref_uv + clampi(mby * 8 + rin + (mvy >> 3), 0, F.CH - 1) * F.pitch
                                : F.ref + clampi(mby * 16 + rin + (mvy >> 2), 0, F.H - 1) * F.pitch;
    const int x0 = chroma ? 2 * (m * 8 + (mvx >> 3)) : m * 16 + (mvx >> 2);
    if (x0 < 0) {
      p = row;
      mode = 1;
      esh = x0 > -16 ? 16 + x0 : 0;
    } else if (x0 > F.W - 16) {
      p = row + F.W - 16;
      mode = 2;
      esh = min(x0 - (F.W - 16), 16);
    } else {
      p = row + x0;
    }
  }
  if (mode == 0) {
    const int sh = static_cast<int>(reinterpret_cast<uintptr_t>(p) & 3);
    const uint4 v = *reinterpret_cast<const uint4_a4 *>(p - sh);
    o.w0 = v.x, o.w1 = v.y, o.w2 = v.z, o.w3 = v.w;
    o.w4 = *reinterpret_cast<const uint32_t *>(p - sh + 16);
    o.shf = sh;
  } else {
    const uint4 v = *reinterpret_cast<const uint4 *>(p);
    o.w0 = v.x, o.w1 = v.y, o.w2 = v.z, o.w3 = v.w, o.w4 = 0;
    o.shf = esh | (mode << 8);
  }
}
__device__ __forceinline__ uint4 finish_row6(bool chroma, bool pcm, const Row6 &o, uint32_t &zero) {
  const int mode = o.shf >> 8, sh = o.shf & 255;
  if (mode == 3) {
    const uint32_t u0 = __builtin_amdgcn_alignbyte(o.w1, o.w0, sh), u1 = __builtin_amdgcn_alignbyte(o.w2, o.w1, sh);
    const uint32_t v0 = __builtin_amdgcn_alignbyte(o.w4, o.w3, sh), v1 = __builtin_amdgcn_alignbyte(o.w5, o.w4, sh);
    zero |= has_zero_byte(u0) | has_zero_byte(u1) | has_zero_byte(v0) | has_zero_byte(v1);
    return interleave_uv(u0, u1, v0, v1);
  }
  if (mode == 0) {
    const uint4 v = make_uint4(__builtin_amdgcn_alignbyte(o.w1, o.w0, sh), __builtin_amdgcn_alignbyte(o.w2, o.w1, sh),
                               __builtin_amdgcn_alignbyte(o.w3, o.w2, sh), __builtin_amdgcn_alignbyte(o.w4, o.w3, sh));
    if (pcm) zero |= has_zero_byte(v.x) | has_zero_byte(v.y) | has_zero_byte(v.z) | has_zero_byte(v.w);
    return v;
  }
  // picture edge: the 16 bytes at the edge against the replicated edge sample
  // (a byte for luma, a Cb/Cr pair for NV12), bytes [sh, sh + 16) of the pair
  uint32_t w[8];
  if (mode == 1) {
    const uint32_t f = chroma ? (o.w0 & 0xffffu) * 0x00010001u : (o.w0 & 0xffu) * 0x01010101u;
    w[0] = w[1] = w[2] = w[3] = f;
    w[4] = o.w0, w[5] = o.w1, w[6] = o.w2, w[7] = o.w3;
  } else {
    const uint32_t g = chroma ? (o.w3 >> 16) * 0x00010001u : (o.w3 >> 24) * 0x01010101u;
    if (sh >= 16) return make_uint4(g, g, g, g);
    w[0] = o.w0, w[1] = o.w1, w[2] = o.w2, w[3] = o.w3;
    w[4] = w[5] = w[6] = w[7] = g;
  }
  const int qd = (sh >> 2) & 3, r = sh & 3;
  uint32_t t[5];
#pragma unroll
  for (int j = 0; j < 5; ++j)
    t[j] = (qd == 0) ? w[j] : (qd == 1) ? w[j + 1] : (qd == 2) ? w[j + 2] : w[j + 3 < 8 ? j + 3 : 7];
  return make_uint4(__builtin_amdgcn_alignbyte(t[1], t[0], r), __builtin_amdgcn_alignbyte(t[2], t[1], r),
                    __builtin_amdgcn_alignbyte(t[3], t[2], r), __builtin_amdgcn_alignbyte(t[4], t[3], r));
}

// ------------------------------------------------ fused decode + scoring
// h264_recon_score<K>: one LANE per (macroblock, group of rows).  A group is
// the K luma rows + K/2 chroma rows of one thumbnail row (K = 2, 4, 8; K = 0
// = plain reconstruction in groups of 4 + 2 rows, nothing scored).  A
// workgroup of 256 lanes covers 256/Q consecutive macroblocks of one frame
// for all Q groups; lanes of a wave take consecutive macroblocks of the same
// group, so every row load and store instruction covers contiguous bytes.
// Each lane issues all of its row loads before using any (memory-level
// parallelism instead of a serial walk), stores the reconstructed rows and,
// while they are in registers, box-sums them into the thumbnail pixels:
// Y'U'V' -> BT.709 RGB, thumbnail luma for the SAD pass, and an LDS
// histogram flushed once per workgroup with global atomics.  The decoded
// frame is never re-read for scoring.
#ifndef VTS_WAVES_PER_EU
#define VTS_WAVES_PER_EU 0
#endif
#if VTS_WAVES_PER_EU
#define VTS_OCCUPANCY __attribute__((amdgpu_waves_per_eu(K == 8 ? 1 : VTS_WAVES_PER_EU)))
#else
#define VTS_OCCUPANCY
#endif

// XCD-aware block order (cdna_hip_programming.md T1, bijective form):
// blocks are dealt round-robin over the 8 XCDs, so remap them so that each
// XCD walks a contiguous range of tiles.  Horizontally adjacent 64-macroblock
// tiles share the 128-byte lines at their seams (the misaligned second load of
// a motion-shifted row); on one XCD the neighbour finds them in its L2.
// Speed only: any placement is correct.
#ifndef VTS_XCD_SWZ
#define VTS_XCD_SWZ 1
#endif
__device__ __forceinline__ int xcd_block(int b, int n) {
#if VTS_XCD_SWZ
  const int q = n >> 3, r = n & 7, x = b & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
#else
  (void)n;
  return b;
#endif
}

template <int K>
__global__ void __launch_bounds__(kReconThreads) VTS_OCCUPANCY h264_recon_score(FusedArgs fa) {
  constexpr int KK = K ? K : 4;      // rows per group
  constexpr int Q = 16 / KK;         // groups per macroblock
  constexpr int G = 16 / KK;         // thumbnail pixels per group row
  constexpr int HK = KK / 2;         // chroma rows per group
  constexpr int MB_PER_WG = kReconThreads / Q;
  __shared__ uint32_t lds_hist[256];
  const ReconArgs &a = fa.r;
  const int mbw = a.mb_width, mbh = a.mb_height, nmb = mbw * mbh;
  const int bid = xcd_block(blockIdx.x, gridDim.x);
  const int fi = bid / fa.wgs_per_frame;
  const int q = threadIdx.x / MB_PER_WG;
  const int mb = (bid - fi * fa.wgs_per_frame) * MB_PER_WG + (threadIdx.x % MB_PER_WG);
  const int4 fr = a.frames[fi];
  const FrameRefs F = frame_refs(a, fr.y);
  const int64_t gframe = fa.frame0 + fr.x;
  // the command load is in flight across the histogram-clearing barrier
  const uint64_t c = mb < nmb ? current_cmd(a.cmd[static_cast<int64_t>(fr.x) * nmb + mb], a.epoch) : 0;
  // and so is the display predecessor's thumbnail (fused SAD, see below)
  constexpr int GW = K ? (16 / K + 3) / 4 : 1;  // thumbnail words per lane
  uint32_t prevw[GW];
#pragma unroll
  for (int i = 0; i < GW; ++i) prevw[i] = 0;
  if constexpr (K != 0) {
    if (fr.z >= 0 && mb < nmb) {
      const int mby = mb / mbw, m = mb - mby * mbw;
      const uint8_t *pt = fa.thumb + static_cast<int64_t>(fr.z) * fa.w * fa.h +
                          static_cast<int64_t>(mby * Q + q) * fa.w + m * G;
      if constexpr (G >= 4) {
#pragma unroll
        for (int i = 0; i < G / 4; ++i) prevw[i] = reinterpret_cast<const uint32_t *>(pt)[i];
      } else {
        prevw[0] = *reinterpret_cast<const uint16_t *>(pt);
      }
    }
  }
  // I pictures (no reference, so every macroblock is I_PCM): a lane reading
  // its rows straight from the elementary stream touches 64 lines per load
  // instruction (consecutive macroblocks' samples lie 386 bytes apart), which
  // made the I-picture launch 1.6x the time of a P level.  Instead the
  // workgroup copies its macroblocks' 384-byte sample blocks into LDS with
  // consecutive lanes on consecutive 16-byte chunks; each lane then reads its
  // rows from LDS.  K = 4 only (24 KB of LDS: 6 workgroups per CU, above the
  // kernel's register-limited 5).
#ifndef VTS_PCM_STAGE
#define VTS_PCM_STAGE 1
#endif
  constexpr bool kStage = K == 4 && VTS_PCM_STAGE;
  constexpr int kPcmChunks = kStage ? MB_PER_WG * 24 : 1;
  __shared__ uint4 pcm_lds[kPcmChunks];
  __shared__ uint64_t pcm_src[kStage ? MB_PER_WG : 1];
  const bool stage = kStage && fr.y < 0;  // uniform over the workgroup
  if constexpr (kStage) {
    if (stage && q == 0)
      pcm_src[threadIdx.x] = (mb < nmb && (c >> 62) == 1) ? (c & 0xffffffffffffull) : ~0ull;
  }
  if constexpr (K != 0) {
    lds_hist[threadIdx.x] = 0;  // kReconThreads == 256
    __syncthreads();
  }
  if constexpr (kStage) {
    if (stage) {
      // branch-free: both aligned 16-byte loads of every chunk in flight,
      // then one funnel shift each (a missing macroblock reads the stream's
      // first bytes; its command fails in the slow path below)
      constexpr int PER = kPcmChunks / kReconThreads;  // 6 chunks per thread
      uint4 lo[PER], hi[PER];
      int sh[PER];
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int i = threadIdx.x + j * kReconThreads;
        const uint64_t src = pcm_src[i / 24];
        const uint8_t *p = a.es + (src != ~0ull ? src + 16 * (i % 24) : 0);
        sh[j] = static_cast<int>(reinterpret_cast<uintptr_t>(p) & 15);
        const uint4 *pa = reinterpret_cast<const uint4 *>(p - sh[j]);
        lo[j] = pa[0];
        hi[j] = pa[1];
      }
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        uint32_t zero_unused = 0;
        pcm_lds[threadIdx.x + j * kReconThreads] = finish_row(false, false, lo[j], hi[j], sh[j], zero_unused);
      }
      __syncthreads();
    }
  }
  uint32_t errs = 0;
  uint32_t sad = 0;  // this lane's share of the frame's thumbnail SAD
  if (mb < nmb) {
    const int mby = mb / mbw, m = mb - mby * mbw;
    uint8_t *dst = a.surf + static_cast<int64_t>(fr.x) * a.frame_stride;
    uint8_t *dst_uv = dst + F.pitch * F.H;
    uint4 yr[KK], cr[HK];
    const uint32_t kind = static_cast<uint32_t>(c >> 62);
    const int mvx = static_cast<int16_t>(c & 0xffff), mvy = static_cast<int16_t>((c >> 16) & 0xffff);
    const int sx = m * 16 + (mvx >> 2), cx = m * 8 + (mvx >> 3);
    const bool pcm = kind == 1;
    // fast paths: I_PCM, and inter with integer-pel chroma.  Vertical
    // clamping is folded into the row index; horizontal clamping at the
    // picture edges loads the edge-most aligned chunk and funnels it against
    // the replicated edge sample, so edge macroblocks (present in almost
    // every wave) do not fall to the per-byte general path.
    const bool fast = pcm || (kind == 2 && F.ref && ((mvx | mvy) & 7) == 0);
    if (fast) {
      // every aligned load is issued before any is used: 16-byte pairs for
      // luma / NV12 rows, 8-byte pairs of the planar Cb and Cr rows of I_PCM
      const uint8_t *pcmb = F.es + static_cast<int64_t>(c & 0xffffffffffffull);
      uint4 lo[KK + HK], hi[KK + HK];
      int shf[KK + HK];  // funnel shift | edge mode << 8 (1 left, 2 right)
      // LDS-staged I_PCM block (I pictures): luma row r = chunk r, Cb row r =
      // bytes 256 + 8r, Cr row r = 320 + 8r; shift 0, so the finish below
      // passes luma through and interleaves the chroma pairs
      const uint4 *blk = pcm_lds + (threadIdx.x % MB_PER_WG) * 24;
      const bool staged = kStage && stage && pcm;
#pragma unroll
      for (int i = 0; i < KK + HK; ++i) {
        if (staged) {
          shf[i] = 0;
          if (i < KK) {
            lo[i] = hi[i] = blk[q * KK + i];
          } else {
            const int r = q * HK + (i - KK);
            const uint4 u = blk[16 + (r >> 1)], v = blk[20 + (r >> 1)];
            lo[i] = (r & 1) ? make_uint4(u.z, u.w, 0, 0) : make_uint4(u.x, u.y, 0, 0);
            hi[i] = (r & 1) ? make_uint4(v.z, v.w, 0, 0) : make_uint4(v.x, v.y, 0, 0);
          }
        } else if (pcm && i >= KK) {
          const uint8_t *pu = pcmb + 256 + 8 * (q * HK + (i - KK));  // Cr row is 64 B on
          const int sh = static_cast<int>(reinterpret_cast<uintptr_t>(pu) & 7);
          const uint2 *au = reinterpret_cast<const uint2 *>(pu - sh);
          const uint2 u0 = au[0], u1 = au[1], v0 = au[8], v1 = au[9];
          shf[i] = sh;
          lo[i] = make_uint4(u0.x, u0.y, u1.x, u1.y);
          hi[i] = make_uint4(v0.x, v0.y, v1.x, v1.y);
        } else {
          const uint4 *pa;
          int sh;
          if (pcm) {
            const uint8_t *p = pcmb + 16 * (q * KK + i);
            sh = static_cast<int>(reinterpret_cast<uintptr_t>(p) & 15);
            pa = reinterpret_cast<const uint4 *>(p - sh);
          } else {
            // row start (16-byte aligned: pitch and W are multiples of 16)
            const uint8_t *row = i < KK
                ? F.ref + clampi(mby * 16 + q * KK + i + (mvy >> 2), 0, F.H - 1) * F.pitch
                : F.ref_uv + clampi(mby * 8 + q * HK + (i - KK) + (mvy >> 3), 0, F.CH - 1) * F.pitch;
            const int x0 = i < KK ? sx : 2 * cx;  // first wanted byte (NV12 rows are W bytes)
            if (x0 < 0) {                         // left edge: [fill x16][row 0..15]
              pa = reinterpret_cast<const uint4 *>(row);
              sh = (x0 > -16 ? 16 + x0 : 0) | (1 << 8);
            } else if (x0 > F.W - 16) {           // right edge: [row W-16..W-1][fill x16]
              pa = reinterpret_cast<const uint4 *>(row + F.W - 16);
              sh = min(x0 - (F.W - 16), 16) | (2 << 8);
            } else {
              const uint8_t *p = row + x0;
              // pointer arithmetic (not an integer round trip) keeps the global
              // address space, so these are global_load_dwordx4, not flat loads
              sh = static_cast<int>(reinterpret_cast<uintptr_t>(p) & 15);
              pa = reinterpret_cast<const uint4 *>(p - sh);
            }
          }
          shf[i] = sh;
          lo[i] = ld_row(pa);
          hi[i] = ld_row(sh >> 8 ? pa : pa + 1);
        }
      }
#pragma unroll
      for (int i = 0; i < KK + HK; ++i) {
        if (!pcm && (shf[i] >> 8)) {
          // replicate the edge sample (a byte for luma, a Cb/Cr pair for NV12)
          const bool luma = i < KK;
          if ((shf[i] >> 8) == 1) {
            const uint32_t f = luma ? (hi[i].x & 0xffu) * 0x01010101u : (hi[i].x & 0xffffu) * 0x00010001u;
            lo[i] = make_uint4(f, f, f, f);
          } else {
            const uint32_t g = luma ? (lo[i].w >> 24) * 0x01010101u : (lo[i].w >> 16) * 0x00010001u;
            hi[i] = make_uint4(g, g, g, g);
            if ((shf[i] & 0xff) == 16) lo[i] = hi[i];
          }
          shf[i] &= 15;
        }
      }
      uint32_t zero = 0;
#pragma unroll
      for (int i = 0; i < KK + HK; ++i) {
        uint4 v;
        if (pcm && i >= KK) {
          const int qd = shf[i] >> 2, r = shf[i] & 3;
          const uint32_t a0 = qd ? lo[i].y : lo[i].x, a1 = qd ? lo[i].z : lo[i].y, a2 = qd ? lo[i].w : lo[i].z;
          const uint32_t b0 = qd ? hi[i].y : hi[i].x, b1 = qd ? hi[i].z : hi[i].y, b2 = qd ? hi[i].w : hi[i].z;
          const uint32_t ux = __builtin_amdgcn_alignbyte(a1, a0, r), uy = __builtin_amdgcn_alignbyte(a2, a1, r);
          const uint32_t vx = __builtin_amdgcn_alignbyte(b1, b0, r), vy = __builtin_amdgcn_alignbyte(b2, b1, r);
          zero |= has_zero_byte(ux) | has_zero_byte(uy) | has_zero_byte(vx) | has_zero_byte(vy);
          v = interleave_uv(ux, uy, vx, vy);
        } else {
          const uint32_t w[8] = {lo[i].x, lo[i].y, lo[i].z, lo[i].w, hi[i].x, hi[i].y, hi[i].z, hi[i].w};
          const int qd = shf[i] >> 2, r = shf[i] & 3;
          uint32_t t[5];
#pragma unroll
          for (int j = 0; j < 5; ++j)
            t[j] = (qd == 0) ? w[j] : (qd == 1) ? w[j + 1] : (qd == 2) ? w[j + 2] : w[j + 3 < 8 ? j + 3 : 7];
          v = make_uint4(__builtin_amdgcn_alignbyte(t[1], t[0], r), __builtin_amdgcn_alignbyte(t[2], t[1], r),
                         __builtin_amdgcn_alignbyte(t[3], t[2], r), __builtin_amdgcn_alignbyte(t[4], t[3], r));
          if (pcm) zero |= has_zero_byte(v.x) | has_zero_byte(v.y) | has_zero_byte(v.z) | has_zero_byte(v.w);
        }
        if (i < KK) yr[i] = v; else cr[i - KK] = v;
      }
      if (pcm && zero) errs |= pcm_rows_epb(pcmb, q, KK, HK);
    } else {
#pragma unroll
      for (int rr = 0; rr < KK; ++rr) yr[rr] = fetch_row(F, c, q * KK + rr, m, mby, errs);
#pragma unroll
      for (int rr = 0; rr < HK; ++rr) cr[rr] = fetch_row(F, c, 16 + q * HK + rr, m, mby, errs);
    }
#pragma unroll
    for (int rr = 0; rr < KK; ++rr) st_row(dst + (mby * 16 + q * KK + rr) * F.pitch + m * 16, yr[rr]);
#pragma unroll
    for (int rr = 0; rr < HK; ++rr) st_row(dst_uv + (mby * 8 + q * HK + rr) * F.pitch + m * 16, cr[rr]);
    if constexpr (K != 0) {
      uint32_t ys[G], us[G], vs[G];
#pragma unroll
      for (int p = 0; p < G; ++p) ys[p] = us[p] = vs[p] = 0;
#pragma unroll
      for (int rr = 0; rr < K; ++rr) add_luma16<K>(yr[rr], ys);
#pragma unroll
      for (int rr = 0; rr < HK; ++rr) add_chroma16<K>(cr[rr], us, vs);
      uint32_t rgb24[G], packed[(G + 3) / 4];
#pragma unroll
      for (int i = 0; i < (G + 3) / 4; ++i) packed[i] = 0;
#pragma unroll
      for (int p = 0; p < G; ++p) {
        const uint32_t y = (ys[p] + K * K / 2) / (K * K);
        const uint32_t u = (us[p] + HK * HK / 2) / (HK * HK);
        const uint32_t v = (vs[p] + HK * HK / 2) / (HK * HK);
        rgb24[p] = bt709_rgb24(y, u, v);
        packed[p / 4] |= y << (8 * (p & 3));
        atomicAdd(&lds_hist[y], 1u);
      }
      const int64_t tpx = static_cast<int64_t>(mby * Q + q) * fa.w + m * G;
      store_rgb<G>(fa.rgb + (gframe * fa.w * fa.h + tpx) * 3, rgb24);
      const int64_t npx = static_cast<int64_t>(fa.w) * fa.h;
      uint8_t *thumb = fa.thumb + static_cast<int64_t>(fr.x) * npx + tpx;
      if constexpr (G >= 4) {
#pragma unroll
        for (int i = 0; i < G / 4; ++i) reinterpret_cast<uint32_t *>(thumb)[i] = packed[i];
      } else {
        *reinterpret_cast<uint16_t *>(thumb) = static_cast<uint16_t>(packed[0]);
      }
      // SAD against the display predecessor's thumbnail (made one or more
      // levels earlier); GOP starts are left to the thumb_sad pass
      if (fr.z >= 0) {
#pragma unroll
        for (int i = 0; i < GW; ++i) sad = sad_u8(packed[i], prevw[i], sad);
      }
    }
  }
  if constexpr (K != 0) {
    if (fr.z >= 0) {  // workgroup SAD -> one 64-bit atomic
      __shared__ uint32_t red[kReconThreads / 64];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) sad += __shfl_xor(sad, off, 64);
      if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sad;
      __syncthreads();
      if (threadIdx.x == 0) {
        uint64_t t = 0;
#pragma unroll
        for (int i = 0; i < kReconThreads / 64; ++i) t += red[i];
        atomicAdd(reinterpret_cast<unsigned long long *>(fa.sad + gframe), static_cast<unsigned long long>(t));
      }
    }
  }
  if constexpr (K != 0) {
    __syncthreads();
    // two bins per 64-bit atomic (a frame's bin total stays below 2^32, so
    // the low count never carries into the high one): half the L2 atomics
    if (threadIdx.x < 128) {
      const uint64_t lo = lds_hist[2 * threadIdx.x], hi = lds_hist[2 * threadIdx.x + 1];
      if (lo | hi)
        atomicAdd(reinterpret_cast<unsigned long long *>(fa.hist + gframe * 256) + threadIdx.x,
                  static_cast<unsigned long long>(lo | (hi << 32)));
    }
  }
  if (errs) atomicOr(a.err, errs);
}

// h264_recon_score6b: the k = 6 kernel with one WAVE per (thumbnail band,
// 63 consecutive macroblock columns).  A band is 6 luma + 3 chroma rows, so
// it spans at most two macroblock rows (two commands); lanes of a wave take
// consecutive macroblocks, so every row load and store instruction covers
// 63 x 16 contiguous bytes, as in the k = 4 kernel.  A 48-column triple of
// macroblocks holds 8 thumbnail pixels: the lane of its first macroblock owns
// pixels 0-2, the second 3-5, the third 6-7; the two pixels that straddle a
// macroblock edge get the neighbour's partial sum through one shuffle (63 =
// 21 triples per wave, so no triple crosses a wave).  No LDS partial sums, no
// LDS atomics except the histogram.  4 waves (4 bands) per workgroup.
constexpr int kK6bCols = 63;
constexpr int kK6bPx = kK6bCols * 16 / 6;  // thumbnail pixels per wave segment (168)

// DEC_E_EPB_IN_PCM if an emulation-prevention byte falls in row `rin` of an
// I_PCM block (a luma row, or the Cb and Cr rows of chroma row rin)
__device__ __noinline__ uint32_t pcm_row_epb(const uint8_t *pcm, bool chroma, int rin) {
  const bool bad = chroma ? (epb_in_pcm(pcm + 256 + 8 * rin, 8, pcm) || epb_in_pcm(pcm + 320 + 8 * rin, 8, pcm))
                          : epb_in_pcm(pcm + 16 * rin, 16, pcm);
  return bad ? DEC_E_EPB_IN_PCM : 0u;
}

__device__ __forceinline__ uint32_t byte_mask(int lo, int hi, int w) {
  // bytes [lo, hi) of a 16-byte chunk that fall in its 32-bit word w
  const int a = min(max(lo - 4 * w, 0), 4), b = min(max(hi - 4 * w, 0), 4);
  const uint32_t upto_b = b >= 4 ? 0xffffffffu : ((1u << (8 * b)) - 1u);
  const uint32_t upto_a = a >= 4 ? 0xffffffffu : ((1u << (8 * a)) - 1u);
  return upto_b & ~upto_a;
}

// add row i of a band (0..5 luma, 6..8 NV12 chroma) into the lane's segment
// box sums: [0] = the left partial [0, b0), [1..3] = the owned pixels
__device__ __forceinline__ void k6_acc_row(int i, int b0, const uint4 row, uint32_t (&ys)[4], uint32_t (&us)[4],
                                           uint32_t (&vs)[4]) {
#pragma unroll
  for (int sgm = 0; sgm < 4; ++sgm) {
    const int lo_b = sgm == 0 ? 0 : b0 + 6 * (sgm - 1);
    const int hi_b = sgm == 0 ? b0 : min(lo_b + 6, 16);
    if (hi_b <= lo_b) continue;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint32_t mk = byte_mask(lo_b, hi_b, w);
      const uint32_t word = w == 0 ? row.x : (w == 1 ? row.y : (w == 2 ? row.z : row.w));
      if (i < 6) {
        ys[sgm] = sad_u8(word & mk, 0u, ys[sgm]);
      } else {
        us[sgm] = sad_u8(word & mk & 0x00ff00ffu, 0u, us[sgm]);
        vs[sgm] = sad_u8(word & mk & 0xff00ff00u, 0u, vs[sgm]);
      }
    }
  }
}
__global__ void __launch_bounds__(256) h264_recon_score6b(FusedArgs fa) {
  constexpr int K = 6, HK = 3;
  __shared__ uint32_t lds_hist[256];
  __shared__ uint32_t red[4];
  __shared__ __attribute__((aligned(16))) uint8_t stage_rgb[4][3 * kK6bPx], stage_th[4][kK6bPx];
  const ReconArgs &a = fa.r;
  const int mbw = a.mb_width, nmb = mbw * a.mb_height;
  const int segs = (mbw + kK6bCols - 1) / kK6bCols;
  const int bid = xcd_block(blockIdx.x, gridDim.x);
  const int fi = bid / fa.wgs_per_frame;
  const int wb = bid - fi * fa.wgs_per_frame;
  const int seg = wb % segs, bg = wb / segs;
  const int lane = threadIdx.x & 63, band = bg * 4 + (threadIdx.x >> 6);
  const int m = seg * kK6bCols + lane;
  const int4 fr = a.frames[fi];
  const FrameRefs F = frame_refs(a, fr.y);
  const int64_t gframe = fa.frame0 + fr.x;
  const int64_t npx = static_cast<int64_t>(fa.w) * fa.h;
  const int r0 = K * band;                                 // first luma row of the band
  const bool active = lane < kK6bCols && m < mbw && r0 < F.H;
  const int mby0 = r0 >> 4, mby1 = min(r0 + K - 1, F.H - 1) >> 4;
  uint64_t c0 = 0, c1 = 0;
  if (active) {
    const uint64_t *cm = a.cmd + static_cast<int64_t>(fr.x) * nmb + m;
    c0 = current_cmd(cm[static_cast<int64_t>(mby0) * mbw], a.epoch);
    c1 = mby1 == mby0 ? c0 : current_cmd(cm[static_cast<int64_t>(mby1) * mbw], a.epoch);
  }
  // owned thumbnail pixels (see above) and the predecessor's bytes, early
  const int j = lane % 3;
  const int pix0 = (m / 3) * 8 + (j == 0 ? 0 : (j == 1 ? 3 : 6));
  const int nown = j == 2 ? 2 : 3;
  const bool scored = active && band < fa.h;
  uint32_t prevb[3] = {0, 0, 0};
  if (scored && fr.z >= 0) {
    const uint8_t *pt = fa.thumb + static_cast<int64_t>(fr.z) * npx + static_cast<int64_t>(band) * fa.w;
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (i < nown && pix0 + i < fa.w) prevb[i] = pt[pix0 + i];
  }
  lds_hist[threadIdx.x] = 0;
  __syncthreads();
  uint32_t errs = 0;
  uint4 rows[K + HK];  // 6 luma rows, then 3 NV12 chroma rows
  uint32_t ys[4] = {0, 0, 0, 0}, us[4] = {0, 0, 0, 0}, vs[4] = {0, 0, 0, 0};  // box sums, [0] = left partial
  const int b0 = j == 0 ? 0 : (j == 1 ? 2 : 4);  // end of the left partial = start of pixel 1
  bool summed = false;
  if (active) {
    uint8_t *dst = a.surf + static_cast<int64_t>(fr.x) * a.frame_stride;
    uint8_t *dst_uv = dst + F.pitch * F.H;
    if (fast_cmd(F, c0) && fast_cmd(F, c1)) {
      Row6 src[K + HK];  // <= 6 dwords per row in flight (48 VGPRs for the 9 rows, not 72)
#pragma unroll
      for (int i = 0; i < K + HK; ++i) {
        const bool chroma = i >= K;
        const int r = chroma ? HK * band + (i - K) : r0 + i;  // luma row / chroma row
        const int mbr = chroma ? r >> 3 : r >> 4;
        const uint64_t c = mbr == mby0 ? c0 : c1;
        const bool pcm = (c >> 62) == 1;
        const uint8_t *pcmb = F.es + static_cast<int64_t>(c & 0xffffffffffffull);
        const int mvx = static_cast<int16_t>(c & 0xffff), mvy = static_cast<int16_t>((c >> 16) & 0xffff);
        if (r < (chroma ? F.CH : F.H)) {
          issue_row6(F, pcmb, pcm, chroma, chroma ? (r & 7) : (r & 15), m, mbr, mvx, mvy, src[i]);
        } else {
          src[i].w0 = src[i].w1 = src[i].w2 = src[i].w3 = src[i].w4 = src[i].w5 = 0;
          src[i].shf = 0;
        }
      }
      uint32_t zero = 0;
#pragma unroll
      for (int i = 0; i < K + HK; ++i) {
        const bool chroma = i >= K;
        const int r = chroma ? HK * band + (i - K) : r0 + i;
        const uint64_t c = (chroma ? r >> 3 : r >> 4) == mby0 ? c0 : c1;
        const uint4 row = finish_row6(chroma, (c >> 62) == 1, src[i], zero);
        if (r < (chroma ? F.CH : F.H)) st_row((chroma ? dst_uv : dst) + static_cast<int64_t>(r) * F.pitch + m * 16, row);
        if (scored) k6_acc_row(i, b0, row, ys, us, vs);
      }
      summed = true;
      if (zero) {  // a zero byte in I_PCM samples: check for emulation prevention exactly
        for (int i = 0; i < K + HK; ++i) {
          const bool chroma = i >= K;
          const int r = chroma ? HK * band + (i - K) : r0 + i;
          const uint64_t c = (chroma ? r >> 3 : r >> 4) == mby0 ? c0 : c1;
          if ((c >> 62) == 1 && r < (chroma ? F.CH : F.H))
            errs |= pcm_row_epb(F.es + static_cast<int64_t>(c & 0xffffffffffffull), chroma, chroma ? (r & 7) : (r & 15));
        }
      }
    } else {
      // general path (sub-pel chroma, errors): rare; one row at a time,
      // stored, then read back for scoring (no runtime-indexed register array)
#pragma unroll 1
      for (int i = 0; i < K + HK; ++i) {
        const bool chroma = i >= K;
        const int r = chroma ? HK * band + (i - K) : r0 + i;
        const int mbr = chroma ? r >> 3 : r >> 4;
        if (r < (chroma ? F.CH : F.H))
          *reinterpret_cast<uint4 *>((chroma ? dst_uv : dst) + static_cast<int64_t>(r) * F.pitch + m * 16) =
              fetch_row(F, mbr == mby0 ? c0 : c1, chroma ? 16 + (r & 7) : (r & 15), m, mbr, errs);
      }
#pragma unroll
      for (int i = 0; i < K + HK; ++i) {
        const bool chroma = i >= K;
        const int r = chroma ? HK * band + (i - K) : r0 + i;
        rows[i] = r < (chroma ? F.CH : F.H)
                      ? *reinterpret_cast<const uint4 *>((chroma ? dst_uv : dst) + static_cast<int64_t>(r) * F.pitch + m * 16)
                      : make_uint4(0, 0, 0, 0);
      }
    }
  }
  // box sums: the left partial (bytes owed to the previous lane's last pixel)
  // and the owned pixels' segments, luma over 6 rows, Cb / Cr over 3
  if (scored && !summed) {
#pragma unroll
    for (int sgm = 0; sgm < 4; ++sgm) {
      // segment sgm: 0 = [0, b0), 1.. = owned pixels [b0 + 6 (sgm-1), +6) clipped to 16
      const int lo_b = sgm == 0 ? 0 : b0 + 6 * (sgm - 1);
      const int hi_b = sgm == 0 ? b0 : min(lo_b + 6, 16);
      if (hi_b <= lo_b) continue;
      uint32_t y = 0, u = 0, v = 0;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const uint32_t mk = byte_mask(lo_b, hi_b, w);
#pragma unroll
        for (int i = 0; i < K; ++i) {
          const uint32_t word = w == 0 ? rows[i].x : (w == 1 ? rows[i].y : (w == 2 ? rows[i].z : rows[i].w));
          y = sad_u8(word & mk, 0u, y);
        }
#pragma unroll
        for (int i = K; i < K + HK; ++i) {
          const uint32_t word = w == 0 ? rows[i].x : (w == 1 ? rows[i].y : (w == 2 ? rows[i].z : rows[i].w));
          u = sad_u8(word & mk & 0x00ff00ffu, 0u, u);
          v = sad_u8(word & mk & 0xff00ff00u, 0u, v);
        }
      }
      ys[sgm] = y;
      us[sgm] = u;
      vs[sgm] = v;
    }
  }
  // the next lane's left partial completes this lane's last pixel
  const uint32_t yn = __shfl_down(ys[0], 1, 64), un = __shfl_down(us[0], 1, 64), vn = __shfl_down(vs[0], 1, 64);
  uint32_t sad = 0;
  if (scored) {
    if (j != 2) {
      ys[3] += yn;
      us[3] += un;
      vs[3] += vn;
    }
    // the wave's RGB / thumbnail bytes go through LDS and leave as dwords
    uint8_t *rgb = stage_rgb[threadIdx.x >> 6] + 3 * (pix0 - kK6bPx * seg);
    uint8_t *thumb = stage_th[threadIdx.x >> 6] + (pix0 - kK6bPx * seg);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (i >= nown || pix0 + i >= fa.w) continue;
      const uint32_t y = (ys[1 + i] + K * K / 2) / (K * K);
      const uint32_t u = (us[1 + i] + HK * HK / 2) / (HK * HK), v = (vs[1 + i] + HK * HK / 2) / (HK * HK);
      const uint32_t c24 = bt709_rgb24(y, u, v);
      rgb[3 * i] = static_cast<uint8_t>(c24);
      rgb[3 * i + 1] = static_cast<uint8_t>(c24 >> 8);
      rgb[3 * i + 2] = static_cast<uint8_t>(c24 >> 16);
      thumb[i] = static_cast<uint8_t>(y);
      atomicAdd(&lds_hist[y], 1u);
      if (fr.z >= 0) sad += y > prevb[i] ? y - prevb[i] : prevb[i] - y;
    }
  }
  if (fr.z >= 0) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) sad += __shfl_xor(sad, off, 64);
    if (lane == 0) red[threadIdx.x >> 6] = sad;
  }
  __syncthreads();
  if (band < fa.h && r0 < F.H) {
    // this wave's segment: pixels [kK6bPx * seg, + np) of thumbnail row `band`
    // (w % 8 == 0, so every row and segment starts on a dword)
    const int np = max(0, min(kK6bPx, fa.w - kK6bPx * seg));
    const int64_t tpx = static_cast<int64_t>(band) * fa.w + kK6bPx * seg;
    const uint32_t *srgb = reinterpret_cast<const uint32_t *>(stage_rgb[threadIdx.x >> 6]);
    const uint32_t *sth = reinterpret_cast<const uint32_t *>(stage_th[threadIdx.x >> 6]);
    uint32_t *grgb = reinterpret_cast<uint32_t *>(fa.rgb + (gframe * npx + tpx) * 3);
    uint32_t *gth = reinterpret_cast<uint32_t *>(fa.thumb + static_cast<int64_t>(fr.x) * npx + tpx);
    for (int d = lane; d < 3 * np / 4; d += 64) grgb[d] = srgb[d];
    if (lane < np / 4) gth[lane] = sth[lane];
  }
  if (fr.z >= 0 && threadIdx.x == 0) {
    const uint64_t t = uint64_t(red[0]) + red[1] + red[2] + red[3];
    if (t) atomicAdd(reinterpret_cast<unsigned long long *>(fa.sad + gframe), static_cast<unsigned long long>(t));
  }
  if (threadIdx.x < 128) {
    const uint64_t lo = lds_hist[2 * threadIdx.x], hi = lds_hist[2 * threadIdx.x + 1];
    if (lo | hi)
      atomicAdd(reinterpret_cast<unsigned long long *>(fa.hist + gframe * 256) + threadIdx.x,
                static_cast<unsigned long long>(lo | (hi << 32)));
  }
  if (errs) atomicOr(a.err, errs);
}

// SAD of each frame's thumbnail luma against its predecessor's (the previous
// window's last thumbnail for the window's first frame) and the score.  One
// workgroup per frame; 16-byte loads, all of a thread's loads issued before
// the SAD (a 320x180 thumbnail is 3 600 uint4 = 14 per thread).
__global__ void __launch_bounds__(256) thumb_sad(ThumbSadArgs t) {
  const int64_t f = t.list ? t.list[blockIdx.x] : blockIdx.x;  // window slot
  const int64_t npx = static_cast<int64_t>(t.w) * t.h;
  const uint8_t *cur = t.thumb + f * npx;
  const uint8_t *prev = f > 0 ? t.thumb + (f - 1) * npx : t.prev_luma;
  const int64_t gf = t.frame0 + f;
  const bool vec = (npx & 15) == 0;  // thumbnail rows are 16-byte aligned in the ring
  if (f == t.n_frames - 1 && t.last_luma) {
    for (int64_t i = threadIdx.x; i < npx / 4; i += blockDim.x)
      reinterpret_cast<uint32_t *>(t.last_luma)[i] = reinterpret_cast<const uint32_t *>(cur)[i];
  }
  if (!prev) {
    if (threadIdx.x == 0) {
      t.sad[gf] = 0;
      t.score[gf] = 0.0f;
    }
    return;
  }
  uint32_t s = 0;
  if (vec) {
    const uint4 *c4 = reinterpret_cast<const uint4 *>(cur), *p4 = reinterpret_cast<const uint4 *>(prev);
    const int64_t n4 = npx / 16;
    constexpr int U = 8;
    for (int64_t i0 = threadIdx.x; i0 < n4; i0 += U * blockDim.x) {
      uint4 a[U], b[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + static_cast<int64_t>(u) * blockDim.x;
        a[u] = i < n4 ? c4[i] : make_uint4(0, 0, 0, 0);
        b[u] = i < n4 ? p4[i] : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        s = sad_u8(a[u].x, b[u].x, s);
        s = sad_u8(a[u].y, b[u].y, s);
        s = sad_u8(a[u].z, b[u].z, s);
        s = sad_u8(a[u].w, b[u].w, s);
      }
    }
  } else {
    for (int64_t i = threadIdx.x; i < npx / 4; i += blockDim.x)
      s = sad_u8(reinterpret_cast<const uint32_t *>(cur)[i], reinterpret_cast<const uint32_t *>(prev)[i], s);
  }
  __shared__ uint32_t red[4];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t total = uint64_t(red[0]) + red[1] + red[2] + red[3];
    t.sad[gf] = total;
    t.score[gf] = static_cast<float>(static_cast<double>(total) / (static_cast<double>(npx) * 255.0));
  }
}

__global__ void __launch_bounds__(256) sad_score(const uint64_t *sad, float *score, int64_t frame0,
                                                int64_t n, double denom) {
  const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (i < n) score[frame0 + i] = static_cast<float>(static_cast<double>(sad[frame0 + i]) / denom);
}

// Zero the fused kernel's per-frame accumulators (256-bin histogram, SAD) of
// a window: 16-byte stores, one per thread (hipMemsetAsync ran this as a
// 256-workgroup fill at ~40 GB/s, 0.5 ms per 10-min 720p window, holding CUs
// while the parser ran).
__global__ void __launch_bounds__(256) clear_accum(uint4 *hist, uint64_t *sad, int64_t n) {
  const int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (i < n * 64) hist[i] = make_uint4(0, 0, 0, 0);
  if (i < n) sad[i] = 0;
}

// ------------------------------------- level-blocked decode + scoring (k = 4)
// h264_recon_score_tb: one workgroup per (GOP chain, macroblock row "band")
// decodes L consecutive GOP levels of that band without sending the levels
// between the first and the last through HBM.  Every frame at level l >= 1 is
// predicted from the frame at level l-1 only, with motion of at most one
// 4-row halo group per level vertically (checked per macroblock; see
// DEC_W_LEVEL_RANGE), so level j of the band needs level j-1 over the band
// widened by one group on each side.  The workgroup therefore reconstructs
// level 0 over the band +- (L-1) groups (full picture width: horizontal
// motion and edge clamping need no halo), from the HBM reference or the
// I_PCM samples, into LDS; each following level over one group less on each
// side, read from and written back to the same LDS rows (all reads of a
// level land in registers before a barrier, then the writes); the last level
// covers the band only.  The band rows of every level are scored exactly as
// h264_recon_score<4> scores them (RGB, thumbnail luma, LDS histogram,
// SAD against the previous level's thumbnail, which the lane still holds).
// HBM traffic per L frames: one reference read + one frame write + the
// scoring outputs, instead of L of each; the halo rows are recomputed
// (1.75x the reconstruction ALU work at L = 4), not re-read.
constexpr int kTbThreads = 512;
constexpr int kTbSlots = 2;  // tasks (macroblock, group) per lane and level
constexpr int kTbHalo = 1;   // halo groups per level: 4 luma / 2 chroma rows

// 16 bytes of an LDS row at byte x0 (any alignment; horizontal clamping at
// the picture edges as issue_row / finish_row do it for HBM rows)
__device__ __forceinline__ uint4 tb_lds_row(const uint8_t *row, int x0, int W, bool chroma) {
  const uint4 *pa;
  int sh;
  if (x0 < 0) {
    pa = reinterpret_cast<const uint4 *>(row);
    sh = (x0 > -16 ? 16 + x0 : 0) | (1 << 8);
  } else if (x0 > W - 16) {
    pa = reinterpret_cast<const uint4 *>(row + W - 16);
    sh = min(x0 - (W - 16), 16) | (2 << 8);
  } else {
    sh = x0 & 15;
    pa = reinterpret_cast<const uint4 *>(row + (x0 - sh));
  }
  const uint4 lo = pa[0];
  const uint4 hi = (sh > 0 && sh < 16) ? pa[1] : lo;  // edges (sh >= 256) use lo only
  uint32_t zero_unused = 0;
  return finish_row(chroma, false, lo, hi, sh, zero_unused);
}

// sub-pel chroma (bilinear eighth-pel) of 8 Cb/Cr pairs from two LDS rows:
// fetch_row's general path (rolled: rare, kept small).
__device__ __forceinline__ uint4 tb_subpel(const uint8_t *ra, const uint8_t *rb, int cx, int fx, int fy, int CW) {
  uint64_t lo8 = 0, hi8 = 0;
#pragma unroll 1
  for (int b = 0; b < 8; ++b) {
    const int xa = clampi(cx + b, 0, CW - 1), xb = clampi(cx + b + 1, 0, CW - 1);
    uint64_t pair = 0;
#pragma unroll
    for (int pl = 0; pl < 2; ++pl) {
      const int A = ra[2 * xa + pl], B = ra[2 * xb + pl], C = rb[2 * xa + pl], D = rb[2 * xb + pl];
      const uint64_t v = static_cast<uint64_t>(
          ((8 - fx) * (8 - fy) * A + fx * (8 - fy) * B + (8 - fx) * fy * C + fx * fy * D + 32) >> 6);
      pair |= v << (8 * pl);
    }
    if (b < 4) lo8 |= pair << (16 * b); else hi8 |= pair << (16 * (b - 4));
  }
  return make_uint4(uint32_t(lo8), uint32_t(lo8 >> 32), uint32_t(hi8), uint32_t(hi8 >> 32));
}

// Same from the previous level held in LDS: luma rows [ly0, ly0 + nl) at
// lds + (y - ly0) W, chroma rows from cy0 at lds + nl W + (cy - cy0) W, of
// which rows [vy0, vy1) / [vc0, vc1) are valid.  A reference row outside them
// sets `range` (the launch's halo is too small for this motion).
__device__ __forceinline__ void tb_group_lds(const uint8_t *lds, int ly0, int cy0, int nl, int W, int H, int vy0,
                                             int vy1, int vc0, int vc1, const uint8_t *es, uint64_t c, int m,
                                             int g, bool has_ref, uint4 *rows, uint32_t &errs, uint32_t &range) {
  const int q = g & 3;
  const uint32_t kind = static_cast<uint32_t>(c >> 62);
  if (kind == 1) {
    FrameRefs F{};
    const uint8_t *pcmb = es + static_cast<int64_t>(c & 0xffffffffffffull);
    uint4 lo[6], hi[6];
    int shf[6];
#pragma unroll
    for (int i = 0; i < 6; ++i)
      issue_row(F, pcmb, true, i >= 4, i < 4 ? 4 * q + i : 2 * q + (i - 4), m, 0, 0, 0, lo[i], hi[i], shf[i]);
    uint32_t zero = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i) rows[i] = finish_row(i >= 4, true, lo[i], hi[i], shf[i], zero);
    if (zero) errs |= pcm_rows_epb(pcmb, q, 4, 2);
    return;
  }
  if (kind != 2 || !has_ref) {
    errs |= kind != 2 ? DEC_E_MISSING_MB : DEC_E_NO_REF;
#pragma unroll
    for (int i = 0; i < 6; ++i) rows[i] = make_uint4(0, 0, 0, 0);
    return;
  }
  const int mvx = static_cast<int16_t>(c & 0xffff), mvy = static_cast<int16_t>((c >> 16) & 0xffff);
  const int x0 = m * 16 + (mvx >> 2);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int sy = clampi(4 * g + r + (mvy >> 2), 0, H - 1);
    if (sy < vy0 || sy >= vy1) {
      range = 1;
      rows[r] = make_uint4(0, 0, 0, 0);
    } else {
      rows[r] = tb_lds_row(lds + (sy - ly0) * W, x0, W, false);
    }
  }
  const int CH = H >> 1, CW = W >> 1;
  const int fx = mvx & 7, fy = mvy & 7;
  const uint8_t *uv = lds + nl * W;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int cy = 2 * g + r + (mvy >> 3);
    const int ya = clampi(cy, 0, CH - 1), yb = fy ? clampi(cy + 1, 0, CH - 1) : ya;
    if (ya < vc0 || ya >= vc1 || yb < vc0 || yb >= vc1) {
      range = 1;
      rows[4 + r] = make_uint4(0, 0, 0, 0);
      continue;
    }
    const uint8_t *ra = uv + (ya - cy0) * W, *rb = uv + (yb - cy0) * W;
    const int cx = m * 8 + (mvx >> 3);
    if ((fx | fy) == 0) {
      rows[4 + r] = tb_lds_row(ra, 2 * cx, W, true);
    } else {
      rows[4 + r] = tb_subpel(ra, rb, cx, fx, fy, CW);
    }
  }
}

#ifndef VTS_TB_WAVES
#define VTS_TB_WAVES 2  // 4 spills (336 B/lane) and measured 1.4x slower
#endif
#ifndef VTS_TB1_WAVES
#define VTS_TB1_WAVES 4
#endif
// S = task slots per lane (1: every level's tasks fit 512 lanes, e.g. L <= 2
// at 720p; 2: up to 1024 tasks)
template <int S>
__global__ void __launch_bounds__(kTbThreads) __attribute__((amdgpu_waves_per_eu(S == 1 ? VTS_TB1_WAVES : VTS_TB_WAVES)))
h264_recon_score_tb(TbArgs ta) {
  extern __shared__ uint4 tb_dyn[];
  __shared__ uint32_t lds_hist[256];
  __shared__ uint32_t red[kTbThreads / 64];
  const FusedArgs &fa = ta.f;
  const ReconArgs &a = fa.r;
  const int mbw = a.mb_width, mbh = a.mb_height, nmb = mbw * mbh;
  const int W = mbw * 16, H = mbh * 16, NG = 4 * mbh;
  const int bid = xcd_block(blockIdx.x, gridDim.x);
  const int chain = bid / mbh, band = bid - chain * mbh;
  const int4 *ch = ta.chains + static_cast<int64_t>(chain) * ta.L;
  int n = 0;
  for (int j = 0; j < ta.L; ++j) n += ch[j].x >= 0 ? 1 : 0;  // valid prefix (host-built)
  // LDS region: the band +- n halo groups (level 0's reference rows); level
  // j is rebuilt in place over the band +- (n-1-j) groups
  const int h0 = n * kTbHalo;
  const int r_lo = max(0, 4 * band - h0), r_hi = min(NG, 4 * band + 4 + h0);
  const int ly0 = 4 * r_lo, cy0 = 2 * r_lo, nl = 4 * (r_hi - r_lo);
  uint8_t *lds = reinterpret_cast<uint8_t *>(tb_dyn);
  const int nb = 4 * mbw;  // band tasks: lanes [0, nb), slot 0, the same at every level
  const int64_t npx = static_cast<int64_t>(fa.w) * fa.h;
  const bool band_lane = static_cast<int>(threadIdx.x) < nb;
  const int bg = 4 * band + static_cast<int>(threadIdx.x) / mbw, bm = static_cast<int>(threadIdx.x) % mbw;
  uint32_t errs = 0, range = 0;
  uint32_t prevw = 0;  // this lane's 4 thumbnail luma bytes of the previous level
  const int4 f0 = ch[0];
  if (band_lane && f0.z >= 0)
    prevw = *reinterpret_cast<const uint32_t *>(fa.thumb + f0.z * npx + static_cast<int64_t>(bg) * fa.w + bm * 4);
  // the task of slot s at level jj: band groups first (lanes keep their band
  // task at every level), then the top and bottom halo groups; and its
  // command, loaded one level ahead so its latency hides behind a level
  auto task = [&](int jj, int s, int &g, int &m) {
    const int h = (n - 1 - jj) * kTbHalo;
    const int g_lo = max(0, 4 * band - h), g_hi = min(NG, 4 * band + 4 + h);
    const int ntask = (g_hi - g_lo) * mbw, top = (4 * band - g_lo) * mbw;
    const int t = static_cast<int>(threadIdx.x) + s * kTbThreads;
    g = -1;
    m = 0;
    if (s < S && t < ntask) {
      if (t < nb) {
        g = 4 * band + t / mbw;
        m = t - (t / mbw) * mbw;
      } else {
        const int u = t - nb;
        const int base = u < top ? g_lo : 4 * band + 4 - top / mbw;
        g = base + u / mbw;
        m = u - (u / mbw) * mbw;
      }
    }
  };
  auto command = [&](int jj, int g, int m) -> uint64_t {
    return g >= 0 ? a.cmd[static_cast<int64_t>(ch[jj].x) * nmb + (g >> 2) * mbw + m] : 0ull;
  };
  int ga, ma, gb, mb2;
  task(0, 0, ga, ma);
  task(0, 1, gb, mb2);
  uint64_t ca = command(0, ga, ma), cb = command(0, gb, mb2);
  // level 0's reference rows, HBM -> LDS, 16 bytes a lane, all in flight
  if (f0.y >= 0) {
    const uint8_t *ref = a.surf + static_cast<int64_t>(f0.y) * a.frame_stride;
    const int cpr = W / 16;                     // chunks per row
    const int nrows = nl + nl / 2, nchunk = nrows * cpr;
    constexpr int kPer = 8;
    for (int i0 = 0; i0 < nchunk; i0 += kPer * kTbThreads) {
      uint4 v[kPer];
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        // past the end: reload the last chunk (branch-free, every load in flight)
        const int i = min(i0 + static_cast<int>(threadIdx.x) + k * kTbThreads, nchunk - 1);
        const int row = i / cpr, col = i - row * cpr;
        const int64_t src = row < nl ? static_cast<int64_t>(ly0 + row) * a.pitch
                                     : static_cast<int64_t>(H + cy0 + (row - nl)) * a.pitch;
        v[k] = *reinterpret_cast<const uint4 *>(ref + src + col * 16);
      }
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const int i = i0 + static_cast<int>(threadIdx.x) + k * kTbThreads;
        if (i < nchunk) reinterpret_cast<uint4 *>(lds)[i] = v[k];  // row r at r * W: W = cpr * 16
      }
    }
  }
  if (threadIdx.x < 256) lds_hist[threadIdx.x] = 0;
  __syncthreads();
  for (int j = 0; j < n; ++j) {
    const int4 fr = ch[j];
    const int hp = (n - j) * kTbHalo;
    const int p_lo = max(0, 4 * band - hp), p_hi = min(NG, 4 * band + 4 + hp);
    const bool last = j == n - 1;
    const int g0 = ga, m0 = ma, g1 = gb, m1 = mb2;
    const uint64_t c0 = current_cmd(ca, a.epoch), c1 = current_cmd(cb, a.epoch);
    if (!last) {  // next level's tasks and commands
      task(j + 1, 0, ga, ma);
      task(j + 1, 1, gb, mb2);
      ca = command(j + 1, ga, ma);
      cb = command(j + 1, gb, mb2);
    }
    auto put = [&](int g, int m, const uint4 (&rows)[6]) {
#pragma unroll
      for (int r = 0; r < 4; ++r) *reinterpret_cast<uint4 *>(lds + (4 * g + r - ly0) * W + m * 16) = rows[r];
#pragma unroll
      for (int r = 0; r < 2; ++r)
        *reinterpret_cast<uint4 *>(lds + nl * W + (2 * g + r - cy0) * W + m * 16) = rows[4 + r];
    };
    static_assert(S == 1 || S == kTbSlots, "one or two task slots");
    // in place: every lane reads level j-1 (the reference rows for j = 0)
    // into registers, barrier, then writes level j
    uint4 ra[6], rb[6];
    const bool has_ref = fr.y >= 0;
    const int vy0 = 4 * p_lo, vy1 = 4 * p_hi, vc0 = 2 * p_lo, vc1 = 2 * p_hi;
    if (g0 >= 0) tb_group_lds(lds, ly0, cy0, nl, W, H, vy0, vy1, vc0, vc1, a.es, c0, m0, g0, has_ref, ra, errs, range);
    if (g1 >= 0) tb_group_lds(lds, ly0, cy0, nl, W, H, vy0, vy1, vc0, vc1, a.es, c1, m1, g1, has_ref, rb, errs, range);
    if (!last) {
      __syncthreads();  // level j-1 fully read before level j overwrites it
      if (g0 >= 0) put(g0, m0, ra);
      if (g1 >= 0) put(g1, m1, rb);
    }
    uint32_t sad = 0;
    const int64_t gframe = fa.frame0 + fr.x;
    if (band_lane) {
      const uint4 *yr = ra, *cr = ra + 4;
      if (ta.keep || last) {
        uint8_t *dst = a.surf + static_cast<int64_t>(fr.x) * a.frame_stride;
        uint8_t *dst_uv = dst + static_cast<int64_t>(a.pitch) * H;
#pragma unroll
        for (int r = 0; r < 4; ++r) st_row(dst + static_cast<int64_t>(4 * bg + r) * a.pitch + bm * 16, yr[r]);
#pragma unroll
        for (int r = 0; r < 2; ++r) st_row(dst_uv + static_cast<int64_t>(2 * bg + r) * a.pitch + bm * 16, cr[r]);
      }
      uint32_t ys[4] = {0, 0, 0, 0}, us[4] = {0, 0, 0, 0}, vs[4] = {0, 0, 0, 0};
#pragma unroll
      for (int r = 0; r < 4; ++r) add_luma16<4>(yr[r], ys);
#pragma unroll
      for (int r = 0; r < 2; ++r) add_chroma16<4>(cr[r], us, vs);
      uint32_t rgb24[4], packed = 0;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const uint32_t y = (ys[p] + 8) / 16, u = (us[p] + 2) / 4, v = (vs[p] + 2) / 4;
        rgb24[p] = bt709_rgb24(y, u, v);
        packed |= y << (8 * p);
        atomicAdd(&lds_hist[y], 1u);
      }
      const int64_t tpx = static_cast<int64_t>(bg) * fa.w + bm * 4;
      store_rgb<4>(fa.rgb + (gframe * npx + tpx) * 3, rgb24);
      *reinterpret_cast<uint32_t *>(fa.thumb + fr.x * npx + tpx) = packed;
      if (fr.z >= 0) sad = sad_u8(packed, prevw, 0u);
      prevw = packed;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) sad += __shfl_xor(sad, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sad;
    __syncthreads();  // scoring (histogram, SAD shares) and the level's LDS rows are complete
    if (threadIdx.x == 0 && fr.z >= 0) {
      uint64_t t = 0;
#pragma unroll
      for (int i = 0; i < kTbThreads / 64; ++i) t += red[i];
      atomicAdd(reinterpret_cast<unsigned long long *>(fa.sad + gframe), static_cast<unsigned long long>(t));
    }
    if (threadIdx.x < 128) {
      const uint64_t lo = lds_hist[2 * threadIdx.x], hi = lds_hist[2 * threadIdx.x + 1];
      if (lo | hi)
        atomicAdd(reinterpret_cast<unsigned long long *>(fa.hist + gframe * 256) + threadIdx.x,
                  static_cast<unsigned long long>(lo | (hi << 32)));
    }
    __syncthreads();
    if (threadIdx.x < 256) lds_hist[threadIdx.x] = 0;
  }
  if (errs | range) atomicOr(a.err, errs | (range ? static_cast<uint32_t>(DEC_W_LEVEL_RANGE) : 0u));
}

}  // namespace

int clear_accum_launch(uint32_t *hist, uint64_t *sad, int64_t n_frames, hipStream_t s) {
  if (n_frames <= 0) return VTS_OK;
  if (reinterpret_cast<uintptr_t>(hist) & 15) return fail(VTS_E_INVALID, "clear_accum: histogram not 16-byte aligned");
  hipLaunchKernelGGL(clear_accum, dim3(static_cast<unsigned>((n_frames * 64 + 255) / 256)), dim3(256), 0, s,
                     reinterpret_cast<uint4 *>(hist), sad, n_frames);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(VTS_E_HIP, "clear_accum launch: %s", hipGetErrorString(e));
  return VTS_OK;
}

int sad_score_launch(const uint64_t *sad, float *score, int64_t frame0, int64_t n_frames,
                     int64_t npx, hipStream_t s) {
  if (n_frames <= 0) return VTS_OK;
  hipLaunchKernelGGL(sad_score, dim3(static_cast<unsigned>((n_frames + 255) / 256)), dim3(256), 0, s, sad,
                     score, frame0, n_frames, static_cast<double>(npx) * 255.0);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(VTS_E_HIP, "sad_score launch: %s", hipGetErrorString(e));
  return VTS_OK;
}

int parse_launch(const ParseArgs &a, hipStream_t s) {
  if (a.n_slices <= 0) return VTS_OK;
  hipLaunchKernelGGL(h264_parse, dim3((a.n_slices + 63) / 64), dim3(64), 0, s, a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(VTS_E_HIP, "h264_parse launch: %s", hipGetErrorString(e));
  return VTS_OK;
}

int fused_launch(const FusedArgs &a, int k, int n_frames, hipStream_t s) {
  if (n_frames <= 0) return VTS_OK;
  if (k == 6) {
    FusedArgs b = a;
    // one wave per (band, 63 macroblock columns), 4 bands per workgroup
    const int bands = (a.r.mb_height * 16 + 5) / 6;
    b.wgs_per_frame = ((a.r.mb_width + kK6bCols - 1) / kK6bCols) * ((bands + 3) / 4);
    hipLaunchKernelGGL(h264_recon_score6b, dim3(n_frames * b.wgs_per_frame), dim3(256), 0, s, b);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(VTS_E_HIP, "h264_recon_score6b launch: %s", hipGetErrorString(e));
    return VTS_OK;
  }
  const int q = (k == 0) ? 4 : 16 / k;
  const int nmb = a.r.mb_width * a.r.mb_height;
  const int mb_per_wg = kReconThreads / q;
  FusedArgs b = a;
  b.wgs_per_frame = (nmb + mb_per_wg - 1) / mb_per_wg;
  const dim3 grid(n_frames * b.wgs_per_frame), block(kReconThreads);
  switch (k) {
    case 0: hipLaunchKernelGGL(h264_recon_score<0>, grid, block, 0, s, b); break;
    case 2: hipLaunchKernelGGL(h264_recon_score<2>, grid, block, 0, s, b); break;
    case 4: hipLaunchKernelGGL(h264_recon_score<4>, grid, block, 0, s, b); break;
    case 8: hipLaunchKernelGGL(h264_recon_score<8>, grid, block, 0, s, b); break;
    default: return fail(VTS_E_INVALID, "fused path needs k in {0,2,4,8}");
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(VTS_E_HIP, "h264_recon_score launch: %s", hipGetErrorString(e));
  return VTS_OK;
}

int thumb_sad_launch(const ThumbSadArgs &t, hipStream_t s) {
  const int64_t n = t.list ? t.n_list : t.n_frames;
  if (n <= 0) return VTS_OK;
  hipLaunchKernelGGL(thumb_sad, dim3(static_cast<unsigned>(n)), dim3(256), 0, s, t);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(VTS_E_HIP, "thumb_sad launch: %s", hipGetErrorString(e));
  return VTS_OK;
}

int tb_lds_bytes(int mb_width, int mb_height, int L) {
  const int groups = std::min(4 * mb_height, 4 + 2 * L * kTbHalo);  // level 0's reference rows
  return groups * 6 * mb_width * 16 + 32;  // + the over-read of a row's second chunk
}

int tb_max_tasks(int mb_width, int mb_height, int L) {
  return std::min(4 * mb_height, 4 + 2 * (L - 1) * kTbHalo) * mb_width;
}

int tb_launch(const TbArgs &a, int n_chains, hipStream_t s) {
  if (n_chains <= 0) return VTS_OK;
  const int mbw = a.f.r.mb_width, mbh = a.f.r.mb_height;
  // shapes the kernel assumes: band tasks in slot 0, all tasks in kTbSlots slots
  if (4 * mbw > kTbThreads || tb_max_tasks(mbw, mbh, a.L) > kTbThreads * kTbSlots || a.L < 1 || a.L > 16)
    return fail(VTS_E_INVALID, "h264_recon_score_tb: %dx%d macroblocks, L=%d out of range", mbw, mbh, a.L);
  const int lds = tb_lds_bytes(mbw, mbh, a.L);
  static bool attr_set = false;
  if (!attr_set) {
    for (const void *k : {reinterpret_cast<const void *>(h264_recon_score_tb<1>),
                          reinterpret_cast<const void *>(h264_recon_score_tb<2>)}) {
      const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
      if (e != hipSuccess) return fail(VTS_E_HIP, "h264_recon_score_tb attribute: %s", hipGetErrorString(e));
    }
    attr_set = true;
  }
  if (lds > 150 * 1024) return fail(VTS_E_INVALID, "h264_recon_score_tb: %d bytes of LDS", lds);
  const dim3 grid(static_cast<unsigned>(n_chains) * mbh), block(kTbThreads);
  if (tb_max_tasks(mbw, mbh, a.L) <= kTbThreads)
    hipLaunchKernelGGL(h264_recon_score_tb<1>, grid, block, static_cast<unsigned>(lds), s, a);
  else
    hipLaunchKernelGGL(h264_recon_score_tb<2>, grid, block, static_cast<unsigned>(lds), s, a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(VTS_E_HIP, "h264_recon_score_tb launch: %s", hipGetErrorString(e));
  return VTS_OK;
}

int recon_launch(const ReconArgs &a, int n_frames, hipStream_t s) {
  FusedArgs f{};
  f.r = a;
  return fused_launch(f, 0, n_frames, s);
}

}  // namespace vts
