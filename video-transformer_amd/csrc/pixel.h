// pixel.h — device helpers shared by the scoring and fused decode kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace vts {

__device__ __forceinline__ uint32_t sad_u8(uint32_t a, uint32_t b, uint32_t acc) {
  return __builtin_amdgcn_sad_u8(a, b, acc);
}

// clamp(floor(x / 256), 0, 255).  The shift is an opaque asm statement: for
// the plain `clamp(x >> 8, 0, 255)` hipcc (ROCm 7.2) selects gfx950's
// v_ashr_pk_u8_i32 for pairs of such values, and those bytes came out wrong
// (saturated as if unshifted; caught by the bit-exact tests).
__device__ __forceinline__ uint32_t shr8_sat(int x) {
  int t;
  asm("v_ashrrev_i32 %0, 8, %1" : "=v"(t) : "v"(x));
  return static_cast<uint32_t>(t < 0 ? 0 : (t > 255 ? 255 : t));
}

// BT.709 limited range, 8-bit fixed point (x256); floor division by 256.
__device__ __forceinline__ uint32_t bt709_rgb24(uint32_t y, uint32_t u, uint32_t v) {
  const int c = static_cast<int>(y) - 16, d = static_cast<int>(u) - 128,
            e = static_cast<int>(v) - 128;
  const uint32_t r = shr8_sat(298 * c + 459 * e + 128);
  const uint32_t g = shr8_sat(298 * c - 55 * d - 136 * e + 128);
  const uint32_t b = shr8_sat(298 * c + 541 * d + 128);
  return r | (g << 8) | (b << 16);
}

// Store G pixels of packed 24-bit RGB (r | g << 8 | b << 16) at dst.  G % 4 ==
// 0 needs 4-byte alignment, G == 2 needs 2-byte alignment.  Shifts only (no
// byte arrays: byte-array packing miscompiled on gfx950 in an earlier build).
template <int G>
__device__ __forceinline__ void store_rgb(uint8_t *dst, const uint32_t *rgb24) {
  if constexpr (G % 4 == 0) {
    uint32_t *d32 = reinterpret_cast<uint32_t *>(dst);
#pragma unroll
    for (int q = 0; q < G / 4; ++q) {
      const uint32_t a0 = rgb24[4 * q], a1 = rgb24[4 * q + 1];
      const uint32_t a2 = rgb24[4 * q + 2], a3 = rgb24[4 * q + 3];
      d32[3 * q + 0] = a0 | (a1 << 24);
      d32[3 * q + 1] = (a1 >> 8) | (a2 << 16);
      d32[3 * q + 2] = (a2 >> 16) | (a3 << 8);
    }
  } else {
    static_assert(G == 2, "G must be 2 or a multiple of 4");
    uint16_t *d16 = reinterpret_cast<uint16_t *>(dst);
    const uint32_t a0 = rgb24[0], a1 = rgb24[1];
    d16[0] = static_cast<uint16_t>(a0 & 0xffffu);
    d16[1] = static_cast<uint16_t>((a0 >> 16) | ((a1 & 0xffu) << 8));
    d16[2] = static_cast<uint16_t>(a1 >> 8);
  }
}

// Box sums over one 16-byte row chunk: luma bytes [p*K, p*K+K) per pixel p,
// and for an NV12 UV row the U (even) / V (odd) bytes of the same span.
template <int K>
__device__ __forceinline__ void add_luma16(const uint4 v, uint32_t *ys) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  if constexpr (K == 2) {
#pragma unroll
    for (int p = 0; p < 8; ++p)
      ys[p] = sad_u8(w[p / 2] & ((p & 1) ? 0xffff0000u : 0x0000ffffu), 0u, ys[p]);
  } else if constexpr (K == 4) {
#pragma unroll
    for (int p = 0; p < 4; ++p) ys[p] = sad_u8(w[p], 0u, ys[p]);
  } else {
    static_assert(K == 8, "K must be 2, 4 or 8");
#pragma unroll
    for (int p = 0; p < 2; ++p) ys[p] = sad_u8(w[2 * p + 1], 0u, sad_u8(w[2 * p], 0u, ys[p]));
  }
}

template <int K>
__device__ __forceinline__ void add_chroma16(const uint4 v, uint32_t *us, uint32_t *vs) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  if constexpr (K == 2) {
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const uint32_t word = w[p / 2] >> ((p & 1) * 16);
      us[p] += word & 0xffu;
      vs[p] += (word >> 8) & 0xffu;
    }
  } else if constexpr (K == 4) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      us[p] = sad_u8(w[p] & 0x00ff00ffu, 0u, us[p]);
      vs[p] = sad_u8((w[p] >> 8) & 0x00ff00ffu, 0u, vs[p]);
    }
  } else {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      us[p] = sad_u8(w[2 * p + 1] & 0x00ff00ffu, 0u, sad_u8(w[2 * p] & 0x00ff00ffu, 0u, us[p]));
      vs[p] = sad_u8((w[2 * p + 1] >> 8) & 0x00ff00ffu, 0u,
                     sad_u8((w[2 * p] >> 8) & 0x00ff00ffu, 0u, vs[p]));
    }
  }
}

}  // namespace vts
