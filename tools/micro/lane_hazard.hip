// Check: does a v_readlane right after a v_writelane of the same VGPR (the
// CABAC parser's LaneTab set / get pattern) read the value just written, on
// gfx950, with no wait states between them?  Variants: the same constant
// lane back to back, lanes in SGPRs (write via m0), the same constant lane
// with one wait state (s_nop 0) between, and another writelane between.  Each
// runs 100 000 dependent rounds on one wave and counts rounds whose read
// differs from the value written.  Inline asm, so the compiler's hazard
// recognizer adds nothing.  Measured (profiles/r06u_lane_hazard.json): back
// to back with constant lanes reads the stale lane (90 000 of 100 000; the
// loop's tenth copy has other instructions between); one wait state, or any
// instruction between, reads the new value.  The compiler puts that s_nop 0
// between a v_writelane and a dependent v_readlane it emits itself
// (llvm.amdgcn.writelane, LaneTab in parse_full.h), so product code is safe.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/lane_hazard.hip -o tools/micro/lane_hazard
#include <hip/hip_runtime.h>

#include <cstdio>

template <int T>
__global__ void __launch_bounds__(64) hazard(uint32_t seed, uint32_t *bad_out) {
  uint32_t v = threadIdx.x;  // the lane table (one VGPR)
  uint32_t bad = 0, x = seed;
  for (int it = 0; it < 100000; ++it) {
    x = x * 1664525u + 1013904223u;
    uint32_t got;
    uint32_t lane = (x >> 7) & 63u;
    if constexpr (T == 0) {  // writelane then readlane, same constant lane, back to back
      asm volatile("v_writelane_b32 %0, %2, 5\n v_readlane_b32 %1, %0, 5" : "+v"(v), "=s"(got) : "s"(x));
      bad += got != x;
    } else if constexpr (T == 1) {  // same SGPR lane index, back to back
      asm volatile("s_mov_b32 m0, %3\n v_writelane_b32 %0, %2, m0\n v_readlane_b32 %1, %0, %3"
                   : "+v"(v), "=s"(got) : "s"(x), "s"(lane) : "m0");
      bad += got != x;
    } else if constexpr (T == 2) {  // same constant lane, one wait state between
      asm volatile("v_writelane_b32 %0, %2, 5\n s_nop 0\n v_readlane_b32 %1, %0, 5" : "+v"(v), "=s"(got) : "s"(x));
      bad += got != x;
    } else {  // readlane of a lane written two rounds earlier (other lanes written between)
      asm volatile("v_writelane_b32 %0, %2, 7\n v_writelane_b32 %0, %3, 9\n v_readlane_b32 %1, %0, 7"
                   : "+v"(v), "=s"(got) : "s"(x), "s"(x ^ 0x5a5a5a5au));
      bad += got != x;
    }
  }
  if (threadIdx.x == 0) bad_out[T] = bad;
}

int main() {
  uint32_t *d = nullptr;
  (void)hipMalloc(&d, 16);
  (void)hipMemset(d, 0xff, 16);
  hipLaunchKernelGGL(hazard<0>, dim3(1), dim3(64), 0, 0, 12345u, d);
  hipLaunchKernelGGL(hazard<1>, dim3(1), dim3(64), 0, 0, 12345u, d);
  hipLaunchKernelGGL(hazard<2>, dim3(1), dim3(64), 0, 0, 12345u, d);
  hipLaunchKernelGGL(hazard<3>, dim3(1), dim3(64), 0, 0, 12345u, d);
  uint32_t h[4];
  (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
  std::printf("{\"same_const_lane\": %u, \"same_sgpr_lane\": %u, \"same_const_lane_nop\": %u, \"other_lane_between\": %u, "
              "\"rounds\": 100000}\n", h[0], h[1], h[2], h[3]);
  return (h[0] | h[1] | h[2] | h[3]) != 0;
}
