// copy_bw.hip — HBM microbenchmark for the fused reconstruct kernel's traffic
// shape (one level launch: 300 frames of 1280x720 NV12 read from a reference
// ring slot, written to the next slot).  Variants isolate what the real
// kernel adds to a plain streaming copy:
//   A linear float4 copy (grid-stride)
//   B macroblock-structured copy: lane per (MB, 4-row group), 6 aligned rows
//   C B + misaligned source (two aligned loads + funnel shift per row)
//   D C + a per-lane 8-byte command load the addresses depend on
// hipcc --offload-arch=gfx950 -O3 copy_bw.hip -o copy_bw && ./copy_bw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int W = 1280, H = 720, PITCH = 1280, MBW = 80, MBH = 45, NMB = MBW * MBH;
constexpr int64_t STRIDE = ((int64_t)PITCH * H * 3 / 2 + 4095) & ~4095ll;

__global__ void copy_linear(const uint4 *__restrict__ s, uint4 *__restrict__ d, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    d[i] = s[i];
}

template <int MODE>
__global__ void __launch_bounds__(256) copy_mb(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                               const uint64_t *__restrict__ cmd, int wgs_per_frame, int shift) {
  extern __shared__ uint32_t occupancy_pad[];  // dynamic LDS limits WGs per CU
  if (threadIdx.x == 1024) occupancy_pad[0] = 0;
  const int fi = blockIdx.x / wgs_per_frame;
  const int q = threadIdx.x / 64;
  const int mb = (blockIdx.x - fi * wgs_per_frame) * 64 + (threadIdx.x % 64);
  if (mb >= NMB) return;
  const int mby = mb / MBW, m = mb - mby * MBW;
  int sh = shift;
  if (MODE >= 3) sh = (int)(cmd[(int64_t)fi * NMB + mb] & 15);
  const uint8_t *ref = src + (int64_t)fi * STRIDE;
  uint8_t *out = dst + (int64_t)fi * STRIDE;
  uint4 v[6];
  if (MODE == 1) {
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int row = i < 4 ? mby * 16 + q * 4 + i : H + mby * 8 + q * 2 + (i - 4);
      v[i] = *reinterpret_cast<const uint4 *>(ref + (int64_t)row * PITCH + m * 16);
    }
  } else {
    uint4 lo[6], hi[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int row = i < 4 ? mby * 16 + q * 4 + i : H + mby * 8 + q * 2 + (i - 4);
      const uint8_t *p = ref + (int64_t)row * PITCH + m * 16 + sh;
      const int s = (int)((uintptr_t)p & 15);
      const uint4 *al = reinterpret_cast<const uint4 *>(p - s);
      lo[i] = al[0];
      hi[i] = al[1];
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const uint32_t w[8] = {lo[i].x, lo[i].y, lo[i].z, lo[i].w, hi[i].x, hi[i].y, hi[i].z, hi[i].w};
      const int s = (int)((uintptr_t)(ref + m * 16 + sh) & 15), qd = s >> 2, r = s & 3;
      uint32_t t[5];
#pragma unroll
      for (int j = 0; j < 5; ++j) t[j] = qd == 0 ? w[j] : qd == 1 ? w[j + 1] : qd == 2 ? w[j + 2] : w[j + 3 < 8 ? j + 3 : 7];
      v[i] = make_uint4(__builtin_amdgcn_alignbyte(t[1], t[0], r), __builtin_amdgcn_alignbyte(t[2], t[1], r),
                        __builtin_amdgcn_alignbyte(t[3], t[2], r), __builtin_amdgcn_alignbyte(t[4], t[3], r));
    }
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int row = i < 4 ? mby * 16 + q * 4 + i : H + mby * 8 + q * 2 + (i - 4);
    *reinterpret_cast<uint4 *>(out + (int64_t)row * PITCH + m * 16) = v[i];
  }
}

int main(int argc, char **argv) {
  const int F = argc > 1 ? atoi(argv[1]) : 300;
  const int reps = 20;
  const int64_t bytes = (int64_t)F * STRIDE + 4096;
  uint8_t *a, *b;
  uint64_t *cmd;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&cmd, (int64_t)F * NMB * 8));
  CK(hipMemset(a, 7, bytes));
  CK(hipMemset(b, 0, bytes));
  CK(hipMemset(cmd, 3, (int64_t)F * NMB * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double frame_bytes = 2.0 * W * H * 1.5;  // read + write, NV12
  auto run = [&](const char *name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-34s %8.4f ms  %7.1f GB/s (read+write NV12 bytes)\n", name, ms, frame_bytes * F / (ms * 1e-3) / 1e9);
    return 0;
  };
  const int64_t n16 = (int64_t)F * STRIDE / 16;
  run("A linear float4 copy", [&] { copy_linear<<<8192, 256>>>((const uint4 *)a, (uint4 *)b, n16); });
  const int wpf = (NMB + 63) / 64;
  run("B MB-structured aligned", [&] { copy_mb<1><<<F * wpf, 256>>>(a, b, cmd, wpf, 0); });
  run("C MB-structured misaligned (sh=6)", [&] { copy_mb<2><<<F * wpf, 256>>>(a, b, cmd, wpf, 6); });
  run("C' MB-structured lo/hi aligned (sh=0)", [&] { copy_mb<2><<<F * wpf, 256>>>(a, b, cmd, wpf, 0); });
  run("D C + dependent command load", [&] { copy_mb<3><<<F * wpf, 256>>>(a, b, cmd, wpf, 0); });
  const int lds_for[] = {20 * 1024, 26 * 1024, 32 * 1024, 40 * 1024, 54 * 1024, 80 * 1024};
  const char *names[] = {"D @ <=8 WG/CU (LDS 20K)", "D @ <=6 WG/CU (LDS 26K)", "D @ <=5 WG/CU (LDS 32K)",
                         "D @ <=4 WG/CU (LDS 40K)", "D @ <=2 WG/CU (LDS 54K)", "D @ 2 WG/CU (LDS 80K)"};
  for (int i = 0; i < 6; ++i)
    run(names[i], [&] { copy_mb<3><<<F * wpf, 256, lds_for[i]>>>(a, b, cmd, wpf, 0); });
  return 0;
}
