// Micro-benchmark: the cost of one CABAC bin on one wave of the general
// decoder's parser (parse_cabac.h, the very engine code the parse kernel
// inlines), with nothing else running.  Modes:
//   0  context-coded bins, context index varying at run time (both lane tables)
//   1  context-coded bins, one constant context
//   2  bypass bins
//   3  residual_block_cabac of 4x4 luma blocks (cat 2) back to back
//   4  residual_block_cabac of 8x8 blocks (cat 5)
// The host runs the same calls on the same bytes to count the bins.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ivideo-transformer_amd/csrc
//         tools/micro/cabac_bins.hip -o /tmp/cabac_bins && /tmp/cabac_bins
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

static unsigned long long g_trace[32];
#if !defined(__HIP_DEVICE_COMPILE__)
#define VTS_PARSE_TRACE(k) (++g_trace[(k)])
#endif
#include "parse_cabac.h"

using namespace vts;
using namespace vts::full;

struct Run {
  const uint8_t *rbsp;
  int32_t len;
  int32_t n;
  int32_t mode;
  uint32_t *bits;  // modes 0-2: every bin, 32 per word (device: lane 0 stores)
};

VTS_HD VTS_INLINE uint32_t run_bins(const Run &r, SynScratch *sc) {
  CabacSyn p{};
  p.sc = sc;
  p.br.init(r.rbsp, r.len, sc->cache);
  p.refresh_lane();
  p.br.reset_at(0);
  p.cab_tables();
  p.cab_init(true, 26);
  p.cab_start();
  uint32_t acc = 0, word = 0;
  for (int i = 0; i < r.n; ++i) {
    if (r.mode <= 2) {
      const uint32_t b = r.mode == 0 ? p.dec(105 + (i % 15)) : (r.mode == 1 ? p.dec(60) : p.bypass());
      acc += b;
      word |= b << (i & 31);
      if ((i & 31) == 31 || i + 1 == r.n) {
#if defined(__HIP_DEVICE_COMPILE__)
        if (threadIdx.x == 0) r.bits[i >> 5] = word;
#else
        r.bits[i >> 5] = word;
#endif
        word = 0;
      }
    } else if (r.mode == 3) {
      for (int k = 0; k < 16; ++k) sc->blk[k] = 0;
      acc += static_cast<uint32_t>(p.residual_t<false>(2, i & 3, 16, sc->blk, 0));
    } else {
      for (int k = 0; k < 64; ++k) sc->blk8[k] = 0;
      acc += static_cast<uint32_t>(p.residual_t<true>(5, 0, 64, sc->blk8, 0));
    }
  }
  return acc;
}

__global__ void __launch_bounds__(64) bins_kernel(Run r, uint32_t *out, unsigned long long *cyc) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[sizeof(SynScratch) + 64];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const uint32_t acc = run_bins(r, reinterpret_cast<SynScratch *>(lds));
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[blockIdx.x] = acc;
    cyc[blockIdx.x] = t1 - t0;
  }
}

int main(int argc, char **argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 200000;
  const int32_t len = 8 << 20;
  std::vector<uint8_t> h(static_cast<size_t>(len) + 256);
  uint32_t x = 12345;
  for (auto &b : h) {
    x = x * 1664525u + 1013904223u;
    b = static_cast<uint8_t>(x >> 24);
  }
  uint8_t *d = nullptr;
  uint32_t *dout = nullptr;
  unsigned long long *dcyc = nullptr;
  (void)hipMalloc(&d, h.size());
  (void)hipMalloc(&dout, 4);
  (void)hipMalloc(&dcyc, 8);
  (void)hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice);
  const char *names[] = {"ctx_var", "ctx_const", "bypass", "res4x4", "res8x8"};
  for (int mode = 0; mode < 5; ++mode) {
    const int nn = mode >= 3 ? n / 40 : n;
    // bins on the host (same bytes, same calls)
    for (auto &t : g_trace) t = 0;
    std::vector<uint8_t> lds(sizeof(SynScratch) + 64);
    std::vector<uint32_t> hbits(static_cast<size_t>(nn) / 32 + 1, 0), dbits(hbits.size(), 0);
    uint32_t *dbits_d = nullptr;
    (void)hipMalloc(&dbits_d, dbits.size() * 4);
    Run hr{h.data(), len, nn, mode, hbits.data()};
    const uint32_t hacc = run_bins(hr, reinterpret_cast<SynScratch *>(lds.data()));
    const unsigned long long bins = g_trace[1] + g_trace[2] + g_trace[3];
    Run r{d, len, nn, mode, dbits_d};
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(bins_kernel, dim3(1), dim3(64), 0, 0, r, dout, dcyc);  // warm-up
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(bins_kernel, dim3(1), dim3(64), 0, 0, r, dout, dcyc);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    uint32_t acc = 0;
    unsigned long long cyc = 0;
    (void)hipMemcpy(&acc, dout, 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(dbits.data(), dbits_d, dbits.size() * 4, hipMemcpyDeviceToHost);
    long first_diff = -1;
    if (mode <= 2)
      for (int i = 0; i < nn && first_diff < 0; ++i)
        if (((hbits[i >> 5] >> (i & 31)) & 1) != ((dbits[i >> 5] >> (i & 31)) & 1)) first_diff = i;
    std::printf("{\"mode\": \"%s\", \"first_diff_bin\": %ld, \"host_acc\": %u, \"dev_acc\": %u}\n", names[mode],
                first_diff, hacc, acc);
    std::printf("{\"mode\": \"%s\", \"calls\": %d, \"bins\": %llu, \"equal\": %s, \"ms\": %.3f, \"ns_per_bin\": %.2f, "
                "\"memtime_per_bin\": %.1f}\n",
                names[mode], nn, bins, acc == hacc ? "true" : "false", ms, ms * 1e6 / static_cast<double>(bins),
                static_cast<double>(cyc) / static_cast<double>(bins));
  }
  return 0;
}
