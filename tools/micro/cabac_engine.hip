// Micro-benchmark: cycles per CABAC decision on one lone wave, product engine
// (parse_cabac.h CabacSyn::dec) against leaner engine variants, on the same
// random bytes; every variant's bins are compared with the product engine's
// on the device.  Variants:
//   prod     CabacSyn::dec (range / offset in VGPRs, four states per dword)
//   sdword   range / offset in SGPRs, one state per dword, branch on the LPS path
//   sdwordc  as sdword with selects instead of the branch
//   vdword   range / offset in VGPRs (as prod), one state per dword
// Modes: const (one context), var (15 contexts in turn), pair (significance /
// last pairs of a 4x4 block map: the next context depends on the bin).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ivideo-transformer_amd/csrc \
//         tools/micro/cabac_engine.hip -o tools/micro/cabac_engine
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "parse_cabac.h"

using namespace vts;
using namespace vts::full;

// ------------------------------------------------------------ lean engines
template <bool kVgpr, bool kBranch>
struct Lean {
  RbspBitsT<kCacheWords> br;
  uint32_t range, val;
  int32_t la;
  LaneTab st[4];  // context c: table c >> 6, lane c & 63, the state (pStateIdx << 1 | valMPS) in the low byte
  LaneTab lps, trn;
  VTS_HD VTS_INLINE uint32_t ev(uint32_t x) { return kVgpr ? VTS_EV(x) : x; }
  VTS_HD VTS_INLINE uint32_t eu(uint32_t x) { return kVgpr ? VTS_EU(x) : x; }
  VTS_HD VTS_INLINE void start(const CabacSyn &p) {
    for (int i = 0; i < 64; ++i) {
      lps.set(i, kCabLanes.lps[i]);
      trn.set(i, kCabLanes.trans[i]);
    }
    // the product's packed states, unpacked: slot q of table t -> context
    for (int t = 0; t < 4; ++t)
      for (int l = 0; l < 64; ++l) {
        const int c = 64 * t + l;
        const int q = CabacSyn::ctx_slot(c), tb = CabacSyn::ctx_tab(c);
        st[t].set(l, (p.st[tb].get(static_cast<uint32_t>(q >> 2)) >> (8 * (q & 3))) & 127u);
      }
    range = ev(510u);
    val = ev(br.bits(32));
    la = 23;
  }
  VTS_HD VTS_INLINE void fill() {
    if (la < 8) {
      val |= br.bits(16) << (7 - la);
      la += 16;
    }
  }
  template <int T>
  VTS_HD VTS_INLINE uint32_t dec(uint32_t lane) {
    const uint32_t s = st[T].get(lane);
    const uint32_t ps = s >> 1, mps = s & 1u;
    const uint32_t lpsr = (lps.get(ps) >> ((range >> 3) & 24u)) & 255u;
    const uint32_t tw = trn.get(ps);
    range -= lpsr;
    const uint32_t rs = range << 23;
    uint32_t bin, ns;
    if (kBranch) {
      if (eu(val >= rs ? 1u : 0u)) {
        val -= rs;
        range = lpsr;
        bin = mps ^ 1u;
        ns = (tw & 127u) ^ mps;
      } else {
        bin = mps;
        ns = ((tw >> 8) & 127u) ^ mps;
      }
    } else {
      const bool l = val >= rs;
      bin = eu(mps ^ (l ? 1u : 0u));
      ns = eu(((tw >> (l ? 0u : 8u)) & 127u) ^ mps);
      val -= l ? rs : 0u;
      range = l ? lpsr : range;
    }
    st[T].set(lane, ns);
    const int n = static_cast<int>(eu(__builtin_clz(range) - 23));
    range <<= n;
    val <<= n;
    la -= n;
    fill();
    return bin;
  }
};

struct Run {
  const uint8_t *rbsp;
  int32_t len;
  int32_t n;
  int32_t mode;     // 0 const, 1 var, 2 pair
  int32_t engine;   // 0 prod, 1 sdword, 2 sdwordc, 3 vdword
  uint32_t *bits;
};

template <class E>
VTS_HD VTS_INLINE uint32_t loop(E &&dec, const Run &r, uint32_t *bits) {
  uint32_t acc = 0, word = 0;
  int k = 0, i = 0, phase = 0;  // pair: position i in the map, phase 0 significance, 1 last
  for (int b = 0; b < r.n; ++b) {
    uint32_t bin;
    if (r.mode == 0) {
      bin = dec(60);
    } else if (r.mode == 1) {
      bin = dec(105 + (b % 15));
    } else {
      bin = dec(phase ? 166 + 15 + i : 105 + 15 + i);  // cat 1 contexts (sig_off 15)
      if (phase == 0) {
        if (bin) phase = 1;
        else if (++i == 15) i = 0;
      } else {
        phase = 0;
        i = bin ? 0 : (i + 1 == 15 ? 0 : i + 1);
      }
    }
    acc += bin;
    word |= bin << (b & 31);
    if ((b & 31) == 31 || b + 1 == r.n) {
#if defined(__HIP_DEVICE_COMPILE__)
      if (threadIdx.x == 0) bits[k] = word;
#else
      bits[k] = word;
#endif
      ++k;
      word = 0;
    }
  }
  (void)i;
  return acc;
}

__global__ void __launch_bounds__(64) engine_kernel(Run r, uint32_t *out, unsigned long long *cyc) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[sizeof(SynScratch) + 64];
  SynScratch *sc = reinterpret_cast<SynScratch *>(lds);
  CabacSyn p{};
  p.sc = sc;
  p.br.init(r.rbsp, r.len, sc->cache);
  p.refresh_lane();
  p.br.reset_at(0);
  p.cab_tables();
  p.cab_init(true, 26);
  unsigned long long t0 = 0, t1 = 0;
  uint32_t acc = 0;
  if (r.engine == 0 && r.mode == 3) {  // 16 decisions per loop trip, nothing else in the loop
    p.cab_start();
    t0 = __builtin_amdgcn_s_memtime();
    for (int b = 0; b < r.n; b += 16) {
#pragma unroll
      for (int k = 0; k < 16; ++k) acc += p.dec(60);
    }
    t1 = __builtin_amdgcn_s_memtime();
  } else if (r.engine == 0 && r.mode == 4) {  // 16 bypass bins per trip
    p.cab_start();
    t0 = __builtin_amdgcn_s_memtime();
    for (int b = 0; b < r.n; b += 16) {
#pragma unroll
      for (int k = 0; k < 16; ++k) acc += p.bypass();
    }
    t1 = __builtin_amdgcn_s_memtime();
  } else if (r.engine == 0) {
    p.cab_start();
    t0 = __builtin_amdgcn_s_memtime();
    acc = loop([&](int c) { return p.dec(c); }, r, r.bits);
    t1 = __builtin_amdgcn_s_memtime();
  } else if (r.engine == 1 || r.engine == 2 || r.engine == 3) {
    auto go = [&](auto &e) {
      e.br = p.br;
      e.start(p);
      t0 = __builtin_amdgcn_s_memtime();
      acc = loop([&](int c) {
        const uint32_t lane = static_cast<uint32_t>(c) & 63u;
        switch (c >> 6) {
          case 0: return e.template dec<0>(lane);
          case 1: return e.template dec<1>(lane);
          case 2: return e.template dec<2>(lane);
          default: return e.template dec<3>(lane);
        }
      }, r, r.bits);
      t1 = __builtin_amdgcn_s_memtime();
    };
    if (r.engine == 1) {
      Lean<false, true> e;
      go(e);
    } else if (r.engine == 2) {
      Lean<false, false> e;
      go(e);
    } else {
      Lean<true, false> e;
      go(e);
    }
  }
  if (threadIdx.x == 0) {
    out[0] = acc;
    cyc[0] = t1 - t0;
  }
}

int main(int argc, char **argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 200000;
  const int32_t len = 1 << 20;
  std::vector<uint8_t> h(static_cast<size_t>(len) + 256);
  uint32_t x = 12345;
  for (auto &b : h) {
    x = x * 1664525u + 1013904223u;
    b = static_cast<uint8_t>(x >> 24);
  }
  uint8_t *d = nullptr;
  uint32_t *dout = nullptr, *dbits = nullptr;
  unsigned long long *dcyc = nullptr;
  const size_t words = static_cast<size_t>(n) / 32 + 1;
  (void)hipMalloc(&d, h.size());
  (void)hipMalloc(&dout, 4);
  (void)hipMalloc(&dcyc, 8);
  (void)hipMalloc(&dbits, words * 4);
  (void)hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice);
  const char *modes[] = {"const", "var", "pair", "const_unrolled16", "bypass_unrolled16"};
  const char *engines[] = {"prod", "sdword", "sdwordc", "vdword"};
  for (int mode = 0; mode < 5; ++mode) {
    std::vector<uint32_t> ref(words), got(words);
    for (int eng = 0; eng < (mode >= 3 ? 1 : 4); ++eng) {
      Run r{d, len, n, mode, eng, dbits};
      hipLaunchKernelGGL(engine_kernel, dim3(1), dim3(64), 0, 0, r, dout, dcyc);  // warm-up
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0, 0);
      hipLaunchKernelGGL(engine_kernel, dim3(1), dim3(64), 0, 0, r, dout, dcyc);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      unsigned long long cyc = 0;
      (void)hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
      (void)hipMemcpy(eng ? got.data() : ref.data(), dbits, words * 4, hipMemcpyDeviceToHost);
      long diff = -1;
      if (eng)
        for (int b = 0; b < n && diff < 0; ++b)
          if (((ref[b >> 5] ^ got[b >> 5]) >> (b & 31)) & 1u) diff = b;
      std::printf("{\"mode\": \"%s\", \"engine\": \"%s\", \"bins\": %d, \"first_diff_vs_prod\": %ld, \"ms\": %.3f, "
                  "\"ns_per_bin\": %.2f, \"memtime_per_bin\": %.1f}\n",
                  modes[mode], engines[eng], n, diff, ms, ms * 1e6 / n, static_cast<double>(cyc) / n);
    }
  }
  return 0;
}
