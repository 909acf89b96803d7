// parse_slice.h — the CAVLC slice parser of the device decoder (h264_parse in
// decode.hip runs one lane of it per slice NAL).  Plain C++ with host+device
// qualifiers so the CPU test suite can also compile it and check its command
// words against the oracle's parser (tests/native/parse_host.cpp,
// oracle/vtseg_oracle.c or_slice_commands) without a GPU.  The product path
// only ever runs it on the GPU.
//
// Output: one 64-bit command per macroblock (h264.h MB_PCM / MB_INTER), the
// reconstruct kernel's input.  Anything outside the subset returns DEC_E_*.
#pragma once
#include <cstdint>

#include "h264.h"

#if defined(__HIPCC__)
#define VTS_HD __host__ __device__
#else
#define VTS_HD
#endif
#define VTS_INLINE inline __attribute__((always_inline))
// A lone parse wave pays ~16-20 cycles for every taken branch and ~2 for a
// fall-through (profiles/r06i_single_wave_issue_latencies.jsonl): rare paths
// (bit-reader refills) are laid out off the common path
#define VTS_UNLIKELY(x) __builtin_expect(!!(x), 0)

namespace vts {

// bytes r..r+3 of the 8-byte little-endian pair (lo, hi): v_alignbyte_b32 on gfx950
VTS_HD VTS_INLINE uint32_t vts_alignbyte(uint32_t hi, uint32_t lo, int r) {
  return static_cast<uint32_t>(((static_cast<uint64_t>(hi) << 32) | lo) >> (8 * (r & 3)));
}
VTS_HD VTS_INLINE int vts_min(int a, int b) { return a < b ? a : b; }
VTS_HD VTS_INLINE int vts_max(int a, int b) { return a > b ? a : b; }

struct alignas(16) Cmd2 {
  uint64_t a, b;
};

// ------------------------------------------------------------ bit reader
// Delivers the RBSP bits of a NAL payload (EBSP) through a left-aligned 64-bit
// window.  Refills take 4 EBSP bytes at a time from a 20-byte register cache;
// a group without any 0x03 byte cannot hold an emulation_prevention_three_byte
// and is appended whole, otherwise it goes byte by byte and the EPBs are
// dropped.  ue()/se() decode with one count-leading-zeros instead of a loop
// per bit.  Positions: `fill - nb` is the RBSP bit index of the next bit.
template <int kW>
struct WinBitsT {
  const uint8_t *base;   // first payload byte (absolute pointer)
  int64_t abs0;          // byte offset of `base` inside the ES buffer
  uint64_t win;          // next bits, MSB first
  int32_t nb;            // valid bits in win
  int32_t fill;          // RBSP bits appended to the window so far (incl. padding)
  int32_t real;          // ... of which real payload bits
  int32_t size;          // payload bytes
  int32_t pos;           // next EBSP byte to append
  int32_t zeros;         // consecutive zero bytes before pos (capped at 2)
  int32_t epb;           // emulation-prevention bytes removed so far
  int32_t epb_next;      // RBSP byte index that followed the last removed EPB
  int32_t cache_at;      // payload index of cache[0] (multiple of 16), -1 none
  uint32_t *cache;       // kW words = 4 (kW - 1) payload bytes + 4 from cache_at: per-lane
                         // scratch (LDS on the device), so the copies at every
                         // control-flow join that register state costs are avoided
  bool err;

  VTS_HD VTS_INLINE void init(const uint8_t *p, int64_t abs, int32_t n, uint32_t *scratch) {
    cache = scratch;
    base = p;
    abs0 = abs;
    size = n;
    win = 0;
    nb = fill = real = pos = zeros = epb = 0;
    epb_next = -1;
    cache_at = -1;
    err = false;
  }
  // 4 payload bytes at i (little endian: byte i in bits 0..7); reads up to 24
  // bytes past the payload (the ES buffer is padded)
  VTS_HD VTS_INLINE uint32_t load4(int32_t i) {
    constexpr int32_t kBlk = 4 * (kW - 1);  // bytes per cache block (16 or 64)
    const int32_t blk = i - (i % kBlk);
    if (blk != cache_at) {
      const uint8_t *pb = base + blk;
      const int sh = static_cast<int>(reinterpret_cast<uintptr_t>(pb) & 3);
      uint32_t t[kW + 1];
      if constexpr (kW > 5) {
        // wave-uniform parse (h264_parse_full): plain loads from a base the
        // compiler can see is dword aligned, all in flight together (as
        // scalar loads from `pb - sh` the compiler once formed an SMEM base of
        // (aligned - 1) + offset 1, which reads the wrong dword; volatile
        // loads, the earlier cure, waited for memory one dword at a time)
        const uint32_t *w = reinterpret_cast<const uint32_t *>(reinterpret_cast<uintptr_t>(pb) & ~uintptr_t(3));
#pragma unroll
        for (int k = 0; k <= kW; ++k) t[k] = w[k];
      } else {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(pb - sh);  // global, not flat
#pragma unroll
        for (int k = 0; k <= kW; ++k) t[k] = w[k];
      }
#pragma unroll
      for (int k = 0; k < kW; ++k) cache[k] = sh ? vts_alignbyte(t[k + 1], t[k], sh) : t[k];
      cache_at = blk;
    }
    const int32_t o = i - blk, q = o >> 2, r = o & 3;
    return vts_alignbyte(cache[q + 1], cache[q], r);
  }
  VTS_HD VTS_INLINE void refill() {  // requires nb <= 32
    const uint32_t v = load4(pos);
    const uint32_t x = v ^ 0x03030303u;
    if (pos + 4 <= size && !((x - 0x01010101u) & ~x & 0x80808080u)) {
      win |= static_cast<uint64_t>(__builtin_bswap32(v)) << (32 - nb);
      nb += 32;
      fill += 32;
      real += 32;
      pos += 4;
      zeros = (v >> 24) ? 0 : (((v >> 16) & 0xffu) ? 1 : 2);
      return;
    }
#pragma unroll 1
    for (int i = 0; i < 4; ++i) {
      if (pos >= size) {  // past the payload: zero padding, flagged if consumed
        nb += 8;
        fill += 8;
        continue;
      }
      const uint32_t b = (v >> (8 * i)) & 0xffu;
      ++pos;
      if (zeros >= 2 && b == 3) {
        ++epb;
        zeros = 0;
        epb_next = real >> 3;
        continue;
      }
      zeros = b ? 0 : vts_min(zeros + 1, 2);
      win |= static_cast<uint64_t>(b) << (56 - nb);
      nb += 8;
      fill += 8;
      real += 8;
    }
  }
  VTS_HD VTS_INLINE void ensure(int n) {  // n <= 32
    while (nb < n) refill();
  }
  VTS_HD VTS_INLINE void skip(int n) {  // n < 64, n <= nb
    win <<= n;
    nb -= n;
  }
  VTS_HD VTS_INLINE uint32_t bits(int n) {  // n <= 32
    if (n == 0) return 0;
    ensure(n);
    const uint32_t v = static_cast<uint32_t>(win >> (64 - n));
    skip(n);
    return v;
  }
  VTS_HD VTS_INLINE uint32_t bit() { return bits(1); }
  VTS_HD VTS_INLINE uint32_t ue() {
    ensure(32);
    const uint32_t p = static_cast<uint32_t>(win >> 32);
    if (p == 0) {  // more than 31 leading zeros
      err = true;
      return 0;
    }
    const int lz = __builtin_clz(p);
    if (lz < 16) {
      const int len = 2 * lz + 1;
      skip(len);
      return (p >> (32 - len)) - 1u;
    }
    skip(lz + 1);
    return ((1u << lz) - 1u) + bits(lz);
  }
  VTS_HD VTS_INLINE int32_t se() {
    const uint32_t k = ue();
    return (k & 1u) ? static_cast<int32_t>((k + 1) >> 1) : -static_cast<int32_t>(k >> 1);
  }
  VTS_HD VTS_INLINE int32_t consumed() const { return fill - nb; }  // RBSP bit index
  VTS_HD VTS_INLINE void align() { skip(nb & 7); }                  // fill is a multiple of 8
  VTS_HD VTS_INLINE bool overrun() const { return consumed() > real; }
  // more_rbsp_data(): the next bit lies before the stop bit.  stop_byte /
  // stop_bit are in the payload (EBSP) domain.  While the window has not
  // reached the stop byte the answer is yes (next bit <= 8 pos < 8 stop_byte
  // <= stop_bit); once it has, every EPB before it has been removed and the
  // stop bit's RBSP index is stop_bit - 8 * epb.
  VTS_HD VTS_INLINE bool more(int32_t stop_byte, int64_t stop_bit) const {
    if (pos < stop_byte) return true;
    return consumed() < stop_bit - 8ll * epb;
  }
  // At a byte boundary: skip n raw bytes (I_PCM samples) and return the ES
  // offset of the first.  Sets epb_hit when an emulation-prevention byte was
  // removed at or after the skip start (it would lie inside the samples).
  VTS_HD VTS_INLINE int64_t skip_raw(int32_t n, bool &epb_hit) {
    const int32_t r = consumed() >> 3;  // RBSP byte index (byte aligned)
    epb_hit = epb_next >= r;
    const int32_t e = r + epb;          // EBSP index: every removed EPB precedes r
    const int64_t off = abs0 + e;
    reset_at(e + n, (r + n) * 8);
    return off;
  }
  // drop the window and continue at payload byte e (RBSP bit index rb)
  VTS_HD VTS_INLINE void reset_at(int32_t e, int32_t rb) {
    pos = e;
    if (pos > size) err = true;
    win = 0;
    nb = 0;
    fill = real = rb;
    const uint32_t w = load4(vts_max(pos - 2, 0));
    const uint32_t b2 = w & 0xffu, b1 = (w >> 8) & 0xffu;
    zeros = (b1 != 0) ? 0 : ((b2 != 0) ? 1 : 2);
  }
};
using WinBits = WinBitsT<5>;

VTS_HD VTS_INLINE int median3(int a, int b, int c) {
  return vts_max(vts_min(a, b), vts_min(vts_max(a, b), c));
}

struct Nb {
  bool avail;
  int ref;
  int mvx, mvy;
};

VTS_HD VTS_INLINE Nb nb_from_cmd(uint64_t c) {
  Nb n{true, -1, 0, 0};
  if ((c >> 62) == 2) {
    n.ref = 0;
    n.mvx = static_cast<int16_t>(c & 0xffff);
    n.mvy = static_cast<int16_t>((c >> 16) & 0xffff);
  }
  return n;
}

// Macroblock commands of one slice, written 32 bytes (4 commands) at a time:
// a lane writing single 8-byte commands at a 640-byte stride from its
// neighbours (one slice per macroblock row) cost 4x the bytes in HBM write
// requests.  Groups are aligned on the absolute command index; partial groups
// (slice edges) fall back to 8-byte stores.
struct CmdWriter {
  uint64_t *cmd;      // frame base
  Cmd2 *e;            // the open group's 4 commands: per-lane scratch (LDS on the device)
  int64_t gbase;      // absolute index (slot * nmb) of cmd[0], for alignment
  uint64_t tag;       // the run's epoch, in bits 48-61 of every command
  int32_t g;          // first frame-relative index of the open group
  uint32_t mask;

  VTS_HD VTS_INLINE void init(uint64_t *c, int64_t gb, Cmd2 *scratch, uint64_t epoch_tag) {
    cmd = c;
    e = scratch;
    tag = epoch_tag;
    gbase = gb;
    g = -1;
    mask = 0;
  }
  VTS_HD VTS_INLINE void flush() {
    if (!mask) return;
    uint64_t *p = cmd + g;
    if (mask == 0xfu) {
      Cmd2 *q = reinterpret_cast<Cmd2 *>(p);  // two 16-byte stores
      q[0] = e[0];
      q[1] = e[1];
    } else {
      const uint64_t *el = reinterpret_cast<const uint64_t *>(e);
      if (mask & 1u) p[0] = el[0];
      if (mask & 2u) p[1] = el[1];
      if (mask & 4u) p[2] = el[2];
      if (mask & 8u) p[3] = el[3];
    }
    mask = 0;
  }
  VTS_HD VTS_INLINE void put(int32_t addr, uint64_t c) {
    const int32_t j = static_cast<int32_t>((gbase + addr) & 3);
    const int32_t ga = addr - j;
    if (ga != g) {
      flush();
      g = ga;
    }
    reinterpret_cast<uint64_t *>(e)[j] = c | tag;
    mask |= 1u << j;
    if (j == 3) flush();
  }
  // command of an earlier macroblock of the slice (neighbour B / C / D)
  VTS_HD VTS_INLINE uint64_t get(int32_t addr) const {
    // both loads, then a select of values: a select of the two pointers
    // would make one flat load (LDS or global)
    const uint64_t in_group = reinterpret_cast<const uint64_t *>(e)[(addr - g) & 3];
    const uint64_t in_memory = cmd[addr];
    return (mask && addr >= g && addr < g + 4) ? in_group : in_memory;
  }
};

// Parse one slice NAL (header byte at es + nal_offset, nal_size bytes) of the
// frame in `slot` into cmd_all[slot * nmb + mb], tagged with `epoch`.
// Returns DEC_E_* bits.
// `scratch` is the lane's private ParseScratch (LDS in h264_parse).
struct ParseScratch {
  Cmd2 cmd[2];         // open command group
  uint32_t cache[6];   // bit reader's byte cache (5 words used)
};

VTS_HD VTS_INLINE uint32_t parse_slice(const uint8_t *es, int64_t nal_offset, int32_t nal_size, int32_t slot,
                                       int32_t ref_slot, const H264DevParams &P, uint64_t *cmd_all,
                                       ParseScratch *scratch, uint32_t epoch = 0) {
  const int nmb = P.mb_width * P.mb_height;
  CmdWriter out;
  out.init(cmd_all + static_cast<int64_t>(slot) * nmb, static_cast<int64_t>(slot) * nmb, scratch->cmd,
           static_cast<uint64_t>(epoch) << kCmdEpochShift);
  uint32_t errs = 0;

  const uint8_t *nal = es + nal_offset;
  const uint32_t hdr = nal[0];
  const int nal_type = hdr & 0x1f, nal_ref_idc = (hdr >> 5) & 3;
  WinBits br;
  br.init(nal + 1, nal_offset + 1, nal_size - 1, scratch->cache);
  // stop bit (rbsp_trailing_bits): last non-zero byte of the NAL
  int32_t last = nal_size - 1;
  while (last > 0 && nal[last] == 0) --last;
  if (last <= 0) return DEC_E_SYNTAX;
  const uint32_t lb = nal[last];
  const int tz = __builtin_ctz(lb);
  const int32_t stop_byte = last - 1;                          // payload domain
  const int64_t stop_bit = int64_t(stop_byte) * 8 + (7 - tz);

  // ---- slice_header (7.3.3)
  const int first_mb = static_cast<int>(br.ue());
  int slice_type = static_cast<int>(br.ue());
  if (slice_type > 4) slice_type -= 5;
  const int pps_id = static_cast<int>(br.ue());
  if (pps_id != P.pps_id) errs |= DEC_E_PPS;
  br.bits(P.log2_max_frame_num);  // frame_num
  if (nal_type == 5) br.ue();      // idr_pic_id
  if (P.poc_type == 0) {
    br.bits(P.log2_max_poc_lsb);
    if (P.bottom_field_pic_order_in_frame_present) br.se();
  } else if (P.poc_type == 1 && !P.delta_pic_order_always_zero) {
    br.se();
    if (P.bottom_field_pic_order_in_frame_present) br.se();
  }
  if (P.redundant_pic_cnt_present) {
    if (br.ue() != 0) errs |= DEC_E_SYNTAX;  // redundant slices are not decoded
  }
  const bool is_p = (slice_type == 0);
  if (!is_p && slice_type != 2) errs |= DEC_E_SLICE_TYPE;
  int num_ref = P.num_ref_idx_l0_default_active;
  if (is_p) {
    if (br.bit()) num_ref = static_cast<int>(br.ue()) + 1;  // override
    if (br.bit()) errs |= DEC_E_REFLIST;                     // ref_pic_list_modification
    if (num_ref != 1) errs |= DEC_E_MULTIREF;
    if (ref_slot < 0) errs |= DEC_E_NO_REF;
  }
  if (nal_ref_idc != 0) {  // dec_ref_pic_marking
    if (nal_type == 5) {
      br.bit();
      br.bit();
    } else if (br.bit()) {
      errs |= DEC_E_MMCO;
    }
  }
  const int qp = P.pic_init_qp + br.se();
  int deblock_idc = 0, alpha_off = 0;
  if (P.deblocking_filter_control_present) {
    deblock_idc = static_cast<int>(br.ue());
    if (deblock_idc != 1) {
      alpha_off = 2 * br.se();
      br.se();
    }
  }
  // Filtering is a no-op only if disabled or every edge's indexA < 16
  // (alpha' = 0): max qPav is the slice QP (I_PCM has qP 0); chroma edges use
  // QPc(QP + chroma_qp_index_offset), which is >= 16 exactly when
  // QP + offset is (QPc(x) = x below 30, >= 29 above).
  const int cqp_up = P.chroma_qp_index_offset > 0 ? P.chroma_qp_index_offset : 0;
  if (deblock_idc != 1 && qp + cqp_up + alpha_off >= 16) errs |= DEC_E_DEBLOCK;
  if (first_mb < 0 || first_mb >= nmb) errs |= DEC_E_SYNTAX;
  if (errs || br.err || br.overrun()) return errs | ((br.err || br.overrun()) ? DEC_E_SYNTAX : 0u);

  // ---- slice_data (7.3.4), CAVLC
  int addr = first_mb;
  const int mbw = P.mb_width;
  int x = addr % mbw, y = addr / mbw;  // position of addr, advanced incrementally
  Nb left{false, -1, 0, 0};  // neighbour A of the current MB within the slice
  bool more = true;
  bool fresh = false;        // window empty at a byte boundary right after I_PCM samples
  while (more && addr < nmb) {
    if (is_p) {
      const int skip = static_cast<int>(br.ue());  // mb_skip_run
      if (br.err || addr + skip > nmb) {
        errs |= DEC_E_SYNTAX;
        break;
      }
      for (int i = 0; i < skip; ++i) {
        // P_Skip motion (8.4.1.1)
        const bool a_ok = x > 0 && addr - 1 >= first_mb;
        const bool b_ok = y > 0 && addr - mbw >= first_mb;
        int mvx = 0, mvy = 0;
        if (a_ok && b_ok) {
          const Nb A = left;
          const Nb B = nb_from_cmd(out.get(addr - mbw));
          if (!(A.ref == 0 && A.mvx == 0 && A.mvy == 0) && !(B.ref == 0 && B.mvx == 0 && B.mvy == 0)) {
            const bool c_ok = x < mbw - 1 && addr - mbw + 1 >= first_mb;
            const bool d_ok = x > 0 && addr - mbw - 1 >= first_mb;
            const Nb C = c_ok ? nb_from_cmd(out.get(addr - mbw + 1))
                              : (d_ok ? nb_from_cmd(out.get(addr - mbw - 1)) : Nb{false, -1, 0, 0});
            const int match = (A.ref == 0) + (B.ref == 0) + (C.ref == 0);
            if (match == 1) {
              mvx = (A.ref == 0) ? A.mvx : (B.ref == 0) ? B.mvx : C.mvx;
              mvy = (A.ref == 0) ? A.mvy : (B.ref == 0) ? B.mvy : C.mvy;
            } else {
              mvx = median3(A.mvx, B.mvx, C.mvx);
              mvy = median3(A.mvy, B.mvy, C.mvy);
            }
          }
        }
        if ((mvx & 3) || (mvy & 3)) errs |= DEC_E_SUBPEL;
        out.put(addr, MB_INTER | (uint64_t(uint16_t(mvx))) | (uint64_t(uint16_t(mvy)) << 16));
        left = Nb{true, 0, mvx, mvy};
        ++addr;
        if (++x == mbw) {
          x = 0;
          ++y;
        }
      }
      if (skip > 0) {
        more = br.more(stop_byte, stop_bit);
        fresh = false;
      }
      if (!more || addr >= nmb) break;
    }
    // ---- I_PCM run speculation: in an I slice, right after an I_PCM
    // macroblock, the next headers sit at a 386-byte stride (mb_type 25 =
    // 9 bits + 7 alignment zeros = 0x0D 0x00, then 384 samples).  Load up to
    // 8 predicted headers at once, verify them in order, commit the matching
    // prefix; anything unexpected falls through to the serial parse below.
    if (!is_p && fresh) {
      uint32_t hit = 0;  // bit j: header j is in range and reads 0x0D 0x00
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t q = static_cast<int64_t>(br.pos) + 386 * j;
        if ((q + 386) * 8 <= stop_bit && addr + j < nmb && nal[1 + q] == 0x0D && nal[2 + q] == 0x00)
          hit |= 1u << j;
      }
      const int ok = __builtin_ctz(~hit);  // matching prefix
      if (ok > 0 && br.zeros < 2) {
        for (int j = 0; j < ok; ++j)
          out.put(addr + j, MB_PCM | static_cast<uint64_t>(br.abs0 + br.pos + 386 * j + 2));
        addr += ok;
        x += ok;
        while (x >= mbw) {
          x -= mbw;
          ++y;
        }
        left = Nb{true, -1, 0, 0};
        br.reset_at(br.pos + 386 * ok, br.consumed() + 386 * 8 * ok);
        more = br.more(stop_byte, stop_bit);
        continue;
      }
    }
    fresh = false;
    // ---- macroblock_layer (7.3.5)
    const int mb_type = static_cast<int>(br.ue());
    if ((!is_p && mb_type == 25) || (is_p && mb_type == 30)) {
      br.align();
      bool hit = false;
      const int64_t off = br.skip_raw(384, hit);
      if (hit) errs |= DEC_E_EPB_IN_PCM;
      out.put(addr, MB_PCM | static_cast<uint64_t>(off));
      left = Nb{true, -1, 0, 0};
      fresh = true;
    } else if (is_p && mb_type == 0) {
      // P_L0_16x16: ref_idx_l0 absent (single reference), mvd_l0, cbp
      const int mvdx = br.se(), mvdy = br.se();
      const uint32_t cbp_code = br.ue();
      if (cbp_code != 0) errs |= DEC_E_RESIDUAL;
      const bool a_ok = x > 0 && addr - 1 >= first_mb;
      const bool b_ok = y > 0 && addr - mbw >= first_mb;
      const bool c_ok = y > 0 && x < mbw - 1 && addr - mbw + 1 >= first_mb;
      const bool d_ok = y > 0 && x > 0 && addr - mbw - 1 >= first_mb;
      Nb A = a_ok ? left : Nb{false, -1, 0, 0};
      Nb B = b_ok ? nb_from_cmd(out.get(addr - mbw)) : Nb{false, -1, 0, 0};
      Nb C = c_ok ? nb_from_cmd(out.get(addr - mbw + 1))
                  : (d_ok ? nb_from_cmd(out.get(addr - mbw - 1)) : Nb{false, -1, 0, 0});
      if (!B.avail && !C.avail && A.avail) B = C = A;
      int px, py;
      const int match = (A.ref == 0) + (B.ref == 0) + (C.ref == 0);
      if (match == 1) {
        px = (A.ref == 0) ? A.mvx : (B.ref == 0) ? B.mvx : C.mvx;
        py = (A.ref == 0) ? A.mvy : (B.ref == 0) ? B.mvy : C.mvy;
      } else {
        px = median3(A.mvx, B.mvx, C.mvx);
        py = median3(A.mvy, B.mvy, C.mvy);
      }
      const int mvx = px + mvdx, mvy = py + mvdy;
      if ((mvx & 3) || (mvy & 3)) errs |= DEC_E_SUBPEL;
      if (mvx < -32768 || mvx > 32767 || mvy < -32768 || mvy > 32767) errs |= DEC_E_SYNTAX;
      out.put(addr, MB_INTER | (uint64_t(uint16_t(mvx))) | (uint64_t(uint16_t(mvy)) << 16));
      left = Nb{true, 0, mvx, mvy};
    } else {
      errs |= DEC_E_MB_TYPE;
      break;
    }
    ++addr;
    if (++x == mbw) {
      x = 0;
      ++y;
    }
    if (br.err || br.overrun()) break;
    more = br.more(stop_byte, stop_bit);
  }
  out.flush();
  if (br.err || br.overrun()) errs |= DEC_E_SYNTAX;
  return errs;
}

}  // namespace vts
