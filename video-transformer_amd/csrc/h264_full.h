// h264_full.h — data shared by the host scheduler (h264_sched.cpp), the
// general device decoder (decode_full.hip) and its CPU harness
// (tests/native/full_host.cpp): the per-slice descriptor the host builds from
// the slice headers, and the per-macroblock record the slice parser writes
// for the reconstruction and deblocking kernels.
//
// The general path decodes progressive 4:2:0 8-bit streams: CAVLC I / P / B
// slices, CABAC I / P slices, 8x8 transforms, explicit and implicit weighted
// prediction, spatial and temporal direct prediction (Baseline without
// FMO/ASO/redundant pictures, Main, High without scaling matrices or
// interlace); DESIGN.md §5b.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define VTS_HD_FULL __host__ __device__
#else
#define VTS_HD_FULL
#endif

namespace vts {

// Slice of a window, as scheduled by the host (window-relative indices).
struct FullSlice {
  int64_t nal_offset;   // NAL header byte inside the device ES buffer
  int32_t nal_size;     // bytes including the header byte
  int32_t slot;         // ring slot of the picture
  int32_t first_mb;
  int32_t data_byte;    // slice_data(): EBSP byte of the payload (after the header byte)
  int32_t data_bit;     // ... and its RBSP bit index
  int32_t is_p;         // 0 I slice, 1 P slice, 2 B slice (kSliceB)
  int32_t qp;           // SliceQPY
  int32_t num_ref;      // num_ref_idx_l0_active (P, B)
  int32_t dbk_idc;      // disable_deblocking_filter_idc
  int32_t dbk_a, dbk_b; // FilterOffsetA / FilterOffsetB
  uint32_t arena;       // CAVLC: first coefficient block reserved for the slice
  uint32_t arena_cap;   // CAVLC: blocks reserved: min(27 x MBs, 3 x NAL bytes + 27) bounds
                        // what CAVLC can code (a stored block costs >= 3 bits).  CABAC
                        // slices take their blocks from the window's arena in chunks
                        // (kArenaChunk) and ignore both fields
  int32_t ext;          // SliceExt of a B slice or a weighted P slice, -1: none
  int16_t ref_slot[32]; // RefPicList0[i] -> ring slot (-1: no reference picture)
};
static_assert(sizeof(FullSlice) == 128, "FullSlice layout");
constexpr int32_t kSliceB = 2;

// What a B slice or an explicitly weighted P slice adds to FullSlice (the
// slices of one picture usually share one record: the host de-duplicates).
struct SliceExt {
  int32_t num_ref1;       // num_ref_idx_l1_active (B)
  int32_t direct_spatial; // direct_spatial_mv_pred_flag
  int32_t wmode;          // 0 default, 1 explicit (pred_weight_table), 2 implicit (8.4.2.3.1)
  int32_t lwd, cwd;       // luma / chroma_log2_weight_denom
  int32_t col_short;      // RefPicList1[0] is a short-term reference picture (colZeroFlag)
  int32_t poc;            // PicOrderCnt(CurrPic)
  uint32_t lt0, lt1;      // bit i: RefPicList0 / 1 [i] is a long-term reference picture
  int32_t _pad[3];
  int16_t ref_slot1[32];  // RefPicList1[i] -> ring slot
  int32_t poc0[32], poc1[32];  // PicOrderCnt of RefPicList0 / 1 [i]
  int16_t w[2][32][6];    // list, index: luma weight, luma offset, Cb weight, Cb offset, Cr weight, Cr offset
};
static_assert(sizeof(SliceExt) == 1136, "SliceExt layout");

struct FullParams {
  int32_t mb_width, mb_height;
  int32_t cip;          // constrained_intra_pred_flag
  int32_t cqp_off;      // chroma_qp_index_offset (Cb)
  int32_t cqp_off2;     // second_chroma_qp_index_offset (Cr)
  int32_t cabac;        // entropy_coding_mode_flag (parse_cabac.h)
  int32_t t8mode;       // transform_8x8_mode_flag
  int32_t bframes;      // the stream has B slices: every macroblock also writes an MbRecB
  int32_t direct8x8;    // direct_8x8_inference_flag
  int32_t has_ext;      // some slice has a SliceExt (B or weighted prediction)
  int32_t scaled;       // scaling matrices other than Flat_16: dequantise from ScaleTab
  int32_t _pad;
};

// Stored coefficient blocks of a macroblock, in parse order = bit order.
enum : uint32_t {
  kBlkI16Dc = 0,        // Intra16x16DCLevel (raster 4x4 of the 16 DC levels)
  kBlkLuma0 = 1,        // + luma4x4BlkIdx (Intra16x16ACLevel / LumaLevel4x4)
  kBlkChromaDc0 = 17,   // + iCbCr (4 levels in entries 0..3)
  kBlkChromaAc0 = 19,   // + 4 * iCbCr + chroma4x4BlkIdx
  kPcmBlocks = 12,      // I_PCM: 384 samples in 12 blocks (256 luma, 64 Cb, 64 Cr)
};

// CABAC: a slice takes coefficient blocks from its window's arena kArenaChunk
// at a time (one atomic add on the window's counter); a macroblock's blocks
// stay in one chunk (MbRec.coef + the popcount of MbRec.blocks below a block's
// bit addresses it), so a chunk with fewer than kMbMaxBlocks left is abandoned
constexpr uint32_t kArenaChunk = 256;
constexpr uint32_t kMbMaxBlocks = 27;  // 16 luma + Intra16x16 DC + 2 chroma DC + 8 chroma AC

// MbRec-parallel intra dependency level of a macroblock that is not intra-predicted
constexpr uint16_t kNoLevel = 0xffff;
constexpr uint8_t kModeT8 = 0x10;  // MbRec.modes: transform_size_8x8_flag

enum : uint8_t {
  kMbInter = 0,
  kMbI4x4 = 1,
  kMbI16 = 2,
  kMbPcm = 3,
  kMbSkip = 4,
};

// 8.5.9 LevelScale4x4 / LevelScale8x8 of a stream: weightScale (Flat_16, the
// Table 7-3 / 7-4 defaults or the stream's scaling lists after fall-back rules
// A and B, 7.4.2.1.1 / 7.4.2.2) times normAdjust.  ls4[list][qP % 6][raster]
// for lists 0..5 = Intra Y, Cb, Cr, Inter Y, Cb, Cr; ls8[list][qP % 6][raster
// 8x8] for lists 0, 1 = Intra Y, Inter Y (4:2:0).
struct ScaleTab {
  int32_t ls4[6][6][16];
  int32_t ls8[2][6][64];
};
// list of a 4x4 block: plane 0 Y, 1 Cb, 2 Cr of an intra or inter macroblock
VTS_HD_FULL inline int scale_list4(bool intra, int plane) { return (intra ? 0 : 3) + plane; }

// One decoded macroblock's syntax (128 bytes).
struct alignas(16) MbRec {
  uint32_t epoch;       // the run's epoch; another value = macroblock absent
  uint32_t slice;       // window slice index (availability: same slice)
  uint32_t coef;        // arena index of the first stored block
  uint32_t blocks;      // stored blocks (kBlk* bits)
  uint8_t type;         // kMb*
  uint8_t qp;           // QPY
  uint8_t cbp;          // coded_block_pattern
  uint8_t modes;        // bits 0-1 Intra16x16PredMode, bits 2-3 intra_chroma_pred_mode,
                        // bit 4 transform_size_8x8_flag (8x8 blocks: 4 consecutive arena
                        // blocks = raster 8x8, kBlkLuma0 + 4 b8 + 0..3 all set)
  int8_t ref[4];        // RefPicList0 index per 8x8 (-1: intra)
  int16_t ref_slot[4];  // its ring slot (the picture identity the deblocking bS compares)
  uint8_t i4[8];        // Intra4x4PredMode of raster 4x4 block b: nibble (b & 1) of byte b >> 1
                        // (Intra_8x8: the 8x8 mode in its four blocks); CABAC inter macroblocks:
                        // Min(|mvd|, 33) of bottom-row block x, component c at byte 2 x + c
  uint8_t nz[16];       // total_coeff of raster luma 4x4 blocks (16 for I_PCM)
  uint8_t nzc[8];       // CAVLC: chroma AC total_coeff, Cb raster 0-3, Cr raster 0-3;
                        // CABAC: bytes 0-3 the coded_block_flag bits (kBlk* numbering,
                        // luma 4x4 by raster index: bit 1 + raster)
  int16_t mv[16][2];    // quarter-sample motion of raster 4x4 blocks
};
static_assert(sizeof(MbRec) == 128, "MbRec layout");

// List-1 half of a macroblock's motion (streams with B slices; same indexing
// as MbRec).  I / P macroblocks: ref1 -1.
constexpr uint8_t kDirect16 = 0x10;  // MbRecB.direct: B_Skip / B_Direct_16x16
struct alignas(16) MbRecB {
  int8_t ref1[4];        // RefPicList1 index per 8x8 (-1: list 1 unused)
  int16_t ref_slot1[4];  // its ring slot
  uint8_t direct;        // bits 0-3: 8x8 quadrants predicted in direct mode; kDirect16
  uint8_t _p[3];
  uint8_t mvd1[8];       // CABAC: Min(|mvdL1|, 33) of bottom-row block x, component c at byte 2 x + c
  uint8_t _q[40];
  int16_t mv1[16][2];    // quarter-sample list-1 motion of raster 4x4 blocks
};
static_assert(sizeof(MbRecB) == 128, "MbRecB layout");

}  // namespace vts
