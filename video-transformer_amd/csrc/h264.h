// h264.h — H.264 parameter sets (host side) and the flattened stream
// parameters the device-side slice parser consumes.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace vts {

struct Sps {
  int profile_idc = 0, constraint_flags = 0, level_idc = 0, sps_id = 0;
  int chroma_format_idc = 1, bit_depth_luma = 8, bit_depth_chroma = 8;
  int log2_max_frame_num = 4, poc_type = 0, log2_max_poc_lsb = 4;
  int delta_pic_order_always_zero = 0;
  int offset_for_non_ref_pic = 0, offset_for_top_to_bottom_field = 0;  // POC type 1 (7.4.2.1.1)
  std::vector<int> offset_for_ref_frame;
  int direct_8x8_inference = 1;
  int max_num_ref_frames = 0, gaps_allowed = 0;
  int mb_width = 0, mb_height = 0, frame_mbs_only = 1;
  int crop_left = 0, crop_right = 0, crop_top = 0, crop_bottom = 0;  // luma samples
  int width() const { return mb_width * 16 - crop_left - crop_right; }
  int height() const { return mb_height * 16 - crop_top - crop_bottom; }
};

struct Pps {
  int pps_id = 0, sps_id = 0, entropy_coding_mode = 0;
  int bottom_field_pic_order_in_frame_present = 0, num_slice_groups = 1;
  int num_ref_idx_l0_default_active = 1, num_ref_idx_l1_default_active = 1;
  int weighted_pred = 0, weighted_bipred_idc = 0, pic_init_qp = 26;
  int chroma_qp_index_offset = 0, deblocking_filter_control_present = 0;
  int constrained_intra_pred = 0, redundant_pic_cnt_present = 0;
  // the High-profile tail (transform_8x8_mode_flag, pic scaling matrix,
  // second_chroma_qp_index_offset) is present: general decoder only
  int has_tail = 0;
};

// Parse an SPS/PPS NAL unit (payload including the one-byte NAL header).
// Return "" on success, else the reason the stream is outside the decoder's
// subset or malformed.
std::string parse_sps(const uint8_t *nal, size_t n, Sps *out);
std::string parse_pps(const uint8_t *nal, size_t n, Pps *out);

// Everything the device slice parser needs, in one POD passed by value.
struct H264DevParams {
  int32_t mb_width, mb_height;
  int32_t log2_max_frame_num;
  int32_t poc_type;
  int32_t log2_max_poc_lsb;
  int32_t delta_pic_order_always_zero;
  int32_t bottom_field_pic_order_in_frame_present;
  int32_t num_ref_idx_l0_default_active;
  int32_t redundant_pic_cnt_present;
  int32_t deblocking_filter_control_present;
  int32_t pic_init_qp;
  int32_t chroma_qp_index_offset;
  int32_t pps_id;
  int32_t _pad;
};

H264DevParams make_dev_params(const Sps &sps, const Pps &pps);

// The subset the device decoder implements (checked per slice on the device):
//   CAVLC, frames only, one SPS/PPS, single reference (refIdx 0),
//   I slices of I_PCM macroblocks; P slices of P_Skip, P_L0_16x16 with
//   integer-pel luma motion and coded_block_pattern 0, and I_PCM;
//   in-loop deblocking disabled (disable_deblocking_filter_idc == 1) or
//   provably inactive (every edge's indexA < 16, so alpha == 0).
enum DecodeError : uint32_t {
  DEC_OK = 0,
  DEC_E_SLICE_TYPE = 1u << 0,     // B/SP/SI slice
  DEC_E_MB_TYPE = 1u << 1,        // macroblock type outside the subset
  DEC_E_RESIDUAL = 1u << 2,       // coded_block_pattern != 0
  DEC_E_SUBPEL = 1u << 3,         // fractional luma motion vector
  DEC_E_MULTIREF = 1u << 4,       // more than one active reference
  DEC_E_SYNTAX = 1u << 5,         // bitstream exhausted / malformed
  DEC_E_DEBLOCK = 1u << 6,        // active deblocking filter
  DEC_E_PPS = 1u << 7,            // unknown pic_parameter_set_id
  DEC_E_MISSING_MB = 1u << 8,     // a macroblock no slice covered
  DEC_E_EPB_IN_PCM = 1u << 9,     // emulation prevention inside PCM samples
  DEC_E_REFLIST = 1u << 10,       // ref_pic_list_modification / weighted pred
  DEC_E_NO_REF = 1u << 11,        // P slice without a preceding reference
  DEC_E_MMCO = 1u << 12,          // adaptive reference marking
  DEC_E_COL_WAIT = 1u << 13,      // merged parse: a B slice's wait for its colocated picture timed out
  DEC_E_ARENA = 1u << 14,         // a slice's coefficient blocks overflowed its arena range (the host
                                  // re-runs the window with the provable bound)
  DEC_E_SCHED = 1u << 15,         // h264_recon_sched: a wait for a reference picture never ended
  // not an error: a level-blocked reconstruct launch met a motion vector
  // reaching beyond its halo; the host re-runs with per-level launches
  DEC_W_LEVEL_RANGE = 1u << 31,
};
std::string describe_decode_error(uint32_t flags);

// Host-side stream writing helpers (synth.cpp), shared with the transcoder:
// Constrained Baseline SPS/PPS NAL units (pic_order_cnt_type 2, 16-bit
// frame_num, one reference, CAVLC, deblocking_filter_control_present) for an
// mbw x mbh macroblock picture cropped by crop_r / crop_b luma samples.
void make_sps_pps(int mbw, int mbh, int crop_r, int crop_b, int level, std::vector<uint8_t> *sps_nal,
                  std::vector<uint8_t> *pps_nal, int chroma_qp_index_offset = 0);
int h264_pick_level(int mbs, double mbps);

// MB command word written by the parser, read by the reconstruct kernel.
//   bits 62-63: 1 = I_PCM (bits 0-47 = byte offset of the 384 PCM bytes in the
//               device elementary-stream buffer), 2 = inter (bits 0-15 mvx,
//               16-31 mvy, quarter-pel, refIdx 0), 0 = not decoded.
constexpr uint64_t MB_PCM = 1ull << 62;
constexpr uint64_t MB_INTER = 2ull << 62;
// bits 48-61: the run's epoch (1..16383).  The reconstruct kernels treat a
// command whose epoch is not the current run's as absent (missing
// macroblock), so the command ring need not be cleared before every parse.
constexpr int kCmdEpochShift = 48;
constexpr uint64_t kCmdEpochMask = 0x3fffull << kCmdEpochShift;
constexpr uint32_t kCmdEpochs = 16383;

}  // namespace vts
