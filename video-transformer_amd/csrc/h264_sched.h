// h264_sched.h — host side of the general decoder: full slice-header parsing
// (7.3.3) and the reference picture bookkeeping of the whole stream (8.2.4
// list initialisation / modification, 8.2.5 sliding window and MMCO), so the
// device parser receives each slice's RefPicList0 as frame indices and starts
// at slice_data().  Also gives every frame the frames it may reference, from
// which the session builds its level schedule.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "h264.h"
#include "h264_full.h"

namespace vts {

struct SchedSlice {
  int64_t frame;
  int64_t nal_offset;   // NAL header byte inside the stream's ES buffer
  int32_t nal_size;
  int32_t first_mb, n_mbs;
  int32_t data_byte;    // slice_data(): EBSP byte of the payload (after the header byte)
  int32_t data_bit;     // ... RBSP bit index
  int32_t is_p, qp, num_ref;  // is_p: 0 I, 1 P, 2 B
  int32_t dbk_idc, dbk_a, dbk_b;
  int64_t ref[32];      // RefPicList0[i] as a frame index, -1 = no reference picture
  // B slices and weighted prediction (h264_full.h SliceExt)
  int32_t num_ref1 = 0, direct_spatial = 0;
  int32_t wmode = 0;    // 0 default, 1 explicit, 2 implicit
  int32_t lwd = 0, cwd = 0;
  int32_t poc = 0;      // PicOrderCnt of the picture
  int32_t col_short = 0;
  uint32_t lt0 = 0, lt1 = 0;
  int64_t ref1[32];     // RefPicList1
  int32_t poc0[32], poc1[32];
  int16_t w[2][32][6];  // pred_weight_table (defaults where absent)
  bool needs_ext() const { return is_p == 2 || wmode != 0; }
};

struct SchedFrame {
  int64_t s0 = 0, ns = 0;   // slices [s0, s0 + ns)
  bool intra = true;        // every slice is an I slice
  bool is_ref = false;      // nal_ref_idc != 0
  bool has_b = false;       // a B slice (direct prediction reads the colocated picture's motion)
  int32_t poc = 0;          // PicOrderCnt after the picture (0 after memory_management_control_operation 5)
  std::vector<int64_t> refs;  // distinct frames in any slice's active RefPicList0 / 1
  std::vector<int64_t> cols;  // distinct RefPicList1[0] of its B slices
};

// Stream facts the general path needs beyond h264.h's Sps / Pps.
// (B slices come with PicOrderCnt 8.2.1, list initialisation 8.2.4.2.3 and
// pred_weight_table 7.3.3.2.)
struct SchedStream {
  int seq_scaling = 0;       // seq_scaling_matrix_present_flag
  int transform_8x8 = 0;     // PPS transform_8x8_mode_flag
  int pic_scaling = 0;       // pic_scaling_matrix_present_flag
  int cqp_off2 = 0;          // second_chroma_qp_index_offset (= chroma_qp_index_offset if absent)
  ScaleTab scale;            // LevelScale4x4 / 8x8 of the active SPS + PPS (flat without matrices)
};

// weightScale4x4 / 8x8 in raster order (w4[list][16], w8[list][64]) -> LevelScale
void scale_tab_build(const uint8_t (*w4)[16], const uint8_t (*w8)[64], ScaleTab *t);

// Parse the High-profile PPS extension (more_rbsp_data part) and the SPS
// scaling flag; "" or the reason the general decoder cannot take the stream.
std::string sched_stream_facts(const std::vector<uint8_t> &sps_nal, const std::vector<uint8_t> &pps_nal,
                               const Sps &sps, const Pps &pps, SchedStream *out);

// frames: per sample (access unit) the byte range [off, off + size) of its
// AVCC NAL units (nal_length_size prefix) inside `es`.  "" or the reason.
std::string sched_build(const Sps &sps, const Pps &pps, const uint8_t *es, const std::vector<int64_t> &off,
                        const std::vector<uint32_t> &size, int nal_length_size,
                        std::vector<SchedFrame> *frames, std::vector<SchedSlice> *slices);

}  // namespace vts
