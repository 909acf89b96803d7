// h264.cpp — SPS / PPS parsing (ITU-T H.264 §7.3.2.1.1, §7.3.2.2).
#include "h264.h"

#include "bitstream.h"

namespace vts {

namespace {

bool is_high_profile(int p) {
  switch (p) {
    case 100: case 110: case 122: case 244: case 44: case 83: case 86:
    case 118: case 128: case 138: case 139: case 134: case 135:
      return true;
    default:
      return false;
  }
}

void skip_scaling_list(BitReader &br, int size) {  // §7.3.2.1.1.1
  int last = 8, next = 8;
  for (int j = 0; j < size; ++j) {
    if (next != 0) {
      const int delta = br.se();
      next = (last + delta + 256) % 256;
    }
    last = (next == 0) ? last : next;
  }
}

}  // namespace

std::string parse_sps(const uint8_t *nal, size_t n, Sps *s) {
  if (n < 4 || (nal[0] & 0x1f) != 7) return "not an SPS NAL";
  BitReader br(nal + 1, n - 1);
  s->profile_idc = static_cast<int>(br.u(8));
  s->constraint_flags = static_cast<int>(br.u(8));
  s->level_idc = static_cast<int>(br.u(8));
  s->sps_id = static_cast<int>(br.ue());
  if (is_high_profile(s->profile_idc)) {
    s->chroma_format_idc = static_cast<int>(br.ue());
    if (s->chroma_format_idc == 3) br.u(1);
    s->bit_depth_luma = 8 + static_cast<int>(br.ue());
    s->bit_depth_chroma = 8 + static_cast<int>(br.ue());
    br.u(1);  // qpprime_y_zero_transform_bypass_flag
    if (br.u(1)) {  // seq_scaling_matrix_present_flag
      const int lists = (s->chroma_format_idc != 3) ? 8 : 12;
      for (int i = 0; i < lists; ++i)
        if (br.u(1)) skip_scaling_list(br, i < 6 ? 16 : 64);
    }
  }
  if (s->chroma_format_idc != 1) return "only 4:2:0 chroma is supported";
  if (s->bit_depth_luma != 8 || s->bit_depth_chroma != 8) return "only 8-bit video is supported";
  s->log2_max_frame_num = 4 + static_cast<int>(br.ue());
  s->poc_type = static_cast<int>(br.ue());
  if (s->poc_type == 0) {
    s->log2_max_poc_lsb = 4 + static_cast<int>(br.ue());
  } else if (s->poc_type == 1) {
    s->delta_pic_order_always_zero = static_cast<int>(br.u(1));
    s->offset_for_non_ref_pic = br.se();
    s->offset_for_top_to_bottom_field = br.se();
    const uint32_t cyc = br.ue();
    if (cyc > 255) return "bad num_ref_frames_in_pic_order_cnt_cycle";
    s->offset_for_ref_frame.clear();
    for (uint32_t i = 0; i < cyc; ++i) s->offset_for_ref_frame.push_back(br.se());
  } else if (s->poc_type != 2) {
    return "bad pic_order_cnt_type";
  }
  s->max_num_ref_frames = static_cast<int>(br.ue());
  s->gaps_allowed = static_cast<int>(br.u(1));
  s->mb_width = 1 + static_cast<int>(br.ue());
  const int map_units = 1 + static_cast<int>(br.ue());
  s->frame_mbs_only = static_cast<int>(br.u(1));
  if (!s->frame_mbs_only) return "interlaced (field) coding is not supported";
  s->mb_height = map_units;
  s->direct_8x8_inference = static_cast<int>(br.u(1));
  if (br.u(1)) {  // frame_cropping_flag; 4:2:0 crop units are 2 samples
    s->crop_left = 2 * static_cast<int>(br.ue());
    s->crop_right = 2 * static_cast<int>(br.ue());
    s->crop_top = 2 * static_cast<int>(br.ue());
    s->crop_bottom = 2 * static_cast<int>(br.ue());
  }
  if (!br.ok()) return "truncated SPS";
  if (s->mb_width <= 0 || s->mb_height <= 0 || s->mb_width > 1024 || s->mb_height > 1024)
    return "bad picture size";
  if (s->width() <= 0 || s->height() <= 0) return "bad cropping";
  return "";
}

std::string parse_pps(const uint8_t *nal, size_t n, Pps *p) {
  if (n < 2 || (nal[0] & 0x1f) != 8) return "not a PPS NAL";
  BitReader br(nal + 1, n - 1);
  p->pps_id = static_cast<int>(br.ue());
  p->sps_id = static_cast<int>(br.ue());
  p->entropy_coding_mode = static_cast<int>(br.u(1));  // CABAC: the general decoder only
  p->bottom_field_pic_order_in_frame_present = static_cast<int>(br.u(1));
  p->num_slice_groups = 1 + static_cast<int>(br.ue());
  if (p->num_slice_groups != 1) return "slice groups (FMO) are not supported";
  p->num_ref_idx_l0_default_active = 1 + static_cast<int>(br.ue());
  p->num_ref_idx_l1_default_active = 1 + static_cast<int>(br.ue());
  p->weighted_pred = static_cast<int>(br.u(1));
  p->weighted_bipred_idc = static_cast<int>(br.u(2));
  p->pic_init_qp = 26 + br.se();
  br.se();  // pic_init_qs_minus26
  p->chroma_qp_index_offset = br.se();
  p->deblocking_filter_control_present = static_cast<int>(br.u(1));
  p->constrained_intra_pred = static_cast<int>(br.u(1));
  p->redundant_pic_cnt_present = static_cast<int>(br.u(1));
  if (!br.ok()) return "truncated PPS";
  p->has_tail = br.more_rbsp_data() ? 1 : 0;
  if (p->weighted_bipred_idc > 2) return "bad weighted_bipred_idc";
  return "";
}

H264DevParams make_dev_params(const Sps &sps, const Pps &pps) {
  H264DevParams d{};
  d.mb_width = sps.mb_width;
  d.mb_height = sps.mb_height;
  d.log2_max_frame_num = sps.log2_max_frame_num;
  d.poc_type = sps.poc_type;
  d.log2_max_poc_lsb = sps.log2_max_poc_lsb;
  d.delta_pic_order_always_zero = sps.delta_pic_order_always_zero;
  d.bottom_field_pic_order_in_frame_present = pps.bottom_field_pic_order_in_frame_present;
  d.num_ref_idx_l0_default_active = pps.num_ref_idx_l0_default_active;
  d.redundant_pic_cnt_present = pps.redundant_pic_cnt_present;
  d.deblocking_filter_control_present = pps.deblocking_filter_control_present;
  d.pic_init_qp = pps.pic_init_qp;
  d.chroma_qp_index_offset = pps.chroma_qp_index_offset;
  d.pps_id = pps.pps_id;
  return d;
}

std::string describe_decode_error(uint32_t f) {
  static const char *names[] = {
      "B/SP/SI slice", "macroblock type outside subset", "residual coefficients",
      "fractional luma motion", "multiple references", "bitstream syntax error",
      "active deblocking filter", "unknown PPS id", "macroblock not covered by any slice",
      "emulation prevention inside I_PCM samples", "reference list modification",
      "P slice without reference frame", "adaptive reference marking (MMCO)",
      "B slice's wait for its colocated picture's parse timed out",
      "coefficient arena range of a slice exceeded",
      "per-picture reconstruction scheduler: a reference picture never finished"};
  std::string s;
  for (int i = 0; i < 16; ++i)
    if (f & (1u << i)) {
      if (!s.empty()) s += ", ";
      s += names[i];
    }
  return s.empty() ? "ok" : s;
}

}  // namespace vts
