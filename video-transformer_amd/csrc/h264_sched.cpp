// h264_sched.cpp — slice headers and reference lists for the general decoder
// (see h264_sched.h).  ITU-T H.264 7.3.3 slice_header(), 7.3.3.1
// ref_pic_list_modification(), 7.3.3.2 pred_weight_table(), 7.3.3.3
// dec_ref_pic_marking(), 8.2.1 picture order count (types 0, 1, 2), 8.2.4
// (reference picture list initialisation for P and B slices in frames, and
// modification), 8.2.5 (IDR, sliding window, MMCO 1-6).
#include "h264_sched.h"

#include "h264_cabac_tables.h"
#include "h264_tables.h"

#include <algorithm>
#include <cstdio>
#include <cstring>

namespace vts {
namespace {

// RBSP reader over a NAL payload that also reports where it is in EBSP bytes
struct HdrReader {
  const uint8_t *p;
  int64_t n;
  int64_t pos = 0;   // next EBSP byte
  int zeros = 0;
  int bitpos = 0;    // bits left in cur
  uint32_t cur = 0;
  int64_t rbits = 0; // RBSP bits consumed
  bool err = false;
  HdrReader(const uint8_t *b, int64_t len) : p(b), n(len) {}
  uint32_t bit() {
    if (bitpos == 0) {
      if (pos >= n) {
        err = true;
        return 0;
      }
      uint32_t v = p[pos];
      if (zeros >= 2 && v == 3) {
        ++pos;
        zeros = 0;
        if (pos >= n) {
          err = true;
          return 0;
        }
        v = p[pos];
      }
      ++pos;
      zeros = v == 0 ? zeros + 1 : 0;
      cur = v;
      bitpos = 8;
    }
    --bitpos;
    ++rbits;
    return (cur >> bitpos) & 1u;
  }
  uint32_t u(int k) {
    uint32_t v = 0;
    for (int i = 0; i < k; ++i) v = (v << 1) | bit();
    return v;
  }
  uint32_t ue() {
    int lz = 0;
    while (!bit()) {
      if (++lz > 31 || err) {
        err = true;
        return 0;
      }
    }
    return lz ? ((1u << lz) - 1u + u(lz)) : 0u;
  }
  int32_t se() {
    const uint32_t k = ue();
    return (k & 1u) ? static_cast<int32_t>((k + 1) / 2) : -static_cast<int32_t>(k / 2);
  }
  // EBSP byte holding the next bit (for a mid-byte position: the current byte)
  int64_t ebsp_byte() const { return bitpos ? pos - 1 : pos; }
};

struct RefPic {
  int64_t frame;
  int frame_num;
  int lt_idx;
  int kind;  // 1 short-term, 2 long-term
  int poc;   // PicOrderCnt
};

bool more_rbsp(const std::vector<uint8_t> &nal, const HdrReader &r) {
  int64_t last = static_cast<int64_t>(nal.size()) - 1;
  while (last > 0 && nal[last] == 0) --last;
  if (last <= 0) return false;
  const int tz = __builtin_ctz(static_cast<uint32_t>(nal[last]));
  const int64_t stop = (last - 1) * 8 + (7 - tz);  // EBSP bit index in the payload
  const int64_t at = r.bitpos ? (r.pos - 1) * 8 + (8 - r.bitpos) : r.pos * 8;
  return at < stop;
}

const uint8_t kDef4[2][16] = VTS_DEFAULT_4x4_DATA;  // Tables 7-3 / 7-4 (scan order)
const uint8_t kDef8[2][64] = VTS_DEFAULT_8x8_DATA;

// 7.3.2.1.1.1 scaling_list(): n values in zig-zag order; true when
// useDefaultScalingMatrixFlag (the first delta leaves nextScale 0)
bool read_scaling_list(HdrReader &r, int n, uint8_t *list) {
  int last = 8, next = 8;
  bool use_default = false;
  for (int j = 0; j < n; ++j) {
    if (next != 0) {
      const int delta = r.se();
      next = (last + delta + 256) % 256;
      use_default = j == 0 && next == 0;
    }
    list[j] = static_cast<uint8_t>(next == 0 ? last : next);
    last = list[j];
  }
  return use_default;
}

// The scaling lists of one parameter set (7.4.2.1.1 / 7.4.2.2): lists 0..5
// 4x4, 6..7 8x8 (4:2:0), present_flag per list; absent lists take the
// fall-back of rule A (SPS: defaults and the previous list) or B (PPS:
// the sequence-level list `seq` for lists 0, 3, 6, 7)
void read_scaling_matrix(HdrReader &r, int n_lists, bool rule_b, const uint8_t (*seq4)[16],
                         const uint8_t (*seq8)[64], uint8_t (*l4)[16], uint8_t (*l8)[64]) {
  for (int i = 0; i < 8; ++i) {
    const bool present = i < n_lists && r.u(1);
    const int inter = (i >= 3 && i < 6) || i == 7 ? 1 : 0;
    if (i < 6) {
      if (present) {
        if (read_scaling_list(r, 16, l4[i])) std::memcpy(l4[i], kDef4[inter], 16);
      } else if (i == 0 || i == 3) {
        std::memcpy(l4[i], rule_b ? seq4[i] : kDef4[inter], 16);
      } else {
        std::memcpy(l4[i], l4[i - 1], 16);
      }
    } else {
      uint8_t *d = l8[i - 6];
      if (present) {
        if (read_scaling_list(r, 64, d)) std::memcpy(d, kDef8[inter], 64);
      } else {
        std::memcpy(d, rule_b ? seq8[i - 6] : kDef8[inter], 64);
      }
    }
  }
}

// 4x4 / 8x8 zig-zag (frame) scan: raster position of coefficient k
const uint8_t kZz4[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
const uint8_t kZz8[64] = VTS_ZZ8_DATA;  // 8.5.7 Table 8-13

}  // namespace

void scale_tab_build(const uint8_t (*w4)[16], const uint8_t (*w8)[64], ScaleTab *t) {
  static const int nv[6][3] = VTS_NORMV_DATA;  // normAdjust4x4 (8.5.9)
  static const int n8[6][6] = VTS_NORM8_DATA;  // normAdjust8x8
  for (int l = 0; l < 6; ++l)
    for (int m = 0; m < 6; ++m)
      for (int k = 0; k < 16; ++k) {
        const int i = k >> 2, j = k & 3;
        const int c = (!(i & 1) && !(j & 1)) ? 0 : (((i & 1) && (j & 1)) ? 1 : 2);
        t->ls4[l][m][k] = w4[l][k] * nv[m][c];
      }
  for (int l = 0; l < 2; ++l)
    for (int m = 0; m < 6; ++m)
      for (int k = 0; k < 64; ++k) {
        t->ls8[l][m][k] = w8[l][k] * n8[m][vts_norm8_class(k >> 3, k & 7)];
      }
}

std::string sched_stream_facts(const std::vector<uint8_t> &sps_nal, const std::vector<uint8_t> &pps_nal,
                               const Sps &sps, const Pps &pps, SchedStream *out) {
  *out = SchedStream{};
  out->cqp_off2 = pps.chroma_qp_index_offset;
  // scaling lists (zig-zag order): sequence level sl4 / sl8 (Flat_16 without
  // seq_scaling_matrix_present_flag), picture level pl4 / pl8
  uint8_t sl4[6][16], sl8[2][64], pl4[6][16], pl8[2][64];
  std::memset(sl4, 16, sizeof(sl4));
  std::memset(sl8, 16, sizeof(sl8));
  {  // SPS: seq_scaling_matrix_present_flag (High profiles only)
    HdrReader r(sps_nal.data() + 1, static_cast<int64_t>(sps_nal.size()) - 1);
    const int prof = static_cast<int>(r.u(8));
    r.u(16);
    r.ue();
    const bool high = prof == 100 || prof == 110 || prof == 122 || prof == 244 || prof == 44 ||
                      prof == 83 || prof == 86 || prof == 118 || prof == 128 || prof == 138 ||
                      prof == 139 || prof == 134 || prof == 135;
    if (high) {
      const uint32_t cf = r.ue();
      if (cf == 3) r.u(1);
      r.ue();
      r.ue();
      r.u(1);
      out->seq_scaling = static_cast<int>(r.u(1));
      if (out->seq_scaling) read_scaling_matrix(r, cf == 3 ? 12 : 8, false, nullptr, nullptr, sl4, sl8);
    }
  }
  {  // PPS: skip to the optional tail (7.3.2.2)
    HdrReader r(pps_nal.data() + 1, static_cast<int64_t>(pps_nal.size()) - 1);
    r.ue();
    r.ue();
    r.u(1);
    r.u(1);
    if (r.ue() != 0) return "slice groups (FMO)";
    r.ue();
    r.ue();
    r.u(1);
    r.u(2);
    r.se();
    r.se();
    r.se();
    r.u(3);
    std::memcpy(pl4, sl4, sizeof(pl4));
    std::memcpy(pl8, sl8, sizeof(pl8));
    if (more_rbsp(pps_nal, r)) {
      out->transform_8x8 = static_cast<int>(r.u(1));
      out->pic_scaling = static_cast<int>(r.u(1));
      // 7.4.2.2: fall-back rule B (the SPS's lists) only when the SPS has
      // its own matrix; rule A (Table 7-3 / 7-4 defaults) otherwise
      if (out->pic_scaling)
        read_scaling_matrix(r, 6 + 2 * out->transform_8x8, out->seq_scaling != 0, sl4, sl8, pl4, pl8);
      out->cqp_off2 = r.se();
    }
    if (r.err) return "truncated PPS";
  }
  // weightScale: the lists in raster order (inverse zig-zag), then LevelScale
  uint8_t w4[6][16], w8[2][64];
  for (int l = 0; l < 6; ++l)
    for (int k = 0; k < 16; ++k) w4[l][kZz4[k]] = pl4[l][k];
  for (int l = 0; l < 2; ++l)
    for (int k = 0; k < 64; ++k) w8[l][kZz8[k]] = pl8[l][k];
  scale_tab_build(w4, w8, &out->scale);
  if (out->transform_8x8 && !pps.entropy_coding_mode) return "8x8 transform with CAVLC (CABAC only)";
  if (pps.redundant_pic_cnt_present) return "redundant pictures";
  return "";
}

std::string sched_build(const Sps &sps, const Pps &pps, const uint8_t *es, const std::vector<int64_t> &off,
                        const std::vector<uint32_t> &size, int nal_len, std::vector<SchedFrame> *frames,
                        std::vector<SchedSlice> *slices) {
  const int nmb = sps.mb_width * sps.mb_height;
  const int max_fn = 1 << sps.log2_max_frame_num;
  const int max_refs = std::max(1, sps.max_num_ref_frames);
  std::vector<RefPic> dpb;
  int prev_ref_fn = 0;
  int max_lt_idx = -1;
  bool have_prev = false;
  // 8.2.1 state carried from the previous picture(s)
  int prev_poc_msb = 0, prev_poc_lsb = 0, prev_fn = 0, prev_fn_offset = 0;
  frames->assign(off.size(), SchedFrame{});
  slices->clear();
  char msg[160];
  for (size_t f = 0; f < off.size(); ++f) {
    SchedFrame &fr = (*frames)[f];
    fr.s0 = static_cast<int64_t>(slices->size());
    int64_t p = off[f];
    const int64_t end = p + size[f];
    bool first = true, idr = false, adaptive = false, lt_ref_flag = false;
    int fn = 0, cur_poc = 0, h_poc_lsb = 0, h_dbot = 0;
    std::vector<std::pair<int, int>> mmco;  // (op, arg) ; op 3/6 carry lt idx in arg2 below
    std::vector<int> mmco_arg2;
    while (p + nal_len <= end) {
      uint32_t len = 0;
      for (int i = 0; i < nal_len; ++i) len = (len << 8) | es[p + i];
      p += nal_len;
      if (len == 0 || p + len > end) return "bad NAL length";
      const uint8_t hdr = es[p];
      const int type = hdr & 31, ref_idc = (hdr >> 5) & 3;
      if (type != 1 && type != 5) {
        if (type >= 2 && type <= 4) return "data partitioning";
        p += len;
        continue;
      }
      HdrReader r(es + p + 1, len - 1);
      SchedSlice s{};
      s.frame = static_cast<int64_t>(f);
      s.nal_offset = p;
      s.nal_size = static_cast<int32_t>(len);
      s.first_mb = static_cast<int32_t>(r.ue());
      int st = static_cast<int>(r.ue());
      if (st > 4) st -= 5;
      if (st > 2) return "SP / SI slices";
      s.is_p = st == 0 ? 1 : (st == 1 ? 2 : 0);
      const bool is_b = s.is_p == 2, inter = s.is_p != 0;
      if (static_cast<int>(r.ue()) != pps.pps_id) return "slice refers to another PPS";
      const int frame_num = static_cast<int>(r.u(sps.log2_max_frame_num));
      if (type == 5) r.ue();  // idr_pic_id
      int poc_lsb = 0, dbot = 0, dpoc0 = 0, dpoc1 = 0;
      if (sps.poc_type == 0) {
        poc_lsb = static_cast<int>(r.u(sps.log2_max_poc_lsb));
        if (pps.bottom_field_pic_order_in_frame_present) dbot = r.se();
      } else if (sps.poc_type == 1 && !sps.delta_pic_order_always_zero) {
        dpoc0 = r.se();
        if (pps.bottom_field_pic_order_in_frame_present) dpoc1 = r.se();
      }
      if (pps.redundant_pic_cnt_present) r.ue();
      if (is_b) s.direct_spatial = static_cast<int>(r.u(1));
      s.num_ref = pps.num_ref_idx_l0_default_active;
      s.num_ref1 = is_b ? pps.num_ref_idx_l1_default_active : 0;
      std::vector<std::pair<int, int>> mods[2];
      if (inter) {
        if (r.u(1)) {
          s.num_ref = static_cast<int>(r.ue()) + 1;
          if (is_b) s.num_ref1 = static_cast<int>(r.ue()) + 1;
        }
        if (s.num_ref > 32 || s.num_ref1 > 32) return "num_ref_idx_active > 32";
        for (int l = 0; l < (is_b ? 2 : 1); ++l)
          if (r.u(1)) {
            for (;;) {
              const int idc = static_cast<int>(r.ue());
              if (idc == 3 || r.err) break;
              if (idc > 2) return "bad modification_of_pic_nums_idc";
              mods[l].emplace_back(idc, static_cast<int>(r.ue()));
              if (mods[l].size() > 64) return "too many list modifications";
            }
          }
      }
      // pred_weight_table (7.3.3.2); absent entries keep the default weights
      s.wmode = is_b ? (pps.weighted_bipred_idc == 1 ? 1 : (pps.weighted_bipred_idc == 2 ? 2 : 0))
                     : (s.is_p == 1 && pps.weighted_pred ? 1 : 0);
      if (s.wmode == 1) {
        s.lwd = static_cast<int>(r.ue());
        s.cwd = static_cast<int>(r.ue());
        if (s.lwd > 7 || s.cwd > 7) return "bad pred_weight_table denominators";
      }
      for (int l = 0; l < 2; ++l)
        for (int i = 0; i < 32; ++i) {
          int16_t *w = s.w[l][i];
          w[0] = static_cast<int16_t>(1 << s.lwd);
          w[2] = w[4] = static_cast<int16_t>(1 << s.cwd);
          w[1] = w[3] = w[5] = 0;
          if (s.wmode != 1 || i >= (l ? s.num_ref1 : s.num_ref)) continue;
          if (r.u(1)) {
            const int lw = r.se(), lo = r.se();
            if (lw < -128 || lw > 127 || lo < -128 || lo > 127) return "pred_weight_table out of range";
            w[0] = static_cast<int16_t>(lw);
            w[1] = static_cast<int16_t>(lo);
          }
          if (r.u(1))
            for (int j = 0; j < 2; ++j) {
              const int cw = r.se(), co = r.se();
              if (cw < -128 || cw > 127 || co < -128 || co > 127) return "pred_weight_table out of range";
              w[2 + 2 * j] = static_cast<int16_t>(cw);
              w[3 + 2 * j] = static_cast<int16_t>(co);
            }
        }
      bool this_adaptive = false, this_lt = false;
      std::vector<std::pair<int, int>> this_mmco;
      std::vector<int> this_arg2;
      if (ref_idc) {
        if (type == 5) {
          r.u(1);
          this_lt = r.u(1) != 0;
        } else if ((this_adaptive = r.u(1) != 0)) {
          for (;;) {
            const int op = static_cast<int>(r.ue());
            if (op == 0 || r.err) break;
            if (op > 6) return "bad MMCO";
            int a1 = 0, a2 = 0;
            if (op == 1 || op == 3) a1 = static_cast<int>(r.ue());
            if (op == 2) a1 = static_cast<int>(r.ue());
            if (op == 3 || op == 6) a2 = static_cast<int>(r.ue());
            if (op == 4) a1 = static_cast<int>(r.ue());
            this_mmco.emplace_back(op, a1);
            this_arg2.push_back(a2);
            if (this_mmco.size() > 66) return "too many MMCOs";
          }
        }
      }
      if (pps.entropy_coding_mode && inter) {
        // only the cabac_init_idc 0 context tables are restated (x264 writes 0)
        if (r.ue() != 0) return "cabac_init_idc 1 or 2 (only the idc 0 context tables are supported)";
      }
      s.qp = pps.pic_init_qp + r.se();
      s.dbk_idc = 0;
      if (pps.deblocking_filter_control_present) {
        s.dbk_idc = static_cast<int>(r.ue());
        if (s.dbk_idc != 1) {
          s.dbk_a = 2 * r.se();
          s.dbk_b = 2 * r.se();
        }
      }
      if (r.err || s.first_mb < 0 || s.first_mb >= nmb || s.qp < 0 || s.qp > 51 || s.dbk_idc > 2 ||
          s.dbk_a < -12 || s.dbk_a > 12 || s.dbk_b < -12 || s.dbk_b > 12)
        return "malformed slice header";
      s.data_byte = static_cast<int32_t>(r.ebsp_byte());
      s.data_bit = static_cast<int32_t>(r.rbits);
      if (first) {
        idr = type == 5;
        fn = frame_num;
        fr.is_ref = ref_idc != 0;
        adaptive = this_adaptive;
        lt_ref_flag = this_lt;
        mmco = this_mmco;
        mmco_arg2 = this_arg2;
        h_poc_lsb = poc_lsb;
        h_dbot = dbot;
        // frame_num continuity (gaps_in_frame_num_value_allowed_flag = 0)
        if (!idr && have_prev) {
          const int want = (prev_ref_fn + 1) % max_fn;
          if (frame_num != want) {
            std::snprintf(msg, sizeof msg, "frame_num gap at frame %zu (%d after %d)", f, frame_num, prev_ref_fn);
            return msg;
          }
        }
        if (!idr && !have_prev) return "stream does not start with an IDR picture";
        if (idr) dpb.clear();
        // PicOrderCnt (8.2.1), frames
        if (sps.poc_type == 0) {
          const int max_lsb = 1 << sps.log2_max_poc_lsb;
          const int pmsb = idr ? 0 : prev_poc_msb, plsb = idr ? 0 : prev_poc_lsb;
          int msb = pmsb;
          if (poc_lsb < plsb && plsb - poc_lsb >= max_lsb / 2) msb = pmsb + max_lsb;
          else if (poc_lsb > plsb && poc_lsb - plsb > max_lsb / 2) msb = pmsb - max_lsb;
          const int top = msb + poc_lsb, bot = top + dbot;
          cur_poc = std::min(top, bot);
        } else {
          const int fno = idr ? 0 : (prev_fn > frame_num ? prev_fn_offset + max_fn : prev_fn_offset);
          if (sps.poc_type == 2) {
            cur_poc = idr ? 0 : (ref_idc ? 2 * (fno + frame_num) : 2 * (fno + frame_num) - 1);
          } else {
            const int ncyc = static_cast<int>(sps.offset_for_ref_frame.size());
            int abs_fn = ncyc ? fno + frame_num : 0;
            if (!ref_idc && abs_fn > 0) --abs_fn;
            int expected = 0;
            if (abs_fn > 0) {
              int delta_cycle = 0;
              for (int v : sps.offset_for_ref_frame) delta_cycle += v;
              const int cyc = (abs_fn - 1) / ncyc, in = (abs_fn - 1) % ncyc;
              expected = cyc * delta_cycle;
              for (int i = 0; i <= in; ++i) expected += sps.offset_for_ref_frame[static_cast<size_t>(i)];
            }
            if (!ref_idc) expected += sps.offset_for_non_ref_pic;
            const int top = expected + dpoc0, bot = top + sps.offset_for_top_to_bottom_field + dpoc1;
            cur_poc = std::min(top, bot);
          }
        }
      } else if (frame_num != fn || (type == 5) != idr) {
        return "slices of one picture disagree";
      }
      first = false;
      s.poc = cur_poc;
      if (inter) fr.intra = false;
      if (is_b) fr.has_b = true;
      // RefPicList0 / 1 (8.2.4.2.1, 8.2.4.2.3 + 8.2.4.3)
      for (int i = 0; i < 32; ++i) {
        s.ref[i] = s.ref1[i] = -1;
        s.poc0[i] = s.poc1[i] = 0;
      }
      if (inter) {
        std::vector<const RefPic *> st_refs, lt_refs;
        for (const RefPic &rp : dpb) (rp.kind == 1 ? st_refs : lt_refs).push_back(&rp);
        auto wrap = [&](const RefPic &rp) { return rp.frame_num > fn ? rp.frame_num - max_fn : rp.frame_num; };
        std::stable_sort(lt_refs.begin(), lt_refs.end(),
                         [](const RefPic *a, const RefPic *b) { return a->lt_idx < b->lt_idx; });
        std::vector<const RefPic *> init[2];
        if (!is_b) {
          std::stable_sort(st_refs.begin(), st_refs.end(),
                           [&](const RefPic *a, const RefPic *b) { return wrap(*a) > wrap(*b); });
          init[0] = st_refs;
        } else {
          std::stable_sort(st_refs.begin(), st_refs.end(),
                           [](const RefPic *a, const RefPic *b) { return a->poc < b->poc; });
          for (auto it = st_refs.rbegin(); it != st_refs.rend(); ++it)
            if ((*it)->poc < cur_poc) init[0].push_back(*it);
          for (const RefPic *rp : st_refs)
            if (rp->poc > cur_poc) init[0].push_back(rp);
          for (const RefPic *rp : st_refs)
            if (rp->poc > cur_poc) init[1].push_back(rp);
          for (auto it = st_refs.rbegin(); it != st_refs.rend(); ++it)
            if ((*it)->poc < cur_poc) init[1].push_back(*it);
        }
        for (int l = 0; l < (is_b ? 2 : 1); ++l) init[l].insert(init[l].end(), lt_refs.begin(), lt_refs.end());
        if (is_b && init[1].size() > 1 && init[0] == init[1]) std::swap(init[1][0], init[1][1]);
        for (int l = 0; l < (is_b ? 2 : 1); ++l) {
          const int n = l ? s.num_ref1 : s.num_ref;
          std::vector<const RefPic *> list(static_cast<size_t>(n) + 1, nullptr);
          for (int i = 0; i < n && i < static_cast<int>(init[l].size()); ++i) list[static_cast<size_t>(i)] = init[l][static_cast<size_t>(i)];
          int pred = fn, ridx = 0;
          for (const auto &md : mods[l]) {
            const RefPic *pic = nullptr;
            if (md.first < 2) {
              const int d = md.second + 1;
              int nowrap = md.first == 0 ? pred - d : pred + d;
              if (nowrap < 0) nowrap += max_fn;
              if (nowrap >= max_fn) nowrap -= max_fn;
              pred = nowrap;
              const int num = nowrap > fn ? nowrap - max_fn : nowrap;
              for (const RefPic *rp : st_refs)
                if (wrap(*rp) == num) pic = rp;
            } else {
              for (const RefPic *rp : lt_refs)
                if (rp->lt_idx == md.second) pic = rp;
            }
            if (!pic) return "list modification names no reference picture";
            for (int c = n; c > ridx; --c) list[static_cast<size_t>(c)] = list[static_cast<size_t>(c - 1)];
            list[static_cast<size_t>(ridx++)] = pic;
            int ni = ridx;
            for (int c = ridx; c <= n; ++c)
              if (list[static_cast<size_t>(c)] != pic) list[static_cast<size_t>(ni++)] = list[static_cast<size_t>(c)];
          }
          // the pointers refer to dpb entries, alive until the marking below
          int64_t *ref = l ? s.ref1 : s.ref;
          int32_t *pocs = l ? s.poc1 : s.poc0;
          uint32_t &lt = l ? s.lt1 : s.lt0;
          for (int i = 0; i < n; ++i) {
            const RefPic *rp = list[static_cast<size_t>(i)];
            ref[i] = rp ? rp->frame : -1;
            pocs[i] = rp ? rp->poc : 0;
            if (rp && rp->kind == 2) lt |= 1u << i;
            if (ref[i] >= 0 && std::find(fr.refs.begin(), fr.refs.end(), ref[i]) == fr.refs.end())
              fr.refs.push_back(ref[i]);
          }
          if (l == 1) {
            if (!list[0]) return "B slice without a colocated picture (RefPicList1[0])";
            s.col_short = list[0]->kind == 1;
            if (std::find(fr.cols.begin(), fr.cols.end(), list[0]->frame) == fr.cols.end())
              fr.cols.push_back(list[0]->frame);
          }
        }
      }
      slices->push_back(s);
      p += len;
    }
    fr.ns = static_cast<int64_t>(slices->size()) - fr.s0;
    if (fr.ns == 0) {
      std::snprintf(msg, sizeof msg, "frame %zu has no slices", f);
      return msg;
    }
    // macroblock counts per slice (slices of a picture in increasing first_mb)
    for (int64_t k = fr.s0; k < fr.s0 + fr.ns; ++k) {
      SchedSlice &s = (*slices)[static_cast<size_t>(k)];
      const int next = (k + 1 < fr.s0 + fr.ns) ? (*slices)[static_cast<size_t>(k + 1)].first_mb : nmb;
      if (next <= s.first_mb) return "slices out of order (ASO) or overlapping";
      s.n_mbs = next - s.first_mb;
    }
    // 8.2.1 state after the picture
    bool mmco5 = false;
    for (const auto &m : mmco) mmco5 |= adaptive && m.first == 5;
    if (sps.poc_type == 0) {
      if (fr.is_ref) {
        if (mmco5) {
          prev_poc_msb = 0;
          prev_poc_lsb = h_dbot < 0 ? -h_dbot : 0;
        } else {
          const int max_lsb = 1 << sps.log2_max_poc_lsb;
          const int pmsb = idr ? 0 : prev_poc_msb, plsb = idr ? 0 : prev_poc_lsb;
          int msb = pmsb;
          if (h_poc_lsb < plsb && plsb - h_poc_lsb >= max_lsb / 2) msb = pmsb + max_lsb;
          else if (h_poc_lsb > plsb && h_poc_lsb - plsb > max_lsb / 2) msb = pmsb - max_lsb;
          prev_poc_msb = msb;
          prev_poc_lsb = h_poc_lsb;
        }
      }
    } else {
      const int fno = idr ? 0 : (prev_fn > fn ? prev_fn_offset + max_fn : prev_fn_offset);
      prev_fn_offset = mmco5 ? 0 : fno;
    }
    prev_fn = mmco5 ? 0 : fn;
    fr.poc = mmco5 ? 0 : cur_poc;
    // reference marking (8.2.5) after the picture
    if (fr.is_ref) {
      RefPic cur{static_cast<int64_t>(f), fn, 0, 1, fr.poc};
      if (idr) {
        dpb.clear();
        if (lt_ref_flag) {
          cur.kind = 2;
          cur.lt_idx = 0;
          max_lt_idx = 0;
        } else {
          max_lt_idx = -1;
        }
        dpb.push_back(cur);
        prev_ref_fn = fn;
      } else {
        bool cur_long = false, reset = false;
        if (adaptive) {
          for (size_t k = 0; k < mmco.size(); ++k) {
            const int op = mmco[k].first, a1 = mmco[k].second, a2 = mmco_arg2[k];
            auto wrap = [&](const RefPic &rp) { return rp.frame_num > fn ? rp.frame_num - max_fn : rp.frame_num; };
            if (op == 1 || op == 3) {
              const int pn = fn - (a1 + 1);
              for (size_t i = 0; i < dpb.size(); ++i)
                if (dpb[i].kind == 1 && wrap(dpb[i]) == pn) {
                  if (op == 1) {
                    dpb.erase(dpb.begin() + static_cast<int64_t>(i));
                  } else {
                    dpb.erase(std::remove_if(dpb.begin(), dpb.end(),
                                             [&](const RefPic &x) { return x.kind == 2 && x.lt_idx == a2; }),
                              dpb.end());
                    for (RefPic &x : dpb)
                      if (x.kind == 1 && wrap(x) == pn) {
                        x.kind = 2;
                        x.lt_idx = a2;
                      }
                  }
                  break;
                }
            } else if (op == 2) {
              dpb.erase(std::remove_if(dpb.begin(), dpb.end(),
                                       [&](const RefPic &x) { return x.kind == 2 && x.lt_idx == a1; }),
                        dpb.end());
            } else if (op == 4) {
              max_lt_idx = a1 - 1;
              dpb.erase(std::remove_if(dpb.begin(), dpb.end(),
                                       [&](const RefPic &x) { return x.kind == 2 && x.lt_idx > max_lt_idx; }),
                        dpb.end());
            } else if (op == 5) {
              dpb.clear();
              max_lt_idx = -1;
              reset = true;
            } else if (op == 6) {
              dpb.erase(std::remove_if(dpb.begin(), dpb.end(),
                                       [&](const RefPic &x) { return x.kind == 2 && x.lt_idx == a2; }),
                        dpb.end());
              cur.kind = 2;
              cur.lt_idx = a2;
              cur_long = true;
            }
          }
        } else {
          int ns = 0;
          for (const RefPic &x : dpb) ns += x.kind == 1;
          if (static_cast<int>(dpb.size()) >= max_refs && ns > 0) {
            size_t o = dpb.size();
            int ow = 0;
            for (size_t i = 0; i < dpb.size(); ++i) {
              if (dpb[i].kind != 1) continue;
              const int w = dpb[i].frame_num > fn ? dpb[i].frame_num - max_fn : dpb[i].frame_num;
              if (o == dpb.size() || w < ow) {
                o = i;
                ow = w;
              }
            }
            dpb.erase(dpb.begin() + static_cast<int64_t>(o));
          }
        }
        if (reset) cur.frame_num = 0;
        (void)cur_long;
        dpb.push_back(cur);
        prev_ref_fn = reset ? 0 : fn;
        if (static_cast<int>(dpb.size()) > 16) return "more than 16 reference frames";
      }
    }
    have_prev = true;
  }
  return "";
}

}  // namespace vts
