// session.h — the per-video device session (vts_ctx) shared by session.hip
// (open / decode + score) and transcode.hip (360p upload transcode).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <thread>
#include <vector>

#include "common.h"
#include "decode.h"
#include "decode_full.h"
#include "h264.h"
#include "devmem.h"
#include "h264_full.h"

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess)                                                          \
      return vts::fail(VTS_E_HIP, "%s failed: %s", #expr, hipGetErrorString(_e));  \
  } while (0)

namespace vts {

struct Window {
  int64_t f0 = 0, f1 = 0;          // frames [f0, f1)
  int64_t s0 = 0, s1 = 0;          // slices [s0, s1), ordered by reconstruct launch
  std::vector<int64_t> lvl_off;    // into level_frames, one entry per reconstruct launch
  std::vector<int32_t> lvl_cnt;
  std::vector<int64_t> lvl_s0;     // first slice (absolute) of each launch's frames
  std::vector<int32_t> chunk_end;  // parse chunk j covers launches [chunk_end[j-1], chunk_end[j])
  std::vector<int32_t> grp;        // interleaved GOP groups: first launch of each (empty = one group)
  int64_t ev0 = 0;                 // first index of this window's events in vts_ctx::lev
  int64_t post_off = 0, post_cnt = 0;  // into post_slots
  // level-blocked schedule (h264_recon_score_tb), when every GOP of the
  // window is a plain P chain: launch i covers chains [tb_off[i], + tb_cnt[i])
  // of tb_L[i] levels each in vts_ctx::tb_chains
  bool tb = false;
  std::vector<int64_t> tb_off;
  std::vector<int32_t> tb_cnt, tb_L;
  int64_t fs0 = 0, fs1 = 0;        // general decoder: slices [fs0, fs1) of vts_ctx::fslices
  int64_t pn0 = 0;                 // general decoder: the window's slot entries in vts_ctx::pneed
  std::vector<int32_t> plv_end;    // general decoder: parse launch j covers window slices
                                   // [plv_end[j-1], plv_end[j]) (B pictures after their colocated picture)
  int64_t ds0 = 0;                 // general decoder, CABAC: the window's entries in vts_ctx::dslots
  std::vector<int32_t> dlv_end;    // ... h264_derive launch j covers entries [dlv_end[j-1], dlv_end[j])
  // CABAC: the window's plong longest slices (porder_m's first entries) parse
  // in a launch of their own, the rest in one beside it, with the derivation
  // of every picture that needs none of the long ones (the first dlv_early[j]
  // entries of derive launch j); 0: one parse launch
  int32_t plong = 0;
  std::vector<int32_t> dlv_early;
};

// Downscaled copy of every decoded frame (transcode.hip), filled by run_all
// after each window's reconstruction when `on`.
struct SmallStore {
  bool on = false;
  int w = 0, h = 0;             // display size (even)
  int cw = 0, ch = 0;           // coded size (16-aligned); NV12, pitch cw, UV at cw * ch
  int64_t stride = 0;           // bytes per frame
  uint8_t *d = nullptr;         // [frame]
  int32_t *d_taps = nullptr;    // area-filter tap tables (transcode.hip area_taps)
  int64_t off[4] = {0, 0, 0, 0};  // luma x, luma y, chroma x, chroma y tables in d_taps
  int taps_x = 0, taps_y = 0, taps_cx = 0, taps_cy = 0;  // taps per output sample
  int32_t tl = 1, tc = 1;       // luma / chroma normalisers
};

}  // namespace vts

namespace vts {
// Host bytes without value-initialisation (a std::vector zero-fills every
// byte of a multi-GB elementary stream before the read overwrites it)
struct HostBytes {
  HostBytes() = default;
  HostBytes(const HostBytes &) = delete;
  HostBytes &operator=(const HostBytes &) = delete;
  // a multi-GB buffer's pages take tens of ms to unmap: freed off the
  // caller's thread (vts_open returned 50-80 ms earlier)
  ~HostBytes() {
    if (n_ >= (int64_t{64} << 20)) std::thread([p = p_]() { std::free(p); }).detach();
    else std::free(p_);
  }
  bool alloc(int64_t n) {
    std::free(p_);
    p_ = static_cast<uint8_t *>(std::malloc(static_cast<size_t>(std::max<int64_t>(n, 1))));
    n_ = p_ ? n : 0;
    return p_ != nullptr;
  }
  uint8_t *data() { return p_; }
  const uint8_t *data() const { return p_; }
  size_t size() const { return static_cast<size_t>(n_); }
  uint8_t operator[](size_t i) const { return p_[i]; }

 private:
  uint8_t *p_ = nullptr;
  int64_t n_ = 0;
};
}  // namespace vts

struct vts_ctx {
  using Sps = vts::Sps;
  using Pps = vts::Pps;
  using H264DevParams = vts::H264DevParams;
  using SliceDesc = vts::SliceDesc;
  using Window = vts::Window;
  int device = 0;
  Sps sps;
  Pps pps;
  H264DevParams prm{};
  vts_video_info info{};
  vts_params params{};
  int k = 4;
  int width = 0, height = 0, pitch = 0, coded_w = 0, coded_h = 0;
  int64_t frame_stride = 0;
  int64_t n_frames = 0;
  std::vector<int64_t> pts;
  std::vector<SliceDesc> slices;
  std::vector<int4> level_frames;
  std::vector<int32_t> post_slots;  // per window: slots whose SAD the thumb_sad pass makes
  std::vector<Window> windows;
  std::vector<int4> tb_chains;      // level-blocked launches: [chain][L] (slot, ref, sad_prev, 0)
  std::vector<uint8_t> tb_last;     // per frame: last level of its chain (kept in HBM)
  int4 *d_tb = nullptr;
  bool tb_off = false;              // a launch met motion beyond its halo: per-level from now on
  bool tb_ran_sparse = false;       // the last run kept only chain-last frames
  int64_t ring_frames = 0;
  int n_rings = 1;
  // device
  uint8_t *d_es = nullptr;
  uint8_t *d_rbsp = nullptr;      // general decoder: slice NAL payloads without EPBs (at ES offsets)
  int32_t *d_rbsp_len = nullptr;  // ... their lengths, per fslice
  int64_t es_bytes = 0;
  SliceDesc *d_slices = nullptr;
  int4 *d_levels = nullptr;
  int32_t *d_post = nullptr;
  uint64_t *d_cmd[2] = {nullptr, nullptr};
  uint8_t *d_surf[2] = {nullptr, nullptr};
  uint8_t *d_ws[2] = {nullptr, nullptr};
  int64_t ws_bytes = 0;
  uint8_t *d_last[2] = {nullptr, nullptr};
  uint32_t *d_err = nullptr;
  float *d_score = nullptr;
  uint64_t *d_sad = nullptr;
  uint32_t *d_hist = nullptr;
  uint8_t *d_rgb = nullptr;       // RGB thumbnails of every frame
  bool fused = false;             // scoring fused into reconstruction
  uint8_t *d_thumb[2] = {nullptr, nullptr};  // fused: [slot][h][w] thumbnail luma
  int64_t thumb_px = 0;
  hipStream_t s_dec = nullptr, s_score = nullptr, s_parse = nullptr;
  // interleaved GOP groups: group g >= 1 reconstructs on s_grp[g - 1] and
  // signals ev_grp[g - 1] when its last launch is done (Window::grp)
  static constexpr int kMaxGroups = 4;
  bool group_parse = false;  // one parse chunk per group (VTS_GROUP_PARSE)
  int recon_groups = 2;  // measured best on MI355X; VTS_RECON_GROUPS overrides
  int general_groups = 2;  // general decoder: GOP groups reconstructing on s_dec / s_grp[g - 1]
                           // (DESIGN.md §5b); VTS_GENERAL_GROUPS (1..4) overrides
  hipStream_t s_grp[kMaxGroups - 1] = {nullptr, nullptr, nullptr};
  int stream_kind = 0;     // the pool its stream set came from (session.hip streams_take)
  hipEvent_t ev_grp[kMaxGroups - 1] = {nullptr, nullptr, nullptr};
  std::vector<hipEvent_t> ev;  // per window: dec start, parsed, decoded, score start, scored, spare
  std::vector<hipEvent_t> lev;  // per window: (start, end) per reconstruct launch, then one per parse chunk
  hipEvent_t ev_start = nullptr, ev_end = nullptr;
  double timings[4] = {0, 0, 0, 0};
  // host time of vts_open by stage (ms, vts_open_timings): 0 demux (moov),
  // 1 device checks, 2 sample read, 3 host schedule, 4 device allocations,
  // 5 elementary-stream upload, 6 other uploads and set-up kernels, 7 total
  double open_ms[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  double open_t = 0;  // seconds (steady clock) of the last lap
  void open_lap(int k);
  int64_t last_window_done = -1;
  // command epochs: run_no counts window runs; a ring is cleared on first use
  // and again before an epoch value could repeat (h264.h kCmdEpochs)
  int64_t run_no = 0;
  int64_t ring_cleared_at[2] = {-1, -1};
  bool have_results = false;
  bool pending = false;            // a run is submitted (vts_run_async) and not yet waited for
  uint32_t *h_err = nullptr;       // pinned: the run's error word, copied back at its end
  std::vector<float> host_scores;
  vts::SmallStore small;       // transcode: downscaled frames (off unless vts_transcode ran)
  // ---- general decoder (decode_full.hip, session_full.hip)
  bool general = false;
  vts::FullParams fprm{};
  vts::ScaleTab scale_tab{};       // LevelScale of the stream (8.5.9; flat without scaling matrices)
  vts::ScaleTab *d_scale = nullptr;
  std::vector<vts::FullSlice> fslices;  // every window's slices (window-relative slots, arena)
  vts::FullSlice *d_fslices = nullptr;
  vts::MbRec *d_recs[2] = {nullptr, nullptr};
  vts::MbRecB *d_recs1[2] = {nullptr, nullptr};  // list-1 halves (streams with B slices)
  std::vector<vts::SliceExt> exts;      // B / weighted slices' SliceExt records (all windows)
  vts::SliceExt *d_exts = nullptr;
  std::vector<int32_t> porder;          // per fslice: parse order inside its launch (longest slice first)
  int32_t *d_porder = nullptr;
  std::vector<int32_t> porder_m;        // per fslice: order inside the window's merged launch
  int32_t *d_porder_m = nullptr;
  std::vector<int32_t> pneed;           // per window frame (ring slot): slices of the picture
  int32_t *d_pneed = nullptr;
  uint32_t *d_pdone[2] = {nullptr, nullptr};  // per ring: slices done per slot (merged parse)
  std::vector<int2> dslots;             // CABAC: the windows' pictures by parse level (h264_derive): ring slot,
                                        // common colocated slot
  int2 *d_dslots = nullptr;
  int intra_kernel = 2;                 // 2: h264_intra_v2; VTS_INTRA=1: h264_intra_full (its LDS fallback)
  int parse_split = 1;                  // CABAC: long slices in a parse launch of their own (VTS_PARSE_SPLIT:
                                        // 0 one launch, 2 the longest eighth whatever the sizes, a test mode)
  std::vector<hipEvent_t> ev_px;        // per window: arena reset done, short parse + early derives done
  hipStream_t s_px = nullptr;           // the short parse's stream: a hardware queue of its own (CU mask of every
                                        // compute unit), made on first use; a stream sharing the parse stream's
                                        // queue would run after the long launch
  bool parse_merged = true;             // VTS_PARSE_MERGE=0: one launch per colocated level
  std::vector<hipEvent_t> ev_bs;  // paced bS: two per level launch of a window (reused window to window)
  // recycled surfaces (keep_frames 0, no transcode): a picture's surface
  // goes back to its GOP group's pool once the last picture predicting from it
  // is reconstructed and its own level is thumbnailed (thumb_pics right after
  // the level on the group's own stream); surf_of[frame] = surface of the
  // frame's window slot, surf_count per ring
  bool surf_pool = false;
  std::vector<int32_t> surf_of;
  int32_t *d_surf_of = nullptr;
  int64_t surf_count = 0;
  std::vector<int64_t> disp;            // presentation rank of each sample (decode order)
  uint16_t *d_ilvl[2] = {nullptr, nullptr};  // intra dependency level per macroblock
  vts::DbkInfo *d_dbk[2] = {nullptr, nullptr};  // deblocking descriptor per macroblock
  int16_t *d_arena[2] = {nullptr, nullptr};
  int64_t arena_blocks = 0;             // per ring (CABAC: the capacity the windows share)
  std::vector<int32_t> fslice_nmbs;     // per fslice: its macroblocks (arena ranges)
  // CABAC: slices take blocks from their window's arena in chunks (h264_full.h
  // kArenaChunk, one counter per window).  The capacity starts at an estimate
  // (arena_q4 quarter blocks per slice byte: 0.75, + 1/8 and a chunk per
  // slice of slack; VTS_ARENA_PER_BYTE = whole blocks per byte, 0 forces the
  // growth; the streams here store 0.46-0.87) and grows, up to arena_bound
  // (32 per byte: every stored block costs at least one bypass bin), when a
  // run reports DEC_E_ARENA, which re-runs it (arena_reruns)
  int arena_q4 = 3;
  int64_t arena_bound = 0;              // per ring: the capacity no valid stream exceeds
  int64_t arena_reruns = 0;
  uint32_t *d_arena_top = nullptr;      // per window: blocks its parse handed out (asked for)
  int64_t dbk_pics = 0;                 // descriptor slots of d_dbk (a ring of two levels per GOP group)
  // kept from open for a later switch to the general decoder (decoder = auto)
  std::vector<int64_t> es_off;          // sample offsets in the ES buffer
  std::vector<uint32_t> sample_size;
  int nal_length_size = 4;
  std::vector<uint8_t> sps_nal, pps_nal;
};

namespace vts {
// Decode + score every window (and downscale when ctx->small.on):
// submit_all enqueues a run, finish_all waits for it (errors, timings, the
// re-runs the device asks for); run_all = both.
int run_all(vts_ctx *c);
int submit_all(vts_ctx *c);
int finish_all(vts_ctx *c);
int finish_subset(vts_ctx *c);
int fetch_scores(vts_ctx *c);
// general decoder: schedule + buffers from the host ES (session_full.hip);
// `sps_nal` / `pps_nal` are the avcC parameter sets
int build_general(vts_ctx *c, const uint8_t *es, const std::vector<int64_t> &es_off,
                  const std::vector<uint32_t> &sizes, int nal_length_size, const std::vector<uint8_t> &sps_nal,
                  const std::vector<uint8_t> &pps_nal);
int run_general(vts_ctx *c);
int submit_general(vts_ctx *c);
int finish_general(vts_ctx *c);
// cheap look at the stream's first pictures: does it need the general decoder?
// the parameter sets alone send the stream to the general decoder
bool general_by_headers(const vts_ctx *c);
bool wants_general(const vts_ctx *c, const uint8_t *es, const std::vector<int64_t> &es_off,
                   const std::vector<uint32_t> &sizes, int nal_length_size);
// downscale the window's frames (transcode.hip)
int small_window(vts_ctx *c, int ring, int64_t f0, int64_t f1, hipStream_t s);
}  // namespace vts
