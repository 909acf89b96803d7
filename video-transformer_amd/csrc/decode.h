// decode.h — host <-> device interface of the H.264 subset decode kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "h264.h"
#include "vtseg.h"

namespace vts {

// One slice NAL unit scheduled for parsing.
struct SliceDesc {
  int64_t nal_offset;  // of the NAL header byte inside the device ES buffer
  int32_t nal_size;    // bytes including the header byte
  int32_t slot;        // frame slot in the window (index into cmd / surfaces)
  int32_t ref_slot;    // slot of the reference picture, -1 for none
  int32_t _pad;
};

struct ParseArgs {
  const uint8_t *es;       // device elementary-stream bytes (+64 B padding)
  const SliceDesc *slices;
  int32_t n_slices;
  uint32_t epoch;          // written into every command (h264.h kCmdEpochMask)
  uint64_t *cmd;           // [slot][mb]
  uint32_t *err;           // DEC_E_* bits
  H264DevParams prm;
};

struct ReconArgs {
  const uint8_t *es;
  const uint64_t *cmd;
  const int4 *frames;      // (slot, ref_slot, sad_prev, 0) per frame of this launch:
                           // sad_prev = slot of the display predecessor when its
                           // thumbnail was made by an earlier launch, else -1
  uint8_t *surf;           // ring of decoded NV12 frames
  int64_t frame_stride;
  int32_t pitch;
  int32_t mb_width, mb_height;
  uint32_t epoch;          // commands of another epoch read as absent
  uint32_t *err;
};

// Fused reconstruct + scoring (k in {2,4,8}, display size == coded size).
struct FusedArgs {
  ReconArgs r;
  int64_t frame0;          // global frame index of window slot 0
  int32_t w, h;            // thumbnail size
  int32_t wgs_per_frame;   // ceil(MBs / 256)
  int32_t _pad;
  uint8_t *thumb;          // [slot][h][w] thumbnail luma
  uint8_t *rgb;            // [global frame][h][w][3]
  uint32_t *hist;          // [global frame][256], zeroed before the window
  uint64_t *sad;           // [global frame], zeroed before the window
};

// Level-blocked fused reconstruct + scoring (k = 4, h264_recon_score_tb).
struct TbArgs {
  FusedArgs f;             // f.r.frames unused
  const int4 *chains;      // [chain][L]: (slot, ref_slot, sad_prev, 0) of L consecutive
                           // GOP levels; slot -1 past the chain's end
  int32_t L;
  int32_t keep;            // store every level's frame (else only each chain's last)
};

struct ThumbSadArgs {
  const uint8_t *thumb;    // [slot][h][w]
  const int32_t *list;     // slots to compute (nullptr = all n_frames)
  int64_t n_list;
  const uint8_t *prev_luma;  // predecessor of slot 0 (nullptr = none)
  uint8_t *last_luma;      // receives slot n_frames-1 (may be nullptr)
  int64_t frame0;
  int64_t n_frames;
  int32_t w, h;
  uint64_t *sad;           // [global frame]
  float *score;
};

// Thumbnails of one list of pictures (general decoder with recycled surfaces):
// thumbnail luma per window slot, RGB and histogram per frame.
struct PicThumbArgs {
  const uint8_t *surf;     // surface pool
  int64_t frame_stride;
  const int32_t *surf_of;  // window slot -> surface (null: the slot)
  const int4 *pics;        // .x = window slot
  int32_t n_pics;
  int32_t w, h;            // thumbnail size
  int32_t pitch, uv_row_offset;
  int32_t chunks_per_row;  // w / G (G = 16 / k bytes, 48 / 6 for k = 6)
  int32_t n_chunks;        // chunks_per_row * h
  int64_t f0;              // frame of window slot 0
  uint8_t *thumb;          // [slot][h][w]
  uint8_t *rgb;            // [frame][h][w][3] (may be null)
  uint32_t *hist;          // [frame][256], zero before (bands add into it; may be null)
};

int parse_launch(const ParseArgs &a, hipStream_t s);
int fused_launch(const FusedArgs &a, int k, int n_frames, hipStream_t s);
int thumb_sad_launch(const ThumbSadArgs &t, hipStream_t s);
// score[frame0 + i] = sad / (w*h*255) for i < n_frames
int sad_score_launch(const uint64_t *sad, float *score, int64_t frame0, int64_t n_frames,
                     int64_t npx, hipStream_t s);
int recon_launch(const ReconArgs &a, int n_frames, hipStream_t s);
// one workgroup per (chain, macroblock row); LDS bytes / tasks per level 0
int tb_launch(const TbArgs &a, int n_chains, hipStream_t s);
int tb_lds_bytes(int mb_width, int mb_height, int L);
int tb_max_tasks(int mb_width, int mb_height, int L);
// hist[0 .. 256 n) = 0, sad[0 .. n) = 0 (hist 16-byte aligned)
int clear_accum_launch(uint32_t *hist, uint64_t *sad, int64_t n_frames, hipStream_t s);
int score_launch(const vts_score_desc *d, hipStream_t stream);
int thumb_pics_launch(const PicThumbArgs &a, int k, hipStream_t s);
int64_t score_workspace_bytes(int32_t width, int32_t height, int32_t k, int64_t n_frames);

}  // namespace vts
