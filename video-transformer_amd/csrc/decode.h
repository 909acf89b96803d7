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
  int32_t _pad;
  uint64_t *cmd;           // [slot][mb]
  uint32_t *err;           // DEC_E_* bits
  H264DevParams prm;
};

struct ReconArgs {
  const uint8_t *es;
  const uint64_t *cmd;
  const int2 *frames;      // (slot, ref_slot) for every frame of this launch
  uint8_t *surf;           // ring of decoded NV12 frames
  int64_t frame_stride;
  int32_t pitch;
  int32_t mb_width, mb_height;
  int32_t _pad;
  uint32_t *err;
};

int parse_launch(const ParseArgs &a, hipStream_t s);
int recon_launch(const ReconArgs &a, int n_frames, hipStream_t s);
int score_launch(const vts_score_desc *d, hipStream_t stream);
int64_t score_workspace_bytes(int32_t width, int32_t height, int32_t k, int64_t n_frames);

}  // namespace vts
