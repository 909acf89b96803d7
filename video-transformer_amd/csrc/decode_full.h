// decode_full.h — host <-> device interface of the general decoder kernels
// (decode_full.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "h264_full.h"

namespace vts {

struct FullParseArgs {
  const uint8_t *rbsp;       // the slice NALs' RBSPs at their ES offsets (nal_unescape_launch)
  const int32_t *rbsp_len;   // RBSP bytes of this launch's slices (parallel to slices)
  const FullSlice *slices;   // this launch's slices
  int32_t n_slices;
  int32_t slice0;            // window index of slices[0] (MbRec.slice)
  uint32_t epoch;
  int32_t _pad;
  MbRec *recs;               // ring: [slot][mb]
  MbRecB *recs1;             // ring: [slot][mb] list-1 halves (P.bframes), else null
  const SliceExt *exts;      // the window's SliceExt records
  uint16_t *ilvl;            // ring: [slot][mb] intra dependency levels
  int16_t *arena;            // ring's coefficient arena
  uint32_t *err;
  const int32_t *order;      // launch-relative slice of workgroup i (longest first), null = i
  // one launch for every slice of the window (merged): a B slice waits until
  // pdone[colocated slot] reaches pneed[colocated slot] (the picture's slice
  // count); every slice adds 1 to pdone[its slot] when its records are out
  uint32_t *pdone;           // per ring slot, zeroed before the launch; null = not merged
  const int32_t *pneed;      // per ring slot
  uint32_t *arena_top;       // CABAC: the window's count of arena blocks handed out (zeroed before the launch)
  uint32_t arena_blocks;     // CABAC: the arena's capacity in blocks
  int32_t _pad2;
  FullParams P;
};

// h264_derive: complete the CABAC parse's syntax records of n pictures (their
// colocated pictures completed by an earlier launch)
struct DeriveArgs {
  const int2 *pics;          // picture i of the launch: (ring slot, its B slices' common colocated
                             // slot RefPicList1[0], or -1: none / they differ)
  MbRec *recs;               // ring: [slot][mb]
  MbRecB *recs1;             // ring: [slot][mb] list-1 halves (P.bframes), else null
  uint16_t *ilvl;            // ring: [slot][mb] intra dependency levels (written)
  const FullSlice *slices;   // the window's slices (MbRec.slice)
  const SliceExt *exts;      // the window's SliceExt records
  uint32_t *err;
  uint32_t epoch;
  int32_t _pad;
  FullParams P;
};

// per macroblock deblocking descriptor (h264_bs_full -> h264_deblock_plane)
struct DbkInfo {
  uint32_t bs[4];   // bS of edge e (0 = the macroblock edge; 0 when it is not filtered) of direction
                    // dir (0 vertical), 4-sample segment seg: nibble (e & 1) * 4 + seg of word dir * 2 + e / 2
  uint32_t qp;      // QPq | QPleft << 8 | QPtop << 16 (I_PCM: 0) | (disable_deblocking_filter_idc == 1) << 24
  int32_t fa, fb;   // FilterOffsetA / B of the macroblock's slice
  uint32_t _pad;
  // Each edge's filter parameters (8.7.2.2, Tables 8-16 / 8-17), resolved by
  // h264_bs_full so the deblocking wavefront reads them instead of deriving
  // them per lane: alpha | beta << 8 | tC0(bS 1, 2, 3) << 16, 21, 26 of the
  // edge's indexA / indexB, 0 when alpha or beta is 0 (the edge never filters).
  uint32_t lv[4];   // luma vertical edges 0..3
  uint32_t lh[4];   // luma horizontal edges 0..3
  uint32_t cv[4];   // chroma vertical: (edge 0, Cb), (edge 0, Cr), (edge 2, Cb), (edge 2, Cr)
  uint32_t ch[4];   // chroma horizontal, the same order
};
static_assert(sizeof(DbkInfo) == 96, "DbkInfo layout");

struct FullReconArgs {
  const int4 *frames;        // (ring slot, descriptor slot in dbk, -, -) per picture of the launch
  const MbRec *recs;
  const MbRecB *recs1;       // list-1 halves (P.bframes), else null
  const SliceExt *exts;      // the window's SliceExt records (FullSlice.ext)
  const uint16_t *ilvl;
  const int16_t *arena;
  const FullSlice *slices;   // the window's slices (MbRec.slice indexes them)
  uint8_t *surf;             // ring of NV12 pictures
  const int32_t *surf_of;    // window slot -> surface index in surf (null: the slot; recycled surfaces)
  int64_t frame_stride;
  int64_t uv_off;            // UV plane offset in a picture (pitch * coded height)
  int32_t pitch;
  uint32_t epoch;
  int32_t deblock;           // 1: h264_deblock_plane after reconstruction (0: none)
  int32_t intra_kernel;      // 1: h264_intra_full, else h264_intra_v2 (where its LDS fits)
  DbkInfo *dbk;              // [descriptor slot][mb] deblocking descriptors: a ring of two levels per GOP
                             // group (bS of level l + 1 is derived while level l deblocks)
  uint32_t *err;
  const ScaleTab *sct;       // LevelScale4x4 / 8x8 (read when P.scaled)
  FullParams P;
};

// 7.4.1 per slice NAL: the payload (after the header byte) without its
// emulation-prevention bytes, at the same offset of rbsp; rbsp_len[i] = its
// length.  Once per session: the parsers then read plain RBSP bits.
int nal_unescape_launch(const uint8_t *es, uint8_t *rbsp, const FullSlice *slices, int32_t n_slices,
                        int32_t *rbsp_len, hipStream_t s);
int parse_full_launch(const FullParseArgs &a, hipStream_t s);
int derive_launch(const DeriveArgs &a, int n_pictures, hipStream_t s);
// a one-wave kernel that returns after `us` microseconds (stream_delay)
int delay_launch(uint32_t us, hipStream_t s);
// deblocking descriptors (bS, QPs) of n_frames pictures: reads only the
// parse's records, so one launch covers a whole window
int bs_full_launch(const FullReconArgs &a, int n_frames, hipStream_t s);
// reconstruction (+ deblocking from bs_full_launch's descriptors when
// a.deblock) of n_frames pictures of one level
int recon_full_launch(const FullReconArgs &a, int n_frames, hipStream_t s, hipEvent_t after_inter = nullptr);

}  // namespace vts
