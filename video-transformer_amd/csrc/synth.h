// synth.h — internals shared by the synthetic stream writers: synth.cpp (the
// I_PCM / P_Skip subset, vts_synth_params.coding 0) and synth_full.cpp (the
// full CAVLC syntax, coding 1).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "vtseg.h"

namespace vts {

struct Pcg32 {  // PCG-XSH-RR 64/32
  uint64_t state, inc;
  explicit Pcg32(uint64_t seed, uint64_t seq = 0x5eedull) : state(0), inc((seq << 1) | 1) {
    next();
    state += seed;
    next();
  }
  uint32_t next() {
    const uint64_t old = state;
    state = old * 6364136223846793005ull + inc;
    const uint32_t xs = static_cast<uint32_t>(((old >> 18) ^ old) >> 27);
    const uint32_t rot = static_cast<uint32_t>(old >> 59);
    return (xs >> rot) | (xs << ((32 - rot) & 31));
  }
  uint32_t below(uint32_t n) { return n ? next() % n : 0; }
  double uniform() { return next() / 4294967296.0; }
};


// One independently coded run of frames [f0, f0 + nf) of the stream: it starts
// with an IDR (a scene cut unless f0 == 0), so chunks concatenate into one
// valid stream.  Samples stay in memory until the MP4 is written.
struct SynthChunk {
  int64_t f0 = 0, nf = 0;
  uint64_t seed = 0;
  int idr_id_base = 0;        // idr_pic_ids 2k, 2k+1: consecutive IDRs across chunks differ
  std::vector<uint8_t> data;  // samples, back to back
  std::vector<uint32_t> size;
  std::vector<uint8_t> sync;
  std::vector<uint32_t> cts;  // composition offsets in frames (B pictures); empty = none
  std::vector<int64_t> cuts;  // global frame indices
  int64_t n_idr = 0;
  uint64_t recon_hash = 0;
  std::string error;          // non-empty: the chunk could not be written
};

// Smooth value-noise texture (two octaves of bilinear random grids + noise)
// of a w x h luma plane and its w/2 x h/2 chroma planes; the subset writer's
// scenes and the full writer's content mode.
void synth_texture(uint8_t *y, uint8_t *u, uint8_t *v, int w, int h, Pcg32 &rng, bool zero_runs);

// Append one NAL unit (header byte + RBSP with emulation prevention) to an
// AVCC sample with a 4-byte length prefix.
void append_nal(std::vector<uint8_t> &sample, uint8_t header, std::vector<uint8_t> &rbsp);

// Full-syntax chunk (synth_full.cpp); SPS / PPS from make_sps_pps_full.
void encode_chunk_full(const vts_synth_params &P, SynthChunk *ck);
void make_sps_pps_full(const vts_synth_params &P, int level, std::vector<uint8_t> *sps_nal,
                       std::vector<uint8_t> *pps_nal);

}  // namespace vts
