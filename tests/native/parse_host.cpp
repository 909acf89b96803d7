// Test-only harness: compiles the device decoder's slice parser
// (video-transformer_amd/csrc/parse_slice.h) for the host so the CPU suite can
// compare its command words with the oracle's parser (tests/test_parse_host.py).
// Never linked into libvtseg.so; the product path runs the parser on the GPU.
#include "parse_slice.h"

extern "C" uint32_t ph_parse_slice(const uint8_t *es, int64_t nal_offset, int32_t nal_size, int32_t slot,
                                   int32_t ref_slot, const int32_t *prm14, uint64_t *cmd_all) {
  vts::H264DevParams P{};
  int32_t *dst = &P.mb_width;  // the POD's int32 fields in declaration order
  for (int i = 0; i < 13; ++i) dst[i] = prm14[i];
  vts::ParseScratch scratch{};
  return vts::parse_slice(es, nal_offset, nal_size, slot, ref_slot, P, cmd_all, &scratch);
}
