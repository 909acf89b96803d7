// Prints the product's CABAC / 8x8-transform tables
// (video-transformer_amd/csrc/h264_cabac_tables.h) as "name i j value" lines
// for tests/test_cabac_tables.py, which compares them with the oracle's own
// transcription (oracle/h264_std_tables.h).  Test-only; never linked.
#include <cstdint>
#include <cstdio>

#include "h264_cabac_tables.h"

static const int8_t kInitI[VTS_CABAC_NCTX][2] = VTS_CABAC_INIT_I_DATA;
static const int8_t kInitP0[VTS_CABAC_NCTX][2] = VTS_CABAC_INIT_P0_DATA;
static const uint8_t kRange[64][4] = VTS_CABAC_RANGE_LPS_DATA;
static const uint8_t kTrans[64] = VTS_CABAC_TRANS_LPS_DATA;
static const uint8_t kSig8[63] = VTS_SIG8x8_DATA;
static const uint8_t kLast8[63] = VTS_LAST8x8_DATA;
static const int kZz8[64] = VTS_ZZ8_DATA;
static const int kNorm8[6][6] = VTS_NORM8_DATA;
static const uint8_t kDef4[2][16] = VTS_DEFAULT_4x4_DATA;
static const uint8_t kDef8[2][64] = VTS_DEFAULT_8x8_DATA;

int main() {
  for (int i = 0; i < VTS_CABAC_NCTX; ++i)
    for (int j = 0; j < 2; ++j) {
      std::printf("init_i %d %d %d\n", i, j, kInitI[i][j]);
      std::printf("init_p0 %d %d %d\n", i, j, kInitP0[i][j]);
    }
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 4; ++j) std::printf("range_lps %d %d %d\n", i, j, kRange[i][j]);
  for (int i = 0; i < 64; ++i) std::printf("trans_lps %d 0 %d\n", i, kTrans[i]);
  for (int i = 0; i < 63; ++i) std::printf("sig8 %d 0 %d\n", i, kSig8[i]);
  for (int i = 0; i < 63; ++i) std::printf("last8 %d 0 %d\n", i, kLast8[i]);
  for (int i = 0; i < 64; ++i) std::printf("zz8 %d 0 %d\n", i, kZz8[i]);
  for (int m = 0; m < 6; ++m)
    for (int c = 0; c < 6; ++c) std::printf("norm8 %d %d %d\n", m, c, kNorm8[m][c]);
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) std::printf("norm8_class %d %d %d\n", i, j, vts_norm8_class(i, j));
  for (int l = 0; l < 2; ++l) {
    for (int k = 0; k < 16; ++k) std::printf("default4 %d %d %d\n", l, k, kDef4[l][k]);
    for (int k = 0; k < 64; ++k) std::printf("default8 %d %d %d\n", l, k, kDef8[l][k]);
  }
  return 0;
}
