// h264_tables.h — constant tables of ITU-T H.264 CAVLC decoding, shared by
// the device decoder (decode_full.hip: parser and reconstruction kernels) and
// the host stream writer (synth_full.cpp).  Codes are (length, value) pairs,
// value = the code's bits read MSB first.  tests/test_h264_tables.py checks
// every entry against the bit strings the oracle keeps as the standard prints
// them (oracle/h264_full_oracle.c), and that each code table is prefix-free.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define VTS_TAB __device__ __constant__ static const
#define VTS_TAB_HOST static const
#else
#define VTS_TAB static const
#define VTS_TAB_HOST static const
#endif

namespace vts {
namespace h264 {

// Table 9-5 coeff_token: [nC class][TotalCoeff][TrailingOnes] -> (len, code);
// class 0: 0<=nC<2, 1: 2<=nC<4, 2: 4<=nC<8, 3: nC == -1 (4:2:0 chroma DC,
// TotalCoeff <= 4).  8<=nC is the 6-bit code ((TotalCoeff-1) << 2 | T1), 3
// for TotalCoeff 0.  len 0 = no such code.
#define VTS_CT_LEN_DATA                                                                            \
  {{{1, 0, 0, 0},     {6, 2, 0, 0},     {8, 6, 3, 0},     {9, 8, 7, 5},     {10, 9, 8, 6},        \
    {11, 10, 9, 7},   {13, 11, 10, 8},  {13, 13, 11, 9},  {13, 13, 13, 10}, {14, 14, 13, 11},     \
    {14, 14, 14, 13}, {15, 15, 14, 14}, {15, 15, 15, 14}, {16, 15, 15, 15}, {16, 16, 16, 15},     \
    {16, 16, 16, 16}, {16, 16, 16, 16}},                                                           \
   {{2, 0, 0, 0},     {6, 2, 0, 0},     {6, 5, 3, 0},     {7, 6, 6, 4},     {8, 6, 6, 4},         \
    {8, 7, 7, 5},     {9, 8, 8, 6},     {11, 9, 9, 6},    {11, 11, 11, 7},  {12, 11, 11, 9},      \
    {12, 12, 12, 11}, {12, 12, 12, 11}, {13, 13, 13, 12}, {13, 13, 13, 13}, {13, 14, 13, 13},     \
    {14, 14, 14, 13}, {14, 14, 14, 14}},                                                           \
   {{4, 0, 0, 0},     {6, 4, 0, 0},     {6, 5, 4, 0},     {6, 5, 5, 4},     {7, 5, 5, 4},         \
    {7, 5, 5, 4},     {7, 6, 6, 4},     {7, 6, 6, 4},     {8, 7, 7, 5},     {8, 8, 7, 6},         \
    {9, 8, 8, 7},     {9, 9, 8, 8},     {9, 9, 9, 8},     {10, 9, 9, 9},    {10, 10, 10, 10},     \
    {10, 10, 10, 10}, {10, 10, 10, 10}},                                                           \
   {{2, 0, 0, 0}, {6, 1, 0, 0}, {6, 6, 3, 0}, {6, 7, 7, 6}, {6, 8, 8, 7}, {0, 0, 0, 0},             \
    {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0},             \
    {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}}}
#define VTS_CT_CODE_DATA                                                                           \
  {{{1, 0, 0, 0},   {5, 1, 0, 0},    {7, 4, 1, 0},    {7, 6, 5, 3},    {7, 6, 5, 3},              \
    {7, 6, 5, 4},   {15, 6, 5, 4},   {11, 14, 5, 4},  {8, 10, 13, 4},  {15, 14, 9, 4},            \
    {11, 10, 13, 12}, {15, 14, 9, 12}, {11, 10, 13, 8}, {15, 1, 9, 12}, {11, 14, 13, 8},          \
    {7, 10, 9, 12}, {4, 6, 5, 8}},                                                                 \
   {{3, 0, 0, 0},   {11, 2, 0, 0},   {7, 7, 3, 0},    {7, 10, 9, 5},   {7, 6, 5, 4},              \
    {4, 6, 5, 6},   {7, 6, 5, 8},    {15, 6, 5, 4},   {11, 14, 13, 4}, {15, 10, 9, 4},            \
    {11, 14, 13, 12}, {8, 10, 9, 8}, {15, 14, 13, 12}, {11, 10, 9, 12}, {7, 11, 6, 8},            \
    {9, 8, 10, 1},  {7, 6, 5, 4}},                                                                 \
   {{15, 0, 0, 0},  {15, 14, 0, 0},  {11, 15, 13, 0}, {8, 12, 14, 12}, {15, 10, 11, 11},          \
    {11, 8, 9, 10}, {9, 14, 13, 9},  {8, 10, 9, 8},   {15, 14, 13, 13}, {11, 14, 10, 12},         \
    {15, 10, 13, 12}, {11, 14, 9, 12}, {8, 10, 13, 8}, {13, 7, 9, 12}, {9, 12, 11, 10},           \
    {5, 8, 7, 6},   {1, 4, 3, 2}},                                                                 \
   {{1, 0, 0, 0}, {7, 1, 0, 0}, {4, 6, 1, 0}, {3, 3, 2, 5}, {2, 3, 2, 0}, {0, 0, 0, 0},             \
    {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0},             \
    {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}}}

// Tables 9-7 / 9-8 total_zeros (4x4 blocks): [TotalCoeff - 1][total_zeros]
#define VTS_TZ_LEN_DATA                                                                            \
  {{1, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 9}, {3, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 6, 6, 6, 6}, \
   {4, 3, 3, 3, 4, 4, 3, 3, 4, 5, 5, 6, 5, 6},       {5, 3, 4, 4, 3, 3, 3, 4, 3, 4, 5, 5, 5},       \
   {4, 4, 4, 3, 3, 3, 3, 3, 4, 5, 4, 5},             {6, 5, 3, 3, 3, 3, 3, 3, 4, 3, 6},             \
   {6, 5, 3, 3, 3, 2, 3, 4, 3, 6},                   {6, 4, 5, 3, 2, 2, 3, 3, 6},                   \
   {6, 6, 4, 2, 2, 3, 2, 5},                         {5, 5, 3, 2, 2, 2, 4},                         \
   {4, 4, 3, 3, 1, 3},                               {4, 4, 2, 1, 3},                               \
   {3, 3, 1, 2},                                     {2, 2, 1},                                     \
   {1, 1}}
#define VTS_TZ_CODE_DATA                                                                           \
  {{1, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 1}, {7, 6, 5, 4, 3, 5, 4, 3, 2, 3, 2, 3, 2, 1, 0}, \
   {5, 7, 6, 5, 4, 3, 4, 3, 2, 3, 2, 1, 1, 0},       {3, 7, 5, 4, 6, 5, 4, 3, 3, 2, 2, 1, 0},       \
   {5, 4, 3, 7, 6, 5, 4, 3, 2, 1, 1, 0},             {1, 1, 7, 6, 5, 4, 3, 2, 1, 1, 0},             \
   {1, 1, 5, 4, 3, 3, 2, 1, 1, 0},                   {1, 1, 1, 3, 3, 2, 2, 1, 0},                   \
   {1, 0, 1, 3, 2, 1, 1, 1},                         {1, 0, 1, 3, 2, 1, 1},                         \
   {0, 1, 1, 2, 1, 3},                               {0, 1, 1, 1, 1},                               \
   {0, 1, 1, 1},                                     {0, 1, 1},                                     \
   {0, 1}}
// Table 9-9a total_zeros (4:2:0 chroma DC): [TotalCoeff - 1][total_zeros]
#define VTS_TZC_LEN_DATA {{1, 2, 3, 3}, {1, 2, 2}, {1, 1}}
#define VTS_TZC_CODE_DATA {{1, 1, 1, 0}, {1, 1, 0}, {1, 0}}
// Table 9-10 run_before: [min(zerosLeft, 7) - 1][run_before]
#define VTS_RB_LEN_DATA                                                                            \
  {{1, 1}, {1, 2, 2}, {2, 2, 2, 2}, {2, 2, 2, 3, 3}, {2, 2, 3, 3, 3, 3}, {2, 3, 3, 3, 3, 3, 3},    \
   {3, 3, 3, 3, 3, 3, 3, 4, 5, 6, 7, 8, 9, 10, 11}}
#define VTS_RB_CODE_DATA                                                                           \
  {{1, 0}, {1, 1, 0}, {3, 2, 1, 0}, {3, 2, 1, 1, 0}, {3, 2, 3, 2, 1, 0}, {3, 0, 1, 3, 2, 5, 4},    \
   {7, 6, 5, 4, 3, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1}}

#define VTS_ZZ_DATA {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15}
#define VTS_CBPI_DATA {47, 31, 15, 0, 23, 27, 29, 30, 7, 11, 13, 14, 39, 43, 45, 46, 16, 3, 5, 10, 12, 19, 21, 26, 28, 35, 37, 42, 44, 1, 2, 4, 8, 17, 18, 20, 24, 6, 9, 22, 25, 32, 33, 34, 36, 40, 38, 41}
#define VTS_CBPP_DATA {0, 16, 1, 2, 4, 8, 32, 3, 5, 10, 12, 15, 47, 7, 11, 13, 14, 6, 9, 31, 35, 37, 42, 44, 33, 34, 36, 40, 39, 43, 45, 46, 17, 18, 20, 24, 19, 21, 26, 28, 23, 27, 29, 30, 22, 25, 38, 41}
#define VTS_NORMV_DATA {{10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}}
#define VTS_QPC_DATA {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 32, 33, 34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39}
#define VTS_ALPHA_DATA {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 4, 4, 5, 6, 7, 8, 9, 10, 12, 13, 15, 17, 20, 22, 25, 28, 32, 36, 40, 45, 50, 56, 63, 71, 80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255}
#define VTS_BETA_DATA {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13, 14, 14, 15, 15, 16, 16, 17, 17, 18, 18}
#define VTS_TC0_DATA { {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 1}, {0, 0, 1}, {0, 0, 1}, {0, 0, 1}, {0, 1, 1}, {0, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 1}, {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 1, 2}, {1, 2, 3}, {1, 2, 3}, {2, 2, 3}, {2, 2, 4}, {2, 3, 4}, {2, 3, 4}, {3, 3, 5}, {3, 4, 6}, {3, 4, 6}, {4, 5, 7}, {4, 5, 8}, {4, 6, 9}, {5, 7, 10}, {6, 8, 11}, {6, 8, 13}, {7, 10, 14}, {8, 11, 16}, {9, 12, 18}, {10, 13, 20}, {11, 15, 23}, {13, 17, 25}}

VTS_TAB_HOST uint8_t kCoeffTokenLen[4][17][4] = VTS_CT_LEN_DATA;
VTS_TAB_HOST uint8_t kCoeffTokenCode[4][17][4] = VTS_CT_CODE_DATA;
VTS_TAB_HOST uint8_t kTotalZerosLen[15][16] = VTS_TZ_LEN_DATA;
VTS_TAB_HOST uint8_t kTotalZerosCode[15][16] = VTS_TZ_CODE_DATA;
VTS_TAB_HOST uint8_t kTotalZerosDcLen[3][4] = VTS_TZC_LEN_DATA;
VTS_TAB_HOST uint8_t kTotalZerosDcCode[3][4] = VTS_TZC_CODE_DATA;
VTS_TAB_HOST uint8_t kRunBeforeLen[7][15] = VTS_RB_LEN_DATA;
VTS_TAB_HOST uint8_t kRunBeforeCode[7][15] = VTS_RB_CODE_DATA;

// 8.5.6 frame zig-zag: scan index -> raster index (row * 4 + column)
VTS_TAB_HOST uint8_t kZigzag4x4[16] = VTS_ZZ_DATA;
// Table 9-4 (chroma_format_idc 1): codeNum -> coded_block_pattern
VTS_TAB_HOST uint8_t kCbpIntra[48] = VTS_CBPI_DATA;
VTS_TAB_HOST uint8_t kCbpInter[48] = VTS_CBPP_DATA;
// luma4x4BlkIdx -> position in 4x4-block units (6.4.3)
VTS_TAB_HOST uint8_t kBlkX[16] = {0, 1, 0, 1, 2, 3, 2, 3, 0, 1, 0, 1, 2, 3, 2, 3};
VTS_TAB_HOST uint8_t kBlkY[16] = {0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3};
// 8.5.9 normAdjust4x4 v[m][0..2]
VTS_TAB_HOST uint8_t kNormV[6][3] = VTS_NORMV_DATA;
// Table 8-15: QPc = f(qPI), qPI in 0..51
VTS_TAB_HOST uint8_t kQpc[52] = VTS_QPC_DATA;
// Tables 8-16 / 8-17: alpha'(indexA), beta'(indexB), tC0'(indexA, bS 1..3)
VTS_TAB_HOST uint8_t kAlpha[52] = VTS_ALPHA_DATA;
VTS_TAB_HOST uint8_t kBeta[52] = VTS_BETA_DATA;
VTS_TAB_HOST uint8_t kTc0[52][3] = VTS_TC0_DATA;

// Device copies (constant memory) of the tables the kernels index at run time,
// from the same data macros.
#if defined(__HIPCC__)
__device__ __constant__ static const uint8_t kdZigzag4x4[16] = VTS_ZZ_DATA;
__device__ __constant__ static const uint8_t kdCbpIntra[48] = VTS_CBPI_DATA;
__device__ __constant__ static const uint8_t kdCbpInter[48] = VTS_CBPP_DATA;
__device__ __constant__ static const uint8_t kdNormV[6][3] = VTS_NORMV_DATA;
__device__ __constant__ static const uint8_t kdQpc[52] = VTS_QPC_DATA;
__device__ __constant__ static const uint8_t kdAlpha[52] = VTS_ALPHA_DATA;
__device__ __constant__ static const uint8_t kdBeta[52] = VTS_BETA_DATA;
__device__ __constant__ static const uint8_t kdTc0[52][3] = VTS_TC0_DATA;
#endif

}  // namespace h264
}  // namespace vts
