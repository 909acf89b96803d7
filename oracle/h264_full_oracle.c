/*
 * h264_full_oracle.c — scalar CPU restatement of ITU-T H.264 decoding for
 * progressive CAVLC streams with I and P slices, used ONLY as the checker of
 * the device decoder (decode_full.hip in the product package).
 *
 * TEST INFRASTRUCTURE.  Only tests/, __graft_entry__.smoke() and bench.py's
 * parity / cpu_baseline legs may load this code; the product never links it.
 * Written from the standard's clauses (cited inline), independently of the
 * product code: its VLC tables are kept as the standard prints them (bit
 * strings per row of Tables 9-5, 9-7..9-10) and tests/test_h264_tables.py
 * checks them against the product's (length, code) arrays.
 *
 * Covered: Baseline-profile decoding without FMO / ASO / redundant slices
 * (and Main/High streams that use no CABAC, B slices, interlace, 8x8
 * transform, scaling matrices or weighted prediction):
 *   7.3     SPS / PPS / slice header / slice data / macroblock layer syntax
 *   8.2.4   reference picture lists (init + modification, short & long term)
 *   8.2.5   reference marking (sliding window, MMCO 1-6)
 *   8.3     Intra_4x4, Intra_16x16, chroma intra prediction, I_PCM
 *   8.4     P motion vector prediction (all partitions, P_Skip), luma
 *           6-tap / quarter-sample and chroma eighth-sample interpolation
 *   8.5     scaling (flat), 4x4 / Hadamard / 2x2 inverse transforms
 *   8.7     deblocking filter (bS, alpha/beta/tC0, idc 0/1/2, offsets)
 *   9.2     CAVLC residual_block (coeff_token, levels, total_zeros, run_before)
 * Output order = decoding order (no B slices; pic_order_cnt is parsed only).
 *
 * Parity: no third-party decoder exists in the image, so this restatement is
 * "parity unpinned" against one; it is cross-checked against the round-1
 * subset oracle (vtseg_oracle.c) on subset streams, against the synthetic
 * writer's own syntax (every slice must end exactly at its stop bit), and it
 * is the reference the GPU decoder must equal bit for bit.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* CABAC / 8x8-transform constants (Tables 9-12..9-33, 9-43, 9-44, 8-16):
 * the oracle's own transcription in the standard's layout, independent of
 * the product's header (tests/test_cabac_tables.py diffs the two) */
#include "h264_std_tables.h"

#define FO_NCTX 460

/* CABAC synthesis mode (fo_cabac_convert, test infrastructure) */
typedef struct fo_enc_s fo_enc;
static fo_enc *g_enc;      /* non-null: synthesis mode */
#define FO_E_FORMAT -8
#define FO_E_UNSUPPORTED -9
#define FO_E_DECODE -12

/* ------------------------------------------------------------------ bits */
typedef struct {
  const uint8_t *p;
  int64_t n, pos;
  int bitpos, zeros, err;
  uint32_t cur;
} fb_t;

static void fb_init(fb_t *b, const uint8_t *p, int64_t n) {
  memset(b, 0, sizeof *b);
  b->p = p;
  b->n = n;
}
static uint32_t fb_byte(fb_t *b) { /* next RBSP byte: 7.4.1 drops 0x03 after 00 00 */
  if (b->pos >= b->n) { b->err = 1; return 0; }
  uint32_t v = b->p[b->pos];
  if (b->zeros >= 2 && v == 3) {
    b->pos++;
    b->zeros = 0;
    if (b->pos >= b->n) { b->err = 1; return 0; }
    v = b->p[b->pos];
  }
  b->pos++;
  b->zeros = v == 0 ? b->zeros + 1 : 0;
  return v;
}
static uint32_t fb_bit(fb_t *b) {
  if (b->bitpos == 0) { b->cur = fb_byte(b); b->bitpos = 8; }
  b->bitpos--;
  return (b->cur >> b->bitpos) & 1u;
}
static uint32_t fb_bits(fb_t *b, int n) {
  uint32_t v = 0;
  for (int i = 0; i < n; i++) v = (v << 1) | fb_bit(b);
  return v;
}
static uint32_t fb_ue(fb_t *b) { /* 9.1 */
  int lz = 0;
  while (!fb_bit(b)) { if (++lz > 31 || b->err) { b->err = 1; return 0; } }
  return lz ? ((1u << lz) - 1u + fb_bits(b, lz)) : 0u;
}
static int32_t fb_se(fb_t *b) { /* 9.1.1 */
  uint32_t k = fb_ue(b);
  return (k & 1) ? (int32_t)((k + 1) / 2) : -(int32_t)(k / 2);
}
static int32_t fb_te(fb_t *b, int range) { /* 9.1: te(v) */
  if (range <= 0) return 0;
  if (range == 1) return !fb_bit(b);
  return (int32_t)fb_ue(b);
}
/* RBSP bit index (EPBs excluded) and the RBSP stop bit of a NAL payload */
static int64_t fb_index(const fb_t *b, int64_t epb_before) {
  (void)epb_before;
  return b->bitpos ? (b->pos - 1) * 8 + (8 - b->bitpos) : b->pos * 8;
}

/* ------------------------------------------------------- VLC tables (9.2) */
/* Table 9-5 coeff_token, one string per (TotalCoeff, TrailingOnes); NULL =
 * no such code.  Columns: 0<=nC<2, 2<=nC<4, 4<=nC<8, nC==-1 (4:2:0 chroma DC).
 * 8<=nC is the 6-bit fixed-length code (9.2.1). */
static const char *const CT[4][17][4] = {
  { /* 0 <= nC < 2 */
    {"1", 0, 0, 0},
    {"000101", "01", 0, 0},
    {"00000111", "000100", "001", 0},
    {"000000111", "00000110", "0000101", "00011"},
    {"0000000111", "000000110", "00000101", "000011"},
    {"00000000111", "0000000110", "000000101", "0000100"},
    {"0000000001111", "00000000110", "0000000101", "00000100"},
    {"0000000001011", "0000000001110", "00000000101", "000000100"},
    {"0000000001000", "0000000001010", "0000000001101", "0000000100"},
    {"00000000001111", "00000000001110", "0000000001001", "00000000100"},
    {"00000000001011", "00000000001010", "00000000001101", "0000000001100"},
    {"000000000001111", "000000000001110", "00000000001001", "00000000001100"},
    {"000000000001011", "000000000001010", "000000000001101", "00000000001000"},
    {"0000000000001111", "000000000000001", "000000000001001", "000000000001100"},
    {"0000000000001011", "0000000000001110", "0000000000001101", "000000000001000"},
    {"0000000000000111", "0000000000001010", "0000000000001001", "0000000000001100"},
    {"0000000000000100", "0000000000000110", "0000000000000101", "0000000000001000"},
  },
  { /* 2 <= nC < 4 */
    {"11", 0, 0, 0},
    {"001011", "10", 0, 0},
    {"000111", "00111", "011", 0},
    {"0000111", "001010", "001001", "0101"},
    {"00000111", "000110", "000101", "0100"},
    {"00000100", "0000110", "0000101", "00110"},
    {"000000111", "00000110", "00000101", "001000"},
    {"00000001111", "000000110", "000000101", "000100"},
    {"00000001011", "00000001110", "00000001101", "0000100"},
    {"000000001111", "00000001010", "00000001001", "000000100"},
    {"000000001011", "000000001110", "000000001101", "00000001100"},
    {"000000001000", "000000001010", "000000001001", "00000001000"},
    {"0000000001111", "0000000001110", "0000000001101", "000000001100"},
    {"0000000001011", "0000000001010", "0000000001001", "0000000001100"},
    {"0000000000111", "00000000001011", "0000000000110", "0000000001000"},
    {"00000000001001", "00000000001000", "00000000001010", "0000000000001"},
    {"00000000000111", "00000000000110", "00000000000101", "00000000000100"},
  },
  { /* 4 <= nC < 8 */
    {"1111", 0, 0, 0},
    {"001111", "1110", 0, 0},
    {"001011", "01111", "1101", 0},
    {"001000", "01100", "01110", "1100"},
    {"0001111", "01010", "01011", "1011"},
    {"0001011", "01000", "01001", "1010"},
    {"0001001", "001110", "001101", "1001"},
    {"0001000", "001010", "001001", "1000"},
    {"00001111", "0001110", "0001101", "01101"},
    {"00001011", "00001110", "0001010", "001100"},
    {"000001111", "00001010", "00001101", "0001100"},
    {"000001011", "000001110", "00001001", "00001100"},
    {"000001000", "000001010", "000001101", "00001000"},
    {"0000001101", "000000111", "000001001", "000001100"},
    {"0000001001", "0000001100", "0000001011", "0000001010"},
    {"0000000101", "0000001000", "0000000111", "0000000110"},
    {"0000000001", "0000000100", "0000000011", "0000000010"},
  },
  { /* nC == -1 */
    {"01", 0, 0, 0},
    {"000111", "1", 0, 0},
    {"000100", "000110", "001", 0},
    {"000011", "0000011", "0000010", "000101"},
    {"000010", "00000011", "00000010", "0000000"},
  },
};

/* Table 9-7 / 9-8: total_zeros for 4x4 blocks, row = TotalCoeff - 1,
 * column = total_zeros */
static const char *const TZ[15][16] = {
  {"1", "011", "010", "0011", "0010", "00011", "00010", "000011", "000010", "0000011",
   "0000010", "00000011", "00000010", "000000011", "000000010", "000000001"},
  {"111", "110", "101", "100", "011", "0101", "0100", "0011", "0010", "00011", "00010",
   "000011", "000010", "000001", "000000"},
  {"0101", "111", "110", "101", "0100", "0011", "100", "011", "0010", "00011", "00010",
   "000001", "00001", "000000"},
  {"00011", "111", "0101", "0100", "110", "101", "100", "0011", "011", "0010", "00010",
   "00001", "00000"},
  {"0101", "0100", "0011", "111", "110", "101", "100", "011", "0010", "00001", "0001",
   "00000"},
  {"000001", "00001", "111", "110", "101", "100", "011", "010", "0001", "001", "000000"},
  {"000001", "00001", "101", "100", "011", "11", "010", "0001", "001", "000000"},
  {"000001", "0001", "00001", "011", "11", "10", "010", "001", "000000"},
  {"000001", "000000", "0001", "11", "10", "001", "01", "00001"},
  {"00001", "00000", "001", "11", "10", "01", "0001"},
  {"0000", "0001", "001", "010", "1", "011"},
  {"0000", "0001", "01", "1", "001"},
  {"000", "001", "1", "01"},
  {"00", "01", "1"},
  {"0", "1"},
};
/* Table 9-9a: total_zeros for 4:2:0 chroma DC, row = TotalCoeff - 1 */
static const char *const TZC[3][4] = {
  {"1", "01", "001", "000"},
  {"1", "01", "00"},
  {"1", "0"},
};
/* Table 9-10: run_before, row = min(zerosLeft, 7) - 1 */
static const char *const RB[7][15] = {
  {"1", "0"},
  {"1", "01", "00"},
  {"11", "10", "01", "00"},
  {"11", "10", "01", "001", "000"},
  {"11", "10", "011", "010", "001", "000"},
  {"11", "000", "001", "011", "010", "101", "100"},
  {"111", "110", "101", "100", "011", "010", "001", "0001", "00001", "000001", "0000001",
   "00000001", "000000001", "0000000001", "00000000001"},
};

/* The strings as (length, value) pairs, converted once when the library
 * loads (matching stays exact: a code is its length and its bits). */
typedef struct {
  int n;
  uint8_t len[68];
  uint32_t val[68];
} fo_vlc;
static fo_vlc VLC_CT[4], VLC_TZ[15], VLC_TZC[3], VLC_RB[7];

static void vlc_make(fo_vlc *t, const char *const *table, int n) {
  t->n = n;
  for (int i = 0; i < n; i++) {
    t->len[i] = 0;
    t->val[i] = 0;
    if (!table[i]) continue;
    for (const char *c = table[i]; *c; c++) {
      t->val[i] = (t->val[i] << 1) | (uint32_t)(*c - '0');
      t->len[i]++;
    }
  }
}

__attribute__((constructor)) static void vlc_init(void) {
  for (int c = 0; c < 4; c++) {
    const char *flat[68];
    for (int r = 0; r < 17; r++)
      for (int k = 0; k < 4; k++) flat[r * 4 + k] = CT[c][r][k];
    vlc_make(&VLC_CT[c], flat, c == 3 ? 20 : 68);
  }
  for (int t = 0; t < 15; t++) vlc_make(&VLC_TZ[t], TZ[t], 16);
  for (int t = 0; t < 3; t++) vlc_make(&VLC_TZC[t], TZC[t], 4);
  for (int r = 0; r < 7; r++) vlc_make(&VLC_RB[r], RB[r], 15);
}

/* Read one code of table t: the entry index, or -1 (no code within 16 bits). */
static int fb_vlc(fb_t *b, const fo_vlc *t) {
  uint32_t v = 0;
  for (int len = 1; len <= 16; len++) {
    v = (v << 1) | fb_bit(b);
    if (b->err) return -1;
    for (int i = 0; i < t->n; i++)
      if (t->len[i] == len && t->val[i] == v) return i;
  }
  return -1;
}

/* Exported for tests/test_h264_tables.py: the standard's strings. */
const char *fo_table_code(int table, int a, int b, int c) {
  switch (table) {
    case 0: return (a >= 0 && a < 4 && b >= 0 && b < 17 && c >= 0 && c < 4) ? CT[a][b][c] : 0;
    case 1: return (a >= 0 && a < 15 && b >= 0 && b < 16) ? TZ[a][b] : 0;
    case 2: return (a >= 0 && a < 3 && b >= 0 && b < 4) ? TZC[a][b] : 0;
    case 3: return (a >= 0 && a < 7 && b >= 0 && b < 15) ? RB[a][b] : 0;
    default: return 0;
  }
}

/* ------------------------------------------------------- other tables */
static const int ZZ4[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15}; /* 8.5.6 frame */
/* Table 9-4 (chroma_format_idc 1): codeNum -> coded_block_pattern */
static const int CBP_INTRA[48] = {47, 31, 15, 0,  23, 27, 29, 30, 7,  11, 13, 14, 39, 43, 45, 46,
                                  16, 3,  5,  10, 12, 19, 21, 26, 28, 35, 37, 42, 44, 1,  2,  4,
                                  8,  17, 18, 20, 24, 6,  9,  22, 25, 32, 33, 34, 36, 40, 38, 41};
static const int CBP_INTER[48] = {0,  16, 1,  2,  4,  8,  32, 3,  5,  10, 12, 15, 47, 7,  11, 13,
                                  14, 6,  9,  31, 35, 37, 42, 44, 33, 34, 36, 40, 39, 43, 45, 46,
                                  17, 18, 20, 24, 19, 21, 26, 28, 23, 27, 29, 30, 22, 25, 38, 41};
/* 8.5.9: normAdjust4x4 v */
static const int NORM_V[6][3] = {{10, 16, 13}, {11, 18, 14}, {13, 20, 16},
                                 {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};
/* Table 8-15: QPc for qPI >= 30 */
static const int QPC_TAB[22] = {29, 30, 31, 32, 32, 33, 34, 34, 35, 35, 36,
                                36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};
/* Table 8-16 / 8-17 */
static const int ALPHA[52] = {0,  0,  0,  0,  0,  0,  0,  0,   0,   0,   0,   0,   0,
                              0,  0,  0,  4,  4,  5,  6,  7,   8,   9,   10,  12,  13,
                              15, 17, 20, 22, 25, 28, 32, 36,  40,  45,  50,  56,  63,
                              71, 80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255};
static const int BETA[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  2,  2,
                             2,  3,  3,  3,  3,  4,  4,  4,  6,  6,  7,  7,  8,  8,  9,  9,  10, 10,
                             11, 11, 12, 12, 13, 13, 14, 14, 15, 15, 16, 16, 17, 17, 18, 18};
static const int TC0[52][3] = {
  {0, 0, 0},   {0, 0, 0},   {0, 0, 0},   {0, 0, 0},  {0, 0, 0},  {0, 0, 0},  {0, 0, 0},
  {0, 0, 0},   {0, 0, 0},   {0, 0, 0},   {0, 0, 0},  {0, 0, 0},  {0, 0, 0},  {0, 0, 0},
  {0, 0, 0},   {0, 0, 0},   {0, 0, 0},   {0, 0, 1},  {0, 0, 1},  {0, 0, 1},  {0, 0, 1},
  {0, 1, 1},   {0, 1, 1},   {1, 1, 1},   {1, 1, 1},  {1, 1, 1},  {1, 1, 1},  {1, 1, 2},
  {1, 1, 2},   {1, 1, 2},   {1, 1, 2},   {1, 2, 3},  {1, 2, 3},  {2, 2, 3},  {2, 2, 4},
  {2, 3, 4},   {2, 3, 4},   {3, 3, 5},   {3, 4, 6},  {3, 4, 6},  {4, 5, 7},  {4, 5, 8},
  {4, 6, 9},   {5, 7, 10},  {6, 8, 11},  {6, 8, 13}, {7, 10, 14}, {8, 11, 16}, {9, 12, 18},
  {10, 13, 20}, {11, 15, 23}, {13, 17, 25}};

/* luma4x4BlkIdx -> (x, y) in 4x4 block units (6.4.3) */
static const int BLK_X[16] = {0, 1, 0, 1, 2, 3, 2, 3, 0, 1, 0, 1, 2, 3, 2, 3};
static const int BLK_Y[16] = {0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3};

static int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }
static int clip1(int v) { return clip3(0, 255, v); }
static int iabs(int v) { return v < 0 ? -v : v; }
static int imin(int a, int b) { return a < b ? a : b; }
static int median3(int a, int b, int c) {
  int mx = a > b ? a : b, mn = a < b ? a : b;
  return c > mx ? mx : (c < mn ? mn : c);
}

/* ------------------------------------------------- parameter sets (7.3.2) */
static int ZZ8[64]; /* 8.5.7 8x8 zig-zag (fo_tables_init) */
static void fo_tables_init(void);
typedef struct {
  int valid, profile_idc, log2_max_frame_num, poc_type, log2_max_poc_lsb, dpoaz;
  int max_num_ref_frames, gaps, mbw, mbh, crop_l, crop_r, crop_t, crop_b;
  int direct8x8;                     /* direct_8x8_inference_flag */
  int off_non_ref, off_t2b, ncycle;  /* POC type 1 (7.4.2.1.1) */
  int off_ref[256];
  uint8_t sl4[6][16], sl8[2][64];    /* sequence-level scaling lists (scan order; 16s when absent) */
  int seq_scaling;                   /* seq_scaling_matrix_present_flag */
} fo_sps;
typedef struct {
  int valid, sps_id, bfpo, num_ref_l0, num_ref_l1, weighted_pred, weighted_bipred, pic_init_qp;
  int cqp_off, cqp_off2, deblock_ctrl, cip, redundant;
  int cabac, t8mode;   /* entropy_coding_mode_flag, transform_8x8_mode_flag */
  int pic_scaling;     /* pic_scaling_matrix_present_flag */
  /* weightScale4x4 / 8x8 in raster order (8.5.6 / 8.5.7 inverse scans of the
     picture's scaling lists): lists Intra Y, Cb, Cr, Inter Y, Cb, Cr / Intra Y, Inter Y */
  uint8_t w4[6][16], w8[2][64];
} fo_pps;

/* 7.3.2.1.1.1 scaling_list(): returns useDefaultScalingMatrixFlag */
static int fo_scaling_list(fb_t *b, int size, uint8_t *list) {
  int last_scale = 8, next_scale = 8, use_default = 0;
  for (int j = 0; j < size; j++) {
    if (next_scale != 0) {
      int delta_scale = fb_se(b);
      next_scale = (last_scale + delta_scale + 256) % 256;
      use_default = (j == 0 && next_scale == 0);
    }
    list[j] = (uint8_t)(next_scale == 0 ? last_scale : next_scale);
    last_scale = list[j];
  }
  return use_default;
}
/* the 8 (4:2:0) scaling lists of an SPS (fall-back rule A) or a PPS (rule
 * B: lists 0, 3, 6, 7 fall back to the SPS's own), Table 7-2; n_sent =
 * how many list flags the parameter set carries */
static void fo_scaling_matrix(fb_t *b, int n_sent, const fo_sps *seq, uint8_t (*l4)[16], uint8_t (*l8)[64]) {
  for (int i = 0; i < 8; i++) {
    int sent = i < n_sent ? (int)fb_bit(b) : 0;
    int size = i < 6 ? 16 : 64, cls = (i < 3 || i == 6) ? 0 : 1; /* 0 intra, 1 inter */
    uint8_t *dst = i < 6 ? l4[i] : l8[i - 6];
    const uint8_t *dflt = i < 6 ? FO_DEFAULT_4x4[cls] : FO_DEFAULT_8x8[cls];
    if (sent) {
      if (fo_scaling_list(b, size, dst)) memcpy(dst, dflt, (size_t)size);
    } else if (i == 0 || i == 3 || i >= 6) { /* rule A: the default; rule B: the SPS's list */
      const uint8_t *src = !seq ? dflt : (i < 6 ? seq->sl4[i] : seq->sl8[i - 6]);
      memcpy(dst, src, (size_t)size);
    } else {                                  /* both rules: the previous list */
      memcpy(dst, l4[i - 1], 16);
    }
  }
}

static int is_high(int p) {
  return p == 100 || p == 110 || p == 122 || p == 244 || p == 44 || p == 83 || p == 86 ||
         p == 118 || p == 128 || p == 138 || p == 139 || p == 134 || p == 135;
}

static int parse_sps(const uint8_t *nal, int64_t n, fo_sps *tab, char *err) {
  fb_t b;
  fb_init(&b, nal + 1, n - 1);
  fo_sps s;
  memset(&s, 0, sizeof s);
  s.profile_idc = (int)fb_bits(&b, 8);
  fb_bits(&b, 16);
  uint32_t id = fb_ue(&b);
  if (id > 31) return FO_E_FORMAT;
  if (is_high(s.profile_idc)) {
    if (fb_ue(&b) != 1) { strcpy(err, "chroma_format_idc != 1"); return FO_E_UNSUPPORTED; }
    if (fb_ue(&b) || fb_ue(&b)) { strcpy(err, "bit depth > 8"); return FO_E_UNSUPPORTED; }
    fb_bit(&b);
  }
  memset(s.sl4, 16, sizeof s.sl4); /* Flat_4x4_16 / Flat_8x8_16 */
  memset(s.sl8, 16, sizeof s.sl8);
  if (is_high(s.profile_idc) && fb_bit(&b)) {
    s.seq_scaling = 1;
    fo_scaling_matrix(&b, 8, NULL, s.sl4, s.sl8);
  }
  s.log2_max_frame_num = (int)fb_ue(&b) + 4;
  s.poc_type = (int)fb_ue(&b);
  if (s.poc_type == 0) {
    s.log2_max_poc_lsb = (int)fb_ue(&b) + 4;
  } else if (s.poc_type == 1) {
    s.dpoaz = (int)fb_bit(&b);
    s.off_non_ref = fb_se(&b);
    s.off_t2b = fb_se(&b);
    uint32_t nc = fb_ue(&b);
    if (nc > 255) return FO_E_FORMAT;
    s.ncycle = (int)nc;
    for (uint32_t i = 0; i < nc; i++) s.off_ref[i] = fb_se(&b);
  }
  s.max_num_ref_frames = (int)fb_ue(&b);
  s.gaps = (int)fb_bit(&b);
  s.mbw = (int)fb_ue(&b) + 1;
  s.mbh = (int)fb_ue(&b) + 1;
  if (!fb_bit(&b)) { strcpy(err, "interlaced (frame_mbs_only_flag 0)"); return FO_E_UNSUPPORTED; }
  s.direct8x8 = (int)fb_bit(&b);
  if (fb_bit(&b)) {
    s.crop_l = 2 * (int)fb_ue(&b);
    s.crop_r = 2 * (int)fb_ue(&b);
    s.crop_t = 2 * (int)fb_ue(&b);
    s.crop_b = 2 * (int)fb_ue(&b);
  }
  if (b.err || s.mbw > 512 || s.mbh > 512) return FO_E_FORMAT;
  s.valid = 1;
  tab[id] = s;
  return 0;
}

static int parse_pps(const uint8_t *nal, int64_t n, fo_pps *tab, const fo_sps *sps_tab, char *err) {
  fb_t b;
  fb_init(&b, nal + 1, n - 1);
  fo_pps p;
  memset(&p, 0, sizeof p);
  uint32_t id = fb_ue(&b);
  if (id > 255) return FO_E_FORMAT;
  p.sps_id = (int)fb_ue(&b);
  p.cabac = (int)fb_bit(&b);
  p.bfpo = (int)fb_bit(&b);
  if (fb_ue(&b)) { strcpy(err, "slice groups (FMO)"); return FO_E_UNSUPPORTED; }
  p.num_ref_l0 = (int)fb_ue(&b) + 1;
  p.num_ref_l1 = (int)fb_ue(&b) + 1;
  p.weighted_pred = (int)fb_bit(&b);
  p.weighted_bipred = (int)fb_bits(&b, 2);
  p.pic_init_qp = 26 + fb_se(&b);
  fb_se(&b); /* pic_init_qs */
  p.cqp_off = fb_se(&b);
  p.deblock_ctrl = (int)fb_bit(&b);
  p.cip = (int)fb_bit(&b);
  p.redundant = (int)fb_bit(&b);
  p.cqp_off2 = p.cqp_off;
  /* more_rbsp_data(): High-profile extension */
  {
    int64_t last = n - 1;
    while (last > 0 && nal[last] == 0) last--;
    int64_t pos_bits = fb_index(&b, 0);
    /* the stop bit lies in the last non-zero byte; compare in EBSP bytes
       (the tail holds no emulation-prevention byte in practice) */
    int tz = 0;
    while (!((nal[last] >> tz) & 1)) tz++;
    int64_t stop = (last - 1) * 8 + (7 - tz);
    const fo_sps *S = &sps_tab[p.sps_id & 31];
    uint8_t l4[6][16], l8[2][64];
    memcpy(l4, S->sl4, sizeof l4); /* no picture-level matrix: the sequence's */
    memcpy(l8, S->sl8, sizeof l8);
    if (pos_bits < stop) {
      p.t8mode = (int)fb_bit(&b);
      p.pic_scaling = (int)fb_bit(&b);
      /* 7.4.2.2: rule B only when the SPS carries seq_scaling_matrix_present_flag
         1; with Flat_16 sequence lists the PPS falls back by rule A */
      if (p.pic_scaling) fo_scaling_matrix(&b, 6 + 2 * p.t8mode, S->seq_scaling ? S : NULL, l4, l8);
      p.cqp_off2 = fb_se(&b);
    }
    fo_tables_init(); /* ZZ8 */
    for (int l = 0; l < 6; l++)
      for (int k = 0; k < 16; k++) p.w4[l][ZZ4[k]] = l4[l][k];
    for (int l = 0; l < 2; l++)
      for (int k = 0; k < 64; k++) p.w8[l][ZZ8[k]] = l8[l][k];
  }
  if (b.err) return FO_E_FORMAT;
  if (p.redundant) { strcpy(err, "redundant pictures"); return FO_E_UNSUPPORTED; }
  p.valid = 1;
  tab[id] = p;
  return 0;
}

/* ------------------------------------------------------------- pictures */
typedef struct {
  uint8_t *y, *u, *v;   /* coded size */
  int frame_num, frame_num_wrap, lt_idx;
  int ref;              /* 0 unused, 1 short-term, 2 long-term */
  int id;               /* identity for bS comparisons */
  int poc;              /* PicOrderCnt (8.2.1) */
  /* motion of the decoded picture, per macroblock x raster 4x4 block, kept
     for the direct prediction of later B pictures (8.4.1.2.1 colocated) */
  int8_t *mref[2];      /* refIdxLX, -1: list unused or intra */
  int16_t *mmv[2];      /* mvLX (x, y) */
  int32_t *mpic[2];     /* id of the picture refIdxLX named */
} fo_pic;

static void pic_free(fo_pic *p) {
  free(p->y); free(p->u); free(p->v);
  for (int l = 0; l < 2; l++) { free(p->mref[l]); free(p->mmv[l]); free(p->mpic[l]); }
  p->y = p->u = p->v = NULL;
  for (int l = 0; l < 2; l++) { p->mref[l] = NULL; p->mmv[l] = NULL; p->mpic[l] = NULL; }
}

typedef struct {
  int type;     /* 0 P inter, 1 I_NxN, 2 I_16x16, 3 I_PCM, 4 P_Skip */
  int slice;    /* slice number in the picture, -1 = not decoded */
  int qp;       /* QPY */
  int cbp;
  int i4[16];   /* Intra4x4PredMode per raster 4x4 block */
  int refidx[2][16];   /* per list, per raster 4x4 block; -1: list unused / intra */
  int refpic[2][16];   /* picture id per list and raster 4x4 block (-1: none) */
  int mv[2][16][2];
  int nz[16];       /* total_coeff per raster luma 4x4 block (8x8 transform: the 8x8's count) */
  int nzc[2][4];    /* chroma AC total_coeff, raster 2x2 */
  int t8;           /* transform_size_8x8_flag (I_NxN with it = I_8x8) */
  int cmode;        /* intra_chroma_pred_mode */
  int mvd[2][16][2];   /* CABAC: mvd_lX per raster 4x4 block (context of later mvds) */
  uint32_t cbf;     /* CABAC coded_block_flag: bit 0 Intra16x16 DC, 1 + raster luma 4x4,
                       17 + iCbCr chroma DC, 19 + 4 iCbCr + raster chroma AC */
  int qpd;          /* mb_qp_delta */
  int direct8;      /* B: 8x8 quadrants predicted in direct mode (B_Skip / B_Direct_16x16: 15 and d16) */
  int d16;          /* B_Skip or B_Direct_16x16 */
} fo_mb;

typedef struct {
  int idc, off_a, off_b;
} fo_slice_dbk;

typedef struct {
  fo_sps sps[32];
  fo_pps pps[256];
  const fo_sps *S;
  const fo_pps *P;
  int mbw, mbh, W, H, nmb;
  fo_pic dpb[17];       /* reference + current */
  int ndpb;
  int next_id;
  fo_mb *mb;
  fo_slice_dbk dbk[4096];
  int nslices;
  int max_lt_idx;       /* -1: no long-term frame indices */
  int prev_ref_frame_num;
  /* 8.2.1 picture order count state */
  int prev_poc_msb, prev_poc_lsb;   /* of the previous reference picture (type 0) */
  int prev_fn_offset, prev_fn;      /* FrameNumOffset / frame_num of the previous picture (types 1, 2) */
  int prev_mmco5;                   /* the previous picture had memory_management_control_operation 5 */
  int flags;
  char *err;
  int64_t enc_pos_qp, enc_pos_data;  /* synthesis: RBSP bit positions in the source slice header */
} fo_dec;

static int fo_fail(fo_dec *d, int rc, const char *msg) {
  if (d->err && !d->err[0]) snprintf(d->err, 200, "%s", msg);
  return rc;
}

/* ------------------------------------------- neighbour locations (6.4.12) */
typedef struct {
  int mb;       /* address or -1 */
  int xw, yw;   /* location inside mb */
} fo_loc;

/* luma (maxW = 16) or chroma (maxW = 8) location (xN, yN) relative to the
 * current macroblock; availability per 6.4.8 (same slice, lower address) */
static fo_loc nb_loc(const fo_dec *d, int cur, int xN, int yN, int maxW, int maxH) {
  fo_loc r = {-1, 0, 0};
  int mx = cur % d->mbw, n = -1;
  if (yN > maxH - 1) return r;
  if (xN < 0 && yN < 0) n = mx > 0 ? cur - d->mbw - 1 : -1;
  else if (xN < 0 && yN < maxH) n = mx > 0 ? cur - 1 : -1;
  else if (xN < maxW && yN < 0) n = cur - d->mbw;
  else if (xN < maxW) n = cur;
  else if (yN < 0) n = mx < d->mbw - 1 ? cur - d->mbw + 1 : -1;
  else return r;
  if (n < 0 || n >= d->nmb) return r;
  if (n != cur && (n > cur || d->mb[n].slice != d->mb[cur].slice)) return r;
  r.mb = n;
  r.xw = (xN + maxW) % maxW;
  r.yw = (yN + maxH) % maxH;
  return r;
}

/* -------------------------------------------------------- CAVLC (9.2) */
static int nc_of(const fo_dec *d, int cur, int blk_x, int blk_y, int chroma, int plane) {
  /* blk_x/blk_y: 4x4 block position (luma 0..3, chroma 0..1) */
  int maxW = chroma ? 8 : 16;
  fo_loc A = nb_loc(d, cur, blk_x * 4 - 1, blk_y * 4, maxW, maxW);
  fo_loc B = nb_loc(d, cur, blk_x * 4, blk_y * 4 - 1, maxW, maxW);
  int nA = 0, nB = 0;
  const fo_loc *L[2] = {&A, &B};
  int *out[2] = {&nA, &nB};
  for (int i = 0; i < 2; i++) {
    if (L[i]->mb < 0) continue;
    const fo_mb *m = &d->mb[L[i]->mb];
    int v;
    if (m->type == 4) v = 0;
    else if (m->type == 3) v = 16;
    else if (chroma) v = m->nzc[plane][(L[i]->yw / 4) * 2 + L[i]->xw / 4];
    else v = m->nz[(L[i]->yw / 4) * 4 + L[i]->xw / 4];
    *out[i] = v;
  }
  if (A.mb >= 0 && B.mb >= 0) return (nA + nB + 1) >> 1;
  if (A.mb >= 0) return nA;
  if (B.mb >= 0) return nB;
  return 0;
}

/* residual_block_cavlc (7.3.5.3.2 / 9.2): coeffLevel[startIdx..endIdx]; returns
 * TotalCoeff or < 0 */
static int residual_block(fb_t *b, int nC, int start, int end, int maxNum, int *coef) {
  for (int i = 0; i < maxNum; i++) coef[i] = 0;
  int tc, t1;
  if (nC >= 8) {
    uint32_t v = fb_bits(b, 6);
    if (v == 3) { tc = 0; t1 = 0; }
    else {
      tc = (int)(v >> 2) + 1;
      t1 = (int)(v & 3);
      if (t1 > tc || (t1 == 3 && tc < 3)) return -1;
    }
  } else {
    int col = nC == -1 ? 3 : (nC < 2 ? 0 : (nC < 4 ? 1 : 2));
    int idx = fb_vlc(b, &VLC_CT[col]);
    if (idx < 0) return -1;
    tc = idx / 4;
    t1 = idx % 4;
  }
  if (tc > maxNum) return -1;
  if (tc == 0) return 0;
  int level[16], run[16];
  int suffixLength = (tc > 10 && t1 < 3) ? 1 : 0;
  for (int i = 0; i < tc; i++) {
    if (i < t1) {
      level[i] = fb_bit(b) ? -1 : 1;
      continue;
    }
    int prefix = 0;
    while (!fb_bit(b)) { if (++prefix > 31 || b->err) return -1; }
    int levelCode = (imin(15, prefix) << suffixLength);
    int size = (prefix == 14 && suffixLength == 0) ? 4 : (prefix >= 15 ? prefix - 3 : suffixLength);
    if (size > 0) levelCode += (int)fb_bits(b, size);
    if (prefix >= 15 && suffixLength == 0) levelCode += 15;
    if (prefix >= 16) levelCode += (1 << (prefix - 3)) - 4096;
    if (i == t1 && t1 < 3) levelCode += 2;
    level[i] = (levelCode % 2 == 0) ? (levelCode + 2) >> 1 : (-levelCode - 1) >> 1;
    if (suffixLength == 0) suffixLength = 1;
    if (iabs(level[i]) > (3 << (suffixLength - 1)) && suffixLength < 6) suffixLength++;
  }
  int zerosLeft = 0;
  if (tc < end - start + 1) {
    int tz;
    tz = fb_vlc(b, maxNum == 4 ? &VLC_TZC[tc - 1] : &VLC_TZ[tc - 1]);
    if (tz < 0) return -1;
    zerosLeft = tz;
  }
  for (int i = 0; i < tc - 1; i++) {
    if (zerosLeft > 0) {
      int rb = fb_vlc(b, &VLC_RB[imin(zerosLeft, 7) - 1]);
      if (rb < 0 || rb > zerosLeft) return -1;
      run[i] = rb;
    } else {
      run[i] = 0;
    }
    zerosLeft -= run[i];
  }
  run[tc - 1] = zerosLeft;
  int coeffNum = -1;
  for (int i = tc - 1; i >= 0; i--) {
    coeffNum += run[i] + 1;
    if (start + coeffNum > end) return -1;
    coef[start + coeffNum] = level[i];
  }
  return tc;
}

/* ------------------------------------------------- transforms (8.5) */
static int qpc_of(int qpy, int off) {
  int qpi = clip3(0, 51, qpy + off);
  return qpi < 30 ? qpi : QPC_TAB[qpi - 30];
}
/* 8.5.9: LevelScale4x4(m, i, j) = weightScale4x4(i, j) * normAdjust4x4(m, i, j);
 * w = the block's weightScale4x4 in raster order */
static int level_scale(const uint8_t *w, int m, int i, int j) {
  int k = ((i & 1) == 0 && (j & 1) == 0) ? 0 : (((i & 1) == 1 && (j & 1) == 1) ? 1 : 2);
  return w[i * 4 + j] * NORM_V[m][k];
}
/* c: 4x4 coefficients in raster (row i, column j); dc_done: c[0] is an
 * already-scaled DC (Intra16x16 / chroma); out r: residual samples */
static void scale_idct4(const int *c, int qp, const uint8_t *w, int dc_done, int *r) {
  int d[16];
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      int k = i * 4 + j;
      if (k == 0 && dc_done) { d[0] = c[0]; continue; }
      int ls = level_scale(w, qp % 6, i, j);
      if (qp >= 24) d[k] = (c[k] * ls) << (qp / 6 - 4);
      else d[k] = (c[k] * ls + (1 << (3 - qp / 6))) >> (4 - qp / 6);
    }
  int f[16], h[16];
  for (int i = 0; i < 4; i++) { /* rows (8.5.12.2) */
    int e0 = d[i * 4 + 0] + d[i * 4 + 2], e1 = d[i * 4 + 0] - d[i * 4 + 2];
    int e2 = (d[i * 4 + 1] >> 1) - d[i * 4 + 3], e3 = d[i * 4 + 1] + (d[i * 4 + 3] >> 1);
    f[i * 4 + 0] = e0 + e3;
    f[i * 4 + 1] = e1 + e2;
    f[i * 4 + 2] = e1 - e2;
    f[i * 4 + 3] = e0 - e3;
  }
  for (int j = 0; j < 4; j++) { /* columns */
    int g0 = f[0 * 4 + j] + f[2 * 4 + j], g1 = f[0 * 4 + j] - f[2 * 4 + j];
    int g2 = (f[1 * 4 + j] >> 1) - f[3 * 4 + j], g3 = f[1 * 4 + j] + (f[3 * 4 + j] >> 1);
    h[0 * 4 + j] = g0 + g3;
    h[1 * 4 + j] = g1 + g2;
    h[2 * 4 + j] = g1 - g2;
    h[3 * 4 + j] = g0 - g3;
  }
  for (int k = 0; k < 16; k++) r[k] = (h[k] + 32) >> 6;
}

/* ------------------------------------------------- intra prediction (8.3) */
/* sample of the current picture at absolute luma/chroma position */
typedef struct {
  int avail;
  int v;
} fo_s;

static int intra_nb_ok(const fo_dec *d, int n) {
  if (n < 0) return 0;
  if (d->P->cip && (d->mb[n].type == 0 || d->mb[n].type == 4)) return 0; /* 8.3.1.2 */
  return 1;
}

/* sample p[x, y] (x, y relative to the block at luma (bx0, by0) of MB cur),
 * luma; block-order availability inside the MB via `done` (raster 4x4 mask) */
static fo_s luma_nb(const fo_dec *d, const fo_pic *pic, int cur, int xo, int yo, int x, int y,
                    int done_mask) {
  fo_s s = {0, 0};
  int xN = xo + x, yN = yo + y;
  fo_loc L = nb_loc(d, cur, xN, yN, 16, 16);
  if (L.mb < 0 || !intra_nb_ok(d, L.mb)) return s;
  if (L.mb == cur) {
    int blk = (L.yw / 4) * 4 + L.xw / 4;
    if (!((done_mask >> blk) & 1)) return s;
  }
  int mx = L.mb % d->mbw, my = L.mb / d->mbw;
  s.avail = 1;
  s.v = pic->y[(int64_t)(my * 16 + L.yw) * d->W + mx * 16 + L.xw];
  return s;
}

static void intra4x4(const fo_dec *d, fo_pic *pic, int cur, int blk, int mode, int done_mask,
                     int pred[16]) {
  int xo = BLK_X[blk] * 4, yo = BLK_Y[blk] * 4;
  int T[9], L[5], tav[8], lav[4], cav; /* T[0] = p[-1,-1], T[1+x] = p[x,-1]; L[1+y] = p[-1,y] */
  fo_s s = luma_nb(d, pic, cur, xo, yo, -1, -1, done_mask);
  cav = s.avail;
  T[0] = L[0] = s.v;
  for (int x = 0; x < 8; x++) {
    s = luma_nb(d, pic, cur, xo, yo, x, -1, done_mask);
    tav[x] = s.avail;
    T[1 + x] = s.v;
  }
  for (int y = 0; y < 4; y++) {
    s = luma_nb(d, pic, cur, xo, yo, -1, y, done_mask);
    lav[y] = s.avail;
    L[1 + y] = s.v;
  }
  if (!tav[4] && tav[3]) /* 8.3.1.2: substitute p[3,-1] for p[4..7,-1] */
    for (int x = 4; x < 8; x++) { T[1 + x] = T[4]; tav[x] = 1; }
  (void)cav;
#define PT(x) T[1 + (x)]
#define PL(y) L[1 + (y)]
  for (int y = 0; y < 4; y++)
    for (int x = 0; x < 4; x++) {
      int v = 128;
      switch (mode) {
        case 0: v = PT(x); break;
        case 1: v = PL(y); break;
        case 2: {
          int ta = tav[0] && tav[1] && tav[2] && tav[3], la = lav[0] && lav[1] && lav[2] && lav[3];
          if (ta && la) v = (PT(0) + PT(1) + PT(2) + PT(3) + PL(0) + PL(1) + PL(2) + PL(3) + 4) >> 3;
          else if (la) v = (PL(0) + PL(1) + PL(2) + PL(3) + 2) >> 2;
          else if (ta) v = (PT(0) + PT(1) + PT(2) + PT(3) + 2) >> 2;
          else v = 128;
          break;
        }
        case 3:
          if (x == 3 && y == 3) v = (PT(6) + 3 * PT(7) + 2) >> 2;
          else v = (PT(x + y) + 2 * PT(x + y + 1) + PT(x + y + 2) + 2) >> 2;
          break;
        case 4:
          if (x > y) v = (PT(x - y - 2) + 2 * PT(x - y - 1) + PT(x - y) + 2) >> 2;
          else if (x < y) v = (PL(y - x - 2) + 2 * PL(y - x - 1) + PL(y - x) + 2) >> 2;
          else v = (PT(0) + 2 * PT(-1) + PL(0) + 2) >> 2;
          break;
        case 5: {
          int z = 2 * x - y;
          if (z >= 0 && !(z & 1)) v = (PT(x - (y >> 1) - 1) + PT(x - (y >> 1)) + 1) >> 1;
          else if (z >= 0) v = (PT(x - (y >> 1) - 2) + 2 * PT(x - (y >> 1) - 1) + PT(x - (y >> 1)) + 2) >> 2;
          else if (z == -1) v = (PL(0) + 2 * PL(-1) + PT(0) + 2) >> 2;
          else v = (PL(y - 1) + 2 * PL(y - 2) + PL(y - 3) + 2) >> 2;
          break;
        }
        case 6: {
          int z = 2 * y - x;
          if (z >= 0 && !(z & 1)) v = (PL(y - (x >> 1) - 1) + PL(y - (x >> 1)) + 1) >> 1;
          else if (z >= 0) v = (PL(y - (x >> 1) - 2) + 2 * PL(y - (x >> 1) - 1) + PL(y - (x >> 1)) + 2) >> 2;
          else if (z == -1) v = (PL(0) + 2 * PL(-1) + PT(0) + 2) >> 2;
          else v = (PT(x - 1) + 2 * PT(x - 2) + PT(x - 3) + 2) >> 2;
          break;
        }
        case 7:
          if (y == 0 || y == 2) v = (PT(x + (y >> 1)) + PT(x + (y >> 1) + 1) + 1) >> 1;
          else v = (PT(x + (y >> 1)) + 2 * PT(x + (y >> 1) + 1) + PT(x + (y >> 1) + 2) + 2) >> 2;
          break;
        case 8: {
          int z = x + 2 * y;
          if (z == 0 || z == 2 || z == 4) v = (PL(y + (x >> 1)) + PL(y + (x >> 1) + 1) + 1) >> 1;
          else if (z == 1 || z == 3) v = (PL(y + (x >> 1)) + 2 * PL(y + (x >> 1) + 1) + PL(y + (x >> 1) + 2) + 2) >> 2;
          else if (z == 5) v = (PL(2) + 3 * PL(3) + 2) >> 2;
          else v = PL(3);
          break;
        }
      }
      pred[y * 4 + x] = v;
    }
#undef PT
#undef PL
}

/* 16x16 luma (8.3.3) or 8x8 chroma (8.3.4) prediction into pred[size*size] */
static void intra_big(const fo_dec *d, fo_pic *pic, int cur, int plane, int mode, int *pred) {
  int chroma = plane > 0, n = chroma ? 8 : 16, W = chroma ? d->W / 2 : d->W;
  const uint8_t *img = plane == 0 ? pic->y : (plane == 1 ? pic->u : pic->v);
  int mx = cur % d->mbw, my = cur / d->mbw;
  int T[17], L[17], ta = 1, la = 1, ca;
  /* neighbour MBs: A (left), B (above), D (above-left) */
  fo_loc A = nb_loc(d, cur, -1, 0, n, n), B = nb_loc(d, cur, 0, -1, n, n), D = nb_loc(d, cur, -1, -1, n, n);
  la = A.mb >= 0 && intra_nb_ok(d, A.mb);
  ta = B.mb >= 0 && intra_nb_ok(d, B.mb);
  ca = D.mb >= 0 && intra_nb_ok(d, D.mb);
  for (int i = 0; i < n; i++) {
    T[1 + i] = ta ? img[(int64_t)(my * n - 1) * W + mx * n + i] : 0;
    L[1 + i] = la ? img[(int64_t)(my * n + i) * W + mx * n - 1] : 0;
  }
  T[0] = L[0] = ca ? img[(int64_t)(my * n - 1) * W + mx * n - 1] : 0;
#define PT(x) T[1 + (x)]
#define PL(y) L[1 + (y)]
  if (!chroma) {
    for (int y = 0; y < 16; y++)
      for (int x = 0; x < 16; x++) {
        int v = 128;
        if (mode == 0) v = PT(x);
        else if (mode == 1) v = PL(y);
        else if (mode == 2) {
          int st = 0, sl = 0;
          for (int i = 0; i < 16; i++) { st += PT(i); sl += PL(i); }
          if (ta && la) v = (st + sl + 16) >> 5;
          else if (la) v = (sl + 8) >> 4;
          else if (ta) v = (st + 8) >> 4;
          else v = 128;
        } else {
          int H = 0, V = 0;
          for (int i = 0; i < 8; i++) {
            H += (i + 1) * (PT(8 + i) - PT(6 - i));
            V += (i + 1) * (PL(8 + i) - PL(6 - i));
          }
          int a = 16 * (PL(15) + PT(15)), bb = (5 * H + 32) >> 6, c = (5 * V + 32) >> 6;
          v = clip1((a + bb * (x - 7) + c * (y - 7) + 16) >> 5);
        }
        pred[y * 16 + x] = v;
      }
  } else {
    for (int y = 0; y < 8; y++)
      for (int x = 0; x < 8; x++) {
        int v = 128;
        if (mode == 0) { /* DC per 4x4 chroma block (8.3.4.1-3) */
          int xO = x & 4, yO = y & 4, st = 0, sl = 0;
          for (int i = 0; i < 4; i++) { st += PT(xO + i); sl += PL(yO + i); }
          if ((xO == 0 && yO == 0) || (xO > 0 && yO > 0)) {
            if (ta && la) v = (st + sl + 4) >> 3;
            else if (la) v = (sl + 2) >> 2;
            else if (ta) v = (st + 2) >> 2;
          } else if (xO > 0 && yO == 0) {
            if (ta) v = (st + 2) >> 2;
            else if (la) v = (sl + 2) >> 2;
          } else {
            if (la) v = (sl + 2) >> 2;
            else if (ta) v = (st + 2) >> 2;
          }
        } else if (mode == 1) v = PL(y);
        else if (mode == 2) v = PT(x);
        else {
          int H = 0, V = 0;
          for (int i = 0; i < 4; i++) {
            H += (i + 1) * (PT(4 + i) - PT(2 - i));
            V += (i + 1) * (PL(4 + i) - PL(2 - i));
          }
          int a = 16 * (PL(7) + PT(7)), bb = (34 * H + 32) >> 6, c = (34 * V + 32) >> 6;
          v = clip1((a + bb * (x - 3) + c * (y - 3) + 16) >> 5);
        }
        pred[y * 8 + x] = v;
      }
  }
#undef PT
#undef PL
}

/* -------------------------------------------- inter prediction (8.4.2.2) */
static int ref_luma(const fo_dec *d, const fo_pic *r, int x, int y) {
  return r->y[(int64_t)clip3(0, d->H - 1, y) * d->W + clip3(0, d->W - 1, x)];
}
static int tap6(int a, int b, int c, int dd, int e, int f) { return a - 5 * b + 20 * c + 20 * dd - 5 * e + f; }

/* luma sample at integer (xi, yi) + fraction (xf, yf) (Table 8-12); only the
 * intermediate values the position needs are formed */
static int luma_sample(const fo_dec *d, const fo_pic *r, int xi, int yi, int xf, int yf) {
#define G(dx, dy) ref_luma(d, r, xi + (dx), yi + (dy))
#define HTAP(dy) tap6(G(-2, dy), G(-1, dy), G(0, dy), G(1, dy), G(2, dy), G(3, dy))
#define VTAP(dx) tap6(G(dx, -2), G(dx, -1), G(dx, 0), G(dx, 1), G(dx, 2), G(dx, 3))
  int Gv = G(0, 0);
  if (!xf && !yf) return Gv;
  int b = 0, h = 0, s = 0, m = 0, j = 0;
  int need_b = (yf == 0 && xf) || (yf == 1 && xf) || (xf == 2);
  int need_h = (xf == 0 && yf) || (xf == 1 && yf) || (yf == 2);
  int need_s = yf == 3 && xf;
  int need_m = xf == 3 && yf;
  int need_j = (xf == 2 && yf) || (yf == 2 && xf);
  if (need_b) b = clip1((HTAP(0) + 16) >> 5);
  if (need_h) h = clip1((VTAP(0) + 16) >> 5);
  if (need_s) s = clip1((HTAP(1) + 16) >> 5);
  if (need_m) m = clip1((VTAP(1) + 16) >> 5);
  if (need_j) j = clip1((tap6(HTAP(-2), HTAP(-1), HTAP(0), HTAP(1), HTAP(2), HTAP(3)) + 512) >> 10);
  int H = xf == 3 && yf == 0 ? G(1, 0) : 0, M = xf == 0 && yf == 3 ? G(0, 1) : 0;
#undef HTAP
#undef VTAP
#undef G
  switch (yf * 4 + xf) {
    case 0 * 4 + 1: return (Gv + b + 1) >> 1;   /* a */
    case 0 * 4 + 2: return b;
    case 0 * 4 + 3: return (H + b + 1) >> 1;    /* c */
    case 1 * 4 + 0: return (Gv + h + 1) >> 1;   /* d */
    case 1 * 4 + 1: return (b + h + 1) >> 1;    /* e */
    case 1 * 4 + 2: return (b + j + 1) >> 1;    /* f */
    case 1 * 4 + 3: return (b + m + 1) >> 1;    /* g */
    case 2 * 4 + 0: return h;
    case 2 * 4 + 1: return (h + j + 1) >> 1;    /* i */
    case 2 * 4 + 2: return j;
    case 2 * 4 + 3: return (j + m + 1) >> 1;    /* k */
    case 3 * 4 + 0: return (M + h + 1) >> 1;    /* n */
    case 3 * 4 + 1: return (h + s + 1) >> 1;    /* p */
    case 3 * 4 + 2: return (j + s + 1) >> 1;    /* q */
    default: return (m + s + 1) >> 1;           /* r */
  }
}

/* predict the w x h luma block at MB-relative (x0, y0) and its chroma */
static void mc_part(const fo_dec *d, const fo_pic *r, int cur, int x0, int y0, int w, int h,
                    int mvx, int mvy, int *py, int *pu, int *pv) {
  int mx = cur % d->mbw, my = cur / d->mbw;
  int xa = mx * 16 + x0, ya = my * 16 + y0;
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++)
      py[(y0 + y) * 16 + x0 + x] =
          luma_sample(d, r, xa + x + (mvx >> 2), ya + y + (mvy >> 2), mvx & 3, mvy & 3);
  int cw = d->W / 2, ch = d->H / 2, xf = mvx & 7, yf = mvy & 7;
  for (int y = 0; y < h / 2; y++)
    for (int x = 0; x < w / 2; x++) {
      int xi = xa / 2 + x + (mvx >> 3), yi = ya / 2 + y + (mvy >> 3);
      int xA = clip3(0, cw - 1, xi), xB = clip3(0, cw - 1, xi + 1);
      int yA = clip3(0, ch - 1, yi), yB = clip3(0, ch - 1, yi + 1);
      for (int pl = 0; pl < 2; pl++) {
        const uint8_t *s = pl ? r->v : r->u;
        int A = s[yA * cw + xA], B = s[yA * cw + xB], C = s[yB * cw + xA], D = s[yB * cw + xB];
        int v = ((8 - xf) * (8 - yf) * A + xf * (8 - yf) * B + (8 - xf) * yf * C + xf * yf * D + 32) >> 6;
        (pl ? pv : pu)[(y0 / 2 + y) * 8 + x0 / 2 + x] = v;
      }
    }
}

/* ---------------------------------------------- MV prediction (8.4.1.3) */
typedef struct {
  int avail;  /* partition available (MB available and already decoded) */
  int ref;    /* -1 when unavailable / intra */
  int mvx, mvy;
} fo_nbmv;

/* neighbour motion data at MB-relative luma location (xN, yN); done_mask =
 * raster 4x4 blocks of the current MB whose motion is already set */
static fo_nbmv nb_mv(const fo_dec *d, int l, int cur, int xN, int yN, int done_mask) {
  fo_nbmv r = {0, -1, 0, 0};
  fo_loc L = nb_loc(d, cur, xN, yN, 16, 16);
  if (L.mb < 0) return r;
  int blk = (L.yw / 4) * 4 + L.xw / 4;
  if (L.mb == cur && !((done_mask >> blk) & 1)) return r;
  r.avail = 1;
  const fo_mb *m = &d->mb[L.mb];
  if (m->type == 1 || m->type == 2 || m->type == 3) return r;
  r.ref = m->refidx[l][blk];
  if (r.ref < 0) return r;   /* predFlagLX 0: refIdxLXN -1, mvLXN 0 */
  r.mvx = m->mv[l][blk][0];
  r.mvy = m->mv[l][blk][1];
  return r;
}

/* mbPart (x0, y0, w, h) in luma samples; shape: 0 generic, 1 16x8, 2 8x16 */
static void mv_pred(const fo_dec *d, int l, int cur, int x0, int y0, int w, int h, int ref, int done_mask,
                    int *px, int *py) {
  fo_nbmv A = nb_mv(d, l, cur, x0 - 1, y0, done_mask);
  fo_nbmv B = nb_mv(d, l, cur, x0, y0 - 1, done_mask);
  fo_nbmv C = nb_mv(d, l, cur, x0 + w, y0 - 1, done_mask);
  if (!C.avail) C = nb_mv(d, l, cur, x0 - 1, y0 - 1, done_mask);
  if (w == 16 && h == 8) {
    if (y0 == 0 && B.ref == ref) { *px = B.mvx; *py = B.mvy; return; }
    if (y0 == 8 && A.ref == ref) { *px = A.mvx; *py = A.mvy; return; }
  } else if (w == 8 && h == 16) {
    if (x0 == 0 && A.ref == ref) { *px = A.mvx; *py = A.mvy; return; }
    if (x0 == 8 && C.ref == ref) { *px = C.mvx; *py = C.mvy; return; }
  }
  if (!B.avail && !C.avail && A.avail) { B = A; C = A; } /* 8.4.1.3.1 */
  int match = (A.ref == ref) + (B.ref == ref) + (C.ref == ref);
  if (match == 1) {
    const fo_nbmv *m = A.ref == ref ? &A : (B.ref == ref ? &B : &C);
    *px = m->mvx;
    *py = m->mvy;
  } else {
    *px = median3(A.mvx, B.mvx, C.mvx);
    *py = median3(A.mvy, B.mvy, C.mvy);
  }
}

/* ---------------------------------------------------- deblocking (8.7) */
static int mb_intra(const fo_mb *m) { return m->type == 1 || m->type == 2 || m->type == 3; }

static int mv_far(const int *a, const int *b) { return iabs(a[0] - b[0]) >= 4 || iabs(a[1] - b[1]) >= 4; }

/* bS for the edge between luma samples p0 (in mb p, raster blk bp) and q0
   (8.7.2.1; reference pictures compared as pictures, not indices, and as the
   set of pictures a bi-predicted block uses) */
static int bs_of(const fo_mb *p, int bp, const fo_mb *q, int bq, int mb_edge) {
  if (mb_intra(p) || mb_intra(q)) return mb_edge ? 4 : 3;
  if (p->nz[bp] || q->nz[bq]) return 2;
  int p0 = p->refpic[0][bp], p1 = p->refpic[1][bp], q0 = q->refpic[0][bq], q1 = q->refpic[1][bq];
  int np = (p0 >= 0) + (p1 >= 0), nq = (q0 >= 0) + (q1 >= 0);
  if (np != nq) return 1;
  if (np == 1) {
    int lp = p0 >= 0 ? 0 : 1, lq = q0 >= 0 ? 0 : 1;
    if ((lp ? p1 : p0) != (lq ? q1 : q0)) return 1;
    return mv_far(p->mv[lp][bp], q->mv[lq][bq]);
  }
  if (!((p0 == q0 && p1 == q1) || (p0 == q1 && p1 == q0))) return 1;
  if (p0 != p1) {
    if (p0 == q0) return mv_far(p->mv[0][bp], q->mv[0][bq]) || mv_far(p->mv[1][bp], q->mv[1][bq]);
    return mv_far(p->mv[0][bp], q->mv[1][bq]) || mv_far(p->mv[1][bp], q->mv[0][bq]);
  }
  return (mv_far(p->mv[0][bp], q->mv[0][bq]) || mv_far(p->mv[1][bp], q->mv[1][bq])) &&
         (mv_far(p->mv[0][bp], q->mv[1][bq]) || mv_far(p->mv[1][bp], q->mv[0][bq]));
}

/* filter one line of samples across an edge; s[k * step] for k = -4..3 (p3..q3) */
static void filter_line(uint8_t *s, int step, int bS, int chroma, int indexA, int alpha, int beta) {
  int p0 = s[-step], p1 = s[-2 * step], q0 = s[0], q1 = s[step];
  if (!(bS > 0 && iabs(p0 - q0) < alpha && iabs(p1 - p0) < beta && iabs(q1 - q0) < beta)) return;
  int p2 = chroma ? 0 : s[-3 * step], q2 = chroma ? 0 : s[2 * step];
  if (bS < 4) {
    int tc0 = TC0[indexA][bS - 1];
    int ap = iabs(p2 - p0), aq = iabs(q2 - q0);
    int tc = chroma ? tc0 + 1 : tc0 + (ap < beta) + (aq < beta);
    int delta = clip3(-tc, tc, (((q0 - p0) << 2) + (p1 - q1) + 4) >> 3);
    s[-step] = (uint8_t)clip1(p0 + delta);
    s[0] = (uint8_t)clip1(q0 - delta);
    if (!chroma) {
      if (ap < beta) s[-2 * step] = (uint8_t)(p1 + clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1));
      if (aq < beta) s[step] = (uint8_t)(q1 + clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1));
    }
  } else {
    if (chroma) {
      s[-step] = (uint8_t)((2 * p1 + p0 + q1 + 2) >> 2);
      s[0] = (uint8_t)((2 * q1 + q0 + p1 + 2) >> 2);
      return;
    }
    int p3 = s[-4 * step], q3 = s[3 * step];
    int ap = iabs(p2 - p0), aq = iabs(q2 - q0);
    int small = iabs(p0 - q0) < ((alpha >> 2) + 2);
    if (ap < beta && small) {
      s[-step] = (uint8_t)((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
      s[-2 * step] = (uint8_t)((p2 + p1 + p0 + q0 + 2) >> 2);
      s[-3 * step] = (uint8_t)((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
    } else {
      s[-step] = (uint8_t)((2 * p1 + p0 + q1 + 2) >> 2);
    }
    if (aq < beta && small) {
      s[0] = (uint8_t)((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
      s[step] = (uint8_t)((p0 + q0 + q1 + q2 + 2) >> 2);
      s[2 * step] = (uint8_t)((2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3);
    } else {
      s[0] = (uint8_t)((2 * q1 + q0 + p1 + 2) >> 2);
    }
  }
}

static void deblock_picture(fo_dec *d, fo_pic *pic) {
  for (int a = 0; a < d->nmb; a++) {
    const fo_mb *q = &d->mb[a];
    const fo_slice_dbk *sd = &d->dbk[q->slice];
    if (sd->idc == 1) continue;
    int mx = a % d->mbw, my = a / d->mbw;
    int left = mx > 0, top = my > 0;
    if (sd->idc == 2) {
      if (left && d->mb[a - 1].slice != q->slice) left = 0;
      if (top && d->mb[a - d->mbw].slice != q->slice) top = 0;
    }
    for (int dir = 0; dir < 2; dir++) {       /* 0: vertical edges, 1: horizontal */
      for (int e = 0; e < 4; e++) {          /* luma edges at 0, 4, 8, 12 */
        if (e == 0 && !(dir ? top : left)) continue;
        int luma_edge = !(q->t8 && (e & 1)); /* 8.7: 8x8 transform: no 4-sample internal luma edges */
        const fo_mb *p = e == 0 ? &d->mb[dir ? a - d->mbw : a - 1] : q;
        int qpp = p->type == 3 ? 0 : p->qp, qpq = q->type == 3 ? 0 : q->qp;
        /* luma */
        if (luma_edge) {
          int qpav = (qpp + qpq + 1) >> 1;
          int iA = clip3(0, 51, qpav + sd->off_a), iB = clip3(0, 51, qpav + sd->off_b);
          for (int k = 0; k < 16; k++) {
            int xq = dir ? k : 4 * e, yq = dir ? 4 * e : k;
            int xp = dir ? xq : (xq + 15) % 16, yp = dir ? (yq + 15) % 16 : yq;
            int bS = bs_of(p, (yp / 4) * 4 + xp / 4, q, (yq / 4) * 4 + xq / 4, e == 0);
            uint8_t *s = pic->y + (int64_t)(my * 16 + yq) * d->W + mx * 16 + xq;
            filter_line(s, dir ? d->W : 1, bS, 0, iA, ALPHA[iA], BETA[iB]);
          }
        }
        /* chroma: edges 0 and 2 (chroma sample 0 and 4) */
        if (e == 0 || e == 2) {
          for (int pl = 0; pl < 2; pl++) {
            int off = pl ? d->P->cqp_off2 : d->P->cqp_off;
            int qpav = (qpc_of(qpp, off) + qpc_of(qpq, off) + 1) >> 1;
            int iA = clip3(0, 51, qpav + sd->off_a), iB = clip3(0, 51, qpav + sd->off_b);
            uint8_t *img = pl ? pic->v : pic->u;
            for (int k = 0; k < 8; k++) {
              /* bS of the corresponding luma sample (chroma k <-> luma 2k) */
              int xq = dir ? 2 * k : 4 * e, yq = dir ? 4 * e : 2 * k;
              int xp = dir ? xq : (xq + 15) % 16, yp = dir ? (yq + 15) % 16 : yq;
              int bS = bs_of(p, (yp / 4) * 4 + xp / 4, q, (yq / 4) * 4 + xq / 4, e == 0);
              int cx = dir ? k : 2 * e, cy = dir ? 2 * e : k;
              uint8_t *s = img + (int64_t)(my * 8 + cy) * (d->W / 2) + mx * 8 + cx;
              filter_line(s, dir ? d->W / 2 : 1, bS, 1, iA, ALPHA[iA], BETA[iB]);
            }
          }
        }
      }
    }
  }
}

/* -------------------------------------------------- reference marking */
static int fo_max_frame_num(const fo_dec *d) { return 1 << d->S->log2_max_frame_num; }

static fo_pic *dpb_find_short(fo_dec *d, int pic_num, int cur_fn) {
  for (int i = 0; i < d->ndpb; i++) {
    fo_pic *p = &d->dpb[i];
    if (p->ref != 1) continue;
    int wrap = p->frame_num > cur_fn ? p->frame_num - fo_max_frame_num(d) : p->frame_num;
    if (wrap == pic_num) return p;
  }
  return NULL;
}
static fo_pic *dpb_find_long(fo_dec *d, int lt_num) {
  for (int i = 0; i < d->ndpb; i++)
    if (d->dpb[i].ref == 2 && d->dpb[i].lt_idx == lt_num) return &d->dpb[i];
  return NULL;
}
static void dpb_compact(fo_dec *d) {
  int j = 0;
  for (int i = 0; i < d->ndpb; i++) {
    if (d->dpb[i].ref) d->dpb[j++] = d->dpb[i];
    else pic_free(&d->dpb[i]);
  }
  d->ndpb = j;
}

typedef struct {
  int nal_type, nal_ref_idc;
  int first_mb, slice_type, pps_id, frame_num, idr_pic_id;
  int poc_lsb, delta_bottom, delta_poc[2];
  int direct_spatial;   /* direct_spatial_mv_pred_flag (B) */
  int num_ref, num_ref1;
  int mod_n, mod_idc[33], mod_val[33];      /* ref_pic_list_modification l0 */
  int mod1_n, mod1_idc[33], mod1_val[33];   /* ... l1 */
  /* pred_weight_table (7.3.3.2): [list][refIdx] luma weight / offset, chroma [Cb, Cr] */
  int lwd, cwd, lw[2][32], lo[2][32], cw[2][32][2], co[2][32][2];
  int lt_ref_flag, adaptive, mmco_n, mmco[66][3];
  int qp, dbk_idc, off_a, off_b;
} fo_hdr;

/* ------------------------------------------------- slice decoding */
typedef struct {
  fo_dec *d;
  fo_pic *cur;
  fo_pic *list[33];     /* RefPicList0 */
  int nlist;
  fo_pic *list1[33];    /* RefPicList1 (B) */
  int nlist1;
  int slice_no;
  int is_b;
  int wmode;            /* 8.4.2.3: 0 default, 1 explicit, 2 implicit weighted prediction */
  const fo_hdr *h;
} fo_ctx;

static int decode_mb(fo_ctx *c, fb_t *b, int addr, int is_p, int *qp, const fo_hdr *h);
static void inter_pred_mb(const fo_ctx *c, int addr, int *py, int *pu, int *pv);

/* 8.5.9: the position class of (i, j) that selects v8x8's column */
static int norm8_class(int i, int j) {
  if (i % 4 == 0 && j % 4 == 0) return 0;
  if (i % 2 == 1 && j % 2 == 1) return 1;
  if (i % 4 == 2 && j % 4 == 2) return 2;
  if ((i % 4 == 0 && j % 2 == 1) || (i % 2 == 1 && j % 4 == 0)) return 3;
  if ((i % 4 == 0 && j % 4 == 2) || (i % 4 == 2 && j % 4 == 0)) return 4;
  return 5;
}

/* 8.5.13: scaling + 8x8 inverse transform of raster coefficients c; w8 =
 * weightScale8x8 (raster), LevelScale8x8 = w8 * normAdjust8x8 (8.5.9) */
static void scale_idct8(const int *c, int qp, const uint8_t *w8, int *r) {
  int d[64], g[64];
  for (int i = 0; i < 8; i++)
    for (int j = 0; j < 8; j++) {
      int ls = w8[i * 8 + j] * FO_V8[qp % 6][norm8_class(i, j)];
      int k = i * 8 + j;
      d[k] = qp >= 36 ? (c[k] * ls) << (qp / 6 - 6) : (c[k] * ls + (1 << (5 - qp / 6))) >> (6 - qp / 6);
    }
  for (int pass = 0; pass < 2; pass++) {
    for (int u = 0; u < 8; u++) {
      int v[8], o[8];
      for (int k = 0; k < 8; k++) v[k] = pass == 0 ? d[u * 8 + k] : g[k * 8 + u];
      int a0 = v[0] + v[4], a4 = v[0] - v[4], a2 = (v[2] >> 1) - v[6], a6 = v[2] + (v[6] >> 1);
      int b0 = a0 + a6, b2 = a4 + a2, b4 = a4 - a2, b6 = a0 - a6;
      int a1 = -v[3] + v[5] - v[7] - (v[7] >> 1), a3 = v[1] + v[7] - v[3] - (v[3] >> 1);
      int a5 = -v[1] + v[7] + v[5] + (v[5] >> 1), a7 = v[3] + v[5] + v[1] + (v[1] >> 1);
      int b1 = a1 + (a7 >> 2), b7 = a7 - (a1 >> 2), b3 = a3 + (a5 >> 2), b5 = (a3 >> 2) - a5;
      o[0] = b0 + b7; o[1] = b2 + b5; o[2] = b4 + b3; o[3] = b6 + b1;
      o[4] = b6 - b1; o[5] = b4 - b3; o[6] = b2 - b5; o[7] = b0 - b7;
      for (int k = 0; k < 8; k++) {
        if (pass == 0) g[u * 8 + k] = o[k];
        else r[k * 8 + u] = (o[k] + 32) >> 6;
      }
    }
  }
}

/* 8.3.2: Intra_8x8 prediction of 8x8 block b8 (raster 0..3) with the
 * reference sample filtering of 8.3.2.2.1 */
static void intra8x8(const fo_dec *d, fo_pic *pic, int cur, int b8, int mode, int done_mask, int pred[64]) {
  int xo = (b8 & 1) * 8, yo = (b8 >> 1) * 8;
  int P_[25], av[25]; /* index 0 = p[-1,-1], 1..16 = p[0..15,-1], 17..24 = p[-1,0..7] */
  fo_s s = luma_nb(d, pic, cur, xo, yo, -1, -1, done_mask);
  av[0] = s.avail; P_[0] = s.v;
  for (int x = 0; x < 16; x++) { s = luma_nb(d, pic, cur, xo, yo, x, -1, done_mask); av[1 + x] = s.avail; P_[1 + x] = s.v; }
  for (int y = 0; y < 8; y++) { s = luma_nb(d, pic, cur, xo, yo, -1, y, done_mask); av[17 + y] = s.avail; P_[17 + y] = s.v; }
  if (!av[9] && av[8]) for (int x = 8; x < 16; x++) { P_[1 + x] = P_[8]; av[1 + x] = 1; }
  int top = av[1], left = av[17], tl = av[0];
  /* filtered samples pt[-1..15] (pt[0] = p'[-1,-1]) and pl[0..7] */
  int T[17] = {0}, L[8] = {0};
  if (top) {
    T[1] = tl ? (P_[0] + 2 * P_[1] + P_[2] + 2) >> 2 : (3 * P_[1] + P_[2] + 2) >> 2;
    for (int x = 1; x < 15; x++) T[1 + x] = (P_[x] + 2 * P_[1 + x] + P_[2 + x] + 2) >> 2;
    T[16] = (P_[15] + 3 * P_[16] + 2) >> 2;
  }
  if (tl) {
    if (top && left) T[0] = (P_[1] + 2 * P_[0] + P_[17] + 2) >> 2;
    else if (top) T[0] = (3 * P_[0] + P_[1] + 2) >> 2;
    else if (left) T[0] = (3 * P_[0] + P_[17] + 2) >> 2;
    else T[0] = P_[0];
  }
  if (left) {
    L[0] = tl ? (P_[0] + 2 * P_[17] + P_[18] + 2) >> 2 : (3 * P_[17] + P_[18] + 2) >> 2;
    for (int y = 1; y < 7; y++) L[y] = (P_[16 + y] + 2 * P_[17 + y] + P_[18 + y] + 2) >> 2;
    L[7] = (P_[23] + 3 * P_[24] + 2) >> 2;
  }
#define PT(x) T[1 + (x)]
#define PL(y) ((y) < 0 ? T[0] : L[(y)])
  for (int y = 0; y < 8; y++)
    for (int x = 0; x < 8; x++) {
      int v = 128;
      switch (mode) {
        case 0: v = PT(x); break;
        case 1: v = PL(y); break;
        case 2: {
          int st = 0, sl = 0;
          for (int i = 0; i < 8; i++) { st += top ? PT(i) : 0; sl += left ? L[i] : 0; }
          if (top && left) v = (st + sl + 8) >> 4;
          else if (left) v = (sl + 4) >> 3;
          else if (top) v = (st + 4) >> 3;
          break;
        }
        case 3:
          if (x == 7 && y == 7) v = (PT(14) + 3 * PT(15) + 2) >> 2;
          else v = (PT(x + y) + 2 * PT(x + y + 1) + PT(x + y + 2) + 2) >> 2;
          break;
        case 4:
          if (x > y) v = (PT(x - y - 2) + 2 * PT(x - y - 1) + PT(x - y) + 2) >> 2;
          else if (x < y) v = (PL(y - x - 2) + 2 * PL(y - x - 1) + PL(y - x) + 2) >> 2;
          else v = (PT(0) + 2 * PT(-1) + PL(0) + 2) >> 2;
          break;
        case 5: {
          int z = 2 * x - y;
          if (z >= 0 && !(z & 1)) v = (PT(x - (y >> 1) - 1) + PT(x - (y >> 1)) + 1) >> 1;
          else if (z >= 0) v = (PT(x - (y >> 1) - 2) + 2 * PT(x - (y >> 1) - 1) + PT(x - (y >> 1)) + 2) >> 2;
          else if (z == -1) v = (PL(0) + 2 * PL(-1) + PT(0) + 2) >> 2;
          else v = (PL(y - 2 * x - 1) + 2 * PL(y - 2 * x - 2) + PL(y - 2 * x - 3) + 2) >> 2;
          break;
        }
        case 6: {
          int z = 2 * y - x;
          if (z >= 0 && !(z & 1)) v = (PL(y - (x >> 1) - 1) + PL(y - (x >> 1)) + 1) >> 1;
          else if (z >= 0) v = (PL(y - (x >> 1) - 2) + 2 * PL(y - (x >> 1) - 1) + PL(y - (x >> 1)) + 2) >> 2;
          else if (z == -1) v = (PL(0) + 2 * PL(-1) + PT(0) + 2) >> 2;
          else v = (PT(x - 2 * y - 1) + 2 * PT(x - 2 * y - 2) + PT(x - 2 * y - 3) + 2) >> 2;
          break;
        }
        case 7:
          if (!(y & 1)) v = (PT(x + (y >> 1)) + PT(x + (y >> 1) + 1) + 1) >> 1;
          else v = (PT(x + (y >> 1)) + 2 * PT(x + (y >> 1) + 1) + PT(x + (y >> 1) + 2) + 2) >> 2;
          break;
        default: {
          int z = x + 2 * y;
          if (z < 13 && !(z & 1)) v = (PL(y + (x >> 1)) + PL(y + (x >> 1) + 1) + 1) >> 1;
          else if (z < 13) v = (PL(y + (x >> 1)) + 2 * PL(y + (x >> 1) + 1) + PL(y + (x >> 1) + 2) + 2) >> 2;
          else if (z == 13) v = (PL(6) + 3 * PL(7) + 2) >> 2;
          else v = PL(7);
          break;
        }
      }
      pred[y * 8 + x] = v;
    }
#undef PT
#undef PL
}

/* reconstruction of a parsed (non-skip, non-PCM) macroblock: prediction +
 * residual (8.3, 8.4, 8.5); coef8 != NULL holds the 8x8 blocks when
 * transform_size_8x8_flag is set */
static int recon_mb(fo_ctx *c, int addr, int (*coef)[16], const int *dcl, int (*cdc)[4], int (*cac)[4][16],
                    int (*coef8)[64], int i16mode, int cmode) {
  fo_dec *d = c->d;
  fo_mb *m = &d->mb[addr];
  fo_pic *pic = c->cur;
  int mx = addr % d->mbw, my = addr / d->mbw;
  int pred_y[256], pred_u[64], pred_v[64];
  int qpy = m->qp;
  uint8_t *Y = pic->y + (int64_t)(my * 16) * d->W + mx * 16;
  if (m->type == 0) {
    /* predict each 4x4 block with its motion (partitions share them;
       interpolation is per sample, so the block size does not matter) */
    inter_pred_mb(c, addr, pred_y, pred_u, pred_v);
    if (m->t8) {
      for (int b8 = 0; b8 < 4; b8++) {
        int r[64], bx = (b8 & 1) * 8, by = (b8 >> 1) * 8;
        scale_idct8(coef8[b8], qpy, d->P->w8[1], r);
        for (int y = 0; y < 8; y++)
          for (int x = 0; x < 8; x++)
            Y[(int64_t)(by + y) * d->W + bx + x] = (uint8_t)clip1(pred_y[(by + y) * 16 + bx + x] + r[y * 8 + x]);
      }
    } else {
      for (int blk = 0; blk < 16; blk++) {
        int r[16], bx = blk % 4, by = blk / 4;
        scale_idct4(coef[blk], qpy, d->P->w4[3], 0, r);
        for (int y = 0; y < 4; y++)
          for (int x = 0; x < 4; x++)
            Y[(int64_t)(by * 4 + y) * d->W + bx * 4 + x] = (uint8_t)clip1(pred_y[(by * 4 + y) * 16 + bx * 4 + x] + r[y * 4 + x]);
      }
    }
  } else if (m->type == 1 && m->t8) {
    int done = 0;
    for (int b8 = 0; b8 < 4; b8++) {
      int bx = (b8 & 1) * 8, by = (b8 >> 1) * 8, pred[64], r[64];
      intra8x8(d, pic, addr, b8, m->i4[(by / 4) * 4 + bx / 4], done, pred);
      scale_idct8(coef8[b8], qpy, d->P->w8[0], r);
      for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) Y[(int64_t)(by + y) * d->W + bx + x] = (uint8_t)clip1(pred[y * 8 + x] + r[y * 8 + x]);
      int r4 = (by / 4) * 4 + bx / 4;
      done |= (1 << r4) | (1 << (r4 + 1)) | (1 << (r4 + 4)) | (1 << (r4 + 5));
    }
  } else if (m->type == 1) {
    int done = 0;
    for (int k = 0; k < 16; k++) {
      int bx = BLK_X[k], by = BLK_Y[k], blk = by * 4 + bx, pred[16], r[16];
      intra4x4(d, pic, addr, k, m->i4[blk], done, pred);
      scale_idct4(coef[blk], qpy, d->P->w4[0], 0, r);
      for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++)
          Y[(int64_t)(by * 4 + y) * d->W + bx * 4 + x] = (uint8_t)clip1(pred[y * 4 + x] + r[y * 4 + x]);
      done |= 1 << blk;
    }
  } else {
    intra_big(d, pic, addr, 0, i16mode, pred_y);
    /* 8.5.10: Intra16x16 DC Hadamard + scaling */
    int f[16], t[16];
    for (int i = 0; i < 4; i++) {
      int a0 = dcl[i * 4 + 0], a1 = dcl[i * 4 + 1], a2 = dcl[i * 4 + 2], a3 = dcl[i * 4 + 3];
      t[i * 4 + 0] = a0 + a1 + a2 + a3;
      t[i * 4 + 1] = a0 + a1 - a2 - a3;
      t[i * 4 + 2] = a0 - a1 - a2 + a3;
      t[i * 4 + 3] = a0 - a1 + a2 - a3;
    }
    for (int j = 0; j < 4; j++) {
      int a0 = t[0 * 4 + j], a1 = t[1 * 4 + j], a2 = t[2 * 4 + j], a3 = t[3 * 4 + j];
      f[0 * 4 + j] = a0 + a1 + a2 + a3;
      f[1 * 4 + j] = a0 + a1 - a2 - a3;
      f[2 * 4 + j] = a0 - a1 - a2 + a3;
      f[3 * 4 + j] = a0 - a1 + a2 - a3;
    }
    int ls = level_scale(d->P->w4[0], qpy % 6, 0, 0);
    for (int k = 0; k < 16; k++) {
      int dc = qpy >= 36 ? (f[k] * ls) << (qpy / 6 - 6) : (f[k] * ls + (1 << (5 - qpy / 6))) >> (6 - qpy / 6);
      coef[k][0] = dc; /* dcY row i col j -> block (x = j, y = i) */
    }
    for (int blk = 0; blk < 16; blk++) {
      int r[16], bx = blk % 4, by = blk / 4;
      scale_idct4(coef[blk], qpy, d->P->w4[0], 1, r);
      for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++)
          Y[(int64_t)(by * 4 + y) * d->W + bx * 4 + x] = (uint8_t)clip1(pred_y[(by * 4 + y) * 16 + bx * 4 + x] + r[y * 4 + x]);
    }
  }
  /* chroma */
  if (m->type != 0) {
    intra_big(d, pic, addr, 1, cmode, pred_u);
    intra_big(d, pic, addr, 2, cmode, pred_v);
  }
  for (int pl = 0; pl < 2; pl++) {
    int qpc = qpc_of(qpy, pl ? d->P->cqp_off2 : d->P->cqp_off);
    int c0 = cdc[pl][0], c1 = cdc[pl][1], c2 = cdc[pl][2], c3 = cdc[pl][3];
    int f[4] = {c0 + c1 + c2 + c3, c0 - c1 + c2 - c3, c0 + c1 - c2 - c3, c0 - c1 - c2 + c3};
    const uint8_t *wc = d->P->w4[(m->type == 0 ? 3 : 0) + 1 + pl]; /* Cb / Cr, intra or inter */
    int ls = level_scale(wc, qpc % 6, 0, 0);
    uint8_t *U = (pl ? pic->v : pic->u) + (int64_t)(my * 8) * (d->W / 2) + mx * 8;
    int *pr = pl ? pred_v : pred_u;
    for (int k = 0; k < 4; k++) {
      int bx = k & 1, by = k >> 1, r[16];
      cac[pl][k][0] = ((f[k] * ls) << (qpc / 6)) >> 5;
      scale_idct4(cac[pl][k], qpc, wc, 1, r);
      for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++)
          U[(int64_t)(by * 4 + y) * (d->W / 2) + bx * 4 + x] = (uint8_t)clip1(pr[(by * 4 + y) * 8 + bx * 4 + x] + r[y * 4 + x]);
    }
  }
  return 0;
}


/* 8.2.1 PicOrderCnt of the picture a slice header belongs to (frames only);
   the "previous picture" state is advanced by poc_advance() after it */
static int pic_order_cnt(const fo_dec *d, const fo_hdr *h) {
  const fo_sps *S = d->S;
  int idr = h->nal_type == 5, maxfn = fo_max_frame_num(d);
  if (S->poc_type == 0) { /* 8.2.1.1 */
    int max_lsb = 1 << S->log2_max_poc_lsb, pmsb = idr ? 0 : d->prev_poc_msb, plsb = idr ? 0 : d->prev_poc_lsb;
    int msb;
    if (h->poc_lsb < plsb && plsb - h->poc_lsb >= max_lsb / 2) msb = pmsb + max_lsb;
    else if (h->poc_lsb > plsb && h->poc_lsb - plsb > max_lsb / 2) msb = pmsb - max_lsb;
    else msb = pmsb;
    int top = msb + h->poc_lsb, bot = top + h->delta_bottom;
    return top < bot ? top : bot;
  }
  int off = idr ? 0 : (d->prev_fn > h->frame_num ? d->prev_fn_offset + maxfn : d->prev_fn_offset);
  if (S->poc_type == 2) { /* 8.2.1.3 */
    if (idr) return 0;
    return h->nal_ref_idc ? 2 * (off + h->frame_num) : 2 * (off + h->frame_num) - 1;
  }
  /* 8.2.1.2 */
  int abs_fn = S->ncycle ? off + h->frame_num : 0;
  if (!h->nal_ref_idc && abs_fn > 0) abs_fn--;
  int expected = 0;
  if (abs_fn > 0) {
    int delta_cycle = 0;
    for (int i = 0; i < S->ncycle; i++) delta_cycle += S->off_ref[i];
    int cyc = (abs_fn - 1) / S->ncycle, in = (abs_fn - 1) % S->ncycle;
    expected = cyc * delta_cycle;
    for (int i = 0; i <= in; i++) expected += S->off_ref[i];
  }
  if (!h->nal_ref_idc) expected += S->off_non_ref;
  int top = expected + h->delta_poc[0], bot = top + S->off_t2b + h->delta_poc[1];
  return top < bot ? top : bot;
}

/* after a picture: the state 8.2.1 keeps for the next one */
static void poc_advance(fo_dec *d, const fo_hdr *h) {
  int idr = h->nal_type == 5, mmco5 = 0, maxfn = fo_max_frame_num(d);
  for (int k = 0; h->adaptive && k < h->mmco_n; k++) mmco5 |= h->mmco[k][0] == 5;
  if (d->S->poc_type == 0) {
    if (h->nal_ref_idc) {
      if (mmco5) { d->prev_poc_msb = 0; d->prev_poc_lsb = h->delta_bottom < 0 ? -h->delta_bottom : 0; }
      else {
        int max_lsb = 1 << d->S->log2_max_poc_lsb;
        int pmsb = idr ? 0 : d->prev_poc_msb, plsb = idr ? 0 : d->prev_poc_lsb, msb;
        if (h->poc_lsb < plsb && plsb - h->poc_lsb >= max_lsb / 2) msb = pmsb + max_lsb;
        else if (h->poc_lsb > plsb && h->poc_lsb - plsb > max_lsb / 2) msb = pmsb - max_lsb;
        else msb = pmsb;
        d->prev_poc_msb = msb;
        d->prev_poc_lsb = h->poc_lsb;
      }
    }
  } else {
    int off = idr ? 0 : (d->prev_fn > h->frame_num ? d->prev_fn_offset + maxfn : d->prev_fn_offset);
    d->prev_fn_offset = mmco5 ? 0 : off;
  }
  d->prev_fn = mmco5 ? 0 : h->frame_num;
  d->prev_mmco5 = mmco5;
}

static int slice_data_cabac(fo_ctx *c, fb_t *b, const fo_hdr *h, int is_p, int64_t stop);

static int decode_slice(fo_dec *d, fo_pic *cur, const uint8_t *nal, int64_t len, int slice_no,
                        int *is_idr_out, fo_hdr *hdr_out) {
  int nal_type = nal[0] & 31, nal_ref_idc = (nal[0] >> 5) & 3;
  int64_t last = len - 1;
  /* trailing cabac_zero_words (0x0000, escaped as 00 00 03) are not RBSP data */
  while (last > 0 && (nal[last] == 0 || (nal[last] == 3 && last >= 2 && nal[last - 1] == 0 && nal[last - 2] == 0)))
    last--;
  if (last <= 0) return fo_fail(d, FO_E_FORMAT, "empty slice NAL");
  int tz = 0;
  while (!((nal[last] >> tz) & 1)) tz++;
  fb_t b;
  fb_init(&b, nal + 1, len - 1);
  /* the stop bit, in the reader's EBSP coordinates (no emulation prevention
     byte can precede a stop byte whose top bit is the stop bit) */
  int64_t stop = (last - 1) * 8 + (7 - tz);
  fo_hdr h;
  memset(&h, 0, sizeof h);
  h.nal_type = nal_type;
  h.nal_ref_idc = nal_ref_idc;
  h.first_mb = (int)fb_ue(&b); /* 7.3.3 */
  h.slice_type = (int)fb_ue(&b) % 5;
  h.pps_id = (int)fb_ue(&b);
  if (h.pps_id > 255 || !d->pps[h.pps_id].valid) return fo_fail(d, FO_E_FORMAT, "unknown PPS");
  const fo_pps *P = &d->pps[h.pps_id];
  if (!d->sps[P->sps_id].valid) return fo_fail(d, FO_E_FORMAT, "unknown SPS");
  const fo_sps *S = &d->sps[P->sps_id];
  if (S->mbw != d->mbw || S->mbh != d->mbh)
    return fo_fail(d, FO_E_UNSUPPORTED, "picture size change");
  d->S = S;
  d->P = P;
  if (h.slice_type > 2) return fo_fail(d, FO_E_UNSUPPORTED, "SP/SI slice");
  int is_b = h.slice_type == 1;
  int is_p = h.slice_type == 0 || is_b;   /* inter slice (P or B) */
  h.frame_num = (int)fb_bits(&b, S->log2_max_frame_num);
  if (nal_type == 5) h.idr_pic_id = (int)fb_ue(&b);
  if (S->poc_type == 0) {
    h.poc_lsb = (int)fb_bits(&b, S->log2_max_poc_lsb);
    if (P->bfpo) h.delta_bottom = fb_se(&b);
  } else if (S->poc_type == 1 && !S->dpoaz) {
    h.delta_poc[0] = fb_se(&b);
    if (P->bfpo) h.delta_poc[1] = fb_se(&b);
  }
  if (is_b) h.direct_spatial = (int)fb_bit(&b);
  h.num_ref = P->num_ref_l0;
  h.num_ref1 = P->num_ref_l1;
  if (is_p) {
    if (fb_bit(&b)) { /* num_ref_idx_active_override_flag */
      h.num_ref = (int)fb_ue(&b) + 1;
      if (is_b) h.num_ref1 = (int)fb_ue(&b) + 1;
    }
    if (h.num_ref > 32 || h.num_ref1 > 32) return fo_fail(d, FO_E_FORMAT, "num_ref_idx");
    for (int l = 0; l < 1 + is_b; l++) {
      int *n = l ? &h.mod1_n : &h.mod_n, *idcs = l ? h.mod1_idc : h.mod_idc, *vals = l ? h.mod1_val : h.mod_val;
      if (fb_bit(&b)) { /* ref_pic_list_modification (7.3.3.1) */
        for (;;) {
          int idc = (int)fb_ue(&b);
          if (idc == 3 || b.err) break;
          if (idc > 2 || *n >= 33) return fo_fail(d, FO_E_FORMAT, "ref list modification");
          idcs[*n] = idc;
          vals[(*n)++] = (int)fb_ue(&b);
        }
      }
    }
  }
  if ((P->weighted_pred && is_p && !is_b) || (P->weighted_bipred == 1 && is_b)) { /* 7.3.3.2 */
    h.lwd = (int)fb_ue(&b);
    h.cwd = (int)fb_ue(&b);
    if (h.lwd > 7 || h.cwd > 7) return fo_fail(d, FO_E_FORMAT, "pred_weight_table denominators");
    for (int l = 0; l < 1 + is_b; l++)
      for (int i = 0; i < (l ? h.num_ref1 : h.num_ref); i++) {
        h.lw[l][i] = 1 << h.lwd;
        h.lo[l][i] = 0;
        if (fb_bit(&b)) {
          h.lw[l][i] = fb_se(&b);
          h.lo[l][i] = fb_se(&b);
        }
        for (int j = 0; j < 2; j++) { h.cw[l][i][j] = 1 << h.cwd; h.co[l][i][j] = 0; }
        if (fb_bit(&b))
          for (int j = 0; j < 2; j++) {
            h.cw[l][i][j] = fb_se(&b);
            h.co[l][i][j] = fb_se(&b);
          }
        if (h.lw[l][i] < -128 || h.lw[l][i] > 127 || h.lo[l][i] < -128 || h.lo[l][i] > 127)
          return fo_fail(d, FO_E_FORMAT, "pred_weight_table");
      }
  }
  if (nal_ref_idc) { /* dec_ref_pic_marking (7.3.3.3) */
    if (nal_type == 5) {
      fb_bit(&b);
      h.lt_ref_flag = (int)fb_bit(&b);
    } else if ((h.adaptive = (int)fb_bit(&b))) {
      for (;;) {
        int op = (int)fb_ue(&b);
        if (op == 0 || b.err) break;
        if (op > 6 || h.mmco_n >= 66) return fo_fail(d, FO_E_FORMAT, "MMCO");
        int *m = h.mmco[h.mmco_n++];
        m[0] = op;
        m[1] = m[2] = 0;
        if (op == 1 || op == 3) m[1] = (int)fb_ue(&b);
        if (op == 2) m[1] = (int)fb_ue(&b);
        if (op == 3 || op == 6) m[2] = (int)fb_ue(&b);
        if (op == 4) m[1] = (int)fb_ue(&b);
      }
    }
  }
  if (g_enc) d->enc_pos_qp = fb_index(&b, 0);
  if (P->cabac && is_p && !g_enc) {
    int idc = (int)fb_ue(&b);
    if (idc != 0) return fo_fail(d, FO_E_UNSUPPORTED, "cabac_init_idc 1/2 (only the idc 0 tables are restated)");
  }
  h.qp = P->pic_init_qp + fb_se(&b);
  if (P->deblock_ctrl) {
    h.dbk_idc = (int)fb_ue(&b);
    if (h.dbk_idc != 1) {
      h.off_a = 2 * fb_se(&b);
      h.off_b = 2 * fb_se(&b);
    }
  }
  if (b.err || h.first_mb >= d->nmb || h.qp < 0 || h.qp > 51 || h.dbk_idc > 2)
    return fo_fail(d, FO_E_FORMAT, "slice header");
  if (is_b && !S->direct8x8 && 0) return fo_fail(d, FO_E_UNSUPPORTED, "direct_8x8_inference_flag 0");
  *is_idr_out = nal_type == 5;
  *hdr_out = h;
  if (slice_no >= 4096) return fo_fail(d, FO_E_UNSUPPORTED, "too many slices");
  d->dbk[slice_no].idc = h.dbk_idc;
  d->dbk[slice_no].off_a = h.off_a;
  d->dbk[slice_no].off_b = h.off_b;
  cur->poc = pic_order_cnt(d, &h);

  fo_ctx c;
  memset(&c, 0, sizeof c);
  c.d = d;
  c.cur = cur;
  c.slice_no = slice_no;
  c.is_b = is_b;
  c.h = hdr_out;
  c.wmode = is_b ? (P->weighted_bipred == 1 ? 1 : (P->weighted_bipred == 2 ? 2 : 0)) : (is_p && P->weighted_pred ? 1 : 0);
  if (is_p) {
    int fn = h.frame_num, maxfn = fo_max_frame_num(d);
    fo_pic *st[17], *lt[17];
    int ns = 0, nl = 0;
    for (int i = 0; i < d->ndpb; i++) {
      fo_pic *p = &d->dpb[i];
      if (p->ref == 1) {
        p->frame_num_wrap = p->frame_num > fn ? p->frame_num - maxfn : p->frame_num;
        st[ns++] = p;
      } else if (p->ref == 2) {
        lt[nl++] = p;
      }
    }
    /* long-term: ascending LongTermPicNum (8.2.4.2.1 / 8.2.4.2.3) */
    for (int i = 1; i < nl; i++)
      for (int j = i; j > 0 && lt[j]->lt_idx < lt[j - 1]->lt_idx; j--) {
        fo_pic *t = lt[j]; lt[j] = lt[j - 1]; lt[j - 1] = t;
      }
    fo_pic *init[2][34];
    int ni[2] = {0, 0};
    if (!is_b) {
      /* 8.2.4.2.1: short-term by descending PicNum, then long-term */
      for (int i = 1; i < ns; i++)
        for (int j = i; j > 0 && st[j]->frame_num_wrap > st[j - 1]->frame_num_wrap; j--) {
          fo_pic *t = st[j]; st[j] = st[j - 1]; st[j - 1] = t;
        }
      for (int i = 0; i < ns; i++) init[0][ni[0]++] = st[i];
    } else {
      /* 8.2.4.2.3: list 0 = POC below the current picture's descending, then
         above ascending; list 1 the other way round; long-term after both */
      for (int i = 1; i < ns; i++)
        for (int j = i; j > 0 && st[j]->poc < st[j - 1]->poc; j--) {
          fo_pic *t = st[j]; st[j] = st[j - 1]; st[j - 1] = t;
        }
      for (int i = ns - 1; i >= 0; i--) if (st[i]->poc < cur->poc) init[0][ni[0]++] = st[i];
      for (int i = 0; i < ns; i++) if (st[i]->poc > cur->poc) init[0][ni[0]++] = st[i];
      for (int i = 0; i < ns; i++) if (st[i]->poc > cur->poc) init[1][ni[1]++] = st[i];
      for (int i = ns - 1; i >= 0; i--) if (st[i]->poc < cur->poc) init[1][ni[1]++] = st[i];
    }
    for (int l = 0; l < 1 + is_b; l++)
      for (int i = 0; i < nl; i++) init[l][ni[l]++] = lt[i];
    if (is_b && ni[1] > 1 && ni[0] == ni[1]) {
      int same = 1;
      for (int i = 0; i < ni[0]; i++) same &= init[0][i] == init[1][i];
      if (same) { fo_pic *t = init[1][0]; init[1][0] = init[1][1]; init[1][1] = t; }
    }
    for (int l = 0; l < 1 + is_b; l++) {
      fo_pic **list = l ? c.list1 : c.list;
      int n = l ? h.num_ref1 : h.num_ref;
      for (int i = 0; i < 33; i++) list[i] = i < ni[l] && i < n ? init[l][i] : NULL;
      /* 8.2.4.3 modification */
      int pred = fn, ridx = 0;
      int mn = l ? h.mod1_n : h.mod_n;
      const int *idcs = l ? h.mod1_idc : h.mod_idc, *vals = l ? h.mod1_val : h.mod_val;
      for (int k = 0; k < mn; k++) {
        fo_pic *pic = NULL;
        int is_long = idcs[k] == 2, num = 0;
        if (!is_long) {
          int abs_diff = vals[k] + 1, nowrap;
          if (idcs[k] == 0) nowrap = pred - abs_diff < 0 ? pred - abs_diff + maxfn : pred - abs_diff;
          else nowrap = pred + abs_diff >= maxfn ? pred + abs_diff - maxfn : pred + abs_diff;
          pred = nowrap;
          num = nowrap > fn ? nowrap - maxfn : nowrap;
          pic = dpb_find_short(d, num, fn);
        } else {
          num = vals[k];
          pic = dpb_find_long(d, num);
        }
        if (!pic) return fo_fail(d, FO_E_DECODE, "modification names no reference picture");
        for (int ci = n; ci > ridx; ci--) list[ci] = list[ci - 1];
        list[ridx++] = pic;
        int ni2 = ridx;
        for (int ci = ridx; ci <= n; ci++) {
          fo_pic *q = list[ci];
          if (q != pic) list[ni2++] = q;
        }
      }
      list[n] = NULL;
      if (l) c.nlist1 = n;
      else c.nlist = n;
    }
  }
  if (is_b && (!c.list1[0] || !c.list1[0]->mref[0]))
    return fo_fail(d, FO_E_DECODE, "B slice without a colocated picture (RefPicList1[0])");

  if (g_enc) d->enc_pos_data = fb_index(&b, 0);
  if (P->cabac) return slice_data_cabac(&c, &b, &h, is_p, stop);
  /* 7.3.4 slice_data */
  int addr = h.first_mb, more = 1, qp = h.qp;
  while (more) {
    if (addr >= d->nmb) return fo_fail(d, FO_E_FORMAT, "macroblock address past the picture");
    if (is_p) {
      int run = (int)fb_ue(&b);
      if (b.err || addr + run > d->nmb) return fo_fail(d, FO_E_FORMAT, "mb_skip_run");
      for (int i = 0; i < run; i++, addr++) {
        if (d->mb[addr].slice >= 0) return fo_fail(d, FO_E_FORMAT, "macroblock decoded twice");
        d->mb[addr].slice = slice_no;
        int rc = decode_mb(&c, NULL, addr, 1, &qp, &h);
        if (rc) return rc;
      }
      if (run > 0) {
        more = fb_index(&b, 0) < stop;
        if (!more) break;
      }
      if (addr >= d->nmb) return fo_fail(d, FO_E_FORMAT, "data after the last macroblock");
    }
    if (d->mb[addr].slice >= 0) return fo_fail(d, FO_E_FORMAT, "macroblock decoded twice");
    d->mb[addr].slice = slice_no;
    int rc = decode_mb(&c, &b, addr, is_p, &qp, &h);
    if (getenv("FO_TRACE"))
      fprintf(stderr, "oracle mb %d type %d cbp %d qp %d bits %lld\n", addr, d->mb[addr].type, d->mb[addr].cbp, qp,
              (long long)fb_index(&b, 0));
    if (rc) return rc;
    if (b.err) return fo_fail(d, FO_E_FORMAT, "bitstream exhausted");
    addr++;
    more = fb_index(&b, 0) < stop;
  }
  if (fb_index(&b, 0) != stop || b.err) return fo_fail(d, FO_E_FORMAT, "slice data does not end at the stop bit");
  return 0;
}

/* ------------------------------------------- B / weighted prediction */
/* Table 7-14: prediction of the two partitions of B mb_type 1..21 (1 Pred_L0,
   2 Pred_L1, 3 BiPred); odd types >= 5 are 8x16, even >= 4 16x8 */
static const uint8_t B_PART[22][2] = {{0, 0}, {1, 0}, {2, 0}, {3, 0}, {1, 1}, {1, 1}, {2, 2}, {2, 2},
                                      {1, 2}, {1, 2}, {2, 1}, {2, 1}, {1, 3}, {1, 3}, {2, 3}, {2, 3},
                                      {3, 1}, {3, 1}, {3, 2}, {3, 2}, {3, 3}, {3, 3}};
/* Table 7-18: B sub_mb_type -> (prediction, shape 0 8x8 / 1 8x4 / 2 4x8 / 3 4x4); prediction 0 = direct */
static const uint8_t B_SUB[13][2] = {{0, 0}, {1, 0}, {2, 0}, {3, 0}, {1, 1}, {1, 2}, {2, 1},
                                     {2, 2}, {3, 1}, {3, 2}, {1, 3}, {2, 3}, {3, 3}};

static void set_mv(const fo_ctx *c, fo_mb *m, int l, int blk, int ref, int mvx, int mvy) {
  fo_pic *const *list = l ? c->list1 : c->list;
  m->refidx[l][blk] = ref;
  m->refpic[l][blk] = ref >= 0 ? list[ref]->id : -1;
  m->mv[l][blk][0] = ref >= 0 ? mvx : 0;
  m->mv[l][blk][1] = ref >= 0 ? mvy : 0;
}

static int min_positive(int x, int y) { return (x >= 0 && y >= 0) ? (x < y ? x : y) : (x > y ? x : y); }

/* 8.4.1.2: direct prediction of the 4x4 blocks in mask (raster bits) */
static int direct_pred(fo_ctx *c, int addr, int mask) {
  fo_dec *d = c->d;
  fo_mb *m = &d->mb[addr];
  const fo_pic *col = c->list1[0];
  int spatial = c->h->direct_spatial;
  int ref[2] = {-1, -1}, mvp[2][2] = {{0, 0}, {0, 0}}, zero = 0;
  if (spatial) { /* 8.4.1.2.2: reference indices and predictors of the 16x16 */
    for (int l = 0; l < 2; l++) {
      fo_nbmv A = nb_mv(d, l, addr, -1, 0, 0), B = nb_mv(d, l, addr, 0, -1, 0), C = nb_mv(d, l, addr, 16, -1, 0);
      if (!C.avail) C = nb_mv(d, l, addr, -1, -1, 0);
      ref[l] = min_positive(A.ref, min_positive(B.ref, C.ref));
    }
    if (ref[0] < 0 && ref[1] < 0) { ref[0] = ref[1] = 0; zero = 1; }
    for (int l = 0; l < 2; l++)
      if (ref[l] >= 0 && !zero) mv_pred(d, l, addr, 0, 0, 16, 16, ref[l], 0, &mvp[l][0], &mvp[l][1]);
  }
  for (int blk = 0; blk < 16; blk++) {
    if (!((mask >> blk) & 1)) continue;
    /* 8.4.1.2.1 colocated 4x4 block (direct_8x8_inference: the macroblock corner of the 8x8) */
    int cb = blk;
    if (d->S->direct8x8) cb = ((blk >> 3) * 3) * 4 + ((blk & 3) >> 1) * 3;
    int ci = addr * 16 + cb, cl = col->mref[0][ci] >= 0 ? 0 : 1;
    int ref_col = col->mref[cl][ci];   /* -1: intra */
    int mvc_x = ref_col < 0 ? 0 : col->mmv[cl][ci * 2], mvc_y = ref_col < 0 ? 0 : col->mmv[cl][ci * 2 + 1];
    if (spatial) {
      int col_zero = col->ref == 1 && ref_col == 0 && mvc_x >= -1 && mvc_x <= 1 && mvc_y >= -1 && mvc_y <= 1;
      for (int l = 0; l < 2; l++) {
        int z = zero || ref[l] < 0 || (ref[l] == 0 && col_zero);
        set_mv(c, m, l, blk, ref[l], z ? 0 : mvp[l][0], z ? 0 : mvp[l][1]);
      }
    } else { /* 8.4.1.2.3 temporal */
      int r0 = 0;
      if (ref_col >= 0) {
        int id = col->mpic[cl][ci];
        r0 = -1;
        for (int i = 0; i < c->nlist && r0 < 0; i++)
          if (c->list[i] && c->list[i]->id == id) r0 = i;
        if (r0 < 0) return fo_fail(d, FO_E_DECODE, "temporal direct: colocated reference not in RefPicList0");
      }
      const fo_pic *p0 = c->list[r0], *p1 = c->list1[0];
      if (!p0) return fo_fail(d, FO_E_DECODE, "temporal direct: no reference picture");
      int tb = clip3(-128, 127, c->cur->poc - p0->poc), td = clip3(-128, 127, p1->poc - p0->poc);
      int m0x, m0y, m1x, m1y;
      if (p0->ref == 2 || td == 0) { m0x = mvc_x; m0y = mvc_y; m1x = m1y = 0; }
      else {
        int tx = (16384 + iabs(td / 2)) / td;
        int dsf = clip3(-1024, 1023, (tb * tx + 32) >> 6);
        m0x = (dsf * mvc_x + 128) >> 8;
        m0y = (dsf * mvc_y + 128) >> 8;
        m1x = m0x - mvc_x;
        m1y = m0y - mvc_y;
      }
      set_mv(c, m, 0, blk, r0, m0x, m0y);
      set_mv(c, m, 1, blk, 0, m1x, m1y);
    }
  }
  return 0;
}

/* mb_pred / sub_mb_pred (7.3.5.1-2) and the motion of a P or B inter macroblock (CAVLC) */
static int inter_mb_cavlc(fo_ctx *c, fb_t *b, int addr, int mb_type) {
  fo_dec *d = c->d;
  fo_mb *m = &d->mb[addr];
  int shape, pm[4] = {1, 1, 1, 1}, ssh[4] = {0, 0, 0, 0}, ref0 = 0;
  if (!c->is_b) {
    shape = mb_type == 0 ? 0 : (mb_type <= 2 ? mb_type : 3);
    ref0 = mb_type == 4;   /* P_8x8ref0 */
  } else if (mb_type == 0) {
    shape = 0;
    pm[0] = 0;             /* B_Direct_16x16 */
  } else if (mb_type <= 3) {
    shape = 0;
    pm[0] = mb_type;
  } else if (mb_type < 22) {
    shape = (mb_type & 1) ? 2 : 1;
    pm[0] = B_PART[mb_type][0];
    pm[1] = B_PART[mb_type][1];
  } else {
    shape = 3;
  }
  int nparts = shape == 0 ? 1 : (shape < 3 ? 2 : 4);
  if (shape == 3)
    for (int k = 0; k < 4; k++) {
      uint32_t v = fb_ue(b);
      if (v > (c->is_b ? 12u : 3u)) return fo_fail(d, FO_E_FORMAT, "sub_mb_type");
      if (c->is_b) { pm[k] = B_SUB[v][0]; ssh[k] = B_SUB[v][1]; }
      else ssh[k] = (int)v;
    }
  int refs[2][4] = {{-1, -1, -1, -1}, {-1, -1, -1, -1}};
  for (int l = 0; l < 1 + c->is_b; l++) {
    int nref = l ? c->nlist1 : c->nlist;
    fo_pic *const *list = l ? c->list1 : c->list;
    for (int k = 0; k < nparts; k++) {
      if (!((pm[k] >> l) & 1)) continue;
      refs[l][k] = (nref > 1 && !ref0) ? fb_te(b, nref - 1) : 0;
      if (refs[l][k] < 0 || refs[l][k] >= nref || !list[refs[l][k]])
        return fo_fail(d, FO_E_DECODE, "ref_idx names no reference picture");
    }
  }
  int mvd[2][4][4][2];
  for (int l = 0; l < 1 + c->is_b; l++)
    for (int k = 0; k < nparts; k++) {
      if (!((pm[k] >> l) & 1)) continue;
      int nsub = shape < 3 ? 1 : (ssh[k] == 0 ? 1 : (ssh[k] == 3 ? 4 : 2));
      for (int q = 0; q < nsub; q++) {
        mvd[l][k][q][0] = fb_se(b);
        mvd[l][k][q][1] = fb_se(b);
      }
    }
  /* motion: partitions in order, both lists of a (sub-)partition before the next */
  int done = 0;
  for (int k = 0; k < nparts; k++) {
    int nsub = 1, pw, ph, x0, y0;
    if (shape == 0) { pw = ph = 16; x0 = y0 = 0; }
    else if (shape == 1) { pw = 16; ph = 8; x0 = 0; y0 = 8 * k; }
    else if (shape == 2) { pw = 8; ph = 16; x0 = 8 * k; y0 = 0; }
    else {
      x0 = 8 * (k & 1);
      y0 = 8 * (k >> 1);
      nsub = ssh[k] == 0 ? 1 : (ssh[k] == 3 ? 4 : 2);
      pw = ssh[k] == 0 || ssh[k] == 1 ? 8 : 4;
      ph = ssh[k] == 0 || ssh[k] == 2 ? 8 : 4;
    }
    if (pm[k] == 0) { /* direct: B_Direct_16x16 or B_Direct_8x8 */
      int bm = 0;
      for (int yy = y0 / 4; yy < (y0 + ph) / 4; yy++)
        for (int xx = x0 / 4; xx < (x0 + pw) / 4; xx++) bm |= 1 << (yy * 4 + xx);
      int rc = direct_pred(c, addr, bm);
      if (rc) return rc;
      done |= bm;
      continue;
    }
    for (int q = 0; q < nsub; q++) {
      int sx = x0, sy = y0;
      if (shape == 3) {
        if (ssh[k] == 1) sy += 4 * q;
        else if (ssh[k] == 2) sx += 4 * q;
        else if (ssh[k] == 3) { sx += 4 * (q & 1); sy += 4 * (q >> 1); }
      }
      for (int l = 0; l < 2; l++) {
        int use = (pm[k] >> l) & 1;
        int vx = 0, vy = 0;
        if (use) {
          int px, py;
          mv_pred(d, l, addr, sx, sy, pw, ph, refs[l][k], done, &px, &py);
          vx = px + mvd[l][k][q][0];
          vy = py + mvd[l][k][q][1];
          if (vx < -32768 || vx > 32767 || vy < -32768 || vy > 32767) return fo_fail(d, FO_E_FORMAT, "mv range");
        }
        for (int yy = sy / 4; yy < (sy + ph) / 4; yy++)
          for (int xx = sx / 4; xx < (sx + pw) / 4; xx++) set_mv(c, m, l, yy * 4 + xx, use ? refs[l][k] : -1, vx, vy);
      }
      for (int yy = sy / 4; yy < (sy + ph) / 4; yy++)
        for (int xx = sx / 4; xx < (sx + pw) / 4; xx++) done |= 1 << (yy * 4 + xx);
    }
  }
  return 0;
}

/* implicit bi-prediction weights (8.4.2.3.1) for refIdxL0 r0, refIdxL1 r1 */
static void implicit_w(const fo_ctx *c, int r0, int r1, int *w0, int *w1) {
  const fo_pic *p0 = c->list[r0], *p1 = c->list1[r1];
  int tb = clip3(-128, 127, c->cur->poc - p0->poc), td = clip3(-128, 127, p1->poc - p0->poc);
  *w0 = *w1 = 32;
  if (td == 0 || p0->ref == 2 || p1->ref == 2) return;
  int tx = (16384 + iabs(td / 2)) / td;
  int dsf = clip3(-1024, 1023, (tb * tx + 32) >> 6);
  if ((dsf >> 2) < -64 || (dsf >> 2) > 128) return;
  *w0 = 64 - (dsf >> 2);
  *w1 = dsf >> 2;
}

/* 8.4.2.3: one predicted sample from the list-0 / list-1 predictions p0, p1
   (r0 / r1 < 0: list unused); pl -1 luma, 0 Cb, 1 Cr */
static int wp_sample(const fo_ctx *c, int pl, int r0, int r1, int p0, int p1) {
  if (c->wmode == 1) {
    const fo_hdr *h = c->h;
    int lwd = pl < 0 ? h->lwd : h->cwd;
    int w0 = 0, o0 = 0, w1 = 0, o1 = 0;
    if (r0 >= 0) { w0 = pl < 0 ? h->lw[0][r0] : h->cw[0][r0][pl]; o0 = pl < 0 ? h->lo[0][r0] : h->co[0][r0][pl]; }
    if (r1 >= 0) { w1 = pl < 0 ? h->lw[1][r1] : h->cw[1][r1][pl]; o1 = pl < 0 ? h->lo[1][r1] : h->co[1][r1][pl]; }
    if (r0 >= 0 && r1 >= 0) return clip1(((p0 * w0 + p1 * w1 + (1 << lwd)) >> (lwd + 1)) + ((o0 + o1 + 1) >> 1));
    int p = r0 >= 0 ? p0 : p1, w = r0 >= 0 ? w0 : w1, o = r0 >= 0 ? o0 : o1;
    if (lwd >= 1) return clip1(((p * w + (1 << (lwd - 1))) >> lwd) + o);
    return clip1(p * w + o);
  }
  if (r0 >= 0 && r1 >= 0) {
    if (c->wmode == 2) {
      int w0, w1;
      implicit_w(c, r0, r1, &w0, &w1);
      return clip1((p0 * w0 + p1 * w1 + 32) >> 6);
    }
    return (p0 + p1 + 1) >> 1;
  }
  return r0 >= 0 ? p0 : p1;
}

/* inter prediction of the whole macroblock from its per-4x4 motion */
static void inter_pred_mb(const fo_ctx *c, int addr, int *py, int *pu, int *pv) {
  const fo_dec *d = c->d;
  const fo_mb *m = &d->mb[addr];
  int ty[2][256], tu[2][64], tv[2][64];
  for (int blk = 0; blk < 16; blk++) {
    int bx = (blk % 4) * 4, by = (blk / 4) * 4;
    int r0 = m->refidx[0][blk], r1 = m->refidx[1][blk];
    for (int l = 0; l < 2; l++) {
      int r = l ? r1 : r0;
      if (r < 0) continue;
      mc_part(d, l ? c->list1[r] : c->list[r], addr, bx, by, 4, 4, m->mv[l][blk][0], m->mv[l][blk][1], ty[l], tu[l],
              tv[l]);
    }
    for (int y = 0; y < 4; y++)
      for (int x = 0; x < 4; x++) {
        int i = (by + y) * 16 + bx + x;
        py[i] = wp_sample(c, -1, r0, r1, ty[0][i], ty[1][i]);
      }
    for (int y = 0; y < 2; y++)
      for (int x = 0; x < 2; x++) {
        int i = (by / 2 + y) * 8 + bx / 2 + x;
        pu[i] = wp_sample(c, 0, r0, r1, tu[0][i], tu[1][i]);
        pv[i] = wp_sample(c, 1, r0, r1, tv[0][i], tv[1][i]);
      }
  }
}

/* macroblock_layer (7.3.5) + reconstruction; b == NULL: P_Skip */
static int decode_mb(fo_ctx *c, fb_t *b, int addr, int is_p, int *qp, const fo_hdr *h) {
  (void)h;
  fo_dec *d = c->d;
  fo_mb *m = &d->mb[addr];
  fo_pic *pic = c->cur;
  int slice = m->slice;
  memset(m, 0, sizeof *m);
  m->slice = slice;
  for (int i = 0; i < 16; i++) {
    m->refidx[0][i] = m->refidx[1][i] = -1;
    m->refpic[0][i] = m->refpic[1][i] = -1;
    m->i4[i] = 2;
  }
  int mx = addr % d->mbw, my = addr / d->mbw;
  int pred_y[256], pred_u[64], pred_v[64];
  if (!b) { /* P_Skip (8.4.1.1) / B_Skip (8.4.1.2) */
    m->type = 4;
    m->qp = *qp;
    if (c->is_b) {
      m->direct8 = 15;
      m->d16 = 1;
      int rc = direct_pred(c, addr, 0xffff);
      if (rc) return rc;
    } else {
      int px = 0, py = 0;
      fo_loc LA = nb_loc(d, addr, -1, 0, 16, 16), LB = nb_loc(d, addr, 0, -1, 16, 16);
      fo_nbmv A = nb_mv(d, 0, addr, -1, 0, 0), B = nb_mv(d, 0, addr, 0, -1, 0);
      if (!(LA.mb < 0 || LB.mb < 0 || (A.ref == 0 && A.mvx == 0 && A.mvy == 0) ||
            (B.ref == 0 && B.mvx == 0 && B.mvy == 0)))
        mv_pred(d, 0, addr, 0, 0, 16, 16, 0, 0, &px, &py);
      if (!c->list[0] || c->nlist < 1) return fo_fail(d, FO_E_DECODE, "P_Skip without a reference picture");
      for (int i = 0; i < 16; i++) set_mv(c, m, 0, i, 0, px, py);
    }
    inter_pred_mb(c, addr, pred_y, pred_u, pred_v);
    for (int y = 0; y < 16; y++)
      for (int x = 0; x < 16; x++) pic->y[(int64_t)(my * 16 + y) * d->W + mx * 16 + x] = (uint8_t)pred_y[y * 16 + x];
    for (int y = 0; y < 8; y++)
      for (int x = 0; x < 8; x++) {
        pic->u[(int64_t)(my * 8 + y) * (d->W / 2) + mx * 8 + x] = (uint8_t)pred_u[y * 8 + x];
        pic->v[(int64_t)(my * 8 + y) * (d->W / 2) + mx * 8 + x] = (uint8_t)pred_v[y * 8 + x];
      }
    return 0;
  }
  int mb_type = (int)fb_ue(b);
  int itype;                 /* I mb_type (0..25) or -1 for inter */
  int intra0 = c->is_b ? 23 : (is_p ? 5 : 0);   /* first intra mb_type (Tables 7-11, 7-13, 7-14) */
  itype = mb_type >= intra0 ? mb_type - intra0 : -1;
  if (itype > 25) return fo_fail(d, FO_E_FORMAT, "mb_type");
  if (itype == 25) { /* I_PCM (7.3.5) */
    m->type = 3;
    m->qp = *qp;
    b->bitpos = 0; /* pcm_alignment_zero_bit */
    for (int y = 0; y < 16; y++)
      for (int x = 0; x < 16; x++) pic->y[(int64_t)(my * 16 + y) * d->W + mx * 16 + x] = (uint8_t)fb_byte(b);
    for (int pl = 0; pl < 2; pl++)
      for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++)
          (pl ? pic->v : pic->u)[(int64_t)(my * 8 + y) * (d->W / 2) + mx * 8 + x] = (uint8_t)fb_byte(b);
    for (int i = 0; i < 16; i++) m->nz[i] = 16;
    for (int i = 0; i < 4; i++) m->nzc[0][i] = m->nzc[1][i] = 16;
    return b->err ? fo_fail(d, FO_E_FORMAT, "I_PCM") : 0;
  }
  int cbp = 0, i16mode = 0, cmode = 0;
  if (itype == 0) { /* I_NxN: 8.3.1.1 mode prediction */
    m->type = 1;
    int prev[16], rem[16];
    for (int k = 0; k < 16; k++) {
      prev[k] = (int)fb_bit(b);
      rem[k] = prev[k] ? 0 : (int)fb_bits(b, 3);
    }
    for (int k = 0; k < 16; k++) {
      int bx = BLK_X[k], by = BLK_Y[k];
      fo_loc LA = nb_loc(d, addr, bx * 4 - 1, by * 4, 16, 16), LB = nb_loc(d, addr, bx * 4, by * 4 - 1, 16, 16);
      int dcf = LA.mb < 0 || LB.mb < 0 ||
                (LA.mb >= 0 && !mb_intra(&d->mb[LA.mb]) && d->P->cip) ||
                (LB.mb >= 0 && !mb_intra(&d->mb[LB.mb]) && d->P->cip);
      int pm;
      if (dcf) pm = 2;
      else {
        const fo_mb *ma = &d->mb[LA.mb], *mb2 = &d->mb[LB.mb];
        int a = ma->type == 1 ? ma->i4[(LA.yw / 4) * 4 + LA.xw / 4] : 2;
        int bb = mb2->type == 1 ? mb2->i4[(LB.yw / 4) * 4 + LB.xw / 4] : 2;
        pm = imin(a, bb);
      }
      int mode = prev[k] ? pm : (rem[k] < pm ? rem[k] : rem[k] + 1);
      m->i4[by * 4 + bx] = mode;
    }
    cmode = (int)fb_ue(b);
  } else if (itype >= 1) { /* I_16x16 (Table 7-11) */
    m->type = 2;
    i16mode = (itype - 1) % 4;
    cbp = (((itype - 1) / 4) % 3) << 4 | (itype >= 13 ? 15 : 0);
    cmode = (int)fb_ue(b);
  } else { /* inter (Tables 7-13, 7-14, 7-17, 7-18) */
    m->type = 0;
    int rc = inter_mb_cavlc(c, b, addr, mb_type);
    if (rc) return rc;
  }
  if (m->type != 2) {
    uint32_t code = fb_ue(b);
    if (code > 47) return fo_fail(d, FO_E_FORMAT, "coded_block_pattern");
    cbp = m->type == 1 ? CBP_INTRA[code] : CBP_INTER[code];
  }
  m->cbp = cbp;
  if ((cbp & 15) || (cbp >> 4) || m->type == 2) {
    int dq = fb_se(b);
    if (dq < -26 || dq > 25) return fo_fail(d, FO_E_FORMAT, "mb_qp_delta");
    *qp = (*qp + dq + 52) % 52;
  }
  m->qp = *qp;
  if (cmode > 3 || (m->type == 2 && i16mode > 3)) return fo_fail(d, FO_E_FORMAT, "intra pred mode");

  /* ---- residual (7.3.5.3), coefficients in raster 4x4 per block */
  int coef[16][16], dcl[16], cdc[2][4], cac[2][4][16];
  memset(coef, 0, sizeof coef);
  memset(dcl, 0, sizeof dcl);
  memset(cdc, 0, sizeof cdc);
  memset(cac, 0, sizeof cac);
  int lvl[16];
  if (m->type == 2) {
    int nC = nc_of(d, addr, 0, 0, 0, 0);
    int tc = residual_block(b, nC, 0, 15, 16, lvl);
    if (tc < 0) return fo_fail(d, FO_E_FORMAT, "Intra16x16DCLevel");
    for (int k = 0; k < 16; k++) dcl[ZZ4[k]] = lvl[k];
  }
  for (int k8 = 0; k8 < 4; k8++)
    for (int k4 = 0; k4 < 4; k4++) {
      int blk = k8 * 4 + k4, bx = BLK_X[blk], by = BLK_Y[blk];
      if (!((cbp >> k8) & 1)) continue;
      int nC = nc_of(d, addr, bx, by, 0, 0);
      int tc;
      if (m->type == 2) {
        tc = residual_block(b, nC, 0, 14, 15, lvl);
        if (tc < 0) return fo_fail(d, FO_E_FORMAT, "Intra16x16ACLevel");
        for (int k = 0; k < 15; k++) coef[by * 4 + bx][ZZ4[k + 1]] = lvl[k];
      } else {
        tc = residual_block(b, nC, 0, 15, 16, lvl);
        if (tc < 0) return fo_fail(d, FO_E_FORMAT, "LumaLevel4x4");
        for (int k = 0; k < 16; k++) coef[by * 4 + bx][ZZ4[k]] = lvl[k];
      }
      m->nz[by * 4 + bx] = tc;
    }
  if (cbp >> 4) {
    for (int pl = 0; pl < 2; pl++) {
      int tc = residual_block(b, -1, 0, 3, 4, lvl);
      if (getenv("FO_TRACE")) fprintf(stderr, "  chroma dc %d tc %d bits %lld\n", pl, tc, (long long)fb_index(b, 0));
      if (tc < 0) return fo_fail(d, FO_E_FORMAT, "ChromaDCLevel");
      for (int k = 0; k < 4; k++) cdc[pl][k] = lvl[k];
    }
  }
  if ((cbp >> 4) & 2) {
    for (int pl = 0; pl < 2; pl++)
      for (int k = 0; k < 4; k++) {
        int bx = k & 1, by = k >> 1;
        int nC = nc_of(d, addr, bx, by, 1, pl);
        int tc = residual_block(b, nC, 0, 14, 15, lvl);
        if (getenv("FO_TRACE")) fprintf(stderr, "  chroma ac %d %d nC %d tc %d bits %lld\n", pl, k, nC, tc, (long long)fb_index(b, 0));
        if (tc < 0) return fo_fail(d, FO_E_FORMAT, "ChromaACLevel");
        for (int j = 0; j < 15; j++) cac[pl][k][ZZ4[j + 1]] = lvl[j];
        m->nzc[pl][k] = tc;
      }
  }
  if (b->err) return fo_fail(d, FO_E_FORMAT, "bitstream exhausted in residual");

  return recon_mb(c, addr, coef, dcl, cdc, cac, NULL, i16mode, cmode);
}

/* ------------------------------------------------------------ CABAC (9.3) */
#define RANGE_LPS FO_RANGE_LPS
#define TRANS_LPS FO_TRANS_LPS
#define SIG8 FO_SIG8_FRAME
#define LAST8 FO_LAST8_FRAME
/* (m, n) by ctxIdx for the I column and cabac_init_idc 0, spread from the
 * standard's per-range listing (h264_std_tables.h); entries the standard
 * leaves undefined for a column stay (0, 0) and are never used by it */
static int8_t CAB_INIT_I[FO_NCTX][2], CAB_INIT_P0[FO_NCTX][2];
/* 8.5.6 / Figure 8-9: frame zig-zag of an 8x8 block, coefficient list index
 * -> raster position, by walking the anti-diagonals alternately */
static int ZZ8[64];
static void fo_tables_init(void) {
  static int done;
  if (done) return;
  for (size_t i = 0; i < sizeof FO_CTX_INIT / sizeof FO_CTX_INIT[0]; i++) {
    const fo_ctx_init *e = &FO_CTX_INIT[i];
    if (e->mi != FO_NA) { CAB_INIT_I[e->ctx][0] = e->mi; CAB_INIT_I[e->ctx][1] = e->ni; }
    CAB_INIT_P0[e->ctx][0] = e->mp;
    CAB_INIT_P0[e->ctx][1] = e->np;
  }
  int k = 0;
  for (int d = 0; d < 15; d++) {        /* d = row + column */
    for (int t = 0; t <= d; t++) {
      int row = (d % 2 == 0) ? d - t : t; /* even diagonals run up-right, odd down-left */
      int col = d - row;
      if (row < 8 && col < 8) ZZ8[k++] = row * 8 + col;
    }
  }
  done = 1;
}

/* the oracle's tables, for tests/test_cabac_tables.py:
 * which 0: CAB_INIT_I (i = ctxIdx, j = 0 m / 1 n; defined[i] in *ok),
 * 1: CAB_INIT_P0, 2: rangeTabLPS[i][j], 3: transIdxLPS[i], 4: Table 9-43
 * significant ctxIdxInc [i], 5: last ctxIdxInc [i], 6: zig-zag [i],
 * 7: normAdjust8x8 v8x8[i][j] (m, class) */
int fo_std_table(int which, int i, int j, int *ok) {
  fo_tables_init();
  *ok = 1;
  switch (which) {
    case 0: case 1:
      for (size_t x = 0; x < sizeof FO_CTX_INIT / sizeof FO_CTX_INIT[0]; x++)
        if (FO_CTX_INIT[x].ctx == i) {
          if (which == 0 && FO_CTX_INIT[x].mi == FO_NA) break;
          return which == 0 ? (j ? FO_CTX_INIT[x].ni : FO_CTX_INIT[x].mi)
                            : (j ? FO_CTX_INIT[x].np : FO_CTX_INIT[x].mp);
        }
      *ok = 0;
      return 0;
    case 2: return FO_RANGE_LPS[i][j];
    case 3: return FO_TRANS_LPS[i];
    case 4: return FO_SIG8_FRAME[i];
    case 5: return FO_LAST8_FRAME[i];
    case 6: return ZZ8[i];
    case 7: return FO_V8[i][j];
    case 8: return FO_DEFAULT_4x4[i][j];   /* Table 7-3: [intra / inter][scan index] */
    case 9: return FO_DEFAULT_8x8[i][j];   /* Table 7-4 */
    default: *ok = 0; return 0;
  }
}

/* CABAC stream synthesis (TEST INFRASTRUCTURE, fo_cabac_convert below): the
 * decoder below runs unchanged, but every bin it asks for is chosen by a
 * seeded random policy and arithmetic-coded (9.3.4) instead of being read, so
 * the bitstream written is exactly what the decoder would have parsed. */
struct fo_enc_s {
  uint8_t *out;            /* bit writer */
  int64_t cap, nbits;
  uint32_t low, range;
  int first, outstanding;
  uint64_t rng;
  int last_mb;             /* end_of_slice_flag is 1 after this macroblock */
  int nref, ref_ones;      /* ref_idx being chosen: entries of the list, ones so far */
  int overflow;
};

static void enc_write(fo_enc *e, int b) {
  if (e->nbits >= e->cap * 8) { e->overflow = 1; return; }
  if (b) e->out[e->nbits >> 3] |= (uint8_t)(0x80 >> (e->nbits & 7));
  e->nbits++;
}
static void enc_put(fo_enc *e, int b) { /* PutBit (9.3.4.2) */
  if (e->first) e->first = 0;
  else enc_write(e, b);
  for (; e->outstanding > 0; e->outstanding--) enc_write(e, !b);
}
static void enc_renorm(fo_enc *e) { /* RenormE */
  while (e->range < 256) {
    if (e->low < 256) enc_put(e, 0);
    else if (e->low >= 512) { e->low -= 512; enc_put(e, 1); }
    else { e->low -= 256; e->outstanding++; }
    e->range <<= 1;
    e->low <<= 1;
  }
}
static uint32_t enc_rand(fo_enc *e) {
  e->rng = e->rng * 6364136223846793005ull + 1442695040888963407ull;
  return (uint32_t)(e->rng >> 33);
}
/* probability (per 1024) of a 1 bin for ctxIdx, by syntax element (Table 9-34) */
static int enc_p1(int ctx) {
  if (ctx >= 11 && ctx <= 13) return 300;   /* mb_skip_flag P */
  if (ctx >= 24 && ctx <= 26) return 300;   /* mb_skip_flag B */
  if (ctx >= 40 && ctx <= 53) return 380;   /* mvd prefix */
  if (ctx >= 60 && ctx <= 63) return 250;   /* mb_qp_delta */
  if (ctx >= 105 && ctx <= 226) return 330; /* significant / last */
  if (ctx >= 227 && ctx <= 275) return 300; /* coeff_abs_level_minus1 */
  if (ctx >= 402 && ctx <= 459) return 330; /* 8x8 significant / last / levels */
  return 512;
}

typedef struct {
  fb_t *b;
  uint32_t range, offset;
  uint8_t state[FO_NCTX], mps[FO_NCTX];
} fo_cab;

static void cab_start(fo_cab *k) { /* 9.3.1.2 */
  k->range = 510;
  if (g_enc) { /* 9.3.4.1 */
    g_enc->low = 0;
    g_enc->range = 510;
    g_enc->first = 1;
    g_enc->outstanding = 0;
    k->offset = 0;
    return;
  }
  k->offset = fb_bits(k->b, 9);
}
static void cab_init(fo_cab *k, int is_i, int qp) { /* 9.3.1.1 */
  fo_tables_init();
  const int8_t(*t)[2] = is_i ? CAB_INIT_I : CAB_INIT_P0;
  for (int i = 0; i < FO_NCTX; i++) {
    int pre = clip3(1, 126, ((t[i][0] * clip3(0, 51, qp)) >> 4) + t[i][1]);
    if (pre <= 63) { k->state[i] = (uint8_t)(63 - pre); k->mps[i] = 0; }
    else { k->state[i] = (uint8_t)(pre - 64); k->mps[i] = 1; }
  }
}
static int cab_dec(fo_cab *k, int ctx) { /* 9.3.3.2.1 DecodeDecision */
  int s = k->state[ctx], bin;
  if (g_enc) { /* synthesis: choose the bin, EncodeDecision (9.3.4.2) */
    fo_enc *e = g_enc;
    if (ctx >= 54 && ctx <= 59) { /* ref_idx: unary, stays inside the list */
      if (ctx <= 57) e->ref_ones = 0;
      bin = e->ref_ones + 1 < e->nref && (int)(enc_rand(e) & 1023) < 300;
      e->ref_ones += bin;
    } else {
      bin = (int)(enc_rand(e) & 1023) < enc_p1(ctx);
    }
    uint32_t lps = RANGE_LPS[s][(e->range >> 6) & 3];
    e->range -= lps;
    if (bin != k->mps[ctx]) {
      e->low += e->range;
      e->range = lps;
      if (s == 0) k->mps[ctx] = (uint8_t)(1 - k->mps[ctx]);
      k->state[ctx] = TRANS_LPS[s];
    } else if (s < 62) {
      k->state[ctx] = (uint8_t)(s + 1);
    }
    enc_renorm(e);
    return bin;
  }
  uint32_t lps = RANGE_LPS[s][(k->range >> 6) & 3];
  k->range -= lps;
  if (k->offset >= k->range) {
    bin = !k->mps[ctx];
    k->offset -= k->range;
    k->range = lps;
    if (s == 0) k->mps[ctx] = (uint8_t)(1 - k->mps[ctx]);
    k->state[ctx] = TRANS_LPS[s];
  } else {
    bin = k->mps[ctx];
    if (s < 62) k->state[ctx] = (uint8_t)(s + 1);
  }
  while (k->range < 256) { /* RenormD */
    k->range <<= 1;
    k->offset = (k->offset << 1) | fb_bit(k->b);
  }
  return bin;
}
static int cab_bypass(fo_cab *k) { /* 9.3.3.2.3 */
  if (g_enc) { /* EncodeBypass (9.3.4.4); suffixes stay short */
    fo_enc *e = g_enc;
    int bin = (int)(enc_rand(e) & 1023) < 350;
    e->low <<= 1;
    if (bin) e->low += e->range;
    if (e->low >= 1024) { enc_put(e, 1); e->low -= 1024; }
    else if (e->low < 512) enc_put(e, 0);
    else { e->low -= 512; e->outstanding++; }
    return bin;
  }
  k->offset = (k->offset << 1) | fb_bit(k->b);
  if (k->offset >= k->range) { k->offset -= k->range; return 1; }
  return 0;
}
static int cab_term(fo_cab *k) { /* 9.3.3.2.2.3: binVal 1 ends parsing without renormalisation */
  if (g_enc) { /* EncodeTerminate (9.3.4.5): 1 only for end_of_slice_flag after the slice's last macroblock */
    fo_enc *e = g_enc;
    int bin = e->last_mb < 0;
    e->range -= 2;
    if (bin) {
      e->low += e->range;
      e->range = 2; /* EncodeFlush */
      enc_renorm(e);
      enc_put(e, (e->low >> 9) & 1);
      enc_write(e, (e->low >> 8) & 1);
      enc_write(e, 1); /* rbsp_stop_one_bit */
    } else {
      enc_renorm(e);
    }
    return bin;
  }
  k->range -= 2;
  if (k->offset >= k->range) return 1;
  while (k->range < 256) {
    k->range <<= 1;
    k->offset = (k->offset << 1) | fb_bit(k->b);
  }
  return 0;
}
static int cab_fl3(fo_cab *k, int ctx) { /* FL, cMax 7: bins least significant first */
  int v = cab_dec(k, ctx);
  v |= cab_dec(k, ctx) << 1;
  v |= cab_dec(k, ctx) << 2;
  return v;
}

/* mb_type of an I macroblock (Table 9-36): prefix ctxIdx 3 (I slice, inc from
 * the neighbours) or the suffix of a P (ctxIdxOffset 17) or B (32) slice's
 * intra mb_type (suffix = its offset); returns 0..25 */
static int cab_i_type(fo_cab *k, int suffix, int inc0) {
  if (!cab_dec(k, suffix ? suffix : 3 + inc0)) return 0; /* I_NxN */
  if (cab_term(k)) return 25;                       /* I_PCM */
  int luma = cab_dec(k, suffix ? suffix + 1 : 6);
  int chroma = cab_dec(k, suffix ? suffix + 2 : 7);
  if (chroma) chroma += cab_dec(k, suffix ? suffix + 2 : 8);
  int pm = cab_dec(k, suffix ? suffix + 3 : 9) << 1;
  pm |= cab_dec(k, suffix ? suffix + 3 : 10);
  return 1 + pm + 4 * chroma + 12 * luma;
}
/* B-slice mb_type (Table 9-37 binarization, ctxIdx 27..35 by Table 9-39):
 * 0 .. 22, or 23 + the intra suffix's mb_type */
static int cab_b_type(fo_cab *k, int inc0) {
  if (!cab_dec(k, 27 + inc0)) return 0;                  /* 0: B_Direct_16x16 */
  if (!cab_dec(k, 27 + 3)) return 1 + cab_dec(k, 27 + 5);  /* 1 0 b: B_L0 / B_L1_16x16 */
  int bits = cab_dec(k, 27 + 4) << 3;
  bits |= cab_dec(k, 27 + 5) << 2;
  bits |= cab_dec(k, 27 + 5) << 1;
  bits |= cab_dec(k, 27 + 5);
  if (bits < 8) return bits + 3;                          /* 1 1 0 x x x: 3 .. 10 */
  if (bits == 13) return 23 + cab_i_type(k, 32, 0);       /* 1 1 1 1 0 1: intra prefix */
  if (bits == 14) return 11;                              /* 1 1 1 1 1 0 */
  if (bits == 15) return 22;                              /* 1 1 1 1 1 1: B_8x8 */
  bits = (bits << 1) | cab_dec(k, 27 + 5);                /* 1 1 1 x x x x: 12 .. 21 */
  return bits - 4;
}
/* B sub_mb_type (Table 9-38 binarization, ctxIdx 36..39): 0 .. 12 */
static int cab_b_sub(fo_cab *k) {
  if (!cab_dec(k, 36)) return 0;                          /* B_Direct_8x8 */
  if (!cab_dec(k, 37)) return 1 + cab_dec(k, 39);         /* B_L0_8x8, B_L1_8x8 */
  int t = 3;
  if (cab_dec(k, 38)) {
    if (cab_dec(k, 39)) return 11 + cab_dec(k, 39);       /* B_L1_4x4, B_Bi_4x4 */
    t += 4;
  }
  t += 2 * cab_dec(k, 39);
  t += cab_dec(k, 39);
  return t;
}
/* mvd_lX component (U prefix cMax 9 + UEG3 suffix + sign, 9.3.2.3), sum =
 * absMvdComp(A) + absMvdComp(B) */
static int cab_mvd(fo_cab *k, int base, int sum) {
  if (!cab_dec(k, base + (sum < 3 ? 0 : (sum > 32 ? 2 : 1)))) return 0;
  static const int inc[8] = {3, 4, 5, 6, 6, 6, 6, 6};
  int v = 1;
  while (v < 9 && cab_dec(k, base + inc[v - 1])) v++;
  if (v >= 9) {
    int kk = 3;
    while (cab_bypass(k)) { v += 1 << kk; if (++kk > 30) return 0; }
    while (kk--) v += cab_bypass(k) << kk;
  }
  return cab_bypass(k) ? -v : v;
}

static const int CBF_OFF[5] = {0, 4, 8, 12, 16};
static const int SIG_OFF[5] = {0, 15, 29, 44, 47};
static const int ABS_OFF[5] = {0, 10, 20, 30, 39};
/* residual_block_cabac (7.3.5.3.3, 9.3.3.1.3) of ctxBlockCat cat: levels in
 * coefficient-list order into lvl; returns the count of non-zero levels
 * (0: coded_block_flag 0) or -1 */
static int cab_residual(fo_cab *k, int cat, int cbf_inc, int maxNum, int *lvl) {
  for (int i = 0; i < maxNum; i++) lvl[i] = 0;
  if (cat != 5 && !cab_dec(k, 85 + CBF_OFF[cat] + cbf_inc)) return 0;
  int sig[64] = {0}, numCoeff = maxNum;
  for (int i = 0; i < numCoeff - 1; i++) {
    int inc = cat == 3 ? imin(i, 2) : i;
    if (cab_dec(k, cat == 5 ? 402 + SIG8[i] : 105 + SIG_OFF[cat] + inc)) {
      sig[i] = 1;
      if (cab_dec(k, cat == 5 ? 417 + LAST8[i] : 166 + SIG_OFF[cat] + inc)) { numCoeff = i + 1; break; }
    }
  }
  sig[numCoeff - 1] = 1;
  int eq1 = 0, gt1 = 0, n = 0, base = cat == 5 ? 426 : 227 + ABS_OFF[cat];
  for (int i = numCoeff - 1; i >= 0; i--) {
    if (!sig[i]) continue;
    int v = 0;
    if (cab_dec(k, base + (gt1 ? 0 : imin(4, 1 + eq1)))) {
      v = 1;
      int inc = 5 + imin(4 - (cat == 3), gt1);
      while (v < 14 && cab_dec(k, base + inc)) v++;
      if (v >= 14) { /* UEG0 suffix */
        int kk = 0;
        while (cab_bypass(k)) { v += 1 << kk; if (++kk > 30) return -1; }
        while (kk--) v += cab_bypass(k) << kk;
      }
    }
    int lv = v + 1;
    if (cab_bypass(k)) lv = -lv;
    lvl[i] = lv;
    if (v == 0) eq1++;
    else gt1++;
    n++;
  }
  return n;
}

/* condTermFlagN of coded_block_flag (9.3.3.1.1.9): neighbour macroblock n
 * (-1 unavailable), transBlockN available (tb), its flag bit */
static int cbf_cond(const fo_dec *d, int cur_intra, int n, int tb, int bit) {
  if (n < 0) return cur_intra;
  const fo_mb *m = &d->mb[n];
  if (m->type == 3) return 1;
  if (!tb || m->type == 4) return 0;
  return (int)((m->cbf >> bit) & 1u);
}
/* coded_block_flag ctxIdxInc of a luma 4x4 block at (x, y) (4x4 units) */
static int cbf_luma_inc(const fo_dec *d, int addr, int x, int y, int intra) {
  int inc = 0;
  for (int nb = 0; nb < 2; nb++) {
    fo_loc L = nb_loc(d, addr, nb ? x * 4 : x * 4 - 1, nb ? y * 4 - 1 : y * 4, 16, 16);
    int tb = 0, bit = 0;
    if (L.mb >= 0) {
      const fo_mb *m = &d->mb[L.mb];
      int b8 = (L.yw / 8) * 2 + L.xw / 8;
      tb = (m->cbp >> b8) & 1;
      bit = 1 + (L.yw / 4) * 4 + L.xw / 4;
    }
    inc += cbf_cond(d, intra, L.mb, tb, bit) << nb;
  }
  return inc;
}
static int cbf_chroma_inc(const fo_dec *d, int addr, int pl, int blk, int dc, int intra) {
  int inc = 0;
  for (int nb = 0; nb < 2; nb++) {
    int x = dc ? 0 : (blk & 1) * 4, y = dc ? 0 : (blk >> 1) * 4;
    fo_loc L = nb_loc(d, addr, nb ? x : x - 1, nb ? y - 1 : y, 8, 8);
    int tb = 0, bit = 0;
    if (L.mb >= 0) {
      const fo_mb *m = &d->mb[L.mb];
      tb = dc ? (m->cbp >> 4) != 0 : (m->cbp >> 4) == 2;
      bit = dc ? 17 + pl : 19 + 4 * pl + (L.yw / 4) * 2 + L.xw / 4;
    }
    inc += cbf_cond(d, intra, L.mb, tb, bit) << nb;
  }
  return inc;
}
/* absMvdComp of list l's neighbouring block (0: unavailable, skip, intra,
   direct or list unused: their mvd is 0) */
static int abs_mvd_at(const fo_dec *d, int l, int addr, int xN, int yN, int comp) {
  fo_loc L = nb_loc(d, addr, xN, yN, 16, 16);
  if (L.mb < 0) return 0;
  const fo_mb *m = &d->mb[L.mb];
  if (m->type != 0) return 0; /* skip, intra */
  return iabs(m->mvd[l][(L.yw / 4) * 4 + L.xw / 4][comp]);
}
/* condTermFlagN of ref_idx_lX (9.3.3.1.1.6): refIdxLX > 0 of an inter
   neighbour block that is not skipped and not predicted in direct mode */
static int ref_gt0_at(const fo_dec *d, int l, int addr, int xN, int yN) {
  fo_loc L = nb_loc(d, addr, xN, yN, 16, 16);
  if (L.mb < 0) return 0;
  const fo_mb *m = &d->mb[L.mb];
  if (m->type != 0) return 0;
  int blk = (L.yw / 4) * 4 + L.xw / 4;
  if ((m->direct8 >> ((blk >> 3) * 2 + ((blk & 3) >> 1))) & 1) return 0;
  return m->refidx[l][blk] > 0;
}
/* Intra NxN mode predictor (8.3.1.1 / 8.3.2.1) of the block whose top-left
 * luma sample is (x0, y0); is8: the current block is 8x8 */
static int intra_pred_mode_pred(const fo_dec *d, int addr, int x0, int y0, int is8) {
  fo_loc LA = nb_loc(d, addr, x0 - 1, y0, 16, 16), LB = nb_loc(d, addr, x0, y0 - 1, 16, 16);
  if (LA.mb < 0 || LB.mb < 0) return 2;
  const fo_mb *ma = &d->mb[LA.mb], *mb2 = &d->mb[LB.mb];
  if (d->P->cip && (!mb_intra(ma) || !mb_intra(mb2))) return 2;
  int modes[2];
  const fo_loc *L[2] = {&LA, &LB};
  const fo_mb *M[2] = {ma, mb2};
  for (int i = 0; i < 2; i++) {
    const fo_mb *m = M[i];
    if (m->type != 1) { modes[i] = 2; continue; }
    if (m->t8 || !is8) { modes[i] = m->i4[(L[i]->yw / 4) * 4 + L[i]->xw / 4]; continue; }
    /* 4x4 neighbour of an 8x8 block: Intra4x4PredMode[luma8x8BlkIdxN * 4 + n], n = 1 (A), 2 (B) */
    int b8 = (L[i]->yw / 8) * 2 + L[i]->xw / 8, idx = b8 * 4 + (i == 0 ? 1 : 2);
    modes[i] = m->i4[BLK_Y[idx] * 4 + BLK_X[idx]];
  }
  return imin(modes[0], modes[1]);
}

/* mb_pred / sub_mb_pred of a B macroblock with CABAC (7.3.5.1-2) and its
   motion; *small: a sub-macroblock partition below 8x8 (or a direct one
   without direct_8x8_inference), which rules out transform_size_8x8_flag */
static int inter_mb_cabac_b(fo_ctx *c, fo_cab *k, int addr, int mb_type, int *small) {
  fo_dec *d = c->d;
  fo_mb *m = &d->mb[addr];
  int shape, pm[4] = {0, 0, 0, 0}, ssh[4] = {0, 0, 0, 0};
  if (mb_type == 0) { /* B_Direct_16x16 */
    m->direct8 = 15;
    m->d16 = 1;
    return direct_pred(c, addr, 0xffff);
  }
  if (mb_type <= 3) { shape = 0; pm[0] = mb_type; }
  else if (mb_type < 22) { shape = (mb_type & 1) ? 2 : 1; pm[0] = B_PART[mb_type][0]; pm[1] = B_PART[mb_type][1]; }
  else {
    shape = 3;
    for (int i = 0; i < 4; i++) {
      int v = cab_b_sub(k);
      pm[i] = B_SUB[v][0];
      ssh[i] = B_SUB[v][1];
      if (pm[i] == 0) {
        m->direct8 |= 1 << i;
        if (!d->S->direct8x8) *small = 1;
      } else if (ssh[i]) {
        *small = 1;
      }
    }
  }
  int nparts = shape == 0 ? 1 : (shape < 3 ? 2 : 4);
  int refs[2][4] = {{-1, -1, -1, -1}, {-1, -1, -1, -1}};
  /* ref_idx_l0 of the partitions, ref_idx_l1, then mvd_l0, mvd_l1 (7.3.5.1 / 7.3.5.2) */
  for (int l = 0; l < 2; l++) {
    int nref = l ? c->nlist1 : c->nlist;
    fo_pic *const *list = l ? c->list1 : c->list;
    for (int i = 0; i < nparts; i++) {
      if (!((pm[i] >> l) & 1)) continue;
      int x0 = shape == 2 || shape == 3 ? 8 * (i & 1) : 0, y0 = shape == 1 ? 8 * i : (shape == 3 ? 8 * (i >> 1) : 0);
      int pw = shape == 0 || shape == 1 ? 16 : 8, ph = shape == 0 || shape == 2 ? 16 : 8;
      int v = 0;
      if (g_enc) { g_enc->nref = 0; while (g_enc->nref < nref && list[g_enc->nref]) g_enc->nref++; }
      if (nref > 1 && cab_dec(k, 54 + ref_gt0_at(d, l, addr, x0 - 1, y0) + 2 * ref_gt0_at(d, l, addr, x0, y0 - 1))) {
        v = 1;
        if (cab_dec(k, 58)) {
          v = 2;
          while (cab_dec(k, 59)) { if (++v > 32) return fo_fail(d, FO_E_FORMAT, "ref_idx"); }
        }
      }
      if (v >= nref || !list[v]) return fo_fail(d, FO_E_DECODE, "ref_idx names no reference picture");
      refs[l][i] = v;
      for (int yy = y0 / 4; yy < (y0 + ph) / 4; yy++)
        for (int xx = x0 / 4; xx < (x0 + pw) / 4; xx++) m->refidx[l][yy * 4 + xx] = v;
    }
  }
  int mvd[2][4][4][2];
  for (int l = 0; l < 2; l++)
    for (int i = 0; i < nparts; i++) {
      if (!((pm[i] >> l) & 1)) continue;
      int nsub = shape < 3 ? 1 : (ssh[i] == 0 ? 1 : (ssh[i] == 3 ? 4 : 2));
      int x0 = shape == 2 || shape == 3 ? 8 * (i & 1) : 0, y0 = shape == 1 ? 8 * i : (shape == 3 ? 8 * (i >> 1) : 0);
      int pw = shape == 0 || shape == 1 ? 16 : 8, ph = shape == 0 || shape == 2 ? 16 : 8;
      if (shape == 3) { pw = ssh[i] == 0 || ssh[i] == 1 ? 8 : 4; ph = ssh[i] == 0 || ssh[i] == 2 ? 8 : 4; }
      for (int q = 0; q < nsub; q++) {
        int sx = x0, sy = y0;
        if (shape == 3) {
          if (ssh[i] == 1) sy += 4 * q;
          else if (ssh[i] == 2) sx += 4 * q;
          else if (ssh[i] == 3) { sx += 4 * (q & 1); sy += 4 * (q >> 1); }
        }
        for (int comp = 0; comp < 2; comp++)
          mvd[l][i][q][comp] = cab_mvd(k, comp ? 47 : 40,
                                       abs_mvd_at(d, l, addr, sx - 1, sy, comp) + abs_mvd_at(d, l, addr, sx, sy - 1, comp));
        for (int yy = sy / 4; yy < (sy + ph) / 4; yy++)
          for (int xx = sx / 4; xx < (sx + pw) / 4; xx++) {
            m->mvd[l][yy * 4 + xx][0] = mvd[l][i][q][0];
            m->mvd[l][yy * 4 + xx][1] = mvd[l][i][q][1];
          }
      }
    }
  /* motion: partitions in order, both lists of a (sub-)partition before the next */
  int done = 0;
  for (int i = 0; i < nparts; i++) {
    int nsub = 1, pw, ph, x0, y0;
    if (shape == 0) { pw = ph = 16; x0 = y0 = 0; }
    else if (shape == 1) { pw = 16; ph = 8; x0 = 0; y0 = 8 * i; }
    else if (shape == 2) { pw = 8; ph = 16; x0 = 8 * i; y0 = 0; }
    else {
      x0 = 8 * (i & 1);
      y0 = 8 * (i >> 1);
      nsub = ssh[i] == 0 ? 1 : (ssh[i] == 3 ? 4 : 2);
      pw = ssh[i] == 0 || ssh[i] == 1 ? 8 : 4;
      ph = ssh[i] == 0 || ssh[i] == 2 ? 8 : 4;
    }
    if (pm[i] == 0) { /* B_Direct_8x8 */
      int bm = 0x33 << ((y0 / 4) * 4 + x0 / 4);
      int rc = direct_pred(c, addr, bm);
      if (rc) return rc;
      done |= bm;
      continue;
    }
    for (int q = 0; q < nsub; q++) {
      int sx = x0, sy = y0;
      if (shape == 3) {
        if (ssh[i] == 1) sy += 4 * q;
        else if (ssh[i] == 2) sx += 4 * q;
        else if (ssh[i] == 3) { sx += 4 * (q & 1); sy += 4 * (q >> 1); }
      }
      for (int l = 0; l < 2; l++) {
        int use = (pm[i] >> l) & 1, vx = 0, vy = 0;
        if (use) {
          int px, py;
          mv_pred(d, l, addr, sx, sy, pw, ph, refs[l][i], done, &px, &py);
          vx = px + mvd[l][i][q][0];
          vy = py + mvd[l][i][q][1];
          if (vx < -32768 || vx > 32767 || vy < -32768 || vy > 32767) return fo_fail(d, FO_E_FORMAT, "mv range");
        }
        for (int yy = sy / 4; yy < (sy + ph) / 4; yy++)
          for (int xx = sx / 4; xx < (sx + pw) / 4; xx++) set_mv(c, m, l, yy * 4 + xx, use ? refs[l][i] : -1, vx, vy);
      }
      for (int yy = sy / 4; yy < (sy + ph) / 4; yy++)
        for (int xx = sx / 4; xx < (sx + pw) / 4; xx++) done |= 1 << (yy * 4 + xx);
    }
  }
  return 0;
}

/* macroblock_layer (7.3.5) with CABAC (not P_Skip) + reconstruction */
static int decode_mb_cabac(fo_ctx *c, fo_cab *k, int addr, int is_p, int *qp, int prev) {
  fo_dec *d = c->d;
  fo_mb *m = &d->mb[addr];
  fo_pic *pic = c->cur;
  int slice = m->slice;
  memset(m, 0, sizeof *m);
  m->slice = slice;
  for (int i = 0; i < 16; i++) {
    m->refidx[0][i] = m->refidx[1][i] = -1;
    m->refpic[0][i] = m->refpic[1][i] = -1;
    m->i4[i] = 2;
  }
  int mx = addr % d->mbw, my = addr / d->mbw;
  int A = nb_loc(d, addr, -1, 0, 16, 16).mb, B = nb_loc(d, addr, 0, -1, 16, 16).mb;
  const fo_mb *ma = A >= 0 ? &d->mb[A] : NULL, *mbb = B >= 0 ? &d->mb[B] : NULL;
  int mb_type, itype;
  if (c->is_b) {
    mb_type = cab_b_type(k, (ma && !ma->d16) + (mbb && !mbb->d16));
    itype = mb_type >= 23 ? mb_type - 23 : -1;
  } else if (is_p) {
    if (cab_dec(k, 14)) {
      itype = cab_i_type(k, 17, 0);
      mb_type = 5 + itype;
    } else {
      itype = -1;
      if (!cab_dec(k, 15)) mb_type = cab_dec(k, 16) ? 3 : 0;
      else mb_type = cab_dec(k, 17) ? 1 : 2;
    }
  } else {
    itype = cab_i_type(k, 0, (ma && ma->type != 1) + (mbb && mbb->type != 1));
    mb_type = itype;
  }
  (void)mb_type;
  if (itype == 25) { /* I_PCM: pcm_alignment_zero_bit, samples, engine restart (9.3.1.2) */
    m->type = 3;
    m->qp = *qp;
    k->b->bitpos = 0;
    for (int y = 0; y < 16; y++)
      for (int x = 0; x < 16; x++) pic->y[(int64_t)(my * 16 + y) * d->W + mx * 16 + x] = (uint8_t)fb_byte(k->b);
    for (int pl = 0; pl < 2; pl++)
      for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++)
          (pl ? pic->v : pic->u)[(int64_t)(my * 8 + y) * (d->W / 2) + mx * 8 + x] = (uint8_t)fb_byte(k->b);
    for (int i = 0; i < 16; i++) m->nz[i] = 16;
    for (int i = 0; i < 4; i++) m->nzc[0][i] = m->nzc[1][i] = 16;
    m->cbp = 0x2f;
    cab_start(k);
    return k->b->err ? fo_fail(d, FO_E_FORMAT, "I_PCM") : 0;
  }
  int cbp = 0, i16mode = 0, cmode = 0, sub[4] = {0, 0, 0, 0}, small = 0;
  if (itype == 0) { /* I_NxN */
    m->type = 1;
    if (d->P->t8mode) m->t8 = cab_dec(k, 399 + (ma && ma->t8) + (mbb && mbb->t8));
    int nb = m->t8 ? 4 : 16, prev_f[16], rem[16];
    for (int i = 0; i < nb; i++) {
      prev_f[i] = cab_dec(k, 68);
      rem[i] = prev_f[i] ? 0 : cab_fl3(k, 69);
    }
    for (int i = 0; i < nb; i++) {
      int x0 = m->t8 ? (i & 1) * 8 : BLK_X[i] * 4, y0 = m->t8 ? (i >> 1) * 8 : BLK_Y[i] * 4;
      int pm = intra_pred_mode_pred(d, addr, x0, y0, m->t8);
      int mode = prev_f[i] ? pm : (rem[i] < pm ? rem[i] : rem[i] + 1);
      if (m->t8) {
        int r = (y0 / 4) * 4 + x0 / 4;
        m->i4[r] = m->i4[r + 1] = m->i4[r + 4] = m->i4[r + 5] = mode;
      } else {
        m->i4[(y0 / 4) * 4 + x0 / 4] = mode;
      }
    }
  } else if (itype >= 1) { /* I_16x16 */
    m->type = 2;
    i16mode = (itype - 1) % 4;
    cbp = (((itype - 1) / 4) % 3) << 4 | (itype >= 13 ? 15 : 0);
  } else if (c->is_b) { /* Table 7-14 */
    m->type = 0;
    int rc = inter_mb_cabac_b(c, k, addr, mb_type, &small);
    if (rc) return rc;
  } else { /* inter, Table 7-13 */
    m->type = 0;
    int nparts = mb_type == 0 ? 1 : (mb_type <= 2 ? 2 : 4), refs[4] = {0, 0, 0, 0};
    if (mb_type == 3) {
      for (int i = 0; i < 4; i++) {
        if (cab_dec(k, 21)) sub[i] = 0;
        else if (!cab_dec(k, 22)) sub[i] = 1;
        else sub[i] = cab_dec(k, 23) ? 2 : 3;
        if (sub[i]) small = 1;
      }
    }
    int nref = c->nlist;
    /* ref_idx_l0 of every partition, then every mvd (7.3.5.1 / 7.3.5.2) */
    for (int i = 0; i < nparts; i++) {
      int x0 = (mb_type == 2 || mb_type == 3) ? 8 * (i & 1) : 0;
      int y0 = mb_type == 1 ? 8 * i : (mb_type == 3 ? 8 * (i >> 1) : 0);
      int pw = mb_type == 0 || mb_type == 1 ? 16 : 8, ph = mb_type == 0 || mb_type == 2 ? 16 : 8;
      if (nref > 1) {
        int v = 0;
        if (g_enc) { g_enc->nref = 0; while (g_enc->nref < nref && c->list[g_enc->nref]) g_enc->nref++; }
        if (cab_dec(k, 54 + ref_gt0_at(d, 0, addr, x0 - 1, y0) + 2 * ref_gt0_at(d, 0, addr, x0, y0 - 1))) {
          v = 1;
          if (cab_dec(k, 58)) {
            v = 2;
            while (cab_dec(k, 59)) { if (++v > 32) return fo_fail(d, FO_E_FORMAT, "ref_idx"); }
          }
        }
        refs[i] = v;
      }
      if (refs[i] >= nref || !c->list[refs[i]]) return fo_fail(d, FO_E_DECODE, "ref_idx names no reference picture");
      for (int yy = y0 / 4; yy < (y0 + ph) / 4; yy++)
        for (int xx = x0 / 4; xx < (x0 + pw) / 4; xx++) {
          m->refidx[0][yy * 4 + xx] = refs[i];
          m->refpic[0][yy * 4 + xx] = c->list[refs[i]]->id;
        }
    }
    int done = 0;
    for (int i = 0; i < nparts; i++) {
      int nsub = 1, pw, ph, x0, y0;
      if (mb_type == 0) { pw = 16; ph = 16; x0 = y0 = 0; }
      else if (mb_type == 1) { pw = 16; ph = 8; x0 = 0; y0 = 8 * i; }
      else if (mb_type == 2) { pw = 8; ph = 16; x0 = 8 * i; y0 = 0; }
      else {
        x0 = 8 * (i & 1);
        y0 = 8 * (i >> 1);
        nsub = sub[i] == 0 ? 1 : (sub[i] == 3 ? 4 : 2);
        pw = sub[i] == 0 || sub[i] == 1 ? 8 : 4;
        ph = sub[i] == 0 || sub[i] == 2 ? 8 : 4;
      }
      for (int s = 0; s < nsub; s++) {
        int sx = x0, sy = y0;
        if (mb_type == 3) {
          if (sub[i] == 1) sy += 4 * s;
          else if (sub[i] == 2) sx += 4 * s;
          else if (sub[i] == 3) { sx += 4 * (s & 1); sy += 4 * (s >> 1); }
        }
        int dmv[2];
        for (int comp = 0; comp < 2; comp++)
          dmv[comp] = cab_mvd(k, comp ? 47 : 40, abs_mvd_at(d, 0, addr, sx - 1, sy, comp) + abs_mvd_at(d, 0, addr, sx, sy - 1, comp));
        int px, py;
        mv_pred(d, 0, addr, sx, sy, pw, ph, refs[i], done, &px, &py);
        int vx = px + dmv[0], vy = py + dmv[1];
        if (vx < -32768 || vx > 32767 || vy < -32768 || vy > 32767) return fo_fail(d, FO_E_FORMAT, "mv range");
        for (int yy = sy / 4; yy < (sy + ph) / 4; yy++)
          for (int xx = sx / 4; xx < (sx + pw) / 4; xx++) {
            int blk = yy * 4 + xx;
            m->mv[0][blk][0] = vx;
            m->mv[0][blk][1] = vy;
            m->mvd[0][blk][0] = dmv[0];
            m->mvd[0][blk][1] = dmv[1];
            done |= 1 << blk;
          }
      }
    }
  }
  if (m->type == 1 || m->type == 2) { /* intra_chroma_pred_mode: TU cMax 3 */
    int inc = 0;
    for (int nb = 0; nb < 2; nb++) {
      const fo_mb *n = nb ? mbb : ma;
      inc += n && (n->type == 1 || n->type == 2) && n->cmode != 0;
    }
    if (cab_dec(k, 64 + inc)) {
      cmode = 1;
      if (cab_dec(k, 67)) {
        cmode = 2;
        if (cab_dec(k, 67)) cmode = 3;
      }
    }
    m->cmode = cmode;
  }
  if (m->type != 2) { /* coded_block_pattern: 4 luma bins (FL), chroma TU (9.3.3.1.1.4) */
    for (int b8 = 0; b8 < 4; b8++) {
      int bx = (b8 & 1) * 8, by = (b8 >> 1) * 8, cond[2];
      for (int nb = 0; nb < 2; nb++) {
        fo_loc L = nb_loc(d, addr, nb ? bx : bx - 1, nb ? by - 1 : by, 16, 16);
        int b8n = (L.yw / 8) * 2 + L.xw / 8;
        if (L.mb < 0) cond[nb] = 0;
        else if (L.mb == addr) cond[nb] = !((cbp >> b8n) & 1);
        else {
          const fo_mb *n = &d->mb[L.mb];
          cond[nb] = n->type == 3 ? 0 : (n->type == 4 ? 1 : !((n->cbp >> b8n) & 1));
        }
      }
      cbp |= cab_dec(k, 73 + cond[0] + 2 * cond[1]) << b8;
    }
    int ca[2], cb2[2];
    for (int nb = 0; nb < 2; nb++) {
      const fo_mb *n = nb ? mbb : ma;
      int cc = !n ? 0 : (n->type == 3 ? 2 : (n->type == 4 ? 0 : n->cbp >> 4));
      ca[nb] = cc != 0;
      cb2[nb] = cc == 2;
    }
    if (cab_dec(k, 77 + ca[0] + 2 * ca[1])) cbp |= (1 + cab_dec(k, 77 + 4 + cb2[0] + 2 * cb2[1])) << 4;
  }
  m->cbp = cbp;
  if (m->type == 0 && (cbp & 15) && d->P->t8mode && !small && !(m->d16 && !d->S->direct8x8))
    m->t8 = cab_dec(k, 399 + (ma && ma->t8) + (mbb && mbb->t8));
  if ((cbp & 15) || (cbp >> 4) || m->type == 2) { /* mb_qp_delta: U of the se mapping */
    const fo_mb *pm = prev >= 0 ? &d->mb[prev] : NULL;
    int inc = pm && pm->type != 4 && pm->type != 3 && (pm->type == 2 || pm->cbp != 0) && pm->qpd != 0;
    int kk = 0;
    if (cab_dec(k, 60 + inc)) {
      kk = 1;
      if (cab_dec(k, 62)) {
        kk = 2;
        while (cab_dec(k, 63)) { if (++kk > 104) return fo_fail(d, FO_E_FORMAT, "mb_qp_delta"); }
      }
    }
    int dq = (kk & 1) ? (kk + 1) / 2 : -(kk / 2);
    if (dq < -26 || dq > 25) return fo_fail(d, FO_E_FORMAT, "mb_qp_delta");
    m->qpd = dq;
    *qp = (*qp + dq + 52) % 52;
  }
  m->qp = *qp;
  /* residual (7.3.5.3): coefficients in raster per block */
  int coef[16][16], dcl[16], cdc[2][4], cac[2][4][16], coef8[4][64], lvl[64];
  memset(coef, 0, sizeof coef);
  memset(dcl, 0, sizeof dcl);
  memset(cdc, 0, sizeof cdc);
  memset(cac, 0, sizeof cac);
  memset(coef8, 0, sizeof coef8);
  int intra = m->type == 1 || m->type == 2;
  if (m->type == 2) {
    int inc = 0;
    for (int nb = 0; nb < 2; nb++) {
      const fo_mb *n = nb ? mbb : ma;
      inc += cbf_cond(d, intra, nb ? B : A, n && n->type == 2, 0) << nb;
    }
    int n = cab_residual(k, 0, inc, 16, lvl);
    if (n < 0) return fo_fail(d, FO_E_FORMAT, "Intra16x16DCLevel");
    for (int i = 0; i < 16; i++) dcl[ZZ4[i]] = lvl[i];
    if (n) m->cbf |= 1u;
  }
  for (int b8 = 0; b8 < 4; b8++) {
    if (!((cbp >> b8) & 1)) continue;
    int r0 = (b8 >> 1) * 8 + (b8 & 1) * 2; /* raster 4x4 index of the 8x8's top-left */
    if (m->t8) {
      int n = cab_residual(k, 5, 0, 64, lvl);
      if (n < 0) return fo_fail(d, FO_E_FORMAT, "LumaLevel8x8");
      for (int i = 0; i < 64; i++) coef8[b8][ZZ8[i]] = lvl[i];
      int rs[4] = {r0, r0 + 1, r0 + 4, r0 + 5};
      for (int j = 0; j < 4; j++) { m->nz[rs[j]] = n; m->cbf |= 1u << (1 + rs[j]); }
      continue;
    }
    for (int i4 = 0; i4 < 4; i4++) {
      int blk = b8 * 4 + i4, bx = BLK_X[blk], by = BLK_Y[blk], r = by * 4 + bx;
      int inc = cbf_luma_inc(d, addr, bx, by, intra);
      int n = m->type == 2 ? cab_residual(k, 1, inc, 15, lvl) : cab_residual(k, 2, inc, 16, lvl);
      if (n < 0) return fo_fail(d, FO_E_FORMAT, "LumaLevel4x4");
      if (m->type == 2) for (int i = 0; i < 15; i++) coef[r][ZZ4[i + 1]] = lvl[i];
      else for (int i = 0; i < 16; i++) coef[r][ZZ4[i]] = lvl[i];
      m->nz[r] = n;
      if (n) m->cbf |= 1u << (1 + r);
    }
  }
  if (cbp >> 4) {
    for (int pl = 0; pl < 2; pl++) {
      int n = cab_residual(k, 3, cbf_chroma_inc(d, addr, pl, 0, 1, intra), 4, lvl);
      if (n < 0) return fo_fail(d, FO_E_FORMAT, "ChromaDCLevel");
      for (int i = 0; i < 4; i++) cdc[pl][i] = lvl[i];
      if (n) m->cbf |= 1u << (17 + pl);
    }
  }
  if ((cbp >> 4) == 2) {
    for (int pl = 0; pl < 2; pl++)
      for (int b = 0; b < 4; b++) {
        int n = cab_residual(k, 4, cbf_chroma_inc(d, addr, pl, b, 0, intra), 15, lvl);
        if (n < 0) return fo_fail(d, FO_E_FORMAT, "ChromaACLevel");
        for (int i = 0; i < 15; i++) cac[pl][b][ZZ4[i + 1]] = lvl[i];
        m->nzc[pl][b] = n;
        if (n) m->cbf |= 1u << (19 + 4 * pl + b);
      }
  }
  if (k->b->err) return fo_fail(d, FO_E_FORMAT, "bitstream exhausted in residual");
  return recon_mb(c, addr, coef, dcl, cdc, cac, coef8, i16mode, cmode);
}

/* 7.3.4 slice_data() with CABAC; stop = the RBSP stop bit (EBSP bit index) */
static int slice_data_cabac(fo_ctx *c, fb_t *b, const fo_hdr *h, int is_p, int64_t stop) {
  fo_dec *d = c->d;
  while (b->bitpos && !g_enc)
    if (!fb_bit(b)) return fo_fail(d, FO_E_FORMAT, "cabac_alignment_one_bit");
  fo_cab k;
  k.b = b;
  cab_init(&k, !is_p, h->qp);
  cab_start(&k);
  int addr = h->first_mb, qp = h->qp, prev = -1;
  for (;;) {
    if (addr >= d->nmb) return fo_fail(d, FO_E_FORMAT, "macroblock address past the picture");
    if (d->mb[addr].slice >= 0) return fo_fail(d, FO_E_FORMAT, "macroblock decoded twice");
    d->mb[addr].slice = c->slice_no;
    int skip = 0;
    if (is_p) {
      int A = nb_loc(d, addr, -1, 0, 16, 16).mb, B = nb_loc(d, addr, 0, -1, 16, 16).mb;
      skip = cab_dec(&k, (c->is_b ? 24 : 11) + (A >= 0 && d->mb[A].type != 4) + (B >= 0 && d->mb[B].type != 4));
    }
    int rc = skip ? decode_mb(c, NULL, addr, 1, &qp, h) : decode_mb_cabac(c, &k, addr, is_p, &qp, prev);
    if (getenv("FO_TRACE"))
      fprintf(stderr, "oracle cabac mb %d type %d cbp %d qp %d t8 %d bits %lld\n", addr, d->mb[addr].type,
              d->mb[addr].cbp, qp, d->mb[addr].t8, (long long)fb_index(b, 0));
    if (rc) return rc;
    if (b->err && !g_enc) return fo_fail(d, FO_E_FORMAT, "bitstream exhausted");
    if (g_enc && addr == g_enc->last_mb) g_enc->last_mb = -1;
    prev = addr++;
    if (cab_term(&k)) break; /* end_of_slice_flag */
  }
  if (g_enc) return 0;
  if (fb_index(b, 0) != stop + 1) return fo_fail(d, FO_E_FORMAT, "CABAC slice data does not end at the stop bit");
  return 0;
}

/* ------------------------------------------------ picture-level driver */
static void mark_refs(fo_dec *d, fo_pic *cur, const fo_hdr *h, int is_idr) {
  int maxfn = fo_max_frame_num(d);
  if (is_idr) {
    for (int i = 0; i < d->ndpb; i++) d->dpb[i].ref = 0;
    if (h->lt_ref_flag) { cur->ref = 2; cur->lt_idx = 0; d->max_lt_idx = 0; }
    else { cur->ref = 1; d->max_lt_idx = -1; }
    dpb_compact(d); /* cur (last in the array) is kept */
    return;
  }
  int cur_to_long = 0;
  if (h->adaptive) {
    for (int k = 0; k < h->mmco_n; k++) {
      const int *op = h->mmco[k];
      int fn = h->frame_num;
      if (op[0] == 1 || op[0] == 3) {
        int picnum = fn - (op[1] + 1);
        fo_pic *p = dpb_find_short(d, picnum, fn);
        if (p) {
          if (op[0] == 1) p->ref = 0;
          else {
            for (int i = 0; i < d->ndpb; i++)
              if (d->dpb[i].ref == 2 && d->dpb[i].lt_idx == op[2]) d->dpb[i].ref = 0;
            p->ref = 2;
            p->lt_idx = op[2];
          }
        }
      } else if (op[0] == 2) {
        fo_pic *p = dpb_find_long(d, op[1]);
        if (p) p->ref = 0;
      } else if (op[0] == 4) {
        d->max_lt_idx = op[1] - 1;
        for (int i = 0; i < d->ndpb; i++)
          if (d->dpb[i].ref == 2 && d->dpb[i].lt_idx > d->max_lt_idx) d->dpb[i].ref = 0;
      } else if (op[0] == 5) {
        for (int i = 0; i < d->ndpb; i++) d->dpb[i].ref = 0;
        d->max_lt_idx = -1;
        cur->frame_num = 0; /* 8.2.1: the picture is treated as frame_num 0 afterwards */
      } else if (op[0] == 6) {
        for (int i = 0; i < d->ndpb; i++)
          if (d->dpb[i].ref == 2 && d->dpb[i].lt_idx == op[2]) d->dpb[i].ref = 0;
        cur->ref = 2;
        cur->lt_idx = op[2];
        cur_to_long = 1;
      }
    }
  } else {
    /* 8.2.5.3 sliding window: at Max(max_num_ref_frames, 1) references, the
       short-term one with the smallest FrameNumWrap goes */
    int ns = 0, nl = 0;
    for (int i = 0; i < d->ndpb; i++) { ns += d->dpb[i].ref == 1; nl += d->dpb[i].ref == 2; }
    int maxr = d->S->max_num_ref_frames > 1 ? d->S->max_num_ref_frames : 1;
    if (ns + nl >= maxr && ns > 0) {
      fo_pic *o = NULL;
      int ow = 0;
      for (int i = 0; i < d->ndpb; i++) {
        fo_pic *p = &d->dpb[i];
        if (p->ref != 1) continue;
        int w = p->frame_num > h->frame_num ? p->frame_num - maxfn : p->frame_num;
        if (!o || w < ow) { o = p; ow = w; }
      }
      o->ref = 0;
    }
  }
  if (!cur_to_long) cur->ref = 1;
  dpb_compact(d);
}

static void out_frame(const fo_dec *d, const fo_pic *p, uint8_t *o) {
  int dw = d->W - d->S->crop_l - d->S->crop_r, dh = d->H - d->S->crop_t - d->S->crop_b;
  for (int j = 0; j < dh; j++)
    memcpy(o + (int64_t)j * dw, p->y + (int64_t)(j + d->S->crop_t) * d->W + d->S->crop_l, (size_t)dw);
  uint8_t *ouv = o + (int64_t)dw * dh;
  for (int j = 0; j < dh / 2; j++)
    for (int i = 0; i < dw / 2; i++) {
      int64_t s = (int64_t)(j + d->S->crop_t / 2) * (d->W / 2) + i + d->S->crop_l / 2;
      ouv[(int64_t)j * dw + 2 * i] = p->u[s];
      ouv[(int64_t)j * dw + 2 * i + 1] = p->v[s];
    }
}

/* Display size of an SPS NAL unit (header byte included).  0 or < 0. */
int fo_dims(const uint8_t *sps, int64_t sn, int *w, int *h) {
  fo_sps tab[32];
  char err[256] = {0};
  memset(tab, 0, sizeof tab);
  int rc = parse_sps(sps, sn, tab, err);
  if (rc) return rc;
  for (int i = 0; i < 32; i++)
    if (tab[i].valid) {
      *w = tab[i].mbw * 16 - tab[i].crop_l - tab[i].crop_r;
      *h = tab[i].mbh * 16 - tab[i].crop_t - tab[i].crop_b;
      return 0;
    }
  return FO_E_FORMAT;
}

/* Decode n AVCC samples (length-prefixed NAL units of nls bytes) with the
 * avcC SPS / PPS; write every frame as display-size NV12 (pitch = width) into
 * out.  flags bit 0: skip the deblocking filter (pre-filter pictures, for
 * staged device bring-up).  Returns 0 or < 0 with *bad_frame and err set. */
/* CABAC synthesis output (fo_cabac_convert) */
typedef struct {
  uint64_t seed;
  int t8;                  /* also switch transform_8x8_mode_flag on */
  uint8_t *out;            /* samples, AVCC (nls-byte lengths) */
  int64_t cap, used;
  int64_t *sizes;          /* per sample */
  uint8_t *pps_out;        /* the converted PPS NAL */
  int64_t pps_len;
} fo_conv;

/* bit writer for the converted headers */
typedef struct { uint8_t *p; int64_t n; } fo_bw;
static void bw_bit(fo_bw *w, int b) {
  if (b) w->p[w->n >> 3] |= (uint8_t)(0x80 >> (w->n & 7));
  w->n++;
}
static void bw_ue(fo_bw *w, uint32_t v) {
  int len = 0;
  while ((v + 1) >> (len + 1)) len++;
  for (int i = 0; i < len; i++) bw_bit(w, 0);
  for (int i = len; i >= 0; i--) bw_bit(w, ((v + 1) >> i) & 1);
}
static void bw_se(fo_bw *w, int v) { bw_ue(w, v > 0 ? (uint32_t)(2 * v - 1) : (uint32_t)(-2 * v)); }
/* RBSP bytes -> NAL payload with emulation_prevention_three_bytes */
static int64_t escape_rbsp(const uint8_t *r, int64_t n, uint8_t *o) {
  int64_t m = 0;
  int zeros = 0;
  for (int64_t i = 0; i < n; i++) {
    if (zeros >= 2 && r[i] <= 3) { o[m++] = 3; zeros = 0; }
    o[m++] = r[i];
    zeros = r[i] == 0 ? zeros + 1 : 0;
  }
  return m;
}
static int64_t unescape_nal(const uint8_t *p, int64_t n, uint8_t *o) {
  int64_t m = 0;
  int zeros = 0;
  for (int64_t i = 0; i < n; i++) {
    if (zeros >= 2 && p[i] == 3) { zeros = 0; continue; }
    o[m++] = p[i];
    zeros = p[i] == 0 ? zeros + 1 : 0;
  }
  return m;
}

static int fo_run(const uint8_t *sps, int64_t sn, const uint8_t *pps, int64_t pn, int nls,
                  const uint8_t *data, const int64_t *offsets, const int64_t *sizes, int64_t n,
                  int flags, uint8_t *out, int64_t *bad_frame, char *err, fo_conv *cv);

int fo_decode(const uint8_t *sps, int64_t sn, const uint8_t *pps, int64_t pn, int nls,
              const uint8_t *data, const int64_t *offsets, const int64_t *sizes, int64_t n,
              int flags, uint8_t *out, int64_t *bad_frame, char *err) {
  return fo_run(sps, sn, pps, pn, nls, data, offsets, sizes, n, flags, out, bad_frame, err, NULL);
}

/* TEST INFRASTRUCTURE: re-code a CAVLC stream's slice data as CABAC.  Every
 * slice keeps its header (cabac_init_idc 0 inserted for P / B slices) and
 * its macroblock range; the macroblock layer is generated by the decoder
 * itself in synthesis mode (g_enc: seeded random syntax, arithmetic-coded as
 * 9.3.4 prescribes), so the stream exercises every CABAC syntax element the
 * decoder parses.  The PPS gets entropy_coding_mode_flag 1 (and, with t8,
 * transform_8x8_mode_flag 1).  out receives the samples (AVCC, nls-byte
 * lengths), out_sizes their sizes, pps_out the PPS NAL; frames (may be
 * null-sized: flags bit 1) the pictures the synthesis decoded.  0 or < 0. */
int fo_cabac_convert(const uint8_t *sps, int64_t sn, const uint8_t *pps, int64_t pn, int nls,
                     const uint8_t *data, const int64_t *offsets, const int64_t *sizes, int64_t n,
                     uint64_t seed, int t8, uint8_t *out, int64_t out_cap, int64_t *out_sizes,
                     uint8_t *pps_out, int64_t *pps_len, uint8_t *frames, int64_t *bad_frame, char *err) {
  fo_conv cv;
  memset(&cv, 0, sizeof cv);
  cv.seed = seed;
  cv.t8 = t8;
  cv.out = out;
  cv.cap = out_cap;
  cv.sizes = out_sizes;
  cv.pps_out = pps_out;
  int rc = fo_run(sps, sn, pps, pn, nls, data, offsets, sizes, n, 0, frames, bad_frame, err, &cv);
  *pps_len = cv.pps_len;
  return rc;
}

static int fo_run(const uint8_t *sps, int64_t sn, const uint8_t *pps, int64_t pn, int nls,
                  const uint8_t *data, const int64_t *offsets, const int64_t *sizes, int64_t n,
                  int flags, uint8_t *out, int64_t *bad_frame, char *err, fo_conv *cv) {
  fo_dec *d = (fo_dec *)calloc(1, sizeof *d);
  if (!d) return FO_E_FORMAT;
  char ebuf[256] = {0};
  d->err = err ? err : ebuf;
  d->err[0] = 0;
  d->flags = flags;
  d->max_lt_idx = -1;
  *bad_frame = -1;
  int rc = parse_sps(sps, sn, d->sps, d->err);
  if (!rc) rc = parse_pps(pps, pn, d->pps, d->sps, d->err);
  if (!rc && cv) { /* the converted PPS, written from the parsed fields */
    for (int id = 0; id < 256; id++) {
      fo_pps *P = &d->pps[id];
      if (!P->valid) continue;
      if (P->pic_scaling) { rc = fo_fail(d, FO_E_UNSUPPORTED, "synthesis: PPS scaling matrices"); break; }
      P->cabac = 1;
      if (cv->t8) P->t8mode = 1;
      uint8_t rb[64];
      memset(rb, 0, sizeof rb);
      fo_bw w = {rb, 0};
      bw_ue(&w, (uint32_t)id);
      bw_ue(&w, (uint32_t)P->sps_id);
      bw_bit(&w, 1);
      bw_bit(&w, P->bfpo);
      bw_ue(&w, 0);
      bw_ue(&w, (uint32_t)(P->num_ref_l0 - 1));
      bw_ue(&w, (uint32_t)(P->num_ref_l1 - 1));
      bw_bit(&w, P->weighted_pred);
      bw_bit(&w, (P->weighted_bipred >> 1) & 1);
      bw_bit(&w, P->weighted_bipred & 1);
      bw_se(&w, P->pic_init_qp - 26);
      bw_se(&w, 0);
      bw_se(&w, P->cqp_off);
      bw_bit(&w, P->deblock_ctrl);
      bw_bit(&w, P->cip);
      bw_bit(&w, 0);
      if (P->t8mode || P->cqp_off2 != P->cqp_off) {
        bw_bit(&w, P->t8mode);
        bw_bit(&w, 0);
        bw_se(&w, P->cqp_off2);
      }
      bw_bit(&w, 1);
      cv->pps_out[0] = pps[0];
      cv->pps_len = 1 + escape_rbsp(rb, (w.n + 7) >> 3, cv->pps_out + 1);
      break;
    }
  }
  int64_t f = 0;
  fo_pic cur;
  memset(&cur, 0, sizeof cur);
  for (int i = 0; i < 32 && !rc; i++)
    if (d->sps[i].valid) {
      d->mbw = d->sps[i].mbw;
      d->mbh = d->sps[i].mbh;
      break;
    }
  d->W = d->mbw * 16;
  d->H = d->mbh * 16;
  d->nmb = d->mbw * d->mbh;
  if (!rc) {
    d->mb = (fo_mb *)calloc((size_t)d->nmb, sizeof(fo_mb));
    if (!d->mb) rc = FO_E_FORMAT;
  }
  int64_t out_size = -1;
  for (f = 0; f < n && !rc; f++) {
    cur.y = (uint8_t *)calloc((size_t)d->W * d->H, 1);
    cur.u = (uint8_t *)calloc((size_t)d->W * d->H / 4, 1);
    cur.v = (uint8_t *)calloc((size_t)d->W * d->H / 4, 1);
    cur.id = ++d->next_id;
    cur.ref = 0;
    for (int a = 0; a < d->nmb; a++) d->mb[a].slice = -1;
    const uint8_t *s = data + offsets[f];
    int64_t pos = 0, end = sizes[f];
    int nslice = 0, is_idr = 0, any_ref = 0;
    fo_hdr h, h0;
    memset(&h0, 0, sizeof h0);
    while (pos + nls <= end && !rc) {
      uint32_t L = 0;
      for (int i = 0; i < nls; i++) L = (L << 8) | s[pos + i];
      pos += nls;
      if (L == 0 || pos + L > end) { rc = fo_fail(d, FO_E_FORMAT, "bad NAL length"); break; }
      int t = s[pos] & 31;
      if ((t == 1 || t == 5) && cv) {
        /* synthesis: source slice as RBSP, its macroblock range from the next slice's first_mb */
        uint8_t *rb = (uint8_t *)malloc((size_t)L + 64), *nb = (uint8_t *)calloc((size_t)L * 4 + 4096, 1);
        uint8_t *eb = (uint8_t *)malloc((size_t)L * 8 + 8192);
        int64_t rn = unescape_nal(s + pos, L, rb);
        memset(rb + rn, 0, 64);
        int last = d->nmb - 1;
        for (int64_t q = pos + L; q + nls <= end; ) {
          uint32_t L2 = 0;
          for (int i = 0; i < nls; i++) L2 = (L2 << 8) | s[q + i];
          q += nls;
          int t2 = s[q] & 31;
          if (t2 == 1 || t2 == 5) {
            fb_t hb;
            fb_init(&hb, s + q + 1, L2 - 1);
            last = (int)fb_ue(&hb) - 1;
            break;
          }
          q += L2;
        }
        fo_enc e;
        memset(&e, 0, sizeof e);
        e.out = (uint8_t *)calloc((size_t)L * 4 + 65536 + (size_t)d->nmb * 1024, 1);
        e.cap = (int64_t)L * 4 + 65536 + (int64_t)d->nmb * 1024;
        e.rng = cv->seed * 0x9E3779B97F4A7C15ull + (uint64_t)f * 1000003u + (uint64_t)nslice * 7919u + 1;
        e.last_mb = last;
        g_enc = &e;
        int idr = 0;
        rc = decode_slice(d, &cur, rb, rn, nslice, &idr, &h);
        g_enc = NULL;
        if (!rc && (e.overflow || e.last_mb != -1)) rc = fo_fail(d, FO_E_DECODE, "synthesis overflow / slice end");
        if (!rc) {
          /* header bits [0, pos_qp) + cabac_init_idc + [pos_qp, pos_data) + alignment ones + CABAC data */
          fo_bw w = {nb, 0};
          const uint8_t *hdr = rb + 1;
          for (int64_t i = 0; i < d->enc_pos_qp; i++) bw_bit(&w, (hdr[i >> 3] >> (7 - (i & 7))) & 1);
          if (h.slice_type != 2) bw_ue(&w, 0);
          for (int64_t i = d->enc_pos_qp; i < d->enc_pos_data; i++) bw_bit(&w, (hdr[i >> 3] >> (7 - (i & 7))) & 1);
          while (w.n & 7) bw_bit(&w, 1);
          for (int64_t i = 0; i < e.nbits; i++) bw_bit(&w, (e.out[i >> 3] >> (7 - (i & 7))) & 1);
          int64_t nbytes = (w.n + 7) >> 3;
          eb[0] = s[pos];
          int64_t en = 1 + escape_rbsp(nb, nbytes, eb + 1);
          if (cv->used + nls + en > cv->cap) rc = fo_fail(d, FO_E_DECODE, "synthesis output full");
          else {
            for (int i = 0; i < nls; i++) cv->out[cv->used++] = (uint8_t)(en >> (8 * (nls - 1 - i)));
            memcpy(cv->out + cv->used, eb, (size_t)en);
            cv->used += en;
            cv->sizes[f] += nls + en;
          }
        }
        free(e.out);
        free(rb);
        free(nb);
        free(eb);
        if (!rc) {
          if (nslice == 0) { h0 = h; is_idr = idr; }
          any_ref |= h.nal_ref_idc != 0;
          nslice++;
        }
      } else if (t == 1 || t == 5) {
        int idr = 0;
        rc = decode_slice(d, &cur, s + pos, L, nslice, &idr, &h);
        if (!rc) {
          if (nslice == 0) { h0 = h; is_idr = idr; }
          any_ref |= h.nal_ref_idc != 0;
          nslice++;
        }
      } else if (t == 7) {
        rc = parse_sps(s + pos, L, d->sps, d->err);
      } else if (t == 8) {
        if (cv) rc = fo_fail(d, FO_E_UNSUPPORTED, "synthesis: in-band PPS");
        else rc = parse_pps(s + pos, L, d->pps, d->sps, d->err);
      } else if (t >= 2 && t <= 4) {
        rc = fo_fail(d, FO_E_UNSUPPORTED, "data partitioning");
      }
      pos += L;
    }
    if (!rc && nslice == 0) rc = fo_fail(d, FO_E_FORMAT, "access unit without a slice");
    for (int a = 0; a < d->nmb && !rc; a++)
      if (d->mb[a].slice < 0) rc = fo_fail(d, FO_E_DECODE, "macroblock not covered by any slice");
    if (rc) break;
    d->nslices = nslice;
    if (!(flags & 1)) deblock_picture(d, &cur);
    /* the picture's motion, for the direct prediction of later B pictures */
    for (int l = 0; l < 2; l++) {
      cur.mref[l] = (int8_t *)malloc((size_t)d->nmb * 16);
      cur.mmv[l] = (int16_t *)malloc((size_t)d->nmb * 32 * sizeof(int16_t));
      cur.mpic[l] = (int32_t *)malloc((size_t)d->nmb * 16 * sizeof(int32_t));
      if (!cur.mref[l] || !cur.mmv[l] || !cur.mpic[l]) { rc = fo_fail(d, FO_E_DECODE, "out of memory"); break; }
      for (int a = 0; a < d->nmb; a++)
        for (int k = 0; k < 16; k++) {
          const fo_mb *m = &d->mb[a];
          int intra = mb_intra(m);
          cur.mref[l][a * 16 + k] = (int8_t)(intra ? -1 : m->refidx[l][k]);
          cur.mpic[l][a * 16 + k] = intra ? -1 : m->refpic[l][k];
          cur.mmv[l][(a * 16 + k) * 2] = (int16_t)m->mv[l][k][0];
          cur.mmv[l][(a * 16 + k) * 2 + 1] = (int16_t)m->mv[l][k][1];
        }
    }
    if (rc) break;
    if (getenv("FO_MVDUMP")) { /* debugging aid: per-block motion, for cross-checks with the writer */
      FILE *df = fopen(getenv("FO_MVDUMP"), "a");
      for (int a = 0; df && a < d->nmb; a++)
        for (int k = 0; k < 16; k++)
          for (int l = 0; l < 2; l++)
            fprintf(df, "%lld %d %d %d %d %d %d\n", (long long)f, a, k, l, d->mb[a].refidx[l][k],
                    d->mb[a].refidx[l][k] >= 0 ? d->mb[a].mv[l][k][0] : 0, d->mb[a].refidx[l][k] >= 0 ? d->mb[a].mv[l][k][1] : 0);
      if (df) fclose(df);
    }
    poc_advance(d, &h0);
    if (d->prev_mmco5) cur.poc = 0; /* 8.2.1: tempPicOrderCnt subtracted */
    int dw = d->W - d->S->crop_l - d->S->crop_r, dh = d->H - d->S->crop_t - d->S->crop_b;
    out_size = (int64_t)dw * dh * 3 / 2;
    out_frame(d, &cur, out + f * out_size);
    if (any_ref) {
      cur.frame_num = h0.frame_num;
      if (d->ndpb >= 17) { rc = fo_fail(d, FO_E_DECODE, "DPB overflow"); break; }
      d->dpb[d->ndpb] = cur;
      mark_refs(d, &d->dpb[d->ndpb++], &h0, is_idr);
      /* mark_refs compacts: the current picture is kept (ref != 0) */
    } else {
      pic_free(&cur);
    }
    memset(&cur, 0, sizeof cur);
  }
  if (rc) {
    *bad_frame = f < n ? f : n - 1;
    pic_free(&cur);
  }
  for (int i = 0; i < d->ndpb; i++) pic_free(&d->dpb[i]);
  free(d->mb);
  free(d);
  return rc;
}
