/*
 * transcode_oracle.c — CPU restatement of the 360p upload transcode
 * (the reference's _compress_video_for_upload,
 * src/analyzer/content_analyzer.py:167-236, runs `ffmpeg -vf scale=-2:360
 * -c:v libx264 -crf 28`).  Used ONLY as a checker.
 *
 * TEST INFRASTRUCTURE.  Only tests/ may load this (through liboracle.so);
 * the product (libvtseg.so, its transcode.hip) never links or calls it.
 * Plain scalar C, written from the definition in DESIGN.md §11, not from the
 * device code.
 *
 * Parity: x264 is absent from this image and the GPU pool, and its output is
 * not a function anything here could restate, so byte parity with the
 * reference's compressed file is UNPINNED.  What is pinned: the output size
 * rule (ffmpeg's scale=-2:H: w = 2 * av_rescale(H, W, 2 * srcH), round to
 * nearest), and — by this oracle — every output byte of the device encoder,
 * and a decode of the output by the oracle decoder equals the encoder's own
 * reconstruction.
 *
 * The encoder:
 *   - area downscale of the display-size NV12 frame to (sw, sh), per axis
 *     weights = overlap of source and destination pixel footprints (gcd
 *     reduced), rounded (sum + T/2) / T, then max(1, .) so that I_PCM data
 *     never holds a zero byte; coded size 16-aligned, edge rows/columns
 *     replicated;
 *   - IDR at frame 0, when the GOP reaches `keyint` frames and (opt-in) at
 *     every scene cut (score > threshold): every macroblock I_PCM;
 *   - P pictures, one slice per macroblock row: per macroblock the integer
 *     luma motion (dx, dy), |dx|,|dy| <= R, of least luma SAD against the
 *     previous reconstructed picture (samples outside it edge-clamped as the
 *     decoder's 8.4.2.2.1 reads them; (0,0)
 *     first, then raster order; first minimum wins); inter (P_L0_16x16 or
 *     P_Skip, no residual) if luma+chroma SAD of its prediction (chroma by
 *     8.4.2.2.2) <= T_mb, else I_PCM.
 *   - residual coding (qp >= 1, the default since round 3): the best motion
 *     is always tried with a quantised residual at QP qp (flat scaling,
 *     chroma_qp_index_offset 0): per 4x4 block the forward core transform
 *     W = Cf X Cf^T, levels sign(W) min(2047, (|W| MF + f) >> qbits),
 *     qbits = 15 + qp / 6, f = 2^qbits / 6, MF by position class; chroma DC
 *     through the 2x2 Hadamard at (qbits + 1, 2f); the reconstruction is the
 *     decoder's (8.5.12 scaling + inverse transform, chroma DC 8.5.11).  A
 *     macroblock stays inter when an upper bound of its residual's CAVLC bits
 *     (every code exact but coeff_token, taken as the longest over the nC
 *     classes) is <= 3072 (the I_PCM payload), else it is I_PCM; P_Skip when
 *     its motion is (0, 0) and nothing is coded.  cbp, mb_qp_delta 0 and
 *     residual_block_cavlc with nC from the left macroblock (the one above is
 *     another slice) as 7.3.5.3 / 9.2.1 write them.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------ sizes */

/* ffmpeg scale=-2:sh: w = av_rescale(sh, W, 2 * H) * 2 (round to nearest). */
int or_small_width(int W, int H, int sh) {
  int64_t a = (int64_t)sh * W, c = 2 * (int64_t)H;
  return (int)((a + c / 2) / c) * 2;
}

static int64_t gcd64(int64_t a, int64_t b) {
  while (b) { int64_t t = a % b; a = b; b = t; }
  return a;
}

/* area weight of source pixel i for destination pixel o (n source -> m dest),
 * divided by g = gcd(n, m) */
static int64_t area_w(int64_t o, int64_t i, int64_t n, int64_t m) {
  int64_t lo = o * n > i * m ? o * n : i * m;
  int64_t hi = (o + 1) * n < (i + 1) * m ? (o + 1) * n : (i + 1) * m;
  return hi > lo ? (hi - lo) / gcd64(n, m) : 0;
}

/* one plane: src (n_x x n_y, pitch sp, element step es) -> dst (coded cx x cy,
 * display m_x x m_y, pitch dp, step ds) */
static void area_plane(const uint8_t *src, int sp, int es, int nx, int ny, uint8_t *dst, int dp,
                       int ds, int mx, int my, int cx, int cy) {
  int64_t tx = nx / gcd64(nx, mx), ty = ny / gcd64(ny, my);
  for (int y = 0; y < cy; y++) {
    int oy = y < my ? y : my - 1;
    for (int x = 0; x < cx; x++) {
      int ox = x < mx ? x : mx - 1;
      int64_t sum = 0;
      for (int j = (int)((int64_t)oy * ny / my); j < ny && (int64_t)j * my < (int64_t)(oy + 1) * ny; j++) {
        int64_t wy = area_w(oy, j, ny, my);
        for (int i = (int)((int64_t)ox * nx / mx); i < nx && (int64_t)i * mx < (int64_t)(ox + 1) * nx; i++)
          sum += wy * area_w(ox, i, nx, mx) * src[(int64_t)j * sp + (int64_t)i * es];
      }
      int64_t T = tx * ty, v = (sum + T / 2) / T;
      dst[(int64_t)y * dp + (int64_t)x * ds] = (uint8_t)(v < 1 ? 1 : v);
    }
  }
}

/* Display-size NV12 (W x H, pitch W) -> coded NV12 (cw x ch, pitch cw, UV at
 * cw * ch) of display size (sw, sh). */
int or_downscale_nv12(const uint8_t *src, int W, int H, uint8_t *dst, int sw, int sh) {
  int cw = (sw + 15) & ~15, ch = (sh + 15) & ~15;
  if (W < 2 || H < 2 || (W & 1) || (H & 1) || sw < 2 || sh < 2 || (sw & 1) || (sh & 1)) return -1;
  area_plane(src, W, 1, W, H, dst, cw, 1, sw, sh, cw, ch);
  const uint8_t *suv = src + (int64_t)W * H;
  uint8_t *duv = dst + (int64_t)cw * ch;
  area_plane(suv, W, 2, W / 2, H / 2, duv, cw, 2, sw / 2, sh / 2, cw / 2, ch / 2);
  area_plane(suv + 1, W, 2, W / 2, H / 2, duv + 1, cw, 2, sw / 2, sh / 2, cw / 2, ch / 2);
  return 0;
}

/* ------------------------------------------------------ bit writer */

typedef struct {
  uint8_t *rbsp;
  int64_t n, cap;
  uint32_t cur;
  int nb;
} or_bw;

static void bw_bit(or_bw *b, uint32_t v) {
  b->cur = (b->cur << 1) | (v & 1u);
  if (++b->nb == 8) {
    if (b->n < b->cap) b->rbsp[b->n] = (uint8_t)b->cur;
    b->n++;
    b->cur = 0;
    b->nb = 0;
  }
}
static void bw_u(or_bw *b, int n, uint32_t v) {
  for (int i = n - 1; i >= 0; i--) bw_bit(b, (v >> i) & 1u);
}
static void bw_ue(or_bw *b, uint32_t v) {
  uint64_t x = (uint64_t)v + 1;
  int len = 0;
  while ((x >> len) > 1) len++;
  for (int i = 0; i < len; i++) bw_bit(b, 0);
  for (int i = len; i >= 0; i--) bw_bit(b, (uint32_t)(x >> i) & 1u);
}
static void bw_se(or_bw *b, int v) { bw_ue(b, v > 0 ? (uint32_t)(2 * v - 1) : (uint32_t)(-2 * v)); }
static void bw_align(or_bw *b) { while (b->nb) bw_bit(b, 0); }
static void bw_trailing(or_bw *b) { bw_bit(b, 1); bw_align(b); }

/* [4-byte length][header][EBSP of rbsp] appended at out[*pos]; returns 0 or -2 */
static int put_nal(uint8_t *out, int64_t cap, int64_t *pos, uint8_t header, const uint8_t *rbsp,
                   int64_t n) {
  int64_t p = *pos + 4, start = p;
  if (p >= cap) return -2;
  out[p++] = header;
  int zeros = 0;
  for (int64_t i = 0; i < n; i++) {
    uint8_t v = rbsp[i];
    if (zeros >= 2 && v <= 3) {
      if (p >= cap) return -2;
      out[p++] = 3;
      zeros = 0;
    }
    if (p >= cap) return -2;
    out[p++] = v;
    zeros = v == 0 ? zeros + 1 : 0;
  }
  int64_t len = p - start;
  out[*pos] = (uint8_t)(len >> 24);
  out[*pos + 1] = (uint8_t)(len >> 16);
  out[*pos + 2] = (uint8_t)(len >> 8);
  out[*pos + 3] = (uint8_t)len;
  *pos = p;
  return 0;
}

/* ------------------------------------------------- parameter sets */

/* Table A-1: smallest level admitting MaxFS / MaxMBPS (levels 3 .. 5.2). */
int or_pick_level(int mbs, double mbps) {
  static const struct { int idc, fs; double mbps; } t[] = {
      {30, 1620, 40500}, {31, 3600, 108000}, {32, 5120, 216000}, {40, 8192, 245760},
      {42, 8704, 522240}, {50, 22080, 589824}, {51, 36864, 983040}, {52, 36864, 2073600}};
  for (int i = 0; i < 8; i++)
    if (mbs <= t[i].fs && mbps <= t[i].mbps) return t[i].idc;
  return 52;
}

/* SPS / PPS NAL units (header byte + EBSP, no length prefix) of the output. */
int or_sps_pps(int mbw, int mbh, int crop_r, int crop_b, int level, uint8_t *sps, int64_t *sn,
               uint8_t *pps, int64_t *pn) {
  uint8_t tmp[64];
  or_bw b = {tmp, 0, sizeof tmp, 0, 0};
  bw_u(&b, 8, 66);      /* profile_idc Baseline */
  bw_u(&b, 8, 0xC0);    /* constraint_set0/1: Constrained Baseline */
  bw_u(&b, 8, (uint32_t)level);
  bw_ue(&b, 0);         /* sps id */
  bw_ue(&b, 12);        /* log2_max_frame_num_minus4: 16-bit frame_num */
  bw_ue(&b, 2);         /* pic_order_cnt_type 2 */
  bw_ue(&b, 1);         /* max_num_ref_frames */
  bw_u(&b, 1, 0);       /* gaps_in_frame_num_value_allowed_flag */
  bw_ue(&b, (uint32_t)(mbw - 1));
  bw_ue(&b, (uint32_t)(mbh - 1));
  bw_u(&b, 1, 1);       /* frame_mbs_only_flag */
  bw_u(&b, 1, 1);       /* direct_8x8_inference_flag */
  if (crop_r || crop_b) {
    bw_u(&b, 1, 1);
    bw_ue(&b, 0);
    bw_ue(&b, (uint32_t)(crop_r / 2));
    bw_ue(&b, 0);
    bw_ue(&b, (uint32_t)(crop_b / 2));
  } else {
    bw_u(&b, 1, 0);
  }
  bw_u(&b, 1, 0);       /* vui_parameters_present_flag */
  bw_trailing(&b);
  uint8_t buf[80];
  int64_t pos = 0;
  if (put_nal(buf, sizeof buf, &pos, 0x67, tmp, b.n)) return -2;
  *sn = pos - 4;
  memcpy(sps, buf + 4, (size_t)*sn);
  or_bw p = {tmp, 0, sizeof tmp, 0, 0};
  bw_ue(&p, 0);         /* pps id */
  bw_ue(&p, 0);         /* sps id */
  bw_u(&p, 1, 0);       /* CAVLC */
  bw_u(&p, 1, 0);       /* bottom_field_pic_order_in_frame_present_flag */
  bw_ue(&p, 0);         /* num_slice_groups_minus1 */
  bw_ue(&p, 0);         /* num_ref_idx_l0_default_active_minus1 */
  bw_ue(&p, 0);         /* num_ref_idx_l1_default_active_minus1 */
  bw_u(&p, 1, 0);       /* weighted_pred_flag */
  bw_u(&p, 2, 0);       /* weighted_bipred_idc */
  bw_se(&p, 0);         /* pic_init_qp_minus26 */
  bw_se(&p, 0);         /* pic_init_qs_minus26 */
  bw_se(&p, 0);         /* chroma_qp_index_offset */
  bw_u(&p, 1, 1);       /* deblocking_filter_control_present_flag */
  bw_u(&p, 1, 0);       /* constrained_intra_pred_flag */
  bw_u(&p, 1, 0);       /* redundant_pic_cnt_present_flag */
  bw_trailing(&p);
  pos = 0;
  if (put_nal(buf, sizeof buf, &pos, 0x68, tmp, p.n)) return -2;
  *pn = pos - 4;
  memcpy(pps, buf + 4, (size_t)*pn);
  return 0;
}

/* ------------------------------------------------------- encoder */

static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
/* Table 9-4 (chroma_format_idc 1), inter column: codeNum -> coded_block_pattern */
static const int CBP_P[48] = {0,  16, 1,  2,  4,  8,  32, 3,  5,  10, 12, 15, 47, 7,  11, 13,
                              14, 6,  9,  31, 35, 37, 42, 44, 33, 34, 36, 40, 39, 43, 45, 46,
                              17, 18, 20, 24, 19, 21, 26, 28, 23, 27, 29, 30, 22, 25, 38, 41};

typedef struct {
  int pcm, mvx, mvy;  /* mv in quarter-pel */
  int cbp;            /* coded_block_pattern of an inter macroblock */
  int16_t lv[384];    /* levels in scan order: luma by luma4x4BlkIdx (16 x 16), Cb / Cr DC (2 x 4),
                         Cb / Cr AC by chroma4x4BlkIdx (8 x 15) */
} or_mb;

/* ------------------------------------------------------ residual coding */

const char *fo_table_code(int table, int a, int b, int c);  /* h264_full_oracle.c: the standard's strings */
static int code_len(int table, int a, int b, int c) {
  const char *s = fo_table_code(table, a, b, c);
  return s ? (int)strlen(s) : -1;
}
static void put_code(or_bw *b, int table, int a, int bb, int c) {
  const char *s = fo_table_code(table, a, bb, c);
  for (; s && *s; s++) bw_bit(b, (uint32_t)(*s - '0'));
}

static const int ZZ[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15}; /* 8.5.6 */
/* luma4x4BlkIdx -> raster 4x4 position (6.4.3) */
static const int BLK_X[16] = {0, 1, 0, 1, 2, 3, 2, 3, 0, 1, 0, 1, 2, 3, 2, 3};
static const int BLK_Y[16] = {0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3};
/* quantisation multipliers by qP % 6 and position class (0: both coordinates
 * even, 1: both odd, 2: mixed); the encoder's choice, the inverse of 8.5.9's
 * v = {10, 16, 13} ... so that (v MF) ~ 2^17 */
static const int MF[6][3] = {{13107, 5243, 8066}, {11916, 4660, 7490}, {10082, 4194, 6554},
                             {9362, 3647, 5825},  {8192, 3355, 5243},  {7282, 2893, 4559}};
static const int NV[6][3] = {{10, 16, 13}, {11, 18, 14}, {13, 20, 16}, {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};
static const int QPC[52] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17,
                            18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 32, 33,
                            34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};
static int pos_class(int i, int j) { return (!(i & 1) && !(j & 1)) ? 0 : ((i & 1) && (j & 1) ? 1 : 2); }

/* W = Cf X Cf^T, Cf = [1 1 1 1; 2 1 -1 -2; 1 -1 -1 1; 1 -2 2 -1]; raster */
static void fwd4(const int *x, int *w) {
  static const int Cf[4][4] = {{1, 1, 1, 1}, {2, 1, -1, -2}, {1, -1, -1, 1}, {1, -2, 2, -1}};
  int t[16];
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 4; k++) {
      int a = 0;
      for (int j = 0; j < 4; j++) a += x[i * 4 + j] * Cf[k][j];
      t[i * 4 + k] = a;
    }
  for (int k = 0; k < 4; k++)
    for (int c = 0; c < 4; c++) {
      int a = 0;
      for (int i = 0; i < 4; i++) a += Cf[k][i] * t[i * 4 + c];
      w[k * 4 + c] = a;
    }
}
static int quant1(int w, int mf, int qbits, int64_t f) {
  int64_t z = ((int64_t)abs(w) * mf + f) >> qbits;
  if (z > 2047) z = 2047;
  return w < 0 ? -(int)z : (int)z;
}
/* 8.5.12.1 scaling (flat) + 8.5.12.2 inverse transform; dc_done: c[0] already scaled */
static void idct4(const int *c, int qp, int dc_done, int *r) {
  int d[16], f[16];
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      int k = i * 4 + j;
      if (k == 0 && dc_done) { d[0] = c[0]; continue; }
      int ls = 16 * NV[qp % 6][pos_class(i, j)];
      d[k] = qp >= 24 ? (c[k] * ls) << (qp / 6 - 4) : (c[k] * ls + (1 << (3 - qp / 6))) >> (4 - qp / 6);
    }
  for (int i = 0; i < 4; i++) {
    int e0 = d[i * 4] + d[i * 4 + 2], e1 = d[i * 4] - d[i * 4 + 2];
    int e2 = (d[i * 4 + 1] >> 1) - d[i * 4 + 3], e3 = d[i * 4 + 1] + (d[i * 4 + 3] >> 1);
    f[i * 4] = e0 + e3; f[i * 4 + 1] = e1 + e2; f[i * 4 + 2] = e1 - e2; f[i * 4 + 3] = e0 - e3;
  }
  for (int j = 0; j < 4; j++) {
    int g0 = f[j] + f[8 + j], g1 = f[j] - f[8 + j];
    int g2 = (f[4 + j] >> 1) - f[12 + j], g3 = f[4 + j] + (f[12 + j] >> 1);
    r[j] = (g0 + g3 + 32) >> 6; r[4 + j] = (g1 + g2 + 32) >> 6;
    r[8 + j] = (g1 - g2 + 32) >> 6; r[12 + j] = (g0 - g3 + 32) >> 6;
  }
}

/* residual_block_cavlc of levels lv[0, maxNum) (scan order) with nC (-1:
 * chroma DC); bits to b, or (b == NULL) only counted; coeff_token counted as
 * the longest code over the nC classes when nC < -1 (the bound) */
static int block_bits(or_bw *b, const int16_t *lv, int maxNum, int nC) {
  int pos[16], lev[16], tc = 0, bits = 0;
  for (int i = maxNum - 1; i >= 0; i--)
    if (lv[i]) { pos[tc] = i; lev[tc++] = lv[i]; }
  int t1 = 0;
  while (t1 < tc && t1 < 3 && (lev[t1] == 1 || lev[t1] == -1)) t1++;
  if (nC < -1) {  /* upper bound over every nC class: Table 9-5 columns and the 6-bit FLC */
    int m = 6;
    for (int c = 0; c < 3; c++) { int l = code_len(0, c, tc, t1); if (l > m) m = l; }
    bits += m;
  } else if (nC >= 8) {
    bits += 6;
    if (b) bw_u(b, 6, tc == 0 ? 3u : (uint32_t)(((tc - 1) << 2) | t1));
  } else {
    int col = nC == -1 ? 3 : (nC < 2 ? 0 : (nC < 4 ? 1 : 2));
    bits += code_len(0, col, tc, t1);
    if (b) put_code(b, 0, col, tc, t1);
  }
  if (tc == 0) return bits;
  for (int i = 0; i < t1; i++) { bits++; if (b) bw_bit(b, lev[i] < 0); }
  int sl = (tc > 10 && t1 < 3) ? 1 : 0;
  for (int i = t1; i < tc; i++) {  /* 9.2.2.1 inverted */
    int level = lev[i];
    int code = level > 0 ? 2 * level - 2 : -2 * level - 1;
    if (i == t1 && t1 < 3) code -= 2;
    int prefix, suffix = 0, ssize = 0;
    if (sl == 0) {
      if (code < 14) prefix = code;
      else if (code < 30) { prefix = 14; suffix = code - 14; ssize = 4; }
      else { prefix = 15; suffix = code - 30; ssize = 12; }
    } else {
      if (code < (15 << sl)) { prefix = code >> sl; suffix = code & ((1 << sl) - 1); ssize = sl; }
      else { prefix = 15; suffix = code - (15 << sl); ssize = 12; }
    }
    bits += prefix + 1 + ssize;
    if (b) {
      for (int z = 0; z < prefix; z++) bw_bit(b, 0);
      bw_bit(b, 1);
      if (ssize) bw_u(b, ssize, (uint32_t)suffix);
    }
    if (sl == 0) sl = 1;
    if (abs(level) > (3 << (sl - 1)) && sl < 6) sl++;
  }
  int zeros = pos[0] + 1 - tc;
  if (tc < maxNum) {
    int t = maxNum == 4 ? 2 : 1;
    bits += code_len(t, tc - 1, zeros, 0);
    if (b) put_code(b, t, tc - 1, zeros, 0);
  }
  for (int i = 0; i < tc - 1 && zeros > 0; i++) {
    int run = pos[i] - pos[i + 1] - 1, row = (zeros < 7 ? zeros : 7) - 1;
    bits += code_len(3, row, run, 0);
    if (b) put_code(b, 3, row, run, 0);
    zeros -= run;
  }
  return bits;
}

/* Quantise the macroblock's residual (src - prediction) at qp, reconstruct
 * into ry / ru / rv (16x16, 8x8, 8x8 samples) and return the residual's
 * CAVLC bit bound; levels and cbp into m. */
static int residual_mb(const uint8_t *sy, const uint8_t *su, const uint8_t *sv, const uint8_t *py,
                       const uint8_t *pu, const uint8_t *pv, int qp, or_mb *m, uint8_t *ry, uint8_t *ru,
                       uint8_t *rv) {
  int qbits = 15 + qp / 6;
  int64_t f = ((int64_t)1 << qbits) / 6;
  int cbp = 0, bound = 0, nz[16];
  memset(m->lv, 0, sizeof m->lv);
  for (int k = 0; k < 16; k++) {  /* luma, luma4x4BlkIdx order */
    int bx = BLK_X[k] * 4, by = BLK_Y[k] * 4, x[16], w[16], z[16], r[16];
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 4; j++) x[i * 4 + j] = sy[(by + i) * 16 + bx + j] - py[(by + i) * 16 + bx + j];
    fwd4(x, w);
    nz[k] = 0;
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 4; j++) {
        z[i * 4 + j] = quant1(w[i * 4 + j], MF[qp % 6][pos_class(i, j)], qbits, f);
        nz[k] |= z[i * 4 + j] != 0;
      }
    for (int s = 0; s < 16; s++) m->lv[16 * k + s] = (int16_t)z[ZZ[s]];
    idct4(z, qp, 0, r);
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 4; j++) {
        int v = py[(by + i) * 16 + bx + j] + r[i * 4 + j];
        ry[(by + i) * 16 + bx + j] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
      }
    if (nz[k]) cbp |= 1 << (k >> 2);
  }
  for (int k8 = 0; k8 < 4; k8++)
    if ((cbp >> k8) & 1)
      for (int k = 4 * k8; k < 4 * k8 + 4; k++) bound += block_bits(NULL, m->lv + 16 * k, 16, -2);
  int qpc = QPC[qp], cqb = 15 + qpc / 6;
  int64_t cf = ((int64_t)1 << cqb) / 6;
  int dcnz = 0, acnz = 0, acz[2][4][16], dcl[2][4];
  for (int pl = 0; pl < 2; pl++) {
    const uint8_t *s = pl ? sv : su, *p = pl ? pv : pu;
    int wdc[4];
    for (int k = 0; k < 4; k++) {
      int bx = (k & 1) * 4, by = (k >> 1) * 4, x[16], w[16];
      for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) x[i * 4 + j] = s[(by + i) * 8 + bx + j] - p[(by + i) * 8 + bx + j];
      fwd4(x, w);
      wdc[k] = w[0];
      acz[pl][k][0] = 0;
      for (int q = 1; q < 16; q++) {
        int i = q >> 2, j = q & 3;
        acz[pl][k][q] = quant1(w[q], MF[qpc % 6][pos_class(i, j)], cqb, cf);
        acnz |= acz[pl][k][q] != 0;
      }
      for (int sidx = 1; sidx < 16; sidx++) m->lv[264 + pl * 60 + k * 15 + sidx - 1] = (int16_t)acz[pl][k][ZZ[sidx]];
    }
    int fd[4] = {wdc[0] + wdc[1] + wdc[2] + wdc[3], wdc[0] - wdc[1] + wdc[2] - wdc[3],
                 wdc[0] + wdc[1] - wdc[2] - wdc[3], wdc[0] - wdc[1] - wdc[2] + wdc[3]};
    for (int k = 0; k < 4; k++) {
      dcl[pl][k] = quant1(fd[k], MF[qpc % 6][0], cqb + 1, 2 * cf);
      dcnz |= dcl[pl][k] != 0;
      m->lv[256 + 4 * pl + k] = (int16_t)dcl[pl][k];
    }
  }
  int cc = acnz ? 2 : (dcnz ? 1 : 0);
  cbp |= cc << 4;
  if (cc) for (int pl = 0; pl < 2; pl++) bound += block_bits(NULL, m->lv + 256 + 4 * pl, 4, -1);
  if (cc == 2) for (int b = 0; b < 8; b++) bound += block_bits(NULL, m->lv + 264 + 15 * b, 15, -2);
  /* chroma reconstruction (8.5.11: DC through the 2x2 transform, then 8.5.12) */
  for (int pl = 0; pl < 2; pl++) {
    const int *c = dcl[pl];
    int F[4] = {c[0] + c[1] + c[2] + c[3], c[0] - c[1] + c[2] - c[3], c[0] + c[1] - c[2] - c[3],
                c[0] - c[1] - c[2] + c[3]};
    const uint8_t *p = pl ? pv : pu;
    uint8_t *rr = pl ? rv : ru;
    for (int k = 0; k < 4; k++) {
      int co[16], r[16], bx = (k & 1) * 4, by = (k >> 1) * 4;
      for (int q = 0; q < 16; q++) co[q] = cc == 2 ? acz[pl][k][q] : 0;
      co[0] = ((F[k] * 16 * NV[qpc % 6][0]) << (qpc / 6)) >> 5;
      idct4(co, qpc, 1, r);
      for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
          int v = p[(by + i) * 8 + bx + j] + r[i * 4 + j];
          rr[(by + i) * 8 + bx + j] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
        }
    }
  }
  /* without a luma 8x8 bit its levels are not coded: the decoder sees zeros */
  for (int k8 = 0; k8 < 4; k8++)
    if (!((cbp >> k8) & 1))
      for (int k = 4 * k8; k < 4 * k8 + 4; k++) {
        int bx = BLK_X[k] * 4, by = BLK_Y[k] * 4;
        for (int i = 0; i < 4; i++)
          for (int j = 0; j < 4; j++) ry[(by + i) * 16 + bx + j] = py[(by + i) * 16 + bx + j];
      }
  m->cbp = cbp;
  return bound;
}

/* prediction of one macroblock from ref (coded NV12 cw x ch), integer luma
 * motion (dx, dy); chroma 8.4.2.2.2 with edge clamping */
static void predict_mb(const uint8_t *ref, int cw, int ch, int mx, int my, int dx, int dy,
                       uint8_t *py, uint8_t *pu, uint8_t *pv) {
  for (int j = 0; j < 16; j++)
    for (int i = 0; i < 16; i++) {
      int sx = clampi(mx * 16 + i + dx, 0, cw - 1), sy = clampi(my * 16 + j + dy, 0, ch - 1);
      py[j * 16 + i] = ref[(int64_t)sy * cw + sx];
    }
  const uint8_t *uv = ref + (int64_t)cw * ch;
  int mvx = 4 * dx, mvy = 4 * dy, fx = mvx & 7, fy = mvy & 7, ccw = cw / 2, cch = ch / 2;
  for (int j = 0; j < 8; j++)
    for (int i = 0; i < 8; i++) {
      int xi = mx * 8 + i + (mvx >> 3), yi = my * 8 + j + (mvy >> 3);
      int xa = clampi(xi, 0, ccw - 1), xb = clampi(xi + 1, 0, ccw - 1);
      int ya = clampi(yi, 0, cch - 1), yb = clampi(yi + 1, 0, cch - 1);
      for (int pl = 0; pl < 2; pl++) {
        int A = uv[(int64_t)ya * cw + 2 * xa + pl], B = uv[(int64_t)ya * cw + 2 * xb + pl];
        int C = uv[(int64_t)yb * cw + 2 * xa + pl], D = uv[(int64_t)yb * cw + 2 * xb + pl];
        int v = ((8 - fx) * (8 - fy) * A + fx * (8 - fy) * B + (8 - fx) * fy * C + fx * fy * D + 32) >> 6;
        (pl ? pv : pu)[j * 8 + i] = (uint8_t)v;
      }
    }
}

/* encode one P picture's decisions and reconstruction (qp >= 1: residual coding) */
static void encode_p(const uint8_t *src, const uint8_t *ref, uint8_t *rec, int cw, int ch, int R,
                     int T, int qp, or_mb *mbs) {
  int mbw = cw / 16, mbh = ch / 16;
  const uint8_t *suv = src + (int64_t)cw * ch;
  uint8_t *ruv = rec + (int64_t)cw * ch;
  int side = 2 * R + 1, ncand = side * side, center = R * side + R;
  for (int my = 0; my < mbh; my++)
    for (int mx = 0; mx < mbw; mx++) {
      int64_t best = -1;
      int bdx = 0, bdy = 0;
      for (int c = 0; c < ncand; c++) {
        int r = c == 0 ? center : (c - 1 < center ? c - 1 : c);
        int dy = r / side - R, dx = r % side - R;
        int x0 = mx * 16 + dx, y0 = my * 16 + dy;
        int64_t s = 0;  /* reference samples outside the picture: edge clamped (8.4.2.2.1) */
        for (int j = 0; j < 16; j++)
          for (int i = 0; i < 16; i++)
            s += abs((int)ref[(int64_t)clampi(y0 + j, 0, ch - 1) * cw + clampi(x0 + i, 0, cw - 1)] -
                     (int)src[(int64_t)(my * 16 + j) * cw + mx * 16 + i]);
        if (best < 0 || s < best) { best = s; bdx = dx; bdy = dy; }
      }
      uint8_t py[256], pu[64], pv[64];
      predict_mb(ref, cw, ch, mx, my, bdx, bdy, py, pu, pv);
      int64_t cost = 0;
      for (int j = 0; j < 16; j++)
        for (int i = 0; i < 16; i++)
          cost += abs((int)py[j * 16 + i] - (int)src[(int64_t)(my * 16 + j) * cw + mx * 16 + i]);
      for (int j = 0; j < 8; j++)
        for (int i = 0; i < 8; i++) {
          int64_t o = (int64_t)(my * 8 + j) * cw + 2 * (mx * 8 + i);
          cost += abs((int)pu[j * 8 + i] - (int)suv[o]) + abs((int)pv[j * 8 + i] - (int)suv[o + 1]);
        }
      or_mb *m = &mbs[my * mbw + mx];
      m->cbp = 0;
      int inter;
      if (qp >= 1) {  /* residual coding: inter unless the residual costs more than I_PCM */
        uint8_t sy[256], su[64], sv[64];
        for (int j = 0; j < 16; j++)
          for (int i = 0; i < 16; i++) sy[j * 16 + i] = src[(int64_t)(my * 16 + j) * cw + mx * 16 + i];
        for (int j = 0; j < 8; j++)
          for (int i = 0; i < 8; i++) {
            int64_t o = (int64_t)(my * 8 + j) * cw + 2 * (mx * 8 + i);
            su[j * 8 + i] = suv[o];
            sv[j * 8 + i] = suv[o + 1];
          }
        uint8_t ry[256], ru[64], rv[64];
        int bound = residual_mb(sy, su, sv, py, pu, pv, qp, m, ry, ru, rv);
        inter = T >= 0 && bound <= 3072;
        if (inter) {
          memcpy(py, ry, 256);
          memcpy(pu, ru, 64);
          memcpy(pv, rv, 64);
        } else {
          m->cbp = 0;
        }
      } else {
        inter = T >= 0 && cost <= T;
      }
      m->pcm = !inter;
      m->mvx = inter ? 4 * bdx : 0;
      m->mvy = inter ? 4 * bdy : 0;
      for (int j = 0; j < 16; j++)
        for (int i = 0; i < 16; i++) {
          int64_t o = (int64_t)(my * 16 + j) * cw + mx * 16 + i;
          rec[o] = inter ? py[j * 16 + i] : src[o];
        }
      for (int j = 0; j < 8; j++)
        for (int i = 0; i < 8; i++) {
          int64_t o = (int64_t)(my * 8 + j) * cw + 2 * (mx * 8 + i);
          ruv[o] = inter ? pu[j * 8 + i] : suv[o];
          ruv[o + 1] = inter ? pv[j * 8 + i] : suv[o + 1];
        }
    }
}

/* residual() of an inter macroblock (7.3.5.3) with nC from the left
 * macroblock (lnz / lnzc: its right-column total_coeff, -1 unavailable) and
 * the blocks above inside this one; cnz / cnzc receive this macroblock's */
static void put_residual(or_bw *b, const or_mb *m, const int *lnz, const int (*lnzc)[2], int *cnz,
                         int (*cnzc)[4]) {
  int cbp = m->cbp;
  for (int i = 0; i < 16; i++) cnz[i] = 0;
  for (int pl = 0; pl < 2; pl++)
    for (int i = 0; i < 4; i++) cnzc[pl][i] = 0;
  for (int k = 0; k < 16; k++) {
    if (!((cbp >> (k >> 2)) & 1)) continue;
    int bx = BLK_X[k], by = BLK_Y[k];
    int na = bx ? cnz[by * 4 + bx - 1] : lnz[by], nb = by ? cnz[(by - 1) * 4 + bx] : -1;
    int nC = (na >= 0 && nb >= 0) ? (na + nb + 1) >> 1 : (na >= 0 ? na : (nb >= 0 ? nb : 0));
    const int16_t *lv = m->lv + 16 * k;
    block_bits(b, lv, 16, nC);
    int tc = 0;
    for (int i = 0; i < 16; i++) tc += lv[i] != 0;
    cnz[by * 4 + bx] = tc;
  }
  if (cbp >> 4)
    for (int pl = 0; pl < 2; pl++) block_bits(b, m->lv + 256 + 4 * pl, 4, -1);
  if ((cbp >> 4) == 2)
    for (int pl = 0; pl < 2; pl++)
      for (int k = 0; k < 4; k++) {
        int bx = k & 1, by = k >> 1;
        int na = bx ? cnzc[pl][by * 2] : lnzc[pl][by], nb = by ? cnzc[pl][bx] : -1;
        int nC = (na >= 0 && nb >= 0) ? (na + nb + 1) >> 1 : (na >= 0 ? na : (nb >= 0 ? nb : 0));
        const int16_t *lv = m->lv + 264 + 60 * pl + 15 * k;
        block_bits(b, lv, 15, nC);
        int tc = 0;
        for (int i = 0; i < 15; i++) tc += lv[i] != 0;
        cnzc[pl][k] = tc;
      }
}

static void put_pcm(or_bw *b, const uint8_t *src, int cw, int ch, int mx, int my) {
  bw_align(b);
  for (int j = 0; j < 16; j++)
    for (int i = 0; i < 16; i++) bw_u(b, 8, src[(int64_t)(my * 16 + j) * cw + mx * 16 + i]);
  const uint8_t *uv = src + (int64_t)cw * ch;
  for (int pl = 0; pl < 2; pl++)
    for (int j = 0; j < 8; j++)
      for (int i = 0; i < 8; i++) bw_u(b, 8, uv[(int64_t)(my * 8 + j) * cw + 2 * (mx * 8 + i) + pl]);
}

/* one picture, one slice per macroblock row, appended to out */
static int write_picture(const uint8_t *src, int cw, int ch, const or_mb *mbs, int idr, int idr_id,
                         int frame_num, int qp, uint8_t *out, int64_t cap, int64_t *pos, uint8_t *rbsp,
                         int64_t rcap, int64_t *stats) {
  int mbw = cw / 16, mbh = ch / 16;
  for (int row = 0; row < mbh; row++) {
    or_bw b = {rbsp, 0, rcap, 0, 0};
    bw_ue(&b, (uint32_t)(row * mbw));  /* first_mb_in_slice */
    bw_ue(&b, idr ? 7 : 5);            /* slice_type I / P (all slices) */
    bw_ue(&b, 0);                      /* pic_parameter_set_id */
    bw_u(&b, 16, (uint32_t)frame_num);
    if (idr) {
      bw_ue(&b, (uint32_t)idr_id);
    } else {
      bw_u(&b, 1, 0);                  /* num_ref_idx_active_override_flag */
      bw_u(&b, 1, 0);                  /* ref_pic_list_modification_flag_l0 */
    }
    if (idr) {
      bw_u(&b, 1, 0);                  /* no_output_of_prior_pics_flag */
      bw_u(&b, 1, 0);                  /* long_term_reference_flag */
    } else {
      bw_u(&b, 1, 0);                  /* adaptive_ref_pic_marking_mode_flag */
    }
    bw_se(&b, qp >= 1 ? qp - 26 : 0);  /* slice_qp_delta: SliceQPY = the residual's QP (pic_init_qp 26) */
    bw_ue(&b, 1);                      /* disable_deblocking_filter_idc */
    uint32_t skip = 0;
    int amv_ok = 0, amvx = 0, amvy = 0;  /* left neighbour A: inter with this mv */
    /* total_coeff of the left macroblock's right column (nC, 9.2.1): -1 none */
    int lnz[4] = {-1, -1, -1, -1}, lnzc[2][2] = {{-1, -1}, {-1, -1}}, cnz[16], cnzc[2][4];
    for (int mx = 0; mx < mbw; mx++) {
      const or_mb *m = &mbs[row * mbw + mx];
      if (idr) {
        bw_ue(&b, 25);
        put_pcm(&b, src, cw, ch, mx, row);
        stats[0]++;
        continue;
      }
      if (m->pcm) {
        bw_ue(&b, skip);
        skip = 0;
        bw_ue(&b, 30);
        put_pcm(&b, src, cw, ch, mx, row);
        amv_ok = 0;
        stats[0]++;
        for (int i = 0; i < 4; i++) lnz[i] = 16;
        for (int pl = 0; pl < 2; pl++) lnzc[pl][0] = lnzc[pl][1] = 16;
        continue;
      }
      if (m->mvx == 0 && m->mvy == 0 && m->cbp == 0) {  /* P_Skip: B unavailable -> mv 0 */
        skip++;
        stats[2]++;
        for (int i = 0; i < 4; i++) lnz[i] = 0;
        for (int pl = 0; pl < 2; pl++) lnzc[pl][0] = lnzc[pl][1] = 0;
      } else {
        int px = amv_ok ? amvx : 0, py = amv_ok ? amvy : 0;  /* 8.4.1.3, only A available */
        bw_ue(&b, skip);
        skip = 0;
        bw_ue(&b, 0);                  /* P_L0_16x16 */
        bw_se(&b, m->mvx - px);
        bw_se(&b, m->mvy - py);
        int code = 0;
        while (CBP_P[code] != m->cbp) code++;
        bw_ue(&b, (uint32_t)code);     /* coded_block_pattern me(v) */
        if (m->cbp) {
          bw_se(&b, 0);                /* mb_qp_delta */
          put_residual(&b, m, lnz, (const int(*)[2])lnzc, cnz, cnzc);
        } else {
          for (int i = 0; i < 16; i++) cnz[i] = 0;
          for (int pl = 0; pl < 2; pl++)
            for (int i = 0; i < 4; i++) cnzc[pl][i] = 0;
        }
        for (int i = 0; i < 4; i++) lnz[i] = cnz[i * 4 + 3];
        for (int pl = 0; pl < 2; pl++) {
          lnzc[pl][0] = cnzc[pl][1];
          lnzc[pl][1] = cnzc[pl][3];
        }
        stats[1]++;
      }
      amv_ok = 1;
      amvx = m->mvx;
      amvy = m->mvy;
    }
    if (skip) bw_ue(&b, skip);
    bw_trailing(&b);
    if (b.n > rcap) return -2;
    if (put_nal(out, cap, pos, idr ? 0x65 : 0x41, rbsp, b.n)) return -2;
  }
  return 0;
}

/* The whole transcode.  frames: n display-size NV12 frames (W x H, pitch W);
 * scores: the scene scores.  out: the concatenated MP4
 * samples (AVCC, 4-byte lengths); sample_off/sample_size/sync per frame;
 * recon (may be NULL): n coded NV12 reconstructions (cw x ch x 1.5 each);
 * stats: [pcm MBs, P_L0_16x16 MBs, P_Skip MBs, IDR pictures].
 * Returns 0, -1 bad argument, -2 capacity, -3 out of memory. */
int or_transcode(const uint8_t *frames, int64_t n, int W, int H, const float *scores, float thr,
                 int idr_at_cuts, int sh, int R, int T, int keyint, int qp, uint8_t *out, int64_t cap, int64_t *sample_off,
                 int64_t *sample_size, uint8_t *sync, uint8_t *recon, int64_t *stats,
                 int64_t *out_len) {
  if (n <= 0 || sh < 2 || (sh & 1) || R < 0 || R > 16 || keyint < 1 || qp > 51) return -1;
  int sw = or_small_width(W, H, sh);
  int cw = (sw + 15) & ~15, ch = (sh + 15) & ~15, mbw = cw / 16, mbh = ch / 16;
  int64_t fsz = (int64_t)cw * ch * 3 / 2, dsz = (int64_t)W * H * 3 / 2;
  uint8_t *src = (uint8_t *)malloc((size_t)fsz), *rec[2];
  rec[0] = (uint8_t *)malloc((size_t)fsz);
  rec[1] = (uint8_t *)malloc((size_t)fsz);
  or_mb *mbs = (or_mb *)calloc((size_t)mbw * mbh, sizeof(or_mb));
  int64_t rcap = 64 + (int64_t)mbw * 420;
  uint8_t *rbsp = (uint8_t *)malloc((size_t)rcap);
  int rc = (src && rec[0] && rec[1] && mbs && rbsp) ? 0 : -3;
  int64_t pos = 0, last_idr = 0, n_idr = 0;
  int cur = 0;
  for (int k = 0; k < 4; k++) stats[k] = 0;
  for (int64_t f = 0; f < n && !rc; f++) {
    or_downscale_nv12(frames + f * dsz, W, H, src, sw, sh);
    int idr = f == 0 || (idr_at_cuts && scores[f] > thr) || f - last_idr >= keyint;
    if (idr) last_idr = f;
    int j = (int)(f - last_idr);
    sample_off[f] = pos;
    sync[f] = (uint8_t)idr;
    if (idr) {
      memcpy(rec[cur], src, (size_t)fsz);
      rc = write_picture(src, cw, ch, mbs, 1, (int)(n_idr & 1), 0, qp, out, cap, &pos, rbsp, rcap, stats);
      n_idr++;
    } else {
      encode_p(src, rec[cur ^ 1], rec[cur], cw, ch, R, T, qp, mbs);
      rc = write_picture(src, cw, ch, mbs, 0, 0, j & 0xffff, qp, out, cap, &pos, rbsp, rcap, stats);
    }
    sample_size[f] = pos - sample_off[f];
    if (recon) memcpy(recon + f * fsz, rec[cur], (size_t)fsz);
    cur ^= 1;
  }
  stats[3] = n_idr;
  *out_len = pos;
  free(src); free(rec[0]); free(rec[1]); free(mbs); free(rbsp);
  return rc;
}
