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

typedef struct { int pcm, mvx, mvy; } or_mb;  /* mv in quarter-pel */

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

/* encode one P picture's decisions and reconstruction */
static void encode_p(const uint8_t *src, const uint8_t *ref, uint8_t *rec, int cw, int ch, int R,
                     int T, or_mb *mbs) {
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
      int inter = T >= 0 && cost <= T;
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
                         int frame_num, uint8_t *out, int64_t cap, int64_t *pos, uint8_t *rbsp,
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
    bw_se(&b, 0);                      /* slice_qp_delta */
    bw_ue(&b, 1);                      /* disable_deblocking_filter_idc */
    uint32_t skip = 0;
    int amv_ok = 0, amvx = 0, amvy = 0;  /* left neighbour A: inter with this mv */
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
        continue;
      }
      if (m->mvx == 0 && m->mvy == 0) {  /* P_Skip: B unavailable -> mv 0 */
        skip++;
        stats[2]++;
      } else {
        int px = amv_ok ? amvx : 0, py = amv_ok ? amvy : 0;  /* 8.4.1.3, only A available */
        bw_ue(&b, skip);
        skip = 0;
        bw_ue(&b, 0);                  /* P_L0_16x16 */
        bw_se(&b, m->mvx - px);
        bw_se(&b, m->mvy - py);
        bw_ue(&b, 0);                  /* coded_block_pattern 0 */
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
                 int idr_at_cuts, int sh, int R, int T, int keyint, uint8_t *out, int64_t cap, int64_t *sample_off,
                 int64_t *sample_size, uint8_t *sync, uint8_t *recon, int64_t *stats,
                 int64_t *out_len) {
  if (n <= 0 || sh < 2 || (sh & 1) || R < 0 || R > 16 || keyint < 1) return -1;
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
      rc = write_picture(src, cw, ch, mbs, 1, (int)(n_idr & 1), 0, out, cap, &pos, rbsp, rcap, stats);
      n_idr++;
    } else {
      encode_p(src, rec[cur ^ 1], rec[cur], cw, ch, R, T, mbs);
      rc = write_picture(src, cw, ch, mbs, 0, 0, j & 0xffff, out, cap, &pos, rbsp, rcap, stats);
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
