/*
 * vtseg.h — C ABI of libvtseg.so, the MI355X-native long-video segmenter.
 *
 * This is the drop-in boundary for the reference's segmenter hot path
 * (shizhenneko/Video-Transformer).  The reference is pure Python and reaches
 * ffprobe/ffmpeg through subprocess; the build keeps the Python call sites
 * (package `vtseg`, same function names and signatures as the reference
 * modules) and puts everything below them behind this header: plain C types,
 * caller-allocated buffers, int status codes, a thread-local error string.
 * No exception crosses the ABI.  ctypes releases the GIL around every call.
 *
 * Entry point → reference interface it replaces:
 *   vts_plan_segments      utils/video_segmenter.py:42-83   plan_segments
 *   vts_plan_with_budget   utils/budget_planner.py:73-194   plan_segments_with_budget
 *   vts_manifest_json      utils/video_segmenter.py:170-218 create_manifest + save_manifest text
 *   vts_probe_duration     utils/video_utils.py:7-38        probe_duration (ffprobe format=duration)
 *   vts_probe_info         utils/video_utils.py:7-38        (same probe, all stream facts)
 *   vts_extract_segment    utils/video_segmenter.py:86-154  extract_segment (ffmpeg -c copy)
 *   vts_add_tracks         analyzer/content_analyzer.py:206-209 (audio kept in the upload copy)
 *   vts_boundary_frames*   (no reference code; video_segmenter.py:157-159 snap_to_keyframe
 *                          is the identity stub this feeds)  segment time -> frame index
 *   vts_open/vts_score/... (no reference code; north_star)   decode + NV12 scene scoring
 *   vts_score_nv12_dev     (no reference code)               the scoring kernel on device NV12
 *   vts_batch_run          pipeline.py:376-393 (the batch loop over analyze_video), as
 *                          vtseg.batch.plan_batch: video i on rank i % world, RCCL exchange
 *   vts_synth_write        (no reference code; tests/test_video_segmenter.py:147-178 builds
 *                          its only synthetic clip with `ffmpeg -f lavfi`, absent here)
 *
 * Status codes: 0 = ok, < 0 = error (see VTS_E_*); vts_last_error() gives a
 * message for the calling thread's last failure.
 */
#ifndef VTSEG_H
#define VTSEG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VTS_ABI_VERSION 8

enum {
  VTS_OK = 0,
  VTS_E_INVALID = -1,        /* bad argument (NULL pointer, bad geometry ...)        */
  VTS_E_CAPACITY = -2,       /* output too small; *n_out holds the size needed       */
  VTS_E_NONTERMINATING = -3, /* the reference loop would never end on this input     */
  VTS_E_RANGE = -4,          /* integer result outside int64 (Python would use bigint) */
  VTS_E_VALUE = -5,          /* Python ValueError (e.g. math.ceil(nan))              */
  VTS_E_OVERFLOW = -6,       /* Python OverflowError (e.g. math.ceil(inf))           */
  VTS_E_IO = -7,             /* file cannot be opened / read / written               */
  VTS_E_FORMAT = -8,         /* container or bitstream not understood                */
  VTS_E_UNSUPPORTED = -9,    /* valid H.264 outside the decoder's supported subset   */
  VTS_E_HIP = -10,           /* HIP runtime error                                    */
  VTS_E_NODEVICE = -11,      /* no usable gfx950 device                              */
  VTS_E_DECODE = -12,        /* bitstream error found by the device-side parser      */
  VTS_E_ZERODIV = -13        /* Python ZeroDivisionError (max_continuations == -1)   */
};

/* ---------------------------------------------------------------- planning */

/* One planned window (reference SegmentInfo, video_segmenter.py:12-18). */
typedef struct vts_segment {
  int64_t segment_id;
  double start;            /* extract window start (core start - overlap)  */
  double end;              /* extract window end   (core end + overlap)    */
  double effective_start;  /* core start                                   */
  double effective_end;    /* core end                                     */
  int64_t flags;           /* bit0: `end` is the duration argument itself,
                              bit1: `effective_end` is the duration argument
                              (lets the host mirror return the caller's int
                              object where the reference does)             */
} vts_segment;

/* plan_segments (video_segmenter.py:42-83), bit-exact double arithmetic in
 * the reference's operation order.  Two-call size query: with out == NULL or
 * cap too small returns VTS_E_CAPACITY and sets *n_out to the count needed.
 * Returns VTS_E_NONTERMINATING where the reference `while` never ends
 * (cursor + segment_seconds == cursor, or duration = +inf). */
int vts_plan_segments(double duration, double segment_seconds,
                      double overlap_seconds, vts_segment *out, int64_t cap,
                      int64_t *n_out);

/* Sync-sample (keyframe) presentation timestamps of the first video track,
 * in *timescale units (edit-list shift applied); anchors for the opt-in
 * keyframe-aware snap_to_keyframe (video_segmenter.py:157-159 stays the
 * identity by default).  Two-call size query. */
int vts_keyframe_pts(const char *path, int64_t *pts, int64_t cap, int64_t *n_out,
                     int64_t *timescale);

/* Manifest JSON (create_manifest + save_manifest, video_segmenter.py:170-218):
 * the text json.dumps(manifest, indent=2, ensure_ascii=True) writes, with the
 * plan from vts_plan_segments.  *_int: the caller's int object's decimal repr
 * (Python ints print as ints: SegmentPlan fields, an int duration), NULL for a
 * float.  segment_dir: str(get_segment_dir(...)) (pathlib-normalised).
 * Two-call size query like vts_plan_segments; VTS_E_INVALID for non-UTF-8. */
typedef struct vts_manifest_args {
  const char *video_id;
  const char *segment_dir;
  const char *created_at;
  double duration;
  const char *duration_int;
  double segment_seconds;
  const char *segment_seconds_int;
  double overlap_seconds;
  const char *overlap_seconds_int;
} vts_manifest_args;

int vts_manifest_json(const vts_manifest_args *args, char *out, int64_t cap, int64_t *len);

/* Budget-planner inputs after the reference's _coerce_int/_coerce_bool and
 * float(threshold) (budget_planner.py:20-40, 95-103); the host mirror does the
 * Python-object coercion and passes plain numbers here. */
typedef struct vts_budget_cfg {
  int64_t default_segment_seconds; /* long_video.default_segment_seconds (480) */
  int64_t overlap_seconds;         /* long_video.overlap_seconds (20)          */
  int64_t min_segment_seconds;     /* long_video.min_segment_seconds (90)      */
  int64_t hard_max_api_calls;      /* long_video.hard_max_api_calls (50)       */
  int64_t max_continuations;       /* analyzer.max_continuations (3)           */
  int64_t retry_times;             /* analyzer.retry_times (0)                 */
  int32_t has_threshold;           /* duration_threshold_seconds parsed?       */
  int32_t consolidate;             /* long_video.consolidate (True)            */
  double duration_threshold_seconds;
} vts_budget_cfg;

/* Reference SegmentPlan (budget_planner.py:9-17). */
typedef struct vts_plan {
  int64_t segment_duration;
  int64_t overlap;
  int64_t num_segments;
  int64_t estimated_calls;
  int64_t available_calls;
  int64_t hard_max_calls;
  int32_t fits_budget;
  int32_t _pad;
} vts_plan;

/* plan_segments_with_budget (budget_planner.py:73-194).  `duration` is the
 * reference's float(duration).  VTS_E_VALUE / VTS_E_OVERFLOW where the
 * reference raises ValueError / OverflowError (NaN / inf durations). */
int vts_plan_with_budget(double duration, const vts_budget_cfg *cfg,
                         int64_t current_api_count, vts_plan *out);

/* Segment time -> frame index.  For each t in times[0..ntimes): the index of
 * the first frame (presentation order) whose pts satisfies
 * pts / timescale >= t, compared exactly in integer arithmetic (no rounding);
 * n_frames when no frame qualifies.  pts must be sorted ascending. */
int vts_boundary_frames_pts(const int64_t *pts, int64_t n_frames,
                            int64_t timescale, const double *times,
                            int64_t ntimes, int64_t *frame_idx);

/* ---------------------------------------------------------------- probing */

typedef struct vts_video_info {
  double duration;            /* == vts_probe_duration                       */
  int64_t duration_us;        /* av_rescale(mvhd.duration, 1e6, mvhd.timescale) */
  int64_t movie_timescale;    /* mvhd                                        */
  int64_t movie_duration;     /* mvhd (movie timescale units)                */
  int64_t track_timescale;    /* mdhd of the first video track               */
  int64_t n_frames;           /* samples of the first video track            */
  int64_t n_sync;             /* stss entries (0 = every sample is sync)     */
  int32_t width, height;      /* display size (SPS crop applied)             */
  int32_t coded_width, coded_height; /* macroblock-aligned size             */
  int32_t profile_idc, level_idc;
  int32_t codec;              /* 1 = H.264/avc1, 0 = other                   */
  int32_t _pad;
} vts_video_info;

/* probe_duration (video_utils.py:7-38).  Parses the ISO-BMFF `moov` box: the
 * value is the one ffprobe prints for `format=duration` on a non-fragmented
 * MP4, (double)av_rescale(mvhd.duration, 1000000, mvhd.timescale) / 1e6.
 * Never fails: returns VTS_OK with *seconds = 0.0 on any error, exactly like
 * the reference (the reason is still available from vts_last_error()). */
int vts_probe_duration(const char *path, double *seconds);

/* All container facts of the first video track. Returns < 0 on error. */
int vts_probe_info(const char *path, vts_video_info *info);

/* extract_segment stream copy (video_segmenter.py:86-154, the `-c copy`
 * branch) for ISO-BMFF input: every track from the sync sample at or before
 * `start` to the last sample presented before `end`, an edit list starting
 * presentation at `start`, moov before mdat (+faststart).  0 = ok. */
int vts_extract_segment(const char *in_path, double start, double end,
                        const char *out_path);

/* Every track of video_path plus every non-video track (audio, subtitles,
 * ...) of src_path, whole and stream-copied, into out_path (moov first).  The
 * upload transcode keeps the source's audio with it, as the reference keeps
 * audio (content_analyzer.py:206-209, -c:a aac -b:a 64k; here a stream copy). */
int vts_add_tracks(const char *video_path, const char *src_path, const char *out_path);

/* ------------------------------------------------- device scoring kernel */

/* Per-frame scene scoring of NV12 frames already in device memory.
 *   thumbnail (w,h) = (width/k, height/k)   (k even, divides width and height)
 *   Y'  = box mean of the k x k luma block,        (sum + k*k/2) / (k*k)
 *   U',V' = box mean of the (k/2)x(k/2) chroma block, rounded the same way
 *   RGB = BT.709 limited-range 8-bit fixed point of (Y',U',V')
 *   hist[256]  = histogram of Y' over the thumbnail (uint32)
 *   sad        = sum |Y'_t - Y'_{t-1}| over the thumbnail (uint64; 0 for the
 *                first frame when prev_luma == NULL)
 *   score      = (float)(sad / (w * h * 255.0))
 * Frame i's Y plane starts at nv12 + i*frame_stride, its interleaved UV plane
 * at + pitch*uv_row_offset.  Outputs are device pointers; any may be NULL
 * except sad/score.  prev_luma (w*h bytes, device) seeds frame 0's SAD and
 * last_luma (w*h bytes, device, may be NULL) receives the last frame's Y'. */
typedef struct vts_score_desc {
  const uint8_t *nv12;       /* device                                      */
  int64_t frame_stride;      /* bytes between frames                        */
  int64_t n_frames;
  int32_t width, height;     /* luma size scored (display size)             */
  int32_t pitch;             /* bytes per row, Y and UV                     */
  int32_t uv_row_offset;     /* UV plane = Y + pitch*uv_row_offset          */
  int32_t k;                 /* downscale factor: 2, 4, 6 or 8              */
  int32_t _pad;
  uint8_t *rgb;              /* n_frames * w*h*3, RGB interleaved           */
  uint32_t *hist;            /* n_frames * 256                              */
  uint64_t *sad;             /* n_frames                                    */
  float *score;              /* n_frames                                    */
  const uint8_t *prev_luma;  /* w*h or NULL                                 */
  uint8_t *last_luma;        /* w*h or NULL                                 */
  uint8_t *workspace;        /* device scratch, vts_score_workspace_bytes() */
  int64_t workspace_bytes;
} vts_score_desc;

int64_t vts_score_workspace_bytes(int32_t width, int32_t height, int32_t k,
                                  int64_t n_frames);
/* Enqueue on `hip_stream` (a hipStream_t, NULL = default stream). */
int vts_score_nv12_dev(const vts_score_desc *desc, void *hip_stream);

/* --------------------------------------------- session: decode + score */

typedef struct vts_ctx vts_ctx;

typedef struct vts_params {
  int32_t k;               /* thumbnail downscale; 0 = auto (4 for <=720p, 6 above) */
  int32_t window_frames;   /* decoded-surface ring size in frames; 0 = auto        */
  int32_t keep_rgb;        /* reserved (RGB thumbnails of every frame are kept)    */
  int32_t n_streams;       /* 1 or 2 (2 = decode/score overlap on two HIP streams) */
  float cut_threshold;     /* scene-cut threshold on score (default 0.08 when <=0) */
  int32_t fused;           /* 0 auto, 1 require, -1 never: fuse scoring into
                              reconstruction (k in {2,4,8}, no cropping)       */
  int32_t gops_per_launch; /* GOPs decoded together per reconstruct launch;
                              <= 0 = all GOPs of the window (fastest measured) */
  int32_t parse_chunks;    /* slice parsing on its own stream in N chunks of
                              launches, chunk j+1 overlapping reconstruction of
                              chunk j; <= 1 (default) = one parse launch */
  int32_t level_block;     /* GOP levels decoded per reconstruct launch (k = 4,
                              fused, GOPs that are plain P chains): 0 (auto)
                              and 1 = one launch per level (fastest measured);
                              n >= 2 = up to n levels per launch with the
                              levels between in LDS */
  int32_t keep_frames;     /* level-blocked launches keep only each block's
                              last frame in HBM (the next block's reference),
                              and the general decoder recycles a picture's
                              surface once it is scored and no longer
                              referenced; 1 = store every decoded frame
                              (vts_get_frame_nv12 of any frame; the
                              transcoder sets it itself)                     */
  int32_t decoder;         /* 0 auto: the I_PCM / integer-motion subset kernels
                              when the stream's headers allow, else (or when
                              the device parser meets syntax outside the
                              subset) the general CAVLC decoder; 1 subset
                              only; 2 general              */
  int32_t _pad;
} vts_params;

/* Demux the file's first H.264 video track on the host (MP4 boxes and NAL
 * length prefixes only), upload the elementary stream to device `device`
 * and prepare the decode schedule.  Fails with VTS_E_UNSUPPORTED for streams
 * outside the device decoder's subset (see DESIGN.md §Decoder subset). */
int vts_open(int device, const char *path, const vts_params *params,
             vts_ctx **out);
/* Same, from an in-memory MP4 image (copied). */
int vts_open_memory(int device, const uint8_t *data, int64_t size,
                    const vts_params *params, vts_ctx **out);
int vts_info(const vts_ctx *ctx, vts_video_info *info);

/* Decode every frame on the device and score it.  Host outputs, each may be
 * NULL except scores; cap must be >= n_frames (else VTS_E_CAPACITY with
 * *n_frames set).  pts is in track timescale units, presentation order. */
int vts_score(vts_ctx *ctx, float *scores, uint32_t *hist, uint64_t *sad,
              int64_t *pts, int64_t cap, int64_t *n_frames);
/* Device-resident variant for benchmarking: decode + score all frames,
 * results stay on the device; returns after the work is enqueued and
 * finished (synchronous). */
int vts_run(vts_ctx *ctx);
/* vts_run split in two: vts_run_async enqueues the run on the session's HIP
 * streams and returns; vts_wait blocks until it is done (errors, timings and
 * any re-run as in vts_run).  Several sessions submitted before any waits
 * share the device (plan_batch).  Entry points that read results wait
 * themselves; vts_close waits for a run nobody waited for. */
int vts_run_async(vts_ctx *ctx);
int vts_wait(vts_ctx *ctx);
/* Scene cut frame indices (score > threshold) of the last vts_score/vts_run. */
int vts_scene_cuts(vts_ctx *ctx, int64_t *frame_idx, int64_t cap,
                   int64_t *n_out);
/* Presentation timestamps of every frame (track timescale, presentation
 * order, the order of every result); host data, no device work.  Two-call
 * size query: with pts == NULL or cap < n_frames returns VTS_E_CAPACITY and
 * sets *n_out.  The batch driver (vtseg.batch.plan_batch) turns scene-cut
 * indices into times with it without copying the per-frame results. */
int vts_frame_pts(const vts_ctx *ctx, int64_t *pts, int64_t cap, int64_t *n_out);
/* Frame index of each segment time (see vts_boundary_frames_pts). */
int vts_boundary_frames(vts_ctx *ctx, const double *times, int64_t n,
                        int64_t *frame_idx);
/* Copy frame i's decoded NV12 (display size, pitch = width) of the most
 * recent window to host; only frames still resident in the ring. */
int vts_get_frame_nv12(vts_ctx *ctx, int64_t frame, uint8_t *out,
                       int64_t out_bytes);
/* RGB thumbnail (w x h x 3, see vts_score_desc) of frame i of the last run. */
int vts_get_thumbnail_rgb(vts_ctx *ctx, int64_t frame, uint8_t *out,
                          int64_t out_bytes);
/* Timing of the last vts_run/vts_score, milliseconds, HIP events:
 * [0] whole, [1] parse, [2] reconstruct, [3] score. */
int vts_last_timings(const vts_ctx *ctx, double *ms4);
/* Device memory released by closed sessions stays mapped in a process-wide
 * cache that later sessions reuse (re-allocating released HBM waits while the
 * driver clears it); this hands device `device`'s cache back to HIP. */
int vts_empty_cache(int device);
/* Bytes of device memory the sessions' allocator has handed out on `device`
 * (open sessions' buffers; the cache's free ranges excluded). */
int64_t vts_device_bytes(int device);
/* Destroy the idle pooled HIP stream sets of `device` (< 0: every device);
 * sets held by open sessions stay.  Returns the number of sets destroyed.
 * Call before process exit when streams should not outlive the library
 * (the Python loader does, at interpreter exit). */
int vts_release_streams(int device);
/* Host time of the vts_open that made ctx, milliseconds, by stage:
 * [0] demux (moov) + device checks, [1] unused, [2] sample read (parallel
 * pread), [3] host decode schedule, [4] device allocations (+ the general
 * decoder's set-up kernels), [5] wait for the elementary-stream upload (it
 * runs on its own thread beside [3] and [4]), [6] the rest, [7] total.
 * Writes min(cap, 8) entries; returns 8. */
int vts_open_timings(const vts_ctx *ctx, double *ms, int32_t cap);
/* Decode schedule facts: what = 0 reconstruct launches per run, 1 windows,
 * 2 slices, 3 ring frames, 4 fused scoring (1/0), 5 / 6 level-blocked
 * launches / chains, 7 chain slots, 8 general decoder (1/0), 9 runs repeated
 * with the bound's CABAC coefficient arena, 10 coefficient blocks per ring,
 * 11 decoded-picture surfaces per ring when the general decoder recycles them
 * (0: one per window frame), 12 the session's HIP stream set (0 plain
 * streams on the process's shared hardware queues, 1 streams with hardware
 * queues of their own: sessions opened beside others, at most 3 such sets
 * per device), 13 CABAC slices parsed in the windows' long-slice launches
 * (0: every window one parse launch); < 0 on error. */
int64_t vts_schedule_info(const vts_ctx *ctx, int32_t what);  /* 8: general decoder in use (1/0) */
int vts_close(vts_ctx *ctx);

/* ------------------------------------------------------------ batch
 * One call per process plans (and with score = 1 decodes + scores) a batch
 * of videos: video i belongs to rank i % world, this process runs its own
 * (at most max_in_flight sessions open at once, every run submitted before
 * earlier ones are waited for), and two all-gathers over RCCL give every
 * rank the whole batch: the per-video records, then the boundary arrays
 * padded to the batch's widths.  Replaces the reference's sequential loop
 * (src/pipeline.py:376-393 -> ContentAnalyzer.analyze_video per URL); the
 * same records and rules as vtseg.batch.plan_batch (a video whose scoring
 * fails is marked and the batch goes on; a planning error fails the call
 * on the rank that meets it, before any exchange).
 *
 * The communicator: vts_rccl_unique_id on one rank, its 128 bytes sent to
 * the others by the host's own means, then vts_rccl_comm_init on every
 * rank (its device, the world size, its rank).  NULL: this process is the
 * whole batch (rank 0 of 1) and nothing is exchanged.  RCCL (librccl.so.1)
 * is loaded on first use. */
#define VTS_RCCL_ID_BYTES 128
int vts_rccl_unique_id(uint8_t *id /* VTS_RCCL_ID_BYTES */);
int vts_rccl_comm_init(int32_t device, int32_t world, int32_t rank, const uint8_t *id, void **comm);
int vts_rccl_comm_destroy(void *comm);

typedef struct vts_batch vts_batch;
typedef struct vts_batch_params {
  int32_t score;             /* 1: decode + score every video (scene cuts, segment frames)  */
  int32_t device;            /* HIP device of this rank                                     */
  int32_t max_in_flight;     /* sessions open at once on this rank; 0 = 4                   */
  int32_t _pad;
  int64_t current_api_count; /* plan_segments_with_budget's current_api_count               */
  void *rccl_comm;           /* vts_rccl_comm_init's, or NULL (one process, no exchange)    */
} vts_batch_params;
/* BatchItem (vtseg/batch.py) without its arrays */
typedef struct vts_batch_record {
  double duration;           /* probe_duration, through the exchange in microseconds      */
  int64_t n_segments;        /* plan_segments windows                                     */
  int64_t n_cuts;            /* scene cuts; -1 when not scored or scoring failed          */
  int32_t rank;              /* rank that processed the video                             */
  int32_t score_failed;      /* 1: scoring failed (vts_batch_error on that rank says why) */
} vts_batch_record;
int vts_batch_run(const char *const *paths, int64_t n, const vts_budget_cfg *cfg,
                  const vts_batch_params *params, vts_batch **out);
int vts_batch_get(const vts_batch *b, int64_t i, vts_batch_record *rec);
/* video i's arrays (score = 1): segment_frames 2 x n_segments ([start, end)
 * frame of each segment's extract window), cut_frames / cut_times n_cuts
 * (presentation time in seconds); each may be NULL */
int vts_batch_arrays(const vts_batch *b, int64_t i, int64_t *segment_frames,
                     int64_t *cut_frames, double *cut_times);
/* the scoring failure of one of this rank's videos ("" otherwise); two-call
 * size query through *len */
int vts_batch_error(const vts_batch *b, int64_t i, char *msg, int64_t cap, int64_t *len);
void vts_batch_free(vts_batch *b);

/* ------------------------------- upload transcode (360p)
 * Replaces the pixel half of ContentAnalyzer._compress_video_for_upload
 * (src/analyzer/content_analyzer.py:167-236: `ffmpeg -vf scale=-2:360
 * -c:v libx264 -crf 28`).  The session's device decoder decodes every frame,
 * an area filter downscales it to (w, height) with w = ffmpeg's scale=-2
 * width, and a device encoder writes H.264 Constrained Baseline: IDR (all
 * I_PCM) every keyint frames (and at scene cuts if asked), P pictures of full-search
 * integer motion (P_L0_16x16 / P_Skip) with a quantised residual (qp), I_PCM
 * where that residual would cost more; one slice per macroblock row; MP4
 * (moov at the end), video only.  DESIGN.md §11. */
typedef struct vts_transcode_params {
  int32_t height;          /* output display height, even; 0 = 360            */
  int32_t search_range;    /* full-search motion range in luma pixels 0..16;
                              < 0 = 0 (zero motion only); 0 = default 8       */
  int32_t max_mb_sad;      /* inter if luma+chroma SAD <= this, else I_PCM;
                              0 = default 1536 (4 per sample; 36 dB PSNR
                              on the synthetic 720p clip); < 0 = all I_PCM */
  int32_t keyint;          /* max frames per GOP; 0 = 250 (x264's default)    */
  float cut_threshold;     /* with idr_at_cuts: IDR where score > this;
                              <= 0 = the session's threshold                  */
  int32_t idr_at_cuts;     /* 1: also an IDR at every scene cut (an IDR is all
                              I_PCM, so off by default: a cut P picture falls
                              back to I_PCM only where motion misses)         */
  int32_t qp;              /* residual coding of P macroblocks at this QP (flat
                              scaling): P_L0_16x16 + quantised 4x4 residual,
                              I_PCM only where the residual's CAVLC bits would
                              exceed the I_PCM payload; 0 = default 28 (the
                              reference's CRF); < 0 = no residual (inter within
                              max_mb_sad, else I_PCM)                        */
} vts_transcode_params;

typedef struct vts_transcode_info {
  int32_t width, height;   /* output display size                              */
  int64_t n_frames;
  int64_t n_idr;
  int64_t pcm_mbs, inter_mbs, skip_mbs;
  int64_t bytes_written;   /* output file size                                 */
  double ms[4];            /* decode+score+downscale (host clock), motion
                              search span (stream 1), slice writing span
                              (stream 2, overlaps the searches), MP4 mux      */
} vts_transcode_info;

/* Transcode the session's video to `out_path`. */
int vts_transcode(vts_ctx *ctx, const char *out_path, const vts_transcode_params *p,
                  vts_transcode_info *info);

/* ------------------------------------------------ synthetic stream writer */

typedef struct vts_synth_params {
  int32_t width, height;        /* multiples of 2; coded size = 16-aligned     */
  int32_t fps_num, fps_den;     /* frame rate, e.g. 30/1                       */
  int64_t n_frames;
  uint64_t seed;                /* PCG32 seed                                   */
  double cut_min_s, cut_max_s;  /* scene length ~ U[cut_min, cut_max] seconds   */
  double gop_max_s;             /* IDR at least every gop_max seconds           */
  int32_t max_motion;           /* |pan| per frame in luma pixels (even)        */
  int32_t slices_per_row;       /* n > 0: n slices per macroblock row; 0: one
                                   slice per picture                            */
  int32_t hash_frames;          /* 1 = compute vts_synth_info.recon_hash        */
  int32_t edge_cases;           /* bit 0: plant runs of zero luma samples in
                                   each scene texture (I_PCM data then holds
                                   emulation-prevention bytes); bit 1: odd-pixel
                                   pans (half-pel chroma, 8.4.2.2.2 bilinear);
                                   max_motion may then be odd; bit 2: the last
                                   picture (if P) loses the slice holding
                                   macroblock row 1 (missing macroblocks);
                                   bit 3: refresh pictures (not scene cuts)
                                   are non-reference non-IDR I pictures, so
                                   the next P picture predicts across them  */
  int32_t chunks;               /* the stream is coded as this many runs of
                                   frames, each starting with an IDR scene cut,
                                   on parallel host threads; 0 = one run per
                                   18 000 frames (10 min at 30 fps; 1 800 for
                                   coding 1)                                    */
  int32_t coding;               /* 0: the I_PCM / P_Skip subset above;
                                   1: full CAVLC syntax, decoded by the general
                                   device decoder: Intra_4x4 / Intra_16x16 /
                                   chroma intra modes, I_PCM, residual blocks
                                   (all coeff_token / level / run codes), P
                                   partitions 16x16 .. 4x4 with quarter-sample
                                   motion, up to 3 reference frames (list
                                   modification, non-reference pictures), QP
                                   changes, the deblocking filter on (idc 0/2,
                                   offsets); bit 4 of edge_cases then turns on
                                   constrained_intra_pred.  Further coding-1
                                   bits: 5 B pictures, 6 / 7 explicit /
                                   implicit weights, 8 temporal direct, 10
                                   CABAC, 11 8x8 transforms, 12 / 13 SPS / PPS
                                   scaling matrices, 14 content mode (with bit
                                   5: pictures coded from textured moving
                                   scenes instead of random syntax)           */
} vts_synth_params;

typedef struct vts_synth_info {
  int64_t bytes_written;
  int64_t n_idr;
  int64_t n_cuts;               /* scene cuts (excluding frame 0)               */
  int64_t timescale;            /* track timescale                              */
  uint64_t recon_hash;          /* sum over frames f, bytes j of the display-size
                                   NV12 frame: b_j * ((j % 65521) + 1) * (f + 1),
                                   mod 2^64 (the encoder's own reconstruction)  */
} vts_synth_info;

/* Write a conforming H.264 (Constrained Baseline, CAVLC, I_PCM intra
 * macroblocks, P_L0_16x16 / P_Skip integer-motion inter macroblocks without
 * residual, deblocking disabled) elementary stream in an MP4 container.
 * cut_frames (may be NULL, cap entries) receives the ground-truth scene-cut
 * frame indices. */
int vts_synth_write(const char *path, const vts_synth_params *p,
                    vts_synth_info *info, int64_t *cut_frames, int64_t cap);

/* ------------------------------------------------------------------ misc */
const char *vts_last_error(void);
int vts_abi_version(void);
/* Number of visible HIP devices (0 when none); never initialises more than
 * the HIP runtime. */
int vts_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* VTSEG_H */
