#include "common.h"
using namespace vts;
extern "C" {
int vts_open(int, const char *, const vts_params *, vts_ctx **) { return fail(VTS_E_UNSUPPORTED, "todo"); }
int vts_open_memory(int, const uint8_t *, int64_t, const vts_params *, vts_ctx **) { return fail(VTS_E_UNSUPPORTED, "todo"); }
int vts_info(const vts_ctx *, vts_video_info *) { return fail(VTS_E_UNSUPPORTED, "todo"); }
int vts_score(vts_ctx *, float *, uint32_t *, uint64_t *, int64_t *, int64_t, int64_t *) { return fail(VTS_E_UNSUPPORTED, "todo"); }
int vts_run(vts_ctx *) { return fail(VTS_E_UNSUPPORTED, "todo"); }
int vts_scene_cuts(vts_ctx *, int64_t *, int64_t, int64_t *) { return fail(VTS_E_UNSUPPORTED, "todo"); }
int vts_boundary_frames(vts_ctx *, const double *, int64_t, int64_t *) { return fail(VTS_E_UNSUPPORTED, "todo"); }
int vts_get_frame_nv12(vts_ctx *, int64_t, uint8_t *, int64_t) { return fail(VTS_E_UNSUPPORTED, "todo"); }
int vts_last_timings(const vts_ctx *, double *) { return fail(VTS_E_UNSUPPORTED, "todo"); }
int vts_close(vts_ctx *) { return 0; }
int vts_synth_write(const char *, const vts_synth_params *, vts_synth_info *, int64_t *, int64_t) { return fail(VTS_E_UNSUPPORTED, "todo"); }
int vts_device_count(void) { return 0; }
}
