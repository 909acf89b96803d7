// probe.cpp — container probing (reference utils/video_utils.py:7-38).
#include <cstring>

#include "common.h"
#include "h264.h"
#include "mp4.h"

namespace vts {

// Fill `info` from a parsed container. Returns VTS_OK or an error code.
int fill_video_info(const Mp4Info &mp4, vts_video_info *info) {
  std::memset(info, 0, sizeof *info);
  info->movie_timescale = mp4.movie_timescale;
  info->movie_duration = mp4.movie_duration;
  if (mp4.has_mvhd) {
    const int64_t us = container_duration_us(mp4);
    if (us >= 0) {
      info->duration_us = us;
      info->duration = static_cast<double>(us) / 1e6;
    }
  }
  if (mp4.video.empty()) return fail(VTS_E_FORMAT, "no video track");
  const Mp4VideoTrack &t = mp4.video.front();
  info->track_timescale = t.timescale;
  info->n_frames = static_cast<int64_t>(t.size.size());
  int64_t nsync = 0;
  if (t.has_stss)
    for (uint8_t s : t.sync) nsync += s;
  info->n_sync = nsync;
  info->width = t.tkhd_width;
  info->height = t.tkhd_height;
  info->codec = (t.codec == "avc1" || t.codec == "avc3") ? 1 : 0;
  if (info->codec && !t.sps.empty()) {
    Sps sps;
    if (parse_sps(t.sps[0].data(), t.sps[0].size(), &sps).empty()) {
      info->width = sps.width();
      info->height = sps.height();
      info->coded_width = sps.mb_width * 16;
      info->coded_height = sps.mb_height * 16;
      info->profile_idc = sps.profile_idc;
      info->level_idc = sps.level_idc;
    }
  }
  return VTS_OK;
}

}  // namespace vts

using namespace vts;

extern "C" int vts_probe_info(const char *path, vts_video_info *info) {
  clear_error();
  if (!path || !info) return fail(VTS_E_INVALID, "NULL argument");
  Mp4Info mp4;
  const std::string e = mp4_parse_file(path, &mp4);
  if (!e.empty()) return fail(VTS_E_FORMAT, "%s", e.c_str());
  return fill_video_info(mp4, info);
}

extern "C" int vts_probe_duration(const char *path, double *seconds) {
  clear_error();
  if (!seconds) return fail(VTS_E_INVALID, "seconds is NULL");
  *seconds = 0.0;  // reference convention: 0.0 on any failure, never an error
  if (!path) {
    fail(VTS_E_INVALID, "path is NULL");
    return VTS_OK;
  }
  Mp4Info mp4;
  const std::string e = mp4_parse_file(path, &mp4);
  if (!e.empty()) {
    fail(VTS_E_FORMAT, "%s", e.c_str());
    return VTS_OK;
  }
  if (!mp4.has_mvhd) {
    fail(VTS_E_FORMAT, "no mvhd");
    return VTS_OK;
  }
  // ffprobe prints 0 duration as "N/A" -> the reference's float() fails -> 0.0
  const int64_t us = container_duration_us(mp4);
  if (us < 0) {
    fail(VTS_E_FORMAT, "fragmented MP4 without samples");
    return VTS_OK;
  }
  *seconds = static_cast<double>(us) / 1e6;
  return VTS_OK;
}

// Presentation timestamps (track timescale, edit-list shift applied as in
// the device session and the remuxer) of the first video track's sync
// samples: the anchors of the opt-in keyframe-aware snap_to_keyframe
// (video_segmenter.py:157-159 is the identity stub).  Two-call size query.
extern "C" int vts_keyframe_pts(const char *path, int64_t *pts, int64_t cap, int64_t *n_out,
                                int64_t *timescale) {
  clear_error();
  if (!path || !n_out || !timescale) return fail(VTS_E_INVALID, "NULL argument");
  Mp4Info mp4;
  const std::string e = mp4_parse_file(path, &mp4);
  if (!e.empty()) return fail(VTS_E_FORMAT, "%s", e.c_str());
  if (mp4.video.empty()) return fail(VTS_E_FORMAT, "no video track");
  const Mp4VideoTrack &t = mp4.video.front();
  int64_t shift = 0;
  for (const EditEntry &ed : t.edits)
    if (ed.media_time >= 0) {
      shift = ed.media_time;
      break;
    }
  *timescale = t.timescale;
  int64_t n = 0;
  for (size_t i = 0; i < t.dts.size(); ++i) {
    if (!t.sync[i]) continue;
    if (pts && n < cap) pts[n] = t.dts[i] + t.cts_offset[i] - shift;
    ++n;
  }
  *n_out = n;
  if (!pts || n > cap) return fail(VTS_E_CAPACITY, "need %lld", static_cast<long long>(n));
  return VTS_OK;
}
