// mp4.h — ISO-BMFF (MP4) demuxer and muxer for H.264 video tracks.
//
// Demux side replaces the container half of `ffprobe`/`ffmpeg` in the
// reference (utils/video_utils.py:9-27 probes `format=duration`;
// utils/video_segmenter.py:118-136 stream-copies): it reads `moov` only, never
// the media payload, and yields the per-sample table (offset, size, dts, cts,
// sync) the device decoder schedules from.
#pragma once
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

namespace vts {

struct EditEntry {
  int64_t segment_duration;  // movie timescale
  int64_t media_time;        // track timescale, -1 = empty edit
};

struct Mp4VideoTrack {       // any track; `video` holds the 'vide' ones
  uint32_t track_id = 0;
  uint32_t handler = 0;       // hdlr handler_type fourcc ('vide', 'soun', ...)
  uint16_t language = 0x55c4; // mdhd packed ISO-639-2 ("und")
  int16_t volume = 0;         // tkhd volume (8.8)
  std::vector<uint8_t> stsd;  // the whole stsd box, copied verbatim on remux
  std::vector<uint8_t> hdlr;  // the whole hdlr box
  std::vector<uint8_t> media_header;  // vmhd / smhd / nmhd box (whole), if any
  int64_t timescale = 0;
  int64_t duration = 0;       // mdhd, track timescale
  int tkhd_width = 0, tkhd_height = 0;
  std::string codec;          // sample entry fourcc ("avc1", "hvc1", ...)
  int nal_length_size = 4;
  std::vector<std::vector<uint8_t>> sps, pps;
  std::vector<int64_t> offset;
  std::vector<uint32_t> size;
  std::vector<int64_t> dts;
  std::vector<int32_t> cts_offset;  // ctts, 0 when absent
  std::vector<uint8_t> sync;        // 1 = sync sample (all 1 when no stss)
  bool has_stss = false;
  bool has_ctts = false;
  std::vector<EditEntry> edits;
};

struct Mp4Info {
  int64_t movie_timescale = 0;
  int64_t movie_duration = 0;
  bool has_mvhd = false;
  bool fragmented = false;   // moof/mvex present: the tracks' sample tables hold
                             // the moov's samples followed by every movie
                             // fragment's (moof/traf/trun), in file order
  int64_t fragment_duration = 0;  // mehd (movie timescale), 0 when absent
  int64_t file_size = 0;
  std::vector<Mp4VideoTrack> video;
  std::vector<Mp4VideoTrack> tracks;  // every track with a sample table, file order
};

// Parse the container from a file path or from memory. "" = ok, else error.
std::string mp4_parse_file(const char *path, Mp4Info *out);
std::string mp4_parse_memory(const uint8_t *data, int64_t size, Mp4Info *out);

// libavformat: s->duration = av_rescale(mvhd.duration, AV_TIME_BASE, timescale)
// (round to nearest, ties away from zero); a timescale <= 0 reads as 1.
int64_t mvhd_duration_us(const Mp4Info &info);
// The container duration ffprobe's format=duration reports, microseconds:
// mvhd's when it is set; for a fragmented file whose mvhd says 0, the
// longest track's samples (first decode time to the last sample's end, each
// track in its own timescale, rounded as above).  -1: none.
int64_t container_duration_us(const Mp4Info &info);

// Stream-copy [start, end) seconds of every track into a new MP4 with moov
// first (ffmpeg -ss S -i IN -t D -c copy -movflags +faststart):
// each track starts at the last sync sample with pts <= start (pts/timescale
// compared exactly), keeps samples with pts < end, and gets an edit list that
// starts presentation at `start`.  "" = ok, else the reason.
std::string mp4_remux_segment(const char *in_path, double start, double end,
                              const char *out_path);

// Every track of video_path plus every non-video track of src_path (audio,
// subtitles ...), whole and stream-copied, into out_path (moov first).  The
// upload transcode keeps the source's audio this way (content_analyzer.py:
// 206-209 keeps it with -c:a aac).  "" = ok, else the reason.
std::string mp4_add_tracks(const char *video_path, const char *src_path, const char *out_path);

// Streaming MP4 writer: ftyp, mdat (64-bit size), moov at the end.
class Mp4Writer {
 public:
  ~Mp4Writer();
  std::string open(const char *path);
  // cts_frames: composition offset (ctts) in sample durations; any non-zero
  // value makes finish() write a ctts box (B-frame reordering)
  std::string add_sample(const uint8_t *data, size_t n, bool sync, uint32_t cts_frames = 0);
  // Raw bytes appended to mdat (samples in any order); *offset = their file
  // offset, for add_sample_at.
  std::string append(const uint8_t *data, size_t n, int64_t *offset);
  // The next sample (decode order) whose n bytes are already in mdat at offset.
  std::string add_sample_at(int64_t offset, size_t n, bool sync);
  // track_timescale / sample_delta: constant frame duration; movie timescale
  // 1000.  sps/pps: NAL units including their header byte.
  std::string finish(int width, int height, int64_t track_timescale,
                     int64_t sample_delta, const std::vector<uint8_t> &sps,
                     const std::vector<uint8_t> &pps);
  int64_t bytes_written() const { return pos_; }

 private:
  FILE *f_ = nullptr;
  int64_t pos_ = 0;
  int64_t mdat_start_ = 0;
  std::vector<int64_t> offsets_;
  std::vector<uint32_t> sizes_;
  std::vector<uint32_t> sync_;
  std::vector<uint32_t> cts_;
  bool any_cts_ = false;
};

}  // namespace vts
