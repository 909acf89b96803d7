// session.hip — vts_open / vts_score / vts_run / vts_close: one video on one GPU.
//
// Host side does only container work (MP4 boxes, NAL length prefixes, the
// first two Exp-Golomb fields of each slice header to know I vs P) and builds
// a static schedule once at open:
//   * windows of whole GOPs (each starts at an intra picture) sized to a
//     decoded-surface ring; a video that fits in kSingleWindowBytes is one
//     window (all GOPs decode in parallel); longer ones get two rings sized
//     from the free HBM;
//   * per window, "levels": level 0 = intra pictures, level L = pictures L
//     references after one; one reconstruct launch per level covers that
//     level of every GOP in the window;
// and uploads the whole elementary stream to HBM.  A run then is pure device
// work per window: memset cmd -> h264_parse (all slices of the window) ->
// one launch per level of h264_recon_score (reconstruct + thumbnail, RGB,
// histogram fused; k in {2,4,8}, no crop) -> thumb_sad, or h264_recon per
// level -> score_runs + score_seams (cropped pictures, k = 6); windows are
// pipelined over two HIP streams and two rings (decode of window i+1
// overlaps scoring of window i).
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "bitstream.h"
#include "common.h"
#include "decode.h"
#include "h264.h"
#include "mp4.h"
#include "session.h"

namespace vts {
int fill_video_info(const Mp4Info &mp4, vts_video_info *info);
}

using namespace vts;

namespace {

constexpr int64_t kSingleWindowBytes = 48ll << 30;  // up to 48 GiB decoded: one window
constexpr int64_t kMinRingBytes = 1ll << 30;        // else two rings of >= 1 GiB
constexpr int64_t kPad = 256;

// Streams outlive sessions, as whole sets: a session's six streams (decode,
// score, parse, three GOP groups) are created one after another — HIP gives
// each new stream the least-used of the process's hardware queues, so the
// six land on six different queues — and go back to a process-wide free list
// per device together, so every later session again gets six streams on six
// queues.  Single streams pooled one by one came back mixed after many
// sessions: two of one session's GOP-group / parse streams could share a
// queue and serialise (general decoder reconstruction 145 -> 239 ms in the
// bench after eight concurrent sessions on 16 queues; 218 -> 288 ms on 4,
// tools/gpu/queue_probe.py).  Sessions open at the same time never share one.
std::mutex g_stream_mu;
// free sets per (device, kind); sets handed out per device
std::map<std::pair<int, int>, std::vector<std::vector<hipStream_t>>> g_stream_sets;
std::map<int, int> g_sets_in_use;
std::map<int, int> g_own_sets;  // CU-masked sets created per device (in use or pooled)
constexpr int kSessionStreams = 3 + (vts_ctx::kMaxGroups - 1);
// at most this many CU-masked sets per device: every one holds six hardware
// queues for good, and a process with many more queues than the GPU maps at
// once is time-sliced across all of them — after the bench's batches had
// left 7 such sets (42 queues) pooled, single sessions ran 2x slower
// (profiles/r06j_bench_default_720p_batch.json); 3 sets, 18 queues, measured
// without a slowdown (r06i)
constexpr int kMaxOwnSets = 3;

// Which kind of stream set a session gets: 0 plain non-blocking streams
// (HIP spreads a process's streams over its GPU_MAX_HW_QUEUES shared hardware
// queues, 4 by default), 1 streams created with a CU mask naming every
// compute unit (HIP backs each with a hardware queue of its own).  A session
// opened while no other holds a set gets plain streams; one opened beside
// others gets its own queues, so concurrent sessions' launches never wait
// behind each other's event barriers in a shared queue.  Measured on 4 queues
// (profiles/r06i_batch_stream_policies.json, 4 content sessions through
// plan_batch): all plain 3.99x one session's step, this policy 2.35x (on 16
// plain queues 2.82x); every set CU-masked also overlaps (1.95x of its own
// step) but one session alone on its own queues is 31 % slower (392 vs 300 ms).
// Beyond kMaxOwnSets CU-masked sets, sessions take plain streams again.
int stream_kind_for(int in_use, bool own_free) { return in_use > 0 && own_free ? 1 : 0; }

int streams_take(vts_ctx *c) {
  std::vector<hipStream_t> set;
  {
    std::lock_guard<std::mutex> lk(g_stream_mu);
    int &in_use = g_sets_in_use[c->device];
    const bool own_free = !g_stream_sets[{c->device, 1}].empty() || g_own_sets[c->device] < kMaxOwnSets;
    const int kind = stream_kind_for(in_use, own_free);
    auto &v = g_stream_sets[{c->device, kind}];
    if (!v.empty()) {
      set = v.back();
      v.pop_back();
    } else {
      set.assign(kSessionStreams, nullptr);
      std::vector<uint32_t> mask;
      if (kind == 1) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || cus <= 0)
          return fail(VTS_E_HIP, "hipDeviceGetAttribute(multiProcessorCount)");
        mask.assign(static_cast<size_t>((cus + 31) / 32), 0u);
        for (int i = 0; i < cus; ++i) mask[static_cast<size_t>(i >> 5)] |= 1u << (i & 31);
      }
      for (auto &x : set) {
        const hipError_t e = kind == 1
                                 ? hipExtStreamCreateWithCUMask(&x, static_cast<uint32_t>(mask.size()), mask.data())
                                 : hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
        if (e != hipSuccess) {
          for (auto &y : set)
            if (y) (void)hipStreamDestroy(y);
          return fail(VTS_E_HIP, "hipStreamCreate");
        }
      }
      if (kind == 1) ++g_own_sets[c->device];
    }
    ++in_use;
    c->stream_kind = kind;
  }
  c->s_dec = set[0];
  c->s_score = set[1];
  c->s_parse = set[2];
  for (int g = 0; g + 1 < vts_ctx::kMaxGroups; ++g) c->s_grp[g] = set[static_cast<size_t>(3 + g)];
  return VTS_OK;
}
void streams_give(vts_ctx *c) {  // every stream idle
  if (!c->s_dec) return;
  std::vector<hipStream_t> set = {c->s_dec, c->s_score, c->s_parse};
  for (int g = 0; g + 1 < vts_ctx::kMaxGroups; ++g) set.push_back(c->s_grp[g]);
  std::lock_guard<std::mutex> lk(g_stream_mu);
  g_stream_sets[{c->device, c->stream_kind}].push_back(set);
  --g_sets_in_use[c->device];
}

}  // namespace

// Destroy the idle pooled stream sets (device < 0: every device).  Sets held
// by open sessions stay.  The library's Python loader calls it at interpreter
// exit: streams left to the HIP runtime's own teardown crashed rocprofv3
// --pmc runs at exit once CU-masked sets existed (__cxa_finalize, rc 139; the
// counter files of the pass were lost — profiles/r06j..r06s bench lines).
extern "C" int vts_release_streams(int device) {
  clear_error();
  std::lock_guard<std::mutex> lk(g_stream_mu);
  int n = 0;
  for (auto &kv : g_stream_sets) {
    if (device >= 0 && kv.first.first != device) continue;
    for (auto &set : kv.second) {
      for (hipStream_t s : set)
        if (s) (void)hipStreamDestroy(s);
      ++n;
      if (kv.first.second == 1) --g_own_sets[kv.first.first];
    }
    kv.second.clear();
  }
  return n;
}

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Read the sample bytes of the track into one contiguous host buffer (the
// elementary stream, uninitialised memory: no zero-fill pass).  Consecutive
// samples that are also consecutive in the file (a video-only mdat; the video
// runs between audio chunks otherwise) are one file range; ranges are cut into
// pieces of <= kReadPiece bytes that kReadThreads threads pread at once (a
// cached file copies at memory bandwidth per thread, one sequential reader was
// the open's largest stage).  A piece holds whole samples; `on_piece(k, s0,
// s1, src)`, when given, runs on the reading thread as soon as piece k
// (samples [s0, s1), their bytes back to back at src) is in memory, after
// `on_plan(n)` announced the n pieces.  With `es` null and `mem` given
// (a mapped file) nothing is copied: src points into `mem`.
constexpr int64_t kReadPiece = 8ll << 20;
int read_threads() {  // 8; VTS_READ_THREADS: 1..64 (measurement)
  static const int n = [] {
    const char *e = std::getenv("VTS_READ_THREADS");
    const int v = e ? std::atoi(e) : 8;
    return v < 1 ? 1 : (v > 64 ? 64 : v);
  }();
  return n;
}

// a read-only private mapping of a whole file (munmap on a detached thread
// for large ones, like HostBytes)
struct FileMap {
  const uint8_t *p = nullptr;
  int64_t n = 0;
  // VTS_OK with p null: not a regular file (the caller reads it instead)
  int open(const char *path) {
    const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return fail(VTS_E_IO, "cannot open %s", path);
    struct stat st {};
    if (::fstat(fd, &st) != 0) {
      ::close(fd);
      return fail(VTS_E_IO, "cannot stat %s", path);
    }
    if (!S_ISREG(st.st_mode) || st.st_size <= 0) {
      ::close(fd);
      return VTS_OK;
    }
    void *m = ::mmap(nullptr, static_cast<size_t>(st.st_size), PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (m == MAP_FAILED) return fail(VTS_E_IO, "cannot map %s", path);
    (void)::madvise(m, static_cast<size_t>(st.st_size), MADV_WILLNEED);
    p = static_cast<const uint8_t *>(m);
    n = st.st_size;
    return VTS_OK;
  }
  ~FileMap() {
    if (!p) return;
    void *m = const_cast<uint8_t *>(p);
    const size_t len = static_cast<size_t>(n);
    if (n >= (int64_t{64} << 20)) std::thread([m, len]() { ::munmap(m, len); }).detach();
    else ::munmap(m, len);
  }
};

struct PieceHooks {
  std::function<void(size_t)> on_plan;
  std::function<void(size_t, int64_t, int64_t, const uint8_t *)> on_piece;
};

int gather_samples(const Mp4VideoTrack &t, const uint8_t *mem, int64_t mem_size, const char *path,
                   HostBytes *es, std::vector<int64_t> *es_off, const PieceHooks *hooks = nullptr) {
  int64_t total = 0;
  for (uint32_t s : t.size) total += s;
  if (!es && !mem) return fail(VTS_E_INVALID, "gather_samples: nowhere to read to");
  if (es) {
    es->alloc(total + kPad);
    std::memset(es->data() + total, 0, kPad);
  }
  es_off->resize(t.size.size());
  struct Piece {
    int64_t file, dst, n, s0, s1;
  };
  std::vector<Piece> pieces;
  int64_t pos = 0;
  for (size_t i = 0; i < t.size.size(); ++i) {
    (*es_off)[i] = pos;
    const int64_t off = t.offset[i], n = t.size[i];
    if (off < 0 || (mem && off + n > mem_size)) return fail(VTS_E_FORMAT, "sample %zu out of file", i);
    if (!pieces.empty() && pieces.back().file + pieces.back().n == off && pieces.back().n + n <= kReadPiece) {
      pieces.back().n += n;
      pieces.back().s1 = static_cast<int64_t>(i) + 1;
    } else {
      pieces.push_back(Piece{off, pos, n, static_cast<int64_t>(i), static_cast<int64_t>(i) + 1});
    }
    pos += n;
  }
  if (hooks && hooks->on_plan) hooks->on_plan(pieces.size());
  if (pieces.empty()) return VTS_OK;
  int fd = -1;
  if (!mem) {
    fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return fail(VTS_E_IO, "cannot open %s", path);
  }
  std::atomic<size_t> next{0};
  std::atomic<int64_t> bad{-1};
  auto worker = [&]() {
    for (size_t k = next++; k < pieces.size() && bad.load() < 0; k = next++) {
      const Piece &pc = pieces[k];
      if (!es) {  // mapped: the piece is where it lies
        if (hooks && hooks->on_piece) hooks->on_piece(k, pc.s0, pc.s1, mem + pc.file);
        continue;
      }
      uint8_t *dst = es->data() + pc.dst;
      if (mem) {
        std::memcpy(dst, mem + pc.file, static_cast<size_t>(pc.n));
      } else {
        int64_t done = 0;
        while (done < pc.n) {
          const ssize_t r = ::pread(fd, dst + done, static_cast<size_t>(pc.n - done), pc.file + done);
          if (r <= 0) {
            bad = pc.dst + done;
            break;
          }
          done += r;
        }
        if (done < pc.n) break;
      }
      if (hooks && hooks->on_piece) hooks->on_piece(k, pc.s0, pc.s1, dst);
    }
  };
  const int nt = static_cast<int>(std::min<size_t>(static_cast<size_t>(read_threads()), pieces.size()));
  std::vector<std::thread> th;
  for (int i = 1; i < nt; ++i) th.emplace_back(worker);
  worker();
  for (auto &x : th) x.join();
  if (fd >= 0) ::close(fd);
  if (bad.load() >= 0) {
    size_t i = 0;
    while (i + 1 < es_off->size() && (*es_off)[i + 1] <= bad.load()) ++i;
    return fail(VTS_E_FORMAT, "cannot read sample %zu", i);
  }
  return VTS_OK;
}

// Elementary-stream upload: host bytes -> pinned staging slots (a
// process-wide pool, allocated once) -> hipMemcpyAsync into HBM (a pageable
// hipMemcpy stages internally, one small chunk at a time, synchronously).
// The threads that push byte ranges copy them into free slots themselves —
// the reading threads, each as its piece lands, so the host copies run eight
// at a time beside the read — and one thread issues the DMA of every filled
// slot and frees slots as their copies complete.  The pool belongs to one
// upload at a time.
constexpr int64_t kStageBytes = 8ll << 20;
constexpr int kStageSlots = 24;
std::mutex g_stage_mu;
uint8_t *g_stage[kStageSlots] = {};

struct EsUpload {
  std::thread th;
  std::mutex mu;
  std::condition_variable cv_dma, cv_slot;
  std::vector<int> free_slots;
  struct Filled {
    int slot;
    int64_t dst, n;
  };
  std::vector<Filled> filled;  // copied into staging, DMA not yet issued
  int pushers = 0;             // push() calls in progress
  bool closed = false, started = false;
  int rc = VTS_OK;
  std::string msg;
  std::unique_lock<std::mutex> pool;  // g_stage_mu while this upload runs

  int start(int device, uint8_t *d_es) {
    pool = std::unique_lock<std::mutex>(g_stage_mu);
    HIP_TRY(hipSetDevice(device));
    for (int i = 0; i < kStageSlots; ++i) {
      if (!g_stage[i]) HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&g_stage[i]), kStageBytes, hipHostMallocDefault));
      free_slots.push_back(i);
    }
    started = true;
    th = std::thread([this, device, d_es]() {
      rc = run(device, d_es);
      if (rc != VTS_OK) msg = last_error();
    });
    return VTS_OK;
  }
  // copy [src, src + n) to device offset dst (on the caller's thread, into
  // staging slots as they come free)
  void push(const uint8_t *src, int64_t dst, int64_t n) {
    if (!started) return;
    {
      std::lock_guard<std::mutex> lk(mu);
      ++pushers;
    }
    for (int64_t off = 0; off < n; off += kStageBytes) {
      int slot;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv_slot.wait(lk, [&] { return !free_slots.empty() || rc != VTS_OK; });
        if (rc != VTS_OK) break;
        slot = free_slots.back();
        free_slots.pop_back();
      }
      const int64_t len = std::min(kStageBytes, n - off);
      std::memcpy(g_stage[slot], src + off, static_cast<size_t>(len));
      {
        std::lock_guard<std::mutex> lk(mu);
        filled.push_back(Filled{slot, dst + off, len});
      }
      cv_dma.notify_one();
    }
    {
      std::lock_guard<std::mutex> lk(mu);
      --pushers;
    }
    cv_dma.notify_one();
  }
  int join() {
    if (started) {
      {
        std::lock_guard<std::mutex> lk(mu);
        closed = true;
      }
      cv_dma.notify_one();
      if (th.joinable()) th.join();
      started = false;
      if (pool.owns_lock()) pool.unlock();
    }
    if (rc != VTS_OK) return fail(rc, "%s", msg.c_str());
    return VTS_OK;
  }
  ~EsUpload() { (void)join(); }

 private:
  int run(int device, uint8_t *d_es) {
    if (hipSetDevice(device) != hipSuccess) return fail(VTS_E_HIP, "hipSetDevice");
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return fail(VTS_E_HIP, "hipStreamCreate");
    hipEvent_t ev[kStageSlots] = {};
    int r = VTS_OK;
    for (int i = 0; i < kStageSlots && r == VTS_OK; ++i)
      if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) r = fail(VTS_E_HIP, "hipEventCreate");
    std::vector<int> inflight;  // slots whose DMA was issued, oldest first
    auto retire_oldest = [&]() {
      const int slot = inflight.front();
      inflight.erase(inflight.begin());
      if (hipEventSynchronize(ev[slot]) != hipSuccess && r == VTS_OK) r = fail(VTS_E_HIP, "staging event");
      {
        std::lock_guard<std::mutex> lk(mu);
        free_slots.push_back(slot);
      }
      cv_slot.notify_all();
    };
    for (;;) {
      std::vector<Filled> work;
      bool done = false;
      {
        std::unique_lock<std::mutex> lk(mu);
        // wake for filled slots, for the end, or (with copies in flight) to
        // hand slots back to waiting pushers
        cv_dma.wait_for(lk, std::chrono::microseconds(200), [&] {
          return !filled.empty() || (closed && pushers == 0) || (!inflight.empty() && free_slots.empty());
        });
        work.swap(filled);
        done = closed && pushers == 0 && work.empty();
        if (r != VTS_OK) rc = r;
      }
      for (const Filled &f : work) {
        if (r == VTS_OK && (hipMemcpyAsync(d_es + f.dst, g_stage[f.slot], static_cast<size_t>(f.n), hipMemcpyHostToDevice, s) != hipSuccess ||
                            hipEventRecord(ev[f.slot], s) != hipSuccess))
          r = fail(VTS_E_HIP, "elementary-stream upload");
        inflight.push_back(f.slot);
      }
      // keep slots coming back: retire the copies that are done, and the
      // oldest when every slot is taken
      while (!inflight.empty() && hipEventQuery(ev[inflight.front()]) == hipSuccess) retire_oldest();
      bool starved;
      {
        std::lock_guard<std::mutex> lk(mu);
        starved = free_slots.empty();
      }
      if (starved && !inflight.empty()) retire_oldest();
      if (done) break;
    }
    while (!inflight.empty()) retire_oldest();
    if (hipStreamSynchronize(s) != hipSuccess && r == VTS_OK) r = fail(VTS_E_HIP, "elementary-stream upload");
    for (auto x : ev)
      if (x) (void)hipEventDestroy(x);
    (void)hipStreamDestroy(s);
    if (r != VTS_OK) {
      std::lock_guard<std::mutex> lk(mu);
      rc = r;
      cv_slot.notify_all();
    }
    return r;
  }
};

// Device buffers of the general decoder (the ES is uploaded when host_es is
// given, else already resident).
int alloc_general(vts_ctx *c) {
  HIP_TRY(hipSetDevice(c->device));
  if (!c->d_es) return fail(VTS_E_INVALID, "elementary stream not resident");
  HIP_TRY(vts::dmalloc(&c->d_fslices, sizeof(FullSlice) * std::max<size_t>(1, c->fslices.size())));
  if (!c->fslices.empty())
    HIP_TRY(hipMemcpy(c->d_fslices, c->fslices.data(), sizeof(FullSlice) * c->fslices.size(), hipMemcpyHostToDevice));
  HIP_TRY(vts::dmalloc(&c->d_scale, sizeof(ScaleTab)));
  HIP_TRY(hipMemcpy(c->d_scale, &c->scale_tab, sizeof(ScaleTab), hipMemcpyHostToDevice));
  // the slice NALs' RBSPs, made once: the parsers read plain bits
  HIP_TRY(vts::dmalloc(&c->d_rbsp, static_cast<size_t>(c->es_bytes)));
  HIP_TRY(vts::dmalloc(&c->d_rbsp_len, sizeof(int32_t) * std::max<size_t>(1, c->fslices.size())));
  VTS_TRY(nal_unescape_launch(c->d_es, c->d_rbsp, c->d_fslices, static_cast<int32_t>(c->fslices.size()),
                              c->d_rbsp_len, nullptr));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(vts::dmalloc(&c->d_porder, sizeof(int32_t) * std::max<size_t>(1, c->porder.size())));
  if (!c->porder.empty())
    HIP_TRY(hipMemcpy(c->d_porder, c->porder.data(), sizeof(int32_t) * c->porder.size(), hipMemcpyHostToDevice));
  HIP_TRY(vts::dmalloc(&c->d_porder_m, sizeof(int32_t) * std::max<size_t>(1, c->porder_m.size())));
  if (!c->porder_m.empty())
    HIP_TRY(hipMemcpy(c->d_porder_m, c->porder_m.data(), sizeof(int32_t) * c->porder_m.size(), hipMemcpyHostToDevice));
  HIP_TRY(vts::dmalloc(&c->d_dslots, sizeof(int2) * std::max<size_t>(1, c->dslots.size())));
  if (!c->dslots.empty())
    HIP_TRY(hipMemcpy(c->d_dslots, c->dslots.data(), sizeof(int2) * c->dslots.size(), hipMemcpyHostToDevice));
  HIP_TRY(vts::dmalloc(&c->d_pneed, sizeof(int32_t) * std::max<size_t>(1, c->pneed.size())));
  if (!c->pneed.empty())
    HIP_TRY(hipMemcpy(c->d_pneed, c->pneed.data(), sizeof(int32_t) * c->pneed.size(), hipMemcpyHostToDevice));
  if (const char *e = std::getenv("VTS_PARSE_MERGE")) c->parse_merged = std::atoi(e) != 0;
  if (const char *e = std::getenv("VTS_INTRA")) c->intra_kernel = std::atoi(e) == 1 ? 1 : 2;
  if (c->fprm.cabac) HIP_TRY(vts::dmalloc(&c->d_arena_top, sizeof(uint32_t) * std::max<size_t>(1, c->windows.size())));
  HIP_TRY(vts::dmalloc(&c->d_exts, sizeof(SliceExt) * std::max<size_t>(1, c->exts.size())));
  if (!c->exts.empty())
    HIP_TRY(hipMemcpy(c->d_exts, c->exts.data(), sizeof(SliceExt) * c->exts.size(), hipMemcpyHostToDevice));
  HIP_TRY(vts::dmalloc(&c->d_levels, sizeof(int4) * std::max<size_t>(1, c->level_frames.size())));
  HIP_TRY(hipMemcpy(c->d_levels, c->level_frames.data(), sizeof(int4) * c->level_frames.size(), hipMemcpyHostToDevice));
  const int64_t nmb = static_cast<int64_t>(c->sps.mb_width) * c->sps.mb_height;
  if (c->surf_pool) {
    HIP_TRY(vts::dmalloc(&c->d_surf_of, sizeof(int32_t) * c->surf_of.size()));
    HIP_TRY(hipMemcpy(c->d_surf_of, c->surf_of.data(), sizeof(int32_t) * c->surf_of.size(), hipMemcpyHostToDevice));
  }
  c->ws_bytes = score_workspace_bytes(c->width, c->height, c->k, c->ring_frames);
  const int64_t tw = (c->width / c->k) * (c->height / c->k);
  for (int r = 0; r < c->n_rings; ++r) {
    HIP_TRY(vts::dmalloc(&c->d_recs[r], static_cast<size_t>(c->ring_frames * nmb) * sizeof(MbRec)));
    if (c->fprm.bframes)
      HIP_TRY(vts::dmalloc(&c->d_recs1[r], static_cast<size_t>(c->ring_frames * nmb) * sizeof(MbRecB)));
    HIP_TRY(vts::dmalloc(&c->d_ilvl[r], static_cast<size_t>(c->ring_frames * nmb) * sizeof(uint16_t)));
    HIP_TRY(vts::dmalloc(&c->d_pdone[r], sizeof(uint32_t) * static_cast<size_t>(std::max<int64_t>(1, c->ring_frames))));
    HIP_TRY(vts::dmalloc(&c->d_dbk[r], static_cast<size_t>(c->dbk_pics * nmb) * sizeof(DbkInfo)));
    HIP_TRY(vts::dmalloc(&c->d_arena[r], static_cast<size_t>(std::max<int64_t>(1, c->arena_blocks)) * 32 + kPad));
    HIP_TRY(vts::dmalloc(&c->d_surf[r], static_cast<size_t>((c->surf_pool ? c->surf_count : c->ring_frames) * c->frame_stride + kPad)));
    if (c->surf_pool) HIP_TRY(vts::dmalloc(&c->d_thumb[r], static_cast<size_t>(c->ring_frames * tw + kPad)));
    HIP_TRY(vts::dmalloc(&c->d_ws[r], static_cast<size_t>(c->ws_bytes)));
    c->ring_cleared_at[r] = -1;
  }
  if (!c->d_last[0])
    for (int r = 0; r < 2; ++r) HIP_TRY(vts::dmalloc(&c->d_last[r], static_cast<size_t>(tw + kPad)));
  if (!c->d_err) HIP_TRY(vts::dmalloc(&c->d_err, sizeof(uint32_t)));
  if (!c->d_score) HIP_TRY(vts::dmalloc(&c->d_score, sizeof(float) * c->n_frames));
  if (!c->d_sad) HIP_TRY(vts::dmalloc(&c->d_sad, sizeof(uint64_t) * c->n_frames));
  if (!c->d_hist) HIP_TRY(vts::dmalloc(&c->d_hist, sizeof(uint32_t) * 256 * c->n_frames));
  c->thumb_px = tw;
  if (!c->d_rgb) HIP_TRY(vts::dmalloc(&c->d_rgb, static_cast<size_t>(3 * tw * c->n_frames + kPad)));
  if (!c->s_dec) VTS_TRY(streams_take(c));
  for (int g = 0; g + 1 < vts_ctx::kMaxGroups; ++g)
    if (!c->ev_grp[g]) HIP_TRY(hipEventCreateWithFlags(&c->ev_grp[g], hipEventDisableTiming));
  for (auto e2 : c->ev)
    if (e2) (void)hipEventDestroy(e2);
  c->ev.assign(c->windows.size() * 6, nullptr);
  for (auto &e2 : c->ev) HIP_TRY(hipEventCreate(&e2));
  if (!c->ev_start) HIP_TRY(hipEventCreate(&c->ev_start));
  if (!c->ev_end) HIP_TRY(hipEventCreate(&c->ev_end));
  return VTS_OK;
}

// decoder = auto: the subset kernels met syntax outside their subset; rebuild
// the schedule for the general decoder from the resident ES.
int switch_to_general(vts_ctx *c) {
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipDeviceSynchronize());
  std::vector<uint8_t> es(static_cast<size_t>(c->es_bytes));
  HIP_TRY(hipMemcpy(es.data(), c->d_es, es.size(), hipMemcpyDeviceToHost));
  auto f = [](void *p) {
    if (p) vts::dfree(p);
  };
  for (int r = 0; r < 2; ++r) {
    f(c->d_cmd[r]);
    f(c->d_thumb[r]);
    f(c->d_surf[r]);
    f(c->d_ws[r]);
    c->d_cmd[r] = nullptr;
    c->d_thumb[r] = nullptr;
    c->d_surf[r] = nullptr;
    c->d_ws[r] = nullptr;
  }
  f(c->d_tb);
  f(c->d_post);
  f(c->d_slices);
  f(c->d_levels);
  c->d_tb = nullptr;
  c->d_post = nullptr;
  c->d_slices = nullptr;
  c->d_levels = nullptr;
  for (auto e2 : c->lev)
    if (e2) (void)hipEventDestroy(e2);
  c->lev.clear();
  c->windows.clear();
  c->level_frames.clear();
  c->slices.clear();
  c->post_slots.clear();
  c->tb_chains.clear();
  VTS_TRY(build_general(c, es.data(), c->es_off, c->sample_size, c->nal_length_size, c->sps_nal, c->pps_nal));
  return alloc_general(c);
}

int build(vts_ctx *c, const Mp4Info &mp4, const uint8_t *mem, int64_t mem_size, const char *path) {
  // interleaved GOP groups per reconstruct level (VTS_RECON_GROUPS, 1..4)
  if (const char *s = std::getenv("VTS_RECON_GROUPS"))
    c->recon_groups = std::max(1, std::min(vts_ctx::kMaxGroups, std::atoi(s)));
  if (const char *s = std::getenv("VTS_GROUP_PARSE")) c->group_parse = std::atoi(s) > 0;
  if (const char *s = std::getenv("VTS_GENERAL_GROUPS")) c->general_groups = std::max(1, std::min(vts_ctx::kMaxGroups, std::atoi(s)));
  VTS_TRY(fill_video_info(mp4, &c->info));
  const Mp4VideoTrack &t = mp4.video.front();
  if (!(t.codec == "avc1" || t.codec == "avc3"))
    return fail(VTS_E_UNSUPPORTED, "codec %s: only H.264 (avc1) is decoded", t.codec.c_str());
  if (t.sps.size() != 1 || t.pps.size() != 1)
    return fail(VTS_E_UNSUPPORTED, "exactly one SPS and one PPS are supported");
  std::string e = parse_sps(t.sps[0].data(), t.sps[0].size(), &c->sps);
  if (!e.empty()) return fail(VTS_E_UNSUPPORTED, "SPS: %s", e.c_str());
  e = parse_pps(t.pps[0].data(), t.pps[0].size(), &c->pps);
  if (!e.empty()) return fail(VTS_E_UNSUPPORTED, "PPS: %s", e.c_str());
  if (c->pps.entropy_coding_mode && c->params.decoder == 1)
    return fail(VTS_E_UNSUPPORTED, "CABAC entropy coding needs the general decoder (decoder = auto / general)");
  if (c->pps.has_tail && c->params.decoder == 1)
    return fail(VTS_E_UNSUPPORTED,
                "a High-profile PPS (8x8 transform / scaling matrix / Cr QP offset) needs the general decoder");
  if (c->sps.crop_left || c->sps.crop_top)
    return fail(VTS_E_UNSUPPORTED, "left/top cropping is not supported");
  c->prm = make_dev_params(c->sps, c->pps);
  c->coded_w = c->sps.mb_width * 16;
  c->coded_h = c->sps.mb_height * 16;
  c->width = c->sps.width();
  c->height = c->sps.height();
  c->pitch = c->coded_w;
  c->frame_stride = (static_cast<int64_t>(c->pitch) * c->coded_h * 3 / 2 + 4095) & ~int64_t(4095);
  c->k = c->params.k > 0 ? c->params.k : (c->height <= 720 ? 4 : 6);
  {
    // h264_recon_score<k>: k in {2,4,8}, display = coded size;
    // h264_recon_score6b: k = 6, any cropping, thumbnail width % 8 == 0
    const bool can_fuse = ((c->k == 2 || c->k == 4 || c->k == 8) && c->width == c->coded_w &&
                           c->height == c->coded_h) ||
                          (c->k == 6 && (c->width / 6) % 8 == 0);
    if (c->params.fused > 0 && !can_fuse)
      return fail(VTS_E_UNSUPPORTED,
                  "fused scoring needs k in {2,4,8} without cropping, or k = 6 with thumbnail width % 8 == 0");
    c->fused = can_fuse && c->params.fused >= 0;
  }
  c->n_frames = static_cast<int64_t>(t.size.size());
  if (c->n_frames == 0) return fail(VTS_E_FORMAT, "video track has no samples");

  // presentation timestamps (sorted: frame i of every result is the i-th in
  // presentation order); with B pictures the decode order differs and only the
  // general decoder reorders (disp = presentation rank of each sample)
  c->pts.resize(static_cast<size_t>(c->n_frames));
  c->disp.resize(static_cast<size_t>(c->n_frames));
  int64_t shift = 0;
  for (const EditEntry &ed : t.edits)
    if (ed.media_time >= 0) {
      shift = ed.media_time;
      break;
    }
  bool reorder = false;
  for (int64_t i = 0; i < c->n_frames; ++i) {
    c->pts[i] = t.dts[i] + t.cts_offset[i] - shift;
    reorder |= i > 0 && c->pts[i] <= c->pts[i - 1];
  }
  {
    std::vector<int64_t> ord(static_cast<size_t>(c->n_frames));
    for (int64_t i = 0; i < c->n_frames; ++i) ord[static_cast<size_t>(i)] = i;
    if (reorder)
      std::stable_sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return c->pts[a] < c->pts[b]; });
    std::vector<int64_t> sorted(static_cast<size_t>(c->n_frames));
    for (int64_t i = 0; i < c->n_frames; ++i) {
      c->disp[static_cast<size_t>(ord[static_cast<size_t>(i)])] = i;
      sorted[static_cast<size_t>(i)] = c->pts[ord[static_cast<size_t>(i)]];
      if (i > 0 && sorted[static_cast<size_t>(i)] == sorted[static_cast<size_t>(i - 1)])
        return fail(VTS_E_FORMAT, "two samples share a presentation time");
    }
    c->pts = sorted;
  }
  if (reorder && c->params.decoder == 1)
    return fail(VTS_E_UNSUPPORTED, "frame reordering (B-frames / ctts) needs the general decoder");
  if ((c->pps.weighted_pred || c->pps.weighted_bipred_idc) && c->params.decoder == 1)
    return fail(VTS_E_UNSUPPORTED, "weighted prediction needs the general decoder");

  // The subset decoder's NAL walk (slice table, intra / reference flags per
  // frame) runs on the reading threads, piece by piece as each is read, into
  // per-piece tables joined in frame order below (a 2-h 720p video is ~10 M
  // slices: walked after the read on one thread it was the open's longest
  // stage).  Skipped when the headers already ask for the general decoder.
  struct Run {
    std::vector<SliceDesc> sl;
    int rc = VTS_OK;
    std::string msg;
    int64_t s0 = 0, s1 = 0;
  };
  std::vector<Run> runs;
  const int L = t.nal_length_size;
  std::vector<int64_t> first_slice(c->n_frames), n_slices(c->n_frames);
  std::vector<uint8_t> intra(c->n_frames, 1), is_ref(c->n_frames, 0);
  HostBytes es;
  std::vector<int64_t> es_off;
  // walk samples [f0, f1), whose bytes lie back to back from src
  auto walk = [&](Run &R, int64_t f0, int64_t f1, const uint8_t *src) {
    const uint8_t *E = src - es_off[f0];  // E + es_off[f]: sample f (device ES offsets)
    R.s0 = f0;
    R.s1 = f1;
    R.sl.reserve(static_cast<size_t>(f1 - f0) * 2);
    for (int64_t f = f0; f < f1; ++f) {
      int64_t p = es_off[f];
      const int64_t end = p + t.size[f];
      first_slice[f] = static_cast<int64_t>(R.sl.size());  // within the piece, rebased below
      while (p + L <= end) {
        uint32_t len = 0;
        for (int i = 0; i < L; ++i) len = (len << 8) | E[p + i];
        p += L;
        if (len == 0 || p + len > end) {
          R.rc = VTS_E_FORMAT;
          R.msg = "bad NAL length in frame " + std::to_string(f);
          return;
        }
        const uint8_t hdr = E[p];
        const int type = hdr & 0x1f;
        if (type == 1 || type == 5) {
          BitReader br(E + p + 1, len - 1);
          br.ue();  // first_mb_in_slice
          uint32_t st = br.ue();
          if (st > 4) st -= 5;
          if (st != 2) intra[f] = 0;
          if ((hdr >> 5) & 3) is_ref[f] = 1;
          SliceDesc sd{};
          sd.nal_offset = p;
          sd.nal_size = static_cast<int32_t>(len);
          R.sl.push_back(sd);
        } else if (type == 7 || type == 8) {
          const std::vector<uint8_t> &ps = (type == 7) ? t.sps[0] : t.pps[0];
          if (ps.size() != len || std::memcmp(ps.data(), E + p, len) != 0) {
            R.rc = VTS_E_UNSUPPORTED;
            R.msg = "in-band parameter set differs from avcC";
            return;
          }
        } else if (type >= 2 && type <= 4) {
          R.rc = VTS_E_UNSUPPORTED;
          R.msg = "data partitioning is not supported";
          return;
        }
        p += len;
      }
      n_slices[f] = static_cast<int64_t>(R.sl.size()) - first_slice[f];
      if (n_slices[f] == 0) {
        R.rc = VTS_E_FORMAT;
        R.msg = "frame " + std::to_string(f) + " has no slices";
        return;
      }
    }
  };
  // (subset only, or auto unless reordering or the parameter sets already
  // send the stream to the general decoder: wants_general's first checks)
  const bool may_subset = c->params.decoder == 1 || (c->params.decoder == 0 && !reorder && !general_by_headers(c));
  // the ES's device buffer first: each piece goes up as soon as it is read
  {
    int64_t total = 0;
    for (uint32_t n : t.size) total += n;
    c->es_bytes = total + kPad;
  }
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(vts::dmalloc(&c->d_es, static_cast<size_t>(c->es_bytes)));
  c->open_lap(4);
  FileMap fmap;  // before `up`: unmapped only after the upload thread has been joined
  EsUpload up;
  PieceHooks hooks;
  int up_rc = VTS_OK;
  hooks.on_plan = [&](size_t n) {
    runs.resize(n);
    up_rc = up.start(c->device, c->d_es);
  };
  hooks.on_piece = [&](size_t k, int64_t s0, int64_t s1, const uint8_t *src) {
    const int64_t end = s1 < c->n_frames ? es_off[s1] : es_off[s1 - 1] + t.size[s1 - 1];
    up.push(src, es_off[s0], end - es_off[s0]);
    if (may_subset) walk(runs[k], s0, s1, src);
  };
  // The subset decoder keeps no host copy of the ES: a file is mapped, the
  // pieces are walked and uploaded where they lie (the copy into a host
  // buffer — 7 GB for a 2-h 720p video, its pages faulted in fresh — was
  // most of the read).  The general decoder's host schedule reads the whole
  // ES, so it gets the host copy (made from the mapping if the first slices
  // send an auto stream there after all).  Only regular files are mapped (a
  // pipe or device is read with pread), and the file must not shrink while
  // vts_open runs (a mapped page past a new end faults).
  if (may_subset && !mem) VTS_TRY(fmap.open(path));
  const uint8_t *src_mem = fmap.p ? fmap.p : mem;
  const int64_t src_size = fmap.p ? fmap.n : mem_size;
  VTS_TRY(gather_samples(t, src_mem, src_size, path, fmap.p ? nullptr : &es, &es_off, &hooks));
  VTS_TRY(up_rc);
  static const uint8_t kZeroPad[kPad] = {};
  up.push(kZeroPad, c->es_bytes - kPad, kPad);  // the zero padding after the last sample
  if (fmap.p && c->params.decoder == 0) {
    // wants_general reads the first pictures' slice headers: a host copy of those
    const size_t n3 = std::min<size_t>(t.size.size(), 3);
    int64_t b3 = 0;
    for (size_t i = 0; i < n3; ++i) b3 += t.size[i];
    es.alloc(b3 + kPad);
    for (size_t i = 0; i < n3; ++i) std::memcpy(es.data() + es_off[i], fmap.p + t.offset[i], t.size[i]);
    std::memset(es.data() + b3, 0, kPad);
  } else if (!fmap.p && static_cast<int64_t>(es.size()) != c->es_bytes) {
    return fail(VTS_E_FORMAT, "elementary stream size");
  }
  c->open_lap(2);
  c->es_off = es_off;
  c->sample_size = t.size;
  c->nal_length_size = t.nal_length_size;
  c->sps_nal = t.sps[0];
  c->pps_nal = t.pps[0];

  // General CAVLC decoder (decode_full.hip) when asked, or when the headers
  // show features outside the subset kernels (deblocking, several references)
  if (c->params.decoder == 2 || reorder ||
      (c->params.decoder == 0 && wants_general(c, es.data(), es_off, t.size, t.nal_length_size))) {
    if (fmap.p) VTS_TRY(gather_samples(t, fmap.p, fmap.n, path, &es, &es_off));  // the whole ES on the host after all
    VTS_TRY(build_general(c, es.data(), es_off, t.size, t.nal_length_size, t.sps[0], t.pps[0]));
    c->open_lap(3);
    VTS_TRY(up.join());
    c->open_lap(5);
    VTS_TRY(alloc_general(c));
    c->open_lap(4);
    return VTS_OK;
  }

  // the pieces' slice tables, joined in frame order (the first failing
  // piece in frame order reports, as one walk would)
  if (!may_subset) return fail(VTS_E_INVALID, "decoder %d: no subset schedule", c->params.decoder);
  {
    for (const Run &R : runs)
      if (R.rc != VTS_OK) return fail(R.rc, "%s", R.msg.c_str());
    const size_t nr = runs.size();
    std::vector<int64_t> base(nr + 1, 0);
    for (size_t r = 0; r < nr; ++r) base[r + 1] = base[r] + static_cast<int64_t>(runs[r].sl.size());
    c->slices.resize(static_cast<size_t>(base[nr]));
    std::atomic<size_t> next{0};
    auto join = [&]() {
      for (size_t r = next++; r < nr; r = next++) {
        for (int64_t f = runs[r].s0; f < runs[r].s1; ++f) first_slice[f] += base[r];
        std::copy(runs[r].sl.begin(), runs[r].sl.end(), c->slices.begin() + base[r]);
      }
    };
    std::vector<std::thread> th;
    for (int i = 1; i < read_threads() && static_cast<size_t>(i) < nr; ++i) th.emplace_back(join);
    join();
    for (auto &x : th) x.join();
  }

  // references and levels (single reference: the latest reference picture)
  std::vector<int64_t> ref(c->n_frames, -1), level(c->n_frames, 0);
  int64_t last_ref = -1;
  for (int64_t f = 0; f < c->n_frames; ++f) {
    if (intra[f]) {
      ref[f] = -1;
      level[f] = 0;
    } else {
      ref[f] = last_ref;  // -1 -> device flags DEC_E_NO_REF
      level[f] = last_ref >= 0 ? level[last_ref] + 1 : 0;
    }
    if (is_ref[f]) last_ref = f;
  }
  // clean[x]: an intra picture no later picture predicts across (a P picture
  // after a non-reference I picture refers to the reference before it).
  // Windows and interleaved GOP groups start only at clean pictures, so no
  // reference crosses a window or a group that reconstructs on another stream.
  std::vector<uint8_t> clean(c->n_frames, 0);
  {
    int64_t min_ref = c->n_frames;  // min ref[y] over y >= x (n_frames: none)
    for (int64_t x = c->n_frames - 1; x >= 0; --x) {
      if (ref[x] >= 0) min_ref = std::min(min_ref, ref[x]);
      clean[x] = intra[x] && min_ref >= x;
    }
  }

  // windows of whole intra-started groups.  Device bytes per window frame:
  // surface + MB commands + thumbnail + scoring workspace share; the rings
  // get half of the HBM left after the whole-video buffers (ES, RGB
  // thumbnails, histograms), capped at kSingleWindowBytes each.
  const int64_t nmb_f = static_cast<int64_t>(c->sps.mb_width) * c->sps.mb_height;
  const int64_t tw_f = static_cast<int64_t>(c->width / c->k) * (c->height / c->k);
  const int64_t per_frame = c->frame_stride + 8 * nmb_f + tw_f +
                            score_workspace_bytes(c->width, c->height, c->k, 1);
  size_t free_b = 0, total_b = 0;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(vts::dmem_free(&free_b, &total_b));
  const int64_t whole = c->es_bytes + c->n_frames * (3 * tw_f + 1024 + 12) + (1ll << 30);
  const int64_t avail = std::max<int64_t>(0, static_cast<int64_t>(free_b) - whole);
  const int64_t ring_budget = std::min(kSingleWindowBytes, std::max(kMinRingBytes, avail / 4));
  int64_t cap;
  if (c->params.window_frames > 0) cap = c->params.window_frames;
  else if (c->n_frames * per_frame <= std::min(kSingleWindowBytes, avail / 2)) cap = c->n_frames;
  else cap = std::max<int64_t>(1, ring_budget / per_frame);
  auto next_intra = [&](int64_t x) {
    while (x < c->n_frames && !clean[x]) ++x;
    return x;
  };
  for (int64_t f = 0; f < c->n_frames;) {
    Window w;
    w.f0 = f;
    int64_t end = next_intra(f + 1);  // the first group is always taken
    while (end < c->n_frames) {
      const int64_t nxt = next_intra(end + 1);
      if (nxt - f > cap) break;
      end = nxt;
    }
    w.f1 = end;
    c->windows.push_back(w);
    f = end;
  }
  for (Window &w : c->windows) c->ring_frames = std::max(c->ring_frames, w.f1 - w.f0);
  c->n_rings = (c->windows.size() > 1 && c->params.n_streams >= 2) ? 2 : 1;

  // level-blocked reconstruction (h264_recon_score_tb): levels per launch
  int tb_L_max = 0;
  c->tb_last.assign(static_cast<size_t>(c->n_frames), 0);
  // Opt-in (level_block >= 2): correct, but measured slower than one launch
  // per level on MI355X, so auto (0) stays per-level.
  if (c->fused && c->k == 4 && c->params.level_block >= 2 && 4 * c->sps.mb_width <= 512) {
    tb_L_max = std::min(c->params.level_block, 16);
    const int lds_cap = 150 * 1024;
    while (tb_L_max >= 2 && (tb_lds_bytes(c->sps.mb_width, c->sps.mb_height, tb_L_max) > lds_cap ||
                             tb_max_tasks(c->sps.mb_width, c->sps.mb_height, tb_L_max) > 1024))
      --tb_L_max;
  }
  // slice slots / ref slots and per-level frame lists
  std::vector<int32_t> launch_of(static_cast<size_t>(c->n_frames), 0);  // launch index within its window
  // per window: the slices' first index per level launch (the slice pass
  // below, on threads: slots and the launch-order sort touch every slice)
  std::vector<std::vector<int64_t>> wcnt(c->windows.size());
  for (size_t wi = 0; wi < c->windows.size(); ++wi) {
    Window &w = c->windows[wi];
    w.s0 = first_slice[w.f0];
    w.s1 = (w.f1 < c->n_frames) ? first_slice[w.f1] : static_cast<int64_t>(c->slices.size());
    int64_t maxl = 0;
    for (int64_t x = w.f0; x < w.f1; ++x) {
      if (ref[x] >= 0 && ref[x] < w.f0)
        return fail(VTS_E_UNSUPPORTED, "reference crosses a window boundary");
      maxl = std::max(maxl, level[x]);
    }
    // GOPs (runs starting at an intra frame) of this window.  Default: every
    // GOP of the window in each level launch.  Grouping GOPs so a launch's
    // output fits the 256 MiB Infinity Cache (the next level's reference reads
    // would hit it) measured slower at every group size on MI355X (the kernel
    // is latency-bound and needs the full launch width):
    // profiles/r01_gop_group_sweep.txt.
    std::vector<int64_t> gop_start;
    for (int64_t x = w.f0; x < w.f1; ++x)
      if (clean[x] || x == w.f0) gop_start.push_back(x);
    int64_t per;
    if (c->params.gops_per_launch < 0) {
      per = static_cast<int64_t>(gop_start.size());
    } else if (c->params.gops_per_launch > 0) {
      per = c->params.gops_per_launch;
    } else {
      // interleaved groups: each group's level launches on its own stream
      const int64_t ng = std::min<int64_t>(c->recon_groups, static_cast<int64_t>(gop_start.size()));
      per = ng > 1 && c->params.parse_chunks <= 1 ? (static_cast<int64_t>(gop_start.size()) + ng - 1) / ng
                                                   : static_cast<int64_t>(gop_start.size());
    }
    const bool grouped = c->fused && c->params.gops_per_launch == 0 && per < static_cast<int64_t>(gop_start.size());
    for (size_t g0 = 0; g0 < gop_start.size(); g0 += static_cast<size_t>(per)) {
      if (grouped) w.grp.push_back(static_cast<int32_t>(w.lvl_off.size()));
      const size_t g1 = std::min(gop_start.size(), g0 + static_cast<size_t>(per));
      const int64_t a = gop_start[g0];
      const int64_t b = (g1 < gop_start.size()) ? gop_start[g1] : w.f1;
      int64_t gmax = 0;
      for (int64_t x = a; x < b; ++x) gmax = std::max(gmax, level[x]);
      std::vector<std::vector<int4>> lv(static_cast<size_t>(gmax + 1));
      for (int64_t x = a; x < b; ++x) {
        // the reconstruct kernel scores SAD against the display predecessor
        // when that thumbnail comes from an earlier level launch
        const bool fused_sad = x > w.f0 && level[x - 1] < level[x];
        lv[level[x]].push_back(make_int4(static_cast<int>(x - w.f0),
                                         ref[x] >= 0 ? static_cast<int>(ref[x] - w.f0) : -1,
                                         fused_sad ? static_cast<int>(x - 1 - w.f0) : -1, 0));
      }
      for (auto &l : lv) {
        if (l.empty()) continue;
        for (const int4 &e : l) launch_of[static_cast<size_t>(w.f0 + e.x)] = static_cast<int32_t>(w.lvl_off.size());
        w.lvl_off.push_back(static_cast<int64_t>(c->level_frames.size()));
        w.lvl_cnt.push_back(static_cast<int32_t>(l.size()));
        c->level_frames.insert(c->level_frames.end(), l.begin(), l.end());
      }
    }
    (void)maxl;
    // Slices in launch order (stable: decode order within a launch), so the
    // slices of launches [a, b) are one contiguous range that a parse chunk
    // can cover while reconstruction of earlier launches runs.
    {
      const int64_t nl = static_cast<int64_t>(w.lvl_off.size());
      std::vector<int64_t> cnt(static_cast<size_t>(nl) + 1, 0);
      for (int64_t x = w.f0; x < w.f1; ++x) cnt[static_cast<size_t>(launch_of[x]) + 1] += n_slices[x];
      for (int64_t l = 0; l < nl; ++l) cnt[l + 1] += cnt[l];
      w.lvl_s0.resize(static_cast<size_t>(nl));
      for (int64_t l = 0; l < nl; ++l) w.lvl_s0[l] = w.s0 + cnt[l];
      wcnt[wi] = cnt;
      // Parse chunks: the first covers launch 0 alone (reconstruction starts
      // as soon as the intra pictures are parsed), the rest split the other
      // launches into runs of about equal slice counts.
      // Default one chunk: overlapping measured no gain on MI355X (the
      // parser's VALU work slows the concurrent reconstruction by as much as
      // it hides, profiles/r01_parse_overlap_ab.txt)
      const int want = c->params.parse_chunks > 0 ? c->params.parse_chunks : 1;
      if (want <= 1 || nl <= 1) {
        w.chunk_end.push_back(static_cast<int32_t>(nl));
      } else {
        w.chunk_end.push_back(1);
        const int64_t rest = cnt[nl] - cnt[1];
        const int64_t per = std::max<int64_t>(1, (rest + want - 2) / (want - 1));
        int64_t acc = 0;
        for (int64_t l = 1; l < nl; ++l) {
          acc += cnt[l + 1] - cnt[l];
          if (acc >= per || l == nl - 1) {
            w.chunk_end.push_back(static_cast<int32_t>(l + 1));
            acc = 0;
          }
        }
      }
      // interleaved groups: optionally one parse chunk per group, so group
      // g's reconstruction starts once its own slices are parsed
      if (w.grp.size() > 1 && c->group_parse && tb_L_max < 2) {
        w.chunk_end.clear();
        for (size_t g = 1; g < w.grp.size(); ++g) w.chunk_end.push_back(w.grp[g]);
        w.chunk_end.push_back(static_cast<int32_t>(nl));
      }
    }
    // thumb_sad pass: frames without a fused SAD, plus the window's last
    // frame (its thumbnail seeds the next window)
    w.post_off = static_cast<int64_t>(c->post_slots.size());
    for (int64_t x = w.f0; x < w.f1; ++x)
      if (!(x > w.f0 && level[x - 1] < level[x]) || x == w.f1 - 1)
        c->post_slots.push_back(static_cast<int32_t>(x - w.f0));
    w.post_cnt = static_cast<int64_t>(c->post_slots.size()) - w.post_off;

    // Level-blocked schedule: every GOP a plain P chain (frame x at level l
    // predicted from x - 1 at level l - 1), k = 4 fused scoring, one parse
    // chunk, all GOPs per launch; L levels per launch while the level-0 halo
    // rows fit the LDS of two workgroups per CU.
    if (tb_L_max >= 2 && c->params.gops_per_launch <= 0 && w.chunk_end.size() == 1) {
      bool chain_ok = true;
      for (int64_t x = w.f0; x < w.f1 && chain_ok; ++x)
        chain_ok = intra[x] ? (level[x] == 0) : (ref[x] == x - 1 && x > w.f0 && level[x] == level[x - 1] + 1);
      if (chain_ok) {
        w.tb = true;
        int64_t lmax = 0;
        for (int64_t x = w.f0; x < w.f1; ++x) lmax = std::max(lmax, level[x]);
        for (int64_t l0 = 0; l0 <= lmax; l0 += tb_L_max) {
          const int L = static_cast<int>(std::min<int64_t>(tb_L_max, lmax + 1 - l0));
          const int64_t off = static_cast<int64_t>(c->tb_chains.size());
          int32_t cnt = 0;
          for (size_t g = 0; g < gop_start.size(); ++g) {
            const int64_t gs = gop_start[g], ge = (g + 1 < gop_start.size()) ? gop_start[g + 1] : w.f1;
            if (ge - gs <= l0) continue;
            for (int j = 0; j < L; ++j) {
              const int64_t x = gs + l0 + j;
              if (x < ge) {
                const bool fused_sad = x > w.f0 && level[x - 1] < level[x];
                c->tb_chains.push_back(make_int4(static_cast<int>(x - w.f0),
                                                 ref[x] >= 0 ? static_cast<int>(ref[x] - w.f0) : -1,
                                                 fused_sad ? static_cast<int>(x - 1 - w.f0) : -1, 0));
                if (x + 1 == ge || j + 1 == L) c->tb_last[static_cast<size_t>(x)] = 1;
              } else {
                c->tb_chains.push_back(make_int4(-1, -1, -1, 0));
              }
            }
            ++cnt;
          }
          w.tb_off.push_back(off);
          w.tb_cnt.push_back(cnt);
          w.tb_L.push_back(L);
        }
      }
    }
  }

  // the slice pass, one window per thread: frame slots, reference slots and
  // the launch-order sort (stable: decode order within a launch), so the
  // slices of launches [a, b) are one contiguous range
  {
    std::atomic<size_t> next{0};
    auto pass = [&]() {
      for (size_t wi = next++; wi < c->windows.size(); wi = next++) {
        const Window &w = c->windows[wi];
        std::vector<SliceDesc> sorted(static_cast<size_t>(w.s1 - w.s0));
        std::vector<int64_t> fill(wcnt[wi].begin(), wcnt[wi].end() - 1);
        for (int64_t x = w.f0; x < w.f1; ++x)
          for (int64_t sl = first_slice[x]; sl < first_slice[x] + n_slices[x]; ++sl) {
            SliceDesc d = c->slices[sl];
            d.slot = static_cast<int32_t>(x - w.f0);
            d.ref_slot = ref[x] >= 0 ? static_cast<int32_t>(ref[x] - w.f0) : -1;
            sorted[static_cast<size_t>(fill[launch_of[x]]++)] = d;
          }
        std::copy(sorted.begin(), sorted.end(), c->slices.begin() + w.s0);
      }
    };
    std::vector<std::thread> th;
    for (size_t i = 1; i < std::min<size_t>(static_cast<size_t>(read_threads()), c->windows.size()); ++i)
      th.emplace_back(pass);
    pass();
    for (auto &x : th) x.join();
  }

  // ---- device allocations and uploads
  c->open_lap(3);
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(vts::dmalloc(&c->d_slices, sizeof(SliceDesc) * c->slices.size()));
  HIP_TRY(hipMemcpy(c->d_slices, c->slices.data(), sizeof(SliceDesc) * c->slices.size(),
                    hipMemcpyHostToDevice));
  HIP_TRY(vts::dmalloc(&c->d_post, sizeof(int32_t) * std::max<size_t>(1, c->post_slots.size())));
  if (!c->post_slots.empty())
    HIP_TRY(hipMemcpy(c->d_post, c->post_slots.data(), sizeof(int32_t) * c->post_slots.size(),
                      hipMemcpyHostToDevice));
  if (!c->tb_chains.empty()) {
    HIP_TRY(vts::dmalloc(&c->d_tb, sizeof(int4) * c->tb_chains.size()));
    HIP_TRY(hipMemcpy(c->d_tb, c->tb_chains.data(), sizeof(int4) * c->tb_chains.size(), hipMemcpyHostToDevice));
  }
  HIP_TRY(vts::dmalloc(&c->d_levels, sizeof(int4) * c->level_frames.size()));
  HIP_TRY(hipMemcpy(c->d_levels, c->level_frames.data(), sizeof(int4) * c->level_frames.size(),
                    hipMemcpyHostToDevice));
  const int64_t nmb = static_cast<int64_t>(c->sps.mb_width) * c->sps.mb_height;
  c->ws_bytes = score_workspace_bytes(c->width, c->height, c->k, c->ring_frames);
  const int64_t tw = (c->width / c->k) * (c->height / c->k);
  for (int r = 0; r < c->n_rings; ++r) {
    HIP_TRY(vts::dmalloc(&c->d_cmd[r], static_cast<size_t>(c->ring_frames * nmb * 8)));
    HIP_TRY(vts::dmalloc(&c->d_surf[r], static_cast<size_t>(c->ring_frames * c->frame_stride + kPad)));
    HIP_TRY(vts::dmalloc(&c->d_ws[r], static_cast<size_t>(c->ws_bytes)));
    if (c->fused) HIP_TRY(vts::dmalloc(&c->d_thumb[r], static_cast<size_t>(c->ring_frames * tw + kPad)));
  }
  for (int r = 0; r < 2; ++r) HIP_TRY(vts::dmalloc(&c->d_last[r], static_cast<size_t>(tw + kPad)));
  HIP_TRY(vts::dmalloc(&c->d_err, sizeof(uint32_t)));
  HIP_TRY(vts::dmalloc(&c->d_score, sizeof(float) * c->n_frames));
  HIP_TRY(vts::dmalloc(&c->d_sad, sizeof(uint64_t) * c->n_frames));
  HIP_TRY(vts::dmalloc(&c->d_hist, sizeof(uint32_t) * 256 * c->n_frames));
  c->thumb_px = tw;
  HIP_TRY(vts::dmalloc(&c->d_rgb, static_cast<size_t>(3 * tw * c->n_frames + kPad)));
  VTS_TRY(streams_take(c));
  for (int g = 1; g < c->recon_groups; ++g) HIP_TRY(hipEventCreateWithFlags(&c->ev_grp[g - 1], hipEventDisableTiming));
  c->ev.resize(c->windows.size() * 6);
  for (auto &e2 : c->ev) HIP_TRY(hipEventCreate(&e2));
  int64_t nlev = 0;
  for (Window &w : c->windows) {
    w.ev0 = nlev;
    nlev += 2 * static_cast<int64_t>(w.lvl_off.size()) + static_cast<int64_t>(w.chunk_end.size());
  }
  c->lev.resize(static_cast<size_t>(nlev));
  for (auto &e2 : c->lev) HIP_TRY(hipEventCreate(&e2));
  HIP_TRY(hipEventCreate(&c->ev_start));
  HIP_TRY(hipEventCreate(&c->ev_end));
  c->open_lap(4);
  VTS_TRY(up.join());
  c->open_lap(5);
  return VTS_OK;
}

int open_common(int device, const Mp4Info &mp4, const uint8_t *mem, int64_t mem_size,
                const char *path, const vts_params *params, vts_ctx **out, double t_start) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(VTS_E_NODEVICE, "no HIP device visible");
  if (device < 0 || device >= ndev) return fail(VTS_E_NODEVICE, "device %d out of range", device);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess)
    return fail(VTS_E_NODEVICE, "hipGetDeviceProperties failed");
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(VTS_E_NODEVICE, "device %d is %s, not gfx950", device, prop.gcnArchName);
  vts_ctx *c = new vts_ctx;
  c->device = device;
  c->open_t = t_start;
  c->open_lap(0);
  if (params) c->params = *params;
  if (c->params.n_streams <= 0) c->params.n_streams = 2;
  if (c->params.cut_threshold <= 0) c->params.cut_threshold = 0.08f;
  const int rc = build(c, mp4, mem, mem_size, path);
  c->open_lap(6);
  for (int i = 0; i < 7; ++i) c->open_ms[7] += c->open_ms[i];
  if (rc != VTS_OK) {
    const std::string msg = last_error();
    vts_close(c);
    last_error() = msg;
    return rc;
  }
  *out = c;
  return VTS_OK;
}

}  // namespace

int vts::run_all(vts_ctx *c) {
  VTS_TRY(submit_all(c));
  return finish_all(c);
}

int vts::finish_all(vts_ctx *c) {
  if (!c->pending) return VTS_OK;
  c->pending = false;
  return c->general ? finish_general(c) : finish_subset(c);
}

// Enqueue one run (every window's decode + score) on the session's streams;
// finish_all waits for it, reads the error word and the timings, and re-runs
// where the device asked for it (level-blocking halo, general decoder, arena).
int vts::submit_all(vts_ctx *c) {
  if (c->pending) VTS_TRY(finish_all(c));
  if (c->general) {
    VTS_TRY(submit_general(c));
    c->pending = true;
    return VTS_OK;
  }
  HIP_TRY(hipSetDevice(c->device));
  if (!c->h_err) HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&c->h_err), sizeof(uint32_t)));
  HIP_TRY(hipMemsetAsync(c->d_err, 0, sizeof(uint32_t), c->s_dec));
  HIP_TRY(hipEventRecord(c->ev_start, c->s_dec));
  HIP_TRY(hipStreamWaitEvent(c->s_score, c->ev_start, 0));
  const int64_t nmb = static_cast<int64_t>(c->sps.mb_width) * c->sps.mb_height;
  hipStream_t sd = c->s_dec;
  // level-blocked launches store every frame only on request (or for the
  // transcoder, which downscales every frame from the ring)
  const bool keep = c->params.keep_frames > 0 || c->small.on;
  c->tb_ran_sparse = false;
  // one window: one stream (nothing to overlap, and HIP event timing of each
  // stage stays on a single queue)
  hipStream_t ss = (c->params.n_streams >= 2 && c->windows.size() > 1) ? c->s_score : c->s_dec;
  const size_t nw = c->windows.size();
  for (size_t wi = 0; wi < nw; ++wi) {
    const Window &w = c->windows[wi];
    const int r = static_cast<int>(wi % c->n_rings);
    hipEvent_t *E = &c->ev[wi * 6];  // 0 parse start, 1 parsed, 2 decoded, 3 score start, 4 scored
    hipEvent_t *LE = &c->lev[static_cast<size_t>(w.ev0)];  // per launch (start, end), then per chunk
    const size_t nl = w.lvl_off.size();
    hipStream_t sp = c->s_parse;
    // the ring's command / surface buffers are free once the window that used
    // them two steps ago has been scored
    if (wi >= static_cast<size_t>(c->n_rings)) {
      HIP_TRY(hipStreamWaitEvent(sd, c->ev[(wi - c->n_rings) * 6 + 4], 0));
      HIP_TRY(hipStreamWaitEvent(sp, c->ev[(wi - c->n_rings) * 6 + 4], 0));
    }
    // Slice parsing on its own stream in chunks of launches: the parser is
    // latency-bound (one lane per slice), reconstruction HBM-bound, so parsing
    // chunk j+1 overlaps reconstructing the launches of chunk j.
    HIP_TRY(hipStreamWaitEvent(sp, c->ev_start, 0));
    HIP_TRY(hipEventRecord(E[0], sp));
    // commands carry the run's epoch; stale ones read as absent, so the ring
    // is cleared only on first use and before an epoch could come round again
    const int64_t run = c->run_no++;
    const uint32_t epoch = 1u + static_cast<uint32_t>(run % kCmdEpochs);
    if (c->ring_cleared_at[r] < 0 || run - c->ring_cleared_at[r] >= kCmdEpochs) {
      HIP_TRY(hipMemsetAsync(c->d_cmd[r], 0, static_cast<size_t>(c->ring_frames * nmb * 8), sp));
      c->ring_cleared_at[r] = run;
    }
    {
      ParseArgs pa{};
      pa.epoch = epoch;
      pa.es = c->d_es;
      pa.cmd = c->d_cmd[r];
      pa.err = c->d_err;
      pa.prm = c->prm;
      int32_t l0 = 0;
      for (size_t j = 0; j < w.chunk_end.size(); ++j) {
        const int32_t l1 = w.chunk_end[j];
        const int64_t a0 = w.lvl_s0[l0];
        const int64_t a1 = (static_cast<size_t>(l1) < nl) ? w.lvl_s0[l1] : w.s1;
        pa.slices = c->d_slices + a0;
        pa.n_slices = static_cast<int32_t>(a1 - a0);
        VTS_TRY(parse_launch(pa, sp));
        HIP_TRY(hipEventRecord(LE[2 * nl + j], sp));
        l0 = l1;
      }
    }
    HIP_TRY(hipEventRecord(E[1], sp));
    ReconArgs ra{};
    ra.es = c->d_es;
    ra.cmd = c->d_cmd[r];
    ra.surf = c->d_surf[r];
    ra.frame_stride = c->frame_stride;
    ra.pitch = c->pitch;
    ra.mb_width = c->sps.mb_width;
    ra.mb_height = c->sps.mb_height;
    ra.epoch = epoch;
    ra.err = c->d_err;
    const int tw = c->width / c->k, th = c->height / c->k;
    FusedArgs fa{};
    if (c->fused) {
      VTS_TRY(clear_accum_launch(c->d_hist + w.f0 * 256, c->d_sad + w.f0, w.f1 - w.f0, sd));
      fa.r = ra;
      fa.frame0 = w.f0;
      fa.w = tw;
      fa.h = th;
      fa.wgs_per_frame = static_cast<int32_t>((nmb + 255) / 256);
      fa.thumb = c->d_thumb[r];
      fa.rgb = c->d_rgb;
      fa.hist = c->d_hist;
      fa.sad = c->d_sad;
    }
    size_t j = 0;
    const bool tb = c->fused && w.tb && !c->tb_off;
    if (tb) {
      // level-blocked launches (one parse chunk: wait for all of it)
      HIP_TRY(hipStreamWaitEvent(sd, LE[2 * nl], 0));
      HIP_TRY(hipEventRecord(LE[0], sd));
      TbArgs ta{};
      ta.f = fa;
      ta.keep = keep ? 1 : 0;
      for (size_t i = 0; i < w.tb_off.size(); ++i) {
        ta.chains = c->d_tb + w.tb_off[i];
        ta.L = w.tb_L[i];
        VTS_TRY(tb_launch(ta, w.tb_cnt[i], sd));
      }
      HIP_TRY(hipEventRecord(LE[2 * (nl - 1) + 1], sd));
    }
    if (!tb && w.grp.size() > 1) {
      // Interleaved GOP groups (one parse chunk): group g's level launches on
      // its own stream, so one group's launch tail overlaps the others' work.
      const int ng = static_cast<int>(w.grp.size());
      // group g waits for its own parse chunk (or the single one)
      const bool per_grp = w.chunk_end.size() == w.grp.size();
      HIP_TRY(hipStreamWaitEvent(sd, LE[2 * nl], 0));
      HIP_TRY(hipEventRecord(LE[0], sd));
      // LE[0] follows clear_accum on sd (this window's histograms / SADs are
      // zeroed before any group adds to them); with per-group parse chunks a
      // group also waits for its own chunk
      for (int g = 1; g < ng; ++g) {
        HIP_TRY(hipStreamWaitEvent(c->s_grp[g - 1], LE[0], 0));
        if (per_grp) HIP_TRY(hipStreamWaitEvent(c->s_grp[g - 1], LE[2 * nl + g], 0));
      }
      for (size_t i = 0;; ++i) {
        bool any = false;
        for (int g = 0; g < ng; ++g) {
          const size_t l = static_cast<size_t>(w.grp[g]) + i;
          const size_t end = g + 1 < ng ? static_cast<size_t>(w.grp[g + 1]) : nl;
          if (l >= end) continue;
          any = true;
          fa.r.frames = c->d_levels + w.lvl_off[l];
          VTS_TRY(fused_launch(fa, c->k, w.lvl_cnt[l], g == 0 ? sd : c->s_grp[g - 1]));
        }
        if (!any) break;
      }
      for (int g = 1; g < ng; ++g) {
        HIP_TRY(hipEventRecord(c->ev_grp[g - 1], c->s_grp[g - 1]));
        HIP_TRY(hipStreamWaitEvent(sd, c->ev_grp[g - 1], 0));
      }
      HIP_TRY(hipEventRecord(LE[2 * (nl - 1) + 1], sd));
    }
    for (size_t l = 0; l < nl && !tb && w.grp.size() <= 1; ++l) {
      if (l == 0 || static_cast<int32_t>(l) == w.chunk_end[j - 1]) {
        HIP_TRY(hipStreamWaitEvent(sd, LE[2 * nl + j++], 0));  // this launch's slices are parsed
        // reconstruct span starts once its first launch may run (a timing
        // event between launches costs ~25 us on ROCm, so only at chunk edges)
        HIP_TRY(hipEventRecord(LE[2 * l], sd));
      }
      if (c->fused) {
        fa.r.frames = c->d_levels + w.lvl_off[l];
        VTS_TRY(fused_launch(fa, c->k, w.lvl_cnt[l], sd));
      } else {
        ra.frames = c->d_levels + w.lvl_off[l];
        VTS_TRY(recon_launch(ra, w.lvl_cnt[l], sd));
      }
      if (l + 1 == nl || static_cast<int32_t>(l + 1) == w.chunk_end[j - 1])
        HIP_TRY(hipEventRecord(LE[2 * l + 1], sd));
    }
    // transcode: the 360p copy of the window's frames, while they are in the ring
    if (c->small.on) VTS_TRY(small_window(c, r, w.f0, w.f1, sd));
    HIP_TRY(hipEventRecord(E[2], sd));
    HIP_TRY(hipStreamWaitEvent(ss, E[2], 0));
    HIP_TRY(hipEventRecord(E[3], ss));
    if (c->fused) {
      ThumbSadArgs t{};
      t.thumb = c->d_thumb[r];
      t.prev_luma = wi > 0 ? c->d_last[(wi - 1) & 1] : nullptr;
      t.last_luma = c->d_last[wi & 1];
      t.frame0 = w.f0;
      t.n_frames = w.f1 - w.f0;
      t.w = tw;
      t.h = th;
      t.sad = c->d_sad;
      t.score = c->d_score;
      t.list = c->d_post + w.post_off;
      t.n_list = w.post_cnt;
      VTS_TRY(thumb_sad_launch(t, ss));
      VTS_TRY(sad_score_launch(c->d_sad, c->d_score, w.f0, w.f1 - w.f0,
                               static_cast<int64_t>(tw) * th, ss));
    } else {
      vts_score_desc d{};
      d.nv12 = c->d_surf[r];
      d.frame_stride = c->frame_stride;
      d.n_frames = w.f1 - w.f0;
      d.width = c->width;
      d.height = c->height;
      d.pitch = c->pitch;
      d.uv_row_offset = c->coded_h;
      d.k = c->k;
      d.rgb = c->d_rgb + 3 * c->thumb_px * w.f0;
      d.hist = c->d_hist + w.f0 * 256;
      d.sad = c->d_sad + w.f0;
      d.score = c->d_score + w.f0;
      d.prev_luma = wi > 0 ? c->d_last[(wi - 1) & 1] : nullptr;
      d.last_luma = c->d_last[wi & 1];
      d.workspace = c->d_ws[r];
      d.workspace_bytes = c->ws_bytes;
      VTS_TRY(score_launch(&d, ss));
    }
    HIP_TRY(hipEventRecord(E[4], ss));
  }
  HIP_TRY(hipStreamWaitEvent(sd, c->ev[(nw - 1) * 6 + 4], 0));
  HIP_TRY(hipMemcpyAsync(c->h_err, c->d_err, sizeof(uint32_t), hipMemcpyDeviceToHost, sd));
  HIP_TRY(hipEventRecord(c->ev_end, sd));
  c->pending = true;
  return VTS_OK;
}

int vts::finish_subset(vts_ctx *c) {
  const size_t nw = c->windows.size();
  const bool keep = c->params.keep_frames > 0 || c->small.on;
  HIP_TRY(hipEventSynchronize(c->ev_end));
  const uint32_t err = *c->h_err;
  // timings
  float ms = 0;
  HIP_TRY(hipEventElapsedTime(&ms, c->ev_start, c->ev_end));
  c->timings[0] = ms;
  c->timings[1] = c->timings[2] = c->timings[3] = 0;
  for (size_t wi = 0; wi < nw; ++wi) {
    hipEvent_t *E = &c->ev[wi * 6];
    float a = 0, s = 0;
    HIP_TRY(hipEventElapsedTime(&a, E[0], E[1]));
    HIP_TRY(hipEventElapsedTime(&s, E[3], E[4]));
    c->timings[1] += a;
    c->timings[3] += s;
    // reconstruct: the spans of each chunk's launches on the decode stream
    // (from after the wait for the chunk's parse to its last launch), so
    // waits for parsing are not counted as kernel time
    const Window &w = c->windows[wi];
    const hipEvent_t *LE = &c->lev[static_cast<size_t>(w.ev0)];
    int32_t l0 = 0;
    for (int32_t l1 : w.chunk_end) {
      float b = 0;
      if (w.grp.size() > 1) {  // interleaved groups: one span over all launches
        if (l1 != w.chunk_end.back()) continue;
        l0 = 0;
      }
      HIP_TRY(hipEventElapsedTime(&b, LE[2 * l0], LE[2 * (l1 - 1) + 1]));
      c->timings[2] += b;
      l0 = l1;
    }
  }
  c->last_window_done = static_cast<int64_t>(nw) - 1;
  if (err & DEC_W_LEVEL_RANGE) {
    // motion beyond a level-blocked launch's halo: redo with one launch per level
    c->tb_off = true;
    return run_all(c);
  }
  for (const Window &w : c->windows) c->tb_ran_sparse |= c->fused && w.tb && !c->tb_off && !keep;
  // decoder = auto: syntax outside the subset kernels -> the general decoder
  constexpr uint32_t kSubsetMiss = DEC_E_MB_TYPE | DEC_E_RESIDUAL | DEC_E_SUBPEL | DEC_E_MULTIREF |
                                   DEC_E_DEBLOCK | DEC_E_REFLIST | DEC_E_MMCO | DEC_E_EPB_IN_PCM;
  if ((err & kSubsetMiss) && c->params.decoder == 0) {  // small.on too: run_general downscales
    VTS_TRY(switch_to_general(c));
    return run_all(c);
  }
  if (err) {
    c->have_results = false;
    return fail(VTS_E_DECODE, "device decoder: %s", describe_decode_error(err).c_str());
  }
  c->have_results = true;
  c->host_scores.clear();
  return VTS_OK;
}

int vts::fetch_scores(vts_ctx *c) {
  VTS_TRY(finish_all(c));  // a submitted run first
  if (!c->host_scores.empty()) return VTS_OK;
  c->host_scores.resize(static_cast<size_t>(c->n_frames));
  HIP_TRY(hipMemcpy(c->host_scores.data(), c->d_score, sizeof(float) * c->n_frames,
                    hipMemcpyDeviceToHost));
  return VTS_OK;
}

extern "C" int vts_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

extern "C" int vts_open(int device, const char *path, const vts_params *params, vts_ctx **out) {
  clear_error();
  if (!path || !out) return fail(VTS_E_INVALID, "NULL argument");
  *out = nullptr;
  const double t0 = now_s();
  Mp4Info mp4;
  const std::string e = mp4_parse_file(path, &mp4);
  if (!e.empty()) return fail(VTS_E_FORMAT, "%s", e.c_str());
  return open_common(device, mp4, nullptr, 0, path, params, out, t0);
}

extern "C" int vts_open_memory(int device, const uint8_t *data, int64_t size, const vts_params *params,
                               vts_ctx **out) {
  clear_error();
  if (!data || size <= 0 || !out) return fail(VTS_E_INVALID, "bad argument");
  *out = nullptr;
  const double t0 = now_s();
  Mp4Info mp4;
  const std::string e = mp4_parse_memory(data, size, &mp4);
  if (!e.empty()) return fail(VTS_E_FORMAT, "%s", e.c_str());
  return open_common(device, mp4, data, size, nullptr, params, out, t0);
}

extern "C" int vts_info(const vts_ctx *c, vts_video_info *info) {
  clear_error();
  if (!c || !info) return fail(VTS_E_INVALID, "NULL argument");
  *info = c->info;
  return VTS_OK;
}

extern "C" int vts_run(vts_ctx *c) {
  clear_error();
  if (!c) return fail(VTS_E_INVALID, "NULL ctx");
  return run_all(c);
}

extern "C" int vts_run_async(vts_ctx *c) {
  clear_error();
  if (!c) return fail(VTS_E_INVALID, "NULL ctx");
  return submit_all(c);
}

extern "C" int vts_wait(vts_ctx *c) {
  clear_error();
  if (!c) return fail(VTS_E_INVALID, "NULL ctx");
  return finish_all(c);
}

extern "C" int vts_score(vts_ctx *c, float *scores, uint32_t *hist, uint64_t *sad, int64_t *pts,
                         int64_t cap, int64_t *n_frames) {
  clear_error();
  if (!c || !n_frames) return fail(VTS_E_INVALID, "NULL argument");
  *n_frames = c->n_frames;
  if (!scores || cap < c->n_frames)
    return fail(VTS_E_CAPACITY, "need %lld frames", static_cast<long long>(c->n_frames));
  VTS_TRY(run_all(c));
  VTS_TRY(fetch_scores(c));
  std::memcpy(scores, c->host_scores.data(), sizeof(float) * c->n_frames);
  if (hist)
    HIP_TRY(hipMemcpy(hist, c->d_hist, sizeof(uint32_t) * 256 * c->n_frames, hipMemcpyDeviceToHost));
  if (sad) HIP_TRY(hipMemcpy(sad, c->d_sad, sizeof(uint64_t) * c->n_frames, hipMemcpyDeviceToHost));
  if (pts) std::memcpy(pts, c->pts.data(), sizeof(int64_t) * c->n_frames);
  return VTS_OK;
}

extern "C" int vts_scene_cuts(vts_ctx *c, int64_t *frame_idx, int64_t cap, int64_t *n_out) {
  clear_error();
  if (!c || !n_out) return fail(VTS_E_INVALID, "NULL argument");
  VTS_TRY(finish_all(c));  // a submitted run completes first
  if (!c->have_results) return fail(VTS_E_INVALID, "run vts_score/vts_run first");
  VTS_TRY(fetch_scores(c));
  int64_t n = 0;
  for (int64_t i = 0; i < c->n_frames; ++i)
    if (c->host_scores[i] > c->params.cut_threshold) {
      if (frame_idx && n < cap) frame_idx[n] = i;
      ++n;
    }
  *n_out = n;
  if (n > cap) return fail(VTS_E_CAPACITY, "need %lld", static_cast<long long>(n));
  return VTS_OK;
}

extern "C" int vts_boundary_frames(vts_ctx *c, const double *times, int64_t n, int64_t *frame_idx) {
  clear_error();
  if (!c) return fail(VTS_E_INVALID, "NULL ctx");
  return vts_boundary_frames_pts(c->pts.data(), c->n_frames, c->info.track_timescale, times, n,
                                 frame_idx);
}

extern "C" int vts_frame_pts(const vts_ctx *c, int64_t *pts, int64_t cap, int64_t *n_out) {
  clear_error();
  if (!c || !n_out) return fail(VTS_E_INVALID, "NULL argument");
  *n_out = c->n_frames;
  if (!pts || cap < c->n_frames) return fail(VTS_E_CAPACITY, "need %lld", static_cast<long long>(c->n_frames));
  std::memcpy(pts, c->pts.data(), sizeof(int64_t) * static_cast<size_t>(c->n_frames));
  return VTS_OK;
}

extern "C" int vts_get_frame_nv12(vts_ctx *c, int64_t frame, uint8_t *out, int64_t out_bytes) {
  clear_error();
  if (!c || !out) return fail(VTS_E_INVALID, "NULL argument");
  VTS_TRY(finish_all(c));
  const int64_t need = static_cast<int64_t>(c->width) * c->height * 3 / 2;
  if (out_bytes < need) return fail(VTS_E_CAPACITY, "need %lld bytes", static_cast<long long>(need));
  if (c->last_window_done < 0) return fail(VTS_E_INVALID, "nothing decoded yet");
  const int64_t first_resident = std::max<int64_t>(0, c->last_window_done - c->n_rings + 1);
  for (int64_t wi = first_resident; wi <= c->last_window_done; ++wi) {
    const Window &w = c->windows[static_cast<size_t>(wi)];
    if (frame < w.f0 || frame >= w.f1) continue;
    if (c->surf_pool)
      return fail(VTS_E_INVALID,
                  "frame %lld is not kept: the general decoder recycles surfaces once a picture is scored "
                  "(open with vts_params.keep_frames = 1, or VTS_SURF_POOL=0)",
                  static_cast<long long>(frame));
    if (c->tb_ran_sparse && w.tb && !c->tb_last[static_cast<size_t>(frame)])
      return fail(VTS_E_INVALID,
                  "frame %lld was decoded in LDS only (level-blocked launches keep each block's last "
                  "frame; open with vts_params.keep_frames = 1 or level_block = 1)",
                  static_cast<long long>(frame));
    const uint8_t *base = c->d_surf[wi % c->n_rings] + (frame - w.f0) * c->frame_stride;
    HIP_TRY(hipMemcpy2D(out, c->width, base, c->pitch, c->width, c->height, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy2D(out + static_cast<int64_t>(c->width) * c->height, c->width,
                        base + static_cast<int64_t>(c->pitch) * c->coded_h, c->pitch, c->width,
                        c->height / 2, hipMemcpyDeviceToHost));
    return VTS_OK;
  }
  return fail(VTS_E_INVALID, "frame %lld is not resident", static_cast<long long>(frame));
}

extern "C" int vts_get_thumbnail_rgb(vts_ctx *c, int64_t frame, uint8_t *out, int64_t out_bytes) {
  clear_error();
  if (!c || !out) return fail(VTS_E_INVALID, "NULL argument");
  VTS_TRY(finish_all(c));
  VTS_TRY(finish_all(c));  // a submitted run completes first
  if (!c->have_results) return fail(VTS_E_INVALID, "run vts_score/vts_run first");
  if (frame < 0 || frame >= c->n_frames) return fail(VTS_E_INVALID, "frame out of range");
  const int64_t need = 3 * c->thumb_px;
  if (out_bytes < need) return fail(VTS_E_CAPACITY, "need %lld bytes", static_cast<long long>(need));
  HIP_TRY(hipMemcpy(out, c->d_rgb + need * frame, static_cast<size_t>(need), hipMemcpyDeviceToHost));
  return VTS_OK;
}

void vts_ctx::open_lap(int k) {
  const double t = now_s();
  open_ms[k] += (t - open_t) * 1e3;
  open_t = t;
}

extern "C" int vts_open_timings(const vts_ctx *c, double *ms, int32_t cap) {
  clear_error();
  if (!c || !ms || cap < 0) return fail(VTS_E_INVALID, "bad argument");
  for (int i = 0; i < std::min(cap, 8); ++i) ms[i] = c->open_ms[i];
  return 8;
}

extern "C" int vts_last_timings(const vts_ctx *c, double *ms4) {
  clear_error();
  if (!c || !ms4) return fail(VTS_E_INVALID, "NULL argument");
  for (int i = 0; i < 4; ++i) ms4[i] = c->timings[i];
  return VTS_OK;
}

extern "C" int64_t vts_schedule_info(const vts_ctx *c, int32_t what) {
  clear_error();
  if (!c) return fail(VTS_E_INVALID, "NULL ctx");
  switch (what) {
    case 0: {
      int64_t n = 0;
      for (const Window &w : c->windows) n += static_cast<int64_t>(w.lvl_off.size());
      return n;
    }
    case 1: return static_cast<int64_t>(c->windows.size());
    case 2: return static_cast<int64_t>(c->slices.size());
    case 3: return c->ring_frames;
    case 4: return c->fused ? 1 : 0;
    case 5: {  // level-blocked launches (0 when the per-level schedule runs)
      if (c->tb_off || !c->fused) return 0;
      int64_t n = 0;
      for (const Window &w : c->windows) n += w.tb ? static_cast<int64_t>(w.tb_off.size()) : 0;
      return n;
    }
    case 6: {  // chains over all level-blocked launches
      if (c->tb_off || !c->fused) return 0;
      int64_t n = 0;
      for (const Window &w : c->windows)
        if (w.tb)
          for (int32_t k : w.tb_cnt) n += k;
      return n;
    }
    case 7: return c->tb_off ? 0 : static_cast<int64_t>(c->tb_chains.size());  // chain slots (levels x chains)
    case 8: return c->general ? 1 : 0;
    case 9: return c->arena_reruns;                 // runs repeated with a larger coefficient arena
    case 10: return c->arena_blocks;                // coefficient blocks per ring (general decoder)
    case 11: return c->surf_pool ? c->surf_count : 0;  // recycled surfaces per ring (general decoder)
    case 12: return c->s_dec ? c->stream_kind : -1;   // stream set: 0 plain, 1 own hardware queues
    case 13: {  // CABAC: slices parsed in the windows' long-slice launches (0: one launch per window)
      int64_t n = 0;
      for (const Window &w : c->windows) n += w.plong;
      return n;
    }
    default: return fail(VTS_E_INVALID, "unknown schedule field %d", what);
  }
}

extern "C" int vts_close(vts_ctx *c) {
  if (!c) return VTS_OK;
  (void)hipSetDevice(c->device);
  if (c->pending && c->ev_end) (void)hipEventSynchronize(c->ev_end);  // a submitted run nobody waited for
  if (c->h_err) (void)hipHostFree(c->h_err);
  if (c->s_dec) (void)hipStreamSynchronize(c->s_dec);
  if (c->s_score) (void)hipStreamSynchronize(c->s_score);
  if (c->s_parse) (void)hipStreamSynchronize(c->s_parse);
  for (hipStream_t g : c->s_grp)
    if (g) (void)hipStreamSynchronize(g);
  auto f = [](void *p) {
    if (p) vts::dfree(p);
  };
  f(c->d_es);
  f(c->d_slices);
  f(c->d_levels);
  f(c->d_tb);
  f(c->d_post);
  for (int r = 0; r < 2; ++r) {
    f(c->d_cmd[r]);
    f(c->d_surf[r]);
    f(c->d_ws[r]);
    f(c->d_last[r]);
    f(c->d_thumb[r]);
  }
  f(c->d_err);
  f(c->d_score);
  f(c->d_sad);
  f(c->d_hist);
  f(c->d_rgb);
  f(c->small.d);
  f(c->small.d_taps);
  f(c->d_fslices);
  f(c->d_rbsp);
  f(c->d_rbsp_len);
  f(c->d_scale);
  f(c->d_exts);
  f(c->d_porder);
  f(c->d_porder_m);
  f(c->d_pneed);
  f(c->d_dslots);
  f(c->d_surf_of);
  f(c->d_arena_top);
  for (int r = 0; r < 2; ++r) {
    f(c->d_recs[r]);
    f(c->d_recs1[r]);
    f(c->d_ilvl[r]);
    f(c->d_pdone[r]);
    f(c->d_dbk[r]);
    f(c->d_arena[r]);
  }
  for (auto e : c->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto e : c->lev)
    if (e) (void)hipEventDestroy(e);
  for (auto e : c->ev_bs)
    if (e) (void)hipEventDestroy(e);
  for (auto e : c->ev_px)
    if (e) (void)hipEventDestroy(e);
  if (c->s_px) {
    (void)hipStreamSynchronize(c->s_px);
    (void)hipStreamDestroy(c->s_px);
  }
  if (c->ev_start) (void)hipEventDestroy(c->ev_start);
  if (c->ev_end) (void)hipEventDestroy(c->ev_end);
  for (int g = vts_ctx::kMaxGroups - 2; g >= 0; --g) {
    if (c->s_grp[g]) (void)hipStreamSynchronize(c->s_grp[g]);
    if (c->ev_grp[g]) (void)hipEventDestroy(c->ev_grp[g]);
  }
  streams_give(c);  // back to the pool as the set it came as
  delete c;
  return VTS_OK;
}
