// batch.cpp — the batch entry points of the C ABI (vtseg.h "batch"): the
// reference's sequential batch loop (src/pipeline.py:376-393 -> one
// ContentAnalyzer.analyze_video per URL) as one call per process, video i on
// rank i % world, records exchanged over RCCL.  The C twin of
// vtseg.batch.plan_batch (same records, same order of work, same failure
// rules), for hosts that drive libvtseg without Python / torch.distributed.
//
// RCCL is loaded on first use (dlopen "librccl.so.1"): a process that never
// passes a communicator never maps it, and a process that already holds one
// (torch's) gets that same library back by its soname.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"
#include "vtseg.h"

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    const hipError_t e_ = (expr);                                                  \
    if (e_ != hipSuccess) return vts::fail(VTS_E_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

namespace vts {
namespace {

// ------------------------------------------------------------ RCCL loader
struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclCommCount) comm_count = nullptr;
  decltype(&ncclCommUserRank) comm_user_rank = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  std::string error;
};

const Rccl &rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char *e = dlerror();
      r.error = std::string("dlopen librccl: ") + (e ? e : "not found");
      return;
    }
    auto sym = [&](auto &fn, const char *name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      if (!fn && r.error.empty()) r.error = std::string("librccl lacks ") + name;
    };
    sym(r.get_unique_id, "ncclGetUniqueId");
    sym(r.comm_init_rank, "ncclCommInitRank");
    sym(r.comm_destroy, "ncclCommDestroy");
    sym(r.comm_count, "ncclCommCount");
    sym(r.comm_user_rank, "ncclCommUserRank");
    sym(r.all_gather, "ncclAllGather");
    sym(r.error_string, "ncclGetErrorString");
  });
  return r;
}

#define RCCL_TRY(call)                                                                              \
  do {                                                                                              \
    const ncclResult_t rc_ = (call);                                                                \
    if (rc_ != ncclSuccess) return fail(VTS_E_HIP, "%s: %s", #call, vts::rccl().error_string(rc_));      \
  } while (0)

struct Comm {
  ncclComm_t comm = nullptr;
  int world = 1, rank = 0, device = 0;
  hipStream_t stream = nullptr;
};

// all-gather of `count` elements of `bytes` each per rank through the
// communicator's device: host in -> host out (world x count)
int all_gather(Comm *c, const void *in, void *out, size_t count, size_t bytes, ncclDataType_t type) {
  HIP_TRY(hipSetDevice(c->device));
  void *din = nullptr, *dout = nullptr;
  const size_t nin = std::max<size_t>(1, count * bytes), nout = nin * static_cast<size_t>(c->world);
  HIP_TRY(hipMalloc(&din, nin));
  if (hipMalloc(&dout, nout) != hipSuccess) {
    (void)hipFree(din);
    return fail(VTS_E_HIP, "hipMalloc (all-gather)");
  }
  int rc = VTS_OK;
  if (hipMemcpyAsync(din, in, count * bytes, hipMemcpyHostToDevice, c->stream) != hipSuccess)
    rc = fail(VTS_E_HIP, "hipMemcpyAsync (all-gather in)");
  if (rc == VTS_OK && count) {
    const ncclResult_t r = rccl().all_gather(din, dout, count, type, c->comm, c->stream);
    if (r != ncclSuccess) rc = fail(VTS_E_HIP, "ncclAllGather: %s", rccl().error_string(r));
  }
  if (rc == VTS_OK && hipMemcpyAsync(out, dout, count * bytes * static_cast<size_t>(c->world), hipMemcpyDeviceToHost,
                                     c->stream) != hipSuccess)
    rc = fail(VTS_E_HIP, "hipMemcpyAsync (all-gather out)");
  if (hipStreamSynchronize(c->stream) != hipSuccess && rc == VTS_OK) rc = fail(VTS_E_HIP, "all-gather stream");
  (void)hipFree(din);
  (void)hipFree(dout);
  return rc;
}

constexpr int kRec = 4;  // int64 per video: n_segments, n_cuts, duration_us, scoring failed (0/1)

}  // namespace
}  // namespace vts

struct vts_batch {
  int64_t n = 0;
  std::vector<vts_batch_record> rec;
  std::vector<std::vector<int64_t>> seg_frames, cut_frames;  // per video (every rank's)
  std::vector<std::vector<double>> cut_times;
  std::map<int64_t, std::string> errors;  // this rank's videos
};

using vts::fail;

extern "C" int vts_rccl_unique_id(uint8_t *id) {
  if (!id) return fail(VTS_E_INVALID, "NULL id");
  const vts::Rccl &r = vts::rccl();
  if (!r.error.empty()) return fail(VTS_E_HIP, "%s", r.error.c_str());
  ncclUniqueId u;
  RCCL_TRY(r.get_unique_id(&u));
  static_assert(sizeof(u) == VTS_RCCL_ID_BYTES, "ncclUniqueId size");
  std::memcpy(id, &u, sizeof u);
  return VTS_OK;
}

extern "C" int vts_rccl_comm_init(int32_t device, int32_t world, int32_t rank, const uint8_t *id, void **comm) {
  if (!id || !comm || world < 1 || rank < 0 || rank >= world) return fail(VTS_E_INVALID, "bad communicator arguments");
  *comm = nullptr;
  const vts::Rccl &r = vts::rccl();
  if (!r.error.empty()) return fail(VTS_E_HIP, "%s", r.error.c_str());
  HIP_TRY(hipSetDevice(device));
  auto *c = new vts::Comm;
  c->world = world;
  c->rank = rank;
  c->device = device;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  const ncclResult_t e = r.comm_init_rank(&c->comm, world, u, rank);
  if (e != ncclSuccess) {
    delete c;
    return fail(VTS_E_HIP, "ncclCommInitRank: %s", r.error_string(e));
  }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    (void)r.comm_destroy(c->comm);
    delete c;
    return fail(VTS_E_HIP, "hipStreamCreate");
  }
  *comm = c;
  return VTS_OK;
}

extern "C" int vts_rccl_comm_destroy(void *comm) {
  if (!comm) return VTS_OK;
  auto *c = static_cast<vts::Comm *>(comm);
  int rc = VTS_OK;
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->comm && vts::rccl().comm_destroy(c->comm) != ncclSuccess) rc = fail(VTS_E_HIP, "ncclCommDestroy");
  delete c;
  return rc;
}

namespace {

struct Local {  // one of this rank's videos
  int64_t j = 0, i = 0;
  double duration = 0;
  std::vector<vts_segment> segs;
  std::vector<int64_t> seg_frames, cut_frames;
  std::vector<double> cut_times;
  int64_t n_cuts = -1;
  bool failed = false;
};

// plan_batch's _segments: plan_segments_with_budget, then plan_segments with
// its segment duration and overlap (none when the duration is <= 0)
int plan_one(Local &v, const vts_budget_cfg *cfg, int64_t api_count) {
  vts_plan plan{};
  int rc = vts_plan_with_budget(v.duration, cfg, api_count, &plan);
  if (rc != VTS_OK) return rc;
  v.segs.clear();
  if (plan.segment_duration <= 0) return VTS_OK;
  int64_t need = 0;
  rc = vts_plan_segments(v.duration, static_cast<double>(plan.segment_duration), static_cast<double>(plan.overlap),
                         nullptr, 0, &need);
  if (rc != VTS_OK && rc != VTS_E_CAPACITY) return rc;
  v.segs.resize(static_cast<size_t>(need));
  return vts_plan_segments(v.duration, static_cast<double>(plan.segment_duration), static_cast<double>(plan.overlap),
                           v.segs.data(), need, &need);
}

}  // namespace

extern "C" int vts_batch_run(const char *const *paths, int64_t n, const vts_budget_cfg *cfg,
                             const vts_batch_params *bp, vts_batch **out) {
  if (!paths || n < 0 || !cfg || !bp || !out) return fail(VTS_E_INVALID, "NULL argument");
  *out = nullptr;
  auto *comm = static_cast<vts::Comm *>(bp->rccl_comm);
  const int world = comm ? comm->world : 1, rank = comm ? comm->rank : 0;
  const int64_t per = (n + world - 1) / world;
  std::vector<Local> mine;
  for (int64_t i = rank, j = 0; i < n; i += world, ++j) {
    Local v;
    v.j = j;
    v.i = i;
    // probe_duration (video_utils.py): the native mvhd rule; no answer -> 0.0
    double s = 0.0;
    if (!paths[i]) return fail(VTS_E_INVALID, "NULL path %lld", static_cast<long long>(i));
    if (vts_probe_duration(paths[i], &s) != VTS_OK || !(s > 0.0)) s = 0.0;
    v.duration = s;
    const int rc = plan_one(v, cfg, bp->current_api_count);
    if (rc != VTS_OK) return rc;
    mine.push_back(std::move(v));
  }
  auto *b = new vts_batch;
  b->n = n;
  if (bp->score) {
    // every local session's run submitted before earlier ones are waited for;
    // at most max_in_flight open at once, an open that fails while others run
    // retried once after they drain; a failure is the video's, never the batch's
    vts_params prm{};
    prm.n_streams = 2;
    prm.cut_threshold = 0.08f;
    struct Running {
      Local *v;
      vts_ctx *ctx;
    };
    std::deque<Running> running;
    auto fail_video = [&](Local &v) {
      b->errors[v.i] = vts_last_error();
      v.failed = true;
      v.n_cuts = -1;
    };
    auto finish_oldest = [&]() {
      Running r = running.front();
      running.pop_front();
      Local &v = *r.v;
      int rc = vts_wait(r.ctx);
      vts_video_info info{};
      std::vector<int64_t> pts;
      if (rc == VTS_OK) rc = vts_info(r.ctx, &info);
      if (rc == VTS_OK) {
        std::vector<int64_t> cuts(static_cast<size_t>(std::max<int64_t>(1, info.n_frames)));
        int64_t nc = 0, np = 0;
        rc = vts_scene_cuts(r.ctx, cuts.data(), info.n_frames, &nc);
        if (rc == VTS_OK) {
          pts.resize(static_cast<size_t>(std::max<int64_t>(1, info.n_frames)));
          rc = vts_frame_pts(r.ctx, pts.data(), info.n_frames, &np);
        }
        if (rc == VTS_OK) {
          std::vector<double> times;
          for (const vts_segment &sg : v.segs) {
            times.push_back(sg.start);
            times.push_back(sg.end);
          }
          v.seg_frames.assign(times.size(), 0);
          if (!times.empty())
            rc = vts_boundary_frames(r.ctx, times.data(), static_cast<int64_t>(times.size()), v.seg_frames.data());
        }
        if (rc == VTS_OK) {
          v.cut_frames.assign(cuts.begin(), cuts.begin() + nc);
          v.cut_times.clear();
          for (int64_t c : v.cut_frames)
            v.cut_times.push_back(static_cast<double>(pts[static_cast<size_t>(c)]) /
                                  static_cast<double>(info.track_timescale));
          v.n_cuts = nc;
        }
      }
      if (rc != VTS_OK) fail_video(v);
      vts_close(r.ctx);
    };
    const int cap = std::max(1, bp->max_in_flight > 0 ? bp->max_in_flight : 4);
    for (Local &v : mine) {
      while (static_cast<int>(running.size()) >= cap) finish_oldest();
      vts_ctx *ctx = nullptr;
      int rc = vts_open(bp->device, paths[v.i], &prm, &ctx);
      if (rc != VTS_OK && !running.empty()) {  // HBM held by the runs in flight: drain, retry once
        while (!running.empty()) finish_oldest();
        rc = vts_open(bp->device, paths[v.i], &prm, &ctx);
      }
      if (rc == VTS_OK) rc = vts_run_async(ctx);
      if (rc != VTS_OK) {
        fail_video(v);
        if (ctx) vts_close(ctx);
        continue;
      }
      running.push_back({&v, ctx});
    }
    while (!running.empty()) finish_oldest();
  }
  // first exchange: the records
  std::vector<int64_t> loc(static_cast<size_t>(per * vts::kRec), 0);
  for (const Local &v : mine) {
    int64_t *r = &loc[static_cast<size_t>(v.j * vts::kRec)];
    r[0] = static_cast<int64_t>(v.segs.size());
    r[1] = bp->score && !v.failed ? v.n_cuts : -1;
    r[2] = static_cast<int64_t>(std::nearbyint(v.duration * 1000000.0));
    r[3] = v.failed ? 1 : 0;
  }
  std::vector<int64_t> g(static_cast<size_t>(world) * loc.size());
  if (comm) {
    const int rc = vts::all_gather(comm, loc.data(), g.data(), loc.size(), sizeof(int64_t), ncclInt64);
    if (rc != VTS_OK) {
      delete b;
      return rc;
    }
  } else {
    g = loc;
  }
  // second exchange: boundary arrays padded to the batch's widths
  std::vector<int64_t> gi;
  std::vector<double> gf;
  int64_t wi = 1, wf = 1;
  if (bp->score) {
    for (int r = 0; r < world; ++r)
      for (int64_t j = 0; j < per; ++j) {
        const int64_t *x = &g[static_cast<size_t>((r * per + j) * vts::kRec)];
        const int64_t nc = std::max<int64_t>(0, x[1]);
        wi = std::max(wi, 2 * x[0] + nc);
        wf = std::max(wf, nc);
      }
    std::vector<int64_t> li(static_cast<size_t>(per * wi), -1);
    std::vector<double> lf(static_cast<size_t>(per * wf), 0.0);
    for (const Local &v : mine) {
      if (v.failed) continue;
      int64_t k = 0;
      for (int64_t x : v.seg_frames) li[static_cast<size_t>(v.j * wi + k++)] = x;
      for (int64_t x : v.cut_frames) li[static_cast<size_t>(v.j * wi + k++)] = x;
      for (size_t q = 0; q < v.cut_times.size(); ++q) lf[static_cast<size_t>(v.j * wf) + q] = v.cut_times[q];
    }
    gi.resize(static_cast<size_t>(world) * li.size());
    gf.resize(static_cast<size_t>(world) * lf.size());
    if (comm) {
      int rc = vts::all_gather(comm, li.data(), gi.data(), li.size(), sizeof(int64_t), ncclInt64);
      if (rc == VTS_OK) rc = vts::all_gather(comm, lf.data(), gf.data(), lf.size(), sizeof(double), ncclFloat64);
      if (rc != VTS_OK) {
        delete b;
        return rc;
      }
    } else {
      gi = li;
      gf = lf;
    }
  }
  b->rec.resize(static_cast<size_t>(n));
  b->seg_frames.resize(static_cast<size_t>(n));
  b->cut_frames.resize(static_cast<size_t>(n));
  b->cut_times.resize(static_cast<size_t>(n));
  for (int64_t i = 0; i < n; ++i) {
    const int r = static_cast<int>(i % world);
    const int64_t j = i / world;
    const int64_t *x = &g[static_cast<size_t>((r * per + j) * vts::kRec)];
    vts_batch_record &o = b->rec[static_cast<size_t>(i)];
    o.duration = static_cast<double>(x[2]) / 1e6;
    o.n_segments = x[0];
    o.n_cuts = x[1];
    o.rank = r;
    o.score_failed = static_cast<int32_t>(x[3]);
    if (bp->score && !x[3]) {
      const int64_t *row = &gi[static_cast<size_t>((r * per + j) * wi)];
      const double *rowf = &gf[static_cast<size_t>((r * per + j) * wf)];
      const int64_t ns = x[0], nc = std::max<int64_t>(0, x[1]);
      b->seg_frames[static_cast<size_t>(i)].assign(row, row + 2 * ns);
      b->cut_frames[static_cast<size_t>(i)].assign(row + 2 * ns, row + 2 * ns + nc);
      b->cut_times[static_cast<size_t>(i)].assign(rowf, rowf + nc);
    }
  }
  *out = b;
  return VTS_OK;
}

extern "C" int vts_batch_get(const vts_batch *b, int64_t i, vts_batch_record *rec) {
  if (!b || !rec || i < 0 || i >= b->n) return fail(VTS_E_INVALID, "bad batch index");
  *rec = b->rec[static_cast<size_t>(i)];
  return VTS_OK;
}

extern "C" int vts_batch_arrays(const vts_batch *b, int64_t i, int64_t *segment_frames, int64_t *cut_frames,
                                double *cut_times) {
  if (!b || i < 0 || i >= b->n) return fail(VTS_E_INVALID, "bad batch index");
  const size_t k = static_cast<size_t>(i);
  if (segment_frames) std::copy(b->seg_frames[k].begin(), b->seg_frames[k].end(), segment_frames);
  if (cut_frames) std::copy(b->cut_frames[k].begin(), b->cut_frames[k].end(), cut_frames);
  if (cut_times) std::copy(b->cut_times[k].begin(), b->cut_times[k].end(), cut_times);
  return VTS_OK;
}

extern "C" int vts_batch_error(const vts_batch *b, int64_t i, char *msg, int64_t cap, int64_t *len) {
  if (!b || i < 0 || i >= b->n) return fail(VTS_E_INVALID, "bad batch index");
  auto it = b->errors.find(i);
  const std::string s = it == b->errors.end() ? std::string() : it->second;
  if (len) *len = static_cast<int64_t>(s.size());
  if (msg && cap > 0) {
    const size_t m = std::min(s.size(), static_cast<size_t>(cap - 1));
    std::memcpy(msg, s.data(), m);
    msg[m] = '\0';
  }
  return VTS_OK;
}

extern "C" void vts_batch_free(vts_batch *b) { delete b; }
