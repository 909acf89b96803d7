"""Benchmark: 720p frames/s decoded+scored per node (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
                    [--config 720p-batch|720p-10min|720p-2h|1080p-2h|480p-60s]
                    [--workload decode_score|score|transcode] [--extras all|none]

One process per GPU: under a launcher (torch.distributed.run) RANK/LOCAL_RANK/
WORLD_SIZE come from the env and must agree with --gpus; a plain
`bench.py --gpus N` starts the N ranks itself through torch.distributed.run
(rendezvous on 127.0.0.1) before it touches the GPU, waits, and exits with
their status (rank 0's JSON line is the output).  Weak scaling: every rank
owns `videos_per_gpu` synthetic videos (video i on rank i mod N, BASELINE
config [3]'s partition) and a step is one call of vtseg.batch.plan_batch over
the whole batch: per local video probe + plan + device decode + score + scene
cuts + boundary frames, then the two all-gathers of the batch (segment / cut
counts and the padded boundary arrays; RCCL over xGMI with NCCL, gloo in the
rehearsal), so every rank ends with the whole batch's segmentation.  No pixel
data crosses GPUs.  The default workload at every N is config [3]'s per-GPU
share, 4 x 10-min 720p (BASELINE config [1]) videos per GPU: N = 8 is exactly
config [3] (32 videos), N = 1 is four config-[1] videos.  `--config 1080p-2h`
is config [4] per GPU (one 2-h 1080p video per rank).

A step's inputs are resident in HBM when the timed region starts: every local
video's session (vts_open: demux, elementary-stream upload, schedule) is open
before the warm-up, and only the per-frame work runs inside it.
  decode_score : device H.264 decode (subset kernels for the synthetic streams)
                 + scoring, through plan_batch
  score        : scoring kernel only, on pre-decoded NV12 frames (one video)
  transcode    : the 360p upload transcode (one video)
Rank 0 prints ONE JSON line (contract in the task statement), including
  roofline     : the dominant kernel; `achieved`/`frac` on SURVEY 8(d)'s
                 algorithmic bytes per frame, kernel time = busy time (union of
                 dispatch intervals) per dispatch from a rocprofv3 kernel trace
                 of this same command (HIP-event value beside it), `traffic`
                 from rocprofv3 PMC passes; the decode-inclusive figure beside;
  parity       : every local video's scores / histograms / SADs, scene cuts,
                 boundary frame indices and the gathered batch records against
                 the C oracle (whole videos at N = 1; a bounded prefix per
                 video for N > 1 unless --parity-frames all), and
                 all_ranks_equal over the ranks;
  cpu_baseline : the oracle's decode + score on the host's cores (the parity
                 pass, timed), N = 1 only;
  extras       : (N = 1, --extras all) `e2e`: file -> segment list through
                 plan_batch with nothing resident (demux, upload, decode,
                 score, results to the host); `long_video`: BASELINE config
                 [2], one 2-h 720p video in streamed two-ring windows;
                 `general`: the general decoder on a 10-min 720p full-syntax
                 noise stream (random syntax: the worst case), and
                 `general_content` on a 10-min 720p content stream (coded
                 moving scenes, synth_content.h: the video-like case), each
                 with per-kernel rooflines, the parse's issue rate, the
                 stream's bits per frame and planted vs detected scene cuts.
The rocprofv3 passes are child processes started before this process touches
the GPU; --profile-dir keeps their summaries.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "video-transformer_amd"))
sys.path.insert(0, str(ROOT / "oracle"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
VALU_SAD_PEAK_TOPS = 256 * 4 * 32 * 4 * 2.4e9 / 1e12  # v_sad_u8 byte-SADs/s (MI355X_MICROARCH.md)
CU_ISSUE_PEAK = 256 * 2.4e9  # instructions/s if every CU issued one per cycle

# BASELINE.json configs, per GPU: name -> (width, height, frames per video,
# videos per GPU, what)
CONFIGS = {
    "720p-batch": (1280, 720, 18000, 4,
                   "BASELINE config [3] per-GPU share: 4 x 10-min 720p MP4 per GPU (config [3] = "
                   "32 videos over 8 GPUs; at N GPUs 4N videos, video i on rank i mod N) through "
                   "vtseg.batch.plan_batch"),
    "720p-10min": (1280, 720, 18000, 1, "BASELINE config [1]: 10-min 720p MP4, one per GPU"),
    "720p-2h": (1280, 720, 216000, 1, "BASELINE config [2]: 2-h 720p, streamed decode "
                                      "(two-ring windows)"),
    "1080p-2h": (1920, 1080, 216000, 1, "BASELINE config [4] per GPU: 2-h 1080p, one per GPU (8 "
                                        "over 8 GPUs), two-stream decode/score overlap"),
    "480p-60s": (640, 480, 1800, 1, "BASELINE config [0] clip (60-s 480p) on the GPU path"),
}
FPS = 30
HD_FRAMES = 54000  # the N = 1 line's 1080p record: a 30-min sample of config [4]'s 2-h video
METRIC = "720p frames/sec decoded+scored per node; segment-index exact-match vs CPU"
# the reference's default analyzer config (config/config.yaml:84-96)
REF_CONFIG = {"analyzer": {"max_continuations": 3, "retry_times": 5,
                           "long_video": {"enabled": True, "default_segment_seconds": 480,
                                          "overlap_seconds": 20, "min_segment_seconds": 90,
                                          "hard_max_api_calls": 50, "consolidate": True,
                                          "duration_threshold_seconds": None}}}


def log(msg: str) -> None:
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def algorithmic_bytes_per_frame(width: int, height: int, k: int) -> int:
    """NV12 read + RGB thumbnail write + thumbnail luma
    write/read + histogram + score."""
    w, h = width // k, height // k
    return int(1.5 * width * height) + 3 * w * h + 2 * w * h + 1024 + 4


def fused_bytes_per_frame(width: int, height: int, k: int) -> int:
    """h264_recon_score: NV12-sized source read (reference picture or I_PCM
    samples) + NV12 frame written + RGB thumbnail + thumbnail luma written and
    the predecessor's read for the fused SAD + histogram + SAD; the frame is
    never re-read for scoring."""
    w, h = width // k, height // k
    return 3 * width * height + 3 * w * h + 2 * w * h + 1024 + 8


def tb_bytes_per_launch(width: int, height: int, k: int, frames: int, chains: int,
                        launches: int, keep: bool = False) -> float:
    """h264_recon_score_tb (level-blocked): per chain of L levels one
    NV12-sized source read (reference picture or I_PCM samples), one NV12
    frame written (the chain's last level; every level with keep) and the
    predecessor thumbnail read once; per frame the RGB thumbnail, thumbnail
    luma written, histogram and SAD.  The levels between a chain's first and
    last stay in LDS and move no HBM bytes."""
    w, h = width // k, height // k
    nv12 = 1.5 * width * height
    per_chain = nv12 + (0 if keep else nv12) + w * h
    per_frame = 3 * w * h + w * h + 1024 + 8 + (nv12 if keep else 0)
    return (chains * per_chain + frames * per_frame) / launches


def host_cores() -> dict:
    """The host cores this process may use: the scheduler affinity set
    (os.sched_getaffinity) and, when the cgroup caps CPU time (cgroup v2
    cpu.max "quota period"), that cap in whole cores.  The CPU baseline runs
    one oracle thread per usable core: all affinity cores, unless the cgroup
    quota grants fewer (more threads than the quota only time-slice)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        quota = None
    return {"affinity": aff, "cgroup_quota": quota, "usable": min(aff, quota) if quota else aff}


def smooth_frames_host(rng, n, width, height):
    frames = np.empty((n, height * 3 // 2, width), np.uint8)
    for i in range(n):
        g = rng.integers(16, 236, size=(height // 32 + 2, width // 32 + 2)).astype(np.float32)
        y = np.kron(g, np.ones((32, 32), np.float32))[:height, :width]
        frames[i, :height] = np.clip(y + rng.normal(0, 4, y.shape), 0, 255).astype(np.uint8)
        c = rng.integers(64, 192, size=(height // 64 + 2, width // 16 + 2)).astype(np.float32)
        frames[i, height:] = np.kron(c, np.ones((32, 16), np.float32))[:height // 2, :width]
    return frames


def cpu_baseline_score(width, height, k, budget_s=10.0):
    """Oracle scorer (scalar C, 1 thread) on a bounded sample of frames
    (score-only workload)."""
    import oracle
    rng = np.random.default_rng(1)
    frames = smooth_frames_host(rng, 8, width, height).reshape(-1)
    stride = width * height * 3 // 2
    t0 = time.perf_counter()
    oracle.score_frames(frames, stride, 8, width, height, width, height, k, want_rgb=True)
    per = (time.perf_counter() - t0) / 8
    n = max(8, min(4000, int(budget_s / max(per, 1e-6))))
    reps = (n + 7) // 8
    t0 = time.perf_counter()
    for _ in range(reps):
        oracle.score_frames(frames, stride, 8, width, height, width, height, k, want_rgb=True)
    dt = time.perf_counter() - t0
    return {"value": round(reps * 8 / dt, 2), "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"{reps * 8} frames {width}x{height} scored by oracle/vtseg_oracle.c "
                      f"or_score_frames (scalar, 1 thread), {dt:.1f} s"}


def cpu_baseline_transcode(path, k, budget_s=15.0):
    """The same transcode on the host, 1 thread: the C oracle decodes and
    scores the first frames of the benchmark video, then or_transcode
    (transcode_oracle.c: area downscale, scalar full search R = 8, slice
    writer) encodes them; a bounded sample sized from a 4-frame probe."""
    import oracle
    m = oracle.read_mp4(path)
    n_all = len(m["sizes"])

    def run(n):
        samples = [m["data"][o:o + z] for o, z in zip(m["offsets"][:n], m["sizes"][:n])]
        frames = oracle.decode_samples(m["sps"][0], m["pps"][0], samples, m["nal_length_size"])
        H, W = frames.shape[1] * 2 // 3, frames.shape[2]
        sc = oracle.score_frames(frames.reshape(-1), frames[0].size, n, W, H, W, H, k,
                                 want_rgb=True)["score"]
        oracle.transcode(frames, W, H, sc)
        return W, H

    t0 = time.perf_counter()
    run(4)
    per = (time.perf_counter() - t0) / 4
    n = max(4, min(n_all, int(budget_s / max(per, 1e-6))))
    t0 = time.perf_counter()
    W, H = run(n)
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 2), "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"first {n} frames ({W}x{H}) of the benchmark video: oracle decode + score + "
                      f"or_transcode (area downscale, scalar full search R=8, CAVLC writer), "
                      f"1 thread, {dt:.1f} s"}


def _kernel_short(name: str) -> str:
    m = re.search(r"(h264_recon_score_tb|h264_recon_score6b?|h264_\w+|thumb_sad|score_\w+)(<\d+>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name.split("(")[0][-60:]


def _busy(intervals: list[tuple[int, int]]) -> tuple[float, float]:
    """(union of the intervals, sum of their lengths) in the trace's units."""
    iv = sorted(intervals)
    tot, (cs, ce) = 0, iv[0]
    for st, en in iv[1:]:
        if st > ce:
            tot, cs, ce = tot + ce - cs, st, en
        else:
            ce = max(ce, en)
    return tot + ce - cs, sum(e - b for b, e in iv)


def profile_passes(argv: list[str], out_dir: Path, keep_dir: Path | None,
                   passes=("trace", "FETCH_SIZE", "WRITE_SIZE"), timeout: int = 240) -> dict:
    """rocprofv3 child runs of this same benchmark (1 timed step each):
      * "trace" = --kernel-trace --stats: per kernel, dispatches, mean dispatch
        duration and busy time (union of the dispatch intervals) per dispatch;
        with two GOP groups two reconstruct dispatches overlap, so the mean
        duration overstates each one's share of the wall time and the busy
        time is the kernel time per launch;
      * a counter name (or a space-separated group of SQ counters) = --pmc
        pass; FETCH_SIZE and WRITE_SIZE need separate passes (3 + 2 TCC slots
        > 4): HBM bytes per dispatch = 2 x FETCH_SIZE (gfx950 tallies wide
        coalesced reads at half their bytes) + WRITE_SIZE, both KiB
        (MI355X_MICROARCH.md, HBM section).
    Started before this process initialises the GPU (no exec from a
    GPU-initialised process), each under its own time limit."""
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not Path(prof).exists():
        return {"error": "rocprofv3 not found"}
    res: dict = {}
    env = dict(os.environ, TMPDIR="/tmp")
    child = [sys.executable, str(Path(__file__).resolve()), *argv, "--steps", "1", "--warmup", "1",
             "--no-cpu-baseline", "--no-pmc", "--no-parity", "--extras", "none"]
    for pi, what in enumerate(passes):
        d = out_dir / f"p{pi}"
        counters = what.split()
        opts = (["--kernel-trace", "--stats"] if what == "trace" else
                ["--kernel-trace", "--pmc", *counters])
        cmd = [prof, *opts, "--output-format", "csv", "-d", str(d), "-o", "run", "--", *child]
        t0 = time.perf_counter()
        try:
            proc = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True,
                                  timeout=timeout)
        except subprocess.TimeoutExpired:
            res["error"] = f"{what} pass timed out"
            continue
        log(f"profile pass {what!r}: rc={proc.returncode}, {time.perf_counter() - t0:.1f} s")
        if proc.returncode != 0:
            res["error"] = f"{what} pass rc={proc.returncode}: {proc.stderr[-300:]}"
            continue
        if what == "trace":
            iv: dict = {}
            for f in d.rglob("*kernel_trace.csv"):
                with open(f) as fh:
                    for r in csv.DictReader(fh):
                        iv.setdefault(_kernel_short(r["Kernel_Name"]), []).append(
                            (int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
            for k, v in iv.items():
                union, total = _busy(v)
                res.setdefault(k, {}).update(dispatches_traced=len(v),
                                             busy_ns_per_dispatch=union / len(v),
                                             busy_ns_total=union,
                                             mean_dispatch_ns=total / len(v))
            if keep_dir is not None:
                keep_dir.mkdir(parents=True, exist_ok=True)
                for f in d.rglob("*kernel_stats.csv"):
                    shutil.copy(f, keep_dir / "kernel_stats.csv")
                rows = sorted(((k, v) for k, v in res.items()
                               if isinstance(v, dict) and "busy_ns_per_dispatch" in v),
                              key=lambda kv: -kv[1]["busy_ns_total"])
                (keep_dir / "kernel_busy.txt").write_text("".join(
                    f"{k}: {v['dispatches_traced']} dispatches, busy (union of intervals) "
                    f"{v['busy_ns_per_dispatch'] / 1e3:.2f} us per dispatch, mean dispatch "
                    f"duration {v['mean_dispatch_ns'] / 1e3:.2f} us\n" for k, v in rows))
            continue
        acc: dict = {}
        for f in d.rglob("*counter_collection.csv"):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if r["Counter_Name"] not in counters:
                        continue
                    acc.setdefault((_kernel_short(r["Kernel_Name"]), r["Counter_Name"]),
                                   []).append(float(r["Counter_Value"]))
        for (k, cn), v in acc.items():
            row = res.setdefault(k, {})
            row[cn] = sum(v) / len(v)
            row[cn + "_total"] = sum(v)
            row["dispatches"] = len(v)
    for k, row in res.items():
        if isinstance(row, dict) and "FETCH_SIZE" in row and "WRITE_SIZE" in row:
            row["hbm_bytes"] = (2 * row["FETCH_SIZE"] + row["WRITE_SIZE"]) * 1024
    if keep_dir is not None:
        keep_dir.mkdir(parents=True, exist_ok=True)
        (keep_dir / "profile_passes.json").write_text(json.dumps(res, indent=1))
    return res


def synth_videos(jobs: list[tuple[Path, int]], width: int, height: int, frames: int,
                 coding: str = "subset", bframes: bool = False, cabac: bool = False,
                 content: bool = False) -> list[dict]:
    """Write the synthetic H.264/MP4 inputs (vts_synth_write; ctypes releases
    the GIL, so the videos are written in parallel)."""
    from vtseg import scene

    def one(job):
        path, seed = job
        if coding == "full":
            # x264-like structure: one slice per picture; with bframes B
            # reference pictures, spatial direct, implicit weighted
            # bi-prediction; with cabac CABAC and the High profile's 8x8
            # transform (x264's defaults: cabac, 8x8dct, b-pyramid, weightb)
            extra = dict(bframes=True, weighted="implicit") if bframes else {}
            if cabac:
                extra.update(cabac=True, transform_8x8=True)
            if content:
                # coded pictures instead of random syntax (synth_content.h);
                # x264's default keyint 250 (~8 s) between refresh IDRs
                extra.update(content=True, gop_max_s=8.0)
            return scene.synth_write(path, width=width, height=height, fps=FPS, n_frames=frames,
                                     seed=seed, coding="full", slices_per_row=0, max_motion=4,
                                     **extra)
        return scene.synth_write(path, width=width, height=height, fps=FPS, n_frames=frames,
                                 seed=seed)

    with ThreadPoolExecutor(max(1, len(jobs))) as ex:
        return list(ex.map(one, jobs))


def parity_check(scorer, path, k: int, segs, threads: int, max_frames: int | None,
                 decoder: str = "subset") -> tuple[dict, dict]:
    """This run's device results against the C oracle (oracle.decode_score_gops,
    GOP-parallel on `threads` host threads): every frame's fp32 score (exact;
    north_star allows |d| <= 1e-4), 256-bin histogram and SAD, the scene cuts,
    and the boundary frame index of every planned segment time (start, end,
    effective start/end of each segment of the reference's plan,
    src/utils/video_segmenter.py:42-83) in exact rationals.  Returns (parity,
    the oracle pass: timing + its pts / cuts for the batch-record check)."""
    import oracle
    res = scorer.score()                     # a full decode + score, results to the host
    cuts = scorer.scene_cuts()
    ref = oracle.decode_score_gops(path, k, threads, max_frames=max_frames, decoder=decoder)
    n = ref["frames"]
    times = [t for sg in segs for t in (sg.start, sg.end, sg.effective_start, sg.effective_end)]
    times = [t for t in times if max_frames is None or t * FPS < n]
    got_idx = scorer.boundary_frames(times) if times else []
    want_idx = oracle.boundary_frames(ref["pts"], ref["timescale"], times) if times else []
    ref_cuts = np.nonzero(ref["score"] > 0.08)[0].tolist()
    dscore = float(np.max(np.abs(res.scores[:n].astype(np.float64) - ref["score"].astype(np.float64))))
    parity = {"frames": n, "of_frames": int(len(res.scores)),
              "scores_equal": bool(np.array_equal(res.scores[:n], ref["score"])),
              "max_abs_score_diff": dscore, "score_tolerance": 1e-4,
              "hist_equal": bool(np.array_equal(res.hist[:n], ref["hist"])),
              "sad_equal": bool(np.array_equal(res.sad[:n], ref["sad"])),
              "scene_cuts": len(ref_cuts),
              "scene_cuts_equal": [c for c in cuts if c < n] == ref_cuts,
              "segment_times": len(times),
              "boundary_frames_equal": list(got_idx) == list(want_idx),
              "pts_equal": res.pts[:n].tolist() == ref["pts"]}
    parity["all_equal"] = all(parity[x] for x in ("scores_equal", "hist_equal", "sad_equal",
                                                  "scene_cuts_equal", "boundary_frames_equal",
                                                  "pts_equal"))
    return parity, {"frames": n, "seconds": ref["seconds"], "threads": threads,
                    "gops": ref["gops"], "width": ref["width"], "height": ref["height"],
                    "pts": ref["pts"], "timescale": ref["timescale"], "cuts": ref_cuts}


def batch_record_check(item, segs, ref: dict, full: bool) -> bool:
    """The gathered BatchItem of a local video against the oracle: segment
    count, every planned segment's [start, end) frame window, the scene-cut
    frames and their times (prefix-restricted when only a prefix was checked)."""
    import oracle
    n = len(ref["pts"])
    if item.n_segments != len(segs) or item.score_failed:
        return False
    times = [t for sg in segs for t in (sg.start, sg.end)]
    want = oracle.boundary_frames(ref["pts"], ref["timescale"], times) if times else []
    got = [x for pair in item.segment_frames for x in pair]
    cut_t = [float(ref["pts"][c]) / ref["timescale"] for c in ref["cuts"]]
    if full:
        return got == want and list(item.cut_frames) == ref["cuts"] and \
            list(item.cut_times) == cut_t and item.n_cuts == len(ref["cuts"])
    keep = [i for i, t in enumerate(times) if t * FPS < n]
    return [got[i] for i in keep] == [want[i] for i in keep] and \
        [c for c in item.cut_frames if c < n] == ref["cuts"]


def kernel_stats_from(prof: dict | None, name: str) -> dict | None:
    row = (prof or {}).get(name)
    return row if isinstance(row, dict) else None


def recon_kernel_name(scorer, k: int) -> str:
    tb = scorer.level_blocks()[0]
    if scorer.fused():
        return ("h264_recon_score_tb" if tb else
                "h264_recon_score6b" if k == 6 else "h264_recon_score<%d>" % k)
    return "score_runs<%d>" % k


def roofline_decode_score(scorers, prof: dict | None, width: int, height: int, k: int,
                          frames_per_video: int) -> dict:
    """Roofline of the dominant kernel over the local videos' sessions: the
    reconstruct+score kernel's time per launch from HIP events on its stream
    (mean of 3 runs per session), replaced by the rocprofv3 trace's busy time
    per dispatch when the trace pass ran."""
    s0 = scorers[0]
    rec, sco, launches = [], [], []
    for v in scorers:
        for _ in range(ROOF_RUNS):
            v.run()
            t = v.timings()
            rec.append(t["reconstruct_ms"])
            sco.append(t["score_ms"])
        launches.append(v.level_blocks()[0] or v.recon_launches())
    tb_launches, tb_chains = s0.level_blocks()
    n_launch = int(np.mean(launches))
    kname = recon_kernel_name(s0, k)
    F = frames_per_video
    if s0.fused():
        kern_ms = float(np.mean(rec)) / n_launch
        frames_per_launch = F / n_launch
    else:
        n_score = max(1, s0.windows())
        kern_ms = float(np.mean(sco)) / n_score
        frames_per_launch = F / n_score
    kern_ms_events = kern_ms
    kern_basis = "HIP events on the kernel's stream"
    prow = kernel_stats_from(prof, kname)
    if prow and "busy_ns_per_dispatch" in prow:
        kern_ms = prow["busy_ns_per_dispatch"] / 1e6
        kern_basis = (f"rocprofv3 --kernel-trace of this command: busy time (union of "
                      f"{prow['dispatches_traced']} dispatch intervals) per dispatch; mean "
                      f"dispatch duration {prow['mean_dispatch_ns'] / 1e3:.2f} us")
    alg_bpf = algorithmic_bytes_per_frame(width, height, k)
    if s0.fused() and tb_launches:
        bytes_per_frame = tb_bytes_per_launch(width, height, k, F, tb_chains, n_launch) / frames_per_launch
    elif s0.fused():
        bytes_per_frame = fused_bytes_per_frame(width, height, k)
    else:
        bytes_per_frame = alg_bpf
    achieved = alg_bpf * frames_per_launch / (kern_ms * 1e-3) / 1e9
    traffic, traffic_note = None, None
    if prof is not None:
        if prow and "hbm_bytes" in prow:
            traffic = round(prow["hbm_bytes"])
            traffic_note = (f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (2xFETCH+WRITE), "
                            f"mean of {prow['dispatches']} dispatches; "
                            f"{traffic / (alg_bpf * frames_per_launch):.3f}x SURVEY 8(d) bytes, "
                            f"{traffic / (bytes_per_frame * frames_per_launch):.3f}x the "
                            f"decode-inclusive bytes")
        else:
            traffic_note = prof.get("error", f"no counters for {kname}")
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "traffic_unit": "bytes/launch", "traffic_source": traffic_note,
            "kernel": kname, "kernel_ms": round(kern_ms, 5), "kernel_ms_basis": kern_basis,
            "kernel_ms_hip_events": round(kern_ms_events, 5),
            "bytes_per_frame": alg_bpf,
            "bytes_basis": "SURVEY 8(d): 1.5*W*H NV12 read + 3*w*h RGB + 2*w*h thumbnail "
                           "luma write/read + 1024 histogram + 4 score",
            "frames_per_launch": round(frames_per_launch, 1)}
    if bytes_per_frame != alg_bpf:
        ach_d = bytes_per_frame * frames_per_launch / (kern_ms * 1e-3) / 1e9
        roof["decode_inclusive"] = {
            "bytes_per_frame": round(bytes_per_frame, 1), "achieved": round(ach_d, 1),
            "frac": round(ach_d / HBM_PEAK_GBS, 4),
            "basis": "the fused decode+score kernel's own bytes: NV12-sized reference/I_PCM "
                     "read + NV12 frame write + RGB + thumbnail luma write + predecessor "
                     "read + histogram + SAD"}
    return roof


# ------------------------------------------------------------ rank launcher

class LaunchError(ValueError):
    """--gpus disagrees with the environment or the machine (exit status 2)."""


def device_count() -> int:
    """GPUs visible to this process without initialising any (on this image
    torch.cuda.device_count() does not create a HIP context)."""
    import torch
    return torch.cuda.device_count()


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_launch_plan(gpus: int, env, ndev: int, backend: str, argv: list[str],
                     port=_free_port) -> tuple[list[str], dict] | None:
    """How `bench.py --gpus N` becomes N rank processes (one per GPU), the
    reference's sequential batch loop (src/pipeline.py:376-393) spread over
    the node.  Returns None when this process is the (only) rank to run:
    N = 1, or a launcher (torch.distributed.run) already set WORLD_SIZE to N.
    Otherwise the torch.distributed.run command that starts N ranks of this
    same script with the same arguments (rendezvous on 127.0.0.1) and its
    environment; the parent only waits, so no process that touched the GPU
    ever execs.  Raises LaunchError when --gpus disagrees with an existing
    WORLD_SIZE, or asks for more GPUs than the machine has (NCCL = RCCL needs
    one GPU per rank; gloo may put several ranks on one GPU as a rehearsal)."""
    if gpus < 1:
        raise LaunchError(f"--gpus {gpus}: at least one GPU")
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            raise LaunchError(f"--gpus {gpus} disagrees with WORLD_SIZE={ws} set by the launcher")
        return None
    if gpus == 1:
        return None
    if backend == "nccl" and gpus > ndev:
        raise LaunchError(f"--gpus {gpus} but only {ndev} GPU(s) visible; RCCL needs one GPU per "
                          f"rank (--dist-backend gloo rehearses several ranks on one GPU)")
    if ndev < 1:
        raise LaunchError(f"--gpus {gpus} but no GPU visible")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1", f"--master-port={port()}",
           str(Path(__file__).resolve()), *argv]
    child_env = dict(env)
    child_env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only (RCCL)
    child_env.setdefault("MASTER_ADDR", "127.0.0.1")
    return cmd, child_env


def relay_ranks(cmd: list[str], env: dict, out=None, err=None) -> int:
    """Run the rank launcher and wait.  Its stdout carries rank 0's JSON line
    and whatever else the ranks print there (gloo announces its peer
    connections on stdout): the JSON line goes to our stdout, everything else
    to stderr, so the contract's one-line output holds.  Returns the
    launcher's exit status."""
    out = out or sys.stdout
    err = err or sys.stderr
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True)
    assert proc.stdout is not None
    for line in proc.stdout:
        (out if line.startswith('{"metric"') else err).write(line)
        (out if line.startswith('{"metric"') else err).flush()
    return proc.wait()


def placement(world: int, ndev: int) -> dict:
    """GPUs a run occupies and ranks per GPU (rank r on GPU LOCAL_RANK % ndev):
    a gloo rehearsal with more ranks than GPUs reports its GPUs as n_gpus,
    never its ranks."""
    n = max(1, min(world, max(ndev, 1)))
    return {"n_gpus": n, "world_size": world, "ranks_per_gpu": round(world / n, 3)}


# --------------------------------------------------------------- extras (N = 1)

ROOF_RUNS = 3             # roofline_decode_score's vts_run calls per session
CHILD_RUNS = 2 + ROOF_RUNS  # a profile child's vts_run calls: warmup 1 + step 1 + the roofline's
GENERAL_PMC = ("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM "
               "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH")


def general_kernel_rooflines(prof: dict, width: int, height: int, k: int, frames: int,
                             mbs_per_frame: int) -> dict:
    """Per-kernel rooflines of the general decoder from a rocprofv3 kernel
    trace (busy time = union of each kernel's dispatch intervals) and an SQ
    instruction-count pass.  Algorithmic bytes per picture (display-size NV12
    = 1.5*W*H):
      h264_inter_full   reference read + NV12 write          3.0*W*H
      h264_intra_v2 / h264_intra_full      NV12 write (intra share)  1.5*W*H
      h264_deblock_plane / _lds / _full   NV12 read + write         3.0*W*H
      score_runs        SURVEY 8(d) bytes                     1.5*W*H + 5*w*h + 1028
    (intra and inter both count the whole picture's write; their sum
    overstates a picture that mixes them, so the sum is not reported).
    h264_parse_full is serial bit parsing: its bound is instruction issue,
    reported as instructions / (256 CUs x 2.4 GHz x busy time).  The child
    ran the whole decode CHILD_RUNS times: busy times and counter totals are
    divided by it (per run)."""
    nv12 = 1.5 * width * height
    w, h = width // k, height // k
    per_pic = {"h264_inter_full": 2 * nv12, "h264_intra_v2": nv12, "h264_intra_full": nv12,
               "h264_deblock_plane": 2 * nv12, "h264_deblock_lds": 2 * nv12, "h264_deblock_full": 2 * nv12,
               f"score_runs<{k}>": nv12 + 5 * w * h + 1028}
    out = {}
    for name, b in per_pic.items():
        row = prof.get(name)
        if not isinstance(row, dict) or "busy_ns_total" not in row:
            continue
        t = row["busy_ns_total"] * 1e-9 / CHILD_RUNS
        ach = b * frames / t / 1e9
        nd = max(1, row["dispatches_traced"] // CHILD_RUNS)
        out[name] = {"bound": "hbm", "busy_ms": round(t * 1e3, 2),
                     "dispatches": row["dispatches_traced"] // CHILD_RUNS,
                     "busy_ms_per_dispatch": round(t * 1e3 / nd, 3), "bytes_per_picture": round(b),
                     "achieved": round(ach, 1), "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBS, 4)}
    pname = "h264_parse_full_cabac" if "h264_parse_full_cabac" in prof else "h264_parse_full"
    row = prof.get(pname)
    if isinstance(row, dict) and "busy_ns_total" in row:
        t = row["busy_ns_total"] * 1e-9 / CHILD_RUNS
        rec = {"bound": "issue", "busy_ms": round(t * 1e3, 2),
               "dispatches": row["dispatches_traced"] // CHILD_RUNS}
        kinds = ["SQ_INSTS_SALU", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM",
                 "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_BRANCH"]
        if all(kk + "_total" in row for kk in kinds):
            insts = sum(row[kk + "_total"] for kk in kinds) / CHILD_RUNS
            mbs = frames * mbs_per_frame * CHILD_RUNS  # per-kind totals below span every run
            rec.update({"instructions": insts, "instructions_per_mb": round(insts * CHILD_RUNS / mbs, 1),
                        "salu_per_mb": round(row["SQ_INSTS_SALU_total"] / mbs, 1),
                        "valu_per_mb": round(row["SQ_INSTS_VALU_total"] / mbs, 1),
                        "lds_per_mb": round(row["SQ_INSTS_LDS_total"] / mbs, 1),
                        "smem_per_mb": round(row["SQ_INSTS_SMEM_total"] / mbs, 1),
                        "vmem_per_mb": round((row["SQ_INSTS_VMEM_RD_total"] + row["SQ_INSTS_VMEM_WR_total"]) / mbs, 1),
                        "branch_per_mb": round(row["SQ_INSTS_BRANCH_total"] / mbs, 1),
                        # the bound: the one scalar ALU a CU's waves share (vector
                        # instructions issue on the CU's four SIMDs beside it)
                        "achieved": round(row["SQ_INSTS_SALU_total"] / CHILD_RUNS / t / 1e9, 2),
                        "unit": "G SALU instructions/s",
                        "peak": CU_ISSUE_PEAK / 1e9,
                        "frac": round(row["SQ_INSTS_SALU_total"] / CHILD_RUNS / t / CU_ISSUE_PEAK, 4),
                        "all_instructions_per_s_G": round(insts / t / 1e9, 2),
                        "peak_basis": "one SALU instruction per CU per cycle: 256 CUs x 2.4 GHz "
                                      "(the scalar unit a CU's waves share)"})
        out[pname] = rec
    return out


def run_single(path: Path, *, gpu: int, k: int, steps: int, threads: int, label: str,
               decoder: str = "auto", prof: dict | None = None, parity: bool = True,
               planted: list[int] | None = None, window_frames: int = 0) -> dict:
    """One video through its session: `steps` timed vts_run calls (inputs
    resident), stage times, the session's HBM (the allocator's bytes handed
    out by its vts_open, and after the runs: a CABAC arena that overflowed
    grew), the dominant kernel's roofline and parity over every frame against
    the oracle; with `planted` (the writer's scene cuts) the device's detected
    cuts beside them."""
    import torch
    from vtseg import _lib
    from vtseg import budget_planner as bp
    from vtseg import scene
    from vtseg import video_segmenter as vs
    L = _lib.lib()
    before = int(L.vts_device_bytes(gpu))
    t0 = time.perf_counter()
    v = scene.VideoScorer(path, device=gpu, decoder=decoder, window_frames=window_frames)
    open_s = time.perf_counter() - t0
    hbm_open = int(L.vts_device_bytes(gpu)) - before
    try:
        F = v.n_frames
        W, H = int(v.info.width), int(v.info.height)
        v.run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            v.run()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        rec = {"label": label, "frames": F, "width": W, "height": H, "steps": steps,
               "value": round(F * steps / el, 1), "unit": "frames/s",
               "ms_per_step": round(el / steps * 1e3, 3), "open_s": round(open_s, 3),
               "open_stages_ms": {k: round(x, 1) for k, x in v.open_timings().items()},
               "decoder": "general" if v.general() else "subset",
               "stage_ms": v.timings(), "recon_launches": v.recon_launches(),
               "windows": v.windows(),
               "hbm_gb_at_open": round(hbm_open / 1e9, 2),
               "hbm_gb_after_runs": round((int(L.vts_device_bytes(gpu)) - before) / 1e9, 2),
               "bits_per_frame": round(Path(path).stat().st_size * 8 / F, 1)}
        if v.general():
            rec["arena_reruns"] = v.arena_reruns()
        if window_frames:
            rec["window_frames"] = window_frames
        if not v.general():
            rec["roofline"] = roofline_decode_score([v], prof, W, H, k, F)
        if planted is not None:
            det = v.scene_cuts()
            ps = set(planted)
            rec["cuts"] = {"planted": len(planted), "detected": len(det),
                           "detected_at_planted": sum(1 for c in det if c in ps),
                           "detected_within_1": sum(1 for c in det if {c - 1, c, c + 1} & ps)}
        if parity:
            duration = float(v.info.duration)
            plan = bp.plan_segments_with_budget(duration, REF_CONFIG, 0)
            segs = vs.plan_segments(duration, plan.segment_duration, plan.overlap)
            par, ct = parity_check(v, path, k, segs, threads, None,
                                   "full" if v.general() else "subset")
            par["oracle"] = ("oracle/h264_full_oracle.c fo_decode" if v.general() else
                             "oracle/vtseg_oracle.c or_decode_samples") + \
                f" + or_score_frames (GOP-parallel, {threads} threads)"
            rec["parity"] = par
            rec["cpu_oracle_frames_per_s"] = round(ct["frames"] / ct["seconds"], 2)
        return rec
    finally:
        v.close()


def general_batch_record(paths: list[Path], gpu: int, threads: int, planted: list[list[int]],
                         n_content: int) -> dict:
    """BATCH config [3]'s per-GPU share on real-syntax streams, resident
    sessions through plan_batch (every session's run submitted before any is
    waited for, vts_run_async): the first n_content paths are video-like CABAC
    B content streams — their batch against one of them alone is the overlap
    figure (`batch_over_single`, HIP's default hardware queues) — the rest
    full-syntax noise streams, run as a mixed batch with half of the content
    sessions (`mixed`: the worst case beside the typical).  Each session's HBM
    (the allocator's bytes handed out by its vts_open, and the mean after the
    runs) and full parity of every video."""
    import torch
    from vtseg import _lib, batch, scene
    from vtseg import budget_planner as bp
    from vtseg import video_segmenter as vs
    L = _lib.lib()
    sessions, hbm = {}, []
    base = int(L.vts_device_bytes(gpu))

    def timed(idx: list[int]) -> tuple[float, list]:
        strs = [str(paths[i]) for i in idx]
        ses = {j: sessions[i] for j, i in enumerate(idx)}
        batch.plan_batch(strs, REF_CONFIG, score=True, sessions=ses)  # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            items = batch.plan_batch(strs, REF_CONFIG, score=True, sessions=ses)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / 3 * 1e3, items

    try:
        for i, p in enumerate(paths):
            before = int(L.vts_device_bytes(gpu))
            sessions[i] = scene.VideoScorer(p, device=gpu)
            hbm.append(int(L.vts_device_bytes(gpu)) - before)
        F = sessions[0].n_frames
        v0 = sessions[0]
        v0.run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            v0.run()
        torch.cuda.synchronize()
        single_ms = (time.perf_counter() - t0) / 3 * 1e3
        content = list(range(n_content))
        batch_ms, items_c = timed(content)
        mixed = list(range(max(1, n_content // 2))) + list(range(n_content, len(paths)))
        mixed_ms, items_m = timed(mixed)
        items = {i: it for i, it in zip(content, items_c)}
        items.update({i: it for i, it in zip(mixed, items_m)})
        hbm_after = int(L.vts_device_bytes(gpu)) - base
        per_video, ok = [], True
        for i, p in enumerate(paths):
            v = sessions[i]
            duration = float(v.info.duration)
            plan = bp.plan_segments_with_budget(duration, REF_CONFIG, 0)
            segs = vs.plan_segments(duration, plan.segment_duration, plan.overlap)
            par, ct = parity_check(v, p, 4, segs, threads, None, "full")
            par["batch_record_equal"] = batch_record_check(items[i], segs, ct, True)
            par["stream"] = "content" if i < n_content else "noise"
            det = set(items[i].cut_frames)
            par["planted_cuts"] = len(planted[i])
            par["planted_cuts_detected"] = sum(1 for c in planted[i] if c in det)
            per_video.append(par)
            ok &= par["all_equal"] and par["batch_record_equal"]
        return {"label": f"BASELINE config [3] per-GPU share on real syntax: {n_content} x 10-min 720p CONTENT "
                         "streams (CABAC, 8x8, B pyramid, implicit weights, deblocking) as resident sessions "
                         "through vtseg.batch.plan_batch, every session's run submitted before any wait, on the "
                         "process's HIP hardware queues as inherited; `mixed`: "
                         f"{len(mixed) - (len(paths) - n_content)} of them with {len(paths) - n_content} "
                         "full-syntax NOISE streams (the worst case for HBM and parse)",
                "videos": n_content, "frames_per_video": F, "steps": 3,
                "value": round(n_content * F / (batch_ms / 1e3), 1), "unit": "frames/s",
                "ms_per_step": round(batch_ms, 2), "single_video_ms": round(single_ms, 2),
                "batch_over_single": round(batch_ms / single_ms, 3),
                "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "unset (HIP default 4)"),
                "mixed": {"videos": [("content" if i < n_content else "noise") for i in mixed],
                          "ms_per_step": round(mixed_ms, 2),
                          "value": round(len(mixed) * F / (mixed_ms / 1e3), 1), "unit": "frames/s"},
                "hbm_gb_per_session": [round(b / 1e9, 2) for b in hbm],
                "hbm_gb_per_session_after_runs": round(hbm_after / len(paths) / 1e9, 2),
                "arena_reruns": [sessions[i].arena_reruns() for i in range(len(paths))],
                "parity": {"all_equal": bool(ok), "videos": per_video}}
    finally:
        for v in sessions.values():
            v.close()


def e2e_record(paths: list[Path], gpu: int) -> dict:
    """File -> segment list with nothing resident: plan_batch over the batch's
    files (per video: native moov probe, plan, vts_open = MP4 demux +
    elementary-stream upload over PCIe + schedule, device decode + score,
    scores to the host, scene cuts, boundary frames, close), then the same
    stages timed one by one on the first video."""
    import torch
    from vtseg import batch, scene
    # the record's inputs are page-cache resident, as it says: read once before
    # the clock starts (the box may have evicted the files since they were
    # written; from disk the same call measured 0.18 -> 1.49 s)
    for p in paths:
        with open(p, "rb") as fh:
            while fh.read(1 << 24):
                pass
    # one untimed call first: a process's first plan_batch over new sessions
    # measured 0.5-2.0 s against 0.19-0.21 s for every later one (the stream
    # pool and the device allocator's cache being set up;
    # profiles/r06ap_e2e_first_call_ab.jsonl); the record is the steady state
    # of a long-running caller, nothing resident between calls
    batch.plan_batch([str(p) for p in paths], REF_CONFIG, score=True, device=gpu)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    items = batch.plan_batch([str(p) for p in paths], REF_CONFIG, score=True, device=gpu)
    dt = time.perf_counter() - t0
    frames = 0
    stages = {}
    for p in paths[:1]:
        t0 = time.perf_counter()
        v = scene.VideoScorer(p, device=gpu)
        t1 = time.perf_counter()
        open_stages = {k: round(x, 1) for k, x in v.open_timings().items()}
        v.run()
        t2 = time.perf_counter()
        cuts = v.scene_cuts()
        v.frame_pts()
        v.boundary_frames([0.0, float(v.info.duration)])
        t3 = time.perf_counter()
        v.close()
        stages = {"open_ms": round((t1 - t0) * 1e3, 1), "open_stages_ms": open_stages,
                  "decode_score_ms": round((t2 - t1) * 1e3, 1),
                  "results_ms": round((t3 - t2) * 1e3, 2), "scene_cuts": len(cuts),
                  "input_bytes": Path(p).stat().st_size,
                  "upload_inclusive_GBps": round(Path(p).stat().st_size / (t1 - t0) / 1e9, 2)}
    for it in items:
        frames += int(round(it.duration * FPS))
    return {"videos": len(paths), "frames": frames, "seconds": round(dt, 3),
            "value": round(frames / dt, 1), "unit": "frames/s",
            "segments": [it.n_segments for it in items], "cuts": [it.n_cuts for it in items],
            "first_video_stages": stages,
            "includes": "per video: moov probe, plan, vts_open (host MP4 demux, elementary-stream "
                        "upload H2D, decode schedule), decode + score, scores D2H, scene cuts, "
                        "boundary frames, close; files in the page cache; the second plan_batch "
                        "call of the process (the first, untimed, sets up its stream pool and "
                        "device allocator)"}


# HIP hardware queues: the bench runs on whatever the process inherits (HIP's
# default 4, which the GPU box exports); sessions opened beside others take
# streams with hardware queues of their own (session.hip streams_take), so
# concurrent sessions overlap without GPU_MAX_HW_QUEUES (round 5 forced 16
# here).  VTS_BENCH_HW_QUEUES sets it for a measurement.
# general-decoder records beyond 10 min: config [2]'s path (a 30-min content
# stream in three windows) and config [4]'s resolution (a 5-min 1080p one)
GLONG_FRAMES = 54000
GLONG_WINDOW = 18000
GHD_FRAMES = 9000


def main() -> None:
    if os.environ.get("VTS_BENCH_HW_QUEUES"):
        os.environ["GPU_MAX_HW_QUEUES"] = os.environ["VTS_BENCH_HW_QUEUES"]
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="decode_score", choices=["decode_score", "score", "transcode"])
    ap.add_argument("--config", default="720p-batch", choices=sorted(CONFIGS),
                    help="BASELINE configuration per GPU; default = config [3]'s per-GPU share "
                         "(4 x 10-min 720p) at every N")
    ap.add_argument("--videos-per-gpu", type=int, default=0, help="override the config's")
    ap.add_argument("--bframes", action="store_true",
                    help="with --coding full: B pictures (x264-like: B references, spatial direct, "
                         "implicit weighted bi-prediction, reordered presentation)")
    ap.add_argument("--coding", default="subset", choices=["subset", "full"],
                    help="synthetic stream syntax: subset = I_PCM + integer-motion P_Skip/P16x16 "
                         "(no residual, deblocking off: the subset kernels); full = intra 4x4/16x16, "
                         "residuals, quarter-sample partitions, 3 references, deblocking on (the "
                         "general decoder)")
    ap.add_argument("--video", default=None,
                    help="comma-separated MP4s (this rank's videos) instead of synthesizing them "
                         "(the rocprofv3 child passes)")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the oracle parity check of the run's results")
    ap.add_argument("--parity-frames", default="auto",
                    help="frames per video the parity pass checks: auto (all at N=1, a 3000-frame "
                         "prefix at N>1), all, or a number")
    ap.add_argument("--extras", default="all", choices=["all", "none"],
                    help="N=1: the e2e / long_video / general sub-records")
    ap.add_argument("--profile-dir", default=None,
                    help="keep the rocprofv3 kernel stats / busy-time summary here")
    ap.add_argument("--frames", type=int, default=None, help="override the config's frames")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--window-frames", type=int, default=0,
                    help="decoded-surface window in frames (vts_params.window_frames); 0 = sized from HBM")
    ap.add_argument("--gops-per-launch", type=int, default=0,
                    help="GOPs per reconstruct launch; <= 0 all GOPs of the window")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse the N>1 path with several ranks on one GPU")
    ap.add_argument("--parse-chunks", type=int, default=1,
                    help="slice-parse chunks overlapped with reconstruction (1 = none, the default)")
    ap.add_argument("--level-block", type=int, default=0,
                    help="GOP levels per reconstruct launch: 0 or 1 = one launch per level (the "
                         "default), >= 2 = the level-blocked kernel (opt-in, DESIGN 4.6)")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the rocprofv3 passes (kernel trace and --pmc) of the headline")
    args = ap.parse_args()

    # --gpus N > 1 with no launcher around us: start the N ranks ourselves
    # (before anything touches the GPU) and exit with their status
    try:
        plan = rank_launch_plan(args.gpus, os.environ, device_count(), args.dist_backend,
                                sys.argv[1:], port=_free_port)
    except LaunchError as exc:
        print(f"bench.py: {exc}", file=sys.stderr, flush=True)
        raise SystemExit(2)
    if plan is not None:
        cmd, env = plan
        log(f"launching {args.gpus} ranks: {' '.join(cmd[:9])} ...")
        raise SystemExit(relay_ranks(cmd, env))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    cw, ch, cf, cvpg, cdesc = CONFIGS[args.config]
    width = args.width or cw
    height = args.height or ch
    F = args.frames or cf
    vpg = args.videos_per_gpu or cvpg
    if args.workload != "decode_score":
        vpg = 1
    n_videos = vpg * world
    local_idx = list(range(rank, n_videos, world))
    k = 4 if height <= 720 else 6
    w, h = width // k, height // k
    stride = width * height * 3 // 2
    hc = host_cores()
    # N = 1: the oracle (parity pass = CPU baseline) on every usable host core;
    # N > 1: each rank's share of them (the parity pass only, no baseline)
    threads = max(1, hc["usable"] // max(1, world))
    extras = args.extras == "all" and world == 1 and args.workload == "decode_score" and \
        not args.no_parity

    # torch first: libvtseg.so must bind to the HIP runtime torch loads (loading
    # libvtseg first hides the device from it); importing torch initialises
    # no GPU, nor does the stream writer below
    import torch
    import torch.distributed as dist
    from vtseg import scene

    # ------------------------------------------------ input videos (host only)
    tmpdir = Path(tempfile.mkdtemp(prefix="vtseg_bench_"))
    all_paths = [tmpdir / f"synth_v{i}.mp4" for i in range(n_videos)]
    if args.workload != "score":
        if args.video:
            given = [Path(p) for p in args.video.split(",")]
            if len(given) != len(local_idx):
                raise SystemExit(f"--video: {len(given)} files for {len(local_idx)} local videos")
            for i, p in zip(local_idx, given):
                all_paths[i] = p
        else:
            t0 = time.perf_counter()
            synth_videos([(all_paths[i], 0x5EED + i) for i in local_idx], width, height, F,
                         args.coding, args.bframes)
            log(f"rank {rank}: wrote {len(local_idx)} synthetic videos in {time.perf_counter() - t0:.1f} s")
    local_paths = [all_paths[i] for i in local_idx]

    # extras' inputs, written before the profile passes (which read them)
    gen_path = long_path = content_path = hd_path = glong_path = ghd_path = None
    gen_info = content_info = glong_info = ghd_info = None
    gb_paths, gb_infos = [], []
    if extras:
        t0 = time.perf_counter()
        gen_path = tmpdir / "general_720p_10min.mp4"
        content_path = tmpdir / "general_content_720p_10min.mp4"
        long_path = tmpdir / "long_720p_2h.mp4"
        hd_path = tmpdir / "hd_1080p_30min.mp4"
        glong_path = tmpdir / "general_content_720p_30min.mp4"
        ghd_path = tmpdir / "general_content_1080p_5min.mp4"
        # config [3]'s share on real syntax: vpg content streams, and the worst
        # case beside them — half of a mixed batch noise streams (VERDICT r05
        # item 4)
        n_noise = max(1, vpg // 2)
        gb_paths = [content_path] + [tmpdir / f"general_content_720p_10min_{i}.mp4" for i in range(1, vpg)]
        gb_noise = [gen_path] + [tmpdir / f"general_720p_10min_{i}.mp4" for i in range(1, n_noise)]
        with ThreadPoolExecutor(12) as ex:
            fa = [ex.submit(synth_videos, [(p, 0x5EED + i)], 1280, 720, 18000, "full", True, True)
                  for i, p in enumerate(gb_noise)]
            fc = [ex.submit(synth_videos, [(p, 0x5EED + i)], 1280, 720, 18000, "full", True, True, True)
                  for i, p in enumerate(gb_paths)]
            fl = ex.submit(synth_videos, [(glong_path, 0x5EED + 100)], 1280, 720, GLONG_FRAMES, "full", True,
                           True, True)
            fh = ex.submit(synth_videos, [(ghd_path, 0x5EED + 200)], 1920, 1080, GHD_FRAMES, "full", True,
                           True, True)
            fb = ex.submit(synth_videos, [(long_path, 0x5EED)], 1280, 720, 216000)
            fd = ex.submit(synth_videos, [(hd_path, 0x5EED)], 1920, 1080, HD_FRAMES)
            noise_infos = [f.result()[0] for f in fa]
            gen_info = noise_infos[0]
            gb_infos = [f.result()[0] for f in fc]
            content_info = gb_infos[0]
            glong_info = fl.result()[0]
            ghd_info = fh.result()[0]
            fb.result()
            fd.result()
        gb_infos = gb_infos + noise_infos
        gb_paths = gb_paths + gb_noise
        log(f"extras inputs written in {time.perf_counter() - t0:.1f} s")

    prof = gprof = None
    if world == 1 and not args.no_pmc and args.workload != "transcode":
        # before anything touches the GPU: the passes are child processes
        child_argv = ["--workload", args.workload, "--config", args.config, "--coding", args.coding,
                      *(["--bframes"] if args.bframes else []),
                      "--videos-per-gpu", str(vpg),
                      "--gops-per-launch", str(args.gops_per_launch),
                      "--parse-chunks", str(args.parse_chunks),
                      "--level-block", str(args.level_block)]
        if args.workload != "score":
            child_argv += ["--video", ",".join(str(p) for p in local_paths)]
        for opt in ("frames", "width", "height"):
            if getattr(args, opt) is not None:
                child_argv += [f"--{opt}", str(getattr(args, opt))]
        pdir = Path(tempfile.mkdtemp(prefix="vtseg_prof_", dir="/tmp"))
        prof = profile_passes(child_argv, pdir,
                              Path(args.profile_dir) if args.profile_dir else None)
        if extras:
            gprof = {}
            for key, gp in (("general", gen_path), ("general_content", content_path)):
                gargv = ["--config", "720p-10min", "--coding", "full", "--bframes", "--video", str(gp)]
                gprof[key] = profile_passes(gargv, pdir / key,
                                            Path(args.profile_dir) / key if args.profile_dir else None,
                                            passes=("trace", GENERAL_PMC))
        shutil.rmtree(pdir, ignore_errors=True)

    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    gpu = local % max(ndev, 1)  # ranks > GPUs only in a gloo rehearsal on one box
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(gpu)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
    device = torch.device("cuda", gpu)
    torch.cuda.set_device(device)
    coll_dev = device if args.dist_backend == "nccl" else torch.device("cpu")
    # N = 1: the step's all-gathers still go through RCCL — a world-size-1
    # NCCL group and plan_batch(always_gather=True) — so the line measures the
    # same collective path every rank of an N > 1 run takes (not the
    # profiler's child passes, which time the kernels only)
    one_rank_group = None
    if world == 1 and args.dist_backend == "nccl" and args.workload == "decode_score" and not args.video:
        try:
            dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                                    world_size=1, device_id=device)
            one_rank_group = "rccl"
        except Exception as exc:  # noqa: BLE001 - reported in the line
            one_rank_group = f"none (RCCL world-size-1 group failed: {type(exc).__name__}: {exc})"
            log(f"RCCL at N=1 unavailable: {exc}")
    gather_always = one_rank_group == "rccl"

    from vtseg import batch
    from vtseg import budget_planner as bp
    from vtseg import video_segmenter as vs

    # ---------------------------------------------------------------- inputs
    scorers: dict = {}
    outs: dict = {}
    if args.workload == "score":
        rng = np.random.default_rng(100 + rank)
        pool = torch.from_numpy(smooth_frames_host(rng, 64, width, height)).to(device)
        reps = (F + 63) // 64
        nv12 = pool.reshape(64, -1).repeat(reps, 1)[:F].contiguous().reshape(-1)
        del pool

        def step():
            outs["r"] = scene.score_nv12(nv12, width=width, height=height, pitch=width,
                                         uv_row_offset=height, frame_stride=stride,
                                         n_frames=F, k=k, out=outs.get("r"),
                                         workspace=outs.get("r", {}).get("_workspace"))
        durations = [F / FPS]
    else:
        t0 = time.perf_counter()
        for i in local_idx:
            scorers[i] = scene.VideoScorer(all_paths[i], device=gpu,
                                           gops_per_launch=args.gops_per_launch,
                                           parse_chunks=args.parse_chunks,
                                           level_block=args.level_block,
                                           window_frames=args.window_frames)
        log(f"rank {rank}: opened {len(scorers)} sessions in {time.perf_counter() - t0:.1f} s")
        F = scorers[local_idx[0]].n_frames
        durations = [float(scorers[i].info.duration) for i in local_idx]

        if args.workload == "transcode":
            out_path = tmpdir / f"small_rank{rank}.mp4"
            v0 = scorers[local_idx[0]]

            def step():
                outs["facts"] = v0.transcode(out_path)
        else:
            str_paths = [str(p) for p in all_paths]

            def step():
                outs["items"] = batch.plan_batch(str_paths, REF_CONFIG, score=True,
                                                 sessions=scorers, always_gather=gather_always)

    def barrier():
        if world > 1:
            dist.barrier()

    # ---------------------------------------------------------------- timing
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    ms_per_step = elapsed / args.steps * 1e3
    total_frames = F * n_videos * args.steps
    value = total_frames / elapsed
    log(f"rank {rank}: {args.steps} steps in {elapsed:.3f} s -> {value:.0f} frames/s")

    # ------------------------------------------- roofline (dominant kernel)
    roof = None
    sl = [scorers[i] for i in local_idx] if scorers else []
    if args.workload == "score":
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 5
        ev0.record()
        for _ in range(reps):
            step()
        ev1.record()
        torch.cuda.synchronize()
        kern_ms = ev0.elapsed_time(ev1) / reps
        alg_bpf = algorithmic_bytes_per_frame(width, height, k)
        achieved = alg_bpf * F / (kern_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                "kernel": "score_runs<%d>" % k, "kernel_ms": round(kern_ms, 5),
                "kernel_ms_basis": "torch events on the current stream (score_nv12 enqueues there)",
                "bytes_per_frame": alg_bpf, "frames_per_launch": F}
    elif args.workload == "transcode":
        # dominant kernel: enc_search<8> (VALU: v_sad_u8, 4 byte-SADs per lane-instruction)
        facts = outs["facts"]
        R = 8
        sw, sh = facts["width"], facts["height"]
        nmb = ((sw + 15) // 16) * ((sh + 15) // 16)
        p_frames = F - facts["n_idr"]
        n_launch = max(1, min(250, F) - 1)
        sad_ops = p_frames * nmb * (2 * R + 1) ** 2 * 256
        kern_ms = facts["search_ms"] / n_launch
        achieved = sad_ops / n_launch / (kern_ms * 1e-3) / 1e12
        roof = {"bound": "valu", "achieved": round(achieved, 2), "peak": VALU_SAD_PEAK_TOPS,
                "unit": "T byte-SAD/s", "frac": round(achieved / VALU_SAD_PEAK_TOPS, 4),
                "traffic": None, "kernel": "enc_search<8>", "kernel_ms": round(kern_ms, 4),
                "sad_ops_per_launch": int(sad_ops / n_launch),
                "frames_per_launch": round(p_frames / n_launch, 1),
                "note": "full-search (2R+1)^2 x 256 byte |a-b| per macroblock, R=8; peak = 256 CUs x "
                        "4 SIMDs x 32 lanes/clk x 4 B (v_sad_u8) x 2.4 GHz"}
    else:
        roof = roofline_decode_score(sl, prof, width, height, k, F)
    roof_decode = None
    if args.workload == "decode_score" and not sl[0].fused():
        t = sl[0].timings()
        n_launch = sl[0].recon_launches()
        rec_ms = t["reconstruct_ms"] / n_launch
        rec_bytes = 3 * width * height
        ach = rec_bytes * (F / n_launch) / (rec_ms * 1e-3) / 1e9
        roof_decode = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                       "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                       "kernel": ("reconstruct level: h264_inter_full + h264_intra_v2 + h264_deblock_plane "
                                  "(h264_bs_full beside the chain)" if sl[0].general() else "h264_recon"),
                       "kernel_ms": round(rec_ms, 4),
                       "launches": n_launch, "bytes_per_frame": rec_bytes,
                       "frames_per_launch": round(F / n_launch, 1)}

    items = outs.get("items")
    counts = [it.n_segments for it in items] if items else None
    stage_info = ({"stage_ms": sl[0].timings(), "recon_launches": sl[0].recon_launches(),
                   "windows": sl[0].windows()} if sl else {})

    # ------------------------------------- parity vs the CPU oracle (+ baseline)
    parity, cpu = None, None
    if args.workload == "decode_score" and not args.no_parity:
        if args.parity_frames == "all":
            maxf = None
        elif args.parity_frames == "auto":
            maxf = None if world == 1 else min(F, 3000)
        else:
            maxf = min(F, int(args.parity_frames))
        dec = "full" if sl[0].general() else "subset"
        per_video, secs, nfr = [], 0.0, 0
        records_ok = True
        for i in local_idx:
            v = scorers[i]
            duration = float(v.info.duration)
            plan = bp.plan_segments_with_budget(duration, REF_CONFIG, 0)
            segs = vs.plan_segments(duration, plan.segment_duration, plan.overlap)
            par, ct = parity_check(v, all_paths[i], k, segs, threads, maxf, dec)
            par["video"] = i
            per_video.append(par)
            secs += ct["seconds"]
            nfr += ct["frames"]
            if items is not None:
                ok = batch_record_check(items[i], segs, ct, maxf is None or ct["frames"] >= F)
                par["batch_record_equal"] = ok
                records_ok &= ok
        parity = {"videos": len(per_video), "frames": nfr, "of_frames": F * len(per_video),
                  "scores_equal": all(p["scores_equal"] for p in per_video),
                  "max_abs_score_diff": max(p["max_abs_score_diff"] for p in per_video),
                  "score_tolerance": 1e-4,
                  "hist_equal": all(p["hist_equal"] for p in per_video),
                  "sad_equal": all(p["sad_equal"] for p in per_video),
                  "scene_cuts": sum(p["scene_cuts"] for p in per_video),
                  "scene_cuts_equal": all(p["scene_cuts_equal"] for p in per_video),
                  "segment_times": sum(p["segment_times"] for p in per_video),
                  "boundary_frames_equal": all(p["boundary_frames_equal"] for p in per_video),
                  "pts_equal": all(p["pts_equal"] for p in per_video),
                  "batch_records_equal": records_ok if items is not None else None,
                  "oracle": ("oracle/h264_full_oracle.c fo_decode" if dec == "full" else
                             "oracle/vtseg_oracle.c or_decode_samples") +
                            f" + or_score_frames (GOP-parallel, {threads} threads)"}
        parity["all_equal"] = all(p["all_equal"] for p in per_video) and \
            (records_ok if items is not None else True)
        if world > 1:
            ok = torch.tensor([1 if parity["all_equal"] else 0], dtype=torch.int32, device=coll_dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            parity["all_ranks_equal"] = bool(ok.item())
            parity["checked_on_each_rank"] = f"{len(per_video)} videos x {nfr // max(1, len(per_video))} frames"
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            cpu = {"value": round(nfr / secs, 2), "unit": "frames/s", "cores": threads, "kind": "port",
                   "host_cores": hc,
                   "note": "the oracle: an unoptimised scalar C restatement of the decoder and scorer used as "
                           "the parity checker, not an ffmpeg-class CPU decoder (ffmpeg, the reference's own "
                           "path, is absent from the image); a GPU / CPU ratio from it says nothing about "
                           "kernel quality",
                   "sample": f"the parity pass: {nfr} frames ({width}x{height}, {len(per_video)} "
                             f"videos) of the benchmark batch decoded by " +
                             ("oracle/h264_full_oracle.c fo_decode" if dec == "full" else
                              "oracle/vtseg_oracle.c or_decode_samples") +
                             f" + scored by or_score_frames, GOP-parallel on {threads} "
                             f"threads = every usable host core (affinity {hc['affinity']}, cgroup "
                             f"quota {hc['cgroup_quota'] or 'none'}), {secs:.1f} s"}
        log(f"rank {rank}: parity all_equal={parity['all_equal']}")
    if rank == 0 and world == 1 and not args.no_cpu_baseline and cpu is None:
        if args.workload == "score":
            cpu = cpu_baseline_score(width, height, k)
        elif args.workload == "transcode":
            cpu = cpu_baseline_transcode(all_paths[0], k)

    # -------------------------------------------------- extras (N = 1 only)
    extra = {}
    if extras:
        try:
            extra["e2e"] = e2e_record(local_paths, gpu)
            log(f"e2e: {extra['e2e']['value']} frames/s")
        except Exception as exc:  # noqa: BLE001 - reported in the line
            extra["e2e"] = {"error": f"{type(exc).__name__}: {exc}"}
        # the batch's sessions give their HBM back before the 2-h video's rings
        for v in sl:
            v.close()
        # the general streams first: after the 2-h video's session its cached
        # segments cannot host the general decoder's ~56 GB coefficient arena,
        # and HBM released to the driver is cleared again before reuse (DESIGN
        # §0 item 4)
        for key, p, label, info in (
                ("general", gen_path, "general decoder, worst case: 10-min 720p x264-structured "
                                      "full-syntax NOISE stream (random syntax decisions and residuals; "
                                      "High profile: CABAC, 8x8 transform and Intra_8x8, B pyramid with "
                                      "B references, spatial direct, implicit weighted bi-prediction, 3 "
                                      "references, deblocking, one slice per picture)", gen_info),
                ("general_content", content_path, "general decoder, video-like: 10-min 720p CONTENT "
                                                  "stream (synth_content.h: textured scenes with planted "
                                                  "cuts, a panning background and moving sprites coded in "
                                                  "closed loop by SAD decisions with quantised residuals; "
                                                  "CABAC, 8x8 transform, B pyramid, implicit weights, "
                                                  "deblocking, keyint ~8 s)", content_info),
                ("general_long", glong_path, f"BASELINE config [2]'s path on real syntax: one "
                                             f"{GLONG_FRAMES / FPS / 60:.0f}-min 720p CONTENT stream "
                                             f"({GLONG_FRAMES} frames, the general decoder in windows of "
                                             f"{GLONG_WINDOW} frames on two rings: parse of window i + 1 "
                                             f"beside the reconstruction of window i)", glong_info),
                ("general_hd", ghd_path, f"BASELINE config [4]'s resolution on real syntax: one "
                                         f"{GHD_FRAMES / FPS / 60:.0f}-min 1080p CONTENT stream "
                                         f"({GHD_FRAMES} frames, coded 1920x1088 with display crop, "
                                         f"thumbnails k=6, general decoder)", ghd_info),
                ("long_video", long_path, "BASELINE config [2]: one 2-h 720p video "
                                          "(216 000 frames), streamed two-ring decode", None),
                ("hd_1080p", hd_path, f"BASELINE config [4] per-GPU share, sampled: one 1080p video of "
                                      f"{HD_FRAMES / FPS / 60:.0f} min ({HD_FRAMES} frames; config [4] is 2 h "
                                      f"per GPU), coded 1920x1088 with display crop, thumbnails k=6, "
                                      f"streamed decode", None)):
            try:
                r = run_single(p, gpu=gpu, k=6 if key in ("hd_1080p", "general_hd") else 4, steps=3,
                               threads=threads, label=label, planted=info["cuts"] if info else None,
                               window_frames=GLONG_WINDOW if key == "general_long" else 0)
                if gprof and gprof.get(key):
                    r["kernels"] = general_kernel_rooflines(gprof[key], 1280, 720, 4, r["frames"],
                                                            80 * 45)
                extra[key] = r
                log(f"{key}: {r['value']} frames/s, parity {r.get('parity', {}).get('all_equal')}")
            except Exception as exc:  # noqa: BLE001 - reported in the line
                extra[key] = {"error": f"{type(exc).__name__}: {exc}"}
        # config [3]'s four general sessions last: their ~196 GB fit beside what
        # the 2-h video's session left cached (carved from its segments, the
        # rest fresh), while before it the 2-h video's 45 GB rings found no
        # cached segment that large, HIP memory ran out and the cache went back
        # to the driver, whose clear then cost the open ~6 s (r05d: alloc_ms
        # 6 230)
        try:
            extra["general_batch"] = general_batch_record(gb_paths, gpu, threads, [x["cuts"] for x in gb_infos],
                                                          n_content=vpg)
            log(f"general_batch: {extra['general_batch']['value']} frames/s, "
                f"x{extra['general_batch']['batch_over_single']} of one video's step, "
                f"mixed {extra['general_batch']['mixed']['value']} frames/s, "
                f"parity {extra['general_batch']['parity']['all_equal']}")
        except Exception as exc:  # noqa: BLE001 - reported in the line
            extra["general_batch"] = {"error": f"{type(exc).__name__}: {exc}"}

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "frames/s",
            **placement(world, ndev),
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u8", "data": "synthetic",
            "config": {"workload": f"{args.workload}: {cdesc}; synthetic H.264 {width}x{height} "
                                   + ("(full syntax" + (", B pictures" if args.bframes else "") + ") "
                                      if args.coding == "full" else "")
                                   + f"@30fps, {vpg} x {F} frames ({F / FPS / 60:.1f} min) per GPU, "
                                   f"thumbnails k={k}",
                       "config_name": args.config,
                       "videos": n_videos, "videos_per_gpu": vpg,
                       "frames_per_video": F, "frames_per_gpu": F * vpg,
                       "width": width, "height": height, "k": k,
                       "parallelism": f"video-per-gpu x{world} (video i on rank i mod {world})",
                       "collectives": ("plan_batch: all_gather_into_tensor of per-video records + "
                                       "padded boundary arrays, " +
                                       (args.dist_backend if world > 1 else
                                        ("rccl (world-size-1 NCCL group, always_gather) at N=1"
                                         if gather_always else (one_rank_group or "none at N=1")))),
                       "segment_counts": counts,
                       "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "unset (HIP default 4)")},
            "roofline": roof,
            "roofline_decode": roof_decode,
            "parity": parity,
            "cpu_baseline": cpu,
        }
        if args.workload == "transcode":
            f = outs["facts"]
            line["metric"] = "720p frames/sec transcoded to 360p (upload compression, SURVEY 8f-2)"
            line["config"]["transcode"] = {kk: (round(v, 3) if isinstance(v, float) else v)
                                           for kk, v in f.items()}
            line["config"]["transcode"]["input_bytes"] = Path(all_paths[0]).stat().st_size
        elif sl:
            line["config"].update(stage_info)
            line["config"]["bits_per_frame"] = round(
                sum(Path(p).stat().st_size for p in local_paths) * 8 / (F * len(local_paths)), 1)
        line.update(extra)
        print(json.dumps(line), flush=True)
    for v in sl:
        v.close()
    if not args.video:
        shutil.rmtree(tmpdir, ignore_errors=True)
    else:
        for p in (gen_path, long_path, hd_path, glong_path, ghd_path, *gb_paths):
            if p is not None:
                Path(p).unlink(missing_ok=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    elif gather_always:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
