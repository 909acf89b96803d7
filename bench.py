"""Benchmark: 720p frames/s decoded+scored per node (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload decode_score|score|transcode]
                    [--config 720p-2h|720p-10min|1080p-2h|480p-60s] [--profile-dir DIR]

One process per GPU (torch.distributed.run for N > 1; RANK/LOCAL_RANK/
WORLD_SIZE from the env, rendezvous on 127.0.0.1).  Weak scaling: every rank
processes its own synthetic video; after each step the ranks all-gather their
per-video segment counts over RCCL (the only collective on this path; no pixel
data crosses GPUs).  The default (N=1) workload is BASELINE config [2], the
largest single-GPU configuration: a 2-h 720p video (216 000 frames at 30 fps),
decoded in streamed two-ring windows.

A step = one pass of the hot path over one whole video with its input already
resident in HBM:
  decode_score : device H.264 subset decode (parse + reconstruct) + scoring
  score        : scoring kernel only, on pre-decoded NV12 frames
  transcode    : the 360p upload transcode
Rank 0 prints ONE JSON line (contract in the task statement), including
  roofline     : the dominant kernel; `achieved`/`frac` on SURVEY 8(d)'s
                 algorithmic bytes per frame, kernel time = busy time (union of
                 dispatch intervals) per dispatch from a rocprofv3 kernel trace
                 of this same command (HIP-event value beside it), `traffic`
                 from rocprofv3 PMC passes; the decode-inclusive figure beside;
  parity       : this run's scores / histograms / SADs, scene cuts and the
                 planned segments' boundary frame indices against the C oracle
                 over the whole video (bounded prefix per rank for N > 1);
  cpu_baseline : the oracle's decode + score on the host's cores (the parity
                 pass, timed), N = 1 only.
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
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "video-transformer_amd"))
sys.path.insert(0, str(ROOT / "oracle"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
VALU_SAD_PEAK_TOPS = 256 * 4 * 32 * 4 * 2.4e9 / 1e12  # v_sad_u8 byte-SADs/s (MI355X_MICROARCH.md)

# BASELINE.json configs runnable per GPU: name -> (width, height, frames, what)
CONFIGS = {
    "720p-10min": (1280, 720, 18000, "BASELINE config [1]: 10-min 720p MP4, one per GPU"),
    "720p-2h": (1280, 720, 216000, "BASELINE config [2]: 2-h 720p, streamed decode "
                                   "(two-ring windows)"),
    "1080p-2h": (1920, 1080, 216000, "BASELINE config [4] per GPU: 2-h 1080p, two-stream "
                                     "decode/score overlap"),
    "480p-60s": (640, 480, 1800, "BASELINE config [0] clip (60-s 480p) on the GPU path"),
}
FPS = 30
METRIC = "720p frames/sec decoded+scored per node; segment-index exact-match vs CPU"


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


def cpu_baseline_decode_score(path, k, budget_s=15.0):
    """The same decode + score on the host: the C oracle's H.264 subset
    decoder (or_decode_samples) and scorer (or_score_frames), GOP-parallel on
    a thread pool (ctypes releases the GIL), over a bounded GOP-aligned sample
    of the benchmark video itself."""
    import ctypes as C
    from concurrent.futures import ThreadPoolExecutor

    import oracle
    m = oracle.read_mp4(path)
    L = oracle.lib()
    prm = oracle.H264Params()
    sps, pps = m["sps"][0], m["pps"][0]
    if L.or_parse_sps_pps(sps, len(sps), pps, len(pps), m["nal_length_size"], C.byref(prm)):
        raise RuntimeError("oracle SPS/PPS")
    W = prm.mb_width * 16 - prm.crop_right
    H = prm.mb_height * 16 - prm.crop_bottom
    data = np.frombuffer(m["data"], np.uint8)
    offs = np.asarray(m["offsets"], np.int64)
    sizes = np.asarray(m["sizes"], np.int64)
    nls = m["nal_length_size"]
    idr = [i for i in range(len(offs)) if data[offs[i] + nls] & 0x1F == 5]
    gops = [(a, b) for a, b in zip(idr, idr[1:] + [len(offs)])]

    def work(g):
        a, b = g
        n = b - a
        out = np.empty((n, H * 3 // 2, W), np.uint8)
        bad = C.c_int64(-1)
        if L.or_decode_samples(C.byref(prm), data.ctypes.data, offs[a:b].ctypes.data,
                               sizes[a:b].ctypes.data, n, out.ctypes.data, C.byref(bad)):
            raise RuntimeError("oracle decode")
        oracle.score_frames(out.reshape(-1), W * H * 3 // 2, n, W, H, W, H, k, want_rgb=True)
        return n

    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    t0 = time.perf_counter()
    per_gop = work(gops[0]) and (time.perf_counter() - t0)
    n_gops = max(1, min(len(gops), int(budget_s * threads / max(per_gop, 1e-6))))
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        frames = sum(ex.map(work, gops[:n_gops]))
    dt = time.perf_counter() - t0
    return {"value": round(frames / dt, 2), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"first {n_gops} GOPs ({frames} frames {W}x{H}) of the benchmark video, "
                      f"decoded by oracle/vtseg_oracle.c or_decode_samples + scored by "
                      f"or_score_frames, GOP-parallel on {threads} threads, {dt:.1f} s"}


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


def profile_passes(argv: list[str], out_dir: Path, keep_dir: Path | None) -> dict:
    """rocprofv3 child runs of this same benchmark (1 timed step each):
      * --kernel-trace --stats: per kernel, dispatches, mean dispatch duration
        and busy time (union of the dispatch intervals) per dispatch; with two
        GOP groups two reconstruct dispatches overlap, so the mean duration
        overstates each one's share of the wall time and the busy time is the
        kernel time per launch;
      * --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes: 3 + 2 TCC
        slots > 4): HBM bytes per dispatch = 2 x FETCH_SIZE (gfx950 tallies
        wide coalesced reads at half their bytes) + WRITE_SIZE, both KiB
        (MI355X_MICROARCH.md, HBM section).
    Started before this process initialises the GPU (no exec from a
    GPU-initialised process), each under its own time limit."""
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not Path(prof).exists():
        return {"error": "rocprofv3 not found"}
    res: dict = {}
    env = dict(os.environ, TMPDIR="/tmp")
    child = [sys.executable, str(Path(__file__).resolve()), *argv, "--steps", "1", "--warmup", "1",
             "--no-cpu-baseline", "--no-pmc", "--no-parity"]
    for what in ("trace", "FETCH_SIZE", "WRITE_SIZE"):
        d = out_dir / what
        opts = (["--kernel-trace", "--stats"] if what == "trace" else
                ["--kernel-trace", "--pmc", what])
        cmd = [prof, *opts, "--output-format", "csv", "-d", str(d), "-o", "run", "--", *child]
        try:
            proc = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True,
                                  timeout=240)
        except subprocess.TimeoutExpired:
            res["error"] = f"{what} pass timed out"
            continue
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
                                             mean_dispatch_ns=total / len(v))
            if keep_dir is not None:
                keep_dir.mkdir(parents=True, exist_ok=True)
                for f in d.rglob("*kernel_stats.csv"):
                    shutil.copy(f, keep_dir / "kernel_stats.csv")
                rows = sorted(((k, v) for k, v in res.items() if "busy_ns_per_dispatch" in v),
                              key=lambda kv: -kv[1]["busy_ns_per_dispatch"] * kv[1]["dispatches_traced"])
                (keep_dir / "kernel_busy.txt").write_text("".join(
                    f"{k}: {v['dispatches_traced']} dispatches, busy (union of intervals) "
                    f"{v['busy_ns_per_dispatch'] / 1e3:.2f} us per dispatch, mean dispatch "
                    f"duration {v['mean_dispatch_ns'] / 1e3:.2f} us\n" for k, v in rows))
            continue
        acc: dict = {}
        for f in d.rglob("*counter_collection.csv"):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if r["Counter_Name"] != what:
                        continue
                    acc.setdefault(_kernel_short(r["Kernel_Name"]), []).append(
                        float(r["Counter_Value"]))
        for k, v in acc.items():
            res.setdefault(k, {})[what] = sum(v) / len(v)
            res[k]["dispatches"] = len(v)
    for k, row in res.items():
        if isinstance(row, dict) and "FETCH_SIZE" in row and "WRITE_SIZE" in row:
            row["hbm_bytes"] = (2 * row["FETCH_SIZE"] + row["WRITE_SIZE"]) * 1024
    if keep_dir is not None:
        (keep_dir / "profile_passes.json").write_text(json.dumps(res, indent=1))
    return res


def parity_check(scorer, path, k: int, duration_s: float, segs, threads: int,
                 max_frames: int | None, decoder: str = "subset") -> tuple[dict, dict]:
    """This run's device results against the C oracle (oracle.decode_score_gops,
    GOP-parallel on `threads` host threads): every frame's fp32 score (exact;
    north_star allows |d| <= 1e-4), 256-bin histogram and SAD, the scene cuts,
    and the boundary frame index of every planned segment time (start, end,
    effective start/end of each segment of the reference's plan,
    src/utils/video_segmenter.py:42-83) in exact rationals.  Returns (parity,
    cpu timing of the oracle pass)."""
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
              "pts_equal": res.pts[:n].tolist() == ref["pts"],
              "oracle": ("oracle/h264_full_oracle.c fo_decode" if decoder == "full" else
                         "oracle/vtseg_oracle.c or_decode_samples") +
                        f" + or_score_frames (GOP-parallel, {threads} threads)"}
    parity["all_equal"] = all(parity[x] for x in ("scores_equal", "hist_equal", "sad_equal",
                                                  "scene_cuts_equal", "boundary_frames_equal",
                                                  "pts_equal"))
    return parity, {"frames": n, "seconds": ref["seconds"], "threads": threads,
                    "gops": ref["gops"], "width": ref["width"], "height": ref["height"]}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="decode_score", choices=["decode_score", "score", "transcode"])
    ap.add_argument("--config", default="720p-2h", choices=sorted(CONFIGS),
                    help="BASELINE configuration (per GPU); the N=1 headline is 720p-2h, the "
                         "largest single-GPU config")
    ap.add_argument("--bframes", action="store_true",
                    help="with --coding full: B pictures (x264-like: B references, spatial direct, "
                         "implicit weighted bi-prediction, reordered presentation)")
    ap.add_argument("--coding", default="subset", choices=["subset", "full"],
                    help="synthetic stream syntax: subset = I_PCM + integer-motion P_Skip/P16x16 "
                         "(no residual, deblocking off: the subset kernels); full = intra 4x4/16x16, "
                         "residuals, quarter-sample partitions, 3 references, deblocking on (the "
                         "general decoder)")
    ap.add_argument("--video", default=None,
                    help="use this MP4 instead of synthesizing one (the rocprofv3 child passes)")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the oracle parity check of the run's results")
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
                    help="GOP levels per reconstruct launch (0 auto = level-blocked kernel where it "
                         "applies, 1 = one launch per level)")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the rocprofv3 --pmc passes that fill roofline.traffic")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    cw, ch, cf, cdesc = CONFIGS[args.config]
    width = args.width or cw
    height = args.height or ch
    F = args.frames or cf
    k = 4 if height <= 720 else 6
    w, h = width // k, height // k
    stride = width * height * 3 // 2

    # torch first: libvtseg.so must bind to the HIP runtime torch loads (loading
    # libvtseg first hides the device from it); importing torch initialises
    # no GPU, nor does the stream writer below
    import torch
    import torch.distributed as dist
    from vtseg import scene

    # ------------------------------------------------ input video (host only)
    tmpdir = tempfile.mkdtemp(prefix="vtseg_bench_")
    path = None
    if args.workload != "score":
        if args.video:
            path = Path(args.video)
        else:
            path = Path(tmpdir) / f"synth_rank{rank}.mp4"
            if args.coding == "full":
                # --bframes: x264-like structure (B reference pictures, spatial
                # direct, implicit weighted bi-prediction, composition offsets)
                extra = dict(bframes=True, weighted="implicit") if args.bframes else {}
                scene.synth_write(path, width=width, height=height, fps=FPS, n_frames=F,
                                  seed=0x5EED + rank, coding="full", slices_per_row=0,
                                  max_motion=4, **extra)
            else:
                scene.synth_write(path, width=width, height=height, fps=FPS, n_frames=F,
                                  seed=0x5EED + rank)

    prof = None
    if world == 1 and not args.no_pmc and args.workload != "transcode":
        # before anything touches the GPU: the passes are child processes
        child_argv = ["--workload", args.workload, "--config", args.config, "--coding", args.coding,
                      *(["--bframes"] if args.bframes else []),
                      "--gops-per-launch", str(args.gops_per_launch),
                      "--parse-chunks", str(args.parse_chunks),
                      "--level-block", str(args.level_block)]
        if path is not None:
            child_argv += ["--video", str(path)]
        for opt in ("frames", "width", "height"):
            if getattr(args, opt) is not None:
                child_argv += [f"--{opt}", str(getattr(args, opt))]
        pdir = Path(tempfile.mkdtemp(prefix="vtseg_prof_", dir="/tmp"))
        prof = profile_passes(child_argv, pdir,
                              Path(args.profile_dir) if args.profile_dir else None)
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

    from vtseg import budget_planner as bp
    from vtseg import video_segmenter as vs

    # ---------------------------------------------------------------- inputs
    scorer = None
    if args.workload == "score":
        rng = np.random.default_rng(100 + rank)
        pool = torch.from_numpy(smooth_frames_host(rng, 64, width, height)).to(device)
        reps = (F + 63) // 64
        nv12 = pool.reshape(64, -1).repeat(reps, 1)[:F].contiguous().reshape(-1)
        del pool
        outs = {}

        def step():
            outs["r"] = scene.score_nv12(nv12, width=width, height=height, pitch=width,
                                         uv_row_offset=height, frame_stride=stride,
                                         n_frames=F, k=k, out=outs.get("r"),
                                         workspace=outs.get("r", {}).get("_workspace"))
        duration_s = F / FPS
    else:
        scorer = scene.VideoScorer(path, device=gpu, gops_per_launch=args.gops_per_launch,
                                   parse_chunks=args.parse_chunks, level_block=args.level_block,
                                   window_frames=args.window_frames)
        duration_s = float(scorer.info.duration)
        F = scorer.n_frames

        if args.workload == "transcode":
            out_path = Path(tmpdir) / f"small_rank{rank}.mp4"
            outs = {}

            def step():
                outs["facts"] = scorer.transcode(out_path)
        else:
            def step():
                scorer.run()

    # per-video segment plan under the reference's default config (config.yaml)
    cfg = {"analyzer": {"max_continuations": 3, "retry_times": 5,
                        "long_video": {"enabled": True, "default_segment_seconds": 480,
                                       "overlap_seconds": 20, "min_segment_seconds": 90,
                                       "hard_max_api_calls": 50, "consolidate": True,
                                       "duration_threshold_seconds": None}}}
    plan = bp.plan_segments_with_budget(duration_s, cfg, 0)
    segs = vs.plan_segments(duration_s, plan.segment_duration, plan.overlap)
    n_segments = len(segs)
    counts_local = torch.tensor([n_segments], dtype=torch.int32, device=coll_dev)
    counts_all = torch.zeros(world, dtype=torch.int32, device=coll_dev)

    def gather_counts():
        if world > 1:
            dist.all_gather_into_tensor(counts_all, counts_local)
        else:
            counts_all.copy_(counts_local)

    def barrier():
        if world > 1:
            dist.barrier()

    # ---------------------------------------------------------------- timing
    for _ in range(args.warmup):
        step()
        gather_counts()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        gather_counts()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    ms_per_step = elapsed / args.steps * 1e3
    total_frames = F * world * args.steps
    value = total_frames / elapsed

    # ------------------------------------------- roofline (dominant kernel)
    roof = None
    tb_launches, tb_chains = 0, 0
    if args.workload == "score":
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 5
        ev0.record()
        for _ in range(reps):
            step()
        ev1.record()
        torch.cuda.synchronize()
        kern_ms = ev0.elapsed_time(ev1) / reps
        kname = "score_runs<4>"
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
        kname = "enc_search<8>"
    else:
        times = []
        for _ in range(3):
            scorer.run()
            times.append(scorer.timings())
        tb_launches, tb_chains = scorer.level_blocks()
        n_launch = tb_launches or scorer.recon_launches()
        fused = scorer.fused()
        rec_ms = float(np.mean([t["reconstruct_ms"] for t in times])) / n_launch
        if fused:
            # dominant kernel = h264_recon_score (decode + score in one pass)
            kern_ms = rec_ms
            kname = ("h264_recon_score_tb" if tb_launches else
                     "h264_recon_score6b" if k == 6 else "h264_recon_score<%d>" % k)
        else:
            # one score_runs launch per window: per-launch time and frames
            n_score = max(1, scorer.windows())
            kern_ms = float(np.mean([t["score_ms"] for t in times])) / n_score
            kname = "score_runs<%d>" % k
    kern_ms_events = kern_ms
    kern_basis = "HIP events on the kernel's stream"
    prow = (prof or {}).get(kname) if isinstance((prof or {}).get(kname), dict) else None
    if args.workload == "decode_score" and prow and "busy_ns_per_dispatch" in prow:
        # the rocprofv3 kernel trace of this same command: union of the
        # dispatch intervals per dispatch (two GOP groups overlap)
        kern_ms = prow["busy_ns_per_dispatch"] / 1e6
        kern_basis = (f"rocprofv3 --kernel-trace of this command: busy time (union of "
                      f"{prow['dispatches_traced']} dispatch intervals) per dispatch; mean "
                      f"dispatch duration {prow['mean_dispatch_ns'] / 1e3:.2f} us")
    alg_bpf = algorithmic_bytes_per_frame(width, height, k)
    if args.workload == "transcode":
        bytes_per_frame = None
        frames_per_launch = p_frames / n_launch
    elif scorer is not None and scorer.fused() and tb_launches:
        frames_per_launch = F / n_launch
        bytes_per_frame = tb_bytes_per_launch(width, height, k, F, tb_chains, n_launch) / frames_per_launch
    elif scorer is not None and scorer.fused():
        bytes_per_frame = fused_bytes_per_frame(width, height, k)
        frames_per_launch = F / n_launch
    elif scorer is not None:
        bytes_per_frame = alg_bpf
        frames_per_launch = F / max(1, scorer.windows())
    else:
        bytes_per_frame = alg_bpf
        frames_per_launch = F
    if args.workload == "transcode":
        achieved = sad_ops / n_launch / (kern_ms * 1e-3) / 1e12
    else:
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
    if args.workload == "transcode":
        roof = {"bound": "valu", "achieved": round(achieved, 2), "peak": VALU_SAD_PEAK_TOPS,
                "unit": "T byte-SAD/s", "frac": round(achieved / VALU_SAD_PEAK_TOPS, 4),
                "traffic": None, "kernel": kname, "kernel_ms": round(kern_ms, 4),
                "sad_ops_per_launch": int(sad_ops / n_launch),
                "frames_per_launch": round(frames_per_launch, 1),
                "note": "full-search (2R+1)^2 x 256 byte |a-b| per macroblock, R=8; peak = 256 CUs x "
                        "4 SIMDs x 32 lanes/clk x 4 B (v_sad_u8) x 2.4 GHz"}
    else:
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
    roof_decode = None
    if args.workload == "decode_score" and not scorer.fused():
        rec_bytes = 3 * width * height
        ach = rec_bytes * (F / n_launch) / (rec_ms * 1e-3) / 1e9
        roof_decode = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                       "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                       "kernel": ("reconstruct level: h264_inter_full + h264_intra_full + h264_bs_full + "
                                  "h264_deblock_full" if scorer.general() else "h264_recon"),
                       "kernel_ms": round(rec_ms, 4),
                       "launches": n_launch, "bytes_per_frame": rec_bytes,
                       "frames_per_launch": round(F / n_launch, 1)}

    counts = counts_all.cpu().tolist()

    # ------------------------------------- parity vs the CPU oracle (+ baseline)
    parity, cpu = None, None
    if args.workload == "decode_score" and not args.no_parity:
        aff = len(os.sched_getaffinity(0))
        threads = max(1, min(16, aff // max(1, world)))
        # N > 1: every rank checks a bounded GOP-aligned prefix of its video
        maxf = None if world == 1 else min(F, 3000)
        dec = "full" if scorer.general() else "subset"
        if dec == "full" and world == 1:
            maxf = min(F, 18000)  # the general oracle decodes ~350 720p frames/s on 16 threads
        parity, ct = parity_check(scorer, path, k, duration_s, segs, threads, maxf, dec)
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            cpu = {"value": round(ct["frames"] / ct["seconds"], 2), "unit": "frames/s",
                   "cores": ct["threads"], "kind": "port",
                   "sample": f"the parity pass: {ct['frames']} frames ({ct['width']}x"
                             f"{ct['height']}, {ct['gops']} GOPs) of the benchmark video decoded by "
                             + ("oracle/h264_full_oracle.c fo_decode" if dec == "full" else
                                "oracle/vtseg_oracle.c or_decode_samples") +
                             f" + scored by or_score_frames, GOP-parallel on {ct['threads']} "
                             f"threads, {ct['seconds']:.1f} s"}
        if world > 1:
            ok = torch.tensor([1 if parity["all_equal"] else 0], dtype=torch.int32, device=coll_dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            parity["all_ranks_equal"] = bool(ok.item())
    if rank == 0 and world == 1 and not args.no_cpu_baseline and cpu is None:
        if args.workload == "score":
            cpu = cpu_baseline_score(width, height, k)
        elif args.workload == "transcode":
            cpu = cpu_baseline_transcode(path, k)
        else:
            cpu = cpu_baseline_decode_score(path, k)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u8", "data": "synthetic",
            "config": {"workload": f"{args.workload}: {cdesc}; synthetic H.264 {width}x{height} "
                                   + ("(full syntax" + (", B pictures" if args.bframes else "") + ") "
                                      if args.coding == "full" else "")
                                   + f"@30fps, {F} frames ({F / FPS / 60:.1f} min) per GPU, "
                                   f"thumbnails k={k}",
                       "config_name": args.config,
                       "frames_per_gpu": F, "width": width, "height": height, "k": k,
                       "parallelism": f"video-per-gpu x{world}",
                       "segment_counts": counts},
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
            line["config"]["transcode"]["input_bytes"] = Path(path).stat().st_size
        elif scorer is not None:
            line["config"]["stage_ms"] = scorer.timings()
            line["config"]["recon_launches"] = scorer.recon_launches()
            line["config"]["windows"] = scorer.windows()
        print(json.dumps(line), flush=True)
    if scorer is not None:
        scorer.close()
    if not args.video:
        shutil.rmtree(tmpdir, ignore_errors=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
