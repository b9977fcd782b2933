"""Benchmark: forward Gaussian-splat rasterization, frames/sec + Msplats/sec.

Headline workload (BASELINE.json configs[2] = SURVEY.md §8(d) C3): 1M synthetic Gaussians,
SH degree 3, 1920x1080, static camera, inputs resident in HBM.  One step = one full frame:
preprocess (EWA + SH) -> device radix depth sort -> binning -> tile sort -> ranges -> blend,
including the per-frame K readback the algorithm needs.  Four frames are in flight by
default (--inflight, `FramePipeline`: frame i on stream / context slot i % 4, one stream per
frame, so the next frames' latency-bound preprocess, sort and binning overlap this frame's
VALU-bound blend; every frame is still rendered in full and bit-identically);
`serial_ms_per_frame` reports one frame at a time.  With --gpus N (one process per GPU,
launched by torch.distributed.run) the frame's 16-px tile rows are split into N strips, every
rank renders its strip and rank 0 gathers the frame over RCCL (strong scaling: the frame is
fixed, N grows).  The untimed diagnostic passes (serial frame time, stage breakdown, in-flight
blend events) run before the W warmup frames, so the K timed frames measure a device that has
been rendering, as a viewer's does.

Prints ONE JSON line on rank 0.  `roofline` is for the dominant kernel (the blend) on the roof
that bounds it, VALU: its instructions per launch (a committed rocprofv3 SQ profile of this
build) over its launch duration from HIP events of a serial pass, with the HBM roof from the
committed FETCH/WRITE counters beside it; `cpu_baseline` times, on rank 0 at N = 1, the
reference's own CPU sort path (renderer_ogl.py:10-19, restated and pinned in oracle/) and the
CPU oracle of the whole forward (oracle/, a C port, OpenMP over the host cores).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import sys
import time

# A strip rank (N > 1) runs RCCL's streams (torch's NCCL stream, RCCL's own) beside its frame
# streams; with HIP's default of 4 hardware queues per process a frame stream would share a
# queue with them (DESIGN.md §5 "Queue budget").  Ranks take 8, set before HIP initialises
# (8 queues measured even at N = 1: profiles/r05z3_ab_hw_queues.txt, r05k_ab_depth_queues.txt).
if int(os.environ.get("WORLD_SIZE", "1")) > 1 and int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from gaussiansplattingviewer_amd import _lib  # noqa: E402
from gaussiansplattingviewer_amd.camera import cuda_camera_inputs, orbit_eye, static_camera  # noqa: E402
from gaussiansplattingviewer_amd.gaussian_data import clustered_scene, synthetic_gaussians  # noqa: E402
from gaussiansplattingviewer_amd.rasterizer import rasterize_gaussians_native, tile_row_pairs  # noqa: E402
from gaussiansplattingviewer_amd.pipeline import FramePipeline  # noqa: E402
from gaussiansplattingviewer_amd.strips import (StripBalancer, StripGather, rank_stream_plan,  # noqa: E402
                                                strip_pixel_rows, strip_rows)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, spec)

CONFIGS = {
    # name: (P, W, H, sh_degree, seed, camera[, scene generator])
    # BASELINE.json configs[0]: the reference's CPU path (numpy sort, renderer_ogl.py:10-19) and
    # the CPU restatement of the blend at 10k / 640x480, timed by cpu_baseline; the HIP forward
    # of the same frame beside it
    "c1": (10_000, 640, 480, 3, 0, "static"),
    "c2": (100_000, 1920, 1080, 0, 1, "static"),
    "c3": (1_000_000, 1920, 1080, 3, 2, "static"),
    "c4": (6_000_000, 3840, 2160, 3, 3, "static"),
    "c5": (1_000_000, 1920, 1080, 3, 2, "orbit"),
    # C3 with a capture-like scene (gaussian_data.clustered_scene): clustered centres, ground
    # plane, background shell, near floaters; depths over 8 float exponents
    "c3r": (1_000_000, 1920, 1080, 3, 7, "static", "clustered"),
}
METRIC = "frames/sec + Msplats/sec, 1M Gaussians @ 1920×1080, 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sim-strip", default=None, metavar="R/N",
                    help="diagnostic, 1 GPU: render only strip R of an N-way partition (no "
                         "gather) to estimate one rank's share of an N-GPU frame")
    ap.add_argument("--blend", default="fast", choices=["exact", "fast"],
                    help="blend arithmetic: GSR_OPT_BLEND_FAST (default) or upstream's exact "
                         "operation order")
    ap.add_argument("--inflight", type=int, default=None,
                    help="frames in flight (FramePipeline: own stream + context slot each); "
                         "1 = serial forwards (default: 4 frames, each on one stream -- strip "
                         "frames below 4M Gaussians with the deferred-K chains; 2 larger strip "
                         "frames, each with its second stream and frame graphs)")
    ap.add_argument("--depth-sort", default="auto", choices=["auto", "lsd", "compact", "msd", "compact-msd"],
                    help="GSR_OPT_DEPTH_SORT: LSD passes, LSD after compacting the kept keys, or "
                         "the MSD pass + per-bucket local sort (auto: compact on strips of >= 4M "
                         "Gaussians, else MSD when the last frame's kept depth keys spanned a "
                         "range of <= 25 bits, else LSD)")
    ap.add_argument("--graphs", type=int, default=None, choices=[0, 1, 2],
                    help="GSR_OPT_FRAME_GRAPHS for every context slot (default: the library's): "
                         "0 direct, 1 recorded graphs, 2 the deferred-K chains launched directly")
    ap.add_argument("--second-stream", type=int, default=None, choices=[0, 1],
                    help="GSR_OPT_SECOND_STREAM of the in-flight frames (default: FramePipeline's "
                         "choice -- off at depth >= 3 without frame graphs)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="CPU-oracle time to sample for cpu_baseline (whole frames; at least one)")
    return ap.parse_args()


class Scene:
    def __init__(self, cfg, dev):
        P, W, H, deg, seed, cam_kind = CONFIGS[cfg][:6]
        self.P, self.W, self.H, self.deg, self.cam_kind = P, W, H, deg, cam_kind
        self.generator = CONFIGS[cfg][6] if len(CONFIGS[cfg]) > 6 else "uniform"
        g = (clustered_scene(P, seed) if self.generator == "clustered"
             else synthetic_gaussians(P, deg, seed))
        self.host = g
        up = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        self.xyz, self.rot, self.scale, self.opacity = up(g.xyz), up(g.rot), up(g.scale), up(g.opacity)
        self.sh = up(g.sh).reshape(P, -1, 3).contiguous()
        self.bg = torch.zeros(3, device=dev)
        self.dev = dev
        self.cams = []
        n_cams = 1000 if cam_kind == "orbit" else 1
        for i in range(n_cams):
            eye = orbit_eye(i, 1000) if cam_kind == "orbit" else (0.0, 0.0, 4.0)
            cam = static_camera(W, H, eye)
            view, proj, campos, tx, ty = cuda_camera_inputs(cam)
            self.cams.append((up(view), up(proj), up(campos), tx, ty, (view, proj, campos)))
            if i == 0:  # the GL view (math layout) the OpenGL backend's sort receives
                self.gl_view0 = np.asarray(cam.get_view_matrix(), dtype=np.float32)

    def render(self, step, tile_rows=None, slot=0, out_color=None, radii=True):
        view, proj, campos, tx, ty, _ = self.cams[step % len(self.cams)]
        return rasterize_gaussians_native(self.bg, self.xyz, None, self.opacity, self.scale,
                                          self.rot, 1.0, None, view, proj, tx, ty, self.H, self.W,
                                          self.sh, self.deg, campos, False, False,
                                          tile_rows=tile_rows, slot=slot, out_color=out_color,
                                          radii=radii)


# Committed rocprofv3 profiles (tools/profile_config.sh on the GPU box, summarised here by
# tools/prof_summary.py and tools/sq_summary.py): per config, the serial kernel trace with HBM
# traffic per launch (FETCH_SIZE x2 + WRITE_SIZE, separate PMC passes) in
# profiles/<tag>_<config>_kernels.json, and the blend's SQ counters in
# profiles/<tag>_<config>_blend_sq.json.  Every profile records the sha256 of the libgsr.so it
# measured; the bench uses only a profile of the library it has loaded (instruction counts and
# traffic belong to one build), else reports null.
PROFILES = os.path.join(REPO, "profiles")
VALU_PEAK_T = 256 * 4 * 32 * 2.4e9 / 1e12  # lane-instructions/s: 256 CUs x 4 SIMD32 x 2.4 GHz
BLEND_KERNEL = "k_blend_q"


def lib_sha16() -> str:
    import hashlib
    return hashlib.sha256(open(_lib.LIB_PATH, "rb").read()).hexdigest()[:16]


def find_profile(config: str, suffix: str):
    """The newest committed profile of this config whose lib_sha16 is the loaded library's."""
    import glob
    sha = lib_sha16()
    best = None
    for path in glob.glob(os.path.join(PROFILES, f"*_{config}_{suffix}.json")):
        try:
            prof = json.load(open(path))
        except (OSError, ValueError):
            continue
        if prof.get("lib_sha16") == sha and (best is None or path > best[0]):
            best = (path, prof)
    return best


def measured_traffic(config: str, kernel: str):
    """HBM bytes per launch of `kernel` from the config's committed PMC profile (FETCH_SIZE
    doubled per the gfx950 calibration, MI355X_MICROARCH.md §HBM, + WRITE_SIZE), with the
    profile's own average launch time; None without a profile of this build."""
    hit = find_profile(config, "kernels")
    if not hit:
        return None
    path, prof = hit
    rec = next((v for name, v in prof["kernels"].items() if name.startswith(kernel)), None)
    if not rec or rec.get("read_bytes_x2") is None or rec.get("write_bytes") is None:
        return None
    return {"bytes": int(rec["read_bytes_x2"] + rec["write_bytes"]),
            "read_bytes_x2": int(rec["read_bytes_x2"]), "write_bytes": int(rec["write_bytes"]),
            "trace_avg_us": round(rec["avg_us"], 2), "source": os.path.relpath(path, REPO)}


def blend_sq(config: str):
    """Per-launch SQ counters of the blend from the config's committed profile, or None."""
    hit = find_profile(config, "blend_sq")
    if not hit:
        return None
    path, prof = hit
    return prof["per_launch"], os.path.relpath(path, REPO)


def blend_roofline(config, launch_ms, launch_ms_inflight, alg_bytes):
    """The blend on the roof that bounds it: VALU (its exponent / composite chain; no dense
    contraction, so no MFMA).  achieved = SQ_INSTS_VALU (wave64 instructions per launch, a
    committed SQ profile of this build and config) x 64 lanes / the live launch time; peak =
    256 CUs x 4 SIMD32 x 32 lanes x 2.4 GHz = 78.6 T lane-instructions/s (the 157.3 TFLOP/s FP32
    vector peak counts an FMA as 2 flops; SQ_INSTS_VALU reads a calibration kernel's known count
    exactly, profiles/r02_valu_calibration.md).  Beside it: the HBM roof from the counters
    (FETCH_SIZE x2 + WRITE_SIZE per launch over the live launch time) and, as a labelled
    diagnostic, SURVEY.md's algorithmic bytes 40 K + 12 W H over the launch time -- omitted when
    above 1, which shows the blend does not read every pair's record (a pixel stops once T <
    1e-4, a quadrant once its 64 pixels have).  frac uses the serial launch time (the kernel on
    an otherwise idle chip); frac_inflight the blend's event time with frames in flight (the
    timed frames' regime, where the next frame's kernels share the CUs)."""
    out = {"bound": "valu", "kernel": "blend", "achieved": None, "peak": round(VALU_PEAK_T, 2),
           "unit": "T lane-instr/s", "frac": None, "traffic": None,
           "launch_ms": round(launch_ms, 5),
           "launch_ms_source": "serial stage pass: HIP events around the kernel on the forward's "
                               "stream, one frame at a time (the committed serial rocprofv3 "
                               "trace agrees); achieved and frac use it",
           "launch_ms_inflight": round(launch_ms_inflight, 5),
           "launch_ms_inflight_source": "blend events of slot 0 in a separate untimed pass with "
                                        "frames in flight"}
    sq = blend_sq(config) if config else None
    if sq:
        c, src = sq
        ach = c["SQ_INSTS_VALU"] * 64 / (launch_ms * 1e-3) / 1e12
        cyc = c["GRBM_GUI_ACTIVE"] / 8  # summed over the 8 XCDs
        ach_if = c["SQ_INSTS_VALU"] * 64 / (launch_ms_inflight * 1e-3) / 1e12
        out.update(achieved=round(ach, 3), frac=round(ach / VALU_PEAK_T, 4),
                   achieved_inflight=round(ach_if, 3), frac_inflight=round(ach_if / VALU_PEAK_T, 4),
                   valu_wave_instr_per_launch=int(c["SQ_INSTS_VALU"]),
                   waves_per_launch=int(c["SQ_WAVES"]),
                   valu_busy=round(c["SQ_INSTS_VALU"] * 2 / 1024 / cyc, 4), sq_source=src)
    else:
        out["note"] = "no committed SQ profile of this build and config: VALU achieved unmeasured"
    tr = measured_traffic(config, BLEND_KERNEL) if config else None
    if tr:
        gbs = tr["bytes"] / (launch_ms * 1e-3) / 1e9
        out["traffic"] = tr["bytes"]
        out["hbm"] = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                      "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4), **tr}
    alg_frac = alg_bytes / (launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
    out["alg_bytes_diag"] = {"bytes_per_launch": int(alg_bytes),
                             "frac_of_hbm": round(alg_frac, 4) if alg_frac <= 1.0 else None,
                             "note": "SURVEY.md 8(d) 40 K + 12 W H: an upper bound on what the "
                                     "blend must read, not a measurement" +
                                     ("" if alg_frac <= 1.0 else
                                      "; above 1 here, so not a bound (omitted)")}
    return out


def algorithmic_bytes(P, P_f, P_v, K, T, W, H, sh_bytes):
    """algorithmic HBM bytes per stage of one frame (the SH read of the
    preprocess is the "color" stage, which runs on the second stream)."""
    return {
        "preprocess": 12 * P + 32 * P_f + 8 * P + 40 * P_v,
        "color": (12 + sh_bytes) * P_v,
        "depth_sort": 16 * P,   # one read + write of (key, id) per Gaussian
        "scan": 8 * P,
        "duplicate": 4 * P + 12 * K,
        "tile_sort": 24 * K,    # one read + write of 12-B pairs (upstream's pair size)
        "ranges": 8 * K + 8 * T,
        "blend": 40 * K + 12 * W * H,
    }


def design_bytes(P, P_f, P_v, K_L, T, W, H, sh_bytes):
    """This design's minimum HBM bytes per frame: what each of its kernels must
    read and write once, with the pair list it really bins (K_L 4-B list words after tight
    binning) -- beside SURVEY.md §8(d)'s upstream model, which charges 12-B pairs for upstream's
    K and a 24-B-per-pair sort that this design does not do."""
    return {
        # xyz; scale + rotation + opacity in the frustum; depth key, {rect, span} record, the
        # blend's 36-B record of a visible Gaussian
        "preprocess": 12 * P + 32 * P_f + 4 * P + 16 * P + 36 * P_v,
        # the rect flag, the SH row and the 12-B colour of a visible Gaussian
        "color": 8 * P + (sh_bytes + 12) * P_v,
        # keys in, (key, id) pairs out and back in, the permutation out
        "depth_sort": 4 * P + 20 * P_v,
        # the permutation and the gathered + written 16-B records
        "scan": 36 * P_v,
        # the permutation and the records in depth order, the list words out
        "duplicate": 20 * P_v + 4 * K_L,
        # the row pass: upsweep read, downsweep read + write
        "tile_sort": 12 * K_L,
        # the second stream's tile counts over the records, the ranges out
        "ranges": 16 * P + 8 * T,
        # a list word and a 48-B record per list entry, the image out
        "blend": 52 * K_L + 12 * W * H,
    }


def host_cpu():
    """CPU model (lscpu "Model name", else /proc/cpuinfo) and the BLAS / OpenMP thread env."""
    model = None
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        model = next((l.split(":", 1)[1].strip() for l in out.splitlines()
                      if l.startswith("Model name")), None)
    except Exception:
        pass
    if model is None and os.path.exists("/proc/cpuinfo"):
        model = next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo")
                      if l.startswith("model name")), None)
    env = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS",
                                          "MKL_NUM_THREADS")}
    return model or platform.processor() or platform.machine(), env


def cpu_baseline(scene, seconds):
    """CPU legs on rank 0's host cores (the checker's code, timed here only as baselines):

    1. the reference's own CPU path -- the OpenGL backend's per-frame depth sort
       `_sort_gaussian_cpu` (renderer_ogl.py:10-19), as restated in `oracle.sort_gaussian_cpu`
       (bit-exact to outputs captured from the reference, tests/golden/sort_backend.npz), on the
       scene's P Gaussians and GL view: one warm-up, then the median of 5 calls;
    2. the full forward on the host cores -- oracle/gsr_oracle.c, the C restatement of the
       upstream rasterizer the viewer's CUDA backend calls, its loops parallel over OpenMP
       threads (OMP_NUM_THREADS: the box's CPU share): whole frames of the same scene and
       camera for `seconds` (at least one frame).  `value` is this leg's frame rate, `cores`
       its thread count;
    3. beside it, one frame of the same forward on one thread (scenes up to 2M Gaussians)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    g = scene.host
    ts = []
    for _ in range(6):
        t0 = time.perf_counter()
        oracle.sort_gaussian_cpu(g.xyz, scene.gl_view0)
        ts.append(time.perf_counter() - t0)
    sort_ms = 1e3 * float(np.median(ts[1:]))
    view, proj, campos = scene.cams[0][5]
    tx, ty = scene.cams[0][3], scene.cams[0][4]

    def frame():
        oracle.forward(g.xyz, g.opacity, view, proj, campos, tx, ty, scene.W, scene.H, shs=g.sh,
                       sh_degree=scene.deg, scales=g.scale, rotations=g.rot)

    threads = oracle.set_threads(0)
    frames, t0 = 0, time.perf_counter()
    while True:
        frame()
        frames += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    single = None
    if scene.P <= 2_000_000:
        oracle.set_threads(1)
        t1 = time.perf_counter()
        frame()
        single = round(1.0 / (time.perf_counter() - t1), 5)
        oracle.set_threads(0)
    model, env = host_cpu()
    return {"value": round(frames / el, 5), "unit": "frames/sec", "cores": threads, "kind": "port",
            "sample": f"{frames} full frame(s) of the {scene.P}-Gaussian {scene.W}x{scene.H} "
                      f"SH{scene.deg} scene through oracle/gsr_oracle.c on {threads} OpenMP "
                      f"threads ({el:.1f} s)",
            "single_thread_frames_per_sec": single,
            "reference_sort": {
                "fn": "renderer_ogl._sort_gaussian_cpu (renderer_ogl.py:10-19) via "
                      "oracle.sort_gaussian_cpu, pinned to reference-captured outputs",
                "ms_median_of_5": round(sort_ms, 3), "calls_per_sec": round(1e3 / sort_ms, 3),
                "P": scene.P, "threads": "numpy argsort is single-threaded; the stacked matmul "
                                         "follows the BLAS / OpenMP env below"},
            "host": {"cpu_model": model, "os_cpu_count": os.cpu_count(),
                     "affinity_cpus": len(os.sched_getaffinity(0)), "thread_env": env}}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        if world == 1:
            raise SystemExit("--gpus > 1 must be launched with torch.distributed.run")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", local))

    scene = Scene(args.config, dev)
    # Frames in flight.  Full frames: four, each on one stream (DESIGN.md decision 13).  Strip
    # frames (a rank of an N-GPU frame, or the simulated strip) of scenes below the compacting
    # sort's 4M Gaussians (the headline's 1M): four one-stream frames too, with the deferred-K
    # chains (GSR_OPT_FRAME_GRAPHS 2: the host does not wait for K in mid-frame) -- C3 strips
    # 10,300-10,450 -> 12,100-12,350 frames/s; larger strips (C4's 6M): two frames with their
    # second streams replaying frame graphs (decision 12), 4 % faster there than four one-stream
    # frames (profiles/r06g_ab_strip_depth.txt)
    strip = world > 1 or bool(args.sim_strip)
    small_strip = strip and scene.P < (4 << 20)
    if args.inflight is None:
        args.inflight = 2 if (strip and not small_strip) else 4
    W, H = scene.W, scene.H
    gy, gx = (H + 15) // 16, (W + 15) // 16
    rows = None
    if args.sim_strip:
        if world > 1:
            raise SystemExit("--sim-strip is a single-process diagnostic")
        sr, sn = (int(x) for x in args.sim_strip.split("/"))
        rows = strip_rows(gy, sn, sr)

    # N > 1: each rank renders its strip of tile rows; rank 0 receives every strip straight
    # into its frame (RCCL send/recv).  The gather of frame i runs asynchronously while frame
    # i+1 renders; the last frame's gather completes inside the timed region.  The strip
    # boundaries follow the blend work: every 8 frames the ranks all-reduce their tile rows'
    # pair counts and re-split (StripBalancer), identically on every rank.
    gather = (StripGather(H, W, world, rank, device=dev, depth=args.inflight + 1)
              if world > 1 else None)
    balancer = StripBalancer(gy, gx, world, rank, device=dev) if world > 1 else None
    # frames in flight: frame i renders on stream i % D with context slot i % D, so the next
    # frame's latency-bound preprocess / sort / binning overlap this frame's blend.  Large strip
    # frames in pairs replay frame graphs (mode 1: with two in flight a strip rank's rate is then
    # steady instead of bimodal run to run, DESIGN.md decision 12); small strip frames launch the
    # deferred-K chains directly on one stream each (mode 2); full frames keep direct launches
    strip_graphs = args.inflight >= 2 and strip and not small_strip
    pipe = None  # (created below: after the serial passes on one GPU)
    if world > 1:
        # RCCL's communicators (and their streams) first: one all-reduce and one gather of an
        # empty frame, so RCCL's streams exist before the frame streams are created and used
        # (a stream's hardware queue is fixed when it is first used)
        warm = torch.zeros((gy,), dtype=torch.int32, device=dev)
        dist.all_reduce(warm)
        gather.submit(gather.next_buffer(strip_pixel_rows(balancer.current[rank], H)[1]),
                      balancer.current)
        gather.finish()
        torch.cuda.synchronize()

    def step(i):
        with pipe.frame() as slot:
            if gather is not None:
                if len(gather.pending) == len(gather.slots) - 1:
                    gather.finish()
                layout = balancer.layout(i)
                mine = layout[rank]
                buf = gather.next_buffer(strip_pixel_rows(mine, H)[1])
                if mine[1] > mine[0]:
                    # a strip rank returns its image only: no radii, so Gaussians that miss the
                    # strip skip the per-Gaussian work (gsr.h gsr_outputs.radii)
                    res = scene.render(i, mine, slot, out_color=buf, radii=False)
                    K = res.num_rendered
                    row_pairs = tile_row_pairs(mine[1] - mine[0], local, slot)
                else:  # more GPUs than tile rows: nothing to render
                    K, row_pairs = 0, torch.zeros((0,), dtype=torch.int32, device=dev)
                gather.submit(buf, layout)
                balancer.observe(i, row_pairs)
                return K
            return scene.render(i, rows, slot, radii=rows is None).num_rendered

    def drain():
        while gather is not None and gather.pending:
            gather.finish()

    lib = _lib.load_library()
    ctxs = [_lib.context(local, slot) for slot in range(args.inflight)]
    ctx = ctxs[0]  # stage timing is read from slot 0 (every D-th frame)
    for c in ctxs:
        opt = lambda o, v: _lib.check(lib.gsr_set_option(c, o, v), "gsr_set_option")  # noqa: E731
        opt(_lib.GSR_OPT_BLEND_FAST, {"exact": 0, "fast": 1}[args.blend])
        opt(_lib.GSR_OPT_DEPTH_SORT,
            {"auto": -1, "lsd": 0, "compact": 1, "msd": 2, "compact-msd": 3}[args.depth_sort])
    # frame graphs: the pipeline's choice (strip frames in flight) unless --graphs; the serial
    # passes render as a caller without the pipeline does (direct launches).  Full frames of
    # small scenes are host-bound (~17 launches per frame): recorded graphs there (C1 +16-28 %,
    # C2 +3-4 %, profiles/r06zb_ab_small_frame_graphs.txt); from 512k Gaussians direct launches
    # (a graph adds ~20 us to a frame's latency, which the 20-frame window pays: C3 -2.6 %,
    # r06h_ab_graphs_one_stream.txt)
    small_frame_graphs = not strip and args.inflight >= 2 and scene.P < (512 << 10)
    graphs_inflight = (args.graphs if args.graphs is not None else
                       1 if (strip_graphs or small_frame_graphs) else 2 if small_strip else 0)
    graphs_serial = args.graphs if args.graphs is not None else 0
    names = _lib.stage_names()
    buf = (ctypes.c_float * len(names))()

    def serial_passes(rows):
        """(2) Serial frame rate: one frame in flight (slot 0, the caller's stream, no gather,
        the second stream on: a lone frame overlaps its own two halves) -- the frame time of a
        viewer that renders each frame before starting the next; (3) the per-stage breakdown
        (events at every stage boundary) of 30 more such forwards."""
        _lib.check(lib.gsr_set_option(ctx, _lib.GSR_OPT_FRAME_GRAPHS, graphs_serial),
                   "gsr_set_option")
        _lib.check(lib.gsr_set_option(ctx, _lib.GSR_OPT_SECOND_STREAM, 1), "gsr_set_option")
        torch.cuda.synchronize()
        n_serial = 100
        t1 = time.perf_counter()
        for i in range(n_serial):
            scene.render(i, rows, radii=rows is None)
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t1) / n_serial
        _lib.check(lib.gsr_set_timing(ctx, 1), "gsr_set_timing")
        torch.cuda.synchronize()
        for i in range(30):
            scene.render(i, rows, radii=rows is None)
        torch.cuda.synchronize()
        _lib.check(lib.gsr_stage_times(ctx, buf, len(names)), "gsr_stage_times")
        _lib.check(lib.gsr_set_timing(ctx, 0), "gsr_set_timing")
        return ms, {n: float(buf[i]) for i, n in enumerate(names)}

    # The untimed diagnostic passes run first, so the device has been rendering for ~200 frames
    # when the timed region starts: a run of 20 timed frames after 5 warmup frames measured
    # 3,160-3,250 frames/s against 3,670-3,720 after 100+ frames of rendering (the same binary;
    # the GPU settles over the first ~30 ms of load), and the metric is the steady frame rate of
    # a viewer that keeps rendering.  Their sizes are fixed (not tied to --steps) for that reason.
    # One GPU: the serial passes come first (after 64 untimed serial frames), before the
    # pipeline's streams exist -- a stream's hardware queue is fixed when it is created, and a
    # second stream created after four one-stream frame streams shared a queue with the caller's
    # stream (serial 0.31 -> 0.6 ms, tools/lab/stream_probe.py).  Strip ranks (N > 1) time them
    # after pass (1), on the split those frames ended with.
    if world == 1:
        for i in range(64):
            scene.render(i, rows, radii=rows is None)
        serial_ms, stage_ms = serial_passes(rows)
    pipe = FramePipeline(args.inflight, dev, graphs=strip_graphs,
                         second_stream=None if args.second_stream is None
                         else bool(args.second_stream))
    for c in ctxs:
        _lib.check(lib.gsr_set_option(c, _lib.GSR_OPT_FRAME_GRAPHS, graphs_inflight),
                   "gsr_set_option")

    # (1) The blend's event time with frames in flight (events around the blend on every 8th
    # forward of slot 0; these frames run on the stream path).
    n_pre = 0
    _lib.check(lib.gsr_set_timing(ctx, 2), "gsr_set_timing")
    for i in range(64):
        step(n_pre + i)
    n_pre += 64
    drain()
    torch.cuda.synchronize()
    _lib.check(lib.gsr_stage_times(ctx, buf, len(names)), "gsr_stage_times")
    _lib.check(lib.gsr_set_timing(ctx, 0), "gsr_set_timing")
    blend_ms_timed = float(buf[names.index("blend")])
    if world > 1:
        if balancer is not None:  # the split these frames ended with (for the serial passes)
            rows = balancer.current[rank]
            if rows[1] <= rows[0]:
                rows = None
        serial_ms, stage_ms = serial_passes(rows)
        _lib.check(lib.gsr_set_option(ctx, _lib.GSR_OPT_FRAME_GRAPHS, graphs_inflight),
                   "gsr_set_option")
        _lib.check(lib.gsr_set_option(ctx, _lib.GSR_OPT_SECOND_STREAM, int(pipe.second_stream)),
                   "gsr_set_option")

    # Warmup: W frames of the timed loop's own kind (in flight, gathered).
    for i in range(args.warmup):
        step(n_pre + i)
    drain()
    torch.cuda.synchronize()

    # Timed region: exactly K frames, no events.
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    K_total = 0
    for i in range(args.steps):
        K_total += step(n_pre + args.warmup + i)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if balancer is not None:  # the split the timed frames ended with (frame statistics below)
        rows = balancer.current[rank]
        if rows[1] <= rows[0]:
            rows = None

    t_max = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    t_max = float(t_max.item())

    # Frame statistics for the algorithmic byte counts (frame 0 of the camera path, full frame).
    res = scene.render(0, rows)
    # the list entries that frame binned (tight binning: fewer than upstream's num_rendered)
    K_list, T_all = ctypes.c_int64(), ctypes.c_int32()
    _lib.check(_lib.load_library().gsr_get_binning(
        _lib.context(local, 0), None, None, None, ctypes.byref(K_list), ctypes.byref(T_all),
        ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "gsr_get_binning")
    P = scene.P
    P_v = int((res.radii > 0).sum().item())
    view = scene.cams[0][0]
    from gaussiansplattingviewer_amd.rasterizer import GaussianRasterizer, GaussianRasterizationSettings
    P_f = int(GaussianRasterizer(GaussianRasterizationSettings(
        H, W, 1.0, 1.0, scene.bg, 1.0, view, scene.cams[0][1], scene.deg, scene.cams[0][2],
        False, False)).markVisible(scene.xyz).sum().item())
    K_mean = K_total / args.steps
    T_strip = ((rows[1] - rows[0]) if rows else gy) * ((W + 15) // 16)
    rows_px = (min(H, rows[1] * 16) - rows[0] * 16) if rows else H
    sh_bytes = 4 * 3 * (scene.deg + 1) ** 2
    alg = algorithmic_bytes(P, P_f, P_v, K_mean, T_strip, W, rows_px, sh_bytes)
    # The roofline kernel is the blend: the largest share of GPU time in the rocprofv3 trace and
    # the last kernel on the frame's critical path.  Its launch duration: the serial stage pass
    # (one frame at a time, events on the forward's stream bracket the kernel alone), which is
    # what the committed serial rocprofv3 trace reports for it; the timed region's blend events
    # (two frames in flight, the other frame's kernels sharing the CUs) are reported beside it.
    dom_ms = stage_ms["blend"]
    default_opts = args.blend == "fast"  # the committed profiles are of the default arithmetic
    # profiles are keyed by config (and the simulated strip: <tag>_<config>-strip<R><N>_*.json)
    prof_key = args.config + (f"-strip{args.sim_strip.replace('/', '')}" if args.sim_strip else "")
    if world > 1:
        prof_key = None  # no profile of a rank's strip of a multi-GPU frame
    roofline = blend_roofline(prof_key if default_opts else None, dom_ms, blend_ms_timed,
                              alg["blend"])
    roofline["frame_alg_gbs"] = round(sum(alg.values()) / (t_max / args.steps) / 1e9, 2)
    # the design's own minimum bytes (frame 0's list length) over the same frame time
    dsg = design_bytes(P, P_f, P_v, int(K_list.value), T_strip, W, rows_px, sh_bytes)
    dsg_gbs = sum(dsg.values()) / (t_max / args.steps) / 1e9
    roofline["frame_design"] = {
        "bytes_per_frame": int(sum(dsg.values())), "gbs": round(dsg_gbs, 2),
        "frac_of_hbm": round(dsg_gbs / HBM_PEAK_GBS, 4),
        "per_stage_bytes": {k: int(v) for k, v in dsg.items()},
        "note": "this design's minimum HBM bytes per frame (bench.design_bytes: the 4-B list "
                "words it bins, one read + write of the depth sort's 8-B pairs, the 48-B blend "
                "records per list entry) over the timed frame time; frame_alg_gbs above is "
                "SURVEY.md 8(d)'s upstream model (12-B pairs, upstream's K), which can exceed "
                "the peak on this design"}
    fps = args.steps / t_max
    line = {
        "metric": METRIC,
        "value": round(fps, 3),
        "unit": "frames/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * t_max / args.steps, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": ("synthetic (%s, seed %d; no PLY offline)" %
                 ("SURVEY.md §8(d) generator" if scene.generator == "uniform" else
                  "gaussian_data.clustered_scene", CONFIGS[args.config][4])),
        "config": {"workload": f"{args.config}: {P} Gaussians ({scene.generator} scene), {W}x{H}, "
                               f"SH degree {scene.deg}, {scene.cam_kind} camera",
                   "gaussians": P, "width": W, "height": H, "sh_degree": scene.deg,
                   "parallelism": (f"SIMULATED strip {args.sim_strip} (diagnostic, no gather)"
                                   if args.sim_strip else
                                   f"image strips x{world}" + (" + RCCL gather" if world > 1 else "")),
                   "blend_arithmetic": args.blend},
        "msplats_per_sec": round(P * fps / 1e6, 2),
        "frame_stats": {"P_frustum": P_f, "P_visible": P_v, "K_pairs_mean": round(K_mean, 1),
                        "K_list_frame0": int(K_list.value), "tiles": T_strip,
                        "note": "K_pairs_mean is upstream's num_rendered (the SURVEY.md §8(d) "
                                "bytes use it: an upper bound); K_list_frame0 the (Gaussian, "
                                "tile) entries frame 0 binned and blended (tight binning on "
                                "full frames keeps only tiles the alpha >= 1/255 ellipse "
                                "reaches); msplats_per_sec counts Gaussians, not pairs"},
        "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
        "stage_ms_note": "HIP events at every stage boundary, separate 30-frame serial pass "
                         "(each event adds a few us); the timed region records no events",
        "inflight": args.inflight,
        "second_stream": pipe.second_stream,
        "streams": {"plan": rank_stream_plan(args.inflight, pipe.second_stream),
                    "priority": "normal (all)",
                    "order": ("the caller's stream and slot 0's second stream in the serial "
                              "passes (that second stream destroyed before the pipeline at "
                              "depth >= 3), then FramePipeline's streams in slot order, first "
                              "used by the in-flight pass" if world == 1 else
                              "RCCL's communicators (warm-up all-reduce + gather), then the "
                              "FramePipeline streams in slot order"),
                    "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                    "note": ("HIP fixes a stream's hardware queue when the stream is first used; "
                             "the plan stays within the process's hw_queues" if world == 1 else
                             "HIP fixes a stream's hardware queue when the stream is first used; "
                             "a rank takes 8 queues so that RCCL's streams do not share the "
                             "frame streams' queues")},
        "timed_after": ("194 serial (64 untimed, 100 for the serial rate, 30 with stage events) "
                        "then 64 in-flight (blend events) untimed diagnostic frames, then the W "
                        "warmup frames" if world == 1 else
                        "64 in-flight (blend events) + 130 serial (rate, stage events) untimed "
                        "diagnostic frames, then the W warmup frames"),
        "strip_layout": (None if balancer is None else
                         {"tile_rows": [list(t) for t in balancer.current],
                          "rebalances": len(balancer.history),
                          "note": "cost-weighted strips (StripBalancer): every 8 frames the "
                                  "ranks all-reduce their tile rows' pair counts and re-split"}),
        "frame_graphs": {"timed_frames": graphs_inflight, "serial_pass": graphs_serial,
                         **{f"slot{c}": _lib.frame_graph_stats(local, c)
                            for c in range(args.inflight)},
                         "note": "GSR_OPT_FRAME_GRAPHS of the in-flight frames (0 direct "
                                 "launches: full frames from 512k Gaussians; 1 recorded graphs: "
                                 "full frames of smaller scenes, and strip frames from 4M "
                                 "Gaussians, two in flight; 2 deferred-K chains on one stream: "
                                 "strip frames below 4M Gaussians) and of the serial pass "
                                 "(direct launches, as a caller without the pipeline)"},
        "serial_ms_per_frame": round(serial_ms, 4),
        "serial_note": "one frame in flight at a time (no FramePipeline overlap), this rank",
        "roofline": roofline,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(scene, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
