#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X LBVH build + ray-traversal path.

Metric (BASELINE.json): Mrays/s, primary + 1 reflection bounce; BVH build Mtris/s;
at 1/2/4/8 GPUs.  Default workload = BASELINE config C5: 10M
synthetic triangles (splitmix64 seed 0x5EED0005, box x,y +-100, z +-50), a
3840x2160 frame, primary rays + 1 bounce.  Multi-GPU: every rank holds the same
scene and builds the same BVH (replicas, deterministic); the frame is split in
8-row bands dealt round-robin to the ranks, and the bands are gathered to rank 0
over RCCL (torch.distributed "nccl") and assembled into the frame.

One step = trace of this rank's bands (primary kernel + bounce kernels) + the
RCCL gather + assembly on rank 0.  Four frames are in flight per rank (--inflight 4):
frame i is traced on stream i % 4 (the context gives each caller stream a trace-buffer
set of its own over the one BVH: rtbvh_trace_band_async), so frame i+1's primary pass
fills the GPU while frame i's bounce walk drains its last long walks; two band buffers keep one gather in flight
(step i's gather overlaps step i+1's trace), and every step's frame is traced,
gathered and assembled before the timed region closes.  The one-frame latency (one
context, frames back to back on one stream) is reported beside it.  The BVH is built once before the timed
loop (the scene is static; replicated build throughput is measured separately and
reported under "build"); the reference's own per-frame semantics -- Graphics.cpp:56 rebuilds
the BVH and traces every frame, behind a fence -- is measured beside it at N = 1
("c5_frame_rebuild", its ms and Mrays/s also at the line's top level), and so is the reference's only
interaction, the eye orbiting by Graphics::onKeyDown every frame ("c5_orbit": rebuild + trace of a new
camera per frame under RTBVH_FLAG_AUTO_WALK | RTBVH_FLAG_GRAPH, frames checked against the reference
order; beside it the same cameras' frames with the eye standing still, and the C5 camera under the
same flags).  value = all rays of the frame (W*H primary + every live bounce ray, summed over ranks) /
max-over-ranks time per step.  The reported traversal is the drop-in's own mode: the certified walks of
RTBVH_FLAG_AUTO_WALK (RTBVH_FLAG_CERTIFIED; DESIGN.md 3: the reference-order frame by construction,
per-ray certificates), its frame checked against the reference order's in this run; the unchecked
walks (exact only when their frame matches, which is checked per run) are reported beside it
(traversal.fastest_identical_*).  Each mode is timed in three interleaved rounds, the median kept.

Parity at the headline size (N = 1, rank 0, inside the cpu_baseline leg): the oracle builds
its own tree of the same 10M triangles (compared with the GPU tree field by field) and traces
the whole 3840x2160 frame on it (OpenMP over rows), which is compared with the GPU frame of
the reported mode pixel for pixel ("parity").

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c5|c3]
       (N > 1 under `torch.distributed.run --nproc-per-node N`).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_HBM_GBS = 8000.0            # MI355X HBM3E spec (MI355X_MICROARCH.md)
# algorithmic bytes per unit of THIS layout (the bytes each walk step requests):
L_REC = 64                       # one 64-B record per step: a QNode / child-pair record / leaf record
L_BOUNCE_RAY = 32 + 8            # bounce walk per ray: the 32-B queue entry read + the 8-B hit record write
L_PRIMARY_PIXEL = 16 + 4         # primary per pixel: colour (16 B) + intensity (4 B) written
L_QUEUE = 32                     # primary per live bounce ray: the queue entry written
# SURVEY.md §8(d) figures (the reference's data per unit of work; the frame_roofline below)
S_INT = 56                       # internal visit: children ids 8 B + two child AABBs 48 B
S_LEAF = 120                     # leaf visit: ids 8 + index 4 + 3 indices 12 + 3 Vertex 96
S_PRIMARY = 56                   # reflectRay record write per primary ray
S_BOUNCE = 112                   # reflectRay record read + write per bounce ray
S_HIT = 72                       # matIndex + Material per hit
S_TEX = 16                       # texel per textured hit
S_BUILD_PER_TRI = 348            # B_build: Morton 80 + sort 160 + Karras 24 + refit 84
# dependent random 64-B record fetches per second on MI355X (scripts/gather_roofline.hip,
# profiles/r01_gather_roofline.jsonl): from HBM / the Infinity Cache (1.25 GiB and 128 MiB
# tables, 2-8 waves/SIMD: 55-56 G/s) and from L2 (2 MiB table: 150 G/s)
GATHER_HBM_RPS = 5.6e10
GATHER_L2_RPS = 1.496e11
WORKLOADS = {
    "c5": dict(name="C5: synthetic 10M tris (seed 0x5EED0005, box 100x100x50), 3840x2160, primary+1 bounce",
               ntris=10_000_000, seed=0x5EED0005, half=(100.0, 100.0, 50.0), W=3840, H=2160, bounces=1),
    "c3": dict(name="C3: Obj/Test.obj (1952 tris), 1920x1080, primary+1 bounce", obj="Test", W=1920, H=1080,
               bounces=1),
    "c2": dict(name="C2: Obj/Image_Test.obj (3072 tris), 1920x1080, primary rays only", obj="Image_Test", W=1920,
               H=1080, bounces=0),
}


def log(msg):
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def make_scene(rt, wl):
    if "obj" in wl:
        return rt.load_npz(os.path.join(REPO, "tests", "golden", "scenes", wl["obj"] + ".npz"))
    return rt.synthetic(wl["ntris"], seed=wl["seed"], half_extent=wl["half"])


def binned_bytes(st, ntris):
    """Algorithmic bytes of the binned primary pass (RTBVH_FLAG_BINNED_PRIMARY): the
    leaf records' 64-B lines once (footprints), the 16-B footprints written and read back, the 16-B
    bin entries written and streamed, the 48-B triangle of every entry past the block test, the 8-B
    per-pixel keys written and read, then the pixel outputs and the bounce queue."""
    entries, survivors = st["bin_entries"]
    return (L_REC * ntris + 2 * 16 * ntris + 2 * 16 * entries + 48 * survivors + 2 * 8 * st["primary_rays"]
            + L_PRIMARY_PIXEL * st["primary_rays"] + L_QUEUE * st["bounce_rays"])


def layout_bytes(st, kernel, wide_primary=False):
    """Algorithmic bytes of one launch in this layout: the records its walk requests (one 64-B
    record per lane step in the per-lane bounce walk; one 64-B record -- two for a 4-wide
    step -- per WAVE step in the packet primary walk, which fetches a record once for its 64
    rays) plus its per-ray inputs and outputs.  Counted with RTBVH_FLAG_COUNT_VISITS."""
    if kernel == "k_primary":
        steps_int, steps_leaf = st["packet_steps"]
        return ((2 if wide_primary else 1) * L_REC * steps_int + L_REC * steps_leaf
                + L_PRIMARY_PIXEL * st["primary_rays"] + L_QUEUE * st["bounce_rays"])
    if kernel == "k_bounce_trav":
        return L_REC * (st["internal_visits"][1] + st["leaf_visits"][1]) + L_BOUNCE_RAY * st["bounce_rays"]
    # k_bounce_shade: queue entry + hit record in, colour read + written, the hit's shading data
    return (32 + 8 + 32) * st["bounce_rays"] + S_HIT * st["hits"][1]


def frame_bytes(st):
    """SURVEY §8(d) frame bytes from REFERENCE-ORDER visit counts."""
    return (S_INT * sum(st["internal_visits"]) + S_LEAF * sum(st["leaf_visits"]) + S_PRIMARY * st["primary_rays"]
            + S_BOUNCE * st["bounce_rays"] + S_HIT * sum(st["hits"]) + S_TEX * st["textured_hits"])


def load_pmc(workload, mode, kernel):
    """The PMC record of `kernel` (per-launch HBM bytes, raw counters and the launch's record
    fetches) from the rocprofv3 passes of the same traversal mode at N = 1
    (profiles/pmc_<workload>_<mode>.json, scripts/make_pmc_json.py), or None."""
    path = os.path.join(REPO, "profiles", f"pmc_{workload}_{mode}.json")
    if not os.path.exists(path):
        return None
    try:
        return json.load(open(path))["kernels"][kernel]
    except Exception:
        return None


def load_pmc_meta(workload, mode):
    """The PMC profile's header (its commit, source directory), or None."""
    path = os.path.join(REPO, "profiles", f"pmc_{workload}_{mode}.json")
    try:
        d = json.load(open(path))
        return {"commit": d.get("commit"), "source": d.get("source")}
    except Exception:
        return None


def build_pmc(workload, mode):
    """Summed per-launch HBM bytes of the build kernels in the same PMC profile, or None."""
    path = os.path.join(REPO, "profiles", f"pmc_{workload}_{mode}.json")
    if not os.path.exists(path):
        return None
    try:
        ks = json.load(open(path))["kernels"]
    except Exception:
        return None
    names = [k for k in ks if k in BUILD_KERNELS]
    if not names:
        return None
    per = {k: ks[k]["hbm_bytes_per_launch"] * BUILD_KERNELS[k] for k in names}
    return {"hbm_bytes": sum(per.values()), "per_kernel_gb": {k: round(v / 1e9, 3) for k, v in per.items()}}


# the build's kernels and their launches per build (the 30-bit sort: 4 passes of 8-bit digits);
# the mesh box (k_bounds) is computed once per scene by rtbvh_set_scene
# (the crossing nodes: k_refit_group + k_qnodes_late since round 6; k_refit_top + k_qnodes_cross in older profiles)
BUILD_KERNELS = {"k_morton": 1, "k_upsweep": 4, "k_scan_rows": 4, "k_downsweep": 4, "k_karras": 1, "k_refit": 1, "k_zrange": 1,
                 "k_refit_group": 1, "k_qnodes_late": 1, "k_refit_top": 1, "k_qnodes_cross": 1}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


NODE_FIELDS = ("parent", "child_l", "child_r", "code", "index", "bb_min", "bb_max")


def affinity_cpus():
    """The CPUs this process may run on (len(os.sched_getaffinity(0))): on the GPU boxes the process's share
    of the host, next to OMP_NUM_THREADS (16 there, set by the box) -- the thread count is the box's cap."""
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return None


def cpu_baseline(rt, scene, ctx, wl, W, H, gpu_frame):
    """The oracle (C++ restatement of the reference path, oracle/) on the GPU box's host cores:
    its own BVH of the bench scene (the parity check of the tree), a single-thread trace
    sample (the timed baseline), the whole frame on all cores (the timed all-cores baseline
    and the pixel parity check of the headline frame), and the reference-faithful 32-pass
    split-sort build on a 1M-triangle sample."""
    from oracle import lib as orc
    wvp, wv = rt.camera_reference(W, H)
    gnodes = ctx.read_bvh()
    osc = orc.Scene(scene.vertices, scene.indices, scene.mat_indices, scene.material_blob)
    parity = {"tolerance_rgb": 1e-4}
    # the all-cores build (SURVEY 8(d) CPU baseline (2)): the reference-faithful path -- Morton,
    # the 32 x 1-bit split sort with 256-wide Blelloch blocks, Karras, refit -- with OpenMP over
    # triangles / groups / nodes / leaves on this process's CPU share (OMP_NUM_THREADS, 16 on the
    # GPU boxes), over the WHOLE bench scene; its tree is the parity tree
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or (os.cpu_count() or 1)
    n_s = 1_000_000
    sub = rt.Scene(scene.vertices[: 3 * n_s], scene.indices[: 3 * n_s], scene.mat_indices[:n_s], scene.materials)
    if "obj" in wl:
        sub = scene
    osub = orc.Scene(sub.vertices, sub.indices, sub.mat_indices, sub.material_blob)
    orc.set_threads(threads)
    try:
        orc.build(osub, wvp, sort_mode=0)   # warm-up (thread pool, page faults), untimed
        t0 = time.perf_counter()
        onodes = orc.build(osc, wvp, sort_mode=0)
        dtb = time.perf_counter() - t0
    finally:
        orc.set_threads(1)
    build_all = {"value": scene.num_tris / dtb / 1e6, "unit": "Mtris/s", "cores": threads,
                 "sample": f"orc_build (Morton + 32 split passes + Karras + refit, OpenMP on {threads} threads) on "
                           f"all {scene.num_tris} triangles of the bench scene, {dtb:.2f} s"}
    parity["tree_nodes"] = int(len(onodes))
    parity["tree_bit_identical"] = bool(all(np.array_equal(gnodes[f], onodes[f]) for f in NODE_FIELDS))
    parity["tree_oracle_s"] = round(dtb, 2)
    del gnodes
    step = 8 if W * H > 4_000_000 else 4
    t0 = time.perf_counter()
    fb1, _, st = orc.trace(osc, onodes, wvp, wv, W, H, wl["bounces"], 0, H, step)
    dt = time.perf_counter() - t0
    rays = st["primary"] + st["bounce"]
    res = {"value": rays / dt / 1e6, "unit": "Mrays/s", "cores": 1, "kind": "port",
           "sample": f"oracle/liboracle.so orc_trace of 1 row in {step} of the same frame, on the oracle's own BVH "
                     f"of the same scene ({st['primary']} primary + {st['bounce']} bounce rays, {dt:.1f} s, 1 thread)",
           "cpu_model": cpu_model(), "host_cpus": os.cpu_count(), "affinity_cpus": affinity_cpus()}
    # BASELINE.md's all-cores variant: the same code, OpenMP over rows, on this process's CPU
    # share, over the WHOLE frame (the parity check)
    orc.set_threads(threads)
    try:
        t0 = time.perf_counter()
        fb, _, st2 = orc.trace(osc, onodes, wvp, wv, W, H, wl["bounces"], 0, H, 1)
        dt2 = time.perf_counter() - t0
    finally:
        orc.set_threads(1)
    res["openmp"] = {"value": (st2["primary"] + st2["bounce"]) / dt2 / 1e6, "unit": "Mrays/s", "cores": threads,
                     "affinity_cpus": affinity_cpus(), "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
                     "sample": f"every row, {st2['primary']} primary + {st2['bounce']} bounce rays, "
                               f"{dt2:.1f} s, OpenMP over rows on {threads} threads (OMP_NUM_THREADS: the "
                               f"process's CPU share, not all {os.cpu_count()} host CPUs)"}
    del onodes
    if gpu_frame is not None:
        diff = np.abs(fb - gpu_frame)
        parity.update({"rows_checked": int(H), "pixels_checked": int(W * H),
                       "frame_bit_identical": bool(np.array_equal(fb, gpu_frame)),
                       "sample_rows_bit_identical": bool(np.array_equal(fb1, gpu_frame[0:H:step])),
                       "pixels_differing": int(np.count_nonzero((fb != gpu_frame).any(axis=2))),
                       "max_abs_diff": float(np.nanmax(diff)) if diff.size else 0.0,
                       "within_tolerance": bool(np.allclose(fb, gpu_frame, atol=1e-4, rtol=0)),
                       "oracle_rays": int(st2["primary"] + st2["bounce"])})
    # build baseline: reference-faithful 32 x 1-bit split sort + Karras + refit on a 1M-triangle sample
    t0 = time.perf_counter()
    orc.build(osub, wvp, sort_mode=0)
    dt = time.perf_counter() - t0
    res["build_mtris_s"] = sub.num_tris / dt / 1e6
    res["build_sample"] = f"orc_build (32 split passes + Karras + refit) on {sub.num_tris} triangles, {dt:.2f} s, 1 thread"
    res["build_openmp"] = build_all
    return res, parity


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c5", choices=["c5", "c3"])
    ap.add_argument("--build-iters", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the C4 build / C3 side measurements")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (the bench); gloo only to rehearse N ranks on one GPU")
    ap.add_argument("--inflight", type=int, default=4, choices=[1, 2, 3, 4],
                    help="frames in flight per rank (one context + stream each)")
    ap.add_argument("--timing-in-flight", action="store_true",
                    help="keep the per-stage HIP events (RTBVH_FLAG_TIMING) in the frames-in-flight loops too (A/B)")
    ap.add_argument("--traversal", default="auto", choices=["auto", "reference"],
                    help="auto: report nearest-first when its frame is identical to the reference order's")
    ap.add_argument("--root-share", type=int, default=None,
                    help="rank 0's band share in 1/16 of another rank's (rtbvh_set_band_deal); default: "
                         "16 at N <= 2, 15 at N <= 4, 13 above (rank 0 also receives and assembles the bands)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")

    import torch
    import torch.distributed as dist

    if args.backend == "gloo":   # rehearsal: every rank on the visible device(s), round-robin
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    def barrier():
        if world > 1:
            dist.barrier()

    import raytracebvh_amd as rt

    wl = WORKLOADS[args.workload]
    W, H, bounces = wl["W"], wl["H"], wl["bounces"]
    t_setup = time.perf_counter()
    scene = make_scene(rt, wl)
    # a real (non-null) torch stream per context: torch's default stream is the null stream
    # (handle 0), and a context given stream 0 creates a private stream of its own, which
    # `with torch.cuda.stream(...)` could not order the RCCL gather after
    stream = torch.cuda.Stream(dev)
    assert stream.cuda_stream != 0
    ctx = rt.Context(device=local, flags=rt.FLAG_TIMING, stream=stream.cuda_stream)
    # the band deal: rank 0 also receives (RCCL) and assembles every other rank's
    # bands, about 0.1 ms per C5 frame whatever N (116 MB in at N = 8), against a rank's ~5.3/N ms
    # of tracing: so it takes 1 - ~2% x N of a share (an estimate until an 8-GPU run measures it)
    share = args.root_share if args.root_share is not None else (16 if world <= 2 else 15 if world <= 4 else 13)
    ctx.set_band_deal(share)
    ctx.set_scene(scene)
    wvp, wv = rt.camera_reference(W, H)
    ctx.set_camera(wvp, wv)
    log(f"scene {scene.num_tris} tris ready in {time.perf_counter() - t_setup:.1f}s (rank {rank}/{world})")

    # ---- BVH build (replicated on every rank), hipEvent-timed
    ctx.build()
    ctx.build()
    ctx.reset_stats()
    for _ in range(args.build_iters):
        ctx.build(sync=False)
    ctx.synchronize()
    bst = ctx.stats()
    build = {"workload": f"{scene.num_tris} tris (bench scene)", "ms": bst["ms_build"],
             "mtris_s": scene.num_tris / (bst["ms_build"] * 1e-3) / 1e6,
             "achieved_gbs": round(S_BUILD_PER_TRI * scene.num_tris / (bst["ms_build"] * 1e-3) / 1e9, 1),
             "stages_ms": dict(zip(["bounds", "morton", "sort", "karras", "refit"],
                                   [round(x, 4) for x in bst["ms_stage"][:5]]))}

    # ---- frames in flight: frame i is traced on streams[i % inflight] (stream 0 is the
    # context's); the context keeps a trace-buffer set per stream, all over the one BVH
    streams = [stream] + [torch.cuda.Stream(dev) for _ in range(args.inflight - 1)]
    ctxs = [ctx]

    # ---- band buffers + RCCL gather plumbing (raytracebvh_amd/tiles.py)
    from raytracebvh_amd.tiles import BandGather
    # one band buffer per frame in flight (>= 2): frame i's RCCL gather overlaps frame i+1's
    # trace (tiles.py), and frames traced concurrently never share a buffer
    g = BandGather(W, H, rank, world, device=dev, nbuf=max(2, args.inflight), root_share=share)
    band = g.band
    # torch fills the new buffers on its current stream; the other contexts' streams are
    # not ordered after it (a late fill overwrote traced pixels in a 3-process rehearsal)
    torch.cuda.synchronize()

    def run(nsteps, inflight):
        """nsteps frames: frame i traced on stream i % inflight into band buffer i % nbuf, then gathered (RCCL, after that stream) and assembled on the same
        stream, so the buffer's next trace waits for its gather; every frame is assembled
        before return."""
        pending = None
        for i in range(nsteps):
            k = i % inflight
            with torch.cuda.stream(streams[k]):
                ctx.trace_band_async(W, H, bounces, rank, world, g.band_buffer(i).data_ptr(),
                                     stream_ptr=streams[k].cuda_stream)
                h = g.gather_async(i)
            if pending is not None:
                with torch.cuda.stream(streams[pending[0] % inflight]):
                    g.assemble(*pending)
            pending = (i, h)
        if pending is not None:
            with torch.cuda.stream(streams[pending[0] % inflight]):
                g.assemble(*pending)
        return g.band_buffer(max(nsteps - 1, 0))

    def timed(flags, inflight=args.inflight):
        """Warm up, then time exactly args.steps steps between barrier + synchronize."""
        # the per-stage HIP events only one frame at a time (the kernels' durations below); in the frames-in-flight
        # loops they are host-clock timed and the events' barriers would only add gaps to the stream they land on
        timing = rt.FLAG_TIMING if inflight == 1 or args.timing_in_flight else 0
        for c in ctxs:
            c.set_flags(timing | flags)
        run(args.warmup, inflight)
        torch.cuda.synchronize()
        st = ctx.stats()
        tot = torch.tensor([st["primary_rays"] + st["bounce_rays"]], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(tot)
        ctx.reset_stats()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        last = run(args.steps, inflight)
        torch.cuda.synchronize()
        t_own = time.perf_counter() - t0   # this rank's own time, before waiting for the others
        barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        own = torch.tensor([t_own / args.steps * 1e3], dtype=torch.float64, device=dev)
        rank_ms = [float(own.item())]
        if world > 1:
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
            allown = [torch.zeros_like(own) for _ in range(world)]
            dist.all_gather(allown, own)
            rank_ms = [round(float(x.item()), 4) for x in allown]
        ms = float(el.item()) / args.steps * 1e3
        rays = float(tot[0].item())
        # the output: the frame assembled on rank 0 (one rank: its band buffer is the frame)
        frame = g.frames[(args.steps - 1) % g.nbuf].clone() if rank == 0 else None
        return dict(ms_step=ms, rays=rays, value=rays / (ms * 1e-3) / 1e6, stats=ctx.stats(),
                    band=last.clone(), frame=frame, rank_ms=rank_ms)

    # reference order (the exact findCollision DFS), nearest-first, and nearest-first on the
    # 4-wide view; a nearest-first number is the headline only if its frame is bit-identical
    # to the reference-order frame of this same run (checked on every rank's bands), and the
    # build above serves all three (one node layout)
    FAST = rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE   # same results as the plain kernels (tests)
    # "certified": RTBVH_FLAG_AUTO_WALK's walks (FLAG_CERTIFIED forces them whatever the size): the binned
    # pass and the 4-wide bounce walk on margin-grown boxes + per-ray certificates
    modes = {"reference-order": FAST, "nearest-first": FAST | rt.FLAG_NEAREST_FIRST,
             "nearest-first-wide": FAST | rt.FLAG_NEAREST_FIRST | rt.FLAG_WIDE_BVH,
             "nearest-first-wide-binned": FAST | rt.FLAG_NEAREST_FIRST | rt.FLAG_WIDE_BVH | rt.FLAG_BINNED_PRIMARY,
             "certified": rt.FLAG_CERTIFIED}
    # three interleaved rounds over the modes, each mode's median run kept (one slow moment on the box --
    # seen as a 15% swing of one mode in one round -- moves no number)
    runs = {m: [] for m in modes}
    for _ in range(3):
        for m, f in modes.items():
            runs[m].append(timed(f))
    res = {m: sorted(rs, key=lambda r: r["ms_step"])[len(rs) // 2] for m, rs in runs.items()}
    ref = res["reference-order"]
    traversal = {"frames_identical": {}}
    use_name = "reference-order"
    for m, r in res.items():
        traversal[m.replace("-", "_") + "_mrays_s"] = round(r["value"], 2)
        traversal[m.replace("-", "_") + "_ms"] = round(r["ms_step"], 4)
        if m == "reference-order":
            continue
        # compared on rank 0's assembled frame (the product), the verdict shared with all ranks
        same = torch.tensor([0.0 if rank != 0 or torch.equal(ref["frame"], r["frame"]) else 1.0], device=dev)
        if world > 1:
            dist.all_reduce(same)
        ident = float(same.item()) == 0.0
        traversal["frames_identical"][m] = ident
        if ident and args.traversal != "reference" and r["ms_step"] < res[use_name]["ms_step"]:
            use_name = m
    # the headline: the certified mode (RTBVH_FLAG_AUTO_WALK's walks at C5: the reference frame by
    # construction; its frame checked above against the reference order's). The fastest mode
    # whose frame equalled the reference order's in this run is reported beside it: the unchecked walks
    # are exact only when containment holds (tests/containment.py), so they are never the headline.
    traversal["fastest_identical_mode"] = use_name
    traversal["fastest_identical_mrays_s"] = round(res[use_name]["value"], 2)
    traversal["fastest_identical_ms"] = round(res[use_name]["ms_step"], 4)
    traversal["runs_ms"] = {m: [round(r["ms_step"], 4) for r in rs] for m, rs in runs.items()}
    if args.traversal != "reference":
        use_name = "certified"
        if not traversal["frames_identical"].get("certified"):   # a bug, never expected: say so loudly
            log("ERROR: the certified frame differs from the reference order's; reporting the reference order")
            use_name = "reference-order"
    use = res[use_name]
    traversal["mode"] = use_name
    # each rank's own ms per step before the closing barrier (rank 0 also receives and assembles the
    # frame): the data the band deal's root_share is fitted to
    traversal["rank_ms_per_step"] = use["rank_ms"]
    mode_flags = modes[use_name]
    rays_per_step, ms_step, value = use["rays"], use["ms_step"], use["value"]
    # one frame at a time (one context, one stream): the per-frame latency, and the kernels'
    # own HIP-event durations without a concurrent frame on the GPU (the roofline below)
    lat = timed(mode_flags, inflight=1)
    tst = lat["stats"]
    traversal["inflight"] = args.inflight
    traversal["one_frame_latency_ms"] = round(lat["ms_step"], 4)
    traversal["one_frame_mrays_s"] = round(lat["value"], 2)
    flag = torch.tensor([0.0 if rank != 0 or torch.equal(lat["frame"], use["frame"]) else 1.0], device=dev)
    if world > 1:
        dist.all_reduce(flag)
    same_lat = float(flag.item()) == 0.0
    if world > 1 and rank == 0:   # the frame assembled from every rank's bands vs one traced whole here
        full = torch.empty((H, W, 4), dtype=torch.float32, device=dev)
        torch.cuda.synchronize()
        ctx.set_flags(rt.FLAG_TIMING | mode_flags)
        ctx.trace_band_async(W, H, bounces, 0, 1, full.data_ptr())
        ctx.synchronize()
        traversal["assembled_frame_identical"] = bool(torch.equal(full, use["frame"]))
    traversal["inflight_frame_identical"] = same_lat
    if not same_lat and rank == 0:
        d = (lat["frame"] != use["frame"]).any(dim=2)
        print(f"[bench] frames in flight differ from one-frame frames: {int(d.sum())} pixels", file=sys.stderr,
              flush=True)

    # ---- visit counts for the byte model (extra, untimed traces of this rank's bands):
    # the chosen mode's own counts, and the reference-order counts of SURVEY §8(d)
    def counts(flags):
        ctx.set_flags(rt.FLAG_TIMING | rt.FLAG_COUNT_VISITS | flags)
        ctx.reset_stats()
        ctx.trace_band_async(W, H, bounces, rank, world, band.data_ptr())
        return ctx.stats()
    cst = counts(mode_flags)
    rst = counts(modes["reference-order"])
    ctx.set_flags(rt.FLAG_TIMING)
    wide = use_name.endswith("wide")
    binned = use_name.endswith("binned") or use_name == "certified"
    kern = {"k_primary": dict(ms=tst["ms_stage"][5],
                              bytes=binned_bytes(cst, scene.num_tris) if binned
                              else layout_bytes(cst, "k_primary", wide_primary=wide))}
    if bounces:   # 1 bounce: the first pass's traversal kernel has its own events
        kern["k_bounce_trav"] = dict(ms=tst["ms_stage"][7], bytes=layout_bytes(cst, "k_bounce_trav"))
        kern["k_bounce_shade"] = dict(ms=tst["ms_stage"][6] - tst["ms_stage"][7],
                                      bytes=layout_bytes(cst, "k_bounce_shade"))
    dom = max(kern, key=lambda k: kern[k]["ms"])
    # HBM traffic: the PMC bytes of each kernel from the rocprofv3 passes of the same mode at N = 1
    # (profiles/pmc_c5_<mode>.json), per record fetch x this launch's record fetches (at N = 1 the
    # profiled launch itself; at N > 1 a rank's launch fetches fewer records)
    recs = {"k_primary": (cst["bin_entries"][0] if binned else
                          sum(cst["packet_steps"]) or (cst["internal_visits"][0] + cst["leaf_visits"][0])),
            "k_bounce_trav": cst["internal_visits"][1] + cst["leaf_visits"][1],
            "k_bounce_shade": cst["bounce_rays"]}
    # per kernel: "requested" = this layout's algorithmic bytes (what the walk asks the memory system
    # for, L2 hits included) per HIP-event second; "frac" = the PMC HBM bytes of the same launch per
    # second over the HBM peak (the fraction north_star asks for)
    for k, v in kern.items():
        v["requested_gbs"] = v["bytes"] / (v["ms"] * 1e-3) / 1e9 if v["ms"] > 0 else 0.0
        v["requested_frac"] = v["requested_gbs"] / PEAK_HBM_GBS
        # the binned primary pass is several kernels: their summed PMC bytes (make_pmc_json.py)
        pm = load_pmc(args.workload, use_name, "k_primary_pass" if k == "k_primary" and binned else k)
        v["traffic"] = None
        v["frac"] = None
        if pm and pm.get("records_per_launch") and recs.get(k):
            v["traffic"] = pm["hbm_bytes_per_launch"] / pm["records_per_launch"] * recs[k]
            v["traffic_gbs"] = v["traffic"] / (v["ms"] * 1e-3) / 1e9 if v["ms"] > 0 else 0.0
            v["frac"] = v["traffic_gbs"] / PEAK_HBM_GBS
    kd = kern[dom]
    measured = kd["traffic"] is not None
    roofline = {"bound": "hbm",
                "achieved": round(kd["traffic_gbs"] if measured else kd["requested_gbs"], 1),
                "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(kd["frac"] if measured else kd["requested_frac"], 4),
                "frac_definition": ("rocprofv3 PMC HBM bytes of the kernel per launch (TCC_EA0 read/write requests "
                                    "x request size, MI355X_MICROARCH.md) / its HIP-event duration / 8 TB/s"
                                    if measured else "no PMC profile for this mode: requested bytes / duration / 8 TB/s"),
                "traffic": kd["traffic"], "kernel": dom, "kernel_ms": round(kd["ms"], 4),
                "algorithmic_bytes": int(kd["bytes"]),
                "requested_gbs": round(kd["requested_gbs"], 1), "requested_frac": round(kd["requested_frac"], 4),
                "bytes_model": "algorithmic_bytes / requested_*: this layout's bytes, 64 B per record fetch (QNode, "
                               "child-pair record, leaf record; a 4-wide primary step = 2) + per-ray queue/hit/colour "
                               "bytes (DESIGN.md 7.1); L2 and the Infinity Cache serve part of them",
                "traffic_source": f"PMC profiles/pmc_{args.workload}_{use_name}.json (N=1, collected at commit "
                                  f"{(load_pmc_meta(args.workload, use_name) or {}).get('commit')}), per record fetch x "
                                  f"this launch's {recs[dom]} record fetches" if measured else None,
                "kernel_trace_source": f"profiles/kernel_stats_{args.workload}_{use_name}.csv: rocprofv3 --kernel-trace "
                                       "--stats of scripts/profile_trace.py in the same mode, one frame at a time, "
                                       "collected in the same GPU call as the PMC file (kernel_ms is this run's "
                                       "HIP-event duration of the same launch, one frame at a time)"}
    if measured:
        roofline["cache_served_frac"] = round(max(0.0, 1.0 - kd["traffic"] / kd["bytes"]), 4)
    pm = load_pmc(args.workload, use_name, dom)
    if dom == "k_bounce_trav" and pm and pm.get("counters", {}).get("TCC_HIT_sum") is not None \
            and pm.get("records_per_launch"):
        # the roofline of a dependent-gather walk, per L2 REQUEST: the measured random-record
        # request rates of L2 and of HBM/Infinity Cache (scripts/gather_roofline.hip) x the PMC
        # L2 hits and misses of the same kernel, scaled to this launch's record fetches
        c = pm["counters"]
        scale = recs[dom] / pm["records_per_launch"]
        hits, miss = c["TCC_HIT_sum"] * scale, c["TCC_MISS_sum"] * scale
        model_ms = (hits / GATHER_L2_RPS + miss / GATHER_HBM_RPS) * 1e3
        roofline["gather"] = {"l2_requests": int(hits + miss), "record_fetches": int(recs[dom]),
                              "l2_hit_frac": round(hits / (hits + miss), 4),
                              "peak_requests_per_s": {"l2": GATHER_L2_RPS, "hbm": GATHER_HBM_RPS},
                              "model_ms": round(model_ms, 4), "kernel_ms": round(kd["ms"], 4),
                              "frac": round(model_ms / kd["ms"], 4)}
    # the build's roofline: SURVEY 8(d)'s 348 B per triangle, and the PMC bytes of its kernels
    bp = build_pmc(args.workload, use_name)
    build_roofline = {"bound": "hbm", "bytes_model": "SURVEY 8(d) B_build = 348 B per triangle",
                      "algorithmic_bytes": int(S_BUILD_PER_TRI * scene.num_tris), "ms": round(bst["ms_build"], 4),
                      "achieved": round(S_BUILD_PER_TRI * scene.num_tris / (bst["ms_build"] * 1e-3) / 1e9, 1),
                      "peak": PEAK_HBM_GBS, "unit": "GB/s"}
    build_roofline["algorithmic_frac"] = round(build_roofline["achieved"] / PEAK_HBM_GBS, 4)
    build_roofline["frac"] = None
    if bp:
        tgbs = bp["hbm_bytes"] / (bst["ms_build"] * 1e-3) / 1e9
        build_roofline.update({"traffic": bp["hbm_bytes"], "traffic_per_kernel_gb": bp["per_kernel_gb"],
                               "traffic_gbs": round(tgbs, 1), "frac": round(tgbs / PEAK_HBM_GBS, 4),
                               "frac_definition": "PMC HBM bytes of the build kernels per build / build ms / 8 TB/s",
                               "traffic_vs_algorithmic": round(bp["hbm_bytes"] / build_roofline["algorithmic_bytes"], 3)})
    fb = frame_bytes(rst)
    # SURVEY 8(d)'s whole-frame figure prices the REFERENCE-ORDER walk's visits; a traversal
    # that visits fewer nodes than that walk can exceed 1 here, so it is reported beside the
    # per-kernel roofline above (own visits), not instead of it
    frame_roofline = {"definition": "SURVEY 8(d): reference-order visit counts x per-unit bytes / trace time: a "
                                    "WORK-EQUIVALENT rate (the reference walk's bytes at this walk's speed), not HBM "
                                    "traffic and not a fraction of the roofline (the roofline above is)",
                      "bytes": int(fb), "trace_ms": round(tst["ms_trace"], 4),
                      "work_equivalent_gbs": round(fb / (tst["ms_trace"] * 1e-3) / 1e9, 1),
                      "work_equivalent_over_peak": round(fb / (tst["ms_trace"] * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)}

    result = None
    if rank == 0:
        extras = {}
        if world == 1 and not args.no_extras:
            # the reference's frame (Graphics.cpp:56, :667-831): rebuild the BVH and trace, one frame
            # at a time behind a fence (rtbvh_compute_bvh is synchronous), in the reported mode;
            # then the same frame replayed as one hipGraph (RTBVH_FLAG_GRAPH)
            # under the drop-in's configuration, RTBVH_FLAG_AUTO_WALK (the certified walks at C5's size:
            # the reference frame by construction), and under the headline's mode (suffix _fastest)
            reb = {"workload": wl["name"] + ", BVH rebuilt every frame",
                   "mode": "RTBVH_FLAG_AUTO_WALK (certified walks)", "mode_fastest": use_name}
            # (no RTBVH_FLAG_TIMING: its ten stage events cost ~0.07 ms of a rebuilt frame)
            for key, fl in (("", rt.FLAG_AUTO_WALK), ("_graph", rt.FLAG_GRAPH | rt.FLAG_AUTO_WALK),
                            ("_fastest", mode_flags), ("_graph_fastest", rt.FLAG_GRAPH | mode_flags)):
                ctx.set_flags(fl)
                ctx.compute_bvh(W, H, bounces)
                ctx.compute_bvh(W, H, bounces)
                nfr = max(5, args.steps // 2)
                t0 = time.perf_counter()
                for _ in range(nfr):
                    ctx.compute_bvh(W, H, bounces)
                dt = (time.perf_counter() - t0) / nfr
                q = ctx.stats()
                rk = q["primary_rays"] + q["bounce_rays"]
                reb["ms_per_frame" + key] = round(dt * 1e3, 4)
                reb["mrays_s" + key] = round(rk / dt / 1e6, 1)
                reb["frames" + key] = nfr
            reb["rays_per_frame"] = int(rk)
            # the same frames pipelined: two contexts (two BVHs, two streams) take alternate frames, each
            # frame still a full rebuild + trace of its own (Graphics.cpp:56 semantics per frame, no
            # work skipped), frame i + 1's build running beside frame i's trace; wall time per frame
            ctx.set_flags(rt.FLAG_AUTO_WALK)
            ctx.synchronize()
            with rt.Context(device=local, flags=rt.FLAG_AUTO_WALK) as cb:
                cb.set_scene(scene)
                cb.set_camera(wvp, wv)
                pair = [ctx, cb]
                for c in pair:   # warm-up
                    c.build(sync=False)
                    c.trace(W, H, bounces, sync=False)
                for c in pair:
                    c.synchronize()
                nfr = max(10, args.steps)
                t0 = time.perf_counter()
                for i in range(nfr):
                    c = pair[i % 2]
                    c.build(sync=False)
                    c.trace(W, H, bounces, sync=False)
                for c in pair:
                    c.synchronize()
                dtp = (time.perf_counter() - t0) / nfr
                reb["ms_per_frame_pipelined2"] = round(dtp * 1e3, 4)
                reb["mrays_s_pipelined2"] = round(rk / dtp / 1e6, 1)
                reb["frames_pipelined2"] = nfr
                reb["pipelined2_frames_identical"] = bool(np.array_equal(cb.read_framebuffer(), ctx.read_framebuffer()))
            extras["c5_frame_rebuild" if args.workload == "c5" else "frame_rebuild"] = reb
            ctx.set_flags(rt.FLAG_TIMING | mode_flags)
            # the reference's only interaction (Graphics::onKeyDown, Graphics.cpp:937-960): every frame the
            # eye orbits by CAM_DELTA and onUpdate re-uploads WVP / WV, then computeBVH (Graphics.cpp:40-56)
            # -- here under the configuration INTEGRATION.md gives the maintainer, AUTO_WALK | GRAPH: a new
            # camera replays the captured frame (the camera is a device buffer) with the certified walks
            orb = {"workload": wl["name"] + ", BVH rebuilt every frame, eye orbiting (VK_LEFT each frame)",
                   "flags": "RTBVH_FLAG_AUTO_WALK | RTBVH_FLAG_GRAPH"}
            with rt.Context(device=local, flags=rt.FLAG_AUTO_WALK | rt.FLAG_GRAPH) as co:
                co.set_scene(scene)
                eye = np.array(rt.EYE_REFERENCE, np.float32)
                cams = []
                nfr = max(10, args.steps)
                for i in range(nfr + 2):   # two warm-up frames (the capture), then the timed ones
                    eye = rt.camera_orbit(eye, rt.KEY_LEFT)
                    cams.append(rt.camera_look(eye, W, H))
                for i in range(2):
                    co.set_camera(*cams[i])
                    co.compute_bvh(W, H, bounces)
                t0 = time.perf_counter()
                for i in range(2, nfr + 2):
                    co.set_camera(*cams[i])
                    co.compute_bvh(W, H, bounces)
                dto = (time.perf_counter() - t0) / nfr
                qo = co.stats()
                caps = int(qo["graph_captures"])
                orb.update({"ms_per_frame": round(dto * 1e3, 4), "frames": nfr,
                            "mrays_s": round((qo["primary_rays"] + qo["bounce_rays"]) / dto / 1e6, 1),
                            "graph_captures": caps, "walk_state": int(qo["walk_state"]),
                            "redo_rays_last_frame": list(qo["redo_rays"]),
                            "vs_c5_frame_rebuild": round(dto * 1e3 / reb["ms_per_frame_graph"], 4)})
                # the same frames with the camera standing still: each timed camera set (and its first
                # frame run) outside the clock, then one frame of it timed -- what a moving camera costs
                # over the frames it renders (the views differ: a rotated eye sees other rays than C5's)
                st_t = 0.0
                for i in range(2, nfr + 2):
                    co.set_camera(*cams[i])
                    co.compute_bvh(W, H, bounces)
                    t0 = time.perf_counter()
                    co.compute_bvh(W, H, bounces)
                    st_t += time.perf_counter() - t0
                dts = st_t / nfr
                # and the reference camera under the same flags (the c5_frame_rebuild frame, certified walks)
                co.set_camera(wvp, wv)
                co.compute_bvh(W, H, bounces)
                t0 = time.perf_counter()
                for _ in range(nfr):
                    co.compute_bvh(W, H, bounces)
                dtr = (time.perf_counter() - t0) / nfr
                orb.update({"same_cameras_static_ms_per_frame": round(dts * 1e3, 4),
                            "vs_same_cameras_static": round(dto / dts, 4),
                            "c5_camera_same_flags_ms_per_frame": round(dtr * 1e3, 4),
                            "vs_c5_camera_same_flags": round(dto / dtr, 4),
                            "graph_captures_after_static": int(co.stats()["graph_captures"]) - caps})
                # frames: the last timed camera and an earlier one, re-rendered (deterministic) against the
                # reference-order frame of the same camera
                checks = []
                for i in (nfr + 1, 2 + nfr // 2):
                    co.set_camera(*cams[i])
                    co.compute_bvh(W, H, bounces)
                    got = co.read_framebuffer()
                    ctx.set_flags(FAST)   # the reference order (the exact findCollision DFS)
                    ctx.set_camera(*cams[i])
                    ctx.compute_bvh(W, H, bounces)
                    checks.append(bool(np.array_equal(got, ctx.read_framebuffer())))
                ctx.set_camera(wvp, wv)
                ctx.set_flags(rt.FLAG_TIMING | mode_flags)
                ctx.build()
                orb["frames_identical_to_reference_order"] = checks
            extras["c5_orbit" if args.workload == "c5" else "orbit"] = orb
        if world == 1 and not args.no_extras and args.workload == "c5":
            # C4: 10M synthetic (seed 0x5EED0004, +-50) build only; C3: Test.obj 1080p primary+1 bounce
            c4 = rt.synthetic(10_000_000, seed=0x5EED0004, half_extent=(50.0, 50.0, 50.0))

            def c4_build(flags):
                with rt.Context(device=local, flags=rt.FLAG_TIMING | flags) as c:
                    c.set_scene(c4)
                    c.set_camera(*rt.camera_reference(1920, 1080))
                    c.build()
                    c.reset_stats()
                    for _ in range(args.build_iters):
                        c.build(sync=False)
                    c.synchronize()
                    return c.stats()
            # the drop-in's configuration (RTBVH_FLAG_AUTO_WALK: the certified walks at this size, whose build
            # writes node boxes instead of node records), and the API's default (reference-order walks: records)
            s4 = c4_build(rt.FLAG_AUTO_WALK)
            s4d = c4_build(0)
            extras["c4_build"] = {"mtris_s": round(10_000_000 / (s4["ms_build"] * 1e-3) / 1e6, 1),
                                  "ms": round(s4["ms_build"], 4),
                                  "achieved_gbs": round(S_BUILD_PER_TRI * 1e7 / (s4["ms_build"] * 1e-3) / 1e9, 1),
                                  "stages_ms": [round(x, 4) for x in s4["ms_stage"][:5]],
                                  "flags": "RTBVH_FLAG_AUTO_WALK (the drop-in's: node boxes, no node records)",
                                  "default_walks": {"ms": round(s4d["ms_build"], 4),
                                                    "mtris_s": round(10_000_000 / (s4d["ms_build"] * 1e-3) / 1e6, 1),
                                                    "stages_ms": [round(x, 4) for x in s4d["ms_stage"][:5]],
                                                    "flags": "none (reference-order walks: node records)"}}
            del c4
            # C3 (Test.obj, primary + 1 bounce) and C2 (Image_Test.obj, primary only): the
            # reference rebuilds and traces every frame (Graphics.cpp:56), so build + trace
            for key in ("c3", "c2"):
                wk = WORKLOADS[key]
                sk = make_scene(rt, wk)
                # the reference-order kernels (the exact findCollision DFS): on these few-thousand-
                # triangle scenes they beat the packet / wide walks (C3 trace 0.28 vs 0.33 ms)
                with rt.Context(device=local, flags=rt.FLAG_TIMING) as c:
                    c.set_scene(sk)
                    c.set_camera(*rt.camera_reference(wk["W"], wk["H"]))
                    c.compute_bvh(wk["W"], wk["H"], wk["bounces"])
                    q = c.stats()
                    c.reset_stats()
                    t0 = time.perf_counter()
                    for _ in range(50):
                        c.compute_bvh(wk["W"], wk["H"], wk["bounces"])
                    dt = (time.perf_counter() - t0) / 50
                    q2 = c.stats()
                # the drop-in's own configuration: AUTO walk + the frame as one hipGraph
                with rt.Context(device=local, flags=rt.FLAG_GRAPH | rt.FLAG_AUTO_WALK) as c:
                    c.set_scene(sk)
                    wvp_k, wv_k = rt.camera_reference(wk["W"], wk["H"])
                    c.set_camera(wvp_k, wv_k)
                    c.compute_bvh(wk["W"], wk["H"], wk["bounces"])   # capture
                    t0 = time.perf_counter()
                    for _ in range(50):
                        c.compute_bvh(wk["W"], wk["H"], wk["bounces"])
                    dtg = (time.perf_counter() - t0) / 50
                    gframe, gtree = c.read_framebuffer(), c.read_bvh()
                rk = q["primary_rays"] + q["bounce_rays"]
                extras[f"{key}_frame"] = {"workload": wk["name"], "rays": int(rk),
                                          "mrays_s_trace": round(rk / (q2["ms_trace"] * 1e-3) / 1e6, 1),
                                          "mrays_s_build_plus_trace_wall": round(rk / dt / 1e6, 1),
                                          "mrays_s_build_plus_trace_wall_graph": round(rk / dtg / 1e6, 1),
                                          "ms_build": round(q2["ms_build"], 4), "ms_trace": round(q2["ms_trace"], 4)}
                if key == "c3":
                    # BASELINE.json's metric is quoted "@1080p" on C3 (Test.obj, primary + 1 reflection
                    # bounce): its own first-class line, in the reference's frame semantics -- rebuild +
                    # trace every frame, synchronously (Graphics.cpp:56, 667-831) -- with its frame and
                    # tree checked against the oracle (OpenMP; cache-resident scene: the roofline is C5's)
                    from oracle import lib as orc
                    osk = orc.Scene(sk.vertices, sk.indices, sk.mat_indices, sk.material_blob)
                    otree = orc.build(osk, wvp_k, sort_mode=0)
                    orc.set_threads(int(os.environ.get("OMP_NUM_THREADS") or 0) or (os.cpu_count() or 1))
                    try:
                        oframe, _, _ = orc.trace(osk, otree, wvp_k, wv_k, wk["W"], wk["H"], wk["bounces"])
                    finally:
                        orc.set_threads(1)
                    extras["c3_1080p"] = {
                        "metric": "Mrays/s primary+1-bounce @1080p (BASELINE.json metric on its own config, C3)",
                        "value": round(rk / dtg / 1e6, 1), "unit": "Mrays/s", "ms_per_frame": round(dtg * 1e3, 4),
                        "higher_is_better": True, "dtype": "f32", "data": "Obj/Test.obj fixture (parsed reference mesh)",
                        "config": {"workload": wk["name"], "width": wk["W"], "height": wk["H"], "bounces": 1,
                                   "triangles": sk.num_tris, "rays_per_frame": int(rk)},
                        "semantics": "rtbvh_compute_bvh per frame (BVH rebuilt + primary + 1 bounce, synchronous, "
                                     "as Graphics::onUpdate -> computeBVH), RTBVH_FLAG_AUTO_WALK | RTBVH_FLAG_GRAPH",
                        "build_ms": round(q2["ms_build"], 4), "trace_ms": round(q2["ms_trace"], 4),
                        "mrays_s_trace_only": round(rk / (q2["ms_trace"] * 1e-3) / 1e6, 1),
                        "parity": {"tree_bit_identical": bool(all(np.array_equal(gtree[f], otree[f])
                                                                  for f in NODE_FIELDS)),
                                   "frame_bit_identical": bool(np.array_equal(gframe, oframe)),
                                   "pixels_checked": int(wk["W"] * wk["H"])}}
        cpu = parity = None
        if world == 1 and not args.no_cpu_baseline:
            log("cpu baseline (oracle, bounded sample) ...")
            gpu_frame = use["frame"].cpu().numpy() if use["frame"] is not None else None
            cpu, parity = cpu_baseline(rt, scene, ctx, wl, W, H, gpu_frame)
            del gpu_frame
        reb = extras.get("c5_frame_rebuild") or extras.get("frame_rebuild") or {}
        orb = extras.get("c5_orbit") or extras.get("orbit") or {}
        result = {
            "metric": "Mrays/s primary+1-bounce (BASELINE.json's metric, on its config C5: 3840x2160, the 1/2/4/8-GPU "
                      "config; the metric's @1080p config C3 is the line c3_1080p); BVH build Mtris/s under build",
            "value": round(value, 2), "unit": "Mrays/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (splitmix64 generator, SURVEY §8(d))" if "obj" not in wl else "Obj/Test.obj fixture",
            "config": {"workload": wl["name"], "width": W, "height": H, "bounces": bounces,
                       "triangles": scene.num_tris, "rays_per_step": int(rays_per_step),
                       "parallelism": f"image bands x{world} + RCCL gather" if world > 1 else "single GPU",
                       "band_deal_root_share": share},
            "value_semantics": "frames in flight (--inflight per rank) traced over one BVH built before the timed "
                               "loop (static scene and camera: the camera-dependent build work -- the clip-space "
                               "transform, the leaf records and pixel footprints -- is part of the build, reported "
                               "under build); the reference's own frame (Graphics.cpp:56: rebuild + trace, "
                               "synchronous, one hipGraph) is c5_frame_rebuild_* under the drop-in's "
                               "RTBVH_FLAG_AUTO_WALK (certified walks; c5_frame_rebuild_fastest_ms in the headline's "
                               "mode), and a moving camera, the same flags, c5_orbit_*",
            "c5_frame_rebuild_ms": reb.get("ms_per_frame_graph"),
            "c5_frame_rebuild_mrays_s": reb.get("mrays_s_graph"),
            "c5_frame_rebuild_fastest_ms": reb.get("ms_per_frame_graph_fastest"),
            "c5_orbit_ms": orb.get("ms_per_frame"),
            "c5_orbit_mrays_s": orb.get("mrays_s"),
            "c5_orbit_vs_same_cameras_static": orb.get("vs_same_cameras_static"),
            "certified_mrays_s": traversal.get("certified_mrays_s"),
            "certified_ms_per_step": traversal.get("certified_ms"),
            "roofline": roofline,
            "build_roofline": build_roofline,
            "parity": parity,
            "kernels": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                        for k, v in kern.items()},
            "visits": {"internal": cst["internal_visits"], "leaf": cst["leaf_visits"], "hits": cst["hits"],
                       "primary_packet_steps": cst["packet_steps"],
                       "reference_order_internal": rst["internal_visits"], "reference_order_leaf": rst["leaf_visits"]},
            "frame_roofline": frame_roofline,
            "traversal": traversal,
            "build": build,
            "cpu_baseline": cpu,
        }
        result.update(extras)
    for c in ctxs:
        c.close()
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
