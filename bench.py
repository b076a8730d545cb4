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
RCCL gather + assembly on rank 0.  Three frames are in flight per rank (--inflight 3):
frame i is traced on stream i % 3 (the context gives each caller stream a trace-buffer
set of its own over the one BVH: rtbvh_trace_band_async), so frame i+1's primary pass
fills the GPU while frame i's bounce walk drains its last long walks; two band buffers keep one gather in flight
(step i's gather overlaps step i+1's trace), and every step's frame is traced,
gathered and assembled before the timed region closes.  The one-frame latency (one
context, frames back to back on one stream) is reported beside it.  The BVH is built once before the timed
loop (the scene is static; replicated build throughput is measured separately and
reported under "build").  value = all rays of the frame (W*H primary + every
live bounce ray, summed over ranks) / max-over-ranks time per step.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c5|c3]
       (N > 1 under `torch.distributed.run --nproc-per-node N`).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_HBM_GBS = 8000.0            # MI355X HBM3E spec (MI355X_MICROARCH.md)
# algorithmic bytes per unit, SURVEY.md §8(d) (the reference's data per unit of work)
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


def trace_bytes(st, kernel, wide=False):
    """Algorithmic bytes of one launch: SURVEY §8(d) per-unit figures x the units that
    launch processes (its own visit counts).  A 4-wide visit tests the four grandchild
    boxes = two binary child-pair records (2 x S_INT)."""
    if kernel == "k_primary":
        return (S_INT * st["internal_visits"][0] + S_LEAF * st["leaf_visits"][0] + S_PRIMARY * st["primary_rays"]
                + S_HIT * st["hits"][0] + S_TEX * st["textured_hits"])
    if kernel == "k_bounce_trav":
        return (2 if wide else 1) * S_INT * st["internal_visits"][1] + S_LEAF * st["leaf_visits"][1]
    # k_bounce_shade
    return S_BOUNCE * st["bounce_rays"] + S_HIT * st["hits"][1]


def frame_bytes(st):
    """SURVEY §8(d) frame bytes from REFERENCE-ORDER visit counts."""
    return (S_INT * sum(st["internal_visits"]) + S_LEAF * sum(st["leaf_visits"]) + S_PRIMARY * st["primary_rays"]
            + S_BOUNCE * st["bounce_rays"] + S_HIT * sum(st["hits"]) + S_TEX * st["textured_hits"])


def load_pmc(workload, mode, kernel, counters=False):
    """Per-launch HBM bytes of `kernel` (or its raw counters) from the PMC passes of the same
    traversal mode (profiles/pmc_<workload>_<mode>.json, written by scripts/make_pmc_json.py)."""
    path = os.path.join(REPO, "profiles", f"pmc_{workload}_{mode}.json")
    if not os.path.exists(path):
        return None
    try:
        k = json.load(open(path))["kernels"][kernel]
        return k["counters"] if counters else k["hbm_bytes_per_launch"]
    except Exception:
        return None


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(rt, scene, ctx, wl, W, H):
    """Oracle (single-thread C++ restatement of the reference path) on a bounded sample."""
    from oracle import lib as orc
    wvp, wv = rt.camera_reference(W, H)
    nodes = ctx.read_bvh()
    osc = orc.Scene(scene.vertices, scene.indices, scene.mat_indices, scene.material_blob)
    step = 8 if W * H > 4_000_000 else 4
    t0 = time.perf_counter()
    _, _, st = orc.trace(osc, nodes, wvp, wv, W, H, wl["bounces"], 0, H, step)
    dt = time.perf_counter() - t0
    rays = st["primary"] + st["bounce"]
    res = {"value": rays / dt / 1e6, "unit": "Mrays/s", "cores": 1, "kind": "port",
           "sample": f"oracle/liboracle.so orc_trace of 1 row in {step} of the same frame and BVH "
                     f"({st['primary']} primary + {st['bounce']} bounce rays, {dt:.1f} s, 1 thread)",
           "cpu_model": cpu_model(), "host_cpus": os.cpu_count()}
    # BASELINE.md's all-cores variant: the same code, OpenMP over rows, on this process's CPU
    # share (OMP_NUM_THREADS, 16 on the GPU boxes), on a 4x larger sample
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or (os.cpu_count() or 1)
    step_all = max(1, step // 4)
    orc.set_threads(threads)
    try:
        t0 = time.perf_counter()
        _, _, st2 = orc.trace(osc, nodes, wvp, wv, W, H, wl["bounces"], 0, H, step_all)
        dt2 = time.perf_counter() - t0
    finally:
        orc.set_threads(1)
    res["all_cores"] = {"value": (st2["primary"] + st2["bounce"]) / dt2 / 1e6, "unit": "Mrays/s", "cores": threads,
                        "sample": f"1 row in {step_all}, {st2['primary']} primary + {st2['bounce']} bounce rays, "
                                  f"{dt2:.1f} s, OpenMP over rows"}
    # build baseline: reference-faithful 32 x 1-bit split sort + Karras + refit on a 1M-triangle sample
    n_s = 1_000_000
    sub = rt.Scene(scene.vertices[: 3 * n_s], scene.indices[: 3 * n_s], scene.mat_indices[:n_s], scene.materials)
    if "obj" in wl:
        sub = scene
    osub = orc.Scene(sub.vertices, sub.indices, sub.mat_indices, sub.material_blob)
    t0 = time.perf_counter()
    orc.build(osub, wvp, sort_mode=0)
    dt = time.perf_counter() - t0
    res["build_mtris_s"] = sub.num_tris / dt / 1e6
    res["build_sample"] = f"orc_build (32 split passes + Karras + refit) on {sub.num_tris} triangles, {dt:.2f} s, 1 thread"
    return res


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
    ap.add_argument("--inflight", type=int, default=3, choices=[1, 2, 3],
                    help="frames in flight per rank (one context + stream each)")
    ap.add_argument("--traversal", default="auto", choices=["auto", "reference"],
                    help="auto: report nearest-first when its frame is identical to the reference order's")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")

    import numpy as np
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
             "stages_ms": dict(zip(["bounds", "morton", "sort", "leaf_karras", "refit"],
                                   [round(x, 4) for x in bst["ms_stage"][:5]]))}

    # ---- frames in flight: frame i is traced on streams[i % inflight] (stream 0 is the
    # context's); the context keeps a trace-buffer set per stream, all over the one BVH
    streams = [stream] + [torch.cuda.Stream(dev) for _ in range(args.inflight - 1)]
    ctxs = [ctx]

    # ---- band buffers + RCCL gather plumbing (raytracebvh_amd/tiles.py)
    from raytracebvh_amd.tiles import BandGather
    # one band buffer per frame in flight (>= 2): frame i's RCCL gather overlaps frame i+1's
    # trace (tiles.py), and frames traced concurrently never share a buffer
    g = BandGather(W, H, rank, world, device=dev, nbuf=max(2, args.inflight))
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
        for c in ctxs:
            c.set_flags(rt.FLAG_TIMING | flags)
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
        barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        ms = float(el.item()) / args.steps * 1e3
        rays = float(tot[0].item())
        # the output: the frame assembled on rank 0 (one rank: its band buffer is the frame)
        frame = g.frames[(args.steps - 1) % g.nbuf].clone() if rank == 0 else None
        return dict(ms_step=ms, rays=rays, value=rays / (ms * 1e-3) / 1e6, stats=ctx.stats(),
                    band=last.clone(), frame=frame)

    # reference order (the exact findCollision DFS), nearest-first, and nearest-first on the
    # 4-wide view; a nearest-first number is the headline only if its frame is bit-identical
    # to the reference-order frame of this same run (checked on every rank's bands), and the
    # build above serves all three (one node layout)
    FAST = rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE   # same results as the plain kernels (tests)
    modes = {"reference-order": FAST, "nearest-first": FAST | rt.FLAG_NEAREST_FIRST,
             "nearest-first-wide": FAST | rt.FLAG_NEAREST_FIRST | rt.FLAG_WIDE_BVH}
    res = {m: timed(f) for m, f in modes.items()}
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
    use = res[use_name]
    traversal["mode"] = use_name
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
    kern = {"k_primary": dict(ms=tst["ms_stage"][5], bytes=trace_bytes(cst, "k_primary"))}
    if bounces:   # 1 bounce: the first pass's traversal kernel has its own events
        kern["k_bounce_trav"] = dict(ms=tst["ms_stage"][7],
                                     bytes=trace_bytes(cst, "k_bounce_trav", wide=use_name.endswith("wide")))
        kern["k_bounce_shade"] = dict(ms=tst["ms_stage"][6] - tst["ms_stage"][7],
                                      bytes=trace_bytes(cst, "k_bounce_shade"))
    dom = max(kern, key=lambda k: kern[k]["ms"])
    for k, v in kern.items():
        v["achieved_gbs"] = v["bytes"] / (v["ms"] * 1e-3) / 1e9 if v["ms"] > 0 else 0.0
    traffic = load_pmc(args.workload, use_name, dom)
    roofline = {"bound": "hbm", "achieved": round(kern[dom]["achieved_gbs"], 1), "peak": PEAK_HBM_GBS,
                "unit": "GB/s", "frac": round(kern[dom]["achieved_gbs"] / PEAK_HBM_GBS, 4),
                "traffic": traffic, "kernel": dom, "kernel_ms": round(kern[dom]["ms"], 4),
                "algorithmic_bytes": int(kern[dom]["bytes"])}
    if traffic:
        # the algorithmic bytes are node/leaf bytes per visit; the upper tree levels stay in
        # L2, so the measured HBM rate (PMC bytes of the same kernel) is the second number
        tg = traffic / (kern[dom]["ms"] * 1e-3) / 1e9
        roofline.update({"traffic_gbs": round(tg, 1), "traffic_frac": round(tg / PEAK_HBM_GBS, 4),
                         "cache_served_frac": round(max(0.0, 1.0 - traffic / kern[dom]["bytes"]), 4)})
    if dom == "k_bounce_trav":
        # the roofline of a dependent-gather walk: one 64-B record per step (QNode or leaf), at
        # the measured random-record rates of L2 and of HBM/Infinity Cache, split by the L2 hit
        # fraction of the same kernel (PMC); frac = model time / measured time
        pc = load_pmc(args.workload, use_name, dom, counters=True)
        recs = cst["internal_visits"][1] + cst["leaf_visits"][1]
        if pc and pc.get("TCC_HIT_sum") is not None and pc.get("TCC_MISS_sum"):
            h = pc["TCC_HIT_sum"] / (pc["TCC_HIT_sum"] + pc["TCC_MISS_sum"])
            model_ms = recs * (h / GATHER_L2_RPS + (1 - h) / GATHER_HBM_RPS) * 1e3
            roofline["gather"] = {"records": int(recs), "l2_hit_frac": round(h, 4),
                                  "peak_records_per_s": {"l2": GATHER_L2_RPS, "hbm": GATHER_HBM_RPS},
                                  "model_ms": round(model_ms, 4), "kernel_ms": round(kern[dom]["ms"], 4),
                                  "frac": round(model_ms / kern[dom]["ms"], 4)}
    fb = frame_bytes(rst)
    # SURVEY 8(d)'s whole-frame figure prices the REFERENCE-ORDER walk's visits; a traversal
    # that visits fewer nodes than that walk can exceed 1 here, so it is reported beside the
    # per-kernel roofline above (own visits), not instead of it
    frame_roofline = {"definition": "SURVEY 8(d): reference-order visit counts x per-unit bytes / trace time "
                                    "(work-equivalent rate; not HBM traffic)",
                      "bytes": int(fb), "trace_ms": round(tst["ms_trace"], 4),
                      "achieved_gbs": round(fb / (tst["ms_trace"] * 1e-3) / 1e9, 1),
                      "frac": round(fb / (tst["ms_trace"] * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)}

    result = None
    if rank == 0:
        extras = {}
        if world == 1 and not args.no_extras and args.workload == "c5":
            # C4: 10M synthetic (seed 0x5EED0004, +-50) build only; C3: Test.obj 1080p primary+1 bounce
            c4 = rt.synthetic(10_000_000, seed=0x5EED0004, half_extent=(50.0, 50.0, 50.0))
            with rt.Context(device=local, flags=rt.FLAG_TIMING) as c:
                c.set_scene(c4)
                c.set_camera(*rt.camera_reference(1920, 1080))
                c.build()
                c.reset_stats()
                for _ in range(args.build_iters):
                    c.build(sync=False)
                c.synchronize()
                s4 = c.stats()
            extras["c4_build"] = {"mtris_s": round(10_000_000 / (s4["ms_build"] * 1e-3) / 1e6, 1),
                                  "ms": round(s4["ms_build"], 4),
                                  "achieved_gbs": round(S_BUILD_PER_TRI * 1e7 / (s4["ms_build"] * 1e-3) / 1e9, 1),
                                  "stages_ms": [round(x, 4) for x in s4["ms_stage"][:5]]}
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
                with rt.Context(device=local, flags=rt.FLAG_GRAPH) as c:   # the frame as one hipGraph
                    c.set_scene(sk)
                    c.set_camera(*rt.camera_reference(wk["W"], wk["H"]))
                    c.compute_bvh(wk["W"], wk["H"], wk["bounces"])   # capture
                    t0 = time.perf_counter()
                    for _ in range(50):
                        c.compute_bvh(wk["W"], wk["H"], wk["bounces"])
                    dtg = (time.perf_counter() - t0) / 50
                rk = q["primary_rays"] + q["bounce_rays"]
                extras[f"{key}_frame"] = {"workload": wk["name"], "rays": int(rk),
                                          "mrays_s_trace": round(rk / (q2["ms_trace"] * 1e-3) / 1e6, 1),
                                          "mrays_s_build_plus_trace_wall": round(rk / dt / 1e6, 1),
                                          "mrays_s_build_plus_trace_wall_graph": round(rk / dtg / 1e6, 1),
                                          "ms_build": round(q2["ms_build"], 4), "ms_trace": round(q2["ms_trace"], 4)}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            log("cpu baseline (oracle, bounded sample) ...")
            cpu = cpu_baseline(rt, scene, ctx, wl, W, H)
        result = {
            "metric": "Mrays/s primary+1-bounce (C5 frame); BVH build Mtris/s under build",
            "value": round(value, 2), "unit": "Mrays/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (splitmix64 generator, SURVEY §8(d))" if "obj" not in wl else "Obj/Test.obj fixture",
            "config": {"workload": wl["name"], "width": W, "height": H, "bounces": bounces,
                       "triangles": scene.num_tris, "rays_per_step": int(rays_per_step),
                       "parallelism": f"image bands x{world} + RCCL gather" if world > 1 else "single GPU"},
            "roofline": roofline,
            "kernels": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                        for k, v in kern.items()},
            "visits": {"internal": cst["internal_visits"], "leaf": cst["leaf_visits"], "hits": cst["hits"],
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
