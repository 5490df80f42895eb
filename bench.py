#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: cost-volume voxels/s (W*H*D per frame = both views)
and ms/frame, 1920x1200 D=128 synthetic pair on one MI355X; D-sharded over N GPUs.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode strong|weak|batch]
    torchrun ... bench.py --gpus N ...   (one process per GPU, RCCL over xGMI)

One step = one frame: both views through the whole path with the images already in HBM
(median, weights, Boruvka MST, tree layout, leaf->root and root->leaf passes, WTA, and for
N>1 the RCCL min+argmin reduce).  Frames are streamed with up to 3 in flight (--inflight): each
in-flight frame has its own context (buffers + HIP stream), so the next frame's prep / MST / layout
runs while the previous frame's tree filter does; every frame is computed in full.  N=1 runs BASELINE config C2 (1920x1200 D=128).  Modes for N>1:
  strong (default): total D = 256 split over N ranks (BASELINE config C4, 32 disparities/GPU at N=8)
  weak            : each rank owns 128 disparities, total D = 128*N, one cross-rank reduce
  batch           : one independent 3840x2160 D=256 pair per rank, no collective (config C5)
Launched without torchrun, --gpus N > 1 starts the N rank processes itself (before any GPU call);
under torchrun, WORLD_SIZE must equal --gpus.  Rank 0 prints ONE JSON line.
"""
import argparse
import math
import json
import os
import socket
import subprocess
import sys
import time

import torch  # noqa: F401  (loaded first: the HIP library then binds to torch's HIP runtime)
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import stereomatch_amd as sm  # noqa: E402
from tools.synth import make_pair  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
CONFIG_NAMES = {(1920, 1200, 128): " (BASELINE C2)", (3840, 2160, 256): " (BASELINE C3)",
                (1920, 1200, 256): " (BASELINE C4 size, unsharded)"}


def host_cpu_info():
    """nproc, the cores this process may use, the CPU model and OMP_NUM_THREADS."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    return dict(nproc=os.cpu_count(), affinity=usable, model=model, OMP_NUM_THREADS=omp)


def cpu_baseline(W, H, D):
    """Oracle (CPU restatement, reference order, fp64) on the benchmarked workload: the full MST build of
    both views (one thread: Kruskal is serial), then all D disparity slices of AGD cost + tree filter +
    WTA with all usable host cores (OpenMP over slices; the box's share: OMP_NUM_THREADS when set).
    Measured in full, no extrapolation.  Test infrastructure, used only as the reported baseline (never
    inside the timed region)."""
    from oracle import oracle as O
    info = host_cpu_info()
    threads = int(info["OMP_NUM_THREADS"] or 0) or info["affinity"]
    threads = max(1, min(threads, info["affinity"]))
    left, right, _ = make_pair(W, H, D, index=0)
    t0 = time.perf_counter()
    trees = [O.build_tree(left), O.build_tree(right)]
    t_tree = time.perf_counter() - t0

    def run(d0, n, nt):
        t0 = time.perf_counter()
        lv, rv = O.cost_agd(left, right, d0, d0 + n, nt)  # OpenMP over slices
        t_cost = time.perf_counter() - t0
        t0 = time.perf_counter()
        for t, vol in zip(trees, (lv, rv)):
            O.tree_filter(W, H, t, vol, d0, True, False, nt)
        return t_cost, time.perf_counter() - t0

    tc, tf = run(0, D, threads)
    frame = t_tree + tc + tf
    return dict(value=W * H * D / frame, unit="voxels/s", cores=threads, kind="port", ms_per_frame=frame * 1e3,
                host=info,
                stages_s=dict(tree_both_views=t_tree, cost=tc, filter_up_down_wta=tf),
                sample="one full %dx%d D=%d frame, both views: MST+BFS (1 thread), AGD cost, tree filter and WTA of "
                       "all %d slices (%d threads, OpenMP over slices); %.0f ms/frame" % (W, H, D, D, threads, frame * 1e3))


PMS_BYTES_PER_EVAL = 24  # data-term gather (2 x f32) + fp64 A_up write + read per node-label


def pms_leg(ctx, left, right, D, iters, oracle):
    """MST_PMS (SM_AGG_PMS): what stereo3dmst() actually runs (Stereo3DMST.cpp:805-904) -- segment forests
    (c=5000, min_size 200), random plane labels, `iters` MST_PMS calls per view (the reference's 100,
    :854), plane disparities -- measured end to end as one frame (host buffers in and out), beside the
    oracle's serial CPU restatement of ONE call per view (rank 0 only).  The roofline of the later calls:
    node-label evaluations they needed (counted on the device, k_pms_count) x PMS_BYTES_PER_EVAL / their
    wall time."""
    p = sm.default_params(aggregator=sm.SM_AGG_PMS, c=5000.0, min_size=200, pms_iters=2, disp_total=D)
    ctx.match(left, right, D, p)  # warm-up (allocations)
    p.pms_iters = iters
    t = time.perf_counter()
    ctx.match(left, right, D, p)
    wall = (time.perf_counter() - t) * 1e3
    st = ctx.pms_stats()
    later_ms = st["iters_ms"]
    alg = st["evals_later"] * PMS_BYTES_PER_EVAL
    out = dict(iters_per_view=iters, frame_s=wall / 1e3, trees=st["ntrees"], host_prep_ms=st["prep_ms"],
               prep_segmentation_ms=st.get("prep_seg_ms"), prep_schedule_forest_ms=st.get("prep_forest_ms"),
               setup_ms=st["setup_ms"], first_call_ms=st["iter0_ms"],
               later_call_ms=later_ms / (iters - 1) if iters > 1 else None,
               later_call_ms_per_view=[m / (iters - 1) for m in st["later_ms_view"]] if iters > 1 else None,
               concurrent_views=bool(st["concurrent_views"]),
               speculative_passes=st["spec_rounds"], serially_run_trees=st["serial_trees"],
               node_label_evals=dict(first_call=st["evals_first"], later_calls=st["evals_later"],
                                     later_calls_reference_count=st["evals_later_ref"],
                                     later_calls_run_on_device=st["evals_later_run"] or None),
               roofline=dict(bound="hbm", kernel="MST_PMS later calls (walks, repairs, cost, update)",
                             bytes_per_eval=PMS_BYTES_PER_EVAL, alg_bytes=alg,
                             achieved=alg / (later_ms * 1e-3) / 1e9 if later_ms > 0 else 0.0, peak=HBM_PEAK_GBS,
                             unit="GB/s", frac=alg / (later_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if later_ms > 0 else 0.0,
                             timing="wall clock of calls 2..%d of both views (host timers around the calls)" % iters),
               what="stereo3dmst's own algorithm, one frame: sm_match with host buffers (images up, maps down), "
                    "host prep + first call (serial) + %d later calls (speculative), both views; measured, "
                    "not extrapolated" % (iters - 1))
    if oracle:
        from oracle import oracle as O
        t = time.perf_counter()
        O.stereo3dmst_pms(left, right, D, iters=1)
        s = time.perf_counter() - t
        out["oracle_one_call_both_views_s"] = s
        out["oracle_note"] = ("oracle/sm_oracle_pms.c, 1 thread (the reference is serial), segmentation + BFS + AGD "
                              "volume + one MST_PMS call per view")
    return out


def stream_frames(ctxs, steps, D, params, retire, split=True, lag=1):
    """Stream `steps` frames over the contexts, frame i on context i mod len(ctxs), keeping up to
    len(ctxs) in flight; retire(c) waits for context c's frame.  split: frame i's tree is enqueued
    (match_begin) before the host waits for frame i-lag's layout and enqueues its filter
    (match_finish), so the GPU never idles on the host; otherwise one match_async per frame.
    lag (1 .. len(ctxs) - 1): frames whose tree is begun but not finished.  1 suits the MST (its
    tree is GPU work that finishes quickly); segment mode's tree has host steps (its worker thread),
    and a larger lag lets that many frames segment at once.  lag len(ctxs) - 1 would retire each
    frame right after finishing it (the host then waits for its whole filter): len(ctxs) - 2 leaves
    the filter one iteration to run."""
    n = len(ctxs)
    if n == 1 or not split:
        for i in range(steps):
            ctxs[i % n].match_async(D, params)  # returns once the frame's filter is enqueued
            if i >= n - 1:
                retire(ctxs[(i - n + 1) % n])
    else:
        lag = max(1, min(lag, n - 1))
        for i in range(steps):
            ctxs[i % n].match_begin(D, params)
            if i >= lag:
                ctxs[(i - lag) % n].match_finish()
            if i >= n - 1:
                retire(ctxs[(i - n + 1) % n])
        for i in range(max(0, steps - lag), steps):
            ctxs[i % n].match_finish()
    for i in range(max(0, steps - n + 1), steps):
        retire(ctxs[i % n])


def segment_leg(ctxs, left, right, D, steps, warmup, c=5000.0, min_size=200, inflight=6):
    """Stereo3DMST's own tree configuration, the segment forest (c = 5000, min_size = 200,
    Stereo3DMST.cpp:831-832), through the per-slice filter on the same pair: streamed ms/frame with
    `inflight` frames in flight (the segment-mode default; each frame segments on its context's worker
    thread) and the single-frame latency.  Reported beside the MST-mode metric, never as it."""
    extra = [sm.Context(ctxs[0].device) for _ in range(max(0, inflight - len(ctxs)))]
    cs = (list(ctxs) + extra)[:inflight]
    for cx in extra:
        cx.upload(left, right)
    p = sm.default_params(c=c, min_size=min_size)
    for cx in cs:
        cx.set_kernel_timing([])
    for _ in range(max(warmup, 1)):
        for cx in cs:
            cx.match_async(D, p)
            cx.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stream_frames(cs, steps, D, p, lambda cx: cx.synchronize(), lag=max(1, len(cs) - 2))
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    lat = []
    for _ in range(3):
        t = time.perf_counter()
        cs[0].match_async(D, p)
        cs[0].synchronize()
        lat.append((time.perf_counter() - t) * 1e3)
    for cx in extra:
        cx.close()
    return dict(ms_per_frame=ms, value=left.shape[0] * left.shape[1] * D / (ms * 1e-3), unit="voxels/s",
                latency_ms=min(lat), frames=steps, frames_in_flight=len(cs), c=c, min_size=min_size,
                what="segment forest (Stereo3DMST's own tree, c=%g, min_size=%d) + per-slice tree filter + WTA, "
                     "both views, same pair; %d frames streamed with %d in flight, latency best of 3"
                     % (c, min_size, steps, len(cs)))


def sm_environment():
    """Every SM_* variable of this process's environment (recorded in the line; refused without --dev)."""
    return {k: v for k, v in os.environ.items() if k.startswith("SM_")}


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """One process per GPU, started before this process touches a GPU (no exec: children)."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


def default_frame_groups(mode, n):
    """Strong mode at N >= 8 ranks: 2 frame groups, else 1."""
    return 2 if (mode == "strong" and n >= 8 and n % 4 == 0) else 1


def rank_plan(args, world, rank, fg_arg=None):
    """This rank's share of a frame: image size, its disparity range and views, and its reduce group
    (stereomatch_amd.partition)."""
    W, H = args.width, args.height
    views, group, gsize, grank = 3, 0, world, rank  # this rank's views and its reduce group
    emu = None
    if args.emulate_rank:  # rank er of en (with en's frame groups: rank er % (en / G) of a group's frames)
        er, en = (int(x) for x in args.emulate_rank.split("/"))
        eg = fg_arg if fg_arg is not None else default_frame_groups("strong", en)
        emu = sm.partition(args.disp, en // eg, er % (en // eg), split_views=args.shard == "vd")
        emu.update(rank=er, nranks=en, frame_groups=eg)
    if world == 1 or args.mode == "weak":
        Dloc = args.disp
        Dtot = Dloc * world if args.mode == "weak" else Dloc
        dbeg = rank * Dloc
    elif args.mode == "strong":
        # frame group fg of G (ranks [fg*Nf, (fg+1)*Nf)) shares frames fg, fg+G, ...; inside it the
        # rank's view / disparity share of those frames; reduce groups are contiguous blocks of gsize
        # ranks, so the global group id is rank // gsize
        Dtot = args.disp
        G = args.frame_groups
        nf = world // G
        fg, lr = divmod(rank, nf)
        part = sm.partition(Dtot, nf, lr, split_views=args.shard == "vd")
        dbeg, Dloc, views = part["d0"], part["D"], part["views"]
        gsize, grank = part["group_size"], part["group_rank"]
        group = fg * (nf // gsize) + part["group"]
    else:  # batch
        Dloc = Dtot = args.disp
        dbeg = 0
    Dtot_frame = Dloc if (args.mode == "batch" or world == 1) else Dtot
    if emu:  # one rank's share of an N-rank frame: its views and slices of the total range
        Dtot = Dtot_frame = args.disp
        dbeg, Dloc, views = emu["d0"], emu["D"], emu["views"]
    fgroups = args.frame_groups if (args.mode == "strong" and world > 1) else 1
    return dict(W=W, H=H, Dloc=Dloc, Dtot=Dtot, Dtot_frame=Dtot_frame, dbeg=dbeg, views=views, group=group, gsize=gsize,
                grank=grank, emu=emu, fgroups=fgroups, fgroup=rank // (world // fgroups))


def setup_comms(ctxs, world, rank, group, gsize, grank, mode, context_cls):
    """One communicator per context (its reduce runs on that context's stream) and reduce group: the
    group's rank 0 creates the unique id, every rank gathers all ids and joins its group leader's."""
    if world == 1 or mode == "batch":
        return
    for c in ctxs:
        ids = [None] * world
        dist.all_gather_object(ids, context_cls.unique_id() if grank == 0 else None)
        leader = next(r for r in range(world) if ids[r] is not None and (r // gsize if gsize < world else 0) == group)
        c.comm_init(gsize, grank, ids[leader])


class StubContext:
    """--plan-only: a context that records its communicator set-up (no GPU)."""
    _n = 0

    def __init__(self, rank):
        self.rank = rank
        self.comm = None

    @staticmethod
    def unique_id():
        StubContext._n += 1
        return ("uid-%d-%d" % (os.getpid(), StubContext._n)).encode().ljust(128, b"\0")

    def comm_init(self, nranks, rank, uid):
        self.comm = dict(nranks=nranks, rank=rank, uid=uid.rstrip(b"\0").decode())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--mode", default=None, choices=["strong", "weak", "batch"],
                    help="N>1 partitioning (default strong = BASELINE C4)")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--disp", type=int, default=None,
                    help="disparities: total (N=1, strong, batch) or per rank (weak); default per config")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host-io", action="store_true")
    ap.add_argument("--segment-c", type=float, default=float("inf"),
                    help="finite: segment mode (Stereo3DMST's c, e.g. 5000) instead of the MST")
    ap.add_argument("--min-size", type=int, default=200)
    ap.add_argument("--aggregator", default="tree", choices=["tree", "guided"],
                    help="cost aggregator: the MST/forest tree filter (default) or the colour guided filter")
    ap.add_argument("--shard", default="vd", choices=["vd", "d"],
                    help="strong mode partition: vd = view groups x disparity shards (even N: half the ranks per "
                         "view, D split inside each group), d = disparity shards of both views")
    ap.add_argument("--frame-groups", type=int, default=None,
                    help="strong mode: split the N ranks into G frame groups of N/G ranks; frames alternate "
                         "between the groups and each group view- and D-shards its frames with its own RCCL "
                         "min+argmin (default: 2 at N >= 8, else 1; 1 = every rank on every frame)")
    ap.add_argument("--emulate-rank", default=None, metavar="R/N",
                    help="one GPU runs rank R's share of an N-rank strong-mode frame (no collective): the per-rank "
                         "cost of the partition, for the multi-GPU estimate in DESIGN.md 7")
    ap.add_argument("--no-split", action="store_true",
                    help="A/B: stream frames with sm_match_async instead of sm_match_begin/finish")
    ap.add_argument("--inflight", type=int, default=0,
                    help="frames in flight (contexts on their own streams); 0 = 3, fewer where memory needs it")
    ap.add_argument("--lag", type=int, default=0,
                    help="frames whose tree is enqueued before the host waits for an earlier frame's layout "
                         "(stream_frames; 0 = 1 in MST mode, inflight - 2 in segment mode)")
    ap.add_argument("--plan-only", action="store_true",
                    help="CPU check: start the ranks, print each rank's share and communicator set-up (stub "
                         "contexts, no GPU), exit")
    ap.add_argument("--no-pms", action="store_true", help="skip the MST_PMS (SM_AGG_PMS) timing leg")
    ap.add_argument("--no-segment", action="store_true",
                    help="skip the segment-mode leg (Stereo3DMST's own forest, reported beside the MST metric)")
    ap.add_argument("--pms-iters", type=int, default=100,
                    help="MST_PMS calls per view in the PMS timing leg (the reference's 100, Stereo3DMST.cpp:854)")
    ap.add_argument("--dev", action="store_true",
                    help="allow SM_* environment variables (a dev library through SM_LIB, tools' A/B runs): the line "
                         "then records them and is marked headline: false")
    args = ap.parse_args()
    sm_env = sm_environment()
    if sm_env and not args.dev:
        # the product library reads no environment variable, but a dev build (SM_LIB) does, and its
        # experiment switches can skip work: a headline is never printed with any of them set
        print("bench.py: refusing to print a headline with SM_* variables set (%s); unset them, or pass --dev "
              "for a line marked headline: false" % ", ".join("%s=%s" % kv for kv in sorted(sm_env.items())),
              file=sys.stderr)
        sys.exit(2)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world), file=sys.stderr)
        sys.exit(2)
    if args.mode is None:
        args.mode = "strong" if world > 1 else "weak"
    big = args.mode == "batch"  # C5: 3840x2160 D=256 pairs
    if args.width is None:
        args.width = 3840 if big else 1920
    if args.height is None:
        args.height = 2160 if big else 1200
    if args.emulate_rank and world != 1:
        print("bench.py: --emulate-rank runs on one GPU without torchrun", file=sys.stderr)
        sys.exit(2)
    if args.disp is None:
        args.disp = 256 if (big or (args.mode == "strong" and world > 1) or args.emulate_rank) else 128
    fg_arg = args.frame_groups
    if args.frame_groups is None:
        args.frame_groups = default_frame_groups(args.mode, world)
    if args.mode == "strong" and (args.frame_groups < 1 or world % args.frame_groups):
        print("bench.py: --frame-groups must divide the rank count", file=sys.stderr)
        sys.exit(2)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    plan = rank_plan(args, world, rank, fg_arg)
    W, H = plan["W"], plan["H"]
    Dloc, Dtot, Dtot_frame, dbeg, views = plan["Dloc"], plan["Dtot"], plan["Dtot_frame"], plan["dbeg"], plan["views"]
    group, gsize, grank, emu = plan["group"], plan["gsize"], plan["grank"], plan["emu"]
    if args.plan_only:  # CPU: the rank's share and its communicator set-up against stub contexts
        ctxs = [StubContext(rank) for _ in range(2)]
        setup_comms(ctxs, world, rank, group, gsize, grank, args.mode, StubContext)
        print(json.dumps(dict(rank=rank, world=world, plan={k: v for k, v in plan.items() if k != "emu"},
                              comms=[c.comm for c in ctxs])), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    # frames in flight: each context is a full pipeline on its own stream; frame i goes to context
    # i % n, so frame i+1's prep / MST / layout overlaps frame i's tree filter on the GPU
    # context footprint (round 6, compact A rows): ~25 B per pixel and padded slice (A_up rows 16, both
    # views; compact A rows + cut-path rows ~5) + ~400 B per pixel (layout, MST); measured by
    # tools/mem_probe.py: 8.26 GB at C2, 53.4 GB at C3 (round 5: 20 B x 2 -> C3 held 2 frames, now 3)
    per_ctx_gb = W * H * (64 * (1 if Dloc <= 64 else 2 if Dloc <= 128 else 4)) * 25 / 1e9 + W * H * 400 / 1e9
    # segment mode: the segmentation's host steps give a frame ~17 ms of latency before its filter,
    # so it keeps more frames in flight (6) and begins lag = inflight - 2 frames ahead (stream_frames)
    seg_mode = math.isfinite(args.segment_c)
    depth = 6 if seg_mode else 3
    inflight = args.inflight if args.inflight > 0 else max(1, min(depth, int(200.0 // per_ctx_gb)))
    ctxs = [sm.Context(local) for _ in range(inflight)]
    setup_comms(ctxs, world, rank, group, gsize, grank, args.mode, sm.Context)
    pair_index = rank if args.mode == "batch" else 0
    left, right, _ = make_pair(W, H, Dtot_frame, index=pair_index)
    for c in ctxs:
        c.upload(left, right)
    params = sm.default_params(disp_begin=dbeg, disp_total=Dtot_frame, c=args.segment_c, min_size=args.min_size,
                               aggregator=sm.SM_AGG_GUIDED if args.aggregator == "guided" else sm.SM_AGG_TREE,
                               views=views)
    torch.cuda.set_device(local)
    ctx = ctxs[0]

    def barrier():
        if world > 1:
            dist.barrier()

    def accumulate(acc, c):
        for k, v in c.kernel_stats().items():
            a = acc.setdefault(k, dict(launches=0, ms=0.0, voxels=0.0, bytes_per_voxel=v["bytes_per_voxel"]))
            a["launches"] += v["launches"]
            a["ms"] += v["ms"]
            a["voxels"] += v["voxels"]

    for _ in range(max(args.warmup, 1)):
        for c in ctxs:
            c.match_async(Dloc, params)
            c.synchronize()
    # roofline kernel: the tree-filter family with the largest summed launch time.  Inside the
    # timed region only its launches carry HIP events (each event record costs GPU time between
    # launches: timing every family adds ~0.14 ms per C2 frame); the other families are timed
    # in a diagnostic pass after the timed region (kernels_ms_per_step, tree_filter)
    warm = {}
    accumulate(warm, ctx)
    dom = max(warm, key=lambda k: warm[k]["ms"])  # (guided aggregator: no tree families, all zero)
    for c in ctxs:
        c.set_kernel_timing([dom])
        c.synchronize()
    barrier()
    torch.cuda.synchronize()
    stage_acc = {}
    kacc = {}

    def retire(c):  # wait for context c's frame; its per-launch HIP-event timings are read here
        c.synchronize()
        for k, v in c.stage_times().items():
            stage_acc[k] = stage_acc.get(k, 0.0) + v
        accumulate(kacc, c)

    clk0 = (time.clock_gettime_ns(time.CLOCK_BOOTTIME), time.monotonic_ns())
    t0 = time.perf_counter()
    # frame groups: the timed region is args.steps frames of the stream; group fg takes frames fg, fg+G, ...
    my_steps = len(range(plan["fgroup"], args.steps, plan["fgroups"]))
    stream_frames(ctxs, my_steps, Dloc, params, retire, split=not args.no_split,
                  lag=args.lag if args.lag > 0 else (max(1, len(ctxs) - 2) if seg_mode else 1))
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    clk1 = (time.clock_gettime_ns(time.CLOCK_BOOTTIME), time.monotonic_ns())
    # the timed region's clock span on stderr: tools/timed_region.py picks this region's launches out of
    # a rocprofv3 kernel trace of the same command (its timestamps are one of these two clocks)
    print("# timed region rank %d boottime_ns %d %d monotonic_ns %d %d" % (rank, clk0[0], clk1[0], clk0[1], clk1[1]),
          file=sys.stderr, flush=True)
    # diagnostic pass, one frame at a time: every family timed (kernels_ms_per_step, tree_filter,
    # roofline.isolated) and the single-frame latency
    for c in ctxs:
        c.set_kernel_timing(None)
    diag_steps = 2
    kall = {}
    lat = []
    for _ in range(diag_steps):
        tl = time.perf_counter()
        ctx.match_async(Dloc, params)
        ctx.synchronize()
        lat.append((time.perf_counter() - tl) * 1e3)
        accumulate(kall, ctx)
    # the filter's wall clock, one frame at a time without per-launch events: stage events around
    # the up and down passes (walkers and chains run concurrently on two streams, so the sum of
    # launch times above counts the overlapped time twice)
    ctx.set_kernel_timing([])
    wall = []
    for _ in range(3):
        ctx.match_async(Dloc, params)
        ctx.synchronize()
        st = ctx.stage_times()
        wall.append(st["up_ms"] + st["down_ms"])
    filt_wall_ms = min(wall)
    # end to end with host buffers (sm_match: image upload + frame + result download over PCIe);
    # reported beside the resident-input value, never as it
    host_io = None
    if not args.no_host_io:
        ctx.match(left, right, Dloc, params)
        barrier()
        th = time.perf_counter()
        nh = 3
        for _ in range(nh):
            ctx.match(left, right, Dloc, params)
        barrier()
        host_ms = (time.perf_counter() - th) * 1e3 / nh
        host_io = {"ms_per_frame": host_ms, "value": W * H * Dtot_frame / (host_ms * 1e-3),
                   "what": "sm_match with host buffers: 2 x %d B images up, disp f32 + idx i32 + min f64 of both "
                           "views down (%d B), synchronous, %d frames" % (W * H * 3, W * H * 16 * 2, nh)}
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    ms_step = elapsed * 1e3 / args.steps
    units_per_step = W * H * (Dtot_frame * (world if args.mode == "batch" else 1))
    value = units_per_step * args.steps / elapsed
    # roofline: the tree-filter kernel family with the largest summed launch time; algorithmic
    # bytes = voxels it processed x SURVEY.md 8(d) bytes/voxel (DESIGN.md "Roofline accounting")
    d = kacc[dom]
    dom_bytes = d["voxels"] * d["bytes_per_voxel"]
    achieved = dom_bytes / (d["ms"] * 1e-3) / 1e9 if d["ms"] > 0 else 0.0
    di = kall[dom]
    iso_ms = di["ms"] / max(di["launches"], 1)
    iso_bytes = di["voxels"] * di["bytes_per_voxel"] / max(di["launches"], 1)
    filt_ms = sum(v["ms"] for v in kall.values()) / diag_steps  # per frame, diagnostic pass
    filt_bytes = sum(v["voxels"] * v["bytes_per_voxel"] for v in kall.values()) / diag_steps
    traffic = None
    traffic_src = None
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tf):
        try:
            with open(tf) as f:
                pj = json.load(f)
            fam = pj.get(dom, {})
            import hashlib
            with open(os.path.join(ROOT, "stereomatch_amd", "libstereomst.so"), "rb") as f:
                cur = hashlib.sha256(f.read()).hexdigest()[:16]
            built = pj.get("_build", "unrecorded")
            traffic_src = dict(file="profiles/pmc_traffic.json", build=built, this_build="libstereomst.so sha256:" + cur,
                               same_build=("sha256:" + cur) in built,
                               note="PMC HBM bytes from a separate rocprofv3 --pmc run (tools/pmc_traffic.py), "
                                    "not measured in this run")
            # PMC HBM bytes of the family per frame over the launches timed here (an empty bucket
            # launches nothing, so both count the same launches)
            if fam.get("hbm_bytes_per_frame") and d["launches"]:
                traffic = fam["hbm_bytes_per_frame"] / (d["launches"] / my_steps)
        except Exception:
            traffic = None
    line = {
        "metric": "cost-volume voxels/s (W*H*D per frame, both views) + ms/frame",
        "value": value,
        "unit": "voxels/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": None if world == 1 else ("weak" if args.mode in ("weak", "batch") else "strong"),
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded slanted-plane stereo pair, tools/synth.py)",
        "config": {"workload": "%dx%d D=%d both views%s%s" % (
                       W, H, Dtot_frame, CONFIG_NAMES.get((W, H, Dtot_frame), ""),
                       " = BASELINE C5's per-GPU pair" if args.mode == "batch" and (W, H, Dtot_frame) == (3840, 2160, 256) else "")
                   if world == 1 else
                   "%dx%d D=%d, %s mode, %s%s%s" % (
                       W, H, Dtot_frame, args.mode,
                       ("%d frame groups of %d ranks (frame i on group i mod %d), each frame: " % (
                           plan["fgroups"], world // plan["fgroups"], plan["fgroups"])) if plan["fgroups"] > 1 else "",
                       ("2 view groups x %d disparity shards of %d slices: each rank one view, %d slices" % (gsize, Dloc, Dloc))
                       if views != 3 else ("%d disparity shards of %d slices, both views per rank" % (
                           world // plan["fgroups"], Dloc))
                       if args.mode == "strong" else "%d disparities/rank, both views" % Dloc,
                       " (BASELINE C4 frame size; C4 names 32 disparities/GPU: here %s)" % (
                           "view groups" if views != 3 else "%d/GPU" % Dloc)
                       if (args.mode == "strong" and (W, H, Dtot_frame) == (1920, 1200, 256)) else
                       " (BASELINE C5: one pair per GPU)" if (args.mode == "batch" and (W, H, Dtot_frame) == (3840, 2160, 256))
                       else ""),
                   "W": W, "H": H, "D": Dtot_frame, "disparities_per_rank": Dloc,
                   "parallelism": "replicas" if args.mode == "batch" else
                   ("%d frame groups x (%s)" % (plan["fgroups"], "view2 x d-shard%d" % gsize if views != 3 else
                                                "d-shard%d" % (world // plan["fgroups"])) if plan["fgroups"] > 1 else
                    "view2 x d-shard%d" % gsize if views != 3 else "d-shard%d" % world),
                   "tree": "MST" if args.segment_c == float("inf") else "segment forest c=%g min_size=%d" % (
                       args.segment_c, args.min_size),
                   "aggregator": args.aggregator,
                   "frames_in_flight": inflight},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "launches_per_step": d["launches"] / my_steps,
                     "alg_bytes_per_launch": dom_bytes / max(d["launches"], 1),
                     "avg_launch_ms": d["ms"] / max(d["launches"], 1),
                     "timing": "HIP events on the launch stream around every %s launch of the timed region, "
                               "%d frames in flight (launches share the GPU with the other frames' work)" % (dom, inflight),
                     "isolated": {"avg_launch_ms": iso_ms, "achieved": iso_bytes / (iso_ms * 1e-3) / 1e9 if iso_ms > 0 else 0.0,
                                  "frac": iso_bytes / (iso_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if iso_ms > 0 else 0.0,
                                  "timing": "diagnostic pass, one frame at a time"},
                     "tree_filter": {"alg_bytes_per_step": filt_bytes, "ms_per_step": filt_ms,
                                     "achieved": filt_bytes / (filt_ms * 1e-3) / 1e9 if filt_ms > 0 else 0.0,
                                     "timing": "diagnostic pass of %d frames after the timed region, every launch timed, "
                                               "launch times summed" % diag_steps,
                                     "wall_ms_per_step": filt_wall_ms,
                                     "wall_achieved": filt_bytes / (filt_wall_ms * 1e-3) / 1e9 if filt_wall_ms > 0 else 0.0,
                                     "wall_frac": filt_bytes / (filt_wall_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if filt_wall_ms > 0 else 0.0,
                                     "wall_timing": "up + down pass spans (stage events), one frame at a time, no per-launch "
                                                    "events, best of 3"},
                     # the whole streamed frame against the same algorithmic bytes (SURVEY 8(d)'s north star:
                     # >= 40 % of HBM peak end to end)
                     "end_to_end": {"alg_bytes_per_step": filt_bytes, "ms_per_step": ms_step,
                                    "achieved": filt_bytes / (ms_step * 1e-3) / 1e9 if ms_step > 0 else 0.0,
                                    "frac": filt_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS if ms_step > 0 else 0.0,
                                    "timing": "the timed region's ms_per_step (frames in flight), all stages included"}},
        "kernels_ms_per_step": {k: v["ms"] / diag_steps for k, v in kall.items()},
        "stages_ms": {k: v / my_steps for k, v in stage_acc.items()},
        "latency_ms_per_frame": min(lat),
        "frames_in_flight": inflight,
        "host_io": host_io,
        "env": sm_env,
        "headline": not sm_env,
    }
    if emu:
        line["emulated_rank"] = dict(emu, note="one rank's share of an N-rank strong-mode frame on one GPU, no "
                                               "collective; value counts the rank's own voxels; with G frame groups "
                                               "the rank takes every G-th frame of the stream, so the stream's "
                                               "ms/frame is ms_per_step / G",
                                     stream_ms_per_frame=ms_step / emu["frame_groups"])
        line["value"] = W * H * Dloc * bin(views).count("1") * args.steps / elapsed
        line["config"]["workload"] = "rank %d/%d of %dx%d D=%d: views %d, slices [%d, %d)" % (
            emu["rank"], emu["nranks"], W, H, Dtot_frame, views, dbeg, dbeg + Dloc)
    if rank == 0 and world == 1 and not args.no_segment and not emu and not seg_mode and args.aggregator == "tree":
        # 6 frames in flight where they fit (the same ~200 GB budget as the main leg: a C3-size pair
        # needs ~85 GB per context, so the batch line's segment leg keeps 2)
        seg_inflight = max(1, min(6, int(200.0 // per_ctx_gb)))
        line["segment"] = segment_leg(ctxs, left, right, Dloc, max(args.steps, 12), args.warmup, inflight=seg_inflight)
    if rank == 0 and world == 1 and not args.no_cpu and not emu:
        line["cpu_baseline"] = cpu_baseline(W, H, Dtot_frame)
    if rank == 0 and world == 1 and not args.no_pms and not emu and args.aggregator == "tree":
        line["pms"] = pms_leg(ctx, left, right, Dtot_frame, max(2, args.pms_iters), not args.no_cpu)
    if rank == 0:
        print(json.dumps(line), flush=True)
    for c in ctxs:
        c.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
