#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: cost-volume voxels/s (W*H*D per frame = both views)
and ms/frame, 1920x1200 D=128 synthetic pair on one MI355X; D-sharded over N GPUs.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode weak|strong|batch]
    torchrun ... bench.py --gpus N ...   (one process per GPU, RCCL over xGMI)

One step = one frame: both views through the whole path with the images already in HBM
(median, weights, Boruvka MST, tree layout, leaf->root and root->leaf passes, WTA, and for
N>1 the RCCL min+argmin reduce).  Modes for N>1:
  weak   (default): each rank owns 128 disparities, total D = 128*N, one cross-rank reduce
  strong          : total D = 256 split over N ranks (BASELINE config C4)
  batch           : one independent pair per rank, no collective (config C5 shape)
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
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


def cpu_baseline(W, H, D, slices, threads):
    """Oracle (CPU restatement, reference order, fp64) on a bounded sample of the workload:
    the full MST build of both views + `slices` disparity slices of cost and tree filter,
    extrapolated to D slices.  Test infrastructure, used only as the reported baseline."""
    from oracle import oracle as O
    left, right, _ = make_pair(W, H, D, index=0)
    t0 = time.perf_counter()
    trees = [O.build_tree(left), O.build_tree(right)]
    t_tree = time.perf_counter() - t0
    d0 = D // 2 - slices // 2
    t0 = time.perf_counter()
    lv, rv = O.cost_agd(left, right, d0, d0 + slices)
    t_cost = time.perf_counter() - t0
    t0 = time.perf_counter()
    for t, vol in zip(trees, (lv, rv)):
        O.tree_filter(W, H, t, vol, d0, True, False, threads)
    t_filter = time.perf_counter() - t0
    frame = t_tree + (t_cost + t_filter) * (D / slices)
    return dict(value=W * H * D / frame, unit="voxels/s", cores=threads, kind="port",
                sample="full %dx%d frame: MST+layout of both views (1 thread) + %d of %d slices of AGD cost (1 thread) "
                       "and tree filter (%d threads, OpenMP over slices), extrapolated to D=%d; stage s: tree %.2f, "
                       "cost %.2f, filter %.2f; est. ms/frame %.0f" % (W, H, slices, D, threads, D, t_tree, t_cost,
                                                                      t_filter, frame * 1e3))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--mode", default="weak", choices=["weak", "strong", "batch"])
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1200)
    ap.add_argument("--disp", type=int, default=128, help="disparities per rank (weak) / total (strong: 256 default)")
    ap.add_argument("--cpu-slices", type=int, default=32)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        args.gpus = world
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    W, H = args.width, args.height
    if world == 1 or args.mode == "weak":
        Dloc = args.disp
        Dtot = Dloc * world if args.mode == "weak" else Dloc
        dbeg = rank * Dloc
    elif args.mode == "strong":
        Dtot = 256 if args.disp == 128 else args.disp
        dbeg, Dloc = sm.shard_range(Dtot, world, rank)
    else:  # batch
        Dloc = Dtot = args.disp
        dbeg = 0
    if args.mode == "batch" or world == 1:
        Dtot_frame = Dloc
    else:
        Dtot_frame = Dtot

    ctx = sm.Context(local)
    if world > 1 and args.mode != "batch":
        uid = [sm.Context.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ctx.comm_init(world, rank, uid[0])
    pair_index = rank if args.mode == "batch" else 0
    left, right, _ = make_pair(W, H, Dtot_frame, index=pair_index)
    ctx.upload(left, right)
    params = sm.default_params(disp_begin=dbeg, disp_total=Dtot_frame)
    torch.cuda.set_device(local)

    def barrier():
        if world > 1:
            dist.barrier()

    def accumulate(acc):
        for k, v in ctx.kernel_stats().items():
            a = acc.setdefault(k, dict(launches=0, ms=0.0, voxels=0.0, bytes_per_voxel=v["bytes_per_voxel"]))
            a["launches"] += v["launches"]
            a["ms"] += v["ms"]
            a["voxels"] += v["voxels"]

    for _ in range(args.warmup):
        ctx.match_async(Dloc, params)
        ctx.synchronize()
    if args.warmup == 0:  # one untimed call to find the dominant kernel family
        ctx.match_async(Dloc, params)
        ctx.synchronize()
    # roofline kernel: the tree-filter family with the largest summed launch time.  Inside the
    # timed region only its launches carry HIP events (each event record costs GPU time between
    # launches: timing every family adds ~0.14 ms per C2 frame); the other families are timed
    # in a diagnostic pass after the timed region (kernels_ms_per_step, tree_filter)
    warm = {}
    accumulate(warm)
    dom = max(warm, key=lambda k: warm[k]["ms"])
    ctx.set_kernel_timing([dom])
    barrier()
    ctx.synchronize()
    torch.cuda.synchronize()
    stage_acc = {}
    kacc = {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.match_async(Dloc, params)
        ctx.synchronize()  # per-step sync: the per-launch HIP-event timings are read here
        for k, v in ctx.stage_times().items():
            stage_acc[k] = stage_acc.get(k, 0.0) + v
        accumulate(kacc)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_kernel_timing(None)
    diag_steps = 2
    kall = {}
    for _ in range(diag_steps):
        ctx.match_async(Dloc, params)
        ctx.synchronize()
        accumulate(kall)
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
    filt_ms = sum(v["ms"] for v in kall.values()) / diag_steps  # per frame, diagnostic pass
    filt_bytes = sum(v["voxels"] * v["bytes_per_voxel"] for v in kall.values()) / diag_steps
    traffic = None
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tf):
        try:
            with open(tf) as f:
                fam = json.load(f).get(dom, {})
            # PMC HBM bytes of the family per frame over the launches timed here (an empty bucket
            # launches nothing, so both count the same launches)
            if fam.get("hbm_bytes_per_frame") and d["launches"]:
                traffic = fam["hbm_bytes_per_frame"] / (d["launches"] / args.steps)
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
        "scaling": "weak" if (args.mode in ("weak", "batch") or world == 1) else "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded slanted-plane stereo pair, tools/synth.py)",
        "config": {"workload": "%dx%d D=%d both views%s" % (W, H, Dtot_frame, CONFIG_NAMES.get((W, H, Dtot_frame), ""))
                   if world == 1 else
                   "%dx%d D=%d, %s mode, %d disparities/rank" % (W, H, Dtot_frame, args.mode, Dloc),
                   "W": W, "H": H, "D": Dtot_frame, "disparities_per_rank": Dloc,
                   "parallelism": "replicas" if args.mode == "batch" else "d-shard%d" % world},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "launches_per_step": d["launches"] / args.steps,
                     "alg_bytes_per_launch": dom_bytes / max(d["launches"], 1),
                     "avg_launch_ms": d["ms"] / max(d["launches"], 1),
                     "tree_filter": {"alg_bytes_per_step": filt_bytes, "ms_per_step": filt_ms,
                                     "achieved": filt_bytes / (filt_ms * 1e-3) / 1e9 if filt_ms > 0 else 0.0,
                                     "timing": "diagnostic pass of %d frames after the timed region, every launch timed" % diag_steps}},
        "kernels_ms_per_step": {k: v["ms"] / diag_steps for k, v in kall.items()},
        "stages_ms": {k: v / args.steps for k, v in stage_acc.items()},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        threads = min(16, os.cpu_count() or 1)
        line["cpu_baseline"] = cpu_baseline(W, H, Dtot_frame, args.cpu_slices, threads)
    if rank == 0:
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
