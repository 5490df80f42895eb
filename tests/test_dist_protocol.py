"""gloo tests (world sizes 2-4) of the D-sharded WTA exchange (sm_api.cpp stage_reduce).

Each rank filters its contiguous disparity shard (the oracle stands in for the per-rank GPU
result, which the -m gpu tests pin to it bit-exactly), then runs the library's two-step
exchange with gloo in place of RCCL: all-reduce MIN of the fp64 minimum cost, the library's own
candidate rule (sm_reduce_candidates: the host form of k_cand / k_cand64, sm_reduce_rule.h), an
all-reduce MIN of the candidates, and the library's finalize (sm_reduce_finalize).  Every rank must
then hold exactly the unsharded strict-< first minimum (PatchMatchStereoGPU.cu:1700-1717,
Stereo3DMST.cpp:177)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _exchange(minc, idx, group=None, disp=None):
    """The library's cross-rank reduce (sm_api.cpp stage_reduce) with gloo in place of RCCL: MIN of the
    minima, the library's candidate rule, MIN of the candidates, the library's finalize.  uint64
    candidates (subpixel) are reduced as int64 with the top bit flipped (an order-preserving map: gloo
    has no unsigned MIN; RCCL reduces ncclUint64)."""
    from stereomatch_amd import _lib as L
    sub = disp is not None
    gmin = torch.from_numpy(minc.copy())
    dist.all_reduce(gmin, op=dist.ReduceOp.MIN, group=group)
    cand = L.reduce_candidates(minc, gmin.numpy(), idx, disp, sub)
    if sub:
        c = torch.from_numpy((cand ^ np.uint64(1 << 63)).view(np.int64).copy())
        dist.all_reduce(c, op=dist.ReduceOp.MIN, group=group)
        gc = c.numpy().view(np.uint64) ^ np.uint64(1 << 63)
    else:
        c = torch.from_numpy(cand.copy())
        dist.all_reduce(c, op=dist.ReduceOp.MIN, group=group)
        gc = c.numpy()
    m, i, d = L.reduce_finalize(gmin.numpy(), gc, sub)
    return (m, i, d) if sub else (m, i)


def _worker(rank, world, port, W, H, D, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from stereomatch_amd import shard_range
        from tools.synth import make_pair
        left, right, _ = make_pair(W, H, D, index=7)
        d0, Dl = shard_range(D, world, rank)
        res = {}
        for v, img in (("left", left), ("right", right)):
            tree = O.build_tree(img)
            lv, rv = O.cost_agd(left, right, d0, d0 + Dl)
            tf = O.tree_filter(W, H, tree, lv if v == "left" else rv, d0, True, False, 2)
            gmin, gidx = _exchange(tf["minc"], tf["idx"])
            res[v] = (gmin, gidx)
        out_q.put((rank, {v: (a.tolist(), b.tolist()) for v, (a, b) in res.items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("W,H,D,world", [(48, 32, 24, 2), (33, 21, 7, 2), (40, 24, 19, 3)])
def test_sharded_wta_exchange_equals_unsharded(W, H, D, world):
    from oracle import oracle as O
    from tools.synth import make_pair
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, D, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    left, right, _ = make_pair(W, H, D, index=7)
    ref = O.match(left, right, D, nthreads=2)
    for r in range(world):
        for v in ("left", "right"):
            gmin, gidx = got[r][v]
            np.testing.assert_array_equal(np.array(gidx, np.int32), ref[v]["idx"])
            np.testing.assert_array_equal(np.array(gmin, np.float64), ref[v]["minc"])


def test_shard_range_partitions():
    from stereomatch_amd import shard_range
    for Dt in (8, 100, 256):
        for G in (1, 2, 3, 8):
            rs = [shard_range(Dt, G, g) for g in range(G)]
            assert rs[0][0] == 0 and sum(n for _, n in rs) == Dt
            assert all(rs[i][0] + rs[i][1] == rs[i + 1][0] for i in range(G - 1))
    with pytest.raises(ValueError):
        shard_range(4, 8, 0)


def _worker_vd(rank, world, port, W, H, D, out_q):
    """View groups x disparity shards (stereomatch_amd.partition, bench.py --shard vd): the rank
    filters its view's shard and the reduce runs inside its view group only."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from stereomatch_amd import partition
        from tools.synth import make_pair
        left, right, _ = make_pair(W, H, D, index=7)
        part = partition(D, world, rank)
        half = part["group_size"]
        groups = [dist.new_group(list(range(g * half, (g + 1) * half))) for g in range(world // half)]
        grp = groups[part["group"]]
        v = "left" if part["views"] == 1 else "right"
        d0, Dl = part["d0"], part["D"]
        tree = O.build_tree(left if v == "left" else right)
        lv, rv = O.cost_agd(left, right, d0, d0 + Dl)
        tf = O.tree_filter(W, H, tree, lv if v == "left" else rv, d0, True, False, 2)
        gmin, gidx = _exchange(tf["minc"], tf["idx"], group=grp)
        out_q.put((rank, (v, gmin.tolist(), gidx.tolist())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("W,H,D,world", [(40, 24, 19, 2), (36, 20, 13, 4)])
def test_view_group_partition_equals_unsharded(W, H, D, world):
    from oracle import oracle as O
    from tools.synth import make_pair
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_vd, args=(r, world, port, W, H, D, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    left, right, _ = make_pair(W, H, D, index=7)
    ref = O.match(left, right, D, nthreads=2)
    seen = set()
    for r in range(world):
        v, gmin, gidx = got[r]
        seen.add(v)
        np.testing.assert_array_equal(np.array(gidx, np.int32), ref[v]["idx"])
        np.testing.assert_array_equal(np.array(gmin, np.float64), ref[v]["minc"])
    assert seen == {"left", "right"}


def test_partition_plans():
    from stereomatch_amd import partition
    # even N: two view groups, each covering the full range in ascending shards
    for Dt, N in ((256, 8), (256, 4), (128, 2), (100, 4), (7, 6)):
        parts = [partition(Dt, N, r) for r in range(N)]
        for g, mask in ((0, 1), (1, 2)):
            mine = [p for p in parts if p["group"] == g]
            assert len(mine) == N // 2 and all(p["views"] == mask for p in mine)
            assert sum(p["D"] for p in mine) == Dt and mine[0]["d0"] == 0
            assert [p["group_rank"] for p in mine] == list(range(N // 2))
    # odd N or split_views=False: both views, D over all ranks
    for N in (1, 3):
        parts = [partition(12, N, r) for r in range(N)]
        assert all(p["views"] == 3 and p["group_size"] == N for p in parts)
    assert partition(256, 8, 5, split_views=False) == dict(views=3, d0=160, D=32, group=0, group_size=8, group_rank=5)
    # one view of more than 128 slices per rank: both views instead (N = 2 at D = 256)
    assert [partition(256, 2, r)["views"] for r in range(2)] == [3, 3]


def _worker_sub(rank, world, port, W, H, D, out_q):
    """Subpixel exchange: each rank's winner carries its disparity (here d - 0.25 * (d % 3), a stand-in
    for the parabola); the lowest index among the ranks holding the minimum must bring its own."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from stereomatch_amd import shard_range
        from tools.synth import make_pair
        left, right, _ = make_pair(W, H, D, index=9)
        d0, Dl = shard_range(D, world, rank)
        tree = O.build_tree(left)
        lv, _ = O.cost_agd(left, right, d0, d0 + Dl)
        tf = O.tree_filter(W, H, tree, lv, d0, True, False, 2)
        disp = (tf["idx"] - 0.25 * (tf["idx"] % 3)).astype(np.float32)
        m, i, d = _exchange(tf["minc"], tf["idx"], disp=disp)
        out_q.put((rank, (m.tolist(), i.tolist(), d.tolist())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_subpixel_exchange_equals_unsharded(world):
    from oracle import oracle as O
    from tools.synth import make_pair
    W, H, D = 36, 22, 17
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_sub, args=(r, world, port, W, H, D, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    left, right, _ = make_pair(W, H, D, index=9)
    tree = O.build_tree(left)
    lv, _ = O.cost_agd(left, right, 0, D)
    ref = O.tree_filter(W, H, tree, lv, 0, True, False, 2)
    rdisp = (ref["idx"] - 0.25 * (ref["idx"] % 3)).astype(np.float32)
    for r in range(world):
        m, i, d = got[r]
        np.testing.assert_array_equal(np.array(i, np.int32), ref["idx"])
        np.testing.assert_array_equal(np.array(m, np.float64), ref["minc"])
        np.testing.assert_array_equal(np.array(d, np.float32), rdisp)
