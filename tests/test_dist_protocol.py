"""World-size-2 gloo test of the D-sharded WTA exchange (sm_api.cpp stage_reduce).

Each rank filters its contiguous disparity shard (the oracle stands in for the per-rank GPU
result, which the -m gpu tests pin to it bit-exactly), then runs the library's two-step
exchange on CPU tensors with gloo: all-reduce MIN of the fp64 minimum cost, candidate = own
global index where the rank's cost equals the global minimum (else INT_MAX, as k_cand), and
all-reduce MIN of the candidates.  Every rank must then hold exactly the unsharded strict-<
first minimum (PatchMatchStereoGPU.cu:1700-1717, Stereo3DMST.cpp:177)."""
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


def _exchange(minc, idx):
    """The library's cross-rank reduce (sm_api.cpp stage_reduce + k_cand + k_finalize)."""
    gmin = torch.from_numpy(minc.copy())
    dist.all_reduce(gmin, op=dist.ReduceOp.MIN)
    cand = torch.where(torch.from_numpy(minc) == gmin, torch.from_numpy(idx), torch.tensor(0x7FFFFFFF, dtype=torch.int32))
    dist.all_reduce(cand, op=dist.ReduceOp.MIN)
    return gmin.numpy(), cand.numpy()


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
