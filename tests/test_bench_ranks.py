"""bench.py's multi-rank orchestration on the CPU: rank spawn (no torchrun), the gloo rendezvous, each
rank's share of the frame (stereomatch_amd.partition) and the per-context, per-view-group communicator
set-up (leader selection, unique ids), driven end to end through `bench.py --gpus N --plan-only` with
stub contexts in place of the GPU (bench.py spawn_ranks, rank_plan, setup_comms)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_plan(n, *extra):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--plan-only"] + list(extra),
                       capture_output=True, text=True, timeout=240, cwd=ROOT,
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1"))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert sorted(x["rank"] for x in lines) == list(range(n))
    return sorted(lines, key=lambda x: x["rank"])


def check_groups(lines, D):
    groups = {}
    for x in lines:
        p = x["plan"]
        groups.setdefault(p["group"], []).append(x)
    for g, members in groups.items():
        members.sort(key=lambda x: x["plan"]["grank"])
        size = members[0]["plan"]["gsize"]
        assert len(members) == size
        assert [m["plan"]["grank"] for m in members] == list(range(size))
        # ascending contiguous shards covering [0, D) of the group's views
        assert members[0]["plan"]["dbeg"] == 0
        for a, b in zip(members, members[1:]):
            assert a["plan"]["dbeg"] + a["plan"]["Dloc"] == b["plan"]["dbeg"]
        assert members[-1]["plan"]["dbeg"] + members[-1]["plan"]["Dloc"] == D
        assert len({m["plan"]["views"] for m in members}) == 1
        # one communicator per context: the same unique id across the group, distinct per context,
        # and every rank joins with the group size and its group rank
        for k in range(len(members[0]["comms"])):
            uids = {m["comms"][k]["uid"] for m in members}
            assert len(uids) == 1
            for m in members:
                assert m["comms"][k]["nranks"] == size and m["comms"][k]["rank"] == m["plan"]["grank"]
        assert len({c["uid"] for c in members[0]["comms"]}) == len(members[0]["comms"])
    return groups


@pytest.mark.parametrize("n", [2, 4])
def test_view_group_plan(n):
    """Strong mode, view groups (default): N = 4 splits into a left and a right group of 2 ranks
    each with 128 slices; N = 2 keeps both views (one view of 256 slices per rank is slower)."""
    lines = run_plan(n)
    groups = check_groups(lines, 256)
    if n == 4:
        assert len(groups) == 2
        assert {groups[g][0]["plan"]["views"] for g in groups} == {1, 2}
        uids = [groups[g][0]["comms"][0]["uid"] for g in groups]
        assert uids[0] != uids[1]  # each group its own communicator
    else:
        assert len(groups) == 1 and lines[0]["plan"]["views"] == 3


def test_disparity_shard_plan():
    lines = run_plan(4, "--shard", "d")
    groups = check_groups(lines, 256)
    assert len(groups) == 1 and all(x["plan"]["views"] == 3 and x["plan"]["Dloc"] == 64 for x in lines)


def test_weak_and_batch_plans():
    weak = run_plan(2, "--mode", "weak")
    assert [x["plan"]["dbeg"] for x in weak] == [0, 128] and all(x["plan"]["Dtot"] == 256 for x in weak)
    batch = run_plan(2, "--mode", "batch")
    assert all(x["comms"] == [None, None] for x in batch)  # replicas: no collective
    assert all((x["plan"]["W"], x["plan"]["H"], x["plan"]["Dloc"]) == (3840, 2160, 256) for x in batch)


def test_frame_group_plan():
    """N = 8 strong mode defaults to 2 frame groups of 4 ranks: each group is a left and a right view
    group of 2 ranks x 128 slices with its own communicators (4 reduce groups in all), and
    --frame-groups 1 keeps every rank on every frame (2 view groups of 4 x 64 slices)."""
    lines = run_plan(8)
    groups = check_groups(lines, 256)
    assert len(groups) == 4
    assert all(x["plan"]["fgroups"] == 2 and x["plan"]["fgroup"] == x["rank"] // 4 for x in lines)
    assert all(x["plan"]["gsize"] == 2 and x["plan"]["Dloc"] == 128 for x in lines)
    assert len({m["comms"][0]["uid"] for m in lines}) == 4
    for fg in (0, 1):
        assert sorted(x["plan"]["views"] for x in lines if x["plan"]["fgroup"] == fg) == [1, 1, 2, 2]
    one = run_plan(8, "--frame-groups", "1")
    groups = check_groups(one, 256)
    assert len(groups) == 2 and all(x["plan"]["Dloc"] == 64 and x["plan"]["fgroups"] == 1 for x in one)
