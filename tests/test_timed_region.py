"""tools/timed_region.py: the launches a kernel trace holds inside bench.py's timed region (the stderr line
"# timed region rank 0 boottime_ns A B monotonic_ns C D") are the ones averaged, on whichever clock the
trace's timestamps use.  Synthetic trace, CPU only."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trace(path, launches):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kind", "Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for name, t0, t1 in launches:
            w.writerow(["KERNEL_DISPATCH", name, t0, t1])


def _run(tmp_path, launches, log_line):
    tr, lg = tmp_path / "trace.csv", tmp_path / "bench.log"
    _trace(tr, launches)
    lg.write_text("noise\n" + log_line + "\n{\"metric\": 1}\n")
    return subprocess.run([sys.executable, os.path.join(ROOT, "tools", "timed_region.py"), str(tr), str(lg), "k_up_walk"],
                          capture_output=True, text=True)


def test_picks_the_region_on_the_boottime_clock(tmp_path):
    walk = "void k_up_walk<2, 3, false>(WalkView, WalkView)"
    launches = [(walk, 100, 1100), (walk, 5000, 5200), (walk, 6000, 6400), (walk, 9000, 12000),
                ("k_meta(LayoutPair, int, int)", 5100, 5150)]
    r = _run(tmp_path, launches, "# timed region rank 0 boottime_ns 4000 8000 monotonic_ns 1 2")
    assert r.returncode == 0, r.stderr
    line = [l for l in r.stdout.splitlines() if l.startswith("k_up_walk")][0]
    assert "2 launches, avg     0.3 us" in line  # (200 + 400) / 2 ns
    assert "whole run:    4 launches" in line
    assert "boottime clock" in r.stdout


def test_falls_back_to_the_monotonic_clock(tmp_path):
    walk = "void k_up_walk<2, 3, false>(WalkView, WalkView)"
    r = _run(tmp_path, [(walk, 50, 150), (walk, 300, 1300)],
             "# timed region rank 0 boottime_ns 10000 20000 monotonic_ns 200 2000")
    assert r.returncode == 0, r.stderr
    assert "monotonic clock" in r.stdout
    assert "1 launches, avg     1.0 us" in r.stdout


def test_no_region_line_is_an_error(tmp_path):
    r = _run(tmp_path, [("k_up_walk", 1, 2)], "no marker here")
    assert r.returncode != 0
