"""Per-kernel-family HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE, run
separately as MI355X_MICROARCH.md "rocprofv3 PMC slots" requires) of `bench.py --steps S --warmup W`.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> <frames|auto> [out.json]
(auto: frames = dispatches of k_prep, one per frame, in the fetch pass)

FETCH_SIZE / WRITE_SIZE are read as KiB per dispatch.  On gfx950 FETCH_SIZE reports half the bytes
of a 16-B/lane streaming read (MI355X_MICROARCH.md "HBM"), so fetch bytes are doubled; the write
side is taken as reported.  k_median (reads and writes exactly 4 B per pixel per view) is reported
beside the families as a sanity check of the units on this box.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

FAMILIES = ["k_up_walk", "k_up_pre", "k_up_chain", "k_down_chain", "k_down_walk", "k_median"]



def frames_of(d):
    """Frames in a rocprofv3 counter-collection directory: k_prep runs once per frame."""
    n = 0
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].startswith("k_prep") and r.get("Dispatch_Id") not in seen:
                seen.add(r.get("Dispatch_Id"))
        n += len(seen)
    return n

def family(name):
    base = name.split("(")[0].replace("void ", "").split("<")[0].strip()
    return base if base in FAMILIES else None


def lib_build_id():
    """sha256 (16 hex) of the library the profiled run loaded, and the time of this summary."""
    import hashlib
    import time
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "stereomatch_amd", "libstereomst.so")
    try:
        with open(path, "rb") as f:
            h = hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        h = "missing"
    return "libstereomst.so sha256:%s %s" % (h, time.strftime("%Y-%m-%d %H:%M"))


def load(d, counter):
    files = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    tot = defaultdict(float)
    disp = defaultdict(set)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            fam = family(r["Kernel_Name"])
            if fam is None:
                continue
            tot[fam] += float(r["Counter_Value"]) * 1024.0
            disp[fam].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    return tot, {k: len(v) for k, v in disp.items()}


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    frames = int(sys.argv[3]) if sys.argv[3] != "auto" else frames_of(fdir)
    out = sys.argv[4] if len(sys.argv) > 4 else "profiles/pmc_traffic.json"
    fetch, nf = load(fdir, "FETCH_SIZE")
    write, nw = load(wdir, "WRITE_SIZE")
    res = {"_note": "HBM bytes per frame and per launch from rocprofv3 FETCH_SIZE (x2, gfx950 16-B/lane "
                    "correction) + WRITE_SIZE over %d frames; see tools/pmc_traffic.py" % frames,
           "_build": lib_build_id()}
    for fam in FAMILIES:
        if fam not in fetch and fam not in write:
            continue
        launches = max(nf.get(fam, 0), nw.get(fam, 0)) / frames
        fb = 2.0 * fetch.get(fam, 0.0) / frames
        wb = write.get(fam, 0.0) / frames
        res[fam] = {"fetch_bytes_per_frame": fb, "write_bytes_per_frame": wb, "hbm_bytes_per_frame": fb + wb,
                    "launches_per_frame": launches,
                    "hbm_bytes_per_launch": (fb + wb) / launches if launches else None,
                    "raw_fetch_kib_per_frame": fetch.get(fam, 0.0) / 1024.0 / frames}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
