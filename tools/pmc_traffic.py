"""Per-stage HBM traffic from rocprofv3 PMC passes -> profiles/pmc_traffic.json.

Usage (on the GPU box, after two separate counter passes of the same bench
command, one with --pmc FETCH_SIZE and one with --pmc WRITE_SIZE):

    python tools/pmc_traffic.py --fetch DIR_F --write DIR_W --dist zipf \
        --size BYTES --out gpurun_out/pmc_traffic.json

FETCH_SIZE / WRITE_SIZE are reported in KiB per dispatch. gfx950 correction
(MI355X_MICROARCH.md, HBM / rocprofv3 section): FETCH_SIZE counts exactly half
of the bytes of wide (16 B per lane) streaming reads. Our own calibration
(tools/microbench/mb_pmc_calib.hip, profiles/r01_pmc_calibration.json) shows
exactly 0.5x for three shapes: coalesced 16-B loads, 64 contiguous bytes per
lane, 64-byte chunks. The doubling is applied PER KERNEL, only to the kernels
whose HBM reads are those shapes (WIDE_READ below); the others (scan kernels,
the index builder's fix-up / select / subs passes, whose reads are 4- or 8-B
accesses of an uncalibrated shape) are reported as counted, and each stage
entry lists which kernels were corrected. WRITE_SIZE is exact for 16-B-per-lane
streaming stores and 4-B stores (calibrated) and is never corrected. The stage
figures are summed over the kernels of a stage and divided by the number of
launches of the stage's marker kernel, so they are per launch of the stage
like bench.py's `achieved`.
"""
import argparse
import csv
import json
import os
from collections import defaultdict

# stage -> (kernels of the stage, kernels that mark one launch of the stage)
# k_scan_* (count scans) are shared by the three-pass pack, the index builder and the index-less
# extract: they are attributed by launch order, to the stage of the kernel launched before them
# (SHARED below), not to a fixed stage.
SHARED = ("k_scan_reduce", "k_scan_tiles", "k_scan_apply")
STAGES = {
    "hist": (("k_hist16", "k_hist16_rng"), ("k_hist16", "k_hist16_rng")),
    "pack": (("k_pack_count", "k_range_dot", "k_range_scan", "k_pack_write", "k_pack_cold", "k_pack_fixed16",
              "k_pack_fixed16_blk"),
             ("k_pack_write", "k_pack_fixed16")),
    "decode": (("k_decode", "k_decode_fixed16", "k_decode_fixed16_blk"), ("k_decode", "k_decode_fixed16")),
    "index": (("k_idx_walk", "k_idx_fixed16", "k_sync_scan", "k_sync_scan2", "k_sync_iter", "k_sync_select",
               "k_sync_subs"),
              ("k_sync_subs", "k_idx_fixed16")),
    "extract": (("k_chain_walk", "k_chain_fix", "k_chain_fix_loop", "k_chain_meta", "k_chain_decode", "k_chain_tail"),
                ("k_chain_decode",)),
}


# kernels whose HBM reads are the calibrated wide shapes (FETCH_SIZE doubled)
WIDE_READ = ("k_hist16", "k_hist16_rng", "k_range_dot", "k_pack_count", "k_pack_write", "k_pack_cold", "k_pack_one",
             "k_pack_fixed16",
             "k_pack_fixed16_blk", "k_decode", "k_decode_fixed16", "k_decode_fixed16_blk", "k_idx_walk", "k_chain_walk",
             "k_chain_decode")


def _is(name, k):
    return k + "<" in name or k + "(" in name


def stage_of(name):
    for st, (keys, _) in STAGES.items():
        if any(_is(name, k) for k in keys):
            return st
    return None


def read_counter(d, counter):
    """Per stage: (corrected bytes, raw bytes, corrected kernel names), launches, and per stage and
    kernel (short name) the corrected bytes."""
    path = os.path.join(d, "run_counter_collection.csv")
    per = defaultdict(float)
    perk = defaultdict(lambda: defaultdict(float))
    raw = defaultdict(float)
    fixed = defaultdict(set)
    calls = defaultdict(set)
    with open(path) as f:
        rows = [r for r in csv.DictReader(f) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    last_stage = None
    for row in rows:
        if True:
            if any(_is(row["Kernel_Name"], k) for k in SHARED):
                st = last_stage  # a count scan belongs to the stage that launched it
            else:
                st = stage_of(row["Kernel_Name"])
                last_stage = st if st is not None else last_stage
            if st is None:
                continue
            v = float(row["Counter_Value"]) * 1024.0
            wide = counter == "FETCH_SIZE" and any(_is(row["Kernel_Name"], k) for k in WIDE_READ)
            per[st] += 2.0 * v if wide else v
            perk[st][short_name(row["Kernel_Name"])] += 2.0 * v if wide else v
            raw[st] += v
            if wide:
                fixed[st].update(k for k in WIDE_READ if _is(row["Kernel_Name"], k))
            if any(_is(row["Kernel_Name"], k) for k in STAGES[st][1]):
                calls[st].add(row["Dispatch_Id"])
    return per, raw, fixed, {k: len(v) for k, v in calls.items()}, perk


def short_name(name):
    """The kernel's name without namespace, template arguments and parameters."""
    n = name.split("(")[0].split("<")[0]
    return n.split("::")[-1].split(" ")[-1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--dist", required=True)
    ap.add_argument("--size", type=int, required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch, fraw, ffixed, fcalls, fk = read_counter(a.fetch, "FETCH_SIZE")
    write, _, _, wcalls, wk = read_counter(a.write, "WRITE_SIZE")
    res = json.load(open(a.out)) if os.path.exists(a.out) else {}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    try:
        bid = open(os.path.join(root, "huffman_amd", "lib", "BUILD_ID")).read().strip()
    except OSError:
        bid = None
    ent = {}
    for st in STAGES:
        if st not in fetch or st not in write:
            continue
        nf, nw = max(fcalls.get(st, 0), 1), max(wcalls.get(st, 0), 1)
        f = fetch[st] / nf
        w = write[st] / nw
        ent[st] = {
            "size": a.size,
            "fetch_bytes_per_launch": round(f),
            "write_bytes_per_launch": round(w),
            "hbm_bytes_per_launch": round(f + w),
            "dispatches": {"fetch_pass": fcalls.get(st, 0), "write_pass": wcalls.get(st, 0)},
            "fetch_size_raw_bytes_per_launch": round(fraw[st] / nf),
            "correction": "fetch = 2 x FETCH_SIZE for the kernels in fetch_doubled (gfx950 wide-read "
                          "undercount, calibrated shapes), FETCH_SIZE as counted for the rest; write = WRITE_SIZE",
            "fetch_doubled": sorted(ffixed[st]),
            "kernels": {k: {"fetch_bytes_per_launch": round(fk[st].get(k, 0.0) / nf),
                            "write_bytes_per_launch": round(wk[st].get(k, 0.0) / nw)}
                        for k in sorted(set(fk[st]) | set(wk[st]))},
            "build_id": bid,
        }
    res.setdefault(a.dist, {}).update(ent)  # a later pass (e.g. the extract-only run) replaces its stages
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({a.dist: ent}))


if __name__ == "__main__":
    main()
