"""
Condense the rocprofv3 output of ``gpurun_prof.sh`` (under ``gpurun_out/``) into the per-round
files committed here:

* ``<round>_<cfg>_kernel_stats.csv`` -- rocprofv3 ``--kernel-trace --stats`` summary (as written by
  rocprofv3; kernel names shortened), graph-replay steps as benched;
* ``<round>_pmc.json`` -- per-launch HBM bytes of each config's dominant kernel from the two PMC
  passes (``--pmc FETCH_SIZE`` and ``--pmc WRITE_SIZE``, separate runs, eager steps), with
  FETCH_SIZE doubled: on gfx950 it reports half the bytes of a coalesced streaming read
  (MI355X_MICROARCH.md, HBM section; confirmed on our own kernels, whose algorithmic read bytes
  are known).

Usage: python profiles/summarize.py r01 [gpurun_out]
"""
from __future__ import annotations

import collections
import csv
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))

DOMINANT = {
    "c2": r"k_site_bcast",
    "c3": r"k_linear",
    "c5": r"mi_site_program|k_group_row",
}


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return name[:120]


def kernel_stats(raw: str, round_tag: str, cfg: str) -> None:
    src = os.path.join(raw, f"stats_{cfg}", "run_kernel_stats.csv")
    if not os.path.exists(src):
        return
    rows = list(csv.DictReader(open(src)))
    out = os.path.join(HERE, f"{round_tag}_{cfg}_kernel_stats.csv")
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs",
                    "MaxNs"])
        for r in rows:
            w.writerow([short(r["Name"]), r["Calls"], r["TotalDurationNs"],
                        f"{float(r['AverageNs']):.1f}", f"{float(r['Percentage']):.2f}",
                        r["MinNs"], r["MaxNs"]])


def counters(raw: str, kind: str, cfg: str):
    src = os.path.join(raw, f"{kind}_{cfg}", "run_counter_collection.csv")
    if not os.path.exists(src):
        return None
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(src)):
        per[(short(r["Kernel_Name"]), int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return per


def pmc(raw: str, round_tag: str) -> None:
    result = {}
    for cfg, pattern in DOMINANT.items():
        fetch = counters(raw, "fetch", cfg)
        write = counters(raw, "write", cfg)
        if fetch is None or write is None:
            continue
        # the dominant launch: matching name, largest grid
        keys = [k for k in fetch if re.search(pattern, k[0])]
        if not keys:
            continue
        key = max(keys, key=lambda k: k[1])
        f = fetch[key]
        wv = write.get(key, [])
        fetch_b = 2.0 * 1024.0 * sum(f) / len(f)            # KB -> B, x2 gfx950 correction
        write_b = 1024.0 * sum(wv) / len(wv) if wv else None
        result[cfg] = {
            "kernel": key[0], "grid_size": key[1], "launches": len(f),
            "fetch_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
            "traffic_bytes_per_launch": fetch_b + (write_b or 0.0),
            "raw_fetch_size_kb": sum(f) / len(f),
            "raw_write_size_kb": (sum(wv) / len(wv)) if wv else None,
        }
    with open(os.path.join(HERE, f"{round_tag}_pmc.json"), "w") as fh:
        json.dump(result, fh, indent=1)


def main() -> None:
    round_tag = sys.argv[1]
    raw = sys.argv[2] if len(sys.argv) > 2 else os.path.join(HERE, "..", "gpurun_out")
    for cfg in ("c2", "c3", "c4", "c5"):
        kernel_stats(raw, round_tag, cfg)
    pmc(raw, round_tag)


if __name__ == "__main__":
    main()
