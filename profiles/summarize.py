"""
Condense the rocprofv3 output of ``gpurun_prof.sh`` (under ``gpurun_out/``) into the per-round
files committed here:

* ``<round>_<cfg>_kernel_stats.csv`` -- rocprofv3 ``--kernel-trace --stats`` summary (as written by
  rocprofv3; kernel names shortened), graph-replay steps as benched;
* ``<round>_pmc.json`` -- per-launch HBM bytes of each config's dominant kernel (and of the step's
  other large kernels, under ``"others"``) from the two PMC passes (``--pmc FETCH_SIZE`` and
  ``--pmc WRITE_SIZE``, separate runs, eager steps), with FETCH_SIZE doubled for vector-memory
  kernels: on gfx950 it reports half the bytes of a coalesced streaming read (MI355X_MICROARCH.md,
  HBM section; confirmed on our own kernels, whose algorithmic read bytes are known, see
  DESIGN.md). The C2 site kernel reads its data through the scalar unit (64-byte s_load), which
  FETCH_SIZE counts in full (4 MB of x -> 4.33 MB raw): no doubling there.
* ``<round>_valu_pmc.json`` -- where the waves' cycles go (``SQ_WAVE_CYCLES`` split into
  ``SQ_ACTIVE_INST_ANY`` / ``SQ_WAIT_ANY`` / ``SQ_WAIT_INST_ANY``, from r03) and issue counters of the VALU-bound kernels (``SQ_INSTS_VALU`` and its
  per-type split, ``GRBM_GUI_ACTIVE``), with the VALU pipe's busy fraction from measured issue
  costs (tools/valu_peak.hip: 2 cycles per wave64 instruction, 4 for v_pk_fma_f32, 8 for a
  transcendental, 6 for v_mad_u64_u32).

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
    "c4": r"k_linear",
    "c5": r"mi_site_program|k_group_row",
}
# raw FETCH_SIZE -> bytes: 2 for vector-memory streaming (the gfx950 correction), 1 for the
# scalar-load C2 kernel (calibrated against its 4 MB of data)
FETCH_SCALE = {"c2": 1.0}
# C5 (VERDICT r03 "What's weak" 3): the fused-draw program's scale is calibrated, not assumed --
# fetch_c5cal / write_c5cal run it at K = 64 (one particle block: every element's inputs read
# exactly once) and the known input bytes divided by the raw FETCH_SIZE give the factor:
# y, b, the guide's loc and unconstrained scale (4 B each) and the shared mask (1 B), n = 1e6.
C5_CAL_BYTES = 1_000_000 * (4 + 4 + 4 + 4 + 1)
# C3 / C4 ("Next round" 2): the linear site kernel's scale from a K = 32 run of C3
# (fetch_c3cal: one particle tile, so X [1e6, 32] and y [1e6] are each read exactly once)
C3_CAL_BYTES = 1_000_000 * (32 * 4 + 4)
OTHERS = r"k_elbo_forward|k_elbo_backward|k_adam_step|k_minibatch_rows|k_finalize"


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


def per_launch(values):
    """Mean over the replayed launches: the second half of a run's launches (the first are the
    eager warm-up steps and the capture's)."""
    if not values:
        return None
    tail = values[len(values) // 2:] if len(values) >= 4 else values
    return sum(tail) / len(tail)


def c5_calibration(raw: str):
    """(scale, raw KB) of the C5 program's FETCH_SIZE from its K = 64 run, or None."""
    fetch = counters(raw, "fetch", "c5cal")
    if not fetch:
        return None
    keys = [k for k in fetch if re.search(DOMINANT["c5"], k[0])]
    if not keys:
        return None
    kb = per_launch(fetch[max(keys, key=lambda k: k[1])])
    return C5_CAL_BYTES / (1024.0 * kb), kb


C4_CAL_BYTES = 65536 * (32 * 4 + 4)


def c4_calibration(raw: str):
    """(scale, raw KB) of the one-stage linear kernel's FETCH_SIZE from C4's own run, or None."""
    fetch = counters(raw, "fetch", "c4")
    if not fetch:
        return None
    keys = [k for k in fetch if re.search(DOMINANT["c4"], k[0])]
    if not keys:
        return None
    kb = per_launch(fetch[max(keys, key=lambda k: k[1])])
    return C4_CAL_BYTES / (1024.0 * kb), kb


def c3_calibration(raw: str):
    """(scale, raw KB) of the linear kernel's FETCH_SIZE from C3's K = 32 run, or None."""
    fetch = counters(raw, "fetch", "c3cal")
    if not fetch:
        return None
    keys = [k for k in fetch if re.search(DOMINANT["c3"], k[0])]
    if not keys:
        return None
    kb = per_launch(fetch[max(keys, key=lambda k: k[1])])
    return C3_CAL_BYTES / (1024.0 * kb), kb


def replay_durations(raw: str, round_tag: str) -> None:
    """Average duration of each config's dominant kernel over the graph-replayed launches of the
    stats run (the second half of its launches: the first are eager warm-up steps), next to the
    bench line's span-stamp kernel_ms -- <round>_kernel_replay.json."""
    out = {}
    for cfg, pattern in DOMINANT.items():
        src = os.path.join(raw, f"stats_{cfg}", "run_kernel_trace.csv")
        if not os.path.exists(src):
            continue
        # (C2: not the reducible-floor variant of the site kernel, SUFF = true)
        rows = [r for r in csv.DictReader(open(src)) if re.search(pattern, r["Kernel_Name"]) and
                not (cfg == "c2" and "true>" in short(r["Kernel_Name"])[-8:])]
        if not rows:
            continue
        grid = max(int(r.get("Grid_Size", 0) or 0) for r in rows)
        rows = [r for r in rows if int(r.get("Grid_Size", 0) or 0) == grid]
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
        tail = d[len(d) // 2:]
        out[cfg] = {"kernel": short(rows[0]["Kernel_Name"]), "grid_size": grid, "launches": len(d),
                    "replay_launches": len(tail), "replay_avg_us": sum(tail) / len(tail),
                    "replay_min_us": min(tail), "replay_max_us": max(tail),
                    "all_avg_us": sum(d) / len(d)}
    with open(os.path.join(HERE, f"{round_tag}_kernel_replay.json"), "w") as fh:
        json.dump(out, fh, indent=1)


def pmc(raw: str, round_tag: str) -> None:
    result = {}
    cal3 = c3_calibration(raw)
    if cal3 is not None:
        FETCH_SCALE["c3"] = cal3[0]
        result["c3_calibration"] = {
            "known_input_bytes": C3_CAL_BYTES, "raw_fetch_size_kb_at_k32": cal3[1],
            "fetch_scale": cal3[0],
            "note": "C3 at K = 32: one particle tile, X and y read once (contiguous rows)"}
    cal4 = c4_calibration(raw)
    if cal4 is not None:
        FETCH_SCALE["c4"] = cal4[0]
        result["c4_calibration"] = {
            "known_input_bytes": C4_CAL_BYTES, "raw_fetch_size_kb": cal4[1], "fetch_scale": cal4[0],
            "note": "C4 as benched (K = 32, one particle group): every gathered row of X and y is "
                    "read by exactly one workgroup, so the known input is the batch's 65536 rows; "
                    "the raw count is about that (random 128-byte row gathers are counted in full, "
                    "unlike C3's streamed rows), hence a scale near 1 -- C3's 1.79 does not apply"}
    cal = c5_calibration(raw)
    if cal is not None:
        FETCH_SCALE["c5"] = cal[0]
        result["c5_calibration"] = {
            "known_input_bytes": C5_CAL_BYTES, "raw_fetch_size_kb_at_k64": cal[1],
            "fetch_scale": cal[0],
            "note": "K = 64: one particle block, each element's inputs read once"}
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
        scale = FETCH_SCALE.get(cfg, 2.0)

        def entry(k, fetch_scale):
            f, wv = per_launch(fetch.get(k, [])), per_launch(write.get(k, []))
            fetch_b = fetch_scale * 1024.0 * f if f is not None else None
            write_b = 1024.0 * wv if wv is not None else None
            return {"kernel": k[0], "grid_size": k[1], "launches": len(fetch.get(k, [])),
                    "fetch_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
                    "traffic_bytes_per_launch": (fetch_b or 0.0) + (write_b or 0.0),
                    "raw_fetch_size_kb": f, "raw_write_size_kb": wv,
                    "fetch_scale": fetch_scale}
        result[cfg] = entry(key, scale)
        result[cfg]["others"] = [entry(k, 2.0) for k in sorted(fetch)
                                 if k != key and re.search(OTHERS, k[0])]
    with open(os.path.join(HERE, f"{round_tag}_pmc.json"), "w") as fh:
        json.dump(result, fh, indent=1)


# issue cost in SIMD cycles per wave64 instruction (tools/valu_peak.hip on MI355X)
COST = {"plain": 2.0, "pk_fma": 4.0, "trans": 8.0, "int64": 6.0}
SIMDS = 1024
XCDS = 8


def valu(raw: str, round_tag: str) -> None:
    result = {}
    for cfg, pattern in DOMINANT.items():
        per = {}
        for kind in ("valu", "vtype", "wait"):
            src = os.path.join(raw, f"{kind}_{cfg}", "run_counter_collection.csv")
            if not os.path.exists(src):
                continue
            rows = [r for r in csv.DictReader(open(src)) if re.search(pattern, r["Kernel_Name"])]
            if not rows:
                continue
            grid = max(int(r["Grid_Size"]) for r in rows)
            acc = collections.defaultdict(list)
            dur = {}
            for r in rows:
                if int(r["Grid_Size"]) != grid:
                    continue
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
                dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            per.update({n: sum(v) / len(v) for n, v in acc.items()})
            per["kernel"] = short(rows[0]["Kernel_Name"])
            per[f"{kind}_us"] = sum(dur.values()) / len(dur) / 1e3
        if "SQ_INSTS_VALU" not in per or "GRBM_GUI_ACTIVE" not in per:
            continue
        cycles = per["GRBM_GUI_ACTIVE"] / XCDS
        us = per.get("vtype_us") or per.get("valu_us") or per.get("wait_us")
        per["clock_ghz"] = cycles / (us * 1e3)
        if "SQ_INSTS_VALU_TRANS_F32" in per:
            trans = per["SQ_INSTS_VALU_TRANS_F32"]
            int64 = per.get("SQ_INSTS_VALU_INT64", 0.0)
            fma = per.get("SQ_INSTS_VALU_FMA_F32", 0.0)
            # the C2 kernel's FMAs are packed (v_pk_fma_f32, 4 cycles); elsewhere scalar
            pk = fma if cfg == "c2" else 0.0
            plain = per["SQ_INSTS_VALU"] - trans - int64 - pk
            busy = (plain * COST["plain"] + pk * COST["pk_fma"] + trans * COST["trans"] +
                    int64 * COST["int64"])
            per["valu_issue_cycles"] = busy
            per["valu_busy"] = busy / (SIMDS * cycles)
        if "SQ_WAVE_CYCLES" in per and per["SQ_WAVE_CYCLES"]:
            # where the waves' cycles go (disjoint: issuing, parked on s_waitcnt / barriers,
            # ready but issue-stalled on a dependency or a busy pipe; MI355X_MICROARCH.md)
            wc = per["SQ_WAVE_CYCLES"]
            for name in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
                if name in per:
                    per[name.lower() + "_frac"] = per[name] / wc
        if "SQ_VALU_MFMA_BUSY_CYCLES" in per:
            per["mfma_busy"] = per["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cycles)
        result[cfg] = per
    with open(os.path.join(HERE, f"{round_tag}_valu_pmc.json"), "w") as fh:
        json.dump(result, fh, indent=1)


def main() -> None:
    round_tag = sys.argv[1]
    raw = sys.argv[2] if len(sys.argv) > 2 else os.path.join(HERE, "..", "gpurun_out")
    for cfg in ("c2", "c3", "c4", "c5"):
        kernel_stats(raw, round_tag, cfg)
    replay_durations(raw, round_tag)
    pmc(raw, round_tag)
    valu(raw, round_tag)


if __name__ == "__main__":
    main()
