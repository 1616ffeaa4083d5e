"""Summarise rocprofv3 PMC passes (tools/pmc_passes.sh output) per kernel.

    python tools/pmc_summary.py gpurun_out/pmc2 [--out profiles/pmc_summary.json]

Per kernel: mean counter values per dispatch, plus derived figures:
  hbm_bytes_per_launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024
      (MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reads half the bytes of a wide
       coalesced read stream, so it is doubled; WRITE_SIZE is exact for 16-B stores;
       both are in KiB)
  mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)
  clock_ghz = GRBM_GUI_ACTIVE / 8 / kernel time
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
from pathlib import Path


def load(root):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{root}/pass*/**/*_counter_collection.csv", recursive=True)):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
            if row["Counter_Name"] in ("GRBM_GUI_ACTIVE",):
                dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    return vals, dur


def short(name):
    if "k_gp_tile" in name:
        if "false" in name:
            return "obs_gemm"
        # the dynamics GP's narrow (de-duplicated rows, 16x256: MT 1) and wide images
        return "dyn_gemm_narrow" if ", 1, 4>" in name else "dyn_gemm"
    return name.split("(")[0].split("::")[-1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--out", default=None)
    ap.add_argument("--commit", default=None, help="commit of the build the passes measured")
    ap.add_argument("--command", default=None, help="the profiled command")
    ap.add_argument("--merge", default=None, help="existing summary to add this one to, under --key")
    ap.add_argument("--key", default=None, help="e.g. config3: stored as <key>_obs_gemm_hbm_bytes_per_launch")
    a = ap.parse_args()
    vals, dur = load(a.root)
    out = {"source": str(a.root), "commit": a.commit, "command": a.command, "kernels": {}}
    for k, d in vals.items():
        if "rocclr" in k:
            continue
        m = {c: sum(v) / len(v) for c, v in d.items()}
        rec = {"name": k, "counters": m}
        if "FETCH_SIZE" in m or "WRITE_SIZE" in m:
            rec["hbm_bytes_per_launch"] = 2 * m.get("FETCH_SIZE", 0.0) * 1024 + m.get("WRITE_SIZE", 0.0) * 1024
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
            rec["mfma_util"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)
        if dur.get(k) and "GRBM_GUI_ACTIVE" in m:
            t = sum(dur[k]) / len(dur[k])
            rec["kernel_ms_profiled"] = t * 1e3
            rec["clock_ghz"] = m["GRBM_GUI_ACTIVE"] / 8 / t / 1e9
        if "SQ_INSTS_MFMA" in m and "SQ_INSTS_VALU" in m:
            rec["valu_per_mfma"] = (m["SQ_INSTS_VALU"] - m["SQ_INSTS_MFMA"]) / max(m["SQ_INSTS_MFMA"], 1)
        if "SQ_WAVE_CYCLES" in m:
            wc = m["SQ_WAVE_CYCLES"]
            rec["wave_cycle_split"] = {x: m.get(x, 0) / wc for x in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY")}
        if "TCC_HIT_sum" in m:
            rec["l2_hit_rate"] = m["TCC_HIT_sum"] / max(m["TCC_HIT_sum"] + m["TCC_MISS_sum"], 1)
        out["kernels"][short(k)] = rec
    obs = out["kernels"].get("obs_gemm", {})
    out["obs_gemm_hbm_bytes_per_launch"] = obs.get("hbm_bytes_per_launch")
    if a.merge and a.key:
        base = json.loads(Path(a.merge).read_text())
        base[a.key] = out
        base[f"{a.key}_obs_gemm_hbm_bytes_per_launch"] = out["obs_gemm_hbm_bytes_per_launch"]
        out = base
    text = json.dumps(out, indent=1)
    if a.out:
        Path(a.out).write_text(text)
    for k, r in out["kernels"].items():
        extra = {x: r[x] for x in ("hbm_bytes_per_launch", "mfma_util", "clock_ghz", "valu_per_mfma",
                                   "wave_cycle_split", "l2_hit_rate") if x in r}
        print(k, json.dumps(extra))


if __name__ == "__main__":
    main()
