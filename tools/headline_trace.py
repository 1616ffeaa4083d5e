"""Headline-only kernel-trace summary: the observation-tile launches of bench.py's timed loop.

    rocprofv3 --kernel-trace --output-format csv -d <dir> -- python bench.py --steps K --warmup W \
        --no-cpu-baseline --spread-steps 0 --replay-steps 0 --no-nodedup
    python tools/headline_trace.py <dir> --steps K --warmup W [--out profiles/rNN/headline_obs.json]

With those flags the bench runs exactly three passes of one filter: W warm-up frames, the K timed
frames, and min(K, 10) stage-breakdown frames, one observation launch (k_gp_tile<d, false>) each.
The summary keeps launches [W, W + K) -- the timed loop -- and reports their duration statistics
(the roofline's launch time), the FLOP rate and peak fraction it implies at the bench's workload,
and per frame the start-to-start time and the GPU time outside the observation launch.  Frames
the bench samples with timing events (every `sample`-th of the timed loop) are flagged, since
their event records idle the GPU for a few microseconds.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import statistics
from pathlib import Path


def load(root):
    rows = []
    for f in sorted(glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def is_obs(name: str) -> bool:
    return "k_gp_tile" in name and ", false" in name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--sample", type=int, default=16, help="bench's event-sampling period of the timed loop")
    ap.add_argument("--flop-per-particle", type=float, default=2000 * 2001 + 2 * 2000 + 2 * 2000 * 62,
                    help="algorithmic FLOP per particle of the observation tile (config 2: 4.254e6)")
    ap.add_argument("--particles", type=int, default=100_000)
    ap.add_argument("--peak", type=float, default=78.6)
    ap.add_argument("--commit", default=None)
    ap.add_argument("--command", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = load(a.root)
    obs = [i for i, r in enumerate(rows) if is_obs(r[2])]
    expect = a.warmup + a.steps + min(a.steps, 10)
    timed = obs[a.warmup:a.warmup + a.steps]
    durs = [(rows[i][1] - rows[i][0]) * 1e-3 for i in timed]       # us
    frames = []
    for k in range(len(timed) - 1):
        i, j = timed[k], timed[k + 1]
        span = (rows[j][0] - rows[i][0]) * 1e-3
        frames.append({"frame": k, "start_to_start_us": span,
                       "non_observation_us": span - (rows[i][1] - rows[i][0]) * 1e-3,
                       "kernels_between": j - i - 1, "sampled": k % a.sample == 0 or (k + 1) % a.sample == 0})
    mean_ms = statistics.mean(durs) / 1e3
    ach = a.flop_per_particle * a.particles / (mean_ms * 1e-3) / 1e12
    unsampled = [f for f in frames if not f["sampled"]]
    out = {
        "source": str(a.root), "commit": a.commit, "command": a.command,
        "observation_launches_in_trace": len(obs), "expected": expect, "count_ok": len(obs) == expect,
        "timed_launches": len(durs),
        "launch_ms": {"mean": mean_ms, "median": statistics.median(durs) / 1e3, "min": min(durs) / 1e3,
                      "max": max(durs) / 1e3, "stdev": statistics.pstdev(durs) / 1e3},
        "achieved_tflops": ach, "peak_tflops": a.peak, "frac": ach / a.peak,
        "flop_per_particle": a.flop_per_particle, "particles": a.particles,
        "frame_us": {"start_to_start_mean": statistics.mean(f["start_to_start_us"] for f in frames),
                     "non_observation_mean": statistics.mean(f["non_observation_us"] for f in frames),
                     "non_observation_mean_unsampled": statistics.mean(f["non_observation_us"] for f in unsampled)
                     if unsampled else None,
                     "non_observation_median": statistics.median(f["non_observation_us"] for f in frames)},
        "kernel": rows[timed[0]][2] if timed else None,
        "frames": frames,
    }
    txt = json.dumps(out, indent=1)
    if a.out:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(txt + "\n")
    print(json.dumps({k: out[k] for k in ("count_ok", "timed_launches", "launch_ms", "frac", "frame_us")}))


if __name__ == "__main__":
    main()
