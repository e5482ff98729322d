#!/usr/bin/env python3
"""Collect bench.py --simulate-world records (one JSON line per rank) into one summary per
configuration: per-rank ms_per_step / host_ms_per_step (/ host_busy_ms_per_step), the slowest
rank, and the host share of the step.

    python scripts/simrank_summary.py profiles/r6/sim --out profiles/r6
"""
import argparse
import glob
import json
import os
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    kinds = {}
    for f in sorted(glob.glob(os.path.join(a.src, "sim_*_r*.json"))):
        m = re.match(r"sim_(.+)_r(\d+)\.json", os.path.basename(f))
        with open(f) as fh:
            lines = [ln for ln in fh if ln.strip()]
        if not m or not lines:
            continue
        rec = json.loads(lines[-1])
        kinds.setdefault(m.group(1), {})[int(m.group(2))] = rec
    for kind, ranks in kinds.items():
        world = next(iter(ranks.values()))["simulated"]["world"]
        rows = {r: {"ms_per_step": v["ms_per_step"], "host_ms_per_step": v.get("host_ms_per_step"),
                    "host_busy_ms_per_step": v.get("host_busy_ms_per_step"),
                    "host_share": round(v["host_ms_per_step"] / v["ms_per_step"], 3)} for r, v in sorted(ranks.items())}
        slow = max(rows, key=lambda r: rows[r]["ms_per_step"])
        out = {"config": kind, "world": world, "ranks_measured": sorted(rows), "per_rank": rows,
               "slowest_rank": slow, "slowest_ms_per_step": rows[slow]["ms_per_step"],
               "max_host_share": max(v["host_share"] for v in rows.values()),
               "model_config": next(iter(ranks.values()))["config"],
               "note": "bench.py --simulate-world: one GPU plays each rank; collectives are same-sized local "
                       "copies (xGMI time not included)"}
        print(f"{kind}: world {world}, ranks {sorted(rows)}, slowest r{slow} {rows[slow]['ms_per_step']} ms, "
              f"max host share {out['max_host_share']}")
        if a.out:
            with open(os.path.join(a.out, f"simrank_{kind}_w{world}.json"), "w") as fh:
                json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
