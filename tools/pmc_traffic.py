"""Summarise rocprofv3 outputs into profiles/<round>_*.json.

Usage (on the GPU box, each rocprofv3 pass in its own run):
  rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -- python3 bench.py ...
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -- python3 bench.py ...
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -- python3 bench.py ...
  python3 tools/pmc_traffic.py --kt gpurun_out/prof_kt --fetch gpurun_out/prof_fetch \
      --write gpurun_out/prof_write --bench gpurun_out/bench_prof.json --out profiles/r01_pmc_traffic.json

HBM bytes per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024: on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced streaming read
(MI355X_MICROARCH.md §HBM); WRITE_SIZE is exact for 16-B/lane stores.  Both
are per dispatch (summed over XCD instances), averaged over the launches.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def _rows(d, pattern):
    out = []
    for p in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


_MULTI = set()  # kernel base names with several template instances in the inputs


def _parts(name):
    m = re.search(r"\b(k_[A-Za-z0-9_]+)(<[^()]*>)?", name)
    if not m:
        return name.split("(")[0], ""
    return m.group(1), (m.group(2) or "").replace(" ", "")


def _short(name):
    """The kernel's base name; with its template arguments when the inputs
    hold several instances of it (e.g. k_ot_merge<4,...> and <8,...>)."""
    base, targs = _parts(name)
    return base + targs if base in _MULTI else base


def _scan_instances(dirs):
    inst = defaultdict(set)
    for d in dirs:
        if not d:
            continue
        for pattern, col in (("*kernel_stats.csv", "Name"), ("*counter_collection.csv", "Kernel_Name")):
            for r in _rows(d, pattern):
                base, targs = _parts(r.get(col, ""))
                inst[base].add(targs)
    _MULTI.update(b for b, t in inst.items() if len(t) > 1)


def counters(d, counter):
    """-> {kernel: [per-dispatch value]} for one counter pass."""
    per = defaultdict(lambda: defaultdict(float))
    for r in _rows(d, "*counter_collection.csv"):
        if r.get("Counter_Name") != counter:
            continue
        k = _short(r.get("Kernel_Name", ""))
        per[k][r.get("Dispatch_Id", r.get("Correlation_Id", ""))] += float(r["Counter_Value"])
    return {k: list(v.values()) for k, v in per.items()}


def kernel_stats(d):
    out = {}
    for r in _rows(d, "*kernel_stats.csv"):
        k = _short(r.get("Name", ""))
        out[k] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                  "total_ns": float(r["TotalDurationNs"]), "pct": float(r.get("Percentage", 0))}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kt")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--sq", help="a pass of SQ_* counters: per-kernel averages per dispatch")
    ap.add_argument("--bench", help="bench.py JSON line of the profiled run")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    res = {"kernels": {}}
    _scan_instances([a.kt, a.fetch, a.write, a.sq])
    if a.sq:
        names = sorted({r["Counter_Name"] for r in _rows(a.sq, "*counter_collection.csv")})
        for n in names:
            for k, v in counters(a.sq, n).items():
                res["kernels"].setdefault(k, {})[n] = sum(v) / len(v)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res["kernels"].get("k_write_cf", {})))
        return
    if a.bench and os.path.exists(a.bench):
        line = [l for l in open(a.bench) if l.startswith("{")][-1]
        b = json.loads(line)
        res["rules"] = b["config"]["rules_per_gpu"]
        res["events"] = b["config"]["events_per_gpu_step"]
        if "windows" in b["config"]:
            res["windows"] = b["config"]["windows"]
        res["bench"] = {k: b[k] for k in ("value", "ms_per_step", "kernel_ms", "roofline")}
    ks = kernel_stats(a.kt) if a.kt else {}
    fe = counters(a.fetch, "FETCH_SIZE") if a.fetch else {}
    wr = counters(a.write, "WRITE_SIZE") if a.write else {}
    for k in sorted(set(ks) | set(fe) | set(wr)):
        e = {}
        if k in ks:
            e.update(ks[k])
        if k in fe and fe[k]:
            e["fetch_kb_per_launch"] = sum(fe[k]) / len(fe[k])
        if k in wr and wr[k]:
            e["write_kb_per_launch"] = sum(wr[k]) / len(wr[k])
        if "fetch_kb_per_launch" in e and "write_kb_per_launch" in e:
            e["hbm_bytes_per_launch"] = 2 * e["fetch_kb_per_launch"] * 1024 + e["write_kb_per_launch"] * 1024
            # without the x2 read correction (stated for 16-B/lane streaming reads;
            # gathers of 8-B words are uncalibrated)
            e["hbm_bytes_raw_per_launch"] = (e["fetch_kb_per_launch"] + e["write_kb_per_launch"]) * 1024
        res["kernels"][k] = e
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res["kernels"].get("k_write_cf", {})))


if __name__ == "__main__":
    main()
