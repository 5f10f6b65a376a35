"""One-line summary of a bench.py JSON line: python3 tools/line.py <file>"""
import json
import sys

d = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]
r = d.get("roofline") or {}
k = {a: round(b, 3) for a, b in (d.get("kernel_ms") or {}).items() if isinstance(b, float) and b > 0.05}
c = d.get("cpu_baseline") or {}
print(sys.argv[1].split("/")[-1], "%.4g %s" % (d["value"], d["unit"]), "ms/step %.3f" % d["ms_per_step"],
      "frac %s" % (round(r["frac"], 3) if "frac" in r else None),
      "traffic %s" % (round(r["traffic"] / 1e9, 2) if r.get("traffic") else None),
      "verified", d.get("verified"), "cpu %.3g" % c.get("value", 0), k)
