"""Median per-launch k_modesum counters of each variant under gpurun_out/<tag>/ (exp_pmc.sh)."""
import collections
import csv
import glob
import json
import sys

root, variants = sys.argv[1], sys.argv[2:]
for v in variants:
    files = glob.glob(f"{root}/{v}/**/*counter_collection.csv", recursive=True)
    agg = collections.defaultdict(float)
    for f in files:
        for r in csv.DictReader(open(f)):
            agg[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
    disp = sorted({d for d, _ in agg})[1:]
    names = sorted({c for _, c in agg})
    med = {c: sorted(agg[(d, c)] for d in disp)[len(disp) // 2] for c in names} if disp else {}
    print(json.dumps({"variant": v, "launches": len(disp), **{k: f"{x:.4g}" for k, x in med.items()}}))
