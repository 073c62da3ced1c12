"""Per-kernel means of tools/gpu/windowed_diag.sh's SQ counter passes.

    python tools/windowed_diag.py TAG   -> profiles/<TAG>_windowed_diag.json

Per kernel and counter: the mean over the kernel's dispatches (each dispatch's value summed over
its instances). The SQ cycle counters count quad-cycles (MI355X_MICROARCH.md); ratios such as
WAIT_ANY / WAVE_CYCLES are what the notes read; TA_BUSY_avr / GRBM_GUI_ACTIVE is the texture
addresser's busy fraction (the vector memory path's issue bound).
"""

import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", tag)
    out = collections.defaultdict(dict)
    for p in ("diag1", "diag2", "diag3"):
        f = os.path.join(src, p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        agg = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (int(r["Dispatch_Id"]), r["Counter_Name"])
            agg[key] += float(r["Counter_Value"])
            names[int(r["Dispatch_Id"])] = short(r["Kernel_Name"])
        per = collections.defaultdict(list)
        for (d, c), v in agg.items():
            per[(names[d], c)].append(v)
        for (k, c), vs in per.items():
            out[k][c] = sum(vs) / len(vs)
    for k, c in out.items():
        w = c.get("SQ_WAVE_CYCLES")
        if w:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if n in c:
                    c["frac_" + n] = c[n] / w
        if c.get("GRBM_GUI_ACTIVE") and "TA_BUSY_avr" in c:
            c["frac_TA_BUSY"] = c["TA_BUSY_avr"] / c["GRBM_GUI_ACTIVE"]
        if c.get("SQ_LDS_IDX_ACTIVE"):
            c["lds_conflict_frac"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"]
    dst = os.path.join(ROOT, "profiles", f"{tag}_windowed_diag.json")
    json.dump({"tag": tag, "kernels": out}, open(dst, "w"), indent=1)
    for k, c in out.items():
        print(k, {n: round(v, 3) for n, v in c.items() if n.startswith(("frac", "lds_"))})


if __name__ == "__main__":
    main(sys.argv[1])
