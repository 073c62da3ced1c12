"""Summarise tools/gpu/windowed_prof.sh's output into profiles/<TAG>_windowed_roofline.json.

    python tools/windowed_summary.py TAG

From the kernel trace: every dispatch between the two k_polarizations markers of
tools/windowed_profile.py (the timed half-steps), per kernel name the calls and time per
half-step (copy engine blits included: "__amd_rocclr_copyBuffer"). From the PMC passes: the HBM
bytes per dispatch of the row / column / reduction kernels (2 FETCH_SIZE + WRITE_SIZE, kB,
MI355X_MICROARCH.md's gfx950 correction), their achieved GB/s over the traced mean duration, and
the fraction of the 8 TB/s HBM peak.
"""

import collections
import csv
import json
import os
import statistics as st
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HBM_PEAK_GBS = 8000.0


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", tag)
    w = json.loads(open(os.path.join(src, "windowed.json")).read().strip().splitlines()[-1])
    steps = int(w["steps"])
    rows = list(csv.DictReader(open(os.path.join(src, "wtrace", "run_kernel_trace.csv"))))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                for r in rows)
    marks = [i for i, e in enumerate(ev) if e[2].startswith("k_polarizations")]
    if len(marks) < 2:
        raise SystemExit("markers not found in the trace")
    a, b = marks[-2], marks[-1]
    span = ev[a + 1:b]
    per = collections.defaultdict(lambda: [0, 0])
    for s, e, n in span:
        per[n][0] += 1
        per[n][1] += e - s
    kernels = {n: {"calls_per_half_step": c / steps, "us_per_half_step": t / steps / 1e3,
                   "us_per_call": t / c / 1e3} for n, (c, t) in
               sorted(per.items(), key=lambda kv: -kv[1][1])}
    wall = (ev[b][0] - ev[a][1]) / steps / 1e3
    # PMC: bytes per dispatch of each kernel (median over the dispatches)
    pmc = collections.defaultdict(dict)
    for p, cname in (("wpmc_fetch", "FETCH_SIZE"), ("wpmc_write", "WRITE_SIZE")):
        f = os.path.join(src, p, "run_counter_collection.csv")
        agg = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != cname:
                continue
            d = int(r["Dispatch_Id"])
            agg[d] += float(r["Counter_Value"])
            names[d] = short(r["Kernel_Name"])
        byk = collections.defaultdict(list)
        for d, v in agg.items():
            byk[names[d]].append(v)
        for n, vs in byk.items():
            pmc[n][cname] = st.median(vs)
    roof = {}
    for n, c in pmc.items():
        if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c or n not in kernels:
            continue
        byts = (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
        us = kernels[n]["us_per_call"]
        gbs = byts / (us * 1e-6) / 1e9
        roof[n] = {"hbm_bytes_per_call": byts, "us_per_call": us, "achieved_gbs": gbs,
                   "frac_of_hbm_peak": gbs / HBM_PEAK_GBS}
    out = {"tag": tag, "workload": w["config"], "N_f": w["N_f"], "steps": steps,
           "ms_per_half_step_host": w["ms_per_half_step"],
           "loglikes_per_s": w["loglikes_per_s"], "us_per_half_step_trace": wall,
           "kernels": kernels, "hbm_roofline": roof,
           "hbm_formula": "(2 FETCH_SIZE + WRITE_SIZE) x 1024 (kB; gfx950 FETCH_SIZE x2), "
                          "median over the kernel's dispatches; time from the kernel trace"}
    dst = os.path.join(ROOT, "profiles", f"{tag}_windowed_roofline.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
