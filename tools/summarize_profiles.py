"""Turn tools/profile_round.sh's raw rocprofv3 output into the committed profiles/ files.

    python tools/summarize_profiles.py r01

writes profiles/<tag>_kernel_stats.csv (the --kernel-trace --stats summary as produced),
profiles/<tag>_bench.json (the bench line of the same round), profiles/<tag>_pmc.json
(per-launch counter values of the mode-sum kernel: k_modesum_batch when the bench line's
config.batch > 1, one launch per batch of waveforms) and profiles/pmc_traffic.json, which bench.py reads
for roofline.traffic. HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (kB units from
rocprofv3): MI355X_MICROARCH.md, section HBM: on gfx950 FETCH_SIZE reports half of the bytes
of wide coalesced reads, WRITE_SIZE reads exactly for 16-B stores.
"""

import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(path):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        agg[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
    disp = sorted({d for d, _ in agg})
    names = sorted({c for _, c in agg})
    # the first dispatch belongs to the workspace-allocating run; use the steady-state median
    out = {}
    for c in names:
        vals = sorted(agg[(d, c)] for d in disp[1:] or disp)
        out[c] = vals[len(vals) // 2]
    return out, len(disp)


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(dst, f"{tag}_kernel_stats.csv"))
    shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, f"{tag}_bench.json"))
    if os.path.exists(os.path.join(src, "td_vs_fd.json")):
        shutil.copy(os.path.join(src, "td_vs_fd.json"), os.path.join(dst, f"{tag}_td_vs_fd.json"))
    pmc = {}
    ndisp = {}
    for p in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_valu"):
        f = os.path.join(src, p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        vals, n = per_dispatch(f)
        pmc.update(vals)
        ndisp[p] = n
    hbm = (2.0 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024.0
    fp64 = None
    if "SQ_INSTS_VALU_FMA_F64" in pmc:
        # FP64 lane operations per launch (an FMA counts 2 FLOP), scaled by the measured lane
        # utilisation of VALU instructions; VALU busy = SQ_ACTIVE_INST_VALU / CUs / GPU cycles
        # (rocprofv3's VALUBusy; GRBM_GUI_ACTIVE is summed over the 8 XCDs here)
        util = pmc["SQ_THREAD_CYCLES_VALU"] / (64.0 * pmc["SQ_ACTIVE_INST_VALU"])
        flops = 64.0 * util * (2.0 * pmc["SQ_INSTS_VALU_FMA_F64"] + pmc["SQ_INSTS_VALU_MUL_F64"]
                               + pmc["SQ_INSTS_VALU_ADD_F64"] + pmc["SQ_INSTS_VALU_TRANS_F64"])
        gpu_cycles = pmc["GRBM_GUI_ACTIVE"] / 8.0
        fp64 = {"flops_per_launch": flops, "lane_utilisation": util,
                "gpu_cycles_per_launch": gpu_cycles,
                "valu_busy": pmc["SQ_ACTIVE_INST_VALU"] / 256.0 / gpu_cycles,
                "fp64_share_of_valu_insts": (pmc["SQ_INSTS_VALU_FMA_F64"]
                                             + pmc["SQ_INSTS_VALU_MUL_F64"]
                                             + pmc["SQ_INSTS_VALU_ADD_F64"]
                                             + pmc["SQ_INSTS_VALU_TRANS_F64"])
                / pmc["SQ_INSTS_VALU"]}
    bench = json.loads(open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1])
    # one launch sums `batch` waveforms (k_modesum_batch; 1 = k_modesum)
    batch = int(bench["config"].get("batch", 1))
    kernel = "k_modesum_batch" if batch > 1 else "k_modesum"
    stats = {}
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
        if kernel in r["Name"] and (batch > 1 or "k_modesum_batch" not in r["Name"]):
            stats = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
    summary = {"tag": tag, "kernel": kernel, "workload": "config2", "batch": batch,
               "caustic": "uniform", "counters_per_launch": pmc, "dispatches": ndisp,
               "hbm_bytes_per_launch": hbm, "hbm_bytes_per_waveform": hbm / batch, "fp64": fp64,
               "hbm_formula": "(2 * FETCH_SIZE + WRITE_SIZE) * 1024 (kB; gfx950 FETCH_SIZE x2)",
               "rocprof_avg_ms": stats.get("avg_ns", 0.0) / 1e6,
               "bench_event_ms": bench["roofline"]["kernel_ms"]}
    json.dump(summary, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1)
    # FP64 FLOP per SPA evaluation (bench.py scales it to its own run's evaluation count)
    cfg = bench["config"]
    evals = (float(cfg["spa_evaluations_per_launch"]) if "spa_evaluations_per_launch" in cfg
             else float(cfg.get("spa_evaluations", 0)) * batch)
    sources = "walkers" if "walker" in str(cfg.get("sources", "")) else "same"
    summary["sources"] = sources
    json.dump(summary, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1)
    if fp64 and evals > 0:
        fp64["flops_per_evaluation"] = fp64["flops_per_launch"] / evals
    import hashlib
    src_sha = hashlib.sha256(open(os.path.join(ROOT, "emri_frequencydomainwaveforms_amd", "csrc",
                                               "emrifd.hip"), "rb").read()).hexdigest()[:16]
    # effective clock of the launch: GPU cycles (GRBM_GUI_ACTIVE over the 8 XCDs) / rocprof time
    clock = (fp64["gpu_cycles_per_launch"] / (stats["avg_ns"] * 1e-9) / 1e9
             if fp64 and stats.get("avg_ns") else None)
    summary["clock_ghz"] = clock
    summary["write_bytes_per_launch"] = pmc["WRITE_SIZE"] * 1024.0
    json.dump(summary, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1)
    json.dump({"workload": "config2", "caustic": "uniform", "kernel": kernel, "batch": batch,
               "sources": sources, "clock_ghz": clock,
               "write_bytes_per_launch": pmc["WRITE_SIZE"] * 1024.0,
               "hbm_bytes_per_launch": hbm, "fp64": fp64, "evaluations_per_launch": evals,
               "src_sha16": src_sha, "source": f"profiles/{tag}_pmc.json"},
              open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
