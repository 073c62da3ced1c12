"""Interleaved end-to-end A/B of library variants through bench.py (GPU box).

    python tools/ab_bench.py ROUNDS NAME[@ARG,...] [NAME[@ARG,...] ...]
    (an ARG of the form env:NAME=VALUE sets the child's environment instead)

Each round runs `bench.py --no-cpu-baseline` once per variant, in a rotated order, each in its
own child process with EFD_LIB pointing at the variant (names as in tools/exp_variants.py:
"base" is the in-tree library, others exp/libemrifd_<NAME>.so). Prints one JSON line per run
and a summary per variant: median waveforms/s and k_modesum ms with a bootstrap 95% interval,
and the median of the per-round ratios to the first variant with its interval (paired rounds
cancel the box-to-box and drift variance that separate runs suffer).
"""

import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from exp_variants import lib_path  # noqa: E402


def run_one(name, extra):
    # NAME[@ARG,ARG...]: the variant's library plus its own bench.py arguments
    lib, _, own = name.partition("@")
    env = dict(os.environ, EFD_LIB=lib_path(lib))
    own = [x for x in own.split(",") if x]
    # "env:NAME=VALUE" items set the child's environment instead of bench.py arguments
    for x in [x for x in own if x.startswith("env:")]:
        k, _, v = x[4:].partition("=")
        env[k] = v
    own = [x for x in own if not x.startswith("env:")]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline",
                        *extra, *own], capture_output=True, text=True, timeout=300, env=env,
                       cwd=ROOT)
    if r.returncode != 0:
        print(json.dumps({"variant": name, "error": r.returncode, "stderr": r.stderr[-1500:]}),
              flush=True)
        sys.exit(1)   # start nothing more on the GPU after a failed run
    j = json.loads(r.stdout.strip().splitlines()[-1])
    return j["value"], j["roofline"]["kernel_ms"]


def ci_median(x, reps=4000, seed=1):
    x = np.asarray(x, dtype=float)
    rng = np.random.default_rng(seed)
    meds = np.median(rng.choice(x, size=(reps, len(x)), replace=True), axis=1)
    return float(np.median(x)), float(np.percentile(meds, 2.5)), float(np.percentile(meds, 97.5))


def main():
    rounds = int(sys.argv[1])
    names = sys.argv[2:]
    extra = os.environ.get("AB_BENCH_ARGS", "").split()
    res = {n: {"value": [], "kernel_ms": []} for n in names}
    for r in range(rounds):
        order = names[r % len(names):] + names[:r % len(names)]
        for n in order:
            v, k = run_one(n, extra)
            res[n]["value"].append(v)
            res[n]["kernel_ms"].append(k)
            print(json.dumps({"round": r, "variant": n, "value": v, "kernel_ms": k}), flush=True)
    ref = names[0]
    for n in names:
        out = {"variant": n, "rounds": rounds}
        for key in ("value", "kernel_ms"):
            m, lo, hi = ci_median(res[n][key])
            out[key] = {"median": m, "ci95": [lo, hi]}
        if n != ref:
            ratio = np.array(res[n]["value"]) / np.array(res[ref]["value"])
            m, lo, hi = ci_median(ratio)
            out["value_ratio_vs_" + ref] = {"median": m, "ci95": [lo, hi]}
        print("SUMMARY " + json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
