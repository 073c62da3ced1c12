"""Diagnostic: config-2 GPU-vs-oracle error at bins [k-W, k+W] for library variants and harmonic
subsets (oracle evaluated on the window only).   python tools/diag_bin2.py K VARIANT..."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
MX = 6.7533643029200836e-18


def child(name, k, W, subset):
    import exp_variants
    os.environ["EFD_LIB"] = exp_variants.lib_path(name)
    import torch
    import bench
    from emri_frequencydomainwaveforms_amd.summation import DeviceInputs, ModeSumEngine
    from oracle import fd_oracle_c
    from oracle.fd_oracle import monotonic_runs
    w = bench.build_workload()
    fk = abs(w["freq"][k])
    sel = np.arange(len(w["m"]))
    if subset == "cover":
        keep = []
        for h, (m, n) in enumerate(zip(w["m"], w["n"])):
            F = m * w["f_phi"] + n * w["f_r"]
            if any(min(F[a], F[b]) < fk < max(F[a], F[b]) for a, b, _ in monotonic_runs(F)):
                keep.append(h)
        sel = np.array(keep)
    elif subset.startswith("half"):
        sel = sel[int(subset[4]) :: 2]
    inp = DeviceInputs.from_host(w["t"], w["amp"][:, sel], w["phi_phi"], w["phi_r"], w["f_phi"],
                                 w["f_r"], w["m"][sel], w["n"][sel], w["ylm_p"][sel],
                                 w["ylm_m"][sel])
    freq = torch.as_tensor(w["freq"], device="cuda")
    eng = ModeSumEngine("uniform")
    S = eng.run(inp, freq, grid_symmetric=True, scale=w["prefactor"]).cpu().numpy()
    km = len(w["freq"]) - 1 - k
    out = {"variant": name, "subset": subset, "K": int(len(sel))}
    for kk, tag in ((k, "k"), (km, "mirror")):
        g = w["freq"][kk - W:kk + W + 1]
        R = fd_oracle_c.modesum(w["t"], w["amp"][:, sel].T, w["phi_phi"], w["phi_r"], w["f_phi"],
                                w["f_r"], w["m"][sel], w["n"][sel], w["ylm_p"][sel],
                                w["ylm_m"][sel], g, w["prefactor"], caustic="uniform",
                                nthreads=16)
        d = np.abs(S[kk - W:kk + W + 1] - R) / MX
        out[tag] = [float(f"{x:.2e}") for x in d]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "child":
        child(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
    else:
        k = int(sys.argv[1])
        for spec in sys.argv[2:]:
            name, _, subset = spec.partition("@")
            subprocess.run([sys.executable, __file__, "child", name, str(k), "10",
                            subset or "all"], check=True)
