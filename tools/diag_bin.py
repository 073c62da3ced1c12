"""Diagnostic: which (m, n) groups make the GPU's config-2 spectrum differ from the C oracle at
a given bin (run on the GPU box; prints one line per group whose own GPU-vs-oracle difference at
the bin exceeds --thresh of the full spectrum's max|S|).

    python tools/diag_bin.py --k 3487815 [--window 12]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, required=True)
    ap.add_argument("--window", type=int, default=12)
    ap.add_argument("--thresh", type=float, default=1e-10)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch
    import bench
    from emri_frequencydomainwaveforms_amd.summation import DeviceInputs, ModeSumEngine
    from oracle import fd_oracle_c
    from oracle.fd_oracle import monotonic_runs
    w = bench.build_workload()
    freq_h = w["freq"]
    freq = torch.as_tensor(freq_h, device="cuda")
    k, W = args.k, args.window
    fk = abs(freq_h[k])
    mx = 6.7533643029200836e-18
    groups = {}
    for h, (m, n) in enumerate(zip(w["m"].tolist(), w["n"].tolist())):
        groups.setdefault((m, n), []).append(h)
    eng = ModeSumEngine("uniform")
    rows = []
    for (m, n), hs in sorted(groups.items()):
        F = m * w["f_phi"] + n * w["f_r"]
        cover = any(min(F[a], F[b]) < s * fk < max(F[a], F[b]) for a, b, _ in monotonic_runs(F) for s in (1, -1))
        if not cover:
            continue
        sel = np.array(hs)
        inp = DeviceInputs.from_host(w["t"], w["amp"][:, sel], w["phi_phi"], w["phi_r"],
                                     w["f_phi"], w["f_r"], w["m"][sel], w["n"][sel],
                                     w["ylm_p"][sel], w["ylm_m"][sel])
        S = eng.run(inp, freq, grid_symmetric=True, scale=w["prefactor"])[k - W:k + W + 1]
        S = S.cpu().numpy()
        R = fd_oracle_c.modesum(w["t"], w["amp"][:, sel].T, w["phi_phi"], w["phi_r"],
                                w["f_phi"], w["f_r"], w["m"][sel], w["n"][sel], w["ylm_p"][sel],
                                w["ylm_m"][sel], freq_h[k - W:k + W + 1], w["prefactor"],
                                caustic="uniform", nthreads=16)
        d = np.abs(S - R) / mx
        if d.max() > args.thresh:
            runs = [(a, b, s) for a, b, s in monotonic_runs(F)]
            dk = float(np.min(np.abs(F - fk)) / (freq_h[1] - freq_h[0]))
            rows.append({"m": m, "n": n, "members": len(hs), "max_err": float(d.max()),
                         "err_at_k": float(d[W]), "max_abs_R": float(np.abs(R).max() / mx),
                         "nearest_knot_bins": dk, "runs": runs,
                         "err": d.tolist()})
            print(json.dumps({kk: v for kk, v in rows[-1].items() if kk != "err"}), flush=True)
    if args.out:
        json.dump(rows, open(args.out, "w"), default=int)


if __name__ == "__main__":
    main()
