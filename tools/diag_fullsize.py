"""Diagnostics: config-2 spectrum of one or more library builds against the C oracle.

    python tools/diag_fullsize.py base [old ...]      # names as in tools/exp_variants.py
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(name, out):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import exp_variants
    os.environ["EFD_LIB"] = exp_variants.lib_path(name)
    import torch
    import bench
    from emri_frequencydomainwaveforms_amd.summation import DeviceInputs, ModeSumEngine
    w = bench.build_workload()
    inp = DeviceInputs.from_host(w["t"], w["amp"], w["phi_phi"], w["phi_r"], w["f_phi"],
                                 w["f_r"], w["m"], w["n"], w["ylm_p"], w["ylm_m"])
    freq = torch.as_tensor(w["freq"], device="cuda")
    S = ModeSumEngine("uniform").run(inp, freq, grid_symmetric=True, scale=w["prefactor"])
    np.save(out, S.cpu().numpy())


def main(names):
    import tempfile
    import bench
    from oracle import fd_oracle_c
    w = bench.build_workload()
    R = fd_oracle_c.modesum(w["t"], w["amp"].T, w["phi_phi"], w["phi_r"], w["f_phi"], w["f_r"],
                            w["m"], w["n"], w["ylm_p"], w["ylm_m"], w["freq"], w["prefactor"],
                            caustic="uniform", nthreads=16)
    mx = np.abs(R).max()
    f = w["freq"]
    for name in names:
        out = os.path.join(tempfile.gettempdir(), f"diag_{name}.npy")
        subprocess.run([sys.executable, __file__, "child", name, out], check=True)
        S = np.load(out)
        d = np.abs(S - R)
        k = int(d.argmax())
        bad = np.nonzero(d > 1e-9 * mx)[0]
        print(f"{name}: max rel {d.max() / mx:.3e} at bin {k} f={f[k]:.6e} |S|={abs(S[k]):.3e} "
              f"|R|={abs(R[k]):.3e}; bins over 1e-9: {len(bad)}; "
              f"f range of those: {f[bad].min() if len(bad) else 0:.4e}..{f[bad].max() if len(bad) else 0:.4e}")
        if len(bad):
            top = bad[np.argsort(-d[bad])[:8]]
            for kk in top:
                print(f"   bin {kk} f={f[kk]:+.6e} |S-R|/max={d[kk]/mx:.2e} |R|/max={abs(R[kk])/mx:.2e}")


if __name__ == "__main__":
    if sys.argv[1] == "child":
        child(sys.argv[2], sys.argv[3])
    else:
        main(sys.argv[1:])
