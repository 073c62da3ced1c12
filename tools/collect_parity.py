"""Collate the GPU parity records (tests write them to $EFD_PARITY_OUT) into one committed file.

    python tools/collect_parity.py gpurun_out/r03d/parity profiles/r03_parity.json
"""
import glob
import json
import os
import sys


def main(src, dst):
    out = {"source": src, "records": {}}
    for f in sorted(glob.glob(os.path.join(src, "*.json"))):
        out["records"][os.path.basename(f)[:-5]] = json.load(open(f))
    json.dump(out, open(dst, "w"), indent=1)
    for name, r in out["records"].items():
        if "max_rel_off_extrap" in r:
            print(f"{name:24s} linearity max dev {r['max_rel_off_extrap']:.2e} of max|S| off the "
                  f"{r['extrap_bins']} extrapolated-term bins ({r['max_rel']:.2e} on them)")
        elif "walkers" in r:
            print(f"{name:24s} walkers {r['walkers']:3d}  max |ll_gpu - ll_oracle| / bound "
                  f"{r['max_err_over_bound']:.2e}")
        else:
            print(f"{name:24s} off-fold max err {r['max_err_off_fold_rel']:.2e} of max|R|; fold bins "
                  f"{r['fold_bins']} (max err/D {r['max_err_over_D_at_folds']:.2f}); extrapolated "
                  f"bins {r.get('extrapolated_bins', 0)} (max err/E "
                  f"{r.get('max_err_over_E_at_extrapolated', 0):.1e}); ok {r['ok']}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
