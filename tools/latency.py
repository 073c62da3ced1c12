"""Single-waveform latency breakdown on the device (config-1 and config-2 shapes).

    python tools/latency.py [--T 1] [--eps 1e-2] [--reps 20]

Prints one JSON line: per-kernel mean durations from HIP events around each phase of one
waveform on one stream (efd_modesum_prepare, efd_modesum_sum with fused h+/hx), the whole
device pipeline with inputs resident, the same plus the host->device upload of the inputs
(DeviceInputs.from_host), and the API call (GenerateEMRIWaveform.__call__) with the host
stand-in upstream memoised. Identifies what bounds one waveform's latency when the mode sum
is small (few harmonics), as in configs 1, 3, 4 and 5.
"""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=float, default=1.0)
    ap.add_argument("--eps", type=float, default=1e-2)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch
    import bench
    from emri_frequencydomainwaveforms_amd.summation import DeviceInputs, ModeSumEngine

    w = bench.build_workload(T=args.T, eps=args.eps)
    freq = torch.as_tensor(w["freq"], device="cuda")
    nf = int(freq.numel())
    k0 = int(np.searchsorted(w["freq"], 0.0))
    hp = torch.view_as_real(torch.empty(nf - k0, dtype=torch.complex128, device="cuda"))
    hc = torch.empty_like(hp)
    eng = ModeSumEngine()
    st = torch.cuda.current_stream().cuda_stream

    def upload():
        return DeviceInputs.from_host(w["t"], w["amp"], w["phi_phi"], w["phi_r"], w["f_phi"],
                                      w["f_r"], w["m"], w["n"], w["ylm_p"], w["ylm_m"])

    inp = upload()

    def ev():
        return torch.cuda.Event(enable_timing=True)

    def phases():
        e = [ev() for _ in range(3)]
        e[0].record()
        eng.launch(inp, freq, None, True, w["prefactor"], stream=st, phase="prepare")
        e[1].record()
        eng.launch(inp, freq, None, True, w["prefactor"], stream=st, hp=hp, hc=hc, k0=k0,
                   phase="sum")
        e[2].record()
        return e

    for _ in range(3):
        phases()
    torch.cuda.synchronize()
    rec = [phases() for _ in range(args.reps)]
    torch.cuda.synchronize()
    prep = float(np.mean([a.elapsed_time(b) for a, b, _ in rec]))
    summ = float(np.mean([b.elapsed_time(c) for _, b, c in rec]))

    def wall(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.reps * 1e3

    def dev_only():
        eng.launch(inp, freq, None, True, w["prefactor"], stream=st, hp=hp, hc=hc, k0=k0)

    def with_upload():
        i2 = upload()
        eng.launch(i2, freq, None, True, w["prefactor"], stream=st, hp=hp, hc=hc, k0=k0)

    print(json.dumps({"workload": f"T={args.T} yr eps={args.eps}", "harmonics": len(w["m"]),
                      "N_f": nf, "prepare_ms": prep, "sum_ms": summ,
                      "pipeline_wall_ms": wall(dev_only),
                      "pipeline_plus_upload_wall_ms": wall(with_upload)}))


if __name__ == "__main__":
    main()
