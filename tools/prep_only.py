"""The headline's preparation alone (no sums beside it): N rounds of efd_modesum_prepare_batch over
bench.py's batch of 8 config-2 waveforms on one stream, synchronised each round, so a kernel
trace (rocprofv3 --kernel-trace) shows each preparation kernel's standalone duration and grid.
With the sums of batch i running beside batch i+1's preparation, every preparation wave holds a
SIMD slot the sum's 4 waves of 128 VGPRs would fill (the sum uses the whole register file), so a
kernel's cost to the sum is about its waves x their lifetime.

    python tools/prep_only.py [ROUNDS]
"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    from emri_frequencydomainwaveforms_amd.summation import (DeviceInputs, ModeSumEngine,
                                                             prepare_batch)
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    ws = bench.build_workloads(8)
    inps = [DeviceInputs.from_host(w["t"], w["amp"], w["phi_phi"], w["phi_r"], w["f_phi"],
                                   w["f_r"], w["m"], w["n"], w["ylm_p"], w["ylm_m"], device=dev)
            for w in ws]
    freq = torch.as_tensor(ws[0]["freq"], device=dev)
    engs = [ModeSumEngine(caustic="uniform") for _ in ws]
    st = torch.cuda.Stream(dev)
    for _ in range(rounds):
        prepare_batch([(e, dict(inp=inps[j], freq=freq, out=None, grid_symmetric=True,
                                scale=ws[j]["prefactor"])) for j, e in enumerate(engs)],
                      stream=st.cuda_stream)
        st.synchronize()
    print("prep_only done", rounds)


if __name__ == "__main__":
    main()
