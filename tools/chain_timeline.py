"""Per-half-step device timeline of the fused likelihood from a rocprofv3 kernel trace
(tools/gpu/chain_trace.sh): for each efd_modesum_prepare_batch chain (k_group_b ... ) the
kernels' durations and the gaps between them, median over the traced half-steps.

    python tools/chain_timeline.py gpurun_out/TAG/tr_config4/run_kernel_trace.csv
"""
import csv
import statistics as st
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].split("<")[0]


def main(path):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                for r in rows)
    # a chain runs from one k_group_b (or k_prep_pcr_b when it groups the harmonics itself) to
    # the last kernel before the next
    chains, cur = [], None
    for s, e, n in ev:
        if n in ("k_ll_tile_const", "vectorized_elementwise_kernel", "__amd_rocclr_copyBuffer"):
            continue
        starts = n == "k_group_b" or (n == "k_prep_pcr_b" and not (cur and cur[-1][2] == "k_group_b"))
        if starts:
            if cur:
                chains.append(cur)
            cur = [(s, e, n)]
        elif cur is not None:
            cur.append((s, e, n))
    chains = chains[len(chains) // 5:]   # skip warm-up
    names = [n for _, _, n in chains[0]]
    chains = [c for c in chains if [n for _, _, n in c] == names]
    print(f"{len(chains)} chains of {len(names)} kernels")
    tot = []
    for i, n in enumerate(names):
        d = st.median((c[i][1] - c[i][0]) / 1e3 for c in chains)
        g = st.median((c[i][0] - c[i - 1][1]) / 1e3 for c in chains) if i else 0.0
        print(f"  {n:24s} gap {g:7.1f} us  run {d:7.1f} us")
    print(f"  chain (first start to last end): "
          f"{st.median((c[-1][1] - c[0][0]) / 1e3 for c in chains):.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
