"""Instruction mix of k_modesum's record loop (the loop holding the fast path's v_rsq_f64).

    python tools/asm_loop.py [hipcc -D flags ...]

Compiles csrc/emrifd.hip for gfx950 to device assembly (/tmp) and prints, for the paired
uniform-K_{1/3} instantiation, the register budget and the counts of VALU / FP64 / LDS / SALU
instructions between the loop header and its back edge.
"""

import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ASM_SRC / ASM_KERNEL: another source file (e.g. an older revision) or kernel symbol prefix
# (the batch sum of config 2: k_modesum_batchILb1ELi1ELi2ELb0E)
SRC = os.environ.get("ASM_SRC") or os.path.join(ROOT, "emri_frequencydomainwaveforms_amd", "csrc",
                                                "emrifd.hip")
KERNEL = os.environ.get("ASM_KERNEL", "k_modesumILb1ELi1E")


def analyse(flags, show=False):
    out = os.path.join(tempfile.gettempdir(), "efd_asm_%d.s" % os.getpid())
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only",
                    "-S", *flags, "-o", out, SRC], check=True, stderr=subprocess.DEVNULL)
    L = open(out).read().split("\n")
    s = next(i for i, l in enumerate(L) if KERNEL in l and not l.startswith(("\t", " ", "."))
             and ":" in l)
    e = next(i for i in range(s, len(L)) if L[i].startswith(".Lfunc_end"))
    body = L[s:e]
    r = next(i for i, l in enumerate(body) if "v_rsq_f64" in l)
    h = max(i for i in range(r) if re.match(r"^\.LBB\d+_\d+:.*Loop Header", body[i]))
    lab = body[h].split(":")[0]
    be = max(i for i, l in enumerate(body) if ("s_cbranch" in l or "s_branch" in l)
             and l.strip().endswith(lab))
    seg = [l.strip() for l in body[h:be + 1]]
    ins = [l.split()[0] for l in seg if l and not l.startswith((";", "."))]
    meta = {}
    for l in L[e:]:
        m = re.match(r"\s+\.(vgpr_count|vgpr_spill_count|sgpr_spill_count|"
                     r"private_segment_fixed_size|group_segment_fixed_size):\s+(\d+)", l)
        if m and KERNEL in "".join(L[max(e, L.index(l) - 40):L.index(l) + 40]):
            meta.setdefault(m.group(1), int(m.group(2)))
    v = [i for i in ins if i.startswith("v_")]
    print(f"flags={' '.join(flags) or '-'}  loop: valu {len(v)} (f64 {sum('f64' in i for i in v)})"
          f"  ds {sum(i.startswith('ds_') for i in ins)}  salu {sum(i.startswith('s_') for i in ins)}"
          f"  scratch {sum('scratch' in i for i in ins)}  calls {sum('swappc' in i for i in ins)}")
    if show:
        for k, c in collections.Counter(ins).most_common():
            print(f"  {c:4d} {k}")
    return v


if __name__ == "__main__":
    args = sys.argv[1:]
    show = "--show" in args
    analyse([a for a in args if a != "--show"], show=show)
