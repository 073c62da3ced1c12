"""Build the oracle's C restatement (oracle/fd_oracle_c.c -> oracle/_build/libfdoracle.so).

Test infrastructure only: the CPU baseline leg of bench.py and tests/ load it.
"""

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "fd_oracle_c.c")
OUTDIR = os.path.join(HERE, "_build")
OUT = os.path.join(OUTDIR, "libfdoracle.so")


def build(force=False, verbose=False):
    if not os.path.exists(SRC):
        return None
    os.makedirs(OUTDIR, exist_ok=True)
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= os.path.getmtime(SRC):
        return OUT
    cmd = ["gcc", "-O3", "-march=x86-64-v3", "-fopenmp", "-fPIC", "-shared", "-std=c11",
           "-o", OUT + ".tmp", SRC, "-lm"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT
