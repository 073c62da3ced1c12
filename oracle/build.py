"""Build the oracle's C restatement (oracle/fd_oracle_c.c -> oracle/_build/libfdoracle.so).

Test infrastructure only: the CPU baseline leg of bench.py and tests/ load it.
"""

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "fd_oracle_c.c")
OUTDIR = os.path.join(HERE, "_build")
OUT = os.path.join(OUTDIR, "libfdoracle.so")
# The same C restatement compiled with FMA contraction: a second rounding realisation of the
# same arithmetic, used by the full-size tests to measure how far rounding alone moves the
# oracle at ill-conditioned (fold) bins. Never a checker on its own.
OUT_FMA = os.path.join(OUTDIR, "libfdoracle_fma.so")


def _build_one(out, extra, force, verbose):
    if not force and os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(SRC):
        return out
    cmd = ["gcc", "-O3", "-march=x86-64-v3", "-fopenmp", "-fPIC", "-shared", "-std=c11", *extra,
           "-o", out + ".tmp", SRC, "-lm"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def build(force=False, verbose=False):
    if not os.path.exists(SRC):
        return None
    os.makedirs(OUTDIR, exist_ok=True)
    _build_one(OUT_FMA, ["-ffp-contract=fast"], force, verbose)
    return _build_one(OUT, [], force, verbose)
