"""Build libemrifd.so in-tree with hipcc for gfx950 (no JIT cache, so the .so travels)."""

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "emrifd.hip")
OUT = os.path.join(HERE, "libemrifd.so")
ARCH = os.environ.get("EFD_OFFLOAD_ARCH", "gfx950")


def build(force=False, verbose=False):
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= os.path.getmtime(SRC):
        hdr = os.path.join(os.path.dirname(HERE), "include", "emrifd.h")
        if not os.path.exists(hdr) or os.path.getmtime(OUT) >= os.path.getmtime(hdr):
            return OUT
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-o", OUT + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))
