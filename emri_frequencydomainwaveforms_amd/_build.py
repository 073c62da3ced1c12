"""Build libemrifd.so in-tree (no JIT cache, so the .so travels with the repo snapshot):

  csrc/emrifd_cpu.cpp -> g++ -O3 -march=x86-64-v4 -fopenmp (the host twin, efd_*_cpu; AVX-512 is
                         on both this container's Sapphire Rapids and the GPU box's EPYC 9575F)
  csrc/emrifd_host.cpp -> g++ -O3: the host upstream stand-ins (trajectory, p0 solve) in C++
  csrc/emrifd_modes.cpp -> g++ -O3 -ffast-math -fopenmp (libmvec; knots over threads for one-at-a-time
                          calls): amplitudes, mode selection
  csrc/emrifd.hip     -> hipcc --offload-arch=gfx950, linked with both objects and libgomp
"""

import glob
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
SRC = os.path.join(CSRC, "emrifd.hip")
CPU_SRC = os.path.join(CSRC, "emrifd_cpu.cpp")
HOST_SRC = os.path.join(CSRC, "emrifd_host.cpp")
MODES_SRC = os.path.join(CSRC, "emrifd_modes.cpp")
OUT = os.path.join(HERE, "libemrifd.so")
OBJDIR = os.path.join(HERE, "build")
ARCH = os.environ.get("EFD_OFFLOAD_ARCH", "gfx950")
CPU_ARCH = os.environ.get("EFD_CPU_ARCH", "x86-64-v4")


def _inputs():
    hdr = os.path.join(os.path.dirname(HERE), "include", "emrifd.h")
    return [SRC, CPU_SRC, HOST_SRC, MODES_SRC, hdr] + glob.glob(os.path.join(CSRC, "*.inc"))


def build(force=False, verbose=False, extra=()):
    if not force and os.path.exists(OUT):
        t = os.path.getmtime(OUT)
        if all(os.path.getmtime(p) <= t for p in _inputs() if os.path.exists(p)):
            return OUT
    os.makedirs(OBJDIR, exist_ok=True)
    obj = os.path.join(OBJDIR, "emrifd_cpu.o")
    hobj = os.path.join(OBJDIR, "emrifd_host.o")
    cpu = ["g++", "-O3", f"-march={CPU_ARCH}", "-fopenmp", "-ffp-contract=off", "-fPIC",
           "-std=c++17", "-c", CPU_SRC, "-o", obj]
    host = ["g++", "-O3", f"-march={CPU_ARCH}", "-ffp-contract=off", "-fPIC", "-std=c++17", "-c",
            HOST_SRC, "-o", hobj]
    mobj = os.path.join(OBJDIR, "emrifd_modes.o")
    modes = ["g++", "-O3", f"-march={CPU_ARCH}", "-ffast-math", "-fopenmp", "-fPIC",
             "-std=c++17", "-c", MODES_SRC, "-o", mobj]
    hip = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", *extra,
           "-o", OUT + ".tmp", obj, hobj, mobj, SRC, "-lgomp", "-lmvec"]
    for cmd in (cpu, host, modes, hip):
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))
