"""Build libemrifd.so in-tree (no JIT cache, so the .so travels with the repo snapshot):

  csrc/emrifd_cpu.cpp -> g++ -O3 -march=x86-64-v4 -fopenmp (the host twin, efd_*_cpu; AVX-512 is
                         on both this container's Sapphire Rapids and the GPU box's EPYC 9575F)
  csrc/emrifd_host.cpp -> g++ -O3 -fopenmp: the host upstream stand-ins (trajectory, p0 solve) in C++
  and the walker batches' staging
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


def source_id():
    """16 hex digits of the SHA-256 over the library's sources (name and contents, sorted): the
    build id compiled into libemrifd.so (efd_build_id)."""
    import hashlib
    h = hashlib.sha256()
    for p in sorted(_inputs()):
        if os.path.exists(p):
            h.update(os.path.basename(p).encode() + b"\0")
            h.update(open(p, "rb").read())
    return h.hexdigest()[:16]


def built_id(path=OUT):
    """The build id tagged into an existing library file (read from its bytes, not loaded), or
    None."""
    try:
        data = open(path, "rb").read()
    except OSError:
        return None
    i = data.find(b"EFD_BUILD_ID=")
    if i < 0:
        return None
    j = data.find(b"\0", i)
    return data[i + 13:j].decode(errors="replace")


def build(force=False, verbose=False, extra=()):
    """Compile libemrifd.so unless the in-tree one was built from exactly these sources (its
    tagged build id equals source_id(): content, not file times, so a library that travelled
    with the tree is reused only when it matches; anything else is rebuilt)."""
    sid = source_id()
    if not force and not extra and built_id() == sid:
        return OUT
    os.makedirs(OBJDIR, exist_ok=True)
    obj = os.path.join(OBJDIR, "emrifd_cpu.o")
    hobj = os.path.join(OBJDIR, "emrifd_host.o")
    cpu = ["g++", "-O3", f"-march={CPU_ARCH}", "-fopenmp", "-ffp-contract=off", "-fPIC",
           "-std=c++17", "-c", CPU_SRC, "-o", obj]
    host = ["g++", "-O3", f"-march={CPU_ARCH}", "-ffp-contract=off", "-fopenmp", "-fPIC",
            "-std=c++17", "-c", HOST_SRC, "-o", hobj]
    mobj = os.path.join(OBJDIR, "emrifd_modes.o")
    modes = ["g++", "-O3", f"-march={CPU_ARCH}", "-ffast-math", "-fopenmp", "-fPIC",
             "-std=c++17", "-c", MODES_SRC, "-o", mobj]
    bid = [f'-DEFD_BUILD_ID="{sid}"'] if not extra else []
    hip = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", *bid,
           *extra,
           "-o", OUT + ".tmp", obj, hobj, mobj, SRC, "-lgomp", "-lmvec"]
    for cmd in (cpu, host, modes, hip):
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))
