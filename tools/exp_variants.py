"""Kernel experiments: build libemrifd.so variants here (CPU), time them on the GPU box.

    python tools/exp_variants.py build NAME[=SRC][:-DFLAG[=V][,-DFLAG2...]] ...   # here, hipcc only
    python tools/exp_variants.py run NAME ...                              # on the GPU box

`build` writes exp/libemrifd_<NAME>.so (git-ignored, travels with gpurun). `run` loads each
variant in its own child process, runs config 2's full device pipeline, and prints one JSON line
per variant: k_modesum ms (HIP events, mean of 5 launches), the spectrum's max deviation from
the in-tree library's (relative to max|S|), and the -DEFD_EXP counters when compiled in.
The variant named "base" is the in-tree library. EXP_T / EXP_EPS select the workload (default
config 2: T = 2 yr, eps = 1e-5).
"""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXP = os.path.join(ROOT, "exp")
SRC = os.path.join(ROOT, "emri_frequencydomainwaveforms_amd", "csrc", "emrifd.hip")
sys.path.insert(0, ROOT)


NWAVE = 4   # waves per k_modesum workgroup


def lib_path(name):
    if name == "base":
        return os.path.join(ROOT, "emri_frequencydomainwaveforms_amd", "libemrifd.so")
    return os.path.join(EXP, f"libemrifd_{name}.so")


def build(specs):
    from emri_frequencydomainwaveforms_amd import _build
    _build.build()   # the host objects (twin, upstream) every variant links, as the in-tree one
    objs = [os.path.join(_build.OBJDIR, o)
            for o in ("emrifd_cpu.o", "emrifd_host.o", "emrifd_modes.o")]
    os.makedirs(EXP, exist_ok=True)
    procs = []
    for spec in specs:
        name, _, flags = spec.partition(":")
        # NAME=SOURCE: another kernel source (e.g. an earlier revision saved under exp/)
        name, _, src = name.partition("=")
        cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               *[f for f in flags.split(",") if f], "-o", lib_path(name), *objs, src or SRC,
               "-lgomp", "-lmvec"]
        print(" ".join(cmd), flush=True)
        procs.append(subprocess.Popen(cmd))
    if any(p.wait() != 0 for p in procs):
        sys.exit("variant build failed")


def child(name, ref_path):
    import ctypes

    import numpy as np
    import torch

    os.environ["EFD_LIB"] = lib_path(name)
    import bench
    from emri_frequencydomainwaveforms_amd.summation import DeviceInputs, ModeSumEngine

    caustic = os.environ.get("EXP_CAUSTIC", "uniform")
    w = bench.build_workload(T=float(os.environ.get("EXP_T", "2")),
                             eps=float(os.environ.get("EXP_EPS", "1e-5")))
    inp = DeviceInputs.from_host(w["t"], w["amp"], w["phi_phi"], w["phi_r"], w["f_phi"],
                                 w["f_r"], w["m"], w["n"], w["ylm_p"], w["ylm_m"])
    freq = torch.as_tensor(w["freq"], device="cuda")
    S = torch.empty(len(w["freq"]), dtype=torch.complex128, device="cuda")
    eng = ModeSumEngine(caustic=caustic)
    eng.run(inp, freq, out=S, grid_symmetric=True, scale=w["prefactor"])
    lib = eng.lib
    has_cnt = hasattr(lib, "efd_exp_counters")
    st = torch.cuda.current_stream().cuda_stream
    fS = torch.view_as_real(S)
    ms = []
    for _ in range(int(os.environ.get("EXP_REPS", "6"))):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        b.record()
        eng.launch(inp, freq, fS, True, w["prefactor"], stream=st,
                   prof_events=(a.cuda_event, b.cuda_event))
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b))
    out = {"variant": name, "kernel_ms": float(np.mean(ms[1:])), "min_ms": float(min(ms[1:])),
           "ok": bool(eng.status(st))}
    Sh = S.cpu().numpy()
    if ref_path and os.path.exists(ref_path):
        R = np.load(ref_path)
        out["max_rel_dev_vs_base"] = float(np.abs(Sh - R).max() / np.abs(R).max())
    elif name == "base" and ref_path:
        np.save(ref_path, Sh)
    if has_cnt and os.environ.get("EXP_TCLK") and "tclk" in name:
        # per-tile wall clock of the last launch (-DEFD_EXP; 100 MHz s_memrealtime ticks):
        # how much of the launch runs below full tile concurrency (the tail)
        nt_ = min(int(os.environ["EXP_TCLK"]), 16384)
        ev = (ctypes.c_uint * 16384)()
        clk = (ctypes.c_ulonglong * 16384)()
        lib.efd_exp_tiles(ev, clk)
        c = np.frombuffer(clk, dtype=np.uint64)[:nt_]
        st0 = (c >> np.uint64(32)).astype(np.int64)
        dur = (c & np.uint64(0xffffffff)).astype(np.int64)
        # the kernel keeps the low 32 bits of the start (100 MHz: wraps every ~43 s); a launch
        # is far shorter than half a wrap, so start times relative to tile 0, taken modulo 2^32
        # into (-2^31, 2^31], are exact even when the wrap falls inside the launch
        rel = (st0 - st0[0]) % (1 << 32)
        rel = np.where(rel > (1 << 31), rel - (1 << 32), rel)
        st0 = rel - rel.min()
        en = st0 + dur
        span = int(en.max())
        grid = np.arange(0, span + 1, max(span // 400, 1))
        conc = np.array([int(((st0 <= g) & (en > g)).sum()) for g in grid])
        full = conc.max()
        below = grid[conc < 0.5 * full]
        if os.environ.get("EXP_TCLK_OUT"):
            np.savez(os.environ["EXP_TCLK_OUT"] + f"_{name}.npz", start=st0, dur=dur,
                     evals=np.frombuffer(ev, dtype=np.uint32)[:nt_].copy())
        out["tiles"] = {"n": nt_, "span_us": span / 100.0, "sum_tile_us": float(dur.sum()) / 100.0,
                        "max_concurrency": int(full),
                        "mean_tile_us": float(dur.mean()) / 100.0,
                        "max_tile_us": float(dur.max()) / 100.0,
                        "p99_tile_us": float(np.percentile(dur, 99)) / 100.0,
                        "last_start_us": float(st0.max()) / 100.0,
                        "us_below_half_concurrency": float(len(below) * (grid[1] - grid[0])) / 100.0,
                        "longest_tiles": [int(i) for i in np.argsort(dur)[-5:]]}
    if has_cnt:
        cnt = (ctypes.c_ulonglong * 40)()   # EXP_NCOUNT (emrifd.hip, -DEFD_EXP)
        lib.efd_exp_counters(cnt)
        runs = 1 + int(os.environ.get("EXP_REPS", "6"))  # counters accumulate over every launch
        out["counters_per_launch"] = {k: cnt[i] / runs for i, k in enumerate(
            ("record_evals", "cold_evals", "cold_lanes", "skips", "lanes_overshoot",
             "lanes_y_mid", "lanes_y_small", "unused", "y_ge153", "y_ge75", "y_ge48",
             "y_ge29", "y_ge23", "y_ge20", "y_ge18", "y_lt18", "cold_wave_evals", "cold_wave_lanes",
             "ov_lt1e-12", "ov_lt1e-9", "ov_lt1e-6", "ov_lt1e-3", "ov_lt1e-1", "ov_ge1e-1",
             "chunk_max_wave_evals", "chunk_wave_evals", "chunks", "segments",
             "tile_hits", "safe_wave_evals", "unused30", "unused31", "records_j1", "records_j2",
             "records_j3", "records_j4", "subbranch_flips", "off_fast_partial", "off_fast_j3",
             "off_fast_uncertified"))}
        c = out["counters_per_launch"]
        if c["chunk_wave_evals"] > 0:
            # wave-time lost at the chunk barriers if every record evaluation cost the same
            out["barrier_idle_frac"] = 1.0 - c["chunk_wave_evals"] / (NWAVE * c["chunk_max_wave_evals"])
    print("EXPRESULT " + json.dumps(out), flush=True)


def run(names):
    import tempfile
    ref = os.path.join(tempfile.gettempdir(), f"exp_base_S_{os.getpid()}.npy")
    if "base" in names:
        names = ["base"] + [n for n in names if n != "base"]
    for name in names:
        r = subprocess.run([sys.executable, __file__, "child", name, ref], capture_output=True,
                           text=True, timeout=300)
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("EXPRESULT ")]
        if r.returncode != 0 or not lines:
            print(json.dumps({"variant": name, "error": r.returncode,
                              "stderr": r.stderr[-2000:]}), flush=True)
            if r.returncode < 0 or r.returncode in (124, 134, 137, 139):
                sys.exit(1)   # a crash: start nothing more on the GPU
            continue
        print(lines[-1][len("EXPRESULT "):], flush=True)


if __name__ == "__main__":
    cmd, rest = sys.argv[1], sys.argv[2:]
    if cmd == "build":
        build(rest)
    elif cmd == "run":
        run(rest)
    elif cmd == "child":
        child(rest[0], rest[1] if len(rest) > 1 else None)
    else:
        sys.exit(__doc__)
