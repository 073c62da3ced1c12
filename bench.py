"""Benchmark: FD EMRI waveforms/s on MI355X (BASELINE.json metric, config 2).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[1]): M = 1e6, mu = 10, e0 = 0.35,
p0 solved so the inspiral lasts 0.99 * Tobs (README's p0 = 12 is overwritten like
emri_pe.py:623-635), Tobs = 2 yr, dt = 10 s (N_f = 6,311,631 two-sided bins), eps = 1e-5
(~3000 harmonics), K_{1/3} uniform SPA (the reference notebook's form). Inputs (sparse
trajectory, amplitudes, Ylm; host stand-ins, NOT FEW physics) are resident in HBM before timing.
One step = a batch of B (--batch, default 8) full FD waveforms on the device, each with its own
workspace and outputs: spline build -> inverse splines -> interval records -> tile lists -> mode
sum -> h+/hx over f >= 0 (the Likelihood path, emri_pe.py:241, for a batch of walkers). With
--pipeline overlap (default) batch i+1's preparation (grouping, splines, records: latency-bound
kernels on few CUs; one efd_modesum_prepare_batch for the B waveforms) runs on a second stream
beside batch i's
mode sums, which run as one launch (efd_modesum_sum_batch: the B waveforms' tiles in one
longest-first dispatch) and write h+/hx themselves (fused polarisations). value counts
waveforms (B per step); --batch 1 runs one efd_modesum_sum per waveform. B = 8 since round 4's
768-lane tiles (paired A/B against 2 / 4 / 6 / 12 / 16: 0.951 / 0.987 / 0.997 / 0.997 / 0.997,
profiles/r04_ab_batch.jsonl); round 3's 512-lane tiles were best at 4.

Multi-GPU: one process per GPU; each rank generates its own waveforms (the walker batch of
emri_pe.py shards with no data-path exchange: weak scaling); value = all ranks' waveforms / the
max over ranks of the timed region.

roofline: the mode-sum kernel (k_modesum_batch, or k_modesum at --batch 1) timed with HIP events
recorded on its own stream around each launch in the timed region. The kernel is bound by the
FP64 vector ALU (output-stationary: each bin written once, ~0.27 GB of HBM traffic per
waveform), so bound = "fp64_valu": achieved = FP64 FLOP per launch (rocprofv3 PMC counters of
the committed profile, per SPA evaluation, times this run's evaluations) / launch time, peak
78.6 TFLOP/s. traffic: HBM bytes per launch from the same PMC pass. SURVEY.md section 8d's
scatter-formulation bytes (32 B per SPA contribution) are reported as scatter_equiv_gbs, a
secondary figure: the kernel never issues that traffic.

few_gen: the drivers' whole GenerateEMRIWaveform call on the same source, one at a time (host
upstream + device pipeline; rank 0 at N = 1), next to the batched device rate.

cpu_baseline: the host twin efd_modesum_cpu (the same algorithm in C++17 + OpenMP, kind "twin")
on this host: all cores on full waveforms, and 1 thread on a subset of harmonics extrapolated by
SPA evaluation count (single_thread). cpu_reference: the oracle's C restatement (per harmonic
and bin, the notebook's construction; the checker) on a subset, extrapolated by contribution
count. Rank 0 at N = 1 only.
"""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "FD waveforms/sec (2 yr, dt=10 s, ~3000 modes) at 1/2/4/8 GPUs; mode-sum HBM GB/s"
HBM_PEAK_GBS = 8000.0
FP64_VALU_PEAK_TFLOPS = 78.6   # MI355X vector FP64 peak (AMD spec: 256 CUs x 128 FLOP/clk x 2.4 GHz)


def build_workload(T=2.0, dt=10.0, eps=1e-5, M=1e6, mu=10.0, e0=0.35, theta=np.pi / 3,
                   phi=-np.pi / 2, dist=1.0, p0=None, Phi_phi0=0.0, Phi_r0=0.0):
    from emri_frequencydomainwaveforms_amd.amplitude import ModeSelector, SyntheticTeukolskyAmplitude
    from emri_frequencydomainwaveforms_amd.constants import Gpc, MRSUN_SI, MTSUN_SI
    from emri_frequencydomainwaveforms_amd.frequencies import get_fundamental_frequencies
    from emri_frequencydomainwaveforms_amd.summation import fd_grid
    from emri_frequencydomainwaveforms_amd.trajectory import EMRIInspiral, get_p_at_t
    from emri_frequencydomainwaveforms_amd.ylm import GetYlms

    traj = EMRIInspiral()
    if p0 is None:
        p0 = get_p_at_t(traj, 0.99 * T, [M, mu, 0.0, e0, 1.0])
    t, p, e, x, pp, pt, pr = traj(M, mu, 0.0, p0, e0, 1.0, Phi_phi0=Phi_phi0, Phi_r0=Phi_r0, T=T)
    amp = SyntheticTeukolskyAmplitude()
    A = amp(p, e)
    ylms = GetYlms(assume_positive_m=True)(amp.l_arr, amp.m_arr, theta, phi)
    keep = ModeSelector(amp.m0mask)(A, ylms, None, eps=eps)
    Kall = amp.num_teuk_modes
    op, _, orr = get_fundamental_frequencies(0.0, p, e, 0.0)
    return dict(t=t, amp=np.ascontiguousarray(A[:, keep]), phi_phi=pp, phi_r=pr,
                f_phi=op / (2 * np.pi * M * MTSUN_SI), f_r=orr / (2 * np.pi * M * MTSUN_SI),
                m=amp.m_arr[keep].astype(np.int32), n=amp.n_arr[keep].astype(np.int32),
                ylm_p=ylms[:Kall][keep], ylm_m=ylms[Kall:][keep],
                prefactor=mu * MRSUN_SI / (dist * Gpc), freq=fd_grid(T, dt),
                params=dict(M=M, mu=mu, p0=float(p0), e0=e0, T=T, dt=dt, eps=eps,
                            Phi_phi0=Phi_phi0, Phi_r0=Phi_r0))


def build_workloads(B, T=2.0, dt=10.0, eps=1e-5, sources="walkers", seed=2601996):
    """B config-2 sources: the source itself, then (sources="walkers") B - 1 draws of emri_pe.py's
    walker start around it, multivariate_normal(truth, cov(covariance.npy) / (2.4 * 6)) in
    (ln M, ln(mu/M), p0, e0, Phi_phi0, Phi_r0) (emri_pe.py:437-444; the covariance is the
    package's data/walker_cov.npy, numpy's Generator with the reference's seed): distinct
    waveforms, each with its own trajectory, harmonic selection and records, as a walker batch
    of the sampler is. sources="same": B copies of the source (rounds 1-3's headline)."""
    w0 = build_workload(T=T, dt=dt, eps=eps)
    if sources == "same" or B == 1:
        return [w0] * B
    from emri_frequencydomainwaveforms_amd import pe
    P = w0["params"]
    truth6 = np.array([np.log(P["M"]), np.log(P["mu"] / P["M"]), P["p0"], P["e0"], 0.0, 0.0])
    cov = np.load(pe._COV, allow_pickle=False) / (2.4 * 6)
    draws = np.random.default_rng(seed).multivariate_normal(truth6, cov, size=B - 1)
    out = [w0]
    for lnM, lnq, p0, e0, pp0, pr0 in draws:
        M = float(np.exp(lnM))
        out.append(build_workload(T=T, dt=dt, eps=eps, M=M, mu=float(M * np.exp(lnq)),
                                  e0=float(e0), p0=float(p0), Phi_phi0=float(pp0),
                                  Phi_r0=float(pr0)))
    return out


# The fixed algorithmic count of the FP64 roofline: FP64 FLOP per SPA evaluation, frozen at the
# value the round-4 end kernel executed (profiles/r04h_pmc.json: (ADD + MUL + 2 FMA + TRANS)_F64
# wave-instructions x 64 lanes x lane utilisation / evaluations = 51.547). An evaluation is one
# (group branch, grid bin) pair (the workspace header's count, set by k_items from the records'
# lane ranges), so evaluations x 51.5 is a property of the workload, not of the kernel build: a
# cut in per-evaluation work shows as a gain in frac instead of a loss.
FLOP_PER_EVAL_FIXED = 51.5


def fp64_roofline(B, n_eval, kern_ms, caustic, sources="walkers"):
    """FP64 VALU roofline of the mode-sum kernel over the 78.6 TFLOP/s vector FP64 peak.

    achieved / frac: the fixed algorithmic count, FLOP_PER_EVAL_FIXED x this launch's SPA
    evaluations / this run's kernel time (HIP events). pmc_instructions: the executed-instruction
    figure beside it, FLOP per evaluation from the committed rocprofv3 PMC pass
    (profiles/pmc_traffic.json, written by tools/summarize_profiles.py: FP64 FMA counts 2,
    MUL/ADD/TRANS 1, times 64 lanes x measured lane utilisation; pmc_matches_build says whether
    that pass was taken on the kernel source being timed). traffic: HBM bytes per launch of the
    same PMC pass (2 FETCH_SIZE + WRITE_SIZE, gfx950 correction)."""
    import hashlib
    flops = FLOP_PER_EVAL_FIXED * n_eval   # n_eval: the launch's SPA evaluations (all B waveforms)
    tf = flops / (kern_ms * 1e-3) / 1e12
    out = {"bound": "fp64_valu", "achieved": tf, "peak": FP64_VALU_PEAK_TFLOPS,
           "unit": "TFLOP/s", "frac": tf / FP64_VALU_PEAK_TFLOPS, "traffic": None,
           "flops_per_launch": flops, "flops_per_evaluation": FLOP_PER_EVAL_FIXED,
           "flops_count": "fixed algorithmic count: 51.5 FP64 FLOP per SPA evaluation "
                          "(profiles/r04h_pmc.json) x evaluations per launch"}
    prof = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(prof):
        return out
    try:
        pj = json.load(open(prof))
        f = pj.get("fp64") or {}
        fpe = f.get("flops_per_evaluation")
        if fpe is None and f.get("flops_per_launch") and pj.get("evaluations_per_launch"):
            fpe = f["flops_per_launch"] / pj["evaluations_per_launch"]
        if fpe is None or pj.get("caustic") != caustic:
            return out
        src = os.path.join(ROOT, "emri_frequencydomainwaveforms_amd", "csrc", "emrifd.hip")
        sha = hashlib.sha256(open(src, "rb").read()).hexdigest()[:16]
        tfi = fpe * n_eval / (kern_ms * 1e-3) / 1e12
        out["pmc_instructions"] = {
            "achieved": tfi, "frac": tfi / FP64_VALU_PEAK_TFLOPS, "flops_per_evaluation": fpe,
            "valu_busy": f.get("valu_busy"), "fp64_share_of_valu_insts":
                f.get("fp64_share_of_valu_insts"), "effective_clock_ghz": pj.get("clock_ghz"),
            "pmc_source": pj.get("source"), "pmc_matches_build": pj.get("src_sha16") == sha}
        if (int(pj.get("batch", 1)) == B and pj.get("workload") == "config2"
                and pj.get("sources", "same") == sources):
            out["traffic"] = pj.get("hbm_bytes_per_launch")
            out["traffic_write"] = pj.get("write_bytes_per_launch")
    except (ValueError, OSError, KeyError, TypeError):
        pass
    return out


def library_info(lib):
    """Which libemrifd.so was timed: its compiled-in build id against the hash of the sources in
    this tree (emri_frequencydomainwaveforms_amd/_build.source_id)."""
    from emri_frequencydomainwaveforms_amd import _build
    bid = lib.efd_build_id().decode()
    return {"build_id": bid, "sources_id": _build.source_id(),
            "matches_sources": bid == _build.source_id()}


def world_size(gpus):
    """The rank count: WORLD_SIZE from the launcher (torch.distributed.run), which must equal
    --gpus. A multi-GPU figure needs the launcher (one process per GPU); `bench.py --gpus 8`
    started without it would time one GPU and print a valid-looking n_gpus = 1 line, so any
    mismatch exits non-zero before touching a GPU."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if gpus != world:
        sys.stderr.write(
            f"bench.py: --gpus {gpus} but WORLD_SIZE={world}: launch one process per GPU with "
            f"python -m torch.distributed.run --nnodes=1 --nproc-per-node {gpus} "
            f"--master-addr 127.0.0.1 --master-port P bench.py --gpus {gpus} ...\n")
        raise SystemExit(2)
    return world


def cpu_baseline(w, seconds=10.0):
    """The host twin (efd_modesum_cpu: the same algorithm as the HIP path in C++17 + OpenMP,
    AVX-512) timed on this box's host cores: all cores on the full waveform (1 warm-up + 3 timed,
    median), and 1 thread on a subset of harmonics sized to ~`seconds`, extrapolated by SPA
    evaluation count (the twin's cost is per evaluation). SURVEY.md section 8(d)."""
    from emri_frequencydomainwaveforms_amd import cputwin
    threads = len(os.sched_getaffinity(0))
    threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))

    def run(sel):
        return cputwin.modesum(w["t"], w["amp"][:, sel], w["phi_phi"], w["phi_r"], w["f_phi"],
                               w["f_r"], w["m"][sel], w["n"][sel], w["ylm_p"][sel],
                               w["ylm_m"][sel], w["freq"], w["prefactor"])
    allh = np.arange(len(w["m"]))
    prev = cputwin.set_threads(threads)
    try:
        run(allh)
        _, ev_all, _ = cputwin.stats()
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            run(allh)
            ts.append(time.perf_counter() - t0)
        t_all = float(np.median(ts))
        cputwin.set_threads(1)
        order = np.argsort(-np.abs(w["amp"]).max(axis=0))   # strongest harmonics first
        k = 16
        while True:
            sel = np.sort(order[:k])
            t0 = time.perf_counter()
            run(sel)
            dt = time.perf_counter() - t0
            _, ev_s, _ = cputwin.stats()
            if dt > 0.5 * seconds or k >= len(order):
                break
            k = min(len(order), int(k * max(2.0, 0.8 * seconds / max(dt, 1e-3))))
    finally:
        cputwin.set_threads(prev)
    one = ev_s / dt / ev_all
    return {"value": 1.0 / t_all, "unit": "waveforms/s", "cores": threads, "kind": "twin",
            "sample": f"full config-2 waveform (3,020 harmonics, {ev_all} SPA evaluations), "
                      f"median of 3 after a warm-up, {t_all:.3f} s each on {threads} threads",
            "single_thread": {"value": one, "unit": "waveforms/s", "cores": 1,
                              "sample": f"{k} of {len(order)} harmonics ({ev_s} of {ev_all} SPA "
                                        f"evaluations) in {dt:.1f} s on 1 thread, extrapolated "
                                        f"by evaluation count"},
            "implementation": "efd_modesum_cpu (csrc/emrifd_cpu.cpp): the HIP path's algorithm "
                              "on the host, C++17 + OpenMP, -O3 -march=x86-64-v4"}


def _host_threads():
    threads = len(os.sched_getaffinity(0))
    return min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))


def twin_job_rate(jobs, unit, seconds=10.0, what=""):
    """The host twin over a list of jobs (BASELINE.md section 2's CPU column for configs 1, 3, 4
    and 5), each job one waveform or one walker's log-likelihood: job() runs it on the host
    (efd_modesum_cpu writing h+/hx over f >= 0 as the device path does, + efd_loglike_cpu for a
    likelihood). All of this rank's cores (the twin's OpenMP over tiles; one warm-up job, then
    the jobs in order until `seconds` or the list ends) and 1 thread (the jobs in order until
    seconds / 2, at least one). The reference's CPU path is the same per-walker loop
    (likelihood.py:246-248), there under mp.Pool(4) (emri_pe.py:545)."""
    from emri_frequencydomainwaveforms_amd import cputwin
    threads = _host_threads()

    def timed(budget):
        n, t0 = 0, time.perf_counter()
        for job in jobs:
            job()
            n += 1
            if time.perf_counter() - t0 > budget:
                break
        return n, time.perf_counter() - t0
    prev = cputwin.set_threads(threads)
    try:
        jobs[0]()
        n_all, t_all = timed(seconds)
        cputwin.set_threads(1)
        n_one, t_one = timed(0.5 * seconds)
    finally:
        cputwin.set_threads(prev)
    return {"value": n_all / t_all, "unit": unit, "cores": threads, "kind": "twin",
            "sample": f"{n_all} of {len(jobs)} {what} in {t_all:.2f} s on {threads} threads",
            "single_thread": {"value": n_one / t_one, "unit": unit, "cores": 1,
                              "sample": f"{n_one} of {len(jobs)} {what} in {t_one:.2f} s on "
                                        f"1 thread"},
            "implementation": "efd_modesum_cpu (+ efd_loglike_cpu): the HIP path's algorithm "
                              "on the host (csrc/emrifd_cpu.cpp, C++17 + OpenMP, -O3 "
                              "-march=x86-64-v4), host upstream prepared beforehand"}


def twin_waveform_job(w):
    """One waveform of a workload dict (build_workload) on the twin: h+/hx over f >= 0."""
    from emri_frequencydomainwaveforms_amd import cputwin
    k0 = int(np.searchsorted(w["freq"], 0.0))

    def job():
        cputwin.modesum(w["t"], w["amp"], w["phi_phi"], w["phi_r"], w["f_phi"], w["f_r"],
                        w["m"], w["n"], w["ylm_p"], w["ylm_m"], w["freq"], w["prefactor"],
                        polarizations=True, k0=k0)
    return job


def twin_likelihood_jobs(s, rows):
    """One job per walker of `rows` (sampled coordinates) for pe.setup's likelihood `s`: the
    walker's template on the twin (its host upstream prepared here, untimed, as the device
    rate's memoised one) and efd_loglike_cpu against the likelihood's own d and w. Returns
    (jobs, logL list the jobs fill)."""
    from emri_frequencydomainwaveforms_amd import cputwin
    from emri_frequencydomainwaveforms_amd.constants import Gpc, MRSUN_SI
    from emri_frequencydomainwaveforms_amd.summation import fd_grid
    from emri_frequencydomainwaveforms_amd.waveform import get_viewing_angles, polarization_angle
    kw = s.kwargs
    grid = np.asarray(kw["f_arr"]) if kw.get("f_arr") is not None else fd_grid(kw["T"], kw["dt"])
    k0 = int(np.searchsorted(grid, 0.0))
    d = s.like._d.cpu().numpy()
    w = s.like._w_templ.cpu().numpy()
    few = s.few
    wg = few.waveform_generator
    out = [None] * len(rows)
    jobs = []
    for i, p14 in enumerate(s.transform.both_transforms(np.asarray(rows))):
        M, mu, _a, p0, e0, _x0, dist, qS, phiS, qK, phiK, pp0, _pt0, pr0 = (float(v) for v in p14)
        theta, phi = get_viewing_angles(qS, phiS, qK, phiK)
        rot = (np.exp(-2j * polarization_angle(qS, phiS, qK, phiK))
               if getattr(few, "frame", None) == "detector" else 1.0)
        u = wg.prepare(M, mu, p0, e0, theta, phi, dist, pp0, pr0, kw["T"], kw["eps"])
        K = len(u["m"])
        scale = complex(rot) * (mu * MRSUN_SI / (dist * Gpc))

        def job(i=i, u=u, K=K, scale=scale):
            hp, hc = cputwin.modesum(u["t"], u["teuk"], u["Phi_phi"], u["Phi_r"], u["f_phi"],
                                     u["f_r"], u["m"], u["n"], u["ylms"][:K], u["ylms"][K:],
                                     grid, scale, polarizations=True, k0=k0)
            out[i] = cputwin.loglike(np.stack([hp, hc]), d, w)
        jobs.append(job)
    return jobs, out


def few_gen_timing(w, reps=10, caustic="uniform"):
    """The drivers' whole call (events around the full few_gen-equivalent
    call; check_mode_by_mode.py:221-229 times `few_gen(*injection_in, **kw)`): the
    GenerateEMRIWaveform("FastSchwarzschildEccentricFlux", output_type="fd") call on config 2's
    source, host upstream (the C++ stand-in trajectory, amplitudes and selection: NOT FEW
    physics) + upload + preparation + mode sum, the two-sided spectrum on the device. 1 warm-up
    + `reps` calls, each bracketed by HIP events on the current stream and a host clock around
    the call and its synchronisation; medians."""
    import torch
    from emri_frequencydomainwaveforms_amd.waveform import GenerateEMRIWaveform
    few = GenerateEMRIWaveform("FastSchwarzschildEccentricFlux",
                               sum_kwargs=dict(pad_output=True, output_type="fd", odd_len=True),
                               use_gpu=True, return_list=False, caustic=caustic)
    P = w["params"]
    # M, mu, a, p0, e0, x0, dist, qS, phiS, qK, phiK, Phi_phi0, Phi_theta0, Phi_r0; the sky and
    # spin angles put the source-frame viewing angles at the workload's (theta, phi) = (pi/3,
    # -pi/2): -R.S = cos(pi/3), so the same ~3,000 harmonics survive eps = 1e-5
    args = (P["M"], P["mu"], 0.0, P["p0"], P["e0"], 1.0, 1.0, np.pi / 3, 0.0, np.pi / 3, np.pi,
            0.0, 0.0, 0.0)
    kw = dict(T=P["T"], dt=P["dt"], eps=P["eps"])
    S = few(*args, **kw)
    torch.cuda.synchronize()
    wall, dev = [], []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record()
        S = few(*args, **kw)
        b.record()
        torch.cuda.synchronize()
        wall.append(time.perf_counter() - t0)
        dev.append(a.elapsed_time(b) * 1e-3)
    ms = float(np.median(wall)) * 1e3
    return {"value": 1e3 / ms, "unit": "waveforms/s", "ms_per_call": ms,
            "events_ms_per_call": float(np.median(dev)) * 1e3, "reps": reps,
            "harmonics": int(len(few.waveform_generator.last_modes[0])), "bins": int(S.numel()),
            "note": "GenerateEMRIWaveform(...)(14 params, T=2, dt=10, eps=1e-5): host stand-in "
                    "upstream (C++, one call at a time) + device pipeline, serial; the batch "
                    "value overlaps many waveforms and excludes the upstream"}


def cpu_reference(w, seconds=5.0):
    """The oracle's C restatement (oracle/fd_oracle_c.c: per harmonic, per bin, the reference
    notebook's construction) on a bounded subset of harmonics, extrapolated by contribution count:
    the checker, timed for reference (it is not the same algorithm as the twin)."""
    from oracle import fd_oracle, fd_oracle_c
    if fd_oracle_c.load() is None:
        return None
    threads = len(os.sched_getaffinity(0))
    threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))
    C_total = fd_oracle.contributions(w["t"], w["f_phi"], w["f_r"], w["m"], w["n"], w["freq"])
    order = np.argsort(-np.abs(w["amp"]).max(axis=0))
    k = 8
    while True:
        sel = order[:k]
        C_s = fd_oracle.contributions(w["t"], w["f_phi"], w["f_r"], w["m"][sel], w["n"][sel],
                                      w["freq"])
        t0 = time.perf_counter()
        fd_oracle_c.modesum(w["t"], w["amp"][:, sel].T, w["phi_phi"], w["phi_r"], w["f_phi"],
                            w["f_r"], w["m"][sel], w["n"][sel], w["ylm_p"][sel], w["ylm_m"][sel],
                            w["freq"], w["prefactor"], caustic="uniform", nthreads=threads)
        dt = time.perf_counter() - t0
        if dt > 0.5 * seconds or k >= len(order):
            break
        k = min(len(order), int(k * max(2.0, 0.8 * seconds / max(dt, 1e-3))))
    return {"value": C_s / dt / C_total, "unit": "waveforms/s", "cores": threads, "kind": "port",
            "sample": f"{k} of {len(order)} harmonics ({C_s} of {C_total} contributions) in "
                      f"{dt:.1f} s on {threads} threads, extrapolated by contribution count"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--caustic", default="uniform", choices=["uniform", "spa"])
    ap.add_argument("--T", type=float, default=2.0)
    ap.add_argument("--eps", type=float, default=1e-5)
    ap.add_argument("--sources", default="walkers", choices=["walkers", "same"],
                    help="the B waveforms of a step: distinct sources from emri_pe.py's walker "
                         "start around config 2's (default), or B copies of config 2's source")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pipeline", default="overlap", choices=["overlap", "serial"],
                    help="overlap: prepare(i+1) on a second stream beside sum(i), fused h+/hx; "
                         "serial: one stream, efd_modesum + efd_polarizations")
    ap.add_argument("--sum-streams", type=int, default=1,
                    help="overlap pipeline: consecutive mode sums alternate over this many streams "
                         "(> 1 lets sum i+1 start during sum i's tail)")
    ap.add_argument("--slots", type=int, default=2,
                    help="overlap pipeline depth: batches in flight (preparation runs up to "
                         "slots - 1 batches ahead of the sum)")
    ap.add_argument("--batch", type=int, default=8,
                    help="overlap pipeline: waveforms per step, their mode sums in one launch "
                         "(efd_modesum_sum_batch; 1 = one efd_modesum_sum per waveform)")
    ap.add_argument("--prep", default="batch", choices=["single", "batch"],
                    help="overlap pipeline: one efd_modesum_prepare_batch over the step's B "
                         "waveforms (9 launches per step), or each waveform's "
                         "efd_modesum_prepare (round 2; 0.993x, 4 paired rounds)")
    ap.add_argument("--sum-priority", type=int, default=0,
                    help="overlap pipeline: torch stream priority of the sum stream (negative = "
                         "higher; the preparation stream keeps the default)")
    ap.add_argument("--prep-priority", type=int, default=0,
                    help="overlap pipeline: torch stream priority of the preparation stream "
                         "(negative = higher)")
    ap.add_argument("--diag-sum-only", action="store_true",
                    help="diagnostic, not the metric: each slot is prepared once in the warm-up, "
                         "then every step runs only the mode sum (the sum-stream ceiling)")
    ap.add_argument("--likelihood", choices=["config4", "config5"], default=None,
                    help="time emri_pe.py's likelihood instead (BASELINE configs 4 / 5): walker "
                         "half-steps through Likelihood (fused mode sum + logL), sharded over the "
                         "ranks by ShardedLikelihood (parameter broadcast + logL all-gather)")
    ap.add_argument("--fused-group", type=int, default=0,
                    help="--likelihood: walkers per fused group (Likelihood.FUSED_GROUP; 0 = its "
                         "default)")
    ap.add_argument("--no-tile-constants", action="store_true",
                    help="--likelihood: empty tiles recompute their logL partial (the A/B "
                         "baseline of efd_loglike_tile_constants)")
    ap.add_argument("--scan", choices=["config3"], default=None,
                    help="time BASELINE config 3's 10x10 (M, e0) scan instead: points round-robin "
                         "over the ranks (parallel.ShardedScan), each rank's p0 solves, host "
                         "upstream and batched device work, per-point records all-gathered")
    ap.add_argument("--api-steps", type=int, default=2,
                    help="--likelihood: half-steps timed with the host upstream in the loop")
    args = ap.parse_args()
    world_size(args.gpus)

    import torch
    import torch.distributed as dist

    if args.likelihood:
        return bench_likelihood(args)
    if args.scan:
        return bench_scan(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", torch.cuda.current_device())

    from emri_frequencydomainwaveforms_amd import _lib
    from emri_frequencydomainwaveforms_amd.summation import (DeviceInputs, ModeSumEngine,
                                                             prepare_batch, sum_batch)

    overlap = args.pipeline == "overlap"
    B = args.batch if overlap else 1
    if not 1 <= B <= _lib.EFD_BATCH_MAX:
        raise SystemExit(f"--batch must be in [1, {_lib.EFD_BATCH_MAX}]")
    ws = build_workloads(B, T=args.T, eps=args.eps, sources=args.sources)
    w = ws[0]
    inps = []
    for wj in ws:
        if inps and wj is ws[0]:
            inps.append(inps[0])
            continue
        inps.append(DeviceInputs.from_host(wj["t"], wj["amp"], wj["phi_phi"], wj["phi_r"],
                                           wj["f_phi"], wj["f_r"], wj["m"], wj["n"], wj["ylm_p"],
                                           wj["ylm_m"], device=dev))
    inp = inps[0]
    freq = torch.as_tensor(w["freq"], device=dev)
    nf = int(freq.numel())
    k0 = int(np.searchsorted(w["freq"], 0.0))
    # Slots of B waveforms (a workspace + h+/hx outputs each). "overlap": batch i+1's
    # preparation (grouping, splines, records: latency-bound kernels on few CUs) runs on the prep
    # stream while batch i's mode sums run on the sum stream, all B in one launch
    # (efd_modesum_sum_batch: one ramp, one tail, no gaps between the B sums); the sums write
    # h+/hx directly (fused polarisations). Every waveform is prepared and summed in full.
    # "serial": one stream, efd_modesum then efd_polarizations (the unfused path).
    slots = []
    for _ in range(max(2, args.slots) if overlap else 1):
        wf = []
        for _ in range(B):
            hp = torch.empty(nf - k0, dtype=torch.complex128, device=dev)
            wf.append(dict(eng=ModeSumEngine(caustic=args.caustic), fhp=torch.view_as_real(hp),
                           fhc=torch.view_as_real(torch.empty_like(hp)),
                           fS=None if overlap else torch.view_as_real(
                               torch.empty(nf, dtype=torch.complex128, device=dev))))
        slots.append(dict(wf=wf, prep_done=torch.cuda.Event(), sum_done=None))
    lib = slots[0]["wf"][0]["eng"].lib
    s_prep = torch.cuda.Stream(dev, priority=args.prep_priority)
    s_sums = [torch.cuda.Stream(dev, priority=args.sum_priority)
              for _ in range(max(1, args.sum_streams))] if overlap else [s_prep]
    s_sum = s_sums[0]

    def step(i, ev=None):
        sl = slots[i % len(slots)]
        pe = (ev[0].cuda_event, ev[1].cuda_event) if ev is not None else (None, None)
        if overlap:
            ss = s_sums[i % len(s_sums)]
            if not (args.diag_sum_only and i >= len(slots)):
                if sl["sum_done"] is not None:    # the slot's previous sums have read it
                    s_prep.wait_event(sl["sum_done"])
                if args.prep == "batch":
                    prepare_batch([(x["eng"], dict(inp=inps[j], freq=freq, out=None,
                                                   grid_symmetric=True,
                                                   scale=ws[j]["prefactor"]))
                                   for j, x in enumerate(sl["wf"])], stream=s_prep.cuda_stream)
                else:
                    for j, x in enumerate(sl["wf"]):
                        x["eng"].launch(inps[j], freq, None, True, ws[j]["prefactor"],
                                        stream=s_prep.cuda_stream, phase="prepare")
                sl["prep_done"].record(s_prep)
                ss.wait_event(sl["prep_done"])
            if B == 1:
                x = sl["wf"][0]
                x["eng"].launch(inp, freq, None, True, w["prefactor"], stream=ss.cuda_stream,
                                prof_events=pe, hp=x["fhp"], hc=x["fhc"], k0=k0, phase="sum")
            else:
                sum_batch([(x["eng"], dict(inp=inps[j], freq=freq, out=None, grid_symmetric=True,
                                           scale=ws[j]["prefactor"], hp=x["fhp"], hc=x["fhc"],
                                           k0=k0)) for j, x in enumerate(sl["wf"])],
                          stream=ss.cuda_stream, prof_events=pe)
            done = torch.cuda.Event()
            done.record(ss)
            sl["sum_done"] = done
        else:
            st = s_prep.cuda_stream
            x = sl["wf"][0]
            x["eng"].launch(inp, freq, x["fS"], True, w["prefactor"], stream=st, prof_events=pe)
            _lib.check(lib.efd_polarizations(x["fS"].data_ptr(), nf, k0, x["fhp"].data_ptr(),
                                             x["fhc"].data_ptr(), st), "efd_polarizations", lib)

    evs = []
    for i in range(args.steps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s_sums[i % len(s_sums)])   # creates the events; the library re-records them
        b.record(s_sums[i % len(s_sums)])   # around k_modesum
        evs.append((a, b))
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i, evs[i])
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    for sl in slots:
        for x in sl["wf"]:
            if not x["eng"].status(s_sum.cuda_stream):
                raise RuntimeError(f"efd_modesum reported a device error: {_lib.last_error(lib)}")
    # per-launch k_modesum duration, live over the timed region (HIP events on the sum stream;
    # with the overlap pipeline the next waveform's preparation kernels share the GPU with it)
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    # idle time of the sum stream between consecutive mode sums (the next sum's start waits for
    # its preparation and for the launch): what the pipeline loses beside the kernel itself
    gaps = [evs[i][1].elapsed_time(evs[i + 1][0]) for i in range(len(evs) - 1)]
    gap_ms = float(np.mean(gaps)) if gaps else 0.0
    # contributions, SPA evaluations and (m, n) groups of one launch (the B waveforms of a slot)
    st_all = [x["eng"].stats(s_sum.cuda_stream) for x in slots[0]["wf"]]
    C = sum(s_[0] for s_ in st_all)
    n_eval = sum(s_[1] for s_ in st_all)
    n_groups = [s_[2] for s_ in st_all]
    n_env = sum(x["eng"].env_evaluations(s_sum.cuda_stream) for x in slots[0]["wf"])

    rank_elapsed = [elapsed]
    if world > 1:
        # every rank's own timed region (the line's value takes the slowest: max over ranks)
        mine = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        allr = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        rank_elapsed = [float(x) for x in allr]
        tt = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(tt[0]), float(tt[1])

    if rank == 0:
        Ks = [int(len(wj["m"])) for wj in ws]
        nts = [int(len(wj["t"])) for wj in ws]
        # SURVEY 8(d)'s algorithmic bytes of the launch's B waveforms (C summed over them)
        b_alg = 32.0 * C + sum(32.0 * (2 * K_ + 4) * nt_ for K_, nt_ in zip(Ks, nts)) \
            + 16.0 * nf * B
        wf_ms = kern_ms / B   # one launch sums B waveforms
        # SURVEY 8(d)'s scatter-formulation bytes: a secondary figure, never the roofline (the
        # output-stationary kernel never makes those accesses, so it exceeds HBM "peak")
        scatter_gbs = b_alg / (kern_ms * 1e-3) / 1e9
        roof = fp64_roofline(B, n_eval, kern_ms, args.caustic, args.sources)
        cpu = cpu_ref = api = None
        if world == 1 and not args.no_cpu_baseline:
            try:
                api = few_gen_timing(w, caustic=args.caustic)
            except Exception as exc:  # not part of the metric: never kill the GPU measurement
                api = {"value": None, "error": repr(exc)}
            try:
                cpu = cpu_baseline(w, seconds=args.cpu_seconds)
            except Exception as exc:  # the baseline must not kill the GPU measurement
                cpu = {"value": None, "error": repr(exc)}
            try:
                cpu_ref = cpu_reference(w)
            except Exception as exc:
                cpu_ref = {"value": None, "error": repr(exc)}
        value = world * args.steps * B / elapsed
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "waveforms/s",
            "n_gpus": world,
            "world_size_rccl": dist.get_world_size() if world > 1 else 1,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "rank_ms_per_step": {"min": min(rank_elapsed) / args.steps * 1e3,
                                 "max": max(rank_elapsed) / args.steps * 1e3,
                                 "per_rank": [x / args.steps * 1e3 for x in rank_elapsed]},
            "waveforms_per_step": B,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (stand-in trajectory/amplitudes; FEW data absent offline)",
            "config": {"workload": "config2: M=1e6 mu=10 e0=0.35 Tobs=2yr dt=10s eps=1e-5 "
                                   f"caustic={args.caustic}",
                       "sources": ("config 2's source + emri_pe walker-start draws "
                                   "(emri_pe.py:437-444)" if args.sources == "walkers"
                                   else "B copies of config 2's source"),
                       "harmonics": Ks, "mn_groups": n_groups, "N_t": nts, "N_f": nf,
                       "contributions_per_launch": C, "spa_evaluations_per_launch": n_eval,
                       "envelope_evaluations_per_launch": n_env,
                       "envelope_share": n_env / n_eval if n_eval else 0.0,
                       "p0": w["params"]["p0"], "parallelism": f"walkers x{world} (no exchange)",
                       "pipeline": args.pipeline + (" (diagnostic: sum only)"
                                                    if args.diag_sum_only else ""),
                       "slots": len(slots), "sum_streams": len(s_sums), "batch": B,
                       "prep": args.prep},
            "roofline": dict(roof, **{
                "kernel": "k_modesum_batch" if B > 1 else "k_modesum",
                "kernel_ms": kern_ms, "kernel_ms_per_waveform": wf_ms,
                "waveforms_per_launch": B,
                "kernel_timing": "HIP events around each k_modesum launch in the timed region "
                                 "(sum stream), mean",
                "spa_evaluations_per_s": n_eval / (kern_ms * 1e-3),
                "contributions_per_s": C / (kern_ms * 1e-3),
                "scatter_equiv_gbs": scatter_gbs,
                "scatter_equiv_note": "SURVEY 8(d) B_alg = 32 C + 32 n_interp N_t + 16 N_f per "
                                      "waveform / kernel time: the reference scatter "
                                      "formulation's traffic, which this kernel never issues "
                                      "(not an HBM roofline)",
                "sum_gap_ms": gap_ms}),
            "cpu_baseline": cpu,
            "cpu_reference": cpu_ref,
            "few_gen": api,
            "library": library_info(lib),
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


LIKE_CONFIGS = {
    # emri_pe.py -Tobs 2 -eps 1e-2 -injectFD 1 -template fd -nwalkers 16 -ntemps 1 (README)
    "config4": dict(Tobs=2.0, dt=10.0, eps=1e-2, nwalkers=16, ntemps=1),
    # ... -downsample 100 -Tobs 4 -nwalkers 128 (BASELINE configs[4])
    "config5": dict(Tobs=4.0, dt=10.0, eps=1e-2, nwalkers=128, ntemps=1, downsample=100),
}


def bench_scan(args):
    """Waveforms/s of config 3's scan (check_mode_by_mode.py:183-229 over BASELINE configs[2]'s
    grid: M = logspace(5, 7, 10), e0 = linspace(0.1, 0.6, 10), mu = 1e-5 M, Tobs = 1 yr, dt =
    10 s, eps = 1e-2), host work included as the config asks: per point the p0 solve for 0.99
    Tobs (get_p_at_t), the stand-in upstream and the device work. The 100 points go round-robin
    over the ranks (parallel.ShardedScan; a fixed grid split over the ranks: strong scaling),
    each rank runs its points through GenerateEMRIWaveform.generate_batch on its own host-core
    share, and the per-point records (power of h+ and hx, max |h+|) are all-gathered. value =
    100 / the max over ranks of a sweep's time (median of `steps` sweeps after `warmup`)."""
    import torch
    import torch.distributed as dist
    from emri_frequencydomainwaveforms_amd import hostcpu
    from emri_frequencydomainwaveforms_amd.parallel import ShardedScan
    from emri_frequencydomainwaveforms_amd.trajectory import EMRIInspiral, get_p_at_t
    from emri_frequencydomainwaveforms_amd.waveform import GenerateEMRIWaveform, _pool
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    share = hostcpu.pin()
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
    T, dt, eps = 1.0, 10.0, 1e-2
    few = GenerateEMRIWaveform("FastSchwarzschildEccentricFlux",
                               sum_kwargs=dict(pad_output=True, output_type="fd", odd_len=True),
                               use_gpu=True, return_list=True)
    traj = EMRIInspiral()
    # injection angles and distance of emri_pe.py:603-617; p0 is solved per point
    params = np.array([[M, 1e-5 * M, 0.0, 0.0, e0, 1.0, 2.4539, 0.2, 0.2, 0.8, 0.8, 1.0, 0.0,
                        3.0] for M in np.logspace(5, 7, 10) for e0 in np.linspace(0.1, 0.6, 10)])

    def p0_of(row):
        return get_p_at_t(traj, 0.99 * T, [row[0], row[1], 0.0, row[4], 1.0])
    scan = ShardedScan(few)
    pool = _pool()
    for _ in range(max(1, args.warmup)):
        scan(params, T=T, dt=dt, eps=eps, p0_solver=p0_of, mapper=pool.map)
    times = []
    for _ in range(args.steps):
        if world > 1:
            dist.barrier()
        res = scan(params, T=T, dt=dt, eps=eps, p0_solver=p0_of, mapper=pool.map)
        times.append(float(res.seconds.max()))
    sweep = float(np.median(times))
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the host twin over the same 100 points (inputs from the same stand-in upstream,
        # prepared beforehand; the upstream's own cost is reported beside it)
        try:
            from emri_frequencydomainwaveforms_amd.waveform import get_viewing_angles
            th, ph = get_viewing_angles(*params[0][7:11])
            t0 = time.perf_counter()
            ws = [build_workload(T=T, dt=dt, eps=eps, M=row[0], mu=row[1], e0=row[4],
                                 p0=float(p0_of(row)), Phi_phi0=row[11], Phi_r0=row[13],
                                 theta=th, phi=ph, dist=row[6]) for row in params]
            up = time.perf_counter() - t0
            cpu = twin_job_rate([twin_waveform_job(w) for w in ws], "waveforms/s",
                                seconds=args.cpu_seconds, what="grid points")
            cpu["host_upstream_s_per_grid_serial"] = up
        except Exception as exc:
            cpu = {"value": None, "error": repr(exc)}
    if rank == 0:
        line = {
            "metric": "FD waveforms/sec (config 3: 10x10 (M, e0) scan, Tobs=1yr, dt=10s, "
                      "eps=1e-2, host p0 solve + upstream included) at 1/2/4/8 GPUs",
            "value": len(params) / sweep, "unit": "waveforms/s", "n_gpus": world,
            "world_size_rccl": dist.get_world_size() if world > 1 else 1,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": sweep * 1e3,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (stand-in trajectory/amplitudes; FEW data absent offline)",
            "config": {"workload": "config3: M=logspace(5,7,10) e0=linspace(0.1,0.6,10) "
                                   "mu=1e-5 M Tobs=1yr dt=10s eps=1e-2",
                       "points": len(params), "points_per_rank":
                           np.bincount(res.owner, minlength=world).tolist(),
                       "parallelism": f"points round-robin x{world} (all-gather of per-point "
                                      "records)" if world > 1 else "1 GPU",
                       "host_cores_rank0": len(share)},
            "rank_seconds_last_sweep": res.seconds.tolist(),
            "sweep_seconds": times,
            "record_checksum": float(np.sum(res.summary[:, :2])),
            "cpu_baseline": cpu,
            "note": "value: 100 points / the max over ranks of one sweep (p0 solves on the "
                    "rank's upstream pool, generate_batch's host upstream and device groups of "
                    "16, per-point records); median over steps",
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def bench_likelihood(args):
    """Log-likelihoods/s of emri_pe.py's sampler calls (configs 4 / 5) over the ranks.

    One step = one red-blue half-step: B = ntemps * nwalkers / 2 walkers (8 for config 4, 64 for
    config 5) from the reference's start distribution (pe.setup), evaluated as Eryn's vectorised
    call does (Likelihood.__call__: transforms, subset, fused mode sum + logL on the device).
    With N ranks, ShardedLikelihood broadcasts the B x 6 parameters from rank 0 (RCCL), every rank
    evaluates its contiguous B / N walkers, and the B logL are all-gathered (RCCL): a fixed batch
    split over the ranks (strong scaling). `value` times the device path: each walker's host
    upstream (the C++ stand-in trajectory and amplitudes) is memoised after the warm-up;
    api_loglikes_per_s times --api-steps half-steps with the upstream in the loop."""
    import torch
    import torch.distributed as dist
    from emri_frequencydomainwaveforms_amd import pe
    from emri_frequencydomainwaveforms_amd.parallel import ShardedLikelihood
    from emri_frequencydomainwaveforms_amd import hostcpu
    from emri_frequencydomainwaveforms_amd.parallel import shard_range
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # this rank's disjoint share of the node's host cores (LOCAL_WORLD_SIZE shares; the upstream
    # pool and the native thread count follow it, not torchrun's OMP_NUM_THREADS=1)
    share = hostcpu.pin()
    host_threads = hostcpu.threads()
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
    cfg = LIKE_CONFIGS[args.likelihood]
    s = pe.setup(**cfg)
    if args.fused_group:
        s.like.FUSED_GROUP = args.fused_group
    if args.no_tile_constants:
        s.like.fused_tile_constants = False
    B = s.half_step
    batches = s.half_steps()
    if world > 1:
        sl = ShardedLikelihood(s.like, broadcast=True, call_kwargs=s.kwargs)
    else:
        sl = lambda p: s.like(p, **s.kwargs)  # noqa: E731

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # the API rate: host upstream in the loop
    sl(batches[0])
    barrier()
    t0 = time.perf_counter()
    for i in range(args.api_steps):
        sl(batches[(i + 1) % len(batches)])
    barrier()
    api = time.perf_counter() - t0
    memo = pe.MemoizedUpstream(s.few.waveform_generator)
    for i in range(max(args.warmup, len(batches))):
        ll = sl(batches[i % len(batches)])
    barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ll = sl(batches[i % len(batches)])
    barrier()
    elapsed = time.perf_counter() - t0
    # per-rank API rate: this rank's walker shard over its own time with the upstream in the loop
    lo, hi = shard_range(B, rank, world)
    mine = dict(rank=rank, walkers_per_step=hi - lo, api_s=api,
                api_loglikes_per_s=args.api_steps * (hi - lo) / api, host_threads=host_threads,
                host_cores=len(share), host_core_range=[min(share), max(share)] if share else None)
    mine["ms_per_step"] = elapsed / args.steps * 1e3
    per_rank = [mine]
    rccl_world = 1
    if world > 1:
        rccl_world = dist.get_world_size()
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
        tt = torch.tensor([elapsed, api], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, api = float(tt[0]), float(tt[1])
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the host twin on the same walkers (all of the start's for config 4, the first
        # half-step's 64 for config 5) against the device logL of the same rows
        try:
            rows = np.concatenate(batches)[:max(B, 16)]
            ll_dev = np.concatenate([np.asarray(sl(rows[i:i + B])) for i in range(0, len(rows), B)])
            jobs, ll_twin = twin_likelihood_jobs(s, rows)
            cpu = twin_job_rate(jobs, "logL/s", seconds=args.cpu_seconds, what="walkers")
            done = [i for i, v in enumerate(ll_twin) if v is not None]
            cpu["twin_vs_device_max_rel_logL"] = float(max(
                abs(ll_twin[i] - ll_dev[i]) / max(1.0, abs(ll_dev[i])) for i in done))
        except Exception as exc:  # the baseline must not kill the GPU measurement
            cpu = {"value": None, "error": repr(exc)}
    if rank == 0:
        line = {
            "metric": f"FD log-likelihoods/sec (emri_pe {args.likelihood}: "
                      f"{'downsample=100 ' if cfg.get('downsample') else ''}Tobs={cfg['Tobs']}yr "
                      f"eps={cfg['eps']} nwalkers={cfg['nwalkers']}) at 1/2/4/8 GPUs",
            "value": args.steps * B / elapsed, "unit": "logL/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (stand-in trajectory/amplitudes; FEW data absent offline)",
            "config": {"workload": f"{args.likelihood}: emri_pe.py Likelihood over red-blue "
                                   f"half-steps of {B} walkers", "walkers_per_step": B,
                       "N_f": s.info.get("N_f"), "N_f_downsampled": s.info.get("N_f_downsampled"),
                       "p0": s.info["p0"], "parallelism": f"walker shards x{world} (RCCL "
                       "broadcast of params + all-gather of logL)" if world > 1 else "1 GPU",
                       "fused_likelihood": bool(s.like.fused_likelihood),
                       "tile_constants": bool(s.like.fused_tile_constants)},
            "api_loglikes_per_s": args.api_steps * B / api,
            "api_per_rank": per_rank,
            "rank_ms_per_step": {"min": min(r["ms_per_step"] for r in per_rank),
                                 "max": max(r["ms_per_step"] for r in per_rank)},
            "world_size_rccl": rccl_world,
            "host_upstream_ms_per_walker": memo.host_s / max(1, len(memo.memo)) * 1e3,
            "ll_truth_walker_sample": float(np.asarray(ll)[0]),
            "cpu_baseline": cpu,
            "note": "value: device path with each walker's host upstream memoised after the "
                    "warm-up (inputs resident); api_loglikes_per_s: the same calls with the "
                    "host stand-in upstream (C++ trajectory, amplitudes, selection on a thread "
                    "pool: NOT FEW physics) in the loop",
        }
        print(json.dumps(line))
    memo.remove()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
