"""Timing of BASELINE.json's other configurations on one MI355X.

    python tools/configs.py [--only 1,3,4,5] [--reps N]

bench.py measures config 2 (the headline line). This tool prints one JSON line per remaining
configuration, each with two rates:

  device   the hot path alone: host upstream (trajectory, amplitudes, Ylm, mode selection --
           this repo's stand-ins, NOT FEW physics) prepared beforehand, inputs resident in HBM,
           HIP-event/synchronised wall time of the device work per waveform;
  api      the drivers' own call (GenerateEMRIWaveform(...)(*14 params), or Likelihood.get_ll
           over the walker batch) end to end, host upstream included.

config 1  M=1e6 mu=10 e0=0.35 Tobs=1 yr dt=10 s eps=1e-2 (check_mode_by_mode.py:221-241 plumbing)
config 3  10x10 grid M = logspace(5, 7), e0 = linspace(0.1, 0.6), mu = 1e-5 M, Tobs=1 yr,
          eps=1e-2, p0 solved for 0.99 Tobs at every point (check_mode_by_mode.py:200-213)
config 4  emri_pe.py: nwalkers=16 ntemps=1 injectFD=1 template=fd Tobs=2 eps=1e-2 on the full
          grid: per proposal half-step B = 8 walkers through Likelihood.get_ll
          (emri_pe.py:381-414, red_blue.py:149-156); walkers = truth + seeded N(0, sigma)
          offsets in (ln M, ln mu, p0, e0, Phi_phi0, Phi_r0) (covariance.npy is not shipped
          to the GPU box; sigma mirrors its scale)
config 5  downsample=100 (emri_pe.py:322-364 grid), Tobs=4, nwalkers=128 -> B = 64 per
          half-step, on one GPU (the 8-GPU sharding is parallel.py's, exercised by bench.py
          --gpus N at round end)

Parity of these configurations against the oracle is tests/test_gpu_configs.py; this tool only
times (it never imports oracle/).
"""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SUM_KW = dict(pad_output=True, output_type="fd", odd_len=True)
NO_CPU = False       # --no-cpu-baseline
HANN_PAIR = False    # --hann-pair: the windowed logL in its mirror-pair form (efd_hann_loglike)
PY_GROUPS = False    # --python-groups: the fused groups' host steps in Python (round 5)
CPU_SECONDS = 8.0    # --cpu-seconds: the host twin's time budget per configuration
# injection angles of emri_pe.py:603-617 (qS, phiS, qK, phiK) and dist = 2.4539 Gpc (:612)
ANGLES = dict(dist=2.4539, qS=0.2, phiS=0.2, qK=0.8, phiK=0.8)


def _params(M, mu, p0, e0, Phi_phi0=1.0, Phi_r0=3.0):
    a = ANGLES
    return [M, mu, 0.0, p0, e0, 1.0, a["dist"], a["qS"], a["phiS"], a["qK"], a["phiK"],
            Phi_phi0, 0.0, Phi_r0]


def _sync():
    import torch
    torch.cuda.synchronize()


def PrepareCache(wg):
    """Memoise the generator's host upstream per parameter set, so a second pass over the same
    walkers times the device work alone (emri_frequencydomainwaveforms_amd.pe.MemoizedUpstream,
    installed on the instance only)."""
    from emri_frequencydomainwaveforms_amd.pe import MemoizedUpstream
    return MemoizedUpstream(wg)


def config1(reps):
    from emri_frequencydomainwaveforms_amd.trajectory import EMRIInspiral, get_p_at_t
    from emri_frequencydomainwaveforms_amd.waveform import GenerateEMRIWaveform
    T, dt, eps = 1.0, 10.0, 1e-2
    few = GenerateEMRIWaveform("FastSchwarzschildEccentricFlux", sum_kwargs=SUM_KW,
                               use_gpu=True, return_list=True)
    p0 = float(get_p_at_t(EMRIInspiral(), 0.99 * T, [1e6, 10.0, 0.0, 0.35, 1.0]))
    prm = _params(1e6, 10.0, p0, 0.35)
    kw = dict(T=T, dt=dt, eps=eps)
    few(*prm, **kw)
    _sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        few(*prm, **kw)
    _sync()
    api = (time.perf_counter() - t0) / reps
    cache = PrepareCache(few.waveform_generator)
    few(*prm, **kw)
    _sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        few(*prm, **kw)
    _sync()
    dev = (time.perf_counter() - t0) / reps
    nf = len(few.waveform_generator.create_waveform.frequency)
    K = len(few.waveform_generator.last_modes[0])
    cpu = None
    if not NO_CPU:
        # the host twin on the same waveform (BASELINE.md section 2's CPU column): the same
        # stand-in upstream, prepared beforehand, then efd_modesum_cpu writing h+/hx
        import bench
        from emri_frequencydomainwaveforms_amd.waveform import get_viewing_angles
        th, ph = get_viewing_angles(ANGLES["qS"], ANGLES["phiS"], ANGLES["qK"], ANGLES["phiK"])
        w = bench.build_workload(T=T, dt=dt, eps=eps, M=1e6, mu=10.0, e0=0.35, p0=p0,
                                 Phi_phi0=1.0, Phi_r0=3.0, theta=th, phi=ph, dist=ANGLES["dist"])
        cpu = bench.twin_job_rate([bench.twin_waveform_job(w)] * 64, "waveforms/s",
                                  seconds=CPU_SECONDS, what="config-1 waveforms")
    return {"config": "config1: M=1e6 mu=10 e0=0.35 Tobs=1yr dt=10s eps=1e-2", "p0": p0,
            "cpu_baseline": cpu,
            "harmonics": K, "N_f": nf, "device_waveforms_per_s": 1.0 / dev,
            "device_ms": dev * 1e3, "api_waveforms_per_s": 1.0 / api, "api_ms": api * 1e3,
            "host_upstream_ms": cache.host_s * 1e3,
            "device_note": "few_gen call with the host upstream memoised: stand-in grouping, "
                           "splines, records, mode sum, h+/hx split and the [h+, hx] stack"}


def config3(reps, slots=4):
    import torch
    import bench
    from emri_frequencydomainwaveforms_amd.summation import WaveformPipeline
    Ms = np.logspace(5, 7, 10)
    e0s = np.linspace(0.1, 0.6, 10)
    T, dt, eps = 1.0, 10.0, 1e-2
    t0 = time.perf_counter()
    ws = [bench.build_workload(T=T, dt=dt, eps=eps, M=M, mu=1e-5 * M, e0=e0)
          for M in Ms for e0 in e0s]
    host_s = time.perf_counter() - t0
    freq = torch.as_tensor(ws[0]["freq"], device="cuda")
    nf = int(freq.numel())
    k0 = int(np.searchsorted(ws[0]["freq"], 0.0))
    hp = torch.view_as_real(torch.empty(nf - k0, dtype=torch.complex128, device="cuda"))
    hc = torch.empty_like(hp)
    # WaveformPipeline: waveform i's whole device chain (input upload from the host arrays,
    # preparation, mode sum with h+/hx) on slot i % slots's stream, several in flight
    pipe = WaveformPipeline(slots)
    hosts = [{k: w[k] for k in ("t", "amp", "phi_phi", "phi_r", "f_phi", "f_r", "m", "n",
                                "ylm_p", "ylm_m")} for w in ws]
    outs = [(torch.empty_like(hp), torch.empty_like(hc)) for _ in range(slots)]

    def sweep():
        for w, host in zip(ws, hosts):
            o = outs[pipe.next_slot()]
            pipe.submit(host, freq, True, w["prefactor"], hp=o[0], hc=o[1], k0=k0)
    sweep()
    _sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        sweep()
    _sync()
    pipe.wait()
    dev_pipe = (time.perf_counter() - t0) / reps

    # batched: groups of 16 grid points, each one packed upload + efd_modesum_prepare_batch on
    # a group stream and one efd_modesum_sum_batch writing every point's h+/hx (two groups in
    # flight; a group's outputs and workspaces are reused after its sum's event)
    from emri_frequencydomainwaveforms_amd.summation import BatchPreparer, sum_batch
    G = 16
    prep = BatchPreparer(group=G, depth=2)
    gouts = [[(torch.empty_like(hp), torch.empty_like(hc)) for _ in range(G)]
             for _ in range(2)]
    s_sum = torch.cuda.Stream()

    def sweep_batched():
        prep.order_after_current()
        s_sum.wait_stream(torch.cuda.current_stream())
        for g0 in range(0, len(ws), G):
            for w, host in zip(ws[g0:g0 + G], hosts[g0:g0 + G]):
                prep.submit(host, freq, True, w["prefactor"], k0=k0, prepare_only=True)
            gi, jobs = prep.flush()
            s_sum.wait_stream(prep.stream(gi))
            sum_batch([(eng, dict(kw, hp=o[0], hc=o[1])) for (eng, kw), o in zip(jobs, gouts[gi])],
                      stream=s_sum.cuda_stream)
            ev = torch.cuda.Event()
            ev.record(s_sum)
            prep.release(gi, ev)
        torch.cuda.current_stream().wait_stream(s_sum)
    sweep_batched()
    _sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        sweep_batched()
    _sync()
    prep.wait()
    dev = (time.perf_counter() - t0) / reps
    K = [len(w["m"]) for w in ws]
    cpu = None
    if not NO_CPU:   # the host twin over the same 100 points' inputs
        cpu = bench.twin_job_rate([bench.twin_waveform_job(w) for w in ws], "waveforms/s",
                                  seconds=CPU_SECONDS, what="grid points")
        cpu["host_upstream_s_per_grid_serial"] = host_s
    # the drivers' scan (check_mode_by_mode.py:183-229): per point the p0 root solve
    # (get_p_at_t) and the whole few_gen call, one at a time, native upstream
    from emri_frequencydomainwaveforms_amd.trajectory import EMRIInspiral, get_p_at_t
    from emri_frequencydomainwaveforms_amd.waveform import GenerateEMRIWaveform
    few = GenerateEMRIWaveform("FastSchwarzschildEccentricFlux", sum_kwargs=SUM_KW,
                               use_gpu=True, return_list=True)
    traj = EMRIInspiral()

    def api_sweep():
        for M in Ms:
            for e0 in e0s:
                p0 = float(get_p_at_t(traj, 0.99 * T, [M, 1e-5 * M, 0.0, e0, 1.0]))
                few(*_params(M, 1e-5 * M, p0, e0), T=T, dt=dt, eps=eps)
    api_sweep()
    _sync()
    t0 = time.perf_counter()
    api_sweep()
    _sync()
    api = time.perf_counter() - t0

    # the same scan with the host work of all points at once on this rank's host cores: the
    # p0 root solves on the upstream thread pool, then GenerateEMRIWaveform.generate_batch
    # (prefetched upstream, device work in groups of 16 writing every point's [h+, hx])
    from emri_frequencydomainwaveforms_amd import hostcpu
    from emri_frequencydomainwaveforms_amd.waveform import _pool
    pts = [(M, e0) for M in Ms for e0 in e0s]
    outb = torch.empty((len(pts), 2, nf - k0), dtype=torch.complex128, device="cuda")

    def api_batched():
        p0s = list(_pool().map(
            lambda me: float(get_p_at_t(traj, 0.99 * T, [me[0], 1e-5 * me[0], 0.0, me[1], 1.0])),
            pts))
        prm = np.array([_params(M, 1e-5 * M, p0, e0) for (M, e0), p0 in zip(pts, p0s)])
        few.generate_batch(prm, outb, T=T, dt=dt, eps=eps)
    api_batched()
    _sync()
    tb = []
    for _ in range(max(1, reps // 2)):
        t0 = time.perf_counter()
        api_batched()
        _sync()
        tb.append(time.perf_counter() - t0)
    api_b = float(np.median(tb))
    return {"config": "config3: 10x10 grid M=logspace(5,7) e0=linspace(0.1,0.6) mu=1e-5 M "
                      "Tobs=1yr dt=10s eps=1e-2", "waveforms": len(ws), "N_f": nf,
            "harmonics_min_max": [min(K), max(K)], "cpu_baseline": cpu,
            "device_waveforms_per_s": len(ws) / dev, "device_ms_per_grid": dev * 1e3,
            "pipeline_waveforms_per_s": len(ws) / dev_pipe,
            "api_waveforms_per_s": len(ws) / api,
            "api_note": "per point: native get_p_at_t + the whole few_gen call, serial",
            "api_batched_waveforms_per_s": len(ws) / api_b,
            "api_batched_host_threads": hostcpu.threads(),
            "api_batched_note": "the 100 p0 solves on the upstream thread pool, then "
                                "GenerateEMRIWaveform.generate_batch: every point's host "
                                "upstream prefetched on the pool, device work in groups of 16, "
                                "each point's [h+, hx] written (median of reps/2 sweeps)",
            "host_upstream_s_per_grid": host_s, "pipeline_slots": slots,
            "device_note": "100 waveforms in groups of 16: one packed upload and one "
                           "efd_modesum_prepare_batch per group on a group stream, one "
                           "efd_modesum_sum_batch writing each point's h+/hx, two groups in "
                           "flight (pipeline_waveforms_per_s: round 2's WaveformPipeline, "
                           f"each waveform's chain on one of {slots} streams); api adds the "
                           "host stand-in upstream incl. the p0 root solve per point"}


def _likelihood_setup(T, eps, downsample, nwalkers, seed=2601996, **extra):
    """emri_pe.py's setup (emri_frequencydomainwaveforms_amd.pe: its angles, distance, phases,
    p0 for 0.99 Tobs, downsampled grid, Likelihood, walker start); the batch is the first
    red-blue half-step of the start, mapped to FEW's 14 parameters by the TransformContainer,
    with walker 0 on the injection (logL = 0 exactly)."""
    from emri_frequencydomainwaveforms_amd import pe
    st = pe.setup(Tobs=T, eps=eps, downsample=downsample, nwalkers=nwalkers, seed=seed,
                  **extra)
    walkers = st.transform.both_transforms(st.half_steps()[0])
    walkers[0] = st.truth14
    return st.few, st.like, walkers, st.kwargs, len(st.f_like)


def config_like(name, T, eps, downsample, nwalkers, reps, slots=4, fused=True, group=None,
                **extra):
    few, like, walkers, kw, nbins = _likelihood_setup(T, eps, downsample, nwalkers, **extra)
    windowed = like.template_model.window is not None
    like.num_streams = slots
    like.fused_likelihood = fused
    if HANN_PAIR:
        like.HANN_LOCAL = False
    if PY_GROUPS:
        like.FUSED_NATIVE_GROUP = False
    if group:
        like.FUSED_GROUP = group
    if os.environ.get("FUSED_DEPTH"):
        like.FUSED_DEPTH = int(os.environ["FUSED_DEPTH"])
    B = len(walkers)
    # warm-up (also the correctness anchor: ll[0] == 0); three calls, so the upstream pool's
    # threads have made their OpenMP teams before the timed calls (the first calls of a fresh
    # process cost several ms more, which a mean over 5 reps otherwise carries)
    for _ in range(3):
        ll = like.get_ll(walkers, **kw)
    _sync()
    # per-call times (get_ll returns host values: each call ends synchronised); the API rate is
    # their median, with the spread reported beside it
    calls = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ll = like.get_ll(walkers, **kw)
        calls.append(time.perf_counter() - t0)
    _sync()
    api = float(np.median(calls))
    cache = PrepareCache(few.waveform_generator)
    like.get_ll(walkers, **kw)
    _sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        ll2 = like.get_ll(walkers, **kw)
    _sync()
    dev = (time.perf_counter() - t0) / reps
    cpu = None
    if not NO_CPU and not windowed:
        # the host twin on the same walkers against the likelihood's own d and w
        import bench
        from emri_frequencydomainwaveforms_amd import pe
        st = pe.setup(Tobs=T, eps=eps, downsample=downsample, nwalkers=nwalkers, **extra)
        jobs, ll_twin = bench.twin_likelihood_jobs(st, st.half_steps()[0])
        cpu = bench.twin_job_rate(jobs, "logL/s", seconds=CPU_SECONDS, what="walkers")
    return {"config": name, "walkers_per_half_step": B, "N_pos": nbins, "cpu_baseline": cpu,
            "device_loglikes_per_s": B / dev, "device_ms_per_half_step": dev * 1e3,
            "api_loglikes_per_s": B / api, "api_ms_per_half_step": api * 1e3,
            "api_ms_per_call_min_max": [min(calls) * 1e3, max(calls) * 1e3],
            "host_upstream_ms_per_walker": cache.host_s / B * 1e3,
            "ll_truth": float(ll[0]), "ll_min": float(np.min(ll)),
            "ll_bitwise_repeatable": bool(np.array_equal(ll, ll2)), "streams": slots,
            "fused_likelihood": fused and not windowed,
            "device_note": "Likelihood.get_ll over the half-step batch with the host upstream "
                           "memoised: " + (
                               "per group of 8 walkers the FD spectra S in one batched mode "
                               "sum, the Hann window's correction as one four-step transform "
                               "pipeline over the rows' supports (efd_hann_convolve) and the "
                               "windowed logL reduced in place (efd_hann_loglike)"
                               if windowed else
                               "per balanced group of up to 16 walkers one packed input "
                               "upload (efd_stage_batch), one efd_modesum_prepare_batch and "
                               "one mode-sum launch with the likelihood fused in (no "
                               "template written); two groups in flight"
                               if fused else
                               "per walker the FD template (input upload, mode sum with h+/hx "
                               "straight into a slot's buffer) + efd_loglike on one of "
                               f"{slots} streams (WaveformPipeline)") +
                           "; one host sync per batch"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="1,3,4,5")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--slots", type=int, default=4, help="WaveformPipeline slots (config 3) "
                    "and Likelihood.num_streams (configs 4, 5)")
    ap.add_argument("--unfused", action="store_true", help="configs 4, 5: templates through "
                    "a buffer + efd_loglike instead of the fused batched likelihood")
    ap.add_argument("--fused-group", type=int, default=0, help="walkers per fused launch "
                    "(Likelihood.FUSED_GROUP; 0 = its default)")
    ap.add_argument("--no-cpu-baseline", action="store_true", help="skip the host twin rates")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--hann-pair", action="store_true", help="windowed config: the logL in "
                    "its mirror-pair form after the transforms (efd_hann_loglike) instead of "
                    "the per-bin form reduced inside them (efd_hann_loglike_local)")
    ap.add_argument("--python-groups", action="store_true", help="configs 4, 5: each fused "
                    "group's staging and launches as Python steps instead of one native call "
                    "(efd_fused_group)")
    args = ap.parse_args()
    global NO_CPU, CPU_SECONDS, HANN_PAIR, PY_GROUPS
    NO_CPU, CPU_SECONDS, HANN_PAIR = args.no_cpu_baseline, args.cpu_seconds, args.hann_pair
    PY_GROUPS = args.python_groups
    which = set(args.only.split(","))
    out = []
    if "1" in which:
        out.append(config1(args.reps))
        print(json.dumps(out[-1]), flush=True)
    if "3" in which:
        out.append(config3(args.reps, args.slots))
        print(json.dumps(out[-1]), flush=True)
    if "4" in which:
        out.append(config_like("config4: emri_pe nwalkers=16 ntemps=1 injectFD=1 template=fd "
                               "Tobs=2yr eps=1e-2 full grid", 2.0, 1e-2, None, 16, args.reps,
                               args.slots, not args.unfused, args.fused_group))
        print(json.dumps(out[-1]), flush=True)
    if "w" in which:
        # test.sh:3: -Tobs 4 -M 3.67e6 -mu 292 -e0 0.579 -eps 1e-2 -template fd -window_flag 1
        out.append(config_like("test.sh windowed: emri_pe Tobs=4yr M=3.67e6 mu=292 e0=0.579 "
                               "eps=1e-2 nwalkers=16 window_flag=1 full grid", 4.0, 1e-2, None,
                               16, args.reps, args.slots, not args.unfused, args.fused_group,
                               M=3670041.7362535275, mu=292.0583167470244,
                               e0=0.5794130830706371, window_flag=True))
        print(json.dumps(out[-1]), flush=True)
    if "5" in which:
        out.append(config_like("config5: emri_pe downsample=100 Tobs=4yr eps=1e-2 "
                               "nwalkers=128 (1 GPU)", 4.0, 1e-2, 100, 128, args.reps,
                               args.slots, not args.unfused, args.fused_group))
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
