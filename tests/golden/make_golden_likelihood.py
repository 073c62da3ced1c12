"""Golden vectors for the likelihood side of the path, produced by the reference's own code.

Run ONLY in the development container (imports Python modules from /root/reference):

    python tests/golden/make_golden_likelihood.py

Imports, unchanged, from /root/reference:
  - LISAanalysistools/lisatools/diagnostic.py: inner_product (:14-157), snr (:160-171)
  - LISAanalysistools/lisatools/sampling/likelihood.py: Likelihood.inject_signal (:80-234),
    get_ll (:236-293), __call__ with `subset` (:295-334); needs Eryn/ on the path
  - FDutils.py: get_sensitivity (:21-33, CubicSpline of LISA_Alloc_Sh.txt), get_convolution
    (:35-47), get_fd_windowed (:66-101); imported with cwd /root/reference because it reads
    './LISA_Alloc_Sh.txt' at import
and evaluates them on seeded synthetic inputs. Only inputs and outputs are written
(tests/golden/likelihood_golden.npz); no reference text is stored.
"""

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def main():
    import matplotlib
    matplotlib.use("Agg")
    sys.path.insert(0, os.path.join(REF, "LISAanalysistools"))
    sys.path.insert(0, os.path.join(REF, "Eryn"))
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    os.chdir(REF)
    try:
        import FDutils
        from lisatools.diagnostic import inner_product, snr
        from lisatools.sampling.likelihood import Likelihood
    finally:
        os.chdir(cwd)
    from scipy.signal.windows import hann

    rng = np.random.default_rng(2601996)
    out = {}

    # ---- PSD table interpolation, incl. f = 0 (first bin of frequency[frequency >= 0])
    dt = 10.0
    nf = 4001
    fpos = np.fft.fftshift(np.fft.fftfreq(2 * nf - 1, dt))[nf - 1:]      # 0 .. ~1/(2 dt)
    out["psd_f"] = fpos
    out["psd"] = FDutils.get_sensitivity(fpos)
    fq = np.geomspace(1e-5, 0.049, 64)
    out["psd_fq"] = fq
    out["psd_q"] = FDutils.get_sensitivity(fq)

    # ---- inner products on a positive grid (bin 0 excluded: PSD(0) is extrapolated)
    f = fpos[1:]
    psd = FDutils.get_sensitivity(f)
    a = [(rng.normal(size=len(f)) + 1j * rng.normal(size=len(f))) * 1e-20 for _ in range(2)]
    b = [x + (rng.normal(size=len(f)) + 1j * rng.normal(size=len(f))) * 3e-21 for x in a]
    out["ip_f"] = f
    out["ip_psd"] = psd
    out["ip_a"] = np.array(a)
    out["ip_b"] = np.array(b)
    out["ip_plain"] = inner_product(a, b, f_arr=f, PSD=psd)
    out["ip_norm"] = inner_product(a, b, f_arr=f, PSD=psd, normalize=True)
    out["ip_norm_sig1"] = inner_product(a, b, f_arr=f, PSD=psd, normalize="sig1")
    out["ip_complex"] = inner_product(a, b, f_arr=f, PSD=psd, complex=True)
    out["ip_chan0"] = inner_product(a[0], b[0], f_arr=f, PSD=psd, normalize=True)
    out["snr_a"] = snr(a, f_arr=f, PSD=psd)
    out["snr_ab"] = snr(a, data=b, f_arr=f, PSD=psd)
    df = f[1] - f[0]
    out["ip_df"] = inner_product(a, b, df=df, PSD=psd)
    # non-uniform (downsampled-style) grid
    fu = np.sort(rng.uniform(1e-4, 0.04, 3001))
    au = [rng.normal(size=len(fu)) + 1j * rng.normal(size=len(fu)) for _ in range(2)]
    bu = [rng.normal(size=len(fu)) + 1j * rng.normal(size=len(fu)) for _ in range(2)]
    psdu = FDutils.get_sensitivity(fu)
    out["ipu_f"], out["ipu_psd"], out["ipu_a"], out["ipu_b"] = fu, psdu, np.array(au), np.array(bu)
    out["ipu_plain"] = inner_product(au, bu, f_arr=fu, PSD=psdu)

    # ---- Likelihood: FD, two channels, f_arr includes f = 0 (noise factor NaN there)
    base = np.array([(rng.normal(size=nf) + 1j * rng.normal(size=nf)) * 1e-20 for _ in range(2)])
    tilt = np.array([(rng.normal(size=nf) + 1j * rng.normal(size=nf)) * 1e-21 for _ in range(2)])

    def template(amp, slope, *args):
        return [amp * base[c] + slope * tilt[c] for c in range(2)]

    truth = np.array([1.0, 0.5])
    like = Likelihood(template, 2, f_arr=fpos, use_gpu=False, subset=2)
    like.inject_signal(data_stream=template(*truth), noise_fn=[FDutils.get_sensitivity] * 2,
                       noise_kwargs=[{}, {}], add_noise=False)
    params = np.array([[1.0, 0.5], [1.01, 0.5], [0.9, -0.2], [1.3, 2.0], [0.0, 0.0]])
    out["ll_f"] = fpos
    out["ll_base"], out["ll_tilt"] = base, tilt
    out["ll_truth"] = truth
    out["ll_params"] = params
    out["ll_noise_factor"] = np.asarray(like.noise_factor)
    out["ll_injection"] = np.asarray(like.injection_channels)
    out["ll_get_ll"] = like.get_ll(params)
    out["ll_call"] = like(params)

    # ---- FD windowing (circular convolution with the window's spectrum)
    nw = 257
    sig = [rng.normal(size=nw) + 1j * rng.normal(size=nw) for _ in range(2)]
    win = hann(nw)
    out["win_sig"] = np.array(sig)
    out["win_window"] = win
    out["win_conv"] = FDutils.get_convolution(np.conj(np.fft.fft(win)), sig[0])
    w0, w1 = FDutils.get_fd_windowed(sig, win)
    out["win_fd"] = np.array([w0, w1])
    wfd = np.fft.fft(win)
    v0, v1 = FDutils.get_fd_windowed(sig, wfd, window_in_fd=True)
    out["win_fd_infd"] = np.array([v0, v1])

    # ---- lisatools' analytic cornish_lisa_psd (sensitivity.py:1227-1286), the notebooks'
    # mismatch weighting, and inner products weighted by it by name (diagnostic.py:81-82),
    # on the positive grid with and without the f = 0 bin (PSD(0) = inf: zero weight there)
    from lisatools.sensitivity import cornish_lisa_psd, get_sensitivity as lt_sensitivity
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        out["cornish_f"] = fpos
        out["cornish_psd"] = cornish_lisa_psd(fpos)
        out["cornish_psd_sky"] = cornish_lisa_psd(fq, sky_averaged=True)
        out["cornish_asd_q"] = lt_sensitivity(fq, sens_fn="cornish_lisa_psd", return_type="ASD")
        out["cornish_char_q"] = lt_sensitivity(fq, sens_fn="cornish_lisa_psd",
                                               return_type="char_strain")
        out["cornish_ip_norm"] = inner_product(a, b, f_arr=f, PSD="cornish_lisa_psd",
                                               normalize=True)
        a0 = [np.concatenate([[1e-20 + 0j], x]) for x in a]
        b0 = [np.concatenate([[2e-20 + 0j], x]) for x in b]
        out["cornish_a0"], out["cornish_b0"] = np.array(a0), np.array(b0)
        out["cornish_ip_f0"] = inner_product(a0, b0, f_arr=fpos, PSD="cornish_lisa_psd",
                                             normalize=True)

    np.savez_compressed(os.path.join(HERE, "likelihood_golden.npz"), **out)
    for k, v in out.items():
        v = np.asarray(v)
        print(k, v.shape, v.dtype, v.ravel()[:2])


if __name__ == "__main__":
    main()
