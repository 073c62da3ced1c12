/*
 * emrifd.h -- C ABI of the MI355X-native FD EMRI mode-sum library (libemrifd.so).
 *
 * Drop-in boundary for the hot path named in BASELINE.json:north_star. In the reference, the
 * FD summation is reached through FastEMRIWaveforms' Python call surface
 *   GenerateEMRIWaveform("FastSchwarzschildEccentricFlux",
 *                        sum_kwargs=dict(pad_output=True, output_type="fd", odd_len=True))
 * (check_mode_by_mode.py:69-83, emri_pe.py:86-105) whose native seam (FEW's Cython wrapper of
 * its FD kernels) is external and absent offline [FEW-ext]. The entry points below are what
 * that seam needs, per SURVEY.md section 8(b):
 *   - efd_spline_build   <- FEW CubicSplineInterpolant build over the sparse trajectory
 *                          (analogue: Tutorial_FD_construction_single_mode.ipynb:558, :594)
 *   - efd_modesum        <- FDInterpolatedModeSum.sum: spline -> SPA per harmonic -> sum over
 *                          harmonics into the two-sided spectrum (notebook :552-623,
 *                          summed over modes; called per waveform at check_mode_by_mode.py:226)
 *   - efd_polarizations  <- the h+/hx split of the 'fd' output (contract
 *                          check_mode_by_mode.py:247: S = h+ - i hx) and mask_positive
 *                          (emri_pe.py:241)
 *   - efd_loglike        <- Likelihood.get_ll's reduction -1/2 * 4 * sum |d - h w|^2
 *                          (LISAanalysistools/lisatools/sampling/likelihood.py:257-274)
 *   - efd_inner_product  <- lisatools inner_product / snr
 *                          (LISAanalysistools/lisatools/diagnostic.py:14-186)
 *
 * Conventions: all arrays are caller-owned DEVICE pointers (HIP, gfx950) unless stated;
 * complex numbers are interleaved (re, im) float64 pairs; every call is asynchronous on the
 * given hipStream_t (NULL = default stream) and never allocates device memory; return value 0
 * on success, negative on error (efd_last_error gives the message). Calls on different
 * streams/devices are independent (no global mutable state except the per-thread error string).
 */
#ifndef EMRIFD_H
#define EMRIFD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EFD_OK 0
#define EFD_ERR_ARG (-1)        /* invalid argument (shape, NULL pointer, unsorted grid...)  */
#define EFD_ERR_HIP (-2)        /* HIP runtime error                                          */
#define EFD_ERR_WORKSPACE (-3)  /* workspace smaller than efd_modesum_workspace_bytes()     */

#define EFD_CAUSTIC_SPA 0       /* plain stationary phase: Q = e^{i sgn(F') 3pi/4} / sqrt|F'| */
#define EFD_CAUSTIC_UNIFORM 1   /* notebook K_{1/3} uniform form (notebook :599-613)          */

/* Library version (major*10000 + minor*100 + patch). */
int efd_version(void);

/* The source hash the library was built from (16 hex digits of the SHA-256 over its sources,
 * emri_frequencydomainwaveforms_amd/_build.py source_id), or "unversioned". Static storage. */
const char* efd_build_id(void);

/* Copies the last error message of the calling thread into buf (NUL-terminated). */
int efd_last_error(char* buf, int len);

/*
 * Batched not-a-knot cubic splines on shared knots x[n] (n >= 2, strictly increasing):
 * y is knot-major [n][ninterp]; coef is written as [n-1][4][ninterp] in scipy PPoly order
 * (c0 highest power): y(x) = ((c0 w + c1) w + c2) w + c3, w = x - x[i].
 * Matches scipy.interpolate.CubicSpline(x, y, bc_type='not-a-knot') including its n = 2
 * (line) and n = 3 (parabola) special cases. One lane per interpolant.
 */
int efd_spline_build(const double* x, int n, const double* y, int ninterp, double* coef,
                     void* stream);

/* Input of one FD mode sum (one waveform). */
typedef struct efd_modesum_args {
    /* sparse trajectory knots, length nt (device) */
    const double* t;          /* [nt] seconds, strictly increasing                           */
    const double* phi_phi;    /* [nt] azimuthal phase                                        */
    const double* phi_r;      /* [nt] radial phase                                           */
    const double* f_phi;      /* [nt] Omega_phi / (2 pi M MTSUN_SI) [Hz]                     */
    const double* f_r;        /* [nt] Omega_r / (2 pi M MTSUN_SI) [Hz]                       */
    int32_t nt;
    /* harmonics (device) */
    const double* amp;        /* complex [nt][K]: Teukolsky amplitude A_k(t_i) (FEW layout)  */
    const int32_t* m;         /* [K] 0 <= m <= 255; m > 0 adds the -m partner branch          */
    const int32_t* n;         /* [K] |n| <= 1023                                              */
    const double* ylm_p;      /* complex [K]: Y_lm                                            */
    const double* ylm_m;      /* complex [K]: (-1)^l Y_{l,-m} (ignored for m = 0)             */
    int32_t K;                /* 1 <= K <= 8192                                               */
    /* frequency grid (device), ascending */
    const double* freq;       /* [nf]                                                         */
    int64_t nf;
    int32_t grid_symmetric;   /* 1 iff freq[nf-1-k] == -freq[k] for all k (mirror pairing)    */
    /* scaling: S *= scale (complex), e.g. mu MRSUN_SI/(dist Gpc) * e^{-2 i psi_pol}           */
    double scale_re, scale_im;
    int32_t caustic;          /* EFD_CAUSTIC_*                                                */
    int32_t accumulate;       /* 1: outputs += new values, 0: outputs = new values            */
    double* out;              /* complex [nf] (device): FEW 'fd' spectrum S = h+ - i hx, or
                               * NULL when only hp/hc are wanted                               */
    /* optional hipEvent_t pair recorded on `stream` around the mode-sum kernel alone (K8), for
     * roofline timing; NULL = not recorded */
    void* prof_begin;
    void* prof_end;
    /* optional fused polarisations (symmetric grids only): complex [nf - k0] each, written as
     * efd_polarizations(S, nf, k0, hp, hc) would, from the registers that hold S (no S round
     * trip through HBM). NULL = not written. */
    double* hp;
    double* hc;
    int64_t k0;
} efd_modesum_args;

/* Bytes of device workspace efd_modesum needs for (nt, K, nf), valid for either grid kind;
 * 0 for an invalid shape (nt < 2 or nt > 1024, K <= 0, nf <= 0). Host-only query. */
size_t efd_modesum_workspace_bytes(int32_t nt, int32_t K, int64_t nf);

/*
 * Full FD mode sum: (m, n) grouping -> spline build (trajectory; group amplitudes
 * sum_l Y A_lmn) -> per-group t(f) inverse splines -> interval records ->
 * segment table -> SPA evaluation with output-stationary accumulation (each tile of frequency
 * bins builds its own record list in LDS). Asynchronous, allocation-free, no host sync, no
 * atomics on the spectrum; bitwise reproducible.
 */
int efd_modesum(const efd_modesum_args* a, void* workspace, size_t workspace_bytes, void* stream);

/*
 * The same call in two phases on possibly different streams (the caller orders them, e.g. with
 * an event): _prepare runs everything up to the tiles' record lists (grouping, splines,
 * inverse splines, interval records, segment table, per-tile key lists and the tiles'
 * longest-first dispatch order; latency-bound),
 * _sum the mode-sum kernel (reads
 * freq, writes out / hp / hc). With two workspaces, waveform i+1's prepare overlaps waveform
 * i's sum. efd_modesum == _prepare then _sum on one stream.
 */
int efd_modesum_prepare(const efd_modesum_args* a, void* workspace, size_t workspace_bytes,
                        void* stream);
int efd_modesum_sum(const efd_modesum_args* a, void* workspace, size_t workspace_bytes,
                    void* stream);

/*
 * _sum for `count` prepared waveforms in one kernel launch (1 <= count <= EFD_BATCH_MAX): the
 * waveforms' tiles interleave in one longest-first dispatch, so the launch's ramp, tail and the
 * gap between launches are shared (a batch of walkers in a likelihood, or of templates). a[i] and
 * workspace[i] are exactly what efd_modesum_sum would take for waveform i (each prepared by
 * efd_modesum_prepare on its own workspace); every a[i] must agree on nf, grid_symmetric, caustic
 * and accumulate. Each waveform's outputs are bitwise those of its own efd_modesum_sum. The
 * profiling events of a[0] bracket the launch; efd_modesum_status / _stats work per workspace.
 * Not part of the reference's interface: an extension for its batched callers.
 */
#define EFD_BATCH_MAX 16
int efd_modesum_sum_batch(const efd_modesum_args* const* a, void* const* workspace,
                          const size_t* workspace_bytes, int32_t count, void* stream);

/*
 * efd_modesum_prepare for `count` waveforms (1 <= count <= EFD_BATCH_MAX) in one chain of
 * launches: each preparation kernel runs once for the batch, its grid's z index picking the
 * waveform (one waveform's launches cost ~10 us of host time and as many dispatches; a
 * likelihood's walker batch pays them once). a[i], workspace[i] are what efd_modesum_prepare
 * would take for waveform i; every a[i] must agree on nf and grid_symmetric and each waveform
 * needs its own workspace. Each workspace ends up bitwise as after its own efd_modesum_prepare
 * (which is this call with count = 1). Not part of the reference's interface: an extension for
 * its batched callers (Likelihood over a walker batch, likelihood.py:246-274).
 */
int efd_modesum_prepare_batch(const efd_modesum_args* const* a, void* const* workspace,
                              const size_t* workspace_bytes, int32_t count, void* stream);

/*
 * efd_modesum_sum_batch with the Gaussian log-likelihood of each waveform fused into the mode
 * sum's epilogue (Likelihood.get_ll over a batch of walkers, likelihood.py:246-274):
 *   out[i] = -1/2 * 4 * sum_c sum_j | d[c][j] - h_c,i[j] * w[c][j] |^2,  c in {+, x},
 *   j over the bins [k0, nf) of the symmetric grid (c = + is h+, c = x is hx, as the fused
 *   polarisations would write them), d complex [2][nf - k0], w real [2][nf - k0]
 * (efd_loglike's terms and rounding), without writing the templates: the registers that hold
 * S(k), S(nf-1-k) feed the reduction, so h+/hx never go through HBM. Every a[i] needs
 * grid_symmetric = 1, accumulate = 0 and the same k0; hp/hc/out of a[i] are still written when
 * non-NULL. out: count device doubles. Per-tile partials live in each workspace; the final
 * reduction has a fixed order (bitwise reproducible; equal to efd_loglike on the written
 * templates to rounding). A waveform whose workspace holds a device-side error flag (see
 * efd_modesum_status) gets out[i] = NaN, and its flags stay set: a caller that finds no NaN
 * needs no status synchronisation, one that does calls efd_modesum_status_batch for the
 * message. An extension for batched likelihood callers.
 */
int efd_modesum_sum_loglike(const efd_modesum_args* const* a, void* const* workspace,
                            const size_t* workspace_bytes, int32_t count, const double* d,
                            const double* w, double* out, void* stream);

/*
 * The fused likelihood's per-tile constants: for each tile of the symmetric grid's paired layout
 * (efd_loglike_tile_count(nf) tiles), that tile's partial of efd_modesum_sum_loglike's sum when
 * the template is zero on all of its bins. They depend on (d, w, nf, k0) only, so a likelihood
 * computes them once; efd_modesum_sum_loglike_ex then gives a tile no harmonic reaches this value
 * instead of re-reading d and w there (at a high f_max most tiles of a sparse spectrum are empty).
 * The result is bitwise efd_modesum_sum_loglike's: the constants are that epilogue's arithmetic on
 * zero sums. tile_const: efd_loglike_tile_count(nf) device doubles. Extensions for batched
 * likelihood callers (likelihood.py:246-274).
 */
int64_t efd_loglike_tile_count(int64_t nf);
int efd_loglike_tile_constants(const double* d, const double* w, int64_t nf, int64_t k0,
                               double* tile_const, void* stream);

/* efd_modesum_sum_loglike with the constants of efd_loglike_tile_constants for the same d, w,
 * nf and k0 (tile_const NULL: efd_modesum_sum_loglike). */
int efd_modesum_sum_loglike_ex(const efd_modesum_args* const* a, void* const* workspace,
                               const size_t* workspace_bytes, int32_t count, const double* d,
                               const double* w, const double* tile_const, double* out,
                               void* stream);

/* Synchronises `stream` and reports errors detected on the device by the calls on this
 * workspace since the previous efd_modesum_status (the flags are sticky across preparations, so
 * a workspace reused by several waveforms before its status is read loses none): a harmonic
 * with more than 8 monotonic frequency runs, or |m| > 255 or |n| > 1023 -> EFD_ERR_ARG; a tile
 * dispatch-order entry out of range in the sum (its bins left unwritten, e.g. a sum run on a
 * workspace another call prepared) -> EFD_ERR_HIP. Reported flags are cleared. */
int efd_modesum_status(const void* workspace, void* stream);

/* Each workspace's lane range [lane_lo, lane_hi) after its preparation: the union of its
 * harmonics' segment lane ranges (on symmetric grids lane l is bin l and its mirror nf-1-l; no
 * term reaches a bin outside), into out[2 i], out[2 i + 1] (device int32), stream-ordered. */
int efd_modesum_lane_ranges(void* const* workspace, int32_t count, int32_t* out, void* stream);

/*
 * efd_modesum_status for `count` workspaces (1 <= count <= EFD_BATCH_MAX) used on `stream`: one
 * gather launch and one synchronisation for a walker batch. flags (optional, int32[count])
 * receives each workspace's error bits (1: more than 8 monotonic runs, 2: |m| > 255 or
 * |n| > 1023, 4: tile dispatch-order entry out of range); the return value and efd_last_error
 * report the first failing waveform. Reported flags are cleared, as by efd_modesum_status.
 */
int efd_modesum_status_batch(void* const* workspace, int32_t count, int32_t* flags,
                             void* stream);

/* Contributions C (harmonic branch x bin pairs, the reference's per-(l, m, n) formulation) of
 * the last efd_modesum on this workspace (for the roofline); synchronises `stream`. */
int efd_modesum_contributions(const void* workspace, int64_t* contributions, void* stream);

/* Statistics of the last efd_modesum on this workspace; synchronises `stream`. contributions as
 * above; evaluations = SPA evaluations actually made (one per (m, n) group branch x bin: every
 * l of a group shares t(f), the phase and the K_{1/3} factor); groups = distinct (m, n).
 * NULL outputs are skipped. */
int efd_modesum_stats(const void* workspace, int64_t* contributions, int64_t* evaluations,
                      int32_t* groups, void* stream);

/* Of those evaluations, the ones made on envelope records (the records whose SPA amplitude and
 * K_{1/3} phase k_items carries as polynomials in t); synchronises `stream`.
 * An extension for the roofline accounting, not part of the reference's interface. */
int efd_modesum_env_evaluations(const void* workspace, int64_t* env_evaluations, void* stream);

/* Input of one time-domain mode sum (one waveform). */
typedef struct efd_td_args {
    /* sparse trajectory knots, length nt (device); as efd_modesum_args */
    const double* t;
    const double* phi_phi;
    const double* phi_r;
    const double* f_phi;
    const double* f_r;
    int32_t nt;
    /* harmonics (device); as efd_modesum_args */
    const double* amp;
    const int32_t* m;
    const int32_t* n;
    const double* ylm_p;
    const double* ylm_m;
    int32_t K;
    /* samples t_i = i dt, 0 <= i < nsamples; zero where t_i > t[nt-1] (FEW pad_output) */
    double dt;
    int64_t nsamples;
    double scale_re, scale_im;  /* h *= scale (complex)                                        */
    int32_t accumulate;         /* 1: outputs += new values, 0: outputs = new values           */
    double* out;                /* complex [nsamples] h = h+ - i hx, or NULL                    */
    double* hp;                 /* real [nsamples] h+, or NULL                                  */
    double* hc;                 /* real [nsamples] hx, or NULL                                  */
    void* prof_begin;           /* optional hipEvent_t pair around the TD kernel alone          */
    void* prof_end;
} efd_td_args;

/* Bytes of device workspace efd_td_modesum needs for (nt, K); 0 for an invalid shape. */
size_t efd_td_workspace_bytes(int32_t nt, int32_t K);

/*
 * Time-domain mode sum <- FEW InterpolatedModeSum, the TD generator the reference compares its
 * FD waveform against (td_gen: check_mode_by_mode.py:85-99, 254-264; Tutorial_FrequencyDomain_
 * Waveforms.ipynb:61-66, 184-188):
 *   h(t_i) = scale * sum_k [ Y+_k A_k(t_i) e^{-i Phi_k(t_i)} + (m_k > 0) Y-_k conj(A_k(t_i))
 *            e^{+i Phi_k(t_i)} ],  Phi_k = m Phi_phi + n Phi_r,
 * with not-a-knot cubic splines of A_k, Phi_phi, Phi_r over the knots. Its DFT,
 * fftshift(fft(h)) dt, is the FD spectrum efd_modesum returns. Asynchronous, allocation-free;
 * efd_modesum_status works on this workspace too.
 */
int efd_td_modesum(const efd_td_args* a, void* workspace, size_t workspace_bytes, void* stream);

/*
 * Asynchronous host -> device copy of `bytes` from `src` (pinned host memory) to `dst` on
 * `stream`: the input upload of a waveform on a pipeline slot's stream, issued through this
 * library's HIP runtime (no host synchronisation). Plumbing for the Python host layer.
 */
int efd_upload(void* dst, const void* src, size_t bytes, void* stream);

/* Host plumbing for batched callers: `bytes` from device memory into (pinned) host memory,
 * asynchronous on `stream` (hipMemcpyAsync). */
int efd_download(void* dst, const void* src, size_t bytes, void* stream);

/* Host plumbing: the `count` streams dst[i] wait for the work queued so far on stream `src`
 * (one event record, one stream wait each; nothing blocks the host). The library's event is
 * per thread and device and re-recorded by each call; waits already enqueued are unaffected. */
int efd_stream_order(void* src, void* const* dst, int32_t count);

/*
 * h+ = (S(f) + conj(S_flip))/2, hx = i (S(f) - conj(S_flip))/2 with S_flip the array reversed
 * (FEW list output). Writes bins [k0, nf) of each (k0 = first bin to keep, e.g. the f >= 0
 * bin for mask_positive) into hp, hc (complex [nf - k0]).
 */
int efd_polarizations(const double* S, int64_t nf, int64_t k0, double* hp, double* hc,
                      void* stream);

/*
 * The spectrum convolved with the reference's Hann window (FDutils.py:66-101 get_fd_windowed
 * with emri_pe.py:261's scipy hann(nf), sym=True) without size-nf DFTs: the windowed spectrum is
 *   S_w[k] = S[k]/2 - (S[k+1] + S[k-1])/4 - (C[k+1] - C[k-1]) / (4 (nf - 1)),   indices mod nf,
 * C = K (*) S the circular convolution with K[m] = -i pi/nf + (pi/nf) cot(pi m/nf),
 * K[0] = i pi (nf-1)/nf (the derivative of the DFT's trigonometric interpolant). C is the caller's
 * linear convolution of each row's support with K on m-point complex64 transforms
 * (fdutils.HannConvolution): rows of S (complex128 [nf], row r at S + 2 r stride doubles);
 * info[r] (4 x uint64 per row, device) = {bits of scale = max(|Re|, |Im|) over the row, first
 * nonzero bin, last nonzero bin + 1, 0} (first = ~0, last = 0 for an all-zero row; a NaN makes
 * the scale NaN); Y complex64 [rows][m], m >= nf + (last - first) - 1.
 *   efd_hann_extent: info from S. lanes (NULL, or device int32 [rows][2] from
 *                    efd_modesum_lane_ranges on the rows' workspaces, symmetric grids): only
 *                    the bins those lanes and their mirrors cover are read.
 *   efd_hann_stage:  Y[r][s] = S[r][first + s] / scale for s < last - first, 0 up to m. The
 *                    caller transforms Y in place: forward, times the lag kernel's spectrum
 *                    (z[t] = K[(t - (m - nf)) mod nf] / m), backward; then
 *                    C[k] = scale Y[r][((k - first) mod nf) + m - nf].
 *   efd_hann_polarizations: h+/hx (efd_polarizations' split) of one row's S_w over bins
 *                    [k0, nf) into hp, hc (complex [nf - k0]).
 *   efd_hann_loglike: efd_loglike of every row's windowed h+/hx against d, w ([2][nf - k0],
 *                    efd_loglike's layout and rounding), out[r] (device doubles [rows],
 *                    rows <= 16); scratch holds rows * EFD_LOGLIKE_SCRATCH doubles. No template
 *                    is written.
 * Replaces: no reference function (the reference convolves each channel with scipy/cupy at
 * FDutils.py:35-47, 95-96).
 */
int efd_hann_extent(const double* S, int64_t stride, int64_t nf, int32_t rows,
                    const int32_t* lanes, uint64_t* info, void* stream);
int efd_hann_stage(const double* S, int64_t stride, int64_t nf, int32_t rows,
                   const uint64_t* info, int64_t m, float* Y, void* stream);
/* efd_hann_stage + the caller's transform pair in one call, for power-of-two m in [2^21, 2^25]
 * (a four-step FFT: column FFTs of length R = m / C with the staging folded in, row FFTs of
 * C with the kernel multiply between forward and inverse, inverse column FFTs; the spectrum is
 * never reordered; C = efd_hann_four_step_cols(m)). kfp: the lag kernel's spectrum / m,
 * complex64 in the four-step order kfp[f_r C + f_c] = kf[f_r + R f_c]. Leaves Y as
 * efd_hann_stage + transforms do. */
int efd_hann_convolve(const double* S, int64_t stride, int64_t nf, int32_t rows,
                      const uint64_t* info, int64_t m, const float* kfp, float* Y, void* stream);
/* The four-step split's row length C that efd_hann_convolve uses for transform length m
 * (R = m / C; kfp's layout above with 8192 replaced by C): 16384 at m = 2^24, else 8192. */
int efd_hann_four_step_cols(int64_t m);
/* The windowed logL with the correction reduced inside efd_hann_convolve's inverse column pass
 * (no correction array written or read back): the reference's per-channel window convolution
 * (FDutils.py:95-96 under emri_pe.py:259-263) followed by Likelihood.get_ll's reduction
 * (likelihood.py:257-274), for a walker group. With the same weight w on both channels the two
 * channels' terms of a kept bin k and of its mirror k' = nf-1-k recombine into one term per bin:
 *   sum_k |d0 - w h+|^2 + |d1 - w hx|^2 = (1/2) sum_j |dl[j] - wl[j] S_w[j]|^2,
 * dl[k] = d0[k] - i d1[k], dl[k'] = conj(d0[k] + i d1[k]), wl = w at both (complex128 [nf + 1]
 * and float64 [nf]; the self-mirror bin kself, or -1, takes its second term from dl[nf]; other
 * bins hold 0). kfd: kfp times 2i sin(2 pi f / m) (the transforms then give the correction's
 * difference C[k+1] - C[k-1] directly); m >= nf + the rows' longest support (a longer support
 * makes the row's logL NaN). out[r] = -2 sum (efd_hann_loglike's value, up to rounding);
 * scratch: rows * efd_hann_loglike_local_partials(m) (<= 4096) doubles. emit (device complex128
 * [nf + 1], rows = 1; dl, out, scratch unused): writes wl[j] S_w[j] (and emit[nf] at kself)
 * instead, the dl of an injection made by this same arithmetic: the logL of the same spectrum
 * against it is exactly 0. */
int efd_hann_loglike_local(const double* S, int64_t stride, int64_t nf, int32_t rows,
                           const uint64_t* info, int64_t m, const float* kfd, float* Y,
                           const double* dl, const double* wl, int64_t kself, double* out,
                           double* scratch, double* emit, void* stream);
/* The partial sums per row efd_hann_loglike_local writes at transform length m (0: not a
 * four-step length). */
int efd_hann_loglike_local_partials(int64_t m);
int efd_hann_polarizations(const double* S, const float* Y, const uint64_t* info, int64_t m,
                           int64_t nf, int64_t k0, double* hp, double* hc, void* stream);

/*
 * Fused Gaussian log-likelihood over nchan channels of nbin bins each:
 *   out = -1/2 * 4 * sum_c sum_k | d[c][k] - h[c][k] * w[c][k] |^2
 * (likelihood.py:257-274 with noise factor w = sqrt(df/S) built at likelihood.py:213-220).
 * h, d complex [nchan][nbin]; w real [nchan][nbin]; out is one device double; scratch holds
 * EFD_LOGLIKE_SCRATCH device doubles. h = NULL gives the data-only term -2 sum |d|^2.
 * Bitwise reproducible (fixed partition and reduction order).
 */
#define EFD_LOGLIKE_SCRATCH 1024
int efd_loglike(const double* h, const double* d, const double* w, int32_t nchan, int64_t nbin,
                double* out, double* scratch, void* stream);
/* the windowed log-likelihood of rows of spectra (see efd_hann_extent above) */
int efd_hann_loglike(const double* S, int64_t stride, const float* Y, const uint64_t* info,
                     int64_t m, int32_t rows, int64_t nf, int64_t k0, const double* d,
                     const double* w, double* out, double* scratch, void* stream);

/*
 * Noise-weighted inner product over nchan channels of nbin bins each:
 *   out[0] + i out[1] = 4 * sum_c sum_k conj(a[c][k]) * b[c][k] * w[c][k]
 * (lisatools diagnostic.py:95-110: right-sum rule, w = diff(f) / PSD with the first spacing
 * repeated; inner_product takes out[0], or both parts with complex=True). a, b complex
 * [nchan][nbin]; w real [nchan][nbin] or NULL (w = 1); out is two device doubles; scratch
 * holds EFD_INNER_SCRATCH device doubles. Bitwise reproducible.
 */
#define EFD_INNER_SCRATCH 2048
int efd_inner_product(const double* a, const double* b, const double* w, int32_t nchan,
                      int64_t nbin, double* out, double* scratch, void* stream);

/*
 * CPU twins: the same algorithm on HOST pointers, C++17 + OpenMP
 * (csrc/emrifd_cpu.cpp, linked into libemrifd.so). Signatures are those of the HIP entry points;
 * `stream`, `workspace` and `scratch` are accepted for parity and ignored (pass NULL / 0). The
 * reference's CPU path is the numpy branch of the same FEW generator (check_mode_by_mode.py:50-60,
 * emri_pe.py:68-80); these twins are the CPU baseline bench.py times at 1 thread and all cores.
 * efd_modesum_cpu: the same grouping, splines, interval records and tile-wise output-stationary
 * sum with the uniform K_{1/3} fast path as efd_modesum, exact IEEE divisions / square roots;
 * synchronous. Errors (EFD_ERR_ARG) are reported by return code + efd_cpu_last_error.
 */
int efd_modesum_cpu(const efd_modesum_args* a, void* workspace, size_t workspace_bytes,
                    void* stream);
/* Counters of the calling thread's last efd_modesum_cpu (as efd_modesum_stats). */
int efd_modesum_cpu_stats(int64_t* contributions, int64_t* evaluations, int32_t* groups);
int efd_spline_build_cpu(const double* x, int n, const double* y, int ninterp, double* coef,
                         void* stream);
int efd_polarizations_cpu(const double* S, int64_t nf, int64_t k0, double* hp, double* hc,
                          void* stream);
int efd_loglike_cpu(const double* h, const double* d, const double* w, int32_t nchan,
                    int64_t nbin, double* out, double* scratch, void* stream);
int efd_inner_product_cpu(const double* a, const double* b, const double* w, int32_t nchan,
                          int64_t nbin, double* out, double* scratch, void* stream);
/* OpenMP threads of the twins (n <= 0: all available); returns the previous setting. */
int efd_cpu_threads(int n);
/* Last error message of the calling thread's CPU-twin call. */
int efd_cpu_last_error(char* buf, int len);

/*
 * Host upstream of the hot path (csrc/emrifd_host.cpp): STAND-IN PHYSICS, NOT FEW (FEW's flux
 * and amplitude data are absent offline). The C++ form of the package's Python stand-ins, with
 * the same equations and integrator (scipy RK45's Dormand-Prince 5(4), step control, dense
 * output and terminal separatrix event). Host pointers, synchronous, thread-safe.
 *
 * efd_host_trajectory <- EMRIInspiral(func="SchwarzEccFlux")(M, mu, 0, p0, e0, 1, T=T)
 *   (check_mode_by_mode.py:34-35): Peters-Mathews fluxes, exact Schwarzschild frequencies; knots
 *   t [s], p, e, Phi_phi, Phi_r and (optional, NULL to skip) f_phi, f_r = Omega / (2 pi M
 *   MTSUN_SI) [Hz], at most max_len (EFD_ERR_WORKSPACE beyond); *nt = knot count.
 * efd_host_p_at_t <- few.utils.utility.get_p_at_t (check_mode_by_mode.py:200-212): p0 whose
 *   inspiral plunges after t_out years (Brent; bracket [lo, hi], <= 0 for the defaults).
 * efd_host_modes <- RomanAmplitude + ModeSelector(eps) (notebook :125-127): the synthetic
 *   amplitude model over the given mode list (l, m, n, seeded phase0 and jitter), selection of
 *   the modes holding (1 - eps) of |A Y|^2 at every knot (+m and -m partner branches, union over
 *   knots) into keep[*nkeep]; with teuk != NULL also their complex amplitudes [nt][*nkeep]
 *   (EFD_ERR_WORKSPACE when 2 nt nkeep > teuk_cap doubles).
 */
int efd_host_trajectory(double M, double mu, double p0, double e0, double Phi_phi0, double Phi_r0,
                        double T, double rtol, double atol, int32_t max_len, double* t, double* p,
                        double* e, double* phi_phi, double* phi_r, double* f_phi, double* f_r,
                        int32_t* nt);
int efd_host_p_at_t(double M, double mu, double e0, double t_out, double rtol, double atol,
                    double xtol, double rtol_root, double lo, double hi, double* p0);
int efd_host_modes(const double* p, const double* e, int32_t nt, const int32_t* l,
                   const int32_t* m, const int32_t* n, const double* phase0, const double* jitter,
                   int32_t nmodes, const double* ylm_p, const double* ylm_m, double eps,
                   int32_t* keep, int32_t* nkeep, double* teuk, int64_t teuk_cap);
/* Threads the calling thread's later efd_host_modes calls spread their knots over (default 1;
 * the setting is per calling thread). Any count gives bitwise the same results. */
int efd_host_set_threads(int32_t n);

/*
 * Host staging of a walker batch for efd_modesum_prepare_batch (not part of the reference's
 * interface; the batched Likelihood's packing step, likelihood.py:246-274 callers): the ten
 * input arrays of walker i (src[10 i + f]: t, phi_phi, phi_r, f_phi, f_r, amp [nt][K] complex,
 * m, n, ylm_p, ylm_m; nt = shape[2 i], K = shape[2 i + 1]) are copied 256-B aligned into the
 * host buffer pin, and args[i] becomes *tmpl with walker i's nt, K, scale (scale[2 i] + i
 * scale[2 i + 1]) and device pointers dev_base + offset (valid after pin is copied to
 * dev_base). *total = bytes needed; EFD_ERR_WORKSPACE (nothing copied) when pin_bytes is less.
 */
int efd_stage_batch(void* pin, size_t pin_bytes, uint64_t dev_base, int32_t count,
                    const uint64_t* src, const int32_t* shape, const double* scale,
                    const efd_modesum_args* tmpl, efd_modesum_args* args, size_t* total);

/*
 * One walker group of the fused likelihood in one call: efd_stage_batch(pin, pin_bytes, dbuf,
 * count, src, shape, scale, tmpl, args, total), the host-to-device copy of pin to dbuf on
 * `stream`, staged_event (a hipEvent_t, or NULL) recorded after it, then
 * efd_modesum_prepare_batch and efd_modesum_sum_loglike_ex(args, workspace, workspace_bytes,
 * d, w, tile_const, out) in launches of EFD_BATCH_MAX walkers on `stream`. EFD_ERR_WORKSPACE
 * with *total set and nothing queued when pin or dbuf is shorter than *total. Not part of the
 * reference's interface: Likelihood.get_ll's per-group host steps (likelihood.py:246-274
 * callers) in one native call.
 */
int efd_fused_group(void* pin, size_t pin_bytes, void* dbuf, size_t dbuf_bytes, int32_t count,
                    const uint64_t* src, const int32_t* shape, const double* scale,
                    const efd_modesum_args* tmpl, efd_modesum_args* args,
                    void* const* workspace, const size_t* workspace_bytes, const double* d,
                    const double* w, const double* tile_const, double* out, void* staged_event,
                    void* stream, size_t* total);

#ifdef __cplusplus
}
#endif

#endif /* EMRIFD_H */
