// emrifd_host.cpp -- the host upstream of the hot path in C++ (linked into libemrifd.so):
// trajectory and p0 root solve for one source.
//
// STAND-IN PHYSICS, NOT FEW: FEW's SchwarzEccFlux trajectory and ROMAN amplitude network need
// data files absent offline. This is the C++ form of this
// package's Python stand-ins, same equations and the same integrator:
//   trajectory.py  Peters-Mathews (quadrupole) fluxes in (p, e), exact Schwarzschild
//                  Omega_phi, Omega_r (frequencies.py: 64-node trapezoid over the relativistic
//                  anomaly) for the phases; scipy's RK45 (Dormand-Prince 5(4), its step-size
//                  control, dense output and terminal-event root) at rtol = atol = 1e-12,
//                  stopping 0.1 outside the separatrix p = 6 + 2e or at T
//                  (EMRIInspiral(func="SchwarzEccFlux"), check_mode_by_mode.py:34-35)
//   get_p_at_t     Brent's root of t_plunge(p0) = t_out (few.utils.utility.get_p_at_t,
//                  check_mode_by_mode.py:200-212)
// (the amplitude stand-in and mode selection are in emrifd_modes.cpp, built with vector math)
// so the drivers' upstream (30-50 ms per walker in numpy/scipy) costs ~1-3 ms per source and
// releases the GIL: the Python layer runs a batch of walkers on a thread pool.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/emrifd.h"

namespace efdhost {

constexpr double MTSUN_SI = 4.925491025543576e-06;
constexpr double YRSID_SI = 31558149.763545603;
constexpr double TWO_PI = 6.283185307179586476925286766559005768;
constexpr double DIST_TO_SEPARATRIX = 0.1;
constexpr int NCHI = 64;

struct CosTable {
    double c[NCHI];
    CosTable() {
        for (int i = 0; i < NCHI; ++i) c[i] = std::cos(TWO_PI * i / NCHI);
    }
};
const CosTable& costab() {
    static const CosTable t;
    return t;
}

// Omega_phi, Omega_r of a Schwarzschild eccentric equatorial orbit (frequencies.py)
inline void fundamental(double p, double e, double& om_phi, double& om_r) {
    const double* c = costab().c;
    double sdt = 0.0, sdphi = 0.0;
    const double k = (p - 2.0) * (p - 2.0) - 4.0 * e * e;
    for (int i = 0; i < NCHI; ++i) {
        const double ec = e * c[i];
        const double den = p - 6.0 - 2.0 * ec;
        const double dphi = std::sqrt(p / den);
        const double q = 1.0 + ec;
        const double dt = p * p / ((p - 2.0 - 2.0 * ec) * q * q) * std::sqrt(k / den);
        sdt += dt;
        sdphi += dphi;
    }
    const double t_r = sdt / NCHI * TWO_PI, phi_r = sdphi / NCHI * TWO_PI;
    om_phi = phi_r / t_r;
    om_r = TWO_PI / t_r;
}

// d/d tau of (p, e, Phi_phi, Phi_r), tau = t / M (trajectory.py _pn_rhs)
inline void rhs(const double* y, double q, double* f) {
    const double p = y[0], e = y[1], e2 = e * e;
    const double a = p / (1.0 - e2);
    const double da = -(64.0 / 5.0) * q / (a * a * a * std::pow(1.0 - e2, 3.5)) *
                      (1.0 + 73.0 / 24.0 * e2 + 37.0 / 96.0 * e2 * e2);
    const double de = -(304.0 / 15.0) * q * e / (a * a * a * a * std::pow(1.0 - e2, 2.5)) *
                      (1.0 + 121.0 / 304.0 * e2);
    f[0] = (1.0 - e2) * da - 2.0 * a * e * de;
    f[1] = de;
    fundamental(p, e, f[2], f[3]);
}

inline double sep_event(const double* y) { return y[0] - (6.0 + 2.0 * y[1]) - DIST_TO_SEPARATRIX; }

// scipy RK45 tableau, error weights and dense-output matrix
constexpr double C[6] = {0.0, 1.0 / 5, 3.0 / 10, 4.0 / 5, 8.0 / 9, 1.0};
constexpr double A[6][5] = {{0, 0, 0, 0, 0},
                            {1.0 / 5, 0, 0, 0, 0},
                            {3.0 / 40, 9.0 / 40, 0, 0, 0},
                            {44.0 / 45, -56.0 / 15, 32.0 / 9, 0, 0},
                            {19372.0 / 6561, -25360.0 / 2187, 64448.0 / 6561, -212.0 / 729, 0},
                            {9017.0 / 3168, -355.0 / 33, 46732.0 / 5247, 49.0 / 176, -5103.0 / 18656}};
constexpr double B[6] = {35.0 / 384, 0.0, 500.0 / 1113, 125.0 / 192, -2187.0 / 6784, 11.0 / 84};
constexpr double E[7] = {-71.0 / 57600, 0.0, 71.0 / 16695, -71.0 / 1920, 17253.0 / 339200,
                         -22.0 / 525, 1.0 / 40};
constexpr double P[7][4] = {
    {1.0, -8048581381.0 / 2820520608, 8663915743.0 / 2820520608, -12715105075.0 / 11282082432},
    {0.0, 0.0, 0.0, 0.0},
    {0.0, 131558114200.0 / 32700410799, -68118460800.0 / 10900136933, 87487479700.0 / 32700410799},
    {0.0, -1754552775.0 / 470086768, 14199869525.0 / 1410260304, -10690763975.0 / 1880347072},
    {0.0, 127303824393.0 / 49829197408, -318862633887.0 / 49829197408, 701980252875.0 / 199316789632},
    {0.0, -282668133.0 / 205662961, 2019193451.0 / 616988883, -1453857185.0 / 822651844},
    {0.0, 40617522.0 / 29380423, -110615467.0 / 29380423, 69997945.0 / 29380423}};
constexpr int NY = 4;

// Brent's method (scipy brentq's algorithm) for f(a), f(b) of opposite signs
template <class F>
double brentq(F f, double xa, double xb, double xtol, double rtol, int maxiter = 100) {
    double xpre = xa, xcur = xb, xblk = 0.0, fblk = 0.0, spre = 0.0, scur = 0.0;
    double fpre = f(xpre), fcur = f(xcur);
    if (fpre == 0.0) return xpre;
    if (fcur == 0.0) return xcur;
    for (int i = 0; i < maxiter; ++i) {
        if (fpre != 0.0 && fcur != 0.0 && (std::signbit(fpre) != std::signbit(fcur))) {
            xblk = xpre;
            fblk = fpre;
            spre = scur = xcur - xpre;
        }
        if (std::fabs(fblk) < std::fabs(fcur)) {
            xpre = xcur; xcur = xblk; xblk = xpre;
            fpre = fcur; fcur = fblk; fblk = fpre;
        }
        const double delta = (xtol + rtol * std::fabs(xcur)) / 2.0;
        const double sbis = (xblk - xcur) / 2.0;
        if (fcur == 0.0 || std::fabs(sbis) < delta) return xcur;
        if (std::fabs(spre) > delta && std::fabs(fcur) < std::fabs(fpre)) {
            double stry;
            if (xpre == xblk) {
                stry = -fcur * (xcur - xpre) / (fcur - fpre);   // interpolate
            } else {                                             // extrapolate
                const double dpre = (fpre - fcur) / (xpre - xcur);
                const double dblk = (fblk - fcur) / (xblk - xcur);
                stry = -fcur * (fblk * dblk - fpre * dpre) / (dblk * dpre * (fblk - fpre));
            }
            if (2.0 * std::fabs(stry) < std::min(std::fabs(spre), 3.0 * std::fabs(sbis) - delta)) {
                spre = scur;   // good short step
                scur = stry;
            } else {
                spre = sbis;   // bisect
                scur = sbis;
            }
        } else {
            spre = sbis;
            scur = sbis;
        }
        xpre = xcur;
        fpre = fcur;
        if (std::fabs(scur) > delta) xcur += scur;
        else xcur += (sbis > 0 ? delta : -delta);
        fcur = f(xcur);
    }
    return xcur;
}

// The sparse inspiral: knots (tau, y) of the accepted RK45 steps, ending at the separatrix event
// or at tau_max. Returns the knot count, -1 past max_len, -2 on a failed step.
int integrate(double p0, double e0, double pp0, double pr0, double q, double tau_max,
              double rtol, double atol, int max_len, std::vector<double>& ts,
              std::vector<double>& ys) {
    ts.clear();
    ys.clear();
    double t = 0.0, y[NY] = {p0, e0, pp0, pr0}, f[NY];
    rhs(y, q, f);
    double h_abs = std::min(1e-3 * tau_max, 1e4);   // first_step (trajectory.py)
    ts.push_back(t);
    ys.insert(ys.end(), y, y + NY);
    double g = sep_event(y);
    double K[7][NY];
    const double err_exp = -1.0 / 5.0;
    while (t < tau_max) {
        const double min_step = 10.0 * std::fabs(std::nextafter(t, INFINITY) - t);
        if (h_abs < min_step) h_abs = min_step;
        bool accepted = false, rejected = false;
        double t_new = t, y_new[NY], f_new[NY], h = 0.0;
        while (!accepted) {
            if (h_abs < min_step) return -2;
            h = h_abs;
            t_new = t + h;
            if (t_new - tau_max > 0) t_new = tau_max;
            h = t_new - t;
            h_abs = std::fabs(h);
            for (int k = 0; k < NY; ++k) K[0][k] = f[k];
            for (int s = 1; s < 6; ++s) {
                double ys_[NY];
                for (int k = 0; k < NY; ++k) {
                    double dy = 0.0;
                    for (int r = 0; r < s; ++r) dy += K[r][k] * A[s][r];
                    ys_[k] = y[k] + dy * h;
                }
                rhs(ys_, q, K[s]);
            }
            for (int k = 0; k < NY; ++k) {
                double acc = 0.0;
                for (int r = 0; r < 6; ++r) acc += K[r][k] * B[r];
                y_new[k] = y[k] + h * acc;
            }
            rhs(y_new, q, f_new);
            for (int k = 0; k < NY; ++k) K[6][k] = f_new[k];
            double en = 0.0;
            for (int k = 0; k < NY; ++k) {
                double ek = 0.0;
                for (int r = 0; r < 7; ++r) ek += K[r][k] * E[r];
                ek *= h;
                const double sc = atol + std::max(std::fabs(y[k]), std::fabs(y_new[k])) * rtol;
                en += (ek / sc) * (ek / sc);
            }
            en = std::sqrt(en) / std::sqrt((double)NY);
            if (en < 1.0) {
                double factor = en == 0.0 ? 10.0 : std::min(10.0, 0.9 * std::pow(en, err_exp));
                if (rejected) factor = std::min(1.0, factor);
                h_abs *= factor;
                accepted = true;
            } else {
                h_abs *= std::max(0.2, 0.9 * std::pow(en, err_exp));
                rejected = true;
            }
        }
        const double g_new = sep_event(y_new);
        if (g >= 0.0 && g_new <= 0.0) {   // terminal event (direction -1): root of the dense output
            double Q[NY][4];
            for (int k = 0; k < NY; ++k)
                for (int c = 0; c < 4; ++c) {
                    double acc = 0.0;
                    for (int r = 0; r < 7; ++r) acc += K[r][k] * P[r][c];
                    Q[k][c] = acc;
                }
            auto sol = [&](double tt, double* out) {
                const double x = (tt - t) / h;
                const double pw[4] = {x, x * x, x * x * x, x * x * x * x};
                for (int k = 0; k < NY; ++k) {
                    double acc = 0.0;
                    for (int c = 0; c < 4; ++c) acc += Q[k][c] * pw[c];
                    out[k] = h * acc + y[k];
                }
            };
            const double eps4 = 4.0 * 2.220446049250313e-16;
            const double te = brentq([&](double tt) { double yy[NY]; sol(tt, yy); return sep_event(yy); },
                                     t, t_new, eps4, eps4);
            double ye[NY];
            sol(te, ye);
            ts.push_back(te);
            ys.insert(ys.end(), ye, ye + NY);
            if ((int)ts.size() > max_len) return -1;
            return (int)ts.size();
        }
        g = g_new;
        t = t_new;
        for (int k = 0; k < NY; ++k) { y[k] = y_new[k]; f[k] = f_new[k]; }
        ts.push_back(t);
        ys.insert(ys.end(), y, y + NY);
        if ((int)ts.size() > max_len) return -1;
    }
    return (int)ts.size();
}

}  // namespace efdhost

extern "C" {

int efd_host_trajectory(double M, double mu, double p0, double e0, double Phi_phi0, double Phi_r0,
                        double T, double rtol, double atol, int32_t max_len, double* t, double* p,
                        double* e, double* phi_phi, double* phi_r, double* f_phi, double* f_r,
                        int32_t* nt) {
    using namespace efdhost;
    if (!t || !p || !e || !phi_phi || !phi_r || !nt || max_len < 2 || !(M > 0) || !(mu > 0))
        return EFD_ERR_ARG;
    if (p0 - (6.0 + 2.0 * e0) <= DIST_TO_SEPARATRIX) return EFD_ERR_ARG;
    const double tscale = M * MTSUN_SI;
    std::vector<double> ts, ys;
    const int n = integrate(p0, e0, Phi_phi0, Phi_r0, mu / M, T * YRSID_SI / tscale, rtol, atol,
                            max_len, ts, ys);
    if (n < 0) return n == -1 ? EFD_ERR_WORKSPACE : EFD_ERR_ARG;
    for (int i = 0; i < n; ++i) {
        t[i] = ts[i] * tscale;
        p[i] = ys[4 * i];
        e[i] = ys[4 * i + 1];
        phi_phi[i] = ys[4 * i + 2];
        phi_r[i] = ys[4 * i + 3];
        if (f_phi && f_r) {
            double op, orr;
            fundamental(p[i], e[i], op, orr);
            f_phi[i] = op / (TWO_PI * M * MTSUN_SI);
            f_r[i] = orr / (TWO_PI * M * MTSUN_SI);
        }
    }
    *nt = n;
    return EFD_OK;
}

int efd_host_p_at_t(double M, double mu, double e0, double t_out, double rtol, double atol,
                    double xtol, double rtol_root, double lo, double hi, double* p0) {
    using namespace efdhost;
    if (!p0 || !(M > 0) || !(mu > 0) || !(t_out > 0)) return EFD_ERR_ARG;
    const double tscale = M * MTSUN_SI;
    const double tau_max = (2.0 * t_out + 1.0) * YRSID_SI / tscale;
    std::vector<double> ts, ys;
    bool bad = false;
    auto f = [&](double pp) {
        const int n = integrate(pp, e0, 0.0, 0.0, mu / M, tau_max, rtol, atol, 1 << 20, ts, ys);
        if (n < 0) { bad = true; return 0.0; }
        return ts[n - 1] * tscale / YRSID_SI - t_out;
    };
    if (!(lo > 0)) lo = 6.0 + 2.0 * e0 + DIST_TO_SEPARATRIX + 1e-3;
    if (!(hi > 0)) hi = 40.0;
    if (f(lo) > 0) return EFD_ERR_ARG;          // t_out shorter than the plunge from the buffer
    while (f(hi) < 0) {
        hi *= 1.5;
        if (hi > 500) return EFD_ERR_ARG;
    }
    *p0 = brentq(f, lo, hi, xtol, std::max(rtol_root, 4 * 2.220446049250313e-16));
    return bad ? EFD_ERR_ARG : EFD_OK;
}

// Staging of a walker batch for efd_modesum_prepare_batch: the ten input arrays of each walker
// (src[10 i + f], f in t, phi_phi, phi_r, f_phi, f_r, amp, m, n, ylm_p, ylm_m; sizes from
// shape[2 i] = nt, shape[2 i + 1] = K) packed 256-B aligned into the pinned buffer, and each
// walker's argument struct (tmpl's grid, caustic and output fields; its own scale and the
// device pointers dev_base + offset, valid once pin has been copied to dev_base). The packing
// costs one memcpy per array instead of a Python slice assignment each.
int efd_stage_batch(void* pin, size_t pin_bytes, uint64_t dev_base, int32_t count,
                    const uint64_t* src, const int32_t* shape, const double* scale,
                    const efd_modesum_args* tmpl, efd_modesum_args* args, size_t* total) {
    if (!src || !shape || !scale || !tmpl || !args || !total || count < 1) return EFD_ERR_ARG;
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    size_t off = 0;
    for (int i = 0; i < count; ++i) {
        const size_t nt = (size_t)shape[2 * i], K = (size_t)shape[2 * i + 1];
        if (shape[2 * i] < 2 || shape[2 * i + 1] < 1) return EFD_ERR_ARG;
        const size_t bytes[10] = {8 * nt, 8 * nt, 8 * nt, 8 * nt, 8 * nt, 16 * nt * K,
                                  4 * K, 4 * K, 16 * K, 16 * K};
        for (int f = 0; f < 10; ++f) off = al(off + bytes[f]);
    }
    *total = off;
    if (!pin || off > pin_bytes) return EFD_ERR_WORKSPACE;
    char* dst = (char*)pin;
    // each walker's offset (the sizes pass above, again), then the copies: walkers over OpenMP
    // threads when the batch is large (config 5's groups of 16: ~2-4 MB, one thread's memcpy
    // bandwidth made the copy most of the group's flush)
    std::vector<size_t> woff((size_t)count + 1, 0);
    for (int i = 0; i < count; ++i) {
        const size_t nt = (size_t)shape[2 * i], K = (size_t)shape[2 * i + 1];
        const size_t bytes[10] = {8 * nt, 8 * nt, 8 * nt, 8 * nt, 8 * nt, 16 * nt * K,
                                  4 * K, 4 * K, 16 * K, 16 * K};
        size_t o = woff[i];
        for (int f = 0; f < 10; ++f) o = al(o + bytes[f]);
        woff[i + 1] = o;
        for (int f = 0; f < 10; ++f)
            if (!src[10 * (size_t)i + f]) return EFD_ERR_ARG;
    }
    const int nth = off >= ((size_t)1 << 20) ? std::min(count, 8) : 1;
#pragma omp parallel for num_threads(nth) schedule(static) if (nth > 1)
    for (int i = 0; i < count; ++i) {
        const size_t nt = (size_t)shape[2 * i], K = (size_t)shape[2 * i + 1];
        const size_t bytes[10] = {8 * nt, 8 * nt, 8 * nt, 8 * nt, 8 * nt, 16 * nt * K,
                                  4 * K, 4 * K, 16 * K, 16 * K};
        uint64_t dp[10];
        size_t o = woff[i];
        for (int f = 0; f < 10; ++f) {
            const void* sp = (const void*)(uintptr_t)src[10 * (size_t)i + f];
            std::memcpy(dst + o, sp, bytes[f]);
            dp[f] = dev_base + o;
            o = al(o + bytes[f]);
        }
        efd_modesum_args& a = args[i];
        a = *tmpl;
        a.t = (const double*)(uintptr_t)dp[0];
        a.phi_phi = (const double*)(uintptr_t)dp[1];
        a.phi_r = (const double*)(uintptr_t)dp[2];
        a.f_phi = (const double*)(uintptr_t)dp[3];
        a.f_r = (const double*)(uintptr_t)dp[4];
        a.amp = (const double*)(uintptr_t)dp[5];
        a.m = (const int32_t*)(uintptr_t)dp[6];
        a.n = (const int32_t*)(uintptr_t)dp[7];
        a.ylm_p = (const double*)(uintptr_t)dp[8];
        a.ylm_m = (const double*)(uintptr_t)dp[9];
        a.nt = (int32_t)nt;
        a.K = (int32_t)K;
        a.scale_re = scale[2 * i];
        a.scale_im = scale[2 * i + 1];
    }
    return EFD_OK;
}

}  // extern "C"
