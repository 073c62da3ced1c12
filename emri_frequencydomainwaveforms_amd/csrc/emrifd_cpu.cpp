// emrifd_cpu.cpp -- host twin of libemrifd.so's FD mode sum: the same algorithm in C++17 with
// OpenMP, on host pointers ("CPU twins efd_*_cpu(...) with identical
// signatures on host pointers"; section 8(d): the CPU baseline is the same algorithm, FP64,
// timed at 1 thread and at all cores).
//
// The reference's CPU path is the numpy/CPU branch of the same FEW generator
// (check_mode_by_mode.py:50-60, emri_pe.py:68-80, FDutils.py:7-17). FEW's CPU backend is absent
// offline, so the twin restates this library's own construction on the CPU:
//   (m, n) grouping, members ascending h                       k_group
//   group amplitudes Bp = sum_l y0 A, Bm = sum_l y1 A           k_group_amp
//   not-a-knot splines: trajectory (Phi_phi, Phi_r, f_phi, f_r, knot slopes of f_phi and f_r),
//   group amplitudes, inverse splines t(F) per monotonic run   k_prep
//   one interval record per (group, knot interval)              k_items
//   output-stationary sum over 768-lane tiles (per-tile record lists, one SPA evaluation per
//   (record, lane) feeding the lane's bin and its mirror), uniform K_{1/3} factor in polar
//   form from the record's series length, sin/cos from the 512-entry table
//                                                               k_tile_keys + k_modesum
//   general path (interval overshoot, small |y|): scipy interval search and the full K_{1/3}
//                                                               spa_general
// Differences from the kernel are rounding only: exact IEEE divisions and square roots in place
// of the reciprocal / rsqrt estimates with Newton steps, and the records' order within a tile.
// Lanes vectorise with `omp simd` (AVX-512 gathers for the sin/cos table); tiles and groups run
// in parallel with OpenMP. Nothing here touches the GPU.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include <omp.h>

#include "../../include/emrifd.h"

namespace efdcpu {

struct double2 {
    double x, y;
};
#define EFD_TABLE static const
#include "spa_tables.inc"
#undef EFD_TABLE

constexpr int TL = 768;             // lanes per tile (the kernel's TILE * BPL)
constexpr int MAXRUNS = 8;
constexpr int MAX_NT = 1024;
constexpr int MAX_K = 8192;
constexpr int FAST_J = 4;
constexpr double FAST_Y = 153.0;
constexpr double PI = 3.141592653589793238462643383279502884;
constexpr double TWO_PI = 6.283185307179586476925286766559005768;
constexpr double VS = 0.18633899812498247470;             // sqrt|KRH_1|
constexpr double FDD_SCALE = 0.29827892638794838654;      // sqrt(3/(2 pi)) |KRH_1|^(1/4)
constexpr double INV_FDD_SCALE = 3.3525667136785156343;
constexpr double KTH0 = -0.069444444444444444444;
// the kernel's cosine on |r| <= pi/512 (emrifd.hip, sincos_tab): minimax line in r^2
constexpr double COS_A = 1.000000000029531;
constexpr double COS_B = -0.5;
constexpr double KTAB_WMIN = 0x1p-8, KTAB_WMAX = 0x1p10;
using std::fabs;
using std::fma;
using std::fmax;
using std::sqrt;
inline double env_rsqrt(double x) { return 1.0 / std::sqrt(x); }
#define EFD_HD
#include "env_fit.inc"
#undef EFD_HD

thread_local std::string g_err;
thread_local int64_t g_stats[3];    // contributions, evaluations, groups of the last call
int g_threads = 0;                  // 0: all of omp_get_max_threads()
int g_env = -1;                     // envelope records: -1 unset (EFD_ENV, default on), 0 off, 1 on
bool env_enabled() {
    if (g_env < 0) {
        const char* e = std::getenv("EFD_ENV");
        g_env = (e && e[0] == '0') ? 0 : 1;
    }
    return g_env != 0;
}

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int nthreads() { return g_threads > 0 ? g_threads : omp_get_max_threads(); }

// ---- not-a-knot cubic spline (scipy.interpolate.CubicSpline; n = 2 line, n = 3 parabola) --
// coef[i][0..3] in PPoly order for interval i; X(i), Y(i) accessors.
template <class FX, class FY>
void spline_nak(int n, FX X, FY Y, double (*coef)[4], std::vector<double>& cp,
                std::vector<double>& dp, std::vector<double>& s) {
    cp.resize(n);
    dp.resize(n);
    s.resize(n);
    if (n == 2) {
        const double sl = (Y(1) - Y(0)) / (X(1) - X(0));
        coef[0][0] = 0.0; coef[0][1] = 0.0; coef[0][2] = sl; coef[0][3] = Y(0);
        return;
    }
    if (n == 3) {
        const double dx0 = X(1) - X(0), dx1 = X(2) - X(1);
        const double sl0 = (Y(1) - Y(0)) / dx0, sl1 = (Y(2) - Y(1)) / dx1;
        s[1] = (dx0 * sl1 + dx1 * sl0) / (dx0 + dx1);
        s[0] = 2.0 * sl0 - s[1];
        s[2] = 2.0 * sl1 - s[1];
    } else {
        {
            const double dx0 = X(1) - X(0), dx1 = X(2) - X(1);
            const double sl0 = (Y(1) - Y(0)) / dx0, sl1 = (Y(2) - Y(1)) / dx1;
            const double d = X(2) - X(0);
            cp[0] = d / dx1;
            dp[0] = (((dx0 + 2.0 * d) * dx1 * sl0 + dx0 * dx0 * sl1) / d) / dx1;
        }
        for (int i = 1; i <= n - 2; ++i) {
            const double dxm = X(i) - X(i - 1), dxi = X(i + 1) - X(i);
            const double slm = (Y(i) - Y(i - 1)) / dxm, sli = (Y(i + 1) - Y(i)) / dxi;
            const double a = dxi, b = 2.0 * (dxm + dxi), c = dxm, r = 3.0 * (dxi * slm + dxm * sli);
            const double mm = b - a * cp[i - 1];
            cp[i] = c / mm;
            dp[i] = (r - a * dp[i - 1]) / mm;
        }
        const double dxm = X(n - 2) - X(n - 3), dxi = X(n - 1) - X(n - 2);
        const double slm = (Y(n - 2) - Y(n - 3)) / dxm, sli = (Y(n - 1) - Y(n - 2)) / dxi;
        const double dd = X(n - 1) - X(n - 3);
        const double r = (dxi * dxi * slm + (2.0 * dd + dxi) * dxm * sli) / dd;
        s[n - 1] = (r - dd * dp[n - 2]) / (dxm - dd * cp[n - 2]);
        for (int i = n - 2; i >= 0; --i) s[i] = dp[i] - cp[i] * s[i + 1];
    }
    for (int i = 0; i < n - 1; ++i) {
        const double dx = X(i + 1) - X(i);
        const double sl = (Y(i + 1) - Y(i)) / dx;
        const double tt = (s[i] + s[i + 1] - 2.0 * sl) / dx;
        coef[i][0] = tt / dx;
        coef[i][1] = (sl - s[i]) / dx - tt;
        coef[i][2] = s[i];
        coef[i][3] = Y(i);
    }
}

inline double cubic(const double* c, double w) {
    return std::fma(std::fma(std::fma(c[0], w, c[1]), w, c[2]), w, c[3]);
}
inline double dcubic(const double* c, double w) {   // scipy's derivative by power sum
    return (c[2] + (2.0 * c[1]) * w) + (3.0 * c[0]) * (w * w);
}

// ---- interval record of one (group, knot interval); the kernel's Item without the padding
struct Rec {
    double gx;
    double ic[4];          // inverse cubic t(g), u = g - gx
    double tj, dtj;        // forward interval [tj, tj + dtj)
    double ph[4];          // Phi_mn(t)
    double fd[3];          // F'(t)
    double fdd[3];         // FDD_SCALE * F''(t)
    double b[2][2][4];     // Bp, Bm (re, im cubics)
    int32_t klo[2], khi[2];
    int32_t jser, fdneg;
    int32_t h, j;          // group, interval (general path)
    // envelope record (env_fit.inc, as k_items): A(w) of degree ENV_DEG and the phase cubic with
    // theta folded in; the general path keeps ph, fd, fdd
    int32_t envc;
    double env[ENV_DEG + 1];
    double phE[4];
};

struct Prep {
    int nt = 0, K = 0, G = 0;
    std::vector<int32_t> gm, gn, gstart, gmem;
    std::vector<double> coefT;   // [ni][4][8]
    std::vector<double> coefA;   // [ni][4][4G]
    std::vector<Rec> recs;       // [G][ni]
    int64_t contributions = 0, evaluations = 0;
};

inline double knotF(const double* fphi, const double* fr, int m, int n, int i) {
    const double a = (double)m * fphi[i];
    const double b = (double)n * fr[i];
    return a + b;   // numpy's m f_phi + n f_r (this file is built without FMA contraction)
}

int prepare(const efd_modesum_args* a, Prep& P, bool paired, int64_t nl, int64_t nl1) {
    const int nt = a->nt, K = a->K, ni = nt - 1;
    P.nt = nt;
    P.K = K;
    // ---- (m, n) groups, members ascending h
    std::vector<int32_t> idx(K);
    std::iota(idx.begin(), idx.end(), 0);
    for (int i = 0; i < K; ++i)
        if (a->m[i] < -256 || a->m[i] > 255 || a->n[i] < -1024 || a->n[i] > 1023)
            return fail(EFD_ERR_ARG, "efd_modesum_cpu: |m| > 255 or |n| > 1023");
    std::stable_sort(idx.begin(), idx.end(), [&](int x, int y) {
        return a->m[x] != a->m[y] ? a->m[x] < a->m[y] : a->n[x] < a->n[y];
    });
    P.gm.clear(); P.gn.clear(); P.gstart.clear();
    for (int p = 0; p < K; ++p) {
        const int h = idx[p];
        if (p == 0 || a->m[h] != a->m[idx[p - 1]] || a->n[h] != a->n[idx[p - 1]]) {
            P.gm.push_back(a->m[h]);
            P.gn.push_back(a->n[h]);
            P.gstart.push_back(p);
        }
    }
    const int G = (int)P.gm.size();
    P.G = G;
    P.gstart.push_back(K);
    P.gmem = idx;
    const double sr = a->scale_re, si = a->scale_im;
    // ---- trajectory splines: Phi_phi, Phi_r, f_phi, f_r, then the knot slopes of f_phi, f_r
    P.coefT.assign((size_t)ni * 32, 0.0);
    std::vector<double> cpv, dpv, sv;
    std::vector<double> tmp((size_t)ni * 4);
    auto X = [&](int i) { return a->t[i]; };
    const double* ys[4] = {a->phi_phi, a->phi_r, a->f_phi, a->f_r};
    std::vector<double> slope((size_t)2 * nt);
    for (int q = 0; q < 6; ++q) {
        const double* y = q < 4 ? ys[q] : slope.data() + (size_t)(q - 4) * nt;
        spline_nak(nt, X, [&](int i) { return y[i]; }, reinterpret_cast<double(*)[4]>(tmp.data()),
                   cpv, dpv, sv);
        for (int i = 0; i < ni; ++i)
            for (int c = 0; c < 4; ++c) P.coefT[((size_t)i * 4 + c) * 8 + q] = tmp[(size_t)i * 4 + c];
        if (q == 2 || q == 3) {   // knot values of the derivative (scipy's derivative PPoly)
            double* o = slope.data() + (size_t)(q - 2) * nt;
            for (int i = 0; i < ni; ++i) o[i] = tmp[(size_t)i * 4 + 2];
            o[nt - 1] = dcubic(&tmp[(size_t)(ni - 1) * 4], a->t[nt - 1] - a->t[nt - 2]);
        }
    }
    // ---- group amplitudes and their splines: coefA[i][c][4g + q]
    P.coefA.assign((size_t)ni * 4 * 4 * G, 0.0);
    std::vector<double> gamp((size_t)nt * 4 * G);
#pragma omp parallel for schedule(static) num_threads(nthreads())
    for (int g = 0; g < G; ++g) {
        const bool partner = P.gm[g] != 0;
        for (int i = 0; i < nt; ++i) {
            double bpr = 0.0, bpi = 0.0, bmr = 0.0, bmi = 0.0;
            for (int p = P.gstart[g]; p < P.gstart[g + 1]; ++p) {
                const int h = P.gmem[p];
                const double ar = a->amp[((size_t)i * K + h) * 2], ai = a->amp[((size_t)i * K + h) * 2 + 1];
                const double vr = a->ylm_p[2 * h], vi = a->ylm_p[2 * h + 1];
                const double y0r = -(sr * vr - si * vi), y0i = -(sr * vi + si * vr);
                bpr += ar * y0r - ai * y0i;
                bpi += ar * y0i + ai * y0r;
                if (partner) {
                    const double ur = a->ylm_m[2 * h], ui = a->ylm_m[2 * h + 1];
                    const double y1r = -(sr * ur - si * ui), y1i = (sr * ui + si * ur);
                    bmr += ar * y1r - ai * y1i;
                    bmi += ar * y1i + ai * y1r;
                }
            }
            double* o = gamp.data() + (size_t)i * 4 * G + 4 * g;
            o[0] = bpr; o[1] = bpi; o[2] = bmr; o[3] = bmi;
        }
    }
#pragma omp parallel num_threads(nthreads())
    {
        std::vector<double> c1, d1, s1, tq((size_t)ni * 4);
#pragma omp for schedule(static)
        for (int q = 0; q < 4 * G; ++q) {
            spline_nak(nt, X, [&](int i) { return gamp[(size_t)i * 4 * G + q]; },
                       reinterpret_cast<double(*)[4]>(tq.data()), c1, d1, s1);
            for (int i = 0; i < ni; ++i)
                for (int c = 0; c < 4; ++c)
                    P.coefA[((size_t)i * 4 + c) * 4 * G + q] = tq[(size_t)i * 4 + c];
        }
    }
    // ---- inverse splines per monotonic run and the interval records
    P.recs.assign((size_t)G * ni, Rec{});
    const double* freq = a->freq;
    const int64_t nf = a->nf;
    const int64_t lim0 = paired ? nl : nf;
    const bool env_on = a->caustic == EFD_CAUSTIC_UNIFORM && env_enabled();
    int bad = 0;
    int64_t evals_total = 0, contrib_total = 0;
#pragma omp parallel num_threads(nthreads()) reduction(+ : evals_total, contrib_total) reduction(| : bad)
    {
        std::vector<double> c1, d1, s1, ti((size_t)nt * 4);
#pragma omp for schedule(dynamic, 4)
        for (int g = 0; g < G; ++g) {
            const int m = P.gm[g], n = P.gn[g];
            const bool partner = m != 0;
            const int64_t lim1 = paired ? nl1 : (partner ? nf : 0);
            // maximal strictly monotonic knot runs [ja, jb) of forward intervals
            int runs[MAXRUNS][3];
            int nrun = 0, cur = 0, ja = 0;
            double Fp = knotF(a->f_phi, a->f_r, m, n, 0);
            for (int j = 0; j <= ni; ++j) {
                int sg = 0;
                double Fn = 0.0;
                if (j < ni) {
                    Fn = knotF(a->f_phi, a->f_r, m, n, j + 1);
                    sg = Fn > Fp ? 1 : (Fn < Fp ? -1 : 0);
                }
                if (sg != cur || j == ni) {
                    if (cur != 0) {
                        if (nrun < MAXRUNS) {
                            runs[nrun][0] = ja; runs[nrun][1] = j; runs[nrun][2] = cur;
                            ++nrun;
                        } else {
                            bad = 1;
                        }
                    }
                    cur = sg;
                    ja = j;
                }
                Fp = Fn;
            }
            Rec* R = P.recs.data() + (size_t)g * ni;
            for (int j = 0; j < ni; ++j) {
                R[j].h = g;
                R[j].j = j;
                R[j].klo[0] = R[j].khi[0] = R[j].klo[1] = R[j].khi[1] = 0;
            }
            for (int r = 0; r < nrun; ++r) {
                const int ra = runs[r][0], rb = runs[r][1], sg = runs[r][2];
                const int npts = rb - ra + 1;
                auto KI = [&](int q) { return sg > 0 ? ra + q : rb - q; };
                spline_nak(npts, [&](int q) { return knotF(a->f_phi, a->f_r, m, n, KI(q)); },
                           [&](int q) { return a->t[KI(q)]; },
                           reinterpret_cast<double(*)[4]>(ti.data()), c1, d1, s1);
                for (int q = 0; q < npts - 1; ++q) {
                    const int jf = sg > 0 ? ra + q : rb - 1 - q;
                    for (int c = 0; c < 4; ++c) R[jf].ic[c] = ti[(size_t)q * 4 + c];
                    R[jf].gx = knotF(a->f_phi, a->f_r, m, n, KI(q));
                }
                const double dm = (double)m, dn = (double)n;
                for (int j = ra; j < rb; ++j) {
                    Rec& it = R[j];
                    it.tj = a->t[j];
                    it.dtj = a->t[j + 1] - a->t[j];
                    for (int c = 0; c < 4; ++c) {
                        const double* ca = P.coefA.data() + ((size_t)j * 4 + c) * 4 * G + 4 * g;
                        it.b[0][0][c] = ca[0]; it.b[0][1][c] = ca[1];
                        it.b[1][0][c] = ca[2]; it.b[1][1][c] = ca[3];
                        const double* ct = P.coefT.data() + ((size_t)j * 4 + c) * 8;
                        it.ph[c] = dm * ct[0] + dn * ct[1];
                    }
                    const double* ct = P.coefT.data() + (size_t)j * 32;
                    const double F0 = dm * ct[2] + dn * ct[3], F1 = dm * ct[10] + dn * ct[11],
                                 F2 = dm * ct[18] + dn * ct[19];
                    it.fd[0] = 3.0 * F0; it.fd[1] = 2.0 * F1; it.fd[2] = F2;
                    const double G0 = dm * ct[4] + dn * ct[5], G1 = dm * ct[12] + dn * ct[13],
                                 G2 = dm * ct[20] + dn * ct[21];
                    it.fdd[0] = FDD_SCALE * (3.0 * G0);
                    it.fdd[1] = FDD_SCALE * (2.0 * G1);
                    it.fdd[2] = FDD_SCALE * G2;
                    // series length from a lower bound of |y| over the interval (k_items)
                    const double dt = it.dtj;
                    auto qv = [](double p0, double p1, double p2, double x) { return (p0 * x + p1) * x + p2; };
                    const double fa = it.fd[2], fb = qv(it.fd[0], it.fd[1], it.fd[2], dt);
                    it.fdneg = qv(it.fd[0], it.fd[1], it.fd[2], 0.5 * dt) < 0.0 ? 1 : 0;
                    double fdmin = std::fmin(std::fabs(fa), std::fabs(fb));
                    if ((fa > 0.0) != (fb > 0.0) || fa == 0.0 || fb == 0.0) fdmin = 0.0;
                    if (it.fd[0] != 0.0) {
                        const double xv = -it.fd[1] / (2.0 * it.fd[0]);
                        if (xv > 0.0 && xv < dt) {
                            const double fv = qv(it.fd[0], it.fd[1], it.fd[2], xv);
                            if ((fv > 0.0) != (fa > 0.0)) fdmin = 0.0;
                            fdmin = std::fmin(fdmin, std::fabs(fv));
                        }
                    }
                    double gmax = std::fmax(std::fabs(G2), std::fabs(qv(3.0 * G0, 2.0 * G1, G2, dt)));
                    if (G0 != 0.0) {
                        const double xv = -(2.0 * G1) / (6.0 * G0);
                        if (xv > 0.0 && xv < dt) gmax = std::fmax(gmax, std::fabs(qv(3.0 * G0, 2.0 * G1, G2, xv)));
                    }
                    const double ymin = gmax > 0.0 ? TWO_PI * fdmin * fdmin * fdmin / (3.0 * gmax * gmax) / 1.1
                                                   : INFINITY;
                    int J = FAST_J;
                    for (int jj = 1; jj < FAST_J; ++jj)
                        if (ymin >= JSER_Y[jj]) { J = jj; break; }
                    it.jser = J;
                    it.envc = 0;
                    if (env_on && ymin >= ENV_MIN_Y) {
                        const double gq[3] = {3.0 * G0, 2.0 * G1, G2};
                        EnvFit E;
                        if (env_fit(it.fd, gq, it.dtj, (it.fdneg & 1) != 0, E)) {
                            it.envc = 1;
                            for (int c = 0; c <= ENV_DEG; ++c) it.env[c] = E.a[c];
                            for (int c = 0; c < 4; ++c) it.phE[c] = it.ph[c] - E.th[c];
                        }
                    }
                    // lane ranges per sub-branch (open at the run's first knot)
                    const double Fj = knotF(a->f_phi, a->f_r, m, n, j);
                    const double Fj1 = knotF(a->f_phi, a->f_r, m, n, j + 1);
                    const double xlo = sg > 0 ? Fj : Fj1, xhi = sg > 0 ? Fj1 : Fj;
                    const bool strict = sg > 0 ? (j == ra) : (j + 1 == rb);
                    auto upper = [&](double v) { return (int64_t)(std::upper_bound(freq, freq + nf, v) - freq); };
                    auto lower = [&](double v) { return (int64_t)(std::lower_bound(freq, freq + nf, v) - freq); };
                    int64_t lo0 = upper(-xhi);
                    int64_t hi0 = strict ? lower(-xlo) : upper(-xlo);
                    int64_t lo1 = strict ? upper(xlo) : lower(xlo);
                    int64_t hi1 = lower(xhi);
                    auto clampr = [](int64_t& lo, int64_t& hi, int64_t lim) {
                        if (lo > lim) lo = lim;
                        if (hi > lim) hi = lim;
                        if (hi < lo) hi = lo;
                    };
                    clampr(lo0, hi0, lim0);
                    clampr(lo1, hi1, lim1);
                    it.klo[0] = (int32_t)lo0; it.khi[0] = (int32_t)hi0;
                    it.klo[1] = (int32_t)lo1; it.khi[1] = (int32_t)hi1;
                    const int mult = paired ? 1 + (partner ? 1 : 0) : 1;
                    const int64_t ev = ((hi0 - lo0) + (hi1 - lo1)) * mult;
                    evals_total += ev;
                    contrib_total += ev * (P.gstart[g + 1] - P.gstart[g]);
                }
            }
        }
    }
    if (bad) return fail(EFD_ERR_ARG, "efd_modesum_cpu: a harmonic has more than 8 monotonic runs");
    P.evaluations = evals_total;
    P.contributions = contrib_total;
    return EFD_OK;
}

// ---- SPA evaluation ------------------------------------------------------------------------
struct SinCosTable {
    double s[512], c[512];
    SinCosTable() {
        for (int i = 0; i < 512; ++i) {
            const long double x = (long double)i * (long double)PI / 256.0L;
            s[i] = (double)sinl(x);
            c[i] = (double)cosl(x);
        }
    }
};
const SinCosTable& sctab() {
    static const SinCosTable t;
    return t;
}

// (R + i I) of the K_{1/3} factor for |y| < FAST_Y (the kernel's kfactor_slow)
void kfactor_slow(double fd, double fdd, double& R, double& I) {
    const double y = TWO_PI * fd * fd * fd / (3.0 * fdd * fdd);
    const double ay = std::fabs(y);
    if (ay * KTAB_WMAX > 1.0) {
        const double ww = 1.0 / ay;
        if (ww < KTAB_WMIN) {
            const double uu = ww * ww;
            double r = KB[FAST_J - 1], im = KC[FAST_J - 1];
            for (int j = FAST_J - 2; j >= 0; --j) {
                r = std::fma(r, uu, KB[j]);
                im = std::fma(im, uu, KC[j]);
            }
            R = r;
            I = ww * im;
        } else {
            uint64_t bits;
            std::memcpy(&bits, &ww, 8);
            const uint32_t hi = (uint32_t)(bits >> 32);
            const int k = (int)((hi >> 18) & 3u);
            const int id = std::min(std::max(4 * ((int)(hi >> 20) - 1023 - KTAB_E_LO) + k, 0), KTAB_N - 1);
            const uint64_t mb = (bits & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull;
            double mm;
            std::memcpy(&mm, &mb, 8);
            const double x = std::fma(8.0, mm, -(double)(9 + 2 * k));
            double r = 0.0, im = 0.0;
            for (int d = KTAB_DEG; d >= 0; --d) {
                r = std::fma(r, x, KTAB[id][d].x);
                im = std::fma(im, x, KTAB[id][d].y);
            }
            R = r;
            I = im;
        }
        if (y < 0.0) I = -I;
        return;
    }
    const double sgn = y > 0 ? 1.0 : -1.0;
    const double q = -0.25 * y * y;
    const int deg = ASC_DEG[std::min(18, (int)ay)];
    double sp = ASC_P[deg], sm = ASC_M[deg];
    for (int k = deg - 1; k >= 0; --k) {
        sp = std::fma(sp, q, ASC_P[k]);
        sm = std::fma(sm, q, ASC_M[k]);
    }
    const double zp = std::cbrt(0.5 * ay), zm = 1.0 / zp;
    constexpr double c6 = 0.86602540378443864676, s6 = 0.5;
    const double ipr = zp * c6 * sp, ipi = -sgn * zp * s6 * sp;
    const double imr = zm * c6 * sm, imi = sgn * zm * s6 * sm;
    constexpr double pref = PI / (2.0 * 0.86602540378443864676);
    const double Kr = pref * (imr - ipr), Ki = pref * (imi - ipi);
    const double sy = std::sin(y), cy = std::cos(y);
    const double kr = Kr * cy + Ki * sy, ki = Ki * cy - Kr * sy;
    const double f = 1.15470053837925152902 * fd / std::fabs(fdd);
    const double qr = -f * ki, qi = f * kr;
    const double am = 1.0 / std::sqrt(std::fabs(fd));
    constexpr double c34 = -0.70710678118654752440;
    const double spr = am * c34, spi = (fd > 0 ? am : -am) * 0.70710678118654752440;
    const double afd = std::fabs(fd);
    R = (qr * spr + qi * spi) * afd;
    I = (qi * spr - qr * spi) * afd;
}

// general path at frequency g of record it (sub-branch s): W and the own / mirror amplitudes
void spa_general(const Rec& it, double g, int s, const Prep& P, const double* t, int caustic,
                 double& wr, double& wi, double xo[2], double zo[2]) {
    const double u = g - it.gx;
    const double tt = cubic(it.ic, u);
    const double wl = tt - it.tj;
    double ph, fd, fdd, b[4];
    const int nt = P.nt, G = P.G;
    if (wl >= 0.0 && wl < it.dtj) {
        for (int q = 0; q < 4; ++q) b[q] = cubic(it.b[q >> 1][q & 1], wl);
        ph = cubic(it.ph, wl);
        fd = std::fma(std::fma(it.fd[0], wl, it.fd[1]), wl, it.fd[2]);
        fdd = INV_FDD_SCALE * std::fma(std::fma(it.fdd[0], wl, it.fdd[1]), wl, it.fdd[2]);
    } else {   // t(g) overshot the record's interval: scipy's interval choice, clamped
        int j = it.j;
        while (j > 0 && tt < t[j]) --j;
        while (j < nt - 2 && tt >= t[j + 1]) ++j;
        const double w = tt - t[j];
        const double* ca = P.coefA.data() + (size_t)j * 4 * 4 * G + 4 * it.h;
        for (int q = 0; q < 4; ++q)
            b[q] = std::fma(std::fma(std::fma(ca[q], w, ca[4 * G + q]), w, ca[8 * G + q]), w, ca[12 * G + q]);
        const double* ct = P.coefT.data() + (size_t)j * 32;
        const double dm = (double)P.gm[it.h], dn = (double)P.gn[it.h];
        const double pc[4] = {dm * ct[0] + dn * ct[1], dm * ct[8] + dn * ct[9],
                              dm * ct[16] + dn * ct[17], dm * ct[24] + dn * ct[25]};
        ph = cubic(pc, w);
        fd = std::fma(std::fma(3.0 * (dm * ct[2] + dn * ct[3]), w, 2.0 * (dm * ct[10] + dn * ct[11])), w,
                      dm * ct[18] + dn * ct[19]);
        fdd = std::fma(std::fma(3.0 * (dm * ct[4] + dn * ct[5]), w, 2.0 * (dm * ct[12] + dn * ct[13])), w,
                       dm * ct[20] + dn * ct[21]);
    }
    // own bin: b[s], mirror: b[1 - s] (Bp = b[0..1], Bm = b[2..3])
    xo[0] = b[2 * s]; xo[1] = b[2 * s + 1];
    zo[0] = b[2 - 2 * s]; zo[1] = b[3 - 2 * s];
    const double amp = fd != 0.0 ? 1.0 / std::sqrt(std::fabs(fd)) : 0.0;
    const double psi = std::fma(TWO_PI * g, tt, -ph) + (fd > 0.0 ? 0.75 * PI : -0.75 * PI);
    double R = 1.0, I = 0.0;
    if (caustic == EFD_CAUSTIC_UNIFORM && fd != 0.0 && fdd != 0.0) {
        const double a2 = amp * amp;
        const double ww = (fd > 0.0 ? 1.0 : -1.0) * (3.0 / TWO_PI) * fdd * fdd * a2 * a2 * a2;
        if (std::fabs(ww) * FAST_Y <= 1.0) {
            const double uu = ww * ww;
            double r = KB[FAST_J - 1], im = KC[FAST_J - 1];
            for (int j = FAST_J - 2; j >= 0; --j) {
                r = std::fma(r, uu, KB[j]);
                im = std::fma(im, uu, KC[j]);
            }
            R = r;
            I = ww * im;
        } else {
            kfactor_slow(fd, fdd, R, I);
        }
    }
    const double sn = std::sin(psi), cs = std::cos(psi);
    wr = amp * (R * cs - I * sn);
    wi = amp * (R * sn + I * cs);
}

// One record's fast-path evaluations over lanes [lo, hi) of a tile (lane i at index i - tlo):
// W (wr, wi), w and the general-path flag, branch-free and vectorised over the lanes.
template <int CAUSTIC, bool J34>
void spa_fast(const Rec& it, int s, const double* fk, int n, double* wr, double* wi, double* wv,
              unsigned char* need) {
    const SinCosTable& T = sctab();
    const double sgn = s ? 1.0 : -1.0;   // g = -f (s = 0) or +f (s = 1)
    const bool neg = it.fdneg != 0;
    const int shift = neg ? -192 : 192;
    const double kth = neg ? -KTH0 / VS : KTH0 / VS;
    constexpr double INV_STEP = 81.48733086305042;
    constexpr double STEP_1 = 0.01227184630308513;
    constexpr double SHIFTER = 6755399441055744.0;
#pragma omp simd
    for (int i = 0; i < n; ++i) {
        const double g = sgn * fk[i];
        const double u = g - it.gx;
        const double tt = std::fma(std::fma(std::fma(it.ic[0], u, it.ic[1]), u, it.ic[2]), u, it.ic[3]);
        const double w = tt - it.tj;
        bool good = (w >= 0.0) & (w < it.dtj);
        const double ph = std::fma(std::fma(std::fma(it.ph[0], w, it.ph[1]), w, it.ph[2]), w, it.ph[3]);
        const double fd = std::fma(std::fma(it.fd[0], w, it.fd[1]), w, it.fd[2]);
        good = good & (neg ? (fd < 0.0) & (fd > -INFINITY) : (fd > 0.0) & (fd < INFINITY));
        const double ampm = good ? 1.0 / std::sqrt(std::fabs(fd)) : 0.0;
        const double psi0 = std::fma(TWO_PI * g, tt, -ph);
        double am = ampm, c0 = COS_A, thn = 0.0, ksc = 0.0;
        if (CAUSTIC == EFD_CAUSTIC_UNIFORM) {
            const double fdds = std::fma(std::fma(it.fdd[0], w, it.fdd[1]), w, it.fdd[2]);
            const double a3 = ampm * ampm * ampm;
            const double t3 = fdds * a3;
            double ww = t3 * t3;   // v = VS / |y|
            if (J34) {
                const bool inr = ww <= VS / FAST_Y;
                good = good & inr;
                ww = inr ? ww : 0.0;
                const double uu = ww * ww;
                const double r = std::fma(45.7, uu * uu, 1.0 - uu);
                thn = ww * std::fma(-14.733333333333333333, uu, 1.0);
                am = good ? ampm * r : 0.0;
            } else {
                c0 = std::fma(-ww, ww, COS_A);
                thn = ww;
            }
            ksc = kth;
        }
        // sin/cos: reduction by pi/256 against the table, short polynomials, angle sum
        const double qs = std::fma(psi0, INV_STEP, SHIFTER);
        const double q = qs - SHIFTER;
        double r = std::fma(-q, STEP_1, psi0);
        r = std::fma(ksc, thn, r);
        const int64_t qi = (int64_t)q;
        const int off = (int)((qi + shift) & 511);
        const double ts = T.s[off], tc = T.c[off];
        const double z = r * r;
        const double sr = std::fma(r * z, -1.6666666666666666e-01, r);
        const double cr = std::fma(z, COS_B, c0);
        const double sn = std::fma(ts, cr, tc * sr);
        const double cs = std::fma(tc, cr, -ts * sr);
        wr[i] = am * cs;
        wi[i] = am * sn;
        wv[i] = w;
        need[i] = !good;
    }
}

// An envelope record's evaluations (k_modesum's spa_env): phase with theta folded into the phase
// cubic, A(w) from its polynomial, no F' / F'' / K_{1/3} arithmetic. Lanes outside the knot
// interval take the general path (the kernel certifies its envelope records have none).
void spa_fast_env(const Rec& it, int s, const double* fk, int n, double* wr, double* wi,
                  double* wv, unsigned char* need) {
    const SinCosTable& T = sctab();
    const double sgn = s ? 1.0 : -1.0;
    const int shift = (it.fdneg & 1) ? -192 : 192;
    constexpr double INV_STEP = 81.48733086305042;
    constexpr double STEP_1 = 0.01227184630308513;
    constexpr double SHIFTER = 6755399441055744.0;
#pragma omp simd
    for (int i = 0; i < n; ++i) {
        const double g = sgn * fk[i];
        const double u = g - it.gx;
        const double tt = std::fma(std::fma(std::fma(it.ic[0], u, it.ic[1]), u, it.ic[2]), u, it.ic[3]);
        const double w = tt - it.tj;
        const bool good = (w >= 0.0) & (w < it.dtj);
        const double ph = std::fma(std::fma(std::fma(it.phE[0], w, it.phE[1]), w, it.phE[2]), w, it.phE[3]);
        const double psi0 = std::fma(TWO_PI * g, tt, -ph);
        double A = it.env[0];
        for (int c = 1; c <= ENV_DEG; ++c) A = std::fma(A, w, it.env[c]);
        const double am = good ? A : 0.0;
        const double qs = std::fma(psi0, INV_STEP, SHIFTER);
        const double q = qs - SHIFTER;
        const double r = std::fma(-q, STEP_1, psi0);
        const int64_t qi = (int64_t)q;
        const int off = (int)((qi + shift) & 511);
        const double ts = T.s[off], tc = T.c[off];
        const double z = r * r;
        const double sr = std::fma(r * z, -1.6666666666666666e-01, r);
        const double cr = std::fma(z, COS_B, COS_A);
        const double sn = std::fma(ts, cr, tc * sr);
        const double cs = std::fma(tc, cr, -ts * sr);
        wr[i] = am * cs;
        wi[i] = am * sn;
        wv[i] = w;
        need[i] = !good;
    }
}

struct TileLists {
    std::vector<int64_t> off;    // [ntiles + 1]
    std::vector<uint32_t> ent;   // (record << 1) | s
};

void build_tile_lists(const Prep& P, int64_t ntiles, TileLists& L) {
    const size_t nrec = P.recs.size();
    std::vector<int64_t> cnt(ntiles + 1, 0);
    for (size_t r = 0; r < nrec; ++r)
        for (int s = 0; s < 2; ++s) {
            const Rec& it = P.recs[r];
            if (it.khi[s] <= it.klo[s]) continue;
            for (int64_t t = it.klo[s] / TL; t <= (it.khi[s] - 1) / TL; ++t) ++cnt[t];
        }
    L.off.assign(ntiles + 1, 0);
    for (int64_t t = 0; t < ntiles; ++t) L.off[t + 1] = L.off[t] + cnt[t];
    L.ent.resize(L.off[ntiles]);
    std::vector<int64_t> pos(L.off.begin(), L.off.end() - 1);
    for (size_t r = 0; r < nrec; ++r)
        for (int s = 0; s < 2; ++s) {
            const Rec& it = P.recs[r];
            if (it.khi[s] <= it.klo[s]) continue;
            for (int64_t t = it.klo[s] / TL; t <= (it.khi[s] - 1) / TL; ++t)
                L.ent[pos[t]++] = (uint32_t)((r << 1) | (size_t)s);
        }
}

int modesum(const efd_modesum_args* a) {
    if (!a) return fail(EFD_ERR_ARG, "efd_modesum_cpu: NULL argument");
    if (!a->t || !a->phi_phi || !a->phi_r || !a->f_phi || !a->f_r || !a->amp || !a->m || !a->n ||
        !a->ylm_p || !a->ylm_m || !a->freq)
        return fail(EFD_ERR_ARG, "efd_modesum_cpu: NULL array");
    const bool pol = a->hp != nullptr || a->hc != nullptr;
    if (pol && (!a->hp || !a->hc || !a->grid_symmetric || a->k0 < 0 || a->k0 > a->nf))
        return fail(EFD_ERR_ARG, "efd_modesum_cpu: hp/hc need both pointers, a symmetric grid and 0 <= k0 <= nf");
    if (!a->out && !pol) return fail(EFD_ERR_ARG, "efd_modesum_cpu: no output (out or hp/hc)");
    if (a->nt < 2 || a->nt > MAX_NT) return fail(EFD_ERR_ARG, "efd_modesum_cpu: nt out of range");
    if (a->K <= 0 || a->K > MAX_K) return fail(EFD_ERR_ARG, "efd_modesum_cpu: K out of range [1, 8192]");
    if (a->nf <= 0 || a->nf >= (int64_t)INT32_MAX) return fail(EFD_ERR_ARG, "efd_modesum_cpu: nf out of range");
    if (a->caustic != EFD_CAUSTIC_SPA && a->caustic != EFD_CAUSTIC_UNIFORM)
        return fail(EFD_ERR_ARG, "efd_modesum_cpu: unknown caustic mode");
    for (int i = 1; i < a->nt; ++i)
        if (!(a->t[i] > a->t[i - 1])) return fail(EFD_ERR_ARG, "efd_modesum_cpu: t not increasing");
    const bool paired = a->grid_symmetric != 0;
    const int64_t nf = a->nf;
    const int64_t nl = paired ? (nf + 1) / 2 : nf;
    const int64_t nl1 = paired ? ((nf % 2) ? nl - 1 : nl) : nf;
    Prep P;
    const int rc = prepare(a, P, paired, nl, nl1);
    if (rc != EFD_OK) return rc;
    g_stats[0] = P.contributions;
    g_stats[1] = P.evaluations;
    g_stats[2] = P.G;
    const int64_t ntiles = (nl + TL - 1) / TL;
    TileLists L;
    build_tile_lists(P, ntiles, L);
    const double* freq = a->freq;
    const int caustic = a->caustic;
    const bool acc = a->accumulate != 0;
    const int64_t k0 = a->k0;
#pragma omp parallel num_threads(nthreads())
    {
        alignas(64) double fk[TL], own_r[TL], own_i[TL], mir_r[TL], mir_i[TL];
        alignas(64) double wr[TL], wi[TL], wv[TL];
        alignas(64) unsigned char need[TL];
#pragma omp for schedule(dynamic, 1)
        for (int64_t tile = 0; tile < ntiles; ++tile) {
            const int64_t tlo = tile * TL;
            const int nln = (int)std::min<int64_t>(TL, nl - tlo);
            for (int i = 0; i < nln; ++i) fk[i] = freq[tlo + i];
            std::fill(own_r, own_r + TL, 0.0);
            std::fill(own_i, own_i + TL, 0.0);
            std::fill(mir_r, mir_r + TL, 0.0);
            std::fill(mir_i, mir_i + TL, 0.0);
            for (int64_t e = L.off[tile]; e < L.off[tile + 1]; ++e) {
                const uint32_t key = L.ent[e];
                const Rec& it = P.recs[key >> 1];
                const int s = (int)(key & 1u);
                const int lo = (int)std::max<int64_t>(it.klo[s] - tlo, 0);
                const int hi = (int)std::min<int64_t>(it.khi[s] - tlo, nln);
                if (hi <= lo) continue;
                const int n = hi - lo;
                if (caustic == EFD_CAUSTIC_UNIFORM) {
                    if (it.envc) spa_fast_env(it, s, fk + lo, n, wr, wi, wv, need);
                    else if (it.jser >= 3) spa_fast<EFD_CAUSTIC_UNIFORM, true>(it, s, fk + lo, n, wr, wi, wv, need);
                    else spa_fast<EFD_CAUSTIC_UNIFORM, false>(it, s, fk + lo, n, wr, wi, wv, need);
                } else {
                    spa_fast<EFD_CAUSTIC_SPA, false>(it, s, fk + lo, n, wr, wi, wv, need);
                }
                // own bin: X = b[s]; mirror: Z = b[1 - s]. s = 0: own += X W, mirror += conj(Z W);
                // s = 1: own += conj(X W), mirror += Z W
                const double* X = &it.b[s][0][0];
                const double* Z = &it.b[1 - s][0][0];
                const double so = s ? -1.0 : 1.0;
#pragma omp simd
                for (int i = 0; i < n; ++i) {
                    const double w = wv[i];
                    const double xr = cubic(X, w), xi = cubic(X + 4, w);
                    const double zr = cubic(Z, w), zi = cubic(Z + 4, w);
                    const int k = lo + i;
                    own_r[k] = std::fma(-xi, wi[i], std::fma(xr, wr[i], own_r[k]));
                    own_i[k] = std::fma(so * xi, wr[i], std::fma(so * xr, wi[i], own_i[k]));
                    mir_r[k] = std::fma(-zi, wi[i], std::fma(zr, wr[i], mir_r[k]));
                    mir_i[k] = std::fma(-so * zi, wr[i], std::fma(-so * zr, wi[i], mir_i[k]));
                }
                for (int i = 0; i < n; ++i) {
                    if (!need[i]) continue;
                    const int k = lo + i;
                    const double g = s ? fk[k] : -fk[k];
                    double cr, ci, xo[2], zo[2];
                    spa_general(it, g, s, P, a->t, caustic, cr, ci, xo, zo);
                    own_r[k] = std::fma(-xo[1], ci, std::fma(xo[0], cr, own_r[k]));
                    own_i[k] = std::fma(so * xo[1], cr, std::fma(so * xo[0], ci, own_i[k]));
                    mir_r[k] = std::fma(-zo[1], ci, std::fma(zo[0], cr, mir_r[k]));
                    mir_i[k] = std::fma(-so * zo[1], cr, std::fma(-so * zo[0], ci, mir_i[k]));
                }
            }
            // outputs: the lane's bin k and, on symmetric grids, its mirror nf - 1 - k
            for (int i = 0; i < nln; ++i) {
                const int64_t k = tlo + i;
                const int64_t km = paired ? nf - 1 - k : k;
                double skr = own_r[i], ski = own_i[i];
                double smr = mir_r[i], smi = mir_i[i];
                if (paired && km == k) {
                    skr += smr; ski += smi;
                    smr = skr; smi = ski;
                }
                if (!paired) { smr = 0.0; smi = 0.0; }
                if (a->out) {
                    double* o = a->out;
                    if (paired && km != k) {
                        o[2 * km] = (acc ? o[2 * km] : 0.0) + smr;
                        o[2 * km + 1] = (acc ? o[2 * km + 1] : 0.0) + smi;
                    }
                    o[2 * k] = (acc ? o[2 * k] : 0.0) + skr;
                    o[2 * k + 1] = (acc ? o[2 * k + 1] : 0.0) + ski;
                }
                if (paired && a->hp) {
                    auto put = [&](int64_t j, double ar, double ai, double br, double bi) {
                        if (j < k0) return;
                        double* hp = a->hp + 2 * (j - k0);
                        double* hc = a->hc + 2 * (j - k0);
                        const double pr = 0.5 * (ar + br), pi = 0.5 * (ai - bi);
                        const double cr = -0.5 * (ai + bi), ci = 0.5 * (ar - br);
                        hp[0] = (acc ? hp[0] : 0.0) + pr;
                        hp[1] = (acc ? hp[1] : 0.0) + pi;
                        hc[0] = (acc ? hc[0] : 0.0) + cr;
                        hc[1] = (acc ? hc[1] : 0.0) + ci;
                    };
                    put(km, smr, smi, skr, ski);
                    if (km != k) put(k, skr, ski, smr, smi);
                }
            }
        }
    }
    return EFD_OK;
}

}  // namespace efdcpu

// ========================================================================================
// C ABI (host pointers; `stream` and workspaces are accepted for signature parity and unused)
// ========================================================================================
extern "C" {

int efd_cpu_threads(int n) {
    const int prev = efdcpu::g_threads;
    efdcpu::g_threads = n > 0 ? n : 0;
    return prev;
}

int efd_cpu_last_error(char* buf, int len) {
    if (!buf || len <= 0) return EFD_ERR_ARG;
    std::snprintf(buf, (size_t)len, "%s", efdcpu::g_err.c_str());
    return EFD_OK;
}

int efd_modesum_cpu(const efd_modesum_args* a, void* workspace, size_t workspace_bytes,
                    void* stream) {
    (void)workspace; (void)workspace_bytes; (void)stream;
    return efdcpu::modesum(a);
}

int efd_modesum_cpu_stats(int64_t* contributions, int64_t* evaluations, int32_t* groups) {
    if (contributions) *contributions = efdcpu::g_stats[0];
    if (evaluations) *evaluations = efdcpu::g_stats[1];
    if (groups) *groups = (int32_t)efdcpu::g_stats[2];
    return EFD_OK;
}

int efd_spline_build_cpu(const double* x, int n, const double* y, int ninterp, double* coef,
                         void* stream) {
    (void)stream;
    if (!x || !y || !coef || n < 2 || ninterp <= 0 || n > efdcpu::MAX_NT)
        return efdcpu::fail(EFD_ERR_ARG, "efd_spline_build_cpu: bad arguments");
    for (int i = 1; i < n; ++i)
        if (!(x[i] > x[i - 1])) return efdcpu::fail(EFD_ERR_ARG, "efd_spline_build_cpu: x not increasing");
#pragma omp parallel num_threads(efdcpu::nthreads())
    {
        std::vector<double> cp, dp, s, tq((size_t)(n - 1) * 4);
#pragma omp for schedule(static)
        for (int q = 0; q < ninterp; ++q) {
            efdcpu::spline_nak(n, [&](int i) { return x[i]; },
                               [&](int i) { return y[(size_t)i * ninterp + q]; },
                               reinterpret_cast<double(*)[4]>(tq.data()), cp, dp, s);
            for (int i = 0; i < n - 1; ++i)
                for (int c = 0; c < 4; ++c) coef[((size_t)i * 4 + c) * ninterp + q] = tq[(size_t)i * 4 + c];
        }
    }
    return EFD_OK;
}

int efd_polarizations_cpu(const double* S, int64_t nf, int64_t k0, double* hp, double* hc,
                          void* stream) {
    (void)stream;
    if (!S || !hp || !hc || nf <= 0 || k0 < 0 || k0 > nf)
        return efdcpu::fail(EFD_ERR_ARG, "efd_polarizations_cpu: bad arguments");
#pragma omp parallel for schedule(static) num_threads(efdcpu::nthreads())
    for (int64_t k = k0; k < nf; ++k) {
        const double ar = S[2 * k], ai = S[2 * k + 1];
        const double br = S[2 * (nf - 1 - k)], bi = S[2 * (nf - 1 - k) + 1];
        const int64_t i = k - k0;
        hp[2 * i] = 0.5 * (ar + br); hp[2 * i + 1] = 0.5 * (ai - bi);
        hc[2 * i] = -0.5 * (ai + bi); hc[2 * i + 1] = 0.5 * (ar - br);
    }
    return EFD_OK;
}

int efd_loglike_cpu(const double* h, const double* d, const double* w, int32_t nchan,
                    int64_t nbin, double* out, double* scratch, void* stream) {
    (void)scratch; (void)stream;
    if (!d || !w || !out || nchan <= 0 || nbin <= 0)
        return efdcpu::fail(EFD_ERR_ARG, "efd_loglike_cpu: bad arguments");
    const int64_t total = (int64_t)nchan * nbin;
    double acc = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : acc) num_threads(efdcpu::nthreads())
    for (int64_t i = 0; i < total; ++i) {
        double rr = d[2 * i], ri = d[2 * i + 1];
        if (h) {
            const double p = h[2 * i] * w[i], q = h[2 * i + 1] * w[i];
            rr -= p;
            ri -= q;
        }
        acc += rr * rr + ri * ri;
    }
    *out = -0.5 * 4.0 * acc;
    return EFD_OK;
}

int efd_inner_product_cpu(const double* a, const double* b, const double* w, int32_t nchan,
                          int64_t nbin, double* out, double* scratch, void* stream) {
    (void)scratch; (void)stream;
    if (!a || !b || !out || nchan <= 0 || nbin <= 0)
        return efdcpu::fail(EFD_ERR_ARG, "efd_inner_product_cpu: bad arguments");
    const int64_t total = (int64_t)nchan * nbin;
    double re = 0.0, im = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : re, im) num_threads(efdcpu::nthreads())
    for (int64_t i = 0; i < total; ++i) {
        const double ww = w ? w[i] : 1.0;
        re += ww * (a[2 * i] * b[2 * i] + a[2 * i + 1] * b[2 * i + 1]);
        im += ww * (a[2 * i] * b[2 * i + 1] - a[2 * i + 1] * b[2 * i]);
    }
    out[0] = 4.0 * re;
    out[1] = 4.0 * im;
    return EFD_OK;
}

}  // extern "C"
