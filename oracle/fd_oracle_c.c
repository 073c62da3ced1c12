/*
 * fd_oracle_c.c -- C restatement of oracle/fd_oracle.py (the reference notebook's FD_waveform,
 * Tutorial_FD_construction_single_mode.ipynb:552-623, summed over harmonics).
 *
 * TEST INFRASTRUCTURE ONLY: tests/ check it against the numpy oracle, and bench.py times it as
 * the CPU baseline ("kind": "port"). The product (libemrifd.so) never links or calls it.
 *
 * Per harmonic (m, n), exactly as the numpy oracle:
 *   F_i = m f_phi_i + n f_r_i                                      notebook :564
 *   Phi(t) = not-a-knot spline of m Phi_phi + n Phi_r               :558-559
 *   A(t) = splines of Re/Im A                                       :587-594
 *   F'(t) = derivative of spline(F); F''(t) = derivative of spline(F'(t_i))   :579-584
 *   per maximal strictly monotonic run of F: t(g) = spline(F_run -> t_run)     :566
 *   parent (+F) at mirror-grid g in (min F, max F), partner (-F) at g in (-max F, -min F)
 *                                                                   :569-572, :607-616
 *   Q = i F'/|F''| K_{1/3}(z) e^z 2/sqrt(3), z = -2 pi i F'^3/(3 F''^2)  ("uniform", :599-608)
 *     or e^{i sgn(F') 3pi/4}/sqrt|F'| ("spa", the leading asymptote)
 *   S(f) = -h_nb(-f) * scale   (FEW's FFT convention)
 * Splines follow scipy.interpolate.CubicSpline (not-a-knot; n = 2 line, n = 3 parabola) and
 * scipy's interval search (x_i <= x < x_{i+1}, clamped at the ends). K_{1/3} of imaginary
 * argument: Hankel asymptotic series for |y| >= 18.4, ascending series below (summed in
 * __float128 above |y| = 5; scipy uses AMOS; agreement ~1e-11 relative, checked in
 * tests/test_oracle_c.py).
 */
#include <complex.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define PI_D 3.14159265358979323846264338327950288
#define TWO_PI_D 6.28318530717958647692528676655900577

/* not-a-knot spline on x[0..n-1] of y (stride ys); coef[4*(n-1)] in PPoly order */
static void spline(const double* x, int n, const double* y, int ys, double* coef, double* cp,
                   double* dp, double* s) {
    if (n == 2) {
        double sl = (y[ys] - y[0]) / (x[1] - x[0]);
        coef[0] = 0.0; coef[1] = 0.0; coef[2] = sl; coef[3] = y[0];
        return;
    }
    if (n == 3) {
        double dx0 = x[1] - x[0], dx1 = x[2] - x[1];
        double sl0 = (y[ys] - y[0]) / dx0, sl1 = (y[2 * ys] - y[ys]) / dx1;
        s[1] = (dx0 * sl1 + dx1 * sl0) / (dx0 + dx1);
        s[0] = 2.0 * sl0 - s[1];
        s[2] = 2.0 * sl1 - s[1];
    } else {
        /* rows as scipy/_cubic.py: row 0 and n-1 not-a-knot, Thomas elimination */
        double dx0 = x[1] - x[0], dx1 = x[2] - x[1];
        double sl0 = (y[ys] - y[0]) / dx0, sl1 = (y[2 * ys] - y[ys]) / dx1;
        double d = x[2] - x[0];
        cp[0] = d / dx1;
        dp[0] = (((dx0 + 2.0 * d) * dx1 * sl0 + dx0 * dx0 * sl1) / d) / dx1;
        for (int i = 1; i <= n - 2; ++i) {
            double dxm = x[i] - x[i - 1], dxi = x[i + 1] - x[i];
            double slm = (y[i * ys] - y[(i - 1) * ys]) / dxm;
            double sli = (y[(i + 1) * ys] - y[i * ys]) / dxi;
            double a = dxi, b = 2.0 * (dxm + dxi), c = dxm, r = 3.0 * (dxi * slm + dxm * sli);
            double mm = b - a * cp[i - 1];
            cp[i] = c / mm;
            dp[i] = (r - a * dp[i - 1]) / mm;
        }
        double dxm = x[n - 2] - x[n - 3], dxi = x[n - 1] - x[n - 2];
        double slm = (y[(n - 2) * ys] - y[(n - 3) * ys]) / dxm;
        double sli = (y[(n - 1) * ys] - y[(n - 2) * ys]) / dxi;
        double dd = x[n - 1] - x[n - 3];
        double a = dd, b = dxm, r = (dxi * dxi * slm + (2.0 * dd + dxi) * dxm * sli) / dd;
        s[n - 1] = (r - a * dp[n - 2]) / (b - a * cp[n - 2]);
        for (int i = n - 2; i >= 0; --i) s[i] = dp[i] - cp[i] * s[i + 1];
    }
    for (int i = 0; i < n - 1; ++i) {
        double dx = x[i + 1] - x[i];
        double sl = (y[(i + 1) * ys] - y[i * ys]) / dx;
        double tt = (s[i] + s[i + 1] - 2.0 * sl) / dx;
        coef[4 * i + 0] = tt / dx;
        coef[4 * i + 1] = (sl - s[i]) / dx - tt;
        coef[4 * i + 2] = s[i];
        coef[4 * i + 3] = y[i * ys];
    }
}

/* scipy find_interval: x_i <= v < x_{i+1}, clamped to [0, n-2] */
static int find_interval(const double* x, int n, double v) {
    if (v >= x[n - 1]) return n - 2;
    if (v <= x[0]) return 0;
    int lo = 0, hi = n - 1;
    while (hi - lo > 1) {
        int mid = (lo + hi) >> 1;
        if (x[mid] <= v) lo = mid; else hi = mid;
    }
    return lo;
}

static inline double cubic(const double* c, double w) { return ((c[0] * w + c[1]) * w + c[2]) * w + c[3]; }
static inline double dcubic(const double* c, double w) { return (3.0 * c[0] * w + 2.0 * c[1]) * w + c[2]; }

/* K_{1/3}(z) e^z for z = -i y */
static double complex kv13_scaled(double y) {
    double ay = fabs(y);
    if (ay >= 18.4) {
        double complex z = -I * y, zi = 1.0 / z, term = 1.0, sum = 1.0;
        double mu = 4.0 / 9.0;
        int N = 40;
        if (ay >= 555.0) N = 6; else if (ay >= 153.0) N = 8; else if (ay >= 75.0) N = 10;
        else if (ay >= 48.0) N = 12; else if (ay >= 29.4) N = 16; else if (ay >= 23.1) N = 20;
        else if (ay >= 20.3) N = 24; else if (ay >= 19.0) N = 28;
        for (int k = 1; k < N; ++k) {
            term *= (mu - (2.0 * k - 1.0) * (2.0 * k - 1.0)) / (8.0 * k) * zi;
            sum += term;
        }
        return csqrt(PI_D / (2.0 * z)) * sum;
    }
    /* The alternating sums cancel: terms reach ~e^|y| / sqrt|y| times the result, so in double
     * the series loses up to 7 digits by |y| = 18 (1e-9 relative error against scipy's AMOS kv,
     * which the notebook calls). Above |y| = 5 they are summed in __float128 and keep ~1e-16
     * (checked against mpmath over 0 < |y| < 18.4; double is good to 7e-16 below 5). */
    double nu = 1.0 / 3.0;
    double spd, smd;
    if (ay < 5.0) {
        double q = -0.25 * y * y;
        double tp = 1.0 / 0.89297951156924921122, tm = 1.0 / 1.35411793942640041695;
        double sp = tp, sm = tm;
        for (int k = 1; k < 200; ++k) {
            tp *= q / (k * (k + nu));
            tm *= q / (k * (k - nu));
            sp += tp;
            sm += tm;
            if (fabs(tp) < 1e-18 * fabs(sp) && fabs(tm) < 1e-18 * fabs(sm)) break;
        }
        spd = sp;
        smd = sm;
    } else {
        __float128 q = -0.25Q * (__float128)y * (__float128)y, nuq = 1.0Q / 3.0Q;
        __float128 tp = 1.0Q / 0.89297951156924921122Q, tm = 1.0Q / 1.35411793942640041695Q;
        __float128 sp = tp, sm = tm;
        for (int k = 1; k < 200; ++k) {
            tp *= q / (k * (k + nuq));
            tm *= q / (k * (k - nuq));
            sp += tp;
            sm += tm;
            if ((tp < 0 ? -tp : tp) < 1e-30Q * (sp < 0 ? -sp : sp) &&
                (tm < 0 ? -tm : tm) < 1e-30Q * (sm < 0 ? -sm : sm))
                break;
        }
        spd = (double)sp;
        smd = (double)sm;
    }
    double complex zh = -I * y / 2.0;
    double complex ip = cpow(zh, nu) * spd, im = cpow(zh, -nu) * smd;
    double complex K = PI_D / (2.0 * sin(PI_D * nu)) * (im - ip);
    return K * cexp(-I * y);
}

static double complex qfactor(double fd, double fdd, int caustic) {
    if (fd == 0.0) return 0.0;
    if (caustic == 0 || fdd == 0.0)
        return cexp(I * (fd > 0 ? 0.75 * PI_D : -0.75 * PI_D)) / sqrt(fabs(fd));
    double y = TWO_PI_D * fd * fd * fd / (3.0 * fdd * fdd);
    return I * fd / fabs(fdd) * kv13_scaled(y) * (2.0 / sqrt(3.0));
}

static int64_t lower_bound(const double* f, int64_t nf, double v) {
    int64_t lo = 0, hi = nf;
    while (lo < hi) { int64_t mid = (lo + hi) >> 1; if (f[mid] < v) lo = mid + 1; else hi = mid; }
    return lo;
}
static int64_t upper_bound(const double* f, int64_t nf, double v) {
    int64_t lo = 0, hi = nf;
    while (lo < hi) { int64_t mid = (lo + hi) >> 1; if (f[mid] <= v) lo = mid + 1; else hi = mid; }
    return lo;
}

/* amp: complex [K][nt] interleaved; ylm_p, ylm_m: complex [K]; out: complex [nf] (written).
 * extrap (optional, real [nf]): per bin, the summed magnitude |term| of the contributions whose
 * t(g) lies outside the trajectory [t_0, t_{nt-1}], where scipy's splines extrapolate (the
 * inverse spline of a nearly flat monotonic run can overshoot the run's times by far). Those
 * terms are part of the construction (CubicSpline extrapolates by default), but their phase
 * comes from cubics evaluated far outside their interval and is numerically undetermined: two
 * faithful evaluations of it agree in magnitude only. The parity tests bound such bins by it. */
int fdo_modesum_ex(const double* t, int nt, const double* amp, const double* phi_phi,
                   const double* phi_r, const double* f_phi, const double* f_r, const int* marr,
                   const int* narr, const double* ylm_p, const double* ylm_m, int K,
                   const double* freq, int64_t nf, double scale_re, double scale_im, int caustic,
                   int nthreads, double* out, double* extrap);
int fdo_modesum(const double* t, int nt, const double* amp, const double* phi_phi,
                const double* phi_r, const double* f_phi, const double* f_r, const int* marr,
                const int* narr, const double* ylm_p, const double* ylm_m, int K,
                const double* freq, int64_t nf, double scale_re, double scale_im, int caustic,
                int nthreads, double* out) {
    return fdo_modesum_ex(t, nt, amp, phi_phi, phi_r, f_phi, f_r, marr, narr, ylm_p, ylm_m, K,
                          freq, nf, scale_re, scale_im, caustic, nthreads, out, NULL);
}

int fdo_modesum_ex(const double* t, int nt, const double* amp, const double* phi_phi,
                   const double* phi_r, const double* f_phi, const double* f_r, const int* marr,
                   const int* narr, const double* ylm_p, const double* ylm_m, int K,
                   const double* freq, int64_t nf, double scale_re, double scale_im, int caustic,
                   int nthreads, double* out, double* extrap) {
    if (nt < 2 || K < 0 || nf <= 0) return -1;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    double complex* S = (double complex*)out;
    memset(out, 0, sizeof(double) * 2 * nf);
    if (extrap) memset(extrap, 0, sizeof(double) * nf);
    int ni = nt - 1;
    double* F = malloc(sizeof(double) * nt);
    double* ph = malloc(sizeof(double) * nt);
    double* ar = malloc(sizeof(double) * nt);
    double* ai = malloc(sizeof(double) * nt);
    double* fdk = malloc(sizeof(double) * nt);
    double* cF = malloc(sizeof(double) * 4 * ni);
    double* cP = malloc(sizeof(double) * 4 * ni);
    double* cAr = malloc(sizeof(double) * 4 * ni);
    double* cAi = malloc(sizeof(double) * 4 * ni);
    double* cD = malloc(sizeof(double) * 4 * ni);
    double* cI = malloc(sizeof(double) * 4 * ni);
    double* xs = malloc(sizeof(double) * nt);
    double* ysv = malloc(sizeof(double) * nt);
    double* w1 = malloc(sizeof(double) * nt);
    double* w2 = malloc(sizeof(double) * nt);
    double* w3 = malloc(sizeof(double) * nt);
    const double complex scale = scale_re + I * scale_im;
    for (int h = 0; h < K; ++h) {
        int m = marr[h], n = narr[h];
        for (int i = 0; i < nt; ++i) {
            F[i] = (double)m * f_phi[i] + (double)n * f_r[i];
            ph[i] = (double)m * phi_phi[i] + (double)n * phi_r[i];
            ar[i] = amp[2 * ((size_t)h * nt + i)];
            ai[i] = amp[2 * ((size_t)h * nt + i) + 1];
        }
        spline(t, nt, F, 1, cF, w1, w2, w3);
        spline(t, nt, ph, 1, cP, w1, w2, w3);
        spline(t, nt, ar, 1, cAr, w1, w2, w3);
        spline(t, nt, ai, 1, cAi, w1, w2, w3);
        for (int i = 0; i < nt; ++i)
            fdk[i] = (i < ni) ? cF[4 * i + 2] : dcubic(cF + 4 * (ni - 1), t[ni] - t[ni - 1]);
        spline(t, nt, fdk, 1, cD, w1, w2, w3);
        const double complex yp = ylm_p[2 * h] + I * ylm_p[2 * h + 1];
        const double complex ym = ylm_m[2 * h] + I * ylm_m[2 * h + 1];
        /* monotonic runs */
        int i0 = 0;
        while (i0 < ni) {
            double d0 = F[i0 + 1] - F[i0];
            int sg = d0 > 0 ? 1 : (d0 < 0 ? -1 : 0);
            if (sg == 0) { ++i0; continue; }
            int j = i0;
            while (j + 1 < ni) {
                double dd = F[j + 2] - F[j + 1];
                int s2 = dd > 0 ? 1 : (dd < 0 ? -1 : 0);
                if (s2 != sg) break;
                ++j;
            }
            int a = i0, b = j + 1, npts = b - a + 1;
            for (int q = 0; q < npts; ++q) {
                int kk = sg > 0 ? a + q : b - q;
                xs[q] = F[kk];
                ysv[q] = t[kk];
            }
            spline(xs, npts, ysv, 1, cI, w1, w2, w3);
            double lo = xs[0], hi = xs[npts - 1];
            for (int br = 0; br < 2; ++br) {
                if (br == 1 && m == 0) break;
                /* parent: g = -freq in (lo, hi); partner: g = -freq in (-hi, -lo), t at -g */
                int64_t k0, k1;
                if (br == 0) { k0 = upper_bound(freq, nf, -hi); k1 = lower_bound(freq, nf, -lo); }
                else { k0 = upper_bound(freq, nf, lo); k1 = lower_bound(freq, nf, hi); }
#pragma omp parallel for schedule(static)
                for (int64_t k = k0; k < k1; ++k) {
                    double g = -freq[k];
                    double ginv = br == 0 ? g : -g;
                    int r = find_interval(xs, npts, ginv);
                    double tt = cubic(cI + 4 * r, ginv - xs[r]);
                    int p = find_interval(t, nt, tt);
                    double w = tt - t[p];
                    double complex A = cubic(cAr + 4 * p, w) + I * cubic(cAi + 4 * p, w);
                    double Ph = cubic(cP + 4 * p, w);
                    double fd = dcubic(cF + 4 * p, w);
                    double fdd = dcubic(cD + 4 * p, w);
                    double complex term;
                    if (br == 0) {
                        term = A * yp * qfactor(fd, fdd, caustic) *
                               cexp(I * (TWO_PI_D * g * tt - Ph));
                    } else {
                        term = conj(A) * ym * qfactor(-fd, -fdd, caustic) *
                               cexp(I * (TWO_PI_D * g * tt + Ph));
                    }
                    S[k] -= term * scale;
                    if (extrap && (tt < t[0] || tt > t[nt - 1])) extrap[k] += cabs(term * scale);
                }
            }
            i0 = b;
        }
    }
    free(F); free(ph); free(ar); free(ai); free(fdk); free(cF); free(cP); free(cAr); free(cAi);
    free(cD); free(cI); free(xs); free(ysv); free(w1); free(w2); free(w3);
    return 0;
}
