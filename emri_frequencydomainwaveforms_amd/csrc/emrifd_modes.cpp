// emrifd_modes.cpp -- the amplitude stand-in and mode selection of the host upstream (linked into
// libemrifd.so; built with -ffast-math so the exponentials vectorise through glibc's libmvec).
//
// STAND-IN PHYSICS, NOT FEW (the ROMAN network's weights are absent offline, SURVEY.md section 2
// row 1c). The C++ form of amplitude.py:
//   SyntheticTeukolskyAmplitude  |A_lmn(p, e)| = 10^(log10(10^core + 10^tail)
//                                + (l + 2)/2 log10(10/p) + jitter_lmn), core = -1 - decay,
//                                tail = -3.6 - 0.085 decay, decay = 0.42 (l - 2) + 0.30 (l - m)
//                                + 0.60 |n - 1.4 m e| / (0.35 + 2.2 e); phase = phase0_lmn
//                                + 0.2 (l - m + 1) 10/p + 0.1 n e (seeded phase0 / jitter in)
//   ModeSelector(eps)            at every trajectory knot, sort |A Y|^2 over the +m branches and
//                                the -m partners, keep them while the power before them is below
//                                (1 - eps) of the total, fold -m picks onto +m, union over knots
//                                (few.utils.modeselector as recalled, notebook :125-127)
// The selection bins the candidate powers by their top 16 bits instead of sorting all ~7,700 per
// knot.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include <omp.h>

#include "../../include/emrifd.h"

namespace {
constexpr double LN10 = 2.302585092994045684017991454684364208;

// |A| of every mode at one knot (vectorised over the modes)
void magnitudes(double p, double e, int nm, const double* c1, const double* dn, const double* dm,
                const double* hl, const double* jit, double* mag) {
    const double invw = 1.0 / (0.35 + 2.2 * e);
    const double pe = 1.4 * e;
    const double lp = std::log10(10.0 / p);
#pragma omp simd
    for (int k = 0; k < nm; ++k) {
        const double decay = c1[k] + 0.60 * std::fabs(dn[k] - dm[k] * pe) * invw;
        const double x = hl[k] * lp + jit[k];
        mag[k] = std::exp(LN10 * (x - 1.0 - decay)) + std::exp(LN10 * (x - 3.6 - 0.085 * decay));
    }
}
// threads for one efd_host_modes call, per calling thread (efd_host_set_threads): the API's
// one-at-a-time calls split the knots over the rank's host cores, and each prefetch pool thread
// sets its share of the pool for the batch it works (pool size / walkers, at least 1)
thread_local int t_threads = 1;
}  // namespace

extern "C" int efd_host_set_threads(int32_t n) {
    t_threads = n < 1 ? 1 : n;
    return EFD_OK;
}

extern "C" int efd_host_modes(const double* p, const double* e, int32_t nt, const int32_t* l,
                              const int32_t* m, const int32_t* n, const double* phase0,
                              const double* jitter, int32_t nmodes, const double* ylm_p,
                              const double* ylm_m, double eps, int32_t* keep, int32_t* nkeep,
                              double* teuk, int64_t teuk_cap) {
    if (!p || !e || !l || !m || !n || !phase0 || !jitter || !ylm_p || !ylm_m || !keep ||
        !nkeep || nt < 1 || nmodes < 1)
        return EFD_ERR_ARG;
    const int nm = nmodes;
    std::vector<double> c1(nm), dn(nm), dm(nm), hl(nm), yp2(nm), ym2(nm);
    std::vector<int32_t> partner_of;   // power index nm + j -> mode (the -m partners)
    for (int k = 0; k < nm; ++k) {
        c1[k] = 0.42 * (l[k] - 2.0) + 0.30 * (double)(l[k] - m[k]);
        dn[k] = n[k];
        dm[k] = m[k];
        hl[k] = 0.5 * (l[k] + 2.0);
        yp2[k] = ylm_p[2 * k] * ylm_p[2 * k] + ylm_p[2 * k + 1] * ylm_p[2 * k + 1];
        ym2[k] = ylm_m[2 * k] * ylm_m[2 * k] + ylm_m[2 * k + 1] * ylm_m[2 * k + 1];
        if (m[k] != 0) partner_of.push_back(k);
    }
    const int np_ = nm + (int)partner_of.size();
    std::vector<unsigned char> kept(nm, 0);
    // the knots' selections are independent and their union is order-free: any thread count
    // gives the same kept set
    const int nth = std::max(1, std::min(t_threads, nt / 4));
#pragma omp parallel num_threads(nth) if (nth > 1)
    {
    std::vector<unsigned char> kept_l(nm, 0);
    std::vector<double> mag(nm), pw(np_), hs;
    std::vector<int32_t> cand(np_), idx(np_), cut(np_), hc;
    std::vector<uint16_t> key(np_);
#pragma omp for schedule(static)
    for (int i = 0; i < nt; ++i) {
        magnitudes(p[i], e[i], nm, c1.data(), dn.data(), dm.data(), hl.data(), jitter, mag.data());
        double total = 0.0;
        for (int k = 0; k < nm; ++k) pw[k] = mag[k] * mag[k] * yp2[k];
        for (size_t j = 0; j < partner_of.size(); ++j) {
            const int k = partner_of[j];
            pw[nm + j] = mag[k] * mag[k] * ym2[k];
        }
        // keep the largest while the sum before them is < (1 - eps) total: the kept set is the
        // top-c, c = min{c : sum of the top c >= threshold}. The c-th largest exceeds
        // eps total / np (the bottom np - c + 1 sum to more than eps total), so only the powers
        // above that floor are candidates; they are binned by their top 16 bits (exponent and 4
        // mantissa bits; 4 interleaved histograms, no store-to-load chains on equal bins), every
        // bin above the one where the running sum from the top crosses the threshold is kept
        // whole, and only that bin is sorted. (Round 4 binned every power by its exponent:
        // 2.4x the time, the histogram's read-modify-write chains and the crossing bin's sort.)
        for (int k = 0; k < np_; ++k) total += pw[k];
        double need = total * (1.0 - eps);
        const double floor_ = eps * total / (double)np_;
        int nc = 0;
        for (int k = 0; k < np_; ++k) {   // branch-free compaction
            cand[nc] = k;
            nc += pw[k] > floor_ ? 1 : 0;
        }
        uint32_t kmin = 0xffffu, kmax = 0u;
        for (int j = 0; j < nc; ++j) {
            uint64_t u;
            std::memcpy(&u, &pw[cand[j]], 8);
            const uint32_t q = (uint32_t)(u >> 48);
            key[j] = (uint16_t)q;
            kmin = std::min(kmin, q);
            kmax = std::max(kmax, q);
        }
        int lo = 0;
        if (nc > 0) {
            const int R = (int)(kmax - kmin) + 1;
            hs.assign(4 * (size_t)R, 0.0);
            hc.assign(4 * (size_t)R, 0);
            for (int j = 0; j < nc; ++j) {
                const int b = (int)(key[j] - kmin) * 4 + (j & 3);
                hs[b] += pw[cand[j]];
                ++hc[b];
            }
            int bcut = -1;
            for (int b = R - 1; b >= 0; --b) {
                const int c = hc[4 * b] + hc[4 * b + 1] + hc[4 * b + 2] + hc[4 * b + 3];
                if (!c) continue;
                const double sb = (hs[4 * b] + hs[4 * b + 1]) + (hs[4 * b + 2] + hs[4 * b + 3]);
                if (sb >= need) { bcut = b; break; }
                need -= sb;
            }
            const int kc = bcut + (int)kmin;
            int nb = 0;
            for (int j = 0; j < nc; ++j) {   // branch-free partition: above / the crossing bin
                const int q = key[j];
                idx[lo] = cand[j];
                lo += q > kc ? 1 : 0;
                cut[nb] = cand[j];
                nb += q == kc ? 1 : 0;
            }
            if (bcut >= 0) {
                std::sort(cut.begin(), cut.begin() + nb, [&](int x, int y) { return pw[x] > pw[y]; });
                for (int j = 0; j < nb && need > 0.0; ++j) {
                    need -= pw[cut[j]];
                    idx[lo++] = cut[j];
                }
            }
        }
        if (lo == 0 && np_ > 0) {   // the largest is always kept
            int best = 0;
            for (int k = 1; k < np_; ++k) best = pw[k] > pw[best] ? k : best;
            idx[lo++] = best;
        }
        for (int k = 0; k < lo; ++k) {
            const int q = idx[k];
            kept_l[q < nm ? q : partner_of[q - nm]] = 1;
        }
    }
#pragma omp critical
    for (int k = 0; k < nm; ++k) kept[k] |= kept_l[k];
    }
    int K = 0;
    for (int k = 0; k < nm; ++k)
        if (kept[k]) keep[K++] = k;
    *nkeep = K;
    if (!teuk) return EFD_OK;
    if ((int64_t)K * nt * 2 > teuk_cap) return EFD_ERR_WORKSPACE;
    // complex amplitudes of the kept modes, [nt][K] (FEW teuk_modes layout)
    std::vector<double> kc1(K), kdn(K), kdm(K), khl(K), kjit(K), kph(K), kdr(K);
    for (int j = 0; j < K; ++j) {
        const int k = keep[j];
        kc1[j] = c1[k]; kdn[j] = dn[k]; kdm[j] = dm[k]; khl[j] = hl[k]; kjit[j] = jitter[k];
        kph[j] = phase0[k];
        kdr[j] = 0.2 * (double)(l[k] - m[k] + 1);
    }
#pragma omp parallel num_threads(nth) if (nth > 1)
    {
    std::vector<double> kmg(K), kph2(K), kc(K), ks(K);
#pragma omp for schedule(static)
    for (int i = 0; i < nt; ++i) {
        magnitudes(p[i], e[i], K, kc1.data(), kdn.data(), kdm.data(), khl.data(), kjit.data(),
                   kmg.data());
        const double q = 10.0 / p[i], ei = e[i];
        double* row = teuk + 2 * (size_t)i * K;
#pragma omp simd
        for (int j = 0; j < K; ++j) kph2[j] = kph[j] + (kdr[j] * q + 0.1 * kdn[j] * ei);
        // cos and sin in separate loops, each vectorised (a joint sincos call is not)
#pragma omp simd
        for (int j = 0; j < K; ++j) kc[j] = std::cos(kph2[j]);
#pragma omp simd
        for (int j = 0; j < K; ++j) ks[j] = std::sin(kph2[j]);
        for (int j = 0; j < K; ++j) {
            row[2 * j] = kmg[j] * kc[j];
            row[2 * j + 1] = kmg[j] * ks[j];
        }
    }
    }
    return EFD_OK;
}
