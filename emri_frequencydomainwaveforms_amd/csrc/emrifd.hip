// emrifd.hip -- MI355X (gfx950, CDNA4) FD EMRI mode-sum: kernels + C ABI (include/emrifd.h).
//
// Hot path (BASELINE.json:north_star): for every
// selected harmonic k = (l, m, n) of the sparse inspiral, the stationary-phase spectrum
//   S(f) = - scale * sum_k [ Y+_k z_k(g) at f = -g ,  Y-_k conj(z_k(g)) at f = +g ]
//   z_k(g) = A_k(t) Q(F', F'') exp(i (2 pi g t - Phi_k(t))),  t = t_k(g) (inverse spline)
// restated from the reference notebook FD_waveform (Tutorial_FD_construction_single_mode.ipynb
// :552-623): Phi_k = m Phi_phi + n Phi_r (:558), F_k = m f_phi + n f_r (:564), t(f) from the
// inverse spline CubicSpline(F, t) (:566), supports (:569-572), F' and F'' spline derivatives
// (:579-584), amplitude spline (:587-594), K_{1/3} factor (:599-613), phases (:615-616).
// The oracle (oracle/fd_oracle.py) states the same maths in numpy; tests pin them together.
//
// Pipeline (one stream per phase, no host sync, no allocation). Preparation
// (efd_modesum_prepare, latency-bound kernels on few CUs, overlapping the previous sum):
//   K0 k_group, k_group_amp  (m, n) groups of the harmonics; per knot, the group amplitudes
//                            Bp = sum_l y0_l A_l, Bm = sum_l y1_l A_l
//   K1-K3 k_prep          one launch, three independent roles by workgroup:
//                         - 1 wave: not-a-knot splines of Phi_phi, Phi_r, f_phi, f_r and of the
//                           knot derivatives f_phi'(t_i), f_r'(t_i) (for F'' as notebook :583)
//                         - 1 lane per group amplitude interpolant (4G lanes), sharing one LDS
//                           factorisation of the knot matrix
//                         - 1 lane per group: F knots, monotonic runs, inverse spline per run
//   K4 k_items            1 thread per (group, knot interval): gathers every cubic the SPA
//                         needs for that interval into one 288-B record + its bin (lane) ranges
//   K5 k_segment_slots    1 thread per (group, run, sub-branch): its segment of records,
//      k_segment_compact  trimmed of clamped empty records; then compacted in slot order;
//      k_seg_tiles        per (segment, tile it covers) the record sub-range reaching the tile
//   K6 k_tile_keys        per tile, its ordered record list (prebuilt keys)
//   K7 k_tile_order       tiles by cost, most expensive first (the sum's dispatch order)
// Mode sum (efd_modesum_sum):
//   K8 k_modesum          OUTPUT-STATIONARY: one 4-wave workgroup per tile of 256*BPL bins;
//                         each lane owns BPL bins (and their mirrors -f when the grid is
//                         symmetric: the +m branch and its -m partner share t(g), the
//                         amplitude/phase splines and sin/cos, so one evaluation feeds two
//                         bins); the tile's record list comes by LDS-DMA from K6 (or is built
//                         in LDS from the segment table, fixed order -> bitwise reproducible),
//                         records stream through a double-buffered LDS stage, and the tile
//                         writes its bins (or h+/hx) once -- no atomics, no host sync.
// The SPA evaluation is FP64 VALU work (phases reach ~1e7 rad); MFMA is not applicable.

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <algorithm>
#include <atomic>
#include <mutex>
#include <cstring>
#include <string>
#include <type_traits>

#include "../../include/emrifd.h"

#define EFD_VERSION 100  // 0.1.0

namespace {

constexpr int TILE = 256;           // threads per workgroup in k_modesum (round 2: 512-thread
                                    // tiles of 8 waves ran 0.974x)
constexpr int NWAVE = TILE / 64;    // waves per workgroup
// bins (lanes) per thread in k_modesum. Round 4: 3 with the own/mirror amplitude cubics split
// (below) fits the 128-VGPR budget without spills in the record loop: config 2 +2.1-2.4% over 2
// (paired A/B, 3 rounds on two boxes, profiles/r04_ab_bpl3.jsonl); 4 spilled (-4%)
#ifndef EFD_BPL
#define EFD_BPL 3   // (an experiment switch: -DEFD_BPL=4)
#endif
constexpr int BPL = EFD_BPL;
constexpr int TILE_LANES = TILE * BPL;  // frequency bins (lanes) per tile
// k_modesum's packed chunk record header (one word per record, read by v_readlane): the
// sub-branch's lane range relative to the tile (HDR_HB bits each), s, the series length J (3
// bits) and Item::fdneg (2 bits)
constexpr int HDR_HB = TILE_LANES < 1024 ? 10 : 11;
constexpr int HDR_S = 2 * HDR_HB, HDR_J = 2 * HDR_HB + 1, HDR_FD = 2 * HDR_HB + 4;
constexpr int XCD_GROUP = 1024 / TILE;  // consecutive tiles per XCD in the dispatch order
constexpr int MAXRUNS = 8;          // monotonic runs per harmonic
// k_segments_one: one 1024-thread workgroup per waveform when its 2 MAXRUNS K segment slots fit
constexpr int SEG1_NT = 1024;
constexpr int SEG1_MAX_K = SEG1_NT / (2 * MAXRUNS);
constexpr int MAX_NT = 1024;        // knots (FEW max_init_len is 1000); bounds LDS staging
constexpr int KEYCAP = 2048;        // record keys per tile pass held in LDS
constexpr int SEGWIN = TILE;        // segments examined per window (tile list build): 4 KB of LDS
                                    // instead of 16 at 4 x TILE, so 4 workgroups fit a CU
constexpr int MAX_K = 8192;         // harmonics per call
// Split tiles of the sparse fused likelihood (K <= SEG1_MAX_K: k_segments_one plans them). A
// tile whose estimated cost (wave-records: records x the 192-lane wave chunks each reaches)
// exceeds the waveform's fair share of the chip is evaluated by BPL workgroups, workgroup j
// taking bin j of every lane over the tile's whole record list (the sub-bin form of
// modesum_tile: each bin's sum in the whole tile's order, so the result is bitwise unsplit);
// the last of them (agent-scope release / acquire, counter per tile) runs the tile's epilogue
// from the bins they stored. A split across the record list instead (every S-th chunk, partial
// sums added by the last) reordered each bin's sum: the injection's logL became -6e-33, not 0.
// Items: the work units of the sparse launch, (tile, bin j, S, slot).
constexpr int SPLIT_ITEM_CAP = 8192;   // items per waveform (union tiles + extra splits)
constexpr int SPLIT_TILE_CAP = 128;    // split tiles per waveform (one slot and counter each)
constexpr int SPLIT_UNION_CAP = 4096;  // union tiles k_segments_one can cost (else no plan)
constexpr int SPLIT_MIN_COST = 48;     // wave-records: tiles below this are never split
constexpr int SPLIT_SLOTS_PER_WF = 64; // the fair share: a waveform's cost / this many workgroups
constexpr double PI = 3.141592653589793238462643383279502884;
constexpr double TWO_PI = 6.283185307179586476925286766559005768;
constexpr double SQRT_3_2PI = 0.69098829894267095480;   // sqrt(3 / (2 pi))
constexpr double INV_SQRT_3_2PI = 1.44720250911653531871; // sqrt(2 pi / 3)
// The records' F'' coefficients carry sqrt(3/(2 pi)) |KRH_1|^(1/4), so the fast path's square
// is v = sqrt|KRH_1| / |y| instead of 1/|y|: rho's leading correction 1 + KRH_1 / y^2 becomes
// 1 - v^2, one FMA (the K_{1/3} series constants below are rescaled to v)
constexpr double VS = 0.18633899812498247470;             // sqrt|KRH_1|
constexpr double FDD_SCALE = 0.29827892638794838654;
constexpr double INV_FDD_SCALE = 3.3525667136785156343;

// Fast-path series length: FAST_J terms of each of R and I/w, exact (truncation < 1e-17) for
// |y| >= FAST_Y (J = 3 -> 555, 4 -> 153, 5 -> 75, 6 -> 48); lanes below FAST_Y take the general
// path, whose K_{1/3} factor comes from the piecewise-polynomial table of kfactor_table.inc.
constexpr int FAST_J = 4;
constexpr double FAST_Y = 153.0;
// Truncation after J terms is KB[J] w^(2J) < 1e-17 for |y| >= JSER_Y[J]; k_items picks the
// smallest J whose bound holds on the whole interval (a lower bound of |y| there).
#define EFD_TABLE __constant__
#include "spa_tables.inc"
// the K_{1/3} factor's polar phase, leading coefficient TH_0 (see KTHN at its use in spa_fast_m)
constexpr double KTH0 = -0.069444444444444444444;   // TH_0
// envelope records (k_items: A(w) polynomial, theta folded into the phase cubic); 1/sqrt from
// the hardware estimate and two Newton steps (~1 ulp; the fit's check needs 1e-11)
__device__ __forceinline__ double env_rsqrt(double x) {
    double y = __builtin_amdgcn_rsq(x);
    y = y * fma(-0.5 * x * y, y, 1.5);
    return y * fma(-0.5 * x * y, y, 1.5);
}
#define EFD_HD __device__
#include "env_fit.inc"
#undef EFD_HD

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            return fail(EFD_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// ----------------------------------------------------------------------------------------
// Data layouts in HBM
// ----------------------------------------------------------------------------------------

// One record per ((m, n) group g, forward knot interval j): everything the SPA needs on the
// bins whose t(g) falls in [t_j, t_{j+1}). All harmonics (l, m, n) of one (m, n) share F, Phi,
// t(f), F', F'', sin/cos and the K_{1/3} factor; only A_lmn Y differs, and the not-a-knot spline
// is linear in its data, so the group carries the two combined amplitude splines
//   Bp(t) = sum_l y0_l A_l(t),  Bm(t) = sum_l y1_l A_l(t)   (y0 = -scale Y+, y1 = conj(-scale Y-))
// and one SPA evaluation serves every l. 288 B (18 pieces of 16 B), staged through LDS.
struct __attribute__((aligned(16))) Item {
    // Field order = the fast path's LDS reads: its first reads are 16-B pairs (ds_read_b128, 4
    // LDS cycles; a misaligned pair takes ds_read2_b64, 8): [gx, ic0] [ic1, ic2] [ic3, tj]
    // [ph0, ph1] [ph2, ph3] [fd0, fd1] [fd2, dtj]; dtj (uncertified records only) rides with fd2
    double gx;        // left end of the inverse-spline interval (ascending F)
    double ic[4];     // t(g) = ((ic0 u + ic1) u + ic2) u + ic3, u = g - gx
    double tj;        // forward interval [tj, tj + dtj)
    double ph[4];     // Phi_mn(t) = m Phi_phi + n Phi_r, w = t - tj (scipy PPoly order)
    double fd[3];     // F'(t)
    double dtj;
    double fdd[3];    // sqrt(3/(2 pi)) F''(t); F'' = derivative of the spline of F'(t_i) (:583)
    int32_t jser;     // K_{1/3} series terms the fast path needs on this interval (1..FAST_J)
    int32_t fdneg;    // F' < 0 at the interval's midpoint: the sign the fast path assumes for
                      // every lane (lanes of the other sign, at a turning point, take the general
                      // path). Also keeps b 16-B aligned, so its cubics come out of LDS by
                      // ds_read_b128 (8 ds_read2_b64 -> ds_read_b128 per record: k_modesum -3%)
    double b[2][2][4];  // b[0] = Bp (re, im cubics), b[1] = Bm: sub-branch s reads b[s] for its
                        // own bin and b[1-s] for the mirror
    int32_t klo[2], khi[2];  // lane ranges per sub-branch s (see k_items)
};
static_assert(sizeof(Item) == 288, "Item must be 288 B");
// Envelope records (k_items, env_fit.inc; Item::jser = 0): the fd, dtj, fdd slots hold the
// ENV_DEG + 1 coefficients of A(w) instead, highest power first, and ph holds Phi - theta. Only
// certified-safe records become envelope records, so nothing that reads fd / dtj / fdd (the
// masked body's tests, the general path) ever meets one.
static_assert(offsetof(Item, dtj) == offsetof(Item, fd) + 24 &&
              offsetof(Item, fdd) == offsetof(Item, fd) + 32 &&
              offsetof(Item, jser) == offsetof(Item, fd) + 8 * (ENV_DEG + 1),
              "envelope coefficients: fd, dtj, fdd contiguous");
// envelope records store A(w) times the sum's cosine constant (COS_A below; static_assert there)
constexpr double ENV_AMP_SCALE = 1.000000000029531;
__host__ __device__ __forceinline__ double* env_of(Item* it) {
    return reinterpret_cast<double*>(reinterpret_cast<char*>(it) + offsetof(Item, fd));
}
__host__ __device__ __forceinline__ const double* env_of(const Item* it) {
    return reinterpret_cast<const double*>(reinterpret_cast<const char*>(it) + offsetof(Item, fd));
}
static_assert(offsetof(Item, ph) % 16 == 0 && offsetof(Item, fd) % 16 == 0 &&
              offsetof(Item, fdd) % 16 == 0, "the fast path's coefficient pairs are 16-B aligned");
constexpr int PIECES = (int)sizeof(Item) / 16;  // 16-B pieces per record
constexpr int B_PIECE = (int)offsetof(Item, b) / 16;   // first piece of b (b[0]: 4, b[1]: 4)
static_assert(offsetof(Item, b) % 16 == 0 && sizeof(Item::b) == 8 * 16, "b: 8 whole pieces");
constexpr int ROUNDS = 2;                        // 16-B pieces per thread per LDS stage
constexpr int NC = (ROUNDS * TILE) / PIECES;     // records per LDS stage

// The error flags (runs_overflow, bad_mn, bad_tile) are sticky: k_group clears only the counters
// of a header it has initialised before (magic == HDR_MAGIC), so an error raised by any call on
// this workspace survives later preparations until efd_modesum_status reports and clears it (a
// pipeline slot reused by several walkers before its status is read loses none of them). A
// header without the magic (fresh device memory) is zeroed whole.
constexpr int64_t HDR_MAGIC = 0x45464448445233LL;   // "EFDHDR3"
struct Header {
    int64_t contributions;      // C of the last call: (l, m, n) branch x bin pairs (k_items)
    int64_t evaluations;        // SPA evaluations: (m, n) group branch x bin pairs
    int32_t runs_overflow;      // set by k_prep when a harmonic has > MAXRUNS monotonic runs
    int32_t groups;             // G: distinct (m, n) of the call (k_group)
    int32_t bad_mn;             // set by k_group when |m| > 255 or |n| > 1023
    int32_t bad_tile;           // set by k_modesum when a dispatch-order entry is out of range
    int64_t magic;              // HDR_MAGIC once k_group has initialised the header
    int32_t lane_lo, lane_hi;   // union [lo, hi) of the segments' lane ranges (k_segment_compact)
    int32_t nitems;             // sparse sum's work items (k_segments_one's split plan), -1: none
    int32_t nsplit;             // split tiles of the plan
    int64_t env_evaluations;    // evaluations on envelope records (k_items; 64 B)
};
static_assert(sizeof(Header) == 64, "Header must be 64 B");


struct Layout {
    size_t header, coefA, coefT, kslope, tscratch, invcp, invdp, runs, items, ranges, seglh,
        seginfo, nseg, slotlh, slotinfo, slotcnt, slottiles, segbase, stb0, stb1, gm, gn, gstart,
        gkeys,
        gmem, gamp, sctab, tkeys, tcnt, tperm, llpart, sitem, scnt, spart, total;
    int64_t stbcap;
    int64_t ntiles, nlanes;
};

__host__ __device__ inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// (also evaluated on the device by the batched preparation kernels: a few dozen scalar integer
// operations per workgroup, so the kernel arguments carry one workspace pointer per waveform)
__host__ __device__ inline Layout make_layout(int32_t nt, int32_t K, int64_t nf, int paired) {
    Layout L{};
    const int64_t ni = nt - 1;
    L.nlanes = paired ? (nf + 1) / 2 : nf;
    L.ntiles = (L.nlanes + TILE_LANES - 1) / TILE_LANES;
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off = align256(off + bytes); return o; };
    L.header = take(sizeof(Header));
    L.coefA = take(sizeof(double) * ni * 4 * 4 * K);   // [ni][4][4K]: Bp re/im, Bm re/im
    L.coefT = take(sizeof(double) * ni * 4 * 8);
    L.kslope = take(sizeof(double) * nt * 2);
    L.tscratch = take(sizeof(double) * nt * 16);
    L.invcp = take(sizeof(double) * nt * K);
    L.invdp = take(sizeof(double) * nt * K);
    L.runs = take(sizeof(int32_t) * 4 * MAXRUNS * K);
    L.items = take(sizeof(Item) * ni * K);
    L.ranges = take(sizeof(int4) * ni * K);
    L.seglh = take(sizeof(int2) * 2 * MAXRUNS * K);
    L.seginfo = take(sizeof(int4) * 2 * MAXRUNS * K);
    L.nseg = take(sizeof(int32_t));
    L.slotlh = take(sizeof(int2) * 2 * MAXRUNS * K);
    L.slotinfo = take(sizeof(int4) * 2 * MAXRUNS * K);
    L.slotcnt = take(sizeof(int32_t) * ((2 * MAXRUNS * K + 255) / 256));
    L.slottiles = take(sizeof(int32_t) * ((2 * MAXRUNS * K + 255) / 256));
    L.segbase = take(sizeof(int32_t) * 2 * MAXRUNS * K);
    // segment-tile boundaries (k_seg_tiles): one (p0, p1) pair per (segment, tile it covers);
    // segments past the capacity keep the bisection
    L.stbcap = 64 * L.ntiles + 4 * (int64_t)(2 * MAXRUNS * K);
    L.stb0 = take(sizeof(int32_t) * (size_t)L.stbcap);
    L.stb1 = take(sizeof(int32_t) * (size_t)L.stbcap);
    L.gm = take(sizeof(int32_t) * K);
    L.gn = take(sizeof(int32_t) * K);
    L.gstart = take(sizeof(int32_t) * (K + 1));
    L.gmem = take(sizeof(int32_t) * K);
    L.gkeys = take(sizeof(unsigned long long) * (size_t)MAX_K);   // k_group's general-case sort
    L.gamp = take(sizeof(double) * nt * 4 * K);
    L.sctab = take(sizeof(double) * 2 * 512);
    L.tkeys = take(sizeof(uint32_t) * (size_t)L.ntiles * KEYCAP);   // prebuilt tile lists
    L.tcnt = take(sizeof(int32_t) * (size_t)L.ntiles);
    L.tperm = take(sizeof(int32_t) * (size_t)L.ntiles);   // cost-ordered dispatch (k_tile_order)
    L.llpart = take(sizeof(double) * (size_t)L.ntiles);   // fused likelihood: per-tile partials
    // the sparse sum's split plan (k_segments_one, K <= SEG1_MAX_K only): items, one arrival
    // counter per split tile, the partial sums of the splits ([slot][lane][4] doubles)
    // (in both layouts: efd_modesum_workspace_bytes sizes by the unpaired one, which must stay
    // the larger)
    const bool plan = K <= SEG1_MAX_K;
    L.sitem = take(plan ? sizeof(int4) * SPLIT_ITEM_CAP : 0);
    L.scnt = take(plan ? sizeof(int32_t) * SPLIT_TILE_CAP : 0);
    L.spart = take(plan ? sizeof(double) * 4 * (size_t)SPLIT_TILE_CAP * TILE_LANES : 0);
    L.total = off;
    return L;
}

// Preparation of up to EFD_BATCH_MAX waveforms per launch (efd_modesum_prepare_batch; a single
// efd_modesum_prepare is a batch of one): blockIdx.z picks the waveform, the grids are sized for
// the batch's largest (nt, K), and each workgroup derives its waveform's workspace layout from
// (nt, K, nf, paired). Every waveform of a batch shares nf and the grid's symmetry.
struct PrepDesc {
    const double *t, *phi_phi, *phi_r, *f_phi, *f_r, *amp, *ylm_p, *ylm_m, *freq;
    const int32_t *m, *n;
    char* ws;
    double sc_re, sc_im;
    int32_t nt, K;
    int32_t lists;   // 1: prebuilt tile lists (k_tile_keys), 3: and cost-ordered dispatch
    int32_t pcr;     // bit 0: k_prep_pcr_b builds the trajectory and inverse splines, bit 1:
                     // and the amplitude splines (else k_prep_b's roles); set per waveform from
                     // its own (N_t, K), so a workspace never depends on its batch
    int32_t env;     // k_items makes envelope records (uniform caustic mode; EFD_ENV=0: none)
};
struct PrepBatch {
    PrepDesc d[EFD_BATCH_MAX];
    int64_t nf, nl, nl1;
    int32_t paired, n;
    int32_t pcr_groups;   // k_prep_pcr_b groups the harmonics itself (k_group_b not launched)
    int32_t seg_lds;      // k_segments_one's dynamic LDS bytes for the ranges table (0: none)
    int32_t split_min;    // k_segments_one: tiles costing at most this (wave-records) stay whole
};
static_assert(sizeof(PrepBatch) <= 3072, "kernel arguments stay well inside 4 KB");

// the waveform of this workgroup: its descriptor and workspace layout
#define PREP_WALKER(B)                                                   \
    const PrepDesc& D = (B).d[blockIdx.z];                                \
    const Layout L = make_layout(D.nt, D.K, (B).nf, (B).paired);          \
    char* const W = D.ws
template <class T>
__device__ __forceinline__ T* ws_at(char* ws, size_t off) { return reinterpret_cast<T*>(ws + off); }

// rows of scratch / knot data fetched per block ahead of the serial spline recurrences
constexpr int SPLINE_PF = 8;   // 16: same, 32: slower (k_prep 110 -> 177 us)

// 1/x for the spline solves: the hardware reciprocal estimate and two Newton steps (5 dependent
// operations, within an ulp) instead of the IEEE division sequence (~10, with the scale and
// fixup steps) on the serial Thomas chains, whose latency sets the preparation's length; the
// coefficients stay within 1e-11 of scipy's (tests/test_gpu_modesum.py), their rounding level
__device__ __forceinline__ double spl_rcp(double x) {
#ifdef EFD_EXP_EXACT_RCP   // experiment: IEEE division (the host twin's), for the HIP = twin study
    return 1.0 / x;
#endif
    double y = __builtin_amdgcn_rcp(x);
    double e = fma(-x, y, 1.0);
    y = fma(y, e, y);
    e = fma(-x, y, 1.0);
    return fma(y, e, y);
}

// ----------------------------------------------------------------------------------------
// Not-a-knot cubic spline solve (scipy.interpolate.CubicSpline semantics)
// ----------------------------------------------------------------------------------------
// Slopes s_i solve the tridiagonal system of scipy/_cubic.py (rows 0 and n-1 encode the
// not-a-knot end conditions); coefficients follow scipy's PPoly construction:
//   tt = (s_i + s_{i+1} - 2 slope_i)/dx_i; c0 = tt/dx_i; c1 = (slope_i - s_i)/dx_i - tt;
//   c2 = s_i; c3 = y_i.
// X(i), Y(i) load knot i; CP/DP are per-lane scratch accessors; OUT(i, c, v) stores.
template <class FX, class FY, class FCP, class FDP, class FOUT>
__device__ void spline_not_a_knot(int n, FX X, FY Y, FCP CP, FDP DP, FOUT OUT) {
    if (n < 2) return;
    if (n == 2) {
        const double dx = X(1) - X(0);
        const double slope = (Y(1) - Y(0)) / dx;
        OUT(0, 0, 0.0); OUT(0, 1, 0.0); OUT(0, 2, slope); OUT(0, 3, Y(0));
        return;
    }
    if (n == 3) {  // parabola through the three points (scipy special case)
        const double dx0 = X(1) - X(0), dx1 = X(2) - X(1);
        const double y0 = Y(0), y1 = Y(1), y2 = Y(2);
        const double sl0 = (y1 - y0) / dx0, sl1 = (y2 - y1) / dx1;
        const double s1 = (dx0 * sl1 + dx1 * sl0) / (dx0 + dx1);
        const double s0 = 2.0 * sl0 - s1, s2 = 2.0 * sl1 - s1;
        double tt = (s0 + s1 - 2.0 * sl0) / dx0;
        OUT(0, 0, tt / dx0); OUT(0, 1, (sl0 - s0) / dx0 - tt); OUT(0, 2, s0); OUT(0, 3, y0);
        tt = (s1 + s2 - 2.0 * sl1) / dx1;
        OUT(1, 0, tt / dx1); OUT(1, 1, (sl1 - s1) / dx1 - tt); OUT(1, 2, s1); OUT(1, 3, y1);
        return;
    }
    // forward sweep (Thomas); row 0
    double x0 = X(0), x1 = X(1), x2 = X(2);
    double y0 = Y(0), y1 = Y(1), y2 = Y(2);
    double dxm = x1 - x0, dxi = x2 - x1;          // dx_{i-1}, dx_i at i = 1
    double slm = (y1 - y0) / dxm, sli = (y2 - y1) / dxi;
    {
        const double d = x2 - x0;
        const double b0 = dxi, c0 = d;
        const double r0 = ((dxm + 2.0 * d) * dxi * slm + dxm * dxm * sli) / d;
        CP(0) = c0 / b0;
        DP(0) = r0 / b0;
    }
    double cpm = CP(0), dpm = DP(0);
    double xi = x2, yi = y2;
    for (int i = 1; i <= n - 2; ++i) {
        // row i: a = dx_i, b = 2(dx_{i-1} + dx_i), c = dx_{i-1}, r = 3(dx_i sl_{i-1} + dx_{i-1} sl_i)
        const double a = dxi, b = 2.0 * (dxm + dxi), c = dxm;
        const double r = 3.0 * (dxi * slm + dxm * sli);
        const double inv = spl_rcp(b - a * cpm);   // one reciprocal on the serial chain
        cpm = c * inv;
        dpm = (r - a * dpm) * inv;
        CP(i) = cpm;
        DP(i) = dpm;
        if (i + 2 <= n - 1) {
            const double xn = X(i + 2), yn = Y(i + 2);
            dxm = dxi; slm = sli;
            dxi = xn - xi; sli = (yn - yi) * spl_rcp(dxi);
            xi = xn; yi = yn;
        }
    }
    // last row (scipy: A[1,-1] = dx[-2], A[-1,-2] = x[-1] - x[-3]): a = x_{n-1} - x_{n-3},
    // b = dx_{n-3}; here dxm = dx_{n-3}, dxi = dx_{n-2}, slm = sl_{n-3}, sli = sl_{n-2}
    double s_next;
    {
        const double d = dxm + dxi;  // x_{n-1} - x_{n-3}
        const double a = X(n - 1) - X(n - 3);
        const double b = dxm;
        const double r = (dxi * dxi * slm + (2.0 * d + dxi) * dxm * sli) / d;
        const double mm = b - a * cpm;
        s_next = (r - a * dpm) / mm;
    }
    // back substitution, emitting interval coefficients from the right. CP/DP may live in
    // global memory: they are fetched PF rows at a time (independent loads, one wait per
    // block) so the serial chain does not pay a memory round trip per row.
    constexpr int PF = SPLINE_PF;
    double xr = X(n - 1), yr = Y(n - 1);
    for (int i0 = n - 2; i0 >= 0; i0 -= PF) {
        double cpb[PF], dpb[PF];
#pragma unroll
        for (int k = 0; k < PF; ++k) {
            const int i = i0 - k;
            cpb[k] = i >= 0 ? CP(i) : 0.0;
            dpb[k] = i >= 0 ? DP(i) : 0.0;
        }
#pragma unroll
        for (int k = 0; k < PF; ++k) {
            const int i = i0 - k;
            if (i < 0) break;
            const double xl = X(i), yl = Y(i);
            const double s_i = dpb[k] - cpb[k] * s_next;
            // one reciprocal for the interval's four quotients (an FP64 division is a ~10-op
            // sequence; x * (1/dx) differs from x / dx by at most an ulp)
            const double rdx = spl_rcp(xr - xl);
            const double sl = (yr - yl) * rdx;
            const double tt = (s_i + s_next - 2.0 * sl) * rdx;
            OUT(i, 0, tt * rdx);
            OUT(i, 1, (sl - s_i) * rdx - tt);
            OUT(i, 2, s_i);
            OUT(i, 3, yl);
            s_next = s_i;
            xr = xl; yr = yl;
        }
    }
}

// derivative of a cubic piece at w (scipy evaluates c2 + 2 c1 w + 3 c0 w^2 by power sum)
__device__ __forceinline__ double dcubic(const double* c, double w) {
    return (c[2] + (2.0 * c[1]) * w) + (3.0 * c[0]) * (w * w);
}

// ----------------------------------------------------------------------------------------
// The same not-a-knot system solved by one wave with parallel cyclic reduction.
// spline_not_a_knot's Thomas sweeps are serial chains of ~2n dependent steps per interpolant,
// with CP/DP round trips through global memory: k_prep took 60-75 us at N_t ~ 100 (the longest
// kernel of a walker's preparation, and the preparation is the latency of small waveforms).
// Here every knot row is a lane's: scipy's two boundary rows are eliminated into rows 1 and
// n-2 (row 0: dx_1 s_0 + (x_2 - x_0) s_1 = r_0, and a_1 = dx_1, so s_0 drops out of row 1
// exactly; the same at the other end), the remaining tridiagonal system in s_1 .. s_{n-2}
// (diagonally dominant: b = 2 (a + c) inside) is normalised to b = 1 and reduced in
// ceil(log2(n - 2)) PCR steps, each row combining its neighbours at distance h:
//   row_k - A_k row_{k-h} - C_k row_{k+h}, renormalised,
// after which every row reads s_k = R_k. The boundary slopes follow from rows 0 and n-1, and
// the interval coefficients are scipy's PPoly construction, in parallel. The slopes agree with
// the Thomas solve to rounding (both are stable on this matrix).
// L: LDS scratch of 7 n doubles; at exit L[0, n) = x, L[n, 2n) = y, L[4n, 5n) = the knot
// slopes s_i. Called by every lane of a one-wave (64-thread) workgroup, 4 <= n <= PCR_NMAX.
// ----------------------------------------------------------------------------------------
constexpr int PCR_RPL = 8;                 // rows per lane
constexpr int PCR_NMAX = 64 * PCR_RPL;     // knots; longer trajectories take the Thomas kernel
// Waveforms of PCR_MAX_K harmonics or more keep the Thomas kernel's amplitude role (one lane per
// interpolant, k_prep_b): their preparation runs beside the previous batch's mode sum, where
// its length is hidden and its CU time is not. One wave per interpolant is ~10x the Thomas
// kernel's wave-time, and with every role on PCR config 2 (3,020 harmonics: 3,139 waves of
// ~10 us, 2,508 of them amplitude splines) lost 1.2% of its rate (paired A/B, ratio 0.988) while
// the latency-bound walker batches gained 6.6% (config 4) and 8.7% (config 5). The trajectory
// and inverse splines (the phases) always take one path for a given N_t, so a harmonic subset
// and the full set share them (the linearity test's 1e-12 bound).
#ifndef PCR_MAX_K
#define PCR_MAX_K 1024
#endif
template <class FX, class FY, class FOUT>
__device__ void pcr_not_a_knot(int n, FX X, FY Y, FOUT OUT, double* L) {
    const int lane = threadIdx.x;
    double* xs = L;
    double* ys = L + n;
    double* dx = L + 2 * n;
    double* sl = L + 3 * n;
    double* A = L + 4 * n;
    double* C = L + 5 * n;
    double* R = L + 6 * n;
    for (int i = lane; i < n; i += 64) {
        xs[i] = X(i);
        ys[i] = Y(i);
    }
    __syncthreads();
    for (int i = lane; i < n - 1; i += 64) {
        const double d = xs[i + 1] - xs[i];
        dx[i] = d;
        sl[i] = (ys[i + 1] - ys[i]) / d;
    }
    __syncthreads();
    const int m = n - 2;   // unknowns s_1 .. s_{n-2}: interior row k holds s_{k+1}
    // scipy's boundary rows: row 0 = (dx_1, x_2 - x_0 | r0), row n-1 = (x_{n-1} - x_{n-3}, dx_{n-3} | rl)
    const double d0 = xs[2] - xs[0];
    const double r0 = ((dx[0] + 2.0 * d0) * dx[1] * sl[0] + dx[0] * dx[0] * sl[1]) / d0;
    const double dl = xs[n - 1] - xs[n - 3];
    const double rl = (dx[n - 2] * dx[n - 2] * sl[n - 3] +
                       (2.0 * dl + dx[n - 2]) * dx[n - 3] * sl[n - 2]) / dl;
    for (int k = lane; k < m; k += 64) {
        const int i = k + 1;
        double a = dx[i], b = 2.0 * (dx[i - 1] + dx[i]), c = dx[i - 1];
        double r = 3.0 * (dx[i] * sl[i - 1] + dx[i - 1] * sl[i]);
        if (i == 1) {       // a_1 = dx_1 = row 0's diagonal: a_1 s_0 = r0 - d0 s_1
            b -= d0;
            a = 0.0;
            r -= r0;
        }
        if (i == n - 2) {   // c_{n-2} = dx_{n-3} = row n-1's diagonal: c s_{n-1} = rl - dl s_{n-2}
            b -= dl;
            c = 0.0;
            r -= rl;
        }
        const double inv = spl_rcp(b);
        A[k] = a * inv;
        C[k] = c * inv;
        R[k] = r * inv;
    }
    __syncthreads();
    for (int h = 1; h < m; h <<= 1) {
        double na[PCR_RPL], nc[PCR_RPL], nr[PCR_RPL];
#pragma unroll
        for (int j = 0; j < PCR_RPL; ++j) {
            if (64 * j >= m) break;    // wave-uniform
            const int k = lane + 64 * j;
            if (k < m) {
                const double ak = A[k], ck = C[k], rk = R[k];
                double al = 0.0, cl = 0.0, rlf = 0.0, ar = 0.0, cr = 0.0, rr = 0.0;
                if (k >= h) { al = A[k - h]; cl = C[k - h]; rlf = R[k - h]; }
                if (k + h < m) { ar = A[k + h]; cr = C[k + h]; rr = R[k + h]; }
                const double inv = spl_rcp(fma(-ck, ar, fma(-ak, cl, 1.0)));
                na[j] = -(ak * al) * inv;
                nc[j] = -(ck * cr) * inv;
                nr[j] = fma(-ck, rr, fma(-ak, rlf, rk)) * inv;
            }
        }
        __syncthreads();   // every row's neighbours read before any row is overwritten
#pragma unroll
        for (int j = 0; j < PCR_RPL; ++j) {
            if (64 * j >= m) break;
            const int k = lane + 64 * j;
            if (k < m) { A[k] = na[j]; C[k] = nc[j]; R[k] = nr[j]; }
        }
        __syncthreads();
    }
    double* S = A;         // knot slopes s_i (A is spent)
    for (int k = lane; k < m; k += 64) S[k + 1] = R[k];
    __syncthreads();
    if (lane == 0) {
        S[0] = (r0 - d0 * S[1]) / dx[1];
        S[n - 1] = (rl - dl * S[n - 2]) / dx[n - 3];
    }
    __syncthreads();
    // scipy's PPoly coefficients per interval (spline_not_a_knot's back-substitution formulas)
    for (int i = lane; i < n - 1; i += 64) {
        const double si = S[i], sn = S[i + 1];
        const double rdx = spl_rcp(xs[i + 1] - xs[i]);
        const double s_l = (ys[i + 1] - ys[i]) * rdx;
        const double tt = (si + sn - 2.0 * s_l) * rdx;
        OUT(i, 0, tt * rdx);
        OUT(i, 1, (s_l - si) * rdx - tt);
        OUT(i, 2, si);
        OUT(i, 3, ys[i]);
    }
    __syncthreads();
}

// ----------------------------------------------------------------------------------------
// K0: (m, n) groups: gm[g], gn[g]; members gmem[gstart[g] .. gstart[g+1]); G = hdr->groups.
// Groups ascend in (m, n), members in harmonic index h (the order every later kernel and the
// oracle's grouping use; a function of (m, n) alone, so everything downstream is deterministic). One 256-thread workgroup with a small LDS footprint: it
// runs while the previous waveform's mode sum holds the GPU, so it must fit where one k_modesum
// workgroup has left a CU (round 1's 1024-thread, 68 KB-LDS bitonic sort needed two to leave the
// same CU at once and waited up to the end of that sum's dispatch, delaying the whole
// preparation chain). Counting sort over the (m, n) box the harmonics span when it has at most
// GB_CAP cells (FEW's l <= 10, |n| <= 30: 21 x 61); otherwise a bitonic sort of (m, n, h) keys
// in the global scratch gkeys. Both give the same groups and member order.
constexpr int GB_CAP = 2048;
__device__ __forceinline__ void header_init(Header* hdr) {
    const bool init = hdr->magic == HDR_MAGIC;
    hdr->contributions = 0;
    hdr->evaluations = 0;
    hdr->env_evaluations = 0;
    hdr->groups = 0;
    hdr->lane_lo = INT32_MAX;   // empty until k_segment_compact's blocks widen it
    hdr->lane_hi = INT32_MIN;
    hdr->nitems = -1;           // no split plan unless k_segments_one makes one
    hdr->nsplit = 0;
    if (!init) {
        hdr->runs_overflow = 0;
        hdr->bad_mn = 0;
        hdr->bad_tile = 0;
        hdr->magic = HDR_MAGIC;
    }
}
__device__ __forceinline__ void group_minmax(int& v_lo, int& v_hi, int* red, int slot) {
    for (int o = 32; o > 0; o >>= 1) {
        v_lo = min(v_lo, __shfl_xor(v_lo, o));
        v_hi = max(v_hi, __shfl_xor(v_hi, o));
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) { red[wave * 4 + slot] = v_lo; red[16 + wave * 4 + slot] = v_hi; }
}
__device__ __forceinline__ void group_body(const int32_t* __restrict__ marr,
                                               const int32_t* __restrict__ narr, int K,
                                               int32_t* __restrict__ gm, int32_t* __restrict__ gn,
                                               int32_t* __restrict__ gstart,
                                               int32_t* __restrict__ gmem,
                                               Header* __restrict__ hdr,
                                               double2* __restrict__ sctab_g,
                                               unsigned long long* __restrict__ gkeys) {
    constexpr int NTH = 256, NW = NTH / 64;
    __shared__ int bcnt[GB_CAP], boff[GB_CAP];
    __shared__ int red[32];
    __shared__ int wsum[2 * NW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // the call's counters start at zero (this is the preparation's first kernel; every later
    // writer runs after it in stream order): no separate hipMemsetAsync per waveform. The error
    // flags stay set until efd_modesum_status clears them (sticky; see Header)
    if (tid == 0) header_init(hdr);
    __syncthreads();
    // k_modesum's (sin, cos)(k pi/256) table, computed once per waveform here and copied into
    // each tile's LDS by LDS-DMA (cheaper than 512 sincospi per tile at small harmonic counts)
    if (sctab_g != nullptr)
        for (int i = tid; i < 512; i += NTH) {
            double sv, cv;
            sincospi((double)i / 256.0, &sv, &cv);
            sctab_g[i] = make_double2(sv, cv);
        }
    auto mval = [&](int i) { return min(max(marr[i], -256), 255); };
    auto nval = [&](int i) { return min(max(narr[i], -1024), 1023); };
    int mlo = INT32_MAX, mhi = INT32_MIN, nlo = INT32_MAX, nhi = INT32_MIN;
    for (int i = tid; i < K; i += NTH) {
        const int m = marr[i], n = narr[i];
        if (m < -256 || m > 255 || n < -1024 || n > 1023) atomicOr(&hdr->bad_mn, 1);
        mlo = min(mlo, mval(i)); mhi = max(mhi, mval(i));
        nlo = min(nlo, nval(i)); nhi = max(nhi, nval(i));
    }
    group_minmax(mlo, mhi, red, 0);
    group_minmax(nlo, nhi, red, 1);
    __syncthreads();
    mlo = red[0]; mhi = red[16]; nlo = red[1]; nhi = red[17];
    for (int w = 1; w < NW; ++w) {
        mlo = min(mlo, red[w * 4]); mhi = max(mhi, red[16 + w * 4]);
        nlo = min(nlo, red[w * 4 + 1]); nhi = max(nhi, red[16 + w * 4 + 1]);
    }
    const int nbn = nhi - nlo + 1;
    const int64_t nb = (int64_t)(mhi - mlo + 1) * nbn;
    if (nb <= GB_CAP) {
        // ---- counting sort over the (m, n) cells: counts, then one pass over the cells (per
        // thread a block of consecutive cells) writes the groups and the cells' offsets
        const int NB = (int)nb;
        auto cell = [&](int i) { return (mval(i) - mlo) * nbn + (nval(i) - nlo); };
        for (int b = tid; b < NB; b += NTH) bcnt[b] = 0;
        __syncthreads();
        for (int i = tid; i < K; i += NTH) atomicAdd(&bcnt[cell(i)], 1);
        __syncthreads();
        const int per = (NB + NTH - 1) / NTH;
        const int b0 = min(NB, tid * per), b1 = min(NB, b0 + per);
        int cm = 0, gmine = 0;
        for (int b = b0; b < b1; ++b) { cm += bcnt[b]; gmine += bcnt[b] > 0; }
        int ci = cm, gi = gmine;   // inclusive wave scans, then across waves
        for (int o = 1; o < 64; o <<= 1) {
            const int vc = __shfl_up(ci, o, 64), vg = __shfl_up(gi, o, 64);
            if (lane >= o) { ci += vc; gi += vg; }
        }
        if (lane == 63) { wsum[wave] = ci; wsum[NW + wave] = gi; }
        __syncthreads();
        int off = ci - cm, g = gi - gmine, G = 0;
        for (int w = 0; w < NW; ++w) {
            if (w < wave) { off += wsum[w]; g += wsum[NW + w]; }
            G += wsum[NW + w];
        }
        for (int b = b0; b < b1; ++b) {
            const int c = bcnt[b];
            boff[b] = off;
            if (c > 0) {
                gm[g] = mlo + b / nbn;
                gn[g] = nlo + b % nbn;
                gstart[g] = off;
                ++g;
            }
            off += c;
        }
        __syncthreads();
        // members into their cells (any order), then each cell sorted by h (l values of one
        // (m, n): a handful of members)
        for (int i = tid; i < K; i += NTH) gmem[atomicAdd(&boff[cell(i)], 1)] = i;
        __syncthreads();
        for (int b = b0; b < b1; ++b) {
            const int c = bcnt[b];
            if (c < 2) continue;
            int32_t* mem = gmem + (boff[b] - c);
            for (int x = 1; x < c; ++x) {
                const int32_t v = mem[x];
                int y = x - 1;
                while (y >= 0 && mem[y] > v) { mem[y + 1] = mem[y]; --y; }
                mem[y + 1] = v;
            }
        }
        if (tid == 0) {
            gstart[G] = K;
            hdr->groups = G;
        }
        return;
    }
    // ---- general (m, n) ranges: bitonic sort of ((m, n) << 32 | h) keys in global scratch
    int P = 1;
    while (P < K) P <<= 1;
    for (int i = tid; i < P; i += NTH) {
        unsigned long long k = ~0ull;
        if (i < K) {
            const unsigned gk = ((unsigned)(mval(i) + 256) << 11) | (unsigned)(nval(i) + 1024);
            k = ((unsigned long long)gk << 32) | (unsigned)i;
        }
        gkeys[i] = k;
    }
    __syncthreads();
    for (int size = 2; size <= P; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = tid; t < P / 2; t += NTH) {
                const int lo = 2 * t - (t & (stride - 1));   // index with bit `stride` clear
                const int hi = lo + stride;
                const bool up = (lo & size) == 0;
                const unsigned long long a = gkeys[lo], b = gkeys[hi];
                if ((a > b) == up) { gkeys[lo] = b; gkeys[hi] = a; }
            }
            __syncthreads();
        }
    }
    // group starts: position p starts a group if its (m, n) differs from p - 1; exclusive scan
    // of the start flags over per-thread blocks of consecutive positions
    const int per = (K + NTH - 1) / NTH;
    const int p0 = min(K, tid * per), p1 = min(K, p0 + per);
    int mine = 0;
    for (int p = p0; p < p1; ++p) mine += (p == 0 || (gkeys[p] >> 32) != (gkeys[p - 1] >> 32));
    int incl = mine;
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int g = incl - mine, G = 0;
    for (int w = 0; w < NW; ++w) {
        if (w < wave) g += wsum[w];
        G += wsum[w];
    }
    for (int p = p0; p < p1; ++p) {
        const unsigned long long k = gkeys[p];
        gmem[p] = (int32_t)(unsigned)(k & 0xffffffffu);
        if (p == 0 || (k >> 32) != (gkeys[p - 1] >> 32)) {
            const unsigned gk = (unsigned)(k >> 32);
            gm[g] = (int32_t)(gk >> 11) - 256;
            gn[g] = (int32_t)(gk & 2047u) - 1024;
            gstart[g] = p;
            ++g;
        }
    }
    if (tid == 0) {
        gstart[G] = K;
        hdr->groups = G;
    }
}
__global__ __launch_bounds__(256) void k_group(const int32_t* __restrict__ marr,
                                               const int32_t* __restrict__ narr, int K,
                                               int32_t* gm, int32_t* gn, int32_t* gstart,
                                               int32_t* gmem, Header* hdr, double2* sctab_g,
                                               unsigned long long* gkeys) {
    group_body(marr, narr, K, gm, gn, gstart, gmem, hdr, sctab_g, gkeys);
}
__global__ __launch_bounds__(256) void k_group_b(const PrepBatch B) {
    PREP_WALKER(B);
    group_body(D.m, D.n, D.K, ws_at<int32_t>(W, L.gm), ws_at<int32_t>(W, L.gn),
               ws_at<int32_t>(W, L.gstart), ws_at<int32_t>(W, L.gmem), ws_at<Header>(W, L.header),
               ws_at<double2>(W, L.sctab), ws_at<unsigned long long>(W, L.gkeys));
}

// K0b: group amplitudes at the knots, one thread per (knot i, group g):
//   Bp = sum_l y0_l A_l(t_i),  Bm = sum_l y1_l A_l(t_i),  y0 = -scale Y+,  y1 = conj(-scale Y-)
// (y1 = 0 for m = 0: no partner), summed in ascending h. gamp is [nt][4K]: (Bp re, Bp im,
// Bm re, Bm im) of group g at 4g. S = -h_nb(-f) * scale: the minus sign and scale live here.
// group_amp_at is the one evaluation: k_group_amp_b stores it for k_prep_b's Thomas roles, and
// k_prep_pcr_b's amplitude waves call it for their own component (no gamp pass, one launch
// fewer in the chain; the same operations in the same order, so the same values).
template <class MEM>
__device__ __forceinline__ double4 group_amp_sum(const double* __restrict__ amp,
                                                 const double* __restrict__ ylm_p,
                                                 const double* __restrict__ ylm_m, double sc_re,
                                                 double sc_im, bool partner, int p0, int p1,
                                                 MEM mem, int K, int i) {
    double bpr = 0.0, bpi = 0.0, bmr = 0.0, bmi = 0.0;
    for (int p = p0; p < p1; ++p) {
        const int h = mem(p);
        const double ar = amp[((size_t)i * K + h) * 2], ai = amp[((size_t)i * K + h) * 2 + 1];
        const double vr = ylm_p[2 * h], vi = ylm_p[2 * h + 1];
        const double y0r = -(sc_re * vr - sc_im * vi), y0i = -(sc_re * vi + sc_im * vr);
        bpr += ar * y0r - ai * y0i;
        bpi += ar * y0i + ai * y0r;
        if (partner) {
            const double ur = ylm_m[2 * h], ui = ylm_m[2 * h + 1];
            const double y1r = -(sc_re * ur - sc_im * ui), y1i = (sc_re * ui + sc_im * ur);
            bmr += ar * y1r - ai * y1i;
            bmi += ar * y1i + ai * y1r;
        }
    }
    return make_double4(bpr, bpi, bmr, bmi);
}
__device__ __forceinline__ double4 group_amp_at(const double* __restrict__ amp,
                                                const double* __restrict__ ylm_p,
                                                const double* __restrict__ ylm_m, double sc_re,
                                                double sc_im, const int32_t* __restrict__ gm,
                                                const int32_t* __restrict__ gstart,
                                                const int32_t* __restrict__ gmem, int K, int i,
                                                int g) {
    return group_amp_sum(amp, ylm_p, ylm_m, sc_re, sc_im, gm[g] != 0, gstart[g], gstart[g + 1],
                         [&](int p) { return gmem[p]; }, K, i);
}
// the grids of k_items and k_group_amp at K >= ITEMS_SPLIT_K: K / ITEMS_PER_THREAD_K threads per
// interval or knot, a thread taking every (K / ITEMS_PER_THREAD_K)-th of the G <= K (m, n) groups
// (config 2's 3,020 harmonics form 627 groups: K-sized grids were ~80% workgroups that exit at
// once, and each held a slot of the sum beside which the next batch is prepared; 1 -> 8:
// +2.2% waveforms/s, r06v, within noise on a slower box, r06w)
#ifndef ITEMS_PER_THREAD_K
#define ITEMS_PER_THREAD_K 8
#endif
constexpr int ITEMS_SPLIT_K = 1024;
__device__ __forceinline__ void group_amp_body(const double* __restrict__ amp,
                                                   const double* __restrict__ ylm_p,
                                                   const double* __restrict__ ylm_m, double sc_re,
                                                   double sc_im, const int32_t* __restrict__ gm,
                                                   const int32_t* __restrict__ gstart,
                                                   const int32_t* __restrict__ gmem, int nt, int K,
                                                   const Header* __restrict__ hdr,
                                                   double* __restrict__ gamp) {
    // (the grid covers K / ITEMS_PER_THREAD_K groups at large K: a thread may take several)
    const int i = blockIdx.y;
    const int G = hdr->groups;
    if (i >= nt) return;
    for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += gridDim.x * blockDim.x) {
        const double4 v = group_amp_at(amp, ylm_p, ylm_m, sc_re, sc_im, gm, gstart, gmem, K, i,
                                       g);
        double* o = gamp + (size_t)i * 4 * K + 4 * g;
        o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
    }
}
__global__ __launch_bounds__(256) void k_group_amp(const double* __restrict__ amp,
                                                   const double* __restrict__ ylm_p,
                                                   const double* __restrict__ ylm_m, double sc_re,
                                                   double sc_im, const int32_t* __restrict__ gm,
                                                   const int32_t* __restrict__ gstart,
                                                   const int32_t* __restrict__ gmem, int nt, int K,
                                                   const Header* __restrict__ hdr,
                                                   double* __restrict__ gamp) {
    group_amp_body(amp, ylm_p, ylm_m, sc_re, sc_im, gm, gstart, gmem, nt, K, hdr, gamp);
}
__global__ __launch_bounds__(256) void k_group_amp_b(const PrepBatch B) {
    PREP_WALKER(B);
    if (D.pcr & 2) return;   // k_prep_pcr_b evaluates this waveform's group amplitudes itself
    group_amp_body(D.amp, D.ylm_p, D.ylm_m, D.sc_re, D.sc_im, ws_at<int32_t>(W, L.gm),
                   ws_at<int32_t>(W, L.gstart), ws_at<int32_t>(W, L.gmem), D.nt, D.K,
                   ws_at<Header>(W, L.header), ws_at<double>(W, L.gamp));
}

// ----------------------------------------------------------------------------------------
// K1: trajectory splines (one wave; lanes 0..3 the knot data, then lanes 4..5 the slopes)
// coefT layout: [interval][coef c][q], q: 0 Phi_phi, 1 Phi_r, 2 f_phi, 3 f_r, 4 f_phi', 5 f_r'
// ----------------------------------------------------------------------------------------
__device__ void traj_splines(const double* __restrict__ t, const double* __restrict__ phi_phi,
                               const double* __restrict__ phi_r, const double* __restrict__ f_phi,
                               const double* __restrict__ f_r, int nt, double* __restrict__ coefT,
                               double* __restrict__ kslope, double* __restrict__ scratch) {
    // the serial Thomas chains read their knots from LDS instead of global memory
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* xs = lds;                 // t
    double* ys = lds + nt;            // 6 interpolants: Phi_phi, Phi_r, f_phi, f_r, f_phi', f_r'
    for (int i = threadIdx.x; i < nt; i += blockDim.x) {
        xs[i] = t[i];
        ys[i] = phi_phi[i];
        ys[nt + i] = phi_r[i];
        ys[2 * nt + i] = f_phi[i];
        ys[3 * nt + i] = f_r[i];
    }
    __syncthreads();
    const int q = threadIdx.x;
    double* cp = scratch + (size_t)q * nt;
    double* dp = scratch + (size_t)(8 + q) * nt;
    auto X = [&](int i) { return xs[i]; };
    auto CP = [&](int i) -> double& { return cp[i]; };
    auto DP = [&](int i) -> double& { return dp[i]; };
    if (q < 4) {
        const double* y = ys + (size_t)q * nt;
        auto Y = [&](int i) { return y[i]; };
        auto OUT = [&](int i, int c, double v) { coefT[((size_t)i * 4 + c) * 8 + q] = v; };
        spline_not_a_knot(nt, X, Y, CP, DP, OUT);
    }
    __syncthreads();
    // knot values of f_phi'(t) and f_r'(t), evaluated like scipy's derivative PPoly at the knots
    for (int idx = threadIdx.x; idx < 2 * nt; idx += blockDim.x) {
        const int qq = 2 + idx / nt, i = idx % nt;
        double v;
        if (i < nt - 1) {
            v = coefT[((size_t)i * 4 + 2) * 8 + qq];
        } else {
            double c[4];
            for (int cc = 0; cc < 4; ++cc) c[cc] = coefT[((size_t)(nt - 2) * 4 + cc) * 8 + qq];
            v = dcubic(c, xs[nt - 1] - xs[nt - 2]);
        }
        ys[(size_t)(4 + idx / nt) * nt + i] = v;
        kslope[idx] = v;
    }
    __syncthreads();
    if (q >= 4 && q < 6) {
        const double* y = ys + (size_t)q * nt;
        auto Y = [&](int i) { return y[i]; };
        auto OUT = [&](int i, int c, double v) { coefT[((size_t)i * 4 + c) * 8 + q] = v; };
        spline_not_a_knot(nt, X, Y, CP, DP, OUT);
    }
}

// ----------------------------------------------------------------------------------------
// K2: shared-knot splines, one lane per interpolant q < count; knot values YF(i, q); coef is
// [n-1][4][stride] (stride >= count). For the mode sum the interpolants are the four real parts
// of the group amplitudes (Bp re, Bp im, Bm re, Bm im of group q/4), summed over the group's
// harmonics as they are read (FEW's teuk_modes[N_t][K] complex layout underneath).
// ----------------------------------------------------------------------------------------
template <class YF>
__device__ void spline_shared(const double* __restrict__ x, int n, YF yf, int count, int stride,
                              double* coef, int64_t scratch_stride, int block) {
    const int ninterp = stride;
    // The not-a-knot matrix depends only on the shared knots: one thread factors it into LDS
    // (cp_i, 1/m_i, a_i of the Thomas sweep), then every lane runs the two division-free
    // recurrences for its right-hand side. DP(i) lives in the c1 slot of interval i of the
    // output (read back, one row ahead, by the back substitution before that row is written).
    // grids are sized for the harmonic count K before the device knows the group count: blocks
    // past the interpolants leave before the shared factorisation (a serial chain of ~n steps)
    if (block * (int)blockDim.x >= count) return;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* xs = lds;
    double* cpl = lds + n;
    double* iml = lds + 2 * n;
    double* all = lds + 3 * n;
    double* ridx = lds + 4 * n;   // 1 / (x_{i+1} - x_i): every lane's quotients by dx_i
    for (int i = threadIdx.x; i < n; i += blockDim.x) xs[i] = x[i];
    __syncthreads();
    for (int i = threadIdx.x; i < n - 1; i += blockDim.x) ridx[i] = spl_rcp(xs[i + 1] - xs[i]);
    if (threadIdx.x == 0 && n >= 4) {
        double dxm = xs[1] - xs[0], dxi = xs[2] - xs[1];
        double d = xs[2] - xs[0];
        cpl[0] = d / dxi; iml[0] = 1.0 / dxi; all[0] = 0.0;
        for (int i = 1; i <= n - 2; ++i) {
            dxm = xs[i] - xs[i - 1];
            dxi = xs[i + 1] - xs[i];
            const double mm = 2.0 * (dxm + dxi) - dxi * cpl[i - 1];
            const double rm = spl_rcp(mm);
            cpl[i] = dxm * rm; iml[i] = rm; all[i] = dxi;
        }
        const double dl = xs[n - 1] - xs[n - 3];
        const double mm = (xs[n - 2] - xs[n - 3]) - dl * cpl[n - 2];
        iml[n - 1] = 1.0 / mm; all[n - 1] = dl; cpl[n - 1] = 0.0;
    }
    __syncthreads();
    const int q = block * blockDim.x + threadIdx.x;
    if (q >= count) return;
    auto Y = [&](int i) { return yf(i, q); };
    auto OUT = [&](int i, int c, double v) { coef[((size_t)i * 4 + c) * ninterp + q] = v; };
    if (n < 4) {
        double* cpbuf = coef;
        double* dpbuf = coef + ninterp;
        auto X = [&](int i) { return xs[i]; };
        auto CP = [&](int i) -> double& { return cpbuf[(size_t)i * scratch_stride + q]; };
        auto DP = [&](int i) -> double& { return dpbuf[(size_t)i * scratch_stride + q]; };
        spline_not_a_knot(n, X, Y, CP, DP, OUT);
        return;
    }
    double* dpbase = coef + ninterp;   // DP(i) at coef[(i*4+1)*ninterp + q]
    auto DPs = [&](int i) -> double& { return dpbase[(size_t)i * scratch_stride + q]; };
    // Global loads (y, and DP on the way back) are issued PF rows at a time, ahead of the
    // serial recurrence, so each block of rows waits for memory once.
    constexpr int PF = SPLINE_PF;
    // forward sweep: dp_i = (r_i - a_i dp_{i-1}) / m_i, r_i from sl_{i-1}, sl_i
    const double y0 = Y(0), y1 = Y(1);
    double yprev = Y(2);
    double dxm = xs[1] - xs[0], dxi = xs[2] - xs[1];
    double slm = (y1 - y0) * ridx[0], sli = (yprev - y1) * ridx[1];
    double dp;
    {
        const double d = xs[2] - xs[0];
        const double r0 = ((dxm + 2.0 * d) * dxi * slm + dxm * dxm * sli) / d;
        dp = r0 * iml[0];
        DPs(0) = dp;
    }
    for (int i0 = 1; i0 <= n - 2; i0 += PF) {
        double yb[PF];   // y_{i+2} for rows i0 .. i0+PF-1
#pragma unroll
        for (int k = 0; k < PF; ++k) {
            const int j = i0 + k + 2;
            yb[k] = j <= n - 1 ? Y(j) : 0.0;
        }
#pragma unroll
        for (int k = 0; k < PF; ++k) {
            const int i = i0 + k;
            if (i > n - 2) break;
            const double r = 3.0 * (dxi * slm + dxm * sli);
            dp = (r - all[i] * dp) * iml[i];
            DPs(i) = dp;
            if (i + 2 <= n - 1) {
                dxm = dxi; slm = sli;
                dxi = xs[i + 2] - xs[i + 1];
                sli = (yb[k] - yprev) * ridx[i + 1];
                yprev = yb[k];
            }
        }
    }
    double s_next;
    {
        const double d = dxm + dxi;
        const double r = (dxi * dxi * slm + (2.0 * d + dxi) * dxm * sli) / d;
        s_next = (r - all[n - 1] * dp) * iml[n - 1];
    }
    // back substitution
    double yr = Y(n - 1);
    for (int i0 = n - 2; i0 >= 0; i0 -= PF) {
        double dpb[PF], ylb[PF];
#pragma unroll
        for (int k = 0; k < PF; ++k) {
            const int i = i0 - k;
            dpb[k] = i >= 0 ? DPs(i) : 0.0;
            ylb[k] = i >= 0 ? Y(i) : 0.0;
        }
#pragma unroll
        for (int k = 0; k < PF; ++k) {
            const int i = i0 - k;
            if (i < 0) break;
            const double yl = ylb[k];
            const double s_i = dpb[k] - cpl[i] * s_next;
            const double rdx = ridx[i];
            const double sl = (yr - yl) * rdx;
            const double tt = (s_i + s_next - 2.0 * sl) * rdx;
            OUT(i, 0, tt * rdx);
            OUT(i, 1, (sl - s_i) * rdx - tt);
            OUT(i, 2, s_i);
            OUT(i, 3, yl);
            s_next = s_i;
            yr = yl;
        }
    }
}

// ----------------------------------------------------------------------------------------
// K3: inverse splines t(F) per monotonic run, one lane per (m, n) group h
// runs[h][r] = (ja, jb, sign, 0): forward intervals [ja, jb), F increasing (+1)/decreasing (-1)
// Item.gx / Item.ic are filled for the intervals of each run.
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ double knotF(const double* f_phi, const double* f_r, int m, int n,
                                        int i) {
    // numpy's m * f_phi + n * f_r, rounded the same way (no FMA contraction)
    return __dadd_rn(__dmul_rn((double)m, f_phi[i]), __dmul_rn((double)n, f_r[i]));
}

__device__ void inverse_splines(const double* __restrict__ t, const double* __restrict__ f_phi,
                                  const double* __restrict__ f_r, const int32_t* __restrict__ marr,
                                  const int32_t* __restrict__ narr, int nt, int K, int G,
                                  int32_t* __restrict__ runs, Item* __restrict__ items,
                                  double* __restrict__ cpbuf, double* __restrict__ dpbuf,
                                  int32_t* __restrict__ err, int block) {
    if (block * (int)blockDim.x >= G) return;   // grid sized for K >= G
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* ts = lds;              // t, f_phi, f_r staged in LDS for the serial chains
    double* fps = lds + nt;
    double* frs = lds + 2 * nt;
    for (int i = threadIdx.x; i < nt; i += blockDim.x) {
        ts[i] = t[i];
        fps[i] = f_phi[i];
        frs[i] = f_r[i];
    }
    __syncthreads();
    const int h = block * blockDim.x + threadIdx.x;   // (m, n) group
    if (h >= G) return;
    const int m = marr[h], n = narr[h];
    const int ni = nt - 1;
    Item* it = items + (size_t)h * ni;
    int32_t* rr = runs + (size_t)h * 4 * MAXRUNS;
    for (int r = 0; r < MAXRUNS; ++r) { rr[4 * r] = 0; rr[4 * r + 1] = 0; rr[4 * r + 2] = 0; }
    int nrun = 0;
    int j = 0;
    double Fprev = knotF(fps, frs, m, n, 0);
    // scan the interval signs and emit maximal strictly monotonic runs
    int cur_sign = 0, ja = 0;
    for (j = 0; j <= ni; ++j) {
        int sg = 0;
        double Fn = 0.0;
        if (j < ni) {
            Fn = knotF(fps, frs, m, n, j + 1);
            sg = (Fn > Fprev) ? 1 : ((Fn < Fprev) ? -1 : 0);
        }
        if (sg != cur_sign || j == ni) {
            if (cur_sign != 0) {  // close run [ja, j)
                if (nrun < MAXRUNS) {
                    rr[4 * nrun] = ja; rr[4 * nrun + 1] = j; rr[4 * nrun + 2] = cur_sign;
                    ++nrun;
                } else {
                    atomicOr(err, 1);
                }
            }
            cur_sign = sg;
            ja = j;
        }
        Fprev = Fn;
    }
    // inverse spline per run: x = F ascending, y = t
    for (int r = 0; r < nrun; ++r) {
        const int a = rr[4 * r], b = rr[4 * r + 1], sg = rr[4 * r + 2];
        const int npts = b - a + 1;
        // ascending index q -> knot index
        auto KI = [&](int qq) { return sg > 0 ? a + qq : b - qq; };
        auto X = [&](int qq) { return knotF(fps, frs, m, n, KI(qq)); };
        auto Y = [&](int qq) { return ts[KI(qq)]; };
        auto CP = [&](int qq) -> double& { return cpbuf[(size_t)(a + qq) * K + h]; };
        auto DP = [&](int qq) -> double& { return dpbuf[(size_t)(a + qq) * K + h]; };
        // ascending interval qq covers knots KI(qq), KI(qq+1) -> forward interval
        auto OUT = [&](int qq, int c, double v) {
            const int jf = sg > 0 ? a + qq : b - 1 - qq;
            it[jf].ic[c] = v;
            if (c == 3) it[jf].gx = X(qq);
        };
        spline_not_a_knot(npts, X, Y, CP, DP, OUT);
    }
}

// K1-K3 fused into one launch: the three spline stages are independent, latency-bound serial
// chains on few workgroups, so running them side by side costs max() instead of sum().
// Block 0: trajectory splines; blocks [1, 1 + nb_amp): amplitude splines (64 interpolants per
// block); the rest: inverse splines (64 harmonics per block).
__device__ __forceinline__ void prep_body(
    const double* __restrict__ t, const double* __restrict__ phi_phi,
    const double* __restrict__ phi_r, const double* __restrict__ f_phi,
    const double* __restrict__ f_r, const double* __restrict__ gamp,
    const int32_t* __restrict__ gm,
    const int32_t* __restrict__ gn, int nt, int K,
    int nb_amp, double* __restrict__ coefT, double* __restrict__ kslope,
    double* __restrict__ tscratch, double* coefA, int32_t* __restrict__ runs,
    Item* __restrict__ items, double* __restrict__ invcp, double* __restrict__ invdp,
    Header* __restrict__ hdr) {
    const int b = blockIdx.x;
    if (b == 0) {
        traj_splines(t, phi_phi, phi_r, f_phi, f_r, nt, coefT, kslope, tscratch);
    } else if (b < 1 + nb_amp) {
        const int G = hdr->groups;
        auto yf = [&](int i, int q) { return gamp[(size_t)i * 4 * K + q]; };
        spline_shared(t, nt, yf, 4 * G, 4 * K, coefA, (int64_t)4 * 4 * K, b - 1);
    } else {
        inverse_splines(t, f_phi, f_r, gm, gn, nt, K, hdr->groups, runs, items, invcp, invdp,
                        &hdr->runs_overflow, b - 1 - nb_amp);
    }
}
__global__ __launch_bounds__(64) void k_prep(
    const double* __restrict__ t, const double* __restrict__ phi_phi,
    const double* __restrict__ phi_r, const double* __restrict__ f_phi,
    const double* __restrict__ f_r, const double* __restrict__ gamp,
    const int32_t* __restrict__ gm,
    const int32_t* __restrict__ gn, int nt, int K,
    int nb_amp, double* __restrict__ coefT, double* __restrict__ kslope,
    double* __restrict__ tscratch, double* coefA, int32_t* __restrict__ runs,
    Item* __restrict__ items, double* __restrict__ invcp, double* __restrict__ invdp,
    Header* __restrict__ hdr) {
    prep_body(t, phi_phi, phi_r, f_phi, f_r, gamp, gm, gn, nt, K, nb_amp, coefT, kslope, tscratch,
              coefA, runs, items, invcp, invdp, hdr);
}
// the grid is sized for the batch's largest K: blocks past this waveform's roles leave at once
__global__ __launch_bounds__(64) void k_prep_b(const PrepBatch B) {
    PREP_WALKER(B);
    const int nb_amp = (4 * D.K + 63) / 64, nb_inv = (D.K + 63) / 64;
    if ((int)blockIdx.x >= 1 + nb_amp + nb_inv) return;
    if (D.pcr & 1) {   // k_prep_pcr_b has the trajectory and inverse roles (and maybe this one)
        const int b = blockIdx.x;
        if (b == 0 || b >= 1 + nb_amp || (D.pcr & 2)) return;
    }
    prep_body(D.t, D.phi_phi, D.phi_r, D.f_phi, D.f_r, ws_at<double>(W, L.gamp),
              ws_at<int32_t>(W, L.gm), ws_at<int32_t>(W, L.gn), D.nt, D.K, nb_amp,
              ws_at<double>(W, L.coefT), ws_at<double>(W, L.kslope), ws_at<double>(W, L.tscratch),
              ws_at<double>(W, L.coefA), ws_at<int32_t>(W, L.runs), ws_at<Item>(W, L.items),
              ws_at<double>(W, L.invcp), ws_at<double>(W, L.invdp), ws_at<Header>(W, L.header));
}

// K1-K3 with one wave per interpolant (parallel cyclic reduction): blocks [0, 4) the trajectory splines (Phi_phi,
// Phi_r, f_phi, f_r; the f_phi and f_r blocks go on to f_phi', f_r' from their own knot
// slopes), [4, 4 + K) the inverse splines of group h = b - 4 < G, [4 + K, 4 + 5K) the group
// amplitude splines (interpolant q = b - 4 - K < 4G; only when Item::pcr bit 1 is set, else the
// grid stops at 4 + K). Blocks past this waveform's G leave at once.
// The same coefficients as k_prep's (scipy's construction, to rounding); for 4 <= N_t <=
// PCR_NMAX (the host takes k_prep_b otherwise). Dynamic LDS: 9 N_t doubles.
struct GroupAmpSrc {   // group_amp_at's operands
    const double *amp, *ylm_p, *ylm_m;
    double sc_re, sc_im;
    const int32_t *gstart, *gmem;
};
// The block's (m, n) group when k_prep_pcr_b groups the harmonics itself (PrepBatch::pcr_groups,
// k_group_b not launched): G, the group's (m, n) and its members in ascending h (LDS)
struct LocalGroups {
    bool on;
    int G, m, n, count;
    const int* mem;
};
__device__ __forceinline__ void prep_pcr_body(
    const double* __restrict__ t, const double* __restrict__ phi_phi,
    const double* __restrict__ phi_r, const double* __restrict__ f_phi,
    const double* __restrict__ f_r, const GroupAmpSrc ga, const LocalGroups lg,
    const int32_t* __restrict__ gm, const int32_t* __restrict__ gn, int nt, int K,
    double* __restrict__ coefT, double* __restrict__ kslope, double* __restrict__ coefA,
    int32_t* __restrict__ runs, Item* __restrict__ items, double* __restrict__ invcp,
    double* __restrict__ invdp, Header* __restrict__ hdr) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    auto X = [&](int i) { return t[i]; };
    if (b < 4) {
        // trajectory spline q; q = 2, 3 continue with the derivative splines 4, 5
        const double* y = b == 0 ? phi_phi : b == 1 ? phi_r : b == 2 ? f_phi : f_r;
        int q = b;
        auto Y = [&](int i) { return y[i]; };
        auto OUT = [&](int i, int c, double v) { coefT[((size_t)i * 4 + c) * 8 + q] = v; };
        pcr_not_a_knot(nt, X, Y, OUT, lds);
        if (b < 2) return;
        // knot values of the derivative, as k_prep takes them: c2 of each interval, and scipy's
        // derivative of the last piece at the last knot (the slopes stay in LDS at [4 nt, 5 nt))
        double* v = lds + 7 * nt;
        const double* xs = lds;
        const double* ys = lds + nt;
        const double* S = lds + 4 * nt;
        for (int i = lane; i < nt; i += 64) {
            double vi;
            if (i < nt - 1) {
                vi = S[i];
            } else {
                const double si = S[nt - 2], sn = S[nt - 1];
                const double rdx = spl_rcp(xs[nt - 1] - xs[nt - 2]);
                const double s_l = (ys[nt - 1] - ys[nt - 2]) * rdx;
                const double tt = (si + sn - 2.0 * s_l) * rdx;
                const double c[4] = {tt * rdx, (s_l - si) * rdx - tt, si, ys[nt - 2]};
                vi = dcubic(c, xs[nt - 1] - xs[nt - 2]);
            }
            v[i] = vi;
            kslope[(size_t)(b - 2) * nt + i] = vi;
        }
        __syncthreads();
        q = b + 2;
        auto YV = [&](int i) { return v[i]; };
        pcr_not_a_knot(nt, X, YV, OUT, lds);
        return;
    }
    const int G = lg.on ? lg.G : hdr->groups;
    if (b >= 4 + K) {
        const int q = b - 4 - K;
        if (q >= 4 * G) return;
        const size_t ninterp = (size_t)4 * K;
        // component q & 3 of group q >> 2 at knot i (group_amp_at; no gamp pass)
        auto Y = [&](int i) {
            const double4 v =
                lg.on ? group_amp_sum(ga.amp, ga.ylm_p, ga.ylm_m, ga.sc_re, ga.sc_im, lg.m != 0,
                                      0, lg.count, [&](int p) { return lg.mem[p]; }, K, i)
                      : group_amp_at(ga.amp, ga.ylm_p, ga.ylm_m, ga.sc_re, ga.sc_im, gm,
                                     ga.gstart, ga.gmem, K, i, q >> 2);
            const int c = q & 3;
            return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w;
        };
        auto OUT = [&](int i, int c, double v) { coefA[((size_t)i * 4 + c) * ninterp + q] = v; };
        pcr_not_a_knot(nt, X, Y, OUT, lds);
        return;
    }
    const int h = b - 4;   // (m, n) group
    if (h >= G) return;
    const int m = lg.on ? lg.m : gm[h], n = lg.on ? lg.n : gn[h];
    const int ni = nt - 1;
    Item* it = items + (size_t)h * ni;
    int32_t* rr = runs + (size_t)h * 4 * MAXRUNS;
    double* Fv = lds + 8 * nt;     // F at the knots (PCR uses [0, 7 npts))
    int* sgv = reinterpret_cast<int*>(lds + 7 * nt);   // sign of F_{j+1} - F_j
    for (int i = lane; i < nt; i += 64) Fv[i] = knotF(f_phi, f_r, m, n, i);
    __shared__ int rrs[4 * MAXRUNS];
    __shared__ int nrun_s;
    __syncthreads();
    for (int j = lane; j < ni; j += 64) {
        const double F0 = Fv[j], F1 = Fv[j + 1];
        sgv[j] = (F1 > F0) ? 1 : ((F1 < F0) ? -1 : 0);
    }
    __syncthreads();
    {
        // maximal strictly monotonic runs, as inverse_splines scans them: a run of sign s != 0
        // starts at j where sgv[j] = s differs from sgv[j - 1] (or j = 0) and ends at the next
        // index whose sign differs (or ni, sign 0); the k-th start and the k-th end are run k's.
        // The wave finds them 64 indices at a time with ballots (lane 0 walking every index
        // serially was a chain of ni dependent LDS reads).
        const unsigned long long below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
        int nst = 0, nen = 0;   // starts / ends in the earlier chunks
        for (int c = 0; c <= ni; c += 64) {
            const int j = c + lane;
            const int sj = j < ni ? sgv[j] : 0;
            const int sp = (j >= 1 && j <= ni) ? sgv[j - 1] : 0;
            const bool st = j < ni && sj != 0 && (j == 0 || sp != sj);
            const bool en = j >= 1 && j <= ni && sp != 0 && sj != sp;
            const unsigned long long bs = __ballot(st), be = __ballot(en);
            if (st) {
                const int r = nst + __popcll(bs & below);
                if (r < MAXRUNS) {
                    rr[4 * r] = rrs[4 * r] = j;
                    rr[4 * r + 2] = rrs[4 * r + 2] = sj;
                }
            }
            if (en) {
                const int r = nen + __popcll(be & below);
                if (r < MAXRUNS) rr[4 * r + 1] = rrs[4 * r + 1] = j;
            }
            nst += __popcll(bs);
            nen += __popcll(be);
        }
        const int nrun = min(nst, MAXRUNS);
        // the unused run slots zeroed (none of them written above)
        if (lane < 4 * MAXRUNS && (lane >> 2) >= nrun && (lane & 3) < 3) {
            rr[lane] = 0;
            rrs[lane] = 0;
        }
        if (lane == 0) {
            // the run-overflow marker (not the header itself: with pcr_groups its
            // initialisation runs in this same launch, block 0, unordered with this block),
            // raised into the header by k_items
            rr[3] = nst > MAXRUNS ? 1 : 0;
            nrun_s = nrun;
        }
    }
    __syncthreads();
    const int nrun = nrun_s;
    for (int r = 0; r < nrun; ++r) {
        const int a = rrs[4 * r], bb = rrs[4 * r + 1], sg = rrs[4 * r + 2];
        const int npts = bb - a + 1;
        auto KI = [&](int qq) { return sg > 0 ? a + qq : bb - qq; };
        auto XF = [&](int qq) { return Fv[KI(qq)]; };
        auto YT = [&](int qq) { return t[KI(qq)]; };
        auto OUT = [&](int qq, int c, double v) {
            const int jf = sg > 0 ? a + qq : bb - 1 - qq;
            it[jf].ic[c] = v;
            if (c == 3) it[jf].gx = XF(qq);
        };
        if (npts >= 4) {
            pcr_not_a_knot(npts, XF, YT, OUT, lds);
        } else {
            if (lane == 0) {   // 2 or 3 knots: the closed forms (no scratch)
                auto CP = [&](int qq) -> double& { return invcp[(size_t)(a + qq) * K + h]; };
                auto DP = [&](int qq) -> double& { return invdp[(size_t)(a + qq) * K + h]; };
                spline_not_a_knot(npts, XF, YT, CP, DP, OUT);
            }
            __syncthreads();
        }
    }
}
// PrepBatch::pcr_groups (every waveform of the batch on the PCR roles with K <= 64): each block
// groups the K harmonics itself, one per lane: a harmonic's group is the rank of its (m, n) among
// the distinct pairs, its place in gmem the count of harmonics of smaller (m, n) plus the members
// of its own before it. The same groups, order and member lists as k_group's counting sort (the
// same clamping and bad_mn rule). Block 0 also writes them (gm, gn, gstart, gmem, G), initialises
// the header and fills the sin/cos table: k_group_b's work, without its launch.
constexpr int PCR_GROUPS_MAX_K = 64;
__device__ __forceinline__ LocalGroups pcr_local_groups(const PrepDesc& D, char* W,
                                                        const Layout& L, int* s_mem) {
    const int lane = threadIdx.x, K = D.K, b = blockIdx.x;
    int m = 0, n = 0, key = INT32_MAX;
    bool bad = false;
    if (lane < K) {
        const int mr = D.m[lane], nr = D.n[lane];
        bad = mr < -256 || mr > 255 || nr < -1024 || nr > 1023;
        m = min(max(mr, -256), 255);
        n = min(max(nr, -1024), 1023);
        key = ((m + 256) << 11) | (n + 1024);
    }
    int less = 0, eqb = 0;   // harmonics of smaller (m, n); of the same (m, n) before this one
    for (int j = 0; j < K; ++j) {
        const int kj = __shfl(key, j, 64);
        less += kj < key;
        eqb += (kj == key) & (j < lane);
    }
    const bool first = lane < K && eqb == 0;
    int rank = 0;   // distinct (m, n) below this one: the group index
    for (int j = 0; j < K; ++j) {
        const int kj = __shfl(key, j, 64);
        const int fj = __shfl(first ? 1 : 0, j, 64);
        rank += fj & (kj < key);
    }
    LocalGroups lg{};
    lg.on = true;
    lg.G = __popcll(__ballot(first));
    lg.mem = s_mem;
    if (b == 0) {
        Header* hdr = ws_at<Header>(W, L.header);
        if (first) {
            ws_at<int32_t>(W, L.gm)[rank] = m;
            ws_at<int32_t>(W, L.gn)[rank] = n;
            ws_at<int32_t>(W, L.gstart)[rank] = less;
        }
        if (lane < K) ws_at<int32_t>(W, L.gmem)[less + eqb] = lane;
        const bool anybad = __ballot(bad) != 0ull;
        if (lane == 0) {
            header_init(hdr);
            ws_at<int32_t>(W, L.gstart)[lg.G] = K;
            hdr->groups = lg.G;
            if (anybad) hdr->bad_mn = 1;
        }
        double2* sctab_g = ws_at<double2>(W, L.sctab);
        for (int i = lane; i < 512; i += 64) {
            double sv, cv;
            sincospi((double)i / 256.0, &sv, &cv);
            sctab_g[i] = make_double2(sv, cv);
        }
    }
    const int g = b < 4 ? -1 : b < 4 + K ? b - 4 : (b - 4 - K) >> 2;
    if (g >= 0 && g < lg.G) {
        const unsigned long long sel = __ballot(first && rank == g);
        const int src = __ffsll((long long)sel) - 1;
        lg.m = __shfl(m, src, 64);
        lg.n = __shfl(n, src, 64);
        const int kg = __shfl(key, src, 64);
        const bool mine = lane < K && key == kg;
        if (mine) s_mem[eqb] = lane;
        lg.count = __popcll(__ballot(mine));
    }
    __syncthreads();
    return lg;
}
__global__ __launch_bounds__(64) void k_prep_pcr_b(const PrepBatch B) {
    PREP_WALKER(B);
    if (!(D.pcr & 1) || (int)blockIdx.x >= 4 + ((D.pcr & 2) ? 5 : 1) * D.K) return;
    const GroupAmpSrc ga{D.amp, D.ylm_p, D.ylm_m, D.sc_re, D.sc_im,
                         ws_at<int32_t>(W, L.gstart), ws_at<int32_t>(W, L.gmem)};
    __shared__ int s_mem[PCR_GROUPS_MAX_K];
    LocalGroups lg{};
    if (B.pcr_groups && (blockIdx.x == 0 || blockIdx.x >= 4))   // (blocks 1-3: trajectory only)
        lg = pcr_local_groups(D, W, L, s_mem);
    prep_pcr_body(D.t, D.phi_phi, D.phi_r, D.f_phi, D.f_r, ga, lg, ws_at<int32_t>(W, L.gm),
                  ws_at<int32_t>(W, L.gn), D.nt, D.K,
                  ws_at<double>(W, L.coefT), ws_at<double>(W, L.kslope), ws_at<double>(W, L.coefA),
                  ws_at<int32_t>(W, L.runs), ws_at<Item>(W, L.items), ws_at<double>(W, L.invcp),
                  ws_at<double>(W, L.invdp), ws_at<Header>(W, L.header));
}

__global__ __launch_bounds__(64) void k_spline_shared(const double* __restrict__ x, int n,
                                                      const double* __restrict__ y, int ninterp,
                                                      double* coef, int64_t scratch_stride) {
    auto yf = [&](int i, int q) { return y[(size_t)i * ninterp + q]; };
    spline_shared(x, n, yf, ninterp, ninterp, coef, scratch_stride, blockIdx.x);
}

// ----------------------------------------------------------------------------------------
// K4: interval records. Lane ranges per sub-branch s over the "lane" index k of the output:
//   s = 0: g = -freq[k];  s = 1: g = +freq[k].
// The inverse interval (ascending) covers g in [x_lo, x_hi), open at the run's first knot
// (notebook supports are open: :569-570; scipy picks the interval x_r <= g < x_{r+1}).
// Paired (symmetric) grids restrict lanes to the non-positive half: s = 0 to [0, nl),
// s = 1 to [0, nl1) (nl1 excludes the f = 0 bin so it is counted once).
// ----------------------------------------------------------------------------------------
// First index with f[i] >= v (UPPER = false) or f[i] > v (UPPER = true) on the sorted grid.
// Starts from the linear-interpolation guess g (exact to +-1 bin on the uniform FEW grids) and
// gallops outward before bisecting, so a typical call reads 2-3 grid values instead of the
// ~23 dependent loads of a plain binary search over 6.3M bins.
template <bool UPPER>
__device__ int64_t grid_bound(const double* __restrict__ f, int64_t nf, double v, int64_t g) {
    auto pred = [&](int64_t i) { return UPPER ? (f[i] > v) : (f[i] >= v); };
    g = g < 0 ? 0 : (g > nf ? nf : g);
    int64_t lo, hi;   // answer in [lo, hi]
    if (g < nf && !pred(g)) {
        lo = g + 1;
        int64_t step = 1;
        while (true) {
            const int64_t p = lo + step - 1;
            if (p >= nf) { hi = nf; break; }
            if (pred(p)) { hi = p; break; }
            lo = p + 1;
            step <<= 1;
        }
    } else {
        hi = g;
        int64_t step = 1;
        while (true) {
            const int64_t p = hi - step;
            if (p < 0) { lo = 0; break; }
            if (pred(p)) { hi = p; step <<= 1; }
            else { lo = p + 1; break; }
        }
    }
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (pred(mid)) hi = mid; else lo = mid + 1;
    }
    return lo;
}

__device__ bool build_item(
    const double* __restrict__ t, const double* __restrict__ f_phi, const double* __restrict__ f_r,
    const int32_t* __restrict__ gm, const int32_t* __restrict__ gn, int ni, int K,
    const double* __restrict__ coefA, const double* __restrict__ coefT,
    const int32_t* __restrict__ runs, const double* __restrict__ freq, int64_t nf, int paired,
    int64_t nl, int64_t nl1, Item* __restrict__ items, int4* __restrict__ ranges, int h, int j,
    unsigned long long& evals, bool env);

// K4: one thread per (group g, knot interval j). Counts both the SPA evaluations the kernel
// makes (per group) and the reference formulation's contributions C (per (l, m, n) harmonic:
// the group's evaluations times its member count).
__device__ __forceinline__ void items_body(const double* __restrict__ t, const double* __restrict__ f_phi,
                        const double* __restrict__ f_r, const int32_t* __restrict__ gm,
                        const int32_t* __restrict__ gn, const int32_t* __restrict__ gstart,
                        int nt, int K, const double* __restrict__ coefA,
                        const double* __restrict__ coefT, const int32_t* __restrict__ runs,
                        const double* __restrict__ freq, int64_t nf, int paired, int64_t nl,
                        int64_t nl1, Item* __restrict__ items, int4* __restrict__ ranges,
                        Header* __restrict__ hdr, bool runs_mark, bool env) {
    const int ni = nt - 1;
    const int G = hdr->groups;
    // the grid is sized for K >= G groups (K / ITEMS_PER_THREAD_K threads per interval at large
    // K): whole blocks past the records leave at once; a thread takes the records gid, gid +
    // the grid's threads, ... (config 2: 627 groups over 377 threads an interval, one or two)
    const int64_t total = (int64_t)ni * G;
    if ((int64_t)blockIdx.x * blockDim.x >= total) return;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    __shared__ unsigned long long red[3][4];
    unsigned long long ev = 0, contrib = 0, eev = 0;
    for (int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; gid < total;
         gid += stride) {
        const int g = (int)(gid % G), j = (int)(gid / G);
        // the PCR inverse splines' run-overflow marker (rr[3]) into the header's sticky flag
        if (runs_mark && j == 0 && runs[(size_t)g * 4 * MAXRUNS + 3] != 0)
            atomicOr(&hdr->runs_overflow, 1);
        unsigned long long e1 = 0;
        const bool envr = build_item(t, f_phi, f_r, gm, gn, ni, K, coefA, coefT, runs, freq, nf,
                                     paired, nl, nl1, items, ranges, g, j, e1, env);
        ev += e1;
        contrib += e1 * (unsigned long long)(gstart[g + 1] - gstart[g]);
        eev += envr ? e1 : 0;
    }
    for (int o = 32; o > 0; o >>= 1) {
        ev += __shfl_xor(ev, o);
        contrib += __shfl_xor(contrib, o);
        eev += __shfl_xor(eev, o);
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = contrib;
        red[1][threadIdx.x >> 6] = ev;
        red[2][threadIdx.x >> 6] = eev;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long c = red[0][0] + red[0][1] + red[0][2] + red[0][3];
        const unsigned long long e = red[1][0] + red[1][1] + red[1][2] + red[1][3];
        const unsigned long long x = red[2][0] + red[2][1] + red[2][2] + red[2][3];
        if (c) atomicAdd((unsigned long long*)&hdr->contributions, c);
        if (e) atomicAdd((unsigned long long*)&hdr->evaluations, e);
        if (x) atomicAdd((unsigned long long*)&hdr->env_evaluations, x);
    }
}
__global__ __launch_bounds__(256) void k_items(const PrepBatch B) {
    PREP_WALKER(B);
    items_body(D.t, D.f_phi, D.f_r, ws_at<int32_t>(W, L.gm), ws_at<int32_t>(W, L.gn),
               ws_at<int32_t>(W, L.gstart), D.nt, D.K, ws_at<double>(W, L.coefA),
               ws_at<double>(W, L.coefT), ws_at<int32_t>(W, L.runs), D.freq, B.nf, B.paired, B.nl,
               B.nl1, ws_at<Item>(W, L.items), ws_at<int4>(W, L.ranges),
               ws_at<Header>(W, L.header), (D.pcr & 1) != 0, D.env != 0);
}

// One interval record of group h; `evals` = its (branch x bin) evaluation count.
// Certified records: a record whose every lane is known to pass the fast path's per-lane validity
// tests -- t(g) inside the record's knot interval and F' of the record's sign, nonzero -- skips
// them (Item::fdneg bit 1, header bit 25): one 64-bit compare and one class test per bin, with
// their ballots and mask arithmetic. Certified here on the device, with the kernel's own
// arithmetic: t(g) is monotonic over the record's g range (its derivative keeps one sign at the
// range's ends and at the derivative's vertex), w = t(g) - t_j at the range's end bins (bitwise
// the values k_modesum computes there) lies inside [0, dtj) with a 1e-6 dtj margin for the
// interior bins' rounding, and F' keeps the record's sign over the whole interval with a margin
// of 1e-12 of its terms. Fold and edge records (overshooting t(g), turning points) keep the
// tests; a safe record's lanes would all have passed them, so the spectrum is bitwise the same.
// FAT(x) = freq[x] (build_item serves the range ends from the grid values it already holds)
template <class FAT>
__device__ bool record_safe(const Item& it, FAT fat, int64_t lo0, int64_t hi0, int64_t lo1,
                            int64_t hi1) {
    // the g range of the lanes: s = 0 lanes k in [lo0, hi0) at g = -freq[k], s = 1 at +freq[k]
    double ga = INFINITY, gb = -INFINITY;
    if (hi0 > lo0) {
        const double fa = fat(0, lo0), fb = fat(1, hi0 - 1);
        ga = fmin(ga, fmin(-fa, -fb));
        gb = fmax(gb, fmax(-fa, -fb));
    }
    if (hi1 > lo1) {
        const double fa = fat(2, lo1), fb = fat(3, hi1 - 1);
        ga = fmin(ga, fmin(fa, fb));
        gb = fmax(gb, fmax(fa, fb));
    }
    if (!(ga <= gb)) return false;   // no lanes (or NaN)
    // the fast path's w at both ends (its exact operations)
    auto wat = [&](double g) {
        const double u = g - it.gx;
        const double tt = fma(fma(fma(it.ic[0], u, it.ic[1]), u, it.ic[2]), u, it.ic[3]);
        return tt - it.tj;
    };
    const double wa = wat(ga), wb = wat(gb);
    const double mg = 1e-6 * it.dtj;
    if (!(fmin(wa, wb) >= mg && fmax(wa, wb) <= it.dtj - mg)) return false;
    // monotonic t(u): t'(u) = 3 c0 u^2 + 2 c1 u + c2 of one sign at both ends and at its vertex
    const double ua = ga - it.gx, ub = gb - it.gx;
    auto dt = [&](double u) { return fma(fma(3.0 * it.ic[0], u, 2.0 * it.ic[1]), u, it.ic[2]); };
    const double da = dt(ua), db = dt(ub);
    if (!((da > 0.0 && db > 0.0) || (da < 0.0 && db < 0.0))) return false;
    if (it.ic[0] != 0.0) {
        const double uv = -it.ic[1] / (3.0 * it.ic[0]);
        if (uv > ua && uv < ub) {
            const double dv = dt(uv);
            if (!((dv > 0.0) == (da > 0.0) && dv != 0.0)) return false;
        }
    }
    // F'(w) = (fd0 w + fd1) w + fd2 of the record's sign on [0, dtj], away from 0
    const double* f = it.fd;
    const double scale = fabs(f[0]) * it.dtj * it.dtj + fabs(f[1]) * it.dtj + fabs(f[2]);
    const double sg = (it.fdneg & 1) ? -1.0 : 1.0;
    auto fq = [&](double x) { return sg * fma(fma(f[0], x, f[1]), x, f[2]); };
    double fmn = fmin(fq(0.0), fq(it.dtj));
    if (f[0] != 0.0) {
        const double xv = -f[1] / (2.0 * f[0]);
        if (xv > 0.0 && xv < it.dtj) fmn = fmin(fmn, fq(xv));
    }
    return fmn > 1e-12 * scale && isfinite(scale);
}

__device__ bool build_item(
    const double* __restrict__ t, const double* __restrict__ f_phi, const double* __restrict__ f_r,
    const int32_t* __restrict__ gm, const int32_t* __restrict__ gn, int ni, int K,
    const double* __restrict__ coefA, const double* __restrict__ coefT,
    const int32_t* __restrict__ runs, const double* __restrict__ freq, int64_t nf, int paired,
    int64_t nl, int64_t nl1, Item* __restrict__ items, int4* __restrict__ ranges, int h, int j,
    unsigned long long& evals, bool env) {
    Item& it = items[(size_t)h * ni + j];
    const int m = gm[h], n = gn[h];
    const int32_t* rr = runs + (size_t)h * 4 * MAXRUNS;
    int run = -1;
    for (int r = 0; r < MAXRUNS; ++r) {
        if (rr[4 * r + 2] != 0 && j >= rr[4 * r] && j < rr[4 * r + 1]) { run = r; break; }
    }
    const int partner = (m != 0) ? 1 : 0;
    evals = 0;
    it.fdneg = 0;
    if (run < 0) {  // flat interval (F_{j+1} == F_j): no support; place empty ranges at 0
        it.klo[0] = it.khi[0] = it.klo[1] = it.khi[1] = 0;
        ranges[(size_t)h * ni + j] = make_int4(0, 0, 0, 0);
        return false;
    }
    const int a = rr[4 * run], sg = rr[4 * run + 2];
    it.tj = t[j];
    it.dtj = t[j + 1] - t[j];
    const double dm = (double)m, dn = (double)n;
    for (int c = 0; c < 4; ++c) {
        const double* ca = coefA + ((size_t)j * 4 + c) * 4 * K + 4 * h;
        it.b[0][0][c] = ca[0];   // Bp re
        it.b[0][1][c] = ca[1];   // Bp im
        it.b[1][0][c] = ca[2];   // Bm re
        it.b[1][1][c] = ca[3];   // Bm im
        const double* ct = coefT + ((size_t)j * 4 + c) * 8;
        it.ph[c] = dm * ct[0] + dn * ct[1];
    }
    // F' = derivative of (m f_phi + n f_r) piece; F'' = derivative of (m f_phi' + n f_r') piece
    double gq[3], ymin_rec;   // F'' quadratic (unscaled) and the |y| bound, for the envelope
    {
        const double* ct = coefT + (size_t)j * 32;
        const double F0 = dm * ct[0 * 8 + 2] + dn * ct[0 * 8 + 3];
        const double F1 = dm * ct[1 * 8 + 2] + dn * ct[1 * 8 + 3];
        const double F2 = dm * ct[2 * 8 + 2] + dn * ct[2 * 8 + 3];
        it.fd[0] = 3.0 * F0; it.fd[1] = 2.0 * F1; it.fd[2] = F2;
        const double G0 = dm * ct[0 * 8 + 4] + dn * ct[0 * 8 + 5];
        const double G1 = dm * ct[1 * 8 + 4] + dn * ct[1 * 8 + 5];
        const double G2 = dm * ct[2 * 8 + 4] + dn * ct[2 * 8 + 5];
        // pre-scaled so the fast path's w = 3 F''^2 / (2 pi |F'|^3) is one square
        it.fdd[0] = FDD_SCALE * (3.0 * G0);
        it.fdd[1] = FDD_SCALE * (2.0 * G1);
        it.fdd[2] = FDD_SCALE * G2;
        // lower bound of |y| = 2 pi |F'|^3 / (3 F''^2) over w in [0, dtj]: min |F'| and max |F''|
        // of the two quadratics from their end points and vertices (F' changing sign -> 0)
        const double dt = it.dtj;
        auto qv = [](double a, double b, double c, double x) { return (a * x + b) * x + c; };
        const double fa = it.fd[2], fb = qv(it.fd[0], it.fd[1], it.fd[2], dt);
        it.fdneg = qv(it.fd[0], it.fd[1], it.fd[2], 0.5 * dt) < 0.0 ? 1 : 0;
        double fdmin = fmin(fabs(fa), fabs(fb));
        if ((fa > 0.0) != (fb > 0.0) || fa == 0.0 || fb == 0.0) fdmin = 0.0;
        if (it.fd[0] != 0.0) {
            const double xv = -it.fd[1] / (2.0 * it.fd[0]);
            if (xv > 0.0 && xv < dt) {
                const double fv = qv(it.fd[0], it.fd[1], it.fd[2], xv);
                if ((fv > 0.0) != (fa > 0.0)) fdmin = 0.0;
                fdmin = fmin(fdmin, fabs(fv));
            }
        }
        double gmax = fmax(fabs(G2), fabs(qv(3.0 * G0, 2.0 * G1, G2, dt)));
        if (G0 != 0.0) {
            const double xv = -(2.0 * G1) / (6.0 * G0);
            if (xv > 0.0 && xv < dt) gmax = fmax(gmax, fabs(qv(3.0 * G0, 2.0 * G1, G2, xv)));
        }
        // 10% margin for the rounding of both bounds and of the kernel's own evaluation
        const double ymin = gmax > 0.0 ? TWO_PI * fdmin * fdmin * fdmin / (3.0 * gmax * gmax) / 1.1
                                       : INFINITY;
        int J = FAST_J;
        for (int jj = 1; jj < FAST_J; ++jj)
            if (ymin >= JSER_Y[jj]) { J = jj; break; }
        it.jser = J;
        gq[0] = 3.0 * G0; gq[1] = 2.0 * G1; gq[2] = G2;
        ymin_rec = ymin;
    }
    // g-interval of this record: [x_lo, x_hi), lower end open at the run's first knot
    const double Fj = knotF(f_phi, f_r, m, n, j), Fj1 = knotF(f_phi, f_r, m, n, j + 1);
    const double xlo = sg > 0 ? Fj : Fj1;
    const double xhi = sg > 0 ? Fj1 : Fj;
    const bool strict_lo = sg > 0 ? (j == a) : (j + 1 == rr[4 * run + 1]);
    // linear-interpolation guess of the grid index of a frequency value
    const double f0 = freq[0], span = freq[nf - 1] - f0;
    const double gsc = span > 0.0 ? (double)(nf - 1) / span : 0.0;
    auto guess = [&](double v) { return (int64_t)floor((v - f0) * gsc); };
    // s = 0: g = -f  ->  f in (-xhi, -xlo]  (or (-xhi, -xlo) if strict)
    // s = 1: g = +f  ->  f in [xlo, xhi)  (or (xlo, xhi))
    // The four bounds' grid values around their guesses are loaded together (one round trip
    // instead of the ~2 dependent ones of each grid_bound in turn); a bound the three values do
    // not settle (a non-uniform grid) takes grid_bound. Same indices either way.
    const double bv[4] = {-xhi, -xlo, xlo, xhi};
    const bool bu[4] = {true, !strict_lo, strict_lo, false};   // UPPER: first f > v, else f >= v
    int64_t bg[4];
    double b3[4][3];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t g = guess(bv[q]);
        bg[q] = g < 0 ? 0 : (g > nf ? nf : g);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t g = bg[q];
        b3[q][0] = freq[g >= 1 ? g - 1 : 0];
        b3[q][1] = freq[g < nf ? g : nf - 1];
        b3[q][2] = freq[g + 1 < nf ? g + 1 : nf - 1];
    }
    int64_t bk[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const double v = bv[q];
        const int64_t g = bg[q];
        auto pred = [&](double x) { return bu[q] ? (x > v) : (x >= v); };
        int64_t k = -1;
        if (!(g >= 1 && pred(b3[q][0]))) {           // f[g - 1] fails: the answer is >= g
            if (g == nf) k = nf;
            else if (pred(b3[q][1])) k = g;
            else if (g + 1 == nf) k = nf;
            else if (pred(b3[q][2])) k = g + 1;
        }
        if (k < 0)
            k = bu[q] ? grid_bound<true>(freq, nf, v, g) : grid_bound<false>(freq, nf, v, g);
        bk[q] = k;
    }
    int64_t lo0 = bk[0], hi0 = bk[1], lo1 = bk[2], hi1 = bk[3];
    const int64_t lim0 = paired ? nl : nf;
    const int64_t lim1 = paired ? nl1 : (partner ? nf : 0);
    auto clampr = [](int64_t& lo, int64_t& hi, int64_t lim) {
        if (lo > lim) lo = lim;
        if (hi > lim) hi = lim;
        if (hi < lo) hi = lo;
    };
    clampr(lo0, hi0, lim0);
    clampr(lo1, hi1, lim1);
    it.klo[0] = (int32_t)lo0; it.khi[0] = (int32_t)hi0;
    it.klo[1] = (int32_t)lo1; it.khi[1] = (int32_t)hi1;
    ranges[(size_t)h * ni + j] = make_int4((int)lo0, (int)hi0, (int)lo1, (int)hi1);
    // freq[x] for a range end x: from bound q's three grid values when x is one of them (the
    // usual case: an end is its bound's answer or the index before), else loaded
    auto fat = [&](int q, int64_t x) {
        const int64_t g = bg[q];
        if (g >= 1 && x == g - 1) return b3[q][0];
        if (g < nf && x == g) return b3[q][1];
        if (g + 1 < nf && x == g + 1) return b3[q][2];
        return freq[x];
    };
    if (record_safe(it, fat, lo0, hi0, lo1, hi1)) it.fdneg |= 2;
    // branch x bin evaluations (on a paired grid one lane serves both the branch and its partner)
    const int mult = paired ? 1 + partner : 1;
    evals = (unsigned long long)((hi0 - lo0) + (hi1 - lo1)) * mult;
    // envelope record (env_fit.inc): a certified-safe record with |y| >= ENV_MIN_Y everywhere
    // whose A(w) and theta(w) polynomials pass the check; its F' / F'' / dtj slots then hold
    // A's coefficients, its phase cubic Phi - theta, and jser = 0 marks it for the sum
    if (env && (it.fdneg & 2) && ymin_rec >= ENV_MIN_Y && evals > 0) {
        EnvFit E;
        if (env_fit(it.fd, gq, it.dtj, (it.fdneg & 1) != 0, E)) {
            // A's coefficients times the cosine polynomial's constant (sincos_tab_amp's cos r =
            // COS_A - r^2/2 then costs one FMA on the scaled amplitude)
            double* e = env_of(&it);
            for (int c = 0; c <= ENV_DEG; ++c) e[c] = E.a[c] * ENV_AMP_SCALE;
            for (int c = 0; c < 4; ++c) it.ph[c] -= E.th[c];
            it.jser = 0;   // the sum's envelope class
            return true;
        }
    }
    return false;
}

// ----------------------------------------------------------------------------------------
// K5: segment table. A segment is (group, monotonic run, sub-branch s) with a non-empty lane
// range; its interval records are consecutive (h * ni + j, j in [ja, jb)) and, walked in lane
// order (j += dir), cover consecutive, disjoint lane ranges. K5a: one thread per (h, run, s)
// slot writes the slot's segment (or an empty marker) into a dense table plus a per-block count;
// K5b compacts the non-empty slots in slot order (block offsets from the counts), so the table
// is deterministic.
// seglh = (lo, hi) lane range; seginfo = (first record, count, dir, s).
// ----------------------------------------------------------------------------------------
// The segment of slot i = (group h, run r, sub-branch sb): its lane range lh and (first record,
// count, dir, s) info, or info.y == 0 when the slot holds none. G = the call's group count.
__device__ __forceinline__ void slot_segment(int i, const int32_t* __restrict__ runs,
                                             const int4* __restrict__ ranges, int nt, int G,
                                             int lim0, int lim1, int2& lh, int4& info) {
    const int h = i / (2 * MAXRUNS), r = (i >> 1) % MAXRUNS, sb = i & 1;
    const int ni = nt - 1;
    lh = make_int2(0, 0);
    info = make_int4(0, 0, 0, 0);
    const int32_t* rr = runs + (size_t)h * 4 * MAXRUNS + 4 * r;
    if (h < G && rr[2] != 0) {
        const int ja = rr[0], jb = rr[1], n = jb - ja;
        const int dir = (sb == 0) ? -rr[2] : rr[2];   // s = 0 walks g downward in lane order
        const int lim = sb ? lim1 : lim0;
        const int4* rg = ranges + (size_t)h * ni;
        // Records whose branch lies outside the lane range are empty and clamped to its
        // ends (lane 0 or lim); they sit at the two ends of the segment in lane order and
        // are trimmed, so the tiles holding lane 0 and lim do not collect all of them.
        int lo = 0, hi = n;                            // first p with khi > 0
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            const int4 v = rg[dir > 0 ? ja + mid : jb - 1 - mid];
            if ((sb ? v.w : v.y) > 0) hi = mid; else lo = mid + 1;
        }
        const int pa = lo;
        hi = n;                                        // first p with klo >= lim
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            const int4 v = rg[dir > 0 ? ja + mid : jb - 1 - mid];
            if ((sb ? v.z : v.x) >= lim) hi = mid; else lo = mid + 1;
        }
        const int pb = lo;
        if (pb > pa) {
            const int4 rf = rg[dir > 0 ? ja + pa : jb - 1 - pa];
            const int4 rl = rg[dir > 0 ? ja + pb - 1 : jb - pb];
            const int klo = sb ? rf.z : rf.x, khi = sb ? rl.w : rl.y;
            if (khi > klo) {
                lh = make_int2(klo, khi);
                const int jfirst = dir > 0 ? ja + pa : jb - pb;   // lowest record index kept
                info = make_int4(h * ni + jfirst, pb - pa, dir, sb);
            }
        }
    }
}
__device__ __forceinline__ void segment_slots_body(const int32_t* __restrict__ runs,
                                                       const int4* __restrict__ ranges, int nt,
                                                       int K, int lim0, int lim1,
                                                       const Header* __restrict__ hdr,
                                                       int2* __restrict__ slot_lh,
                                                       int4* __restrict__ slot_info,
                                                       int32_t* __restrict__ blockcnt,
                                                       int32_t* __restrict__ blocktiles) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    __shared__ int wc[4], wt[4];
    int ntl = 0;   // tiles the slot's segment covers
    bool valid = false;
    if (i < K * MAXRUNS * 2) {
        const int G = hdr->groups;
        int2 lh;
        int4 info;
        slot_segment(i, runs, ranges, nt, G, lim0, lim1, lh, info);
        slot_lh[i] = lh;
        slot_info[i] = info;
        valid = info.y > 0;
        if (valid) ntl = (lh.y - 1) / TILE_LANES - lh.x / TILE_LANES + 1;
    }
    const unsigned long long bal = __ballot(valid);
    int tsum = ntl;
    for (int o = 32; o > 0; o >>= 1) tsum += __shfl_xor(tsum, o);
    if ((threadIdx.x & 63) == 0) {
        wc[threadIdx.x >> 6] = __popcll(bal);
        wt[threadIdx.x >> 6] = tsum;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        blockcnt[blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
        blocktiles[blockIdx.x] = wt[0] + wt[1] + wt[2] + wt[3];
    }
}
// slot blocks of one waveform: (2 MAXRUNS K + 255) / 256; the grid has the batch's largest count
__device__ __forceinline__ int slot_blocks(int K) { return (2 * MAXRUNS * K + 255) / 256; }
__global__ __launch_bounds__(256) void k_segment_slots(const PrepBatch B) {
    PREP_WALKER(B);
    if ((int)blockIdx.x >= slot_blocks(D.K)) return;
    segment_slots_body(ws_at<int32_t>(W, L.runs), ws_at<int4>(W, L.ranges), D.nt, D.K,
                       (int)(B.paired ? B.nl : B.nf), (int)(B.paired ? B.nl1 : B.nf),
                       ws_at<Header>(W, L.header), ws_at<int2>(W, L.slotlh),
                       ws_at<int4>(W, L.slotinfo), ws_at<int32_t>(W, L.slotcnt),
                       ws_at<int32_t>(W, L.slottiles));
}

// one workgroup per slot block: its output offset is the sum of the earlier blocks' counts
// Segment-tile boundaries: segment s covers tiles [t0, t1] (t0 = lo / TILE_LANES); its
// (p0, p1) pairs for those tiles sit at stb[toff(s) .. toff(s) + t1 - t0] in compacted segment
// order, and segbase[s] = toff(s) - t0 (so the pair of tile t is stb[segbase[s] + t]), or
// SEG_NO_STB when the pairs would pass the capacity (that segment keeps the bisection).
constexpr int32_t SEG_NO_STB = INT32_MIN;
__device__ __forceinline__ void segment_compact_body(const int2* __restrict__ slot_lh,
                                                         const int4* __restrict__ slot_info,
                                                         const int32_t* __restrict__ blockcnt,
                                                         const int32_t* __restrict__ blocktiles,
                                                         int nslot, int64_t stbcap,
                                                         int2* __restrict__ seglh,
                                                         int4* __restrict__ seginfo,
                                                         int32_t* __restrict__ segbase,
                                                         int32_t* __restrict__ nseg, int nblk,
                                                         Header* __restrict__ hdr) {
    __shared__ int wc[4];
    __shared__ int64_t wt[4];
    __shared__ int2 wr[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int blk = blockIdx.x;
    int before = 0;
    int64_t tbefore = 0;
    for (int b = tid; b < blk; b += 256) { before += blockcnt[b]; tbefore += blocktiles[b]; }
    for (int o = 32; o > 0; o >>= 1) {
        before += __shfl_xor(before, o);
        tbefore += __shfl_xor(tbefore, o);
    }
    if (lane == 0) { wc[wave] = before; wt[wave] = tbefore; }
    __syncthreads();
    const int base = wc[0] + wc[1] + wc[2] + wc[3];
    const int64_t tbase = wt[0] + wt[1] + wt[2] + wt[3];
    __syncthreads();
    const int i = blk * 256 + tid;
    int4 info = make_int4(0, 0, 0, 0);
    int2 lh = make_int2(0, 0);
    if (i < nslot) { info = slot_info[i]; lh = slot_lh[i]; }
    const bool valid = info.y > 0;
    const int ntl = valid ? (lh.y - 1) / TILE_LANES - lh.x / TILE_LANES + 1 : 0;
    // exclusive scan of the tile counts over the block's slots (slot order)
    int incl = ntl;
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    const unsigned long long bal = __ballot(valid);
    if (lane == 63) wt[wave] = incl;
    if (lane == 0) wc[wave] = __popcll(bal);
    __syncthreads();
    int pos = base;
    int64_t toff = tbase + incl - ntl;
    for (int w = 0; w < wave; ++w) { pos += wc[w]; toff += wt[w]; }
    pos += __popcll(bal & ((1ull << lane) - 1ull));
    if (valid) {
        seglh[pos] = lh;
        seginfo[pos] = info;
        segbase[pos] = (toff + ntl <= stbcap) ? (int32_t)(toff - lh.x / TILE_LANES)
                                                         : SEG_NO_STB;
    }
    if (blk == nblk - 1 && tid == 0) *nseg = base + wc[0] + wc[1] + wc[2] + wc[3];
    // the union of the block's segment lane ranges into the header: k_modesum's tiles outside
    // it skip the list build (one block-wide min / max, two global atomics per block)
    int lo = valid ? lh.x : INT32_MAX, hi = valid ? lh.y : INT32_MIN;
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, __shfl_xor(lo, o));
        hi = max(hi, __shfl_xor(hi, o));
    }
    if (lane == 0) wr[wave] = make_int2(lo, hi);
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < 4; ++w) { lo = min(lo, wr[w].x); hi = max(hi, wr[w].y); }
        if (lo < hi) {
            atomicMin(&hdr->lane_lo, lo);
            atomicMax(&hdr->lane_hi, hi);
        }
    }
}
__global__ __launch_bounds__(256) void k_segment_compact(const PrepBatch B) {
    PREP_WALKER(B);
    const int nblk = slot_blocks(D.K);
    if ((int)blockIdx.x >= nblk) return;
    segment_compact_body(ws_at<int2>(W, L.slotlh), ws_at<int4>(W, L.slotinfo),
                         ws_at<int32_t>(W, L.slotcnt), ws_at<int32_t>(W, L.slottiles),
                         2 * MAXRUNS * D.K, L.stbcap, ws_at<int2>(W, L.seglh),
                         ws_at<int4>(W, L.seginfo), ws_at<int32_t>(W, L.segbase),
                         ws_at<int32_t>(W, L.nseg), nblk, ws_at<Header>(W, L.header));
}

// One workgroup per segment (grid-stride): for every record p of the segment in lane order
// (and the end marker p = n), the tiles t of [t0, t1] whose first record reaching them is p
// (p0(t) = first p with khi > t*TL) and whose first record past them is p (p1(t) = first p with
// klo >= (t+1)*TL). Lane ranges are monotone in p, so each tile gets exactly one of each: the
// same answers as k_modesum's bisection, from two loads instead of ~2 log2(n) dependent ones.
__device__ __forceinline__ int div_floor_nn(int64_t a) { return (int)(a / TILE_LANES); }   // a >= 0
// record p (0 <= p <= n: n is the end marker) of the segment (lh, info) with pair base sbase
__device__ __forceinline__ void seg_tiles_record(const int4* __restrict__ ranges, int2 lh,
                                                 int4 info, int32_t sbase, int p,
                                                 int32_t* __restrict__ stb0,
                                                 int32_t* __restrict__ stb1) {
    const int base = info.x, n = info.y, dir = info.z, sb = info.w;
    const int t0 = lh.x / TILE_LANES, t1 = (lh.y - 1) / TILE_LANES;
    auto rng = [&](int q) {   // (klo, khi) of record q in lane order
        const int4 rg = ranges[base + (dir > 0 ? q : n - 1 - q)];
        return sb ? make_int2(rg.z, rg.w) : make_int2(rg.x, rg.y);
    };
    const int2 cur = p < n ? rng(p) : make_int2(0, 0);
    const int2 prv = p > 0 ? rng(p - 1) : make_int2(0, 0);
    // p0: khi_{p-1} <= t TL < khi_p
    int a = p > 0 ? (int)((prv.y + TILE_LANES - 1) / TILE_LANES) : t0;
    int b = p < n ? (cur.y > 0 ? div_floor_nn(cur.y - 1) : -1) : t1;
    for (int t = max(a, t0); t <= min(b, t1); ++t) stb0[sbase + t] = p;
    // p1: klo_{p-1} < (t+1) TL <= klo_p
    a = p > 0 ? div_floor_nn(prv.x) : t0;
    b = p < n ? div_floor_nn(cur.x) - 1 : t1;
    for (int t = max(a, t0); t <= min(b, t1); ++t) stb1[sbase + t] = p;
}
__device__ __forceinline__ void seg_tiles_body(const int4* __restrict__ ranges,
                                                   const int2* __restrict__ seglh,
                                                   const int4* __restrict__ seginfo,
                                                   const int32_t* __restrict__ segbase,
                                                   const int32_t* __restrict__ nsegp,
                                                   int32_t* __restrict__ stb0,
                                                   int32_t* __restrict__ stb1) {
    const int nseg = *nsegp;
    for (int sg = blockIdx.x; sg < nseg; sg += gridDim.x) {
        const int32_t sbase = segbase[sg];
        if (sbase == SEG_NO_STB) continue;
        const int2 lh = seglh[sg];
        const int4 info = seginfo[sg];
        for (int p = threadIdx.x; p <= info.y; p += blockDim.x)
            seg_tiles_record(ranges, lh, info, sbase, p, stb0, stb1);
    }
}
__global__ __launch_bounds__(256) void k_seg_tiles(const PrepBatch B) {
    PREP_WALKER(B);
    seg_tiles_body(ws_at<int4>(W, L.ranges), ws_at<int2>(W, L.seglh), ws_at<int4>(W, L.seginfo),
                   ws_at<int32_t>(W, L.segbase), ws_at<int32_t>(W, L.nseg),
                   ws_at<int32_t>(W, L.stb0), ws_at<int32_t>(W, L.stb1));
}

// K5 in one workgroup per waveform when its 2 MAXRUNS K slots fit one (K <= 64: the walker
// batches' sparse spectra): the slots' segments, their compaction in slot order (block scans in
// place of k_segment_compact's per-block offsets), the lane union, then the tile pairs of every
// (segment, record) (k_seg_tiles' work flattened over the workgroup: a record's segment found by
// bisection of the segments' record offsets in LDS). The same tables as the three kernels, in
// one launch instead of three.
constexpr int64_t SEG1_LDS_CAP = 40 * 1024;   // bytes of staged ranges (+ 33 KB static LDS)
__device__ __forceinline__ int seg1_excl_scan(int v, int* wsum, int& total) {
    constexpr int NW = SEG1_NT / 64;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int incl = v;
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(incl, o, 64);
        if (lane >= o) incl += u;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int before = 0;
    total = 0;
    for (int w = 0; w < NW; ++w) {
        const int x = wsum[w];
        if (w < wave) before += x;
        total += x;
    }
    __syncthreads();   // wsum free for the next scan
    return before + incl - v;
}
__global__ __launch_bounds__(SEG1_NT) void k_segments_one(const PrepBatch B) {
    PREP_WALKER(B);
    constexpr int NW = SEG1_NT / 64;
    __shared__ int wsum[NW];
    __shared__ int2 wr[NW];
    __shared__ int2 s_lh[SEG1_NT];
    __shared__ int4 s_info[SEG1_NT];
    __shared__ int32_t s_base[SEG1_NT];
    __shared__ int32_t s_roff[SEG1_NT];
    Header* hdr = ws_at<Header>(W, L.header);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nslot = 2 * MAXRUNS * D.K;   // <= SEG1_NT (host: every waveform has K <= SEG1_MAX_K)
    // the interval records' lane ranges staged in LDS when they fit (one coalesced pass): the
    // slots' bisections and the tile pairs then read LDS instead of chains of global loads
    extern __shared__ int4 s_rg[];
    const int ni = D.nt - 1;
    const int4* ranges = ws_at<int4>(W, L.ranges);
    if ((int64_t)D.K * ni * (int64_t)sizeof(int4) <= (int64_t)B.seg_lds) {
        const int nrec = hdr->groups * ni;
        for (int i = tid; i < nrec; i += SEG1_NT) s_rg[i] = ranges[i];
        __syncthreads();
        ranges = s_rg;
    }
    int2 lh = make_int2(0, 0);
    int4 info = make_int4(0, 0, 0, 0);
    if (tid < nslot)
        slot_segment(tid, ws_at<int32_t>(W, L.runs), ranges, D.nt, hdr->groups,
                     (int)(B.paired ? B.nl : B.nf), (int)(B.paired ? B.nl1 : B.nf), lh, info);
    const bool valid = info.y > 0;
    const int ntl = valid ? (lh.y - 1) / TILE_LANES - lh.x / TILE_LANES + 1 : 0;
    int nseg, ntot;
    const int pos = seg1_excl_scan(valid ? 1 : 0, wsum, nseg);
    const int toff = seg1_excl_scan(ntl, wsum, ntot);
    int32_t sbase = SEG_NO_STB;
    if (valid) {
        sbase = ((int64_t)toff + ntl <= L.stbcap) ? (int32_t)(toff - lh.x / TILE_LANES)
                                                  : SEG_NO_STB;
        ws_at<int2>(W, L.seglh)[pos] = lh;
        ws_at<int4>(W, L.seginfo)[pos] = info;
        ws_at<int32_t>(W, L.segbase)[pos] = sbase;
        s_lh[pos] = lh;
        s_info[pos] = info;
        s_base[pos] = sbase;
    }
    int nrec_all;
    const int nrec = (valid && sbase != SEG_NO_STB) ? info.y + 1 : 0;
    const int roff = seg1_excl_scan(nrec, wsum, nrec_all);
    if (valid) s_roff[pos] = roff;
    // the lane union (k_segment_compact's, one workgroup: no atomics)
    int lo = valid ? lh.x : INT32_MAX, hi = valid ? lh.y : INT32_MIN;
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, __shfl_xor(lo, o));
        hi = max(hi, __shfl_xor(hi, o));
    }
    if (lane == 0) wr[wave] = make_int2(lo, hi);
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < NW; ++w) { lo = min(lo, wr[w].x); hi = max(hi, wr[w].y); }
        if (lo < hi) {
            hdr->lane_lo = lo;
            hdr->lane_hi = hi;
        }
        *ws_at<int32_t>(W, L.nseg) = nseg;
    }
    int32_t* stb0 = ws_at<int32_t>(W, L.stb0);
    int32_t* stb1 = ws_at<int32_t>(W, L.stb1);
    // the sparse sum's split plan (paired grids, i.e. the fused likelihood): every union tile's
    // cost in wave-records, from the same (segment, record) pairs. Possible when the union fits
    // SPLIT_UNION_CAP tiles and every segment has its tile pairs (else nitems stays -1)
    __shared__ int s_cost[SPLIT_UNION_CAP];
    __syncthreads();   // wr[] (the union) is complete
    int ulo = INT32_MAX, uhi = INT32_MIN;
    for (int w = 0; w < NW; ++w) { ulo = min(ulo, wr[w].x); uhi = max(uhi, wr[w].y); }
    const int ut0 = ulo < uhi ? ulo / TILE_LANES : 0;
    const int nut = ulo < uhi ? (uhi - 1) / TILE_LANES - ut0 + 1 : 0;
    const bool plan = B.paired && nut > 0 && nut <= SPLIT_UNION_CAP &&
                      !__syncthreads_or(valid && sbase == SEG_NO_STB);
    if (plan)
        for (int i = tid; i < nut; i += SEG1_NT) s_cost[i] = 0;
    __syncthreads();
    for (int f = tid; f < nrec_all; f += SEG1_NT) {
        int a = 0, b = nseg - 1;   // the last segment q with s_roff[q] <= f
        while (a < b) {
            const int mid = (a + b + 1) >> 1;
            if (s_roff[mid] <= f) a = mid; else b = mid - 1;
        }
        const int p = f - s_roff[a];
        seg_tiles_record(ranges, s_lh[a], s_info[a], s_base[a], p, stb0, stb1);
        if (plan && p < s_info[a].y) {
            // record p's cost per tile it reaches: the 64 BPL-lane wave chunks it touches there
            // (modesum_tile evaluates a record on every wave whose bins it reaches)
            const int4 in = s_info[a];
            const int4 rg = ranges[in.x + (in.z > 0 ? p : in.y - 1 - p)];
            const int klo = in.w ? rg.z : rg.x, khi = in.w ? rg.w : rg.y;
            if (khi > klo) {
                constexpr int WL = 64 * BPL;
                for (int t = klo / TILE_LANES; t <= (khi - 1) / TILE_LANES; ++t) {
                    const int a0 = max(klo, t * TILE_LANES), b0 = min(khi, (t + 1) * TILE_LANES);
                    atomicAdd(&s_cost[t - ut0], (b0 - 1) / WL - a0 / WL + 1);
                }
            }
        }
    }
    if (!plan) return;
    __syncthreads();
    // each thread takes SPLIT_UNION_CAP / SEG1_NT consecutive union tiles
    constexpr int PER = SPLIT_UNION_CAP / SEG1_NT;
    int64_t csum = 0;
    for (int i = 0; i < PER; ++i) {
        const int u = tid * PER + i;
        csum += u < nut ? s_cost[u] : 0;
    }
    for (int o = 32; o > 0; o >>= 1) csum += __shfl_xor(csum, o);
    __shared__ int64_t s_csum[NW];
    if (lane == 0) s_csum[wave] = csum;
    __syncthreads();
    int64_t total = 0;
    for (int w = 0; w < NW; ++w) total += s_csum[w];
    // the fair share of one workgroup: the waveform's cost over SPLIT_SLOTS_PER_WF workgroups
    // (a walker group of 16 then fills the chip's ~1,024 resident slots); a tile above it (and
    // above B.split_min) is split into its BPL bins
    const int64_t share = max((int64_t)B.split_min, total / SPLIT_SLOTS_PER_WF);
    int nS[PER];
    int my_items = 0, my_split = 0;
    for (int i = 0; i < PER; ++i) {
        const int u = tid * PER + i;
        const int S = (u < nut && s_cost[u] > share) ? BPL : 1;
        nS[i] = u < nut ? S : 0;
        my_items += nS[i];
        my_split += S > 1 ? 1 : 0;
    }
    // no tile above the share (config 4's full grid: costs within 1.5x of the median): no plan,
    // and none of the scans below
    if (!__syncthreads_or(my_split > 0)) return;
    int n_items, n_split;
    const int io = seg1_excl_scan(my_items, wsum, n_items);
    const int po = seg1_excl_scan(my_split, wsum, n_split);
    if (n_split == 0 || n_items > SPLIT_ITEM_CAP || n_split > SPLIT_TILE_CAP)
        return;   // nothing to split, or past the plan's capacity: the plain tile loop
    int4* items = ws_at<int4>(W, L.sitem);
    int32_t* cnt = ws_at<int32_t>(W, L.scnt);
    int ii = io, sp = po;
    for (int i = 0; i < PER; ++i) {
        const int u = tid * PER + i, S = nS[i];
        for (int j = 0; j < S; ++j)
            items[ii + j] = make_int4(ut0 + u, (j << 16) | S, S > 1 ? sp : -1, S > 1 ? sp : -1);
        if (S > 1) {
            cnt[sp] = 0;
            ++sp;
        }
        ii += S;
    }
    if (tid == 0) {
        hdr->nitems = n_items;
        hdr->nsplit = n_split;
    }
}

// ----------------------------------------------------------------------------------------
// SPA arithmetic
// ----------------------------------------------------------------------------------------

// sin/cos of a phase up to |x| ~ 1e9 rad: two-term FMA Cody-Waite reduction by pi/2 (the
// third term, q * 1.5e-33, is below half an ulp of r for |q| < 2^31) and fdlibm's kernel
// polynomials on [-pi/4, pi/4]. The quadrant is applied with a select (odd q swaps sin/cos)
// and sign-bit flips, all branch-free.
__device__ __forceinline__ double flip_sign_if(double v, int flip_bit_2) {
    // flip_bit_2 is 0 or 2: moves to bit 63
    return __longlong_as_double(__double_as_longlong(v) ^
                                ((unsigned long long)(unsigned)flip_bit_2 << 62));
}
__device__ __forceinline__ void sincos_big(double x, double& s, double& c) {
    constexpr double INV_PIO2 = 6.36619772367581382433e-01;
    constexpr double PIO2_1 = 1.57079632679489655800e+00;   // first 53 bits of pi/2
    constexpr double PIO2_2 = 6.12323399573676603587e-17;   // pi/2 - PIO2_1
    const double q = rint(x * INV_PIO2);
    double r = fma(-q, PIO2_1, x);
    r = fma(-q, PIO2_2, r);
    const int iq = (int)q;
    const double z = r * r;
    // fdlibm __kernel_sin / __kernel_cos coefficients
    const double ps = fma(z, fma(z, fma(z, fma(z, fma(z, 1.58969099521155010221e-10,
                       -2.50507602534068634195e-08), 2.75573137070700676789e-06),
                       -1.98412698298579493134e-04), 8.33333333332248946124e-03),
                       -1.66666666666666324348e-01);
    const double sr = fma(r * z, ps, r);
    const double pc = fma(z, fma(z, fma(z, fma(z, fma(z, -1.13596475577881948265e-11,
                       2.08757232129817482790e-09), -2.75573143513906633035e-07),
                       2.48015872894767294178e-05), -1.38888888888741095749e-03),
                       4.16666666666666019037e-02);
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    const double cr = w + (((1.0 - w) - hz) + z * z * pc);
    const bool odd = (iq & 1) != 0;
    s = flip_sign_if(odd ? cr : sr, iq & 2);
    c = flip_sign_if(odd ? sr : cr, (iq + 1) & 2);
}

// sin/cos for the fast path: reduce by pi/256 against a 512-entry table of
// (sin, cos)(k pi/256) held in LDS, then short Taylor polynomials on |r| <= pi/512 (sin to r^3:
// truncation r^5/120 < 7.4e-14, far below the ~1e-9 rad rounding of phases that reach 1e7 rad;
// cos to r^4: < 1e-16) and the angle-sum formula: ~13 FP64 operations
// instead of ~26 plus the quadrant logic of sincos_big. `shift` (an integer number of table
// steps) is added to the angle exactly, through the table index. Valid for |x| < 2^31 pi/256.
// The reduction is one FMA against the leading 53 bits of the step: the dropped q * STEP_2 is
// < 3.9e-17 |x|, below half an ulp of x itself (the rounding every phase already carries), and
// one FMA less on the longest dependency chain of an evaluation (k_modesum +1.2-1.6%, the
// spectrum moves by 8e-12 of max|S| at config 2).
constexpr int SCTAB = 512;
// The cosine on |r| <= pi/512 as COS_A - z/2 (z = r^2) with the constant chosen
// minimax (max error 2.95e-11 = half the dropped z^2/24 at r = pi/512; mpmath), one FMA instead
// of the r^4 Taylor form's two. 2.95e-11 of a term is far below the ~1e-9 rad rounding every
// term's phase already carries (phases reach 1e7 rad). The slope stays -0.5 (an inline
// constant: the free minimax slope, 7.4e-12, cost an SGPR pair and VGPR moves in the record
// loop). COS_A is the constant callers pass as c0 (J <= 2 records fold rho - 1 into it:
// fma(-v, v, COS_A) = COS_A rho to 2e-20).
constexpr double COS_A = 1.000000000029531;
constexpr double COS_B = -0.5;
static_assert(COS_A == ENV_AMP_SCALE, "envelope amplitudes carry COS_A (k_items)");
__device__ __forceinline__ void sincos_tab(double x, int shift, const double2* __restrict__ tab,
                                           double& s, double& c, double extra = 0.0,
                                           bool use_extra = false, double extra_scale = 1.0,
                                           double c0 = COS_A) {
    constexpr double INV_STEP = 81.48733086305042;       // 256 / pi
    constexpr double STEP_1 = 0.01227184630308513;       // pi/256, leading part
    // q = nearest integer to x / step via the 1.5 * 2^52 shifter: its low word is q itself
    // (two's complement), so neither rint nor a float->int conversion is needed
    constexpr double SHIFTER = 6755399441055744.0;
    const double qs = fma(x, INV_STEP, SHIFTER);
    const double q = qs - SHIFTER;
    double r = fma(-q, STEP_1, x);
    // a small angle (|extra_scale * extra| < 1e-3) added after the reduction
    if (use_extra) r = fma(extra_scale, extra, r);
    const int qi = __double2loint(qs);
    // (sin, cos)((q + shift) pi/256), addressed in bytes: v_lshl_add + v_and
    const uint32_t off = ((uint32_t)qi * 16u + (uint32_t)shift * 16u) & (uint32_t)(16 * (SCTAB - 1));
    const double2 t = *reinterpret_cast<const double2*>(reinterpret_cast<const char*>(tab) + off);
    const double z = r * r;
    const double sr = fma(r * z, -1.6666666666666666e-01, r);
    // c0: the cosine polynomial's constant term (1, or a factor 1 + O(1e-9) folded in by the
    // caller: rho (1 + d) E to within |d| |sr| < 3e-12, see spa_fast_m)
    const double cr = fma(z, COS_B, c0);
    s = fma(t.x, cr, t.y * sr);
    c = fma(t.y, cr, -t.x * sr);
}

// amp (sin, cos)(x + shift pi/256) for the envelope records, in the tangent form: with the
// table's (sin a, cos a), sin(a + r) = cos r (sin a + cos a tan r) and cos(a + r) =
// cos r (cos a - sin a tan r), so the amplitude multiplies cos r once instead of both outputs.
// tan r = r + r^3/3 (dropped 2 r^5/15 <= 1.1e-12 at |r| <= pi/512); cos r as sincos_tab's minimax
// COS_A - r^2/2, with COS_A already in the record's amplitude (k_items: amp = COS_A A) so that
// amp cos r = amp (1 + h), h = -r^2/2 (the product's -1/2 from the output modifier, IEEE mode
// off in k_modesum as for rsqrt_pos_sum; COS_A h against h: 6e-16 relative). 11 FP64 operations
// against sincos_tab's 11 plus the two products.
__device__ __forceinline__ void sincos_tab_amp(double x, int shift,
                                               const double2* __restrict__ tab, double amp,
                                               double& wr, double& wi) {
    constexpr double INV_STEP = 81.48733086305042;       // 256 / pi
    constexpr double STEP_1 = 0.01227184630308513;       // pi/256, leading part
    constexpr double SHIFTER = 6755399441055744.0;
    const double qs = fma(x, INV_STEP, SHIFTER);
    const double q = qs - SHIFTER;
    const double r = fma(-q, STEP_1, x);
    const int qi = __double2loint(qs);
    const uint32_t off = ((uint32_t)qi * 16u + (uint32_t)shift * 16u) & (uint32_t)(16 * (SCTAB - 1));
    const double2 t = *reinterpret_cast<const double2*>(reinterpret_cast<const char*>(tab) + off);
    double h;
    asm("v_mul_f64 %0, -%1, %2 div:2" : "=v"(h) : "v"(r), "v"(r));
    const double tr = fma(r * h, -0.6666666666666666, r);
    const double ac = fma(amp, h, amp);
    wi = ac * fma(t.y, tr, t.x);
    wr = ac * fma(-t.x, tr, t.y);
}

// 1/sqrt(x) for finite x > 0 inside k_modesum: the hardware estimate plus one Newton
// (second-order) correction, relative error ~1e-15 (the OCML sequence's third-order step costs
// one more FP64 operation for the last bits; the SPA amplitude needs no more; callers mask
// x <= 0), with the halving on the FMA's output modifier: e/2 comes straight out of
// v_fma_f64 ... div:2, one FP64 operation fewer. The output modifiers apply only with IEEE mode
// off and FP64 denormals flushed (tools/rsq_omod_check.hip: otherwise the modifier is silently
// ignored), which modesum_tile sets in the MODE register; the compiler never emits them itself in
// IEEE mode, hence the inline asm. Only for k_modesum's mode.
__device__ __forceinline__ double rsqrt_pos_sum(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double h;
    asm("v_fma_f64 %0, -%1, %2, 1.0 div:2" : "=v"(h) : "v"(x * y), "v"(y));
    return fma(y, h, y);
}

// Q factor. The mirror-convention term of one branch is A Y Q e^{i(2 pi g t - Phi)} with
//   SPA:      Q_spa = e^{i sgn(F') 3 pi/4} / sqrt|F'|
//   uniform:  Q = i F'/|F''| K_{1/3}(z) e^{z} 2/sqrt(3),  z = -i y,  y = 2 pi F'^3 / (3 F''^2)
//             (notebook :599-608). Since i F'/|F''| sqrt(pi/(2z)) 2/sqrt(3) == Q_spa exactly,
//             Q = Q_spa * sum_k a_k (i w)^k,  w = 1/y, a_k the Hankel asymptotic coefficients
//             of K_{1/3}: a_k = a_{k-1} (4/9 - (2k-1)^2) / (8k).
// The kernel folds arg(Q_spa) into the phase and multiplies A by the series (R + i I).
// Series split: R = sum_j b_j u^j, I = w sum_j c_j u^j, u = w^2, b_j = (-1)^j a_{2j},
// c_j = (-1)^j a_{2j+1}. With 6 terms the truncation is < 1e-17 for |y| >= 555 (fast path);
// smaller |y| (hours before plunge, turning points) takes kfactor_slow.



// G(w) from the table of tools/gen_kfactor_table.py for w = 1/|y| in [2^KTAB_E_LO, 2^KTAB_E_HI)
// (y > 0; for y < 0 the caller negates I): interval (binade e, quarter k) from the bits of w,
// local variable x = 8 m - (9 + 2k) in [-1, 1) exact (m = mantissa in [1, 2)), then one Horner
// chain of KTAB_DEG FMAs each for Re and Im. Max error 1.1e-16 against mpmath. Outside the range
// the interval index is clamped (callers mask or never get there).
constexpr double KTAB_WMIN = 0x1p-8, KTAB_WMAX = 0x1p10;
static_assert(KTAB_E_LO == -8 && KTAB_E_HI == 10, "KTAB_WMIN/WMAX follow the table's range");
__device__ __forceinline__ void kfactor_tab(double ww, double& R, double& I) {
    const uint32_t hi = (uint32_t)__double2hiint(ww);
    const int k = (int)((hi >> 18) & 3u);
    const int idx = min(max(4 * ((int)(hi >> 20) - 1023 - KTAB_E_LO) + k, 0), KTAB_N - 1);
    const double m = __hiloint2double((int)((hi & 0x000FFFFFu) | 0x3FF00000u), __double2loint(ww));
    const double x = fma(8.0, m, -(double)(9 + 2 * k));
    const double2* c = KTAB[idx];
    // coefficients in groups of KTAB_GRP pairs: a compiler barrier between groups keeps the
    // loads from being hoisted all at once (the general path runs inside k_modesum's 128-VGPR
    // budget)
    constexpr int KTAB_GRP = 4;
    static_assert((KTAB_DEG + 1) % KTAB_GRP == 0, "whole coefficient groups");
    double r = 0.0, im = 0.0;
#pragma unroll
    for (int g = KTAB_DEG + 1 - KTAB_GRP; g >= 0; g -= KTAB_GRP) {
        double2 cc[KTAB_GRP];
#pragma unroll
        for (int j = 0; j < KTAB_GRP; ++j) cc[j] = c[g + j];
#pragma unroll
        for (int j = KTAB_GRP - 1; j >= 0; --j) {
            r = fma(r, x, cc[j].x);
            im = fma(im, x, cc[j].y);
        }
        asm volatile("" ::: "memory");
    }
    R = r;
    I = im;
}

template <int J>
__device__ __forceinline__ void kseries(double ww, double& R, double& I) {
    if (J == 1) {
        R = 1.0;
        I = ww * KC[0];
        return;
    }
    const double uu = ww * ww;
    double r = KB[J - 1], im = KC[J - 1];
#pragma unroll
    for (int j = J - 2; j >= 0; --j) {
        r = fma(r, uu, KB[j]);
        im = fma(im, uu, KC[j]);
    }
    R = r;
    I = ww * im;
}
__device__ __forceinline__ void kseries_fast(double ww, double& R, double& I) {
    kseries<FAST_J>(ww, R, I);
}

// Ascending-series coefficients of kfactor_slow, c+-_k = 1 / (k! Gamma(k + 1 +- 1/3)) (the
// recurrence c_k = c_(k-1) / (k (k +- 1/3)) evaluated once, in double), and the Horner degree
// for |y| < i + 1 (next term < 1e-19 of the leading one); |y| < 18.4 needs at most 41.

// (R + i I) for |y| < FAST_Y: the table (kfactor_tab) down to |y| = 2^-10, below that the
// ascending series K = pi/(2 sin(pi/3)) (I_{-1/3} - I_{1/3}) divided by Q_spa.
__device__ __noinline__ void kfactor_slow(double fd, double fdd, double& R, double& I) {
    const double y = TWO_PI * fd * fd * fd / (3.0 * fdd * fdd);
    const double ay = fabs(y);
    if (ay * KTAB_WMAX > 1.0) {   // |y| > 2^-10: asymptotic series above 256, else the table
        const double ww = 1.0 / ay;
        if (ww < KTAB_WMIN) kseries<FAST_J>(ww, R, I);
        else kfactor_tab(ww, R, I);
        if (y < 0.0) I = -I;
        return;
    }
    // ascending series for K_{1/3}(z), z = -i y; K~ = K e^{z}: sp, sm = sum_k c+-_k q^k,
    // q = -y^2/4, by Horner to the degree |y| needs (no divisions, no convergence test)
    const double sgn = y > 0 ? 1.0 : -1.0;
    const double q = -0.25 * y * y;
    const int deg = ASC_DEG[min(18, (int)ay)];
    double sp = ASC_P[deg], sm = ASC_M[deg];
    for (int k = deg - 1; k >= 0; --k) {
        sp = fma(sp, q, ASC_P[k]);
        sm = fma(sm, q, ASC_M[k]);
    }
    const double zp = cbrt(0.5 * ay);     // (|y|/2)^{1/3}
    const double zm = 1.0 / zp;
    constexpr double c6 = 0.86602540378443864676, s6 = 0.5;  // cos, sin(pi/6)
    const double ipr = zp * c6 * sp, ipi = -sgn * zp * s6 * sp;
    const double imr = zm * c6 * sm, imi = sgn * zm * s6 * sm;
    constexpr double pref = PI / (2.0 * 0.86602540378443864676);
    const double Kr = pref * (imr - ipr), Ki = pref * (imi - ipi);
    double sy, cy;
    sincos(y, &sy, &cy);
    const double kr = Kr * cy + Ki * sy;   // K e^{-i y}
    const double ki = Ki * cy - Kr * sy;
    // Q = i f K~, f = (2/sqrt3) F'/|F''|; (R + iI) = Q / Q_spa = Q conj(Q_spa) |F'|
    const double f = 1.15470053837925152902 * fd / fabs(fdd);
    const double qr = -f * ki, qi = f * kr;
    const double a = 1.0 / sqrt(fabs(fd));
    constexpr double c34 = -0.70710678118654752440;
    const double sr = a * c34, si = (fd > 0 ? a : -a) * 0.70710678118654752440;
    const double afd = fabs(fd);
    R = (qr * sr + qi * si) * afd;
    I = (qi * sr - qr * si) * afd;
}

// Generic (slow-path) evaluation of group h's forward splines at t when t(g) overshoots the
// record's interval: search the knot and gather the cubic pieces directly.
struct FwdEval {
    double b[4];   // Bp re, Bp im, Bm re, Bm im
    double ph, fd, fdd;
};
__device__ __noinline__ FwdEval forward_generic(double tt, const double* __restrict__ t, int nt,
                                                int jhint, int h, int K, int m, int n,
                                                const double* __restrict__ coefA,
                                                const double* __restrict__ coefT) {
    // scipy: interval i with t_i <= tt < t_{i+1}, clamped to [0, nt-2] (extrapolation). t(g)
    // overshoots the record's interval jhint by little, so walk from there (1-2 loads).
    int j = jhint;
    while (j > 0 && tt < t[j]) --j;
    while (j < nt - 2 && tt >= t[j + 1]) ++j;
    const double w = tt - t[j];
    auto cub = [&](double c0, double c1, double c2, double c3) {
        return fma(fma(fma(c0, w, c1), w, c2), w, c3);
    };
    const double* ca = coefA + (size_t)j * 4 * 4 * K + 4 * h;
    const double* ct = coefT + (size_t)j * 32;
    const double dm = (double)m, dn = (double)n;
    FwdEval e;
    for (int q = 0; q < 4; ++q) e.b[q] = cub(ca[q], ca[4 * K + q], ca[8 * K + q], ca[12 * K + q]);
    e.ph = cub(dm * ct[0] + dn * ct[1], dm * ct[8] + dn * ct[9], dm * ct[16] + dn * ct[17],
               dm * ct[24] + dn * ct[25]);
    const double F0 = dm * ct[2] + dn * ct[3], F1 = dm * ct[10] + dn * ct[11],
                 F2 = dm * ct[18] + dn * ct[19];
    e.fd = fma(fma(3.0 * F0, w, 2.0 * F1), w, F2);
    const double G0 = dm * ct[4] + dn * ct[5], G1 = dm * ct[12] + dn * ct[13],
                 G2 = dm * ct[20] + dn * ct[21];
    e.fdd = fma(fma(3.0 * G0, w, 2.0 * G1), w, G2);
    return e;
}

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
// the thread index made opaque at a use site: values derived from it are recomputed there instead
// of being hoisted to the kernel's prologue as loop invariants (which, live across the record
// loop's cold call, were spilled to scratch by every wave)
__device__ __forceinline__ int opq(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

__device__ __forceinline__ double cubic(const double* __restrict__ c, double w) {
    return fma(fma(fma(c[0], w, c[1]), w, c[2]), w, c[3]);
}

// The fast path's K_{1/3} factor in polar form, G = rho e^{i theta}: log G of the Hankel series,
// re-expanded as rho = sum_j RH_j u^j and theta = w sum_j TH_j u^j (y > 0; theta is odd in y),
// u = w^2, TH = {-0.069444444444444444444, 0.035525977366255144033, -0.11095169967421124829,
// 0.85188445191064930488}. The first omitted terms fall below 1e-17 at the same |y| bounds as
// KB / KC (JSER_Y), so a record's series length J serves both forms. theta is added to the
// reduced sin/cos argument (|r| <= pi/512, where it costs no rounding) and rho scales the
// amplitude: two FP64 operations fewer per evaluation than rotating by (R + iI). theta comes out
// in units of its leading coefficient (thn = theta / TH_0), so the add of theta to the reduced
// angle is one FMA with TH_0 (with the sign of F' and the v rescaling: RecSign::kth).
//   - Records of series length 3 take the fourth terms too (below 1e-17 on their intervals, by the
//     choice of J), so J = 3 and J = 4 share one real branch (the compiler otherwise if-converts
//     the J >= 4 increments and merges the results with 4 v_cndmask per evaluation).
//   - theta is an angle added to phases that reach 1e7 rad and carry ~1e-9 rad of rounding, so
//     its series stops at terms below 1e-13 rad instead of the 1e-17 (relative) that picks J for
//     rho, an amplitude factor: for J <= 2 records (|y| >= 8.7e3, 82% of records) the KTHN1 term
//     is at most 0.0694 * 0.512 |w|^3 = 5.4e-14 rad and theta = TH_0 w; for J >= 3 the KTHN3
//     term is at most 4.2e-16 rad (|y| >= 153).
// Lane predicates as wave masks in scalar registers: every VALU instruction issues in 4 cycles
// per wave64, an FP64 FMA's cost, so the fast path's per-lane booleans (lane range: 2 integer
// compares per bin; the |y| test of a series-length-4 record; the any-lane test of the general
// path) are masks: the lane range from the record's bounds in SALU (lane_range_mask), each
// comparison's result taken by ballot (the compare itself writes the mask), the |y| test only in
// a wave-uniform branch for records that need it, and the masks combined in SALU.
// lanes l of the wave with lo <= l < hi (wave-uniform bounds, any range). Selects, not a clamp:
// min/max of a uniform value becomes v_med3 + v_readfirstlane (2 VALU), the selects stay SALU.
__device__ __forceinline__ uint64_t lanes_below(int32_t x) {
    const uint64_t m = x >= 64 ? ~0ull : ((1ull << (x & 63)) - 1ull);
    return x <= 0 ? 0ull : m;
}
__device__ __forceinline__ uint64_t lane_range_mask(int32_t lo, int32_t hi) {
    return lanes_below(hi) & ~lanes_below(lo);
}
// The sign of F' is the record's (Item::fdneg, wave-uniform), so the table shift and the angle's
// sign are scalar values: one v_cmp_class (F' of the record's sign, nonzero) replaces an |F'| > 0
// compare, a per-lane sign compare, a shift select and a copysign (lanes whose F' has the other
// sign, at turning points, take the general path). The class test is inline asm: the builtin's
// boolean is turned into a VGPR and compared back (2 VALU) before a ballot.
struct RecSign {
    int32_t fdcls;   // v_cmp_class mask: F' normal or subnormal of the record's sign
    int32_t shift;   // sign(F') 3 pi / 4 in table steps
    double kth;      // theta = kth * min(|thn|, 1): KTH0 with the sign of F'
    bool safe;       // every lane passes the interval and sign tests (record_safe)
};
// bits: Item::fdneg (bit 0: F' < 0, bit 1: safe record)
__device__ __forceinline__ RecSign rec_sign(uint32_t bits) {
    const bool fdneg = bits & 1u;
    RecSign r;
    r.safe = (bits & 2u) != 0;
    r.fdcls = fdneg ? 0x018 : 0x180;
    r.shift = fdneg ? -192 : 192;
    r.kth = fdneg ? -KTH0 / VS : KTH0 / VS;
    return r;
}
// lanes where v_cmp_class_f64(x, cls) holds, as a wave mask
__device__ __forceinline__ uint64_t class_mask(double x, int32_t cls) {
    uint64_t m;
    asm volatile("v_cmp_class_f64_e64 %0, %1, %2" : "=s"(m) : "v"(x), "s"(cls));
    return m;
}
// Masking the fast path's amplitude: k_modesum runs with FP64 denormals
// flushed (modesum_tile sets the MODE register; no value of the sum comes near 1e-308), so
// clearing the high word alone turns any amp -- inf and NaN included -- into a denormal that
// every later FP64 operation reads as +0: one v_cndmask_b32 instead of two for the 64-bit
// select, with bitwise the same W (+0 either way).
__device__ __forceinline__ double ftz_select(bool ok, double v) {
    return __hiloint2double(ok ? __double2hiint(v) : 0, __double2loint(v));
}
// A wave-uniform test of the record header, re-derived in SALU at each use: the empty asm
// makes the header word "new" to the compiler, so the test is an s_and + s_cmp on the SGPR
// instead of a boolean kept alive across the bins' blocks, which the compiler turned into a
// VGPR and back (v_cndmask + v_cmp, 2 VALU) for every bin after the first.
__device__ __forceinline__ bool hdr_test(uint32_t ha, uint32_t mask) {
    asm volatile("" : "+s"(ha));
    return (ha & mask) != 0;
}
__device__ __forceinline__ bool hdr_j3(uint32_t ha) {   // the record's series length J >= 3
    asm volatile("" : "+s"(ha));
    return ((ha >> HDR_J) & 7u) >= 3u;
}
__device__ __forceinline__ bool hdr_j4(uint32_t ha) {   // J >= 4
    asm volatile("" : "+s"(ha));
    return ((ha >> HDR_J) & 7u) >= 4u;
}
// The common record class on its own straight-line body: certified safe, series length J <= 2
// and covering the wave's whole 64 BPL-lane chunk (every lane evaluates, every lane passes the
// interval and sign tests), so no lane mask, no amplitude select and no series branch:
// spa_fast_m's J <= 2 arithmetic, bitwise the same values (config 2: kernel 5.128 -> 4.978 ms
// per launch of 8, +3.2% waveforms/s, 3 paired rounds, profiles/r05d_ab_fastpath.jsonl)
__device__ __forceinline__ void spa_simple(const Item* __restrict__ it, double sfk, double stfk,
                                           const double2* __restrict__ sct, const RecSign& rs,
                                           double& wr, double& wi, double& w) {
    const double u = sfk - it->gx;
    const double tt = fma(fma(fma(it->ic[0], u, it->ic[1]), u, it->ic[2]), u, it->ic[3]);
    w = tt - it->tj;
    const double ph = fma(fma(fma(it->ph[0], w, it->ph[1]), w, it->ph[2]), w, it->ph[3]);
    const double fd = fma(fma(it->fd[0], w, it->fd[1]), w, it->fd[2]);
    const double amp = rsqrt_pos_sum(fabs(fd));
    const double psi0 = fma(stfk, tt, -ph);
    const double fdds = fma(fma(it->fdd[0], w, it->fdd[1]), w, it->fdd[2]);
    const double a3 = amp * amp * amp;
    const double t3 = fdds * a3;
    const double ww = t3 * t3;
    double sn, cs;
    sincos_tab(psi0, rs.shift, sct, sn, cs, ww, true, rs.kth, fma(-ww, ww, COS_A));
    wr = amp * cs;
    wi = amp * sn;
}
// The same for series length J = 3 (16% of config 2's records): spa_fast_m's J >= 3 branch with
// every lane active and in range (k_items gives J = 3 only when |y| >= 555 / 1.1 on the whole
// interval, far inside FAST_Y = 153), bitwise its values (+1.8% config 2, CI 1.006-1.023, 3
// paired rounds, profiles/r05g_ab_fast3.jsonl)
__device__ __forceinline__ void spa_simple3(const Item* __restrict__ it, double sfk, double stfk,
                                            const double2* __restrict__ sct, const RecSign& rs,
                                            double& wr, double& wi, double& w) {
    const double u = sfk - it->gx;
    const double tt = fma(fma(fma(it->ic[0], u, it->ic[1]), u, it->ic[2]), u, it->ic[3]);
    w = tt - it->tj;
    const double ph = fma(fma(fma(it->ph[0], w, it->ph[1]), w, it->ph[2]), w, it->ph[3]);
    const double fd = fma(fma(it->fd[0], w, it->fd[1]), w, it->fd[2]);
    const double amp = rsqrt_pos_sum(fabs(fd));
    const double psi0 = fma(stfk, tt, -ph);
    const double fdds = fma(fma(it->fdd[0], w, it->fdd[1]), w, it->fdd[2]);
    const double a3 = amp * amp * amp;
    const double t3 = fdds * a3;
    const double ww = t3 * t3;
    const double uu = ww * ww;
    const double r = fma(45.7, uu * uu, 1.0 - uu);
    const double thn = ww * fma(-14.733333333333333333, uu, 1.0);
    const double am = amp * r;
    double sn, cs;
    sincos_tab(psi0, rs.shift, sct, sn, cs, thn, true, rs.kth, COS_A);
    wr = am * cs;
    wi = am * sn;
}
// Envelope records (k_items, env_fit.inc; Item::jser = 0, always certified safe): the phase with
// theta already in the record's phase cubic and the amplitude A(w) = rho / sqrt|F'| from its
// degree-ENV_DEG polynomial, for the NB bins of the lane. 26 FP64 operations per bin instead of
// spa_simple's 36 (the sin/cos in sincos_tab_amp's tangent form): no F', F'' quadratics, no 1/sqrt|F'| Newton step, no 1/|y| and no angle or rho
// fold in the sin/cos.
// MASK: the record covers the wave's chunk only partly; lanes outside am[i] get A = +0 (flushed).
template <bool MASK, int NB>
__device__ __forceinline__ void env_record(const Item* __restrict__ it, const double* fk,
                                           const double* tfk, const double2* __restrict__ sct,
                                           const RecSign& rs, const uint64_t* am, double* wr,
                                           double* wi, double* w) {
    const double* e = env_of(it);
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const double u = fk[i] - it->gx;
        const double tt = fma(fma(fma(it->ic[0], u, it->ic[1]), u, it->ic[2]), u, it->ic[3]);
        w[i] = tt - it->tj;
        const double ph = fma(fma(fma(it->ph[0], w[i], it->ph[1]), w[i], it->ph[2]), w[i], it->ph[3]);
        const double psi0 = fma(tfk[i], tt, -ph);
        double amp = e[0];
#pragma unroll
        for (int c = 1; c <= ENV_DEG; ++c) amp = fma(amp, w[i], e[c]);
        if (MASK) amp = ftz_select(__builtin_amdgcn_inverse_ballot_w64(am[i]), amp);
        sincos_tab_amp(psi0, rs.shift, sct, amp, wr[i], wi[i]);
    }
}
template <int CAUSTIC>
__device__ __forceinline__ void spa_fast_m(const Item* __restrict__ it, double sfk, double stfk,
                                           uint32_t ha, uint64_t actm,
                                           const double2* __restrict__ sct,
                                           const RecSign& rs, double& wr, double& wi, double& w,
                                           uint64_t& needm) {
    const double u = sfk - it->gx;
    const double tt = fma(fma(fma(it->ic[0], u, it->ic[1]), u, it->ic[2]), u, it->ic[3]);
    w = tt - it->tj;
    const double ph = fma(fma(fma(it->ph[0], w, it->ph[1]), w, it->ph[2]), w, it->ph[3]);
    const double fd = fma(fma(it->fd[0], w, it->fd[1]), w, it->fd[2]);
    const double afd = fabs(fd);
    uint64_t goodm = ~0ull;
    if (!hdr_test(ha, 2u << HDR_FD)) {   // wave-uniform: a record k_items could not certify tests every lane
        asm volatile("");
        goodm = __builtin_amdgcn_ballot_w64((unsigned long long)__double_as_longlong(w) <
                                            (unsigned long long)__double_as_longlong(it->dtj)) &
                class_mask(fd, rs.fdcls);
    }
    // F' = 0 gives amp = NaN here; every quantity it reaches is selected away below
    const double amp = rsqrt_pos_sum(afd);
    const double psi0 = fma(stfk, tt, -ph);
    double sn, cs;
    if (CAUSTIC == EFD_CAUSTIC_UNIFORM) {
        static_assert(FAST_J == 4, "early mask: the J >= 3 branch covers J = 3 and 4");
        // The amplitude is masked before it enters 1/|y|: masked lanes get amp = +0 (inf and
        // NaN included), so w = 0, theta = 0 and rho = 1 there and the angle stays finite with no
        // clamp; for J <= 3 records every in-interval lane is within the series' range, so
        // nothing else needs masking. J <= 2 (82% of records): rho - 1 = KRH_1 w^2 < 4.6e-10
        // goes into the cosine polynomial's constant term instead of a multiply of the
        // amplitude (rho E to within |rho - 1| |sr| < 3e-12, a rotation far below the phases'
        // 1e-9 rad rounding). J >= 3 (18%) tests |y| >= FAST_Y, clamps w for the lanes past it
        // and masks their amplitude again.
        const double ampm = ftz_select(__builtin_amdgcn_inverse_ballot_w64(actm & goodm), amp);
        const double fdds = fma(fma(it->fdd[0], w, it->fdd[1]), w, it->fdd[2]);
        const double a3 = ampm * ampm * ampm;
        const double t3 = fdds * a3;
        double ww = t3 * t3;   // 1/|y|
        double am, c0, thn;
        if (hdr_j3(ha)) {   // J >= 3: wave-uniform; a real branch (see KTH0's notes)
            asm volatile("");
            // the |y| >= FAST_Y test only matters for J = 4 (J = 3 lanes pass it by their
            // record's bound), but a nested J test's condition crossed the join as a per-lane
            // boolean (v_cndmask + v_cmp for every record)
            // |w| <= 1/153: rho's KRH_3 term (< 2.2e-14) and theta's KTHN_2 term (< 1.3e-12 rad)
            // are below the accuracy of the rest of the evaluation
            // ww = v = VS w: rho = 1 - v^2 + (KRH_2 / KRH_1^2) v^4, theta / (TH_0 / VS) =
            // v (1 + (KTHN_1 / |KRH_1|) v^2)
            // lanes past the series' range get w = +0 (high word cleared, flushed): finite
            // angle, masked amplitude below; one v_cndmask instead of fmin's max + min
            const uint64_t inrange = __builtin_amdgcn_ballot_w64(ww <= VS / FAST_Y);
            goodm &= inrange;
            ww = ftz_select(__builtin_amdgcn_inverse_ballot_w64(inrange), ww);
            const double uu = ww * ww;
            const double r = fma(45.7, uu * uu, 1.0 - uu);
            thn = ww * fma(-14.733333333333333333, uu, 1.0);
            am = ftz_select(__builtin_amdgcn_inverse_ballot_w64(actm & goodm), ampm * r);
            c0 = COS_A;
        } else {
            c0 = fma(-ww, ww, COS_A);   // (1 + KRH_1 w^2) COS_A = (1 - v^2) COS_A
            thn = ww;
            am = ampm;
        }
        sincos_tab(psi0, rs.shift, sct, sn, cs, thn, true, rs.kth, c0);
        wr = am * cs;
        wi = am * sn;
    } else {
        const bool ok = __builtin_amdgcn_inverse_ballot_w64(actm & goodm);
        const double am = ftz_select(ok, amp);
        sincos_tab(psi0, rs.shift, sct, sn, cs);
        wr = am * cs;
        wi = am * sn;
    }
    needm = actm & ~goodm;
}

#ifdef EFD_EXP
// record evals, cold-path evals, cold lanes, skips; cold lanes by cause: overshoot, 18.4 <= |y| <
// FAST_Y, |y| < 18.4
// Experiment build (-DEFD_EXP, tools/exp_variants.py): counters and per-tile clocks. Never in the
// product library (tests/test_abi.py checks that efd_exp_* is not exported).
constexpr int EXP_NCOUNT = 40;
__device__ unsigned long long g_exp_count[EXP_NCOUNT];  // [8..15]: |y| bands of kfactor_slow's J;
// [16, 17]: cold wave evaluations / lanes (one-body kernel); [18..23]: overshoot bands of
// max(-w, w - dtj) / dtj: < 1e-12, 1e-9, 1e-6, 1e-3, 1e-1, larger; [24, 25, 26]: chunk barrier
// balance: sum over chunks of the busiest wave's record evaluations, of all waves' evaluations,
// and the number of chunks; [27, 28]: segment table size, hits per tile summed (k_tile_keys);
// [29]: wave-records of certified-safe records; [32..35]: wave-records by series length J = 1..4,
// [36]: sub-branch flips; [37..39]: wave-records off the straight-line path by cause (partial
// coverage, J >= 3, not certified; a record may count in several)
__device__ unsigned int g_exp_tile[16384];       // record evaluations per tile (first 16384)
__device__ unsigned long long g_exp_tclk[16384];  // wall clock (s_memrealtime) per tile
#endif

// General (cold) path: scipy interval selection for t(g) and the full K_{1/3} evaluation.
// Returns W and both group amplitudes at t(g), the own bin's first (b[0], b[1]: the staged
// record's b[0]; from the spline coefficients, Bp for s = 0 and Bm for s = 1).
struct ColdEval {
    double wr, wi, b[4];
};
template <int CAUSTIC>
__device__ __noinline__ ColdEval spa_general(const Item* __restrict__ it, double g, int s, int h,
                                             int jrec,
                                             const double* __restrict__ t, int nt, int K,
                                             const int32_t* __restrict__ gm,
                                             const int32_t* __restrict__ gn,
                                             const double* __restrict__ coefA,
                                             const double* __restrict__ coefT) {
    const double u = g - it->gx;
    const double tt = fma(fma(fma(it->ic[0], u, it->ic[1]), u, it->ic[2]), u, it->ic[3]);
    double ph, fd, fdd;
    ColdEval c;
    const double wl = tt - it->tj;
    if (wl >= 0.0 && wl < it->dtj) {
        const double w = wl;
        for (int q = 0; q < 4; ++q) c.b[q] = cubic(it->b[q >> 1][q & 1], w);
        ph = fma(fma(fma(it->ph[0], w, it->ph[1]), w, it->ph[2]), w, it->ph[3]);
        fd = fma(fma(it->fd[0], w, it->fd[1]), w, it->fd[2]);
        fdd = INV_FDD_SCALE * fma(fma(it->fdd[0], w, it->fdd[1]), w, it->fdd[2]);
    } else {  // t(g) overshot the record's knot interval: evaluate like scipy
#ifdef EFD_EXP
        atomicAdd(&g_exp_count[4], 1ull);
        {
            const double ov = fmax(-wl, wl - it->dtj) / it->dtj;
            const int band = ov < 1e-12 ? 18 : ov < 1e-9 ? 19 : ov < 1e-6 ? 20 : ov < 1e-3 ? 21
                           : ov < 1e-1 ? 22 : 23;
            atomicAdd(&g_exp_count[band], 1ull);
        }
#endif
        const FwdEval fe = forward_generic(tt, t, nt, jrec, h, K, gm[h], gn[h], coefA, coefT);
        for (int q = 0; q < 4; ++q) c.b[q] = fe.b[s ? q ^ 2 : q];
        ph = fe.ph; fd = fe.fd; fdd = fe.fdd;
    }
    const double amp = fd != 0.0 ? rsqrt(fabs(fd)) : 0.0;
    const double psi = fma(TWO_PI * g, tt, -ph) + (fd > 0.0 ? 0.75 * PI : -0.75 * PI);
    double R = 1.0, I = 0.0;
    if (CAUSTIC == EFD_CAUSTIC_UNIFORM && fd != 0.0 && fdd != 0.0) {
        const double a2 = amp * amp;
        const double a6 = a2 * a2 * a2;
        const double ww = (fd > 0.0 ? 1.0 : -1.0) * (3.0 / TWO_PI) * fdd * fdd * a6;
        if (fabs(ww) * FAST_Y <= 1.0) {
            kseries_fast(ww, R, I);
        } else {
#ifdef EFD_EXP
            atomicAdd(&g_exp_count[fabs(ww) * 18.4 <= 1.0 ? 5 : 6], 1ull);
            {
                const double ay = 1.0 / fabs(ww);
                const int band = ay >= 153.0 ? 8 : ay >= 75.0 ? 9 : ay >= 48.0 ? 10 : ay >= 29.4 ? 11
                               : ay >= 23.1 ? 12 : ay >= 20.3 ? 13 : ay >= 18.4 ? 14 : 15;
                atomicAdd(&g_exp_count[band], 1ull);
            }
#endif
            kfactor_slow(fd, fdd, R, I);
        }
    }
    double sn, cs;
    sincos_big(psi, sn, cs);
    c.wr = amp * (R * cs - I * sn);
    c.wi = amp * (R * sn + I * cs);
    return c;
}

// Accumulation of one evaluation into the lane's two bins. X is the own bin's group amplitude
// (b[S]), Z the mirror's (b[1-S]):
//   S = 0: own += X W,        mirror += conj(Z W)   (parent at f = -g, partner at the mirror)
//   S = 1: own += conj(X W),  mirror += Z W
template <int S, bool PAIRED>
__device__ __forceinline__ void accumulate(double wr, double wi, double xr, double xi, double zr,
                                           double zi, double& own_r, double& own_i,
                                           double& mir_r, double& mir_i) {
    own_r = fma(xr, wr, own_r);
    own_r = fma(-xi, wi, own_r);
    own_i = fma(S ? -xr : xr, wi, own_i);
    own_i = fma(S ? -xi : xi, wr, own_i);
    if (PAIRED) {
        mir_r = fma(zr, wr, mir_r);
        mir_r = fma(-zi, wi, mir_r);
        mir_i = fma(S ? zr : -zr, wi, mir_i);
        mir_i = fma(S ? zi : -zi, wr, mir_i);
    }
}

// One 16-B LDS-DMA piece per lane: global src (per lane) -> LDS dst (wave-uniform base + 16 B x
// lane). Issued through inline asm: the compiler's waitcnt pass treats the
// intrinsic's LDS write as possibly aliasing later ds_reads, so each wave waited for its prefetch
// of the next stage at the first record of every chunk (s_waitcnt vmcnt at the loop head). Hidden
// from that pass, the DMA is retired only by the explicit vmcnt(0) before each chunk barrier and
// at the end of the cold block (whose spill reloads would otherwise leave a vmcnt wait at the
// loop head): bitwise the same spectrum, ratio 1.005 (CI 1.002-1.015, 8 rounds). Round 1 measured
// the same idea as neutral (1.148 vs 1.14 ms) while the cold block's reloads still kept a vmcnt
// wait at the loop head. M0 (the DMA's LDS base) is set inside the asm: the k_modesum instances
// have no other M0 user (checked in their ISA), hence the local -Winline-asm silence.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void glds16(const uint4* src, uint4* dst) {
    const uint32_t base = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(dst));
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                 :
                 : "v"(src), "s"(base)
                 : "memory", "m0");
}
#pragma clang diagnostic pop

// ----------------------------------------------------------------------------------------
// K8: the mode sum. One workgroup (4 waves) per tile of TILE * BPL frequency bins ("lanes");
// wave w owns the contiguous chunk [tile_base + w*64*BPL, +64*BPL) and lane l its bins
// chunk + 64 i + l (i < BPL). The tile's list of interval records is sorted in LDS (fixed
// summation order -> bitwise reproducible), then streamed through a double-buffered LDS stage:
// the whole workgroup streams the next NC records global -> LDS (global_load_lds, 16 B per lane)
// while the waves evaluate the current NC from LDS (broadcast reads; no dependent global latency
// in the loop).
// Each record feeds BPL independent, branch-free evaluations per lane (one per (m, n) group:
// every l of the group at once); lanes needing the general path get W = 0 there and add their
// term in a cold block. The sub-branch S of a record is wave-uniform: each S has its own copy of
// the evaluation (compile-time signs and LDS offsets).
// ----------------------------------------------------------------------------------------
// The tile's LDS, one object for every instantiation a kernel inlines (a kernel holding both the
// whole-tile and the sub-bin form of modesum_tile allocates it once, not twice)
struct TileLds {
    uint32_t keys[KEYCAP];
    Item stage[2][NC];
    int part[TILE];
    int hits[SEGWIN], hp0[SEGWIN], hcnt[SEGWIN], hoff[SEGWIN];
    int wcnt[(SEGWIN / TILE) * NWAVE];
    double2 sctab[SCTAB];   // (sin, cos)(k pi/128) for sincos_tab
#ifdef EFD_EXP
    int wimb[2][NWAVE];     // records each wave evaluated in a chunk (barrier balance)
#endif
};
__device__ __forceinline__ TileLds& tile_lds() {
    __shared__ TileLds lds;
    return lds;
}

template <bool PAIRED>
__device__ __forceinline__ void tile_epilogue(
    double (&own_r)[BPL], double (&own_i)[BPL], double (&mir_r)[BPL], double (&mir_i)[BPL],
    int32_t w_lo, int lane, int wave, int tid, int64_t nlanes, int64_t nf, int64_t k0,
    int accumulate_out, double* __restrict__ out, double* __restrict__ hp,
    double* __restrict__ hc, const double* __restrict__ lld, const double* __restrict__ llw,
    double* __restrict__ llpart, int64_t tile);

template <bool PAIRED, int CAUSTIC, int NB = BPL>
// 4 waves per SIMD (<= 128 VGPRs, 19 spilled, all outside the fast path's FMA chains): with
// 37.6 KB of LDS per workgroup 4 workgroups fit a CU, and the fourth wave hides more FP64
// latency than the spills cost (config 2: 1.00 ms against 1.09 ms at 3 waves / 147 VGPRs;
// 5 waves with a one-round stage: 1.07 ms)
#ifndef EFD_WAVES_PER_EU
#define EFD_WAVES_PER_EU 4
#endif
// 1: the tiles' record lists are built by k_tile_keys in the preparation phase and DMA'd in by
// the sum; tiles whose list needs more than one KEYCAP pass or has more than TK_HITS segments
// (tcnt = -1) build it in the sum as before. 0: always in the sum.
// sum dispatch order from k_tile_order: 0 = fixed (f = 0 outward), 1 = tiles longest first
__device__ __forceinline__ void modesum_tile(
    const Item* __restrict__ items, const int4* __restrict__ ranges,
    const int2* __restrict__ seglh, const int4* __restrict__ seginfo,
    const int32_t* __restrict__ nsegp, const double* __restrict__ freq, int64_t nf,
    int64_t nlanes, int64_t ntiles, int nt, int K, const int32_t* __restrict__ gm,
    const int32_t* __restrict__ gn, const double* __restrict__ t,
    const double* __restrict__ coefA, const double* __restrict__ coefT,
    const double2* __restrict__ sctab_g, const uint32_t* __restrict__ tkeys,
    const int32_t* __restrict__ tcnt, const int32_t* __restrict__ tperm,
    const int32_t* __restrict__ segbase, const int32_t* __restrict__ stb0,
    const int32_t* __restrict__ stb1, Header* __restrict__ hdr, int accumulate_out,
    double* __restrict__ out, double* __restrict__ hp, double* __restrict__ hc, int64_t k0,
    // fused likelihood (efd_modesum_sum_loglike; paired grids): d complex, w real [2][nf - k0];
    // the tile writes sum_c sum_j |d[c][j] - h_c[j] w[c][j]|^2 over its bins j >= k0 to
    // llpart[tile]. lld = NULL: not computed.
    const double* __restrict__ lld, const double* __restrict__ llw, double* __restrict__ llpart,
    // fused likelihood: the partial of a tile with no record (h = 0 on its bins), the same for
    // every walker (efd_loglike_tile_constants); NULL: such tiles compute it
    const double* __restrict__ llconst,
    int64_t b,     // b: this workgroup's place in the waveform's dispatch order
    bool direct = false,     // b is the tile itself (k_modesum_batch's sparse form)
    // NB < BPL: a split tile (k_segments_one's plan; sparse form), the sub-bin form. This
    // workgroup evaluates bins ioff .. ioff + NB - 1 of every lane (all of the tile's records, in
    // the whole tile's order, so each bin's sum is bitwise the whole tile's), stores them in the
    // tile's slot spart, and the last of the BPL / NB workgroups (arrival counter *scnt) loads
    // the slot and runs the epilogue
    int ioff = 0, double* __restrict__ spart = nullptr, int32_t* __restrict__ scnt = nullptr) {
    static_assert(NB == BPL || NB == 1, "sub-bin form: one bin per lane");
    TileLds& L_ = tile_lds();
    uint32_t* const keys = L_.keys;
    Item (*const stage)[NC] = L_.stage;
    int* const part = L_.part;
    int* const hits = L_.hits;
    int* const hp0 = L_.hp0;
    int* const hcnt = L_.hcnt;
    int* const hoff = L_.hoff;
    int* const wcnt = L_.wcnt;
    double2* const sctab = L_.sctab;
#ifdef EFD_EXP
    int (*const wimb)[NWAVE] = L_.wimb;
#endif
    if (NB == BPL) ioff = 0;
    // Tile order. Blocks are dealt round-robin over the 8 XCDs; XCD x = b % 8 here gets groups
    // of XCD_GROUP consecutive tiles (neighbouring tiles share interval records, which then hit
    // in that XCD's L2) interleaved with the other XCDs' groups, so every XCD sees the same mix
    // of dense (low |f|) and empty (near Nyquist) tiles. The lane order runs from -Nyquist to
    // f = 0, so walking it backwards dispatches the dense band first and the cheap high-|f|
    // tiles last (short tail). The grid is padded to a multiple of 8 * XCD_GROUP.
    // With a cost order (tperm, k_tile_order) block b takes the b-th most expensive tile instead:
    // longest-first dispatch, so the launch does not end on expensive tiles started late;
    // consecutive blocks (similar cost) land on different XCDs.
    int64_t tile;
    if (direct) {
        tile = b;
    } else if (tperm != nullptr) {
        if (b >= ntiles) return;   // grid padding
        tile = tperm[b];
        if ((uint64_t)tile >= (uint64_t)ntiles) {
            // a corrupt or stale order entry: never index past the grid, and make
            // efd_modesum_status report it (the tile's bins would be left unwritten)
            if (threadIdx.x == 0) hdr->bad_tile = 1;
            return;
        }
    } else {
        // (the padded per-waveform grid, not gridDim: a batched launch holds several)
        const int64_t gq = 8 * XCD_GROUP, ngrid = (ntiles + gq - 1) / gq * gq;
        const int64_t r = b >> 3, grp = r / XCD_GROUP;
        const int64_t lin = (grp * 8 + (b & 7)) * XCD_GROUP + (r % XCD_GROUP);
        tile = ngrid - 1 - lin;
        if (tile >= ntiles) return;
    }
#ifdef EFD_EXP
    const unsigned long long t_start = wall_clock64();
#endif
    // MODE.FP_DENORM[3:2] (FP64/FP16) = 0: flush denormal inputs and outputs (ftz_select). The
    // mode is per wave and set from the kernel descriptor at every wave launch.
    __builtin_amdgcn_s_setreg(1 | (6 << 6) | (1 << 11), 0);   // hwreg(HW_REG_MODE, 6, 2)
    // MODE.IEEE = 0 (rsqrt_pos_sum's output modifier). Nothing here depends on IEEE mode's NaN
    // rules: the one min (fmin(|thn|, 1)) sees quiet NaNs at most and returns 1 in either mode.
    __builtin_amdgcn_s_setreg(1 | (9 << 6), 0);               // hwreg(HW_REG_MODE, 9, 1)
    // tid / lane are re-derived from tid0 through opq at the top of each loop and of the
    // epilogue, so nothing derived from them is live across the record loop's cold call (the
    // prologue's scratch stores of such values, 7 KB per wave, are gone)
    const int tid0 = threadIdx.x;
    int tid = tid0;
    int lane = tid & 63;
    const int ni = nt - 1;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform
    // Prebuilt record list: k_tile_keys, launched in the preparation phase, stored this tile's
    // keys when they fit in one KEYCAP pass (tcnt >= 0); they come in by LDS-DMA with the sin/cos
    // table and the build below is skipped. Same keys in the same order as the build below, so
    // the sum is bitwise the in-kernel build's.
    const int pre = tcnt != nullptr ? tcnt[tile] : -1;
    const int32_t tlo = (int32_t)(tile * TILE_LANES), thi = tlo + TILE_LANES;
    // a tile outside the union of the segments' lane ranges has no record: no list to build
    const int nseg = (pre < 0 && (hdr->lane_hi <= tlo || hdr->lane_lo >= thi))
                         ? 0 : *nsegp;
    // a tile that can have records (a prebuilt list, or segments to search): block-uniform. Tiles
    // without read neither their frequencies nor the sin/cos table
    const bool anyrec = pre > 0 || (pre < 0 && nseg > 0);
    bool seen = pre > 0;   // records evaluated (the fused likelihood's constant otherwise)
    // the (sin, cos) table: k_group's copy, global -> LDS by LDS-DMA (lane-linear pieces), with
    // a prebuilt list's keys
    static_assert(SCTAB % TILE == 0, "sin/cos table copy: whole rounds");
    if (anyrec) {
        if (pre > 0) {
            static_assert(KEYCAP % (4 * TILE) == 0, "key copy: whole rounds of 16-B pieces");
#pragma unroll
            for (int rd = 0; rd < KEYCAP / (4 * TILE); ++rd) {
                const int pc = rd * TILE + tid;                     // 16-B piece = 4 keys
                if (4 * pc < pre)
                    glds16(reinterpret_cast<const uint4*>(tkeys + (size_t)tile * KEYCAP) + pc,
                           reinterpret_cast<uint4*>(keys) + rd * TILE + wave * 64);
            }
        }
#pragma unroll
        for (int rd = 0; rd < SCTAB / TILE; ++rd)
            glds16(reinterpret_cast<const uint4*>(sctab_g) + rd * TILE + tid,
                   reinterpret_cast<uint4*>(sctab) + rd * TILE + wave * 64);
        __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0)
        __syncthreads();
    }

    // ---- the tile's record list, built in LDS from the segment table (no global list, no
    // atomics). Segments are taken in windows of SEGWIN: (1) each thread tests SEGWIN/TILE
    // segments (strided, coalesced) for overlap with the tile, and a ballot compaction keeps the
    // hits in segment order; (2) one thread per hit bisects that segment's records for the
    // sub-range [p0, p0 + n) reaching into the tile; (3) a block scan places the keys. Keys go to
    // keys[] until KEYCAP, then the chunked evaluation below drains them. The summation order
    // (segment, then lane order) is fixed, so the result is bitwise reproducible.
    const int32_t w_lo = (int32_t)(tile * TILE_LANES + wave * 64 * BPL);
    // the bins this workgroup evaluates in the wave's chunk: [e_lo, e_hi), NB per lane
    const int32_t e_lo = w_lo + 64 * ioff;
    const int32_t e_hi = e_lo + 64 * NB;
    double fk[NB], tfk[NB];
    double own_r[NB], own_i[NB], mir_r[NB], mir_i[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int32_t k = e_lo + 64 * i + lane;
        fk[i] = (anyrec && k < nlanes) ? freq[k] : 0.0;
        tfk[i] = TWO_PI * fk[i];
        own_r[i] = own_i[i] = mir_r[i] = mir_i[i] = 0.0;
    }
    // Sub-branch sign state (wave-uniform): fk, tfk hold g = -+f, 2 pi g of the sub-branch s_cur
    // and own_i, mir_i hold sg * (the true sums), sg = -1 for s_cur = 1. A record of the other
    // sub-branch flips the 4 BPL registers in place (one v_xor each) instead of making signed
    // copies of fk, tfk, wi, wr for every record (16 VALU per record); negation commutes with
    // round-to-nearest, so the sums are bitwise those of the signed-copy form.
    int s_cur = 0;
#pragma unroll
    for (int i = 0; i < NB; ++i) { fk[i] = -fk[i]; tfk[i] = -tfk[i]; }   // s = 0: g = -f

    // staging: a record is PIECES pieces of 16 B; NC records take at most ROUNDS pieces per thread.
    // The pieces go global -> LDS directly (gfx950 global_load_lds_dwordx4: no VGPR staging,
    // nothing held across the evaluation loop). The LDS destination of one wave-instruction is
    // a wave-uniform base + 16 B x lane, so piece p = round * TILE + 64 wave + lane of the chunk
    // lands at ((uint4*)stage[buf])[p], i.e. record p / PIECES, piece p % PIECES; its global
    // source is per lane.
    static_assert(PIECES * NC <= ROUNDS * TILE, "staging: at most ROUNDS 16-B pieces per thread");
#define EFD_GLDS(c, buf)                                                                      \
    do {                                                                                      \
        _Pragma("unroll") for (int rd_ = 0; rd_ < ROUNDS; ++rd_) {                            \
            const int p_ = rd_ * TILE + tid;                                                  \
            const int r_ = p_ / PIECES, q_ = p_ - r_ * PIECES;                                \
            if (r_ < NC && (c) * NC + r_ < cnt) {                                             \
                const uint32_t key_ = keys[(c) * NC + r_];                                    \
                /* sub-branch 1: b[0] and b[1] trade places in the stage, so the own bin's */ \
                /* amplitudes are always at b[0] (fixed LDS offsets in the hot loop) */       \
                const int qs_ = ((key_ & 1u) && q_ >= B_PIECE && q_ < B_PIECE + 8)            \
                                    ? ((q_ - B_PIECE + 4) & 7) + B_PIECE : q_;                \
                const uint4* src_ = reinterpret_cast<const uint4*>(items + (key_ >> 1)) + qs_; \
                uint4* dst_ = reinterpret_cast<uint4*>(&stage[(buf)][0]) + rd_ * TILE + wave * 64; \
                glds16(src_, dst_);                                                           \
            }                                                                                 \
        }                                                                                     \
    } while (0)

    int win = 0;        // next segment window
    int nhit = 0;       // overlapping segments of the current window
    int wtotal = 0;     // keys of the current window
    int wdone = 0;      // keys of the current window already written
    int nkeys = pre > 0 ? pre : 0;   // keys waiting in keys[]
    while (true) {
        // ---- fill keys[] (block-uniform control flow)
        while (pre < 0 && nkeys < KEYCAP) {
            tid = opq(tid0);
            lane = tid & 63;
            if (wdone == wtotal) {                 // need a new window of segments
                if (win >= nseg) break;
                // (1) overlap test + ordered compaction: every thread tests its SEGWIN/TILE
                // segments, one barrier publishes the per-(row, wave) counts
                constexpr int ROWS = SEGWIN / TILE;
                unsigned long long bal[ROWS];
#pragma unroll
                for (int row = 0; row < ROWS; ++row) {
                    const int sgi = win + row * TILE + tid;
                    bool hit = false;
                    if (sgi < nseg) {
                        const int2 lh = seglh[sgi];
                        hit = lh.y > tlo && lh.x < thi;
                    }
                    bal[row] = __ballot(hit);
                    if (lane == 0) wcnt[row * NWAVE + wave] = __popcll(bal[row]);
                }
                __syncthreads();
                nhit = 0;
#pragma unroll
                for (int row = 0; row < ROWS; ++row) {
                    int before = nhit;
                    for (int w = 0; w < wave; ++w) before += wcnt[row * NWAVE + w];
                    if ((bal[row] >> lane) & 1ull) {
                        const unsigned long long below = bal[row] & ((1ull << lane) - 1ull);
                        hits[before + __popcll(below)] = win + row * TILE + tid;
                    }
#pragma unroll
                    for (int w = 0; w < NWAVE; ++w) nhit += wcnt[row * NWAVE + w];
                }
                __syncthreads();
                if (nhit == 0) {                   // nothing of this window reaches the tile
                    win += SEGWIN;
                    wtotal = wdone = 0;
                    continue;
                }
                win += SEGWIN;
                // (2) each hit segment's records reaching into the tile: [p0, p1) from the
                // segment-tile boundaries of k_seg_tiles, or by bisection
                for (int i = tid; i < nhit; i += TILE) {
                    const int32_t sbase = segbase[hits[i]];
                    if (sbase != SEG_NO_STB) {
                        const int q0 = stb0[sbase + tile], q1 = stb1[sbase + tile];
                        hp0[i] = q0;
                        hcnt[i] = max(q1 - q0, 0);
                        continue;
                    }
                    const int4 info = seginfo[hits[i]];
                    const int base = info.x, n = info.y, dir = info.z, sb = info.w;
                    int lo = 0, hi = n;            // first p (lane order) with khi > tlo
                    while (lo < hi) {
                        const int mid = (lo + hi) >> 1;
                        const int4 rg = ranges[base + (dir > 0 ? mid : n - 1 - mid)];
                        if ((sb ? rg.w : rg.y) > tlo) hi = mid; else lo = mid + 1;
                    }
                    const int p0 = lo;
                    hi = n;                        // first p with klo >= thi
                    while (lo < hi) {
                        const int mid = (lo + hi) >> 1;
                        const int4 rg = ranges[base + (dir > 0 ? mid : n - 1 - mid)];
                        if ((sb ? rg.z : rg.x) >= thi) hi = mid; else lo = mid + 1;
                    }
                    hp0[i] = p0;
                    hcnt[i] = lo - p0;
                }
                __syncthreads();
                // (3) exclusive scan of the counts (serial per thread over a block of hits,
                // then a wave scan and one barrier for the wave totals)
                const int hper = (nhit + TILE - 1) / TILE;
                const int h0 = min(nhit, tid * hper), h1 = min(nhit, h0 + hper);
                int mine = 0;
                for (int i = h0; i < h1; ++i) mine += hcnt[i];
                int incl = mine;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int v = __shfl_up(incl, o, 64);
                    if (lane >= o) incl += v;
                }
                if (lane == 63) part[wave] = incl;
                __syncthreads();
                int woff = 0, wsum = 0;
#pragma unroll
                for (int w = 0; w < NWAVE; ++w) {
                    woff += w < wave ? part[w] : 0;
                    wsum += part[w];
                }
                int run_off = woff + incl - mine;
                for (int i = h0; i < h1; ++i) { hoff[i] = run_off; run_off += hcnt[i]; }
                wtotal = wsum;
                wdone = 0;
                __syncthreads();
                continue;
            }
            // write keys [wdone, wdone + take) of this window at keys[nkeys ...], scattered by
            // the bijection x -> x * P mod take (P prime, take % P != 0): a segment's records
            // cover neighbouring lanes, i.e. mostly one wave, and unscattered a chunk of NC
            // consecutive records would keep one wave busy while the others wait at its barrier
            const int take = min(KEYCAP - nkeys, wtotal - wdone);
            const int P = (take % 97) ? 97 : 101;
            for (int i = tid; i < nhit; i += TILE) {
                const int o = hoff[i], c = hcnt[i];
                const int lo = max(o, wdone), hi = min(o + c, wdone + take);
                if (lo >= hi) continue;
                const int4 info = seginfo[hits[i]];
                for (int g = lo; g < hi; ++g) {
                    const int p = hp0[i] + (g - o);
                    const int j = info.z > 0 ? p : info.y - 1 - p;
                    keys[nkeys + (int)(((unsigned)(g - wdone) * (unsigned)P) % (unsigned)take)] =
                        ((uint32_t)(info.x + j) << 1) | (uint32_t)info.w;
                }
            }
            nkeys += take;
            wdone += take;
            __syncthreads();
        }
        if (nkeys == 0) break;

        // ---- evaluate the nkeys records in chunks of NC through the double-buffered stage
        const int cnt = nkeys;
        const int nchunk = (cnt + NC - 1) / NC;
        seen = true;
        tid = opq(tid0);
        lane = tid & 63;
        EFD_GLDS(0, 0);
        __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0): this wave's LDS-DMA pieces landed
        __syncthreads();

        for (int c = 0; c < nchunk; ++c) {
            tid = opq(tid0);
            lane = tid & 63;
            // buffer (c+1)&1 was last read in chunk c-1, which every wave finished before the
            // barrier that closed it: chunk c+1's pieces stream in meanwhile
            if (c + 1 < nchunk) EFD_GLDS(c + 1, (c + 1) & 1);
            const int nin = (int)rfl((uint32_t)min(NC, cnt - c * NC));   // loop bound in an SGPR
            const Item* stg = stage[c & 1];
            // the chunk's record headers, one lane per record, read from LDS once per chunk and
            // packed into one word: the sub-branch's lane range clamped to the tile, relative
            // to its first lane (HB bits each), s and the series length: hdr = lo | hi << HB |
            // s << 2 HB | jser << (2 HB + 1) | fdneg << (2 HB + 4). Each record then takes one v_readlane (a VALU instruction,
            // as costly as an FMA) instead of an LDS round trip and 5 address / readfirstlane
            // operations (round 1), or two readlanes of absolute bounds (round 2 first form).
            static_assert(FAST_J < 8, "header: jser in 3 bits");
            constexpr int HB = TILE_LANES < 1024 ? 10 : 11;   // bits of a tile-relative bound
            constexpr uint32_t HM = (1u << HB) - 1u;
            static_assert(TILE_LANES < 2048 && 2 * HB + 6 <= 32, "header: one 32-bit word");
            uint32_t hdr = 0;
            if (lane < nin) {
                const uint32_t kl = keys[c * NC + lane];
                const int sl = (int)(kl & 1);
                const Item* il = stg + lane;
                const uint32_t lo = (uint32_t)min(max(il->klo[sl] - tlo, 0), TILE_LANES);
                const uint32_t hi = (uint32_t)min(max(il->khi[sl] - tlo, 0), TILE_LANES);
                hdr = lo | (hi << HB) | ((uint32_t)sl << (2 * HB)) |
                      ((uint32_t)il->jser << (2 * HB + 1)) | ((uint32_t)il->fdneg << (2 * HB + 4));
            }
#ifdef EFD_EXP
            int nev = 0;
            if (c > 0 && tid == 0) {
                int mx = 0, sm = 0;
                for (int w = 0; w < NWAVE; ++w) { mx = max(mx, wimb[(c - 1) & 1][w]); sm += wimb[(c - 1) & 1][w]; }
                atomicAdd(&g_exp_count[24], (unsigned long long)mx);
                atomicAdd(&g_exp_count[25], (unsigned long long)sm);
                atomicAdd(&g_exp_count[26], 1ull);
            }
#endif
            for (int ii = 0; ii < nin; ++ii) {
                const uint32_t ha = (uint32_t)__builtin_amdgcn_readlane((int)hdr, ii);
                const int s = (int)((ha >> (2 * HB)) & 1u);
                const int32_t klo = tlo + (int32_t)(ha & HM);
                const int32_t khi = tlo + (int32_t)((ha >> HB) & HM);
                const Item* it = stg + ii;
                if (khi <= e_lo || klo >= e_hi) {              // misses this wave's bins
#ifdef EFD_EXP
                    if (lane == 0) atomicAdd(&g_exp_count[3], 1ull);
#endif
                    continue;
                }
#ifdef EFD_EXP
                ++nev;
                if (lane == 0) {
                    atomicAdd(&g_exp_count[0], 1ull);
                    if (tile < 16384) atomicAdd(&g_exp_tile[tile], 1u);
                }
#endif
                bool anyneed = false;
                bool need[NB];
                {
                    // one body: sub-branch sign (the register state above) and series length as
                    // wave-uniform values
#ifdef EFD_EXP   // records by series length [32..35], sub-branch flips [36]
                    if (lane == 0) {
                        atomicAdd(&g_exp_count[31 + min((int)((ha >> (2 * HB + 1)) & 7u), 4)], 1ull);
                        if (s != s_cur) atomicAdd(&g_exp_count[36], 1ull);
                    }
#endif
                    if (s != s_cur) {
#pragma unroll
                        for (int i = 0; i < NB; ++i) {
                            fk[i] = -fk[i];
                            tfk[i] = -tfk[i];
                            own_i[i] = -own_i[i];
                            mir_i[i] = -mir_i[i];
                        }
                        s_cur = s;
                    }
                    const int J = CAUSTIC == EFD_CAUSTIC_UNIFORM ? (int)((ha >> (2 * HB + 1)) & 7u) : FAST_J;
                    // the stage holds b[s] at b[0] (EFD_GLDS swaps the halves for s = 1)
                    const double* xo = &it->b[0][0][0];
                    const double* xm = &it->b[1][0][0];
                    double wr[NB], wi[NB], w[NB];
                    uint64_t needm[NB], needany = 0;
                    const RecSign rs = rec_sign((ha >> (2 * HB + 4)) & 3u);
#ifdef EFD_EXP   // [29]: wave-records of certified-safe records
                    if (lane == 0 && rs.safe) atomicAdd(&g_exp_count[29], 1ull);
#endif
#ifdef EFD_EXP   // [37]: partial coverage of the wave's bins, [38]: J >= 3, [39]: not certified
                    if (lane == 0) {
                        if ((e_lo - klo) < 0 || (khi - e_hi) < 0) atomicAdd(&g_exp_count[37], 1ull);
                        if (((ha >> HDR_J) & 7u) >= 3u) atomicAdd(&g_exp_count[38], 1ull);
                        if (!((ha >> (HDR_FD + 1)) & 1u)) atomicAdd(&g_exp_count[39], 1ull);
                    }
#endif
                    // envelope records (series length field 0): the straight envelope body when
                    // the record covers the wave's whole chunk, else the same with a lane mask
                    if (CAUSTIC == EFD_CAUSTIC_UNIFORM && !hdr_test(ha, 7u << HDR_J)) {
                        if (!hdr_test((uint32_t)((e_lo - klo) | (khi - e_hi)) >> 31, 1u)) {
                            env_record<false, NB>(it, fk, tfk, sctab, rs, nullptr, wr, wi, w);
                        } else {
                            uint64_t am[NB];
#pragma unroll
                            for (int i = 0; i < NB; ++i) {
                                const int32_t base = e_lo + 64 * i;
                                am[i] = lane_range_mask(klo - base, khi - base);
                            }
                            env_record<true, NB>(it, fk, tfk, sctab, rs, am, wr, wi, w);
                        }
#pragma unroll
                        for (int i = 0; i < NB; ++i) need[i] = false;
                    } else
                    // certified safe, J <= 2 and covering the whole chunk: the straight-line
                    // evaluation (no lane masks, amplitude selects or series branch); the
                    // amplitude cubics and accumulation below are shared
                    if (CAUSTIC == EFD_CAUSTIC_UNIFORM &&
                        !hdr_test(((uint32_t)((e_lo - klo) | (khi - e_hi)) >> 31) |
                                  ((((ha >> HDR_J) & 7u) + 5u) >> 3) |
                                  (((ha >> (HDR_FD + 1)) & 1u) ^ 1u), 1u)) {
#pragma unroll
                        for (int i = 0; i < NB; ++i) {
                            spa_simple(it, fk[i], tfk[i], sctab, rs, wr[i], wi[i], w[i]);
                            need[i] = false;
                        }
                    } else
                    if (CAUSTIC == EFD_CAUSTIC_UNIFORM &&
                        !hdr_test(((uint32_t)((e_lo - klo) | (khi - e_hi)) >> 31) |
                                  (((((ha >> HDR_J) & 7u) ^ 3u) + 7u) >> 3) |
                                  (((ha >> (HDR_FD + 1)) & 1u) ^ 1u), 1u)) {
#pragma unroll
                        for (int i = 0; i < NB; ++i) {
                            spa_simple3(it, fk[i], tfk[i], sctab, rs, wr[i], wi[i], w[i]);
                            need[i] = false;
                        }
                    } else
#pragma unroll
                    for (int i = 0; i < NB; ++i) {
                        const int32_t base = e_lo + 64 * i;
                        const uint64_t am = lane_range_mask(klo - base, khi - base);
                        spa_fast_m<CAUSTIC>(it, fk[i], tfk[i], ha, am, sctab, rs,
                                            wr[i], wi[i], w[i], needm[i]);
                        need[i] = __builtin_amdgcn_inverse_ballot_w64(needm[i]);
                        needany |= needm[i];
                    }
                    anyneed = needany != 0;
                    // the own bins' amplitude cubics (b[0], 16 VGPRs) first, then the mirrors'
                    // (b[1], read after a compiler fence so they can reuse the registers)
#pragma unroll
                    for (int i = 0; i < NB; ++i) {
                        const double xr = cubic(xo, w[i]), xi = cubic(xo + 4, w[i]);
                        own_r[i] = fma(xr, wr[i], own_r[i]);
                        own_r[i] = fma(-xi, wi[i], own_r[i]);
                        own_i[i] = fma(xr, wi[i], own_i[i]);
                        own_i[i] = fma(xi, wr[i], own_i[i]);
                    }
                    if (PAIRED) {
                        asm volatile("" ::: "memory");
#pragma unroll
                        for (int i = 0; i < NB; ++i) {
                            const double zr = cubic(xm, w[i]), zi = cubic(xm + 4, w[i]);
                            mir_r[i] = fma(zr, wr[i], mir_r[i]);
                            mir_r[i] = fma(-zi, wi[i], mir_r[i]);
                            mir_i[i] = fma(-zr, wi[i], mir_i[i]);
                            mir_i[i] = fma(-zi, wr[i], mir_i[i]);
                        }
                    }
                    if (__builtin_expect(anyneed, 0)) {   // cold: general path, some lanes
#ifdef EFD_EXP
                        {
                            unsigned long long nl_ = 0;
#pragma unroll
                            for (int i = 0; i < NB; ++i) nl_ += __popcll(__ballot(need[i]));
                            if (lane == 0) {
                                atomicAdd(&g_exp_count[16], 1ull);
                                atomicAdd(&g_exp_count[17], nl_);
                            }
                        }
#endif
                        const uint32_t key = rfl(keys[c * NC + ii]);
                        const int hg = (int)((key >> 1) / (uint32_t)ni);
                        const int jr = (int)((key >> 1) - (uint32_t)hg * (uint32_t)ni);
                        // the bins' g = -+f are reloaded from the grid around the calls (and
                        // fk, tfk after them), so they are not live across the calls: the
                        // caller-saved copies the kernel's prologue stored for every wave go
                        const int ln = opq(tid0) & 63;
#pragma unroll
                        for (int i = 0; i < NB; ++i) {
                            if (need[i]) {
                                const double f = freq[e_lo + 64 * i + ln];   // k < nlanes here
                                const ColdEval ce = spa_general<CAUSTIC>(
                                    it, s_cur ? f : -f, s, hg, jr, t, nt, K, gm, gn, coefA, coefT);
                                accumulate<0, PAIRED>(ce.wr, ce.wi, ce.b[0], ce.b[1], ce.b[2],
                                                      ce.b[3], own_r[i], own_i[i], mir_r[i],
                                                      mir_i[i]);
                            }
                        }
                        {
                            const int ln2 = opq(tid0) & 63;
#pragma unroll
                            for (int i = 0; i < NB; ++i) {
                                const int32_t k = e_lo + 64 * i + ln2;
                                const double f = k < nlanes ? freq[k] : 0.0;
                                fk[i] = s_cur ? f : -f;
                                tfk[i] = TWO_PI * fk[i];
                            }
                        }
                        // the cold block's reloads retired here, so the loop head needs no
                        // vmcnt wait (which would also wait for the hidden LDS-DMA)
                        __builtin_amdgcn_s_waitcnt(0x0f70);
                    }
                }
            }
#ifdef EFD_EXP
            if (lane == 0) wimb[c & 1][wave] = nev;
#endif
            // retire this wave's LDS-DMA pieces, then the barrier publishes chunk c+1's stage
            __builtin_amdgcn_s_waitcnt(0x0f70);
            __syncthreads();
        }
        nkeys = 0;
        if (pre >= 0) break;   // a prebuilt list is the whole list
    }
#undef EFD_GLDS
    if constexpr (NB < BPL) {
        // the sub-bin form: this workgroup's bins (true signs) to the tile's slot, then the
        // arrival count (cdna_hip_programming.md's in-launch split-K reduction: plain stores ->
        // every wave's vmcnt(0) -> barrier -> lane 0 agent release -> vmcnt(0) -> relaxed agent
        // fetch_add; the last arriver: agent acquire -> vmcnt(0) -> barrier -> plain loads;
        // correct for any placement of the workgroups over XCDs and CUs). Each bin's sum is
        // complete here (all the tile's records, in its order): the slot is a handover, not a
        // reduction, so the spectrum is bitwise the whole tile's
        if (s_cur)
#pragma unroll
            for (int i = 0; i < NB; ++i) { own_i[i] = -own_i[i]; mir_i[i] = -mir_i[i]; }
        const int lt = opq(tid0);
        const int lw = lt >> 6, ll = lt & 63;
        double2* slot = reinterpret_cast<double2*>(spart);
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int li = lw * 64 * BPL + 64 * (ioff + i) + ll;
            slot[2 * li] = make_double2(own_r[i], own_i[i]);
            slot[2 * li + 1] = make_double2(mir_r[i], mir_i[i]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (lt == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const int arrived = __hip_atomic_fetch_add(scnt, 1, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
            const int last = arrived == BPL / NB - 1;
            if (last) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                // re-armed for a later sum on the same preparation (k_segments_one zeroes it too)
                __hip_atomic_store(scnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            part[0] = last;   // "I am last", through an LDS array the tile already has
        }
        __syncthreads();
        if (!part[0]) return;
        const double2* s0 = reinterpret_cast<const double2*>(spart);
        double a_r[BPL], a_i[BPL], m_r[BPL], m_i[BPL];
#pragma unroll
        for (int i = 0; i < BPL; ++i) {
            const int li = lw * 64 * BPL + 64 * i + ll;
            const double2 a = s0[2 * li], m = s0[2 * li + 1];
            a_r[i] = a.x; a_i[i] = a.y; m_r[i] = m.x; m_i[i] = m.y;
        }
        tile_epilogue<PAIRED>(a_r, a_i, m_r, m_i, w_lo, ll, lw, lt, nlanes, nf, k0,
                              accumulate_out, out, hp, hc, lld, llw, llpart, tile);
    } else {
        if (PAIRED && llconst != nullptr && !seen && out == nullptr && hp == nullptr) {
            // no record reached this tile: h = 0 on its bins, whose likelihood partial is the
            // walker-independent one k_ll_tile_const computed with this epilogue's arithmetic
            if (tid == 0) llpart[tile] = llconst[tile];
            return;
        }
        if (s_cur)
#pragma unroll
            for (int i = 0; i < BPL; ++i) { own_i[i] = -own_i[i]; mir_i[i] = -mir_i[i]; }
        tid = opq(tid0);
        tile_epilogue<PAIRED>(own_r, own_i, mir_r, mir_i, w_lo, tid & 63, wave, tid, nlanes, nf,
                              k0, accumulate_out, out, hp, hc, lld, llw, llpart, tile);
    }
#ifdef EFD_EXP
    if (threadIdx.x == 0 && tile < 16384)
        g_exp_tclk[tile] = ((t_start & 0xffffffffull) << 32) | ((wall_clock64() - t_start) & 0xffffffffull);
#endif
}

// The tile's epilogue (whole tile, or the last arriver of a sub-bin split): the spectrum S,
// the symmetric grid's h+ / hx, and the fused likelihood's partial of the tile
template <bool PAIRED>
__device__ __forceinline__ void tile_epilogue(
    double (&own_r)[BPL], double (&own_i)[BPL], double (&mir_r)[BPL], double (&mir_i)[BPL],
    int32_t w_lo, int lane, int wave, int tid, int64_t nlanes, int64_t nf, int64_t k0,
    int accumulate_out, double* __restrict__ out, double* __restrict__ hp,
    double* __restrict__ hc, const double* __restrict__ lld, const double* __restrict__ llw,
    double* __restrict__ llpart, int64_t tile) {
    // S is written when out != NULL; on a symmetric grid h+ and hx of bins [k0, nf) are written
    // straight from the registers when hp != NULL (the lane holds S(k) and S(nf-1-k), the two
    // halves of efd_polarizations' flip), so the likelihood path never stores S
    double2* o = reinterpret_cast<double2*>(out);
    double2* php = reinterpret_cast<double2*>(hp);
    double2* phc = reinterpret_cast<double2*>(hc);
    double llacc = 0.0;   // fused likelihood: this lane's sum of |d - h w|^2
#pragma unroll
    for (int i = 0; i < BPL; ++i) {
        const int64_t k = w_lo + 64 * i + lane;
        if (k >= nlanes) continue;
        const int64_t km = PAIRED ? nf - 1 - k : k;
        double2 sk = make_double2(own_r[i], own_i[i]);
        double2 sm = make_double2(mir_r[i], mir_i[i]);
        if (PAIRED && km == k) {
            sk.x += sm.x;
            sk.y += sm.y;
            sm = sk;
        }
        if (o) {
            if (PAIRED && km != k) {
                double2 vm = sm;
                if (accumulate_out) { const double2 p = o[km]; vm.x += p.x; vm.y += p.y; }
                o[km] = vm;
            }
            double2 v = sk;
            if (accumulate_out) { const double2 p = o[k]; v.x += p.x; v.y += p.y; }
            o[k] = v;
        }
        if (PAIRED && (php || lld)) {
            // h+ = (a + conj b)/2, hx = i (a - conj b)/2 with a = S(j), b = S(nf-1-j)
            auto put = [&](int64_t j, double2 a, double2 b) {
                if (j < k0) return;
                double2 vp = make_double2(0.5 * (a.x + b.x), 0.5 * (a.y - b.y));
                double2 vc = make_double2(-0.5 * (a.y + b.y), 0.5 * (a.x - b.x));
                if (lld) {
                    // d - h w rounded like efd_loglike (product rounded, then difference: no
                    // contraction), so a template equal to the injection gives exactly 0
#pragma clang fp contract(off)
                    const int64_t q = j - k0, nb = nf - k0;
                    const double2 d0 = reinterpret_cast<const double2*>(lld)[q];
                    const double2 d1 = reinterpret_cast<const double2*>(lld)[nb + q];
                    const double w0 = llw[q], w1 = llw[nb + q];
                    const double r0 = d0.x - vp.x * w0, i0 = d0.y - vp.y * w0;
                    const double r1 = d1.x - vc.x * w1, i1 = d1.y - vc.y * w1;
                    llacc = fma(r0, r0, fma(i0, i0, llacc));
                    llacc = fma(r1, r1, fma(i1, i1, llacc));
                }
                if (!php) return;
                if (accumulate_out) {
                    const double2 pp = php[j - k0], pc = phc[j - k0];
                    vp.x += pp.x; vp.y += pp.y; vc.x += pc.x; vc.y += pc.y;
                }
                php[j - k0] = vp;
                phc[j - k0] = vc;
            };
            put(km, sm, sk);
            if (km != k) put(k, sk, sm);
        }
    }
    if (PAIRED && lld) {
        // the tile's partial in a fixed order: a butterfly over each wave, then the waves in turn
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) llacc += __shfl_xor(llacc, o, 64);
        __shared__ double llw4[NWAVE];
        if (lane == 0) llw4[wave] = llacc;
        __syncthreads();
        if (tid == 0) {
            double t = 0.0;
#pragma unroll
            for (int w = 0; w < NWAVE; ++w) t += llw4[w];
            llpart[tile] = t;
        }
    }
}

#define EFD_MODESUM_PARAMS                                                                    \
    const Item* __restrict__ items, const int4* __restrict__ ranges,                          \
        const int2* __restrict__ seglh, const int4* __restrict__ seginfo,                     \
        const int32_t* __restrict__ nsegp, const double* __restrict__ freq, int64_t nf,       \
        int64_t nlanes, int64_t ntiles, int nt, int K, const int32_t* __restrict__ gm,        \
        const int32_t* __restrict__ gn, const double* __restrict__ t,                         \
        const double* __restrict__ coefA, const double* __restrict__ coefT,                   \
        const double2* __restrict__ sctab_g, const uint32_t* __restrict__ tkeys,              \
        const int32_t* __restrict__ tcnt, const int32_t* __restrict__ tperm,                  \
        const int32_t* __restrict__ segbase, const int32_t* __restrict__ stb0,                \
        const int32_t* __restrict__ stb1, Header* __restrict__ hdr, int accumulate_out,       \
        double* __restrict__ out, double* __restrict__ hp, double* __restrict__ hc, int64_t k0
#define EFD_MODESUM_ARGS                                                                      \
    items, ranges, seglh, seginfo, nsegp, freq, nf, nlanes, ntiles, nt, K, gm, gn, t, coefA,  \
        coefT, sctab_g, tkeys, tcnt, tperm, segbase, stb0, stb1, hdr, accumulate_out, out, hp,  \
        hc, k0

// K8: the mode sum (one workgroup per tile; prebuilt lists when tcnt is given)
template <bool PAIRED, int CAUSTIC, int BPL>
__global__ __launch_bounds__(TILE) __attribute__((amdgpu_waves_per_eu(EFD_WAVES_PER_EU, 8)))
void k_modesum(EFD_MODESUM_PARAMS) {
    modesum_tile<PAIRED, CAUSTIC>(EFD_MODESUM_ARGS, nullptr, nullptr, nullptr, nullptr,
                                       (int64_t)blockIdx.x);
}

// K8 over a batch of prepared waveforms in one launch (efd_modesum_sum_batch): workgroup g takes
// waveform g mod n at place g / n of that waveform's dispatch order, so the waveforms' tiles
// interleave longest-first and one launch's ramp, tail and inter-launch gap are shared by n
// waveforms. Each waveform keeps its own workspace and outputs; its tiles run exactly the code of
// a single launch (bitwise the same spectrum). The per-waveform pointers travel in the kernel
// arguments (n <= EFD_BATCH_MAX), read with wave-uniform scalar loads. Config 2 (bench.py, 2
// rounds): 1,238 waveforms/s one sum per launch; 2 / 4 / 8 / 16 per launch 1,311 / 1,331 /
// 1,291 / 1,288 (k_modesum 0.781 -> 0.742 ms per waveform at 4; past 4 the concurrent
// waveforms' records outgrow the caches). Waveform-major order (each waveform's longest-first
// order in turn) measured 1,288 / 1,290 / 1,226 / 1,187.
struct BatchDesc {
    const Item* items;
    const int4* ranges;
    const int2* seglh;
    const int4* seginfo;
    const int32_t* nseg;
    const double* freq;
    const int32_t* gm;
    const int32_t* gn;
    const double* t;
    const double* coefA;
    const double* coefT;
    const double2* sctab;
    const uint32_t* tkeys;
    const int32_t* tcnt;
    const int32_t* tperm;
    const int32_t* segbase;
    const int32_t* stb0;
    const int32_t* stb1;
    Header* hdr;
    double* out;
    double* hp;
    double* hc;
    double* llpart;
    int64_t k0;
    int32_t nt, K;
};
struct SumBatch {
    BatchDesc d[EFD_BATCH_MAX];
    int32_t n;
};
static_assert(sizeof(SumBatch) <= 3584, "batch descriptors must fit the kernel arguments");
// One waveform's logL from its tile partials p (with llconst: tiles outside the lane union take
// their constants): each thread's tiles i, i + 256, ... added in that order, then a tree; out =
// -1/2 * 4 * sum, or NaN when the workspace holds a device-side error flag (the flags stay set:
// efd_modesum_status_batch reports and clears them), so a caller that finds no NaN in the batch
// needs no status synchronisation. 256 threads.
__device__ __forceinline__ void ll_final_reduce(const double* __restrict__ p,
                                                const Header* __restrict__ h,
                                                const double* __restrict__ llconst,
                                                int64_t ntiles, double* __restrict__ out) {
    __shared__ double red[256];
    int64_t t0 = 0, t1 = ntiles - 1;
    if (llconst != nullptr) {
        const int32_t lo = h->lane_lo, hi = h->lane_hi;
        t0 = lo < hi ? lo / TILE_LANES : ntiles;
        t1 = lo < hi ? (int64_t)(hi - 1) / TILE_LANES : -1;
    }
    auto val = [&](int64_t i) { return (i < t0 || i > t1) ? llconst[i] : p[i]; };
    // four loads in flight at a time
    double acc = 0.0;
    int64_t i = threadIdx.x;
    for (; i + 3 * 256 < ntiles; i += 4 * 256) {
        const double v0 = val(i), v1 = val(i + 256), v2 = val(i + 512), v3 = val(i + 768);
        acc += v0;
        acc += v1;
        acc += v2;
        acc += v3;
    }
    for (; i < ntiles; i += 256) acc += val(i);
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const bool bad = h->runs_overflow | h->bad_mn | h->bad_tile;
        *out = bad ? __longlong_as_double(0x7ff8000000000000LL) : -0.5 * 4.0 * red[0];
    }
}
// SPARSE (the fused likelihood with tile constants, no written outputs): only the tiles inside the
// union of the waveform's segment lane ranges ([lane_lo, lane_hi) in its header, k_segment_compact)
// are visited, by nper workgroups per waveform striding over them; k_ll_final takes the constant
// of every tile outside. (Folding k_ll_final into the launch's last workgroup per waveform, with
// agent-scope partial stores and a completion count, made config 4's sum 6 us longer than the two
// kernels: the reduction then runs in the launch's tail.) A sparse spectrum (config 4: 15 harmonics cover 576 of 6,164 tiles) then
// launches a few hundred workgroups per walker instead of one per tile.
template <bool PAIRED, int CAUSTIC, int BPL, bool SPARSE>
__global__ __launch_bounds__(TILE) __attribute__((amdgpu_waves_per_eu(EFD_WAVES_PER_EU, 8)))
void k_modesum_batch(const SumBatch batch, int64_t nf, int64_t nlanes, int64_t ntiles,
                     int accumulate_out, const double* __restrict__ lld,
                     const double* __restrict__ llw, const double* __restrict__ llconst,
                     int64_t nper) {
    const int n = batch.n;
    int w;
    int64_t pos;
    if (lld == nullptr) {
        w = (int)(blockIdx.x % (unsigned)n);
        pos = blockIdx.x / (unsigned)n;
    } else {
        // fused likelihood: the n waveforms of one dispatch place run back to back on one XCD
        // (workgroups are dealt round-robin over the 8 XCDs, x = g mod 8), so the tile's data
        // and weights (48 B per bin, the same for every walker) come from HBM once and from
        // that XCD's L2 for the other n - 1 walkers; place p*8 + x keeps each waveform's
        // place-to-XCD assignment that of a single launch
        const unsigned g = blockIdx.x, r = g >> 3;
        w = (int)(r % (unsigned)n);
        pos = (int64_t)(r / (unsigned)n) * 8 + (g & 7u);
    }
    const BatchDesc& d = batch.d[w];
    if constexpr (SPARSE) {
        const int32_t nit = d.hdr->nitems;
        if (nit > 0) {
            // k_segments_one's split plan: items (tile, bin j, S, slot = counter); S = BPL: the
            // sub-bin form, one bin of every lane per workgroup
            const Layout L = make_layout(d.nt, d.K, nf, 1);
            char* W = reinterpret_cast<char*>(d.hdr);
            const int4* items = ws_at<const int4>(W, L.sitem);
            for (int64_t it = pos; it < nit; it += nper) {
                const int4 e = items[it];
                const int S = e.y & 0xffff, j = e.y >> 16;
                if (S > 1)
                    modesum_tile<PAIRED, CAUSTIC, 1>(
                        d.items, d.ranges, d.seglh, d.seginfo, d.nseg, d.freq, nf, nlanes, ntiles,
                        d.nt, d.K, d.gm, d.gn, d.t, d.coefA, d.coefT, d.sctab, d.tkeys, d.tcnt,
                        d.tperm, d.segbase, d.stb0, d.stb1, d.hdr, accumulate_out, d.out, d.hp,
                        d.hc, d.k0, lld, llw, d.llpart, llconst, e.x, true, j,
                        ws_at<double>(W, L.spart) + (size_t)e.z * TILE_LANES * 4,
                        ws_at<int32_t>(W, L.scnt) + e.w);
                else
                    modesum_tile<PAIRED, CAUSTIC>(
                        d.items, d.ranges, d.seglh, d.seginfo, d.nseg, d.freq, nf, nlanes, ntiles,
                        d.nt, d.K, d.gm, d.gn, d.t, d.coefA, d.coefT, d.sctab, d.tkeys, d.tcnt,
                        d.tperm, d.segbase, d.stb0, d.stb1, d.hdr, accumulate_out, d.out, d.hp,
                        d.hc, d.k0, lld, llw, d.llpart, llconst, e.x, true);
                __syncthreads();   // the next tile's LDS writes after every wave's last reads
            }
            return;
        }
        const int32_t lo = d.hdr->lane_lo, hi = d.hdr->lane_hi;
        if (lo < hi) {
            const int64_t t1 = min((int64_t)(hi - 1) / TILE_LANES, ntiles - 1);
            for (int64_t tile = lo / TILE_LANES + pos; tile <= t1; tile += nper) {
                modesum_tile<PAIRED, CAUSTIC>(
                    d.items, d.ranges, d.seglh, d.seginfo, d.nseg, d.freq, nf, nlanes, ntiles,
                    d.nt, d.K, d.gm, d.gn, d.t, d.coefA, d.coefT, d.sctab, d.tkeys, d.tcnt,
                    d.tperm, d.segbase, d.stb0, d.stb1, d.hdr, accumulate_out, d.out, d.hp, d.hc,
                    d.k0, lld, llw, d.llpart, llconst, tile, true);
                __syncthreads();   // the next tile's LDS writes after every wave's last reads
            }
        }
        return;
    }
    modesum_tile<PAIRED, CAUSTIC>(
        d.items, d.ranges, d.seglh, d.seginfo, d.nseg, d.freq, nf, nlanes, ntiles, d.nt, d.K,
        d.gm, d.gn, d.t, d.coefA, d.coefT, d.sctab, d.tkeys, d.tcnt, d.tperm, d.segbase, d.stb0,
        d.stb1, d.hdr, accumulate_out, d.out, d.hp, d.hc, d.k0, lld, llw, d.llpart, llconst, pos);
}

// The fused likelihood's partial of a tile whose waveform has no record on it (every bin's
// h = 0): modesum_tile's epilogue with zero accumulators, the same operations in the same order,
// so a tile that takes it (llconst) gives bitwise what computing it would. Depends on the grid
// (nf, the paired tile layout), k0, d and w only: once per likelihood.
template <int BPL>
__global__ __launch_bounds__(TILE) void k_ll_tile_const(const double* __restrict__ lld,
                                                        const double* __restrict__ llw,
                                                        int64_t nf, int64_t nlanes, int64_t k0,
                                                        double* __restrict__ llconst) {
    const int64_t tile = blockIdx.x;
    // modesum_tile's FP modes, so the epilogue's arithmetic rounds the same
    __builtin_amdgcn_s_setreg(1 | (6 << 6) | (1 << 11), 0);
    __builtin_amdgcn_s_setreg(1 | (9 << 6), 0);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int32_t w_lo = (int32_t)(tile * TILE_LANES + wave * 64 * BPL);
    double llacc = 0.0;
#pragma unroll
    for (int i = 0; i < BPL; ++i) {
        const int64_t k = w_lo + 64 * i + lane;
        if (k >= nlanes) continue;
        const int64_t km = nf - 1 - k;
        double2 sk = make_double2(0.0, 0.0);
        double2 sm = make_double2(0.0, 0.0);
        if (km == k) {
            sk.x += sm.x;
            sk.y += sm.y;
            sm = sk;
        }
        auto put = [&](int64_t j, double2 a, double2 b) {
            if (j < k0) return;
            double2 vp = make_double2(0.5 * (a.x + b.x), 0.5 * (a.y - b.y));
            double2 vc = make_double2(-0.5 * (a.y + b.y), 0.5 * (a.x - b.x));
            {
#pragma clang fp contract(off)
                const int64_t q = j - k0, nb = nf - k0;
                const double2 d0 = reinterpret_cast<const double2*>(lld)[q];
                const double2 d1 = reinterpret_cast<const double2*>(lld)[nb + q];
                const double w0 = llw[q], w1 = llw[nb + q];
                const double r0 = d0.x - vp.x * w0, i0 = d0.y - vp.y * w0;
                const double r1 = d1.x - vc.x * w1, i1 = d1.y - vc.y * w1;
                llacc = fma(r0, r0, fma(i0, i0, llacc));
                llacc = fma(r1, r1, fma(i1, i1, llacc));
            }
        };
        put(km, sm, sk);
        if (km != k) put(k, sk, sm);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) llacc += __shfl_xor(llacc, o, 64);
    __shared__ double llw4[NWAVE];
    if (lane == 0) llw4[wave] = llacc;
    __syncthreads();
    if (tid == 0) {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < NWAVE; ++w) t += llw4[w];
        llconst[tile] = t;
    }
}

// Fused likelihood, second stage: waveform i's out[i] = -1/2 * 4 * (sum of its tiles' partials),
// one workgroup per waveform, fixed order (a strided pass per thread, then a tree)
struct LlBatch {
    const double* part[EFD_BATCH_MAX];
    const Header* hdr[EFD_BATCH_MAX];
    double* out;
    const double* llconst;   // sparse sum: the constants of the tiles outside each lane union
    int64_t ntiles;
    int32_t n;
};
// efd_modesum_status_batch: each workspace's error flags (bit 0 runs_overflow, 1 bad_mn,
// 2 bad_tile) into out[i], and the reported flags cleared (sticky until reported; see Header)
struct StatusBatch {
    Header* h[EFD_BATCH_MAX];
    int32_t n;
};
// efd_modesum_lane_ranges: each workspace's [lane_lo, lane_hi) (k_segment_compact's union of the
// segments' lane ranges) into out[2 i], out[2 i + 1]
__global__ __launch_bounds__(64) void k_lane_gather(const StatusBatch sb, int32_t* out) {
    const int i = threadIdx.x;
    if (i >= sb.n) return;
    out[2 * i] = sb.h[i]->lane_lo;
    out[2 * i + 1] = sb.h[i]->lane_hi;
}
__global__ __launch_bounds__(64) void k_status_gather(const StatusBatch sb, int32_t* out) {
    const int i = threadIdx.x;
    if (i >= sb.n) return;
    Header* h = sb.h[i];
    const int32_t f = (h->runs_overflow ? 1 : 0) | (h->bad_mn ? 2 : 0) | (h->bad_tile ? 4 : 0);
    out[i] = f;
    if (f) {
        h->runs_overflow = 0;
        h->bad_mn = 0;
        h->bad_tile = 0;
    }
}

__global__ __launch_bounds__(256) void k_ll_final(const LlBatch lb) {
    ll_final_reduce(lb.part[blockIdx.x], lb.hdr[blockIdx.x], lb.llconst, lb.ntiles,
                           lb.out + blockIdx.x);
}

// K6: the tiles' record lists, built in the preparation phase (k_modesum DMAs them in). The same
// keys in the same order as the sum's own build (segments in table order; each segment's records
// reaching the tile, [p0, p1) from the segment-tile boundaries or by bisection; the keys of each
// SEGWIN window of segment ids scattered by x -> P x mod n over that window), computed in one
// pass over the tile's hits instead of window by window: the segment table is read in batches
// of 8 windows per barrier, the hits' boundaries and counts in one round of loads, one block
// scan places them, and each thread then writes keys found by bisection over the hit offsets.
// The sum's build waits for every window's loads, scans and barriers in turn (~7.7 us per tile
// alone at config 2, 37 us for the launch); this kernel shares the GPU with the previous
// waveform's sum, so its resident time is what it costs. Tiles with more than TK_HITS hits or
// KEYCAP keys get tcnt = -1 and build in the sum.
constexpr int TK_HITS = TILE;
constexpr int TK_ROWS = 8;   // windows of the segment table per barrier
__device__ __forceinline__ void tile_keys_body(
    const int4* __restrict__ ranges, const int2* __restrict__ seglh,
    const int4* __restrict__ seginfo, const int32_t* __restrict__ nsegp,
    const int32_t* __restrict__ segbase, const int32_t* __restrict__ stb0,
    const int32_t* __restrict__ stb1, int64_t ntiles, uint32_t* __restrict__ tkeys,
    int32_t* __restrict__ tcnt) {
    static_assert(SEGWIN == TILE, "one segment per thread and window row");
    __shared__ int hits[TK_HITS], hp0[TK_HITS], hcnt[TK_HITS], hoff[TK_HITS], hws[TK_HITS],
        hwt[TK_HITS];
    __shared__ int4 hinfo[TK_HITS];
    __shared__ int wcnt[TK_ROWS * NWAVE];
    __shared__ int part[NWAVE];
    const int64_t tile = blockIdx.x;
    if (tile >= ntiles) return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int32_t tlo = (int32_t)(tile * TILE_LANES), thi = tlo + TILE_LANES;
    const int nseg = *nsegp;
#ifdef EFD_EXP   // segment table size [27], hits per tile summed [28]
    if (tile == 0 && tid == 0) atomicAdd(&g_exp_count[27], (unsigned long long)nseg);
#endif
    // (1) the segments overlapping the tile, in table order
    int nhit = 0;
    for (int base = 0; base < nseg; base += TK_ROWS * TILE) {
        unsigned long long bal[TK_ROWS];
#pragma unroll
        for (int r = 0; r < TK_ROWS; ++r) {
            const int sgi = base + r * TILE + tid;
            bool hit = false;
            if (sgi < nseg) {
                const int2 lh = seglh[sgi];
                hit = lh.y > tlo && lh.x < thi;
            }
            bal[r] = __ballot(hit);
            if (lane == 0) wcnt[r * NWAVE + wave] = __popcll(bal[r]);
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < TK_ROWS; ++r) {
            int before = nhit;
            for (int w = 0; w < wave; ++w) before += wcnt[r * NWAVE + w];
            if ((bal[r] >> lane) & 1ull) {
                const int pos = before + __popcll(bal[r] & ((1ull << lane) - 1ull));
                if (pos < TK_HITS) hits[pos] = base + r * TILE + tid;
            }
#pragma unroll
            for (int w = 0; w < NWAVE; ++w) nhit += wcnt[r * NWAVE + w];
        }
        __syncthreads();
    }
#ifdef EFD_EXP
    if (tid == 0) atomicAdd(&g_exp_count[28], (unsigned long long)nhit);
#endif
    if (nhit > TK_HITS) {
        if (tid == 0) tcnt[tile] = -1;
        return;
    }
    // (2) each hit's records reaching into the tile: [p0, p1)
    int c = 0;
    if (tid < nhit) {
        const int sg = hits[tid];
        const int32_t sbase = segbase[sg];
        const int4 info = seginfo[sg];
        int p0 = 0;
        if (sbase != SEG_NO_STB) {
            p0 = stb0[sbase + tile];
            c = max(stb1[sbase + tile] - p0, 0);
        } else {
            const int base = info.x, n = info.y, dir = info.z, sb = info.w;
            int lo = 0, hi = n;            // first p (lane order) with khi > tlo
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                const int4 rg = ranges[base + (dir > 0 ? mid : n - 1 - mid)];
                if ((sb ? rg.w : rg.y) > tlo) hi = mid; else lo = mid + 1;
            }
            p0 = lo;
            hi = n;                        // first p with klo >= thi
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                const int4 rg = ranges[base + (dir > 0 ? mid : n - 1 - mid)];
                if ((sb ? rg.z : rg.x) >= thi) hi = mid; else lo = mid + 1;
            }
            c = lo - p0;
        }
        hp0[tid] = p0;
        hcnt[tid] = c;
        hinfo[tid] = info;
    }
    // (3) exclusive scan of the counts
    int incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    if (lane == 63) part[wave] = incl;
    __syncthreads();
    int total = 0, woff = 0;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) {
        woff += w < wave ? part[w] : 0;
        total += part[w];
    }
    if (total > KEYCAP) {
        if (tid == 0) tcnt[tile] = -1;
        return;
    }
    if (tid < nhit) hoff[tid] = woff + incl - c;
    __syncthreads();
    // (4) each hit's SEGWIN window: where its keys start and how many it holds (the scatter's
    // range). Hits are in table order, so a window's hits are consecutive: the window's start
    // is a max-scan of the offsets at window starts, its end a min-scan from the right of the
    // offsets past window ends
    {
        const int w = tid < nhit ? hits[tid] / SEGWIN : INT32_MAX;
        const bool first = tid < nhit && (tid == 0 || hits[tid - 1] / SEGWIN != w);
        const bool last = tid < nhit && (tid == nhit - 1 || hits[tid + 1] / SEGWIN != w);
        int st = first ? woff + incl - c : INT32_MIN;       // this hit's offset = hoff[tid]
        int en = last ? woff + incl : INT32_MAX;            // hoff[tid] + hcnt[tid]
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int vs = __shfl_up(st, o, 64), ve = __shfl_down(en, o, 64);
            if (lane >= o) st = max(st, vs);
            if (lane + o < 64) en = min(en, ve);
        }
        if (lane == 63) hws[wave] = st;   // wave carries (hws, hwt reused as scratch)
        if (lane == 0) hwt[wave] = en;
        __syncthreads();
        for (int v = 0; v < wave; ++v) st = max(st, hws[v]);
        for (int v = NWAVE - 1; v > wave; --v) en = min(en, hwt[v]);
        __syncthreads();
        if (tid < nhit) {
            hws[tid] = st;
            hwt[tid] = en - st;
        }
    }
    __syncthreads();
    // (5) the keys: position g of the list lies in hit i (bisection over the offsets)
    uint32_t* out = tkeys + (size_t)tile * KEYCAP;
    for (int g = tid; g < total; g += TILE) {
        int lo = 0, hi = nhit - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (hoff[mid] <= g) lo = mid; else hi = mid - 1;
        }
        const int4 info = hinfo[lo];
        const int p = hp0[lo] + (g - hoff[lo]);
        const int j = info.z > 0 ? p : info.y - 1 - p;
        const int ws = hws[lo], take = hwt[lo];
        const int P = (take % 97) ? 97 : 101;
        out[ws + (int)(((unsigned)(g - ws) * (unsigned)P) % (unsigned)take)] =
            ((uint32_t)(info.x + j) << 1) | (uint32_t)info.w;
    }
    if (tid == 0) tcnt[tile] = total;
}
__global__ __launch_bounds__(TILE) void k_tile_keys(const PrepBatch B) {
    PREP_WALKER(B);
    if (D.lists == 0) return;
    tile_keys_body(ws_at<int4>(W, L.ranges), ws_at<int2>(W, L.seglh), ws_at<int4>(W, L.seginfo),
                   ws_at<int32_t>(W, L.nseg), ws_at<int32_t>(W, L.segbase),
                   ws_at<int32_t>(W, L.stb0), ws_at<int32_t>(W, L.stb1), L.ntiles,
                   ws_at<uint32_t>(W, L.tkeys), ws_at<int32_t>(W, L.tcnt));
}
#undef EFD_MODESUM_PARAMS
#undef EFD_MODESUM_ARGS

// K7: dispatch order for the sum, most expensive tiles first (longest-processing-time list
// scheduling). Cost = the tile's record count from k_tile_keys (tcnt; -1, a list over one
// KEYCAP pass, is the most expensive class), bucketed at quarter octaves: a counting sort in
// LDS by one workgroup. The order within a bucket follows LDS atomics and may vary from run to
// run; it changes only which block runs a tile, never a tile's arithmetic, so the spectrum is
// bitwise the same in every order.
constexpr int ORDER_BUCKETS = 64;
__device__ __forceinline__ int tile_cost_bucket(int32_t c) {
    if (c < 0) return ORDER_BUCKETS - 1;
    const float l = __log2f((float)c + 1.0f) * 4.0f;
    return min((int)l, ORDER_BUCKETS - 2);
}
// Wave-aggregated LDS atomic: the lanes of a wave holding the same bucket take one add by their
// lowest lane (a tile list's neighbours mostly share a bucket, so one add serves many lanes
// instead of a contended add per lane); returns the old value plus the lane's rank among them.
__device__ __forceinline__ int wave_bucket_add(int* hist, int bucket, bool valid) {
    const int lane = threadIdx.x & 63;
    unsigned long long todo = __ballot(valid);
    int res = 0;
    while (todo) {
        const int leader = __ffsll((long long)todo) - 1;
        const int bl = __shfl(bucket, leader, 64);
        const unsigned long long same = __ballot(valid && bucket == bl) & todo;
        int base = 0;
        if (lane == leader) base = atomicAdd(&hist[bl], __popcll(same));
        base = __shfl(base, leader, 64);
        if ((same >> lane) & 1ull) res = base + __popcll(same & ((1ull << lane) - 1ull));
        todo &= ~same;
    }
    return res;
}
__device__ __forceinline__ void tile_order_body(const int32_t* __restrict__ tcnt,
                                                int64_t ntiles, int32_t* __restrict__ tperm) {
    __shared__ int hist[ORDER_BUCKETS];
    const int tid = threadIdx.x;
    if (tid < ORDER_BUCKETS) hist[tid] = 0;
    __syncthreads();
    // the first 16 x 1024 tiles' buckets stay in registers: one round of independent loads
    // instead of a dependent load-atomic chain per pass (the sort sits on the preparation
    // phase's critical path at small harmonic counts); every lane of a wave runs the same
    // number of passes (wave_bucket_add's ballots need the whole wave)
    constexpr int PER = 16;
    int bk[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int64_t i = tid + (int64_t)q * 1024;
        bk[q] = i < ntiles ? tile_cost_bucket(tcnt[i]) : -1;
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) wave_bucket_add(hist, bk[q], bk[q] >= 0);
    const int64_t npass = (ntiles + 1023) / 1024;
    for (int64_t p = PER; p < npass; ++p) {
        const int64_t i = tid + p * 1024;
        const int bkt = i < ntiles ? tile_cost_bucket(tcnt[i]) : 0;
        wave_bucket_add(hist, bkt, i < ntiles);
    }
    __syncthreads();
    if (tid == 0) {   // exclusive scan, most expensive bucket first
        int acc = 0;
        for (int q = ORDER_BUCKETS - 1; q >= 0; --q) { const int h = hist[q]; hist[q] = acc; acc += h; }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int pos = wave_bucket_add(hist, bk[q], bk[q] >= 0);
        if (bk[q] >= 0) tperm[pos] = (int32_t)(tid + q * 1024);
    }
    for (int64_t p = PER; p < npass; ++p) {
        const int64_t i = tid + p * 1024;
        const int bkt = i < ntiles ? tile_cost_bucket(tcnt[i]) : 0;
        const int pos = wave_bucket_add(hist, bkt, i < ntiles);
        if (i < ntiles) tperm[pos] = (int32_t)i;
    }
}
__global__ __launch_bounds__(1024) void k_tile_order(const PrepBatch B) {
    PREP_WALKER(B);
    if (D.lists != 3) return;
    tile_order_body(ws_at<int32_t>(W, L.tcnt), L.ntiles, ws_at<int32_t>(W, L.tperm));
}

// ----------------------------------------------------------------------------------------
// K9: TD mode sum (FEW's InterpolatedModeSum [FEW-ext]; the reference's comparison path,
// check_mode_by_mode.py:85-99, 254-264). Sample-stationary: each
// thread owns TD_SPL samples t_i = i dt (strided by the block, so loads and stores coalesce).
// The (m, n) groups of k_group are walked in descending (m, n) order and, per m, summed by
// Horner's rule in z = e^{-i Phi_r}:
//   h(t) = - sum_m [ b_m P_m + conj(b_m Q_m) ],   b_m = e^{-i (m Phi_phi + n0 Phi_r)},
//   P_m = sum_n Bp_mn(t) z^(n - n0),  Q_m = sum_n Bm_mn(t) z^(n - n0),  n0 = min n of m,
// so a group costs its four amplitude cubics and two complex multiply-adds (20 FP64 FMAs); a
// sample pays one sin/cos for z and one per distinct m. Bp, Bm are k_group_amp's group
// amplitudes (they carry -scale Y+ and conj(-scale Y-): hence the leading minus, and the
// partner term conj(Bm e^{-i Phi}) = scale Y- conj(A) e^{+i Phi}). A gap in n multiplies by z
// once more per missing n. The knot interval is wave-uniform except in the few waves that
// straddle a knot; those read the amplitude coefficients per lane.
// ----------------------------------------------------------------------------------------
constexpr int TD_THREADS = 256;
constexpr int TD_SPL = 4;   // samples per thread

// scipy's interval choice: i with t_i <= x < t_{i+1}, clamped to [0, nt - 2]
__device__ __forceinline__ int knot_interval(const double* __restrict__ t, int nt, double x) {
    int lo = 0, hi = nt - 1;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (t[mid] <= x) lo = mid; else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(TD_THREADS) void k_td_modesum(
    const double* __restrict__ t, int nt, const double* __restrict__ coefT,
    const double* __restrict__ coefA, const int32_t* __restrict__ gm,
    const int32_t* __restrict__ gn, int K, const Header* __restrict__ hdr, double dt,
    int64_t ns, int accumulate_out, double* __restrict__ out, double* __restrict__ hp,
    double* __restrict__ hc) {
    const int64_t s_base = (int64_t)blockIdx.x * (TD_THREADS * TD_SPL) + threadIdx.x;
    const double t_end = t[nt - 1];
    const int G = hdr->groups;
    double w[TD_SPL], pphi[TD_SPL], pr[TD_SPL], zr[TD_SPL], zi[TD_SPL];
    int jj[TD_SPL];
    bool valid[TD_SPL];
    bool any_valid = false;
#pragma unroll
    for (int i = 0; i < TD_SPL; ++i) {
        const int64_t s = s_base + (int64_t)i * TD_THREADS;
        const double ts = (double)s * dt;
        valid[i] = s < ns && ts <= t_end;
        any_valid |= valid[i];
        // samples past the end share the last interval, keeping the wave uniform there
        jj[i] = valid[i] ? knot_interval(t, nt, ts) : nt - 2;
        w[i] = valid[i] ? ts - t[jj[i]] : 0.0;
        const double* ct = coefT + (size_t)jj[i] * 32;
        pphi[i] = fma(fma(fma(ct[0], w[i], ct[8]), w[i], ct[16]), w[i], ct[24]);
        pr[i] = fma(fma(fma(ct[1], w[i], ct[9]), w[i], ct[17]), w[i], ct[25]);
        double sn, cs;
        sincos_big(pr[i], sn, cs);
        zr[i] = cs;
        zi[i] = -sn;
    }
    double Hr[TD_SPL], Hi[TD_SPL];
#pragma unroll
    for (int i = 0; i < TD_SPL; ++i) Hr[i] = Hi[i] = 0.0;

    if (__any(any_valid) && G > 0) {
        const int j0 = (int)rfl((uint32_t)jj[0]);
        bool same = true;
#pragma unroll
        for (int i = 0; i < TD_SPL; ++i) same &= jj[i] == j0;
        const size_t row = (size_t)4 * 4 * K;   // doubles per interval of coefA
        auto run = [&](auto UNI) {
            constexpr bool U = decltype(UNI)::value;
            double Pr[TD_SPL], Pi[TD_SPL], Qr[TD_SPL], Qi[TD_SPL];
#pragma unroll
            for (int i = 0; i < TD_SPL; ++i) Pr[i] = Pi[i] = Qr[i] = Qi[i] = 0.0;
            auto flush = [&](int m, int n0) {
#pragma unroll
                for (int i = 0; i < TD_SPL; ++i) {
                    double sn, cs;
                    sincos_big(fma((double)m, pphi[i], (double)n0 * pr[i]), sn, cs);
                    const double br = cs, bi = -sn;   // b = e^{-i (m Phi_phi + n0 Phi_r)}
                    // b P + conj(b Q)
                    Hr[i] += (br * Pr[i] - bi * Pi[i]) + (br * Qr[i] - bi * Qi[i]);
                    Hi[i] += (br * Pi[i] + bi * Pr[i]) - (br * Qi[i] + bi * Qr[i]);
                    Pr[i] = Pi[i] = Qr[i] = Qi[i] = 0.0;
                }
            };
            int cur_m = gm[G - 1], nprev = gn[G - 1];
            for (int g = G - 1; g >= 0; --g) {
                const int m = gm[g], n = gn[g];
                int d = nprev - n;
                if (m != cur_m) {
                    flush(cur_m, nprev);
                    cur_m = m;
                    d = 1;   // P = Q = 0: the Horner step below reduces to P = Bp
                }
                nprev = n;
                for (; d > 1; --d) {   // missing n between two groups of this m
#pragma unroll
                    for (int i = 0; i < TD_SPL; ++i) {
                        const double a = Pr[i], b = Qr[i];
                        Pr[i] = fma(a, zr[i], -Pi[i] * zi[i]);
                        Pi[i] = fma(a, zi[i], Pi[i] * zr[i]);
                        Qr[i] = fma(b, zr[i], -Qi[i] * zi[i]);
                        Qi[i] = fma(b, zi[i], Qi[i] * zr[i]);
                    }
                }
#pragma unroll
                for (int i = 0; i < TD_SPL; ++i) {
                    const double* ca = coefA + (size_t)(U ? j0 : jj[i]) * row + 4 * g;
                    const double wi = w[i];
                    const double bpr = fma(fma(fma(ca[0], wi, ca[4 * K]), wi, ca[8 * K]), wi, ca[12 * K]);
                    const double bpi = fma(fma(fma(ca[1], wi, ca[4 * K + 1]), wi, ca[8 * K + 1]), wi, ca[12 * K + 1]);
                    const double bmr = fma(fma(fma(ca[2], wi, ca[4 * K + 2]), wi, ca[8 * K + 2]), wi, ca[12 * K + 2]);
                    const double bmi = fma(fma(fma(ca[3], wi, ca[4 * K + 3]), wi, ca[8 * K + 3]), wi, ca[12 * K + 3]);
                    // P = P z + Bp, Q = Q z + Bm
                    const double a = Pr[i], b = Qr[i];
                    Pr[i] = fma(a, zr[i], fma(-Pi[i], zi[i], bpr));
                    Pi[i] = fma(a, zi[i], fma(Pi[i], zr[i], bpi));
                    Qr[i] = fma(b, zr[i], fma(-Qi[i], zi[i], bmr));
                    Qi[i] = fma(b, zi[i], fma(Qi[i], zr[i], bmi));
                }
            }
            flush(cur_m, nprev);
        };
        if (__all(same)) run(std::integral_constant<bool, true>{});
        else run(std::integral_constant<bool, false>{});
    }

    double2* o = reinterpret_cast<double2*>(out);
#pragma unroll
    for (int i = 0; i < TD_SPL; ++i) {
        const int64_t s = s_base + (int64_t)i * TD_THREADS;
        if (s >= ns) continue;
        // h = h+ - i hx = -H (zero past the trajectory's end: pad_output)
        double vr = valid[i] ? -Hr[i] : 0.0, vi = valid[i] ? -Hi[i] : 0.0;
        if (o) {
            double2 v = make_double2(vr, vi);
            if (accumulate_out) { const double2 p = o[s]; v.x += p.x; v.y += p.y; }
            o[s] = v;
        }
        if (hp) hp[s] = accumulate_out ? hp[s] + vr : vr;
        if (hc) hc[s] = accumulate_out ? hc[s] - vi : -vi;
    }
}

// h+ / hx split with FEW's array flip
__global__ void k_polarizations(const double2* __restrict__ S, int64_t nf, int64_t k0,
                                double2* __restrict__ hp, double2* __restrict__ hc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t k = k0 + i;
    if (k >= nf) return;
    const double2 a = S[k], b = S[nf - 1 - k];
    // h+ = (a + conj b)/2 ; hx = i (a - conj b)/2
    hp[i] = make_double2(0.5 * (a.x + b.x), 0.5 * (a.y - b.y));
    hc[i] = make_double2(-0.5 * (a.y + b.y), 0.5 * (a.x - b.x));
}

// ---- The Hann window's convolution (fdutils.HannConvolution; efd_hann_*). A row's correction
// C = K (*) S (circular, mod nf) is the linear convolution of the row's support [first, last) with
// the lag kernel, on m-point transforms (m >= nf + (last - first) - 1): the caller's Y[s] holds
// S[first + s] / scale for s < last - first, zero up to m (efd_hann_stage), and after its
// transforms (the kernel's spectrum includes 1/m) C[k] = scale Y[((k - first) mod nf) + m - nf].
// info[r] = {bits of scale = max(|Re|, |Im|), first nonzero bin, last nonzero bin + 1, 0}; a
// NaN anywhere in the row makes the scale NaN (the bit pattern orders above every finite
// value), so the row's outputs are NaN.
__global__ void k_hann_info_init(uint64_t* __restrict__ info, int32_t rows) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    info[4 * r + 0] = 0;
    info[4 * r + 1] = ~0ull;
    info[4 * r + 2] = 0;
    info[4 * r + 3] = 0;
}
// lanes (optional, int32 [rows][2]): each row's paired-grid lane range from its mode sum
// (efd_modesum_lane_ranges); bins outside {l, nf-1-l : lo <= l < hi} hold no term, so the scan
// covers [min(lo, nf-hi), max(hi, nf-lo)) only
__global__ __launch_bounds__(256) void k_hann_extent(const double2* __restrict__ S, int64_t stride,
                                                     int64_t nf, const int32_t* __restrict__ lanes,
                                                     uint64_t* __restrict__ info) {
    const double2* row = S + (int64_t)blockIdx.y * stride;
    int64_t k_lo = 0, k_hi = nf;
    if (lanes != nullptr) {
        const int64_t llo = lanes[2 * blockIdx.y], lhi = lanes[2 * blockIdx.y + 1];
        if (llo >= lhi) {
            k_hi = 0;   // no segment: an all-zero row
        } else {
            k_lo = max((int64_t)0, min(llo, nf - lhi));
            k_hi = min(nf, max(lhi, nf - llo));
        }
    }
    uint64_t mx = 0, lo = ~0ull, hi = 0;
#pragma unroll 8
    for (int64_t k = k_lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < k_hi;
         k += (int64_t)gridDim.x * blockDim.x) {
        const double2 v = row[k];
        const uint64_t bx = (uint64_t)__double_as_longlong(fabs(v.x));
        const uint64_t by = (uint64_t)__double_as_longlong(fabs(v.y));
        mx = max(mx, max(bx, by));
        if ((bx | by) != 0) {          // nonzero (or NaN)
            lo = min(lo, (uint64_t)k);
            hi = (uint64_t)k + 1;      // k grows along the thread's stride
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mx = max(mx, (uint64_t)__shfl_xor((unsigned long long)mx, o, 64));
        lo = min(lo, (uint64_t)__shfl_xor((unsigned long long)lo, o, 64));
        hi = max(hi, (uint64_t)__shfl_xor((unsigned long long)hi, o, 64));
    }
    // the block's 4 waves through LDS, then one thread's 3 atomics per block (a few hundred
    // per row: contention on the row's 3 words stays small)
    __shared__ uint64_t red[3][4];
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][wv] = mx;
        red[1][wv] = lo;
        red[2][wv] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < 4; ++i) {
            mx = max(mx, red[0][i]);
            lo = min(lo, red[1][i]);
            hi = max(hi, red[2][i]);
        }
        uint64_t* in = info + 4 * blockIdx.y;
        if (mx) atomicMax((unsigned long long*)&in[0], (unsigned long long)mx);
        if (hi) {
            atomicMin((unsigned long long*)&in[1], (unsigned long long)lo);
            atomicMax((unsigned long long*)&in[2], (unsigned long long)hi);
        }
    }
}
struct HannRow {
    int64_t first, len;
    double scale;   // 0 for an all-zero row (its Y is zero)
};
__device__ __forceinline__ HannRow hann_row(const uint64_t* __restrict__ info, int r) {
    HannRow h;
    const uint64_t lo = info[4 * r + 1], hi = info[4 * r + 2];
    h.first = hi ? (int64_t)lo : 0;
    h.len = hi ? (int64_t)(hi - lo) : 0;
    h.scale = __longlong_as_double((long long)info[4 * r + 0]);
    return h;
}
__global__ __launch_bounds__(256) void k_hann_stage(const double2* __restrict__ S, int64_t stride,
                                                    const uint64_t* __restrict__ info, int64_t m,
                                                    float2* __restrict__ Y) {
    const int r = blockIdx.y;
    const HannRow h = hann_row(info, r);
    const double2* row = S + (int64_t)r * stride + h.first;
    float2* y = Y + (int64_t)r * m;
    const double inv = h.scale == 0.0 ? 0.0 : 1.0 / h.scale;   // NaN scale: NaN row
    const bool bad = h.len > m;     // the host sized m from info: never, but never write past Y
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < m;
         s += (int64_t)gridDim.x * blockDim.x) {
        float2 v = make_float2(0.f, 0.f);
        if (bad) {
            v = make_float2(__int_as_float(0x7fc00000), 0.f);
        } else if (s < h.len) {
            const double2 x = row[s];
            v = make_float2((float)(x.x * inv), (float)(x.y * inv));
        }
        y[s] = v;
    }
}
// ---- The Hann correction's convolution as one four-step FFT pipeline (efd_hann_convolve).
// Y = ifft_m(fft_m(y) * kf) for power-of-two m = R * C, C = 8192, R = m / C (256..4096), in
// complex64, with y the scaled support of each row (efd_hann_stage's values, computed on the
// fly). Index s = C r + c (row r, column c), frequency f = f_r + R f_c:
//   (A) columns: length-R FFT over r of every column c, times w_m^(c f_r)   -> [f_r][c]
//   (B) rows:    length-C FFT over c of every row f_r gives X[f_r + R f_c] at [f_r][f_c]; times
//                the lag kernel's spectrum in the same order (kfp[f_r C + f_c] = kf[f_r + R f_c],
//                1/m included); inverse length-C FFT                           -> [f_r][c]
//   (C) columns: times w_m^(-c f_r), inverse length-R FFT over f_r          -> [r][c] = Y[s]
// The spectrum is never put in natural order: the two transposes on each side of rocFFT's
// 2^24-point transform (five kernels per direction) and the separate stage and multiply passes
// are gone; three passes over Y remain. Stockham radix-8 passes (a radix-4 or -2 one last) in
// LDS, ~70 KB per workgroup so two share a CU (one's global loads overlap the other's
// transforms), twiddles from __sincosf (absolute error ~5e-7: the correction needs ~3 digits).
constexpr int FC_C = 8192;             // row length (LDS: 8192 x 8 B + 1/16 padding = 68 KB)
constexpr int FC_NT = 512;             // threads of a column or row workgroup
constexpr float FC_2PI = 6.283185307179586f;
constexpr float FC_SQRT_HALF = 0.70710678118654752f;

// complex64 values as 2-wide float vectors: the arithmetic below compiles to packed FP32
// instructions (v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32, one issue slot per complex add or
// half a complex multiply), about half the VALU instructions of scalar float2 code
typedef float fcv __attribute__((ext_vector_type(2)));
__device__ __forceinline__ fcv cmulf(fcv a, fcv b) {
    const fcv t = a.xx * b;
    return __builtin_elementwise_fma(a.yy, b.yx * (fcv){-1.0f, 1.0f}, t);
}
// x times -i (SIGN -1) or +i (SIGN +1)
template <int SIGN>
__device__ __forceinline__ fcv cmuli(fcv x) {
    return x.yx * (SIGN < 0 ? (fcv){1.0f, -1.0f} : (fcv){-1.0f, 1.0f});
}
// natural-order DFTs of 4 and 8 points in registers, exp(SIGN 2 pi i n k / N)
template <int SIGN>
__device__ __forceinline__ void fc_dft4(fcv& a0, fcv& a1, fcv& a2, fcv& a3) {
    const fcv t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3;
    const fcv t3 = cmuli<SIGN>(a1 - a3);
    a0 = t0 + t2;
    a1 = t1 + t3;
    a2 = t0 - t2;
    a3 = t1 - t3;
}
template <int SIGN>
__device__ __forceinline__ void fc_dft8(fcv* v) {
    fcv e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
    fcv o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
    fc_dft4<SIGN>(e0, e1, e2, e3);
    fc_dft4<SIGN>(o0, o1, o2, o3);
    // o_k times w8^k, w8 = (1 + SIGN i) / sqrt 2: w8 o = (o + SIGN i o) / sqrt 2,
    // w8^3 o = (-o + SIGN i o) / sqrt 2
    o1 = FC_SQRT_HALF * (o1 + cmuli<SIGN>(o1));
    o2 = cmuli<SIGN>(o2);
    o3 = FC_SQRT_HALF * (cmuli<SIGN>(o3) - o3);
    v[0] = e0 + o0;
    v[1] = e1 + o1;
    v[2] = e2 + o2;
    v[3] = e3 + o3;
    v[4] = e0 - o0;
    v[5] = e1 - o1;
    v[6] = e2 - o2;
    v[7] = e3 - o3;
}
// element e of line j in LDS: columns pass [e][j] rows padded to NCOL + 1, rows pass one line
// with a pad element every 16
template <int NCOL>
struct FcColIdx {
    // (2 columns: no pad, so m = 2^25's 4096-row blocks fit two workgroups per CU; 8 columns: no
    // pad either, the reads of 4 lines x 8 columns by 32 lanes then fill the 64 banks (the pad
    // of 9 made them 2-way, r05z5: 0.47 of the LDS cycles conflicts) and only the first
    // pass's stores, 2 lines x 8 columns per 16-lane group at 8 lines apart, are 2-way)
    static constexpr int STRIDE = (NCOL > 2 && NCOL != 8) ? NCOL + 1 : NCOL;
    __device__ __forceinline__ int operator()(int j, int e) const { return e * STRIDE + j; }
};
struct FcRowIdx {
    __device__ __forceinline__ int operator()(int, int e) const { return e + (e >> 4); }
};

// One Stockham pass of radix RAD over 2^LOGL lines of length L held in LDS (in place: every
// thread reads its butterflies into registers, barrier, writes). SIGN -1: forward.
template <int RAD, int SIGN, int NITEM, int LOGL, class Idx>
__device__ __forceinline__ void fc_pass(fcv* sm, int L, int lgNs, Idx idx) {
    fcv v[NITEM][RAD];
    const int Ns = 1 << lgNs;
    const int tid = threadIdx.x;
    const int bfly = L / RAD;
#pragma unroll
    for (int q = 0; q < NITEM; ++q) {
        const int item = tid + q * FC_NT;
        const int j = item & ((1 << LOGL) - 1), b = item >> LOGL;
        const int k = b & (Ns - 1);
#pragma unroll
        for (int r = 0; r < RAD; ++r) v[q][r] = sm[idx(j, b + r * bfly)];
        if (lgNs > 0) {
            float sn, cs;
            // 2 pi k / (Ns RAD): the power-of-two division as an exponent shift
            __sincosf((float)SIGN * FC_2PI * ldexpf((float)k, -(lgNs + (RAD == 8 ? 3 : RAD == 4 ? 2 : 1))),
                      &sn, &cs);
            const fcv w1 = {cs, sn};
            fcv w = w1;
#pragma unroll
            for (int r = 1; r < RAD; ++r) {
                v[q][r] = cmulf(v[q][r], w);
                if (r + 1 < RAD) w = cmulf(w, w1);
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NITEM; ++q) {
        const int item = tid + q * FC_NT;
        const int j = item & ((1 << LOGL) - 1), b = item >> LOGL;
        const int d = ((b >> lgNs) << lgNs) * RAD + (b & (Ns - 1));
        if (RAD == 8) {
            fc_dft8<SIGN>(v[q]);
        } else if (RAD == 4) {
            fc_dft4<SIGN>(v[q][0], v[q][1], v[q][2], v[q][3]);
        } else {
            const fcv a0 = v[q][0], a1 = v[q][1];
            v[q][0] = a0 + a1;
            v[q][1] = a0 - a1;
        }
#pragma unroll
        for (int r = 0; r < RAD; ++r) sm[idx(j, d + r * Ns)] = v[q][r];
    }
    __syncthreads();
}

// the whole length-L transform of 2^LOGL lines (natural order in, natural order out): radix-8
// passes, then one radix-4 or radix-2 pass for the rest
template <int SIGN, int L, int LOGL, class Idx>
__device__ __forceinline__ void fc_fft(fcv* sm, Idx idx) {
    constexpr int N8 = ((L / 8) << LOGL) / FC_NT;
    static_assert(((L / 8) << LOGL) % FC_NT == 0, "radix-8 butterflies: whole rounds per thread");
    int lg = 0;
#pragma unroll 1
    for (; (8 << lg) <= L; lg += 3) fc_pass<8, SIGN, N8, LOGL>(sm, L, lg, idx);
    if ((4 << lg) == L) fc_pass<4, SIGN, ((L / 4) << LOGL) / FC_NT, LOGL>(sm, L, lg, idx);
    else if ((2 << lg) == L) fc_pass<2, SIGN, ((L / 2) << LOGL) / FC_NT, LOGL>(sm, L, lg, idx);
}

template <int R>
struct FcCols {
    static constexpr int NCOL = R >= 4096 ? 2 : R >= 2048 ? 4 : R >= 1024 ? 8 : 16;
    static constexpr int LOGL = NCOL == 2 ? 1 : NCOL == 4 ? 2 : NCOL == 8 ? 3 : 4;
};

// (A) and (C): NCOL columns per workgroup. FWD: load the scaled support of row blockIdx.y
// straight from S (efd_hann_stage's values), forward FFT, twiddle, store. Inverse: load,
// conjugate twiddle, inverse FFT, store in natural order.
// (<= 128 VGPRs: two 8-wave workgroups per CU, 4 waves per SIMD)
template <bool FWD, int R, int C = FC_C>
__global__ __launch_bounds__(FC_NT) __attribute__((amdgpu_waves_per_eu(4, 8)))
void k_fc_cols(const double2* __restrict__ S, int64_t stride, const uint64_t* __restrict__ info,
               float2* __restrict__ Yv) {
    constexpr int NCOL = FcCols<R>::NCOL, LOGL = FcCols<R>::LOGL;
    constexpr int64_t M = (int64_t)R * C;
    constexpr int NQ = R * NCOL / FC_NT;   // elements per thread
    static_assert(R * NCOL % FC_NT == 0, "whole rounds of elements per thread");
    __shared__ fcv sm[R * FcColIdx<NCOL>::STRIDE];
    fcv* Y = reinterpret_cast<fcv*>(Yv);
    const FcColIdx<NCOL> idx;
    const int row = blockIdx.y;
    // XCD-aware column blocks: workgroups are dealt round-robin over the 8 XCDs (x = b mod 8),
    // so XCD x takes the contiguous eighth [x G/8, (x+1) G/8) of the G column blocks in order;
    // a block's rows are NCOL * 8 or 16 B wide, and the neighbouring blocks sharing their
    // 128-B lines then hit the same L2
    constexpr int G = C / NCOL;
    static_assert(G % 8 == 0, "column blocks: a multiple of the 8 XCDs");
    const int c0 = ((blockIdx.x & 7) * (G / 8) + (blockIdx.x >> 3)) * NCOL;
    fcv* y = Y + (int64_t)row * M;
    if (FWD) {
        const HannRow h = hann_row(info, row);
        const double inv = h.scale == 0.0 ? 0.0 : 1.0 / h.scale;
        const double2* src = S + (int64_t)row * stride + h.first;
        const bool bad = h.len > M;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int i = threadIdx.x + q * FC_NT;
            const int e = i / NCOL, j = i % NCOL;
            const int64_t s = (int64_t)e * C + c0 + j;
            fcv v = {0.f, 0.f};
            if (bad) {
                v = (fcv){__int_as_float(0x7fc00000), 0.f};
            } else if (s < h.len) {
                const double2 x = src[s];
                v = (fcv){(float)(x.x * inv), (float)(x.y * inv)};
            }
            sm[idx(j, e)] = v;
        }
        __syncthreads();
        fc_fft<-1, R, LOGL>(sm, idx);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int i = threadIdx.x + q * FC_NT;
            const int e = i / NCOL, j = i % NCOL;   // e = f_r
            const int c = c0 + j;
            const uint32_t p = (uint32_t)c * (uint32_t)e;   // < C R = M: no reduction
            float sn, cs;
            __sincosf(-FC_2PI * ((float)p * (1.0f / (float)M)), &sn, &cs);
            y[(int64_t)e * C + c] = cmulf(sm[idx(j, e)], (fcv){cs, sn});
        }
    } else {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int i = threadIdx.x + q * FC_NT;
            const int e = i / NCOL, j = i % NCOL;   // e = f_r
            const int c = c0 + j;
            const uint32_t p = (uint32_t)c * (uint32_t)e;   // < C R = M: no reduction
            float sn, cs;
            __sincosf(FC_2PI * ((float)p * (1.0f / (float)M)), &sn, &cs);
            sm[idx(j, e)] = cmulf(y[(int64_t)e * C + c], (fcv){cs, sn});
        }
        __syncthreads();
        fc_fft<1, R, LOGL>(sm, idx);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int i = threadIdx.x + q * FC_NT;
            const int e = i / NCOL, j = i % NCOL;
            y[(int64_t)e * C + c0 + j] = sm[idx(j, e)];
        }
    }
}

// (B): one row f_r per workgroup: forward FFT, times the kernel's spectrum, inverse FFT, as
// three register stages per direction with two LDS exchanges between them (8192 = 32 x 16 x 16):
//   forward  (A) thread t = n2 (n = n2 + 256 n1): DFT-32 over n1, times w_8192^(n2 k1)
//            (B) task (k1, n2a) (n2 = n2a + 16 n2b): DFT-16 over n2b, times w_256^(n2a k2a)
//            (C) task (k1, k2a): DFT-16 over n2a -> X[k1 + 32 k2a + 512 k2b], natural index k
//   times the kernel's spectrum at k, then the transpose of the same steps: the inverse of (C) on
//   the same task's registers (no exchange), of (B), of (A) -> x[n2 + 256 n1], natural order.
// Four exchanges of 64 KB per row instead of the Stockham passes' ten (five radix-8/2 passes per
// direction, each a 64-KB LDS read and write) and the multiply's own pass; every exchange is
// bank-conflict free (exchange 1: rows of 257 elements, lanes along k1 at stride 514 words;
// exchange 2: [k2a][n2a][k1], lanes along k1). Twiddle powers from two __sincosf (w, w^8).
constexpr int FR_NT = 256;     // threads of the row workgroup (32 elements each)
constexpr int FR_S1 = 257;     // exchange 1: LDS row stride of [k1][n2] (elements)
// cos and sin of 2 pi j / 32
constexpr float FC_COS32[32] = {
    1.000000000e+00f, 9.807852804e-01f, 9.238795325e-01f, 8.314696123e-01f, 7.071067812e-01f,
    5.555702330e-01f, 3.826834324e-01f, 1.950903220e-01f, 0.0f, -1.950903220e-01f,
    -3.826834324e-01f, -5.555702330e-01f, -7.071067812e-01f, -8.314696123e-01f,
    -9.238795325e-01f, -9.807852804e-01f, -1.000000000e+00f, -9.807852804e-01f,
    -9.238795325e-01f, -8.314696123e-01f, -7.071067812e-01f, -5.555702330e-01f,
    -3.826834324e-01f, -1.950903220e-01f, 0.0f, 1.950903220e-01f, 3.826834324e-01f,
    5.555702330e-01f, 7.071067812e-01f, 8.314696123e-01f, 9.238795325e-01f, 9.807852804e-01f};
// w_N^j = exp(SIGN 2 pi i j / N) for N = 16, 32 (compile-time j: constant-folded)
template <int SIGN, int N>
__device__ __forceinline__ fcv fc_w(int j) {
    const int q = (j * (32 / N)) & 31;
    return (fcv){FC_COS32[q], (float)SIGN * FC_COS32[(q + 24) & 31]};
}
// natural-order DFT-16 (4 x 4) and DFT-32 (4 x 8) in registers, exp(SIGN 2 pi i n k / N)
template <int SIGN>
__device__ __forceinline__ void fc_dft16(fcv* v) {
    fcv t[4][4];
#pragma unroll
    for (int n1 = 0; n1 < 4; ++n1) {   // DFT-4 over n2 of x[n1 + 4 n2]
        fcv a0 = v[n1], a1 = v[n1 + 4], a2 = v[n1 + 8], a3 = v[n1 + 12];
        fc_dft4<SIGN>(a0, a1, a2, a3);
        t[n1][0] = a0; t[n1][1] = a1; t[n1][2] = a2; t[n1][3] = a3;
    }
#pragma unroll
    for (int n1 = 1; n1 < 4; ++n1)
#pragma unroll
        for (int k1 = 1; k1 < 4; ++k1) t[n1][k1] = cmulf(t[n1][k1], fc_w<SIGN, 16>(n1 * k1));
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {   // DFT-4 over n1 -> X[k1 + 4 k2]
        fcv a0 = t[0][k1], a1 = t[1][k1], a2 = t[2][k1], a3 = t[3][k1];
        fc_dft4<SIGN>(a0, a1, a2, a3);
        v[k1] = a0; v[k1 + 4] = a1; v[k1 + 8] = a2; v[k1 + 12] = a3;
    }
}
template <int SIGN>
__device__ __forceinline__ void fc_dft32(fcv* v) {
    fcv t[8][4];
#pragma unroll
    for (int n1 = 0; n1 < 8; ++n1) {   // DFT-4 over n2 of x[n1 + 8 n2]
        fcv a0 = v[n1], a1 = v[n1 + 8], a2 = v[n1 + 16], a3 = v[n1 + 24];
        fc_dft4<SIGN>(a0, a1, a2, a3);
        t[n1][0] = a0; t[n1][1] = a1; t[n1][2] = a2; t[n1][3] = a3;
    }
#pragma unroll
    for (int n1 = 1; n1 < 8; ++n1)
#pragma unroll
        for (int k1 = 1; k1 < 4; ++k1) t[n1][k1] = cmulf(t[n1][k1], fc_w<SIGN, 32>(n1 * k1));
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {   // DFT-8 over n1 -> X[k1 + 4 k2]
        fcv e[8];
#pragma unroll
        for (int n1 = 0; n1 < 8; ++n1) e[n1] = t[n1][k1];
        fc_dft8<SIGN>(e);
#pragma unroll
        for (int k2 = 0; k2 < 8; ++k2) v[k1 + 4 * k2] = e[k2];
    }
}
// v[j] *= w^j, j = 0 .. N-1, w = exp(i theta): powers from w and w^8 (at most 3 + 7 products)
template <int N>
__device__ __forceinline__ void fc_twiddle_pow(fcv* v, float theta) {
    float s1, c1, s8, c8;
    __sincosf(theta, &s1, &c1);
    __sincosf(8.0f * theta, &s8, &c8);
    const fcv w1 = {c1, s1}, w8 = {c8, s8};
    fcv p[8];
    p[0] = (fcv){1.0f, 0.0f};
    p[1] = w1;
#pragma unroll
    for (int j = 2; j < 8; ++j) p[j] = cmulf(p[j - 1], w1);
    fcv b = (fcv){1.0f, 0.0f};
#pragma unroll
    for (int a = 0; a < N / 8; ++a) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (a + j > 0) v[8 * a + j] = cmulf(v[8 * a + j], a == 0 ? p[j] : (j == 0 ? b : cmulf(b, p[j])));
        b = a == 0 ? w8 : cmulf(b, w8);
    }
}
// v[j] *= w0 w^j, j = 0 .. N-1, w = exp(i theta): fc_twiddle_pow with the constant factor w0
// folded into the powers (8 products instead of N)
template <int N>
__device__ __forceinline__ void fc_twiddle_pow_from(fcv* v, fcv w0, float theta) {
    float s1, c1, s8, c8;
    __sincosf(theta, &s1, &c1);
    __sincosf(8.0f * theta, &s8, &c8);
    const fcv w1 = {c1, s1}, w8 = {c8, s8};
    fcv p[8];
    p[0] = w0;
#pragma unroll
    for (int j = 1; j < 8; ++j) p[j] = cmulf(p[j - 1], w1);
    fcv b = (fcv){1.0f, 0.0f};
#pragma unroll
    for (int a = 0; a < N / 8; ++a) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[8 * a + j] = cmulf(v[8 * a + j], a == 0 ? p[j] : cmulf(b, p[j]));
        b = a == 0 ? w8 : cmulf(b, w8);
    }
}
__global__ __launch_bounds__(FR_NT)
void k_fc_rows(const float2* __restrict__ kfpv, int64_t m, int rows, float2* __restrict__ Yv) {
    static_assert(FC_C == 32 * 16 * 16 && FR_NT == 256, "row transform: 8192 = 32 x 16 x 16");
    __shared__ fcv sm[32 * FR_S1];   // exchange 1 [k1][n2] (stride 257); exchange 2 [k2a][n2a][k1]
    const fcv* kfp = reinterpret_cast<const fcv*>(kfpv);
    fcv* Y = reinterpret_cast<fcv*>(Yv);
    // (row f_r, walker) pairs: XCD x = b mod 8 takes the contiguous eighth of them in f_r-major
    // order, so a kernel-spectrum row is read from HBM once per XCD and from its L2 for the
    // group's other walkers (gridDim.x = R * rows, a multiple of 8)
    const int64_t npair = (int64_t)gridDim.x;
    const int64_t p = (int64_t)(blockIdx.x & 7) * (npair >> 3) + (blockIdx.x >> 3);
    const int fr = (int)(p / rows), wk = (int)(p - (int64_t)fr * rows);
    fcv* y = Y + (int64_t)wk * m + (int64_t)fr * FC_C;
    const fcv* kr = kfp + (int64_t)fr * FC_C;
    const int t = threadIdx.x;
    constexpr float W8192 = FC_2PI / 8192.0f, W256 = FC_2PI / 256.0f;
    {   // forward (A): n2 = t
        fcv v[32];
#pragma unroll
        for (int n1 = 0; n1 < 32; ++n1) v[n1] = y[t + 256 * n1];
        fc_dft32<-1>(v);
        fc_twiddle_pow<32>(v, -W8192 * (float)t);
#pragma unroll
        for (int k1 = 0; k1 < 32; ++k1) sm[k1 * FR_S1 + t] = v[k1];
    }
    __syncthreads();
    fcv u[2][16];
#pragma unroll
    for (int h = 0; h < 2; ++h) {   // forward (B): task (k1, n2a)
        const int q = t + 256 * h, k1 = q & 31, n2a = q >> 5;
#pragma unroll
        for (int n2b = 0; n2b < 16; ++n2b) u[h][n2b] = sm[k1 * FR_S1 + n2a + 16 * n2b];
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int q = t + 256 * h, k1 = q & 31, n2a = q >> 5;
        fc_dft16<-1>(u[h]);
        fc_twiddle_pow<16>(u[h], -W256 * (float)n2a);
#pragma unroll
        for (int k2a = 0; k2a < 16; ++k2a) sm[(k2a * 16 + n2a) * 32 + k1] = u[h][k2a];
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {   // forward (C), the kernel's spectrum, inverse (C): (k1, k2a)
        const int q = t + 256 * h, k1 = q & 31, k2a = q >> 5;
#pragma unroll
        for (int n2a = 0; n2a < 16; ++n2a) u[h][n2a] = sm[(k2a * 16 + n2a) * 32 + k1];
        fc_dft16<-1>(u[h]);
#pragma unroll
        for (int k2b = 0; k2b < 16; ++k2b)
            u[h][k2b] = cmulf(u[h][k2b], kr[k1 + 32 * k2a + 512 * k2b]);
        fc_dft16<1>(u[h]);
        fc_twiddle_pow<16>(u[h], W256 * (float)k2a);
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int q = t + 256 * h, k1 = q & 31, k2a = q >> 5;
#pragma unroll
        for (int n2a = 0; n2a < 16; ++n2a) sm[(k2a * 16 + n2a) * 32 + k1] = u[h][n2a];
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {   // inverse (B): task (k1, n2a)
        const int q = t + 256 * h, k1 = q & 31, n2a = q >> 5;
#pragma unroll
        for (int k2a = 0; k2a < 16; ++k2a) u[h][k2a] = sm[(k2a * 16 + n2a) * 32 + k1];
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int q = t + 256 * h, k1 = q & 31, n2a = q >> 5;
        fc_dft16<1>(u[h]);   // -> n2b
        // times w_8192^(-n2 k1), n2 = n2a + 16 n2b: w^(n2a k1) (w^(16 k1))^n2b
        float s0, c0;
        __sincosf(W8192 * (float)(n2a * k1), &s0, &c0);
        const fcv w0 = {c0, s0};
#pragma unroll
        for (int n2b = 0; n2b < 16; ++n2b) u[h][n2b] = cmulf(u[h][n2b], w0);
        fc_twiddle_pow<16>(u[h], W8192 * 16.0f * (float)k1);
#pragma unroll
        for (int n2b = 0; n2b < 16; ++n2b) sm[k1 * FR_S1 + n2a + 16 * n2b] = u[h][n2b];
    }
    __syncthreads();
    {   // inverse (A): n2 = t -> x[n2 + 256 n1]
        fcv v[32];
#pragma unroll
        for (int k1 = 0; k1 < 32; ++k1) v[k1] = sm[k1 * FR_S1 + t];
        fc_dft32<1>(v);
#pragma unroll
        for (int n1 = 0; n1 < 32; ++n1) y[t + 256 * n1] = v[n1];
    }
}

// (B) for rows of C = 16384 (m = 2^24 as 1024 x 16384: wider column segments, 128 B of S and 64 B
// of Y per row of a column block), register-staged as k_fc_rows with 512 threads of 32 elements
// (16384 = 32 x 32 x 16; n = n2 + 512 n1, n2 = n2a + 16 n2b; k = k1 + 32 k2a + 1024 k2b): forward
// (A) thread n2: DFT-32 over n1, times w_16384^(n2 k1); (B) task (k1, n2a): DFT-32 over n2b,
// times w_512^(n2a k2a); (C) task (k1, k2a), two per thread: DFT-16 over n2a; the kernel's
// spectrum; the transposed steps back. (Round 5 also kept complex exchanges with 128 KB of LDS,
// one workgroup per CU: 650 against 575-579 us, r05z; deleted in round 6.)
constexpr int FC_C16 = 16384;
// Every exchange in two passes (real parts, then imaginary parts) through a float array: 69.6 KB of LDS and at most 128 VGPRs, so two workgroups share a CU and one's
// loads and stores overlap the other's transforms (one per CU leaves HBM idle while it
// computes). Exchange 1 [k1][n2] stride 513, exchange 2 [k2a][n2a][k1] unpadded: every b32
// access of a 32-lane bank group hits 32 distinct banks (ds_read_b32 / ds_write_b32 bank
// (a/4) mod 32; stride 514 read exchange 1 2-way, r05z5: 0.20 of the LDS cycles conflicts).
constexpr int FR16_T1 = 513, FR16_T2 = 512;
__global__ __launch_bounds__(FC_NT) __attribute__((amdgpu_waves_per_eu(4, 8)))
void k_fc_rows16k_h(const float2* __restrict__ kfpv, int64_t m, int rows, float2* __restrict__ Yv) {
    static_assert(FC_NT == 512 && FC_C16 == 32 * 32 * 16, "16384 = 32 x 32 x 16, 512 threads");
    __shared__ float sf[32 * (FR16_T1 > FR16_T2 ? FR16_T1 : FR16_T2)];
    const fcv* kfp = reinterpret_cast<const fcv*>(kfpv);
    fcv* Y = reinterpret_cast<fcv*>(Yv);
    const int64_t npair = (int64_t)gridDim.x;
    const int64_t p = (int64_t)(blockIdx.x & 7) * (npair >> 3) + (blockIdx.x >> 3);
    const int fr = (int)(p / rows), wk = (int)(p - (int64_t)fr * rows);
    fcv* y = Y + (int64_t)wk * m + (int64_t)fr * FC_C16;
    const fcv* kr = kfp + (int64_t)fr * FC_C16;
    const int t = threadIdx.x;
    const int kb = t & 31, nb = t >> 5;
    constexpr float W16K = FC_2PI / 16384.0f, W512 = FC_2PI / 512.0f;
    fcv v[32], u[32], w[2][16];
#pragma unroll
    for (int n1 = 0; n1 < 32; ++n1) v[n1] = y[t + 512 * n1];
    fc_dft32<-1>(v);   // forward (A): n2 = t
    fc_twiddle_pow<32>(v, -W16K * (float)t);
#pragma unroll
    for (int c = 0; c < 2; ++c) {   // exchange 1 -> (B) task (k1 = kb, n2a = nb)
#pragma unroll
        for (int k1 = 0; k1 < 32; ++k1) sf[k1 * FR16_T1 + t] = c ? v[k1].y : v[k1].x;
        __syncthreads();
#pragma unroll
        for (int n2b = 0; n2b < 32; ++n2b) {
            const float x = sf[kb * FR16_T1 + nb + 16 * n2b];
            if (c) u[n2b].y = x; else u[n2b].x = x;
        }
        __syncthreads();
    }
    fc_dft32<-1>(u);
    fc_twiddle_pow<32>(u, -W512 * (float)nb);
#pragma unroll
    for (int c = 0; c < 2; ++c) {   // exchange 2 -> (C) tasks (k1, k2a)
#pragma unroll
        for (int k2a = 0; k2a < 32; ++k2a) sf[k2a * FR16_T2 + nb * 32 + kb] = c ? u[k2a].y : u[k2a].x;
        __syncthreads();
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int q = t + 512 * h, k1 = q & 31, k2a = q >> 5;
#pragma unroll
            for (int n2a = 0; n2a < 16; ++n2a) {
                const float x = sf[k2a * FR16_T2 + n2a * 32 + k1];
                if (c) w[h][n2a].y = x; else w[h][n2a].x = x;
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {   // forward (C), the kernel's spectrum, inverse (C)
        const int q = t + 512 * h, k1 = q & 31, k2a = q >> 5;
        fc_dft16<-1>(w[h]);
#pragma unroll
        for (int k2b = 0; k2b < 16; ++k2b)
            w[h][k2b] = cmulf(w[h][k2b], kr[k1 + 32 * k2a + 1024 * k2b]);
        fc_dft16<1>(w[h]);
        fc_twiddle_pow<16>(w[h], W512 * (float)k2a);
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {   // exchange 2 back -> inverse (B)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int q = t + 512 * h, k1 = q & 31, k2a = q >> 5;
#pragma unroll
            for (int n2a = 0; n2a < 16; ++n2a)
                sf[k2a * FR16_T2 + n2a * 32 + k1] = c ? w[h][n2a].y : w[h][n2a].x;
        }
        __syncthreads();
#pragma unroll
        for (int k2a = 0; k2a < 32; ++k2a) {
            const float x = sf[k2a * FR16_T2 + nb * 32 + kb];
            if (c) u[k2a].y = x; else u[k2a].x = x;
        }
        __syncthreads();
    }
    fc_dft32<1>(u);   // -> n2b, times w_16384^(-n2 k1)
    {
        float s0, c0;
        __sincosf(W16K * (float)(nb * kb), &s0, &c0);
        fc_twiddle_pow_from<32>(u, (fcv){c0, s0}, W16K * 16.0f * (float)kb);
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {   // exchange 1 back -> inverse (A): n2 = t
#pragma unroll
        for (int n2b = 0; n2b < 32; ++n2b) sf[kb * FR16_T1 + nb + 16 * n2b] = c ? u[n2b].y : u[n2b].x;
        __syncthreads();
#pragma unroll
        for (int k1 = 0; k1 < 32; ++k1) {
            const float x = sf[k1 * FR16_T1 + t];
            if (c) v[k1].y = x; else v[k1].x = x;
        }
        if (c == 0) __syncthreads();
    }
    fc_dft32<1>(v);
    // the store offsets from an opaque copy of t: else the compiler keeps the loads' 32
    // addresses live across the kernel (spilled to scratch)
    int to = t;
    __asm__ volatile("" : "+v"(to));
#pragma unroll
    for (int n1 = 0; n1 < 32; ++n1) y[to + 512 * n1] = v[n1];
}

// (A) for R = 1024 with rows of C = 16384 (m = 2^24 as 1024 x 16384), NCOL = 8 columns per
// workgroup, register-staged (1024 = 16 x 8 x 8; n = n2 + 64 n1, n2 = n2a + 8 n2b; k = k1 + 16 k2a
// + 128 k2b): task (j, n2): DFT-16 over n1, times w_1024^(n2 k1); (B) tasks (j, k1, n2a), two per
// thread: DFT-8 over n2b, times w_64^(n2a k2a); (C) tasks (j, k1, k2a), two per thread: DFT-8
// over n2a -> f_r = k. Exchange 1 [k1][n2][j], exchange 2 [k1][k2a][n2a (pad to 9)][j]: lanes
// along j then n2a / k2a, conflict-free. 252 against the Stockham kernel's 369 us (r05z3). The
// inverse columns stay on the Stockham kernel k_fc_cols<false, 1024, 16384>: the staged inverse
// measured 549 against 476 us (r05z3; deleted in round 6).
constexpr int FCD_R = 1024, FCD_NCOL = 8, FCD_S2 = 9;
__global__ __launch_bounds__(FC_NT) __attribute__((amdgpu_waves_per_eu(4, 8)))
void k_fc_cols1024(const double2* __restrict__ S, int64_t stride, const uint64_t* __restrict__ info,
                   float2* __restrict__ Yv) {
    static_assert(FC_NT == 512 && FCD_R * FCD_NCOL == 16 * FC_NT, "16 elements per thread");
    constexpr int C = FC_C16;
    constexpr int64_t M = (int64_t)FCD_R * C;
    // exchange 1: 16 x 64 x 8 = 8192; exchange 2: 16 x 8 x 9 x 8 = 9216 elements (73.7 KB)
    __shared__ fcv sm[16 * 8 * FCD_S2 * FCD_NCOL];
    fcv* Y = reinterpret_cast<fcv*>(Yv);
    const int row = blockIdx.y;
    constexpr int G = C / FCD_NCOL;
    static_assert(G % 8 == 0, "column blocks: a multiple of the 8 XCDs");
    const int c0 = ((blockIdx.x & 7) * (G / 8) + (blockIdx.x >> 3)) * FCD_NCOL;
    fcv* y = Y + (int64_t)row * M;
    const int t = threadIdx.x;
    const int j = t & 7;
    const int c = c0 + j;
    constexpr float W1024 = FC_2PI / 1024.0f, W64 = FC_2PI / 64.0f;
    auto e1 = [](int k1, int n2, int jj) { return (k1 * 64 + n2) * FCD_NCOL + jj; };
    auto e2 = [](int k1, int k2a, int n2a, int jj) {
        return ((k1 * 8 + k2a) * FCD_S2 + n2a) * FCD_NCOL + jj;
    };
    {
        const HannRow h = hann_row(info, row);
        const double inv = h.scale == 0.0 ? 0.0 : 1.0 / h.scale;
        const double2* src = S + (int64_t)row * stride + h.first;
        const bool bad = h.len > M;
        {   // (A): task (j, n2)
            const int n2 = t >> 3;
            fcv v[16];
#pragma unroll
            for (int n1 = 0; n1 < 16; ++n1) {
                const int64_t s = (int64_t)(n2 + 64 * n1) * C + c;
                fcv x = {0.f, 0.f};
                if (bad) {
                    x = (fcv){__int_as_float(0x7fc00000), 0.f};
                } else if (s < h.len) {
                    const double2 d = src[s];
                    x = (fcv){(float)(d.x * inv), (float)(d.y * inv)};
                }
                v[n1] = x;
            }
            fc_dft16<-1>(v);
            fc_twiddle_pow<16>(v, -W1024 * (float)n2);
#pragma unroll
            for (int k1 = 0; k1 < 16; ++k1) sm[e1(k1, n2, j)] = v[k1];
        }
        __syncthreads();
        fcv u[2][8];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {   // (B): tasks (j, n2a, k1)
            const int q = t + FC_NT * hh, n2a = (q >> 3) & 7, k1 = q >> 6;
#pragma unroll
            for (int n2b = 0; n2b < 8; ++n2b) u[hh][n2b] = sm[e1(k1, n2a + 8 * n2b, j)];
        }
        __syncthreads();
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            const int q = t + FC_NT * hh, n2a = (q >> 3) & 7, k1 = q >> 6;
            fc_dft8<-1>(u[hh]);
            fc_twiddle_pow<8>(u[hh], -W64 * (float)n2a);
#pragma unroll
            for (int k2a = 0; k2a < 8; ++k2a) sm[e2(k1, k2a, n2a, j)] = u[hh][k2a];
        }
        __syncthreads();
        int to = t;   // opaque: no store address kept live from (A)
        __asm__ volatile("" : "+v"(to));
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {   // (C): tasks (j, k2a, k1)
            const int q = to + FC_NT * hh, k2a = (q >> 3) & 7, k1 = q >> 6;
            fcv w[8];
#pragma unroll
            for (int a = 0; a < 8; ++a) w[a] = sm[e2(k1, k2a, a, j)];
            fc_dft8<-1>(w);
#pragma unroll
            for (int k2b = 0; k2b < 8; ++k2b) {
                const int fr = k1 + 16 * k2a + 128 * k2b;
                const uint32_t pp = (uint32_t)c * (uint32_t)fr;   // < C R = M: no reduction
                float sn, cs;
                __sincosf(-FC_2PI * ((float)pp * (1.0f / (float)M)), &sn, &cs);
                y[(int64_t)fr * C + c] = cmulf(w[k2b], (fcv){cs, sn});
            }
        }
    }
}

// S_w at bin k: the 3-point stencil on S and the correction's difference (neighbours mod nf).
// S is zero outside the row's support [first, first + len) (cyclic; efd_hann_extent's bounds),
// so it is read only there: the support is ~40% of test.sh's grid, and the skipped reads were
// half of the reduction's HBM bytes (the correction C = Y is nonzero everywhere)
__device__ __forceinline__ double2 hann_sw(const double2* __restrict__ S,
                                           const float2* __restrict__ Y, int64_t nf, int64_t k,
                                           double c, int64_t first, int64_t len, int64_t off) {
    const int64_t kp = k + 1 < nf ? k + 1 : 0, km = k > 0 ? k - 1 : nf - 1;
    int64_t qp = kp - first, qm = km - first, q0 = k - first;
    qp += qp < 0 ? nf : 0;
    qm += qm < 0 ? nf : 0;
    q0 += q0 < 0 ? nf : 0;
    const double2 z = make_double2(0.0, 0.0);
    const double2 s = q0 < len ? S[k] : z, sp = qp < len ? S[kp] : z, sm = qm < len ? S[km] : z;
    const float2 cp = Y[qp + off], cm = Y[qm + off];
    return make_double2(0.5 * s.x - 0.25 * (sp.x + sm.x) - c * ((double)cp.x - (double)cm.x),
                        0.5 * s.y - 0.25 * (sp.y + sm.y) - c * ((double)cp.y - (double)cm.y));
}
// h+ = (a + conj b)/2, hx = i (a - conj b)/2 of the windowed spectrum at k (a) and nf-1-k (b)
__device__ __forceinline__ void hann_pol(const double2* __restrict__ S,
                                         const float2* __restrict__ Y, int64_t nf, int64_t k,
                                         double c, int64_t first, int64_t len, int64_t off,
                                         double2& vp, double2& vc) {
    const double2 a = hann_sw(S, Y, nf, k, c, first, len, off);
    const double2 b = hann_sw(S, Y, nf, nf - 1 - k, c, first, len, off);
    vp = make_double2(0.5 * (a.x + b.x), 0.5 * (a.y - b.y));
    vc = make_double2(-0.5 * (a.y + b.y), 0.5 * (a.x - b.x));
}
__global__ void k_hann_polarizations(const double2* __restrict__ S, const float2* __restrict__ Y,
                                     const uint64_t* __restrict__ info, int64_t m, int64_t nf,
                                     int64_t k0, double2* __restrict__ hp,
                                     double2* __restrict__ hc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t k = k0 + i;
    if (k >= nf) return;
    const HannRow h = hann_row(info, 0);
    const double c = h.scale / (4.0 * (double)(nf - 1));
    double2 vp, vc;
    hann_pol(S, Y, nf, k, c, h.first, h.len, m - nf, vp, vc);
    hp[i] = vp;
    hc[i] = vc;
}
// the windowed templates' log-likelihood partials of every row: efd_loglike's terms (d - h w,
// product rounded then difference) for both channels of every bin [k0, nf). One workgroup per
// (bin chunk, row): a thread holds one row's sum (70 VGPRs, 7 waves per SIMD: the loads of many
// waves in flight; the earlier form kept all rows' sums and loads in one thread, 233 VGPRs and
// 2 waves per SIMD, 0.53 of HBM). The rows of a chunk are consecutive workgroups of one XCD
// (workgroup b runs on XCD b mod 8), so d and w (48 B per bin, the same for every row) come from
// HBM once and from that XCD's L2 for the other rows. part[row * nchunk + chunk].
constexpr int HANN_ROWS_MAX = 16;
// RPT rows per workgroup (rows = RPT x the row groups; a thread reads its bin's d and w once
// for all of them: 48 B of the ~176 a bin-row loads from L1/L2). The rows of a chunk's row
// groups are consecutive workgroups of one XCD as with one row each; every row's partial sums
// the same bins in the same order, so the output is bitwise that of RPT = 1.
template <int RPT>
__global__ __launch_bounds__(256) void k_hann_loglike_partial(
    const double2* __restrict__ S, int64_t stride, const float2* __restrict__ Y,
    const uint64_t* __restrict__ info, int64_t m, int64_t nf, int64_t k0,
    const double2* __restrict__ d, const double* __restrict__ w, int rows, int nchunk,
    double* __restrict__ part) {
#pragma clang fp contract(off)
    const int ngr = rows / RPT;
    const int j = (int)(blockIdx.x >> 3);
    const int r0 = (j % ngr) * RPT, chunk = (int)(blockIdx.x & 7) + 8 * (j / ngr);
    double c[RPT];
    int64_t first[RPT], len[RPT];
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
        const HannRow h = hann_row(info, r0 + q);
        c[q] = h.scale / (4.0 * (double)(nf - 1));
        first[q] = h.first;
        len[q] = h.len;
    }
    const int64_t nb = nf - k0;
    double acc[RPT];
#pragma unroll
    for (int q = 0; q < RPT; ++q) acc[q] = 0.0;
    for (int64_t i = (int64_t)chunk * 256 + threadIdx.x; i < nb; i += (int64_t)nchunk * 256) {
        const double2 d0 = d[i], d1 = d[nb + i];
        const double w0 = w[i], w1 = w[nb + i];
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            double2 vp, vc;
            hann_pol(S + (int64_t)(r0 + q) * stride, Y + (int64_t)(r0 + q) * m, nf, k0 + i, c[q],
                     first[q], len[q], m - nf, vp, vc);
            const double x0 = d0.x - vp.x * w0, y0 = d0.y - vp.y * w0;
            const double x1 = d1.x - vc.x * w1, y1 = d1.y - vc.y * w1;
            acc[q] = fma(x0, x0, fma(y0, y0, acc[q]));
            acc[q] = fma(x1, x1, fma(y1, y1, acc[q]));
        }
    }
    // a butterfly over each wave, then the 4 waves in turn (fixed order)
    __shared__ double red[RPT][4];
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
        double a = acc[q];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
        if ((threadIdx.x & 63) == 0) red[q][threadIdx.x >> 6] = a;
    }
    __syncthreads();
    if (threadIdx.x < RPT && chunk < nchunk) {
        const int q = threadIdx.x;
        part[(int64_t)(r0 + q) * nchunk + chunk] = ((red[q][0] + red[q][1]) + red[q][2]) + red[q][3];
    }
}

// (C) with the windowed logL fused in (efd_hann_loglike_local). Per bin the two channels' terms
// of a bin k and of its mirror k' = nf-1-k combine into one term on each (with the same weight
// w on both channels, p = d0 - w h+, q = d1 - w hx: |p|^2 + |q|^2 = (|p - iq|^2 + |p + iq|^2)/2,
// p - iq = (d0 - i d1) - w S_w[k], p + iq = (d0 + i d1) - w conj(S_w[k'])), so the logL is
//   (1/2) sum_j |dl[j] - wl[j] S_w[j]|^2 over the whole grid
// with dl[k] = d0 - i d1 (k >= k0), dl[k'] = conj(d0 + i d1), wl = w at both (the caller's
// layout: fdutils.HannConvolution.local_data; the self-mirror bin kself takes its second term
// from dl[nf]). Every term is local to its bin, so the inverse column pass reduces them as it
// produces the correction: the correction array is neither written nor read back.
// The pipeline's kernel spectrum carries the difference factor 2i sin(2 pi f / m), so the
// transform yields Dc[s] = Y[s+1] - Y[s-1] directly (no neighbour column needed): valid for
// s in [m - nf, m - 1) when m >= nf + len, and at s = m - 1 (bin u = nf - 1, whose +1 neighbour
// wraps to u = 0) Y[m] = Y[0] differs from C(u = 0) = Y[m - nf] by y[0] (K[(-(m-nf)) mod nf] -
// K[0]) alone (kfix = K[0] - K[(-(m-nf)) mod nf], added back). emit (one row): write
// dl[j] = wl[j] S_w[j] (and dl[nf] = dl[kself]) instead, the data of an injection made by this
// same arithmetic (its logL against itself is then exactly 0).
// Workgroups: 1-D, b -> XCD b mod 8; XCD x takes column blocks [x G/8, (x+1) G/8) and on it the
// rows of one column block are consecutive, so dl / wl (24 B a bin, the same for every row) come
// from HBM once and from the XCD's L2 for the other rows. part[row * G + column block], halved.
// one element of the fused logL: bin offset u >= 0 from the row's first bin, its differenced
// correction dvf (the transform's output), its prefetched data dv and weight w
struct HannLl {
    const double2* Sr;   // the row of S
    int nfi, first, len;
    double cc, scale;    // e / 4 times the row's scale (NaN: aliased row); the scale
    double2 kfix;
    const double2* dl;
    int64_t kself, nf;
    double2* emit;
};
__device__ __forceinline__ void hann_ll_elem(const HannLl& x, int u, fcv dvf, double2 dv, double w,
                                             double& acc) {
#pragma clang fp contract(off)
    const double2 z = make_double2(0.0, 0.0);
    double dx = (double)dvf.x, dy = (double)dvf.y;
    if (u == x.nfi - 1 && x.len > 0) {   // the +1 neighbour wraps: Y[0] -> C(u = 0)
        const double inv = 1.0 / x.scale;
        const double2 s0 = x.Sr[x.first];
        const double yx = s0.x * inv, yy = s0.y * inv;
        dx += yx * x.kfix.x - yy * x.kfix.y;
        dy += yx * x.kfix.y + yy * x.kfix.x;
    }
    int k = u + x.first;
    k -= k >= x.nfi ? x.nfi : 0;
    const int kp = k + 1 < x.nfi ? k + 1 : 0, km = k > 0 ? k - 1 : x.nfi - 1;
    const int qp = u + 1 < x.nfi ? u + 1 : 0, qm = u > 0 ? u - 1 : x.nfi - 1;
    const double2 s = u < x.len ? x.Sr[k] : z, sp = qp < x.len ? x.Sr[kp] : z,
                  sn = qm < x.len ? x.Sr[km] : z;
    const double wx = 0.5 * s.x - 0.25 * (sp.x + sn.x) - x.cc * dx;
    const double wy = 0.5 * s.y - 0.25 * (sp.y + sn.y) - x.cc * dy;
    if (x.emit != nullptr) {
        const double2 o = make_double2(wx * w, wy * w);
        x.emit[k] = o;
        if (k == x.kself) x.emit[x.nf] = o;
        return;
    }
    const double rx = dv.x - wx * w, ry = dv.y - wy * w;
    acc = fma(rx, rx, fma(ry, ry, acc));
    if (k == x.kself) {
        const double2 d2 = x.dl[x.nf];
        const double tx = d2.x - wx * w, ty = d2.y - wy * w;
        acc = fma(tx, tx, fma(ty, ty, acc));
    }
}
// the row's context (hann_row) for hann_ll_elem
__device__ __forceinline__ HannLl hann_ll_ctx(const double2* S, int64_t stride,
                                              const uint64_t* info, int row, int64_t M,
                                              int64_t nf, const double2* dl, int64_t kself,
                                              double2 kfix, double2* emit) {
    const HannRow h = hann_row(info, row);
    HannLl x;
    x.Sr = S + (int64_t)row * stride;
    x.nfi = (int)nf;
    x.first = (int)h.first;
    x.len = (int)h.len;
    // a support longer than m - nf leaves Y[m - nf - 1] aliased: the row's logL is NaN
    x.cc = h.len > M - nf ? __longlong_as_double(0x7ff8000000000000ll)
                          : h.scale / (4.0 * (double)(nf - 1));
    x.scale = h.scale;
    x.kfix = kfix;
    x.dl = dl;
    x.kself = kself;
    x.nf = nf;
    x.emit = emit;
    return x;
}
// the workgroup's partial (wave butterflies, then the waves in order): part[row G + cb], halved
__device__ __forceinline__ void hann_ll_store(double acc, double* red, double* part, int64_t at) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int wv = 0; wv < (int)(blockDim.x >> 6); ++wv) t += red[wv];
        part[at] = 0.5 * t;
    }
}
template <int R, int C>
__global__ __launch_bounds__(FC_NT) __attribute__((amdgpu_waves_per_eu(4, 8)))
void k_fc_cols_ll(const double2* __restrict__ S, int64_t stride, const uint64_t* __restrict__ info,
                  const float2* __restrict__ Yv, int64_t nf, const double2* __restrict__ dl,
                  const double* __restrict__ wl, int64_t kself, double2 kfix, int rows,
                  double* __restrict__ part, double2* __restrict__ emit) {
#pragma clang fp contract(off)
    constexpr int NCOL = FcCols<R>::NCOL, LOGL = FcCols<R>::LOGL;
    constexpr int64_t M = (int64_t)R * C;
    constexpr int NQ = R * NCOL / FC_NT;
    static_assert(R * NCOL % FC_NT == 0, "whole rounds of elements per thread");
    constexpr int G = C / NCOL;
    static_assert(G % 8 == 0, "column blocks: a multiple of the 8 XCDs");
    __shared__ fcv sm[R * FcColIdx<NCOL>::STRIDE];
    __shared__ double red[FC_NT / 64];
    const fcv* Y = reinterpret_cast<const fcv*>(Yv);
    const FcColIdx<NCOL> idx;
    const int q8 = (int)(blockIdx.x >> 3);
    const int row = q8 % rows, cb = (int)(blockIdx.x & 7) * (G / 8) + q8 / rows;
    const int c0 = cb * NCOL;
    const fcv* y = Y + (int64_t)row * M;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int i = threadIdx.x + q * FC_NT;
        const int e = i / NCOL, j = i % NCOL;
        const uint32_t p = (uint32_t)(c0 + j) * (uint32_t)e;
        float sn, cs;
        __sincosf(FC_2PI * ((float)p * (1.0f / (float)M)), &sn, &cs);
        sm[idx(j, e)] = cmulf(y[(int64_t)e * C + c0 + j], (fcv){cs, sn});
    }
    __syncthreads();
    fc_fft<1, R, LOGL>(sm, idx);
    const HannLl x = hann_ll_ctx(S, stride, info, row, M, nf, dl, kself, kfix, emit);
    const int offi = (int)(M - nf);
    // the elements' data (dl, wl) requested QH at a time before any of them is used: QH loads
    // of each in flight per thread (the epilogue is latency-bound otherwise, one round trip per
    // few elements; all 16 at once spill past 128 VGPRs); indices fit 32 bits (nf < 2^31,
    // m <= 2^25)
    constexpr int QH = NQ >= 8 ? 8 : NQ;
    static_assert(NQ % QH == 0, "whole rounds of prefetched elements");
    double acc = 0.0;
#pragma unroll
    for (int q0 = 0; q0 < NQ; q0 += QH) {
        double2 dv[QH];
        double wv[QH];
#pragma unroll
        for (int t = 0; t < QH; ++t) {
            const int i = threadIdx.x + (q0 + t) * FC_NT;
            const int u = (i / NCOL) * C + c0 + i % NCOL - offi;
            int k = u + x.first;
            k -= k >= x.nfi ? x.nfi : 0;
            dv[t] = make_double2(0.0, 0.0);
            wv[t] = 0.0;
            if (u >= 0) {
                wv[t] = wl[k];
                if (emit == nullptr) dv[t] = dl[k];
            }
        }
#pragma unroll
        for (int t = 0; t < QH; ++t) {
            const int i = threadIdx.x + (q0 + t) * FC_NT;
            const int e = i / NCOL, j = i % NCOL;
            const int u = e * C + c0 + j - offi;   // the correction's bin offset from first
            if (u >= 0) hann_ll_elem(x, u, sm[idx(j, e)], dv[t], wv[t], acc);
        }
    }
    if (emit != nullptr) return;
    hann_ll_store(acc, red, part, (int64_t)row * G + cb);
}

// fused log-likelihood partials: one workgroup per chunk, then a second pass
__global__ void k_loglike_partial(const double2* __restrict__ h, const double2* __restrict__ d,
                                  const double* __restrict__ w, int64_t total,
                                  double* __restrict__ part) {
    // d - h*w rounded like the reference's numpy (product rounded, then difference): no FMA
    // contraction here, so a template equal to the injection gives exactly 0
#pragma clang fp contract(off)
    __shared__ double red[256];
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const double2 dv = d[i];
        const double ww = w[i];
        double rr = dv.x, ri = dv.y;
        if (h) {
            const double2 hv = h[i];
            rr -= hv.x * ww;
            ri -= hv.y * ww;
        }
        acc = fma(rr, rr, fma(ri, ri, acc));
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// (one row per workgroup: partials part[row * np ...], out[row])
__global__ void k_loglike_final(const double* __restrict__ part, int np, double* __restrict__ out) {
    part += (int64_t)blockIdx.x * np;
    out += blockIdx.x;
    __shared__ double red[256];
    double acc = 0.0;
    for (int i = threadIdx.x; i < np; i += blockDim.x) acc += part[i];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = -0.5 * 4.0 * red[0];
}

// noise-weighted inner product partials: sum conj(a) b w (complex), one pair per workgroup
__global__ void k_inner_partial(const double2* __restrict__ a, const double2* __restrict__ b,
                                const double* __restrict__ w, int64_t total,
                                double2* __restrict__ part) {
    __shared__ double rre[256], rim[256];
    double accr = 0.0, acci = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const double2 av = a[i], bv = b[i];
        const double ww = w ? w[i] : 1.0;
        // conj(a) b = (ar br + ai bi) + i (ar bi - ai br)
        accr = fma(ww, fma(av.x, bv.x, av.y * bv.y), accr);
        acci = fma(ww, fma(av.x, bv.y, -av.y * bv.x), acci);
    }
    rre[threadIdx.x] = accr;
    rim[threadIdx.x] = acci;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            rre[threadIdx.x] += rre[threadIdx.x + s];
            rim[threadIdx.x] += rim[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = make_double2(rre[0], rim[0]);
}

__global__ void k_inner_final(const double2* __restrict__ part, int np, double scale,
                              double2* __restrict__ out) {
    __shared__ double rre[256], rim[256];
    double accr = 0.0, acci = 0.0;
    for (int i = threadIdx.x; i < np; i += blockDim.x) {
        accr += part[i].x;
        acci += part[i].y;
    }
    rre[threadIdx.x] = accr;
    rim[threadIdx.x] = acci;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            rre[threadIdx.x] += rre[threadIdx.x + s];
            rim[threadIdx.x] += rim[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = make_double2(scale * rre[0], scale * rim[0]);
}

}  // namespace

// ========================================================================================
// C ABI
// ========================================================================================
extern "C" {

int efd_version(void) { return EFD_VERSION; }

// The sources' hash this library was compiled from (_build.source_id(), passed by _build.py as
// -DEFD_BUILD_ID), kept as a tagged string so the build can check an existing binary without
// loading it: a shipped .so is reused only when its tag matches the sources at hand.
#ifndef EFD_BUILD_ID
#define EFD_BUILD_ID "unversioned"
#endif
__attribute__((used)) static const char efd_build_tag[] = "EFD_BUILD_ID=" EFD_BUILD_ID;
const char* efd_build_id(void) { return efd_build_tag + 13; }

#ifdef EFD_EXP
int efd_exp_counters(unsigned long long* out) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_exp_count), sizeof(unsigned long long) * EXP_NCOUNT));
    return EFD_OK;
}
int efd_exp_tiles(unsigned int* out, unsigned long long* clk) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_exp_tile), sizeof(unsigned int) * 16384));
    HIP_TRY(hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_exp_tclk), sizeof(unsigned long long) * 16384));
    return EFD_OK;
}
#endif

int efd_last_error(char* buf, int len) {
    if (!buf || len <= 0) return EFD_ERR_ARG;
    std::snprintf(buf, (size_t)len, "%s", g_err.c_str());
    return EFD_OK;
}


// the split plan's cost floor (k_segments_one): SPLIT_MIN_COST, or EFD_SPLIT_MIN_COST when set
// (read per preparation; -1 splits every tile of the union: the tests' bitwise check of the
// sub-bin form)
static int32_t split_min_cost() {
    const char* e = getenv("EFD_SPLIT_MIN_COST");
    if (!e || !*e) return SPLIT_MIN_COST;
    const long long x = atoll(e);
    return x >= -1 && x <= (1 << 30) ? (int32_t)x : SPLIT_MIN_COST;
}

int efd_spline_build(const double* x, int n, const double* y, int ninterp, double* coef,
                     void* stream) {
    if (!x || !y || !coef || n < 2 || ninterp <= 0 || n > MAX_NT)
        return fail(EFD_ERR_ARG, "efd_spline_build: bad arguments");
    const int threads = 64;   // spline_shared assumes 64-thread blocks
    const int blocks = (ninterp + threads - 1) / threads;
    hipLaunchKernelGGL(k_spline_shared, dim3(blocks), dim3(threads), sizeof(double) * 5 * n,
                       (hipStream_t)stream, x, n, y, ninterp, coef, (int64_t)4 * ninterp);
    HIP_TRY(hipGetLastError());
    return EFD_OK;
}

size_t efd_modesum_workspace_bytes(int32_t nt, int32_t K, int64_t nf) {
    if (nt < 2 || nt > MAX_NT || K <= 0 || K > MAX_K || nf <= 0) return 0;
    return make_layout(nt, K, nf, 0).total;  // unpaired has the most tiles
}

// Workgroup slots k_modesum has resident at once on the current device (CUs x workgroups per
// CU from the occupancy query), cached per device. A grid with no more tiles than that starts
// every tile together, so there is no dispatch order to choose and k_tile_order is skipped (it
// would only lengthen the preparation: config 5's 43-tile downsampled grid lost 5.7% of its rate
// to it). The kernels' shapes do not depend on the caustic mode or pairing.
static int64_t resident_tile_slots() {
    constexpr int MAX_DEV = 64;
    static std::atomic<int64_t> cache[MAX_DEV];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEV) return 1024;
    int64_t v = cache[dev].load(std::memory_order_relaxed);
    if (v > 0) return v;
    int cus = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, reinterpret_cast<const void*>(&k_modesum<true, EFD_CAUSTIC_UNIFORM, BPL>),
            TILE, 0) != hipSuccess || cus <= 0 || per_cu <= 0)
        return 1024;   // MI355X: 256 CUs x 4 workgroups (LDS-bound)
    v = (int64_t)cus * per_cu;
    cache[dev].store(v, std::memory_order_relaxed);
    return v;
}

// Longest-first dispatch (k_tile_order) for one waveform: only when its tiles outnumber the
// resident slots and it has at least ORDER_MIN_K harmonics. With few harmonics the tiles' record
// lists are short and even, and the sort's ~9 us on the preparation chain cost more than the
// order saved: configs 1 and 3 (tens of harmonics, 3,082 tiles) ran 7% faster without it
// (2,147 / 2,122 vs 2,023 / 1,944 and 8,182 / 8,231 vs 7,777 / 7,410 waveforms/s, two rounds),
// while config 2 (3,020 harmonics) keeps +0.2% (paired A/B, ratio 1.002, CI 1.001-1.003).
// prepare and sum see the same arguments, so they agree on whether tperm exists.
constexpr int32_t ORDER_MIN_K = 1024;
// Prebuilt tile lists (k_tile_keys) from LISTS_MIN_K harmonics up; below, the sum builds
// them itself (short lists: one window pass per tile). With tens of harmonics (eps = 1e-2) the
// in-sum build is cheaper than k_tile_keys' pass over every tile in the batched likelihood:
// config 4's walker groups (bench.py --likelihood, 3 interleaved pairs) 11,253 -> 13,416 logL/s;
// configs 1 / 3 (tools/configs.py, 2 interleaved pairs) 2,938 vs 2,897 and 8,166 vs 7,996
// waveforms/s (neutral), config 5 40,729 vs 39,648 (neutral); config 2 (3,020 harmonics) keeps
// the prebuilt lists.
constexpr int32_t LISTS_MIN_K = 1024;
// (the environment variable EFD_LISTS_MIN_K, read once per process, overrides it:
// a tuning knob; prepare and sum read the same value, so they agree on whether lists exist)
static int32_t lists_min_k() {
    static const int32_t v = [] {
        const char* e = std::getenv("EFD_LISTS_MIN_K");
        return e ? (int32_t)std::atoi(e) : LISTS_MIN_K;
    }();
    return v;
}
static bool use_prebuilt(int32_t K) { return K >= lists_min_k(); }
// Envelope records (k_items, env_fit.inc) in the uniform caustic mode; EFD_ENV=0 (read once per
// process) builds none: the A/B and parity switch of DESIGN.md's round-6 study. prepare decides
// per waveform and the sum follows the records (Item::jser), so they always agree.
static bool env_records() {
    static const bool v = [] {
        const char* e = std::getenv("EFD_ENV");
        return !(e && e[0] == '0');
    }();
    return v;
}
static bool use_cost_order(const Layout& L, int32_t K) {
    return use_prebuilt(K) && K >= ORDER_MIN_K &&
           L.ntiles > resident_tile_slots();
}

// argument checks of efd_modesum / _prepare / _sum (phase as in modesum_impl)
static int check_modesum_args(const efd_modesum_args* a, const void* workspace, int phase) {
    if (!a || !workspace) return fail(EFD_ERR_ARG, "efd_modesum: NULL argument");
    if (!a->t || !a->phi_phi || !a->phi_r || !a->f_phi || !a->f_r || !a->amp || !a->m ||
        !a->n || !a->ylm_p || !a->ylm_m || !a->freq)
        return fail(EFD_ERR_ARG, "efd_modesum: NULL array");
    const bool pol = a->hp != nullptr || a->hc != nullptr;
    if (pol && (!a->hp || !a->hc || !a->grid_symmetric || a->k0 < 0 || a->k0 > a->nf))
        return fail(EFD_ERR_ARG, "efd_modesum: hp/hc need both pointers, a symmetric grid and "
                                 "0 <= k0 <= nf");
    if ((phase & 2) && !a->out && !pol)
        return fail(EFD_ERR_ARG, "efd_modesum: no output (out or hp/hc)");
    if (a->nt < 2 || a->nt > MAX_NT) return fail(EFD_ERR_ARG, "efd_modesum: nt out of range");
    if (a->K <= 0 || a->K > MAX_K) return fail(EFD_ERR_ARG, "efd_modesum: K out of range [1, 8192]");
    if (a->nf <= 0 || a->nf >= (int64_t)INT32_MAX)
        return fail(EFD_ERR_ARG, "efd_modesum: nf out of range");
    if (a->caustic != EFD_CAUSTIC_SPA && a->caustic != EFD_CAUSTIC_UNIFORM)
        return fail(EFD_ERR_ARG, "efd_modesum: unknown caustic mode");
    return EFD_OK;
}

// Preparation (K0-K6) of `count` waveforms in one chain of launches; blockIdx.z = waveform.
// efd_modesum_prepare and efd_modesum's first phase are a batch of one.
static int prepare_batch_impl(const char* fn, const efd_modesum_args* const* a,
                              void* const* workspace, const size_t* workspace_bytes,
                              int32_t count, void* stream) {
    const std::string F(fn);
    if (!a || !workspace || !workspace_bytes) return fail(EFD_ERR_ARG, F + ": NULL argument");
    if (count < 1 || count > EFD_BATCH_MAX)
        return fail(EFD_ERR_ARG, F + ": count out of range [1, EFD_BATCH_MAX]");
    PrepBatch B{};
    B.n = count;
    int ntmax = 0, Kmax = 0, nimax = 0, ntmax_pcr = 0, pcr_blocks = 0;
    bool any_pcr = false, any_thomas = false;
    int64_t items_max = 0, ntiles = 0;
    bool any_lists = false, any_order = false;
    for (int i = 0; i < count; ++i) {
        const efd_modesum_args* ai = a[i];
        const int rc = check_modesum_args(ai, workspace[i], 1);
        if (rc != EFD_OK) return rc;
        if (ai->nf != a[0]->nf || (ai->grid_symmetric != 0) != (a[0]->grid_symmetric != 0))
            return fail(EFD_ERR_ARG, F + ": nf and grid_symmetric must agree across the batch");
        const int paired = ai->grid_symmetric ? 1 : 0;
        const Layout L = make_layout(ai->nt, ai->K, ai->nf, paired);
        if (workspace_bytes[i] < L.total)
            return fail(EFD_ERR_WORKSPACE, F + ": workspace too small (see "
                                               "efd_modesum_workspace_bytes)");
        for (int j = 0; j < i; ++j)
            if (workspace[j] == workspace[i])
                return fail(EFD_ERR_ARG, F + ": one workspace per waveform");
        PrepDesc& d = B.d[i];
        d.t = ai->t; d.phi_phi = ai->phi_phi; d.phi_r = ai->phi_r; d.f_phi = ai->f_phi;
        d.f_r = ai->f_r; d.amp = ai->amp; d.ylm_p = ai->ylm_p; d.ylm_m = ai->ylm_m;
        d.freq = ai->freq; d.m = ai->m; d.n = ai->n;
        d.ws = (char*)workspace[i];
        d.sc_re = ai->scale_re; d.sc_im = ai->scale_im;
        d.nt = ai->nt; d.K = ai->K;
        d.lists = use_prebuilt(ai->K) ? (use_cost_order(L, ai->K) ? 3 : 1) : 0;
        d.env = (ai->caustic == EFD_CAUSTIC_UNIFORM && env_records()) ? 1 : 0;
        any_lists |= d.lists != 0;
        any_order |= d.lists == 3;
#ifdef EFD_EXP_NO_PCR   // experiment: every waveform on the Thomas kernels (the twin's solve order)
        const bool pcr = false;
#else
        const bool pcr = ai->nt >= 4 && ai->nt <= PCR_NMAX;
#endif
        d.pcr = pcr ? (ai->K < PCR_MAX_K ? 3 : 1) : 0;
        if (pcr) {
            any_pcr = true;
            ntmax_pcr = std::max(ntmax_pcr, ai->nt);
            pcr_blocks = std::max(pcr_blocks, 4 + (d.pcr == 3 ? 5 : 1) * ai->K);
        }
        if (d.pcr != 3) any_thomas = true;
        ntmax = std::max(ntmax, ai->nt);
        Kmax = std::max(Kmax, ai->K);
        nimax = std::max(nimax, ai->nt - 1);
        // (G <= K groups; at large K each thread may take several records: config 2's 3,020
        // harmonics form 627 groups, so a K-sized grid was 79% workgroups that exit at once)
        const int64_t per = ai->K >= ITEMS_SPLIT_K ? ITEMS_PER_THREAD_K : 1;
        items_max = std::max(items_max, ((int64_t)(ai->nt - 1) * ai->K + per - 1) / per);
        if (i == 0) {
            B.paired = paired;
            B.nf = ai->nf;
            B.nl = L.nlanes;
            B.nl1 = paired ? ((ai->nf % 2) ? L.nlanes - 1 : L.nlanes) : ai->nf;
            ntiles = L.ntiles;
        }
    }
    (void)nimax;
    hipStream_t st = (hipStream_t)stream;
    const unsigned nz = (unsigned)count;
    // K0: (m, n) groups (in k_prep_pcr_b's blocks when the batch allows) and, for the Thomas
    // kernel's amplitude role, their amplitudes at the knots (the PCR amplitude waves evaluate
    // their own)
    B.pcr_groups = (!any_thomas && Kmax <= PCR_GROUPS_MAX_K) ? 1 : 0;
    {
        if (!B.pcr_groups) {
            hipLaunchKernelGGL(k_group_b, dim3(1, 1, nz), dim3(256), 0, st, B);
            HIP_TRY(hipGetLastError());
        }
        if (any_thomas) {
            const int gper = Kmax >= ITEMS_SPLIT_K ? ITEMS_PER_THREAD_K : 1;
            hipLaunchKernelGGL(k_group_amp_b, dim3((Kmax / gper + 255) / 256, ntmax, nz),
                               dim3(256), 0, st, B);
            HIP_TRY(hipGetLastError());
        }
    }
    // K1-K3: trajectory splines, group amplitude splines, inverse splines (one fused launch;
    // grids sized for G = K, blocks past the device-side G return at once)
    {
        if (any_pcr) {   // one wave per interpolant, parallel cyclic reduction (prep_pcr_body)
            hipLaunchKernelGGL(k_prep_pcr_b, dim3(pcr_blocks, 1, nz), dim3(64),
                               sizeof(double) * 9 * ntmax_pcr, st, B);
            HIP_TRY(hipGetLastError());
        }
        if (any_thomas) {
            const int nb = 1 + (4 * Kmax + 63) / 64 + (Kmax + 63) / 64;
            hipLaunchKernelGGL(k_prep_b, dim3(nb, 1, nz), dim3(64), sizeof(double) * 7 * ntmax,
                               st, B);
            HIP_TRY(hipGetLastError());
        }
    }
    // K4: interval records
    {
        const int64_t blocks = (items_max + 255) / 256;
        hipLaunchKernelGGL(k_items, dim3((unsigned)blocks, 1, nz), dim3(256), 0, st, B);
        HIP_TRY(hipGetLastError());
    }
    // K5: segment table
    if (Kmax <= SEG1_MAX_K) {
        // the largest ranges table of the batch that fits SEG1_LDS_CAP (K N_t int4s at most)
        int64_t need = 0;
        for (int i = 0; i < count; ++i) {
            const int64_t b = (int64_t)a[i]->K * (a[i]->nt - 1) * 16;
            if (b <= SEG1_LDS_CAP) need = std::max(need, b);
        }
        B.seg_lds = (int32_t)need;
        B.split_min = split_min_cost();
        hipLaunchKernelGGL(k_segments_one, dim3(1, 1, nz), dim3(SEG1_NT), (size_t)B.seg_lds, st,
                           B);
        HIP_TRY(hipGetLastError());
    } else {
        const int nslot = Kmax * MAXRUNS * 2;
        const int nblk = (nslot + 255) / 256;
        hipLaunchKernelGGL(k_segment_slots, dim3(nblk, 1, nz), dim3(256), 0, st, B);
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_segment_compact, dim3(nblk, 1, nz), dim3(256), 0, st, B);
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_seg_tiles, dim3((unsigned)std::min(nslot, 1024), 1, nz), dim3(256),
                           0, st, B);
        HIP_TRY(hipGetLastError());
    }
    // K6: the tiles' record lists (k_tile_keys): moves the latency-bound build out of the mode
    // sum into the preparation phase, which overlaps the previous waveform's sum in a two-stream
    // pipeline
    if (any_lists) {
        hipLaunchKernelGGL(k_tile_keys, dim3((unsigned)ntiles, 1, nz), dim3(TILE), 0, st, B);
        HIP_TRY(hipGetLastError());
    }
    if (any_order) {
        hipLaunchKernelGGL(k_tile_order, dim3(1, 1, nz), dim3(1024), 0, st, B);
        HIP_TRY(hipGetLastError());
    }
    return EFD_OK;
}

// phase: 1 = prepare (K0-K6), 2 = sum (K8), 3 = both
static int modesum_impl(const efd_modesum_args* a, void* workspace, size_t workspace_bytes,
                        void* stream, int phase) {
    {
        const int rc = check_modesum_args(a, workspace, phase);
        if (rc != EFD_OK) return rc;
    }
    const int paired = a->grid_symmetric ? 1 : 0;
    const Layout L = make_layout(a->nt, a->K, a->nf, paired);
    if (workspace_bytes < L.total)
        return fail(EFD_ERR_WORKSPACE, "efd_modesum: workspace too small (see efd_modesum_workspace_bytes)");

    hipStream_t st = (hipStream_t)stream;
    char* ws = (char*)workspace;
    Header* hdr = (Header*)(ws + L.header);
    const Item* items = (const Item*)(ws + L.items);
    const int4* ranges = (const int4*)(ws + L.ranges);
    const int2* seglh = (const int2*)(ws + L.seglh);
    const int4* seginfo = (const int4*)(ws + L.seginfo);
    const int32_t* nseg = (const int32_t*)(ws + L.nseg);
    const int32_t* gm = (const int32_t*)(ws + L.gm);
    const int32_t* gn = (const int32_t*)(ws + L.gn);
    const double* coefA = (const double*)(ws + L.coefA);
    const double* coefT = (const double*)(ws + L.coefT);
    const double2* sctab_g = (const double2*)(ws + L.sctab);
    const uint32_t* tkeys = (const uint32_t*)(ws + L.tkeys);
    int32_t* tcnt = (int32_t*)(ws + L.tcnt);
    const int32_t* segbase = (const int32_t*)(ws + L.segbase);
    const int32_t* stb0 = (const int32_t*)(ws + L.stb0);
    const int32_t* stb1 = (const int32_t*)(ws + L.stb1);
    const int nt = a->nt, K = a->K;
    const int64_t nf = a->nf;
    const int64_t nl = L.nlanes;

    if (phase & 1) {
        const int rc = prepare_batch_impl("efd_modesum_prepare", &a, &workspace, &workspace_bytes,
                                          1, stream);
        if (rc != EFD_OK) return rc;
    }
    // K8: mode sum
    if (phase & 2) {
        const int64_t gq = 8 * XCD_GROUP;
        const dim3 grid((unsigned)((L.ntiles + gq - 1) / gq * gq)), block(TILE);
        const int acc = a->accumulate ? 1 : 0;
        if (a->prof_begin) HIP_TRY(hipEventRecord((hipEvent_t)a->prof_begin, st));
        int32_t* tcnt_sum = use_prebuilt(K) ? tcnt : nullptr;
        const int32_t* tperm =
            use_cost_order(L, K)
                ? (const int32_t*)(ws + L.tperm) : nullptr;
#define EFD_LAUNCH(P, C)                                                                      \
    hipLaunchKernelGGL((k_modesum<P, C, BPL>), grid, block, 0, st, items, ranges, seglh,          \
                       seginfo, nseg, a->freq, nf, nl, L.ntiles, nt, K, gm, gn, a->t, coefA,      \
                       coefT, sctab_g, tkeys, tcnt_sum, tperm, segbase, stb0, stb1, hdr, acc,      \
                       a->out, a->hp, a->hc, a->k0)
        if (paired) {
            if (a->caustic == EFD_CAUSTIC_UNIFORM) EFD_LAUNCH(true, EFD_CAUSTIC_UNIFORM);
            else EFD_LAUNCH(true, EFD_CAUSTIC_SPA);
        } else {
            if (a->caustic == EFD_CAUSTIC_UNIFORM) EFD_LAUNCH(false, EFD_CAUSTIC_UNIFORM);
            else EFD_LAUNCH(false, EFD_CAUSTIC_SPA);
        }
#undef EFD_LAUNCH
        HIP_TRY(hipGetLastError());
        if (a->prof_end) HIP_TRY(hipEventRecord((hipEvent_t)a->prof_end, st));
    }
    return EFD_OK;
}

int efd_modesum(const efd_modesum_args* a, void* workspace, size_t workspace_bytes, void* stream) {
    return modesum_impl(a, workspace, workspace_bytes, stream, 3);
}

int efd_modesum_prepare(const efd_modesum_args* a, void* workspace, size_t workspace_bytes,
                        void* stream) {
    return modesum_impl(a, workspace, workspace_bytes, stream, 1);
}

int efd_modesum_prepare_batch(const efd_modesum_args* const* a, void* const* workspace,
                              const size_t* workspace_bytes, int32_t count, void* stream) {
    return prepare_batch_impl("efd_modesum_prepare_batch", a, workspace, workspace_bytes, count,
                              stream);
}

int efd_modesum_sum(const efd_modesum_args* a, void* workspace, size_t workspace_bytes,
                    void* stream) {
    return modesum_impl(a, workspace, workspace_bytes, stream, 2);
}

// efd_modesum_sum_batch, and efd_modesum_sum_loglike when d != NULL (paired grids: the tiles
// write their likelihood partials, k_ll_final turns each waveform's into out[i])
constexpr int64_t SPARSE_WG = 4096;   // workgroups of a sparse launch, all waveforms
// (EFD_SPARSE_WG overrides it: an experiment switch for paired A/B runs, read once)
static int64_t sparse_wg() {
    static const int64_t v = [] {
        const char* e = getenv("EFD_SPARSE_WG");
        const long long x = e ? atoll(e) : 0;
        return x >= 64 && x <= (1 << 20) ? (int64_t)x : SPARSE_WG;
    }();
    return v;
}
int sum_batch_impl(const char* fn, const efd_modesum_args* const* a, void* const* workspace,
                   const size_t* workspace_bytes, int32_t count, const double* d, const double* w,
                   double* llout, void* stream, const double* llconst = nullptr) {
    const std::string F(fn);
    if (!a || !workspace || !workspace_bytes)
        return fail(EFD_ERR_ARG, F + ": NULL argument");
    if (count < 1 || count > EFD_BATCH_MAX)
        return fail(EFD_ERR_ARG, F + ": count out of range [1, EFD_BATCH_MAX]");
    SumBatch batch{};
    batch.n = count;
    Layout L0{};
    for (int i = 0; i < count; ++i) {
        const efd_modesum_args* ai = a[i];
        // (the fused likelihood needs no written output)
        const int rc = check_modesum_args(ai, workspace[i], d ? 0 : 2);
        if (rc != EFD_OK) return rc;
        if (ai->nf != a[0]->nf || (ai->grid_symmetric != 0) != (a[0]->grid_symmetric != 0) ||
            ai->caustic != a[0]->caustic || (ai->accumulate != 0) != (a[0]->accumulate != 0))
            return fail(EFD_ERR_ARG, F + ": nf, grid_symmetric, caustic and accumulate must agree "
                                         "across the batch");
        if (d && (!ai->grid_symmetric || ai->accumulate || ai->k0 != a[0]->k0 || ai->k0 < 0 ||
                  ai->k0 >= ai->nf))
            return fail(EFD_ERR_ARG, F + ": the fused likelihood needs a symmetric grid, "
                                         "accumulate = 0 and one 0 <= k0 < nf for the batch");
        const int paired = ai->grid_symmetric ? 1 : 0;
        const Layout L = make_layout(ai->nt, ai->K, ai->nf, paired);
        if (workspace_bytes[i] < L.total)
            return fail(EFD_ERR_WORKSPACE, F + ": workspace too small (see "
                                               "efd_modesum_workspace_bytes)");
        if (i == 0) L0 = L;
        char* ws = (char*)workspace[i];
        BatchDesc& d = batch.d[i];
        d.items = (const Item*)(ws + L.items);
        d.ranges = (const int4*)(ws + L.ranges);
        d.seglh = (const int2*)(ws + L.seglh);
        d.seginfo = (const int4*)(ws + L.seginfo);
        d.nseg = (const int32_t*)(ws + L.nseg);
        d.freq = ai->freq;
        d.gm = (const int32_t*)(ws + L.gm);
        d.gn = (const int32_t*)(ws + L.gn);
        d.t = ai->t;
        d.coefA = (const double*)(ws + L.coefA);
        d.coefT = (const double*)(ws + L.coefT);
        d.sctab = (const double2*)(ws + L.sctab);
        d.tkeys = (const uint32_t*)(ws + L.tkeys);
        d.tcnt = use_prebuilt(ai->K) ? (const int32_t*)(ws + L.tcnt) : nullptr;
        d.tperm = use_cost_order(L, ai->K)
                      ? (const int32_t*)(ws + L.tperm) : nullptr;
        d.segbase = (const int32_t*)(ws + L.segbase);
        d.stb0 = (const int32_t*)(ws + L.stb0);
        d.stb1 = (const int32_t*)(ws + L.stb1);
        d.hdr = (Header*)(ws + L.header);
        d.out = ai->out;
        d.hp = ai->hp;
        d.hc = ai->hc;
        d.llpart = (double*)(ws + L.llpart);
        d.k0 = ai->k0;
        d.nt = ai->nt;
        d.K = ai->K;
    }
    hipStream_t st = (hipStream_t)stream;
    // the sparse form (k_modesum_batch): the fused likelihood with tile constants, nothing
    // written, and in-kernel lists (below 1,024 harmonics: the sparse spectra; denser ones keep
    // the longest-first order over every tile)
    bool sparse = d != nullptr && llconst != nullptr && a[0]->grid_symmetric;
    for (int i = 0; i < count && sparse; ++i)
        sparse = !a[i]->out && !a[i]->hp && !a[i]->hc && !use_prebuilt(a[i]->K) &&
                 !use_cost_order(make_layout(a[i]->nt, a[i]->K, a[i]->nf, 1), a[i]->K);
    const int64_t gq = 8 * XCD_GROUP;
    int64_t nper = 0;
    if (sparse) {
        // workgroups per waveform: a multiple of 8 (one XCD place each), ~SPARSE_WG in all. With
        // a possible split plan (K <= SEG1_MAX_K: k_segments_one; its item count is on the
        // device) the whole share, so every item of a plan gets its own workgroup (those past
        // the items exit at once)
        const int64_t cap = std::max<int64_t>(64, (sparse_wg() / count + 7) / 8 * 8);
        bool planned = true;
        for (int i = 0; i < count; ++i) planned = planned && a[i]->K <= SEG1_MAX_K;
        nper = planned ? cap : std::min<int64_t>((L0.ntiles + 7) / 8 * 8, cap);
    }
    const int64_t nblk = sparse ? nper * count : (L0.ntiles + gq - 1) / gq * gq * count;
    if (nblk > (int64_t)UINT32_MAX) return fail(EFD_ERR_ARG, F + ": grid too large");
    const dim3 grid((unsigned)nblk), block(TILE);
    const int acc = a[0]->accumulate ? 1 : 0;
    if (a[0]->prof_begin) HIP_TRY(hipEventRecord((hipEvent_t)a[0]->prof_begin, st));
#define EFD_LAUNCH(P, C)                                                                      \
    do {                                                                                      \
        if (sparse)                                                                           \
            hipLaunchKernelGGL((k_modesum_batch<P, C, BPL, true>), grid, block, 0, st, batch,  \
                               a[0]->nf, L0.nlanes, L0.ntiles, acc, d, w, llconst, nper);     \
        else                                                                                  \
            hipLaunchKernelGGL((k_modesum_batch<P, C, BPL, false>), grid, block, 0, st, batch, \
                               a[0]->nf, L0.nlanes, L0.ntiles, acc, d, w,                     \
                               d ? llconst : nullptr, (int64_t)0);                            \
    } while (0)
    if (a[0]->grid_symmetric) {
        if (a[0]->caustic == EFD_CAUSTIC_UNIFORM) EFD_LAUNCH(true, EFD_CAUSTIC_UNIFORM);
        else EFD_LAUNCH(true, EFD_CAUSTIC_SPA);
    } else {
        if (a[0]->caustic == EFD_CAUSTIC_UNIFORM) EFD_LAUNCH(false, EFD_CAUSTIC_UNIFORM);
        else EFD_LAUNCH(false, EFD_CAUSTIC_SPA);
    }
#undef EFD_LAUNCH
    HIP_TRY(hipGetLastError());
    if (d) {
        LlBatch lb{};
        lb.n = count;
        lb.ntiles = L0.ntiles;
        for (int i = 0; i < count; ++i) {
            lb.part[i] = batch.d[i].llpart;
            lb.hdr[i] = (const Header*)workspace[i];
        }
        lb.out = llout;
        lb.llconst = sparse ? llconst : nullptr;
        hipLaunchKernelGGL(k_ll_final, dim3((unsigned)count), dim3(256), 0, st, lb);
        HIP_TRY(hipGetLastError());
    }
    if (a[0]->prof_end) HIP_TRY(hipEventRecord((hipEvent_t)a[0]->prof_end, st));
    return EFD_OK;
}

int efd_modesum_sum_batch(const efd_modesum_args* const* a, void* const* workspace,
                          const size_t* workspace_bytes, int32_t count, void* stream) {
    return sum_batch_impl("efd_modesum_sum_batch", a, workspace, workspace_bytes, count, nullptr,
                          nullptr, nullptr, stream);
}

int efd_modesum_sum_loglike(const efd_modesum_args* const* a, void* const* workspace,
                            const size_t* workspace_bytes, int32_t count, const double* d,
                            const double* w, double* out, void* stream) {
    if (!d || !w || !out) return fail(EFD_ERR_ARG, "efd_modesum_sum_loglike: NULL d, w or out");
    return sum_batch_impl("efd_modesum_sum_loglike", a, workspace, workspace_bytes, count, d, w,
                          out, stream);
}

int64_t efd_loglike_tile_count(int64_t nf) {
    if (nf < 1) return 0;
    return make_layout(2, 1, nf, 1).ntiles;
}

int efd_loglike_tile_constants(const double* d, const double* w, int64_t nf, int64_t k0,
                               double* tile_const, void* stream) {
    if (!d || !w || !tile_const)
        return fail(EFD_ERR_ARG, "efd_loglike_tile_constants: NULL d, w or tile_const");
    if (nf < 1 || k0 < 0 || k0 >= nf)
        return fail(EFD_ERR_ARG, "efd_loglike_tile_constants: need nf >= 1 and 0 <= k0 < nf");
    const Layout L = make_layout(2, 1, nf, 1);
    if (L.ntiles > (int64_t)UINT32_MAX) return fail(EFD_ERR_ARG, "efd_loglike_tile_constants: grid too large");
    hipLaunchKernelGGL(k_ll_tile_const<BPL>, dim3((unsigned)L.ntiles), dim3(TILE), 0,
                       (hipStream_t)stream, d, w, nf, L.nlanes, k0, tile_const);
    HIP_TRY(hipGetLastError());
    return EFD_OK;
}

int efd_modesum_sum_loglike_ex(const efd_modesum_args* const* a, void* const* workspace,
                               const size_t* workspace_bytes, int32_t count, const double* d,
                               const double* w, const double* tile_const, double* out,
                               void* stream) {
    if (!d || !w || !out)
        return fail(EFD_ERR_ARG, "efd_modesum_sum_loglike_ex: NULL d, w or out");
    return sum_batch_impl("efd_modesum_sum_loglike_ex", a, workspace, workspace_bytes, count, d,
                          w, out, stream, tile_const);
}

// One walker group of the fused likelihood in one call (Likelihood.get_ll's per-group host
// path, likelihood.py:246-274 callers): efd_stage_batch into pin, the copy to dbuf, staged_event
// recorded after it (the pinned buffer's reuse waits on it), efd_modesum_prepare_batch and
// efd_modesum_sum_loglike_ex in launches of EFD_BATCH_MAX walkers, all on `stream`: the five
// ctypes transitions and the argument handling of the Python steps in one.
int efd_fused_group(void* pin, size_t pin_bytes, void* dbuf, size_t dbuf_bytes, int32_t count,
                    const uint64_t* src, const int32_t* shape, const double* scale,
                    const efd_modesum_args* tmpl, efd_modesum_args* args,
                    void* const* workspace, const size_t* workspace_bytes, const double* d,
                    const double* w, const double* tile_const, double* out, void* staged_event,
                    void* stream, size_t* total) {
    if (count < 1 || !args || !workspace || !workspace_bytes || !d || !w || !out || !total)
        return fail(EFD_ERR_ARG, "efd_fused_group: bad arguments");
    const int rs = efd_stage_batch(pin, pin_bytes, (uint64_t)(uintptr_t)dbuf, count, src, shape,
                                   scale, tmpl, args, total);
    if (rs == EFD_ERR_WORKSPACE || (rs == EFD_OK && (!dbuf || *total > dbuf_bytes)))
        return EFD_ERR_WORKSPACE;   // the caller grows pin / dbuf to *total and calls again
    if (rs != EFD_OK) return fail(rs, "efd_fused_group: staging failed (efd_stage_batch)");
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(hipMemcpyAsync(dbuf, pin, *total, hipMemcpyHostToDevice, st));
    if (staged_event) HIP_TRY(hipEventRecord((hipEvent_t)staged_event, st));
    const efd_modesum_args* ap[EFD_BATCH_MAX];
    for (int32_t c0 = 0; c0 < count; c0 += EFD_BATCH_MAX) {
        const int32_t cnt = std::min<int32_t>(EFD_BATCH_MAX, count - c0);
        for (int32_t i = 0; i < cnt; ++i) ap[i] = &args[c0 + i];
        const int rc = efd_modesum_prepare_batch(ap, workspace + c0, workspace_bytes + c0, cnt,
                                                 stream);
        if (rc != EFD_OK) return rc;
    }
    for (int32_t c0 = 0; c0 < count; c0 += EFD_BATCH_MAX) {
        const int32_t cnt = std::min<int32_t>(EFD_BATCH_MAX, count - c0);
        for (int32_t i = 0; i < cnt; ++i) ap[i] = &args[c0 + i];
        const int rc = efd_modesum_sum_loglike_ex(ap, workspace + c0, workspace_bytes + c0, cnt,
                                                  d, w, tile_const, out + c0, stream);
        if (rc != EFD_OK) return rc;
    }
    return EFD_OK;
}

int efd_modesum_status(const void* workspace, void* stream) {
    if (!workspace) return fail(EFD_ERR_ARG, "efd_modesum_status: NULL workspace");
    Header h{};
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    HIP_TRY(hipMemcpy(&h, workspace, sizeof(Header), hipMemcpyDeviceToHost));
    if (h.runs_overflow != 0 || h.bad_mn != 0 || h.bad_tile != 0) {
        // reported once: clear the sticky flags (the stream is idle, so nothing races this)
        char* w = (char*)const_cast<void*>(workspace);
        HIP_TRY(hipMemset(w + offsetof(Header, runs_overflow), 0, sizeof(int32_t)));
        HIP_TRY(hipMemset(w + offsetof(Header, bad_mn), 0, 2 * sizeof(int32_t)));
    }
    if (h.runs_overflow != 0)
        return fail(EFD_ERR_ARG, "efd_modesum: a harmonic has more than 8 monotonic runs");
    if (h.bad_mn != 0)
        return fail(EFD_ERR_ARG, "efd_modesum: |m| > 255 or |n| > 1023");
    if (h.bad_tile != 0)
        return fail(EFD_ERR_HIP, "efd_modesum: a tile dispatch-order entry was out of range "
                                 "(prepare/sum workspace mismatch?); bins were left unwritten");
    return EFD_OK;
}

int efd_modesum_lane_ranges(void* const* workspace, int32_t count, int32_t* out, void* stream) {
    if (!workspace || !out || count < 1 || count > EFD_BATCH_MAX)
        return fail(EFD_ERR_ARG, "efd_modesum_lane_ranges: NULL argument or count out of range "
                                 "[1, EFD_BATCH_MAX]");
    StatusBatch sb{};
    sb.n = count;
    for (int i = 0; i < count; ++i) {
        if (!workspace[i]) return fail(EFD_ERR_ARG, "efd_modesum_lane_ranges: NULL workspace");
        sb.h[i] = (Header*)workspace[i];
    }
    hipLaunchKernelGGL(k_lane_gather, dim3(1), dim3(64), 0, (hipStream_t)stream, sb, out);
    HIP_TRY(hipGetLastError());
    return EFD_OK;
}

int efd_modesum_status_batch(void* const* workspace, int32_t count, int32_t* flags,
                             void* stream) {
    if (!workspace || count < 1 || count > EFD_BATCH_MAX)
        return fail(EFD_ERR_ARG, "efd_modesum_status_batch: NULL workspaces or count out of "
                                 "range [1, EFD_BATCH_MAX]");
    StatusBatch sb{};
    sb.n = count;
    for (int i = 0; i < count; ++i) {
        if (!workspace[i]) return fail(EFD_ERR_ARG, "efd_modesum_status_batch: NULL workspace");
        sb.h[i] = (Header*)workspace[i];
    }
    // one gather kernel writing into mapped host memory, one synchronisation: the flags of a
    // walker batch cost what one efd_modesum_status costs
    static std::mutex mu;
    static int32_t* host = nullptr;
    std::lock_guard<std::mutex> lock(mu);
    if (!host) HIP_TRY(hipHostMalloc((void**)&host, sizeof(int32_t) * EFD_BATCH_MAX,
                                     hipHostMallocMapped));
    int32_t* dev = nullptr;
    HIP_TRY(hipHostGetDevicePointer((void**)&dev, host, 0));
    hipLaunchKernelGGL(k_status_gather, dim3(1), dim3(64), 0, (hipStream_t)stream, sb, dev);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    int first = -1;
    for (int i = 0; i < count; ++i) {
        const int32_t f = ((volatile int32_t*)host)[i];
        if (flags) flags[i] = f;
        if (f && first < 0) first = i;
    }
    if (first < 0) return EFD_OK;
    const int32_t f = host[first];
    const std::string w = "efd_modesum (waveform " + std::to_string(first) + " of the batch): ";
    if (f & 1) return fail(EFD_ERR_ARG, w + "a harmonic has more than 8 monotonic runs");
    if (f & 2) return fail(EFD_ERR_ARG, w + "|m| > 255 or |n| > 1023");
    return fail(EFD_ERR_HIP, w + "a tile dispatch-order entry was out of range (prepare/sum "
                                 "workspace mismatch?); bins were left unwritten");
}

int efd_modesum_contributions(const void* workspace, int64_t* contributions, void* stream) {
    if (!workspace || !contributions) return fail(EFD_ERR_ARG, "NULL argument");
    Header h{};
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    HIP_TRY(hipMemcpy(&h, workspace, sizeof(Header), hipMemcpyDeviceToHost));
    *contributions = h.contributions;
    return EFD_OK;
}

int efd_modesum_stats(const void* workspace, int64_t* contributions, int64_t* evaluations,
                      int32_t* groups, void* stream) {
    if (!workspace) return fail(EFD_ERR_ARG, "NULL argument");
    Header h{};
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    HIP_TRY(hipMemcpy(&h, workspace, sizeof(Header), hipMemcpyDeviceToHost));
    if (contributions) *contributions = h.contributions;
    if (evaluations) *evaluations = h.evaluations;
    if (groups) *groups = h.groups;
    return EFD_OK;
}

int efd_modesum_env_evaluations(const void* workspace, int64_t* env_evaluations, void* stream) {
    if (!workspace || !env_evaluations) return fail(EFD_ERR_ARG, "NULL argument");
    Header h{};
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    HIP_TRY(hipMemcpy(&h, workspace, sizeof(Header), hipMemcpyDeviceToHost));
    *env_evaluations = h.env_evaluations;
    return EFD_OK;
}

// TD workspace: the FD layout's grouping and spline buffers only (no records, no tile lists)
struct TdLayout {
    size_t header, coefA, coefT, kslope, tscratch, gm, gn, gstart, gmem, gkeys, gamp, total;
};
static TdLayout make_td_layout(int32_t nt, int32_t K) {
    TdLayout L{};
    const int64_t ni = nt - 1;
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off = align256(off + bytes); return o; };
    L.header = take(sizeof(Header));
    L.coefA = take(sizeof(double) * ni * 4 * 4 * K);
    L.coefT = take(sizeof(double) * ni * 4 * 8);
    L.kslope = take(sizeof(double) * nt * 2);
    L.tscratch = take(sizeof(double) * nt * 16);
    L.gm = take(sizeof(int32_t) * K);
    L.gn = take(sizeof(int32_t) * K);
    L.gstart = take(sizeof(int32_t) * (K + 1));
    L.gmem = take(sizeof(int32_t) * K);
    L.gkeys = take(sizeof(unsigned long long) * (size_t)MAX_K);
    L.gamp = take(sizeof(double) * nt * 4 * K);
    L.total = off;
    return L;
}

size_t efd_td_workspace_bytes(int32_t nt, int32_t K) {
    if (nt < 2 || nt > MAX_NT || K <= 0 || K > MAX_K) return 0;
    return make_td_layout(nt, K).total;
}

int efd_td_modesum(const efd_td_args* a, void* workspace, size_t workspace_bytes, void* stream) {
    if (!a || !workspace) return fail(EFD_ERR_ARG, "efd_td_modesum: NULL argument");
    if (!a->t || !a->phi_phi || !a->phi_r || !a->f_phi || !a->f_r || !a->amp || !a->m ||
        !a->n || !a->ylm_p || !a->ylm_m)
        return fail(EFD_ERR_ARG, "efd_td_modesum: NULL array");
    if (!a->out && !a->hp && !a->hc)
        return fail(EFD_ERR_ARG, "efd_td_modesum: no output (out, hp or hc)");
    if (a->nt < 2 || a->nt > MAX_NT) return fail(EFD_ERR_ARG, "efd_td_modesum: nt out of range");
    if (a->K <= 0 || a->K > MAX_K)
        return fail(EFD_ERR_ARG, "efd_td_modesum: K out of range [1, 8192]");
    if (a->nsamples <= 0 || a->nsamples > ((int64_t)1 << 40))
        return fail(EFD_ERR_ARG, "efd_td_modesum: nsamples out of range");
    if (!(a->dt > 0.0)) return fail(EFD_ERR_ARG, "efd_td_modesum: dt must be > 0");
    const TdLayout L = make_td_layout(a->nt, a->K);
    if (workspace_bytes < L.total)
        return fail(EFD_ERR_WORKSPACE,
                    "efd_td_modesum: workspace too small (see efd_td_workspace_bytes)");
    hipStream_t st = (hipStream_t)stream;
    char* ws = (char*)workspace;
    Header* hdr = (Header*)(ws + L.header);
    double* coefA = (double*)(ws + L.coefA);
    double* coefT = (double*)(ws + L.coefT);
    int32_t* gm = (int32_t*)(ws + L.gm);
    int32_t* gn = (int32_t*)(ws + L.gn);
    int32_t* gstart = (int32_t*)(ws + L.gstart);
    int32_t* gmem = (int32_t*)(ws + L.gmem);
    double* gamp = (double*)(ws + L.gamp);
    const int nt = a->nt, K = a->K;

    HIP_TRY(hipMemsetAsync(hdr, 0, sizeof(Header), st));
    hipLaunchKernelGGL(k_group, dim3(1), dim3(256), 0, st, a->m, a->n, K, gm, gn, gstart, gmem,
                       hdr, (double2*)nullptr, (unsigned long long*)(ws + L.gkeys));
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_group_amp, dim3((K + 255) / 256, nt), dim3(256), 0, st, a->amp, a->ylm_p,
                       a->ylm_m, a->scale_re, a->scale_im, gm, gstart, gmem, nt, K, hdr, gamp);
    HIP_TRY(hipGetLastError());
    // k_prep's first two roles only (trajectory splines, group amplitude splines): the grid
    // stops before the inverse-spline blocks, which the TD sum does not need
    const int nb_amp = (4 * K + 63) / 64;
    hipLaunchKernelGGL(k_prep, dim3(1 + nb_amp), dim3(64), sizeof(double) * 7 * nt, st, a->t,
                       a->phi_phi, a->phi_r, a->f_phi, a->f_r, gamp, gm, gn, nt, K, nb_amp, coefT,
                       (double*)(ws + L.kslope), (double*)(ws + L.tscratch), coefA,
                       (int32_t*)nullptr, (Item*)nullptr, (double*)nullptr, (double*)nullptr, hdr);
    HIP_TRY(hipGetLastError());
    const int64_t per_block = (int64_t)TD_THREADS * TD_SPL;
    const int64_t nblk = (a->nsamples + per_block - 1) / per_block;
    if (nblk > 0x7fffffffLL) return fail(EFD_ERR_ARG, "efd_td_modesum: too many samples");
    if (a->prof_begin) HIP_TRY(hipEventRecord((hipEvent_t)a->prof_begin, st));
    hipLaunchKernelGGL(k_td_modesum, dim3((unsigned)nblk), dim3(TD_THREADS), 0, st, a->t, nt,
                       coefT, coefA, gm, gn, K, hdr, a->dt, a->nsamples, a->accumulate ? 1 : 0,
                       a->out, a->hp, a->hc);
    HIP_TRY(hipGetLastError());
    if (a->prof_end) HIP_TRY(hipEventRecord((hipEvent_t)a->prof_end, st));
    return EFD_OK;
}

int efd_upload(void* dst, const void* src, size_t bytes, void* stream) {
    if (bytes == 0) return EFD_OK;
    if (!dst || !src) return fail(EFD_ERR_ARG, "efd_upload: NULL pointer");
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
    return EFD_OK;
}

int efd_download(void* dst, const void* src, size_t bytes, void* stream) {
    if (bytes == 0) return EFD_OK;
    if (!dst || !src) return fail(EFD_ERR_ARG, "efd_download: NULL pointer");
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
    return EFD_OK;
}

int efd_stream_order(void* src, void* const* dst, int32_t count) {
    if (count < 0 || (count > 0 && !dst))
        return fail(EFD_ERR_ARG, "efd_stream_order: need count >= 0 and a stream array");
    if (count == 0) return EFD_OK;
    // one event per thread and device, re-recorded each call: a wait already enqueued keeps the
    // record it saw (stream-wait semantics), so reuse never loosens an earlier ordering
    // The event belongs to the source stream's device (not the caller's current device, which
    // may have changed since the streams were made): created and recorded with that device
    // current, the caller's device restored afterwards.
    constexpr int MAX_DEV = 64;
    thread_local hipEvent_t ev[MAX_DEV] = {};
    int cur = 0, dev = 0;
    HIP_TRY(hipGetDevice(&cur));
    dev = cur;
    if (src) HIP_TRY(hipStreamGetDevice((hipStream_t)src, &dev));
    if (dev < 0 || dev >= MAX_DEV) return fail(EFD_ERR_ARG, "efd_stream_order: device index");
    if (dev != cur) HIP_TRY(hipSetDevice(dev));
    hipError_t e = hipSuccess;
    if (!ev[dev]) e = hipEventCreateWithFlags(&ev[dev], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(ev[dev], (hipStream_t)src);
    for (int32_t i = 0; e == hipSuccess && i < count; ++i)
        if (dst[i] != src) e = hipStreamWaitEvent((hipStream_t)dst[i], ev[dev], 0);
    if (dev != cur) HIP_TRY(hipSetDevice(cur));
    HIP_TRY(e);
    return EFD_OK;
}

int efd_polarizations(const double* S, int64_t nf, int64_t k0, double* hp, double* hc,
                      void* stream) {
    if (!S || !hp || !hc || nf <= 0 || k0 < 0 || k0 > nf)
        return fail(EFD_ERR_ARG, "efd_polarizations: bad arguments");
    const int64_t cnt = nf - k0;
    if (cnt == 0) return EFD_OK;
    const int threads = 256;
    const int64_t blocks = (cnt + threads - 1) / threads;
    hipLaunchKernelGGL(k_polarizations, dim3((unsigned)blocks), dim3(threads), 0,
                       (hipStream_t)stream, (const double2*)S, nf, k0, (double2*)hp, (double2*)hc);
    HIP_TRY(hipGetLastError());
    return EFD_OK;
}

static bool hann_rows_ok(const char* fn, const void* S, int64_t stride, int64_t nf,
                         int32_t rows) {
    if (!S || nf < 3 || rows < 1 || rows > 65535 || stride < nf) {
        fail(EFD_ERR_ARG, std::string(fn) + ": bad arguments");
        return false;
    }
    return true;
}
int efd_hann_extent(const double* S, int64_t stride, int64_t nf, int32_t rows,
                    const int32_t* lanes, uint64_t* info, void* stream) {
    if (!hann_rows_ok("efd_hann_extent", S, stride, nf, rows) || !info)
        return fail(EFD_ERR_ARG, "efd_hann_extent: bad arguments");
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_hann_info_init, dim3((unsigned)((rows + 63) / 64)), dim3(64), 0, st, info,
                       rows);
    HIP_TRY(hipGetLastError());
    // (with lane ranges the rows' supports are a fraction of the grid: fewer workgroups; each
    // block's 3 atomics on its row's words serialise, so the grid stays small -- 512 blocks a
    // row took 94 against 44 us for 32, r05z8 -- and the loop is unrolled for loads in flight)
    const int64_t cap = lanes ? std::max(16, 512 / rows) : std::max(64, 1024 / rows);
    const int64_t blocks = std::min<int64_t>(cap, (nf + 255) / 256);
    hipLaunchKernelGGL(k_hann_extent, dim3((unsigned)blocks, (unsigned)rows), dim3(256), 0, st,
                       (const double2*)S, stride, nf, lanes, info);
    HIP_TRY(hipGetLastError());
    return EFD_OK;
}
int efd_hann_stage(const double* S, int64_t stride, int64_t nf, int32_t rows,
                   const uint64_t* info, int64_t m, float* Y, void* stream) {
    if (!hann_rows_ok("efd_hann_stage", S, stride, nf, rows) || !info || !Y || m < nf)
        return fail(EFD_ERR_ARG, "efd_hann_stage: bad arguments");
    const int64_t blocks = std::min<int64_t>(4096, (m + 255) / 256);
    hipLaunchKernelGGL(k_hann_stage, dim3((unsigned)blocks, (unsigned)rows), dim3(256), 0,
                       (hipStream_t)stream, (const double2*)S, stride, info, m, (float2*)Y);
    HIP_TRY(hipGetLastError());
    return EFD_OK;
}
// the four-step split's row length C for a transform length m (the lag kernel's spectrum is
// laid out [f_r][f_c], R = m / C): 16384 at m = 2^24 (1024 x 16384: the column kernels read
// 128 B segments, r05z; the 2048 x 8192 split measured 1.08 against 0.73 ms of column passes and
// was deleted in round 6), else 8192
int efd_hann_four_step_cols(int64_t m) {
    return m == ((int64_t)1 << 24) ? FC_C16 : FC_C;
}
// the four-step pipeline for power-of-two m in [2^21, 2^25]: forward columns (staging folded
// in) and rows (the kernel spectrum kfp between the row transforms), then either the inverse
// columns (Y = the correction, efd_hann_convolve) or the inverse columns with the windowed logL
// reduced in place (ll != nullptr: efd_hann_loglike_local)
}  // extern "C"
struct HannLocal {
    const double2* dl;
    const double* wl;
    int64_t kself;
    double2 kfix;
    double* part;
    double2* emit;
};
template <int RR, int CC>
static int hann_pipeline(const double* S, int64_t stride, int64_t nf, int32_t rows,
                         const uint64_t* info, const float* kfp, float* Y, const HannLocal* ll,
                         hipStream_t st) {
    constexpr int NC = FcCols<RR>::NCOL;
    constexpr int64_t M = (int64_t)RR * CC;
    float2* y = (float2*)Y;
    if constexpr (CC == FC_C16) {
        static_assert(RR == FCD_R && NC == FCD_NCOL, "1024 x 16384 split");
        hipLaunchKernelGGL(k_fc_cols1024, dim3(CC / NC, (unsigned)rows), dim3(FC_NT), 0, st,
                           (const double2*)S, stride, info, y);
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_fc_rows16k_h, dim3(RR * (unsigned)rows), dim3(FC_NT), 0, st,
                           (const float2*)kfp, M, (int)rows, y);
    } else {
        hipLaunchKernelGGL((k_fc_cols<true, RR, CC>), dim3(CC / NC, (unsigned)rows), dim3(FC_NT),
                           0, st, (const double2*)S, stride, info, y);
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_fc_rows, dim3(RR * (unsigned)rows), dim3(FR_NT), 0, st,
                           (const float2*)kfp, M, (int)rows, y);
    }
    HIP_TRY(hipGetLastError());
    if (ll == nullptr) {
        hipLaunchKernelGGL((k_fc_cols<false, RR, CC>), dim3(CC / NC, (unsigned)rows),
                           dim3(FC_NT), 0, st, (const double2*)nullptr, (int64_t)0,
                           (const uint64_t*)nullptr, y);
    } else {
        hipLaunchKernelGGL((k_fc_cols_ll<RR, CC>), dim3((CC / NC) * (unsigned)rows), dim3(FC_NT),
                           0, st, (const double2*)S, stride, info, (const float2*)y, nf, ll->dl,
                           ll->wl, ll->kself, ll->kfix, (int)rows, ll->part, ll->emit);
    }
    HIP_TRY(hipGetLastError());
    return EFD_OK;
}
static int hann_pipeline_m(const double* S, int64_t stride, int64_t nf, int32_t rows,
                           const uint64_t* info, int64_t m, const float* kfp, float* Y,
                           const HannLocal* ll, hipStream_t st) {
    if (m == ((int64_t)1 << 24))
        return hann_pipeline<(1 << 24) / FC_C16, FC_C16>(S, stride, nf, rows, info, kfp, Y, ll, st);
    switch (m / FC_C) {   // R = 2048 is m = 2^24, the 1024 x 16384 split above
        case 256: return hann_pipeline<256, FC_C>(S, stride, nf, rows, info, kfp, Y, ll, st);
        case 512: return hann_pipeline<512, FC_C>(S, stride, nf, rows, info, kfp, Y, ll, st);
        case 1024: return hann_pipeline<1024, FC_C>(S, stride, nf, rows, info, kfp, Y, ll, st);
        case 4096: return hann_pipeline<4096, FC_C>(S, stride, nf, rows, info, kfp, Y, ll, st);
        default: return fail(EFD_ERR_ARG, "efd_hann_convolve: no four-step split for this m");
    }
}
extern "C" {
static bool hann_four_step_m(int64_t m, int64_t nf) {
    return m >= nf && m >= ((int64_t)1 << 21) && m <= ((int64_t)1 << 25) && (m & (m - 1)) == 0;
}
int efd_hann_convolve(const double* S, int64_t stride, int64_t nf, int32_t rows,
                      const uint64_t* info, int64_t m, const float* kfp, float* Y, void* stream) {
    if (!hann_rows_ok("efd_hann_convolve", S, stride, nf, rows) || !info || !kfp || !Y ||
        !hann_four_step_m(m, nf))
        return fail(EFD_ERR_ARG, "efd_hann_convolve: bad arguments (m: a power of two in "
                                 "[2^21, 2^25], >= nf)");
    return hann_pipeline_m(S, stride, nf, rows, info, m, kfp, Y, nullptr, (hipStream_t)stream);
}
int efd_hann_loglike_local_partials(int64_t m) {
    if (m == ((int64_t)1 << 24)) return FC_C16 / FcCols<(1 << 24) / FC_C16>::NCOL;
    switch (m / FC_C) {
        case 256: return FC_C / FcCols<256>::NCOL;
        case 512: return FC_C / FcCols<512>::NCOL;
        case 1024: return FC_C / FcCols<1024>::NCOL;
        case 4096: return FC_C / FcCols<4096>::NCOL;
        default: return 0;
    }
}
int efd_hann_loglike_local(const double* S, int64_t stride, int64_t nf, int32_t rows,
                           const uint64_t* info, int64_t m, const float* kfd, float* Y,
                           const double* dl, const double* wl, int64_t kself, double* out,
                           double* scratch, double* emit, void* stream) {
    const int np = hann_four_step_m(m, nf) ? efd_hann_loglike_local_partials(m) : 0;
    if (!hann_rows_ok("efd_hann_loglike_local", S, stride, nf, rows) || !info || !kfd || !Y ||
        !wl || np == 0 || kself < -1 || kself >= nf ||
        (emit ? rows != 1 : (!dl || !out || !scratch || rows > HANN_ROWS_MAX)))
        return fail(EFD_ERR_ARG, "efd_hann_loglike_local: bad arguments (m: a power of two in "
                                 "[2^21, 2^25], >= nf; rows <= 16, or 1 with emit)");
    // kfix = K[0] - K[(-(m - nf)) mod nf], K[j] = -i pi/nf + (pi/nf) cot(pi j/nf), K[0] = i pi
    // (nf - 1)/nf (fdutils.HannConvolution.kernel_spectrum's lag kernel)
    const double pn = M_PI / (double)nf;
    const int64_t jw = ((-(m - nf)) % nf + nf) % nf;
    double2 kfix = make_double2(0.0, pn * (double)(nf - 1));
    if (jw != 0) {
        kfix.x -= pn / std::tan(pn * (double)jw);
        kfix.y += pn;
    } else {
        kfix = make_double2(0.0, 0.0);
    }
    hipStream_t st = (hipStream_t)stream;
    const HannLocal ll{(const double2*)dl, wl, kself, kfix, scratch, (double2*)emit};
    const int rc = hann_pipeline_m(S, stride, nf, rows, info, m, kfd, Y, &ll, st);
    if (rc != EFD_OK || emit) return rc;
    hipLaunchKernelGGL(k_loglike_final, dim3((unsigned)rows), dim3(256), 0, st, scratch, np, out);
    HIP_TRY(hipGetLastError());
    return EFD_OK;
}
int efd_hann_polarizations(const double* S, const float* Y, const uint64_t* info, int64_t m,
                           int64_t nf, int64_t k0, double* hp, double* hc, void* stream) {
    if (!S || !Y || !info || !hp || !hc || nf < 3 || m < nf || k0 < 0 || k0 > nf)
        return fail(EFD_ERR_ARG, "efd_hann_polarizations: bad arguments");
    const int64_t cnt = nf - k0;
    if (cnt == 0) return EFD_OK;
    const int threads = 256;
    const int64_t blocks = (cnt + threads - 1) / threads;
    hipLaunchKernelGGL(k_hann_polarizations, dim3((unsigned)blocks), dim3(threads), 0,
                       (hipStream_t)stream, (const double2*)S, (const float2*)Y, info, m, nf, k0,
                       (double2*)hp, (double2*)hc);
    HIP_TRY(hipGetLastError());
    return EFD_OK;
}
int efd_hann_loglike(const double* S, int64_t stride, const float* Y, const uint64_t* info,
                     int64_t m, int32_t rows, int64_t nf, int64_t k0, const double* d,
                     const double* w, double* out, double* scratch, void* stream) {
    if (!hann_rows_ok("efd_hann_loglike", S, stride, nf, rows) || !Y || !info || !d || !w ||
        !out || !scratch || m < nf || k0 < 0 || k0 >= nf || rows > HANN_ROWS_MAX)
        return fail(EFD_ERR_ARG, "efd_hann_loglike: bad arguments (rows <= 16)");
    const int64_t nb = nf - k0;
    const int threads = 256;
    // chunks: a multiple of 8 (one per XCD in turn), at most EFD_LOGLIKE_SCRATCH per row
    const int np = (int)std::min<int64_t>(EFD_LOGLIKE_SCRATCH,
                                          ((nb + threads - 1) / threads + 7) / 8 * 8);
    hipStream_t st = (hipStream_t)stream;
    static_assert(EFD_LOGLIKE_SCRATCH % 8 == 0, "chunks: whole rounds of the 8 XCDs");
    // two rows a workgroup when the rows pair up (d and w read once for both: 362 -> 318 us,
    // r05zr; an odd row count takes one row a workgroup)
    const int rpt = (rows % 2 == 0) ? 2 : 1;
    hipLaunchKernelGGL(rpt == 2 ? k_hann_loglike_partial<2> : k_hann_loglike_partial<1>,
                       dim3((unsigned)(np * (rows / rpt))), dim3(threads), 0, st,
                       (const double2*)S, stride, (const float2*)Y, info, m, nf, k0,
                       (const double2*)d, w, (int)rows, np, scratch);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_loglike_final, dim3((unsigned)rows), dim3(256), 0, st, scratch, np, out);
    HIP_TRY(hipGetLastError());
    return EFD_OK;
}

int efd_loglike(const double* h, const double* d, const double* w, int32_t nchan, int64_t nbin,
                double* out, double* scratch, void* stream) {
    if (!d || !w || !out || !scratch || nchan <= 0 || nbin <= 0)
        return fail(EFD_ERR_ARG, "efd_loglike: bad arguments");
    const int64_t total = (int64_t)nchan * nbin;
    const int threads = 256;
    const int np = (int)std::min<int64_t>(EFD_LOGLIKE_SCRATCH, (total + threads - 1) / threads);
    hipStream_t st = (hipStream_t)stream;
    // fixed partition + fixed reduction tree: bitwise reproducible
    hipLaunchKernelGGL(k_loglike_partial, dim3(np), dim3(threads), 0, st, (const double2*)h,
                       (const double2*)d, w, total, scratch);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_loglike_final, dim3(1), dim3(256), 0, st, scratch, np, out);
    HIP_TRY(hipGetLastError());
    return EFD_OK;
}

int efd_inner_product(const double* a, const double* b, const double* w, int32_t nchan,
                      int64_t nbin, double* out, double* scratch, void* stream) {
    if (!a || !b || !out || !scratch || nchan <= 0 || nbin <= 0)
        return fail(EFD_ERR_ARG, "efd_inner_product: bad arguments");
    const int64_t total = (int64_t)nchan * nbin;
    const int threads = 256;
    const int np = (int)std::min<int64_t>(EFD_INNER_SCRATCH / 2, (total + threads - 1) / threads);
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_inner_partial, dim3(np), dim3(threads), 0, st, (const double2*)a,
                       (const double2*)b, w, total, (double2*)scratch);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_inner_final, dim3(1), dim3(256), 0, st, (const double2*)scratch, np,
                       4.0, (double2*)out);
    HIP_TRY(hipGetLastError());
    return EFD_OK;
}

}  // extern "C"
