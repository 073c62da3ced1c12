// Checks whether v_fma_f64 honours the div:2 output modifier, without and with FP64 denormals
// flushed by s_setreg (MODE.FP_DENORM[3:2]). MI355X: it does not in either mode (eh/e = 1; the
// kernels run in IEEE mode, where the output modifiers are not applied):
// hipcc --offload-arch=gfx950 -O3 tools/rsq_omod_check.hip -o /tmp/rsq_omod
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
template <int FTZ>
__global__ void k(const double* x, double* out, int n) {
    if (FTZ >= 1) __builtin_amdgcn_s_setreg(1 | (6 << 6) | (1 << 11), 0);
    if (FTZ >= 2) __builtin_amdgcn_s_setreg(1 | (9 << 6), 0);   // MODE.IEEE = 0
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double xv = x[i];
    const double y = __builtin_amdgcn_rsq(xv);
    const double e = fma(-xv * y, y, 1.0);
    out[4 * i] = fma(y * e, 0.5, y);
    double eh;
    asm volatile("v_fma_f64 %0, -%1, %2, 1.0 div:2" : "=v"(eh) : "v"(xv * y), "v"(y));
    out[4 * i + 1] = fma(y, eh, y);
    out[4 * i + 2] = y;
    out[4 * i + 3] = eh / e;
}
int main() {
    const int n = 1 << 16;
    double *x, *o;
    hipMallocManaged(&x, n * sizeof(double));
    hipMallocManaged(&o, 4 * n * sizeof(double));
    for (int i = 0; i < n; ++i) x[i] = std::ldexp(1.0 + (double)i / n, (i % 97) - 48);
  for (int ftz = 0; ftz < 3; ++ftz) {
    if (ftz == 2) hipLaunchKernelGGL(k<2>, dim3(n / 256), dim3(256), 0, 0, x, o, n);
    else if (ftz == 1) hipLaunchKernelGGL(k<1>, dim3(n / 256), dim3(256), 0, 0, x, o, n);
    else hipLaunchKernelGGL(k<0>, dim3(n / 256), dim3(256), 0, 0, x, o, n);
    hipDeviceSynchronize();
    double m0 = 0, m1 = 0, my = 0, rmin = 1e9, rmax = -1e9;
    for (int i = 0; i < n; ++i) {
        long double ex = 1.0L / sqrtl((long double)x[i]);
        m0 = fmax(m0, (double)fabsl((o[4 * i] - ex) / ex));
        m1 = fmax(m1, (double)fabsl((o[4 * i + 1] - ex) / ex));
        my = fmax(my, (double)fabsl((o[4 * i + 2] - ex) / ex));
        if (std::isfinite(o[4 * i + 3])) { rmin = fmin(rmin, o[4 * i + 3]); rmax = fmax(rmax, o[4 * i + 3]); }
    }
    printf("ftz %d rel err: newton %.3e  omod %.3e  rsq %.3e  eh/e in [%.6f, %.6f]\n", ftz, m0, m1,
           my, rmin, rmax);
  }
    return 0;
}
