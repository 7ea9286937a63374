// Micro-benchmark (diagnostic, not product): single-wave issue cost of fp64 /
// fp32 FMA chains on gfx950, and the accuracy of the raw v_rcp_f64.
// Build: hipcc --offload-arch=gfx950 -O3 -o fp64_issue fp64_issue.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

template <typename T, int CH>
__global__ void chains(T* out, long long* cyc, int iters) {
    T a[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = (T)(threadIdx.x + c) * (T)1e-3;
    const T m = (T)0.999999, k = (T)1e-7;
    long long t0 = clock64();
    for (int i = 0; i < iters; i += 32) {
#pragma unroll
        for (int u = 0; u < 32; ++u)
#pragma unroll
            for (int c = 0; c < CH; ++c) a[c] = fma(a[c], m, k);
    }
    long long t1 = clock64();
    T s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += a[c];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void rcp_raw(const double* x, double* r, int n) {
    int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) r[i] = __builtin_amdgcn_rcp(x[i]);
}

template <typename T, int CH>
double run(int iters) {
    T* o;
    long long* c;
    hipMalloc(&o, 64 * sizeof(T));
    hipMalloc(&c, sizeof(long long));
    hipLaunchKernelGGL((chains<T, CH>), dim3(1), dim3(64), 0, 0, o, c, iters);
    hipLaunchKernelGGL((chains<T, CH>), dim3(1), dim3(64), 0, 0, o, c, iters);
    long long h;
    hipMemcpy(&h, c, sizeof(h), hipMemcpyDeviceToHost);
    hipFree(o);
    hipFree(c);
    return (double)h / ((double)iters * CH);
}

int main() {
    const int it = 4096;
    printf("cycles per FMA (clock64), one wave64 on one SIMD:\n");
    printf("  f64 chains=1 %.2f  2 %.2f  4 %.2f  8 %.2f\n", run<double, 1>(it), run<double, 2>(it), run<double, 4>(it),
           run<double, 8>(it));
    printf("  f32 chains=1 %.2f  2 %.2f  4 %.2f  8 %.2f\n", run<float, 1>(it), run<float, 2>(it), run<float, 4>(it),
           run<float, 8>(it));
    const int n = 1 << 22;
    double *hx = (double*)malloc(n * 8), *hr = (double*)malloc(n * 8);
    srand(1);
    for (int i = 0; i < n; ++i) {
        double m = 1.0 + (double)rand() / RAND_MAX;
        int e = rand() % 200 - 100;
        hx[i] = ldexp(m, e) * ((rand() & 1) ? 1 : -1);
    }
    double *dx, *dr;
    hipMalloc(&dx, n * 8);
    hipMalloc(&dr, n * 8);
    hipMemcpy(dx, hx, n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(rcp_raw, dim3(n / 256), dim3(256), 0, 0, dx, dr, n);
    hipMemcpy(hr, dr, n * 8, hipMemcpyDeviceToHost);
    double maxulp = 0;
    long exact = 0;
    for (int i = 0; i < n; ++i) {
        double ref = 1.0 / hx[i];
        double ulp = fabs(nextafter(ref, INFINITY) - ref);
        double e = fabs(hr[i] - ref) / ulp;
        maxulp = e > maxulp ? e : maxulp;
        exact += (hr[i] == ref);
    }
    for (int nn : {1, 2}) {
        double me = 0;
        for (int i = 0; i < n; ++i) {
            double r = hr[i], x = hx[i];
            for (int k = 0; k < nn; ++k) {
                double e = fma(-x, r, 1.0);
                r = fma(r, e, r);
            }
            double ref = 1.0 / x;
            double ulp = fabs(nextafter(ref, INFINITY) - ref);
            me = fmax(me, fabs(r - ref) / ulp);
        }
        printf("v_rcp_f64 + %d Newton: max error %.3g ulp\n", nn, me);
    }
    printf("v_rcp_f64 raw: max error %.3g ulp, correctly rounded %.4f\n", maxulp, (double)exact / n);
    return 0;
}
