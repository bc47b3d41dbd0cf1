#include <hip/hip_runtime.h>
#include <cstdio>
// one wave: N steps of the TD chain (mul, min, add), 1 or 2 independent chains per lane
template <int ILP>
__global__ void chain(const double* y, double* out, long long* cyc, int n) {
    double w[ILP], mn[ILP];
    for (int c = 0; c < ILP; c++) { w[c] = y[threadIdx.x + c]; mn[c] = 1.0; }
    const double oma = 0.97;
    double yy = y[threadIdx.x + 7];
    long long t0 = clock64();
    for (int k = 0; k < n; k++) {
#pragma unroll
        for (int c = 0; c < ILP; c++) {
            double t;
            asm volatile("v_mul_f64 %[t], %[w], %[oma]\n\t"
                "v_min_f64 %[mn], %[mn], |%[w]|\n\t"
                "v_add_f64 %[w], %[t], %[y]"
                : [w] "+v"(w[c]), [mn] "+v"(mn[c]), [t] "=&v"(t)
                : [oma] "v"(oma), [y] "v"(yy));
        }
    }
    long long t1 = clock64();
    double s = 0; for (int c = 0; c < ILP; c++) s += w[c] + mn[c];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
int main() {
    double *y, *o; long long* c;
    hipMalloc(&y, 1024 * 8); hipMalloc(&o, 1024 * 8); hipMalloc(&c, 8);
    hipMemset(y, 0, 1024 * 8);
    const int n = 100000;
    long long h;
    chain<1><<<1, 64>>>(y, o, c, n); hipDeviceSynchronize();
    chain<1><<<1, 64>>>(y, o, c, n); hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("ILP1: %.1f cycles per step (clock64)\n", (double)h / n);
    chain<2><<<1, 64>>>(y, o, c, n); hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("ILP2: %.1f cycles per step-pair\n", (double)h / n);
    chain<4><<<1, 64>>>(y, o, c, n); hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("ILP4: %.1f cycles per 4 steps\n", (double)h / n);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0); chain<1><<<1, 64>>>(y, o, c, n); hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("ILP1 wall: %.1f ns per step\n", ms * 1e6 / n);
    return 0;
}
