// Diagnostic build of the rollout kernel (per-wave timestamps) — NOT product code.
// hipcc --offload-arch=gfx950 -O3 -DOTH_DIAG -x hip tools/diag/rollout_diag.cpp -o rollout_diag
#include "../../subproc_amd/csrc/othello.hip"
#include <cstdio>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
    long long n = argc > 1 ? atoll(argv[1]) : (1 << 20);
    int reps = argc > 2 ? atoi(argv[2]) : 5;
    uint64_t *fb; int8_t* df; uint8_t* pl; int64_t* hist; unsigned long long* diag;
    CK(hipMalloc(&fb, n * 16)); CK(hipMalloc(&df, n)); CK(hipMalloc(&pl, n)); CK(hipMalloc(&hist, 133 * 8));
    const long long maxw = 1 << 20;
    CK(hipMalloc(&diag, maxw * 32));
    uint64_t* work; CK(hipMalloc(&work, 8)); CK(hipMemset(work, 0, 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_diag), &diag, sizeof(diag)));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int r = 0; r < reps; r++) {
        CK(hipMemset(hist, 0, 133 * 8));
        CK(hipMemset(diag, 0, maxw * 32));
        CK(hipEventRecord(e0, 0));
        int st = oth_rollout(nullptr, nullptr, 0x5EED, (uint64_t)r * n, 0, 10, fb, df, pl, nullptr, hist, work, n, nullptr);
        CK(hipEventRecord(e1, 0));
        CK(hipDeviceSynchronize());
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<long long> h(133); CK(hipMemcpy(h.data(), hist, 133 * 8, hipMemcpyDeviceToHost));
        std::vector<unsigned long long> d(maxw * 4); CK(hipMemcpy(d.data(), diag, maxw * 32, hipMemcpyDeviceToHost));
        long long waves = 0; unsigned long long t0 = ~0ull, t1 = 0; double life = 0; double it = 0; unsigned long long maxit = 0, minit = ~0ull;
        std::vector<double> lifes;
        for (long long w = 0; w < maxw; w++) { if (!d[4*w+1]) continue; waves++; t0 = std::min(t0, d[4*w]); t1 = std::max(t1, d[4*w+1]); }
        std::vector<double> starts, ends;
        double issued = 0, useful = 0;
        for (long long w = 0; w < maxw; w++) { if (!d[4*w+1]) continue; double l = (d[4*w+1]-d[4*w]) / 100.0; life += l; lifes.push_back(l); const unsigned long long wi = d[4*w+3] >> 32, li = d[4*w+3] & 0xffffffffull; issued += 64.0 * wi; useful += li; it += wi; maxit = std::max(maxit, wi); minit = std::min(minit, wi); starts.push_back((d[4*w]-t0)/100.0); ends.push_back((d[4*w+1]-t0)/100.0);}
        printf("lane-plies: issued %.0f (64 x the waves' ply steps), useful %.0f (the lanes' own), idle %.2f%%\n", issued, useful, 100.0 * (1.0 - useful / issued));
        std::sort(lifes.begin(), lifes.end()); std::sort(starts.begin(), starts.end()); std::sort(ends.begin(), ends.end());
        printf("n=%lld status=%d ms=%.3f env-steps=%lld -> %.3e steps/s | waves=%lld span_us=%.1f life_us avg=%.1f p5=%.1f p50=%.1f p95=%.1f max=%.1f | start_us p50=%.1f p95=%.1f max=%.1f | end_us p5=%.1f p50=%.1f | wave ply steps avg=%.1f min=%llu max=%llu\n",
               n, st, ms, h[132], h[132] / (ms * 1e-3), waves, (t1 - t0) / 100.0, life / waves, lifes[waves*5/100], lifes[waves/2], lifes[waves*95/100], lifes.back(), starts[waves/2], starts[waves*95/100], starts.back(), ends[waves*5/100], ends[waves/2], it / waves, minit, maxit);
    }
    return 0;
}
