// A C++ host driving the C-ABI directly (no Python, no torch): one batch of
// random-policy self-play and one batched step, as a C/C++ caller of
// include/othello.h would.  Build and run:
//   hipcc --offload-arch=gfx950 -O2 -Iinclude examples/rollout_host.cpp \
//         -Lsubproc_amd/lib -lsubproc_amd_hip -Wl,-rpath,$PWD/subproc_amd/lib -o rollout_host
//   ./rollout_host 65536
// Prints the histogram summary and the first final board (compare with the oracle).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "othello.h"

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)
#define OTH(x)                                                                         \
    do {                                                                               \
        int s_ = (x);                                                                  \
        if (s_ != OTH_OK) {                                                            \
            std::fprintf(stderr, "oth call failed: %d at line %d\n", s_, __LINE__);   \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? std::atoll(argv[1]) : 65536;
    const uint64_t seed = 0x5EED;
    std::printf("%s\n", oth_version());
    hipStream_t st;
    CK(hipStreamCreate(&st));
    uint64_t* fb;
    int64_t* hist;
    CK(hipMalloc(&fb, n * 16));
    CK(hipMalloc(&hist, OTH_HIST_BINS * sizeof(int64_t)));
    uint64_t* work;  // the rollouts' batch counter: zeroed once, left at 0 by every launch
    CK(hipMalloc(&work, sizeof(uint64_t)));
    CK(hipMemsetAsync(work, 0, sizeof(uint64_t), st));
    CK(hipMemsetAsync(hist, 0, OTH_HIST_BINS * sizeof(int64_t), st));
    OTH(oth_rollout(nullptr, nullptr, seed, 0, OTH_POLICY_RANDOM, 0, fb, nullptr, nullptr, nullptr, hist, work, n,
                    st));

    // one batched step on the opening: every game plays d3 (square 19)
    uint64_t* boards;
    uint8_t *turn, *move;
    int8_t* ret;
    CK(hipMalloc(&boards, n * 16));
    CK(hipMalloc(&turn, n));
    CK(hipMalloc(&move, n));
    CK(hipMalloc(&ret, n));
    OTH(oth_reset(boards, turn, nullptr, n, st));
    CK(hipMemsetAsync(move, 19, n, st));
    OTH(oth_step(boards, turn, move, boards, turn, nullptr, nullptr, ret, nullptr, n, st));

    std::vector<int64_t> h(OTH_HIST_BINS);
    std::vector<uint64_t> b0(2);
    int8_t r0 = 0;
    CK(hipMemcpyAsync(h.data(), hist, OTH_HIST_BINS * sizeof(int64_t), hipMemcpyDeviceToHost, st));
    CK(hipMemcpyAsync(b0.data(), fb, 16, hipMemcpyDeviceToHost, st));
    CK(hipMemcpyAsync(&r0, ret, 1, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    int64_t games = 0;
    for (int d = 0; d <= 128; d++) games += h[d];
    std::printf("games %lld black %lld white %lld draws %lld env-steps %lld\n", (long long)games, (long long)h[129],
                (long long)h[130], (long long)h[131], (long long)h[132]);
    std::printf("game0 final black %016llx white %016llx\n", (unsigned long long)b0[0], (unsigned long long)b0[1]);
    std::printf("step d3 ret %d\n", (int)r0);
    CK(hipFree(fb));
    CK(hipFree(hist));
    CK(hipFree(boards));
    CK(hipFree(turn));
    CK(hipFree(move));
    CK(hipFree(ret));
    CK(hipStreamDestroy(st));
    return 0;
}
