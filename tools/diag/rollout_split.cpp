// Diagnostic experiment (NOT product code): does splitting each 64-game batch
// into two half-game work units, so that any wave may continue a half-played
// batch, shorten the per-launch tail of the random rollout?
//
// Units 0..B-1 play the first kSplit plies of batch u and save the 64 game
// states (32 B each); units B..2B-1 resume batch u-B from those states.  All
// first halves are dequeued before any second half and every wave is
// resident, so a second half waits only for a first half that is running; the
// wait is capped (a wave that gives up records an error instead of hanging).
// The result must equal oth_rollout's histogram bit for bit (same RNG
// streams).
//   hipcc --offload-arch=gfx950 -O3 -x hip tools/diag/rollout_split.cpp -o tools/diag/rollout_split
//   ./tools/diag/rollout_split 1048576 5 [split_ply]
#include "../../subproc_amd/csrc/othello.hip"

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

namespace {
struct GState {
    u64 P, O;
    u32 rng_state, rng_inc;
    u32 packed;  // side | ply << 8 | passed << 16 | active << 17
    u32 pad;
};

__device__ __forceinline__ u64 ld_agent(const u64* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(u64* p, u64 v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kBlock, 4) void split_kernel(u64 seed_state, u64 game_id0, int64_t n_, int split,
                                                          unsigned long long* work, unsigned* ready, GState* scratch,
                                                          long long* hist, unsigned* errors) {
    __shared__ unsigned long long hist_s[OTH_HIST_BINS];
    __shared__ uint8_t kth_tab[256 * 8];
    __shared__ u64 rays[kTabRows * 64];
    for (int k = threadIdx.x; k < OTH_HIST_BINS; k += kBlock) hist_s[k] = 0;
    kth_table_init(kth_tab);
    ray_table_init(rays);
    __syncthreads();
    const int lane = lane_id();
    const u64 n = (u64)n_;
    const u64 B = (n + 63) / 64;
    u64 plies_sum = 0;
    for (;;) {
        u64 u = 0;
        if (lane == 0) u = atomicAdd(work, 1ull);
        u = __shfl(u, 0);
        if (u >= 2 * B) break;
        const bool second = u >= B;
        const u64 b = second ? u - B : u;
        const u64 g = b * 64 + lane;
        bool active = g < n;
        u64 P = OPEN_BLACK, O = OPEN_WHITE;
        u32 side = OTH_BLACK, ply = 0;
        bool passed = false;
        GameRng rng;
        if (!second) {
            if (active) rng.init(game_key(seed_state, game_id0 + g));
        } else {
            if (lane == 0) {
                unsigned spins = 0;
                while (__hip_atomic_load(&ready[b], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0) {
                    __builtin_amdgcn_s_sleep(2);
                    if (++spins > (1u << 26)) {
                        atomicAdd(errors, 1u);
                        break;
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            __atomic_thread_fence(__ATOMIC_ACQUIRE);
            if (active) {
                u64* s = reinterpret_cast<u64*>(scratch + g);
                P = ld_agent(s);
                O = ld_agent(s + 1);
                const u64 r = ld_agent(s + 2), k = ld_agent(s + 3);
                rng.state = (u32)r;
                rng.inc = (u32)(r >> 32);
                side = (u32)k & 0xFF;
                ply = ((u32)k >> 8) & 0xFF;
                passed = (k >> 16) & 1;
                active = (k >> 17) & 1;
            }
        }
        while (__ballot(active && (second || (int)ply < split))) {
            if (!active || (!second && (int)ply >= split)) continue;
            Position pos;
            analyse(P, O, pos);
            const u64 legal = pos.legal;
            if (legal == 0) {
                if (passed) {
                    const u64 bl = side == OTH_BLACK ? P : O, wh = side == OTH_BLACK ? O : P;
                    const int d = __popcll(bl) - __popcll(wh);
                    atomicAdd(&hist_s[d + 64], 1ull);
                    atomicAdd(&hist_s[d > 0 ? 129 : (d < 0 ? 130 : 131)], 1ull);
                    plies_sum += ply;
                    active = false;
                } else {
                    passed = true;
                    const u64 t = P;
                    P = O;
                    O = t;
                    side ^= 3u;
                }
                continue;
            }
            if (passed) {
                ply++;
                passed = false;
            }
            const u32 sq = pick_legal(legal, rng, kth_tab);
            const u64 mv = square_bit(sq, rays);
            const u64 f = flips_rays(sq, mv, run_sets(pos), rays);
            const u64 np = andn(O, f);
            O = P | f | mv;
            P = np;
            side ^= 3u;
            ply++;
        }
        if (!second) {
            if (g < n) {
                u64* s = reinterpret_cast<u64*>(scratch + g);
                st_agent(s, P);
                st_agent(s + 1, O);
                st_agent(s + 2, ((u64)rng.inc << 32) | rng.state);
                st_agent(s + 3, (u64)side | ((u64)ply << 8) | ((u64)passed << 16) | ((u64)active << 17));
            }
            __atomic_thread_fence(__ATOMIC_RELEASE);
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) __hip_atomic_store(&ready[b], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    for (int off = 32; off >= 1; off >>= 1) plies_sum += __shfl_xor(plies_sum, off);
    if (lane == 0) atomicAdd(&hist_s[132], (unsigned long long)plies_sum);
    __syncthreads();
    for (int k = threadIdx.x; k < OTH_HIST_BINS; k += kBlock)
        if (hist_s[k]) atomicAdd((unsigned long long*)&hist[k], hist_s[k]);
}
}  // namespace

int main(int argc, char** argv) {
    const long long n = argc > 1 ? atoll(argv[1]) : (1 << 20);
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const int split = argc > 3 ? atoi(argv[3]) : 30;
    const long long B = (n + 63) / 64;
    int64_t *hist, *hist_ref;
    unsigned long long* work;
    unsigned *ready, *errors;
    GState* scratch;
    CK(hipMalloc(&hist, 133 * 8));
    CK(hipMalloc(&hist_ref, 133 * 8));
    CK(hipMalloc(&work, 8));
    CK(hipMalloc(&ready, B * 4));
    CK(hipMalloc(&errors, 4));
    CK(hipMalloc(&scratch, n * sizeof(GState)));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const unsigned grid = (unsigned)std::min<long long>((n + 255) / 256, (long long)cus * 5);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < reps; r++) {
        const unsigned long long gid0 = (unsigned long long)r * n;
        CK(hipMemset(hist_ref, 0, 133 * 8));
        CK(hipEventRecord(e0, 0));
        static uint64_t* ref_work = nullptr;
        if (!ref_work) { CK(hipMalloc(&ref_work, 8)); CK(hipMemset(ref_work, 0, 8)); }
        int st = oth_rollout(nullptr, nullptr, 0x5EED, gid0, 0, 0, nullptr, nullptr, nullptr, nullptr, hist_ref, ref_work,
                             n, nullptr);
        CK(hipEventRecord(e1, 0));
        CK(hipDeviceSynchronize());
        float ms_ref;
        CK(hipEventElapsedTime(&ms_ref, e0, e1));
        CK(hipMemset(hist, 0, 133 * 8));
        CK(hipMemset(work, 0, 8));
        CK(hipMemset(ready, 0, B * 4));
        CK(hipMemset(errors, 0, 4));
        CK(hipEventRecord(e0, 0));
        split_kernel<<<grid, kBlock>>>(mix64(0x5EED + GOLDEN64), gid0, n, split, work, ready, scratch, (long long*)hist,
                                       errors);
        CK(hipEventRecord(e1, 0));
        CK(hipDeviceSynchronize());
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<long long> h(133), hr(133);
        unsigned err = 0;
        CK(hipMemcpy(h.data(), hist, 133 * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hr.data(), hist_ref, 133 * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&err, errors, 4, hipMemcpyDeviceToHost));
        printf("n=%lld split=%d st=%d ref %.3f ms  split %.3f ms  (%.3fx)  hist %s  wait-errors %u\n", n, split, st,
               ms_ref, ms, ms_ref / ms, h == hr ? "identical" : "DIFFERENT", err);
    }
    return 0;
}
