// grid_sync.hip — what a kernel boundary costs against a grid barrier inside one
// persistent launch, at the engine's grid sizes (a config-3 solve is
// ~3,500 dependent launches of ~10 µs).
//
//   A  back-to-back launches of a kernel of G workgroups × 256 threads whose waves
//      read one window of frontier flags (121k flag bytes in all, every flag 0)
//      and exit: the per-launch floor of a sparse round or sweep;
//   B  one cooperative launch of G workgroups running K grid-stride passes over the
//      same flags, a grid barrier after each (agent-scope release before the
//      arrival, acquire after), in three barrier shapes:
//        0 flat: every workgroup polls the arrival counter;
//        1 flat + release word: the last arrival bumps a generation word, the
//          others poll it;
//        2 per-XCD then global: arrivals count per XCD (blockIdx % 8), the last of
//          each XCD arrives at the global counter, whose last arrival bumps the
//          generation word.
// Every spin has a wall-clock deadline (s_memrealtime, 100 MHz), so a grid that
// could not be co-resident ends instead of hanging.
//
//   hipcc --offload-arch=gfx950 -O3 tools/calib/grid_sync.hip -o /tmp/grid_sync && /tmp/grid_sync
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            return 1;                                                              \
        }                                                                          \
    } while (0)

constexpr int NFLAG = 121252;

__device__ __forceinline__ int scan_flags(const unsigned char* flags, int vb, int nvb, unsigned char* out) {
    // one 64-byte window per wave, grid-stride over the windows
    const int lane = threadIdx.x & 63;
    const int nw = (NFLAG + 63) / 64;
    int any = 0;
    for (int w = vb * 4 + (threadIdx.x >> 6); w < nw; w += nvb * 4) {
        const int i = w * 64 + lane;
        const int f = i < NFLAG ? flags[i] : 0;
        if (__ballot(f != 0)) any = 1;
    }
    if (any && threadIdx.x == 0) out[vb] = 1;
    return any;
}

__global__ __launch_bounds__(256) void k_launch(const unsigned char* flags, unsigned char* out) {
    scan_flags(flags, blockIdx.x, gridDim.x, out);
}

__device__ __forceinline__ bool spin_until(const unsigned* w, unsigned target, unsigned long long deadline) {
    while (__hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() > deadline) return false;
    }
    return true;
}
// relaxed polling (no cache invalidation per poll), one acquire fence once it passes
__device__ __forceinline__ bool spin_relaxed(const unsigned* w, unsigned target, unsigned long long deadline) {
    while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() > deadline) return false;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    return true;
}

template <int SHAPE>
__global__ __launch_bounds__(256) void k_persist(const unsigned char* flags, unsigned char* out, unsigned* sync,
                                                 int k, unsigned long long* tout, int* timeout) {
    const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + 300000000ULL;   // 3 s
    __shared__ int bad;
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    unsigned* ctr = sync;            // flat counter
    unsigned* gen = sync + 16;       // generation word
    unsigned* xc = sync + 32;        // per-XCD counters (stride 16 words: separate lines)
    const int G = gridDim.x;
    const int x = blockIdx.x & 7;
    const int per_x = G / 8 + ((G & 7) > x ? 1 : 0);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 1; i <= k; ++i) {
        scan_flags(flags, blockIdx.x, G, out);
        __syncthreads();
        if (threadIdx.x == 0) {
            bool ok = true;
            if (SHAPE == 0) {
                __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                ok = spin_until(ctr, (unsigned)G * (unsigned)i, deadline);
            } else if (SHAPE == 1) {
                const unsigned old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
                if (old == (unsigned)G * (unsigned)i - 1)
                    __hip_atomic_store(gen, (unsigned)i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                else
                    ok = spin_until(gen, (unsigned)i, deadline);
            } else if (SHAPE == 3) {   // flat, relaxed polling
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = spin_relaxed(ctr, (unsigned)G * (unsigned)i, deadline);
            } else if (SHAPE == 4) {   // flat + generation word, relaxed polling
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                const unsigned old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (old == (unsigned)G * (unsigned)i - 1)
                    __hip_atomic_store(gen, (unsigned)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else
                    ok = spin_relaxed(gen, (unsigned)i, deadline);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            } else if (SHAPE == 5) {   // no fences at all (the floor of the arrival / poll traffic)
                const unsigned old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (old == (unsigned)G * (unsigned)i - 1)
                    __hip_atomic_store(gen, (unsigned)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else
                    while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)i) {
                        __builtin_amdgcn_s_sleep(1);
                        if (__builtin_amdgcn_s_memrealtime() > deadline) { ok = false; break; }
                    }
            } else {
                const unsigned old = __hip_atomic_fetch_add(xc + 16 * x, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
                if (old == (unsigned)per_x * (unsigned)i - 1) {
                    const unsigned o2 = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
                    if (o2 == 8u * (unsigned)i - 1)
                        __hip_atomic_store(gen, (unsigned)i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                    else
                        ok = spin_until(gen, (unsigned)i, deadline);
                } else {
                    ok = spin_until(gen, (unsigned)i, deadline);
                }
            }
            if (!ok) bad = 1;
        }
        __syncthreads();
        if (bad) break;
    }
    if (threadIdx.x == 0) {
        if (bad) atomicOr(timeout, 1);
        tout[blockIdx.x] = __builtin_amdgcn_s_memrealtime() - t0;
    }
}

int main() {
    unsigned char *flags, *out;
    unsigned* sync;
    unsigned long long* tout;
    int* timeout;
    CK(hipMalloc(&flags, NFLAG));
    CK(hipMalloc(&out, 1 << 16));
    CK(hipMalloc(&sync, 4096));
    CK(hipMalloc(&tout, 8192 * sizeof(unsigned long long)));
    CK(hipMalloc(&timeout, sizeof(int)));
    CK(hipMemset(flags, 0, NFLAG));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::printf("{\"rows\": [\n");
    bool first = true;
    const int L = 2000;
    for (int G : {256, 2304}) {
        for (int rep = 0; rep < 1; ++rep) {
            for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(k_launch, dim3(G), dim3(256), 0, 0, flags, out);
            CK(hipEventRecord(a, 0));
            for (int i = 0; i < L; ++i) hipLaunchKernelGGL(k_launch, dim3(G), dim3(256), 0, 0, flags, out);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            std::printf("%s {\"mode\": \"launches\", \"workgroups\": %d, \"rep\": %d, \"us_per_step\": %.3f}",
                        first ? "" : ",\n", G, rep, ms * 1000.0 / L);
            first = false;
        }
    }
    int dev = 0, ncu = 0, per_cu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_persist<2>, 256, 0));
    const int K = 2000;
    for (int shape = 3; shape < 6; ++shape) {
        for (int G : {64, 128, 256, 512}) {
            if (G > ncu * per_cu) continue;
            for (int rep = 0; rep < 2; ++rep) {
                CK(hipMemset(sync, 0, 4096));
                CK(hipMemset(timeout, 0, sizeof(int)));
                int k = K;
                void* args[] = {&flags, &out, &sync, &k, &tout, &timeout};
                const void* fn = shape == 3 ? (const void*)k_persist<3>
                                 : shape == 4 ? (const void*)k_persist<4> : (const void*)k_persist<5>;
                CK(hipEventRecord(a, 0));
                CK(hipLaunchCooperativeKernel(fn, dim3(G), dim3(256), args, 0, 0));
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                int to = 0;
                CK(hipMemcpy(&to, timeout, sizeof(int), hipMemcpyDeviceToHost));
                std::vector<unsigned long long> h(G);
                CK(hipMemcpy(h.data(), tout, G * sizeof(unsigned long long), hipMemcpyDeviceToHost));
                unsigned long long mx = 0;
                for (auto t : h) mx = t > mx ? t : mx;
                std::printf(",\n {\"mode\": \"barrier\", \"shape\": %d, \"workgroups\": %d, \"rep\": %d, "
                            "\"us_per_step\": %.3f, \"event_us_per_step\": %.3f, \"timeout\": %d}",
                            shape, G, rep, mx / 100.0 / K, ms * 1000.0 / K, to);
            }
        }
    }
    std::printf("\n], \"cus\": %d, \"blocks_per_cu\": %d}\n", ncu, per_cu);
    return 0;
}
