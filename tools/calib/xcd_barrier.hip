// xcd_barrier.hip — the cost of a cross-CU barrier among N workgroups of ONE XCD
// (the number DESIGN §8 needs before spreading a cell over several CUs).
//
// Workgroups are dealt round-robin over the 8 XCDs (blockIdx.x % 8), so a launch of
// 8·N workgroups of which only blockIdx.x % 8 == 0 stay puts N of them on one XCD;
// the rest exit at once. The N workgroups then run K barriers: thread 0 adds 1 to
// an arrival counter (agent-scope atomic, resolved in that XCD's L2) and spins with
// relaxed loads until the counter reaches N·k, then a workgroup barrier. Every spin
// is bounded by a wall-clock deadline (s_memrealtime, 100 MHz), so a grid that could
// not be co-resident ends instead of hanging.
//
//   hipcc --offload-arch=gfx950 -O3 tools/calib/xcd_barrier.hip -o /tmp/xcd_barrier && /tmp/xcd_barrier
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

__global__ __launch_bounds__(1024) void k_barriers(unsigned* ctr, int n, int k, int stride,
                                                   unsigned long long* out, int* timeout) {
    if (blockIdx.x % stride) return;   // keep one XCD's share (or every block when stride = 1)
    const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + 200000000ULL;   // 2 s
    __shared__ int bad;
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 1; i <= k; ++i) {
        if (threadIdx.x == 0) {
            __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned target = (unsigned)n * (unsigned)i;
            while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() > deadline) {
                    bad = 1;
                    break;
                }
            }
        }
        __syncthreads();
        if (bad) break;
    }
    if (threadIdx.x == 0) {
        if (bad) atomicOr(timeout, 1);
        out[blockIdx.x / stride] = __builtin_amdgcn_s_memrealtime() - t0;
    }
}

int main() {
    unsigned* ctr;
    unsigned long long* out;
    int* timeout;
    CK(hipMalloc(&ctr, sizeof(unsigned)));
    CK(hipMalloc(&out, 256 * sizeof(unsigned long long)));
    CK(hipMalloc(&timeout, sizeof(int)));
    const int K = 2000;
    std::printf("{\"barriers_per_run\": %d, \"rows\": [\n", K);
    bool first = true;
    for (int stride : {8, 1}) {          // 8: N workgroups on one XCD; 1: N workgroups over all XCDs
        for (int n : {2, 4, 8, 16, 32}) {
            if (stride == 1 && n < 8) continue;
            for (int rep = 0; rep < 3; ++rep) {
                CK(hipMemset(ctr, 0, sizeof(unsigned)));
                CK(hipMemset(timeout, 0, sizeof(int)));
                CK(hipMemset(out, 0, 256 * sizeof(unsigned long long)));
                hipLaunchKernelGGL(k_barriers, dim3(n * stride), dim3(1024), 0, 0, ctr, n, K, stride, out, timeout);
                CK(hipGetLastError());
                CK(hipDeviceSynchronize());
                int to = 0;
                std::vector<unsigned long long> h(n);
                CK(hipMemcpy(&to, timeout, sizeof(int), hipMemcpyDeviceToHost));
                CK(hipMemcpy(h.data(), out, n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
                unsigned long long mx = 0;
                for (auto t : h) mx = t > mx ? t : mx;
                std::printf("%s {\"workgroups\": %d, \"placement\": \"%s\", \"rep\": %d, \"us_per_barrier\": %.3f, \"timeout\": %d}",
                            first ? "" : ",\n", n, stride == 8 ? "one XCD" : "all XCDs", rep, mx / 100.0 / K, to);
                first = false;
            }
        }
    }
    std::printf("\n]}\n");
    return 0;
}
