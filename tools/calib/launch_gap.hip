// launch_gap.hip — the GPU's idle time between a host round trip's kernels: the
// engine's cycle loop waits for each cycle's control snapshot, decides, and
// enqueues the next cycle, and the config-3 kernel trace shows ~23 µs between
// the cycle's last kernel and the next cycle's first.
//
//   mode 0  kernel A; event; host waits on the event; host launches kernel B
//   mode 1  the same with a hold kernel behind the event: the GPU spins on a flag in
//           pinned host memory (bounded by a 2 ms deadline) while the host waits on
//           the event, launches B (queued behind the hold) and then sets the flag
//
// A and B stamp s_memrealtime (100 MHz) at entry and exit; the gap is B's entry
// minus A's exit, the median over 400 round trips.
//
//   hipcc --offload-arch=gfx950 -O3 tools/calib/launch_gap.hip -o /tmp/launch_gap && /tmp/launch_gap
#include <hip/hip_runtime.h>

#include <algorithm>
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

__global__ void k_stamp(unsigned long long* t, int i) {
    if (blockIdx.x == 0 && threadIdx.x == 0) t[2 * i] = __builtin_amdgcn_s_memrealtime();
    // a little work so the kernel is not empty
    __shared__ int x;
    if (threadIdx.x == 0) x = i;
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x == 0) t[2 * i + 1] = __builtin_amdgcn_s_memrealtime() + (x & 0);
}

__global__ void k_hold(const volatile unsigned* flag, unsigned want, int* timeouts) {
    if (threadIdx.x != 0) return;
    const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + 200000ULL;   // 2 ms
    while (__hip_atomic_load(const_cast<const unsigned*>(flag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != want) {
        __builtin_amdgcn_s_sleep(2);
        if (__builtin_amdgcn_s_memrealtime() > deadline) {
            atomicAdd(timeouts, 1);
            return;
        }
    }
}

int main() {
    const int N = 400;
    unsigned long long* t;
    int* tmo;
    unsigned* flag;
    CK(hipMalloc(&t, 2 * (N + 1) * sizeof(unsigned long long)));
    CK(hipMalloc(&tmo, sizeof(int)));
    CK(hipHostMalloc(&flag, sizeof(unsigned), hipHostMallocCoherent | hipHostMallocMapped));
    unsigned* dflag = nullptr;
    CK(hipHostGetDevicePointer((void**)&dflag, flag, 0));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t ev;
    CK(hipEventCreate(&ev));
    std::printf("{\"rows\": [");
    for (int mode = 0; mode < 2; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipMemset(tmo, 0, sizeof(int)));
            *flag = 0;
            hipLaunchKernelGGL(k_stamp, dim3(256), dim3(256), 0, st, t, 0);
            for (int i = 1; i <= N; ++i) {
                CK(hipEventRecord(ev, st));
                if (mode == 1) hipLaunchKernelGGL(k_hold, dim3(1), dim3(64), 0, st, dflag, (unsigned)i, tmo);
                CK(hipEventSynchronize(ev));
                hipLaunchKernelGGL(k_stamp, dim3(256), dim3(256), 0, st, t, i);
                if (mode == 1) __atomic_store_n(flag, (unsigned)i, __ATOMIC_RELEASE);
            }
            CK(hipStreamSynchronize(st));
            std::vector<unsigned long long> h(2 * (N + 1));
            CK(hipMemcpy(h.data(), t, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
            int to = 0;
            CK(hipMemcpy(&to, tmo, sizeof(int), hipMemcpyDeviceToHost));
            std::vector<double> gap;
            for (int i = 1; i <= N; ++i) gap.push_back((double)(h[2 * i] - h[2 * i - 1]) / 100.0);
            std::sort(gap.begin(), gap.end());
            std::printf("%s\n {\"mode\": %d, \"rep\": %d, \"gap_us_p10\": %.2f, \"gap_us_p50\": %.2f, \"gap_us_p90\": %.2f, "
                        "\"hold_timeouts\": %d}",
                        (mode || rep) ? "," : "", mode, rep, gap[N / 10], gap[N / 2], gap[9 * N / 10], to);
        }
    }
    std::printf("\n]}\n");
    return 0;
}
