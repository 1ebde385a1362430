// FETCH_SIZE / WRITE_SIZE calibration for the solver's access widths on gfx950.
// Known byte counts: coalesced 4-B and 8-B streams, random 8-B gathers, 8-B
// streaming stores and no-return 8-B atomics, over a 1 GiB table (past the
// 256 MiB Infinity Cache, so every line comes from HBM once). Run under
//   rocprofv3 --pmc FETCH_SIZE -- ./calib_fetch   (and WRITE_SIZE, TCC_EA0_ATOMIC…)
// and divide the counter by the printed byte count of each kernel.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

__global__ void k_stream8(const long long* __restrict__ a, long long n, long long* __restrict__ out) {
    long long s = 0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        s += a[i];
    if (s == 0x7fffffffffffLL) out[0] = s;
}
__global__ void k_stream4(const int* __restrict__ a, long long n, long long* __restrict__ out) {
    long long s = 0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        s += a[i];
    if (s == 0x7fffffffffffLL) out[0] = s;
}
__global__ void k_gather8(const long long* __restrict__ a, long long n, long long loads, long long* __restrict__ out) {
    long long s = 0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < loads;
         i += (long long)gridDim.x * blockDim.x) {
        unsigned long long h = (unsigned long long)i * 0x9E3779B97F4A7C15ULL;
        h ^= h >> 29;
        s += a[h % (unsigned long long)n];
    }
    if (s == 0x7fffffffffffLL) out[0] = s;
}
__global__ void k_store8(long long* __restrict__ a, long long n) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        a[i] = i;
}
__global__ void k_atomic8(long long* __restrict__ a, long long n, long long ops) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < ops;
         i += (long long)gridDim.x * blockDim.x) {
        unsigned long long h = (unsigned long long)i * 0x9E3779B97F4A7C15ULL;
        h ^= h >> 29;
        __hip_atomic_fetch_add(&a[h % (unsigned long long)n], 1LL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

int main() {
    const long long n8 = 1LL << 27;   // 1 GiB of int64
    long long *a, *out;
    CK(hipMalloc(&a, n8 * 8));
    CK(hipMalloc(&out, 8));
    CK(hipMemset(a, 1, n8 * 8));
    const int grid = 8192, blk = 256;
    const long long loads = 1LL << 24;   // 16 Mi gathers / atomics
    hipLaunchKernelGGL(k_stream8, dim3(grid), dim3(blk), 0, 0, a, n8, out);
    hipLaunchKernelGGL(k_stream4, dim3(grid), dim3(blk), 0, 0, (const int*)a, 2 * n8, out);
    hipLaunchKernelGGL(k_gather8, dim3(grid), dim3(blk), 0, 0, a, n8, loads, out);
    hipLaunchKernelGGL(k_store8, dim3(grid), dim3(blk), 0, 0, a, n8);
    hipLaunchKernelGGL(k_atomic8, dim3(grid), dim3(blk), 0, 0, a, n8, loads);
    CK(hipDeviceSynchronize());
    std::printf("{\"k_stream8\": %lld, \"k_stream4\": %lld, \"k_gather8\": %lld, \"k_gather8_loads\": %lld, "
                "\"k_store8\": %lld, \"k_atomic8_ops\": %lld}\n",
                n8 * 8, n8 * 8, loads * 8, loads, n8 * 8, loads);
    CK(hipFree(a));
    CK(hipFree(out));
    return 0;
}
