// Micro-benchmark (diagnostic): the cost of handing one body's velocities from one wave to another
// wave of the same workgroup through LDS -- the exchange a two-wave island solve
// would put on its chain at every cross-wave Gauss-Seidel dependency.
//   flag: wave 0 writes 64 lanes + a release flag, wave 1 spins on the flag (acquire), reads, replies
//   barrier: the same ping-pong with __syncthreads between the halves
// Prints cycles (s_memtime) per one-way handoff; `blocks` workgroups run at once (1: a lone pair).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(128) void k_flag(int iters, unsigned long long* out, float* sink) {
    __shared__ float val[2][64];
    __shared__ int flag[2];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (threadIdx.x < 2) flag[threadIdx.x] = 0;
    __syncthreads();
    float x = (float)l;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 1; i <= iters; ++i) {
        if (w == 0) {
            val[0][l] = x;
            __hip_atomic_store(&flag[0], i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            for (int g = 0; g < (1 << 22) && __hip_atomic_load(&flag[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < i; ++g) {}
            x = val[1][l] + 1.0f;
        } else {
            for (int g = 0; g < (1 << 22) && __hip_atomic_load(&flag[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < i; ++g) {}
            x = val[0][l] + 1.0f;
            val[1][l] = x;
            __hip_atomic_store(&flag[1], i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[blockIdx.x * 128 + threadIdx.x] = x;
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(128) void k_barrier(int iters, unsigned long long* out, float* sink) {
    __shared__ float val[2][64];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    float x = (float)l;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 1; i <= iters; ++i) {
        if (w == 0) val[0][l] = x;
        __syncthreads();
        if (w == 1) { x = val[0][l] + 1.0f; val[1][l] = x; }
        __syncthreads();
        if (w == 0) x = val[1][l] + 1.0f;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[blockIdx.x * 128 + threadIdx.x] = x;
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

template <typename K> static void run(K kern, const char* name, int blocks, unsigned long long* d, float* s) {
    const int iters = 2000;
    static unsigned long long h[4096];
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(128), 0, 0, iters, d, s);
        if (hipDeviceSynchronize() != hipSuccess) { printf("%s: launch failed\n", name); return; }
    }
    (void)hipMemcpy(h, d, (size_t)blocks * 8, hipMemcpyDeviceToHost);
    double mx = 0, sum = 0;
    for (int b = 0; b < blocks; ++b) { sum += (double)h[b]; if (h[b] > mx) mx = (double)h[b]; }
    printf("%-8s blocks %5d: cycles per one-way handoff mean %7.1f max %7.1f\n", name, blocks,
           sum / blocks / (2.0 * iters), mx / (2.0 * iters));
}

int main() {
    unsigned long long* d; float* s;
    if (hipMalloc(&d, 4096 * 8) != hipSuccess || hipMalloc(&s, 4096 * 128 * 4) != hipSuccess) return 1;
    for (int blocks : {1, 256, 1024}) {
        run(k_flag, "flag", blocks, d, s);
        run(k_barrier, "barrier", blocks, d, s);
    }
    return 0;
}
