// Micro-benchmark (diagnostic): cycles per b2Rot::Set (mrp::rot) on one wave, wave-uniform and
// per-lane inputs, in a dependent chain.  hipcc --offload-arch=gfx950 -O3 -ffp-contract=off
// -fno-fast-math -fno-gpu-flush-denormals-to-zero tools/micro/rotbench.hip -o /tmp/rotbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../gym_puzzles_amd/csrc/mrp_math.h"
using namespace mrp;

__global__ void k(int n, float a0, int uniform, unsigned long long* out, float* sink) {
    float a = uniform ? a0 : a0 + 1e-3f * threadIdx.x;
    float acc = 0.0f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
        Rot q = rot(a);
        acc += q.s;
        a = a + q.c * 1e-6f;   // dependent chain through the angle
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[threadIdx.x] = acc + a;
    if (threadIdx.x == 0) out[0] = t1 - t0;
}
__global__ void kbase(int n, float a0, unsigned long long* out, float* sink) {
    float a = a0, acc = 0.0f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) { acc += a; a = a + a * 1e-6f; }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[threadIdx.x] = acc + a;
    if (threadIdx.x == 0) out[0] = t1 - t0;
}
int main() {
    unsigned long long* d; float* s; hipMalloc(&d, 8); hipMalloc(&s, 256 * 4);
    const float angles[] = {0.3f, 2.5f, 40.0f, 200.0f};
    for (float a0 : angles)
        for (int u = 1; u >= 0; --u) {
            unsigned long long c[2];
            for (int rep = 0; rep < 2; ++rep) {
                hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, 10000, a0, u, d, s);
                hipDeviceSynchronize();
                hipMemcpy(&c[rep], d, 8, hipMemcpyDeviceToHost);
            }
            printf("angle %7.2f %s: %.1f cycles per rot\n", a0, u ? "uniform " : "per-lane", c[1] / 10000.0);
        }
    unsigned long long c;
    hipLaunchKernelGGL(kbase, dim3(1), dim3(64), 0, 0, 10000, 0.3f, d, s);
    hipDeviceSynchronize();
    hipMemcpy(&c, d, 8, hipMemcpyDeviceToHost);
    printf("loop baseline (2 dependent f32 ops): %.1f cycles per iteration\n", c / 10000.0);
    return 0;
}
