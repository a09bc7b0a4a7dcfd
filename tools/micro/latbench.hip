// Micro-benchmark (diagnostic): dependent vs independent f32 VALU chains on one wave (cycles per op).
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CH>
__global__ void k(int n, float x, unsigned long long* out, float* sink) {
    float a[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = x + c + threadIdx.x;
    const float m = 1.0000001f, b = 1e-7f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#pragma unroll
            for (int c = 0; c < CH; ++c) { a[c] = a[c] * m; a[c] = a[c] + b; }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0; for (int c = 0; c < CH; ++c) s += a[c];
    sink[threadIdx.x] = s;
    if (threadIdx.x == 0) out[0] = t1 - t0;
}
template <int CH> void run(unsigned long long* d, float* s, int waves) {
    unsigned long long c[2];
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k<CH>, dim3(1), dim3(64 * waves), 0, 0, 1000, 1.0f, d, s);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(&c[rep], d, 8, hipMemcpyDeviceToHost);
    }
    printf("%d chain(s), %d wave(s) in the block: %.2f cycles per op per chain-step (%.2f cycles per issued op)\n", CH, waves,
           c[1] / (1000.0 * 16 * 2), c[1] / (1000.0 * 16 * 2 * CH));
}
int main() {
    unsigned long long* d; float* s;
    (void)hipMalloc(&d, 8); (void)hipMalloc(&s, 1024 * 4);
    run<1>(d, s, 1); run<2>(d, s, 1); run<4>(d, s, 1); run<8>(d, s, 1);
    run<1>(d, s, 4); run<1>(d, s, 8); run<1>(d, s, 16);
    return 0;
}
