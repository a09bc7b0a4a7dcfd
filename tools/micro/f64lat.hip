// Micro-benchmark (diagnostic): one wave's dependent-chain cost of the f64 / f32 operations that
// b2Rot::Set (mrp::rot) is built from, and of rot variants that shorten its chain, on a
// wave-uniform angle (the position passes' case: every lane rotates lane i's angle).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math -fno-gpu-flush-denormals-to-zero \
//         tools/micro/f64lat.hip -o tools/micro/f64lat
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../gym_puzzles_amd/csrc/mrp_math.h"
using namespace mrp;

constexpr int N = 4096;

__global__ void k_fma64(double a0, unsigned long long* out, double* sink) {
    double a = a0 + 1e-9 * threadIdx.x, b = 1.0000001, c = 1e-9;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
    for (int i = 0; i < N; ++i) a = fma(a, b, c);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[threadIdx.x] = a;
    if (threadIdx.x == 0) out[0] = t1 - t0;
}
__global__ void k_mul64(double a0, unsigned long long* out, double* sink) {
    double a = a0 + 1e-9 * threadIdx.x, b = 1.0000001;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
    for (int i = 0; i < N; ++i) a = a * b;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[threadIdx.x] = a;
    if (threadIdx.x == 0) out[0] = t1 - t0;
}
__global__ void k_fma32(float a0, unsigned long long* out, float* sink) {
    float a = a0 + 1e-6f * threadIdx.x, b = 1.0000001f, c = 1e-9f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
    for (int i = 0; i < N; ++i) a = __builtin_fmaf(a, b, c);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[threadIdx.x] = a;
    if (threadIdx.x == 0) out[0] = t1 - t0;
}
__global__ void k_cvt(float a0, unsigned long long* out, float* sink) {   // f32 -> f64 -> f32 round trip
    float a = a0 + 1e-6f * threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
    for (int i = 0; i < N; ++i) { double d = a; a = (float)(d * 1.0000001); }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[threadIdx.x] = a;
    if (threadIdx.x == 0) out[0] = t1 - t0;
}
// rot_fast with the quadrant predicted (n_pred, e.g. the previous call's quadrant): the polynomials
// start from fma(-n_pred, pi/2, x) at once, the exact quadrant is computed beside them and a rare
// wave-uniform branch redoes the reduction when the prediction was wrong (same bits as rot_fast)
__device__ __forceinline__ Rot rot_pred(float y, int& npred) {
    const double x = y;
    const double xr = fma(-(double)npred, SC_HPI, x);
    const double r = x * SC_HPI_INV;
    const int n = ((int32_t)r + 0x800000) >> 24;
    Rot q;
    if (__builtin_amdgcn_readfirstlane(n) == npred) {
        const int m = npred;
        const double xs = ((m + 1) & 2) ? -xr : xr;
        const double x2 = xr * xr;
        const double x3 = xs * x2;
        const double s1 = fma(x2, SC_S3, SC_S2);
        const double x7 = x3 * x2;
        const double ss = fma(x3, SC_S1, xs);
        const float ps = (float)fma(x7, s1, ss);
        const double x4 = x2 * x2;
        const double c2 = fma(x2, SC_C4, SC_C3);
        const double c1 = fma(x2, SC_C1, SC_C0);
        const double x6 = x4 * x2;
        const double cc = fma(x4, SC_C2, c1);
        const float pc0 = (float)fma(x6, c2, cc);
        const float pc = (m & 2) ? -pc0 : pc0;
        const bool odd = (m & 1) != 0;
        const bool tiny = abstop12(y) < abstop12(0x1p-12f);
        q.s = tiny ? y : (odd ? pc : ps);
        q.c = tiny ? 1.0f : (odd ? ps : pc);
    } else {
        npred = __builtin_amdgcn_readfirstlane(n);
        q = rot_fast(y);
    }
    return q;
}
// glibc's small-argument branch alone (|y| < pi/4, n = 0): no reduction
__device__ __forceinline__ Rot rot_small(float y) {
    const double x = y, x2 = x * x;
    Rot q;
    q.s = sincos_poly(x, x2, false, 0);
    q.c = sincos_poly(x, x2, false, 1);
    if (abstop12(y) < abstop12(0x1p-12f)) { q.s = y; q.c = 1.0f; }
    return q;
}

// rot chain: the angle of the next call depends on the previous result (as in the position passes)
template <int V>
__global__ void k_rot(float a0, unsigned long long* out, float* sink) {
    float a = __builtin_amdgcn_readfirstlane(__float_as_int(a0)) ? a0 : a0;
    float acc = 0.0f;
    int npred = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N / 16; ++i) {
        const float u = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(a)));   // wave-uniform (SGPR)
        Rot q;
        if (V == 0) q = rot(u);
        else if (V == 1) q = rot_fast(u);
        else if (V == 2) q = rot_pred(u, npred);
        else q = rot_small(u);
        acc += q.s;
        a = u + q.c * 1e-7f;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[threadIdx.x] = acc + a;
    if (threadIdx.x == 0) out[0] = t1 - t0;
}

int main() {
    unsigned long long* d; double* sd; float* sf;
    hipMalloc(&d, 8); hipMalloc(&sd, 64 * 8); hipMalloc(&sf, 64 * 4);
    unsigned long long c;
    auto rd = [&](const char* what, double per) {
        hipDeviceSynchronize();
        hipMemcpy(&c, d, 8, hipMemcpyDeviceToHost);
        printf("%-44s %8.1f cycles per op\n", what, c / per);
    };
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_fma64, dim3(1), dim3(64), 0, 0, 1.0, d, sd); rd("v_fma_f64 dependent chain", N);
        hipLaunchKernelGGL(k_mul64, dim3(1), dim3(64), 0, 0, 1.0, d, sd); rd("v_mul_f64 dependent chain", N);
        hipLaunchKernelGGL(k_fma32, dim3(1), dim3(64), 0, 0, 1.0f, d, sf); rd("v_fma_f32 dependent chain", N);
        hipLaunchKernelGGL(k_cvt, dim3(1), dim3(64), 0, 0, 1.0f, d, sf); rd("cvt f32->f64, mul_f64, cvt f64->f32 (3 ops)", N);
        const float angles[] = {0.3f, 2.5f, 40.0f};
        for (float a0 : angles) {
            char buf[96];
            hipLaunchKernelGGL(k_rot<0>, dim3(1), dim3(64), 0, 0, a0, d, sf);
            snprintf(buf, sizeof buf, "rot (angle %.1f, wave-uniform, chained)", a0); rd(buf, N / 16);
            hipLaunchKernelGGL(k_rot<1>, dim3(1), dim3(64), 0, 0, a0, d, sf);
            snprintf(buf, sizeof buf, "rot_fast (angle %.1f, wave-uniform, chained)", a0); rd(buf, N / 16);
            hipLaunchKernelGGL(k_rot<2>, dim3(1), dim3(64), 0, 0, a0, d, sf);
            snprintf(buf, sizeof buf, "rot_pred (angle %.1f, wave-uniform, chained)", a0); rd(buf, N / 16);
            if (a0 < 0.7f) {
                hipLaunchKernelGGL(k_rot<3>, dim3(1), dim3(64), 0, 0, a0, d, sf);
                snprintf(buf, sizeof buf, "rot_small (angle %.1f, wave-uniform, chained)", a0); rd(buf, N / 16);
            }
        }
    }
    return 0;
}
