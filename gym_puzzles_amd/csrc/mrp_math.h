// mrp_math.h -- float32 vector math with Box2D v2.3 operation order, glibc-faithful
// sinf/cosf, and the counter RNG.  Compiled for gfx950 device code and for the host
// (geometry tables); both sides MUST be built with -ffp-contract=off and without
// fast-math so every expression rounds exactly like the box2d-py engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MRP_HD __host__ __device__ __forceinline__

namespace mrp {

struct V2 { float x, y; };
struct Rot { float s, c; };
struct Xf { V2 p; Rot q; };

MRP_HD V2 v2(float x, float y) { V2 r; r.x = x; r.y = y; return r; }
MRP_HD V2 vadd(V2 a, V2 b) { return v2(a.x + b.x, a.y + b.y); }
MRP_HD V2 vsub(V2 a, V2 b) { return v2(a.x - b.x, a.y - b.y); }
MRP_HD V2 vmul(float s, V2 a) { return v2(s * a.x, s * a.y); }   // b2Vec2 operator*(float, b2Vec2)
MRP_HD V2 vneg(V2 a) { return v2(-a.x, -a.y); }
MRP_HD float vdot(V2 a, V2 b) { return a.x * b.x + a.y * b.y; }
MRP_HD float vcross(V2 a, V2 b) { return a.x * b.y - a.y * b.x; }
MRP_HD V2 vcross_vs(V2 a, float s) { return v2(s * a.y, -s * a.x); }
MRP_HD V2 vcross_sv(float s, V2 a) { return v2(-s * a.y, s * a.x); }
MRP_HD float vlensq(V2 a) { return a.x * a.x + a.y * a.y; }
MRP_HD float vlen(V2 a) { return sqrtf(a.x * a.x + a.y * a.y); }
MRP_HD float vnormalize(V2& a) {
    float length = sqrtf(a.x * a.x + a.y * a.y);
    if (length < 1.1920928955078125e-7f) return 0.0f;   // b2_epsilon = FLT_EPSILON
    float inv = 1.0f / length;
    a.x *= inv; a.y *= inv;
    return length;
}
MRP_HD float fmin_(float a, float b) { return a < b ? a : b; }
MRP_HD float fmax_(float a, float b) { return a > b ? a : b; }
MRP_HD float fclamp(float a, float lo, float hi) { return fmax_(lo, fmin_(a, hi)); }
MRP_HD V2 vmin(V2 a, V2 b) { return v2(fmin_(a.x, b.x), fmin_(a.y, b.y)); }
MRP_HD V2 vmax(V2 a, V2 b) { return v2(fmax_(a.x, b.x), fmax_(a.y, b.y)); }
MRP_HD V2 mul_rv(Rot q, V2 v) { return v2(q.c * v.x - q.s * v.y, q.s * v.x + q.c * v.y); }
MRP_HD V2 mulT_rv(Rot q, V2 v) { return v2(q.c * v.x + q.s * v.y, -q.s * v.x + q.c * v.y); }
MRP_HD V2 mul_xv(Xf T, V2 v) {
    float x = (T.q.c * v.x - T.q.s * v.y) + T.p.x;
    float y = (T.q.s * v.x + T.q.c * v.y) + T.p.y;
    return v2(x, y);
}
MRP_HD V2 mulT_xv(Xf T, V2 v) {
    float px = v.x - T.p.x, py = v.y - T.p.y;
    return v2(T.q.c * px + T.q.s * py, -T.q.s * px + T.q.c * py);
}
MRP_HD Rot mulT_rr(Rot q, Rot r) { Rot o; o.s = q.c * r.s - q.s * r.c; o.c = q.c * r.c + q.s * r.s; return o; }
MRP_HD Xf mulT_xx(Xf A, Xf B) { Xf C; C.q = mulT_rr(A.q, B.q); C.p = mulT_rv(A.q, vsub(B.p, A.p)); return C; }

// Packed pairs for the solver loops: a native 2 x f32 vector, so the x and y halves of one
// b2Vec2 operation issue as ONE v_pk_add_f32 / v_pk_mul_f32 (two IEEE f32 operations, each
// rounded exactly like the scalar one; -ffp-contract=off keeps v_pk_fma_f32 out).  Broadcasts,
// half swaps and negations fold into the instruction's op_sel / neg modifiers.  Every helper
// computes each component with the operations, operands and order of its V2 counterpart above:
//   pcross_sv(s, r) = s * (-r.y, r.x) = (-(s*r.y), s*r.x) = vcross_sv(s, r)  (negation is exact)
//   pcross(a, b)    = (a * b.yx).x - (a * b.yx).y = a.x*b.y - a.y*b.x      = vcross(a, b)
//   pcrossp(pperp(a), b) = a.x*b.y + -(a.y*b.x)                           = vcross(a, b)
//   pdot(a, b)      = (a * b).x + (a * b).y                               = vdot(a, b)
//   pmul_rv(q, v)   = (c,s)*v.x + (-s,c)*v.y = (c*vx - s*vy, s*vx + c*vy)  = mul_rv(q, v)
typedef float P2 __attribute__((ext_vector_type(2)));
MRP_HD P2 p2(float x, float y) { P2 r = {x, y}; return r; }
MRP_HD P2 pbc(float s) { P2 r = {s, s}; return r; }
MRP_HD P2 pperp(P2 r) { P2 o = {-r.y, r.x}; return o; }
MRP_HD P2 pcross_sv(float s, P2 r) { return pbc(s) * pperp(r); }
MRP_HD float pcross(P2 a, P2 b) { const P2 p = a * b.yx; return p.x - p.y; }
// cross(a, b) from ap = pperp(a): ap * b = (-(a.y*b.x), a.x*b.y), and a.x*b.y + -(a.y*b.x) is
// a.x*b.y - a.y*b.x exactly; with the arms stored as perps, pcross_sv(s, a) is one pbc(s) * ap
MRP_HD float pcrossp(P2 ap, P2 b) { const P2 p = ap * b; return p.y + p.x; }
MRP_HD float pdot(P2 a, P2 b) { const P2 p = a * b; return p.x + p.y; }
MRP_HD P2 pmul_rv(Rot q, P2 v) { const P2 cs = {q.c, q.s}, sc = {-q.s, q.c}; return cs * pbc(v.x) + sc * pbc(v.y); }

// ---------------------------------------------------------------------------------------
// sinf / cosf, bit-exact with glibc >= 2.28's FMA code path (sysdeps/ieee754/flt-32
// s_sinf.c / s_cosf.c, the variant glibc's ifunc selects on every FMA-capable x86-64 CPU).
// Verified exhaustively against the host glibc 2.35 sinf/cosf over all 4,278,190,080
// finite float inputs (tests/test_sincos.py re-checks a strided subset).  Box2D calls
// sinf/cosf in every b2Rot::Set, so sharing one exact implementation is what makes the
// GPU trajectory bitwise equal to the CPU one.
// ---------------------------------------------------------------------------------------
// Coefficients are immediate operands (no table in memory: a data-dependent table pick
// compiles to global loads on the device).  glibc's second table (__sincosf_table[1]) is
// the first with c0..c4 negated and the same s1..s3, so "table 1" is the table-0 polynomial
// with its (exactly representable) result negated; `sign[n & 3]` is {+1, -1, -1, +1}.
constexpr double SC_HPI_INV = 0x1.45F306DC9C883p+23, SC_HPI = 0x1.921FB54442D18p0;
constexpr double SC_C0 = 0x1p0, SC_C1 = -0x1.ffffffd0c621cp-2, SC_C2 = 0x1.55553e1068f19p-5,
                 SC_C3 = -0x1.6c087e89a359dp-10, SC_C4 = 0x1.99343027bf8c3p-16;
constexpr double SC_S1 = -0x1.555545995a603p-3, SC_S2 = 0x1.1107605230bc4p-7, SC_S3 = -0x1.994eb3774cf24p-13;

MRP_HD double sc_sign(int n) { return ((n + 1) & 2) ? -1.0 : 1.0; }   // glibc sign[n & 3]

MRP_HD uint32_t f2u(float f) { union { float f; uint32_t u; } x; x.f = f; return x.u; }
MRP_HD float u2f(uint32_t u) { union { float f; uint32_t u; } x; x.u = u; return x.f; }
MRP_HD uint32_t abstop12(float x) { return (f2u(x) >> 20) & 0x7ff; }

// glibc sinf_poly; `neg` selects the second coefficient table (cos branch negated)
MRP_HD float sincos_poly(double x, double x2, bool neg, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = fma(x2, SC_S3, SC_S2);
        double x7 = x3 * x2;
        double s = fma(x3, SC_S1, x);
        return (float)fma(x7, s1, s);
    } else {
        double x4 = x2 * x2;
        double c2 = fma(x2, SC_C4, SC_C3);
        double c1 = fma(x2, SC_C1, SC_C0);
        double x6 = x4 * x2;
        double c = fma(x4, SC_C2, c1);
        float r = (float)fma(x6, c2, c);
        return neg ? -r : r;   // fma/round-to-nearest are odd: negated coefficients negate exactly
    }
}

MRP_HD double reduce_fast(double x, int* np) {
    double r = x * SC_HPI_INV;
    int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return fma(-(double)n, SC_HPI, x);
}

MRP_HD double reduce_large(uint32_t xi, int* np) {
    // bits of 2/pi (glibc __inv_pio4)
    const uint32_t inv_pio4[24] = {0xa2, 0xa2f9, 0xa2f983, 0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
        0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0,
        0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041};
    const uint32_t* arr = &inv_pio4[(xi >> 26) & 15];
    int shift = (xi >> 23) & 7;
    uint64_t n, res0, res1, res2;
    xi = (xi & 0xffffff) | 0x800000;
    xi <<= shift;
    res0 = xi * arr[0];
    res1 = (uint64_t)xi * arr[4];
    res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    n = (res0 + (1ULL << 61)) >> 62;
    res0 -= n << 62;
    double x = (double)(int64_t)res0;
    *np = (int)n;
    return x * 0x1.921FB54442D18p-62;
}

MRP_HD float g_sinf(float y) {
    double x = y, s; int n;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        s = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return y;
        return sincos_poly(x, s, false, 0);
    } else if (abstop12(y) < abstop12(120.0f)) {
        x = reduce_fast(x, &n);
        s = sc_sign(n);
        return sincos_poly(x * s, x * x, (n & 2) != 0, n);
    } else if (abstop12(y) < abstop12(__builtin_inff())) {
        uint32_t xi = f2u(y); int sign = xi >> 31;
        x = reduce_large(xi, &n);
        s = sc_sign(n + sign);
        return sincos_poly(x * s, x * x, ((n + sign) & 2) != 0, n);
    }
    return (y - y) / (y - y);
}

MRP_HD float g_cosf(float y) {
    double x = y, s; int n;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        double x2 = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
        return sincos_poly(x, x2, false, 1);
    } else if (abstop12(y) < abstop12(120.0f)) {
        x = reduce_fast(x, &n);
        s = sc_sign(n);
        return sincos_poly(x * s, x * x, (n & 2) != 0, n ^ 1);
    } else if (abstop12(y) < abstop12(__builtin_inff())) {
        uint32_t xi = f2u(y); int sign = xi >> 31;
        x = reduce_large(xi, &n);
        s = sc_sign(n + sign);
        return sincos_poly(x * s, x * x, ((n + sign) & 2) != 0, n ^ 1);
    }
    return (y - y) / (y - y);
}

// b2Rot::Set for |angle| < 120 without branches: glibc's fast-reduction path evaluated for every
// input below 120 (for |y| < pi/4 that path reduces with n = 0, xr = fma(-0.0, pi/2, x) = x, sign
// +1, which is exactly glibc's small-argument branch), both polynomials always, the quadrant
// picks and glibc's |y| < 2^-12 early returns as selects.  The same double operations in the same
// order as g_sinf / g_cosf, so bit-identical to them; no scalar branch and no VALU -> SALU round
// trip on the dependency chain (the branchy form took 430 cycles per call on one wave, serially
// dependent calls; this form exists because the position passes call it once per contact point).
MRP_HD Rot rot_fast(float y) {
    const double x = y;
    const double r = x * SC_HPI_INV;
    const int n = ((int32_t)r + 0x800000) >> 24;
    const double xr = fma(-(double)n, SC_HPI, x);
    const double xs = ((n + 1) & 2) ? -xr : xr;   // x * sign[n & 3] (an exact negation)
    const double x2 = xr * xr;                      // (x * s) * (x * s) == x * x
    // sin polynomial of xs (glibc sinf_poly, even n)
    const double x3 = xs * x2;
    const double s1 = fma(x2, SC_S3, SC_S2);
    const double x7 = x3 * x2;
    const double ss = fma(x3, SC_S1, xs);
    const float ps = (float)fma(x7, s1, ss);
    // cos polynomial (odd n): depends on x2 only
    const double x4 = x2 * x2;
    const double c2 = fma(x2, SC_C4, SC_C3);
    const double c1 = fma(x2, SC_C1, SC_C0);
    const double x6 = x4 * x2;
    const double cc = fma(x4, SC_C2, c1);
    const float pc0 = (float)fma(x6, c2, cc);
    const float pc = (n & 2) ? -pc0 : pc0;          // the negated second table
    const bool odd = (n & 1) != 0;
    const bool tiny = abstop12(y) < abstop12(0x1p-12f);
    Rot q;
    q.s = tiny ? y : (odd ? pc : ps);
    q.c = tiny ? 1.0f : (odd ? ps : pc);
    return q;
}

// b2Rot::Set(angle) = {sinf(angle), cosf(angle)}: g_sinf and g_cosf fused over one range
// reduction (the reduction and the sign pick are the same function of the input in both, so
// each result is bit-identical to its standalone routine).
MRP_HD Rot rot_slow(float y) {
    Rot q;
    double x = y;
    int n;
    const uint32_t t = abstop12(y);
    if (t < abstop12(0x1.921FB6p-1f)) {
        if (t < abstop12(0x1p-12f)) { q.s = y; q.c = 1.0f; return q; }
        const double x2 = x * x;
        q.s = sincos_poly(x, x2, false, 0);
        q.c = sincos_poly(x, x2, false, 1);
    } else if (t < abstop12(120.0f)) {
        x = reduce_fast(x, &n);
        const double s = sc_sign(n);
        q.s = sincos_poly(x * s, x * x, (n & 2) != 0, n);
        q.c = sincos_poly(x * s, x * x, (n & 2) != 0, n ^ 1);
    } else if (t < abstop12(__builtin_inff())) {
        const uint32_t xi = f2u(y);
        const int sign = xi >> 31;
        x = reduce_large(xi, &n);
        const double s = sc_sign(n + sign);
        q.s = sincos_poly(x * s, x * x, ((n + sign) & 2) != 0, n);
        q.c = sincos_poly(x * s, x * x, ((n + sign) & 2) != 0, n ^ 1);
    } else {
        q.s = (y - y) / (y - y);
        q.c = q.s;
    }
    return q;
}

// the entry point.  On the device: the fast form, straight-line, for every input; glibc's other
// branches (Payne-Hanek reduction at 120 rad and above, inf / NaN) replace its result on the lanes
// that need them, behind one wave-uniform test that is almost never taken (same bits; the branch in
// front of the fast form cost a chained call 338 cycles against 226, tools/micro/f64lat.hip; slowest
// lane-steps alone 1.5 % shorter in v0 / Heavy-v0 / v2, profiles/r6_rot_late_ab.txt)
MRP_HD Rot rot(float y) {
#if defined(__HIP_DEVICE_COMPILE__)
    Rot q = rot_fast(y);   // v_cvt_i32_f64 clamps the reduction of |y| >= 120; rot_slow replaces those
    const bool big = !(abstop12(y) < abstop12(120.0f));
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(big) != 0, 0)) {
        if (big) q = rot_slow(y);
    }
    return q;
#else
    if (abstop12(y) < abstop12(120.0f)) return rot_fast(y);
    return rot_slow(y);
#endif
}

// b2Rot::Set(+-0) = {+-0, 1} exactly (glibc's sinf / cosf return y and 1 below 2^-12): when no
// active lane's angle is nonzero (a static body's sweep in the TOI iterations, a body whose angle
// never left zero such as a v0 agent with invI = 0) the wave skips the polynomials; otherwise rot().
// The position passes keep rot(): their rotation memo already answers +0.
MRP_HD Rot rot_z(float y) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (__builtin_amdgcn_ballot_w64(y != 0.0f) == 0) { Rot q; q.s = y; q.c = 1.0f; return q; }
#endif
    return rot(y);
}

// ---------------------------------------------------------------------------------------
// Counter-based RNG for on-device resets and synthetic actions (pure integer SplitMix64
// mixing; identical on host and device, so the CPU oracle can replay device resets).
// ---------------------------------------------------------------------------------------
MRP_HD uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}
MRP_HD double rng_u01(uint64_t seed, uint64_t lane, uint64_t stream, uint64_t counter) {
    uint64_t h = splitmix64(seed ^ splitmix64(lane ^ splitmix64(stream ^ splitmix64(counter))));
    return (double)(h >> 11) * 0x1.0p-53;
}

}  // namespace mrp
