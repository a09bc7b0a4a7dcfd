// Exhaustive host check (diagnostic): mrp::rot / rot_fast / rot_slow against the host glibc
// sinf / cosf over every float bit pattern (NaN inputs: both NaN).  Build:
//   hipcc -O2 -ffp-contract=off -fno-fast-math -fopenmp tools/micro/rot_exhaustive.cpp -o /tmp/rot_exhaustive
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include "../../gym_puzzles_amd/csrc/mrp_math.h"

static bool same(float a, float b) {
    if (std::isnan(a) && std::isnan(b)) return true;
    uint32_t x, y;
    std::memcpy(&x, &a, 4); std::memcpy(&y, &b, 4);
    return x == y;
}
int main() {
    long long bad = 0, bad_fast = 0;
#pragma omp parallel for reduction(+ : bad, bad_fast) schedule(dynamic, 1 << 16)
    for (long long u = 0; u <= 0xffffffffLL; ++u) {
        const uint32_t b = (uint32_t)u;
        float y;
        std::memcpy(&y, &b, 4);
        const float s = sinf(y), c = cosf(y);
        const mrp::Rot q = mrp::rot(y);
        if (!same(q.s, s) || !same(q.c, c)) {
            if (bad < 10) printf("rot mismatch at %08x (%a): %a %a vs glibc %a %a\n", b, y, q.s, q.c, s, c);
            ++bad;
        }
        if (mrp::abstop12(y) < mrp::abstop12(120.0f)) {
            const mrp::Rot f = mrp::rot_fast(y);
            if (!same(f.s, s) || !same(f.c, c)) ++bad_fast;
        }
    }
    printf("rot mismatches: %lld; rot_fast mismatches below 120: %lld (all 2^32 inputs)\n", bad, bad_fast);
    return bad || bad_fast ? 1 : 0;
}
