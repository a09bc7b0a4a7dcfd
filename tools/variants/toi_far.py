# A/B (round 6): the TOI candidate scan skips b2TimeOfImpact for pairs whose cores stay provably farther
# apart over the sweep than the touching band (the only TOI output toi_event reads is state == touching
# and its t; every other state gives alpha = 1), so the skipped pairs' alphas are the same bits.
EDITS = [("mrp_world.h", "    // b2TimeOfImpact; state 3 == e_touching\n", r'''    // A box around one body's core over its sweep (beta in [0, 1]): every vertex sits at
    // p(beta) + R(angle(beta)) (v - lc), p linear between c0 and c.  A body whose angle is 0 at both ends
    // (static bodies, the v0 agents) has R = identity, so its vertex offsets bound it directly;
    // otherwise every vertex lies within max |v - lc| of p(beta).  Rounding moves the box by ulps.
    __device__ __forceinline__ static void sweep_box(const DProxy& p, const SweepV& s, V2& lo, V2& hi) {
        const float px0 = fmin_(s.c0x, s.cx), px1 = fmax_(s.c0x, s.cx), py0 = fmin_(s.c0y, s.cy), py1 = fmax_(s.c0y, s.cy);
        if (s.a0 == 0.0f && s.a == 0.0f) {
            float xlo = 3.0e38f, xhi = -3.0e38f, ylo = 3.0e38f, yhi = -3.0e38f;
            for (int k = 0; k < p.count; ++k) {
                const float rx = p.v[k].x - s.lcx, ry = p.v[k].y - s.lcy;
                xlo = fmin_(xlo, rx); xhi = fmax_(xhi, rx); ylo = fmin_(ylo, ry); yhi = fmax_(yhi, ry);
            }
            lo = v2(px0 + xlo, py0 + ylo); hi = v2(px1 + xhi, py1 + yhi);
        } else {
            float r2 = 0.0f;
            for (int k = 0; k < p.count; ++k) {
                const float rx = p.v[k].x - s.lcx, ry = p.v[k].y - s.lcy;
                r2 = fmax_(r2, rx * rx + ry * ry);
            }
            const float R = sqrtf(r2);
            lo = v2(px0 - R, py0 - R); hi = v2(px1 + R, py1 + R);
        }
    }
    // true when b2TimeOfImpact cannot report e_touching for this pair: it does so only at a time t1 whose
    // core distance (GJK's, >= the true distance up to rounding; or the separation function's, which at
    // t1 is at least GJK's distance) is within target + tolerance, and the sweep boxes are farther apart
    // than that plus a margin of 0.05 m (10 linear slops, far above any rounding of these coordinates).
    // NaN coordinates never skip.
    __device__ __forceinline__ static bool toi_far(const DProxy& pA, const SweepV& sA, const DProxy& pB, const SweepV& sB) {
        V2 aLo, aHi, bLo, bHi;
        sweep_box(pA, sA, aLo, aHi);
        sweep_box(pB, sB, bLo, bHi);
        const float gx = fmax_(fmax_(aLo.x - bHi.x, bLo.x - aHi.x), 0.0f);
        const float gy = fmax_(fmax_(aLo.y - bHi.y, bLo.y - aHi.y), 0.0f);
        const float target = fmax_(LINEAR_SLOP, pA.radius + pB.radius - 3.0f * LINEAR_SLOP);
        const float thr = target + 0.25f * LINEAR_SLOP + 0.05f;
        return gx * gx + gy * gy > thr * thr;
    }
    // b2TimeOfImpact; state 3 == e_touching
'''),
         ("mrp_world.h", "                sh.u.toi.tout[i] = time_of_impact(pA, pB, sh.u.toi.tsA[i], sh.u.toi.tsB[i]);\n",
          r'''                const SweepV sA = sh.u.toi.tsA[i], sB = sh.u.toi.tsB[i];
                TOIOut o;
                o.state = 4; o.t = 1.0f;   // e_separated: what b2TimeOfImpact returns for such a pair
                if (!toi_far(pA, sA, pB, sB)) o = time_of_impact(pA, pB, sA, sB);
                sh.u.toi.tout[i] = o;
''')]
