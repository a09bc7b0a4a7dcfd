# A/B (round 6): rot() evaluates the straight-line fast form for every input and replaces its result
# by glibc's other branches (Payne-Hanek at 120 rad and above, inf / NaN) only on the lanes that need
# them, behind one wave-uniform test.  Same bits; the branch in front of the fast form cost a chained
# call 338 cycles against 226 (tools/micro/f64lat.hip).
EDITS = [("mrp_math.h", '''MRP_HD Rot rot(float y) {
    if (abstop12(y) < abstop12(120.0f)) return rot_fast(y);
    return rot_slow(y);
}''', '''MRP_HD Rot rot(float y) {
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
}''')]
