# DIAGNOSTIC ONLY (not exact): b2Rot::Set misses of the position passes' memos replaced by a 3-op
# approximation, so posbench / the phase table show the rotations' share of a position point update.
EDITS = [("mrp_world.h", "            const P2 q = rot_cs(angle);\n", "            const P2 q = p2(1.0f - 0.5f * angle * angle, angle);\n")]
