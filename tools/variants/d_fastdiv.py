# DIAGNOSTIC ONLY (not exact): the position update's impulse -C / K with the hardware reciprocal
# instead of the correctly rounded division, so posbench shows the division's share of a point update.
EDITS = [("mrp_world.h", "            const float impulse = K > 0.0f ? -Cc / K : 0.0f;\n",
          "            const float impulse = K > 0.0f ? -Cc * __builtin_amdgcn_rcpf(K) : 0.0f;\n")]
