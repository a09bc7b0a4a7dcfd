# DIAGNOSTIC (exact, slower): the position passes' memos never hit (b2Rot::Set on every lookup but +0),
# so posbench shows what the memo saves.
EDITS = [("mrp_world.h", "            if (b == k0) { next1 = true; return q0; }   // least recently used entry is replaced\n", ""),
         ("mrp_world.h", "            if (b == k1) { next1 = false; return q1; }\n", ""),
         ("mrp_world.h", "            if (uni(b == k0)) { next1 = true; return q0; }\n", ""),
         ("mrp_world.h", "            if (uni(b == k1)) { next1 = false; return q1; }\n", "")]
