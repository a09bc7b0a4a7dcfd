# A/B (round 6): MRP_FRESH_REGS (late values made where used, the thread id opaque per island / TOI pass)
# on the Heavy-v0, v2 and 3-block units as well (v0 and v3 already build with it).
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from gym_puzzles_amd.build import UNIT_FLAGS  # noqa: E402

EDITS = []
FLAGS = {u: list(UNIT_FLAGS.get(u, [])) + ["-DMRP_FRESH_REGS=1"] for u in ("mrp_env1.hip", "mrp_env2.hip", "mrp_env4.hip")}
