# A/B (round 6): the branch-free block-solver selection on the lanes path only (MRP_VEL_BFREE_LANES, as v0
# builds) for Heavy-v0 and v3, whose round-5 A/B covered only the form on both paths (-1.0 % / -4.9 %).
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from gym_puzzles_amd.build import UNIT_FLAGS  # noqa: E402

EDITS = []
FLAGS = {u: list(UNIT_FLAGS.get(u, [])) + ["-DMRP_VEL_BFREE=1", "-DMRP_VEL_BFREE_LANES=1"] for u in ("mrp_env1.hip", "mrp_env5.hip")}
