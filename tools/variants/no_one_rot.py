# A/B (round 6): v0 / Heavy-v0 with the position passes' rotation memo instead of the ONE_ROT form
# (-DMRP_ONE_ROT=0 on their units, every other flag as build.py sets it).
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from gym_puzzles_amd.build import UNIT_FLAGS  # noqa: E402

EDITS = []
FLAGS = {u: list(UNIT_FLAGS.get(u, [])) + ["-DMRP_ONE_ROT=0"] for u in ("mrp_env0.hip", "mrp_env1.hip")}
