# A/B (round 6): Heavy-v0's k_step held to 2 waves per SIMD (launch bounds; at most 256 VGPRs) -- the
# final round-6 unit uses 266, which leaves one wave per SIMD although its 20 KB of LDS allow two.
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from gym_puzzles_amd.build import UNIT_FLAGS  # noqa: E402

EDITS = []
FLAGS = {"mrp_env1.hip": list(UNIT_FLAGS.get("mrp_env1.hip", [])) + ["-DMRP_STEP_WAVES_PER_EU=2"]}
