# A/B (round 6): v0's and v3's k_step at 2 waves per SIMD (launch bounds; a 256-VGPR budget instead of
# 168).  Their launches are bounded by the slowest lane-step, not by residency (v0: mean lane-step 83 K
# cycles x 4096 lanes over 2048 resident waves is 166 K cycles, against 877 K for the slowest), so the
# question is whether the wider budget shortens the serial chain.
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from gym_puzzles_amd.build import UNIT_FLAGS  # noqa: E402

EDITS = []
FLAGS = {u: list(UNIT_FLAGS[u]) + ["-DMRP_STEP_WAVES_PER_EU=2"] for u in ("mrp_env0.hip", "mrp_env5.hip")}
