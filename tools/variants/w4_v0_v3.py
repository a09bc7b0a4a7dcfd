# A/B (round 6): v0's and v3's k_step at 4 waves per SIMD (launch bounds; a 128-VGPR budget instead of
# 168): every lane of a 4096-lane batch resident at once.  Round 6 found v0's steady state (steps 501-700,
# whole episode) residency-bound (two waves per SIMD: -7 %), the driver window bounded by the slowest
# lane-step; round 3 measured the driver window level at 4 waves (with spills).
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from gym_puzzles_amd.build import UNIT_FLAGS  # noqa: E402

EDITS = []
FLAGS = {u: list(UNIT_FLAGS[u]) + ["-DMRP_STEP_WAVES_PER_EU=4"] for u in ("mrp_env0.hip", "mrp_env5.hip")}
