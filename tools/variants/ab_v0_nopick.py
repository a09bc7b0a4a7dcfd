# A/B (round 6): v0 without the two-ballot case test / cross-product tangent speed
# (MRP_VEL_PICK2, MRP_VEL_VTCROSS), keeping the branch-free selection on its lanes path.
EDITS = []
FLAGS = {"mrp_env0.hip": ["-DMRP_LANES_PAIRS=1", "-mllvm", "-amdgpu-sched-strategy=iterative-ilp", "-DMRP_FRESH_REGS=1",
                          "-DMRP_VEL_BFREE=2", "-DMRP_VEL_BFREE_LANES=1"]}
