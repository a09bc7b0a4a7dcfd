# A/B (round 6): v0 without the branch-free selection on its lanes path
# (MRP_VEL_BFREE_LANES), keeping the two-ballot case test and the cross-product tangent speed.
EDITS = []
FLAGS = {"mrp_env0.hip": ["-DMRP_LANES_PAIRS=1", "-mllvm", "-amdgpu-sched-strategy=iterative-ilp", "-DMRP_FRESH_REGS=1",
                          "-DMRP_VEL_PICK2=1", "-DMRP_VEL_VTCROSS=1"]}
