# A/B (round 6): v0 with neither round-5 velocity change (round 4's case loop).
EDITS = []
FLAGS = {"mrp_env0.hip": ["-DMRP_LANES_PAIRS=1", "-mllvm", "-amdgpu-sched-strategy=iterative-ilp", "-DMRP_FRESH_REGS=1"]}
