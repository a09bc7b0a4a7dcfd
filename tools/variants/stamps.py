# the per-phase timing diagnostic build (-DMRP_STAMPS) of the listed env units (tools/phase_profile.py)
EDITS = []
DEFINES = ["MRP_STAMPS"]
