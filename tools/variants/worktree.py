# the working tree's sources as they are (with MRP_VARIANT_WORKTREE=1): an A/B library of the listed env units
EDITS = []
