#!/bin/bash
# Register use / spills of every k_step instantiation in a built env unit object (CPU only):
#   tools/kernel_regs.sh gym_puzzles_amd/build/libmrp.so.obj/mrp_env0.hip.o
set -euo pipefail
O=$1
T=$(mktemp -d)
B=/opt/rocm/lib/llvm/bin
$B/llvm-objcopy --dump-section .hip_fatbin=$T/fb.bin "$O" /dev/null
$B/clang-offload-bundler --unbundle --type=o --input=$T/fb.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/dev.co
$B/llvm-readobj --notes $T/dev.co | grep -E "\.name:|\.vgpr_count|\.vgpr_spill_count|\.sgpr_count|\.sgpr_spill_count|private_segment_fixed_size" \
  | awk '/\.name:/ {n=$2} /private_segment/ {p=$2} /sgpr_count/ {s=$2} /sgpr_spill/ {ss=$2} /vgpr_count/ {v=$2} /vgpr_spill/ {vs=$2; if (n ~ /k_step/) printf "%s vgpr %s (spill %s) sgpr %s (spill %s) scratch %s\n", n, v, vs, s, ss, p}'
rm -rf $T
