#!/bin/bash
# Register use of the gfx950 kernels of one object: scripts/kmeta.sh build/device.o [name-regex]
set -e
OBJ=$1; PAT=${2:-.}
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$B/llvm-objcopy -O binary --only-section=.hip_fatbin "$OBJ" $T/fat.bin
$B/clang-offload-bundler -type=o -targets=hipv4-amdgcn-amd-amdhsa--gfx950 -input=$T/fat.bin -output=$T/dev.co -unbundle
$B/llvm-readelf --notes $T/dev.co | grep -E "^\s+\.name:|\.vgpr_count|\.vgpr_spill_count|\.private_segment_fixed_size|\.group_segment_fixed_size" \
  | paste - - - - - | grep -E "$PAT" | sed 's/  */ /g'
rm -rf $T
