#!/bin/bash
# Device-only gfx950 assembly of one csrc file (fast register / spill audit, no link):
#   tools/dev_asm.sh gemm64 [kernel-substring ...]
set -e
cd "$(dirname "$0")/.."
src=llmctl/ops/csrc/$1.hip; shift
out=build/asm/$(basename "$src" .hip).s
mkdir -p build/asm
TI=$(python -c "from torch.utils.cpp_extension import include_paths; print(' '.join('-I'+p for p in include_paths()))")
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -D__HIP_PLATFORM_AMD__ -DUSE_ROCM \
  -Wno-unused-result -Wno-deprecated-declarations -Wno-return-type -Illmctl/ops/csrc $TI "$src" -o "$out"
python tools/kernel_audit.py "$out" "$@"
