#!/bin/bash
# Tools-only A/B builds of csrc/attention.hip: one small .so per variant,
#   bash tools/ab_attn.sh <name> <attention.hip path> [extra hipcc flags...]  -> ab/attn/<name>.so
# timed interleaved in one process by tools/ab_attn.py.
set -e
name=$1; src=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
out=${AB_OUT:-$root/tools/abso}; mkdir -p "$out"
inc="-I $root/include -I $root/ai-laryngeal-video-based-classifier_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $inc -Wno-unused-result "$@" -c "$src" -o "$out/$name.o" 2>/dev/null
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -c "$root/tools/ab_attn_stub.cpp" -o "$out/stub.o"
# attention.hip dispatches S <= 256 to attention_short.hip's launcher: link the tree's copy
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $inc -c "$root/ai-laryngeal-video-based-classifier_amd/csrc/attention_short.hip" -o "$out/short.o" 2>/dev/null
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$out/$name.so" "$out/$name.o" "$out/short.o" "$out/stub.o"
echo "$out/$name.so"
