#!/bin/bash
# Build an A/B variant library from a git revision of the kernel sources:
#   bash tools/ab_build.sh <rev> <name>   ->  ab/<name>/libvclip.so
# (every csrc/*.hip and common.hpp at <rev>; used by tools/ab_attn.py / ab_gemm.py to
# time two builds interleaved in ONE process, cdna_hip_programming.md rule 24)
set -e
rev=$1; name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
pkg=ai-laryngeal-video-based-classifier_amd
d=${AB_OUT:-$root/ab}/$name
rm -rf "$d"; mkdir -p "$d/csrc" "$d/include"
for f in $(git -C "$root" ls-tree --name-only "$rev" $pkg/csrc/); do
  git -C "$root" show "$rev:$f" > "$d/csrc/$(basename $f)"
done
git -C "$root" show "$rev:include/vclip.h" > "$d/include/vclip.h"
tl=$(python -c 'import torch,os;print(os.path.join(os.path.dirname(torch.__file__),"lib"))')
objs=()
for s in "$d"/csrc/*.hip; do
  o=${s%.hip}.o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I "$d/include" -I "$d/csrc" -Wno-unused-result \
    -munsafe-fp-atomics -c "$s" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$d/libvclip.so" "${objs[@]}" -L"$tl" -Wl,-rpath,"$tl"
echo "$d/libvclip.so"
