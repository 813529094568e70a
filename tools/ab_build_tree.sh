#!/bin/bash
# Build an A/B variant library from the WORKING TREE's kernel sources with one file replaced:
#   bash tools/ab_build_tree.sh <name> [csrc-file-name replacement-path]  ->  ab/<name>/libvclip.so
set -e
name=$1; f=$2; rep=$3
root=$(cd "$(dirname "$0")/.." && pwd)
pkg=$root/ai-laryngeal-video-based-classifier_amd
d=$root/ab/$name
rm -rf "$d"; mkdir -p "$d/csrc" "$d/include"
cp $pkg/csrc/*.hip $pkg/csrc/*.hpp "$d/csrc/"; cp $root/include/vclip.h "$d/include/"
[ -n "$f" ] && cp "$rep" "$d/csrc/$f"
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
