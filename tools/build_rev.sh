#!/bin/bash
# Build libskgehip.so from the csrc/ + include/ of a git revision into
# scikit-kge_amd/build_abl/<name>/ (for same-box A/B runs via SKGE_LIB_PATH).
# Usage: tools/build_rev.sh <name> <rev> [extra hipcc flags...]
set -e
name=$1; rev=$2; shift 2
root="$(cd "$(dirname "$0")/.." && pwd)"
tmp=$(mktemp -d)
git -C "$root" archive "$rev" scikit-kge_amd/csrc include | tar -x -C "$tmp"
out="$root/scikit-kge_amd/build_abl/$name"
mkdir -p "$out"
for f in "$tmp"/scikit-kge_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -c "$f" \
    -o "$out/$(basename "$f" .hip).o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/libskgehip.so" "$out"/*.o
rm -rf "$tmp"
echo "built $out/libskgehip.so from $rev"
