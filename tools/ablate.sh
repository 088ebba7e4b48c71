#!/bin/bash
# Build timing-only ablation variants of libskgehip.so (NOT correct builds):
#   build_abl/<name>/libskgehip.so   compiled with -D<FLAG>
# Used to price one piece of a kernel (e.g. the relation-row atomics).
set -e
cd "$(dirname "$0")/../scikit-kge_amd"
for v in "$@"; do
  name=${v%%=*}; flag=${v#*=}
  mkdir -p build_abl/$name
  rm -f build_abl/$name/*.o
  pids=()
  for f in csrc/*.hip; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -D$flag -c $f -o build_abl/$name/$(basename $f .hip).o &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait $p || { echo "variant $name: a source failed to compile" >&2; exit 1; }; done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined -o build_abl/$name/libskgehip.so build_abl/$name/*.o
  echo "built build_abl/$name"
done
