#!/bin/bash
# Build compile-time variants of librt_hip.so for A/B timing
# (scripts/bench_variants.py).  Usage: scripts/variants.sh name:"-DFLAG=.." ...
# (tile widths: -DRT_TILE_NARROW=.. / -DRT_TILE_WIDE=.., not RT_TILE_W)
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
C="$R/opencl-ray-tracer_amd/csrc"; V="$R/opencl-ray-tracer_amd/variants"
mkdir -p "$V"
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -mllvm -amdgpu-kernarg-preload-count=16 -I$R/include"
make -s -C "$C" rt_scene.o rt_scene_device.o rt_args.o
pids=()
for spec in "$@"; do
  name="${spec%%:*}"; flags="${spec#*:}"
  ( /opt/rocm/bin/hipcc $HIPFLAGS $flags -c -o "$V/$name.o" "$C/rt_device.hip" &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$V/librt_hip_$name.so" "$V/$name.o" "$C/rt_scene_device.o" "$C/rt_scene.o" "$C/rt_args.o" &&
    rm -f "$V/$name.o" && echo "built $name ($flags)" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
