#!/bin/bash
# Build (here: BUILD=1) and run the kernarg-preload probe.
set -eu
cd "$(dirname "$0")"
if [ "${BUILD:-0}" = "1" ]; then
  H=/opt/rocm/bin/hipcc; F="-O3 --offload-arch=gfx950 -fgpu-rdc"
  $H $F -c preload_kern.hip -DKNAME=probe_plain -o k_plain.o
  $H $F -c preload_kern.hip -DKNAME=probe_pre -mllvm -amdgpu-kernarg-preload-count=16 -o k_pre.o
  $H $F -c preload_main.hip -o main.o
  $H -fgpu-rdc --hip-link --offload-arch=gfx950 main.o k_plain.o k_pre.o -o preload_probe
  exit 0
fi
timeout -k 10 60 ./preload_probe
