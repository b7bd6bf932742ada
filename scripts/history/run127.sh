#!/bin/bash
# Access-shape read-bandwidth microbench (built on the CPU side:
#   hipcc -O3 --offload-arch=gfx950 scripts/bw_shapes.hip -o build/bw_shapes)
source scripts/gpu_check.sh
step bw_shapes 120 ./build/bw_shapes
