#!/bin/bash
# build tools/probes/phase_micro variants: build_micro.sh NAME [-DFLAG ...]
cd "$(dirname "$0")"
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Wno-unused-result -Wno-unused-value "$@" -o phase_micro_$name phase_micro.hip
