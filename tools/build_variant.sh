#!/bin/bash
# Build an experimental variant of the solver library next to the product one:
#   tools/build_variant.sh NAME [-DFLAG ...]  ->  safe-autonomous-driving-mpc_amd/libmpcqp_NAME.so
# (timed against the product build with tools/ab_probe.py; never loaded by the product)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off ${SCHED--mllvm -amdgpu-sched-strategy=iterative-ilp} -Wno-unused-result \
  -Wno-unused-value -Wno-pass-failed "$@" -o "$R/safe-autonomous-driving-mpc_amd/libmpcqp_$name.so" \
  "$R/safe-autonomous-driving-mpc_amd/csrc/mpcqp.hip"
