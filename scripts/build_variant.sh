#!/usr/bin/env bash
# Build an A/B variant of libcfd_amd.so with extra compile flags:
#   scripts/build_variant.sh NAME "-DFOO=1"  ->  computational-fluid-dynamics_amd/libcfd_amd_NAME.so
set -e
cd "$(dirname "$0")/../computational-fluid-dynamics_amd"
name=$1; shift
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -I../include"
/opt/rocm/bin/hipcc $F "$@" -c csrc/solver.hip -o /tmp/solver_$name.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 /tmp/solver_$name.o csrc/comm.o csrc/vtk.o csrc/params.o -o libcfd_amd_$name.so -ldl -Wl,-rpath,/opt/rocm/lib
echo built libcfd_amd_$name.so
