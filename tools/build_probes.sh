#!/bin/bash
# Native probes for the GPU box, built here (hipcc cross-compiles gfx950) into tools/bin
# (git-ignored; travels with the gpurun snapshot): the copy-engine probe and the native step
# driver (links the in-tree libdmlp.so).
set -e
cd "$(dirname "$0")/.."
PKG=distributed_machine_learning_project_amd
mkdir -p tools/bin
hipcc --offload-arch=gfx950 -O2 tests/native/copy_kind_probe.cpp -o tools/bin/copy_kind_probe
hipcc --offload-arch=gfx950 -O2 -std=c++17 tests/native/step_driver.cpp -I$PKG/csrc -L$PKG -ldmlp \
    -Wl,-rpath,'$ORIGIN/../../'$PKG -o tools/bin/step_driver
hipcc --offload-arch=gfx950 -O2 tests/native/h2d_bw.cpp -o tools/bin/h2d_bw
