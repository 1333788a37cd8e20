#!/bin/bash
# Experiment builds of the denoiser: libvxpt_<name>.so = libvxpt.so with csrc/denoise.hip (or another
# source, path relative to the package) compiled with extra flags.
# Usage (in this container): tools/den_variants.sh name:"-DFLAG ..."[:source] ...
# Load one on the GPU box with VXPT_LIB=real-time-path-tracing-voxel-blocks_amd/libvxpt_<name>.so.
set -e
cd "$(dirname "$0")/../real-time-path-tracing-voxel-blocks_amd"
make -s libvxpt.so
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-function -Wno-unused-variable"
OTHERS=$(ls build/*.o | grep -v denoise.hip.o)
for spec in "$@"; do
    name=${spec%%:*}; rest=${spec#*:}; extra=${rest%%:*}; src=csrc/denoise.hip
    [ "$rest" != "$extra" ] && src=${rest#*:}
    mkdir -p build/var
    /opt/rocm/bin/hipcc $FLAGS $extra -Icsrc -x hip -c -o build/var/denoise_$name.o $src
    /opt/rocm/bin/hipcc $FLAGS -shared -o libvxpt_$name.so build/var/denoise_$name.o $OTHERS -L/opt/rocm/lib -lrccl -lz
    echo "built libvxpt_$name.so ($extra)"
done
