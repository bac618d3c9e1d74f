#!/bin/bash
# An instrumented copy of libddm_amd.so (DDM_WALK_PROFILE), for DDM_AMD_LIB=... runs.
set -e
cd "$(dirname "$0")/../distributed-drift-detection_amd/csrc"
make -j8 >/dev/null
mkdir -p /tmp/profbuild
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -mcode-object-version=5 \
    -DDDM_WALK_PROFILE -c shuffle.hip -o /tmp/profbuild/shuffle.o
cd ../build
TL=$(python3 -c "import os,torch;print(os.path.join(os.path.dirname(torch.__file__),'lib'))")
objs=$(ls *.o | grep -v '^shuffle.o$')
g++ -shared -o ../ddm_amd/libddm_amd_prof.so $objs /tmp/profbuild/shuffle.o -L$TL -l:libamdhip64.so -Wl,-rpath,$TL -Wl,--no-undefined
