#!/bin/bash
# A variant of libddm_amd.so with one source rebuilt under extra flags:
#   tools/build_variant.sh <name> <source.hip> <flags...>  ->  ddm_amd/libddm_amd_<name>.so
set -e
name=$1; src=$2; shift 2
cd "$(dirname "$0")/../distributed-drift-detection_amd/csrc"
make -j8 >/dev/null
mkdir -p /tmp/variant_$name
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -mcode-object-version=5 \
    "$@" -c $src -o /tmp/variant_$name/${src%.hip}.o
cd ../build
TL=$(python3 -c "import os,torch;print(os.path.join(os.path.dirname(torch.__file__),'lib'))")
objs=$(ls *.o | grep -v "^${src%.hip}.o$")
g++ -shared -o ../ddm_amd/libddm_amd_$name.so $objs /tmp/variant_$name/${src%.hip}.o -L$TL -l:libamdhip64.so -Wl,-rpath,$TL -Wl,--no-undefined
