#!/bin/bash
# A/B build: libhgx.so with one source recompiled under extra flags, written
# to tools/_ab/<name>.so (load with HGX_LIB_PATH). Usage:
#   tools/build_variant.sh NAME SOURCE.hip "-DFOO=1 ..."
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; flags=$3
mkdir -p tools/_ab
python -m hypergraphembedding_amd.build > /dev/null
objs=""
for o in hypergraphembedding_amd/_build/*.o; do
  if [ "$(basename $o)" = "$(basename $src).o" ]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Wno-pass-failed $flags -c hypergraphembedding_amd/csrc/$(basename $src) -o tools/_ab/$name.o 2>/dev/null
    objs="$objs tools/_ab/$name.o"
  else
    objs="$objs $o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/_ab/$name.so $objs
echo tools/_ab/$name.so
