#!/bin/bash
# Development helper: link libcpx variants with one translation unit (SRC, default k_texture)
# compiled under extra defines.
#   [SRC=k_conv] tools/build_variants.sh name1 "-DFOO=1" [name2 "-DBAR" ...]  ->  tools/_var/libcpx_<name>.so
set -e
SRC=${SRC:-k_texture}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/image-processing-suite_amd/csrc
make -C "$CS" -j8 >/dev/null
mkdir -p "$ROOT/tools/_var"
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off $defs \
    -c "$CS/$SRC.hip" -o "/tmp/ktv_$name.o"
  objs=$(ls "$CS"/*.o | grep -v "$SRC.o")
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$ROOT/tools/_var/libcpx_$name.so" $objs "/tmp/ktv_$name.o"
  echo "built tools/_var/libcpx_$name.so ($defs)"
done
