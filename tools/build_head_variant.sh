#!/bin/bash
# Development helper: link a libcpx variant whose translation unit SRC (default k_texture) is
# taken from git revision REV (default HEAD) -> tools/_var/libcpx_<name>.so, for same-box A/B timing.
#   [SRC=k_texture] [REV=HEAD] [DEFS="-D..."] tools/build_head_variant.sh name
set -e
SRC=${SRC:-k_texture}
REV=${REV:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/image-processing-suite_amd/csrc
make -C "$CS" -j8 >/dev/null
mkdir -p "$ROOT/tools/_var"
git -C "$ROOT" show "$REV:image-processing-suite_amd/csrc/$SRC.hip" > "$CS/_rev_$SRC.hip"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off $DEFS \
  -c "$CS/_rev_$SRC.hip" -o "/tmp/rev_$1.o"
rm -f "$CS/_rev_$SRC.hip"
objs=$(ls "$CS"/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$ROOT/tools/_var/libcpx_$1.so" $objs "/tmp/rev_$1.o"
echo "built tools/_var/libcpx_$1.so ($SRC.hip @ $REV)"
