#!/bin/bash
# Build libvtseg variants that differ only in decode_full.hip compile-time
# switches (-D flags of an experiment), for same-box A/B timing: tools/exp/lib_<name>.so.
#   bash tools/exp/build_full_variants.sh name:-DFLAG ...
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
PKG=$ROOT/video-transformer_amd
B=$PKG/build
mkdir -p $B/exp
OTHERS=$(ls $B/*.o | grep -v decode_full.hip.o)
build() {
  name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$ROOT/include -I$PKG/csrc -munsafe-fp-atomics "$@" -c $PKG/csrc/decode_full.hip -o $B/exp/decode_full_$name.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $ROOT/tools/exp/lib_$name.so $B/exp/decode_full_$name.o $OTHERS -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
}
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  build $name $flags &
done
wait
ls -la $ROOT/tools/exp/*.so
