#!/bin/bash
# Build an experimental variant of the library with one kernel source replaced:
#   tools/build_variant.sh <name> <replaced csrc file name> <variant source> [extra hipcc flags]
# -> tauv-vision_amd/lib/variants/<name>.so (load it with TV_LIB=...)
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT/tauv-vision_amd"
name=$1; target=$2; src=$(realpath "$ROOT/$3"); shift 3
mkdir -p build/var_$name lib/variants
objs=""
for f in $(sed -n "s/^SRC := //p" Makefile); do
  b=$(basename $f)
  if [ "$b" = "$target" ]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Icsrc "$@" -x hip -c "$src" -o build/var_$name/$b.o
    objs="$objs build/var_$name/$b.o"
  else
    objs="$objs build/$b.o"
  fi
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o lib/variants/$name.so $objs
echo lib/variants/$name.so
