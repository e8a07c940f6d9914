#!/bin/bash
# Build a tuning variant of libpsgd.so into powersgd_amd/_lib_v/<name>/libpsgd.so, recompiling
# only the given objects with the extra flags (the rest copied from the default build).
# usage: tools/build_variant.sh <name> "<EXTRA flags>" <obj.hip|obj.cpp> ...
set -e
name=$1; extra=$2; shift 2
cd "$(dirname "$0")/../powersgd_amd/csrc"
make -s -j8 >/dev/null
vdir=../_build_v/$name
rm -rf "$vdir"; mkdir -p "$vdir"
cp ../_build/*.o "$vdir"/
for src in "$@"; do rm -f "$vdir/$src.o"; done
make -s -j8 OBJDIR="$vdir" OUT="../_lib_v/$name/libpsgd.so" EXTRA="$extra" "../_lib_v/$name/libpsgd.so"
echo "built _lib_v/$name ($extra)"
