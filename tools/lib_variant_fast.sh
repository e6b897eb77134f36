#!/bin/bash
# Like tools/lib_variant.sh, but rebuilds only the named objects with the extra defines and links them
# with the tree's other objects (copied from build/obj): the conv instantiations are not recompiled.
#   tools/lib_variant_fast.sh NAME "-DSDP_X=1" "merge aux"  ->  tools/_var/NAME/libsdp.so
set -eu
cd "$(dirname "$0")/.."
NAME=$1; DEFS=$2; OBJS=$3
D=tools/_var/$NAME
B=simultaneous-diffusion-for-pointclouds_amd/build/obj
[ -d $B ] || { echo "build the library first ($B missing)"; exit 1; }
rm -rf $D; mkdir -p $D/obj
cp -p $B/*.o $D/obj/
for o in $OBJS; do rm -f $D/obj/$o.o; done
make -C simultaneous-diffusion-for-pointclouds_amd/csrc -j${JOBS:-8} OBJDIR=$PWD/$D/obj OUT=$PWD/$D/libsdp.so EXTRA="$DEFS" > $D/build.log 2>&1 \
  || { tail -30 $D/build.log; exit 1; }
rm -rf $D/obj
echo "built $D/libsdp.so ($DEFS; rebuilt: $OBJS)"
