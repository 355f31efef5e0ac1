#!/bin/bash
# Build an A/B variant of libwgsr.so: csrc/ with the files in $2 (a directory
# of replacement .hip/.h sources) substituted -> lib/variants/$1.so.
# Run a bench against it with WGSR_LIB=wildgs-slam-blackwell_amd/lib/variants/$1.so.
# Extra compiler flags (e.g. -DNAME=value) come from $VFLAGS; $2 may be an empty directory.
set -e
name=$1; over=$2
root=$(cd "$(dirname "$0")/.." && pwd)
pkg=$root/wildgs-slam-blackwell_amd
tmp=$(mktemp -d)
cp $pkg/csrc/* $tmp/
cp $over/* $tmp/ 2>/dev/null || true
mkdir -p $pkg/lib/variants $tmp/obj
for f in $tmp/*.hip; do
  extra=""; [ "$(basename $f)" = raster_bwd.hip ] && extra="${BWD_FLAGS--fno-slp-vectorize}"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=gfx950 ${VFLAGS:-} $extra -I$tmp -I$root/include -c $f -o $tmp/obj/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o $pkg/lib/variants/$name.so $tmp/obj/*.o
rm -rf $tmp
echo built $pkg/lib/variants/$name.so
