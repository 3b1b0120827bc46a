#!/bin/bash
# Build libfdhip.so with extra compile flags into abvar/NAME.so (A/B variants for tools/gpu_session.sh).
# usage: tools/build_variant.sh NAME "XFLAGS"
set -e
name=$1
shift
root=$(cd "$(dirname "$0")/.." && pwd)
out=/tmp/fd_variant_$name
make -s -C "$root/feature_detector_amd/csrc" -j8 OUT=$out XFLAGS="$*" > /dev/null
mkdir -p "$root/abvar"
cp $out/libfdhip.so "$root/abvar/$name.so"
echo "abvar/$name.so ($*)"
