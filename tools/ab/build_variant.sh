#!/bin/bash
# Build a product-library variant with extra -D flags into tools/_ab/ (A/B against the product
# without the A/B build's probes):  tools/ab/build_variant.sh NAME -DNH_X=1 [...]
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/../.." && pwd)
tmp=$(mktemp -d /tmp/nhvar.XXXX)
mkdir -p "$tmp/nano-hevc_amd/nano_hevc"
cp -r "$root/include" "$tmp/"
cp -r "$root/nano-hevc_amd/Makefile" "$root/nano-hevc_amd/csrc" "$tmp/nano-hevc_amd/"
make -s -j8 -C "$tmp/nano-hevc_amd" HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall $*" \
  nano_hevc/libnanohevc.so
cp "$tmp/nano-hevc_amd/nano_hevc/libnanohevc.so" "$root/tools/_ab/libnanohevc_$name.so"
rm -rf "$tmp"
echo "tools/_ab/libnanohevc_$name.so"
