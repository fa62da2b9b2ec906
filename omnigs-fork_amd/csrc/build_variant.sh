#!/bin/bash
# Build a variant of libomnigs_raster.so with extra compile flags, for kernel A/B runs on the GPU box:
#   omnigs-fork_amd/csrc/build_variant.sh NAME -DOMR_FWD_BANDS=2 ...   ->  omnigs-fork_amd/lib/exp/NAME.so
# bench.py picks it up with OMR_LIB_PATH=omnigs-fork_amd/lib/exp/NAME.so (see rasterizer.py).
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
NAME=${1:?variant name}
shift
OUT=$HERE/../lib/exp
OBJ=$OUT/obj_$NAME
mkdir -p "$OBJ"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-rdc -Wall -Wno-unused-function"
pids=()
SRCS=$(sed -n 's/^SRCS := //p' "$HERE/Makefile" | sed 's/\.hip//g')
for f in $SRCS; do
    EXTRA=""
    [ "$f" = render_bwd ] && EXTRA="-ffp-contract=fast -fno-slp-vectorize"
    [ "$f" = render_fwd ] && EXTRA="-fno-slp-vectorize"
    /opt/rocm/bin/hipcc $FLAGS $EXTRA "$@" -c "$HERE/$f.hip" -o "$OBJ/$f.o" &
    pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/$NAME.so" "$OBJ"/*.o
echo "$OUT/$NAME.so"
