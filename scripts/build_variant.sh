#!/bin/bash
# Build an A/B variant of libpdplqr.so with extra -D flags into pdp-lqr_amd/build/variants/.
# usage: scripts/build_variant.sh NAME [-DFOO=1 ...]     (CPU side; the .so travels with gpurun)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
C=$ROOT/pdp-lqr_amd/csrc
SRCS=$(sed -n 's/^SRCS := //p' "$C/Makefile")
OUTD=${VARIANT_DIR:-$ROOT/pdp-lqr_amd/build/variants}
mkdir -p "$OUTD"
cd "$C"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I"$ROOT/include" -mllvm -amdgpu-mfma-vgpr-form \
  "$@" -shared -o "$OUTD/libpdplqr_$NAME.so" $SRCS
