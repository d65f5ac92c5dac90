#!/bin/bash
# Build an A/B variant of the library: fisdf/libfisdf_<name>.so with extra hipcc flags on the
# listed sources (default zgemm.hip); the other objects are the default build's.
#   bash tools/build_variant.sh NAME "-DFISDF_PREREAD=1" [zgemm.hip fft.hip ...]
set -e
NAME=$1; FL=$2; shift 2
SRCS=${@:-zgemm.hip}
cd "$(dirname "$0")/../fft-isdf-scratch_amd/csrc"
make -s
D=/tmp/fisdf_var_$NAME
mkdir -p $D
OBJS=""
for s in api zgemm zgemm_wide fft pchol linalg ao; do
  if [[ " $SRCS " == *" $s.hip "* ]]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function \
      -I../../include -mllvm -amdgpu-mfma-vgpr-form=1 $FL -c $s.hip -o $D/$s.o
    OBJS="$OBJS $D/$s.o"
  else
    OBJS="$OBJS $s.o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS -ldl -o ../fisdf/libfisdf_$NAME.so
echo "built fisdf/libfisdf_$NAME.so ($FL on $SRCS)"
