#!/bin/bash
# Build the committed tree's library (git REV, default HEAD) as fisdf/libfisdf_<name>.so for an
# A/B against the working tree:  bash tools/build_base.sh [REV] [name]
set -e
REV=${1:-HEAD}; NAME=${2:-base}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=/tmp/fisdf_base_$NAME
rm -rf $D && mkdir -p $D
git -C $ROOT archive $REV fft-isdf-scratch_amd/csrc include | tar -x -C $D
make -s -C $D/fft-isdf-scratch_amd/csrc -j8 OUT=$ROOT/fft-isdf-scratch_amd/fisdf/libfisdf_$NAME.so
echo "built fisdf/libfisdf_$NAME.so from $REV"
