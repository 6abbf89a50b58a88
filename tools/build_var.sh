#!/bin/bash
# tools/build_var.sh NAME SRC "DEFINES" -- build the library with one source file compiled with
# extra defines into build/var/NAME.so (every other object from the in-tree build). For A/B runs
# on the GPU box: RMIMO_LIB=$PWD/build/var/NAME.so python bench.py ...
set -e
NAME=$1; SRC=${2:-decode_stream.hip}; DEFS=$3
cd "$(dirname "$0")/../rub_mimo_amd/csrc"
OBJ=../../build/obj
OUT=../../build/abl
VAR=../../build/var
mkdir -p $VAR
mkdir -p $OUT
make -j8 >/dev/null
base=$(basename $SRC .hip)
base=$(basename $base .cpp)
FLAGS=""
case $base in sync_kernels|synth_kernels) FLAGS="-ffp-contract=off" ;; esac
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -I../../include \
  $FLAGS $DEFS -c $SRC -o $OUT/${base}_$NAME.o
objs=$(ls $OBJ/*.o | grep -v "/$base.o\$")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $VAR/$NAME.so $objs $OUT/${base}_$NAME.o
echo "built $VAR/$NAME.so"
