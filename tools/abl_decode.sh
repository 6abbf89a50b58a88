#!/bin/bash
# tools/abl_decode.sh -- build timing-ablation variants of the streaming decode into
# build/abl/<name>.so (outputs are wrong by construction; for stage timing only).
# On the GPU box: for v in base nostore nodma nofft; do RMIMO_LIB=build/abl/$v.so python bench.py ...
set -e
cd "$(dirname "$0")/../rub_mimo_amd/csrc"
OBJ=../../build/obj
OUT=../../build/abl
mkdir -p $OUT
make -j8 >/dev/null
for v in ${VARIANTS:-base nostore nodma nofft nostore_nodma nodemap}; do
  case $v in
    base) D="" ;;
    nostore) D="-DDS_ABL_NOSTORE" ;;
    nodma) D="-DDS_ABL_NODMA" ;;
    nofft) D="-DDS_ABL_NOFFT" ;;
    nostore_nodma) D="-DDS_ABL_NOSTORE -DDS_ABL_NODMA" ;;
    nodemap) D="-DDS_ABL_NODEMAP" ;;
    all_off) D="-DDS_ABL_NOSTORE -DDS_ABL_NODMA -DDS_ABL_NODEMAP" ;;
  esac
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include $D $EXTRA \
    -c decode_stream.hip -o $OUT/ds_$v.o
  objs=$(ls $OBJ/*.o | grep -v '/decode_stream.o$')
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $OUT/$v.so $objs $OUT/ds_$v.o
done
ls -la $OUT/*.so
