#!/bin/bash
# tools/abl_search.sh -- timing-ablation builds of est_kernels.hip into build/abl/s_<name>.so
set -e
cd "$(dirname "$0")/../rub_mimo_amd/csrc"
OBJ=../../build/obj
OUT=../../build/abl
mkdir -p $OUT
make -j8 >/dev/null
for v in ${VARIANTS:-nols noinv}; do
  case $v in
    nols) D="-DSL_ABL_NOLS" ;;
    noinv) D="-DSL_ABL_NOINV" ;;
    both) D="-DSL_ABL_NOLS -DSL_ABL_NOINV" ;;
    nofwd) D="-DSL_ABL_NOLS -DSL_ABL_NOINV -DSL_ABL_NOFWD" ;;     # loads + scoring only
    noload) D="-DSL_ABL_NOLS -DSL_ABL_NOINV -DSL_ABL_NOFWD -DSL_ABL_NOLOAD" ;;   # scoring only
    lslds) D="-DSL_ABL_LSLDS" ;;                                 # LS transform batched in LDS
    lsonly) D="-DSL_ABL_NOINV -DSL_ABL_NOFWD" ;;                 # loads + scoring + LS
  esac
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include $D \
    -c est_kernels.hip -o $OUT/est_$v.o
  objs=$(ls $OBJ/*.o | grep -v '/est_kernels.o$')
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $OUT/s_$v.so $objs $OUT/est_$v.o
done
