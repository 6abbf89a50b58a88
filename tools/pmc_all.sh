#!/bin/bash
# tools/pmc_all.sh TAG [bench args...] -- the standard PMC passes over the decode kernels
# (one rocprofv3 run per pass; FETCH_SIZE and WRITE_SIZE in passes of their own)
R=$(cd "$(dirname "$0")/.." && pwd)
tag=$1; shift
set -e
"$R/tools/pmc_run.sh" "${tag}_sqa" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "$@"
"$R/tools/pmc_run.sh" "${tag}_sqb" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE" "$@"
"$R/tools/pmc_run.sh" "${tag}_fetch" "FETCH_SIZE" "$@"
"$R/tools/pmc_run.sh" "${tag}_write" "WRITE_SIZE" "$@"
"$R/tools/pmc_run.sh" "${tag}_tcc" "TCC_HIT_sum TCC_MISS_sum" "$@"
