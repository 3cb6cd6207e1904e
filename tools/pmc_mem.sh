#!/bin/bash
# tools/pmc_mem.sh <out_dir> <lib or ""> : memory-side counter passes over perf_fresh (20 M config-3 events)
out=$1; lib=$2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
if [ -n "$lib" ]; then export EBD_LIB=$PWD/ebpf-discovery_amd/build/variants/libebd_amd_$lib.so; fi
run() { n=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$out/$n" -o p --output-format csv -- python3 tools/perf_fresh.py --reps 1 || exit $?; }
run a FETCH_SIZE TCC_HIT_sum
run b TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_MISS_sum
run c TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAIT_INST_ANY
run d SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU
python3 tools/pmc_summary.py "$out" k_fresh
