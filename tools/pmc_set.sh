#!/bin/bash
# tools/pmc_set.sh <out_dir> <perf_fresh args...>: counter passes (one rocprofv3 --pmc run each,
# within the per-block limits) over tools/perf_fresh.py; summarise with tools/pmc_summary.py.
out=$1; shift
export TMPDIR=/tmp
run() { timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$out/$1" -o p --output-format csv -- python3 tools/perf_fresh.py $ARGS; }
ARGS="$*"
set -e
run SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS
run SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU
run TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum
run TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum
