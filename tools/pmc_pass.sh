#!/bin/bash
# tools/pmc_pass.sh <out_dir> <lib or ""> <counters...>: one rocprofv3 counter pass over
# tools/perf_fresh.py (one cold + one timed submit of 20 M config-3 events).
out=$1; lib=$2; shift 2
if [ -n "$lib" ]; then export EBD_LIB=$lib; fi
rocprofv3 --pmc "$@" -d "$out" -o p --output-format csv -- python tools/perf_fresh.py --reps 1
