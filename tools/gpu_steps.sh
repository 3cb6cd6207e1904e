#!/bin/bash
# Runs GPU steps in order on the gpurun box, each under its own time limit.
# Usage: tools/gpu_steps.sh "<name>:<timeout_s>:<command>" ...
# Stops at the first step that faults, aborts, segfaults or times out (exit 124/134/137/139
# or a negative signal); an ordinary failure (exit 1, e.g. a failing assert) does not stop
# the remaining steps.  Logs go to gpurun_out/<name>.log.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
status=0
for spec in "$@"; do
	name="${spec%%:*}"; rest="${spec#*:}"; tmo="${rest%%:*}"; cmd="${rest#*:}"
	echo "=== [$name] (limit ${tmo}s) $cmd" | tee -a gpurun_out/steps.log
	start=$(date +%s)
	timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
	rc=$?
	echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
	tail -n 5 "gpurun_out/$name.log"
	if [ $rc -ne 0 ]; then status=$rc; fi
	# a GPU fault reported as an ordinary failure (pytest exit 1) still ends the call
	if grep -qE "illegal memory access|APERTURE_VIOLATION|Memory access fault" "gpurun_out/$name.log"; then
		echo "=== stopping: step $name hit a GPU fault" | tee -a gpurun_out/steps.log
		exit 99
	fi
	case $rc in
		0|1|2|5) ;;
		*) echo "=== stopping: step $name ended with $rc" | tee -a gpurun_out/steps.log; exit $rc ;;
	esac
done
exit $status
