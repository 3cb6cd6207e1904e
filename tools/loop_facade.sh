#!/bin/bash
# Runs the C++ facade test binary on the GPU several times (a check of a flaky result, not of a
# fault: any exit status other than 0 or 1 ends the loop at once).
n=${1:-20}
fails=0
for k in $(seq 1 "$n"); do
	timeout -k 5 60 tests/cpp/build/facade_test gpu > "gpurun_out/cpp_loop_$k.log" 2>&1
	rc=$?
	if [ $rc -eq 1 ]; then
		fails=$((fails + 1))
		echo "run $k: checks failed"
		tail -4 "gpurun_out/cpp_loop_$k.log"
	elif [ $rc -ne 0 ]; then
		echo "run $k ended with $rc: stopping"
		exit $rc
	fi
done
echo "runs $n, failed $fails"
