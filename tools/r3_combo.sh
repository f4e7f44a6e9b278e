#!/bin/bash
# tests, then (unless a GPU step crashed or timed out) the measurement passes
# Usage: bash tools/r3_combo.sh <tag> "<pytest files>" <prof modes...>
tag=$1; files=$2; shift 2
bash tools/r3_run.sh $tag tests "$files"
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc: stopping"; exit $rc; fi
for m in "$@"; do
  bash tools/r3_prof.sh $tag $m || exit $?
done
exit $rc
