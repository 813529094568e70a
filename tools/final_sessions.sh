#!/bin/bash
# Round-end evidence on ONE build: for each mode in $MODES, tools/profile_round.sh (kernel traces of the
# headline command, HBM traffic and SQ counter passes, then the bench line citing them) into
# gpurun_out/${ROUND}_${mode}/.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
ROUND=${ROUND:-r05f}
for m in ${MODES:-fwd train}; do
  tag=${ROUND}_$m
  echo "== session $tag"
  TAG=$tag MODE=$m bash tools/profile_round.sh > gpurun_out/$tag.log 2>&1
  rc=$?; tail -3 gpurun_out/$tag.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/$tag.log; exit $rc; }
done
echo "== done"
