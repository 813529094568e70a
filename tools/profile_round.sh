#!/bin/bash
# One GPU session that produces every number a bench line cites, from ONE build, on the configuration
# the bench TIMES (round 5: the headline split -- 2 HIP streams, graph replay; before, one stream):
#   bench JSON (bench.py --mode $MODE), rocprofv3 kernel-trace stats + per-dispatch timeline of the
#   headline command alone (tools/headline.py: exactly the kernels of the timed region), HBM traffic per
#   kernel (FETCH_SIZE x2 / WRITE_SIZE passes), SQ / GRBM counter groups, each pass on that command.
#   TAG=r05_fwd MODE=fwd bash tools/profile_round.sh      -> gpurun_out/$TAG/...
# Copy the summaries into profiles/ afterwards (tools/collect_profiles.py $TAG).
set -o pipefail
TAG=${TAG:-r05}
MODE=${MODE:-fwd}
OUT=gpurun_out/$TAG
mkdir -p $OUT
STEPS=${STEPS:-20}
BENCH_ARGS=${BENCH_ARGS:-}
if [ "$MODE" = "train" ]; then
  PROF="bench.py --mode train --steps 3 --warmup 1 --no-cpu-baseline"
  TRACE="bench.py --mode train --steps $STEPS --no-cpu-baseline"
else
  # counters and the per-kernel durations bench.py's roofline is checked against: the headline's own
  # launches serialised on one stream (--serial 1, as bench.py times them); the concurrent headline
  # (2 streams, graph replay) gets its own trace and timeline
  PROF="tools/headline.py --mode $MODE --steps 2 --warmup 1 --serial 1"
  TRACE="tools/headline.py --mode $MODE --steps $STEPS --serial 1"
  HTRACE="tools/headline.py --mode $MODE --steps $STEPS"
fi
# the profiled command, recorded beside its outputs (tools/collect_profiles.py stamps it and the
# bench mode on every summary: bench.py cites only counters of its own build AND mode)
echo "python3 $PROF" > $OUT/pmc_command.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
echo "== kernel trace: $TRACE"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 $TRACE > $OUT/trace.log 2>&1
rc=$?; tail -2 $OUT/trace.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$HTRACE" ]; then
  echo "== headline kernel trace: $HTRACE"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/htrace -o run --output-format csv -- \
    python3 $HTRACE > $OUT/htrace.log 2>&1
  rc=$?; tail -2 $OUT/htrace.log; [ $rc -eq 0 ] || exit $rc
  python3 tools/trace_timeline.py $OUT/htrace > $OUT/timeline.json; rc=$?; [ $rc -eq 0 ] || exit $rc
fi
echo "== traffic"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- \
    python3 $PROF > $OUT/pmc_$c.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pmc $c failed rc=$rc"; tail -5 $OUT/pmc_$c.log; exit $rc; }
done
echo "== pmc groups"
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_g$i -o run -- \
    python3 $PROF > $OUT/pmc_g$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pmc group $i failed rc=$rc"; tail -5 $OUT/pmc_g$i.log; exit $rc; }
done
# the bench line LAST, citing this session's counters (collected here under gpurun_out/$TAG/prof with the
# names they get in profiles/)
python3 tools/collect_profiles.py $TAG --dst $OUT/prof > /dev/null || exit 1
if [ -z "$NO_BENCH" ]; then
  echo "== bench"
  VCLIP_PROFILES=$OUT/prof timeout -k 10 400 python3 bench.py --mode $MODE --steps $STEPS $BENCH_ARGS > $OUT/bench.log 2>&1
  rc=$?; tail -c 400 $OUT/bench.log; echo; [ $rc -eq 0 ] || exit $rc
  grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
fi
echo "== done"
