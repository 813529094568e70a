#!/bin/bash
# One GPU session that produces every number the headline bench line cites, from ONE build:
#   bench JSON, rocprofv3 kernel-trace stats of the same bench command on one HIP stream (--streams 1:
#   the bench's roofline pass runs there, so the trace's per-launch durations are the ones its HIP
#   events time; under two streams kernels share the CUs), HBM traffic per kernel
#   (FETCH_SIZE x2 / WRITE_SIZE passes), attention + GEMM PMC counters.
#   TAG=r02_v1 bash tools/profile_round.sh      -> gpurun_out/$TAG/...
# Copy the summaries into profiles/ afterwards (tools/collect_profiles.py).
set -o pipefail
TAG=${TAG:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
STEPS=${STEPS:-20}
BENCH_ARGS=${BENCH_ARGS:-}
echo "== bench"
timeout -k 10 300 python3 bench.py --steps $STEPS $BENCH_ARGS > $OUT/bench.log 2>&1
rc=$?; tail -c 600 $OUT/bench.log; echo; [ $rc -eq 0 ] || exit $rc
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
# the profiled command, recorded beside its outputs (tools/collect_profiles.py stamps it and the
# bench mode on every summary: bench.py cites only counters of its own build AND mode)
echo "python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --streams 1 $BENCH_ARGS" > $OUT/pmc_command.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
echo "== kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 bench.py --steps $STEPS --no-cpu-baseline --streams 1 $BENCH_ARGS > $OUT/trace.log 2>&1
rc=$?; tail -2 $OUT/trace.log; [ $rc -eq 0 ] || exit $rc
[ -n "$NO_PMC" ] && { echo "== done (no pmc)"; exit 0; }
echo "== traffic"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --streams 1 $BENCH_ARGS > $OUT/pmc_$c.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pmc $c failed rc=$rc"; tail -5 $OUT/pmc_$c.log; exit $rc; }
done
echo "== pmc groups"
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_g$i -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --streams 1 $BENCH_ARGS > $OUT/pmc_g$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pmc group $i failed rc=$rc"; tail -5 $OUT/pmc_g$i.log; exit $rc; }
done
echo "== done"
