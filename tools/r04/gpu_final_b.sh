# round 4 final, part B: TimeSformer-B and Swin-T profile sessions (bench, kernel trace, traffic, counters)
set -o pipefail
TAG=r04_timesformer BENCH_ARGS="--mode timesformer" bash tools/profile_round.sh || exit $?
TAG=r04_swin BENCH_ARGS="--mode swin" bash tools/profile_round.sh
