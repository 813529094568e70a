# round 4 final, part C: ResNet3D-50 (automatic conv ring A/B, then the profile session) and the ViViT
# train-step profile session
set -o pipefail
mkdir -p gpurun_out/r04_final
timeout -k 10 400 python -u tools/r04/ab_resnet3d_ring.py '{"s2": 2, "s3": 2, "s4": 2, "s5": 2}' '{}' --rounds 8 > gpurun_out/r04_final/ab_ring_auto.log 2>&1; rc=$?
cat gpurun_out/r04_final/ab_ring_auto.log; [ $rc -eq 0 ] || exit $rc
TAG=r04_resnet3d BENCH_ARGS="--mode resnet3d" bash tools/profile_round.sh || exit $?
TAG=r04_train BENCH_ARGS="--mode train" bash tools/profile_round.sh
