# round 4 final, part C: ResNet3D-50 and ViViT train-step profile sessions
set -o pipefail
TAG=r04_resnet3d BENCH_ARGS="--mode resnet3d" bash tools/profile_round.sh || exit $?
TAG=r04_train BENCH_ARGS="--mode train" bash tools/profile_round.sh
