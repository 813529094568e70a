# round 4 batch 8: ResNet3D stream count (graph replay, one process), then the final-build TimeSformer-B
# and Swin-T profile sessions
set -o pipefail
T=${TAG:-r04_b8}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 300 python -u tools/r04/ab_streams_family.py resnet3d 2 3 4 --rounds 6 > $OUT/ab_streams_r3d.log 2>&1; rc=$?
cat $OUT/ab_streams_r3d.log; [ $rc -eq 0 ] || exit $rc
bash tools/r04/gpu_final_b.sh
