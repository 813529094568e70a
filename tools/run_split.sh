set -o pipefail
O=gpurun_out/r05_split; mkdir -p $O
timeout -k 10 300 python tools/ab_split_sizes.py 8,8 10,6 9,7 --family timesformer --rounds 10 > $O/tsf.txt 2>&1 || { tail -20 $O/tsf.txt; exit 1; }
cat $O/tsf.txt
timeout -k 10 300 python tools/ab_split_sizes.py 2,2 3,1 --family resnet3d --rounds 10 > $O/r3d.txt 2>&1 || { tail -20 $O/r3d.txt; exit 1; }
cat $O/r3d.txt
timeout -k 10 300 python tools/ab_split_sizes.py 4,4 5,3 --rounds 16 > $O/vivit3.txt 2>&1 || { tail -20 $O/vivit3.txt; exit 1; }
cat $O/vivit3.txt
