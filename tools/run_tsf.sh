set -o pipefail
O=gpurun_out/r05_tsf; mkdir -p $O
timeout -k 10 200 python tools/pp_check.py --cfgs 8,15,4,24 --only tsf_fc1_B8,fc2_B4 --rounds 7 > $O/pp.txt 2>&1 || { tail -20 $O/pp.txt; exit 1; }
cat $O/pp.txt
timeout -k 10 400 python tools/ab_family_cfg.py timesformer '{}' '{"fc1": 8}' '{"fc2": 24}' '{"qkv_temporal": 8, "qkv_spatial": 8}' > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
