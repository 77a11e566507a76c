#!/bin/bash
# round 3 session 2: zarrs_ome end to end at 2048^3 u16 — device-resident, the reference's store
# loop, and the octant split over 2 and 4 processes sharing device 0 (one-GPU rehearsal)
set -u
OUT=gpurun_out/r3s2l
mkdir -p $OUT
timeout -k 10 900 python3 -u tools/bench_ome_e2e.py --size 2048 --levels 5 --threads 16 --gpus 2 4 > $OUT/ome_e2e.json 2> $OUT/ome_e2e.err || { tail $OUT/ome_e2e.err; exit 1; }
cut -c1-1500 $OUT/ome_e2e.json
for v in ty16 ty32 ty8 ty16 ty32 ty8; do timeout -k 10 180 tools/tg4r_$v $v >> $OUT/tg4r.txt 2>&1 || { cat $OUT/tg4r.txt; exit 1; }; done
cat $OUT/tg4r.txt
