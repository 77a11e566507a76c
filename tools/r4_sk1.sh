#!/bin/bash
# round 4: LDS-DMA skeleton sweep (tools/skel2.hip) beside the round-3 skeleton on one box
set -e
cd tools/bin
timeout -k 10 60 ./sk2_pd4 2048 512 1
for b in sk_base sk_ent; do timeout -k 10 60 ./$b 2048 98304; done
for v in pd2 pd3 pd4 pd6 pd8 pd4nt pd4noring pd4noxch; do timeout -k 10 60 ./sk2_$v 2048 512; done
timeout -k 10 60 ./sk2_pd4 2048 256
