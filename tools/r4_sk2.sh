#!/bin/bash
set -e
cd tools/bin
timeout -k 10 60 ./sk2_pd2 2048 512 1
for b in sk_base sk_ent; do timeout -k 10 60 ./$b 2048 98304; done
for v in pd2 pd3 pd2l pd3l pd3p pd2lp pd4lp pd2 pd3; do timeout -k 10 60 ./sk2_$v 2048 512; done
timeout -k 10 60 ./sk_base 2048 98304
