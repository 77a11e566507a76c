#!/bin/bash
set -e
for g in "2 4" "4 2" "8 1"; do
  timeout -k 10 400 python -u tools/bench_ops.py --only tshare --reps 3 --t-groups $g
done
