#!/bin/bash
# Round 5, call AJ: the earlier-tuned knobs of the headline kernel re-checked with the two-step
# prefetch: s_setprio off (prio0), P4 after P12 (ord0), 4 outputs per P4 item (k4), idle waves
# not branching around P4 (ws0); tools/timek.hip 2048^3 r=4.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5aj.txt
cd tools/exp
for rep in 1 2 3; do for v in s0 prio0 ord0 k4 ws0; do timeout -k 10 90 ./tk_$v 2048 $v 512 >> $O || exit 1; done; done
