#!/bin/bash
# Round-4 final profiling pass (GPU box, repo root): headline bench + kernel trace + PMC traffic
# keyed to this build (tools/prof_final.sh), the --share G/8 proxies with their own share-keyed
# PMC traffic, and the config T share counter passes.
set -u
O=gpurun_out/r4_final
tools/prof_final.sh r4_final || exit 1
cp $O/pmc_traffic.json profiles/pmc_traffic.json
for G in 0 3 7; do
  PASSES="fetch write" tools/profile_pmc.sh $O/share$G --share $G/8 --steps 1 --warmup 0 --parity-chunks 0 || exit 1
  python3 tools/make_traffic_json.py $O/share$G profiles/pmc_traffic.json 2048 4 $G/8 || exit 1
done
cp profiles/pmc_traffic.json $O/pmc_traffic_all.json
for G in 0 3 7; do
  timeout -k 10 300 python3 bench.py --share $G/8 --no-cpu-baseline > $O/share$G.json 2> $O/share$G.err || exit 1
done
tools/profile_pmc_tshare.sh $O/tshare_pmc || exit 1
echo done
