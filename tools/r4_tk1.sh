#!/bin/bash
set -e
cd tools/bin
for v in "tk_base 0" "tk_base 32" "tk_base 64" "tk_m0 0" "tk_m0 32" "tk_k3e 0" "tk_base 0" "tk_base 32"; do
  set -- $v; timeout -k 10 90 ./$1 2048 "$1_pad$2" 512 $2
done
