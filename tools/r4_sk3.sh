#!/bin/bash
set -e
cd tools/bin
for b in sk_base_a2 sk_base_a16 sk_base_a17 sk_base_a18 sk_base_a0 sk_ent sk_ent_a16 sk_base_a2 sk_base_a16; do timeout -k 10 60 ./$b 2048 98304; done
for a in 2 16 17 18 2 16; do timeout -k 10 90 ./tk_a$a 2048 aux$a 512; done
