#!/bin/bash
# round 6: configs[2] loop with the SNAC stream confined to a CU subset (MORPHEUS_MX_SNAC_CUS)
set -o pipefail
O=gpurun_out/r06_cumask; mkdir -p $O
run() { tag=$1; shift; env "$@" timeout -k 10 240 python -u scripts/snac_share.py > $O/$tag.log 2>&1 || exit 1; }
run base A=1
run c64s4 MORPHEUS_MX_SNAC_CUS=64:4
run c64s1 MORPHEUS_MX_SNAC_CUS=64:1
run c32s8 MORPHEUS_MX_SNAC_CUS=32:8
run c128s2 MORPHEUS_MX_SNAC_CUS=128:2
run c64s4x MORPHEUS_MX_SNAC_CUS=64:4 MORPHEUS_MX_DECODE_CUS_REST=1
